"""MI355X-native drop-in for REPIC's ``get_cliques`` consensus stage.

Host package: ingest (BOX parsing, pairing, global ids), batch packing, writers and the
``get_cliques`` subcommand plugin; the hot path itself is ``librepic_gc.so`` (HIP, gfx950).
"""
__version__ = "0.1.0"
