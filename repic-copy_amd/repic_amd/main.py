"""``repic``-compatible CLI dispatcher (reference repic/main.py:11-34).

Registers the same subcommand plugin protocol: ``get_cliques`` (the hot path) and its
consumer ``run_ilp`` (exact set packing on the device instead of Gurobi, so nothing here
imports gurobipy).  The workflow drivers (``iter_config``, ``iter_pick``) stay with the
reference package.
"""
from __future__ import annotations

import argparse

from . import __version__
from .commands import get_cliques, run_ilp


def main(argv=None):
    parser = argparse.ArgumentParser()
    parser.add_argument("--version", action="version", version=f"REPIC-MI355X {__version__}")
    sub = parser.add_subparsers(title="commands", dest="command", required=True)
    for module in (get_cliques, run_ilp):
        p = sub.add_parser(module.name)
        module.add_arguments(p)
        p.set_defaults(func=module.main)
    args = parser.parse_args(argv)
    args.func(args)


if __name__ == "__main__":
    main()
