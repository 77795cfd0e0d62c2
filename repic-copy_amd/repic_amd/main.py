"""``repic``-compatible CLI dispatcher (reference repic/main.py:11-34).

Registers the same subcommand plugin protocol.  Only ``get_cliques`` is implemented here
(the hot path); the other reference subcommands (``run_ilp``, ``iter_config``,
``iter_pick``) are unchanged consumers/callers and stay with the reference package, so this
module never imports gurobipy.
"""
from __future__ import annotations

import argparse

from . import __version__
from .commands import get_cliques


def main(argv=None):
    parser = argparse.ArgumentParser()
    parser.add_argument("--version", action="version", version=f"REPIC-MI355X {__version__}")
    sub = parser.add_subparsers(title="commands", dest="command", required=True)
    for module in (get_cliques,):
        p = sub.add_parser(module.name)
        module.add_arguments(p)
        p.set_defaults(func=module.main)
    args = parser.parse_args(argv)
    args.func(args)


if __name__ == "__main__":
    main()
