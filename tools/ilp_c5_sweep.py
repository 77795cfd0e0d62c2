#!/usr/bin/env python3
"""run_ilp on one complete C5 micrograph (the device path's get_cliques output) at several
node budgets: sections, status, certified gap, objective and wall time per budget.

  RGC_ILP_DEBUG=1 python tools/ilp_c5_sweep.py [node_limit ...]
"""
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "repic-copy_amd"))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "tests"))

import numpy as np  # noqa: E402


def main():
    from test_ilp import _c5_model
    from repic_amd import _lib
    from repic_amd.ilp import solve_batch
    A, w = _c5_model()
    limits = [int(a) for a in sys.argv[1:]] or [0]
    for nl in limits:
        ctx = _lib.Context(0)
        t0 = time.time()
        xs, st, g = solve_batch(ctx, [A], [w], node_limit=nl, statuses=True, gaps=True,
                                timing=True)
        dt = time.time() - t0
        secs = [(n, round(ms, 1)) for n, ms in ctx.kernel_times()]
        ctx.close()
        obj = float(np.asarray(w, np.float64)[xs[0] == 1].sum())
        print(f"node_limit {nl}: status {st[0]} gap {g[0]:.3e} objective {obj:.6f} "
              f"wall {dt:.2f} s sections {secs}", flush=True)


if __name__ == "__main__":
    main()
