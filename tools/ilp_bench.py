#!/usr/bin/env python3
"""run_ilp throughput: the set-packing ILP of a whole batch of C2
micrographs (their get_cliques constraint matrices, computed on the device first) solved
exactly in one rgc_ilp_solve call, beside HiGHS (scipy.optimize.milp, the oracle's exact
solver; Gurobi is not installed) on a bounded sample, 1 process.

  python tools/ilp_bench.py [--config C2] [--n_mg 10000] [--reps 3]

Prints one JSON line: micrographs/s of the solve (host packing excluded / included), per-stage
device ms (HIP events), and the CPU leg.  Every sampled micrograph's objective is checked
against HiGHS.
"""
from __future__ import annotations

import argparse
import json
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "repic-copy_amd"))
sys.path.insert(0, ROOT)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--config", default="C2")
    ap.add_argument("--n_mg", type=int, default=10000)
    ap.add_argument("--reps", type=int, default=3)
    ap.add_argument("--cpu-budget", type=float, default=10.0)
    args = ap.parse_args()
    from scipy.sparse import coo_matrix

    from repic_amd import _lib, synth
    from repic_amd.ilp import solve_batch
    from repic_amd.pipeline import Batch, run_batch
    cfg = synth.SynthConfig(**synth.CONFIGS[args.config], seed=0)
    batch = Batch.pack(cfg.k, cfg.box, synth.batch(cfg, args.n_mg))
    ctx = _lib.Context(0)
    res = run_batch(ctx, batch)
    mats = []
    weights = []
    for r in res:
        C = len(r.w)
        mats.append(coo_matrix((np.ones(C * cfg.k, np.int64),
                                (r.rows.reshape(-1), np.repeat(np.arange(C), cfg.k))),
                               shape=(int(r.n_vert), C)))
        weights.append(r.w)
    solve_batch(ctx, mats[:16], weights[:16])                      # warm-up
    walls, stages = [], []
    for _ in range(args.reps):
        t0 = time.perf_counter()
        xs, exact = solve_batch(ctx, mats, weights, timing=True)
        walls.append(time.perf_counter() - t0)
        stages.append(dict(ctx.kernel_times()))
    dev = {k_: float(np.median([s[k_] for s in stages])) for k_ in stages[0]}
    dev_ms = sum(v for k_, v in dev.items() if k_ != "d2h_x")
    from oracle import ilp_ref
    t0 = time.perf_counter()
    n = 0
    for (A, w), x in zip(zip(mats, weights), xs):
        _, obj = ilp_ref.milp(A, w)
        got = float(np.sum(np.asarray(w, np.float64)[x == 1]))
        assert abs(got - obj) <= 1e-12 * obj, (n, got, obj)
        n += 1
        if time.perf_counter() - t0 > args.cpu_budget:
            break
    cdt = time.perf_counter() - t0
    cols = sum(m.shape[1] for m in mats)
    print(json.dumps({
        "metric": f"run_ilp micrographs/s ({args.config}, exact set packing)",
        "value": args.n_mg / (dev_ms * 1e-3), "unit": "micrographs/s", "n_mg": args.n_mg,
        "cliques": cols, "device_ms": dev_ms, "stage_ms": dev,
        "call_wall_ms": float(np.median(walls)) * 1e3,
        "micrographs_per_s_call": args.n_mg / float(np.median(walls)),
        "all_proven_optimal": bool(all(exact)),
        "cpu_baseline": {"value": n / cdt, "unit": "micrographs/s", "cores": 1,
                         "kind": "HiGHS (scipy.optimize.milp, gap 0); Gurobi not installed",
                         "sample": f"{n} micrographs, {cdt:.1f} s, every objective equal to "
                                   f"the device solver's"},
    }), flush=True)
    ctx.close()


if __name__ == "__main__":
    main()
