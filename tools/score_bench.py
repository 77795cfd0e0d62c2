#!/usr/bin/env python3
"""score_detections throughput: C2-like micrograph pairs (4096^2 px, ~300
ground-truth and ~330 picked boxes of 180 px) scored in one batched raster launch, beside
the oracle's numpy masks (the reference's algorithm, score_detections.py:16-48) on 1 core.

  python tools/score_bench.py [--pairs 2000] [--reps 5]

Prints one JSON line: pairs/s, Mpixel/s per mask, kernel ms (HIP events), the reference's
mask traffic it avoids (two int16 H x W masks written and read back: 8 B per pixel), and the
CPU leg.
"""
from __future__ import annotations

import argparse
import json
import os
import sys
import time
import warnings

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "repic-copy_amd"))
sys.path.insert(0, ROOT)


def make_pairs(n, seed=0, W=4096, H=4096, box=180):
    rng = np.random.default_rng(seed)
    out = []
    for _ in range(n):
        c = rng.uniform(0, [W - box, H - box], (300, 2))
        g = np.concatenate([np.rint(c), np.full((300, 2), float(box)),
                            rng.uniform(0.3, 1, (300, 1))], axis=1)
        keep = rng.random(300) < 0.9
        pk = np.rint(c[keep] + rng.normal(0, 0.08 * box, (int(keep.sum()), 2)))
        fp = np.rint(rng.uniform(0, [W - box, H - box], (60, 2)))
        pk = np.concatenate([pk, fp])
        p = np.concatenate([pk, np.full((len(pk), 2), float(box)),
                            rng.uniform(0, 1, (len(pk), 1))], axis=1)
        out.append((g, p))
    return out


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--pairs", type=int, default=2000)
    ap.add_argument("--reps", type=int, default=5)
    ap.add_argument("--cpu-budget", type=float, default=10.0)
    args = ap.parse_args()
    from repic_amd import score_detections as sd
    pairs = make_pairs(args.pairs)
    W = H = 4096
    sd.score_pairs(pairs[:8], mrc_w=W, mrc_h=H)                    # warm-up
    kms, walls = [], []
    for _ in range(args.reps):
        t0 = time.perf_counter()
        res, kt = sd.score_pairs(pairs, mrc_w=W, mrc_h=H, timing=True)
        walls.append(time.perf_counter() - t0)
        kms.append(kt["k_score_raster"])
    k = float(np.median(kms))
    wall = float(np.median(walls))
    px = args.pairs * W * H
    from oracle import score_ref
    t0 = time.perf_counter()
    n = 0
    for g, p in pairs:
        with warnings.catch_warnings():
            warnings.simplefilter("ignore")
            want = score_ref.get_segmentation_scores([tuple(r) for r in g.tolist()],
                                                     [tuple(r) for r in p.tolist()], None, W, H)
        assert tuple(want) == tuple(res[n]), n
        n += 1
        if time.perf_counter() - t0 > args.cpu_budget:
            break
    cdt = time.perf_counter() - t0
    print(json.dumps({
        "metric": "score_detections pairs/s (4096^2 micrographs, ~300 GT + ~330 picks of 180 px)",
        "value": args.pairs / (k * 1e-3), "unit": "pairs/s", "pairs": args.pairs,
        "kernel_ms": k, "call_wall_ms": wall * 1e3,
        "pairs_per_s_call": args.pairs / wall,
        "gpixel_per_s_per_mask": px / (k * 1e-3) / 1e9,
        "avoided_mask_bytes_per_pair": 8 * W * H,
        "equivalent_gbs": 8 * px / (k * 1e-3) / 1e9,
        "cpu_baseline": {"value": n / cdt, "unit": "pairs/s", "cores": 1, "kind": "port",
                         "sample": f"{n} pairs, oracle numpy masks (reference algorithm), "
                                   f"{cdt:.1f} s, every one bit-identical to the GPU result"},
    }), flush=True)


if __name__ == "__main__":
    main()
