#!/usr/bin/env python3
"""Host restatement of the fused kernel's P1 grid plan and P2 2x3 stencil (rgc_fused.hip): every
pair with JI > 0.3 (reference get_cliques.py:40-46, 64-65) must fall in the stencil of its box.

Columns >= 1.08 B wide, rows >= 0.54 B tall; a box searches its column and the neighbouring
column on the side of its half of the column (f32 product, as the kernel), rows cy-1..cy+1.
Random micrographs with integer, fractional and near-threshold clustered coordinates.

The large-micrograph route's k1_bin / k2_pairs plan (f64 keys, row height h, column width 2 h
within bin_budget) is restated by plan_large / missed_large.

  python tools/stencil_check.py [seed] [micrographs] [large]
"""
import sys

import numpy as np

f32 = np.float32


def rcp(v):
    return f32(1.0) / f32(v)


def plan(xs, ys, B, n_budget_boxes, K=1):
    nmax = ((n_budget_boxes + 63) // 64) * 64
    mnx, mny = xs.min(), ys.min()
    ex, ey = xs.max() - mnx, ys.max() - mny
    budget = (4 * nmax + 4) // K
    fex, fey = f32(ex), f32(ey)
    rb = rcp(budget)
    fch = f32(max(f32(0.54 * B) * f32(1.000001), np.sqrt(f32(0.5) * fex * fey * rb),
                  max(f32(0.5) * fex, fey) * rb))
    while True:
        iry = rcp(fch)
        fx = int(np.floor(fex * (f32(0.5) * iry))) + 1
        fy = int(np.floor(fey * iry)) + 1
        if fx <= budget and fy <= budget and fx * fy <= budget:
            break
        fch = f32(fch * f32(1.0625))
    icly = float(rcp(fch))
    icl = 0.5 * icly
    if icl * (1.08 * B) > 1:
        icl = 1 / (1.08 * B)
    if icly * (0.54 * B) > 1:
        icly = 1 / (0.54 * B)
    return mnx, mny, icl, icly, fx, fy


def missed(xs, ys, B):
    """(missed pairs, JI > 0.3 pairs) of one micrograph."""
    mnx, mny, icl, icly, gx, gy = plan(xs, ys, B, len(xs))
    u = (xs - mnx).astype(f32) * f32(icl)
    cx = np.minimum(np.floor(u).astype(int), gx - 1)
    cy = np.minimum(np.floor(((ys - mny).astype(f32) * f32(icly))).astype(int), gy - 1)
    c0 = cx - ((u - cx.astype(f32)) < f32(0.5)).astype(int)
    miss = tot = 0
    for i in range(len(xs)):
        ox = np.maximum((np.minimum(xs[i], xs) + B) - np.maximum(xs[i], xs), 0)
        oy = np.maximum((np.minimum(ys[i], ys) + B) - np.maximum(ys[i], ys), 0)
        inter = ox * oy
        e = np.flatnonzero(inter / ((2 * B * B) - inter) > 0.3)
        e = e[e != i]
        tot += len(e)
        ok = ((cx[e] == c0[i]) | (cx[e] == c0[i] + 1)) & (np.abs(cy[e] - cy[i]) <= 1)
        miss += int((~ok).sum())
    return miss, tot


def plan_large(xs, ys, B, n, K=1):
    """k1_bin's plan (rgc_kernels.hip, the large-micrograph route): f64, row height h, column
    width 2 h, K gx gy <= bin_budget(n)."""
    budget = min(2 * n + 64, 65528)
    per = budget // K
    mnx, mny = xs.min(), ys.min()
    ex, ey = xs.max() - mnx, ys.max() - mny
    h = max(0.54 * B * (1.0 + 1e-9), np.sqrt(0.5 * ex * ey / per), max(0.5 * ex, ey) / per)
    while True:
        fx, fy = np.floor(ex / (2.0 * h)) + 1.0, np.floor(ey / h) + 1.0
        if fx * fy <= per:
            break
        h *= 1.0625
    icl, icly = 1.0 / (2.0 * h), 1.0 / h
    if icl * (1.08 * B) > 1.0:
        icl = 1.0 / (1.08 * B)
    if icly * (0.54 * B) > 1.0:
        icly = 1.0 / (0.54 * B)
    return mnx, mny, icl, icly, int(fx), int(fy)


def missed_large(xs, ys, B):
    """(missed pairs, JI > 0.3 pairs) of k2_pairs' stencil (f64 keys and half test)."""
    mnx, mny, icl, icly, gx, gy = plan_large(xs, ys, B, len(xs))
    u = (xs - mnx) * icl
    cx = np.minimum(np.floor(u), gx - 1).astype(int)
    cy = np.minimum(np.floor((ys - mny) * icly), gy - 1).astype(int)
    c0 = cx - ((u - cx) < 0.5).astype(int)
    miss = tot = 0
    for i in range(len(xs)):
        ox = np.maximum((np.minimum(xs[i], xs) + B) - np.maximum(xs[i], xs), 0)
        oy = np.maximum((np.minimum(ys[i], ys) + B) - np.maximum(ys[i], ys), 0)
        inter = ox * oy
        e = np.flatnonzero(inter / ((2 * B * B) - inter) > 0.3)
        e = e[e != i]
        tot += len(e)
        ok = ((cx[e] == c0[i]) | (cx[e] == c0[i] + 1)) & (np.abs(cy[e] - cy[i]) <= 1)
        miss += int((~ok).sum())
    return miss, tot


def run(seed=0, n_mg=300, large=False):
    rng = np.random.default_rng(seed)
    M = T = 0
    for it in range(n_mg):
        B = float(rng.choice([180, 64, 176, 37, 13, 1000, 2.5]))
        n = int(rng.integers(50, 1500))
        W = float(rng.choice([4096, 1000, 200, 50000]))
        kind = it % 3
        xs, ys = rng.uniform(0, W, n), rng.uniform(0, W, n)
        if kind == 0:
            xs, ys = np.rint(xs), np.rint(ys)
        if kind == 2:   # clusters at offsets just inside the 7/13 B edge limit
            base = rng.uniform(0, W, (n // 4, 2))
            d = (7 / 13) * B * (1 - rng.uniform(0, 1e-3, (n // 4, 2))) * rng.choice([-1, 1], (n // 4, 2))
            pts = np.concatenate([base, base + d, base + d * [1, 0], base + d * [0, 1]])
            xs, ys = pts[:, 0], pts[:, 1]
        m, t = (missed_large if large else missed)(xs, ys, B)
        M += m
        T += t
    return M, T


if __name__ == "__main__":
    seed = int(sys.argv[1]) if len(sys.argv) > 1 else 0
    n = int(sys.argv[2]) if len(sys.argv) > 2 else 300
    m, t = run(seed, n, len(sys.argv) > 3 and sys.argv[3] == "large")
    print(f"missed {m} of {t} JI > 0.3 pairs")
    sys.exit(1 if m else 0)
