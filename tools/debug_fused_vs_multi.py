#!/usr/bin/env python3
"""Debug helper: run one synthetic batch through the fused kernel and the multi-kernel path
and print the first cliques whose outputs differ (canonical column order)."""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "repic-copy_amd"))
import numpy as np  # noqa: E402

from repic_amd import _lib, synth  # noqa: E402
from repic_amd.pipeline import Batch, run_batch  # noqa: E402

n_true = int(sys.argv[1]) if len(sys.argv) > 1 else 600
n_mg = int(sys.argv[2]) if len(sys.argv) > 2 else 8
multi = len(sys.argv) > 3 and sys.argv[3] == "multi"
cfg = synth.SynthConfig(k=3, n_true=n_true, box=180, width=4096, height=4096, dup=0.1, seed=7)
mgs = synth.batch(cfg, n_mg)
b = Batch.pack(cfg.k, cfg.box, mgs)
ctx = _lib.Context(0)
ra = run_batch(ctx, b, members=True, multi_out=multi)
rb = run_batch(ctx, b, members=True, multi_out=multi, no_fused=True)
bad = 0
for m in range(n_mg):
    a, c = ra[m], rb[m]
    n = int(b.box_off[(m + 1) * 3] - b.box_off[m * 3])
    assert a.status == c.status, (m, a.status, c.status)
    pa = np.lexsort(a.rows.T[::-1])
    pc = np.lexsort(c.rows.T[::-1])
    assert np.array_equal(a.rows[pa], c.rows[pc]), m
    for fld in ("w", "conf", "consensus", "members", "order"):
        va, vc = getattr(a, fld), getattr(c, fld)
        if va is None:
            continue
        va, vc = va[pa], vc[pc]
        diff = np.nonzero((va != vc).reshape(len(va), -1).any(axis=1))[0]
        for j in diff[:5]:
            mem = va[j] if fld == "members" else a.members[pa][j]
            print(f"mg {m} n {n} fld {fld} clique {j}: fused {va[j]} multi {vc[j]} members {mem}"
                  f" xy {[(b.x[g], b.y[g]) for g in mem]}")
        bad += len(diff)
print("mismatching entries:", bad)
ctx.close()
