#!/usr/bin/env python3
"""Per-phase cycle shares of the fused kernel from the diagnostic build (RGC_STAMPS).

  REPIC_GC_LIB=abl/librepic_gc_diag.so python tools/phase_stamps.py [C2] [n_mg]

Prints, per phase, mean / p50 / p99 s_memtime cycles per workgroup, and the workgroup
timeline (first start, last end) to see how many occupancy rounds the launch took.
Shares only: the stamps add a barrier per phase (never quote this build's run time).
"""
import ctypes as C
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "repic-copy_amd"))
os.environ.setdefault("REPIC_GC_LIB", os.path.join(ROOT, "abl/librepic_gc_diag.so"))

import numpy as np  # noqa: E402

from repic_amd import _lib, synth  # noqa: E402
from repic_amd.pipeline import Batch  # noqa: E402

cfg_name = sys.argv[1] if len(sys.argv) > 1 else "C2"
n_mg = int(sys.argv[2]) if len(sys.argv) > 2 else 10000
cfg = synth.SynthConfig(**synth.CONFIGS[cfg_name], seed=0)
batch = Batch.pack(cfg.k, cfg.box, synth.batch(cfg, n_mg))
ctx = _lib.Context(0)
for _ in range(3):
    r = ctx.run(batch.n_mg, cfg.k, cfg.box, batch.box_off, batch.id_base, batch.x, batch.y,
                batch.score, 0)
f = _lib.lib.rgc_diag_stamps
f.argtypes = [C.c_void_p, C.POINTER(C.c_uint64), C.c_int64]
f.restype = C.c_int64
n = f(ctx._p, None, 0)
buf = (C.c_uint64 * n)()
f(ctx._p, buf, n)
SLOTS = 16 + 13 * 16   # rgc_kernels.h STAMP_SLOTS
raw = np.frombuffer(buf, dtype=np.uint64).reshape(-1, SLOTS).astype(np.int64)
st = raw[:, :13]
nch, ncl = raw[:, 14], raw[:, 15]
print(f"BFS root chunks per micrograph: mean {nch.mean():.2f} p50 {np.median(nch):.0f} "
      f"max {nch.max()} (0 = per-root DFS fallback: {(nch == 0).sum()}); cliques mean {ncl.mean():.0f}")
names = ["P0 load+bbox", "P1 grid+sort", "P2a count", "P2b fwd scan", "P2c fill",
         "P3a union", "P3b CC stats", "P4a DFS+queue", "P4b scan+reserve", "P5 rank",
         "P6a score staging", "P6b epilogue"]
valid = (st != 0).all(axis=1)
d = np.diff(st[valid], axis=1)
tot = d.sum(axis=1)
print(f"{cfg_name}: {n_mg} micrographs, {valid.sum()} complete WGs, cliques {r.n_cliques}")
for i, nm in enumerate(names):
    print(f"  {nm:18s} mean {d[:, i].mean():9.0f}  p50 {np.median(d[:, i]):9.0f}  "
          f"p99 {np.percentile(d[:, i], 99):9.0f}  share {d[:, i].sum() / tot.sum():6.1%}")
# barrier waits: slot 16 + 16 (i + 1) + w = cycles wave w waited in the workgroup barriers of
# phase i (timed barriers of the diagnostic build).  Per phase: the mean wave's barrier-wait
# share of the phase, and the spread of the waves' waits (max - min: the skew between the
# first and last wave to arrive, summed over the phase's barriers)
bw = raw[valid, 16:].reshape(-1, 13, 16)[:, 1:, :]
nw = int(max(1, (bw.sum(axis=(0, 1)) > 0).sum()))
bw = bw[:, :, :nw].astype(np.float64)
print(f"  barrier waits ({nw} waves per workgroup): share of phase cycles, mean wave / "
      f"skew (max - min wave) / phase")
rows = []
for i, nm in enumerate(names):
    ph = d[:, i].astype(np.float64)
    mean_w = bw[:, i, :].mean(axis=1)
    skew = bw[:, i, :].max(axis=1) - bw[:, i, :].min(axis=1)
    share = mean_w.sum() / max(ph.sum(), 1)
    sk = skew.sum() / max(ph.sum(), 1)
    rows.append((nm, d[:, i].sum() / tot.sum(), share, sk))
    print(f"  {nm:18s} phase share {d[:, i].sum() / tot.sum():6.1%}  barrier-wait {share:6.1%}  "
          f"skew {sk:6.1%}  (of the whole WG: {mean_w.sum() / tot.sum():6.1%})")
allw = sum(bw[:, i, :].mean(axis=1).sum() for i in range(len(names)))
print(f"  all phases: waves wait in barriers {allw / tot.sum():.1%} of the workgroup's cycles")
print(f"  per-WG total cycles: mean {tot.mean():.0f} p50 {np.median(tot):.0f} p99 {np.percentile(tot, 99):.0f}")
span = st[valid, 12].max() - st[valid, 0].min()
print(f"  launch span {span} cycles; sum(WG cycles)/span = {tot.sum() / span:.1f} concurrent WGs")

# workgroup timeline from s_memrealtime (slot 13: end << 32 | start, 100 MHz): concurrency over
# the launch and the tail (time while fewer than 90 % of the peak workgroups are resident)
rt = raw[valid, 13].astype(np.uint64)
t0 = (rt & np.uint64(0xFFFFFFFF)).astype(np.int64)
t1 = (rt >> np.uint64(32)).astype(np.int64)
t1 = np.where(t1 < t0, t1 + (1 << 32), t1)
base = t0.min()
t0, t1 = t0 - base, t1 - base
ev = np.concatenate([np.stack([t0, np.ones_like(t0)], 1), np.stack([t1, -np.ones_like(t1)], 1)])
ev = ev[np.lexsort((ev[:, 1], ev[:, 0]))]
conc = np.cumsum(ev[:, 1])
tt = ev[:, 0]
peak = conc.max()
dur = (t1.max()) * 10e-3   # us
wg_us = (t1 - t0) * 10e-3
below = tt[conc >= 0.9 * peak]
tail = (t1.max() - below.max()) * 10e-3 if len(below) else 0.0
ramp = below.min() * 10e-3 if len(below) else 0.0
area = np.sum(np.diff(tt) * conc[:-1]) * 10e-3
print(f"  timeline: span {dur:.1f} us, peak {peak} resident WGs, mean {area / dur:.0f}; "
      f"WG time mean {wg_us.mean():.1f} us p50 {np.median(wg_us):.1f} p99 {np.percentile(wg_us, 99):.1f}; "
      f"ramp to 90% {ramp:.1f} us, tail below 90% {tail:.1f} us")
