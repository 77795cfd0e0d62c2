#!/usr/bin/env python3
"""Host-side cost of one bench step (C2): ms/step with and without F_TIMING events, without
the per-step kernel_times() query, and the bare rgc_run call vs its fused kernel time.

  python tools/host_overhead.py [C2] [n_mg] [steps]
"""
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "repic-copy_amd"))

import numpy as np  # noqa: E402
import torch  # noqa: E402

from repic_amd import _lib, synth  # noqa: E402
from repic_amd.pipeline import Batch  # noqa: E402

cfg_name = sys.argv[1] if len(sys.argv) > 1 else "C2"
n_mg = int(sys.argv[2]) if len(sys.argv) > 2 else 10000
steps = int(sys.argv[3]) if len(sys.argv) > 3 else 30
cfg = synth.SynthConfig(**synth.CONFIGS[cfg_name], seed=0)
batch = Batch.pack(cfg.k, cfg.box, synth.batch(cfg, n_mg))
dev = torch.device("cuda", 0)
dx, dy, ds = (torch.from_numpy(a).to(dev) for a in (batch.x, batch.y, batch.score))
dbo = torch.from_numpy(batch.box_off.astype(np.int32)).to(dev)
did = torch.from_numpy(np.ascontiguousarray(batch.id_base, dtype=np.int64)).to(dev)
torch.cuda.synchronize()
ctx = _lib.Context(0, torch.cuda.current_stream(dev).cuda_stream)


def run(flags):
    return ctx.run(batch.n_mg, cfg.k, cfg.box, batch.box_off, batch.id_base, dx.data_ptr(),
                   dy.data_ptr(), ds.data_ptr(), _lib.F_DEVICE_INPUTS | flags,
                   dev_meta=(dbo.data_ptr(), did.data_ptr()))


def timed(label, flags, query):
    for _ in range(5):
        run(flags)
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    kt = 0.0
    for _ in range(steps):
        run(flags)
        if query:
            kt += dict(ctx.kernel_times()).get("k_fused", 0.0)
    torch.cuda.synchronize()
    ms = (time.perf_counter() - t0) / steps * 1e3
    print(f"{label:40s} {ms:8.4f} ms/step" + (f"   k_fused {kt / steps:.4f} ms" if query else ""))
    return ms


for rep in range(2):
    timed("timing events + kernel_times()", _lib.F_TIMING, True)
    timed("timing events, no query", _lib.F_TIMING, False)
    timed("no timing", 0, False)
# host-only cost of the Python wrapper around rgc_run (ctypes + Result)
t0 = time.perf_counter()
for _ in range(steps):
    r = run(0)
times = []
for _ in range(steps):
    a = time.perf_counter()
    r = run(0)
    times.append(time.perf_counter() - a)
print(f"rgc_run call wall: min {min(times) * 1e3:.4f} median {np.median(times) * 1e3:.4f} ms")
