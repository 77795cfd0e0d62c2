#!/usr/bin/env python3
"""Where the time between two pipelined C2 steps goes (bench.py's loop: two contexts on one
stream, submit(i+1) before wait(i)): wall ms per step with and without F_TIMING events, and
the host time of submit() and wait().

  python tools/step_gap.py [C2] [n_mg] [steps]
"""
import json
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
dx, dy, ds = (torch.from_numpy(v).to(dev) for v in (batch.x, batch.y, batch.score))
dbo = torch.from_numpy(batch.box_off.astype(np.int32)).to(dev)
did = torch.from_numpy(np.ascontiguousarray(batch.id_base, dtype=np.int64)).to(dev)
torch.cuda.synchronize()
stream = torch.cuda.Stream(dev).cuda_stream
ctxs = [_lib.Context(0, stream), _lib.Context(0, stream)]
t_sub, t_wait = [], []


def submit(c, timing):
    t = time.perf_counter()
    c.submit(batch.n_mg, cfg.k, cfg.box, batch.box_off, batch.id_base, dx.data_ptr(),
             dy.data_ptr(), ds.data_ptr(),
             _lib.F_DEVICE_INPUTS | _lib.F_LAZY_STATS | (_lib.F_TIMING if timing else 0),
             dev_meta=(dbo.data_ptr(), did.data_ptr()))
    t_sub.append(time.perf_counter() - t)


def run(n, timing):
    submit(ctxs[0], timing)
    for i in range(n):
        if i + 1 < n:
            submit(ctxs[(i + 1) % 2], timing)
        t = time.perf_counter()
        ctxs[i % 2].wait()
        t_wait.append(time.perf_counter() - t)


out = {}
for timing in (True, False, True, False):
    run(5, timing)
    torch.cuda.synchronize()
    t_sub.clear()
    t_wait.clear()
    t0 = time.perf_counter()
    run(steps, timing)
    torch.cuda.synchronize()
    ms = (time.perf_counter() - t0) * 1e3 / steps
    key = "timing" if timing else "no_timing"
    out.setdefault(key, []).append({"ms_per_step": round(ms, 4),
                                    "submit_us": round(1e6 * float(np.median(t_sub)), 1),
                                    "wait_us": round(1e6 * float(np.median(t_wait)), 1)})
for c in ctxs:
    c.close()
print(json.dumps(out))
