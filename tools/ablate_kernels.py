#!/usr/bin/env python3
"""Per-kernel device times (median over interleaved rounds) of every library under
abl/ and the product build on one synthetic batch.

  python tools/ablate_kernels.py C5 16 7
"""
import ctypes as C
import glob
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "repic-copy_amd"))
import numpy as np  # noqa: E402

from repic_amd import _lib, synth  # noqa: E402
from repic_amd.pipeline import Batch  # noqa: E402

cfg_name = sys.argv[1] if len(sys.argv) > 1 else "C5"
n_mg = int(sys.argv[2]) if len(sys.argv) > 2 else 16
rounds = int(sys.argv[3]) if len(sys.argv) > 3 else 7
cfg = synth.SynthConfig(**synth.CONFIGS[cfg_name], seed=0)
batch = Batch.pack(cfg.k, cfg.box, synth.batch(cfg, n_mg))
libs = sorted(glob.glob(os.path.join(ROOT, "abl/*.so"))) + [_lib.LIB_PATH]


class Runner:
    def __init__(self, path):
        self.lib = C.CDLL(path)
        self.lib.rgc_ctx_create.argtypes = [C.c_int, C.c_void_p, C.POINTER(C.c_void_p)]
        self.lib.rgc_run.argtypes = [C.c_void_p, C.POINTER(_lib.BatchIn), C.POINTER(_lib.BatchOut)]
        self.lib.rgc_kernel_times.argtypes = [C.c_void_p, C.c_int, C.POINTER(C.c_float),
                                              C.POINTER(C.c_char_p)]
        self.ctx = C.c_void_p()
        assert self.lib.rgc_ctx_create(0, None, C.byref(self.ctx)) == 0

    def run(self):
        bi = _lib.BatchIn(batch.n_mg, cfg.k, cfg.box, _lib.F_TIMING,
                          batch.box_off.ctypes.data, batch.id_base.ctypes.data,
                          C.c_void_p(batch.x.ctypes.data), C.c_void_p(batch.y.ctypes.data),
                          C.c_void_p(batch.score.ctypes.data))
        bo = _lib.BatchOut()
        assert self.lib.rgc_run(self.ctx, C.byref(bi), C.byref(bo)) == 0
        n = self.lib.rgc_kernel_times(self.ctx, 0, None, None)
        ms = (C.c_float * n)()
        nm = (C.c_char_p * n)()
        self.lib.rgc_kernel_times(self.ctx, n, ms, nm)
        out = {}
        for i in range(n):
            out[nm[i].decode()] = out.get(nm[i].decode(), 0.0) + ms[i]
        return out


runners = [Runner(p) for p in libs]
for r in runners:
    r.run()
times = {p: [] for p in libs}
for _ in range(rounds):
    for p, r in zip(libs, runners):
        times[p].append(r.run())
names = sorted({k for p in libs for t in times[p] for k in t})
print(f"{cfg_name} {n_mg} micrographs: per-kernel device ms (median of {rounds}, interleaved)")
print(f"{'kernel':18s}" + "".join(f"{os.path.basename(p)[11:24]:>14s}" for p in libs))
for k in names:
    print(f"{k:18s}" + "".join(f"{np.median([t.get(k, 0.0) for t in times[p]]):14.4f}" for p in libs))
