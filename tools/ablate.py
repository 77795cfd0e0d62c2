#!/usr/bin/env python3
"""Marginal cost of each fused-kernel phase: time the ablation builds (kernel stops after
phase N) and the product build on the same batch, interleaved in one process.

  make -C repic-copy_amd/csrc ablate && python tools/ablate.py [C2] [n_mg] [rounds] [lib.so]
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

cfg_name = sys.argv[1] if len(sys.argv) > 1 else "C2"
n_mg = int(sys.argv[2]) if len(sys.argv) > 2 else 10000
rounds = int(sys.argv[3]) if len(sys.argv) > 3 else 7
# (C2_frac: C2 with 3-decimal coordinates, bench.py's by_config entry of that name)
cfg = synth.SynthConfig(**synth.CONFIGS[cfg_name.replace("_frac", "")], seed=0,
                        frac=cfg_name.endswith("_frac"))
batch = Batch.pack(cfg.k, cfg.box, synth.batch(cfg, n_mg))
libs = sorted(glob.glob(os.path.join(ROOT, "abl/*.so"))) + [_lib.LIB_PATH]
if len(sys.argv) > 4:   # one library only (per-phase PMC passes: tools/gpu_pmc_ablate.sh)
    libs = [sys.argv[4]]


class Runner:
    def __init__(self, path):
        self.lib = C.CDLL(path)
        self.lib.rgc_ctx_create.argtypes = [C.c_int, C.c_void_p, C.POINTER(C.c_void_p)]
        self.lib.rgc_run.argtypes = [C.c_void_p, C.POINTER(_lib.BatchIn), C.POINTER(_lib.BatchOut)]
        self.lib.rgc_kernel_times.argtypes = [C.c_void_p, C.c_int, C.POINTER(C.c_float),
                                              C.POINTER(C.c_char_p)]
        self.ctx = C.c_void_p()
        assert self.lib.rgc_ctx_create(0, None, C.byref(self.ctx)) == 0
        self.keep = [batch.box_off, batch.id_base, batch.x, batch.y, batch.score]

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
        # device time of the hot path: every recorded kernel except the copies (the fused
        # route: k_fused + k_fused_ties; the large route: its whole kernel pipeline)
        return sum(ms[i] for i in range(n)
                   if nm[i] not in (b"d2h", b"h2d_meta", b"d2h_stats", b"h2d"))


runners = [Runner(p) for p in libs]
for r in runners:
    r.run()
times = {p: [] for p in libs}
for _ in range(rounds):
    for p, r in zip(libs, runners):
        times[p].append(r.run())
prev = 0.0
print(f"{cfg_name} {n_mg} micrographs: device ms (median of {rounds}, interleaved)")
for p in libs:
    t = float(np.median(times[p]))
    print(f"  {os.path.basename(p):28s} {t:8.3f} ms   (+{t - prev:7.3f})")
    prev = t
