#!/usr/bin/env python3
"""Device time of the hot path on fractional-coordinate micrographs (the f64 "wide" layout of
the fused kernel) beside the same configuration with integer coordinates (the f32 layout the
bench configs take).  Library timing events, median of R runs, inputs on the host (rgc_run's
general path: the first f32 pass defers every fractional micrograph to the f64 pass).

  python tools/frac_bench.py [C2] [n_mg] [rounds]
"""
import json
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
ctx = _lib.Context(0)
out = {"config": cfg_name, "micrographs": n_mg}
for frac in (False, True):
    cfg = synth.SynthConfig(**synth.CONFIGS[cfg_name], frac=frac, seed=0)
    b = Batch.pack(cfg.k, cfg.box, synth.batch(cfg, n_mg))
    ts, parts = [], {}
    for it in range(rounds + 1):
        r = ctx.run(b.n_mg, cfg.k, cfg.box, b.box_off, b.id_base, b.x, b.y, b.score, _lib.F_TIMING)
        kt = ctx.kernel_times()
        dev = sum(ms for nm, ms in kt if nm not in ("d2h", "h2d", "h2d_meta", "d2h_stats"))
        if it:
            ts.append(dev)
            for nm, ms in kt:
                parts[nm] = parts.get(nm, 0.0) + ms / rounds
    key = "fractional" if frac else "integer"
    out[key] = {"device_ms": round(float(np.median(ts)), 4), "cliques": int(r.n_cliques),
                "parts_ms": {k: round(v, 4) for k, v in parts.items()}}
ctx.close()
print(json.dumps(out))
