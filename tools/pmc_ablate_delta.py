#!/usr/bin/env python3
"""Per-phase marginal PMC counts from a tools/gpu_pmc_ablate.sh log (stopN builds + product).

  python tools/pmc_ablate_delta.py LOG
"""
import sys

cur, d = None, {}
for line in open(sys.argv[1]):
    if line.startswith("== librepic"):
        cur = line.split()[1]
        d[cur] = {}
    elif cur and "avg=" in line:
        d[cur][line.split()[0]] = float(line.split("avg=")[1])
def _phase(name):   # stopN; two-digit N = sub-phase N % 10 of phase N // 10 (stop21 < stop2)
    v = int(name.split("stop")[1])
    return v if v < 10 else (v // 10 - 1) + (v % 10) / 10


order = sorted((k for k in d if "stop" in k), key=_phase) + ["librepic_gc"]
keys = [k for k in ("SQ_INSTS_VALU", "SQ_INSTS_SALU", "SQ_INSTS_LDS", "SQ_WAVE_CYCLES",
                    "SQ_WAIT_ANY", "SQ_LDS_BANK_CONFLICT", "SQ_ACTIVE_INST_VALU",
                    "SQ_THREAD_CYCLES_VALU") if any(k in v for v in d.values())]
lane = "SQ_ACTIVE_INST_VALU" in keys and "SQ_THREAD_CYCLES_VALU" in keys
print(f"{'phase':22s}" + "".join(f"{k[3:]:>16s}" for k in keys) +
      ("   lane_eff" if lane else "") + "   (millions, marginal)")
prev = {}
for o in order:
    v = d[o]
    row = f"{o:22s}" + "".join(f"{(v[k] - prev.get(k, 0)) / 1e6:16.1f}" for k in keys)
    if lane:
        da = v["SQ_ACTIVE_INST_VALU"] - prev.get("SQ_ACTIVE_INST_VALU", 0)
        dt = v["SQ_THREAD_CYCLES_VALU"] - prev.get("SQ_THREAD_CYCLES_VALU", 0)
        row += f"   {dt / (64 * da) if da > 0 else float('nan'):8.2f}"
    print(row)
    prev = v
print(f"{'total':22s}" + "".join(f"{prev[k] / 1e6:16.1f}" for k in keys) +
      (f"   {prev['SQ_THREAD_CYCLES_VALU'] / (64 * prev['SQ_ACTIVE_INST_VALU']):8.2f}" if lane else ""))
