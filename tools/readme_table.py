#!/usr/bin/env python3
"""README / DESIGN measurement table from a bench.py line with by_config (one JSON line).

  python tools/readme_table.py profiles/r04z_bench_default.json
"""
import json
import sys

d = json.load(open(sys.argv[1]))
rows = [("C2", d["value"], d["ms_per_step"], d["roofline"]["kernel_ms_per_step"], d["roofline"])]
for c, e in d.get("by_config", {}).items():
    if c == "C2":
        continue
    rows.append((c, e["value"], e["ms_per_step"], e["kernel_ms"], e["roofline"]))
print("| config | micrographs/s | ms/step (kernel) | frac (B_alg / 8 TB/s) | HBM traffic / step | bound |")
print("|---|---|---|---|---|---|")
for c, v, ms, km, r in rows:
    t = r.get("traffic")
    ts = f"{t / 1e6:.0f} MB" if isinstance(t, (int, float)) else "-"
    vs = f"{v / 1e6:.2f} M" if v >= 1e6 else f"{v / 1e3:.1f} k"
    print(f"| {c} | {vs} | {ms:.3f} ({km:.3f}) | {r['frac']:.3f} | {ts} | {r.get('bound')} |")
cb = d.get("cpu_baseline")
if cb:
    print(f"\nCPU baseline (C2): {cb['value']:.2f} micrographs/s on {cb['cores']} core ({cb['kind']}); "
          f"{cb.get('parallel', {}).get('value', 0):.1f} on 16")
