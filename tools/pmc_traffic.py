#!/usr/bin/env python3
"""Per-kernel HBM traffic and issue/stall counters from rocprofv3 PMC CSVs (one counter group
per pass: FETCH_SIZE and WRITE_SIZE separately, per MI355X_MICROARCH.md §HBM), folded into
one JSON that bench.py matches to its own library build (sha256) and workload (config).

MI355X_MICROARCH.md §HBM: FETCH_SIZE / WRITE_SIZE are in KiB (x1024 -> bytes).  FETCH_SIZE
reads exactly 1/2 of a wide (16 B/lane) coalesced streaming read on gfx950; our kernels read
4-8 B per lane in gathers, a width the guide leaves uncalibrated, so the fetch side is
reported raw (x1024) and flagged, not doubled.

SQ_WAVE_CYCLES / SQ_WAIT_* count quad-cycles (guide); SQ_ACTIVE_INST_VALU does NOT: on gfx950
it equals SQ_INSTS_VALU, an instruction count, and a wave64 VALU instruction takes 2 SIMD
cycles when >= 2 waves per SIMD are ready (calibrated by tools/probe/valu_cal.hip,
profiles/r05a_valu_calibration.json: the saturated 8-waves/SIMD probe reads 0.85 with the
factor 2 and an impossible 1.70 with the factor 4 used until round 4).  GRBM_GUI_ACTIVE is
summed over the 8 XCDs.  Derived per kernel:
  valu_busy  = 2 * SQ_ACTIVE_INST_VALU / (GRBM_GUI_ACTIVE / 8 * 1024 SIMDs)
  wait_any   = SQ_WAIT_ANY / SQ_WAVE_CYCLES          (share of resident wave time stalled)
  waves_per_cu = 4 * SQ_WAVE_CYCLES / (GRBM_GUI_ACTIVE / 8 * 256 CUs)
  lane_eff   = SQ_THREAD_CYCLES_VALU / (64 * SQ_ACTIVE_INST_VALU)   (when collected)

  python tools/pmc_traffic.py DIR LIB.so OUT.json [CONFIG] [STEPS]
    DIR holds fetch.csv / write.csv (required) and any of sqa.csv sqb.csv grbm.csv lane.csv;
    STEPS = hot-path steps the profiled command ran (bench warmup + steps): "step_traffic" is
    then every kernel's bytes summed over the run / STEPS (the multi-kernel route's roofline)
  python tools/pmc_traffic.py FETCH.csv WRITE.csv LIB.so OUT.json [CONFIG]   (traffic only)
"""
import csv
import hashlib
import json
import os
import re
import sys
from collections import defaultdict

# rocprof kernel name -> bench.py event name
NAMES = [(r"k5_cliques<\d+, true>", "k5_cliques_fill"), (r"k5_cliques<\d+, false>", "k5_cliques_count"),
         (r"k2_pairs<true>", "k2_pairs_fill"), (r"k2_pairs<false>", "k2_pairs_count"),
         (r"k_fused<", "k_fused"), (r"k7_rows<", "k7_rows"), (r"rgc::(k\w+)", None),
         (r"rgc::(scan_\w+)\(", None)]
N_XCD, N_CU, N_SIMD = 8, 256, 1024
VALU_CYCLES = 2     # SIMD cycles per wave64 VALU instruction (profiles/r05a_valu_calibration.json)


def event_name(kname):
    for pat, name in NAMES:
        m = re.search(pat, kname)
        if m:
            return name or m.group(1)
    return None


def per_kernel(path, counters=None, total=False):
    """{event name: {counter: mean value per launch}} of one CSV (total=True: the sum over
    launches and the launch count instead)."""
    acc = defaultdict(lambda: defaultdict(list))
    for r in csv.DictReader(open(path)):
        n = event_name(r["Kernel_Name"])
        if n and (counters is None or r["Counter_Name"] in counters):
            acc[n][r["Counter_Name"]].append(float(r["Counter_Value"]))
    if total:
        return {k: {c: (sum(v), len(v)) for c, v in d.items()} for k, d in acc.items()}
    return {k: {c: sum(v) / len(v) for c, v in d.items()} for k, d in acc.items()}


def derive(c):
    out = {}
    g = c.get("GRBM_GUI_ACTIVE")
    if g:
        per_xcd = g / N_XCD
        if "SQ_ACTIVE_INST_VALU" in c:
            out["valu_busy"] = VALU_CYCLES * c["SQ_ACTIVE_INST_VALU"] / (per_xcd * N_SIMD)
        if "SQ_WAVE_CYCLES" in c:
            out["waves_per_cu"] = 4 * c["SQ_WAVE_CYCLES"] / (per_xcd * N_CU)
    if c.get("SQ_WAVE_CYCLES") and "SQ_WAIT_ANY" in c:
        out["wait_any"] = c["SQ_WAIT_ANY"] / c["SQ_WAVE_CYCLES"]
    if c.get("SQ_ACTIVE_INST_VALU") and "SQ_THREAD_CYCLES_VALU" in c:
        out["lane_eff"] = c["SQ_THREAD_CYCLES_VALU"] / (64 * c["SQ_ACTIVE_INST_VALU"])
    return out


def main(argv):
    if os.path.isdir(argv[0]):
        d, lib, out = argv[0], argv[1], argv[2]
        config = argv[3] if len(argv) > 3 else "C2"
        steps = int(argv[4]) if len(argv) > 4 else None
        entry = argv[5] if len(argv) > 5 else config
        fetch, write = os.path.join(d, "fetch.csv"), os.path.join(d, "write.csv")
        extra = [os.path.join(d, f"{n}.csv") for n in ("sqa", "sqb", "grbm", "lane", "occ", "lds")]
        extra = [p for p in extra if os.path.exists(p)]
    else:
        fetch, write, lib, out = argv[:4]
        config = argv[4] if len(argv) > 4 else "C2"
        entry = config
        steps = None
        extra = []
    f = per_kernel(fetch, {"FETCH_SIZE"})
    w = per_kernel(write, {"WRITE_SIZE"})
    cnt = defaultdict(dict)
    for p in extra:
        for k, d in per_kernel(p).items():
            cnt[k].update(d)
    sha = hashlib.sha256(open(lib, "rb").read()).hexdigest()
    kernels = {}
    for k in sorted(set(f) | set(w)):
        fb = f.get(k, {}).get("FETCH_SIZE")
        wb = w.get(k, {}).get("WRITE_SIZE")
        e = {"fetch": None if fb is None else fb * 1024.0,
             "write": None if wb is None else wb * 1024.0}
        e["traffic"] = (e["fetch"] or 0.0) + (e["write"] or 0.0)
        if k in cnt:
            e["counters"] = cnt[k]
            e["derived"] = derive(cnt[k])
        kernels[k] = e
    # entry: the bench.py by_config name (the batch size: C4_100k is C4 at 100k micrographs)
    res = {"lib_sha256": sha, "config": config, "entry": entry, "unit": "bytes per launch",
           "note": "FETCH_SIZE*1024 (raw, uncalibrated width) + WRITE_SIZE*1024; counters are "
                   "per-launch means, derived ratios per tools/pmc_traffic.py",
           "kernels": kernels}
    if steps:
        ft = per_kernel(fetch, {"FETCH_SIZE"}, total=True)
        wt = per_kernel(write, {"WRITE_SIZE"}, total=True)
        tot = sum(v["FETCH_SIZE"][0] for v in ft.values()) + \
            sum(v["WRITE_SIZE"][0] for v in wt.values())
        res["steps"] = steps
        res["step_traffic"] = tot * 1024.0 / steps
        res["launches"] = {k: v["FETCH_SIZE"][1] for k, v in ft.items()}
    json.dump(res, open(out, "w"), indent=1)
    for k, v in sorted(kernels.items(), key=lambda kv: -kv[1]["traffic"]):
        dv = " ".join(f"{a}={b:.3f}" for a, b in v.get("derived", {}).items())
        print(f"{k:22s} fetch={v['fetch'] or 0:14.0f} write={v['write'] or 0:14.0f} {dv}")


if __name__ == "__main__":
    main(sys.argv[1:])
