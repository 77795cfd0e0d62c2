#!/usr/bin/env python3
"""Per-kernel HBM traffic from rocprofv3 PMC CSVs (separate FETCH_SIZE / WRITE_SIZE passes).

MI355X_MICROARCH.md §HBM: FETCH_SIZE / WRITE_SIZE are in KiB (x1024 -> bytes).  FETCH_SIZE
reads exactly 1/2 of a wide (16 B/lane) coalesced streaming read on gfx950; our kernels read
4-8 B per lane in gathers, a width the guide leaves uncalibrated, so the fetch side is
reported raw (x1024) and flagged, not doubled.

  python tools/pmc_traffic.py FETCH.csv WRITE.csv LIB.so OUT.json [CONFIG]

CONFIG (default C2) is recorded so bench.py only quotes traffic measured on its own workload.
"""
import csv
import hashlib
import json
import re
import sys
from collections import defaultdict

# rocprof kernel name -> bench.py event name
NAMES = [(r"k5_cliques<\d+, true>", "k5_cliques_fill"), (r"k5_cliques<\d+, false>", "k5_cliques_count"),
         (r"k2_pairs<true>", "k2_pairs_fill"), (r"k2_pairs<false>", "k2_pairs_count"),
         (r"k_fused<", "k_fused"), (r"k7_rows<", "k7_rows"), (r"rgc::(k\w+)\(", None),
         (r"rgc::(scan_\w+)\(", None)]


def event_name(kname):
    for pat, name in NAMES:
        m = re.search(pat, kname)
        if m:
            return name or m.group(1)
    return None


def per_kernel(path, counter):
    acc = defaultdict(list)
    for r in csv.DictReader(open(path)):
        if r["Counter_Name"] != counter:
            continue
        n = event_name(r["Kernel_Name"])
        if n:
            acc[n].append(float(r["Counter_Value"]) * 1024.0)
    return {k: sum(v) / len(v) for k, v in acc.items()}


def main(fetch, write, lib, out, config="C2"):
    f, w = per_kernel(fetch, "FETCH_SIZE"), per_kernel(write, "WRITE_SIZE")
    sha = hashlib.sha256(open(lib, "rb").read()).hexdigest()
    res = {"lib_sha256": sha, "config": config, "unit": "bytes per launch",
           "note": "FETCH_SIZE*1024 (raw, uncalibrated width) + WRITE_SIZE*1024",
           "kernels": {k: {"fetch": f.get(k), "write": w.get(k),
                           "traffic": (f.get(k) or 0.0) + (w.get(k) or 0.0)}
                       for k in sorted(set(f) | set(w))}}
    json.dump(res, open(out, "w"), indent=1)
    for k, v in sorted(res["kernels"].items(), key=lambda kv: -kv[1]["traffic"]):
        print(f"{k:22s} fetch={v['fetch'] or 0:14.0f} write={v['write'] or 0:14.0f}")


if __name__ == "__main__":
    main(*sys.argv[1:6])
