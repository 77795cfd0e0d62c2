#!/usr/bin/env python3
"""Average PMC counter values per kernel from rocprofv3 --pmc CSVs.

  python tools/pmc_summary.py KERNEL_SUBSTR file1.csv [file2.csv ...]
"""
import csv
import sys
from collections import defaultdict

sub = sys.argv[1]
acc = defaultdict(list)
for f in sys.argv[2:]:
    for r in csv.DictReader(open(f)):
        if sub in r["Kernel_Name"]:
            acc[r["Counter_Name"]].append(float(r["Counter_Value"]))
for k, v in sorted(acc.items()):
    print(f"{k:28s} n={len(v):3d} avg={sum(v) / len(v):16.1f}")
