#!/usr/bin/env python3
"""Calibrate the CPU baseline: the oracle's faithful per-pair loop (oracle/cpu_ref.py, what
bench.py's ``cpu_baseline`` times on the GPU box) against the REAL reference
``repic get_cliques`` on the same inputs, in THIS container (the reference never travels to
the GPU box).  Test/measurement infrastructure only.

  python tools/calibrate_cpu.py [--c2 6] > profiles/r02_cpu_calibration.json

Reference time per micrograph = its own ``<base>_runtime.tsv`` seconds column (the time of
get_cliques.py:132-229 for that micrograph, interpreter start-up excluded); the port is timed
around ``cpu_ref.micrograph(..., faithful=True)`` on the same parsed boxes and ids.
"""
from __future__ import annotations

import argparse
import glob
import json
import os
import sys
import tempfile
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "repic-copy_amd"))
sys.path.insert(0, os.path.join(ROOT, "tests", "golden"))
sys.path.insert(0, ROOT)

from make_golden import run_reference  # noqa: E402  (the one file that runs the reference)


def ref_seconds(in_dir, box):
    out = tempfile.mkdtemp(prefix="calib_ref_")
    order, exc, r = run_reference(in_dir, out, box, ())
    assert exc is None, r.stderr[-2000:]
    secs = {}
    for f in glob.glob(os.path.join(out, "*_runtime.tsv")):
        base = os.path.basename(f)[:-len("_runtime.tsv")]
        secs[base] = float(open(f).read().split("\t")[0])
    return order, secs


def port_seconds(in_dir, box, order):
    """cpu_ref faithful loop on the reference's micrographs, in its processing order, with the
    global ids the reference assigned (box_id counts every loaded box in that order)."""
    from oracle import cpu_ref
    from repic_amd.ingest import DirIndex, list_methods, parse_many
    methods = list_methods(in_dir)
    idx = DirIndex(in_dir, methods)
    secs, nid = {}, 0
    for base in order:
        paths = [os.path.join(in_dir, methods[0], base + ".box")]
        paths += [os.path.join(in_dir, m, idx.glob(m, f"*{base}*")[0]) for m in methods[1:]]
        coords = []
        for pf in parse_many(paths):
            coords.append([(float(a), float(b), float(c), nid + i)
                           for i, (a, b, c) in enumerate(zip(pf.x.tolist(), pf.y.tolist(),
                                                             list(pf.s)))])
            nid += pf.n
        t0 = time.perf_counter()
        cpu_ref.micrograph(coords, box, methods, faithful=True)
        secs[base] = time.perf_counter() - t0
    return secs


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--c2", type=int, default=6, help="C2 micrographs to time")
    args = ap.parse_args()
    from repic_amd import synth
    rows = {}
    c1 = os.path.join(ROOT, "tests", "golden", "inputs_10017")
    c2 = tempfile.mkdtemp(prefix="calib_c2_")
    synth.write_box_dirs(c2, synth.SynthConfig(**synth.CONFIGS["C2"], seed=0), args.c2)
    for name, d, box in (("C1", c1, 180), ("C2", c2, 180)):
        order, rs = ref_seconds(d, box)
        ps = port_seconds(d, box, order)
        r_tot, p_tot = sum(rs.values()), sum(ps[b] for b in rs)
        rows[name] = {"micrographs": len(rs), "reference_s": r_tot, "port_s": p_tot,
                      "reference_mg_per_s": len(rs) / r_tot, "port_mg_per_s": len(rs) / p_tot,
                      "port_over_reference_rate": r_tot / p_tot}
    print(json.dumps({"what": "cpu_ref faithful loop vs the real reference get_cliques, same "
                              "inputs, 1 core, this container (runtime.tsv seconds)",
                      "python": sys.version.split()[0], "configs": rows}, indent=1))


if __name__ == "__main__":
    main()
