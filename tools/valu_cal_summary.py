#!/usr/bin/env python3
"""Fold tools/gpu_valu_cal.sh's output (plain timings + PMC passes of tools/probe/valu_cal)
into the calibration record: per (dependent?, waves/SIMD) the known VALU instruction count,
SQ_INSTS_VALU, SQ_ACTIVE_INST_VALU, GRBM_GUI_ACTIVE and the SIMD cycles per instruction.

  python tools/valu_cal_summary.py gpurun_out/TAG OUT.json
"""
import collections
import csv
import json
import os
import sys

N_XCD, N_SIMD = 8, 1024


def load(path):
    d = collections.OrderedDict()
    for r in csv.DictReader(open(path)):
        if "k_valu" not in r["Kernel_Name"]:
            continue
        key = int(r["Dispatch_Id"])
        e = d.setdefault(key, {"dep": "k_valu<true>" in r["Kernel_Name"],
                               "threads": int(r["Grid_Size"])})
        e[r["Counter_Name"]] = float(r["Counter_Value"])
    return list(d.values())


def main(src, out):
    plain = json.load(open(os.path.join(src, "plain.json")))
    a, b = load(os.path.join(src, "a.csv")), load(os.path.join(src, "b.csv"))
    cus = plain["cus"]
    per_wave = plain["iters"] * 8            # v_add_u32 in the loop of one wave
    rows = []
    for ea, eb in zip(a, b):
        waves = ea["threads"] // 64
        wps = waves // (cus * 4)
        per_xcd = ea["GRBM_GUI_ACTIVE"] / N_XCD
        insts = ea["SQ_INSTS_VALU"]
        t = [r for r in plain["runs"] if r["dep"] == int(ea["dep"]) and r["waves_per_simd"] == wps
             and r["rep"] > 0]
        wall = sum(r["wall_ms"] for r in t) / len(t)
        clk = sum(r["clock_ghz"] for r in t) / len(t)
        rows.append({
            "dependent_chain": ea["dep"], "waves_per_simd": wps, "waves": waves,
            "loop_valu_per_wave": per_wave, "SQ_INSTS_VALU": insts,
            "SQ_ACTIVE_INST_VALU": ea["SQ_ACTIVE_INST_VALU"],
            "active_equals_insts": ea["SQ_ACTIVE_INST_VALU"] == insts,
            "lanes_per_inst": eb["SQ_THREAD_CYCLES_VALU"] / insts,
            "GRBM_GUI_ACTIVE_per_xcd": per_xcd,
            "simd_cycles_per_valu_inst_grbm": per_xcd * N_SIMD / insts,
            "wall_ms": wall, "clock_ghz": clk,
            "simd_cycles_per_valu_inst_wall": wall * 1e-3 * clk * 1e9 * N_SIMD / insts,
            "valu_busy_4cyc_formula": 4 * insts / (per_xcd * N_SIMD),
            "valu_busy_2cyc_formula": 2 * insts / (per_xcd * N_SIMD),
        })
    res = {"probe": "tools/probe/valu_cal.hip", "source": src, "cus": cus, "runs": rows,
           "conclusion": "SQ_ACTIVE_INST_VALU equals SQ_INSTS_VALU (an instruction count, not "
                         "quad-cycles); with >= 2 waves per SIMD independent wave64 v_add_u32 "
                         "issue at ~2 SIMD cycles each (the 8-wave kernel including ramp and "
                         "tail: see simd_cycles_per_valu_inst_*), one wave alone at ~4-5: "
                         "valu_busy = 2 * SQ_INSTS_VALU / (GRBM_GUI_ACTIVE / 8 * 1024 SIMDs)"}
    json.dump(res, open(out, "w"), indent=1)
    for r in rows:
        print(f"dep={int(r['dependent_chain'])} wps={r['waves_per_simd']} "
              f"cyc/inst grbm={r['simd_cycles_per_valu_inst_grbm']:.2f} "
              f"wall={r['simd_cycles_per_valu_inst_wall']:.2f} busy4={r['valu_busy_4cyc_formula']:.2f} "
              f"busy2={r['valu_busy_2cyc_formula']:.2f} lanes={r['lanes_per_inst']:.1f}")


if __name__ == "__main__":
    main(*sys.argv[1:3])
