"""A/B of bench.py's pipelined loop with both contexts on one stream (the default: kernels
serialised) against one stream per context (step i+1's workgroups fill step i's drain tail).
Interleaved rounds, median wall ms per step per config.  Run on the GPU box:

    python tools/streams_ab.py C2 C3 C4 C5 > gpurun_out/streams_ab.txt
"""
import argparse
import os
import statistics
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "repic-copy_amd"))

import bench  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("configs", nargs="+")
    ap.add_argument("--rounds", type=int, default=5)
    ap.add_argument("--steps", type=int, default=20)
    ap.add_argument("--depth", type=int, default=0,
                    help="also time DEPTH contexts in flight, each on its own stream")
    a = ap.parse_args()
    args = argparse.Namespace(seed=0)
    env = bench.Env(args)
    for name in a.configs:
        config, n_mg = bench.BY_CONFIG[name]
        legs = [(1, 2), (2, 2)] + ([(2, a.depth)] if a.depth > 2 else [])
        ms = {lg: [] for lg in legs}
        for _ in range(a.rounds):
            for s_, d_ in legs:
                rep, _, _ = bench.measure(args, env, config, n_mg, a.steps, 4, streams=s_,
                                          depth=d_)
                ms[(s_, d_)].append(rep["ms_per_step"])
        m1 = statistics.median(ms[(1, 2)])
        print(f"{name} {n_mg} micrographs: wall ms per step (median of {a.rounds}, interleaved)")
        for (s_, d_), v in ms.items():
            m = statistics.median(v)
            label = "one stream" if s_ == 1 else f"{d_} streams"
            print(f"  {label:14s}  {m:8.4f} ms   {v}   ({(m / m1 - 1) * 100:+.1f} %)", flush=True)


if __name__ == "__main__":
    main()
