#!/usr/bin/env python3
"""File-to-file throughput of the drop-in CLI (what a user of ``repic get_cliques`` runs):
BOX text in, the five per-micrograph output files out, on one GPU.

  python tools/file_bench.py [--config C2] [--n_mg 10000] [--threads T] [--workdir DIR]
  python tools/file_bench.py --index-only --n_mg 100000 --tiny   # §8(f)3 directory index

Writes the synthetic BOX directories first (seeded SURVEY.md §8(d) generator, not timed),
then times ``repic_amd.commands.get_cliques.main`` end to end (directory index + parse +
device + pickles/TSV) and reports its phases.  Prints one JSON line.  Never the bench
``value``: the reference's only published number is of this kind (README.md:60), so it is
reported beside the HBM-resident headline.
"""
from __future__ import annotations

import argparse
import json
import os
import shutil
import sys
import tempfile
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "repic-copy_amd"))


def _write_inputs(root, cfg, n_mg, threads):
    """Write the BOX dirs with a process pool (generation is not what is measured)."""
    from concurrent.futures import ProcessPoolExecutor

    from repic_amd import synth
    step = max(1, n_mg // (4 * threads))
    with ProcessPoolExecutor(threads) as ex:
        futs = [ex.submit(synth.write_box_dirs, root, cfg, min(step, n_mg - s), None, s)
                for s in range(0, n_mg, step)]
        for f in futs:
            f.result()


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--config", default="C2")
    ap.add_argument("--n_mg", type=int, default=10000)
    ap.add_argument("--threads", type=int, default=None)
    ap.add_argument("--workdir", default=None)
    ap.add_argument("--tiny", action="store_true",
                    help="4 true particles per micrograph: directory-index / per-file scale test")
    ap.add_argument("--index-only", action="store_true",
                    help="time the directory index and micrograph pairing only (no GPU)")
    args = ap.parse_args()

    from repic_amd import synth
    threads = args.threads or min(16, len(os.sched_getaffinity(0)))
    kw = dict(synth.CONFIGS[args.config])
    if args.tiny:
        kw["n_true"] = 4
    cfg = synth.SynthConfig(**kw, seed=0)
    work = tempfile.mkdtemp(prefix="rgc_f2f_", dir=args.workdir)
    out = {"metric": "file-to-file micrographs/s (repic get_cliques CLI, 1 GPU)",
           "config": args.config + (" tiny (n_true=4)" if args.tiny else ""),
           "n_mg": args.n_mg, "k": cfg.k, "threads": threads}
    try:
        in_dir = os.path.join(work, "in")
        t0 = time.perf_counter()
        _write_inputs(in_dir, cfg, args.n_mg, threads)
        out["gen_s"] = time.perf_counter() - t0
        out["input_bytes"] = sum(e.stat().st_size for p in os.scandir(in_dir)
                                 for e in os.scandir(p.path))

        from repic_amd.ingest import DirIndex, list_methods, micrograph_names
        t0 = time.perf_counter()
        methods = list_methods(in_dir)
        index = DirIndex(in_dir, methods)
        names = micrograph_names(index, methods)
        for n in names:   # the reference's per-micrograph partner globs (get_cliques.py:121)
            base = n.replace(".box", "")
            for m in methods[1:]:
                assert len(index.glob(m, f"*{base}*")) == 1
        out["index_s"] = time.perf_counter() - t0
        out["index_us_per_mg"] = out["index_s"] / args.n_mg * 1e6
        if args.index_only:
            print(json.dumps(out), flush=True)
            return

        import repic_amd.commands.get_cliques as gc
        p = argparse.ArgumentParser()
        gc.add_arguments(p)
        cli = p.parse_args([in_dir, os.path.join(work, "out"), str(cfg.box),
                            "--threads", str(threads)])
        # warm the device context / kernels on a tiny copy first (not timed)
        warm = os.path.join(work, "warm")
        synth.write_box_dirs(warm, cfg, 2)
        wa = p.parse_args([warm, os.path.join(work, "warm_out"), str(cfg.box)])
        with open(os.devnull, "w") as dn:
            so = sys.stdout
            sys.stdout = dn
            try:
                gc.main(wa)
                t0 = time.perf_counter()
                gc.main(cli)
                wall = time.perf_counter() - t0
            finally:
                sys.stdout = so
        st = dict(gc.LAST_RUN)
        out.update({"value": args.n_mg / wall, "unit": "micrographs/s", "wall_s": wall,
                    "phases_s": {k_: round(v, 4) for k_, v in st.items() if k_.endswith("_s")},
                    "cliques": st.get("cliques"), "edges": st.get("edges"),
                    "output_files": len(os.listdir(os.path.join(work, "out")))})
        print(json.dumps(out), flush=True)
    finally:
        shutil.rmtree(work, ignore_errors=True)


if __name__ == "__main__":
    main()
