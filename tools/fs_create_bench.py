#!/usr/bin/env python3
"""File-creation rate in ONE directory (what bounds the CLI's writes: 5 files per micrograph
in out_dir, reference get_cliques.py:215-229), 1 vs P processes, io.open vs os.open."""
import json
import os
import sys
import tempfile
import time
from concurrent.futures import ProcessPoolExecutor

PAYLOAD = b"x" * 4096


def work(d, start, n, mode):
    t = time.perf_counter()
    for i in range(start, start + n):
        p = os.path.join(d, f"f{i:07d}.pickle")
        if mode == "io":
            with open(p, "wb") as f:
                f.write(PAYLOAD)
        else:
            fd = os.open(p, os.O_WRONLY | os.O_CREAT | os.O_TRUNC, 0o644)
            os.write(fd, PAYLOAD)
            os.close(fd)
    return time.perf_counter() - t


def main():
    n = int(sys.argv[1]) if len(sys.argv) > 1 else 20000
    base = sys.argv[2] if len(sys.argv) > 2 else None
    out = {}
    for procs in (1, 4, 16):
        for mode in ("io", "os"):
            d = tempfile.mkdtemp(dir=base)
            t0 = time.perf_counter()
            with ProcessPoolExecutor(procs) as ex:
                futs = [ex.submit(work, d, r * (n // procs), n // procs, mode) for r in range(procs)]
                [f.result() for f in futs]
            dt = time.perf_counter() - t0
            out[f"{mode}_p{procs}"] = round(n / dt)
            os.system(f"rm -rf {d}")
    print(json.dumps({"files_per_s": out, "n": n, "dir": base or tempfile.gettempdir()}))


if __name__ == "__main__":
    main()
