#!/usr/bin/env python3
"""Golden fixtures for score_detections, produced by the REAL reference in THIS container.

Test infrastructure only (the reference never travels to the GPU box).  Imports
/root/reference/repic/utils/score_detections.py (``get_segmentation_scores``,
score_detections.py:16-48) and coord_converter.py (``process_conversion``, the BOX reader the
reference's command line uses) and records, for seeded synthetic inputs:

* ``score/cases.npz`` + ``score/meta.json``: boxes (x, y, w, h, conf) of every case, its
  arguments, and the reference's (prec, rec, f1, pos_frac) as float64 bit patterns and types;
* ``score/files/*.box`` + the arrays ``process_conversion`` read from them.

  python tests/golden/make_score_golden.py
"""
from __future__ import annotations

import json
import os
import shutil
import sys
import warnings

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
OUT = os.path.join(HERE, "score")
sys.path.insert(0, "/root/reference/repic/utils")

import score_detections as ref  # noqa: E402  (reference module)
from coord_converter import Box, process_conversion  # noqa: E402


def _boxes(rng, n, W, H, size, frac=False, spread=0):
    x = rng.uniform(-spread, W - size + spread, n)
    y = rng.uniform(-spread, H - size + spread, n)
    if frac:
        x = np.round(x * 2) / 2          # exact .5 values: Python round() goes to even
        y = np.round(y * 2) / 2
    else:
        x, y = np.rint(x), np.rint(y)
    w = np.full(n, float(size))
    h = np.full(n, float(size))
    c = rng.uniform(0, 1, n)
    return np.stack([x, y, w, h, c], axis=1)


def cases():
    rng = np.random.default_rng(11)
    out = []
    out.append(("int_small", _boxes(rng, 30, 512, 512, 40), _boxes(rng, 40, 512, 512, 40), {}))
    out.append(("thresh", _boxes(rng, 30, 512, 512, 40), _boxes(rng, 40, 512, 512, 40),
                {"conf_thresh": 0.5}))
    out.append(("half_neg_edges", _boxes(rng, 40, 600, 500, 64, True, 80),
                _boxes(rng, 50, 600, 500, 64, True, 80), {}))
    out.append(("given_dims_crop", _boxes(rng, 40, 800, 800, 100, True, 50),
                _boxes(rng, 40, 800, 800, 100, True, 50), {"mrc_w": 700, "mrc_h": 650}))
    g = _boxes(rng, 20, 400, 400, 30)
    p = g.copy()
    p[:, 0] += 200.0                     # disjoint picks: tp = 0 -> prec = rec = 0, f1 = 0.0
    out.append(("disjoint", g, p, {"mrc_w": 800, "mrc_h": 400}))
    out.append(("all_below_thresh", g, _boxes(rng, 10, 400, 400, 30), {"conf_thresh": 2.0}))
    odd = _boxes(rng, 25, 300, 300, 20)
    odd[::3, 2] = 0.0                    # zero width
    odd[1::5, 3] = -7.0                  # negative height
    odd[2::4, 2] = 2.5                   # round(2.5) = 2
    out.append(("odd_sizes", odd, _boxes(rng, 25, 300, 300, 20), {}))
    out.append(("empty_gt", np.zeros((0, 5)), _boxes(rng, 10, 300, 300, 20), {}))
    for i in range(2):                   # C2-like: 4096^2, ~300 true + picks of box 180
        out.append((f"mg4096_{i}", _boxes(rng, 300, 4096, 4096, 180),
                    _boxes(rng, 330, 4096, 4096, 180), {"mrc_w": 4096, "mrc_h": 4096}))
    out.append(("mg4096_inferred", _boxes(rng, 300, 4096, 4096, 180),
                _boxes(rng, 330, 4096, 4096, 180), {"conf_thresh": 0.3}))
    return out


BOX_FILES = {
    "plain.box": "10\t20\t64\t64\t0.5\n30.5\t40\t64\t64\t0.25\n",
    "header.box": "x y w h conf\n_junk 1\n12 14 32 32 0.9\n\n15 17 32 32 0.1\n",
    "four_cols.box": "100 100 50 50\n200 210 50 50\n",
    "neg.box": "-10 -20 40 40 1e-3\n5 6 40 40 0.75\n",
}


def main():
    shutil.rmtree(OUT, ignore_errors=True)
    os.makedirs(os.path.join(OUT, "files"))
    meta, arrays = {"cases": []}, {}
    for name, g, p, kw in cases():
        gb = [Box(*r) for r in g.tolist()]
        pb = [Box(*r) for r in p.tolist()]
        with warnings.catch_warnings():
            warnings.simplefilter("ignore")
            res = ref.get_segmentation_scores(gb, pb, **kw)
        arrays[name + "_gt"] = g
        arrays[name + "_pk"] = p
        meta["cases"].append({"name": name, "kwargs": kw,
                              "result_hex": [float(v).hex() for v in res],
                              "result_type": [type(v).__name__ for v in res]})
    for fname, text in BOX_FILES.items():
        path = os.path.join(OUT, "files", fname)
        with open(path, "w") as f:
            f.write(text)
        df = list(process_conversion([path], "box", "box", out_dir=None, quiet=True).values())[0]
        if "conf" not in df.columns:
            df["conf"] = 1
        arrays["file_" + fname] = df[["x", "y", "w", "h", "conf"]].to_numpy(dtype=np.float64)
    np.savez(os.path.join(OUT, "cases.npz"), **arrays)
    with open(os.path.join(OUT, "meta.json"), "w") as f:
        json.dump(meta, f, indent=1)
    print(f"wrote {len(meta['cases'])} cases and {len(BOX_FILES)} BOX files to {OUT}")


if __name__ == "__main__":
    main()
