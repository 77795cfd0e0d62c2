"""Helpers shared by the parity tests: load golden cases, canonicalise an output dir.

Canonical form: constraint-matrix columns sorted by their
sorted row tuple; ``w``, ``conf`` and consensus coordinates permuted alongside.  Rows
are already canonical (rank of the vertex by (x, y, id)).
"""
from __future__ import annotations

import json
import os
import pickle
import sys

import numpy as np

TESTS = os.path.dirname(os.path.abspath(__file__))
GOLDEN = os.path.join(TESTS, "golden")
sys.path.insert(0, GOLDEN)

from cases import CASES, materialise  # noqa: E402
from make_golden import canon_matrix, tree_digest  # noqa: E402


def load_case(name):
    d = os.path.join(GOLDEN, name)
    with open(os.path.join(d, "meta.json")) as f:
        meta = json.load(f)
    with np.load(os.path.join(d, "data.npz"), allow_pickle=False) as z:
        data = {k: z[k] for k in z.files}
    return meta, data


def golden_cases():
    return sorted(n for n in CASES if os.path.exists(os.path.join(GOLDEN, n, "meta.json")))


def make_inputs(name, root):
    meta, _ = load_case(name)
    in_dir = os.path.join(root, "in")
    materialise(CASES[name], in_dir)
    assert tree_digest(in_dir) == meta["input_sha256"], "fixture inputs not reproduced"
    return in_dir


def read_outputs(out_dir, meta):
    """Read an output directory in the golden's micrograph order -> (mgs, arrays)."""
    multi = "--multi_out" in meta["flags"]
    mgs = []
    acc = {k: [] for k in ("rows", "w", "conf", "cx", "cy", "cid", "mo_x", "mo_y", "mo_id",
                           "ap_j", "ap_x", "ap_y", "ap_w", "ap_id")}
    for g in meta["micrographs"]:
        base = g["base"]
        rec = {"base": base}
        mat = os.path.join(out_dir, base + "_constraint_matrix.pickle")
        if os.path.exists(os.path.join(out_dir, base + ".box")):
            rec["status"] = "skip"
            assert os.path.getsize(os.path.join(out_dir, base + ".box")) == 0
        elif os.path.exists(mat):
            rec["status"] = "ok"
            with open(mat, "rb") as f:
                A = pickle.load(f)
            with open(mat.replace("_constraint_matrix", "_weight_vector"), "rb") as f:
                w = pickle.load(f)
            with open(mat.replace("_constraint_matrix", "_consensus_confidences"), "rb") as f:
                conf = pickle.load(f)
            with open(mat.replace("_constraint_matrix", "_consensus_coords"), "rb") as f:
                coords = pickle.load(f)
            with open(mat.replace("_constraint_matrix.pickle", "_runtime.tsv")) as f:
                line = f.read()
            assert line.endswith("\n") and line.count("\n") == 1
            tsv = line.rstrip("\n").split("\t")
            float(tsv[0])
            assert type(w).__name__ == "ndarray" and w.dtype == np.float32
            assert conf.dtype == np.float32
            assert A.format == "coo" and A.data.dtype == np.int64
            assert np.all(A.data == 1)
            rec["coo_index_dtype"] = str(A.row.dtype)
            perm, R = canon_matrix(A)
            V, C = A.shape
            rec.update(V=int(V), C=int(C), k=int(R.shape[1]) if C else 0,
                       cc_max=int(tsv[1]), cc_cnt=int(tsv[2]))
            acc["rows"].append(R.reshape(-1).astype(np.int32))
            acc["w"].append(w[perm].view(np.uint32))
            acc["conf"].append(conf[perm].view(np.uint32))
            if multi:
                assert isinstance(coords, list)
                cl = coords[1:1 + C]
                for j in perm:
                    assert isinstance(cl[j], list)
                    for (x, y, i) in cl[j]:
                        assert type(x) is float and type(y) is float and type(i) is int
                        acc["mo_x"].append(x); acc["mo_y"].append(y); acc["mo_id"].append(i)
                tail = coords[1 + C:]
                rec["n_appended"] = len(tail)
                for row in tail:
                    j = [t for t, v in enumerate(row) if v is not None]
                    assert len(j) == 1
                    x, y, wt, i = row[j[0]]
                    acc["ap_j"].append(j[0]); acc["ap_x"].append(x); acc["ap_y"].append(y)
                    acc["ap_w"].append(float(wt)); acc["ap_id"].append(i)
            else:
                assert isinstance(coords, list)
                for j in perm:
                    x, y, i = coords[j]
                    assert type(x) is float and type(y) is float and type(i) is int
                    acc["cx"].append(x); acc["cy"].append(y); acc["cid"].append(i)
        else:
            rec["status"] = "absent"
        mgs.append(rec)
    dtypes = {"rows": np.int32, "w": np.uint32, "conf": np.uint32, "cx": np.float64,
              "cy": np.float64, "cid": np.int64, "mo_x": np.float64, "mo_y": np.float64,
              "mo_id": np.int64, "ap_j": np.int32, "ap_x": np.float64, "ap_y": np.float64,
              "ap_w": np.float64, "ap_id": np.int64}
    out = {}
    for k, v in acc.items():
        if v:
            out[k] = (np.concatenate(v) if isinstance(v[0], np.ndarray)
                      else np.array(v, dtype=dtypes[k]))
    return mgs, out


def assert_matches_golden(meta, data, mgs, arrays):
    """Bit-exact comparison of canonicalised outputs against the golden."""
    exc = meta["exception"]
    for g, m in zip(meta["micrographs"], mgs):
        want = g["status"]
        got = m["status"]
        if want in ("crash", "missing"):
            assert got == "absent", (g["base"], got)
            continue
        assert got == want, (g["base"], want, got)
        if want == "ok":
            for key in ("V", "C", "k", "cc_max", "cc_cnt", "coo_index_dtype"):
                assert m[key] == g[key], (g["base"], key, g[key], m[key])
            if "n_appended" in g:
                assert m["n_appended"] == g["n_appended"], g["base"]
    for key, want in data.items():
        got = arrays.get(key)
        assert got is not None, key
        assert got.dtype == want.dtype and got.shape == want.shape, (key, got.shape, want.shape)
        if got.dtype.kind == "f":
            assert np.array_equal(got.view(np.uint64), want.view(np.uint64)), key
        else:
            assert np.array_equal(got, want), key
    for key in arrays:
        assert key in data, f"unexpected output array {key}"
    return exc
