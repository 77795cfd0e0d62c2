#!/usr/bin/env python3
"""Generate golden fixtures by running the REAL reference `get_cliques` in THIS container.

This script is test infrastructure.  It is the only file that touches /root/reference,
and only at fixture-generation time (the reference never travels to the GPU box).  For
each case it:

1. materialises the input BOX directories (the EMPIAR-10017 example set committed under
   ``inputs_10017/``, or files written by our seeded generator ``repic_amd.synth`` plus
   the listed mutations),
2. runs ``repic.commands.get_cliques.main`` (reference ``get_cliques.py:72-229``) in a
   fresh process (the global ``box_id`` counter, ``common.py:23``, must start at 0),
3. unpickles the outputs it wrote (``get_cliques.py:215-229``) and stores them in a
   canonical form: constraint-matrix columns sorted by their sorted row tuple, with
   ``w``, ``conf`` and consensus coordinates permuted alongside (the raw column order is
   CPython set-iteration order).

Outputs per case: ``<case>/meta.json`` and ``<case>/data.npz`` (numeric arrays only,
loadable with ``allow_pickle=False``).  The processing order (readdir order of the first
picker's directory) is recorded, because global box ids depend on it; the parity tests
replay that order.

Usage:  python tests/golden/make_golden.py [case ...]
"""
from __future__ import annotations

import hashlib
import json
import os
import pickle
import shutil
import subprocess
import sys
import tempfile

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
REPO = os.path.dirname(os.path.dirname(HERE))
sys.path.insert(0, os.path.join(REPO, "repic-copy_amd"))
sys.path.insert(0, HERE)

from cases import CASES, materialise  # noqa: E402

REFERENCE = "/root/reference"
DRIVER = (
    "import sys, argparse\n"
    f"sys.path.insert(0, {REFERENCE!r})\n"
    "import repic.commands.get_cliques as gc\n"
    "p = argparse.ArgumentParser(); gc.add_arguments(p)\n"
    "gc.main(p.parse_args(sys.argv[1:]))\n"
)


def run_reference(in_dir, out_dir, box, flags):
    env = dict(os.environ, PYTHONDONTWRITEBYTECODE="1", MPLBACKEND="Agg")
    cmd = [sys.executable, "-c", DRIVER, in_dir, out_dir, str(box)] + list(flags)
    r = subprocess.run(cmd, cwd="/tmp", env=env, capture_output=True, text=True)
    order = [ln.strip()[4:-4] for ln in r.stdout.splitlines()
             if ln.startswith("--- ") and ln.rstrip().endswith(" ---")]
    exc = None
    if r.returncode != 0:
        last = [ln for ln in r.stderr.strip().splitlines() if ln.strip()][-1]
        exc = last.split(":")[0].strip()
    return order, exc, r


def canon_matrix(A):
    """Return (perm, canonical rows[C,k]) with columns sorted by sorted row tuple."""
    A = A.tocoo()
    C = A.shape[1]
    rows = A.row.astype(np.int64)
    cols = A.col.astype(np.int64)
    o = np.lexsort((rows, cols))
    rows, cols = rows[o], cols[o]
    k = len(rows) // C if C else 0
    R = rows.reshape(C, k) if C else np.zeros((0, 0), np.int64)
    assert C == 0 or np.all(cols.reshape(C, k) == np.arange(C)[:, None])
    perm = np.lexsort(R.T[::-1]) if C else np.zeros(0, np.int64)
    return perm, R[perm]


def collect(case, out_dir, order, exc, methods):
    multi = "--multi_out" in case.get("flags", ())
    mgs, arrays = [], {k: [] for k in (
        "rows", "w", "conf", "cx", "cy", "cid", "mo_x", "mo_y", "mo_id",
        "ap_j", "ap_x", "ap_y", "ap_w", "ap_id")}
    for base in order:
        rec = {"base": base}
        skip = os.path.join(out_dir, base + ".box")
        mat = os.path.join(out_dir, base + "_constraint_matrix.pickle")
        if os.path.exists(skip):
            rec["status"] = "skip"
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
                tsv = f.read().split("\t")
            assert w.dtype == np.float32 and conf.dtype == np.float32
            assert A.data.dtype == np.int64, A.data.dtype
            rec["coo_index_dtype"] = str(A.row.dtype)
            perm, R = canon_matrix(A)
            V, C = A.shape
            rec.update(V=int(V), C=int(C), k=int(R.shape[1]) if C else 0,
                       cc_max=int(tsv[1]), cc_cnt=int(tsv[2]))
            arrays["rows"].append(R.reshape(-1).astype(np.int32))
            arrays["w"].append(w[perm].view(np.uint32))
            arrays["conf"].append(conf[perm].view(np.uint32))
            if multi:
                assert list(coords[0]) == list(methods)
                cl = coords[1:1 + C]
                for j in perm:
                    for (x, y, i) in cl[j]:
                        arrays["mo_x"].append(np.float64(x)); arrays["mo_y"].append(np.float64(y))
                        arrays["mo_id"].append(np.int64(i))
                tail = coords[1 + C:]
                rec["n_appended"] = len(tail)
                for row in tail:
                    j = [t for t, v in enumerate(row) if v is not None]
                    assert len(j) == 1
                    x, y, wt, i = row[j[0]]
                    arrays["ap_j"].append(np.int32(j[0])); arrays["ap_x"].append(np.float64(x))
                    arrays["ap_y"].append(np.float64(y)); arrays["ap_w"].append(np.float64(wt))
                    arrays["ap_id"].append(np.int64(i))
            else:
                for j in perm:
                    x, y, i = coords[j]
                    assert type(x) is float and type(y) is float and type(i) is int
                    arrays["cx"].append(np.float64(x)); arrays["cy"].append(np.float64(y))
                    arrays["cid"].append(np.int64(i))
        else:
            rec["status"] = "crash" if exc else "missing"
        mgs.append(rec)
    out = {}
    for k, v in arrays.items():
        if not v:
            continue
        out[k] = np.concatenate(v) if isinstance(v[0], np.ndarray) else np.array(v)
    return mgs, out


def tree_digest(root):
    h = hashlib.sha256()
    for dp, dn, fn in sorted(os.walk(root)):
        dn.sort()
        for f in sorted(fn):
            p = os.path.join(dp, f)
            h.update(os.path.relpath(p, root).encode())
            with open(p, "rb") as fh:
                h.update(fh.read())
    return h.hexdigest()


def ji_vectors(n=4000, seed=7):
    """Known-answer vectors for the reference calc_jaccard (get_cliques.py:40-46)."""
    env = dict(os.environ, PYTHONDONTWRITEBYTECODE="1", MPLBACKEND="Agg")
    rng = np.random.default_rng(seed)
    B = rng.choice([1, 7, 64, 176, 180, 500], size=n)
    x = rng.normal(0, 300, size=n)
    x[: n // 2] = np.rint(x[: n // 2])
    dx = rng.normal(0, 0.4, size=n) * B
    dy = rng.normal(0, 0.4, size=n) * B
    y = rng.uniform(-1000, 5000, size=n)
    a = x + dx
    b = y + dy
    a[n // 4: n // 2] = np.rint(a[n // 4: n // 2])
    tmp = tempfile.mkdtemp()
    np.save(os.path.join(tmp, "in.npy"), np.stack([x, y, a, b, B.astype(np.float64)]))
    code = (
        "import sys, numpy as np\n"
        f"sys.path.insert(0, {REFERENCE!r})\n"
        "import repic.commands.get_cliques as gc\n"
        f"X = np.load({os.path.join(tmp, 'in.npy')!r})\n"
        "out = [gc.calc_jaccard(float(x), float(y), float(a), float(b), int(B)) for x, y, a, b, B in X.T]\n"
        f"np.save({os.path.join(tmp, 'out.npy')!r}, np.array(out, dtype=np.float64))\n"
    )
    subprocess.run([sys.executable, "-c", code], cwd="/tmp", env=env, check=True)
    out = np.load(os.path.join(tmp, "out.npy"))
    shutil.rmtree(tmp)
    os.makedirs(os.path.join(HERE, "ji_kat"), exist_ok=True)
    np.savez_compressed(os.path.join(HERE, "ji_kat", "data.npz"), x=x, y=y, a=a, b=b,
                        B=B.astype(np.int64), ji=out)


def make_case(name):
    case = CASES[name]
    tmp = tempfile.mkdtemp(prefix="golden_")
    try:
        in_dir = os.path.join(tmp, "in")
        out_dir = os.path.join(tmp, "out")
        materialise(case, in_dir)
        digest = tree_digest(in_dir)
        methods = sorted([d for d in os.listdir(in_dir) if os.path.isdir(os.path.join(in_dir, d))],
                         key=str)
        # readdir order of every picker directory (glob order inside the reference run)
        listing = {m: os.listdir(os.path.join(in_dir, m)) for m in methods}
        order, exc, r = run_reference(in_dir, out_dir, case["box"], case.get("flags", ()))
        mgs, arrays = collect(case, out_dir, order, exc, methods)
        meta = {"case": name, "box": case["box"], "flags": list(case.get("flags", ())),
                "methods": methods, "listing": listing, "order": order, "exception": exc,
                "input_sha256": digest, "micrographs": mgs}
        d = os.path.join(HERE, name)
        os.makedirs(d, exist_ok=True)
        with open(os.path.join(d, "meta.json"), "w") as f:
            json.dump(meta, f, indent=1)
        np.savez_compressed(os.path.join(d, "data.npz"), **arrays)
        n_ok = sum(m["status"] == "ok" for m in mgs)
        print(f"{name}: {len(order)} micrographs ({n_ok} ok), exception={exc}, "
              f"cliques={sum(m.get('C', 0) for m in mgs)}", flush=True)
        if exc is None and r.returncode != 0:
            print(r.stderr[-2000:])
    finally:
        shutil.rmtree(tmp)


def main(argv):
    names = argv or list(CASES)
    if not argv or "ji_kat" in argv:
        ji_vectors()
        names = [n for n in names if n != "ji_kat"]
    for n in names:
        make_case(n)


if __name__ == "__main__":
    main(sys.argv[1:])
