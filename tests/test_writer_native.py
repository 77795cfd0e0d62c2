"""Native output writer (csrc/out_write.cpp, rgc_write_outputs) vs the Python writer
(reference get_cliques.py:204-229 objects through pickle.HIGHEST_PROTOCOL).  CPU only.

* every file's bytes equal pickle.dumps of the reference-typed object with its FRAME opcodes
  removed (the only difference: framing is optional and the native writer emits none), and
  the unpickled objects are equal (values and dtypes) - including large micrographs whose
  Python pickles span several frames and ids across every pickle int encoding
* runtime.tsv text equals the Python writer's (CPython str(float) for the seconds)
* a write error is reported as OSError naming the micrograph
"""
import os
import pickle
import pickletools

import numpy as np
import pytest

from repic_amd import writers


def _unframed(b: bytes) -> bytes:
    cut = [pos for op, arg, pos in pickletools.genops(b) if op.name == "FRAME"]
    out, last = [], 0
    for p in cut:
        out.append(b[last:p])
        last = p + 9
    out.append(b[last:])
    return b"".join(out)


def _group(rng, sizes, k):
    C = int(sum(sizes))
    V = 3 * max(sizes) * k + 5
    items = [(f"mg_{i:04d}", n, V, int(rng.integers(1, 99)), int(rng.integers(1, 999)),
              float(rng.choice([0.25, 1e-5, 3.0, 123.456789, 7e-3])), None)
             for i, n in enumerate(sizes)]
    w = rng.random(C).astype(np.float32)
    conf = rng.random(C).astype(np.float32)
    rows = np.sort(rng.integers(0, V, (C, k)), axis=1).astype(np.int32)
    cx = np.round(rng.random(C) * 4096, int(rng.integers(0, 4)))
    cy = rng.random(C) * 4096
    cid = rng.choice(np.array([0, 200, 256, 40000, 65536, 2**31 - 1, 2**31, 3 * 10**12]),
                     C).astype(np.int64) + rng.integers(0, 3, C)
    return items, w, conf, rows, cx, cy, cid


@pytest.mark.parametrize("k,sizes", [(3, [1, 2, 535, 7]), (5, [1583, 3]), (8, [12000, 1])])
def test_native_writer_matches_python(tmp_path, k, sizes):
    fmt = writers.native_format()
    assert fmt is not None, "native writer self-test failed for the installed numpy/scipy"
    rng = np.random.default_rng(k)
    items, w, conf, rows, cx, cy, cid = _group(rng, sizes, k)
    a, b = tmp_path / "native", tmp_path / "python"
    a.mkdir()
    b.mkdir()
    writers.write_group_native(fmt, str(a), items, w, conf, rows, cx, cy, cid)
    writers.write_group(str(b), items, w, conf, rows, cx, cy, cid)
    names = sorted(os.listdir(b))
    assert names == sorted(os.listdir(a)) and len(names) == 5 * len(sizes)
    for f in names:
        na, nb = (a / f).read_bytes(), (b / f).read_bytes()
        if f.endswith(".tsv"):
            assert na == nb, f
            continue
        assert na == _unframed(nb), f
        oa, ob = pickle.loads(na), pickle.loads(nb)
        assert type(oa) is type(ob)
        if isinstance(ob, np.ndarray):
            assert oa.dtype == ob.dtype and np.array_equal(oa.view(np.uint32), ob.view(np.uint32))
        elif isinstance(ob, list):
            assert oa == ob and all(type(x) is tuple for x in oa)
        else:
            assert oa.shape == ob.shape
            for u, v in ((oa.row, ob.row), (oa.col, ob.col), (oa.data, ob.data)):
                assert u.dtype == v.dtype and np.array_equal(u, v)


def test_native_writer_skip_and_error(tmp_path):
    fmt = writers.native_format()
    rng = np.random.default_rng(1)
    items, w, conf, rows, cx, cy, cid = _group(rng, [4, 6], 3)
    items = [("skipped", -1, 0, 0, 0, 0.0, None)] + items
    writers.write_group_native(fmt, str(tmp_path), items, w, conf, rows, cx, cy, cid)
    assert (tmp_path / "skipped.box").read_bytes() == b""
    assert len(os.listdir(tmp_path)) == 11
    with pytest.raises(OSError) as ei:
        writers.write_group_native(fmt, str(tmp_path / "missing_dir"), items[1:], w, conf, rows,
                                   cx, cy, cid)
    assert "mg_0000" in str(ei.value)
