"""Pin the CPU oracle against the reference's own outputs (golden fixtures).

The fixtures were produced by running reference ``get_cliques`` in the development
container (``tests/golden/make_golden.py``); this file checks the restatement in
``oracle/cpu_ref.py`` reproduces them bit-exactly (canonical column order).
"""
import builtins
import os

import numpy as np
import pytest

from golden_util import assert_matches_golden, golden_cases, load_case, make_inputs, read_outputs
from oracle import cpu_ref

FAST = [c for c in golden_cases() if not c.startswith("c1_10017") and c not in ("syn_k4",)]
SLOW = [c for c in golden_cases() if c not in FAST]


def _run(name, tmp_path, faithful=False):
    meta, data = load_case(name)
    in_dir = make_inputs(name, str(tmp_path))
    out_dir = os.path.join(str(tmp_path), "out")
    exc = None
    try:
        cpu_ref.run_dir(in_dir, out_dir, meta["box"], get_cc="--get_cc" in meta["flags"],
                        multi_out="--multi_out" in meta["flags"], listing=meta["listing"],
                        faithful=faithful)
    except Exception as e:  # noqa: BLE001 - exception class is part of the contract
        exc = e
    if meta["exception"]:
        assert exc is not None, "reference crashed, oracle did not"
        assert isinstance(exc, getattr(builtins, meta["exception"])), (meta["exception"], exc)
    else:
        assert exc is None, exc
    mgs, arrays = read_outputs(out_dir, meta)
    assert_matches_golden(meta, data, mgs, arrays)


@pytest.mark.parametrize("name", FAST)
def test_oracle_matches_reference(name, tmp_path):
    _run(name, tmp_path)


@pytest.mark.parametrize("name", SLOW)
def test_oracle_matches_reference_large(name, tmp_path):
    _run(name, tmp_path)


def test_oracle_faithful_loop_matches(tmp_path):
    """The timed (per-pair numpy) baseline path gives the same outputs."""
    _run("skips", tmp_path, faithful=True)


def test_jaccard_known_answers():
    """calc_jaccard KAT vectors (reference get_cliques.py:40-46), f64 bit-exact."""
    with np.load(os.path.join(os.path.dirname(__file__), "golden", "ji_kat", "data.npz")) as z:
        x, y, a, b, B, ji = (z[k] for k in ("x", "y", "a", "b", "B", "ji"))
    got = np.array([cpu_ref.jaccard(float(x[i]), float(y[i]), float(a[i]), float(b[i]), int(B[i]))
                    for i in range(len(x))])
    assert np.array_equal(got.view(np.uint64), ji.view(np.uint64))
    # vectorised form, same op order
    xo = np.maximum((np.minimum(x, a) + B) - np.maximum(x, a), 0.0)
    yo = np.maximum((np.minimum(y, b) + B) - np.maximum(y, b), 0.0)
    inter = xo * yo
    vec = inter / ((2 * B.astype(np.float64) ** 2) - inter)
    assert np.array_equal(vec.view(np.uint64), ji.view(np.uint64))


def _vec_vs_ref(mg, box, get_cc=False, idb=1000):
    """oracle/cpu_vec.py (full-size checker) against oracle/cpu_ref.py, bit-exact."""
    from oracle import cpu_vec
    k = len(mg)
    coords, nid = [], idb
    for (x, y, s) in mg:
        coords.append([(float(a), float(b), float(c), nid + i)
                       for i, (a, b, c) in enumerate(zip(x, y, s))])
        nid += len(x)
    o = cpu_ref.micrograph(coords, box, [f"p{i}" for i in range(k)], get_cc=get_cc)
    X, Y, S = (np.concatenate([m[i] for m in mg]) for i in range(3))
    v = cpu_vec.micrograph(X, Y, S, [len(m[0]) for m in mg], box, get_cc=get_cc, id_base=idb)
    A = o["A"].tocoo()
    C = A.shape[1]
    orows = np.sort(A.row[np.argsort(A.col, kind="stable")].reshape(C, k), axis=1)
    po, pv = np.lexsort(orows.T[::-1]), np.lexsort(v["rows"].T[::-1])
    assert (o["cc_max"], o["cc_cnt"]) == (v["cc_max"], v["cc_cnt"])
    assert np.array_equal(orows[po], v["rows"][pv])
    assert np.array_equal(o["w"][po].view(np.uint32), v["w"][pv].view(np.uint32))
    assert np.array_equal(o["conf"][po].view(np.uint32), v["conf"][pv].view(np.uint32))
    got = [(float(X[g]), float(Y[g]), idb + int(g)) for g in v["consensus"][pv]]
    assert got == [o["consensus"][i] for i in po]
    return C


@pytest.mark.parametrize("cfg_name,n,extra", [
    ("C2", 3, {}), ("C2", 2, {"frac": True, "dup": 0.2}), ("C4", 2, {"logit": (1,)}),
    ("C3", 1, {})])
def test_vectorised_oracle_matches_scalar(cfg_name, n, extra):
    from repic_amd import synth
    from repic_amd.ingest import sigmoid
    cfg = synth.SynthConfig(**{**synth.CONFIGS[cfg_name], **extra}, seed=5)
    for mg in synth.batch(cfg, n):
        mg = [(x, y, sigmoid(s) if s.min() < 0 else s) for (x, y, s) in mg]
        assert _vec_vs_ref(mg, cfg.box) > 0
        _vec_vs_ref(mg, cfg.box, get_cc=True)


def test_vectorised_oracle_matches_scalar_c5_window():
    """A 768^2 window of a full C5 micrograph (k = 8, duplicates -> degree ties)."""
    from repic_amd import synth
    cfg = synth.SynthConfig(**synth.CONFIGS["C5"], seed=0)
    mg = synth.batch(cfg, 1)[0]
    win = []
    for (x, y, s) in mg:
        m = (x >= 1000) & (x < 1768) & (y >= 1000) & (y < 1768)
        win.append((x[m], y[m], s[m]))
    assert _vec_vs_ref(win, cfg.box) > 5000
