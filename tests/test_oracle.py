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
