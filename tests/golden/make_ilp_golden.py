"""HiGHS optima of the set-packing problems the run_ilp GPU tests solve (tests/test_ilp.py).

The GPU tests compare the device solver (rgc_ilp.hip) with HiGHS (oracle/ilp_ref.milp, relative
gap 0) on the same models.  The large ones (C3 micrographs, C5 windows with components of
>10k cliques) take seconds to minutes of CPU per solve on the GPU box, so their optima are
computed once here and committed: ``ilp_highs.npz`` maps a sha256 of each model (shape, COO
rows/cols, f32 weights) to the HiGHS objective and its packing (chosen column indices).
``tests/test_ilp.py:highs`` fails for a model that is not in the file (no live solves on the
GPU box).

    python tests/golden/make_ilp_golden.py
"""
from __future__ import annotations

import hashlib
import os
import sys

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(os.path.dirname(HERE))
OUT = os.path.join(HERE, "ilp_highs.npz")


def model_key(A, w) -> str:
    """sha256 of the model: shape, columns' sorted rows, f32 weights."""
    from scipy.sparse import csc_matrix
    A = csc_matrix(A)
    A.sort_indices()
    h = hashlib.sha256()
    h.update(np.asarray(A.shape, np.int64).tobytes())
    h.update(np.asarray(A.indptr, np.int64).tobytes())
    h.update(np.asarray(A.indices, np.int64).tobytes())
    h.update(np.asarray(w, np.float32).tobytes())
    return h.hexdigest()[:32]


def load():
    """{key: (objective, chosen column indices)} from ilp_highs.npz ({} if absent)."""
    if not os.path.exists(OUT):
        return {}
    out = {}
    with np.load(OUT, allow_pickle=False) as z:
        keys, obj, off, idx = z["keys"], z["obj"], z["off"], z["idx"]
    for i, k in enumerate(keys.tolist()):
        out[k] = (float(obj[i]), idx[off[i]:off[i + 1]])
    return out


def main():
    sys.path[:0] = [os.path.join(ROOT, "tests"), ROOT, os.path.join(ROOT, "repic-copy_amd")]
    import time

    import test_ilp
    from oracle import ilp_ref
    probs = (test_ilp.golden_problems() + test_ilp.golden_problems("syn_k4") +
             test_ilp.golden_problems("syn_k5") + test_ilp.synthetic_problems("C2", 60) +
             test_ilp.synthetic_problems("C4", 20) + test_ilp.synthetic_problems("C3", 3) +
             test_ilp._c5_window_problems(640, 2))
    keys, obj, idx, off = [], [], [], [0]
    t0 = time.time()
    for A, w in probs:
        k = model_key(A, w)
        if k in keys:
            continue
        x, o = ilp_ref.milp(A, w)
        keys.append(k)
        obj.append(o)
        sel = np.flatnonzero(x).astype(np.int32)
        idx.append(sel)
        off.append(off[-1] + len(sel))
    np.savez_compressed(OUT, keys=np.array(keys), obj=np.array(obj, np.float64),
                        off=np.array(off, np.int64), idx=np.concatenate(idx))
    print(f"{len(keys)} models, {time.time() - t0:.1f} s -> {OUT}")


if __name__ == "__main__":
    main()
