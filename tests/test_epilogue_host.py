"""The device ILP epilogue (rgc_device.h ``epilogue<K>``, compiled for the host through the
``rgc_test_epilogue`` hook) against the reference's semantics, restated with the live CPython
set (this interpreter is the oracle's CPython 3.10):

* consensus = first node of maximal weighted degree in networkx node-iteration order, i.e. the
  iteration order of ``set(sorted(clique))`` (get_cliques.py:182-183 -> coreviews.py
  FilterAtlas.__iter__), or graph insertion order for tiny graphs;
* degree = left-to-right f64 sum of member JIs in increasing picker order;
* conf = f32(median(scores)), w = f32(f64(conf) * median(JIs))  (get_cliques.py:186-190).

Tie-heavy inputs: duplicate / equal coordinates and JIs drawn from a small set.
"""
import itertools
import random

import numpy as np

from repic_amd import _lib


def _ref(xs, ys, ss, ids, ji, set_order, ins):
    k = len(xs)
    keys = [(xs[i], ys[i], ids[i]) for i in range(k)]
    idx = {kk: i for i, kk in enumerate(keys)}
    if set_order:
        it = [idx[u] for u in set(sorted(keys))]
    else:
        it = sorted(range(k), key=lambda i: ins[i])
    best, best_deg = None, None
    for i in it:
        d = 0
        for q in range(k):
            if q != i:
                d = d + ji[min(i, q)][max(i, q)]
        if best is None or d > best_deg:
            best, best_deg = i, d
    conf = np.float32(np.median([ss[i] for i in it]))
    eji = [ji[a][b] for a, b in itertools.combinations(range(k), 2)]
    w = np.float32(conf * np.median(eji))
    return best, it, w, conf


def test_device_epilogue_matches_reference_semantics():
    rng = random.Random(5)
    n_tie = 0
    for trial in range(6000):
        k = rng.randint(2, 8)
        set_order = trial % 4 != 0
        xs = [float(rng.choice([10, 11, 12, rng.randint(0, 4000)])) for _ in range(k)]
        ys = [float(rng.choice([10, 11, rng.randint(0, 4000)])) for _ in range(k)]
        if trial % 5 == 0:
            xs = [rng.choice([1.5, 2.25]) for _ in range(k)]
        base = rng.randint(0, 10 ** 6)
        ids = sorted(rng.sample(range(base, base + 40), k))
        ss = [rng.choice([0.5, 0.75, rng.random()]) for _ in range(k)]
        vals = [0.3125, 0.5, 0.40625, rng.uniform(0.3, 1.0)]
        ji = [[0.0] * k for _ in range(k)]
        for a in range(k):
            for b in range(a + 1, k):
                ji[a][b] = rng.choice(vals)
        ins = rng.sample(range(1 << 40), k)
        want = _ref(xs, ys, ss, ids, ji, set_order, ins)
        got = _lib.test_epilogue(xs, ys, ss, ids, ji, set_order, ins)
        degs = [sum(ji[min(i, q)][max(i, q)] for q in range(k) if q != i) for i in range(k)]
        n_tie += degs.count(max(degs)) > 1
        assert got[0] == want[0], (trial, got, want)
        assert got[1] == want[1], (trial, got, want)
        assert got[2].view(np.uint32) == want[2].view(np.uint32), (trial, got, want)
        assert got[3].view(np.uint32) == want[3].view(np.uint32), (trial, got, want)
    assert n_tie > 500
