"""Property tests on the EXACT batches bench.py times (same generator, seed and micrograph
count per step as ``bench.DEFAULT_MG``): C2 10k, C3 4k, C4 12.5k (one eighth of the
config-4 100k batch) and C5 64.  These are too large for the oracle, so they check the
size-independent invariants of the reference's output (get_cliques.py:160-202):

* every clique has one box per picker, inside the micrograph owning its output range;
* every pair of members has JI > 0.3, recomputed in f64 with the reference op order
  (calc_jaccard, get_cliques.py:40-46);
* cliques are unique (checked as strict lexicographic order inside each micrograph's range,
  the library's deterministic column order, with a sort-based fallback);
* COO rows strictly ascending per clique and < V of the micrograph;
* 0 < w <= conf (w = f32(conf * median JI), median JI in (0.3, 1]).
"""
import os
import sys

import numpy as np
import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

CHUNK = 1 << 22


def _ji(xa, ya, xb, yb, B):
    xo = np.maximum((np.minimum(xa, xb) + B) - np.maximum(xa, xb), 0.0)
    yo = np.maximum((np.minimum(ya, yb) + B) - np.maximum(ya, yb), 0.0)
    inter = xo * yo
    return inter / (2 * B * B - inter)


def check_properties(batch, r, k, box):
    from repic_amd import _lib
    assert (r.status == _lib.OK).all()
    C = int(r.n_cliques)
    cnt, base = r.clique_cnt.astype(np.int64), r.clique_base.astype(np.int64)
    assert C == int(cnt.sum()) and (cnt > 0).all()
    o = np.argsort(base, kind="stable")
    ends = base[o] + cnt[o]
    assert base[o][0] == 0 and (base[o][1:] == ends[:-1]).all() and ends[-1] == C
    B = float(box)
    mgc = batch.box_off[::k].astype(np.int64)     # first box of each micrograph (+ total)
    for c0 in range(0, C, CHUNK):
        c1 = min(C, c0 + CHUNK)
        sl = slice(c0, c1)
        mem = r.members[sl].astype(np.int64)
        # owner micrograph of each column, from the tiled output ranges
        pos = np.searchsorted(ends, np.arange(c0, c1), side="right")
        mg = o[pos]
        assert (np.searchsorted(mgc, mem[:, 0], side="right") - 1 == mg).all()
        for p in range(k):
            lo = batch.box_off[mg * k + p]
            hi = batch.box_off[mg * k + p + 1]
            assert ((mem[:, p] >= lo) & (mem[:, p] < hi)).all()
        X, Y = batch.x[mem], batch.y[mem]
        for a in range(k):
            for b in range(a + 1, k):
                ji = _ji(X[:, a], Y[:, a], X[:, b], Y[:, b], B)
                assert (ji > 0.3).all(), (a, b)
        # unique: strictly increasing lexicographically inside a micrograph's range
        if c1 - c0 > 1:
            d = np.diff(mem, axis=0)
            first = np.argmax(d != 0, axis=1)
            inc = d[np.arange(len(d)), first] > 0
            same_mg = mg[1:] == mg[:-1]
            if not (inc | ~same_mg).all():
                for m in np.unique(mg):
                    mm = mem[mg == m]
                    assert len(np.unique(mm, axis=0)) == len(mm)
        rows = r.rows[sl]
        assert (np.diff(rows, axis=1) > 0).all()
        assert (rows[:, 0] >= 0).all() and (rows[:, -1] < r.n_vert[mg]).all()
        w, conf = r.w[sl], r.conf[sl]
        assert (w > 0).all() and (w <= conf).all()
        # conf = f32(median of member scores): inside [min, max] of the members' scores
        S = batch.score[mem]
        assert (conf >= S.min(axis=1).astype(np.float32)).all()
        assert (conf <= S.max(axis=1).astype(np.float32)).all()
    return C


@pytest.mark.gpu
@pytest.mark.parametrize("cfg_name", ["C2", "C3", "C4", "C5"])
def test_gpu_bench_step_properties(cfg_name):
    import bench
    from repic_amd import _lib, synth
    from repic_amd.pipeline import Batch
    cfg = synth.SynthConfig(**synth.CONFIGS[cfg_name], seed=0)
    n_mg = bench.DEFAULT_MG[cfg_name]
    batch = Batch.pack(cfg.k, cfg.box, synth.batch(cfg, n_mg))
    ctx = _lib.Context(0)
    try:
        r = ctx.run(batch.n_mg, cfg.k, cfg.box, batch.box_off, batch.id_base, batch.x, batch.y,
                    batch.score, _lib.F_HOST_OUTPUTS | _lib.F_MEMBERS)
        C = check_properties(batch, r, cfg.k, cfg.box)
        # lower bounds from SURVEY.md §8(d)'s per-micrograph clique counts
        want = {"C2": 500, "C3": 12000, "C4": 1200, "C5": 700000}[cfg_name]
        assert C > want * n_mg, (C, n_mg)
    finally:
        ctx.close()


def _fake_result(batch, mgs, k, box):
    """A Result-shaped namespace built by the vectorised oracle (checker self-test)."""
    from types import SimpleNamespace
    from oracle import cpu_vec
    mem, rows, w, conf, nv, cnt = [], [], [], [], [], []
    for m, mg in enumerate(mgs):
        x, y, s = (np.concatenate([t[i] for t in mg]) for i in range(3))
        o = cpu_vec.micrograph(x, y, s, [len(t[0]) for t in mg], box,
                               id_base=int(batch.id_base[m]))
        mem.append(o["members"] + int(batch.box_off[m * k]))
        rows.append(o["rows"])
        w.append(o["w"])
        conf.append(o["conf"])
        nv.append(o["V"])
        cnt.append(len(o["w"]))
    cnt = np.array(cnt, np.int64)
    return SimpleNamespace(status=np.zeros(len(mgs), np.int32), n_cliques=int(cnt.sum()),
                           clique_cnt=cnt, clique_base=np.cumsum(cnt) - cnt,
                           members=np.concatenate(mem).astype(np.int32),
                           rows=np.concatenate(rows).astype(np.int32), w=np.concatenate(w),
                           conf=np.concatenate(conf), n_vert=np.array(nv, np.int32))


def test_property_checker_accepts_oracle_and_rejects_faults():
    """CPU self-test of check_properties: the oracle's own output passes; a swapped member,
    a duplicated clique and a w > conf each fail."""
    from repic_amd import synth
    from repic_amd.pipeline import Batch
    cfg = synth.SynthConfig(**synth.CONFIGS["C2"], seed=0)
    mgs = synth.batch(cfg, 3)
    batch = Batch.pack(cfg.k, cfg.box, mgs)
    r = _fake_result(batch, mgs, cfg.k, cfg.box)
    assert check_properties(batch, r, cfg.k, cfg.box) == r.n_cliques
    for fault in ("member", "dup", "w"):
        f = _fake_result(batch, mgs, cfg.k, cfg.box)
        if fault == "member":
            f.members[5, 1] = f.members[400, 1]
        elif fault == "dup":
            f.members[7] = f.members[6]
        else:
            f.w[9] = np.nextafter(f.conf[9], np.float32(2))
        with pytest.raises(AssertionError):
            check_properties(batch, f, cfg.k, cfg.box)
