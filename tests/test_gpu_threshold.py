"""The JI > 0.3 edge decision on the device (reference get_cliques.py:40-46, 64-65, 138).

The kernels decide ``I > (6/13) B^2`` without a division and evaluate the reference quotient
``I / ((2 B^2) - I)`` only inside a 2^-40 band around the threshold; the f32-coordinate
layout adds a conservative ``|dx|, |dy| >= 0.54 B`` reject.  These tests feed pairs to both
routes (fused f32 / f64 layouts and the multi-kernel path) through the C-ABI's RGC_F_EDGES
hook and require the reference's edge decisions and bit-identical f64 JIs:

* the 4000 ``calc_jaccard`` known-answer vectors produced by the reference itself
  (tests/golden/ji_kat, non-integer and negative coordinates, B in {1, 7, 64, 176, 180, 500});
* every integer offset (dx, dy) for B in {13, 26, 180}: exact ties I = 6 B^2 / 13 (JI
  rounds to the f64 0.3, so no edge) and their +-1 pixel neighbours;
* non-integer offsets stepped in single ulps (and 2^-m relative) around the threshold.

Each pair is one micrograph of two pickers with one box each.
"""
import os

import numpy as np
import pytest

pytestmark = pytest.mark.gpu

KAT = os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden", "ji_kat", "data.npz")


def _ref_ji(x, y, a, b, B):
    """calc_jaccard's f64 op order (same as oracle/cpu_ref.jaccard, vectorised)."""
    xo = np.maximum((np.minimum(x, a) + B) - np.maximum(x, a), 0.0)
    yo = np.maximum((np.minimum(y, b) + B) - np.maximum(y, b), 0.0)
    inter = xo * yo
    return inter / (np.float64(2 * B * B) - inter)


def _device_edges(x, y, a, b, B, no_fused):
    """One micrograph per pair -> {pair index: device JI} of the pairs the device keeps."""
    from repic_amd import _lib
    n = len(x)
    X = np.stack([x, a], axis=1).reshape(-1)
    Y = np.stack([y, b], axis=1).reshape(-1)
    S = np.full(2 * n, 0.5)
    box_off = np.arange(2 * n + 1, dtype=np.int64)
    id_base = np.arange(0, 2 * n, 2, dtype=np.int64)
    fl = _lib.F_HOST_OUTPUTS | _lib.F_EDGES | (_lib.F_NO_FUSED if no_fused else 0)
    ctx = _lib.Context(0)
    r = ctx.run(n, 2, B, box_off, id_base, X, Y, S, fl)
    u, v, ji = ctx.last_edges()
    st = np.array(r.status)
    ctx.close()
    assert len(u) == int(r.n_edges)
    assert (u % 2 == 0).all() and (v == u + 1).all()
    m = u // 2
    assert len(np.unique(m)) == len(m)
    # status agrees with the edge list: OK (the edge is the 2-clique) or NO_EDGES
    want = np.full(n, _lib.NO_EDGES)
    want[m] = _lib.OK
    assert np.array_equal(st, want)
    return dict(zip(m.tolist(), ji))


def _check(x, y, a, b, B, ji_want=None):
    x, y, a, b = (np.ascontiguousarray(v, dtype=np.float64) for v in (x, y, a, b))
    ji_ref = _ref_ji(x, y, a, b, B)
    if ji_want is not None:
        assert np.array_equal(ji_ref.view(np.uint64), ji_want.view(np.uint64))
    edge = (np.abs(x - a) <= B) & (ji_ref > 0.3)            # get_cliques.py:64-65
    for no_fused in (False, True):
        got = _device_edges(x, y, a, b, B, no_fused)
        assert sorted(got) == np.nonzero(edge)[0].tolist(), ("no_fused", no_fused)
        idx = np.array(sorted(got), dtype=np.int64)
        dev = np.array([got[i] for i in idx])
        assert np.array_equal(dev.view(np.uint64), ji_ref[idx].view(np.uint64))
    return int(edge.sum())


def test_device_edges_match_reference_kat():
    with np.load(KAT) as z:
        x, y, a, b, B, ji = (z[k] for k in ("x", "y", "a", "b", "B", "ji"))
    n_edges = 0
    for bv in np.unique(B):
        s = B == bv
        n_edges += _check(x[s], y[s], a[s], b[s], int(bv), ji[s])
    assert n_edges > 1000


@pytest.mark.parametrize("B", [13, 26, 180])
def test_device_edges_integer_grid_exact_ties(B):
    """Every integer offset: f32 layout, exact ties at I = 6 B^2 / 13 included."""
    d = np.arange(-B - 1, B + 2, dtype=np.float64)
    dx, dy = (v.reshape(-1) for v in np.meshgrid(d, d))
    x0, y0 = 1000.0, 2000.0
    a, b = x0 + dx, y0 + dy
    x, y = np.full_like(a, x0), np.full_like(b, y0)
    inter = np.maximum(B - np.abs(dx), 0) * np.maximum(B - np.abs(dy), 0)
    ties = 13 * inter == 6 * B * B
    if B % 13 == 0:
        assert ties.sum() >= 4   # JI == 0.3 exactly (f64): must NOT be an edge
        assert not (_ref_ji(x, y, a, b, B)[ties] > 0.3).any()
    _check(x, y, a, b, B)


@pytest.mark.parametrize("B", [13, 26, 176, 180])
def test_device_edges_ulp_steps_around_threshold(B):
    """Non-integer coordinates (f64 layout): the y offset stepped in single ulps and in
    2^-m relative steps around the threshold offset 7B/13 (and along the I = 6B^2/13 curve
    for random x overlaps), on both sides of the 2^-40 band."""
    rng = np.random.default_rng(B)
    t = 7.0 * B / 13.0
    offs = [t]
    for j in range(1, 65):
        offs += [np.nextafter(offs[-1], np.inf)]
    lo = [t]
    for j in range(1, 65):
        lo += [np.nextafter(lo[-1], -np.inf)]
    offs = offs + lo[1:]
    offs += [t * (1 + s * 2.0 ** -m) for m in range(20, 53) for s in (-1, 1)]
    offs = np.array(offs)
    # random x overlaps xo in (0.55 B, B); y offset from the threshold curve yo = I* / xo
    xo = rng.uniform(0.55 * B, B, 200)
    yo = (6.0 * B * B / 13.0) / xo
    jit = rng.integers(-40, 41, 200).astype(np.float64)
    dy2 = (B - yo) * (1 + jit * 2.0 ** -45)
    dx = np.concatenate([np.zeros(len(offs)), B - xo])
    dy = np.concatenate([offs, dy2])
    x0, y0 = 512.25, 700.5
    sign = np.where(rng.random(len(dx)) < 0.5, -1.0, 1.0)
    a, b = x0 + sign * dx, y0 - sign * dy
    x, y = np.full_like(a, x0), np.full_like(b, y0)
    n = _check(x, y, a, b, B)
    assert 0 < n < len(x)
