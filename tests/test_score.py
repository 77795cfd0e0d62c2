"""score_detections (reference repic/utils/score_detections.py:16-48).

CPU: the oracle (oracle/score_ref.py) and the BOX reader against the reference's own outputs
(tests/golden/score, made by tests/golden/make_score_golden.py).  GPU: the raster kernel
(rgc_score.hip through rgc_score_pairs) against the golden outputs and the oracle, bit-exact
(the scores are ratios of exact pixel counts, computed with the reference's numpy scalars).
"""
import json
import os
import warnings

import numpy as np
import pytest

HERE = os.path.dirname(os.path.abspath(__file__))
GOLD = os.path.join(HERE, "golden", "score")


def _cases():
    meta = json.load(open(os.path.join(GOLD, "meta.json")))
    arr = np.load(os.path.join(GOLD, "cases.npz"))
    for c in meta["cases"]:
        yield c, arr[c["name"] + "_gt"], arr[c["name"] + "_pk"]


def _same(got, case):
    want = [float.fromhex(h) for h in case["result_hex"]]
    for g, w, t in zip(got, want, case["result_type"]):
        assert type(g).__name__ == t, (case["name"], type(g), t)
        assert (np.isnan(g) and np.isnan(w)) or float(g).hex() == w.hex(), (case["name"], g, w)


def _recs(a):
    return [tuple(r) for r in a.tolist()]


def test_oracle_matches_reference_golden():
    from oracle import score_ref
    for case, g, p in _cases():
        with warnings.catch_warnings():
            warnings.simplefilter("ignore")
            got = score_ref.get_segmentation_scores(_recs(g), _recs(p), **case["kwargs"])
        _same(got, case)


def test_box_reader_matches_reference_process_conversion():
    from repic_amd.score_detections import read_box_file
    arr = np.load(os.path.join(GOLD, "cases.npz"))
    files = sorted(os.listdir(os.path.join(GOLD, "files")))
    assert files
    for f in files:
        got = read_box_file(os.path.join(GOLD, "files", f))
        want = arr["file_" + f]
        assert got.shape == want.shape and np.array_equal(got, want), f


def test_slice_normalisation_matches_numpy():
    """Host side of the device boundary: numpy slice bounds of arr[y:y+h, x:x+w]."""
    from repic_amd.score_detections import _mask_slices
    rng = np.random.default_rng(0)
    H, W = 37, 53
    x = rng.integers(-80, 80, 400).astype(float)
    y = rng.integers(-60, 60, 400).astype(float)
    w = rng.integers(-10, 70, 400).astype(float)
    h = rng.integers(-10, 70, 400).astype(float)
    s = _mask_slices(x, y, w, h, H, W)
    a = np.zeros((H, W), np.int16)
    b = np.zeros((H, W), np.int16)
    for xi, yi, wi, hi in zip(x.astype(int), y.astype(int), w.astype(int), h.astype(int)):
        a[yi:yi + hi, xi:xi + wi] = 1
    for r0, r1, c0, c1 in s:
        assert 0 <= r0 < r1 <= H and 0 <= c0 < c1 <= W
        b[r0:r1, c0:c1] = 1
    assert np.array_equal(a, b)


@pytest.mark.gpu
def test_gpu_scores_match_reference_golden():
    from repic_amd import score_detections as sd
    for case, g, p in _cases():
        with warnings.catch_warnings():
            warnings.simplefilter("ignore")
            got = sd.get_segmentation_scores(_recs(g), _recs(p), **case["kwargs"])
        _same(got, case)


@pytest.mark.gpu
def test_gpu_batched_scores_match_oracle():
    """Many pairs in one launch (mixed sizes, thresholds applied per call), vs the oracle."""
    from oracle import score_ref
    from repic_amd import score_detections as sd
    rng = np.random.default_rng(3)
    pairs = []
    for i in range(24):
        W, H = int(rng.integers(64, 1500)), int(rng.integers(64, 1500))
        sz = int(rng.integers(4, 200))
        def mk(n):
            x = rng.uniform(-sz, W, n).round(1)
            y = rng.uniform(-sz, H, n).round(1)
            return np.stack([x, y, np.full(n, float(sz)), np.full(n, float(sz)),
                             rng.uniform(0, 1, n)], axis=1)
        pairs.append((mk(int(rng.integers(0, 60))), mk(int(rng.integers(1, 80)))))
    for thr in (None, 0.4):
        got = sd.score_pairs(pairs, conf_thresh=thr)
        for (g, p), r in zip(pairs, got):
            with warnings.catch_warnings():
                warnings.simplefilter("ignore")
                want = score_ref.get_segmentation_scores(_recs(g), _recs(p), thr)
            for a, b in zip(r, want):
                assert type(a) is type(b)
                assert (np.isnan(a) and np.isnan(b)) or a == b


@pytest.mark.gpu
def test_gpu_score_cli(tmp_path):
    """The command line (score_detections.py:51-140) end to end on BOX files."""
    from oracle import score_ref
    from repic_amd import score_detections as sd
    rng = np.random.default_rng(5)
    gdir, pdir = tmp_path / "gt", tmp_path / "pk"
    gdir.mkdir()
    pdir.mkdir()
    want = {}
    for i in range(3):
        g = np.stack([rng.integers(0, 900, 50), rng.integers(0, 900, 50), np.full(50, 64),
                      np.full(50, 64), rng.uniform(0, 1, 50)], axis=1)
        p = g.copy()
        p[:, :2] += rng.integers(-20, 20, (50, 2))
        for d, a, nm in ((gdir, g, f"mg{i}.box"), (pdir, p, f"mg{i}_picked.box")):
            with open(d / nm, "w") as f:
                for r in a:
                    f.write(f"{int(r[0])}\t{int(r[1])}\t64\t64\t{float(r[4])!r}\n")
        want[f"mg{i}"] = score_ref.get_segmentation_scores(_recs(g.astype(float)),
                                                          _recs(p.astype(float)), 0.2)
    out = tmp_path / "out"
    sd.main(["-g"] + [str(f) for f in sorted(gdir.iterdir())] +
            ["-p"] + [str(f) for f in sorted(pdir.iterdir())] + ["-c", "0.2", "--out_dir", str(out)])
    lines = open(out / "particle_set_comp.tsv").read().splitlines()
    assert lines[0] == "filename\tprecision\trecall\tf1\tpos_frac"
    for ln in lines[1:]:
        name, *vals = ln.split("\t")
        assert vals == [str(v) for v in want[name]]
