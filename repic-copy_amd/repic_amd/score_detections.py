"""``score_detections`` — precision / recall / F1 of picked particle sets, MI355X raster.

Same interface as the reference module (repic/utils/score_detections.py):
``get_segmentation_scores(gt_boxes, pckr_boxes, conf_thresh=None, mrc_w=None, mrc_h=None)``
returns ``(prec, rec, f1, pos_frac)`` with the reference's numpy scalar types, and the command
line (``-g``, ``-p``, ``-c``, ``--height``, ``--width``, ``--verbose``, ``--out_dir``) writes the
same ``particle_set_comp.tsv``.  The (H x W) int16 masks the reference paints
(score_detections.py:28-41) are never materialised: ``librepic_gc.so``'s ``rgc_score_pairs``
paints 1-bit tiles in LDS and returns three pixel counts per pair (rgc_score.hip), many
micrograph pairs per launch (``score_pairs``).  No CPU fallback: the library must load.
"""
from __future__ import annotations

import argparse
import ctypes as C
import os
import re
from collections import namedtuple
from pathlib import Path

import numpy as np

from . import _lib

# the reference's coordinate record (coord_converter.py:50-51: conf defaults to 0)
Box = namedtuple("Box", ["x", "y", "w", "h", "conf"])
Box.__new__.__defaults__ = (0,)


class ScoreIn(C.Structure):
    _fields_ = [("n_pairs", C.c_int64), ("height", C.c_void_p), ("width", C.c_void_p),
                ("gt_off", C.c_void_p), ("pk_off", C.c_void_p), ("boxes", C.c_void_p),
                ("flags", C.c_uint32)]


_lib.lib.rgc_score_pairs.argtypes = [C.c_void_p, C.POINTER(ScoreIn), C.c_void_p]
_lib.lib.rgc_score_pairs.restype = C.c_int


def _py_round(v):
    """Python ``round(v)`` of each value (score_detections.py:31,36): half to even -> int."""
    v = np.asarray(v)
    if v.dtype.kind in "iu":
        return v.astype(np.int64)
    v = v.astype(np.float64)
    if not np.isfinite(v).all():
        raise ValueError("cannot convert float NaN or infinity to integer")
    return np.rint(v).astype(np.int64)


def _slice_bounds(a, n):
    """Python slice.indices for step 1: negative values wrap once, then clamp to [0, n]."""
    return np.where(a < 0, np.maximum(a + n, 0), np.minimum(a, n))


def _as_cols(boxes):
    """(x, y, w, h, conf) columns of a box list (namedtuples / tuples) or a (n, >=4) array."""
    if isinstance(boxes, np.ndarray):
        a = boxes
        conf = a[:, 4] if a.shape[1] > 4 else np.zeros(len(a))
        return a[:, 0], a[:, 1], a[:, 2], a[:, 3], conf
    if not len(boxes):
        z = np.zeros(0)
        return z, z, z, z, z
    cols = list(zip(*[tuple(b) for b in boxes]))
    conf = cols[4] if len(cols) > 4 else [0] * len(boxes)
    return tuple(np.asarray(c) for c in cols[:4]) + (np.asarray(conf, dtype=np.float64),)


def _mask_slices(x, y, w, h, H, W):
    """Non-empty numpy slices [r0, r1) x [c0, c1) of ``arr[y:y+h, x:x+w] = 1``."""
    xi, yi, wi, hi = (_py_round(v) for v in (x, y, w, h))
    r0, r1 = _slice_bounds(yi, H), _slice_bounds(yi + hi, H)
    c0, c1 = _slice_bounds(xi, W), _slice_bounds(xi + wi, W)
    keep = (r0 < r1) & (c0 < c1)
    return np.stack([r0[keep], r1[keep], c0[keep], c1[keep]], axis=1).astype(np.int32)


def _scores(counts, H, W):
    """score_detections.py:43-48 on the three pixel counts, same numpy scalar arithmetic."""
    gsum, num_pos, tp = (np.int64(v) for v in counts)
    pos_frac = num_pos / (H * W)
    prec = 0.0 if (tp == num_pos == 0.0) else (tp / num_pos)
    rec = tp / gsum
    f1 = 0.0 if (prec == rec == 0.0) else ((2 * prec * rec) / (prec + rec))
    return prec, rec, f1, pos_frac


_CTX = None


def _ctx():
    global _CTX
    if _CTX is None:
        _CTX = _lib.Context(int(os.environ.get("LOCAL_RANK", "0")))
    return _CTX


def score_pairs(pairs, conf_thresh=None, mrc_w=None, mrc_h=None, ctx=None, timing=False):
    """Batched ``get_segmentation_scores`` over (gt_boxes, pckr_boxes) pairs: one device call.
    Returns a list of (prec, rec, f1, pos_frac); with ``timing`` also the kernel ms."""
    ctx = ctx or _ctx()
    Hs, Ws, gts, pks = [], [], [], []
    for gt, pk in pairs:
        g = _as_cols(gt)
        p = _as_cols(pk)
        # mrc_w / mrc_h default: round(max(x + w)) over every box, thresholded or not (:22-26)
        W = mrc_w if mrc_w is not None else int(_py_round(np.max(np.concatenate(
            [g[0] + g[2], p[0] + p[2]]))))
        H = mrc_h if mrc_h is not None else int(_py_round(np.max(np.concatenate(
            [g[1] + g[3], p[1] + p[3]]))))
        if H < 0 or W < 0:
            raise ValueError("negative dimensions are not allowed")
        if conf_thresh is not None:
            keep = ~(p[4] < conf_thresh)          # b.conf < conf_thresh -> skipped (:35-36)
            p = tuple(c[keep] for c in p)
        gts.append(_mask_slices(*g[:4], H, W))
        pks.append(_mask_slices(*p[:4], H, W))
        Hs.append(H)
        Ws.append(W)
    # every pair's ground-truth boxes, then every pair's picks
    npairs = len(Hs)
    z = np.zeros((0, 4), np.int32)
    boxes = np.ascontiguousarray(np.concatenate(gts + pks + [z]), dtype=np.int32)
    ng = np.cumsum([0] + [len(v) for v in gts]).astype(np.int64)
    gt_arr = ng
    pk_arr = (ng[-1] + np.cumsum([0] + [len(v) for v in pks])).astype(np.int64)
    H = np.asarray(Hs, dtype=np.int64)
    W = np.asarray(Ws, dtype=np.int64)
    counts = np.zeros((npairs, 3), dtype=np.int64)
    si = ScoreIn(npairs, H.ctypes.data, W.ctypes.data, gt_arr.ctypes.data, pk_arr.ctypes.data,
                 boxes.ctypes.data, _lib.F_TIMING if timing else 0)
    ctx._retire()   # a live Result of an earlier run keeps its host buffers
    _lib._check(_lib.lib.rgc_score_pairs(ctx._p, C.byref(si), counts.ctypes.data))
    out = [_scores(counts[i], int(H[i]), int(W[i])) for i in range(npairs)]
    if timing:
        return out, dict(ctx.kernel_times())
    return out


def get_segmentation_scores(gt_boxes, pckr_boxes, conf_thresh=None, mrc_w=None, mrc_h=None):
    """score_detections.py:16-48 for one pair (prec, rec, f1, pos_frac)."""
    return score_pairs([(gt_boxes, pckr_boxes)], conf_thresh, mrc_w, mrc_h)[0]


# ----------------------------------------------------------------------------- command line
def read_box_file(path):
    """BOX file -> (n, 5) float array x, y, w, h, conf, as the reference reads it with
    coord_converter.process_conversion([path], "box", "box") (tsv_to_df, coord_converter.py:
    200-243): leading lines are skipped up to the first one that does not start with "_" and
    contains a digit; whitespace-separated columns; rows without any numeric value dropped;
    a missing conf column becomes 1 (score_detections.py:118-120)."""
    import pandas as pd
    start = 0
    with open(path) as f:
        for i, line in enumerate(f):
            if not line.startswith("_") and re.search("[0-9]", line):
                start = i
                break
    try:
        df = pd.read_csv(path, sep=r"\s+", header=None, skip_blank_lines=True, skiprows=start)
    except pd.errors.EmptyDataError:
        return np.zeros((0, 5))

    def numeric(v):
        try:
            float(v)
            return True
        except (TypeError, ValueError):
            return False
    df = df[[any(numeric(v) for v in row.dropna()) for _, row in df.iterrows()]]
    cols = [df[c].to_numpy(dtype=np.float64) for c in df.columns[:5]]
    if len(cols) < 5:
        cols.append(np.ones(len(df)))
    return np.stack(cols[:5], axis=1) if len(df) else np.zeros((0, 5))


def main(argv=None):
    ap = argparse.ArgumentParser(
        description="Score detections between ground truth and particle picker coordinate "
                    "sets, matching files by name (BOX format).")
    ap.add_argument("-g", help="Ground truth particle coordinate file(s)", nargs="+", required=True)
    ap.add_argument("-p", help="Particle picker coordinate file(s)", nargs="+", required=True)
    ap.add_argument("-c", help="Confidence threshold", type=float)
    ap.add_argument("--height", help="Micrograph height (pixels)", type=int, default=None)
    ap.add_argument("--width", help="Micrograph width (pixels)", type=int, default=None)
    ap.add_argument("--verbose", help="Print individual boxfile pair scores", action="store_true")
    ap.add_argument("--out_dir", help="file path to output directory", type=str)
    a = ap.parse_args(argv)
    # score_detections.py:87-90, including its quirk: an existing --out_dir is ignored
    if a.out_dir is not None and not os.path.exists(a.out_dir):
        os.makedirs(a.out_dir)
    else:
        a.out_dir = os.path.dirname(a.p[0])
    gt_names = [Path(f).stem.lower() for f in a.g if f.endswith(".box")]
    pk_names = [Path(f).stem.lower() for f in a.p if f.endswith(".box")]
    matches = [g for g in gt_names if sum(p.startswith(g) for p in pk_names) > 0]
    if a.verbose:
        print(f"Found {len(matches)} boxfile matches\n")
    assert len(matches) > 0, "No paired ground truth and picker particle sets found"
    pairs = []
    for m in matches:
        gp = next(f for f in a.g if Path(f).stem.lower() == m)
        pp = next(f for f in a.p if Path(f).stem.lower().startswith(m))
        pairs.append((read_box_file(gp), read_box_file(pp)))
    scores = score_pairs(pairs, a.c, a.width, a.height)
    rows = []
    for m, (prec, rec, f1, pos) in zip(matches, scores):
        if a.verbose:
            print(f"{m} - precision: {prec:.3f} recall: {rec:.3f} F1-score: {f1:.3f}")
        rows.append((m, prec, rec, f1, pos))
    with open(os.path.join(a.out_dir, "particle_set_comp.tsv"), "wt") as o:
        o.write("\t".join(["filename", "precision", "recall", "f1", "pos_frac"]) + "\n")
        for e in rows:
            o.write("\t".join(str(v) for v in e) + "\n")


if __name__ == "__main__":
    main()
