"""CPU oracle for score_detections (TEST INFRASTRUCTURE ONLY: imported by tests/ and the
score bench's CPU leg, never by the product path).

Restates reference repic/utils/score_detections.py:16-48 ``get_segmentation_scores`` with
numpy: the same int16 (H x W) masks painted by slice assignment, the same reductions and the
same scalar arithmetic.  Pinned by tests/golden/score/ (outputs of the real reference on the
same inputs, tests/golden/make_score_golden.py).
"""
from __future__ import annotations

import numpy as np


def get_segmentation_scores(gt_boxes, pckr_boxes, conf_thresh=None, mrc_w=None, mrc_h=None):
    """``gt_boxes`` / ``pckr_boxes``: sequences of (x, y, w, h, conf) records."""
    if mrc_w is None:                                            # :22-26
        mrc_w = round(max([b[0] + b[2] for b in list(gt_boxes) + list(pckr_boxes)]))
    if mrc_h is None:
        mrc_h = round(max([b[1] + b[3] for b in list(gt_boxes) + list(pckr_boxes)]))
    gt_arr = np.zeros((mrc_h, mrc_w), dtype=np.int16)           # :28-30
    pk_arr = np.zeros((mrc_h, mrc_w), dtype=np.int16)
    for b in gt_boxes:                                           # :31-33
        x, y, w, h = round(b[0]), round(b[1]), round(b[2]), round(b[3])
        gt_arr[y:y + h, x:x + w] = 1
    for b in pckr_boxes:                                         # :34-38
        if conf_thresh is not None and b[4] < conf_thresh:
            continue
        x, y, w, h = round(b[0]), round(b[1]), round(b[2]), round(b[3])
        pk_arr[y:y + h, x:x + w] = 1
    num_pos = np.sum(pk_arr)                                     # :41-46
    pos_frac = num_pos / pk_arr.size
    tp = np.sum(gt_arr * pk_arr)
    prec = 0.0 if (tp == num_pos == 0.0) else (tp / num_pos)
    rec = tp / np.sum(gt_arr)
    f1 = 0.0 if (prec == rec == 0.0) else ((2 * prec * rec) / (prec + rec))
    return prec, rec, f1, pos_frac
