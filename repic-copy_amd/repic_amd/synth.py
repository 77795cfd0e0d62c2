"""Seeded synthetic particle-pick generator (SURVEY.md §8(d) "Configs as synthetic inputs").

Model: ``n_true`` true particle centres uniform in ``[0, W-B] x [0, H-B]``.  Each of
``k`` pickers keeps each centre with probability ``keep``, jitters it by
N(0, (jit*B)^2) and rounds to an integer pixel; it then adds ``fp*n_true`` uniform
false positives and, with probability ``dup`` per box, an exact duplicate box (this
creates tied Jaccard degrees, exercising the consensus tie-break of
``get_cliques.py:182-183``).  One extra centre is planted exactly in every picker so
each micrograph has at least one k-clique (the reference crashes on zero cliques,
``get_cliques.py:203``).  Scores are U(0.3, 1.0); pickers listed in ``logit`` get
Topaz-like log-likelihood scores N(2, 2) (negative values trigger the sigmoid branch of
``common.py:92-94``).

The same generator feeds the golden fixtures (written as BOX text files) and the bench
(kept in memory), so both see the same distribution.
"""
from __future__ import annotations

import os
from dataclasses import dataclass, field

import numpy as np


@dataclass
class SynthConfig:
    k: int = 3
    n_true: int = 300
    box: int = 180
    width: int = 4096
    height: int = 4096
    keep: float = 0.9
    jit: float = 0.08
    fp: float = 0.1
    dup: float = 0.0
    logit: tuple = ()
    frac: bool = False          # non-integer coordinates (3 decimals)
    header: tuple = ()          # pickers whose files get a text header line
    seed: int = 0


# BASELINE.json configs[1..4]; C1 is the EMPIAR-10017 example set.
CONFIGS = {
    "C2": dict(k=3, n_true=300, box=180, width=4096, height=4096, keep=0.9, jit=0.08, fp=0.1),
    "C3": dict(k=4, n_true=1000, box=176, width=3838, height=3710, keep=0.9, jit=0.08, fp=0.1),
    "C4": dict(k=5, n_true=300, box=180, width=4096, height=4096, keep=0.9, jit=0.08, fp=0.1),
    "C5": dict(k=8, n_true=3000, box=64, width=4096, height=4096, keep=0.95, jit=0.06, fp=0.05,
               dup=0.15),
}


def _picker_boxes(rng, cfg: SynthConfig, centres, planted, p):
    B = cfg.box
    keep = rng.random(len(centres)) < cfg.keep
    pts = centres[keep] + rng.normal(0.0, cfg.jit * B, size=(int(keep.sum()), 2))
    n_fp = int(round(cfg.fp * cfg.n_true))
    fps = rng.uniform((0.0, 0.0), (cfg.width - B, cfg.height - B), size=(n_fp, 2))
    pts = np.concatenate([pts, fps], axis=0)
    if cfg.dup > 0:
        d = rng.random(len(pts)) < cfg.dup
        pts = np.concatenate([pts, pts[d]], axis=0)
    pts = pts[rng.permutation(len(pts))]
    if cfg.frac:
        pts = np.round(pts + rng.random(pts.shape), 3)
    else:
        pts = np.rint(pts)
    pts = np.concatenate([planted[None, :], pts], axis=0)
    if p in cfg.logit:
        sc = rng.normal(2.0, 2.0, size=len(pts))
    else:
        sc = rng.uniform(0.3, 1.0, size=len(pts))
    return pts[:, 0].copy(), pts[:, 1].copy(), sc


def micrograph(rng, cfg: SynthConfig):
    """Return a list of k (x, y, score) float64 triples for one micrograph."""
    B = cfg.box
    centres = rng.uniform((0.0, 0.0), (cfg.width - B, cfg.height - B), size=(cfg.n_true, 2))
    planted = np.rint(rng.uniform((0.0, 0.0), (cfg.width - B, cfg.height - B)))
    return [_picker_boxes(rng, cfg, centres, planted, p) for p in range(cfg.k)]


def batch(cfg: SynthConfig, n_mg: int, start: int = 0):
    """In-memory batch: list of micrographs (each a list of k (x, y, s) triples).

    Micrograph i uses its own stream ``default_rng([seed, start + i])`` so that shards
    generated on different ranks are identical to one big batch.
    """
    out = []
    for i in range(start, start + n_mg):
        rng = np.random.default_rng([cfg.seed, i])
        out.append(micrograph(rng, cfg))
    return out


def _fmt_coord(v: float, frac: bool) -> str:
    return repr(float(v)) if frac else str(int(v))


def write_box_dirs(root: str, cfg: SynthConfig, n_mg: int, names=None, start: int = 0):
    """Write ``root/picker{p}/mg{i:06d}.box`` files (EMAN BOX: x y w h score)."""
    names = names or [f"picker{p}" for p in range(cfg.k)]
    for p in range(cfg.k):
        os.makedirs(os.path.join(root, names[p]), exist_ok=True)
    for i, mg in enumerate(batch(cfg, n_mg, start)):
        for p, (x, y, s) in enumerate(mg):
            lines = []
            if p in cfg.header:
                lines.append("x\ty\tw\th\tscore\n")
            for xi, yi, si in zip(x.tolist(), y.tolist(), s.tolist()):
                lines.append(f"{_fmt_coord(xi, cfg.frac)}\t{_fmt_coord(yi, cfg.frac)}\t"
                             f"{cfg.box}\t{cfg.box}\t{si!r}\n")
            with open(os.path.join(root, names[p], f"mg{start + i:06d}.box"), "w") as f:
                f.writelines(lines)
    return names
