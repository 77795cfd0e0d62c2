"""ORACLE (vectorised) — numpy restatement of REPIC ``get_cliques`` for FULL-SIZE checks.

TEST INFRASTRUCTURE ONLY: imported by ``tests/`` (never by the product path).  It computes
the same per-micrograph results as ``oracle/cpu_ref.py`` (which is pinned bit-exactly to the
reference's golden outputs) with array operations instead of per-node Python loops, so the
GPU path can be compared with it at BASELINE.json's full sizes (C3: ~4k boxes / ~14k
cliques, C5: ~27k boxes / ~1M 8-cliques per micrograph) where ``cpu_ref`` takes minutes.
``tests/test_oracle.py`` pins it against ``cpu_ref`` (and so, transitively, the reference).

Restated reference semantics (reference repic/commands/get_cliques.py):
* JI pairs (:40-46, :59-69, :134-138): a grid with cell = box size finds every candidate
  (JI > 0.3 needs |dx|, |dy| < 0.54 B); JI in the reference's f64 operation order
  ``max((min(x,a) + B) - max(x,a), 0)`` ... ``I / ((2 B^2) - I)``; strict ``> 0.3``.
* CC stats (:145-149): components over boxes with >= 1 edge (scipy csgraph).
* cliques (:49-56, :160-161): the graph is k-partite, so size-k maximal cliques are the
  one-box-per-picker k-tuples that are pairwise adjacent (level-by-level extension).
* rows (:164, :193): rank of a clique vertex by (x, y, id).
* conf / w (:169-170, :186-190): ``f32(np.median(scores))``, ``f32(f64(conf) * np.median(JIs))``.
* consensus (:182-183): largest weighted degree (naive left-to-right f64 sum in increasing
  picker order = networkx adjacency order); ties go to the first tied member in the
  iteration order of the real CPython ``set(sorted(clique))`` (this interpreter), which is
  networkx's node order when ``2k < |G|`` (the only case this module accepts).
* ``--get_cc`` (:151-156): largest CC, ties -> the component whose first node in graph
  insertion order (edge enumeration order, u before v) comes first.
"""
from __future__ import annotations

import numpy as np
from scipy.sparse import coo_matrix
from scipy.sparse.csgraph import connected_components

THRESHOLD = 0.3   # get_cliques.py:138


def jaccard(x, y, a, b, box):
    """calc_jaccard (get_cliques.py:40-46), elementwise, same f64 op order."""
    xo = np.maximum((np.minimum(x, a) + box) - np.maximum(x, a), 0.0)
    yo = np.maximum((np.minimum(y, b) + box) - np.maximum(y, b), 0.0)
    inter = xo * yo
    with np.errstate(divide="ignore", invalid="ignore"):
        return inter / (np.float64(2 * box ** 2) - inter)


def edges(x, y, pick, box):
    """All JI > 0.3 pairs (u, v) with pick[u] < pick[v] (local indices), and their JI."""
    n = len(x)
    fin = np.isfinite(x) & np.isfinite(y)
    idx = np.nonzero(fin)[0]
    if len(idx) == 0 or box <= 0:
        return np.zeros(0, np.int64), np.zeros(0, np.int64), np.zeros(0)
    x0, y0 = x[idx].min(), y[idx].min()
    cx = np.floor((x[idx] - x0) / box).astype(np.int64)
    cy = np.floor((y[idx] - y0) / box).astype(np.int64)
    gy = int(cy.max()) + 3
    key = (cx + 1) * gy + (cy + 1)
    order = np.argsort(key, kind="stable")
    skey, sidx = key[order], idx[order]
    us, vs = [], []
    for dx in (-1, 0, 1):
        for dy in (-1, 0, 1):
            tk = key + dx * gy + dy
            lo = np.searchsorted(skey, tk, "left")
            hi = np.searchsorted(skey, tk, "right")
            cnt = hi - lo
            tot = int(cnt.sum())
            if tot == 0:
                continue
            src = np.repeat(idx, cnt)
            start = np.repeat(lo - (np.cumsum(cnt) - cnt), cnt)
            dst = sidx[start + np.arange(tot)]
            keep = pick[src] < pick[dst]
            us.append(src[keep])
            vs.append(dst[keep])
    u = np.concatenate(us) if us else np.zeros(0, np.int64)
    v = np.concatenate(vs) if vs else np.zeros(0, np.int64)
    pre = np.abs(x[u] - x[v]) <= box                       # get_cliques.py:64
    ji = jaccard(x[u], y[u], x[v], y[v], box)
    ok = pre & (ji > THRESHOLD)
    u, v, ji = u[ok], v[ok], ji[ok]
    o = np.lexsort((v, u))
    assert n < (1 << 31)
    return u[o].astype(np.int64), v[o].astype(np.int64), ji[o]


def micrograph(x, y, score, counts, box, get_cc=False, id_base=0):
    """One micrograph: ``x``/``y``/``score`` f64 in picker-major file order, ``counts[p]`` boxes
    of picker p; box i has global id ``id_base + i`` (the hash in the consensus tie-break).

    Returns dict: status ("ok" | "no_edges" | "no_cliques"), cc_max, cc_cnt, n_edges,
    members (C, k) local indices in lexicographic order, rows (C, k) ascending, w, conf
    (float32), consensus (C,) local index of the consensus member, V.
    """
    x = np.asarray(x, np.float64)
    y = np.asarray(y, np.float64)
    score = np.asarray(score, np.float64)
    k = len(counts)
    n = len(x)
    pb = np.concatenate([[0], np.cumsum(counts)]).astype(np.int64)
    pick = np.repeat(np.arange(k), counts)
    u, v, eji = edges(x, y, pick, box)
    out = {"n_edges": len(u)}
    if len(u) == 0:
        out["status"] = "no_edges"
        return out
    # connected components over graph nodes
    g = coo_matrix((np.ones(len(u)), (u, v)), shape=(n, n))
    _, lab = connected_components(g, directed=False)
    nodes = np.unique(np.concatenate([u, v]))
    sizes = np.bincount(lab[nodes])
    sizes = sizes[sizes > 0]
    out["cc_max"], out["cc_cnt"] = int(sizes.max()), int(len(sizes))
    allowed = np.ones(n, bool)
    if get_cc:
        # graph insertion order: edges enumerated by (picker pair, a index, b index), u then v
        pair = pick[u] * k + pick[v]
        eo = np.lexsort((v, u, pair))
        seq = np.stack([u[eo], v[eo]], axis=1).reshape(-1)
        first_nodes, first_pos = np.unique(seq, return_index=True)
        lab_n = lab[first_nodes]
        csize = np.bincount(lab[nodes], minlength=lab.max() + 1)
        big = np.nonzero(csize == csize.max())[0]
        # earliest-inserted node of each largest component
        best, best_pos = None, None
        for c in big:
            p = first_pos[lab_n == c].min()
            if best_pos is None or p < best_pos:
                best, best_pos = c, p
        allowed = lab == best
    # forward CSR keyed by (u, picker of v): edges are sorted by (u, v), v picker-major
    ekey = u * k + pick[v]
    # level-by-level extension (lexicographic prefixes)
    roots = np.unique(u[pick[u] == 0])
    roots = roots[allowed[roots]]
    P = roots[:, None]
    eset = u * n + v   # sorted (u major, then v)
    for D in range(1, k):
        last = P[:, D - 1]
        want = last * k + D
        lo = np.searchsorted(ekey, want, "left")
        hi = np.searchsorted(ekey, want, "right")
        cnt = hi - lo
        tot = int(cnt.sum())
        if tot == 0:
            P = np.zeros((0, D + 1), np.int64)
            break
        rep = np.repeat(np.arange(len(P)), cnt)
        start = np.repeat(lo - (np.cumsum(cnt) - cnt), cnt)
        cand = v[start + np.arange(tot)]
        ok = allowed[cand]
        for q in range(D - 1):
            kk = P[rep, q] * n + cand
            pos = np.searchsorted(eset, kk)
            pos = np.minimum(pos, len(eset) - 1)
            ok &= eset[pos] == kk
        P = np.concatenate([P[rep[ok]], cand[ok][:, None]], axis=1)
    if len(P) == 0:
        out["status"] = "no_cliques"
        return out
    C = len(P)
    # rows: rank of each clique vertex by (x, y, id)
    verts = np.unique(P)
    o = np.lexsort((verts, y[verts], x[verts]))
    rank = np.empty(n, np.int64)
    rank[verts[o]] = np.arange(len(verts))
    rows = np.sort(rank[P], axis=1)
    # conf / w
    conf = np.median(score[P], axis=1).astype(np.float32)
    pairs = [(a, b) for a in range(k) for b in range(a + 1, k)]
    J = np.empty((C, len(pairs)))
    for t, (a, b) in enumerate(pairs):
        J[:, t] = jaccard(x[P[:, a]], y[P[:, a]], x[P[:, b]], y[P[:, b]], box)
    w = (conf.astype(np.float64) * np.median(J, axis=1)).astype(np.float32)
    # consensus: weighted degree, naive sum in increasing picker order
    deg = np.zeros((C, k))
    for i in range(k):
        d = np.zeros(C)
        for q in range(k):
            if q == i:
                continue
            t = pairs.index((min(i, q), max(i, q)))
            d = d + J[:, t]
        deg[:, i] = d
    n_nodes = len(nodes)
    assert 2 * k < n_nodes, "cpu_vec handles the set-order case (2k < |G|) only"
    mx = deg.max(axis=1)
    ntop = (deg == mx[:, None]).sum(axis=1)
    cons = P[np.arange(C), deg.argmax(axis=1)]
    for j in np.nonzero(ntop > 1)[0]:
        keyn = {(float(x[m]), float(y[m]), id_base + int(m)): t for t, m in enumerate(P[j])}
        tup = tuple(sorted(keyn))
        for node in set(tup):   # CPython set iteration order
            t = keyn[node]
            if deg[j, t] == mx[j]:
                cons[j] = P[j, t]
                break
    out.update(status="ok", members=P, rows=rows, w=w, conf=conf, consensus=cons,
               V=int(len(verts)), n_nodes=int(n_nodes))
    return out
