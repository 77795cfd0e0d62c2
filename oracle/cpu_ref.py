"""ORACLE — CPU restatement of REPIC ``get_cliques`` (TEST INFRASTRUCTURE ONLY).

Only ``tests/``, ``__graft_entry__.smoke()`` and ``bench.py``'s ``cpu_baseline`` leg may
import this module, and only as the checker / the timed CPU baseline.  The product path
(``repic-copy_amd/repic_amd``) never imports it.

It restates the semantics of the reference hot path without networkx:

* BOX parsing           -> ``parse_box``         (reference ``common.py:71-114``)
* Jaccard index         -> ``jaccard``            (``get_cliques.py:40-46``)
* pair loop + threshold -> ``edges_faithful`` / ``edges_vectorised`` (``:59-69``, ``:134-138``)
* graph + CC stats      -> ``Micrograph.graph``   (``:30-37``, ``:142-149``)
* largest-CC filter     -> ``--get_cc``           (``:151-156``)
* size-k cliques        -> one-box-per-picker k-tuples (``:49-56``, ``:160-161``; the graph
                           is k-partite, so every maximal clique of size k is exactly such
                           a tuple)
* ILP structures        -> ``Micrograph.ilp``     (``:164-202``)
* writers               -> ``run_dir``            (``:72-130``, ``:204-229``)

Parity is pinned against golden fixtures produced by running the reference itself in the
development container (``tests/golden/make_golden.py``); see ``tests/test_oracle.py``.
"""
from __future__ import annotations

import fnmatch
import itertools
import os
import pickle
import shutil
import time
from pathlib import Path

import numpy as np
from scipy.sparse import coo_matrix

THRESHOLD = 0.3   # get_cliques.py:138


# --------------------------------------------------------------------------- parsing
def _is_float(tok: str) -> bool:
    """common.py:44-51 check_float."""
    try:
        float(tok)
    except ValueError:
        return False
    return True


def parse_box(path: str):
    """Return ``(x, y, w)`` lists for one BOX file, raising what common.py:71-99 raises.

    * first token of line 1 not a float -> that line is a header and is skipped (:79-80)
    * rows are zipped column-wise: the SHORTEST row must have exactly 5 tokens (:81)
    * x / y tokens that are not floats are dropped, weights must all be floats (:87-89)
    * if min(weights) < 0 (NaN-propagating np.min), weights -> numpy sigmoid (:92-94)
    * len(x) != len(y) -> AssertionError (:96); coords = zip(x, y, w) (truncating)
    * an empty first line -> IndexError (caller treats it as "skip micrograph")
    """
    with open(path, "rt") as f:
        if _is_float(f.readline().rstrip().split()[0]):
            f.seek(0)
        X, Y, H, W, weights = zip(*[ln.strip().split() for ln in f])
    X = [float(v) for v in X if _is_float(v)]
    Y = [float(v) for v in Y if _is_float(v)]
    weights = [float(v) for v in weights]
    if np.min(weights) < 0:
        weights = [1.0 / (1.0 + np.exp(-1.0 * v)) for v in weights]
    assert len(X) == len(Y), "unequal number of x and y elements"
    n = min(len(X), len(Y), len(weights))
    return X[:n], Y[:n], weights[:n]


# --------------------------------------------------------------------------- Jaccard
def jaccard(x, y, a, b, box):
    """get_cliques.py:40-46 with the same f64 operation order (np.min/np.max on 2-lists)."""
    xo = np.max([(np.min([x, a]) + box - np.max([x, a])), 0])
    yo = np.max([(np.min([y, b]) + box - np.max([y, b])), 0])
    inter = xo * yo
    return inter / ((2 * box ** 2) - inter)


def edges_faithful(P, Q, box):
    """Per-pair loop with the reference's structure (get_cliques.py:59-69).

    ``P``/``Q`` are lists of (x, y, w, id).  Returns [(i, j, ji)] with i/j file indices.
    This is the timed CPU baseline: it pays the same per-pair numpy overheads.
    """
    out = []
    for i, (x, y, _, _) in enumerate(P):
        for j, (a, b, _, _) in enumerate(Q):
            if np.abs(x - a) <= box:
                ji = jaccard(x, y, a, b, box)
                if ji > THRESHOLD:
                    out.append((i, j, ji))
    return out


def edges_vectorised(P, Q, box):
    """Same edge set and bit-identical JI as ``edges_faithful`` (same IEEE op order)."""
    if not P or not Q:
        return []
    px = np.array([p[0] for p in P]); py = np.array([p[1] for p in P])
    qx = np.array([q[0] for q in Q]); qy = np.array([q[1] for q in Q])
    out = []
    # chunk rows to bound memory
    step = max(1, 4_000_000 // max(1, len(Q)))
    for s in range(0, len(P), step):
        x = px[s:s + step, None]; y = py[s:s + step, None]
        pre = np.abs(x - qx[None, :]) <= box
        xo = np.maximum((np.minimum(x, qx[None, :]) + box) - np.maximum(x, qx[None, :]), 0.0)
        yo = np.maximum((np.minimum(y, qy[None, :]) + box) - np.maximum(y, qy[None, :]), 0.0)
        inter = xo * yo
        with np.errstate(divide="ignore", invalid="ignore"):
            ji = inter / (np.float64(2 * box ** 2) - inter)
        ii, jj = np.nonzero(pre & (ji > THRESHOLD))
        out.extend(zip((ii + s).tolist(), jj.tolist(), ji[ii, jj].tolist()))
    return out


# --------------------------------------------------------------------------- micrograph
class NoEdges(ValueError):
    """The reference raises ValueError from np.max([]) (get_cliques.py:148)."""


class NoCliques(UnboundLocalError):
    """The reference raises UnboundLocalError at ``del ... clique`` (get_cliques.py:203)."""


def micrograph(coords, box, methods, get_cc=False, multi_out=False, faithful=False):
    """Run one micrograph.  ``coords[p]`` = list of (x, y, w, id) in file order.

    Returns a dict with ``w``, ``conf`` (float32), ``consensus`` (list), ``A``
    (coo_matrix), ``cc_max``, ``cc_cnt``; raises NoEdges / NoCliques like the reference.
    """
    k = len(coords)
    key = [[(float(c[0]), float(c[1]), int(c[3])) for c in P] for P in coords]
    score = [[c[2] for c in P] for P in coords]
    edge_fn = edges_faithful if faithful else edges_vectorised

    # graph (get_cliques.py:30-37, 134-143): insertion-ordered adjacency like networkx
    adj: dict = {}
    name: dict = {}
    weight: dict = {}
    for (j, l) in itertools.combinations(range(k), 2):
        for (i1, i2, ji) in edge_fn(coords[j], coords[l], box):
            u, v = key[j][i1], key[l][i2]
            ji = np.float64(ji)
            for n, p, i, nm in ((u, j, i1, methods[0]), (v, l, i2, methods[1])):
                adj.setdefault(n, {})
                name[n] = nm               # add_nodes_to_graph names with node_names[0/1]
                weight[n] = score[p][i]
            adj[u][v] = ji
            adj[v][u] = ji
    picker_of = {key[p][i]: p for p in range(k) for i in range(len(key[p]))}

    # connected components in discovery order (networkx connected_components)
    seen, comps = set(), []
    for n in adj:
        if n in seen:
            continue
        comp, stack = [], [n]
        seen.add(n)
        while stack:
            u = stack.pop()
            comp.append(u)
            for v in adj[u]:
                if v not in seen:
                    seen.add(v)
                    stack.append(v)
        comps.append(comp)
    sizes = [len(c) for c in comps]
    if not sizes:
        raise NoEdges("zero-size array to reduction operation maximum which has no identity")
    cc_max, cc_cnt = int(np.max(sizes)), len(sizes)
    allowed = None
    if get_cc:
        best = max(range(len(comps)), key=lambda i: (sizes[i], -i))
        allowed = set(comps[best])

    # size-k cliques = pairwise-adjacent one-box-per-picker tuples
    by_picker = [[n for n in adj if picker_of[n] == p and (allowed is None or n in allowed)]
                 for p in range(k)]
    cliques = []

    def extend(chosen):
        p = len(chosen)
        if p == k:
            cliques.append(tuple(sorted(chosen)))
            return
        if p == 0:
            cands = by_picker[0]
        else:
            cands = [v for v in adj[chosen[0]] if picker_of[v] == p
                     and (allowed is None or v in allowed)]
        for v in cands:
            if all(v in adj[c] for c in chosen):
                extend(chosen + [v])

    extend([])
    if not cliques:
        raise NoCliques("local variable 'clique' referenced before assignment")

    # ILP structures (get_cliques.py:164-202)
    n = len(cliques)
    verts = sorted(set(sum(cliques, ())))
    row_of = {v: r for r, v in enumerate(verts)}
    conf = np.zeros(n, dtype=np.float32)
    w = np.zeros(n, dtype=np.float32)
    out_coords, rows, cols = [], [], []
    graph_order = {u: r for r, u in enumerate(adj)}
    n_graph = len(adj)
    for j, cl in enumerate(cliques):
        members = set(cl)
        # FilterAtlas.__iter__: set order when 2*|nodes| < |G|, else graph insertion order
        if 2 * len(members) < n_graph:
            it = [u for u in members]
        else:
            it = sorted(members, key=graph_order.__getitem__)
        if multi_out:
            out_coords.append(sorted(it, key=lambda u: name[u]))
        else:
            best, best_deg = None, None
            for u in it:
                deg = 0
                for v, ji in adj[u].items():
                    if v in members:
                        deg = deg + ji
                if best is None or deg > best_deg:
                    best, best_deg = u, deg
            out_coords.append(best)
        conf[j] = np.median([weight[u] for u in it])
        eji = [adj[a][b] for a, b in itertools.combinations(cl, 2)]
        w[j] = conf[j] * np.median(eji)
        cols.extend([j] * k)
        rows.extend(row_of[u] for u in cl)
    A = coo_matrix(([1] * len(cols), (rows, cols)), shape=(len(verts), n))
    if multi_out:
        out_coords = [list(methods)] + out_coords
        if not get_cc:
            in_cl = set(v for c in out_coords for v in c)
            for p in range(k):
                four = [(c[0], c[1], c[2], c[3]) for c in coords[p]]
                for val in set(four).difference(in_cl):
                    e = [None] * k
                    e[p] = val
                    out_coords.append(e)
    return {"w": w, "conf": conf, "consensus": out_coords, "A": A,
            "cc_max": cc_max, "cc_cnt": cc_cnt}


# --------------------------------------------------------------------------- directory driver
def _glob(dir_path, pattern, listing=None):
    """glob.glob(os.path.join(dir_path, pattern)) in readdir order (hidden names skipped)."""
    if listing is not None and os.path.basename(dir_path) in listing:
        names = listing[os.path.basename(dir_path)]
    else:
        try:
            names = os.listdir(dir_path)
        except (FileNotFoundError, NotADirectoryError):
            return []
    return [os.path.join(dir_path, n) for n in names
            if not n.startswith(".") and fnmatch.fnmatchcase(n, pattern)]


def load_coords(pattern_dir, pattern, next_id, listing=None):
    """common.py:71-114 get_box_coords(return_weights=True) -> (coords, next_id)."""
    files = _glob(pattern_dir, pattern, listing)
    if not files:
        raise UnboundLocalError("local variable 'i' referenced before assignment")
    for f in files:
        X, Y, W = parse_box(f)
    assert len(files) == 1, "multiple BOX files found using pattern"
    coords = [(x, y, w, i) for i, (x, y, w) in enumerate(zip(X, Y, W), next_id)]
    return coords, coords[-1][-1] + 1      # IndexError when empty (-> skip)


def run_dir(in_dir, out_dir, box, get_cc=False, multi_out=False, listing=None,
            faithful=False, quiet=True):
    """Directory-level restatement of get_cliques.main (get_cliques.py:72-229)."""
    assert os.path.exists(in_dir), "Error - input directory does not exist"
    if Path(out_dir).is_dir():
        shutil.rmtree(out_dir)
    methods = sorted([os.path.basename(v) for v in _glob(in_dir, "*") if os.path.isdir(v)],
                     key=str)
    Path(out_dir).mkdir(parents=True, exist_ok=True)
    start_method, n = None, None
    box_file = None
    for method in methods:
        for box_file in _glob(os.path.join(in_dir, method), "*.box", listing):
            tmp = f"*{os.path.basename(box_file).replace('.box', '')}*"
            n = sum(len(_glob(os.path.join(in_dir, m), tmp, listing)) for m in methods)
            break
        if n is None:
            raise UnboundLocalError("local variable 'n' referenced before assignment")
        if n == len(methods):
            start_method = method
            break
    assert start_method is not None, "Error - particle file names cannot be paired across methods"
    if box_file is None:
        raise UnboundLocalError("local variable 'box_file' referenced before assignment")
    next_id = 0
    for box_file in _glob(os.path.join(in_dir, methods[0]), "*.box", listing):
        start = time.time()
        base = os.path.basename(box_file).replace(".box", "")
        try:
            coords = []
            c, next_id = load_coords(os.path.dirname(box_file), os.path.basename(box_file),
                                     next_id, None)
            coords.append(c)
            for m in methods[1:]:
                c, next_id = load_coords(os.path.join(in_dir, m), f"*{base}*", next_id, listing)
                coords.append(c)
        except (UnboundLocalError, IndexError):
            open(os.path.join(out_dir, base + ".box"), "wt").close()
            continue
        res = micrograph(coords, box, methods, get_cc, multi_out, faithful)
        for label, val in zip(["weight_vector", "consensus_coords", "consensus_confidences",
                               "constraint_matrix"],
                              [res["w"], res["consensus"], res["conf"], res["A"]]):
            with open(os.path.join(out_dir, f"{base}_{label}.pickle"), "wb") as o:
                pickle.dump(val, o, protocol=pickle.HIGHEST_PROTOCOL)
        with open(os.path.join(out_dir, f"{base}_runtime.tsv"), "wt") as o:
            o.write(f"{time.time() - start}\t{res['cc_max']}\t{res['cc_cnt']}\n")
