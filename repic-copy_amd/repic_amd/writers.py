"""Per-micrograph output files, exactly the set the reference writes.

reference get_cliques.py:125-129 (skip -> empty ``<base>.box``) and :204-229:
``<base>_weight_vector.pickle`` (float32[C]), ``<base>_consensus_coords.pickle`` (list of
``(x, y, id)`` tuples, or the ``--multi_out`` table), ``<base>_consensus_confidences.pickle``
(float32[C]), ``<base>_constraint_matrix.pickle`` (scipy ``coo_matrix``, int64 data, int32
indices, shape (V, C)) and ``<base>_runtime.tsv`` ("seconds\\tlargest CC\\tnumber of CCs").
All pickles use ``pickle.HIGHEST_PROTOCOL`` so the unchanged ``run_ilp`` reads them.
"""
from __future__ import annotations

import os
import pickle
from concurrent.futures import ThreadPoolExecutor

import numpy as np
from scipy.sparse import coo_matrix

LABELS = ("weight_vector", "consensus_coords", "consensus_confidences", "constraint_matrix")


def write_skip(out_dir: str, base: str):
    with open(os.path.join(out_dir, base + ".box"), "wt"):
        pass


def constraint_matrix(rows: np.ndarray, n_vert: int):
    """coo_matrix(([1]*nnz, (rows, cols)), shape=(V, C)) with cols = [j]*k (:192-202)."""
    C, k = rows.shape
    cols = np.repeat(np.arange(C, dtype=np.int32), k)
    data = np.ones(C * k, dtype=np.int64)
    return coo_matrix((data, (rows.reshape(-1).astype(np.int32), cols)), shape=(n_vert, C))


def consensus_coords(x, y, ids):
    return list(zip(x.tolist(), y.tolist(), ids.tolist()))


def multi_out_coords(methods, member_tuples, order, k, get_cc, picker_coords):
    """--multi_out table (get_cliques.py:175-178, 206-213).

    Members are sorted by the node attribute "name" that add_nodes_to_graph (:30-37)
    assigns: every node is (re)named ``node_names[0]`` when added as the first box of a
    pair and ``node_names[1]`` as the second, so clique members of pickers 0..k-2 end up
    ``methods[0]`` and the picker k-1 member ``methods[1]``; sorted() is stable, so the
    former keep networkx's node iteration order (``order``).
    """
    rows = [list(methods)]
    for j in range(len(member_tuples)):
        mt = member_tuples[j]
        first = [mt[p] for p in order[j] if p != k - 1]
        rows.append(first + [mt[k - 1]])
    if not get_cc:
        clique_set = set([val for clique in rows for val in clique])
        for p in range(k):
            for val in set(picker_coords[p]).difference(clique_set):
                e = [None] * k
                e[p] = val
                rows.append(e)
    return rows


def write_micrograph(out_dir, base, w, coords, conf, A, seconds, cc_max, cc_cnt):
    for label, val in zip(LABELS, (w, coords, conf, A)):
        with open(os.path.join(out_dir, f"{base}_{label}.pickle"), "wb") as o:
            pickle.dump(val, o, protocol=pickle.HIGHEST_PROTOCOL)
    with open(os.path.join(out_dir, f"{base}_runtime.tsv"), "wt") as o:
        o.write("\t".join([str(seconds), str(cc_max), str(cc_cnt)]) + "\n")


class Writer:
    """Thread-pooled writer: file creation dominates the per-micrograph output cost and
    releases the GIL, so writes of different micrographs overlap.  ``close()`` waits for
    every pending write and re-raises the first I/O error."""

    def __init__(self, threads=None):
        self.threads = threads or min(16, (os.cpu_count() or 1))
        self._pool = ThreadPoolExecutor(max_workers=self.threads) if self.threads > 1 else None
        self._futs = []
        self._bases = set()

    def _submit(self, fn, *args):
        base = args[1]
        if base in self._bases:      # same output name twice: keep the reference's order
            self._drain()
        self._bases.add(base)
        if self._pool is None:
            fn(*args)
        else:
            self._futs.append(self._pool.submit(fn, *args))
            if len(self._futs) > 4 * self.threads:
                self._drain(len(self._futs) // 2)

    def _drain(self, n=None):
        n = len(self._futs) if n is None else n
        done, self._futs = self._futs[:n], self._futs[n:]
        for f in done:
            f.result()

    def skip(self, out_dir, base):
        self._submit(write_skip, out_dir, base)

    def micrograph(self, *args):
        self._submit(write_micrograph, *args)

    def close(self):
        try:
            self._drain()
        finally:
            if self._pool is not None:
                self._pool.shutdown(wait=True)
