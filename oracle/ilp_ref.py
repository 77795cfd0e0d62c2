"""CPU oracle for run_ilp's set packing (TEST INFRASTRUCTURE ONLY: imported by tests/ and the
ILP bench's CPU leg, never by the product path).

The reference solves, per micrograph, max w.x s.t. A x <= 1, x binary with Gurobi
(repic/commands/run_ilp.py:50-63).  gurobipy is not installed here, so parity against Gurobi
itself is UNPINNED; the model is restated for two independent exact solvers instead:
``milp`` (scipy.optimize.milp = HiGHS branch and cut, relative gap 0) and ``brute_force``
(every subset of each conflict component, for small components), which pin each other in
tests/test_ilp.py.
"""
from __future__ import annotations

import itertools

import numpy as np
from scipy.optimize import Bounds, LinearConstraint, milp as _milp
from scipy.sparse import csr_matrix
from scipy.sparse.csgraph import connected_components


def milp(A, w):
    """HiGHS on the reference model: returns (x uint8, objective f64 = sum of chosen w)."""
    A = csr_matrix(A)
    n = A.shape[1]
    w = np.asarray(w, dtype=np.float64)
    res = _milp(-w, integrality=np.ones(n), bounds=Bounds(0, 1),
                constraints=[LinearConstraint(A, -np.inf, 1)],
                options={"mip_rel_gap": 0.0, "presolve": True})
    assert res.status == 0, res.message
    x = (res.x > 0.5).astype(np.uint8)
    return x, float(np.sum(w[x == 1]))


def components(A):
    """Conflict components: columns sharing a row (a box) are connected."""
    B = csr_matrix(A).T.tocsr()
    G = B @ B.T
    return connected_components(G, directed=False)


def brute_force(A, w, max_comp=18):
    """Exact optimum by enumerating every packing of every conflict component (<= max_comp
    columns each); returns (x, objective) or None if a component is larger."""
    A = csr_matrix(A)
    w = np.asarray(w, dtype=np.float64)
    nc, lab = components(A)
    x = np.zeros(A.shape[1], np.uint8)
    cols = A.T.tocsr()
    for c in range(nc):
        mem = np.flatnonzero(lab == c)
        if len(mem) > max_comp:
            return None
        rows = [set(cols[j].indices.tolist()) for j in mem]
        best, best_s = -1.0, ()
        for r in range(len(mem) + 1):
            for sub in itertools.combinations(range(len(mem)), r):
                used = set()
                ok = True
                for i in sub:
                    if used & rows[i]:
                        ok = False
                        break
                    used |= rows[i]
                if ok:
                    s = float(sum(w[mem[i]] for i in sub))
                    if s > best:
                        best, best_s = s, sub
        for i in best_s:
            x[mem[i]] = 1
    return x, float(np.sum(w[x == 1]))


def is_packing(A, x):
    return bool(np.max(csr_matrix(A) @ np.asarray(x, np.float64)) <= 1)
