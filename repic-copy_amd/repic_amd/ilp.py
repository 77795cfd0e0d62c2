"""Exact max-weight set packing on the device (the ILP of reference run_ilp.py:50-63).

``solve_batch`` packs many micrographs' constraint matrices into one CSC problem (rows are
offset per micrograph, so micrographs never share a row) and calls ``rgc_ilp_solve``
(rgc_ilp.hip): conflict components by union-find, one thread per component of <= 64 cliques,
one wavefront per larger one, exact branch and bound.  No CPU fallback.
"""
from __future__ import annotations

import ctypes as C

import numpy as np

from . import _lib


class IlpIn(C.Structure):
    _fields_ = [("n_cols", C.c_int64), ("n_rows", C.c_int64), ("col_ptr", C.c_void_p),
                ("row_idx", C.c_void_p), ("w", C.c_void_p), ("node_limit", C.c_int64),
                ("flags", C.c_uint32), ("gap", C.c_void_p), ("time_limit_s", C.c_double)]


_lib.lib.rgc_ilp_solve.argtypes = [C.c_void_p, C.POINTER(IlpIn), C.c_void_p, C.c_void_p]
_lib.lib.rgc_ilp_solve.restype = C.c_int


def pack(mats):
    """CSC arrays of a batch of sparse (V_m x C_m) matrices: (col_ptr, row_idx, n_rows,
    col_off) with micrograph m's rows offset by the rows of the ones before it."""
    ptrs, idxs, col_off, row0, nnz0 = [np.zeros(1, np.int64)], [], [0], 0, 0
    for A in mats:
        csc = A.tocsc()
        ptrs.append(csc.indptr[1:].astype(np.int64) + nnz0)
        idxs.append(csc.indices.astype(np.int64) + row0)
        nnz0 += int(csc.indptr[-1])
        row0 += A.shape[0]
        col_off.append(col_off[-1] + A.shape[1])
    col_ptr = np.concatenate(ptrs)
    row_idx = (np.concatenate(idxs) if idxs else np.zeros(0, np.int64)).astype(np.int32)
    return col_ptr, row_idx, row0, np.asarray(col_off, np.int64)


# component statuses (include/repic_gc.h RGC_ILP_*)
NODE_LIMIT, OPTIMAL, GAP_OK, HEURISTIC = 0, 1, 2, 3


def mg_status(ex, gap=0.0, primal=0.0):
    """A micrograph's status.  OPTIMAL when every conflict component was proven optimal;
    else GAP_OK when the summed dual-bound gaps of its components are within 1e-4 of its
    objective - the relative MIPGap at which Gurobi reports the micrograph's model optimal
    (run_ilp.py:50-63 solves one model per micrograph, default parameters); else the weakest
    component status (HEURISTIC < NODE_LIMIT)."""
    if len(ex) == 0 or (ex == OPTIMAL).all():
        return OPTIMAL
    if gap <= 1e-4 * abs(primal):
        return GAP_OK
    for st in (HEURISTIC, NODE_LIMIT):
        if (ex == st).any():
            return st
    return GAP_OK


def solve_batch(ctx, mats, weights, node_limit=0, timing=False, statuses=False, gaps=False):
    """Returns (x list of uint8 arrays, exact list of bool): per micrograph the chosen
    columns and whether every component was proven optimal (with ``statuses``: the
    micrograph status codes, mg_status, instead of the bools; with ``gaps`` also the
    micrograph's relative gap bound, sum of component gaps / objective).  The search is
    bounded by ``node_limit`` nodes per component (0: the library default) and nothing else,
    so the result is the same on every run and device."""
    col_ptr, row_idx, n_rows, col_off = pack(mats)
    w = np.ascontiguousarray(np.concatenate([np.asarray(v, np.float64).ravel() for v in weights])
                             if weights else np.zeros(0), dtype=np.float64)
    nc = len(col_ptr) - 1
    assert len(w) == nc, (len(w), nc)
    if n_rows >= 2 ** 31 or nc >= 2 ** 31:
        raise _lib.RGCError("batch too large for 32-bit row / column ids")
    x = np.zeros(nc, np.uint8)
    ex = np.zeros(nc, np.uint8)
    gp = np.zeros(nc, np.float64)
    si = IlpIn(nc, n_rows, col_ptr.ctypes.data, row_idx.ctypes.data, w.ctypes.data,
               int(node_limit), _lib.F_TIMING if timing else 0, gp.ctypes.data,
               0.0)   # (time_limit_s: ignored since ABI 9)
    ctx._retire()   # a live Result of an earlier run keeps its host buffers
    _lib._check(_lib.lib.rgc_ilp_solve(ctx._p, C.byref(si), x.ctypes.data, ex.ctypes.data))
    xs = [x[col_off[m]:col_off[m + 1]] for m in range(len(mats))]
    st, rel = [], []
    for m in range(len(mats)):
        a, b = col_off[m], col_off[m + 1]
        primal = float(w[a:b][x[a:b] == 1].sum())
        g = float(gp[a:b].sum())
        st.append(mg_status(ex[a:b], g, primal))
        rel.append(g / primal if primal > 0 else (0.0 if g == 0 else float("inf")))
    if statuses:
        return (xs, st, rel) if gaps else (xs, st)
    return xs, [s_ == OPTIMAL for s_ in st]
