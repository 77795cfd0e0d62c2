"""ctypes binding of ``librepic_gc.so`` (C-ABI declared in ``include/repic_gc.h``).

The library is built in-tree by ``repic-copy_amd/csrc/Makefile`` (``__graft_entry__.build``).
Importing this module without the built library raises ImportError: there is no CPU
fallback for the hot path.
"""
from __future__ import annotations

import ctypes as C
import os
import weakref

import numpy as np

_HERE = os.path.dirname(os.path.abspath(__file__))
# REPIC_GC_LIB selects the diagnostic build (librepic_gc_diag.so) for tools/phase_stamps.py
LIB_PATH = os.environ.get("REPIC_GC_LIB") or os.path.join(_HERE, "librepic_gc.so")

if not os.path.exists(LIB_PATH):
    raise ImportError(
        f"{LIB_PATH} is missing: build it with `make -C repic-copy_amd/csrc` "
        "(or __graft_entry__.build()); the get_cliques hot path has no CPU fallback")

lib = C.CDLL(LIB_PATH)

F_GET_CC, F_MULTI_OUT, F_DEVICE_INPUTS, F_HOST_OUTPUTS, F_TIMING = 1, 2, 4, 8, 16
F_MEMBERS, F_NO_FUSED, F_DEVICE_META, F_EDGES = 32, 64, 128, 256
F_LAZY_STATS = 512   # ABI 6: per-micrograph outputs fetched on first use (rgc_fetch_stats)
OK, NO_EDGES, NO_CLIQUES = 0, 1, 2
PARSE_OK, PARSE_INDEX, PARSE_VALUE, PARSE_ASSERT, PARSE_FALLBACK, PARSE_OSERROR = range(6)
MAX_K = 8

_i32p = C.POINTER(C.c_int32)
_i64p = C.POINTER(C.c_int64)
_f64p = C.POINTER(C.c_double)
_f32p = C.POINTER(C.c_float)
_u8p = C.POINTER(C.c_uint8)


class BatchIn(C.Structure):
    _fields_ = [("n_mg", C.c_int32), ("k", C.c_int32), ("box_size", C.c_int64),
                ("flags", C.c_uint32), ("box_off", C.c_void_p), ("id_base", C.c_void_p),
                ("x", C.c_void_p), ("y", C.c_void_p), ("score", C.c_void_p),
                ("dev_box_off", C.c_void_p), ("dev_id_base", C.c_void_p)]


class BatchOut(C.Structure):
    _fields_ = [("n_boxes", C.c_int64), ("n_edges", C.c_int64), ("n_cliques", C.c_int64),
                ("status", _i32p), ("cc_max", _i32p), ("cc_cnt", _i32p), ("n_nodes", _i32p),
                ("n_vert", _i32p), ("n_edges_mg", _i64p), ("clique_base", _i64p),
                ("clique_cnt", _i64p),
                ("rows", C.c_void_p), ("w", C.c_void_p), ("conf", C.c_void_p),
                ("consensus", C.c_void_p), ("members", C.c_void_p), ("order", C.c_void_p)]


class Parsed(C.Structure):
    _fields_ = [("n_files", C.c_int64), ("status", _i32p), ("off", _i64p), ("x", _f64p),
                ("y", _f64p), ("score", _f64p), ("sigmoid", _u8p)]


class PickleFmt(C.Structure):
    _fields_ = [("arr_mod", C.c_char_p), ("arr_fn", C.c_char_p), ("dtype_mod", C.c_char_p),
                ("dtype_cls", C.c_char_p), ("coo_mod", C.c_char_p), ("coo_cls", C.c_char_p),
                ("maxprint", C.c_int32)]


class WriteIn(C.Structure):
    _fields_ = [("out_dir", C.c_char_p), ("n_mg", C.c_int32), ("k", C.c_int32),
                ("bases", C.POINTER(C.c_char_p)), ("clique_off", C.c_void_p),
                ("n_vert", C.c_void_p), ("cc_max", C.c_void_p), ("cc_cnt", C.c_void_p),
                ("seconds", C.c_void_p), ("w", C.c_void_p), ("conf", C.c_void_p),
                ("rows", C.c_void_p), ("cx", C.c_void_p), ("cy", C.c_void_p),
                ("cid", C.c_void_p)]


lib.rgc_abi_version.restype = C.c_int
lib.rgc_last_error.restype = C.c_char_p
lib.rgc_device_count.argtypes = [C.POINTER(C.c_int)]
lib.rgc_ctx_create.argtypes = [C.c_int, C.c_void_p, C.POINTER(C.c_void_p)]
lib.rgc_ctx_destroy.argtypes = [C.c_void_p]
lib.rgc_ctx_set_copy_stream.argtypes = [C.c_void_p, C.c_void_p]
lib.rgc_ctx_destroy.restype = None
lib.rgc_run.argtypes = [C.c_void_p, C.POINTER(BatchIn), C.POINTER(BatchOut)]
lib.rgc_submit.argtypes = [C.c_void_p, C.POINTER(BatchIn)]
lib.rgc_wait.argtypes = [C.c_void_p, C.POINTER(BatchOut)]
lib.rgc_fetch_stats.argtypes = [C.c_void_p]
lib.rgc_detach_host.argtypes = [C.c_void_p, C.POINTER(C.c_void_p)]
lib.rgc_host_block_free.argtypes = [C.c_void_p]
lib.rgc_host_block_free.restype = None
lib.rgc_last_edges.argtypes = [C.c_void_p, C.POINTER(_i32p), C.POINTER(_i32p),
                               C.POINTER(_f64p)]
lib.rgc_last_edges.restype = C.c_int64
lib.rgc_kernel_times.argtypes = [C.c_void_p, C.c_int, _f32p, C.POINTER(C.c_char_p)]
lib.rgc_parse_files.argtypes = [C.POINTER(C.c_char_p), C.c_int64, C.c_int,
                                C.POINTER(C.POINTER(Parsed))]
lib.rgc_parsed_free.argtypes = [C.POINTER(Parsed)]
lib.rgc_parsed_free.restype = None
lib.rgc_py_hash_node.argtypes = [C.c_double, C.c_double, C.c_int64]
lib.rgc_py_hash_node.restype = C.c_uint64
lib.rgc_py_set_order.argtypes = [C.POINTER(C.c_uint64), C.c_int, C.POINTER(C.c_int8)]
lib.rgc_test_epilogue.argtypes = [C.c_int, _f64p, _f64p, _f64p, C.POINTER(C.c_int64), _f64p,
                                  C.c_int, C.POINTER(C.c_uint64), C.POINTER(C.c_int),
                                  C.POINTER(C.c_int8), _f32p, _f32p]

lib.rgc_write_outputs.argtypes = [C.POINTER(PickleFmt), C.POINTER(WriteIn), C.c_int,
                                  C.POINTER(C.c_int64)]
lib.rgc_pickle_bytes.argtypes = [C.POINTER(PickleFmt), C.POINTER(WriteIn), C.c_int, C.c_int,
                                 C.c_void_p, C.c_int64, C.POINTER(C.c_int64)]
lib.rgc_py_float_repr.argtypes = [C.c_double, C.c_char_p, C.c_int]

EXPORTS = ["rgc_abi_version", "rgc_last_error", "rgc_device_count", "rgc_ctx_create",
           "rgc_ctx_destroy", "rgc_ctx_set_copy_stream", "rgc_run", "rgc_submit", "rgc_wait", "rgc_fetch_stats", "rgc_detach_host", "rgc_host_block_free", "rgc_kernel_times", "rgc_last_edges", "rgc_parse_files",
           "rgc_parsed_free", "rgc_py_hash_node", "rgc_py_set_order", "rgc_test_epilogue",
           "rgc_score_pairs", "rgc_ilp_solve", "rgc_write_outputs", "rgc_pickle_bytes",
           "rgc_py_float_repr"]


class RGCError(RuntimeError):
    pass


def _check(rc):
    if rc < 0:
        raise RGCError(lib.rgc_last_error().decode(errors="replace"))
    return rc


def abi_version() -> int:
    return lib.rgc_abi_version()


def ilp_big_max() -> int:
    """Largest conflict component (cliques) the run_ilp branch and bound searches
    (rgc_ilp.hip ILP_BIG); larger ones are certified, not searched."""
    return 4096


# ----------------------------------------------------------------------------- parsing
def parse_files(paths, n_threads=None):
    """Parse BOX files with the C++ parser -> (status[n], off[n+1], x, y, score, sigmoid)."""
    n = len(paths)
    arr = (C.c_char_p * max(n, 1))(*[os.fsencode(p) for p in paths])
    out = C.POINTER(Parsed)()
    if n_threads is None:
        n_threads = min(16, os.cpu_count() or 1)
    _check(lib.rgc_parse_files(arr, n, int(n_threads), C.byref(out)))
    # the library-owned x / y / score arrays are handed out without a copy: each numpy view's
    # base is a ctypes array holding the owner, which frees them when the last view is gone
    owner = _ParsedOwner(out)
    P = out.contents
    status = np.ctypeslib.as_array(P.status, shape=(n,)).copy() if n else np.zeros(0, np.int32)
    off = np.ctypeslib.as_array(P.off, shape=(n + 1,)).copy()
    tot = int(off[-1])
    if tot:
        x, y, s = (owner.view(p, tot) for p in (P.x, P.y, P.score))
    else:
        x = y = s = np.zeros(0, np.float64)
    sig = (np.ctypeslib.as_array(P.sigmoid, shape=(n,)).astype(bool) if n
           else np.zeros(0, bool))
    return status, off, x, y, s, sig


class _ParsedOwner:
    """Frees an rgc_parsed once no numpy view of its arrays is left."""

    def __init__(self, ptr):
        self.ptr = ptr

    def view(self, p, n):
        ca = (C.c_double * n).from_address(C.cast(p, C.c_void_p).value)
        ca._owner = self
        return np.frombuffer(ca, dtype=np.float64)

    def __del__(self):
        try:
            lib.rgc_parsed_free(self.ptr)
        except Exception:  # noqa: BLE001 - interpreter shutdown
            pass


# ----------------------------------------------------------------------------- CPython set order
def py_hash_node(x: float, y: float, node_id: int) -> int:
    return int(lib.rgc_py_hash_node(x, y, node_id))


def py_set_order(hashes):
    n = len(hashes)
    h = (C.c_uint64 * max(n, 1))(*[int(v) & 0xFFFFFFFFFFFFFFFF for v in hashes])
    o = (C.c_int8 * max(n, 1))()
    _check(lib.rgc_py_set_order(h, n, o))
    return [o[i] for i in range(n)]


def test_epilogue(x, y, score, ids, ji, set_order=True, ins=None):
    """The device ILP epilogue of one clique, run on the host (test hook):
    -> (consensus member index, node-iteration order, w, conf)."""
    k = len(x)
    f = lambda a: np.ascontiguousarray(a, dtype=np.float64)  # noqa: E731
    xa, ya, sa, ja = f(x), f(y), f(score), f(np.asarray(ji).reshape(k * k))
    ia = np.ascontiguousarray(ids, dtype=np.int64)
    insa = None if ins is None else (C.c_uint64 * k)(*[int(v) for v in ins])
    arg = C.c_int(0)
    ordr = (C.c_int8 * k)()
    w, conf = C.c_float(0), C.c_float(0)
    p64 = lambda a: a.ctypes.data_as(_f64p)  # noqa: E731
    _check(lib.rgc_test_epilogue(k, p64(xa), p64(ya), p64(sa),
                                 ia.ctypes.data_as(C.POINTER(C.c_int64)), p64(ja),
                                 int(set_order), insa, C.byref(arg), ordr, C.byref(w),
                                 C.byref(conf)))
    return arg.value, [ordr[i] for i in range(k)], np.float32(w.value), np.float32(conf.value)


# ----------------------------------------------------------------------------- device context
def device_count() -> int:
    n = C.c_int(0)
    _check(lib.rgc_device_count(C.byref(n)))
    return n.value


class _HostLease:
    """Owner of one run's host output buffers.  Every numpy view a :class:`Result` hands out
    keeps it alive.  While the context still owns the buffers (``block`` None) nothing is
    done; once the context moves on (next run, ILP / score call, close) while this lease is
    still referenced, the context detaches the buffers into ``block`` (rgc_detach_host, ABI 7)
    and they are freed here when the last view is gone."""

    __slots__ = ("block", "__weakref__")

    def __init__(self):
        self.block = None

    def view(self, p, ct, n):
        """numpy view of n elements of ctypes type ct at address p, owned by this lease"""
        ca = (ct * n).from_address(p)
        ca._owner = self
        return np.ctypeslib.as_array(ca)

    def __del__(self):
        if self.block:
            try:
                lib.rgc_host_block_free(self.block)
            except Exception:  # noqa: BLE001 - interpreter shutdown
                pass


class Context:
    """One device + stream; owns the device workspace arena (grow-only)."""

    def __init__(self, device: int = 0, stream: int | None = None):
        self._p = C.c_void_p()
        _check(lib.rgc_ctx_create(int(device), C.c_void_p(stream or 0), C.byref(self._p)))
        self.device = device
        self._pending = None
        self._lease = None   # weakref to the _HostLease of the last Result

    def set_copy_stream(self, stream: int):
        """Stream of the per-micrograph stats copy of non-lazy submits (0: the null stream);
        by default all contexts share one copy stream per device (rgc_ctx_set_copy_stream)."""
        _check(lib.rgc_ctx_set_copy_stream(self._p, C.c_void_p(stream or 0)))

    def _retire(self):
        """Before anything that may reuse or free the context's host buffers: if the last
        Result (or any array taken from it) is still referenced, hand its buffers over to it."""
        ref = self._lease
        lease = ref() if ref is not None else None
        if lease is not None and lease.block is None and self._p:
            h = C.c_void_p()
            # (the lease is dropped only once the hand-over succeeded: after a failed detach
            # the next retire, or close(), tries again)
            _check(lib.rgc_detach_host(self._p, C.byref(h)))
            lease.block = h.value
        self._lease = None

    def _result(self, bo, n_mg, k, flags, lazy_ctx=None):
        lease = _HostLease()
        self._lease = weakref.ref(lease)
        return Result(bo, n_mg, k, flags, lazy_ctx, lease)

    def close(self):
        if self._p:
            if self._pending is None:
                self._retire()
            lib.rgc_ctx_destroy(self._p)
            self._p = C.c_void_p()

    def __del__(self):
        try:
            self.close()
        except Exception:  # noqa: BLE001
            pass

    def run(self, n_mg, k, box_size, box_off, id_base, x, y, score, flags=F_HOST_OUTPUTS,
            dev_meta=None):
        """Run the batched pipeline.  ``box_off``/``id_base`` are host int64 arrays;
        ``x``/``y``/``score`` are host float64 arrays, or device pointers (ints) with
        ``F_DEVICE_INPUTS``.  ``dev_meta`` = (device pointer of box_off as int32, device
        pointer of id_base) sets ``F_DEVICE_META``: the offsets are not uploaded per run.
        Returns a :class:`Result`; its host arrays stay valid as long as they are referenced
        (rgc_detach_host hands them over when the context moves on)."""
        bi, keep, flags = self._batch_in(n_mg, k, box_size, box_off, id_base, x, y, score, flags,
                                         dev_meta)
        self._retire()
        bo = BatchOut()
        _check(lib.rgc_run(self._p, C.byref(bi), C.byref(bo)))
        del keep
        return self._result(bo, n_mg, k, flags)

    def submit(self, n_mg, k, box_size, box_off, id_base, x, y, score, flags=F_HOST_OUTPUTS,
               dev_meta=None):
        """``run`` without waiting (rgc_submit): the batch is enqueued on the context's stream
        and :meth:`wait` returns its :class:`Result`.  One submission in flight per context;
        two contexts overlap the host side of batch i+1 with the device work of batch i, and on
        two streams also the two batches' kernels (bench.py's default).  A batch that needs the
        general path (large micrographs) runs on the context's worker thread until ``wait``.
        The arrays passed in must stay alive until ``wait`` (kept here)."""
        bi, keep, flags = self._batch_in(n_mg, k, box_size, box_off, id_base, x, y, score, flags,
                                         dev_meta)
        self._retire()
        _check(lib.rgc_submit(self._p, C.byref(bi)))
        self._pending = (keep, n_mg, k, flags)

    def wait(self):
        if self._pending is None:
            raise RGCError("rgc_wait: no submission in flight on this context")
        bo = BatchOut()
        keep, n_mg, k, flags = self._pending
        self._pending = None
        _check(lib.rgc_wait(self._p, C.byref(bo)))
        del keep
        return self._result(bo, n_mg, k, flags, self)

    def _batch_in(self, n_mg, k, box_size, box_off, id_base, x, y, score, flags, dev_meta):
        # (kept lean: this runs once per batch inside the bench's timed region)
        if not (type(box_off) is np.ndarray and box_off.dtype == np.int64
                and box_off.flags.c_contiguous):
            box_off = np.ascontiguousarray(box_off, dtype=np.int64)
        if not (type(id_base) is np.ndarray and id_base.dtype == np.int64
                and id_base.flags.c_contiguous):
            id_base = np.ascontiguousarray(id_base, dtype=np.int64)
        assert box_off.shape == (n_mg * k + 1,) and id_base.shape == (n_mg,)
        keep = [box_off, id_base]
        if flags & F_DEVICE_INPUTS:
            px, py, ps = int(x), int(y), int(score)
        else:
            x, y, score = (np.ascontiguousarray(v, dtype=np.float64) for v in (x, y, score))
            n = int(box_off[-1]) if len(box_off) else 0
            assert x.shape == y.shape == score.shape == (n,)
            keep += [x, y, score]
            px, py, ps = x.ctypes.data, y.ctypes.data, score.ctypes.data
        dbo = did = None
        if dev_meta is not None:
            flags |= F_DEVICE_META
            dbo, did = int(dev_meta[0]), int(dev_meta[1])
        bi = BatchIn(n_mg, k, int(box_size), flags, box_off.ctypes.data, id_base.ctypes.data,
                     px, py, ps, dbo, did)
        return bi, keep, flags

    def last_edges(self):
        """Test hook: (u, v, ji) copies of the JI > 0.3 edges of the last run with F_EDGES
        (batch box indices; order unspecified)."""
        u, v, j = _i32p(), _i32p(), _f64p()
        n = _check(lib.rgc_last_edges(self._p, C.byref(u), C.byref(v), C.byref(j)))
        if n == 0:
            return np.zeros(0, np.int32), np.zeros(0, np.int32), np.zeros(0)
        return (np.ctypeslib.as_array(u, shape=(n,)).copy(),
                np.ctypeslib.as_array(v, shape=(n,)).copy(),
                np.ctypeslib.as_array(j, shape=(n,)).copy())

    def kernel_times(self):
        n = lib.rgc_kernel_times(self._p, 0, None, None)
        ms = (C.c_float * max(n, 1))()
        names = (C.c_char_p * max(n, 1))()
        lib.rgc_kernel_times(self._p, n, ms, names)
        return [(names[i].decode(), float(ms[i])) for i in range(n)]


class Result:
    """Host view of one rgc_run.  Per-micrograph and per-clique arrays are numpy views of
    pinned memory (per-clique arrays: device pointers without F_HOST_OUTPUTS).  The host views
    stay valid, with this run's values, for as long as they (or this Result) are referenced:
    each holds the run's :class:`_HostLease`, and the context hands the buffers over to it
    (rgc_detach_host) instead of reusing or freeing them.  Device pointers follow the C-ABI
    rule: valid until the next run on the context."""

    _PER_MG = {"status": ("status", np.int32), "cc_max": ("cc_max", np.int32),
               "cc_cnt": ("cc_cnt", np.int32), "n_nodes": ("n_nodes", np.int32),
               "n_vert": ("n_vert", np.int32), "n_edges_mg": ("n_edges_mg", np.int64),
               "clique_base": ("clique_base", np.int64), "clique_cnt": ("clique_cnt", np.int64)}

    def __getattr__(self, name):
        # per-micrograph arrays are built on first use (views, no copy)
        spec = Result._PER_MG.get(name)
        if spec is None:
            raise AttributeError(name)
        field, dt = spec
        dt = np.dtype(dt)
        if self._lazy is not None:   # F_LAZY_STATS: copied from HBM on first use
            # (once the buffers were detached, rgc_detach_host has fetched them already)
            if self._lease.block is None:
                _check(lib.rgc_fetch_stats(self._lazy._p))
            self._lazy = None
        p = getattr(self._bo, field)
        if not self.n_mg or not p:
            v = np.zeros(0, dt)
        else:
            addr = C.cast(p, C.c_void_p).value
            ct = {4: C.c_int32, 8: C.c_int64}[dt.itemsize]
            v = self._lease.view(addr, ct, self.n_mg).view(dt)
        setattr(self, name, v)
        return v

    def __init__(self, bo: BatchOut, n_mg: int, k: int, flags: int, ctx=None, lease=None):
        self._bo = bo
        self._lease = lease if lease is not None else _HostLease()
        self._lazy = ctx if (flags & F_LAZY_STATS) and ctx is not None else None
        self.n_mg, self.k = n_mg, k
        self.n_boxes, self.n_edges, self.n_cliques = bo.n_boxes, bo.n_edges, bo.n_cliques
        C_ = int(self.n_cliques)
        if flags & F_HOST_OUTPUTS:
            def h(p, ct, n):
                if not n or not p:
                    return np.zeros(n, dtype=np.dtype(ct))
                return self._lease.view(C.cast(p, C.c_void_p).value, ct, n)
            self.rows = h(bo.rows, C.c_int32, C_ * k).reshape(C_, k)
            self.w = h(bo.w, C.c_float, C_)
            self.conf = h(bo.conf, C.c_float, C_)
            self.consensus = h(bo.consensus, C.c_int32, C_)
            self.members = (h(bo.members, C.c_int32, C_ * k).reshape(C_, k)
                            if (flags & (F_MULTI_OUT | F_MEMBERS)) else None)
            self.order = (h(bo.order, C.c_uint8, C_ * k).reshape(C_, k)
                          if (flags & F_MULTI_OUT) else None)
        else:
            self.rows, self.w, self.conf = bo.rows, bo.w, bo.conf
            self.consensus, self.members, self.order = bo.consensus, bo.members, bo.order
