"""Per-micrograph output files, exactly the set the reference writes.

reference get_cliques.py:125-129 (skip -> empty ``<base>.box``) and :204-229:
``<base>_weight_vector.pickle`` (float32[C]), ``<base>_consensus_coords.pickle`` (list of
``(x, y, id)`` tuples, or the ``--multi_out`` table), ``<base>_consensus_confidences.pickle``
(float32[C]), ``<base>_constraint_matrix.pickle`` (scipy ``coo_matrix``, int64 data, int32
indices, shape (V, C)) and ``<base>_runtime.tsv`` ("seconds\\tlargest CC\\tnumber of CCs").
All pickles use ``pickle.HIGHEST_PROTOCOL`` so the unchanged ``run_ilp`` reads them.

Plain micrographs are written by the library's native writer (``rgc_write_outputs``,
csrc/out_write.cpp: the same pickle opcodes, emitted in C++ from threads without the GIL) once
``native_format()`` has checked its bytes against ``pickle.dumps`` of the same objects for the
installed numpy / scipy; otherwise (and for ``--multi_out`` tables and skipped micrographs)
Python pickles them.
"""
from __future__ import annotations

import os
import time
import pickle
from concurrent.futures import ThreadPoolExecutor

import numpy as np
from scipy.sparse import coo_matrix

LABELS = ("weight_vector", "consensus_coords", "consensus_confidences", "constraint_matrix")
# coo_matrix.__dict__ keys the native writer emits (scipy >= 1.13 layout)
_COO_KEYS = ["_shape", "maxprint", "coords", "data", "has_canonical_format"]
_NATIVE = None


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


def write_micrograph_raw(out_dir, base, w, conf, rows, n_vert, cx, cy, cid, coords, seconds,
                         cc_max, cc_cnt):
    """write_micrograph from the device results: the consensus tuples and the COO matrix are
    built here (in the writer thread or process), not on the submitting thread."""
    if coords is None:
        coords = consensus_coords(cx, cy, cid)
    write_micrograph(out_dir, base, w, coords, conf, constraint_matrix(rows, n_vert), seconds,
                     cc_max, cc_cnt)


def _strip_frame(b: bytes) -> bytes:
    """pickle.dumps output without its FRAME opcode (one frame for small objects)."""
    return b[:2] + b[11:] if len(b) > 11 and b[2] == 0x95 else b


def _fmt_from_installed():
    """rgc_pickle_fmt from the installed numpy / scipy, or None if their pickle layout is not
    the one csrc/out_write.cpp emits."""
    from . import _lib
    a = np.zeros(2, np.float32)
    fn, args = a.__reduce_ex__(pickle.HIGHEST_PROTOCOL)
    dt = np.dtype(np.float32).__reduce__()
    A = constraint_matrix(np.zeros((1, 2), np.int32), 1)
    if (len(args) != 4 or args[3] != "C" or dt[0] is not np.dtype
            or list(A.__dict__) != _COO_KEYS or dt[2][:2] != (3, "<")):
        return None
    keep = [x.encode() for x in (fn.__module__, fn.__name__, dt[0].__module__, dt[0].__name__,
                                 type(A).__module__, type(A).__name__)]
    f = _lib.PickleFmt(*keep, int(A.maxprint))
    return f, keep


def _write_in(out_dir, bases, k, offs, n_vert, cc_max, cc_cnt, seconds, w, conf, rows, cx, cy,
              cid):
    """rgc_write_in over contiguous arrays (returned with everything it points into)."""
    import ctypes as C

    from . import _lib
    arrs = [np.ascontiguousarray(offs, np.int64), np.ascontiguousarray(n_vert, np.int32),
            np.ascontiguousarray(cc_max, np.int32), np.ascontiguousarray(cc_cnt, np.int32),
            np.ascontiguousarray(seconds, np.float64), np.ascontiguousarray(w, np.float32),
            np.ascontiguousarray(conf, np.float32), np.ascontiguousarray(rows, np.int32),
            np.ascontiguousarray(cx, np.float64), np.ascontiguousarray(cy, np.float64),
            np.ascontiguousarray(cid, np.int64)]
    bs = (C.c_char_p * max(1, len(bases)))(*[os.fsencode(b) for b in bases])
    wi = _lib.WriteIn(os.fsencode(out_dir), len(bases), k, bs, *[a.ctypes.data for a in arrs])
    return wi, (arrs, bs)


def native_format():
    """The native writer's format (cached), after a byte-for-byte check of all four pickles of
    sample micrographs (ids across the pickle's int encodings, 1 and 1001 cliques) against
    pickle.dumps; None when the check fails or the library is unavailable."""
    global _NATIVE
    if _NATIVE is not None:
        return _NATIVE or None
    _NATIVE = False
    try:
        import ctypes as C

        from . import _lib
        got = _fmt_from_installed()
        if got is None:
            return None
        fmt, keep = got
        rng = np.random.default_rng(5)
        k = 3
        cnt = [1, 1001, 4]
        offs = np.concatenate([[0], np.cumsum(cnt)])
        C_ = int(offs[-1])
        w = rng.random(C_).astype(np.float32)
        conf = rng.random(C_).astype(np.float32)
        rows = np.sort(rng.integers(0, 300, (C_, k)), axis=1).astype(np.int32)
        cx = np.round(rng.random(C_) * 4000, 3)
        cy = rng.random(C_) * 1e-7
        cid = rng.choice(np.array([0, 255, 256, 65535, 65536, 2**31 - 1, 2**31, 2**40], np.int64),
                         C_)
        n_vert = np.array([300, 65536, 3000], np.int32)
        wi, hold = _write_in("/nonexistent", ["a", "b", "c"], k, offs, n_vert, [1, 2, 3],
                             [4, 5, 6], [0.5, 1e-5, 1e17], w, conf, rows, cx, cy, cid)
        for m in range(3):
            c0, c1 = int(offs[m]), int(offs[m + 1])
            objs = (w[c0:c1], consensus_coords(cx[c0:c1], cy[c0:c1], cid[c0:c1]), conf[c0:c1],
                    constraint_matrix(rows[c0:c1], int(n_vert[m])))
            for which, obj in enumerate(objs):
                want = _strip_frame(pickle.dumps(obj, protocol=pickle.HIGHEST_PROTOCOL))
                n = C.c_int64()
                buf = C.create_string_buffer(len(want) + 64)
                rc = _lib.lib.rgc_pickle_bytes(C.byref(fmt), C.byref(wi), m, which, buf,
                                               len(want) + 64, C.byref(n))
                if rc != 0 or buf.raw[:n.value] != want:
                    return None
        for v in (0.0, 1.5, 2.0, 1e-4, 1e-5, 1e16, 1e17, 123.456, 1 / 3, 2.5e-300):
            b = C.create_string_buffer(64)
            if _lib.lib.rgc_py_float_repr(v, b, 64) < 0 or b.value.decode() != str(v):
                return None
        _NATIVE = (fmt, keep)
    except Exception:  # noqa: BLE001 - any failure: Python writer
        _NATIVE = False
    return _NATIVE or None


def write_group_native(fmt, out_dir, items, w, conf, rows, cx, cy, cid):
    """write_group through rgc_write_outputs (one thread; callers run groups in parallel):
    skipped micrographs get their empty .box from Python."""
    import ctypes as C

    from . import _lib
    bases, offs, nv, cm, cc, sec = [], [0], [], [], [], []
    for base, n, n_vert, cc_max, cc_cnt, seconds, coords in items:
        if n < 0:
            write_skip(out_dir, base)
            continue
        assert coords is None
        bases.append(base)
        offs.append(offs[-1] + n)
        nv.append(n_vert)
        cm.append(cc_max)
        cc.append(cc_cnt)
        sec.append(seconds)
    if not bases:
        return
    k = rows.shape[1] if rows.ndim == 2 else 1
    wi, hold = _write_in(out_dir, bases, k, offs, nv, cm, cc, sec, w, conf, rows, cx, cy, cid)
    bad = C.c_int64(-1)
    rc = _lib.lib.rgc_write_outputs(C.byref(fmt[0]), C.byref(wi), 1, C.byref(bad))
    if rc != 0:
        b = bases[bad.value] if 0 <= bad.value < len(bases) else out_dir
        raise OSError(-rc, os.strerror(-rc), os.path.join(out_dir, b))


def _write_chunk(items):
    """Writer-process task: a chunk of (kind, args) writes, in order."""
    for kind, args in items:
        if kind == 0:
            write_skip(*args)
        elif kind == 1:
            write_micrograph_raw(*args)
        else:
            write_group(*args)
    return len(items)


def write_group(out_dir, items, w, conf, rows, cx, cy, cid):
    """Writer task for a group of micrographs in reference order, from flat arrays over the
    group's cliques (micrograph by micrograph): ``items`` = (base, n_cliques, n_vert, cc_max,
    cc_cnt, seconds, coords) per micrograph, or (base, -1, ...) for a skipped one (empty
    ``<base>.box``); ``coords`` is the prebuilt --multi_out table, else None and the
    consensus tuples come from cx / cy / cid."""
    c0 = 0
    for base, n, n_vert, cc_max, cc_cnt, seconds, coords in items:
        if n < 0:
            write_skip(out_dir, base)
            continue
        c1 = c0 + n
        write_micrograph_raw(out_dir, base, w[c0:c1], conf[c0:c1], rows[c0:c1], n_vert,
                             cx[c0:c1] if coords is None else None,
                             cy[c0:c1] if coords is None else None,
                             cid[c0:c1] if coords is None else None, coords, seconds, cc_max,
                             cc_cnt)
        c0 = c1


# the files written per micrograph (get_cliques.py:123-130, 215-229): the empty <base>.box
# of a skip, or the four pickles and the runtime.tsv of a micrograph with cliques
SKIP_FILES = (".box",)
OK_FILES = ("_weight_vector.pickle", "_consensus_coords.pickle",
            "_consensus_confidences.pickle", "_constraint_matrix.pickle", "_runtime.tsv")


class Writer:
    """Pooled writer.  Pickling the per-micrograph objects holds the GIL, so large runs write
    from a pool of spawned processes (started early, chunks of ``chunk`` micrographs per
    task, raw arrays shipped, objects built in the worker); small runs use threads (file
    creation releases the GIL).  ``close()`` waits for every pending write and re-raises the
    first I/O error, so the files of every micrograph before a crash exist, as in the
    reference."""

    def __init__(self, threads=None, processes=False, chunk=32, native=True):
        self.threads = threads or min(16, (os.cpu_count() or 1))
        # the native writer needs no interpreter per worker: threads instead of processes
        self.native = native_format() if native else None
        if self.native is not None:
            # file creation in one directory serialises on its inode lock: a few writer
            # threads saturate it (more only contend); RGC_WRITER_THREADS overrides
            self.threads = max(1, min(self.threads, int(os.environ.get("RGC_WRITER_THREADS", 4))))
        self.procs = bool(processes) and self.threads > 1 and self.native is None
        self.chunk = chunk
        if self.procs:
            import multiprocessing as mp
            from concurrent.futures import ProcessPoolExecutor
            self._pool = ProcessPoolExecutor(self.threads, mp_context=mp.get_context("spawn"))
            for _ in range(self.threads):   # start the workers now: they import while the
                self._pool.submit(_write_chunk, [])   # device runs
        else:
            self._pool = ThreadPoolExecutor(max_workers=self.threads) if self.threads > 1 else None
        self._futs = []
        self._bases = set()
        self._items = []
        # (base, suffixes) of every file set handed to the pool, in submission order
        self.written = []
        # optional timeline: ("write", first base, submit, done) seconds after t0, per group
        self.spans, self.t0 = None, 0.0

    def _submit(self, kind, args):
        base = args[1]
        if base in self._bases:      # same output name twice: keep the reference's order
            self._flush()
            self._drain()
        self._bases.add(base)
        if self._pool is None:
            _write_chunk([(kind, args)])
        elif self.procs:
            self._items.append((kind, args))
            if len(self._items) >= self.chunk:
                self._flush()
        else:
            self._futs.append(self._pool.submit(_write_chunk, [(kind, args)]))
        if len(self._futs) > 4 * self.threads:
            self._drain(len(self._futs) // 2)

    def _flush(self):
        if self._items:
            self._futs.append(self._pool.submit(_write_chunk, self._items))
            self._items = []

    def _drain(self, n=None):
        n = len(self._futs) if n is None else n
        done, self._futs = self._futs[:n], self._futs[n:]
        for f in done:
            f.result()

    def skip(self, out_dir, base):
        self.written.append((base, SKIP_FILES))
        self._submit(0, (out_dir, base))

    def micrograph(self, out_dir, base, w, conf, rows, n_vert, cx, cy, cid, coords, seconds,
                   cc_max, cc_cnt):
        self.written.append((base, OK_FILES))
        self._submit(1, (out_dir, base, w, conf, rows, n_vert, cx, cy, cid, coords, seconds,
                         cc_max, cc_cnt))

    def group(self, out_dir, items, w, conf, rows, cx, cy, cid):
        """A group of micrographs (write_group) as one task; a base name already written
        earlier in the run waits for every pending write first (the reference's order)."""
        names = [it[0] for it in items]
        if any(b in self._bases for b in names):
            self._flush()
            self._drain()
        self._bases.update(names)
        self.written.extend((it[0], SKIP_FILES if it[1] < 0 else OK_FILES) for it in items)
        args = (out_dir, items, w, conf, rows, cx, cy, cid)
        t_sub = time.time()
        if self.native is not None and all(it[6] is None for it in items):
            if self._pool is None:
                write_group_native(self.native, *args)
                self._span(names, t_sub)
                return
            self._futs.append(self._pool.submit(write_group_native, self.native, *args))
        elif self._pool is None:
            write_group(*args)
            self._span(names, t_sub)
            return
        else:
            self._flush()
            self._futs.append(self._pool.submit(_write_chunk, [(2, args)]))
        if self.spans is not None:
            self._futs[-1].add_done_callback(lambda f, n=names, t=t_sub: self._span(n, t))
        if len(self._futs) > 4 * self.threads:
            self._drain(len(self._futs) // 2)

    def _span(self, names, t_sub):
        if self.spans is not None and names:
            self.spans.append(("write", names[0], t_sub - self.t0, time.time() - self.t0))

    def close(self):
        try:
            if self._pool is not None:
                self._flush()
            self._drain()
        finally:
            if self._pool is not None:
                self._pool.shutdown(wait=True)
