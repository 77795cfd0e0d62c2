"""BOX ingest: picker discovery, micrograph pairing, parsing and global box ids.

Mirrors the reference's file handling exactly (reference repic/commands/get_cliques.py
:74-130 and repic/utils/common.py:54-114) but replaces the O(M^2) per-micrograph
``glob('*base*')`` directory scans (get_cliques.py:94,121) with a one-pass directory index:

* ``glob.glob(dir/pattern)`` semantics = names of ``os.listdir(dir)`` in readdir order, hidden
  names skipped, matched with ``fnmatch.fnmatchcase``.  ``*base*`` for a base without glob
  magic characters is a substring test, answered from a substring index built once per
  (directory, base length); other patterns fall back to fnmatch over the listing.
* The C++ parser (``rgc_parse_files``) reproduces ``get_box_coords``' acceptance rules; files
  it flags as FALLBACK (non-ASCII bytes) are parsed here with Python's own str/float.
* Scores of a file with ``min(score) < 0`` go through the numpy sigmoid
  ``1 / (1 + np.exp(-s))`` (common.py:92-94), on the host, with numpy, so the bits match.
* Global box ids follow the reference's process-wide counter (common.py:23,108-112),
  including ids consumed by pickers loaded before a micrograph was skipped.
"""
from __future__ import annotations

import fnmatch
import os
from dataclasses import dataclass, field

import numpy as np

from . import _lib

_MAGIC = set("*?[")


def _has_magic(s: str) -> bool:
    return any(c in _MAGIC for c in s)


class DirIndex:
    """readdir-order listing of each picker directory with fast ``*base*`` lookups."""

    def __init__(self, in_dir: str, methods, listing=None):
        self.in_dir = in_dir
        self.names = {}
        for m in methods:
            if listing is not None and m in listing:
                names = list(listing[m])
            else:
                try:
                    names = os.listdir(os.path.join(in_dir, m))
                except (FileNotFoundError, NotADirectoryError):
                    names = []
            self.names[m] = [n for n in names if not n.startswith(".")]
        self._sub = {}

    def glob(self, method: str, pattern: str):
        """Names in ``method`` matching ``pattern`` (glob.glob semantics, readdir order)."""
        names = self.names.get(method, [])
        if pattern.startswith("*") and pattern.endswith("*") and len(pattern) >= 2:
            base = pattern[1:-1]
            if not _has_magic(base):
                return self._contains(method, base)
        return [n for n in names if fnmatch.fnmatchcase(n, pattern)]

    def _contains(self, method, base):
        L = len(base)
        if L == 0:
            return list(self.names.get(method, []))
        key = (method, L)
        idx = self._sub.get(key)
        if idx is None:
            idx = {}
            for pos, n in enumerate(self.names.get(method, [])):
                seen = set()
                for i in range(len(n) - L + 1):
                    s = n[i:i + L]
                    if s not in seen:
                        seen.add(s)
                        idx.setdefault(s, []).append(pos)
            self._sub[key] = idx
        names = self.names[method]
        return [names[p] for p in idx.get(base, ())]


def list_methods(in_dir: str):
    """Picker subdirectories, sorted by str (get_cliques.py:81-82)."""
    out = []
    for n in os.listdir(in_dir):
        if n.startswith("."):
            continue
        if os.path.isdir(os.path.join(in_dir, n)):
            out.append(n)
    return sorted(out, key=str)


def probe_start_method(index: DirIndex, methods):
    """The "start_method" probe of get_cliques.py:86-103 (same exceptions)."""
    start, n, seen_file = None, None, False
    for method in methods:
        files = index.glob(method, "*.box")
        if files:
            seen_file = True
            base = files[0].replace(".box", "")
            n = sum(len(index.glob(m, f"*{base}*")) for m in methods)
        if n is None:
            raise UnboundLocalError("local variable 'n' referenced before assignment")
        if n == len(methods):
            start = method
            break
    if start is None:
        raise AssertionError("Error - particle file names cannot be paired across methods")
    if not seen_file:
        raise UnboundLocalError("local variable 'box_file' referenced before assignment")
    return start


# ----------------------------------------------------------------------------- parsing
def _is_float(tok: str) -> bool:
    try:
        float(tok)
    except ValueError:
        return False
    return True


def _py_parse(path):
    """Python-semantics parse for files the C++ parser hands back (non-ASCII bytes)."""
    with open(path, "rt") as f:
        if _is_float(f.readline().rstrip().split()[0]):
            f.seek(0)
        X, Y, H, W, weights = zip(*[ln.strip().split() for ln in f])
    X = [float(v) for v in X if _is_float(v)]
    Y = [float(v) for v in Y if _is_float(v)]
    weights = [float(v) for v in weights]
    sig = bool(np.min(weights) < 0)
    assert len(X) == len(Y), "Error - unequal number of 'x' and 'y' elements"
    n = min(len(X), len(Y), len(weights))
    if n == 0:
        raise IndexError("list index out of range")
    return (np.array(X[:n], np.float64), np.array(Y[:n], np.float64),
            np.array(weights[:n], np.float64), sig)


class ParsedFile:
    __slots__ = ("exc", "x", "y", "s", "sigmoid")

    def __init__(self, exc=None, x=None, y=None, s=None, sigmoid=False):
        self.exc, self.x, self.y, self.s, self.sigmoid = exc, x, y, s, sigmoid

    @property
    def n(self):
        return 0 if self.x is None else len(self.x)


_EXC = {
    _lib.PARSE_INDEX: lambda p: IndexError("list index out of range"),
    _lib.PARSE_VALUE: lambda p: ValueError(f"malformed BOX file: {p}"),
    _lib.PARSE_ASSERT: lambda p: AssertionError("Error - unequal number of 'x' and 'y' elements"),
}


def parse_many(paths, n_threads=None):
    """Parse files (deduplicated by caller) -> list[ParsedFile]."""
    status, off, x, y, s, sig = _lib.parse_files(paths, n_threads)
    out = []
    for i, p in enumerate(paths):
        st = int(status[i])
        if st == _lib.PARSE_OK:
            xs, ys, ss = x[off[i]:off[i + 1]], y[off[i]:off[i + 1]], s[off[i]:off[i + 1]]
            out.append(ParsedFile(None, xs, ys, ss, bool(sig[i])))
        elif st == _lib.PARSE_FALLBACK:
            try:
                xs, ys, ss, sg = _py_parse(p)
                out.append(ParsedFile(None, xs, ys, ss, sg))
            except Exception as e:  # noqa: BLE001 - reproduced exception is the contract
                out.append(ParsedFile(e))
        elif st == _lib.PARSE_OSERROR:
            try:
                open(p, "rt").close()
                out.append(ParsedFile(OSError(f"cannot read {p}")))
            except OSError as e:
                out.append(ParsedFile(e))
        else:
            out.append(ParsedFile(_EXC[st](p)))
    return out


def sigmoid(s):
    """common.py:94 ``1. / (1. + np.exp(-1. * val))`` with numpy, elementwise."""
    return 1.0 / (1.0 + np.exp(-1.0 * s))


# ----------------------------------------------------------------------------- plan
@dataclass
class Micrograph:
    base: str                      # basename with every ".box" removed (get_cliques.py:112)
    files: list = field(default_factory=list)   # k lists of matching paths
    status: str = "ok"             # ok | skip | crash
    exc: BaseException | None = None
    id_base: int = 0
    coords: list = field(default_factory=list)  # k ParsedFile (ok micrographs; plan())
    slot: int = -1                 # index among the chunk's ok micrographs (plan_chunk())


def _glob_path_itself(path: str):
    """glob.glob(path) for the first picker's own file (get_cliques.py:120)."""
    d, name = os.path.split(path)
    if not _has_magic(name):
        return [path] if os.path.lexists(path) else []
    try:
        names = os.listdir(d)
    except OSError:
        return []
    return [os.path.join(d, n) for n in names
            if not n.startswith(".") and fnmatch.fnmatchcase(n, name)]


def micrograph_names(index: DirIndex, methods):
    """First-picker BOX files in readdir order = the reference's processing order (:108)."""
    return index.glob(methods[0], "*.box")


def plan(in_dir, methods, index: DirIndex, order=None, n_threads=None):
    """Enumerate micrographs in reference order, parse their files and assign box ids.

    ``order`` restricts/reorders the first-picker file names (a shard).  Ids start at 0 for
    the first listed micrograph; a sharded caller adds its global offset.  Returns
    ``(micrographs, crash_index, consumed)``: processing stops at the first micrograph that
    would crash the reference (its exception in ``exc``); skipped micrographs still consume
    the ids of the pickers loaded before the failing one.
    """
    first = order if order is not None else micrograph_names(index, methods)
    mgs = []
    for name in first:
        base = name.replace(".box", "")
        path0 = os.path.join(in_dir, methods[0], name)
        files = [_glob_path_itself(path0)]
        for m in methods[1:]:
            files.append([os.path.join(in_dir, m, n) for n in index.glob(m, f"*{base}*")])
        mgs.append(Micrograph(base=base, files=files))
    uniq = {}
    for mg in mgs:
        for fl in mg.files:
            for p in fl:
                uniq.setdefault(p, len(uniq))
    paths = list(uniq)
    parsed = parse_many(paths, n_threads) if paths else []
    next_id = 0
    crash = None
    for i, mg in enumerate(mgs):
        mg.id_base = next_id
        coords = []
        try:
            for fl in mg.files:
                if not fl:
                    raise UnboundLocalError("local variable 'i' referenced before assignment")
                pf = None
                for p in fl:
                    pf = parsed[uniq[p]]
                    if pf.exc is not None:
                        raise pf.exc
                if len(fl) > 1:
                    raise AssertionError("Error - multiple BOX files found using pattern")
                coords.append(pf)
                next_id += pf.n
        except (UnboundLocalError, IndexError):
            mg.status = "skip"
            continue
        except BaseException as e:  # noqa: BLE001
            mg.status, mg.exc = "crash", e
            crash = i
            break
        mg.coords = [ParsedFile(None, c.x, c.y, sigmoid(c.s) if c.sigmoid else c.s, c.sigmoid)
                     for c in coords]
    if crash is not None:
        mgs = mgs[:crash + 1]
    return mgs, crash, next_id


# ----------------------------------------------------------------------------- chunked plan
class Chunk:
    """One chunk of the reference-order micrograph list, planned and parsed.

    ``mgs``: Micrograph records (status ok / skip / crash; ok ones carry ``id_base`` and
    ``slot``, their index in ``batch``).  ``batch``: the packed ok micrographs
    (pipeline.Batch; None when there is none).  ``sig``: per (ok micrograph, picker) sigmoid
    flag (the --multi_out table keeps numpy scalars for mapped scores).  ``consumed``: box ids
    consumed (skips included).  ``crash``: index in ``mgs`` of the micrograph at which the
    reference raises (its exception in ``exc``; the chunk ends there), else None.
    """

    def __init__(self, mgs, batch, sig, consumed, crash):
        self.mgs, self.batch, self.sig, self.consumed, self.crash = mgs, batch, sig, consumed, crash

    def shift_ids(self, off):
        """Add a global id offset (a shard's exclusive prefix) to every id of the chunk."""
        for mg in self.mgs:
            mg.id_base += off
        if self.batch is not None:
            self.batch.id_base = self.batch.id_base + off


def resolve(in_dir, methods, index: DirIndex, names):
    """Micrograph records with their k lists of matching paths (get_cliques.py:108-122)."""
    mgs = []
    d0 = os.path.join(in_dir, methods[0])
    others = [(m, os.path.join(in_dir, m)) for m in methods[1:]]
    for name in names:
        base = name.replace(".box", "")
        files = [_glob_path_itself(os.path.join(d0, name))]
        for m, dm in others:
            files.append([os.path.join(dm, n) for n in index.glob(m, f"*{base}*")])
        mgs.append(Micrograph(base=base, files=files))
    return mgs


def plan_chunk(in_dir, methods, index: DirIndex, names, k, box_size, next_id=0,
               n_threads=None):
    """Resolve, parse (C++ parser, GIL released) and pack one chunk of micrographs, giving
    box ids from ``next_id`` on (the process-wide counter of common.py:23,108-112).

    Fast path (the common case: every micrograph has exactly one file per picker, all files
    distinct and parsed OK): the parser's flat arrays are already the batch layout
    (micrograph-major, picker order, file order), so ids and offsets are two cumsums.  Any
    other chunk takes the per-micrograph loop of :func:`plan`'s semantics."""
    from .pipeline import Batch
    mgs = resolve(in_dir, methods, index, names)
    uniq = {}
    single = True
    for mg in mgs:
        for fl in mg.files:
            if len(fl) != 1:
                single = False
            for p in fl:
                uniq.setdefault(p, len(uniq))
    paths = list(uniq)
    if not paths:
        st = np.zeros(0, np.int32)
        off = np.zeros(1, np.int64)
        x = y = sc = np.zeros(0)
        sg = np.zeros(0, bool)
    else:
        st, off, x, y, sc, sg = _lib.parse_files(paths, n_threads)
        if bool((st == _lib.PARSE_FALLBACK).any()):
            st, off, x, y, sc, sg = _splice_fallback(paths, st, off, x, y, sc, sg)
    nf = len(paths)
    if (single and mgs and nf == len(mgs) * k and
            bool((st == _lib.PARSE_OK).all())):
        cnt = np.diff(off)
        if bool((cnt > 0).all()):
            per_mg = cnt.reshape(-1, k).sum(axis=1)
            id_base = next_id + np.concatenate([[0], np.cumsum(per_mg)[:-1]])
            if sg.any():
                sc = sc.copy()
                m = np.repeat(sg, cnt)
                sc[m] = sigmoid(sc[m])
            for i, mg in enumerate(mgs):
                mg.id_base = int(id_base[i])
                mg.slot = i
            batch = Batch(k, box_size, off, id_base, x, y, sc)
            return Chunk(mgs, batch, sg.reshape(-1, k), next_id + int(per_mg.sum()), None)
    # general path: per micrograph, in order (skips consume ids; the first crash ends it)
    crash = None
    ok_files = []
    for i, mg in enumerate(mgs):
        mg.id_base = next_id
        fidx = []
        try:
            for fl in mg.files:
                if not fl:
                    raise UnboundLocalError("local variable 'i' referenced before assignment")
                f = None
                for pth in fl:
                    f = uniq[pth]
                    if st[f] != _lib.PARSE_OK:
                        raise _parsed_exc(int(st[f]), pth)
                if len(fl) > 1:
                    raise AssertionError("Error - multiple BOX files found using pattern")
                fidx.append(f)
                next_id += int(off[f + 1] - off[f])
        except (UnboundLocalError, IndexError):
            mg.status = "skip"
            continue
        except BaseException as e:  # noqa: BLE001 - reproduced exception is the contract
            mg.status, mg.exc = "crash", e
            crash = i
            break
        mg.slot = len(ok_files)
        ok_files.append(fidx)
    if crash is not None:
        mgs = mgs[:crash + 1]
    if not ok_files:
        return Chunk(mgs, None, np.zeros((0, k), bool), next_id, crash)
    fl = np.array(ok_files, np.int64).reshape(-1)
    cnt = off[fl + 1] - off[fl]
    box_off = np.concatenate([[0], np.cumsum(cnt)]).astype(np.int64)
    src = np.repeat(off[fl] - box_off[:-1], cnt) + np.arange(int(box_off[-1]))
    bsig = sg[fl]
    sc2 = sc[src]
    if bsig.any():
        m = np.repeat(bsig, cnt)
        sc2[m] = sigmoid(sc2[m])
    ok = [mg for mg in mgs if mg.status == "ok"]
    batch = Batch(k, box_size, box_off, np.array([mg.id_base for mg in ok], np.int64),
                  x[src], y[src], sc2)
    return Chunk(mgs, batch, bsig.reshape(-1, k), next_id, crash)


def _splice_fallback(paths, st, off, x, y, sc, sg):
    """Files the C++ parser handed back (non-ASCII bytes) parsed with Python's own str/float
    semantics and spliced into the flat arrays (status OK, or the status of the exception
    class they raise; rare, so rebuilt with concatenations)."""
    st = st.copy()
    sg = sg.copy()
    parts = []
    for f, pth in enumerate(paths):
        seg = (x[off[f]:off[f + 1]], y[off[f]:off[f + 1]], sc[off[f]:off[f + 1]])
        if st[f] == _lib.PARSE_FALLBACK:
            try:
                xs, ys, ss, sgf = _py_parse(pth)
                seg = (xs, ys, ss)
                st[f], sg[f] = _lib.PARSE_OK, sgf
            except Exception as e:  # noqa: BLE001
                # skip-class exceptions by status; any other re-raised by _parsed_exc's re-parse
                st[f] = {IndexError: _lib.PARSE_INDEX}.get(type(e), _lib.PARSE_FALLBACK)
                seg = (np.zeros(0), np.zeros(0), np.zeros(0))
        parts.append(seg)
    cnt = np.array([len(p[0]) for p in parts], np.int64)
    off = np.concatenate([[0], np.cumsum(cnt)]).astype(np.int64)
    cat = lambda j: np.concatenate([p[j] for p in parts]) if parts else np.zeros(0)  # noqa: E731
    return st, off, cat(0), cat(1), cat(2), sg


def _parsed_exc(st, path):
    """The exception the reference raises for a file the C++ parser flagged (or, for
    FALLBACK / OSERROR files, Python's own parse of it)."""
    if st == _lib.PARSE_FALLBACK:
        try:
            _py_parse(path)
        except Exception as e:  # noqa: BLE001
            return e
        return None
    if st == _lib.PARSE_OSERROR:
        try:
            open(path, "rt").close()
            return OSError(f"cannot read {path}")
        except OSError as e:
            return e
    return _EXC[st](path)
