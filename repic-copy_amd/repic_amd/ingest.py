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
    coords: list = field(default_factory=list)  # k ParsedFile (ok micrographs)


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
