"""CPU tests of the single-rank streaming driver (repic_amd.commands.get_cliques._Run.stream):
parser thread | device | writer.  The device stage is replaced by a stub that reports a
per-micrograph status, so the test exercises the queue hand-off and the failure semantics of
the reference (get_cliques.py:145-148, 203: the exception is raised at the first failing
micrograph, after the files of every earlier micrograph exist) without a GPU."""
import argparse
import os
import threading
import time

import numpy as np
import pytest

from golden_util import load_case, make_inputs

from repic_amd import _lib
from repic_amd.commands import get_cliques as gc
from repic_amd.ingest import DirIndex, list_methods, micrograph_names


class _FakeRes:
    def __init__(self, status):
        self.status = status
        self.clique_cnt = np.zeros(len(status), np.int64)


class _FakeWriter:
    def __init__(self):
        self.bases = []
        self.closed = 0

    def group(self, out_dir, items, *arrays):
        self.bases.extend(it[0] for it in items)

    def close(self):
        self.closed += 1


def _run(tmp_path, chunk_mg, fail_at, delay=0.0):
    """Stream the 10017 inputs in chunks of ``chunk_mg`` micrographs; the stub device reports
    NO_EDGES for the ``fail_at``-th ok micrograph (None: never).  Returns (exception, written
    bases, ok bases in order)."""
    meta, _ = load_case("c1_10017")
    in_dir = make_inputs("c1_10017", str(tmp_path))
    methods = list_methods(in_dir)
    index = DirIndex(in_dir, methods, meta["listing"])
    names = micrograph_names(index, methods)
    args = argparse.Namespace(in_dir=in_dir, out_dir=str(tmp_path / "out"), box_size=meta["box"],
                              multi_out=False, get_cc=False, threads=2, chunk_mg=chunk_mg)
    run = gc._Run(args, None, methods, index, names, 0)
    seen = []

    def device(ch):
        time.sleep(delay)   # let the parser run ahead and fill the queue
        st = np.full(max(1, len(ch.mgs)), _lib.OK, np.int32)
        for mg in ch.mgs:
            if mg.status == "ok":
                if fail_at is not None and len(seen) == fail_at:
                    st[mg.slot] = _lib.NO_EDGES
                seen.append(mg.base)
        ch.res = _FakeRes(st)

    run.device = device
    w = _FakeWriter()
    # the group assembly reads the device arrays: record the bases only
    run._submit_group = lambda ch, items, slots, writer: writer.group(None, items)
    exc = None
    try:
        run.stream(w)
    except Exception as e:  # noqa: BLE001 - the class is part of the contract
        exc = e
    return exc, w.bases, seen


@pytest.mark.timeout(60)
@pytest.mark.parametrize("chunk_mg", [1, 4, 5])
def test_stream_raises_at_failing_micrograph_without_hanging(tmp_path, chunk_mg):
    """A device-detected failure in the first chunk while the parser has queued the rest (and
    is blocked on the end sentinel) must raise, not deadlock (the join waited on a full queue
    before the fix)."""
    done = {}

    def body():
        done["r"] = _run(tmp_path, chunk_mg, fail_at=0, delay=0.3)

    th = threading.Thread(target=body, daemon=True)
    th.start()
    th.join(30)
    assert not th.is_alive(), "stream() did not return after a failing micrograph"
    exc, written, seen = done["r"]
    assert isinstance(exc, ValueError), exc
    assert written == []                 # nothing after (or at) the failing micrograph


@pytest.mark.timeout(60)
def test_stream_writes_every_earlier_micrograph_before_raising(tmp_path):
    exc, written, seen = _run(tmp_path, 2, fail_at=5)
    assert isinstance(exc, ValueError), exc
    assert written == seen[:5]


@pytest.mark.timeout(60)
def test_stream_without_failure_writes_all(tmp_path):
    exc, written, seen = _run(tmp_path, 3, fail_at=None)
    assert exc is None
    assert written == seen and len(seen) == 12
