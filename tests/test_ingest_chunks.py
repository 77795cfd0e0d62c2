"""CPU tests of the chunked ingest (repic_amd.ingest.plan_chunk) that the pipelined CLI runs:
for every golden input set (reference get_cliques.py:108-130 + common.py:71-114 semantics) and
any chunk size, chunk-by-chunk planning must reproduce the whole-list plan(): the same
micrograph statuses and exception classes, the same global box ids (skips consume ids), and
the same packed coordinates / sigmoid-mapped scores, bit for bit."""
import os

import numpy as np
import pytest

from golden_util import golden_cases, load_case, make_inputs

from repic_amd.ingest import DirIndex, list_methods, micrograph_names, plan, plan_chunk


def _chunks(in_dir, methods, index, names, k, box, size):
    out, nid = [], 0
    for c0 in range(0, len(names), size):
        ch = plan_chunk(in_dir, methods, index, names[c0:c0 + size], k, box, nid, 2)
        out.append(ch)
        nid = ch.consumed
        if ch.crash is not None:
            break
    return out, nid


@pytest.mark.parametrize("name", golden_cases())
@pytest.mark.parametrize("size", [1, 3, 1024])
def test_plan_chunk_matches_plan(name, size, tmp_path):
    meta, _ = load_case(name)
    in_dir = make_inputs(name, str(tmp_path))
    methods = list_methods(in_dir)
    if len(methods) < 2:
        pytest.skip("k = 1 case (the reference raises before any micrograph)")
    index = DirIndex(in_dir, methods, meta["listing"])
    try:
        names = micrograph_names(index, methods)
    except Exception:  # noqa: BLE001
        pytest.skip("listing not replayable here")
    k = len(methods)
    ref, crash, consumed = plan(in_dir, methods, index, order=names, n_threads=2)
    chunks, nid = _chunks(in_dir, methods, index, names, k, meta["box"], size)
    got = [mg for ch in chunks for mg in ch.mgs]
    assert [m.base for m in got] == [m.base for m in ref]
    assert [m.status for m in got] == [m.status for m in ref]
    assert nid == consumed
    for a, b in zip(got, ref):
        if b.status == "crash":
            assert type(a.exc) is type(b.exc)
        if b.status == "ok":
            assert a.id_base == b.id_base
    # packed coordinates / scores of the ok micrographs, in order
    for ch in chunks:
        oks = [mg for mg in ch.mgs if mg.status == "ok"]
        if not oks:
            assert ch.batch is None
            continue
        by_base = {}
        for r in ref:
            by_base.setdefault(r.base, []).append(r)
        b = ch.batch
        for mg in oks:
            r = [x for x in by_base[mg.base] if x.id_base == mg.id_base][0]
            assert int(b.id_base[mg.slot]) == r.id_base
            for p in range(k):
                lo, hi = int(b.box_off[mg.slot * k + p]), int(b.box_off[mg.slot * k + p + 1])
                c = r.coords[p]
                for got_a, want_a in ((b.x[lo:hi], c.x), (b.y[lo:hi], c.y), (b.score[lo:hi], c.s)):
                    assert np.array_equal(np.asarray(got_a).view(np.uint64),
                                          np.asarray(want_a).view(np.uint64))
                assert bool(ch.sig[mg.slot, p]) == bool(c.sigmoid)
