"""CPU tests (gloo, world size 2) of the sharded CLI driver (get_cliques._Run.sharded): the
shard is parsed, the ranks exchange their consumed ids, then chunks stream through the device
(a stub here, no GPU) with their writes handed to the writer pool, so the writes of one chunk
overlap the device work of the next.  On a failure the ranks agree on the first failing
micrograph; files of micrographs from it on are removed, the owning rank raises the
reference's exception and every earlier micrograph's files exist (get_cliques.py:145-148,203).
"""
import json
import os
import subprocess
import sys

import pytest

from test_distributed import ROOT, _free_port

CODE = r"""
import argparse, json, os, sys, time
import numpy as np
from golden_util import load_case
from repic_amd import _lib
from repic_amd.commands import get_cliques as gc

root, fail_at, foreign = sys.argv[1], int(sys.argv[2]), sys.argv[3] == "1"
meta, _ = load_case("c1_10017")
args = argparse.Namespace(in_dir=os.path.join(root, "in"), out_dir=os.path.join(root, "out"),
                          box_size=meta["box"], multi_out=False, get_cc=False, threads=2,
                          chunk_mg=2, batch_boxes=1 << 25, device=None, listing=meta["listing"])

class Res:
    def __init__(self, st):
        self.status = st
        self.n_edges_mg = np.zeros(len(st), np.int64)
        self.clique_cnt = np.zeros(len(st), np.int64)

def device(self, ch):
    time.sleep(0.3)                 # the writes of the previous chunk land meanwhile
    if foreign:                     # files this run never writes (e.g. an earlier run_ilp's)
        for mg in ch.mgs:
            with open(os.path.join(self.args.out_dir, mg.base + "_runtime.tsv"), "w") as f:
                f.write("foreign\n")
    st = np.full(max(1, len(ch.mgs)), _lib.OK, np.int32)
    for i, mg in enumerate(ch.mgs):
        if mg.status == "ok" and ch.first + i == fail_at:
            st[mg.slot] = _lib.NO_EDGES
    ch.res = Res(st)

def submit(self, ch, items, slots, writer):
    # every micrograph as an empty <base>.box (a skip record): the stub has no device arrays
    z = np.zeros(0)
    writer.group(self.args.out_dir, [(it[0], -1, 0, 0, 0, 0.0, None) for it in items], z, z,
                 np.zeros((0, 3), np.int32), z, z, np.zeros(0, np.int64))

gc._Run.device = device
gc._Run._submit_group = submit
import torch.distributed as dist
dist.init_process_group("gloo")
exc = None
try:
    gc._main(args, None, 2, dist.get_rank())
except Exception as e:
    exc = type(e).__name__
print(json.dumps({"exc": exc, "spans": gc.LAST_RUN.get("spans", [])}))
dist.destroy_process_group()
"""


def _run(tmp_path, fail_at, foreign=False):
    from golden_util import make_inputs
    make_inputs("c1_10017", str(tmp_path))
    port = _free_port()
    procs = []
    for r in range(2):
        env = dict(os.environ, WORLD_SIZE="2", RANK=str(r), LOCAL_RANK="0",
                   MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), RGC_CLI_GLOO="1",
                   PYTHONPATH=os.pathsep.join([ROOT, os.path.join(ROOT, "repic-copy_amd"),
                                               os.path.join(ROOT, "tests")]))
        procs.append(subprocess.Popen([sys.executable, "-c", CODE, str(tmp_path), str(fail_at),
                                       "1" if foreign else "0"],
                                      env=env, stdout=subprocess.PIPE, stderr=subprocess.PIPE,
                                      text=True))
    out = []
    for p in procs:
        o, e = p.communicate(timeout=240)
        assert p.returncode == 0, e[-3000:]
        out.append(json.loads(o.strip().splitlines()[-1]))
    return out


def _names():
    from golden_util import load_case
    meta, _ = load_case("c1_10017")
    return [g["base"] for g in meta["micrographs"]]


@pytest.mark.timeout(300)
def test_sharded_stream_overlaps_device_and_writes(tmp_path):
    res = _run(tmp_path, -1)
    assert [r["exc"] for r in res] == [None, None]
    written = sorted(f[:-4] for f in os.listdir(tmp_path / "out") if f.endswith(".box"))
    assert written == sorted(_names())
    for r in res:
        sp = r["spans"]
        dev = [s for s in sp if s[0] == "device"]
        wr = [s for s in sp if s[0] == "write"]
        assert len(dev) >= 2 and wr
        # some write of an earlier chunk is in flight while a later chunk is on the device
        assert any(w[2] < d[3] and w[3] > d[2] for w in wr for d in dev[1:]), sp


@pytest.mark.timeout(300)
@pytest.mark.parametrize("fail_at", [3, 9])
def test_sharded_stream_failure_removes_later_files(tmp_path, fail_at):
    """fail_at: global micrograph index of a NO_EDGES micrograph (rank 0's shard: rank 1's
    optimistic writes are removed again; rank 1's shard: rank 0 completes)."""
    res = _run(tmp_path, fail_at)
    excs = [r["exc"] for r in res]
    assert "ValueError" in excs and excs.count("ValueError") == 1
    # the listing replays the reference's order: the golden's micrograph order
    names = _names()
    written = sorted(f[:-4] for f in os.listdir(tmp_path / "out") if f.endswith(".box"))
    assert written == sorted(names[:fail_at])


@pytest.mark.timeout(300)
def test_sharded_failure_cleanup_removes_only_written_files(tmp_path):
    """the cleanup after a failure removes only the files the writer wrote for the
    micrographs from the failing one on (here each one's empty .box), never other files of
    those names (here a <base>_runtime.tsv the run did not write)."""
    fail_at = 3
    res = _run(tmp_path, fail_at, foreign=True)
    assert [r["exc"] for r in res].count("ValueError") == 1
    names = _names()
    out = tmp_path / "out"
    assert sorted(f[:-4] for f in os.listdir(out) if f.endswith(".box")) == sorted(names[:fail_at])
    # every chunk the device saw created a foreign runtime.tsv; none of them was removed
    kept = {f[:-len("_runtime.tsv")] for f in os.listdir(out) if f.endswith("_runtime.tsv")}
    assert set(names[fail_at:]) & kept, kept
    for b in kept:
        assert open(out / (b + "_runtime.tsv")).read() == "foreign\n"
