"""Multi-process (world size 2) tests of the sharded path.

CPU (gloo): shard bounds, the global box-id offset exchange, counter reduction and the
first-failure agreement (repic_amd/dist.py).  GPU: the full CLI under two ranks (both on
cuda:0) reproduces the single-process goldens, including ids consumed by skipped
micrographs in an earlier shard and a crash in the middle of the list.
"""
import json
import os
import socket
import subprocess
import sys

import numpy as np
import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _spawn(code, world, extra_env=None, timeout=240):
    port = _free_port()
    procs = []
    for r in range(world):
        env = dict(os.environ, WORLD_SIZE=str(world), RANK=str(r), LOCAL_RANK="0",
                   MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port),
                   PYTHONPATH=os.pathsep.join([ROOT, os.path.join(ROOT, "repic-copy_amd"),
                                               os.path.join(ROOT, "tests")]))
        env.update(extra_env or {})
        procs.append(subprocess.Popen([sys.executable, "-c", code], env=env,
                                      stdout=subprocess.PIPE, stderr=subprocess.PIPE, text=True))
    outs = []
    for p in procs:
        o, e = p.communicate(timeout=timeout)
        outs.append((p.returncode, o, e))
    return outs


def test_shard_bounds_balanced():
    from repic_amd.dist import shard_bounds
    for n in (0, 1, 7, 100):
        for world in (1, 2, 3, 8):
            w = np.random.default_rng(n + world).integers(1, 10, size=n)
            b = shard_bounds(w, world)
            assert len(b) == world + 1 and b[0] == 0 and b[-1] == n
            assert all(b[i] <= b[i + 1] for i in range(world))


def test_shard_bounds_pair_work_skewed_within_one_over_world():
    """Skewed micrograph list (a few crowded micrographs among many small ones): contiguous
    shards by pair_work (get_cliques.py:135-138 work per micrograph) are within max item /
    ideal of a perfect split, i.e. no shard exceeds ideal + the largest single micrograph."""
    from repic_amd.dist import pair_work, shard_bounds
    rng = np.random.default_rng(7)
    for world in (2, 4, 8):
        for n, crowded in ((2000, 3000), (20000, 1000)):
            sizes = [[int(v) for v in rng.integers(100, 400, 3)] for _ in range(n)]
            for i in rng.choice(n, n // 100, replace=False):
                sizes[i] = [crowded] * 3            # C3-like crowded micrographs (1 %)
            w = np.array([1.0 + pair_work(s) for s in sizes])
            b = shard_bounds(w, world)
            ideal = w.sum() / world
            loads = [w[b[r]:b[r + 1]].sum() for r in range(world)]
            # a contiguous split overshoots by at most one micrograph
            assert max(loads) <= ideal + w.max()
            if w.max() <= ideal / world:    # items small next to a shard: within 1/world
                assert max(loads) <= ideal * (1 + 1.0 / world)


def test_cli_backend_choice(monkeypatch):
    """The CLI's collectives: gloo when ranks share a GPU (or none is visible), gloo + RCCL
    for device tensors when every local rank owns one GPU."""
    from repic_amd import _lib
    from repic_amd.commands import get_cliques as gc
    monkeypatch.setattr(_lib, "device_count", lambda: 8)
    monkeypatch.setenv("LOCAL_WORLD_SIZE", "8")
    assert gc._dist_backend(8) == "cpu:gloo,cuda:nccl"
    monkeypatch.setenv("LOCAL_WORLD_SIZE", "2")
    monkeypatch.setattr(_lib, "device_count", lambda: 1)
    assert gc._dist_backend(2) == "gloo"
    monkeypatch.setattr(_lib, "device_count", lambda: (_ for _ in ()).throw(_lib.RGCError("x")))
    assert gc._dist_backend(2) == "gloo"


CPU_CODE = r"""
import json, os, torch.distributed as dist
from repic_amd.dist import exclusive_offsets, reduce_counts, first_failure
dist.init_process_group("gloo")
r = dist.get_rank()
off, tot = exclusive_offsets(100 + 7 * r)
cnt = reduce_counts([1, r, 10])
ff = first_failure(None if r == 0 else 5 + r)
ff2 = first_failure(None)
print(json.dumps({"off": off, "tot": tot, "cnt": cnt, "ff": ff, "ff2": ff2}))
dist.destroy_process_group()
"""


def test_gloo_world2_exchanges():
    outs = _spawn(CPU_CODE, 2)
    res = []
    for rc, o, e in outs:
        assert rc == 0, e[-2000:]
        res.append(json.loads(o.strip().splitlines()[-1]))
    assert res[0]["off"] == 0 and res[1]["off"] == 100
    assert res[0]["tot"] == res[1]["tot"] == 207
    assert res[0]["cnt"] == res[1]["cnt"] == [2, 1, 20]
    assert res[0]["ff"] == res[1]["ff"] == 6
    assert res[0]["ff2"] is None and res[1]["ff2"] is None


GPU_CODE = r"""
import argparse, builtins, json, os, sys
from golden_util import load_case, make_inputs
from repic_amd.commands import get_cliques
name, root = sys.argv[1], sys.argv[2]
meta, data = load_case(name)
in_dir = os.path.join(root, "in")
out_dir = os.path.join(root, "out")
a = argparse.Namespace(in_dir=in_dir, out_dir=out_dir, box_size=meta["box"],
                       multi_out="--multi_out" in meta["flags"], get_cc="--get_cc" in meta["flags"],
                       batch_boxes=1 << 25, threads=None, device=0, listing=meta["listing"])
exc = None
try:
    get_cliques.main(a)
except Exception as e:
    exc = type(e).__name__
    import traceback; traceback.print_exc()
print(json.dumps({"exc": exc}))
"""


@pytest.mark.gpu
@pytest.mark.parametrize("name", ["c1_10017", "skips", "crash_noedges", "ties_getcc"])
def test_cli_two_ranks_match_golden(name, tmp_path):
    from golden_util import assert_matches_golden, load_case, make_inputs, read_outputs
    meta, data = load_case(name)
    make_inputs(name, str(tmp_path))
    port = _free_port()
    procs = []
    for r in range(2):
        env = dict(os.environ, WORLD_SIZE="2", RANK=str(r), LOCAL_RANK="0",
                   MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port),
                   PYTHONPATH=os.pathsep.join([ROOT, os.path.join(ROOT, "repic-copy_amd"),
                                               os.path.join(ROOT, "tests")]))
        procs.append(subprocess.Popen([sys.executable, "-c", GPU_CODE, name, str(tmp_path)],
                                      env=env, stdout=subprocess.PIPE, stderr=subprocess.PIPE,
                                      text=True))
    excs = []
    for p in procs:
        o, e = p.communicate(timeout=600)
        assert p.returncode == 0, e[-3000:]
        excs.append(json.loads(o.strip().splitlines()[-1])["exc"])
        if excs[-1] is not None and excs[-1] != meta["exception"]:
            raise AssertionError(e[-3000:])
    if meta["exception"]:
        assert meta["exception"] in excs
    else:
        assert excs == [None, None]
    mgs, arrays = read_outputs(os.path.join(str(tmp_path), "out"), meta)
    assert_matches_golden(meta, data, mgs, arrays)


def test_bench_self_launch_rank_layout():
    """`python bench.py --gpus N` with no launcher env spawns N ranks (RANK = LOCAL_RANK = r,
    WORLD_SIZE = N, rendezvous on 127.0.0.1); a --gpus / WORLD_SIZE mismatch is an error."""
    env = {k: v for k, v in os.environ.items()
           if k not in ("WORLD_SIZE", "RANK", "LOCAL_RANK", "MASTER_PORT")}
    r = subprocess.run([sys.executable, os.path.join(ROOT, "bench.py"), "--gpus", "3",
                        "--launch-check"], env=env, capture_output=True, text=True, timeout=120)
    assert r.returncode == 0, r.stderr
    got = sorted((json.loads(line) for line in r.stdout.strip().splitlines()),
                 key=lambda d: int(d["RANK"]))
    assert [(d["RANK"], d["LOCAL_RANK"], d["WORLD_SIZE"], d["MASTER_ADDR"]) for d in got] == \
        [(str(i), str(i), "3", "127.0.0.1") for i in range(3)]
    r = subprocess.run([sys.executable, os.path.join(ROOT, "bench.py"), "--gpus", "4",
                        "--launch-check"], env=dict(env, WORLD_SIZE="2"), capture_output=True,
                       text=True, timeout=120)
    assert r.returncode != 0 and "WORLD_SIZE=2" in r.stderr


@pytest.mark.gpu
def test_bench_self_launch_two_ranks():
    """`python bench.py --gpus 2` with no launcher: two self-spawned ranks (both on cuda:0 over
    gloo on the 1-GPU test box) report n_gpus 2 and the totals of the 120-micrograph union."""
    env = {k: v for k, v in os.environ.items()
           if k not in ("WORLD_SIZE", "RANK", "LOCAL_RANK", "MASTER_PORT")}
    env.update(RGC_BENCH_DEVICE="0", RGC_DIST_BACKEND="gloo")
    r = subprocess.run([sys.executable, os.path.join(ROOT, "bench.py"), "--gpus", "2", "--n_mg",
                        "60", "--steps", "2", "--warmup", "1", "--no-cpu-baseline"], env=env,
                       capture_output=True, text=True, timeout=240)
    assert r.returncode == 0, r.stderr[-3000:]
    lines = [json.loads(s) for s in r.stdout.strip().splitlines() if s.startswith("{")]
    assert len(lines) == 1
    d = lines[0]
    assert d["n_gpus"] == 2 and d["totals"]["micrographs"] == 120 and d["value"] > 0


@pytest.mark.gpu
def test_bench_two_ranks_one_gpu():
    """bench.py's sharded path (id-offset all_gather, max-over-ranks timing, counter
    all_reduce) with two ranks on cuda:0 over gloo: the totals equal one rank's run over the
    union of the shards."""
    def run(world, n_mg):
        port = _free_port()
        procs = []
        for r in range(world):
            env = dict(os.environ, WORLD_SIZE=str(world), RANK=str(r), LOCAL_RANK=str(r),
                       MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), RGC_BENCH_DEVICE="0",
                       RGC_DIST_BACKEND="gloo")
            procs.append(subprocess.Popen(
                [sys.executable, os.path.join(ROOT, "bench.py"), "--gpus", str(world), "--n_mg",
                 str(n_mg), "--steps", "2", "--warmup", "1", "--no-cpu-baseline"],
                env=env, stdout=subprocess.PIPE, stderr=subprocess.PIPE, text=True))
        outs = [p.communicate(timeout=240) for p in procs]
        for p, (o, e) in zip(procs, outs):
            assert p.returncode == 0, e[-3000:]
        return json.loads(outs[0][0].strip().splitlines()[-1])
    two = run(2, 60)
    one = run(1, 120)
    assert two["n_gpus"] == 2 and two["value"] > 0 and two["scaling"] == "weak"
    assert two["totals"] == one["totals"]
    assert two["totals"]["micrographs"] == 120


@pytest.mark.gpu
def test_bench_fixed_batch_two_ranks():
    """The strong-scaling entry: `bench.py --gpus 2 --by-config C4_100k_fixed` (two
    self-spawned ranks on cuda:0 over gloo) splits ONE 100k-micrograph C4 batch 50k / 50k and
    reports its total of 100k micrographs per step, scaling "strong"."""
    env = {k: v for k, v in os.environ.items()
           if k not in ("WORLD_SIZE", "RANK", "LOCAL_RANK", "MASTER_PORT")}
    env.update(RGC_BENCH_DEVICE="0", RGC_DIST_BACKEND="gloo")
    r = subprocess.run([sys.executable, os.path.join(ROOT, "bench.py"), "--gpus", "2",
                        "--config", "C2", "--n_mg", "20", "--by-config", "C4_100k_fixed",
                        "--steps", "2", "--warmup", "1", "--no-cpu-baseline"], env=env,
                       capture_output=True, text=True, timeout=280)
    assert r.returncode == 0, r.stderr[-3000:]
    lines = [json.loads(s) for s in r.stdout.strip().splitlines() if s.startswith("{")]
    assert len(lines) == 1
    e = lines[0]["by_config"]["C4_100k_fixed"]
    assert e["totals"]["micrographs"] == 100000 and e["micrographs_per_step"] == 100000
    assert e["scaling"] == "strong" and e["micrographs_per_gpu"] == 50000 and e["value"] > 0
