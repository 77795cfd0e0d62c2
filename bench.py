#!/usr/bin/env python3
"""Benchmark of the MI355X get_cliques hot path (BASELINE.json metric: micrographs/s).

A "step" is one pass of the whole hot path (bin -> JI pairs -> graph/CC -> k-cliques +
ILP epilogue -> constraint-matrix rows) over one batch of synthetic micrographs already
resident in HBM.  Default workload = BASELINE.json configs[1] (C2: 10k micrographs x 3
pickers x ~300 boxes, box 180, 4096^2) per GPU; multi-GPU runs shard micrographs across
ranks (weak scaling, no collective in the hot path).

  python bench.py [--gpus N] [--steps K] [--warmup W] [--config C2|C3|C4|C5] [--n_mg M]

Prints ONE JSON line on rank 0 (driver contract), with "roofline" (dominant kernel, HIP
events around each launch) and "cpu_baseline" (the oracle's faithful per-pair loop on a
bounded sample, 1 core).  Steps are pipelined on three contexts, each on its own stream, so
that step i+1's workgroups run in step i's drain tail (--streams 1 serialises two contexts on
one stream); the roofline's per-launch durations then come from serialised steps timed after
the timed region.
"""
from __future__ import annotations

import argparse
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.join(ROOT, "repic-copy_amd"))
sys.path.insert(0, ROOT)

import numpy as np  # noqa: E402

HBM_PEAK_GBS = 8000.0   # MI355X_MICROARCH.md: HBM3E 8.0 TB/s spec

DEFAULT_MG = {"C2": 10000, "C3": 4000, "C4": 12500, "C5": 64}
# by_config entries: name -> (BASELINE config, micrographs per GPU).  C4_100k is the north-star
# batch (BASELINE configs[3]: 100k micrographs, 5 pickers) on ONE GPU, the 1-GPU point of the
# 1 -> 8 curve; C4 is its 12.5k-micrograph per-GPU shard at 8 GPUs.
# C5_256: the large-micrograph route at 256 micrographs per step (its per-micrograph kernels,
# one workgroup per micrograph, fill 64 of 256 CUs at C5's 64 per step)
BY_CONFIG = {"C2": ("C2", 10000), "C3": ("C3", 4000), "C4": ("C4", 12500), "C5": ("C5", 64),
             "C4_100k": ("C4", 100000), "C5_256": ("C5", 256),
             # strong scaling: ONE fixed 100k-micrograph C4 batch (the
             # north-star batch) split over the ranks, 100k / N each; at N = 1 it is C4_100k
             "C4_100k_fixed": ("C4", 100000),
             # C2 with fractional coordinates (3 decimals, as converted STAR / CBOX picks give):
             # the fused kernel's f64 layout (untimed on the line before)
             "C2_frac": ("C2", 10000)}
ENTRY_KW = {"C2_frac": {"frac": True}}   # generator overrides of an entry
FIXED_TOTAL = {"C4_100k_fixed"}   # entries whose micrograph count is the whole job's, not per GPU
# file-to-file entries (the CLI on BOX text, one GPU, rank 0 of a 1-GPU run): C1 = the
# reference's own EMPIAR-10017 example (12 micrographs, BASELINE configs[0]), C2_f2f = 10k
# synthetic C2 micrographs written as BOX text first (not timed)
F2F_ENTRIES = ("C1", "C2_f2f")
# the reference's C1 rate (the survey's run of the reference itself, 1 core,
# 34.75 s for the 12 micrographs; README.md:60 quotes "1-3 mins")
REF_C1_RATE = 0.345
# hardware queues per process on the MI355X boxes (GPU_MAX_HW_QUEUES); the bench's streams:
# `depth` launch streams + torch's null stream, which also carries the non-lazy stats copies
HW_QUEUES = 4


def fixed_shard(total, world, rank):
    """(start, count) of rank's contiguous share of a fixed batch of ``total`` micrographs:
    sizes differ by at most one, the first ``total % world`` ranks take the extra one."""
    base, extra = divmod(total, world)
    start = rank * base + min(rank, extra)
    return start, base + (1 if rank < extra else 0)


def stream_plan(depth):
    """Streams (hardware queues) one bench process uses: a launch stream per context in flight
    plus the null stream (torch's default; rgc_ctx_set_copy_stream(ctx, 0) for any copy the
    library issues off the launch stream; non-lazy runs' stats come from the ties kernel on
    the launch stream), no other copy stream.  Must fit HW_QUEUES, or streams share queues in
    creation order (round 5: the stats-copy variant ran 68 % slower on the driver's box with 7
    streams)."""
    plan = {"launch_streams": depth, "null_stream": 1, "copy_streams": 0}
    plan["total"] = plan["launch_streams"] + plan["null_stream"] + plan["copy_streams"]
    assert plan["total"] <= HW_QUEUES, plan
    return plan


def fused_compulsory_bytes(N, C, k, V, n_mg):
    """Bytes the fused kernel must move at minimum: read x, y (16 B/box) and the scores of
    clique vertices (8 B/vertex); write rows (4k), w, conf, consensus (12) per clique and the
    48-B per-micrograph stats."""
    return 16 * N + 8 * V + C * (4 * k + 12) + 48 * n_mg


def alg_bytes(name, N, E, C, k, V, n_mg=0):
    """Algorithmic HBM bytes of one step of each kernel.  The fused kernel
    runs the whole hot path, so its figure is SURVEY.md §8(d)'s per-micrograph B_alg summed
    over the micrographs it processes."""
    table = {
        "k_fused": pipeline_bytes(N, E, C, k),
        "k1_bin": 16 * N + 30 * N,                       # read x,y; write sorted SoA + maps
        "k2_pairs_count": 21 * N + 4 * N,                # read sx,sy,spick,sbox; write count
        "k2_pairs_fill": 21 * N + 8 * N + 12 * E,        # + offsets; write (dst, JI) per edge
        "k4_union": 8 * N + 4 * E + 1 * N,               # offsets, targets, node flags
        "k4_compress": 1 * N + 8 * N,                    # flags, parent read/write
        "k4_stats": 1 * N + 8 * N,
        "k5_cliques_count": 13 * N + 12 * E + 4 * N,     # roots' CSR walk; write counts
        "k5_cliques_fill": 13 * N + 12 * E + 24 * V + C * (5 * k + 12),
        "k7_rank": 1 * N + 20 * V,
        "k7_rows": 12 * k * C,
    }
    return table.get(name)


def pipeline_bytes(N, E, C, k):
    """B_alg = 28 N + 32 E + C (20 k + 12) for the whole hot path."""
    return 28 * N + 32 * E + C * (20 * k + 12)


def pmc_record(entry):
    """The newest profiles/*_traffic.json written by tools/pmc_traffic.py for THIS library
    build (sha256 must match) on THIS entry (its by_config name, which fixes the batch size:
    files without an "entry" key were taken at the config's bench size, so they stand for the
    entry named like the config, and files without a "config" were C2 runs), as (record, file
    name), else (None, None)."""
    import glob
    import hashlib
    from repic_amd import _lib
    sha = hashlib.sha256(open(_lib.LIB_PATH, "rb").read()).hexdigest()
    for f in sorted(glob.glob(os.path.join(ROOT, "profiles", "*_traffic.json")), reverse=True):
        try:
            d = json.load(open(f))
        except (OSError, ValueError):
            continue
        if d.get("lib_sha256") == sha and d.get("entry", d.get("config", "C2")) == entry:
            return d, os.path.basename(f)
    return None, None


def roofline_evidence(rec, kernel, alg_bytes, kernel_ms, dv_kernel=None):
    """(traffic bytes per launch/step, measured HBM fraction, limiter text) from the config's
    committed counters; the limiter names what the counters show, not a fixed claim.  The
    multi-kernel route's issue counters are those of dv_kernel, its longest kernel (the same
    ones derived_bound reads)."""
    if rec is None:
        return None, None, ("unmeasured for this library build: no profiles/*_traffic.json "
                            "with its sha256 for this config")
    if kernel == "k_fused":
        k = rec.get("kernels", {}).get("k_fused")
        if k is None:
            return None, None, "no k_fused counters in the matching PMC file"
        traffic, dv = k["traffic"], k.get("derived", {})
    else:
        traffic = rec.get("step_traffic")
        dv = rec.get("kernels", {}).get(dv_kernel, {}).get("derived", {}) if dv_kernel else {}
        if traffic is None:
            return None, None, "no per-step traffic in the matching PMC file"
    hbm = traffic / (kernel_ms * 1e-3) / 1e9 / HBM_PEAK_GBS
    parts = [f"measured HBM traffic {traffic / 1e6:.0f} MB/launch = {traffic / alg_bytes:.2f}x "
             f"B_alg, {hbm * HBM_PEAK_GBS / 1e3:.2f} TB/s = {100 * hbm:.0f}% of peak"]
    if "valu_busy" in dv:
        parts.append(f"VALU busy {100 * dv['valu_busy']:.0f}%")
    if "wait_any" in dv:
        parts.append(f"waves stalled {100 * dv['wait_any']:.0f}% of resident time")
    if "waves_per_cu" in dv:
        parts.append(f"{dv['waves_per_cu']:.1f} resident waves/CU")
    if "lane_eff" in dv:
        parts.append(f"VALU lane efficiency {100 * dv['lane_eff']:.0f}%")
    if dv and kernel != "k_fused":
        parts.append(f"issue counters of {dv_kernel}, the route's longest kernel")
    bound = ("VALU issue" if dv.get("valu_busy", 0) > 0.6 and hbm < 0.5 else
             "HBM bandwidth" if hbm >= 0.5 else "latency (neither VALU nor HBM saturated)")
    if not dv:
        bound = "HBM bandwidth" if hbm >= 0.5 else "not HBM bandwidth (issue counters not collected)"
    return traffic, hbm, f"{bound}: " + "; ".join(parts)


def _cpu_model():
    try:
        with open("/proc/cpuinfo") as f:
            for line in f:
                if line.startswith("model name"):
                    return line.split(":", 1)[1].strip()
    except OSError:
        pass
    return "unknown"


def _oracle_loop(cfg, mgs, budget_s, id0=0):
    """Oracle faithful per-pair loop (oracle/cpu_ref.py, same structure as the reference's
    get_jaccard, get_cliques.py:59-69) over ``mgs`` until ``budget_s`` has elapsed."""
    from oracle import cpu_ref
    methods = [f"picker{p}" for p in range(cfg.k)]
    t0 = time.perf_counter()
    n, nid = 0, id0
    for mg in mgs:
        coords = []
        for (x, y, s) in mg:
            coords.append([(float(a), float(b), float(c), nid + i)
                           for i, (a, b, c) in enumerate(zip(x.tolist(), y.tolist(), s.tolist()))])
            nid += len(x)
        cpu_ref.micrograph(coords, cfg.box, methods, faithful=True)
        n += 1
        if time.perf_counter() - t0 > budget_s:
            break
    return n, time.perf_counter() - t0


def _oracle_worker(cfg_kw, start, n_max, budget_s):
    """One process of the parallel CPU baseline: its own disjoint micrograph shard."""
    from repic_amd import synth
    cfg = synth.SynthConfig(**cfg_kw)
    mgs = synth.batch(cfg, n_max, start=start)
    return _oracle_loop(cfg, mgs, budget_s)


def _pair_loop_sample(cfg, mg, budget_s):
    """BASELINE.md §3 for C5 (one micrograph takes far longer than any bench budget): time the
    oracle's faithful per-pair loop (get_cliques.py:59-69, >= 97 % of the reference's time on
    C1) over the first rows of every picker pair's outer loop for ``budget_s`` in all, and
    extrapolate each pair to its full outer loop.  Later stages (graph, cliques, epilogue) are
    not timed, so the returned micrograph time UNDERSTATES the reference's (the CPU rate is an
    upper bound)."""
    import itertools

    from oracle import cpu_ref
    P = []
    nid = 0
    for (x, y, s) in mg:
        P.append([(float(a), float(b), float(c), nid + i)
                  for i, (a, b, c) in enumerate(zip(x.tolist(), y.tolist(), s.tolist()))])
        nid += len(x)
    pairs = list(itertools.combinations(range(cfg.k), 2))
    per = budget_s / len(pairs)
    est, rows_done, rows_all = 0.0, 0, 0
    for (j, l) in pairs:
        t0 = time.perf_counter()
        r = 0
        step = max(1, len(P[j]) // 200)
        while r < len(P[j]) and time.perf_counter() - t0 < per:
            cpu_ref.edges_faithful(P[j][r:r + step], P[l], cfg.box)
            r += step
        dt = time.perf_counter() - t0
        r = min(r, len(P[j]))
        est += dt * len(P[j]) / max(r, 1)
        rows_done += r
        rows_all += len(P[j])
    return est, rows_done, rows_all


def cpu_baseline(cfg, mgs, budget_s=12.0, procs=None, config=None):
    """1 process (the reference is single-threaded) and P processes on disjoint micrograph
    shards, P = this host's CPU share capped at 16 (the GPU box's share).
    C5 (a micrograph takes tens of minutes): one micrograph's pair loop, sampled and
    extrapolated (_pair_loop_sample), 1 process only."""
    if config == "C5":
        est, done, tot = _pair_loop_sample(cfg, mgs[0], budget_s)
        return {"value": 1.0 / est, "unit": "micrographs/s", "cores": 1, "kind": "port",
                "sample": f"1 micrograph: faithful per-pair loop (get_cliques.py:59-69) over "
                          f"{done} of {tot} outer-loop boxes across all {cfg.k * (cfg.k - 1) // 2} "
                          f"picker pairs in ~{budget_s:.0f} s, extrapolated to the whole pair "
                          f"loop ({est:.0f} s per micrograph); graph/clique/epilogue stages not "
                          f"timed, so this rate is an upper bound on the reference's",
                "cpu_model": _cpu_model()}
    n, dt = _oracle_loop(cfg, mgs, budget_s)
    out = {"value": n / dt, "unit": "micrographs/s", "cores": 1, "kind": "port",
           "sample": f"{n} micrographs of this workload, oracle faithful per-pair loop "
                     f"(reference get_jaccard structure), 1 process, {dt:.1f} s",
           "cpu_model": _cpu_model()}
    P = procs or min(16, len(os.sched_getaffinity(0)))
    if P > 1:
        import dataclasses
        import multiprocessing as mp
        from concurrent.futures import ProcessPoolExecutor
        per = max(2, int(2 * n / dt * budget_s))      # more than one process gets through
        kw = dataclasses.asdict(cfg)
        t0 = time.perf_counter()
        with ProcessPoolExecutor(P, mp_context=mp.get_context("spawn")) as ex:
            futs = [ex.submit(_oracle_worker, kw, 1_000_000 + i * per, per, budget_s)
                    for i in range(P)]
            res = [f.result() for f in futs]
        wall = time.perf_counter() - t0
        tot = sum(r[0] for r in res)
        out["parallel"] = {
            "value": sum(r[0] / r[1] for r in res), "unit": "micrographs/s", "cores": P,
            "sample": f"{tot} micrographs, {P} processes on disjoint shards of the same "
                      f"generator, ~{budget_s:.0f} s each ({wall:.1f} s wall incl. start-up)"}
    return out


def _free_port():
    import socket
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    port = s.getsockname()[1]
    s.close()
    return port


def self_launch(n):
    """``--gpus N`` without a torch.distributed launcher: start N fresh child processes of this
    script, one per GPU (RANK = LOCAL_RANK = r, WORLD_SIZE = N, rendezvous on 127.0.0.1), and
    exit with the worst child status.  Runs before anything touches the GPU (the parent never
    initialises HIP); rank 0's JSON line reaches the inherited stdout."""
    import subprocess
    port = os.environ.get("MASTER_PORT") or str(_free_port())
    procs = []
    for r in range(n):
        env = dict(os.environ, WORLD_SIZE=str(n), RANK=str(r), LOCAL_RANK=str(r),
                   LOCAL_WORLD_SIZE=str(n), MASTER_ADDR="127.0.0.1", MASTER_PORT=port)
        procs.append(subprocess.Popen([sys.executable, os.path.abspath(__file__)] + sys.argv[1:],
                                      env=env))
    # a failed rank would leave the others blocked in a collective: stop them (our own
    # children, by handle)
    while True:
        rcs = [p.poll() for p in procs]
        bad = [rc for rc in rcs if rc not in (None, 0)]
        if bad:
            for p in procs:
                if p.poll() is None:
                    p.terminate()
            for p in procs:
                try:
                    p.wait(timeout=30)
                except subprocess.TimeoutExpired:
                    p.kill()
            return bad[0]
        if all(rc == 0 for rc in rcs):
            return 0
        time.sleep(0.05)


def derived_bound(rec, kernel, alg_bytes, kernel_ms, dv_kernel="k_fused"):
    """The roofline class the counters put this kernel in (the same evidence as ``limiter``):
    "hbm" when the measured HBM bandwidth is >= 50 % of peak, "valu" when the VALU pipe is
    busy > 60 % of the time, "latency" otherwise; "unmeasured" without counters for this
    library build.  Throughput is priced against HBM either way (no contraction, no MFMA).
    The issue counters are those of ``dv_kernel`` (the multi-kernel route: its longest
    kernel)."""
    if rec is None:
        return "unmeasured"
    traffic, hbm, _ = roofline_evidence(rec, kernel, alg_bytes, kernel_ms)
    if hbm is None:
        return "unmeasured"
    dv = rec.get("kernels", {}).get(dv_kernel, {}).get("derived", {})
    if hbm >= 0.5:
        return "hbm"
    if dv.get("valu_busy", 0.0) > 0.6:
        return "valu"
    return "latency" if dv else "unmeasured"


TIME_EVERY = 4   # pipelined steps: one in TIME_EVERY carries the HIP timing events
SER_STEPS = 8    # two-stream runs: serialised steps timed with HIP events for the roofline
# steps in flight (contexts, one stream each): three against two, with each run's stats copy
# on its own launch stream, C2 -1.5 %, C4 -1.3 %, C3 -0.6 %, C5 -4.7 % (the large route syncs
# on the host once per clique level; profiles/r05w_ab_copy_on_stream.txt)
PIPE_DEPTH_DEFAULT = 3
PIPE_DEPTH = {}


class Env:
    """Rank layout and devices of this bench process (one GPU per rank over RCCL)."""

    def __init__(self, args):
        import torch
        self.world = int(os.environ.get("WORLD_SIZE", "1"))
        self.rank = int(os.environ.get("RANK", "0"))
        local = int(os.environ.get("LOCAL_RANK", "0"))
        # RGC_BENCH_DEVICE / RGC_DIST_BACKEND: test hooks (two ranks on one GPU over gloo);
        # the driver's runs use one GPU per rank over RCCL ("nccl")
        self.local = int(os.environ.get("RGC_BENCH_DEVICE", local))
        self.backend = os.environ.get("RGC_DIST_BACKEND", "nccl")
        self.dist = None
        self.streams = None   # measure(): the two library streams, created on first use
        if self.world > 1:
            import torch.distributed as dist
            torch.cuda.set_device(self.local)
            if self.backend == "nccl":
                dist.init_process_group("nccl", device_id=torch.device("cuda", self.local))
            else:
                dist.init_process_group(self.backend)
            self.dist = dist
        self.dev = torch.device("cuda", self.local)
        # collective tensors
        self.cdev = self.dev if self.backend == "nccl" else torch.device("cpu")


def pipelined_steps(ctxs, submit, n, timing, ktimes=None):
    """n steps over the contexts round-robin with len(ctxs) of them in flight: step i is
    submitted on ctxs[i % d] once step i - d + 1 has been waited for (d = len(ctxs)); returns
    the last step's Result.  ``submit(ctx, timed)`` enqueues one step.  HIP timing events cost
    ~5 us of idle GPU each between launches (tools/step_gap.py: ~15 us per C2 step with the
    three per step), so with ``timing`` every TIME_EVERY-th step carries them and ``ktimes``
    sums those steps' kernel times (count in "__steps")."""
    def timed(i):
        return timing and i % TIME_EVERY == 0

    nd = len(ctxs)
    r = None
    for j in range(min(nd - 1, n)):
        submit(ctxs[j], timed(j))
    for i in range(n):
        # drop step i-1's Result before its context is reused: a Result still referenced at
        # the next submit makes the context hand its host buffers over to it
        r = None
        if i + nd - 1 < n:
            submit(ctxs[(i + nd - 1) % nd], timed(i + nd - 1))
        c = ctxs[i % nd]
        r = c.wait()
        if ktimes is not None and timed(i):
            ktimes["__steps"] = ktimes.get("__steps", 0) + 1
            for name, ms in c.kernel_times():
                ktimes[name] = ktimes.get(name, 0.0) + ms
    return r


def measure(args, env, config, n_mg, steps, warmup, host_io=False, no_pipeline=False,
            lazy_stats=True, streams=1, depth=None, entry=None, fixed_total=None):
    """Time ``steps`` steps of the hot path over one synthetic batch of ``config`` (n_mg
    micrographs per rank, inputs resident in HBM; with ``fixed_total``, this rank's share of
    one batch of that many micrographs): barrier + synchronize on both sides, max over ranks.
    ``entry`` names the workload for its PMC record (default: the config).  Returns (report
    dict, cfg, this rank's micrographs)."""
    import torch

    from repic_amd import _lib, synth
    from repic_amd.pipeline import Batch

    dist, world, rank, dev, cdev = env.dist, env.world, env.rank, env.dev, env.cdev
    depth = depth or PIPE_DEPTH.get(config, PIPE_DEPTH_DEFAULT)
    entry = entry or config
    cfg = synth.SynthConfig(**dict(synth.CONFIGS[config], **ENTRY_KW.get(entry, {})),
                            seed=args.seed)
    t_gen = time.time()
    # this rank's shard of one big batch (identical to packing synth.batch's list; large
    # batches are generated by a process pool)
    start = rank * n_mg
    if fixed_total is not None:   # strong scaling: a share of one fixed batch
        start, n_mg = fixed_shard(fixed_total, world, rank)
    procs = min(16, len(os.sched_getaffinity(0))) if n_mg * cfg.n_true * cfg.k >= 2_000_000 else 1
    batch = Batch.from_counts(cfg.k, cfg.box, *synth.packed(cfg, n_mg, start=start, procs=procs))
    # the first micrographs as per-picker arrays, for the CPU baseline's sample
    mgs = synth.batch(cfg, min(n_mg, 64 if config != "C3" else 8), start=start)
    t_gen = time.time() - t_gen
    # the one exchange of the sharded path: global box-id offsets
    if dist is not None:
        tot = torch.tensor([batch.n_boxes], dtype=torch.int64, device=cdev)
        allt = [torch.zeros_like(tot) for _ in range(world)]
        dist.all_gather(allt, tot)
        id_off = int(sum(int(t.item()) for t in allt[:rank]))
        batch.id_base = batch.id_base + id_off

    # inputs resident in HBM (torch only for the allocation / handoff)
    dx = torch.from_numpy(batch.x).to(dev)
    dy = torch.from_numpy(batch.y).to(dev)
    ds = torch.from_numpy(batch.score).to(dev)
    # per-micrograph offsets too (int32 box offsets, int64 id bases): nothing crosses PCIe
    # on the way in; the host copies are only read for launch planning
    dbo = torch.from_numpy(batch.box_off.astype(np.int32)).to(dev)
    did = torch.from_numpy(np.ascontiguousarray(batch.id_base, dtype=np.int64)).to(dev)
    torch.cuda.synchronize()
    # one explicit stream for every context (torch's default stream handle is 0, with which
    # each context would create its own stream, and two in-flight steps would run their
    # kernels concurrently: more throughput, but per-launch kernel times that overlap)
    # (the process's streams, created once: every measure() runs on the same ones; with the
    # null stream they fit the hardware queues, stream_plan)
    stream_plan(depth)
    if env.streams is None:
        env.streams = [torch.cuda.Stream(dev), torch.cuda.Stream(dev)]
    while len(env.streams) < depth:   # (experiments: tools/streams_ab.py --depth)
        env.streams.append(torch.cuda.Stream(dev))
    tstream = env.streams[0]
    stream = tstream.cuda_stream
    ctx = _lib.Context(env.local, stream)
    flags = _lib.F_DEVICE_INPUTS
    # pipelined steps (default): `depth` contexts in flight (rgc_submit / rgc_wait), so the host
    # side of step i+1 (planning, launch) overlaps the device work of step i; every step runs
    # the whole hot path into its own context's outputs and is waited for.  streams=2 (default):
    # each context on a stream of its own, so step i+1's workgroups fill the CUs step i's
    # drain tail leaves idle; streams=1: two contexts on one stream, kernels serialised
    pipeline = not (host_io or no_pipeline)
    if pipeline and streams == 2:
        ctxs = [ctx] + [_lib.Context(env.local, env.streams[j].cuda_stream)
                        for j in range(1, depth)]
    else:
        ctxs = [ctx, _lib.Context(env.local, stream)] if pipeline else [ctx]
    # (non-lazy runs get their stats from the ties kernel on the launch stream; any copy the
    # library still issues goes to the null stream: no extra hardware queue)
    for c in ctxs:
        c.set_copy_stream(0)

    def step(timing=False):
        if host_io:
            return ctx.run(batch.n_mg, cfg.k, cfg.box, batch.box_off, batch.id_base,
                           batch.x, batch.y, batch.score,
                           _lib.F_HOST_OUTPUTS | (_lib.F_TIMING if timing else 0))
        return ctx.run(batch.n_mg, cfg.k, cfg.box, batch.box_off, batch.id_base,
                       dx.data_ptr(), dy.data_ptr(), ds.data_ptr(),
                       flags | (_lib.F_TIMING if timing else 0),
                       dev_meta=(dbo.data_ptr(), did.data_ptr()))

    def submit(c, timing):
        # per-micrograph stats stay in HBM like the per-clique outputs (rgc_wait copies only
        # the run's totals; the last step's stats are fetched after the timed region)
        c.submit(batch.n_mg, cfg.k, cfg.box, batch.box_off, batch.id_base,
                 dx.data_ptr(), dy.data_ptr(), ds.data_ptr(),
                 flags | (_lib.F_LAZY_STATS if lazy_stats else 0) |
                 (_lib.F_TIMING if timing else 0),
                 dev_meta=(dbo.data_ptr(), did.data_ptr()))

    def steps_run(n, timing, ktimes=None):
        """n steps; returns the last step's Result"""
        r = None
        if not pipeline:
            for _ in range(n):
                r = step(timing)
                if ktimes is not None:
                    for name, ms in ctx.kernel_times():
                        ktimes[name] = ktimes.get(name, 0.0) + ms
            return r
        return pipelined_steps(ctxs, submit, n, timing, ktimes)

    overlap = pipeline and streams == 2
    try:
        if warmup:
            steps_run(warmup, False)
        if dist is not None:
            dist.barrier()
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        ktimes = {}
        # overlapping steps: no timing events in the timed region (a launch's events would span
        # the other stream's workgroups too); the per-launch durations come from the
        # serialised leg below
        r = steps_run(steps, not overlap, ktimes)
        torch.cuda.synchronize()
        if dist is not None:
            dist.barrier()
        elapsed = time.perf_counter() - t0
        N, E, C = int(r.n_boxes), int(r.n_edges), int(r.n_cliques)
        V = int(r.n_vert.sum())
        r = None
        if overlap:
            # the roofline's per-launch kernel durations: SER_STEPS steps on one context, one
            # stream, each launch alone on the GPU (HIP events around every kernel)
            ktimes = {"__steps": SER_STEPS}
            for _ in range(SER_STEPS):
                step(True)
                for name, ms in ctx.kernel_times():
                    ktimes[name] = ktimes.get(name, 0.0) + ms
    finally:
        for c in ctxs:
            c.close()
    if dist is not None:
        t = torch.tensor([elapsed], dtype=torch.float64, device=cdev)
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        elapsed = float(t.item())
        # single end-of-run reduction of node-level counts over RCCL/xGMI
        cnt = torch.tensor([n_mg, E, C], dtype=torch.int64, device=cdev)
        dist.all_reduce(cnt)
        tot_mg, tot_e, tot_c = (int(v) for v in cnt.tolist())
    else:
        tot_mg, tot_e, tot_c = n_mg, E, C

    value = tot_mg * steps / elapsed
    nt = ktimes.pop("__steps", steps)   # steps that carried timing events
    avg = {k_: v / nt for k_, v in ktimes.items()}
    dev_ms = sum(v for k_, v in avg.items() if k_ not in ("d2h", "h2d_meta", "d2h_stats"))
    pipe = pipeline_bytes(N, E, C, cfg.k)
    if avg.get("k_fused", 0.0) >= 0.5 * dev_ms:
        # fused route: one kernel runs the whole hot path (plus k_fused_ties, the CPython
        # set-order tie-breaks it hands off), its B_alg is the pipeline's
        dom = "k_fused"
        dom_bytes = alg_bytes(dom, N, E, C, cfg.k, V, n_mg)
        dom_ms = avg[dom] + avg.get("k_fused_ties", 0.0)
    else:
        # large-micrograph route (C3, C5): SURVEY.md §8(d) prices the whole route,
        # achieved = sum B_alg / device time of all its kernels (rocprof: their sum)
        dom = "pipeline (multi-kernel route: " + max(avg, key=avg.get) + " largest)"
        dom_bytes = pipe
        dom_ms = dev_ms
    achieved = dom_bytes / (dom_ms * 1e-3) / 1e9
    rec, traffic_src = pmc_record(entry)
    kind = "k_fused" if dom == "k_fused" else "route"
    dv_kernel = "k_fused" if kind == "k_fused" else max(avg, key=avg.get)
    traffic, hbm_frac, limiter = roofline_evidence(rec, kind, dom_bytes, dom_ms, dv_kernel)
    out = {
        "value": value, "unit": "micrographs/s", "n_gpus": world, "steps": steps,
        "warmup": warmup, "ms_per_step": elapsed / steps * 1e3,
        "config": {"workload": f"{entry}: {dict(synth.CONFIGS[config], **ENTRY_KW.get(entry, {}))}",
                   "micrographs_per_gpu": n_mg if fixed_total is None else fixed_total / world,
                   "micrographs_per_step": tot_mg,
                   "scaling": "weak" if fixed_total is None else "strong",
                   "k": cfg.k, "box_size": cfg.box,
                   "boxes_per_gpu": N, "edges_per_gpu": E, "cliques_per_gpu": C,
                   "parallelism": f"dp{world} (micrograph shards)",
                   "io": "host buffers over PCIe (--host-io)" if host_io else "HBM-resident",
                   "steps_in_flight": len(ctxs) if pipeline else 1,
                   "streams": len(ctxs) if overlap else 1,
                   "stream_plan": stream_plan(depth)},
        "edges_per_sec": tot_e * steps / elapsed,
        "totals": {"micrographs": tot_mg, "edges": tot_e, "cliques": tot_c},
        "roofline": {"bound": derived_bound(rec, kind, dom_bytes, dom_ms, dv_kernel),
                     "priced_against": "hbm (no contraction: no MFMA roofline applies)",
                     "kernel": dom, "achieved": achieved,
                     # the limiter (and bound) come from this build's committed PMC counters
                     "limiter": limiter,
                     "peak": HBM_PEAK_GBS, "unit": "GB/s", "frac": achieved / HBM_PEAK_GBS,
                     "traffic": traffic, "traffic_source": traffic_src,
                     "hbm_frac_measured": hbm_frac,
                     "alg_bytes_per_step": dom_bytes, "alg_bytes_formula":
                         "SURVEY.md 8(d): 28 N + 32 E + C (20 k + 12)",
                     "compulsory_bytes_per_step": fused_compulsory_bytes(N, C, cfg.k, V, n_mg),
                     "kernel_ms_per_step": dom_ms,
                     # the same bytes over the wall time per step (steps overlapping on two
                     # streams finish faster than one launch alone)
                     "frac_step_wall": dom_bytes / (elapsed / steps) / 1e9 / HBM_PEAK_GBS,
                     "timed_steps": (f"HIP events on {nt} serialised steps (one context, one "
                                     f"stream) after the {steps} timed steps, which overlap on "
                                     f"{len(ctxs)} streams" if overlap else
                                     f"HIP events on {nt} of the {steps} timed steps"),
                     "kernel_ms_parts": {k_: round(avg[k_], 5) for k_ in ("k_fused", "k_fused_ties")
                                         if k_ in avg} if dom == "k_fused" else None},
        "pipeline": {"device_ms_per_step": dev_ms, "alg_bytes": pipe,
                     "achieved_gbs": pipe / (dev_ms * 1e-3) / 1e9,
                     "frac": pipe / (dev_ms * 1e-3) / 1e9 / HBM_PEAK_GBS,
                     "kernel_ms": {k_: round(v, 4) for k_, v in sorted(avg.items())}},
        "gen_s": t_gen, "gen_procs": procs,
    }
    return out, cfg, mgs


def by_config_entry(rep):
    """The compact per-config record of the by_config key."""
    r = rep["roofline"]
    return {"value": rep["value"], "unit": rep["unit"], "ms_per_step": rep["ms_per_step"],
            "kernel_ms": r["kernel_ms_per_step"], "kernel": r["kernel"],
            "steps": rep["steps"], "warmup": rep["warmup"],
            "micrographs_per_gpu": rep["config"]["micrographs_per_gpu"],
            "micrographs_per_step": rep["config"]["micrographs_per_step"],
            "scaling": rep["config"]["scaling"],
            "edges_per_sec": rep["edges_per_sec"], "totals": rep["totals"],
            "roofline": {"frac": r["frac"], "achieved": r["achieved"], "bound": r["bound"],
                         "traffic": r["traffic"], "traffic_source": r["traffic_source"],
                         "hbm_frac_measured": r["hbm_frac_measured"], "limiter": r["limiter"],
                         "alg_bytes_per_step": r["alg_bytes_per_step"]},
            "kernel_ms_by_name": rep["pipeline"]["kernel_ms"]}


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=30)
    ap.add_argument("--warmup", type=int, default=10)
    ap.add_argument("--config", default="C2")
    ap.add_argument("--n_mg", type=int, default=None, help="micrographs per GPU")
    ap.add_argument("--seed", type=int, default=0)
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--cpu-budget", type=float, default=12.0)
    ap.add_argument("--host-io", action="store_true",
                    help="PCIe-inclusive variant (never the headline value): host x/y/score and "
                         "offsets are uploaded and every per-clique output is copied back to "
                         "pinned host memory inside each step")
    ap.add_argument("--no-pipeline", action="store_true",
                    help="synchronous rgc_run per step instead of contexts in flight")
    ap.add_argument("--streams", type=int, choices=(1, 2), default=2,
                    help="pipelined steps: 2 (default) puts each context in flight (three) on a "
                         "stream of its own, so step i+1 runs in step i's drain tail; 1 "
                         "serialises two contexts on one stream (the rocprof evidence command: "
                         "per-launch durations that do not overlap)")
    ap.add_argument("--by-config", default=None,
                    help="comma-separated by_config entries (BY_CONFIG names) also timed in this "
                         "run (default: every other BASELINE config at its bench size plus "
                         "C4_100k, when --n_mg is not given; 'none' to skip)")
    ap.add_argument("--by-config-cpu-budget", type=float, default=6.0,
                    help="seconds of the 1-core CPU baseline sample per by_config entry (0: none)")
    ap.add_argument("--no-variants", action="store_true",
                    help="skip stats_copy_variant (profiling runs: only the headline's launches)")
    ap.add_argument("--launch-check", action="store_true", help=argparse.SUPPRESS)
    args = ap.parse_args()

    if "WORLD_SIZE" not in os.environ and args.gpus > 1:
        sys.exit(self_launch(args.gpus))
    world = int(os.environ.get("WORLD_SIZE", "1"))
    if world != args.gpus:
        sys.exit(f"bench.py: --gpus {args.gpus} but WORLD_SIZE={world}")
    if args.launch_check:   # test hook: the launcher's rank layout, no GPU work
        print(json.dumps({k_: os.environ.get(k_) for k_ in
                          ("RANK", "LOCAL_RANK", "WORLD_SIZE", "MASTER_ADDR")}), flush=True)
        return

    env = Env(args)
    n_mg = args.n_mg or DEFAULT_MG[args.config]
    rep, cfg, mgs = measure(args, env, args.config, n_mg, args.steps, args.warmup,
                            host_io=args.host_io, no_pipeline=args.no_pipeline,
                            streams=args.streams)
    out = {"metric": "micrographs/sec (get_cliques, whole node) at 1/2/4/8 MI355X; % HBM roofline"}
    out.update(rep)
    out.update({"higher_is_better": True, "scaling": "weak", "vs_baseline": None,
                "dtype": "f64", "data": "synthetic (seeded SURVEY.md §8(d) generator)",
                "stats_copy": "per-micrograph stats stay in HBM during the timed steps "
                              "(RGC_F_LAZY_STATS, since round 4): each step copies its 128-B "
                              "cursor block; see stats_copy_variant for the rate with every "
                              "step's per-micrograph stats copied to the host"})
    # the other BASELINE configs in the same run (same steps / warmup, their bench sizes:
    # C4 at the 100k / 8-GPU shard of 12.5k micrographs per GPU, C4_100k the whole north-star
    # batch on this GPU), each with a 1-core CPU baseline sample on rank 0
    if args.by_config is None:
        extra = [] if args.n_mg else [c for c in ("C2", "C3", "C4", "C5", "C4_100k", "C5_256",
                                                  "C4_100k_fixed", "C2_frac", "C1", "C2_f2f")
                                      if c != args.config]
    elif args.by_config.lower() == "none":
        extra = []
    else:
        extra = [c.strip() for c in args.by_config.split(",") if c.strip()]
    cpu_rank0 = env.rank == 0 and world == 1
    if extra and not args.host_io:
        byc = {args.config: by_config_entry(rep)}
        cpu_of = {}
        for name in extra:
            if name in F2F_ENTRIES:
                # file to file: the CLI on one GPU (rank 0 of a 1-GPU run only)
                if world == 1:
                    byc[name] = f2f_entry(name, cpu=cpu_rank0 and not args.no_cpu_baseline
                                          and args.by_config_cpu_budget > 0,
                                          cpu_budget=args.by_config_cpu_budget)
                continue
            config, n_c = BY_CONFIG[name]
            if name in FIXED_TOTAL and world == 1 and "C4_100k" in byc:
                # one GPU: the fixed 100k batch IS C4_100k's (same micrographs, same steps)
                byc[name] = dict(byc["C4_100k"], scaling="strong", same_run_as="C4_100k")
                continue
            r_c, cfg_c, mgs_c = measure(args, env, config, n_c, args.steps, args.warmup,
                                        no_pipeline=args.no_pipeline, streams=args.streams,
                                        entry=name,
                                        fixed_total=n_c if name in FIXED_TOTAL else None)
            byc[name] = by_config_entry(r_c)
            if cpu_rank0 and args.by_config_cpu_budget > 0 and not args.no_cpu_baseline:
                if config not in cpu_of:
                    cpu_of[config] = cpu_baseline(cfg_c, mgs_c, args.by_config_cpu_budget,
                                                  procs=1, config=config)
                cb = dict(cpu_of[config])
                if n_c >= 50000:
                    cb["glob_pairing"] = glob_pairing_term(n_c, cfg_c.k)
                byc[name]["cpu_baseline"] = cb
        out["by_config"] = byc
    if cpu_rank0 and not args.no_cpu_baseline:
        out["cpu_baseline"] = cpu_baseline(cfg, mgs, args.cpu_budget, config=args.config)
        if "by_config" in out:
            out["by_config"][args.config]["cpu_baseline"] = out["cpu_baseline"]
    if (not args.host_io and not args.no_pipeline and not args.no_variants
            and n_mg == DEFAULT_MG.get(args.config)):
        # the rate with every step's per-micrograph stats copied to the host (what
        # the CLI reads), next to the headline's lazy-stats rate
        r_s, _, _ = measure(args, env, args.config, n_mg, args.steps, args.warmup,
                            lazy_stats=False, streams=args.streams)
        out["stats_copy_variant"] = {"value": r_s["value"], "ms_per_step": r_s["ms_per_step"],
                                     "note": "same workload, per-micrograph stats (48 B each) "
                                             "copied to pinned host memory in every step"}
    if env.rank == 0:
        print(json.dumps(out), flush=True)
    if env.dist is not None:
        env.dist.destroy_process_group()


def _cli_run(in_dir, out_dir, box, threads=None):
    """One run of the drop-in CLI (repic_amd.commands.get_cliques.main), stdout silenced;
    returns (wall seconds, its LAST_RUN phase record)."""
    import repic_amd.commands.get_cliques as gc
    p = argparse.ArgumentParser()
    gc.add_arguments(p)
    argv = [in_dir, out_dir, str(box)] + (["--threads", str(threads)] if threads else [])
    cli = p.parse_args(argv)
    so = sys.stdout
    with open(os.devnull, "w") as dn:
        sys.stdout = dn
        try:
            t0 = time.perf_counter()
            gc.main(cli)
            wall = time.perf_counter() - t0
        finally:
            sys.stdout = so
    return wall, dict(gc.LAST_RUN)


def _c1_cpu_sample(in_dir, budget_s):
    """The oracle's faithful per-micrograph path (oracle/cpu_ref.py, the reference's
    get_jaccard loop structure) on the 10017 micrographs, parsed (untimed) by the product's
    ingest plan, until ``budget_s`` has elapsed: (micrographs, seconds) on 1 core."""
    from oracle import cpu_ref
    from repic_amd import ingest
    methods = ingest.list_methods(in_dir)
    mgs, _, _ = ingest.plan(in_dir, methods, ingest.DirIndex(in_dir, methods))
    t0 = time.perf_counter()
    n = 0
    for mg in mgs:
        if mg.status != "ok":
            continue
        nid, coords = mg.id_base, []
        for pf in mg.coords:
            coords.append([(float(a), float(b), float(c), nid + i)
                           for i, (a, b, c) in enumerate(zip(pf.x, pf.y, pf.s))])
            nid += pf.n
        cpu_ref.micrograph(coords, 180, methods, faithful=True)
        n += 1
        if time.perf_counter() - t0 > budget_s:
            break
    return n, time.perf_counter() - t0


def f2f_entry(name, cpu=True, cpu_budget=6.0):
    """File-to-file rate of the drop-in CLI (BOX text in, the five files per micrograph out),
    never the headline: C1 = the reference's EMPIAR-10017 example (tests/golden/inputs_10017,
    12 micrographs; a warm-up run, then the median of 5 timed runs, each into a fresh output
    directory) beside the reference's own rate on it; C2_f2f = 10k C2 micrographs written as
    BOX text to /tmp first (not timed), then one timed CLI run (a first run: the writes of 50k
    fresh files depend on the file system's state)."""
    import shutil
    import tempfile
    work = tempfile.mkdtemp(prefix="rgc_bench_f2f_", dir="/tmp")
    try:
        if name == "C1":
            in_dir = os.path.join(ROOT, "tests", "golden", "inputs_10017")
            n_mg, box = 12, 180
            _cli_run(in_dir, os.path.join(work, "warm"), box)
            walls, last = [], None
            for i in range(5):
                w, last = _cli_run(in_dir, os.path.join(work, f"out{i}"), box)
                walls.append(w)
            wall = float(np.median(walls))
            out = {"value": n_mg / wall, "unit": "micrographs/s (file to file)",
                   "micrographs": n_mg, "wall_s": wall, "wall_s_runs": walls,
                   "workload": "EMPIAR-10017 example (BASELINE configs[0]): crYOLO / deepPicker "
                               "/ topaz BOX, box 180, the reference's own input files",
                   "phases_s": {k_: round(v, 4) for k_, v in last.items() if k_.endswith("_s")},
                   "cliques": last.get("cliques"),
                   "reference_cpu": {"value": REF_C1_RATE, "unit": "micrographs/s",
                                     "cores": 1, "kind": "reference",
                                     "source": "BASELINE.md §2: the reference's get_cliques run "
                                               "on these files, 1 core (34.75 s)"}}
            out["vs_reference_cpu"] = out["value"] / REF_C1_RATE
            if cpu:
                n, dt = _c1_cpu_sample(in_dir, cpu_budget)
                out["cpu_baseline"] = {"value": n / dt, "unit": "micrographs/s", "cores": 1,
                                       "kind": "port", "cpu_model": _cpu_model(),
                                       "sample": f"{n} of the 12 micrographs, oracle faithful "
                                                 f"path, 1 process, {dt:.1f} s"}
            return out
        from repic_amd import synth
        sys.path.insert(0, os.path.join(ROOT, "tools"))
        from file_bench import _write_inputs as write_inputs
        cfg = synth.SynthConfig(**synth.CONFIGS["C2"], seed=0)
        n_mg = 10000
        threads = min(16, len(os.sched_getaffinity(0)))
        in_dir = os.path.join(work, "in")
        t0 = time.perf_counter()
        write_inputs(in_dir, cfg, n_mg, threads)
        gen = time.perf_counter() - t0
        warm = os.path.join(work, "warm")
        synth.write_box_dirs(warm, cfg, 2)
        _cli_run(warm, os.path.join(work, "warm_out"), cfg.box)
        wall, last = _cli_run(in_dir, os.path.join(work, "out"), cfg.box, threads)
        return {"value": n_mg / wall, "unit": "micrographs/s (file to file)",
                "micrographs": n_mg, "wall_s": wall, "gen_s": gen, "threads": threads,
                "workload": "C2 (10k synthetic micrographs x 3 pickers as BOX text in /tmp, "
                            "box 180), first run",
                "phases_s": {k_: round(v, 4) for k_, v in last.items() if k_.endswith("_s")},
                "cliques": last.get("cliques"), "edges": last.get("edges")}
    finally:
        shutil.rmtree(work, ignore_errors=True)


def glob_pairing_term(n_mg, k, sample=20000):
    """BASELINE.md §3 for C4 at 100k: the reference pairs each micrograph with its partner
    files by ``glob(in/methods[p]/*{base}*)`` (get_cliques.py:94,121), a scan of the whole
    picker directory per call: M (k - 1) calls of O(M) each.  Timed here on a directory of
    ``sample`` empty files named like the synthetic ones, scaled linearly to M files; the
    CPU baseline's per-micrograph rate above excludes it."""
    import glob
    import tempfile
    with tempfile.TemporaryDirectory(dir="/tmp") as d:
        for i in range(sample):
            open(os.path.join(d, f"mg{i:06d}.box"), "w").close()
        t0 = time.perf_counter()
        reps = 5
        for r in range(reps):
            assert len(glob.glob(os.path.join(d, f"*mg{(r * 3571) % sample:06d}*"))) == 1
        per = (time.perf_counter() - t0) / reps
    per_m = per * n_mg / sample
    return {"seconds_per_glob_at_M": per_m, "calls": n_mg * (k - 1),
            "total_hours": per_m * n_mg * (k - 1) / 3600.0,
            "sample": f"glob over a directory of {sample} files: {per * 1e3:.2f} ms per call, "
                      f"scaled linearly to {n_mg} files; not part of the CPU rate"}


if __name__ == "__main__":
    main()
