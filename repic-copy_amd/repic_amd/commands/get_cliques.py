"""``repic get_cliques`` — drop-in subcommand, MI355X hot path.

Same plugin protocol as the reference module (reference repic/commands/get_cliques.py:13-27,72):
``name``, ``add_arguments(parser)``, ``main(args)``; same positional arguments and flags;
same side effects (``out_dir`` deleted and recreated, the same five files per micrograph,
an empty ``<base>.box`` for skipped micrographs) and the same exception classes at the same
micrograph when the reference would crash.  The work between parsing and writing runs as
batched HIP kernels (``librepic_gc.so``); there is no CPU fallback.

Extra options (do not change outputs): ``--batch_boxes`` (boxes per device batch),
``--threads`` (host parser threads), ``--device``.
"""
from __future__ import annotations

import argparse
import os
import shutil
import sys
import time
from pathlib import Path

import numpy as np

from .. import _lib
from ..dist import agree, pair_work, reduce_counts, shard_bounds
from ..ingest import DirIndex, list_methods, micrograph_names, plan, probe_start_method
from ..pipeline import Batch, run_batch, split_batches
from ..writers import Writer, multi_out_coords

name = "get_cliques"

# phase seconds and totals of the last run in this process (tools/file_bench.py reads them)
LAST_RUN: dict = {}
# micrographs per rank from which the writer uses processes instead of threads
PROC_WRITER_MIN = 512


def add_arguments(parser):
    """Same CLI surface as the reference (get_cliques.py:16-27) plus tuning knobs."""
    parser.add_argument("in_dir",
                        help="path to input directory containing subdirectories of particle coordinate files ")
    parser.add_argument("out_dir",
                        help="path to output directory (WARNING - script will delete directory if it exists)")
    parser.add_argument("box_size", type=int,
                        help="particle detection box size (in int[pixels])")
    parser.add_argument("--multi_out", action="store_true",
                        help="set output of cliques to be members sorted by picker name")
    parser.add_argument("--get_cc", action="store_true",
                        help="filters cliques for those in the largest Connected Component (CC)")
    parser.add_argument("--batch_boxes", type=int, default=1 << 25,
                        help="max boxes per device batch (does not change outputs)")
    parser.add_argument("--threads", type=int, default=None,
                        help="host BOX-parser threads (does not change outputs)")
    parser.add_argument("--device", type=int, default=None,
                        help="HIP device (default: $LOCAL_RANK or 0)")
    # tests only: JSON {picker: [names in readdir order]} replayed instead of os.listdir, so
    # global box ids (and the consensus tie-breaks) match a recorded reference run
    parser.add_argument("--listing", type=_load_listing, default=None, help=argparse.SUPPRESS)


def _load_listing(path):
    import json
    with open(path) as f:
        return json.load(f)


def _del_dir(path):
    p = Path(path)
    if p.exists() and p.is_dir():
        shutil.rmtree(p)


def _dist_env():
    world = int(os.environ.get("WORLD_SIZE", "1"))
    return world, int(os.environ.get("RANK", "0")), int(os.environ.get("LOCAL_RANK", "0"))


def main(args):
    """get_cliques.py:72-229 semantics; under torchrun (WORLD_SIZE > 1) every rank takes a
    contiguous shard of the micrographs on its own GPU."""
    assert os.path.exists(args.in_dir), "Error - input directory does not exist"
    world, rank, local = _dist_env()
    dev = args.device if getattr(args, "device", None) is not None else local
    # the HIP context is created before torch.distributed is imported (a child that
    # initialised gloo first could not see the device on the GPU pool)
    ctx = _lib.Context(dev)
    try:
        _main(args, ctx, world, rank)
    finally:
        ctx.close()


def _methods_after_reset(in_dir, out_dir):
    """The picker list the reference will see once out_dir is deleted (get_cliques.py:77-82):
    out_dir itself is not a picker even when it lies inside in_dir."""
    out = os.path.realpath(out_dir)
    return [m for m in list_methods(in_dir)
            if os.path.realpath(os.path.join(in_dir, m)) != out]


def _shard_weights(in_dir, methods, index, names):
    """Per-micrograph pair-loop work estimate (sum over picker pairs of the product of the BOX
    file sizes, a proxy for n_j * n_l) for balanced contiguous shards."""
    w = np.empty(len(names))
    for i, name in enumerate(names):
        base = name.replace(".box", "")
        sizes = []
        for p, m in enumerate(methods):
            fl = [name] if p == 0 else index.glob(m, f"*{base}*")
            try:
                sizes.append(sum(os.stat(os.path.join(in_dir, m, f)).st_size for f in fl))
            except OSError:
                sizes.append(0)
        w[i] = 1.0 + pair_work(sizes)
    return w


def _main(args, ctx, world, rank):
    t_start = time.time()
    dist = None
    if world > 1:
        import torch.distributed as dist
        if not dist.is_initialized():
            dist.init_process_group("gloo")   # control-plane only: a few int64 per rank
    assert os.path.exists(args.in_dir), "Error - input directory does not exist"
    # checked before anything is deleted: the device kernels are compiled for k <= MAX_K
    k_pre = len(_methods_after_reset(args.in_dir, args.out_dir))
    if k_pre > _lib.MAX_K:
        raise _lib.RGCError(f"{k_pre} picker directories in {args.in_dir}: this build supports "
                            f"at most {_lib.MAX_K} (no output was deleted or written)")
    if rank == 0:
        _del_dir(args.out_dir)
    if dist is not None:
        dist.barrier()
    methods = list_methods(args.in_dir)
    Path(args.out_dir).mkdir(parents=True, exist_ok=True)
    listing = getattr(args, "listing", None)     # tests: replay a recorded readdir order
    index = DirIndex(args.in_dir, methods, listing)
    start = probe_start_method(index, methods)
    if rank == 0:
        print(f"Using {start} BOX files as starting point")
    names = micrograph_names(index, methods)
    t_index = time.time() - t_start
    lo, hi = 0, len(names)
    # large runs write from spawned processes, started now so they import during the parse
    # and the device work
    writer = Writer(getattr(args, "threads", None),
                    processes=len(names) >= PROC_WRITER_MIN * max(1, world))
    if dist is not None:
        b = shard_bounds(_shard_weights(args.in_dir, methods, index, names), world)
        lo, hi = b[rank], b[rank + 1]
    k = len(methods)
    t_plan = time.time()
    mgs, results, err, consumed = [], {}, None, 0
    try:
        mgs, crash, consumed = plan(args.in_dir, methods, index, order=names[lo:hi],
                                    n_threads=getattr(args, "threads", None))
    except Exception as e:  # noqa: BLE001 - re-raised by agree() after the exchange
        err = e
    if dist is not None:
        # global box-id offset of this shard (the one data exchange), with failure agreement
        cons = agree(err, [consumed])
        id_off = sum(c[0] for c in cons[:rank])
        for mg in mgs:
            mg.id_base += id_off
    elif err is not None:
        raise err
    ok = [mg for mg in mgs if mg.status == "ok"]
    t_plan = time.time() - t_plan
    t_dev = 0.0
    n_edges = n_cliques = 0
    try:
        if ok:
            counts = [sum(c.n for c in mg.coords) for mg in ok]
            for m0, m1 in split_batches(counts, getattr(args, "batch_boxes", 1 << 25)):
                part = ok[m0:m1]
                batch = Batch.pack(k, args.box_size, [[(c.x, c.y, c.s) for c in mg.coords]
                                                     for mg in part],
                                   id_bases=[mg.id_base for mg in part])
                t0 = time.time()
                res = run_batch(ctx, batch, get_cc=args.get_cc, multi_out=args.multi_out)
                t_dev += time.time() - t0
                for j, mg in enumerate(part):
                    results[id(mg)] = (batch, j, res[j])
                    n_edges += res[j].n_edges
                    n_cliques += len(res[j].w)
    except Exception as e:  # noqa: BLE001
        if dist is None:
            raise
        err = e
    # first micrograph (global index) at which the reference would raise
    fail = None
    if err is None:
        for i, mg in enumerate(mgs):
            if mg.status == "crash" or (mg.status == "ok" and
                                        results[id(mg)][2].status != _lib.OK):
                fail = lo + i
                break
    if dist is not None:
        big = np.iinfo(np.int64).max
        rows = agree(err, [big if fail is None else fail])
        gfail = min(r[0] for r in rows)
        gfail = None if gfail == big else gfail
    else:
        gfail = fail
    share = (t_plan + t_dev) / max(1, len(mgs))
    t_write = time.time()
    try:
        _write_all(args, mgs, results, methods, k, lo, fail, gfail, share, writer)
    finally:
        writer.close()
        LAST_RUN.clear()
        LAST_RUN.update(index_s=t_index, parse_s=t_plan, device_s=t_dev,
                        write_s=time.time() - t_write, total_s=time.time() - t_start,
                        micrographs=len(ok), edges=n_edges, cliques=n_cliques)
        if dist is not None:
            # node-level counters: one reduction at the end of the run
            tot = reduce_counts([len(ok), n_edges, n_cliques])
            if rank == 0:
                print(f"get_cliques: {tot[0]} micrographs, {tot[1]} edges, {tot[2]} cliques "
                      f"on {world} ranks")
    sys.stdout.flush()


def _write_all(args, mgs, results, methods, k, lo, fail, gfail, share, writer):
    """Write outputs in reference order; raise the reference's exception where it would."""
    for i, mg in enumerate(mgs):
        if gfail is not None and lo + i > gfail:
            break
        if gfail is not None and lo + i == gfail and fail != gfail:
            break
        print(f"\n--- {mg.base} ---\n")
        if mg.status == "skip":
            print("Skipping micrograph - not all methods have picked particles...")
            writer.skip(args.out_dir, mg.base)
            continue
        if mg.status == "crash":
            raise mg.exc
        t0 = time.time()
        batch, j, r = results[id(mg)]
        if r.status == _lib.NO_EDGES:
            raise ValueError("zero-size array to reduction operation maximum which has no identity")
        if r.status == _lib.NO_CLIQUES:
            raise UnboundLocalError("local variable 'clique' referenced before assignment")
        b0 = int(batch.box_off[j * k])
        idb = int(batch.id_base[j]) - b0
        cx = cy = cid = coords = None
        if args.multi_out:
            def tup(g):
                return (float(batch.x[g]), float(batch.y[g]), idb + int(g))
            member_tuples = [[tup(g) for g in row] for row in r.members.tolist()]
            picker_coords = []
            for p, c in enumerate(mg.coords):
                ids = range(idb + int(batch.box_off[j * k + p]),
                            idb + int(batch.box_off[j * k + p + 1]))
                ws = list(c.s) if c.sigmoid else c.s.tolist()
                picker_coords.append(list(zip(c.x.tolist(), c.y.tolist(), ws, ids)))
            coords = multi_out_coords(methods, member_tuples, r.order.tolist(), k, args.get_cc,
                                      picker_coords)
        else:
            g = r.consensus.astype(np.int64)
            cx, cy, cid = batch.x[g], batch.y[g], idb + g
        writer.micrograph(args.out_dir, mg.base, r.w, r.conf, r.rows, r.n_vert, cx, cy, cid,
                          coords, share + (time.time() - t0), r.cc_max, r.cc_cnt)
