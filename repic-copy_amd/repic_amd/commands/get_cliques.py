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
from ..ingest import DirIndex, list_methods, micrograph_names, plan_chunk, probe_start_method
from ..pipeline import split_batches
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
    """Per-micrograph pair-loop work estimate for balanced contiguous shards (SURVEY.md
    §8(e)): 1 + s^2 * k (k - 1) / 2 from the size s of the micrograph's picker-0 BOX file (a
    proxy for sum over picker pairs of n_j * n_l, get_cliques.py:135-138).  One stat per
    micrograph, from a thread pool (os.stat releases the GIL); no partner lookups."""
    from concurrent.futures import ThreadPoolExecutor
    d0 = os.path.join(in_dir, methods[0])

    def size(name):
        try:
            return os.stat(os.path.join(d0, name)).st_size
        except OSError:
            return 0
    with ThreadPoolExecutor(16) as ex:
        s = np.fromiter(ex.map(size, names, chunksize=256), np.float64, len(names))
    k = len(methods)
    return 1.0 + s * s * (k * (k - 1) / 2.0)


def _main(args, ctx, world, rank):
    t_start = time.time()
    dist = None
    if world > 1:
        import torch.distributed as dist
        if not dist.is_initialized():
            dist.init_process_group(_dist_backend(world))
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
    if dist is not None:
        b = shard_bounds(_shard_weights(args.in_dir, methods, index, names), world)
        lo, hi = b[rank], b[rank + 1]
    run = _Run(args, ctx, methods, index, names[lo:hi], lo)
    # optimistic sharded writes need distinct output names: a failure's cleanup must never
    # remove a file an earlier micrograph of another shard also wrote
    run.unique_bases = len({n.replace(".box", "") for n in names}) == len(names)
    writer = None
    try:
        # large runs write from spawned processes, started now so they import during the
        # parse and the device work
        writer = Writer(getattr(args, "threads", None),
                        processes=len(names) >= PROC_WRITER_MIN * max(1, world))
        if dist is None:
            run.stream(writer)
        else:
            run.sharded(writer, dist, rank)
    finally:
        t_w = time.time()
        if writer is not None:
            writer.close()
        run.stats["write_tail_s"] = time.time() - t_w
        LAST_RUN.clear()
        LAST_RUN.update(index_s=t_index, total_s=time.time() - t_start, **run.stats)
        if dist is not None and run.stats.get("reduce", True):
            # node-level counters: one reduction at the end of the run, over
            # RCCL when every rank owns its own GPU
            st = run.stats
            tot = reduce_counts([st["micrographs"], st["edges"], st["cliques"]],
                                device=_counter_device(ctx))
            if rank == 0:
                print(f"get_cliques: {tot[0]} micrographs, {tot[1]} edges, {tot[2]} cliques "
                      f"on {world} ranks")
    sys.stdout.flush()


def _distinct_gpus(world):
    """True when every rank of this node can own its own GPU (LOCAL_RANK < device count and
    the node's ranks fit the devices), so collectives can run over RCCL."""
    try:
        lw = int(os.environ.get("LOCAL_WORLD_SIZE", world))
        return 0 < lw <= _lib.device_count() and os.environ.get("RGC_CLI_GLOO") is None
    except Exception:  # noqa: BLE001
        return False


def _dist_backend(world):
    """Control-plane collectives (a few int64 per rank) on gloo; with one GPU per rank the
    device tensors of the end-of-run counter reduction go over RCCL."""
    return "cpu:gloo,cuda:nccl" if _distinct_gpus(world) else "gloo"


def _counter_device(ctx):
    import torch
    import torch.distributed as dist
    if "nccl" in str(dist.get_backend()).lower():
        torch.cuda.set_device(ctx.device)
        return torch.device("cuda", ctx.device)
    return None


# micrographs per pipeline chunk (parse of chunk i+1 | device chunk i | writes of chunk i-1)
CHUNK_MG = 1024
# micrographs per writer task
GROUP_MG = 64
# ... or fewer when their cliques reach this many: a group is one writer thread's task, so a
# chunk of large micrographs (C5: ~1 M cliques each) is spread over the writer threads instead
# of leaving one thread a multi-second tail
GROUP_CLIQUES = 1 << 18


class _Run:
    """One rank's pass over its micrographs, chunk by chunk (reference get_cliques.py:108-229
    order and failure semantics)."""

    def __init__(self, args, ctx, methods, index, names, lo):
        self.args, self.ctx, self.methods, self.index = args, ctx, methods, index
        self.names, self.lo = names, lo
        self.k = len(methods)
        self.stats = dict(parse_s=0.0, device_s=0.0, write_s=0.0, micrographs=0, edges=0,
                          cliques=0, chunks=0)
        self.chunk = max(1, int(getattr(args, "chunk_mg", None) or CHUNK_MG))

    # -- stages
    def plan_chunks(self):
        """Planned chunks in order (the id counter runs across them); stops after a crash."""
        nid = 0
        for c0 in range(0, len(self.names), self.chunk):
            t0 = time.time()
            ch = plan_chunk(self.args.in_dir, self.methods, self.index,
                            self.names[c0:c0 + self.chunk], self.k, self.args.box_size, nid,
                            getattr(self.args, "threads", None))
            ch.first = self.lo + c0
            ch.parse_s = time.time() - t0
            nid = ch.consumed
            yield ch
            if ch.crash is not None:
                return

    def device(self, ch):
        """Device results of a chunk's ok micrographs (flat host copies)."""
        ch.res = None
        if ch.batch is None:
            return
        t0 = time.time()
        b = ch.batch
        for m0, m1 in split_batches(np.diff(b.box_off[::self.k]).tolist(),
                                    getattr(self.args, "batch_boxes", 1 << 25)):
            part = b if (m0 == 0 and m1 == b.n_mg) else b.slice(m0, m1)
            r = _FlatResult(self.ctx, part, self.args.get_cc, self.args.multi_out,
                            getattr(self.args, "no_fused", False))
            ch.res = r if ch.res is None else ch.res.append(r, int(b.box_off[m0 * self.k]))
        self.stats["device_s"] += time.time() - t0
        ok = ch.res.status == _lib.OK
        self.stats["edges"] += int(ch.res.n_edges_mg[ok].sum())
        self.stats["cliques"] += int(ch.res.clique_cnt[ok].sum())

    def first_failure(self, ch):
        """Index in ch.mgs of the first micrograph at which the reference raises, or None."""
        for i, mg in enumerate(ch.mgs):
            if mg.status == "crash" or (mg.status == "ok" and
                                        ch.res.status[mg.slot] != _lib.OK):
                return i
        return None

    def write(self, ch, writer, stop=None):
        """Print and write the chunk's micrographs in order up to ``stop`` (exclusive), in
        groups; returns the micrograph the reference would raise at (if it is < stop)."""
        mgs = ch.mgs if stop is None else ch.mgs[:stop]
        share = (ch.parse_s + getattr(ch, "dev_s", 0.0)) / max(1, len(ch.mgs))
        t0 = time.time()
        items, slots = [], []
        gcl = 0
        raise_at = None
        for i, mg in enumerate(mgs):
            print(f"\n--- {mg.base} ---\n")
            if mg.status == "skip":
                print("Skipping micrograph - not all methods have picked particles...")
                items.append((mg.base, -1, 0, 0, 0, 0.0, None))
                slots.append(-1)
            elif mg.status == "crash" or ch.res.status[mg.slot] != _lib.OK:
                raise_at = mg
                break
            else:
                items.append((mg.base, 0, 0, 0, 0, share, None))
                slots.append(mg.slot)
                gcl += int(ch.res.clique_cnt[mg.slot])
                self.stats["micrographs"] += 1
            if len(items) >= GROUP_MG or gcl >= GROUP_CLIQUES:
                self._submit_group(ch, items, slots, writer)
                items, slots = [], []
                gcl = 0
        if items:
            self._submit_group(ch, items, slots, writer)
        self.stats["write_s"] += time.time() - t0
        return raise_at

    @staticmethod
    def raise_for(mg, ch):
        if mg.status == "crash":
            raise mg.exc
        st = ch.res.status[mg.slot]
        if st == _lib.NO_EDGES:
            raise ValueError("zero-size array to reduction operation maximum which has no identity")
        raise UnboundLocalError("local variable 'clique' referenced before assignment")

    def _submit_group(self, ch, items, slots, writer):
        r, b, k = ch.res, ch.batch, self.k
        sl = np.array([s for s in slots if s >= 0], np.int64)
        if len(sl):
            cnt = r.clique_cnt[sl]
            base = r.clique_base[sl]
            tot = int(cnt.sum())
            idx = np.repeat(base - (np.cumsum(cnt) - cnt), cnt) + np.arange(tot)
            g = r.consensus[idx].astype(np.int64)
            idb = b.id_base[sl] - b.box_off[sl * k]
            w, conf, rows = r.w[idx], r.conf[idx], r.rows[idx]
            cx, cy, cid = b.x[g], b.y[g], g + np.repeat(idb, cnt)
        else:
            cnt = np.zeros(0, np.int64)
            w = conf = cx = cy = np.zeros(0)
            rows = np.zeros((0, k), np.int32)
            cid = np.zeros(0, np.int64)
        out, j = [], 0
        for it, s in zip(items, slots):
            if s < 0:
                out.append(it)
                continue
            coords = self._multi_out_coords(ch, s) if self.args.multi_out else None
            out.append((it[0], int(cnt[j]), int(r.n_vert[s]), int(r.cc_max[s]), int(r.cc_cnt[s]),
                        it[5], coords))
            j += 1
        writer.group(self.args.out_dir, out, w, conf, rows, cx, cy, cid)

    def _multi_out_coords(self, ch, s):
        """--multi_out table of ok micrograph slot s (get_cliques.py:175-178, 206-213)."""
        r, b, k = ch.res, ch.batch, self.k
        c0, c1 = int(r.clique_base[s]), int(r.clique_base[s] + r.clique_cnt[s])
        idb = int(b.id_base[s]) - int(b.box_off[s * k])

        def tup(g):
            return (float(b.x[g]), float(b.y[g]), idb + int(g))
        member_tuples = [[tup(g) for g in row] for row in r.members[c0:c1].tolist()]
        picker_coords = []
        for p in range(k):
            p0, p1 = int(b.box_off[s * k + p]), int(b.box_off[s * k + p + 1])
            sc = b.score[p0:p1]
            ws = list(sc) if ch.sig[s, p] else sc.tolist()
            picker_coords.append(list(zip(b.x[p0:p1].tolist(), b.y[p0:p1].tolist(), ws,
                                          range(idb + p0, idb + p1))))
        return multi_out_coords(self.methods, member_tuples, r.order[c0:c1].tolist(), k,
                                self.args.get_cc, picker_coords)

    # -- drivers
    def stream(self, writer):
        """Single rank: a parser thread plans chunk i+1 (the C++ parse releases the GIL) while
        this thread runs chunk i on the device and hands its writes to the writer pool."""
        import queue
        import threading
        q = queue.Queue(maxsize=2)
        stop = threading.Event()

        def put(item):
            """Queue ``item`` unless the consumer has stopped (it raised, or is done): every
            put, the end sentinel and a parser exception included, gives up once ``stop`` is
            set, so the join below cannot wait on a full queue nobody reads."""
            while not stop.is_set():
                try:
                    q.put(item, timeout=0.1)
                    return True
                except queue.Full:
                    continue
            return False

        def produce():
            try:
                for ch in self.plan_chunks():
                    if not put(ch):
                        return
            except BaseException as e:  # noqa: BLE001 - re-raised by the consumer
                put(e)
                return
            put(None)

        th = threading.Thread(target=produce, name="rgc-parse", daemon=True)
        th.start()
        try:
            while True:
                ch = q.get()
                if ch is None:
                    break
                if isinstance(ch, BaseException):
                    raise ch
                self.stats["parse_s"] += ch.parse_s
                self.stats["chunks"] += 1
                t0 = time.time()
                self.device(ch)
                ch.dev_s = time.time() - t0
                bad = self.write(ch, writer)
                if bad is not None:
                    writer.close()        # every earlier micrograph's files exist first
                    self.raise_for(bad, ch)
        finally:
            stop.set()
            th.join()

    def sharded(self, writer, dist, rank):
        """One shard of a multi-rank run.  The shard's global id offset needs every lower
        shard's consumed ids, so the shard is parsed first (all ranks in parallel) and one
        all-gather exchanges the counts; then chunks stream through the device with their
        writes handed to the writer pool (device of chunk i+1 overlaps the writes of chunk i).
        Writes are optimistic: a rank does not wait for the lower ranks' outcome.  The ranks
        agree on the first failing micrograph at the end; files of micrographs at or after
        it are removed again (the reference never wrote them), the rank owning it raises the
        reference's exception, and every earlier micrograph's files exist."""
        t_run = time.time()
        spans = self.stats.setdefault("spans", [])
        chunks, err = [], None
        try:
            for ch in self.plan_chunks():
                self.stats["parse_s"] += ch.parse_s
                spans.append(("parse", ch.first, time.time() - ch.parse_s - t_run,
                              time.time() - t_run))
                chunks.append(ch)
        except Exception as e:  # noqa: BLE001 - re-raised by agree() after the exchange
            err = e
        consumed = chunks[-1].consumed if chunks else 0
        cons = agree(err, [consumed])
        id_off = sum(c[0] for c in cons[:rank])
        fail, stop_ch = None, None
        optimistic = getattr(self, "unique_bases", True)
        writer.spans, writer.t0 = spans, t_run
        done = []
        try:
            for ch in chunks:
                ch.shift_ids(id_off)
                t0 = time.time()
                self.device(ch)
                ch.dev_s = time.time() - t0
                spans.append(("device", ch.first, t0 - t_run, time.time() - t_run))
                self.stats["chunks"] += 1
                done.append(ch)
                i = self.first_failure(ch)
                if optimistic:
                    self.write(ch, writer, i)        # up to its first failure (exclusive)
                if i is not None:
                    fail = ch.first + i
                    stop_ch = (ch, ch.mgs[i])
                    break
        except Exception as e:  # noqa: BLE001
            err = e
        big = np.iinfo(np.int64).max
        rows = agree(err, [big if fail is None else fail])
        gfail = min(r_[0] for r_ in rows)
        if not optimistic:       # (duplicate output names) writes only up to the agreed failure
            for ch in done:
                if gfail < ch.first:
                    break
                self.write(ch, writer, gfail - ch.first if gfail < ch.first + len(ch.mgs)
                           else None)
        if gfail == big:
            return
        # a micrograph raises: every pending write lands first, then the files of the
        # micrographs from the failing one on are removed (this shard's part of them)
        writer.close()
        if optimistic:
            # exactly the files the writer wrote for those micrographs (Writer.written)
            gi = {mg.base: ch.first + i for ch in done for i, mg in enumerate(ch.mgs)}
            _remove_outputs(self.args.out_dir, [(b, sfx) for b, sfx in writer.written
                                                if gi.get(b, -1) >= gfail])
        if fail == gfail:
            self.raise_for(stop_ch[1], stop_ch[0])


def _remove_outputs(out_dir, written):
    """Remove files this run wrote: ``written`` = (base, suffixes) pairs, the empty
    <base>.box of a skip or the four pickles and the runtime.tsv of a micrograph with
    cliques.  Nothing else in out_dir is touched (e.g. a run_ilp <base>.box)."""
    for b, sufs in written:
        for suf in sufs:
            try:
                os.remove(os.path.join(out_dir, b + suf))
            except FileNotFoundError:
                pass


class _FlatResult:
    """Host copies of one device run's outputs (the library's buffers are reused by the next
    run, which may start before these are written)."""

    PER_MG = ("status", "cc_max", "cc_cnt", "n_vert", "n_edges_mg", "clique_base", "clique_cnt")

    def __init__(self, ctx, batch, get_cc, multi_out, no_fused=False):
        flags = _lib.F_HOST_OUTPUTS
        if no_fused:
            flags |= _lib.F_NO_FUSED
        if get_cc:
            flags |= _lib.F_GET_CC
        if multi_out:
            flags |= _lib.F_MULTI_OUT
        r = ctx.run(batch.n_mg, batch.k, batch.box_size, batch.box_off, batch.id_base, batch.x,
                    batch.y, batch.score, flags)
        for f in self.PER_MG:
            setattr(self, f, np.array(getattr(r, f)))
        self.rows, self.w, self.conf = r.rows.copy(), r.w.copy(), r.conf.copy()
        self.consensus = r.consensus.copy()
        self.members = r.members.copy() if r.members is not None else None
        self.order = r.order.copy() if r.order is not None else None

    def append(self, o, box0):
        """Concatenate a later sub-batch's result (its box indices start at box0)."""
        C = len(self.w)
        for f in self.PER_MG:
            setattr(self, f, np.concatenate([getattr(self, f), getattr(o, f)]))
        self.clique_base[-len(o.status):] += C
        self.rows = np.concatenate([self.rows, o.rows])
        self.w = np.concatenate([self.w, o.w])
        self.conf = np.concatenate([self.conf, o.conf])
        self.consensus = np.concatenate([self.consensus, o.consensus + box0])
        if self.members is not None:
            self.members = np.concatenate([self.members, o.members + box0])
            self.order = np.concatenate([self.order, o.order]) if self.order is not None else None
        return self
