"""GPU parity: the HIP path (through the C-ABI) against the reference's golden outputs and the
CPU oracle.  Bit-exact: clique sets, constraint matrices, float32 weights / confidences,
consensus coordinates (canonical column order); f64 Jaccard indices enter
only through those outputs, so the 1e-12 relative tolerance of BASELINE.json is met with 0.
"""
import argparse
import builtins
import os

import numpy as np
import pytest

from golden_util import assert_matches_golden, golden_cases, load_case, make_inputs, read_outputs

pytestmark = pytest.mark.gpu


def _args(in_dir, out_dir, meta, **kw):
    a = argparse.Namespace(in_dir=in_dir, out_dir=out_dir, box_size=meta["box"],
                           multi_out="--multi_out" in meta["flags"],
                           get_cc="--get_cc" in meta["flags"], batch_boxes=1 << 25,
                           threads=None, device=None, listing=meta["listing"])
    for k_, v in kw.items():
        setattr(a, k_, v)
    return a


def _run_case(name, tmp_path, no_fused=False, **kw):
    from repic_amd.commands import get_cliques
    meta, data = load_case(name)
    in_dir = make_inputs(name, str(tmp_path))
    out_dir = os.path.join(str(tmp_path), "out")
    exc = None
    try:
        get_cliques.main(_args(in_dir, out_dir, meta, no_fused=no_fused, **kw))
    except Exception as e:  # noqa: BLE001 - the exception class is part of the contract
        exc = e
    if meta["exception"]:
        assert exc is not None and isinstance(exc, getattr(builtins, meta["exception"])), exc
    else:
        assert exc is None, repr(exc)
    mgs, arrays = read_outputs(out_dir, meta)
    assert_matches_golden(meta, data, mgs, arrays)


@pytest.mark.parametrize("name", golden_cases())
def test_gpu_matches_reference_golden(name, tmp_path):
    _run_case(name, tmp_path)


@pytest.mark.parametrize("name", golden_cases())
def test_gpu_multikernel_path_matches_reference_golden(name, tmp_path):
    """The multi-kernel path (used for micrographs too large for the fused kernel's LDS)."""
    _run_case(name, tmp_path, no_fused=True)


@pytest.mark.parametrize("name", ["c1_10017", "syn_k3", "skips", "ties_getcc"])
def test_gpu_multi_batch_split(name, tmp_path):
    """Splitting the micrographs over several device batches changes nothing."""
    _run_case(name, tmp_path, batch_boxes=2000)


@pytest.mark.parametrize("name", ["c1_10017", "c1_10017_multi", "skips", "crash_nocliques",
                                  "ties_getcc"])
def test_gpu_process_writer_matches_reference_golden(name, tmp_path, monkeypatch):
    """Large runs write through spawned writer processes (chunks of micrographs): same files,
    and on a crash the outputs of every micrograph before it exist, as in the reference."""
    from repic_amd.commands import get_cliques
    monkeypatch.setattr(get_cliques, "PROC_WRITER_MIN", 1)
    _run_case(name, tmp_path, threads=4)


# ----------------------------------------------------------------------------- vs oracle
def _oracle_mg(mg, box, methods, id_base, get_cc=False):
    from oracle import cpu_ref
    coords, nid = [], id_base
    for (x, y, s) in mg:
        coords.append([(float(a), float(b), float(c), nid + i)
                       for i, (a, b, c) in enumerate(zip(x, y, s))])
        nid += len(x)
    return cpu_ref.micrograph(coords, box, methods, get_cc=get_cc)


def _canon(rows, w, conf, cons_xyid):
    perm = np.lexsort(np.asarray(rows).T[::-1]) if len(rows) else np.zeros(0, int)
    return (np.asarray(rows)[perm], np.asarray(w)[perm].view(np.uint32),
            np.asarray(conf)[perm].view(np.uint32), [cons_xyid[i] for i in perm])


def _check_vs_oracle(mgs, k, box, get_cc=False, no_fused=False):
    from repic_amd import _lib
    from repic_amd.pipeline import Batch, run_batch
    batch = Batch.pack(k, box, mgs)
    ctx = _lib.Context(0)
    res = run_batch(ctx, batch, get_cc=get_cc, no_fused=no_fused)
    methods = [f"picker{p}" for p in range(k)]
    for m, mg in enumerate(mgs):
        o = _oracle_mg(mg, box, methods, int(batch.id_base[m]), get_cc)
        r = res[m]
        assert r.status == _lib.OK
        assert (r.cc_max, r.cc_cnt) == (o["cc_max"], o["cc_cnt"])
        A = o["A"].tocoo()
        C = A.shape[1]
        orows = np.sort(A.row[np.argsort(A.col, kind="stable")].reshape(C, k), axis=1)
        assert r.n_vert == A.shape[0] and len(r.w) == C
        b0 = int(batch.box_off[m * k])
        idb = int(batch.id_base[m]) - b0
        gcons = [(float(batch.x[g]), float(batch.y[g]), idb + int(g)) for g in r.consensus]
        a = _canon(orows, o["w"], o["conf"], o["consensus"])
        b = _canon(r.rows, r.w, r.conf, gcons)
        assert np.array_equal(a[0], b[0])
        assert np.array_equal(a[1], b[1]) and np.array_equal(a[2], b[2])
        assert a[3] == b[3]
    ctx.close()


@pytest.mark.parametrize("cfg_name,n_mg,get_cc,no_fused", [
    ("C2", 24, False, False), ("C2", 8, True, False), ("C4", 6, False, False),
    ("C2", 8, False, True), ("C3", 2, False, False), ("C3", 1, True, False)])
def test_gpu_matches_oracle_synthetic(cfg_name, n_mg, get_cc, no_fused):
    from repic_amd import synth
    from repic_amd.ingest import sigmoid
    cfg = synth.SynthConfig(**synth.CONFIGS[cfg_name], seed=5, logit=(1,))
    mgs = synth.batch(cfg, n_mg)
    mgs = [[(x, y, sigmoid(s) if s.min() < 0 else s) for (x, y, s) in mg] for mg in mgs]
    _check_vs_oracle(mgs, cfg.k, cfg.box, get_cc, no_fused)


def _dense_clusters(k, per, n_clusters, seed, box=100):
    """Clusters of `per` near-duplicate boxes per picker: per**k cliques per cluster, far more
    cliques than boxes (the fused kernel's clique queue overflows -> chunked DFS re-walk)."""
    rng = np.random.default_rng(seed)
    cx = rng.uniform(0, 3000, n_clusters).round()
    cy = rng.uniform(0, 3000, n_clusters).round()
    mg = []
    for _ in range(k):
        x = np.concatenate([c + rng.integers(-3, 4, per) for c in cx]).astype(np.float64)
        y = np.concatenate([c + rng.integers(-3, 4, per) for c in cy]).astype(np.float64)
        s = rng.uniform(0.3, 1.0, len(x))
        mg.append((x, y, s))
    return mg


@pytest.mark.parametrize("k,per,n_clusters", [(3, 12, 3), (5, 4, 2), (8, 3, 1), (4, 2, 40)])
def test_gpu_dense_clusters_match_oracle(k, per, n_clusters):
    mgs = [_dense_clusters(k, per, n_clusters, seed) for seed in range(2)]
    _check_vs_oracle(mgs, k, 100)
    _check_vs_oracle(mgs, k, 100, get_cc=True)
    _check_vs_oracle(mgs, k, 100, no_fused=True)


@pytest.mark.parametrize("box,shift,frac", [(64, 0, False), (255, 0, False), (256, 0, False),
                                             (300, 0, False), (100, 0, True), (100, 18000, False),
                                             (100, -17000, False)])
def test_gpu_large_route_epilogue_paths(box, shift, frac):
    """k5_epilogue's paths on the multi-kernel route: packed-u16 clique pairs (integer
    coordinates in [-16384, 16383], integer B <= 255), one float clique at a time (B > 255,
    or a pair with a partner outside that range), f64 (fractional coordinates); odd and even
    clique counts."""
    mgs = []
    for seed in range(3):
        mg = _dense_clusters(4, 3, 9 + seed, seed, box=box)
        out = []
        for p, (x, y, s) in enumerate(mg):
            x, y = x.copy(), y.copy()
            if shift:
                x[: len(x) // 3] += shift   # some clusters out of the u16 range
            if frac and p == 1:
                x += 0.5
            out.append((x, y, s))
        mgs.append(out)
    _check_vs_oracle(mgs, 4, box, no_fused=True)
    _check_vs_oracle(mgs, 4, box, no_fused=True, get_cc=True)


def test_gpu_full_c2_properties():
    """Full BASELINE config #2 (10k micrographs): size-independent invariants."""
    from repic_amd import _lib, synth
    from repic_amd.pipeline import Batch
    cfg = synth.SynthConfig(**synth.CONFIGS["C2"], seed=0)
    batch = Batch.pack(cfg.k, cfg.box, synth.batch(cfg, 10000))
    ctx = _lib.Context(0)
    r = ctx.run(batch.n_mg, cfg.k, cfg.box, batch.box_off, batch.id_base, batch.x, batch.y,
                batch.score, _lib.F_HOST_OUTPUTS | _lib.F_MEMBERS)
    assert (r.status == 0).all()
    C = int(r.n_cliques)
    assert C == int(r.clique_cnt.sum()) and C > 10000 * 300
    # micrograph ranges tile [0, C) without overlap
    o = np.argsort(r.clique_base)
    assert (r.clique_base[o][1:] == (r.clique_base + r.clique_cnt)[o][:-1]).all()
    mem = r.members.astype(np.int64)
    # members: one box per picker, inside their micrograph (the one owning the range)
    mg_of = np.repeat(o, r.clique_cnt[o])   # ranges tile [0, C) in base order
    assert (np.searchsorted(batch.box_off[::cfg.k], mem[:, 0], side="right") - 1 == mg_of).all()
    for p in range(cfg.k):
        lo = batch.box_off[mg_of * cfg.k + p]
        hi = batch.box_off[mg_of * cfg.k + p + 1]
        assert ((mem[:, p] >= lo) & (mem[:, p] < hi)).all()
    # every pair of members overlaps with JI > 0.3 (f64, reference op order)
    B = float(cfg.box)
    for a in range(cfg.k):
        for b in range(a + 1, cfg.k):
            xa, ya, xb, yb = batch.x[mem[:, a]], batch.y[mem[:, a]], batch.x[mem[:, b]], batch.y[mem[:, b]]
            xo = np.maximum((np.minimum(xa, xb) + B) - np.maximum(xa, xb), 0.0)
            yo = np.maximum((np.minimum(ya, yb) + B) - np.maximum(ya, yb), 0.0)
            inter = xo * yo
            assert (inter / (2 * B * B - inter) > 0.3).all()
    # rows ascending and within [0, V)
    rows = r.rows
    assert (np.diff(rows, axis=1) > 0).all()
    vm = r.n_vert[mg_of]
    assert (rows[:, -1] < vm).all() and (rows[:, 0] >= 0).all()
    # cliques unique
    assert len(np.unique(mem, axis=0)) == C
    # weight = f32(f64(conf) * median JI) >= 0.3 * conf; conf is a member's score median
    assert (r.w > 0).all() and (r.w <= r.conf).all()
    ctx.close()


def _check_vs_vec(mgs, k, box, get_cc=False, no_fused=False, ctx=None):
    """Every output of the HIP path against the vectorised oracle (oracle/cpu_vec.py, pinned
    to oracle/cpu_ref.py), bit-exact, at full BASELINE sizes: clique member sets, COO rows,
    float32 w / conf, consensus box, CC stats."""
    from oracle import cpu_vec
    from repic_amd import _lib
    from repic_amd.pipeline import Batch, run_batch
    batch = Batch.pack(k, box, mgs)
    own = ctx is None
    if own:
        ctx = _lib.Context(0)
    res = run_batch(ctx, batch, get_cc=get_cc, no_fused=no_fused, members=True)
    # without members in the outputs (what the CLI and the bench ask for) the large route
    # derives each clique's members inside its epilogue (k5_leaf_epi): the same outputs,
    # compared in the canonical order of the rows (a clique's sorted vertex ranks)
    res_nm = run_batch(ctx, batch, get_cc=get_cc, no_fused=no_fused, members=False)
    n_cl = 0
    for m, mg in enumerate(mgs):
        b0 = int(batch.box_off[m * k])
        x, y, s = (np.concatenate([t[i] for t in mg]) for i in range(3))
        o = cpu_vec.micrograph(x, y, s, [len(t[0]) for t in mg], box, get_cc=get_cc,
                               id_base=int(batch.id_base[m]))
        r = res[m]
        assert o["status"] == "ok" and r.status == _lib.OK
        assert (r.cc_max, r.cc_cnt) == (o["cc_max"], o["cc_cnt"])
        assert r.n_edges == o["n_edges"] and r.n_vert == o["V"]
        mem = r.members.astype(np.int64) - b0
        assert mem.shape == o["members"].shape, (mem.shape, o["members"].shape)
        p = np.lexsort(mem.T[::-1])      # oracle members are already lexicographic
        assert np.array_equal(mem[p], o["members"])
        assert np.array_equal(r.rows[p], o["rows"])
        assert np.array_equal(r.w[p].view(np.uint32), o["w"].view(np.uint32))
        assert np.array_equal(r.conf[p].view(np.uint32), o["conf"].view(np.uint32))
        assert np.array_equal(r.consensus[p].astype(np.int64) - b0, o["consensus"])
        q = res_nm[m]
        assert q.members is None and len(q.w) == len(p)
        po = np.lexsort(o["rows"].T[::-1])
        pq = np.lexsort(q.rows.T[::-1])
        assert np.array_equal(q.rows[pq], o["rows"][po])
        assert np.array_equal(q.w[pq].view(np.uint32), o["w"][po].view(np.uint32))
        assert np.array_equal(q.conf[pq].view(np.uint32), o["conf"][po].view(np.uint32))
        assert np.array_equal(q.consensus[pq].astype(np.int64) - b0, o["consensus"][po])
        assert (q.status, q.cc_max, q.cc_cnt, q.n_vert) == (r.status, r.cc_max, r.cc_cnt, r.n_vert)
        n_cl += len(p)
    if own:
        ctx.close()
    return n_cl


def _c5_window(mg, x0, y0, W):
    out = []
    for (x, y, s) in mg:
        m = (x >= x0) & (x < x0 + W) & (y >= y0) & (y < y0 + W)
        out.append((x[m], y[m], s[m]))
    return out


def test_gpu_c5_full_size_matches_vectorised_oracle():
    """BASELINE config #5 (8 pickers, ~27.5k boxes and ~1M 8-cliques per micrograph, B = 64):
    two full-size micrographs through the large-micrograph route, every output bit-exact
    against the vectorised oracle (get_cliques.py:49-56,160-202 clique explosion)."""
    from repic_amd import synth
    cfg = synth.SynthConfig(**synth.CONFIGS["C5"], seed=0)
    mgs = synth.batch(cfg, 2)
    assert sum(len(t[0]) for t in mgs[0]) > 25000
    n = _check_vs_vec(mgs, cfg.k, cfg.box)
    assert n > 1_000_000


def test_gpu_c5_windows_match_reference_oracle():
    """C5 windows small enough for the scalar oracle (pinned to the reference's goldens):
    768^2 px (~1k boxes, ~7k cliques) and 1024^2 px (~1.8k boxes, ~39k cliques), on the
    fused route and on the large-micrograph route."""
    from repic_amd import synth
    cfg = synth.SynthConfig(**synth.CONFIGS["C5"], seed=0)
    base = synth.batch(cfg, 2)
    wins = [_c5_window(base[0], 1000, 1000, 768), _c5_window(base[1], 2500, 300, 768),
            _c5_window(base[0], 1000, 1000, 1024)]
    _check_vs_oracle(wins, cfg.k, cfg.box)
    _check_vs_oracle(wins[:2], cfg.k, cfg.box, no_fused=True)


@pytest.mark.parametrize("cfg_name,n_mg,get_cc", [("C3", 16, False), ("C3", 4, True),
                                                   ("C4", 200, False), ("C2", 400, False)])
def test_gpu_full_size_configs_match_vectorised_oracle(cfg_name, n_mg, get_cc):
    """Full-size C2/C3/C4 micrographs (same generator and seed as bench.py), bit-exact."""
    from repic_amd import synth
    cfg = synth.SynthConfig(**synth.CONFIGS[cfg_name], seed=0)
    _check_vs_vec(synth.batch(cfg, n_mg), cfg.k, cfg.box, get_cc=get_cc)


def test_gpu_mixed_batch_routes():
    """One batch whose micrographs take every route: f32-layout fused pass, f64 relaunch
    (coordinates not exact in f32), large-LDS relaunch (dense clusters), BFS overflow into
    the DFS re-walk, and the multi-kernel path (more boxes than the fused kernel's LDS)."""
    from repic_amd import synth
    cfg = synth.SynthConfig(**synth.CONFIGS["C2"], seed=11)
    base = synth.batch(cfg, 6)
    mgs = [base[0], base[1]]
    # non-f32-exact coordinates
    mgs.append([(x + 0.001, y - 0.0005, s) for (x, y, s) in base[2]])
    # dense near-duplicate clusters (many more cliques than boxes)
    mgs.append(_dense_clusters(3, 10, 4, seed=7))
    mgs.append(base[3])
    # a large micrograph: too many boxes for the fused kernel
    big = synth.SynthConfig(k=3, n_true=1500, box=60, width=4096, height=4096, keep=0.9,
                            jit=0.08, fp=0.1, seed=12)
    mgs.append(synth.batch(big, 1)[0])
    mgs.append(base[4])
    _check_vs_oracle(mgs, 3, 100)
    _check_vs_oracle(mgs, 3, 100, get_cc=True)


def test_gpu_device_resident_inputs_and_offsets():
    """F_DEVICE_INPUTS + F_DEVICE_META (the bench's HBM-resident handoff: coordinates, scores,
    box offsets and id bases already on the device) give the same outputs as host inputs, on
    a batch that takes every route (fused f32/f64, multi-kernel gather of the big micrograph).
    Runs in a child process: torch's bundled HIP runtime must initialise before the library's
    (as in bench.py), and this test process already created library contexts."""
    import subprocess
    import sys
    here = os.path.dirname(os.path.abspath(__file__))
    root = os.path.dirname(here)
    env = dict(os.environ, PYTHONPATH=os.pathsep.join(
        [root, os.path.join(root, "repic-copy_amd"), here, os.environ.get("PYTHONPATH", "")]))
    r = subprocess.run([sys.executable, "-c",
                        "import test_gpu_parity as t; t._device_meta_check(); print('OK')"],
                       env=env, capture_output=True, text=True, timeout=110)
    assert r.returncode == 0 and r.stdout.strip().endswith("OK"), r.stdout + r.stderr


@pytest.mark.parametrize("streams", [1, 2])
def test_gpu_submit_wait_pipelined_contexts(streams):
    """rgc_submit / rgc_wait (ABI 3) on two contexts sharing one stream, or on a stream each
    (bench.py's default: consecutive steps' launches overlap), the bench's pipelined steps:
    every batch's outputs equal rgc_run's.  Batches cover the single-launch fast path, a
    micrograph that needs the f64 pass (the fast path falls back at rgc_wait) and a batch with
    a large micrograph (general path at rgc_submit).  Child process as above."""
    import subprocess
    import sys
    here = os.path.dirname(os.path.abspath(__file__))
    root = os.path.dirname(here)
    env = dict(os.environ, PYTHONPATH=os.pathsep.join(
        [root, os.path.join(root, "repic-copy_amd"), here, os.environ.get("PYTHONPATH", "")]))
    r = subprocess.run([sys.executable, "-c",
                        f"import test_gpu_parity as t; t._submit_wait_check({streams}); "
                        "print('OK')"],
                       env=env, capture_output=True, text=True, timeout=110)
    assert r.returncode == 0 and r.stdout.strip().endswith("OK"), r.stdout + r.stderr


def _d2h(ptr, n, dtype):
    """copy n elements of a device array to numpy (HIP runtime through ctypes)"""
    import ctypes
    hip = ctypes.CDLL("libamdhip64.so")
    out = np.empty(n, dtype=dtype)
    if n:
        rc = hip.hipMemcpy(ctypes.c_void_p(out.ctypes.data), ctypes.c_void_p(int(ptr)),
                           ctypes.c_size_t(out.nbytes), ctypes.c_int(2))
        assert rc == 0, rc
    return out


def _submit_wait_check(streams=1):
    import torch
    torch.cuda.init()

    from repic_amd import _lib, synth
    from repic_amd.pipeline import Batch
    cfg = synth.SynthConfig(**synth.CONFIGS["C2"], seed=21)
    b1 = Batch.pack(3, 180, synth.batch(cfg, 300))
    m2 = synth.batch(cfg, 40, start=300)
    m2[7] = [(x + 0.25, y, s) for (x, y, s) in m2[7]]          # f64 pass: wait falls back
    b2 = Batch.pack(3, 180, m2)
    big = synth.SynthConfig(k=3, n_true=1800, box=60, width=4096, height=4096, keep=0.9,
                            jit=0.08, fp=0.1, seed=22)
    b3 = Batch.pack(3, 180, synth.batch(cfg, 20, start=400) + synth.batch(big, 1))
    dev = torch.device("cuda", 0)
    fl = _lib.F_MEMBERS | _lib.F_GET_CC
    per_mg = ("status", "cc_max", "cc_cnt", "n_vert", "clique_cnt")
    per_cl = (("rows", np.int32, 3), ("w", np.float32, 1), ("conf", np.float32, 1),
              ("consensus", np.int32, 1), ("members", np.int32, 3))

    def snap(r, on_dev):
        d = {f: np.array(getattr(r, f)) for f in per_mg}
        C = int(r.n_cliques)
        # batch totals (the fast path sums the edges after the launch, k_fused_ties)
        d["tot"] = (int(r.n_edges), C, int(np.asarray(r.n_edges_mg).sum()))
        for f, dt, w in per_cl:
            v = getattr(r, f)
            v = _d2h(v, C * w, dt) if on_dev else np.asarray(v).reshape(-1)
            v = v.reshape(C, w) if w > 1 else v
            d[f] = [v[int(b0):int(b0) + int(n)].copy() for b0, n in zip(r.clique_base, r.clique_cnt)]
        return d

    ref_ctx = _lib.Context(0)
    refs, dev_in = [], []
    for b in (b1, b2, b3):
        refs.append(snap(ref_ctx.run(b.n_mg, 3, 180, b.box_off, b.id_base, b.x, b.y, b.score,
                                     fl | _lib.F_HOST_OUTPUTS), False))
        t = [torch.from_numpy(np.ascontiguousarray(v)).to(dev) for v in (b.x, b.y, b.score)]
        t.append(torch.from_numpy(b.box_off.astype(np.int32)).to(dev))
        t.append(torch.from_numpy(np.ascontiguousarray(b.id_base, dtype=np.int64)).to(dev))
        dev_in.append(t)
    torch.cuda.synchronize()
    stream = torch.cuda.current_stream(dev).cuda_stream
    s2 = torch.cuda.Stream(dev) if streams == 2 else None
    ctxs = [_lib.Context(0, stream), _lib.Context(0, s2.cuda_stream if s2 else stream)]

    def submit(c, i, lazy=False):
        # lazy: ABI 6 F_LAZY_STATS (the bench's steps): per-micrograph outputs fetched from HBM
        # when the Result first reads them
        b, t = (b1, b2, b3)[i], dev_in[i]
        c.submit(b.n_mg, 3, 180, b.box_off, b.id_base, t[0].data_ptr(), t[1].data_ptr(),
                 t[2].data_ptr(), fl | _lib.F_DEVICE_INPUTS | _lib.F_TIMING |
                 (_lib.F_LAZY_STATS if lazy else 0),
                 dev_meta=(t[3].data_ptr(), t[4].data_ptr()))

    # one run in flight per context: wait() with nothing pending raises, and while a submit is
    # pending, run / submit on the same context are refused (its buffers are in use)
    try:
        ctxs[0].wait()
        raise AssertionError("wait() without a submission did not raise")
    except _lib.RGCError:
        pass
    submit(ctxs[0], 0)
    for call in (lambda: submit(ctxs[0], 1),
                 lambda: ctxs[0].run(b1.n_mg, 3, 180, b1.box_off, b1.id_base, b1.x, b1.y,
                                     b1.score, fl | _lib.F_HOST_OUTPUTS)):
        try:
            call()
            raise AssertionError("call on a busy context did not raise")
        except _lib.RGCError as e:
            assert "awaits rgc_wait" in str(e)
    ctxs[0].wait()

    order = [0, 1, 2, 0, 2, 1, 0, 1, 0]
    submit(ctxs[0], order[0])
    for j, i in enumerate(order):
        if j + 1 < len(order):
            submit(ctxs[(j + 1) % 2], order[j + 1], lazy=j + 1 >= 6)
        got = snap(ctxs[j % 2].wait(), True)
        for f in per_mg:
            np.testing.assert_array_equal(got[f], refs[i][f], err_msg=f"{f} batch {i}")
        assert got["tot"] == refs[i]["tot"], (got["tot"], refs[i]["tot"])
        for f, _, _ in per_cl:
            for a, e in zip(got[f], refs[i][f]):
                np.testing.assert_array_equal(a.view(np.uint8), e.view(np.uint8), err_msg=f)
        assert any(n == "k_fused" for n, _ in ctxs[j % 2].kernel_times())
    for c in ctxs + [ref_ctx]:
        c.close()


def _device_meta_check():
    import torch
    torch.cuda.init()   # torch's HIP runtime first (bench.py order)

    from repic_amd import _lib, synth
    from repic_amd.pipeline import Batch
    cfg = synth.SynthConfig(**synth.CONFIGS["C2"], seed=13)
    base = synth.batch(cfg, 4)
    big = synth.SynthConfig(k=3, n_true=1500, box=60, width=4096, height=4096, keep=0.9,
                            jit=0.08, fp=0.1, seed=14)
    mgs = [base[0], [(x + 0.001, y, s) for (x, y, s) in base[1]], _dense_clusters(3, 10, 4, 9),
           synth.batch(big, 1)[0], base[2], base[3]]
    batch = Batch.pack(3, 100, mgs)
    fl = _lib.F_HOST_OUTPUTS | _lib.F_MEMBERS
    ctx = _lib.Context(0)
    a = ctx.run(batch.n_mg, 3, 100, batch.box_off, batch.id_base, batch.x, batch.y,
                batch.score, fl)
    per_mg = ("status", "cc_max", "cc_cnt", "n_vert", "clique_cnt")
    per_cl = ("rows", "w", "conf", "consensus", "members")

    def snap(r):
        # micrograph ranges are reserved atomically (their order varies); content per range
        # is deterministic
        d = {f: np.array(getattr(r, f)) for f in per_mg}
        for f in per_cl:
            v = np.asarray(getattr(r, f))
            d[f] = [v[int(b0):int(b0) + int(n)].copy()
                    for b0, n in zip(r.clique_base, r.clique_cnt)]
        return d

    ref = snap(a)
    dev = torch.device("cuda", 0)
    dx, dy, ds = (torch.from_numpy(np.ascontiguousarray(v)).to(dev)
                  for v in (batch.x, batch.y, batch.score))
    dbo = torch.from_numpy(batch.box_off.astype(np.int32)).to(dev)
    did = torch.from_numpy(np.ascontiguousarray(batch.id_base, dtype=np.int64)).to(dev)
    torch.cuda.synchronize()
    b = ctx.run(batch.n_mg, 3, 100, batch.box_off, batch.id_base, dx.data_ptr(),
                dy.data_ptr(), ds.data_ptr(), fl | _lib.F_DEVICE_INPUTS,
                dev_meta=(dbo.data_ptr(), did.data_ptr()))
    assert (a.n_edges, a.n_cliques) == (b.n_edges, b.n_cliques)
    got = snap(b)
    for f in per_mg:
        assert np.array_equal(ref[f], got[f]), f
    for f in per_cl:
        assert all(np.array_equal(u, v) for u, v in zip(ref[f], got[f])), f
    assert sum(len(v) for v in got["w"]) == int(b.n_cliques)
    ctx.close()


def test_gpu_cli_end_to_end_subprocess(tmp_path):
    """`python -m repic_amd.main get_cliques <in> <out> 180` as a separate process (argparse,
    dispatcher, exit status) on EMPIAR-10017 reproduces the reference's golden outputs."""
    import json
    import subprocess
    import sys
    name = "c1_10017"
    meta, data = load_case(name)
    in_dir = make_inputs(name, str(tmp_path))
    out_dir = os.path.join(str(tmp_path), "out")
    lst = os.path.join(str(tmp_path), "listing.json")
    with open(lst, "w") as f:
        json.dump(meta["listing"], f)
    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    env = dict(os.environ, PYTHONPATH=os.pathsep.join([os.path.join(root, "repic-copy_amd"),
                                                       os.environ.get("PYTHONPATH", "")]))
    r = subprocess.run([sys.executable, "-m", "repic_amd.main", "get_cliques", in_dir, out_dir,
                        str(meta["box"]), "--listing", lst], env=env, capture_output=True,
                       text=True, timeout=300)
    assert r.returncode == 0, r.stderr[-3000:]
    assert "Using crYOLO BOX files as starting point" in r.stdout
    mgs, arrays = read_outputs(out_dir, meta)
    assert_matches_golden(meta, data, mgs, arrays)
    # a crash case exits non-zero with the reference's exception class
    meta2, _ = load_case("crash_noedges")
    in2 = make_inputs("crash_noedges", str(tmp_path / "c2"))
    r = subprocess.run([sys.executable, "-m", "repic_amd.main", "get_cliques", in2,
                        os.path.join(str(tmp_path), "out2"), str(meta2["box"])], env=env,
                       capture_output=True, text=True, timeout=300)
    assert r.returncode != 0 and "ValueError" in r.stderr


def test_gpu_result_views_outlive_next_run_and_close():
    """Result arrays are views of pinned host memory the context owns; a Result still
    referenced when the context moves on keeps its buffers (rgc_detach_host, ABI 7): a
    coo_matrix built from ``r.rows`` reads the same values after a second, larger run (which
    grows and would otherwise free or overwrite those buffers) and after ``close()``.  The
    r04e segfault was this read after close (reference get_cliques.py:192-202 builds the COO
    from the same rows)."""
    from scipy.sparse import coo_matrix

    from repic_amd import _lib, synth
    from repic_amd.pipeline import Batch
    cfg = synth.SynthConfig(**synth.CONFIGS["C2"], seed=3)
    small = Batch.pack(cfg.k, cfg.box, synth.batch(cfg, 4))
    big = Batch.pack(cfg.k, cfg.box, synth.batch(cfg, 400, start=4))
    ctx = _lib.Context(0)
    r = ctx.run(small.n_mg, cfg.k, cfg.box, small.box_off, small.id_base, small.x, small.y,
                small.score, _lib.F_HOST_OUTPUTS)
    C, V0 = int(r.clique_cnt[0]), int(r.n_vert[0])
    b0 = int(r.clique_base[0])
    rows = r.rows[b0:b0 + C].reshape(-1)
    A = coo_matrix((np.ones(C * cfg.k, np.int64), (rows, np.repeat(np.arange(C), cfg.k))),
                   shape=(V0, C))
    want_rows, want_w, want_st = rows.copy(), r.w.copy(), r.status.copy()
    r2 = ctx.run(big.n_mg, cfg.k, cfg.box, big.box_off, big.id_base, big.x, big.y, big.score,
                 _lib.F_HOST_OUTPUTS)
    assert int(r2.n_cliques) > 50 * int(r.n_cliques)       # the host buffers had to grow
    assert (r.rows[b0:b0 + C].reshape(-1) == want_rows).all() and (r.w == want_w).all()
    del r2
    ctx.close()
    assert (A.row == want_rows).all() and (A.tocsc().indices.size == C * cfg.k)
    assert (r.status == want_st).all() and (r.w == want_w).all()
    assert (A.toarray().sum(axis=0) == cfg.k).all()


def test_gpu_lazy_stats_result_survives_next_submit():
    """F_LAZY_STATS: a Result whose per-micrograph block was not fetched yet, still referenced
    at the next submit on its context, gets its own run's stats (fetched at the hand-over),
    not the newer run's (stale lazy stats).  Child process as above (torch's HIP
    runtime first)."""
    import subprocess
    import sys
    here = os.path.dirname(os.path.abspath(__file__))
    root = os.path.dirname(here)
    env = dict(os.environ, PYTHONPATH=os.pathsep.join(
        [root, os.path.join(root, "repic-copy_amd"), here, os.environ.get("PYTHONPATH", "")]))
    r = subprocess.run([sys.executable, "-c",
                        "import test_gpu_parity as t; t._lazy_survive_check(); print('OK')"],
                       env=env, capture_output=True, text=True, timeout=110)
    assert r.returncode == 0 and r.stdout.strip().endswith("OK"), r.stdout + r.stderr


def _lazy_survive_check():
    import torch
    torch.cuda.init()

    from repic_amd import _lib, synth
    from repic_amd.pipeline import Batch
    cfg = synth.SynthConfig(**synth.CONFIGS["C2"], seed=5)
    a = Batch.pack(cfg.k, cfg.box, synth.batch(cfg, 6))
    b = Batch.pack(cfg.k, cfg.box, synth.batch(cfg, 9, start=6))
    dev = []
    for bt in (a, b):
        dev.append([torch.from_numpy(v).cuda() for v in (bt.x, bt.y, bt.score)] +
                   [torch.from_numpy(bt.box_off.astype(np.int32)).cuda(),
                    torch.from_numpy(bt.id_base.astype(np.int64)).cuda()])
    torch.cuda.synchronize()
    stream = torch.cuda.Stream()
    ctx = _lib.Context(0, stream.cuda_stream)
    ref = ctx.run(a.n_mg, cfg.k, cfg.box, a.box_off, a.id_base, a.x, a.y, a.score, 0)
    want = ref.clique_cnt.copy()
    del ref

    def sub(bt, d):
        ctx.submit(bt.n_mg, cfg.k, cfg.box, bt.box_off, bt.id_base, d[0].data_ptr(),
                   d[1].data_ptr(), d[2].data_ptr(), _lib.F_DEVICE_INPUTS | _lib.F_LAZY_STATS,
                   dev_meta=(d[3].data_ptr(), d[4].data_ptr()))
    sub(a, dev[0])
    ra = ctx.wait()
    sub(b, dev[1])
    rb = ctx.wait()
    assert len(ra.clique_cnt) == a.n_mg and (ra.clique_cnt == want).all(), (ra.clique_cnt, want)
    assert len(rb.clique_cnt) == b.n_mg and (rb.clique_cnt > 0).all()
    ctx.close()


def test_gpu_submit_worker_error_and_reuse():
    """A batch on rgc_submit's general path runs on the context's worker thread: its error
    (box_size above 2^26) comes back from rgc_wait with the worker's message, and the context
    then runs further submissions (general path: a micrograph too large for the fused kernel)
    with outputs equal to rgc_run's."""
    from repic_amd import _lib, synth
    from repic_amd.pipeline import Batch
    cfg = synth.SynthConfig(**synth.CONFIGS["C2"], seed=31)
    big = synth.SynthConfig(k=3, n_true=1800, box=60, width=4096, height=4096, keep=0.9,
                            jit=0.08, fp=0.1, seed=32)
    b = Batch.pack(3, 180, synth.batch(cfg, 5) + synth.batch(big, 1))
    fl = _lib.F_HOST_OUTPUTS | _lib.F_MEMBERS
    ctx = _lib.Context(0)
    try:
        ctx.submit(b.n_mg, 3, 1 << 27, b.box_off, b.id_base, b.x, b.y, b.score, fl)
        with pytest.raises(_lib.RGCError, match="box_size"):
            ctx.wait()
        def snap(r):
            # micrograph ranges are reserved atomically (their order varies); the content of
            # each range is deterministic
            d = {f: np.array(getattr(r, f)) for f in ("status", "clique_cnt")}
            for f in ("rows", "w", "conf", "consensus", "members"):
                v = np.asarray(getattr(r, f))
                d[f] = [v[int(b0):int(b0) + int(n)].copy()
                        for b0, n in zip(r.clique_base, r.clique_cnt)]
            return d

        want = snap(ctx.run(b.n_mg, 3, 180, b.box_off, b.id_base, b.x, b.y, b.score, fl))
        for _ in range(2):
            ctx.submit(b.n_mg, 3, 180, b.box_off, b.id_base, b.x, b.y, b.score, fl)
            got = snap(ctx.wait())
            for f, v in want.items():
                if isinstance(v, list):
                    assert len(got[f]) == len(v)
                    for a, e in zip(got[f], v):
                        np.testing.assert_array_equal(a, e, err_msg=f)
                else:
                    np.testing.assert_array_equal(got[f], v, err_msg=f)
    finally:
        ctx.close()
