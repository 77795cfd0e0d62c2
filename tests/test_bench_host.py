"""CPU tests of bench.py's host-side reporting: the roofline limiter / measured HBM fraction
derived from a PMC record, and the C5 sampled CPU baseline."""
import os
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

import bench  # noqa: E402


def test_roofline_evidence_from_counters():
    rec = {"kernels": {"k_fused": {"traffic": 346e6, "derived": {
        "valu_busy": 0.867, "wait_any": 0.541, "waves_per_cu": 26.0, "lane_eff": 0.62}}}}
    traffic, hbm, lim = bench.roofline_evidence(rec, "k_fused", 995e6, 0.54)
    assert traffic == 346e6
    assert hbm == pytest.approx(346e6 / 0.54e-3 / 8e12)
    assert lim.startswith("VALU issue:")
    for frag in ("0.35x B_alg", "VALU busy 87%", "stalled 54%", "lane efficiency 62%"):
        assert frag in lim, (frag, lim)
    # an HBM-saturating kernel is labelled as such
    rec2 = {"kernels": {"k_fused": {"traffic": 4.4e9, "derived": {"valu_busy": 0.3}}}}
    assert bench.roofline_evidence(rec2, "k_fused", 4e9, 1.0)[2].startswith("HBM bandwidth")
    # multi-kernel route: per-step traffic over the route's device time
    rec3 = {"step_traffic": 2e9, "kernels": {}}
    t, h, lim3 = bench.roofline_evidence(rec3, "route", 8e9, 8.0)
    assert t == 2e9 and h == pytest.approx(2e9 / 8e-3 / 8e12)
    # no matching file: said so, no numbers
    t, h, lim4 = bench.roofline_evidence(None, "k_fused", 1.0, 1.0)
    assert t is None and h is None and "unmeasured" in lim4


def test_c5_cpu_baseline_is_sampled_and_bounded():
    sys.path.insert(0, os.path.join(ROOT, "repic-copy_amd"))
    import time

    from repic_amd import synth
    cfg = synth.SynthConfig(**synth.CONFIGS["C5"], seed=0)
    mgs = synth.batch(cfg, 1)
    t0 = time.perf_counter()
    cb = bench.cpu_baseline(cfg, mgs, budget_s=1.5, procs=1, config="C5")
    assert time.perf_counter() - t0 < 10
    assert cb["cores"] == 1 and cb["kind"] == "port" and 0 < cb["value"] < 0.1
    assert "extrapolated" in cb["sample"] and "upper bound" in cb["sample"]


def test_roofline_bound_follows_the_counters():
    """roofline.bound is derived from the same counters as the limiter, never a literal."""
    valu = {"kernels": {"k_fused": {"traffic": 243e6, "derived": {"valu_busy": 0.9}}}}
    assert bench.derived_bound(valu, "k_fused", 995e6, 0.48) == "valu"
    lat = {"kernels": {"k_fused": {"traffic": 2.4e9, "derived": {"valu_busy": 0.54}}}}
    assert bench.derived_bound(lat, "k_fused", 7.5e9, 3.4) == "latency"
    hbm = {"kernels": {"k_fused": {"traffic": 4.4e9, "derived": {"valu_busy": 0.3}}}}
    assert bench.derived_bound(hbm, "k_fused", 4e9, 1.0) == "hbm"
    assert bench.derived_bound(None, "k_fused", 1.0, 1.0) == "unmeasured"
    assert bench.derived_bound({"step_traffic": 2e9}, "route", 8e9, 8.0, "k5l") == "unmeasured"
    route = {"step_traffic": 2e9, "kernels": {"k5_epilogue": {"derived": {"valu_busy": 0.7}}}}
    assert bench.derived_bound(route, "route", 8e9, 8.0, "k5_epilogue") == "valu"


class _StubCtx:
    """submit / wait bookkeeping of one library context (one run in flight, as rgc_submit)"""

    def __init__(self, name, log):
        self.name, self.log, self.pending = name, log, None

    def submit(self, step, timed):
        assert self.pending is None, "submit on a context with a run in flight"
        self.pending = (step, timed)
        self.log.append(("submit", self.name, step))

    def wait(self):
        assert self.pending is not None, "wait without a submission"
        step, timed = self.pending
        self.pending = None
        self.log.append(("wait", self.name, step))
        return ("result", step)

    def kernel_times(self):
        return [("k_fused", 1.0)] if self.pending is None else []


@pytest.mark.parametrize("depth,n", [(1, 5), (2, 7), (3, 7), (3, 2), (2, 1)])
def test_pipelined_steps_order_and_depth(depth, n):
    """bench.pipelined_steps: steps in order, at most ``depth`` in flight, each context waited
    for before it is reused, the last step's result returned, timing on every TIME_EVERY-th."""
    log = []
    ctxs = [_StubCtx(f"c{j}", log) for j in range(depth)]
    count = iter(range(10 ** 6))

    def submit(c, timed):
        c.submit(next(count), timed)

    kt = {}
    r = bench.pipelined_steps(ctxs, submit, n, True, kt)
    assert r == ("result", n - 1)
    subs = [e for e in log if e[0] == "submit"]
    waits = [e for e in log if e[0] == "wait"]
    assert [e[2] for e in subs] == list(range(n)) and [e[2] for e in waits] == list(range(n))
    assert all(e[1] == f"c{e[2] % depth}" for e in subs + waits)
    in_flight = 0
    for e in log:
        in_flight += 1 if e[0] == "submit" else -1
        assert 0 <= in_flight <= depth
    assert in_flight == 0
    assert kt.get("__steps", 0) == len(range(0, n, bench.TIME_EVERY))


@pytest.mark.parametrize("total,world", [(100000, 1), (100000, 2), (100000, 3), (100000, 8),
                                         (7, 8), (12, 5)])
def test_fixed_shard_splits_one_batch(total, world):
    """C4_100k_fixed (strong scaling): the ranks' shares of the fixed batch are contiguous,
    cover it exactly once and differ by at most one micrograph."""
    shares = [bench.fixed_shard(total, world, r) for r in range(world)]
    assert shares[0][0] == 0
    for (s0, n0), (s1, _) in zip(shares, shares[1:]):
        assert s0 + n0 == s1
    assert sum(n for _, n in shares) == total
    assert max(n for _, n in shares) - min(n for _, n in shares) <= 1


def test_stream_plan_fits_the_hardware_queues():
    """bench.py's streams fit GPU_MAX_HW_QUEUES (4): the default depth's launch streams plus
    the null stream (which also carries the non-lazy stats copies), no separate copy stream."""
    plan = bench.stream_plan(bench.PIPE_DEPTH_DEFAULT)
    assert plan["total"] <= bench.HW_QUEUES == 4
    assert plan["copy_streams"] == 0 and plan["launch_streams"] == bench.PIPE_DEPTH_DEFAULT
    with pytest.raises(AssertionError):
        bench.stream_plan(bench.HW_QUEUES)


def test_pmc_record_is_keyed_by_entry(tmp_path, monkeypatch):
    """Counters are looked up by by_config ENTRY: a record taken at C4's bench size (no
    "entry" key) stands for C4, never for C4_100k or C4_100k_fixed (other batch sizes)."""
    import hashlib
    import json
    lib = tmp_path / "lib.so"
    lib.write_bytes(b"x")
    sha = hashlib.sha256(b"x").hexdigest()
    prof = tmp_path / "profiles"
    prof.mkdir()
    (prof / "a_c4_traffic.json").write_text(json.dumps({"lib_sha256": sha, "config": "C4"}))
    (prof / "b_c4_100k_traffic.json").write_text(json.dumps(
        {"lib_sha256": sha, "config": "C4", "entry": "C4_100k"}))
    (prof / "c_c2_traffic.json").write_text(json.dumps({"lib_sha256": sha}))
    sys.path.insert(0, os.path.join(ROOT, "repic-copy_amd"))
    from repic_amd import _lib
    monkeypatch.setattr(_lib, "LIB_PATH", str(lib))
    monkeypatch.setattr(bench, "ROOT", str(tmp_path))
    assert bench.pmc_record("C4")[1] == "a_c4_traffic.json"
    assert bench.pmc_record("C4_100k")[1] == "b_c4_100k_traffic.json"
    assert bench.pmc_record("C4_100k_fixed") == (None, None)
    assert bench.pmc_record("C2")[1] == "c_c2_traffic.json"
    assert bench.pmc_record("C5_256") == (None, None)
