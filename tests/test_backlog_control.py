"""The burst planner's backlog control is a bounded state (plugins.gpu.planner.observe_time):
measured feedback sets each GPU's relative speed (a window median of measured / predicted
ratios), speeds scale the carried predicted increments, and the relative backlog is clipped --
so one outlier is absorbed, a persistently slow GPU converges to a steady smaller share, and
no GPU with free units ever receives zero pods of a burst because of carried backlog.

This is the CPU counterpart of the hardware direction test
(tests/test_gpu_native.py::test_planner_feedback_moves_work_off_a_really_slower_gpu, which
failed on the round-4 driver box with an undamped integrator, GPUTEST_r04.json)."""
import numpy as np
import pytest

from k8s_gpu_scheduler_amd import _native
from k8s_gpu_scheduler_amd.models import workloads as W
from k8s_gpu_scheduler_amd.parallel import podbench as PB

has_core = _native.core() is not None
pytestmark = pytest.mark.skipif(not has_core, reason="_core not built")


def _run(epochs: int, slow=(1.0, 1.0), outlier=None, seed: int = 5, noise: float = 0.03):
    """2-GPU control plane (2 pods per GPU per burst: the planner may put 0-4 pods on a GPU),
    each GPU's group "runs" for its co-run model duration x slow[g] x (1 +- noise); outlier =
    (epoch, gpu, extra ms) added to one measured busy time.  Returns per-epoch (pods per GPU,
    GPU 1 work share, backlog spread, plan-visible spread)."""
    cp = PB.ControlPlane(n_gpus=2, pods_per_gpu=2, iters=20, seed=seed, balance=1.0, plan_bursts=True,
                         plan_tolerance=0.3, slo_objective="corun", corun_sigma=0.05, plan_carry=1.0)
    planner = cp.plugin.planner
    model = cp.corun.base
    rng = np.random.default_rng(seed)
    keys = [(PB.NODE, 0), (PB.NODE, 1)]
    out = []
    for e in range(epochs):
        cp.finish_live()
        arr = cp.schedule_epoch()
        runs = {g: PB._runs_for(arr, g) for g in (0, 1)}
        work = {g: sum(model.alone_ms[model.wid(r.workload)] * r.iters for r in runs[g]) for g in (0, 1)}
        pods = np.full((2, PB.POD_F * PB.MAX_PODS_GPU), -1.0)
        for g in (0, 1):
            rs = runs[g]
            if not rs:
                continue
            d = model.group_durations([model.wid(r.workload) for r in rs], [r.iters for r in rs])
            d = np.asarray(d) * slow[g] * (1.0 + noise * rng.uniform(-1, 1, len(rs)))
            if outlier is not None and outlier[0] == e and outlier[1] == g:
                d = d + outlier[2]
            for i, (r, ms) in enumerate(zip(rs, d)):
                pods[g, i * PB.POD_F:(i + 1) * PB.POD_F] = [W.INDEX[r.workload], r.iters / (ms / 1e3), -1, -1, -1]
        cp._plan_feedback(pods)
        bl = [planner.backlog.get(k, 0.0) for k in keys]
        base = planner.plan_base(keys)
        out.append(((len(runs[0]), len(runs[1])), work[1] / max(work[0] + work[1], 1e-9),
                    max(bl) - min(bl), float(base.max() - base.min())))
    return out, planner


def test_single_outlier_is_absorbed_without_a_zero_pod_burst():
    base, _ = _run(24)
    hit, planner = _run(24, outlier=(10, 1, 50.0))
    assert all(min(n) > 0 for n, _, _, _ in hit), [n for n, *_ in hit]
    # a +50 ms outlier (~10 bursts of work) on one epoch: the window median ignores it, so
    # within 3 bursts the plans are back to the undisturbed run's
    assert [n for n, *_ in hit[14:]] == [n for n, *_ in base[14:]]
    assert max(s for *_, s in hit) <= planner.SPREAD_CLIP * planner._burst_ms * 1.5 + 1e-6


def test_persistent_slowdown_converges_to_a_steady_share():
    res, planner = _run(200, slow=(1.0, 1.1))
    assert all(min(n) > 0 for n, _, _, _ in res)
    share = np.array([s for _, s, _, _ in res])
    spread = np.array([b for _, _, b, _ in res])
    # bounded state: the stored relative backlog never exceeds its clip
    assert spread.max() <= planner.STORE_CLIP * planner._burst_ms * 1.5 + 1e-6, spread.max()
    # steady: the slow GPU's mean share over the last 100 bursts is below half and the two
    # 50-burst halves agree (no drift, no divergence)
    a, b = share[100:150].mean(), share[150:].mean()
    assert share[100:].mean() < 0.49, share[100:].mean()
    assert abs(a - b) < 0.03, (a, b)
    assert planner.rel_speeds([(PB.NODE, 0), (PB.NODE, 1)])[1] > 1.03


def test_uniform_slowdown_changes_no_plan():
    base, _ = _run(30)
    slow, _ = _run(30, slow=(1.15, 1.15))
    assert [n for n, *_ in slow] == [n for n, *_ in base]


def test_speed_is_a_clipped_window_median():
    from k8s_gpu_scheduler_amd.plugins.gpu.planner import BurstPlanner
    p = BurstPlanner.__new__(BurstPlanner)
    p.carry, p._speed_obs, p.stats = 1.0, {}, {}
    g = ("n", 0)
    p.observe_time(g, 10.0, 11.0)
    p.observe_time(g, 10.0, 500.0)          # outlier, clipped to SPEED_CLIP[1]
    assert p.speed(g) == 1.0                # fewer than SPEED_MIN_OBS observations
    p.observe_time(g, 10.0, 11.0)
    assert p.speed(g) == pytest.approx(1.1)
    p.observe_time(g, 0.0, 5.0)             # no prediction: ignored
    assert len(p._speed_obs[g]) == 3


def test_released_pods_leave_the_slot_timeline_and_the_feedback():
    """unreserved / deleted pods were never removed from the slot chains (phantom
    work forever) and their predicted durations outlived them in the completion feedback."""
    from k8s_gpu_scheduler_amd.api import objects as O
    from k8s_gpu_scheduler_amd.plugins.gpu.planner import BurstPlanner
    from k8s_gpu_scheduler_amd.plugins.gpu.timeline import SlotTimeline

    class _FB:
        def __init__(self):
            self.forgot = []

        def forget(self, k):
            self.forgot.append(k)
    p = BurstPlanner.__new__(BurstPlanner)
    p.timeline, p.feedback, p.drop_on_delete = SlotTimeline(depth=6, phantoms=2), _FB(), True
    g = ("n", 0)
    pods = {n: O.make_pod(n, gpu_cu=64) for n in ("a", "b", "c")}
    for i, n in enumerate(pods):
        p.timeline.place(g, (2 * i, 2), O.key(pods[n]), 0, 20.0, 1.0)
    p.released(pods["a"], "unreserve")
    p.released(pods["b"], "delete")
    fin = pods["c"]
    fin["status"] = {"phase": "Succeeded", "containerStatuses": [{"state": {"terminated": {
        "startedAt": "2026-01-01T00:00:01Z", "finishedAt": "2026-01-01T00:00:31Z"}}}]}
    p.released(fin, "terminal")
    ch = p.timeline.chains(g)
    keys = [k for c in ch.values() for k, _, _ in c]
    assert keys == [O.key(fin)]
    (_, s, e), = [x for c in ch.values() for x in c]
    assert e - s == pytest.approx(30000.0)                 # measured from its container times (ms)
    # a 2-s span of whole-second kubelet timestamps is quantisation noise: dropped, not measured
    short = O.make_pod("s", gpu_cu=64)
    p.timeline.place(g, (4, 2), O.key(short), 0, 20.0, 1.0)
    short["status"] = {"phase": "Succeeded", "containerStatuses": [{"state": {"terminated": {
        "startedAt": "2026-01-01T00:01:01Z", "finishedAt": "2026-01-01T00:01:03Z"}}}]}
    p.released(short, "terminal")
    assert O.key(short) not in [k for c in p.timeline.chains(g).values() for k, _, _ in c]
    assert p.feedback.forgot == [O.key(pods["a"]), O.key(pods["b"])]
    # the pipelined bench keeps deleted in-flight pods (its executor measures them)
    p.drop_on_delete = False
    p.timeline.place(g, (0, 2), "default/d", 0, 20.0, 1.0)
    p.released(O.make_pod("d", gpu_cu=64), "delete")
    assert "default/d" in [k for c in p.timeline.chains(g).values() for k, _, _ in c]


def test_direction_arrivals_stay_in_band_with_a_40pct_slower_gpu():
    """The hardware direction test's arrivals (seed 5) with GPU 1 running 1.4x the model's
    time: with measured speeds scaling the plan's makespans (native plan_corun `speed`) each
    burst is balanced in measured time, so GPU 1's share of epochs 6-11 stays within
    [0.15, 0.5] (target 1 / 2.4 = 0.42) -- without it the carried backlog pulled work back one
    burst late (0.34 / 0.48 / 0.57 on MI355X)."""
    res, planner = _run(12, slow=(1.0, 1.4), seed=5)
    share = np.array([s for _, s, _, _ in res])[6:]
    assert share.min() >= 0.15 and share.max() <= 0.5, share
    assert abs(share.mean() - 1 / 2.4) < 0.05, share
    assert all(min(n) > 0 for n, *_ in res)


# ---- the speed gate must see a 10-20 % slower GPU at realistic noise.
# Round 5's gate (every one of 7 window observations on the slow side) left GPU 1's share at
# 0.50 with +-8 % noise; the rank test (planner.rank_z, SPEED_Z) is the statistical decision.
# A single run's 60-burst share moves by +-0.015 with the arrival / noise seed (4-pod bursts
# split discretely and the SLO objective picks among near-balanced splits), so the bars are on
# the mean over five seeds; seed 5 is the harness run VERDICT r5 quoted (round-5 gate: 0.504 /
# 0.497 / 0.500 for the three cases below).
SEEDS = (5, 6, 7, 8, 9)


def _share(res, start=60):
    return float(np.mean([s for _, s, _, _ in res][start:]))


def _mean_share(slow, noise):
    return float(np.mean([_share(_run(120, slow=slow, noise=noise, seed=sd)[0]) for sd in SEEDS]))


def test_ten_percent_slower_gpu_is_seen_at_8pct_noise():
    res, _ = _run(120, slow=(1.0, 1.1), noise=0.08)
    assert _share(res) <= 0.485, _share(res)             # fair 0.5, target 1 / 2.1 = 0.476
    assert all(min(n) > 0 for n, *_ in res)
    assert _mean_share((1.0, 1.1), 0.08) <= 0.4875       # five seeds: 0.486 (round 5: ~0.50)


def test_twenty_percent_slower_gpu_is_seen_at_15pct_noise():
    assert _mean_share((1.0, 1.2), 0.15) <= 0.47         # target 1 / 2.2 = 0.455; five seeds 0.463


def test_identical_gpus_at_8pct_noise_plan_as_if_noiseless():
    assert abs(_mean_share((1.0, 1.0), 0.08) - 0.5) <= 0.01
    same = []
    for sd in SEEDS:
        quiet, _ = _run(120, noise=0.0, seed=sd)
        noisy, _ = _run(120, noise=0.08, seed=sd)
        same.append(sum(a[0] == b[0] for a, b in zip(quiet, noisy)) / len(quiet))
    assert np.mean(same) >= 0.9 and min(same) >= 0.85, same


def test_rank_z_separates_shifted_windows_only():
    from k8s_gpu_scheduler_amd.plugins.gpu.planner import rank_z
    rng = np.random.default_rng(0)
    same = [abs(rank_z(1 + 0.08 * rng.uniform(-1, 1, 16), 1 + 0.08 * rng.uniform(-1, 1, 48))) for _ in range(400)]
    # identical distributions: |z| >= 2.33 in about 2 % of draws
    assert np.mean(np.array(same) >= 2.33) < 0.05
    slow = [rank_z(1.1 * (1 + 0.08 * rng.uniform(-1, 1, 16)), 1 + 0.08 * rng.uniform(-1, 1, 48)) for _ in range(100)]
    assert min(slow) > 2.33
    assert rank_z(np.array([1.0, 1.0]), np.array([1.0, 1.0])) == 0.0
    assert rank_z(np.array([]), np.array([1.0])) == 0.0


def test_direction_twin_over_seeds():
    """The 40 %-slower direction case over five arrival seeds: GPU 1's mean share of epochs 6-11
    within 0.06 of the 1 / 2.4 target for every seed and within 0.02 on average (round 6 gate:
    0.37-0.46 per seed, 0.419 on average)."""
    ms = []
    for sd in SEEDS:
        res, _ = _run(12, slow=(1.0, 1.4), seed=sd)
        ms.append(float(np.mean([s for _, s, _, _ in res][6:])))
    assert all(abs(m - 1 / 2.4) < 0.06 for m in ms), ms
    assert abs(np.mean(ms) - 1 / 2.4) < 0.02, ms
