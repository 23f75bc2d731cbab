"""The slot-pipeline side of the co-run model: the native chained simulation (chain_times),
the slot planner (plan_slots), the scheduler's slot timelines (plugins.gpu.timeline), the
model-driven pipeline executor (parallel.modelpipe) and the pipelined virtual node's replay
(tools/pipelined_vn.py)."""
import os
import sys

import numpy as np
import pytest

from k8s_gpu_scheduler_amd import _native
from k8s_gpu_scheduler_amd.models import corun as CR
from k8s_gpu_scheduler_amd.parallel.executor import PodRun
from k8s_gpu_scheduler_amd.plugins.gpu.timeline import SlotTimeline

core = _native.core()
has_chain = core is not None and hasattr(core, "chain_times")
I32 = np.int32
NEG = -1e300
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _toy():
    # memwl presses on memwl only, cmpwl on cmpwl only; 1 ms per iteration alone
    return CR.CorunModel(["memwl", "cmpwl"], [1.0, 1.0], np.array([[0.0, 1.0], [1.0, 0.0]]),
                         np.array([[0.0, 1.0], [1.0, 0.0]]), {"version": "toy"})


@pytest.mark.skipif(not has_chain, reason="_core not built")
def test_chain_times_chains_a_slot_and_matches_the_group_simulation():
    m = _toy()
    # slot A: memwl (10 it) then memwl (5 it); slot B: memwl (10 it) from t=0
    wid = np.array([0, 0, 0], I32)
    it = np.array([10.0, 5.0, 10.0])
    st, fin = core.chain_times(wid, it, np.array([0.0, NEG, 0.0]), np.array([-1, 0, -1], I32), m.alone_ms,
                               m.coupling())
    # both first pods share (rate 1/2) until t=20; the chained pod then runs alone 5 ms
    assert np.allclose(st, [0.0, 20.0, 0.0]) and np.allclose(fin, [20.0, 25.0, 20.0])
    # without chaining it is the multi-way group simulation with staggered starts
    rng = np.random.default_rng(1)
    full = CR.CorunModel.load()
    for _ in range(20):
        k = int(rng.integers(2, 7))
        w = rng.integers(0, len(full.names), k).astype(I32)
        its = rng.integers(5, 40, k).astype(float)
        s0 = np.sort(rng.uniform(0, 3, k))
        _, f1 = core.chain_times(w, its, s0, np.full(k, -1, I32), full.alone_ms, full.coupling())
        f2 = full.group_times(list(w), list(its), list(s0))
        assert np.allclose(f1, f2, rtol=1e-9, atol=1e-9)


@pytest.mark.skipif(not has_chain, reason="_core not built")
def test_plan_slots_puts_the_complementary_pod_next_to_the_inflight_one():
    """Slot 1 runs a measured memory-bound pod until t=10; slot 0 is free.  A new memory pod
    on slot 0 would share HBM with it (500 it/s < its 800 SLO); the planner puts the compute
    pod there and the memory pod on slot 1, after the in-flight one: both meet their SLOs."""
    m = _toy()
    sl, st, fin, exp, spread, min_spread = core.plan_slots(
        np.array([0], I32), np.array([10.0]), np.array([0.0]), np.array([-1], I32), np.array([10.0]),
        np.array([0.0]), np.array([-1, -1], I32), np.array([0.0, 10.0]),
        np.array([0, 1], I32), np.array([10.0, 10.0]), np.array([800.0, 800.0]), np.full(2, NEG),
        m.alone_ms, m.coupling(), 0.0, 100.0, 720)
    assert list(sl) == [1, 0]
    assert exp == pytest.approx(2.0)
    assert np.allclose(fin[1:], [20.0, 10.0])               # memwl after the in-flight pod; cmpwl alongside
    # the tight spread limit keeps the most even assignment even if it meets fewer SLOs
    sl2 = core.plan_slots(
        np.array([0], I32), np.array([10.0]), np.array([0.0]), np.array([-1], I32), np.array([10.0]),
        np.array([0.0]), np.array([-1, -1], I32), np.array([0.0, 10.0]),
        np.array([0, 1], I32), np.array([10.0, 10.0]), np.array([800.0, 800.0]), np.full(2, NEG),
        m.alone_ms, m.coupling(), 0.0, 0.0, 720)[0]
    assert len(set(sl2)) == 2


def _random_slot_case(rng, W):
    """plan_slots inputs shaped like an 8-GPU bench epoch's: measured pinned pods, per-slot chains
    of unmeasured ones, 4 slots, 2-4 new pods (often repeating a workload), 2 phantoms per slot."""
    S = 4
    wid, it, st, prev, pin, slo = [], [], [], [], [], []
    for _ in range(int(rng.integers(0, 8))):                    # measured, pinned
        s0 = float(rng.uniform(-30, 0))
        wid.append(int(rng.integers(0, W))), it.append(20.0), st.append(s0), prev.append(-1)
        pin.append(s0 + float(rng.uniform(1, 40))), slo.append(float(rng.uniform(0, 900)))
    tail = []
    for q in range(S):
        p = -1
        for j in range(int(rng.integers(0, 4))):               # unmeasured chain on slot q
            wid.append(int(rng.integers(0, W))), it.append(20.0), pin.append(0.0)
            slo.append(float(rng.uniform(0, 900)))
            st.append(float(rng.uniform(-5, 5)) if j == 0 else NEG), prev.append(p)
            p = len(wid) - 1
        tail.append(p)
    free = rng.uniform(0, 10, S)
    n = int(rng.integers(2, 5))
    nw = rng.integers(0, W, n)
    nw[1] = nw[0]                                               # a repeated workload
    nslo = np.where(nw == nw[0], 400.0, rng.uniform(100, 900, n))
    ph_off = np.arange(0, 2 * S + 1, 2, dtype=np.int64)
    ph_w = rng.integers(0, W, 2 * S).astype(I32)
    return ((np.array(wid, I32), np.array(it), np.array(st), np.array(prev, I32), np.array(pin), np.array(slo),
             np.array(tail, I32), free, nw.astype(I32), np.full(n, 20.0), nslo, np.full(n, NEG)),
            (ph_off, ph_w, np.full(2 * S, 20.0)))


def _brute_slots(args, ph, alone, cmat, sigma, tol):
    """Reference: every injective assignment simulated with chain_times, plan_slots' rule."""
    import itertools
    from math import erfc, log, sqrt
    cw, ci, cs, cp, cpin, cslo, tail, free, nw, ni, nslo, nrel = args
    ph_off, ph_w, ph_i = ph
    m, n, S = len(cw), len(nw), len(tail)
    res = []
    for perm in itertools.permutations(range(S), n):
        w, it, s0, pv, pe, sl = list(cw), list(ci), list(cs), list(cp), list(cpin), list(cslo)
        last = list(tail)
        for j, s in enumerate(perm):
            w.append(nw[j]), it.append(ni[j]), sl.append(nslo[j]), pe.append(0.0)
            pv.append(tail[s]), s0.append(nrel[j] if tail[s] >= 0 else max(free[s], nrel[j]))
            last[s] = m + j
        for q in range(S):
            p = last[q]
            for x in range(ph_off[q], ph_off[q + 1]):
                w.append(ph_w[x]), it.append(ph_i[x]), sl.append(0.0), pe.append(0.0)
                pv.append(p), s0.append(NEG if p >= 0 else free[q])
                p = len(w) - 1
        st, fin = core.chain_times(np.array(w, I32), np.array(it), np.array(s0), np.array(pv, I32), alone, cmat,
                                   np.array(pe))[:2]
        e = 0.0
        for i in range(len(w)):
            if (i < m and pv[i] < 0 and pe[i] > s0[i]) or sl[i] <= 0 or it[i] <= 0 or fin[i] >= 1e299:
                continue
            t = it[i] / max(fin[i] - st[i], 1e-12) * 1e3
            e += 0.5 * erfc(-log(max(t, 1e-12) / sl[i]) / (sigma * sqrt(2.0)))
        ends = []
        for s in range(S):
            x = free[s] if tail[s] < 0 else fin[tail[s]]
            for j, sj in enumerate(perm):
                if sj == s:
                    x = fin[m + j]
            ends.append(x)
        res.append((perm, e, max(ends) - min(ends)))
    min_sp = min(r[2] for r in res)
    best, be, bs = None, -1.0, 1e300
    for perm, e, sp in res:
        if sp > min_sp + tol + 1e-9:
            continue
        if e > be + 1e-9 or (e > be - 1e-9 and sp < bs - 1e-9):
            best, be, bs = perm, e, sp
    return list(best), be, bs


@pytest.mark.skipif(not has_chain, reason="_core not built")
def test_plan_slots_fast_forward_and_twin_pruning_match_the_full_enumeration():
    """plan_slots simulates the context prefix before the first new pod can start once
    (fast_forward) and skips assignments that only permute identical new pods; both give the
    assignment, expected SLOs met and spread of simulating every assignment in full."""
    full = CR.CorunModel.load()
    rng = np.random.default_rng(7)
    for _ in range(60):
        args, ph = _random_slot_case(rng, len(full.names))
        ref = _brute_slots(args, ph, full.alone_ms, full.coupling(), 0.05, 2.0)
        for ff in (True, False):
            sl, st, fin, exp, spread, _ = core.plan_slots(*args, full.alone_ms, full.coupling(), 0.05, 2.0, 720,
                                                          *ph, fast_forward=ff)
            assert list(sl) == ref[0] and exp == pytest.approx(ref[1], abs=1e-9) and \
                spread == pytest.approx(ref[2], abs=1e-9), (ff, list(sl), ref)


def test_slot_timeline_chains_unmeasured_pods_and_pins_measured_ones():
    tl = SlotTimeline(depth=4, phantoms=2)
    g = ("n0", 0)
    tl.next_burst()
    tl.place(g, (0, 2), "a", 0, 10.0, 500.0)
    tl.place(g, (2, 2), "b", 1, 10.0, 0.0)
    tl.next_burst()
    tl.place(g, (0, 2), "c", 1, 5.0, 0.0)
    assert tl.measure(g, 0, 0.0, 12.0) and tl.measure(g, 2, 0.0, 8.0)
    assert not tl.measure(g, 6, 0.0, 1.0) and tl.unmatched == 1
    ctx = tl.context(g, [(0, 2), (2, 2), (4, 2)])
    keys = ctx["keys"]
    # the unmeasured "c" starts when slot 0's last measured pod ("a") ended; "b" ended before
    # that window, so slot 1 is free from its end
    i_c = keys.index("c")
    assert ctx["prev"][i_c] == -1 and ctx["start"][i_c] == pytest.approx(12.0)
    assert list(ctx["slot_tail"]) == [i_c, -1, -1]
    assert ctx["slot_free"][1] == pytest.approx(8.0)
    # phantoms: each candidate slot continues with its own recent workloads (2 per slot)
    assert list(ctx["ph_off"]) == [0, 2, 4, 6]


@pytest.mark.skipif(not has_chain, reason="_core not built")
def test_model_pipeline_executor_runs_slots_back_to_back():
    from k8s_gpu_scheduler_amd.parallel.modelpipe import ModelPipelineExecutor
    ex = ModelPipelineExecutor(model=_toy(), noise=0.0, host_ms=0.0)
    e1 = [PodRun(0, "memwl", 0, 2, 10), PodRun(1, "cmpwl", 2, 2, 10)]
    e2 = [PodRun(2, "memwl", 0, 2, 5)]
    # the toy names are not catalog workloads: borrow two catalog entries for the FLOP / byte
    # accounting the executor keeps
    import k8s_gpu_scheduler_amd.parallel.modelpipe as MP
    cat = MP.W.CATALOG
    MP.W.CATALOG = {"memwl": cat["onnx_mobilenet_1024"], "cmpwl": cat["onnx_resnet50_1024"]}
    try:
        ex.launch_epoch(e1)
        ex.launch_epoch(e2)
        ex.wait_epoch(e1)
        ex.wait_epoch(e2)
    finally:
        MP.W.CATALOG = cat
    # memwl and cmpwl do not couple: 10 ms each; the chained memwl then runs 5 ms alone
    assert e1[0].ms == pytest.approx(10.0) and e1[1].ms == pytest.approx(10.0)
    assert e2[0].start.t == pytest.approx(10.0) and e2[0].ms == pytest.approx(5.0)
    assert ex.elapsed_ms == pytest.approx(15.0)


def test_pipelined_vn_coupled_release_and_sim_replay():
    sys.path.insert(0, os.path.join(ROOT, "tools"))
    import pipelined_vn as PV
    # GPU 1 collects epoch 0 at 9 ms, GPU 0 at 5: with lookahead 1, epoch 2's broadcast waits
    # for both (9), epoch 3's for epoch 1 (max 14, 12)
    rel = PV.coupled_release([[5.0, 12.0, 20.0, 30.0], [9.0, 14.0, 19.0, 25.0]], 1)
    assert rel == [0.0, 0.0, 9.0, 14.0]
    if not has_chain:
        return
    from k8s_gpu_scheduler_amd.models import workloads as W
    from k8s_gpu_scheduler_amd.parallel.modelpipe import ModelPipelineExecutor
    w = W.INDEX["onnx_mobilenet_1024"]
    epochs = [{"timed": e > 0, "arr": [[0, 2 * s, 2, w, 20, 1, 0] for s in range(4)] +
               [[1, 0, 2, w, 20, 1, 0]]} for e in range(4)]
    out = PV.replay_gpu(ModelPipelineExecutor(noise=0.0), epochs, 0, 2)
    assert out["pods"] == 12 and out["slo_ok"] == 12 and out["span_ms"] > 0
    assert len(out["done_ms"]) == 4 and out["done_ms"] == sorted(out["done_ms"])
    gated = PV.replay_gpu(ModelPipelineExecutor(noise=0.0), epochs, 0, 2, release=[0.0, 0.0, 0.0, 50.0])
    assert gated["done_ms"][3] > 50.0 > out["done_ms"][3]


@pytest.mark.skipif(core is None, reason="_core not built")
def test_lpt_slot_policy_levels_the_slot_streams_at_one_gpu():
    """plan_slots='lpt': the scheduler itself puts each epoch's pods, longest predicted work
    first, on the slot with the least cumulative work -- the longest pod is not always on
    slot 0 (the first-fit order the executor used to re-slot), and the four slot streams'
    cumulative work stays within one pod's work of each other."""
    from k8s_gpu_scheduler_amd.parallel import podbench as PB
    cp = PB.ControlPlane(n_gpus=1, pods_per_gpu=4, iters=20, seed=3, balance=1.0, plan_bursts=True,
                         plan_tolerance=0.3, slo_objective="corun", corun_sigma=0.05, plan_carry=1.0,
                         plan_slots="lpt")
    pl = cp.plugin.planner
    model = cp.plugin.corun_model()
    longest_slot = set()
    max_work = 0.0
    for _ in range(24):
        cp.finish_live()
        arr = cp.schedule_epoch()
        rows = [r for r in arr if r[0] >= 0]
        assert sorted(int(r[1]) for r in rows) == [0, 2, 4, 6]
        work = [float(model.alone_ms[int(r[3])]) * float(r[4]) for r in rows]
        max_work = max(max_work, max(work))
        longest_slot.add(int(rows[int(np.argmax(work))][1]))
    st = cp.planner_stats()
    assert st["slot_policy"] == "lpt" and st["slot_pods"] == 96
    assert len(longest_slot) >= 3
    assert st["slot_work_spread_ms"] <= max_work + 1e-9


@pytest.mark.skipif(not has_chain, reason="_core not built")
def test_plan_corun_pipeline_phantoms_shape_and_no_op():
    """plan_corun's pipeline context may carry one phantom (the slot's likely next pod) per
    free slot; with every phantom absent (-1) the plan equals the phantom-free plan, and a
    phantom that presses on the burst's memory pods changes the predicted SLOs it plans on."""
    m = _toy()
    args = dict(units=np.full(4, 2, I32), wid=np.array([0, 0, 1, 1], I32), iters=np.array([20.0, 20.0, 5.0, 5.0]),
                slo=np.array([900.0, 900.0, 0.0, 0.0]), dev_gpu=np.array([0, 1], I32), dev_free=np.array([4, 4], I32),
                res_off=np.zeros(3, np.int64), r_wid=np.zeros(0, I32), r_iters=np.zeros(0), r_slo=np.zeros(0),
                alone_ms=m.alone_ms, cmat=m.coupling(), tolerance=1.0)
    six = (np.array([0, 0, 0], np.int64), np.zeros(0, I32), np.zeros(0), np.zeros(0),
           np.array([0, 2, 4], np.int64), np.zeros(4))
    dev0 = np.array([0, 0, 1, 1], I32)
    base = list(core.plan_corun(dev0, pipe=six, **args))
    none = six + (np.full(4, -1, I32), np.zeros(4))
    assert list(core.plan_corun(dev0, pipe=none, **args)) == base
    # each memory pod beside a compute pod is the only plan meeting both 900 it/s SLOs
    assert base[0] != base[1] and base[2] != base[3]
    with pytest.raises(RuntimeError):
        core.plan_corun(dev0, pipe=six + (np.full(3, -1, I32), np.zeros(3)), **args)
    # memory-pressing phantoms behind every slot: the short compute pods' slots continue with
    # memory pods, which co-run with the long memory pods -- still a valid full plan
    mem = six + (np.zeros(4, I32), np.full(4, 20.0))
    out = list(core.plan_corun(dev0, pipe=mem, **args))
    assert sorted(out) == [0, 0, 1, 1]


@pytest.mark.skipif(core is None, reason="_core not built")
def test_control_plane_lowers_planning_effort_when_it_paces_the_gpus():
    """ControlPlane(adaptive=True): scheduling back to back (the pipeline period is the
    scheduling time itself) drives the planner to its cheapest effort level; with ample time
    between requests it climbs back to the configured plan."""
    import time as _t
    from k8s_gpu_scheduler_amd.parallel import podbench as PB
    cp = PB.ControlPlane(n_gpus=2, pods_per_gpu=4, iters=20, seed=1, balance=1.0, plan_bursts=True,
                         plan_tolerance=0.3, slo_objective="corun", corun_sigma=0.05, plan_carry=1.0,
                         plan_slots="auto", adaptive=True)
    pl = cp.plugin.planner
    assert pl.effort == 0 and pl.pipe_phantoms and pl.slot_policy == "auto"
    for _ in range(24):
        cp.finish_live()
        cp.schedule_epoch()
    assert pl.effort == 3 and pl.slot_policy == "lpt" and not pl.pipe_eval and pl.sweeps == 1
    assert pl.stats["bursts"] > 0           # level 3 still plans bursts (one sweep per phase)
    for _ in range(60):
        cp.finish_live()
        _t.sleep(0.08)
        cp.schedule_epoch()
    assert pl.effort == 0 and pl.slot_policy == "auto" and pl.pipe_phantoms
    st = cp.planner_stats()
    assert set(st["effort_epochs"]) == {"0", "1", "2", "3"}


@pytest.mark.skipif(core is None, reason="_core not built")
def test_adaptive_effort_jumps_to_the_level_predicted_to_fit():
    """A control plane whose scheduling takes the whole period (it paces the GPUs) jumps from
    level 0 straight to the first level whose predicted cost fits 80 % of the period (level 2:
    0.69 of level 0's cost; level 1's 0.81 does not fit), after two consecutive over-threshold
    checks; the request intervals right after the change are not sampled; with room again it
    climbs back one level."""
    from k8s_gpu_scheduler_amd.parallel import podbench as PB
    cp = PB.ControlPlane(n_gpus=2, pods_per_gpu=4, iters=20, seed=1, balance=1.0, plan_bursts=True,
                         plan_tolerance=0.3, slo_objective="corun", corun_sigma=0.05, plan_carry=1.0,
                         plan_slots="auto", adaptive=True)
    pl = cp.plugin.planner
    ctl = cp._effort                          # the planner's EffortController, fed with periods
    cp.epoch = 10
    t = [0.0]

    def step(period_ms, cost_ms):
        t[0] += period_ms / 1e3
        cp._adapt_effort(t[0])
        ctl.add_cost(cost_ms / 1e3)

    levels = []
    for _ in range(8):
        step(10, 10)
        levels.append(pl.effort)
        if pl.effort:
            break
    # the first decision: as soon as two samples are in, one jump (later ones wait for three
    # samples and two over-threshold checks)
    assert levels[:2] == [0, 0] and levels[-1] == 2 and 1 not in levels
    assert not ctl._allowed and ctl._settle == ctl.settle_n == 3
    for _ in range(ctl.settle_n):
        step(2, 7.5)                          # queued requests arrive back to back: not sampled
    assert not ctl._allowed and pl.effort == 2
    for _ in range(6):
        step(10, 7.5)                         # 75 % of the period (between up and down): stays
    assert pl.effort == 2
    for _ in range(6):
        step(20, 7.5)                         # 38 %: level 1 (81 / 69 x 7.5 = 8.8 ms) fits 80 % of 20
    assert pl.effort == 1


@pytest.mark.skipif(not (has_chain and hasattr(core, "plan_slots_async")), reason="_core not built")
def test_async_slot_plans_give_the_synchronous_placements():
    """The burst planner starts the GPUs' slot plans on the native batch thread and resolves each
    when its pod is planned (planner.slots_async): an 8-GPU control plane at the bench defaults
    makes exactly the placements -- GPU, slot, policy -- of the synchronous slot plans, epoch by
    epoch, with the measured timelines fed back in between."""
    sys.path.insert(0, os.path.join(ROOT, "tools"))
    import virtual_node_bench as V
    from k8s_gpu_scheduler_amd.parallel.podbench import ControlPlane
    # (the online co-run learner off, as in the bench: its background refits land at wall-clock
    # dependent epochs)
    bench = dict(balance=1.0, plan_bursts=True, plan_tolerance=0.3, slo_objective="corun", corun_sigma=0.05,
                 plan_carry=1.0, plan_feedback=True, plan_slots="auto", learn_corun=False)
    runs = {}
    for async_ in (True, False):
        V.N_GPUS = 8
        V.SIM.update(on=True, sigma=0.05, rng=np.random.default_rng(0), speed=[])
        cp = ControlPlane(8, 4, 20, 0, **bench)
        cp.plugin.planner.slots_async = async_
        # one LPT arrival window: the queue's wall-clock windows could split an epoch's
        # arrivals differently in the two runs (a different scheduling order, not a different
        # slot plan)
        cp.plugin.args.lpt_window_s = 1e9
        arrs = []
        for _ in range(14):
            cp.finish_live()
            arr = cp.schedule_epoch()
            arrs.append(np.array(arr, copy=True))
            V.epoch(cp, None, arr, "t")
        st = cp.planner_stats()
        runs[async_] = (arrs, st["model_slot_plans"], st["slot_pods"])
    assert runs[True][1] == runs[False][1] > 0 and runs[True][2] == runs[False][2]
    for a, b in zip(runs[True][0], runs[False][0]):
        assert np.array_equal(a, b)


def test_pacing_probe_adds_its_busy_wait_to_the_epoch_cost(monkeypatch):
    """GPUSCHED_CP_EXTRA_MS (tools/archive/gpu_cp_knee.sh): every epoch's schedule takes at least the
    added busy wait, and the effort rule's cost samples include it."""
    from k8s_gpu_scheduler_amd.parallel import podbench as PB
    monkeypatch.setenv("GPUSCHED_CP_EXTRA_MS", "4")
    cp = PB.ControlPlane(n_gpus=1, pods_per_gpu=4, iters=20, seed=1, balance=1.0, plan_bursts=True,
                         plan_tolerance=0.3, slo_objective="corun", corun_sigma=0.05, plan_carry=1.0,
                         plan_slots="auto", adaptive=True, effort_up=0.65, effort_target=0.75)
    assert cp.extra_s == 0.004
    assert (cp._effort.up, cp._effort.target) == (0.65, 0.75)
    for _ in range(3):
        cp.finish_live()
        cp.schedule_epoch()
    assert cp.sched_s >= 3 * 0.004
    assert min(cp._effort._costs) >= 0.004


def test_effort_level_table_and_its_override(monkeypatch):
    """BurstPlanner.EFFORT_LEVELS: level 1 keeps the pipeline phantoms with a quarter of the
    sweeps; GPUSCHED_EFFORT_LEVELS replaces the table (experiments) and is validated."""
    from k8s_gpu_scheduler_amd.parallel import podbench as PB
    from k8s_gpu_scheduler_amd.plugins.gpu.planner import BurstPlanner
    cp = PB.ControlPlane(n_gpus=2, pods_per_gpu=4, iters=20, seed=1, balance=1.0, plan_bursts=True,
                         plan_tolerance=0.3, slo_objective="corun", corun_sigma=0.05, plan_carry=1.0,
                         plan_slots="auto", adaptive=False)
    pl = cp.plugin.planner
    sweeps = pl._configured[0]
    pl.set_effort(1)
    assert pl.pipe_phantoms and pl.pipe_eval and pl.slot_policy == "auto" and pl.sweeps == max(1, sweeps // 4)
    pl.set_effort(2)
    assert not pl.pipe_phantoms and not pl.pipe_eval and pl.slot_policy == "lpt" and pl.sweeps == max(1, sweeps // 2)
    monkeypatch.setenv("GPUSCHED_EFFORT_LEVELS", "1,1,1,1;2,0,1,1;2,0,0,0;0,0,0,0")
    pl.set_effort(1)                      # round 5's first level 1
    assert not pl.pipe_phantoms and pl.pipe_eval and pl.sweeps == max(1, sweeps // 2)
    monkeypatch.setenv("GPUSCHED_EFFORT_LEVELS", "1,1,1,1;2,0,1,1")
    with pytest.raises(ValueError):
        BurstPlanner._effort_levels()
    monkeypatch.delenv("GPUSCHED_EFFORT_LEVELS")
    pl.set_effort(0)
    assert pl.pipe_phantoms and pl.sweeps == sweeps
