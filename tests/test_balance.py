"""Least-predicted-load balancing across a node's GPUs, longest-work-first queue sort and
the observed work-cost model (telemetry.workcost).

The ranks of a multi-GPU job are coupled (here: the bench's per-epoch placement broadcast),
so the busiest GPU sets the pace; the GPU plugin's balance term spreads predicted GPU time
evenly, the queueSort orders a burst longest-first (LPT list scheduling)."""
import json
import os
import subprocess
import sys

import pytest

from k8s_gpu_scheduler_amd.api import constants as C
from k8s_gpu_scheduler_amd.api import objects as O
from k8s_gpu_scheduler_amd.framework.config import default_gpu_config
from k8s_gpu_scheduler_amd.framework.queue import QueuedPodInfo
from k8s_gpu_scheduler_amd.framework.scheduler import Scheduler
from k8s_gpu_scheduler_amd.kube.client import FakeCluster
from k8s_gpu_scheduler_amd.plugins import full_registry
from k8s_gpu_scheduler_amd.plugins.gpu.devices import DeviceLedger, synth_uuid
from k8s_gpu_scheduler_amd.plugins.gpu.plugin import GPUPlugin
from k8s_gpu_scheduler_amd.telemetry.cache import TelemetryCache
from k8s_gpu_scheduler_amd.telemetry.workcost import WorkCostModel

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


class _Pred:
    """Predictions: 'big' workloads run 1 iteration/s on a whole GPU, 'small' 10/s."""

    def configurations(self, name):
        tput = 1.0 if "big" in name else 10.0
        return {f"{p}P_{C.MI355X}": tput / p for p in (1, 2, 4, 8)}

    def interference(self, name):
        return {}


def _world(args, queue_sort=True, workcost=None):
    fc = FakeCluster()
    fc.create("nodes", O.make_node("n0", gpus=4))
    ledger = DeviceLedger()
    extras = {"ledger": ledger, "telemetry": TelemetryCache(stale_s=0), "predictions": _Pred()}
    if workcost is not None:
        extras["workcost"] = workcost
    s = Scheduler(fc, default_gpu_config(args, disable_defaults=True, queue_sort=queue_sort), full_registry(),
                  bind_async=False, seed=0, extras=extras)
    s.start_informers()
    return fc, s, ledger


def _pod(name, iters=10):
    return O.make_pod(name, gpu_cu=64, env={C.ENV_ITERATIONS: str(iters)})


def _loads(ledger):
    return ledger.gpu_work("n0")


def test_ledger_tracks_predicted_work_per_gpu():
    led = DeviceLedger()
    fc = FakeCluster()
    fc.create("nodes", O.make_node("n0", gpus=2))
    from k8s_gpu_scheduler_amd.plugins.gpu.devices import devices_for_node
    led.set_devices("n0", devices_for_node(fc.get("nodes", "n0")))
    u0, u1 = synth_uuid("n0", 0), synth_uuid("n0", 1)
    assert led.reserve("n0", "ns/a", "a", 0, [(u0, 0, 2, 1.0, False)], work=3.0)
    assert led.reserve("n0", "ns/b", "b", 0, [(u0, 2, 2, 1.0, False)], work=1.5)
    assert led.reserve("n0", "ns/c", "c", 0, [(u0, 4, 2, 0.0, False), (u1, 0, 2, 0.0, False)], work=2.0)
    assert led.gpu_work("n0") == {0: 5.5, 1: 1.0}
    led.release("ns/a")
    assert led.gpu_work("n0") == {0: 2.5, 1: 1.0}
    led.release("ns/b")
    led.release("ns/c")
    assert led.gpu_work("n0") == {0: 0.0, 1: 0.0}


def test_pod_work_from_predictions_and_observed_cost():
    p = GPUPlugin({"w_balance": 1.0}, None, predictions=_Pred())
    conf = _Pred().configurations("big-x")
    assert p.pod_work(_pod("big-x", iters=20), conf) == pytest.approx(20.0)
    svc = O.make_pod("big-svc", gpu_cu=64, slo=0.25)            # service: SLO x s/iter
    assert p.pod_work(svc, conf) == pytest.approx(0.25)
    assert p.pod_work(_pod("nothing"), {}) == 0.0
    wc = WorkCostModel(alpha=0.5)
    wc.observe("big", 0.2)
    p.workcost = wc                                           # observed co-run cost wins
    assert p.pod_work(_pod("big-x", iters=20), conf) == pytest.approx(4.0)
    wc.observe("big", 0.4)                                    # EWMA
    assert p.pod_work(_pod("big-x", iters=20), conf) == pytest.approx(20 * 0.3)


def test_workcost_label_resolution_prefers_longest_label():
    wc = WorkCostModel()
    wc.observe("onnx_resnet50_1024", 1.0)
    wc.observe("onnx_resnet50_10240", 2.0)
    assert wc.seconds_per_iter("onnx-resnet50-10240-e1-p3") == 2.0
    assert wc.seconds_per_iter("onnx-resnet50-1024-e1-p3") == 1.0
    assert wc.seconds_per_iter("busybox-abc") is None
    wc.observe("x", -1.0)                                     # ignored
    assert "x" not in wc.snapshot()


def test_balance_spreads_predicted_work_over_gpus():
    """4 big (10 s) + 12 small (1 s) pods, 4 GPUs x 4 slots: least-loaded + LPT puts one
    big pod on each GPU; without the term bin-packing stacks the big pods."""
    fc, s, ledger = _world({"w_slo": 0.0, "w_pack": 0.25, "w_telemetry": 0.0, "w_balance": 1.0})
    names = [f"small-{i}" for i in range(12)] + [f"big-{i}" for i in range(4)]
    for n in names:
        fc.create("pods", _pod(n))
    s.schedule_pending()
    loads = _loads(ledger)
    assert sorted(loads.values()) == pytest.approx([13.0] * 4)
    fc2, s2, ledger2 = _world({"w_slo": 0.0, "w_pack": 0.25, "w_telemetry": 0.0, "w_balance": 0.0},
                              queue_sort=False)
    for n in names:
        fc2.create("pods", _pod(n))
    s2.schedule_pending()
    assert max(_loads(ledger2).values()) >= 31.0              # 3 big + 1 small on one GPU


def test_lpt_queue_sort_orders_burst_longest_first_with_windows():
    p = GPUPlugin({"lpt_window_s": 1.0}, None, predictions=_Pred())
    a = QueuedPodInfo(_pod("small-a"), timestamp=10.1)
    b = QueuedPodInfo(_pod("big-b"), timestamp=10.5)
    c = QueuedPodInfo(_pod("big-c"), timestamp=11.2)          # next window
    hi = QueuedPodInfo(O.make_pod("small-hi", gpu_cu=64, priority=5), timestamp=12.0)
    order = sorted([a, b, c, hi], key=p._sort_key)
    assert [O.name(x.pod) for x in order] == ["small-hi", "big-b", "small-a", "big-c"]
    assert p.less(b, a) and not p.less(a, b)


def test_bench_sim_balance_flag_and_cost_learning():
    from k8s_gpu_scheduler_amd.parallel.podbench import ControlPlane, main
    r = main(["--sim", "--gpus", "4", "--steps", "3", "--warmup", "1", "--balance", "1"])
    assert r["config"]["balance"] == 1.0 and r["unscheduled"] == 0
    cp = ControlPlane(n_gpus=2, pods_per_gpu=4, iters=20, seed=0, balance=1.0)
    import numpy as np
    from k8s_gpu_scheduler_amd.parallel.podbench import TELE
    per_gpu = np.zeros((2, TELE))
    per_gpu[0, 4:6] = (0.5, 2)                                # workload 0: 2 pods, 0.25 s/iter mean
    cp.update_telemetry(per_gpu, 10.0)
    from k8s_gpu_scheduler_amd.models import workloads as W
    assert cp.workcost.snapshot()[W.NAMES[0]] == pytest.approx(0.25)


@pytest.mark.slow
def test_bench_timed_sim_four_ranks_balance_improves_throughput(tmp_path):
    """Rehearsal of the coupled multi-rank run (gloo, modelled device time): spreading
    predicted work must not lose throughput against plain bin-packing."""
    best = {}
    # wall-clock timed runs on a shared CPU: further interleaved pairs (best of each arm) absorb
    # a load spike during one run (other test processes under pytest -n, a cold page cache after
    # a native rebuild); the modelled epoch (--sim-scale 4, ~26 ms) leaves the control plane room
    # on a loaded CPU, so the comparison is of placements, not of scheduling speed
    for attempt in range(5):
        for bal in (0, 1):
            env = dict(os.environ, CUDA_VISIBLE_DEVICES="", HIP_VISIBLE_DEVICES="")
            cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", "--nproc-per-node=4",
                   "--master-addr", "127.0.0.1", "--master-port", str(29621 + bal + 2 * attempt),
                   os.path.join(ROOT, "bench.py"),
                   "--sim-timed", "--sim-scale", "4", "--gpus", "4", "--steps", "16", "--warmup", "3",
                   "--balance", str(bal), "--plan-bursts", "0"]
            p = subprocess.run(cmd, capture_output=True, text=True, timeout=300, env=env, cwd=ROOT)
            assert p.returncode == 0, p.stderr[-3000:]
            r = json.loads([l for l in p.stdout.splitlines() if l.startswith("{")][0])
            assert bal == 0 or r["unscheduled"] == 0
            best[bal] = max(best.get(bal, 0.0), r["value"])
        if best[1] >= 0.97 * best[0]:
            break
    assert best[1] >= 0.97 * best[0], best


def test_batch_filter_and_score_match_node_at_a_time():
    """framework.runtime.find_feasible/run_score with the plugins' batch forms give the
    same feasible set, first-failure statuses and scores as the node-at-a-time loop."""
    from k8s_gpu_scheduler_amd.framework.config import default_gpu_config
    from k8s_gpu_scheduler_amd.framework.interface import CycleState
    fc = FakeCluster()
    for i in range(40):
        kw = {}
        if i % 7 == 3:
            kw["taints"] = [{"key": "dedicated", "value": "x", "effect": "NoSchedule"}]
        if i % 5 == 1:
            kw["labels_"] = {"zone": "b"}
        node = O.make_node(f"n{i:02d}", gpus=2 if i % 3 else 1, cpu="4" if i % 4 == 2 else "64")
        if kw.get("taints"):
            node["spec"]["taints"] = kw["taints"]
        if kw.get("labels_"):
            node["metadata"]["labels"].update(kw["labels_"])
        if i % 11 == 5:
            node["spec"]["unschedulable"] = True
        fc.create("nodes", node)
    s = Scheduler(fc, default_gpu_config({"w_balance": 1.0}), full_registry(), bind_async=False, seed=0,
                  extras={"ledger": DeviceLedger(), "telemetry": TelemetryCache(stale_s=0), "predictions": _Pred()})
    s.start_informers()
    for i in range(30):                              # load some GPUs
        fc.create("pods", O.make_pod(f"warm-{i}", gpu_cu=128, cpu="1"))
    s.schedule_pending()
    fw = s.frameworks[C.SCHEDULER_NAME]
    seen_plugins = set()
    pods = [O.make_pod("q1", gpu_cu=64, cpu="8"), O.make_pod("q2", gpu_cu=256, node_selector={"zone": "b"}),
            O.make_pod("q3", gpus=2), O.make_pod("q4", gpu_cu=64, tolerations=[{"key": "dedicated",
                                                                                 "operator": "Exists"}])]
    for pod in pods:
        for limit in (0, 3, 7):
            nodes = s.cache.snapshot().list()
            s._snapshot = s.cache.snapshot()
            st1 = CycleState()
            fw.run_pre_filter(st1, pod)
            feas1, failed1 = fw.find_feasible(st1, pod, nodes, limit)
            st2 = CycleState()
            fw.run_pre_filter(st2, pod)
            feas2, failed2 = [], {}
            for ni in nodes:                         # reference: one node at a time
                r = fw.run_filter(st2, pod, ni)
                if r.ok:
                    feas2.append(ni)
                    if limit and len(feas2) >= limit:
                        break
                else:
                    failed2[ni.name] = r
            assert [n.name for n in feas1] == [n.name for n in feas2], (O.name(pod), limit)
            assert {k: (v.code, v.plugin, v.reasons) for k, v in failed1.items()} == \
                   {k: (v.code, v.plugin, v.reasons) for k, v in failed2.items()}
            seen_plugins |= {v.plugin for v in failed1.values()}
            if len(feas1) > 1 and limit == 0:
                fw.run_pre_score(st1, pod, feas1)
                batch, ok = fw.run_score(st1, pod, feas1)
                assert ok.ok
                per_node = {}
                for p in fw.points["score"]:
                    if p.name() in st1.skip_score_plugins:
                        continue
                    per_node[p.name()] = [p.score(st1, pod, n.name)[0] for n in feas1]
                got = st1.read("framework/per-plugin-scores")
                for name, vals in per_node.items():
                    raw = [ns.score for ns in got[name]]
                    if name != "GPU":                # GPU's list is normalized in place
                        assert raw == vals, name
    assert {"TaintToleration", "NodeResourcesFit", "NodeAffinity", "NodeUnschedulable"} <= seen_plugins, seen_plugins


def test_lpt_sort_key_follows_requeue_timestamp():
    p = GPUPlugin({"lpt_window_s": 1.0}, None, predictions=_Pred())
    a = QueuedPodInfo(_pod("big-a"), timestamp=10.0)
    b = QueuedPodInfo(_pod("small-b"), timestamp=20.0)
    assert p.less(a, b)
    a.timestamp = 30.0                       # a was requeued after b arrived
    assert p.less(b, a)


def test_complement_term_prefers_the_gpu_with_the_other_roofline_class():
    """weightComplement: a stream-bound pod joins the GPU running an MFMA-bound pod rather
    than an idle GPU (balanced MFMA/HBM time after placement scores 100, one-sided 0), and
    without the term the balance-free plugin packs by unit fill alone."""
    def place(w_complement):
        fc = FakeCluster()
        fc.create("nodes", O.make_node("n0", gpus=2))
        ledger = DeviceLedger()
        split = {"gemmy": (1.0, 0.0), "streamy": (0.0, 1.0)}
        extras = {"ledger": ledger, "telemetry": TelemetryCache(stale_s=0), "predictions": _Pred(),
                  "roofline": lambda n: next((v for k, v in split.items() if k in n), None)}
        s = Scheduler(fc, default_gpu_config({"w_complement": w_complement, "w_pack": 0.0, "w_slo": 0.0,
                                              "w_balance": 1.0}, disable_defaults=True),
                      full_registry(), bind_async=False, seed=0, extras=extras)
        s.start_informers()
        for name in ("big-gemmy-0", "big-streamy-0"):
            fc.create("pods", _pod(name))
            s.schedule_pending()
        return {use.name: st.device.gpu for st in ledger.devices("n0") for use in st.pods.values()}
    g = place(3.0)
    assert g["big-gemmy-0"] == g["big-streamy-0"]
    g = place(0.0)                      # balance alone spreads the two pods
    assert g["big-gemmy-0"] != g["big-streamy-0"]


def test_executor_balances_burstable_slots_by_cumulative_work():
    """DeviceExecutor._balance (CPU-testable part): each epoch's same-size Burstable pods go
    longest first onto the slot with the least cumulative work, so the slot that first-fit
    always hands the epoch's longest pod does not become the pipeline's bottleneck; masked
    (Guaranteed) pods keep their slots."""
    import types
    from k8s_gpu_scheduler_amd.parallel.executor import DeviceExecutor, PodRun
    ex = types.SimpleNamespace(_slot_work={}, pod_work=lambda r: {"a": 4.0, "b": 3.0, "c": 2.0, "d": 1.0}[r.pod_id])
    tot = {}
    for e in range(8):
        runs = [PodRun(p, "onnx_resnet50_1024", u, 2, 20, masked=False) for p, u in zip("abcd", (0, 2, 4, 6))]
        DeviceExecutor._balance(ex, runs)
        assert sorted(r.first_unit for r in runs) == [0, 2, 4, 6]
        for r in runs:
            tot[r.first_unit] = tot.get(r.first_unit, 0.0) + ex.pod_work(r)
    assert max(tot.values()) - min(tot.values()) <= 4.0          # first-fit: 32 vs 8
    g = [PodRun("a", "x", 0, 2, 20, masked=True), PodRun("b", "x", 2, 2, 20, masked=True)]
    DeviceExecutor._balance(ex, g)
    assert [r.first_unit for r in g] == [0, 2]
