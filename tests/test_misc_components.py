"""Smaller components: recommender smoke client/helpers, metrics logger, host-sanitizer
build of the native host modules, discovery helpers, workload catalog, C++ core
unit-fit search."""
import os

import numpy as np
import pytest

from k8s_gpu_scheduler_amd.agent.metrics_logger import COLUMNS, log_metrics
from k8s_gpu_scheduler_amd.api import constants as C
from k8s_gpu_scheduler_amd.api import objects as O
from k8s_gpu_scheduler_amd.kube.client import FakeCluster
from k8s_gpu_scheduler_amd.kube.resources import Resources
from k8s_gpu_scheduler_amd.models import workloads as W
from k8s_gpu_scheduler_amd.models.imputers import SVDImputer
from k8s_gpu_scheduler_amd.recommender.metrics import holdout_score, masked_mean_error, read_timer
from k8s_gpu_scheduler_amd.recommender.smoke import find_max_ind_for_node
from k8s_gpu_scheduler_amd.utils import discovery as D

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def test_find_max_ind_for_node():
    cols = ["1P_A30", "2P_A30", "4P_A30", "1P_V100"]
    assert find_max_ind_for_node(cols, [624.9, 538.5, 397.6, 725.0], "A30") == ("1P_A30", 624.9)


def test_imputation_metrics():
    t = np.array([[1.0, np.nan], [3.0, 4.0]])
    assert masked_mean_error(t, np.array([[1, 2], [3, 4]]), np.array([[1, 2.5], [3, 4]])) == 0.5
    rng = np.random.default_rng(0)
    X = rng.normal(size=(40, 2)) @ rng.normal(size=(2, 6))
    assert holdout_score(lambda: SVDImputer(k=2), X) < 0.3
    assert read_timer(3725) == "Elapsed Time: 1 hours, 2 minutes and 5 seconds."


def test_metrics_logger(tmp_path):
    out = tmp_path / "m.tsv"
    n = log_metrics(lambda: [{"index": 0, "power_w": 700, "gfx_activity": 50, "temp_c": 60},
                             {"index": 1, "power_w": 300}], str(out), period_s=0, max_samples=3)
    assert n == 6
    lines = out.read_text().splitlines()
    assert lines[0].split("\t") == COLUMNS and len(lines) == 7


def test_discovery_reference_semantics():
    fc = FakeCluster()
    fc.create("nodes", O.make_node("k8s-aferik-master", address="10.1.2.3"))
    fc.create("nodes", O.make_node("worker", address="10.9.9.9"))
    fc.create("pods", O.make_pod("redis-0", ns="redis", node_name="worker", phase="Running"))
    res = Resources(fc, "redis")
    assert D.find_nodes_ip_from_pod(res, "-0") == [{"worker": "10.9.9.9"}]
    # parity: GetNode ignores its argument and returns the master (reference nodes.go:29)
    assert D.find_nodes_ip_from_pod(res, "-0", parity_master="k8s-aferik-master") == \
        [{"k8s-aferik-master": "10.1.2.3"}]
    ep = D.Endpoints().discover(fc)
    assert ep.redis == f"10.9.9.9:{C.REDIS_NODEPORT}" and ep.recommender == ""
    assert D.exists(["GPU-a", "MIG-b"], "MIG") == 1 and D.exists(["x"], "y") == -1
    assert D.remove(["a", "b", "c"], 1) == ["a", "c"]
    with pytest.raises(ValueError):
        D.check(ValueError("boom"))


def test_workload_catalog_shapes_are_kernel_legal():
    assert len(W.CATALOG) == 18
    for w in W.CATALOG.values():
        for o in w.ops:
            if o.kind == "gemm":
                assert o.M % 64 == 0 and o.N % 64 == 0 and o.K % 64 == 0
            else:
                assert o.n_floats % 4 == 0
    assert W.workload_for_pod("mlperf-gpu-onnx-ssd-mobilenet-2048-x").name == "onnx_ssd_mobilenet_2048"
    assert W.workload_for_pod("tensorflow-resnet50-4096-e1-p2").name == "tensorflow_resnet50_4096"
    idx, cols, conf, icols, intf = W.analytic_tables()
    assert cols == ["1P_MI355X", "2P_MI355X", "4P_MI355X", "8P_MI355X"]
    assert all(r[0] > r[-1] > 0 for r in conf)                    # more share -> more throughput


def test_measured_tables_are_consistent():
    from k8s_gpu_scheduler_amd.recommender.tables import Table
    p = os.path.join(ROOT, "k8s_gpu_scheduler_amd", "data", "configurations_mi355x.tsv")
    if not os.path.exists(p):
        pytest.skip("tables not measured yet")
    t = Table.read_tsv(p)
    assert set(t.index) == set(W.NAMES)
    assert not np.isnan(t.values).any() and (t.values > 0).all()


def test_core_find_units_matches_python():
    from k8s_gpu_scheduler_amd import _native
    from k8s_gpu_scheduler_amd.plugins.gpu.devices import Device, DeviceState
    core = _native.core()
    if core is None:
        pytest.skip("_core not built")
    rng = np.random.default_rng(3)
    masks, states = [], []
    for _ in range(200):
        used = rng.random(8) < 0.4
        st = DeviceState(Device("u", "n", 0))
        st.used_units = list(map(bool, used))
        states.append(st)
        masks.append(sum(1 << i for i, b in enumerate(used) if b))
    for n in (1, 2, 4, 8):
        got = core.find_units(np.array(masks, dtype=np.uint64), np.full(len(masks), 8, np.int32), n)
        want = [st._find_units(n) for st in states]
        assert [(-1 if w is None else w) for w in want] == list(got)


@pytest.mark.slow
def test_host_modules_build_with_sanitizers(tmp_path):
    """ASan+UBSan build of the host-only native modules."""
    from k8s_gpu_scheduler_amd._native import build as B
    out = B.build(force=True, asan=True, only=("_core",))
    assert out and out[0].endswith(".so") and "_asan" in out[0]
    os.remove(out[0])


def test_sampler_thread_is_race_free_under_tsan(tmp_path):
    """The amd-smi sampler's thread/ring contract (native/smi/sampler.h) under
    ThreadSanitizer: start/stop/drain from several threads."""
    from k8s_gpu_scheduler_amd._native import build as B
    rc, out = B.sampler_tsan_test(str(tmp_path))
    assert rc == 0 and "ok drained=" in out, out[-3000:]


@pytest.mark.slow
def test_host_modules_build_with_tsan():
    from k8s_gpu_scheduler_amd._native import build as B
    out = B.build(force=True, only=("_core",), san_kind="tsan")
    assert out and "_tsan" in out[0]
    os.remove(out[0])


def test_gc_settle_freezes_the_startup_objects():
    """utils.gctune.settle: one collection, then the surviving objects leave the collector's
    scans (the control plane's start-up state) and the gen-0 threshold is raised."""
    import gc
    from k8s_gpu_scheduler_amd.utils import gctune
    before = gc.get_threshold()
    try:
        gctune.settle(gen0=12345)
        assert gc.get_freeze_count() > 0
        assert gc.get_threshold()[0] >= 12345
    finally:
        gc.unfreeze()
        gc.set_threshold(*before)
