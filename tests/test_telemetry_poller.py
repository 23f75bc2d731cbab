"""Scheduler-side live telemetry: agent exporter -> (Prometheus | direct scrape) -> poller ->
TelemetryCache -> GPU plugin Score (reference reads DCGM series through Prometheus,
pkg/prom/fetch_prom_metrics/prom_metrics.go:63-118, gpu_plugins.go:162-300)."""
import socket
import time

from k8s_gpu_scheduler_amd.api import constants as C
from k8s_gpu_scheduler_amd.api import objects as O
from k8s_gpu_scheduler_amd.telemetry.cache import TelemetryCache
from k8s_gpu_scheduler_amd.telemetry.exporter import GpuExporter
from k8s_gpu_scheduler_amd.telemetry.fake_prom import FakePrometheus
from k8s_gpu_scheduler_amd.telemetry.poller import (PromSource, ScrapeSource, TelemetryPoller, make_source,
                                                    samples_from_series)

UUIDS = {0: "GPU-aaaa", 1: "GPU-bbbb"}
SAMPLES = [{"index": 0, "gfx_activity": 95.0, "umc_activity": 40.0, "vram_used_mb": 1000.0,
            "vram_total_mb": 294912.0, "power_w": 900.0, "temp_c": 80.0, "xgmi_write_bps": 5e9},
           {"index": 1, "gfx_activity": 0.0, "umc_activity": 0.0, "vram_used_mb": 10.0,
            "vram_total_mb": 294912.0, "power_w": 150.0, "temp_c": 40.0}]


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _exporter():
    exp = GpuExporter("node-a", "amd-gpu-exporter-x")
    exp.observe_samples(SAMPLES, UUIDS)
    return exp


def test_samples_from_series_groups_by_node_and_uuid():
    got = samples_from_series([
        ("amd_gpu_gfx_activity", {"node": "n", "UUID": "u"}, 0.5, 1.0),
        ("amd_gpu_vram_used_mb", {"node": "n", "UUID": "u"}, 100.0, 0.0),
        ("amd_gpu_vram_free_mb", {"node": "n", "UUID": "u"}, 900.0, 0.0),
        ("amd_gpu_gfx_activity", {"UUID": "no-node"}, 0.5, 0.0)])
    assert list(got) == [("n", "u")]
    smp, age = got[("n", "u")]
    assert smp.gfx_activity == 0.5 and smp.vram_total_mb == 1000.0 and age == 1.0


def test_prometheus_source_fills_cache():
    prom = FakePrometheus().start()
    try:
        prom.ingest_exposition(_exporter().render().decode())
        cache = TelemetryCache(stale_s=5)
        p = TelemetryPoller(cache, PromSource(prom.url))
        assert p.poll_once() == 2
        s0, s1 = cache.get("node-a", "GPU-aaaa"), cache.get("node-a", "GPU-bbbb")
        assert abs(s0.gfx_activity - 0.95) < 1e-9 and s1.gfx_activity == 0.0
        assert s0.power_w == 900.0 and s0.xgmi_tx_bps == 5e9 and s0.vram_used_mb == 1000.0
        # one instant query per AMD series, like the reference's fan-out
        assert set(q.split("{")[0] for q in prom.queries) >= set(C.AMD_METRICS[:5])
    finally:
        prom.stop()


def test_scrape_source_and_outage_goes_stale():
    exp = _exporter()
    port = _free_port()
    exp.serve(port, "127.0.0.1")
    cache = TelemetryCache(stale_s=0.3)
    p = TelemetryPoller(cache, ScrapeSource([f"http://127.0.0.1:{port}/metrics"]))
    assert p.poll_once() == 2
    assert cache.get("node-a", "GPU-aaaa").gfx_activity > 0.9
    # exporter unreachable: the poll fails, nothing is written, old samples age out
    bad = TelemetryPoller(cache, ScrapeSource([f"http://127.0.0.1:{_free_port()}/metrics"], timeout_s=0.2))
    assert bad.poll_once() == 0 and bad.failures == 1
    time.sleep(0.4)
    assert cache.get("node-a", "GPU-aaaa") is None and cache.node("node-a") == {}


def test_make_source_prefers_scrape():
    assert isinstance(make_source("http://p:1", "http://a:2/metrics"), ScrapeSource)
    assert isinstance(make_source("http://p:1", ""), PromSource)
    assert make_source("", "") is None


def test_busy_device_loses_score_through_the_poller():
    """A node with two GPUs; the exporter reports GPU 0 at 95 % and GPU 1 idle: after one
    poll the fractional pod lands on GPU 1; with telemetry stale both tie on packing."""
    from k8s_gpu_scheduler_amd.framework.config import default_gpu_config
    from k8s_gpu_scheduler_amd.framework.scheduler import Scheduler
    from k8s_gpu_scheduler_amd.kube.client import FakeCluster
    from k8s_gpu_scheduler_amd.plugins import full_registry
    from k8s_gpu_scheduler_amd.plugins.gpu.devices import synth_uuid
    fc = FakeCluster(sync_watch=True, auto_run=True)
    fc.create("nodes", O.make_node("node-a", gpus=2))
    uuids = {g: synth_uuid("node-a", g) for g in range(2)}
    exp = GpuExporter("node-a", "exp")
    exp.observe_samples(SAMPLES, uuids)
    prom = FakePrometheus().start()
    try:
        prom.ingest_exposition(exp.render().decode())
        cache = TelemetryCache(stale_s=30)
        cfg = default_gpu_config({"w_slo": 0.0, "w_pack": 1.0, "w_telemetry": 1.0}, disable_defaults=True)
        sched = Scheduler(fc, cfg, full_registry(), bind_async=False, record_events=False, seed=1,
                          extras={"telemetry": cache})
        sched.start_informers()
        TelemetryPoller(cache, PromSource(prom.url)).poll_once()
        fc.create("pods", O.make_pod("p0", gpu_cu=64, gpu_mem_gib=4))
        res = sched.schedule_pending()
        assert res and res[0].node == "node-a"
        pod = fc.get("pods", "p0", "default")
        assert O.annotations(pod)[C.ANNOT_DEVICES] == uuids[1]
    finally:
        prom.stop()
