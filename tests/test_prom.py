"""Prometheus query client + exporter.

Ports the reference's hermetic tests as behaviour tests:
* Test_Request (reference pkg/prom/requests/request_test.go): mock server, path
  api/v1/query, `{"test":"mock"}\n` body, 400 when `query` is missing;
* Test_ParseResponse (reference pkg/prom/fetch_prom_metrics/prom_metrics_test.go) on the
  reference's own fixture files (read in place).  Case 2 in the reference expects an empty
  UUID although the fixture carries one and ParseResponse sets it -- it fails there
  (SURVEY.md §2.9 #14); here the UUID is asserted as parsed.
"""
import os

import pytest

from k8s_gpu_scheduler_amd.api import constants as C
from k8s_gpu_scheduler_amd.telemetry.exporter import GpuExporter
from k8s_gpu_scheduler_amd.telemetry.fake_prom import FakePrometheus, parse_selector
from k8s_gpu_scheduler_amd.telemetry.prom import (Requests, ResponseNotOK, create_url, dcgm_prom_instant_query,
                                                  instant_query, metrics_by_device, parse_response)

REF = "/root/reference/pkg/prom/test_data"


def test_create_url():
    assert create_url("http://h:30090/", "api/v1/query", {"query": "X"}) == "http://h:30090/api/v1/query?query=X"
    assert create_url("http://h:1/base", "/api/v1/query", {}) == "http://h:1/base/api/v1/query"


def test_request_against_mock():
    srv = FakePrometheus(mock=True).start()
    try:
        req = Requests(srv.url)
        assert req.request("api/v1/query", {"query": "DCGM_FI_DEV_GPU_UTIL"}) == b'{"test": "mock"}\n'
        with pytest.raises(ResponseNotOK):
            req.request("api/v1/query", {"query": ""})
    finally:
        srv.stop()


def test_parse_response_reference_fixtures():
    mock = os.path.join(REF, "prom_response_mock.txt")
    empty = os.path.join(REF, "empty_response.txt")
    if not os.path.isfile(mock):
        pytest.skip("reference fixtures not mounted")
    assert parse_response(None) is None
    assert parse_response(b"") is None
    rows = parse_response(open(mock, "rb").read())
    assert [r.exporter for r in rows] == ["dcgm-exporter-1673788700-8xg5s", "dcgm-exporter-1673788700-9g6m5",
                                          "dcgm-exporter-1673788700-cf9nx", "dcgm-exporter-1673788700-pcpm7"]
    assert all(r.metric_name == "DCGM_FI_DEV_FB_FREE" and r.value == "4005" for r in rows)
    assert all(r.uuid == "GPU-ae76674e-a8e1-63c6-0b52-bc04a80cb290" and r.gpu_i_id == "" for r in rows)
    assert parse_response(open(empty, "rb").read()) is None


def test_selector_parser():
    assert parse_selector('amd_gpu_gfx_activity{pod="x",gpu!="1"}') == \
        ("amd_gpu_gfx_activity", [("pod", "=", "x"), ("gpu", "!=", "1")])


def test_exporter_to_query_roundtrip():
    exp = GpuExporter("node-a", "amd-gpu-exporter-abc", dcgm_compat=True)
    exp.observe_samples([{"index": 0, "gfx_activity": 75, "umc_activity": 10, "vram_used_mb": 1024,
                          "vram_total_mb": 294912, "temp_c": 55, "power_w": 900},
                         {"index": 1, "gfx_activity": 5, "vram_used_mb": 0, "vram_total_mb": 294912}],
                        {0: "GPU-0", 1: "GPU-1"})
    prom = FakePrometheus().start()
    try:
        assert prom.ingest_exposition(exp.render().decode()) > 0
        rows = instant_query(prom.url, '{pod="amd-gpu-exporter-abc"}')
        by = metrics_by_device(rows)
        assert by["GPU-0"]["amd_gpu_gfx_activity"] == pytest.approx(0.75)
        assert by["GPU-1"]["amd_gpu_vram_free_mb"] == pytest.approx(294912)
        dc = metrics_by_device(dcgm_prom_instant_query(prom.url, '{pod="amd-gpu-exporter-abc"}'))
        assert dc["GPU-0"]["DCGM_FI_PROF_GR_ENGINE_ACTIVE"] == pytest.approx(0.75)
        assert set(dc["GPU-0"]) == set(C.DCGM_METRICS)
        assert instant_query(prom.url, '{pod="other"}') == []
    finally:
        prom.stop()


def test_query_timeout_is_bounded():
    # nothing listening -> empty result quickly, no exception (reference logs & skips)
    import time
    t = time.time()
    assert instant_query("http://127.0.0.1:9", "", timeout_s=0.2) == []
    assert time.time() - t < 3


def test_scheduler_metrics_exporter():
    from k8s_gpu_scheduler_amd.api import objects as O
    from k8s_gpu_scheduler_amd.framework.config import default_gpu_config
    from k8s_gpu_scheduler_amd.framework.scheduler import Scheduler
    from k8s_gpu_scheduler_amd.kube.client import FakeCluster
    from k8s_gpu_scheduler_amd.plugins import full_registry
    from k8s_gpu_scheduler_amd.telemetry.exporter import GpuExporter, attach_scheduler_metrics
    fc = FakeCluster()
    fc.create("nodes", O.make_node("n", gpus=1))
    s = Scheduler(fc, default_gpu_config({}), full_registry(), bind_async=False)
    s.start_informers()
    exp = GpuExporter("n")
    stop = attach_scheduler_metrics(exp, s, period_s=0.05)
    for i in range(3):
        fc.create("pods", O.make_pod(f"p{i}", gpu_cu=128))
    s.schedule_pending()
    import time
    time.sleep(0.2)
    stop()
    txt = exp.render().decode()
    assert 'gpusched_pods_scheduled_total{result="scheduled"} 2.0' in txt
    assert 'gpusched_pods_scheduled_total{result="unschedulable"} 1.0' in txt
    assert "gpusched_scheduling_latency_seconds_count 3.0" in txt
    assert 'gpusched_extension_point_mean_us{point="score"}' in txt


def test_scheduler_http_endpoint_health_and_metrics():
    """kube-scheduler's serving paths: /metrics, /healthz, /livez, /readyz (ready once the
    informer caches synced; liveness fails when the started scheduling loop died)."""
    import urllib.error
    import urllib.request
    from k8s_gpu_scheduler_amd.api import objects as O
    from k8s_gpu_scheduler_amd.framework.config import default_gpu_config
    from k8s_gpu_scheduler_amd.framework.scheduler import Scheduler
    from k8s_gpu_scheduler_amd.kube.client import FakeCluster
    from k8s_gpu_scheduler_amd.plugins import full_registry
    from k8s_gpu_scheduler_amd.telemetry.exporter import GpuExporter, SchedulerHTTP, attach_scheduler_metrics
    fc = FakeCluster()
    fc.create("nodes", O.make_node("n", gpus=1))
    s = Scheduler(fc, default_gpu_config({}), full_registry(), bind_async=False)
    exp = GpuExporter("n")
    stop = attach_scheduler_metrics(exp, s, period_s=0.05)
    http = SchedulerHTTP(exp, s, 0, "127.0.0.1").start()

    def get(path):
        try:
            with urllib.request.urlopen(f"http://127.0.0.1:{http.port}{path}", timeout=5) as r:
                return r.status, r.read().decode()
        except urllib.error.HTTPError as e:
            return e.code, ""
    try:
        assert get("/healthz") == (200, "ok") and get("/livez")[0] == 200
        assert get("/readyz")[0] == 503                     # informers not synced yet
        s.start_informers()
        assert get("/readyz") == (200, "ok")
        fc.create("pods", O.make_pod("p0", gpu_cu=64))
        s.schedule_pending()
        code, body = get("/metrics")
        assert code == 200 and 'gpusched_pods_scheduled_total{result="scheduled"} 1.0' in body
        assert get("/nope")[0] == 404
    finally:
        stop()
        http.stop()
