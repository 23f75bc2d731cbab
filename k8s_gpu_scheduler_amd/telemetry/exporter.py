"""Prometheus exporter for MI355X telemetry and scheduler metrics.

The reference *consumes* dcgm-exporter series (reference
pkg/prom/fetch_prom_metrics/prom_metrics.go:63-70) and exports nothing of its own
(SURVEY.md §5.5).  This exporter publishes, per GPU (labels `gpu`, `UUID`, `node`,
`pod` = exporter pod name so the reference's `{pod="<exporter>"}` filter works):

  amd_gpu_gfx_activity, amd_gpu_umc_activity  (0..1, DCGM_FI_PROF_GR_ENGINE_ACTIVE /
                                               DCGM_FI_DEV_MEM_COPY_UTIL analogs)
  amd_gpu_temperature_hotspot                 (C,  DCGM_FI_DEV_GPU_TEMP)
  amd_gpu_vram_used_mb / amd_gpu_vram_free_mb (MB, DCGM_FI_DEV_FB_USED / _FREE)
  amd_gpu_power_watts, amd_gpu_xgmi_{tx,rx}_bytes (rate, B/s)
  amd_gpu_ecc_uncorrectable_total, amd_gpu_ecc_correctable_total (accumulated counts)
  amd_gpu_healthy                             (1/0, the agent's health verdict, agent/health.py)

per pod (labels `pod`, `node`): amd_gpu_pod_hbm_used_gib / _cap_gib / amd_gpu_pod_hbm_overuse
(the agent's per-process attribution against the pod's HBM share);

optionally the same values under the DCGM names (`dcgm_compat=True`), and scheduler
series: pods scheduled, scheduling latency histogram, SLO attainment, per-extension-point
latency.
"""
from __future__ import annotations

from typing import Dict, Iterable, Optional

from prometheus_client import CollectorRegistry, Counter, Gauge, Histogram, generate_latest, start_http_server

from ..api import constants as C


class GpuExporter:
    def __init__(self, node: str, exporter_pod: str = "amd-gpu-exporter", dcgm_compat: bool = False,
                 registry: Optional[CollectorRegistry] = None):
        self.node, self.pod, self.dcgm_compat = node, exporter_pod, dcgm_compat
        self.registry = registry or CollectorRegistry()
        lab = ["gpu", "UUID", "node", "pod"]
        self.g: Dict[str, Gauge] = {m: Gauge(m, m, lab, registry=self.registry) for m in C.AMD_METRICS}
        self.dcgm: Dict[str, Gauge] = {}
        if dcgm_compat:
            self.dcgm = {m: Gauge(m, m, lab, registry=self.registry) for m in C.DCGM_METRICS}
        self.sched_pods = Counter("gpusched_pods_scheduled", "pods bound by the scheduler", ["result"],
                                  registry=self.registry)
        self.sched_latency = Histogram("gpusched_scheduling_latency_seconds", "pod scheduling latency",
                                       buckets=(1e-4, 3e-4, 1e-3, 3e-3, 1e-2, 3e-2, 0.1, 0.3, 1, 3),
                                       registry=self.registry)
        self.slo = Gauge("gpusched_slo_attainment", "fraction of pods meeting their SLO", registry=self.registry)
        self.ext = Gauge("gpusched_extension_point_mean_us", "mean latency per extension point", ["point"],
                         registry=self.registry)
        self.plan_level = Gauge("gpusched_plan_effort_level", "burst planner effort level (0 = full)", ["profile"],
                                registry=self.registry)
        self.plan_ms = Gauge("gpusched_plan_ms", "wall time of the last burst plan", ["profile"],
                             registry=self.registry)
        self.ecc = {k: Gauge(f"amd_gpu_ecc_{k}_total", f"accumulated {k} ECC errors", lab, registry=self.registry)
                    for k in ("uncorrectable", "correctable")}
        self.healthy = Gauge("amd_gpu_healthy", "1 if the node agent considers the device healthy", lab,
                             registry=self.registry)
        plab = ["pod", "node"]
        self.pod_hbm = Gauge("amd_gpu_pod_hbm_used_gib", "VRAM held by a pod's processes (amd-smi process list)",
                             plab, registry=self.registry)
        self.pod_hbm_cap = Gauge("amd_gpu_pod_hbm_cap_gib", "the pod's HBM share (amd.com/gpu-memory request)",
                                 plab, registry=self.registry)
        self.pod_overuse = Gauge("amd_gpu_pod_hbm_overuse", "1 if the pod holds more VRAM than its HBM share",
                                 plab, registry=self.registry)

    def observe_samples(self, samples: Iterable[Dict[str, float]], uuids: Dict[int, str]) -> None:
        for s in samples:
            idx = int(s.get("index", 0))
            lv = (str(idx), uuids.get(idx, ""), self.node, self.pod)
            gfx = max(0.0, float(s.get("gfx_activity", 0.0))) / 100.0
            umc = max(0.0, float(s.get("umc_activity", 0.0))) / 100.0
            used = max(0.0, float(s.get("vram_used_mb", 0.0)))
            total = max(used, float(s.get("vram_total_mb", C.MI355X_HBM_GIB * 1024)))
            vals = {"amd_gpu_gfx_activity": gfx, "amd_gpu_umc_activity": umc,
                    "amd_gpu_temperature_hotspot": float(s.get("temp_c", 0.0)),
                    "amd_gpu_vram_used_mb": used, "amd_gpu_vram_free_mb": total - used,
                    "amd_gpu_power_watts": float(s.get("power_w", 0.0)),
                    "amd_gpu_xgmi_tx_bytes": float(s.get("xgmi_write_bps", 0.0)),
                    "amd_gpu_xgmi_rx_bytes": float(s.get("xgmi_read_bps", 0.0))}
            for m, v in vals.items():
                self.g[m].labels(*lv).set(v)
            for k, gauge in self.ecc.items():
                v = float(s.get(f"ecc_{k}", -1))
                if v >= 0:
                    gauge.labels(*lv).set(v)
            if self.dcgm:
                for dm, am in C.DCGM_TO_AMD.items():
                    self.dcgm[dm].labels(*lv).set(vals[am])

    def observe_pod_hbm(self, pod: str, used_gib: float, cap_gib: float, tolerance_gib: float = 0.25) -> None:
        self.pod_hbm.labels(pod, self.node).set(used_gib)
        self.pod_hbm_cap.labels(pod, self.node).set(cap_gib)
        self.pod_overuse.labels(pod, self.node).set(1.0 if cap_gib > 0 and used_gib > cap_gib + tolerance_gib else 0.0)

    def observe_health(self, healthy: Dict[int, bool], uuids: Dict[int, str]) -> None:
        for idx, ok in healthy.items():
            self.healthy.labels(str(idx), uuids.get(idx, ""), self.node, self.pod).set(1.0 if ok else 0.0)

    def observe_scheduler(self, scheduled: int = 0, failed: int = 0, latencies=(), slo: Optional[float] = None,
                          ext: Optional[Dict[str, Dict[str, float]]] = None) -> None:
        if scheduled:
            self.sched_pods.labels("scheduled").inc(scheduled)
        if failed:
            self.sched_pods.labels("unschedulable").inc(failed)
        for l in latencies:
            self.sched_latency.observe(l)
        if slo is not None:
            self.slo.set(slo)
        for p, d in (ext or {}).items():
            self.ext.labels(p).set(d.get("mean_us", 0.0))

    def observe_planner(self, profile: str, level: int, plan_ms: Optional[float]) -> None:
        self.plan_level.labels(profile).set(level)
        if plan_ms is not None:
            self.plan_ms.labels(profile).set(plan_ms)

    def render(self) -> bytes:
        return generate_latest(self.registry)

    def serve(self, port: int = 9400, addr: str = "0.0.0.0") -> None:
        start_http_server(port, addr, registry=self.registry)


def observe_planner(exporter: "GpuExporter", profile: str, fw) -> None:
    """The GPU plugin's burst-planner effort level and last plan time (if it has a planner)."""
    try:
        plugin = fw.plugin(C.PLUGIN_NAME)
    except Exception:
        return
    pl = getattr(plugin, "planner", None)
    if pl is not None:
        exporter.observe_planner(profile, pl.effort, pl.stats.get("plan_ms_last"))


def attach_scheduler_metrics(exporter: "GpuExporter", sched, period_s: float = 5.0):
    """Feed a Scheduler's results into the exporter's scheduler series: every result
    (bound / unschedulable, latency) as it happens, per-extension-point mean latency every
    `period_s`.  Returns a stop() callable."""
    import threading
    prev = sched.on_result

    def on_result(res):
        if res.status.ok and res.node:
            exporter.observe_scheduler(scheduled=1, latencies=(res.latency_s,))
        else:
            exporter.observe_scheduler(failed=1, latencies=(res.latency_s,))
        if prev is not None:
            prev(res)
    sched.on_result = on_result
    stop = threading.Event()

    def loop():
        while not stop.wait(period_s):
            ext = {}
            for name, fw in sched.frameworks.items():
                ext.update(fw.metrics.summary())
                observe_planner(exporter, name, fw)
            exporter.observe_scheduler(ext=ext)
    threading.Thread(target=loop, daemon=True, name="sched-metrics").start()
    return stop.set


class SchedulerHTTP:
    """The scheduler's HTTP endpoint (kube-scheduler serves the same paths): /metrics (the
    exporter's registry), /healthz and /livez (200 while the process serves; 500 once the
    scheduling loop that was started has died), /readyz (200 once the informer caches have
    synced and, under leader election, this replica leads or stands by -- 503 before)."""

    def __init__(self, exporter: "GpuExporter", sched, port: int, addr: str = "0.0.0.0"):
        import threading
        from http.server import BaseHTTPRequestHandler, ThreadingHTTPServer
        outer = self
        self.exporter, self.sched = exporter, sched

        class H(BaseHTTPRequestHandler):
            def log_message(self, *a):
                pass

            def do_GET(self):
                path = self.path.split("?", 1)[0].rstrip("/")
                if path == "/metrics":
                    code, ctype, body = 200, "text/plain; version=0.0.4", outer.exporter.render()
                elif path in ("/healthz", "/livez", "/readyz"):
                    ok = outer.ready() if path == "/readyz" else outer.alive()
                    code, ctype, body = (200 if ok else (503 if path == "/readyz" else 500)), "text/plain", \
                        (b"ok" if ok else b"not ok")
                else:
                    code, ctype, body = 404, "text/plain", b"not found"
                self.send_response(code)
                self.send_header("Content-Type", ctype)
                self.send_header("Content-Length", str(len(body)))
                self.end_headers()
                self.wfile.write(body)
        self.server = ThreadingHTTPServer((addr, port), H)
        self.port = self.server.server_address[1]
        self._thread = threading.Thread(target=self.server.serve_forever, daemon=True, name="sched-http")

    def alive(self) -> bool:
        t = getattr(self.sched, "_thread", None)
        stopped = getattr(self.sched, "_stop", None)
        return t is None or t.is_alive() or (stopped is not None and stopped.is_set())

    def ready(self) -> bool:
        return bool(getattr(self.sched, "_started", False)) and self.alive()

    def start(self) -> "SchedulerHTTP":
        self._thread.start()
        return self

    def stop(self) -> None:
        self.server.shutdown()
        self.server.server_close()
