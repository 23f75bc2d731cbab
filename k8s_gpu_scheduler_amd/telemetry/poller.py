"""Scheduler-side live telemetry: poll the node agents' GPU series into the TelemetryCache.

The reference scheduler reads DCGM series through Prometheus (`DcgmPromInstantQuery`: five
concurrent instant queries, 1 s timeout; reference
pkg/prom/fetch_prom_metrics/prom_metrics.go:63-118, called from
pkg/plugins/gpu_plugin/gpu_plugins.go:162-300) -- synchronously, inside Score.  Here a
background thread of the scheduler process does the reading, so Score stays free of I/O:

  * `PromSource`   -- the same instant queries against Prometheus (`telemetry.prom`), AMD
                      series names (`amd_gpu_*`, published by the agents' exporter), one query
                      per metric fanned out concurrently, grouped by the `node` / `UUID` labels;
  * `ScrapeSource` -- no Prometheus in between: scrape the agents' `/metrics` endpoints
                      directly (Prometheus text format).

Every poll turns each (node, UUID) into a `DeviceSample` (gfx/umc activity, VRAM used/total,
power, temperature, xGMI tx/rx) stamped with the series' own age, so the cache's `stale_s`
drops data from an agent that stopped reporting and the GPU plugin degrades to
prediction/packing-only scoring during a telemetry outage.
"""
from __future__ import annotations

import logging
import threading
import time
import urllib.request
from typing import Callable, Dict, Iterable, List, Optional, Sequence, Tuple

from ..api import constants as C
from .cache import DeviceSample, TelemetryCache

log = logging.getLogger(__name__)

# (metric name, labels, value, age in seconds)
Series = Tuple[str, Dict[str, str], float, float]

_FIELDS = {"amd_gpu_gfx_activity": "gfx_activity", "amd_gpu_umc_activity": "umc_activity",
           "amd_gpu_vram_used_mb": "vram_used_mb", "amd_gpu_power_watts": "power_w",
           "amd_gpu_temperature_hotspot": "temp_c", "amd_gpu_xgmi_tx_bytes": "xgmi_tx_bps",
           "amd_gpu_xgmi_rx_bytes": "xgmi_rx_bps"}


class PromSource:
    """Instant queries against a Prometheus server (reference query path, AMD names)."""

    def __init__(self, url: str, timeout_s: float = C.PROM_TIMEOUT_S, metrics: Sequence[str] = tuple(C.AMD_METRICS),
                 selector: str = ""):
        self.url, self.timeout_s, self.metrics, self.selector = url, timeout_s, tuple(metrics), selector

    def fetch(self) -> List[Series]:
        from .prom import instant_query
        now = time.time()
        out = []
        for r in instant_query(self.url, self.selector, self.metrics, self.timeout_s):
            try:
                v = float(r.value)
            except ValueError:
                continue
            out.append((r.metric_name, r.labels, v, max(0.0, now - r.ts) if r.ts else 0.0))
        return out


class ScrapeSource:
    """Direct scrape of exporter endpoints (`http://<agent>:9400/metrics`)."""

    def __init__(self, urls: Callable[[], Iterable[str]] | Sequence[str], timeout_s: float = C.PROM_TIMEOUT_S):
        self._urls = urls
        self.timeout_s = timeout_s

    def urls(self) -> List[str]:
        return list(self._urls() if callable(self._urls) else self._urls)

    def fetch(self) -> List[Series]:
        from prometheus_client.parser import text_string_to_metric_families
        out: List[Series] = []
        for u in self.urls():
            try:
                with urllib.request.urlopen(u, timeout=self.timeout_s) as r:
                    txt = r.read().decode()
            except Exception as e:
                log.debug("scrape %s failed: %s", u, e)
                continue
            for fam in text_string_to_metric_families(txt):
                for smp in fam.samples:
                    if smp.name in _FIELDS or smp.name == "amd_gpu_vram_free_mb":
                        out.append((smp.name, dict(smp.labels), float(smp.value), 0.0))
        return out


def samples_from_series(series: Iterable[Series]) -> Dict[Tuple[str, str], Tuple[DeviceSample, float]]:
    """{(node, UUID): (sample, age_s)}; series without a node or UUID label are skipped."""
    acc: Dict[Tuple[str, str], Dict[str, float]] = {}
    ages: Dict[Tuple[str, str], float] = {}
    for name, labels, value, age in series:
        node, uuid = labels.get("node", ""), labels.get("UUID", "")
        if not node or not uuid:
            continue
        k = (node, uuid)
        acc.setdefault(k, {})[name] = value
        ages[k] = max(ages.get(k, 0.0), age)
    out = {}
    for k, m in acc.items():
        if "amd_gpu_gfx_activity" not in m and "amd_gpu_vram_used_mb" not in m:
            continue
        kw = {f: m[n] for n, f in _FIELDS.items() if n in m}
        used = m.get("amd_gpu_vram_used_mb", 0.0)
        if "amd_gpu_vram_free_mb" in m:
            kw["vram_total_mb"] = used + m["amd_gpu_vram_free_mb"]
        out[k] = (DeviceSample(**kw), ages.get(k, 0.0))
    return out


class TelemetryPoller:
    """Background thread: every `period_s`, fetch from `source` into `cache`.

    A failed or empty poll leaves the cache untouched; samples then age out after the
    cache's `stale_s`, which is how an outage degrades Score (never an exception in it)."""

    def __init__(self, cache: TelemetryCache, source, period_s: float = 2.0):
        self.cache, self.source, self.period_s = cache, source, period_s
        self.polls = self.failures = 0
        self.last_ok = 0.0
        self.last_count = 0
        self._stop = threading.Event()
        self._thread: Optional[threading.Thread] = None

    def poll_once(self) -> int:
        self.polls += 1
        try:
            series = self.source.fetch()
        except Exception as e:
            self.failures += 1
            log.debug("telemetry poll failed: %s", e)
            return 0
        got = samples_from_series(series)
        now = time.monotonic()
        for (node, uuid), (smp, age) in got.items():
            smp.ts = now - age
            self.cache.update(node, uuid, smp)
        if got:
            self.last_ok = time.time()
        else:
            self.failures += 1
        self.last_count = len(got)
        return len(got)

    def run(self) -> None:
        while not self._stop.is_set():
            self.poll_once()
            self._stop.wait(self.period_s)

    def start(self) -> "TelemetryPoller":
        self._thread = threading.Thread(target=self.run, daemon=True, name="telemetry-poller")
        self._thread.start()
        return self

    def stop(self) -> None:
        self._stop.set()
        if self._thread is not None:
            self._thread.join(timeout=5)


def make_source(prometheus: str = "", scrape: str = "", timeout_s: float = C.PROM_TIMEOUT_S):
    """`scrape` (comma-separated exporter URLs) wins over `prometheus` (server URL)."""
    if scrape:
        return ScrapeSource([u.strip() for u in scrape.split(",") if u.strip()], timeout_s)
    if prometheus:
        return PromSource(prometheus, timeout_s)
    return None
