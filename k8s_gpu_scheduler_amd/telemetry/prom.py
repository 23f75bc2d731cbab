"""Prometheus HTTP query client.

Same behaviour as the reference's `requests.Requests` and `metrics.ParseResponse` /
`DcgmPromInstantQuery` (reference pkg/prom/requests/metrics_request.go:18-88,
pkg/prom/fetch_prom_metrics/prom_metrics.go:14-118):

* `create_url(base, path, params)` joins the path and appends `?k=v&k2=v2` (the reference
  does not URL-escape PromQL; here values ARE escaped -- a `{pod="x"}` filter otherwise
  produces an invalid URL);
* `Requests.request` issues a GET with a timeout (1 s default) and returns the body, or
  raises `ResponseNotOK` on non-200;
* `parse_response` turns a Prometheus vector reply into `Response` rows
  (metric name, exporter pod, value string, GPU_I_ID, UUID); empty body or empty result
  -> None;
* `instant_query(url, filter)` fans the metric queries out concurrently and concatenates
  the parsed rows (the reference's 5 goroutines).  AMD series names are queried by
  default; `metrics=DCGM_METRICS` reproduces the reference's query set.
"""
from __future__ import annotations

import json
import urllib.error
import urllib.parse
import urllib.request
from concurrent.futures import ThreadPoolExecutor
from dataclasses import dataclass, field
from typing import Dict, List, Optional, Sequence

from ..api import constants as C


class ResponseNotOK(Exception):
    def __init__(self, status: int, text: str = ""):
        super().__init__(f"response not ok. {status} {text}")
        self.status = status


@dataclass
class Response:
    metric_name: str = ""
    exporter: str = ""
    value: str = ""
    gpu_i_id: str = ""
    uuid: str = ""
    # every label of the series and the sample's unix timestamp (the reference keeps only
    # the five fields above; the scheduler's poller also needs `node`/`gpu` and the age)
    labels: Dict[str, str] = field(default_factory=dict, compare=False, repr=False)
    ts: float = field(default=0.0, compare=False, repr=False)


def create_url(base_url: str, upath: str, params: Dict[str, str]) -> str:
    u = urllib.parse.urlsplit(base_url)
    path = "/".join(p.strip("/") for p in (u.path, upath) if p.strip("/"))
    url = urllib.parse.urlunsplit((u.scheme, u.netloc, "/" + path, "", ""))
    if params:
        url += "?" + urllib.parse.urlencode(params)
    return url


class Requests:
    def __init__(self, base_url: str, timeout_s: float = C.PROM_TIMEOUT_S):
        self.base_url, self.timeout_s = base_url, timeout_s

    def request(self, upath: str, params: Dict[str, str]) -> bytes:
        url = create_url(self.base_url, upath, params)
        try:
            with urllib.request.urlopen(url, timeout=self.timeout_s) as r:
                if r.status != 200:
                    raise ResponseNotOK(r.status)
                return r.read()
        except urllib.error.HTTPError as e:
            raise ResponseNotOK(e.code, e.reason) from None


def parse_response(body: Optional[bytes]) -> Optional[List[Response]]:
    if not body:
        return None
    doc = json.loads(body)
    results = doc["data"]["result"]
    if not results:
        return None
    out = []
    for r in results:
        m = r["metric"]
        out.append(Response(metric_name=m["__name__"], exporter=m.get("pod", ""), value=str(r["value"][1]),
                            gpu_i_id=m.get("GPU_I_ID", ""), uuid=m.get("UUID", ""), labels=dict(m),
                            ts=float(r["value"][0])))
    return out


def instant_query(url: str, filter_: str = "", metrics: Sequence[str] = tuple(C.AMD_METRICS[:5]),
                  timeout_s: float = C.PROM_TIMEOUT_S) -> List[Response]:
    req = Requests(url, timeout_s)

    def one(metric: str) -> List[Response]:
        try:
            return parse_response(req.request("api/v1/query", {"query": metric + filter_})) or []
        except Exception:
            return []          # the reference logs and skips failed queries
    with ThreadPoolExecutor(len(metrics) or 1) as ex:
        parts = list(ex.map(one, metrics))
    return [r for p in parts for r in p]


def dcgm_prom_instant_query(url: str, filter_: str = "") -> List[Response]:
    """Reference-compatible query set (DCGM series names)."""
    return instant_query(url, filter_, C.DCGM_METRICS)


def metrics_by_device(responses: List[Response], uuids: Optional[List[str]] = None) -> Dict[str, Dict[str, float]]:
    """{uuid-or-GPU_I_ID: {metric: value}} like GetDcgmMetricsForNode
    (reference gpu_plugins.go:279-299)."""
    out: Dict[str, Dict[str, float]] = {}
    for r in responses:
        k = r.gpu_i_id or r.uuid
        try:
            out.setdefault(k, {})[r.metric_name] = float(r.value)
        except ValueError:
            continue
    return out
