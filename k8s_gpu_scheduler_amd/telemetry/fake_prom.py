"""Fake Prometheus HTTP API (instant queries) for tests and local e2e runs.

The reference tests its HTTP client against an `httptest.NewServer` that routes
`/api/v1/query` to a mock returning `{"test":"mock"}` (400 when `query` is missing;
reference pkg/prom/requests/request_test.go:25-39,76-88).  This server supports that mock
mode and a real mode: series are pushed with `set(metric, labels, value)` (or scraped
from a GpuExporter) and `/api/v1/query?query=METRIC{k="v",...}` returns a Prometheus
vector reply filtered by the label matchers (=, !=, =~).
"""
from __future__ import annotations

import json
import re
import threading
import time
from http.server import BaseHTTPRequestHandler, ThreadingHTTPServer
from typing import Dict, List, Optional, Tuple
from urllib.parse import parse_qs, urlsplit

_SEL = re.compile(r'^\s*([a-zA-Z_:][a-zA-Z0-9_:]*)\s*(?:\{(.*)\})?\s*$')
_MATCH = re.compile(r'\s*([a-zA-Z_][a-zA-Z0-9_]*)\s*(=~|!=|=)\s*"((?:[^"\\]|\\.)*)"\s*,?')


def parse_selector(q: str) -> Tuple[str, List[Tuple[str, str, str]]]:
    m = _SEL.match(q)
    if not m:
        raise ValueError(f"unsupported query {q!r}")
    name, body = m.group(1), m.group(2) or ""
    matchers = [(a, op, v) for a, op, v in _MATCH.findall(body)]
    return name, matchers


class FakePrometheus:
    def __init__(self, mock: bool = False, host: str = "127.0.0.1", port: int = 0):
        self.mock = mock
        self.series: Dict[Tuple[str, Tuple[Tuple[str, str], ...]], float] = {}
        self._lock = threading.Lock()
        self.queries: List[str] = []
        outer = self

        class H(BaseHTTPRequestHandler):
            def log_message(self, *a):  # quiet
                pass

            def do_GET(self):
                u = urlsplit(self.path)
                if u.path.strip() != "/api/v1/query":
                    self.send_response(404)
                    self.end_headers()
                    return
                qs = parse_qs(u.query)
                q = (qs.get("query") or [""])[0]
                status, body = outer.handle(q)
                raw = (json.dumps(body) + "\n").encode() if outer.mock else json.dumps(body).encode()
                self.send_response(status)
                self.send_header("Content-Type", "application/json")
                self.send_header("Content-Length", str(len(raw)))
                self.end_headers()
                self.wfile.write(raw)

        self.httpd = ThreadingHTTPServer((host, port), H)
        self.httpd.daemon_threads = True
        self._t: Optional[threading.Thread] = None

    @property
    def url(self) -> str:
        h, p = self.httpd.server_address[:2]
        return f"http://{h}:{p}"

    def start(self) -> "FakePrometheus":
        self._t = threading.Thread(target=self.httpd.serve_forever, daemon=True)
        self._t.start()
        return self

    def stop(self) -> None:
        self.httpd.shutdown()
        self.httpd.server_close()

    def set(self, metric: str, labels: Dict[str, str], value: float) -> None:
        with self._lock:
            self.series[(metric, tuple(sorted(labels.items())))] = float(value)

    def handle(self, q: str):
        self.queries.append(q)
        if self.mock:
            if not q:
                return 400, {}
            return 200, {"test": "mock"}
        if not q:
            return 400, {"status": "error", "errorType": "bad_data", "error": "no query"}
        try:
            name, matchers = parse_selector(q)
        except ValueError as e:
            return 400, {"status": "error", "errorType": "bad_data", "error": str(e)}
        res = []
        now = time.time()
        with self._lock:
            for (m, labs), v in self.series.items():
                if m != name:
                    continue
                ld = dict(labs)
                ok = True
                for k, op, val in matchers:
                    have = ld.get(k, "")
                    if op == "=" and have != val or op == "!=" and have == val or \
                            op == "=~" and not re.fullmatch(val, have):
                        ok = False
                        break
                if ok:
                    met = {"__name__": m, **ld}
                    res.append({"metric": met, "value": [now, repr(v) if not float(v).is_integer() else str(int(v))]})
        return 200, {"status": "success", "data": {"resultType": "vector", "result": res}}

    def ingest_exposition(self, text: str) -> int:
        """Load a Prometheus text exposition (e.g. GpuExporter.render())."""
        n = 0
        for ln in text.splitlines():
            if not ln or ln.startswith("#"):
                continue
            m = re.match(r'^([a-zA-Z_:][a-zA-Z0-9_:]*)(?:\{(.*)\})?\s+(\S+)', ln)
            if not m:
                continue
            labs = dict((a, v) for a, _, v in _MATCH.findall(m.group(2) or ""))
            try:
                self.set(m.group(1), labs, float(m.group(3)))
                n += 1
            except ValueError:
                continue
        return n
