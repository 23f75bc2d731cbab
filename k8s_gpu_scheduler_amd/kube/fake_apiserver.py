"""HTTP front-end over FakeCluster speaking the apiserver REST dialect.

Lets the real `RestClient`, the standalone scheduler process, the node agent and the
extender run end to end against an in-memory cluster (the reference has no fake
apiserver at all -- SURVEY.md §4).  Implements exactly the paths `kube.rest` uses:
collection GET (with label/field selectors and `?watch=1` streaming), item
GET/PUT/PATCH/DELETE, POST create, POST pods/{name}/binding.
"""
from __future__ import annotations

import json
import re
import threading
from http.server import BaseHTTPRequestHandler, ThreadingHTTPServer
from typing import Optional
from urllib.parse import parse_qs, urlsplit

from .client import ApiError, FakeCluster

_CORE = re.compile(r"^/api/v1(?:/namespaces/(?P<ns>[^/]+))?/(?P<res>pods|nodes|configmaps|events|namespaces|"
                   r"persistentvolumeclaims|persistentvolumes|services|replicationcontrollers)"
                   r"(?:/(?P<name>[^/]+))?(?:/(?P<sub>binding|status|eviction))?$")
_COORD = re.compile(r"^/apis/(?:coordination\.k8s\.io|storage\.k8s\.io|apps|policy)/v1(?:/namespaces/(?P<ns>[^/]+))?/"
                    r"(?P<res>leases|storageclasses|csinodes|replicasets|statefulsets|poddisruptionbudgets)"
                    r"(?:/(?P<name>[^/]+))?$")
_PT = {"application/json-patch+json": "json", "application/merge-patch+json": "merge",
       "application/strategic-merge-patch+json": "strategic"}


class FakeApiServer:
    def __init__(self, cluster: Optional[FakeCluster] = None, host: str = "127.0.0.1", port: int = 0,
                 token: str = ""):
        self.cluster = cluster or FakeCluster(sync_watch=False)
        self.token = token
        outer = self

        class H(BaseHTTPRequestHandler):
            protocol_version = "HTTP/1.1"

            def log_message(self, *a):
                pass

            def _send(self, code: int, body) -> None:
                raw = json.dumps(body).encode()
                self.send_response(code)
                self.send_header("Content-Type", "application/json")
                self.send_header("Content-Length", str(len(raw)))
                self.end_headers()
                self.wfile.write(raw)

            def _err(self, e: ApiError) -> None:
                self._send(e.code, {"kind": "Status", "apiVersion": "v1", "status": "Failure",
                                    "message": e.message, "reason": e.reason, "code": e.code})

            def _route(self):
                u = urlsplit(self.path)
                m = _CORE.match(u.path) or _COORD.match(u.path)
                if not m:
                    return None, None
                return m.groupdict(), {k: v[0] for k, v in parse_qs(u.query).items()}

            def _auth(self) -> bool:
                if outer.token and self.headers.get("Authorization") != f"Bearer {outer.token}":
                    self._send(401, {"kind": "Status", "code": 401, "reason": "Unauthorized"})
                    return False
                return True

            def _body(self):
                n = int(self.headers.get("Content-Length") or 0)
                return json.loads(self.rfile.read(n)) if n else None

            def do_GET(self):
                if not self._auth():
                    return
                r, q = self._route()
                if r is None:
                    return self._send(404, {"kind": "Status", "code": 404, "reason": "NotFound"})
                c = outer.cluster
                try:
                    if r["name"]:
                        return self._send(200, c.get(r["res"], r["name"], r["ns"]))
                    if q.get("watch") in ("1", "true"):
                        return self._watch(r, q)
                    items, rv = c.list(r["res"], r["ns"], q.get("labelSelector"), q.get("fieldSelector"))
                    self._send(200, {"kind": "List", "apiVersion": "v1", "metadata": {"resourceVersion": rv},
                                     "items": items})
                except ApiError as e:
                    self._err(e)

            def _watch(self, r, q):
                c = outer.cluster
                try:
                    it = c.watch(r["res"], r["ns"], q.get("resourceVersion", ""),
                                 float(q.get("timeoutSeconds", "30")))
                except ApiError as e:
                    self.send_response(200)
                    self.send_header("Content-Type", "application/json")
                    self.send_header("Transfer-Encoding", "chunked")
                    self.end_headers()
                    self._chunk(json.dumps({"type": "ERROR", "object": {"kind": "Status", "code": e.code,
                                                                         "message": e.message}}).encode() + b"\n")
                    self._chunk(b"")
                    return
                self.send_response(200)
                self.send_header("Content-Type", "application/json")
                self.send_header("Transfer-Encoding", "chunked")
                self.end_headers()
                try:
                    for ev in it:
                        self._chunk(json.dumps({"type": ev["type"], "object": ev["object"]}).encode() + b"\n")
                    self._chunk(b"")
                except (BrokenPipeError, ConnectionResetError):
                    pass

            def _chunk(self, data: bytes) -> None:
                self.wfile.write(b"%x\r\n%s\r\n" % (len(data), data))
                self.wfile.flush()

            def do_POST(self):
                if not self._auth():
                    return
                r, q = self._route()
                if r is None:
                    return self._send(404, {"code": 404})
                body = self._body()
                try:
                    if r.get("sub") == "binding":
                        outer.cluster.bind(r["ns"], r["name"], body["target"]["name"],
                                           body.get("metadata", {}).get("uid", ""),
                                           body.get("metadata", {}).get("annotations"))
                        return self._send(201, {"kind": "Status", "status": "Success", "code": 201})
                    if r.get("sub") == "eviction":
                        outer.cluster.evict(r["ns"], r["name"])
                        return self._send(201, {"kind": "Status", "status": "Success", "code": 201})
                    self._send(201, outer.cluster.create(r["res"], body, r["ns"]))
                except ApiError as e:
                    self._err(e)

            def do_PUT(self):
                if not self._auth():
                    return
                r, q = self._route()
                try:
                    self._send(200, outer.cluster.update(r["res"], self._body(), r["ns"]))
                except ApiError as e:
                    self._err(e)

            def do_PATCH(self):
                if not self._auth():
                    return
                r, q = self._route()
                pt = _PT.get(self.headers.get("Content-Type", ""), "merge")
                try:
                    self._send(200, outer.cluster.patch(r["res"], r["name"], self._body(), pt, r["ns"]))
                except ApiError as e:
                    self._err(e)

            def do_DELETE(self):
                if not self._auth():
                    return
                r, q = self._route()
                self._body()
                try:
                    outer.cluster.delete(r["res"], r["name"], r["ns"])
                    self._send(200, {"kind": "Status", "status": "Success"})
                except ApiError as e:
                    self._err(e)

        self.httpd = ThreadingHTTPServer((host, port), H)
        self.httpd.daemon_threads = True
        self._t: Optional[threading.Thread] = None

    @property
    def url(self) -> str:
        h, p = self.httpd.server_address[:2]
        return f"http://{h}:{p}"

    def start(self) -> "FakeApiServer":
        self._t = threading.Thread(target=self.httpd.serve_forever, daemon=True, name="fake-apiserver")
        self._t.start()
        return self

    def stop(self) -> None:
        self.cluster.close_watches()
        self.httpd.shutdown()
        self.httpd.server_close()

    def kubeconfig(self, path: str) -> str:
        doc = {"apiVersion": "v1", "kind": "Config", "current-context": "fake",
               "clusters": [{"name": "fake", "cluster": {"server": self.url}}],
               "users": [{"name": "fake", "user": {"token": self.token} if self.token else {}}],
               "contexts": [{"name": "fake", "context": {"cluster": "fake", "user": "fake"}}]}
        import yaml
        with open(path, "w") as f:
            yaml.safe_dump(doc, f)
        return path
