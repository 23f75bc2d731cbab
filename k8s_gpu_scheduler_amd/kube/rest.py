"""REST client for a real Kubernetes apiserver (in-cluster service account or kubeconfig).

The reference uses client-go (`rest.InClusterConfig` / `clientcmd.BuildConfigFromFlags`,
reference pkg/resources/pods.go:182-212, utils/utils.go:110-122).  The Python
`kubernetes` package is not available, so the handful of core/v1 + coordination/v1
endpoints the scheduler needs are spoken directly: list/get/create/update/patch
(json-patch, merge-patch, strategic-merge-patch)/delete, pods/binding, and streaming
watches (`?watch=1&resourceVersion=`), with HTTP status -> ApiError mapping
(404 NotFound, 409 Conflict/AlreadyExists, 410 Gone).
"""
from __future__ import annotations

import base64
import json
import os
import ssl
import tempfile
import urllib.error
import urllib.parse
import urllib.request
from dataclasses import dataclass
from typing import Any, Dict, Iterator, Optional

import yaml

from .client import AlreadyExists, ApiError, Conflict, Gone, KubeClient, NotFound, TooManyRequests, WatchEvent

Obj = Dict[str, Any]
SA_DIR = "/var/run/secrets/kubernetes.io/serviceaccount"

GROUP_PATH = {"pods": "/api/v1", "nodes": "/api/v1", "configmaps": "/api/v1", "events": "/api/v1",
              "namespaces": "/api/v1", "leases": "/apis/coordination.k8s.io/v1",
              "persistentvolumeclaims": "/api/v1", "persistentvolumes": "/api/v1",
              "storageclasses": "/apis/storage.k8s.io/v1", "csinodes": "/apis/storage.k8s.io/v1",
              "services": "/api/v1", "replicationcontrollers": "/api/v1", "replicasets": "/apis/apps/v1",
              "statefulsets": "/apis/apps/v1", "poddisruptionbudgets": "/apis/policy/v1"}
CLUSTER_SCOPED = {"nodes", "namespaces", "persistentvolumes", "storageclasses", "csinodes"}
PATCH_CT = {"json": "application/json-patch+json", "merge": "application/merge-patch+json",
            "strategic": "application/strategic-merge-patch+json"}


@dataclass
class RestConfig:
    host: str
    token: str = ""
    ca_file: str = ""
    cert_file: str = ""
    key_file: str = ""
    insecure: bool = False
    timeout_s: float = 10.0

    @classmethod
    def in_cluster(cls) -> "RestConfig":
        h, p = os.environ.get("KUBERNETES_SERVICE_HOST"), os.environ.get("KUBERNETES_SERVICE_PORT")
        if not h or not p:
            raise RuntimeError("not running in a cluster (KUBERNETES_SERVICE_HOST/PORT unset)")
        with open(os.path.join(SA_DIR, "token")) as f:
            tok = f.read().strip()
        host = f"https://[{h}]:{p}" if ":" in h else f"https://{h}:{p}"
        return cls(host, tok, os.path.join(SA_DIR, "ca.crt"))

    @classmethod
    def from_kubeconfig(cls, path: str, context: Optional[str] = None) -> "RestConfig":
        with open(os.path.expanduser(path)) as f:
            kc = yaml.safe_load(f)
        ctx_name = context or kc.get("current-context")
        ctx = next(c["context"] for c in kc["contexts"] if c["name"] == ctx_name)
        cluster = next(c["cluster"] for c in kc["clusters"] if c["name"] == ctx["cluster"])
        user = next((u["user"] for u in kc.get("users", []) if u["name"] == ctx.get("user")), {}) or {}

        def materialise(data_key: str, file_key: str, src: Dict[str, Any]) -> str:
            if src.get(file_key):
                return src[file_key]
            if src.get(data_key):
                fd, p = tempfile.mkstemp(prefix="kc-")
                with os.fdopen(fd, "wb") as out:
                    out.write(base64.b64decode(src[data_key]))
                return p
            return ""
        return cls(host=cluster["server"], token=user.get("token", ""),
                   ca_file=materialise("certificate-authority-data", "certificate-authority", cluster),
                   cert_file=materialise("client-certificate-data", "client-certificate", user),
                   key_file=materialise("client-key-data", "client-key", user),
                   insecure=bool(cluster.get("insecure-skip-tls-verify")))


def _raise_for(code: int, body: bytes) -> None:
    msg = body.decode(errors="replace")[:500]
    try:
        reason = json.loads(body).get("reason", "")
    except Exception:
        reason = ""
    if code == 404:
        raise NotFound(msg)
    if code == 409:
        raise AlreadyExists(msg) if reason == "AlreadyExists" else Conflict(msg)
    if code == 410:
        raise Gone(msg)
    if code == 429:
        raise TooManyRequests(msg)
    raise ApiError(code, reason or "Error", msg)


class RestClient(KubeClient):
    def __init__(self, cfg: RestConfig):
        self.cfg = cfg
        ctx = None
        if cfg.host.startswith("https"):
            ctx = ssl.create_default_context(cafile=cfg.ca_file or None)
            if cfg.insecure:
                ctx.check_hostname = False
                ctx.verify_mode = ssl.CERT_NONE
            if cfg.cert_file:
                ctx.load_cert_chain(cfg.cert_file, cfg.key_file or None)
        self._ctx = ctx

    @classmethod
    def auto(cls, kubeconfig: str = "") -> "RestClient":
        if kubeconfig:
            return cls(RestConfig.from_kubeconfig(kubeconfig))
        try:
            return cls(RestConfig.in_cluster())
        except Exception:
            return cls(RestConfig.from_kubeconfig(os.environ.get("KUBECONFIG", "~/.kube/config")))

    # ------------------------------------------------------------------ plumbing
    def _path(self, resource: str, namespace: Optional[str], name: str = "", sub: str = "") -> str:
        base = GROUP_PATH[resource]
        if resource in CLUSTER_SCOPED or namespace is None:
            p = f"{base}/{resource}"
        else:
            p = f"{base}/namespaces/{urllib.parse.quote(namespace)}/{resource}"
        if name:
            p += "/" + urllib.parse.quote(name)
        if sub:
            p += "/" + sub
        return p

    def _req(self, method: str, path: str, body: Any = None, ctype: str = "application/json",
             query: Optional[Dict[str, str]] = None, timeout: Optional[float] = None):
        url = self.cfg.host.rstrip("/") + path
        if query:
            url += "?" + urllib.parse.urlencode(query)
        data = None if body is None else json.dumps(body).encode()
        rq = urllib.request.Request(url, data=data, method=method)
        rq.add_header("Accept", "application/json")
        if data is not None:
            rq.add_header("Content-Type", ctype)
        if self.cfg.token:
            rq.add_header("Authorization", f"Bearer {self.cfg.token}")
        try:
            return urllib.request.urlopen(rq, timeout=timeout or self.cfg.timeout_s, context=self._ctx)
        except urllib.error.HTTPError as e:
            _raise_for(e.code, e.read())

    def _json(self, *a, **kw) -> Obj:
        with self._req(*a, **kw) as r:
            raw = r.read()
        return json.loads(raw) if raw else {}

    # ------------------------------------------------------------------ KubeClient
    def list(self, resource, namespace=None, label_selector=None, field_selector=None):
        q = {}
        if label_selector:
            q["labelSelector"] = label_selector if isinstance(label_selector, str) else ",".join(
                f"{k}={v}" for k, v in (label_selector.get("matchLabels") or {}).items())
        if field_selector:
            q["fieldSelector"] = field_selector
        doc = self._json("GET", self._path(resource, namespace), query=q)
        from .client import KIND_OF
        kind = KIND_OF[resource]
        items = doc.get("items") or []
        for it in items:
            it.setdefault("kind", kind)
        return items, doc.get("metadata", {}).get("resourceVersion", "")

    def get(self, resource, name, namespace=None):
        return self._json("GET", self._path(resource, namespace or "default", name))

    def create(self, resource, obj, namespace=None):
        ns = namespace or obj.get("metadata", {}).get("namespace") or "default"
        return self._json("POST", self._path(resource, ns), obj)

    def update(self, resource, obj, namespace=None):
        md = obj.get("metadata", {})
        ns = namespace or md.get("namespace") or "default"
        return self._json("PUT", self._path(resource, ns, md["name"]), obj)

    def patch(self, resource, name, patch, patch_type="json", namespace=None):
        return self._json("PATCH", self._path(resource, namespace or "default", name), patch, PATCH_CT[patch_type])

    def delete(self, resource, name, namespace=None, grace_period_seconds=None):
        body = None if grace_period_seconds is None else {"kind": "DeleteOptions", "apiVersion": "v1",
                                                           "gracePeriodSeconds": grace_period_seconds}
        self._json("DELETE", self._path(resource, namespace or "default", name), body)

    def bind(self, namespace, pod_name, node_name, pod_uid="", annotations=None):
        md = {"name": pod_name, "namespace": namespace}
        if pod_uid:
            md["uid"] = pod_uid
        if annotations:
            md["annotations"] = dict(annotations)
        body = {"apiVersion": "v1", "kind": "Binding", "metadata": md,
                "target": {"apiVersion": "v1", "kind": "Node", "name": node_name}}
        self._json("POST", self._path("pods", namespace, pod_name, "binding"), body)

    def evict(self, namespace, pod_name, grace_period_seconds=None):
        body = {"apiVersion": "policy/v1", "kind": "Eviction", "metadata": {"name": pod_name, "namespace": namespace}}
        if grace_period_seconds is not None:
            body["deleteOptions"] = {"gracePeriodSeconds": grace_period_seconds}
        self._json("POST", self._path("pods", namespace, pod_name, "eviction"), body)

    def watch(self, resource, namespace=None, resource_version="", timeout_s=None):
        q = {"watch": "1", "allowWatchBookmarks": "true"}
        if resource_version:
            q["resourceVersion"] = resource_version
        if timeout_s:
            q["timeoutSeconds"] = str(max(1, int(timeout_s)))
        resp = self._req("GET", self._path(resource, namespace), query=q,
                         timeout=(timeout_s or 300) + 5)

        def it() -> Iterator[WatchEvent]:
            with resp:
                for line in resp:
                    line = line.strip()
                    if not line:
                        continue
                    ev = json.loads(line)
                    if ev.get("type") == "ERROR":
                        st = ev.get("object") or {}
                        if st.get("code") == 410:
                            raise Gone(st.get("message", ""))
                    yield WatchEvent(type=ev.get("type"), object=ev.get("object"))
        return it()
