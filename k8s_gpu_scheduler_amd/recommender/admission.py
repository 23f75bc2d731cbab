"""Request right-sizing at admission: the resize loop of BASELINE config 5.

Pods' GPU requests are rewritten when they are CREATED -- requests of a running pod are
immutable, which is why Kubernetes' Vertical Pod Autoscaler also resizes through a mutating
admission webhook.  The loop:

  node agent / executor --samples--> Redis history (per workload, `schema.history_key`)
  pod CREATE --> ResizeAdmission.mutate --> recommend() (recommender.resize) over that
  history + the configuration predictions --> new amd.com/gpu-cu / amd.com/gpu-memory
  requests (and limits, when the pod had them: QoS class is preserved) + the
  `gpu-scheduler.amd.com/resized-request` annotation recording from/to/reason.

History is keyed by WORKLOAD, not pod: a new pod has no history of its own, so it inherits
what earlier pods of the same workload measured (the same catalog-name substring rule the
recommender uses for its rows, reference recom_server.py:67-71; an explicit
`gpu-scheduler.amd.com/workload` annotation wins).

Front-ends: `FakeCluster.add_admission("pods", ResizeAdmission(...))` (in-process, tests and
bench), and `webhook_handler` -- an AdmissionReview v1 (admission.k8s.io/v1) JSON handler
returning a base64 JSONPatch -- for a real apiserver's MutatingWebhookConfiguration.
The reference has no resize path.
"""
from __future__ import annotations

import base64
import json
import logging
from typing import Any, Callable, Dict, List, Optional, Tuple

from ..api import constants as C
from ..api import objects as O
from ..store import schema
from .resize import ResizeAdvice, recommend

log = logging.getLogger(__name__)
Obj = Dict[str, Any]
ANNOT_RESIZE_OPT = C.ANNOT_PREFIX + "resize"          # "off" opts a pod out


def workload_key(pod: Obj) -> str:
    ann = O.annotations(pod).get(C.ANNOT_WORKLOAD)
    if ann:
        return ann
    try:
        from ..models.workloads import workload_for_pod
        return workload_for_pod(O.name(pod)).name
    except KeyError:
        return O.name(pod)


class RedisHistory:
    """Per-workload sample store on the agent's Redis (`gpusched:hist:<workload>`)."""

    def __init__(self, redis: Any, keep: int = 256):
        self.redis, self.keep = redis, keep

    def append(self, workload: str, sample: Dict[str, Any]) -> None:
        schema.append_history(self.redis, workload, sample, keep=self.keep)

    def read(self, workload: str) -> List[Dict[str, Any]]:
        return schema.read_history(self.redis, workload, last=self.keep)


class ResizeAdmission:
    def __init__(self, history: Callable[[str], List[Dict[str, Any]]],
                 predictions: Optional[Callable[[str], Optional[Dict[str, float]]]] = None,
                 model: str = C.MI355X, min_samples: int = 3, shrink_only: bool = False,
                 slo_margin: float = 0.15):
        self.history = history
        self.predictions = predictions
        self.model = model
        self.min_samples = min_samples
        self.shrink_only = shrink_only
        # headroom over the SLO for co-runner interference (a share's throughput is
        # profiled or observed, but the next pod may land beside a heavier neighbour)
        self.slo_margin = slo_margin
        self.stats = {"seen": 0, "resized": 0, "cu_before": 0, "cu_after": 0}

    def advise(self, pod: Obj) -> Optional[ResizeAdvice]:
        g, cu, mem = O.gpu_request(pod, cached=False)
        if g or cu <= 0 or O.annotations(pod).get(ANNOT_RESIZE_OPT, "") == "off":
            return None                     # whole-GPU and non-GPU pods are not resized
        key = workload_key(pod)
        conf = None
        if self.predictions is not None:
            try:
                conf = self.predictions(O.name(pod))
            except Exception as e:
                log.debug("predictions for %s unavailable: %s", key, e)
        adv = recommend(self.history(key), cu, mem, O.pod_slo(pod), conf, self.model,
                        slo_margin=self.slo_margin, min_samples=self.min_samples)
        if self.shrink_only and adv.cu > cu:
            adv = ResizeAdvice(cu, adv.hbm_gib, adv.samples, adv.reason + " (shrink only)")
        return adv

    def patch_ops(self, pod: Obj) -> Tuple[List[Dict[str, Any]], Optional[ResizeAdvice]]:
        """JSONPatch (RFC 6902) ops that apply the advice to the pod's first container."""
        adv = self.advise(pod)
        self.stats["seen"] += 1
        if adv is None:
            return [], None
        g, cu, mem = O.gpu_request(pod, cached=False)
        self.stats["cu_before"] += cu
        self.stats["cu_after"] += adv.cu
        if adv.cu == cu and (adv.hbm_gib == mem or not mem):
            return [], adv
        ctr = (O.containers(pod) or [{}])[0]
        res = ctr.get("resources") or {}
        ops: List[Dict[str, Any]] = []
        if "resources" not in ctr:
            ops.append({"op": "add", "path": "/spec/containers/0/resources", "value": {}})
        for section in ("requests", "limits"):
            cur = res.get(section)
            if section == "limits" and (cur is None or C.RESOURCE_GPU_CU not in cur):
                continue                    # Burstable stays Burstable
            if cur is None:
                ops.append({"op": "add", "path": f"/spec/containers/0/resources/{section}", "value": {}})
            base = f"/spec/containers/0/resources/{section}/"
            ops.append({"op": "add", "path": base + C.RESOURCE_GPU_CU.replace("/", "~1"), "value": str(adv.cu)})
            if mem or section == "requests":
                ops.append({"op": "add", "path": base + C.RESOURCE_GPU_MEM.replace("/", "~1"),
                            "value": O.format_quantity(adv.hbm_gib)})
        note = json.dumps({"from": {"cu": cu, "hbm_gib": mem}, "to": {"cu": adv.cu, "hbm_gib": adv.hbm_gib},
                           "samples": adv.samples, "reason": adv.reason}, separators=(",", ":"))
        if not O.annotations(pod):
            ops.append({"op": "add", "path": "/metadata/annotations", "value": {}})
        ops.append({"op": "add", "path": "/metadata/annotations/" + C.ANNOT_RESIZED.replace("/", "~1"), "value": note})
        self.stats["resized"] += 1
        return ops, adv

    def mutate(self, pod: Obj) -> Obj:
        """In-process admission (FakeCluster hook): returns the mutated pod."""
        from ..kube.patch import apply_json_patch
        ops, _ = self.patch_ops(pod)
        if not ops:
            return pod
        O.forget_requests(pod)
        return apply_json_patch(pod, ops)

    __call__ = mutate


def webhook_handler(adm: Any, review: Dict[str, Any]) -> Dict[str, Any]:
    """admission.k8s.io/v1 AdmissionReview in -> AdmissionReview out (JSONPatch)."""
    req = review.get("request") or {}
    uid = req.get("uid", "")
    resp: Dict[str, Any] = {"uid": uid, "allowed": True}
    try:
        if req.get("kind", {}).get("kind") == "Pod" and req.get("operation", "CREATE") == "CREATE":
            ops, adv = adm.patch_ops(req.get("object") or {})
            if ops:
                resp["patchType"] = "JSONPatch"
                resp["patch"] = base64.b64encode(json.dumps(ops).encode()).decode()
    except Exception as e:  # never block pod creation on a recommender problem
        log.warning("resize admission failed open: %s", e)
        resp["warnings"] = [f"gpu resize skipped: {e}"]
    return {"apiVersion": "admission.k8s.io/v1", "kind": "AdmissionReview", "response": resp}


class AdmissionServer:
    """HTTP(S) front-end for `webhook_handler` (POST /mutate).  The apiserver only calls
    webhooks over TLS: pass certfile/keyfile (the deploy manifest mounts them from a
    Secret); plain HTTP is for tests and local runs."""

    def __init__(self, adm: Any, host: str = "0.0.0.0", port: int = 8443,
                 certfile: str = "", keyfile: str = "", routes: Optional[Dict[str, Any]] = None):
        # POST /mutate -> adm; extra paths -> their own admission (anything with patch_ops)
        paths = {"/mutate": adm, **(routes or {})}
        import threading
        from http.server import BaseHTTPRequestHandler, ThreadingHTTPServer

        class H(BaseHTTPRequestHandler):
            protocol_version = "HTTP/1.1"

            def log_message(self, *a):
                pass

            def _send(self, code: int, body: bytes, ctype: str = "application/json") -> None:
                self.send_response(code)
                self.send_header("Content-Type", ctype)
                self.send_header("Content-Length", str(len(body)))
                self.end_headers()
                self.wfile.write(body)

            def do_GET(self):
                if self.path.rstrip("/") in ("/healthz", "/readyz"):
                    self._send(200, b"ok", "text/plain")
                else:
                    self._send(404, b"")

            def do_POST(self):
                target = paths.get(self.path.rstrip("/"))
                if target is None:
                    self._send(404, b"")
                    return
                n = int(self.headers.get("Content-Length") or 0)
                try:
                    review = json.loads(self.rfile.read(n) or b"{}")
                    self._send(200, json.dumps(webhook_handler(target, review)).encode())
                except json.JSONDecodeError as e:
                    self._send(400, json.dumps({"error": str(e)}).encode())

        self.httpd = ThreadingHTTPServer((host, port), H)
        self.httpd.daemon_threads = True
        self.tls = bool(certfile)
        if certfile:
            import ssl
            ctx = ssl.SSLContext(ssl.PROTOCOL_TLS_SERVER)
            ctx.load_cert_chain(certfile, keyfile or None)
            self.httpd.socket = ctx.wrap_socket(self.httpd.socket, server_side=True)
        self._threading = threading

    @property
    def url(self) -> str:
        h, p = self.httpd.server_address[:2]
        return f"{'https' if self.tls else 'http'}://{h}:{p}"

    def start(self) -> "AdmissionServer":
        self._threading.Thread(target=self.httpd.serve_forever, daemon=True, name="resize-webhook").start()
        return self

    def stop(self) -> None:
        self.httpd.shutdown()
        self.httpd.server_close()
