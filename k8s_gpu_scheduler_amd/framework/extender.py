"""kube-scheduler extender front-end (HTTP/JSON).

The reference compiles its plugin INTO a kube-scheduler binary (reference
cmd/scheduler/main.go:20-22).  Without Go, a stock kube-scheduler can still drive this
framework through the scheduler-extender protocol: configure
`extenders: [{urlPrefix: http://gpu-sched-extender:8888, filterVerb: filter,
prioritizeVerb: prioritize, bindVerb: bind, weight: ..., nodeCacheCapable: false}]`.

  POST /filter      ExtenderArgs{Pod, Nodes{items}|NodeNames} -> ExtenderFilterResult
  POST /prioritize  ExtenderArgs -> HostPriorityList [{Host, Score}] (0..10, MaxExtenderPriority)
  POST /bind        ExtenderBindingArgs{PodName, PodNamespace, PodUID, Node} -> ExtenderBindingResult
The same Framework (profile plugins incl. GPU: Filter/Score/NormalizeScore, then
Reserve+PreBind at bind time) runs behind every verb against the informer cache.
"""
from __future__ import annotations

import json
import threading
from http.server import BaseHTTPRequestHandler, ThreadingHTTPServer
from typing import Any, Dict, List, Optional

from ..api import objects as O
from .interface import CycleState
from .scheduler import Scheduler

MAX_EXTENDER_PRIORITY = 10


class Extender:
    def __init__(self, scheduler: Scheduler, scheduler_name: Optional[str] = None):
        self.s = scheduler
        self.fw = scheduler.frameworks[scheduler_name] if scheduler_name else next(iter(scheduler.frameworks.values()))
        self._lock = threading.Lock()

    def _nodes(self, args: Dict[str, Any]) -> List[Any]:
        snap = self.s.cache.snapshot()
        self.s._snapshot = snap
        names = args.get("NodeNames") or args.get("nodenames")
        if names is None:
            items = (args.get("Nodes") or args.get("nodes") or {}).get("items") or []
            names = [O.name(n) for n in items]
        return [ni for ni in (snap.get(n) for n in names) if ni is not None]

    def filter(self, args: Dict[str, Any]) -> Dict[str, Any]:
        pod = args.get("Pod") or args.get("pod")
        with self._lock:
            nodes = self._nodes(args)
            state = CycleState()
            st = self.fw.run_pre_filter(state, pod)
            if not st.ok:
                return {"Nodes": None, "NodeNames": [], "FailedNodes": {n.name: st.message() for n in nodes},
                        "Error": ""}
            ok, failed = self.fw.find_feasible(state, pod, nodes)
        res: Dict[str, Any] = {"NodeNames": [n.name for n in ok], "FailedNodes": {k: v.message() for k, v in failed.items()},
                               "FailedAndUnresolvableNodes": {}, "Error": ""}
        if args.get("Nodes"):
            keep = set(res["NodeNames"])
            res["Nodes"] = {"items": [n for n in args["Nodes"]["items"] if O.name(n) in keep]}
        return res

    def prioritize(self, args: Dict[str, Any]) -> List[Dict[str, Any]]:
        pod = args.get("Pod") or args.get("pod")
        with self._lock:
            nodes = self._nodes(args)
            state = CycleState()
            self.fw.run_pre_filter(state, pod)
            feas, _ = self.fw.find_feasible(state, pod, nodes)
            if not feas:
                return [{"Host": n.name, "Score": 0} for n in nodes]
            self.fw.run_pre_score(state, pod, feas)
            scores, st = self.fw.run_score(state, pod, feas)
        if not st.ok:
            return [{"Host": n.name, "Score": 0} for n in nodes]
        hi = max((s.score for s in scores), default=0) or 1
        by = {s.name: s.score for s in scores}
        return [{"Host": n.name, "Score": int(by.get(n.name, 0) * MAX_EXTENDER_PRIORITY // hi)} for n in nodes]

    def bind(self, args: Dict[str, Any]) -> Dict[str, Any]:
        ns = args.get("PodNamespace") or "default"
        name = args.get("PodName")
        node = args.get("Node")
        try:
            pod = self.s.client.get("pods", name, ns)
        except Exception as e:
            return {"Error": f"get pod: {e}"}
        with self._lock:
            self.s._snapshot = self.s.cache.snapshot()
            state = CycleState()
            st = self.fw.run_pre_filter(state, pod)
            ni = self.s._snapshot.get(node)
            if ni is None:
                return {"Error": f"unknown node {node}"}
            if st.ok:
                st = self.fw.run_filter(state, pod, ni)
            if st.ok:
                self.fw.run_pre_score(state, pod, [ni])
                self.fw.run_score(state, pod, [ni])
                self.s.cache.assume_pod(pod, node)
                st = self.fw.run_reserve(state, pod, node)
            if not st.ok:
                self.fw.run_unreserve(state, pod, node)
                self.s.cache.forget_pod(pod)
                return {"Error": st.message() or "reserve failed"}
        st = self.fw.run_pre_bind(state, pod, node)
        if st.ok:
            st = self.fw.run_bind(state, pod, node)
        if not st.ok:
            self.fw.run_unreserve(state, pod, node)
            self.s.cache.forget_pod(pod)
            return {"Error": st.message()}
        self.s.cache.finish_binding(pod)
        self.fw.run_post_bind(state, pod, node)
        return {"Error": ""}


class ExtenderServer:
    def __init__(self, extender: Extender, host: str = "0.0.0.0", port: int = 8888):
        ext = extender

        class H(BaseHTTPRequestHandler):
            protocol_version = "HTTP/1.1"

            def log_message(self, *a):
                pass

            def do_POST(self):
                n = int(self.headers.get("Content-Length") or 0)
                try:
                    args = json.loads(self.rfile.read(n) or b"{}")
                    verb = self.path.rstrip("/").rsplit("/", 1)[-1]
                    if verb == "filter":
                        out = ext.filter(args)
                    elif verb == "prioritize":
                        out = ext.prioritize(args)
                    elif verb == "bind":
                        out = ext.bind(args)
                    else:
                        self.send_response(404)
                        self.send_header("Content-Length", "0")
                        self.end_headers()
                        return
                    code = 200
                except Exception as e:
                    out, code = {"Error": str(e)}, 500
                raw = json.dumps(out).encode()
                self.send_response(code)
                self.send_header("Content-Type", "application/json")
                self.send_header("Content-Length", str(len(raw)))
                self.end_headers()
                self.wfile.write(raw)

        self.httpd = ThreadingHTTPServer((host, port), H)
        self.httpd.daemon_threads = True

    @property
    def url(self) -> str:
        h, p = self.httpd.server_address[:2]
        return f"http://{h}:{p}"

    def start(self) -> "ExtenderServer":
        threading.Thread(target=self.httpd.serve_forever, daemon=True, name="extender").start()
        return self

    def stop(self) -> None:
        self.httpd.shutdown()
        self.httpd.server_close()
