"""Kubernetes API client interface + the in-memory FakeCluster apiserver.

The reference talks to the apiserver through client-go (informers, listers, REST writes;
reference pkg/resources/pods.go, nodes.go, gpu_plugins.go:785-795) and has **no** fake
for tests (SURVEY.md §4 "Gaps").  Here `KubeClient` is the one interface every layer
uses; `FakeCluster` implements it in memory with resourceVersion bookkeeping, optimistic
concurrency, JSON/merge patches, the pods/binding subresource, field/label selectors,
watch fan-out and fault-injection hooks; `kube.rest.RestClient` implements it against a
real apiserver (in-cluster service account or kubeconfig).
"""
from __future__ import annotations

import itertools
import queue
import threading
import time
from typing import Any, Callable, Dict, Iterator, List, Optional, Tuple

from ..api import objects as O
from .patch import apply_json_patch, apply_merge_patch, match_field_selector, match_label_selector

Obj = Dict[str, Any]

NAMESPACED = {"pods": True, "configmaps": True, "events": True, "leases": True,
              "nodes": False, "namespaces": False,
              # storage (kube-scheduler's volume plugins: framework.volume_plugins)
              "persistentvolumeclaims": True, "persistentvolumes": False, "storageclasses": False,
              "csinodes": False,
              # workload owners (SelectorSpread, ServiceAffinity, PodTopologySpread system defaults)
              "services": True, "replicationcontrollers": True, "replicasets": True, "statefulsets": True,
              "poddisruptionbudgets": True}
KIND_OF = {"poddisruptionbudgets": "PodDisruptionBudget", "pods": "Pod", "configmaps": "ConfigMap", "events": "Event", "leases": "Lease",
           "nodes": "Node", "namespaces": "Namespace", "persistentvolumeclaims": "PersistentVolumeClaim",
           "persistentvolumes": "PersistentVolume", "storageclasses": "StorageClass", "csinodes": "CSINode",
           "services": "Service", "replicationcontrollers": "ReplicationController", "replicasets": "ReplicaSet",
           "statefulsets": "StatefulSet"}
API_VERSION_OF = {"poddisruptionbudgets": "policy/v1", "leases": "coordination.k8s.io/v1", "storageclasses": "storage.k8s.io/v1",
                  "csinodes": "storage.k8s.io/v1", "replicasets": "apps/v1", "statefulsets": "apps/v1"}


class ApiError(Exception):
    def __init__(self, code: int, reason: str, message: str = ""):
        super().__init__(f"{code} {reason}: {message}")
        self.code, self.reason, self.message = code, reason, message


class NotFound(ApiError):
    def __init__(self, message: str = ""):
        super().__init__(404, "NotFound", message)


class TooManyRequests(ApiError):
    """429: an eviction the pod's PodDisruptionBudget does not allow right now."""

    def __init__(self, message: str = ""):
        super().__init__(429, "TooManyRequests", message)


class Conflict(ApiError):
    def __init__(self, message: str = ""):
        super().__init__(409, "Conflict", message)


class AlreadyExists(ApiError):
    def __init__(self, message: str = ""):
        super().__init__(409, "AlreadyExists", message)


class Gone(ApiError):
    """410: the requested resourceVersion is too old for a watch."""

    def __init__(self, message: str = ""):
        super().__init__(410, "Gone", message)


class WatchEvent(dict):
    """{"type": ADDED|MODIFIED|DELETED|BOOKMARK|ERROR, "object": obj}"""


class KubeClient:
    """The apiserver operations the framework needs."""

    def list(self, resource: str, namespace: Optional[str] = None, label_selector: Any = None,
             field_selector: Optional[str] = None) -> Tuple[List[Obj], str]:
        raise NotImplementedError

    def get(self, resource: str, name: str, namespace: Optional[str] = None) -> Obj:
        raise NotImplementedError

    def create(self, resource: str, obj: Obj, namespace: Optional[str] = None) -> Obj:
        raise NotImplementedError

    def update(self, resource: str, obj: Obj, namespace: Optional[str] = None) -> Obj:
        raise NotImplementedError

    def patch(self, resource: str, name: str, patch: Any, patch_type: str = "json",
              namespace: Optional[str] = None) -> Obj:
        raise NotImplementedError

    def delete(self, resource: str, name: str, namespace: Optional[str] = None,
               grace_period_seconds: Optional[int] = None) -> None:
        raise NotImplementedError

    def bind(self, namespace: str, pod_name: str, node_name: str, pod_uid: str = "",
             annotations: Optional[Dict[str, str]] = None) -> None:
        """POST pods/binding; Binding.metadata.annotations are copied onto the pod by the
        apiserver (BindingREST), which is how the scheduler attaches per-pod assignment
        annotations without a separate PATCH."""
        raise NotImplementedError

    def evict(self, namespace: str, pod_name: str, grace_period_seconds: Optional[int] = None) -> None:
        """POST pods/eviction (policy/v1 Eviction): a delete that honours the pod's
        PodDisruptionBudgets -- raises TooManyRequests (429) when a budget forbids it."""
        raise NotImplementedError

    def watch(self, resource: str, namespace: Optional[str] = None, resource_version: str = "",
              timeout_s: Optional[float] = None) -> Iterator[WatchEvent]:
        raise NotImplementedError

    # conveniences --------------------------------------------------------------------
    def create_event(self, involved: Obj, reason: str, message: str, type_: str = "Normal") -> None:
        ns = O.namespace(involved)
        ev = {"apiVersion": "v1", "kind": "Event",
              "metadata": {"generateName": f"{O.name(involved)}.", "namespace": ns},
              "involvedObject": {"kind": involved.get("kind", "Pod"), "name": O.name(involved),
                                 "namespace": ns, "uid": O.uid(involved)},
              "reason": reason, "message": message, "type": type_,
              "source": {"component": "gpu-scheduler"}}
        try:
            self.create("events", ev, ns)
        except ApiError:
            pass


class FakeCluster(KubeClient):
    """In-memory apiserver.

    * `sync_watch=True` (default) delivers watch events inline to `subscribe()`rs, so
      informer-driven tests are deterministic and thread-free; `watch()` iterators are
      always queue-backed.
    * Fault injection: `fail_next(op, resource, exc, times)` and `latency_s`.
    * `auto_run=True` moves bound pods to phase Running (the kubelet's job).
    """

    def __init__(self, sync_watch: bool = True, auto_run: bool = True, history: int = 1000):
        self._lock = threading.RLock()
        self._store: Dict[str, Dict[str, Obj]] = {r: {} for r in NAMESPACED}
        self._rv = itertools.count(1)
        self._cur_rv = 0
        self._subs: Dict[str, List[Callable[[WatchEvent], None]]] = {r: [] for r in NAMESPACED}
        self._admission: Dict[str, List[Callable[[Obj], Obj]]] = {}
        self._queues: Dict[str, List[Tuple[Optional[str], "queue.Queue[Optional[WatchEvent]]"]]] = {
            r: [] for r in NAMESPACED}
        self._history: Dict[str, List[Tuple[int, WatchEvent]]] = {r: [] for r in NAMESPACED}
        self._history_len = history
        self._faults: List[List[Any]] = []
        self.sync_watch = sync_watch
        self.auto_run = auto_run
        self.latency_s = 0.0
        self.bindings: List[Tuple[str, str, str]] = []
        self.evictions: List[Tuple[str, str]] = []
        self.calls: Dict[str, int] = {}

    # ------------------------------------------------------------------ fault injection
    def fail_next(self, op: str, resource: str, exc: Exception, times: int = 1) -> None:
        with self._lock:
            self._faults.append([op, resource, exc, times])

    def _maybe_fail(self, op: str, resource: str) -> None:
        self.calls[op] = self.calls.get(op, 0) + 1
        if self.latency_s:
            time.sleep(self.latency_s)
        for f in self._faults:
            if f[0] == op and f[1] == resource and f[3] > 0:
                f[3] -= 1
                raise f[2]

    # ------------------------------------------------------------------ internals
    def _k(self, resource: str, name: str, namespace: Optional[str]) -> str:
        if NAMESPACED[resource]:
            return f"{namespace or 'default'}/{name}"
        return name

    def _bump(self, obj: Obj) -> None:
        rv = next(self._rv)
        self._cur_rv = rv
        O.meta(obj)["resourceVersion"] = str(rv)

    def _emit(self, resource: str, typ: str, obj: Obj) -> None:
        # Copy-on-write store: every mutation installs a NEW object and never touches a
        # stored one in place, so the stored object itself is shared (no copy) by the
        # history, every inline subscriber and every watch queue.  Like client-go's shared
        # informer cache, consumers must treat watched objects as read-only; get()/list()
        # still hand out private copies.
        ev = WatchEvent(type=typ, object=obj)
        h = self._history[resource]
        h.append((int(O.resource_version(obj) or self._cur_rv), ev))
        if len(h) > self._history_len:
            del h[: len(h) - self._history_len]
        for cb in list(self._subs[resource]):
            cb(ev)
        ns_obj = O.namespace(obj) if NAMESPACED[resource] else None
        for ns, q in list(self._queues[resource]):
            if ns is None or ns == ns_obj:
                q.put(ev)

    @property
    def resource_version(self) -> str:
        return str(self._cur_rv)

    # ------------------------------------------------------------------ KubeClient
    def list(self, resource, namespace=None, label_selector=None, field_selector=None):
        with self._lock:
            self._maybe_fail("list", resource)
            out = []
            for k, obj in self._store[resource].items():
                if NAMESPACED[resource] and namespace and O.namespace(obj) != namespace:
                    continue
                if not match_label_selector(O.labels(obj), label_selector):
                    continue
                if not match_field_selector(obj, field_selector):
                    continue
                out.append(O.deepcopy(obj))
            return out, str(self._cur_rv)

    def get(self, resource, name, namespace=None):
        with self._lock:
            self._maybe_fail("get", resource)
            obj = self._store[resource].get(self._k(resource, name, namespace))
            if obj is None:
                raise NotFound(f"{resource} {namespace}/{name}")
            return O.deepcopy(obj)

    def add_admission(self, resource: str, fn: Callable[[Obj], Obj]) -> None:
        """Mutating admission hook on CREATE (the in-process analog of a
        MutatingWebhookConfiguration): fn(obj) -> obj, run in registration order."""
        self._admission.setdefault(resource, []).append(fn)

    def create(self, resource, obj, namespace=None, owned=False):
        """owned=True: the caller hands the object over (never touches it again) and does
        not need the stored copy back -- skips both defensive copies (bulk arrivals)."""
        with self._lock:
            self._maybe_fail("create", resource)
            if not owned:
                obj = O.deepcopy(obj)
            for fn in self._admission.get(resource, ()):
                obj = fn(obj)
            md = O.meta(obj)
            if NAMESPACED[resource]:
                md["namespace"] = namespace or md.get("namespace") or "default"
            if not md.get("name") and md.get("generateName"):
                md["name"] = f"{md['generateName']}{next(self._rv):x}"
            k = self._k(resource, md["name"], md.get("namespace"))
            if k in self._store[resource]:
                raise AlreadyExists(f"{resource} {k}")
            md.setdefault("uid", f"uid-{resource}-{md['name']}-{next(self._rv)}")
            md.setdefault("creationTimestamp", time.strftime("%Y-%m-%dT%H:%M:%SZ", time.gmtime()))
            obj.setdefault("kind", KIND_OF[resource])
            obj.setdefault("apiVersion", API_VERSION_OF.get(resource, "v1"))
            if resource == "pods":
                obj.setdefault("status", {}).setdefault("phase", "Pending")
            self._bump(obj)
            self._store[resource][k] = obj
            self._emit(resource, "ADDED", obj)
            return None if owned else O.deepcopy(obj)

    def update(self, resource, obj, namespace=None):
        with self._lock:
            self._maybe_fail("update", resource)
            md = obj.get("metadata", {})
            k = self._k(resource, md.get("name", ""), namespace or md.get("namespace"))
            cur = self._store[resource].get(k)
            if cur is None:
                raise NotFound(f"{resource} {k}")
            rv = md.get("resourceVersion")
            if rv and rv != O.resource_version(cur):
                raise Conflict(f"{resource} {k}: resourceVersion {rv} != {O.resource_version(cur)}")
            new = O.deepcopy(obj)
            O.meta(new)["uid"] = O.uid(cur)
            if NAMESPACED[resource]:
                O.meta(new)["namespace"] = O.namespace(cur)
            self._bump(new)
            self._store[resource][k] = new
            self._emit(resource, "MODIFIED", new)
            return O.deepcopy(new)

    def patch(self, resource, name, patch, patch_type="json", namespace=None):
        with self._lock:
            self._maybe_fail("patch", resource)
            k = self._k(resource, name, namespace)
            cur = self._store[resource].get(k)
            if cur is None:
                raise NotFound(f"{resource} {k}")
            if patch_type == "json":
                new = apply_json_patch(cur, patch)
            elif patch_type in ("merge", "strategic"):
                new = apply_merge_patch(cur, patch)
            else:
                raise ApiError(415, "UnsupportedMediaType", patch_type)
            O.meta(new)["name"] = O.name(cur)
            O.meta(new)["uid"] = O.uid(cur)
            self._bump(new)
            self._store[resource][k] = new
            self._emit(resource, "MODIFIED", new)
            return O.deepcopy(new)

    def delete(self, resource, name, namespace=None, grace_period_seconds=None):
        with self._lock:
            self._maybe_fail("delete", resource)
            k = self._k(resource, name, namespace)
            obj = self._store[resource].pop(k, None)
            if obj is None:
                raise NotFound(f"{resource} {k}")
            self._bump(obj)
            self._emit(resource, "DELETED", obj)

    def bind(self, namespace, pod_name, node_name, pod_uid="", annotations=None):
        with self._lock:
            self._maybe_fail("bind", "pods")
            k = self._k("pods", pod_name, namespace)
            pod = self._store["pods"].get(k)
            if pod is None:
                raise NotFound(f"pods {k}")
            if pod_uid and O.uid(pod) != pod_uid:
                raise Conflict(f"pod {k} uid changed")
            if O.node_name_of(pod):
                raise Conflict(f"pod {k} is already assigned to node {O.node_name_of(pod)}")
            node = self._store["nodes"].get(node_name)
            if node is None:
                raise NotFound(f"nodes {node_name}")
            # path copy: stored objects are never mutated in place (copy-on-write store,
            # see _emit), so only the sub-objects the binding changes are copied
            new = dict(pod)
            new["spec"] = dict(pod.get("spec") or {}, nodeName=node_name)
            md = new["metadata"] = dict(pod.get("metadata") or {})
            if annotations:
                md["annotations"] = dict(md.get("annotations") or {}, **annotations)
            st = new["status"] = dict(pod.get("status") or {})
            st["conditions"] = list(st.get("conditions") or []) + [{"type": "PodScheduled", "status": "True"}]
            if self.auto_run:
                st["phase"] = "Running"
            self._bump(new)
            self._store["pods"][k] = new
            self.bindings.append((namespace, pod_name, node_name))
            self._emit("pods", "MODIFIED", new)

    def evict(self, namespace, pod_name, grace_period_seconds=None):
        """The eviction subresource: refused (429) while a PodDisruptionBudget selecting the
        pod has status.disruptionsAllowed == 0, else the pod is deleted and the budget's
        allowance drops by one (the disruption controller would recompute it)."""
        with self._lock:
            self._maybe_fail("evict", "pods")
            pod = self._store["pods"].get(self._k("pods", pod_name, namespace))
            if pod is None:
                raise NotFound(f"pods {namespace}/{pod_name}")
            budgets = [b for b in self._store["poddisruptionbudgets"].values()
                       if O.namespace(b) == namespace
                       and match_label_selector(O.labels(pod), (b.get("spec") or {}).get("selector") or {})]
            for b in budgets:
                if int((b.get("status") or {}).get("disruptionsAllowed", 0)) <= 0:
                    raise TooManyRequests(f"Cannot evict pod as it would violate the pod's disruption budget "
                                          f"{O.name(b)}")
            for b in budgets:
                st = b.setdefault("status", {})
                st["disruptionsAllowed"] = int(st.get("disruptionsAllowed", 0)) - 1
            self.evictions.append((namespace, pod_name))
        self.delete("pods", pod_name, namespace, grace_period_seconds)

    def set_pod_phase(self, namespace: str, pod_name: str, phase: str) -> Obj:
        return self.patch("pods", pod_name, {"status": {"phase": phase}}, "merge", namespace)

    def subscribe(self, resource: str, cb: Callable[[WatchEvent], None]) -> Callable[[], None]:
        """Inline (synchronous) watch used by informers on a FakeCluster."""
        with self._lock:
            self._subs[resource].append(cb)

        def cancel() -> None:
            with self._lock:
                if cb in self._subs[resource]:
                    self._subs[resource].remove(cb)
        return cancel

    def watch(self, resource, namespace=None, resource_version="", timeout_s=None):
        q: "queue.Queue[Optional[WatchEvent]]" = queue.Queue()
        with self._lock:
            if resource_version:
                rv = int(resource_version)
                hist = self._history[resource]
                if hist and rv < hist[0][0] - 1 and rv < self._cur_rv:
                    raise Gone(f"resourceVersion {rv} is too old")
                for hrv, ev in hist:
                    if hrv > rv:
                        obj = ev["object"]
                        if namespace is None or not NAMESPACED[resource] or O.namespace(obj) == namespace:
                            q.put(WatchEvent(type=ev["type"], object=O.deepcopy(obj)))
            entry = (namespace, q)
            self._queues[resource].append(entry)
        deadline = None if timeout_s is None else time.monotonic() + timeout_s

        def it() -> Iterator[WatchEvent]:
            try:
                while True:
                    rem = None if deadline is None else max(0.0, deadline - time.monotonic())
                    if rem == 0.0:
                        return
                    try:
                        ev = q.get(timeout=rem if rem is not None else 0.5)
                    except queue.Empty:
                        if deadline is None:
                            continue
                        return
                    if ev is None:
                        return
                    yield ev
            finally:
                with self._lock:
                    if entry in self._queues[resource]:
                        self._queues[resource].remove(entry)
        return it()

    def close_watches(self) -> None:
        with self._lock:
            for r in self._queues:
                for _, q in self._queues[r]:
                    q.put(None)

    # ------------------------------------------------------------------ snapshot/restore
    def dump(self) -> Dict[str, List[Obj]]:
        with self._lock:
            return {r: [O.deepcopy(o) for o in objs.values()] for r, objs in self._store.items()}

    def load(self, state: Dict[str, List[Obj]]) -> None:
        for r, objs in state.items():
            for o in objs:
                self.create(r, o, o.get("metadata", {}).get("namespace"))
