"""Pod / ConfigMap / Node helpers.

Same operations as the reference's `resources.Descriptor` and `PatchNodeParam`
(reference pkg/resources/pods.go:20-212, pkg/resources/nodes.go:15-68), re-designed:

* reads go through informer listers when given, else straight to the client;
* `list_pods` honours its field selector (the reference ignores it, pods.go:54-61) and
  never panics;
* `get_node` uses its argument (the reference always reads "k8s-aferik-master",
  nodes.go:29 -- reproduce with `parity_master=`);
* ConfigMap updates retry on 409 Conflict (read-modify-write with resourceVersion).
"""
from __future__ import annotations

import json
import random
import threading
import time
from typing import Any, Dict, List, Optional, Tuple

from ..api import objects as O
from .client import Conflict, KubeClient, NotFound
from .informer import Lister

Obj = Dict[str, Any]


class Resources:
    def __init__(self, client: KubeClient, namespace: str = "", field_selector: str = "",
                 pod_lister: Optional[Lister] = None, cm_lister: Optional[Lister] = None,
                 node_lister: Optional[Lister] = None):
        self.client = client
        self.namespace = namespace or "default"     # reference pods.go:183-185
        self.field_selector = field_selector
        self.pod_lister = pod_lister
        self.cm_lister = cm_lister
        self.node_lister = node_lister

    # ---------------------------------------------------------------- pods
    def list_pods(self, all_namespaces: bool = False) -> List[Obj]:
        ns = None if all_namespaces else self.namespace
        if self.pod_lister is not None:
            return self.pod_lister.list(ns, field_selector=self.field_selector or None)
        items, _ = self.client.list("pods", ns, field_selector=self.field_selector or None)
        return items

    def get(self, pod_name: str) -> Optional[Obj]:
        if self.pod_lister is not None:
            return self.pod_lister.get(pod_name, self.namespace)
        try:
            return self.client.get("pods", pod_name, self.namespace)
        except NotFound:
            return None

    def patch_pod(self, pod_name: str, operator_type: str, operator_path: str,
                  operator_data: Dict[str, Any]) -> Obj:
        """JSON-patch one op per key at `operator_path + key` (reference pods.go:63-85)."""
        ops = [{"op": operator_type, "path": operator_path + k, "value": v}
               for k, v in operator_data.items()]
        return self.client.patch("pods", pod_name, ops, "json", self.namespace)

    def annotate_pod(self, pod_name: str, annotations: Dict[str, str]) -> Obj:
        return self.client.patch("pods", pod_name, {"metadata": {"annotations": annotations}},
                                 "merge", self.namespace)

    def delete_pod(self, pod_name: str, grace_period_seconds: int = 0) -> None:
        self.client.delete("pods", pod_name, self.namespace, grace_period_seconds)

    # ---------------------------------------------------------------- configmaps
    def get_config_map(self, cm_name: str) -> Optional[Obj]:
        if self.cm_lister is not None:
            cm = self.cm_lister.get(cm_name, self.namespace)
            if cm is not None:
                return cm
        try:
            return self.client.get("configmaps", cm_name, self.namespace)
        except NotFound:
            return None

    def create_config_map(self, cm_name: str, data: Dict[str, str]) -> Obj:
        return self.client.create("configmaps", O.make_config_map(cm_name, data, self.namespace),
                                  self.namespace)

    def update_config_map(self, cm_name: str, data: Dict[str, str], overwrite: bool = True,
                          retries: int = 10) -> Optional[Obj]:
        """Merge `data` into a ConfigMap (reference pods.go:98-121).  Writers in this
        process are serialised per ConfigMap (concurrent binding cycles of pods that share
        one -- the reference's busybox replicas share `game-demo`, SURVEY §2.9 #6 -- would
        otherwise mostly conflict with each other); other writers are handled with
        optimistic retries and a short jittered backoff."""
        with _cm_lock(self.namespace, cm_name):
            return self._update_config_map(cm_name, data, overwrite, retries)

    def _update_config_map(self, cm_name: str, data: Dict[str, str], overwrite: bool, retries: int) -> Optional[Obj]:
        for attempt in range(retries):
            if attempt:
                time.sleep(random.uniform(0.0, 0.002 * (2 ** min(attempt, 6))))
            try:
                cm = self.client.get("configmaps", cm_name, self.namespace)
            except NotFound:
                return None
            d = cm.setdefault("data", {}) or {}
            cm["data"] = d
            changed = False
            for k, v in data.items():
                if k in d and not overwrite:
                    continue
                if d.get(k) != v:
                    d[k] = v
                    changed = True
            if not changed:
                return cm
            try:
                return self.client.update("configmaps", cm, self.namespace)
            except Conflict:
                continue
        raise Conflict(f"configmap {cm_name}: too many conflicts")

    def upsert_config_map(self, cm_name: str, data: Dict[str, str]) -> Obj:
        cm = self.update_config_map(cm_name, data, True)
        if cm is None:
            cm = self.create_config_map(cm_name, data)
        return cm

    def append_to_existing_config_maps_in_pod(self, pod_name: str, data: Dict[str, str],
                                              overwrite: bool = True, pod: Optional[Obj] = None) -> int:
        """Merge `data` into every envFrom ConfigMap of the pod (reference pods.go:156-174).
        Returns how many ConfigMaps were updated."""
        pod = pod or self.get(pod_name)
        if not pod:
            return 0
        n = 0
        for cm_name in O.env_from_config_maps(pod):
            if self.update_config_map(cm_name, data, overwrite) is not None:
                n += 1
        return n

    # ---------------------------------------------------------------- nodes
    def get_node(self, node_name: str, parity_master: Optional[str] = None) -> Optional[Obj]:
        target = parity_master or node_name
        if self.node_lister is not None:
            n = self.node_lister.get(target)
            if n is not None:
                return n
        try:
            return self.client.get("nodes", target)
        except NotFound:
            return None

    def label_node(self, node_name: str, new_labels: Dict[str, str], operator_type: str = "replace",
                   parity_master: Optional[str] = None) -> Obj:
        """Replace the node's whole label map with (current ∪ new) via JSON patch
        (reference nodes.go:39-68 -- which reads the labels from the hard-coded master)."""
        src = self.get_node(node_name, parity_master) or {}
        lab = dict(O.labels(src))
        lab.update(new_labels)
        ops = [{"op": operator_type, "path": "/metadata/labels", "value": lab}]
        return self.client.patch("nodes", node_name, ops, "json")

    def taint_node(self, node_name: str, key: str, value: str = "true", effect: str = "NoSchedule") -> Obj:
        node = self.client.get("nodes", node_name)
        taints = [t for t in O.node_taints(node) if t.get("key") != key]
        taints.append({"key": key, "value": value, "effect": effect})
        return self.client.patch("nodes", node_name, {"spec": {"taints": taints}}, "merge")

    def untaint_node(self, node_name: str, key: str) -> Obj:
        node = self.client.get("nodes", node_name)
        taints = [t for t in O.node_taints(node) if t.get("key") != key]
        return self.client.patch("nodes", node_name, {"spec": {"taints": taints}}, "merge")


_CM_LOCKS: Dict[Tuple[str, str], threading.Lock] = {}
_CM_LOCKS_GUARD = threading.Lock()


def _cm_lock(namespace: str, name: str) -> threading.Lock:
    with _CM_LOCKS_GUARD:
        lk = _CM_LOCKS.get((namespace, name))
        if lk is None:
            lk = _CM_LOCKS[(namespace, name)] = threading.Lock()
        return lk


def patch_payload(op: str, path: str, data: Dict[str, Any]) -> bytes:
    return json.dumps([{"op": op, "path": path + k, "value": v} for k, v in data.items()]).encode()
