"""Persistent-volume controller for the fake cluster: the kube-controller-manager half of
volume binding that the scheduler's VolumeBinding plugin (framework.volume_plugins) relies
on.  In a real cluster this is kube-controller-manager's PV controller plus an external
provisioner; here it keeps the fake apiserver's claims and volumes consistent so scheduler
tests and local stacks can schedule pods with PersistentVolumeClaims:

  * a PV whose claimRef names an unbound claim -> bind both (claim.spec.volumeName, both
    phases Bound, pv.kubernetes.io/bind-completed);
  * an unbound Immediate-mode claim -> bind it to the smallest matching available PV, or
    provision one when its StorageClass has a provisioner;
  * an unbound claim carrying volume.kubernetes.io/selected-node (set by the scheduler's
    PreBind for WaitForFirstConsumer classes) -> provision a PV pinned to that node
    (node affinity on kubernetes.io/hostname) and bind it.
"""
from __future__ import annotations

import threading
from typing import Any, Dict, Optional

from ..api import objects as O
from ..framework.volume_plugins import (ANNOT_BIND_COMPLETED, ANNOT_SELECTED_NODE, NO_PROVISIONER, _claim_class,
                                        claim_is_bound, parse_storage, pv_matches_claim)
from .client import FakeCluster, NotFound

Obj = Dict[str, Any]


class PVController:
    def __init__(self, client: Any):
        self.client = client
        self._busy = threading.local()
        self._cancel = []
        self._stop = threading.Event()
        self._thread: Optional[threading.Thread] = None
        self.provisioned = 0

    # ------------------------------------------------------------------ reconcile
    def _bind(self, pvc: Obj, pv: Obj) -> None:
        ns, cname, vname = O.namespace(pvc), O.name(pvc), O.name(pv)
        if not (pv.get("spec") or {}).get("claimRef"):
            self.client.patch("persistentvolumes", vname, {"spec": {"claimRef": {
                "kind": "PersistentVolumeClaim", "namespace": ns, "name": cname, "uid": O.uid(pvc)}}}, "merge")
        self.client.patch("persistentvolumes", vname, {"status": {"phase": "Bound"}}, "merge")
        self.client.patch("persistentvolumeclaims", cname, {
            "metadata": {"annotations": {ANNOT_BIND_COMPLETED: "yes"}},
            "spec": {"volumeName": vname}, "status": {"phase": "Bound"}}, "merge", ns)

    def _provision(self, pvc: Obj, node: str) -> None:
        spec = pvc.get("spec") or {}
        pv = {"metadata": {"name": f"pvc-{O.uid(pvc) or O.name(pvc)}", "labels": {}},
              "spec": {"capacity": {"storage": ((spec.get("resources") or {}).get("requests") or {}).get("storage", "1Gi")},
                       "accessModes": list(spec.get("accessModes") or ["ReadWriteOnce"]),
                       "storageClassName": _claim_class(pvc),
                       "volumeMode": spec.get("volumeMode") or "Filesystem",
                       "persistentVolumeReclaimPolicy": "Delete",
                       "claimRef": {"kind": "PersistentVolumeClaim", "namespace": O.namespace(pvc),
                                    "name": O.name(pvc), "uid": O.uid(pvc)}}}
        if node:
            pv["spec"]["nodeAffinity"] = {"required": {"nodeSelectorTerms": [{"matchExpressions": [
                {"key": "kubernetes.io/hostname", "operator": "In", "values": [node]}]}]}}
        created = self.client.create("persistentvolumes", pv)
        self.provisioned += 1
        self._bind(pvc, created if created is not None else self.client.get("persistentvolumes", pv["metadata"]["name"]))

    def reconcile(self) -> None:
        """One pass over every claim and volume (idempotent)."""
        pvs = self.client.list("persistentvolumes")[0]
        by_name = {O.name(v): v for v in pvs}
        for pvc in self.client.list("persistentvolumeclaims")[0]:
            if claim_is_bound(pvc) and (pvc.get("status") or {}).get("phase") == "Bound":
                continue
            ns, cname = O.namespace(pvc), O.name(pvc)
            ref = next((v for v in pvs if ((v.get("spec") or {}).get("claimRef") or {}).get("name") == cname
                        and (v["spec"]["claimRef"].get("namespace") or "default") == ns), None)
            want = (pvc.get("spec") or {}).get("volumeName")
            if ref is None and want:
                ref = by_name.get(want)
            if ref is not None:
                self._bind(pvc, ref)
                continue
            node = O.annotations(pvc).get(ANNOT_SELECTED_NODE, "")
            sc = self._class(_claim_class(pvc))
            delayed = sc is not None and sc.get("volumeBindingMode") == "WaitForFirstConsumer"
            if delayed and not node:
                continue                            # waits for the scheduler to pick a node
            if not delayed:
                free = [v for v in pvs if not (v.get("spec") or {}).get("claimRef") and pv_matches_claim(v, pvc)]
                if free:
                    best = min(free, key=lambda v: parse_storage(v["spec"].get("capacity", {}).get("storage")))
                    self._bind(pvc, best)
                    pvs = self.client.list("persistentvolumes")[0]
                    continue
            if sc is not None and (sc.get("provisioner") or NO_PROVISIONER) != NO_PROVISIONER:
                self._provision(pvc, node)
                pvs = self.client.list("persistentvolumes")[0]

    def _class(self, name: str) -> Optional[Obj]:
        if not name:
            return None
        try:
            return self.client.get("storageclasses", name)
        except NotFound:
            return None

    # ------------------------------------------------------------------ running
    def _on_event(self, ev) -> None:
        if getattr(self._busy, "on", False):        # our own writes re-enter: one pass is enough
            return
        self._busy.on = True
        try:
            self.reconcile()
        finally:
            self._busy.on = False

    def start(self, period_s: float = 0.2) -> "PVController":
        """FakeCluster: reconcile inline on every claim / volume event; any other client:
        a polling thread."""
        if isinstance(self.client, FakeCluster):
            for r in ("persistentvolumeclaims", "persistentvolumes"):
                self._cancel.append(self.client.subscribe(r, self._on_event))
            self.reconcile()
            return self

        def loop():
            while not self._stop.wait(period_s):
                try:
                    self.reconcile()
                except Exception:
                    pass
        self._thread = threading.Thread(target=loop, name="pv-controller", daemon=True)
        self._thread.start()
        return self

    def stop(self) -> None:
        for c in self._cancel:
            c()
        self._cancel = []
        self._stop.set()
