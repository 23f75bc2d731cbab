"""kube-scheduler's volume plugins: VolumeBinding, VolumeRestrictions, VolumeZone and
NodeVolumeLimits (CSI).

The reference's scheduler is the stock kube-scheduler v1.21 plus the GPU plugin (reference
cmd/scheduler/main.go:15-28), so pods with PersistentVolumeClaims keep working there: claims
must exist, bound volumes must be reachable from the node, WaitForFirstConsumer claims are
bound to a matching volume on the chosen node (or provisioned there), and per-node attach
limits hold.  Same semantics here, on the framework's extension points:

  VolumeBinding      PreFilter: resolve the pod's claims (missing / deleting claim or an
                     unbound Immediate-mode claim -> UnschedulableAndUnresolvable).
                     Filter: every bound claim's PV node affinity matches the node; every
                     delayed claim finds the smallest available matching PV (class, capacity,
                     access modes, volume mode, claim selector, PV node affinity) not already
                     taken in this cycle or assumed by an earlier one -- or its StorageClass
                     can provision there (provisioner set, allowedTopologies match).
                     Reserve/Unreserve: assume / forget the chosen PVs so later cycles do
                     not pick them before the API catches up.  PreBind: PV claimRef (static)
                     or the claim's selected-node annotation (dynamic), then wait (bounded,
                     `bindTimeoutSeconds`) until the PV controller reports every claim Bound.
  VolumeRestrictions an in-line GCE PD / AWS EBS / RBD / iSCSI disk already mounted read-write
                     on the node, or a ReadWriteOncePod claim already in use, conflicts.
  VolumeZone         a bound PV's topology.kubernetes.io/{zone,region} labels (multi-zone
                     values joined by "__") must contain the node's label value.
  NodeVolumeLimits   CSI volumes on the node (distinct driver + volume handle, incl. the
                     pod's) may not exceed the node's CSINode allocatable count per driver.
  EBSLimits, GCEPDLimits, AzureDiskLimits, CinderLimits
                     the in-tree attach limits: distinct AWS EBS / GCE PD / Azure disk /
                     Cinder volumes (in-line or through a bound claim's PV, plus unbound
                     claims whose class provisions that type) may not exceed the node's
                     `attachable-volumes-*` allocatable, else the upstream default (EBS 39,
                     25 on Nitro instance types; GCE PD 16; Azure 16; Cinder 256;
                     KUBE_MAX_PD_VOLS overrides).  A plugin migrated to CSI on the node
                     (CSINode storage.alpha.kubernetes.io/migrated-plugins) is left to
                     NodeVolumeLimits.

Each plugin returns Skip at PreFilter for pods without volumes of its kind, so ordinary pods
(and the cross-cycle node-result cache) are unaffected.  `kube.pv_controller` is the PV
controller half for the fake cluster (bind + a provisioner).
"""
from __future__ import annotations

import os
import re
import threading
import time
from typing import Any, Dict, List, Optional, Set, Tuple

from ..api import objects as O
from ..kube.patch import match_label_selector
from .interface import FilterPlugin, PreBindPlugin, PreFilterPlugin, ReservePlugin, Status
from .score_plugins import node_selector_term_matches

Obj = Dict[str, Any]

ANNOT_SELECTED_NODE = "volume.kubernetes.io/selected-node"
ANNOT_BIND_COMPLETED = "pv.kubernetes.io/bind-completed"
NO_PROVISIONER = "kubernetes.io/no-provisioner"
ZONE_LABELS = ("topology.kubernetes.io/zone", "topology.kubernetes.io/region",
               "failure-domain.beta.kubernetes.io/zone", "failure-domain.beta.kubernetes.io/region")


def parse_storage(q: Any) -> float:
    return O.parse_quantity(q) if q not in (None, "") else 0.0


def pod_claim_names(pod: Obj) -> List[str]:
    return [v["persistentVolumeClaim"]["claimName"] for v in (pod.get("spec") or {}).get("volumes") or []
            if (v.get("persistentVolumeClaim") or {}).get("claimName")]


def pv_node_affinity_matches(pv: Obj, node: Obj) -> bool:
    req = (((pv.get("spec") or {}).get("nodeAffinity") or {}).get("required") or {})
    terms = req.get("nodeSelectorTerms") or []
    return not terms or any(node_selector_term_matches(node, t) for t in terms)


def _claim_class(pvc: Obj) -> str:
    sc = (pvc.get("spec") or {}).get("storageClassName")
    if sc is None:
        sc = O.annotations(pvc).get("volume.beta.kubernetes.io/storage-class", "")
    return sc or ""


def _pv_class(pv: Obj) -> str:
    return (pv.get("spec") or {}).get("storageClassName") or ""


def claim_is_bound(pvc: Obj) -> bool:
    return bool((pvc.get("spec") or {}).get("volumeName")) and \
        ((pvc.get("status") or {}).get("phase") in (None, "", "Bound"))


def pv_matches_claim(pv: Obj, pvc: Obj) -> bool:
    """The persistent-volume controller's findMatchingVolume predicate (without node affinity)."""
    spec, cspec = pv.get("spec") or {}, pvc.get("spec") or {}
    if O.meta(pv).get("deletionTimestamp"):
        return False
    ref = spec.get("claimRef")
    if ref and (ref.get("name") != O.name(pvc) or ref.get("namespace", "default") != O.namespace(pvc)):
        return False
    if _pv_class(pv) != _claim_class(pvc):
        return False
    if (spec.get("volumeMode") or "Filesystem") != (cspec.get("volumeMode") or "Filesystem"):
        return False
    if not set(cspec.get("accessModes") or []) <= set(spec.get("accessModes") or []):
        return False
    need = parse_storage(((cspec.get("resources") or {}).get("requests") or {}).get("storage"))
    have = parse_storage((spec.get("capacity") or {}).get("storage"))
    if have < need:
        return False
    sel = cspec.get("selector")
    return not sel or match_label_selector(O.labels(pv), sel)


class _Claims:
    __slots__ = ("bound", "delayed", "pvcs")

    def __init__(self):
        self.bound: List[Tuple[Obj, Obj]] = []      # (pvc, pv)
        self.delayed: List[Obj] = []                # WaitForFirstConsumer claims to bind
        self.pvcs: List[Obj] = []


class VolumeBinding(PreFilterPlugin, FilterPlugin, ReservePlugin, PreBindPlugin):
    NAME = "VolumeBinding"
    _KEY = "VolumeBinding/claims"
    _DEC = "VolumeBinding/decisions"        # node -> [(pvc key, pv name or "" = provision)]

    def __init__(self, args=None, handle=None):
        args = args or {}
        self.handle = handle
        self.bind_timeout_s = float(args.get("bindTimeoutSeconds", 600))
        self._assumed: Dict[str, str] = {}          # pv name -> claim key (assumed, API pending)
        self._pod_assumed: Dict[str, List[str]] = {}
        self._lock = threading.Lock()
        self._inf = None
        if handle is not None:
            try:
                f = handle.informer_factory
                self._inf = (f.persistent_volume_claims(), f.persistent_volumes(), f.storage_classes())
            except AttributeError:
                self._inf = None

    # ------------------------------------------------------------------ lookups
    def _pvc(self, ns: str, name: str) -> Optional[Obj]:
        if self._inf is not None:
            return self._inf[0].lister.get(name, ns)
        try:
            return self.handle.client.get("persistentvolumeclaims", name, ns)
        except Exception:
            return None

    def _pv(self, name: str) -> Optional[Obj]:
        if self._inf is not None:
            return self._inf[1].lister.get(name)
        try:
            return self.handle.client.get("persistentvolumes", name)
        except Exception:
            return None

    def _pvs(self) -> List[Obj]:
        if self._inf is not None:
            return self._inf[1].lister.list()
        return self.handle.client.list("persistentvolumes")[0]

    def _class(self, name: str) -> Optional[Obj]:
        if not name:
            return None
        if self._inf is not None:
            return self._inf[2].lister.get(name)
        try:
            return self.handle.client.get("storageclasses", name)
        except Exception:
            return None

    def _delayed(self, pvc: Obj) -> bool:
        sc = self._class(_claim_class(pvc))
        return sc is not None and sc.get("volumeBindingMode") == "WaitForFirstConsumer"

    # ------------------------------------------------------------------ PreFilter / Filter
    def pre_filter(self, state, pod):
        if not (pod.get("spec") or {}).get("volumes"):
            return Status.skip()
        names = pod_claim_names(pod)
        if not names:
            return Status.skip()
        cl = _Claims()
        for n in names:
            pvc = self._pvc(O.namespace(pod), n)
            if pvc is None:
                return Status.unschedulable(f'persistentvolumeclaim "{n}" not found', self.NAME, True)
            if O.meta(pvc).get("deletionTimestamp"):
                return Status.unschedulable(f'persistentvolumeclaim "{n}" is being deleted', self.NAME, True)
            cl.pvcs.append(pvc)
            vol = (pvc.get("spec") or {}).get("volumeName")
            if vol and claim_is_bound(pvc):
                pv = self._pv(vol)
                if pv is None:
                    return Status.unschedulable(f'pvc "{n}" bound to non-existent pv "{vol}"', self.NAME, True)
                cl.bound.append((pvc, pv))
            elif self._delayed(pvc):
                cl.delayed.append(pvc)
            else:
                return Status.unschedulable("pod has unbound immediate PersistentVolumeClaims", self.NAME, True)
        state.write(self._KEY, cl)
        state.write(self._DEC, {})
        return None

    def filter(self, state, pod, node_info):
        cl: Optional[_Claims] = state.read(self._KEY)
        if cl is None:
            return None
        node = node_info.node
        for _, pv in cl.bound:
            if not pv_node_affinity_matches(pv, node):
                return Status.unschedulable("node(s) had volume node affinity conflict", self.NAME, True)
        if not cl.delayed:
            return None
        taken: Set[str] = set()
        decisions = []
        with self._lock:
            assumed = dict(self._assumed)
        pvs = self._pvs()
        for pvc in cl.delayed:
            ckey = O.key(pvc)
            want = (pvc.get("spec") or {}).get("volumeName")
            best = None
            for pv in pvs:
                nm = O.name(pv)
                if nm in taken or (nm in assumed and assumed[nm] != ckey):
                    continue
                if want and nm != want:
                    continue
                if not pv_matches_claim(pv, pvc) or not pv_node_affinity_matches(pv, node):
                    continue
                if best is None or parse_storage(pv["spec"].get("capacity", {}).get("storage")) < \
                        parse_storage(best["spec"].get("capacity", {}).get("storage")):
                    best = pv
            if best is not None:
                taken.add(O.name(best))
                decisions.append((ckey, O.name(best)))
                continue
            sc = self._class(_claim_class(pvc))
            prov = (sc or {}).get("provisioner") or NO_PROVISIONER
            if want or prov == NO_PROVISIONER or not self._topology_allows(sc, node):
                return Status.unschedulable("node(s) didn't find available persistent volumes to bind", self.NAME)
            decisions.append((ckey, ""))            # dynamic provisioning on this node
        state.read(self._DEC)[node_info.name] = decisions
        return None

    @staticmethod
    def _topology_allows(sc: Optional[Obj], node: Obj) -> bool:
        terms = (sc or {}).get("allowedTopologies") or []
        if not terms:
            return True
        lab = O.labels(node)
        for t in terms:
            if all(lab.get(e.get("key")) in (e.get("values") or []) for e in t.get("matchLabelExpressions") or []):
                return True
        return False

    # ------------------------------------------------------------------ Reserve / PreBind
    def reserve(self, state, pod, node_name):
        decs = state.read(self._DEC)
        if not decs:
            return None
        dec = decs.get(node_name)
        if not dec:
            return None
        with self._lock:
            for ckey, pv in dec:
                if pv and self._assumed.get(pv, ckey) != ckey:
                    return Status.unschedulable("persistent volume was taken by another pod", self.NAME)
            taken = [pv for _, pv in dec if pv]
            for ckey, pv in dec:
                if pv:
                    self._assumed[pv] = ckey
            self._pod_assumed[O.key(pod)] = taken
        return None

    def unreserve(self, state, pod, node_name):
        with self._lock:
            for pv in self._pod_assumed.pop(O.key(pod), []):
                self._assumed.pop(pv, None)

    def pre_bind(self, state, pod, node_name):
        decs = state.read(self._DEC)
        if not decs:
            return None
        dec = decs.get(node_name)
        if not dec:
            return None
        client = self.handle.client
        ns = O.namespace(pod)
        try:
            for ckey, pv in dec:
                cname = ckey.split("/", 1)[1]
                if pv:
                    pvc = self._pvc(ns, cname)
                    client.patch("persistentvolumes", pv, {"spec": {"claimRef": {
                        "kind": "PersistentVolumeClaim", "namespace": ns, "name": cname,
                        "uid": O.uid(pvc) if pvc else ""}}}, "merge")
                else:
                    client.patch("persistentvolumeclaims", cname,
                                 {"metadata": {"annotations": {ANNOT_SELECTED_NODE: node_name}}}, "merge", ns)
        except Exception as e:
            return Status.error(f"binding volumes: {e}", self.NAME)
        deadline = time.monotonic() + self.bind_timeout_s
        pending = [ckey.split("/", 1)[1] for ckey, _ in dec]
        while pending:
            try:
                pending = [c for c in pending
                           if not claim_is_bound(client.get("persistentvolumeclaims", c, ns))]
            except Exception as e:
                return Status.error(f"checking volume bindings: {e}", self.NAME)
            if not pending:
                break
            if time.monotonic() > deadline:
                return Status.error(f"timed out waiting for volume binding of {pending}", self.NAME)
            time.sleep(0.05)
        with self._lock:                         # the API now records the bindings
            for pv in self._pod_assumed.pop(O.key(pod), []):
                self._assumed.pop(pv, None)
        return None


# ---------------------------------------------------------------------------- VolumeRestrictions
def _inline_disks(pod: Obj) -> List[Tuple[str, str, bool]]:
    """(kind, identity, read-only) of the pod's in-line disks that conflict upstream."""
    out = []
    for v in (pod.get("spec") or {}).get("volumes") or []:
        if v.get("gcePersistentDisk"):
            d = v["gcePersistentDisk"]
            out.append(("gce", d.get("pdName", ""), bool(d.get("readOnly"))))
        elif v.get("awsElasticBlockStore"):
            out.append(("ebs", v["awsElasticBlockStore"].get("volumeID", ""), False))   # EBS: never shared
        elif v.get("rbd"):
            d = v["rbd"]
            out.append(("rbd", f"{','.join(sorted(d.get('monitors') or []))}/{d.get('pool', 'rbd')}/{d.get('image', '')}",
                        bool(d.get("readOnly"))))
        elif v.get("iscsi"):
            d = v["iscsi"]
            out.append(("iscsi", f"{d.get('iqn', '')}/{d.get('lun', 0)}", bool(d.get("readOnly"))))
    return out


class VolumeRestrictions(PreFilterPlugin, FilterPlugin):
    NAME = "VolumeRestrictions"
    _KEY = "VolumeRestrictions/state"

    def __init__(self, args=None, handle=None):
        self.handle = handle
        self._rwop: Dict[str, Set[str]] = {}        # ReadWriteOncePod claim key -> pods using it
        self._uses: Dict[str, List[str]] = {}       # pod key -> its ReadWriteOncePod claim keys
        self._claims_inf = None
        if handle is not None:
            try:
                self._claims_inf = handle.informer_factory.persistent_volume_claims()
                handle.informer_factory.pods().add_event_handler(self._on_pod, lambda o, n: self._on_pod(n),
                                                                 self._on_pod_delete)
            except AttributeError:
                pass

    def _rwop_claims(self, pod: Obj) -> List[str]:
        out = []
        for n in pod_claim_names(pod):
            pvc = self._claims_inf.lister.get(n, O.namespace(pod)) if self._claims_inf is not None else None
            if pvc is not None and "ReadWriteOncePod" in ((pvc.get("spec") or {}).get("accessModes") or []):
                out.append(f"{O.namespace(pod)}/{n}")
        return out

    def _on_pod(self, pod: Obj) -> None:
        vols = (pod.get("spec") or {}).get("volumes")
        if not vols and not self._uses:
            return                                  # the common case: no claims anywhere
        self._on_pod_delete(pod)
        if vols and O.node_name_of(pod) and not O.is_terminal(pod):
            claims = self._rwop_claims(pod)
            if claims:
                self._uses[O.key(pod)] = claims
                for c in claims:
                    self._rwop.setdefault(c, set()).add(O.key(pod))

    def _on_pod_delete(self, pod: Obj) -> None:
        k = O.key(pod)
        for c in self._uses.pop(k, ()):
            users = self._rwop.get(c)
            if users is not None:
                users.discard(k)
                if not users:
                    del self._rwop[c]

    def pre_filter(self, state, pod):
        if not (pod.get("spec") or {}).get("volumes"):
            return Status.skip()
        disks = _inline_disks(pod)
        claims = self._rwop_claims(pod) if pod_claim_names(pod) else []
        if not disks and not claims:
            return Status.skip()
        me = O.key(pod)
        for c in claims:
            if self._rwop.get(c, set()) - {me}:
                return Status.unschedulable("node has pod using PersistentVolumeClaim with the same name and "
                                            "ReadWriteOncePod access mode", self.NAME, True)
        state.write(self._KEY, disks)
        return None

    def filter(self, state, pod, node_info):
        disks = state.read(self._KEY)
        if not disks:
            return None
        used = [d for other in node_info.pods.values() for d in _inline_disks(other)]
        for kind, ident, ro in disks:
            for k2, i2, ro2 in used:
                if kind == k2 and ident == i2 and not (ro and ro2 and kind != "ebs"):
                    return Status.unschedulable("node(s) had no available disk", self.NAME)
        return None


# ---------------------------------------------------------------------------- VolumeZone
class VolumeZone(PreFilterPlugin, FilterPlugin):
    NAME = "VolumeZone"
    _KEY = "VolumeZone/pvs"

    def __init__(self, args=None, handle=None):
        self.vb = VolumeBinding(None, None)
        self.vb.handle = handle
        self.vb._inf = None
        if handle is not None:
            try:
                f = handle.informer_factory
                self.vb._inf = (f.persistent_volume_claims(), f.persistent_volumes(), f.storage_classes())
            except AttributeError:
                pass

    def pre_filter(self, state, pod):
        if not (pod.get("spec") or {}).get("volumes"):
            return Status.skip()
        names = pod_claim_names(pod)
        if not names:
            return Status.skip()
        zoned = []
        for n in names:
            pvc = self.vb._pvc(O.namespace(pod), n)
            vol = (pvc.get("spec") or {}).get("volumeName") if pvc else None
            pv = self.vb._pv(vol) if vol else None
            if pv is not None and any(k in O.labels(pv) for k in ZONE_LABELS):
                zoned.append(pv)
        if not zoned:
            return Status.skip()
        state.write(self._KEY, zoned)
        return None

    def filter(self, state, pod, node_info):
        lab = O.labels(node_info.node)
        for pv in state.read(self._KEY) or []:
            for k in ZONE_LABELS:
                v = O.labels(pv).get(k)
                if v is None:
                    continue
                if lab.get(k) not in set(v.split("__")):
                    return Status.unschedulable("node(s) had no available volume zone", self.NAME, True)
        return None


# ---------------------------------------------------------------------------- NodeVolumeLimits (CSI)
class NodeVolumeLimits(PreFilterPlugin, FilterPlugin):
    NAME = "NodeVolumeLimits"
    _KEY = "NodeVolumeLimits/volumes"

    def __init__(self, args=None, handle=None):
        self.vb = VolumeZone(None, handle).vb
        self._csinodes = None
        if handle is not None:
            try:
                self._csinodes = handle.informer_factory.csi_nodes()
            except AttributeError:
                pass

    def _csi_volumes(self, pod: Obj) -> List[Tuple[str, str]]:
        out = []
        for n in pod_claim_names(pod):
            pvc = self.vb._pvc(O.namespace(pod), n)
            vol = (pvc.get("spec") or {}).get("volumeName") if pvc else None
            pv = self.vb._pv(vol) if vol else None
            csi = ((pv or {}).get("spec") or {}).get("csi")
            if csi:
                out.append((csi.get("driver", ""), csi.get("volumeHandle", "")))
        for v in (pod.get("spec") or {}).get("volumes") or []:
            if v.get("csi"):                       # in-line (ephemeral) CSI volume
                out.append((v["csi"].get("driver", ""), f"{O.key(pod)}/{v.get('name', '')}"))
        return out

    def pre_filter(self, state, pod):
        vols = self._csi_volumes(pod) if (pod.get("spec") or {}).get("volumes") else []
        if not vols:
            return Status.skip()
        state.write(self._KEY, vols)
        return None

    def filter(self, state, pod, node_info):
        new = state.read(self._KEY) or []
        csinode = self._csinodes.lister.get(node_info.name) if self._csinodes is not None else None
        if csinode is None:
            return None
        limits = {d.get("name"): int((d.get("allocatable") or {}).get("count"))
                  for d in (csinode.get("spec") or {}).get("drivers") or []
                  if (d.get("allocatable") or {}).get("count") is not None}
        attached: Dict[str, Set[str]] = {}
        for other in node_info.pods.values():
            for drv, h in self._csi_volumes(other):
                attached.setdefault(drv, set()).add(h)
        for drv, h in new:
            attached.setdefault(drv, set()).add(h)
        for drv, vols in attached.items():
            if drv in limits and len(vols) > limits[drv]:
                return Status.unschedulable("node(s) exceed max volume count", self.NAME)
        return None


# ---------------------------------------------------------------------------- in-tree volume limits
_EBS_NITRO = re.compile(r"^[cmr]5.*|t3|z1d")
_MIGRATED_ANNOT = "storage.alpha.kubernetes.io/migrated-plugins"


class _InTreeLimits(PreFilterPlugin, FilterPlugin):
    """Base of the non-CSI attach-limit filters (upstream nodevolumelimits/non_csi.go)."""
    VOLUME = ""            # pod volume source / PV spec key
    ID = ""                # field naming the volume inside that source
    PROVISIONER = ""       # in-tree provisioner of dynamically provisioned volumes
    ALLOCATABLE = ""       # node allocatable key
    PLUGIN = ""            # in-tree plugin name (CSI migration annotation)
    DEFAULT_MAX = 0

    def __init__(self, args=None, handle=None):
        self.vb = VolumeZone(None, handle).vb
        self._csinodes = None
        self._key = f"{self.NAME}/volumes"
        if handle is not None:
            try:
                self._csinodes = handle.informer_factory.csi_nodes()
            except AttributeError:
                pass

    def _ids(self, pod: Obj, with_unbound: bool) -> Set[str]:
        out: Set[str] = set()
        ns = O.namespace(pod)
        for v in (pod.get("spec") or {}).get("volumes") or []:
            src = v.get(self.VOLUME)
            if src:
                out.add(str(src.get(self.ID, "")))
                continue
            claim = (v.get("persistentVolumeClaim") or {}).get("claimName")
            if not claim:
                continue
            pvc = self.vb._pvc(ns, claim)
            if pvc is None:
                continue
            vol = (pvc.get("spec") or {}).get("volumeName")
            if vol:
                src = ((self.vb._pv(vol) or {}).get("spec") or {}).get(self.VOLUME)
                if src:
                    out.add(str(src.get(self.ID, "")))
            elif with_unbound:
                sc = self.vb._class(_claim_class(pvc))
                if sc is not None and sc.get("provisioner") == self.PROVISIONER:
                    out.add(f"{ns}/{claim}-unbound")        # one new volume, identity unknown yet
        return out

    def _max(self, node: Obj) -> int:
        env = os.environ.get("KUBE_MAX_PD_VOLS", "")
        if env.isdigit() and int(env) > 0:
            return int(env)
        alloc = ((node.get("status") or {}).get("allocatable") or {}).get(self.ALLOCATABLE)
        if alloc is not None:
            return int(O.parse_quantity(alloc))
        return self._default_max(node)

    def _default_max(self, node: Obj) -> int:
        return self.DEFAULT_MAX

    def _migrated(self, node_name: str) -> bool:
        csinode = self._csinodes.lister.get(node_name) if self._csinodes is not None else None
        if csinode is None:
            return False
        return self.PLUGIN in O.annotations(csinode).get(_MIGRATED_ANNOT, "").split(",")

    def pre_filter(self, state, pod):
        if not (pod.get("spec") or {}).get("volumes"):
            return Status.skip()
        ids = self._ids(pod, True)
        if not ids:
            return Status.skip()
        state.write(self._key, ids)
        return None

    def filter(self, state, pod, node_info):
        new = state.read(self._key)
        if not new or self._migrated(node_info.name):
            return None
        attached: Set[str] = set()
        for other in node_info.pods.values():
            if (other.get("spec") or {}).get("volumes"):
                attached |= self._ids(other, False)
        extra = len(new - attached)
        if extra and len(attached) + extra > self._max(node_info.node):
            return Status.unschedulable("node(s) exceed max volume count", self.NAME)
        return None


class EBSLimits(_InTreeLimits):
    NAME = "EBSLimits"
    VOLUME, ID = "awsElasticBlockStore", "volumeID"
    PROVISIONER, ALLOCATABLE, PLUGIN = "kubernetes.io/aws-ebs", "attachable-volumes-aws-ebs", "kubernetes.io/aws-ebs"
    DEFAULT_MAX = 39

    def _default_max(self, node: Obj) -> int:
        lab = O.labels(node)
        itype = lab.get("node.kubernetes.io/instance-type") or lab.get("beta.kubernetes.io/instance-type") or ""
        return 25 if itype and _EBS_NITRO.match(itype) else 39


class GCEPDLimits(_InTreeLimits):
    NAME = "GCEPDLimits"
    VOLUME, ID = "gcePersistentDisk", "pdName"
    PROVISIONER, ALLOCATABLE, PLUGIN = "kubernetes.io/gce-pd", "attachable-volumes-gce-pd", "kubernetes.io/gce-pd"
    DEFAULT_MAX = 16


class AzureDiskLimits(_InTreeLimits):
    NAME = "AzureDiskLimits"
    VOLUME, ID = "azureDisk", "diskName"
    PROVISIONER, ALLOCATABLE, PLUGIN = ("kubernetes.io/azure-disk", "attachable-volumes-azure-disk",
                                        "kubernetes.io/azure-disk")
    DEFAULT_MAX = 16


class CinderLimits(_InTreeLimits):
    NAME = "CinderLimits"
    VOLUME, ID = "cinder", "volumeID"
    PROVISIONER, ALLOCATABLE, PLUGIN = "kubernetes.io/cinder", "attachable-volumes-cinder", "kubernetes.io/cinder"
    DEFAULT_MAX = 256
