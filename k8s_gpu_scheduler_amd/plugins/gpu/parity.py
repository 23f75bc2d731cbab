"""Parity mode: the reference's `Logic`, `GetSLOs`, `reconfigure` and `PostBind`,
behaviour-for-behaviour (reference pkg/plugins/gpu_plugin/gpu_plugins.go:87-160,
357-453, 455-777, 843-926), including the quirks SURVEY.md §2.9 lists (Score side
effects, shuffled UUIDs, the A30 "empty node" test comparing NodeName to the pod name,
the always-all-4g reconfigure choice, random-UUID PostBind, "2"-before-"4" MPS mapping).
Two deliberate deviations, both configurable: the reconfigure poll is bounded
(`reconfigure_timeout_s`, the reference loops forever, §2.9 #3) and a missing
Redis/Prometheus returns an error instead of `klog.Fatal` killing the process.
"""
from __future__ import annotations

import logging
import random
import threading
import time
from typing import TYPE_CHECKING, Any, Dict, List

from ...api import constants as C
from ...api import objects as O
from ...kube.resources import Resources
from ...store import schema
from ...utils import discovery
from .scoring import Resident, mps_env, pick_mps_config, reconfigure_choice, score_devices

if TYPE_CHECKING:
    from .plugin import GPUPlugin

log = logging.getLogger(__name__)
Obj = Dict[str, Any]

_A30_MUTEX = threading.Lock()           # reference gpu_plugins.go:46,480,496


class ParityLogic:
    def __init__(self, plugin: "GPUPlugin"):
        self.p = plugin
        self.rng = random.Random(plugin.args.seed)

    # ---------------------------------------------------------------- plumbing
    @property
    def client(self):
        return self.p.handle.client

    def _res(self, ns: str, field_selector: str = "") -> Resources:
        inf = getattr(self.p.handle, "informer_factory", None)
        pl = inf.pods().lister if inf is not None else None
        cl = inf.config_maps().lister if inf is not None else None
        nl = inf.nodes().lister if inf is not None else None
        return Resources(self.client, ns, field_selector, pl, cl, nl)

    def _redis(self):
        if self.p.redis is not None:
            return self.p.redis
        master = self.p.args.parity_master or None
        ips = discovery.find_nodes_ip_from_pod(self._res(C.REDIS_NAMESPACE), C.REDIS_POD_SUBSTR,
                                               parity_master=master)
        if not ips:
            return None
        from ...store.resp import Redis
        ip = list(ips[0].values())[-1]
        self.p.redis = Redis.connect(f"{ip}:{C.REDIS_NODEPORT}", self.p.args.redis_password)
        return self.p.redis

    def _conf(self, name: str) -> Dict[str, float]:
        return self.p.predictions.configurations(name) if self.p.predictions else {}

    def _intf(self, name: str) -> Dict[str, float]:
        return self.p.predictions.interference(name) if self.p.predictions else {}

    # ---------------------------------------------------------------- GetSLOs
    def get_slos(self, node_name: str, uuids: List[str]) -> Dict[str, Dict[str, float]]:
        """map[uuid]map[podName]SLO for Running pods in ns "default" (the reference's
        resources.New("") namespace) whose first envFrom ConfigMap holding
        CUDA_VISIBLE_DEVICES names one of the node's UUIDs (gpu_plugins.go:87-160)."""
        res = self._res("default", f"spec.nodeName={node_name}")
        uuid_set = set(uuids)
        out: Dict[str, Dict[str, float]] = {}
        # the reference's ListPods ignores the field selector (pods.go:54-61)
        for pod in Resources(res.client, "default", "", res.pod_lister, res.cm_lister).list_pods():
            if O.phase(pod) != "Running":
                continue
            uuid = ""
            for cm_name in O.env_from_config_maps(pod, first_container_only=True):
                cm = res.get_config_map(cm_name)
                if cm is None:
                    continue
                v = (cm.get("data") or {}).get(C.ENV_CUDA_VISIBLE)
                if v is not None:
                    uuid = v
                    break
            if not uuid or uuid not in uuid_set:
                continue
            raw = O.get_env(pod, C.ENV_SLO)
            if raw == "":
                continue
            out.setdefault(uuid, {})[O.name(pod)] = float(raw)   # ValueError propagates like Go
        return out

    # ---------------------------------------------------------------- reconfigure (A30)
    def reconfigure(self, node_name: str, slo: float, pod: Obj) -> None:
        r = self._redis()
        conf = self._conf(O.name(pod))
        idx = reconfigure_choice(conf, slo, "A30", fixed=False)
        res = self._res(C.REDIS_NAMESPACE)
        res.label_node(node_name, {C.LABEL_MIG_CONFIG: C.MIG_CONFIGS[idx]}, "replace",
                       parity_master=self.p.args.parity_master or None)
        prof = None
        for q in res.list_pods():
            if C.PROFILER_POD_SUBSTR in O.name(q) and O.node_name_of(q) == node_name:
                prof = q
                break
        if prof is not None:
            res.delete_pod(O.name(prof), 0)
        if r is None:
            return
        val = r.get_or(node_name)
        deadline = time.monotonic() + self.p.args.reconfigure_timeout_s
        poll = getattr(self.p, "reconfigure_poll_s", C.RECONFIGURE_POLL_S)
        time.sleep(poll)
        while r.get_or(node_name) == val:
            if time.monotonic() > deadline:
                log.warning("reconfigure of %s: UUIDs did not change within %.0fs", node_name,
                            self.p.args.reconfigure_timeout_s)
                return
            time.sleep(poll)

    # ---------------------------------------------------------------- Logic
    def logic(self, node_name: str, pod: Obj) -> int:
        score = C.MIN_NODE_SCORE
        selected = ""
        raw = O.get_env(pod, C.ENV_SLO)
        try:
            cur_slo = float(raw) if raw else 0.0
        except ValueError:
            cur_slo = 0.0
        node = self.p.handle.snapshot().get(node_name)
        node_obj = node.node if node is not None else {"metadata": {"name": node_name}}
        model = O.node_gpu_model(node_obj, parity_names=True)
        r = self._redis()
        pod_res = self._res(O.namespace(pod))
        if model == "A30":
            with _A30_MUTEX:
                empty = True
                for q in pod_res.list_pods():
                    if O.phase(q) in ("Running", "Pending") and O.node_name_of(q) == O.name(pod):
                        empty = False       # compares NodeName to the pod's *name* (quirk #2)
                        break
                if empty and r is not None and self.p.args.parity_reconfigure:
                    try:
                        self.reconfigure(node_name, cur_slo, pod)
                    except Exception as e:   # the reference ignores the error (:494)
                        log.info("reconfigure failed: %s", e)
        if r is None:
            # DCGM/Prometheus fallback; the reference computes then returns 0 (:508-527)
            return 0
        uuids = schema.read_uuids(r, node_name) or []
        slos = self.get_slos(node_name, uuids)
        if model:
            if self.p.args.parity_shuffle:
                self.rng.shuffle(uuids)
            # The reference scores UUID by UUID with the recommender calls and the V100
            # ConfigMap write inside the loop (:558-757); the calls and side effects are
            # kept per UUID here, and the scores are then computed as one batch
            # (scoring.score_devices -> the native C++ core on busy nodes), identical numerics.
            col = f"{len(uuids)}P_{model}"
            per_uuid = []
            pred, intf = -1.0, {}
            for uuid in uuids:
                residents = [Resident(n, s, self._conf(n), self._intf(f"{n}_{model}"))
                             for n, s in (slos.get(uuid) or {}).items()]
                conf = self._conf(O.name(pod))
                pred = -1.0
                if model == "A30":
                    pred = conf.get(col, 0.0)          # missing key -> zero value (:637)
                elif model == "V100":
                    idx, pred = pick_mps_config(conf, cur_slo, "V100")
                    pod_res.append_to_existing_config_maps_in_pod(O.name(pod), {f"MPS_{node_name}": idx}, True)
                intf = self._intf(f"{O.name(pod)}_{model}") if pred != -1 else {}
                # residents are excluded from their own interference sum; the incoming pod
                # is never a resident here (it is not Running on this UUID).
                per_uuid.append((uuid, residents))
            scores = score_devices([r for _, r in per_uuid], O.name(pod), cur_slo, pred, intf, col)
            for (uuid, _), tmp in zip(per_uuid, scores):
                if int(tmp) > score:
                    score = int(tmp)
                    selected = uuid
        pod_res.append_to_existing_config_maps_in_pod(O.name(pod), {node_name: selected}, True)
        return score

    # ---------------------------------------------------------------- PostBind
    def post_bind(self, pod: Obj, node_name: str) -> None:
        r = self._redis()
        if r is None:
            raise RuntimeError("Redis not found")       # klog.Fatal in the reference (:852)
        uuids = schema.read_uuids(r, node_name)
        if uuids is None:
            raise RuntimeError(f"Error occured in redis.Get() in PostBind: no key {node_name}")
        names = O.env_from_config_maps(pod, first_container_only=True)
        res = self._res(O.namespace(pod))
        cm = res.get_config_map(names[0]) if names else None
        if cm is None or not uuids:
            return
        uuid = uuids[self.rng.randrange(len(uuids))]
        mem, thr = "", ""
        for k, v in (cm.get("data") or {}).items():
            if k == node_name:
                uuid = v
            elif k == f"MPS_{node_name}":
                mem, thr = mps_env(v)
        if uuid:
            res.append_to_existing_config_maps_in_pod(O.name(pod), {
                C.ENV_CUDA_VISIBLE: uuid, C.ENV_MPS_MEM: mem, C.ENV_MPS_THREADS: thr}, True)
