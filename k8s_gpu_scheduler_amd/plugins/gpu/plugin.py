"""The "GPU" scheduler plugin for MI355X nodes.

Reference: `type GPU` implementing Score + NormalizeScore + PostBind
(reference pkg/plugins/gpu_plugin/gpu_plugins.go:39-44,779-926).  Two modes:

* ``mode: parity`` -- reproduces the reference behaviour exactly (`parity.ParityLogic`):
  node model from the node name, UUIDs from Redis, residents' SLOs from their
  ConfigMaps' CUDA_VISIBLE_DEVICES, one recommender RPC per lookup, shuffled UUIDs,
  ConfigMap writes inside Score, A30 MIG reconfigure, random-UUID PostBind with MPS env.
  Used to pass the SURVEY §2.7.4 parity vectors.

* ``mode: fixed`` (default) -- the MI355X design, fixing SURVEY §2.9 #1-#10:
  PreFilter parses the GPU request (whole GPUs / partitions, or fractional CUs + HBM);
  Filter checks per-device capacity in the ledger (32-CU mask-word units + HBM) and, for
  multi-GPU pods, an xGMI clique (`topology.select_gpu_set`); PreScore fetches the
  incoming pod's predictions once; Score evaluates every candidate device with the
  reference's SLO/interference objective (the `scoring.device_score` terms, evaluated
  incrementally from a cached per-device resident summary, `scoring.fast_device_score`)
  blended with unit-packing and live telemetry terms -- no I/O, no side effects;
  NormalizeScore is the reference's min-max; Reserve/Unreserve commit the device choice
  to the ledger; PreBind writes the device env (ROCR_VISIBLE_DEVICES, HIP_VISIBLE_DEVICES,
  HSA_CU_MASK, HBM cap; reference CUDA_* keys with `compatEnv`) into the pod's envFrom
  ConfigMaps and annotations *before* bind, so the container starts with it (§2.9 #7).
"""
from __future__ import annotations

import dataclasses
import json
import logging
import math
import random
import threading
import time
from dataclasses import dataclass, field
from typing import Any, Dict, List, Optional, Tuple

from ...api import constants as C
from ...api import objects as O
from ...framework.interface import (CycleState, FilterPlugin, NodeScore, PostBindPlugin, PreBindPlugin,
                                    PreFilterPlugin, PreScorePlugin, QueueSortPlugin, ReservePlugin, ScoreExtensions,
                                    ScorePlugin, Status, min_max_normalize)
from ...kube.resources import Resources
from ...recommender.client import CachedPredictions, PredictionProvider, RecommenderClient, RpcPredictions
from ...telemetry.cache import TelemetryCache
from .devices import (CUS_PER_XCD, Device, DeviceLedger, DeviceState, cu_slice_mask, devices_for_node,
                      hsa_cu_mask_ranges)
from .scoring import DeviceSummary, build_device_summary, fast_device_score, workload_column
from .topology import XGMI_GPU_BPS, Topology, select_gpu_set

log = logging.getLogger(__name__)
Obj = Dict[str, Any]

_REQ = "GPU/request"
_PRED = "GPU/predictions"
_CHOICE = "GPU/choice"
_CANDS = "GPU/candidates"
_SIG = "GPU/signature"
_PLAN = "GPU/plan"
BIND_ANNOTATIONS = "bind/annotations"


@dataclass
class GpuRequest:
    whole: int = 0          # whole devices (GPUs or partitions)
    units: int = 0          # XCD units for a fractional pod
    cu: int = 0
    hbm_gib: float = 0.0
    slo: float = 0.0
    gpu_pod: bool = False
    burstable: bool = False
    implicit: bool = False  # SLO env only, no amd.com/* request: GPU preferred, not required
    isolated: bool = False  # needs its own compute partition (ANNOT_ISOLATION = "partition")
    part_cus: int = 0       # ... of this many CUs (0 = not sized yet)
    part_min: bool = False  # part_cus is a floor (SLO-sized): any larger free partition will do
    iters: float = 0.0      # iterations of a batch pod (ITERATIONS env; 0 = long-running service)


PARTITION_SIZES = tuple(C.MI355X_CUS // p for p in sorted(C.COMPUTE_PARTITIONS.values(), reverse=True))  # 32..256


def partition_size(cus: int) -> int:
    """Smallest MI355X compute-partition size (CPX 32 .. SPX 256 CUs) holding `cus`."""
    for s in PARTITION_SIZES:
        if cus <= s:
            return s
    return C.MI355X_CUS


@dataclass
class Choice:
    node: str
    allocs: List[Tuple[str, int, int, float, bool]] = field(default_factory=list)  # uuid,u0,n,hbm,whole
    score: float = 0.0
    devices: List[Device] = field(default_factory=list)
    burstable: bool = False


@dataclass
class GPUArgs:
    mode: str = "fixed"
    w_slo: float = 1.0
    w_pack: float = 1.0
    w_telemetry: float = 0.5
    # least-predicted-load across a node's GPUs: each resident pod's predicted GPU time
    # (ITERATIONS / predicted whole-GPU throughput, or SLO / throughput for services)
    w_balance: float = 0.0
    # roofline complementarity: prefer the GPU whose residents plus this pod split their
    # predicted time most evenly between MFMA-bound and HBM-bound work (needs a roofline
    # provider in the handle extras: name -> (mfma s, hbm s) per iteration)
    w_complement: float = 0.0
    # queueSort (when GPU is the profile's queueSort plugin): pods arriving in the same
    # window are popped longest-predicted-work first (LPT), older windows first
    lpt_window_s: float = 1.0
    # plan a burst of pending fractional pods jointly (plugins.gpu.planner): pairings that
    # keep predicted SLOs under interference, within planTolerance of the balanced load
    plan_bursts: bool = False
    plan_tolerance: float = 0.05
    # "slo": most predicted SLOs met first, then the lower busier GPU; "load": the lower
    # interference-adjusted load of the busier GPU first, SLO count as the tie-break
    plan_objective: str = "slo"
    # SLO objective of Score: "auto" = the co-run constraint when the prediction provider
    # serves a co-run model (models.corun), else the reference's per-pod terms; "corun" /
    # "terms" force one.  Co-run constraint: a device whose GPU group would, with this pod,
    # miss fewer predicted SLOs always ranks first (bands by the number of NEW misses), the
    # other terms (packing, balance by predicted group makespan, telemetry) order a band.
    slo_objective: str = "auto"
    # headroom the co-run model's predicted throughput must clear over an SLO to count as met
    # (its held-out error is ~9 %: without headroom a plan that just meets an SLO on paper
    # misses it about half the time)
    corun_margin: float = 0.0
    # the burst planner's soft objective: expected SLOs met when the model's log error is
    # N(0, sigma^2) (held-out: mean |log error| 0.093 -> sigma ~0.12); 0 = hard counts
    corun_sigma: float = 0.0
    # co-run planner backlog carry: each GPU's predicted work from earlier bursts beyond the
    # least-loaded GPU's is carried into the next plans (multiplied by this factor per burst;
    # 0 = every burst planned on its own).  In a pipelined multi-GPU job the busiest GPU's
    # CUMULATIVE work paces the run, and per-burst slack for SLOs otherwise random-walks
    plan_carry: float = 0.0
    # co-run planner: also choose each planned pod's CU slot on its GPU, simulating the GPU's
    # slot pipelines (in-flight pods of earlier placements, measured ones pinned; see
    # plugins.gpu.timeline) -- the most expected SLOs met among slot assignments whose slot
    # ends stay within slotSpreadMs of the most even assignment's
    plan_slots: Any = False           # "" / False: off, "lpt", "model" / True (planner.BurstPlanner)
    # per-burst planning budget (ms; 0 = none): each burst plan's wall time is measured and the
    # planner's effort level follows it (planner.EffortController: a burst over budget -> the
    # cheapest level predicted to fit, under half of it -> one level back up); exported as
    # gpusched_plan_effort_level / gpusched_plan_ms
    plan_budget_ms: float = 0.0
    slot_spread_ms: float = 2.0
    slot_sigma: float = 0.2
    pack: str = "binpack"             # binpack (MostAllocated) | spread (LeastAllocated) | random
    model: str = C.MI355X
    default_cu: int = 64              # implied request for SLO-only pods (reference-style pods)
    compat_env: bool = True
    predictions: str = "cache"        # cache | rpc | none
    recommender: str = ""
    redis: str = ""
    redis_password: str = C.REDIS_PASSWORD
    prometheus: str = ""
    parity_master: str = ""
    parity_reconfigure: bool = True
    reconfigure_timeout_s: float = 60.0
    parity_shuffle: bool = True
    seed: Optional[int] = None
    # partition controller (plugins.gpu.partitioner): "auto" re-partitions idle nodes for
    # pending pods that ask for an isolated partition; "off" never requests a change
    partitioning: str = "auto"
    # an SLO-only pod (no amd.com/* request) whose SLO no fractional share can meet -- its
    # predicted throughput at the default share is below it -- becomes an isolated-partition
    # request sized from its predictions (the reference drives the MIG layout from every A30
    # pod's predictions, gpu_plugins.go:357-399,478-496)
    slo_partitioning: bool = True
    partition_period_s: float = 2.0
    partition_backoff_s: float = 600.0     # a node that refused / failed a mode is not asked again for it

    @classmethod
    def from_dict(cls, d: Dict[str, Any]) -> "GPUArgs":
        a = cls()
        alias = {"weightSLO": "w_slo", "weightPack": "w_pack", "weightTelemetry": "w_telemetry",
                 "weightBalance": "w_balance", "weightComplement": "w_complement",
                 "lptWindowSeconds": "lpt_window_s",
                 "planBursts": "plan_bursts", "planTolerance": "plan_tolerance",
                 "planObjective": "plan_objective", "sloObjective": "slo_objective", "corunMargin": "corun_margin", "corunSigma": "corun_sigma",
                 "planCarry": "plan_carry", "planSlots": "plan_slots", "planBudgetMs": "plan_budget_ms", "slotSpreadMs": "slot_spread_ms", "slotSigma": "slot_sigma",
                 "defaultCU": "default_cu", "compatEnv": "compat_env", "redisPassword": "redis_password",
                 "parityMaster": "parity_master", "parityReconfigure": "parity_reconfigure",
                 "reconfigureTimeoutSeconds": "reconfigure_timeout_s", "parityShuffle": "parity_shuffle",
                 "partitionPeriodSeconds": "partition_period_s", "sloPartitioning": "slo_partitioning", "partitionBackoffSeconds": "partition_backoff_s"}
        for k, v in (d or {}).items():
            k = alias.get(k, k)
            if hasattr(a, k):
                setattr(a, k, v)
        return a


class GPUPlugin(QueueSortPlugin, PreFilterPlugin, FilterPlugin, PreScorePlugin, ScorePlugin, ScoreExtensions, ReservePlugin,
                PreBindPlugin, PostBindPlugin):
    NAME = C.PLUGIN_NAME

    def __init__(self, args: Optional[Dict[str, Any]] = None, handle: Any = None,
                 predictions: Optional[PredictionProvider] = None, redis: Any = None,
                 telemetry: Optional[TelemetryCache] = None, ledger: Optional[DeviceLedger] = None):
        self.args = GPUArgs.from_dict(args or {})
        self.handle = handle
        extras = getattr(handle, "extras", {}) if handle is not None else {}
        self.telemetry = telemetry or extras.get("telemetry") or TelemetryCache()
        self.ledger = ledger or extras.get("ledger") or DeviceLedger()
        self.redis = redis if redis is not None else extras.get("redis")
        self.predictions = predictions or extras.get("predictions")
        self.workcost = extras.get("workcost")      # telemetry.workcost.WorkCostModel (optional)
        self.roofline = extras.get("roofline")      # name -> (mfma s, hbm s) per iteration, or None
        # native node scoring: interned names / interference columns and per-node packs
        self._name_ids: Dict[str, int] = {}
        self._col_ids: Dict[str, int] = {}
        self._packs: Dict[str, Tuple[Any, Dict[str, Any]]] = {}
        self._pack_seen: Dict[str, Any] = {}
        self._xvec_memo: Any = None
        self._core_mod: Any = False
        self._weights_vec: Any = None
        import numpy as _np
        self._empty_vec = _np.zeros(0)
        self._mfma_frac: Dict[str, Optional[float]] = {}
        self.topologies: Dict[str, Topology] = dict(extras.get("topologies") or {})
        self._resident_memo: Dict[str, Tuple[Dict[str, float], Dict[str, float]]] = {}
        self._col_memo: Dict[str, Optional[str]] = {}
        self._cands_memo: Dict[str, Tuple[Any, List[Tuple[DeviceState, int]]]] = {}
        self._score_memo: Dict[str, Tuple[Any, Optional[Choice]]] = {}
        self._col_cache: Dict[Tuple[int, int], str] = {}
        self._pending_by_key: Dict[str, Obj] = {}
        self._corun_packs: Dict[str, Tuple[Any, Dict[str, Any]]] = {}
        self.planner = None
        if self.args.plan_bursts:
            from .planner import BurstPlanner
            self.planner = BurstPlanner(self, self.args.plan_tolerance, objective=self.args.plan_objective,
                                        carry=self.args.plan_carry, slots=self.args.plan_slots,
                                        spread_ms=float(self.args.slot_spread_ms),
                                        slot_sigma=float(self.args.slot_sigma))
            self.planner.set_budget(float(self.args.plan_budget_ms or 0.0))
        self._pred_version: Any = None
        self._lock = threading.RLock()
        self._rng = random.Random(self.args.seed)
        self._client: Optional[RecommenderClient] = None
        self.SCORE_DOES_IO = self.args.mode == "parity"
        if self.predictions is None and self.args.recommender and self.args.predictions != "none":
            self._client = RecommenderClient(self.args.recommender)
            self.predictions = (RpcPredictions(self._client) if self.args.predictions == "rpc"
                                else CachedPredictions(self._client))
        if self.redis is None and self.args.redis:
            from ...store.resp import Redis
            self.redis = Redis.connect(self.args.redis, self.args.redis_password)
        self.parity = None
        if self.args.mode == "parity":
            from .parity import ParityLogic
            self.parity = ParityLogic(self)
        self.partitioner = None
        if handle is not None:
            self._wire_informers()
            if self.args.mode != "parity" and self.args.partitioning == "auto":
                from .partitioner import PartitionController
                self.partitioner = PartitionController(self, period_s=self.args.partition_period_s,
                                                       backoff_s=self.args.partition_backoff_s)

    # ------------------------------------------------------------------ wiring
    def _wire_informers(self) -> None:
        try:
            inf = self.handle.informer_factory
        except AttributeError:
            return
        inf.nodes().add_event_handler(self._on_node, lambda o, n: self._on_node(n), None)
        inf.pods().add_event_handler(self._on_pod, lambda o, n: self._on_pod(n), self._on_pod_delete)

    def _on_node(self, node: Obj) -> None:
        name = O.name(node)
        uuids, descs = None, None
        if self.redis is not None:
            try:
                from ...store import schema
                uuids = schema.read_uuids(self.redis, name)
                descs = schema.read_devices(self.redis, name)
                topo = self.redis.get_or(schema.topology_key(name))
                if topo:
                    self.topologies[name] = Topology.from_json(json.loads(topo))
            except Exception as e:
                log.debug("redis inventory for %s unavailable: %s", name, e)
        devs = devices_for_node(node, uuids, descs)
        self.ledger.set_devices(name, devs)
        if name not in self.topologies:
            n_gpu = max((d.gpu for d in devs), default=-1) + 1
            if n_gpu:
                self.topologies[name] = Topology.fully_connected(n_gpu)

    def _on_pod(self, pod: Obj) -> None:
        """Rebuild reservations of assigned pods from their annotations (scheduler restart
        recovery) and release finished ones."""
        if O.is_terminal(pod):
            fb = getattr(self.planner, "feedback", None) if self.planner is not None else None
            if fb is not None:
                fb.completed(pod)       # measured vs predicted time -> its GPU's measured speed
            if self.planner is not None:
                self.planner.released(pod, "terminal")
            self.ledger.release(O.key(pod))
            return
        node = O.node_name_of(pod)
        ann = O.annotations(pod).get(C.ANNOT_DEVICES)
        if not node or not ann or self.ledger.placement(O.key(pod)) is not None:
            return
        try:
            allocs = json.loads(O.annotations(pod).get(C.ANNOT_DEVICE_INDICES, "[]"))
            allocs = [tuple(a) for a in allocs]
        except json.JSONDecodeError:
            return
        if allocs:
            if not self.ledger.has_node(node):
                # informers may deliver pods before their node (start order): load the node
                try:
                    self._on_node(self.handle.client.get("nodes", node))
                except Exception as e:
                    log.debug("recovery: node %s of %s unavailable: %s", node, O.key(pod), e)
            work = self.pod_work(pod, self._pod_predictions(O.name(pod))[0])
            self.ledger.reserve(node, O.key(pod), O.name(pod), O.pod_slo(pod), allocs, work=work,
                                iters=float(O.pod_iterations(pod)))

    def _on_pod_delete(self, pod: Obj) -> None:
        fb = getattr(self.planner, "feedback", None) if self.planner is not None else None
        terminal = O.is_terminal(pod)
        if fb is not None:
            if terminal:
                fb.completed(pod)
            fb.forget(O.key(pod))
        self.ledger.release(O.key(pod))
        if self.planner is not None:
            self.planner.released(pod, "terminal" if terminal else "delete")
            self.planner.consume(O.key(pod))

    # ------------------------------------------------------------------ request
    def parse_request(self, pod: Obj) -> GpuRequest:
        g, cu, mem = O.gpu_request(pod)
        slo = O.pod_slo(pod)
        r = GpuRequest(slo=slo, hbm_gib=mem, burstable=O.gpu_qos(pod) == "Burstable",
                       iters=float(O.pod_iterations(pod)))
        ann = O.annotations(pod)
        if ann.get(C.ANNOT_ISOLATION) == "partition":
            # one whole compute partition of the requested (or controller-chosen) size
            size = cu if cu > 0 else int(float(ann.get(C.ANNOT_PARTITION_CUS) or 0))
            r.isolated, r.gpu_pod, r.whole = True, True, 1
            r.part_cus = partition_size(size) if size > 0 else 0
            r.cu = r.part_cus
            return r
        if cu > 0:
            r.cu = min(cu, C.MI355X_CUS)
            r.units = max(1, math.ceil(r.cu / CUS_PER_XCD))
            r.gpu_pod = True
        elif g > 0:
            r.whole = g
            r.gpu_pod = True
        elif mem > 0 or slo > 0:
            r.cu = self.args.default_cu
            r.units = max(1, math.ceil(r.cu / CUS_PER_XCD))
            r.gpu_pod = True
            # the reference scores every SLO-labelled pod but never filters one out
            # (busybox on a CPU-only cluster still schedules): only an explicit
            # amd.com/* request makes the GPU a hard requirement
            r.implicit = mem <= 0
            size = self.slo_partition_size(pod, slo) if (r.implicit and slo > 0) else None
            if size:
                # a floor, not an exact shape: a busy SPX node's free 256-CU GPU meets the SLO
                # better than a 128-CU partition the controller may never get to cut
                r.isolated, r.whole, r.implicit, r.part_min = True, 1, False, True
                r.part_cus = r.cu = size
                r.units = 0
                return r
        # round fractional units up to a power of two (aligned XCD groups)
        if r.units:
            p = 1
            while p < r.units:
                p *= 2
            r.units = min(p, C.MI355X_XCDS)
            r.cu = r.units * CUS_PER_XCD
        return r

    def slo_partition_size(self, pod: Obj, slo: float) -> Optional[int]:
        """CUs of the isolated partition an SLO-only pod needs when no fractional share can
        meet its SLO (predicted throughput at the default share below the SLO), sized like
        the reference's MIG choice: the smallest partition whose prediction still meets it
        (partitioner.size_from_predictions); None = a fractional share will do, or no
        predictions (then the reference's behaviour: score it, never filter it)."""
        if not self.args.slo_partitioning or self.predictions is None or self.args.mode == "parity":
            return None
        conf = self._pod_predictions(O.name(pod))[0]
        if not conf:
            return None
        share = conf.get(self._col(max(1, math.ceil(self.args.default_cu / CUS_PER_XCD)), C.MI355X_XCDS))
        if share is None or share >= slo:
            return None
        from .partitioner import size_from_predictions
        return size_from_predictions(conf, slo, self.args.model)

    # ------------------------------------------------------------------ extension points
    def pre_filter(self, state: CycleState, pod: Obj) -> Optional[Status]:
        if self.parity is not None:
            return None
        req = self.parse_request(pod)
        state.write(_REQ, req)
        if not req.gpu_pod:
            return Status.skip()
        return None

    def filter(self, state: CycleState, pod: Obj, node_info: Any) -> Optional[Status]:
        if self.parity is not None:
            return None
        req: GpuRequest = state.read(_REQ) or self.parse_request(pod)
        node = node_info.node
        for t in O.node_taints(node):
            if t.get("key") == C.TAINT_PARTITIONING:
                return Status.unschedulable("node is being re-partitioned", self.NAME)
            if t.get("key") == C.TAINT_PROBING:
                return Status.unschedulable("node's GPU fabric is being probed", self.NAME)
        if not self.ledger.has_node(node_info.name):
            self._on_node(node)
        if req.isolated and not req.part_cus:
            return Status.unschedulable("waiting for partition sizing", self.NAME)
        removed = getattr(node_info, "removed", None)
        if removed:                 # preemption what-if: victims' units/HBM released
            if self._fits_without(req, node_info.name, removed):
                return None
            return Status.unschedulable("insufficient free GPU units/HBM even without lower-priority pods", self.NAME)
        choice = self._best_choice(state, pod, req, node_info.name, scoring=False)
        if choice is None and req.isolated:
            mode = C.PARTITIONS_TO_MODE.get(C.MI355X_CUS // req.part_cus, "?")
            return Status.unschedulable(f"no free {mode} partition ({req.part_cus} CUs)", self.NAME)
        if choice is None and not req.implicit:
            return Status.unschedulable("insufficient free GPU units/HBM or no xGMI clique", self.NAME)
        return None

    def filter_nodes(self, state: CycleState, pod: Obj, node_infos: List[Any]) -> List[Optional[Status]]:
        """Batch Filter (framework chunked filtering): the request is parsed once; nodes
        under a preemption what-if or not yet in the ledger take the per-node path."""
        if self.parity is not None:
            return [None] * len(node_infos)
        req: GpuRequest = state.read(_REQ) or self.parse_request(pod)
        if req.isolated:                # rare: the per-node path (with its partition messages)
            return [self.filter(state, pod, ni) for ni in node_infos]
        out: List[Optional[Status]] = []
        memo = state.read(_CANDS)
        if memo is None:
            memo = {}
            state.write(_CANDS, memo)
        node_gen, cmemo, has_node = self.ledger.node_gen, self._cands_memo, self.ledger.has_node
        frac = not req.whole
        for ni in node_infos:
            nn = ni.name
            if getattr(ni, "removed", None) or not has_node(nn) or O.node_taints(ni.node):
                out.append(self.filter(state, pod, ni))
                continue
            if frac:                    # inline memo hit of _best_choice(scoring=False)
                hit = cmemo.get(nn)
                if hit is not None and hit[0] == (node_gen.get(nn, 0), req.units, req.hbm_gib):
                    memo[nn] = hit[1]
                    ok = bool(hit[1])
                else:
                    ok = self._best_choice(state, pod, req, nn, scoring=False) is not None
            else:
                ok = self._best_choice(state, pod, req, nn, scoring=False) is not None
            out.append(None if ok or req.implicit else
                       Status.unschedulable("insufficient free GPU units/HBM or no xGMI clique", self.NAME))
        return out

    def planned_node(self, state: CycleState, pod: Obj) -> Optional[str]:
        """The node of this pod's burst plan, if one was made (the framework then filters only
        that node and skips Score: with this plugin's weight the plan decides anyway)."""
        if self.planner is None or self.parity is not None:
            return None
        hit = self.planner.plans.get(O.key(pod))
        return hit[0] if hit is not None else None

    def pre_score(self, state: CycleState, pod: Obj, nodes: List[Any]) -> Optional[Status]:
        if self.parity is not None:
            return None
        req: GpuRequest = state.read(_REQ)
        if req is None or not req.gpu_pod:
            return Status.skip()
        state.write(_PRED, self._pod_predictions(O.name(pod)))
        state.write(_CHOICE, {})
        if self.planner is not None and req.units and not req.whole:
            try:
                plan = self.planner.plan(pod, [n.name for n in nodes])
            except Exception as e:          # planning is an optimisation: never fail the cycle
                log.warning("burst planning failed: %s", e)
                plan = None
            state.write(_PLAN, plan)
        return None

    def score(self, state: CycleState, pod: Obj, node_name: str) -> Tuple[int, Optional[Status]]:
        if self.parity is not None:
            try:
                return self.parity.logic(node_name, pod), None
            except Exception as e:
                return 0, Status.error(f"Error in Logic() in Score(): {e}", self.NAME)
        req: GpuRequest = state.read(_REQ) or self.parse_request(pod)
        choice = self._apply_plan(state, req, node_name, self._best_choice(state, pod, req, node_name, scoring=True))
        if choice is None:
            return 0, None
        choices = state.read(_CHOICE)
        if choices is None:
            choices = {}
            state.write(_CHOICE, choices)
        choices[node_name] = choice
        return max(C.MIN_NODE_SCORE, min(C.MAX_NODE_SCORE, int(choice.score))), None

    def score_nodes(self, state: CycleState, pod: Obj, names: List[str]) -> Tuple[List[int], Optional[Status]]:
        """Batch Score over every feasible node (fixed mode; parity mode does I/O per node
        and keeps the per-node path)."""
        req: GpuRequest = state.read(_REQ) or self.parse_request(pod)
        choices = state.read(_CHOICE)
        if choices is None:
            choices = {}
            state.write(_CHOICE, choices)
        out = []
        lo, hi = C.MIN_NODE_SCORE, C.MAX_NODE_SCORE
        sig = self._pod_ctx(state, pod, req)[4] if not req.whole else None
        plan = state.read(_PLAN)
        node_gen, smemo, tele = self.ledger.node_gen, self._score_memo, self.telemetry
        use_t, stale = bool(self.args.w_telemetry), tele.stale_s
        for nn in names:
            hit = smemo.get(nn) if sig is not None else None
            if hit is not None:         # inline memo hit of _best_choice(scoring=True)
                tv = tele.node_version(nn) if use_t else 0
                skey = ((node_gen.get(nn, 0), req.units, req.hbm_gib),
                        (tv, int(time.monotonic()) if (tv and stale) else 0), sig)
                if hit[0] != skey:
                    hit = None
            planned = self._planned_choice(state, req, nn, plan) if plan is not None else None
            if planned is not None:         # the plan decides on its node: no scoring needed
                choice = planned
            else:
                choice = hit[1] if hit is not None else self._best_choice(state, pod, req, nn, scoring=True)
                if plan is not None:
                    choice = self._apply_plan(state, req, nn, choice)
            if choice is None:
                out.append(0)
                continue
            choices[nn] = choice
            out.append(max(lo, min(hi, int(choice.score))))
        return out, None

    def cache_signature(self, state: CycleState, pod: Obj, phase: str) -> Any:
        """Cycle-cache signature (framework.fastpath): everything a node's Filter verdict or
        raw Score depends on besides that node's ledger entry, telemetry samples and
        NodeInfo, which report their changes to the change log.  None = not cacheable:
        parity mode (I/O in Score), the burst planner (couples nodes), random packing."""
        if self.parity is not None or self.planner is not None:
            return None
        req: GpuRequest = state.read(_REQ) or self.parse_request(pod)
        rsig = (req.whole, req.units, req.cu, req.hbm_gib, req.isolated, req.part_cus, req.implicit, req.gpu_pod,
                req.iters, req.part_min and self._larger_ok(req))
        if phase != "score":
            return rsig
        if self.args.pack == "random":
            return None
        tele = self.telemetry
        # samples age out after stale_s: a per-second token bounds how long a cached score
        # can outlive its telemetry (the per-node memo uses the same granularity)
        tok = int(time.monotonic()) if (self.args.w_telemetry and tele.stale_s and tele.updates) else 0
        if req.whole:
            return rsig, tok
        sig = self._pod_ctx(state, pod, req)[4]
        return None if sig is None else (rsig, sig, tok, self._pred_version, id(self.corun_model()))

    def _planned_choice(self, state: CycleState, req: GpuRequest, node: str, plan: Any) -> Optional[Choice]:
        """The plan's device on its node as a top-scored Choice, if it is still a candidate."""
        pnode, puuid = plan[0], plan[1]
        pu0 = plan[2] if len(plan) > 2 else None
        if node != pnode:
            return None
        for st, u0 in (state.read(_CANDS) or {}).get(node) or []:
            if st.device.uuid == puuid:
                # the planned CU slot when it is still free (else the ledger's best fit)
                if pu0 is not None and pu0 + req.units <= len(st.used_units) and \
                        not any(st.used_units[pu0:pu0 + req.units]):
                    u0 = pu0
                return Choice(node, [(puuid, u0, req.units, req.hbm_gib, False)], float(C.MAX_NODE_SCORE),
                              [st.device])
        return None

    def _apply_plan(self, state: CycleState, req: GpuRequest, node: str,
                    choice: Optional[Choice]) -> Optional[Choice]:
        """Burst plan (planner.BurstPlanner): the planned device on the planned node scores
        100 and everything else below it; a stale plan (device no longer a candidate)
        leaves the normal choice."""
        plan = state.read(_PLAN)
        if plan is None:
            return choice
        if node == plan[0]:
            return self._planned_choice(state, req, node, plan) or choice
        if choice is not None and choice.score > C.MAX_NODE_SCORE - 1:
            choice = dataclasses.replace(choice, score=float(C.MAX_NODE_SCORE - 1))
        return choice

    NORMALIZE = "minmax"        # what normalize_score does (the cycle cache re-does it natively)

    def score_extensions(self) -> ScoreExtensions:
        return self

    def normalize_score(self, state: CycleState, pod: Obj, scores: List[NodeScore]) -> Optional[Status]:
        min_max_normalize(scores)
        return None

    def reserve(self, state: CycleState, pod: Obj, node_name: str) -> Optional[Status]:
        if self.parity is not None:
            return None
        req: GpuRequest = state.read(_REQ)
        if req is None or not req.gpu_pod:
            return None
        choice = (state.read(_CHOICE) or {}).get(node_name)
        if choice is None:
            plan = state.read(_PLAN)
            if plan is not None:            # a planned pod that skipped Score (planned_node)
                choice = self._planned_choice(state, req, node_name, plan)
        if choice is None:
            choice = self._best_choice(state, pod, req, node_name, scoring=True)
        if choice is not None:
            choice = dataclasses.replace(choice, burstable=req.burstable)   # memoised object: copy
        elif req.implicit:
            return None                 # no free GPU share: runs without one
        work = self.pod_work(pod, (state.read(_PRED) or self._pod_predictions(O.name(pod)))[0]) \
            if choice is not None else 0.0
        if choice is None or not self.ledger.reserve(node_name, O.key(pod), O.name(pod), req.slo, choice.allocs,
                                                     work=work, iters=req.iters):
            return Status.unschedulable("GPU capacity changed before reserve", self.NAME)
        state.write(_CHOICE + "/reserved", choice)
        if self.planner is not None:
            self.planner.placed(pod, node_name, choice, req)
            self.planner.consume(O.key(pod))
        return None

    def unreserve(self, state: CycleState, pod: Obj, node_name: str) -> None:
        if self.parity is not None:
            return
        self.ledger.release(O.key(pod))
        if self.planner is not None:
            self.planner.released(pod, "unreserve")
            self.planner.consume(O.key(pod))

    def pre_bind(self, state: CycleState, pod: Obj, node_name: str) -> Optional[Status]:
        if self.parity is not None:
            return None
        choice: Optional[Choice] = state.read(_CHOICE + "/reserved")
        if choice is None:
            return None
        env = self.device_env(choice)
        ann = {C.ANNOT_DEVICES: ",".join(a[0] for a in choice.allocs),
               C.ANNOT_DEVICE_INDICES: json.dumps([list(a) for a in choice.allocs]),
               C.ANNOT_CU_MASK: env.get(C.ENV_CU_MASK, "")}
        res = Resources(self.handle.client, O.namespace(pod))
        try:
            # Env into the pod's envFrom ConfigMaps BEFORE the bind (the kubelet reads them
            # at container creation -- fixes the reference's PostBind race).
            # Only into ConfigMaps no other live pod references: replicas sharing one
            # ConfigMap (reference deploy/busybox: 4 replicas -> one `game-demo`) would
            # overwrite each other's device (§2.9 #6); there the device identity is removed
            # and delivered per pod (Binding annotations -> device-plugin Allocate env).
            cms = O.env_from_config_maps(pod)
            if cms:
                shared = self._shared_config_maps(pod, cms)
                for cm in cms:
                    if cm in shared:
                        self._strip_device_env(res, cm, env)
                    else:
                        res.update_config_map(cm, env, True)
        except Exception as e:
            return Status.error(f"PreBind: writing device assignment failed: {e}", self.NAME)
        # The per-pod assignment annotations ride on the Binding itself (the apiserver
        # copies Binding.metadata.annotations onto the pod), saving one PATCH per pod.
        bind_ann = state.read(BIND_ANNOTATIONS) or {}
        bind_ann.update(ann)
        state.write(BIND_ANNOTATIONS, bind_ann)
        state.write("GPU/env", env)
        return None

    def _shared_config_maps(self, pod: Obj, cms: List[str]) -> set:
        """envFrom ConfigMaps of `pod` that another non-terminal pod (bound or pending) of the
        namespace also references."""
        ns, me = O.namespace(pod), O.key(pod)
        try:
            others = self.handle.informer_factory.pods().lister.list(namespace=ns)
        except Exception:
            others = self.handle.client.list("pods", ns)[0]
        want = set(cms)
        out = set()
        for p in others:
            if O.key(p) == me or O.is_terminal(p):
                continue
            out |= want & set(O.env_from_config_maps(p))
            if out == want:
                break
        return out

    @staticmethod
    def _strip_device_env(res: Resources, cm: str, env: Dict[str, str]) -> None:
        cur = res.get_config_map(cm)
        data = (cur or {}).get("data") or {}
        stale = [k for k in env if k in data]
        if stale:       # JSON merge patch: null deletes the key
            res.client.patch("configmaps", cm, {"data": {k: None for k in stale}}, "merge", res.namespace)

    def post_bind(self, state: CycleState, pod: Obj, node_name: str) -> None:
        if self.parity is not None:
            self.parity.post_bind(pod, node_name)

    def close(self) -> None:
        if self._client is not None:
            self._client.close()

    # ------------------------------------------------------------------ env
    def device_env(self, choice: Choice) -> Dict[str, str]:
        """Container env for a placement.  ROCR_VISIBLE_DEVICES filters the devices the ROCm
        runtime enumerates, so every index after it is RELATIVE to that list: HIP sees the
        pod's devices as 0..n-1, and HSA_CU_MASK addresses its (single) fractional device as
        GPU 0, in ROCr's `<gpu>:<cu ranges>` syntax.  The physical GPU indices stay in the
        device-indices annotation."""
        devs = {d.uuid: d for d in choice.devices}
        uuids = [a[0] for a in choice.allocs]
        env = {C.ENV_ROCR_VISIBLE: ",".join(uuids), C.ENV_HIP_VISIBLE: ",".join(str(i) for i in range(len(uuids)))}
        frac = [a for a in choice.allocs if not a[4]]
        if frac:
            u, u0, n, hbm, _ = frac[0]
            env[C.ENV_HBM_LIMIT] = f"{hbm:g}"
            if not choice.burstable:
                d = devs.get(u)
                first = (d.first_xcd if d else 0) + u0
                env[C.ENV_CU_MASK] = f"{uuids.index(u)}:{hsa_cu_mask_ranges(cu_slice_mask(first, n))}"
        if self.args.compat_env:
            env[C.ENV_CUDA_VISIBLE] = env[C.ENV_ROCR_VISIBLE]
            if frac:
                n = frac[0][2]
                env[C.ENV_MPS_THREADS] = str(int(100 * n / C.MI355X_XCDS))
                env[C.ENV_MPS_MEM] = f"0={int(frac[0][3] * 1024)}MB" if frac[0][3] else ""
            else:
                env[C.ENV_MPS_THREADS] = ""
                env[C.ENV_MPS_MEM] = ""
        return env

    # ------------------------------------------------------------------ queue sort
    def less(self, a: Any, b: Any) -> bool:
        """QueueSort: priority first (PrioritySort), then arrival window, then the longest
        predicted work first inside a window -- longest-processing-time-first list
        scheduling, which with the least-loaded balance term keeps a burst of pods evenly
        spread over a node's GPUs.  Windows keep the order a strict weak ordering and
        bound how long a short pod can be overtaken (one window)."""
        ka, kb = self._sort_key(a), self._sort_key(b)
        return ka < kb

    def sort_key(self, pi: Any) -> Tuple[int, int, float, float]:
        """Total-order key of `less` (the scheduling queue keys its heap with it)."""
        return self._sort_key(pi)

    def _sort_key(self, pi: Any) -> Tuple[int, int, float, float]:
        d = pi.__dict__
        hit = d.get("_gpu_sort")
        if hit is not None and hit[0] is pi.pod and hit[2] == pi.timestamp:
            return hit[1]
        pod = pi.pod
        w = self.args.lpt_window_s
        window = int(pi.timestamp // w) if w > 0 else 0
        work = self.pod_work(pod, self._pod_predictions(O.name(pod))[0]) if w > 0 else 0.0
        key = (-O.priority(pod), window, -work, pi.timestamp)
        d["_gpu_sort"] = (pod, key, pi.timestamp)    # requeueing restamps the pod: recompute
        return key

    def pod_work(self, pod: Obj, conf: Dict[str, float]) -> float:
        """Predicted whole-GPU time of a pod: ITERATIONS x seconds per iteration for a
        batch pod, SLO x seconds per iteration (the GPU fraction it needs) for a service;
        0 without a prediction.  Seconds per iteration come from the observed co-run cost
        of the pod's workload (telemetry.workcost, fed by the executors) when there is
        one, else 1 / the predicted whole-GPU throughput (Burstable co-running pods share
        every CU, so the whole-GPU rate is the denominator for the load they add)."""
        spi = self.workcost.seconds_per_iter(O.name(pod)) if self.workcost is not None else None
        if spi is None:
            tput = (conf.get(f"1P_{self.args.model}") or 0.0) if conf else 0.0
            if tput <= 0:
                return 0.0
            spi = 1.0 / tput
        iters = O.pod_iterations(pod)
        return (iters if iters > 0 else O.pod_slo(pod)) * spi

    # ------------------------------------------------------------------ predictions
    def _pod_predictions(self, name: str) -> Tuple[Dict[str, float], Dict[str, float]]:
        if self.predictions is None:
            return {}, {}
        ver_fn = getattr(self.predictions, "version", None)
        ver = ver_fn() if ver_fn is not None else None
        with self._lock:
            if ver != self._pred_version:       # a new model version: forget memoised lookups
                self._pred_version = ver
                self._resident_memo.clear()
                self._col_memo.clear()
                self._score_memo.clear()
                self.ledger.invalidate_summaries()
            hit = self._resident_memo.get(name)
        if hit is not None:
            return hit
        try:
            conf = self.predictions.configurations(name)
            intf = self.predictions.interference(f"{name}_{self.args.model}")
        except Exception as e:  # recommender down -> degrade to packing/telemetry
            log.debug("predictions for %s unavailable: %s", name, e)
            return {}, {}
        with self._lock:
            if len(self._resident_memo) > 65536:
                self._resident_memo.clear()
            self._resident_memo[name] = (conf, intf)
        return conf, intf

    # ------------------------------------------------------------------ device choice
    def _col(self, units: int, dev_units: int) -> str:
        k = (units, dev_units)
        c = self._col_cache.get(k)
        if c is None:
            c = self._col_cache[k] = f"{max(1, dev_units // max(units, 1))}P_{self.args.model}"
        return c

    def _workload_col(self, name: str, intf: Dict[str, float]) -> Optional[str]:
        hit = self._col_memo.get(name, False)
        if hit is False:
            hit = workload_column(name, intf) if intf else None
            if len(self._col_memo) > 65536:
                self._col_memo.clear()
            self._col_memo[name] = hit
        return hit

    def _device_summary(self, st: DeviceState) -> DeviceSummary:
        res = []
        for use in st.pods.values():
            conf, intf = self._pod_predictions(use.name)
            res.append((use.name, use.slo, conf.get(self._col(use.units[1], st.device.units)), intf))
        return build_device_summary(res)

    def _best_choice(self, state: CycleState, pod: Obj, req: GpuRequest, node: str,
                     scoring: bool) -> Optional[Choice]:
        """Best device choice on one node.  The returned Choice may be the memoised
        object itself (never mutated before Reserve, which copies it)."""
        if req.whole:
            states = self.ledger.devices(node)
            return self._whole_choice(req, node, states) if states else None
        memo = state.read(_CANDS)
        if memo is None:
            memo = {}
            state.write(_CANDS, memo)
        cands = memo.get(node)
        # Across cycles a node's candidates and best choice only change when its ledger
        # entry (node_gen) or its telemetry changes, so large clusters -- where almost
        # every node is untouched between two pods -- reuse them (the equivalence-cache
        # idea of kube-scheduler, keyed by node version x request signature).
        ckey = (self.ledger.node_gen.get(node, 0), req.units, req.hbm_gib)
        if cands is None:
            hit = self._cands_memo.get(node)
            if hit is not None and hit[0] == ckey:
                cands = hit[1]
            else:
                states = self.ledger.devices(node)
                cands = []
                for st in states:
                    if not st.device.healthy or st.hbm_free + 1e-6 < req.hbm_gib:
                        continue
                    u0 = st.find_units(req.units)
                    if u0 is None:
                        continue
                    cands.append((st, u0))
                self._cands_memo[node] = (ckey, cands)
            memo[node] = cands      # Filter computes, Score reuses (same cycle snapshot)
        if not cands:
            return None
        if not scoring:
            st, u0 = cands[0]
            return Choice(node, [(st.device.uuid, u0, req.units, req.hbm_gib, False)], 0.0, [st.device])
        name, conf, intf, work, sig = self._pod_ctx(state, pod, req)
        skey = None
        if sig is not None:
            tv = self.telemetry.node_version(node) if self.args.w_telemetry else 0
            tkey = (tv, int(time.monotonic()) if (tv and self.telemetry.stale_s) else 0)
            skey = (ckey, tkey, sig)
            hit = self._score_memo.get(node)
            if hit is not None and hit[0] == skey:
                return hit[1]
        best = self._score_cands(node, cands, req, name, conf, intf, work)
        if skey is not None:
            self._score_memo[node] = (skey, best)
        return best

    def _pod_ctx(self, state: CycleState, pod: Obj, req: GpuRequest) -> Tuple[str, Dict[str, float],
                                                                              Dict[str, float], float, Any]:
        """Pod-level inputs of Score, computed once per cycle: predictions, predicted work
        and the memo signature -- everything the score depends on besides the node (the
        request and the incoming pod's workload row, not its name); None = no memo
        (random packing)."""
        ctx = state.read(_SIG)
        if ctx is not None:
            return ctx
        a = self.args
        name = O.name(pod)
        conf, intf = state.read(_PRED) or self._pod_predictions(name)
        work = self.pod_work(pod, conf) if (a.w_balance or a.w_complement) else 0.0
        sig = None
        if a.pack != "random":
            x_col = self._workload_col(name, intf) if intf else None
            sig = (req.units, req.hbm_gib, req.slo, req.iters, work, x_col,
                   self.mfma_fraction(name) if a.w_complement else None,
                   tuple(sorted(conf.items())) if conf else (),
                   () if x_col is not None or not intf else tuple(sorted(intf.items())))
        ctx = (name, conf, intf, work, sig)
        state.write(_SIG, ctx)
        return ctx

    def _core(self) -> Any:
        if self._core_mod is False:
            try:
                from ... import _native
                self._core_mod = _native.core()
            except Exception:
                self._core_mod = None
            if self._core_mod is not None and not hasattr(self._core_mod, "NodePack"):
                self._core_mod = None           # an older build
        return self._core_mod

    def mfma_fraction(self, name: str) -> Optional[float]:
        """Share of a workload's alone time that is MFMA-bound (roofline provider), memoised."""
        hit = self._mfma_frac.get(name, False)
        if hit is False:
            rf = self.roofline(name) if self.roofline is not None else None
            hit = None if not rf or sum(rf) <= 0 else rf[0] / (rf[0] + rf[1])
            if len(self._mfma_frac) > 65536:
                self._mfma_frac.clear()
            self._mfma_frac[name] = hit
        return hit

    def _gpu_roofline(self, node: str) -> Dict[int, Tuple[float, float]]:
        """Per physical GPU: predicted MFMA-bound and HBM-bound seconds of its residents."""
        out: Dict[int, Tuple[float, float]] = {}
        for st in self.ledger.devices(node):
            m, h = out.get(st.device.gpu, (0.0, 0.0))
            for use in st.pods.values():
                f = self.mfma_fraction(use.name)
                if f is not None:
                    m += use.work * f
                    h += use.work * (1.0 - f)
            out[st.device.gpu] = (m, h)
        return out

    # ------------------------------------------------------------------ native node scoring
    native_score = True          # score a node's candidates in C++ (_core.score_node) when built
    NATIVE_MIN_CANDS = 2

    def _summary(self, st: DeviceState) -> DeviceSummary:
        d = st.__dict__
        ver = d.get("_ver", 0)
        hit = d.get("_slo")
        if hit is not None and hit[0] == ver:
            return hit[1]
        summ = self._device_summary(st)          # version-tagged like find_units' memo
        d["_slo"] = (ver, summ)
        return summ

    def _intern(self, table: Dict[str, int], key: str) -> int:
        i = table.get(key)
        if i is None:
            i = table[key] = len(table)
        return i

    def _node_pack(self, node: str, states: List[DeviceState]) -> Dict[str, Any]:
        """Flat arrays of a node's device states for `_core.score_node`, rebuilt only when the
        node's ledger entry (node_gen) or the prediction version changes."""
        import numpy as np
        key = (self.ledger.node_gen.get(node, 0), self._pred_version, self.args.w_complement)
        hit = self._packs.get(node)
        if hit is not None and hit[0] == key and len(hit[1]["uuid"]) == len(states):
            return hit[1]
        names, cols = self._name_ids, self._col_ids
        t_off, t_name, t_slo, t_pred, t_base, rows = [0], [], [], [], [], []
        k_off, k_name, k_col = [0], [], []
        for st in states:
            summ = self._summary(st)
            for nm, slo, pred, base, row in summ.terms:
                t_name.append(self._intern(names, nm))
                t_slo.append(slo)
                t_pred.append(pred)
                t_base.append(base)
                rows.append({self._intern(cols, c): v for c, v in row.items()})
            t_off.append(len(t_name))
            for nm, c in summ.cols:
                k_name.append(self._intern(names, nm))
                k_col.append(self._intern(cols, c))
            k_off.append(len(k_name))
        n_col = len(cols)
        t_rows = np.zeros((len(rows), n_col), np.float64)
        for t, r in enumerate(rows):
            for c, v in r.items():
                t_rows[t, c] = v
        n_gpu = max((st.device.gpu for st in states), default=-1) + 1
        tot, used = [0] * n_gpu, [0] * n_gpu
        for st in states:
            tot[st.device.gpu] += st.device.units
            used[st.device.gpu] += st.device.units - st.free_units
        loads = self.ledger.gpu_work(node)
        roof = self._gpu_roofline(node) if self.args.w_complement else {}
        pack = {"uuid": {st.device.uuid: i for i, st in enumerate(states)},
                "t_off": np.asarray(t_off, np.int64), "t_name": np.asarray(t_name, np.int32),
                "t_slo": np.asarray(t_slo, np.float64), "t_pred": np.asarray(t_pred, np.float64),
                "t_base": np.asarray(t_base, np.float64), "t_rows": t_rows,
                "k_off": np.asarray(k_off, np.int64), "k_name": np.asarray(k_name, np.int32),
                "k_col": np.asarray(k_col, np.int32),
                "dev_gpu": np.asarray([st.device.gpu for st in states], np.int32),
                "gpu_tot": np.asarray(tot, np.int32), "gpu_used": np.asarray(used, np.int32),
                "gpu_load": np.asarray([loads.get(g, 0.0) for g in range(n_gpu)], np.float64),
                "roof_m": np.asarray([roof.get(g, (0.0, 0.0))[0] for g in range(n_gpu)], np.float64),
                "roof_h": np.asarray([roof.get(g, (0.0, 0.0))[1] for g in range(n_gpu)], np.float64),
                "max_load": max(loads.values(), default=0.0), "cands": {},
                "no_tele": (np.zeros(len(states), np.int8), np.zeros(len(states)), np.zeros(len(states)))}
        pack["native"] = self._core().NodePack(
            pack["t_off"], pack["t_name"], pack["t_slo"], pack["t_pred"], pack["t_base"], pack["t_rows"],
            pack["k_off"], pack["k_name"], pack["k_col"], pack["dev_gpu"], pack["gpu_tot"], pack["gpu_used"],
            pack["gpu_load"], pack["roof_m"], pack["roof_h"])
        if len(self._packs) > 65536:
            self._packs.clear()
        self._packs[node] = (key, pack)
        return pack

    def _pack_ready(self, node: str) -> bool:
        key = (self.ledger.node_gen.get(node, 0), self._pred_version, self.args.w_complement)
        hit = self._packs.get(node)
        if hit is not None and hit[0] == key:
            return True
        if self._pack_seen.get(node) == key:
            return True
        if len(self._pack_seen) > 65536:
            self._pack_seen.clear()
        self._pack_seen[node] = key
        return False

    def _x_vector(self, intf: Dict[str, float]):
        """The incoming pod's interference row as a dense vector over interned column ids."""
        import numpy as np
        key = id(intf)
        hit = self._xvec_memo
        if hit is not None and hit[0] == key and hit[1] is intf and len(hit[2]) == len(self._col_ids):
            return hit[2]
        for c in intf:
            self._intern(self._col_ids, c)
        v = np.zeros(len(self._col_ids), np.float64)
        for c, x in intf.items():
            v[self._col_ids[c]] = x
        self._xvec_memo = (key, intf, v)
        return v

    def _score_cands_native(self, core: Any, node: str, cands: List[Tuple[DeviceState, int]], req: GpuRequest,
                            name: str, conf: Dict[str, float], intf: Dict[str, float], work: float,
                            states: List[DeviceState]) -> Optional[Choice]:
        import numpy as np
        a = self.args
        pack = self._node_pack(node, states)
        slo_on = bool(a.w_slo and req.slo > 0 and conf)
        x_col_name = self._workload_col(name, intf) if slo_on else None
        # candidate indices and the pod's prediction per candidate: memoised per candidate
        # list object (itself memoised per node version x request) and prediction table
        ck = (id(cands), id(conf) if slo_on else 0, req.units)
        hit = pack["cands"].get(ck)
        if hit is None or hit[0] is not cands:
            uidx = pack["uuid"]
            cand = np.asarray([uidx[st.device.uuid] for st, _ in cands], np.int32)
            xp = np.asarray([conf.get(self._col(req.units, st.device.units), -1.0) for st, _ in cands]
                            if slo_on else [-1.0] * len(cands), np.float64)
            if len(pack["cands"]) > 64:
                pack["cands"].clear()
            hit = pack["cands"][ck] = (cands, cand, xp)
        _, cand, xp = hit
        x_vec = self._x_vector(intf) if slo_on else self._empty_vec
        D = len(states)
        samples = self.telemetry.node(node) if a.w_telemetry else {}
        if not samples:
            tele_ok, gfx, vfree = pack["no_tele"]
        else:
            tele_ok = np.zeros(D, np.int8)
            gfx = np.zeros(D)
            vfree = np.zeros(D)
            for i, st in enumerate(states):
                smp = samples.get(st.device.uuid)
                if smp is not None:
                    tele_ok[i] = 1
                    gfx[i] = smp.gfx_activity
                    vfree[i] = smp.vram_total_mb - smp.vram_used_mb
        xf = self.mfma_fraction(name) if a.w_complement else None
        flags = (1 if slo_on else 0) | (2 if a.pack == "binpack" else 0) | (4 if a.w_balance else 0) | \
            (8 if xf is not None and work > 0 else 0)
        top = pack["max_load"] + work if a.w_balance else 0.0
        x_name = self._name_ids.get(name, -1)
        x_col = self._intern(self._col_ids, x_col_name) if x_col_name is not None else -1
        wt = self._weights_vec
        if wt is None:
            wt = self._weights_vec = np.asarray([a.w_slo, a.w_pack, a.w_balance, a.w_complement, a.w_telemetry],
                                                np.float64)
        best_i, best_sc = pack["native"].score(
            cand, xp, tele_ok, gfx, vfree, x_vec, x_name, x_col, float(req.slo), int(req.units), float(work),
            float(top), float(xf) if xf is not None else 0.0, float(req.hbm_gib * 1024), wt, flags)
        if best_i < 0:
            return None
        st, u0 = cands[best_i]
        return Choice(node, [(st.device.uuid, u0, req.units, req.hbm_gib, False)], best_sc, [st.device])

    def _score_cands(self, node: str, cands: List[Tuple[DeviceState, int]], req: GpuRequest, name: str,
                     conf: Dict[str, float], intf: Dict[str, float], work: float = 0.0) -> Optional[Choice]:
        a = self.args
        states = self.ledger.devices(node)
        if a.w_slo and a.pack != "random":
            model = self.corun_model()
            if model is not None:
                choice = self._score_cands_corun(node, cands, req, name, states, model)
                if choice is not None:
                    return choice
        if self.native_score and a.pack != "random" and len(cands) >= self.NATIVE_MIN_CANDS:
            core = self._core()
            # the node's pack is built on the SECOND score of one node version: a node that
            # changes after every placement (a single busy node) stays on the Python path,
            # where building the pack would cost more than it saves
            if core is not None and self._pack_ready(node):
                return self._score_cands_native(core, node, cands, req, name, conf, intf, work, states)
        slo_scores: List[Optional[float]] = [None] * len(cands)
        if a.w_slo and req.slo > 0 and conf:
            x_col = self._workload_col(name, intf)
            for i, (st, _) in enumerate(cands):
                summ = self._summary(st)
                slo_scores[i] = fast_device_score(summ, name, x_col, req.slo,
                                                  conf.get(self._col(req.units, st.device.units), -1.0), intf)
        if a.pack == "random":
            st, u0 = cands[self._rng.randrange(len(cands))]
            return Choice(node, [(st.device.uuid, u0, req.units, req.hbm_gib, False)], 50.0, [st.device])
        # per-GPU inputs once per call (a node has <= 8 GPUs; candidates share them)
        fill: Dict[int, Tuple[int, int]] = {}
        if a.w_pack:
            for s2 in states:
                t, u = fill.get(s2.device.gpu, (0, 0))
                fill[s2.device.gpu] = (t + s2.device.units, u + s2.device.units - s2.free_units)
        loads: Optional[Dict[int, float]] = None
        top = 0.0
        if a.w_balance:
            loads = self.ledger.gpu_work(node)
            top = max(loads.values(), default=0.0) + work
        roof: Optional[Dict[int, Tuple[float, float]]] = None
        xf = self.mfma_fraction(name) if a.w_complement else None
        if xf is not None and work > 0:
            roof = self._gpu_roofline(node)
        samples = self.telemetry.node(node) if a.w_telemetry else {}
        binpack = a.pack == "binpack"
        hbm_mb = req.hbm_gib * 1024
        best_i, best_sc = -1, 0.0
        for i, (st, u0) in enumerate(cands):
            num = den = 0.0
            if slo_scores[i] is not None:
                num += a.w_slo * slo_scores[i]
                den += a.w_slo
            g = st.device.gpu
            if a.w_pack:
                tot, used = fill[g]
                frac = (used + req.units) / max(tot, 1)
                num += a.w_pack * (100.0 * frac if binpack else 100.0 * (1.0 - frac))
                den += a.w_pack
            if loads is not None:
                # 100 on the least-loaded GPU after placement relative to the node's
                # busiest; equal loads (or no prediction) tie
                num += a.w_balance * (100.0 * (1.0 - (loads.get(g, 0.0) + work) / top) if top > 0 else 100.0)
                den += a.w_balance
            if roof is not None:
                # 100 when the GPU's MFMA-bound and HBM-bound predicted time are equal after
                # placement (the most room for the two phases to overlap), 0 when one-sided
                m, h = roof.get(g, (0.0, 0.0))
                m, h = m + work * xf, h + work * (1.0 - xf)
                num += a.w_complement * 100.0 * (min(m, h) / max(m, h) if max(m, h) > 0 else 1.0)
                den += a.w_complement
            if samples:
                smp = samples.get(st.device.uuid)
                if smp is not None:
                    hbm_ok = 1.0 if smp.vram_total_mb - smp.vram_used_mb >= hbm_mb else 0.0
                    num += a.w_telemetry * 100.0 * (1.0 - min(1.0, smp.gfx_activity)) * hbm_ok
                    den += a.w_telemetry
            sc = num / den if den > 0 else 0.0
            if best_i < 0 or sc > best_sc:
                best_i, best_sc = i, sc
        if best_i < 0:
            return None
        st, u0 = cands[best_i]
        return Choice(node, [(st.device.uuid, u0, req.units, req.hbm_gib, False)], best_sc, [st.device])

    # ------------------------------------------------------------------ co-run SLO objective
    def corun_model(self) -> Any:
        """The co-run model of the prediction provider (models.corun.CorunModel) when Score
        uses the co-run constraint, else None."""
        if self.args.slo_objective == "terms" or self.predictions is None:
            return None
        fn = getattr(self.predictions, "corun", None)
        return fn() if fn is not None else None

    @staticmethod
    def corun_group_key(st: DeviceState) -> Tuple[int, ...]:
        """Pods that co-run: every fractional pod on a physical GPU in SPX (they share its CUs
        and HBM), only the pods of one partition on a partitioned GPU."""
        d = st.device
        return (d.gpu,) if d.partitions <= 1 else (d.gpu, d.partition)

    def _corun_pack(self, node: str, states: List[DeviceState], model: Any) -> Optional[Dict[str, Any]]:
        """A node's co-run groups (residents per group as CSR arrays) and their current SLO
        misses / makespans, memoised per node version x model."""
        import numpy as np
        key = (self.ledger.node_gen.get(node, 0), id(model), len(states), self.args.corun_margin)
        hit = self._corun_packs.get(node)
        if hit is not None and hit[0] == key:
            return hit[1]
        core = self._core()
        if core is None or not hasattr(core, "corun_gpu_eval"):
            return None
        gids: Dict[Tuple[int, ...], int] = {}
        dev_group: Dict[str, int] = {}
        for st in states:
            dev_group[st.device.uuid] = gids.setdefault(self.corun_group_key(st), len(gids))
        per: List[List[Tuple[int, float, float]]] = [[] for _ in gids]
        seen = set()
        for st in states:
            g = dev_group[st.device.uuid]
            for k, use in st.pods.items():
                if (k, g) in seen:
                    continue
                seen.add((k, g))
                w = model.wid(use.name)
                if w >= 0:                  # a workload the model does not know is not modelled
                    per[g].append((w, use.iters, use.slo * (1.0 + self.args.corun_margin)))
        off = np.zeros(len(per) + 1, np.int64)
        off[1:] = np.cumsum([len(m) for m in per])
        flat = [x for m in per for x in m]
        r_wid = np.asarray([x[0] for x in flat], np.int32)
        r_iters = np.asarray([x[1] for x in flat], np.float64)
        r_slo = np.asarray([x[2] for x in flat], np.float64)
        if max((len(m) for m in per), default=0) >= 64:
            return None
        bad, mk = core.corun_groups_eval(off, r_wid, r_iters, r_slo, model.alone_ms, model.coupling())
        pack = {"dev_group": dev_group, "off": off, "r_wid": r_wid, "r_iters": r_iters, "r_slo": r_slo,
                "bad": bad, "mk": mk, "mk_max": float(mk.max(initial=0.0))}
        if len(self._corun_packs) > 65536:
            self._corun_packs.clear()
        self._corun_packs[node] = (key, pack)
        return pack

    @staticmethod
    def corun_band(new_bad: int, blend: float) -> float:
        """Score band of a placement causing `new_bad` predicted SLO misses (its own or its
        co-runners'): [50, 100) with none, [50/(k+1), 50/k) with k -- strictly ordered by k;
        `blend` (0..100, the packing / balance / telemetry terms) orders inside a band."""
        k = max(0, int(new_bad))
        lo = 50.0 / (k + 1)
        hi = 100.0 if k == 0 else 50.0 / k
        return lo + (hi - lo) * min(max(blend, 0.0), 100.0) / 100.0 * 0.999

    def _score_cands_corun(self, node: str, cands: List[Tuple[DeviceState, int]], req: GpuRequest, name: str,
                           states: List[DeviceState], model: Any) -> Optional[Choice]:
        """Co-run constraint Score of one node's candidate devices (see GPUArgs.slo_objective):
        each candidate's co-run group is simulated with and without the pod (native
        corun_gpu_eval); new predicted SLO misses pick the band, packing / makespan balance /
        telemetry order within it.  None = the pod's workload is unknown to the model."""
        import numpy as np
        xw = model.wid(name)
        if xw < 0:
            return None
        pack = self._corun_pack(node, states, model)
        if pack is None:
            return None
        a = self.args
        dg = pack["dev_group"]
        cg = np.asarray([dg[st.device.uuid] for st, _ in cands], np.int32)
        ug, inv = np.unique(cg, return_inverse=True)
        bb, ba, mb, ma, _ = self._core().corun_gpu_eval(
            pack["off"], pack["r_wid"], pack["r_iters"], pack["r_slo"], int(xw), float(req.iters),
            float(req.slo) * (1.0 + a.corun_margin),
            ug.astype(np.int32), model.alone_ms, model.coupling())
        top = max(pack["mk_max"], float(ma.max(initial=0.0)))
        fill: Dict[int, Tuple[int, int]] = {}
        if a.w_pack:
            for s2 in states:
                t, u = fill.get(s2.device.gpu, (0, 0))
                fill[s2.device.gpu] = (t + s2.device.units, u + s2.device.units - s2.free_units)
        samples = self.telemetry.node(node) if a.w_telemetry else {}
        binpack = a.pack == "binpack"
        hbm_mb = req.hbm_gib * 1024
        best_i, best_sc = -1, 0.0
        for i, (st, u0) in enumerate(cands):
            j = int(inv[i])
            num = den = 0.0
            g = st.device.gpu
            if a.w_pack:
                tot, used = fill[g]
                frac = (used + req.units) / max(tot, 1)
                num += a.w_pack * (100.0 * frac if binpack else 100.0 * (1.0 - frac))
                den += a.w_pack
            if a.w_balance:
                # the group's predicted makespan after placement against the node's longest
                num += a.w_balance * (100.0 * (1.0 - float(ma[j]) / top) if top > 0 else 100.0)
                den += a.w_balance
            if samples:
                smp = samples.get(st.device.uuid)
                if smp is not None:
                    hbm_ok = 1.0 if smp.vram_total_mb - smp.vram_used_mb >= hbm_mb else 0.0
                    num += a.w_telemetry * 100.0 * (1.0 - min(1.0, smp.gfx_activity)) * hbm_ok
                    den += a.w_telemetry
            sc = self.corun_band(int(ba[j]) - int(bb[j]), num / den if den > 0 else 100.0)
            if best_i < 0 or sc > best_sc:
                best_i, best_sc = i, sc
        st, u0 = cands[best_i]
        return Choice(node, [(st.device.uuid, u0, req.units, req.hbm_gib, False)], best_sc, [st.device])

    def _fits_without(self, req: GpuRequest, node: str, removed: Any) -> bool:
        """Would the request fit if the pods in `removed` released their devices?  Works on
        copies of the node's device states; the ledger itself is untouched."""
        sim: List[DeviceState] = []
        for st in self.ledger.devices(node):
            c = DeviceState(st.device, list(st.used_units), st.hbm_used, dict(st.pods))
            for key in removed:
                use = c.pods.pop(key, None)
                if use is not None:
                    u0, n = use.units
                    for u in range(u0, u0 + n):
                        c.used_units[u] = False
                    c.hbm_used = max(0.0, c.hbm_used - use.hbm_gib)
            sim.append(c)
        if req.whole:
            return self._whole_choice(req, node, sim) is not None
        return any(c.device.healthy and c.hbm_free + 1e-6 >= req.hbm_gib and c._find_units(req.units) is not None
                   for c in sim)

    def _larger_ok(self, req: GpuRequest) -> bool:
        """An SLO-sized pod may take a larger free partition when no node can be cut to its
        size soon: no partition controller, or the controller found no idle node to
        re-partition for it (every node busy / changing / backed off).  Otherwise it waits
        for the exact size, so whole GPUs are not spent on half-GPU pods."""
        if not req.part_min:
            return False
        pc = self.partitioner
        return pc is None or req.part_cus in pc.stuck

    def _whole_choice(self, req: GpuRequest, node: str, states: List[DeviceState]) -> Optional[Choice]:
        larger = req.isolated and self._larger_ok(req)
        free = [st for st in states if st.device.healthy and not st.pods
                and st.hbm_free + 1e-6 >= req.hbm_gib / max(req.whole, 1)
                and (not req.isolated or st.device.cus == req.part_cus
                     or (larger and st.device.cus >= req.part_cus))]
        if len(free) < req.whole:
            return None
        per = req.hbm_gib / max(req.whole, 1)
        parts = states[0].device.partitions
        if req.whole == 1:
            # single device: least-fragmenting = the GPU with the most used devices
            used_per_gpu: Dict[int, int] = {}
            for st in states:
                if st.pods:
                    used_per_gpu[st.device.gpu] = used_per_gpu.get(st.device.gpu, 0) + 1
            # (an SLO-sized floor: the smallest partition that holds it first)
            free.sort(key=lambda s: (s.device.cus if req.part_min else 0, -used_per_gpu.get(s.device.gpu, 0),
                                     s.device.gpu, s.device.partition))
            pick = free[:1]
            return Choice(node, [(s.device.uuid, 0, s.device.units, per, True) for s in pick], 100.0,
                          [s.device for s in pick])
        topo = self.topologies.get(node) or Topology.fully_connected(max(s.device.gpu for s in states) + 1)
        by_gpu: Dict[int, DeviceState] = {}
        if parts > 1:
            # Multi-device pod on a partitioned node: its devices go to DISTINCT physical
            # GPUs forming an xGMI clique (select_gpu_set on the physical GPUs), and never to
            # a GPU whose partitions already serve another multi-device pod -- all partitions
            # of a GPU share its 7 xGMI links, so two such pods' collectives would contend
            # (SURVEY.md §5.8 item 3).  Per GPU the lowest free partition is taken.
            taken = self._multi_device_gpus(states)
            for st in sorted(free, key=lambda s: (s.device.gpu, s.device.partition)):
                if st.device.gpu not in taken:
                    by_gpu.setdefault(st.device.gpu, st)
        else:
            by_gpu = {st.device.gpu: st for st in free}
        load: Dict[int, float] = {}
        if self.args.w_telemetry:
            for g, st in by_gpu.items():
                smp = self.telemetry.get(node, st.device.uuid)
                if smp is not None:
                    load[g] = max(smp.xgmi_tx_bps, smp.xgmi_rx_bps) / XGMI_GPU_BPS
        sel = select_gpu_set(topo, list(by_gpu), req.whole, load)
        if sel is None:
            return None
        gpus, quality = sel
        pick = [by_gpu[g] for g in gpus]
        return Choice(node, [(s.device.uuid, 0, s.device.units, per, True) for s in pick], 100.0 * quality,
                      [s.device for s in pick])

    def _multi_device_gpus(self, states: List[DeviceState]) -> set:
        """Physical GPUs hosting a device of a pod that holds more than one device."""
        out = set()
        for st in states:
            for key in st.pods:
                pl = self.ledger.placement(key)
                if pl is not None and len(pl[1]) > 1:
                    out.add(st.device.gpu)
                    break
        return out


def register(registry: Any) -> None:
    registry.register(C.PLUGIN_NAME, lambda args, handle: GPUPlugin(args, handle))
