"""Framework runtime: instantiates a profile's plugins and runs the extension points.

Mirrors upstream kube-scheduler's frameworkruntime (which the reference links via
`app.NewSchedulerCommand(app.WithPlugin(...))`, reference cmd/scheduler/main.go:20-22):
filter fan-out, Score over feasible nodes (parallel, bounded by `parallelism`),
ScoreExtensions.NormalizeScore, per-plugin weights, Reserve in order / Unreserve in
reverse order, Permit, PreBind, the first non-Skip Bind plugin, PostBind.
"""
from __future__ import annotations

from ..api import constants as C

import logging
import time
from concurrent.futures import ThreadPoolExecutor
from typing import Any, Callable, Dict, List, Optional, Tuple

from ..api.constants import MAX_NODE_SCORE, MIN_NODE_SCORE
from .config import Profile
from .interface import EXTENSION_POINTS, Code, CycleState, NodeScore, Status, as_status

log = logging.getLogger(__name__)
Obj = Dict[str, Any]
PluginFactory = Callable[[Dict[str, Any], Any], Any]


class Registry(dict):
    """plugin name -> factory(args, handle)"""

    def register(self, name: str, factory: PluginFactory) -> None:
        if name in self:
            raise ValueError(f"plugin {name} already registered")
        self[name] = factory

    def merge(self, other: Dict[str, PluginFactory]) -> "Registry":
        for k, v in other.items():
            self.register(k, v)
        return self


class Metrics:
    """Per-extension-point latency accounting (SURVEY §5.5 'scheduler spans')."""

    def __init__(self) -> None:
        self.ext_ns: Dict[str, int] = {}
        self.ext_calls: Dict[str, int] = {}

    def add(self, point: str, ns: int) -> None:
        self.ext_ns[point] = self.ext_ns.get(point, 0) + ns
        self.ext_calls[point] = self.ext_calls.get(point, 0) + 1

    def summary(self) -> Dict[str, Dict[str, float]]:
        return {k: {"calls": self.ext_calls[k], "mean_us": self.ext_ns[k] / 1e3 / max(self.ext_calls[k], 1)}
                for k in self.ext_ns}


class Framework:
    def __init__(self, profile: Profile, registry: Registry, handle: Any, parallelism: int = 16):
        self.profile = profile
        self.handle = handle
        self.parallelism = max(1, parallelism)
        self.metrics = Metrics()
        self._instances: Dict[str, Any] = {}
        self.points: Dict[str, List[Any]] = {}
        self.weights: Dict[str, int] = {}
        for point, cls in EXTENSION_POINTS.items():
            lst = []
            for ref in profile.enabled(point):
                if ref.name not in registry:
                    raise KeyError(f"plugin {ref.name!r} (at {point}) is not registered")
                inst = self._instances.get(ref.name)
                if inst is None:
                    inst = registry[ref.name](profile.args(ref.name), handle)
                    self._instances[ref.name] = inst
                if not isinstance(inst, cls):
                    raise TypeError(f"plugin {ref.name} does not implement {point}")
                lst.append(inst)
                if point == "score":
                    self.weights[ref.name] = ref.weight
            self.points[point] = lst
        self._pool: Optional[ThreadPoolExecutor] = None
        self._filter_forms: Optional[Tuple[List[Any], List[Any]]] = None   # (plugins, batch forms)
        self.score_in_parallel = any(getattr(p, "SCORE_DOES_IO", False) for p in self.points["score"])
        # plan hints: a score plugin that may already have decided a pod's node (the GPU plugin's
        # burst plan, `planned_node`) short-cuts the cycle -- Filter on that node only, no Score --
        # but only when its weight makes one point of its score outweigh every other score
        # plugin's whole range, i.e. when Score could not pick another feasible node anyway
        # (the deployed profile: GPU 10100 vs the in-tree plugins' 1-2 each x 100)
        self._hinters: List[Any] = []
        for p in self.points["score"]:
            if not hasattr(p, "planned_node"):
                continue
            others = sum(self.weights.get(q.name(), 1) for q in self.points["score"] if q is not p)
            if self.weights.get(p.name(), 1) > others * C.MAX_NODE_SCORE:
                self._hinters.append(p)

    @property
    def scheduler_name(self) -> str:
        return self.profile.scheduler_name

    def plugin(self, name: str) -> Any:
        return self._instances.get(name)

    def pool(self) -> ThreadPoolExecutor:
        if self._pool is None:
            self._pool = ThreadPoolExecutor(self.parallelism, thread_name_prefix="sched-par")
        return self._pool

    def _timed(self, point: str, fn: Callable[[], Any]) -> Any:
        t0 = time.perf_counter_ns()
        try:
            return fn()
        finally:
            self.metrics.add(point, time.perf_counter_ns() - t0)

    def plan_hint(self, state: CycleState, pod: Obj) -> Optional[str]:
        """The node a dominant score plugin has already planned for `pod` (None: none)."""
        for p in self._hinters:
            n = p.planned_node(state, pod)
            if n:
                return n
        return None

    # ---------------------------------------------------------------- queue sort
    def queue_sort_less(self) -> Optional[Callable[[Any, Any], bool]]:
        qs = self.points["queueSort"]
        return qs[0].less if qs else None

    def queue_sort_key(self) -> Optional[Callable[[Any], Any]]:
        """The queueSort plugin's `sort_key(pod_info)` when it offers one (a key whose `<`
        is exactly its `less`); None = the queue compares with `less`."""
        qs = self.points["queueSort"]
        return getattr(qs[0], "sort_key", None) if qs else None

    # ---------------------------------------------------------------- filter
    # extension points are timed as a whole (kube-scheduler's framework_extension_point_duration);
    # per-plugin clocks cost two clock reads and a metrics update per plugin per pod
    def run_pre_filter(self, state: CycleState, pod: Obj) -> Status:
        t0 = time.perf_counter_ns()
        try:
            for p in self.points["preFilter"]:
                r = p.pre_filter(state, pod)
                if r is None:
                    continue
                s = as_status(r)
                if s.code == Code.SKIP:
                    state.skip_filter_plugins.add(p.name())
                    continue
                if not s.ok:
                    s.plugin = s.plugin or p.name()
                    return s
            return Status.success()
        finally:
            self.metrics.add("preFilter", time.perf_counter_ns() - t0)

    def run_filter(self, state: CycleState, pod: Obj, node_info: Any) -> Status:
        for p in self.points["filter"]:
            if p.name() in state.skip_filter_plugins:
                continue
            s = as_status(p.filter(state, pod, node_info))
            if not s.ok:
                s.plugin = s.plugin or p.name()
                return s
        return Status.success()

    def find_feasible(self, state: CycleState, pod: Obj, nodes: List[Any],
                      limit: int = 0) -> Tuple[List[Any], Dict[str, Status]]:
        """Filter nodes in order; with limit > 0 stop once that many are feasible (the
        scheduler passes a rotated node list, kube-scheduler's nextStartNodeIndex).

        Nodes go through the filter plugins a chunk at a time: a plugin with a batch form
        (`filter_nodes(state, pod, node_infos) -> [Status|None]`) is called once per chunk
        with the nodes still alive, so pod-side work (requests, tolerations, selectors) is
        hoisted out of the per-node loop.  Each node's status is still that of the FIRST
        failing plugin, and with a limit the feasible list is cut exactly where the
        node-at-a-time loop would have stopped -- identical results."""
        t0 = time.perf_counter_ns()
        feasible: List[Any] = []
        failed: Dict[str, Status] = {}
        if state.skip_filter_plugins:
            plugins = [p for p in self.points["filter"] if p.name() not in state.skip_filter_plugins]
            batch = [getattr(p, "filter_nodes", None) for p in plugins]
        else:
            if self._filter_forms is None:
                ps = list(self.points["filter"])
                self._filter_forms = (ps, [getattr(p, "filter_nodes", None) for p in ps])
            plugins, batch = self._filter_forms
        chunk = max(16, min(256, limit * 2)) if limit else 256
        processed = 0
        i, n, done = 0, len(nodes), False
        while i < n and not done:
            part = nodes[i:i + chunk]
            i += chunk
            res: List[Optional[Status]] = [None] * len(part)
            alive = list(range(len(part)))
            for p, bf in zip(plugins, batch):
                if not alive:
                    break
                if bf is not None:
                    sts = bf(state, pod, [part[j] for j in alive])
                else:
                    sts = [p.filter(state, pod, part[j]) for j in alive]
                nxt = []
                for j, s in zip(alive, sts):
                    if s is None or s.ok:
                        nxt.append(j)
                    else:
                        s.plugin = s.plugin or p.name()
                        res[j] = s
                alive = nxt
            for j, ni in enumerate(part):
                processed += 1
                s = res[j]
                if s is None:
                    feasible.append(ni)
                    if limit and len(feasible) >= limit:
                        done = True
                        break
                else:
                    failed[ni.name] = s
        self.metrics.add("filter", time.perf_counter_ns() - t0)
        state.write("framework/nodes-processed", processed)
        return feasible, failed

    def run_post_filter(self, state: CycleState, pod: Obj, failed: Dict[str, Status]) -> Tuple[Optional[str], Status]:
        """First plugin that nominates a node (or declares the pod unresolvable) wins."""
        last = Status.unschedulable("no postFilter plugin made the pod schedulable")
        for p in self.points["postFilter"]:
            nominated, s = p.post_filter(state, pod, failed)
            if nominated or s.ok or s.code == Code.UNSCHEDULABLE_AND_UNRESOLVABLE:
                return nominated, s
            last = s
        return None, last

    # ---------------------------------------------------------------- score
    def run_pre_score(self, state: CycleState, pod: Obj, nodes: List[Any]) -> Status:
        for p in self.points["preScore"]:
            s = as_status(self._timed("preScore", lambda p=p: p.pre_score(state, pod, nodes)))
            if s.code == Code.SKIP:
                state.skip_score_plugins.add(p.name())
                continue
            if not s.ok:
                s.plugin = s.plugin or p.name()
                return s
        return Status.success()

    def run_score(self, state: CycleState, pod: Obj, nodes: List[Any]) -> Tuple[List[NodeScore], Status]:
        """Returns the weighted total per node (sum over plugins of normalized*weight)."""
        t0 = time.perf_counter_ns()
        plugins = [p for p in self.points["score"] if p.name() not in state.skip_score_plugins]
        names = [n.name for n in nodes]
        per_plugin: Dict[str, List[NodeScore]] = {}
        for p in plugins:
            batch = getattr(p, "score_nodes", None)
            if batch is not None and not getattr(p, "SCORE_DOES_IO", False):
                # batch form: one call for every feasible node
                vals, bst = batch(state, pod, names)
                if bst is not None and not bst.ok:
                    bst.plugin = bst.plugin or p.name()
                    return [], bst
                per_plugin[p.name()] = [NodeScore(nn, int(v)) for nn, v in zip(names, vals)]
                continue

            def one(nn: str, p=p) -> Tuple[int, Status]:
                sc, st = p.score(state, pod, nn)
                return int(sc), as_status(st)
            if self.score_in_parallel and len(names) > 1 and getattr(p, "SCORE_DOES_IO", False):
                results = list(self.pool().map(one, names))
            else:
                results = [one(nn) for nn in names]
            lst = []
            for nn, (sc, st) in zip(names, results):
                if not st.ok:
                    st.plugin = st.plugin or p.name()
                    return [], st
                lst.append(NodeScore(nn, sc))
            per_plugin[p.name()] = lst
        for p in plugins:
            ext = p.score_extensions()
            if ext is not None:
                s = as_status(ext.normalize_score(state, pod, per_plugin[p.name()]))
                if not s.ok:
                    s.plugin = s.plugin or p.name()
                    return [], s
        totals = [NodeScore(nn, 0) for nn in names]
        for p in plugins:
            w = self.weights.get(p.name(), 1)
            for i, ns in enumerate(per_plugin[p.name()]):
                if not (MIN_NODE_SCORE <= ns.score <= MAX_NODE_SCORE):
                    return [], Status.error(f"plugin {p.name()} returned invalid score {ns.score} for {ns.name}",
                                            p.name())
                totals[i].score += ns.score * w
        self.metrics.add("score", time.perf_counter_ns() - t0)
        state.write("framework/per-plugin-scores", per_plugin)
        return totals, Status.success()

    # ---------------------------------------------------------------- reserve .. postBind
    def run_reserve(self, state: CycleState, pod: Obj, node: str) -> Status:
        t0 = time.perf_counter_ns()
        try:
            for p in self.points["reserve"]:
                r = p.reserve(state, pod, node)
                if r is None:
                    continue
                s = as_status(r)
                if not s.ok:
                    s.plugin = s.plugin or p.name()
                    return s
            return Status.success()
        finally:
            self.metrics.add("reserve", time.perf_counter_ns() - t0)

    def run_unreserve(self, state: CycleState, pod: Obj, node: str) -> None:
        for p in reversed(self.points["reserve"]):
            try:
                p.unreserve(state, pod, node)
            except Exception as e:  # never let unreserve failures mask the original error
                log.warning("unreserve %s failed: %s", p.name(), e)

    def run_permit(self, state: CycleState, pod: Obj, node: str) -> Tuple[Status, float]:
        """Upstream semantics: any rejection wins; otherwise, if some plugins asked to wait,
        the pod becomes a waiting pod until each of them allows it (handle.allow) or the
        longest of their timeouts passes; their names are left in the cycle state."""
        wait = 0.0
        waiting: List[str] = []
        for p in self.points["permit"]:
            s, timeout = p.permit(state, pod, node)
            s = as_status(s)
            if s.code == Code.WAIT:
                wait = max(wait, timeout)
                waiting.append(p.name())
                continue
            if not s.ok:
                s.plugin = s.plugin or p.name()
                return s, 0.0
        state.write("framework/permit-waiting", waiting)
        return (Status(Code.WAIT) if waiting else Status.success()), wait

    def run_pre_bind(self, state: CycleState, pod: Obj, node: str) -> Status:
        t0 = time.perf_counter_ns()
        try:
            for p in self.points["preBind"]:
                r = p.pre_bind(state, pod, node)
                if r is None:
                    continue
                s = as_status(r)
                if not s.ok:
                    s.plugin = s.plugin or p.name()
                    return s
            return Status.success()
        finally:
            self.metrics.add("preBind", time.perf_counter_ns() - t0)

    def run_bind(self, state: CycleState, pod: Obj, node: str) -> Status:
        for p in self.points["bind"]:
            s = as_status(self._timed("bind", lambda p=p: p.bind(state, pod, node)))
            if s.code == Code.SKIP:
                continue
            if not s.ok:
                s.plugin = s.plugin or p.name()
            return s
        return Status.error("no bind plugin bound the pod")

    def run_post_bind(self, state: CycleState, pod: Obj, node: str) -> None:
        for p in self.points["postBind"]:
            try:
                self._timed("postBind", lambda p=p: p.post_bind(state, pod, node))
            except Exception as e:
                log.warning("postBind %s failed: %s", p.name(), e)

    def close(self) -> None:
        if self._pool is not None:
            self._pool.shutdown(wait=False)
        for inst in self._instances.values():
            c = getattr(inst, "close", None)
            if callable(c):
                c()
