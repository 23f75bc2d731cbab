"""The scheduler: informers -> queue -> scheduling cycle -> binding cycle.

Upstream kube-scheduler's scheduleOne, which the reference inherits unchanged
("kube-scheduler scheduleOne → Filter → RunScorePlugins → NormalizeScore
→ selectHost → Reserve/Permit → PreBind → Bind → PostBind"), re-implemented for the
standalone `gpu-scheduler`:

* pods with `spec.schedulerName` in our profiles are queued (reference pods opt in via
  `schedulerName: gpu-scheduler`, deploy/busybox/busybox.yaml:17);
* the scheduling cycle takes a cache snapshot, filters, scores, picks the host with the
  reservoir-sampled max (upstream selectHost), assumes the pod and runs Reserve/Permit;
* the binding cycle (PreBind, Bind, PostBind) runs async on a worker pool or inline
  (`bind_async=False`, used by the bench and tests); failures Unreserve + forget + requeue.
"""
from __future__ import annotations

import logging
import random
import threading
import time
from concurrent.futures import ThreadPoolExecutor
from dataclasses import dataclass, field
from typing import Any, Callable, Dict, List, Optional

from ..api import constants as C
from ..api import objects as O
from ..kube.client import KubeClient
from ..kube.informer import SharedInformerFactory
from .cache import SchedulerCache, Snapshot
from .changes import ChangeLog
from .fastpath import NodeResultCache
from .config import SchedulerConfig
from .interface import Code, CycleState, Status
from .queue import QueuedPodInfo, SchedulingQueue
from .runtime import Framework, Registry

log = logging.getLogger(__name__)
Obj = Dict[str, Any]


@dataclass
class ScheduleResult:
    pod_key: str
    node: str = ""
    status: Status = field(default_factory=Status.success)
    scores: Dict[str, int] = field(default_factory=dict)
    evaluated: int = 0
    feasible: int = 0
    latency_s: float = 0.0
    bound: bool = False
    nominated: str = ""         # node nominated by a PostFilter (preemption)


class Handle:
    """What plugins can reach (framework.Handle in upstream)."""

    def __init__(self, scheduler: "Scheduler"):
        self._s = scheduler

    @property
    def client(self) -> KubeClient:
        return self._s.client

    @property
    def informer_factory(self) -> SharedInformerFactory:
        return self._s.informers

    @property
    def cache(self) -> SchedulerCache:
        return self._s.cache

    def snapshot(self) -> Snapshot:
        return self._s.current_snapshot()

    def event(self, obj: Obj, reason: str, message: str, type_: str = "Normal") -> None:
        if self._s.record_events:
            self.client.create_event(obj, reason, message, type_)

    @property
    def extras(self) -> Dict[str, Any]:
        return self._s.extras

    def pending_pods(self) -> List[Obj]:
        """Pods in the active queue -- what a plugin may plan jointly with the current one."""
        return self._s.queue.active_pods()

    def framework_for(self, pod: Obj) -> Optional["Framework"]:
        return self._s.frameworks.get(O.scheduler_name(pod))

    # waiting pods (Permit -> WAIT), upstream framework.Handle's WaitingPod API
    def get_waiting_pod(self, pod_key: str) -> Optional["WaitingPod"]:
        return self._s.waiting_pods().get(pod_key)

    def iterate_over_waiting_pods(self) -> List["WaitingPod"]:
        return list(self._s.waiting_pods().values())

    def allow(self, pod_key: str, plugin: str) -> bool:
        return self._s.allow_waiting(pod_key, plugin)

    def reject(self, pod_key: str, plugin: str, message: str) -> bool:
        return self._s.reject_waiting(pod_key, plugin, message)


@dataclass
class WaitingPod:
    """A reserved pod held at Permit until every waiting plugin allows it (then its binding
    cycle runs) or one rejects it / the deadline passes (then it is unreserved and
    requeued).  `ctx` = (framework, state, queued pod info, host, result, t0)."""
    key: str
    pod: Obj
    node: str
    pending: set
    deadline: float
    ctx: tuple = ()


class Scheduler:
    def __init__(self, client: KubeClient, config: SchedulerConfig, registry: Registry,
                 bind_async: bool = True, bind_workers: int = 16, record_events: bool = True,
                 seed: Optional[int] = None, extras: Optional[Dict[str, Any]] = None,
                 informers: Optional[SharedInformerFactory] = None):
        self.client = client
        self.config = config
        self.cache = SchedulerCache()
        self.informers = informers or SharedInformerFactory(client)
        self.extras: Dict[str, Any] = dict(extras or {})
        self.telemetry_poller: Any = None      # telemetry.poller.TelemetryPoller (CLI wiring)
        self.record_events = record_events
        self.handle = Handle(self)
        self.frameworks: Dict[str, Framework] = {}
        self._snapshot: Optional[Snapshot] = None
        self._next_start = 0
        for prof in config.profiles:
            self.frameworks[prof.scheduler_name] = Framework(prof, registry, self.handle, config.parallelism)
        first = next(iter(self.frameworks.values()))
        self.queue = SchedulingQueue(self._queue_less(first), config.pod_initial_backoff_s,
                                     config.pod_max_backoff_s, sort_key=first.queue_sort_key())
        self.bind_async = bind_async
        self._bind_pool = ThreadPoolExecutor(bind_workers, thread_name_prefix="bind") if bind_async else None
        self._rng = random.Random(seed)
        self._stop = threading.Event()
        self._thread: Optional[threading.Thread] = None
        self._results_lock = threading.Lock()
        self.results: List[ScheduleResult] = []
        self.keep_results = True
        self.on_result: Optional[Callable[[ScheduleResult], None]] = None
        self.stats = {"scheduled": 0, "unschedulable": 0, "errors": 0, "bind_failures": 0}
        self._pending_binds = 0
        self._bind_cv = threading.Condition()
        self._started = False
        self._waiting: Dict[str, WaitingPod] = {}
        self._waiting_lock = threading.RLock()
        # cross-cycle node-result cache (framework.fastpath): every source of node-local
        # scheduling state reports changed nodes to one change log
        self.changes = ChangeLog()
        self.cache.changes.attach(self.changes)
        # HTTP extenders this scheduler calls (config `extenders:`, framework.extender_client)
        from .extender_client import HTTPExtender
        self.extenders = [HTTPExtender(c) for c in getattr(config, "extenders", None) or []]
        self.fast_path = not self.extenders     # the node-result cache cannot see extender verdicts
        self.fast_min_nodes = 16      # below this the per-cycle signature work costs more than it saves
        self.plan_hints = True        # planned pods skip Score (Framework.plan_hint)
        self.plan_hint_hits = 0
        self._fast: Dict[str, NodeResultCache] = {}
        for name, fw in self.frameworks.items():
            for inst in fw._instances.values():
                for attr in ("ledger", "telemetry"):
                    fan = getattr(getattr(inst, attr, None), "changes", None)
                    if fan is not None and hasattr(fan, "attach"):
                        fan.attach(self.changes)
            nc = NodeResultCache(fw, self.changes)
            nc.fw_rng = self._rng
            self._fast[name] = nc

    @staticmethod
    def _queue_less(fw: Framework):
        less = fw.queue_sort_less()
        return less

    # ---------------------------------------------------------------- event wiring
    def _responsible(self, pod: Obj) -> bool:
        return O.scheduler_name(pod) in self.frameworks

    def _on_pod_add(self, pod: Obj) -> None:
        if O.node_name_of(pod):
            self.cache.add_pod(pod)
        elif self._responsible(pod) and not O.is_terminal(pod):
            self.queue.add(pod)

    def _on_pod_update(self, old: Obj, new: Obj) -> None:
        if O.node_name_of(new):
            if O.is_terminal(new):
                self.cache.remove_pod(new)
                self.queue.move_all_to_active_or_backoff("PodTerminated")
            else:
                self.cache.update_pod(new)
        elif self._responsible(new) and not O.is_terminal(new):
            if O.resource_version(old) != O.resource_version(new):
                self.queue.update(new)

    def _on_pod_delete(self, pod: Obj) -> None:
        if O.node_name_of(pod):
            self.cache.remove_pod(pod)
            self.queue.move_all_to_active_or_backoff("AssignedPodDelete")
        else:
            self.queue.delete(pod)

    def _on_node_add(self, node: Obj) -> None:
        self.cache.add_node(node)
        self.queue.move_all_to_active_or_backoff("NodeAdd")

    def _on_node_update(self, old: Obj, new: Obj) -> None:
        self.cache.update_node(new)
        self.queue.move_all_to_active_or_backoff("NodeUpdate")

    def _on_node_delete(self, node: Obj) -> None:
        self.cache.remove_node(node)

    def start_informers(self) -> None:
        if self._started:
            return
        self._started = True
        pods, nodes = self.informers.pods(), self.informers.nodes()
        self.informers.config_maps()
        nodes.add_event_handler(self._on_node_add, self._on_node_update, self._on_node_delete)
        pods.add_event_handler(self._on_pod_add, self._on_pod_update, self._on_pod_delete)
        self.informers.start()
        self.informers.wait_for_cache_sync()

    # ---------------------------------------------------------------- cycle
    def current_snapshot(self) -> Snapshot:
        if self._snapshot is None:
            self._snapshot = self.cache.snapshot()
        return self._snapshot

    # kube-scheduler's adaptive sampling (pkg/scheduler/schedule_one.go numFeasibleNodesToFind)
    MIN_FEASIBLE_NODES = 100
    MIN_FEASIBLE_PERCENT = 5

    def num_feasible_nodes_to_find(self, n: int) -> int:
        if n < self.MIN_FEASIBLE_NODES:
            return n
        pct = self.config.percentage_of_nodes_to_score
        if pct <= 0:
            pct = max(self.MIN_FEASIBLE_PERCENT, 50 - n // 125)
        if pct >= 100:
            return n
        return max(self.MIN_FEASIBLE_NODES, n * pct // 100)

    def _select_host(self, scores: List[Any]) -> str:
        """Uniformly random among the nodes tied at the maximum (upstream selectHost's
        reservoir sample has the same distribution); one draw, as the cycle cache's."""
        if not scores:
            return ""
        best = max(ns.score for ns in scores)
        ties = [ns.name for ns in scores if ns.score == best]
        return ties[0] if len(ties) == 1 else ties[self._rng.randrange(len(ties))]

    def schedule_one(self, pi: QueuedPodInfo) -> ScheduleResult:
        t0 = time.perf_counter()
        pod = pi.pod
        fw = self.frameworks.get(O.scheduler_name(pod))
        res = ScheduleResult(O.key(pod))
        if fw is None:
            res.status = Status.error("no profile for scheduler " + O.scheduler_name(pod))
            return res
        fast = self._fast.get(O.scheduler_name(pod)) \
            if self.fast_path and len(self.cache._nodes) >= self.fast_min_nodes else None
        cursor = fast.cursor() if fast is not None else None     # before the snapshot
        self._snapshot = self.cache.snapshot()
        state = CycleState()
        nodes = self._snapshot.list()
        st = fw.run_pre_filter(state, pod)
        if not st.ok:
            return self._fail(pi, fw, state, res, st, t0)
        # a planned pod (framework.plan_hint: the GPU plugin's burst plan, whose weight decides
        # Score): Filter on the planned node only and no Score; a stale plan (node gone or no
        # longer feasible) falls through to the full cycle
        hint = fw.plan_hint(state, pod) if (self.plan_hints and not self.extenders) else None
        if hint is not None:
            ni = self._snapshot.get(hint)
            if ni is not None:
                feasible, _ = fw.find_feasible(state, pod, [ni], 0)
                if feasible:
                    st = fw.run_pre_score(state, pod, feasible)
                    if not st.ok:
                        return self._fail(pi, fw, state, res, st, t0)
                    res.evaluated, res.feasible = 1, 1
                    self.plan_hint_hits += 1
                    return self._assume_and_bind(fw, state, pi, pod, hint, res, t0)
        limit = self.num_feasible_nodes_to_find(len(nodes))
        sampled = limit < len(nodes)
        got = fast.schedule(state, pod, self._snapshot, self._next_start % len(nodes) if sampled else 0,
                            limit if sampled else 0, cursor) if fast is not None and nodes else None
        if got is not None:
            host, processed, n_feasible, scores = got
            self._next_start = (self._next_start + processed) % len(nodes)
            res.evaluated, res.feasible, res.scores = processed, n_feasible, scores
            return self._assume_and_bind(fw, state, pi, pod, host, res, t0)
        if limit < len(nodes):
            start = self._next_start % len(nodes)
            nodes = nodes[start:] + nodes[:start]
        feasible, failed = fw.find_feasible(state, pod, nodes, limit if limit < len(nodes) else 0)
        processed = state.read("framework/nodes-processed") or len(nodes)
        if nodes:
            self._next_start = (self._next_start + processed) % len(nodes)
        res.evaluated = processed
        if feasible and self.extenders:
            feasible, st = self._extender_filter(pod, feasible, failed)
            if st is not None:
                return self._fail(pi, fw, state, res, st, t0)
        res.feasible = len(feasible)
        if not feasible:
            nominated, pst = fw.run_post_filter(state, pod, failed)
            reasons = sorted({m for s in failed.values() for m in s.reasons})
            msg = f"0/{len(nodes)} nodes are available: " + ", ".join(reasons) if nodes else "no nodes available"
            if pst.message():
                msg += f"; postFilter: {pst.message()}"
            res.nominated = nominated or ""
            return self._fail(pi, fw, state, res, Status.unschedulable(msg), t0)
        if len(feasible) == 1 and not fw.points["score"]:
            host = feasible[0].name
        else:
            st = fw.run_pre_score(state, pod, feasible)
            if not st.ok:
                return self._fail(pi, fw, state, res, st, t0)
            scores, st = fw.run_score(state, pod, feasible)
            if not st.ok:
                return self._fail(pi, fw, state, res, st, t0)
            if self.extenders:
                self._extender_prioritize(pod, feasible, scores)
            res.scores = {s.name: s.score for s in scores}
            host = self._select_host(scores)
        return self._assume_and_bind(fw, state, pi, pod, host, res, t0)

    # ---------------------------------------------------------------- extenders
    def _extender_filter(self, pod: Obj, feasible: List[Any], failed: Dict[str, Status]):
        """Each interested extender narrows the feasible set in turn; (nodes, error status)."""
        from .extender_client import ExtenderError
        for ext in self.extenders:
            if not feasible:
                break
            if not ext.is_interested(pod):
                continue
            try:
                feasible, bad, unresolvable = ext.filter(pod, feasible)
            except ExtenderError as e:
                if ext.is_ignorable:
                    log.warning("skipping ignorable extender: %s", e)
                    continue
                return feasible, Status.error(str(e))
            for name, why in bad.items():
                failed[name] = Status.unschedulable(why or "rejected by extender", ext.name)
            for name, why in unresolvable.items():
                failed[name] = Status.unschedulable(why or "rejected by extender", ext.name, True)
        return feasible, None

    def _extender_prioritize(self, pod: Obj, feasible: List[Any], scores: List[Any]) -> None:
        from .extender_client import ExtenderError, MAX_EXTENDER_PRIORITY
        extra: Dict[str, int] = {}
        for ext in self.extenders:
            if not ext.cfg.prioritize_verb or not ext.is_interested(pod):
                continue
            try:
                got = ext.prioritize(pod, feasible)
            except ExtenderError as e:     # upstream ignores prioritize errors
                log.warning("extender prioritize failed: %s", e)
                continue
            for host, v in got.items():
                extra[host] = extra.get(host, 0) + v * ext.cfg.weight * (C.MAX_NODE_SCORE // MAX_EXTENDER_PRIORITY)
        for ns in scores:
            ns.score += extra.get(ns.name, 0)

    def _assume_and_bind(self, fw: Framework, state: CycleState, pi: QueuedPodInfo, pod: Obj, host: str,
                         res: ScheduleResult, t0: float) -> ScheduleResult:
        # assume + reserve
        self.cache.assume_pod(pod, host)
        st = fw.run_reserve(state, pod, host)
        if not st.ok:
            fw.run_unreserve(state, pod, host)
            self.cache.forget_pod(pod)
            return self._fail(pi, fw, state, res, st, t0)
        st, wait = fw.run_permit(state, pod, host)
        if not st.ok and st.code != Code.WAIT:
            fw.run_unreserve(state, pod, host)
            self.cache.forget_pod(pod)
            return self._fail(pi, fw, state, res, st, t0)
        res.node = host
        self._snapshot = None
        if st.code == Code.WAIT:
            pending = set(state.read("framework/permit-waiting") or [])
            key = O.key(pod)
            wp = WaitingPod(key, pod, host, pending, time.monotonic() + max(0.0, wait),
                            (fw, state, pi, host, res, t0))
            with self._waiting_lock:
                self._waiting[key] = wp
            res.status = Status(Code.WAIT, ["waiting on permit: " + ",".join(sorted(pending))])
            return res
        self._start_binding(fw, state, pi, host, res, t0)
        return res

    # ---------------------------------------------------------------- waiting pods
    def waiting_pods(self) -> Dict[str, WaitingPod]:
        with self._waiting_lock:
            return dict(self._waiting)

    def allow_waiting(self, pod_key: str, plugin: str) -> bool:
        with self._waiting_lock:
            wp = self._waiting.get(pod_key)
            if wp is None:
                return False
            wp.pending.discard(plugin)
            if wp.pending:
                return True
            del self._waiting[pod_key]
        fw, state, pi, host, res, t0 = wp.ctx
        res.status = Status.success()
        self._start_binding(fw, state, pi, host, res, t0)
        return True

    def reject_waiting(self, pod_key: str, plugin: str, message: str) -> bool:
        with self._waiting_lock:
            wp = self._waiting.pop(pod_key, None)
        if wp is None:
            return False
        fw, state, pi, host, res, t0 = wp.ctx
        fw.run_unreserve(state, wp.pod, host)
        self.cache.forget_pod(wp.pod)
        res.node = ""
        st = Status.unschedulable(f"rejected at permit by {plugin}: {message}", plugin)
        self._fail(pi, fw, state, res, st, t0)
        return True

    def expire_waiting(self) -> int:
        """Reject waiting pods whose permit deadline passed (called by the loops)."""
        now = time.monotonic()
        with self._waiting_lock:
            late = [wp for wp in self._waiting.values() if wp.deadline <= now]
        for wp in late:
            self.reject_waiting(wp.key, ",".join(sorted(wp.pending)) or "permit", "timed out waiting on permit")
        return len(late)

    def _start_binding(self, fw: Framework, state: CycleState, pi: QueuedPodInfo, host: str,
                       res: ScheduleResult, t0: float) -> None:
        if self._bind_pool is not None:
            with self._bind_cv:
                self._pending_binds += 1
            self._bind_pool.submit(self._binding_cycle, fw, state, pi, host, res, t0)
        else:
            self._binding_cycle(fw, state, pi, host, res, t0)

    def _binding_cycle(self, fw: Framework, state: CycleState, pi: QueuedPodInfo, host: str,
                       res: ScheduleResult, t0: float) -> None:
        pod = pi.pod
        try:
            st = fw.run_pre_bind(state, pod, host)
            if st.ok:
                binder = next((e for e in self.extenders if e.is_binder and e.is_interested(pod)), None)
                if binder is not None:
                    from .extender_client import ExtenderError
                    try:
                        binder.bind(pod, host)
                    except ExtenderError as e:
                        st = Status.error(str(e))
                else:
                    st = fw.run_bind(state, pod, host)
            if not st.ok:
                fw.run_unreserve(state, pod, host)
                self.cache.forget_pod(pod)
                self.stats["bind_failures"] += 1
                res.status = st
                self.handle.event(pod, "FailedScheduling", f"Binding rejected: {st.message()}", "Warning")
                self.queue.add_unschedulable(pi)
            else:
                self.cache.finish_binding(pod)
                self.queue.done(pod)
                res.bound = True
                self.stats["scheduled"] += 1
                self.handle.event(pod, "Scheduled", f"Successfully assigned {O.key(pod)} to {host}")
                fw.run_post_bind(state, pod, host)
        except Exception as e:  # keep the loop alive
            log.exception("binding cycle failed")
            fw.run_unreserve(state, pod, host)
            self.cache.forget_pod(pod)
            res.status = Status.error(str(e))
            self.stats["errors"] += 1
            self.queue.add_unschedulable(pi)
        finally:
            res.latency_s = time.perf_counter() - t0
            self._record(res)
            if self._bind_pool is not None:
                with self._bind_cv:
                    self._pending_binds -= 1
                    self._bind_cv.notify_all()

    def _fail(self, pi: QueuedPodInfo, fw: Framework, state: CycleState, res: ScheduleResult,
              st: Status, t0: float) -> ScheduleResult:
        res.status = st
        res.latency_s = time.perf_counter() - t0
        if st.code == Code.ERROR:
            self.stats["errors"] += 1
            log.warning("scheduling %s failed: %s", res.pod_key, st.message())
        else:
            self.stats["unschedulable"] += 1
        self.handle.event(pi.pod, "FailedScheduling", st.message(), "Warning")
        self.queue.add_unschedulable(pi)
        self._snapshot = None
        self._record(res)
        return res

    def _record(self, res: ScheduleResult) -> None:
        if self.keep_results:
            with self._results_lock:
                self.results.append(res)
        if self.on_result:
            self.on_result(res)

    # ---------------------------------------------------------------- loops
    def schedule_pending(self, max_pods: Optional[int] = None, timeout_s: float = 0.0) -> List[ScheduleResult]:
        """Drain the active queue synchronously (tests / bench)."""
        out = []
        while max_pods is None or len(out) < max_pods:
            if self._waiting:
                self.expire_waiting()
            pi = self.queue.pop(timeout_s)
            if pi is None:
                break
            out.append(self.schedule_one(pi))
        return out

    def wait_for_binds(self, timeout_s: float = 30.0) -> bool:
        deadline = time.monotonic() + timeout_s
        with self._bind_cv:
            while self._pending_binds > 0:
                rem = deadline - time.monotonic()
                if rem <= 0:
                    return False
                self._bind_cv.wait(rem)
        return True

    def run(self) -> None:
        self.start_informers()
        from ..utils.gctune import settle
        settle()                            # the synced caches to the permanent GC generation
        last_cleanup = time.monotonic()
        while not self._stop.is_set():
            pi = self.queue.pop(0.2)
            if self._waiting:
                self.expire_waiting()
            if time.monotonic() - last_cleanup > 1.0:
                self.cache.cleanup_expired()
                last_cleanup = time.monotonic()
            if pi is None:
                continue
            try:
                self.schedule_one(pi)
            except Exception:
                log.exception("schedule_one crashed")
                self.queue.add_unschedulable(pi)

    def start(self) -> None:
        self._thread = threading.Thread(target=self.run, name="scheduler", daemon=True)
        self._thread.start()

    def stop(self) -> None:
        self._stop.set()
        self.queue.close()
        if self._thread:
            self._thread.join(timeout=5)
        if self._bind_pool:
            self._bind_pool.shutdown(wait=True)
        for fw in self.frameworks.values():
            fw.close()
        self.informers.stop()
