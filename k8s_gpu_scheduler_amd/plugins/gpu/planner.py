"""Joint placement of a burst of fractional GPU pods ("plan bursts").

The reference scores one pod at a time against the residents already on each device
(reference pkg/plugins/gpu_plugin/gpu_plugins.go:558-757), so a burst of pods arriving
together is placed greedily: whichever pod comes first takes the device that suits it,
and later pods get what is left -- co-locating workloads whose predicted interference
breaks their SLOs even when a different pairing would satisfy everyone.  On an 8-GPU
MI355X node a burst of 32 quarter-GPU pods fills every slot, so the *pairing* is the
whole decision.

At the first cycle of a burst (PreScore of a pod with no plan), the GPU plugin plans the
pod together with every pending fractional pod of the queue:

1. an initial feasible assignment: longest predicted work first onto the least-loaded GPU
   with free units / HBM (the balance objective);
2. the native core (`_core.plan_assignment`) improves it with pairwise swaps that raise the
   number of pods -- incoming and resident -- predicted to meet their SLO under the
   interference of their co-residents (the reference's `SLO > pred - intf` test), or keep
   that number and lower the busier GPU's interference-adjusted load (alone work stretched
   by the predicted slowdown `pred / (pred - intf)`: complementary pairs finish sooner),
   never letting a GPU's adjusted load exceed the initial plan's busiest GPU by more than
   `planTolerance`.

The plan is a hint: each pod still runs the full Filter/Score/Reserve cycle; Score ranks
the planned device first and every other choice after it, and a plan that no longer fits
(capacity taken meanwhile) is simply ignored.

With a co-run model (models.corun, served by the recommender) the plan is made on it
instead (`_plan_corun`, native `_core.plan_corun`): every GPU's pod group is simulated as a
whole, so the objective sees what the pairwise table cannot -- how long each co-runner
runs and how asymmetric the contention is.  Phase A balances the predicted group makespans
(the slowest GPU paces a coupled multi-GPU epoch), phase B then maximises the number of
pods -- burst and residents -- predicted to meet their SLO without letting any GPU's
makespan exceed (1 + planTolerance) x the balanced plan's longest.

With `planCarry` > 0 the planner also remembers how much predicted work each GPU took in
earlier bursts beyond the least-loaded GPU (its backlog, decayed by planCarry per burst) and
plans on backlog + makespan: the SLO phase's slack then evens out over bursts instead of
random-walking onto one GPU, whose cumulative work paces a pipelined multi-GPU job
(tools/virtual_node_bench.py replays the bench's launch-ahead pipeline over measured groups).
Measured feedback (bench epochs, cluster completions) never enters the backlog as raw ms: it
sets a per-GPU speed that scales the GPU's future increments, and the backlog is clipped
(`observe_time` and the constants above it) -- a bounded state, not an integrator.
"""
from __future__ import annotations

import os
from typing import Any, Dict, List, Optional, Tuple

import numpy as np

from ...api import objects as O
from ...recommender.tables import find_index_for_request
from .scoring import workload_column

Obj = Dict[str, Any]


def _median(xs) -> float:
    """Median of a short sequence (np.median costs ~100 us a call: 8 groups per burst)."""
    v = sorted(xs)
    n = len(v)
    return float(v[n // 2]) if n % 2 else 0.5 * (v[n // 2 - 1] + v[n // 2])


def rank_z(x: np.ndarray, y: np.ndarray) -> float:
    """Mann-Whitney z of sample x against sample y (normal approximation, ties counted half):
    > 0 when x tends to be larger.  O((n + m) log m) through a sorted y."""
    nx, ny = len(x), len(y)
    if nx == 0 or ny == 0:
        return 0.0
    ys = np.sort(y)
    lo = np.searchsorted(ys, x, "left")
    hi = np.searchsorted(ys, x, "right")
    u = float(lo.sum() + 0.5 * (hi - lo).sum())
    sd = (nx * ny * (nx + ny + 1) / 12.0) ** 0.5
    return (u - 0.5 * nx * ny) / sd if sd > 0 else 0.0


class EffortController:
    """Planning-effort control: keeps the burst planner's cost inside what it may take.

    Each decision compares the mean cost of the last plans at the current level with the mean
    time they were ALLOWED -- in the bench the interval between schedule requests (the GPUs'
    pipeline period: a control plane slower than that paces its GPUs), in a cluster the
    configured per-burst budget (`planBudgetMs`).  Over `down` x the allowed time on `patience`
    consecutive checks it jumps to the cheapest level predicted to fit `target` x (LEVEL_COST:
    measured relative cost per level), below `up` x it steps back one level if that level is
    predicted to fit; right after a change it re-measures (costs at the new level only; the
    first `settle` allowed-time samples, which still carry the old pace, are not taken).  The
    first decision acts on two samples without patience: a control plane that paces its GPUs
    from the start would carry that backlog into a timed region (rehearsed at 8 GPUs on the box
    CPU: profiles/archive/r04_cp_rehearsal/jump_first/)."""

    # relative cost of an epoch's scheduling per effort level (box CPU, 8 GPUs, tools/cp_timing.py
    # and tools/archive/gpu_cp_levels.sh: 5.78 / 4.68 / 4.09 ms, profiles/r05_cp_levels/; level 3 3.59 of
    # 5.75, profiles/r05_cp2/; round 4: 8.1 / 6.3 / 4.5 / 4.1)
    LEVEL_COST = (1.0, 0.81, 0.69, 0.63)

    def __init__(self, planner: "BurstPlanner", down: float = 0.85, up: float = 0.5, target: float = 0.7,
                 settle: int = 3, window: int = 6):
        import collections
        self.planner = planner
        self.down, self.up, self.target, self.settle_n = down, up, target, settle
        self._allowed: "collections.deque[float]" = collections.deque(maxlen=window)
        self._costs: "collections.deque[float]" = collections.deque(maxlen=window)
        self._settle = 0
        self._over = 0
        self._changed = False
        self.level_samples: Dict[int, int] = {}
        self.changes = 0
        self.debug = None            # callable(str) for a decision trace

    def add_cost(self, cost_s: float) -> None:
        self._costs.append(float(cost_s))

    def add_allowed(self, allowed_s: float) -> None:
        """One sample of the time a plan may take (skipped while settling after a change)."""
        if self._settle > 0:
            self._settle -= 1
            return
        self._allowed.append(float(allowed_s))

    def decide(self) -> int:
        """Act on the windows; returns the (possibly new) level."""
        pl = self.planner
        cur = pl.effort
        first = not self._changed
        need = 2 if first else 3
        if len(self._allowed) >= need and len(self._costs) >= need:
            allowed = sum(self._allowed) / len(self._allowed)
            cost = sum(self._costs) / len(self._costs)
            share = cost / max(allowed, 1e-12)
            base = cost / self.LEVEL_COST[min(cur, len(self.LEVEL_COST) - 1)]

            def fits(level: int) -> bool:
                return base * self.LEVEL_COST[min(level, len(self.LEVEL_COST) - 1)] <= self.target * allowed
            new = cur
            self._over = self._over + 1 if share > self.down else 0
            if self._over >= (1 if first else 2) and cur < pl.MAX_EFFORT:
                new = next((lv for lv in range(cur + 1, pl.MAX_EFFORT + 1) if fits(lv)), pl.MAX_EFFORT)
            elif share < self.up and cur > 0 and fits(cur - 1):
                new = cur - 1
            if self.debug is not None:
                self.debug(f"level {cur}->{new} share {share:.2f} allowed {[round(x * 1e3, 2) for x in self._allowed]} "
                           f"cost {[round(x * 1e3, 2) for x in self._costs]}")
            if new != cur:
                pl.set_effort(new)
                self._costs.clear()
                self._allowed.clear()
                self._settle = self.settle_n
                self._over = 0
                self._changed = True
                self.changes += 1
        self.level_samples[pl.effort] = self.level_samples.get(pl.effort, 0) + 1
        return pl.effort


class BurstPlanner:
    # sweeps: improvement passes of the native planners -- 4 and 8 plan alike (8-GPU pipelined
    # simulation, 3 seeds: 64.8 vs 65.3 % SLOs met, same pods/s) at half the control-plane time
    def __init__(self, plugin: Any, tolerance: float = 0.05, sweeps: int = 4, objective: str = "slo",
                 carry: float = 0.0, slots: Any = False, spread_ms: float = 2.0, slot_sigma: float = 0.2):
        if objective not in ("slo", "load"):
            raise ValueError(f"plan objective must be 'slo' or 'load', not {objective!r}")
        if not 0.0 <= carry <= 1.0:
            raise ValueError(f"plan carry must be in [0, 1], not {carry!r}")
        self.carry = carry
        self.backlog: Dict[Tuple, float] = {}             # co-run group key -> predicted ms
        self.last_increments: Dict[Tuple, float] = {}     # the last burst's predicted ms per group
        self._last_scaled: Dict[Tuple, float] = {}        # ... scaled by the groups' measured speeds
        self._speed_obs: Dict[Tuple, Any] = {}            # group -> recent measured / predicted ratios
        self._burst_ms = 0.0                              # a balanced burst's per-group work (EMA)
        self.plugin = plugin
        self.tolerance = tolerance
        self.load_first = objective == "load"
        self.sweeps = sweeps
        # pod key -> (node, device uuid, first CU-slice unit or None)
        self.plans: Dict[str, Tuple[str, str, Optional[int]]] = {}
        self.planned_bursts = 0
        # CU-slot planning on each GPU's pipeline (plugins.gpu.timeline): with a co-run model,
        # every planned pod also gets its slot -- the one whose predicted co-runners (the slot
        # pipelines' in-flight pods) let the most pods meet their SLOs, within spread_ms of the
        # most even slot ends (a slot running ahead idles once the pipeline's window is used up)
        # slots: "" (off: the ledger's best-fit unit range), "lpt" (each GPU's planned pods,
        # longest predicted work first, onto the CU slot with the least cumulative predicted
        # work -- the slot streams of a pipelined GPU stay level), "model" (the co-run model's
        # simulation of the slot pipelines, below); True = "model"
        # "auto": "model" when the plan spans several GPU groups (the model then also gives the
        # GPU choice each group's in-flight pipeline), "lpt" on a single GPU, where the slot
        # permutation is the only freedom and levelling measured better on MI355X
        self.slot_policy = "model" if slots is True else (slots or "")
        if self.slot_policy not in ("", "off", "lpt", "model", "auto"):
            raise ValueError(f"slot policy must be off, lpt, model or auto, not {slots!r}")
        if self.slot_policy == "off":
            self.slot_policy = ""
        self._slot_work: Dict[Tuple[str, int, int], float] = {}    # (device, first unit, units) -> ms
        self.timeline = None
        if self.slot_policy in ("model", "auto"):
            from .timeline import SlotTimeline
            # 2 phantom pods per slot: 65.6 % SLOs met vs 65.3 with 3 and 64.3 with 1 (8-GPU
            # pipelined simulation, 3 seeds), a smaller pipeline simulation per candidate
            self.timeline = SlotTimeline(depth=6, phantoms=2)
        self.spread_ms = spread_ms
        # model error of a slot plan's predictions: a pod's co-runners are partly pods placed
        # AFTER it, unknown at planning time (MI355X bench traces: mean |log error| ~0.2 with
        # the phantom continuation, vs ~0.06 once the co-runners are measured)
        self.slot_sigma = slot_sigma
        self.pipe_eval = True        # plan_corun's SLO phase on the GPUs' pipelines (timeline)
        self.pipe_phantoms = True    # ... with each slot's next (phantom) pod chained after its new one
        self.sweeps_b: Optional[int] = None     # SLO-phase sweeps (None: `sweeps`)
        # effort level (set_effort, EFFORT_LEVELS): 0 = as configured, 1 = a quarter of the
        # sweeps (phantoms kept), 2 = half the sweeps, no phantoms, slot levelling instead of the
        # model's slot plans and no pipeline evaluation, 3 = also one sweep per phase -- a control
        # plane that falls behind its GPUs trades plan quality for time.  (Dropping burst plans altogether is NOT cheaper at 8
        # GPUs: Score then evaluates the co-run groups of every candidate GPU per pod, 22.6 vs
        # 17.0 ms per epoch for level 2 in tools/cp_timing.py, at greedy's SLOs.)
        self.effort = 0
        self._configured = (self.sweeps, self.slot_policy)
        self._pool = None
        if self.timeline is not None:
            from concurrent.futures import ThreadPoolExecutor
            # the GPUs' slot plans can run side by side (native, without the interpreter lock;
            # GPUSCHED_SLOT_THREADS=n).  Off by default since the slot planner's context
            # fast-forward: at ~0.05 ms per GPU the threads' interpreter-lock hand-offs cost
            # more than they overlap (box CPU, 8 GPUs, tools/cp_breakdown.py: 1.0-2.0 ms of
            # slot planning per epoch on 8 threads vs ~0.4 ms of native work)
            n = max(1, min(8, int(os.environ.get("GPUSCHED_SLOT_THREADS", "1"))))
            self._pool = ThreadPoolExecutor(n, thread_name_prefix="slot-plan") if n > 1 else None
        # measured backlog feedback from pod completions (plugins.gpu.feedback; deployed
        # clusters -- the bench corrects per collected epoch instead)
        self.feedback = None
        if carry > 0:
            from .feedback import CompletionFeedback
            self.feedback = CompletionFeedback(self)
        # slot_plans / slot_pods: every slot plan (lpt or model); the model_* fields and the spread
        # / predicted-met sums only for the co-run model's slot plans (_plan_slots)
        self.stats = {"bursts": 0, "slot_plans": 0, "slot_pods": 0, "model_slot_plans": 0, "model_slot_pods": 0,
                      "slot_pred_met": 0, "slot_spread_ms": 0.0, "slot_min_spread_ms": 0.0}
        self.budget_ms = 0.0
        self.budget: Optional[EffortController] = None
        # slot plans still running on the native batch thread (_plan_slots): resolved when one of
        # their pods is asked for (plan), before the next burst and before stats are read
        import os as _os
        self.slots_async = _os.environ.get("GPUSCHED_SLOTS_ASYNC", "1") != "0"
        self._slot_pending: Optional[Dict[str, Any]] = None
        self._slot_job_of: Dict[str, int] = {}
        import time
        self.clock = time.perf_counter          # plan timing (a test may script it)

    MAX_EFFORT = 3

    def set_budget(self, budget_ms: float) -> None:
        """A deployed scheduler's per-burst planning budget (planBudgetMs; 0 = none): every burst
        plan's own wall time is measured and the effort level follows EffortController against
        the budget (over it: down to the level predicted to fit 80 % of it; under half of it:
        back up)."""
        self.budget_ms = float(budget_ms)
        self.budget = EffortController(self, down=1.0, up=0.5, target=0.8, settle=0) if budget_ms > 0 else None

    def _timed_plan(self, fn, *args) -> Any:
        """Run one burst plan; with a budget, feed its wall time to the effort controller."""
        n0 = self.stats["bursts"]
        t0 = self.clock()
        out = fn(*args)
        dt = self.clock() - t0
        if self.stats["bursts"] == n0:
            return out                   # nothing was planned (no burst): not a plan sample
        self.stats["plan_ms_last"] = round(dt * 1e3, 3)
        self.stats["plan_ms_sum"] = self.stats.get("plan_ms_sum", 0.0) + dt * 1e3
        self.stats["plans_timed"] = self.stats.get("plans_timed", 0) + 1
        if self.budget is not None:
            self.budget.add_cost(dt)
            self.budget.add_allowed(self.budget_ms / 1e3)
            self.budget.decide()
        return out

    # what each effort level plans with: (sweep divisor -- 0: one sweep --, pipeline phantoms,
    # pipeline evaluation, model slot plans).  Level 1 keeps the phantoms and drops sweeps: on
    # the 8-GPU pipelined virtual node (MI355X, profiles/r05_pvn_levels/) the phantoms carry the
    # SLO quality (level 1 with phantoms and 1 sweep: 60.4 % SLOs, the full plan 60.2 %, round
    # 5's first level 1 -- 2 sweeps, no phantoms -- 57.7 %, at the same pods/s; 59.5 vs 60.9 %
    # in a 3-seed rerun, profiles/r05_pvn_final/) and the sweeps the cost (box CPU: 4.68 vs
    # 5.02 ms per 8-GPU epoch, profiles/r05_cp_levels/)
    EFFORT_LEVELS = ((1, True, True, True), (4, True, True, True), (2, False, False, False), (0, False, False, False))

    @classmethod
    def _effort_levels(cls) -> Tuple[Tuple[int, bool, bool, bool], ...]:
        # experiments: GPUSCHED_EFFORT_LEVELS="1,1,1,1;2,0,1,1;2,0,0,0;0,0,0,0"
        env = os.environ.get("GPUSCHED_EFFORT_LEVELS")
        if not env:
            return cls.EFFORT_LEVELS
        rows = tuple(tuple(int(x) for x in r.split(",")) for r in env.split(";"))
        if len(rows) != cls.MAX_EFFORT + 1 or any(len(r) != 4 for r in rows):
            raise ValueError(f"GPUSCHED_EFFORT_LEVELS needs {cls.MAX_EFFORT + 1} rows of 4 fields: {env!r}")
        return tuple((r[0], bool(r[1]), bool(r[2]), bool(r[3])) for r in rows)

    def set_effort(self, level: int) -> None:
        level = max(0, min(self.MAX_EFFORT, int(level)))
        sweeps, slots = self._configured
        self.effort = level
        div, phantoms, pipe_eval, model_slots = self._effort_levels()[level]
        self.sweeps = 1 if div == 0 else max(1, sweeps // div)
        self.pipe_phantoms = phantoms
        self.pipe_eval = pipe_eval
        if slots in ("model", "auto"):
            self.slot_policy = slots if model_slots else "lpt"
        self.stats["effort_changes"] = self.stats.get("effort_changes", 0) + 1

    # ---------------------------------------------------------------- inputs
    def _matrix(self) -> Optional[Tuple[List[str], List[str], np.ndarray]]:
        tables = getattr(self.plugin.predictions, "tables", None)
        if tables is None:
            return None
        _, intf = tables()
        if intf is None or not intf.index:
            return None
        key = (id(intf), intf.version)
        hit = getattr(self, "_mcache", None)
        if hit is None or hit[0] != key:
            m = np.asarray([[intf.by_label[r].get(c, 0.0) for c in intf.columns] for r in intf.index], dtype=np.float64)
            self._mcache = hit = (key, (list(intf.index), list(intf.columns), np.nan_to_num(m)))
            # a pod's interference lookup returns its row's dict object: row index by identity
            self._row_of = {id(intf.by_label[r]): i for i, r in enumerate(intf.index)}
            self._col_of = {c: j for j, c in enumerate(intf.columns)}
        return hit[1]

    def _ids(self, name: str, index: List[str], columns: List[str]) -> Tuple[int, int]:
        """(interference row, column) of a pod: the row from the identity of the row dict its
        (memoised) prediction lookup returned, the column by the recommender's substring
        rule."""
        _, intf = self.plugin._pod_predictions(name)
        r = self._row_of.get(id(intf), -1) if intf else -1
        if r < 0 and intf:
            lab = find_index_for_request(f"{name}_{self.plugin.args.model}".replace("-", "_"), index)
            r = index.index(lab) if lab else -1
        c = self.plugin._workload_col(name, intf) if intf else workload_column(name, dict.fromkeys(columns))
        return r, self._col_of.get(c, -1) if c is not None else -1

    # ---------------------------------------------------------------- plan
    def plan(self, pod: Obj, nodes: List[str]) -> Optional[Tuple[str, str]]:
        """Plan `pod` with the pending fractional pods over the devices of `nodes` (the
        pod's feasible nodes); returns its (node, device uuid)."""
        key = O.key(pod)
        hit = self.plans.get(key)
        if hit is not None:
            j = self._slot_job_of.get(key)
            if j is not None:
                self._resolve_slots(j)
                hit = self.plans.get(key)
            return hit
        from ... import _native
        core = _native.core()
        model = self.plugin.corun_model()
        if model is not None and core is not None and hasattr(core, "plan_corun"):
            return self._timed_plan(self._plan_corun, pod, nodes, model, core)
        mat = self._matrix()
        if core is None or mat is None or not hasattr(core, "plan_assignment"):
            return None
        index, columns, M = mat
        plugin = self.plugin
        placed = [(nd, st) for nd in nodes for st in plugin.ledger.devices(nd) if st.device.healthy]
        if not placed:
            return None
        states = [st for _, st in placed]
        owner = [nd for nd, _ in placed]
        # the burst: this pod + pending fractional pods of this scheduler not planned yet
        burst, seen = [], {key}
        for p in [pod] + list(plugin.handle.pending_pods() if plugin.handle is not None else []):
            k = O.key(p)
            if (k in seen and p is not pod) or k in self.plans or O.node_name_of(p):
                continue
            seen.add(k)
            req = plugin.parse_request(p)
            if req.units and not req.whole and req.gpu_pod:
                burst.append((p, req))
        if len(burst) < 2:
            return None
        dev_index = {(owner[d], st.device.uuid): d for d, st in enumerate(states)}
        gkeys = sorted({(owner[d], st.device.gpu) for d, st in enumerate(states)})
        gpos = {g: i for i, g in enumerate(gkeys)}
        gof = [gpos[(owner[d], st.device.gpu)] for d, st in enumerate(states)]
        free_units = [st.free_units for st in states]
        free_hbm = [st.hbm_free for st in states]
        load = [0.0] * len(gkeys)
        res_dev, res_row, res_col, res_slo, res_pred = [], [], [], [], []
        for d, st in enumerate(states):
            load[gof[d]] += st.work
            for use in st.pods.values():
                conf, _ = plugin._pod_predictions(use.name)
                r, c = self._ids(use.name, index, columns)
                res_dev.append(d)
                res_row.append(r)
                res_col.append(c)
                res_slo.append(use.slo)
                res_pred.append(conf.get(plugin._col(use.units[1], st.device.units), -1.0) if conf else -1.0)
        # pods planned earlier and still pending hold their capacity / interfere as residents
        for k, (n, u) in self.plans.items():
            d = dev_index.get((n, u))
            if d is None:
                continue
            p = plugin._pending_by_key.get(k)
            if p is None:
                continue
            req = plugin.parse_request(p)
            free_units[d] -= req.units
            free_hbm[d] -= req.hbm_gib
            conf, _ = plugin._pod_predictions(O.name(p))
            r, c = self._ids(O.name(p), index, columns)
            res_dev.append(d)
            res_row.append(r)
            res_col.append(c)
            res_slo.append(req.slo)
            res_pred.append(conf.get(plugin._col(req.units, states[d].device.units), -1.0) if conf else -1.0)
            load[gof[d]] += plugin.pod_work(p, conf)
        base_load = list(load)
        # 1. initial assignment: longest predicted work first, least-loaded GPU with room
        items = []
        for p, req in burst:
            conf, _ = plugin._pod_predictions(O.name(p))
            items.append((plugin.pod_work(p, conf), p, req, conf))
        items.sort(key=lambda t: -t[0])
        assign: List[Tuple[Any, Any, Any, int, float]] = []
        # equal loads are broken by a per-burst rotation of the device order: a fixed order
        # would hand the same GPU the longest pod of every burst, and any bias in the
        # predicted work would then pile up on that GPU across epochs (in a pipelined
        # multi-GPU job the per-GPU totals, not one epoch's, pace the ranks)
        rot = (self.planned_bursts * 5 + 1) % max(len(states), 1)
        nst = len(states)
        for work, p, req, conf in items:
            best = None
            for d, st in enumerate(states):
                if free_units[d] < req.units or free_hbm[d] + 1e-6 < req.hbm_gib:
                    continue
                k2 = (load[gof[d]], (d - rot) % nst)
                if best is None or k2 < best[0]:
                    best = (k2, d)
            if best is None:
                continue                      # does not fit now: left to the normal cycle
            d = best[1]
            free_units[d] -= req.units
            free_hbm[d] -= req.hbm_gib
            load[gof[d]] += work
            assign.append((p, req, conf, d, work))
        if len(assign) < 2:
            return None
        n = len(assign)
        dev = np.array([a[3] for a in assign], dtype=np.int32)
        units = np.array([a[1].units for a in assign], dtype=np.int32)
        rows, cols, slo, pred, work = [], [], [], [], []
        for p, req, conf, d, w in assign:
            r, c = self._ids(O.name(p), index, columns)
            rows.append(r)
            cols.append(c)
            slo.append(req.slo)
            pred.append(conf.get(plugin._col(req.units, states[d].device.units), -1.0) if conf else -1.0)
            work.append(w)
        out = core.plan_assignment(
            dev, units, np.array(rows, dtype=np.int32), np.array(cols, dtype=np.int32),
            np.array(slo, dtype=np.float64), np.array(pred, dtype=np.float64), np.array(work, dtype=np.float64),
            np.array(gof, dtype=np.int32), np.array(base_load, dtype=np.float64),
            np.array(res_dev, dtype=np.int32), np.array(res_row, dtype=np.int32), np.array(res_col, dtype=np.int32),
            np.array(res_slo, dtype=np.float64), np.array(res_pred, dtype=np.float64), M, 0.0,
            self.sweeps, float(self.tolerance), int(self.load_first))
        for (p, _, _, _, _), d in zip(assign, out[:n]):
            self.plans[O.key(p)] = (owner[int(d)], states[int(d)].device.uuid)
            plugin._pending_by_key[O.key(p)] = p
        self.planned_bursts += 1
        return self.plans.get(key)

    # ---------------------------------------------------------------- co-run plan
    def _burst(self, pod: Obj) -> List[Tuple[Obj, Any]]:
        """This pod + the pending fractional pods of this scheduler not planned yet."""
        plugin = self.plugin
        key = O.key(pod)
        burst, seen = [], {key}
        for p in [pod] + list(plugin.handle.pending_pods() if plugin.handle is not None else []):
            k = O.key(p)
            if (k in seen and p is not pod) or k in self.plans or O.node_name_of(p):
                continue
            seen.add(k)
            req = plugin.parse_request(p)
            if req.units and not req.whole and req.gpu_pod:
                burst.append((p, req))
        return burst

    def _plan_corun(self, pod: Obj, nodes: List[str], model: Any, core: Any) -> Optional[Tuple[str, str]]:
        plugin = self.plugin
        key = O.key(pod)
        self._resolve_slots()
        placed = [(nd, st) for nd in nodes for st in plugin.ledger.devices(nd) if st.device.healthy]
        if not placed:
            return None
        states = [st for _, st in placed]
        owner = [nd for nd, _ in placed]
        burst = [(p, r) for p, r in self._burst(pod) if model.wid(O.name(p)) >= 0]
        if len(burst) < 2 or not any(O.key(p) == key for p, _ in burst):
            return None
        gkey = {}
        dev_group = []
        for nd, st in placed:
            dev_group.append(gkey.setdefault((nd,) + plugin.corun_group_key(st), len(gkey)))
        n_groups = len(gkey)
        if n_groups < 2 and not self.slot_policy:
            return None                     # one co-run group (one GPU) and no slots to plan
        free_units = [st.free_units for st in states]
        free_hbm = [st.hbm_free for st in states]
        per: List[List[Tuple[int, float, float]]] = [[] for _ in range(n_groups)]
        margin = 1.0 + plugin.args.corun_margin      # SLOs as the model must predict them
        seen = set()
        for d, st in enumerate(states):
            g = dev_group[d]
            for k, use in st.pods.items():
                if (k, g) in seen:
                    continue
                seen.add((k, g))
                w = model.wid(use.name)
                if w >= 0:
                    per[g].append((w, use.iters, use.slo * margin))
        dev_index = {(owner[d], st.device.uuid): d for d, st in enumerate(states)}
        # pods planned earlier and still pending hold their capacity and co-run as residents
        for k, (n, u) in self.plans.items():
            d = dev_index.get((n, u))
            p = plugin._pending_by_key.get(k)
            if d is None or p is None:
                continue
            req = plugin.parse_request(p)
            free_units[d] -= req.units
            free_hbm[d] -= req.hbm_gib
            w = model.wid(O.name(p))
            if w >= 0:
                per[dev_group[d]].append((w, req.iters, req.slo * margin))
        # initial assignment: longest predicted work first onto the group with the least
        # predicted work that has room (units and HBM)
        load = [sum(model.alone_ms[w] * (it if it > 0 else 0.0) for w, it, _ in m) for m in per]
        items = sorted(((model.alone_ms[model.wid(O.name(p))] * max(r.iters, 0.0), p, r) for p, r in burst),
                       key=lambda t: -t[0])
        rot = (self.planned_bursts * 5 + 1) % max(len(states), 1)
        nst = len(states)
        assign = []
        for work, p, r in items:
            best = None
            for d in range(nst):
                if free_units[d] < r.units or free_hbm[d] + 1e-6 < r.hbm_gib:
                    continue
                k2 = (load[dev_group[d]], (d - rot) % nst)
                if best is None or k2 < best[0]:
                    best = (k2, d)
            if best is None:
                continue
            d = best[1]
            free_units[d] -= r.units
            free_hbm[d] -= r.hbm_gib
            load[dev_group[d]] += work
            assign.append((p, r, d))
        if len(assign) < 2:
            return None
        self._burst_unit = min((r.units for _, r, _ in assign if r.units), default=0)
        if max((len(m) for m in per), default=0) + len(assign) > 64:
            return None
        off = np.zeros(n_groups + 1, np.int64)
        off[1:] = np.cumsum([len(m) for m in per])
        flat = [x for m in per for x in m]
        dev0 = np.array([d for _, _, d in assign], np.int32)
        units = np.array([r.units for _, r, _ in assign], np.int32)
        # capacity before the burst (the native planner subtracts the initial assignment)
        cap = np.array(free_units, np.int32)
        np.add.at(cap, dev0, units)
        hbm = np.array([r.hbm_gib for _, r, _ in assign], np.float64)
        cap_hbm = np.array(free_hbm, np.float64)
        np.add.at(cap_hbm, dev0, hbm)
        gkeys = sorted(gkey, key=gkey.get)
        base = self.plan_base(gkeys) if self.carry > 0 else None
        r_wid = np.array([x[0] for x in flat], np.int32)
        r_iters = np.array([x[1] for x in flat], np.float64)
        r_slo = np.array([x[2] for x in flat], np.float64)
        pipe = self._pipe_context(gkey, states, owner, dev_group, model, core) if (self.timeline is not None and self.pipe_eval) else None
        if n_groups >= 2:
            out = core.plan_corun(
                dev0, units, np.array([model.wid(O.name(p)) for p, _, _ in assign], np.int32),
                np.array([r.iters for _, r, _ in assign], np.float64),
                np.array([r.slo * margin for _, r, _ in assign], np.float64),
                np.array(dev_group, np.int32), cap, off, r_wid, r_iters, r_slo,
                model.alone_ms, model.coupling(), self.sweeps, float(self.tolerance), 0,
                float(plugin.args.corun_sigma), base, pipe, hbm, cap_hbm,
                -1 if self.sweeps_b is None else int(self.sweeps_b),
                np.array(self.rel_speeds(gkeys), np.float64) if self._speed_obs else None)
            if self.carry > 0:
                self._carry(gkeys, per, assign, out, dev_group, model, core, off, r_wid, r_iters, r_slo)
        else:
            out = dev0
        slot_of: Dict[str, int] = {}
        if self.timeline is not None:
            self.timeline.next_burst()
        if self.slot_policy == "model" or (self.slot_policy == "auto" and n_groups >= 2):
            self._trigger_key = key
            slot_of = self._plan_slots(assign, out, states, owner, dev_group, model, core, margin)
        elif self.slot_policy in ("lpt", "auto"):
            slot_of = self._lpt_slots(assign, out, states, model)
        for (p, _, _), d in zip(assign, out):
            self.plans[O.key(p)] = (owner[int(d)], states[int(d)].device.uuid, slot_of.get(O.key(p)))
            plugin._pending_by_key[O.key(p)] = p
        self.planned_bursts += 1
        self.stats["bursts"] += 1
        return self.plans.get(key)

    # ---------------------------------------------------------------- slot plan
    def _free_slots(self, st: Any, n: int, busy: set) -> List[Tuple[int, int]]:
        align = 1
        while align < n:
            align *= 2
        return [(u, n) for u in range(0, st.device.units - n + 1, align)
                if not any(st.used_units[u:u + n]) and u not in busy]

    def _taken_slots(self) -> Dict[str, set]:
        """First units of the slots planned for still-pending pods, per device."""
        self._resolve_slots()
        taken: Dict[str, set] = {}
        for k, pl in self.plans.items():
            if len(pl) > 2 and pl[2] is not None and k in self.plugin._pending_by_key:
                taken.setdefault(pl[1], set()).add(pl[2])
        return taken

    def _lpt_slots(self, assign, out, states, model) -> Dict[str, int]:
        """slot policy "lpt": per device, its planned pods of one size longest predicted work
        (co-run model alone time x iterations) first, each onto the free slot whose stream has
        the least cumulative predicted work so far (ties: the lower slot).  On a pipelined GPU
        the slot streams then stay level over the epochs (a first-fit order gives slot 0 the
        longest pod of every burst, and the pipeline waits on it); replaces the bench
        executor's SLO-blind re-slotting, which ran after the scheduler had decided."""
        by_dev: Dict[int, List[Tuple[Any, Any]]] = {}
        for (p, r, _), d in zip(assign, out):
            by_dev.setdefault(int(d), []).append((p, r))
        taken = self._taken_slots()
        res: Dict[str, int] = {}
        for d, items in by_dev.items():
            st = states[d]
            uuid = st.device.uuid
            sizes = {r.units for _, r in items}
            if len(sizes) != 1:
                continue
            n = sizes.pop()
            slots = [u for u, _ in self._free_slots(st, n, taken.get(uuid, set()))]
            if len(slots) < len(items):
                continue
            work = {O.key(p): float(model.alone_ms[model.wid(O.name(p))]) * max(r.iters, 1.0) for p, r in items}
            for p, r in sorted(items, key=lambda x: -work[O.key(x[0])]):
                u = min(slots, key=lambda s: (self._slot_work.get((uuid, s, n), 0.0), s))
                slots.remove(u)
                res[O.key(p)] = u
                self._slot_work[(uuid, u, n)] = self._slot_work.get((uuid, u, n), 0.0) + work[O.key(p)]
            self.stats["slot_plans"] += 1
            self.stats["slot_pods"] += len(items)
        return res

    def _pipe_context(self, gkey: Dict[Tuple, int], states, owner, dev_group, model, core) -> Any:
        """plan_corun's `pipe`: per GPU group of one device, its timeline's in-flight pods
        (pinned at measured / predicted intervals) and its free slots' free times."""
        if not hasattr(core, "chain_times"):
            return None
        n_groups = len(gkey)
        ndev = [0] * n_groups
        dev_of = [-1] * n_groups
        for d, g in enumerate(dev_group):
            ndev[g] += 1
            dev_of[g] = d
        unit = getattr(self, "_burst_unit", 0)       # the burst's smallest slot size (_plan_corun)
        c_off, f_off = [0], [0]
        parts = []                                   # per GPU: (w, start, end, free, ph wid, ph iters)
        nc = nf = 0
        for g in range(n_groups):
            d = dev_of[g]
            if ndev[g] == 1 and unit > 0:
                st = states[d]
                slots = self._free_slots(st, unit, set())
                p = self.timeline.pipeline((owner[d],) + self.plugin.corun_group_key(st), slots, model, core,
                                           with_phantoms=True)
                parts.append(p)
                nc += len(p[0])
                nf += len(p[3])
            c_off.append(nc)
            f_off.append(nf)
        if not nc and not nf:
            return None

        def cat(i, dt):
            return np.concatenate([p[i] for p in parts]).astype(dt, copy=False)
        out = (np.asarray(c_off, np.int64), cat(0, np.int32), cat(1, np.float64), cat(2, np.float64),
               np.asarray(f_off, np.int64), cat(3, np.float64))
        if self.pipe_phantoms:
            # per free slot, the workload its stream runs next (-1: none), chained after the
            # slot's new pod (native plan_corun)
            out += (cat(4, np.int32), cat(5, np.float64))
        return out

    def _plan_slots(self, assign, out, states, owner, dev_group, model, core, margin: float) -> Dict[str, int]:
        """CU slot of every planned pod on its GPU: the GPU's slot pipelines (the timeline's
        in-flight pods, measured ones pinned) plus the new pods, every injective assignment
        simulated (native plan_slots).  Only for a GPU group of one device whose new pods
        share one size; anything else keeps the ledger's best-fit slot."""
        if not hasattr(core, "plan_slots"):
            return {}
        plugin = self.plugin
        trigger = getattr(self, "_trigger_key", None)
        per_group_devs: Dict[int, int] = {}
        for g in dev_group:
            per_group_devs[g] = per_group_devs.get(g, 0) + 1
        by_dev: Dict[int, List[Tuple[Any, Any]]] = {}
        for (p, r, _), d in zip(assign, out):
            by_dev.setdefault(int(d), []).append((p, r))
        taken = self._taken_slots()
        res: Dict[str, int] = {}
        jobs = []
        for d, items in by_dev.items():
            st = states[d]
            if per_group_devs.get(dev_group[d], 0) != 1:
                continue
            sizes = {r.units for _, r in items}
            if len(sizes) != 1:
                continue
            n = sizes.pop()
            slots = self._free_slots(st, n, taken.get(st.device.uuid, set()))
            if len(slots) < len(items):
                continue
            gk = (owner[d],) + plugin.corun_group_key(st)
            ctx = self.timeline.context(gk, slots)
            if len(ctx["wid"]) + len(items) + len(ctx["ph_wid"]) > 64:
                continue
            nw = np.array([model.wid(O.name(p)) for p, _ in items], np.int32)
            args = (ctx["wid"], ctx["iters"], ctx["start"], ctx["prev"], ctx["pin"], ctx["slo"], ctx["slot_tail"],
                    ctx["slot_free"], nw, np.array([r.iters for _, r in items], np.float64),
                    np.array([r.slo * margin for _, r in items], np.float64), np.full(len(items), -1e300),
                    model.alone_ms, model.coupling(), float(self.slot_sigma), float(self.spread_ms), 720,
                    ctx["ph_off"], ctx["ph_wid"], ctx["ph_iters"])
            jobs.append((items, slots, ctx, args))
        # the GPUs' slot plans are independent; only the first pod's is needed now.  Async (the
        # default): one native batch thread runs them, the triggering pod's GPU first, while the
        # burst's other pods go through their cycles; each is resolved when its pod is planned
        # (plan), so the ~0.1 ms per GPU overlaps the Python scheduling work instead of adding to
        # it.  Else: on the planner's worker threads (GPUSCHED_SLOT_THREADS) or in turn.
        if self.slots_async and len(jobs) > 1 and hasattr(core, "plan_slots_async"):
            first = next((i for i, jb in enumerate(jobs) if any(O.key(p) == trigger for p, _ in jb[0])), 0)
            jobs.insert(0, jobs.pop(first))
            batch = core.plan_slots_async([tuple(jb[3]) + (True,) for jb in jobs])
            self._slot_pending = {"batch": batch, "jobs": jobs, "margin": margin, "left": set(range(len(jobs)))}
            for j, jb in enumerate(jobs):
                for p, _ in jb[0]:
                    self._slot_job_of[O.key(p)] = j
            res.update(self._slot_result(0, self._batch_result(batch, 0)))
            return res
        if len(jobs) > 1 and self._pool is not None:
            outs = list(self._pool.map(lambda j: core.plan_slots(*j[3]), jobs))
        else:
            outs = [core.plan_slots(*j[3]) for j in jobs]
        for jb, out in zip(jobs, outs):
            res.update(self._apply_slot_plan(jb, out, margin))
        return res

    def _apply_slot_plan(self, job, out, margin: float) -> Dict[str, int]:
        """One GPU's slot plan: the pods' slots, and the slot-plan stats."""
        items, slots, ctx, _ = job
        sl, st0, fin, exp, spread, min_spread = out
        res = {}
        for (p, _), s in zip(items, sl):
            res[O.key(p)] = slots[int(s)][0]
        self.stats["slot_plans"] += 1
        self.stats["slot_pods"] += len(items)
        self.stats["model_slot_plans"] += 1
        self.stats["model_slot_pods"] += len(items)
        # the new pods predicted to meet their SLO on the chosen slots (hard counts; `exp`
        # also covers the unmeasured context pods the choice re-predicts)
        m0 = len(ctx["wid"])
        for j, (_, r) in enumerate(items):
            d_ms = float(fin[m0 + j] - st0[m0 + j])
            if r.slo <= 0 or (d_ms > 0 and r.iters / d_ms * 1e3 >= r.slo * margin):
                self.stats["slot_pred_met"] += 1
        self.stats["slot_spread_ms"] += float(spread)
        self.stats["slot_min_spread_ms"] += float(min_spread)
        return res

    @staticmethod
    def _batch_result(batch, j: int):
        """Job j of an async slot batch; None (the ledger's best-fit slots) if it failed -- the
        slot plan only refines a placement, and its error would surface in a later pod's cycle."""
        try:
            return batch.result(j)
        except Exception as e:
            import logging
            logging.getLogger(__name__).warning("slot plan %d failed: %s (best-fit slots)", j, e)
            return None

    def _slot_result(self, j: int, out) -> Dict[str, int]:
        pend = self._slot_pending
        pend["left"].discard(j)
        res = self._apply_slot_plan(pend["jobs"][j], out, pend["margin"]) if out is not None else {}
        for p, _ in pend["jobs"][j][0]:
            self._slot_job_of.pop(O.key(p), None)
        if not pend["left"]:
            pend["batch"].join()
            self._slot_pending = None
        return res

    def _resolve_slots(self, j: Optional[int] = None) -> None:
        """Collect pending async slot plans (job j, or all) into the pods' plans."""
        pend = self._slot_pending
        if pend is None:
            return
        for i in ([j] if j is not None else sorted(pend["left"])):
            if i not in pend["left"]:
                continue
            for k, u0 in self._slot_result(i, self._batch_result(pend["batch"], i)).items():
                pl = self.plans.get(k)
                if pl is not None:
                    self.plans[k] = (pl[0], pl[1], u0)
            if self._slot_pending is None:
                break

    def flush(self) -> None:
        """Finish every pending slot plan (stats readers; tests)."""
        self._resolve_slots()

    def placed(self, pod: Obj, node: str, choice: Any, req: Any) -> None:
        """Reserve: the pod took `choice` -- append it to its GPU's slot timeline, and record
        its predicted duration next to its co-residents for the completion feedback."""
        if (self.timeline is None and self.feedback is None) or choice is None:
            return
        model = self.plugin.corun_model()
        if model is None:
            return
        w = model.wid(O.name(pod))
        frac = [a for a in choice.allocs if not a[4]]
        if w < 0 or len(frac) != 1:
            return
        uuid, u0, n = frac[0][0], frac[0][1], frac[0][2]
        st = next((s for s in self.plugin.ledger.devices(node) if s.device.uuid == uuid), None)
        if st is None:
            return
        group = (node,) + self.plugin.corun_group_key(st)
        if self.feedback is not None and req.iters > 0:
            mem = [(k, model.wid(u.name), u.iters) for s in self.plugin.ledger.devices(node)
                   if (node,) + self.plugin.corun_group_key(s) == group for k, u in s.pods.items()]
            mem = [(k, wi, it) for k, wi, it in mem if wi >= 0 and it > 0]
            keys = [k for k, _, _ in mem]
            if O.key(pod) in keys and len(mem) <= 64:
                # every member's prediction is refreshed with the group as it now stands: a pod
                # placed earlier co-runs with this one too
                d = model.group_durations([wi for _, wi, _ in mem], [it for _, _, it in mem])
                self.feedback.expect(O.key(pod), group, float(d[keys.index(O.key(pod))]))
                for k, x in zip(keys, d):
                    if k != O.key(pod):
                        self.feedback.refresh(k, group, float(x))
        if self.timeline is None:
            return
        margin = 1.0 + self.plugin.args.corun_margin
        self.timeline.place((node,) + self.plugin.corun_group_key(st), (u0, n), O.key(pod), w, req.iters,
                            req.slo * margin)

    # ------------------------------------------------------------ backlog control
    # The backlog is a bounded state (round 4's plain integrator of measured-minus-predicted
    # deltas kept every outlier forever: one lazily captured HIP graph inside a measured pod
    # made a GPU's relative backlog exceed a whole burst, and phase A handed the next burst
    # entirely to its sibling, GPUTEST_r04.json):
    #  * measurements never enter the backlog as ms; they set each group's SPEED, the window
    #    median of its last SPEED_WINDOW measured / predicted ratios (each clipped to
    #    SPEED_CLIP), relative to the median group, with a dead band -- one outlier does not move
    #    a median, a persistently slower GPU does after SPEED_MIN_OBS observations;
    #  * a burst's predicted increments enter the backlog scaled by the group's speed, so a GPU
    #    10 % slower is planned as if its pods were 10 % longer (its steady share is then the
    #    one that levels the measured work, not a diverging integral);
    #  * the stored relative backlog is clipped to STORE_CLIP x a balanced burst's per-group
    #    work (anti-windup when capacity leaves the plan no way to even it out), and the plans
    #    see at most SPREAD_CLIP x that (a tighter clip of 0.5 / 1.0 bursts cost the 8-GPU
    #    simulated pipeline 1-4 % pods/s: the carry needs about two bursts of range to even out
    #    the SLO phase's slack); the native planner itself never empties a GPU of a burst that
    #    has a pod for every GPU (plan_corun), so carried backlog cannot starve a GPU.
    SPEED_WINDOW = 16
    SPEED_MIN_OBS = 3
    SPEED_CLIP = (0.5, 2.0)
    SPEED_DEADBAND = 0.02
    # A group's speed counts only when a rank test says its window differs from the other
    # groups' pooled windows: Mann-Whitney U, two-sided, |z| >= SPEED_Z (alpha 0.02), after
    # SPEED_TEST_MIN observations.  Round 5 required EVERY one of 7 window observations on the
    # group's side of the median group -- at the ~8 % epoch-to-epoch noise of identical GPUs'
    # pipelined busy times (which had scattered their "speeds" and cost the 8-GPU simulated
    # pipeline 4-8 % pods/s) that gate also hid a GPU 10-20 % slower (VERDICT r5 weak #2:
    # shares 0.50 instead of 0.476 / 0.455).  The rank test is distribution-free (heavy-tailed
    # pipeline noise included) and sees a persistent 10 % slowdown at +-8 % noise within a
    # window, while identical GPUs pass it about twice per 100 decisions.
    SPEED_Z = 2.33
    SPEED_TEST_MIN = 5
    # before SPEED_TEST_MIN observations the normal approximation cannot reach SPEED_Z; a large
    # shift (|r - 1| >= SPEED_EARLY_EFFECT) whose window lies wholly beyond every other
    # group's observations counts from SPEED_MIN_OBS on (a GPU 40 % slower, seen in 3 epochs)
    SPEED_EARLY_EFFECT = 0.1
    SPREAD_CLIP = 2.0
    STORE_CLIP = 4.0

    def observe_time(self, group: Tuple, predicted_ms: float, measured_ms: float) -> None:
        """Measured feedback: `group` ran work predicted at `predicted_ms` in `measured_ms`
        (the bench: a GPU's busy time for a collected epoch; a cluster: a finished pod's run
        time normalised by the node-wide median ratio, plugins.gpu.feedback)."""
        if self.carry <= 0 or not (predicted_ms > 0 and measured_ms > 0):
            return
        import collections
        lo, hi = self.SPEED_CLIP
        q = self._speed_obs.get(group)
        if q is None:
            q = self._speed_obs[group] = collections.deque(maxlen=self.SPEED_WINDOW)
        q.append(min(hi, max(lo, measured_ms / predicted_ms)))
        self.stats["speed_obs"] = self.stats.get("speed_obs", 0) + 1

    def speed(self, group: Tuple) -> float:
        """The group's measured / predicted time ratio (1.0 until SPEED_MIN_OBS observations)."""
        q = self._speed_obs.get(group)
        if not q or len(q) < self.SPEED_MIN_OBS:
            return 1.0
        return _median(q)

    def rel_speeds(self, gkeys: List[Tuple]) -> List[float]:
        """Each group's speed over the median group's (a uniform slowdown changes nothing), 1.0
        inside the dead band -- and 1.0 unless the group's window differs from the other groups'
        pooled windows by a rank test in the same direction (SPEED_Z): a GPU that is really
        slower shifts its whole window, while the pipeline's epoch-to-epoch accounting noise
        scatters identical GPUs' windows around each other."""
        stamp = (self.stats.get("speed_obs", 0), tuple(gkeys))
        hit = getattr(self, "_rel_cache", None)
        if hit is not None and hit[0] == stamp:
            return list(hit[1])
        s = [self.speed(k) for k in gkeys]
        med = _median(s) if s else 1.0
        wins = [np.asarray(self._speed_obs.get(k) or (), np.float64) for k in gkeys]
        out = []
        for i, x in enumerate(s):
            r = x / med if med > 0 else 1.0
            x = wins[i]
            others = [w for j, w in enumerate(wins) if j != i and len(w)]
            if abs(r - 1.0) < self.SPEED_DEADBAND or len(x) < self.SPEED_MIN_OBS or not others:
                out.append(1.0)
                continue
            y = np.concatenate(others)
            if len(x) < self.SPEED_TEST_MIN:
                sep = x.min() > y.max() if r > 1.0 else x.max() < y.min()
                out.append(r if sep and abs(r - 1.0) >= self.SPEED_EARLY_EFFECT else 1.0)
                continue
            z = rank_z(x, y)
            out.append(r if (z >= self.SPEED_Z and r > 1.0) or (z <= -self.SPEED_Z and r < 1.0) else 1.0)
        self._rel_cache = (stamp, tuple(out))
        return out

    def plan_base(self, gkeys: List[Tuple]) -> np.ndarray:
        """The relative backlog the plan sees per group, clipped to SPREAD_CLIP x a balanced
        burst's per-group work."""
        raw = [self.backlog.get(k, 0.0) for k in gkeys]
        lo = min(raw) if raw else 0.0
        cap = self.SPREAD_CLIP * self._burst_ms if self._burst_ms > 0 else 0.0
        return np.array([min(x - lo, cap) for x in raw], np.float64)

    def _carry(self, gkeys, per, assign, out, dev_group, model, core, off, r_wid, r_iters, r_slo) -> None:
        """Backlog bookkeeping after a co-run plan: each group's predicted makespan increase
        from this burst (residents alone before, residents + planned pods after), scaled by
        its measured relative speed, is added to its backlog; backlogs decay by `carry` per
        burst, are kept relative to the least loaded group (only differences steer the plan)
        and clipped (anti-windup, above)."""
        if len(r_wid):
            _, mk0 = core.corun_groups_eval(off, r_wid, r_iters, r_slo, model.alone_ms, model.coupling())
        else:                               # no residents anywhere (e.g. every GPU drained)
            mk0 = np.zeros(len(gkeys))
        groups = [list(m) for m in per]
        for (p, r, _), d in zip(assign, out):
            groups[dev_group[int(d)]].append((model.wid(O.name(p)), r.iters, r.slo))
        off1 = np.zeros(len(groups) + 1, np.int64)
        off1[1:] = np.cumsum([len(m) for m in groups])
        flat1 = [x for m in groups for x in m]
        _, mk1 = core.corun_groups_eval(off1, np.array([x[0] for x in flat1], np.int32),
                                        np.array([x[1] for x in flat1], np.float64),
                                        np.array([x[2] for x in flat1], np.float64), model.alone_ms, model.coupling())
        self.last_increments = {}
        self._last_scaled = {}
        speeds = self.rel_speeds(gkeys)
        incs = []
        for g, k in enumerate(gkeys):
            inc = max(float(mk1[g]) - float(mk0[g]), 0.0)
            incs.append(inc)
            self.last_increments[k] = inc
            self._last_scaled[k] = inc * speeds[g]
            self.backlog[k] = self.carry * self.backlog.get(k, 0.0) + inc * speeds[g]
        mean_inc = sum(incs) / len(incs) if incs else 0.0
        if mean_inc > 0:
            self._burst_ms = mean_inc if self._burst_ms <= 0 else 0.5 * (self._burst_ms + mean_inc)
        lo = min(self.backlog[k] for k in gkeys)
        cap = self.STORE_CLIP * self._burst_ms if self._burst_ms > 0 else float("inf")
        for k in gkeys:
            self.backlog[k] = min(self.backlog[k] - lo, cap)

    def realign(self) -> None:
        """Every group has drained (e.g. a pipelined job synchronised its GPUs): the carried
        backlog is void, except the last planned burst, which has not run yet.  The measured
        speeds are a property of the GPUs and stay."""
        if self.timeline is not None:
            self.timeline.realign()
        self.backlog = dict(self._last_scaled or self.last_increments)
        if self.backlog:
            lo = min(self.backlog.values())
            for k in self.backlog:
                self.backlog[k] -= lo

    def consume(self, pod_key: str) -> None:
        self.plans.pop(pod_key, None)
        self.plugin._pending_by_key.pop(pod_key, None)

    # the pipelined bench deletes its pods right after scheduling them to free the ledger while
    # they still run on the executor, whose measured intervals own the timeline: it turns this off
    drop_on_delete = True

    def released(self, pod: Obj, how: str) -> None:
        """A placed pod left the plan's view.  how: "unreserve" (it never ran there), "delete"
        (deleted before finishing) or "terminal" (it ran; its container times measure its
        timeline entry).  Keeps phantom work out of the slot chains and stale predictions out
        of the completion feedback."""
        key = O.key(pod)
        if how != "terminal" and self.feedback is not None:
            self.feedback.forget(key)
        tl = self.timeline
        if tl is None:
            return
        if how == "unreserve" or (how == "delete" and self.drop_on_delete):
            tl.drop(key)
        elif how == "terminal":
            from .feedback import QUANTISED_MIN_SPAN_S, container_span
            span = container_span(pod, QUANTISED_MIN_SPAN_S)
            if span is not None:
                tl.measure_key(key, span[0] * 1e3, span[1] * 1e3)
            elif self.drop_on_delete:
                tl.drop(key)
