"""Per-GPU CU-slot timelines: which pods run on each slot, in order, and when they ran.

A fractional pod holds a CU slot (an aligned run of CU-slice units, plugins.gpu.devices).
When a slot's pods run back to back -- the bench's executor keeps a stream per slot and a
launch-ahead pipeline of epochs, and a node whose pods queue behind a slot's previous
occupant behaves the same -- a pod's co-runners are not only the pods placed with it but
whatever the OTHER slots run during its lifetime: the tails of earlier placements and the
heads of later ones.  Scoring a placement against the pods "resident" at that moment (the
reference's model, pkg/plugins/gpu_plugin/gpu_plugins.go:558-757) then mispredicts exactly
the overlap that decides its SLO.

`SlotTimeline` keeps, per co-run group (a physical GPU, or one partition of it), each slot's
chain of placed pods.  Measured intervals (the executor's per-pod start / end) pin pods that
already ran; the unmeasured ones are chained: each starts when its slot predecessor ends.
`context()` turns a group's timeline into the arrays of the native pipeline simulation
(`_core.chain_times` / `_core.plan_slots`, native/core/corun.cpp), which the burst planner
uses to choose the slot of every new pod (plugins.gpu.planner).
"""
from __future__ import annotations

import threading
from typing import Any, Dict, Hashable, List, Optional, Sequence, Tuple

import numpy as np

NEG = -1e300
Slot = Tuple[int, int]          # (first unit, units)


class _Entry:
    __slots__ = ("key", "wid", "iters", "slo", "burst", "start", "end")

    def __init__(self, key: str, wid: int, iters: float, slo: float, burst: int):
        self.key, self.wid, self.iters, self.slo, self.burst = key, wid, iters, slo, burst
        self.start: Optional[float] = None
        self.end: Optional[float] = None


class SlotTimeline:
    """Slot chains per co-run group.  `depth` bounds how many unmeasured pods a chain keeps
    (without measurements -- no executor feedback -- older ones are taken as finished)."""

    def __init__(self, depth: int = 4, phantoms: int = 3):
        self.depth = depth
        self.phantoms = phantoms
        self._g: Dict[Hashable, Dict[Slot, List[_Entry]]] = {}
        self._lock = threading.Lock()
        self.burst = 0
        self.measured = 0
        self.unmatched = 0
        self._ver = 0                   # bumped by every change: context() results are memoised on it
        self._ctx_memo: Dict[Any, Dict[str, Any]] = {}

    # ------------------------------------------------------------------ updates
    def next_burst(self) -> int:
        self.burst += 1
        return self.burst

    def place(self, group: Hashable, slot: Slot, key: str, wid: int, iters: float, slo: float) -> None:
        """A pod was placed on `slot` of `group` (after every pod placed there before)."""
        self._ver += 1
        with self._lock:
            chain = self._g.setdefault(group, {}).setdefault(tuple(slot), [])
            chain.append(_Entry(key, int(wid), float(iters), float(slo), self.burst))
            unmeasured = [e for e in chain if e.end is None]
            while len(unmeasured) > self.depth:
                chain.remove(unmeasured.pop(0))

    def measure(self, group: Hashable, first_unit: int, start: float, end: float) -> bool:
        """The oldest unmeasured pod on the slot starting at `first_unit` ran [start, end)
        (times on the group's executor clock; a slot's pods run in placement order)."""
        self._ver += 1
        with self._lock:
            slots = self._g.get(group)
            if not slots:
                self.unmatched += 1
                return False
            for slot, chain in slots.items():
                if slot[0] != first_unit:
                    continue
                for e in chain:
                    if e.end is None:
                        e.start, e.end = float(start), float(end)
                        self.measured += 1
                        return True
            self.unmatched += 1
            return False

    def drop(self, key: str) -> bool:
        """Remove a pod that will not run on its slot (unreserved, or deleted before it ran):
        left in its chain it would be simulated as phantom work forever."""
        self._ver += 1
        with self._lock:
            for slots in self._g.values():
                for chain in slots.values():
                    for i, e in enumerate(chain):
                        if e.key == key:
                            del chain[i]
                            return True
        return False

    def measure_key(self, key: str, start: float, end: float) -> bool:
        """A pod identified by key ran [start, end) (a cluster's producer: the pod's container
        startedAt / finishedAt on the wall clock, instead of the executor's per-slot order)."""
        self._ver += 1
        with self._lock:
            for slots in self._g.values():
                for chain in slots.values():
                    for e in chain:
                        if e.key == key:
                            e.start, e.end = float(start), float(end)
                            self.measured += 1
                            return True
        return False

    def realign(self) -> None:
        """Every group drained (e.g. a pipelined job synchronised its GPUs): only each group's
        latest burst -- placed, not run yet -- remains, starting from an idle GPU."""
        self._ver += 1
        with self._lock:
            for g, slots in self._g.items():
                last = max((e.burst for ch in slots.values() for e in ch), default=None)
                for s in list(slots):
                    keep = [e for e in slots[s] if e.burst == last]
                    for e in keep:
                        e.start = e.end = None
                    slots[s] = keep

    def forget(self, group: Hashable) -> None:
        self._ver += 1
        with self._lock:
            self._g.pop(group, None)

    # ------------------------------------------------------------------ queries
    def chains(self, group: Hashable) -> Dict[Slot, List[Tuple[str, Optional[float], Optional[float]]]]:
        with self._lock:
            return {s: [(e.key, e.start, e.end) for e in ch] for s, ch in self._g.get(group, {}).items()}

    def context(self, group: Hashable, slots: Sequence[Slot]) -> Dict[str, Any]:
        """Memoised `_context` (the planner asks twice per burst and GPU: for plan_corun's
        pipeline evaluation and for the slot plan)."""
        key = (group, tuple(tuple(x) for x in slots), self._ver)
        hit = self._ctx_memo.get(key)
        if hit is None:
            if len(self._ctx_memo) > 256:
                self._ctx_memo.clear()
            hit = self._ctx_memo[key] = self._context(group, slots)
        return hit

    def _context(self, group: Hashable, slots: Sequence[Slot]) -> Dict[str, Any]:
        """The group's pipeline as plan_slots arrays: pinned measured pods that overlap the
        unmeasured ones, then every slot's unmeasured pods chained; slot_tail / slot_free for
        the candidate `slots`.  Times are relative to the group's clock: measured ends where
        there are any, else 0 (nothing ran yet)."""
        with self._lock:
            chains = {s: list(ch) for s, ch in self._g.get(group, {}).items()}
        last_end: Dict[Slot, float] = {}
        for s, ch in chains.items():
            ends = [e.end for e in ch if e.end is not None]
            if ends:
                last_end[s] = ends[-1]
        # a slot with no measured pod yet starts from the earliest point the group is known at
        origin = min(last_end.values()) if last_end else 0.0
        head: Dict[Slot, float] = {s: last_end.get(s, origin) for s in set(chains) | set(map(tuple, slots))}
        open_: Dict[Slot, List[_Entry]] = {s: [e for e in ch if e.end is None] for s, ch in chains.items()}
        starts = [head[s] for s, es in open_.items() if es]
        t_lo = min(starts) if starts else (min(head.values()) if head else 0.0)
        wid: List[int] = []
        it: List[float] = []
        st: List[float] = []
        prev: List[int] = []
        pin: List[float] = []
        slo: List[float] = []
        keys: List[str] = []
        # measured pods still running after the first unmeasured one starts: pinned co-runners
        with self._lock:
            for s, ch in chains.items():
                for e in ch:
                    if e.end is not None and e.end > t_lo and e.start is not None:
                        wid.append(e.wid), it.append(e.iters), st.append(e.start), prev.append(-1)
                        pin.append(e.end), slo.append(e.slo), keys.append(e.key)
            # prune: measured pods that ended before the window, except each slot's last one
            for s, ch in self._g.get(group, {}).items():
                lm = max((i for i, e in enumerate(ch) if e.end is not None), default=-1)
                ch[:] = [e for i, e in enumerate(ch) if e.end is None or i == lm or e.end > t_lo]
        tail: Dict[Slot, int] = {}
        for s, es in open_.items():
            p = -1
            for j, e in enumerate(es):
                wid.append(e.wid), it.append(e.iters), slo.append(e.slo), keys.append(e.key), pin.append(0.0)
                if j == 0:
                    st.append(head[s]), prev.append(-1)
                else:
                    st.append(NEG), prev.append(p)
                p = len(wid) - 1
            if p >= 0:
                tail[s] = p
        cand = [tuple(s) for s in slots]
        # phantom continuation per candidate slot: its own most recent pods, newest first
        # (the pods placed after this burst co-run with its tails; native plan_slots)
        recent_all = [e for ch in chains.values() for e in ch[-self.phantoms:]]
        ph_off, ph_wid, ph_it = [0], [], []
        for sl_ in cand:
            hist = list(reversed(chains.get(sl_, [])[-self.phantoms:])) or list(reversed(recent_all))
            for j in range(self.phantoms if hist else 0):
                e = hist[j % len(hist)]
                ph_wid.append(e.wid)
                ph_it.append(e.iters)
            ph_off.append(len(ph_wid))
        return {"ph_off": np.asarray(ph_off, np.int64), "ph_wid": np.asarray(ph_wid, np.int32),
                "ph_iters": np.asarray(ph_it, np.float64),"wid": np.asarray(wid, np.int32), "iters": np.asarray(it, np.float64),
                "start": np.asarray(st, np.float64), "prev": np.asarray(prev, np.int32),
                "pin": np.asarray(pin, np.float64), "slo": np.asarray(slo, np.float64), "keys": keys,
                "slot_tail": np.asarray([tail.get(s, -1) for s in cand], np.int32),
                "slot_free": np.asarray([head.get(s, origin) for s in cand], np.float64),
                "slots": cand}

    def pipeline(self, group: Hashable, slots: Sequence[Slot], model: Any, core: Any, with_phantoms: bool = False
                 ) -> Tuple[np.ndarray, ...]:
        """The group's in-flight pods as pinned co-runners for the burst planner: (workload
        ids, start, end) -- measured intervals, and predicted ones (the chained pipeline
        simulated with `model`) for pods that have not run yet -- restricted to what is still
        running once the first candidate slot frees; and the candidate `slots`' free times,
        ascending (native plan_corun's `pipe`)."""
        ctx = self.context(group, slots)
        k = len(ctx["wid"])
        # with_phantoms: per free slot (in free-time order) the first phantom of that slot --
        # the workload its stream most likely runs next (its own most recent one), which the
        # planner chains after the slot's new pod: a long pod co-runs with the NEXT epoch's
        # pods too, and without them its predicted co-runners thin out and it looks safe
        po = ctx["ph_off"]
        has = po[1:] > po[:-1]
        first = np.minimum(po[:-1], max(len(ctx["ph_wid"]) - 1, 0))
        ph_w = np.where(has, ctx["ph_wid"][first] if len(ctx["ph_wid"]) else -1, -1).astype(np.int32)
        ph_i = np.where(has, ctx["ph_iters"][first] if len(ctx["ph_iters"]) else 0.0, 0.0)
        if k == 0:
            order = np.argsort(ctx["slot_free"], kind="stable")
            free = ctx["slot_free"][order]
            out = (np.zeros(0, np.int32), np.zeros(0), np.zeros(0), free)
            return out + ((ph_w[order], ph_i[order]) if with_phantoms else ())
        st, fin = core.chain_times(ctx["wid"], ctx["iters"], ctx["start"], ctx["prev"], model.alone_ms,
                                   model.coupling(), ctx["pin"])
        tail = ctx["slot_tail"]
        free = np.where(tail >= 0, fin[np.maximum(tail, 0)], ctx["slot_free"])
        order = np.argsort(free, kind="stable")
        free = free[order]
        t0 = float(free[0]) if len(free) else 0.0
        keep = (fin > t0) & (fin < 1e299) & (st < 1e299)
        out = (ctx["wid"][keep], st[keep], fin[keep], free)
        return out + ((ph_w[order], ph_i[order]) if with_phantoms else ())
