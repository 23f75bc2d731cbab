"""Cross-cycle node-result cache: the scheduling cycle at cluster scale.

A cycle filters and scores every node for one pod.  For a node whose scheduling state did
not change since the previous cycle (framework.changes), and a pod that presents the same
*signature* to every enabled plugin, those results cannot differ -- the equivalence-class
idea of kube-scheduler's old equivalence cache, applied to the whole Filter+Score pipeline.
So per signature the cache keeps, for every node in snapshot order, its filter verdict and
each score plugin's raw score in flat arrays; a cycle re-runs the real plugins only on the
nodes touched since the entry's last cycle (normally just the node the previous pod went
to) and hands the arrays to the native core (`_core.select_nodes`, native/core/score.cpp),
which does the rotated, sampled feasible scan (numFeasibleNodesToFind), min-max
normalisation, weighting and the max-tie set in C++.  Python work per pod is O(changed
nodes), not O(nodes).

Results are identical to the node-at-a-time path (framework.runtime find_feasible +
run_score + Scheduler._select_host): the same plugins compute every cached value, the scan
order and the sample cut are the same, and ties are broken by the same RNG draw
(tests/test_fastpath.py runs both paths side by side).

A plugin takes part by implementing `cache_signature(state, pod, phase) -> hashable | None`
(phase "filter", "preScore" or "score"): everything its per-node result depends on besides
node-local state that reports to the change log; None (or no method) sends the cycle down
the ordinary path -- e.g. inter-pod affinity and topology spreading, whose verdicts depend
on other nodes' pods, or the GPU plugin's burst planner.
"""
from __future__ import annotations

import time
from collections import OrderedDict
from typing import Any, Dict, List, Optional, Tuple

import numpy as np

from .changes import ChangeLog
from .interface import CycleState, MAX_NODE_SCORE, MIN_NODE_SCORE, as_status

Obj = Dict[str, Any]


def _plugin_sigs(plugins, skip, state, pod, phase) -> Optional[tuple]:
    out = []
    for p in plugins:
        if p.name() in skip:
            continue
        f = getattr(p, "cache_signature", None)
        if f is None:
            return None
        s = f(state, pod, phase)
        if s is None:
            return None
        out.append((p.name(), s))
    return tuple(out)


def select_nodes_py(feasible: np.ndarray, raw: np.ndarray, norm: np.ndarray, weights: np.ndarray,
                    start: int, limit: int) -> tuple:
    """Pure-Python twin of `_core.select_nodes` (no native build)."""
    n = len(feasible)
    order = [(start + i) % n for i in range(n)] if n else []
    feas, unknown, processed = [], [], 0
    for i in order:
        processed += 1
        if feasible[i] < 0:
            unknown.append(i)
        elif feasible[i]:
            feas.append(i)
        if limit and len(feas) + len(unknown) >= limit:
            break
    e = np.asarray([], np.int32)
    if unknown:
        return processed, e, np.asarray([], np.int64), e, -1, np.asarray(unknown, np.int32)
    tot = [0] * len(feas)
    for p in range(raw.shape[0]):
        vals = [int(raw[p, i]) for i in feas]
        if norm[p] and vals:
            lo, hi = min(vals), max(vals)
            vals = [0 if hi == lo else ((v - lo) * 100) // (hi - lo) for v in vals]
        for k, v in enumerate(vals):
            if not (MIN_NODE_SCORE <= v <= MAX_NODE_SCORE):
                return processed, np.asarray(feas), np.asarray(tot), e, p, e
            tot[k] += v * int(weights[p])
    best = max(tot) if tot else 0
    ties = [k for k, t in enumerate(tot) if t == best] if tot else []
    return processed, np.asarray(feas, np.int32), np.asarray(tot, np.int64), np.asarray(ties, np.int32), -1, e


class _Entry:
    __slots__ = ("names", "feasible", "raw", "seq", "epoch", "snap")

    def __init__(self, names: List[str], n_score: int, seq: int, epoch: int):
        self.names = names
        self.feasible = np.full(len(names), -1, np.int8)       # -1 = not evaluated
        self.raw = np.zeros((n_score, len(names)), np.int64)
        self.seq = seq
        self.epoch = epoch
        self.snap = None


class NodeResultCache:
    """One per scheduling profile (Framework)."""
    MAX_ENTRIES = 32

    def __init__(self, fw: Any, log: ChangeLog):
        self.fw = fw
        self.log = log
        self._entries: "OrderedDict[tuple, _Entry]" = OrderedDict()
        self.stats = {"cycles": 0, "fallback": 0, "rescored": 0}
        try:
            from .. import _native
            core = _native.core()
            self._select = core.select_nodes if core is not None else select_nodes_py
        except Exception:
            self._select = select_nodes_py

    def cursor(self) -> Tuple[int, int]:
        """Read BEFORE the cycle's snapshot: every change after it is re-examined next cycle."""
        return self.log.seq, self.log.epoch

    def schedule(self, state: CycleState, pod: Obj, snapshot: Any, start: int, limit: int,
                 cursor: Tuple[int, int]) -> Optional[Tuple[str, int, int, Dict[str, int]]]:
        """(host, nodes processed, feasible count, total score per feasible node) or None
        when the cycle must take the ordinary path (a plugin without a cache signature, no
        feasible node -- the failure path wants per-node reasons --, or a plugin error)."""
        fw = self.fw
        nodes = snapshot.list()
        if not nodes:
            return None
        fsig = _plugin_sigs(fw.points["filter"], state.skip_filter_plugins, state, pod, "filter")
        if fsig is None:
            return self._fallback()
        seq, epoch = cursor
        st = fw.run_pre_score(state, pod, [])
        # a PreScore plugin that skipped itself contributes nothing to this cycle's scores
        if not st.ok or _plugin_sigs(fw.points["preScore"], state.skip_score_plugins, state, pod, "preScore") is None:
            return self._fallback()
        score_plugins = [p for p in fw.points["score"] if p.name() not in state.skip_score_plugins]
        ssig = _plugin_sigs(score_plugins, (), state, pod, "score")
        if ssig is None:
            return self._fallback()
        key = (fsig, ssig, tuple(sorted(state.skip_filter_plugins)), tuple(sorted(state.skip_score_plugins)))
        ent = self._entries.get(key)
        if ent is not None:
            self._entries.move_to_end(key)
        dirty: Optional[set] = None
        if ent is not None and ent.epoch == epoch and ent.snap is not None and len(ent.names) == len(nodes):
            dirty = self.log.since(ent.seq)
        if dirty is None:                       # new entry, compacted log or node set changed
            ent = _Entry([ni.name for ni in nodes], len(score_plugins), seq, epoch)
            self._entries[key] = ent
            while len(self._entries) > self.MAX_ENTRIES:
                self._entries.popitem(last=False)
        else:                                   # touched nodes: evaluate again when the scan needs them
            index = snapshot.index()
            for n in dirty:
                i = index.get(n)
                if i is not None:
                    ent.feasible[i] = -1
        ent.seq, ent.epoch, ent.snap = seq, epoch, snapshot
        self._find_ns = 0
        norm = []
        for p in score_plugins:
            ext = p.score_extensions()
            if ext is None:
                norm.append(0)
            elif getattr(ext, "NORMALIZE", None) == "minmax":
                norm.append(1)
            else:                               # a normalisation the native core does not know
                return self._fallback()
        norm = np.asarray(norm, np.int8)
        weights = np.asarray([fw.weights.get(p.name(), 1) for p in score_plugins], np.int64)
        t0 = time.perf_counter_ns()
        score_ns = 0
        while True:
            processed, feas, tot, ties, bad, unknown = self._select(ent.feasible, ent.raw, norm, weights, start, limit)
            if len(unknown) == 0:
                break
            # evaluate exactly the nodes the sampled scan reached (in scan order), then rescan
            if not self._recompute(state, pod, ent, nodes, unknown.tolist(), score_plugins):
                self._entries.pop(key, None)
                return self._fallback()
            self.stats["rescored"] += len(unknown)
            score_ns += self._score_ns
        self.stats["cycles"] += 1
        fw.metrics.add("score", time.perf_counter_ns() - t0 - self._find_ns + score_ns)
        if bad >= 0 or len(feas) == 0:
            self._entries.pop(key, None)
            return self._fallback()
        pick = int(ties[0]) if len(ties) == 1 else int(ties[self.fw_rng.randrange(len(ties))])
        names = ent.names
        scores = {names[i]: int(t) for i, t in zip(feas.tolist(), tot.tolist())}
        state.write("framework/nodes-processed", int(processed))
        return names[int(feas[pick])], int(processed), len(feas), scores

    fw_rng: Any = None      # the scheduler's RNG (set by Scheduler): same draws as _select_host
    _score_ns = 0
    _find_ns = 0

    def _fallback(self):
        self.stats["fallback"] += 1
        return None

    def _recompute(self, state: CycleState, pod: Obj, ent: _Entry, nodes: List[Any], idx: List[int],
                   score_plugins: List[Any]) -> bool:
        """Re-run the real Filter and Score plugins on the nodes at `idx`."""
        fw = self.fw
        self._score_ns = 0
        infos = [nodes[i] for i in idx]
        t0 = time.perf_counter_ns()
        feasible, _ = fw.find_feasible(state, pod, infos, 0)
        self._find_ns += time.perf_counter_ns() - t0
        ok = {ni.name for ni in feasible}
        fe = ent.feasible
        for i, ni in zip(idx, infos):
            fe[i] = 1 if ni.name in ok else 0
        if not feasible:
            return True
        fidx = [i for i, ni in zip(idx, infos) if ni.name in ok]
        names = [ni.name for ni in feasible]
        t0 = time.perf_counter_ns()
        for k, p in enumerate(score_plugins):
            batch = getattr(p, "score_nodes", None)
            if batch is not None and not getattr(p, "SCORE_DOES_IO", False):
                vals, st = batch(state, pod, names)
                if st is not None and not st.ok:
                    return False
            else:
                vals = []
                for nn in names:
                    v, st = p.score(state, pod, nn)
                    if not as_status(st).ok:
                        return False
                    vals.append(int(v))
            ent.raw[k, fidx] = np.asarray(vals, np.int64)
        self._score_ns = time.perf_counter_ns() - t0
        return True
