"""CPU stand-in for the bench's GPU pipeline, driven by the co-run model ("model pipeline").

`parallel.executor.DeviceExecutor` runs each CU slot's pods back to back on the slot's stream;
the bench keeps `lookahead` epochs in flight, so a pod's co-runners are whatever the other
slots run meanwhile -- pods of its own epoch and of the neighbouring ones.  This executor
reproduces that on the CPU: every launched pod is appended to its slot's chain with a release
time (the simulated host clock when it was enqueued), and `wait_epoch` advances the simulated
GPU with the multi-way co-run model (native `chain_times`: the fluid model with chained slot
starts) until the epoch's pods have finished.  Pods that finished by then are final and stay
pinned to their interval; pods still running are re-simulated when later pods join, which is
exact because no later pod can start before the epoch finished (the host enqueues them after).

The "truth" can differ from the scheduler's model: per-pod lognormal noise on the work
(`noise` sigma, drawn once per pod) and a perturbed coupling matrix (`perturb` sigma on the
log of u and v), so a policy tuned on the model is judged against something it does not know.
Times are on a simulated clock (ms); `elapsed_ms` is the simulated wall time.

Used by `bench.py --sim --sim-model` and tests; the co-run model it simulates is
models.corun (data/corun_mi355x.json, fitted on MI355X measurements).
"""
from __future__ import annotations

from typing import Any, Dict, List, Optional, Tuple

import numpy as np

from ..models import workloads as W

NEG = -1e300


class _Ev:
    """A simulated HIP event: a time on the executor's clock."""
    __slots__ = ("t",)

    def __init__(self, t: float = 0.0):
        self.t = t

    def elapsed_time(self, other: "_Ev") -> float:
        return other.t - self.t

    def query(self) -> bool:
        return True


class ModelPipelineExecutor:
    def __init__(self, model: Any = None, noise: float = 0.05, perturb: float = 0.0, seed: int = 0,
                 host_ms: float = 0.05):
        from ..models.corun import CorunModel, _native_core
        base = model or CorunModel.load() or CorunModel.prior()
        rng = np.random.default_rng(seed + 7919)
        if perturb > 0:
            base = base.copy_with(base.u * np.exp(rng.normal(0, perturb, base.u.shape)),
                                  base.v * np.exp(rng.normal(0, perturb, base.v.shape)), f"{base.version}+perturbed")
        self.truth = base
        self.core = _native_core()
        if self.core is None or not hasattr(self.core, "chain_times"):
            raise RuntimeError("model pipeline needs the native core (_core.chain_times)")
        self.noise, self.rng, self.host_ms = noise, rng, host_ms
        self.now = 0.0                           # simulated host clock (ms), shared by every GPU
        self.clock = _Ev(0.0)                     # reference event of the executor clock
        self.gpus: Dict[int, _Gpu] = {}           # one pipeline per GPU (PodRun.gpu, default 0)
        self.flops_done = 0.0
        self.bytes_done = 0.0
        self.pending: List[Any] = []
        self.balance_slots = False                # the executor-side LPT slot balancing (A/B)
        self._slot_work: Dict[int, Dict[Tuple[int, int], float]] = {}

    # -- the DeviceExecutor surface the bench uses
    def warm(self, runs) -> None:
        pass

    def _gpu(self, r) -> "_Gpu":
        g = int(getattr(r, "gpu", 0))
        st = self.gpus.get(g)
        if st is None:
            st = self.gpus[g] = _Gpu(self)
        return st

    def launch_epoch(self, runs) -> None:
        if self.balance_slots:
            from .executor import lpt_balance
            by: Dict[int, List[Any]] = {}
            for r in runs:
                by.setdefault(int(getattr(r, "gpu", 0)), []).append(r)
            for g, rs in by.items():
                lpt_balance(rs, self._slot_work.setdefault(g, {}))
        for r in runs:
            mult = float(np.exp(self.rng.normal(0.0, self.noise))) if self.noise > 0 else 1.0
            self._gpu(r).launch(r, self.truth.wid(r.workload), r.iters * mult, self.now + self.host_ms)
            r.start, r.end = _Ev(), _Ev()
            w = W.CATALOG[r.workload]
            self.flops_done += w.flops * r.iters
            self.bytes_done += w.bytes * r.iters
        self.pending = runs

    def wait_epoch(self, runs) -> None:
        """Every GPU runs until its pods of this epoch finished; the host (which waits for all
        of them, as the ranks meet at the next placement broadcast) continues at the last."""
        if not runs:
            return
        by: Dict[int, List[Any]] = {}
        for r in runs:
            by.setdefault(int(getattr(r, "gpu", 0)), []).append(r)
        t = max(self.gpus[g].wait(rs) for g, rs in by.items())
        for r in runs:
            p = self._gpu(r).pods[r._sim_idx]
            r.start.t, r.end.t = p[4], p[5]
            r.ms = p[5] - p[4]
        self.now = max(self.now, t) + self.host_ms

    def wait_all(self) -> None:
        for g in self.gpus.values():
            g.simulate()

    def collect(self, runs) -> Dict[str, float]:
        busy = sum(r.ms * r.n_units for r in runs)
        ok = sum(1 for r in runs if r.slo <= 0 or r.throughput >= r.slo)
        if runs:
            span = max(r.end.t for r in runs) - min(r.start.t for r in runs)
        else:
            span = 0.0
        return {"pods": float(len(runs)), "busy_unit_ms": busy, "span_ms": span, "slo_ok": float(ok)}

    @property
    def elapsed_ms(self) -> float:
        return self.now

    def close(self) -> None:
        pass


class _Gpu:
    """One GPU's slot pipelines."""

    def __init__(self, ex: ModelPipelineExecutor):
        self.ex = ex
        # per pod: [wid, work iters, release, prev pod index or -1, start, fin, final]
        self.pods: List[List[Any]] = []
        self.slot_last: Dict[int, int] = {}       # unit -> index of the last pod that used it
        self._first_open = 0                      # pods before this index are all final

    def launch(self, r, wid: int, work_iters: float, release: float) -> None:
        prev = -1
        for u in range(r.first_unit, r.first_unit + r.n_units):
            j = self.slot_last.get(u, -1)
            if j > prev:
                prev = j
        idx = len(self.pods)
        self.pods.append([wid, work_iters, release, prev, None, None, False])
        for u in range(r.first_unit, r.first_unit + r.n_units):
            self.slot_last[u] = idx
        r._sim_idx = idx

    def simulate(self) -> None:
        """Re-simulate every non-final pod (final pods overlapping them are pinned)."""
        open_ = [i for i in range(self._first_open, len(self.pods)) if not self.pods[i][6]]
        if not open_:
            return
        def earliest(i: int) -> float:
            p = self.pods[i]
            q = p[3]
            if q >= 0 and not self.pods[q][6]:
                return float("inf")           # chained behind an open pod: starts later
            return max(p[2], self.pods[q][5] if q >= 0 else NEG)
        t_lo = min(earliest(i) for i in open_)
        pinned = [i for i in range(self._first_open, len(self.pods))
                  if self.pods[i][6] and self.pods[i][5] > t_lo]
        members = pinned + open_
        pos = {i: k for k, i in enumerate(members)}
        k = len(members)
        if k > 64:
            raise RuntimeError("model pipeline: more than 64 pods in flight on one GPU")
        wid = np.empty(k, np.int32)
        it = np.empty(k)
        st = np.empty(k)
        prev = np.full(k, -1, np.int32)
        pin = np.zeros(k)
        for m, i in enumerate(members):
            p = self.pods[i]
            wid[m], it[m] = p[0], p[1]
            if p[6]:                            # final: pinned to its interval
                st[m], pin[m] = p[4], p[5]
            elif p[3] >= 0 and p[3] in pos and not self.pods[p[3]][6]:
                prev[m], st[m] = pos[p[3]], p[2]        # chained behind an open pod (release)
            else:
                pf = self.pods[p[3]][5] if p[3] >= 0 else NEG
                st[m] = max(p[2], pf)
        s, f = self.ex.core.chain_times(wid, it, st, prev, self.ex.truth.alone_ms, self.ex.truth.coupling(), pin)
        for m, i in enumerate(members):
            if not self.pods[i][6]:
                self.pods[i][4], self.pods[i][5] = float(s[m]), float(f[m])

    def wait(self, runs) -> float:
        """Simulate until this GPU's pods of `runs` finished; returns when the last did."""
        self.simulate()
        t = max(self.pods[r._sim_idx][5] for r in runs)
        for p in self.pods[self._first_open:]:
            if p[5] is not None and p[5] <= t + 1e-9:
                p[6] = True
        while self._first_open < len(self.pods) and self.pods[self._first_open][6]:
            # keep final pods that still overlap open ones (pinned co-runners)
            if any(not q[6] and q[4] is not None and q[4] < self.pods[self._first_open][5]
                   for q in self.pods[self._first_open + 1:]):
                break
            self._first_open += 1
        return t
