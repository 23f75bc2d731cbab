"""Per-GPU pod executor ("kubelet + container runtime" of the bench and e2e tests).

One process per GPU.  The executor receives the scheduler's placements for its device
(pod id, workload, CU-slice unit range, iterations), runs each pod's kernel mix on a HIP
stream whose CU mask is exactly the pod's CU slices (ops.cumask.MaskedStream), and measures
per-pod device time with HIP events.  Pods are ordered on the device per CU-slice unit
(a pod waits for the previous occupant of each of its units), so the scheduler's
capacity model (a unit is free when its previous pod finishes) holds without host
synchronisation: the host can schedule epoch t+1 while the GPU executes epoch t.

Working buffers are allocated once per (workload, slot) and reused -- a warm container.
"""
from __future__ import annotations

import os
import time
from dataclasses import dataclass
from typing import Dict, List, Optional, Tuple

import torch

from ..models.workloads import Op, Workload, get as workload_by_name
from ..ops import loadgen
from ..plugins.gpu.devices import CUS_PER_XCD as CUS_PER_UNIT, cu_slice_mask


@dataclass
class PodRun:
    pod_id: int
    workload: str
    first_unit: int
    n_units: int
    iters: int
    slo: float = 0.0
    masked: bool = True          # Guaranteed QoS: hard CU mask; Burstable: accounted share only
    start: Optional[torch.cuda.Event] = None
    end: Optional[torch.cuda.Event] = None
    ms: float = 0.0
    gpu: int = 0                 # the node's GPU index (simulated executors keep one pipeline per GPU)
    policy: int = 0              # kernel policy from the scheduler: 1 = wide GEMM tiles (whole-chip budget)

    @property
    def throughput(self) -> float:
        return self.iters / (self.ms / 1e3) if self.ms > 0 else 0.0


class _Buffers:
    def __init__(self, w: Workload, device: torch.device):
        self.ops: List[Tuple[Op, tuple]] = []
        g = torch.Generator(device="cpu").manual_seed(hash(w.name) & 0xFFFF)
        for o in w.ops:
            if o.is_gemm:
                a = ((torch.rand(o.M, o.K, generator=g) * 2 - 1).to(torch.bfloat16)).to(device)
                bt = ((torch.rand(o.N, o.K, generator=g) * 2 - 1).to(torch.bfloat16) * 0.05).to(device)
                if o.kind == "gemm8":                   # e4m3 operands (weights scaled into range)
                    a, bt = a.to(loadgen.FP8), (bt * 16).to(loadgen.FP8)
                bias = torch.zeros(o.N, dtype=torch.float32, device=device)
                c = torch.empty(o.M, o.N, dtype=torch.bfloat16, device=device)
                self.ops.append((o, (a, bt, bias, c)))
            else:
                x = torch.ones(o.n_floats, dtype=torch.float32, device=device)
                y = torch.ones(o.n_floats, dtype=torch.float32, device=device)
                z = torch.ones(o.n_floats, dtype=torch.float32, device=device)
                self.ops.append((o, (x, y, z)))


def enqueue_ops(bufs: _Buffers, iters: int, st, budget: int, blocks: int = 0) -> None:
    """`iters` iterations of a workload's op list on stream `st` (GEMM tiles sized for `budget`
    CUs, 0 = the whole chip)."""
    for _ in range(iters):
        for o, t in bufs.ops:
            if o.kind == "gemm":
                a, bt, bias, c = t
                loadgen.gemm(a, bt, out=c, bias=bias, relu=o.relu, stream=st, cu_budget=budget)
            elif o.kind == "gemm8":
                a, bt, bias, c = t
                loadgen.gemm_fp8(a, bt, out=c, bias=bias, relu=o.relu, stream=st, cu_budget=budget)
            else:
                x, y, z = t
                loadgen.triad(x, y, z, 1.0001, blocks=blocks, stream=st)


def lpt_balance(runs: List[PodRun], slot_work: Dict[Tuple[int, int], float], work=None) -> None:
    """Reassign the slots of each group of same-size Burstable pods of this epoch: longest pod
    first onto the slot with the least cumulative work (ties: the lower slot).  `slot_work`
    ((first unit, units) -> cumulative work) is the caller's running state."""
    work = work or DeviceExecutor.pod_work
    groups: Dict[int, List[PodRun]] = {}
    for r in runs:
        if not r.masked:
            groups.setdefault(r.n_units, []).append(r)
    for n, rs in groups.items():
        if len(rs) < 2:
            continue
        slots = sorted(r.first_unit for r in rs)
        if len(set(slots)) != len(slots):
            continue
        for r in sorted(rs, key=work, reverse=True):
            u = min(slots, key=lambda s: (slot_work.get((s, n), 0.0), s))
            slots.remove(u)
            r.first_unit = u
            slot_work[(u, n)] = slot_work.get((u, n), 0.0) + work(r)


class DeviceExecutor:
    # co-run launch policy (tools/pod_mix.py measures these on the catalog mix):
    #   gemm_share   -- tell the GEMM tile picker the pod's CU share instead of the chip
    #   triad_blocks -- workgroups per stream-kernel launch (0 = the kernel's default)
    #   (capping the stream kernels at k workgroups per CU of the pod's share was measured and
    #   dropped: 380 / 509 / 550 pods/s at k = 1 / 2 / 4 vs 586 uncapped, profiles/archive/r03_triad_cap_ab.json)
    gemm_share = True
    triad_blocks = 0
    #   use_graphs   -- replay each pod's whole kernel sequence (iters x ops) as one captured
    #                   HIP graph on the pod's stream (captured once per workload/slot)
    use_graphs = False
    #   balance_slots -- (off by default; an A/B arm) re-slot each epoch's same-size Burstable
    #                   pods longest first onto the slot stream with the least cumulative work
    #                   (LPT).  It was round 3's default: +1.5 % pods/s over the scheduler's
    #                   first-fit slots, but blind to SLOs (-9 points of SLO attainment).  The
    #                   scheduler now chooses each pod's slot itself on its model of the slot
    #                   pipelines (plugins.gpu.timeline, --plan-slots), and the executor runs
    #                   every pod on the slot it was given (MI355X, 20 steps x 3 interleaved:
    #                   603.5 pods/s / 56.25 % SLOs vs 600.7 / 53.75 % for LPT re-slotting,
    #                   gpurun_out r04_slots_ab20 -> profiles/archive/r04_slots_ab/)
    balance_slots = os.environ.get("GPUSCHED_BALANCE_SLOTS", "0") == "1"

    def __init__(self, device: int = 0, use_cu_masks: bool = True, units_per_gpu: int = 8):
        self.device = device
        self.dev = torch.device("cuda", device)
        self.use_cu_masks = use_cu_masks
        self.units = units_per_gpu
        self._streams: Dict[Tuple[int, int], object] = {}
        self._bufs: Dict[Tuple[str, int, int], _Buffers] = {}
        self._last_events: List[torch.cuda.Event] = []
        self._unit_last: Dict[int, Tuple[Tuple[int, int], torch.cuda.Event]] = {}
        # (workload, units, iterations) of every pod launched, per epoch -- not the PodRuns: those
        # hold two HIP events each, and a long run would keep every one of them alive
        self.epoch_pods: List[List[Tuple[str, int, int]]] = []
        self._graphs: Dict[Tuple, "torch.cuda.CUDAGraph"] = {}
        self.lazy_captures = 0           # graphs captured by launch_epoch (not warm()): outside pod timing
        self.flops_done = 0.0
        self.bytes_done = 0.0
        self._slot_work: Dict[Tuple[int, int], float] = {}     # (first unit, units) -> cumulative work
        # the executor's clock: pod start / end events are reported as ms after this event
        # (the co-run learner rebuilds which pods of neighbouring epochs overlapped)
        self.clock = torch.cuda.Event(enable_timing=True)
        self.clock.record(torch.cuda.current_stream(self.device))

    def stream_for(self, first_unit: int, n_units: int, masked: bool = True):
        key = (first_unit, n_units, masked)
        st = self._streams.get(key)
        if st is None:
            if self.use_cu_masks and masked:
                from ..ops.cumask import MaskedStream
                st = MaskedStream(cu_slice_mask(first_unit, n_units), self.device)
            else:
                st = _PlainStream(self.device)
            self._streams[key] = st
        return st

    # one buffer set per workload instead of per (workload, slot): ~1/4 of the HBM, for
    # multi-rank rehearsals that map every rank onto one GPU (GPUSCHED_FORCE_DEVICE);
    # co-running pods of one workload then share operands (load generation only)
    shared_buffers = os.environ.get("GPUSCHED_SHARED_BUFFERS", "") == "1"

    def buffers(self, w: Workload, first_unit: int, n_units: int) -> _Buffers:
        k = (w.name, 0, 0) if self.shared_buffers else (w.name, first_unit, n_units)
        b = self._bufs.get(k)
        if b is None:
            b = _Buffers(w, self.dev)
            self._bufs[k] = b
        return b

    def warm(self, placements: List[PodRun]) -> None:
        """Pre-create streams/buffers -- and, with use_graphs, capture the pods' graphs --
        outside any timed region."""
        for p in placements:
            st = self.stream_for(p.first_unit, p.n_units, p.masked)
            bufs = self.buffers(workload_by_name(p.workload), p.first_unit, p.n_units)
            if self.use_graphs:
                self._graph_for(p, bufs, st.stream, self._budget(p))
        torch.cuda.synchronize(self.device)

    def _budget(self, r: PodRun) -> int:
        if r.policy == 1:
            return 0                     # wide: tiles for the whole chip (more, smaller workgroups)
        return r.n_units * CUS_PER_UNIT if self.gemm_share else 0   # the pod's CU share

    def _enqueue_ops(self, r: PodRun, bufs: "_Buffers", st, budget: int) -> None:
        enqueue_ops(bufs, r.iters, st, budget, self.triad_blocks)

    def _graph_for(self, r: PodRun, bufs: "_Buffers", st, budget: int) -> "torch.cuda.CUDAGraph":
        """One HIP graph per (workload, unit slot, QoS, iters): captured on the pod's own
        stream, so replaying it there keeps the stream's CU mask and its ordering."""
        k = (r.workload, r.first_unit, r.n_units, r.masked, r.iters, budget, self.triad_blocks)
        g = self._graphs.get(k)
        if g is None:
            torch.cuda.synchronize(self.device)
            g = torch.cuda.CUDAGraph()
            with torch.cuda.graph(g, stream=st):
                self._enqueue_ops(r, bufs, st, budget)
            torch.cuda.synchronize(self.device)
            self._graphs[k] = g
        return g

    def launch_epoch(self, runs: List[PodRun]) -> None:
        """Enqueue one epoch's pods; returns immediately (async).

        Ordering is per CU-slice unit, not per epoch: a pod waits (device-side) only for
        the last pod that occupied any of ITS units on another stream; pods reusing the
        same unit range share a stream and are ordered by it.  So a slot whose pod
        finished early starts its next pod at once instead of idling until the slowest
        pod of the epoch completes (work-conserving), while two pods never overlap on the
        same CUs -- exactly the ledger's capacity model."""
        if self.balance_slots:
            self._balance(runs)
        # buffers, streams and (with use_graphs) graphs of every pod are made BEFORE any pod's
        # start event is recorded: a lazy capture synchronises the device and captures on the
        # host, and inside a pod's [start, end) it would be measured as that pod's run time --
        # an outlier the planner's feedback would read as a slow GPU (GPUTEST_r04.json)
        prep = []
        for r in runs:
            w = workload_by_name(r.workload)
            bufs = self.buffers(w, r.first_unit, r.n_units)
            budget = self._budget(r)
            st = self.stream_for(r.first_unit, r.n_units, r.masked).stream
            g = None
            if self.use_graphs:
                n0 = len(self._graphs)
                g = self._graph_for(r, bufs, st, budget)
                self.lazy_captures += len(self._graphs) - n0
            prep.append((w, bufs, budget, g))
        for r, (w, bufs, budget, g) in zip(runs, prep):
            key = (r.first_unit, r.n_units, r.masked)
            r.start = torch.cuda.Event(enable_timing=True)
            r.end = torch.cuda.Event(enable_timing=True)
            st = self.stream_for(*key).stream
            waited = set()
            for u in range(r.first_unit, r.first_unit + r.n_units):
                last = self._unit_last.get(u)
                if last is not None and last[0] != key and id(last[1]) not in waited:
                    # a stream-wait is a barrier packet pending on this pod's queue until the
                    # previous occupant ends -- it slows the queue sharing its hardware pipe
                    # (see wait_all); skip it when that pod has already finished
                    if not last[1].query():
                        st.wait_event(last[1])
                    waited.add(id(last[1]))
            r.start.record(st)
            if g is not None:
                with torch.cuda.stream(st):
                    g.replay()
            else:
                self._enqueue_ops(r, bufs, st, budget)
            r.end.record(st)
            for u in range(r.first_unit, r.first_unit + r.n_units):
                self._unit_last[u] = (key, r.end)
            self.flops_done += w.flops * r.iters
            self.bytes_done += w.bytes * r.iters
        self._last_events = [ev for _, ev in {id(e): (k, e) for k, e in self._unit_last.values()}.values()]
        self.epoch_pods.append([(r.workload, r.n_units, r.iters) for r in runs])

    @staticmethod
    def pod_work(r: PodRun) -> float:
        """Relative work of a pod (its kernels' roofline time alone on the GPU x iterations)."""
        from ..models.workloads import roofline_seconds
        return roofline_seconds(workload_by_name(r.workload), 1.0) * max(r.iters, 1)

    def _balance(self, runs: List[PodRun]) -> None:
        lpt_balance(runs, self._slot_work, self.pod_work)

    # host poll period while waiting for an epoch's end events
    poll_s = 20e-6

    def wait_epoch(self, runs: List[PodRun]) -> None:
        """Host-wait until every pod of an epoch finished (its end events), by polling the
        events (wakes within tens of microseconds; never a stream-wait, see wait_all)."""
        for r in runs:
            ev = r.end
            if ev is None:
                continue
            while not ev.query():
                time.sleep(self.poll_s)

    def wait_all(self) -> None:
        """Host-wait until every enqueued pod finished, by polling their end events.

        Never by making another stream wait on them: a stream-wait leaves a barrier packet
        pending on that stream's hardware queue for as long as the pods run, and the queue of
        the pod stream sharing its hardware pipe is then served at about half rate -- with
        the default stream joined on 4 co-running pods, the 4th pod stream took 6.0 ms instead
        of 3.5 and the group 6.2 ms instead of 3.7 (profiles/archive/r03_queue_fairness/README.md)."""
        for ev in self._last_events:
            while not ev.query():
                time.sleep(self.poll_s)

    def collect(self, runs: List[PodRun]) -> Dict[str, float]:
        """After a sync: per-pod times + busy accounting for one epoch."""
        busy_unit_ms = 0.0
        t_first, t_last = None, None
        slo_ok = 0
        for r in runs:
            r.ms = r.start.elapsed_time(r.end)
            busy_unit_ms += r.ms * r.n_units
            if r.slo <= 0 or r.throughput >= r.slo:
                slo_ok += 1
        if runs:
            starts = [r.start for r in runs]
            ends = [r.end for r in runs]
            t0 = starts[0]
            t_first = min(t0.elapsed_time(s) for s in starts)
            t_last = max(t0.elapsed_time(e) for e in ends)
        span = (t_last - t_first) if runs else 0.0
        return {"pods": float(len(runs)), "busy_unit_ms": busy_unit_ms, "span_ms": span,
                "slo_ok": float(slo_ok)}

    def close(self) -> None:
        torch.cuda.synchronize(self.device)
        self._graphs.clear()
        for s in self._streams.values():
            s.close()
        self._streams.clear()


class _PlainStream:
    def __init__(self, device: int):
        self.stream = torch.cuda.Stream(device=device)

    def close(self) -> None:
        pass
