"""The node agent's background fabric probes: per-pair xGMI copy rates and RCCL bus-bandwidth
checks of the GPU sets multi-GPU pods were placed on.

Both probes need idle GPUs and take seconds (a child process opens a GPU context on every
device it measures), so they run on their own thread, never inside the agent's step: its
inventory publishing, HBM checks and profile ingestion keep their period.  Each probe

  1. starts only when the GPUs it measures are idle (no process in amd-smi's list, no
     non-terminal pod bound to them);
  2. taints the node `amd.com/fabric-probe=NoSchedule` while it runs, so no pod binds to the
     GPUs mid-probe and shares them with 256 MiB peer-copy buffers or RCCL rings;
  3. re-checks idleness afterwards and throws the result away if anything started meanwhile
     (a pod that ignored the taint, a process outside Kubernetes): a contended measurement
     would mark a healthy link degraded.

Set checks close SURVEY §5.8 item 4 as far as one node allows: the topology Filter picks an
xGMI clique from the pairwise copy rates (plugins.gpu.topology.select_gpu_set), and once a
multi-GPU pod has run on a set, the agent validates THAT set with RCCL all-reduce
(parallel.rccl_probe, one rank per GPU, in a child process when the pod has finished).  A set
whose bus bandwidth falls below `frac` x the median of this node's sets of the same size (or
below an absolute per-link floor) is published as bad (`bad_sets` in
`gpusched:topology:<node>`), and select_gpu_set ranks every candidate containing it after
the healthy ones.

The reference has no multi-GPU pods and no fabric view (reference
pkg/plugins/gpu_plugin/gpu_plugins.go:915 places one UUID per pod).
"""
from __future__ import annotations

import json
import logging
import os
import subprocess
import sys
import threading
import time
from typing import Any, Callable, Dict, List, Optional, Sequence, Tuple

from ..api import constants as C
from ..api import objects as O

log = logging.getLogger(__name__)

GpuSet = Tuple[int, ...]


def set_probe_in_child(gpus: Sequence[int], mib: int = 64, iters: int = 10, timeout_s: float = 180.0,
                       env: Optional[Dict[str, str]] = None) -> Optional[Dict[str, Any]]:
    """RCCL all-reduce over `gpus` (one rank per GPU, parallel.rccl_probe) in a child process
    that sees only those GPUs; the probe's JSON, or None on failure."""
    e = dict(os.environ if env is None else env)
    e["HIP_VISIBLE_DEVICES"] = ",".join(str(g) for g in gpus)
    e.setdefault("HSA_ENABLE_IPC_MODE_LEGACY", "0")
    e.setdefault("MASTER_ADDR", "127.0.0.1")
    cmd = [sys.executable, "-m", "k8s_gpu_scheduler_amd.parallel.rccl_probe", "--gpus", str(len(gpus)),
           "--sizes", f"{mib}M", "--iters", str(iters), "--ops", "all_reduce"]
    try:
        p = subprocess.run(cmd, capture_output=True, text=True, timeout=timeout_s, env=e)
    except (OSError, subprocess.TimeoutExpired) as ex:
        log.warning("RCCL set probe %s failed to run: %s", list(gpus), ex)
        return None
    if p.returncode != 0:
        log.warning("RCCL set probe %s exited %d: %s", list(gpus), p.returncode, p.stderr[-500:])
        return None
    for line in reversed(p.stdout.strip().splitlines()):
        if line.startswith("{"):
            try:
                return json.loads(line)
            except ValueError:
                break
    log.warning("RCCL set probe %s: no JSON in its output", list(gpus))
    return None


def busbw_of(res: Optional[Dict[str, Any]]) -> Optional[float]:
    """Largest all-reduce bus bandwidth (GB/s) of a probe result."""
    if not res:
        return None
    vals = [float(r["busbw_gbps"]) for r in res.get("results", []) if r.get("op") == "all_reduce"]
    return max(vals) if vals else None


class SetChecker:
    """Which GPU sets to validate, and the verdicts.

    frac: a set is bad below frac x the median bus bandwidth of this node's checked sets of
    the same size (once there are at least 3 of them); floor_link_gbps: and always below
    (k - 1) x this per-link rate (a k-GPU ring crosses k - 1 links per GPU; 20 GB/s is far
    below a healthy MI355X xGMI link, ~153 GB/s, and catches a link down to PCIe rates)."""

    # a probe that ran on idle GPUs but produced no result (child crash, RCCL hang until the
    # timeout, no JSON) is not retried at once: after the first failure the set waits
    # retry_s (doubling per failure); after max_failures it is published as bad -- a set on
    # which RCCL cannot complete an all-reduce is not a set to place a ring on
    def __init__(self, probe: Callable[[Sequence[int]], Optional[Dict[str, Any]]] = set_probe_in_child,
                 recheck_s: float = 3600.0, frac: float = 0.6, floor_link_gbps: float = 20.0, keep: int = 64,
                 clock: Callable[[], float] = time.time, retry_s: float = 300.0, max_failures: int = 2):
        self.probe = probe
        self.recheck_s = recheck_s
        self.retry_s = retry_s
        self.max_failures = max_failures
        self.failures: Dict[GpuSet, int] = {}
        self._retry_at: Dict[GpuSet, float] = {}
        self.frac = frac
        self.floor_link_gbps = floor_link_gbps
        self.keep = keep
        self.clock = clock
        self.results: Dict[GpuSet, Dict[str, Any]] = {}
        self._queue: List[GpuSet] = []
        self._lock = threading.Lock()

    def note(self, gpus: Sequence[int]) -> bool:
        """A multi-GPU pod was placed on `gpus`: queue the set unless checked recently."""
        s = tuple(sorted(int(g) for g in gpus))
        if len(s) < 2:
            return False
        with self._lock:
            r = self.results.get(s)
            if s in self._queue or (r is not None and self.clock() - r["ts"] < self.recheck_s):
                return False
            if self.clock() < self._retry_at.get(s, 0.0):
                return False
            self._queue.append(s)
            return True

    def pending(self) -> List[GpuSet]:
        with self._lock:
            return list(self._queue)

    def record(self, gpus: GpuSet, res: Optional[Dict[str, Any]]) -> Optional[Dict[str, Any]]:
        with self._lock:
            if gpus in self._queue:
                self._queue.remove(gpus)
            bw = busbw_of(res)
            if bw is None:
                return self._failed(gpus)
            self.failures.pop(gpus, None)
            self._retry_at.pop(gpus, None)
            self.results[gpus] = {"gpus": list(gpus), "busbw_gbps": round(bw, 1), "ts": self.clock()}
            if len(self.results) > self.keep:
                oldest = min(self.results, key=lambda s: self.results[s]["ts"])
                self.results.pop(oldest)
            self._judge()
            return dict(self.results.get(gpus, {})) or None

    def _failed(self, gpus: GpuSet) -> Optional[Dict[str, Any]]:
        """(lock held) A probe of `gpus` ran and failed: back off, or after max_failures
        publish the set as bad."""
        n = self.failures.get(gpus, 0) + 1
        self.failures[gpus] = n
        if n < self.max_failures:
            self._retry_at[gpus] = self.clock() + self.retry_s * 2 ** (n - 1)
            return None
        self._retry_at.pop(gpus, None)
        self.failures.pop(gpus, None)
        self.results[gpus] = {"gpus": list(gpus), "busbw_gbps": 0.0, "ts": self.clock(), "failed": True}
        self._judge()
        return dict(self.results[gpus])

    def _judge(self) -> None:
        """(Re)judge every set against its size's median: a set checked before its peers
        existed is re-judged as they arrive."""
        by_k: Dict[int, List[float]] = {}
        for s, r in self.results.items():
            if not r.get("failed"):
                by_k.setdefault(len(s), []).append(r["busbw_gbps"])
        for s, r in self.results.items():
            vals = sorted(by_k.get(len(s), []))
            med = vals[len(vals) // 2] if len(vals) >= 3 else None
            floor = (len(s) - 1) * self.floor_link_gbps
            r["floor_gbps"] = floor
            r["median_gbps"] = med
            r["ok"] = bool(not r.get("failed") and r["busbw_gbps"] >= floor and
                           (med is None or r["busbw_gbps"] >= self.frac * med))

    def bad_sets(self) -> List[List[int]]:
        with self._lock:
            return [list(s) for s, r in sorted(self.results.items()) if not r["ok"]]

    def to_json(self) -> List[Dict[str, Any]]:
        with self._lock:
            return [dict(r) for _, r in sorted(self.results.items())]


class ProbeWorker:
    """Runs the agent's fabric probe and set checks on a background thread (see module doc)."""

    def __init__(self, agent: Any, sets: Optional[SetChecker] = None, period_s: float = 5.0, taint: bool = True):
        self.agent = agent
        self.sets = sets
        self.period_s = period_s
        self.taint = taint
        self.discarded = 0
        self.ran: List[str] = []
        self.failed: List[str] = []
        self.retry_s = 300.0             # fabric probe back-off after a failed run (doubling)
        self._fabric_failures = 0
        self._fabric_retry_at = 0.0
        self._stop = threading.Event()
        self._thread: Optional[threading.Thread] = None

    # ---------------------------------------------------------------- idleness
    def _gpu_of_uuid(self) -> Dict[str, int]:
        return {d["uuid"]: int(d.get("gpu", i)) for i, d in enumerate(self.agent.source.devices())}

    def busy(self, gpus: Optional[Sequence[int]] = None) -> List[str]:
        """Why (some of) `gpus` are not idle (None = any GPU of the node)."""
        if gpus is None:
            return self.agent.busy_reasons()
        want = set(int(g) for g in gpus)
        out = []
        for i, d in enumerate(self.agent.source.devices()):
            if int(d.get("gpu", i)) not in want:
                continue
            for p in self.agent.source.processes(i):
                if not self.agent._is_own_process(int(p.get("pid", 0))):
                    out.append(f"gpu{d.get('gpu', i)}: pid {p.get('pid')}")
        client = self.agent.client
        if client is not None:
            try:
                pods, _ = client.list("pods", field_selector=f"spec.nodeName={self.agent.node}")
            except Exception as e:
                return out + [f"cannot list pods on the node: {e}"]
            g_of = self._gpu_of_uuid()
            for p in pods:
                if O.is_terminal(p):
                    continue
                devs = [u for u in (O.annotations(p).get(C.ANNOT_DEVICES) or "").split(",") if u]
                if any(g_of.get(u) in want for u in devs):
                    out.append(f"pod {O.key(p)}")
        return out

    # ---------------------------------------------------------------- pods -> sets
    def note_pods(self, pods: Optional[List[Dict[str, Any]]] = None) -> int:
        """Queue the GPU set of every multi-GPU pod bound to the node."""
        if self.sets is None or self.agent.client is None:
            return 0
        if pods is None:
            pods, _ = self.agent.client.list("pods", field_selector=f"spec.nodeName={self.agent.node}")
        g_of = self._gpu_of_uuid()
        n = 0
        for p in pods:
            devs = [u for u in (O.annotations(p).get(C.ANNOT_DEVICES) or "").split(",") if u]
            gpus = sorted({g_of[u] for u in devs if u in g_of})
            if len(gpus) >= 2 and self.sets.note(gpus):
                n += 1
        return n

    # ---------------------------------------------------------------- one probe
    DEFERRED, DISCARDED, RAN = "deferred", "discarded", "ran"

    def _exclusive(self, what: str, gpus: Optional[Sequence[int]], fn: Callable[[], Any]) -> Tuple[str, Any]:
        """(outcome, result): fn() with the node tainted, only from idle GPUs and only kept when
        they are still idle afterwards.  outcome: DEFERRED (busy before: not run), DISCARDED
        (busy afterwards: result thrown away, the probe is still due) or RAN (result = fn()'s,
        None when the probe itself failed)."""
        reasons = self.busy(gpus)
        if reasons:
            log.info("%s deferred: GPUs busy (%s)", what, "; ".join(reasons[:3]))
            return self.DEFERRED, None
        res_api = None
        if self.taint and self.agent.client is not None:
            from ..kube.resources import Resources
            res_api = Resources(self.agent.client, "default")
            try:
                res_api.taint_node(self.agent.node, C.TAINT_PROBING, what.split()[0], "NoSchedule")
            except Exception as e:
                log.warning("%s: tainting %s failed (%s): not probing", what, self.agent.node, e)
                return self.DEFERRED, None
        try:
            out = fn()
        finally:
            if res_api is not None:
                try:
                    res_api.untaint_node(self.agent.node, C.TAINT_PROBING)
                except Exception as e:
                    log.warning("%s: untainting %s failed: %s", what, self.agent.node, e)
        after = self.busy(gpus)
        if after:
            self.discarded += 1
            log.warning("%s: GPUs became busy during the probe (%s): result discarded", what, "; ".join(after[:3]))
            return self.DISCARDED, None
        self.ran.append(what)
        return self.RAN, out

    def tick(self) -> Optional[str]:
        """Run at most one due probe; returns what ran ('fabric' / 'set 0,1,2,3') or None."""
        ag = self.agent
        fab = getattr(ag, "fabric", None)
        if fab is not None and fab.due and time.time() >= self._fabric_retry_at:
            how, res = self._exclusive("fabric", None, fab.probe)
            if how != self.DEFERRED:
                if how == self.RAN:
                    # done either way: a failed probe (child crash / timeout / no JSON) must
                    # not re-taint the node and re-run every period_s forever -- it is retried
                    # after a doubling back-off (the last good topology stays published)
                    fab.due = False
                    if res is not None:
                        self._fabric_failures = 0
                        fab.last = res
                        from .fabric import degraded_pairs
                        bad = degraded_pairs(res.get("bw_gbps") or [])
                        if bad:
                            log.warning("fabric on %s: degraded GPU pairs %s", ag.node, bad)
                        ag.publish_topology()
                    else:
                        self._fabric_failures += 1
                        self.failed.append("fabric")
                        self._fabric_retry_at = time.time() + self.retry_s * 2 ** min(self._fabric_failures - 1, 6)
                        fab.due = True
                        log.warning("fabric probe on %s failed (%d in a row): retry in %.0f s", ag.node,
                                    self._fabric_failures, self._fabric_retry_at - time.time())
                return "fabric"
        if self.sets is not None:
            for s in self.sets.pending():
                how, res = self._exclusive(f"set {','.join(map(str, s))}", s, lambda s=s: self.sets.probe(s))
                if how == self.DEFERRED:
                    continue
                if how == self.RAN:
                    # a failed probe is recorded too (back-off, then a bad set): it leaves the queue
                    doc = self.sets.record(s, res)
                    if res is None:
                        self.failed.append(f"set {','.join(map(str, s))}")
                    if doc is not None and not doc["ok"]:
                        log.warning("RCCL set check on %s: GPUs %s at %.1f GB/s busbw%s: degraded", ag.node,
                                    doc["gpus"], doc["busbw_gbps"], " (probe failed)" if doc.get("failed") else "")
                    if doc is not None:
                        ag.publish_topology()
                return f"set {','.join(map(str, s))}"
        return None

    # ---------------------------------------------------------------- thread
    def run(self) -> None:
        while not self._stop.is_set():
            try:
                self.tick()
            except Exception as e:
                log.warning("background probe failed: %s", e)
            self._stop.wait(self.period_s)

    def start(self) -> "ProbeWorker":
        if self._thread is None:
            self._thread = threading.Thread(target=self.run, daemon=True, name="fabric-probes")
            self._thread.start()
        return self

    def stop(self) -> None:
        self._stop.set()
        if self._thread is not None:
            self._thread.join(timeout=5)
