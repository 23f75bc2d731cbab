"""Per-pod GPU profiling sidecar: rocprofv3 around the container, summary into Redis.

BASELINE's north star: "the profiler sidecar samples rocprof counters per pod into Redis
and the recommender resizes GPU requests from that history".  The reference's profiler only
enumerates UUIDs (pkg/profiler/profile_gpu.sh:3-13); its per-workload throughput matrices were
measured offline.  Here a launched pod (agent.launcher.PodLauncher) can run under

  rocprofv3 --kernel-trace --stats --output-format csv -d <dir> -o run -- <container argv>

(the program directly after `--`, no shell or env hop), or, in a separate mode, under
`rocprofv3 --pmc <counters>` (counters are never combined with trace domains).  The CSVs are
summarised -- GPU busy time, kernel count, the top kernels, busy fraction of the pod's wall
time, counter totals -- and appended to the pod's workload history
(`schema.history_key(<workload>)`), next to the CU share it ran on, which is exactly what
`recommender.resize.recommend` / the resize admission webhook read.
"""
from __future__ import annotations

import csv
import logging
import os
import shutil
import tempfile
import time
from typing import Any, Callable, Dict, List, Optional, Tuple

from ..api import constants as C
from ..api import objects as O
from ..recommender.admission import RedisHistory, workload_key
from .launcher import LaunchResult, PodLauncher

ROCPROF = shutil.which("rocprofv3") or "/opt/rocm/bin/rocprofv3"
log = logging.getLogger(__name__)


# kernel-name markers of matrix-core (MFMA) work: this framework's GEMMs (gs::gemm_*),
# hipBLASLt / Tensile (Cijk_*), rocBLAS, composable_kernel / MIOpen implicit-GEMM convolutions,
# flash attention
MFMA_KERNEL_MARKERS = ("gemm", "cijk_", "mfma", "matmul", "igemm", "conv", "fmha", "attn", "xdl", "wmma")


def is_mfma_kernel(name: str) -> bool:
    n = name.lower()
    return any(m in n for m in MFMA_KERNEL_MARKERS)


def summarize_kernel_stats(path: str, top: int = 5) -> Dict[str, Any]:
    """Busy time, calls, the top kernels and `mfma_share`: the fraction of kernel time in
    matrix-core kernels (by name) -- the resource shape the co-run model's cold start
    (models.coldstart) places an unseen workload by."""
    rows = list(csv.DictReader(open(path)))
    tot_ns = sum(float(r.get("TotalDurationNs", 0) or 0) for r in rows)
    mfma_ns = sum(float(r.get("TotalDurationNs", 0) or 0) for r in rows if is_mfma_kernel(r.get("Name", "")))
    calls = sum(int(float(r.get("Calls", 0) or 0)) for r in rows)
    rows.sort(key=lambda r: -float(r.get("TotalDurationNs", 0) or 0))
    out = {"gpu_busy_ms": tot_ns / 1e6, "kernels": calls,
           "top": [{"name": r["Name"][:120], "calls": int(float(r["Calls"])),
                    "ms": float(r["TotalDurationNs"]) / 1e6} for r in rows[:top]]}
    if tot_ns > 0:
        out["mfma_share"] = round(mfma_ns / tot_ns, 4)
    return out


def summarize_counters(path: str) -> Dict[str, float]:
    tot: Dict[str, float] = {}
    for r in csv.DictReader(open(path)):
        k = r.get("Counter_Name", "")
        tot[k] = tot.get(k, 0.0) + float(r.get("Counter_Value", 0) or 0)
    return tot


class ProfiledLauncher(PodLauncher):
    """PodLauncher whose containers run under rocprofv3; each finished pod appends one
    profile sample to its workload's history."""

    def __init__(self, *a: Any, history: Optional[RedisHistory] = None, mode: str = "trace",
                 counters: Optional[List[str]] = None, keep_dir: str = "", **kw: Any):
        super().__init__(*a, **kw)
        if mode not in ("trace", "pmc"):
            raise ValueError("mode must be 'trace' or 'pmc'")
        self.history = history
        self.mode = mode
        self.counters = counters or ["SQ_WAVES", "SQ_BUSY_CU_CYCLES", "SQ_INSTS_VALU_MFMA_MOPS_BF16"]
        self.keep_dir = keep_dir
        self.samples: Dict[str, Dict[str, Any]] = {}

    def run(self, pod: Dict[str, Any]) -> LaunchResult:
        work = tempfile.mkdtemp(prefix="podprof-", dir=os.environ.get("TMPDIR") or None)
        out_dir = os.path.join(work, "prof")
        inner = self.command_for

        def wrapped(p: Dict[str, Any]) -> List[str]:
            ctr = O.containers(p)[0] if O.containers(p) else {}
            argv = (inner(p) if inner else None) or \
                (list(ctr.get("command") or []) + list(ctr.get("args") or [])) or self.command
            prof = [ROCPROF, "--output-format", "csv", "-d", out_dir, "-o", "run"]
            prof += ["--kernel-trace", "--stats"] if self.mode == "trace" else ["--pmc", *self.counters]
            return prof + ["--"] + list(argv)
        self.command_for = wrapped
        # rocprofv3 keeps its scratch in the working directory and TMPDIR: both go to the
        # per-pod temp dir; the package stays importable through PYTHONPATH
        pkg_root = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
        old_cwd, old_env = self.cwd, dict(self.extra_env)
        self.cwd = work
        self.extra_env.update({"TMPDIR": work, "PYTHONPATH": os.pathsep.join(
            x for x in (pkg_root, self.base_env.get("PYTHONPATH", "")) if x)})
        t0 = time.time()
        try:
            res = super().run(pod)
        finally:
            self.command_for = inner
            self.cwd, self.extra_env = old_cwd, old_env
        wall = time.time() - t0
        sample: Dict[str, Any] = {"ts": t0, "wall_s": wall, "rc": res.rc}
        try:
            for root, _, files in os.walk(out_dir):
                for f in files:
                    if f.endswith("kernel_stats.csv"):
                        sample.update(summarize_kernel_stats(os.path.join(root, f)))
                    elif f.endswith("counter_collection.csv"):
                        sample["counters"] = summarize_counters(os.path.join(root, f))
            if "gpu_busy_ms" in sample:
                sample["busy_frac"] = min(1.0, sample["gpu_busy_ms"] / 1e3 / max(wall, 1e-9))
            g, cu, mem = O.gpu_request(pod)
            sample["cu"] = cu or (g * C.MI355X_CUS)
            if mem:
                sample["hbm_gib"] = mem
            self.samples[O.key(pod)] = sample
            if self.history is not None:
                self.history.append(workload_key(pod), sample)
        finally:
            if self.keep_dir:
                dst = os.path.join(self.keep_dir, O.name(pod))
                shutil.rmtree(dst, ignore_errors=True)
                if os.path.isdir(out_dir):
                    shutil.copytree(out_dir, dst)
            shutil.rmtree(work, ignore_errors=True)
        return res


def _workgroups(r: Dict[str, str]) -> Optional[int]:
    """Workgroups of one kernel-trace dispatch (rocprofv3 grid and workgroup sizes are in
    work-items per dimension); None when the row has no sizes."""
    n = 1
    for d in ("X", "Y", "Z"):
        g, w = r.get(f"Grid_Size_{d}"), r.get(f"Workgroup_Size_{d}")
        if g in (None, "") or w in (None, ""):
            if d == "X":
                return None
            continue
        g, w = int(float(g)), max(1, int(float(w)))
        n *= max(1, -(-g // w))
    return n


def summarize_kernel_trace(path: str, cus: int = C.MI355X_CUS) -> Dict[str, Any]:
    """Span (first kernel start .. last kernel end) and busy time (union of kernel intervals)
    of a rocprofv3 kernel_trace.csv, in ms; `cu_fill`: the kernel-time-weighted fraction of
    the chip's CUs the dispatches occupy (min(1, workgroups / CUs)) -- the co-run cold start's
    footprint feature (models.coldstart)."""
    iv = []
    fw = ft = 0.0
    for r in csv.DictReader(open(path)):
        try:
            a, b = int(r["Start_Timestamp"]), int(r["End_Timestamp"])
        except (KeyError, ValueError):
            continue
        iv.append((a, b))
        try:
            wg = _workgroups(r)
        except ValueError:
            wg = None
        if wg is not None and b > a:
            fw += (b - a) * min(1.0, wg / cus)
            ft += b - a
    if not iv:
        return {}
    iv.sort()
    first_ns, last_ns = iv[0][0], max(b for _, b in iv)
    busy, cs, ce = 0, iv[0][0], iv[0][1]
    for a, b in iv[1:]:
        if a > ce:
            busy += ce - cs
            cs, ce = a, b
        else:
            ce = max(ce, b)
    busy += ce - cs
    span = last_ns - first_ns
    out = {"span_ms": span / 1e6, "busy_union_ms": busy / 1e6, "first_ns": first_ns, "last_ns": last_ns}
    if ft > 0:
        out["cu_fill"] = round(fw / ft, 4)
    return out


class ProfileIngestor:
    """Node-agent side of the profiling webhook (agent.profile_webhook): every finished
    rocprofv3 output directory under the hostPath -- <root>/<ns>/<pod>/<uid>/<container>/<tag>
    -- becomes one sample of the pod's workload history (what the resize admission reads):
    GPU busy time, kernel count, top kernels, the kernel span and busy fraction, the CU share
    and HBM it was admitted with, and -- for a batch pod with ITERATIONS -- its throughput
    (iterations / GPU-busy time: the union of its kernel intervals, not the span -- rocprofv3's
    per-dispatch tracing adds host gaps between an eagerly launching pod's kernels that the
    unprofiled pod does not have).  A directory is finished when rocprofv3 has written its
    stats (kernel_stats.csv, or counter_collection.csv for a PMC pass); ingested ones are
    removed, so each run is counted once.

    `pod_lookup(ns, name)` (the agent's API client): a directory is ingested for a pod that
    exists with that UID on this node -- defence in depth behind the webhook's per-container
    subPathExpr mount; the pod's own workload annotation names the history it goes to.  A pod
    that no longer exists (deleted after it ran) keeps its run only if the agent saw that
    exact (namespace, name, UID) on this node (`note_pods`, fed by the agent's per-step pod
    list): its directory is then ingested under the name rule's workload while younger than
    `orphan_grace_s`; an unprovable orphan is dropped (a forged directory must not
    feed another workload's history).  Files over `max_file_bytes` are not read.  With a `corun` observer
    (agent.corun_observer.CorunObserver) each traced pod's kernel interval on its device is
    also recorded, so pods that overlapped on one GPU become co-run observations."""

    def __init__(self, root: str, history: RedisHistory, keep_dir: str = "",
                 pod_lookup: Optional[Callable[[str, str], Optional[Dict[str, Any]]]] = None,
                 node: str = "", corun: Any = None, max_file_bytes: int = 64 << 20,
                 orphan_grace_s: float = 3600.0):
        # a directory whose pod object is already gone (a Job pod garbage-collected or
        # TTL-deleted before this pass) is still that pod's: only its own container could write
        # there (the webhook's per-container subPathExpr mount names it by namespace, name and
        # UID).  It is ingested under the name rule's workload while younger than
        # orphan_grace_s; older orphans are dropped
        self.orphan_grace_s = orphan_grace_s
        self.root = root
        self.history = history
        self.keep_dir = keep_dir
        self.pod_lookup = pod_lookup
        self.node = node
        self.corun = corun
        self.max_file_bytes = max_file_bytes
        self.ingested: List[Dict[str, Any]] = []
        self.rejected: List[str] = []
        # uid -> (namespace, name, last seen) of pods the agent saw bound to this node
        self.seen: Dict[str, Tuple[str, str, float]] = {}
        # callback(uid, busy ms) for the agent's busy-ms annotation (agent.busy)
        self.on_busy: Optional[Callable[[str, float], None]] = None

    def note_pods(self, pods: List[Dict[str, Any]]) -> None:
        """The pods bound to this node right now (any phase): the UIDs an orphaned profile
        directory may belong to."""
        now = time.time()
        for p in pods:
            u = O.uid(p)
            if u:
                self.seen[u] = (O.namespace(p), O.name(p), now)
        if len(self.seen) > 65536:
            for u in [u for u, v in self.seen.items() if now - v[2] > self.orphan_grace_s]:
                self.seen.pop(u, None)

    def _finished(self) -> List[Tuple[str, List[str]]]:
        out = []
        if not os.path.isdir(self.root):
            return out
        for dirpath, _, files in os.walk(self.root):
            rel = os.path.relpath(dirpath, self.root).split(os.sep)
            if len(rel) != 5:
                continue
            if any(f.endswith("kernel_stats.csv") or f.endswith("counter_collection.csv") for f in files):
                out.append((dirpath, rel))
        return out

    def _owner(self, ns: str, name: str, uid: str, d: str = "") -> Tuple[bool, Optional[Dict[str, Any]]]:
        """(accept, pod object or None)."""
        if self.pod_lookup is None:
            return True, None
        try:
            pod = self.pod_lookup(ns, name)
        except Exception as e:          # apiserver blip: keep the directory for the next pass
            raise RuntimeError(f"pod lookup failed: {e}") from e
        if pod is None:                 # gone (deleted after it ran): an orphan within its grace
            try:
                age = time.time() - os.path.getmtime(d) if d else float("inf")
            except OSError:
                age = float("inf")
            known = self.seen.get(uid)
            provable = known is not None and known[:2] == (ns, name)
            return provable and age <= self.orphan_grace_s, None
        if O.uid(pod) != uid:           # a different pod of that name: never this directory's
            return False, None
        if self.node and O.node_name_of(pod) not in ("", self.node):
            return False, None
        return True, pod

    def _drop(self, d: str) -> None:
        shutil.rmtree(d, ignore_errors=True)
        # drop the now-empty parents (<uid>/<container>) so the tree does not grow
        for up in (os.path.dirname(d), os.path.dirname(os.path.dirname(d))):
            try:
                os.rmdir(up)
            except OSError:
                break

    def step(self) -> int:
        from .profile_webhook import parse_tag
        n = 0
        for d, (ns, name, uid, container, tag) in self._finished():
            try:
                ok, owner = self._owner(ns, name, uid, d)
            except RuntimeError as e:
                log.warning("profile %s: %s", d, e)
                continue
            if not ok:
                log.warning("profile %s: no pod %s/%s with uid %s on this node: dropped", d, ns, name, uid)
                self.rejected.append(d)
                self._drop(d)
                continue
            sample: Dict[str, Any] = {"ts": time.time(), "pod": f"{ns}/{name}", "uid": uid, "container": container,
                                      "source": "rocprof"}
            req = parse_tag(tag)
            for root, _, files in os.walk(d):
                for f in files:
                    p = os.path.join(root, f)
                    try:
                        if os.path.getsize(p) > self.max_file_bytes:
                            log.warning("profile %s: %s larger than %d bytes: skipped", d, f, self.max_file_bytes)
                            continue
                        if f.endswith("kernel_stats.csv"):
                            sample.update(summarize_kernel_stats(p))
                        elif f.endswith("kernel_trace.csv"):
                            sample.update(summarize_kernel_trace(p))
                        elif f.endswith("counter_collection.csv"):
                            sample["counters"] = summarize_counters(p)
                    except (OSError, csv.Error, KeyError, ValueError) as e:
                        log.warning("profile %s: %s unreadable: %s", d, f, e)
            if "cu" in req:
                sample["cu"] = int(req["cu"])
            if req.get("hbm_gib"):
                sample["hbm_gib"] = req["hbm_gib"]
            span = sample.get("span_ms")
            if span:
                sample["busy_frac"] = min(1.0, sample.get("busy_union_ms", 0.0) / span)
                sample["cu_busy"] = sample["busy_frac"]
                if req.get("iters"):
                    busy = sample.get("busy_union_ms") or span
                    sample["throughput"] = req["iters"] / (busy / 1e3)
            # the pod's own workload name (its annotation) when the object is known; the name
            # rule of recommender.admission.workload_key otherwise
            pod = owner or {"metadata": {"name": name, "namespace": ns, "annotations": {}}}
            wl = workload_key(pod)
            first, last = sample.pop("first_ns", None), sample.pop("last_ns", None)
            busy_ms = sample.get("busy_union_ms") or sample.get("gpu_busy_ms")
            if self.on_busy is not None and busy_ms:
                self.on_busy(uid, float(busy_ms))
            try:
                self.history.append(wl, sample)
            except Exception as e:          # Redis blip: keep the directory for the next pass
                log.warning("profile %s: history append failed: %s", d, e)
                continue
            if self.corun is not None and first is not None and last is not None and last > first:
                try:
                    self.corun.add(pod, wl, float(req.get("iters", 0.0)), int(first), int(last),
                                   mfma_share=sample.get("mfma_share"), cu_fill=sample.get("cu_fill"))
                except Exception as e:
                    log.warning("profile %s: co-run record failed: %s", d, e)
            self.ingested.append(sample)
            n += 1
            if self.keep_dir:
                dst = os.path.join(self.keep_dir, ns, name, uid, container)
                shutil.rmtree(dst, ignore_errors=True)
                shutil.copytree(d, dst)
            self._drop(d)
        return n
