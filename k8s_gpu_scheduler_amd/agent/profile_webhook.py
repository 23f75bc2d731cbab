"""Per-pod rocprofv3 profiling for kubelet-started containers: a mutating admission webhook.

The reference's profiler DaemonSet only enumerates device UUIDs (reference
pkg/profiler/profile_gpu.sh:3-13, deploy/profiler/client-daemonset.yaml:1-38); its per-GPU
metrics sampler exists but is never called (pkg/profiler/parse_smi_metrics.py:23-42).  The
MI355X build's north star wants kernel-level history per workload, so that the resize
recommender sizes requests from what pods actually ran.  A DaemonSet cannot wrap a container
the kubelet starts, but admission can rewrite what the kubelet will start:

  pod CREATE (label gpu-scheduler.amd.com/profile=trace) --> ProfileInjector.patch_ops:
    every container with an explicit `command` runs as
      rocprofv3 --kernel-trace --stats --output-format csv -o run -- <command> <args>
                -d /gpusched-prof/<tag>
    (the program directly after `--`: no shell, no env hop -- the profiler's preloaded
    library must see the real program); the hostPath volume (/var/lib/gpusched/prof) is
    mounted with `subPathExpr: <ns>/<pod>/<uid>/<container>` (namespace, name and UID from
    the downward API: a controller's pod may get its generated name after admission), so a
    container sees only its own directory -- it cannot read, overwrite or forge another pod's
    profiles; <tag> records the request the pod was admitted with (CU share, HBM, iterations:
    `cu64-hbm8-it20`), so the agent can attribute a profile even after the pod object is gone
    (a pod deleted after it ran is ingested under its name's workload within the ingestor's
    orphan grace period, pod_profiler.ProfileIngestor);
  the container exits --> rocprofv3 writes run_kernel_stats.csv / run_kernel_trace.csv
    into the hostPath --> the node agent (pod_profiler.ProfileIngestor, NodeAgent.step)
    summarises each finished directory into the pod's WORKLOAD history in Redis
    (`gpusched:hist:<workload>`), which the resize admission reads.

A container without `command` (image ENTRYPOINT) is left alone -- its argv is not in the pod
spec -- unless the pod names it in the annotation `gpu-scheduler.amd.com/profile-argv`
(JSON list).  PMC counters are never combined with trace domains (the pool's rule and
rocprofv3's own limits): `profile=pmc` with `gpu-scheduler.amd.com/profile-counters`
(comma separated) runs a counter pass instead of a trace.
"""
from __future__ import annotations

import json
import logging
from typing import Any, Dict, List, Optional, Tuple

from ..api import constants as C
from ..api import objects as O

log = logging.getLogger(__name__)
Obj = Dict[str, Any]

LABEL_PROFILE = C.ANNOT_PREFIX + "profile"           # label (objectSelector) and annotation: trace | pmc
ANNOT_PROFILE_ARGV = C.ANNOT_PREFIX + "profile-argv"
ANNOT_PROFILE_COUNTERS = C.ANNOT_PREFIX + "profile-counters"
ANNOT_PROFILED = C.ANNOT_PREFIX + "profiled"         # set by the webhook: containers wrapped
HOST_DIR = "/var/lib/gpusched/prof"
MOUNT = "/gpusched-prof"
VOLUME = "gpusched-prof"
UID_ENV = "GPUSCHED_POD_UID"
NAME_ENV = "GPUSCHED_POD_NAME"
NS_ENV = "GPUSCHED_POD_NAMESPACE"


def request_tag(pod: Obj) -> str:
    """`cu<CUs>-hbm<GiB>-it<iterations>` of the pod as admitted (whole GPUs count 256 CUs each)."""
    g, cu, mem = O.gpu_request(pod, cached=False)
    cus = cu or g * C.MI355X_CUS
    return f"cu{int(cus)}-hbm{mem:g}-it{O.pod_iterations(pod):g}"


def parse_tag(tag: str) -> Dict[str, float]:
    out: Dict[str, float] = {}
    for part in tag.split("-"):
        for key, pre in (("cu", "cu"), ("hbm_gib", "hbm"), ("iters", "it")):
            if part.startswith(pre):
                try:
                    out[key] = float(part[len(pre):])
                except ValueError:
                    pass
                break
    return out


DEFAULT_COUNTERS = ("SQ_WAVES", "SQ_BUSY_CU_CYCLES", "SQ_INSTS_VALU_MFMA_MOPS_BF16")


def profile_mode(pod: Obj) -> Optional[str]:
    v = O.labels(pod).get(LABEL_PROFILE) or O.annotations(pod).get(LABEL_PROFILE) or ""
    v = v.strip().lower()
    return v if v in ("trace", "pmc") else None


def wrap_argv(argv: List[str], out_dir: str, mode: str = "trace", counters: Optional[List[str]] = None,
              rocprof: str = "rocprofv3") -> List[str]:
    """rocprofv3 command line around a container argv (program directly after `--`)."""
    prof = [rocprof, "--output-format", "csv", "-d", out_dir, "-o", "run"]
    prof += ["--kernel-trace", "--stats"] if mode == "trace" else ["--pmc", *(counters or DEFAULT_COUNTERS)]
    return prof + ["--"] + list(argv)


class ProfileInjector:
    def __init__(self, rocprof: str = "rocprofv3", host_dir: str = HOST_DIR):
        self.rocprof = rocprof
        self.host_dir = host_dir
        self.stats = {"seen": 0, "wrapped": 0, "skipped_no_command": 0}

    def patch_ops(self, pod: Obj) -> Tuple[List[Dict[str, Any]], Optional[Dict[str, Any]]]:
        """JSONPatch ops wrapping the opted-in pod's containers (empty = leave the pod)."""
        self.stats["seen"] += 1
        mode = profile_mode(pod)
        if mode is None or O.annotations(pod).get(ANNOT_PROFILED):
            return [], None
        ann = O.annotations(pod)
        explicit: Optional[List[str]] = None
        if ann.get(ANNOT_PROFILE_ARGV):
            try:
                explicit = [str(x) for x in json.loads(ann[ANNOT_PROFILE_ARGV])]
            except (ValueError, TypeError):
                log.warning("%s: bad %s annotation", O.key(pod), ANNOT_PROFILE_ARGV)
        counters = [c.strip() for c in ann.get(ANNOT_PROFILE_COUNTERS, "").split(",") if c.strip()] or None
        spec = pod.get("spec") or {}
        ops: List[Dict[str, Any]] = []
        wrapped: List[str] = []
        tag = request_tag(pod)
        for i, ctr in enumerate(spec.get("containers") or []):
            cmd = list(ctr.get("command") or [])
            if not cmd and explicit and i == 0:
                cmd = explicit                      # the full argv: the image's args go too
                if ctr.get("args"):
                    ops.append({"op": "remove", "path": f"/spec/containers/{i}/args"})
            elif not cmd:
                self.stats["skipped_no_command"] += 1
                continue
            name = ctr.get("name") or f"c{i}"
            out = f"{MOUNT}/{tag}"
            # the container args stay where they are: kubelet runs command + args, so the
            # original program and its arguments follow `--` unchanged
            ops.append({"op": "add", "path": f"/spec/containers/{i}/command",
                        "value": wrap_argv(cmd, out, mode, counters, self.rocprof)})
            if "env" not in ctr:
                ops.append({"op": "add", "path": f"/spec/containers/{i}/env", "value": []})
            for env, field in ((UID_ENV, "metadata.uid"), (NAME_ENV, "metadata.name"), (NS_ENV, "metadata.namespace")):
                ops.append({"op": "add", "path": f"/spec/containers/{i}/env/-", "value": {
                    "name": env, "valueFrom": {"fieldRef": {"fieldPath": field}}}})
            if "volumeMounts" not in ctr:
                ops.append({"op": "add", "path": f"/spec/containers/{i}/volumeMounts", "value": []})
            ops.append({"op": "add", "path": f"/spec/containers/{i}/volumeMounts/-",
                        "value": {"name": VOLUME, "mountPath": MOUNT,
                                  # only this container's own directory of the hostPath
                                  "subPathExpr": f"$({NS_ENV})/$({NAME_ENV})/$({UID_ENV})/{name}"}})
            wrapped.append(name)
        if not wrapped:
            return [], None
        if "volumes" not in spec:
            ops.append({"op": "add", "path": "/spec/volumes", "value": []})
        ops.append({"op": "add", "path": "/spec/volumes/-", "value": {
            "name": VOLUME, "hostPath": {"path": self.host_dir, "type": "DirectoryOrCreate"}}})
        if not ann:
            ops.append({"op": "add", "path": "/metadata/annotations", "value": {}})
        ops.append({"op": "add", "path": "/metadata/annotations/" + ANNOT_PROFILED.replace("/", "~1"),
                    "value": ",".join(wrapped)})
        self.stats["wrapped"] += 1
        return ops, {"mode": mode, "containers": wrapped, "tag": tag}

    def mutate(self, pod: Obj) -> Obj:
        """In-process admission (FakeCluster.add_admission): the mutated pod."""
        from ..kube.patch import apply_json_patch
        ops, _ = self.patch_ops(pod)
        return apply_json_patch(pod, ops) if ops else pod

    __call__ = mutate


class ChainAdmission:
    """Several mutating admissions behind one webhook endpoint: each sees the pod as the
    previous ones left it, and their JSONPatches are concatenated in order."""

    def __init__(self, *admissions: Any):
        self.admissions = [a for a in admissions if a is not None]

    def patch_ops(self, pod: Obj) -> Tuple[List[Dict[str, Any]], Any]:
        from ..kube.patch import apply_json_patch
        all_ops: List[Dict[str, Any]] = []
        infos = []
        cur = pod
        for a in self.admissions:
            ops, info = a.patch_ops(cur)
            if ops:
                cur = apply_json_patch(cur, ops)
                all_ops += ops
            infos.append(info)
        return all_ops, infos

    def mutate(self, pod: Obj) -> Obj:
        from ..kube.patch import apply_json_patch
        ops, _ = self.patch_ops(pod)
        if not ops:
            return pod
        O.forget_requests(pod)
        return apply_json_patch(pod, ops)

    __call__ = mutate
