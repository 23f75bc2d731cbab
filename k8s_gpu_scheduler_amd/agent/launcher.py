"""Pod launcher: a minimal kubelet for one node.

The reference relies on the real kubelet to read the pod's envFrom ConfigMaps at container
creation (its PostBind writes CUDA_VISIBLE_DEVICES there, reference
pkg/plugins/gpu_plugin/gpu_plugins.go:910-920) and on the NVIDIA runtime to expose the
device.  This launcher plays both roles for tests, the fake cluster and bare-metal runs: it
picks up pods bound to its node, builds the container environment the way the kubelet does
(container `env`, then `envFrom` ConfigMaps, then the device plugin's allocation, which here
is the scheduler's assignment annotations: devices -> ROCR_VISIBLE_DEVICES, cu-mask ->
HSA_CU_MASK) and runs the container command as a child process, then reports the pod phase
(Succeeded / Failed) through the API.

The default command is `agent.container_probe`, which prints what the process sees of the
GPU (visible devices, CUs its kernels ran on): SURVEY §7.4's "the pod saw exactly the one
assigned device".
"""
from __future__ import annotations

import json
import logging
import os
import subprocess
import sys
import time
from dataclasses import dataclass, field
from typing import Callable, Dict, List, Optional

from ..api import constants as C
from ..api import objects as O
from ..kube.client import KubeClient, NotFound

log = logging.getLogger(__name__)
Obj = Dict[str, object]

DEFAULT_COMMAND = [sys.executable, "-m", "k8s_gpu_scheduler_amd.agent.container_probe"]
# environment of the launcher that a container must not inherit (it would override or
# contradict the pod's device assignment)
_SCRUB = (C.ENV_ROCR_VISIBLE, C.ENV_HIP_VISIBLE, C.ENV_CU_MASK, C.ENV_CUDA_VISIBLE, "GPU_DEVICE_ORDINAL",
          "OMPI_COMM_WORLD_LOCAL_RANK", "LOCAL_RANK", "RANK", "WORLD_SIZE")


@dataclass
class LaunchResult:
    pod_key: str
    rc: int
    stdout: str = ""
    stderr: str = ""
    env: Dict[str, str] = field(default_factory=dict)

    def json(self) -> Optional[dict]:
        for line in reversed(self.stdout.strip().splitlines()):
            try:
                return json.loads(line)
            except json.JSONDecodeError:
                continue
        return None


_VAR = None


def _rfc3339(t: float) -> str:
    """The kubelet's container timestamp format: UTC, whole seconds."""
    return time.strftime("%Y-%m-%dT%H:%M:%SZ", time.gmtime(t))


def _expand(s: str, env: Dict[str, str]) -> str:
    """Kubernetes' $(VAR) expansion (an undefined reference stays as written, $$ escapes)."""
    global _VAR
    if "$(" not in s and "$$" not in s:
        return s
    if _VAR is None:
        import re
        _VAR = re.compile(r"\$\$|\$\(([A-Za-z_][A-Za-z0-9_.-]*)\)")
    return _VAR.sub(lambda m: "$" if m.group(0) == "$$" else env.get(m.group(1), m.group(0)), s)


def _field_ref(pod: Obj, path: str) -> Optional[str]:
    """Downward API fieldRef values a kubelet resolves for env."""
    if path == "metadata.name":
        return O.name(pod)
    if path == "metadata.namespace":
        return O.namespace(pod)
    if path == "metadata.uid":
        return O.uid(pod)
    if path == "spec.nodeName":
        return O.node_name_of(pod) or ""
    if path.startswith("metadata.annotations['") or path.startswith("metadata.labels['"):
        key = path.split("['", 1)[1].rstrip("']")
        return (O.annotations(pod) if path.startswith("metadata.annotations") else O.labels(pod)).get(key, "")
    return None


class PodLauncher:
    def __init__(self, client: KubeClient, node_name: str, command: Optional[List[str]] = None,
                 timeout_s: float = 120.0, base_env: Optional[Dict[str, str]] = None,
                 command_for: Optional[Callable[[Obj], List[str]]] = None):
        self.client = client
        self.node = node_name
        self.command = command or DEFAULT_COMMAND
        self.command_for = command_for
        self.timeout_s = timeout_s
        base = dict(os.environ if base_env is None else base_env)
        for k in _SCRUB:
            base.pop(k, None)
        self.base_env = base
        self.launched: Dict[str, LaunchResult] = {}
        self.cwd: Optional[str] = None              # container working directory (None = ours)
        self.extra_env: Dict[str, str] = {}         # runtime-injected env (not the pod's)
        self.running: Dict[int, str] = {}           # pid of a running container -> pod UID

    # ------------------------------------------------------------------ env
    def env_for(self, pod: Obj) -> Dict[str, str]:
        """Container env, kubelet order: env entries, then envFrom ConfigMaps (a key from env
        wins), then the device allocation from the assignment annotations."""
        ns = O.namespace(pod)
        env: Dict[str, str] = {}
        ctr = O.containers(pod)[0] if O.containers(pod) else {}
        from_cms: Dict[str, str] = {}
        for ref in ctr.get("envFrom") or []:
            name = (ref.get("configMapRef") or {}).get("name")
            if not name:
                continue
            try:
                cm = self.client.get("configmaps", name, ns)
            except NotFound:
                if (ref.get("configMapRef") or {}).get("optional"):
                    continue
                raise
            from_cms.update({k: str(v) for k, v in (cm.get("data") or {}).items()})
        env.update(from_cms)
        for e in ctr.get("env") or []:
            if "value" in e:
                env[e["name"]] = _expand(str(e["value"]), env)
            elif "valueFrom" in e:
                v = _field_ref(pod, ((e.get("valueFrom") or {}).get("fieldRef") or {}).get("fieldPath", ""))
                if v is not None:
                    env[e["name"]] = v
        ann = O.annotations(pod)
        devices = ann.get(C.ANNOT_DEVICES, "")
        if devices:
            uuids = [u for u in devices.split(",") if u]
            env.setdefault(C.ENV_ROCR_VISIBLE, ",".join(uuids))
            env.setdefault(C.ENV_HIP_VISIBLE, ",".join(str(i) for i in range(len(uuids))))
            if ann.get(C.ANNOT_CU_MASK):
                env.setdefault(C.ENV_CU_MASK, ann[C.ANNOT_CU_MASK])
        return env

    # ------------------------------------------------------------------ run
    def run(self, pod: Obj) -> LaunchResult:
        key = O.key(pod)
        env = self.env_for(pod)
        ctr = O.containers(pod)[0] if O.containers(pod) else {}
        argv = (self.command_for(pod) if self.command_for else None) or \
            (list(ctr.get("command") or []) + list(ctr.get("args") or [])) or self.command
        # kubelet: $(VAR) in command/args expands from the container env; a process runtime
        # has no mount namespace, so hostPath volumeMounts become path rewrites
        mounts = self.host_mounts(pod, ctr, env)
        argv = [self._remap(_expand(a, env), mounts) for a in argv]
        for mp, hp in mounts.items():
            os.makedirs(self.host_root + hp, exist_ok=True)     # hostPath type DirectoryOrCreate
        full_env = dict(self.base_env)
        full_env.update(self.extra_env)
        full_env.update(env)
        started = time.time()
        try:
            proc = subprocess.Popen(argv, env=full_env, stdout=subprocess.PIPE, stderr=subprocess.PIPE, text=True,
                                    cwd=self.cwd)
        except OSError as e:
            res = LaunchResult(key, 127, "", str(e), env)
        else:
            # the running container's pid -> pod UID (what a cgroup lookup gives a node agent)
            self.running[proc.pid] = O.uid(pod)
            try:
                out, err = proc.communicate(timeout=self.timeout_s)
                res = LaunchResult(key, proc.returncode, out, err, env)
            except subprocess.TimeoutExpired:
                proc.kill()
                out, err = proc.communicate()
                res = LaunchResult(key, -9, out or "", (err or "") + "\ntimeout", env)
            finally:
                self.running.pop(proc.pid, None)
        self.launched[key] = res
        phase = "Succeeded" if res.rc == 0 else "Failed"
        # as the kubelet reports it: RFC 3339 at whole seconds
        term = {"exitCode": res.rc, "startedAt": _rfc3339(started), "finishedAt": _rfc3339(time.time())}
        status = {"phase": phase, "containerStatuses": [{"name": (O.containers(pod) or [{}])[0].get("name", "main"),
                                                         "state": {"terminated": term}}]}
        try:
            self.client.patch("pods", O.name(pod), {"status": status}, "merge", O.namespace(pod))
        except NotFound:
            pass
        return res

    @staticmethod
    def host_mounts(pod: Obj, ctr: Obj, env: Optional[Dict[str, str]] = None) -> Dict[str, str]:
        """mountPath -> hostPath of the container's hostPath volume mounts (with its subPath,
        or its subPathExpr expanded from the container env, as the kubelet does; a sub-path
        that is absolute or climbs out with `..` is refused, as the kubelet refuses it)."""
        vols = {v.get("name"): (v.get("hostPath") or {}).get("path") for v in (pod.get("spec") or {}).get("volumes") or []}
        out = {}
        for m in ctr.get("volumeMounts") or []:
            hp = vols.get(m.get("name"))
            if not hp or not m.get("mountPath"):
                continue
            sub = m.get("subPath") or (_expand(m["subPathExpr"], env or {}) if m.get("subPathExpr") else "")
            if sub:
                if sub.startswith("/") or ".." in sub.split("/") or "$(" in sub:
                    raise ValueError(f"volumeMount {m.get('name')}: bad sub-path {sub!r}")
                hp = hp.rstrip("/") + "/" + sub
            out[m["mountPath"].rstrip("/")] = hp
        return out

    def _remap(self, arg: str, mounts: Dict[str, str]) -> str:
        for mp, hp in sorted(mounts.items(), key=lambda kv: -len(kv[0])):
            if arg == mp or arg.startswith(mp + "/"):
                return self.host_root + hp + arg[len(mp):]
        return arg

    host_root = ""      # prefix for hostPath volumes (tests point it at a scratch directory)

    def run_bound(self) -> List[LaunchResult]:
        """Launch every pod bound to this node that has not run yet (one pass)."""
        pods, _ = self.client.list("pods", field_selector=f"spec.nodeName={self.node}")
        out = []
        for pod in pods:
            if O.key(pod) in self.launched or O.is_terminal(pod):
                continue
            out.append(self.run(pod))
        return out
