"""One-process-per-GPU self-launcher (no torchrun needed).

`python bench.py --gpus N` (and `rccl_probe --gpus N`) without a torch.distributed
environment start N fresh worker processes here, one per GPU, each with
RANK / LOCAL_RANK / WORLD_SIZE / LOCAL_WORLD_SIZE / MASTER_ADDR / MASTER_PORT set exactly
as `torch.distributed.run --nnodes 1 --nproc-per-node N` would.  The parent never touches
the GPU: it only counts devices (`torch.cuda.device_count()` does not initialise HIP on
this image) and waits, so no GPU-initialised process ever execs, and a request for more
GPUs than the host has fails fast with a non-zero exit instead of silently measuring one.
If any rank fails, the others are stopped and the first failure's exit code is returned.
"""
from __future__ import annotations

import os
import signal
import socket
import subprocess
import sys
import time
from typing import Dict, List, Optional, Sequence


class LaunchError(RuntimeError):
    pass


def free_port(host: str = "127.0.0.1") -> int:
    s = socket.socket()
    s.bind((host, 0))
    p = s.getsockname()[1]
    s.close()
    return p


def visible_gpu_count() -> int:
    """GPUs this process could use, counted without initialising HIP."""
    try:
        import torch
        return int(torch.cuda.device_count())
    except Exception:
        return 0


def in_distributed_env(env: Optional[Dict[str, str]] = None) -> bool:
    env = os.environ if env is None else env
    return "WORLD_SIZE" in env and int(env.get("WORLD_SIZE", "1")) >= 1 and "RANK" in env


def rank_env(rank: int, world: int, port: int, base: Optional[Dict[str, str]] = None) -> Dict[str, str]:
    env = dict(os.environ if base is None else base)
    env.update({"RANK": str(rank), "LOCAL_RANK": str(rank), "WORLD_SIZE": str(world),
                "LOCAL_WORLD_SIZE": str(world), "GROUP_RANK": "0", "MASTER_ADDR": "127.0.0.1",
                "MASTER_PORT": str(port)})
    env.setdefault("HSA_ENABLE_IPC_MODE_LEGACY", "0")     # dmabuf IPC only on this host driver
    return env


def spawn(cmd: Sequence[str], world: int, require_gpus: bool = True, poll_s: float = 0.05,
          timeout_s: Optional[float] = None) -> int:
    """Run `cmd` as `world` ranks; returns 0 or the first failing rank's exit code."""
    if world < 1:
        raise LaunchError(f"world size must be >= 1 (got {world})")
    if require_gpus:
        have = visible_gpu_count()
        if have < world:
            print(f"[launch] {world} GPU ranks requested but only {have} GPU(s) visible; refusing to run "
                  f"(no silent fallback to fewer GPUs)", file=sys.stderr, flush=True)
            return 2
    port = free_port()
    procs: List[subprocess.Popen] = []
    for r in range(world):
        procs.append(subprocess.Popen(list(cmd), env=rank_env(r, world, port), start_new_session=False))
    t0 = time.monotonic()
    rc = 0
    try:
        while True:
            codes = [p.poll() for p in procs]
            bad = [c for c in codes if c not in (None, 0)]
            if bad:
                rc = bad[0]
                break
            if all(c == 0 for c in codes):
                break
            if timeout_s is not None and time.monotonic() - t0 > timeout_s:
                print(f"[launch] ranks still running after {timeout_s:.0f}s; stopping them", file=sys.stderr)
                rc = 124
                break
            time.sleep(poll_s)
    except KeyboardInterrupt:
        rc = 130
    if rc:
        _stop(procs)
    for p in procs:
        try:
            p.wait(timeout=60)
        except subprocess.TimeoutExpired:
            p.kill()
            p.wait()
    if rc < 0:                  # killed by a signal: report it the way a shell would
        rc = 128 - rc
    return rc


def _stop(procs: List[subprocess.Popen], grace_s: float = 15.0) -> None:
    for p in procs:
        if p.poll() is None:
            try:
                p.send_signal(signal.SIGTERM)
            except OSError:
                pass
    t = time.monotonic()
    while time.monotonic() - t < grace_s and any(p.poll() is None for p in procs):
        time.sleep(0.05)
    for p in procs:
        if p.poll() is None:
            p.kill()


def self_launch_script(script: str, argv: Sequence[str], world: int, require_gpus: bool = True) -> int:
    return spawn([sys.executable, "-u", script, *argv], world, require_gpus)


def self_launch_module(module: str, argv: Sequence[str], world: int, require_gpus: bool = True) -> int:
    return spawn([sys.executable, "-u", "-m", module, *argv], world, require_gpus)
