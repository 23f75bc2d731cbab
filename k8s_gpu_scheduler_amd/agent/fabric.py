"""Measured xGMI fabric bandwidth per GPU pair, published for multi-GPU placement.

The reference places single devices only (reference pkg/plugins/gpu_plugin/gpu_plugins.go:915)
and has no fabric view.  On an 8xMI355X node every pair is one xGMI hop, so the static link
matrix (amdsmi link type / hops / weight) rarely discriminates -- but a link that trained
at a lower width or speed, or retimers that degrade, do: RCCL rings are per-link bound
(SURVEY.md §5.8 item 4), so one slow pair slows every collective of a pod placed across it.

The node agent therefore measures a device-to-device copy rate for every ordered GPU pair
(`hipMemcpyPeerAsync` between the two devices' HBM, native/hip/p2p.hip) at start-up and
after partition changes -- only while the node's GPUs are idle, and in a CHILD process, so
the agent itself never holds a GPU context -- and publishes the matrix with the topology
(`gpusched:topology:<node>`, key "bw_gbps").  The GPU plugin's `select_gpu_set` steers
multi-GPU pods away from sets containing a degraded pair and otherwise breaks ties on the
set's slowest pair.

    python -m k8s_gpu_scheduler_amd.agent.fabric [--mib 256] [--iters 10]   (prints JSON)
"""
from __future__ import annotations

import argparse
import json
import logging
import subprocess
import sys
from typing import Any, Callable, Dict, List, Optional

log = logging.getLogger(__name__)


def measure(mib: int = 256, iters: int = 10) -> Dict[str, Any]:
    """In THIS process (opens a GPU context on every device): the peer-access matrix and
    GB/s of every ordered pair (the diagonal = the device's own HBM copy rate)."""
    from .. import _native
    h = _native.hip(required=True)
    n = h.device_count()
    acc = h.peer_access_matrix()
    bw = [[0.0] * n for _ in range(n)]
    for i in range(n):
        for j in range(n):
            if i == j or acc[i * n + j]:
                bw[i][j] = round(h.peer_copy_gbps(i, j, mib << 20, iters), 1)
    return {"n": n, "peer_access": [[int(acc[i * n + j]) for j in range(n)] for i in range(n)], "bw_gbps": bw,
            "bytes": mib << 20, "iters": iters}


def measure_in_child(mib: int = 256, iters: int = 10, timeout_s: float = 120.0,
                     env: Optional[Dict[str, str]] = None) -> Optional[Dict[str, Any]]:
    """`measure` in a child process (the caller never initialises the GPU); None on failure."""
    try:
        p = subprocess.run([sys.executable, "-m", "k8s_gpu_scheduler_amd.agent.fabric", "--mib", str(mib),
                            "--iters", str(iters)], capture_output=True, text=True, timeout=timeout_s, env=env)
    except (OSError, subprocess.TimeoutExpired) as e:
        log.warning("fabric probe failed to run: %s", e)
        return None
    if p.returncode != 0:
        log.warning("fabric probe exited %d: %s", p.returncode, p.stderr[-500:])
        return None
    try:
        return json.loads(p.stdout.strip().splitlines()[-1])
    except (ValueError, IndexError) as e:
        log.warning("fabric probe output unreadable: %s", e)
        return None


class FabricProber:
    """Agent side: when to probe (never with busy GPUs), what to publish."""

    def __init__(self, probe: Callable[[], Optional[Dict[str, Any]]] = measure_in_child):
        self.probe = probe
        self.last: Optional[Dict[str, Any]] = None
        self.due = True                  # at start-up, and again after a partition change

    def invalidate(self) -> None:
        self.due = True

    def maybe_probe(self, busy: Callable[[], List[str]]) -> Optional[Dict[str, Any]]:
        if not self.due:
            return None
        reasons = busy()
        if reasons:
            log.info("fabric probe deferred: GPUs busy (%s)", "; ".join(reasons[:3]))
            return None
        res = self.probe()
        self.due = False
        if res is not None:
            self.last = res
        return res


def degraded_pairs(bw: List[List[float]], frac: float = 0.5) -> List[tuple]:
    """Ordered pairs whose measured rate is below `frac` x the median off-diagonal rate."""
    vals = sorted(v for i, r in enumerate(bw) for j, v in enumerate(r) if i != j and v > 0)
    if not vals:
        return []
    med = vals[len(vals) // 2]
    return [(i, j) for i, r in enumerate(bw) for j, v in enumerate(r) if i != j and 0 <= v < frac * med]


def main(argv=None) -> int:
    ap = argparse.ArgumentParser(description="per-pair device copy bandwidth (JSON)")
    ap.add_argument("--mib", type=int, default=256)
    ap.add_argument("--iters", type=int, default=10)
    a = ap.parse_args(argv)
    print(json.dumps(measure(a.mib, a.iters)), flush=True)
    return 0


if __name__ == "__main__":
    raise SystemExit(main())
