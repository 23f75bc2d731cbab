"""xGMI-topology-aware selection of GPU sets for multi-GPU pods
(BASELINE config 4: "one 4-GPU pod placed on an xGMI-connected quad").

The reference never places multi-GPU pods (one UUID per pod).  On an
8xMI355X node every GPU pair has a direct xGMI link (7 links x ~153 GB/s per GPU), so
adjacency alone rarely discriminates; the selection therefore ranks candidate sets by:

1. hard requirement: every pair is 1 xGMI hop (from the agent's amdsmi link matrix,
   `topo_get_link_type`/hops; assumed fully connected only when no matrix is published);
2. NUMA locality: all GPUs on one NUMA node/socket (host staging stays local);
3. best fit: take GPUs from the NUMA domain with the fewest free GPUs that still fits,
   so larger future requests keep a whole domain;
4. measured fabric (agent.fabric, `bw_gbps`): a set containing a degraded pair (copy rate
   below half the node's median pair), or containing a GPU set whose RCCL all-reduce check
   failed after a multi-GPU pod ran on it (agent.probes, `bad_sets`), ranks after every set
   without one, and among the
   rest the set whose slowest pair is fastest wins (quantised to 5 % of the median, so
   measurement noise does not reorder healthy sets) -- ring collectives run at the pace
   of their slowest link;
5. least live xGMI traffic on the set's GPUs (telemetry: amd-smi per-link accumulators,
   quantised to 10 % of a GPU's 7-link capacity so noise does not reorder equal sets);
6. lowest total link weight (amdsmi `topo_get_link_weight`), then lowest indices.
A set is only eligible if each GPU is entirely free (no fractional residents): RCCL
rings of a multi-GPU pod are per-link bound and a co-located partition pod would share
that GPU's links.
"""
from __future__ import annotations

import itertools
from dataclasses import dataclass, field
from typing import Dict, List, Optional, Sequence, Tuple


@dataclass
class Topology:
    n: int
    link_type: List[List[str]] = field(default_factory=list)     # "XGMI" | "PCIE" | "SELF"
    hops: List[List[int]] = field(default_factory=list)
    weight: List[List[int]] = field(default_factory=list)
    numa: List[int] = field(default_factory=list)
    bw: List[List[float]] = field(default_factory=list)               # measured GB/s per ordered pair
    bad_sets: List[List[int]] = field(default_factory=list)           # RCCL set checks below par (agent.probes)

    @classmethod
    def fully_connected(cls, n: int = 8, numa_split: bool = True) -> "Topology":
        lt = [["SELF" if i == j else "XGMI" for j in range(n)] for i in range(n)]
        hops = [[0 if i == j else 1 for j in range(n)] for i in range(n)]
        w = [[0 if i == j else 15 for j in range(n)] for i in range(n)]
        numa = [0 if (not numa_split or i < n // 2) else 1 for i in range(n)]
        return cls(n, lt, hops, w, numa)

    @classmethod
    def from_json(cls, d: Dict) -> "Topology":
        n = int(d["n"])
        return cls(n, d.get("link_type") or [], d.get("hops") or [], d.get("weight") or [], d.get("numa") or [0] * n,
                   d.get("bw_gbps") or [], [list(map(int, b)) for b in d.get("bad_sets") or []])

    def to_json(self) -> Dict:
        out = {"n": self.n, "link_type": self.link_type, "hops": self.hops, "weight": self.weight, "numa": self.numa}
        if self.bw:
            out["bw_gbps"] = self.bw
        if self.bad_sets:
            out["bad_sets"] = self.bad_sets
        return out

    def pair_bw(self, i: int, j: int) -> Optional[float]:
        """Measured rate of the slower direction of a pair (None = not measured)."""
        if not self.bw or max(i, j) >= len(self.bw):
            return None
        a, b = self.bw[i][j], self.bw[j][i]
        return min(a, b) if a > 0 and b > 0 else None

    def bw_median(self) -> Optional[float]:
        vals = sorted(v for i in range(len(self.bw)) for j in range(len(self.bw))
                      if i != j and (v := self.pair_bw(i, j)) is not None)
        return vals[len(vals) // 2] if vals else None

    def connected(self, i: int, j: int) -> bool:
        if i == j:
            return True
        if self.link_type and self.link_type[i][j] != "XGMI":
            return False
        if self.hops and self.hops[i][j] > 1:
            return False
        return True


def is_clique(topo: Topology, gpus: Sequence[int]) -> bool:
    return all(topo.connected(a, b) for a, b in itertools.combinations(gpus, 2))


XGMI_GPU_BPS = 7 * 153e9        # one MI355X: 7 xGMI links x ~153 GB/s per direction


def select_gpu_set(topo: Topology, free_gpus: Sequence[int], k: int,
                   link_load: Optional[Dict[int, float]] = None) -> Optional[Tuple[List[int], float]]:
    """Best k-GPU xGMI clique among `free_gpus`; returns (gpus, quality in [0,1]) or None.
    link_load: per-GPU xGMI utilisation in [0, 1] (live telemetry), optional."""
    free = sorted(set(free_gpus))
    if k <= 0 or len(free) < k:
        return None
    numa_of = {g: (topo.numa[g] if g < len(topo.numa) else 0) for g in free}
    free_per_numa: Dict[int, int] = {}
    for g in free:
        free_per_numa[numa_of[g]] = free_per_numa.get(numa_of[g], 0) + 1
    best: Optional[Tuple[Tuple, List[int]]] = None
    med = topo.bw_median() if k > 1 else None
    combos = itertools.combinations(free, k)
    for combo in combos:
        if not is_clique(topo, combo):
            continue
        domains = {numa_of[g] for g in combo}
        same_numa = len(domains) == 1
        fit = min(free_per_numa[d] for d in domains) if same_numa else 99
        wsum = sum(topo.weight[a][b] if topo.weight else 0 for a, b in itertools.combinations(combo, 2))
        load = sum(round(10 * min(1.0, max(0.0, (link_load or {}).get(g, 0.0)))) for g in combo)
        degraded, bw_q = 0, 0
        if med:
            slowest = min((topo.pair_bw(a, b) or med) for a, b in itertools.combinations(combo, 2))
            degraded = 1 if slowest < 0.5 * med else 0
            bw_q = -round(20 * slowest / med)
        # a set whose RCCL bus bandwidth was measured below par: any superset has its rings
        if any(set(b) <= set(combo) for b in topo.bad_sets):
            degraded = 1
        key = (degraded, 0 if same_numa else 1, fit, bw_q, load, wsum, combo)
        if best is None or key < best[0]:
            best = (key, list(combo))
    if best is None:
        return None
    same = best[0][1] == 0
    quality = (1.0 if same else 0.6) * (1.0 if best[0][2] in (k, 99) else 0.9) * (0.5 if best[0][0] else 1.0)
    return best[1], quality
