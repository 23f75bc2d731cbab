"""Synthetic pod workloads (the "model families" the scheduler places).

The reference characterises 18 MLPerf-style inference workloads -- {onnx, tensorflow} x
{mobilenet, resnet50, ssd_mobilenet} x batch {1024, 2048, 4096} -- only through their
measured throughput per GPU share (reference
pkg/recommender/recommender/configurations_train.ods) and pairwise interference
(interference_train.ods).  There are no model binaries to run here, so each workload is
re-created as a kernel mix with the same *character* on MI355X, built from the native
load kernels (ops.loadgen):

  resnet50       compute-bound: a chain of bf16 MFMA GEMMs (+bias+ReLU fused)
  mobilenet      memory-bound: HBM triad passes (depthwise-like) + one small GEMM
  ssd_mobilenet  mixed: GEMMs and HBM streaming in similar proportion

The batch suffix scales the GEMM M dimension and the streamed bytes; the framework prefix
selects a different layer shape (onnx: 2048-wide, tensorflow: 1536/2560-wide).  One
*iteration* ("query batch") runs the op list once; a pod's throughput is iterations/s,
its SLO a minimum iterations/s -- the same semantics as the reference's SLO env
(SURVEY.md §2.7.1).
"""
from __future__ import annotations

from dataclasses import dataclass
from typing import Dict, List, Optional, Tuple


@dataclass(frozen=True)
class Op:
    kind: str              # "gemm" (bf16) | "gemm8" (fp8 e4m3, bf16 out) | "triad"
    M: int = 0
    N: int = 0
    K: int = 0
    relu: bool = True
    n_floats: int = 0      # triad

    @property
    def is_gemm(self) -> bool:
        return self.kind in ("gemm", "gemm8")

    @property
    def flops(self) -> float:
        return 2.0 * self.M * self.N * self.K if self.is_gemm else 2.0 * self.n_floats

    @property
    def bytes(self) -> float:
        if self.kind == "gemm":
            return 2.0 * (self.M * self.K + self.N * self.K + self.M * self.N)
        if self.kind == "gemm8":
            return 1.0 * (self.M * self.K + self.N * self.K) + 2.0 * self.M * self.N
        return 12.0 * self.n_floats

    def mfma_rate(self) -> float:
        """MFMA throughput relative to bf16 (the fp8 MFMA does twice the work per clock)."""
        return 2.0 if self.kind == "gemm8" else 1.0


@dataclass(frozen=True)
class Workload:
    name: str
    family: str                  # resnet50 | mobilenet | ssd_mobilenet
    framework: str               # onnx | tensorflow
    batch: int
    ops: Tuple[Op, ...]
    hbm_gib: float               # declared footprint (request)

    @property
    def flops(self) -> float:
        return sum(o.flops for o in self.ops)

    @property
    def bytes(self) -> float:
        return sum(o.bytes for o in self.ops)

    @property
    def intensity(self) -> float:
        return self.flops / max(self.bytes, 1.0)


def _mk(framework: str, family: str, batch: int) -> Workload:
    wide = 2048 if framework == "onnx" else 2560
    narrow = 1024 if framework == "onnx" else 1536
    m = batch                                         # 1024 / 2048 / 4096
    if family == "resnet50":
        ops = (Op("gemm", m, wide, wide), Op("gemm", m, wide, wide), Op("gemm", m, wide, wide))
        hbm = 8.0
    elif family == "mobilenet":
        ops = (Op("triad", n_floats=m * 16384), Op("triad", n_floats=m * 16384),
               Op("gemm", m, narrow, narrow))
        hbm = 4.0
    else:  # ssd_mobilenet
        ops = (Op("gemm", m, wide, narrow), Op("triad", n_floats=m * 16384), Op("gemm", m, narrow, wide))
        hbm = 6.0
    return Workload(f"{framework}_{family}_{batch}", family, framework, batch, ops, hbm * (batch / 1024) ** 0.5)


FRAMEWORKS = ("onnx", "tensorflow")
FAMILIES = ("mobilenet", "resnet50", "ssd_mobilenet")
BATCHES = (1024, 2048, 4096)

CATALOG: Dict[str, Workload] = {}
for _fw in FRAMEWORKS:
    for _fa in FAMILIES:
        for _b in BATCHES:
            _w = _mk(_fw, _fa, _b)
            CATALOG[_w.name] = _w
NAMES: List[str] = sorted(CATALOG)
INDEX: Dict[str, int] = {n: i for i, n in enumerate(NAMES)}

# Workloads OUTSIDE the reference's 18 (no configuration / interference rows, no co-run rows
# in data/corun_mi355x.json): kernel mixes the catalog does not have, runnable by the executor
# and the pod entrypoint, and what the co-run model's cold start is checked on
# (models.coldstart, tools/corun_extra_groups.py -> profiles/r05_coldstart/):
#   fp8_llm_2048     three fp8 GEMMs 2048 x 4096 x 4096 (LLM-projection-like, MFMA-bound on
#                    the block-scaled fp8 MFMA the catalog never uses)
#   triad_only_2048  three HBM stream passes, no GEMM at all
EXTRA: Dict[str, Workload] = {
    "fp8_llm_2048": Workload("fp8_llm_2048", "llm_fp8", "hip", 2048, (Op("gemm8", 2048, 4096, 4096),) * 3, 1.0),
    "triad_only_2048": Workload("triad_only_2048", "stream", "hip", 2048,
                                (Op("triad", n_floats=2048 * 16384),) * 3, 1.0),
}


def get(name: str) -> Workload:
    """A catalog or extra workload by exact name."""
    w = CATALOG.get(name)
    if w is None:
        w = EXTRA.get(name)
    if w is None:
        raise KeyError(name)
    return w


def workload_for_pod(pod_name: str) -> Workload:
    """Same matching rule as the recommender: first catalog name that is a substring of
    the pod name with '-' -> '_' (reference recom_server.py:67-71); the extra workloads after
    the catalog."""
    nm = pod_name.replace("-", "_")
    for table in (CATALOG, EXTRA):
        for n in sorted(table, key=len, reverse=True):
            if n in nm:
                return table[n]
    raise KeyError(pod_name)


def roofline_split(pod_name: str, tflops: float = 1.0e3, tbps: float = 6.0) -> Optional[Tuple[float, float]]:
    """(MFMA-bound s, HBM-bound s) of one iteration of the pod's workload alone on a whole
    GPU (GEMMs at `tflops`, stream passes at `tbps`); None for a pod outside the catalog.
    The GPU plugin's complementarity term reads this (extras "roofline")."""
    try:
        w = workload_for_pod(pod_name)
    except KeyError:
        return None
    m = sum(o.flops / o.mfma_rate() for o in w.ops if o.is_gemm) / (tflops * 1e12)
    h = sum(o.bytes for o in w.ops if not o.is_gemm) / (tbps * 1e12)
    return m, h


# ---------------------------------------------------------------- analytic predictions
CUS = 256                          # MI355X compute units
POD_CU_BUDGET = 64                 # a bench pod's GEMM tile budget (2 CU-slice units x 32 CUs)


# block tile (BM, BN) of the native GEMM kernels (native/hip/loadgen.hip kTileBM / kTileBN)
_TILE = {1: (128, 128), 2: (64, 128), 3: (64, 64), 4: (256, 256), 10: (256, 256)}


def default_gemm_workgroups(M: int, N: int, K: int, cu_budget: int = 0, fp8: bool = False) -> int:
    """Workgroups the native GEMM launches for this shape under the DEFAULT kernel policy
    (policy 10, or 1: the same grids -- tile 14 launches tile 10's; no forced tile, split-K off)
    -- a pure-Python copy of pick_gemm_tile /
    resolve_gemm_tile / fp8_tile_128 (native/hip/loadgen.hip), so the CU-fill feature needs no
    HIP build and never reads the process-wide tile settings.  Pinned against the
    native picker in tests/test_gemm_policy_picker.py."""
    alone = cu_budget <= 0 or cu_budget >= CUS
    budget = CUS if alone else cu_budget
    if fp8:
        need = 2 * CUS if alone else cu_budget
        big = M % 128 == 0 and N % 128 == 0 and (M // 128) * (N // 128) >= need
        return (M // 128) * (N // 128) if big else (M // 64) * (N // 64)
    per_cu = 2 if alone else 1
    if M % 256 == 0 and N % 256 == 0 and (M // 256) * (N // 256) >= budget:
        t = 10
    elif (M // 128) * (N // 128) >= per_cu * budget:
        t = 1
    elif (M // 64) * (N // 128) >= per_cu * budget and N % 128 == 0:
        t = 2
    else:
        t = 3
    if t == 10 and K < 128:
        t = 4
    bm, bn = _TILE[t]
    if M % bm or N % bn:
        bm, bn = _TILE[3]
    return (M // bm) * (N // bn)


def cu_fill(w: Workload, cu_budget: int = POD_CU_BUDGET) -> Optional[float]:
    """Fraction of the chip's CUs the workload's kernels occupy, weighted by their (roofline)
    time: min(1, workgroups / CUs) per kernel -- GEMM workgroups as the native tile picker
    launches them for `cu_budget` under the default policy (default_gemm_workgroups), the
    stream kernels' 8192 blocks fill the chip.  A pod that leaves CUs idle alone leaves
    co-runners room; one that fills the chip alone presses on and suffers from every co-runner
    (models.coldstart)."""
    t = f = 0.0
    for o in w.ops:
        dt = roofline_seconds(Workload(w.name, w.family, w.framework, w.batch, (o,), 0.0), 1.0)
        if o.is_gemm:
            fo = min(1.0, default_gemm_workgroups(o.M, o.N, o.K, cu_budget, o.kind == "gemm8") / CUS)
        else:
            fo = 1.0
        t += dt
        f += dt * fo
    return f / t if t > 0 else None


def roofline_seconds(w: Workload, share: float, peak_tflops: float = 1100.0, hbm_tbps: float = 5.5,
                     share_bw_exp: float = 0.6) -> float:
    """Per-iteration time on a `share` of the GPU's XCDs.  Compute scales linearly with
    the share; a CU subset can still pull a super-linear fraction of HBM bandwidth
    (share**share_bw_exp).  Defaults are measured MI355X rates of the native kernels
    (gemm ~1.1 PF on a whole chip, triad ~5.5 TB/s); `profile_workloads` replaces this
    with measurements."""
    t = 0.0
    for o in w.ops:
        if o.is_gemm:
            t += max(o.flops / (peak_tflops * o.mfma_rate() * 1e12 * share),
                     o.bytes / (hbm_tbps * 1e12 * share ** share_bw_exp))
        else:
            t += o.bytes / (hbm_tbps * 1e12 * share ** share_bw_exp)
    return t


def analytic_tables(model: str = "MI355X", parts=(1, 2, 4, 8)) -> Tuple[List[str], List[str], List[List[float]],
                                                                         List[str], List[List[float]]]:
    """(conf_index, conf_cols, conf_values, intf_cols, intf_values) -- configuration
    throughput (iterations/s) per partition share and pairwise interference (throughput
    lost when co-located on the same GPU: HBM contention between memory-heavy kernels),
    in the reference's matrix layout."""
    idx = list(NAMES)
    cols = [f"{p}P_{model}" for p in parts]
    conf = [[1.0 / roofline_seconds(CATALOG[n], 1.0 / p) for p in parts] for n in idx]
    intf_vals = []
    for n in idx:
        a = CATALOG[n]
        base = 1.0 / roofline_seconds(a, 0.25)
        mem_a = min(1.0, 1.0 / max(a.intensity / 100.0, 1e-3))
        row = []
        for m in idx:
            b = CATALOG[m]
            mem_b = min(1.0, 1.0 / max(b.intensity / 100.0, 1e-3))
            row.append(base * 0.25 * mem_a * mem_b)
        intf_vals.append(row)
    return idx, cols, conf, list(idx), intf_vals
