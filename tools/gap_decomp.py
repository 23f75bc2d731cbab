"""Where the bench's step time goes against its floors.

Replays the TIMED pods of one bench run (`bench.py --dump-placements F`, the driver's seed /
steps / warmup) on one MI355X in several regimes, interleaved `--reps` times, and calibrates the
amd-smi UMC activity that the bench samples against triads of known bandwidth:

  replay            the pods through the bench's DeviceExecutor (4 Burstable slot streams,
                    unit-ordered, HIP graphs): the bench's device work without its host / control
                    plane; `replay_nograph` the same from eager launches (the filtered replays'
                    reference)
  replay_gemm       the same pods and slots with the stream kernels left out (GEMMs only)
  replay_triad      ... with the GEMMs left out (stream kernels only)
  serial_share      every kernel of every pod, in pod order, on ONE stream (no co-running),
                    GEMM tiles for the pod's 64-CU share as in the bench
  serial_full       the same with whole-chip GEMM tiles (the lone-kernel picker)
  triad_serial      only the stream kernels, one stream (the HBM time at the lone rate)
  gemm_serial_full  only the GEMMs, one stream, whole-chip tiles (the MFMA time at the lone rate)
  gemm_serial_share only the GEMMs, one stream, share tiles
  split_full        two streams side by side: every triad on one, every GEMM (whole-chip tiles)
                    on the other -- the best overlap of the two kinds when pod order is free
  split_share       the same with the share tiles, GEMMs spread over 4 streams by pod slot
  mask_split_<u>    triads on a stream CU-masked to u of the 8 units, GEMMs on the other 8-u
                    units (tiles for those CUs): disjoint CU partitions

and `triad_units_<u>` (a 768 MB triad on u masked units: bandwidth vs CUs) and `umc_cal` (a
triad at several grid sizes for ~0.4 s each: achieved TB/s vs amd-smi umc_activity).

Writes --out (JSON) and prints one line per regime.  Read by tools/gap_report.py.
"""
from __future__ import annotations

import argparse
import json
import os
import sys
import time

# the bench's hardware-queue limit (bench.py).  Measured (profiles/r06_gap/): the same replay
# runs 7.32 ms / step under a limit of 32 with ~20 streams alive in the process vs 6.75 / 6.69
# under 16 / 8 with 5 -- every regime family below therefore runs in its own process with only
# the streams it uses (the 4 slot streams, or 2 masked ones)
os.environ.setdefault("GPU_MAX_HW_QUEUES", "16")
from typing import Callable, Dict, List

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

import torch  # noqa: E402

from k8s_gpu_scheduler_amd.models import workloads as W  # noqa: E402
from k8s_gpu_scheduler_amd.ops import loadgen  # noqa: E402
from k8s_gpu_scheduler_amd.ops.cumask import MaskedStream  # noqa: E402
from k8s_gpu_scheduler_amd.parallel.executor import DeviceExecutor, PodRun  # noqa: E402
from k8s_gpu_scheduler_amd.parallel.podbench import build_parser, gpu_executor  # noqa: E402
from k8s_gpu_scheduler_amd.plugins.gpu.devices import CUS_PER_XCD as CUS_PER_UNIT, cu_slice_mask  # noqa: E402


class KindExecutor(DeviceExecutor):
    """DeviceExecutor whose pods run only one kind of op ('gemm' / 'triad'; '' = all)."""
    kind = ""

    def _enqueue_ops(self, r, bufs, st, budget):
        for _ in range(r.iters):
            for o, t in bufs.ops:
                if self.kind == "gemm" and not o.is_gemm or self.kind == "triad" and o.is_gemm:
                    continue
                _one(o, t, st, budget, self.triad_blocks)


def _one(o, t, st, budget: int, blocks: int = 0) -> None:
    if o.kind == "gemm":
        a, bt, bias, c = t
        loadgen.gemm(a, bt, out=c, bias=bias, relu=o.relu, stream=st, cu_budget=budget)
    elif o.kind == "gemm8":
        a, bt, bias, c = t
        loadgen.gemm_fp8(a, bt, out=c, bias=bias, relu=o.relu, stream=st, cu_budget=budget)
    else:
        x, y, z = t
        loadgen.triad(x, y, z, 1.0001, blocks=blocks, stream=st)


def timed(fn: Callable[[], None]) -> float:
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    fn()
    torch.cuda.synchronize()
    return (time.perf_counter() - t0) * 1e3


def main() -> None:
    ap = argparse.ArgumentParser()
    ap.add_argument("--placements", required=True)
    ap.add_argument("--reps", type=int, default=3)
    ap.add_argument("--out", default="gpurun_out/gap/decomp.json")
    ap.add_argument("--mask-units", default="", help="mask_split regimes for these unit counts (own process)")
    ap.add_argument("--triad-units", action="store_true", help="triad TB/s vs masked units")
    ap.add_argument("--umc-cal", action="store_true", help="triad TB/s vs amd-smi umc_activity")
    ap.add_argument("--extra-streams", default="", help="K:before|after -- K idle streams that each "
                    "dispatch one tiny kernel (so get a hardware queue) before / after the slot streams")
    ap.add_argument("--bench-args", default="", help="bench.py flags for the executor's kernel policy, "
                    "e.g. '--gemm-policy 8'")
    ap.add_argument("--passes", type=int, default=1,
                    help="back-to-back passes per timed regime run; amd-smi umc is averaged over the "
                         "last half of the run (its firmware moving average lags a regime change)")
    ap.add_argument("--only", default="", help="comma-separated regime names to run (default: all)")
    args = ap.parse_args()
    dump = json.load(open(args.placements))
    names = dump["workloads"]
    epochs = [e["arr"] for e in dump["epochs"] if e["timed"]]
    pods = [(names[int(r[3])], int(r[1]), int(r[2]), int(r[4])) for ep in epochs for r in ep if int(r[0]) == 0]
    steps = len(epochs)
    torch.cuda.set_device(0)
    ba = build_parser().parse_args(args.bench_args.split())
    ex = gpu_executor(ba, 0)
    kx = KindExecutor(0)
    kx.use_graphs = False
    kx.triad_blocks = ex.triad_blocks
    extra = []

    def make_extra() -> None:
        k = int(args.extra_streams.split(":")[0])
        for _ in range(k):
            st = torch.cuda.Stream()
            with torch.cuda.stream(st):
                torch.zeros(1, device="cuda").add_(1)
            extra.append(st)
        torch.cuda.synchronize()
    if args.extra_streams.endswith(":before"):
        make_extra()
    mask_units = [int(x) for x in args.mask_units.split(",") if x]
    core = not mask_units and not args.triad_units and not args.umc_cal
    if core:
        ex.warm([PodRun(0, wl, u, n, it, masked=False) for wl, u, n, it in pods])
    else:                                               # operands only: no slot streams / queues
        for wl, u, n, it in pods:
            ex.buffers(W.get(wl), u, n)
    kx._bufs, kx._streams = ex._bufs, ex._streams       # the same operands and slot streams
    if args.extra_streams.endswith(":after"):
        make_extra()
    flops = sum(W.get(wl).flops * it for wl, _, _, it in pods)
    mbytes = sum(W.get(wl).bytes * it for wl, _, _, it in pods)
    tri_bytes = sum(sum(o.bytes for o in W.get(wl).ops if not o.is_gemm) * it for wl, _, _, it in pods)

    def epochs_runs() -> List[List[PodRun]]:
        out, i = [], 0
        for ep in epochs:
            rs = []
            for r in ep:
                if int(r[0]) != 0:
                    continue
                rs.append(PodRun(i, names[int(r[3])], int(r[1]), int(r[2]), int(r[4]), masked=False))
                i += 1
            out.append(rs)
        return out

    def replay(e: DeviceExecutor, kind: str = "", ahead: int = 0) -> Callable[[], None]:
        """ahead = 0: every epoch enqueued at once; L > 0: the bench's launch-ahead pipeline (epoch
        e is launched once epoch e-L-1 has finished, host-polled as the bench's collect)."""
        def f() -> None:
            if isinstance(e, KindExecutor):
                e.kind = kind
            pending = []
            for rs in epochs_runs():
                e.launch_epoch(rs)
                pending.append(rs)
                while ahead and len(pending) > ahead:
                    e.wait_epoch(pending.pop(0))
            e.wait_all()
        return f

    # serial / split regimes reuse the 4 slot streams (no extra hardware queues)
    s_aux = [ex.stream_for(u, 2, False).stream for u in (0, 2, 4, 6)] if core else []
    s_main = s_aux[0] if core else None
    s_tri = torch.cuda.Stream() if core else None       # split_share's triads (a 5th stream)

    def serial(kind: str, share: bool) -> Callable[[], None]:
        def f() -> None:
            for wl, u, n, it in pods:
                bufs = ex.buffers(W.get(wl), u, n)
                for _ in range(it):
                    for o, t in bufs.ops:
                        if kind == "gemm" and not o.is_gemm or kind == "triad" and o.is_gemm:
                            continue
                        _one(o, t, s_main, n * CUS_PER_UNIT if share else 0)
        return f

    def split(share: bool, tri_st=None, gemm_st=None, gemm_budget: int = 0) -> Callable[[], None]:
        def f() -> None:
            ts = tri_st or (s_tri if share else s_aux[0])
            for wl, u, n, it in pods:
                bufs = ex.buffers(W.get(wl), u, n)
                gs = gemm_st or (s_aux[u // 2 % 4] if share else s_aux[1])
                b = n * CUS_PER_UNIT if share else gemm_budget
                for _ in range(it):
                    for o, t in bufs.ops:
                        _one(o, t, gs if o.is_gemm else ts, b)
        return f

    regimes: Dict[str, Callable[[], None]] = {} if not core else {
        "replay": replay(ex),
        "replay_la2": replay(ex, "", 2),
        "replay_nograph": replay(kx, ""),
        "replay_gemm": replay(kx, "gemm"),
        "replay_triad": replay(kx, "triad"),
        "serial_share": serial("", True),
        "serial_full": serial("", False),
        "triad_serial": serial("triad", False),
        "gemm_serial_full": serial("gemm", False),
        "gemm_serial_share": serial("gemm", True),
        "split_full": split(False),
        "split_share": split(True),
    }
    masked: Dict[int, tuple] = {}
    for u in mask_units:
        ts = MaskedStream(cu_slice_mask(0, u))
        gs = MaskedStream(cu_slice_mask(u, 8 - u))
        masked[u] = (ts, gs)
        regimes[f"mask_split_{u}"] = split(False, ts.stream, gs.stream, (8 - u) * CUS_PER_UNIT)

    if args.only:
        keep = set(args.only.split(","))
        regimes = {k: v for k, v in regimes.items() if k in keep}
    smi = None
    try:
        from k8s_gpu_scheduler_amd.telemetry.smi_sampler import ActivitySampler
        smi = ActivitySampler([0], 0.005)
        if not smi.start():
            print("amd-smi sampler off:", smi.error, flush=True)
            smi = None
    except Exception as e:              # calibration is optional; timings are not
        print("amd-smi sampler off:", e, flush=True)
        smi = None

    for f in regimes.values():          # one untimed pass each (graphs, queues, clocks)
        f()
    res: Dict[str, Dict[str, object]] = {k: {"ms": []} for k in regimes}
    for rep in range(args.reps):
        for k, f in regimes.items():
            w0 = time.time()
            ms = timed(lambda: [f() for _ in range(args.passes)]) / args.passes
            w1 = time.time()
            res[k]["ms"].append(round(ms, 3))
            if smi is not None:
                smi.poll()
                s = smi.summary(0.5 * (w0 + w1), w1)
                res[k].setdefault("umc", []).append(s["umc_activity_pct_mean"])
                res[k].setdefault("gfx", []).append(s["gfx_activity_pct_mean"])
        print(f"rep {rep}: " + ", ".join(f"{k} {v['ms'][-1]:.1f}" for k, v in res.items()), flush=True)
    for k, v in res.items():
        v["ms_per_step"] = round(min(v["ms"]) / steps, 4)
        v["ms_per_step_median"] = round(sorted(v["ms"])[len(v["ms"]) // 2] / steps, 4)

    # triad bandwidth vs masked CU units (768 MB per pass)
    n = 64 << 20
    x, y, z = (torch.ones(n, device="cuda") for _ in range(3))
    tb = {}
    for u in ((1, 2, 3, 4, 5, 6, 8) if args.triad_units else ()):
        ms_ = MaskedStream(cu_slice_mask(0, u))

        def tri(st=ms_.stream) -> None:
            for _ in range(20):
                loadgen.triad(x, y, z, 1.0001, stream=st)
        tri()
        best = min(timed(tri) for _ in range(3))
        tb[u] = round(12.0 * n * 20 / (best / 1e3) / 1e12, 3)
        ms_.close()
    print("triad TB/s by masked units:", tb, flush=True)

    cal = []
    if smi is not None and args.umc_cal:
        for blocks in (32, 64, 128, 256, 512, 8192):
            def tri2(b=blocks) -> None:
                loadgen.triad(x, y, z, 1.0001, blocks=b)
            tri2()
            torch.cuda.synchronize()
            w0 = time.time()
            t0 = time.perf_counter()
            k = 0
            while time.perf_counter() - t0 < 0.45:
                for _ in range(8):
                    tri2()
                k += 8
                torch.cuda.synchronize()
            el = time.perf_counter() - t0
            w1 = time.time()
            smi.poll()
            s = smi.summary(w0 + 0.1, w1)         # skip the moving average's ramp
            cal.append({"blocks": blocks, "tbps": round(12.0 * n * k / el / 1e12, 3),
                        "umc_pct": s["umc_activity_pct_mean"], "gfx_pct": s["gfx_activity_pct_mean"],
                        "samples": s["samples"]})
            print("umc cal", cal[-1], flush=True)
    if smi is not None:
        smi.stop()
    for ts, gs in masked.values():
        ts.close()
        gs.close()
    out = {"steps": steps, "pods": len(pods), "model_flops_per_step": flops / steps,
           "model_bytes_per_step": mbytes / steps, "triad_bytes_per_step": tri_bytes / steps,
           "regimes": res, "triad_tbps_by_units": tb, "umc_calibration": cal,
           "placements": args.placements, "reps": args.reps}
    os.makedirs(os.path.dirname(args.out) or ".", exist_ok=True)
    json.dump(out, open(args.out, "w"), indent=1)
    for k, v in res.items():
        print(f"{k:20s} {v['ms_per_step']:.3f} ms/step  umc {v.get('umc')}", flush=True)
    ex.close()


if __name__ == "__main__":
    main()
