"""Kernel time shares of the bench's TIMED region from a rocprofv3 kernel trace.

`rocprofv3 --kernel-trace --output-format csv` of a bench run with GPUSCHED_PROFILE_MARKERS set:
the bench launches a marker kernel (xcd_probe_kernel) right before and right after its timed
epochs, so only the dispatches between the two markers count -- the pre-warm loop, buffer fills,
graph captures and warm-up epochs are left out (rocprofv3 --stats covers the whole process).
Per kernel family: dispatches, summed kernel time, share, and the union of kernel intervals
(engine-active time) next to the window's wall span.  Also reports the traced run's pods/s from
its bench log line, since a traced run is host-bound: compare it with the untraced bench before
reading co-run behaviour into it.

Usage: trace_kernel_summary.py <kernel_trace.csv> [bench log with the JSON line] -> JSON on stdout.
"""
from __future__ import annotations

import csv
import json
import sys
from collections import defaultdict

MARKER = "xcd_probe_kernel"


def family(name: str) -> str:
    if "256_8ph" in name:
        return "gemm_256x256_8phase"
    if "256_w4l" in name:
        tparams = name.split("(")[0].rstrip(">").split(",")
        bn = tparams[4].strip() if len(tparams) > 4 else "256"
        bm = tparams[5].strip() if len(tparams) > 5 else "256"
        return f"gemm_{bm}x{bn}_4wave"
    if "gemm_bf16_nt_kernel" in name:
        return "gemm_tile_" + name.split("<", 1)[1].split(",")[0].strip() + "x" + name.split(",")[1].strip()
    if "gemm_fp8" in name:
        return "gemm_fp8"
    if "splitk_reduce" in name:
        return "splitk_reduce"
    if "stream_triad" in name:
        return "stream_triad"
    if MARKER in name:
        return "marker"
    return "other"


def summarize(path: str) -> dict:
    rows = list(csv.DictReader(open(path)))
    key_s = "Start_Timestamp" if "Start_Timestamp" in rows[0] else "Start_Time"
    key_e = "End_Timestamp" if "End_Timestamp" in rows[0] else "End_Time"
    rows.sort(key=lambda r: int(r[key_s]))
    marks = [i for i, r in enumerate(rows) if MARKER in r.get("Kernel_Name", "")]
    if len(marks) >= 2:
        lo, hi = marks[0], marks[-1]
        t0, t1 = int(rows[lo][key_e]), int(rows[hi][key_s])
        sel = [r for r in rows[lo + 1:hi] if MARKER not in r.get("Kernel_Name", "")]
    else:
        sel = rows
        t0 = min(int(r[key_s]) for r in rows)
        t1 = max(int(r[key_e]) for r in rows)
    tot = defaultdict(float)
    cnt = defaultdict(int)
    iv = []
    for r in sel:
        s, e = int(r[key_s]), int(r[key_e])
        f = family(r.get("Kernel_Name", ""))
        tot[f] += (e - s) / 1e6
        cnt[f] += 1
        iv.append((s, e))
    iv.sort()
    busy, cur_s, cur_e = 0.0, None, None
    for s, e in iv:
        if cur_e is None or s > cur_e:
            if cur_e is not None:
                busy += cur_e - cur_s
            cur_s, cur_e = s, e
        else:
            cur_e = max(cur_e, e)
    if cur_e is not None:
        busy += cur_e - cur_s
    all_ms = sum(tot.values())
    return {"timed_window": len(marks) >= 2, "window_ms": round((t1 - t0) / 1e6, 3),
            "engine_active_ms": round(busy / 1e6, 3),
            "families": {f: {"dispatches": cnt[f], "kernel_ms": round(v, 3), "share_pct": round(100 * v / all_ms, 2)}
                         for f, v in sorted(tot.items(), key=lambda kv: -kv[1])}}


def main() -> None:
    out = summarize(sys.argv[1])
    if len(sys.argv) > 2:
        for line in open(sys.argv[2]):
            if line.startswith("{") and '"metric"' in line:
                d = json.loads(line)
                out["traced_run"] = {"pods_per_s": d["value"], "ms_per_step": d["ms_per_step"],
                                     "cu_share_occupancy_pct": d.get("cu_share_occupancy_pct")}
    print(json.dumps(out, indent=1))


if __name__ == "__main__":
    main()
