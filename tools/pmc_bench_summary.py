"""Aggregate tools/gpu_pmc_bench.sh's rocprofv3 counter CSVs per kernel family, over the TIMED
region only: the bench (GPUSCHED_PROFILE_MARKERS) launches a marker kernel (xcd_probe_kernel)
right before and right after its timed epochs, and only dispatches between the two markers of a
run count -- warm-up epochs, buffer fills and the pre-warm loop are left out.

Per family: dispatches, MFMA-busy share of the busy CUs' SIMD cycles, HBM bytes read / written
(FETCH_SIZE x 2 -- on gfx950 FETCH_SIZE counts half the bytes of 16-B-per-lane streaming reads,
MI355X_MICROARCH.md "HBM" -- and WRITE_SIZE), and next to them the COMPULSORY bytes of the timed
pods' ops of that family (models.workloads.Op.bytes: A + B + C once per GEMM, 8 B read + 4 B
written per triad element), with the measured / compulsory ratio.  Writes summary.json."""
import csv
import glob
import json
import os
import sys
from collections import defaultdict

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
if ROOT not in sys.path:
    sys.path.insert(0, ROOT)

MARKER = "xcd_probe_kernel"
TILE_FAMILY = {1: "gemm_tile_128x128", 2: "gemm_tile_64x128", 3: "gemm_tile_64x64", 4: "gemm_tile_256x256",
               5: "gemm_tile_256x128", 6: "gemm_tile_128x128", 7: "gemm_tile_64x128", 8: "gemm_tile_256x128",
               9: "gemm_256x256_8phase", 10: "gemm_256x256_8phase", 13: "gemm_256x128_8phase",
               14: "gemm_256x256_4wave", 15: "gemm_256x128_4wave", 16: "gemm_128x128_4wave"}


def family(name: str) -> str:
    if "256_8ph" in name:
        return "gemm_256x256_8phase"
    if "256_w4l" in name:
        tparams = name.split("(")[0].rstrip(">").split(",")
        bn = tparams[4].strip() if len(tparams) > 4 else "256"
        bm = tparams[5].strip() if len(tparams) > 5 else "256"
        return f"gemm_{bm}x{bn}_4wave"
    if "gemm_bf16_nt_kernel" in name:
        return "gemm_tile_" + name.split("<", 1)[1].split(",")[0] + "x" + name.split(",")[1].strip()
    if "stream_triad" in name:
        return "stream_triad"
    if MARKER in name:
        return "marker"
    return "other"


def _rows(f: str):
    with open(f) as fh:
        return list(csv.DictReader(fh))


def timed_window(rows) -> tuple:
    """(first, last) dispatch id strictly inside the two marker dispatches (None: no markers)."""
    ids = sorted(int(r["Dispatch_Id"]) for r in rows if MARKER in r.get("Kernel_Name", ""))
    ids = sorted(set(ids))
    if len(ids) < 2:
        return None
    return ids[0], ids[-1]


def compulsory(pods_file: str) -> dict:
    """Compulsory HBM bytes per family of the timed pods' ops (the tile picker decides which
    GEMM family an op runs on: the pod's CU share as its budget, as the executor passes it)."""
    from k8s_gpu_scheduler_amd.models.workloads import CATALOG
    from k8s_gpu_scheduler_amd import _native
    h = _native.hip(required=True)
    d = json.load(open(pods_file))
    out = defaultdict(lambda: {"read": 0.0, "write": 0.0})
    for wl, n_units, iters in d["pods"]:
        budget = n_units * 32 if d.get("gemm_share", True) else 0
        for o in CATALOG[wl].ops:
            if o.kind == "gemm":
                t = h.pick_gemm_tile(o.M, o.N, budget)
                fam = TILE_FAMILY.get(t, "gemm_tile_64x64")
                out[fam]["read"] += 2.0 * (o.M * o.K + o.N * o.K) * iters
                out[fam]["write"] += 2.0 * o.M * o.N * iters
            else:
                out["stream_triad"]["read"] += 8.0 * o.n_floats * iters
                out["stream_triad"]["write"] += 4.0 * o.n_floats * iters
    return out


def main(root: str) -> None:
    agg = defaultdict(lambda: defaultdict(float))
    disp = defaultdict(set)
    windows = {}
    for f in sorted(glob.glob(os.path.join(root, "p*", "**", "*counter_collection.csv"), recursive=True)):
        rows = _rows(f)
        win = timed_window(rows)
        windows[f] = win
        for row in rows:
            did = int(row["Dispatch_Id"])
            if win is not None and not (win[0] < did < win[1]):
                continue
            fam = family(row.get("Kernel_Name", ""))
            if fam == "marker":
                continue
            agg[fam][row["Counter_Name"]] += float(row["Counter_Value"])
            disp[fam].add((f, did))
    comp = {}
    pods = os.path.join(root, "timed_pods.json")
    if os.path.exists(pods):
        try:
            comp = compulsory(pods)
        except Exception as e:           # no GPU module here: measured side only
            print("compulsory bytes unavailable:", e, file=sys.stderr)
    out = {}
    tot_bytes = sum(c.get("FETCH_SIZE", 0.0) * 2 + c.get("WRITE_SIZE", 0.0) for c in agg.values()) * 1024
    for fam, c in sorted(agg.items()):
        d = {"counters": {k: round(v, 1) for k, v in c.items()}}
        if c.get("SQ_VALU_MFMA_BUSY_CYCLES") is not None and c.get("SQ_BUSY_CU_CYCLES"):
            # MFMA busy per SIMD cycle of the CUs that were busy
            d["mfma_busy_of_busy_cu_pct"] = round(100 * c["SQ_VALU_MFMA_BUSY_CYCLES"] / (4 * c["SQ_BUSY_CU_CYCLES"]), 1)
        rd = c.get("FETCH_SIZE", 0.0) * 2 * 1024 if "FETCH_SIZE" in c else None
        wr = c.get("WRITE_SIZE", 0.0) * 1024 if "WRITE_SIZE" in c else None
        if rd is not None:
            d["hbm_read_gib"] = round(rd / 2 ** 30, 3)
        if wr is not None:
            d["hbm_write_gib"] = round(wr / 2 ** 30, 3)
        if tot_bytes > 0 and rd is not None and wr is not None:
            d["share_of_measured_bytes_pct"] = round(100.0 * (rd + wr) / tot_bytes, 2)
        if fam in comp:
            cr, cw = comp[fam]["read"], comp[fam]["write"]
            d["compulsory_read_gib"] = round(cr / 2 ** 30, 3)
            d["compulsory_write_gib"] = round(cw / 2 ** 30, 3)
            if rd is not None and cr > 0:
                d["read_over_compulsory"] = round(rd / cr, 3)
            if wr is not None and cw > 0:
                d["write_over_compulsory"] = round(wr / cw, 3)
        d["dispatches_per_pass"] = len(disp[fam]) // max(1, len({f for f, _ in disp[fam]}))
        out[fam] = d
    out["note"] = ("rocprofv3 --pmc, one counter group per bench run (bench.py --steps S --warmup 1 "
                   "--control-plane inline --graphs 0 --prewarm-ms 0, GPUSCHED_PROFILE_MARKERS); only the "
                   "dispatches between the two marker kernels of each run (the timed epochs) are counted; kernels "
                   "are serialised under --pmc, so these are per-kernel totals, not co-run; hbm_read = FETCH_SIZE x 2 "
                   "(gfx950 calibration), compulsory bytes from the timed pods' ops (models.workloads)")
    out["timed_windows"] = {os.path.relpath(f, root): w for f, w in windows.items()}
    json.dump(out, open(os.path.join(root, "summary.json"), "w"), indent=1)
    print(json.dumps(out, indent=1))


if __name__ == "__main__":
    main(sys.argv[1])
