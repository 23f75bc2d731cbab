"""Aggregate tools/gpu_pmc_bench.sh's rocprofv3 counter CSVs per kernel family: dispatches,
MFMA-busy share, HBM bytes read / written (FETCH_SIZE / WRITE_SIZE, KiB), next to the bytes the
speed-of-light model charges those kernels (models.workloads.Op.bytes).  Writes summary.json."""
import csv
import glob
import json
import os
import sys
from collections import defaultdict


def family(name: str) -> str:
    if "256_8ph" in name:
        return "gemm_256x256_8phase"
    if "gemm_bf16_nt_kernel" in name:
        return "gemm_tile_" + name.split("<", 1)[1].split(",")[0] + "x" + name.split(",")[1].strip()
    if "stream_triad" in name:
        return "stream_triad"
    return "other"


def main(root: str) -> None:
    agg = defaultdict(lambda: defaultdict(float))
    disp = defaultdict(set)
    for f in glob.glob(os.path.join(root, "p*", "**", "*counter_collection.csv"), recursive=True):
        with open(f) as fh:
            for row in csv.DictReader(fh):
                fam = family(row.get("Kernel_Name", ""))
                agg[fam][row["Counter_Name"]] += float(row["Counter_Value"])
                disp[fam].add((f, row.get("Dispatch_Id")))
    out = {}
    for fam, c in sorted(agg.items()):
        d = {"counters": {k: round(v, 1) for k, v in c.items()}}
        if c.get("GRBM_GUI_ACTIVE") and c.get("SQ_VALU_MFMA_BUSY_CYCLES") is not None and c.get("SQ_BUSY_CU_CYCLES"):
            # MFMA busy per SIMD cycle of the CUs that were busy
            d["mfma_busy_of_busy_cu_pct"] = round(100 * c["SQ_VALU_MFMA_BUSY_CYCLES"] / (4 * c["SQ_BUSY_CU_CYCLES"]), 1)
        if "FETCH_SIZE" in c:
            d["hbm_read_gib"] = round(c["FETCH_SIZE"] * 1024 / 2 ** 30, 2)
        if "WRITE_SIZE" in c:
            d["hbm_write_gib"] = round(c["WRITE_SIZE"] * 1024 / 2 ** 30, 2)
        out[fam] = d
    out["note"] = ("rocprofv3 --pmc per counter group in its own bench run (bench.py --steps 4 --warmup 1 "
                   "--control-plane inline --graphs 0 --prewarm-ms 0); kernels serialised under --pmc")
    json.dump(out, open(os.path.join(root, "summary.json"), "w"), indent=1)
    print(json.dumps(out, indent=1))


if __name__ == "__main__":
    main(sys.argv[1])
