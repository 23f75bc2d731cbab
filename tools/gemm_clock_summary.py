"""Summarise tools/gpu_gemm_clock.sh: per GEMM kernel, median duration, clock (GRBM_GUI_ACTIVE
/ 8 XCDs / duration), MFMA busy per SIMD-cycle, LDS instructions, wait fractions."""
import csv
import json
import statistics as st
import sys
from collections import defaultdict

D = sys.argv[1] if len(sys.argv) > 1 else "gpurun_out/clk"
SHAPE = [int(x) for x in sys.argv[2:5]] if len(sys.argv) > 4 else [8192, 8192, 8192]


def kind(name):
    if "gemm_bf16_nt_256_8ph" in name:
        return "own_tile10"
    if "gemm_bf16_nt_256_4w" in name:
        return "own_4wave"
    if "Cijk" in name:
        return "hipblaslt"
    return None


out = defaultdict(lambda: defaultdict(list))
for pas in ("a", "b"):
    for r in csv.DictReader(open(f"{D}/{pas}/run_counter_collection.csv")):
        k = kind(r["Kernel_Name"])
        if k:
            dur = (int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) * 1e-9
            out[k][r["Counter_Name"]].append(float(r["Counter_Value"]))
            out[k]["_dur_" + pas + r["Counter_Name"]].append(dur)
dur = defaultdict(list)
for r in csv.DictReader(open(f"{D}/t/run_kernel_trace.csv")):
    k = kind(r["Kernel_Name"])
    if k:
        dur[k].append((int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) * 1e-9)
flop = 2.0 * SHAPE[0] * SHAPE[1] * SHAPE[2]
res = {}
for k, c in out.items():
    med = {n: st.median(v) for n, v in c.items() if not n.startswith("_dur")}
    d_a = st.median(c["_dur_aGRBM_GUI_ACTIVE"])
    t = st.median(dur[k])
    res[k] = {
        "median_us_trace": round(t * 1e6, 1),
        "tflops_trace": round(flop / t / 1e12, 1),
        "clock_ghz_pmc_run": round(med["GRBM_GUI_ACTIVE"] / 8 / d_a / 1e9, 3),
        "mfma_busy_per_simd": round(med["SQ_VALU_MFMA_BUSY_CYCLES"] / (1024 * med["GRBM_GUI_ACTIVE"] / 8), 3),
        "busy_cu_frac": round(med["SQ_BUSY_CU_CYCLES"] / (256 * med["GRBM_GUI_ACTIVE"] / 8), 3),
        "insts_lds": med["SQ_INSTS_LDS"],
        "lds_bank_conflict": med.get("SQ_LDS_BANK_CONFLICT"),
        "wait_any_frac": round(med["SQ_WAIT_ANY"] / med["SQ_WAVE_CYCLES"], 3),
        "wait_lds_frac": round(med["SQ_WAIT_INST_LDS"] / med["SQ_WAVE_CYCLES"], 3),
        "wave_cycles": med["SQ_WAVE_CYCLES"],
        "raw": med,
    }
print(json.dumps({"shape": SHAPE, "kernels": res}, indent=1))
