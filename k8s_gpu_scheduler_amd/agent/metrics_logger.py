"""Per-GPU power / utilisation / temperature logger.

Reference: `parse_smi_metrics.py` polls `nvidia-smi --query-gpu=power.draw,
utilization.gpu,temperature.gpu` every second into a DataFrame and writes `test.ods`
(TSV) on SIGINT (reference pkg/profiler/parse_smi_metrics.py:23-42; unused there).
Here the samples come from the native amd-smi sampler (`_smi`), every GPU, and the TSV
gets one row per (timestamp, gpu).

  python -m k8s_gpu_scheduler_amd.agent.metrics_logger --out metrics.tsv --period 1
"""
from __future__ import annotations

import argparse
import signal
import time
from typing import Callable, List, Optional

COLUMNS = ["ts", "gpu", "power_w", "gfx_activity", "umc_activity", "temp_c", "vram_used_mb"]


def log_metrics(sample: Callable[[], list], out: str, period_s: float = 1.0, max_samples: int = 0,
                stop: Optional[Callable[[], bool]] = None) -> int:
    rows: List[List[str]] = []
    n = 0
    while not (stop and stop()):
        ts = time.time()
        for s in sample():
            rows.append([f"{ts:.3f}", str(s.get("index", 0))] +
                        [f"{float(s.get(k, 0.0)):.2f}" for k in COLUMNS[2:]])
        n += 1
        if max_samples and n >= max_samples:
            break
        time.sleep(period_s)
    with open(out, "w") as f:
        f.write("\t".join(COLUMNS) + "\n")
        for r in rows:
            f.write("\t".join(r) + "\n")
    return len(rows)


def main(argv: Optional[List[str]] = None) -> int:
    ap = argparse.ArgumentParser()
    ap.add_argument("--out", default="metrics.tsv")
    ap.add_argument("--period", type=float, default=1.0)
    ap.add_argument("--samples", type=int, default=0)
    a = ap.parse_args(argv)
    from .devices import SmiSource
    src = SmiSource()
    flag = {"stop": False}
    signal.signal(signal.SIGINT, lambda *x: flag.__setitem__("stop", True))
    n = log_metrics(src.samples, a.out, a.period, a.samples, lambda: flag["stop"])
    print(f"wrote {n} rows to {a.out}")
    return 0


if __name__ == "__main__":
    raise SystemExit(main())
