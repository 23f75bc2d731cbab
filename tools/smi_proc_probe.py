"""What amd-smi's per-process list reports for a BUSY process on this box (VERDICT r5 item 3:
a millisecond busy-time producer for the completion feedback).

A child runs back-to-back bf16 GEMMs for ~3 s (HIP-event timed, so its true GPU busy ms is
known); the parent samples `processes()` every 0.1 s and records every field of the child's
entry (the child appears under its HOST pid, found as the pid new to the list).  Writes
gpurun_out/smi_proc_probe.json."""
from __future__ import annotations

import json
import os
import subprocess
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

CHILD = r"""
import sys, time, torch
sys.path.insert(0, %r)
from k8s_gpu_scheduler_amd.ops import loadgen
a = torch.rand(4096, 4096, device='cuda').to(torch.bfloat16); bt = torch.rand(4096, 4096, device='cuda').to(torch.bfloat16)
c = torch.empty(4096, 4096, device='cuda', dtype=torch.bfloat16)
loadgen.gemm(a, bt, out=c); torch.cuda.synchronize()
print('ready', flush=True)
e0 = torch.cuda.Event(enable_timing=True); e1 = torch.cuda.Event(enable_timing=True)
e0.record(); t0 = time.time()
while time.time() - t0 < 3.0:
    for _ in range(32):
        loadgen.gemm(a, bt, out=c)
    torch.cuda.synchronize()
e1.record(); torch.cuda.synchronize()
print('busy_ms', e0.elapsed_time(e1), flush=True)
time.sleep(1.0)
"""


def main() -> None:
    from k8s_gpu_scheduler_amd.agent.devices import SmiSource
    src = SmiSource()
    n = len(src.devices())

    def procs():
        return [dict(p, dev=i) for i in range(n) for p in src.processes(i)]
    before = {p["pid"] for p in procs()}
    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    child = subprocess.Popen([sys.executable, "-c", CHILD % root], stdout=subprocess.PIPE, text=True)
    samples = []
    assert "ready" in child.stdout.readline()
    t0 = time.time()
    while child.poll() is None and time.time() - t0 < 20:
        now = time.time() - t0
        for p in procs():
            if p["pid"] not in before:
                samples.append(dict(p, t=round(now, 3)))
        time.sleep(0.1)
    out = child.stdout.read()
    busy = [float(x.split()[1]) for x in out.splitlines() if x.startswith("busy_ms")]
    os.makedirs("gpurun_out", exist_ok=True)
    res = {"child_busy_ms": busy[0] if busy else None, "samples": samples,
           "gfx_ns_max": max((s.get("gfx_ns", 0) for s in samples), default=0),
           "cu_occupancy_max": max((s.get("cu_occupancy", 0) for s in samples), default=0)}
    json.dump(res, open("gpurun_out/smi_proc_probe.json", "w"), indent=1, default=str)
    print(json.dumps({k: v for k, v in res.items() if k != "samples"}), "samples", len(samples), flush=True)


if __name__ == "__main__":
    main()
