"""What a container sees of the GPU: the devices the ROCm runtime enumerates under the
pod's env (ROCR_VISIBLE_DEVICES / HIP_VISIBLE_DEVICES) and the CUs its kernels actually run
on (HSA_CU_MASK).  The default command of `agent.launcher.PodLauncher` -- the in-container
check of SURVEY §7.4 ("the pod saw exactly the one assigned device").

  python -m k8s_gpu_scheduler_amd.agent.container_probe [--work N]   -> one JSON line on stdout
"""
from __future__ import annotations

import json
import os
import sys


def probe(blocks: int = 4096) -> dict:
    from .. import _native
    h = _native.hip(required=True)
    out = {"env": {k: os.environ.get(k, "") for k in ("ROCR_VISIBLE_DEVICES", "HIP_VISIBLE_DEVICES",
                                                        "HSA_CU_MASK", "CUDA_VISIBLE_DEVICES",
                                                        "GPU_SCHED_HBM_LIMIT_GIB")}}
    devs = h.query_all()
    out["count"] = len(devs)
    out["devices"] = [{"rocr_uuid": d.get("rocr_uuid", ""), "pci": d.get("pci", ""), "cus": d["cus"]} for d in devs]
    if devs:
        s = h.create_stream(0)
        try:
            raw = h.probe_xcd(s, blocks)
        finally:
            h.destroy_stream(s)
        slots = set()
        per_xcc: dict = {}
        for i in range(blocks):
            xcc, hw = raw[2 * i] & 0xF, raw[2 * i + 1]
            slot = (xcc, (hw >> 13) & 0x7, (hw >> 12) & 0x1, (hw >> 8) & 0xF)
            slots.add(slot)
            per_xcc.setdefault(xcc, set()).add(slot)
        out["cus_used"] = len(slots)
        out["cus_per_xcc"] = {str(k): len(v) for k, v in sorted(per_xcc.items())}
    return out


def work(iters: int) -> dict:
    """A little real load (MFMA GEMM + HBM stream) so a profiled pod has kernels to trace."""
    import torch
    from ..ops import loadgen
    # operands generated on the host: device-side RNG kernels (hiprand, shipped with the torch
    # wheel's ROCm) crashed under the system rocprofv3's kernel tracer on the box
    g = torch.Generator().manual_seed(0)
    a = (torch.rand(2048, 2048, generator=g) - 0.5).to(torch.bfloat16).cuda()
    bt = (torch.rand(2048, 2048, generator=g) - 0.5).to(torch.bfloat16).cuda()
    x, y, z = (torch.ones(1 << 22).cuda() for _ in range(3))
    for _ in range(iters):
        loadgen.gemm(a, bt, relu=True)
        loadgen.triad(x, y, z, 1.5)
    torch.cuda.synchronize()
    return {"work_iters": iters}


def main() -> int:
    try:
        out = probe()
        n = int(sys.argv[sys.argv.index("--work") + 1]) if "--work" in sys.argv else 0
        if n > 0:
            out.update(work(n))
        print(json.dumps(out), flush=True)
        return 0
    except Exception as e:  # report, do not crash silently
        print(json.dumps({"error": str(e)}), flush=True)
        return 1


if __name__ == "__main__":
    sys.exit(main())
