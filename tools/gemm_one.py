"""Run one GEMM shape/tile repeatedly (profiling target for rocprofv3 --pmc)."""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402

from k8s_gpu_scheduler_amd import _native  # noqa: E402
from k8s_gpu_scheduler_amd.ops import loadgen  # noqa: E402

M, N, K, tile, reps = (int(x) for x in (sys.argv[1:6] if len(sys.argv) > 5 else (4096, 2048, 2048, 1, 20)))
_native.hip().set_gemm_tile(tile)
a = (torch.rand(M, K, device="cuda") * 2 - 1).to(torch.bfloat16)
bt = (torch.rand(N, K, device="cuda") * 2 - 1).to(torch.bfloat16)
c = torch.empty(M, N, device="cuda", dtype=torch.bfloat16)
bias = torch.zeros(N, device="cuda")
for _ in range(reps):
    loadgen.gemm(a, bt, out=c, bias=bias, relu=True)
torch.cuda.synchronize()
print("done", M, N, K, tile)
