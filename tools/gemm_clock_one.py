"""One process, two GEMMs of one shape: the own lone-GEMM kernel (tile 10) and torch.matmul
(hipBLASLt), each `reps` times -- the profiling target for a per-dispatch clock / MFMA-busy
comparison (rocprofv3 --pmc GRBM_GUI_ACTIVE ... --kernel-trace: clock = GRBM_GUI_ACTIVE / 8 XCDs
/ kernel duration)."""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402

from k8s_gpu_scheduler_amd import _native  # noqa: E402
from k8s_gpu_scheduler_amd.ops import loadgen  # noqa: E402

M, N, K, tile, reps = (int(x) for x in (sys.argv[1:6] if len(sys.argv) > 5 else (8192, 8192, 8192, 10, 10)))
_native.hip().set_gemm_tile(tile)
a = (torch.rand(M, K, device="cuda") * 2 - 1).to(torch.bfloat16)
bt = (torch.rand(N, K, device="cuda") * 2 - 1).to(torch.bfloat16)
c = torch.empty(M, N, device="cuda", dtype=torch.bfloat16)
for _ in range(reps):
    loadgen.gemm(a, bt, out=c)
torch.cuda.synchronize()
for _ in range(reps):
    torch.matmul(a, bt.t(), out=c)
torch.cuda.synchronize()
print("done", M, N, K, tile)
