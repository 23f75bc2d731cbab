#!/bin/bash
# Round 6: the 4-wave GEMM with its odd waves issuing LDS-DMA in the odd MFMA groups (--w4-parity):
# numerics, lone timing next to the default placement, 3 interleaved bench rounds.
cd "${GRAFT_REPO_ROOT:-.}"
O=gpurun_out/r06_parity; mkdir -p $O
timeout -k 10 120 python3 -u -c "
import torch
from k8s_gpu_scheduler_amd import _native
from k8s_gpu_scheduler_amd.ops import loadgen
h = _native.hip(required=True)
h.set_w4_parity(1)
for (M, N, K) in [(256, 256, 128), (512, 768, 320), (2048, 2048, 4096), (4096, 4096, 640)]:
    a = (torch.rand(M, K, device='cuda') * 2 - 1).to(torch.bfloat16)
    bt = (torch.rand(N, K, device='cuda') * 2 - 1).to(torch.bfloat16)
    b = torch.randn(N, device='cuda')
    ref = torch.relu(a.float() @ bt.float().T + b)
    for budget in (0, 64):
        h.set_gemm_tile(14 if budget == 0 else 0)
        for _ in range(3):
            out = loadgen.gemm(a, bt, bias=b, relu=True, cu_budget=budget)
            err = (out.float() - ref).abs().max().item()
            assert err <= 0.01 * ref.abs().max().item() + 1e-2, (M, N, K, budget, err)
        print(M, N, K, budget, err, flush=True)
h.set_gemm_tile(0); h.set_w4_parity(0)
print('numerics ok')
" > $O/numerics.log 2>&1 || exit $?
timeout -k 10 200 python3 -u tools/gemm_w4_probe.py 8192 8192 8192 30 > $O/probe.log 2>&1 || exit $?
for r in 1 2 3; do
  for pa in 1 0; do
    timeout -k 10 150 python3 bench.py --steps 20 --warmup 5 --w4-parity $pa > $O/b_pa${pa}_r$r.json 2> $O/b_pa${pa}_r$r.err || exit $?
  done
done
echo done
