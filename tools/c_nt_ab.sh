#!/bin/bash
# Non-temporal GEMM output stores (set_c_nontemporal / --c-nt): bit-exact check vs plain stores,
# lone + co-run GEMM mix (+ big lone shapes), bench interleaved at the driver's shape.
cd "${GRAFT_REPO_ROOT:-.}"
mkdir -p gpurun_out/cnt
timeout -k 10 120 python - > gpurun_out/cnt/check.log 2>&1 <<'PY' || exit $?
import torch
from k8s_gpu_scheduler_amd import _native
from k8s_gpu_scheduler_amd.ops import loadgen
h = _native.hip(required=True)
for M, N, K in ((4096, 2560, 2560), (1024, 2048, 1024), (8192, 8192, 2048)):
    a = (torch.rand(M, K, device="cuda") * 2 - 1).to(torch.bfloat16)
    bt = (torch.rand(N, K, device="cuda") * 2 - 1).to(torch.bfloat16)
    b = torch.randn(N, device="cuda")
    h.set_c_nontemporal(0)
    c0 = loadgen.gemm(a, bt, bias=b, relu=True)
    h.set_c_nontemporal(1)
    c1 = loadgen.gemm(a, bt, bias=b, relu=True)
    torch.cuda.synchronize()
    assert torch.equal(c0, c1), (M, N, K)
h.set_c_nontemporal(0)
print("nt C stores bit-exact")
PY
cat gpurun_out/cnt/check.log
timeout -k 10 400 python -u tools/gemm_knob_mix.py set_c_nontemporal big > gpurun_out/cnt/mix.log 2>&1 || exit $?
cat gpurun_out/cnt/mix.log
for i in 1 2 3; do
  for x in 0 1; do
    timeout -k 10 200 python bench.py --steps 20 --warmup 5 --c-nt $x > gpurun_out/cnt/b_${x}_${i}.log 2>&1 || exit $?
    echo "c_nt=$x run=$i $(grep '^{' gpurun_out/cnt/b_${x}_${i}.log | python -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["value"], d["ms_per_step"], d["achieved_tflops"], d.get("slo_attainment_pct"))')"
  done
done
