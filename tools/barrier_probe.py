"""How much do the 8-phase GEMM's barriers cost?  Times the production steady-state loop
(mode 0, same code as tile 10) against a copy with half of its barriers removed (mode 1 --
racy, wrong results by design, timing only) on lone 4096^3 / 8192^3 GEMMs.  Builds
tools/hip/barrier_probe.hip into a throwaway .so under /tmp.  Writes gpurun_out/barrier_probe.json."""
import ctypes
import json
import os
import subprocess
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

import torch  # noqa: E402

HERE = os.path.dirname(os.path.abspath(__file__))


def build(so):
    src = os.path.join(HERE, "hip", "barrier_probe.hip")
    subprocess.run(["/opt/rocm/bin/hipcc", "--offload-arch=gfx950", "-O3", "-std=c++17", "-shared", "-fPIC",
                    f"-I{os.path.join(HERE, '..', 'native', 'hip')}", "-I/usr/include/python3.10",
                    f"-I{__import__('pybind11').get_include()}", src, "-o", so], check=True)


def main():
    so = os.path.join(HERE, "hip", "barrier_probe.so")
    if not os.path.exists(so):
        build(so)
    lib = ctypes.CDLL(so)
    lib.probe_launch.argtypes = [ctypes.c_int, ctypes.c_void_p, ctypes.c_void_p, ctypes.c_void_p, ctypes.c_int,
                                 ctypes.c_int, ctypes.c_int, ctypes.c_void_p]
    out = {}
    for (M, N, K) in [(4096, 4096, 4096), (8192, 8192, 8192), (8192, 8192, 2048)]:
        a = (torch.rand(M, K, device="cuda") * 2 - 1).to(torch.bfloat16)
        bt = (torch.rand(N, K, device="cuda") * 2 - 1).to(torch.bfloat16)
        c = torch.empty(M, N, device="cuda", dtype=torch.bfloat16)
        st = torch.cuda.current_stream().cuda_stream
        res = {0: [], 1: []}
        for _ in range(3):
            for mode in (0, 1):
                for _ in range(3):
                    assert lib.probe_launch(mode, a.data_ptr(), bt.data_ptr(), c.data_ptr(), M, N, K, st) == 0
                torch.cuda.synchronize()
                e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
                e0.record()
                for _ in range(20):
                    lib.probe_launch(mode, a.data_ptr(), bt.data_ptr(), c.data_ptr(), M, N, K, st)
                e1.record()
                torch.cuda.synchronize()
                res[mode].append(round(2 * M * N * K / (e0.elapsed_time(e1) / 20) / 1e9, 1))
        row = {"tile10_tflops": sorted(res[0])[1], "half_barriers_tflops": sorted(res[1])[1]}
        out[f"{M}x{N}x{K}"] = row
        print(M, N, K, row, flush=True)
    os.makedirs("gpurun_out", exist_ok=True)
    json.dump(out, open("gpurun_out/barrier_probe.json", "w"), indent=1)


if __name__ == "__main__":
    main()
