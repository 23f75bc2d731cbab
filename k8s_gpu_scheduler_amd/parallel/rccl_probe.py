"""RCCL-over-xGMI placement probe (BASELINE config 4: validate that a multi-GPU pod's
GPU set gives its collectives full Infinity Fabric bandwidth).

The reference never places multi-GPU pods.  The topology Filter picks
an xGMI clique; this probe measures it: run under torch.distributed (backend "nccl" =
RCCL on ROCm), one rank per GPU of the candidate set, and time all-reduce / all-gather /
reduce-scatter over a size sweep.  Reported bus bandwidth follows the nccl-tests
convention (all-reduce busbw = algbw * 2(n-1)/n); on an 8xMI355X node one ring is bound
by a single ~153 GB/s xGMI link per direction, and RCCL's multi-channel rings spread a
k-GPU set over k-1 links per GPU.

  python -m k8s_gpu_scheduler_amd.parallel.rccl_probe --gpus 4 --sizes 1M,64M,512M
  (or under torchrun --nproc-per-node 4; --gpus N outside torchrun spawns the N ranks)
"""
from __future__ import annotations

import argparse
import json
import os
import sys
import time
from typing import Dict, List, Optional

import torch
import torch.distributed as dist


def _parse_size(s: str) -> int:
    s = s.strip().upper()
    mult = {"K": 1 << 10, "M": 1 << 20, "G": 1 << 30}
    return int(float(s[:-1]) * mult[s[-1]]) if s[-1] in mult else int(s)


def bus_factor(op: str, n: int) -> float:
    if n <= 1:
        return 1.0
    return {"all_reduce": 2.0 * (n - 1) / n, "all_gather": (n - 1) / n,
            "reduce_scatter": (n - 1) / n}[op]


def probe(sizes: List[int], ops=("all_reduce", "all_gather", "reduce_scatter"), iters: int = 20,
          warmup: int = 5, group=None) -> List[Dict[str, float]]:
    n = dist.get_world_size(group)
    dev = torch.device("cuda", torch.cuda.current_device())
    out = []
    for nbytes in sizes:
        numel = max(n, nbytes // 2 // n * n)            # bf16 elements, divisible by n
        x = torch.ones(numel, dtype=torch.bfloat16, device=dev)
        shard = torch.empty(numel // n, dtype=torch.bfloat16, device=dev)
        for op in ops:
            def run():
                if op == "all_reduce":
                    dist.all_reduce(x, group=group)
                elif op == "all_gather":
                    dist.all_gather_into_tensor(x, shard, group=group)
                else:
                    dist.reduce_scatter_tensor(shard, x, group=group)
            for _ in range(warmup):
                run()
            torch.cuda.synchronize()
            dist.barrier(group=group)
            t0 = time.perf_counter()
            for _ in range(iters):
                run()
            torch.cuda.synchronize()
            dt = (time.perf_counter() - t0) / iters
            t = torch.tensor([dt], device=dev)
            dist.all_reduce(t, op=dist.ReduceOp.MAX, group=group)
            dt = float(t)
            algbw = numel * 2 / dt / 1e9
            out.append({"op": op, "bytes": numel * 2, "n": n, "time_us": dt * 1e6, "algbw_gbps": algbw,
                        "busbw_gbps": algbw * bus_factor(op, n)})
    return out


def main(argv: Optional[List[str]] = None) -> int:
    ap = argparse.ArgumentParser()
    ap.add_argument("--sizes", default="1M,16M,256M")
    ap.add_argument("--iters", type=int, default=20)
    ap.add_argument("--gpus", type=int, default=1,
                    help="ranks (one per GPU); outside torchrun the probe spawns them itself")
    ap.add_argument("--ops", default="all_reduce,all_gather,reduce_scatter")
    ap.add_argument("--out", default="")
    a = ap.parse_args(argv)
    if "WORLD_SIZE" not in os.environ and a.gpus > 1:
        from .launch import self_launch_module
        return self_launch_module(__name__ if __name__ != "__main__" else "k8s_gpu_scheduler_amd.parallel.rccl_probe",
                                  list(argv if argv is not None else sys.argv[1:]), a.gpus)
    world = int(os.environ.get("WORLD_SIZE", "1"))
    if world > 1 and torch.cuda.device_count() < world:
        raise SystemExit(f"WORLD_SIZE {world} but only {torch.cuda.device_count()} GPU(s) visible")
    local = int(os.environ.get("LOCAL_RANK", "0"))
    torch.cuda.set_device(local)
    if not dist.is_initialized():
        if "WORLD_SIZE" not in os.environ:
            os.environ.update({"WORLD_SIZE": "1", "RANK": "0", "MASTER_ADDR": "127.0.0.1",
                               "MASTER_PORT": os.environ.get("MASTER_PORT", "29581")})
        dist.init_process_group("nccl", device_id=torch.device("cuda", local))
    res = probe([_parse_size(s) for s in a.sizes.split(",")], ops=tuple(o for o in a.ops.split(",") if o),
                iters=a.iters)
    if dist.get_rank() == 0:
        txt = json.dumps({"world": dist.get_world_size(), "results": res})
        print(txt, flush=True)
        if a.out:
            with open(a.out, "w") as f:
                f.write(txt)
    dist.destroy_process_group()
    return 0


if __name__ == "__main__":
    raise SystemExit(main())
