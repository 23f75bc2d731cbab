"""The pod-arrival benchmark and its distributed path on CPU (gloo, simulated executor).

The driver runs `bench.py` under torch.distributed.run with one rank per GPU; here the
same code path runs with world_size 2 on gloo so placement broadcast, telemetry
all-gather and the max-over-ranks timing are exercised without a GPU.
"""
import json
import os
import subprocess
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def test_bench_sim_single_process():
    from k8s_gpu_scheduler_amd.parallel.podbench import main
    r = main(["--sim", "--gpus", "4", "--steps", "3", "--warmup", "1"])
    assert r["n_gpus"] == 4 and r["config"]["global_batch"] == 16 and r["unscheduled"] == 0
    assert r["value"] > 0 and r["simulated"] is True
    for k in ("metric", "value", "unit", "n_gpus", "steps", "warmup", "ms_per_step", "higher_is_better",
              "scaling", "vs_baseline", "dtype", "data", "config"):
        assert k in r
    # speed-of-light bookkeeping: the floor at the hardware peaks is below the floor at the
    # measured-best rates, and both are positive for a run that did work
    floor = r["roofline_floor_ms_per_step"]
    assert 0 < floor["peak"] <= floor["achievable"]
    assert r["sol_pct"]["peak"] <= r["sol_pct"]["achievable"] and r["achieved_hbm_tbps_per_gpu"] > 0


def test_bench_pinned_effort_level_is_recorded_and_held():
    """--plan-effort pins the planner's level (the simulated bench never adapts): the JSON's
    config records the level and that adaptation was off, and every epoch ran at that level."""
    from k8s_gpu_scheduler_amd.parallel.podbench import main
    r = main(["--sim", "--gpus", "2", "--steps", "3", "--warmup", "1", "--plan-effort", "2"])
    assert r["config"]["plan_effort"] == 2 and r["config"]["cp_adaptive"] == 0
    assert "cp_effort_down" not in r["config"]
    assert set(r["planner"]["effort_epochs"]) == {"2"} and r["planner"]["slot_policy"] == "lpt"


def test_bench_random_policy_runs():
    from k8s_gpu_scheduler_amd.parallel.podbench import main
    r = main(["--sim", "--gpus", "2", "--steps", "2", "--warmup", "1", "--policy", "random"])
    assert r["config"]["policy"] == "random" and r["unscheduled"] == 0


@pytest.mark.slow
def test_bench_two_ranks_gloo(tmp_path):
    out = tmp_path / "r.json"
    env = dict(os.environ, CUDA_VISIBLE_DEVICES="", HIP_VISIBLE_DEVICES="")
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", "--nproc-per-node=2",
           "--master-addr", "127.0.0.1", "--master-port", "29611", os.path.join(ROOT, "bench.py"),
           "--sim", "--gpus", "2", "--steps", "3", "--warmup", "1", "--out", str(out)]
    p = subprocess.run(cmd, capture_output=True, text=True, timeout=300, env=env, cwd=ROOT)
    assert p.returncode == 0, p.stderr[-3000:]
    lines = [l for l in p.stdout.splitlines() if l.startswith("{")]
    assert len(lines) == 1                        # rank 0 prints exactly one JSON line
    r = json.loads(lines[0])
    assert r["n_gpus"] == 2 and r["config"]["parallelism"] == "dp2" and r["config"]["global_batch"] == 8
    assert json.loads(out.read_text())["value"] == r["value"]


def test_resize_loop_clears_backlog_sim():
    """Config 5 (simulated executor): with the admission loop the over-requested pods are
    shrunk to what their SLO needs, so the backlog that builds without it disappears."""
    from k8s_gpu_scheduler_amd.parallel import resize_loop
    on = resize_loop.run(n_gpus=2, epochs=15, rate=3.0, sim=True, resize=True)
    off = resize_loop.run(n_gpus=2, epochs=15, rate=3.0, sim=True, resize=False)
    assert on["created"] == off["created"]
    assert on["completed"] > off["completed"] and on["final_backlog"] < off["final_backlog"]
    assert on["mean_cu_request_placed"] < 128 and on["admission"]["resized"] > 0
    # the history the admission resized from was written by the node agent's per-process path
    assert on["history"]["samples"] == on["completed"]


def test_dead_control_plane_raises_instead_of_hanging():
    """A crashed control-plane process must fail the bench (torchrun then stops every
    rank), never leave rank 0 blocked at the next schedule forever."""
    from k8s_gpu_scheduler_amd.parallel.controlplane_proc import ControlPlaneProc
    cp = ControlPlaneProc(n_gpus=1, pods_per_gpu=2, iters=2, seed=0)
    try:
        assert cp.schedule_epoch().shape == (2, 8)
        cp.request_schedule()
        cp._p.kill()
        cp._p.join()
        with pytest.raises((RuntimeError, OSError)):
            # the child may have answered the request before the kill landed: that
            # buffered reply is returned once, the next read must then raise
            cp.get_schedule()
            cp.get_schedule()
        with pytest.raises((RuntimeError, OSError)):
            cp.schedule_epoch()
    finally:
        cp._outstanding = 0
        cp.close()


def _bench(args, timeout=300):
    env = dict(os.environ, CUDA_VISIBLE_DEVICES="", HIP_VISIBLE_DEVICES="")
    for k in ("WORLD_SIZE", "RANK", "LOCAL_RANK", "MASTER_ADDR", "MASTER_PORT"):
        env.pop(k, None)
    return subprocess.run([sys.executable, os.path.join(ROOT, "bench.py"), *args], capture_output=True, text=True,
                          timeout=timeout, env=env, cwd=ROOT)


def test_bench_sim_gpus4_without_torchrun_reports_4():
    """`python bench.py --sim --gpus 4` (no torchrun): N simulated GPUs, one JSON line."""
    p = _bench(["--sim", "--gpus", "4", "--steps", "2", "--warmup", "1"])
    assert p.returncode == 0, p.stderr[-3000:]
    lines = [l for l in p.stdout.splitlines() if l.startswith("{")]
    assert len(lines) == 1
    r = json.loads(lines[0])
    assert r["n_gpus"] == 4 and r["config"]["parallelism"] == "dp4"


@pytest.mark.slow
def test_bench_self_launches_one_process_per_rank():
    """`--launch spawn` without torchrun: the parent starts N rank processes itself (here
    gloo ranks of the simulated executor) -- the path `bench.py --gpus N` takes on a GPU
    host, where the parent never touches the GPU."""
    p = _bench(["--sim", "--launch", "spawn", "--gpus", "2", "--steps", "2", "--warmup", "1"])
    assert p.returncode == 0, p.stderr[-3000:]
    lines = [l for l in p.stdout.splitlines() if l.startswith("{")]
    assert len(lines) == 1                        # only rank 0 prints
    r = json.loads(lines[0])
    assert r["n_gpus"] == 2 and r["config"]["parallelism"] == "dp2" and r["config"]["global_batch"] == 8


def test_bench_more_gpus_than_visible_fails_fast():
    """No silent clamp: asking for 2 GPUs on a host with fewer fails with rc != 0."""
    import time
    t = time.time()
    p = _bench(["--gpus", "2", "--steps", "1", "--warmup", "0"], timeout=120)
    assert p.returncode != 0
    assert "GPU" in p.stderr and not [l for l in p.stdout.splitlines() if l.startswith("{")]
    assert time.time() - t < 60


def test_launcher_propagates_rank_failure():
    from k8s_gpu_scheduler_amd.parallel.launch import spawn
    code = "import os,sys,time; r=int(os.environ['RANK']); time.sleep(0.2*r); sys.exit(3 if r==1 else 0)"
    assert spawn([sys.executable, "-c", code], 2, require_gpus=False) == 3
    code = ("import os; assert os.environ['WORLD_SIZE']=='3' and os.environ['MASTER_ADDR']=='127.0.0.1'; "
            "assert os.environ['RANK']==os.environ['LOCAL_RANK']")
    assert spawn([sys.executable, "-c", code], 3, require_gpus=False) == 0


def test_bench_dist_single_takes_the_collective_path():
    """--dist-single: a 1-rank process group runs the multi-rank collective code (broadcast,
    all-gather, all-reduce, barriers) -- on a 1-GPU box that is the RCCL path of the scaling run."""
    from k8s_gpu_scheduler_amd.parallel.podbench import main
    import torch.distributed as dist
    r = main(["--sim", "--dist-single", "1", "--steps", "3", "--warmup", "1", "--control-plane", "inline"])
    assert r["n_gpus"] == 1 and r["value"] > 0 and r["unscheduled"] == 0
    assert not dist.is_initialized() and "WORLD_SIZE" not in os.environ
    with pytest.raises(SystemExit):
        main(["--sim", "--dist-single", "1", "--gpus", "2", "--steps", "1", "--warmup", "0"])


@pytest.mark.gpu
def test_bench_rccl_collective_path_on_gpu(tmp_path):
    """The scaling run's collective code over RCCL on one MI355X: bench.py --dist-single runs a
    1-rank nccl group (placement broadcast on the side stream, telemetry all-gather, result
    all-reduce / all-gather, barriers, destroy) through the real HIP executor."""
    out = tmp_path / "b.json"
    env = dict(os.environ)
    env.pop("WORLD_SIZE", None)
    p = subprocess.run([sys.executable, os.path.join(ROOT, "bench.py"), "--dist-single", "1", "--steps", "5",
                        "--warmup", "2", "--out", str(out)], env=env, capture_output=True, text=True, timeout=240)
    assert p.returncode == 0, p.stderr[-2000:]
    r = json.loads(out.read_text())
    assert r["n_gpus"] == 1 and r["simulated"] is False and r["value"] > 0 and r["unscheduled"] == 0
