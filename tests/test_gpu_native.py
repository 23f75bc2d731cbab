"""Native HIP layer on a real MI355X (run with `-m gpu` on the box).

Numerics of every HIP kernel are checked against a plain PyTorch fp32 reference of the
same op.  The HIP module is loaded unconditionally (no fallback): if it is missing these
tests fail loudly.
"""
import json
import os

import pytest
import torch

pytestmark = pytest.mark.gpu
OUT = os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "gpurun_out")


@pytest.fixture(scope="module")
def hip():
    from k8s_gpu_scheduler_amd import _native
    return _native.hip(required=True)


def test_device_query(hip):
    devs = hip.query_all()
    assert devs and devs[0]["arch"].startswith("gfx950")
    assert devs[0]["cus"] == 256 and devs[0]["total_mem"] > 250 * 2**30 and devs[0]["warp"] == 64


@pytest.mark.parametrize("M,N,K,relu,bias", [(128, 128, 64, False, False), (256, 384, 192, True, True),
                                             (1024, 2048, 2048, True, False), (2048, 1024, 4096, False, True)])
def test_gemm_matches_fp32_reference(M, N, K, relu, bias):
    from k8s_gpu_scheduler_amd.ops import loadgen
    g = torch.Generator(device="cuda").manual_seed(M + N + K)
    a = torch.randn(M, K, device="cuda", generator=g).to(torch.bfloat16)
    bt = torch.randn(N, K, device="cuda", generator=g).to(torch.bfloat16)
    b = torch.randn(N, device="cuda", generator=g) if bias else None
    out = loadgen.gemm(a, bt, bias=b, relu=relu)
    ref = a.float() @ bt.float().T + (b if bias else 0)
    if relu:
        ref = torch.relu(ref)
    err = (out.float() - ref).abs().max().item()
    assert err <= 0.01 * ref.abs().max().item() + 1e-2, err


@pytest.mark.parametrize("tile", [1, 2, 3, 4, 5, 6, 7, 8, 11, 12, 13])
def test_gemm_every_tile_variant(tile):
    from k8s_gpu_scheduler_amd import _native
    from k8s_gpu_scheduler_amd.ops import loadgen
    h = _native.hip()
    h.set_gemm_tile(tile)
    try:
        for (M, N, K) in [(256, 256, 128), (384, 640, 320), (1024, 1536, 1536), (512, 768, 2048)]:
            a = torch.randn(M, K, device="cuda").to(torch.bfloat16)
            bt = torch.randn(N, K, device="cuda").to(torch.bfloat16)
            b = torch.randn(N, device="cuda")
            out = loadgen.gemm(a, bt, bias=b, relu=True)
            ref = torch.relu(a.float() @ bt.float().T + b)
            assert (out.float() - ref).abs().max().item() <= 0.01 * ref.abs().max().item() + 1e-2
    finally:
        h.set_gemm_tile(0)


@pytest.mark.parametrize("tile", [9, 10, 11, 12, 13, 14, 15, 16])
def test_gemm_256_8phase_numerics_and_race_screen(tile):
    """The 8-phase 256x256 kernel (tile 9; tile 10 = its steady-state loop peeled), and the
    128x128 multi-stage kernels (11, 12: 3 / 4 LDS stages, counted vmcnt), and the 8-phase
    schedule on a 256x128 block (13: unequal half-tile glds counts in the waits), and the 4-wave
    kernel with AGPR-tied inline-asm MFMAs (14: 5-slot LDS ring, one barrier per K-tile; the
    accumulator fences are what keep its bias / ReLU epilogue right; 15: the same on a 256 x 128
    block, unequal A / B glds counts; 16: on a 128 x 128 block, two blocks per CU): every
    K-tile count from the minimum (2) through odd
    counts (the buffer parity flips) to long loops, several grid sizes, each shape run
    repeatedly -- a mis-counted vmcnt or a restage too early shows up as rare wrong tiles
    (guide §5 'A sync-structure edit makes a NEW template'), so every run is checked against
    an fp32 reference, and A = I with an asymmetric B pins the C layout."""
    from k8s_gpu_scheduler_amd import _native
    from k8s_gpu_scheduler_amd.ops import loadgen
    h = _native.hip()
    h.set_gemm_tile(tile)
    try:
        for (M, N, K) in [(256, 256, 64), (256, 256, 128), (256, 512, 192), (512, 256, 320), (768, 1024, 1024),
                          (512, 512, 384), (2048, 2048, 4096), (4096, 4096, 640), (1024, 512, 1088)]:
            g = torch.Generator(device="cuda").manual_seed(M * 7 + N * 3 + K)
            a = (torch.rand(M, K, device="cuda", generator=g) * 2 - 1).to(torch.bfloat16)
            bt = (torch.rand(N, K, device="cuda", generator=g) * 2 - 1).to(torch.bfloat16)
            b = torch.randn(N, device="cuda", generator=g)
            ref = torch.relu(a.float() @ bt.float().T + b)
            tol = 0.01 * ref.abs().max().item() + 1e-2
            out = torch.empty(M, N, device="cuda", dtype=torch.bfloat16)
            for _ in range(6):
                out.fill_(float("nan"))
                loadgen.gemm(a, bt, out=out, bias=b, relu=True)
                err = (out.float() - ref).abs().max().item()
                assert err <= tol, (M, N, K, err)
        n = 256
        eye = torch.eye(n, device="cuda", dtype=torch.bfloat16)
        asym = (torch.arange(n * n, device="cuda", dtype=torch.float32).reshape(n, n) % 97).to(torch.bfloat16)
        assert torch.equal(loadgen.gemm(eye, asym).float(), asym.float().T)
    finally:
        h.set_gemm_tile(0)


@pytest.mark.parametrize("M,N,K,relu,bias", [(2048, 4096, 8192, True, True), (1024, 1024, 8192, False, False),
                                             (512, 768, 4096, True, False), (256, 256, 2048, False, True)])
def test_gemm_split_k_matches_fp32_reference(hip, M, N, K, relu, bias):
    """Split-K (opt-in, set_split_k): lone GEMMs whose 256x256 tiles leave CUs idle run the 8-phase
    kernel per K slice -> fp32 partials -> reduce + bias + ReLU; repeated runs screen for
    ordering races."""
    from k8s_gpu_scheduler_amd.ops import loadgen
    hip.set_split_k(-1)
    try:
        _split_k_case(hip, loadgen, M, N, K, relu, bias)
    finally:
        hip.set_split_k(0)


def _split_k_case(hip, loadgen, M, N, K, relu, bias):
    assert hip.pick_split_k(M, N, K) > 1
    g = torch.Generator(device="cuda").manual_seed(M + 3 * N + K)
    a = (torch.rand(M, K, device="cuda", generator=g) * 2 - 1).to(torch.bfloat16)
    bt = (torch.rand(N, K, device="cuda", generator=g) * 2 - 1).to(torch.bfloat16)
    b = torch.randn(N, device="cuda", generator=g) if bias else None
    ref = a.float() @ bt.float().T + (b if bias else 0)
    if relu:
        ref = torch.relu(ref)
    tol = 0.01 * ref.abs().max().item() + 1e-2
    out = torch.empty(M, N, device="cuda", dtype=torch.bfloat16)
    for _ in range(4):
        out.fill_(float("nan"))
        loadgen.gemm(a, bt, out=out, bias=b, relu=relu)
        assert (out.float() - ref).abs().max().item() <= tol


@pytest.mark.parametrize("M,N,K,relu,bias", [(1024, 2560, 2560, True, True), (1024, 1536, 1536, True, False),
                                             (1024, 1024, 2048, False, True)])
def test_gemm_corun_split_k_policy8_matches_fp32_reference(hip, M, N, K, relu, bias):
    """Arm 8: a co-running pod's GEMM at its 64-CU share, too small for one
    256 x 256 tile per CU, runs split along K on the 8-phase kernel (2-4 slices) -> fp32 partials ->
    reduce; checked against fp32 PyTorch with the race screen's repeated runs."""
    from k8s_gpu_scheduler_amd.ops import loadgen
    hip.set_gemm_policy(8)
    try:
        assert hip.pick_split_k(M, N, K, 64) > 1
        g = torch.Generator(device="cuda").manual_seed(M + 5 * N + K)
        a = (torch.rand(M, K, device="cuda", generator=g) * 2 - 1).to(torch.bfloat16)
        bt = (torch.rand(N, K, device="cuda", generator=g) * 2 - 1).to(torch.bfloat16)
        b = torch.randn(N, device="cuda", generator=g) if bias else None
        ref = a.float() @ bt.float().T + (b if bias else 0)
        if relu:
            ref = torch.relu(ref)
        tol = 0.01 * ref.abs().max().item() + 1e-2
        out = torch.empty(M, N, device="cuda", dtype=torch.bfloat16)
        for _ in range(4):
            out.fill_(float("nan"))
            loadgen.gemm(a, bt, out=out, bias=b, relu=relu, cu_budget=64)
            assert (out.float() - ref).abs().max().item() <= tol
    finally:
        hip.set_gemm_policy(10)


@pytest.mark.parametrize("M,N,K", [(4096, 2560, 2560), (2048, 2560, 1536), (4096, 2048, 1024)])
def test_gemm_share_capped_policy9_matches_fp32_reference(hip, M, N, K):
    """Arm 9: a co-running pod's 8-phase GEMM with more 256 x 256 tiles than its 64-CU share runs as
    back-to-back launches of whole tile rows (<= 64 tiles each); every row slice lands in the
    right place (fp32 PyTorch reference, repeated runs)."""
    from k8s_gpu_scheduler_amd.ops import loadgen
    hip.set_gemm_policy(9)
    try:
        assert hip.pick_gemm_tile(M, N, 64) == 10
        g = torch.Generator(device="cuda").manual_seed(M + 7 * N + K)
        a = (torch.rand(M, K, device="cuda", generator=g) * 2 - 1).to(torch.bfloat16)
        bt = (torch.rand(N, K, device="cuda", generator=g) * 2 - 1).to(torch.bfloat16)
        b = torch.randn(N, device="cuda", generator=g)
        ref = torch.relu(a.float() @ bt.float().T + b)
        tol = 0.01 * ref.abs().max().item() + 1e-2
        out = torch.empty(M, N, device="cuda", dtype=torch.bfloat16)
        for _ in range(3):
            out.fill_(float("nan"))
            loadgen.gemm(a, bt, out=out, bias=b, relu=True, cu_budget=64)
            assert (out.float() - ref).abs().max().item() <= tol
    finally:
        hip.set_gemm_policy(10)


@pytest.mark.parametrize("policy,small_tile", [(11, 15), (13, 16)])
def test_gemm_corun_policy11_13_four_wave_matches_fp32_reference(hip, policy, small_tile):
    """Arms 11 / 13: arm 10, plus co-running GEMMs too small for 256 x 256 tiles on the 4-wave
    kernel at 256 x 128 (tile 15) / 128 x 128 (tile 16) -- fp32 PyTorch reference, repeated runs."""
    from k8s_gpu_scheduler_amd.ops import loadgen
    hip.set_gemm_policy(policy)
    try:
        for M, N, K, tile in [(1024, 2048, 1024, small_tile), (1024, 2560, 2560, small_tile), (4096, 4096, 512, 14)]:
            assert hip.pick_gemm_tile(M, N, 64) == tile
            g = torch.Generator(device="cuda").manual_seed(M + 3 * N + K)
            a = (torch.rand(M, K, device="cuda", generator=g) * 2 - 1).to(torch.bfloat16)
            bt = (torch.rand(N, K, device="cuda", generator=g) * 2 - 1).to(torch.bfloat16)
            b = torch.randn(N, device="cuda", generator=g)
            ref = torch.relu(a.float() @ bt.float().T + b)
            tol = 0.01 * ref.abs().max().item() + 1e-2
            out = torch.empty(M, N, device="cuda", dtype=torch.bfloat16)
            for _ in range(3):
                out.fill_(float("nan"))
                loadgen.gemm(a, bt, out=out, bias=b, relu=True, cu_budget=64)
                assert (out.float() - ref).abs().max().item() <= tol, (M, N, K)
    finally:
        hip.set_gemm_policy(10)


@pytest.mark.parametrize("prio", [0, 1])
def test_gemm_corun_policy10_four_wave_matches_fp32_reference(hip, prio):
    """Arm 10: a co-running pod's GEMM that fills its share with 256 x 256 tiles runs the 4-wave
    kernel (tile 14), in the XCD-block tile order, with and without whole-kernel priority; the
    unaligned-C fallback takes the 8-phase kernel (fp32 PyTorch reference, repeated runs)."""
    from k8s_gpu_scheduler_amd.ops import loadgen
    hip.set_gemm_policy(10)
    hip.set_w4_prio(prio)
    try:
        for M, N, K in [(4096, 4096, 1024), (2048, 2560, 2560), (8192, 2048, 192)]:
            assert hip.pick_gemm_tile(M, N, 64) == 14
            g = torch.Generator(device="cuda").manual_seed(M + 5 * N + K + prio)
            a = (torch.rand(M, K, device="cuda", generator=g) * 2 - 1).to(torch.bfloat16)
            bt = (torch.rand(N, K, device="cuda", generator=g) * 2 - 1).to(torch.bfloat16)
            b = torch.randn(N, device="cuda", generator=g)
            ref = torch.relu(a.float() @ bt.float().T + b)
            tol = 0.01 * ref.abs().max().item() + 1e-2
            out = torch.empty(M, N, device="cuda", dtype=torch.bfloat16)
            for _ in range(3):
                out.fill_(float("nan"))
                loadgen.gemm(a, bt, out=out, bias=b, relu=True, cu_budget=64)
                assert (out.float() - ref).abs().max().item() <= tol, (M, N, K)
        # C rows 8-B but not 16-B aligned: the 8-phase kernel instead (a forced tile 14 would raise)
        M, N, K = 1024, 1024, 512
        a = (torch.rand(M, K, device="cuda") * 2 - 1).to(torch.bfloat16)
        bt = (torch.rand(N, K, device="cuda") * 2 - 1).to(torch.bfloat16)
        wide = torch.empty(M, N + 4, device="cuda", dtype=torch.bfloat16)
        out = wide[:, 4:]
        loadgen.gemm(a, bt, out=out, cu_budget=64)
        torch.testing.assert_close(out.float(), a.float() @ bt.float().T, atol=0.1, rtol=0.02)
    finally:
        hip.set_w4_prio(0)
        hip.set_gemm_policy(10)


@pytest.mark.parametrize("slice_", [0, 1])
def test_gemm_split_k_layout_identity(hip, slice_):
    """A = I placed in K slice 0 or 1 (zeros elsewhere) with an asymmetric B: pins the C layout
    and each slice's K offset exactly."""
    from k8s_gpu_scheduler_amd.ops import loadgen
    n, K = 256, 2048
    hip.set_split_k(-1)
    try:
        _split_k_identity(hip, loadgen, n, K, slice_)
    finally:
        hip.set_split_k(0)


def _split_k_identity(hip, loadgen, n, K, slice_):
    assert hip.pick_split_k(n, n, K) == 2
    a = torch.zeros(n, K, device="cuda", dtype=torch.bfloat16)
    a[:, slice_ * 1024:slice_ * 1024 + n] = torch.eye(n, device="cuda", dtype=torch.bfloat16)
    asym = (torch.arange(n * n, device="cuda", dtype=torch.float32).reshape(n, n) % 97).to(torch.bfloat16)
    bt = torch.zeros(n, K, device="cuda", dtype=torch.bfloat16)
    bt[:, slice_ * 1024:slice_ * 1024 + n] = asym
    assert torch.equal(loadgen.gemm(a, bt).float(), asym.float().T)


def test_gemm_layout_identity_asymmetric():
    """A = I with an asymmetric B catches row/col swaps in the C write (guide §3)."""
    from k8s_gpu_scheduler_amd.ops import loadgen
    n = 256
    a = torch.eye(n, device="cuda", dtype=torch.bfloat16)
    bt = (torch.arange(n * n, device="cuda", dtype=torch.float32).reshape(n, n) % 97).to(torch.bfloat16)
    out = loadgen.gemm(a, bt)
    assert torch.equal(out.float(), bt.float().T)


@pytest.mark.parametrize("M,N,K,relu,bias", [(64, 64, 128, False, False), (128, 128, 256, True, True),
                                             (384, 640, 384, False, True), (1024, 2048, 2048, True, False),
                                             (4096, 4096, 1024, False, False)])
def test_gemm_fp8_matches_fp32_reference(M, N, K, relu, bias):
    """Block-scaled fp8 MFMA GEMM (unit scales) vs fp32 matmul of the same e4m3fn values
    (both 64x64 and 128x128 tiles are hit by these shapes)."""
    from k8s_gpu_scheduler_amd.ops import loadgen
    g = torch.Generator(device="cuda").manual_seed(M + 3 * N + K)
    a = torch.randn(M, K, device="cuda", generator=g).to(loadgen.FP8)
    bt = torch.randn(N, K, device="cuda", generator=g).to(loadgen.FP8)
    b = torch.randn(N, device="cuda", generator=g) if bias else None
    out = loadgen.gemm_fp8(a, bt, bias=b, relu=relu)
    ref = a.float() @ bt.float().T + (b if bias else 0)
    if relu:
        ref = torch.relu(ref)
    err = (out.float() - ref).abs().max().item()
    assert err <= 0.01 * ref.abs().max().item() + 1e-2, err


def test_gemm_fp8_layout_identity_asymmetric():
    """A = I (exact in e4m3) with an asymmetric integer B (0..15, exact in e4m3 and bf16)
    pins the C layout and the k pairing of the A/B fragments: the result must be exact."""
    from k8s_gpu_scheduler_amd.ops import loadgen
    for n in (128, 256, 640):
        a = torch.eye(n, device="cuda").to(loadgen.FP8)
        bt = (torch.arange(n * n, device="cuda", dtype=torch.float32).reshape(n, n) % 16).to(loadgen.FP8)
        assert torch.equal(loadgen.gemm_fp8(a, bt).float(), bt.float().T), n
    with pytest.raises(ValueError):
        loadgen.gemm_fp8(torch.zeros(128, 64, device="cuda").to(loadgen.FP8),
                         torch.zeros(128, 64, device="cuda").to(loadgen.FP8))


def test_gemm_rejects_bad_shapes():
    from k8s_gpu_scheduler_amd.ops import loadgen
    a = torch.zeros(100, 64, device="cuda", dtype=torch.bfloat16)
    with pytest.raises(ValueError):
        loadgen.gemm(a, torch.zeros(128, 64, device="cuda", dtype=torch.bfloat16))
    with pytest.raises(ValueError):
        loadgen.gemm(torch.zeros(128, 96, device="cuda", dtype=torch.bfloat16),
                     torch.zeros(128, 96, device="cuda", dtype=torch.bfloat16))


def test_triad_matches_reference():
    from k8s_gpu_scheduler_amd.ops import loadgen
    n = 1 << 22
    b, c = torch.rand(n, device="cuda"), torch.rand(n, device="cuda")
    a = torch.empty_like(b)
    loadgen.triad(a, b, c, 2.5)
    torch.testing.assert_close(a, b + 2.5 * c)


def test_triad_variants_match_reference():
    """Every selectable stream-kernel variant on a length that leaves a partial unrolled trip
    (fp32 reference b + s*c)."""
    from k8s_gpu_scheduler_amd import _native
    from k8s_gpu_scheduler_amd.ops import loadgen
    h = _native.hip(required=True)
    n = (1 << 20) + 4 * 123
    b, c = torch.rand(n, device="cuda"), torch.rand(n, device="cuda")
    ref = b + 1.5 * c
    try:
        for v in range(11):
            h.set_triad_variant(v)
            a = torch.full_like(b, -1.0)
            loadgen.triad(a, b, c, 1.5)
            torch.testing.assert_close(a, ref, msg=f"variant {v}")
        with pytest.raises(Exception):
            h.set_triad_variant(11)
    finally:
        h.set_triad_variant(6)


def test_cu_mask_slices_map_to_all_xccs():
    """A 2-word mask = 64 CUs = 8 CUs on each of the 8 XCCs (measured mapping)."""
    from k8s_gpu_scheduler_amd.ops.cumask import probe_xcd_map
    from k8s_gpu_scheduler_amd.plugins.gpu.devices import cu_slice_mask
    r = probe_xcd_map(cu_slice_mask(2, 2), 2048)
    assert sorted(r["cus_per_xcc"]) == list(range(8))
    assert all(v == 8 for v in r["cus_per_xcc"].values()), r


def test_masked_stream_gemm_correct_and_slower():
    from k8s_gpu_scheduler_amd.ops import loadgen
    from k8s_gpu_scheduler_amd.ops.cumask import MaskedStream
    from k8s_gpu_scheduler_amd.plugins.gpu.devices import cu_slice_mask
    n = 4096
    a = torch.randn(n, n, device="cuda").to(torch.bfloat16)
    bt = torch.randn(n, n, device="cuda").to(torch.bfloat16)
    ms = MaskedStream(cu_slice_mask(0, 1))           # 32 CUs
    try:
        def run(stream):
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            s = stream or torch.cuda.current_stream()
            e0.record(s)
            for _ in range(5):
                out = loadgen.gemm(a, bt, stream=stream)
            e1.record(s)
            torch.cuda.synchronize()
            return e0.elapsed_time(e1), out
        run(None)
        t_full, o1 = run(None)
        t_mask, o2 = run(ms.stream)
        assert torch.equal(o1, o2)
        assert t_mask > 2.5 * t_full, (t_mask, t_full)
    finally:
        ms.close()


def test_executor_epoch_and_bench_smoke():
    from k8s_gpu_scheduler_amd.parallel.executor import DeviceExecutor, PodRun
    ex = DeviceExecutor(0)
    runs = [PodRun(i, w, 2 * i, 2, 2, 1.0) for i, w in
            enumerate(["onnx_resnet50_1024", "onnx_mobilenet_1024", "tensorflow_ssd_mobilenet_1024",
                       "onnx_resnet50_2048"])]
    ex.launch_epoch(runs)
    torch.cuda.synchronize()
    st = ex.collect(runs)
    assert st["pods"] == 4 and all(r.ms > 0 for r in runs) and st["busy_unit_ms"] > 0
    ex.close()
    from k8s_gpu_scheduler_amd.parallel.podbench import main
    r = main(["--steps", "2", "--warmup", "1"])
    assert r["value"] > 0 and not r["simulated"] and r["unscheduled"] == 0


def _direction_run(slow: float, epochs: int, first: int):
    """The N-GPU bench's planner path on hardware: a 2-GPU control plane (co-run planner +
    backlog carry + measured feedback) plans each epoch; each GPU's group runs on the MI355X in
    turn (isolated, the bench's executor), and GPU 1's pods really run `slow` x the iterations
    the model is told -- a GPU slower than its sibling.  Returns (planner, GPU 1 shares of epochs
    >= first, backlog spreads, GPU 0 group errors, state printer)."""
    import numpy as np
    from k8s_gpu_scheduler_amd.models import workloads as W
    from k8s_gpu_scheduler_amd.parallel import podbench as PB
    from k8s_gpu_scheduler_amd.parallel.executor import PodRun
    cp = PB.ControlPlane(n_gpus=2, pods_per_gpu=2, iters=20, seed=5, balance=1.0, plan_bursts=True,
                         plan_tolerance=0.3, slo_objective="corun", corun_sigma=0.05, plan_carry=1.0)
    planner = cp.plugin.planner
    model = cp.corun.base if cp.corun is not None else planner.plugin.corun_model()
    ex = PB.gpu_executor(PB.build_parser().parse_args([]), 0)
    # every slot a pod of either GPU can land on, at both iteration counts (as the bench warms)
    for it in sorted({20, int(round(20 * slow))}):
        ex.warm([PodRun(0, wl, u, 2, it, masked=False) for wl in W.NAMES for u in (0, 2, 4, 6)])
    share, errs, spreads = [], [], []
    fed = {}
    orig = planner.observe_time

    def spy(group, pred, meas):
        fed.setdefault(group, []).append(round(meas / pred, 3))
        orig(group, pred, meas)
    planner.observe_time = spy

    def state(e):
        keys = sorted(planner.backlog)
        return (f"epoch {e} backlog {planner.backlog} speeds {[planner.speed(k) for k in keys]} "
                f"rel {planner.rel_speeds(keys) if keys else None} fed {fed} shares {np.round(share, 3)}")
    for e in range(epochs):
        cp.finish_live()
        arr = cp.schedule_epoch()
        per_gpu = np.zeros((2, PB.TELE))
        per_gpu[:, PB.SMI0:] = -1.0
        runs = {g: PB._runs_for(arr, g) for g in (0, 1)}
        assert runs[0] and runs[1], (arr, state(e))           # no GPU starved of a whole burst
        if planner.backlog:
            spreads.append(max(planner.backlog.values()) - min(planner.backlog.values()))
        work = {g: sum(model.alone_ms[model.wid(r.workload)] * r.iters for r in runs[g]) for g in (0, 1)}
        if e >= first:
            share.append(work[1] / (work[0] + work[1]))
        for r in runs[1]:
            r.iters = int(round(r.iters * slow))    # the slower GPU: work the model does not see
        for g in (0, 1):                            # each GPU's group in isolation, in turn
            ex.launch_epoch(runs[g])
            ex.wait_all()
            ex.collect(runs[g])
            per_gpu[g, PB.POD0:PB.SMI0] = PB._pod_rows(runs[g], ex.clock)
            if g == 0 and e >= 1:
                wall = max(ex.clock.elapsed_time(r.end) for r in runs[g]) - \
                    min(ex.clock.elapsed_time(r.start) for r in runs[g])
                pred = float(np.max(model.group_times([model.wid(r.workload) for r in runs[g]],
                                                      [r.iters for r in runs[g]])))
                errs.append(abs(pred - wall) / wall)
        cp.update_telemetry(per_gpu, 1.0)
    ex.close()
    print(state(epochs), "group errors", np.round(errs, 3), "backlog spreads", np.round(spreads, 2),
          "lazy captures", ex.lazy_captures)
    return planner, share, spreads, errs, state


def test_planner_feedback_moves_work_off_a_really_slower_gpu():
    """DIRECTION on hardware, GPU 1 40 % slower: after 12 epochs the measured feedback must have
    raised GPU 1's measured speed ratio over GPU 0's and moved planned work off it, without ever
    starving a GPU of a whole burst (the backlog is bounded, planner.observe_time); and the co-run
    model's predicted group times must be within 15 % of the measured ones for >= 80 % of GPU 0's
    (unslowed) groups."""
    import numpy as np
    from k8s_gpu_scheduler_amd.parallel import podbench as PB
    planner, share, spreads, errs, state = _direction_run(1.4, 12, 6)
    g0, g1 = (PB.NODE, 0), (PB.NODE, 1)
    assert planner.speed(g1) > 1.2 * planner.speed(g0), state(12)      # GPU 1 measured slower
    # (a burst is 4 pods of unequal length, so a single burst's share is one of a handful of
    # discrete splits around the 1 / 2.4 target: GPU 1 takes one pod or two.  Round 6's rank-test
    # gate decides from the third observation on for a shift this large; on MI355X the bursts of
    # epochs 6-11 read 0.34-0.49 in two runs and 0.148-0.485 in a third, where GPU 1 took only
    # the burst's shortest pod once (round 5 saw the same 0.148) -- a starved GPU would be 0.
    # The backlog carry answers light bursts with heavier ones: with the 4-wave co-run GEMM
    # (round 6) two runs read 0.25 -> 0.572 and 0.198 -> 0.551, 0.515 at means 0.41 / 0.40 (the
    # 1.45x measured speed targets 0.41).  So the direction is judged on the mean, and a single
    # burst only has to stay clear of starvation (>= 0.12) and of dumping work on the slow GPU
    # (<= 0.6))
    assert 0.3 < float(np.mean(share)) < 0.5 and min(share) >= 0.12 and max(share) <= 0.6, state(12)
    # bounded: never more than the planner's stored clip of a balanced burst's work
    assert max(spreads) <= planner.STORE_CLIP * planner._burst_ms + 1e-6, (spreads, state(12))
    assert np.mean(np.asarray(errs) <= 0.15) >= 0.8, errs


def test_planner_feedback_sees_a_15pct_slower_gpu():
    """the same hardware path with GPU 1 only 15 % slower -- the size of a
    power-capped or noisy-neighbour GPU, which round 5's all-observations gate could not see
    through pipeline noise.  The rank-test gate must pass GPU 1's speed to the plans (rel speed
    above GPU 0's).  (Which share that buys is a CPU-test property over many bursts and seeds,
    tests/test_backlog_control.py: over 8 bursts of 4 pods the split is too discrete -- the CPU
    twin of this case reads 0.48-0.51 -- so here it only must not starve either GPU.)"""
    import numpy as np
    from k8s_gpu_scheduler_amd.parallel import podbench as PB
    planner, share, spreads, _, state = _direction_run(1.15, 16, 8)
    g0, g1 = (PB.NODE, 0), (PB.NODE, 1)
    rel = planner.rel_speeds([g0, g1])
    assert planner.speed(g1) > 1.07 * planner.speed(g0), state(16)
    assert rel[1] > rel[0], state(16)                                    # the gate passed it on
    assert 0.3 < float(np.mean(share)) < 0.55 and min(share) > 0.0, state(16)
    assert max(spreads) <= planner.STORE_CLIP * planner._burst_ms + 1e-6, (spreads, state(16))


def test_rccl_probe_single_rank(tmp_path, monkeypatch):
    """RCCL path of the placement probe (world size 1 on the 1-GPU box)."""
    import json
    from k8s_gpu_scheduler_amd.parallel import rccl_probe
    for k in ("WORLD_SIZE", "RANK", "MASTER_ADDR", "MASTER_PORT"):
        monkeypatch.delenv(k, raising=False)
    monkeypatch.setenv("MASTER_PORT", "29587")
    out = tmp_path / "p.json"
    assert rccl_probe.main(["--sizes", "1M,8M", "--iters", "3", "--out", str(out)]) == 0
    res = json.loads(out.read_text())["results"]
    assert {r["op"] for r in res} == {"all_reduce", "all_gather", "reduce_scatter"}
    assert all(r["time_us"] > 0 for r in res)


def test_als_imputer_on_gpu():
    import numpy as np
    from k8s_gpu_scheduler_amd.models.imputers import ALSImputer
    rng = np.random.default_rng(1)
    X = rng.normal(size=(200, 2)) @ rng.normal(size=(2, 16)) + 5
    M = X.copy()
    hide = rng.random(X.shape) < 0.2
    M[hide] = np.nan
    out = ALSImputer(k=2, device="cuda").fit(M).predict(M)
    assert np.abs(out[hide] - X[hide]).mean() < 0.5


def test_peer_matrix_and_smi():
    from k8s_gpu_scheduler_amd import _native
    m = _native.hip().peer_access_matrix()
    n = _native.hip().device_count()
    assert len(m) == n * n and all(m[i * n + i] == 1 for i in range(n))
    smi = _native.smi()
    assert smi is not None
    s = smi.Smi()
    if not s.init():
        pytest.skip(f"amd-smi unavailable on this box: {s.error()}")
    assert s.count() >= 1
    samples = s.sample()
    assert samples and samples[0]["vram_total_mb"] > 0
    # health inputs: the device answers; ECC counts are reported (or -1 if unsupported)
    assert samples[0]["responsive"] is True
    assert all(samples[0][k] >= -1 for k in ("ecc_correctable", "ecc_uncorrectable", "ecc_deferred"))
    from k8s_gpu_scheduler_amd.agent.health import HealthMonitor
    hm = HealthMonitor()
    hm.update(samples, [{"uuid": f"dev{i}"} for i in range(len(samples))])
    assert hm.unhealthy() == {}, hm.unhealthy()         # a working box is healthy
    topo = s.topology()
    assert topo["n"] == s.count()
    s.shutdown()


def test_pod_sees_only_its_assignment_end_to_end():
    """SURVEY §7.4 slice: HIP-enumerated devices -> node agent -> Redis -> scheduler ->
    assignment annotations -> launcher (mini-kubelet) -> container process.  The container
    sees exactly its device (by ROCr id), and a Guaranteed fractional pod's kernels run only
    on its CU slice (HSA_CU_MASK); a Burstable one is not masked."""
    import json
    import os
    import subprocess
    import sys
    from k8s_gpu_scheduler_amd.agent.agent import NodeAgent
    from k8s_gpu_scheduler_amd.agent.devices import HipSource
    from k8s_gpu_scheduler_amd.agent.launcher import PodLauncher
    from k8s_gpu_scheduler_amd.api import constants as C
    from k8s_gpu_scheduler_amd.api import objects as O
    from k8s_gpu_scheduler_amd.framework.config import default_gpu_config
    from k8s_gpu_scheduler_amd.framework.scheduler import Scheduler
    from k8s_gpu_scheduler_amd.kube.client import FakeCluster
    from k8s_gpu_scheduler_amd.plugins import full_registry
    from k8s_gpu_scheduler_amd.store.fake_redis import FakeRedisBackend, FakeRedisEngine
    from k8s_gpu_scheduler_amd.store.resp import Redis
    node = "mi355x-box"
    src = HipSource()
    devs = src.devices()
    assert devs and all(d["uuid"].startswith("GPU-") and len(d["uuid"]) == 20 for d in devs), devs
    r = Redis(FakeRedisBackend(FakeRedisEngine()))
    NodeAgent(node, r, src).publish()
    fc = FakeCluster()
    fc.create("nodes", O.make_node(node, gpus=len(devs)))
    s = Scheduler(fc, default_gpu_config({"compat_env": False}), full_registry(), bind_async=False, seed=0,
                  extras={"redis": r})
    s.start_informers()
    la = PodLauncher(fc, node, timeout_s=240)
    res = {}
    # the box has one GPU: two fractional pods share it, then (after they finish and are
    # deleted) one whole-GPU pod
    for batch in ([O.make_pod("guar", gpu_cu=64, gpu_mem_gib=8), O.make_pod("burst", gpu_cu=64, gpu_limits=False)],
                  [O.make_pod("whole", gpus=1)]):
        for p in batch:
            fc.create("pods", p)
        sr = s.schedule_pending()
        assert all(x.status.ok for x in sr), [x.status.message() for x in sr]
        res.update({x.pod_key.split("/")[1]: x for x in la.run_bound()})
        keep = {k: O.annotations(fc.get("pods", k, "default")) for k in [O.name(p) for p in batch]}
        for p in batch:
            fc.delete("pods", O.name(p), "default")
        res.update({k + "/ann": v for k, v in keep.items()})
    names = ("whole", "guar", "burst")
    out = {k: (res[k].json() or {"rc": res[k].rc, "stderr": res[k].stderr[-2000:]}) for k in names}
    os.makedirs("gpurun_out", exist_ok=True)
    with open("gpurun_out/e2e_container_view.json", "w") as f:
        json.dump({k: {"env": res[k].env, "seen": out[k]} for k in names}, f, indent=1)
    for k in names:
        assert res[k].rc == 0, out[k]
        ann = res[k + "/ann"]
        assert out[k]["count"] == 1 and out[k]["devices"][0]["rocr_uuid"] == ann[C.ANNOT_DEVICES], out[k]
    assert out["whole"]["cus_used"] == 256 and out["burst"]["cus_used"] == 256, out
    assert out["guar"]["cus_used"] == 64 and set(out["guar"]["cus_per_xcc"].values()) == {8}, out["guar"]
    # a device id that is not on the node hides every GPU (the env really filters)
    env = dict(os.environ, ROCR_VISIBLE_DEVICES="GPU-0000000000000000")
    p = subprocess.run([sys.executable, "-m", "k8s_gpu_scheduler_amd.agent.container_probe"], env=env,
                       capture_output=True, text=True, timeout=240)
    assert json.loads(p.stdout.strip().splitlines()[-1]).get("count", 0) == 0, p.stdout + p.stderr


def test_executor_graph_replay_matches_eager():
    """A pod's kernel sequence captured as one HIP graph and replayed on its (CU-masked)
    stream produces the same outputs as eager launches."""
    from k8s_gpu_scheduler_amd.models.workloads import CATALOG
    from k8s_gpu_scheduler_amd.parallel.executor import DeviceExecutor, PodRun
    wl = "onnx_ssd_mobilenet_1024"          # gemm + triad + gemm
    outs = {}
    for graphs in (False, True):
        ex = DeviceExecutor(0)
        ex.use_graphs = graphs
        runs = [PodRun(0, wl, 2, 2, 3, masked=True), PodRun(1, wl, 4, 2, 3, masked=False)]
        ex.warm(runs)
        ex.launch_epoch(runs)
        ex.wait_epoch(runs)
        assert all(r.start.elapsed_time(r.end) > 0 for r in runs)
        bufs = ex.buffers(CATALOG[wl], 2, 2)
        outs[graphs] = [t[3].float().clone() if o.kind == "gemm" else t[0].clone() for o, t in bufs.ops]
        assert (len(ex._graphs) == 2) == graphs
        ex.close()
    for a, b in zip(outs[False], outs[True]):
        assert torch.equal(a, b)


def test_executor_runs_extra_workloads_fp8_and_triad_only():
    """The workloads outside the catalog (models.workloads.EXTRA) run through the executor's
    captured graphs: the fp8 GEMMs' output equals the eager fp8 kernel on the same operands, and
    the triad-only pod streams its passes."""
    from k8s_gpu_scheduler_amd.models import workloads as W
    from k8s_gpu_scheduler_amd.ops import loadgen
    from k8s_gpu_scheduler_amd.parallel.executor import DeviceExecutor, PodRun
    ex = DeviceExecutor(0)
    ex.use_graphs = True
    runs = [PodRun(0, "fp8_llm_2048", 0, 2, 2, masked=False), PodRun(1, "triad_only_2048", 2, 2, 2, masked=False)]
    ex.warm(runs)
    ex.launch_epoch(runs)
    ex.wait_epoch(runs)
    assert all(r.start.elapsed_time(r.end) > 0 for r in runs)
    o, (a, bt, bias, c) = ex.buffers(W.get("fp8_llm_2048"), 0, 2).ops[0]
    assert o.kind == "gemm8" and a.dtype == loadgen.FP8
    ref = loadgen.gemm_fp8(a, bt, bias=bias, relu=True, cu_budget=64)
    torch.cuda.synchronize()
    assert torch.equal(c, ref)
    x, y, z = ex.buffers(W.get("triad_only_2048"), 2, 2).ops[0][1]
    assert torch.allclose(x, y + 1.0001 * z)
    ex.close()


def test_executor_serves_four_co_running_pod_streams_equally():
    """Four identical Burstable pods co-run on four streams and finish within a few percent of
    each other.  (A stream-wait pending on another hardware queue while they ran made the 4th
    stream ~1.8x slower: profiles/archive/r03_queue_fairness/README.md; wait_all waits from the host.)"""
    from k8s_gpu_scheduler_amd.parallel.executor import DeviceExecutor, PodRun
    wl = "onnx_resnet50_2048"
    ex = DeviceExecutor(0)
    ex.use_graphs = True
    ex.warm([PodRun(i, wl, 2 * i, 2, 20, masked=False) for i in range(4)])
    per = [[] for _ in range(4)]
    for _ in range(5):
        runs = [PodRun(i, wl, 2 * i, 2, 20, masked=False) for i in range(4)]
        ex.launch_epoch(runs)
        ex.wait_all()
        assert all(r.end.query() for r in runs)
        for i, r in enumerate(runs):
            per[i].append(r.start.elapsed_time(r.end))
    ex.close()
    med = sorted(sorted(p)[2] for p in per)
    assert med[-1] / med[0] < 1.2, per


def test_profiled_pod_writes_rocprof_history():
    """Profiler sidecar on the box: the pod runs under rocprofv3 --kernel-trace --stats and
    its kernel time lands in the workload's Redis history (what the resize loop reads)."""
    import sys
    from k8s_gpu_scheduler_amd.agent.devices import synthetic_node
    from k8s_gpu_scheduler_amd.agent.agent import NodeAgent
    from k8s_gpu_scheduler_amd.agent.pod_profiler import ProfiledLauncher
    from k8s_gpu_scheduler_amd.api import objects as O
    from k8s_gpu_scheduler_amd.framework.config import default_gpu_config
    from k8s_gpu_scheduler_amd.framework.scheduler import Scheduler
    from k8s_gpu_scheduler_amd.kube.client import FakeCluster
    from k8s_gpu_scheduler_amd.plugins import full_registry
    from k8s_gpu_scheduler_amd.recommender.admission import RedisHistory
    from k8s_gpu_scheduler_amd.store.fake_redis import FakeRedisBackend, FakeRedisEngine
    from k8s_gpu_scheduler_amd.store.resp import Redis
    r = Redis(FakeRedisBackend(FakeRedisEngine()))
    NodeAgent("box", r, synthetic_node(1, node="box")).publish()
    fc = FakeCluster()
    fc.create("nodes", O.make_node("box", gpus=1))
    s = Scheduler(fc, default_gpu_config({}), full_registry(), bind_async=False, extras={"redis": r})
    s.start_informers()
    fc.create("pods", O.make_pod("onnx-resnet50-1024-prof", gpu_cu=256))
    assert all(x.status.ok for x in s.schedule_pending())
    hist = RedisHistory(r)
    la = ProfiledLauncher(fc, "box", timeout_s=300, history=hist,
                          command=[sys.executable, "-m", "k8s_gpu_scheduler_amd.agent.container_probe", "--work", "30"])
    # the synthetic node's UUIDs are not this box's ROCr ids: run unfiltered
    la.env_for = lambda pod: {}
    (res,) = la.run_bound()
    assert res.rc == 0, res.stderr[-3000:]
    (h,) = hist.read("onnx_resnet50_1024")
    assert h["gpu_busy_ms"] > 0 and h["kernels"] >= 60, h
    assert any("gemm_bf16" in k["name"] for k in h["top"]), h["top"]


def test_profile_webhook_pod_under_rocprof_lands_in_redis_history(tmp_path):
    """The deployable per-pod profiler end to end on the box: the admission webhook wraps an
    opted-in pod's container in rocprofv3 (agent.profile_webhook), the kubelet-style launcher
    resolves the downward-API env / $(VAR)s / hostPath and runs it (ops.podrun: the workload's
    native GEMM + stream kernels), and the node agent's ingestor turns the finished output
    directory into the workload's Redis history -- GEMM kernels included."""
    import sys
    from k8s_gpu_scheduler_amd.agent import profile_webhook as PW
    from k8s_gpu_scheduler_amd.agent.launcher import PodLauncher
    from k8s_gpu_scheduler_amd.agent.pod_profiler import ROCPROF, ProfileIngestor
    from k8s_gpu_scheduler_amd.api import constants as C
    from k8s_gpu_scheduler_amd.api import objects as O
    from k8s_gpu_scheduler_amd.kube.client import FakeCluster
    from k8s_gpu_scheduler_amd.recommender.admission import RedisHistory
    from k8s_gpu_scheduler_amd.store.fake_redis import FakeRedisBackend, FakeRedisEngine
    from k8s_gpu_scheduler_amd.store.resp import Redis
    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    fc = FakeCluster()
    fc.create("nodes", O.make_node("box", gpus=1))
    fc.add_admission("pods", PW.ProfileInjector(rocprof=ROCPROF))
    pod = O.make_pod("onnx-resnet50-1024-wh", gpu_cu=64, gpu_mem_gib=8, env={C.ENV_ITERATIONS: "30"},
                     labels_={PW.LABEL_PROFILE: "trace"}, node_name="box", phase="Running")
    pod["spec"]["containers"][0]["command"] = [sys.executable, "-m", "k8s_gpu_scheduler_amd.ops.podrun"]
    pod["spec"]["containers"][0]["args"] = ["--workload", "onnx_resnet50_1024", "--cu-budget", "64"]
    fc.create("pods", pod)
    pod = fc.get("pods", "onnx-resnet50-1024-wh", "default")
    assert pod["spec"]["containers"][0]["command"][0] == ROCPROF
    la = PodLauncher(fc, "box", timeout_s=300)
    la.host_root = str(tmp_path)
    la.cwd = str(tmp_path)
    la.extra_env = {"TMPDIR": str(tmp_path), "PYTHONPATH": root}
    res = la.run(pod)
    assert res.rc == 0, res.stderr[-3000:]
    r = Redis(FakeRedisBackend(FakeRedisEngine()))
    ing = ProfileIngestor(str(tmp_path) + PW.HOST_DIR, RedisHistory(r))
    assert ing.step() == 1
    (h,) = RedisHistory(r).read("onnx_resnet50_1024")
    assert h["source"] == "rocprof" and h["cu"] == 64 and h["uid"] == O.uid(pod)
    assert any("gemm_bf16" in k["name"] for k in h["top"]), h["top"]
    assert h["kernels"] >= 90 and h["span_ms"] > 0 and h["throughput"] > 0 and 0 < h["busy_frac"] <= 1.0
    with open(os.path.join(OUT, "profile_webhook_sample.json"), "w") as f:
        json.dump(h, f, indent=1)


def test_resize_loop_fed_by_rocprof_history(tmp_path):
    """Config 5 on the deployed path: Poisson pods run as processes under the webhook's
    rocprofv3, the agent's ingestor writes their kernel-level samples to the workload
    history, and the resize admission of later pods reads them."""
    from k8s_gpu_scheduler_amd.parallel.resize_loop import run
    out = run(epochs=4, rate=2.0, request_cu=128, iters=10, resize=True, history="rocprof", workdir=str(tmp_path))
    with open(os.path.join(OUT, "resize_loop_rocprof.json"), "w") as f:
        json.dump(out, f, indent=1)
    assert out["failed_pods"] == 0, out
    assert out["completed"] > 0 and out["history"]["samples"] == out["history"]["profiled_pods"] > 0, out
    assert out["admission"]["seen"] >= out["created"]


def test_fabric_probe_single_device_publishes(tmp_path):
    """The agent's fabric probe on the box (agent.fabric): run in a child process (the agent
    never holds a GPU context), it measures every visible device's copy rate -- here one
    MI355X, so the diagonal (its own HBM copy) -- and the agent publishes it with the
    topology without error."""
    from k8s_gpu_scheduler_amd.agent.agent import NodeAgent
    from k8s_gpu_scheduler_amd.agent.devices import synthetic_node
    from k8s_gpu_scheduler_amd.agent.fabric import FabricProber, measure_in_child
    from k8s_gpu_scheduler_amd.store import schema
    from k8s_gpu_scheduler_amd.store.fake_redis import FakeRedisBackend, FakeRedisEngine
    from k8s_gpu_scheduler_amd.store.resp import Redis
    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    env = dict(os.environ, PYTHONPATH=root)
    res = measure_in_child(mib=64, iters=5, env=env)
    assert res is not None and res["n"] >= 1
    assert all(res["bw_gbps"][i][i] > 100.0 for i in range(res["n"])), res
    r = Redis(FakeRedisBackend(FakeRedisEngine()))
    ag = NodeAgent("box", r, synthetic_node(1, node="box"),
                   fabric=FabricProber(lambda: measure_in_child(mib=64, iters=5, env=env)))
    ag.publish()
    assert ag.probe_fabric()
    topo = json.loads(r.get(schema.topology_key("box")))
    assert topo["bw_gbps"][0][0] > 100.0
    with open(os.path.join(OUT, "fabric_probe.json"), "w") as f:
        json.dump(res, f, indent=1)


def test_rccl_set_check_runs_in_background_worker_and_reaches_topology(tmp_path):
    """agent.probes on the box: the background worker runs the RCCL set check
    (parallel.rccl_probe in a child process restricted to the set's GPUs) with the node
    tainted, and the verdict reaches `gpusched:topology:<node>`.  One MI355X here, so the
    set is {GPU 0} through a 1-rank RCCL communicator: the path, not a multi-GPU rate."""
    from k8s_gpu_scheduler_amd.agent.agent import NodeAgent
    from k8s_gpu_scheduler_amd.agent.devices import synthetic_node
    from k8s_gpu_scheduler_amd.agent.probes import SetChecker, busbw_of, set_probe_in_child
    from k8s_gpu_scheduler_amd.api import constants as C
    from k8s_gpu_scheduler_amd.api import objects as O
    from k8s_gpu_scheduler_amd.kube.client import FakeCluster
    from k8s_gpu_scheduler_amd.store import schema
    from k8s_gpu_scheduler_amd.store.fake_redis import FakeRedisBackend, FakeRedisEngine
    from k8s_gpu_scheduler_amd.store.resp import Redis
    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    env = dict(os.environ, PYTHONPATH=root, MASTER_PORT="29623")
    fc = FakeCluster()
    fc.create("nodes", O.make_node("box", gpus=1))
    taints = []

    def probe(gpus):
        taints.append([t["key"] for t in O.node_taints(fc.get("nodes", "box"))])
        return set_probe_in_child(gpus, mib=64, iters=5, timeout_s=100, env=env)
    sets = SetChecker(probe)
    r = Redis(FakeRedisBackend(FakeRedisEngine()))
    ag = NodeAgent("box", r, synthetic_node(1, node="box"), client=fc, set_checks=sets)
    ag.publish()
    sets._queue.append((0,))                 # a one-GPU "set" (note() takes >= 2 GPUs)
    assert ag.probes.tick() == "set 0"
    assert taints == [[C.TAINT_PROBING]] and not O.node_taints(fc.get("nodes", "box"))
    topo = json.loads(r.get(schema.topology_key("box")))
    (chk,) = topo["set_checks"]
    assert chk["gpus"] == [0] and chk["busbw_gbps"] > 0 and chk["ok"], chk
    with open(os.path.join(OUT, "rccl_set_check.json"), "w") as f:
        json.dump(topo["set_checks"], f, indent=1)


def test_device_plugin_allocates_real_device_nodes():
    """Device plugin on the real inventory (amd-smi / HIP): every advertised GPU resolves to
    its own /dev/dri/renderD* through sysfs, and Allocate hands a container /dev/kfd plus
    that node."""
    import os
    from k8s_gpu_scheduler_amd.agent import deviceplugin as dp
    from k8s_gpu_scheduler_amd.agent.devices import best_source
    inv = best_source().devices()
    assert inv, "no devices enumerated"
    for d in inv:
        d["healthy"] = True
    nodes = [dp.render_nodes(str(d.get("bdf", ""))) for d in inv]
    assert all(n and all(os.path.exists(p) for p in n) for n in nodes), nodes
    if all(d.get("bdf") for d in inv):
        assert all(len(n) == 1 for n in nodes) and len({n[0] for n in nodes}) == len(nodes)
    plugin = dp.DevicePlugin("amd.com/gpu", "box", lambda: inv)
    req = dp.AllocateRequest()
    req.container_requests.add(devices_ids=[inv[0]["uuid"]])
    resp = plugin.Allocate(req, None).container_responses[0]
    paths = [x.host_path for x in resp.devices]
    assert paths[0] == "/dev/kfd" and nodes[0][0] in paths
    assert resp.envs["ROCR_VISIBLE_DEVICES"] == inv[0]["uuid"]


def test_agent_exports_real_telemetry_to_prometheus():
    """BASELINE config 2: the node agent on the real MI355X (amd-smi source) publishes the
    device to Redis and its telemetry to the Prometheus exporter under the AMD and the
    DCGM-compatible names the reference queries (reference prom_metrics.go:64-70), with the
    device UUID label; the health verdict gauge is 1."""
    from k8s_gpu_scheduler_amd.agent.agent import NodeAgent
    from k8s_gpu_scheduler_amd.agent.devices import SmiSource
    from k8s_gpu_scheduler_amd.store import schema
    from k8s_gpu_scheduler_amd.store.fake_redis import FakeRedisBackend, FakeRedisEngine
    from k8s_gpu_scheduler_amd.store.resp import Redis
    from k8s_gpu_scheduler_amd.telemetry.exporter import GpuExporter
    try:
        src = SmiSource()
    except RuntimeError as e:
        pytest.skip(f"amd-smi unavailable: {e}")
    r = Redis(FakeRedisBackend(FakeRedisEngine()))
    ex = GpuExporter("box", dcgm_compat=True)
    ag = NodeAgent("box", r, src, exporter=ex)
    ag.step()
    uuids = schema.read_uuids(r, "box")
    assert uuids and all(u.startswith("GPU-") for u in uuids)
    text = ex.render().decode()
    for m in ("amd_gpu_gfx_activity", "amd_gpu_vram_used_mb", "amd_gpu_temperature_hotspot",
              "DCGM_FI_PROF_GR_ENGINE_ACTIVE", "DCGM_FI_DEV_FB_FREE", "amd_gpu_healthy"):
        assert f"{m}{{" in text, m
    assert f'UUID="{uuids[0]}"' in text
    assert any(l.startswith("amd_gpu_healthy{") and l.endswith(" 1.0") for l in text.splitlines())


def test_xcd_dispatch_and_tile_orders_bit_exact():
    """Blocks b and b + 8 run on the same XCD, the residues on distinct XCDs (HW_REG_XCC_ID):
    what the XCD-block tile order relies on; the XCD-block order is bit-exact vs the GROUP_M
    order, and the removed study knobs (XCD confinement, non-temporal C) are gone from the
    module so no runtime setting can select them."""
    from k8s_gpu_scheduler_amd import _native
    from k8s_gpu_scheduler_amd.ops import loadgen
    h = _native.hip(required=True)
    ids = torch.full((4096,), -1, dtype=torch.int32, device="cuda")
    h.xcd_probe(ids.data_ptr(), 4096, torch.cuda.current_stream().cuda_stream)
    torch.cuda.synchronize()
    # round-robin dispatch: blocks b and b + 8 share an XCD and the 8 residues cover the 8 XCDs
    # (the rotation -- which XCD gets block 0 -- depends on what was dispatched before)
    xcd_of = {}
    for b, x in enumerate(ids.cpu().tolist()):
        xcd_of.setdefault(b % 8, set()).add(x)
    assert all(len(v) == 1 for v in xcd_of.values()), xcd_of
    assert sorted(next(iter(v)) for v in xcd_of.values()) == list(range(8)), xcd_of
    M, N, K = 2048, 1536, 1024
    a = (torch.rand(M, K, device="cuda") * 2 - 1).to(torch.bfloat16)
    bt = ((torch.rand(N, K, device="cuda") * 2 - 1) * 0.05).to(torch.bfloat16)
    bias = torch.randn(N, device="cuda")
    y, z = torch.rand(1 << 20, device="cuda"), torch.rand(1 << 20, device="cuda")
    try:
        h.set_gemm_tile(10)
        # a co-running pod's GEMM (CU budget 64) takes the XCD-block order, a lone one the plain
        # GROUP_M order (set_lone_plain_order); every order computes the same bits
        ref = loadgen.gemm(a, bt, bias=bias, relu=True, cu_budget=64)
        tref = torch.empty_like(y)
        loadgen.triad(tref, y, z, 1.5)
        torch.testing.assert_close(ref.float(), torch.relu(a.float() @ bt.float().T + bias), atol=0.1, rtol=0.02)
        assert torch.equal(loadgen.gemm(a, bt, bias=bias, relu=True), ref)
        h.set_lone_plain_order(0)
        assert torch.equal(loadgen.gemm(a, bt, bias=bias, relu=True), ref)
        h.set_lone_plain_order(1)
        h.set_xcd_blocks(0)
        assert torch.equal(loadgen.gemm(a, bt, bias=bias, relu=True, cu_budget=64), ref)
        h.set_xcd_blocks(1)
        torch.testing.assert_close(tref, y + 1.5 * z)
        for gone in ("set_xcd_mask", "set_c_nontemporal", "set_triad_aux"):
            assert not hasattr(h, gone), gone
        for bad in (17, 18, -1):                  # (tiles 11-13 exist since round 5, 14-16 since round 6)
            with pytest.raises(Exception):
                h.set_gemm_tile(bad)
    finally:
        h.set_xcd_blocks(1)
        h.set_lone_plain_order(1)
        h.set_gemm_tile(0)
