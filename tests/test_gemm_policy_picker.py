"""The native GEMM tile picker per `--gemm-policy` arm (host code only, no GPU).

ADVICE r5: the arm-3/4 branch of pick_gemm_tile tested `policy >= 3`, so arms 5-7 ran tile 8
and the bench A/B of tile 13 never executed it.  Every arm's tile is pinned here on the bench's
shapes: a quarter-GPU pod (64-CU budget) with a GEMM too small for one 256x256 tile per CU
(1024 x 2048) and one large enough (4096 x 4096), and a lone GEMM (whole chip)."""
import pytest

from k8s_gpu_scheduler_amd import _native

h = _native.hip(required=False)
pytestmark = pytest.mark.skipif(h is None, reason="HIP extension not built")

# policy -> tile for M=1024, N=2048 at a 64-CU budget
SMALL = {0: 1, 1: 1, 2: 1, 3: 5, 4: 8, 5: 11, 6: 12, 7: 13, 8: 1, 9: 1, 10: 1, 11: 15, 12: 14, 13: 16}


@pytest.fixture(autouse=True)
def _restore():
    yield
    h.set_gemm_policy(10)                                      # the default since round 6
    h.set_gemm_tile(0)


@pytest.mark.parametrize("policy", sorted(SMALL))
def test_small_corun_gemm_tile_per_policy(policy):
    h.set_gemm_policy(policy)
    assert h.pick_gemm_tile(1024, 2048, 64) == SMALL[policy]


@pytest.mark.parametrize("policy", range(14))
def test_large_corun_and_lone_gemm_tiles(policy):
    h.set_gemm_policy(policy)
    # enough 256x256 tiles for the share: the 8-phase kernel for every policy but 0 (128x128) and
    # 10 (the 4-wave kernel)
    assert h.pick_gemm_tile(4096, 4096, 64) == {0: 1, 10: 14, 11: 14, 12: 14, 13: 14}.get(policy, 10)
    # a lone GEMM that fills the chip: tile 4 under policy 2, else the 8-phase kernel
    assert h.pick_gemm_tile(8192, 8192, 0) == (4 if policy == 2 else 10)


def test_forced_tile_overrides_policy():
    h.set_gemm_policy(7)
    h.set_gemm_tile(3)
    assert h.pick_gemm_tile(1024, 2048, 64) == 3


def test_policy8_splits_small_corun_gemms_along_k():
    """Arm 8: a co-running GEMM with fewer 256 x 256 tiles than its share's
    CUs runs the 8-phase kernel split along K; shapes the tile already fills are not split, and
    lone GEMMs keep the lone rule (off by default)."""
    h.set_gemm_policy(8)
    assert h.pick_split_k(1024, 2560, 2560, 64) == 2           # 40 tiles -> 80 blocks
    assert h.gemm_workgroups(1024, 2560, 2560, 64, False, True) == 80
    assert h.splitk_workspace_floats(1024, 2560, 2560, 64) == 2 * 1024 * 2560
    assert h.pick_split_k(1024, 1536, 1536, 64) == 3           # 24 tiles, slices of 512
    assert h.pick_split_k(1024, 1024, 1024, 64) == 2           # 4 slices would be 256 deep
    assert h.pick_split_k(2048, 2560, 2560, 64) == 1           # 80 tiles fill the share
    assert h.pick_split_k(1024, 2560, 2560, 0) == 1            # lone: split-K stays off
    h.set_gemm_policy(1)
    assert h.pick_split_k(1024, 2560, 2560, 64) == 1


def test_python_default_tile_rule_matches_the_native_picker():
    """models.workloads.default_gemm_workgroups (the CU-fill feature's HIP-free copy of the default
    policy) against the native picker on every catalog / extra GEMM at the bench's share, a lone
    launch and a half share."""
    from k8s_gpu_scheduler_amd.models import workloads as W
    shapes = {(o.M, o.N, o.K, o.kind == "gemm8") for w in list(W.CATALOG.values()) + list(W.EXTRA.values())
              for o in w.ops if o.is_gemm}
    shapes |= {(256, 256, 64, False), (192, 320, 256, False), (8192, 8192, 8192, False), (640, 384, 128, False)}
    for policy in (10, 1):                                     # tile 14 launches tile 10's grid
        h.set_gemm_policy(policy)
        for M, N, K, fp8 in sorted(shapes):
            for budget in (0, 64, 128, 32):
                assert W.default_gemm_workgroups(M, N, K, budget, fp8) == h.gemm_workgroups(M, N, K, budget, fp8), \
                    (policy, M, N, K, budget, fp8)


def test_four_wave_study_tile_is_forced_only():
    """Tile 14 (the 4-wave 256 x 256 kernel of the round-6 lone-GEMM study) runs only when forced or
    under the co-run arm 10: no other policy picks it on any shape / budget, it launches one
    256-thread block per 256 x 256 tile, falls back to tile 4 below two K-tiles, and its timing
    probes are range-checked."""
    for policy in range(10):
        h.set_gemm_policy(policy)
        for M, N in [(1024, 2048), (4096, 4096), (8192, 8192), (2048, 1024)]:
            for budget in (0, 32, 64, 128):
                assert h.pick_gemm_tile(M, N, budget) != 14
    h.set_gemm_policy(10)
    assert h.pick_gemm_tile(8192, 8192, 0) == 10               # arm 10 leaves lone GEMMs alone
    assert h.gemm_workgroups(4096, 4096, 1024, 64, False, False) == 256
    h.set_gemm_policy(1)
    h.set_gemm_tile(14)
    assert h.pick_gemm_tile(1024, 2048, 64) == 14
    assert h.gemm_workgroups(8192, 8192, 8192, 0, False, False) == 32 * 32
    assert h.gemm_workgroups(512, 512, 64, 0, False, False) == 4       # K < 128 -> tile 4, same grid
    with pytest.raises(Exception):
        h.set_gemm_tile(17)
    h.set_gemm_tile(15)                                        # its 256 x 128 sibling (policy 11)
    assert h.gemm_workgroups(1024, 2048, 1024, 64, False, False) == 4 * 16
    h.set_gemm_tile(0)
    for bad in (-1, 4):
        with pytest.raises(Exception):
            h.set_w4_probe(bad)
    h.set_w4_probe(0)


def test_default_policy_is_the_four_wave_corun_arm():
    h.set_gemm_tile(0)
    h.set_gemm_policy(10)
    assert h.pick_gemm_tile(4096, 4096, 64) == 14 and h.pick_gemm_tile(8192, 8192, 0) == 10
