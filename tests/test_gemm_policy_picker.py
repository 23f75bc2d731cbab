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
SMALL = {0: 1, 1: 1, 2: 1, 3: 5, 4: 8, 5: 11, 6: 12, 7: 13}


@pytest.fixture(autouse=True)
def _restore():
    yield
    h.set_gemm_policy(1)
    h.set_gemm_tile(0)


@pytest.mark.parametrize("policy", sorted(SMALL))
def test_small_corun_gemm_tile_per_policy(policy):
    h.set_gemm_policy(policy)
    assert h.pick_gemm_tile(1024, 2048, 64) == SMALL[policy]


@pytest.mark.parametrize("policy", range(8))
def test_large_corun_and_lone_gemm_tiles(policy):
    h.set_gemm_policy(policy)
    # enough 256x256 tiles for the share: the 8-phase kernel for every policy but 0
    assert h.pick_gemm_tile(4096, 4096, 64) == (1 if policy == 0 else 10)
    # a lone GEMM that fills the chip: tile 4 under policy 2, else the 8-phase kernel
    assert h.pick_gemm_tile(8192, 8192, 0) == (4 if policy == 2 else 10)


def test_forced_tile_overrides_policy():
    h.set_gemm_policy(7)
    h.set_gemm_tile(3)
    assert h.pick_gemm_tile(1024, 2048, 64) == 3
