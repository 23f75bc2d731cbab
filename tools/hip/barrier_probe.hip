// TIMING PROBE ONLY (not product code): the 8-phase GEMM's steady-state loop with half of its
// barriers removed (MODE 1) -- wrong results by design (WAR races on the LDS buffers) -- to
// bound what the per-phase barriers cost.  Built and run by tools/barrier_probe.py.
#include "../../native/hip/loadgen.hip"

namespace gs {
template <bool RELU, bool BIAS, bool PEEL = false, bool WIDE = false, bool SPLIT = false, int MODE = 0>
__global__ void __launch_bounds__(512, 1)
gemm_8ph_probe(const __bf16* __restrict__ A, const __bf16* __restrict__ Bt, __bf16* __restrict__ C,
                     const float* __restrict__ bias, int M, int N, int K, int lda, int ldb, int ldc,
                     float* __restrict__ ws = nullptr) {
  constexpr int HALF = 128 * 64 * 2;               // bytes of one half-tile image
  constexpr int BUF = 4 * HALF;                    // one K-tile: A0 A1 B0 B1
  constexpr int OA0 = 0, OA1 = HALF, OB0 = 2 * HALF, OB1 = 3 * HALF;
  __shared__ __attribute__((aligned(16))) char smem[2 * BUF];

  int nwg = gridDim.x;
  int b = blockIdx.x;
  int split = 0;
  if constexpr (SPLIT) {
    nwg = (M / 256) * (N / 256);                   // tiles; the S slices of one tile are nwg apart
    split = b / nwg;
    b -= split * nwg;
    A += (size_t)split * K;
    Bt += (size_t)split * K;
  }
  const int xcd = b % kXcds;
  const int q = nwg / kXcds, rem = nwg % kXcds;
  const int wgid = (xcd < rem ? xcd * (q + 1) : rem * (q + 1) + (xcd - rem) * q) + b / kXcds;
  const int tiles_m = M / 256, tiles_n = N / 256;
  const int per_group = GROUP_M * tiles_n;
  const int group = wgid / per_group;
  const int first_m = group * GROUP_M;
  const int gsize = min(tiles_m - first_m, GROUP_M);
  const int m0 = (first_m + (wgid % per_group) % gsize) * 256;
  const int n0 = ((wgid % per_group) / gsize) * 256;

  const int wave = __builtin_amdgcn_readfirstlane(threadIdx.x / kWave);
  const int lane = threadIdx.x & (kWave - 1);
  const int wr = wave >> 2, wc = wave & 3;
  const int frow = lane & 15, fk = lane >> 4;

  f32x4 acc[2][4][2][2];                           // [h][mi][g][nj]
#pragma unroll
  for (int h = 0; h < 2; ++h)
#pragma unroll
    for (int i = 0; i < 4; ++i)
#pragma unroll
      for (int g = 0; g < 2; ++g)
#pragma unroll
        for (int j = 0; j < 2; ++j) acc[h][i][g][j] = f32x4{0.f, 0.f, 0.f, 0.f};
  bf16x8 ar[2][4], b0r[2][2], b1r[2][2];            // [kk][mi], [kk][nj]

  const int T = K / 64;
  const int last_stage = 4 * T - 6;                // global phase of the last glds
  // half-tile j of K-tile u: A rows (j = 0, 3) or B rows (j = 1, 2)
  auto stage = [&](int u, int j) {
    char* dst = smem + (u & 1) * BUF + (j == 0 ? OA0 : j == 3 ? OA1 : j == 1 ? OB0 : OB1);
    if (j == 0 || j == 3)
      stage_tile<128, 512, 64>(A, lda, m0 + (j == 3 ? 128 : 0), u * 64, dst, wave, lane);
    else
      stage_tile<128, 512, 64>(Bt, ldb, n0 + (j == 2 ? 128 : 0), u * 64, dst, wave, lane);
  };
  auto read_a = [&](const char* half) {
#pragma unroll
    for (int kk = 0; kk < 2; ++kk)
#pragma unroll
      for (int i = 0; i < 4; ++i) ar[kk][i] = lds_frag<64>(half, wr * 64 + i * 16 + frow, kk * 4 + fk);
  };
  auto read_b = [&](const char* half, bf16x8 (&br)[2][2]) {
#pragma unroll
    for (int kk = 0; kk < 2; ++kk)
#pragma unroll
      for (int j = 0; j < 2; ++j) br[kk][j] = lds_frag<64>(half, wc * 32 + j * 16 + frow, kk * 4 + fk);
  };
  auto barrier = [] {
    __builtin_amdgcn_sched_barrier(0);
    __builtin_amdgcn_s_barrier();
    __builtin_amdgcn_sched_barrier(0);
  };
  auto mfma_quadrant = [&](int h, int g, bf16x8 (&br)[2][2]) {
    __builtin_amdgcn_s_setprio(1);
#pragma unroll
    for (int kk = 0; kk < 2; ++kk)
#pragma unroll
      for (int i = 0; i < 4; ++i)
#pragma unroll
        for (int j = 0; j < 2; ++j)
          acc[h][i][g][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(br[kk][j], ar[kk][i], acc[h][i][g][j], 0, 0, 0);
    __builtin_amdgcn_s_setprio(0);
  };
  // loads allowed in flight at the wait of global phase p: the glds of phases p-2 .. p
  // that exist (2 per phase)
  auto inflight = [&](int p) { return 2 * max(0, min(3, last_stage - p + 3)); };

  // prologue: K-tile 0 and half-tiles A0, B0 of K-tile 1 (phases -5 .. 0)
#pragma unroll
  for (int j = 0; j < 4; ++j) stage(0, j);
  stage(1, 0);
  stage(1, 1);
  wait_vmcnt<4>();                                 // K-tile 0 landed; K-tile 1's A0/B0 in flight
  barrier();
  if (wr == 1) barrier();                          // group 1 runs one barrier behind

  int t0 = 0;
  if constexpr (PEEL) {
    // Steady state (t <= T-3): every phase stages its half-tile and three half-tiles stay in
    // flight, so the waits are the constant vmcnt(6) and nothing branches -- the generic
    // loop below only runs the last two K-tiles, where the pipeline drains.
    for (; t0 + 2 < T; ++t0) {
      const char* cur = smem + (t0 & 1) * BUF;
      read_b(cur + OB0, b0r);
      __builtin_amdgcn_sched_barrier(0);
      read_a(cur + OA0);
      stage(t0 + 1, 2);
      barrier();
      mfma_quadrant(0, 0, b0r);
      if (MODE == 0) barrier();
      read_b(cur + OB1, b1r);
      stage(t0 + 1, 3);
      wait_vmcnt<6>();
      if (MODE == 0) barrier();
      mfma_quadrant(0, 1, b1r);
      barrier();
      read_a(cur + OA1);
      stage(t0 + 2, 0);
      barrier();
      mfma_quadrant(1, 1, b1r);
      if (MODE == 0) barrier();
      stage(t0 + 2, 1);
      wait_vmcnt<6>();
      if (MODE == 0) barrier();
      mfma_quadrant(1, 0, b0r);
      barrier();
    }
  }
  for (int t = t0; t < T; ++t) {
    const char* cur = smem + (t & 1) * BUF;
    const int p0 = 4 * t;
    // phase 1: (0,0)
    read_b(cur + OB0, b0r);
    __builtin_amdgcn_sched_barrier(0);
    read_a(cur + OA0);
    if (t + 1 < T) stage(t + 1, 2);
    barrier();
    mfma_quadrant(0, 0, b0r);
    barrier();
    // phase 2: (0,1)
    read_b(cur + OB1, b1r);
    if (t + 1 < T) stage(t + 1, 3);
    wait_vmcnt_rt(inflight(p0 + 2));
    barrier();
    mfma_quadrant(0, 1, b1r);
    barrier();
    // phase 3: (1,1)
    read_a(cur + OA1);
    if (t + 2 < T) stage(t + 2, 0);
    barrier();
    mfma_quadrant(1, 1, b1r);
    barrier();
    // phase 4: (1,0)
    if (t + 2 < T) stage(t + 2, 1);
    wait_vmcnt_rt(inflight(p0 + 4));
    barrier();
    mfma_quadrant(1, 0, b0r);
    barrier();
  }
  if (wr == 0) barrier();                          // balance the barrier count

  if constexpr (SPLIT) {
    // fp32 partial tile (D = C^T layout: 4 consecutive columns of one row per lane, 16-B stores)
    float* P = ws + (size_t)split * M * N;
#pragma unroll
    for (int g = 0; g < 2; ++g)
#pragma unroll
      for (int j = 0; j < 2; ++j) {
        const int col = n0 + g * 128 + wc * 32 + j * 16 + fk * 4;
#pragma unroll
        for (int h = 0; h < 2; ++h)
#pragma unroll
          for (int i = 0; i < 4; ++i) {
            const int row = m0 + h * 128 + wr * 64 + i * 16 + frow;
            *reinterpret_cast<f32x4*>(P + (size_t)row * N + col) = acc[h][i][g][j];
          }
      }
    return;
  }

  if constexpr (WIDE) {
    // Wide epilogue (wide_put / wide_store): the whole 256x256 bf16 block tile is assembled in
    // LDS (exactly the 128 KiB the K loop used; every wave is past its last LDS read and every
    // LDS-DMA has retired -- the drained pipeline's vmcnt(0) -- once the now-aligned wave
    // groups meet at one more barrier), then whole 512-B rows go out with 16-B stores: 16
    // coalesced stores per lane instead of 32 scattered 8-B ones (the scattered tail cost
    // 7-20 % of the kernel at K = 8192 .. 2048).
    barrier();
#pragma unroll
    for (int g = 0; g < 2; ++g)
#pragma unroll
      for (int j = 0; j < 2; ++j) {
        const int col = g * 128 + wc * 32 + j * 16 + fk * 4;
        f32x4 bv = f32x4{0.f, 0.f, 0.f, 0.f};
        if (BIAS) bv = *reinterpret_cast<const f32x4*>(bias + n0 + col);
#pragma unroll
        for (int h = 0; h < 2; ++h)
#pragma unroll
          for (int i = 0; i < 4; ++i) {
            f32x4 v = acc[h][i][g][j] + bv;
            bf16x4 o;
#pragma unroll
            for (int r = 0; r < 4; ++r) o[r] = (__bf16)(RELU ? (v[r] > 0.f ? v[r] : 0.f) : v[r]);
            wide_put<256>(smem, h * 128 + wr * 64 + i * 16 + frow, col, o);
          }
      }
    __syncthreads();
    wide_store<256, 256, 512>(smem, C, ldc, m0, n0);
    return;
  }

  // epilogue (D = C^T layout, as in gemm_bf16_nt_kernel): lane holds 4 consecutive columns
#pragma unroll
  for (int g = 0; g < 2; ++g)
#pragma unroll
    for (int j = 0; j < 2; ++j) {
      const int col = n0 + g * 128 + wc * 32 + j * 16 + fk * 4;
      f32x4 bv = f32x4{0.f, 0.f, 0.f, 0.f};
      if (BIAS) bv = *reinterpret_cast<const f32x4*>(bias + col);
#pragma unroll
      for (int h = 0; h < 2; ++h)
#pragma unroll
        for (int i = 0; i < 4; ++i) {
          const int row = m0 + h * 128 + wr * 64 + i * 16 + frow;
          f32x4 v = acc[h][i][g][j] + bv;
          bf16x4 o;
#pragma unroll
          for (int r = 0; r < 4; ++r) o[r] = (__bf16)(RELU ? (v[r] > 0.f ? v[r] : 0.f) : v[r]);
          *reinterpret_cast<bf16x4*>(C + (size_t)row * ldc + col) = o;
        }
    }
}


}  // namespace gs

extern "C" int probe_launch(int mode, const void* A, const void* B, void* C, int M, int N, int K, void* stream) {
  const dim3 grid((M / 256) * (N / 256)), block(512);
  auto s = reinterpret_cast<hipStream_t>(stream);
  auto a = reinterpret_cast<const __bf16*>(A);
  auto b = reinterpret_cast<const __bf16*>(B);
  auto c = reinterpret_cast<__bf16*>(C);
  if (M % 256 || N % 256 || K % 64 || K < 256) return 1;
  if (mode == 0)
    hipLaunchKernelGGL((gs::gemm_8ph_probe<false, false, true, true, false, 0>), grid, block, 0, s, a, b, c, nullptr, M,
                       N, K, K, K, N, nullptr);
  else
    hipLaunchKernelGGL((gs::gemm_8ph_probe<false, false, true, true, false, 1>), grid, block, 0, s, a, b, c, nullptr, M,
                       N, K, K, K, N, nullptr);
  return hipGetLastError() == hipSuccess ? 0 : 2;
}
