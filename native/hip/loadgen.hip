// Load-generator kernels: the GPU work a scheduled pod performs on its XCDs.
//
// The reference has no GPU code; its pods are external MLPerf-style
// inference containers whose throughput the recommender matrices describe
// (pkg/recommender/recommender/configurations_train.ods).  The MI355X build needs real,
// controllable load on the chip to measure "achieved node GPU-util %" (BASELINE.json), so
// each synthetic workload is a mix of:
//
//  * gemm_bf16_nt -- C[M,N] = act(A[M,K] . Bt[N,K]^T (+bias)), bf16 in / f32 accumulate /
//    bf16 out, on MFMA (v_mfma_f32_16x16x32_bf16).  Block tiles 64x64 .. 256x256 (4 or 8
//    waves; 64x64 or 128x64 per wave) picked per shape; both operands staged global->LDS with 16-byte
//    global_load_lds (no VGPR round trip) into a double-buffered, XOR-swizzled LDS image
//    (bank-conflict-free ds_read_b128 fragment reads); stage of tile t+1 is issued before
//    the MFMAs of tile t; XCD-aware bijective block remap + grouped tile order for L2 reuse.
//    Epilogue fuses bias + ReLU and stores packed bf16x4.
//  * stream_triad -- a = b + s*c over float4 (16 B/lane) -- the HBM-bound pod phase.
#include <cstdint>

#include "api.h"
#include "common.h"

namespace gs {

typedef __bf16 bf16x8 __attribute__((ext_vector_type(8)));
typedef float f32x4 __attribute__((ext_vector_type(4)));
typedef __bf16 bf16x4 __attribute__((ext_vector_type(4)));

constexpr int BK = 64;
constexpr int GROUP_M = 8;

typedef const void __attribute__((address_space(1)))* gptr_t;
typedef void __attribute__((address_space(3)))* lptr_t;

// Issue the glds for one ROWS x KT bf16 tile (rows [r0, r0+ROWS), k [k0, k0+KT)) of a
// row-major matrix with leading dimension ld (elements).  A row is KT*2 bytes = KT/8 16-byte
// chunks; logical chunk kc of row r lands at physical chunk kc ^ ((r >> 1) & (KT/8 - 1)).
// The LDS image itself is lane-linear (glds requirement), so the swizzle is applied on the
// per-lane SOURCE address (rule: linear dest + permuted source + same permutation on read).
// For KT = 64 (128-B rows) and KT = 32 (64-B rows) this makes every 16-lane group of a
// ds_read_b128 fragment read (rows r..r+15, one logical chunk) hit 16 distinct 16-B bank
// slots: conflict-free (checked against the gfx950 ds_read_b128 lane groups; PMC
// SQ_LDS_BANK_CONFLICT = 0, profiles/r01_gemm_pmc.json).
template <int ROWS, int NT, int KT = BK>
__device__ __forceinline__ void stage_tile(const __bf16* __restrict__ g, int ld, int r0, int k0,
                                           char* lds_tile, int wave, int lane) {
  constexpr int CH = KT / 8;          // 16-byte chunks per row
  constexpr int SH = CH == 8 ? 3 : 2;
#pragma unroll
  for (int i = 0; i < ROWS * KT * 2 / 16 / NT; ++i) {
    const int chunk = i * NT + wave * 64 + lane;
    const int r = chunk >> SH;
    const int p = chunk & (CH - 1);
    const int kc = p ^ ((r >> 1) & (CH - 1));
    const __bf16* src = g + (size_t)(r0 + r) * ld + k0 + kc * 8;
    char* dst = lds_tile + (i * NT + wave * 64) * 16;  // wave-uniform base
    __builtin_amdgcn_global_load_lds((gptr_t)src, (lptr_t)dst, 16, 0, 0);
  }
}

template <int KT = BK>
__device__ __forceinline__ bf16x8 lds_frag(const char* lds_tile, int row, int kchunk) {
  const int phys = kchunk ^ ((row >> 1) & (KT / 8 - 1));
  return *reinterpret_cast<const bf16x8*>(lds_tile + row * (KT * 2) + phys * 16);
}

// Block tile BM x BN, WGM x WGN waves, each wave (BM/WGM) x (BN/WGN) = MI x NJ MFMA 16x16
// tiles.  Register reuse (LDS read bytes per FLOP) is set by the WAVE tile and global->LDS
// traffic per FLOP by the BLOCK tile (the 256x256 variant, 8 waves of 128x64, moves ~40 %
// fewer LDS bytes per FLOP than 128x128).  Counters at 8192^3 (profiles/r01_gemm_pmc.json):
// no LDS bank conflicts, LDS array ~30 % busy, waves waiting ~26 % of their cycles -- the
// 2-stage loop is bound by the wait for the next tile, which STAGES >= 3 (counted vmcnt,
// raw s_barrier, glds issued two tiles ahead) attacks.  Small tiles exist so that the
// small-M GEMMs of the workload catalog still launch >= 256 workgroups (one per CU).
//
// The MFMA is issued with the B fragment as its first operand, so each lane's 4
// accumulator registers are 4 CONSECUTIVE output columns of one row (D = C^T layout:
// col = lane&15 -> m, row = (lane>>4)*4 + r -> n): the epilogue stores 8-byte packed bf16x4
// (4x fewer store instructions than one bf16 per register) and loads bias as float4.
// s_waitcnt with only the vmcnt field constrained (expcnt = 7, lgkmcnt = 15 = no wait);
// gfx9 encoding: vmcnt[3:0] -> bits 3:0, vmcnt[5:4] -> bits 15:14.
template <int N>
__device__ __forceinline__ void wait_vmcnt() {
  static_assert(N >= 0 && N < 64, "vmcnt range");
  __builtin_amdgcn_s_waitcnt((N & 0xF) | ((N >> 4) << 14) | (0x7 << 4) | (0xF << 8));
}

template <int BM, int BN, int WGM, int WGN, int OCC, bool RELU, bool BIAS, int STAGES = 2, int KT = BK,
          bool HOIST = false>
__global__ void __launch_bounds__(WGM * WGN * 64, OCC)
gemm_bf16_nt_kernel(const __bf16* __restrict__ A, const __bf16* __restrict__ Bt, __bf16* __restrict__ C,
                    const float* __restrict__ bias, int M, int N, int K, int lda, int ldb, int ldc) {
  constexpr int NT = WGM * WGN * 64;
  static_assert(KT == 32 || KT == 64, "K tile");
  constexpr int A_BYTES = BM * KT * 2, B_BYTES = BN * KT * 2;
  constexpr int WTM = BM / WGM, WTN = BN / WGN;       // wave tile
  constexpr int MI = WTM / 16, NJ = WTN / 16;
  static_assert(BM * KT * 2 / 16 % NT == 0 && BN * KT * 2 / 16 % NT == 0, "stage split");
  static_assert(STAGES >= 2 && STAGES <= 4, "stages");
  constexpr int LOADS = (BM + BN) * KT * 2 / 16 / NT;    // glds per thread per K-tile
  __shared__ __attribute__((aligned(16))) char smem[STAGES * (A_BYTES + B_BYTES)];

  // ---- XCD-aware bijective remap, then grouped (GROUP_M) tile order ----------------
  const int nwg = gridDim.x;
  const int b = blockIdx.x;
  const int xcd = b % kXcds;
  const int q = nwg / kXcds, rem = nwg % kXcds;
  const int wgid = (xcd < rem ? xcd * (q + 1) : rem * (q + 1) + (xcd - rem) * q) + b / kXcds;
  const int tiles_m = M / BM, tiles_n = N / BN;
  const int per_group = GROUP_M * tiles_n;
  const int group = wgid / per_group;
  const int first_m = group * GROUP_M;
  const int gsize = min(tiles_m - first_m, GROUP_M);
  const int tm = first_m + (wgid % per_group) % gsize;
  const int tn = (wgid % per_group) / gsize;
  const int m0 = tm * BM, n0 = tn * BN;

  const int wave = __builtin_amdgcn_readfirstlane(threadIdx.x / kWave);
  const int lane = threadIdx.x & (kWave - 1);
  const int wm = wave / WGN, wn = wave % WGN;

  f32x4 acc[MI][NJ];
#pragma unroll
  for (int i = 0; i < MI; ++i)
#pragma unroll
    for (int j = 0; j < NJ; ++j) acc[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};

  auto tileA = [&](int buf) { return smem + buf * (A_BYTES + B_BYTES); };
  auto tileB = [&](int buf) { return smem + buf * (A_BYTES + B_BYTES) + A_BYTES; };

  const int nt = K / KT;
  const int frow = lane & 15;
  const int fk = lane >> 4;
  auto compute = [&](const char* a_t, const char* b_t) {
    if constexpr (HOIST) {
      // every fragment of the K tile is read before the first MFMA: the MFMAs of k-step 0
      // wait only for their own reads (counted lgkmcnt), k-step 1's reads fly under them
      bf16x8 af[KT / 32][MI], bf[KT / 32][NJ];
#pragma unroll
      for (int kk = 0; kk < KT / 32; ++kk) {
#pragma unroll
        for (int j = 0; j < NJ; ++j) bf[kk][j] = lds_frag<KT>(b_t, wn * WTN + j * 16 + frow, kk * 4 + fk);
#pragma unroll
        for (int i = 0; i < MI; ++i) af[kk][i] = lds_frag<KT>(a_t, wm * WTM + i * 16 + frow, kk * 4 + fk);
      }
      __builtin_amdgcn_s_setprio(1);
#pragma unroll
      for (int kk = 0; kk < KT / 32; ++kk)
#pragma unroll
        for (int i = 0; i < MI; ++i)
#pragma unroll
          for (int j = 0; j < NJ; ++j)
            acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(bf[kk][j], af[kk][i], acc[i][j], 0, 0, 0);
      __builtin_amdgcn_s_setprio(0);
      return;
    }
#pragma unroll
    for (int kk = 0; kk < KT / 32; ++kk) {
      bf16x8 af[MI], bf[NJ];
#pragma unroll
      for (int j = 0; j < NJ; ++j) bf[j] = lds_frag<KT>(b_t, wn * WTN + j * 16 + frow, kk * 4 + fk);
#pragma unroll
      for (int i = 0; i < MI; ++i) af[i] = lds_frag<KT>(a_t, wm * WTM + i * 16 + frow, kk * 4 + fk);
      __builtin_amdgcn_s_setprio(1);
#pragma unroll
      for (int i = 0; i < MI; ++i)
#pragma unroll
        for (int j = 0; j < NJ; ++j)
          acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(bf[j], af[i], acc[i][j], 0, 0, 0);
      __builtin_amdgcn_s_setprio(0);
    }
  };
  auto stage = [&](int t, int buf) {
    stage_tile<BM, NT, KT>(A, lda, m0, t * KT, tileA(buf), wave, lane);
    stage_tile<BN, NT, KT>(Bt, ldb, n0, t * KT, tileB(buf), wave, lane);
  };

  if constexpr (STAGES == 2) {
    stage(0, 0);
    __syncthreads();
    int buf = 0;
    for (int t = 0; t < nt; ++t) {
      if (t + 1 < nt) stage(t + 1, buf ^ 1);   // issue tile t+1 before the MFMAs of tile t
      compute(tileA(buf), tileB(buf));
      __syncthreads();   // tile t+1 landed (vmcnt(0) before the barrier) and tile t fully read
      buf ^= 1;
    }
  } else {
    // Prologue: tiles 0 .. STAGES-2 in flight.  Iteration t: wait until only the tiles
    // after t are outstanding (counted vmcnt -- loads retire in order), barrier (every
    // thread's part of tile t landed AND every wave finished reading tile t-1, whose
    // buffer tile t+STAGES-1 reuses), issue tile t+STAGES-1, compute tile t.
#pragma unroll
    for (int p = 0; p < STAGES - 1; ++p)
      if (p < nt) stage(p, p);
    for (int t = 0; t < nt; ++t) {
      const int ahead = nt - 1 - t;             // tiles after t already issued (<= STAGES-2)
      if (ahead >= STAGES - 2) {
        wait_vmcnt<LOADS * (STAGES - 2)>();
      } else if (STAGES == 4 && ahead == 1) {
        wait_vmcnt<LOADS>();
      } else {
        wait_vmcnt<0>();
      }
      __builtin_amdgcn_sched_barrier(0);
      __builtin_amdgcn_s_barrier();
      __builtin_amdgcn_sched_barrier(0);
      if (t + STAGES - 1 < nt) stage(t + STAGES - 1, (t + STAGES - 1) % STAGES);
      compute(tileA(t % STAGES), tileB(t % STAGES));
    }
  }

  // ---- epilogue (D = C^T layout): row m = lane&15, cols n..n+3 = (lane>>4)*4 + r ----
#pragma unroll
  for (int j = 0; j < NJ; ++j) {
    const int col = n0 + wn * WTN + j * 16 + fk * 4;
    f32x4 bv = f32x4{0.f, 0.f, 0.f, 0.f};
    if (BIAS) bv = *reinterpret_cast<const f32x4*>(bias + col);
#pragma unroll
    for (int i = 0; i < MI; ++i) {
      const int row = m0 + wm * WTM + i * 16 + frow;
      f32x4 v = acc[i][j] + bv;
      bf16x4 o;
#pragma unroll
      for (int r = 0; r < 4; ++r) o[r] = (__bf16)(RELU ? (v[r] > 0.f ? v[r] : 0.f) : v[r]);
      *reinterpret_cast<bf16x4*>(C + (size_t)row * ldc + col) = o;
    }
  }
}

__global__ void __launch_bounds__(256) stream_triad_kernel(float4* __restrict__ a, const float4* __restrict__ b,
                                                           const float4* __restrict__ c, float s, size_t n4) {
  size_t i = (size_t)blockIdx.x * blockDim.x + threadIdx.x;
  const size_t stride = (size_t)gridDim.x * blockDim.x;
  for (; i < n4; i += stride) {
    float4 x = b[i], y = c[i];
    a[i] = make_float4(x.x + s * y.x, x.y + s * y.y, x.z + s * y.z, x.w + s * y.w);
  }
}

// Unrolled variant: each thread moves U float4 per trip with all loads issued before
// any store (U outstanding 16-B loads per stream per lane), block-contiguous so every
// load instruction is one coalesced 1 KiB wave access; NT selects non-temporal
// (streaming) loads/stores so the one-touch stream does not evict L2/MALL lines.
template <int U, bool NT>
__global__ void __launch_bounds__(256) stream_triad_u(float4* __restrict__ a_, const float4* __restrict__ b_,
                                                      const float4* __restrict__ c_, float s, size_t n4) {
  auto a = reinterpret_cast<f32x4*>(a_);
  auto b = reinterpret_cast<const f32x4*>(b_);
  auto c = reinterpret_cast<const f32x4*>(c_);
  const size_t tile = (size_t)blockDim.x * U;
  const size_t step = (size_t)gridDim.x * tile;
  for (size_t base = (size_t)blockIdx.x * tile + threadIdx.x; base < n4; base += step) {
    f32x4 x[U], y[U];
#pragma unroll
    for (int k = 0; k < U; ++k) {
      const size_t i = base + (size_t)k * blockDim.x;
      if (i < n4) {
        if (NT) {
          x[k] = __builtin_nontemporal_load(b + i);
          y[k] = __builtin_nontemporal_load(c + i);
        } else {
          x[k] = b[i];
          y[k] = c[i];
        }
      }
    }
#pragma unroll
    for (int k = 0; k < U; ++k) {
      const size_t i = base + (size_t)k * blockDim.x;
      if (i < n4) {
        const f32x4 r = x[k] + s * y[k];
        if (NT)
          __builtin_nontemporal_store(r, a + i);
        else
          a[i] = r;
      }
    }
  }
}

// 6 = auto: working set (3 arrays) <= 96 MiB -> cached 2x-unrolled loads (the stream
// stays in the 256 MiB Infinity Cache across iterations: 7.1 TB/s measured), larger ->
// non-temporal 4x (6.5 TB/s vs 6.1 for torch.add) -- profiles/r01_kernel_bench.json.
static int g_triad_variant = 6;

void set_triad_variant(int v) {
  if (v < 0 || v > 6) throw std::runtime_error("triad variant must be 0..6");
  g_triad_variant = v;
}

static void check_align(const void* p, const char* what) {
  if (reinterpret_cast<uintptr_t>(p) % 16 != 0) throw std::runtime_error(std::string(what) + " must be 16-byte aligned");
}

template <int BM, int BN, int WGM, int WGN, int OCC, int STAGES = 2, int KT = BK, bool HOIST = false>
static void launch_gemm(const __bf16* A, const __bf16* B, __bf16* Cp, const float* bp, int M, int N, int K, int lda,
                        int ldb, int ldc, bool relu, hipStream_t s) {
  const dim3 grid((M / BM) * (N / BN)), block(WGM * WGN * 64);
  if (relu && bp)
    hipLaunchKernelGGL((gemm_bf16_nt_kernel<BM, BN, WGM, WGN, OCC, true, true, STAGES, KT, HOIST>), grid, block, 0, s, A, B, Cp, bp, M, N,
                       K, lda, ldb, ldc);
  else if (relu)
    hipLaunchKernelGGL((gemm_bf16_nt_kernel<BM, BN, WGM, WGN, OCC, true, false, STAGES, KT, HOIST>), grid, block, 0, s, A, B, Cp, bp, M, N,
                       K, lda, ldb, ldc);
  else if (bp)
    hipLaunchKernelGGL((gemm_bf16_nt_kernel<BM, BN, WGM, WGN, OCC, false, true, STAGES, KT, HOIST>), grid, block, 0, s, A, B, Cp, bp, M, N,
                       K, lda, ldb, ldc);
  else
    hipLaunchKernelGGL((gemm_bf16_nt_kernel<BM, BN, WGM, WGN, OCC, false, false, STAGES, KT, HOIST>), grid, block, 0, s, A, B, Cp, bp, M,
                       N, K, lda, ldb, ldc);
}

// 0 = auto, 1 = 128x128 (4 waves, 2/CU), 2 = 64x128, 3 = 64x64,
// 4 = 256x256 (8 waves of 128x64, 1/CU), 5 = 256x128 (8 waves of 64x64, 1/CU)
static int g_gemm_tile = 0;
// (Measured and dropped: 128x128 with 2 waves of 128x64 and 128x256 with 4 waves of
// 64x128 -- fewer LDS bytes per FLOP, but 753 / 670 TF vs 783 TF for 128x128 on the co-run
// mix: profiles/r01_gemm_tiles_with_2wave_variants.json.)
// 6 = 128x128 without hoisted reads (A/B reference); 7 = 64x128, 3 stages (2/CU);
// 8 = 256x128 8 waves, 3 stages.
// Measured (profiles/r01_gemm_tiles.json): correct, but none beats 128x128 / 2 stages / 2 per CU
// (4096x2048x2048: 697 / 783 / 898 vs 954 TF; co-run mix 659 / 682 / 733 vs 795 TF): the extra
// stage costs the second resident block, which hid the tile wait just as well.
// (Also measured and dropped: 128x128 with a 32-deep K tile, 2 and 3 stages -- 4 / 3 blocks
// per CU, 687 / 704 TF on the co-run mix: twice the barriers per FLOP cost more than the
// extra residency hides; profiles/r01_gemm_tiles_bk32.json.)
// Tiles 1, 3 and 4 read all fragments of a K tile before its first MFMA (HOIST): +0-7 % over
// the per-k-step reads on the catalog shapes, 4096^3 1105 vs 1047 TF; for 64x128 it is mixed
// (profiles/r01_gemm_tiles_hoist.json), so that tile keeps per-k-step reads.  Tile 6 is the
// non-hoisted 128x128 kept as the A/B reference.
static const int kTileBM[9] = {0, 128, 64, 64, 256, 256, 128, 64, 256};
static const int kTileBN[9] = {0, 128, 128, 64, 256, 128, 128, 128, 128};

void set_gemm_tile(int t) {
  if (t < 0 || t > 8) throw std::runtime_error("gemm tile must be 0..8");
  g_gemm_tile = t;
}

int pick_gemm_tile(int M, int N, int cu_budget) {
  if (g_gemm_tile) return g_gemm_tile;
  // cu_budget = CUs this GEMM can expect to own: the whole chip for a lone kernel, the
  // pod's CU share when pods run side by side (0 = whole chip).  Measured
  // (profiles/r01_gemm_tiles.json): a lone kernel wants >= 2 workgroups per CU of the
  // 64/128-wide tiles (fill beats per-block efficiency) and the 256x256 tile only when it
  // still fills every CU (4096^3: 1172 vs 1089 TF); co-running pods want the largest
  // tile that gives one workgroup per CU of their share -- the other pods' kernels fill
  // the rest of the chip -- 128x128 on the whole catalog mix: 784 vs 715 TF aggregate.
  const bool alone = cu_budget <= 0 || cu_budget >= kCus;
  const int budget = alone ? kCus : cu_budget;
  const int per_cu = alone ? 2 : 1;
  if (alone && (M % 256 == 0) && (N % 256 == 0) && (M / 256) * (N / 256) >= budget) return 4;
  if ((M / 128) * (N / 128) >= per_cu * budget) return 1;
  if ((M / 64) * (N / 128) >= per_cu * budget && N % 128 == 0) return 2;
  return 3;
}

void gemm_bf16_nt(uintptr_t a, uintptr_t bt, uintptr_t c, uintptr_t bias, int M, int N, int K, int lda, int ldb,
                  int ldc, bool relu, uintptr_t stream, int cu_budget) {
  // Host-side shape checks: the kernel has no bounds checks by design.
  if (M <= 0 || N <= 0 || K <= 0) throw std::runtime_error("gemm: empty shape");
  if (M % 64 || N % 64 || K % BK) throw std::runtime_error("gemm: M,N must be multiples of 64 and K of 64");
  if (lda < K || ldb < K || ldc < N || lda % 8 || ldb % 8) throw std::runtime_error("gemm: bad leading dims");
  check_align(reinterpret_cast<void*>(a), "A");
  check_align(reinterpret_cast<void*>(bt), "Bt");
  auto s = reinterpret_cast<hipStream_t>(stream);
  auto A = reinterpret_cast<const __bf16*>(a);
  auto B = reinterpret_cast<const __bf16*>(bt);
  auto Cp = reinterpret_cast<__bf16*>(c);
  auto bp = reinterpret_cast<const float*>(bias);
  if (ldc % 4 || reinterpret_cast<uintptr_t>(c) % 8) throw std::runtime_error("gemm: C rows must be 8-byte aligned");
  if (bias) check_align(reinterpret_cast<void*>(bias), "bias");
  int t = pick_gemm_tile(M, N, cu_budget);
  if (M % kTileBM[t] || N % kTileBN[t]) t = 3;   // 64x64 always divides (checked above)
  switch (t) {
    case 1: launch_gemm<128, 128, 2, 2, 2, 2, 64, true>(A, B, Cp, bp, M, N, K, lda, ldb, ldc, relu, s); break;
    case 2: launch_gemm<64, 128, 2, 2, 2>(A, B, Cp, bp, M, N, K, lda, ldb, ldc, relu, s); break;
    case 4: launch_gemm<256, 256, 2, 4, 1, 2, 64, true>(A, B, Cp, bp, M, N, K, lda, ldb, ldc, relu, s); break;
    case 5: launch_gemm<256, 128, 4, 2, 1>(A, B, Cp, bp, M, N, K, lda, ldb, ldc, relu, s); break;
    case 6: launch_gemm<128, 128, 2, 2, 2>(A, B, Cp, bp, M, N, K, lda, ldb, ldc, relu, s); break;
    case 7: launch_gemm<64, 128, 2, 2, 2, 3>(A, B, Cp, bp, M, N, K, lda, ldb, ldc, relu, s); break;
    case 8: launch_gemm<256, 128, 4, 2, 1, 3>(A, B, Cp, bp, M, N, K, lda, ldb, ldc, relu, s); break;
    default: launch_gemm<64, 64, 2, 2, 2, 2, 64, true>(A, B, Cp, bp, M, N, K, lda, ldb, ldc, relu, s); break;
  }
  HIP_CHECK(hipGetLastError());
}

void stream_triad(uintptr_t a, uintptr_t b, uintptr_t c, float s, size_t n_floats, int blocks, uintptr_t stream) {
  if (n_floats % 4) throw std::runtime_error("triad: n must be a multiple of 4");
  check_align(reinterpret_cast<void*>(a), "a");
  check_align(reinterpret_cast<void*>(b), "b");
  check_align(reinterpret_cast<void*>(c), "c");
  if (blocks <= 0) blocks = 8192;
  auto st = reinterpret_cast<hipStream_t>(stream);
  auto A = reinterpret_cast<float4*>(a);
  auto B = reinterpret_cast<const float4*>(b);
  auto Cc = reinterpret_cast<const float4*>(c);
  const size_t n4 = n_floats / 4;
  int variant = g_triad_variant;
  if (variant == 6) variant = (n_floats * 12 <= (size_t)96 << 20) ? 1 : 3;
  switch (variant) {
    case 0: hipLaunchKernelGGL(stream_triad_kernel, dim3(blocks), dim3(256), 0, st, A, B, Cc, s, n4); break;
    case 1: hipLaunchKernelGGL((stream_triad_u<2, false>), dim3(blocks), dim3(256), 0, st, A, B, Cc, s, n4); break;
    case 2: hipLaunchKernelGGL((stream_triad_u<4, false>), dim3(blocks), dim3(256), 0, st, A, B, Cc, s, n4); break;
    case 3: hipLaunchKernelGGL((stream_triad_u<4, true>), dim3(blocks), dim3(256), 0, st, A, B, Cc, s, n4); break;
    case 4: hipLaunchKernelGGL((stream_triad_u<8, true>), dim3(blocks), dim3(256), 0, st, A, B, Cc, s, n4); break;
    default: hipLaunchKernelGGL((stream_triad_u<2, true>), dim3(blocks), dim3(256), 0, st, A, B, Cc, s, n4); break;
  }
  HIP_CHECK(hipGetLastError());
}

}  // namespace gs
