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
//    the MFMAs of tile t; XCD-aware bijective block remap + XCD-block tile order for L2 reuse.
//    Epilogue fuses bias + ReLU and stores packed bf16x4.  Lone large GEMMs use a separate
//    256x256 "8-phase" kernel (gemm_bf16_nt_256_8ph: two staggered wave groups, one
//    half-tile of glds per phase, counted vmcnt).
//  * gemm_fp8_nt -- the same GEMM with OCP e4m3fn operands on the block-scaled
//    v_mfma_scale_f32_16x16x128_f8f6f4 (unit scales): 2x the bf16 MFMA rate.
//  * stream_triad -- a = b + s*c over float4 (16 B/lane) -- the HBM-bound pod phase.
//
// Launch settings (set_gemm_policy, set_gemm_tile, set_split_k, set_wide_epilogue,
// set_xcd_blocks, set_xcd_group, set_triad_variant) are process-wide values read on the launching host thread when a kernel is
// enqueued (a captured HIP graph keeps the values of its capture).  One host thread per rank
// launches every pod kernel (parallel.executor), so they are plain statics; the defaults are
// the measured winners; every selectable variant computes the same result (GPU-tested against
// fp32 PyTorch), the rest of the A/B record lives in profiles/.
#include <algorithm>
#include <cstdint>
#include <type_traits>

#include "api.h"
#include "common.h"

namespace gs {

typedef __bf16 bf16x8 __attribute__((ext_vector_type(8)));
typedef float f32x4 __attribute__((ext_vector_type(4)));
typedef __bf16 bf16x4 __attribute__((ext_vector_type(4)));

constexpr int BK = 64;
constexpr int GROUP_M = 8;

// Block index -> output tile.  Workgroups b and b + 8 run on the same XCD (round-robin dispatch;
// which XCD takes block 0 rotates with earlier dispatches -- tests/test_gpu_native.py reads
// HW_REG_XCC_ID), so the XCD-aware bijective remap first makes each XCD's workgroups one
// contiguous range of wgid.
// xmap = 0: GROUP_M-row grouped order over the whole grid (an XCD's range is a tall 8-row
// strip of tiles).  xmap = px | (gm << 8): the tile grid is cut into px x (8 / px) equal
// rectangles, XCD x walks rectangle x (gm-row grouped order inside), so the A row-strips and B column-strips
// one XCD's L2 has to fetch are those of a near-square block: on the co-run catalog shapes
// 18-33 % fewer strips per XCD than the tall strip (pick_xcd_map; the host only passes px when
// both dimensions divide and the grid is a multiple of 8).
__device__ __forceinline__ void tile_coords(int b, int nwg, int tiles_m, int tiles_n, int xmap, int& tm, int& tn) {
  const int xcd = b % kXcds;
  const int q = nwg / kXcds, rem = nwg % kXcds;
  const int wgid = (xcd < rem ? xcd * (q + 1) : rem * (q + 1) + (xcd - rem) * q) + b / kXcds;
  if (xmap & 0xFF) {
    const int px = xmap & 0xFF, GM = (xmap >> 8) & 0xFF;     // bands, rows per group inside the block
    const int py = kXcds / px;
    const int bm = tiles_m / px, bn = tiles_n / py;
    const int per = bm * bn;
    const int x = wgid / per, l = wgid - x * per;
    const int per_group = GM * bn;
    const int g = l / per_group;
    const int gsize = min(bm - g * GM, GM);
    const int r = l - g * per_group;
    tm = (x / py) * bm + g * GM + r % gsize;
    tn = (x % py) * bn + r / gsize;
    return;
  }
  const int per_group = GROUP_M * tiles_n;
  const int group = wgid / per_group;
  const int first_m = group * GROUP_M;
  const int gsize = min(tiles_m - first_m, GROUP_M);
  tm = first_m + (wgid % per_group) % gsize;
  tn = (wgid % per_group) / gsize;
}

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

// XCC id of the executing workgroup (HW_REG_XCC_ID): tests/test_gpu_native.py reads it through
// xcd_probe to check the round-robin block -> XCD dispatch the tile order relies on.
__device__ __forceinline__ int xcc_id() { return __builtin_amdgcn_s_getreg((3 << 11) | 20) & 0xF; }

__global__ void xcd_probe_kernel(int* out) {
  if (threadIdx.x == 0) out[blockIdx.x] = xcc_id();
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

// Wide epilogue of a BM x BN block tile (all kernels below): the bf16 tile is assembled in the
// (then idle) staging LDS and stored as whole rows with 16-B stores instead of each lane's
// scattered 8-B pieces (the D = C^T layout gives a lane 4 consecutive columns of one row).
// Image: row r at r * BN * 2 bytes; its 8-B slot s (4 columns) at slot s ^ ((r & MASK) << 1)
// with MASK = min(15, BN / 8 - 1): a ds_write_b64 lane group (16 rows, one column) spreads
// over 8 bank pairs (2-way), and the 16-B chunk c of row r stays whole at chunk c ^ (r & MASK)
// for the ds_read_b128 pass.  Caller: every wave past its last LDS read, no LDS-DMA in flight.
template <int BN>
__device__ __forceinline__ void wide_put(char* img, int row, int col, bf16x4 o) {
  constexpr int MASK = (BN / 8 - 1) < 15 ? (BN / 8 - 1) : 15;
  const int slot = (col >> 2) ^ ((row & MASK) << 1);
  *reinterpret_cast<bf16x4*>(img + row * (BN * 2) + slot * 8) = o;
}

template <int BM, int BN, int NT>
__device__ __forceinline__ void wide_store(const char* img, __bf16* __restrict__ C, int ldc, int m0, int n0) {
  constexpr int MASK = (BN / 8 - 1) < 15 ? (BN / 8 - 1) : 15;
  constexpr int CPR = BN / 8;                           // 16-B chunks per row
  static_assert(BM * CPR % NT == 0, "wide epilogue split");
#pragma unroll
  for (int k = 0; k < BM * CPR / NT; ++k) {
    const int id = k * NT + (int)threadIdx.x;
    const int row = id / CPR, c = id % CPR;
    const bf16x8 v = *reinterpret_cast<const bf16x8*>(img + row * (BN * 2) + ((c ^ (row & MASK)) << 4));
    *reinterpret_cast<bf16x8*>(C + (size_t)(m0 + row) * ldc + n0 + c * 8) = v;
  }
}

template <int BM, int BN, int WGM, int WGN, int OCC, bool RELU, bool BIAS, int STAGES = 2, int KT = BK,
          bool HOIST = false, bool WIDE = false>
__global__ void __launch_bounds__(WGM * WGN * 64, OCC)
gemm_bf16_nt_kernel(const __bf16* __restrict__ A, const __bf16* __restrict__ Bt, __bf16* __restrict__ C,
                    const float* __restrict__ bias, int M, int N, int K, int lda, int ldb, int ldc, int xmap) {
  constexpr int NT = WGM * WGN * 64;
  static_assert(KT == 32 || KT == 64, "K tile");
  constexpr int A_BYTES = BM * KT * 2, B_BYTES = BN * KT * 2;
  constexpr int WTM = BM / WGM, WTN = BN / WGN;       // wave tile
  constexpr int MI = WTM / 16, NJ = WTN / 16;
  static_assert(BM * KT * 2 / 16 % NT == 0 && BN * KT * 2 / 16 % NT == 0, "stage split");
  static_assert(STAGES >= 2 && STAGES <= 4, "stages");
  constexpr int LOADS = (BM + BN) * KT * 2 / 16 / NT;    // glds per thread per K-tile
  __shared__ __attribute__((aligned(16))) char smem[STAGES * (A_BYTES + B_BYTES)];

  // ---- XCD-aware tile order (tile_coords) -------------------------------------------
  int tm, tn;
  tile_coords(blockIdx.x, gridDim.x, M / BM, N / BN, xmap, tm, tn);
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

  if constexpr (WIDE) {
    static_assert(BM * BN * 2 <= STAGES * (A_BYTES + B_BYTES), "wide epilogue image exceeds the staging LDS");
    __syncthreads();                          // every wave past its last fragment read
#pragma unroll
    for (int j = 0; j < NJ; ++j) {
      const int col = wn * WTN + j * 16 + fk * 4;
      f32x4 bv = f32x4{0.f, 0.f, 0.f, 0.f};
      if (BIAS) bv = *reinterpret_cast<const f32x4*>(bias + n0 + col);
#pragma unroll
      for (int i = 0; i < MI; ++i) {
        f32x4 v = acc[i][j] + bv;
        bf16x4 o;
#pragma unroll
        for (int r = 0; r < 4; ++r) o[r] = (__bf16)(RELU ? (v[r] > 0.f ? v[r] : 0.f) : v[r]);
        wide_put<BN>(smem, wm * WTM + i * 16 + frow, col, o);
      }
    }
    __syncthreads();
    wide_store<BM, BN, NT>(smem, C, ldc, m0, n0);
    return;
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

// ---------------------------------------------------------------------------------------
// FP8 (OCP e4m3fn) GEMM: C[M,N] = act(A[M,K] . Bt[N,K]^T (+bias)), fp8 in / f32 accumulate /
// bf16 out, on the block-scaled MFMA v_mfma_scale_f32_16x16x128_f8f6f4 with unit scales
// (e8m0 127 = 2^0): twice the bf16 rate per clock (MI355X_MICROARCH.md "Matrix cores"),
// where the non-scaled 16x16x32 fp8 form only matches bf16.  A K tile is 128 fp8 = 128 B per
// row -- byte for byte the bf16 kernel's 64-deep tile -- so staging reuses stage_tile (the
// fp8 rows are moved as 16-byte chunks through a bf16 view with half the K) and the same
// XOR-swizzled, conflict-free LDS image.  One MFMA consumes a whole K tile: lane group
// fk = lane>>4 supplies 32 k values, read as the two 16-B chunks 2fk and 2fk+1 of its row.
// Which k a lane byte stands for does not matter as long as A and B agree (they are read
// with the same map), so no k permutation is needed.  Epilogue as the bf16 kernel (D = C^T
// layout, packed bf16x4 stores, fused bias + ReLU).
typedef int i32x8 __attribute__((ext_vector_type(8)));
typedef int i32x4 __attribute__((ext_vector_type(4)));
constexpr int kUnitScale = 0x7F7F7F7F;   // e8m0 1.0 in every byte (any OPSEL picks 127)

__device__ __forceinline__ i32x8 lds_frag_fp8(const char* lds_tile, int row, int fk) {
  const i32x4 lo = __builtin_bit_cast(i32x4, lds_frag<BK>(lds_tile, row, 2 * fk));
  const i32x4 hi = __builtin_bit_cast(i32x4, lds_frag<BK>(lds_tile, row, 2 * fk + 1));
  return i32x8{lo[0], lo[1], lo[2], lo[3], hi[0], hi[1], hi[2], hi[3]};
}

template <int BM, int BN, int WGM, int WGN, int OCC, bool RELU, bool BIAS>
__global__ void __launch_bounds__(WGM * WGN * 64, OCC)
gemm_fp8_nt_kernel(const uint8_t* __restrict__ A8, const uint8_t* __restrict__ B8, __bf16* __restrict__ C,
                   const float* __restrict__ bias, int M, int N, int K, int lda, int ldb, int ldc) {
  constexpr int NT = WGM * WGN * 64;
  constexpr int KT8 = 128;                             // fp8 elements (bytes) per K tile
  constexpr int A_BYTES = BM * KT8, B_BYTES = BN * KT8;
  constexpr int WTM = BM / WGM, WTN = BN / WGN;
  constexpr int MI = WTM / 16, NJ = WTN / 16;
  static_assert(A_BYTES / 16 % NT == 0 && B_BYTES / 16 % NT == 0, "stage split");
  __shared__ __attribute__((aligned(16))) char smem[2 * (A_BYTES + B_BYTES)];
  // bf16 views of the fp8 rows for the 16-byte glds staging (K and ld halved)
  const __bf16* A = reinterpret_cast<const __bf16*>(A8);
  const __bf16* Bt = reinterpret_cast<const __bf16*>(B8);
  const int lda2 = lda / 2, ldb2 = ldb / 2;

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
  const int frow = lane & 15;
  const int fk = lane >> 4;
  auto stage = [&](int t, int buf) {
    stage_tile<BM, NT, BK>(A, lda2, m0, t * BK, tileA(buf), wave, lane);
    stage_tile<BN, NT, BK>(Bt, ldb2, n0, t * BK, tileB(buf), wave, lane);
  };
  auto compute = [&](const char* a_t, const char* b_t) {
    i32x8 af[MI], bf[NJ];
#pragma unroll
    for (int j = 0; j < NJ; ++j) bf[j] = lds_frag_fp8(b_t, wn * WTN + j * 16 + frow, fk);
#pragma unroll
    for (int i = 0; i < MI; ++i) af[i] = lds_frag_fp8(a_t, wm * WTM + i * 16 + frow, fk);
    __builtin_amdgcn_s_setprio(1);
#pragma unroll
    for (int i = 0; i < MI; ++i)
#pragma unroll
      for (int j = 0; j < NJ; ++j)
        acc[i][j] = __builtin_amdgcn_mfma_scale_f32_16x16x128_f8f6f4(bf[j], af[i], acc[i][j], 0, 0, 0, kUnitScale,
                                                                      0, kUnitScale);
    __builtin_amdgcn_s_setprio(0);
  };
  const int nt = K / KT8;
  stage(0, 0);
  __syncthreads();
  int buf = 0;
  for (int t = 0; t < nt; ++t) {
    if (t + 1 < nt) stage(t + 1, buf ^ 1);
    compute(tileA(buf), tileB(buf));
    __syncthreads();
    buf ^= 1;
  }
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

// ---------------------------------------------------------------------------------------
// 256x256 "8-phase" GEMM for lone, large GEMMs (a whole-GPU Guaranteed pod): 8 waves as
// 2 (M) x 4 (N) groups, one block per CU, 128 KiB LDS = 2 K-tile buffers x {A0, A1, B0, B1}
// half-tiles of 128 rows x 64 k.  Wave (wr, wc) owns rows h*128 + wr*64 + [0, 64) and
// columns g*128 + wc*32 + [0, 32) for h, g in {0, 1}, so a (h, g) output quadrant touches
// only half-tiles A_h and B_g.  Each K-tile is 4 phases, each phase = its fragment reads,
// ONE half-tile of glds (2 x 16 B per thread), a barrier, 16 MFMAs, a barrier:
//
//   phase 1: quadrant (0,0)  reads A0 (8 x ds_read_b128) + B0 (4, kept in registers)
//   phase 2: quadrant (0,1)  reads B1 (4)
//   phase 3: quadrant (1,1)  reads A1 (8)
//   phase 4: quadrant (1,0)  no reads (A1 and B0 already in registers)
//
// Half-tile j (A0, B0, B1, A1 = 0..3) of K-tile u is staged in global phase 4u - 5 + j
// (K-tile u runs phases 4u+1 .. 4u+4; the prologue covers the phases <= 0), so every half-tile
// is restaged >= 2 phases after its last read of K-tile u-2 (WAR with the two wave groups
// staggered by one barrier) and is retired by a counted vmcnt at phase 2 or 4 at least one
// phase before its first read (RAW): three half-tiles stay in flight (vmcnt(6)) in steady
// state, fewer as the K loop drains.  The wr = 1 group runs one barrier behind the wr = 0
// group, so on every SIMD (one wave of each group) one wave issues its reads and glds
// while the other runs MFMAs.
__device__ __forceinline__ void wait_vmcnt_rt(int n) {
  // s_waitcnt takes an immediate: n (loads allowed in flight) is 0 .. 6
  if (n >= 6) wait_vmcnt<6>();
  else if (n == 5) wait_vmcnt<5>();
  else if (n == 4) wait_vmcnt<4>();
  else if (n == 3) wait_vmcnt<3>();
  else if (n == 2) wait_vmcnt<2>();
  else if (n == 1) wait_vmcnt<1>();
  else wait_vmcnt<0>();
}

// SPLIT (split-K for lone GEMMs with fewer 256x256 tiles than CUs, e.g. tall-K 2048x4096x8192):
// the grid is tiles x S; block (s, tile) multiplies the K slice [s*K, (s+1)*K) (K = the slice
// length here) and stores its fp32 partial tile to ws[s] (row-major, ld = N) instead of C;
// splitk_reduce then sums the S partials, adds bias, applies the activation and writes bf16.
//
// BN = 128: the same 8-phase schedule on a 256 x 128 block tile (tile 13) for the GEMMs of a
// co-running pod that are too small to give every CU of its share a 256 x 256 tile (the
// catalog's M = 1024 layers at a 64-CU share): B half-tiles are 64 rows (one glds per thread
// instead of two), each wave owns 128 x 32 outputs (one 16-column fragment per B half), and the
// counted waits follow the unequal half-tile sizes (inflight_8ph).  Half the blocks of the
// 128 x 128 tile, each staging 85 FLOP per byte instead of 64, with the two staggered wave groups
// of the 8-phase kernel instead of one lock-step group.
template <int BN>
struct Tile8ph {
  static constexpr int HALF_A = 128 * 64 * 2;          // bytes of an A half-tile image (128 rows x 64 k)
  static constexpr int HALF_B = (BN / 2) * 64 * 2;     // a B half-tile (BN/2 rows x 64 k)
  static constexpr int BUF = 2 * HALF_A + 2 * HALF_B;  // one K-tile: A0 A1 B0 B1
  static constexpr int OA0 = 0, OA1 = HALF_A, OB0 = 2 * HALF_A, OB1 = 2 * HALF_A + HALF_B;
  static constexpr int NJ = BN / 128;                  // 16-column fragments per wave per B half
  static constexpr int WCOLS = BN / 8;                 // columns per wave per B half
  static constexpr int GA = 2, GB = BN / 128;          // glds per thread for an A / B half-tile
};

// glds (per thread) allowed in flight at the counted wait of global phase p: those of phases
// p-2 .. p that exist (phase q stages half-tile j = (q + 5) mod 4 -- A0, B0, B1, A1 for j = 0..3
// -- and nothing after last_stage)
template <int BN>
__device__ __forceinline__ int inflight_8ph(int p, int last_stage) {
  int n = 0;
#pragma unroll
  for (int q = p - 2; q <= p; ++q) {
    if (q > last_stage) continue;
    const int j = ((q + 5) % 4 + 4) % 4;
    n += (j == 0 || j == 3) ? Tile8ph<BN>::GA : Tile8ph<BN>::GB;
  }
  return n;
}

template <bool RELU, bool BIAS, bool PEEL = false, bool WIDE = false, bool SPLIT = false, int BN = 256>
__global__ void __launch_bounds__(512, 1)
gemm_bf16_nt_256_8ph(const __bf16* __restrict__ A, const __bf16* __restrict__ Bt, __bf16* __restrict__ C,
                     const float* __restrict__ bias, int M, int N, int K, int lda, int ldb, int ldc, int xmap,
                     float* __restrict__ ws = nullptr) {
  static_assert(BN == 256 || BN == 128, "8-phase block tile is 256 x 256 or 256 x 128");
  using TL = Tile8ph<BN>;
  constexpr int BUF = TL::BUF;
  constexpr int OA0 = TL::OA0, OA1 = TL::OA1, OB0 = TL::OB0, OB1 = TL::OB1;
  constexpr int NJ = TL::NJ;
  __shared__ __attribute__((aligned(16))) char smem[2 * BUF];

  int nwg = gridDim.x;
  int b = blockIdx.x;
  int split = 0;
  if constexpr (SPLIT) {
    nwg = (M / 256) * (N / BN);                    // tiles; the S slices of one tile are nwg apart
    split = b / nwg;
    b -= split * nwg;
    A += (size_t)split * K;
    Bt += (size_t)split * K;
  }
  int tm, tn;
  tile_coords(b, nwg, M / 256, N / BN, xmap, tm, tn);
  const int m0 = tm * 256, n0 = tn * BN;

  const int wave = __builtin_amdgcn_readfirstlane(threadIdx.x / kWave);
  const int lane = threadIdx.x & (kWave - 1);
  const int wr = wave >> 2, wc = wave & 3;
  const int frow = lane & 15, fk = lane >> 4;

  f32x4 acc[2][4][2][NJ];                          // [h][mi][g][nj]
#pragma unroll
  for (int h = 0; h < 2; ++h)
#pragma unroll
    for (int i = 0; i < 4; ++i)
#pragma unroll
      for (int g = 0; g < 2; ++g)
#pragma unroll
        for (int j = 0; j < NJ; ++j) acc[h][i][g][j] = f32x4{0.f, 0.f, 0.f, 0.f};
  bf16x8 ar[2][4], b0r[2][NJ], b1r[2][NJ];          // [kk][mi], [kk][nj]

  const int T = K / 64;
  const int last_stage = 4 * T - 6;                // global phase of the last glds
  // half-tile j of K-tile u: A rows (j = 0, 3) or B rows (j = 1, 2)
  auto stage = [&](int u, int j) {
    char* dst = smem + (u & 1) * BUF + (j == 0 ? OA0 : j == 3 ? OA1 : j == 1 ? OB0 : OB1);
    if (j == 0 || j == 3)
      stage_tile<128, 512, 64>(A, lda, m0 + (j == 3 ? 128 : 0), u * 64, dst, wave, lane);
    else
      stage_tile<BN / 2, 512, 64>(Bt, ldb, n0 + (j == 2 ? BN / 2 : 0), u * 64, dst, wave, lane);
  };
  auto read_a = [&](const char* half) {
#pragma unroll
    for (int kk = 0; kk < 2; ++kk)
#pragma unroll
      for (int i = 0; i < 4; ++i) ar[kk][i] = lds_frag<64>(half, wr * 64 + i * 16 + frow, kk * 4 + fk);
  };
  auto read_b = [&](const char* half, bf16x8 (&br)[2][NJ]) {
#pragma unroll
    for (int kk = 0; kk < 2; ++kk)
#pragma unroll
      for (int j = 0; j < NJ; ++j) br[kk][j] = lds_frag<64>(half, wc * TL::WCOLS + j * 16 + frow, kk * 4 + fk);
  };
  auto barrier = [] {
    __builtin_amdgcn_sched_barrier(0);
    __builtin_amdgcn_s_barrier();
    __builtin_amdgcn_sched_barrier(0);
  };
  auto mfma_quadrant = [&](int h, int g, bf16x8 (&br)[2][NJ]) {
    __builtin_amdgcn_s_setprio(1);
#pragma unroll
    for (int kk = 0; kk < 2; ++kk)
#pragma unroll
      for (int i = 0; i < 4; ++i)
#pragma unroll
        for (int j = 0; j < NJ; ++j)
          acc[h][i][g][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(br[kk][j], ar[kk][i], acc[h][i][g][j], 0, 0, 0);
    __builtin_amdgcn_s_setprio(0);
  };
  // loads allowed in flight at the wait of global phase p: the glds of phases p-2 .. p that
  // exist (BN = 256: 2 per phase; BN = 128: 2 for an A half, 1 for a B half)
  auto inflight = [&](int p) { return inflight_8ph<BN>(p, last_stage); };
  // steady state: phase 2 of a K-tile waits with B0, B1, A1 in flight; phase 4 with A1, A0, B0
  constexpr int STEADY2 = 2 * TL::GB + TL::GA;
  constexpr int STEADY4 = 2 * TL::GA + TL::GB;

  // prologue: K-tile 0 and half-tiles A0, B0 of K-tile 1 (phases -5 .. 0)
#pragma unroll
  for (int j = 0; j < 4; ++j) stage(0, j);
  stage(1, 0);
  stage(1, 1);
  wait_vmcnt<TL::GA + TL::GB>();                   // K-tile 0 landed; K-tile 1's A0/B0 in flight
  barrier();
  if (wr == 1) barrier();                          // group 1 runs one barrier behind

  int t0 = 0;
  if constexpr (PEEL) {
    // Steady state (t <= T-3): every phase stages its half-tile and three half-tiles stay in
    // flight, so the waits are constant counts and nothing branches -- the generic loop below
    // only runs the last two K-tiles, where the pipeline drains.
    for (; t0 + 2 < T; ++t0) {
      const char* cur = smem + (t0 & 1) * BUF;
      read_b(cur + OB0, b0r);
      __builtin_amdgcn_sched_barrier(0);
      read_a(cur + OA0);
      stage(t0 + 1, 2);
      barrier();
      mfma_quadrant(0, 0, b0r);
      barrier();
      read_b(cur + OB1, b1r);
      stage(t0 + 1, 3);
      wait_vmcnt<STEADY2>();
      barrier();
      mfma_quadrant(0, 1, b1r);
      barrier();
      read_a(cur + OA1);
      stage(t0 + 2, 0);
      barrier();
      mfma_quadrant(1, 1, b1r);
      barrier();
      stage(t0 + 2, 1);
      wait_vmcnt<STEADY4>();
      barrier();
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
      for (int j = 0; j < NJ; ++j) {
        const int col = n0 + g * (BN / 2) + wc * TL::WCOLS + j * 16 + fk * 4;
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
    // Wide epilogue (wide_put / wide_store): the whole 256 x BN bf16 block tile is assembled in
    // LDS (at most the LDS the K loop used; every wave is past its last LDS read and every
    // LDS-DMA has retired -- the drained pipeline's vmcnt(0) -- once the now-aligned wave
    // groups meet at one more barrier), then whole rows go out with 16-B stores: coalesced
    // stores instead of scattered 8-B ones (the scattered tail cost 7-20 % of the 256 x 256
    // kernel at K = 8192 .. 2048).
    static_assert(256 * BN * 2 <= 2 * BUF, "wide epilogue image exceeds the staging LDS");
    barrier();
#pragma unroll
    for (int g = 0; g < 2; ++g)
#pragma unroll
      for (int j = 0; j < NJ; ++j) {
        const int col = g * (BN / 2) + wc * TL::WCOLS + j * 16 + fk * 4;
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
            wide_put<BN>(smem, h * 128 + wr * 64 + i * 16 + frow, col, o);
          }
      }
    __syncthreads();
    wide_store<256, BN, 512>(smem, C, ldc, m0, n0);
    return;
  }

  // epilogue (D = C^T layout, as in gemm_bf16_nt_kernel): lane holds 4 consecutive columns
#pragma unroll
  for (int g = 0; g < 2; ++g)
#pragma unroll
    for (int j = 0; j < NJ; ++j) {
      const int col = n0 + g * (BN / 2) + wc * TL::WCOLS + j * 16 + fk * 4;
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

// Tile 14 (built for the lone-GEMM study; the co-run default since round 6,
// policy 10): the 256 x 256 block tile on FOUR waves of 128 x 128 -- hipBLASLt's shape
// (profiles/r05_lone_gemm_pmc/: 0.25 LDS reads per MFMA instead of the 8-phase kernel's 0.375).
// Tiles 15 / 16 are the same kernel on 256 x 128 / 128 x 128 blocks (A/B knobs).  Round 5's versions of this
// structure stalled once per K-tile (1,016 TF) or spilled: the compiler kept a VGPR copy of the
// 256 accumulators next to the AGPRs.  Here the MFMA is inline asm with the accumulator tied to
// an AGPR ("+a"), so the accumulators cannot leave the AGPR file.
__device__ __forceinline__ void mfma_agpr(f32x4& acc, const bf16x8& b, const bf16x8& a) {
  asm volatile("v_mfma_f32_16x16x32_bf16 %0, %1, %2, %0" : "+a"(acc) : "v"(b), "v"(a));
}

// The compiler cannot see that the asm above is an MFMA, so it cannot insert the wait states
// between an MFMA and a VALU access of its accumulator: these fences pin them.  An empty volatile
// asm that "modifies" every accumulator keeps the compiler's own accumulator accesses on their
// side of it (volatile asm statements keep their order).  agpr_after_init: after the accumulators'
// bias / zero fill, before the first MFMA; agpr_before_read: after the last MFMA, before the
// epilogue reads.
template <int NI, int NJ>
__device__ __forceinline__ void agpr_fence(f32x4 (&acc)[NI][NJ]) {
#pragma unroll
  for (int i = 0; i < NI; ++i)
#pragma unroll
    for (int j = 0; j < NJ; ++j) asm volatile("" : "+a"(acc[i][j]));
}
template <int NI, int NJ>
__device__ __forceinline__ void agpr_after_init(f32x4 (&acc)[NI][NJ]) {
  agpr_fence(acc);
  asm volatile("s_nop 7" ::: "memory");
}
template <int NI, int NJ>
__device__ __forceinline__ void agpr_before_read(f32x4 (&acc)[NI][NJ]) {
  asm volatile("s_nop 7\n\ts_nop 7\n\ts_nop 7" ::: "memory");
  agpr_fence(acc);
}

// The schedule: 64-deep operand tiles in a 5-slot LDS ring.  Timing probes of a first version
// (32-deep sub-tiles in 4 slots, one barrier per 32 k; profiles/r06_lone_gemm/): its LDS-DMA cost
// the single wave per SIMD ~0.22 ms of 0.79 at 8192^3, and fetching 8 rows x 128 B per
// instruction (whole cache lines) instead of 16 rows x 64 B saved ~0.09 ms of that.  So the
// operand tiles here are BM / BN rows x 64 k (128-B rows, stage_tile's KT = 64 image and swizzle):
// A_t and B_t take ring slots (2t) % 5 and (2t+1) % 5 of the larger tile's size (256 x 256: 32 KiB
// each, 160 KiB = the CU's whole LDS; 128 x 128: 80 KiB, two blocks per CU).  K-tile t runs two
// halves of (BM / 32) x (BN / 32) MFMAs (64 at 256 x 256):
//   h0: MFMAs of k-step 0 (fragment set 0), reads of k-step 1 into set 1, glds of A_{t+2}
//       (into B_{t-1}'s slot);
//   lgkmcnt(0) + vmcnt (A_{t+1}, B_{t+1} landed; A_{t+2} may fly) + ONE barrier;
//   h1: MFMAs of k-step 1 (set 1), reads of K-tile t+1's k-step 0 into set 0, glds of B_{t+2}
//       (into A_t's slot).
// The barrier certifies for every wave that A_{t+1} / B_{t+1} landed (RAW for h1's reads) and
// that every read of A_t and B_{t-1} retired (WAR for the next two glds groups), so one barrier
// per 128 MFMAs suffices.
// PRIO (A/B arm, set_w4_prio): the waves run at s_setprio 1 from start to end, ahead of co-resident
// stream waves of other pods in the SIMD's issue arbitration.
template <bool RELU, bool BIAS, int PROBE = 0, bool PRIO = false, int BN = 256, int BM = 256>
__global__ void __launch_bounds__(256, BM == 128 ? 2 : 1)
gemm_bf16_nt_256_w4l(const __bf16* __restrict__ A, const __bf16* __restrict__ Bt, __bf16* __restrict__ C,
                     const float* __restrict__ bias, int M, int N, int K, int lda, int ldb, int ldc, int xmap) {
  static_assert((BM == 256 && (BN == 256 || BN == 128)) || (BM == 128 && BN == 128),
                "4-wave block tile is 256 x 256, 256 x 128 or 128 x 128");
  constexpr int KT = 64, NSLOT = 5;
  constexpr int SLOT = (BM > BN ? BM : BN) * KT * 2;  // one ring slot: the larger operand tile
  constexpr int GA = BM * KT * 2 / 16 / 256;       // glds per thread for an A tile (8 or 4)
  constexpr int GB = BN * KT * 2 / 16 / 256;       // ... for a B tile (8 or 4)
  constexpr int WM = BM / 2, WN = BN / 2;          // wave tile (2 x 2 waves)
  constexpr int NI = WM / 16, NJ = WN / 16;        // 16-row / 16-column fragments per wave
  constexpr int NG = NI * NJ / 4;                  // groups of 4 MFMAs per half
  __shared__ __attribute__((aligned(16))) char smem[NSLOT * SLOT];

  int tm, tn;
  tile_coords(blockIdx.x, gridDim.x, M / BM, N / BN, xmap, tm, tn);
  const int m0 = tm * BM, n0 = tn * BN;
  const int wave = __builtin_amdgcn_readfirstlane(threadIdx.x / kWave);
  const int lane = threadIdx.x & (kWave - 1);
  const int wr = wave >> 1, wc = wave & 1;
  const int frow = lane & 15, fk = lane >> 4;

  // the accumulators start at the bias (D = C^T layout: 4 consecutive columns per lane), so the
  // epilogue holds no bias registers (at BN = 256 that kept the kernel at 148 VGPRs instead of 129)
  f32x4 acc[NI][NJ];
#pragma unroll
  for (int j = 0; j < NJ; ++j) {
    f32x4 b0 = f32x4{0.f, 0.f, 0.f, 0.f};
    if constexpr (BIAS) b0 = *reinterpret_cast<const f32x4*>(bias + n0 + wc * WN + j * 16 + fk * 4);
#pragma unroll
    for (int i = 0; i < NI; ++i) acc[i][j] = b0;
  }
  agpr_after_init(acc);
  if constexpr (PRIO) __builtin_amdgcn_s_setprio(1);
  // BN = 256: one A fragment set.  The MFMAs run row by row, so A fragment i is dead after row i
  // and the next k-step's fragment i is read into the same registers right behind it; B keeps two
  // sets.  96 fragment VGPRs instead of 128 put the kernel at 384 registers, so three 38-VGPR
  // stream waves of other pods fit beside each of its waves instead of two.
  constexpr bool SINGLE_A = NI == 8 && NJ == 8;
  bf16x8 fa[SINGLE_A ? 1 : 2][NI], fb[2][NJ];
  const int T = K / KT;                             // >= 2

  // piece q of operand tile X_u (B if isb): rows (q * 256 + wave * 64 + lane) >> 3, 8 per
  // instruction, by buffer_load ... lds through one descriptor per operand block: the per-thread
  // part is one 32-bit voffset per operand ((r >> 1) & 7 does not depend on q), the piece and
  // K-tile parts an SGPR soffset (the global_load_lds form with 64-bit per-lane addresses: within
  // 1-2 %, profiles/r06_lone_gemm/)
  const int rr = (wave * 64 + lane) >> 3, kq = ((wave * 64 + lane) & 7) ^ ((rr >> 1) & 7);
  const int voA = rr * lda * 2 + kq * 16, voB = rr * ldb * 2 + kq * 16;
  const auto rsA = __builtin_amdgcn_make_buffer_rsrc(const_cast<__bf16*>(A + (size_t)m0 * lda), 0, BM * lda * 2, 0x00020000);
  const auto rsB = __builtin_amdgcn_make_buffer_rsrc(const_cast<__bf16*>(Bt + (size_t)n0 * ldb), 0, BN * ldb * 2, 0x00020000);
  auto glds = [&](int u, bool isb, int q) {
    char* dst = smem + ((2 * u + (isb ? 1 : 0)) % NSLOT) * SLOT + (q * 256 + wave * 64) * 16;
    const int so = q * 32 * (isb ? ldb : lda) * 2 + u * KT * 2;
    __builtin_amdgcn_raw_ptr_buffer_load_lds(isb ? rsB : rsA, (lptr_t)dst, 16, isb ? voB : voA, so, 0, 0);
  };
  auto slot = [&](int u, bool isb) -> const char* { return smem + ((2 * u + (isb ? 1 : 0)) % NSLOT) * SLOT; };
  auto barrier = [] {
    __builtin_amdgcn_sched_barrier(0);
    __builtin_amdgcn_s_barrier();
    __builtin_amdgcn_sched_barrier(0);
  };

  // prologue: A_0 B_0 A_1 B_1 in flight; wait for A_0 / B_0; k-step 0 of K-tile 0 into set 0
#pragma unroll
  for (int u = 0; u < 2; ++u)
  {
#pragma unroll
    for (int q = 0; q < GA; ++q) glds(u, false, q);
#pragma unroll
    for (int q = 0; q < GB; ++q) glds(u, true, q);
  }
  wait_vmcnt<GA + GB>();
  barrier();
#pragma unroll
  for (int q = 0; q < NI; ++q) fa[0][q] = lds_frag<KT>(smem, wr * WM + q * 16 + frow, fk);
#pragma unroll
  for (int q = 0; q < NJ; ++q) fb[0][q] = lds_frag<KT>(smem + SLOT, wc * WN + q * 16 + frow, fk);

  // (Measured and removed: the four waves issuing their LDS-DMA pieces at different points -- in
  // pairs at groups w, w + 4, ... for wave w (1,277 vs 1,483 TF/s lone, -2.7 % pods/s) or the odd
  // waves in the odd groups (1,282 vs 1,493, -2.2 %); the waves' lockstep issue is the faster one,
  // profiles/r06_lone_gemm/stagger/, parity/.)
  // one half: 8 x NJ MFMAs on set S (k-step S of K-tile t) in NG groups of 4; the 8 + NJ reads of
  // (RU, k-step S^1) into set S^1 when RD, spread evenly (BN = 256: one per group); the glds of
  // operand tile (t+2, X = S) when ST, spread evenly (BN = 256: every second group; other
  // placements -- the glds in the odd groups, reads and glds in separate halves -- measured
  // 1-2 % slower, profiles/r06_lone_gemm/)
  auto half = [&](auto sc, auto rdc, auto stc, int t) {
    constexpr int S = decltype(sc)::value;
    constexpr bool RD = decltype(rdc)::value, ST = decltype(stc)::value;
    const int ru = S == 0 ? t : t + 1;             // h0 reads k-step 1 of t, h1 k-step 0 of t+1
    const char* ta = slot(ru, false);
    const char* tb = slot(ru, true);
    constexpr int NR = NI + NJ, NS = S == 0 ? GA : GB;
    constexpr int SA = SINGLE_A ? 0 : S;           // A set in use
#pragma unroll
    for (int g = 0; g < NG; ++g) {
#pragma unroll
      for (int m = 0; m < 4; ++m) {
        const int i = (g * 4 + m) / NJ, j = (g * 4 + m) % NJ;
        mfma_agpr(acc[i][j], fb[S][j], fa[SA][i]);
      }
      if constexpr (RD && SINGLE_A) {              // row g/2 done: its next A fragment; B at even groups
        if (g & 1) fa[0][g >> 1] = lds_frag<KT>(ta, wr * WM + (g >> 1) * 16 + frow, (S ^ 1) * 4 + fk);
        else fb[S ^ 1][g >> 1] = lds_frag<KT>(tb, wc * WN + (g >> 1) * 16 + frow, (S ^ 1) * 4 + fk);
      } else if constexpr (RD) {
#pragma unroll
        for (int q = 0; q < NR; ++q) {
          if (q * NG / NR != g) continue;
          if (q < NI) fa[S ^ 1][q] = lds_frag<KT>(ta, wr * WM + q * 16 + frow, (S ^ 1) * 4 + fk);
          else fb[S ^ 1][q - NI] = lds_frag<KT>(tb, wc * WN + (q - NI) * 16 + frow, (S ^ 1) * 4 + fk);
        }
      }
      if constexpr (ST) {
#pragma unroll
        for (int p = 0; p < NS; ++p)
          if (p * NG / NS == g) glds(t + 2, S == 1, p);
      }
      __builtin_amdgcn_sched_barrier(0);
    }
  };
  auto sync = [&](auto wc_) {
    __builtin_amdgcn_s_waitcnt(0xC07F);            // lgkmcnt(0): this wave's reads retired
    wait_vmcnt<decltype(wc_)::value>();
    barrier();
  };
  using I0 = std::integral_constant<int, 0>;
  using I1 = std::integral_constant<int, 1>;
  using IG = std::integral_constant<int, GA>;      // A_{t+2} (staged in h0) may fly at the sync
  using Y = std::true_type;
  using F = std::false_type;
  // PROBE (timing study only): bit 0 drops the steady loop's glds, bit 1 its reads (wrong results)
  using SR = std::integral_constant<bool, !(PROBE & 2)>;
  using SS = std::integral_constant<bool, !(PROBE & 1)>;
  int t = 0;
  for (; t + 3 <= T; ++t) {                         // steady: stages A_{t+2}, B_{t+2}
    half(I0{}, SR{}, SS{}, t);
    sync(IG{});
    half(I1{}, SR{}, SS{}, t);
  }
  if (t + 2 == T) {                                 // K-tile T-2: nothing left to stage
    half(I0{}, Y{}, F{}, t);
    sync(I0{});
    half(I1{}, Y{}, F{}, t);
    ++t;
  }
  half(I0{}, Y{}, F{}, t);                          // K-tile T-1
  half(I1{}, F{}, F{}, t);
  agpr_before_read(acc);
  __builtin_amdgcn_s_waitcnt(0xC07F);
  barrier();

#pragma unroll
  for (int j = 0; j < NJ; ++j) {
    const int col = wc * WN + j * 16 + fk * 4;
#pragma unroll
    for (int i = 0; i < NI; ++i) {
      const f32x4 v = acc[i][j];
      bf16x4 o;
#pragma unroll
      for (int r = 0; r < 4; ++r) o[r] = (__bf16)(RELU ? (v[r] > 0.f ? v[r] : 0.f) : v[r]);
      wide_put<BN>(smem, wr * WM + i * 16 + frow, col, o);
    }
  }
  __syncthreads();
  wide_store<BM, BN, 256>(smem, C, ldc, m0, n0);
}

// C[m, n..n+3] = act(sum_s ws[s][m, n..n+3] + bias) as bf16 -- the split-K epilogue (float4 in,
// bf16x4 out, grid-stride over M*N/4).
template <bool RELU, bool BIAS>
__global__ void __launch_bounds__(256) splitk_reduce(const float* __restrict__ ws, int S, int M, int N,
                                                     const float* __restrict__ bias, __bf16* __restrict__ C,
                                                     int ldc) {
  const size_t mn = (size_t)M * N, n4 = mn / 4;
  for (size_t q = (size_t)blockIdx.x * blockDim.x + threadIdx.x; q < n4; q += (size_t)gridDim.x * blockDim.x) {
    const size_t e = q * 4;
    f32x4 v = *reinterpret_cast<const f32x4*>(ws + e);
    for (int sp = 1; sp < S; ++sp) v += *reinterpret_cast<const f32x4*>(ws + (size_t)sp * mn + e);
    const int m = (int)(e / N), n = (int)(e % N);
    if (BIAS) v += *reinterpret_cast<const f32x4*>(bias + n);
    bf16x4 o;
#pragma unroll
    for (int r = 0; r < 4; ++r) o[r] = (__bf16)(RELU ? (v[r] > 0.f ? v[r] : 0.f) : v[r]);
    *reinterpret_cast<bf16x4*>(C + (size_t)m * ldc + n) = o;
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
// WT: the result goes out with `global_store_dwordx4 ... sc1` (write-through, the line is DROPPED
// from the XCD's L2, MI355X_MICROARCH.md "stores of each flavour") instead of a non-temporal store
// (which keeps the line in L2): a one-touch output stream then does not evict the co-running
// GEMMs' operand panels from L2 (round-6 A/B, variant 8).  Vector stores only.
template <int U, bool NT, bool WT = false>
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
        if (WT)
          asm volatile("global_store_dwordx4 %0, %1, off sc1" : : "v"(a + i), "v"(r) : "memory");
        else if (NT)
          __builtin_nontemporal_store(r, a + i);
        else
          a[i] = r;
      }
    }
  }
}

void xcd_probe(uintptr_t out, int blocks, uintptr_t stream) {
  hipLaunchKernelGGL(xcd_probe_kernel, dim3(blocks), dim3(64), 0, reinterpret_cast<hipStream_t>(stream),
                     reinterpret_cast<int*>(out));
  HIP_CHECK(hipGetLastError());
}

// 6 = auto: working set (3 arrays) <= 96 MiB -> cached 2x-unrolled loads (the stream
// stays in the 256 MiB Infinity Cache across iterations: 7.1 TB/s measured), larger ->
// non-temporal 4x (6.5 TB/s vs 6.1 for torch.add) -- profiles/r01_kernel_bench.json.
static int g_triad_variant = 6;

// 5 = non-temporal 2x (22 VGPRs), 7 = non-temporal 3x (<= 32 VGPRs): a triad wave small enough
// to fit beside an 8-phase GEMM block's 2 x 240 VGPRs per SIMD (the 4x variant's 38 VGPRs do
// not, so a CU running a 256 x 256 GEMM block takes no triad wave at all; round 6 A/B)
void set_triad_variant(int v) {
  if (v < 0 || v > 10) throw std::runtime_error("triad variant must be 0..10 (6 = auto)");
  g_triad_variant = v;
}

static void check_align(const void* p, const char* what) {
  if (reinterpret_cast<uintptr_t>(p) % 16 != 0) throw std::runtime_error(std::string(what) + " must be 16-byte aligned");
}

template <int BM, int BN, int WGM, int WGN, int OCC, int STAGES, int KT, bool HOIST, bool WIDE>
static void launch_gemm_v(const __bf16* A, const __bf16* B, __bf16* Cp, const float* bp, int M, int N, int K, int lda,
                          int ldb, int ldc, bool relu, hipStream_t s) {
  const dim3 grid((M / BM) * (N / BN)), block(WGM * WGN * 64);
  const int xmap = pick_xcd_map(M / BM, N / BN);
  if (relu && bp)
    hipLaunchKernelGGL((gemm_bf16_nt_kernel<BM, BN, WGM, WGN, OCC, true, true, STAGES, KT, HOIST, WIDE>), grid, block, 0, s,
                       A, B, Cp, bp, M, N, K, lda, ldb, ldc, xmap);
  else if (relu)
    hipLaunchKernelGGL((gemm_bf16_nt_kernel<BM, BN, WGM, WGN, OCC, true, false, STAGES, KT, HOIST, WIDE>), grid, block, 0,
                       s, A, B, Cp, bp, M, N, K, lda, ldb, ldc, xmap);
  else if (bp)
    hipLaunchKernelGGL((gemm_bf16_nt_kernel<BM, BN, WGM, WGN, OCC, false, true, STAGES, KT, HOIST, WIDE>), grid, block, 0,
                       s, A, B, Cp, bp, M, N, K, lda, ldb, ldc, xmap);
  else
    hipLaunchKernelGGL((gemm_bf16_nt_kernel<BM, BN, WGM, WGN, OCC, false, false, STAGES, KT, HOIST, WIDE>), grid, block, 0,
                       s, A, B, Cp, bp, M, N, K, lda, ldb, ldc, xmap);
}

// XCD-block tile order (tile_coords): 1 = on (px chosen per grid), 0 = the GROUP_M order over
// the whole grid (A/B knob).
static int g_xcd_blocks = 1;
static int g_xcd_group = 4;         // tile rows per group inside an XCD block
void set_xcd_blocks(int on) { g_xcd_blocks = on ? 1 : 0; }
// lone 8-phase GEMMs (whole-chip budget) in the plain GROUP_M order (1, default) or the same
// order as co-running pods (0, A/B knob)
static int g_lone_plain_order = 1;
void set_lone_plain_order(int on) { g_lone_plain_order = on ? 1 : 0; }

void set_xcd_group(int rows) {
  if (rows < 1 || rows > 64) throw std::runtime_error("xcd group rows must be 1..64");
  g_xcd_group = rows;
}

// px (XCD-block rows, 8 / px columns) minimising the strips one XCD fetches, A rows + B
// columns of its block, among the splits that divide the grid; 0 = none (legacy order).
int pick_xcd_map(int tiles_m, int tiles_n) {
  if (!g_xcd_blocks || (tiles_m * tiles_n) % kXcds) return 0;
  int best = 0, best_cost = 1 << 30;
  for (int px = 1; px <= kXcds; px *= 2) {
    const int py = kXcds / px;
    if (tiles_m % px || tiles_n % py) continue;
    const int cost = tiles_m / px + tiles_n / py;
    if (cost < best_cost) best = px, best_cost = cost;
  }
  return best ? best | (g_xcd_group << 8) : 0;
}

// Wide (LDS-staged, 16-B row stores) epilogue whenever C rows are 16-B aligned; g_wide_epi = 0
// keeps the scattered 8-B epilogue (A/B knob).
static int g_wide_epi = 1;

void set_wide_epilogue(int on) { g_wide_epi = on ? 1 : 0; }

static bool wide_ok(const __bf16* Cp, int ldc) {
  return g_wide_epi && ldc % 8 == 0 && reinterpret_cast<uintptr_t>(Cp) % 16 == 0;
}

template <int BM, int BN, int WGM, int WGN, int OCC, int STAGES = 2, int KT = BK, bool HOIST = false>
static void launch_gemm(const __bf16* A, const __bf16* B, __bf16* Cp, const float* bp, int M, int N, int K, int lda,
                        int ldb, int ldc, bool relu, hipStream_t s) {
  if (wide_ok(Cp, ldc))
    launch_gemm_v<BM, BN, WGM, WGN, OCC, STAGES, KT, HOIST, true>(A, B, Cp, bp, M, N, K, lda, ldb, ldc, relu, s);
  else
    launch_gemm_v<BM, BN, WGM, WGN, OCC, STAGES, KT, HOIST, false>(A, B, Cp, bp, M, N, K, lda, ldb, ldc, relu, s);
}

template <bool PEEL, bool WIDE, int BN = 256>
static void launch_8ph_v(const __bf16* A, const __bf16* B, __bf16* Cp, const float* bp, int M, int N, int K, int lda,
                         int ldb, int ldc, bool relu, hipStream_t s, dim3 grid, dim3 block, bool lone) {
  // a lone GEMM (the whole chip) takes the plain GROUP_M order: 0.936 vs 0.913 of hipBLASLt at
  // 4096^3, 0.94 vs 0.916 at 4096x8192x4096, 0.935 vs 0.918 at 8192^2x2048, 0.914 vs 0.92 at 8192^3
  // (7 interleaved rounds, profiles/r04_gemm_xcd/); co-running pods keep the XCD-block order
  // (+2.6 % bench pods/s, profiles/r02_xcd_block_order_ab.txt)
  const int xmap = lone ? 0 : pick_xcd_map(M / 256, N / BN);
  if (relu && bp)
    hipLaunchKernelGGL((gemm_bf16_nt_256_8ph<true, true, PEEL, WIDE, false, BN>), grid, block, 0, s, A, B, Cp, bp, M, N, K, lda, ldb, ldc, xmap, nullptr);
  else if (relu)
    hipLaunchKernelGGL((gemm_bf16_nt_256_8ph<true, false, PEEL, WIDE, false, BN>), grid, block, 0, s, A, B, Cp, bp, M, N, K, lda, ldb, ldc, xmap, nullptr);
  else if (bp)
    hipLaunchKernelGGL((gemm_bf16_nt_256_8ph<false, true, PEEL, WIDE, false, BN>), grid, block, 0, s, A, B, Cp, bp, M, N, K, lda, ldb, ldc, xmap, nullptr);
  else
    hipLaunchKernelGGL((gemm_bf16_nt_256_8ph<false, false, PEEL, WIDE, false, BN>), grid, block, 0, s, A, B, Cp, bp, M, N, K, lda, ldb, ldc, xmap, nullptr);
}

// tile 9 = the original 8-phase kernel; 10 = peeled steady-state loop + wide LDS-staged
// epilogue (when C rows are 16-B aligned, else the 8-B epilogue); 13 = tile 10's schedule on a
// 256 x 128 block tile
template <bool PEEL, int BN = 256>
static void launch_8ph(const __bf16* A, const __bf16* B, __bf16* Cp, const float* bp, int M, int N, int K, int lda,
                       int ldb, int ldc, bool relu, hipStream_t s, dim3 grid, dim3 block, bool lone) {
  const bool wide = PEEL && wide_ok(Cp, ldc);
  if (wide)
    launch_8ph_v<PEEL, true, BN>(A, B, Cp, bp, M, N, K, lda, ldb, ldc, relu, s, grid, block, lone);
  else
    launch_8ph_v<PEEL, false, BN>(A, B, Cp, bp, M, N, K, lda, ldb, ldc, relu, s, grid, block, lone);
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
// 9 = 256x256 8-phase (gemm_bf16_nt_256_8ph; needs K >= 128); 10 = the same with the
// steady-state K loop peeled (constant vmcnt, no per-phase stage conditions).
// (Measured and removed: a 256x256 kernel with 4 waves of 128x128 wave tiles, 3-4 LDS stages --
// slower than the 8-phase kernel at every catalog shape, profiles/r02_gemm_4wave_study.json.)
// 11 / 12 = 128x128 with 3 / 4 LDS stages (counted vmcnt, glds issued 2 / 3 K-tiles ahead): a
// co-running pod's small GEMM gets ~1 block per CU of its share, so its 4 waves (one per SIMD)
// must hide the MALL / HBM latency of the next tiles by depth, not by a second resident block.
// 13 = 256x128 8-phase (gemm_bf16_nt_256_8ph<..., BN = 128>, peeled + wide epilogue; K >= 128)
// 14 = 256x256 on 4 waves of 128x128 with AGPR-tied inline-asm MFMAs, 64-deep operand tiles in a
// 5-slot LDS ring (gemm_bf16_nt_256_w4l).  Forced only (K >= 128, C rows 16-B aligned): the
// lone-GEMM study of profiles/r06_lone_gemm/, level with tile 10; the co-run default since
// round 6, policy 10).  15 = the same kernel on a 256x128 block (wave tile 128 x 64; policy 11);
// 16 = on a 128x128 block (wave tile 64 x 64, 80 KiB ring, 2 blocks per CU; policy 13).
// (Also measured and removed: tile 14's schedule on v_mfma_f32_32x32x16_bf16 -- half the MFMA
// instructions, exact, but 1,434 vs 1,483 TF/s at 8192^3, profiles/r06_lone_gemm/mfma32/.)  (Also measured there and
// removed: 32-deep sub-tiles in 4 slots with one barrier per 32 or per 64 k, and register-staged
// global loads -- 5-15 % behind.)
static const int kTileBM[17] = {0, 128, 64, 64, 256, 256, 128, 64, 256, 256, 256, 128, 128, 256, 256, 256, 128};
static const int kTileBN[17] = {0, 128, 128, 64, 256, 128, 128, 128, 128, 256, 256, 128, 128, 128, 256, 128, 128};

// Tile policy.  Lone GEMMs that still get one block per CU use the 8-phase 256x256 with the
// peeled steady-state loop (tile 10; tile 9 4096^3 1306 vs 1109 TF for tile 4, 8192^3 1434 vs
// 1211, profiles/r01_gemm_big.json; peeling: +5-6 % over tile 9 on every shape,
// profiles/r02_gemm_big_peeled.json).  1 = default: co-running pods whose CU share the 256x256
// tile fills use it too -- +3.2 % pods/s in the bench once the wide epilogue and the peeled loop
// landed and every pod stream got its own HW queue (interleaved A/B, profiles/r02_gemm_share_ab.txt;
// in round 1, with the older kernels, it had been even: profiles/r01_gemm_policy_ab.txt).
// 0 = co-running pods always take the 128x128 / 2-per-CU picker.  2 = tile 4 instead of tile
// 10 for lone GEMMs.
// Default 10 since round 6: arm 1's tiles, except co-running GEMMs the 256x256 tile fills run the
// 4-wave kernel (tile 14) -- 606.3 vs 596.4 pods/s, SLOs 61.8 vs 59.0 % over 5 interleaved bench
// rounds on MI355X (600.6 vs 587.1 over 3 on another box; profiles/r06_w4corun/).
static int g_gemm_policy = 10;
// split-K for lone GEMMs whose 256x256 tiles leave CUs idle: -1 = auto (up to 8 slices), 0 = off,
// 2..8 = at most that many slices.  Off by default: on the tall-K 2048x4096x8192 the split
// kernel itself runs at ~1540 TF, but the fp32 partials + reduce pass (~144 MB of traffic) put
// the whole GEMM at 1162 TF vs 1210 for the 128x128 tile and 1290 for hipBLASLt
// (profiles/r02_gemm_big_splitk.json); a fused last-arriver fixup would need cross-XCD L2
// coherence for the partials.
static int g_split_k = 0;

void set_gemm_policy(int p) {
  if (p < 0 || p > 13) throw std::runtime_error("gemm policy must be 0..13");
  g_gemm_policy = p;
}

static int g_w4_probe = 0;
static int g_w4_prio = 0;


void set_w4_prio(int on) { g_w4_prio = on ? 1 : 0; }
void set_w4_probe(int mask) {
  if (mask < 0 || mask > 3) throw std::runtime_error("w4 probe must be 0..3");
  g_w4_probe = mask;
}

void set_gemm_tile(int t) {
  if (t < 0 || t > 16) throw std::runtime_error("gemm tile must be 0..16");
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
  const bool fits256 = (M % 256 == 0) && (N % 256 == 0) && (M / 256) * (N / 256) >= budget;
  if (alone && fits256) return g_gemm_policy == 2 ? 4 : 10;
  // 10 (A/B arm, round 6): such co-running GEMMs on the 4-wave kernel (tile 14) -- one wave per
  // SIMD at 416 registers and no LDS left over, so up to three 32-VGPR stream waves of the other
  // pods fit on each of its SIMDs, where the 8-phase kernel's two 240-register waves leave room
  // for one
  if (!alone && fits256 && (g_gemm_policy == 10 || g_gemm_policy == 11 || g_gemm_policy == 13)) return 14;
  // 12 (A/B arm): every co-running GEMM the 256 x 256 tile divides on the 4-wave kernel, even with
  // fewer tiles than its share's CUs (the other pods' stream waves take the rest)
  if (!alone && g_gemm_policy == 12 && M % 256 == 0 && N % 256 == 0) return 14;
  // 11 (A/B arm): arm 10, and a co-running GEMM too small for that but filling its share with
  // 256 x 128 blocks on the same 4-wave kernel (tile 15) instead of the 128 x 128 tile
  if (!alone && g_gemm_policy == 11 && M % 256 == 0 && N % 128 == 0 && (M / 256) * (N / 128) >= budget) return 15;
  if (!alone && fits256 && g_gemm_policy >= 1) return 10;
  // 3 / 4 (A/B arms): a co-running GEMM too small for one 256x256 tile per CU of its share
  // takes 256x128 (8 waves, 2 / 3 LDS stages) when that still gives every CU of the share a
  // block -- twice the arithmetic intensity per staged byte of 128x128 (85 vs 64 FLOP/B)
  // (exactly 3 / 4: arms 5-7 below are other tiles, and a `>= 3` test here used to shadow them)
  if (!alone && (g_gemm_policy == 3 || g_gemm_policy == 4) && M % 256 == 0 && N % 128 == 0 &&
      (M / 256) * (N / 128) >= budget)
    return g_gemm_policy == 3 ? 5 : 8;
  // 7: the co-running small GEMM on the 256x128 8-phase kernel when that gives every CU of the
  // share a block
  if (!alone && g_gemm_policy == 7 && M % 256 == 0 && N % 128 == 0 && (M / 256) * (N / 128) >= budget) return 13;
  // 5 / 6 (A/B arms): the co-running small GEMM's 128x128 tile with 3 / 4 LDS stages
  if (!alone && (g_gemm_policy == 5 || g_gemm_policy == 6) && M % 128 == 0 && N % 128 == 0 &&
      (M / 128) * (N / 128) >= budget)
    return g_gemm_policy == 5 ? 11 : 12;
  // 13 (A/B arm): arm 10, and the co-running GEMMs the 128 x 128 tile fills on the 4-wave kernel
  // at 128 x 128 (tile 16) instead of the compiler-scheduled tile 1
  if (!alone && g_gemm_policy == 13 && (M / 128) * (N / 128) >= budget) return 16;
  if ((M / 128) * (N / 128) >= per_cu * budget) return 1;
  if ((M / 64) * (N / 128) >= per_cu * budget && N % 128 == 0) return 2;
  return 3;
}

// Split-K factor for a lone GEMM (cu_budget 0 / whole chip): the 8-phase 256x256 kernel with
// S K-slices when its tiles leave CUs idle -- tiles x S <= CUs, every slice >= 1024 deep and a
// multiple of 64 -- else 1.  Needs an fp32 workspace of S*M*N floats (splitk_workspace_floats).
int pick_split_k(int M, int N, int K, int cu_budget) {
  if (g_gemm_tile) return 1;
  const bool alone = cu_budget <= 0 || cu_budget >= kCus;
  // policy 8 (A/B arm): a co-running pod's GEMM with fewer 256 x 256 tiles
  // than CUs in its share runs the 8-phase kernel split S ways along K (S = tiles needed to
  // cover the share, at most 4, every slice >= 512 deep), fp32 partials reduced by
  // splitk_reduce, instead of the 128 x 128 tile
  if (!alone && g_gemm_policy == 8) {
    if (M % 256 || N % 256) return 1;
    const int tiles = (M / 256) * (N / 256);
    if (tiles >= cu_budget) return 1;
    int S = std::min(4, (cu_budget + tiles - 1) / tiles);
    while (S > 1 && (K % (64 * S) != 0 || K / S < 512)) --S;
    return S;
  }
  if (g_split_k == 0) return 1;
  if (!alone) return 1;
  if (M % 256 || N % 256) return 1;
  const int tiles = (M / 256) * (N / 256);
  if (tiles * 2 > kCus) return 1;
  int S = std::min(g_split_k > 0 ? g_split_k : 8, kCus / tiles);
  while (S > 1 && (K % (64 * S) != 0 || K / S < 1024)) --S;
  return S;
}

size_t splitk_workspace_floats(int M, int N, int K, int cu_budget) {
  const int S = pick_split_k(M, N, K, cu_budget);
  return S > 1 ? (size_t)S * M * N : 0;
}

void set_split_k(int s) {
  if (s < -1 || s > 8) throw std::runtime_error("split_k must be 0 (off) .. 8, or -1 (auto)");
  g_split_k = s == 1 ? 0 : s;
}

template <bool RELU, bool BIAS>
static void launch_splitk(const __bf16* A, const __bf16* B, __bf16* Cp, const float* bp, float* ws, int S, int M,
                          int N, int K, int lda, int ldb, int ldc, hipStream_t s) {
  const dim3 grid((M / 256) * (N / 256) * S), block(512);
  hipLaunchKernelGGL((gemm_bf16_nt_256_8ph<false, false, true, false, true>), grid, block, 0, s, A, B, Cp, bp, M, N,
                     K / S, lda, ldb, ldc, 0, ws);
  const size_t n4 = (size_t)M * N / 4;
  const int rblocks = (int)std::min<size_t>((n4 + 255) / 256, 8192);
  hipLaunchKernelGGL((splitk_reduce<RELU, BIAS>), dim3(rblocks), dim3(256), 0, s, ws, S, M, N, bp, Cp, ldc);
}

// the tile gemm_bf16_nt launches for this shape (pick_gemm_tile + the kernels' shape limits)
static int resolve_gemm_tile(int M, int N, int K, int cu_budget) {
  int t = pick_gemm_tile(M, N, cu_budget);
  if ((t == 9 || t == 10) && K < 128) t = 4;     // the 8-phase prologue stages two K-tiles
  if (t == 13 && K < 128) t = 5;
  if (t == 14 && K < 128) t = 4;
  if (t == 15 && K < 128) t = 5;
  if (t == 16 && K < 128) t = 1;
  if (M % kTileBM[t] || N % kTileBN[t]) t = 3;   // 64x64 always divides (checked by the caller)
  return t;
}

// fp8 fill rule, as the bf16 picker: 128x128 when it gives every CU of the budget a block (two
// for a lone kernel), else 64x64
static bool fp8_tile_128(int M, int N, int cu_budget) {
  const bool alone = cu_budget <= 0 || cu_budget >= kCus;
  const int need = alone ? 2 * kCus : cu_budget;
  return M % 128 == 0 && N % 128 == 0 && (M / 128) * (N / 128) >= need;
}

int gemm_workgroups(int M, int N, int K, int cu_budget, bool fp8, bool split_workspace) {
  if (M <= 0 || N <= 0 || K <= 0 || M % 64 || N % 64) throw std::runtime_error("gemm_workgroups: bad shape");
  if (fp8) return fp8_tile_128(M, N, cu_budget) ? (M / 128) * (N / 128) : (M / 64) * (N / 64);
  const int S = split_workspace ? pick_split_k(M, N, K, cu_budget) : 1;
  if (S > 1) return (M / 256) * (N / 256) * S;
  const int t = resolve_gemm_tile(M, N, K, cu_budget);
  return (M / kTileBM[t]) * (N / kTileBN[t]);
}

void gemm_bf16_nt(uintptr_t a, uintptr_t bt, uintptr_t c, uintptr_t bias, int M, int N, int K, int lda, int ldb,
                  int ldc, bool relu, uintptr_t stream, int cu_budget, uintptr_t workspace, size_t workspace_floats) {
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
  const int S = workspace ? pick_split_k(M, N, K, cu_budget) : 1;
  if (S > 1) {
    if (workspace_floats < (size_t)S * M * N) throw std::runtime_error("gemm: split-K workspace too small");
    check_align(reinterpret_cast<void*>(workspace), "workspace");
    auto ws = reinterpret_cast<float*>(workspace);
    if (relu && bp) launch_splitk<true, true>(A, B, Cp, bp, ws, S, M, N, K, lda, ldb, ldc, s);
    else if (relu) launch_splitk<true, false>(A, B, Cp, bp, ws, S, M, N, K, lda, ldb, ldc, s);
    else if (bp) launch_splitk<false, true>(A, B, Cp, bp, ws, S, M, N, K, lda, ldb, ldc, s);
    else launch_splitk<false, false>(A, B, Cp, bp, ws, S, M, N, K, lda, ldb, ldc, s);
    HIP_CHECK(hipGetLastError());
    return;
  }
  const int t = resolve_gemm_tile(M, N, K, cu_budget);
  switch (t) {
    case 1: launch_gemm<128, 128, 2, 2, 2, 2, 64, true>(A, B, Cp, bp, M, N, K, lda, ldb, ldc, relu, s); break;
    case 2: launch_gemm<64, 128, 2, 2, 2>(A, B, Cp, bp, M, N, K, lda, ldb, ldc, relu, s); break;
    case 4: launch_gemm<256, 256, 2, 4, 1, 2, 64, true>(A, B, Cp, bp, M, N, K, lda, ldb, ldc, relu, s); break;
    case 5: launch_gemm<256, 128, 4, 2, 1>(A, B, Cp, bp, M, N, K, lda, ldb, ldc, relu, s); break;
    case 6: launch_gemm<128, 128, 2, 2, 2>(A, B, Cp, bp, M, N, K, lda, ldb, ldc, relu, s); break;
    case 7: launch_gemm<64, 128, 2, 2, 2, 3>(A, B, Cp, bp, M, N, K, lda, ldb, ldc, relu, s); break;
    case 8: launch_gemm<256, 128, 4, 2, 1, 3>(A, B, Cp, bp, M, N, K, lda, ldb, ldc, relu, s); break;
    case 11: launch_gemm<128, 128, 2, 2, 1, 3, 64, true>(A, B, Cp, bp, M, N, K, lda, ldb, ldc, relu, s); break;
    case 12: launch_gemm<128, 128, 2, 2, 1, 4, 64, true>(A, B, Cp, bp, M, N, K, lda, ldb, ldc, relu, s); break;
    case 9:
    case 10: {
      const bool lone = g_lone_plain_order && (cu_budget <= 0 || cu_budget >= kCus);
      // policy 9 (A/B arm, round 6): a co-running pod's 8-phase GEMM with more 256 x 256 tiles than
      // its CU share runs as back-to-back launches of whole tile rows of at most `cu_budget` tiles
      // each, so it never holds more CUs than its share and the other pods' stream kernels keep
      // the rest of the chip (profiles/r06_gap/: GEMM time not hidden under the streams is the
      // largest term of the step)
      const bool co = cu_budget > 0 && cu_budget < kCus;
      if (t == 10 && co && g_gemm_policy == 9 && (M / 256) * (N / 256) > cu_budget) {
        const int rows = std::max(1, cu_budget / (N / 256)) * 256;
        const dim3 block(512);
        for (int m0 = 0; m0 < M; m0 += rows) {
          const int mm = std::min(rows, M - m0);
          const dim3 g((mm / 256) * (N / 256));
          launch_8ph<true>(A + (size_t)m0 * lda, B, Cp + (size_t)m0 * ldc, bp, mm, N, K, lda, ldb, ldc, relu, s, g,
                           block, false);
        }
        break;
      }
      const dim3 grid((M / 256) * (N / 256)), block(512);
      if (t == 10)
        launch_8ph<true>(A, B, Cp, bp, M, N, K, lda, ldb, ldc, relu, s, grid, block, lone);
      else
        launch_8ph<false>(A, B, Cp, bp, M, N, K, lda, ldb, ldc, relu, s, grid, block, lone);
      break;
    }
    case 13: {
      const dim3 grid((M / 256) * (N / 128)), block(512);
      const bool lone = g_lone_plain_order && (cu_budget <= 0 || cu_budget >= kCus);
      launch_8ph<true, 128>(A, B, Cp, bp, M, N, K, lda, ldb, ldc, relu, s, grid, block, lone);
      break;
    }
    case 14:
    case 15:
    case 16: {
      if (!wide_ok(Cp, ldc)) {
        if (g_gemm_tile == t) throw std::runtime_error("gemm tiles 14-16: C rows must be 16-byte aligned");
        if (t == 14)                                // a policy on an unaligned C: the 8-phase kernels
          launch_8ph<true>(A, B, Cp, bp, M, N, K, lda, ldb, ldc, relu, s, dim3((M / 256) * (N / 256)), dim3(512), false);
        else if (t == 15)
          launch_8ph<true, 128>(A, B, Cp, bp, M, N, K, lda, ldb, ldc, relu, s, dim3((M / 256) * (N / 128)), dim3(512), false);
        else
          launch_gemm<128, 128, 2, 2, 2, 2, 64, true>(A, B, Cp, bp, M, N, K, lda, ldb, ldc, relu, s);
        break;
      }
      if ((size_t)256 * std::max(lda, ldb) * 2 >= ((size_t)1 << 31))
        throw std::runtime_error("gemm tiles 14-16: a 256-row operand block must span < 2 GiB");
      const int bm = t == 16 ? 128 : 256, bn = t == 14 ? 256 : 128;
      const dim3 grid((M / bm) * (N / bn)), block(256);
      const bool lone = g_lone_plain_order && (cu_budget <= 0 || cu_budget >= kCus);
      const int xmap = lone ? 0 : pick_xcd_map(M / bm, N / bn);
      decltype(&gemm_bf16_nt_256_w4l<false, false>) k;
      if (t == 16)
        k = relu ? (bp ? gemm_bf16_nt_256_w4l<true, true, 0, false, 128, 128> : gemm_bf16_nt_256_w4l<true, false, 0, false, 128, 128>)
                 : (bp ? gemm_bf16_nt_256_w4l<false, true, 0, false, 128, 128> : gemm_bf16_nt_256_w4l<false, false, 0, false, 128, 128>);
      else if (t == 15)
        k = relu ? (bp ? gemm_bf16_nt_256_w4l<true, true, 0, false, 128> : gemm_bf16_nt_256_w4l<true, false, 0, false, 128>)
                 : (bp ? gemm_bf16_nt_256_w4l<false, true, 0, false, 128> : gemm_bf16_nt_256_w4l<false, false, 0, false, 128>);
      else if (g_w4_probe)   // timing probes: steady-loop LDS-DMA (1), reads (2) or both (3) dropped
        k = g_w4_probe == 1 ? gemm_bf16_nt_256_w4l<false, false, 1>
            : g_w4_probe == 2 ? gemm_bf16_nt_256_w4l<false, false, 2> : gemm_bf16_nt_256_w4l<false, false, 3>;
      else if (g_w4_prio)
        k = relu ? (bp ? gemm_bf16_nt_256_w4l<true, true, 0, true> : gemm_bf16_nt_256_w4l<true, false, 0, true>)
                 : (bp ? gemm_bf16_nt_256_w4l<false, true, 0, true> : gemm_bf16_nt_256_w4l<false, false, 0, true>);
      else
        k = relu ? (bp ? gemm_bf16_nt_256_w4l<true, true> : gemm_bf16_nt_256_w4l<true, false>)
                 : (bp ? gemm_bf16_nt_256_w4l<false, true> : gemm_bf16_nt_256_w4l<false, false>);
      hipLaunchKernelGGL(k, grid, block, 0, s, A, B, Cp, bp, M, N, K, lda, ldb, ldc, xmap);
      break;
    }
    default: launch_gemm<64, 64, 2, 2, 2, 2, 64, true>(A, B, Cp, bp, M, N, K, lda, ldb, ldc, relu, s); break;
  }
  HIP_CHECK(hipGetLastError());
}

template <int BM, int BN, int WGM, int WGN, int OCC>
static void launch_gemm_fp8(const uint8_t* A, const uint8_t* B, __bf16* Cp, const float* bp, int M, int N, int K,
                            int lda, int ldb, int ldc, bool relu, hipStream_t s) {
  const dim3 grid((M / BM) * (N / BN)), block(WGM * WGN * 64);
  if (relu && bp)
    hipLaunchKernelGGL((gemm_fp8_nt_kernel<BM, BN, WGM, WGN, OCC, true, true>), grid, block, 0, s, A, B, Cp, bp, M, N,
                       K, lda, ldb, ldc);
  else if (relu)
    hipLaunchKernelGGL((gemm_fp8_nt_kernel<BM, BN, WGM, WGN, OCC, true, false>), grid, block, 0, s, A, B, Cp, bp, M,
                       N, K, lda, ldb, ldc);
  else if (bp)
    hipLaunchKernelGGL((gemm_fp8_nt_kernel<BM, BN, WGM, WGN, OCC, false, true>), grid, block, 0, s, A, B, Cp, bp, M,
                       N, K, lda, ldb, ldc);
  else
    hipLaunchKernelGGL((gemm_fp8_nt_kernel<BM, BN, WGM, WGN, OCC, false, false>), grid, block, 0, s, A, B, Cp, bp, M,
                       N, K, lda, ldb, ldc);
}

void gemm_fp8_nt(uintptr_t a, uintptr_t bt, uintptr_t c, uintptr_t bias, int M, int N, int K, int lda, int ldb,
                 int ldc, bool relu, uintptr_t stream, int cu_budget) {
  if (M <= 0 || N <= 0 || K <= 0) throw std::runtime_error("gemm_fp8: empty shape");
  if (M % 64 || N % 64 || K % 128) throw std::runtime_error("gemm_fp8: M,N must be multiples of 64 and K of 128");
  if (lda < K || ldb < K || ldc < N || lda % 16 || ldb % 16) throw std::runtime_error("gemm_fp8: bad leading dims");
  check_align(reinterpret_cast<void*>(a), "A");
  check_align(reinterpret_cast<void*>(bt), "Bt");
  if (ldc % 4 || reinterpret_cast<uintptr_t>(c) % 8) throw std::runtime_error("gemm_fp8: C rows must be 8-byte aligned");
  if (bias) check_align(reinterpret_cast<void*>(bias), "bias");
  auto s = reinterpret_cast<hipStream_t>(stream);
  auto A = reinterpret_cast<const uint8_t*>(a);
  auto B = reinterpret_cast<const uint8_t*>(bt);
  auto Cp = reinterpret_cast<__bf16*>(c);
  auto bp = reinterpret_cast<const float*>(bias);
  if (fp8_tile_128(M, N, cu_budget))
    launch_gemm_fp8<128, 128, 2, 2, 2>(A, B, Cp, bp, M, N, K, lda, ldb, ldc, relu, s);
  else
    launch_gemm_fp8<64, 64, 2, 2, 2>(A, B, Cp, bp, M, N, K, lda, ldb, ldc, relu, s);
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
  // 9 / 10 (A/B arms): write-through stores only for the largest streams (arrays >= 256 / 128 MiB,
  // where a lone sc1 stream gains most), non-temporal below
  if (variant == 9 || variant == 10) variant = n_floats * 4 >= ((size_t)(variant == 9 ? 256 : 128) << 20) ? 8 : 3;
  switch (variant) {
    case 0: hipLaunchKernelGGL(stream_triad_kernel, dim3(blocks), dim3(256), 0, st, A, B, Cc, s, n4); break;
    case 1: hipLaunchKernelGGL((stream_triad_u<2, false>), dim3(blocks), dim3(256), 0, st, A, B, Cc, s, n4); break;
    case 2: hipLaunchKernelGGL((stream_triad_u<4, false>), dim3(blocks), dim3(256), 0, st, A, B, Cc, s, n4); break;
    case 3: hipLaunchKernelGGL((stream_triad_u<4, true>), dim3(blocks), dim3(256), 0, st, A, B, Cc, s, n4); break;
    case 4: hipLaunchKernelGGL((stream_triad_u<8, true>), dim3(blocks), dim3(256), 0, st, A, B, Cc, s, n4); break;
    case 7: hipLaunchKernelGGL((stream_triad_u<3, true>), dim3(blocks), dim3(256), 0, st, A, B, Cc, s, n4); break;
    case 8: hipLaunchKernelGGL((stream_triad_u<4, true, true>), dim3(blocks), dim3(256), 0, st, A, B, Cc, s, n4); break;
    default: hipLaunchKernelGGL((stream_triad_u<2, true>), dim3(blocks), dim3(256), 0, st, A, B, Cc, s, n4); break;
  }
  HIP_CHECK(hipGetLastError());
}

}  // namespace gs
