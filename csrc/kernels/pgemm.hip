// Prefill / encoder GEMM for gfx950:  Y[M, N] = X[M, K] . W[N, K]^T  (bf16 in, fp32 accumulate),
// with the elementwise op that follows each projection fused into the epilogue.
//
// Shapes: the decoder's prefill projections (M = prompt tokens of a batch, thousands to tens of
// thousands; N, K = 4096 .. 28672) and the sentence encoders' (M = tokens of an embedding batch,
// N, K = 384 .. 3072).  Compute bound: 256 x 256 output tile per workgroup, 128 FLOP per staged
// byte, so each CU must keep ~55 GB/s of X and W arriving through L2 while its MFMAs run.
//
//   * workgroup = 8 waves (2 along M x 4 along N), 512 threads, one workgroup per CU (launch
//     bound 1), each wave a 128 x 64 output block: 8 x 4 accumulator tiles of 16 x 16
//     (v_mfma_f32_16x16x32_bf16, 128 accumulator VGPRs);
//   * K in 64-deep tiles, both operands staged global -> LDS by LDS-DMA (`global_load_lds_dwordx4`,
//     written in asm: hipcc orders nothing behind it and never drains it before an ordinary load),
//     two LDS stages of 64 KB: the DMA of tile t+1 runs under the MFMAs of tile t, one barrier per
//     tile (its counted wait retires tile t's DMA and the previous tile's ds_reads together);
//   * each LDS image is 256 rows x 128 B, XOR-swizzled through the SOURCE address (chunk c of row r
//     at r * 128 + ((c ^ (r & 7)) << 4)), so the 16-row ds_read_b128 fragment reads are
//     bank-conflict free (guide rule 21 / T2) -- the same image as the decode GEMM's X stage;
//   * operands swapped in the MFMA (W fragment as A, X fragment as B) so each lane's accumulator
//     holds 4 CONSECUTIVE output columns of one row: the epilogue stores 8 bytes per lane straight
//     from registers, and SwiGLU's gate/up pairs are one lane swap (v_permlane32_swap) away;
//   * blockIdx -> tile: bijective XCD remap (guide T1), then groups of 8 M-tiles sweep the N-tiles,
//     so the ~32 workgroups resident on one XCD share X rows and W rows in that XCD's L2.
//
// Epilogues: bf16; + bias (encoder qkv); + bias -> GELU(erf) (encoder FFN up); SwiGLU over 8-row
// interleaved gate/up weights (decoder gate_up, reference.interleave_gate_up) -> [M, N/2].
//
// Bounds: K % 64 == 0, N % 64 == 0, ldo % 4 == 0; M and N need not be tile multiples (rows past
// the edge read the last valid row, their results are never stored).  X, W byte spans < 4 GiB
// (32-bit DMA offsets).
#include <atomic>
#include <type_traits>

#include "common.h"

namespace {

typedef __attribute__((address_space(3))) void pg_lds_t;

// PG_F32: the fp32 accumulators themselves (row stride ldo in floats): a tensor-parallel row-parallel
// projection's partial, all-reduced in fp32 and rounded to bf16 once, as TP = 1 rounds the full sum
enum { PG_BF16 = 0, PG_BIAS = 1, PG_BIAS_GELU = 2, PG_SWIGLU = 3, PG_F32 = 4 };

constexpr int PG_BM = 256, PG_BN = 256, PG_BK = 64;
constexpr int PG_STAGE = (PG_BM + PG_BN) * PG_BK * 2;   // 64 KB: A image then B image
constexpr int PG_GROUP_M = 8;

// One 1-KB LDS-DMA piece from sbase + voff (per lane): lane l's 16 bytes land at lds_addr + 16 l.
// SGPR base + 32-bit VGPR offset (one VGPR per piece instead of a 64-bit pointer).  M0 is saved and
// restored inside the statement (guide §5.7).
__device__ __forceinline__ void pg_glds16(uint32_t voff, const void* sbase, uint32_t lds_addr) {
  unsigned keep;
  asm volatile(
      "s_mov_b32 %0, m0\n\ts_mov_b32 m0, %3\n\ts_nop 0\n\tglobal_load_lds_dwordx4 %1, %2\n\ts_mov_b32 m0, %0"
      : "=&s"(keep)
      : "v"(voff), "s"(sbase), "s"(lds_addr)
      : "memory");
}

__device__ __forceinline__ float pg_gelu(float v) { return 0.5f * v * (1.f + erff(v * 0.70710678118654752f)); }

__device__ __forceinline__ float pg_bfr(float v) { return bf2f(f2bf(v)); }

// SwiGLU of one 4-value accumulator group (16-row n-tile = 8 gate rows then 8 up rows: lanes
// g = 0, 1 hold gate columns, lanes g = 2, 3 -- lane ^ 32 -- the matching up columns).  One VALU lane
// swap (v_permlane32_swap, common.h) of (v[0], v[2]) gives every lane a (gate, up) pair -- element 0
// in lanes g < 2, element 2 in lanes g >= 2 -- and one of (v[1], v[3]) elements 1 / 3, so every lane
// computes two outputs (no idle lane half, no LDS-crossbar shuffles) and returns them packed: output
// columns pg_swiglu_col(g) + {0, 1} of the n-tile's 8.  Same values and rounding as the unfused
// GEMM -> silu_mul path: bf16 of gate and up, silu(g) * u in fp32.
__device__ __forceinline__ uint32_t pg_swiglu2(const float (&v)[4]) {
  float g0 = v[0], u0 = v[2], g1 = v[1], u1 = v[3];
  swap32(g0, u0);
  swap32(g1, u1);
  auto f = [](float gate, float up) {
    const float gg = pg_bfr(gate);
    return gg * __builtin_amdgcn_rcpf(1.f + __expf(-gg)) * pg_bfr(up);
  };
  return pack2bf(f(g0, u0), f(g1, u1));
}

__device__ __forceinline__ int pg_swiglu_col(int g) { return 4 * (g & 1) + 2 * (g >> 1); }

// Epilogue of every kernel here: lane holds rows m = mw + 16 i + (lane & 15), columns
// n = nw + 16 j + 4 (lane >> 4) + 0..3 of the wave's 128 x 16 NJ block.
template <int EPI, int NJ>
__device__ __forceinline__ void pg_epilogue(const f32x4_t (&acc)[8][NJ], const uint16_t* __restrict__ bias,
                                            uint16_t* __restrict__ out, int M, int N, int ldo, int mw, int nw) {
  const int lane = threadIdx.x & 63;
  const int g = lane >> 4;
#pragma unroll
  for (int i = 0; i < 8; ++i) {
    const int m = mw + i * 16 + (lane & 15);
#pragma unroll
    for (int j = 0; j < NJ; ++j) {
      const int nb = nw + j * 16;   // n-tile base
      const int n = nb + 4 * g;
      float v[4] = {acc[i][j][0], acc[i][j][1], acc[i][j][2], acc[i][j][3]};
      if constexpr (EPI == PG_SWIGLU) {
        // bf16 rounding of g and u as the unfused GEMM -> silu_mul path
        const uint32_t y = pg_swiglu2(v);
        if (m < M && nb < N) *reinterpret_cast<uint32_t*>(out + (size_t)m * ldo + nb / 2 + pg_swiglu_col(g)) = y;
      } else if constexpr (EPI == PG_F32) {
        if (m < M && n < N)
          *reinterpret_cast<float4*>(reinterpret_cast<float*>(out) + (size_t)m * ldo + n) = make_float4(v[0], v[1], v[2], v[3]);
      } else {
        if (m < M && n < N) {
          if constexpr (EPI == PG_BIAS || EPI == PG_BIAS_GELU) {
            const uint2 bb = *reinterpret_cast<const uint2*>(bias + n);
            v[0] += __uint_as_float(bb.x << 16);
            v[1] += __uint_as_float(bb.x & 0xffff0000u);
            v[2] += __uint_as_float(bb.y << 16);
            v[3] += __uint_as_float(bb.y & 0xffff0000u);
          }
          if constexpr (EPI == PG_BIAS_GELU) {
#pragma unroll
            for (int e = 0; e < 4; ++e) v[e] = pg_gelu(v[e]);
          }
          *reinterpret_cast<uint2*>(out + (size_t)m * ldo + n) = make_uint2(pack2bf(v[0], v[1]), pack2bf(v[2], v[3]));
        }
      }
    }
  }
}

// LDS-staged epilogue of one wave's 128 x 64 accumulator tile (bf16 and SwiGLU outputs only): the
// values go to the wave's private 16-KB LDS region (8-byte writes, 16-byte units XOR-swizzled by the
// row), come back as 16-byte row pieces and leave as full 128-byte (bf16: 64 output columns) or
// 64-byte (SwiGLU: 32 output columns) row segments -- instead of 8-byte pieces with 32 / 16 bytes
// contiguous per row (and half the lanes idle for SwiGLU).  Same values, same rounding as
// pg_epilogue.  The caller guarantees no other wave reads or DMAs into that region any more.
template <int EPI>
__device__ __forceinline__ void pg_epilogue_staged(const f32x4_t (&acc)[8][4], uint16_t* __restrict__ out, int M,
                                                   int N, int ldo, int mw, int nw, char* region) {
  const int lane = threadIdx.x & 63;
  const int g = lane >> 4, rl = lane & 15;
  constexpr int OC = EPI == PG_SWIGLU ? 32 : 64;     // output columns of this wave
  constexpr int UPR = OC / 8;                         // 16-byte units per row
  constexpr int RB = OC * 2;                          // bytes per staged row
#pragma unroll
  for (int i = 0; i < 8; ++i) {
    const int r = 16 * i + rl;
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      float v[4] = {acc[i][j][0], acc[i][j][1], acc[i][j][2], acc[i][j][3]};
      if constexpr (EPI == PG_SWIGLU) {
        // output columns 8 j + pg_swiglu_col(g) .. +1: unit j
        const int unit = j ^ (r & (UPR - 1));
        *reinterpret_cast<uint32_t*>(region + r * RB + unit * 16 + 2 * pg_swiglu_col(g)) = pg_swiglu2(v);
      } else {
        // columns 16 j + 4 g .. +3: unit 2 j + (g >> 1), half g & 1
        const int unit = (2 * j + (g >> 1)) ^ (r & (UPR - 1));
        *reinterpret_cast<uint2*>(region + r * RB + unit * 16 + (g & 1) * 8) =
            make_uint2(pack2bf(v[0], v[1]), pack2bf(v[2], v[3]));
      }
    }
  }
  __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
  __builtin_amdgcn_wave_barrier();
  __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
  constexpr int RPI = 64 / UPR;                       // rows per store instruction
  const int ncol0 = EPI == PG_SWIGLU ? nw / 2 : nw;   // first output column of this wave
#pragma unroll
  for (int s = 0; s < 128 / RPI; ++s) {
    const int r = RPI * s + lane / UPR, unit = lane % UPR;
    const uint4 val = *reinterpret_cast<const uint4*>(region + r * RB + ((unit ^ (r & (UPR - 1))) * 16));
    const int m = mw + r, n = ncol0 + unit * 8;
    if (m < M && n < (EPI == PG_SWIGLU ? N / 2 : N))
      *reinterpret_cast<uint4*>(out + (size_t)m * ldo + n) = val;
  }
}

template <int EPI>
__global__ void __launch_bounds__(512, 1)
    pgemm_kernel(const uint16_t* __restrict__ X, const uint16_t* __restrict__ W, const uint16_t* __restrict__ bias,
                 uint16_t* __restrict__ out, int M, int N, int K, int ldo, int tiles_m, int tiles_n) {
  __shared__ __attribute__((aligned(16))) char smem[2 * PG_STAGE];
  const int lane = threadIdx.x & 63;
  const int w = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  const int wr = w >> 2, wc = w & 3;

  // ---- tile of this workgroup: XCD-local id, then GROUP_M-row groups sweeping the N tiles
  const int nwg = tiles_m * tiles_n;
  const int id = xcd_remap(blockIdx.x, nwg);
  const int per_group = PG_GROUP_M * tiles_n;
  const int first_m = (id / per_group) * PG_GROUP_M;
  const int gsz = min(tiles_m - first_m, PG_GROUP_M);
  const int in_group = id % per_group;
  const int m0 = (first_m + in_group % gsz) * PG_BM;
  const int n0 = (in_group / gsz) * PG_BN;

  // ---- DMA sources: piece p = 8 i + w (i = 0..3) covers image rows 8p .. 8p+7 of A and of B
  const int prow = lane >> 3, pch = (lane & 7) ^ prow;   // image row & 7 == prow for every piece
  uint32_t va[4], vb[4];
#pragma unroll
  for (int i = 0; i < 4; ++i) {
    const int r = 8 * (8 * i + w) + prow;
    va[i] = ((uint32_t)min(m0 + r, M - 1) * (uint32_t)K + 8u * pch) * 2u;
    vb[i] = ((uint32_t)min(n0 + r, N - 1) * (uint32_t)K + 8u * pch) * 2u;
  }
  const uint32_t lds0 = __builtin_amdgcn_readfirstlane((uint32_t)(uintptr_t)(pg_lds_t*)smem + w * 1024);
  auto issue = [&](int t, int s) {
    const uint16_t* xa = X + (size_t)t * PG_BK;
    const uint16_t* wb = W + (size_t)t * PG_BK;
    const uint32_t la = lds0 + s * PG_STAGE;
#pragma unroll
    for (int i = 0; i < 4; ++i) pg_glds16(va[i], xa, la + i * 8192);
#pragma unroll
    for (int i = 0; i < 4; ++i) pg_glds16(vb[i], wb, la + PG_BM * 128 + i * 8192);
  };

  f32x4_t acc[8][4];
#pragma unroll
  for (int i = 0; i < 8; ++i)
#pragma unroll
    for (int j = 0; j < 4; ++j) acc[i][j] = f32x4_t{0.f, 0.f, 0.f, 0.f};

  // fragment reads: row (lane & 15) of a 16-row tile, 16-byte chunk 4 kk + (lane >> 4) of the
  // 32-deep half kk, through the image swizzle (row & 7 == lane & 7)
  const int frow = (lane & 15) * 128;
  const int nk = K / PG_BK;
  issue(0, 0);
  for (int t = 0; t < nk; ++t) {
    // tile t's DMA (the only one in flight) retired and the previous tile's ds_reads done, in
    // every wave: after this barrier stage t & 1 is readable and stage (t + 1) & 1 writable
    asm volatile("s_waitcnt vmcnt(0) lgkmcnt(0)\n\ts_barrier" ::: "memory");
    if (t + 1 < nk) issue(t + 1, (t + 1) & 1);
    const char* sa = smem + (t & 1) * PG_STAGE + wr * 128 * 128 + frow;
    const char* sb = smem + (t & 1) * PG_STAGE + PG_BM * 128 + wc * 64 * 128 + frow;
#pragma unroll
    for (int kk = 0; kk < 2; ++kk) {
      const int ch = ((4 * kk + (lane >> 4)) ^ (lane & 7)) << 4;
      bf16x8_t af[8], bw[4];
#pragma unroll
      for (int i = 0; i < 8; ++i) af[i] = *reinterpret_cast<const bf16x8_t*>(sa + i * 16 * 128 + ch);
#pragma unroll
      for (int j = 0; j < 4; ++j) bw[j] = *reinterpret_cast<const bf16x8_t*>(sb + j * 16 * 128 + ch);
#pragma unroll
      for (int i = 0; i < 8; ++i)
#pragma unroll
        for (int j = 0; j < 4; ++j) acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(bw[j], af[i], acc[i][j], 0, 0, 0);
    }
  }

  pg_epilogue<EPI>(acc, bias, out, M, N, ldo, m0 + wr * 128, n0 + wc * 64);
}


// ---- v2: BK = 32 ring of R LDS slots ------------------------------------------------------------
// Same tile, waves and epilogue as pgemm_kernel; the K loop is a ring instead of a 2-stage double
// buffer.  A slot is one 32-deep K step of both operands: A image then B image, 256 rows x 64 B
// each (32 KB).  Step t's MFMAs run on fragments read from LDS during step t - 1, so the LDS reads
// of step t + 1 overlap them.  At the top of step t each wave waits (counted vmcnt) for ITS DMA of
// step t + 1 with the later steps left in flight and retires its ds_reads of step t (lgkmcnt(0));
// then one raw barrier: step t + 1 is readable everywhere and step t's slot (in registers in every
// wave) is free, so the DMA of step t + R goes into it right away.  A slot's DMA thus has R - 1
// steps of MFMA work (~1k cycles per step per SIMD pair) to land, against one 64-deep tile in the
// 2-stage kernel: what that kernel waits for at its vmcnt(0) (guide "Pipelining across barriers").
//
// 64-B image rows: 4 rows share a 256-B bank row, so the 16-row fragment read (lane: row
// lane & 15, chunk lane >> 4) is swizzled as chunk' = chunk ^ f((row >> 2) & 3), f = 0,3,2,1: every
// ds_read_b128 lane group then covers the 16 bank slots of one bank row exactly once.  The DMA
// writes lane-linear (16-row x 64-B piece per wave instruction), so the swizzle goes on its source
// chunk (guide rule 21).
constexpr int PR_BK = 32;
constexpr int PR_SLOT = (PG_BM + PG_BN) * PR_BK * 2;   // 32 KB

__device__ __forceinline__ int pr_f(int x) { return (4 - x) & 3; }

template <int EPI, int R>
__global__ void __launch_bounds__(512, 1)
    pgemm_ring_kernel(const uint16_t* __restrict__ X, const uint16_t* __restrict__ W,
                      const uint16_t* __restrict__ bias, uint16_t* __restrict__ out, int M, int N, int K, int ldo,
                      int tiles_m, int tiles_n) {
  __shared__ __attribute__((aligned(16))) char smem[R * PR_SLOT];
  const int lane = threadIdx.x & 63;
  const int w = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  const int wr = w >> 2, wc = w & 3;

  const int nwg = tiles_m * tiles_n;
  const int id = xcd_remap(blockIdx.x, nwg);
  const int per_group = PG_GROUP_M * tiles_n;
  const int first_m = (id / per_group) * PG_GROUP_M;
  const int gsz = min(tiles_m - first_m, PG_GROUP_M);
  const int in_group = id % per_group;
  const int m0 = (first_m + in_group % gsz) * PG_BM;
  const int n0 = (in_group / gsz) * PG_BN;

  // ---- DMA: wave w moves pieces w and w + 8 of A (image rows 16 p .. 16 p + 15) and of B;
  // lane l lands at row l >> 2, slot chunk l & 3 of its piece
  const int prow = lane >> 2, pch = (lane & 3) ^ pr_f((prow >> 2) & 3);
  uint32_t va[2], vb[2];
#pragma unroll
  for (int i = 0; i < 2; ++i) {
    const int r = 16 * (w + 8 * i) + prow;
    va[i] = ((uint32_t)min(m0 + r, M - 1) * (uint32_t)K + 8u * pch) * 2u;
    vb[i] = ((uint32_t)min(n0 + r, N - 1) * (uint32_t)K + 8u * pch) * 2u;
  }
  const uint32_t lds0 = __builtin_amdgcn_readfirstlane((uint32_t)(uintptr_t)(pg_lds_t*)smem + w * 1024);
  auto issue = [&](int t, int s) {
    const uint16_t* xa = X + (size_t)t * PR_BK;
    const uint16_t* wb = W + (size_t)t * PR_BK;
    const uint32_t la = lds0 + s * PR_SLOT;
    pg_glds16(va[0], xa, la);
    pg_glds16(va[1], xa, la + 8192);
    pg_glds16(vb[0], wb, la + PG_BM * 64);
    pg_glds16(vb[1], wb, la + PG_BM * 64 + 8192);
  };

  f32x4_t acc[8][4];
#pragma unroll
  for (int i = 0; i < 8; ++i)
#pragma unroll
    for (int j = 0; j < 4; ++j) acc[i][j] = f32x4_t{0.f, 0.f, 0.f, 0.f};

  const int frow = (lane & 15) * 64;
  const int ch = ((lane >> 4) ^ pr_f(((lane & 15) >> 2) & 3)) << 4;
  const char* ra = smem + wr * 128 * 64 + frow + ch;
  const char* rb = smem + PG_BM * 64 + wc * 64 * 64 + frow + ch;
  const int nk = K / PR_BK;
  // Fragments of step t are read from LDS during step t - 1's MFMAs.  B (4 fragments) is
  // double-buffered and read first; A fragment i is re-read in place right after its last MFMA of
  // the step (sched_barrier pins each read there: hoisted, the reads would double the live
  // fragments and spill).  The reads of the last step's "next" fragments touch a slot nobody
  // writes any more and are never used (branch-free MFMA stream).
  bf16x8_t af[8], bq[2][4];
  auto rd_a = [&](int s, int i) { return *reinterpret_cast<const bf16x8_t*>(ra + s * PR_SLOT + i * 16 * 64); };
  auto rd_b = [&](int s, int j) { return *reinterpret_cast<const bf16x8_t*>(rb + s * PR_SLOT + j * 16 * 64); };
  // Wait (own DMAs) for step t + 1 with the steps after it left in flight, retire this wave's
  // ds_reads, then the barrier: step t + 1 readable everywhere, slot of step t free.
  auto sync_next = [&](int t) {
    const int ahead = min(nk - 2 - t, R - 2);
    if (ahead >= 3)
      asm volatile("s_waitcnt vmcnt(12) lgkmcnt(0)\n\ts_barrier" ::: "memory");
    else if (ahead == 2)
      asm volatile("s_waitcnt vmcnt(8) lgkmcnt(0)\n\ts_barrier" ::: "memory");
    else if (ahead == 1)
      asm volatile("s_waitcnt vmcnt(4) lgkmcnt(0)\n\ts_barrier" ::: "memory");
    else
      asm volatile("s_waitcnt vmcnt(0) lgkmcnt(0)\n\ts_barrier" ::: "memory");
  };
#define PR_STEP(T, S, S1, BC, BN)                                                                         \
  do {                                                                                                   \
    if ((T) + 1 < nk) {                                                                                  \
      sync_next(T);                                                                                      \
      if ((T) + R < nk) issue((T) + R, S);                                                               \
    }                                                                                                    \
    _Pragma("unroll") for (int j = 0; j < 4; ++j) BN[j] = rd_b(S1, j);                                  \
    __builtin_amdgcn_sched_barrier(0);                                                                   \
    __builtin_amdgcn_s_setprio(1);                                                                       \
    _Pragma("unroll") for (int i = 0; i < 8; ++i) {                                                      \
      _Pragma("unroll") for (int j = 0; j < 4; ++j) acc[i][j] =                                          \
          __builtin_amdgcn_mfma_f32_16x16x32_bf16(BC[j], af[i], acc[i][j], 0, 0, 0);                     \
      af[i] = rd_a(S1, i);                                                                               \
      __builtin_amdgcn_sched_barrier(0);                                                                 \
    }                                                                                                    \
    __builtin_amdgcn_s_setprio(0);                                                                       \
  } while (0)
  for (int t = 0; t < R && t < nk; ++t) issue(t, t);
  {
    const int ahead = min(nk - 1, R - 1);   // step 0 landed, steps 1 .. ahead in flight
    if (ahead >= 4)
      asm volatile("s_waitcnt vmcnt(16)\n\ts_barrier" ::: "memory");
    else if (ahead == 3)
      asm volatile("s_waitcnt vmcnt(12)\n\ts_barrier" ::: "memory");
    else if (ahead == 2)
      asm volatile("s_waitcnt vmcnt(8)\n\ts_barrier" ::: "memory");
    else if (ahead == 1)
      asm volatile("s_waitcnt vmcnt(4)\n\ts_barrier" ::: "memory");
    else
      asm volatile("s_waitcnt vmcnt(0)\n\ts_barrier" ::: "memory");
  }
#pragma unroll
  for (int j = 0; j < 4; ++j) bq[0][j] = rd_b(0, j);
#pragma unroll
  for (int i = 0; i < 8; ++i) af[i] = rd_a(0, i);
  int s = 0;   // ring slot of step t
  for (int t = 0; t < nk; t += 2) {
    const int s1 = (s == R - 1) ? 0 : s + 1;
    const int s2 = (s1 == R - 1) ? 0 : s1 + 1;
    PR_STEP(t, s, s1, bq[0], bq[1]);
    PR_STEP(t + 1, s1, s2, bq[1], bq[0]);   // nk is even (K % 64 == 0)
    s = s2;
  }
#undef PR_STEP
  pg_epilogue<EPI>(acc, bias, out, M, N, ldo, m0 + wr * 128, n0 + wc * 64);
}


// ---- v3: ping-pong of two wave groups over half-tile LDS-DMA stages ------------------------------
// The 2-stage kernel above waits 30-35 % of its cycles (profiles/r03s2_pmc_pgemm_vs_hipblaslt.txt):
// every wave reaches the tile's vmcnt(0) + barrier at once, then all read LDS at once, and nothing
// covers either.  Here the 8 waves are two groups of 4 (waves 0-3, 4-7: one of each on every SIMD),
// run one barrier apart, so on each SIMD one wave's MFMA segment covers its partner's load segment
// (LDS-DMA issue, fragment ds_reads, counted vmcnt) and the matrix pipe never waits for either
// (guide §5 "The 256² 8-phase template", MI355X_MICROARCH "Two waves per SIMD").
//
//   * tile 256 x 256, BK = 64; wave (grp, wc) owns output rows 128 grp .. +128, cols 64 wc .. +64;
//   * a K-tile is 4 half-tiles of 16 KB: X0 = X tile rows {0-63, 128-191}, X1 = {64-127, 192-255},
//     W0 = W rows 0-127, W1 = W rows 128-255; two K-tile buffers = 128 KB of LDS;
//   * K-tile kt runs in two segments of 32 MFMAs per wave: A (X0 and both W halves: the wave's first
//     64 rows) and B (X1: its last 64 rows, W fragments kept in registers);
//   * stream of half-tiles: segment A of tile kt issues tile kt+1's {W1, X1}, segment B issues tile
//     kt+2's {X0, W0} -- each into a half whose last reader (either group) retired its ds_reads
//     (lgkmcnt(0)) before the barrier that precedes the issue; counted vmcnt(8) / vmcnt(6) leave
//     2-3 half-tiles of DMA in flight per wave (48-64 KB per CU) and retire exactly what the next
//     segment reads, one barrier (two for the lagging group) ahead of the read;
//   * X image: 128 rows x 128 B per half, chunk c of image row r at r*128 + ((c ^ (r & 7)) << 4)
//     (swizzled through the DMA SOURCE address, guide rule 21), 8-row x 128-B pieces;
//   * W: row-major as X, or fragment-packed (the decode GEMM's cfc_dgemm_pack layout, wnw = its
//     bn / 16): every 16-row x 32-k MFMA fragment is 1 KB contiguous in lane order, so each DMA piece
//     is one whole fragment and its ds_read_b128 at lane * 16 is conflict free -- one weight copy
//     serves prefill and decode.
constexpr int PP_HALF = 128 * 128;        // bytes of one half-tile (128 rows x 64 k bf16)
constexpr int PP_BUF = 4 * PP_HALF;       // X0 X1 W0 W1

__device__ __forceinline__ void pp_barrier() { asm volatile("s_barrier" ::: "memory"); }

template <int N>
__device__ __forceinline__ void pp_wait_barrier() {
  asm volatile("s_waitcnt vmcnt(%0) lgkmcnt(0)\n\ts_barrier" ::"i"(N) : "memory");
}

// PF: probe flags (scripts/bench_pgemm.py --probe; 0 in production): 1 = no s_setprio, 2 = static
// priority 1 for group 1 instead of per-segment flips.  gm = M-tiles per N sweep of the tile order.
template <int EPI, bool PACKED, int PF = 0>
__global__ void __launch_bounds__(512, 1)
    pgemm_pp_kernel(const uint16_t* __restrict__ X, const uint16_t* __restrict__ W, const uint16_t* __restrict__ bias,
                    uint16_t* __restrict__ out, int M, int N, int K, int ldo, int tiles_m, int tiles_n, int wnw,
                    int gm = PG_GROUP_M) {
  __shared__ __attribute__((aligned(16))) char smem[2 * PP_BUF];
  const int lane = threadIdx.x & 63;
  const int w = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  const int grp = w >> 2, wc = w & 3;

  const int nwg = tiles_m * tiles_n;
  const int id = xcd_remap(blockIdx.x, nwg);
  const int per_group = gm * tiles_n;
  const int first_m = (id / per_group) * gm;
  const int gsz = min(tiles_m - first_m, gm);
  const int in_group = id % per_group;
  const int m0 = (first_m + in_group % gsz) * PG_BM;
  const int n0 = (in_group / gsz) * PG_BN;
  const int nk = K / PG_BK;

  // ---- DMA sources.  X: pieces w and w + 8 of half h = image rows 8 p .. 8 p + 7 (lane: row
  // lane >> 3, chunk lane & 7 through the swizzle; image row r is tile row (r >> 6) * 128 + 64 h + (r & 63))
  uint32_t vx[2][2], vw[2][2];
#pragma unroll
  for (int h = 0; h < 2; ++h)
#pragma unroll
    for (int i = 0; i < 2; ++i) {
      const int r = 8 * (w + 8 * i) + (lane >> 3);
      const int trow = (r >> 6) * 128 + 64 * h + (r & 63);
      const int c = (lane & 7) ^ (r & 7);
      vx[h][i] = ((uint32_t)min(m0 + trow, M - 1) * (uint32_t)K + 8u * c) * 2u;
    }
  // W half h, pieces w and w + 8.  Packed: piece f = fragment (n-tile f >> 1 of the half, k group
  // f & 1 of the K-tile); its 1 KB sits at ((g / wnw) * K/32 + kg) * wnw + g % wnw fragments
  // (cfc_dgemm_pack).  Row-major: as X, image row r = W tile row 128 h + r.
  const int kg_all = K / 32;
#pragma unroll
  for (int h = 0; h < 2; ++h)
#pragma unroll
    for (int i = 0; i < 2; ++i) {
      if constexpr (PACKED) {
        const int f = w + 8 * i;
        const int g = min(n0 / 16 + 8 * h + (f >> 1), N / 16 - 1);
        vw[h][i] = (uint32_t)(((g / wnw) * kg_all + (f & 1)) * wnw + g % wnw) * 1024u + 16u * lane;
      } else {
        const int r = 8 * (w + 8 * i) + (lane >> 3);
        const int c = (lane & 7) ^ (r & 7);
        vw[h][i] = ((uint32_t)min(n0 + 128 * h + r, N - 1) * (uint32_t)K + 8u * c) * 2u;
      }
    }
  const uint32_t lds0 = __builtin_amdgcn_readfirstlane((uint32_t)(uintptr_t)(pg_lds_t*)smem + w * 1024);
  // per K-tile advance of the W source: 2 fragments of every 16-row group (packed) or 64 columns
  const size_t wstep = PACKED ? (size_t)2 * wnw * 512 : (size_t)PG_BK;
  auto issue_x = [&](int kt, int h) {
    const uint16_t* src = X + (size_t)kt * PG_BK;
    const uint32_t la = lds0 + (kt & 1) * PP_BUF + h * PP_HALF;
    pg_glds16(vx[h][0], src, la);
    pg_glds16(vx[h][1], src, la + 8192);
  };
  auto issue_w = [&](int kt, int h) {
    const uint16_t* src = W + (size_t)kt * wstep;
    const uint32_t la = lds0 + (kt & 1) * PP_BUF + (2 + h) * PP_HALF;
    pg_glds16(vw[h][0], src, la);
    pg_glds16(vw[h][1], src, la + 8192);
  };

  f32x4_t acc[8][4];
#pragma unroll
  for (int i = 0; i < 8; ++i)
#pragma unroll
    for (int j = 0; j < 4; ++j) acc[i][j] = f32x4_t{0.f, 0.f, 0.f, 0.f};

  // fragment reads.  X: image row 64 grp + 16 i + (lane & 15) of the half, chunk 4 kk + (lane >> 4)
  // through the swizzle (row & 7 == lane & 7).  W n-tile T = 4 wc + j lies in half T >> 3.
  const int xrd = (64 * grp + (lane & 15)) * 128;
  const int sw = lane & 7;
  auto rd_x = [&](int buf, int h, int i, int kk) {
    return *reinterpret_cast<const bf16x8_t*>(smem + buf + h * PP_HALF + xrd + i * 16 * 128 +
                                              (((4 * kk + (lane >> 4)) ^ sw) << 4));
  };
  auto rd_w = [&](int buf, int j, int kk) {
    const int T = 4 * wc + j;
    const char* half = smem + buf + (2 + (T >> 3)) * PP_HALF;
    if constexpr (PACKED) {
      return *reinterpret_cast<const bf16x8_t*>(half + (2 * (T & 7) + kk) * 1024 + 16 * lane);
    } else {
      return *reinterpret_cast<const bf16x8_t*>(half + (16 * (T & 7) + (lane & 15)) * 128 +
                                                (((4 * kk + (lane >> 4)) ^ sw) << 4));
    }
  };

  // W1E (PF & 32): tile kt+2's W1 half is issued with its X0 / W0 in segment B of tile kt (its slot is
  // free once both groups' segment-A reads of tile kt retired) instead of in segment A of tile kt+1,
  // so every half has ~2 segments between its issue and the wait that retires it (was 1 for W1).
  constexpr bool W1E = (PF & 32) != 0;
  // ---- prologue: tile 0 whole, tile 1's {X0, W0} (+ W1); tile 0's X0 / W0 / W1 landed in every wave
  issue_x(0, 0);
  issue_w(0, 0);
  issue_w(0, 1);
  issue_x(0, 1);
  if (nk > 1) {
    issue_x(1, 0);
    issue_w(1, 0);
    if constexpr (W1E) {
      issue_w(1, 1);
      pp_wait_barrier<8>();
    } else {
      pp_wait_barrier<6>();
    }
  } else {
    pp_wait_barrier<2>();
  }
  if (grp == 1) pp_barrier();   // the stagger: group 1 runs one barrier behind group 0
  if constexpr ((PF & 2) != 0) {
    if (grp == 1) __builtin_amdgcn_s_setprio(1);
  }
  constexpr bool FLIP = (PF & 3) == 0;

  // ablation probes (never in production): 4 = no LDS-DMA in the loop, 8 = no fragment ds_reads
  // (fragments of tile 0 reused, kept live), 16 = no MFMA (fragments kept live)
  constexpr bool DMA = (PF & 4) == 0, RD = (PF & 8) == 0, MM = (PF & 16) == 0;
  bf16x8_t wf[4][2], xf[4][2];
  if constexpr (!RD) {
#pragma unroll
    for (int j = 0; j < 4; ++j)
#pragma unroll
      for (int kk = 0; kk < 2; ++kk) wf[j][kk] = rd_w(0, j, kk);
#pragma unroll
    for (int i = 0; i < 4; ++i)
#pragma unroll
      for (int kk = 0; kk < 2; ++kk) xf[i][kk] = rd_x(0, 0, i, kk);
  }
  auto keep = [&]() {
#pragma unroll
    for (int j = 0; j < 4; ++j)
#pragma unroll
      for (int kk = 0; kk < 2; ++kk) asm volatile("" : "+v"(wf[j][kk]), "+v"(xf[j][kk]));
  };
  for (int kt = 0; kt < nk; ++kt) {
    const int buf = (kt & 1) * PP_BUF;
    // ======== segment A: load part (tile kt+1's W1 / X1 into the other buffer; fragments)
    if (DMA && kt + 1 < nk) {
      if constexpr (!W1E) issue_w(kt + 1, 1);
      issue_x(kt + 1, 1);
    }
    if constexpr (RD) {
#pragma unroll
      for (int j = 0; j < 4; ++j)
#pragma unroll
        for (int kk = 0; kk < 2; ++kk) wf[j][kk] = rd_w(buf, j, kk);
#pragma unroll
      for (int i = 0; i < 4; ++i)
#pragma unroll
        for (int kk = 0; kk < 2; ++kk) xf[i][kk] = rd_x(buf, 0, i, kk);
    } else {
      keep();
    }
    // retire tile kt's X1 (segment B reads it) and this wave's ds_reads
    if (DMA && kt + 1 < nk) pp_wait_barrier<8>();
    else pp_wait_barrier<0>();
    __builtin_amdgcn_sched_barrier(0);
    if constexpr (FLIP) __builtin_amdgcn_s_setprio(1);
    if constexpr (MM) {
#pragma unroll
      for (int kk = 0; kk < 2; ++kk)
#pragma unroll
        for (int i = 0; i < 4; ++i)
#pragma unroll
          for (int j = 0; j < 4; ++j)
            acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(wf[j][kk], xf[i][kk], acc[i][j], 0, 0, 0);
    } else {
      keep();
    }
    if constexpr (FLIP) __builtin_amdgcn_s_setprio(0);
    __builtin_amdgcn_sched_barrier(0);
    pp_barrier();
    // ======== segment B: load part (tile kt+2's X0 / W0 into this buffer's free halves)
    if (DMA && kt + 2 < nk) {
      issue_x(kt + 2, 0);
      issue_w(kt + 2, 0);
      if constexpr (W1E) issue_w(kt + 2, 1);
    }
    if constexpr (RD) {
#pragma unroll
      for (int i = 0; i < 4; ++i)
#pragma unroll
        for (int kk = 0; kk < 2; ++kk) xf[i][kk] = rd_x(buf, 1, i, kk);
    } else {
      keep();
    }
    // retire tile kt+1's X0 / W0 / W1 (next segment A reads them)
    if (DMA && kt + 2 < nk) pp_wait_barrier<W1E ? 8 : 6>();
    else if (DMA && kt + 1 < nk) pp_wait_barrier<2>();
    else pp_wait_barrier<0>();
    __builtin_amdgcn_sched_barrier(0);
    if constexpr (FLIP) __builtin_amdgcn_s_setprio(1);
    if constexpr (MM) {
#pragma unroll
      for (int kk = 0; kk < 2; ++kk)
#pragma unroll
        for (int i = 0; i < 4; ++i)
#pragma unroll
          for (int j = 0; j < 4; ++j)
            acc[4 + i][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(wf[j][kk], xf[i][kk], acc[4 + i][j], 0, 0, 0);
    } else {
      keep();
    }
    if constexpr (FLIP) __builtin_amdgcn_s_setprio(0);
    __builtin_amdgcn_sched_barrier(0);
    pp_barrier();
  }
  if constexpr (!MM) {      // the ablation's outputs depend on its fragments (nothing is dead code)
#pragma unroll
    for (int j = 0; j < 4; ++j) acc[0][j] += __builtin_bit_cast(f32x4_t, wf[j][0]) + __builtin_bit_cast(f32x4_t, xf[j][1]);
  }

  // wave rows: segment A's m-tiles i = tile rows 128 grp + 16 i, segment B's = 128 grp + 64 + 16 i.
  // STG (PF & 64): the bf16 / SwiGLU outputs leave through LDS as whole row segments.  After this
  // wave's last barrier of the loop no wave reads LDS any more (the lagging group's last reads were
  // retired before it) and every DMA landed, so each wave may use its own 16-KB slice.
  // staged stores for the bf16 epilogue; SwiGLU (half the columns, 8-byte pieces) measured 0.7 %
  // faster with the direct stores once its math was spread over both lane halves
  constexpr bool STG = (PF & 64) != 0 && EPI == PG_BF16;
  if constexpr (STG)
    pg_epilogue_staged<EPI>(acc, out, M, N, ldo, m0 + grp * 128, n0 + wc * 64, smem + w * 16384);
  else
    pg_epilogue<EPI>(acc, bias, out, M, N, ldo, m0 + grp * 128, n0 + wc * 64);
  if (grp == 0) pp_barrier();   // matches group 1's stagger barrier
}

// ---- v4: the ping-pong kernel made persistent (packed W; bf16 and SwiGLU epilogues) ----------------
// Fitting t = a + b K over K = 1k..8k at M = 16384 (scripts/probe_pgemm_k.py, profiles/
// r06_pgemm_k.jsonl) puts a fixed ~7 us (qkv) to ~16-20 us (gate_up) on every wave of 256 tiles:
// each new workgroup starts with an idle prologue (its first two K-tiles' DMA round trip, every CU
// at once) and ends with a store tail nothing covers.  Here one workgroup per CU walks the tiles
// vb = blockIdx.x, + gridDim.x, ... (the same XCD-remapped order, so the same XCD sees the same
// tiles), and the half-tile stream simply runs on across the tile boundary: the last two K-tiles of
// a tile issue the next tile's first ones with its DMA offsets (the slot-free analysis of the stream
// is per position, so it holds unchanged), and the epilogue stores of tile t are issued without a
// drain while tile t+1's first DMA is in flight.
//   * interior wave blocks store with exactly S unconditional stores (16 x 16 B staged bf16, 8 x 16 B
//     staged SwiGLU, 32 without staging; the counts are pinned by tests/test_ppp_isa.py), and the
//     waits of the next tile's K-tile 0 keep those S stores outstanding (vmcnt(8 + S), or 2 + S in
//     segment B of a two-K-tile last tile); the next waits see them older than the DMA they retire,
//     so the stores have one MFMA segment to drain;
//   * an edge block (rows past M / columns past N) stores through pg_epilogue and drains (vmcnt(0));
//   * the steady K-tiles (kt + 2 < nk) run a branch-free copy of the K step; only the last two run
//     the copy whose DMA continues into the next tile (its offsets computed there), so the loop
//     the MFMAs wait on carries no tile-boundary logic (71 scalar instructions per K-tile, "pp" 102);
//   * STG: the interior block leaves as whole row segments (bf16 128 B, SwiGLU 64 B) through a
//     private 4-KB LDS region per wave (the 32 KB the stream's two 64-KB buffers leave free), 32 /
//     64 rows at a time -- what "pps" does with the stream's own buffers, which stay busy here.
constexpr int PPP_REGION = 4096;   // bytes of one wave's staging region (STG)

// The epilogue stores are compiler-issued (full exec, unconditional: exactly one global_store_dwordx2
// / _dwordx4 each, checked in the ISA): a store of more than 8 bytes needs wait states before its
// registers are rewritten, which the compiler inserts only for instructions it can see.
__device__ __forceinline__ void ppp_st4(void* p, uint32_t v) { *reinterpret_cast<uint32_t*>(p) = v; }

__device__ __forceinline__ void ppp_st8(void* p, uint2 v) { *reinterpret_cast<uint2*>(p) = v; }

__device__ __forceinline__ void ppp_st16(void* p, uint4 v) { *reinterpret_cast<uint4*>(p) = v; }

template <int EPI, bool STG = false>
__global__ void __launch_bounds__(512, 1)
    pgemm_ppp_kernel(const uint16_t* __restrict__ X, const uint16_t* __restrict__ W, uint16_t* __restrict__ out,
                     int M, int N, int K, int ldo, int tiles_m, int tiles_n, int wnw, int gm) {
  static_assert(EPI == PG_BF16 || EPI == PG_SWIGLU, "bf16 / SwiGLU epilogues");
  // epilogue store instructions per wave in the interior (counted in the next tile's first waits):
  // staged bf16 16 x 16 B (128 rows x 128 B), staged SwiGLU 8 x 16 B (128 rows x 64 B), else 32
  constexpr int PPP_S = STG ? (EPI == PG_SWIGLU ? 8 : 16) : 32;
  __shared__ __attribute__((aligned(16))) char smem[2 * PP_BUF + (STG ? 8 * PPP_REGION : 0)];
  const int lane = threadIdx.x & 63;
  const int w = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  const int grp = w >> 2, wc = w & 3;
  const int nwg = tiles_m * tiles_n, G = gridDim.x;
  const int per_group = gm * tiles_n;
  const int nk = K / PG_BK, kg_all = K / 32;

  auto coords = [&](int vb, int& m0, int& n0) {
    const int id = xcd_remap(vb, nwg);
    const int first_m = (id / per_group) * gm;
    const int gsz = min(tiles_m - first_m, gm);
    const int in_group = id % per_group;
    m0 = (first_m + in_group % gsz) * PG_BM;
    n0 = (in_group / gsz) * PG_BN;
  };
  // DMA source offsets of one tile (as pgemm_pp_kernel, packed W)
  auto offsets = [&](int m0, int n0, uint32_t (&vx)[2][2], uint32_t (&vw)[2][2]) {
#pragma unroll
    for (int h = 0; h < 2; ++h)
#pragma unroll
      for (int i = 0; i < 2; ++i) {
        const int r = 8 * (w + 8 * i) + (lane >> 3);
        const int trow = (r >> 6) * 128 + 64 * h + (r & 63);
        const int c = (lane & 7) ^ (r & 7);
        vx[h][i] = ((uint32_t)min(m0 + trow, M - 1) * (uint32_t)K + 8u * c) * 2u;
        const int f = w + 8 * i;
        const int g = min(n0 / 16 + 8 * h + (f >> 1), N / 16 - 1);
        vw[h][i] = (uint32_t)(((g / wnw) * kg_all + (f & 1)) * wnw + g % wnw) * 1024u + 16u * lane;
      }
  };
  int vb = blockIdx.x, m0, n0, m0n = 0, n0n = 0;
  uint32_t vx[2][2], vw[2][2], nx[2][2], nwv[2][2];
  coords(vb, m0, n0);
  offsets(m0, n0, vx, vw);
  bool has_next = vb + G < nwg;
  if (has_next) coords(vb + G, m0n, n0n);   // its DMA offsets: computed where first needed (MODE 1)
  const uint32_t lds0 = __builtin_amdgcn_readfirstlane((uint32_t)(uintptr_t)(pg_lds_t*)smem + w * 1024);
  const size_t wstep = (size_t)2 * wnw * 512;
  auto issue_x = [&](int kt, int slot, const uint32_t (&o)[2][2], int h) {
    const uint16_t* src = X + (size_t)kt * PG_BK;
    const uint32_t la = lds0 + slot * PP_BUF + h * PP_HALF;
    pg_glds16(o[h][0], src, la);
    pg_glds16(o[h][1], src, la + 8192);
  };
  auto issue_w = [&](int kt, int slot, const uint32_t (&o)[2][2], int h) {
    const uint16_t* src = W + (size_t)kt * wstep;
    const uint32_t la = lds0 + slot * PP_BUF + (2 + h) * PP_HALF;
    pg_glds16(o[h][0], src, la);
    pg_glds16(o[h][1], src, la + 8192);
  };
  const int xrd = (64 * grp + (lane & 15)) * 128;
  const int sw = lane & 7;
  auto rd_x = [&](int buf, int h, int i, int kk) {
    return *reinterpret_cast<const bf16x8_t*>(smem + buf + h * PP_HALF + xrd + i * 16 * 128 +
                                              (((4 * kk + (lane >> 4)) ^ sw) << 4));
  };
  auto rd_w = [&](int buf, int j, int kk) {
    const int T = 4 * wc + j;
    return *reinterpret_cast<const bf16x8_t*>(smem + buf + (2 + (T >> 3)) * PP_HALF + (2 * (T & 7) + kk) * 1024 +
                                              16 * lane);
  };

  // prologue (nk >= 2, checked by the launcher): K-tile 0 whole, K-tile 1's X0 / W0 / W1
  issue_x(0, 0, vx, 0);
  issue_w(0, 0, vw, 0);
  issue_w(0, 0, vw, 1);
  issue_x(0, 0, vx, 1);
  issue_x(1, 1, vx, 0);
  issue_w(1, 1, vw, 0);
  issue_w(1, 1, vw, 1);
  pp_wait_barrier<8>();
  if (grp == 1) pp_barrier();   // the stagger: group 1 runs one barrier behind group 0

  f32x4_t acc[8][4];
  bf16x8_t wf[4][2], xf[4][2];
  int par = 0;          // LDS slot of K-tile 0 of the current tile (stream position parity)
  bool st = false;      // S epilogue stores of the previous tile still counted in vmcnt
  for (;;) {
#pragma unroll
    for (int i = 0; i < 8; ++i)
#pragma unroll
      for (int j = 0; j < 4; ++j) acc[i][j] = f32x4_t{0.f, 0.f, 0.f, 0.f};
    // K-tile kt of this tile.  TAIL false: kt + 2 < nk (this tile's DMA only, no branches); TAIL
    // true: the last two K-tiles, whose DMA issues continue into the next tile (its K-tile 0 in
    // segment B of kt = nk - 2 and segment A of kt = nk - 1, its K-tile 1 in segment B of nk - 1).
    // Each wait keeps exactly the younger operations that exist in flight: A retires X1(kt) under
    // [X0 W0 W1 (kt+1), held stores, X1 (kt+1)]; B retires X0 W0 W1 (kt+1) under [held stores,
    // X1 (kt+1), X0 W0 W1 (kt+2)], where a position past this tile exists only with a next tile.
    auto step = [&](int kt, auto tail_tag, bool held) {
      constexpr bool TAIL = decltype(tail_tag)::value;
      const int s0 = (kt + par) & 1, s1 = s0 ^ 1;   // slots of K-tiles kt (and kt + 2), kt + 1
      const int buf = s0 * PP_BUF;
      const bool e1 = !TAIL || kt + 1 < nk || has_next;   // position kt + 1 exists
      // ======== segment A: position kt+1's X1; fragments of K-tile kt
      if (!TAIL || kt + 1 < nk) issue_x(kt + 1, s1, vx, 1);
      else if (has_next) issue_x(0, s1, nx, 1);
#pragma unroll
      for (int j = 0; j < 4; ++j)
#pragma unroll
        for (int kk = 0; kk < 2; ++kk) wf[j][kk] = rd_w(buf, j, kk);
#pragma unroll
      for (int i = 0; i < 4; ++i)
#pragma unroll
        for (int kk = 0; kk < 2; ++kk) xf[i][kk] = rd_x(buf, 0, i, kk);
      if (held) pp_wait_barrier<8 + PPP_S>();   // (held: kt = 0, so kt + 1 exists)
      else if (e1) pp_wait_barrier<8>();
      else pp_wait_barrier<0>();
      __builtin_amdgcn_sched_barrier(0);
#pragma unroll
      for (int kk = 0; kk < 2; ++kk)
#pragma unroll
        for (int i = 0; i < 4; ++i)
#pragma unroll
          for (int j = 0; j < 4; ++j)
            acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(wf[j][kk], xf[i][kk], acc[i][j], 0, 0, 0);
      __builtin_amdgcn_sched_barrier(0);
      pp_barrier();
      // ======== segment B: position kt+2's X0 / W0 / W1 (slot s0); K-tile kt's X1 fragments
      if constexpr (!TAIL) {
        issue_x(kt + 2, s0, vx, 0);
        issue_w(kt + 2, s0, vw, 0);
        issue_w(kt + 2, s0, vw, 1);
      } else if (has_next) {
        // the next tile's offsets, live from kt = nk - 2 to the tile switch only
        if (kt == nk - 2) offsets(m0n, n0n, nx, nwv);
        issue_x(kt + 2 - nk, s0, nx, 0);
        issue_w(kt + 2 - nk, s0, nwv, 0);
        issue_w(kt + 2 - nk, s0, nwv, 1);
      }
#pragma unroll
      for (int i = 0; i < 4; ++i)
#pragma unroll
        for (int kk = 0; kk < 2; ++kk) xf[i][kk] = rd_x(buf, 1, i, kk);
      const bool e2 = !TAIL || has_next;   // position kt + 2 exists
      if (held) {
        if (e2) pp_wait_barrier<8 + PPP_S>();
        else pp_wait_barrier<2 + PPP_S>();
      } else if (e2) {
        pp_wait_barrier<8>();
      } else if (e1) {
        pp_wait_barrier<2>();
      } else {
        pp_wait_barrier<0>();
      }
      __builtin_amdgcn_sched_barrier(0);
#pragma unroll
      for (int kk = 0; kk < 2; ++kk)
#pragma unroll
        for (int i = 0; i < 4; ++i)
#pragma unroll
          for (int j = 0; j < 4; ++j)
            acc[4 + i][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(wf[j][kk], xf[i][kk], acc[4 + i][j], 0, 0, 0);
      __builtin_amdgcn_sched_barrier(0);
      pp_barrier();
    };
    int kt = 0;
    for (; kt < nk - 2; ++kt) step(kt, std::false_type{}, st && kt == 0);
    for (; kt < nk; ++kt) step(kt, std::true_type{}, st && kt == 0);
    // ---- epilogue of this tile (no LDS: the next tile's DMA is already landing there)
    const int mw = m0 + grp * 128, nw0 = n0 + wc * 64;
    if (mw + 128 <= M && nw0 + 64 <= N) {
      const int g = lane >> 4;
#pragma unroll
      for (int i = 0; i < 8; ++i) {
        const int m = mw + i * 16 + (lane & 15);
#pragma unroll
        for (int j = 0; j < 4; ++j) {
          const int nb = nw0 + j * 16;
          float v[4] = {acc[i][j][0], acc[i][j][1], acc[i][j][2], acc[i][j][3]};
          if constexpr (EPI == PG_SWIGLU && !STG) {
            ppp_st4(out + (size_t)m * ldo + nb / 2 + pg_swiglu_col(g), pg_swiglu2(v));
          } else if constexpr (!STG) {
            ppp_st8(out + (size_t)m * ldo + nb + 4 * g, make_uint2(pack2bf(v[0], v[1]), pack2bf(v[2], v[3])));
          }
        }
      }
      if constexpr (STG && EPI == PG_SWIGLU) {
        // 2 chunks of 64 rows (m-tiles 4q .. 4q+3): 64-byte rows (32 output columns), 16-byte units
        // XOR-swizzled by the row (4 per row); each lane's two outputs (4 bytes) land at column
        // 8 j + pg_swiglu_col(g) of the chunk row, read back as whole units, stored as 64-byte row
        // segments (8 x 16 B per wave instead of 32 x 4 B)
        char* region = smem + 2 * PP_BUF + w * PPP_REGION;
        const int rl = lane & 15;
#pragma unroll
        for (int q = 0; q < 2; ++q) {
#pragma unroll
          for (int ii = 0; ii < 4; ++ii) {
            const int r = 16 * ii + rl;
#pragma unroll
            for (int j = 0; j < 4; ++j) {
              const f32x4_t& a = acc[4 * q + ii][j];
              const float v[4] = {a[0], a[1], a[2], a[3]};
              *reinterpret_cast<uint32_t*>(region + r * 64 + ((j ^ (r & 3)) << 4) + 2 * pg_swiglu_col(g)) =
                  pg_swiglu2(v);
            }
          }
          __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
          __builtin_amdgcn_wave_barrier();
          __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
#pragma unroll
          for (int s4 = 0; s4 < 4; ++s4) {
            const int r = 16 * s4 + (lane >> 2), unit = lane & 3;
            const uint4 val = *reinterpret_cast<const uint4*>(region + r * 64 + ((unit ^ (r & 3)) << 4));
            ppp_st16(out + (size_t)(mw + 64 * q + r) * ldo + nw0 / 2 + unit * 8, val);
          }
          __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
          __builtin_amdgcn_wave_barrier();
          __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
        }
      } else if constexpr (STG) {
        // 4 chunks of 32 rows (m-tiles 2q, 2q+1): 16-byte units XOR-swizzled by the row (8 per row),
        // written as 8-byte halves, read back as whole units, stored as 128-byte row segments
        char* region = smem + 2 * PP_BUF + w * PPP_REGION;
        const int rl = lane & 15;
#pragma unroll
        for (int q = 0; q < 4; ++q) {
#pragma unroll
          for (int ii = 0; ii < 2; ++ii) {
            const int r = 16 * ii + rl;
#pragma unroll
            for (int j = 0; j < 4; ++j) {
              const f32x4_t& a = acc[2 * q + ii][j];
              const int unit = (2 * j + (g >> 1)) ^ (r & 7);
              *reinterpret_cast<uint2*>(region + r * 128 + unit * 16 + (g & 1) * 8) =
                  make_uint2(pack2bf(a[0], a[1]), pack2bf(a[2], a[3]));
            }
          }
          __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
          __builtin_amdgcn_wave_barrier();
          __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
#pragma unroll
          for (int s4 = 0; s4 < 4; ++s4) {
            const int r = 8 * s4 + (lane >> 3), unit = lane & 7;
            const uint4 val = *reinterpret_cast<const uint4*>(region + r * 128 + ((unit ^ (r & 7)) << 4));
            ppp_st16(out + (size_t)(mw + 32 * q + r) * ldo + nw0 + unit * 8, val);
          }
          // the next chunk rewrites the region: every lane's reads of this one returned (the stores
          // above consumed them), and the wave's LDS operations stay in order
          __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
          __builtin_amdgcn_wave_barrier();
          __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
        }
      }
      st = true;
    } else {
      pg_epilogue<EPI>(acc, nullptr, out, M, N, ldo, mw, nw0);
      asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
      st = false;
    }
    if (!has_next) break;
    par ^= nk & 1;
    vb += G;
    m0 = m0n;
    n0 = n0n;
#pragma unroll
    for (int h = 0; h < 2; ++h)
#pragma unroll
      for (int i = 0; i < 2; ++i) {
        vx[h][i] = nx[h][i];
        vw[h][i] = nwv[h][i];
      }
    has_next = vb + G < nwg;
    if (has_next) coords(vb + G, m0n, n0n);
  }
  if (grp == 0) pp_barrier();   // matches group 1's stagger barrier
}


// ---- encoder sub-layer epilogue: Y = LayerNorm(X . W^T + bias + residual) --------------------------
// The post-LN BERT projections whose output width is the hidden size (o-proj K = hidden, FFN down
// K = 4 x hidden) for hidden NC16 x 16 (384: MiniLM / bge-small).  A workgroup owns WHOLE rows: a
// 128-row x N tile, so the row statistics of the LayerNorm are reduced inside it (waves' partial
// sums through LDS) and the normalised row is written once -- no bf16 round trip of the projection
// output and no separate residual + LayerNorm pass.
//   * 8 waves = 2 (M) x 4 (N), wave tile 64 rows x N/4 columns: acc[4][NC16/4] tiles of 16 x 16;
//   * K in 64-deep tiles, A (128 rows) and B (N rows) images staged by LDS-DMA in 8-row x 128-B
//     pieces, XOR-swizzled through the source address as the 2-stage kernel, two LDS stages;
//   * epilogue numerics as the unfused path: projection rounded to bf16, then bias + residual and
//     the LayerNorm in fp32 (mean and E[x^2] - mean^2 over the row), gamma / beta, bf16 store.
template <int NC16>
__global__ void __launch_bounds__(512, 1)
    pgemm_ln_kernel(const uint16_t* __restrict__ X, const uint16_t* __restrict__ W, const uint16_t* __restrict__ bias,
                    const uint16_t* __restrict__ residual, const uint16_t* __restrict__ gamma,
                    const uint16_t* __restrict__ beta, uint16_t* __restrict__ out, int M, int K, float eps) {
  constexpr int N = NC16 * 16, BM = 128, JT = NC16 / 4;           // JT column tiles per wave
  constexpr int STAGE = (BM + N) * PG_BK * 2;
  constexpr int PA = BM / 8 / 8, PB = N / 8 / 8;                  // DMA pieces per wave per stage
  static_assert(NC16 % 4 == 0 && N % 64 == 0, "N = 64 k, split over 4 waves in 16-column tiles");
  static_assert(2 * STAGE <= 160 * 1024, "two stages must fit the LDS");
  __shared__ __attribute__((aligned(16))) char smem[2 * STAGE];
  const int lane = threadIdx.x & 63;
  const int w = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  const int wr = w >> 2, wc = w & 3;
  const int m0 = blockIdx.x * BM;

  const int prow = lane >> 3, pch = (lane & 7) ^ prow;
  uint32_t va[PA], vb[PB];
#pragma unroll
  for (int i = 0; i < PA; ++i) va[i] = ((uint32_t)min(m0 + 8 * (8 * i + w) + prow, M - 1) * (uint32_t)K + 8u * pch) * 2u;
#pragma unroll
  for (int i = 0; i < PB; ++i) vb[i] = ((uint32_t)(8 * (8 * i + w) + prow) * (uint32_t)K + 8u * pch) * 2u;
  const uint32_t lds0 = __builtin_amdgcn_readfirstlane((uint32_t)(uintptr_t)(pg_lds_t*)smem + w * 1024);
  auto issue = [&](int t, int s) {
    const uint16_t* xa = X + (size_t)t * PG_BK;
    const uint16_t* wb = W + (size_t)t * PG_BK;
    const uint32_t la = lds0 + s * STAGE;
#pragma unroll
    for (int i = 0; i < PA; ++i) pg_glds16(va[i], xa, la + i * 8192);
#pragma unroll
    for (int i = 0; i < PB; ++i) pg_glds16(vb[i], wb, la + BM * 128 + i * 8192);
  };

  f32x4_t acc[4][JT];
#pragma unroll
  for (int i = 0; i < 4; ++i)
#pragma unroll
    for (int j = 0; j < JT; ++j) acc[i][j] = f32x4_t{0.f, 0.f, 0.f, 0.f};
  const int frow = (lane & 15) * 128;
  const int nk = K / PG_BK;
  issue(0, 0);
  for (int t = 0; t < nk; ++t) {
    asm volatile("s_waitcnt vmcnt(0) lgkmcnt(0)\n\ts_barrier" ::: "memory");
    if (t + 1 < nk) issue(t + 1, (t + 1) & 1);
    const char* sa = smem + (t & 1) * STAGE + wr * 64 * 128 + frow;
    const char* sb = smem + (t & 1) * STAGE + BM * 128 + wc * (N / 4) * 128 + frow;
#pragma unroll
    for (int kk = 0; kk < 2; ++kk) {
      const int ch = ((4 * kk + (lane >> 4)) ^ (lane & 7)) << 4;
      bf16x8_t af[4], bw[JT];
#pragma unroll
      for (int i = 0; i < 4; ++i) af[i] = *reinterpret_cast<const bf16x8_t*>(sa + i * 16 * 128 + ch);
#pragma unroll
      for (int j = 0; j < JT; ++j) bw[j] = *reinterpret_cast<const bf16x8_t*>(sb + j * 16 * 128 + ch);
#pragma unroll
      for (int i = 0; i < 4; ++i)
#pragma unroll
        for (int j = 0; j < JT; ++j) acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(bw[j], af[i], acc[i][j], 0, 0, 0);
    }
  }

  // ---- epilogue: lane holds rows m0 + 64 wr + 16 i + (lane & 15), columns n0w + 16 j + 4 g + e
  const int g = lane >> 4;
  const int n0w = wc * (N / 4);
  float s1[4], s2[4];
#pragma unroll
  for (int i = 0; i < 4; ++i) {
    const int m = m0 + wr * 64 + i * 16 + (lane & 15);
    s1[i] = s2[i] = 0.f;
#pragma unroll
    for (int j = 0; j < JT; ++j) {
      const int n = n0w + j * 16 + 4 * g;
      const uint2 bb = *reinterpret_cast<const uint2*>(bias + n);
      uint2 rr = make_uint2(0u, 0u);
      if (m < M) rr = *reinterpret_cast<const uint2*>(residual + (size_t)m * N + n);
      float v[4];
      v[0] = pg_bfr(acc[i][j][0]) + __uint_as_float(bb.x << 16) + __uint_as_float(rr.x << 16);
      v[1] = pg_bfr(acc[i][j][1]) + __uint_as_float(bb.x & 0xffff0000u) + __uint_as_float(rr.x & 0xffff0000u);
      v[2] = pg_bfr(acc[i][j][2]) + __uint_as_float(bb.y << 16) + __uint_as_float(rr.y << 16);
      v[3] = pg_bfr(acc[i][j][3]) + __uint_as_float(bb.y & 0xffff0000u) + __uint_as_float(rr.y & 0xffff0000u);
#pragma unroll
      for (int e = 0; e < 4; ++e) {
        acc[i][j][e] = v[e];
        s1[i] += v[e];
        s2[i] += v[e] * v[e];
      }
    }
    // the row's 4 column groups of this wave (lanes l, l ^ 16, l ^ 32, l ^ 48)
    s1[i] = xor16_sum(s1[i]);
    s1[i] = xor32_sum(s1[i]);
    s2[i] = xor16_sum(s2[i]);
    s2[i] = xor32_sum(s2[i]);
  }
  // the 4 waves of a row band through LDS: red[wc][row][2] (the stages are free after the barrier)
  float* red = reinterpret_cast<float*>(smem);
  __syncthreads();
  if (g == 0) {
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      const int r = wr * 64 + i * 16 + (lane & 15);
      red[(wc * BM + r) * 2] = s1[i];
      red[(wc * BM + r) * 2 + 1] = s2[i];
    }
  }
  __syncthreads();
#pragma unroll
  for (int i = 0; i < 4; ++i) {
    const int r = wr * 64 + i * 16 + (lane & 15);
    const int m = m0 + r;
    float t1 = 0.f, t2 = 0.f;
#pragma unroll
    for (int q = 0; q < 4; ++q) {
      t1 += red[(q * BM + r) * 2];
      t2 += red[(q * BM + r) * 2 + 1];
    }
    const float mean = t1 * (1.f / N);
    const float rstd = rsqrtf(fmaxf(t2 * (1.f / N) - mean * mean, 0.f) + eps);
    if (m >= M) continue;
#pragma unroll
    for (int j = 0; j < JT; ++j) {
      const int n = n0w + j * 16 + 4 * g;
      const uint2 gg = *reinterpret_cast<const uint2*>(gamma + n);
      const uint2 be = *reinterpret_cast<const uint2*>(beta + n);
      const float y0 = (acc[i][j][0] - mean) * rstd * __uint_as_float(gg.x << 16) + __uint_as_float(be.x << 16);
      const float y1 = (acc[i][j][1] - mean) * rstd * __uint_as_float(gg.x & 0xffff0000u) + __uint_as_float(be.x & 0xffff0000u);
      const float y2 = (acc[i][j][2] - mean) * rstd * __uint_as_float(gg.y << 16) + __uint_as_float(be.y << 16);
      const float y3 = (acc[i][j][3] - mean) * rstd * __uint_as_float(gg.y & 0xffff0000u) + __uint_as_float(be.y & 0xffff0000u);
      *reinterpret_cast<uint2*>(out + (size_t)m * N + n) = make_uint2(pack2bf(y0, y1), pack2bf(y2, y3));
    }
  }
}

// ---- v4: four waves of 128 x 128, one per SIMD, software-pipelined -----------------------------
// The library's shape of the same tile (hipBLASLt MT256x256x64, 4 waves: profiles/
// r03s2_pmc_pgemm_vs_hipblaslt.txt): a wave owns a 128 x 128 output block (64 accumulator tiles,
// 256 registers -- the AGPR half of the file), so each MFMA costs half the LDS fragment bytes of the
// 8-wave kernels' 128 x 64 blocks (16 ds_read_b128 per 64 MFMAs) -- less LDS traffic and less
// energy per flop, which is what the clock under DVFS rewards (guide §5.4 rule 28).  With one wave
// per SIMD nothing else covers its waits, so the wave pipelines itself:
//   * K in 32-deep steps through a ring of 4 LDS stages (X image 256 rows x 64 B + W image 16
//     fragments, 32 KB per stage); the DMA of step t + 4 is issued at the top of step t into the
//     stage step t just vacated: three steps (~3k cycles of MFMA) to land;
//   * fragments of step t + 1 are read from LDS into the second register set DURING step t's 64
//     MFMAs (one ds_read_b128 per 3 MFMAs, all issued by MFMA 45 so they land before the step
//     ends); the step's 8 DMA pieces are interleaved the same way;
//   * one barrier per step, behind a counted vmcnt (step t + 1's DMA; t + 2, t + 3 stay in flight)
//     and lgkmcnt(0) (step t + 1's fragments in registers, every read of stage t % 4 retired).
// X image: 64-B rows (16-row x 64-B DMA pieces), chunk c of row r at r*64 + ((c ^ f((r >> 2) & 3)) << 4),
// f = 0,3,2,1: conflict-free 16-row fragment reads (the ring kernel's image).  W: packed fragments
// (1 KB each, lane order) or a row-major image like X.
constexpr int W4_BK = 32;
constexpr int W4_STAGE = (PG_BM + PG_BN) * W4_BK * 2;   // 32 KB
constexpr int W4_NS = 4;

template <int EPI, bool PACKED>
__global__ void __launch_bounds__(256, 1)
    pgemm_w4_kernel(const uint16_t* __restrict__ X, const uint16_t* __restrict__ W, const uint16_t* __restrict__ bias,
                    uint16_t* __restrict__ out, int M, int N, int K, int ldo, int tiles_m, int tiles_n, int wnw) {
  __shared__ __attribute__((aligned(16))) char smem[W4_NS * W4_STAGE];
  const int lane = threadIdx.x & 63;
  const int w = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  const int wr = w >> 1, wc = w & 1;

  const int nwg = tiles_m * tiles_n;
  const int id = xcd_remap(blockIdx.x, nwg);
  const int per_group = PG_GROUP_M * tiles_n;
  const int first_m = (id / per_group) * PG_GROUP_M;
  const int gsz = min(tiles_m - first_m, PG_GROUP_M);
  const int in_group = id % per_group;
  const int m0 = (first_m + in_group % gsz) * PG_BM;
  const int n0 = (in_group / gsz) * PG_BN;
  const int ns = K / W4_BK;                       // even (K % 64 == 0)

  // ---- DMA sources: pieces p = w + 4 i (i = 0..3) of each image.  X piece = image rows 16 p ..
  // 16 p + 15 (lane: row lane >> 2, slot lane & 3 through the swizzle)
  const int prow = lane >> 2, pch = (lane & 3) ^ pr_f((prow >> 2) & 3);
  uint32_t vx[4], vw[4];
  const int kg_all = K / 32;
#pragma unroll
  for (int i = 0; i < 4; ++i) {
    const int p = w + 4 * i;
    vx[i] = ((uint32_t)min(m0 + 16 * p + prow, M - 1) * (uint32_t)K + 8u * pch) * 2u;
    if constexpr (PACKED) {
      const int g = min(n0 / 16 + p, N / 16 - 1);
      vw[i] = (uint32_t)((g / wnw) * kg_all * wnw + g % wnw) * 1024u + 16u * lane;
    } else {
      vw[i] = ((uint32_t)min(n0 + 16 * p + prow, N - 1) * (uint32_t)K + 8u * pch) * 2u;
    }
  }
  const uint32_t lds0 = __builtin_amdgcn_readfirstlane((uint32_t)(uintptr_t)(pg_lds_t*)smem + w * 1024);
  const size_t wstep = PACKED ? (size_t)wnw * 512 : (size_t)W4_BK;   // per step: one k group / 32 columns
  auto issue_piece = [&](int t, int i) {        // piece i (0..3: X, 4..7: W) of step t
    const uint32_t la = lds0 + (t & (W4_NS - 1)) * W4_STAGE;
    if (i < 4) pg_glds16(vx[i], X + (size_t)t * W4_BK, la + i * 4096);
    else pg_glds16(vw[i - 4], W + (size_t)t * wstep, la + PG_BM * 64 + (i - 4) * 4096);
  };

  f32x4_t acc[8][8];
#pragma unroll
  for (int i = 0; i < 8; ++i)
#pragma unroll
    for (int j = 0; j < 8; ++j) acc[i][j] = f32x4_t{0.f, 0.f, 0.f, 0.f};

  // fragment reads of step t: X m-tile i = image rows 16 (8 wr + i) + (lane & 15); W n-tile j
  const int fr = lane & 15;
  const int xch = ((lane >> 4) ^ pr_f((fr >> 2) & 3)) << 4;
  const char* xrd = smem + (wr * 128 + fr) * 64 + xch;
  const char* wrd = PACKED ? smem + PG_BM * 64 + wc * 8 * 1024 + 16 * lane : smem + PG_BM * 64 + (wc * 128 + fr) * 64 + xch;
  auto rd_x = [&](int t, int i) {
    return *reinterpret_cast<const bf16x8_t*>(xrd + (t & (W4_NS - 1)) * W4_STAGE + i * 16 * 64);
  };
  auto rd_w = [&](int t, int j) {
    return *reinterpret_cast<const bf16x8_t*>(wrd + (t & (W4_NS - 1)) * W4_STAGE + j * (PACKED ? 1024 : 16 * 64));
  };

  // ---- prologue: steps 0..3 issued, step 0 landed everywhere, its fragments in set A
#pragma unroll
  for (int t = 0; t < W4_NS; ++t)
    if (t < ns)
#pragma unroll
      for (int i = 0; i < 8; ++i) issue_piece(t, i);
  {
    const int ahead = min(ns - 1, W4_NS - 1);     // steps issued after step 0
    if (ahead >= 3) pp_wait_barrier<24>();
    else if (ahead == 2) pp_wait_barrier<16>();
    else pp_wait_barrier<8>();
  }
  bf16x8_t fa_x[8], fa_w[8], fb_x[8], fb_w[8];
#pragma unroll
  for (int i = 0; i < 8; ++i) fa_x[i] = rd_x(0, i);
#pragma unroll
  for (int j = 0; j < 8; ++j) fa_w[j] = rd_w(0, j);

  // One step: wait for step t + 1's DMA and every wave's reads of stage t, barrier, DMA of step
  // t + 4 into stage t, 64 MFMAs on (cx, cw) with step t + 1's fragments read into (nx, nw).
#define W4_STEP(T, CX, CW, NX, NWF)                                                                     \
  do {                                                                                                  \
    const int t_ = (T);                                                                                 \
    const int ahead_ = min(ns - 1, t_ + 3) - (t_ + 1);    /* steps issued after step t+1 */            \
    if (ahead_ >= 2) pp_wait_barrier<16>();                                                             \
    else if (ahead_ == 1) pp_wait_barrier<8>();                                                         \
    else pp_wait_barrier<0>();                                                                          \
    const bool more_ = t_ + 1 < ns, dma_ = t_ + W4_NS < ns;                                             \
    __builtin_amdgcn_sched_barrier(0);                                                                  \
    _Pragma("unroll") for (int q = 0; q < 16; ++q) {                                                    \
      _Pragma("unroll") for (int e = 0; e < 4; ++e) {                                                   \
        const int mm = 4 * q + e, i = mm >> 3, j = mm & 7;                                              \
        acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(CW[j], CX[i], acc[i][j], 0, 0, 0);          \
      }                                                                                                 \
      if (q < 12) {                                                                                     \
        if (more_) {                                                                                    \
          if (q < 8) NX[q] = rd_x(t_ + 1, q);                                                           \
          else NWF[q - 8] = rd_w(t_ + 1, q - 8);                                                        \
          if (q >= 8) NWF[q - 4] = rd_w(t_ + 1, q - 4);                                                 \
        }                                                                                               \
        if (q < 8 && dma_) issue_piece(t_ + W4_NS, q);                                                  \
      }                                                                                                 \
      __builtin_amdgcn_sched_barrier(0);                                                                \
    }                                                                                                   \
  } while (0)

  for (int t = 0; t < ns; t += 2) {
    W4_STEP(t, fa_x, fa_w, fb_x, fb_w);
    W4_STEP(t + 1, fb_x, fb_w, fa_x, fa_w);
  }
#undef W4_STEP

  pg_epilogue<EPI>(acc, bias, out, M, N, ldo, m0 + wr * 128, n0 + wc * 128);
}

// production probe flags of the ping-pong kernel: no s_setprio (measured 1.5-2.5 % faster than the
// per-segment flips on all four headline shapes, profiles/r04_pgemm_pp_probes.jsonl pf1 vs pf0) and
// W1-early (+0.6-1.7 %: qkv 580 -> 571 us, o 384 -> 378, gate_up 2665 -> 2631, down 1311 -> 1299;
// profiles/r04_pgemm_w1e.jsonl)
constexpr int PP_PF = 1 | 32;

// compute units of the current device (the persistent kernel's grid), looked up once per device
// (relaxed atomics: concurrent first calls store the same value)
int pg_cus() {
  static std::atomic<int> cus[64];
  int dev = 0;
  if (hipGetDevice(&dev) != hipSuccess || dev < 0 || dev >= 64) return 256;
  int n = cus[dev].load(std::memory_order_relaxed);
  if (n == 0) {
    if (hipDeviceGetAttribute(&n, hipDeviceAttributeMultiprocessorCount, dev) != hipSuccess || n < 1) n = 256;
    cus[dev].store(n, std::memory_order_relaxed);
  }
  return n;
}

// LDS-staged 16-byte epilogue stores in the persistent kernel (bf16 and SwiGLU)
constexpr bool PPP_STG = true;

// M-tiles per N sweep of the persistent kernel's tile order.  Measured (scripts/probe_ppp_gm.py,
// profiles/r06_ppp_gm.jsonl, gm 2 / 4 / 8 / 16): 8 is best on qkv, o and gate_up; the long-K,
// narrow-N down projection (K = 14336, 16 N-tiles) runs 2.3 % faster at 4 (round 4 saw the same
// on the one-tile kernel: r04_pgemm_pp_probes.jsonl)
int ppp_group_m(int tiles_n, int K) { return (K >= 8192 && tiles_n <= 16) ? 4 : PG_GROUP_M; }

template <int EPI>
int ppp_launch(const uint16_t* xp, const uint16_t* wp, uint16_t* op, int M, int N, int K, int ldo, int wnw, int gm,
               bool stg, hipStream_t stream) {
  const int tm = (M + PG_BM - 1) / PG_BM, tn = (N + PG_BN - 1) / PG_BN;
  if (stg)
    pgemm_ppp_kernel<EPI, true><<<min(tm * tn, pg_cus()), 512, 0, stream>>>(xp, wp, op, M, N, K, ldo, tm, tn, wnw, gm);
  else
    pgemm_ppp_kernel<EPI, false><<<min(tm * tn, pg_cus()), 512, 0, stream>>>(xp, wp, op, M, N, K, ldo, tm, tn, wnw, gm);
  return (int)hipGetLastError();
}

template <int EPI>
int pgemm_launch(const void* x, const void* w, const void* bias, void* out, int M, int N, int K, int ldo,
                 int variant, int wnw, hipStream_t stream) {
  const int tm = (M + PG_BM - 1) / PG_BM, tn = (N + PG_BN - 1) / PG_BN;
  const uint16_t *xp = (const uint16_t*)x, *wp = (const uint16_t*)w, *bp = (const uint16_t*)bias;
  uint16_t* op = (uint16_t*)out;
  if (wnw > 0) {   // fragment-packed W: the ping-pong (default) or the 4-wave kernel
    if (variant == 4) pgemm_w4_kernel<EPI, true><<<tm * tn, 256, 0, stream>>>(xp, wp, bp, op, M, N, K, ldo, tm, tn, wnw);
    else if (variant == 5)   // LDS-staged bf16 / SwiGLU epilogue
      pgemm_pp_kernel<EPI, true, PP_PF | 64><<<tm * tn, 512, 0, stream>>>(xp, wp, bp, op, M, N, K, ldo, tm, tn, wnw);
    else if (variant == 6) {   // persistent: one workgroup per CU walking the tiles
      // (bias epilogues and K < 128 take the non-persistent kernel)
      if constexpr (EPI == PG_BF16 || EPI == PG_SWIGLU) {
        if (K >= 2 * PG_BK) return ppp_launch<EPI>(xp, wp, op, M, N, K, ldo, wnw, ppp_group_m(tn, K), PPP_STG, stream);
      }
      pgemm_pp_kernel<EPI, true, PP_PF><<<tm * tn, 512, 0, stream>>>(xp, wp, bp, op, M, N, K, ldo, tm, tn, wnw);
    }
    else pgemm_pp_kernel<EPI, true, PP_PF><<<tm * tn, 512, 0, stream>>>(xp, wp, bp, op, M, N, K, ldo, tm, tn, wnw);
    return (int)hipGetLastError();
  }
  switch (variant) {
    case 0: pgemm_ring_kernel<EPI, 5><<<tm * tn, 512, 0, stream>>>(xp, wp, bp, op, M, N, K, ldo, tm, tn); break;
    case 1: pgemm_kernel<EPI><<<tm * tn, 512, 0, stream>>>(xp, wp, bp, op, M, N, K, ldo, tm, tn); break;
    case 2: pgemm_ring_kernel<EPI, 4><<<tm * tn, 512, 0, stream>>>(xp, wp, bp, op, M, N, K, ldo, tm, tn); break;
    case 3: pgemm_pp_kernel<EPI, false, PP_PF><<<tm * tn, 512, 0, stream>>>(xp, wp, bp, op, M, N, K, ldo, tm, tn, 1); break;
    case 4: pgemm_w4_kernel<EPI, false><<<tm * tn, 256, 0, stream>>>(xp, wp, bp, op, M, N, K, ldo, tm, tn, 1); break;
    case 5: pgemm_pp_kernel<EPI, false, PP_PF | 64><<<tm * tn, 512, 0, stream>>>(xp, wp, bp, op, M, N, K, ldo, tm, tn, 1); break;
    case 6: pgemm_pp_kernel<EPI, false, PP_PF><<<tm * tn, 512, 0, stream>>>(xp, wp, bp, op, M, N, K, ldo, tm, tn, 1); break;
    default: return (int)hipErrorInvalidValue;
  }
  return (int)hipGetLastError();
}

// fp32 output: the ping-pong kernel only (packed or row-major W)
int pgemm_launch_f32(const void* x, const void* w, void* out, int M, int N, int K, int ldo, int wnw,
                     hipStream_t stream) {
  const int tm = (M + PG_BM - 1) / PG_BM, tn = (N + PG_BN - 1) / PG_BN;
  const uint16_t *xp = (const uint16_t*)x, *wp = (const uint16_t*)w;
  uint16_t* op = (uint16_t*)out;
  if (wnw > 0) pgemm_pp_kernel<PG_F32, true, PP_PF><<<tm * tn, 512, 0, stream>>>(xp, wp, nullptr, op, M, N, K, ldo, tm, tn, wnw);
  else pgemm_pp_kernel<PG_F32, false, PP_PF><<<tm * tn, 512, 0, stream>>>(xp, wp, nullptr, op, M, N, K, ldo, tm, tn, 1);
  return (int)hipGetLastError();
}

}  // namespace

// epi & 15: 0 bf16, 1 + bias, 2 + bias -> GELU, 3 SwiGLU (out [M, N/2]); epi >> 4: K-loop variant
// for a row-major W (0 BK = 32 ring of 5 slots, 1 the 2-stage BK = 64 kernel, 2 ring of 4 slots,
// 3 the ping-pong kernel, 5 the same with the LDS-staged bf16 / SwiGLU epilogue, 6 the persistent
// ping-pong kernel for a packed W -- the ping-pong kernel otherwise); ldo = output row stride.  wnw > 0: W is in the decode GEMM's
// fragment-packed layout for bn = 16 wnw (cfc_dgemm_pack; N % (16 wnw) == 0) and runs on the
// ping-pong kernel whatever the variant.
CFC_API int cfc_pgemm(const void* x, const void* w, const void* bias, void* out, int M, int N, int K, int epi_v,
                      int ldo, int wnw, hipStream_t stream) {
  const int epi = epi_v & 15, variant = epi_v >> 4;
  if (M < 1 || N < 64 || K < 64 || K % 64 || N % 64 || ldo % 4 || (epi != 3 && ldo < N) ||
      (epi == 3 && ldo < N / 2) || (uint64_t)M * K * 2 >= (1ull << 32) || (uint64_t)N * K * 2 >= (1ull << 32) ||
      ((epi == 1 || epi == 2) && bias == nullptr) || wnw < 0 || (wnw > 0 && N % (16 * wnw)))
    return (int)hipErrorInvalidValue;
  switch (epi) {
    case 0: return pgemm_launch<PG_BF16>(x, w, bias, out, M, N, K, ldo, variant, wnw, stream);
    case 1: return pgemm_launch<PG_BIAS>(x, w, bias, out, M, N, K, ldo, variant, wnw, stream);
    case 2: return pgemm_launch<PG_BIAS_GELU>(x, w, bias, out, M, N, K, ldo, variant, wnw, stream);
    case 3: return pgemm_launch<PG_SWIGLU>(x, w, bias, out, M, N, K, ldo, variant, wnw, stream);
    case 4: return pgemm_launch_f32(x, w, out, M, N, K, ldo, wnw, stream);
    default: return (int)hipErrorInvalidValue;
  }
}

// Timing probe only (scripts/bench_pgemm.py --probe): the ping-pong kernel, bf16 epilogue, packed W
// (wnw > 0), probe flags pf (see pgemm_pp_kernel) and tile-order group gm.
CFC_API int cfc_pgemm_probe(const void* x, const void* w, void* out, int M, int N, int K, int wnw, int pf, int gm,
                            hipStream_t stream) {
  if (M < 1 || K % 64 || N % 64 || wnw < 1 || N % (16 * wnw) || gm < 1) return (int)hipErrorInvalidValue;
  const int tm = (M + PG_BM - 1) / PG_BM, tn = (N + PG_BN - 1) / PG_BN;
  const uint16_t *xp = (const uint16_t*)x, *wp = (const uint16_t*)w;
  uint16_t* op = (uint16_t*)out;
#define PP_PROBE(F) pgemm_pp_kernel<PG_BF16, true, F><<<tm * tn, 512, 0, stream>>>(xp, wp, nullptr, op, M, N, K, N, tm, tn, wnw, gm); break;
  switch (pf) {
    case 0: PP_PROBE(0)
    case 1: PP_PROBE(1)
    case 2: PP_PROBE(2)
    case 5: PP_PROBE(5)
    case 9: PP_PROBE(9)
    case 13: PP_PROBE(13)
    case 17: PP_PROBE(17)
    case 21: PP_PROBE(21)
    case 33: PP_PROBE(33)
    case 97: PP_PROBE(97)
    default: return (int)hipErrorInvalidValue;
  }
#undef PP_PROBE
  return (int)hipGetLastError();
}

// Timing probe only (scripts/probe_ppp_gm.py): the persistent kernel (packed W, bf16 or SwiGLU
// epilogue: epi 0 / 3, +16 for register-direct instead of LDS-staged stores) with an explicit
// tile-order group gm (M-tiles per N sweep).
CFC_API int cfc_pgemm_ppp_probe(const void* x, const void* w, void* out, int M, int N, int K, int epi_s, int ldo,
                                int wnw, int gm, hipStream_t stream) {
  const int epi = epi_s & 15;
  const bool stg = (epi_s & 16) == 0;   // +16: register-direct epilogue stores
  if (M < 1 || K < 2 * PG_BK || K % 64 || N % 64 || wnw < 1 || N % (16 * wnw) || gm < 1 || (epi != 0 && epi != 3) ||
      ldo < (epi == 3 ? N / 2 : N) || ldo % 4 || (uint64_t)M * K * 2 >= (1ull << 32) || (uint64_t)N * K * 2 >= (1ull << 32))
    return (int)hipErrorInvalidValue;
  const uint16_t *xp = (const uint16_t*)x, *wp = (const uint16_t*)w;
  uint16_t* op = (uint16_t*)out;
  return epi == 0 ? ppp_launch<PG_BF16>(xp, wp, op, M, N, K, ldo, wnw, gm, stg, stream)
                  : ppp_launch<PG_SWIGLU>(xp, wp, op, M, N, K, ldo, wnw, gm, stg, stream);
}

// Y[M, N] = LayerNorm(X[M, K] . W[N, K]^T + bias + residual) * gamma + beta, N = 384 (the encoder
// hidden sizes this kernel is built for), K % 64 == 0; out may not alias residual or X.
CFC_API int cfc_pgemm_ln(const void* x, const void* w, const void* bias, const void* residual, const void* gamma,
                         const void* beta, void* out, int M, int N, int K, float eps, hipStream_t stream) {
  if (M < 1 || K < 64 || K % 64 || N != 384 || (uint64_t)M * K * 2 >= (1ull << 32) || !bias || !residual || !gamma ||
      !beta || out == residual || out == x)
    return (int)hipErrorInvalidValue;
  pgemm_ln_kernel<24><<<(M + 127) / 128, 512, 0, stream>>>(
      (const uint16_t*)x, (const uint16_t*)w, (const uint16_t*)bias, (const uint16_t*)residual, (const uint16_t*)gamma,
      (const uint16_t*)beta, (uint16_t*)out, M, K, eps);
  return (int)hipGetLastError();
}
