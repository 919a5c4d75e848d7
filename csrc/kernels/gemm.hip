// Split-K reduce kernels for the decode GEMM (dgemm.hip) and the library split-K path, and the
// GEMV for single-stream / small-batch decode (M <= 4).
#include "common.h"

namespace {

// Reduce the split-K partials [split][M][N] -> bf16 Y (mode 0) or silu(gate) * up for the
// 8-row interleaved gate/up layout (mode 1, output width N/2).  One thread per 4 output columns.
__global__ void __launch_bounds__(256) splitk_reduce_kernel(const float* __restrict__ part, int split, int M, int N,
                                                            int mode, uint16_t* __restrict__ out, int ldo) {
  const int m = blockIdx.y;
  const int c4 = (blockIdx.x * 256 + threadIdx.x) * 4;   // column (mode 0) / gate column (mode 1)
  if (mode == 0) {
    if (c4 >= N) return;
    float4 s = make_float4(0.f, 0.f, 0.f, 0.f);
    for (int p = 0; p < split; ++p) {
      const float4 v = *reinterpret_cast<const float4*>(part + ((size_t)p * M + m) * N + c4);
      s.x += v.x; s.y += v.y; s.z += v.z; s.w += v.w;
    }
    uint2 o;
    o.x = pack2bf(s.x, s.y);
    o.y = pack2bf(s.z, s.w);
    *reinterpret_cast<uint2*>(out + (size_t)m * ldo + c4) = o;
  } else {
    const int F = N >> 1;
    if (c4 >= F) return;
    const int gcol = 16 * (c4 >> 3) + (c4 & 7), ucol = gcol + 8;
    float4 gs = make_float4(0.f, 0.f, 0.f, 0.f), us = gs;
    for (int p = 0; p < split; ++p) {
      const float* row = part + ((size_t)p * M + m) * N;
      const float4 a = *reinterpret_cast<const float4*>(row + gcol);
      const float4 b = *reinterpret_cast<const float4*>(row + ucol);
      gs.x += a.x; gs.y += a.y; gs.z += a.z; gs.w += a.w;
      us.x += b.x; us.y += b.y; us.z += b.z; us.w += b.w;
    }
    // bf16-round the projection outputs first: the rounding points of GEMM -> silu_mul
    auto sl = [](float x) { x = bf2f(f2bf(x)); return x / (1.f + __expf(-x)); };
    auto rb = [](float x) { return bf2f(f2bf(x)); };
    uint2 o;
    o.x = pack2bf(sl(gs.x) * rb(us.x), sl(gs.y) * rb(us.y));
    o.y = pack2bf(sl(gs.z) * rb(us.z), sl(gs.w) * rb(us.w));
    *reinterpret_cast<uint2*>(out + (size_t)m * ldo + c4) = o;
  }
}

// Reduce partials + residual add + RMSNorm, one block per row (N = hidden, N / 8 <= 1024 threads):
//   h = sum_p part[p][m] + residual[m];  residual[m] <- bf16(h);  out[m] = bf16(norm(bf16(h)) * w)
// (the rounding sequence of rmsnorm_kernel with add_residual, so fused and unfused decode agree).
// SPLIT is a template parameter so every partial, the residual and the norm weight are loaded
// up front with no per-split branch: a runtime-count loop made the compiler wait for each split's
// loads before issuing the next (one dependent L2/HBM round trip per split).
template <int SPLIT>
__global__ void __launch_bounds__(1024) splitk_residual_rmsnorm_kernel(const float* __restrict__ part, int split_rt,
                                                                       int M, int N, uint16_t* __restrict__ residual,
                                                                       const uint16_t* __restrict__ w, float eps,
                                                                       uint16_t* __restrict__ out) {
  __shared__ float red[16];
  const int m = blockIdx.x, c = threadIdx.x;      // c: 8-column group
  const int split = SPLIT > 0 ? SPLIT : split_rt;
  const bool act = c * 8 < N;
  float v[8];
  float ss = 0.f;
  uint4 rr = make_uint4(0, 0, 0, 0), wv = make_uint4(0, 0, 0, 0);
  float s[8] = {0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f};
  uint4* rp = reinterpret_cast<uint4*>(residual + (size_t)m * N) + c;
  if (act) {
    rr = *rp;
    wv = reinterpret_cast<const uint4*>(w)[c];
    if constexpr (SPLIT > 0) {
      float4 a[SPLIT], b[SPLIT];
#pragma unroll
      for (int p = 0; p < SPLIT; ++p) {
        const float4* row = reinterpret_cast<const float4*>(part + ((size_t)p * M + m) * N + c * 8);
        a[p] = row[0];
        b[p] = row[1];
      }
#pragma unroll
      for (int p = 0; p < SPLIT; ++p) {
        s[0] += a[p].x; s[1] += a[p].y; s[2] += a[p].z; s[3] += a[p].w;
        s[4] += b[p].x; s[5] += b[p].y; s[6] += b[p].z; s[7] += b[p].w;
      }
    } else {
      float4 a = make_float4(0.f, 0.f, 0.f, 0.f), b = a;
      slab_sum8(part, split, (size_t)M * N, (size_t)m * N + c * 8, a, b);
      s[0] = a.x; s[1] = a.y; s[2] = a.z; s[3] = a.w; s[4] = b.x; s[5] = b.y; s[6] = b.z; s[7] = b.w;
    }
    float r[8];
    unpack8(rr, r);
    // the projection output is rounded to bf16 first (as the unfused path stores it), then added
#pragma unroll
    for (int j = 0; j < 8; ++j) v[j] = bf2f(f2bf(s[j])) + r[j];
    const uint4 pk = pack8(v);
    *rp = pk;
    unpack8(pk, v);
#pragma unroll
    for (int j = 0; j < 8; ++j) ss += v[j] * v[j];
  }
  ss = block_sum(ss, red);
  const float inv = rsqrtf(ss / (float)N + eps);
  if (act) {
    float gw[8], o[8];
    unpack8(wv, gw);
#pragma unroll
    for (int j = 0; j < 8; ++j) o[j] = v[j] * inv * gw[j];
    reinterpret_cast<uint4*>(out + (size_t)m * N)[c] = pack8(o);
  }
}


// ---------------------------------------------------------------------------------------------
// GEMV for single-stream / small-batch decode (M <= 4): Y[M, N] = X[M, K] . W[N, K]^T.
//
// At M <= 4 a projection is a pure weight stream (0.5-2 flop per byte): no MFMA, no LDS.  Each
// wave owns GV_RW = 2 rows of W and walks K in 512-element chunks (one 16-B load per lane per row);
// GV_CPI = 8 chunks (16 x 16 B per lane, 16 KB per wave) are issued before any FMA so every wave
// keeps its whole K=4096 slice in flight at once, and nontemporal loads keep the once-read weights
// out of L2.  X rows are read from global (L2-resident, re-read once per wave = M/2 of W's bytes).
// The 64 lane partials are summed with a butterfly.  Epilogues: fp32 store (feeds the residual +
// RMSNorm reduce kernel with split = 1), bf16 store, or SwiGLU over the 8-row interleaved gate/up
// weights (the wave's two rows are gate row j and up row j of output column j).
// Grid: one 4-wave block per 8 W rows (4 output columns for SwiGLU) -> 512-3584 blocks for the
// 7B shapes, i.e. >= 2 blocks per CU.
constexpr int GV_RW = 2;
constexpr int GV_CPI = 8;   // chunks in flight per row (4 for M > 2, to stay within 128 VGPRs + AGPRs)
constexpr int GV_CHUNK = 512;
enum { GV_F32 = 0, GV_BF16 = 1, GV_SWIGLU = 2 };
typedef unsigned int gv_u32x4 __attribute__((ext_vector_type(4)));

__device__ __forceinline__ uint4 gv_stream(const uint16_t* p) {
  const gv_u32x4 v = __builtin_nontemporal_load(reinterpret_cast<const gv_u32x4*>(p));
  return make_uint4(v.x, v.y, v.z, v.w);
}

__device__ __forceinline__ float dot8(const uint4 a, const uint4 b) {
  float fa[8], fb[8];
  unpack8(a, fa);
  unpack8(b, fb);
  float s = 0.f;
#pragma unroll
  for (int j = 0; j < 8; ++j) s = fmaf(fa[j], fb[j], s);
  return s;
}

template <int MT, int EPI, int CPI = (MT > 2 ? GV_CPI / 2 : GV_CPI)>
__global__ void __launch_bounds__(256) gemv_kernel(const uint16_t* __restrict__ X, const uint16_t* __restrict__ W,
                                                   int N, int K, float* __restrict__ yf, uint16_t* __restrict__ yb,
                                                   int ldo, int ncols) {
  const int lane = threadIdx.x & 63;
  const int col = blockIdx.x * 4 + (threadIdx.x >> 6);   // output column group of this wave
  if (col >= ncols) return;
  int rows[GV_RW];
  if constexpr (EPI == GV_SWIGLU) {
    rows[0] = 16 * (col >> 3) + (col & 7);    // gate row of output column `col` (8-row groups)
    rows[1] = rows[0] + 8;                    // matching up row
  } else {
    rows[0] = GV_RW * col;
    rows[1] = GV_RW * col + 1;
  }
  float acc[GV_RW][MT];
#pragma unroll
  for (int r = 0; r < GV_RW; ++r)
#pragma unroll
    for (int m = 0; m < MT; ++m) acc[r][m] = 0.f;

  for (int k0 = 0; k0 < K; k0 += CPI * GV_CHUNK) {
    uint4 w[GV_RW][CPI], x[MT][CPI];
#pragma unroll
    for (int c = 0; c < CPI; ++c) {
      const int k = k0 + c * GV_CHUNK + lane * 8;
#pragma unroll
      for (int r = 0; r < GV_RW; ++r)
        w[r][c] = k < K ? gv_stream(W + (size_t)rows[r] * K + k) : make_uint4(0, 0, 0, 0);
    }
#pragma unroll
    for (int c = 0; c < CPI; ++c) {
      const int k = k0 + c * GV_CHUNK + lane * 8;
#pragma unroll
      for (int m = 0; m < MT; ++m)
        x[m][c] = k < K ? *reinterpret_cast<const uint4*>(X + (size_t)m * K + k) : make_uint4(0, 0, 0, 0);
    }
#pragma unroll
    for (int c = 0; c < CPI; ++c)
#pragma unroll
      for (int r = 0; r < GV_RW; ++r)
#pragma unroll
        for (int m = 0; m < MT; ++m) acc[r][m] += dot8(w[r][c], x[m][c]);
  }
#pragma unroll
  for (int r = 0; r < GV_RW; ++r)
#pragma unroll
    for (int m = 0; m < MT; ++m) acc[r][m] = wave_sum(acc[r][m]);
  if (lane != 0) return;
#pragma unroll
  for (int m = 0; m < MT; ++m) {
    if constexpr (EPI == GV_SWIGLU) {
      const float g = bf2f(f2bf(acc[0][m])), u = bf2f(f2bf(acc[1][m]));   // bf16 GEMM output, as unfused
      yb[(size_t)m * ldo + col] = f2bf(g / (1.f + __expf(-g)) * u);
    } else if constexpr (EPI == GV_BF16) {
      *reinterpret_cast<uint32_t*>(yb + (size_t)m * ldo + rows[0]) = pack2bf(acc[0][m], acc[1][m]);
    } else {
      *reinterpret_cast<float2*>(yf + (size_t)m * N + rows[0]) = make_float2(acc[0][m], acc[1][m]);
    }
  }
}

// GEMV over the decode GEMM's fragment-packed weight (cfc_dgemm_pack, bn = 16 NW): the B <= 4
// decode path when only the packed copy of a projection exists (one weight copy for prefill,
// batched and single-stream decode).  A packed fragment = 16 W rows x 32 k, lane l holding row
// l & 15, k = 8 (l >> 4) .. +8 -- one 16-byte load per lane, 1 KB per wave instruction; a bn-row
// tile is kg-major: the NW fragments of one kg (NW KB) are contiguous, then the next kg.
//   * workgroup (tile, s) streams k-slice s of one tile: the tile's kg range split S ways, each
//     slice ONE contiguous run of (KG / S) NW KB; its 4 waves take U consecutive kg each per
//     step (a step of the workgroup = 4 U NW contiguous KB), all U NW loads of a step in flight
//     at once (nontemporal buffer loads), one 16-byte activation load per kg shared by the NW
//     fragments of that kg;
//   * S > 1 (host: gemv_packed_split, tiles x S ~ 1024 workgroups) writes fp32 slice partials
//     part[S, M, N] that the consumer sums -- the split-K reduce the decode already runs: RoPE / KV
//     write from slabs for qkv, the residual + RMSNorm reduce for o / down.  A first build summed
//     them in-kernel (last workgroup of a tile, agent-scope fence + ticket): the agent-scope
//     release writes back the whole L2 per workgroup on gfx950 and the GEMV fell to 0.5-2 TB/s
//     (profiles/r04_gemv_bench_fence.jsonl);
//   * the first build -- one workgroup per 16-row group, its waves each streaming one group's
//     1 KB pieces at NW KB stride -- reached 4.0 TB/s at 4 waves x 8 KB in flight and 3.8 TB/s at
//     8 x 16 KB: scattered 1 KB pieces, not bytes in flight, were the limit (single-stream
//     Mistral-7B 261-276 tok/s vs 330 on the row-major GEMV, profiles/r04_latency*);
//   * per lane acc[NW][M]: two xor-shuffles sum the lanes of a row, LDS the 4 waves; epilogues
//     (S = 1) as cfc_gemv: fp32 / bf16 / SwiGLU over the 8-row interleaved gate/up groups (rows
//     16 g + r and 16 g + 8 + r -> output column 8 g + r); fp32 with S > 1 = the slab of slice s.
// The residual + RMSNorm that produces this GEMV's input, folded into its prologue (XN): the
// input is the previous projection's fp32 k-slice slabs, and every workgroup rebuilds the whole
// normalised row in LDS -- h = bf16(bf16(sum of slabs) + residual), x = bf16(h rsqrt(mean h^2 +
// eps) w) -- with the reduce kernel's exact arithmetic (slabs summed in order, the sum of squares
// as its 64-lane waves and their in-order total), so x is bit-identical to
// cfc_splitk_residual_rmsnorm's.  Workgroup 0 stores h to res_out (a different buffer from
// res_in: the other workgroups are still reading it).  The first step's weight loads are issued
// before the prologue, so its slab reads hide under the weight stream instead of a launch.
struct GvNorm {
  const float* part;
  int split;
  const uint16_t* res_in;
  uint16_t* res_out;
  const uint16_t* w;
  float eps;
};

template <int NW, int MT, int WAVES, bool XN>
__global__ void __launch_bounds__(64 * WAVES) gemv_tile_kernel(const uint16_t* __restrict__ X,
                                                        const uint16_t* __restrict__ Wp, int N, int K, int S, int epi,
                                                        float* __restrict__ yf, uint16_t* __restrict__ yb, int ldo,
                                                        GvNorm nm) {
  constexpr int U = MT > 2 ? 2 : (NW >= 7 ? 3 : 4);
  constexpr int R = NW * MT * 16;                  // (group, m, row) values of one tile
  __shared__ float red[WAVES][R];
  extern __shared__ uint4 xs[];                    // XN: the normalised rows [MT][K] (bf16)
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6, q = lane >> 4;
  const int tile = blockIdx.x / S, s = blockIdx.x - tile * S;
  const int KG = K / 32;
  const int kb = s * KG / S, ke = (s + 1) * KG / S;
  const uint16_t* base = Wp + (size_t)tile * KG * NW * 512;
  const uint32_t lo = __builtin_amdgcn_readfirstlane((uint32_t)(uintptr_t)base);
  const uint32_t hi = __builtin_amdgcn_readfirstlane((uint32_t)((uintptr_t)base >> 32));
  const __amdgpu_buffer_rsrc_t rs = __builtin_amdgcn_make_buffer_rsrc(
      (void*)(((uintptr_t)hi << 32) | lo), (short)0, (int)((size_t)KG * NW * 1024), 0x00020000);
  const int voff = 16 * lane;
  float acc[NW][MT];
#pragma unroll
  for (int j = 0; j < NW; ++j)
#pragma unroll
    for (int m = 0; m < MT; ++m) acc[j][m] = 0.f;
#define GVT_LOAD_W(K0)                                                                                 \
  uint4 wv[U][NW];                                                                                     \
  _Pragma("unroll") for (int u = 0; u < U; ++u) {                                                      \
    const int kg = min((K0) + u, ke - 1);          /* tail: re-read the last kg, weight 0 below */     \
    _Pragma("unroll") for (int j = 0; j < NW; ++j) {                                                   \
      const gv_u32x4 v = __builtin_amdgcn_raw_buffer_load_b128(rs, voff + j * 1024, kg * NW * 1024, 2); \
      wv[u][j] = make_uint4(v.x, v.y, v.z, v.w);                                                       \
    }                                                                                                  \
  }
#define GVT_DOT(K0)                                                                                    \
  {                                                                                                    \
    uint4 xv[U][MT];                                                                                   \
    _Pragma("unroll") for (int u = 0; u < U; ++u) {                                                    \
      const int kg = min((K0) + u, ke - 1);                                                            \
      _Pragma("unroll") for (int m = 0; m < MT; ++m) {                                                 \
        if constexpr (XN) xv[u][m] = xs[(m * K + 32 * kg + 8 * q) >> 3];                              \
        else xv[u][m] = *reinterpret_cast<const uint4*>(X + (size_t)m * K + 32 * kg + 8 * q);          \
      }                                                                                                \
    }                                                                                                  \
    _Pragma("unroll") for (int u = 0; u < U; ++u) {                                                    \
      if ((K0) + u < ke) {                                                                             \
        _Pragma("unroll") for (int j = 0; j < NW; ++j)                                                 \
          _Pragma("unroll") for (int m = 0; m < MT; ++m) acc[j][m] += dot8(wv[u][j], xv[u][m]);       \
      }                                                                                                \
    }                                                                                                  \
  }
  if constexpr (!XN) {
    for (int k0 = kb + w * U; k0 < ke; k0 += WAVES * U) {
      GVT_LOAD_W(k0)
      GVT_DOT(k0)
    }
  } else {
    // every wave runs the same step count (a wave past the slice re-reads its last kg, masked), so
    // all of them reach the prologue's barriers; the first step's weight loads go out before it.
    // (Issuing the prologue's first slab / residual / norm loads ahead of the weights, so its wait
    // does not include the weight stream, needs ~64 more VGPRs: it spilled and measured slower.)
    __shared__ float red_ss[MT][32];
    const int nsteps = (ke - kb + WAVES * U - 1) / (WAVES * U);
    for (int st = 0; st < nsteps; ++st) {
      const int k0 = kb + st * WAVES * U + w * U;
      GVT_LOAD_W(k0)
      if (st == 0) {
        const int G = K / 8, nvw = (G + 63) / 64;  // the reduce kernel's block: one 8-column group per thread
        for (int m = 0; m < MT; ++m) {
          for (int vw = w; vw < nvw; vw += WAVES) {
            const int c = vw * 64 + lane;
            float ss = 0.f;
            if (c < G) {
              float4 a = make_float4(0.f, 0.f, 0.f, 0.f), b = a;
              slab_sum8(nm.part, nm.split, (size_t)MT * K, (size_t)m * K + 8 * c, a, b);
              const float sv[8] = {a.x, a.y, a.z, a.w, b.x, b.y, b.z, b.w};
              float r[8], v[8];
              unpack8(*reinterpret_cast<const uint4*>(nm.res_in + (size_t)m * K + 8 * c), r);
#pragma unroll
              for (int j = 0; j < 8; ++j) v[j] = bf2f(f2bf(sv[j])) + r[j];
              const uint4 pk = pack8(v);
              xs[(m * K + 8 * c) >> 3] = pk;
              if (blockIdx.x == 0) *reinterpret_cast<uint4*>(nm.res_out + (size_t)m * K + 8 * c) = pk;
              unpack8(pk, v);
#pragma unroll
              for (int j = 0; j < 8; ++j) ss += v[j] * v[j];
            }
            ss = wave_sum(ss);
            if (lane == 0) red_ss[m][vw] = ss;
          }
        }
        __syncthreads();
        for (int idx = threadIdx.x; idx < MT * G; idx += 64 * WAVES) {
          const int m = idx / G, c = idx - m * G;
          float t = 0.f;
          for (int i = 0; i < nvw; ++i) t += red_ss[m][i];
          const float inv = rsqrtf(t / (float)K + nm.eps);
          float v[8], gw[8], o[8];
          unpack8(xs[idx], v);
          unpack8(reinterpret_cast<const uint4*>(nm.w)[c], gw);
#pragma unroll
          for (int j = 0; j < 8; ++j) o[j] = v[j] * inv * gw[j];
          xs[idx] = pack8(o);
        }
        __syncthreads();
      }
      GVT_DOT(k0)
    }
  }
#undef GVT_LOAD_W
#undef GVT_DOT
#pragma unroll
  for (int j = 0; j < NW; ++j)
#pragma unroll
    for (int m = 0; m < MT; ++m) {
      acc[j][m] = xor16_sum(acc[j][m]);
      acc[j][m] = xor32_sum(acc[j][m]);
    }
  if (q == 0) {
#pragma unroll
    for (int j = 0; j < NW; ++j)
#pragma unroll
      for (int m = 0; m < MT; ++m) red[w][(j * MT + m) * 16 + lane] = acc[j][m];
  }
  __syncthreads();
  const int row0 = tile * NW * 16;
  // t = (j MT + m) 16 + r  ->  row row0 + 16 j + r of batch row m
  for (int t = threadIdx.x; t < R; t += 64 * WAVES) {
    float v = red[0][t];
#pragma unroll
    for (int ww = 1; ww < WAVES; ++ww) v += red[ww][t];
    red[0][t] = v;
  }
  __syncthreads();
  if (epi == GV_SWIGLU) {
    for (int t = threadIdx.x; t < R / 2; t += 64 * WAVES) {
      const int r = t & 7, jm = t >> 3, j = jm / MT, m = jm - j * MT;
      const float gg = bf2f(f2bf(red[0][jm * 16 + r])), uu = bf2f(f2bf(red[0][jm * 16 + 8 + r]));
      yb[(size_t)m * ldo + 8 * (tile * NW + j) + r] = f2bf(gg / (1.f + __expf(-gg)) * uu);
    }
  } else {
    for (int t = threadIdx.x; t < R; t += 64 * WAVES) {
      const int r = t & 15, jm = t >> 4, j = jm / MT, m = jm - j * MT;
      const int row = row0 + 16 * j + r;
      if (epi == GV_BF16) yb[(size_t)m * ldo + row] = f2bf(red[0][t]);
      else yf[((size_t)s * MT + m) * N + row] = red[0][t];
    }
  }
}
}  // namespace

// mode 0: out[M, N] bf16 = sum of partials; mode 1: out[M, N/2] = silu(gate) * up (interleaved).
CFC_API int cfc_splitk_reduce(const float* part, int split, int M, int N, int mode, void* out, int ldo,
                              hipStream_t stream) {
  if (N % 4 || M <= 0 || (mode == 1 && N % 16)) return -1;
  const int cols = mode == 0 ? N : N / 2;
  dim3 grid((cols / 4 + 255) / 256, M);
  splitk_reduce_kernel<<<grid, 256, 0, stream>>>(part, split, M, N, mode, (uint16_t*)out, ldo);
  return CFC_CHECK_LAUNCH();
}

CFC_API int cfc_splitk_residual_rmsnorm(const float* part, int split, int M, int N, void* residual, const void* w,
                                        float eps, void* out, hipStream_t stream) {
  if (N % 8 || N / 8 > 1024 || M <= 0 || split <= 0) return -1;
  const int threads = ((N / 8 + 63) / 64) * 64;
#define SRR_ARGS part, split, M, N, (uint16_t*)residual, (const uint16_t*)w, eps, (uint16_t*)out
  switch (split) {
    case 1: splitk_residual_rmsnorm_kernel<1><<<M, threads, 0, stream>>>(SRR_ARGS); break;
    case 2: splitk_residual_rmsnorm_kernel<2><<<M, threads, 0, stream>>>(SRR_ARGS); break;
    case 4: splitk_residual_rmsnorm_kernel<4><<<M, threads, 0, stream>>>(SRR_ARGS); break;
    case 8: splitk_residual_rmsnorm_kernel<8><<<M, threads, 0, stream>>>(SRR_ARGS); break;
    default: splitk_residual_rmsnorm_kernel<0><<<M, threads, 0, stream>>>(SRR_ARGS); break;
  }
#undef SRR_ARGS
  return CFC_CHECK_LAUNCH();
}

// M <= 4 GEMV. epi 0: fp32 [M, N] into yf; 1: bf16 into yb (row stride ldo); 2: SwiGLU over the
// interleaved gate/up W -> bf16 [M, N/2] into yb.  N even (epi 2: N % 16 == 0), K % 8 == 0.
CFC_API int cfc_gemv(const void* x, const void* w, int M, int N, int K, int epi, float* yf, void* yb, int ldo,
                     hipStream_t stream) {
  if (M < 1 || M > 4 || N <= 0 || N % 2 || K <= 0 || K % 8) return -1;
  if (epi == GV_SWIGLU && N % 16) return -1;
  if ((epi == GV_F32 && !yf) || (epi != GV_F32 && !yb)) return -2;
  const int ncols = epi == GV_SWIGLU ? N / 2 : N / GV_RW;
  const dim3 grid((ncols + 3) / 4);
#define GV_ARGS (const uint16_t*)x, (const uint16_t*)w, N, K, yf, (uint16_t*)yb, ldo, ncols
#define GV_CASE(MT)                                                                          \
  case MT:                                                                                   \
    if (epi == GV_F32) gemv_kernel<MT, GV_F32><<<grid, 256, 0, stream>>>(GV_ARGS);           \
    else if (epi == GV_BF16) gemv_kernel<MT, GV_BF16><<<grid, 256, 0, stream>>>(GV_ARGS);    \
    else if (epi == GV_SWIGLU) gemv_kernel<MT, GV_SWIGLU><<<grid, 256, 0, stream>>>(GV_ARGS); \
    else return -3;                                                                          \
    break;
  switch (M) { GV_CASE(1) GV_CASE(2) GV_CASE(3) GV_CASE(4) }
#undef GV_CASE
#undef GV_ARGS
  return CFC_CHECK_LAUNCH();
}

namespace {
template <int NW, int MT, int WAVES, bool XN>
void gemv_tile_go(dim3 grid, hipStream_t stream, const uint16_t* x, const uint16_t* wp, int N, int K, int split, int epi,
                  float* yf, uint16_t* yb, int ldo, const GvNorm& nm) {
  const size_t lds = XN ? (size_t)MT * K * 2 : 0;
  if constexpr (XN) {
    static bool raised = false;                    // dynamic LDS past 64 KB (Llama-70B rows at M = 4)
    if (!raised) {
      hipFuncSetAttribute(reinterpret_cast<const void*>(&gemv_tile_kernel<NW, MT, WAVES, XN>),
                          hipFuncAttributeMaxDynamicSharedMemorySize, 96 * 1024);
      raised = true;
    }
  }
  gemv_tile_kernel<NW, MT, WAVES, XN><<<grid, 64 * WAVES, lds, stream>>>(x, wp, N, K, split, epi, yf, yb, ldo, nm);
}

template <int NW, int MT>
void gemv_tile_launch(dim3 grid, int waves, hipStream_t stream, const uint16_t* x, const uint16_t* wp, int N, int K,
                      int split, int epi, float* yf, uint16_t* yb, int ldo, const GvNorm& nm) {
  const bool xn = nm.part != nullptr;
#define GVT(WV)                                                                                    \
  if (xn) gemv_tile_go<NW, MT, WV, true>(grid, stream, x, wp, N, K, split, epi, yf, yb, ldo, nm);  \
  else gemv_tile_go<NW, MT, WV, false>(grid, stream, x, wp, N, K, split, epi, yf, yb, ldo, nm);
  if (waves == 4) { GVT(4) }
  else if (waves == 8) { GVT(8) }
  else if constexpr (MT == 1) { GVT(16) }         // 16 waves: 4 per SIMD, so <= 128 VGPRs -- single-row only
#undef GVT
}
}  // namespace

// M <= 4 GEMV over a fragment-packed W (cfc_dgemm_pack layout for bn = 16 nw, nw in {4, 6, 7, 8}):
// epilogues as cfc_gemv; split > 1 (fp32 only): yf = slabs [split, M, N] of the k-slice partial
// sums.  N % (16 nw) == 0, K % 32 == 0, 1 <= split <= K / 32.
CFC_API int cfc_gemv_packed(const void* x, const void* wp, int M, int N, int K, int nw, int epi, float* yf, void* yb,
                            int ldo, int split, int waves, const float* xpart, int xsplit, const void* res_in,
                            void* res_out, const void* norm_w, float eps, hipStream_t stream) {
  if (M < 1 || M > 4 || N <= 0 || nw <= 0 || N % (16 * nw) || K <= 0 || K % 32) return -1;
  if ((epi == GV_F32 && !yf) || (epi != GV_F32 && !yb) || epi < 0 || epi > 2) return -2;
  if (split < 1 || split > K / 32 || (split > 1 && epi != GV_F32)) return -4;
  if (waves != 4 && waves != 8 && !(waves == 16 && M == 1)) return -5;
  // the fused-norm prologue holds the first step's weights across the slab sums: <= 8 waves (VGPRs)
  if (xpart ? (xsplit < 1 || !res_in || !res_out || !norm_w || res_in == res_out || K > 8192 || waves > 8) : !x)
    return -6;
  const GvNorm nm{xpart, xsplit, (const uint16_t*)res_in, (uint16_t*)res_out, (const uint16_t*)norm_w, eps};
  const dim3 grid((N / (16 * nw)) * split);
#define GVP_ARGS (const uint16_t*)x, (const uint16_t*)wp, N, K, split, epi, yf, (uint16_t*)yb, ldo, nm
#define GVP_CASE(NW)                                                                         \
  case NW:                                                                                   \
    switch (M) {                                                                             \
      case 1: gemv_tile_launch<NW, 1>(grid, waves, stream, GVP_ARGS); break;                 \
      case 2: gemv_tile_launch<NW, 2>(grid, waves, stream, GVP_ARGS); break;                 \
      case 3: gemv_tile_launch<NW, 3>(grid, waves, stream, GVP_ARGS); break;                 \
      default: gemv_tile_launch<NW, 4>(grid, waves, stream, GVP_ARGS); break;                \
    }                                                                                        \
    break;
  switch (nw) {
    GVP_CASE(4) GVP_CASE(6) GVP_CASE(7) GVP_CASE(8)
    default: return -3;
  }
#undef GVP_CASE
#undef GVP_ARGS
  return CFC_CHECK_LAUNCH();
}
