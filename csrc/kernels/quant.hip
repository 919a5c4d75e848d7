// ggml block-quantized weights on gfx950: dequantization to bf16 (checkpoint loading) and the
// weight-only quantized GEMV that runs single-stream / small-batch decode straight from the
// quantized blocks (the reference's summarizer is a Q4_K_M GGUF served by llama.cpp,
// docker-compose.infra.yml:296-298; runtime/gguf.py reads the file).
//
// GPU layouts (repacked on the host, ops/kernels.py:_planar): planar, every plane row-major
// [N, ...], so the 16-B loads of one wave instruction are contiguous (the ggml 144 / 210-byte
// blocks interleave headers with quants, which halved the streaming rate -- measured).  Within
// a 32-weight chunk c the nibble plane holds byte i = q[32c + i] | q[32c + 16 + i] << 4.
//   Q4_K: NIB [N][K/2], HDR [N][K/256][16] (ggml fp16 d, fp16 dmin, 12 bytes of 6-bit scales/mins)
//   Q6_K: NIB [N][K/2] (low 4 bits), HI [N][K/4] (chunk c: dword h, byte b, bits 2f..2f+1 = top
//         2 bits of weight 16h + 4f + b), SC [N][K/16] int8, D [N][K/256] fp16
//   Q8_0: Q [N][K] int8, D [N][K/32] fp16
//
// Quantized GEMV, M <= 4 rows of bf16 X (decode): a projection at M <= 4 is a pure weight stream
// and the quantized weights are 3.6x (Q4_K) / 2.4x (Q6_K) fewer bytes than bf16.  One wave owns
// two output rows (for SwiGLU: gate row j and up row j) and walks K in 32-weight units, 8 units
// per 256-weight block, all units of the row issued before any arithmetic (whole rows in flight).
// The arithmetic stays in bf16 x fp32 (no int8 activation quantization, unlike llama.cpp's mmvq):
// nibbles become bf16 values 128 + q by ONE v_perm_b32 each pair (byte q under exponent byte 0x43),
// v_dot2c_f32_bf16 accumulates (128 + q) . x, and the 128 . sum(x) offset, the block scale and
// the min are applied once per 16-32 weights:
//     sum_i (d sc q_i - dmin m) x_i = d sc (S - 128 X) - dmin m X,  S = sum (128 + q_i) x_i, X = sum x_i.
#include <algorithm>

#include "common.h"

namespace {

enum { QT_Q4K = 12, QT_Q6K = 14, QT_Q8_0 = 8 };
enum { QE_F32 = 0, QE_BF16 = 1, QE_SWIGLU = 2 };
constexpr int Q6K_GPU_BYTES = 224;

typedef __bf16 bf16x2_t __attribute__((ext_vector_type(2)));
typedef unsigned int q_u32x4 __attribute__((ext_vector_type(4)));

__device__ __forceinline__ uint4 q_stream(const void* p) {   // once-read weights: nontemporal
  const q_u32x4 v = __builtin_nontemporal_load(reinterpret_cast<const q_u32x4*>(p));
  return make_uint4(v.x, v.y, v.z, v.w);
}
__device__ __forceinline__ float h2f(uint16_t h) { return (float)__builtin_bit_cast(_Float16, h); }
__device__ __forceinline__ float dot2(uint32_t a, uint32_t b, float c) {
  return __builtin_amdgcn_fdot2_f32_bf16(__builtin_bit_cast(bf16x2_t, a), __builtin_bit_cast(bf16x2_t, b), c, false);
}
// bytes q0..q3 of w (each < 128) -> bf16 pairs (128 + q0, 128 + q1) and (128 + q2, 128 + q3)
__device__ __forceinline__ uint32_t pair_lo(uint32_t w) { return __builtin_amdgcn_perm(0x43434343u, w, 0x04010400u); }
__device__ __forceinline__ uint32_t pair_hi(uint32_t w) { return __builtin_amdgcn_perm(0x43434343u, w, 0x04030402u); }
constexpr uint32_t BF16_ONES = 0x3F803F80u;

__device__ __forceinline__ uint32_t byte_of(uint32_t v, int k) { return (v >> (8 * k)) & 0xffu; }

// get_scale_min_k4 on the 12 scale bytes held in three dwords (s0 = bytes 0-3, s1 = 4-7, s2 = 8-11),
// j runtime: shifts, not a byte array (a runtime-indexed register array would go to scratch)
__device__ __forceinline__ void scale_min_k4r(int j, uint32_t s0, uint32_t s1, uint32_t s2, int& d, int& m) {
  if (j < 4) {
    d = byte_of(s0, j) & 63;
    m = byte_of(s1, j) & 63;
  } else {
    const int k = j - 4;
    d = (byte_of(s2, k) & 0xF) | ((byte_of(s0, k) >> 6) << 4);
    m = (byte_of(s2, k) >> 4) | ((byte_of(s1, k) >> 6) << 4);
  }
}

__device__ __forceinline__ void scale_min_k4(int j, const uint8_t* q, int& d, int& m) {
  if (j < 4) {
    d = q[j] & 63;
    m = q[j + 4] & 63;
  } else {
    d = (q[j + 4] & 0xF) | ((q[j - 4] >> 6) << 4);
    m = (q[j + 4] >> 4) | ((q[j] >> 6) << 4);
  }
}

// ------------------------------------------------------------------------------------------------
// Per-unit loads and math.  A unit is one 32-weight chunk c of a row; plane p of tensor base b
// starts at b + off[p].  x holds the chunk's 32 bf16 activations (4 x 16 B), X their two 16-run
// sums (shared by every row of the wave).
__device__ __forceinline__ void xsum32(const uint4 (&x)[4], float (&X)[2]) {
  float a = 0.f, b = 0.f;
  a = dot2(BF16_ONES, x[0].x, a); a = dot2(BF16_ONES, x[0].y, a); a = dot2(BF16_ONES, x[0].z, a);
  a = dot2(BF16_ONES, x[0].w, a); a = dot2(BF16_ONES, x[1].x, a); a = dot2(BF16_ONES, x[1].y, a);
  a = dot2(BF16_ONES, x[1].z, a); a = dot2(BF16_ONES, x[1].w, a);
  b = dot2(BF16_ONES, x[2].x, b); b = dot2(BF16_ONES, x[2].y, b); b = dot2(BF16_ONES, x[2].z, b);
  b = dot2(BF16_ONES, x[2].w, b); b = dot2(BF16_ONES, x[3].x, b); b = dot2(BF16_ONES, x[3].y, b);
  b = dot2(BF16_ONES, x[3].z, b); b = dot2(BF16_ONES, x[3].w, b);
  X[0] = a;
  X[1] = b;
}

// S over 16 weights whose 6-or-4-bit values sit one per byte in dwords q[0..3] (weights 4f + b),
// against the 16 bf16 of xa (weights 0-7) and xb (8-15)
__device__ __forceinline__ float dot16b(const uint32_t (&q)[4], uint4 xa, uint4 xb) {
  float S = 0.f;
  S = dot2(pair_lo(q[0]), xa.x, S); S = dot2(pair_hi(q[0]), xa.y, S);
  S = dot2(pair_lo(q[1]), xa.z, S); S = dot2(pair_hi(q[1]), xa.w, S);
  S = dot2(pair_lo(q[2]), xb.x, S); S = dot2(pair_hi(q[2]), xb.y, S);
  S = dot2(pair_lo(q[3]), xb.z, S); S = dot2(pair_hi(q[3]), xb.w, S);
  return S;
}

template <int K>
__device__ __forceinline__ uint32_t quad_bcast(uint32_t v) {   // lane 4q + K's value to all lanes of quad q
  return (uint32_t)__builtin_amdgcn_mov_dpp((int)v, K * 0x55, 0xF, 0xF, false);
}

template <int T>
struct Unit;

template <>
struct Unit<QT_Q4K> {
  uint4 nib, hdr;
  uint32_t hw;   // header dword (c & 3) of the chunk's block; the 8 lanes of a block hold chunks
                 // c = 8b..8b+7, so each quad holds the block's dwords 0..3 (DPP broadcast)
  __device__ __forceinline__ void load(const uint8_t* base, int row, int c, int K, const size_t* off) {
    nib = q_stream(base + (size_t)row * (K / 2) + 16 * c);
    hw = *reinterpret_cast<const uint32_t*>(base + off[0] + (size_t)row * (K / 16) + 16 * (c >> 3) + 4 * (c & 3));
  }
  __device__ __forceinline__ void gather_header() {
    hdr = make_uint4(quad_bcast<0>(hw), quad_bcast<1>(hw), quad_bcast<2>(hw), quad_bcast<3>(hw));
  }
  __device__ __forceinline__ float dot(int c, const uint4 (&x)[4], const float (&X)[2]) const {
#ifdef QG_MEMONLY   // probe build (scripts/probes/qgemv_probe.py): the loads without the arithmetic
    return __uint_as_float((nib.x ^ nib.y ^ nib.z ^ nib.w ^ hdr.x ^ hdr.w) & 0x3fffffffu) * X[0];
#endif
    int sc, mn;
    scale_min_k4r(c & 7, hdr.y, hdr.z, hdr.w, sc, mn);
    const float d = h2f((uint16_t)(hdr.x & 0xffff)) * (float)sc, m = h2f((uint16_t)(hdr.x >> 16)) * (float)mn;
    const uint32_t lo[4] = {nib.x & 0x0F0F0F0Fu, nib.y & 0x0F0F0F0Fu, nib.z & 0x0F0F0F0Fu, nib.w & 0x0F0F0F0Fu};
    const uint32_t hi[4] = {(nib.x >> 4) & 0x0F0F0F0Fu, (nib.y >> 4) & 0x0F0F0F0Fu, (nib.z >> 4) & 0x0F0F0F0Fu,
                            (nib.w >> 4) & 0x0F0F0F0Fu};
    const float S = dot16b(lo, x[0], x[1]) + dot16b(hi, x[2], x[3]);
    return d * (S - 128.f * (X[0] + X[1])) - m * (X[0] + X[1]);
  }
};

template <>
struct Unit<QT_Q6K> {
  uint4 nib;
  uint2 hi;
  uint32_t sc2, dd;
  __device__ __forceinline__ void load(const uint8_t* base, int row, int c, int K, const size_t* off) {
    nib = q_stream(base + (size_t)row * (K / 2) + 16 * c);
    hi = *reinterpret_cast<const uint2*>(base + off[0] + (size_t)row * (K / 4) + 8 * c);
    sc2 = *reinterpret_cast<const uint16_t*>(base + off[1] + (size_t)row * (K / 16) + 2 * c);
    dd = *reinterpret_cast<const uint16_t*>(base + off[2] + (size_t)row * (K / 128) + 2 * (c >> 3));
  }
  __device__ __forceinline__ void gather_header() {}
  __device__ __forceinline__ float dot(int c, const uint4 (&x)[4], const float (&X)[2]) const {
    const uint32_t n[4] = {nib.x, nib.y, nib.z, nib.w};
    uint32_t q0[4], q1[4];
#pragma unroll
    for (int f = 0; f < 4; ++f) {
      q0[f] = (n[f] & 0x0F0F0F0Fu) | (((hi.x >> (2 * f)) & 0x03030303u) << 4);
      q1[f] = ((n[f] >> 4) & 0x0F0F0F0Fu) | (((hi.y >> (2 * f)) & 0x03030303u) << 4);
    }
    const float s0 = (float)(int8_t)(sc2 & 0xff), s1 = (float)(int8_t)(sc2 >> 8);
    // q - 32 = (128 + q) - 160
    return h2f((uint16_t)dd) * (s0 * (dot16b(q0, x[0], x[1]) - 160.f * X[0]) +
                                s1 * (dot16b(q1, x[2], x[3]) - 160.f * X[1]));
  }
};

template <>
struct Unit<QT_Q8_0> {
  uint4 a, b;
  uint32_t dd;
  __device__ __forceinline__ void load(const uint8_t* base, int row, int c, int K, const size_t* off) {
    const uint8_t* q = base + (size_t)row * K + 32 * c;
    a = q_stream(q);
    b = q_stream(q + 16);
    dd = *reinterpret_cast<const uint16_t*>(base + off[0] + (size_t)row * (K / 16) + 2 * c);
  }
  __device__ __forceinline__ void gather_header() {}
  __device__ __forceinline__ float dot(int c, const uint4 (&x)[4], const float (&X)[2]) const {
    // int8 q -> u = q ^ 0x80 = q + 128 in 0..255 = 16 hi + lo: both nibbles go through the same
    // bf16 (128 + n) pairs as Q4_K, so sum q x = 16 S_hi + S_lo - (16 * 128 + 128 + 128) sum x
    const uint32_t w0[4] = {a.x ^ 0x80808080u, a.y ^ 0x80808080u, a.z ^ 0x80808080u, a.w ^ 0x80808080u};
    const uint32_t w1[4] = {b.x ^ 0x80808080u, b.y ^ 0x80808080u, b.z ^ 0x80808080u, b.w ^ 0x80808080u};
    uint32_t l0[4], h0[4], l1[4], h1[4];
#pragma unroll
    for (int f = 0; f < 4; ++f) {
      l0[f] = w0[f] & 0x0F0F0F0Fu;
      h0[f] = (w0[f] >> 4) & 0x0F0F0F0Fu;
      l1[f] = w1[f] & 0x0F0F0F0Fu;
      h1[f] = (w1[f] >> 4) & 0x0F0F0F0Fu;
    }
    // bytes of a (w0) are weights 0-15 (x[0], x[1]), of b (w1) weights 16-31 (x[2], x[3])
    const float S = 16.f * (dot16b(h0, x[0], x[1]) + dot16b(h1, x[2], x[3])) + dot16b(l0, x[0], x[1]) +
                    dot16b(l1, x[2], x[3]);
    return h2f((uint16_t)dd) * (S - 2304.f * (X[0] + X[1]));
  }
};

// X in LDS, 16-B chunks XOR-swizzled: lane l reads chunks 4l + i, i = 0..3 (one ds_read_b128 per
// i); bits 4-5 of the chunk index go into bits 0-1 so the 16 lanes of a bank group hit 16 slots.
__device__ __forceinline__ int xswz(int c) { return c ^ ((c >> 4) & 3); }

// Quantized GEMV: blocks of 4 waves; wave w owns groups of R rows (SwiGLU: R/2 gate rows + the
// matching R/2 up rows); the block stages X (M x K bf16) in LDS first, so the x reads are ds_reads
// (lgkmcnt) and the vmcnt waits only ever cover weight loads.  A lane takes UPI 32-weight chunks
// of every row of its group per stage, all loads unconditional (clamped indices: a branch around
// a load makes hipcc wait vmcnt(0) at the join).
template <int T, int MT, int EPI, int R, int UPI, int KS>
__global__ void __launch_bounds__(256) qgemv_kernel(const uint16_t* __restrict__ X, const uint8_t* __restrict__ W,
                                                    const uint8_t* __restrict__ W2, size_t o1, size_t o2, size_t o3,
                                                    int ngroups, int K, float* __restrict__ yf,
                                                    uint16_t* __restrict__ yb, int ldo) {
  using U = Unit<T>;
  extern __shared__ uint4 xs[];
  const size_t off[3] = {o1, o2, o3};
  const int tid = threadIdx.x, lane = tid & 63, w = tid >> 6;
  // KS waves share one row group and split its K range (long rows: more waves in flight)
  const int g = blockIdx.x * (4 / KS) + w / KS, kp = w % KS;
  const int cpr = K / 8, units = K / 32;
  const int ubeg = kp * (units / KS), uend = ubeg + units / KS;
  {  // X -> LDS
    const int total = MT * cpr;
    for (int c0 = 0; c0 < total; c0 += 256 * 4) {
      uint4 v[4];
#pragma unroll
      for (int i = 0; i < 4; ++i) v[i] = reinterpret_cast<const uint4*>(X)[min(c0 + i * 256 + tid, total - 1)];
#pragma unroll
      for (int i = 0; i < 4; ++i) {
        const int c = c0 + i * 256 + tid;
        xs[c < total ? (c / cpr) * cpr + xswz(c % cpr) : total] = v[i];   // surplus -> pad slot
      }
    }
  }
  __syncthreads();
  const int gc = min(g, ngroups - 1);   // idle waves of the last block stream a real group (no branch)
  constexpr int RH = EPI == QE_SWIGLU ? R / 2 : R;
  const uint8_t* base[R];
  int rowi[R];
#pragma unroll
  for (int r = 0; r < R; ++r) {
    base[r] = (EPI == QE_SWIGLU && r >= RH) ? W2 : W;
    rowi[r] = EPI == QE_SWIGLU ? gc * RH + (r % RH) : gc * R + r;
  }
  float acc[R][MT];
#pragma unroll
  for (int r = 0; r < R; ++r)
#pragma unroll
    for (int m = 0; m < MT; ++m) acc[r][m] = 0.f;
  for (int u0 = ubeg; u0 < uend; u0 += UPI * 64) {
    U wv[UPI][R];
#pragma unroll
    for (int i = 0; i < UPI; ++i)
#pragma unroll
      for (int r = 0; r < R; ++r) wv[i][r].load(base[r], rowi[r], min(u0 + i * 64 + lane, uend - 1), K, off);
#pragma unroll
    for (int i = 0; i < UPI; ++i) {
      const int u = u0 + i * 64 + lane;
      const bool live = u < uend;
      const int uc = live ? u : uend - 1;
#pragma unroll
      for (int r = 0; r < R; ++r) wv[i][r].gather_header();
#pragma unroll
      for (int m = 0; m < MT; ++m) {
        uint4 x[4];
#pragma unroll
        for (int q = 0; q < 4; ++q) x[q] = xs[m * cpr + xswz(4 * uc + q)];
        float xsm[2];
        xsum32(x, xsm);
#pragma unroll
        for (int r = 0; r < R; ++r) {
          const float v = wv[i][r].dot(uc, x, xsm);
          acc[r][m] += live ? v : 0.f;
        }
      }
    }
  }
#pragma unroll
  for (int r = 0; r < R; ++r)
#pragma unroll
    for (int m = 0; m < MT; ++m) acc[r][m] = wave_sum(acc[r][m]);
  if constexpr (KS > 1) {   // the K parts meet in LDS (after the X image: all waves are past it)
    __syncthreads();
    float* red = reinterpret_cast<float*>(xs);
    if (lane == 0) {
#pragma unroll
      for (int r = 0; r < R; ++r)
#pragma unroll
        for (int m = 0; m < MT; ++m) red[(w * R + r) * MT + m] = acc[r][m];
    }
    __syncthreads();
    if (kp != 0) return;
#pragma unroll
    for (int r = 0; r < R; ++r)
#pragma unroll
      for (int m = 0; m < MT; ++m) {
        float v = 0.f;
#pragma unroll
        for (int k = 0; k < KS; ++k) v += red[((w + k) * R + r) * MT + m];
        acc[r][m] = v;
      }
  }
  if (lane != 0 || g >= ngroups) return;
#pragma unroll
  for (int m = 0; m < MT; ++m) {
    if constexpr (EPI == QE_SWIGLU) {
#pragma unroll
      for (int r = 0; r < RH; ++r) {
        const float gt = bf2f(f2bf(acc[r][m])), up = bf2f(f2bf(acc[r + RH][m]));   // bf16 projections, as unfused
        yb[(size_t)m * ldo + g * RH + r] = f2bf(gt / (1.f + __expf(-gt)) * up);
      }
    } else {
#pragma unroll
      for (int r = 0; r < R; r += 2) {
        if constexpr (EPI == QE_BF16)
          *reinterpret_cast<uint32_t*>(yb + (size_t)m * ldo + g * R + r) = pack2bf(acc[r][m], acc[r + 1][m]);
        else
          *reinterpret_cast<float2*>(yf + (size_t)m * ldo + g * R + r) = make_float2(acc[r][m], acc[r + 1][m]);
      }
    }
  }
}

// ------------------------------------------------------------------------------------------------
// Dequantization of RAW ggml blocks (as stored in the file, any alignment) to bf16: one thread
// per output weight (load-time only; byte loads, L1/L2 absorb the re-reads of block headers).
__device__ __forceinline__ uint16_t ld16(const uint8_t* p) { return (uint16_t)(p[0] | (p[1] << 8)); }

__global__ void dequant_kernel(const uint8_t* __restrict__ raw, int type, long long n, uint16_t* __restrict__ out) {
  const long long i = (long long)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n) return;
  float v = 0.f;
  switch (type) {
    case 0: v = reinterpret_cast<const float*>(raw)[i]; break;                         // F32
    case 1: v = h2f(ld16(raw + 2 * i)); break;                                          // F16
    case 30: out[i] = ld16(raw + 2 * i); return;                                        // BF16
    case 8: {                                                                           // Q8_0
      const uint8_t* b = raw + (i >> 5) * 34;
      v = h2f(ld16(b)) * (float)(int8_t)b[2 + (i & 31)];
      break;
    }
    case 2: {                                                                           // Q4_0
      const uint8_t* b = raw + (i >> 5) * 18;
      const int j = i & 31;
      const int q = j < 16 ? (b[2 + j] & 0xF) : (b[2 + j - 16] >> 4);
      v = h2f(ld16(b)) * (float)(q - 8);
      break;
    }
    case 3: {                                                                           // Q4_1
      const uint8_t* b = raw + (i >> 5) * 20;
      const int j = i & 31;
      const int q = j < 16 ? (b[4 + j] & 0xF) : (b[4 + j - 16] >> 4);
      v = h2f(ld16(b)) * (float)q + h2f(ld16(b + 2));
      break;
    }
    case 6:
    case 7: {                                                                           // Q5_0 / Q5_1
      const int size = type == 6 ? 22 : 24, o = type == 6 ? 2 : 4;
      const uint8_t* b = raw + (i >> 5) * size;
      const uint32_t qh = b[o] | (b[o + 1] << 8) | (b[o + 2] << 16) | ((uint32_t)b[o + 3] << 24);
      const int j = i & 31;
      const int q = j < 16 ? ((b[o + 4 + j] & 0xF) | (((qh >> j) << 4) & 0x10))
                           : ((b[o + 4 + j - 16] >> 4) | ((qh >> (j - 16 + 12)) & 0x10));
      v = type == 6 ? h2f(ld16(b)) * (float)(q - 16) : h2f(ld16(b)) * (float)q + h2f(ld16(b + 2));
      break;
    }
    case 12:
    case 13: {                                                                          // Q4_K / Q5_K
      const int size = type == 12 ? 144 : 176;
      const uint8_t* b = raw + (i >> 8) * size;
      const int w = i & 255, j = w >> 6, hi = (w >> 5) & 1, l = w & 31;
      int s, m;
      scale_min_k4(2 * j + hi, b + 4, s, m);
      const uint8_t* qs = b + (type == 12 ? 16 : 48) + 32 * j;
      int q = hi ? (qs[l] >> 4) : (qs[l] & 0xF);
      if (type == 13) q += ((b[16 + l] >> (2 * j + hi)) & 1) << 4;
      v = h2f(ld16(b)) * (float)s * (float)q - h2f(ld16(b + 2)) * (float)m;
      break;
    }
    case 14: {                                                                          // Q6_K
      const uint8_t* b = raw + (i >> 8) * 210;
      const int w = i & 255, hh = w >> 7, k = (w >> 5) & 3, l = w & 31;
      const uint8_t L = b[64 * hh + (k & 1) * 32 + l];
      const int low = (k < 2 ? L : (L >> 4)) & 0xF;
      const int q = (low | (((b[128 + 32 * hh + l] >> (2 * k)) & 3) << 4)) - 32;
      v = h2f(ld16(b + 208)) * (float)(int8_t)b[192 + 8 * hh + 2 * k + (l >> 4)] * (float)q;
      break;
    }
    default: v = __int_as_float(0x7fc00000); break;
  }
  out[i] = f2bf(v);
}

int g_qg_rows = 0, g_qg_ks = 0;   // probe overrides (cfc_qgemv_config); 0 = automatic

template <int T, int EPI, int MT, int R, int KS>
int qgemv_launch_rk(const uint16_t* x, const uint8_t* w, const uint8_t* w2, const size_t* off, int N, int K,
                    float* yf, uint16_t* yb, int ldo, hipStream_t st) {
  const int rows = EPI == QE_SWIGLU ? 2 * N : N;
  if (rows % R || (K / 32) % KS) return -1;
  const int ngroups = rows / R;
  const size_t lds = (size_t)MT * K * 2 + 16;   // + the pad slot surplus X writes land in
  if (lds > 160 * 1024 || (KS > 1 && lds < 4 * R * MT * sizeof(float))) return -5;
  constexpr int GPB = 4 / KS;                  // row groups per block
  qgemv_kernel<T, MT, EPI, R, (MT == 1 ? 2 : 1), KS><<<(ngroups + GPB - 1) / GPB, 256, lds, st>>>(
      x, w, w2, off[0], off[1], off[2], ngroups, K, yf, yb, ldo);
  return CFC_CHECK_LAUNCH();
}

template <int T, int EPI, int MT>
int qgemv_launch(const uint16_t* x, const uint8_t* w, const uint8_t* w2, const size_t* off, int N, int K, float* yf,
                 uint16_t* yb, int ldo, hipStream_t st) {
  // measured on MI355X (scripts/probes/qgemv_probe.py, profiles/qgemv_probe_r02.jsonl): long rows
  // (down: K = 14336) split K over 2 waves, so the few row groups still put enough waves (and
  // bytes) in flight; short-K shapes with few rows (q, k, v, o) take 2 rows per wave (twice the
  // waves); the wide ones (gate/up, lm_head) 4
  const int ks = g_qg_ks ? g_qg_ks : (K >= 8192 ? 2 : 1);
  const int r = g_qg_rows ? g_qg_rows : ((K < 8192 && (EPI == QE_SWIGLU ? 2 * N : N) <= 8192) ? 2 : 4);
  if constexpr (MT == 1) {
    if (r == 2) {
      if (ks == 4) return qgemv_launch_rk<T, EPI, MT, 2, 4>(x, w, w2, off, N, K, yf, yb, ldo, st);
      if (ks == 2) return qgemv_launch_rk<T, EPI, MT, 2, 2>(x, w, w2, off, N, K, yf, yb, ldo, st);
      return qgemv_launch_rk<T, EPI, MT, 2, 1>(x, w, w2, off, N, K, yf, yb, ldo, st);
    }
    if (ks == 2) return qgemv_launch_rk<T, EPI, MT, 4, 2>(x, w, w2, off, N, K, yf, yb, ldo, st);
  }
  if (ks == 4) return qgemv_launch_rk<T, EPI, MT, 4, 4>(x, w, w2, off, N, K, yf, yb, ldo, st);
  return qgemv_launch_rk<T, EPI, MT, 4, 1>(x, w, w2, off, N, K, yf, yb, ldo, st);
}

template <int T, int EPI>
int qgemv_dispatch(int M, const uint16_t* x, const uint8_t* w, const uint8_t* w2, const size_t* off, int N, int K,
                   float* yf, uint16_t* yb, int ldo, hipStream_t st) {
  switch (M) {
    case 1: return qgemv_launch<T, EPI, 1>(x, w, w2, off, N, K, yf, yb, ldo, st);
    case 2: return qgemv_launch<T, EPI, 2>(x, w, w2, off, N, K, yf, yb, ldo, st);
    case 3: return qgemv_launch<T, EPI, 3>(x, w, w2, off, N, K, yf, yb, ldo, st);
    case 4: return qgemv_launch<T, EPI, 4>(x, w, w2, off, N, K, yf, yb, ldo, st);
    default: return -1;
  }
}

template <int T>
int qgemv_epi(int epi, int M, const uint16_t* x, const uint8_t* w, const uint8_t* w2, const size_t* off, int N, int K,
              float* yf, uint16_t* yb, int ldo, hipStream_t st) {
  switch (epi) {
    case QE_F32: return qgemv_dispatch<T, QE_F32>(M, x, w, w2, off, N, K, yf, yb, ldo, st);
    case QE_BF16: return qgemv_dispatch<T, QE_BF16>(M, x, w, w2, off, N, K, yf, yb, ldo, st);
    case QE_SWIGLU: return qgemv_dispatch<T, QE_SWIGLU>(M, x, w, w2, off, N, K, yf, yb, ldo, st);
    default: return -3;
  }
}

}  // namespace

// Y[M, N] = X[M, K] . W^T for ggml-quantized W in the planar GPU layouts above, 1 <= M <= 4.
//   w: the tensor's buffer (plane 0 at w, planes 1..3 at w + o1 / o2 / o3), type 12 / 14 / 8
//   (Q4_K / Q6_K / Q8_0); epi 0: fp32 into yf; 1: bf16 into yb; 2: SwiGLU -- w gate, w2 up (same
//   shape and plane offsets), out[M][N] = silu(gate) * up into yb.  ldo = output row stride.
CFC_API int cfc_qgemv(const void* x, int M, int N, int K, int type, const void* w, const void* w2, long long o1,
                      long long o2, long long o3, int epi, float* yf, void* yb, int ldo, hipStream_t stream) {
  if (M < 1 || M > 4 || N <= 0 || K <= 0 || K % 256 || !w) return -1;
  if (epi == QE_SWIGLU && (!w2 || !yb)) return -2;
  if ((epi == QE_F32 && !yf) || (epi != QE_F32 && !yb)) return -2;
  const size_t off[3] = {(size_t)o1, (size_t)o2, (size_t)o3};
  const auto* xp = (const uint16_t*)x;
  const auto *wp = (const uint8_t*)w, *w2p = (const uint8_t*)w2;
  auto* ybp = (uint16_t*)yb;
  switch (type) {
    case QT_Q4K: return qgemv_epi<QT_Q4K>(epi, M, xp, wp, w2p, off, N, K, yf, ybp, ldo, stream);
    case QT_Q6K: return qgemv_epi<QT_Q6K>(epi, M, xp, wp, w2p, off, N, K, yf, ybp, ldo, stream);
    case QT_Q8_0: return qgemv_epi<QT_Q8_0>(epi, M, xp, wp, w2p, off, N, K, yf, ybp, ldo, stream);
    default: return -4;
  }
}

// probe hook: rows per wave (2 / 4) and K split (1 / 2 / 4) of the quantized GEMV; 0 = automatic
CFC_API void cfc_qgemv_config(int rows, int ks) {
  g_qg_rows = rows;
  g_qg_ks = ks;
}

// raw ggml blocks (file layout) -> bf16[n]
CFC_API int cfc_dequant_bf16(const void* raw, int type, long long n, void* out, hipStream_t stream) {
  if (n <= 0) return -1;
  switch (type) {
    case 0: case 1: case 2: case 3: case 6: case 7: case 8: case 12: case 13: case 14: case 30: break;
    default: return -4;
  }
  const long long blocks = (n + 255) / 256;
  dequant_kernel<<<(unsigned)blocks, 256, 0, stream>>>((const uint8_t*)raw, type, n, (uint16_t*)out);
  return CFC_CHECK_LAUNCH();
}
