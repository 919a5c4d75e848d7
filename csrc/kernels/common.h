// Shared device helpers for the gfx950 (CDNA4) kernels of copilot_for_consensus_amd.
//
// Conventions used by every kernel in this directory:
//   * bf16 tensors are passed as `const uint16_t*` / `uint16_t*` (raw bits) and converted with
//     the helpers below; vector loads go through 16-byte `uint4` (8 bf16) whenever the row
//     length allows it (guide §6 Guideline 13: scalar bf16 loads cost 2-2.5x).
//   * Wavefront = 64 lanes; block sizes are multiples of 64.
//   * Every launcher is `extern "C"` and takes an explicit hipStream_t so PyTorch's current
//     stream (and therefore hipGraph capture) is honoured.
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

#define CFC_API extern "C" __attribute__((visibility("default")))

typedef __bf16 bf16x8_t __attribute__((ext_vector_type(8)));
typedef __bf16 bf16x4_t __attribute__((ext_vector_type(4)));
typedef float f32x4_t __attribute__((ext_vector_type(4)));
typedef float f32x16_t __attribute__((ext_vector_type(16)));

__device__ __forceinline__ float bf2f(uint16_t v) { return __uint_as_float(((uint32_t)v) << 16); }

// Round-to-nearest-even f32 -> bf16 (NaN preserved by forcing a quiet NaN payload).
__device__ __forceinline__ uint16_t f2bf(float f) {
  uint32_t u = __float_as_uint(f);
  if ((u & 0x7fffffffu) > 0x7f800000u) return 0x7fc0;
  u += 0x7fffu + ((u >> 16) & 1u);
  return (uint16_t)(u >> 16);
}

__device__ __forceinline__ uint32_t pack2bf(float a, float b) {
  return (uint32_t)f2bf(a) | ((uint32_t)f2bf(b) << 16);
}

__device__ __forceinline__ void unpack8(const uint4 v, float* f) {
  f[0] = __uint_as_float(v.x << 16); f[1] = __uint_as_float(v.x & 0xffff0000u);
  f[2] = __uint_as_float(v.y << 16); f[3] = __uint_as_float(v.y & 0xffff0000u);
  f[4] = __uint_as_float(v.z << 16); f[5] = __uint_as_float(v.z & 0xffff0000u);
  f[6] = __uint_as_float(v.w << 16); f[7] = __uint_as_float(v.w & 0xffff0000u);
}

__device__ __forceinline__ uint4 pack8(const float* f) {
  uint4 r;
  r.x = pack2bf(f[0], f[1]); r.y = pack2bf(f[2], f[3]);
  r.z = pack2bf(f[4], f[5]); r.w = pack2bf(f[6], f[7]);
  return r;
}

// gfx950 lane swaps, VALU only (a __shfl_xor is an LDS-crossbar ds_bpermute: LDS issue, lgkmcnt wait):
// v_permlane32_swap trades lanes 32-63 of a with lanes 0-31 of b; v_permlane16_swap trades the odd
// 16-lane rows of a with the even rows of b.  With a = b = x every lane then holds its own value in one
// result and its lane ^ 32 (^ 16) partner's in the other, so one butterfly step of a commutative op is
// one swap + one op -- the same bits as x op __shfl_xor(x, 32 / 16).
__device__ __forceinline__ void swap32(float& a, float& b) {
  const auto r = __builtin_amdgcn_permlane32_swap(__float_as_uint(a), __float_as_uint(b), false, false);
  a = __uint_as_float(r[0]);
  b = __uint_as_float(r[1]);
}

__device__ __forceinline__ void swap16(float& a, float& b) {
  const auto r = __builtin_amdgcn_permlane16_swap(__float_as_uint(a), __float_as_uint(b), false, false);
  a = __uint_as_float(r[0]);
  b = __uint_as_float(r[1]);
}

__device__ __forceinline__ float xor32_sum(float x) { float a = x, b = x; swap32(a, b); return a + b; }
__device__ __forceinline__ float xor32_max(float x) { float a = x, b = x; swap32(a, b); return fmaxf(a, b); }
__device__ __forceinline__ float xor16_sum(float x) { float a = x, b = x; swap16(a, b); return a + b; }
__device__ __forceinline__ float xor16_max(float x) { float a = x, b = x; swap16(a, b); return fmaxf(a, b); }

__device__ __forceinline__ float wave_sum(float v) {
  v = xor32_sum(v);
  v = xor16_sum(v);
#pragma unroll
  for (int o = 8; o > 0; o >>= 1) v += __shfl_xor(v, o, 64);
  return v;
}

__device__ __forceinline__ float wave_max(float v) {
  v = xor32_max(v);
  v = xor16_max(v);
#pragma unroll
  for (int o = 8; o > 0; o >>= 1) v = fmaxf(v, __shfl_xor(v, o, 64));
  return v;
}

// Block-wide sum for blockDim.x <= 1024 (multiple of 64). `red` must hold >= 16 floats.
__device__ __forceinline__ float block_sum(float v, float* red) {
  const int lane = threadIdx.x & 63, wid = threadIdx.x >> 6, nw = blockDim.x >> 6;
  v = wave_sum(v);
  __syncthreads();
  if (lane == 0) red[wid] = v;
  __syncthreads();
  float t = 0.f;
  for (int i = 0; i < nw; ++i) t += red[i];
  return t;
}

// Block-wide max, same contract as block_sum.
__device__ __forceinline__ float block_max(float v, float* red) {
  const int lane = threadIdx.x & 63, wid = threadIdx.x >> 6, nw = blockDim.x >> 6;
  v = wave_max(v);
  __syncthreads();
  if (lane == 0) red[wid] = v;
  __syncthreads();
  float t = red[0];
  for (int i = 1; i < nw; ++i) t = fmaxf(t, red[i]);
  return t;
}

// XCD-aware bijective remap of a 1-D block id (guide §5 "XCD swizzle must be bijective"):
// consecutive logical tiles land on the same XCD so neighbouring tiles share that XCD's L2.
__device__ __forceinline__ int xcd_remap(int orig, int nwg) {
  const int q = nwg / 8, r = nwg % 8, xcd = orig % 8;
  return (xcd < r ? xcd * (q + 1) : r * (q + 1) + (xcd - r) * q) + orig / 8;
}

// ---------------------------------------------------------------------------------------------
// FP8 KV cache (OCP e4m3fn -- gfx950's v_cvt_pk_fp8_f32 / v_cvt_pk_f32_fp8 format, max 448; NOT
// MI300's fnuz).  Values are clamped to +-448 before conversion so the cache never holds NaN.
// fp8 -> f32 -> bf16 is exact (e4m3's 3 mantissa bits and exponent range fit bf16).
typedef __bf16 bf16x2v_t __attribute__((ext_vector_type(2)));
typedef float f32x2v_t __attribute__((ext_vector_type(2)));

__device__ __forceinline__ uint32_t cvt_pk_bf16_f32(float a, float b) {
  return __builtin_bit_cast(uint32_t, __builtin_convertvector(f32x2v_t{a, b}, bf16x2v_t));
}
__device__ __forceinline__ float fp8_clamp(float x) { return fminf(fmaxf(x, -448.f), 448.f); }
__device__ __forceinline__ uint32_t pack4_fp8(float a, float b, float c, float d) {
  const uint32_t r = __builtin_amdgcn_cvt_pk_fp8_f32(fp8_clamp(a), fp8_clamp(b), 0, false);
  return __builtin_amdgcn_cvt_pk_fp8_f32(fp8_clamp(c), fp8_clamp(d), r, true);
}
__device__ __forceinline__ uint2 pack8_fp8(const float* f) {
  return make_uint2(pack4_fp8(f[0], f[1], f[2], f[3]), pack4_fp8(f[4], f[5], f[6], f[7]));
}
__device__ __forceinline__ uint8_t f2fp8(float x) {
  return (uint8_t)(__builtin_amdgcn_cvt_pk_fp8_f32(fp8_clamp(x), 0.f, 0, false) & 0xff);
}
// 8 fp8 (in a uint2) -> 8 bf16 (bits, in a uint4), same element order
__device__ __forceinline__ uint4 fp8x8_to_bf16x8(uint2 v) {
  const auto a = __builtin_amdgcn_cvt_pk_f32_fp8(v.x, false), b = __builtin_amdgcn_cvt_pk_f32_fp8(v.x, true);
  const auto c = __builtin_amdgcn_cvt_pk_f32_fp8(v.y, false), d = __builtin_amdgcn_cvt_pk_f32_fp8(v.y, true);
  uint4 r;
  r.x = cvt_pk_bf16_f32(a[0], a[1]); r.y = cvt_pk_bf16_f32(b[0], b[1]);
  r.z = cvt_pk_bf16_f32(c[0], c[1]); r.w = cvt_pk_bf16_f32(d[0], d[1]);
  return r;
}

// ---------------------------------------------------------------------------------------------
// Decode RoPE + paged KV write, shared by rope_kv_kernel (elementwise.hip) and the decode attention
// kernel that does it in its prologue (attention.hip), so both write bit-identical caches.
// Cache layouts (attention.hip header): K [blk][kvh][32][D]; V transposed [blk][kvh][4][D][8] (slot
// position p = 8 g' + j' of row d at kv_v_off(d, p)) with key (16 hi + 4 g + j) of a block at slot
// position 8 g + 4 hi + j.
constexpr int CFC_KV_BS = 32;

__device__ __forceinline__ int kv_v_slot(int key_in_block) {
  const int hi = key_in_block >> 4, g = (key_in_block >> 2) & 3, j = (key_in_block & 3) + 4 * hi;
  return 8 * g + j;
}

// Element offset of (d, slot position p) inside one (block, kv head) V tile, stored as
// [4 slot groups][D][8 slots]: the 8 positions 8g..8g+7 of one d (one P.V MFMA fragment) are 16
// contiguous bytes, and one token's column touches D * 2 B / 128 B = 16 cache lines (bf16, D = 128)
// instead of 64 in a [D][32] tile -- the decode step's V write costs by lines dirtied
// (profiles/ROOFLINE.md, round 6).
__device__ __forceinline__ int kv_v_off(int d, int p, int D) { return (p >> 3) * (D * 8) + d * 8 + (p & 7); }

// 8 consecutive qkv values of token row element offset `off`: from the bf16 qkv, or summed from
// `split` fp32 split-K slabs of the decode GEMM (slab stride `slab` elements) and rounded to bf16
// -- the same values splitk_reduce would have written, without the round trip
// a += sum_p part[p slab + off .. + 4], b += ... [+ 4 .. + 8], p ascending: the split-K slab sum of
// one 8-column group.  Loads go out 8 slabs at a time (a plain loop waits one load latency per
// slab: 12 us for 32 slabs of a 4096-wide row in one workgroup, profiles/r04_latprof_*).
__device__ __forceinline__ void slab_sum8(const float* part, int split, size_t slab, size_t off, float4& a,
                                          float4& b) {
  for (int p0 = 0; p0 < split; p0 += 8) {
    float4 x[8], y[8];
#pragma unroll
    for (int u = 0; u < 8; ++u) {
      const size_t o = (size_t)min(p0 + u, split - 1) * slab + off;
      x[u] = *reinterpret_cast<const float4*>(part + o);
      y[u] = *reinterpret_cast<const float4*>(part + o + 4);
    }
#pragma unroll
    for (int u = 0; u < 8; ++u) {
      if (p0 + u < split) {
        a.x += x[u].x; a.y += x[u].y; a.z += x[u].z; a.w += x[u].w;
        b.x += y[u].x; b.y += y[u].y; b.z += y[u].z; b.w += y[u].w;
      }
    }
  }
}

__device__ __forceinline__ void qkv_load8(const uint16_t* qkv, const float* part, int split, size_t slab, size_t off,
                                          float* f) {
  if (part == nullptr) {
    unpack8(*reinterpret_cast<const uint4*>(qkv + off), f);
    return;
  }
  float4 a = make_float4(0.f, 0.f, 0.f, 0.f), b = a;
  slab_sum8(part, split, slab, off, a, b);
  f[0] = bf2f(f2bf(a.x)); f[1] = bf2f(f2bf(a.y)); f[2] = bf2f(f2bf(a.z)); f[3] = bf2f(f2bf(a.w));
  f[4] = bf2f(f2bf(b.x)); f[5] = bf2f(f2bf(b.y)); f[6] = bf2f(f2bf(b.z)); f[7] = bf2f(f2bf(b.w));
}

// qkv_load8 of two offsets with every load of both in flight at once (4 slabs of each per round):
// the two halves a RoPE rotation pairs no longer wait one slab round trip after the other
// (rope_kv_kernel at B = 128 decode, split 4: 11.2 us in the step).  Same sums, same order.
__device__ __forceinline__ void qkv_load8x2(const uint16_t* qkv, const float* part, int split, size_t slab,
                                            size_t off_a, size_t off_b, float* fa, float* fb) {
  if (part == nullptr) {
    const uint4 ua = *reinterpret_cast<const uint4*>(qkv + off_a), ub = *reinterpret_cast<const uint4*>(qkv + off_b);
    unpack8(ua, fa);
    unpack8(ub, fb);
    return;
  }
  float4 a0 = make_float4(0.f, 0.f, 0.f, 0.f), a1 = a0, b0 = a0, b1 = a0;
  for (int p0 = 0; p0 < split; p0 += 4) {
    float4 x[4][4];
#pragma unroll
    for (int u = 0; u < 4; ++u) {
      const size_t o = (size_t)min(p0 + u, split - 1) * slab;
      x[u][0] = *reinterpret_cast<const float4*>(part + o + off_a);
      x[u][1] = *reinterpret_cast<const float4*>(part + o + off_a + 4);
      x[u][2] = *reinterpret_cast<const float4*>(part + o + off_b);
      x[u][3] = *reinterpret_cast<const float4*>(part + o + off_b + 4);
    }
#pragma unroll
    for (int u = 0; u < 4; ++u) {
      if (p0 + u < split) {
        a0.x += x[u][0].x; a0.y += x[u][0].y; a0.z += x[u][0].z; a0.w += x[u][0].w;
        a1.x += x[u][1].x; a1.y += x[u][1].y; a1.z += x[u][1].z; a1.w += x[u][1].w;
        b0.x += x[u][2].x; b0.y += x[u][2].y; b0.z += x[u][2].z; b0.w += x[u][2].w;
        b1.x += x[u][3].x; b1.y += x[u][3].y; b1.z += x[u][3].z; b1.w += x[u][3].w;
      }
    }
  }
  const float sa[8] = {a0.x, a0.y, a0.z, a0.w, a1.x, a1.y, a1.z, a1.w};
  const float sb[8] = {b0.x, b0.y, b0.z, b0.w, b1.x, b1.y, b1.z, b1.w};
#pragma unroll
  for (int j = 0; j < 8; ++j) {
    fa[j] = bf2f(f2bf(sa[j]));
    fb[j] = bf2f(f2bf(sb[j]));
  }
}

// Rotate-half RoPE of the c-th 8-vector of each half of one head (head row at element offset
// `head_off`); cs = cos_sin + position * half * 2 (cos, sin interleaved).  pa / pb: bf16 results
// for [c*8, c*8+8) and [half + c*8, ...).
__device__ __forceinline__ void rope_rot8(const uint16_t* qkv, const float* part, int split, size_t slab,
                                          size_t head_off, int half, int c, const float* cs, uint4& pa, uint4& pb) {
  const float4* c4 = reinterpret_cast<const float4*>(cs + (size_t)c * 16);
  float csv[16];
#pragma unroll
  for (int j = 0; j < 4; ++j) {
    const float4 t = c4[j];
    csv[4 * j] = t.x; csv[4 * j + 1] = t.y; csv[4 * j + 2] = t.z; csv[4 * j + 3] = t.w;
  }
  float a[8], b[8], ra[8], rb[8];
  qkv_load8x2(qkv, part, split, slab, head_off + c * 8, head_off + half + c * 8, a, b);
#pragma unroll
  for (int j = 0; j < 8; ++j) {
    const float cv = csv[2 * j], sv = csv[2 * j + 1];
    ra[j] = a[j] * cv - b[j] * sv;
    rb[j] = b[j] * cv + a[j] * sv;
  }
  pa = pack8(ra);
  pb = pack8(rb);
}

// Roped key 8-vectors (c of each half) of kv-head kh into cache slot `slot`.  F8: e4m3 of the bf16
// value times inv_k (rounded to bf16 first: the values the bf16 cache would hold).
template <bool F8>
__device__ __forceinline__ void kv_write_k(void* k_cache, int slot, int kh, int Hkv, int D, int c, uint4 pa, uint4 pb,
                                           float inv_k) {
  const int half = D / 2, blk = slot / CFC_KV_BS, off = slot % CFC_KV_BS;
  const size_t e0 = (((size_t)blk * Hkv + kh) * CFC_KV_BS + off) * D;
  if constexpr (F8) {
    float qa[8], qb[8];
    unpack8(pa, qa);
    unpack8(pb, qb);
#pragma unroll
    for (int j = 0; j < 8; ++j) { qa[j] *= inv_k; qb[j] *= inv_k; }
    uint8_t* dst = reinterpret_cast<uint8_t*>(k_cache) + e0;
    *reinterpret_cast<uint2*>(dst + c * 8) = pack8_fp8(qa);
    *reinterpret_cast<uint2*>(dst + half + c * 8) = pack8_fp8(qb);
  } else {
    uint16_t* dst = reinterpret_cast<uint16_t*>(k_cache) + e0;
    *reinterpret_cast<uint4*>(dst + c * 8) = pa;
    *reinterpret_cast<uint4*>(dst + half + c * 8) = pb;
  }
}

// V 8-vector c (elements [8c, 8c+8)) of kv-head kh into the transposed cache at slot `slot`:
// eight 1-2 byte stores, each into a different 32-slot row (a partial cache line).  VM: 0 plain
// stores; 1 write-through (the partial lines leave L2 during the kernel instead of at its end);
// 2 nontemporal.
template <bool F8, int VM = 0>
__device__ __forceinline__ void kv_write_v(void* v_cache, int slot, int kh, int Hkv, int D, int c, uint4 val,
                                           float inv_v) {
  const int blk = slot / CFC_KV_BS, off = slot % CFC_KV_BS;
  const size_t e0 = ((size_t)blk * Hkv + kh) * D * CFC_KV_BS + kv_v_off(c * 8, kv_v_slot(off), D);
  const uint16_t* e = reinterpret_cast<const uint16_t*>(&val);
  if constexpr (F8) {
    uint8_t* dst = reinterpret_cast<uint8_t*>(v_cache) + e0;
#pragma unroll
    for (int j = 0; j < 8; ++j) {
      const uint8_t b = f2fp8(bf2f(e[j]) * inv_v);
      if constexpr (VM == 1) __hip_atomic_store(dst + j * 8, b, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      else if constexpr (VM == 2) __builtin_nontemporal_store(b, dst + j * 8);
      else dst[j * 8] = b;
    }
  } else {
    uint16_t* dst = reinterpret_cast<uint16_t*>(v_cache) + e0;
#pragma unroll
    for (int j = 0; j < 8; ++j) {
      const uint16_t h = e[j];
      if constexpr (VM == 1) __hip_atomic_store(dst + j * 8, h, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      else if constexpr (VM == 2) __builtin_nontemporal_store(h, dst + j * 8);
      else dst[j * 8] = h;
    }
  }
}

#define CFC_CHECK_LAUNCH() (int)hipGetLastError()
