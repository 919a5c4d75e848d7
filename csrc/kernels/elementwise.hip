// Memory-bound fused elementwise kernels for the decoder/encoder hot path:
//   * RoPE (rotate-half, host-precomputed cos/sin table) fused with the paged KV-cache write
//   * SwiGLU activation (silu(gate) * up) on the fused gate|up projection output
//   * bias + GELU (erf) for the BERT FFN
//   * token-embedding gather
//   * greedy argmax / Gumbel-max temperature sampling + on-device decode-state advance, so a
//     whole decode step (and the EOS/stop check) replays from a hipGraph with no
//     host synchronisation.
// All loads/stores are 16-byte vectors (guide §6 Guideline 13).
#include "common.h"

namespace {

constexpr int KV_BS = CFC_KV_BS;

__device__ __forceinline__ int v_slot(int key_in_block) { return kv_v_slot(key_in_block); }

// qkv: [T, (Hq + 2*Hkv) * D] (q heads | k heads | v heads), positions [T], slots [T] (-1 = skip
// cache write), cos_sin [max_pos][D/2][2] fp32 (cos, sin interleaved); the per-item math lives in
// common.h (rope_rot8 / kv_write_k / kv_write_v), shared with the fused decode attention.
template <bool F8, int VM = 0>
__global__ void __launch_bounds__(64) rope_kv_kernel(const uint16_t* __restrict__ qkv, const int32_t* __restrict__ positions,
                                                     const int32_t* __restrict__ slots, const float* __restrict__ cos_sin,
                                                     uint16_t* __restrict__ q_out, void* __restrict__ k_cache,
                                                     void* __restrict__ v_cache, int Hq, int Hkv, int D,
                                                     int write_v, float inv_k, float inv_v,
                                                     const float* __restrict__ part = nullptr, int split = 0) {
  // grid = (T, ceil(items / 64)): one 8-element item per thread -- (Hq + Hkv) * D/16 rotation
  // items then Hkv * D/8 V items -- so a decode batch of 128 tokens is ~900 blocks, not 128.
  // write_v = 0: V goes through v_cache_runs_kernel instead (prefill: whole blocks, 16-B stores).
  // F8: the caches hold e4m3 of value * inv_k / inv_v (the attention kernels scale back).
  const int tok = blockIdx.x;
  const int half = D / 2, nv = half / 8;  // 8-element vectors per half-head
  const int n_rot = (Hq + Hkv) * nv;
  const int n_v = write_v ? Hkv * (D / 8) : 0;
  const int it = blockIdx.y * 64 + threadIdx.x;
  if (it >= n_rot + n_v) return;
  const int stride = (Hq + 2 * Hkv) * D;
  const size_t row0 = (size_t)tok * stride, slab = (size_t)gridDim.x * stride;
  const int slot = slots[tok];
  if (it < n_rot) {
    const int head = it / nv, c = it - head * nv;  // head < Hq: query, else key (head - Hq)
    uint4 pa, pb;
    rope_rot8(qkv, part, split, slab, row0 + (size_t)head * D, half, c,
              cos_sin + (size_t)positions[tok] * half * 2, pa, pb);
    if (head < Hq) {
      uint16_t* dst = q_out + ((size_t)tok * Hq + head) * D;
      *reinterpret_cast<uint4*>(dst + c * 8) = pa;
      *reinterpret_cast<uint4*>(dst + half + c * 8) = pb;
    } else if (slot >= 0) {
      kv_write_k<F8>(k_cache, slot, head - Hq, Hkv, D, c, pa, pb, inv_k);
    }
  } else if (slot >= 0) {
    const int v = it - n_rot;
    const int kh = v / (D / 8), c = v % (D / 8);
    float vf[8];
    qkv_load8(qkv, part, split, slab, row0 + (size_t)(Hq + Hkv + kh) * D + c * 8, vf);
    kv_write_v<F8, VM>(v_cache, slot, kh, Hkv, D, c, pack8(vf), inv_v);
  }
}

// Prefill V-cache writer.  One workgroup per (run, kv-head); a run = consecutive tokens that land
// in ONE cache block at consecutive offsets (runs[r] = {first token, count, block, first offset},
// built on the host from the slots).  The run's V rows are staged in LDS and written out as the
// block's transposed, slot-permuted image: a full run (32 tokens) as 16-byte stores of whole
// 8-slot chunks, a partial run (chunk edges, prefix-cache continuations) per element so the
// block's other slots are left untouched.  Replaces the 2-byte scattered stores of the per-token
// path (1.85 TB/s effective for rope_kv at a prefill chunk, profiles/elementwise_bw_probe_r01.log).
template <bool F8>
__global__ void __launch_bounds__(256) v_cache_runs_kernel(const uint16_t* __restrict__ qkv,
                                                           const int32_t* __restrict__ runs,
                                                           void* __restrict__ v_cache, int Hq, int Hkv, int D,
                                                           float inv_v) {
  __shared__ __attribute__((aligned(16))) uint16_t sv[KV_BS][256 + 8];
  const int r = blockIdx.x, kh = blockIdx.y, tid = threadIdx.x;
  const int t0 = runs[4 * r], n = runs[4 * r + 1], blk = runs[4 * r + 2], off0 = runs[4 * r + 3];
  const int nc = D / 8;
  const size_t stride = (size_t)(Hq + 2 * Hkv) * D;
  for (int i = tid; i < n * nc; i += 256) {
    const int j = i / nc, c = i - j * nc;
    *reinterpret_cast<uint4*>(&sv[off0 + j][c * 8]) =
        *reinterpret_cast<const uint4*>(qkv + (size_t)(t0 + j) * stride + (size_t)(Hq + Hkv + kh) * D + c * 8);
  }
  __syncthreads();
  const size_t e0 = ((size_t)blk * Hkv + kh) * D * KV_BS;   // [4][D][8 slots] (common.h kv_v_off)
  if (n == KV_BS) {
    for (int i = tid; i < D * 4; i += 256) {
      const int d = i >> 2, g = i & 3;
      uint16_t e[8];
#pragma unroll
      for (int j = 0; j < 8; ++j) e[j] = sv[16 * (j >> 2) + 4 * g + (j & 3)][d];   // key held by slot 8g + j
      if constexpr (F8) {
        float f[8];
#pragma unroll
        for (int j = 0; j < 8; ++j) f[j] = bf2f(e[j]) * inv_v;
        *reinterpret_cast<uint2*>(reinterpret_cast<uint8_t*>(v_cache) + e0 + kv_v_off(d, 8 * g, D)) = pack8_fp8(f);
      } else {
        uint4 v;
        v.x = e[0] | ((uint32_t)e[1] << 16); v.y = e[2] | ((uint32_t)e[3] << 16);
        v.z = e[4] | ((uint32_t)e[5] << 16); v.w = e[6] | ((uint32_t)e[7] << 16);
        *reinterpret_cast<uint4*>(reinterpret_cast<uint16_t*>(v_cache) + e0 + kv_v_off(d, 8 * g, D)) = v;
      }
    }
  } else {
    for (int i = tid; i < n * D; i += 256) {
      const int j = i / D, d = i - j * D, off = off0 + j;
      if constexpr (F8)
        reinterpret_cast<uint8_t*>(v_cache)[e0 + kv_v_off(d, v_slot(off), D)] = f2fp8(bf2f(sv[off][d]) * inv_v);
      else
        reinterpret_cast<uint16_t*>(v_cache)[e0 + kv_v_off(d, v_slot(off), D)] = sv[off][d];
    }
  }
}

// out[t, f] = silu(gate[t, f]) * up[t, f].  Layout of gu[t]: [gate | up] halves, or (interleave)
// 8-column groups [gate 8t..8t+7 | up 8t..8t+7] -- the layout the decode GEMM's fused
// SwiGLU epilogue needs, so prefill and decode share one weight copy.  grid = (cols/8/256, T).
__global__ void silu_mul_kernel(uint16_t* __restrict__ out, const uint16_t* __restrict__ gu, int F, int interleave) {
  const int t = blockIdx.y;
  const int c = blockIdx.x * blockDim.x + threadIdx.x;   // 8-column group of the output
  if (c >= (F >> 3)) return;
  const int gc = interleave ? 2 * c : c;          // 8-row gate/up groups: chunk 2c gate, 2c+1 up
  const int uc = interleave ? 2 * c + 1 : c + (F >> 3);
  const uint4* row = reinterpret_cast<const uint4*>(gu + (size_t)t * 2 * F);
  float a[8], b[8], r[8];
  unpack8(row[gc], a);
  unpack8(row[uc], b);
#pragma unroll
  for (int j = 0; j < 8; ++j) r[j] = a[j] / (1.f + __expf(-a[j])) * b[j];
  reinterpret_cast<uint4*>(out + (size_t)t * F)[c] = pack8(r);
}

// SwiGLU fused with the per-row FP8 quantisation of its output (the down projection's input in
// W8A8 mode): one 1024-thread workgroup per row, the row's products held in registers between
// the amax reduction and the e4m3 conversion.  Values are rounded to bf16 first, so the result
// equals silu_mul -> quant_fp8_rows bit for bit.  F <= 1024 * 8 * SQ_MAX_VEC.
constexpr int SQ_MAX_VEC = 4;
__global__ void __launch_bounds__(1024) silu_mul_fp8_kernel(uint8_t* __restrict__ out, float* __restrict__ scale,
                                                           const uint16_t* __restrict__ gu, int F, int interleave) {
  __shared__ float red[16];
  const int t = blockIdx.x;
  const uint4* row = reinterpret_cast<const uint4*>(gu + (size_t)t * 2 * F);
  float r[SQ_MAX_VEC][8];
  float amax = 0.f;
#pragma unroll
  for (int i = 0; i < SQ_MAX_VEC; ++i) {
    const int c = threadIdx.x + i * 1024;
    if (c < (F >> 3)) {
      const int gc = interleave ? 2 * c : c;
      const int uc = interleave ? 2 * c + 1 : c + (F >> 3);
      float a[8], b[8];
      unpack8(row[gc], a);
      unpack8(row[uc], b);
#pragma unroll
      for (int j = 0; j < 8; ++j) {
        r[i][j] = bf2f(f2bf(a[j] / (1.f + __expf(-a[j])) * b[j]));
        amax = fmaxf(amax, fabsf(r[i][j]));
      }
    }
  }
  amax = block_max(amax, red);
  const float s = amax > 0.f ? amax / 448.f : 1.f, rs = 1.f / s;
  if (threadIdx.x == 0) scale[t] = s;
  uint2* orow = reinterpret_cast<uint2*>(out + (size_t)t * F);
#pragma unroll
  for (int i = 0; i < SQ_MAX_VEC; ++i) {
    const int c = threadIdx.x + i * 1024;
    if (c < (F >> 3)) {
#pragma unroll
      for (int j = 0; j < 8; ++j) r[i][j] *= rs;
      orow[c] = pack8_fp8(r[i]);
    }
  }
}

// Per-row (per-token) FP8 quantisation for the W8A8 linear path: scale[r] = max|x[r,:]| / 448,
// out[r,:] = e4m3fn(x[r,:] / scale[r]) (OCP e4m3 via gfx950's v_cvt_pk_fp8_f32, saturating).
// One 256-thread workgroup per row; the row stays in registers between the amax pass and the
// conversion (K <= 256 * 8 * QR_MAX_VEC), so it is read from HBM once.
constexpr int QR_MAX_VEC = 16;   // up to 32768 columns
__global__ void __launch_bounds__(256) quant_fp8_rows_kernel(const uint16_t* __restrict__ x, uint8_t* __restrict__ out,
                                                            float* __restrict__ scale, int K) {
  const int r = blockIdx.x, t = threadIdx.x;
  const int nvec = K >> 3;
  const uint4* row = reinterpret_cast<const uint4*>(x + (size_t)r * K);
  uint4 v[QR_MAX_VEC];
  float amax = 0.f;
#pragma unroll
  for (int j = 0; j < QR_MAX_VEC; ++j) {
    const int c = t + 256 * j;
    if (c < nvec) {
      v[j] = row[c];
      float f[8];
      unpack8(v[j], f);
#pragma unroll
      for (int e = 0; e < 8; ++e) amax = fmaxf(amax, fabsf(f[e]));
    }
  }
  __shared__ float red[4];
  amax = wave_max(amax);
  if ((t & 63) == 0) red[t >> 6] = amax;
  __syncthreads();
  amax = fmaxf(fmaxf(red[0], red[1]), fmaxf(red[2], red[3]));
  const float s = amax > 0.f ? amax / 448.f : 1.f;
  const float inv = 1.f / s;
  if (t == 0) scale[r] = s;
  uint2* orow = reinterpret_cast<uint2*>(out + (size_t)r * K);
#pragma unroll
  for (int j = 0; j < QR_MAX_VEC; ++j) {
    const int c = t + 256 * j;
    if (c < nvec) {
      float f[8];
      unpack8(v[j], f);
#pragma unroll
      for (int e = 0; e < 8; ++e) f[e] *= inv;
      orow[c] = pack8_fp8(f);
    }
  }
}

// out[t, f] = gelu_erf(x[t, f] + bias[f])   (in place allowed)
__global__ void bias_gelu_kernel(uint16_t* __restrict__ out, const uint16_t* __restrict__ x,
                                 const uint16_t* __restrict__ bias, int T, int F) {
  const int nvec = F / 8;
  const size_t total = (size_t)T * nvec;
  for (size_t i = blockIdx.x * (size_t)blockDim.x + threadIdx.x; i < total; i += (size_t)gridDim.x * blockDim.x) {
    const size_t c = i % nvec;
    float a[8], b[8];
    unpack8(reinterpret_cast<const uint4*>(x)[i], a);
    if (bias) unpack8(reinterpret_cast<const uint4*>(bias)[c], b);
    else {
#pragma unroll
      for (int j = 0; j < 8; ++j) b[j] = 0.f;
    }
#pragma unroll
    for (int j = 0; j < 8; ++j) {
      const float v = a[j] + b[j];
      a[j] = 0.5f * v * (1.f + erff(v * 0.70710678118654752f));
    }
    reinterpret_cast<uint4*>(out)[i] = pack8(a);
  }
}

// out[t, :] = table[ids[t], :]
__global__ void embedding_kernel(uint16_t* __restrict__ out, const uint16_t* __restrict__ table,
                                 const int32_t* __restrict__ ids, int T, int dim) {
  const int nvec = dim / 8;
  const int t = blockIdx.x;
  const uint4* src = reinterpret_cast<const uint4*>(table + (size_t)ids[t] * dim);
  uint4* dst = reinterpret_cast<uint4*>(out + (size_t)t * dim);
  for (int c = threadIdx.x; c < nvec; c += blockDim.x) dst[c] = src[c];
}

__device__ __forceinline__ uint32_t hash_u32(uint32_t x) {
  x ^= x >> 16; x *= 0x7feb352dU; x ^= x >> 15; x *= 0x846ca68bU; x ^= x >> 16;
  return x;
}

// NaN logits rank as -inf in both samplers, so an all-NaN row still yields a defined token (the
// lowest index) instead of an index that matched no comparison.
__device__ __forceinline__ float logit_nan_as_ninf(float x) { return x != x ? -INFINITY : x; }

// One workgroup per row. temperature <= 0 => greedy argmax (lowest index wins ties);
// otherwise Gumbel-max sampling: argmax(logit/T + Gumbel(seed, step, row, idx)), which draws
// exactly from softmax(logit/T).  `step` is read from device memory so graph replays advance it.
__global__ void __launch_bounds__(1024) sample_kernel(const uint16_t* __restrict__ logits, int V, float temperature,
                                                     uint32_t seed, const int32_t* __restrict__ step_ptr,
                                                     int32_t* __restrict__ out_ids) {
  const int row = blockIdx.x;
  const uint16_t* lr = logits + (size_t)row * V;
  const uint32_t step = step_ptr ? (uint32_t)*step_ptr : 0u;
  float best = -INFINITY;
  int best_i = 0x7fffffff;
  const int nvec = (V % 8 == 0) ? V / 8 : 0;  // 16-byte row alignment needed for vector loads
  const bool sample = temperature > 0.f;
  const float inv_t = sample ? 1.f / temperature : 1.f;
  auto score = [&](float x, int idx) -> float {
    x = logit_nan_as_ninf(x);
    if (!sample) return x;
    const uint32_t h = hash_u32(seed ^ hash_u32(step * 0x9E3779B9u ^ hash_u32(row * 0x85EBCA6Bu ^ (uint32_t)idx)));
    const float u = ((h >> 8) + 0.5f) * (1.f / 16777216.f);
    return x * inv_t - __logf(-__logf(u));
  };
  // 1024 threads x 4 independent 16-B loads in flight: a 32k-vocab row is one memory round trip
  // (the previous 256-thread loop was 16 dependent ones: 16 us per decode step at B = 1)
  for (int c0 = threadIdx.x; c0 < nvec; c0 += 4 * blockDim.x) {
    uint4 raw[4];
#pragma unroll
    for (int u = 0; u < 4; ++u) {
      const int c = c0 + u * blockDim.x;
      raw[u] = c < nvec ? reinterpret_cast<const uint4*>(lr)[c] : make_uint4(0, 0, 0, 0);
    }
#pragma unroll
    for (int u = 0; u < 4; ++u) {
      const int c = c0 + u * blockDim.x;
      if (c >= nvec) break;
      float v[8];
      unpack8(raw[u], v);
#pragma unroll
      for (int j = 0; j < 8; ++j) {
        const int idx = c * 8 + j;
        const float x = score(v[j], idx);
        if (x > best || (x == best && idx < best_i)) { best = x; best_i = idx; }
      }
    }
  }
  for (int idx = nvec * 8 + threadIdx.x; idx < V; idx += blockDim.x) {  // tail (V % 8)
    const float x = score(bf2f(lr[idx]), idx);
    if (x > best || (x == best && idx < best_i)) { best = x; best_i = idx; }
  }
  __shared__ float sb[16];
  __shared__ int si[16];
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) {
    const float ob = __shfl_xor(best, o, 64);
    const int oi = __shfl_xor(best_i, o, 64);
    if (ob > best || (ob == best && oi < best_i)) { best = ob; best_i = oi; }
  }
  const int lane = threadIdx.x & 63, wid = threadIdx.x >> 6;
  if (lane == 0) { sb[wid] = best; si[wid] = best_i; }
  __syncthreads();
  if (threadIdx.x == 0) {
    for (int i = 1; i < (int)(blockDim.x >> 6); ++i)
      if (sb[i] > best || (sb[i] == best && si[i] < best_i)) { best = sb[i]; best_i = si[i]; }
    // an all-NaN / all -inf row matches no comparison: emit token 0 instead of an index past the
    // vocabulary (the next step's embedding gather would read outside the table)
    out_ids[row] = (unsigned)best_i < (unsigned)V ? best_i : 0;
  }
}

// Truncated sampling with llama.cpp's default chain (its server's /completion, which the reference
// calls with only temperature 0.7): top-k -> top-p -> min-p on the raw logits, then temperature
// and a draw from the survivors (Gumbel-max with the same counter-based RNG as sample_kernel).
// One 256-thread workgroup per row, no host sync (graph-capturable):
//   1. radix-select the key of the k-th largest logit (4 passes of 256-bin LDS histograms over the
//      order-preserving uint32 image of the float), 2. gather the k largest into LDS (ties at the
//      threshold by ascending index), 3. sort them (value desc, index asc), 4. top-p / min-p cut on
//      the sorted survivors, 5. Gumbel-max over the kept ones.
#define SK_CAP 256

__device__ __forceinline__ uint32_t order_key(float f) {
  const uint32_t u = __float_as_uint(f);
  return (u & 0x80000000u) ? ~u : (u | 0x80000000u);
}

__global__ void __launch_bounds__(256) sample_topk_kernel(const uint16_t* __restrict__ logits, int V, float temperature,
                                                          int top_k, float top_p, float min_p, uint32_t seed,
                                                          const int32_t* __restrict__ step_ptr,
                                                          int32_t* __restrict__ out_ids) {
  const int row = blockIdx.x, tid = threadIdx.x;
  const uint16_t* lr = logits + (size_t)row * V;
  const uint32_t step = step_ptr ? (uint32_t)*step_ptr : 0u;
  const int K = max(1, min(top_k > 0 ? top_k : SK_CAP, min(V, SK_CAP)));
  __shared__ uint32_t hist[256];
  __shared__ uint32_t s_prefix, s_remaining;
  __shared__ float cv[SK_CAP];
  __shared__ int ci[SK_CAP];
  __shared__ int s_n;
  __shared__ float sv[SK_CAP];
  __shared__ int si[SK_CAP];
  __shared__ int s_keep;
  __shared__ int tie_i[4][SK_CAP];
  __shared__ int tie_n[4];

  // 1. radix select: key of the K-th largest element
  uint32_t prefix = 0, mask = 0, remaining = (uint32_t)K;
  for (int shift = 24; shift >= 0; shift -= 8) {
    hist[tid] = 0;
    __syncthreads();
    for (int i = tid; i < V; i += 256) {
      const uint32_t k = order_key(logit_nan_as_ninf(bf2f(lr[i])));
      if ((k & mask) == prefix) atomicAdd(&hist[(k >> shift) & 0xFF], 1u);
    }
    __syncthreads();
    if (tid == 0) {
      uint32_t cum = 0;
      int b = 255;
      for (; b > 0; --b) {
        if (cum + hist[b] >= remaining) break;
        cum += hist[b];
      }
      s_prefix = prefix | ((uint32_t)b << shift);
      s_remaining = remaining - cum;
    }
    __syncthreads();
    prefix = s_prefix;
    remaining = s_remaining;
    mask |= 0xFFu << shift;
  }
  // 2. gather: every key > threshold (fewer than K, any order: ranked below), then the `remaining`
  //    lowest-index keys == threshold -- each wave scans a quarter of the row in index order with
  //    ballots, so ties are taken by ascending index exactly like the reference
  if (tid == 0) s_n = 0;
  __syncthreads();
  for (int i = tid; i < V; i += 256) {
    const float f = logit_nan_as_ninf(bf2f(lr[i]));
    if (order_key(f) > prefix) {
      const int slot = atomicAdd(&s_n, 1);
      cv[slot] = f;
      ci[slot] = i;
    }
  }
  {
    const int w = tid >> 6, lane = tid & 63;
    const int lo = (int)(((int64_t)V * w) / 4), hi = (int)(((int64_t)V * (w + 1)) / 4);
    int found = 0;
    for (int base = lo; base < hi && found < (int)remaining; base += 64) {
      const int i = base + lane;
      const bool tie = i < hi && order_key(logit_nan_as_ninf(bf2f(lr[i]))) == prefix;
      const unsigned long long m = __ballot(tie);
      if (tie) {
        const int pos = found + __popcll(m & ((1ull << lane) - 1ull));
        if (pos < (int)remaining) tie_i[w][pos] = i;
      }
      found += __popcll(m);
    }
    if (lane == 0) tie_n[w] = min(found, (int)remaining);
  }
  __syncthreads();
  if (tid == 0) {
    int n0 = s_n;
    for (int w = 0; w < 4 && n0 < K; ++w)
      for (int j = 0; j < tie_n[w] && n0 < K; ++j) { ci[n0] = tie_i[w][j]; cv[n0] = logit_nan_as_ninf(bf2f(lr[tie_i[w][j]])); ++n0; }
    s_n = n0;
  }
  __syncthreads();
  const int n = s_n;
  // 3. rank = position in (value desc, index asc); keep rank < K
  if (tid < n) {
    const float v = cv[tid];
    const int id = ci[tid];
    int rank = 0;
    for (int j = 0; j < n; ++j) rank += (cv[j] > v) || (cv[j] == v && ci[j] < id);
    if (rank < K) { sv[rank] = v; si[rank] = id; }
  }
  __syncthreads();
  const int kk = min(n, K);
  // 4. top-p over softmax(logits) of the sorted survivors, min-p relative to the best (always >= 1 kept)
  if (tid == 0) {
    const float top = sv[0];
    float z = 0.f;
    for (int j = 0; j < kk; ++j) z += __expf(sv[j] - top);
    const float minp_logit = min_p > 0.f ? top + __logf(min_p) : -INFINITY;
    float cum = 0.f;
    int keep = 0;
    for (; keep < kk; ++keep) {
      if (keep > 0 && sv[keep] < minp_logit) break;
      cum += __expf(sv[keep] - top) / z;
      if (cum >= top_p) { ++keep; break; }
    }
    s_keep = max(1, min(keep, kk));
  }
  __syncthreads();
  // 5. temperature + Gumbel-max over the kept candidates (greedy if temperature <= 0)
  if (tid < 64) {
    float best = -INFINITY;
    int best_i = 0x7fffffff;
    for (int j = tid; j < s_keep; j += 64) {
      float x = sv[j];
      if (temperature > 0.f) {
        const uint32_t h = hash_u32(seed ^ hash_u32(step * 0x9E3779B9u ^ hash_u32(row * 0x85EBCA6Bu ^ (uint32_t)si[j])));
        const float u = ((h >> 8) + 0.5f) * (1.f / 16777216.f);
        x = x / temperature - __logf(-__logf(u));
      }
      if (x > best || (x == best && si[j] < best_i)) { best = x; best_i = si[j]; }
    }
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) {
      const float ob = __shfl_xor(best, o, 64);
      const int oi = __shfl_xor(best_i, o, 64);
      if (ob > best || (ob == best && oi < best_i)) { best = ob; best_i = oi; }
    }
    if (tid == 0) out_ids[row] = (unsigned)best_i < (unsigned)V ? best_i : 0;  // never outside the vocabulary
  }
}

// Advance the per-sequence decode state after sampling (one thread per sequence):
//   tokens[b][step] = next[b]; input_ids[b] = next[b]; positions[b]++; ctx_lens[b]++;
//   slots[b] = block_tables[b][pos/32]*32 + pos%32; done[b] |= next[b] in stop_ids.
// Thread 0 of block 0 also bumps the device step counter.
// Stop strings on the device (runtime/stops.py builds the tables): per token id the first L bytes
// it adds to the decoded text, its last H = L - 1 bytes, its byte length and whether a stop lies
// entirely inside it; per slot the last H bytes generated so far (wlen -1 = nothing yet, so a
// SentencePiece leading space is dropped as decode() does) and `keep` = tokens through the
// stop-completing one.  n_str == 0: no stop strings (the pointers are null).
struct StopTab {
  const uint8_t* head;
  const uint8_t* tail;
  const int32_t* tlen;
  const uint8_t* contains;
  const uint8_t* stops;
  const int32_t* stop_lens;
  int n_str, L, H, strip;
  uint8_t* win;
  int32_t* wlen;
  int32_t* keep;
};

// Feed token `tok` to slot b's window; true when a stop string now ends inside the token's bytes
// (a stop within the token, or one straddling the window and the token's first bytes).
__device__ bool stop_feed(const StopTab& t, int b, int tok) {
  uint8_t* w = t.win + (size_t)b * t.H;
  int wl = t.wlen[b];
  const bool fresh = wl < 0;
  if (fresh) wl = 0;
  const uint8_t* hd = t.head + (size_t)tok * t.L;
  int n = t.tlen[tok], off = 0;
  if (fresh && t.strip && n > 0 && hd[0] == ' ') { off = 1; n -= 1; }
  bool hit = t.contains[tok] != 0;
  for (int s = 0; s < t.n_str && !hit; ++s) {
    const uint8_t* sp = t.stops + (size_t)s * t.L;
    const int ls = t.stop_lens[s];
    for (int j = 1; j < ls && !hit; ++j) {   // j bytes from the window's end, ls - j from the token
      if (j > wl || ls - j > n) continue;
      bool ok = true;
      for (int q = 0; q < j && ok; ++q) ok = w[wl - j + q] == sp[q];
      for (int q = 0; q < ls - j && ok; ++q) ok = hd[off + q] == sp[j + q];
      hit = ok;
    }
  }
  if (n >= t.H) {
    const uint8_t* tl = t.tail + (size_t)tok * t.H;
    for (int q = 0; q < t.H; ++q) w[q] = tl[q];
    wl = t.H;
  } else if (n > 0) {
    const int kb = min(wl, t.H - n);
    for (int q = 0; q < kb; ++q) w[q] = w[wl - kb + q];
    for (int q = 0; q < n; ++q) w[kb + q] = hd[off + q];
    wl = kb + n;
  }
  t.wlen[b] = (fresh && n == 0) ? -1 : wl;
  return hit;
}

__global__ void decode_advance_kernel(const int32_t* __restrict__ next, int32_t* __restrict__ tokens, int max_new,
                                      int32_t* __restrict__ step_ptr, int32_t* __restrict__ input_ids,
                                      int32_t* __restrict__ positions, int32_t* __restrict__ ctx_lens,
                                      int32_t* __restrict__ slots, const int32_t* __restrict__ block_tables,
                                      int max_blocks, int32_t* __restrict__ done, const int32_t* __restrict__ stop_ids,
                                      int n_stop, int B, StopTab st) {
  const int b = blockIdx.x * blockDim.x + threadIdx.x;
  const int step = *step_ptr;
  __syncthreads();
  if (b < B) {
    const int tok = next[b];
    if (step < max_new) tokens[(size_t)b * max_new + step] = tok;
    input_ids[b] = tok;
    const int pos = positions[b] + 1;
    positions[b] = pos;
    ctx_lens[b] = pos + 1;
    slots[b] = block_tables[(size_t)b * max_blocks + pos / KV_BS] * KV_BS + pos % KV_BS;
    int d = done[b];
    if (st.n_str > 0 && !d && stop_feed(st, b, tok)) {
      d = 1;
      st.keep[b] = step + 1;   // tokens 0..step kept; the text is cut at the stop by the caller
    }
    for (int i = 0; i < n_stop; ++i) d |= (tok == stop_ids[i]);
    done[b] = d;
  }
  if (b == 0) *step_ptr = step + 1;
}

// Continuous batching: every slot carries its own generated-token count and limit.  Active,
// unfinished slots record the sampled token at tokens[b][gen[b]], advance their position and KV
// slot, and finish on a stop id or when gen reaches limit.  Finished / empty slots are frozen:
// their token, position and KV slot stay put (an empty slot points at the engine's scratch block),
// so the fixed-shape captured step can keep running over them.
__global__ void decode_advance_cb_kernel(const int32_t* __restrict__ next, int32_t* __restrict__ tokens, int cap,
                                         int32_t* __restrict__ gen, const int32_t* __restrict__ limit,
                                         int32_t* __restrict__ input_ids, int32_t* __restrict__ positions,
                                         int32_t* __restrict__ ctx_lens, int32_t* __restrict__ slots,
                                         const int32_t* __restrict__ block_tables, int max_blocks,
                                         int32_t* __restrict__ done, const int32_t* __restrict__ stop_ids, int n_stop,
                                         int B, StopTab st) {
  const int b = blockIdx.x * blockDim.x + threadIdx.x;
  if (b >= B || done[b]) return;
  const int tok = next[b];
  const int g = gen[b];
  if (g < cap) tokens[(size_t)b * cap + g] = tok;
  gen[b] = g + 1;
  int d = g + 1 >= limit[b];
  for (int i = 0; i < n_stop; ++i) d |= (tok == stop_ids[i]);
  if (st.n_str > 0 && stop_feed(st, b, tok)) {
    d = 1;
    st.keep[b] = g + 1;
  }
  done[b] = d;
  if (d) return;
  input_ids[b] = tok;
  const int pos = positions[b] + 1;
  positions[b] = pos;
  ctx_lens[b] = pos + 1;
  slots[b] = block_tables[(size_t)b * max_blocks + pos / KV_BS] * KV_BS + pos % KV_BS;
}

inline int ew_grid(size_t total) {
  size_t g = (total + 255) / 256;
  return (int)(g > 4096 ? 4096 : (g == 0 ? 1 : g));
}

}  // namespace

// decode V-cache store mode for the rope_kv launches (kv_write_v's VM: 0 plain, 1 write-through,
// 2 nontemporal); read at launch, so a captured graph keeps the mode it was captured with
static int g_kv_vstore_mode = 0;

CFC_API int cfc_set_kv_vstore_mode(int mode) {
  if (mode < 0 || mode > 2) return -1;
  g_kv_vstore_mode = mode;
  return 0;
}

CFC_API int cfc_rope_kv_write(const void* qkv, const int32_t* positions, const int32_t* slots, const float* cos_sin,
                              void* q_out, void* k_cache, void* v_cache, int T, int Hq, int Hkv, int head_dim,
                              int write_v, hipStream_t stream) {
  if (head_dim % 16 != 0 || T < 0) return -1;
  if (T == 0) return 0;
  const int items = (Hq + Hkv) * (head_dim / 16) + (write_v ? Hkv * (head_dim / 8) : 0);
  const dim3 grid(T, (items + 63) / 64);
  const auto* x = (const uint16_t*)qkv;
  if (write_v && g_kv_vstore_mode == 1)
    rope_kv_kernel<false, 1><<<grid, 64, 0, stream>>>(x, positions, slots, cos_sin, (uint16_t*)q_out, k_cache,
                                                      v_cache, Hq, Hkv, head_dim, 1, 1.f, 1.f);
  else if (write_v && g_kv_vstore_mode == 2)
    rope_kv_kernel<false, 2><<<grid, 64, 0, stream>>>(x, positions, slots, cos_sin, (uint16_t*)q_out, k_cache,
                                                      v_cache, Hq, Hkv, head_dim, 1, 1.f, 1.f);
  else
    rope_kv_kernel<false><<<grid, 64, 0, stream>>>(x, positions, slots, cos_sin, (uint16_t*)q_out, k_cache, v_cache,
                                                   Hq, Hkv, head_dim, write_v, 1.f, 1.f);
  return CFC_CHECK_LAUNCH();
}

// FP8 (e4m3fn) KV cache: k/v stored as value * inv_k / inv_v
CFC_API int cfc_rope_kv_write_fp8(const void* qkv, const int32_t* positions, const int32_t* slots,
                                  const float* cos_sin, void* q_out, void* k_cache, void* v_cache, int T, int Hq,
                                  int Hkv, int head_dim, int write_v, float inv_k, float inv_v, hipStream_t stream) {
  if (head_dim % 16 != 0 || T < 0) return -1;
  if (T == 0) return 0;
  const int items = (Hq + Hkv) * (head_dim / 16) + (write_v ? Hkv * (head_dim / 8) : 0);
  rope_kv_kernel<true><<<dim3(T, (items + 63) / 64), 64, 0, stream>>>(
      (const uint16_t*)qkv, positions, slots, cos_sin, (uint16_t*)q_out, k_cache, v_cache, Hq, Hkv, head_dim, write_v,
      inv_k, inv_v);
  return CFC_CHECK_LAUNCH();
}

// runs: [R][4] int32 {first token, count (1..32), cache block, first offset (count + offset <= 32)}
CFC_API int cfc_v_cache_write_runs(const void* qkv, const int32_t* runs, int R, void* v_cache, int Hq, int Hkv,
                                   int head_dim, hipStream_t stream) {
  if (head_dim % 8 != 0 || head_dim > 256 || R < 0) return -1;
  if (R == 0) return 0;
  v_cache_runs_kernel<false><<<dim3(R, Hkv), 256, 0, stream>>>((const uint16_t*)qkv, runs, v_cache, Hq, Hkv,
                                                               head_dim, 1.f);
  return CFC_CHECK_LAUNCH();
}

CFC_API int cfc_v_cache_write_runs_fp8(const void* qkv, const int32_t* runs, int R, void* v_cache, int Hq, int Hkv,
                                       int head_dim, float inv_v, hipStream_t stream) {
  if (head_dim % 8 != 0 || head_dim > 256 || R < 0) return -1;
  if (R == 0) return 0;
  v_cache_runs_kernel<true><<<dim3(R, Hkv), 256, 0, stream>>>((const uint16_t*)qkv, runs, v_cache, Hq, Hkv, head_dim,
                                                              inv_v);
  return CFC_CHECK_LAUNCH();
}

CFC_API int cfc_decode_advance_cb(const int32_t* next, int32_t* tokens, int cap, int32_t* gen, const int32_t* limit,
                                  int32_t* input_ids, int32_t* positions, int32_t* ctx_lens, int32_t* slots,
                                  const int32_t* block_tables, int max_blocks, int32_t* done, const int32_t* stop_ids,
                                  int n_stop, int B, const uint8_t* head, const uint8_t* tail, const int32_t* tlen,
                                  const uint8_t* contains, const uint8_t* stops, const int32_t* stop_lens, int n_str,
                                  int L, int H, int strip, uint8_t* win, int32_t* wlen, int32_t* keep,
                                  hipStream_t stream) {
  if (B <= 0) return 0;
  if (n_str > 0 && (L < 1 || H < 1 || L > 32 || !head || !tail || !tlen || !contains || !stops || !stop_lens ||
                    !win || !wlen || !keep))
    return -1;
  const StopTab st{head, tail, tlen, contains, stops, stop_lens, n_str, L, H, strip, win, wlen, keep};
  decode_advance_cb_kernel<<<(B + 255) / 256, 256, 0, stream>>>(next, tokens, cap, gen, limit, input_ids, positions,
                                                                 ctx_lens, slots, block_tables, max_blocks, done,
                                                                 stop_ids, n_stop, B, st);
  return CFC_CHECK_LAUNCH();
}

CFC_API int cfc_quant_fp8_rows(void* out, float* scale, const void* x, int M, int K, hipStream_t stream) {
  if (K % 8 != 0 || K > 256 * 8 * QR_MAX_VEC || M < 0) return -1;
  if (M == 0) return 0;
  quant_fp8_rows_kernel<<<M, 256, 0, stream>>>((const uint16_t*)x, (uint8_t*)out, scale, K);
  return CFC_CHECK_LAUNCH();
}

CFC_API int cfc_silu_mul(void* out, const void* gu, int T, int F, int interleave, hipStream_t stream) {
  if (F % 8 != 0 || T > 65535) return -1;
  if (T == 0) return 0;
  silu_mul_kernel<<<dim3((F / 8 + 255) / 256, T), 256, 0, stream>>>((uint16_t*)out, (const uint16_t*)gu, F, interleave);
  return CFC_CHECK_LAUNCH();
}

CFC_API int cfc_silu_mul_fp8(void* out, float* scale, const void* gu, int T, int F, int interleave,
                             hipStream_t stream) {
  if (F % 8 != 0 || F > 1024 * 8 * SQ_MAX_VEC || T < 0) return -1;
  if (T == 0) return 0;
  silu_mul_fp8_kernel<<<T, 1024, 0, stream>>>((uint8_t*)out, scale, (const uint16_t*)gu, F, interleave);
  return CFC_CHECK_LAUNCH();
}

CFC_API int cfc_bias_gelu(void* out, const void* x, const void* bias, int T, int F, hipStream_t stream) {
  if (F % 8 != 0) return -1;
  if (T == 0) return 0;
  bias_gelu_kernel<<<ew_grid((size_t)T * F / 8), 256, 0, stream>>>((uint16_t*)out, (const uint16_t*)x,
                                                                   (const uint16_t*)bias, T, F);
  return CFC_CHECK_LAUNCH();
}

CFC_API int cfc_embedding(void* out, const void* table, const int32_t* ids, int T, int dim, hipStream_t stream) {
  if (dim % 8 != 0) return -1;
  if (T == 0) return 0;
  embedding_kernel<<<T, 256, 0, stream>>>((uint16_t*)out, (const uint16_t*)table, ids, T, dim);
  return CFC_CHECK_LAUNCH();
}

// top_k <= 0: no top-k cut (candidates still capped at SK_CAP = 256); top_p >= 1 / min_p <= 0 disable those.
CFC_API int cfc_sample_truncated(const void* logits, int B, int V, float temperature, int top_k, float top_p,
                                 float min_p, uint32_t seed, const int32_t* step_ptr, int32_t* out_ids,
                                 hipStream_t stream) {
  if (B == 0) return 0;
  if (V <= 0 || top_p <= 0.f) return -1;
  sample_topk_kernel<<<B, 256, 0, stream>>>((const uint16_t*)logits, V, temperature, top_k, top_p, min_p, seed,
                                            step_ptr, out_ids);
  return CFC_CHECK_LAUNCH();
}

CFC_API int cfc_sample(const void* logits, int B, int V, float temperature, uint32_t seed, const int32_t* step_ptr,
                       int32_t* out_ids, hipStream_t stream) {
  if (B == 0) return 0;
  sample_kernel<<<B, 1024, 0, stream>>>((const uint16_t*)logits, V, temperature, seed, step_ptr, out_ids);
  return CFC_CHECK_LAUNCH();
}

CFC_API int cfc_decode_advance(const int32_t* next, int32_t* tokens, int max_new, int32_t* step_ptr, int32_t* input_ids,
                               int32_t* positions, int32_t* ctx_lens, int32_t* slots, const int32_t* block_tables,
                               int max_blocks, int32_t* done, const int32_t* stop_ids, int n_stop, int B,
                               const uint8_t* head, const uint8_t* tail, const int32_t* tlen, const uint8_t* contains,
                               const uint8_t* stops, const int32_t* stop_lens, int n_str, int L, int H, int strip,
                               uint8_t* win, int32_t* wlen, int32_t* keep, hipStream_t stream) {
  if (B <= 0) return 0;
  if (B > 1024) return -1;  // single workgroup: the step counter bump must not race other blocks
  if (n_str > 0 && (L < 1 || H < 1 || L > 32 || !head || !tail || !tlen || !contains || !stops || !stop_lens ||
                    !win || !wlen || !keep))
    return -1;
  const StopTab st{head, tail, tlen, contains, stops, stop_lens, n_str, L, H, strip, win, wlen, keep};
  decode_advance_kernel<<<1, ((B + 63) / 64) * 64, 0, stream>>>(next, tokens, max_new, step_ptr, input_ids, positions,
                                                               ctx_lens, slots, block_tables, max_blocks, done,
                                                               stop_ids, n_stop, B, st);
  return CFC_CHECK_LAUNCH();
}

// Decode: RoPE + K/V cache write straight from the qkv projection's fp32 split-K slabs
// part [split][T][(Hq + 2 Hkv) D] (dgemm "part" epilogue) -- the reduce kernel folded in.
CFC_API int cfc_rope_kv_write_part(const float* part, int split, const int32_t* positions, const int32_t* slots,
                                   const float* cos_sin, void* q_out, void* k_cache, void* v_cache, int T, int Hq,
                                   int Hkv, int head_dim, int fp8, float inv_k, float inv_v, hipStream_t stream) {
  if (head_dim % 16 != 0 || T < 0 || split < 1 || part == nullptr) return -1;
  if (T == 0) return 0;
  const int items = (Hq + Hkv) * (head_dim / 16) + Hkv * (head_dim / 8);
  const dim3 grid(T, (items + 63) / 64);
#define ROPE_PART(F8, VM)                                                                                          \
  rope_kv_kernel<F8, VM><<<grid, 64, 0, stream>>>(nullptr, positions, slots, cos_sin, (uint16_t*)q_out, k_cache,   \
                                                  v_cache, Hq, Hkv, head_dim, 1, F8 ? inv_k : 1.f, F8 ? inv_v : 1.f, \
                                                  part, split)
  switch (g_kv_vstore_mode * 2 + (fp8 ? 1 : 0)) {
    case 2: ROPE_PART(false, 1); break;
    case 3: ROPE_PART(true, 1); break;
    case 4: ROPE_PART(false, 2); break;
    case 5: ROPE_PART(true, 2); break;
    case 1: ROPE_PART(true, 0); break;
    default: ROPE_PART(false, 0); break;
  }
#undef ROPE_PART
  return CFC_CHECK_LAUNCH();
}
