// Vector-search kernels: HBM-resident flat index scan + exact top-k, and the encoder's
// pooling/normalisation epilogue.
//
// Replaces the reference's vector-store hot paths: InMemoryVectorStore's python cosine loop
// (adapters/copilot_vectorstore/copilot_vectorstore/inmemory.py:106-119), FAISS IndexFlatL2 /
// IVFFlat (faiss_store.py:101-111,214) and Qdrant query_points (qdrant_store.py:371).
//
//   * cfc_knn_scores: scores[q][n] = <x_n, q>  (or -||x_n - q||^2) for <= 16 queries, one pass
//     over the bf16 index with MFMA 16x16x32 (queries are the B columns, index rows stream
//     straight from HBM into the A operand: the GEMV regime of guide §5 table, last row).
//   * cfc_topk: exact per-query top-k by 4-pass 8-bit radix select in LDS per chunk; applied
//     recursively on the candidates until one chunk remains.
//   * cfc_l2_normalize: rows -> unit length (+ fp32 norms), used on insert for cosine.
//   * cfc_pool: masked mean / CLS pooling over varlen sequences (+ optional L2 normalise):
//     the SentenceTransformer Pooling+Normalize modules.
#include "common.h"

namespace {

__device__ __forceinline__ bf16x8_t as_bf16x8(uint4 v) { return __builtin_bit_cast(bf16x8_t, v); }

template <int KC>  // KC = D / 32 MFMA k-steps
__global__ void __launch_bounds__(256) knn_scores_kernel(const uint16_t* __restrict__ X, const uint16_t* __restrict__ Q,
                                                         int N, int nq, const float* __restrict__ xnorm2,
                                                         const float* __restrict__ qnorm2, float* __restrict__ out) {
  constexpr int D = KC * 32;
  const int lane = threadIdx.x & 63;
  const int col = lane & 15, g = lane >> 4;
  const bool qv = col < nq;
  bf16x8_t qf[KC];
  {
    const uint16_t* qr = Q + (size_t)(qv ? col : 0) * D;
#pragma unroll
    for (int c = 0; c < KC; ++c)
      qf[c] = as_bf16x8(qv ? *reinterpret_cast<const uint4*>(qr + 32 * c + 8 * g) : make_uint4(0, 0, 0, 0));
  }
  const float qn = (qnorm2 && qv) ? qnorm2[col] : 0.f;
  const int ngroups = (N + 15) / 16;
  const int wave_global = (blockIdx.x * blockDim.x + threadIdx.x) >> 6;
  const int nwaves = (gridDim.x * blockDim.x) >> 6;
  for (int grp = wave_global; grp < ngroups; grp += nwaves) {
    const int r0 = grp * 16;
    const int r = min(r0 + col, N - 1);
    const uint16_t* xr = X + (size_t)r * D;
    uint4 a[KC];
#pragma unroll
    for (int c = 0; c < KC; ++c) a[c] = *reinterpret_cast<const uint4*>(xr + 32 * c + 8 * g);
    f32x4_t acc = {0.f, 0.f, 0.f, 0.f};
#pragma unroll
    for (int c = 0; c < KC; ++c) acc = __builtin_amdgcn_mfma_f32_16x16x32_bf16(as_bf16x8(a[c]), qf[c], acc, 0, 0, 0);
    if (qv) {
      const int rb = r0 + 4 * g;
      float v[4];
#pragma unroll
      for (int i = 0; i < 4; ++i) {
        v[i] = acc[i];
        if (xnorm2) v[i] = -(xnorm2[min(rb + i, N - 1)] + qn - 2.f * v[i]);
      }
      float* orow = out + (size_t)col * N;
      if (rb + 3 < N && (N & 3) == 0) {
        *reinterpret_cast<float4*>(orow + rb) = make_float4(v[0], v[1], v[2], v[3]);
      } else {
#pragma unroll
        for (int i = 0; i < 4; ++i)
          if (rb + i < N) orow[rb + i] = v[i];
      }
    }
  }
}

__device__ __forceinline__ uint32_t f2key(float f) {
  const uint32_t u = __float_as_uint(f);
  return (u & 0x80000000u) ? ~u : (u | 0x80000000u);
}
__device__ __forceinline__ float key2f(uint32_t k) {
  return __uint_as_float((k & 0x80000000u) ? (k & 0x7fffffffu) : ~k);
}

constexpr int TOPK_CHUNK = 8192;

// grid = (nchunks, nq), block = 256.  in: [nq][n] fp32 scores (row stride ld), optional idx_in
// [nq][n] int64 ids; out: [nq][nchunks][k] (unordered within a chunk).
__global__ void __launch_bounds__(256) topk_chunk_kernel(const float* __restrict__ in, const int64_t* __restrict__ idx_in,
                                                         int n, int ld, int k, float* __restrict__ out_v,
                                                         int64_t* __restrict__ out_i) {
  __shared__ uint32_t keys[TOPK_CHUNK];
  __shared__ uint32_t hist[256];
  __shared__ uint32_t s_prefix, s_need, s_cnt_gt, s_cnt_eq;
  const int chunk = blockIdx.x, qi = blockIdx.y, tid = threadIdx.x;
  const int beg = chunk * TOPK_CHUNK;
  const int len = min(TOPK_CHUNK, n - beg);
  const float* src = in + (size_t)qi * ld + beg;
  for (int i = tid; i < len; i += 256) keys[i] = f2key(src[i]);
  const int kk = min(k, len);
  if (tid == 0) { s_prefix = 0; s_need = kk; }
  __syncthreads();
  uint32_t mask = 0;
  for (int shift = 24; shift >= 0; shift -= 8) {
    hist[tid] = 0;
    __syncthreads();
    const uint32_t prefix = s_prefix;
    for (int i = tid; i < len; i += 256) {
      const uint32_t key = keys[i];
      if ((key & mask) == prefix) atomicAdd(&hist[(key >> shift) & 255u], 1u);
    }
    __syncthreads();
    if (tid == 0) {
      uint32_t need = s_need, acc = 0;
      int d = 255;
      for (; d > 0; --d) {
        if (acc + hist[d] >= need) break;
        acc += hist[d];
      }
      s_need = need - acc;
      s_prefix = prefix | ((uint32_t)d << shift);
    }
    mask |= 255u << shift;
    __syncthreads();
  }
  const uint32_t thr = s_prefix;
  const uint32_t need_eq = s_need;
  if (tid == 0) { s_cnt_gt = 0; s_cnt_eq = 0; }
  __syncthreads();
  float* ov = out_v + ((size_t)qi * gridDim.x + chunk) * k;
  int64_t* oi = out_i + ((size_t)qi * gridDim.x + chunk) * k;
  const uint32_t n_gt = (uint32_t)kk - need_eq;
  for (int i = tid; i < len; i += 256) {
    const uint32_t key = keys[i];
    int slot = -1;
    if (key > thr) slot = (int)atomicAdd(&s_cnt_gt, 1u);
    else if (key == thr) {
      const uint32_t e = atomicAdd(&s_cnt_eq, 1u);
      if (e < need_eq) slot = (int)(n_gt + e);
    }
    if (slot >= 0) {
      ov[slot] = key2f(key);
      oi[slot] = idx_in ? idx_in[(size_t)qi * ld + beg + i] : (int64_t)(beg + i);
    }
  }
  for (int s = kk + tid; s < k; s += 256) { ov[s] = -INFINITY; oi[s] = -1; }
}

__global__ void __launch_bounds__(256) l2_normalize_kernel(uint16_t* __restrict__ out, const uint16_t* __restrict__ in,
                                                           float* __restrict__ norms2, int dim) {
  __shared__ float red[16];
  const int row = blockIdx.x;
  const int nvec = dim / 8;
  const uint4* src = reinterpret_cast<const uint4*>(in + (size_t)row * dim);
  float ss = 0.f;
  for (int c = threadIdx.x; c < nvec; c += blockDim.x) {
    float v[8];
    unpack8(src[c], v);
#pragma unroll
    for (int j = 0; j < 8; ++j) ss += v[j] * v[j];
  }
  ss = block_sum(ss, red);
  if (norms2 && threadIdx.x == 0) norms2[row] = ss;
  const float inv = ss > 0.f ? rsqrtf(ss) : 0.f;
  if (!out) return;
  uint4* dst = reinterpret_cast<uint4*>(out + (size_t)row * dim);
  for (int c = threadIdx.x; c < nvec; c += blockDim.x) {
    float v[8];
    unpack8(src[c], v);
#pragma unroll
    for (int j = 0; j < 8; ++j) v[j] *= inv;
    dst[c] = pack8(v);
  }
}

// grid = nseq, block = 256. mode 0: masked mean over the sequence's tokens; 1: CLS (first
// token); 2: unmasked mean over a fixed padded length (HF provider parity,
// huggingface_provider.py:101) -- identical to 0 for packed varlen input.
__global__ void __launch_bounds__(256) pool_kernel(float* __restrict__ out_f32, uint16_t* __restrict__ out_bf16,
                                                   const uint16_t* __restrict__ hidden,
                                                   const int32_t* __restrict__ cu_seqlens, int dim, int mode,
                                                   int normalize) {
  __shared__ float red[16];
  extern __shared__ __attribute__((aligned(16))) float acc[];  // dim floats
  const int s = blockIdx.x;
  const int beg = cu_seqlens[s], len = cu_seqlens[s + 1] - beg;
  const int cnt = mode == 1 ? min(len, 1) : len;
  for (int d = threadIdx.x; d < dim; d += blockDim.x) {
    float sum = 0.f;
    for (int t = 0; t < cnt; ++t) sum += bf2f(hidden[(size_t)(beg + t) * dim + d]);
    acc[d] = cnt > 0 ? sum / (float)cnt : 0.f;
  }
  __syncthreads();
  float ss = 0.f;
  for (int d = threadIdx.x; d < dim; d += blockDim.x) ss += acc[d] * acc[d];
  ss = block_sum(ss, red);
  const float inv = (normalize && ss > 0.f) ? rsqrtf(ss) : 1.f;
  for (int d = threadIdx.x; d < dim; d += blockDim.x) {
    const float v = acc[d] * inv;
    if (out_f32) out_f32[(size_t)s * dim + d] = v;
    if (out_bf16) out_bf16[(size_t)s * dim + d] = f2bf(v);
  }
}

}  // namespace

CFC_API int cfc_knn_scores(const void* X, const void* Q, int N, int nq, int dim, const float* xnorm2,
                           const float* qnorm2, float* out, hipStream_t stream) {
  if (nq < 1 || nq > 16 || dim % 32 != 0 || N <= 0) return -1;
  const int groups = (N + 15) / 16;
  int blocks = (groups + 3) / 4;
  if (blocks > 256 * 16) blocks = 256 * 16;
#define KS(KC) knn_scores_kernel<KC><<<blocks, 256, 0, stream>>>((const uint16_t*)X, (const uint16_t*)Q, N, nq, xnorm2, qnorm2, out)
  switch (dim / 32) {
    case 4: KS(4); break;     // 128
    case 8: KS(8); break;     // 256
    case 12: KS(12); break;   // 384 (MiniLM, bge-small)
    case 16: KS(16); break;   // 512
    case 24: KS(24); break;   // 768 (bge-base, mpnet)
    case 32: KS(32); break;   // 1024 (bge-large)
    default: return -2;
  }
#undef KS
  return CFC_CHECK_LAUNCH();
}

// One radix-select pass: in [nq][n] (row stride ld) -> out [nq][ceil(n/8192)][k].
CFC_API int cfc_topk_pass(const float* in, const int64_t* idx_in, int nq, int n, int ld, int k, float* out_v,
                          int64_t* out_i, hipStream_t stream) {
  if (k <= 0 || k > 2048 || n <= 0) return -1;
  const int nchunks = (n + TOPK_CHUNK - 1) / TOPK_CHUNK;
  topk_chunk_kernel<<<dim3(nchunks, nq), 256, 0, stream>>>(in, idx_in, n, ld, k, out_v, out_i);
  return CFC_CHECK_LAUNCH();
}

CFC_API int cfc_topk_chunk_size() { return TOPK_CHUNK; }

CFC_API int cfc_l2_normalize(void* out, const void* in, float* norms2, int rows, int dim, hipStream_t stream) {
  if (dim % 8 != 0) return -1;
  if (rows == 0) return 0;
  l2_normalize_kernel<<<rows, dim >= 2048 ? 256 : 64, 0, stream>>>((uint16_t*)out, (const uint16_t*)in, norms2, dim);
  return CFC_CHECK_LAUNCH();
}

CFC_API int cfc_pool(float* out_f32, void* out_bf16, const void* hidden, const int32_t* cu_seqlens, int nseq, int dim,
                     int mode, int normalize, hipStream_t stream) {
  if (nseq == 0) return 0;
  pool_kernel<<<nseq, 256, dim * sizeof(float), stream>>>(out_f32, (uint16_t*)out_bf16, (const uint16_t*)hidden,
                                                          cu_seqlens, dim, mode, normalize);
  return CFC_CHECK_LAUNCH();
}
