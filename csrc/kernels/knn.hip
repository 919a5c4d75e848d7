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
//   * cfc_knn_topk / cfc_ivf_topk: the scan and the top-k FUSED: each workgroup scores its
//     1024-row chunk against its queries into LDS and radix-selects every query's k best there,
//     so only k candidates per (query, chunk) reach HBM (never the [nq, N] score matrix); the
//     IVF form takes (query, probed list, chunk) work items from a device list-offset table in
//     one launch.  The candidates are merged by cfc_topk_pass.
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

// ------------------------------------------------------------------ fused scan + top-k
constexpr int KT_ROWS = 1024;   // rows per workgroup chunk (scores [nqb][KT_ROWS] fp32 in LDS)

// Wave-level exact top-k of sc[0..len) (LDS, len <= KT_ROWS): every lane holds 16 keys in
// registers (row lane + 64 j); the k-th largest key is found bit by bit, MSB first, from wave-wide
// counts of keys >= the candidate (32 rounds of 16 compare-ballot-popcounts, all in SGPRs/VALU) --
// no LDS: a radix histogram's atomics serialise here because one chunk's scores share their top
// key bytes, and a shuffle-tree sum pays an LDS round trip per level.
// Writes exactly k slots (ov/oi; -inf / -1 padding when len < k).
template <int ROWS>
__device__ __forceinline__ void wave_topk(const float* sc, int len, int k, int64_t row0, const int64_t* ids, float* ov, int64_t* oi,
                          uint32_t* /*unused*/) {
  const int lane = threadIdx.x & 63;
  const int kk = min(k, len);
  uint32_t key[ROWS / 64];
#pragma unroll
  for (int j = 0; j < ROWS / 64; ++j) {
    const int i = lane + 64 * j;
    key[j] = i < len ? f2key(sc[i]) : 0u;
  }
  uint32_t thr = 0;
  if (kk > 0) {
    for (int b = 31; b >= 0; --b) {
      const uint32_t cand = thr | (1u << b);
      int c = 0;
#pragma unroll
      for (int j = 0; j < ROWS / 64; ++j) c += __popcll(__ballot(key[j] >= cand));
      if (c >= kk) thr = cand;                 // wave-uniform decision
    }
  }
  int gt = 0;
#pragma unroll
  for (int j = 0; j < ROWS / 64; ++j) gt += __popcll(__ballot(key[j] > thr));
  const uint32_t n_gt = (uint32_t)gt;
  const uint32_t need = (uint32_t)kk - n_gt;   // keys == thr to take (>= 1 when kk > 0)
  uint32_t base_gt = 0, base_eq = 0;
  const uint64_t below = (lane == 0) ? 0ull : (~0ull >> (64 - lane));
#pragma unroll
  for (int j = 0; j < ROWS / 64; ++j) {
    const int i = lane + 64 * j;
    const bool g = kk > 0 && i < len && key[j] > thr, e = kk > 0 && i < len && key[j] == thr;
    const uint64_t bg = __ballot(g), be = __ballot(e);
    int slot = -1;
    if (g) slot = (int)(base_gt + __popcll(bg & below));
    else if (e) {
      const uint32_t q = base_eq + __popcll(be & below);
      if (q < need) slot = (int)(n_gt + q);
    }
    if (slot >= 0) {
      ov[slot] = key2f(key[j]);
      oi[slot] = ids ? ids[row0 + i] : row0 + i;
    }
    base_gt += __popcll(bg);
    base_eq += __popcll(be);
  }
  for (int s2 = kk + lane; s2 < k; s2 += 64) { ov[s2] = -INFINITY; oi[s2] = -1; }
}

// Work item = a chunk of <= ROWS consecutive rows and a set of queries (qsel < 0: all nq, else
// query qsel only).  Flat: blockIdx.x = chunk, queries all.  IVF (probe != null): blockIdx.x =
// (q * nprobe + j) * maxc + c -> list probe[q][j], its chunk c.  out_v/out_i: [nq][nslots][k].
// ROWS per workgroup: the scores of all its queries sit in LDS between the scan and the select, so
// with many queries the chunk is shorter (knn_flat_rows) -- more workgroups resident per CU, one
// workgroup's select overlapping the others' scans.
template <int KC, int ROWS>
__global__ void __launch_bounds__(256) knn_topk_kernel(const uint16_t* __restrict__ X, const uint16_t* __restrict__ Q,
                                                       int N, int nq, const float* __restrict__ xnorm2,
                                                       const float* __restrict__ qnorm2,
                                                       const uint8_t* __restrict__ alive, int k, int row_lo,
                                                       const int32_t* __restrict__ probe, int nprobe, int maxc,
                                                       const int64_t* __restrict__ list_off, int nslots,
                                                       float* __restrict__ out_v, int64_t* __restrict__ out_i) {
  constexpr int D = KC * 32;
  extern __shared__ __attribute__((aligned(16))) float kt_smem[];
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
  int lo, hi, q0, nqb, slot;
  if (probe == nullptr) {
    lo = row_lo + blockIdx.x * ROWS;
    hi = min(N, lo + ROWS);
    q0 = 0;
    nqb = nq;
    slot = blockIdx.x;
  } else {
    const int c = blockIdx.x % maxc, qj = blockIdx.x / maxc;
    q0 = qj / nprobe;
    nqb = 1;
    slot = (qj % nprobe) * maxc + c;
    const int l = probe[qj];
    lo = (int)list_off[l] + c * ROWS;
    hi = min((int)list_off[l + 1], lo + ROWS);
  }
  const int len = max(0, hi - lo);
  float* sc = kt_smem;                                        // [nqb][ROWS]
  uint32_t* hist = reinterpret_cast<uint32_t*>(kt_smem + nqb * ROWS) + 256 * w;
  if (len > 0) {
    const int col = lane & 15, g = lane >> 4;
    const bool qv = col < nqb;
    bf16x8_t qf[KC];
    const uint16_t* qr = Q + (size_t)(q0 + (qv ? col : 0)) * D;
#pragma unroll
    for (int c = 0; c < KC; ++c)
      qf[c] = as_bf16x8(qv ? *reinterpret_cast<const uint4*>(qr + 32 * c + 8 * g) : make_uint4(0, 0, 0, 0));
    const float qn = (qnorm2 && qv) ? qnorm2[q0 + col] : 0.f;
    const int ngroups = (len + 15) / 16;
    for (int grp = w; grp < ngroups; grp += 4) {
      const int r0 = lo + grp * 16;
      const int r = min(r0 + col, hi - 1);
      const uint16_t* xr = X + (size_t)r * D;
      uint4 a[KC];
#pragma unroll
      for (int c = 0; c < KC; ++c) a[c] = *reinterpret_cast<const uint4*>(xr + 32 * c + 8 * g);
      f32x4_t acc = {0.f, 0.f, 0.f, 0.f};
#pragma unroll
      for (int c = 0; c < KC; ++c) acc = __builtin_amdgcn_mfma_f32_16x16x32_bf16(as_bf16x8(a[c]), qf[c], acc, 0, 0, 0);
      if (qv) {
#pragma unroll
        for (int i = 0; i < 4; ++i) {
          const int row = r0 + 4 * g + i;
          if (row < hi) {
            float v = acc[i];
            if (xnorm2) v = -(xnorm2[row] + qn - 2.f * v);
            if (alive && !alive[row]) v = -INFINITY;
            sc[col * ROWS + (row - lo)] = v;
          }
        }
      }
    }
  }
  __syncthreads();
  for (int qi = w; qi < nqb; qi += 4) {
    const size_t o = ((size_t)(q0 + qi) * nslots + slot) * k;
    wave_topk<ROWS>(sc + qi * ROWS, len, k, lo, nullptr, out_v + o, out_i + o, hist);
  }
}

// ------------------------------------------------------------------ streamed scan + top-k (large k)
// With a large k the per-chunk candidates of knn_topk_kernel are a big share of the rows (k = 150
// from 512-row chunks: 29 % of the index written as candidates and read again by the merge).  Here
// a workgroup (8 waves; two workgroups per CU = 4 waves per SIMD) scans a long span (KS_SPAN rows) in
// KS_SUB-row sub-chunks and keeps, per query, a
// candidate buffer in LDS behind a running threshold: only rows scoring above the k-th best key
// the buffer held at its last cut are appended, and when the next sub-chunk could overflow the
// buffer it is cut back to its exact top k (the threshold rises).  k candidates per query leave
// per KS_SPAN rows (0.9 % at k = 150).  Rows equal to the threshold that arrive after a cut are
// skipped: the buffer already holds k keys >= it, so the result is exact up to tie order.
constexpr int KS_SUB = 256, KS_CAP = 512, KS_SPAN = 16384;

// keys held KS_CAP / 64 per lane (entry lane + 64 j; 0 = empty): the exact kk-th largest
__device__ __forceinline__ uint32_t ks_kth(const uint32_t* key, int kk) {
  uint32_t thr = 0;
  for (int b = 31; b >= 0; --b) {
    const uint32_t cand = thr | (1u << b);
    int c = 0;
#pragma unroll
    for (int j = 0; j < KS_CAP / 64; ++j) c += __popcll(__ballot(key[j] >= cand));
    if (c >= kk) thr = cand;                 // wave-uniform decision
  }
  return thr;
}

// Cut a query's buffer (cnt > kk entries) to its exact top kk, in place (wave-level; every entry is
// in registers before the first write).  Returns the kk-th largest key (the new threshold).
__device__ __forceinline__ uint32_t ks_cut(uint32_t* bk, uint32_t* br, int cnt, int kk) {
  const int lane = threadIdx.x & 63;
  uint32_t key[KS_CAP / 64], row[KS_CAP / 64];
#pragma unroll
  for (int j = 0; j < KS_CAP / 64; ++j) {
    const int i = lane + 64 * j;
    key[j] = i < cnt ? bk[i] : 0u;
    row[j] = i < cnt ? br[i] : 0u;
  }
  const uint32_t thr = ks_kth(key, kk);
  int gt = 0;
#pragma unroll
  for (int j = 0; j < KS_CAP / 64; ++j) gt += __popcll(__ballot(key[j] > thr));
  const uint32_t need = (uint32_t)(kk - gt);
  const uint64_t below = (lane == 0) ? 0ull : (~0ull >> (64 - lane));
  uint32_t base_gt = 0, base_eq = 0;
#pragma unroll
  for (int j = 0; j < KS_CAP / 64; ++j) {
    const bool g = key[j] > thr, e = key[j] == thr && key[j] != 0u;
    const uint64_t bg = __ballot(g), be = __ballot(e);
    int slot = -1;
    if (g) slot = (int)(base_gt + __popcll(bg & below));
    else if (e) {
      const uint32_t q = base_eq + __popcll(be & below);
      if (q < need) slot = gt + (int)q;
    }
    if (slot >= 0) { bk[slot] = key[j]; br[slot] = row[j]; }
    base_gt += __popcll(bg);
    base_eq += __popcll(be);
  }
  return thr;
}

template <int KC>
__global__ void __launch_bounds__(512) knn_topk_stream_kernel(const uint16_t* __restrict__ X,
                                                              const uint16_t* __restrict__ Q, int N, int nq,
                                                              const float* __restrict__ xnorm2,
                                                              const float* __restrict__ qnorm2,
                                                              const uint8_t* __restrict__ alive, int k, int row_lo,
                                                              float* __restrict__ out_v, int64_t* __restrict__ out_i) {
  constexpr int D = KC * 32;
  __shared__ float sc[16 * KS_SUB];                                        // 16 KB scores
  __shared__ uint32_t bk[16 * KS_CAP], br[16 * KS_CAP];                     // 64 KB buffers
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
  const int lo = row_lo + blockIdx.x * KS_SPAN, hi = min(N, lo + KS_SPAN);
  const int col = lane & 15, g = lane >> 4;
  const bool qv = col < nq;
  bf16x8_t qf[KC];
  const uint16_t* qrow = Q + (size_t)(qv ? col : 0) * D;
#pragma unroll
  for (int c = 0; c < KC; ++c)
    qf[c] = as_bf16x8(qv ? *reinterpret_cast<const uint4*>(qrow + 32 * c + 8 * g) : make_uint4(0, 0, 0, 0));
  const float qn = (qnorm2 && qv) ? qnorm2[col] : 0.f;
  const uint64_t below = (lane == 0) ? 0ull : (~0ull >> (64 - lane));
  int cnt[2] = {0, 0};                // this wave's queries w, w + 8 (wave-uniform)
  uint32_t thr[2] = {0u, 0u};
  for (int s0 = lo; s0 < hi; s0 += KS_SUB) {
    const int s1 = min(hi, s0 + KS_SUB), len = s1 - s0;
    const int ngroups = (len + 15) / 16;
    for (int grp = w; grp < ngroups; grp += 8) {
      const int r0 = s0 + grp * 16;
      const int r = min(r0 + col, s1 - 1);
      const uint16_t* xr = X + (size_t)r * D;
      uint4 a[KC];
#pragma unroll
      for (int c = 0; c < KC; ++c) a[c] = *reinterpret_cast<const uint4*>(xr + 32 * c + 8 * g);
      f32x4_t acc = {0.f, 0.f, 0.f, 0.f};
#pragma unroll
      for (int c = 0; c < KC; ++c) acc = __builtin_amdgcn_mfma_f32_16x16x32_bf16(as_bf16x8(a[c]), qf[c], acc, 0, 0, 0);
      if (qv) {
#pragma unroll
        for (int i = 0; i < 4; ++i) {
          const int row = r0 + 4 * g + i;
          if (row < s1) {
            float v = acc[i];
            if (xnorm2) v = -(xnorm2[row] + qn - 2.f * v);
            if (alive && !alive[row]) v = -INFINITY;
            sc[col * KS_SUB + (row - s0)] = v;
          }
        }
      }
    }
    __syncthreads();
#pragma unroll
    for (int t = 0; t < 2; ++t) {
      const int qi = w + 8 * t;
      if (qi < nq) {
        uint32_t* qk = bk + qi * KS_CAP;
        uint32_t* qr = br + qi * KS_CAP;
#pragma unroll
        for (int j = 0; j < KS_SUB / 64; ++j) {
          const int i = lane + 64 * j;
          const uint32_t key = i < len ? f2key(sc[qi * KS_SUB + i]) : 0u;
          const bool p = i < len && key > thr[t];
          const uint64_t b = __ballot(p);
          if (p) {
            const int slot = cnt[t] + __popcll(b & below);
            qk[slot] = key;
            qr[slot] = (uint32_t)(s0 - lo + i);
          }
          cnt[t] += __popcll(b);
        }
        if (cnt[t] > KS_CAP - KS_SUB) {        // the next sub-chunk might not fit: cut to k (k <= 256)
          thr[t] = ks_cut(qk, qr, cnt[t], k);
          cnt[t] = k;
        }
      }
    }
    __syncthreads();                              // sc is the next sub-chunk's
  }
#pragma unroll
  for (int t = 0; t < 2; ++t) {
    const int qi = w + 8 * t;
    if (qi < nq) {
      uint32_t* qk = bk + qi * KS_CAP;
      uint32_t* qr = br + qi * KS_CAP;
      int n = cnt[t];
      if (n > k) {
        ks_cut(qk, qr, n, k);
        n = k;
      }
      const size_t o = ((size_t)qi * gridDim.x + blockIdx.x) * k;
      for (int s2 = lane; s2 < k; s2 += 64) {
        out_v[o + s2] = s2 < n ? key2f(qk[s2]) : -INFINITY;
        out_i[o + s2] = s2 < n ? (int64_t)lo + qr[s2] : -1;
      }
    }
  }
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

namespace {
// rows per flat-scan workgroup for nq queries and top-k: the [nq][ROWS] fp32 score tile stays at
// <= 16-32 KB of LDS (several workgroups per CU overlap one chunk's select with the others' scans),
// and for a large k the chunk grows so the k candidates it emits stay a small share of its rows
// (the candidate arrays are written and merged: k = 150 from 256-row chunks is 59 % of the index).
// Measured on 100M x 384: 1 query 2048 rows 12.6 ms (6.1 TB/s) vs 1024 rows 14.1 ms; 16 queries
// 256 rows 14.1 ms vs 1024 rows 23.6 ms (k = 10), 512 rows 20.7 ms vs 256 rows 22.8 ms (k = 150).
// k > 32 and more than 4 queries: the streamed kernel, k candidates per KS_SPAN rows (up to 4
// queries the 2048-row chunks already keep k = 150 at 7 % of the rows, and the streamed kernel's two
// workgroups per CU scan slower: 1 query, k = 150: 14.8 ms vs 12.6, profiles/r04_bench_knn_*).
constexpr int knn_flat_rows(int nq, int k) {
  return nq <= 4 ? 2048 : k > 32 ? KS_SPAN : nq <= 8 ? 512 : 256;
}

template <int KC>
int knn_topk_launch(const void* X, const void* Q, int N, int nq, const float* xnorm2, const float* qnorm2,
                    const uint8_t* alive, int k, int row_lo, const int32_t* probe, int nprobe, int maxc,
                    const int64_t* list_off, int nslots, float* out_v, int64_t* out_i, int blocks, int nqb,
                    int rows, hipStream_t stream) {
  const size_t lds = (size_t)nqb * rows * 4 + 4 * 256 * 4;
#define KTL(R) knn_topk_kernel<KC, R><<<blocks, 256, lds, stream>>>((const uint16_t*)X, (const uint16_t*)Q, N, nq, \
      xnorm2, qnorm2, alive, k, row_lo, probe, nprobe, maxc, list_off, nslots, out_v, out_i)
  switch (rows) {
    case 2048: KTL(2048); break;
    case 1024: KTL(1024); break;
    case 512: KTL(512); break;
    case 256: KTL(256); break;
    default: return -3;
  }
#undef KTL
  return CFC_CHECK_LAUNCH();
}

int knn_topk_dispatch(int dim, const void* X, const void* Q, int N, int nq, const float* xnorm2, const float* qnorm2,
                      const uint8_t* alive, int k, int row_lo, const int32_t* probe, int nprobe, int maxc,
                      const int64_t* list_off, int nslots, float* out_v, int64_t* out_i, int blocks, int nqb,
                      int rows, hipStream_t stream) {
#define KT(KC) return knn_topk_launch<KC>(X, Q, N, nq, xnorm2, qnorm2, alive, k, row_lo, probe, nprobe, maxc, \
                                          list_off, nslots, out_v, out_i, blocks, nqb, rows, stream)
  switch (dim / 32) {
    case 4: KT(4);
    case 8: KT(8);
    case 12: KT(12);
    case 16: KT(16);
    case 24: KT(24);
    case 32: KT(32);
    default: return -2;
  }
#undef KT
}
}  // namespace

// Flat index, rows [row_lo, N): candidates out [nq][ceil((N - row_lo) / cfc_knn_flat_rows(nq, k))][k]
// (unsorted within a chunk; merge with cfc_topk_pass).  nq <= 16, k <= 256; alive: optional uint8 row mask.
CFC_API int cfc_knn_topk(const void* X, const void* Q, int N, int row_lo, int nq, int dim, const float* xnorm2,
                         const float* qnorm2, const uint8_t* alive, int k, float* out_v, int64_t* out_i,
                         hipStream_t stream) {
  if (nq < 1 || nq > 16 || dim % 32 != 0 || N <= row_lo || row_lo < 0 || k < 1 || k > 256) return -1;
  const int rows = knn_flat_rows(nq, k);
  const int nch = (N - row_lo + rows - 1) / rows;
  if (rows == KS_SPAN) {
#define KS(KC) \
  case KC: \
    knn_topk_stream_kernel<KC><<<nch, 512, 0, stream>>>((const uint16_t*)X, (const uint16_t*)Q, N, nq, xnorm2, qnorm2, \
                                                       alive, k, row_lo, out_v, out_i); \
    return CFC_CHECK_LAUNCH();
    switch (dim / 32) {
      KS(4) KS(8) KS(12) KS(16) KS(24) KS(32)
      default: return -2;
    }
#undef KS
  }
  return knn_topk_dispatch(dim, X, Q, N, nq, xnorm2, qnorm2, alive, k, row_lo, nullptr, 1, 1, nullptr, nch, out_v,
                           out_i, nch, nq, rows, stream);
}

// rows per IVF list chunk (one workgroup each)
CFC_API int cfc_knn_topk_rows() { return KT_ROWS; }
// rows per flat-scan workgroup for nq queries and top-k (the candidate count of cfc_knn_topk)
CFC_API int cfc_knn_flat_rows(int nq, int k) { return knn_flat_rows(nq, k); }

// IVF: probe [nq][nprobe] list ids, list_off [nlist + 1] row offsets (rows grouped by list), maxc =
// max chunks of any list.  One launch of nq * nprobe * maxc workgroups; candidates out
// [nq][nprobe * maxc][k].
CFC_API int cfc_ivf_topk(const void* X, const void* Q, int N, int nq, int dim, const float* xnorm2,
                         const float* qnorm2, const uint8_t* alive, const int32_t* probe, int nprobe,
                         const int64_t* list_off, int maxc, int k, float* out_v, int64_t* out_i, hipStream_t stream) {
  if (nq < 1 || nprobe < 1 || maxc < 1 || dim % 32 != 0 || k < 1 || k > 256) return -1;
  const long blocks = (long)nq * nprobe * maxc;
  if (blocks > (1L << 30)) return -1;
  return knn_topk_dispatch(dim, X, Q, N, nq, xnorm2, qnorm2, alive, k, 0, probe, nprobe, maxc, list_off,
                           nprobe * maxc, out_v, out_i, (int)blocks, 1, KT_ROWS, stream);
}
