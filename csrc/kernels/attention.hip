// Attention kernels for gfx950 (CDNA4), bf16 in / fp32 accumulate on MFMA 16x16x32.
//
//   * paged decode attention (GQA, split-K over context partitions + LSE combine)
//   * varlen causal prefill attention over the paged KV cache (flash-style online softmax)
//   * varlen bidirectional encoder attention (BERT / MiniLM / BGE, head_dim 32 or 64)
//
// They replace the attention inside the engines the reference drives over HTTP
// (Ollama /api/generate: local_llm_summarizer.py:107; llama.cpp /completion:
// llamacpp_summarizer.py:108) and inside SentenceTransformer.encode
// (sentence_transformer_provider.py:93).  The reference itself has no kernels.
//
// Layout decisions (MI355X-first, not a CUDA translation):
//   * "Swapped" products: S^T = K . Q^T and O^T = V^T . P^T.  With the 16x16x32 C/D map
//     (col = lane&15, row = 4*(lane>>4)+i) every lane then owns ONE query column, so the
//     online-softmax max/sum are lane-local plus two xor-shuffles, and the S^T accumulator is
//     already the P^T B-operand of the next MFMA (guide §3 "accumulator as the next operand").
//   * KV cache block = 32 tokens = one MFMA k-step.  K is stored [blk][kvh][32][D] (row = key),
//     V is stored TRANSPOSED in slot groups, [blk][kvh][4 groups g][D][8] (common.h kv_v_off), with
//     the keys of each block permuted so that slot 8g+j holds key perm(g,j) = (j<4 ? 4g+j : 16+4g+j-4).
//     That is exactly the key order a lane holds in its S^T registers, so the V^T A-operand is one
//     contiguous 16-byte load per lane (no LDS transpose, no ds_read_tr needed) in both decode
//     (straight from HBM) and prefill; and one decode token's V column dirties 16 cache lines
//     ([D][32] rows: 64), which is what its write costs the step.
//   * LDS tiles are XOR-swizzled for conflict-free ds_read_b128 (guide §5.5 T2); the swizzles
//     were derived against the gfx950 ds_read_b128 lane groups {0-3,12-15,20-27}, ...
#include "common.h"
#include <stdlib.h>

namespace {

constexpr int KV_BS = 32;          // tokens per KV-cache block
constexpr float LOG2E = 1.4426950408889634f;

__device__ __forceinline__ bf16x8_t as_bf16x8(uint4 v) { return __builtin_bit_cast(bf16x8_t, v); }

__device__ __forceinline__ f32x4_t mfma16(bf16x8_t a, bf16x8_t b, f32x4_t c) {
  return __builtin_amdgcn_mfma_f32_16x16x32_bf16(a, b, c, 0, 0, 0);
}

// P^T fragment for keys [32ks, 32ks+32): {p[2ks][0..3], p[2ks+1][0..3]} as bf16.
__device__ __forceinline__ bf16x8_t pack_p(const f32x4_t& a, const f32x4_t& b) {
  uint4 u;
  u.x = pack2bf(a[0], a[1]); u.y = pack2bf(a[2], a[3]);
  u.z = pack2bf(b[0], b[1]); u.w = pack2bf(b[2], b[3]);
  return as_bf16x8(u);
}

// ------------------------------------------------------------------------------------------
// Paged decode attention.
// grid = (P partitions, Hkv, B); block = 256 (4 waves).  Each wave walks the partition's KV
// blocks with stride 4, K/V fragments straight from HBM into VGPRs (guide: "GEMV / M<=16 decode:
// load straight to VGPRs"), next block prefetched while the current one is in the MFMAs.
// The G = Hq/Hkv query heads of the kv-head share every K/V byte (GQA packing: the G heads are
// the MFMA's B columns).
// ------------------------------------------------------------------------------------------
typedef unsigned int u32x4_t __attribute__((ext_vector_type(4)));

// 16-byte KV load; NT = non-temporal (streamed once per step: keep it out of the caches' LRU so the
// shared-prefix blocks and the weights stay resident)
template <bool NT>
__device__ __forceinline__ uint4 kv_load(const uint16_t* p) {
  if constexpr (NT) {
    const u32x4_t v = __builtin_nontemporal_load(reinterpret_cast<const u32x4_t*>(p));
    return make_uint4(v.x, v.y, v.z, v.w);
  } else {
    return *reinterpret_cast<const uint4*>(p);
  }
}

typedef unsigned int u32x2_t __attribute__((ext_vector_type(2)));

// 8-byte load of 8 fp8 KV values (the FP8 cache's fragment)
template <bool NT>
__device__ __forceinline__ uint2 kv_load8(const uint8_t* p) {
  if constexpr (NT) {
    const u32x2_t v = __builtin_nontemporal_load(reinterpret_cast<const u32x2_t*>(p));
    return make_uint2(v.x, v.y);
  } else {
    return *reinterpret_cast<const uint2*>(p);
  }
}

// Raw KV fragment as loaded (bf16: 16 B; fp8: 8 B) and its bf16x8 MFMA operand.  The fp8 ->
// bf16 conversion happens at the MFMA, so a prefetched block's loads stay in flight.
template <bool F8> struct KvFrag { typedef uint4 raw; };
template <> struct KvFrag<true> { typedef uint2 raw; };
__device__ __forceinline__ bf16x8_t kv_operand(uint4 r) { return as_bf16x8(r); }
__device__ __forceinline__ bf16x8_t kv_operand(uint2 r) { return as_bf16x8(fp8x8_to_bf16x8(r)); }

// ROPE: the decode step's RoPE + KV write happens in the prologue (DecRope below): every workgroup
// ropes the G query heads it needs straight from the qkv projection output (bf16, or the decode
// GEMM's fp32 split-K slabs) into LDS, and the workgroup whose KV range holds the sequence's last
// block writes the new key / value into the cache first -- the separate rope_kv launch, its q
// round trip through HBM and its dependency edge disappear.  Same helpers (common.h) as
// rope_kv_kernel, so the cache bytes and q values are identical to the two-kernel path.
// Workgroup barrier that orders LDS only: global loads and stores issued before it stay in flight
// (__syncthreads waits for every outstanding vector-memory operation first).
__device__ __forceinline__ void lds_barrier() {
  __builtin_amdgcn_fence(__ATOMIC_RELEASE, "workgroup", "local");
  __builtin_amdgcn_s_barrier();
  __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "workgroup", "local");
}

// Element e (0..7) of a bf16x8 fragment replaced by the bf16 bits h (register selects, no scratch).
__device__ __forceinline__ uint4 set_bf16(uint4 v, int e, uint32_t h) {
  const int wi = e >> 1;
  const bool hi = e & 1;
  auto put = [&](uint32_t x, int i) -> uint32_t {
    return i != wi ? x : hi ? ((x & 0xffffu) | (h << 16)) : ((x & 0xffff0000u) | h);
  };
  return make_uint4(put(v.x, 0), put(v.y, 1), put(v.z, 2), put(v.w, 3));
}

struct DecRope {
  const uint16_t* qkv;     // [B, (Hq + 2 Hkv) D] bf16, or nullptr with part
  const float* part;       // [split, B, (Hq + 2 Hkv) D] fp32 split-K slabs
  int split;
  const int32_t* positions;
  const int32_t* slots;    // -1: no cache write
  const float* cos_sin;
  float inv_k, inv_v;
  int probe;               // timing ablations only (cfc_set_decode_rope_probe); 0 in production
};

// One KV block's K fragments (bf16: 8 x 16 B per lane; fp8: 4 x 16 B) and V^T fragments (8) of
// kv-head block `base` (elements), loaded nontemporal (NT) or through the caches.
template <bool NT, bool F8>
__device__ __forceinline__ void dec_load_blk(const void* kc, const void* vc, size_t base, int col, int g, uint4* kk,
                                             typename KvFrag<F8>::raw* vv) {
  constexpr int D = 128;
  if constexpr (F8) {
    const uint8_t* kb = reinterpret_cast<const uint8_t*>(kc) + base;
#pragma unroll
    for (int st = 0; st < 2; ++st)
#pragma unroll
      for (int pp = 0; pp < 2; ++pp)
        kk[st * 2 + pp] = kv_load<NT>(reinterpret_cast<const uint16_t*>(kb + (16 * st + col) * D + 64 * pp + 16 * g));
#pragma unroll
    for (int dt = 0; dt < 8; ++dt)
      vv[dt] = kv_load8<NT>(reinterpret_cast<const uint8_t*>(vc) + base + kv_v_off(16 * dt + col, 8 * g, D));
  } else {
#pragma unroll
    for (int st = 0; st < 2; ++st)
#pragma unroll
      for (int c = 0; c < 4; ++c)
        kk[st * 4 + c] = kv_load<NT>(reinterpret_cast<const uint16_t*>(kc) + base + (16 * st + col) * D + 32 * c + 8 * g);
#pragma unroll
    for (int dt = 0; dt < 8; ++dt)
      vv[dt] = kv_load<NT>(reinterpret_cast<const uint16_t*>(vc) + base + kv_v_off(16 * dt + col, 8 * g, D));
  }
}

// NT: the KV stream is read nontemporal (each block once per step, kept out of the caches' LRU) --
// except the first *shared_blocks blocks of every sequence (shared_blocks: device int, may be null):
// the prefix-cache blocks that every sequence of the batch maps to the SAME physical blocks (system
// prompt + template head, ~10 blocks of a 2.9k-token context).  Those go through L2 / MALL, so the
// 128 sequences' reads of them cost one HBM read instead of 128.
template <int G, bool NT, bool F8 = false, bool ROPE = false>
__global__ void __launch_bounds__(256, F8 ? 2 : 1) paged_decode_kernel(
    const uint16_t* __restrict__ q, const void* __restrict__ kc, const void* __restrict__ vc,
    const int32_t* __restrict__ block_tables, const int32_t* __restrict__ ctx_lens, float scale_log2, int Hkv,
    int max_blocks, int part_blocks, int P, int window, float v_scale, float* __restrict__ part_o,
    float* __restrict__ part_ml, uint16_t* __restrict__ out, DecRope rp, const int32_t* __restrict__ shared_blocks) {
  // F8: kc / vc hold e4m3 of K / k_scale and V / v_scale; k_scale is folded into scale_log2 by the
  // host, v_scale multiplies the output here
  typedef typename KvFrag<F8>::raw Raw;
  constexpr int D = 128;
  const int p = blockIdx.x, h = blockIdx.y, b = blockIdx.z;
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
  const int col = lane & 15, g = lane >> 4;
  const int Hq = Hkv * G;
  const int ctx = ctx_lens[b];
  const int nblk = (ctx + KV_BS - 1) / KV_BS;
  // sliding window (window > 0): the query at position ctx-1 sees keys [ctx - window, ctx)
  const int key_lo = window > 0 ? max(0, ctx - window) : 0;
  const int blk_lo = key_lo / KV_BS;
  // part_blocks > 0: fixed-size partitions of the block table; <= 0: the sequence's OWN blocks
  // split into P near-equal ranges (balanced per sequence whatever its length -- no nearly empty
  // tail partitions, and P can stay small, so each workgroup streams a long run of KV)
  const int blk0 = part_blocks > 0 ? max(blk_lo, p * part_blocks)
                                   : blk_lo + (int)(((int64_t)p * (nblk - blk_lo)) / P);
  const int blk1 = part_blocks > 0 ? min(nblk, p * part_blocks + part_blocks)
                                   : blk_lo + (int)(((int64_t)(p + 1) * (nblk - blk_lo)) / P);

  __shared__ float sm_o[4][D][17];
  __shared__ float sm_m[4][16], sm_l[4][16];

  // Q^T B-operand: lane holds Q[head h*G+col][dq(c) .. +7]; columns >= G are zero.  bf16 cache:
  // dq(c) = 32c + 8g.  FP8 cache: the head dim is visited in the order that lets ONE 16-byte load
  // carry two k-steps of a key row (64 contiguous bytes per row per wave instruction, as the bf16
  // loads have): dq(c) = 64(c >> 1) + 16g + 8(c & 1) -- any d order works as long as Q and K agree.
  __shared__ __attribute__((aligned(16))) uint16_t sm_q[ROPE ? G : 1][D];
  f32x4_t o[8];
#pragma unroll
  for (int i = 0; i < 8; ++i) o[i] = f32x4_t{0.f, 0.f, 0.f, 0.f};
  float m = -INFINITY, l = 0.f;

  const int32_t* bt = block_tables + (size_t)b * max_blocks;
  const size_t head_stride = (size_t)KV_BS * D;  // elements per (block, kv-head)

  // K fragments: bf16 -> 8 x 16 B (st, c); fp8 -> 4 x 16 B (st, pair p of k-steps 2p, 2p+1)
  constexpr int NK = F8 ? 4 : 8;
  uint4 kr[NK];
  Raw vr[8];
  const int temporal = (NT && shared_blocks != nullptr) ? shared_blocks[0] : 0;   // blocks read cached
  auto load_blk = [&](int bi, uint4* kk, Raw* vv) {
    const size_t base = ((size_t)bt[bi] * Hkv + h) * head_stride;
    if (NT && bi >= temporal) dec_load_blk<NT, F8>(kc, vc, base, col, g, kk, vv);
    else dec_load_blk<false, F8>(kc, vc, base, col, g, kk, vv);
  };
  // K operand of (st, k-step c)
  auto kop = [&](const uint4* kk, int st, int c) -> bf16x8_t {
    if constexpr (F8) {
      const uint4 r = kk[st * 2 + (c >> 1)];
      return kv_operand((c & 1) ? make_uint2(r.z, r.w) : make_uint2(r.x, r.y));
    } else {
      return as_bf16x8(kk[st * 4 + c]);
    }
  };

  // ROPE, bf16 cache (PATCH): the new key / value make no round trip through memory inside the
  // step.  The prologue ropes q and k into LDS and writes the new key's cache row (256 contiguous
  // bytes, whole lines); the wave that streams the sequence's last block patches the new slot's K
  // and V into the fragments it loaded and stores the V^T slot group holding the new key back (16
  // full lines; the write costs the step by lines dirtied, scripts/probe_decode_rope_fused.py).
  // Every wave issues its first block before the prologue, so that block's HBM latency overlaps
  // the slab reads.  FP8 keeps the write-then-read order: the prologue writes K and V and the wave
  // whose first block receives them loads it after the barrier.
  constexpr bool PATCH = ROPE && !F8;
  __shared__ __attribute__((aligned(16))) uint16_t sm_kv[PATCH ? 2 : 1][PATCH ? D : 1];
  const int slot = ROPE ? rp.slots[b] : -1;
  const bool owner = ROPE && slot >= 0 && blk0 <= nblk - 1 && nblk - 1 < blk1;   // holds the new key's block
  int bi = blk0 + w;
  const bool early = ROPE && bi < blk1 && (PATCH || !(owner && bi == nblk - 1));
  if (early) load_blk(bi, kr, vr);
  if constexpr (ROPE) {
    constexpr int NV = D / 16;    // 8-vectors per half-head
    const size_t stride = (size_t)(Hq + 2 * Hkv) * D;
    const size_t row0 = (size_t)b * stride, slab = (size_t)gridDim.z * stride;
    const float* cs = rp.cos_sin + (size_t)rp.positions[b] * (D / 2) * 2;
    const int t = threadIdx.x;
    if (t < (G + 1) * NV) {
      const int hh = t / NV, c = t - hh * NV;   // hh < G: query head h*G + hh; hh == G: key head h
      if (hh < G || owner) {
        uint4 pa, pb;
        rope_rot8(rp.qkv, rp.part, rp.split, slab, row0 + (size_t)(hh < G ? h * G + hh : Hq + h) * D, D / 2, c, cs,
                  pa, pb);
        if (hh < G) {
          *reinterpret_cast<uint4*>(&sm_q[hh][c * 8]) = pa;
          *reinterpret_cast<uint4*>(&sm_q[hh][D / 2 + c * 8]) = pb;
        } else {
          if (!(rp.probe & 1)) kv_write_k<F8>(const_cast<void*>(kc), slot, h, Hkv, D, c, pa, pb, rp.inv_k);
          if constexpr (PATCH) {
            *reinterpret_cast<uint4*>(&sm_kv[0][c * 8]) = pa;
            *reinterpret_cast<uint4*>(&sm_kv[0][D / 2 + c * 8]) = pb;
          }
        }
      }
    } else if (owner && t < (G + 1) * NV + D / 8) {
      const int c = t - (G + 1) * NV;
      float vf[8];
      qkv_load8(rp.qkv, rp.part, rp.split, slab, row0 + (size_t)(Hq + Hkv + h) * D + c * 8, vf);
      if constexpr (PATCH) *reinterpret_cast<uint4*>(&sm_kv[1][c * 8]) = pack8(vf);
      else kv_write_v<F8>(const_cast<void*>(vc), slot, h, Hkv, D, c, pack8(vf), rp.inv_v);
    }
    // workgroup-scope release / acquire: sm_q / sm_kv to every wave and (FP8) the cache stores above
    // to this workgroup's KV loads below (same CU).  PATCH reads nothing back from memory, so its
    // barrier orders LDS only: the early KV loads and the key-row store stay in flight across it.
    if constexpr (PATCH) lds_barrier();
    else __syncthreads();
  }
  bf16x8_t qf[4];
  {
    const bool valid = col < G;
    const uint16_t* qr = ROPE ? &sm_q[valid ? col : 0][0] : q + ((size_t)b * Hq + h * G + (valid ? col : 0)) * D;
#pragma unroll
    for (int c = 0; c < 4; ++c) {
      const int dq = F8 ? 64 * (c >> 1) + 16 * g + 8 * (c & 1) : 32 * c + 8 * g;
      uint4 v = valid ? *reinterpret_cast<const uint4*>(qr + dq) : make_uint4(0, 0, 0, 0);
      qf[c] = as_bf16x8(v);
    }
  }

  if (bi < blk1 && !early) load_blk(bi, kr, vr);
  for (; bi < blk1; bi += 4) {
    uint4 kn[NK];
    Raw vn[8];
    const bool more = bi + 4 < blk1;
    if (more) load_blk(bi + 4, kn, vn);
    if constexpr (PATCH) {
      if (owner && bi == nblk - 1) {
        const int sn = slot % KV_BS;
        // K row sn: lanes col == sn % 16 of fragment half st = sn / 16 hold its d-chunks 32c + 8g
        if (col == (sn & 15)) {
#pragma unroll
          for (int st = 0; st < 2; ++st)
            if (st == (sn >> 4))
#pragma unroll
              for (int c = 0; c < 4; ++c) kr[st * 4 + c] = *reinterpret_cast<const uint4*>(&sm_kv[0][32 * c + 8 * g]);
        }
        // V^T column of key sn: stored at slot position ps = kv_v_slot(sn), i.e. element ps % 8 of
        // the lanes g == ps / 8 (rows d = 16 dt + col)
        const int ps = kv_v_slot(sn);
        if (g == (ps >> 3)) {
#pragma unroll
          for (int dt = 0; dt < 8; ++dt) vr[dt] = set_bf16(vr[dt], ps & 7, sm_kv[1][16 * dt + col]);
        }
        // the new key's slot group of the V^T tile back to the cache: the lanes g == ps / 8 store
        // their 8 x 16-byte pieces, the group's 16 full cache lines
        uint16_t* vt = reinterpret_cast<uint16_t*>(const_cast<void*>(vc)) + ((size_t)bt[bi] * Hkv + h) * head_stride;
        if (g != (ps >> 3)) {
        } else if (rp.probe & 4) {
#pragma unroll
          for (int dt = 0; dt < 8; ++dt) {
            const uint4 v = vr[dt];
            __builtin_nontemporal_store(u32x4_t{v.x, v.y, v.z, v.w},
                                        reinterpret_cast<u32x4_t*>(vt + kv_v_off(16 * dt + col, 8 * g, D)));
          }
        } else if (!(rp.probe & 2)) {
#pragma unroll
          for (int dt = 0; dt < 8; ++dt) *reinterpret_cast<uint4*>(vt + kv_v_off(16 * dt + col, 8 * g, D)) = vr[dt];
        }
      }
    }

    f32x4_t s[2];
#pragma unroll
    for (int st = 0; st < 2; ++st) {
      s[st] = f32x4_t{0.f, 0.f, 0.f, 0.f};
#pragma unroll
      for (int c = 0; c < 4; ++c) s[st] = mfma16(kop(kr, st, c), qf[c], s[st]);
    }
    const int key0 = bi * KV_BS;
    float tmax = -INFINITY;
#pragma unroll
    for (int st = 0; st < 2; ++st)
#pragma unroll
      for (int i = 0; i < 4; ++i) {
        const int key = key0 + 16 * st + 4 * g + i;
        float v = s[st][i] * scale_log2;
        v = key < ctx && key >= key_lo ? v : -INFINITY;
        s[st][i] = v;
        tmax = fmaxf(tmax, v);
      }
    tmax = xor16_max(tmax);
    tmax = xor32_max(tmax);
    const float mn = fmaxf(m, tmax);
    const float alpha = exp2f(m - mn);
    float rs = 0.f;
#pragma unroll
    for (int st = 0; st < 2; ++st)
#pragma unroll
      for (int i = 0; i < 4; ++i) { const float e = exp2f(s[st][i] - mn); s[st][i] = e; rs += e; }
    rs = xor16_sum(rs);
    rs = xor32_sum(rs);
    l = l * alpha + rs;
    m = mn;
    const bf16x8_t pf = pack_p(s[0], s[1]);
#pragma unroll
    for (int dt = 0; dt < 8; ++dt) {
      o[dt] *= alpha;
      o[dt] = mfma16(kv_operand(vr[dt]), pf, o[dt]);
    }
    if (more) {
#pragma unroll
      for (int i = 0; i < 8; ++i) {
        if (i < NK) kr[i] = kn[i];
        vr[i] = vn[i];
      }
    }
  }

  // Combine the 4 waves through LDS.  Lane (col, g) holds O^T[d = 16dt + 4g + i][col].
#pragma unroll
  for (int dt = 0; dt < 8; ++dt)
#pragma unroll
    for (int i = 0; i < 4; ++i) sm_o[w][16 * dt + 4 * g + i][col] = o[dt][i];
  if (g == 0) { sm_m[w][col] = m; sm_l[w][col] = l; }
  // PATCH: the V^T tile store of the last block stays in flight (a full barrier would wait for its
  // write acknowledgement here, once per workgroup, behind the chip-wide KV read stream)
  if constexpr (PATCH) lds_barrier();
  else __syncthreads();

  for (int idx = threadIdx.x; idx < G * D; idx += 256) {
    const int qh = idx / D, d = idx % D;
    float M = -INFINITY;
#pragma unroll
    for (int ww = 0; ww < 4; ++ww) M = fmaxf(M, sm_m[ww][qh]);
    float L = 0.f, O = 0.f;
    if (M != -INFINITY) {
#pragma unroll
      for (int ww = 0; ww < 4; ++ww) {
        const float f = exp2f(sm_m[ww][qh] - M);
        L += sm_l[ww][qh] * f;
        O += sm_o[ww][d][qh] * f;
      }
    }
    const int head = h * G + qh;
    O *= v_scale;
    if (P == 1) {
      out[((size_t)b * Hq + head) * D + d] = f2bf(L > 0.f ? O / L : 0.f);
    } else {
      const size_t pi = ((size_t)b * Hq + head) * P + p;
      part_o[pi * D + d] = O;
      if (d == 0) { part_ml[pi * 2] = M; part_ml[pi * 2 + 1] = L; }
    }
  }
}

// grid = (Hq, B), block = 128: merge the P partition results of one (seq, head).
__global__ void __launch_bounds__(128) decode_combine_kernel(const float* __restrict__ part_o,
                                                             const float* __restrict__ part_ml, int P, int Hq,
                                                             uint16_t* __restrict__ out) {
  // Small-batch decode runs with up to ~64 partitions per head: the (m, l) pairs are loaded by all
  // 128 threads at once and the weights exp2(m_p - M) / L go through LDS, so the only per-thread
  // loop is P independent part_o loads (unrolled) instead of three dependent P-long chains.
  constexpr int D = 128, PMAX = 256;
  __shared__ float wsh[PMAX];
  __shared__ float red[2];
  const int head = blockIdx.x, b = blockIdx.y, d = threadIdx.x;
  const size_t base = ((size_t)b * Hq + head) * P;
  const int lane = d & 63, wid = d >> 6;
  float O = 0.f, Ltot = 0.f, Mrun = -INFINITY;
  for (int p0 = 0; p0 < P; p0 += PMAX) {   // one pass for P <= 256
    const int np = min(PMAX, P - p0);
    float mloc = -INFINITY;
    for (int i = d; i < np; i += 128) mloc = fmaxf(mloc, part_ml[(base + p0 + i) * 2]);
    mloc = wave_max(mloc);
    if (lane == 0) red[wid] = mloc;
    __syncthreads();
    const float M = fmaxf(red[0], red[1]);
    __syncthreads();
    float lsum = 0.f;
    for (int i = d; i < np; i += 128) {
      const float mp = part_ml[(base + p0 + i) * 2];
      const float f = (M == -INFINITY || mp == -INFINITY) ? 0.f : exp2f(mp - M);
      wsh[i] = f;
      lsum += part_ml[(base + p0 + i) * 2 + 1] * f;
    }
    lsum = wave_sum(lsum);
    if (lane == 0) red[wid] = lsum;
    __syncthreads();
    const float L = red[0] + red[1];
    float o = 0.f;
#pragma unroll 8
    for (int i = 0; i < np; ++i) o += part_o[(base + p0 + i) * D + d] * wsh[i];
    __syncthreads();
    // merge this pass into the running (O, L, Mrun); every thread holds the same M, L
    if (p0 == 0) {
      O = o; Ltot = L; Mrun = M;
    } else {
      const float Mn = fmaxf(Mrun, M);
      const float a = Mrun == -INFINITY ? 0.f : exp2f(Mrun - Mn), c = M == -INFINITY ? 0.f : exp2f(M - Mn);
      O = O * a + o * c; Ltot = Ltot * a + L * c; Mrun = Mn;
    }
  }
  out[((size_t)b * Hq + head) * D + d] = f2bf(Ltot > 0.f ? O / Ltot : 0.f);
}

// ------------------------------------------------------------------------------------------
// Varlen causal prefill over the paged cache (D = 128).
// grid = (n_tiles, Hq); block = 512 = 8 waves x 16 query rows = 128-row query tile.
// Tile t covers query rows [tile_q0[t], +128) of sequence tile_seq[t]; those rows sit at
// positions ctx - q_len + row (chunked prefill / prefix reuse: keys come from the cache).
//   * K tile (64 keys x 128) and V^T tile (2 blocks x 128 x 32) double-buffered in LDS and shared
//     by all 8 waves; register-staged (next tile's loads issue before this tile's MFMAs, LDS
//     writes after -- guide §5.5 T14); one barrier per tile.
//   * <= 128 VGPRs so two workgroups (16 waves, 4 per SIMD) share a CU: one wave's softmax VALU
//     overlaps another's MFMAs (a 1-wave-per-SIMD build of this loop was VALU-serialised).
//   * VALU trimmed: Q is pre-scaled by softmax_scale*log2(e) once (scores come out of the MFMA
//     in the exp2 domain), the causal mask is applied only on tiles that cross the diagonal, and
//     the O rescale is deferred until the running max grows by > RESCALE_THR (guide T13; P is
//     then bounded by 2^THR, exact after the final 1/l).
//   * The host orders tiles heaviest-first (most keys) so the causal triangle drains evenly.
// ------------------------------------------------------------------------------------------
constexpr int PF_KT = 64;     // keys per tile
#ifndef CFC_PF_QK_PIPE
#define CFC_PF_QK_PIPE 1
#endif
constexpr int PF_QK_PIPE = CFC_PF_QK_PIPE;
#ifndef CFC_PF_V_EARLY
#define CFC_PF_V_EARLY 1
#endif
constexpr int PF_V_EARLY = CFC_PF_V_EARLY;   // prefill v5: V fragments of the first PF_V_EARLY half-tiles read before the softmax (2: 251 VGPRs, 1 % slower, profiles/r05_ab_prefill_attn_vearly2_rejected.log)
   // prefill v5: K fragments of a half-tile read ahead of its MFMAs
constexpr int PF_WAVES = 8;
constexpr int PF_ROWS = 16 * PF_WAVES;
constexpr float RESCALE_THR = 8.0f;

__device__ __forceinline__ int k_lds_off(int row, int ch) { return row * 256 + ((ch ^ (row & 15)) << 4); }
__device__ __forceinline__ int v_lds_off(int blk, int d, int ch) {
  return blk * 128 * 64 + d * 64 + ((ch ^ (((d >> 3) & 1) << 1)) << 4);
}

template <int MINW>
__global__ void __launch_bounds__(512, MINW) prefill_paged_kernel(
    const uint16_t* __restrict__ q, const uint16_t* __restrict__ kc, const uint16_t* __restrict__ vc,
    const int32_t* __restrict__ block_tables, const int32_t* __restrict__ cu_q, const int32_t* __restrict__ ctx_lens,
    const int32_t* __restrict__ tile_seq, const int32_t* __restrict__ tile_q0, float scale_log2, int Hq, int Hkv,
    int max_blocks, uint16_t* __restrict__ out) {
  constexpr int D = 128;
  extern __shared__ __attribute__((aligned(16))) char smem[];
  // LDS: [K buf0 16K][K buf1 16K][V buf0 16K][V buf1 16K]
  const int t = blockIdx.x, hq = blockIdx.y;
  const int G = Hq / Hkv, hk = hq / G;
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6, tid = threadIdx.x;
  const int col = lane & 15, g = lane >> 4;
  const int s = tile_seq[t], qs = tile_q0[t];
  const int q_begin = cu_q[s], q_len = cu_q[s + 1] - q_begin;
  const int ctx = ctx_lens[s];
  const int pos_base = ctx - q_len;
  const int row_last = min(qs + PF_ROWS - 1, q_len - 1);
  const int kend = pos_base + row_last + 1;  // keys [0, kend) are needed by this tile
  const int ntiles = (kend + PF_KT - 1) / PF_KT;
  const int32_t* bt = block_tables + (size_t)s * max_blocks;

  const int my_row = qs + 16 * w + col;
  const int my_pos = pos_base + my_row;
  const int wave_min_pos = pos_base + qs + 16 * w;
  bf16x8_t qf[4];
  {
    const int rr = min(my_row, q_len - 1);
    const uint16_t* qr = q + ((size_t)(q_begin + rr) * Hq + hq) * D;
#pragma unroll
    for (int c = 0; c < 4; ++c) {
      float f[8];
      unpack8(*reinterpret_cast<const uint4*>(qr + 32 * c + 8 * g), f);
#pragma unroll
      for (int j = 0; j < 8; ++j) f[j] *= scale_log2;
      qf[c] = as_bf16x8(pack8(f));
    }
  }

  uint4 kst[2], vst[2];
  auto gload = [&](int kt) {
#pragma unroll
    for (int i = 0; i < 2; ++i) {
      const int id = tid + 512 * i;
      {  // K: row = id>>4 (key within tile), ch = id&15
        const int row = id >> 4, ch = id & 15, key = kt * PF_KT + row;
        if (key < kend) {
          const int blk = bt[key / KV_BS];
          kst[i] = *reinterpret_cast<const uint4*>(kc + (((size_t)blk * Hkv + hk) * KV_BS + (key % KV_BS)) * D + ch * 8);
        } else {
          kst[i] = make_uint4(0, 0, 0, 0);
        }
      }
      {  // V^T: blk_i = id>>9, d = (id>>2)&127, ch = id&3
        const int bi = id >> 9, d = (id >> 2) & 127, ch = id & 3;
        const int key0 = kt * PF_KT + bi * KV_BS;
        if (key0 < kend) {
          const int blk = bt[key0 / KV_BS];
          vst[i] = *reinterpret_cast<const uint4*>(vc + ((size_t)blk * Hkv + hk) * D * KV_BS + kv_v_off(d, 8 * ch, D));
        } else {
          vst[i] = make_uint4(0, 0, 0, 0);
        }
      }
    }
  };
  auto lwrite = [&](int buf) {
#pragma unroll
    for (int i = 0; i < 2; ++i) {
      const int id = tid + 512 * i;
      *reinterpret_cast<uint4*>(smem + buf * 16384 + k_lds_off(id >> 4, id & 15)) = kst[i];
      *reinterpret_cast<uint4*>(smem + 32768 + buf * 16384 + v_lds_off(id >> 9, (id >> 2) & 127, id & 3)) = vst[i];
    }
  };

  f32x4_t o[8];
#pragma unroll
  for (int i = 0; i < 8; ++i) o[i] = f32x4_t{0.f, 0.f, 0.f, 0.f};
  float m = -INFINITY, l = 0.f;

  gload(0);
  lwrite(0);
  __syncthreads();
  for (int kt = 0; kt < ntiles; ++kt) {
    const int cur = kt & 1;
    const bool more = kt + 1 < ntiles;
    if (more) gload(kt + 1);

    const char* kb = smem + cur * 16384;
    const char* vb = smem + 32768 + cur * 16384;
    const int key0 = kt * PF_KT;
    // tiles wholly above this wave's rows (possible only in the last tiles): skip the math
    if (key0 <= wave_min_pos + 15) {
      f32x4_t sc[4];
#pragma unroll
      for (int st = 0; st < 4; ++st) {
        sc[st] = f32x4_t{0.f, 0.f, 0.f, 0.f};
        const int row = 16 * st + col;
#pragma unroll
        for (int c = 0; c < 4; ++c)
          sc[st] = mfma16(as_bf16x8(*reinterpret_cast<const uint4*>(kb + k_lds_off(row, 4 * c + g))), qf[c], sc[st]);
      }
      if (key0 + PF_KT - 1 > wave_min_pos) {  // diagonal tile: causal mask
#pragma unroll
        for (int st = 0; st < 4; ++st)
#pragma unroll
          for (int i = 0; i < 4; ++i)
            if (key0 + 16 * st + 4 * g + i > my_pos) sc[st][i] = -INFINITY;
      }
      float tmax = fmaxf(fmaxf(fmaxf(sc[0][0], sc[0][1]), fmaxf(sc[0][2], sc[0][3])),
                         fmaxf(fmaxf(sc[1][0], sc[1][1]), fmaxf(sc[1][2], sc[1][3])));
      tmax = fmaxf(tmax, fmaxf(fmaxf(fmaxf(sc[2][0], sc[2][1]), fmaxf(sc[2][2], sc[2][3])),
                               fmaxf(fmaxf(sc[3][0], sc[3][1]), fmaxf(sc[3][2], sc[3][3]))));
      tmax = xor16_max(tmax);
      tmax = xor32_max(tmax);
      // deferred rescale: keep the old max unless some row of the wave grew by > THR
      if (!__all(tmax - m <= RESCALE_THR)) {
        const float mn = fmaxf(m, tmax);
        const float mref = mn == -INFINITY ? 0.f : mn;
        const float alpha = exp2f(m - mref);
        l *= alpha;
#pragma unroll
        for (int dt = 0; dt < 8; ++dt) o[dt] *= alpha;
        m = mn;
      }
      const float mref = m == -INFINITY ? 0.f : m;
      float rs = 0.f;
#pragma unroll
      for (int st = 0; st < 4; ++st)
#pragma unroll
        for (int i = 0; i < 4; ++i) { const float e = exp2f(sc[st][i] - mref); sc[st][i] = e; rs += e; }
      rs = xor16_sum(rs);
      rs = xor32_sum(rs);
      l += rs;
#pragma unroll
      for (int ks = 0; ks < 2; ++ks) {
        const bf16x8_t pf = pack_p(sc[2 * ks], sc[2 * ks + 1]);
#pragma unroll
        for (int dt = 0; dt < 8; ++dt)
          o[dt] = mfma16(as_bf16x8(*reinterpret_cast<const uint4*>(vb + v_lds_off(ks, 16 * dt + col, g))), pf, o[dt]);
      }
    }
    if (more) lwrite(cur ^ 1);
    __syncthreads();
  }

  if (my_row < q_len) {
    const float inv = l > 0.f ? 1.f / l : 0.f;
    uint16_t* orow = out + ((size_t)(q_begin + my_row) * Hq + hq) * D;
#pragma unroll
    for (int dt = 0; dt < 8; ++dt) {
      uint2 pk;
      pk.x = pack2bf(o[dt][0] * inv, o[dt][1] * inv);
      pk.y = pack2bf(o[dt][2] * inv, o[dt][3] * inv);
      *reinterpret_cast<uint2*>(orow + 16 * dt + 4 * g) = pk;
    }
  }
}

// ------------------------------------------------------------------------------------------
// Prefill v4: 4 waves x 32 query rows on v_mfma_f32_32x32x16_bf16 (128-row tiles, as v3).
//   * S^T = K . Q^T per 32-key half-tile: A = K rows from LDS, B = Q^T from registers (8 k-steps
//     over D = 128).  C/D of 32x32: col = lane & 31 (query), row = 8(i>>2) + 4(lane>>5) + (i&3)
//     (key), so each lane owns one query row's scores for 16 of every 32 keys (the other 16 in
//     lane ^ 32): row max / sum = 31 local ops + one xor-32 shuffle.
//   * O^T = V^T . P^T: the S^T accumulator IS the P^T B-operand (guide §3: k-step s of a 32-key
//     tile = registers 8s..8s+7, key order 16s + 8(j>>2) + 4h + (j&3)); the V^T LDS image stores
//     each d row's 64 keys in exactly that slot order, so the A fragment is one ds_read_b128.
//     The cache's V^T blocks are in the decode (16x16) slot order; the permutation to the 32x32
//     order is applied while writing the LDS image (two 8-byte stores per 16-byte load).
//   * K / V^T tiles (64 keys) double-buffered in LDS, register-staged (loads for tile t+1 issued
//     before tile t's MFMAs, LDS writes after), one barrier per tile; deferred rescale as in v3.
//   * vs v3 (16x16x32, 16 rows/wave): every LDS fragment byte now feeds twice the FLOPs.
// ------------------------------------------------------------------------------------------
__device__ __forceinline__ f32x16_t mfma32(bf16x8_t a, bf16x8_t b, f32x16_t c) {
  return __builtin_amdgcn_mfma_f32_32x32x16_bf16(a, b, c, 0, 0, 0);
}

// V^T image: row d (64 keys = 128 B), 16-byte chunk c at d*128 + ((c ^ (d & 7)) << 4)
__device__ __forceinline__ int v4_off(int d, int c) { return d * 128 + ((c ^ (d & 7)) << 4); }

template <int MINW>
__global__ void __launch_bounds__(256, MINW) prefill_paged_kernel_v4(
    const uint16_t* __restrict__ q, const uint16_t* __restrict__ kc, const uint16_t* __restrict__ vc,
    const int32_t* __restrict__ block_tables, const int32_t* __restrict__ cu_q, const int32_t* __restrict__ ctx_lens,
    const int32_t* __restrict__ tile_seq, const int32_t* __restrict__ tile_q0, float scale_log2, int Hq, int Hkv,
    int max_blocks, uint16_t* __restrict__ out) {
  constexpr int D = 128;
  extern __shared__ __attribute__((aligned(16))) char smem[];
  // LDS: [K buf0 16K][K buf1 16K][V buf0 16K][V buf1 16K]
  const int t = blockIdx.x, hq = blockIdx.y;
  const int G = Hq / Hkv, hk = hq / G;
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6, tid = threadIdx.x;
  const int l32 = lane & 31, hi = lane >> 5;
  const int s = tile_seq[t], qs = tile_q0[t];
  const int q_begin = cu_q[s], q_len = cu_q[s + 1] - q_begin;
  const int ctx = ctx_lens[s];
  const int pos_base = ctx - q_len;
  const int row_last = min(qs + PF_ROWS - 1, q_len - 1);
  const int kend = pos_base + row_last + 1;
  const int ntiles = (kend + PF_KT - 1) / PF_KT;
  const int32_t* bt = block_tables + (size_t)s * max_blocks;

  const int my_row = qs + 32 * w + l32;
  const int my_pos = pos_base + my_row;
  const int wave_min_pos = pos_base + qs + 32 * w;
  // Q^T B-operand, pre-scaled into the exp2 domain: k-step ks holds Q[row][16ks + 8hi .. +7]
  bf16x8_t qf[8];
  {
    const int rr = min(my_row, q_len - 1);
    const uint16_t* qr = q + ((size_t)(q_begin + rr) * Hq + hq) * D;
#pragma unroll
    for (int ks = 0; ks < 8; ++ks) {
      float f[8];
      unpack8(*reinterpret_cast<const uint4*>(qr + 16 * ks + 8 * hi), f);
#pragma unroll
      for (int j = 0; j < 8; ++j) f[j] *= scale_log2;
      qf[ks] = as_bf16x8(pack8(f));
    }
  }

  // staging: 1024 16-B pieces of K + 1024 of V per tile, 4 + 4 per thread
  uint4 kst[4], vst[4];
  auto gload = [&](int kt) {
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      const int id = tid + 256 * i;
      {  // K: row = id >> 4 (key in tile), chunk = id & 15
        const int row = id >> 4, ch = id & 15, key = kt * PF_KT + row;
        kst[i] = key < kend ? *reinterpret_cast<const uint4*>(
                                  kc + (((size_t)bt[key / KV_BS] * Hkv + hk) * KV_BS + (key % KV_BS)) * D + ch * 8)
                            : make_uint4(0, 0, 0, 0);
      }
      {  // V^T: block bi = id >> 9, d = (id >> 2) & 127, cache chunk g = id & 3 (slots 8g..8g+7)
        const int bi = id >> 9, d = (id >> 2) & 127, g = id & 3;
        const int key0 = kt * PF_KT + bi * KV_BS;
        vst[i] = key0 < kend ? *reinterpret_cast<const uint4*>(
                                   vc + ((size_t)bt[key0 / KV_BS] * Hkv + hk) * D * KV_BS + kv_v_off(d, 8 * g, D))
                             : make_uint4(0, 0, 0, 0);
      }
    }
  };
  auto lwrite = [&](int buf) {
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      const int id = tid + 256 * i;
      *reinterpret_cast<uint4*>(smem + buf * 16384 + k_lds_off(id >> 4, id & 15)) = kst[i];
      // cache slots 8g..8g+3 hold keys 4g..4g+3 and 8g+4..8g+7 hold keys 16+4g..16+4g+3; in the
      // 32x32 order key k of a 32-block sits at slot 16(k>>4) + 8((k>>2)&1) + 4((k&15)>>3) + (k&3)
      const int bi = id >> 9, d = (id >> 2) & 127, g = id & 3;
      const int base = 32 * bi + 8 * (g & 1) + 4 * (g >> 1);        // slot of key 4g (s = 0)
      char* vrow = smem + 32768 + buf * 16384;
      const uint2 lo = make_uint2(vst[i].x, vst[i].y), hi2 = make_uint2(vst[i].z, vst[i].w);
      *reinterpret_cast<uint2*>(vrow + v4_off(d, base >> 3) + (base & 7) * 2) = lo;
      *reinterpret_cast<uint2*>(vrow + v4_off(d, (base + 16) >> 3) + ((base + 16) & 7) * 2) = hi2;
    }
  };

  f32x16_t o[4];
#pragma unroll
  for (int i = 0; i < 4; ++i)
#pragma unroll
    for (int r = 0; r < 16; ++r) o[i][r] = 0.f;
  float m = -INFINITY, l = 0.f;

  gload(0);
  lwrite(0);
  __syncthreads();
  for (int kt = 0; kt < ntiles; ++kt) {
    const int cur = kt & 1;
    const bool more = kt + 1 < ntiles;
    if (more) gload(kt + 1);

    const char* kb = smem + cur * 16384;
    const char* vb = smem + 32768 + cur * 16384;
    const int key0 = kt * PF_KT;
    if (key0 <= wave_min_pos + 31) {
      f32x16_t sc[2];
#pragma unroll
      for (int hf = 0; hf < 2; ++hf) {
#pragma unroll
        for (int r = 0; r < 16; ++r) sc[hf][r] = 0.f;
        const int row = 32 * hf + l32;
#pragma unroll
        for (int ks = 0; ks < 8; ++ks)
          sc[hf] = mfma32(as_bf16x8(*reinterpret_cast<const uint4*>(kb + k_lds_off(row, 2 * ks + hi))), qf[ks], sc[hf]);
      }
      if (key0 + PF_KT - 1 > wave_min_pos) {  // diagonal tile: causal mask
#pragma unroll
        for (int hf = 0; hf < 2; ++hf)
#pragma unroll
          for (int r = 0; r < 16; ++r)
            if (key0 + 32 * hf + 8 * (r >> 2) + 4 * hi + (r & 3) > my_pos) sc[hf][r] = -INFINITY;
      }
      float tmax = -INFINITY;
#pragma unroll
      for (int hf = 0; hf < 2; ++hf)
#pragma unroll
        for (int r = 0; r < 16; ++r) tmax = fmaxf(tmax, sc[hf][r]);
      tmax = xor32_max(tmax);
      if (!__all(tmax - m <= RESCALE_THR)) {
        const float mn = fmaxf(m, tmax);
        const float mref = mn == -INFINITY ? 0.f : mn;
        const float alpha = exp2f(m - mref);
        l *= alpha;
#pragma unroll
        for (int dt = 0; dt < 4; ++dt) o[dt] *= alpha;
        m = mn;
      }
      const float mref = m == -INFINITY ? 0.f : m;
      float rs = 0.f;
#pragma unroll
      for (int hf = 0; hf < 2; ++hf)
#pragma unroll
        for (int r = 0; r < 16; ++r) { const float e = exp2f(sc[hf][r] - mref); sc[hf][r] = e; rs += e; }
      rs = xor32_sum(rs);
      l += rs;
#pragma unroll
      for (int hf = 0; hf < 2; ++hf)
#pragma unroll
        for (int ss = 0; ss < 2; ++ss) {
          uint4 u;
          u.x = pack2bf(sc[hf][8 * ss + 0], sc[hf][8 * ss + 1]);
          u.y = pack2bf(sc[hf][8 * ss + 2], sc[hf][8 * ss + 3]);
          u.z = pack2bf(sc[hf][8 * ss + 4], sc[hf][8 * ss + 5]);
          u.w = pack2bf(sc[hf][8 * ss + 6], sc[hf][8 * ss + 7]);
          const bf16x8_t pf = as_bf16x8(u);
          const int c = 4 * hf + 2 * ss + hi;     // V^T chunk of slots 32hf + 16ss + 8hi .. +7
#pragma unroll
          for (int dt = 0; dt < 4; ++dt)
            o[dt] = mfma32(as_bf16x8(*reinterpret_cast<const uint4*>(vb + v4_off(32 * dt + l32, c))), pf, o[dt]);
        }
    }
    if (more) lwrite(cur ^ 1);
    __syncthreads();
  }

  if (my_row < q_len) {
    const float inv = l > 0.f ? 1.f / l : 0.f;
    uint16_t* orow = out + ((size_t)(q_begin + my_row) * Hq + hq) * D;
#pragma unroll
    for (int dt = 0; dt < 4; ++dt)
#pragma unroll
      for (int rg = 0; rg < 4; ++rg) {   // registers 4rg..4rg+3 = d 32dt + 8rg + 4hi + 0..3
        uint2 pk;
        pk.x = pack2bf(o[dt][4 * rg] * inv, o[dt][4 * rg + 1] * inv);
        pk.y = pack2bf(o[dt][4 * rg + 2] * inv, o[dt][4 * rg + 3] * inv);
        *reinterpret_cast<uint2*>(orow + 32 * dt + 8 * rg + 4 * hi) = pk;
      }
  }
}

// ------------------------------------------------------------------------------------------
// Prefill v5 (default): GQA-packed 8-wave tiles on v_mfma_f32_32x32x16_bf16.
// grid = (n_tiles, Hkv); block = 512 = 8 waves, 2 per SIMD.  A tile is QR = 256 / G query rows of
// ONE sequence for ALL G query heads of kv-head hk: wave w takes head hk*G + (w % G) and rows
// 32 (w / G) .. +31.  Every K/V byte staged in LDS therefore feeds 256 query rows (8 waves), and
// the tile spans only 256/G positions, so at G = 4 the causal diagonal idles 4x fewer rows than a
// 256-row single-head tile would.
//   * LDS per KV tile (64 keys): K 64 x 256 B (16-B chunk c of key r at r*256 + ((c ^ (r&15))<<4))
//     and V^T 128 d-rows x 128 B copied AS STORED in the cache (decode slot order).  The decode
//     order already fits the 32x32 PV: cache chunk g of a 32-key block holds keys {4g..4g+3,
//     16+4g..16+4g+3}, all with key bit 2 == g&1, which is exactly the half-wave (lane>>5) that holds
//     them in the S^T accumulator; so k-step s of half hf uses chunk 4hf + 2s + hi for the A operand
//     and accumulator registers {4s..4s+3, 8+4s..8+4s+3} as the B operand -- one ds_read_b128 and
//     one in-lane pack, no permutation anywhere.  V swizzle c ^ ((d>>1)&7) ^ ((d&1)<<2): the
//     ds_read_b128 lane groups and the 8-lane ds_write_b128 groups are both conflict-free.
//   * register-staged double buffer, one barrier per tile (loads for tile t+1 issued before tile
//     t's MFMAs, LDS writes after); Q pre-scaled into the exp2 domain; deferred rescale
//     (RESCALE_THR); row max / sum across the two half-waves with v_permlane32_swap (no LDS
//     bpermute); per-lane partial row sums combined once at the end; v_exp_f32 / v_cvt_pk_bf16_f32
//     directly; waves 4-7 at static priority 1 (the younger half loses VALU arbitration otherwise).
// ------------------------------------------------------------------------------------------
typedef __bf16 bf16x2_t __attribute__((ext_vector_type(2)));
typedef float f32x2_t __attribute__((ext_vector_type(2)));

__device__ __forceinline__ uint32_t cvt_pk_bf16(float a, float b) {
  return __builtin_bit_cast(uint32_t, __builtin_convertvector(f32x2_t{a, b}, bf16x2_t));
}
// value of lane l ^ 32 combined with lane l's own (both halves get the same result)
__device__ __forceinline__ float pair_max(float x) {
  const auto r = __builtin_amdgcn_permlane32_swap(__float_as_uint(x), __float_as_uint(x), false, false);
  return fmaxf(__uint_as_float(r[0]), __uint_as_float(r[1]));
}
__device__ __forceinline__ float pair_sum(float x) {
  const auto r = __builtin_amdgcn_permlane32_swap(__float_as_uint(x), __float_as_uint(x), false, false);
  return __uint_as_float(r[0]) + __uint_as_float(r[1]);
}
// reductions over the 4 lanes l, l^16, l^32, l^48 (one MFMA 16x16 output column): two VALU
// permlane swaps instead of two ds_bpermute round trips
__device__ __forceinline__ float quad_max(float x) {
  const auto r = __builtin_amdgcn_permlane16_swap(__float_as_uint(x), __float_as_uint(x), false, false);
  return pair_max(fmaxf(__uint_as_float(r[0]), __uint_as_float(r[1])));
}
__device__ __forceinline__ float quad_sum(float x) {
  const auto r = __builtin_amdgcn_permlane16_swap(__float_as_uint(x), __float_as_uint(x), false, false);
  return pair_sum(__uint_as_float(r[0]) + __uint_as_float(r[1]));
}
__device__ __forceinline__ int v5_off(int d, int c) { return d * 128 + ((c ^ ((d >> 1) & 7) ^ ((d & 1) << 2)) << 4); }

template <int G, bool F8 = false>
__global__ void __launch_bounds__(512, 2) prefill_gqa_kernel(
    const uint16_t* __restrict__ q, const void* __restrict__ kc, const void* __restrict__ vc,
    const int32_t* __restrict__ block_tables, const int32_t* __restrict__ cu_q, const int32_t* __restrict__ ctx_lens,
    const int32_t* __restrict__ tile_seq, const int32_t* __restrict__ tile_q0, float scale_log2, int Hq, int Hkv,
    int max_blocks, int window, float v_scale, int xcd_local, uint16_t* __restrict__ out) {
  // F8: e4m3 caches (K / k_scale folded into scale_log2 by the host, V / v_scale rescaled at the
  // output); tiles are widened to bf16 at the LDS write, so the MFMA loop is the bf16 one
  constexpr int D = 128;
  constexpr int QR = 256 / G;      // query rows per tile
  extern __shared__ __attribute__((aligned(16))) char smem[];
  // LDS: [K buf0 16K][K buf1 16K][V buf0 16K][V buf1 16K]
  // xcd_local: the (tile, kv-head) grid is XCD-remapped so each XCD takes a contiguous run of the
  // kv-head-major order -- with Hkv a multiple of 8 one XCD serves whole kv-heads and its L2 holds
  // only their K/V, instead of every XCD touching every head's K/V
  int t = blockIdx.x, hk = blockIdx.y;
  if (xcd_local) {
    const int lin = xcd_remap(blockIdx.y * gridDim.x + blockIdx.x, gridDim.x * gridDim.y);
    hk = lin / gridDim.x;
    t = lin - hk * gridDim.x;
  }
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6, tid = threadIdx.x;
  const int l32 = lane & 31, hi = lane >> 5;
  const int hq = hk * G + (w % G);
  const int rsub = w / G;
  const int s = tile_seq[t], qs = tile_q0[t];
  const int q_begin = cu_q[s], q_len = cu_q[s + 1] - q_begin;
  const int ctx = ctx_lens[s];
  const int pos_base = ctx - q_len;
  const int row_last = min(qs + QR - 1, q_len - 1);
  const int kend = pos_base + row_last + 1;         // keys [0, kend) are needed by this tile
  const int ntiles = (kend + PF_KT - 1) / PF_KT;
  // sliding window: row at position p sees keys (p - window, p]; the tile's first row bounds it
  const int kt_begin = window > 0 ? max(0, pos_base + qs - window + 1) / PF_KT : 0;
  const int32_t* bt = block_tables + (size_t)s * max_blocks;

  if (__builtin_amdgcn_readfirstlane(threadIdx.x) >= 256) __builtin_amdgcn_s_setprio(1);

  const int my_row = qs + 32 * rsub + l32;
  const int my_pos = pos_base + my_row;
  const int wave_min_pos = pos_base + qs + 32 * rsub;
  // Q^T B-operand, pre-scaled: k-step ks holds Q[row][16ks + 8hi .. +7]
  bf16x8_t qf[8];
  {
    const int rr = min(my_row, q_len - 1);
    const uint16_t* qr = q + ((size_t)(q_begin + rr) * Hq + hq) * D;
#pragma unroll
    for (int ks = 0; ks < 8; ++ks) {
      float f[8];
      unpack8(*reinterpret_cast<const uint4*>(qr + 16 * ks + 8 * hi), f);
      uint4 u;
      u.x = cvt_pk_bf16(f[0] * scale_log2, f[1] * scale_log2);
      u.y = cvt_pk_bf16(f[2] * scale_log2, f[3] * scale_log2);
      u.z = cvt_pk_bf16(f[4] * scale_log2, f[5] * scale_log2);
      u.w = cvt_pk_bf16(f[6] * scale_log2, f[7] * scale_log2);
      qf[ks] = as_bf16x8(u);
    }
  }

  // staging: tile kt = cache blocks 2kt, 2kt+1; piece i of a thread is block 2kt+i, bytes 16 tid ..
  // of both its K image [32][128] and its V^T image [128][32] (each 8 KB contiguous).  The block id
  // is workgroup-uniform (scalar load) and the data loads are UNCONDITIONAL (a block past kend
  // re-reads the last needed block; its V is zeroed at the LDS write), so no per-lane select
  // makes the compiler wait for the loads inside the issue sequence -- they stay in flight across
  // the tile's MFMAs.
  const int nb_need = (kend + KV_BS - 1) / KV_BS;
  uint4 ks0, ks1, vs0, vs1;     // named (not an array): an array here is kept in scratch
  auto gload = [&](int kt) {
    const int b0 = bt[min(2 * kt, nb_need - 1)], b1 = bt[min(2 * kt + 1, nb_need - 1)];
    if constexpr (F8) {
      // 8 KB of K and 8 KB of V per tile: one 16-B piece of each per thread; block = tid >> 8
      const size_t base = ((size_t)(tid >> 8 ? b1 : b0) * Hkv + hk) * (KV_BS * D) + 16 * (tid & 255);
      ks0 = *reinterpret_cast<const uint4*>(reinterpret_cast<const uint8_t*>(kc) + base);
      vs0 = *reinterpret_cast<const uint4*>(reinterpret_cast<const uint8_t*>(vc) + base);
    } else {
      const size_t base0 = ((size_t)b0 * Hkv + hk) * (KV_BS * D) + 8 * tid;
      const size_t base1 = ((size_t)b1 * Hkv + hk) * (KV_BS * D) + 8 * tid;
      ks0 = *reinterpret_cast<const uint4*>(reinterpret_cast<const uint16_t*>(kc) + base0);
      vs0 = *reinterpret_cast<const uint4*>(reinterpret_cast<const uint16_t*>(vc) + base0);
      ks1 = *reinterpret_cast<const uint4*>(reinterpret_cast<const uint16_t*>(kc) + base1);
      vs1 = *reinterpret_cast<const uint4*>(reinterpret_cast<const uint16_t*>(vc) + base1);
    }
  };
  auto lwrite = [&](int buf, int kt) {
    char* kb = smem + buf * 16384;
    char* vb = smem + 32768 + buf * 16384;
    const bool z0 = kt * PF_KT >= kend, z1 = kt * PF_KT + KV_BS >= kend;
    if constexpr (F8) {
      const int b = tid >> 8, e = tid & 255;
      const int key = (e >> 3) + 32 * b, ch = 2 * (e & 7);          // 16 d values = bf16 chunks ch, ch+1
      *reinterpret_cast<uint4*>(kb + k_lds_off(key, ch)) = fp8x8_to_bf16x8(make_uint2(ks0.x, ks0.y));
      *reinterpret_cast<uint4*>(kb + k_lds_off(key, ch + 1)) = fp8x8_to_bf16x8(make_uint2(ks0.z, ks0.w));
      // 16 bytes of the [4][D][8] tile = slot chunk e >> 6 of rows d, d + 1
      const int d = 2 * (e & 63), c = 4 * b + (e >> 6);
      const bool z = b ? z1 : z0;
      const uint4 zero = make_uint4(0, 0, 0, 0);
      *reinterpret_cast<uint4*>(vb + v5_off(d, c)) = z ? zero : fp8x8_to_bf16x8(make_uint2(vs0.x, vs0.y));
      *reinterpret_cast<uint4*>(vb + v5_off(d + 1, c)) = z ? zero : fp8x8_to_bf16x8(make_uint2(vs0.z, vs0.w));
    } else {
      *reinterpret_cast<uint4*>(kb + k_lds_off(tid >> 4, tid & 15)) = ks0;
      *reinterpret_cast<uint4*>(kb + k_lds_off((tid >> 4) + 32, tid & 15)) = ks1;
      // element 8 tid of the [4][D][8] tile = slot chunk tid >> 7 of row tid & 127
      *reinterpret_cast<uint4*>(vb + v5_off(tid & 127, tid >> 7)) = z0 ? make_uint4(0, 0, 0, 0) : vs0;
      *reinterpret_cast<uint4*>(vb + v5_off(tid & 127, 4 + (tid >> 7))) = z1 ? make_uint4(0, 0, 0, 0) : vs1;
    }
  };

  f32x16_t o[4];
#pragma unroll
  for (int i = 0; i < 4; ++i)
#pragma unroll
    for (int r = 0; r < 16; ++r) o[i][r] = 0.f;
  float m = -INFINITY, l = 0.f;   // l: this lane's partial row sum (its 32 of every 64 keys)
  // l in 4 interleaved partial sums: one serial chain of 32 dependent v_add_f32 per tile was
  // on the critical path between the exp2s and the next tile (ISA); summed once at the end
  float lp[4] = {0.f, 0.f, 0.f, 0.f};

  gload(kt_begin);
  lwrite(kt_begin & 1, kt_begin);
  __syncthreads();
  for (int kt = kt_begin; kt < ntiles; ++kt) {
    const int cur = kt & 1;
    const bool more = kt + 1 < ntiles;
    if (more) gload(kt + 1);

    const char* kb = smem + cur * 16384;
    const char* vb = smem + 32768 + cur * 16384;
    const int key0 = kt * PF_KT;
    const bool below = window > 0 && key0 + PF_KT - 1 <= wave_min_pos - window;  // all keys out of window
    if (key0 <= wave_min_pos + 31 && !below) {     // else every key of the tile is masked for this wave
      // scores come out of the MFMA already shifted by the running max (the accumulator starts at
      // -m): a tile that needs no rescale goes straight to exp2, without 32 subtractions per lane
      const float mref0 = m == -INFINITY ? 0.f : m;
      f32x16_t sc[2];
      if constexpr (PF_QK_PIPE == 2) {
        // both halves' 16 K fragments in flight before the 16 MFMAs (246 VGPRs; measured equal to
        // one half at a time, profiles/r05_ab_prefill_attn_qkpipe2.log)
        uint4 kf[2][8];
#pragma unroll
        for (int hf = 0; hf < 2; ++hf)
#pragma unroll
          for (int ks = 0; ks < 8; ++ks)
            kf[hf][ks] = *reinterpret_cast<const uint4*>(kb + k_lds_off(32 * hf + l32, 2 * ks + hi));
#pragma unroll
        for (int hf = 0; hf < 2; ++hf) {
#pragma unroll
          for (int r = 0; r < 16; ++r) sc[hf][r] = -mref0;
#pragma unroll
          for (int ks = 0; ks < 8; ++ks) sc[hf] = mfma32(as_bf16x8(kf[hf][ks]), qf[ks], sc[hf]);
        }
        __builtin_amdgcn_sched_group_barrier(0x100, 16, 0);
        __builtin_amdgcn_sched_group_barrier(0x008, 16, 0);
      } else
#pragma unroll
      for (int hf = 0; hf < 2; ++hf) {
#pragma unroll
        for (int r = 0; r < 16; ++r) sc[hf][r] = -mref0;
        const int row = 32 * hf + l32;
        // all 8 K fragments of the half in flight before its MFMA chain (PF_QK_PIPE): left to
        // itself hipcc issued read -> lgkmcnt(0) -> MFMA sixteen times, one LDS round trip each
        if constexpr (PF_QK_PIPE) {
          uint4 kf[8];
#pragma unroll
          for (int ks = 0; ks < 8; ++ks) kf[ks] = *reinterpret_cast<const uint4*>(kb + k_lds_off(row, 2 * ks + hi));
#pragma unroll
          for (int ks = 0; ks < 8; ++ks) sc[hf] = mfma32(as_bf16x8(kf[ks]), qf[ks], sc[hf]);
          __builtin_amdgcn_sched_group_barrier(0x100, 8, 0);   // 8 DS reads, then
          __builtin_amdgcn_sched_group_barrier(0x008, 8, 0);   // the 8 MFMAs (counted lgkmcnt waits)
        } else {
#pragma unroll
          for (int ks = 0; ks < 8; ++ks)
            sc[hf] = mfma32(as_bf16x8(*reinterpret_cast<const uint4*>(kb + k_lds_off(row, 2 * ks + hi))), qf[ks],
                            sc[hf]);
        }
      }
      // the first half's 8 V^T fragments read now, under the softmax's VALU work (PF_V_EARLY)
      uint4 vf0[2][2][4];
      if constexpr (PF_V_EARLY) {
#pragma unroll
        for (int hf = 0; hf < PF_V_EARLY; ++hf)
#pragma unroll
          for (int ss = 0; ss < 2; ++ss)
#pragma unroll
            for (int dt = 0; dt < 4; ++dt)
              vf0[hf][ss][dt] = *reinterpret_cast<const uint4*>(vb + v5_off(32 * dt + l32, 4 * hf + 2 * ss + hi));
      }
      if (key0 + PF_KT - 1 > wave_min_pos) {  // diagonal tile: causal mask
#pragma unroll
        for (int hf = 0; hf < 2; ++hf)
#pragma unroll
          for (int r = 0; r < 16; ++r)
            if (key0 + 32 * hf + 8 * (r >> 2) + 4 * hi + (r & 3) > my_pos) sc[hf][r] = -INFINITY;
      }
      if (window > 0 && key0 <= wave_min_pos + 31 - window) {  // window edge: keys <= pos - window
#pragma unroll
        for (int hf = 0; hf < 2; ++hf)
#pragma unroll
          for (int r = 0; r < 16; ++r)
            if (key0 + 32 * hf + 8 * (r >> 2) + 4 * hi + (r & 3) <= my_pos - window) sc[hf][r] = -INFINITY;
      }
      // the tile's row max minus mref0: two interleaved v_max3 chains (16 instructions for 32
      // values; the pairwise form compiled to 16 v_max + 8 v_max3)
      float ta = fmaxf(fmaxf(sc[0][0], sc[0][1]), sc[0][2]);
      float tb = fmaxf(fmaxf(sc[1][0], sc[1][1]), sc[1][2]);
#pragma unroll
      for (int r = 3; r < 15; r += 2) {
        ta = fmaxf(fmaxf(ta, sc[0][r]), sc[0][r + 1]);
        tb = fmaxf(fmaxf(tb, sc[1][r]), sc[1][r + 1]);
      }
      float tmax = fmaxf(fmaxf(ta, sc[0][15]), fmaxf(tb, sc[1][15]));
      tmax = pair_max(tmax);
      if (!__all(m != -INFINITY && tmax <= RESCALE_THR)) {
        const float mn = fmaxf(m, mref0 + tmax);
        const float alpha = __builtin_amdgcn_exp2f(m - (mn == -INFINITY ? 0.f : mn));
#pragma unroll
        for (int u = 0; u < 4; ++u) lp[u] *= alpha;
#pragma unroll
        for (int dt = 0; dt < 4; ++dt) o[dt] *= alpha;
        m = mn;
        const float shift = (m == -INFINITY ? 0.f : m) - mref0;
#pragma unroll
        for (int hf = 0; hf < 2; ++hf)
#pragma unroll
          for (int r = 0; r < 16; ++r) sc[hf][r] -= shift;
      }
#pragma unroll
      for (int hf = 0; hf < 2; ++hf)
#pragma unroll
        for (int r = 0; r < 16; ++r) {
          const float e = __builtin_amdgcn_exp2f(sc[hf][r]);
          sc[hf][r] = e;
          lp[r & 3] += e;
        }
#pragma unroll
      for (int hf = 0; hf < 2; ++hf)
#pragma unroll
        for (int ss = 0; ss < 2; ++ss) {
          uint4 u;
          u.x = cvt_pk_bf16(sc[hf][4 * ss + 0], sc[hf][4 * ss + 1]);
          u.y = cvt_pk_bf16(sc[hf][4 * ss + 2], sc[hf][4 * ss + 3]);
          u.z = cvt_pk_bf16(sc[hf][8 + 4 * ss + 0], sc[hf][8 + 4 * ss + 1]);
          u.w = cvt_pk_bf16(sc[hf][8 + 4 * ss + 2], sc[hf][8 + 4 * ss + 3]);
          const bf16x8_t pf = as_bf16x8(u);
          const int c = 4 * hf + 2 * ss + hi;
#pragma unroll
          for (int dt = 0; dt < 4; ++dt)
            o[dt] = mfma32(as_bf16x8(hf < PF_V_EARLY ? vf0[hf][ss][dt]
                                                     : *reinterpret_cast<const uint4*>(vb + v5_off(32 * dt + l32, c))),
                           pf, o[dt]);
        }
    }
    if (more) lwrite(cur ^ 1, kt + 1);
    __syncthreads();
  }

  l = pair_sum((lp[0] + lp[1]) + (lp[2] + lp[3]));
  if (my_row < q_len) {
    const float inv = l > 0.f ? v_scale / l : 0.f;
    uint16_t* orow = out + ((size_t)(q_begin + my_row) * Hq + hq) * D;
#pragma unroll
    for (int dt = 0; dt < 4; ++dt)
#pragma unroll
      for (int rg = 0; rg < 4; ++rg) {   // registers 4rg..4rg+3 = d 32dt + 8rg + 4hi + 0..3
        uint2 pk;
        pk.x = cvt_pk_bf16(o[dt][4 * rg] * inv, o[dt][4 * rg + 1] * inv);
        pk.y = cvt_pk_bf16(o[dt][4 * rg + 2] * inv, o[dt][4 * rg + 3] * inv);
        *reinterpret_cast<uint2*>(orow + 32 * dt + 8 * rg + 4 * hi) = pk;
      }
  }
}

// ------------------------------------------------------------------------------------------
// Varlen bidirectional encoder attention (BERT family), D in {32, 64}, S <= 512.
// Input qkv is the fused projection output [T, 3*H*D] (q | k | v, head-major inside each).
// 1-D grid over (query tile, head), XCD-remapped; block = 256 = 4 waves, tile = ENC_ROWS = 256
// query rows (wave w: rows 64w .. 64w+63 as ENC_R = 4 groups of 16).  The WHOLE key/value range
// of the sequence is staged once in LDS per block (K row-major, V transposed with the per-32-key
// slot permutation) -- with 256-row tiles a MiniLM sequence (S <= 256) stages its K/V once per
// head instead of once per 64 rows -- then every wave runs the swapped-product online softmax:
// each 32-key K / V fragment is read from LDS once and reused by the wave's 4 row groups.
// Softmax: Q is pre-scaled by scale*log2(e) at load, the key mask runs only on the sequence's
// last (partial) 32-key tile, exponentials are v_exp_f32 (inputs <= 0).
// ------------------------------------------------------------------------------------------
constexpr int ENC_R = 4;               // 16-row query groups per wave
constexpr int ENC_ROWS = 64 * ENC_R;   // query rows per workgroup

template <int D>
__global__ void __launch_bounds__(256) encoder_attn_kernel(const uint16_t* __restrict__ qkv,
                                                           const int32_t* __restrict__ cu_seqlens,
                                                           const int32_t* __restrict__ tile_seq,
                                                           const int32_t* __restrict__ tile_q0, float scale_log2,
                                                           int H, uint16_t* __restrict__ out) {
  constexpr int NC = D / 8;         // 16-byte chunks per K row
  constexpr int KSTEPS = D / 32;    // MFMA k-steps over head_dim
  constexpr int DT = D / 16;        // 16-wide output column tiles
  extern __shared__ __attribute__((aligned(16))) char smem[];
  // logical block = tile * H + head, XCD-remapped: every (query tile, head) block of a sequence
  // lands on ONE XCD, so the sequence's fused qkv rows (all heads share each 128-B line) are
  // fetched from HBM once into that XCD's L2 instead of once per XCD.
  const int lb = xcd_remap(blockIdx.x, gridDim.x);
  const int t = lb / H, h = lb - t * H;
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6, tid = threadIdx.x;
  const int col = lane & 15, g = lane >> 4;
  const int s = tile_seq[t], qs = tile_q0[t];
  const int beg = cu_seqlens[s], S = cu_seqlens[s + 1] - beg;
  const int Spad = (S + 127) & ~127;       // V^T rows hold Spad slots (multiple of 128 => >=16 chunks)
  const int row_stride = 3 * H * D;
  char* klds = smem;                              // [Spad][D]  bf16, swizzled per 16-row group
  char* vlds = smem + (size_t)Spad * D * 2;       // [D][Spad]  bf16, slot-permuted, swizzled

  // K rows: chunk ch of row r at r*D*2 + ((ch ^ sw(r)) * 16).
  auto koff = [&](int r, int ch) -> int {
    if constexpr (D == 32) return r * 64 + ((ch ^ (((r >> 3) & 1) << 1)) << 4);
    else return r * 128 + ((ch ^ (r & 7)) << 4);
  };
  // V^T element (d, slot): row d has Spad*2 bytes; 16-byte chunk c = slot>>3 swizzled by d&15.
  auto voff_chunk = [&](int d, int c) -> int { return d * Spad * 2 + ((c ^ (d & 15)) << 4); };

  // Q fragments first (pre-scaled), so their loads overlap the K/V staging below
  const int wrow0 = qs + 64 * w;
  const int ng = min(ENC_R, max(0, (S - wrow0 + 15) >> 4));   // row groups with >= 1 row (wave-uniform)
  bf16x8_t qf[ENC_R][KSTEPS];
#pragma unroll
  for (int rg = 0; rg < ENC_R; ++rg) {
    const int r = min(wrow0 + 16 * rg + col, S - 1);
    const uint16_t* qr = qkv + (size_t)(beg + r) * row_stride + h * D;
#pragma unroll
    for (int c = 0; c < KSTEPS; ++c) {
      float f[8];
      unpack8(*reinterpret_cast<const uint4*>(qr + 32 * c + 8 * g), f);
      uint4 u;
      u.x = pack2bf(f[0] * scale_log2, f[1] * scale_log2);
      u.y = pack2bf(f[2] * scale_log2, f[3] * scale_log2);
      u.z = pack2bf(f[4] * scale_log2, f[5] * scale_log2);
      u.w = pack2bf(f[6] * scale_log2, f[7] * scale_log2);
      qf[rg][c] = as_bf16x8(u);
    }
  }

  // K / V staging: every thread issues SB chunk loads of K and of V before any LDS write, so one
  // memory round trip covers SB chunks (a load -> write -> load loop pays the latency per chunk)
  constexpr int SB = 4;
  const int nchunks = Spad * NC;
  for (int id0 = tid; id0 < nchunks; id0 += 256 * SB) {
    uint4 kv[SB], vv[SB];
#pragma unroll
    for (int b = 0; b < SB; ++b) {
      const int id = id0 + 256 * b, r = id / NC, ch = id % NC;
      kv[b] = make_uint4(0, 0, 0, 0);
      vv[b] = make_uint4(0, 0, 0, 0);
      if (id < nchunks && r < S) {
        const uint16_t* base = qkv + (size_t)(beg + r) * row_stride;
        kv[b] = *reinterpret_cast<const uint4*>(base + H * D + h * D + ch * 8);
        vv[b] = *reinterpret_cast<const uint4*>(base + 2 * H * D + h * D + ch * 8);
      }
    }
#pragma unroll
    for (int b = 0; b < SB; ++b) {
      const int id = id0 + 256 * b, r = id / NC, ch = id % NC;
      if (id >= nchunks) break;
      *reinterpret_cast<uint4*>(klds + koff(r, ch)) = kv[b];
      // scatter V row r (d = ch*8 .. +7) into V^T at the permuted slot of key r
      const int kin = r & 31, hi = kin >> 4, gg = (kin >> 2) & 3, jj = (kin & 3) + 4 * hi;
      const int slot = (r & ~31) + 8 * gg + jj;
      const uint16_t* ve = reinterpret_cast<const uint16_t*>(&vv[b]);
#pragma unroll
      for (int e = 0; e < 8; ++e) {
        const int d = ch * 8 + e;
        *reinterpret_cast<uint16_t*>(vlds + voff_chunk(d, slot >> 3) + (slot & 7) * 2) = ve[e];
      }
    }
  }
  __syncthreads();
  if (ng == 0) return;   // no barrier follows

  f32x4_t o[ENC_R][DT];
  float m[ENC_R], l[ENC_R];
#pragma unroll
  for (int rg = 0; rg < ENC_R; ++rg) {
    m[rg] = -INFINITY;
    l[rg] = 0.f;
#pragma unroll
    for (int i = 0; i < DT; ++i) o[rg][i] = f32x4_t{0.f, 0.f, 0.f, 0.f};
  }

  for (int k0 = 0; k0 < S; k0 += 32) {
    bf16x8_t kf[2][KSTEPS];
#pragma unroll
    for (int st = 0; st < 2; ++st)
#pragma unroll
      for (int c = 0; c < KSTEPS; ++c)
        kf[st][c] = as_bf16x8(*reinterpret_cast<const uint4*>(klds + koff(k0 + 16 * st + col, 4 * c + g)));
    bf16x8_t vf[DT];
#pragma unroll
    for (int dt = 0; dt < DT; ++dt)
      vf[dt] = as_bf16x8(*reinterpret_cast<const uint4*>(vlds + voff_chunk(16 * dt + col, (k0 >> 3) + g)));
    const bool tail = k0 + 32 > S;

#pragma unroll
    for (int rg = 0; rg < ENC_R; ++rg) {
      if (rg >= ng) break;
      f32x4_t sc[2];
#pragma unroll
      for (int st = 0; st < 2; ++st) {
        sc[st] = f32x4_t{0.f, 0.f, 0.f, 0.f};
#pragma unroll
        for (int c = 0; c < KSTEPS; ++c) sc[st] = mfma16(kf[st][c], qf[rg][c], sc[st]);
      }
      if (tail) {
#pragma unroll
        for (int st = 0; st < 2; ++st)
#pragma unroll
          for (int i = 0; i < 4; ++i)
            if (k0 + 16 * st + 4 * g + i >= S) sc[st][i] = -INFINITY;
      }
      float tmax = fmaxf(fmaxf(fmaxf(sc[0][0], sc[0][1]), fmaxf(sc[0][2], sc[0][3])),
                         fmaxf(fmaxf(sc[1][0], sc[1][1]), fmaxf(sc[1][2], sc[1][3])));
      tmax = quad_max(tmax);
      // deferred rescale (guide T13, as in the prefill kernel): O and l are rescaled only when the
      // running max grows by more than RESCALE_THR, not on every 32-key step -- the per-step
      // multiply of O (held in AGPRs) cost a read / multiply / write per register
      if (!__all(tmax - m[rg] <= RESCALE_THR)) {
        const float mn = fmaxf(m[rg], tmax);
        const float alpha = __builtin_amdgcn_exp2f(m[rg] - (mn == -INFINITY ? 0.f : mn));
        l[rg] *= alpha;
#pragma unroll
        for (int dt = 0; dt < DT; ++dt) o[rg][dt] *= alpha;
        m[rg] = mn;
      }
      const float mref = m[rg] == -INFINITY ? 0.f : m[rg];
      float rs = 0.f;
#pragma unroll
      for (int st = 0; st < 2; ++st)
#pragma unroll
        for (int i = 0; i < 4; ++i) {
          const float e = __builtin_amdgcn_exp2f(sc[st][i] - mref);
          sc[st][i] = e;
          rs += e;
        }
      rs = quad_sum(rs);
      l[rg] += rs;
      const bf16x8_t pf = pack_p(sc[0], sc[1]);
#pragma unroll
      for (int dt = 0; dt < DT; ++dt) o[rg][dt] = mfma16(vf[dt], pf, o[rg][dt]);
    }
  }

#pragma unroll
  for (int rg = 0; rg < ENC_R; ++rg) {
    const int my_row = wrow0 + 16 * rg + col;
    if (rg < ng && my_row < S) {
      const float inv = l[rg] > 0.f ? 1.f / l[rg] : 0.f;
      uint16_t* orow = out + ((size_t)(beg + my_row) * H + h) * D;
#pragma unroll
      for (int dt = 0; dt < DT; ++dt) {
        uint2 pk;
        pk.x = pack2bf(o[rg][dt][0] * inv, o[rg][dt][1] * inv);
        pk.y = pack2bf(o[rg][dt][2] * inv, o[rg][dt][3] * inv);
        *reinterpret_cast<uint2*>(orow + 16 * dt + 4 * g) = pk;
      }
    }
  }
}

}  // namespace

// q: [B, Hq, 128] bf16; caches per layer as documented above; out: [B, Hq, 128] bf16.
// part_o / part_ml: fp32 workspaces of B*Hq*P*128 and B*Hq*P*2 floats (unused when P == 1).
template <bool F8>
static int launch_paged_decode(const void* q, const void* k_cache, const void* v_cache, const int32_t* block_tables,
                               const int32_t* ctx_lens, int B, int Hq, int Hkv, int head_dim, int max_blocks,
                               int part_blocks, int P, float scale, int window, float v_scale, float* part_o,
                               float* part_ml, void* out, hipStream_t stream, const DecRope* rope = nullptr,
                               const int32_t* shared_blocks = nullptr) {
  if (head_dim != 128 || Hq % Hkv != 0 || B <= 0 || P <= 0 || window < 0) return -1;
  if (rope != nullptr && ((rope->qkv == nullptr) == (rope->part == nullptr) || (rope->part && rope->split < 1) ||
                          !rope->positions || !rope->slots || !rope->cos_sin))
    return -1;
  const DecRope rp = rope ? *rope : DecRope{};
  const int G = Hq / Hkv;
  dim3 grid(P, Hkv, B);
  const float sl2 = scale * LOG2E;
#define DEC_ARGS (const uint16_t*)q, k_cache, v_cache, block_tables, ctx_lens, sl2, Hkv, max_blocks, part_blocks, P, \
    window, v_scale, part_o, part_ml, (uint16_t*)out, rp, shared_blocks
  // nontemporal KV loads for large batches (B=128: 6.5 vs 5.9 TB/s; B=8: 3.8 vs 4.2 -- there the
  // plain loads win), profiles/decode_attn_partitions_r01.log; CFC_DECODE_NT=0/1 forces either
  static const int nt_env = [] { const char* e = getenv("CFC_DECODE_NT"); return e ? atoi(e) : -1; }();
  const bool nt = nt_env >= 0 ? nt_env != 0 : B >= 32;
#define DEC_CASE(GG) \
  case GG: \
    if (rope) { \
      if (nt) paged_decode_kernel<GG, true, F8, true><<<grid, 256, 0, stream>>>(DEC_ARGS); \
      else paged_decode_kernel<GG, false, F8, true><<<grid, 256, 0, stream>>>(DEC_ARGS); \
    } else { \
      if (nt) paged_decode_kernel<GG, true, F8><<<grid, 256, 0, stream>>>(DEC_ARGS); \
      else paged_decode_kernel<GG, false, F8><<<grid, 256, 0, stream>>>(DEC_ARGS); \
    } \
    break;
  switch (G) {
    DEC_CASE(1) DEC_CASE(2) DEC_CASE(4) DEC_CASE(8) DEC_CASE(16)
    default: return -3;
  }
#undef DEC_CASE
#undef DEC_ARGS
  if (P > 1) decode_combine_kernel<<<dim3(Hq, B), 128, 0, stream>>>(part_o, part_ml, P, Hq, (uint16_t*)out);
  return CFC_CHECK_LAUNCH();
}

// q: [B, Hq, 128] bf16; caches per layer as documented above; out: [B, Hq, 128] bf16.
// part_o / part_ml: fp32 workspaces of B*Hq*P*128 and B*Hq*P*2 floats (unused when P == 1).
// shared_blocks (device int32, may be null): leading blocks of every sequence read through the
// caches (the batch's shared prefix blocks), the rest nontemporal.
CFC_API int cfc_paged_decode_attention(const void* q, const void* k_cache, const void* v_cache,
                                       const int32_t* block_tables, const int32_t* ctx_lens, int B, int Hq, int Hkv,
                                       int head_dim, int max_blocks, int part_blocks, int P, float scale, int window,
                                       float* part_o, float* part_ml, void* out, const int32_t* shared_blocks,
                                       hipStream_t stream) {
  return launch_paged_decode<false>(q, k_cache, v_cache, block_tables, ctx_lens, B, Hq, Hkv, head_dim, max_blocks,
                                    part_blocks, P, scale, window, 1.f, part_o, part_ml, out, stream, nullptr,
                                    shared_blocks);
}

// Timing ablations of the fused decode RoPE (scripts/probe_decode_rope_fused.py): bit 1 skips the new
// key's cache row, bit 2 the V^T slot-group store, bit 4 makes that store nontemporal.  Results are wrong
// with bits 1 / 2 set; production never sets it.
static int g_dec_rope_probe = 0;
CFC_API int cfc_set_decode_rope_probe(int bits) {
  g_dec_rope_probe = bits;
  return 0;
}

// Decode attention with the step's RoPE + KV write in its prologue (DecRope).  qkv [B, (Hq+2Hkv)*128]
// bf16 OR part [split, B, (Hq+2Hkv)*128] fp32 slabs (exactly one non-null); positions / slots [B];
// fp8 != 0: e4m3 caches (K / k_scale, V / v_scale).  Writes out [B, Hq, 128]; q never leaves the chip.
CFC_API int cfc_paged_decode_rope_attention(const void* qkv, const float* part, int split, const int32_t* positions,
                                            const int32_t* slots, const float* cos_sin, void* k_cache, void* v_cache,
                                            const int32_t* block_tables, const int32_t* ctx_lens, int B, int Hq,
                                            int Hkv, int head_dim, int max_blocks, int part_blocks, int P, float scale,
                                            int window, int fp8, float k_scale, float v_scale, float* part_o,
                                            float* part_ml, void* out, const int32_t* shared_blocks,
                                            hipStream_t stream) {
  const DecRope rp{(const uint16_t*)qkv, part, split, positions, slots, cos_sin, 1.f / k_scale, 1.f / v_scale,
                   g_dec_rope_probe};
  if (fp8)
    return launch_paged_decode<true>(nullptr, k_cache, v_cache, block_tables, ctx_lens, B, Hq, Hkv, head_dim,
                                     max_blocks, part_blocks, P, scale * k_scale, window, v_scale, part_o, part_ml,
                                     out, stream, &rp, shared_blocks);
  return launch_paged_decode<false>(nullptr, k_cache, v_cache, block_tables, ctx_lens, B, Hq, Hkv, head_dim,
                                    max_blocks, part_blocks, P, scale, window, 1.f, part_o, part_ml, out, stream, &rp,
                                    shared_blocks);
}

// FP8 (e4m3fn) caches holding K / k_scale and V / v_scale
CFC_API int cfc_paged_decode_attention_fp8(const void* q, const void* k_cache, const void* v_cache,
                                           const int32_t* block_tables, const int32_t* ctx_lens, int B, int Hq,
                                           int Hkv, int head_dim, int max_blocks, int part_blocks, int P, float scale,
                                           int window, float k_scale, float v_scale, float* part_o, float* part_ml,
                                           void* out, const int32_t* shared_blocks, hipStream_t stream) {
  return launch_paged_decode<true>(q, k_cache, v_cache, block_tables, ctx_lens, B, Hq, Hkv, head_dim, max_blocks,
                                   part_blocks, P, scale * k_scale, window, v_scale, part_o, part_ml, out, stream,
                                   nullptr, shared_blocks);
}

CFC_API int cfc_prefill_tile_rows() { return PF_ROWS; }

static int prefill_variant() {
  static const int v = [] { const char* e = getenv("CFC_PREFILL_VARIANT"); return e ? atoi(e) : 5; }();
  return v;
}
static int prefill_xcd_local() {
  static const int v = [] { const char* e = getenv("CFC_PREFILL_XCD"); return e ? atoi(e) : 1; }();
  return v;
}

// Query rows per tile the default prefill kernel expects for Hq / Hkv heads (the host tiler's
// granularity): 256 / G on the GQA-packed kernel, else PF_ROWS.
CFC_API int cfc_prefill_rows(int Hq, int Hkv) {
  if (Hkv <= 0 || Hq % Hkv) return PF_ROWS;
  const int G = Hq / Hkv;
  const bool v5 = prefill_variant() == 5 && (G == 1 || G == 2 || G == 4 || G == 8);
  return v5 ? 256 / G : PF_ROWS;
}

CFC_API int cfc_prefill_attention(const void* q, const void* k_cache, const void* v_cache, const int32_t* block_tables,
                                  const int32_t* cu_q, const int32_t* ctx_lens, const int32_t* tile_seq,
                                  const int32_t* tile_q0, int n_tiles, int tile_rows, int Hq, int Hkv, int head_dim,
                                  int max_blocks, float scale, int window, void* out, hipStream_t stream) {
  if (head_dim != 128 || Hkv <= 0 || Hq % Hkv != 0 || window < 0) return -1;
  if (tile_rows != cfc_prefill_rows(Hq, Hkv)) return -2;     // tiles cut for another kernel
  if (n_tiles <= 0) return 0;
  const size_t lds = 65536;
  const int G = Hq / Hkv;
#define PF_ARGS (const uint16_t*)q, (const uint16_t*)k_cache, (const uint16_t*)v_cache, block_tables, cu_q, ctx_lens, \
    tile_seq, tile_q0, scale * LOG2E, Hq, Hkv, max_blocks, (uint16_t*)out
#define PF5_ARGS (const uint16_t*)q, k_cache, v_cache, block_tables, cu_q, ctx_lens, \
    tile_seq, tile_q0, scale * LOG2E, Hq, Hkv, max_blocks, window, 1.f, prefill_xcd_local(), (uint16_t*)out
  if (tile_rows != PF_ROWS || (G * tile_rows == 256 && prefill_variant() == 5)) {
    // 5: GQA-packed 8-wave kernel (default)
    const dim3 grid(n_tiles, Hkv);
    switch (G) {
      case 1: prefill_gqa_kernel<1><<<grid, 512, lds, stream>>>(PF5_ARGS); break;
      case 2: prefill_gqa_kernel<2><<<grid, 512, lds, stream>>>(PF5_ARGS); break;
      case 4: prefill_gqa_kernel<4><<<grid, 512, lds, stream>>>(PF5_ARGS); break;
      case 8: prefill_gqa_kernel<8><<<grid, 512, lds, stream>>>(PF5_ARGS); break;
      default: return -3;
    }
    return CFC_CHECK_LAUNCH();
  }
  if (window > 0) return -4;     // sliding window: GQA-packed kernel only
  // legacy single-head 128-row kernels: 0 = v3 <=128 VGPRs (2 workgroups / CU); 1 = v3 <=256 VGPRs;
  // 2/3 = v4 (32x32 MFMA, 2 / 1 WG per CU)
  const int variant = prefill_variant();
  if (variant == 1) prefill_paged_kernel<2><<<dim3(n_tiles, Hq), 512, lds, stream>>>(PF_ARGS);
  else if (variant == 2) prefill_paged_kernel_v4<2><<<dim3(n_tiles, Hq), 256, lds, stream>>>(PF_ARGS);
  else if (variant == 3) prefill_paged_kernel_v4<1><<<dim3(n_tiles, Hq), 256, lds, stream>>>(PF_ARGS);
  else prefill_paged_kernel<4><<<dim3(n_tiles, Hq), 512, lds, stream>>>(PF_ARGS);
#undef PF_ARGS
#undef PF5_ARGS
  return CFC_CHECK_LAUNCH();
}

// FP8 (e4m3fn) caches holding K / k_scale and V / v_scale; GQA-packed kernel only (G in 1,2,4,8)
CFC_API int cfc_prefill_attention_fp8(const void* q, const void* k_cache, const void* v_cache,
                                      const int32_t* block_tables, const int32_t* cu_q, const int32_t* ctx_lens,
                                      const int32_t* tile_seq, const int32_t* tile_q0, int n_tiles, int tile_rows,
                                      int Hq, int Hkv, int head_dim, int max_blocks, float scale, int window,
                                      float k_scale, float v_scale, void* out, hipStream_t stream) {
  if (head_dim != 128 || Hkv <= 0 || Hq % Hkv != 0 || window < 0) return -1;
  const int G = Hq / Hkv;
  if (!(G == 1 || G == 2 || G == 4 || G == 8) || tile_rows * G != 256) return -2;
  if (n_tiles <= 0) return 0;
  const dim3 grid(n_tiles, Hkv);
#define PF8_ARGS (const uint16_t*)q, k_cache, v_cache, block_tables, cu_q, ctx_lens, tile_seq, tile_q0, \
    scale * k_scale * LOG2E, Hq, Hkv, max_blocks, window, v_scale, prefill_xcd_local(), (uint16_t*)out
  switch (G) {
    case 1: prefill_gqa_kernel<1, true><<<grid, 512, 65536, stream>>>(PF8_ARGS); break;
    case 2: prefill_gqa_kernel<2, true><<<grid, 512, 65536, stream>>>(PF8_ARGS); break;
    case 4: prefill_gqa_kernel<4, true><<<grid, 512, 65536, stream>>>(PF8_ARGS); break;
    default: prefill_gqa_kernel<8, true><<<grid, 512, 65536, stream>>>(PF8_ARGS); break;
  }
#undef PF8_ARGS
  return CFC_CHECK_LAUNCH();
}

CFC_API int cfc_encoder_rows() { return ENC_ROWS; }

CFC_API int cfc_encoder_attention(const void* qkv, const int32_t* cu_seqlens, const int32_t* tile_seq,
                                  const int32_t* tile_q0, int n_tiles, int tile_rows, int H, int head_dim,
                                  int max_seqlen, float scale, void* out, hipStream_t stream) {
  if (tile_rows != ENC_ROWS) return -3;          // tiles cut for another kernel revision
  if (n_tiles <= 0) return 0;
  if (max_seqlen > 512) return -2;
  const int spad = (max_seqlen + 127) & ~127;
  const size_t lds = (size_t)spad * head_dim * 2 * 2;
  if (head_dim == 32) {
    encoder_attn_kernel<32><<<dim3(n_tiles * H), 256, lds, stream>>>((const uint16_t*)qkv, cu_seqlens, tile_seq, tile_q0,
                                                                    scale * LOG2E, H, (uint16_t*)out);
  } else if (head_dim == 64) {
    encoder_attn_kernel<64><<<dim3(n_tiles * H), 256, lds, stream>>>((const uint16_t*)qkv, cu_seqlens, tile_seq, tile_q0,
                                                                    scale * LOG2E, H, (uint16_t*)out);
  } else {
    return -1;
  }
  return CFC_CHECK_LAUNCH();
}
