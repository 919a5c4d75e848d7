// Decode GEMM for gfx950 at batch sizes 5..256:  Y[M, N] = X[M, K] . W[N, K]^T  (bf16 in, fp32 acc).
//
// At decode a projection is a weight stream: W (14-235 MB per projection, the whole layer per
// token step) is read exactly once while X (M x K, <= 7 MB) stays in L2.  At M = 128 every weight
// byte carries 128 flops, so each CU must keep ~12 B/clk of W arriving AND run its MFMAs at ~40 %
// of peak.  What the measurements on this chip said (scripts/bench_dgemm.py --ablate):
//   * with the MFMAs removed an LDS-ring kernel was exactly as fast -- the limit is how the W bytes
//     are fetched, not the math;
//   * an LDS-DMA W ring (4-6 stages in flight per CU) stayed at ~4.1-4.5 TB/s however deep.
// So here W never touches LDS:
//
//   * workgroup = BN/16 compute waves + 2 X-loader waves, tile = ALL M rows (BM = 64/128/256) x BN
//     W rows (BN = 64..128, chosen per shape so ~256 workgroups run: one per CU);
//   * compute wave w owns 16 W rows and loads its B fragments straight from HBM into a D-stage
//     register ring (D = 8 x 64-deep K stages = 16 KB per wave in flight, the GEMV's depth).  Its
//     only vector-memory instructions are those loads, so hipcc's own counted vmcnt waits are
//     exact and never drain the ring; every load is unconditional (the tail re-reads the last
//     stage) so no branch joins force a vmcnt(0) (round-2 finding);
//   * X (an L2 hit, shared by all compute waves) is staged by the 2 loader waves with LDS-DMA
//     (`global_load_lds_dwordx4`, written in asm so hipcc orders nothing behind it) into an
//     NSX-slot LDS ring; only the loaders wait on vmcnt for it (counted, in one asm statement with
//     the s_barrier), so the X and W streams never serialise each other through the in-order
//     vmcnt counter;
//   * the X image is lane-linear per DMA piece and XOR-swizzled through the SOURCE address: chunk
//     c of row r at r*128 + ((c ^ (r & 7)) << 4), so the 16-row ds_read_b128 A-fragment reads are
//     bank-conflict free (guide rule 21 / T2);
//   * split-K over the grid for the small-N projections; blocks are remapped XCD-locally so the
//     blocks of one XCD share a K slice and therefore the same X slice in that XCD's L2 (guide T1);
//   * epilogues: fp32 split-K partials (reduced by the residual + RMSNorm / SwiGLU reduce), bf16,
//     or SwiGLU over gate/up weights interleaved in 8-row groups (each 16-row n-tile = 8 gate +
//     8 up rows, so silu(g) * u is one lane swap away; same bf16 rounding points as
//     GEMM -> silu_mul).
//
// MFMA maps (guide §3): A = X rows (m on lane & 15, k = 8 * (lane >> 4) + j), B = W rows (n on
// lane & 15, same k); C/D: n = lane & 15, m = 4 * (lane >> 4) + i.
#include "common.h"

namespace {

typedef __attribute__((address_space(3))) void dg_lds_t;
typedef unsigned int dg_u32x4 __attribute__((ext_vector_type(4)));

// X-loader waves per workgroup: fill the workgroup up to 8 waves (2 per SIMD, 256 VGPRs each), at
// least one
template <int BN>
constexpr int dg_loaders() { return BN / 16 >= 7 ? 1 : 8 - BN / 16 > 2 ? 2 : 8 - BN / 16; }
// DG_PART_WT: the split-K slabs stored write-through (sc1): they reach memory while the kernel
// runs instead of as dirty L2 lines the kernel boundary must write back before the consumer (the
// residual + RMSNorm reduce, rope_kv) may start -- MI355X_MICROARCH "boundary": +B / 6 TB/s behind
// B dirty bytes, 2.8-3.8 us behind 12.6-16.8 MB of fp32 partials.
enum { DG_PART = 0, DG_BF16 = 1, DG_SILU = 2, DG_PART_WT = 3 };

// MX (ablation 64): two X-loader waves and an 8-slot X ring whatever BN -- one loader wave's
// vmcnt window (63 pieces = 3 stages at BM = 128) may cap the X stream of the wide-BN shapes.
template <int BM, int BN, bool MX = false>
struct DgShape {
  static constexpr int NW = BN / 16;                  // compute waves
  static constexpr int LOADERS = MX ? 2 : dg_loaders<BN>();
  static constexpr int WAVES = NW + LOADERS;
  static constexpr int MT = BM / 16;                  // m-tiles per compute wave
  // W register ring depth (64-deep stages); 9 waves (BN = 128) leave 168 VGPRs per lane
  static constexpr int D = BM == 256 ? 4 : (WAVES > 8 ? 6 : 8);
  static constexpr int XSTAGE = BM * 128;             // X bytes per 64-deep stage
  static constexpr int XP = BM / 8 / LOADERS;         // 1-KB DMA pieces per loader wave per stage
  // X ring slots (64-128 KB); a loader keeps NSX - 2 stages in flight at its wait, and vmcnt
  // counts at most 63 of its pieces
  static constexpr int NSX_BASE = MX ? 8 : (BM == 256 ? 4 : (BM == 128 ? 6 : 8));
  static constexpr int NSX = (NSX_BASE - 2 <= 63 / XP ? NSX_BASE : 2 + 63 / XP);
};

__device__ __forceinline__ f32x4_t dg_mfma(uint4 a, uint4 b, f32x4_t c) {
  return __builtin_amdgcn_mfma_f32_16x16x32_bf16(__builtin_bit_cast(bf16x8_t, a), __builtin_bit_cast(bf16x8_t, b),
                                                 c, 0, 0, 0);
}

// One 1-KB LDS-DMA piece: lane l's 16 source bytes land at lds_addr + 16 l.  Inline asm, so hipcc
// sees no LDS write to order the compute waves' ds_reads behind; M0 (compiler-reserved) is saved
// and restored inside the statement (guide §5.7).
__device__ __forceinline__ void dg_glds16(const void* gsrc, uint32_t lds_addr) {
  unsigned keep;
  asm volatile("s_mov_b32 %0, m0\n\ts_mov_b32 m0, %2\n\ts_nop 0\n\tglobal_load_lds_dwordx4 %1, off\n\ts_mov_b32 m0, %0"
               : "=&s"(keep)
               : "v"(gsrc), "s"(lds_addr)
               : "memory");
}

// loader waves: s_waitcnt vmcnt(n) + s_barrier as ONE statement (n = DMA pieces still allowed in flight)
template <int N>
__device__ __forceinline__ void dg_wait_barrier() {
  asm volatile("s_waitcnt vmcnt(%0)\n\ts_barrier" ::"i"(N) : "memory");
}

template <int P, int MAXA>
__device__ __forceinline__ void dg_wait_ahead(int ahead) {
  if constexpr (MAXA == 0) {
    dg_wait_barrier<0>();
  } else {
    if (ahead >= MAXA) dg_wait_barrier<MAXA * P>();
    else dg_wait_ahead<P, MAXA - 1>(ahead);
  }
}

// compute waves: their W loads stay in flight across the barrier; their LDS reads of the previous
// stage are retired first (hipcc may sink the MFMA that waits for them below an asm statement),
// so the loaders' next DMA into that slot cannot overtake them
__device__ __forceinline__ void dg_barrier() { asm volatile("s_waitcnt lgkmcnt(0)\n\ts_barrier" ::: "memory"); }

// per-lane part of the offset in voff (one VGPR for the whole ring), the wave-uniform stage part in
// soff (an SGPR)
template <bool NT>
__device__ __forceinline__ uint4 dg_ldw_buf(__amdgpu_buffer_rsrc_t rs, int voff, int soff) {
  const dg_u32x4 v = __builtin_amdgcn_raw_buffer_load_b128(rs, voff, soff, NT ? 2 : 0);
  return make_uint4(v.x, v.y, v.z, v.w);
}

template <bool NT>
__device__ __forceinline__ uint4 dg_ldw(const uint16_t* p) {
  if constexpr (NT) {
    const dg_u32x4 v = __builtin_nontemporal_load(reinterpret_cast<const dg_u32x4*>(p));
    return make_uint4(v.x, v.y, v.z, v.w);
  } else {
    return *reinterpret_cast<const uint4*>(p);
  }
}

// ABL: ablation builds for the timing probes only (scripts/bench_dgemm.py --ablate); 0 in production.
//   1 = no X DMA, 2 = no ds_read / MFMA (W loads kept live), 4 = no K-order rotation,
//   16 = X first: the loaders' first X stages enter the CU's memory pipeline before the compute
//   waves' W ring fill (one extra barrier), so the first MFMAs do not wait behind ~96 KB of W;
//   32 = contiguous W pieces: wave w loads fragments 2w, 2w+1 of the stage's 2 NW KB region (one
//   2-KB run per wave) instead of its own group's two 1-KB fragments NW KB apart (wrong sums);
//   64 = two X-loader waves + an 8-slot X ring (DgShape MX);
//   256 = the round-5 tail (re-reads the last stage instead of issuing no loads);
//   128 = no workgroup barrier in the compute waves' stage loop (with 1 only: the loader waves
//   return at once) -- is the per-stage lockstep of the compute waves what slows the W stream?
// PACKED: W in the fragment-packed layout of cfc_dgemm_pack for this BN: tile-major, then 32-deep
// k group, then wave: Wp[N/BN][K/32][BN/16][64][8], so the 16 rows x 32 k of one MFMA B fragment
// are 1 KB contiguous in lane order and a workgroup's whole W slice (BN rows x its K range) is ONE
// contiguous span that its waves read front to back, 2 KB each per stage.  Measured
// (scripts/probes_stream.py, probes_flat.py): row-major fragments (16 rows x 64 B per instruction,
// 8 KB row stride) stream at 3.8-4.2 TB/s however deep the ring; contiguous 1-KB pieces at
// 6.0 TB/s from the same 224-256 workgroups.  Packed loads are buffer loads (32-bit offsets into
// the workgroup's span) so the cache policy can be set: NTW = nontemporal for these once-read
// bytes (guide "nt-weights").
template <int BM, int BN, int EPI, bool NTW, int ABL = 0, bool PACKED = true>
__global__ void __launch_bounds__((64 * DgShape<BM, BN, (ABL & 64) != 0>::WAVES), 1)
    dgemm_kernel(const uint16_t* __restrict__ X, const uint16_t* __restrict__ W, int M, int N, int K, int ntiles,
                 int split, float* __restrict__ part, uint16_t* __restrict__ out, int ldo) {
  using S = DgShape<BM, BN, (ABL & 64) != 0>;
  constexpr int NW = S::NW;
  constexpr int D = S::D;
  __shared__ __attribute__((aligned(16))) char smem[S::NSX * S::XSTAGE];
  const int lane = threadIdx.x & 63;
  const int w = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);

  // logical block: the blocks of one XCD take consecutive ids, i.e. (mostly) one K slice
  const int lid = xcd_remap(blockIdx.x, gridDim.x);
  const int ks = lid / ntiles, tile = lid % ntiles;
  const int n0 = tile * BN, m0 = blockIdx.y * BM;
  const int nks = K >> 6;
  const int kb = (int)((long)ks * nks / split), ke = (int)((long)(ks + 1) * nks / split);
  const int nst = ke - kb;
  const int kq = lane >> 4;         // 8-element k group within a 32-deep MFMA step
  // K-order rotation: workgroup `lid` walks its K slice starting at stage `rot` and wraps around,
  // so the ~256 concurrent workgroups read different K offsets of their rows at any moment instead
  // of all hitting the same power-of-2-strided address set in lock step (the sum is order-free)
  const int rot = (ABL & 4) ? 0 : (int)((unsigned)lid * 37u % (unsigned)nst);
  auto phys = [&](int s) { s += rot; return s >= nst ? s - nst : s; };

  constexpr bool NOBAR = (ABL & 128) != 0;
  // XT: the MFMA's A operand is the W fragment, B the X fragment (probe 512: the round-5
  // orientation, X as A, one output element per lane per row -> 4-byte epilogue stores)
  constexpr bool XT = (ABL & 512) == 0;
  static_assert(!NOBAR || (ABL & 1), "no-barrier probe only without the X stream");
  if (w >= NW) {
    if constexpr (NOBAR) return;
    // ---------------- X loader wave, LDS-DMA: rows 8 XP l .. 8 XP (l+1) - 1 of the X stage image
    const int l = w - NW;
    const int prow = lane >> 3, pch = (lane & 7) ^ prow;   // row & 7 == prow for every piece
    const uint16_t* xsrc[S::XP];
#pragma unroll
    for (int i = 0; i < S::XP; ++i) {
      const int m = min(m0 + 8 * S::XP * l + 8 * i + prow, M - 1);   // rows past M: results dropped
      xsrc[i] = X + (size_t)m * K + (size_t)kb * 64 + 8 * pch;
    }
    const uint32_t lds0 =
        __builtin_amdgcn_readfirstlane((uint32_t)(uintptr_t)(dg_lds_t*)smem + 8 * S::XP * l * 128);
    auto issue = [&](int st, int slot) {
      if constexpr ((ABL & 1) != 0) return;
#pragma unroll
      for (int i = 0; i < S::XP; ++i) dg_glds16(xsrc[i] + phys(st) * 64, lds0 + slot * S::XSTAGE + i * 1024);
    };
#pragma unroll
    for (int p = 0; p < S::NSX - 1; ++p)
      if (p < nst) issue(p, p);
    if constexpr ((ABL & 16) != 0) asm volatile("s_barrier" ::: "memory");
    int slot = 0;
    for (int st = 0; st < nst; ++st) {
      if constexpr ((ABL & 1) != 0) dg_wait_barrier<0>();
      else dg_wait_ahead<S::XP, S::NSX - 2>(nst - 1 - st);
      // the slot read in iteration st-1 is free once every wave passed this barrier
      if (st + S::NSX - 1 < nst) issue(st + S::NSX - 1, slot == 0 ? S::NSX - 1 : slot - 1);
      slot = slot + 1 == S::NSX ? 0 : slot + 1;
    }
    return;
  }

  // ---------------- compute wave w: W rows n0 + 16 w + (lane & 15)
  uint4 ring[D][2];
  // packed: the workgroup's span, tile n0 / BN over all of K (split slices are sub-ranges of it),
  // as a buffer descriptor built from wave-uniform values (guide T20: no waterfall loops)
  const uint16_t* span = W + (size_t)(n0 / BN) * ((size_t)BN * K);
  const uint32_t span_lo = __builtin_amdgcn_readfirstlane((uint32_t)(uintptr_t)span);
  const uint32_t span_hi = __builtin_amdgcn_readfirstlane((uint32_t)((uintptr_t)span >> 32));
  const __amdgpu_buffer_rsrc_t wrs = __builtin_amdgcn_make_buffer_rsrc(
      (void*)(((uintptr_t)span_hi << 32) | span_lo), (short)0, PACKED ? BN * K * 2 : 0, 0x00020000);
  const int wvoff = lane * 16;                                                   // per-lane byte offset
  const int wsoff = __builtin_amdgcn_readfirstlane(((kb * 2) * NW + ((ABL & 32) ? 2 * w : w)) * 1024);
  // row-major: this lane's row and k offset
  const uint16_t* wp = W + (size_t)(n0 + 16 * w + (lane & 15)) * K + (size_t)kb * 64 + 8 * kq;
  // stage s of this lane: the kk = 0 and kk = 1 halves of its B fragments
  auto load_stage = [&](int s, uint4 (&dst)[2]) {
    if constexpr (PACKED) {
      const int so = __builtin_amdgcn_readfirstlane(wsoff + s * 2 * NW * 1024);
      dst[0] = dg_ldw_buf<NTW>(wrs, wvoff, so);
      dst[1] = dg_ldw_buf<NTW>(wrs, wvoff, so + ((ABL & 32) ? 1024 : NW * 1024));
    } else {
      dst[0] = dg_ldw<NTW>(wp + s * 64);
      dst[1] = dg_ldw<NTW>(wp + s * 64 + 32);
    }
  };
  // packed: logical stage s of the slice, or -- past its end -- zeros from an out-of-range buffer
  // offset (no memory access); the condition is wave-uniform, so this is a scalar select, no branch
  auto load_stage_past = [&](int s, uint4 (&dst)[2]) {
    const int so = __builtin_amdgcn_readfirstlane(s < nst ? wsoff + phys(s) * 2 * NW * 1024 : 0x40000000);
    dst[0] = dg_ldw_buf<NTW>(wrs, wvoff, so);
    dst[1] = dg_ldw_buf<NTW>(wrs, wvoff, so + ((ABL & 32) ? 1024 : NW * 1024));
  };
  if constexpr ((ABL & 16) != 0) asm volatile("s_barrier" ::: "memory");
#pragma unroll
  for (int p = 0; p < D; ++p) {
    if constexpr (PACKED && (ABL & 256) == 0) load_stage_past(p, ring[p]);
    else load_stage(phys(min(p, nst - 1)), ring[p]);
  }
  f32x4_t acc[S::MT];
#pragma unroll
  for (int i = 0; i < S::MT; ++i) acc[i] = f32x4_t{0.f, 0.f, 0.f, 0.f};

  const int xoff = (lane & 15) * 128;
  const int sw = lane & 7;
  int xslot = 0;
  auto compute = [&](const uint4 (&b)[2]) {
    if constexpr ((ABL & 2) != 0) {
      asm volatile("" ::"v"(__builtin_bit_cast(dg_u32x4, b[0])), "v"(__builtin_bit_cast(dg_u32x4, b[1])));
    } else {
      const char* ximg = smem + xslot * S::XSTAGE + xoff;
#pragma unroll
      for (int kk = 0; kk < 2; ++kk) {
        const int chunk = ((4 * kk + kq) ^ sw) << 4;
#pragma unroll
        for (int i = 0; i < S::MT; ++i) {
          const uint4 a = *reinterpret_cast<const uint4*>(ximg + i * 16 * 128 + chunk);
          // W fragment as the A operand: the 16 x 16 output tile comes out with four consecutive
          // W rows (output columns) of one X row per lane -> 16-byte epilogue stores
          acc[i] = XT ? dg_mfma(b[kk], a, acc[i]) : dg_mfma(a, b[kk], acc[i]);
        }
      }
    }
    xslot = xslot + 1 == S::NSX ? 0 : xslot + 1;
  };

  // Stage s lives in ring slot s % D; after computing stage s the slot is refilled with stage
  // s + D.  Every load is unconditional (a branch around a load makes hipcc drain the ring at the
  // join), so the last D refills of a slice name stages past its end: on the packed path they are
  // buffer loads at an offset past the descriptor's range, which return zeros without touching
  // memory (round 5 and before re-read the last stage D times instead: up to half of a small
  // slice's loads, e.g. 8 redundant 2-KB stages per wave of qkv's 16 at split 4).  The ring is never
  // read past the slice (the tail computes only real stages).
  constexpr bool TAIL_RELOAD = (ABL & 256) != 0;    // probe: the round-5 re-reading tail
  int st = 0;
  for (; st + D <= nst; st += D) {
#pragma unroll
    for (int u = 0; u < D; ++u) {
      if constexpr (!NOBAR) dg_barrier();   // X stage st+u is in LDS
      compute(ring[u]);
      if constexpr (PACKED && !TAIL_RELOAD) load_stage_past(st + u + D, ring[u]);
      else load_stage(phys(min(st + u + D, nst - 1)), ring[u]);
    }
  }
#pragma unroll
  for (int u = 0; u < D; ++u) {
    if (st + u < nst) {
      if constexpr (!NOBAR) dg_barrier();
      compute(ring[u]);
    }
  }

  if constexpr (XT) {
    // ---- epilogue: lane holds X row m0 + 16 i + (lane & 15) at the four consecutive W rows (output
    // columns) n0 + 16 w + 4 (lane >> 4) + r, r = 0..3 -- one 16-byte (fp32) / 8-byte (bf16) store per
    // lane and m-tile, 16 rows x 64 B per wave instruction (the round-5 orientation stored 4 bytes
    // per lane: 4x the store instructions, the epilogue's store-issue tail of a small-N projection)
    const int mr = m0 + (lane & 15);
    const int nq = n0 + 16 * w + 4 * kq;
    if constexpr (EPI == DG_SILU) {
      // 8-row interleave: W rows 0-7 of each 16-row group are gate, 8-15 the matching up rows, so the
      // lanes with kq < 2 hold gate rows and lane ^ 32 the up rows of the same output columns.  One
      // VALU lane swap (v_permlane32_swap) of (acc[0], acc[2]) hands every lane a (gate, up) pair --
      // column 0 in lanes kq < 2, column 2 in lanes kq >= 2 -- and one of (acc[1], acc[3]) columns
      // 1 / 3: each lane computes and stores two outputs
      const int oc = (n0 >> 1) + 8 * w + 4 * (kq & 1) + 2 * (kq >> 1);
      auto silu_mul = [](float gate, float up) {
        const float gt = bf2f(f2bf(gate)), u = bf2f(f2bf(up));
        return gt / (1.f + __expf(-gt)) * u;
      };
#pragma unroll
      for (int i = 0; i < S::MT; ++i) {
        float g0 = acc[i][0], u0 = acc[i][2], g1 = acc[i][1], u1 = acc[i][3];
        swap32(g0, u0);
        swap32(g1, u1);
        const int m = mr + 16 * i;
        if (m < M) *reinterpret_cast<uint32_t*>(out + (size_t)m * ldo + oc) = pack2bf(silu_mul(g0, u0), silu_mul(g1, u1));
      }
    } else if constexpr (EPI == DG_PART_WT) {
      // write-through (sc1) 16-byte stores through a buffer descriptor of the slab array (the
      // guide's R1 form: the consumer kernel reads them from memory, no dirty lines at the boundary)
      const uint32_t lo = __builtin_amdgcn_readfirstlane((uint32_t)(uintptr_t)part);
      const uint32_t hi = __builtin_amdgcn_readfirstlane((uint32_t)((uintptr_t)part >> 32));
      const __amdgpu_buffer_rsrc_t prs = __builtin_amdgcn_make_buffer_rsrc(
          (void*)(((uintptr_t)hi << 32) | lo), (short)0, 0x7fffffff, 0x00020000);
#pragma unroll
      for (int i = 0; i < S::MT; ++i) {
        const int m = mr + 16 * i;
        if (m < M) {
          const dg_u32x4 v = {__float_as_uint(acc[i][0]), __float_as_uint(acc[i][1]), __float_as_uint(acc[i][2]),
                              __float_as_uint(acc[i][3])};
          __builtin_amdgcn_raw_buffer_store_b128(v, prs, (int)((((size_t)ks * M + m) * N + nq) * 4), 0, 16);
        }
      }
    } else {
#pragma unroll
      for (int i = 0; i < S::MT; ++i) {
        const int m = mr + 16 * i;
        if (m < M) {
          if constexpr (EPI == DG_PART)
            *reinterpret_cast<float4*>(part + ((size_t)ks * M + m) * N + nq) =
                make_float4(acc[i][0], acc[i][1], acc[i][2], acc[i][3]);
          else
            *reinterpret_cast<uint2*>(out + (size_t)m * ldo + nq) =
                make_uint2(pack2bf(acc[i][0], acc[i][1]), pack2bf(acc[i][2], acc[i][3]));
        }
      }
    }
    return;
  }
  // ---- epilogue (round-5 orientation): lane holds rows m0 + 16 i + 4 (lane >> 4) + r of W row n
  const int n = n0 + 16 * w + (lane & 15);
  const int mb = m0 + 4 * kq;
  if constexpr (EPI == DG_SILU) {
    // 8-row interleave: lanes 0-7 of each 16 hold gate rows, lanes 8-15 the matching up rows
    const bool gate = (lane & 8) == 0;
    const int oc = (n0 >> 1) + 8 * w + (lane & 7);
#pragma unroll
    for (int i = 0; i < S::MT; ++i)
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        const float up = __shfl_xor(acc[i][r], 8, 64);
        const int m = mb + 16 * i + r;
        if (gate && m < M) {
          const float gt = bf2f(f2bf(acc[i][r])), u = bf2f(f2bf(up));
          out[(size_t)m * ldo + oc] = f2bf(gt / (1.f + __expf(-gt)) * u);
        }
      }
  } else {
#pragma unroll
    for (int i = 0; i < S::MT; ++i)
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        const int m = mb + 16 * i + r;
        if (m < M) {
          if constexpr (EPI == DG_PART) part[((size_t)ks * M + m) * N + n] = acc[i][r];
          else if constexpr (EPI == DG_PART_WT) {    // vector store with sc1 (agent-scope relaxed)
            // the element goes through a scalar temporary: __builtin_bit_cast of the vector element
            // expression acc[i][r] itself compiled to element 0 for every r (hipcc, ROCm 7.2)
            const float v = acc[i][r];
            __hip_atomic_store(reinterpret_cast<uint32_t*>(part + ((size_t)ks * M + m) * N + n), __float_as_uint(v),
                               __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
          }
          else out[(size_t)m * ldo + n] = f2bf(acc[i][r]);
        }
      }
  }
}

constexpr bool DG_NT = true;    // nontemporal packed weight stream (bench_dgemm --ablate: ~10 % faster)

template <int BM, int BN, bool NTW, int ABL, bool PK>
int dgemm_launch_bn(const void* x, const void* w, int M, int N, int K, int split, int epi, float* part, void* out,
                    int ldo, hipStream_t stream) {
  const int ntiles = N / BN;
  const dim3 grid(ntiles * split, (M + BM - 1) / BM);
  const int threads = 64 * DgShape<BM, BN, (ABL & 64) != 0>::WAVES;
#define DG_ARGS (const uint16_t*)x, (const uint16_t*)w, M, N, K, ntiles, split, part, (uint16_t*)out, ldo
  switch (epi) {
    case DG_PART: dgemm_kernel<BM, BN, DG_PART, NTW, ABL, PK><<<grid, threads, 0, stream>>>(DG_ARGS); break;
    case DG_PART_WT: dgemm_kernel<BM, BN, DG_PART_WT, NTW, ABL, PK><<<grid, threads, 0, stream>>>(DG_ARGS); break;
    case DG_BF16: dgemm_kernel<BM, BN, DG_BF16, NTW, ABL, PK><<<grid, threads, 0, stream>>>(DG_ARGS); break;
    case DG_SILU: dgemm_kernel<BM, BN, DG_SILU, NTW, ABL, PK><<<grid, threads, 0, stream>>>(DG_ARGS); break;
    default: return -3;
  }
#undef DG_ARGS
  return 0;
}

template <int BM, bool NTW, int ABL, bool PK>
int dgemm_launch_pk(const void* x, const void* w, int M, int N, int K, int split, int epi, int bn, float* part,
                    void* out, int ldo, hipStream_t stream) {
  switch (bn) {
    case 64: return dgemm_launch_bn<BM, 64, NTW, ABL, PK>(x, w, M, N, K, split, epi, part, out, ldo, stream);
    case 96: return dgemm_launch_bn<BM, 96, NTW, ABL, PK>(x, w, M, N, K, split, epi, part, out, ldo, stream);
    case 112: return dgemm_launch_bn<BM, 112, NTW, ABL, PK>(x, w, M, N, K, split, epi, part, out, ldo, stream);
    case 128: return dgemm_launch_bn<BM, 128, NTW, ABL, PK>(x, w, M, N, K, split, epi, part, out, ldo, stream);
    default: return -5;
  }
}

// packed weights stream nontemporal (NTW); row-major ones keep the default policy
template <int BM, int ABL = 0>
int dgemm_launch(const void* x, const void* w, int M, int N, int K, int split, int epi, int bn, int packed,
                 float* part, void* out, int ldo, hipStream_t stream) {
  return packed ? dgemm_launch_pk<BM, DG_NT, ABL, true>(x, w, M, N, K, split, epi, bn, part, out, ldo, stream)
                : dgemm_launch_pk<BM, false, ABL, false>(x, w, M, N, K, split, epi, bn, part, out, ldo, stream);
}

// Fragment-pack a row-major W[N][K] for workgroups of nw = BN/16 waves:
// Wp[t][kg][w][l][j] = W[BN t + 16 w + (l & 15)][32 kg + 8 (l >> 4) + j].  One thread per 16-B piece.
__global__ void dgemm_pack_kernel(const uint16_t* __restrict__ W, uint16_t* __restrict__ Wp, int N, int K, int nw) {
  const size_t i = (size_t)blockIdx.x * 256 + threadIdx.x;
  const size_t total = (size_t)N * K / 8;
  if (i >= total) return;
  const int l = (int)(i & 63);
  const size_t frag = i >> 6;
  const int kgs = K / 32;
  const int w = (int)(frag % nw);
  const size_t t2 = frag / nw;
  const int kg = (int)(t2 % kgs), t = (int)(t2 / kgs);
  const int row = 16 * (t * nw + w) + (l & 15);
  const uint4 v = *reinterpret_cast<const uint4*>(W + (size_t)row * K + 32 * kg + 8 * (l >> 4));
  reinterpret_cast<uint4*>(Wp)[i] = v;
}

int dgemm_check(int M, int N, int K, int split, int epi, int bn, const float* part, const void* out, int ldo) {
  if (M <= 0 || N <= 0 || K <= 0 || K % 64 || split < 1 || split > K / 64) return -1;
  if (bn != 64 && bn != 96 && bn != 112 && bn != 128) return -5;
  if (N % bn) return -1;
  const bool slabs = epi == DG_PART || epi == DG_PART_WT;
  if (!slabs && split != 1) return -2;
  if ((slabs && !part) || (!slabs && !out)) return -2;
  // the epilogue stores 4 consecutive outputs per lane: 16-byte fp32 / 8-byte bf16 aligned rows
  if ((slabs && ((uintptr_t)part & 15)) || (!slabs && (((uintptr_t)out & 7) || ldo % 4))) return -2;
  return 0;
}

}  // namespace

// Which row tile (64 / 128 / 256) a batch of M rows runs with (M > 256 loops 256-row tiles over grid.y).
CFC_API int cfc_dgemm_bm(int M) { return M <= 64 ? 64 : (M <= 128 ? 128 : 256); }

// epi 0: fp32 split-K partials into part[split][M][N]; 1: bf16 into out (row stride ldo, split 1);
// 2: SwiGLU over 8-row interleaved gate/up W -> bf16 [M, N/2] into out (split 1); 3: as 0 with
// write-through (sc1) slab stores.
// bn (W rows per workgroup) in {64, 96, 112, 128}, N % bn == 0, K % 64 == 0, 1 <= split <= K / 64.
// packed: w is in the fragment-packed layout cfc_dgemm_pack wrote for this same bn (else row-major [N][K]).
CFC_API int cfc_dgemm(const void* x, const void* w, int M, int N, int K, int split, int epi, int bn, int packed,
                      float* part, void* out, int ldo, hipStream_t stream) {
  if (const int e = dgemm_check(M, N, K, split, epi, bn, part, out, ldo)) return e;
  int rc;
  switch (cfc_dgemm_bm(M)) {
    case 64: rc = dgemm_launch<64>(x, w, M, N, K, split, epi, bn, packed, part, out, ldo, stream); break;
    case 128: rc = dgemm_launch<128>(x, w, M, N, K, split, epi, bn, packed, part, out, ldo, stream); break;
    default: rc = dgemm_launch<256>(x, w, M, N, K, split, epi, bn, packed, part, out, ldo, stream); break;
  }
  return rc ? rc : CFC_CHECK_LAUNCH();
}

// Row-major W[N][K] bf16 -> the fragment-packed layout for bn-row workgroups (same size; the
// packed weight is only valid with that bn).  N % bn == 0, bn % 16 == 0, K % 64 == 0.
CFC_API int cfc_dgemm_pack(const void* w, void* wp, int N, int K, int bn, hipStream_t stream) {
  if (N <= 0 || K <= 0 || bn <= 0 || bn % 16 || N % bn || K % 64 || w == wp) return -1;
  const size_t pieces = (size_t)N * K / 8;
  dgemm_pack_kernel<<<(unsigned)((pieces + 255) / 256), 256, 0, stream>>>((const uint16_t*)w, (uint16_t*)wp, N, K,
                                                                           bn / 16);
  return CFC_CHECK_LAUNCH();
}

// Timing probe only (scripts/bench_dgemm.py --ablate): split-K partial GEMM at BM = 128 on a
// packed weight, ablation bits `abl` (1 no X DMA, 2 no MFMA, 4 no K rotation); +8 = default
// (not nontemporal) cache policy on the weight stream.
CFC_API int cfc_dgemm_ablate(const void* x, const void* w, int M, int N, int K, int split, int bn, int abl,
                             float* part, hipStream_t stream) {
  if (M > 128 || (abl & ~1023)) return -1;
  if (const int e = dgemm_check(M, N, K, split, DG_PART, bn, part, nullptr, N)) return e;
  int rc;
  switch (abl) {
#define DG_ABL(A, NT) rc = dgemm_launch_pk<128, NT, A, true>(x, w, M, N, K, split, 0, bn, part, nullptr, 0, stream); break;
    case 0: DG_ABL(0, true)
    case 1: DG_ABL(1, true)
    case 2: DG_ABL(2, true)
    case 3: DG_ABL(3, true)
    case 4: DG_ABL(4, true)
    case 7: DG_ABL(7, true)
    case 8: DG_ABL(0, false)
    case 11: DG_ABL(3, false)
    case 16: DG_ABL(16, true)
    case 32: DG_ABL(32, true)
    case 35: DG_ABL(35, true)
    case 64: DG_ABL(64, true)
    case 96: DG_ABL(96, true)
    case 129: DG_ABL(129, true)
    case 131: DG_ABL(131, true)
    case 256: DG_ABL(256, true)
    case 259: DG_ABL(259, true)
    case 512: DG_ABL(512, true)
#undef DG_ABL
    default: return -3;
  }
  return rc ? rc : CFC_CHECK_LAUNCH();
}
