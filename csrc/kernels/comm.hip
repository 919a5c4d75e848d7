// One-shot all-reduce over IPC-mapped peer buffers (xGMI point-to-point), for the latency-bound
// tensor-parallel decode collectives (64 per token, each B x hidden bf16).
//
// Every rank owns ONE shared region, allocated uncached (fine-grained: stores write through and
// remote loads are never served from a stale L2 line) and exported with hipIpcGetMemHandle:
//
//   [ signals: CFC_AR_MAX_BLOCKS x CFC_AR_MAX_RANKS int32 ][ staging parity 0 ][ staging parity 1 ]
//   [ key area parity 0 ][ key area parity 1 ]
//
// Call k, block b (each block owns one contiguous slice of the tensor):
//   1. copy its slice of the input into this rank's staging[k & 1];
//   2. system-scope release, then store epoch k into signals[b][me] of EVERY peer (remote store);
//   3. poll this rank's signals[b][j] >= k for every peer j (system-scope acquire loads);
//   4. read slice b of every rank's staging[k & 1] (remote loads over xGMI), sum in fp32 in a
//      fixed rank order (bitwise identical on every rank), write the output slice.
// Double-buffering by parity makes one barrier per call sufficient: a peer that reached call k+1
// has finished kernel k (same stream), so nobody still reads staging[(k+2) & 1]'s previous use.
// Epochs live in a per-rank device array (one counter per block), so the launch has fixed
// arguments and is captured into the decode hipGraph like any other kernel.  Every sum-type call
// (any size, either kernel) launches all CFC_AR_SUM_BLOCKS blocks and the idle ones only advance
// their epoch: all blocks' epochs stay equal, so a call's parity is one per call whatever its
// size or row mapping, and a block of call k+1 can never write a staging region a peer's block of
// call k (another slice layout, same parity) may still be reading.
//
// The same protocol also reduces per-row int64 keys with MAX (the TP greedy lm_head: each vocab
// shard's (max logit, argmax) packed into one order-preserving key, so the decode graph needs no
// logits all-gather): it owns the last signal block and its own double-buffered key area, so its
// epochs never interleave with the sum's slices.  Every spin is bounded:
// on timeout the block records an error and exits, so a missing peer fails the call instead of
// hanging the GPU.
#include "common.h"

#define CFC_AR_MAX_RANKS 8
#define CFC_AR_MAX_BLOCKS 64
#define CFC_AR_SIGNAL_BYTES (CFC_AR_MAX_BLOCKS * CFC_AR_MAX_RANKS * 4)
#define CFC_AR_SPIN_LIMIT (1u << 22)   // ~1 us per uncached poll: a few seconds, then fail
#define CFC_AR_SUM_BLOCKS (CFC_AR_MAX_BLOCKS - 1)   // the last signal block belongs to the key-max
#define CFC_AR_KEY_ROWS 1024
#define CFC_AR_KEY_BYTES (CFC_AR_KEY_ROWS * 8)

struct ArPeers {
  char* base[CFC_AR_MAX_RANKS];  // each rank's shared region, mapped into this process
};

namespace {

__device__ __forceinline__ void store_signal(int* p, int v) {
  __hip_atomic_store(p, v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
}

__device__ __forceinline__ int load_signal(const int* p) {
  return __hip_atomic_load(p, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
}

template <int NR>
__global__ void __launch_bounds__(256) oneshot_allreduce_kernel(const uint16_t* __restrict__ in,
                                                                uint16_t* __restrict__ out, int64_t n8,
                                                                ArPeers peers, int rank, int64_t staging_bytes,
                                                                int* __restrict__ epochs, int* __restrict__ err,
                                                                int nact) {
  const int b = blockIdx.x;
  if (b >= nact) {                  // idle block: keeps its epoch (and so the parity) in step
    if (threadIdx.x == 0) epochs[b] += 1;
    return;
  }
  __shared__ int s_epoch, s_ok;
  if (threadIdx.x == 0) {
    s_epoch = epochs[b] + 1;
    s_ok = 1;
  }
  __syncthreads();
  const int epoch = s_epoch;
  const int64_t per = (n8 + nact - 1) / nact;
  const int64_t v0 = (int64_t)b * per, v1 = min(n8, v0 + per);
  const int64_t parity_off = CFC_AR_SIGNAL_BYTES + (int64_t)(epoch & 1) * staging_bytes;

  // 1. publish this rank's slice (uncached region: the stores write through)
  uint4* mine = reinterpret_cast<uint4*>(peers.base[rank] + parity_off);
  const uint4* src = reinterpret_cast<const uint4*>(in);
  for (int64_t v = v0 + threadIdx.x; v < v1; v += blockDim.x) mine[v] = src[v];
  __threadfence_system();  // every storing wave drains + releases its own stores
  __syncthreads();

  // 2. arrive at every peer (after the barrier: all of this block's slice is visible)
  if (threadIdx.x < NR) {
    int* sig = reinterpret_cast<int*>(peers.base[threadIdx.x]) + b * CFC_AR_MAX_RANKS + rank;
    store_signal(sig, epoch);
  }
  // 3. wait for every peer's arrival (lane j waits for rank j)
  if (threadIdx.x < NR) {
    const int* sig = reinterpret_cast<const int*>(peers.base[rank]) + b * CFC_AR_MAX_RANKS + threadIdx.x;
    unsigned spins = 0;
    while (load_signal(sig) < epoch) {
      __builtin_amdgcn_s_sleep(2);
      if (++spins > CFC_AR_SPIN_LIMIT) {
        s_ok = 0;
        break;
      }
    }
  }
  __syncthreads();
  __threadfence_system();  // acquire on every wave before its remote loads
  if (!s_ok) {
    if (threadIdx.x == 0) {
      atomicAdd(err, 1);
      epochs[b] = epoch;  // stay in step with peers that did arrive
    }
    return;
  }

  // 4. reduce slice b of every rank's staging buffer, fixed rank order -> identical on all ranks
  const uint4* st[NR];
#pragma unroll
  for (int r = 0; r < NR; ++r) st[r] = reinterpret_cast<const uint4*>(peers.base[r] + parity_off);
  uint4* dst = reinterpret_cast<uint4*>(out);
  for (int64_t v = v0 + threadIdx.x; v < v1; v += blockDim.x) {
    uint4 x[NR];
#pragma unroll
    for (int r = 0; r < NR; ++r) x[r] = st[r][v];  // all NR loads in flight before the adds
    float acc[8], f[8];
    unpack8(x[0], acc);
#pragma unroll
    for (int r = 1; r < NR; ++r) {
      unpack8(x[r], f);
#pragma unroll
      for (int i = 0; i < 8; ++i) acc[i] += f[i];
    }
    dst[v] = pack8(acc);
  }
  if (threadIdx.x == 0) epochs[b] = epoch;
}

// Max of int64 keys[n] over the ranks -> out_ids[i] = 0xffffffff - (low 32 bits of the max key).
// One block of 256 threads; signal block CFC_AR_SUM_BLOCKS; key area after the two staging buffers.
template <int NR>
__global__ void __launch_bounds__(256) oneshot_keymax_kernel(const int64_t* __restrict__ keys,
                                                             int32_t* __restrict__ out_ids, int n, ArPeers peers,
                                                             int rank, int64_t staging_bytes,
                                                             int* __restrict__ epochs, int* __restrict__ err) {
  constexpr int b = CFC_AR_SUM_BLOCKS;
  __shared__ int s_epoch, s_ok;
  if (threadIdx.x == 0) {
    s_epoch = epochs[b] + 1;
    s_ok = 1;
  }
  __syncthreads();
  const int epoch = s_epoch;
  const int64_t area = CFC_AR_SIGNAL_BYTES + 2 * staging_bytes + (int64_t)(epoch & 1) * CFC_AR_KEY_BYTES;
  int64_t* mine = reinterpret_cast<int64_t*>(peers.base[rank] + area);
  for (int i = threadIdx.x; i < n; i += blockDim.x) mine[i] = keys[i];
  __threadfence_system();
  __syncthreads();
  if (threadIdx.x < NR) {
    int* sig = reinterpret_cast<int*>(peers.base[threadIdx.x]) + b * CFC_AR_MAX_RANKS + rank;
    store_signal(sig, epoch);
  }
  if (threadIdx.x < NR) {
    const int* sig = reinterpret_cast<const int*>(peers.base[rank]) + b * CFC_AR_MAX_RANKS + threadIdx.x;
    unsigned spins = 0;
    while (load_signal(sig) < epoch) {
      __builtin_amdgcn_s_sleep(2);
      if (++spins > CFC_AR_SPIN_LIMIT) {
        s_ok = 0;
        break;
      }
    }
  }
  __syncthreads();
  __threadfence_system();
  if (!s_ok) {
    if (threadIdx.x == 0) {
      atomicAdd(err, 1);
      epochs[b] = epoch;
    }
    return;
  }
  for (int i = threadIdx.x; i < n; i += blockDim.x) {
    int64_t best = reinterpret_cast<const int64_t*>(peers.base[0] + area)[i];
#pragma unroll
    for (int r = 1; r < NR; ++r) {
      const int64_t k = reinterpret_cast<const int64_t*>(peers.base[r] + area)[i];
      best = k > best ? k : best;
    }
    out_ids[i] = (int32_t)(0xffffffffu - (uint32_t)(best & 0xffffffff));
  }
  if (threadIdx.x == 0) epochs[b] = epoch;
}

// One-shot all-reduce of fp32 split-K slabs + residual + RMSNorm (tensor-parallel decode, the
// row-parallel o / down projections).  TP = 1 runs "decode GEMM -> fp32 k-slice slabs ->
// splitk_residual_rmsnorm" (gemm.hip): the projection is rounded to bf16 ONCE, after the fp32 sum of
// every slab.  Here each rank holds the slabs of its K shard; the kernel sums them (fp32, slab
// order), exchanges the fp32 row sums through the peers' staging buffers, adds the ranks' sums in
// fixed rank order (fp32) and then applies exactly the reduce kernel's epilogue:
//   h = bf16(bf16(sum) + residual); residual <- h; out = bf16(h * rsqrt(mean(h^2) + eps) * w).
// So the only difference from TP = 1 is the association of the fp32 sum -- no extra bf16 rounding of
// the per-rank partials, and one launch replaces reduce + all-reduce + RMSNorm (three).  A block
// owns whole rows (rows b, b + nb, ...; N / 8 threads, one 8-column group each), so the row
// statistic of the norm is a block reduction after the exchange; the signal protocol, parities and
// bounded spins are oneshot_allreduce_kernel's (the staging rows are fp32: B x N x 4 bytes).
template <int NR>
__global__ void __launch_bounds__(1024) oneshot_ar_residual_rmsnorm_kernel(
    const float* __restrict__ part, int split, int M, int N, uint16_t* __restrict__ residual,
    const uint16_t* __restrict__ w, float eps, uint16_t* __restrict__ out, ArPeers peers, int rank,
    int64_t staging_bytes, int* __restrict__ epochs, int* __restrict__ err, int nb) {
  __shared__ float red[16];
  __shared__ int s_epoch, s_ok;
  const int b = blockIdx.x, c = threadIdx.x;    // c: 8-column group of a row
  if (b >= nb) {                    // idle block: keeps its epoch (and so the parity) in step
    if (threadIdx.x == 0) epochs[b] += 1;
    return;
  }
  if (threadIdx.x == 0) {
    s_epoch = epochs[b] + 1;
    s_ok = 1;
  }
  __syncthreads();
  const int epoch = s_epoch;
  const int64_t parity_off = CFC_AR_SIGNAL_BYTES + (int64_t)(epoch & 1) * staging_bytes;
  const bool act = c * 8 < N;
  const size_t slab = (size_t)M * N;

  // 1. this rank's fp32 row sums of its slabs -> own staging (uncached region: stores write through)
  float* mine = reinterpret_cast<float*>(peers.base[rank] + parity_off);
  for (int m = b; m < M; m += nb) {
    if (act) {
      float4 a = make_float4(0.f, 0.f, 0.f, 0.f), bb = a;
      slab_sum8(part, split, slab, (size_t)m * N + c * 8, a, bb);
      float4* dst = reinterpret_cast<float4*>(mine + (size_t)m * N + c * 8);
      dst[0] = a;
      dst[1] = bb;
    }
  }
  __threadfence_system();
  __syncthreads();
  // 2. arrive at every peer; 3. wait for every peer's arrival (lane j waits for rank j)
  if (threadIdx.x < NR) {
    int* sig = reinterpret_cast<int*>(peers.base[threadIdx.x]) + b * CFC_AR_MAX_RANKS + rank;
    store_signal(sig, epoch);
  }
  if (threadIdx.x < NR) {
    const int* sig = reinterpret_cast<const int*>(peers.base[rank]) + b * CFC_AR_MAX_RANKS + threadIdx.x;
    unsigned spins = 0;
    while (load_signal(sig) < epoch) {
      __builtin_amdgcn_s_sleep(2);
      if (++spins > CFC_AR_SPIN_LIMIT) {
        s_ok = 0;
        break;
      }
    }
  }
  __syncthreads();
  __threadfence_system();
  if (!s_ok) {
    if (threadIdx.x == 0) {
      atomicAdd(err, 1);
      epochs[b] = epoch;
    }
    return;
  }
  // 4. rows b, b + nb, ...: fixed-rank-order fp32 sum, then the reduce kernel's epilogue
  for (int m = b; m < M; m += nb) {
    float v[8];
    float ss = 0.f;
    uint4 wv = make_uint4(0, 0, 0, 0);
    uint4* rp = reinterpret_cast<uint4*>(residual + (size_t)m * N) + c;
    if (act) {
      float4 x[NR][2];
#pragma unroll
      for (int r = 0; r < NR; ++r) {      // every rank's loads in flight before the adds
        const float4* src = reinterpret_cast<const float4*>(peers.base[r] + parity_off) + ((size_t)m * N + c * 8) / 4;
        x[r][0] = src[0];
        x[r][1] = src[1];
      }
      const uint4 rr = *rp;
      wv = reinterpret_cast<const uint4*>(w)[c];
      float s8[8] = {x[0][0].x, x[0][0].y, x[0][0].z, x[0][0].w, x[0][1].x, x[0][1].y, x[0][1].z, x[0][1].w};
#pragma unroll
      for (int r = 1; r < NR; ++r) {
        s8[0] += x[r][0].x; s8[1] += x[r][0].y; s8[2] += x[r][0].z; s8[3] += x[r][0].w;
        s8[4] += x[r][1].x; s8[5] += x[r][1].y; s8[6] += x[r][1].z; s8[7] += x[r][1].w;
      }
      float rf[8];
      unpack8(rr, rf);
#pragma unroll
      for (int j = 0; j < 8; ++j) v[j] = bf2f(f2bf(s8[j])) + rf[j];
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
  if (threadIdx.x == 0) epochs[b] = epoch;
}

}  // namespace

// Shared region: signals + two staging buffers of `staging_bytes` + two key areas, uncached, zeroed.
CFC_API int cfc_ar_region_bytes(int64_t staging_bytes, int64_t* out) {
  if (staging_bytes <= 0 || staging_bytes % 16) return -1;
  *out = CFC_AR_SIGNAL_BYTES + 2 * staging_bytes + 2 * CFC_AR_KEY_BYTES;
  return 0;
}

CFC_API int cfc_ar_key_rows() { return CFC_AR_KEY_ROWS; }

CFC_API int cfc_ar_alloc(int64_t bytes, void** ptr) {
  hipError_t e = hipExtMallocWithFlags(ptr, (size_t)bytes, hipDeviceMallocUncached);
  if (e != hipSuccess) return (int)e;
  return (int)hipMemset(*ptr, 0, (size_t)bytes);
}

CFC_API int cfc_ar_free(void* ptr) { return (int)hipFree(ptr); }

CFC_API int cfc_ar_ipc_handle_size() { return (int)sizeof(hipIpcMemHandle_t); }

CFC_API int cfc_ar_ipc_handle(void* ptr, void* handle_out) {
  return (int)hipIpcGetMemHandle(reinterpret_cast<hipIpcMemHandle_t*>(handle_out), ptr);
}

CFC_API int cfc_ar_ipc_open(const void* handle, void** ptr) {
  hipIpcMemHandle_t h;
  __builtin_memcpy(&h, handle, sizeof(h));
  return (int)hipIpcOpenMemHandle(ptr, h, hipIpcMemLazyEnablePeerAccess);
}

CFC_API int cfc_ar_ipc_close(void* ptr) { return (int)hipIpcCloseMemHandle(ptr); }

// epochs arrays are CFC_AR_MAX_BLOCKS long; the sum uses at most CFC_AR_SUM_BLOCKS blocks
CFC_API int cfc_ar_max_blocks() { return CFC_AR_MAX_BLOCKS; }

// in/out: n bf16 (n % 8 == 0, 16-byte aligned, n * 2 <= staging_bytes); bases: `world` device
// pointers (this process's mapping of each rank's region, bases[rank] = own); epochs: int32
// [CFC_AR_MAX_BLOCKS] zero-initialised device array private to this rank; err: device int32.
CFC_API int cfc_oneshot_allreduce(const void* in, void* out, int64_t n, const void* const* bases, int world,
                                  int rank, int64_t staging_bytes, int blocks, int* epochs, int* err,
                                  hipStream_t stream) {
  if (world < 1 || world > CFC_AR_MAX_RANKS || rank < 0 || rank >= world) return -1;
  if (n <= 0 || n % 8 || n * 2 > staging_bytes || blocks < 1 || blocks > CFC_AR_SUM_BLOCKS) return -2;
  if (((uintptr_t)in | (uintptr_t)out) & 15) return -3;
  ArPeers peers{};
  for (int r = 0; r < world; ++r) peers.base[r] = (char*)bases[r];
  const int64_t n8 = n / 8;
  const int64_t want = (n8 + 255) / 256;
  const int nb = (int)(want < blocks ? want : blocks);
#define AR_CASE(NR) \
  case NR: \
    oneshot_allreduce_kernel<NR><<<CFC_AR_SUM_BLOCKS, 256, 0, stream>>>((const uint16_t*)in, (uint16_t*)out, n8, \
                                                                        peers, rank, staging_bytes, epochs, err, nb); \
    break;
  switch (world) {
    AR_CASE(1) AR_CASE(2) AR_CASE(3) AR_CASE(4) AR_CASE(5) AR_CASE(6) AR_CASE(7) AR_CASE(8)
    default: return -1;
  }
#undef AR_CASE
  return CFC_CHECK_LAUNCH();
}

// keys: n int64 (n <= CFC_AR_KEY_ROWS) per rank; out_ids: n int32 = 0xffffffff - low word of the
// max key over the ranks.  Same region / epochs / err as cfc_oneshot_allreduce.
CFC_API int cfc_oneshot_keymax(const int64_t* keys, int32_t* out_ids, int n, const void* const* bases, int world,
                               int rank, int64_t staging_bytes, int* epochs, int* err, hipStream_t stream) {
  if (world < 1 || world > CFC_AR_MAX_RANKS || rank < 0 || rank >= world) return -1;
  if (n <= 0 || n > CFC_AR_KEY_ROWS) return -2;
  ArPeers peers{};
  for (int r = 0; r < world; ++r) peers.base[r] = (char*)bases[r];
#define KM_CASE(NR) \
  case NR: \
    oneshot_keymax_kernel<NR><<<1, 256, 0, stream>>>(keys, out_ids, n, peers, rank, staging_bytes, epochs, err); \
    break;
  switch (world) {
    KM_CASE(1) KM_CASE(2) KM_CASE(3) KM_CASE(4) KM_CASE(5) KM_CASE(6) KM_CASE(7) KM_CASE(8)
    default: return -1;
  }
#undef KM_CASE
  return CFC_CHECK_LAUNCH();
}


// part: this rank's fp32 k-slice slabs [split, M, N] (its K shard of a row-parallel projection);
// residual (bf16 [M, N], updated in place), w (bf16 [N]), out (bf16 [M, N]) as
// cfc_splitk_residual_rmsnorm, with the projection summed over the TP group in fp32 first.
// M * N * 4 <= staging_bytes, N % 8 == 0, N <= 8192; blocks = row groups (<= CFC_AR_SUM_BLOCKS).
CFC_API int cfc_oneshot_ar_residual_rmsnorm(const float* part, int split, int M, int N, void* residual, const void* w,
                                            float eps, void* out, const void* const* bases, int world, int rank,
                                            int64_t staging_bytes, int blocks, int* epochs, int* err,
                                            hipStream_t stream) {
  if (world < 1 || world > CFC_AR_MAX_RANKS || rank < 0 || rank >= world) return -1;
  if (M <= 0 || N <= 0 || N % 8 || N / 8 > 1024 || split < 1 || (int64_t)M * N * 4 > staging_bytes) return -2;
  if (blocks < 1 || blocks > CFC_AR_SUM_BLOCKS) return -2;
  if ((((uintptr_t)part | (uintptr_t)residual | (uintptr_t)out | (uintptr_t)w) & 15)) return -3;
  ArPeers peers{};
  for (int r = 0; r < world; ++r) peers.base[r] = (char*)bases[r];
  const int nb = M < blocks ? M : blocks;
  const int threads = ((N / 8 + 63) / 64) * 64;
#define ARN_CASE(NR) \
  case NR: \
    oneshot_ar_residual_rmsnorm_kernel<NR><<<CFC_AR_SUM_BLOCKS, threads, 0, stream>>>(part, split, M, N, \
        (uint16_t*)residual, (const uint16_t*)w, eps, (uint16_t*)out, peers, rank, staging_bytes, epochs, err, nb); \
    break;
  switch (world) {
    ARN_CASE(1) ARN_CASE(2) ARN_CASE(3) ARN_CASE(4) ARN_CASE(5) ARN_CASE(6) ARN_CASE(7) ARN_CASE(8)
    default: return -1;
  }
#undef ARN_CASE
  return CFC_CHECK_LAUNCH();
}
