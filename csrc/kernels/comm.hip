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
// arguments and is captured into the decode hipGraph like any other kernel.
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
                                                                int* __restrict__ epochs, int* __restrict__ err) {
  const int b = blockIdx.x;
  __shared__ int s_epoch, s_ok;
  if (threadIdx.x == 0) {
    s_epoch = epochs[b] + 1;
    s_ok = 1;
  }
  __syncthreads();
  const int epoch = s_epoch;
  const int64_t per = (n8 + gridDim.x - 1) / gridDim.x;
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
    oneshot_allreduce_kernel<NR><<<nb, 256, 0, stream>>>((const uint16_t*)in, (uint16_t*)out, n8, peers, rank, \
                                                         staging_bytes, epochs, err); \
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
