// Probe only (not part of libcfc_kernels): how fast can 8-wave workgroups stream a row-major
// [N, K] bf16 weight matrix, as a function of the per-instruction access shape?  Each wave owns
// 16 rows; one load instruction covers RPI rows x (1024 / RPI) contiguous bytes per row (lane l:
// row l / (64 / RPI), 16-B chunk l % (64 / RPI)).  RPI = 16 is the MFMA B-fragment shape
// (16 rows x 64 B), RPI = 1 the GEMV shape (1 KB of one row).  D steps of 16 rows x (1024/RPI) B
// stay in flight per wave.  ROT: workgroups start at different K offsets.
#include <hip/hip_runtime.h>
#include <stdint.h>

template <int RPI, int D, bool ROT>
__global__ void __launch_bounds__(512) stream_kernel(const uint16_t* __restrict__ W, int N, int K, float* out) {
  constexpr int LPR = 64 / RPI;                  // lanes per row
  constexpr int BPR = 16 * LPR;                  // bytes per row per instruction
  constexpr int IPS = 16 / RPI;                  // instructions per step (16 rows)
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
  const int row0 = blockIdx.x * 128 + 16 * w;
  const int nsteps = K * 2 / BPR;
  const int rot = ROT ? (int)((blockIdx.x * 37u) % (unsigned)nsteps) : 0;
  const uint16_t* base = W + (size_t)(row0 + lane / LPR) * K + (lane % LPR) * 8;
  uint4 ring[D][IPS];
  auto ld = [&](int s, uint4 (&dst)[IPS]) {
    s += rot; if (s >= nsteps) s -= nsteps;
#pragma unroll
    for (int i = 0; i < IPS; ++i) dst[i] = *reinterpret_cast<const uint4*>(base + (size_t)i * RPI * K + s * (BPR / 2));
  };
#pragma unroll
  for (int p = 0; p < D; ++p) ld(p < nsteps ? p : nsteps - 1, ring[p]);
  unsigned acc = 0;
  int st = 0;
  for (; st + D <= nsteps; st += D) {
#pragma unroll
    for (int u = 0; u < D; ++u) {
#pragma unroll
      for (int i = 0; i < IPS; ++i) acc ^= ring[u][i].x + ring[u][i].y + ring[u][i].z + ring[u][i].w;
      ld(min(st + u + D, nsteps - 1), ring[u]);
    }
  }
#pragma unroll
  for (int u = 0; u < D; ++u)
#pragma unroll
    for (int i = 0; i < IPS; ++i) acc ^= ring[u][i].x;
  if (acc == 0x12345678u) out[0] = 1.f;
}

#define SP_CASE(R, DD, RT)                                                                          \
  if (rpi == R && d == DD && rot == RT) {                                                           \
    stream_kernel<R, DD, RT><<<N / 128, 512, 0, st>>>((const uint16_t*)w, N, K, out);               \
    return (int)hipGetLastError();                                                                  \
  }
extern "C" int stream_probe(const void* w, int N, int K, int rpi, int d, int rot, float* out, hipStream_t st) {
  if (N % 128) return -1;
  SP_CASE(1, 2, 0) SP_CASE(1, 2, 1) SP_CASE(2, 2, 1) SP_CASE(2, 4, 1) SP_CASE(4, 4, 1) SP_CASE(4, 8, 1)
  SP_CASE(8, 8, 1) SP_CASE(8, 16, 1) SP_CASE(16, 16, 0) SP_CASE(16, 16, 1) SP_CASE(16, 32, 1) SP_CASE(16, 8, 1)
  return -2;
}

// Flat stream: the matrix read as one contiguous byte array.  Workgroup b of G owns a contiguous
// span; its NWV waves interleave 1-KB pieces (wave w takes pieces w, w+NWV, ...) with F pieces in
// flight per wave.  Upper bound for any weight-stream layout at a given grid and concurrency.
template <int F>
__global__ void __launch_bounds__(512) flat_kernel(const uint4* __restrict__ W, size_t n16, int nwv, float* out) {
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
  if (w >= nwv) return;
  const size_t pieces = n16 / 64;
  const size_t per = (pieces + gridDim.x - 1) / gridDim.x;
  const size_t p0 = blockIdx.x * per, p1 = min(pieces, p0 + per);
  unsigned acc = 0;
  size_t p = p0 + w;
  uint4 r[F];
  for (; p + (size_t)(F - 1) * nwv < p1; p += (size_t)F * nwv) {
#pragma unroll
    for (int i = 0; i < F; ++i) r[i] = W[(p + (size_t)i * nwv) * 64 + lane];
#pragma unroll
    for (int i = 0; i < F; ++i) acc ^= r[i].x + r[i].y + r[i].z + r[i].w;
  }
  for (; p < p1; p += nwv) acc ^= W[p * 64 + lane].x;
  if (acc == 0x12345678u) out[0] = 1.f;
}

extern "C" int flat_probe(const void* w, size_t bytes, int grid, int nwv, int f, float* out, hipStream_t st) {
  const size_t n16 = bytes / 16;
  switch (f) {
    case 4: flat_kernel<4><<<grid, 64 * nwv, 0, st>>>((const uint4*)w, n16, nwv, out); break;
    case 8: flat_kernel<8><<<grid, 64 * nwv, 0, st>>>((const uint4*)w, n16, nwv, out); break;
    case 16: flat_kernel<16><<<grid, 64 * nwv, 0, st>>>((const uint4*)w, n16, nwv, out); break;
    default: return -2;
  }
  return (int)hipGetLastError();
}
