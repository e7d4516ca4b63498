// Diagnostic: what rocprofv3's FETCH_SIZE counter reports on gfx950 for known traffic, per
// access pattern - the correction tools/prof.py applies (x2) was derived for wide streaming
// reads (MI355X_MICROARCH.md); k_bwd_tail's dZ1 traffic is 128-byte gathers (VERDICT r05
// weak #2 asked whether x2 holds for them).  Each kernel reads a known number of DISTINCT
// bytes once, from a 1 GiB buffer (beyond L2 and the 256 MB Infinity Cache):
//   k_fp_stream    16 B per lane, consecutive (a wide streaming read)
//   k_fp_gather<P> P-byte pieces (P / 16 lanes, 16 B each) at a permuted piece index
//                  (piece k -> (k * 40503 + 7) mod pieces: distinct, scattered)
//   hipcc --offload-arch=gfx950 -O3 -shared -fPIC tools/fetch_probe.hip -o tools/libfetchprobe.so
#include <hip/hip_runtime.h>
#include <cstdint>

typedef unsigned int v4u __attribute__((ext_vector_type(4)));

__global__ __launch_bounds__(256) void k_fp_stream(const v4u* __restrict__ buf, int64_t n16, unsigned* out) {
  unsigned acc = 0;
  for (int64_t i = int64_t(blockIdx.x) * 256 + threadIdx.x; i < n16; i += int64_t(gridDim.x) * 256) {
    const v4u v = buf[i];
    acc ^= v.x ^ v.y ^ v.z ^ v.w;
  }
  if (acc == 0x9E3779B9u) out[0] = acc;
}

template <int P>
__global__ __launch_bounds__(256) void k_fp_gather(const v4u* __restrict__ buf, int64_t pieces, int64_t count,
                                                   unsigned* out) {
  constexpr int L = P / 16;   // lanes per piece
  unsigned acc = 0;
  const int64_t groups = int64_t(gridDim.x) * (256 / L);
  for (int64_t k = int64_t(blockIdx.x) * (256 / L) + threadIdx.x / L; k < count; k += groups) {
    const int64_t piece = (k * 40503 + 7) % pieces;
    const v4u v = buf[piece * L + threadIdx.x % L];
    acc ^= v.x ^ v.y ^ v.z ^ v.w;
  }
  if (acc == 0x9E3779B9u) out[0] = acc;
}

extern "C" int fp_stream(const void* buf, int64_t bytes, unsigned* out, void* s) {
  hipLaunchKernelGGL(k_fp_stream, dim3(4096), dim3(256), 0, (hipStream_t)s, (const v4u*)buf, bytes / 16, out);
  return hipGetLastError();
}
extern "C" int fp_gather(int piece_bytes, const void* buf, int64_t bytes, int64_t count, unsigned* out, void* s) {
  const int64_t pieces = bytes / piece_bytes;
  switch (piece_bytes) {
    case 64: hipLaunchKernelGGL(k_fp_gather<64>, dim3(4096), dim3(256), 0, (hipStream_t)s, (const v4u*)buf, pieces, count, out); break;
    case 128: hipLaunchKernelGGL(k_fp_gather<128>, dim3(4096), dim3(256), 0, (hipStream_t)s, (const v4u*)buf, pieces, count, out); break;
    case 256: hipLaunchKernelGGL(k_fp_gather<256>, dim3(4096), dim3(256), 0, (hipStream_t)s, (const v4u*)buf, pieces, count, out); break;
    default: return -1;
  }
  return hipGetLastError();
}
