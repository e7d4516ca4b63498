// Diagnostic for VERDICT r05 item 1 (the per-XCD persistent chain): does a latency-bound
// gather chain that hits its XCD's L2 escape the slowdown the paced pass over X inflicts on the
// chain's kernels (conv2 20.7 -> 81 us in-step), and does that L2 content survive a kernel
// boundary?  The chain's loads are 256-byte rows (64 fp32, one aggregation neighbour) in
// dependent rounds; the pass is 16-B non-temporal loads over ~600 MB.
//
//   k_l2_warm   each block reads every row of its XCD's part of the table (HW_REG_XCC_ID)
//   k_l2_chain  each wave runs `steps` dependent rounds of 8 row gathers (two 16-B loads per
//               lane, 4 rows per load: 16 lanes per row), the next rows picked from a hash of
//               what lane 0 loaded; rows from part (xcc + shift) % 8: shift 0 = the XCD's own
//               (warmed) part, 4 = a part another XCD warmed.  warm=1 warms inside the same
//               launch first (block-local: the block reads the whole part, then a barrier).
//               Per wave, wall_clock64 (100 MHz) brackets the dependent rounds only.
//   k_l2_stream the pass: `passes` non-temporal sweeps over X.
//   hipcc --offload-arch=gfx950 -O3 -shared -fPIC tools/l2_stream_probe.hip -o tools/libl2streamprobe.so
#include <hip/hip_runtime.h>
#include <cstdint>

typedef unsigned int v4u __attribute__((ext_vector_type(4)));
typedef float v4f __attribute__((ext_vector_type(4)));

__device__ __forceinline__ unsigned xcc_id() { return __builtin_amdgcn_s_getreg((3 << 11) | 20) & 7u; }
__device__ __forceinline__ unsigned hash32(unsigned x) {
  x ^= x >> 16; x *= 0x7feb352dU; x ^= x >> 15; x *= 0x846ca68bU; x ^= x >> 16;
  return x;
}

__global__ __launch_bounds__(256) void k_l2_warm(const v4f* __restrict__ table, int part_rows, float* sink) {
  const unsigned x = xcc_id();
  const v4f* p = table + int64_t(x) * part_rows * 16;
  v4f acc = {0, 0, 0, 0};
  for (int i = threadIdx.x; i < part_rows * 16; i += 256) acc += p[i];
  if (acc.x == 1234.5f) sink[0] = acc.y;
}

__global__ __launch_bounds__(256) void k_l2_chain(const v4f* __restrict__ table, int part_rows, int shift, int warm,
                                                  int steps, int64_t* __restrict__ times, float* sink) {
  const unsigned x = xcc_id();
  if (warm) {
    const v4f* w = table + int64_t(x) * part_rows * 16;
    v4f a = {0, 0, 0, 0};
    for (int i = threadIdx.x; i < part_rows * 16; i += 256) a += w[i];
    if (a.x == 1234.5f) sink[1] = a.y;
    __syncthreads();
  }
  const v4f* p = table + int64_t((x + shift) & 7) * part_rows * 16;
  const int lane = threadIdx.x & 63, sub = lane >> 4, c = lane & 15;
  const int wave = blockIdx.x * 4 + (threadIdx.x >> 6);
  unsigned st = hash32(wave * 2654435761u + 17);
  v4f acc = {0, 0, 0, 0};
  const int64_t t0 = wall_clock64();
  for (int s = 0; s < steps; ++s) {
    const unsigned r0 = hash32(st * 8 + sub * 2) & unsigned(part_rows - 1);
    const unsigned r1 = hash32(st * 8 + sub * 2 + 1) & unsigned(part_rows - 1);
    const v4f a = p[int64_t(r0) * 16 + c];
    const v4f b = p[int64_t(r1) * 16 + c];
    acc += a + b;
    st = hash32(st ^ __builtin_amdgcn_readfirstlane(__float_as_uint(a.x) ^ __float_as_uint(b.y)));
  }
  const int64_t t1 = wall_clock64();
  if (lane == 0) times[wave] = t1 - t0;
  if (acc.x == 1234.5f) sink[2] = acc.y;
}

// four 16-B loads in flight per lane (the pass keeps several in flight too)
__global__ __launch_bounds__(256) void k_l2_stream(const v4u* __restrict__ buf, int64_t n16, int passes, unsigned* out) {
  unsigned acc = 0;
  const int64_t step = int64_t(gridDim.x) * 256;
  for (int p = 0; p < passes; ++p)
    for (int64_t i = int64_t(blockIdx.x) * 256 + threadIdx.x; i < n16; i += 4 * step) {
      v4u v[4];
#pragma unroll
      for (int u = 0; u < 4; ++u) v[u] = __builtin_nontemporal_load(buf + min(i + u * step, n16 - 1));
#pragma unroll
      for (int u = 0; u < 4; ++u) acc ^= v[u].x ^ v[u].y ^ v[u].z ^ v[u].w;
    }
  if (acc == 0x9E3779B9u) out[0] = acc;
}

extern "C" int l2_wallclock_khz() {
  int v = 0;
  if (hipDeviceGetAttribute(&v, hipDeviceAttributeWallClockRate, 0) != hipSuccess) return -1;
  return v;
}
// a stream on the CUs i with (i % every == every - 1) != complement (every <= 1: no mask)
extern "C" int l2_stream_create(int every, int complement, void** out) {
  hipStream_t st;
  if (every <= 1) {
    if (hipStreamCreateWithFlags(&st, hipStreamNonBlocking) != hipSuccess) return -1;
  } else {
    hipDeviceProp_t prop;
    if (hipGetDeviceProperties(&prop, 0) != hipSuccess) return -1;
    const int ncu = prop.multiProcessorCount;
    uint32_t mask[16] = {0};
    if (ncu > 512) return -2;
    for (int i = 0; i < ncu; ++i)
      if ((i % every == every - 1) != bool(complement)) mask[i / 32] |= 1u << (i % 32);
    if (hipExtStreamCreateWithCUMask(&st, uint32_t((ncu + 31) / 32), mask) != hipSuccess) return -3;
  }
  *out = st;
  return 0;
}
extern "C" int l2_warm(const void* table, int part_rows, float* sink, int blocks, void* s) {
  hipLaunchKernelGGL(k_l2_warm, dim3(blocks), dim3(256), 0, (hipStream_t)s, (const v4f*)table, part_rows, sink);
  return hipGetLastError();
}
extern "C" int l2_chain(const void* table, int part_rows, int shift, int warm, int steps, int blocks, int64_t* times,
                        float* sink, void* s) {
  hipLaunchKernelGGL(k_l2_chain, dim3(blocks), dim3(256), 0, (hipStream_t)s, (const v4f*)table, part_rows, shift, warm,
                     steps, times, sink);
  return hipGetLastError();
}
extern "C" int l2_stream(const void* buf, int64_t bytes, int passes, int blocks, unsigned* out, void* s) {
  hipLaunchKernelGGL(k_l2_stream, dim3(blocks), dim3(256), 0, (hipStream_t)s, (const v4u*)buf, bytes / 16, passes, out);
  return hipGetLastError();
}
