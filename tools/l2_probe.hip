// Diagnostic: does an XCD's L2 keep lines written by the previous kernel on the same
// stream?  Kernel W: block b writes slice (b % 8) of a 16 MB buffer (2 MB per slice,
// block b lands on XCD b % 8 under round-robin placement); kernel R: block b reads slice
// (b + shift) % 8 - shift 0 reads what its own XCD wrote, shift 1 what another wrote.
// Timed with events (python tools/l2_probe.py) and under rocprofv3 --pmc FETCH_SIZE.
//   hipcc --offload-arch=gfx950 -O3 -shared -fPIC tools/l2_probe.hip -o tools/libl2probe.so
#include <hip/hip_runtime.h>
#include <cstdint>

constexpr int kSlices = 8;

__global__ void k_l2_write(float4* __restrict__ buf, int64_t per_slice, int blocks_per_slice, float v) {
  const int slice = blockIdx.x % kSlices, j = blockIdx.x / kSlices;
  float4* p = buf + int64_t(slice) * per_slice;
  for (int64_t i = int64_t(j) * blockDim.x + threadIdx.x; i < per_slice; i += int64_t(blocks_per_slice) * blockDim.x)
    p[i] = make_float4(v, v, v, v);
}

__global__ void k_l2_read(const float4* __restrict__ buf, int64_t per_slice, int blocks_per_slice, int shift,
                          float* out) {
  const int slice = (blockIdx.x + shift) % kSlices, j = blockIdx.x / kSlices;
  const float4* p = buf + int64_t(slice) * per_slice;
  float acc = 0.f;
  for (int64_t i = int64_t(j) * blockDim.x + threadIdx.x; i < per_slice; i += int64_t(blocks_per_slice) * blockDim.x) {
    const float4 v = p[i];
    acc += v.x + v.y + v.z + v.w;
  }
  if (acc == 123.456f) out[0] = acc;
}

extern "C" int l2p_write(void* buf, int64_t bytes, int blocks_per_slice, float v, void* s) {
  hipLaunchKernelGGL(k_l2_write, dim3(kSlices * blocks_per_slice), dim3(256), 0, (hipStream_t)s,
                     (float4*)buf, bytes / 16 / kSlices, blocks_per_slice, v);
  return hipGetLastError();
}
extern "C" int l2p_read(void* buf, int64_t bytes, int blocks_per_slice, int shift, float* out, void* s) {
  hipLaunchKernelGGL(k_l2_read, dim3(kSlices * blocks_per_slice), dim3(256), 0, (hipStream_t)s,
                     (const float4*)buf, bytes / 16 / kSlices, blocks_per_slice, shift, out);
  return hipGetLastError();
}
