// Diagnostic side-stream jobs for tools/interfere_probe.py: what kind of concurrent
// activity slows the latency-bound training chain (CU occupancy / clocks, L2 or
// Infinity-Cache traffic, HBM streaming, page-translation pressure)?
//   hipcc --offload-arch=gfx950 -O3 -shared -fPIC tools/interfere.hip -o tools/libinterfere.so
#include <hip/hip_runtime.h>
#include <cstdint>

// ALU only: every lane runs `iters` dependent FMA rounds (no memory traffic)
__global__ void k_alu(int iters, float* out) {
  float a = threadIdx.x * 1e-3f, b = 1.0001f, c = 0.9999f;
  for (int i = 0; i < iters; ++i) {
    a = fmaf(a, b, c);
    b = fmaf(b, c, a * 1e-9f);
  }
  if (a == 12345.f) out[0] = b;
}

// reads n16 16-byte words of buf `reps` times, grid-stride (lane-contiguous)
__global__ void k_read(const uint4* __restrict__ buf, int64_t n16, int reps, uint32_t* out) {
  uint32_t acc = 0;
  const int64_t stride = int64_t(gridDim.x) * blockDim.x;
  for (int r = 0; r < reps; ++r)
    for (int64_t i = int64_t(blockIdx.x) * blockDim.x + threadIdx.x; i < n16; i += stride) {
      const uint4 v = buf[i];
      acc ^= v.x ^ v.y ^ v.z ^ v.w;
    }
  if (acc == 0x9e3779b9u) out[0] = acc;
}

// page-hopping reads: each lane reads one 16-byte word per 64 KiB page, walking the
// buffer; little bandwidth, many distinct pages (translation pressure)
__global__ void k_pages(const uint4* __restrict__ buf, int64_t n16, int reps, uint32_t* out) {
  uint32_t acc = 0;
  const int64_t step = 4096;  // 64 KiB in 16-byte words
  const int64_t lanes = int64_t(gridDim.x) * blockDim.x;
  const int64_t t = int64_t(blockIdx.x) * blockDim.x + threadIdx.x;
  for (int r = 0; r < reps; ++r)
    for (int64_t p = t; p * step < n16; p += lanes) {
      const uint4 v = buf[(p * step + r * 17) % n16];
      acc ^= v.x;
    }
  if (acc == 0x9e3779b9u) out[0] = acc;
}

extern "C" int ifr_alu(int blocks, int iters, float* out, void* stream) {
  hipLaunchKernelGGL(k_alu, dim3(blocks), dim3(256), 0, (hipStream_t)stream, iters, out);
  return hipGetLastError();
}
extern "C" int ifr_read(const void* buf, int64_t bytes, int blocks, int reps, uint32_t* out, void* stream) {
  hipLaunchKernelGGL(k_read, dim3(blocks), dim3(256), 0, (hipStream_t)stream,
                     (const uint4*)buf, bytes / 16, reps, out);
  return hipGetLastError();
}
extern "C" int ifr_pages(const void* buf, int64_t bytes, int blocks, int reps, uint32_t* out, void* stream) {
  hipLaunchKernelGGL(k_pages, dim3(blocks), dim3(256), 0, (hipStream_t)stream,
                     (const uint4*)buf, bytes / 16, reps, out);
  return hipGetLastError();
}

// the same streaming read through a buffer descriptor with cache policy AUX on every
// load (gfx950 CPol bits: 1 = sc0, 2 = nt, 16 = sc1): does the policy of the stream
// change what it costs the chain beside it (Infinity-Cache allocation, queueing)?
template <int AUX>
__global__ void k_read_pol(const uint4* __restrict__ buf, int64_t n16, int reps, uint32_t* out) {
  uint32_t acc = 0;
  const __amdgpu_buffer_rsrc_t rs = __builtin_amdgcn_make_buffer_rsrc(
      const_cast<uint4*>(buf), 0, uint32_t(n16 * 16 > 0xffffffffll ? 0xffffffffll : n16 * 16), 0x00020000);
  const int64_t stride = int64_t(gridDim.x) * blockDim.x;
  for (int r = 0; r < reps; ++r)
    for (int64_t i = int64_t(blockIdx.x) * blockDim.x + threadIdx.x; i < n16; i += 4 * stride) {
      typedef unsigned int u4 __attribute__((ext_vector_type(4)));
      u4 v[4];
#pragma unroll
      for (int u = 0; u < 4; ++u)
        v[u] = __builtin_amdgcn_raw_buffer_load_b128(rs, uint32_t((i + u * stride) * 16), 0, AUX);
#pragma unroll
      for (int u = 0; u < 4; ++u) acc ^= v[u].x ^ v[u].y ^ v[u].z ^ v[u].w;
    }
  if (acc == 0x9e3779b9u) out[0] = acc;
}

extern "C" int ifr_read_pol(const void* buf, int64_t bytes, int blocks, int reps, int aux, uint32_t* out,
                            void* stream) {
  const uint4* b = (const uint4*)buf;
  hipStream_t s = (hipStream_t)stream;
  const int64_t n = bytes / 16;
  switch (aux) {
    case 0: hipLaunchKernelGGL(k_read_pol<0>, dim3(blocks), dim3(256), 0, s, b, n, reps, out); break;
    case 1: hipLaunchKernelGGL(k_read_pol<1>, dim3(blocks), dim3(256), 0, s, b, n, reps, out); break;
    case 2: hipLaunchKernelGGL(k_read_pol<2>, dim3(blocks), dim3(256), 0, s, b, n, reps, out); break;
    case 3: hipLaunchKernelGGL(k_read_pol<3>, dim3(blocks), dim3(256), 0, s, b, n, reps, out); break;
    case 16: hipLaunchKernelGGL(k_read_pol<16>, dim3(blocks), dim3(256), 0, s, b, n, reps, out); break;
    case 17: hipLaunchKernelGGL(k_read_pol<17>, dim3(blocks), dim3(256), 0, s, b, n, reps, out); break;
    case 18: hipLaunchKernelGGL(k_read_pol<18>, dim3(blocks), dim3(256), 0, s, b, n, reps, out); break;
    case 19: hipLaunchKernelGGL(k_read_pol<19>, dim3(blocks), dim3(256), 0, s, b, n, reps, out); break;
    default: return -1;
  }
  return hipGetLastError();
}

// device buffers with an allocation flag (0 = hipMalloc default / coarse-grained,
// 1 = fine-grained, 3 = uncached): does the placement of a streamed buffer change what
// its stream costs the chain (cache pollution)?
extern "C" void* ifr_alloc(int64_t bytes, int flags) {
  void* p = nullptr;
  if (flags == 0) { if (hipMalloc(&p, bytes) != hipSuccess) return nullptr; }
  else if (hipExtMallocWithFlags(&p, bytes, unsigned(flags)) != hipSuccess) return nullptr;
  if (hipMemset(p, 1, bytes) != hipSuccess) return nullptr;
  return p;
}
extern "C" int ifr_free(void* p) { return hipFree(p); }
