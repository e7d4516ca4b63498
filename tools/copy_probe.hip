// Streaming ceiling probe: how fast can one kernel read 614 MB and write 614 MB on this
// box (the byte count of the 5000-wide aggregation A_hat . X at N = 30,720)?  Variants:
// grid-stride float4 copy with default / non-temporal loads and stores, various grids.
//   hipcc --offload-arch=gfx950 -O3 -o tools/copy_probe tools/copy_probe.hip && tools/copy_probe
#include <hip/hip_runtime.h>
#include <stdio.h>

typedef float f32x4 __attribute__((ext_vector_type(4)));

template <int LD, int ST, int UNROLL>
__global__ __launch_bounds__(256) void k_copy(const f32x4* __restrict__ a, f32x4* __restrict__ b, size_t n) {
  const size_t stride = size_t(gridDim.x) * 256 * UNROLL;
  for (size_t i = size_t(blockIdx.x) * 256 * UNROLL + threadIdx.x; i < n; i += stride) {
    f32x4 v[UNROLL];
#pragma unroll
    for (int u = 0; u < UNROLL; ++u) {
      const size_t k = i + size_t(u) * 256;
      const size_t kk = k < n ? k : n - 1;
      v[u] = LD ? __builtin_nontemporal_load(a + kk) : a[kk];
    }
#pragma unroll
    for (int u = 0; u < UNROLL; ++u) {
      const size_t k = i + size_t(u) * 256;
      if (k < n) {
        if (ST) __builtin_nontemporal_store(v[u], b + k);
        else b[k] = v[u];
      }
    }
  }
}

template <int LD, int ST, int UNROLL>
static void run(const char* name, const f32x4* a, f32x4* b, size_t n, int blocks) {
  hipEvent_t e0, e1;
  hipEventCreate(&e0);
  hipEventCreate(&e1);
  for (int i = 0; i < 3; ++i) hipLaunchKernelGGL((k_copy<LD, ST, UNROLL>), dim3(blocks), dim3(256), 0, 0, a, b, n);
  hipEventRecord(e0, 0);
  const int it = 20;
  for (int i = 0; i < it; ++i) hipLaunchKernelGGL((k_copy<LD, ST, UNROLL>), dim3(blocks), dim3(256), 0, 0, a, b, n);
  hipEventRecord(e1, 0);
  hipEventSynchronize(e1);
  float ms = 0;
  hipEventElapsedTime(&ms, e0, e1);
  ms /= it;
  printf("%-28s blocks %6d  %7.1f us  %6.0f GB/s (read+write)\n", name, blocks, ms * 1e3,
         2.0 * n * 16 / (ms * 1e-3) / 1e9);
}

// row-structured copies of a [rows, 5000] fp32 matrix (the aggregation's shape):
// a wave copies RPW consecutive rows, each as SL slices of Q float4 per lane (SL*Q*64*4
// floats >= 5000), one slice per wave; blockDim 256.
template <int Q, int RPW>
__global__ __launch_bounds__(256) void k_rows(const float* __restrict__ a, float* __restrict__ b, int rows, int F, int slices) {
  const int lane = threadIdx.x & 63;
  const long w = long(blockIdx.x) * 4 + (threadIdx.x >> 6);
  const long chunk = w / slices;
  const int s = int(w % slices);
  const long r0 = chunk * RPW;
  if (r0 >= rows) return;
#pragma unroll 1
  for (int k = 0; k < RPW; ++k) {
    const long r = r0 + k;
    if (r >= rows) break;
    f32x4 v[Q];
#pragma unroll
    for (int j = 0; j < Q; ++j) {
      const int c = s * Q * 256 + (j * 64 + lane) * 4;
      const int cc = c < F ? c : 0;
      v[j] = __builtin_nontemporal_load(reinterpret_cast<const f32x4*>(a + r * F + cc));
    }
#pragma unroll
    for (int j = 0; j < Q; ++j) {
      const int c = s * Q * 256 + (j * 64 + lane) * 4;
      if (c < F) __builtin_nontemporal_store(v[j], reinterpret_cast<f32x4*>(b + r * F + c));
    }
  }
}

template <int Q, int RPW>
static void run_rows(const char* name, const float* a, float* b, int rows, int F) {
  const int slices = (F + Q * 256 - 1) / (Q * 256);
  const long waves = long((rows + RPW - 1) / RPW) * slices;
  const int blocks = int((waves + 3) / 4);
  hipEvent_t e0, e1;
  hipEventCreate(&e0);
  hipEventCreate(&e1);
  for (int i = 0; i < 3; ++i) hipLaunchKernelGGL((k_rows<Q, RPW>), dim3(blocks), dim3(256), 0, 0, a, b, rows, F, slices);
  hipEventRecord(e0, 0);
  const int it = 20;
  for (int i = 0; i < it; ++i) hipLaunchKernelGGL((k_rows<Q, RPW>), dim3(blocks), dim3(256), 0, 0, a, b, rows, F, slices);
  hipEventRecord(e1, 0);
  hipEventSynchronize(e1);
  float ms = 0;
  hipEventElapsedTime(&ms, e0, e1);
  ms /= it;
  printf("rows Q=%2d RPW=%2d %-10s blocks %6d  %7.1f us  %6.0f GB/s (read+write)\n", Q, RPW, name, blocks,
         ms * 1e3, 2.0 * rows * F * 4 / (ms * 1e-3) / 1e9);
}

int main() {
  const size_t bytes = size_t(30720) * 5000 * 4;
  const size_t n = bytes / 16;
  f32x4 *a, *b;
  hipMalloc(&a, bytes);
  hipMalloc(&b, bytes);
  hipMemset(a, 1, bytes);
  hipMemset(b, 0, bytes);
  for (int blocks : {1024, 2048, 4096, 8192}) {
    run<0, 0, 4>("default ld / default st x4", a, b, n, blocks);
    run<1, 1, 4>("nt ld / nt st x4", a, b, n, blocks);
    run<0, 1, 4>("default ld / nt st x4", a, b, n, blocks);
    run<1, 1, 8>("nt ld / nt st x8", a, b, n, blocks);
  }
  run<1, 1, 1>("nt ld / nt st x1 (1 per thread)", a, b, n, int((n + 255) / 256));
  run<0, 0, 1>("default x1 (1 per thread)", a, b, n, int((n + 255) / 256));
  const float* af = reinterpret_cast<const float*>(a);
  float* bf = reinterpret_cast<float*>(b);
  run_rows<20, 1>("", af, bf, 30720, 5000);
  run_rows<20, 8>("", af, bf, 30720, 5000);
  run_rows<10, 1>("", af, bf, 30720, 5000);
  run_rows<10, 8>("", af, bf, 30720, 5000);
  run_rows<5, 1>("", af, bf, 30720, 5000);
  run_rows<5, 8>("", af, bf, 30720, 5000);
  run_rows<2, 1>("", af, bf, 30720, 5000);
  run_rows<1, 1>("", af, bf, 30720, 5000);
  return 0;
}
