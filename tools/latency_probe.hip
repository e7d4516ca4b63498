// Diagnostic: per-launch cost of back-to-back dependent kernels on one stream and the
// cost of a dependent global-memory round trip, on the device this runs on.
#include <hip/hip_runtime.h>
#include <cstdio>
#include <vector>

__global__ void k_empty() {}

// each thread follows `hops` dependent loads through a random permutation
__global__ void k_chase(const int* __restrict__ next, int hops, int* out, int n) {
  int i = (blockIdx.x * blockDim.x + threadIdx.x) % n;
  for (int h = 0; h < hops; ++h) i = next[i];
  if (i == -1) out[0] = i;
}

static float time_it(int reps, void (*launch)(hipStream_t), hipStream_t s) {
  hipEvent_t a, b;
  hipEventCreate(&a); hipEventCreate(&b);
  launch(s);
  hipStreamSynchronize(s);
  hipEventRecord(a, s);
  for (int r = 0; r < reps; ++r) launch(s);
  hipEventRecord(b, s);
  hipEventSynchronize(b);
  float ms = 0; hipEventElapsedTime(&ms, a, b);
  return ms * 1000.f / reps;
}

static int* g_next; static int* g_out; static int g_n; static int g_hops; static int g_grid;
static void l_empty1(hipStream_t s) { hipLaunchKernelGGL(k_empty, dim3(1), dim3(64), 0, s); }
static void l_emptyN(hipStream_t s) { hipLaunchKernelGGL(k_empty, dim3(g_grid), dim3(256), 0, s); }
static void l_chase(hipStream_t s) { hipLaunchKernelGGL(k_chase, dim3(g_grid), dim3(256), 0, s, g_next, g_hops, g_out, g_n); }

int main() {
  hipStream_t s; hipStreamCreateWithFlags(&s, hipStreamNonBlocking);
  g_n = 16 << 20;   // 64 MB of int: beyond L2, inside the Infinity Cache
  std::vector<int> perm(g_n);
  for (int i = 0; i < g_n; ++i) perm[i] = i;
  unsigned x = 12345;
  for (int i = g_n - 1; i > 0; --i) { x = x * 1664525u + 1013904223u; int j = x % (i + 1); std::swap(perm[i], perm[j]); }
  hipMalloc(&g_next, g_n * sizeof(int)); hipMalloc(&g_out, 64);
  hipMemcpy(g_next, perm.data(), g_n * sizeof(int), hipMemcpyHostToDevice);
  printf("empty kernel, 1 block          : %6.2f us/launch\n", time_it(200, l_empty1, s));
  for (int gsz : {256, 1024, 4096, 16384}) {
    g_grid = gsz;
    printf("empty kernel, %5d x 256       : %6.2f us/launch\n", gsz, time_it(200, l_emptyN, s));
  }
  for (int hops : {1, 2, 4, 8, 16}) {
    g_hops = hops; g_grid = 1024;
    printf("chase %2d dependent loads, 1024 x 256 : %7.2f us/launch\n", hops, time_it(50, l_chase, s));
  }
  {   // the same 200 empty launches captured in a hipGraph and replayed
    hipGraph_t g; hipGraphExec_t ge;
    hipStreamBeginCapture(s, hipStreamCaptureModeGlobal);
    for (int r = 0; r < 200; ++r) hipLaunchKernelGGL(k_empty, dim3(256), dim3(256), 0, s);
    hipStreamEndCapture(s, &g);
    hipGraphInstantiate(&ge, g, nullptr, nullptr, 0);
    hipGraphLaunch(ge, s); hipStreamSynchronize(s);
    hipEvent_t a, b; hipEventCreate(&a); hipEventCreate(&b);
    hipEventRecord(a, s);
    for (int k = 0; k < 5; ++k) hipGraphLaunch(ge, s);
    hipEventRecord(b, s); hipEventSynchronize(b);
    float ms = 0; hipEventElapsedTime(&ms, a, b);
    printf("empty kernel, 256 x 256, hipGraph : %6.2f us/kernel\n", ms * 1000.f / 1000.f);
  }
  for (int hops : {1, 4, 16}) {
    g_hops = hops; g_grid = 16;
    printf("chase %2d dependent loads,   16 x 256 : %7.2f us/launch\n", hops, time_it(50, l_chase, s));
  }
  return 0;
}
