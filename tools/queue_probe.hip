// Diagnostic: do kernels on streams created back to back run concurrently once many
// streams already exist (e.g. torch's stream pools)?  Prints the wall time of one spin
// kernel per stream launched together vs. one alone.
#include <hip/hip_runtime.h>
#include <chrono>
#include <cstdio>
#include <cstdlib>
#include <vector>

__global__ void spin(long long cycles, int* out) {
  long long t0 = clock64();
  while (clock64() - t0 < cycles) {}
  if (threadIdx.x == 0) out[blockIdx.x] = 1;
}

static double run(std::vector<hipStream_t>& ss, int* buf, long long cyc) {
  hipDeviceSynchronize();
  auto t0 = std::chrono::high_resolution_clock::now();
  for (auto s : ss) hipLaunchKernelGGL(spin, dim3(8), dim3(64), 0, s, cyc, buf);
  hipDeviceSynchronize();
  auto t1 = std::chrono::high_resolution_clock::now();
  return std::chrono::duration<double, std::micro>(t1 - t0).count();
}

int main(int argc, char** argv) {
  int pre = argc > 1 ? atoi(argv[1]) : 0;   // streams created first (a "pool")
  int* buf;
  hipMalloc(&buf, 1024 * sizeof(int));
  std::vector<hipStream_t> pool(pre);
  for (auto& s : pool) hipStreamCreateWithFlags(&s, hipStreamNonBlocking);
  std::vector<hipStream_t> lanes(3);
  for (auto& s : lanes) hipStreamCreateWithFlags(&s, hipStreamNonBlocking);
  const long long cyc = 200000;   // ~100 us
  std::vector<hipStream_t> one{lanes[0]};
  run(one, buf, cyc);
  double t1 = run(one, buf, cyc);
  for (int n = 2; n <= 3; ++n) {
    std::vector<hipStream_t> v(lanes.begin(), lanes.begin() + n);
    double tn = run(v, buf, cyc);
    printf("pre=%d streams=%d: one %.0f us, %d together %.0f us (%s)\n", pre, n, t1, n, tn,
           tn < 1.5 * t1 ? "concurrent" : "serialised");
  }
  if (pre > 0) {   // a pool stream together with lane 0
    std::vector<hipStream_t> v{pool[0], lanes[0]};
    double tn = run(v, buf, cyc);
    printf("pre=%d pool[0]+lane0 together %.0f us (%s)\n", pre, tn, tn < 1.5 * t1 ? "concurrent" : "serialised");
    std::vector<hipStream_t> w{pool[pre - 1], lanes[0]};
    tn = run(w, buf, cyc);
    printf("pre=%d pool[last]+lane0 together %.0f us (%s)\n", pre, tn, tn < 1.5 * t1 ? "concurrent" : "serialised");
  }
  return 0;
}
