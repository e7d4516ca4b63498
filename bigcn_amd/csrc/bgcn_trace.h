// Diagnostic builds only (-DBGCN_BLOCK_TRACE, tools/block_trace.py): every wave of an
// instrumented kernel records {kernel id, block, start, end, CU} with the device's
// constant-rate clock, so a kernel's span can be split into wave lifetimes, dispatch
// spread and tail.  One record buffer per translation unit, read by bgcn_bt_read_<tu>.
#pragma once
#include <hip/hip_runtime.h>
#include <cstdint>

#ifdef BGCN_BLOCK_TRACE
namespace bgcn {
namespace {
// one region of kBtWaves wave slots per kernel slot (kid / 10 for the role ids 70..83);
// a wave writes its own slot (no atomics: a shared counter serialises thousands of waves)
constexpr unsigned kBtKernels = 16, kBtWaves = 1u << 14;
__device__ unsigned long long g_bt[kBtKernels * kBtWaves * 4];
__device__ unsigned long long g_btm[kBtKernels * kBtWaves * 4];   // intermediate marks
__device__ unsigned int g_bt_on;
__device__ __forceinline__ unsigned bt_slot(unsigned kid) {
  const unsigned ks = kid >= 70 ? kid / 10 : kid;
  const unsigned w = ((blockIdx.y * gridDim.x + blockIdx.x) * ((blockDim.x + 63) / 64) + (threadIdx.x >> 6));
  return (ks >= kBtKernels || w >= kBtWaves) ? ~0u : ks * kBtWaves + w;
}
__device__ __forceinline__ void bt_mark(unsigned kid, int j) {
  if ((threadIdx.x & 63) != 0 || g_bt_on == 0) return;
  const unsigned s = bt_slot(kid);
  if (s != ~0u) g_btm[s * 4 + j] = uint64_t(wall_clock64());
}
__device__ __forceinline__ void bt_record(unsigned kid, long long t0, long long c0) {
  if ((threadIdx.x & 63) != 0 || g_bt_on == 0) return;
  const long long t1 = wall_clock64();
  const long long c1 = clock64();
  const unsigned ks = kid >= 70 ? kid / 10 : kid;
  const unsigned w = ((blockIdx.y * gridDim.x + blockIdx.x) * ((blockDim.x + 63) / 64) + (threadIdx.x >> 6));
  if (ks >= kBtKernels || w >= kBtWaves) return;
  const unsigned s = ks * kBtWaves + w;
  const unsigned xcc = __builtin_amdgcn_s_getreg((3 << 11) | 20) & 15u;   // HW_REG_XCC_ID
  g_bt[s * 4 + 0] = (uint64_t(kid) << 48) | (uint64_t(blockIdx.y) << 32) | blockIdx.x;
  g_bt[s * 4 + 1] = uint64_t(t0);
  g_bt[s * 4 + 2] = uint64_t(t1);
  g_bt[s * 4 + 3] = (uint64_t(uint32_t(c1 - c0)) << 32) | (uint64_t(xcc) << 24) | (uint64_t(__smid() & 0xffff) << 8) |
                    (threadIdx.x >> 6);
}
}  // namespace
}  // namespace bgcn
#define BT_BEGIN const long long bt_t0_ = wall_clock64(), bt_c0_ = clock64();
#define BT_END(kid) bgcn::bt_record(kid, bt_t0_, bt_c0_)
#define BT_MARK(kid, j) bgcn::bt_mark(kid, j)
// host side of one translation unit: copy out (all slots; empty ones are zero), clear,
// enable / disable recording
#define BT_READER(tu)                                                                        \
  extern "C" int bgcn_bt_read_##tu(unsigned long long* out, unsigned cap, int enable) {     \
    const unsigned n = bgcn::kBtKernels * bgcn::kBtWaves;                                    \
    if (hipDeviceSynchronize() != hipSuccess) return -1;                                    \
    if (out && cap >= n &&                                                                   \
        hipMemcpyFromSymbol(out, HIP_SYMBOL(bgcn::g_bt), size_t(n) * 32) != hipSuccess)      \
      return -1;                                                                             \
    void* p = nullptr;                                                                       \
    if (hipGetSymbolAddress(&p, HIP_SYMBOL(bgcn::g_bt)) != hipSuccess ||                     \
        hipMemset(p, 0, size_t(n) * 32) != hipSuccess)                                       \
      return -1;                                                                             \
    if (out && cap >= 2 * n &&                                                               \
        hipMemcpyFromSymbol(out + size_t(n) * 4, HIP_SYMBOL(bgcn::g_btm), size_t(n) * 32) != hipSuccess) \
      return -1;                                                                             \
    if (hipGetSymbolAddress(&p, HIP_SYMBOL(bgcn::g_btm)) != hipSuccess ||                    \
        hipMemset(p, 0, size_t(n) * 32) != hipSuccess)                                       \
      return -1;                                                                             \
    const unsigned on = enable ? 1u : 0u;                                                    \
    (void)hipMemcpyToSymbol(HIP_SYMBOL(bgcn::g_bt_on), &on, sizeof(on));                     \
    (void)hipDeviceSynchronize();                                                            \
    return out && cap >= n ? int(n) : 0;                                                     \
  }
#else
#define BT_BEGIN
#define BT_END(kid)
#define BT_MARK(kid, j)
#define BT_READER(tu)
#endif
