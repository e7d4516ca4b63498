// K8: torch_scatter.scatter_mean(src, index, dim=0) forward / backward.
// Reference call sites: model/Twitter/BiGCN_Twitter.py:65,113; model/Weibo/BiGCN_Weibo.py:43,73.
// torch_scatter semantics: out[b] = sum_{index[i]=b} src[i] / max(count_b, 1).
//
// PyG batches are sorted by tree, so the common path is a deterministic segmented
// mean.  The kernel pair below decides on the device (no host sync): k_check_sorted
// sets a flag, the segmented kernels run when the index is sorted and the atomic
// kernels (any order; float atomics) run otherwise - each returns immediately when
// it is not the selected path.
#include "bgcn_common.h"

namespace bgcn {
namespace {

// flags[0] = 1 if index is NOT non-decreasing; *status |= 1 if any index is out of range
__global__ void k_check(const int64_t* __restrict__ index, int64_t n, int64_t B,
                        int32_t* __restrict__ flags, int32_t* __restrict__ status) {
  int64_t i = int64_t(blockIdx.x) * blockDim.x + threadIdx.x;
  if (i >= n) return;
  int64_t v = index[i];
  if ((v < 0 || v >= B) && status) atomicOr(status, 1);
  if (i > 0 && index[i - 1] > v) atomicOr(&flags[0], 1);
}

__global__ void k_seg_bounds(const int64_t* __restrict__ index, int64_t n, int64_t B,
                             const int32_t* __restrict__ flags, int64_t* __restrict__ bounds) {
  if (flags[0]) return;
  int64_t b = int64_t(blockIdx.x) * blockDim.x + threadIdx.x;
  if (b > B) return;
  int64_t lo = 0, hi = n;
  while (lo < hi) {
    int64_t mid = (lo + hi) >> 1;
    if (index[mid] < b) lo = mid + 1; else hi = mid;
  }
  bounds[b] = lo;
}

// one block per (segment, 256-column slice); rows of the segment split over 4 phases
__global__ __launch_bounds__(256) void k_seg_mean(const float* __restrict__ src, int64_t ld_src,
                                                  int64_t n, int C, int64_t B,
                                                  const int32_t* __restrict__ flags,
                                                  const int64_t* __restrict__ bounds,
                                                  float* __restrict__ out, int64_t ld_out,
                                                  float* __restrict__ count) {
  if (flags[0]) return;
  __shared__ float red[4][64];
  const int64_t b = blockIdx.x;
  const int c = blockIdx.y * 64 + (threadIdx.x & 63), ph = threadIdx.x >> 6;
  int64_t beg = bounds[b], end = bounds[b + 1];
  // indices outside [0, B) (sorted to the ends) are excluded by the bounds
  float acc = 0.f;
  if (c < C)
    for (int64_t i = beg + ph; i < end; i += 4) acc += src[i * ld_src + c];
  red[ph][threadIdx.x & 63] = acc;
  __syncthreads();
  if (ph == 0 && c < C) {
    float s = red[0][threadIdx.x] + red[1][threadIdx.x] + red[2][threadIdx.x] + red[3][threadIdx.x];
    float cnt = float(end - beg > 0 ? end - beg : 1);
    out[b * ld_out + c] = s / cnt;
    if (c == 0 && count) count[b] = cnt;
  }
}

__global__ void k_atomic_zero(const int32_t* __restrict__ flags, float* __restrict__ out,
                              int64_t ld_out, int64_t B, int C, float* __restrict__ count) {
  if (!flags[0]) return;
  int64_t idx = int64_t(blockIdx.x) * blockDim.x + threadIdx.x;
  if (idx >= B * C) return;
  int64_t b = idx / C;
  out[b * ld_out + idx % C] = 0.f;
  if (idx % C == 0) count[b] = 0.f;
}

__global__ void k_atomic_sum(const float* __restrict__ src, int64_t ld_src,
                             const int64_t* __restrict__ index, int64_t n, int C, int64_t B,
                             const int32_t* __restrict__ flags, float* __restrict__ out,
                             int64_t ld_out, float* __restrict__ count) {
  if (!flags[0]) return;
  int64_t idx = int64_t(blockIdx.x) * blockDim.x + threadIdx.x;
  if (idx >= n * C) return;
  int64_t i = idx / C;
  int c = int(idx % C);
  int64_t b = index[i];
  if (b < 0 || b >= B) return;
  atomicAdd(&out[b * ld_out + c], src[i * ld_src + c]);
  if (c == 0) atomicAdd(&count[b], 1.f);
}

__global__ void k_atomic_div(const int32_t* __restrict__ flags, float* __restrict__ out,
                             int64_t ld_out, int64_t B, int C, float* __restrict__ count) {
  if (!flags[0]) return;
  int64_t b = int64_t(blockIdx.x) * blockDim.y + threadIdx.y;
  if (b >= B) return;
  float cnt = fmaxf(count[b], 1.f);
  for (int c = threadIdx.x; c < C; c += blockDim.x) out[b * ld_out + c] /= cnt;
  if (threadIdx.x == 0) count[b] = cnt;
}

__global__ void k_mean_bwd(const float* __restrict__ dout, int64_t ld_dout,
                           const int64_t* __restrict__ index, const float* __restrict__ count,
                           int64_t n, int C, int64_t B, float* __restrict__ dsrc, int64_t ld_dsrc) {
  int64_t idx = int64_t(blockIdx.x) * blockDim.x + threadIdx.x;
  if (idx >= n * C) return;
  int64_t i = idx / C;
  int c = int(idx % C);
  int64_t b = index[i];
  float g = 0.f;
  if (b >= 0 && b < B) g = dout[b * ld_dout + c] / count[b];
  dsrc[i * ld_dsrc + c] = g;
}

}  // namespace

size_t scatter_ws_size(int64_t B) { return 256 + size_t(B + 1) * sizeof(int64_t); }

int scatter_mean_fwd_impl(const float* src, int64_t ld_src, const int64_t* index, int64_t n,
                          int32_t C, int64_t B, float* out, int64_t ld_out, float* count,
                          int32_t* status, void* ws, size_t ws_bytes, hipStream_t s) {
  BGCN_CHECK_ARG(n >= 0 && C > 0 && B > 0, "bad shape");
  BGCN_CHECK_ARG(out && count, "null pointer (count is required)");
  BGCN_CHECK_ARG(n == 0 || (src && index), "null src/index");
  BGCN_CHECK_ARG(ld_src >= C && ld_out >= C, "bad leading dimension");
  BGCN_CHECK_ARG(ws && ws_bytes >= scatter_ws_size(B), "workspace too small");
  int32_t* flags = static_cast<int32_t*>(ws);  // [0] unsorted
  int64_t* bounds = reinterpret_cast<int64_t*>(static_cast<char*>(ws) + 256);
  BGCN_CHECK_HIP(hipMemsetAsync(flags, 0, 16, s));
  if (n > 0) {
    hipLaunchKernelGGL(k_check, dim3(grid_for(n, 256)), dim3(256), 0, s, index, n, B, flags,
                       status);
    BGCN_CHECK_LAUNCH();
  }
  hipLaunchKernelGGL(k_seg_bounds, dim3(grid_for(B + 1, 256)), dim3(256), 0, s, index, n, B,
                     flags, bounds);
  BGCN_CHECK_LAUNCH();
  hipLaunchKernelGGL(k_seg_mean, dim3(unsigned(B), unsigned((C + 63) / 64)), dim3(256), 0, s, src,
                     ld_src, n, C, B, flags, bounds, out, ld_out, count);
  BGCN_CHECK_LAUNCH();
  hipLaunchKernelGGL(k_atomic_zero, dim3(grid_for(B * C, 256)), dim3(256), 0, s, flags, out,
                     ld_out, B, C, count);
  BGCN_CHECK_LAUNCH();
  if (n > 0) {
    hipLaunchKernelGGL(k_atomic_sum, dim3(grid_for(n * C, 256)), dim3(256), 0, s, src, ld_src,
                       index, n, C, B, flags, out, ld_out, count);
    BGCN_CHECK_LAUNCH();
  }
  hipLaunchKernelGGL(k_atomic_div, dim3(grid_for(B, 4)), dim3(64, 4), 0, s, flags, out, ld_out,
                     B, C, count);
  BGCN_CHECK_LAUNCH();
  return BGCN_OK;
}

int scatter_mean_bwd_impl(const float* dout, int64_t ld_dout, const int64_t* index,
                          const float* count, int64_t n, int32_t C, int64_t B, float* dsrc,
                          int64_t ld_dsrc, hipStream_t s) {
  BGCN_CHECK_ARG(n >= 0 && C > 0 && B > 0, "bad shape");
  if (n == 0) return BGCN_OK;
  BGCN_CHECK_ARG(dout && index && count && dsrc, "null pointer");
  hipLaunchKernelGGL(k_mean_bwd, dim3(grid_for(n * C, 256)), dim3(256), 0, s, dout, ld_dout, index,
                     count, n, C, B, dsrc, ld_dsrc);
  BGCN_CHECK_LAUNCH();
  return BGCN_OK;
}

}  // namespace bgcn

extern "C" size_t bgcn_scatter_mean_workspace_size(int64_t B) {
  return bgcn::scatter_ws_size(B);
}

extern "C" int bgcn_scatter_mean_fwd(const float* src, int64_t ld_src, const int64_t* index,
                                     int64_t n, int32_t C, int64_t B, float* out, int64_t ld_out,
                                     float* count, int32_t* status, void* workspace,
                                     size_t workspace_bytes, bgcn_stream_t stream) {
  return bgcn::scatter_mean_fwd_impl(src, ld_src, index, n, C, B, out, ld_out, count, status,
                                     workspace, workspace_bytes,
                                     reinterpret_cast<hipStream_t>(stream));
}

extern "C" int bgcn_scatter_mean_bwd(const float* dout, int64_t ld_dout, const int64_t* index,
                                     const float* count, int64_t n, int32_t C, int64_t B,
                                     float* dsrc, int64_t ld_dsrc, bgcn_stream_t stream) {
  return bgcn::scatter_mean_bwd_impl(dout, ld_dout, index, count, n, C, B, dsrc, ld_dsrc,
                                     reinterpret_cast<hipStream_t>(stream));
}
