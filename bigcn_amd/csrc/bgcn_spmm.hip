// K3/K4: normalised neighbour aggregation out = A_hat * in (+ bias, relu).
//
// Replaces PyG MessagePassing.propagate for GCNConv (message = norm * x_j,
// aggr = 'add': index_select(x, row) * norm -> scatter_add to col) and its
// autograd backward (the same product over the transposed CSR).  Call sites in
// the reference: every GCNConv at model/Twitter/BiGCN_Twitter.py:42,56,92,105.
//
// Load balance: propagation trees are extremely skewed (TD rows have <= 2
// entries, a BU star root can have thousands).  The nnz range is cut into equal
// chunks of NPG entries, one chunk per lane group (merge path over the COO row
// array).  A group writes every row it owns completely; a row that crosses a chunk
// boundary leaves one partial per chunk it touches, and a fixup pass sums those
// partials in chunk order (deterministic, no atomics).
//
// Narrow kernel (F = 64 / 128): a group = F/4 lanes, one float4 per lane.
// Wide kernel (any F, e.g. the 5000-dim standalone aggregation): a group = one
// 256-thread block, blockIdx.y tiles F in 1024-float slices.
#include "bgcn_common.h"

namespace bgcn {
namespace {

constexpr int NPG = 32;  // CSR entries per lane group

// Partial record per (group, slot): slot 0 = head row (started before the chunk),
// slot 1 = tail row (started inside the chunk, ends after it).
template <int LANES>
__global__ __launch_bounds__(256) void k_spmm_narrow(
    const int32_t* __restrict__ ptr, const int32_t* __restrict__ rowid,
    const int32_t* __restrict__ col, const float* __restrict__ w, int64_t rows,
    const float* __restrict__ in, int64_t ld_in, float* __restrict__ out, int64_t ld_out,
    const float* __restrict__ bias, int epi, float* __restrict__ part, int64_t ngroups) {
  constexpr int GPB = 256 / LANES;  // groups per block
  const int lane = threadIdx.x % LANES;
  const int64_t g = int64_t(blockIdx.x) * GPB + threadIdx.x / LANES;
  if (g >= ngroups) return;
  const int64_t nnz = ptr[rows];
  const int64_t p0 = g * NPG;
  if (p0 >= nnz) return;
  const int64_t p1 = min<int64_t>(p0 + NPG, nnz);
  const int fo = lane * 4;
  const float4 bv = bias ? ld4(bias + fo) : f4zero();

  // prefetch the chunk's (row, col, w) into registers of the group's lanes
  // (LANES >= 16, NPG = 32 -> at most 2 entries per lane)
  constexpr int EPL = (NPG + LANES - 1) / LANES;
  int32_t r_l[EPL], c_l[EPL];
  float w_l[EPL];
#pragma unroll
  for (int q = 0; q < EPL; ++q) {
    int64_t p = p0 + q * LANES + lane;
    bool v = p < p1;
    r_l[q] = v ? rowid[p] : -1;
    c_l[q] = v ? col[p] : 0;
    w_l[q] = v ? w[p] : 0.f;
  }
  const int base_lane = ((threadIdx.x & 63) / LANES) * LANES;  // group's first lane in the wave
  auto bc_i = [&](int32_t v, int src) { return __shfl(v, base_lane + src, 64); };
  auto bc_f = [&](float v, int src) { return __shfl(v, base_lane + src, 64); };

  float4 acc = f4zero();
  int32_t cur = -1;
  const int n = int(p1 - p0);
  // entries are processed in blocks of 8 to keep 8 row loads in flight
  for (int k0 = 0; k0 < NPG; k0 += 8) {
    if (k0 >= n) break;
    float4 v[8];
    int32_t rr[8];
    float ww[8];
#pragma unroll
    for (int u = 0; u < 8; ++u) {
      int k = k0 + u;
      int q = k / LANES, src = k % LANES;
      int32_t rk = -1, ck = 0;
      float wk = 0.f;
#pragma unroll
      for (int qq = 0; qq < EPL; ++qq) {
        int32_t rv = bc_i(r_l[qq], src), cv = bc_i(c_l[qq], src);
        float wv = bc_f(w_l[qq], src);
        if (qq == q) { rk = rv; ck = cv; wk = wv; }
      }
      rr[u] = k < n ? rk : -1;
      ww[u] = wk;
      v[u] = k < n ? ld4(in + int64_t(ck) * ld_in + fo) : f4zero();
    }
#pragma unroll
    for (int u = 0; u < 8; ++u) {
      int32_t r = rr[u];
      if (r < 0) break;
      if (r != cur) {
        if (cur >= 0) {
          // flush `cur`: it ended inside this chunk (it is not the last row touched)
          int64_t rs = ptr[cur];
          if (rs >= p0) {
            float4 o = f4add(acc, bv);
            if (epi & BGCN_EPI_RELU) o = f4relu(o);
            st4(out + int64_t(cur) * ld_out + fo, o);
          } else {
            st4(part + (g * 2 + 0) * (LANES * 4) + fo, acc);
          }
        }
        cur = r;
        acc = f4zero();
      }
      acc = f4fma(ww[u], v[u], acc);
    }
  }
  if (cur >= 0) {
    int64_t rs = ptr[cur], re = ptr[cur + 1];
    if (rs >= p0 && re <= p1) {
      float4 o = f4add(acc, bv);
      if (epi & BGCN_EPI_RELU) o = f4relu(o);
      st4(out + int64_t(cur) * ld_out + fo, o);
    } else if (rs < p0) {
      st4(part + (g * 2 + 0) * (LANES * 4) + fo, acc);  // head (may also extend past p1)
    } else {
      st4(part + (g * 2 + 1) * (LANES * 4) + fo, acc);  // tail
    }
  }
}

// One lane group per chunk boundary g*NPG (g >= 1): if the row containing entry
// g*NPG started before it and its last entry lies in chunk g's... last chunk,
// this group sums tail[g0] + head[g0+1..g1] and writes the row.
template <int LANES>
__global__ __launch_bounds__(256) void k_spmm_fixup(
    const int32_t* __restrict__ ptr, const int32_t* __restrict__ rowid, int64_t rows,
    float* __restrict__ out, int64_t ld_out, const float* __restrict__ bias, int epi,
    const float* __restrict__ part, int64_t ngroups, int F) {
  constexpr int GPB = 256 / LANES;
  const int lane = threadIdx.x % LANES;
  const int64_t g = int64_t(blockIdx.x) * GPB + threadIdx.x / LANES;
  if (g < 1 || g >= ngroups) return;
  const int64_t nnz = ptr[rows];
  const int64_t pb = g * NPG;
  if (pb >= nnz) return;
  const int32_t r = rowid[pb];
  const int64_t rs = ptr[r], re = ptr[r + 1];
  if (rs >= pb) return;                      // row starts at the boundary: no crossing
  const int64_t g0 = rs / NPG, g1 = (re - 1) / NPG;
  if (g1 != g) return;                       // only the row's last chunk does the fixup
  for (int fo = lane * 4; fo < F; fo += LANES * 4) {
    float4 acc = ld4(part + (g0 * 2 + 1) * int64_t(F) + fo);
    for (int64_t q = g0 + 1; q <= g1; ++q) acc = f4add(acc, ld4(part + (q * 2 + 0) * int64_t(F) + fo));
    float4 o = f4add(acc, bias ? ld4(bias + fo) : f4zero());
    if (epi & BGCN_EPI_RELU) o = f4relu(o);
    st4(out + int64_t(r) * ld_out + fo, o);
  }
}

// Wide kernel: block = one chunk of NPG entries, blockIdx.y = 1024-float slice.
__global__ __launch_bounds__(256) void k_spmm_wide(
    const int32_t* __restrict__ ptr, const int32_t* __restrict__ rowid,
    const int32_t* __restrict__ col, const float* __restrict__ w, int64_t rows,
    const float* __restrict__ in, int64_t ld_in, float* __restrict__ out, int64_t ld_out, int F,
    const float* __restrict__ bias, int epi, float* __restrict__ part) {
  __shared__ int32_t s_r[NPG], s_c[NPG];
  __shared__ float s_w[NPG];
  const int64_t g = blockIdx.x;
  const int64_t nnz = ptr[rows];
  const int64_t p0 = g * NPG;
  if (p0 >= nnz) return;
  const int64_t p1 = min<int64_t>(p0 + NPG, nnz);
  const int n = int(p1 - p0);
  if (threadIdx.x < NPG) {
    int64_t p = p0 + threadIdx.x;
    bool v = p < p1;
    s_r[threadIdx.x] = v ? rowid[p] : -1;
    s_c[threadIdx.x] = v ? col[p] : 0;
    s_w[threadIdx.x] = v ? w[p] : 0.f;
  }
  __syncthreads();
  const int fo = blockIdx.y * 1024 + threadIdx.x * 4;
  const bool act = fo < F;
  const float4 bv = (bias && act) ? ld4(bias + fo) : f4zero();
  float4 acc = f4zero();
  int32_t cur = -1;
  for (int k0 = 0; k0 < n; k0 += 8) {
    float4 v[8];
#pragma unroll
    for (int u = 0; u < 8; ++u) {
      int k = k0 + u;
      v[u] = (k < n && act) ? ld4(in + int64_t(s_c[k]) * ld_in + fo) : f4zero();
    }
#pragma unroll
    for (int u = 0; u < 8; ++u) {
      int k = k0 + u;
      if (k >= n) break;
      int32_t r = s_r[k];
      if (r != cur) {
        if (cur >= 0 && act) {
          if (ptr[cur] >= p0) {
            float4 o = f4add(acc, bv);
            if (epi & BGCN_EPI_RELU) o = f4relu(o);
            st4(out + int64_t(cur) * ld_out + fo, o);
          } else {
            st4(part + (g * 2 + 0) * int64_t(F) + fo, acc);
          }
        }
        cur = r;
        acc = f4zero();
      }
      acc = f4fma(s_w[k], v[u], acc);
    }
  }
  if (cur >= 0 && act) {
    int64_t rs = ptr[cur], re = ptr[cur + 1];
    if (rs >= p0 && re <= p1) {
      float4 o = f4add(acc, bv);
      if (epi & BGCN_EPI_RELU) o = f4relu(o);
      st4(out + int64_t(cur) * ld_out + fo, o);
    } else if (rs < p0) {
      st4(part + (g * 2 + 0) * int64_t(F) + fo, acc);
    } else {
      st4(part + (g * 2 + 1) * int64_t(F) + fo, acc);
    }
  }
}

}  // namespace

size_t spmm_ws_size(int64_t capacity, int32_t F) {
  int64_t ngroups = (capacity + NPG - 1) / NPG;
  return size_t(ngroups) * 2 * size_t(F) * sizeof(float) + 256;
}

int spmm_impl(const int32_t* ptr, const int32_t* row, const int32_t* col, const float* w,
              int64_t rows, int64_t capacity, const float* in, int64_t ld_in, float* out,
              int64_t ld_out, int32_t F, const float* bias, int epi, void* ws, size_t ws_bytes,
              hipStream_t stream) {
  BGCN_CHECK_ARG(rows > 0 && capacity >= rows, "bad rows/capacity");
  BGCN_CHECK_ARG(F > 0 && F % 4 == 0, "F must be a positive multiple of 4");
  BGCN_CHECK_ARG(ld_in % 4 == 0 && ld_out % 4 == 0 && ld_in >= F && ld_out >= F,
                 "ld must be >= F and a multiple of 4");
  BGCN_CHECK_ARG((reinterpret_cast<uintptr_t>(in) & 15) == 0 &&
                     (reinterpret_cast<uintptr_t>(out) & 15) == 0 &&
                     (!bias || (reinterpret_cast<uintptr_t>(bias) & 15) == 0),
                 "in/out/bias must be 16-byte aligned");
  BGCN_CHECK_ARG(ws && ws_bytes >= spmm_ws_size(capacity, F), "workspace too small");
  float* part = static_cast<float*>(ws);
  const int64_t ngroups = (capacity + NPG - 1) / NPG;
  if (F == 64 || F == 128) {
    if (F == 64) {
      constexpr int L = 16;
      hipLaunchKernelGGL((k_spmm_narrow<L>), dim3(grid_for(ngroups, 256 / L)), dim3(256), 0,
                         stream, ptr, row, col, w, rows, in, ld_in, out, ld_out, bias, epi, part,
                         ngroups);
      BGCN_CHECK_LAUNCH();
      hipLaunchKernelGGL((k_spmm_fixup<L>), dim3(grid_for(ngroups, 256 / L)), dim3(256), 0,
                         stream, ptr, row, rows, out, ld_out, bias, epi, part, ngroups, F);
    } else {
      constexpr int L = 32;
      hipLaunchKernelGGL((k_spmm_narrow<L>), dim3(grid_for(ngroups, 256 / L)), dim3(256), 0,
                         stream, ptr, row, col, w, rows, in, ld_in, out, ld_out, bias, epi, part,
                         ngroups);
      BGCN_CHECK_LAUNCH();
      hipLaunchKernelGGL((k_spmm_fixup<L>), dim3(grid_for(ngroups, 256 / L)), dim3(256), 0,
                         stream, ptr, row, rows, out, ld_out, bias, epi, part, ngroups, F);
    }
    BGCN_CHECK_LAUNCH();
    return BGCN_OK;
  }
  hipLaunchKernelGGL(k_spmm_wide, dim3(unsigned(ngroups), unsigned((F + 1023) / 1024)), dim3(256),
                     0, stream, ptr, row, col, w, rows, in, ld_in, out, ld_out, F, bias, epi,
                     part);
  BGCN_CHECK_LAUNCH();
  hipLaunchKernelGGL((k_spmm_fixup<64>), dim3(grid_for(ngroups, 4)), dim3(256), 0, stream, ptr,
                     row, rows, out, ld_out, bias, epi, part, ngroups, F);
  BGCN_CHECK_LAUNCH();
  return BGCN_OK;
}

}  // namespace bgcn

extern "C" size_t bgcn_spmm_workspace_size(int64_t capacity, int32_t F) {
  return bgcn::spmm_ws_size(capacity, F);
}

extern "C" int bgcn_spmm(const int32_t* ptr, const int32_t* row, const int32_t* col,
                         const float* w, int64_t rows, int64_t capacity, const float* in,
                         int64_t ld_in, float* out, int64_t ld_out, int32_t F, const float* bias,
                         int epilogue, void* workspace, size_t workspace_bytes,
                         bgcn_stream_t stream) {
  return bgcn::spmm_impl(ptr, row, col, w, rows, capacity, in, ld_in, out, ld_out, F, bias,
                         epilogue, workspace, workspace_bytes,
                         reinterpret_cast<hipStream_t>(stream));
}
