// K1: gcn_norm + add_remaining_self_loops + CSR construction (both orientations).
//
// Restates PyG >= 2.0 gcn_norm(improved=False, add_self_loops=True,
// flow='source_to_target') as used by every GCNConv call of the reference
// (model/Twitter/BiGCN_Twitter.py:42,56,92,105; explicit call form at
// explain_PHEME.py:62-63), with the PyG 1.3.2 source-degree convention selectable.
//
// Plan (deterministic, no float atomics):
//   1. keys: key_t[e] = target, key_s[e] = source, or N for self loops / invalid
//      edges (sorted to the end and dropped); value = e.
//   2. two stable LSD radix sorts (rocPRIM) -> edges grouped by target / by source
//      in their original order (the order PyG's scatter-add sums them in).
//   3. per node: segment bounds by binary search, weighted degree, D^-1/2, row
//      pointers (each row gets one extra slot for its self loop, placed last),
//      self-loop entries.
//   4. per sorted edge: CSR entry at position j + key (j = sorted position).
#include <cstring>

#include <rocprim/rocprim.hpp>

#include "bgcn_common.h"

namespace bgcn {
namespace {

__global__ void k_edge_keys(const int64_t* __restrict__ ei, int64_t E, int64_t N,
                            uint32_t* __restrict__ key_t, uint32_t* __restrict__ key_s,
                            uint32_t* __restrict__ val, int32_t* __restrict__ status) {
  int64_t e = int64_t(blockIdx.x) * blockDim.x + threadIdx.x;
  if (e >= E) return;
  int64_t src = ei[e], dst = ei[E + e];
  bool valid = src >= 0 && src < N && dst >= 0 && dst < N;
  if (!valid && status) atomicOr(status, 1);
  bool keep = valid && src != dst;  // existing self loops are replaced by the appended ones
  key_t[e] = keep ? uint32_t(dst) : uint32_t(N);
  key_s[e] = keep ? uint32_t(src) : uint32_t(N);
  val[e] = uint32_t(e);
}

__device__ __forceinline__ int64_t lower_bound_u32(const uint32_t* a, int64_t n, uint32_t x) {
  int64_t lo = 0, hi = n;
  while (lo < hi) {
    int64_t mid = (lo + hi) >> 1;
    if (a[mid] < x) lo = mid + 1; else hi = mid;
  }
  return lo;
}

// One thread per node i in [0, N].  Thread N only writes the terminal pointers.
__global__ void k_nodes(const uint32_t* __restrict__ st_keys, const uint32_t* __restrict__ st_vals,
                        const uint32_t* __restrict__ ss_keys, const uint32_t* __restrict__ ss_vals,
                        const float* __restrict__ ew, int64_t E, int64_t N, int degree_on,
                        float* __restrict__ dinv, int32_t* __restrict__ t_ptr,
                        int32_t* __restrict__ s_ptr) {
  int64_t i = int64_t(blockIdx.x) * blockDim.x + threadIdx.x;
  if (i > N) return;
  int64_t t0 = lower_bound_u32(st_keys, E, uint32_t(i));
  int64_t s0 = lower_bound_u32(ss_keys, E, uint32_t(i));
  t_ptr[i] = int32_t(t0 + i);
  s_ptr[i] = int32_t(s0 + i);
  if (i == N) return;
  const uint32_t* keys = degree_on == BGCN_DEGREE_ON_COL ? st_keys : ss_keys;
  const uint32_t* vals = degree_on == BGCN_DEGREE_ON_COL ? st_vals : ss_vals;
  int64_t a = degree_on == BGCN_DEGREE_ON_COL ? t0 : s0;
  int64_t b = lower_bound_u32(keys, E, uint32_t(i + 1));
  // scatter_add over the final edge list in order: real edges, then the loop (w=1)
  float deg = 0.f;
  if (ew) {
    for (int64_t j = a; j < b; ++j) deg += ew[vals[j]];
  } else {
    for (int64_t j = a; j < b; ++j) deg += 1.f;
  }
  deg += 1.f;
  float d = deg > 0.f ? 1.0f / sqrtf(deg) : 0.f;  // pow(-0.5); inf -> 0
  if (isinf(d)) d = 0.f;
  dinv[i] = d;
}

__global__ void k_self_loops(const int32_t* __restrict__ t_ptr, const int32_t* __restrict__ s_ptr,
                             const float* __restrict__ dinv, int64_t N,
                             int32_t* __restrict__ t_row, int32_t* __restrict__ t_col,
                             float* __restrict__ t_w, int32_t* __restrict__ s_row,
                             int32_t* __restrict__ s_col, float* __restrict__ s_w) {
  int64_t i = int64_t(blockIdx.x) * blockDim.x + threadIdx.x;
  if (i >= N) return;
  float d = dinv[i];
  float w = (d * 1.0f) * d;  // dinv[row] * w * dinv[col]
  int32_t pt = t_ptr[i + 1] - 1, ps = s_ptr[i + 1] - 1;
  t_row[pt] = int32_t(i); t_col[pt] = int32_t(i); t_w[pt] = w;
  s_row[ps] = int32_t(i); s_col[ps] = int32_t(i); s_w[ps] = w;
}

// One thread per sorted edge position j (both orientations).
__global__ void k_fill(const int64_t* __restrict__ ei, const float* __restrict__ ew, int64_t E,
                       int64_t N, const uint32_t* __restrict__ st_keys,
                       const uint32_t* __restrict__ st_vals, const uint32_t* __restrict__ ss_keys,
                       const uint32_t* __restrict__ ss_vals, const float* __restrict__ dinv,
                       int32_t* __restrict__ t_row, int32_t* __restrict__ t_col,
                       float* __restrict__ t_w, int32_t* __restrict__ s_row,
                       int32_t* __restrict__ s_col, float* __restrict__ s_w) {
  int64_t j = int64_t(blockIdx.x) * blockDim.x + threadIdx.x;
  if (j >= E) return;
  uint32_t kt = st_keys[j];
  if (kt < uint32_t(N)) {
    uint32_t e = st_vals[j];
    int64_t src = ei[e];
    float w = ew ? ew[e] : 1.f;
    int64_t pos = j + kt;
    t_row[pos] = int32_t(kt);
    t_col[pos] = int32_t(src);
    t_w[pos] = (dinv[src] * w) * dinv[kt];
  }
  uint32_t ks = ss_keys[j];
  if (ks < uint32_t(N)) {
    uint32_t e = ss_vals[j];
    int64_t dst = ei[E + e];
    float w = ew ? ew[e] : 1.f;
    int64_t pos = j + ks;
    s_row[pos] = int32_t(ks);
    s_col[pos] = int32_t(dst);
    s_w[pos] = (dinv[ks] * w) * dinv[dst];
  }
}

int key_bits(int64_t N) {
  int bits = 1;
  while ((int64_t(1) << bits) <= N) ++bits;  // keys in [0, N]
  return bits;
}

struct GraphWs {
  uint32_t *key_t, *key_s, *val, *st_keys, *st_vals, *ss_keys, *ss_vals;
  float* dinv;
  void* sort_tmp;
  size_t sort_bytes;
};

size_t sort_tmp_bytes(int64_t E, int64_t N) {
  size_t bytes = 0;
  if (E == 0) return 0;
  (void)rocprim::radix_sort_pairs(nullptr, bytes, (uint32_t*)nullptr, (uint32_t*)nullptr,
                            (uint32_t*)nullptr, (uint32_t*)nullptr, size_t(E), 0, key_bits(N));
  return bytes;
}

size_t carve_graph_ws(Carve& c, int64_t E, int64_t N, GraphWs* g) {
  size_t e = size_t(E > 0 ? E : 1);
  GraphWs t;
  t.key_t = c.take<uint32_t>(e);
  t.key_s = c.take<uint32_t>(e);
  t.val = c.take<uint32_t>(e);
  t.st_keys = c.take<uint32_t>(e);
  t.st_vals = c.take<uint32_t>(e);
  t.ss_keys = c.take<uint32_t>(e);
  t.ss_vals = c.take<uint32_t>(e);
  t.dinv = c.take<float>(size_t(N > 0 ? N : 1));
  t.sort_bytes = sort_tmp_bytes(E, N);
  t.sort_tmp = c.take<char>(t.sort_bytes > 0 ? t.sort_bytes : 1);
  if (g) *g = t;
  return c.off;
}

}  // namespace

int build_graph_impl(const int64_t* ei, const float* ew, int64_t E, int64_t N, int degree_on,
                     int32_t* t_ptr, int32_t* t_row, int32_t* t_col, float* t_w, int32_t* s_ptr,
                     int32_t* s_row, int32_t* s_col, float* s_w, int32_t* status, void* ws,
                     size_t ws_bytes, hipStream_t stream) {
  BGCN_CHECK_ARG(N > 0 && N < (int64_t(1) << 31) - 1, "num_nodes out of range");
  BGCN_CHECK_ARG(E >= 0 && E + N < (int64_t(1) << 31), "num_edges out of range");
  BGCN_CHECK_ARG(degree_on == BGCN_DEGREE_ON_COL || degree_on == BGCN_DEGREE_ON_ROW,
                 "degree_on must be 0 (col) or 1 (row)");
  BGCN_CHECK_ARG(t_ptr && t_row && t_col && t_w && s_ptr && s_row && s_col && s_w,
                 "null output pointer");
  BGCN_CHECK_ARG(E == 0 || ei, "null edge_index");
  Carve c(ws, ws_bytes);
  GraphWs g;
  carve_graph_ws(c, E, N, &g);
  BGCN_CHECK_ARG(c.ok() && ws, "workspace too small");
  const int blk = 256;
  if (E > 0) {
    hipLaunchKernelGGL(k_edge_keys, dim3(grid_for(E, blk)), dim3(blk), 0, stream, ei, E, N,
                       g.key_t, g.key_s, g.val, status);
    BGCN_CHECK_LAUNCH();
    int bits = key_bits(N);
    size_t tb = g.sort_bytes;
    BGCN_CHECK_HIP(rocprim::radix_sort_pairs(g.sort_tmp, tb, g.key_t, g.st_keys, g.val,
                                             g.st_vals, size_t(E), 0, bits, stream));
    tb = g.sort_bytes;
    BGCN_CHECK_HIP(rocprim::radix_sort_pairs(g.sort_tmp, tb, g.key_s, g.ss_keys, g.val,
                                             g.ss_vals, size_t(E), 0, bits, stream));
  }
  hipLaunchKernelGGL(k_nodes, dim3(grid_for(N + 1, blk)), dim3(blk), 0, stream, g.st_keys,
                     g.st_vals, g.ss_keys, g.ss_vals, ew, E, N, degree_on, g.dinv, t_ptr, s_ptr);
  BGCN_CHECK_LAUNCH();
  hipLaunchKernelGGL(k_self_loops, dim3(grid_for(N, blk)), dim3(blk), 0, stream, t_ptr, s_ptr,
                     g.dinv, N, t_row, t_col, t_w, s_row, s_col, s_w);
  BGCN_CHECK_LAUNCH();
  if (E > 0) {
    hipLaunchKernelGGL(k_fill, dim3(grid_for(E, blk)), dim3(blk), 0, stream, ei, ew, E, N,
                       g.st_keys, g.st_vals, g.ss_keys, g.ss_vals, g.dinv, t_row, t_col, t_w,
                       s_row, s_col, s_w);
    BGCN_CHECK_LAUNCH();
  }
  return BGCN_OK;
}

size_t graph_ws_size(int64_t E, int64_t N) {
  Carve c(nullptr, 0);
  carve_graph_ws(c, E, N, nullptr);
  return c.off + 256;
}

}  // namespace bgcn

extern "C" size_t bgcn_graph_workspace_size(int64_t num_edges, int64_t num_nodes) {
  return bgcn::graph_ws_size(num_edges, num_nodes);
}

extern "C" int bgcn_build_graph(const int64_t* edge_index, const float* edge_weight,
                                int64_t num_edges, int64_t num_nodes, int degree_on,
                                int32_t* t_ptr, int32_t* t_row, int32_t* t_col, float* t_w,
                                int32_t* s_ptr, int32_t* s_row, int32_t* s_col, float* s_w,
                                int32_t* status, void* workspace, size_t workspace_bytes,
                                bgcn_stream_t stream) {
  return bgcn::build_graph_impl(edge_index, edge_weight, num_edges, num_nodes, degree_on, t_ptr,
                                t_row, t_col, t_w, s_ptr, s_row, s_col, s_w, status, workspace,
                                workspace_bytes, reinterpret_cast<hipStream_t>(stream));
}
