// K1: gcn_norm + add_remaining_self_loops + CSR construction (both orientations).
//
// Restates PyG >= 2.0 gcn_norm(improved=False, add_self_loops=True,
// flow='source_to_target') as used by every GCNConv call of the reference
// (model/Twitter/BiGCN_Twitter.py:42,56,92,105; explicit call form at
// explain_PHEME.py:62-63), with the PyG 1.3.2 source-degree convention selectable:
//   * existing self loops are removed and one loop (i, i) per node is appended after
//     the edges (its weight = the removed loop's weight, else 1);
//   * deg[i] = sum of edge weights at the target (col) - or source (row) - of i;
//   * norm_e = deg^-1/2[src] * w_e * deg^-1/2[dst]  (inf -> 0).
//
// Both orientations are stable counting sorts of the edge list (entries of a row keep
// edge order, the self loop last = PyG's scatter-add summation order), built with no
// float atomics and no general sort:
//   count (int atomics) -> exclusive scan (3 launches) -> place.
// Placement: when every key's edges form one contiguous run in edge order (always the
// case for propagation trees: TD edges are sorted by (parent, child), each child has one
// parent; BU is the flip) an edge's rank in its row is e - run_start(key).  Otherwise a
// device-side flag selects the general placement (atomic slots + an O(d) rank per entry
// that restores edge order).  The choice is made on the device: no host sync.
//
// Several graphs are built per launch sequence (blockIdx.y = graph): the fused step
// builds TD and BU together.
#include "bgcn_graph_body.h"

namespace bgcn {
namespace {

__global__ __launch_bounds__(kGraphThreads) void k_count(GraphBatch gb) {
  graph_count_body(gb, gb.g[blockIdx.y], int(blockIdx.x));
}

__global__ __launch_bounds__(kScanThreads) void k_scan_lb(GraphBatch gb) {
  graph_scan_body(gb, gb.g[blockIdx.y]);
}

__global__ __launch_bounds__(kGraphThreads) void k_fill_nodes(GraphBatch gb, int nfill) {
  graph_fill_nodes_body(gb, gb.g[blockIdx.y], int(blockIdx.x), nfill);
}

__global__ __launch_bounds__(kGraphThreads) void k_rank_norm(GraphBatch gb, int ne, int nn) {
  graph_rank_norm_body(gb, gb.g[blockIdx.y], int(blockIdx.x), ne, nn);
}

// ---- the multi-block scan (N > kScanSingleMax) and the edge-weighted steps
// block partial sums of (cnt + 1) and of (cnt > 0) over [0, N)
__global__ __launch_bounds__(kScanThreads) void k_scan_blocks(GraphBatch gb) {
  GraphIO& G = gb.g[blockIdx.y];
  const int64_t N = gb.N;
  const int64_t base = int64_t(blockIdx.x) * kScanChunk;
  int st = 0, ss = 0, dt = 0, ds = 0;
  for (int k = 0; k < kScanItems; ++k) {
    int64_t i = base + int64_t(k) * kScanThreads + threadIdx.x;
    if (i < N) {
      int ct = G.cnt_t[i], cs = G.cnt_s[i];
      st += ct + 1; ss += cs + 1; dt += ct > 0; ds += cs > 0;
    }
  }
  __shared__ int red[4][kScanThreads];
  red[0][threadIdx.x] = st; red[1][threadIdx.x] = ss; red[2][threadIdx.x] = dt; red[3][threadIdx.x] = ds;
  __syncthreads();
  for (int o = kScanThreads / 2; o > 0; o >>= 1) {
    if (threadIdx.x < o)
      for (int q = 0; q < 4; ++q) red[q][threadIdx.x] += red[q][threadIdx.x + o];
    __syncthreads();
  }
  if (threadIdx.x < 4) G.bsum[int64_t(blockIdx.x) * 4 + threadIdx.x] = red[threadIdx.x][0];
}

// exclusive scan of the block sums (one block per graph); grouped flags
__global__ __launch_bounds__(kScanThreads) void k_scan_top(GraphBatch gb, int nb) {
  GraphIO& G = gb.g[blockIdx.y];
  __shared__ int sh[2][kScanThreads];
  __shared__ int carry[2];
  __shared__ int dist[2];
  if (threadIdx.x < 2) { carry[threadIdx.x] = 0; dist[threadIdx.x] = 0; }
  __syncthreads();
  for (int c0 = 0; c0 < nb; c0 += kScanThreads) {
    int b = c0 + threadIdx.x;
    int vt = b < nb ? G.bsum[b * 4 + 0] : 0, vs = b < nb ? G.bsum[b * 4 + 1] : 0;
    int dt = b < nb ? G.bsum[b * 4 + 2] : 0, ds = b < nb ? G.bsum[b * 4 + 3] : 0;
    sh[0][threadIdx.x] = vt; sh[1][threadIdx.x] = vs;
    __syncthreads();
    for (int o = 1; o < kScanThreads; o <<= 1) {   // Hillis-Steele inclusive scan
      int a0 = threadIdx.x >= o ? sh[0][threadIdx.x - o] : 0;
      int a1 = threadIdx.x >= o ? sh[1][threadIdx.x - o] : 0;
      __syncthreads();
      sh[0][threadIdx.x] += a0; sh[1][threadIdx.x] += a1;
      __syncthreads();
    }
    if (b < nb) {   // exclusive offsets, reuse the bsum slots 0/1
      G.bsum[b * 4 + 0] = carry[0] + sh[0][threadIdx.x] - vt;
      G.bsum[b * 4 + 1] = carry[1] + sh[1][threadIdx.x] - vs;
    }
    atomicAdd(&dist[0], dt);
    atomicAdd(&dist[1], ds);
    __syncthreads();
    if (threadIdx.x == 0) {
      carry[0] += sh[0][kScanThreads - 1];
      carry[1] += sh[1][kScanThreads - 1];
    }
    __syncthreads();
  }
  if (threadIdx.x == 0) {
    bool clean = G.flags[2] == 0;
    G.flags[3] = (clean && G.flags[0] == dist[0]) ? 1 : 0;
    G.flags[4] = (clean && G.flags[1] == dist[1]) ? 1 : 0;
  }
}

// row pointers: ptr[i] = offset + local exclusive scan of (cnt + 1); ptr[N] = total
__global__ __launch_bounds__(kScanThreads) void k_scan_write(GraphBatch gb) {
  GraphIO& G = gb.g[blockIdx.y];
  const int64_t N = gb.N;
  const int64_t base = int64_t(blockIdx.x) * kScanChunk + int64_t(threadIdx.x) * kScanItems;
  // thread-contiguous items for the write pass
  int vt[kScanItems], vs[kScanItems];
  int st = 0, ss = 0;
  for (int k = 0; k < kScanItems; ++k) {
    int64_t i = base + k;
    vt[k] = i < N ? G.cnt_t[i] + 1 : 0;
    vs[k] = i < N ? G.cnt_s[i] + 1 : 0;
    st += vt[k]; ss += vs[k];
  }
  __shared__ int sh[2][kScanThreads];
  sh[0][threadIdx.x] = st; sh[1][threadIdx.x] = ss;
  __syncthreads();
  for (int o = 1; o < kScanThreads; o <<= 1) {
    int a0 = threadIdx.x >= o ? sh[0][threadIdx.x - o] : 0;
    int a1 = threadIdx.x >= o ? sh[1][threadIdx.x - o] : 0;
    __syncthreads();
    sh[0][threadIdx.x] += a0; sh[1][threadIdx.x] += a1;
    __syncthreads();
  }
  int ot = G.bsum[int64_t(blockIdx.x) * 4 + 0] + sh[0][threadIdx.x] - st;
  int os = G.bsum[int64_t(blockIdx.x) * 4 + 1] + sh[1][threadIdx.x] - ss;
  for (int k = 0; k < kScanItems; ++k) {
    int64_t i = base + k;
    if (i < N) { G.t_ptr[i] = ot; G.s_ptr[i] = os; }
    if (i == N) { G.t_ptr[N] = ot; G.s_ptr[N] = os; }
    ot += vt[k]; os += vs[k];
  }
}

// grouped: direct placement.  general: atomic slot + eid (ordered by k_fill_rank).
__global__ void k_fill(GraphBatch gb) {
  GraphIO& G = gb.g[blockIdx.y];
  const int64_t e = int64_t(blockIdx.x) * blockDim.x + threadIdx.x;
  if (e >= G.E) return;
  int64_t src, dst;
  bool valid;
  if (!edge_kept(G.ei, G.E, gb.N, e, src, dst, valid)) return;
  const float w = G.ew ? G.ew[e] : 1.f;
  if (G.flags[3]) {
    int64_t p = G.t_ptr[dst] + (e - G.run_t[dst]);
    G.t_row[p] = int32_t(dst); G.t_col[p] = int32_t(src); G.t_w[p] = w;
  } else {
    int64_t p = G.t_ptr[dst] + atomicAdd(&G.cur_t[dst], 1);
    G.tmp_t[p] = int32_t(e);
  }
  if (G.flags[4]) {
    int64_t p = G.s_ptr[src] + (e - G.run_s[src]);
    G.s_row[p] = int32_t(src); G.s_col[p] = int32_t(dst); G.s_w[p] = w;
  } else {
    int64_t p = G.s_ptr[src] + atomicAdd(&G.cur_s[src], 1);
    G.tmp_s[p] = int32_t(e);
  }
}

// general path only: rank = number of entries of the row with a smaller edge id
__global__ void k_fill_rank(GraphBatch gb) {
  GraphIO& G = gb.g[blockIdx.y];
  if (G.flags[3] && G.flags[4]) return;
  const int64_t e = int64_t(blockIdx.x) * blockDim.x + threadIdx.x;
  if (e >= G.E) return;
  int64_t src, dst;
  bool valid;
  if (!edge_kept(G.ei, G.E, gb.N, e, src, dst, valid)) return;
  const float w = G.ew ? G.ew[e] : 1.f;
  if (!G.flags[3]) {
    int64_t a = G.t_ptr[dst], n = G.cnt_t[dst];
    int r = 0;
    for (int64_t q = 0; q < n; ++q) r += G.tmp_t[a + q] < e;
    G.t_row[a + r] = int32_t(dst); G.t_col[a + r] = int32_t(src); G.t_w[a + r] = w;
  }
  if (!G.flags[4]) {
    int64_t a = G.s_ptr[src], n = G.cnt_s[src];
    int r = 0;
    for (int64_t q = 0; q < n; ++q) r += G.tmp_s[a + q] < e;
    G.s_row[a + r] = int32_t(src); G.s_col[a + r] = int32_t(dst); G.s_w[a + r] = w;
  }
}

// self loops (raw loop weight) + degree + D^-1/2
__global__ void k_nodes(GraphBatch gb) {
  GraphIO& G = gb.g[blockIdx.y];
  const int64_t i = int64_t(blockIdx.x) * blockDim.x + threadIdx.x;
  if (i >= gb.N) return;
  const int le = G.loop_eid[i];
  const float lw = (le > 0 && G.ew) ? G.ew[le - 1] : 1.f;
  const int64_t pt = G.t_ptr[i + 1] - 1, ps = G.s_ptr[i + 1] - 1;
  // rows of more than kPlanChunk entries: aggregated by a block each (SpmmPlan)
  if (pt + 1 - G.t_ptr[i] > kPlanChunk) G.long_t[atomicAdd(&G.nlong[0], 1)] = int32_t(i);
  if (ps + 1 - G.s_ptr[i] > kPlanChunk) G.long_s[atomicAdd(&G.nlong[1], 1)] = int32_t(i);
  G.t_row[pt] = int32_t(i); G.t_col[pt] = int32_t(i); G.t_w[pt] = lw;
  G.s_row[ps] = int32_t(i); G.s_col[ps] = int32_t(i); G.s_w[ps] = lw;
  // scatter_add over the final edge list in order (real edges, then the loop)
  const bool col = gb.degree_on == BGCN_DEGREE_ON_COL;
  float deg = 0.f;
  if (G.ew) {
    const int64_t a = col ? G.t_ptr[i] : G.s_ptr[i];
    const float* wr = col ? G.t_w : G.s_w;
    for (int64_t p = a; p < (col ? pt : ps); ++p) deg += wr[p];
  } else {
    deg = float(col ? G.cnt_t[i] : G.cnt_s[i]);   // unit weights: the count (exact in fp32)
  }
  deg += lw;
  float d = 1.0f / sqrtf(deg);  // pow(-0.5)
  if (isinf(d)) d = 0.f;
  G.dinv[i] = d;
}

// chunk bounds of a plan: lo = the entry where chunk g starts (a long row at the boundary
// is skipped), hi = where it ends (a long row is excluded)
__device__ __forceinline__ int2 plan_bounds(const int32_t* ptr, const int32_t* row, int64_t nnz, int64_t g) {
  const int64_t p0 = g * kPlanGrid, p1 = p0 + kPlanGrid;
  int lo = int(nnz), hi = int(nnz);
  if (p0 < nnz) {
    const int32_t r = row[p0];
    const int32_t rs = ptr[r], re = ptr[r + 1];
    lo = re - rs > kPlanChunk ? re : rs;
  }
  if (p1 < nnz) hi = ptr[row[p1]];
  return make_int2(lo, hi);
}

__global__ void k_normalize(GraphBatch gb) {
  GraphIO& G = gb.g[blockIdx.y];
  const int64_t p = int64_t(blockIdx.x) * blockDim.x + threadIdx.x;
  // the plans' chunk bounds, chunk g = thread p (the first ngroups threads; rows are
  // final here, k_nodes wrote the self loops)
  if (G.bnd_t && p < (G.E + gb.N + kPlanGrid - 1) / kPlanGrid) {
    G.bnd_t[p] = plan_bounds(G.t_ptr, G.t_row, G.t_ptr[gb.N], p);
    G.bnd_s[p] = plan_bounds(G.s_ptr, G.s_row, G.s_ptr[gb.N], p);
  }
  if (p >= int64_t(G.t_ptr[gb.N])) {
    // the unused tail of the capacity (dropped self loops, invalid edges): row -1 marks
    // it for the aggregation kernels, which then need not read the entry count first
    if (p < G.E + gb.N) {
      G.t_row[p] = -1; G.t_col[p] = 0; G.t_w[p] = 0.f;
      G.s_row[p] = -1; G.s_col[p] = 0; G.s_w[p] = 0.f;
    }
    return;
  }
  // dinv[row] * w * dinv[col] with row = source, col = target (PyG order)
  G.t_w[p] = (G.dinv[G.t_col[p]] * G.t_w[p]) * G.dinv[G.t_row[p]];
  G.s_w[p] = (G.dinv[G.s_row[p]] * G.s_w[p]) * G.dinv[G.s_col[p]];
}

// ---- gcn_norm backward: the gradient w.r.t. edge_weight (EBGCN learns its edge weights,
// model/Twitter/EBGCN.py:101-102 sigmoid -> GCNConv(..., edge_weight) at :84,178).
// With g_e = <dout[dst_e], h[src_e]> (dL/dnorm_e), norm_e = dis[src] w_e dis[dst] and
// dis = deg^-1/2 (deg[k] = the weights summed at k's target - or source - side, its loop
// included):
//   S[k]         = sum_{e: src=k} g_e norm_e + sum_{e: dst=k} g_e norm_e
//                = <dout[k], (A h)[k]> + <h[k], (A^T dout)[k]>     (row dots, no gathers)
//   dL/ddeg[k]   = -1/2 dis[k]^2 S[k]          (0 where dis = 0: the masked inf)
//   dL/dw_e      = g_e dis[src] dis[dst] + dL/ddeg[key_e]            (key = dst, or src)
//   an input self loop (its weight is the node's loop weight, add_remaining_self_loops):
//   dL/dw_e      = <dout[k], h[k]> dis[k]^2 + dL/ddeg[k]
// One 16-lane group per node / per edge, float4 over the (padded) feature width.
struct EwArgs {
  const int64_t* ei;
  int64_t E, N;
  int degree_on;
  const float *dinv, *h, *agg, *dout, *dz;
  int64_t ld;
  int F4;
  float *dldeg, *lgrad, *dw;
};

__device__ __forceinline__ float dot4(float4 a, float4 b) {
  return fmaf(a.x, b.x, fmaf(a.y, b.y, fmaf(a.z, b.z, a.w * b.w)));
}
__device__ __forceinline__ float sum16(float v) {
#pragma unroll
  for (int m = 8; m >= 1; m >>= 1) v += __shfl_xor(v, m, 16);
  return v;
}

__global__ __launch_bounds__(256) void k_ew_nodes(EwArgs a) {
  const int64_t k = (int64_t(blockIdx.x) * blockDim.x + threadIdx.x) / 16;
  const int l = threadIdx.x & 15;
  if (k >= a.N) return;   // group-uniform
  float s1 = 0.f, s2 = 0.f, s3 = 0.f;
  for (int c = 4 * l; c < a.F4; c += 64) {
    const float4 d = ld4(a.dout + k * a.ld + c), h = ld4(a.h + k * a.ld + c);
    s1 += dot4(d, ld4(a.agg + k * a.ld + c));
    s2 += dot4(h, ld4(a.dz + k * a.ld + c));
    s3 += dot4(d, h);
  }
  s1 = sum16(s1); s2 = sum16(s2); s3 = sum16(s3);
  if (l == 0) {
    const float dis = a.dinv[k];
    const float dld = dis > 0.f ? -0.5f * dis * dis * (s1 + s2) : 0.f;
    a.dldeg[k] = dld;
    a.lgrad[k] = s3 * dis * dis + dld;
  }
}

__global__ __launch_bounds__(256) void k_ew_edges(EwArgs a) {
  const int64_t e = (int64_t(blockIdx.x) * blockDim.x + threadIdx.x) / 16;
  const int l = threadIdx.x & 15;
  if (e >= a.E) return;   // group-uniform
  const int64_t src = a.ei[e], dst = a.ei[a.E + e];
  const bool valid = src >= 0 && src < a.N && dst >= 0 && dst < a.N;
  if (!valid || src == dst) {
    if (l == 0) a.dw[e] = valid ? a.lgrad[src] : 0.f;   // an input loop: the loop weight's gradient
    return;
  }
  float s = 0.f;
  for (int c = 4 * l; c < a.F4; c += 64) s += dot4(ld4(a.dout + dst * a.ld + c), ld4(a.h + src * a.ld + c));
  s = sum16(s);
  if (l == 0)
    a.dw[e] = s * a.dinv[src] * a.dinv[dst] + a.dldeg[a.degree_on == BGCN_DEGREE_ON_COL ? dst : src];
}

}  // namespace

size_t graph_carve(Carve& c, int64_t E, int64_t N, GraphIO* G, size_t* zero_bytes) {
  const size_t n = size_t(N > 0 ? N : 1), cap = size_t(E + N > 0 ? E + N : 1);
  const int64_t nb = (N + 1 + kScanChunk - 1) / kScanChunk;
  GraphIO t{};
  // zero-initialised block first (one memset)
  t.cnt_t = c.take<int32_t>(n);
  t.cnt_s = c.take<int32_t>(n);
  t.cur_t = c.take<int32_t>(n);
  t.cur_s = c.take<int32_t>(n);
  t.loop_eid = c.take<int32_t>(n);
  t.flags = c.take<int32_t>(8);
  t.nlong = c.take<int32_t>(2);
  t.lb = c.take<uint64_t>(size_t(graph_scan_tiles(N)));
  t.run_t = c.take<int32_t>(n);
  t.run_s = c.take<int32_t>(n);
  t.tmp_t = c.take<int32_t>(cap);
  t.tmp_s = c.take<int32_t>(cap);
  t.bsum = c.take<int32_t>(size_t(nb) * 4);
  t.dinv = c.take<float>(n);
  const size_t ng = (cap + kPlanGrid - 1) / kPlanGrid;
  t.bnd_t = c.take<int2>(ng);
  t.bnd_s = c.take<int2>(ng);
  t.long_t = c.take<int32_t>(n);
  t.long_s = c.take<int32_t>(n);
  if (G) *G = t;
  if (zero_bytes) *zero_bytes = size_t(reinterpret_cast<char*>(t.run_t) - reinterpret_cast<char*>(t.cnt_t));
  return c.off;
}

size_t graph_ws_size(int64_t E, int64_t N) {
  Carve c(nullptr, 0);
  graph_carve(c, E, N, nullptr, nullptr);
  return c.off + 256;
}

int graph_batch_setup(const GraphArgs* ga, int count, int64_t N, int degree_on, GraphBatch* out,
                      size_t zero_bytes[kMaxGraphs], const int64_t* batch) {
  BGCN_CHECK_ARG(count >= 1 && count <= kMaxGraphs, "1 or 2 graphs per call");
  BGCN_CHECK_ARG(N > 0 && N < (int64_t(1) << 31) - 1, "num_nodes out of range");
  BGCN_CHECK_ARG(degree_on == BGCN_DEGREE_ON_COL || degree_on == BGCN_DEGREE_ON_ROW,
                 "degree_on must be 0 (col) or 1 (row)");
  GraphBatch gb{};
  gb.N = N;
  gb.degree_on = degree_on;
  gb.batch = batch;
  for (int k = 0; k < count; ++k) {
    const GraphArgs& a = ga[k];
    BGCN_CHECK_ARG(a.E >= 0 && a.E + N < (int64_t(1) << 31), "num_edges out of range");
    BGCN_CHECK_ARG(a.t_ptr && a.t_row && a.t_col && a.t_w && a.s_ptr && a.s_row && a.s_col && a.s_w,
                   "null output pointer");
    BGCN_CHECK_ARG(a.E == 0 || a.ei, "null edge_index");
    BGCN_CHECK_ARG(a.ws && a.ws_bytes >= graph_ws_size(a.E, N), "workspace too small");
    Carve c(a.ws, a.ws_bytes);
    GraphIO& G = gb.g[k];
    graph_carve(c, a.E, N, &G, &zero_bytes[k]);
    G.ei = a.ei; G.ew = a.ew; G.E = a.E;
    G.t_ptr = a.t_ptr; G.t_row = a.t_row; G.t_col = a.t_col; G.t_w = a.t_w;
    G.s_ptr = a.s_ptr; G.s_row = a.s_row; G.s_col = a.s_col; G.s_w = a.s_w;
    G.status = a.status;
  }
  *out = gb;
  return BGCN_OK;
}

int build_graphs_impl(const GraphArgs* ga, int count, int64_t N, int degree_on, hipStream_t s,
                      const int64_t* batch) {
  BGCN_CHECK_ARG(count >= 1 && count <= kMaxGraphs, "1 or 2 graphs per call");
  BGCN_CHECK_ARG(N > 0 && N < (int64_t(1) << 31) - 1, "num_nodes out of range");
  BGCN_CHECK_ARG(degree_on == BGCN_DEGREE_ON_COL || degree_on == BGCN_DEGREE_ON_ROW,
                 "degree_on must be 0 (col) or 1 (row)");
  GraphBatch gb{};
  gb.N = N;
  gb.degree_on = degree_on;
  gb.batch = batch;
  int64_t Emax = 0;
  for (int k = 0; k < count; ++k) {
    const GraphArgs& a = ga[k];
    BGCN_CHECK_ARG(a.E >= 0 && a.E + N < (int64_t(1) << 31), "num_edges out of range");
    BGCN_CHECK_ARG(a.t_ptr && a.t_row && a.t_col && a.t_w && a.s_ptr && a.s_row && a.s_col && a.s_w,
                   "null output pointer");
    BGCN_CHECK_ARG(a.E == 0 || a.ei, "null edge_index");
    BGCN_CHECK_ARG(a.ws && a.ws_bytes >= graph_ws_size(a.E, N), "workspace too small");
    Carve c(a.ws, a.ws_bytes);
    GraphIO& G = gb.g[k];
    size_t zero_bytes = 0;
    graph_carve(c, a.E, N, &G, &zero_bytes);
    G.ei = a.ei; G.ew = a.ew; G.E = a.E;
    G.t_ptr = a.t_ptr; G.t_row = a.t_row; G.t_col = a.t_col; G.t_w = a.t_w;
    G.s_ptr = a.s_ptr; G.s_row = a.s_row; G.s_col = a.s_col; G.s_w = a.s_w;
    G.status = a.status;
    BGCN_CHECK_HIP(hipMemsetAsync(G.cnt_t, 0, zero_bytes, s));
    Emax = a.E > Emax ? a.E : Emax;
  }
  const unsigned gy = unsigned(count);
  const int blk = 256;
  const int64_t nb = (N + 1 + kScanChunk - 1) / kScanChunk;
  bool weighted = false;
  for (int k = 0; k < count; ++k) weighted = weighted || ga[k].ew != nullptr;
  if (Emax > 0) {
    hipLaunchKernelGGL(k_count, dim3(grid_for(Emax, blk), gy), dim3(blk), 0, s, gb);
    BGCN_CHECK_LAUNCH();
  }
  if (!weighted) {   // count -> scan -> fill_nodes -> rank_norm (bgcn_graph_body.h)
    hipLaunchKernelGGL(k_scan_lb, dim3(unsigned(graph_scan_tiles(N)), gy), dim3(kScanThreads), 0, s, gb);
    BGCN_CHECK_LAUNCH();
    const int ne = graph_edge_blocks(Emax), nn = graph_node_blocks(N), np = graph_pos_blocks(Emax, N);
    hipLaunchKernelGGL(k_fill_nodes, dim3(unsigned(ne + nn), gy), dim3(kGraphThreads), 0, s, gb, ne);
    BGCN_CHECK_LAUNCH();
    hipLaunchKernelGGL(k_rank_norm, dim3(unsigned(ne + nn + np), gy), dim3(kGraphThreads), 0, s, gb, ne, nn);
    BGCN_CHECK_LAUNCH();
    return BGCN_OK;
  }
  hipLaunchKernelGGL(k_scan_blocks, dim3(unsigned(nb), gy), dim3(kScanThreads), 0, s, gb);
  BGCN_CHECK_LAUNCH();
  hipLaunchKernelGGL(k_scan_top, dim3(1, gy), dim3(kScanThreads), 0, s, gb, int(nb));
  BGCN_CHECK_LAUNCH();
  hipLaunchKernelGGL(k_scan_write, dim3(unsigned(nb), gy), dim3(kScanThreads), 0, s, gb);
  BGCN_CHECK_LAUNCH();
  if (Emax > 0) {
    hipLaunchKernelGGL(k_fill, dim3(grid_for(Emax, blk), gy), dim3(blk), 0, s, gb);
    BGCN_CHECK_LAUNCH();
    hipLaunchKernelGGL(k_fill_rank, dim3(grid_for(Emax, blk), gy), dim3(blk), 0, s, gb);
    BGCN_CHECK_LAUNCH();
  }
  hipLaunchKernelGGL(k_nodes, dim3(grid_for(N, blk), gy), dim3(blk), 0, s, gb);
  BGCN_CHECK_LAUNCH();
  hipLaunchKernelGGL(k_normalize, dim3(grid_for(Emax + N, blk), gy), dim3(blk), 0, s, gb);
  BGCN_CHECK_LAUNCH();
  return BGCN_OK;
}

void graph_pair_plans(void* ws, size_t ws_bytes, int64_t Etd, int64_t Ebu, int64_t N, SpmmPlan td[2],
                      SpmmPlan bu[2]) {
  const size_t half = ws_bytes / 2 / 256 * 256;
  char* base = static_cast<char*>(ws);
  for (int k = 0; k < 2; ++k) {
    Carve c(base + k * half, half);
    GraphIO G{};
    graph_carve(c, k == 0 ? Etd : Ebu, N, &G, nullptr);
    SpmmPlan* o = k == 0 ? td : bu;
    o[0] = SpmmPlan{G.bnd_t, G.long_t, G.nlong};
    o[1] = SpmmPlan{G.bnd_s, G.long_s, G.nlong + 1};
  }
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
  bgcn::GraphArgs a{edge_index, edge_weight, num_edges, t_ptr, t_row, t_col, t_w,
                    s_ptr, s_row, s_col, s_w, status, workspace, workspace_bytes};
  return bgcn::build_graphs_impl(&a, 1, num_nodes, degree_on, reinterpret_cast<hipStream_t>(stream), nullptr);
}

extern "C" int bgcn_graph_pair_plans(const void* workspace, size_t workspace_bytes, int64_t td_num_edges,
                                     int64_t bu_num_edges, int64_t num_nodes, bgcn_spmm_plan td[2],
                                     bgcn_spmm_plan bu[2]) {
  if (!workspace || !td || !bu || num_nodes <= 0 || td_num_edges < 0 || bu_num_edges < 0)
    return bgcn::fail(BGCN_EINVAL, "bad arguments");
  const int64_t e = td_num_edges > bu_num_edges ? td_num_edges : bu_num_edges;
  if (workspace_bytes < 2 * bgcn::align_up(bgcn::graph_ws_size(e, num_nodes), 256))
    return bgcn::fail(BGCN_EINVAL, "workspace smaller than the build's");
  bgcn::SpmmPlan p[2][2];
  bgcn::graph_pair_plans(const_cast<void*>(workspace), workspace_bytes, td_num_edges, bu_num_edges, num_nodes,
                         p[0], p[1]);
  for (int o = 0; o < 2; ++o) {
    td[o] = bgcn_spmm_plan{p[0][o].bnd, p[0][o].longs, p[0][o].nlong};
    bu[o] = bgcn_spmm_plan{p[1][o].bnd, p[1][o].longs, p[1][o].nlong};
  }
  return BGCN_OK;
}

extern "C" size_t bgcn_graph_pair_workspace_size(int64_t td_num_edges, int64_t bu_num_edges,
                                                int64_t num_nodes) {
  int64_t e = td_num_edges > bu_num_edges ? td_num_edges : bu_num_edges;
  return 2 * bgcn::align_up(bgcn::graph_ws_size(e, num_nodes), 256);
}

namespace bgcn {
void graph_pair_args(const int64_t* td_ei, int64_t Etd, const int64_t* bu_ei, int64_t Ebu,
                     const bgcn_csr_out* td, const bgcn_csr_out* bu, int32_t* status, void* workspace,
                     size_t workspace_bytes, GraphArgs a[2]) {
  const size_t half = workspace_bytes / 2 / 256 * 256;
  char* ws = static_cast<char*>(workspace);
  a[0] = GraphArgs{td_ei, nullptr, Etd, td->t_ptr, td->t_row, td->t_col, td->t_w, td->s_ptr,
                   td->s_row, td->s_col, td->s_w, status, ws, half};
  a[1] = GraphArgs{bu_ei, nullptr, Ebu, bu->t_ptr, bu->t_row, bu->t_col, bu->t_w, bu->s_ptr,
                   bu->s_row, bu->s_col, bu->s_w, status, ws ? ws + half : nullptr, half};
}
}  // namespace bgcn

extern "C" int bgcn_build_graph_pair(const int64_t* td_edge_index, int64_t td_num_edges,
                                     const int64_t* bu_edge_index, int64_t bu_num_edges,
                                     int64_t num_nodes, int degree_on, const bgcn_csr_out* td,
                                     const bgcn_csr_out* bu, const int64_t* batch, int32_t* status,
                                     void* workspace, size_t workspace_bytes, bgcn_stream_t stream) {
  using bgcn::GraphArgs;
  if (!td || !bu) return bgcn::fail(BGCN_EINVAL, "null csr descriptor");
  const size_t half = workspace_bytes / 2 / 256 * 256;
  char* ws = static_cast<char*>(workspace);
  GraphArgs a[2] = {
      {td_edge_index, nullptr, td_num_edges, td->t_ptr, td->t_row, td->t_col, td->t_w, td->s_ptr,
       td->s_row, td->s_col, td->s_w, status, ws, half},
      {bu_edge_index, nullptr, bu_num_edges, bu->t_ptr, bu->t_row, bu->t_col, bu->t_w, bu->s_ptr,
       bu->s_row, bu->s_col, bu->s_w, status, ws ? ws + half : nullptr, half}};
  return bgcn::build_graphs_impl(a, 2, num_nodes, degree_on, reinterpret_cast<hipStream_t>(stream), batch);
}

extern "C" int bgcn_graph_dinv(const void* workspace, size_t workspace_bytes, int64_t num_edges, int64_t num_nodes,
                               const float** dinv) {
  if (!workspace || !dinv || num_nodes <= 0 || num_edges < 0) return bgcn::fail(BGCN_EINVAL, "bad arguments");
  if (workspace_bytes < bgcn::graph_ws_size(num_edges, num_nodes))
    return bgcn::fail(BGCN_EINVAL, "workspace smaller than the build's");
  bgcn::Carve c(const_cast<void*>(workspace), workspace_bytes);
  bgcn::GraphIO G{};
  bgcn::graph_carve(c, num_edges, num_nodes, &G, nullptr);
  *dinv = G.dinv;
  return BGCN_OK;
}

extern "C" size_t bgcn_edge_weight_grad_workspace_size(int64_t num_nodes) {
  return num_nodes > 0 ? 2 * bgcn::align_up(size_t(num_nodes) * sizeof(float), 256) + 256 : 0;
}

extern "C" int bgcn_edge_weight_grad(const int64_t* edge_index, int64_t num_edges, int64_t num_nodes, int degree_on,
                                     const float* dinv, const float* h, const float* agg, const float* dout,
                                     const float* dz, int64_t ld, int32_t F, float* d_edge_weight, void* workspace,
                                     size_t workspace_bytes, bgcn_stream_t stream) {
  using namespace bgcn;
  BGCN_CHECK_ARG(num_nodes > 0 && num_edges >= 0 && F > 0 && F % 4 == 0 && ld >= F && ld % 4 == 0,
                 "bad sizes (F and ld: multiples of 4)");
  BGCN_CHECK_ARG(degree_on == BGCN_DEGREE_ON_COL || degree_on == BGCN_DEGREE_ON_ROW, "bad degree_on");
  BGCN_CHECK_ARG(dinv && h && agg && dout && dz && (num_edges == 0 || (edge_index && d_edge_weight)), "null pointer");
  BGCN_CHECK_ARG(workspace && workspace_bytes >= bgcn_edge_weight_grad_workspace_size(num_nodes),
                 "workspace too small");
  Carve c(workspace, workspace_bytes);
  EwArgs a{edge_index, num_edges, num_nodes, degree_on, dinv, h, agg, dout, dz, ld, int(F),
           c.take<float>(size_t(num_nodes)), c.take<float>(size_t(num_nodes)), d_edge_weight};
  hipStream_t s = reinterpret_cast<hipStream_t>(stream);
  hipLaunchKernelGGL(k_ew_nodes, dim3(grid_for(num_nodes * 16, 256)), dim3(256), 0, s, a);
  BGCN_CHECK_LAUNCH();
  if (num_edges > 0) {
    hipLaunchKernelGGL(k_ew_edges, dim3(grid_for(num_edges * 16, 256)), dim3(256), 0, s, a);
    BGCN_CHECK_LAUNCH();
  }
  return BGCN_OK;
}
