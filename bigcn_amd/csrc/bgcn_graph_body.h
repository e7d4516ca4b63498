// K1 device bodies (gcn_norm + add_remaining_self_loops + CSR, both orientations):
// shared by the generic graph build (bgcn_graph.hip) and the fused step's batch
// preparation, which runs them as roles of merged launches (bgcn_sparse.hip).
//
// Unweighted graphs (every GCNConv of the BiGCN path) take four steps:
//   count        per edge: target / source counts (int atomics), run starts
//   scan         exclusive scan of (count + 1) -> row pointers, "grouped" flags
//   fill_nodes   per edge: placement (run rank when grouped, else an atomic slot);
//                per node: the self loop (last in its row), D^-1/2, long-row lists
//   rank_norm    per edge: the normalised weight at its final slot (general path: the
//                rank that restores edge order); per node: the loop's weight; the
//                capacity tail (row -1) and the aggregation plans' chunk bounds
// Edge-weighted graphs keep the older fill / fill_rank / nodes / normalize split
// (bgcn_graph.hip): their degree sums the placed weights in row order.
#pragma once

#include "bgcn_common.h"

namespace bgcn {

constexpr int kMaxGraphs = 2;
constexpr int kScanThreads = 256, kScanItems = 4, kScanChunk = kScanThreads * kScanItems;
constexpr int kGraphThreads = 256;     // block size of the per-edge / per-node bodies

struct GraphIO {
  const int64_t* ei;
  const float* ew;
  int64_t E;
  int32_t *t_ptr, *t_row, *t_col;
  float* t_w;
  int32_t *s_ptr, *s_row, *s_col;
  float* s_w;
  int32_t* status;
  // scratch
  int32_t *cnt_t, *cnt_s, *cur_t, *cur_s, *loop_eid;  // zero-initialised block
  int32_t* flags;   // [0] runs_t [1] runs_s [2] excluded [3] grouped_t [4] grouped_s (weighted
                    // path) [5] keys_t [6] keys_s [7] scan ticket (unweighted path)
  uint64_t* lb;                                          // [tiles] look-back words (zeroed block)
  int32_t *run_t, *run_s;                                // run start per key
  int32_t *tmp_t, *tmp_s;                                // general path: eid per slot
  int32_t* bsum;                                         // [nb][4]: sum_t, sum_s, distinct_t, distinct_s
  float* dinv;
  int32_t* nlong;                                        // [2] long rows t / s (zeroed block)
  int2 *bnd_t, *bnd_s;                                   // aggregation plans (SpmmPlan)
  int32_t *long_t, *long_s;
};

struct GraphBatch {
  GraphIO g[kMaxGraphs];
  int64_t N;
  int degree_on;
  const int64_t* batch;   // optional [N] tree ids: an edge across trees sets BGCN_STATUS_CROSS_TREE
};

__device__ __forceinline__ bool edge_kept(const int64_t* ei, int64_t E, int64_t N, int64_t e,
                                          int64_t& src, int64_t& dst, bool& valid) {
  src = ei[e];
  dst = ei[E + e];
  valid = src >= 0 && src < N && dst >= 0 && dst < N;
  return valid && src != dst;
}

// count: edge e = bid * blockDim + thread.  Run-start counters are wave-aggregated
// (ballot + popcount, one atomic per wave): in a propagation tree nearly every edge
// starts a run, and per-edge atomics on one address serialise.
// Per-node counts are wave-aggregated too: the edges of one node come in runs (a BU star
// root's children, a TD parent's), and a run inside a wave adds its length with one
// atomic from its first lane instead of one atomic per edge on the same address.
__device__ __forceinline__ void add_runs(int32_t* __restrict__ cnt, bool keep, int64_t key) {
  const int lane = threadIdx.x & (kWave - 1);
  const int64_t pkey = __shfl_up(key, 1, kWave);
  const bool pkeep = __shfl_up(int(keep), 1, kWave) != 0;
  const bool lead = keep && (lane == 0 || !pkeep || pkey != key);
  const uint64_t km = __ballot(keep), lm = __ballot(lead);
  if (lead) {
    const uint64_t after = lane == kWave - 1 ? 0ull : (lm >> (lane + 1)) << (lane + 1);
    const int next = after ? __builtin_ctzll(after) : kWave;   // the next run's first lane
    const uint64_t span = (next == kWave ? ~0ull : ((1ull << next) - 1ull)) & ~((1ull << lane) - 1ull);
    atomicAdd(&cnt[key], __popcll(km & span));
  }
}

__device__ inline void graph_count_body(const GraphBatch& gb, const GraphIO& G, int bid) {
  const int64_t e = int64_t(bid) * blockDim.x + threadIdx.x;
  const int64_t N = gb.N;
  bool start_t = false, start_s = false;
  bool kept = false;
  int64_t ksrc = 0, kdst = 0;
  if (e < G.E) {
    int64_t src, dst;
    bool valid;
    const bool keep = edge_kept(G.ei, G.E, N, e, src, dst, valid);
    if (!valid) {
      if (G.status) atomicOr(G.status, 1);
      atomicOr(&G.flags[2], 1);
    } else if (!keep) {  // an input self loop: removed, its weight becomes the loop weight
      if (G.ew) atomicMax(&G.loop_eid[src], int32_t(e + 1));  // (last wins; unweighted: 1)
      // run-based ranks (e - run start) hold unless the loop sits inside a run of its
      // own node, i.e. the next edge is a kept edge at that node; a loop between runs of
      // other nodes shows up as a surplus run start (the scan's check)
      if (e + 1 < G.E) {
        int64_t ns, nd;
        bool nv;
        if (edge_kept(G.ei, G.E, N, e + 1, ns, nd, nv) && (ns == src || nd == src))
          atomicOr(&G.flags[2], 1);
      }
    } else {
      kept = true;
      ksrc = src;
      kdst = dst;
      // a propagation tree's edges stay inside it (PyG collation); the fused readout
      // backward needs to know when they do not (bgcn.h BGCN_STATUS_CROSS_TREE)
      if (gb.batch && G.status && gb.batch[src] != gb.batch[dst]) atomicOr(G.status, BGCN_STATUS_CROSS_TREE);
      int64_t psrc = -1, pdst = -1;
      if (e > 0) {
        bool pv;
        edge_kept(G.ei, G.E, N, e - 1, psrc, pdst, pv);
      }
      start_t = e == 0 || pdst != dst;
      start_s = e == 0 || psrc != src;
      if (start_t) G.run_t[dst] = int32_t(e);
      if (start_s) G.run_s[src] = int32_t(e);
    }
  }
  add_runs(G.cnt_t, kept, kdst);
  add_runs(G.cnt_s, kept, ksrc);
  const int nt = __popcll(__ballot(start_t)), ns = __popcll(__ballot(start_s));
  if ((threadIdx.x & (kWave - 1)) == 0) {
    if (nt) atomicAdd(&G.flags[0], nt);
    if (ns) atomicAdd(&G.flags[1], ns);
  }
}

// Single-pass scan with decoupled look-back: ptr[i] = sum_{j < i} (cnt[j] + 1) for both
// orientations, ptr[N] = the total; blocks take tiles of kScanTile nodes in the order
// they start (a ticket, flags[7]), so a tile's predecessors are running or done.  A
// tile publishes its aggregate at once and its inclusive prefix once known, both as
// one 8-byte word {flag:2 | t:31 | s:31} (an agent-scope atomic store: the payload is
// the flag, no fence); one wave reads up to 64 predecessors' words at a time, sums the
// aggregates back to the nearest inclusive prefix.  The keys-with-edges counts behind
// the grouped flags go to flags[5] / flags[6] (int atomics); the later steps derive the
// flags from them.  lb[] and flags[5..7] must be zero before the launch.
constexpr int kScanPer = 8;
constexpr int kScanTile = kScanThreads * kScanPer;
constexpr uint64_t kLbAgg = 1ull << 62, kLbInc = 2ull << 62;
// tiles covering indices [0, N] (ptr[N] is written by the tile holding index N)
__host__ __device__ inline int64_t graph_scan_tiles(int64_t N) { return N / kScanTile + 1; }

__device__ inline void graph_scan_body(const GraphBatch& gb, const GraphIO& G) {
  __shared__ int ticket;
  __shared__ int wsum[2][kScanThreads / kWave];
  __shared__ int wdist[2][kScanThreads / kWave];
  __shared__ int excl[2];
  const int64_t N = gb.N;
  const int tid = threadIdx.x, lane = tid & (kWave - 1), wv = tid / kWave;
  constexpr int nw = kScanThreads / kWave;
  if (tid == 0) ticket = atomicAdd(&G.flags[7], 1);
  __syncthreads();
  const int tile = ticket;
  const int64_t base = int64_t(tile) * kScanTile + int64_t(tid) * kScanPer;
  int ct[kScanPer], cs[kScanPer];
#pragma unroll
  for (int k = 0; k < kScanPer; ++k) {
    const int64_t i = min<int64_t>(base + k, N - 1);
    ct[k] = G.cnt_t[i];
    cs[k] = G.cnt_s[i];
  }
  int lt = 0, ls = 0, dt = 0, ds = 0;
#pragma unroll
  for (int k = 0; k < kScanPer; ++k) {
    const bool in = base + k < N;
    dt += in && ct[k] > 0;
    ds += in && cs[k] > 0;
    ct[k] = in ? ct[k] + 1 : 0;
    cs[k] = in ? cs[k] + 1 : 0;
    lt += ct[k];
    ls += cs[k];
  }
  int it = lt, is = ls;
  for (int o = 1; o < kWave; o <<= 1) {
    const int x = __shfl_up(it, o, kWave), y = __shfl_up(is, o, kWave);
    if (lane >= o) { it += x; is += y; }
  }
  for (int o = kWave / 2; o > 0; o >>= 1) {
    dt += __shfl_xor(dt, o, kWave);
    ds += __shfl_xor(ds, o, kWave);
  }
  if (lane == kWave - 1) { wsum[0][wv] = it; wsum[1][wv] = is; }
  if (lane == 0) { wdist[0][wv] = dt; wdist[1][wv] = ds; }
  __syncthreads();
  int ot = it - lt, os = is - ls, at = 0, as = 0, nt = 0, ns = 0;
#pragma unroll
  for (int w = 0; w < nw; ++w) {
    ot += w < wv ? wsum[0][w] : 0;
    os += w < wv ? wsum[1][w] : 0;
    at += wsum[0][w];
    as += wsum[1][w];
    nt += wdist[0][w];
    ns += wdist[1][w];
  }
  uint64_t* lb = G.lb;
  if (wv == 0) {
    if (lane == 0) {
      if (nt) atomicAdd(&G.flags[5], nt);
      if (ns) atomicAdd(&G.flags[6], ns);
      const uint64_t mine = (uint64_t(uint32_t(at)) << 31) | uint64_t(uint32_t(as));
      __hip_atomic_store(lb + tile, (tile == 0 ? kLbInc : kLbAgg) | mine, __ATOMIC_RELAXED,
                         __HIP_MEMORY_SCOPE_AGENT);
    }
    int pt = 0, ps = 0;
    if (tile > 0) {   // look back, 64 predecessors per round (uniform loop)
      int j = tile - 1;
      unsigned spins = 0;
      for (;;) {
        const int q = j - lane;
        const uint64_t w = q >= 0 ? __hip_atomic_load(lb + q, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT)
                                  : kLbInc;   // before tile 0: an empty inclusive prefix
        const uint64_t fl = w >> 62;
        const uint64_t ready = __ballot(fl != 0), inc = __ballot(fl == 2);
        // lanes up to the nearest inclusive prefix must all be published
        const int stop = inc ? __builtin_ctzll(inc) : kWave;   // first lane (nearest) with a prefix
        const uint64_t need = stop >= kWave - 1 ? ~0ull : ((2ull << stop) - 1ull);
        if ((ready & need) != need) {
          if (++spins > (1u << 22)) {   // a lost predecessor: flag the graph, never hang
            if (lane == 0 && G.status) atomicOr(G.status, kStatusInternal);
            break;
          }
          __builtin_amdgcn_s_sleep(1);
          continue;
        }
        const bool take = lane <= stop;
        int vt = take ? int((w >> 31) & 0x7fffffffu) : 0, vs = take ? int(w & 0x7fffffffu) : 0;
        for (int o = kWave / 2; o > 0; o >>= 1) {
          vt += __shfl_xor(vt, o, kWave);
          vs += __shfl_xor(vs, o, kWave);
        }
        pt += vt;
        ps += vs;
        if (stop < kWave) break;
        j -= kWave;
      }
      if (lane == 0)
        __hip_atomic_store(lb + tile, kLbInc | (uint64_t(uint32_t(pt + at)) << 31) | uint64_t(uint32_t(ps + as)),
                           __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    }
    if (lane == 0) { excl[0] = pt; excl[1] = ps; }
  }
  __syncthreads();
  ot += excl[0];
  os += excl[1];
#pragma unroll
  for (int k = 0; k < kScanPer; ++k) {
    const int64_t i = base + k;
    if (i < N) { G.t_ptr[i] = ot; G.s_ptr[i] = os; }
    if (i == N) { G.t_ptr[N] = ot; G.s_ptr[N] = os; }
    ot += ct[k];
    os += cs[k];
  }
}

// grouped flags (every key's edges one contiguous run, nothing excluded), from the
// count step's run starts and the scan's keys-with-edges counts
__device__ __forceinline__ bool graph_grouped_t(const GraphIO& G) {
  return G.flags[2] == 0 && G.flags[0] == G.flags[5];
}
__device__ __forceinline__ bool graph_grouped_s(const GraphIO& G) {
  return G.flags[2] == 0 && G.flags[1] == G.flags[6];
}

// fill_nodes, unweighted graphs.  Blocks [0, nfill): edge e - grouped: its final slot
// ptr + (e - run start) gets (row, col); general: an atomic slot records e (rank_norm
// orders them).  Blocks from nfill: node i - the self loop (weight 1) last in both of
// its rows, D^-1/2 of (count + 1), and rows of more than kPlanChunk entries listed for
// the aggregation plans.
__device__ inline void graph_fill_nodes_body(const GraphBatch& gb, const GraphIO& G, int bid, int nfill) {
  if (bid < nfill) {
    const int64_t e = int64_t(bid) * blockDim.x + threadIdx.x;
    if (e >= G.E) return;
    int64_t src, dst;
    bool valid;
    if (!edge_kept(G.ei, G.E, gb.N, e, src, dst, valid)) return;
    if (graph_grouped_t(G)) {
      const int64_t p = G.t_ptr[dst] + (e - G.run_t[dst]);
      G.t_row[p] = int32_t(dst); G.t_col[p] = int32_t(src);
    } else {
      G.tmp_t[G.t_ptr[dst] + atomicAdd(&G.cur_t[dst], 1)] = int32_t(e);
    }
    if (graph_grouped_s(G)) {
      const int64_t p = G.s_ptr[src] + (e - G.run_s[src]);
      G.s_row[p] = int32_t(src); G.s_col[p] = int32_t(dst);
    } else {
      G.tmp_s[G.s_ptr[src] + atomicAdd(&G.cur_s[src], 1)] = int32_t(e);
    }
    return;
  }
  const int64_t i = int64_t(bid - nfill) * blockDim.x + threadIdx.x;
  if (i >= gb.N) return;
  const int64_t pt = G.t_ptr[i + 1] - 1, ps = G.s_ptr[i + 1] - 1;
  if (pt + 1 - G.t_ptr[i] > kPlanChunk) G.long_t[atomicAdd(&G.nlong[0], 1)] = int32_t(i);
  if (ps + 1 - G.s_ptr[i] > kPlanChunk) G.long_s[atomicAdd(&G.nlong[1], 1)] = int32_t(i);
  G.t_row[pt] = int32_t(i); G.t_col[pt] = int32_t(i);
  G.s_row[ps] = int32_t(i); G.s_col[ps] = int32_t(i);
  // scatter_add of unit weights over the final edge list: the count (exact in fp32) + the loop
  const bool col = gb.degree_on == BGCN_DEGREE_ON_COL;
  const float deg = float(col ? G.cnt_t[i] : G.cnt_s[i]) + 1.f;
  float d = 1.0f / sqrtf(deg);  // pow(-0.5)
  if (isinf(d)) d = 0.f;
  G.dinv[i] = d;
}

// chunk bounds of a plan: lo = the entry where chunk g starts (a long row at the boundary
// is skipped), hi = where it ends (a long row is excluded).  row_of(p) = the row holding
// entry p (every row has its self loop, so rows are never empty).
__device__ __forceinline__ int32_t row_of(const int32_t* ptr, int64_t N, int64_t p) {
  int64_t lo = 0, hi = N - 1;   // largest r with ptr[r] <= p
  while (lo < hi) {
    const int64_t mid = (lo + hi + 1) >> 1;
    if (ptr[mid] <= p) lo = mid; else hi = mid - 1;
  }
  return int32_t(lo);
}
__device__ __forceinline__ int2 plan_bounds_ptr(const int32_t* ptr, int64_t N, int64_t nnz, int64_t g) {
  const int64_t p0 = g * kPlanGrid, p1 = p0 + kPlanGrid;
  int lo = int(nnz), hi = int(nnz);
  if (p0 < nnz) {
    const int32_t r = row_of(ptr, N, p0);
    const int32_t rs = ptr[r], re = ptr[r + 1];
    lo = re - rs > kPlanChunk ? re : rs;
  }
  if (p1 < nnz) hi = ptr[row_of(ptr, N, p1)];
  return make_int2(lo, hi);
}

__device__ __forceinline__ int2 plan_bounds_row(const int32_t* ptr, const int32_t* row, int64_t nnz,
                                               int64_t g) {
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

// rank_norm, unweighted graphs.  Blocks [0, ne): edge e - its normalised weight
// dinv[src] * 1 * dinv[dst] (PyG order) at its final slot in both orientations (general
// path: the slot of rank = number of the row's entries with a smaller edge id, which
// restores edge order).  Blocks [ne, ne + nn): node i - its self loop's weight.  Blocks
// from ne + nn: entry position p - the unused capacity tail (row -1: the aggregation
// kernels then need not read the entry count) and, for p < ngroups, the plans' chunk
// bounds (from the row pointers alone).
__device__ inline void graph_rank_norm_body(const GraphBatch& gb, const GraphIO& G, int bid, int ne,
                                            int nn) {
  const int64_t N = gb.N;
  if (bid < ne) {
    const int64_t e = int64_t(bid) * blockDim.x + threadIdx.x;
    if (e >= G.E) return;
    int64_t src, dst;
    bool valid;
    if (!edge_kept(G.ei, G.E, N, e, src, dst, valid)) return;
    const float wn = (G.dinv[src] * 1.f) * G.dinv[dst];
    if (graph_grouped_t(G)) {
      G.t_w[G.t_ptr[dst] + (e - G.run_t[dst])] = wn;
    } else {
      const int64_t a = G.t_ptr[dst], n = G.cnt_t[dst];
      int r = 0;
      for (int64_t q = 0; q < n; ++q) r += G.tmp_t[a + q] < e;
      G.t_row[a + r] = int32_t(dst); G.t_col[a + r] = int32_t(src); G.t_w[a + r] = wn;
    }
    if (graph_grouped_s(G)) {
      G.s_w[G.s_ptr[src] + (e - G.run_s[src])] = wn;
    } else {
      const int64_t a = G.s_ptr[src], n = G.cnt_s[src];
      int r = 0;
      for (int64_t q = 0; q < n; ++q) r += G.tmp_s[a + q] < e;
      G.s_row[a + r] = int32_t(src); G.s_col[a + r] = int32_t(dst); G.s_w[a + r] = wn;
    }
    return;
  }
  if (bid < ne + nn) {
    const int64_t i = int64_t(bid - ne) * blockDim.x + threadIdx.x;
    if (i >= N) return;
    const float d = G.dinv[i], wn = (d * 1.f) * d;
    G.t_w[G.t_ptr[i + 1] - 1] = wn;
    G.s_w[G.s_ptr[i + 1] - 1] = wn;
    return;
  }
  const int64_t p = int64_t(bid - ne - nn) * blockDim.x + threadIdx.x;
  const int64_t nnz = G.t_ptr[N];   // == s_ptr[N]
  if (G.bnd_t && p < (G.E + N + kPlanGrid - 1) / kPlanGrid) {
    // grouped: every row entry is already final (fill_nodes), read the row of a slot;
    // general: this launch is still placing entries, find the row from the pointers
    G.bnd_t[p] = graph_grouped_t(G) ? plan_bounds_row(G.t_ptr, G.t_row, nnz, p)
                                    : plan_bounds_ptr(G.t_ptr, N, nnz, p);
    G.bnd_s[p] = graph_grouped_s(G) ? plan_bounds_row(G.s_ptr, G.s_row, nnz, p)
                                    : plan_bounds_ptr(G.s_ptr, N, nnz, p);
  }
  if (p >= nnz && p < G.E + N) {
    G.t_row[p] = -1; G.t_col[p] = 0; G.t_w[p] = 0.f;
    G.s_row[p] = -1; G.s_col[p] = 0; G.s_w[p] = 0.f;
  }
}

// block counts of the unweighted steps for E edges and N nodes
__host__ inline int graph_edge_blocks(int64_t E) { return int((E + kGraphThreads - 1) / kGraphThreads); }
__host__ inline int graph_node_blocks(int64_t N) { return int((N + kGraphThreads - 1) / kGraphThreads); }
__host__ inline int graph_pos_blocks(int64_t E, int64_t N) {
  return int((E + N + kGraphThreads - 1) / kGraphThreads);
}

size_t graph_ws_size(int64_t E, int64_t N);
struct GraphArgs {
  const int64_t* ei; const float* ew; int64_t E;
  int32_t *t_ptr, *t_row, *t_col; float* t_w;
  int32_t *s_ptr, *s_row, *s_col; float* s_w;
  int32_t* status; void* ws; size_t ws_bytes;
};
// the GraphBatch of 1-2 graphs without launching anything; zero_bytes[k]: the prefix of
// graph k's workspace (at gb.g[k].cnt_t) that must be zero before the count step
int graph_batch_setup(const GraphArgs* ga, int count, int64_t N, int degree_on, GraphBatch* out,
                      size_t zero_bytes[kMaxGraphs], const int64_t* batch = nullptr);
// GraphArgs of bgcn_build_graph_pair's layout (two workspace halves)
void graph_pair_args(const int64_t* td_ei, int64_t Etd, const int64_t* bu_ei, int64_t Ebu,
                     const bgcn_csr_out* td, const bgcn_csr_out* bu, int32_t* status, void* workspace,
                     size_t workspace_bytes, GraphArgs a[2]);
// carve a graph's workspace (bgcn_graph.hip); zero_bytes = the prefix that must be zero
// before the count step
size_t graph_carve(Carve& c, int64_t E, int64_t N, GraphIO* G, size_t* zero_bytes);

}  // namespace bgcn
