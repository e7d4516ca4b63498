// DropEdge on the device: the per-tree edge subsampling the reference runs in its
// DataLoader workers (Process/dataset.py:68-90, BiGraphDataset.__getitem__):
//
//   poslist = sorted(random.sample(range(E_t), int(E_t * (1 - droprate))))
//   edges   = edges[poslist]                         (only when droprate > 0)
//
// for every tree t of a collated batch, independently per direction (TD with
// tddroprate over [parent, child]; BU with budroprate over the flipped list).  The
// build keeps the distribution - a uniform random subset of exactly
// int(E_t * (1 - rate)) edges (the count computed in double, as Python does), in the
// original order - and replaces Python's Mersenne Twister with a counter-based key:
// edge e of the list gets the 32-bit key drop_key(seed, dir, e) and the k smallest
// (key, e) pairs of its tree are kept.  With keys i.i.d. uniform that is a uniform
// k-subset; the selection is a deterministic function of (seed, dir, list), restated
// bit for bit by the oracle (oracle/bigcn_oracle.py drop_edges).
//
// Layout: the list is [2, E] int64 in collation order, every tree's edges contiguous
// and trees ascending (PyG Batch concatenation).  k_drop_bounds finds every tree's edge
// range from the tree boundaries of the list (edge-parallel, no search); one block per
// (tree, list) then finds its tree's k-th smallest key by a 4-pass 8-bit radix select
// over keys recomputed from the hash (no key storage: 4 passes cost 4 hashes per edge,
// not HBM traffic) and writes the kept edges (compact form: block-wide ordered scan
// after the kept counts of the preceding trees).
//
// Two output forms:
//   compact: the kept edges, in order, into [2, ld] (ld >= kept count);
//   masked : [2, E]; within each tree's range its kept edges first (in order), then
//            every dropped edge (s, d) as the self loop (d, d).  gcn_norm's
//            add_remaining_self_loops removes input self loops, so the K1 graph of the
//            masked list equals that of the compacted one (unweighted), the prepared-batch
//            path never needs the kept count on the host, and K1's run-based placement
//            stays valid (no loop inside a node's run of edges).
#include "bgcn_drop_body.h"
#include "bgcn_internal.h"

namespace bgcn {
namespace {

// standalone launches (bgcn_drop_edges): 1024-thread blocks, blockIdx.y = list
__global__ __launch_bounds__(kDropThreads) void k_drop_bounds(DropList l0, DropList l1,
                                                              const int64_t* __restrict__ batch,
                                                              int64_t N, int64_t B,
                                                              int64_t* __restrict__ eptr,
                                                              int32_t* __restrict__ status) {
  drop_bounds_body(blockIdx.y == 0 ? l0 : l1, int(blockIdx.y), batch, N, B, eptr, status, int(blockIdx.x));
}

__global__ __launch_bounds__(kDropThreads) void k_drop_select(DropList l0, DropList l1,
                                                              const int64_t* __restrict__ batch,
                                                              int64_t N, int64_t B, uint64_t seed,
                                                              const int64_t* __restrict__ eptr,
                                                              int32_t masked,
                                                              int64_t* __restrict__ counts,
                                                              int32_t* __restrict__ status) {
  drop_select_body(blockIdx.y == 0 ? l0 : l1, int(blockIdx.y), int64_t(blockIdx.x), batch, N, B, seed,
                   eptr, masked, counts, status);
}

}  // namespace

size_t drop_ws_size(int64_t B) {
  Carve c(nullptr, 0);
  c.take<int64_t>(size_t(2 * (B + 1)));
  return c.off + 256;
}

int drop_edges_impl(const int64_t* td, int64_t Etd, int64_t* td_out, int64_t ld_td, double td_rate,
                    const int64_t* bu, int64_t Ebu, int64_t* bu_out, int64_t ld_bu, double bu_rate,
                    const int64_t* batch, int64_t N, int64_t B, uint64_t seed, int masked,
                    int64_t* counts, int32_t* status, void* ws, size_t ws_bytes, hipStream_t s) {
  BGCN_CHECK_ARG(N >= 1 && B >= 1 && Etd >= 0 && Ebu >= 0, "bad sizes");
  BGCN_CHECK_ARG(batch, "null batch");
  BGCN_CHECK_ARG(!td || (td_out && (Etd == 0 || ld_td >= 1)), "bad TD list / output");
  BGCN_CHECK_ARG(!bu || (bu_out && (Ebu == 0 || ld_bu >= 1)), "bad BU list / output");
  BGCN_CHECK_ARG(!masked || ((!td || ld_td >= Etd) && (!bu || ld_bu >= Ebu)),
                 "masked output needs ld >= E");
  BGCN_CHECK_ARG(td_rate < 1.0 && bu_rate < 1.0, "droprate must be < 1");
  BGCN_CHECK_ARG(ws && ws_bytes >= drop_ws_size(B), "workspace too small");
  if (counts) BGCN_CHECK_HIP(hipMemsetAsync(counts, 0, 2 * sizeof(int64_t), s));
  if (!td && !bu) return BGCN_OK;
  Carve c(ws, ws_bytes);
  int64_t* eptr = c.take<int64_t>(size_t(2 * (B + 1)));
  // the lists actually present, packed first; their counts land in counts[0] / [1]
  DropList l[2];
  int lists = 0;
  int64_t* cnt[2] = {counts, counts ? counts + 1 : nullptr};
  int slot[2];
  if (td) { l[lists] = DropList{td, Etd, td_out, ld_td, td_rate, 0u}; slot[lists++] = 0; }
  if (bu) { l[lists] = DropList{bu, Ebu, bu_out, ld_bu, bu_rate, 1u}; slot[lists++] = 1; }
  if (lists == 1) l[1] = l[0];
  const int64_t Emax = std::max(l[0].E, l[1].E);
  hipLaunchKernelGGL(k_drop_bounds, dim3(unsigned((Emax + kDropThreads) / kDropThreads), unsigned(lists)),
                     dim3(kDropThreads), 0, s, l[0], l[1], batch, N, B, eptr, status);
  BGCN_CHECK_LAUNCH();
  // counts are written per list index; map a lone BU list onto counts[1]
  int64_t* cbase = (lists == 1 && slot[0] == 1) ? cnt[1] : cnt[0];
  hipLaunchKernelGGL(k_drop_select, dim3(unsigned(B), unsigned(lists)), dim3(kDropThreads), 0, s,
                     l[0], l[1], batch, N, B, seed, eptr, masked, cbase, status);
  BGCN_CHECK_LAUNCH();
  return BGCN_OK;
}

}  // namespace bgcn

extern "C" size_t bgcn_drop_edges_workspace_size(int64_t num_graphs) {
  return bgcn::drop_ws_size(num_graphs);
}

extern "C" int bgcn_drop_edges(const int64_t* td_edge_index, int64_t td_num_edges, double td_droprate,
                               int64_t* td_out, int64_t ld_td_out, const int64_t* bu_edge_index,
                               int64_t bu_num_edges, double bu_droprate, int64_t* bu_out,
                               int64_t ld_bu_out, const int64_t* batch, int64_t num_nodes,
                               int64_t num_graphs, uint64_t seed, int32_t masked, int64_t* counts,
                               int32_t* status, void* workspace, size_t workspace_bytes,
                               bgcn_stream_t stream) {
  return bgcn::drop_edges_impl(td_edge_index, td_num_edges, td_out, ld_td_out, td_droprate,
                               bu_edge_index, bu_num_edges, bu_out, ld_bu_out, bu_droprate, batch,
                               num_nodes, num_graphs, seed, masked, counts, status, workspace,
                               workspace_bytes, reinterpret_cast<hipStream_t>(stream));
}
