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
// and trees ascending (PyG Batch concatenation).  One launch plans the batch (tree edge
// ranges by binary search over batch[src], kept counts, output offsets); one block per
// (tree, list) then finds its tree's k-th smallest key by a 4-pass 8-bit radix select
// over keys recomputed from the hash (no key storage: 4 passes cost 4 hashes per edge,
// not HBM traffic) and writes the kept edges with a block-wide ordered scan.
//
// Two output forms:
//   compact: the kept edges, in order, into [2, ld] (ld >= kept count);
//   masked : [2, E] in place order, each dropped edge (s, d) written as the self loop
//            (d, d).  gcn_norm's add_remaining_self_loops removes input self loops, so
//            the K1 graph of the masked list equals that of the compacted one and the
//            prepared-batch path never needs the kept count on the host.
#include "bgcn_common.h"
#include "bgcn_internal.h"

namespace bgcn {
namespace {

constexpr int kDropThreads = 256;
constexpr int kPlanThreads = 1024;

// splitmix64 finaliser of (seed, dir, e) with a salt that separates it from the
// dropout keep words (keep_word) drawn from the same step seed
__device__ __forceinline__ uint32_t drop_key(uint64_t seed, uint32_t dir, uint64_t e) {
  uint64_t z = (seed ^ 0xD1B54A32D192ED03ull) + 0x9E3779B97F4A7C15ull * (((e << 1) | dir) + 1ull);
  z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ull;
  z = (z ^ (z >> 27)) * 0x94D049BB133111EBull;
  z ^= z >> 31;
  return uint32_t(z >> 32);
}

// int(E_t * (1 - rate)) as Python computes it (double multiply, truncation)
__device__ __forceinline__ int64_t kept_count(int64_t et, double rate) {
  if (!(rate > 0.0)) return et;
  const double v = __dmul_rn(double(et), __dsub_rn(1.0, rate));
  return v <= 0.0 ? 0 : int64_t(v);
}

struct DropList {
  const int64_t* ei;   // [2, E] (row stride E)
  int64_t E;
  int64_t* out;        // [2, ld]
  int64_t ld;
  double rate;
  uint32_t dir;
};

// tree id of edge e (batch[src], clamped so a bad index cannot read out of bounds)
__device__ __forceinline__ int64_t edge_tree(const int64_t* ei, const int64_t* batch, int64_t N,
                                             int64_t e) {
  int64_t s = ei[e];
  s = s < 0 ? 0 : (s >= N ? N - 1 : s);
  return batch[s];
}

// eptr[d][t] = first edge of tree t in list d (eptr[d][0] = 0, eptr[d][B] = E);
// koff[d][t] = exclusive prefix of the kept counts; counts[d] = total kept.
__global__ __launch_bounds__(kPlanThreads) void k_drop_plan(DropList l0, DropList l1,
                                                            const int64_t* __restrict__ batch,
                                                            int64_t N, int64_t B,
                                                            int64_t* __restrict__ eptr,
                                                            int64_t* __restrict__ koff,
                                                            int64_t* __restrict__ counts) {
  const DropList& L = blockIdx.x == 0 ? l0 : l1;
  int64_t* ep = eptr + int64_t(blockIdx.x) * (B + 1);
  int64_t* ko = koff + int64_t(blockIdx.x) * (B + 1);
  __shared__ int64_t wsum[kPlanThreads / kWave];
  __shared__ int64_t carry;
  const int tid = threadIdx.x, lane = tid & (kWave - 1), wv = tid / kWave;
  if (tid == 0) carry = 0;
  // edge ranges first (every block thread binary-searches its trees)
  for (int64_t t = tid; t <= B; t += kPlanThreads) {
    int64_t lo = 0, hi = L.E;
    if (t == 0) hi = 0;
    else if (t == B) lo = L.E;
    while (lo < hi) {
      const int64_t mid = (lo + hi) >> 1;
      if (edge_tree(L.ei, batch, N, mid) < t) lo = mid + 1; else hi = mid;
    }
    ep[t] = lo;
  }
  __syncthreads();
  // kept counts and their exclusive scan, 1024 trees per round
  for (int64_t base = 0; base < B; base += kPlanThreads) {
    const int64_t t = base + tid;
    int64_t k = 0;
    if (t < B) {
      const int64_t et = ep[t + 1] - ep[t];
      k = kept_count(et > 0 ? et : 0, L.rate);
    }
    int64_t incl = k;
    for (int o = 1; o < kWave; o <<= 1) {
      const int64_t v = __shfl_up(incl, o, kWave);
      if (lane >= o) incl += v;
    }
    if (lane == kWave - 1) wsum[wv] = incl;
    __syncthreads();
    int64_t before = carry;
    for (int w = 0; w < wv; ++w) before += wsum[w];
    if (t < B) ko[t] = before + incl - k;
    __syncthreads();
    if (tid == kPlanThreads - 1) carry = before + incl;
    __syncthreads();
  }
  if (tid == 0) {
    ko[B] = carry;
    if (counts) counts[blockIdx.x] = carry;
  }
}

// block-wide exclusive scan of 0/1 flags (4 waves); returns the prefix, *total the sum
__device__ __forceinline__ int block_scan01(bool f, int* wtot, int* total) {
  const int tid = threadIdx.x, lane = tid & (kWave - 1), wv = tid / kWave;
  const uint64_t m = __ballot(f);
  const int below = __builtin_popcountll(m & ((1ull << lane) - 1ull));
  if (lane == 0) wtot[wv] = __builtin_popcountll(m);
  __syncthreads();
  int pre = 0, tot = 0;
#pragma unroll
  for (int w = 0; w < kDropThreads / kWave; ++w) {
    pre += w < wv ? wtot[w] : 0;
    tot += wtot[w];
  }
  __syncthreads();
  *total = tot;
  return pre + below;
}

// grid (B, lists): block (t, d) selects and writes tree t of list d
__global__ __launch_bounds__(kDropThreads) void k_drop_select(DropList l0, DropList l1,
                                                              const int64_t* __restrict__ batch,
                                                              int64_t N, int64_t B, uint64_t seed,
                                                              const int64_t* __restrict__ eptr,
                                                              const int64_t* __restrict__ koff,
                                                              int32_t masked,
                                                              int32_t* __restrict__ status) {
  const DropList& L = blockIdx.y == 0 ? l0 : l1;
  const int64_t t = blockIdx.x;
  const int64_t* ep = eptr + int64_t(blockIdx.y) * (B + 1);
  const int64_t* ko = koff + int64_t(blockIdx.y) * (B + 1);
  const int64_t e0 = ep[t], e1 = ep[t + 1];
  const int64_t et = e1 > e0 ? e1 - e0 : 0;
  const int64_t k = kept_count(et, L.rate);
  const int tid = threadIdx.x, lane = tid & (kWave - 1);

  __shared__ int32_t hist[256];
  __shared__ uint32_t sel[2];  // threshold key, rank among ties
  __shared__ int wtot[kDropThreads / kWave];
  __shared__ int64_t run;

  // radix select of the (k-1)-th smallest key (0 < k < et only)
  uint32_t T = 0xffffffffu;
  int64_t r = 0;
  const bool select = k > 0 && k < et;
  if (select) {
    uint32_t prefix = 0, mask = 0;
    r = k - 1;
    for (int shift = 24; shift >= 0; shift -= 8) {
      hist[tid] = 0;
      __syncthreads();
      for (int64_t e = e0 + tid; e < e1; e += kDropThreads) {
        const uint32_t h = drop_key(seed, L.dir, uint64_t(e));
        if ((h & mask) == prefix) atomicAdd(&hist[(h >> shift) & 255u], 1);
      }
      __syncthreads();
      if (tid < kWave) {   // wave 0: lane l owns bins 4l..4l+3
        int c[4], s = 0;
#pragma unroll
        for (int j = 0; j < 4; ++j) { c[j] = hist[4 * lane + j]; s += c[j]; }
        int incl = s;
        for (int o = 1; o < kWave; o <<= 1) {
          const int v = __shfl_up(incl, o, kWave);
          if (lane >= o) incl += v;
        }
        const uint64_t over = __ballot(int64_t(incl) > r);
        const int hit = __builtin_ctzll(over);   // r < total, so some lane crosses
        if (lane == hit) {
          int64_t rr = r - (incl - s);   // < s: the crossing bin is one of this lane's
          int j = 0;
          while (j < 3 && rr >= c[j]) { rr -= c[j]; ++j; }
          sel[0] = uint32_t(4 * lane + j);
          sel[1] = uint32_t(rr);
        }
      }
      __syncthreads();
      prefix |= sel[0] << shift;
      mask |= 255u << shift;
      r = sel[1];
      __syncthreads();
    }
    T = prefix;
  }

  if (tid == 0) run = 0;
  __syncthreads();
  const int64_t* src = L.ei;
  const int64_t* dst = L.ei + L.E;
  int64_t* o0 = L.out;
  int64_t* o1 = L.out + L.ld;
  bool bad = e1 < e0;   // trees out of order: some edges are in no tree's range
  for (int64_t base = e0; base < e1; base += kDropThreads) {
    const int64_t e = base + tid;
    const bool valid = e < e1;
    bool keep = false;
    int64_t s = 0, d = 0;
    if (valid) {
      s = src[e];
      d = dst[e];
      const bool inb = s >= 0 && s < N && d >= 0 && d < N;
      bad |= !inb || batch[inb ? s : 0] != t || batch[inb ? d : 0] != t;
      if (k == et) {
        keep = true;
      } else if (select) {
        const uint32_t h = drop_key(seed, L.dir, uint64_t(e));
        if (h < T) {
          keep = true;
        } else if (h == T) {   // ties in edge order (rare): rank among equal keys
          int64_t eq = 0;
          for (int64_t j = e0; j < e; ++j) eq += drop_key(seed, L.dir, uint64_t(j)) == T;
          keep = eq <= r;
        }
      }
    }
    if (masked) {
      if (valid) {
        o0[e] = keep ? s : d;
        o1[e] = d;
      }
    } else {
      int total;
      const int pos = block_scan01(keep, wtot, &total);
      const int64_t q = ko[t] + run + pos;
      if (keep) {
        if (q < L.ld) { o0[q] = s; o1[q] = d; } else bad = true;
      }
      __syncthreads();
      if (tid == 0) run += total;
      __syncthreads();
    }
  }
  if (__ballot(bad) && lane == 0 && status) atomicOr(status, 1);
}

}  // namespace

size_t drop_ws_size(int64_t B) {
  Carve c(nullptr, 0);
  c.take<int64_t>(size_t(2 * (B + 1)));
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
  Carve c(ws, ws_bytes);
  int64_t* eptr = c.take<int64_t>(size_t(2 * (B + 1)));
  int64_t* koff = c.take<int64_t>(size_t(2 * (B + 1)));
  // an absent list is planned as an empty one (its counts come out 0)
  DropList l0{td, td ? Etd : 0, td_out, ld_td, td_rate, 0u};
  DropList l1{bu, bu ? Ebu : 0, bu_out, ld_bu, bu_rate, 1u};
  if (!td) l0.ei = bu ? bu : td;
  if (!bu) l1.ei = l0.ei;
  if (!l0.ei) return BGCN_OK;  // nothing to do
  hipLaunchKernelGGL(k_drop_plan, dim3(2), dim3(kPlanThreads), 0, s, l0, l1, batch, N, B, eptr,
                     koff, counts);
  BGCN_CHECK_LAUNCH();
  const int lists = bu ? 2 : 1;
  if (!td) {  // BU only: run it as list 0 of the launch
    hipLaunchKernelGGL(k_drop_select, dim3(unsigned(B), 1), dim3(kDropThreads), 0, s, l1, l1, batch,
                       N, B, seed, eptr + (B + 1), koff + (B + 1), masked, status);
  } else {
    hipLaunchKernelGGL(k_drop_select, dim3(unsigned(B), unsigned(lists)), dim3(kDropThreads), 0, s,
                       l0, l1, batch, N, B, seed, eptr, koff, masked, status);
  }
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
