// DropEdge device bodies (bgcn_drop.hip's standalone launches and the fused step's
// batch preparation, bgcn_sparse.hip).  See bgcn_drop.hip for the algorithm.
#pragma once

#include "bgcn_common.h"

namespace bgcn {

constexpr int kDropThreads = 1024;   // standalone launches: one block per tree, big trees bound it
constexpr int kDropMaxWaves = 16;

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

// tree id of edge e (batch[src], clamped to [0, B] so a bad index cannot read or
// write out of bounds; edges of a bad tree id are flagged by k_drop_select)
__device__ __forceinline__ int64_t edge_tree(const int64_t* ei, const int64_t* batch, int64_t N,
                                             int64_t B, int64_t e) {
  int64_t s = ei[e];
  s = s < 0 ? 0 : (s >= N ? N - 1 : s);
  const int64_t t = batch[s];
  return t < 0 ? 0 : (t > B ? B : t);
}

// eptr[d][t] = first edge of tree t in list d (eptr[d][0] = 0, eptr[d][B] = E), from
// the tree boundaries of the list: edge-parallel, one dependent load (no search).
// Edge e = bid * blockDim + thread of list d.
__device__ inline void drop_bounds_body(const DropList& L, int d, const int64_t* __restrict__ batch,
                                        int64_t N, int64_t B, int64_t* __restrict__ eptr,
                                        int32_t* __restrict__ status, int bid) {
  const int64_t e = int64_t(bid) * blockDim.x + threadIdx.x;
  if (e > L.E) return;
  int64_t* ep = eptr + int64_t(d) * (B + 1);
  const int64_t tp = e > 0 ? edge_tree(L.ei, batch, N, B, e - 1) : -1;
  const int64_t tc = e < L.E ? edge_tree(L.ei, batch, N, B, e) : B;
  for (int64_t t = tp + 1; t <= tc; ++t) ep[t] = e;   // trees (tp, tc] start at e
  if (tc < tp && status) atomicOr(status, 1);          // trees out of order
}

// block-wide exclusive scan of 0/1 flags; returns the prefix, *total the sum
__device__ __forceinline__ int block_scan01(bool f, int* wtot, int* total) {
  const int tid = threadIdx.x, lane = tid & (kWave - 1), wv = tid / kWave;
  const int nwv = int(blockDim.x) / kWave;
  const uint64_t m = __ballot(f);
  const int below = __builtin_popcountll(m & ((1ull << lane) - 1ull));
  if (lane == 0) wtot[wv] = __builtin_popcountll(m);
  __syncthreads();
  int pre = 0, tot = 0;
  for (int w = 0; w < nwv; ++w) {
    pre += w < wv ? wtot[w] : 0;
    tot += wtot[w];
  }
  __syncthreads();
  *total = tot;
  return pre + below;
}

// block (t, d) selects and writes tree t of list d (any block size, <= 1024 threads)
__device__ inline void drop_select_body(const DropList& L, int d, int64_t t,
                                        const int64_t* __restrict__ batch, int64_t N, int64_t B,
                                        uint64_t seed, const int64_t* __restrict__ eptr, int32_t masked,
                                        int64_t* __restrict__ counts, int32_t* __restrict__ status) {
  const int64_t* ep = eptr + int64_t(d) * (B + 1);
  const int tid = threadIdx.x, lane = tid & (kWave - 1);
  const int nth = int(blockDim.x), nwv = nth / kWave;
  const auto clampE = [&](int64_t v) { return v < 0 ? int64_t(0) : (v > L.E ? L.E : v); };
  const int64_t e0 = clampE(ep[t]), e1 = clampE(ep[t + 1]);
  const int64_t et = e1 > e0 ? e1 - e0 : 0;
  const int64_t k = kept_count(et, L.rate);

  __shared__ int32_t hist[256];
  __shared__ int64_t sel[3];  // digit, rank among ties, number of ties
  __shared__ int wtot[kDropMaxWaves];
  __shared__ int64_t red[kDropMaxWaves];
  __shared__ int64_t run;

  // compact output offset: kept counts of the trees before t (all trees for the total)
  int64_t off = 0;
  if (!masked) {
    int64_t part = 0, all = 0;
    for (int64_t u = tid; u < B; u += nth) {
      const int64_t a = clampE(ep[u]), b = clampE(ep[u + 1]);
      const int64_t ku = kept_count(b > a ? b - a : 0, L.rate);
      if (u < t) part += ku;
      all += ku;
    }
    for (int o = kWave / 2; o > 0; o >>= 1) {
      part += __shfl_xor(part, o, kWave);
      all += __shfl_xor(all, o, kWave);
    }
    if (lane == 0) red[tid / kWave] = part;
    __syncthreads();
    for (int w = 0; w < nwv; ++w) off += red[w];
    __syncthreads();
    if (lane == 0) red[tid / kWave] = all;
    __syncthreads();
    if (tid == 0 && t == B - 1 && counts) {
      int64_t tot = 0;
      for (int w = 0; w < nwv; ++w) tot += red[w];
      counts[d] = tot;
    }
  }

  // radix select of the (k-1)-th smallest key (0 < k < et only); afterwards the kept
  // set is {h < T} plus the first r+1 (in edge order) of the `ties` edges with h == T
  uint32_t T = 0xffffffffu;
  int64_t r = 0, ties = 1;
  const bool select = k > 0 && k < et;
  if (select) {
    uint32_t prefix = 0, mask = 0;
    r = k - 1;
    for (int shift = 24; shift >= 0; shift -= 8) {
      if (tid < 256) hist[tid] = 0;
      __syncthreads();
      for (int64_t e = e0 + tid; e < e1; e += nth) {
        const uint32_t h = drop_key(seed, L.dir, uint64_t(e));
        if ((h & mask) == prefix) atomicAdd(&hist[(h >> shift) & 255u], 1);
      }
      __syncthreads();
      if (tid < kWave) {   // wave 0: lane l owns bins 4l..4l+3
        int c[4], sum = 0;
#pragma unroll
        for (int j = 0; j < 4; ++j) { c[j] = hist[4 * lane + j]; sum += c[j]; }
        int incl = sum;
        for (int o = 1; o < kWave; o <<= 1) {
          const int v = __shfl_up(incl, o, kWave);
          if (lane >= o) incl += v;
        }
        const uint64_t over = __ballot(int64_t(incl) > r);
        const int hit = __builtin_ctzll(over);   // r < candidates, so some lane crosses
        if (lane == hit) {
          int64_t rr = r - (incl - sum);   // < sum: the crossing bin is one of this lane's
          int j = 0;
          while (j < 3 && rr >= c[j]) { rr -= c[j]; ++j; }
          sel[0] = 4 * lane + j;
          sel[1] = rr;
          sel[2] = c[j];
        }
      }
      __syncthreads();
      prefix |= uint32_t(sel[0]) << shift;
      mask |= 255u << shift;
      r = sel[1];
      ties = sel[2];
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
  bool bad = false;
  int64_t tie_run = 0;   // ties seen in earlier chunks (uniform)
  for (int64_t base = e0; base < e1; base += nth) {
    const int64_t e = base + tid;
    const bool valid = e < e1;
    int64_t sv = 0, dv = 0;
    uint32_t h = 0xffffffffu;
    if (valid) {
      sv = src[e];
      dv = dst[e];
      const bool inb = sv >= 0 && sv < N && dv >= 0 && dv < N;
      bad |= !inb || batch[inb ? sv : 0] != t || batch[inb ? dv : 0] != t;
      if (select) h = drop_key(seed, L.dir, uint64_t(e));
    }
    const bool eq = valid && select && h == T;
    int64_t tie_rank = 0;
    if (ties > 1) {   // rare: rank among equal keys by a block scan (uniform branch)
      int tot;
      tie_rank = tie_run + block_scan01(eq, wtot, &tot);
      tie_run += tot;
    }
    const bool keep = valid && (k == et || (select && (h < T || (eq && tie_rank <= r))));
    int total;
    const int pos = block_scan01(keep, wtot, &total);
    if (masked) {   // the tree's kept edges first, in order; then its dropped ones as loops
      if (valid) {
        const int64_t kept_before = run + pos;
        const int64_t q = keep ? e0 + kept_before : e0 + k + ((e - e0) - kept_before);
        o0[q] = keep ? sv : dv;
        o1[q] = dv;
      }
    } else {
      const int64_t q = off + run + pos;
      if (keep) {
        if (q < L.ld) { o0[q] = sv; o1[q] = dv; } else bad = true;
      }
    }
    __syncthreads();
    if (tid == 0) run += total;
    __syncthreads();
  }
  if (__ballot(bad) && lane == 0 && status) atomicOr(status, 1);
}


}  // namespace bgcn
