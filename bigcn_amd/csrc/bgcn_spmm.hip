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
// Narrow kernel (F = 64 / 128): a group = F/4 lanes, one float4 per lane; the
// chunk's (row, col, w) triples are loaded once (one entry per lane) and broadcast
// with cross-lane shuffles; 8 neighbour rows are in flight per group.
// Wide kernel (F > 128, e.g. the 5000-dim standalone aggregation): a group = one wave
// per (chunk, 256-float column slice).
// Up to two problems (the fused step's TD and BU graphs) share one launch
// (blockIdx.y / blockIdx.z = problem).
#include "bgcn_internal.h"
#include "bgcn_trace.h"

namespace bgcn {

namespace {

constexpr int NPG = 16;  // CSR entries per lane group
static_assert(NPG == kPlanChunk, "K1's plans use the narrow kernel's chunk grid");

__device__ __forceinline__ float4 epilogue(float4 acc, float4 bias, int epi) {
  float4 o = f4add(acc, bias);
  return (epi & BGCN_EPI_RELU) ? f4relu(o) : o;
}

// Partial record per (group, slot): slot 0 = head row (started before the chunk),
// slot 1 = tail row (started inside the chunk, ends after it).
template <int LANES>
__global__ __launch_bounds__(256) void k_spmm_narrow(SpmmBatch sb) {
  static_assert(LANES >= NPG, "one entry per lane");
  const SpmmProb& P = sb.p[blockIdx.y];
  constexpr int GPB = 256 / LANES;  // groups per block
  const int lane = threadIdx.x % LANES;
  const int64_t g = int64_t(blockIdx.x) * GPB + threadIdx.x / LANES;
  if (g >= P.ngroups) return;
  const int64_t cap = P.capacity;
  const int64_t p0 = g * NPG;
  const int64_t p1 = min<int64_t>(p0 + NPG, cap);
  const int fo = lane * 4;
  const float4 bv = P.bias ? ld4(P.bias + fo) : f4zero();

  // entry k of the chunk lives in lane k of the group.  Whether the first row started
  // before the chunk / the last row runs past it is read off the neighbouring entries
  // (row[p0-1], row[p1]) - loaded alongside the chunk, so no dependent loads: entries
  // past the valid count carry row -1 (K1), so the count itself is never read.
  const bool mine = lane < NPG && p0 + lane < cap;
  const int64_t pl = min<int64_t>(p0 + lane, cap - 1);   // clamped, unconditional
  const int32_t r_ld = P.row[pl], c_ld = P.col[pl];
  const float w_ld = P.w[pl];
  const int32_t r_l = mine ? r_ld : -1;
  const int32_t c_l = mine ? c_ld : 0;
  const float w_l = mine ? w_ld : 0.f;
  const int32_t prev_ld = P.row[p0 > 0 ? p0 - 1 : 0], next_ld = P.row[min<int64_t>(p1, cap - 1)];
  const int32_t prev_row = p0 > 0 ? prev_ld : -1;
  const int32_t next_row = p1 < cap ? next_ld : -1;
  const int n = int(p1 - p0);
  const int base_lane = ((threadIdx.x & 63) / LANES) * LANES;  // group's first lane in the wave

  float4 acc = f4zero();
  int32_t cur = -1;
  bool cur_head = false;  // cur started before p0
  for (int k0 = 0; k0 < n; k0 += 8) {
    float4 v[8];
    int32_t rr[8];
    float ww[8];
#pragma unroll
    for (int u = 0; u < 8; ++u) {
      const int src = base_lane + k0 + u;  // k0 + u < NPG <= LANES
      const int32_t rk = __shfl(r_l, src, 64);
      const int32_t ck = __shfl(c_l, src, 64);
      ww[u] = __shfl(w_l, src, 64);
      rr[u] = rk;
      // unconditional gather (ck = 0 for padding entries): a guarded load would compile
      // to a branch with its own wait and serialise the eight loads
      const float4 t = ld4(P.in + int64_t(ck) * P.ld_in + fo);
      v[u] = rk >= 0 ? t : f4zero();
    }
#pragma unroll
    for (int u = 0; u < 8; ++u) {
      const int32_t r = rr[u];
      if (r < 0) break;
      if (r != cur) {
        if (cur >= 0) {
          // `cur` ended inside this chunk (a later entry belongs to another row)
          if (!cur_head) st4_chain(P.out, int64_t(cur) * P.ld_out + fo, epilogue(acc, bv, sb.epi));
          else st4(P.part + (g * 2 + 0) * (LANES * 4) + fo, acc);
        }
        cur_head = cur < 0 && r == prev_row;
        cur = r;
        acc = f4zero();
      }
      acc = f4fma(ww[u], v[u], acc);
    }
  }
  if (cur >= 0) {
    const bool ends = next_row != cur;
    if (!cur_head && ends) st4_chain(P.out, int64_t(cur) * P.ld_out + fo, epilogue(acc, bv, sb.epi));
    else if (cur_head) st4(P.part + (g * 2 + 0) * (LANES * 4) + fo, acc);  // head (may also extend past p1)
    else st4(P.part + (g * 2 + 1) * (LANES * 4) + fo, acc);               // tail
  }
}

// Planned narrow aggregation (F = 64, the fused step): with K1's SpmmPlan no row is split,
// so no fixup launch follows.  Blocks [0, nchunk) hold 64 groups of 16 lanes; group g
// aggregates chunk g's complete short rows [bnd.x, bnd.y) (<= 31 entries, two per lane,
// broadcast by shuffles, 8 gathers in flight).  Blocks [nchunk, nchunk + nlongblk) take
// the long rows longs[j], j = block, block + nlongblk, ...: the 64 groups sum entries
// q, q + 64, ... of the row (8 in flight) and combine their partials in LDS in group
// order (deterministic; a row's sum does not depend on which block takes it).
#ifndef BGCN_ROWS_THREADS
#define BGCN_ROWS_THREADS 512   // 1024-thread blocks ran one per CU (block trace)
#endif
constexpr int kRowsThreads = BGCN_ROWS_THREADS;
#ifndef BGCN_ROWS_WPE
#define BGCN_ROWS_WPE 1   // minimum waves per SIMD the compiler budgets registers for (A/B knob)
#endif
constexpr int64_t kPlanMaxEntries = int64_t(1) << 30;   // capacity (E + N) up to which plans are used
constexpr int kRowsGroups = kRowsThreads / 16;

// kSign (SpmmBatch::sg): the input rows are the readout's dH2, generated from the H2 sign
// words of the gathered rows (8 bytes per neighbour instead of a 256-byte row) and scaled
// per output row by its tree's dhead / count (the rows of one chunk mostly share one or two
// trees: the first and the last entry's tree scales are loaded with the entries).
__device__ __forceinline__ float4 sign_bits(uint64_t wd, int lane) {
  return make_float4(float((wd >> lane) & 1ull), float((wd >> (16 + lane)) & 1ull),
                     float((wd >> (32 + lane)) & 1ull), float((wd >> (48 + lane)) & 1ull));
}
__device__ __forceinline__ float4 tree_scale(const SpmmSign& sg, int64_t b, int hoff, int fo) {
  b = min<int64_t>(max<int64_t>(b, 0), sg.B - 1);   // ids out of range: status bit (K1 / head)
  const float cnt = float(max(sg.tree_ptr[b + 1] - sg.tree_ptr[b], 1));
  const float4 dh = ld4(sg.dhead + b * kHeadIn + hoff + fo);
  return make_float4(dh.x / cnt, dh.y / cnt, dh.z / cnt, dh.w / cnt);
}

#ifndef BGCN_SIGN_XT
#define BGCN_SIGN_XT 1   // A/B only: 0 drops the cross-tree check (wrong for edges across trees)
#endif
// kXt (kSign with an edge across trees: the graph build's BGCN_STATUS_CROSS_TREE, never set
// by PyG collation): every gathered row is scaled by its own tree, the output row not.  The
// kernel branches on the status word once per block into separate instantiations: a
// run-time test inside the gather loop made the compiler wait for each gather before the
// next (the sign-word aggregation ran 1.3-1.8x the plain one's time)
template <bool kSign, bool kXt>
__device__ __forceinline__ void rows_chunk(const SpmmBatch& sb, const SpmmProb& P, int64_t g, int hoff,
                                           const uint64_t* __restrict__ sgn) {
  constexpr int LANES = 16;
  const int lane = threadIdx.x % LANES;
  const int fo = lane * 4;
  const int base_lane = ((threadIdx.x & 63) / LANES) * LANES;
  const int2 bd = P.plan.bnd[g];
  const int n = bd.y - bd.x;                       // <= 2 * LANES - 1; <= 0: no rows
  if (n <= 0) return;
  const float4 bv = P.bias ? ld4(P.bias + fo) : f4zero();
  // entries bd.x + lane and bd.x + 16 + lane (clamped, unconditional; masked by n)
  const int64_t e0 = min<int64_t>(bd.x + lane, P.capacity - 1);
  const int64_t e1 = min<int64_t>(bd.x + LANES + lane, P.capacity - 1);
  const int32_t r0 = P.row[e0], c0 = P.col[e0], r1 = P.row[e1], c1 = P.col[e1];
  const float w0 = P.w[e0], w1 = P.w[e1];
  // kSign: the trees of the chunk's first and last rows and their scales
  int32_t bA = 0, bZ = 0;   // tree ids (< B)
  float4 gA = f4zero(), gZ = f4zero();
  // kSign: the tree of each entry's row, loaded with the entries (a row's tree is then at
  // hand when the row finishes - no dependent load per row)
  int32_t bb0 = 0, bb1 = 0;
  if constexpr (kSign && !kXt) {
    bb0 = int32_t(sb.sg.batch[max(r0, 0)]);
    bb1 = int32_t(sb.sg.batch[max(r1, 0)]);
    bA = __shfl(bb0, base_lane, 64);
    bZ = __shfl(n > LANES ? bb1 : bb0, base_lane + ((n - 1) & (LANES - 1)), 64);
    gA = tree_scale(sb.sg, bA, hoff, fo);
    gZ = tree_scale(sb.sg, bZ, hoff, fo);
  }
  auto finish = [&](int32_t r, float4 acc, int32_t b) {
    if constexpr (kSign && kXt) {
      st4_chain(P.out, int64_t(r) * P.ld_out + fo, acc);
    } else if constexpr (kSign) {
      const float4 gs = b == bA ? gA : (b == bZ ? gZ : tree_scale(sb.sg, b, hoff, fo));
      st4_chain(P.out, int64_t(r) * P.ld_out + fo,
          make_float4(acc.x * gs.x, acc.y * gs.y, acc.z * gs.z, acc.w * gs.w));
    } else {
      st4_chain(P.out, int64_t(r) * P.ld_out + fo, epilogue(acc, bv, sb.epi));
    }
  };
  float4 acc = f4zero();
  int32_t cur = -1;
  int32_t curb = 0;
  if constexpr (kXt) {   // rare (no PyG batch has it): one entry at a time, few registers
    for (int k = 0; k < n; ++k) {
      const int src = base_lane + (k & (LANES - 1));
      const bool hi = k >= LANES;
      const int32_t r = __shfl(hi ? r1 : r0, src, 64);
      const int32_t ck = __shfl(hi ? c1 : c0, src, 64);
      const float w = __shfl(hi ? w1 : w0, src, 64);
      const float4 v = f4mul(sign_bits(sgn[int64_t(ck) * 2], lane), tree_scale(sb.sg, sb.sg.batch[ck], hoff, fo));
      if (r != cur) {
        if (cur >= 0) finish(cur, acc, 0);
        cur = r;
        acc = f4zero();
      }
      acc = f4fma(w, v, acc);
    }
    if (cur >= 0) finish(cur, acc, 0);
    return;
  }
  for (int k0 = 0; k0 < n; k0 += 8) {
    float4 v[8];
    int32_t rr[8];
    int32_t bk[8];
    float ww[8];
#pragma unroll
    for (int u = 0; u < 8; ++u) {
      const int k = k0 + u;                        // < 32
      const int src = base_lane + (k & (LANES - 1));
      const bool hi = k >= LANES;                  // uniform
      const int32_t rk = __shfl(hi ? r1 : r0, src, 64);
      const int32_t ck = __shfl(hi ? c1 : c0, src, 64);
      ww[u] = __shfl(hi ? w1 : w0, src, 64);
      if constexpr (kSign && !kXt) bk[u] = __shfl(hi ? bb1 : bb0, src, 64);
      else bk[u] = 0;
      rr[u] = k < n ? rk : -1;
      if constexpr (kSign)
        v[u] = sign_bits(sgn[int64_t(ck) * 2], lane);    // unconditional (ck is a real row)
      else
        v[u] = ld4(P.in + int64_t(ck) * P.ld_in + fo);   // unconditional (ck is a real row)
    }
#pragma unroll
    for (int u = 0; u < 8; ++u) {
      const int32_t r = rr[u];
      if (r < 0) break;
      if (r != cur) {
        if (cur >= 0) finish(cur, acc, curb);
        cur = r;
        curb = bk[u];
        acc = f4zero();
      }
      acc = f4fma(ww[u], v[u], acc);
    }
  }
  if (cur >= 0) finish(cur, acc, curb);
}

// long rows: one block per row (the 32 groups of 16 lanes sum entries q, q + 32, ... and
// combine their partials in LDS in group order)
template <bool kSign, bool kXt>
__device__ __forceinline__ void rows_long(const SpmmBatch& sb, const SpmmProb& P, int64_t nchunk, int nlongblk,
                                          int hoff, const uint64_t* __restrict__ sgn,
                                          float4 (*red)[16]) {
  constexpr int LANES = 16;
  const int lane = threadIdx.x % LANES, grp = threadIdx.x / LANES;
  const int fo = lane * 4;
  const int nl = *P.plan.nlong;
  for (int j = int(blockIdx.x - nchunk); j < nl; j += nlongblk) {
    const int32_t r = P.plan.longs[j];
    const int64_t rs = P.ptr[r], re = P.ptr[r + 1];
    float4 gs = f4zero();
    if constexpr (kSign) gs = kXt ? make_float4(1.f, 1.f, 1.f, 1.f) : tree_scale(sb.sg, sb.sg.batch[r], hoff, fo);
    float4 acc = f4zero();
    int64_t e = rs + grp;
    for (; !kXt && e + 7 * kRowsGroups < re; e += 8 * kRowsGroups) {
      float4 v[8];
      float ww[8];
#pragma unroll
      for (int u = 0; u < 8; ++u) {
        const int64_t eu = e + u * kRowsGroups;
        ww[u] = P.w[eu];
        if constexpr (kSign)
          v[u] = sign_bits(sgn[int64_t(P.col[eu]) * 2], lane);
        else
          v[u] = ld4(P.in + int64_t(P.col[eu]) * P.ld_in + fo);
      }
#pragma unroll
      for (int u = 0; u < 8; ++u) acc = f4fma(ww[u], v[u], acc);
    }
    for (; e < re; e += kRowsGroups) {
      if constexpr (kSign) {
        float4 v = sign_bits(sgn[int64_t(P.col[e]) * 2], lane);
        if constexpr (kXt) v = f4mul(v, tree_scale(sb.sg, sb.sg.batch[P.col[e]], hoff, fo));
        acc = f4fma(P.w[e], v, acc);
      } else
        acc = f4fma(P.w[e], ld4(P.in + int64_t(P.col[e]) * P.ld_in + fo), acc);
    }
    red[grp][lane] = acc;
    __syncthreads();
    if (grp == 0) {
      float4 t = red[0][lane];
#pragma unroll 8
      for (int q = 1; q < kRowsGroups; ++q) t = f4add(t, red[q][lane]);
      if constexpr (kSign) {
        st4_chain(P.out, int64_t(r) * P.ld_out + fo, make_float4(t.x * gs.x, t.y * gs.y, t.z * gs.z, t.w * gs.w));
      } else {
        const float4 bv = P.bias ? ld4(P.bias + fo) : f4zero();
        st4_chain(P.out, int64_t(r) * P.ld_out + fo, epilogue(t, bv, sb.epi));
      }
    }
    __syncthreads();
  }
}

template <bool kSign>
__global__ __launch_bounds__(kRowsThreads) __attribute__((amdgpu_waves_per_eu(BGCN_ROWS_WPE))) void k_spmm_rows(SpmmBatch sb, int64_t nchunk, int nlongblk) {
  BT_BEGIN
  const SpmmProb& P = sb.p[blockIdx.y];
  const int hoff = blockIdx.y == 0 ? kHeadIn / 2 : 0;   // kSign: TD's r1 block sits after BU's
  const uint64_t* sgn = sb.sg.sgn + blockIdx.y;      // kSign: this problem's word of row j
  __shared__ float4 red[kRowsGroups][16];
  const bool xt = kSign && BGCN_SIGN_XT && (*sb.sg.tree_status[blockIdx.y] & BGCN_STATUS_CROSS_TREE) != 0;
  if (int64_t(blockIdx.x) < nchunk) {
    // XCD-contiguous chunk ranges: a tree's rows and the neighbours they gather stay in one
    // L2 (the launch pads gridDim.x to a multiple of 8)
    const int64_t g = int64_t(xcd_contig(int(blockIdx.x), int(nchunk))) * kRowsGroups + threadIdx.x / 16;
    if (g >= (P.capacity + kPlanGrid - 1) / kPlanGrid) return;
    if (xt) rows_chunk<kSign, true>(sb, P, g, hoff, sgn);
    else rows_chunk<kSign, false>(sb, P, g, hoff, sgn);
    BT_END(3);
    return;
  }
  if (xt) rows_long<kSign, true>(sb, P, nchunk, nlongblk, hoff, sgn, red);
  else rows_long<kSign, false>(sb, P, nchunk, nlongblk, hoff, sgn, red);
  if (*P.plan.nlong > int(blockIdx.x - nchunk)) BT_END(4);
}

// Fixup, F <= 128: one block per SG = 256/LANES chunk boundaries, sub-group s checking
// boundary blockIdx.x*SG + s + 1.  A row that crosses it and ends in that chunk gets its
// partials tail[g0], head[g0+1..g1] summed in chunk order and is written: by the
// sub-group itself when it has <= kSmall pieces (TD rows, most BU rows), by the whole
// block otherwise (a BU star root spans hundreds of chunks: sub-group q takes items
// q, q+SG, ..., combined in a fixed order).  Deterministic; one row's sum is the same
// either way.
template <int LANES>
__global__ __launch_bounds__(256) void k_spmm_fixup_narrow(SpmmBatch sb) {
  constexpr int SG = 256 / LANES;
  constexpr int kSmall = 8;                  // pieces a sub-group sums on its own
  __shared__ float4 red[SG][LANES];
  __shared__ int32_t big[SG];                // rows of > kSmall pieces found by sub-group s
  const SpmmProb& P = sb.p[blockIdx.y];
  const int s = threadIdx.x / LANES, fo = (threadIdx.x % LANES) * 4;
  const float4 bv = P.bias ? ld4(P.bias + fo) : f4zero();
  auto item = [&](int64_t g0, int64_t j) {   // item 0 = tail[g0], item j = head[g0 + j]
    return ld4(P.part + ((g0 + j) * 2 + (j == 0 ? 1 : 0)) * (LANES * 4) + fo);
  };
  // sub-group s checks boundary g = blockIdx.x * SG + s + 1
  const int64_t g = int64_t(blockIdx.x) * SG + s + 1;
  int32_t mine = -1;
  if (g < P.ngroups) {
    const int64_t pb = g * NPG;              // < capacity (g < ngroups)
    const int32_t r = P.row[pb], rp = P.row[pb - 1];
    if (r >= 0 && rp == r) {                 // a row crossing the boundary ...
      const int64_t rs = P.ptr[r], re = P.ptr[r + 1];
      const int64_t g0 = rs / NPG, g1 = (re - 1) / NPG;
      if (g1 == g) {                         // ... whose last piece is chunk g
        const int64_t m = g1 - g0 + 1;
        if (m <= kSmall) {                   // sequential sum, all loads in flight
          float4 v[kSmall];
#pragma unroll
          for (int j = 0; j < kSmall; ++j) v[j] = item(g0, j < m ? j : 0);
          float4 acc = v[0];
#pragma unroll
          for (int j = 1; j < kSmall; ++j)
            if (j < m) acc = f4add(acc, v[j]);
          st4_chain(P.out, int64_t(r) * P.ld_out + fo, epilogue(acc, bv, sb.epi));
        } else {
          mine = r;
        }
      }
    }
  }
  if (fo == 0) big[s] = mine;
  __syncthreads();
  // rows of many pieces (BU star roots): the whole block, sub-group q takes items
  // q, q+SG, ..., combined in a fixed order (deterministic)
  for (int t = 0; t < SG; ++t) {
    const int32_t r = big[t];
    if (r < 0) continue;                     // uniform
    const int64_t rs = P.ptr[r], re = P.ptr[r + 1];
    const int64_t g0 = rs / NPG, g1 = (re - 1) / NPG;
    const int64_t m = g1 - g0 + 1;
    float4 acc = f4zero();
    int64_t j = s;
    for (; j + 3 * SG < m; j += 4 * SG) {
      float4 v[4];
#pragma unroll
      for (int u = 0; u < 4; ++u) v[u] = item(g0, j + u * SG);
#pragma unroll
      for (int u = 0; u < 4; ++u) acc = f4add(acc, v[u]);
    }
    for (; j < m; j += SG) acc = f4add(acc, item(g0, j));
    red[s][threadIdx.x % LANES] = acc;
    __syncthreads();
    if (s == 0) {
      float4 sum = red[0][threadIdx.x];
#pragma unroll
      for (int q = 1; q < SG; ++q) sum = f4add(sum, red[q][threadIdx.x]);
      st4_chain(P.out, int64_t(r) * P.ld_out + fo, epilogue(sum, bv, sb.epi));
    }
    __syncthreads();
  }
}

// Wide aggregation (F > 128, e.g. the 5000-dim A_hat . X).  HBM-bound: every X row is
// needed by its own output row and by its neighbours' (parent / children); the output is
// written once.  Chunks of NPGW entries (merge path as above) are row-aligned for rows of
// <= NPGW entries (the nominal boundary g * NPGW moves back to the start of the row it
// falls in), so only long rows (BU star roots) leave partial rows for the fixup pass.
#ifndef BGCN_NPGW
#define BGCN_NPGW 16
#endif
constexpr int NPGW = BGCN_NPGW;
constexpr int kWideSlice = 1024;   // fixup slice (floats)
constexpr int kWaveBlock = 256;    // 4 waves per block

// first entry of chunk g: g*NPGW, or the start of the row containing it when that row
// is short (<= NPGW entries, never split)
__device__ __forceinline__ int64_t wide_chunk_start(const SpmmProb& P, int64_t g, int64_t nnz) {
  const int64_t p = g * NPGW;
  if (p >= nnz) return nnz;
  const int32_t r = P.row[p];
  const int64_t rs = P.ptr[r], re = P.ptr[r + 1];
  return re - rs <= NPGW ? rs : p;
}


// Slice kernel: one short-lived wave per (chunk, 256-float column slice), one float4 per
// lane.  Measured on MI355X (tools/copy_probe.hip, profiles/r01_agg_variants.txt):
// HBM streams fastest when the work is cut into small units that the dispatcher hands
// out in address order, so the bytes in flight form ONE compact moving window (a copy of
// 1 KB per wave: 6.3-6.5 TB/s) - not when each wave or block sweeps its own run of rows
// (8 rows per wave: 4.8-4.9 TB/s; a block-per-CU sweep and a wave-per-row-slice sweep of
// this aggregation ran at 4.6-4.9 TB/s, this kernel at 5.0-5.4).  Waves
// u = g*S + s, so the S slices of chunk g run side by side and read its rows whole.
//   * the chunk's entries sit one per lane (plus the entries just before / after it) and
//     are broadcast with readlane, so row changes, source rows and weights are
//     wave-uniform; every X / output row is addressed through a buffer descriptor
//     (scalar base, hardware range check at F);
//   * 16 source slices in flight per wave: entries are loaded in groups of 8, two
//     groups ahead; loads of padding entries go through a zero-size buffer descriptor
//     (no memory traffic), so every load is unconditional and the waits stay exact;
//   * default-policy X loads (parent / child re-reads hit L2 / the Infinity Cache: the
//     non-temporal variant measured 13-29 % slower), non-temporal output stores.
constexpr int kSliceGroup = 8;

__global__ __launch_bounds__(kWaveBlock) void k_spmm_slice(SpmmBatch sb, int slices) {
  const SpmmProb& P = sb.p[blockIdx.y];
  const int F = sb.F;
  const int lane = threadIdx.x & 63;
  // (blocks renumbered XCD-contiguously, each XCD sweeping its eighth of the rows so that
  // re-reads stay in its L2, measured slower: TD 243 vs 230 us, BU 258 vs 245)
  const int64_t wv = int64_t(blockIdx.x) * 4 + (threadIdx.x >> 6);
  const int64_t g = wv / slices;
  if (g >= P.ngroups) return;
  const int s = int(wv % slices);
  const int64_t nnz = P.ptr[sb.rows];
  const int64_t p0 = wide_chunk_start(P, g, nnz), p1 = wide_chunk_start(P, g + 1, nnz);
  const int n = __builtin_amdgcn_readfirstlane(int(p1 - p0));   // <= 2 * NPGW, wave-uniform
  int64_t pm = lane < 2 * NPGW ? p0 + lane : (lane == 2 * NPGW ? p0 - 1 : p1);
  pm = min<int64_t>(max<int64_t>(pm, 0), nnz - 1);
  const int32_t r_l = P.row[pm], c_l = P.col[pm];
  const float w_l = P.w[pm];
  const int32_t prev_row = p0 > 0 ? __builtin_amdgcn_readlane(r_l, 2 * NPGW) : -1;
  const int32_t next_row = p1 < nnz ? __builtin_amdgcn_readlane(r_l, 2 * NPGW + 1) : -1;
  const uint32_t voff = uint32_t(s * 256 + lane * 4) * 4u;
  const uint32_t rowbytes = uint32_t(F) * 4u;
  typedef u32x4 raw4;
  raw4 A[kSliceGroup], Bq[kSliceGroup];
  float4 acc = f4zero();
  const auto load8 = [&](raw4* dst, int k0) {   // entries k0..k0+7; past n: no traffic
#pragma unroll
    for (int u = 0; u < kSliceGroup; ++u) {
      const int k = k0 + u;
      const int32_t c = __builtin_amdgcn_readlane(c_l, k < 2 * NPGW ? k : 0);
      const __amdgpu_buffer_rsrc_t rs = row_rsrc(P.in + int64_t(c) * P.ld_in, k < n ? rowbytes : 0u);
      dst[u] = __builtin_amdgcn_raw_buffer_load_b128(rs, voff, 0, 0);
    }
  };
  const auto store = [&](float* row, bool fin) {
    const __amdgpu_buffer_rsrc_t rs = row_rsrc(row, rowbytes);
    float4 o = acc;
    if (fin) {
      if (P.bias) {
        const raw4 b = __builtin_amdgcn_raw_buffer_load_b128(row_rsrc(P.bias, rowbytes), voff, 0, 0);
        o = f4add(o, make_float4(__uint_as_float(b.x), __uint_as_float(b.y), __uint_as_float(b.z),
                                 __uint_as_float(b.w)));
      }
      if (sb.epi & BGCN_EPI_RELU) o = f4relu(o);
    }
    const raw4 v = {__float_as_uint(o.x), __float_as_uint(o.y), __float_as_uint(o.z), __float_as_uint(o.w)};
    if (fin) __builtin_amdgcn_raw_buffer_store_b128(v, rs, voff, 0, kAuxNT);
    else __builtin_amdgcn_raw_buffer_store_b128(v, rs, voff, 0, 0);
  };
  int32_t cur = -1;
  bool cur_head = false;
  const auto consume8 = [&](const raw4* src, int k0) {
#pragma unroll
    for (int u = 0; u < kSliceGroup; ++u) {
      const int k = k0 + u;
      if (k >= n) break;                       // uniform
      const int32_t r = __builtin_amdgcn_readlane(r_l, k);
      const float w = __int_as_float(__builtin_amdgcn_readlane(__float_as_int(w_l), k));
      if (r != cur) {
        if (cur >= 0) {
          if (!cur_head) store(P.out + int64_t(cur) * P.ld_out, true);
          else store(P.part + (g * 2 + 0) * int64_t(F), false);
        }
        cur_head = cur < 0 && r == prev_row;
        cur = r;
        acc = f4zero();
      }
      const float4 x = make_float4(__uint_as_float(src[u].x), __uint_as_float(src[u].y),
                                   __uint_as_float(src[u].z), __uint_as_float(src[u].w));
      acc = f4fma(w, x, acc);
    }
  };
  static_assert(2 * NPGW <= 4 * kSliceGroup, "four groups cover a chunk");
  load8(A, 0);
  load8(Bq, 8);
  consume8(A, 0);
  if (n > 16) {                                // uniform; typical chunks stop here
    load8(A, 16);
    consume8(Bq, 8);
    load8(Bq, 24);
    consume8(A, 16);
    consume8(Bq, 24);
  } else {
    consume8(Bq, 8);
  }
  if (cur >= 0) {
    const bool ends = next_row != cur;
    if (!cur_head && ends) store(P.out + int64_t(cur) * P.ld_out, true);
    else if (cur_head) store(P.part + (g * 2 + 0) * int64_t(F), false);
    else store(P.part + (g * 2 + 1) * int64_t(F), false);
  }
}

// Wide fixup: one block per (chunk boundary g*NPGW, 1024-float slice): if the row at the
// boundary started before it and this is its last chunk, sum tail[g0] + head[g0+1..g]
// in chunk order (four loads in flight) and write the row.
__global__ __launch_bounds__(256) void k_spmm_fixup_wide(SpmmBatch sb) {
  const SpmmProb& P = sb.p[blockIdx.z];
  const int64_t g = int64_t(blockIdx.x) + 1;
  if (g >= P.ngroups) return;
  const int64_t nnz = P.ptr[sb.rows];
  const int64_t pb = g * NPGW;
  if (pb >= nnz) return;
  const int32_t r = P.row[pb];
  if (P.row[pb - 1] != r) return;
  const int64_t rs = P.ptr[r], re = P.ptr[r + 1];
  if (re - rs <= NPGW) return;               // short rows are never split (wide_chunk_start)
  const int64_t g0 = rs / NPGW, g1 = (re - 1) / NPGW;
  if (g1 != g) return;
  const int F = sb.F;
  const int fo = blockIdx.y * kWideSlice + threadIdx.x * 4;
  if (fo >= F) return;
  float4 acc = ld4(P.part + (g0 * 2 + 1) * int64_t(F) + fo);
  int64_t q = g0 + 1;
  for (; q + 3 <= g1; q += 4) {
    float4 v[4];
#pragma unroll
    for (int u = 0; u < 4; ++u) v[u] = ld4(P.part + ((q + u) * 2 + 0) * int64_t(F) + fo);
#pragma unroll
    for (int u = 0; u < 4; ++u) acc = f4add(acc, v[u]);
  }
  for (; q <= g1; ++q) acc = f4add(acc, ld4(P.part + (q * 2 + 0) * int64_t(F) + fo));
  st4_chain(P.out, int64_t(r) * P.ld_out + fo, epilogue(acc, P.bias ? ld4(P.bias + fo) : f4zero(), sb.epi));
}

}  // namespace

// chunk size of the kernel family spmm_batch_impl picks for width F
static int npg_for(int32_t F) { return (F == 64 || F == 128) ? NPG : NPGW; }

size_t spmm_ws_size(int64_t capacity, int32_t F) {
  const int64_t ngroups = (capacity + npg_for(F) - 1) / npg_for(F);
  return size_t(ngroups) * 2 * size_t(F) * sizeof(float) + 256;
}

static bool a16(const void* p) { return (reinterpret_cast<uintptr_t>(p) & 15) == 0; }


// Whether spmm_batch_impl takes K1's plans (k_spmm_rows) for these problems.  The plan pays
// off while long rows are few and short (one block each): measured on the fused step
// beside the next batch's preparation, Twitter15-sized batches (E + N = 55k) 0.356 vs
// 0.362 ms per step; with 1024-thread row blocks (one per CU) Weibo-sized ones (188k)
// lost (0.85 vs 0.77 ms), with 512-thread blocks they win too (weibo_bf16 0.698-0.700 vs
// 0.719, synth1024_bf16 0.853 vs 0.867: profiles/r02_plan_ab.txt).  BGCN_SPMM_PLAN=0/1
// forces either form (A/B runs; read per call: tests switch it).
bool spmm_planned(const SpmmBatch& sb, int count) {
  bool planned = sb.F == 64;
  int64_t capmax = 0;
  for (int k = 0; k < count; ++k) {
    planned = planned && sb.p[k].plan.bnd && sb.p[k].plan.longs && sb.p[k].plan.nlong;
    capmax = sb.p[k].capacity > capmax ? sb.p[k].capacity : capmax;
  }
  const char* pe = std::getenv("BGCN_SPMM_PLAN");
  const int plan_env = pe ? atoi(pe) : -1;
  return planned && (plan_env == 1 || (plan_env != 0 && capmax <= kPlanMaxEntries));
}

// count problems (1 or 2) described by sb.p[0..count), each with its own part buffer
int spmm_batch_impl(SpmmBatch& sb, int count, hipStream_t stream) {
  const int F = sb.F;
  BGCN_CHECK_ARG(count == 1 || count == 2, "1 or 2 problems per launch");
  BGCN_CHECK_ARG(sb.rows > 0, "bad rows");
  BGCN_CHECK_ARG(F > 0 && F % 4 == 0, "F must be a positive multiple of 4");
  int64_t gmax = 0;
  for (int k = 0; k < count; ++k) {
    const SpmmProb& P = sb.p[k];
    BGCN_CHECK_ARG(P.ptr && P.row && P.col && P.w && (P.in || sb.sg.sgn) && P.out && P.part, "null pointer");
    BGCN_CHECK_ARG(P.ld_in % 4 == 0 && P.ld_out % 4 == 0 && P.ld_in >= F && P.ld_out >= F,
                   "ld must be >= F and a multiple of 4");
    BGCN_CHECK_ARG(a16(P.in) && a16(P.out) && (!P.bias || a16(P.bias)) && a16(P.part),
                   "in/out/bias must be 16-byte aligned");
    gmax = P.ngroups > gmax ? P.ngroups : gmax;
  }
  if (gmax == 0) return BGCN_OK;
  const unsigned gy = unsigned(count);
  int64_t capmax = 0;
  for (int k = 0; k < count; ++k) capmax = sb.p[k].capacity > capmax ? sb.p[k].capacity : capmax;
  const bool planned = spmm_planned(sb, count);
  BGCN_CHECK_ARG(!sb.sg.sgn || (planned && count == 2 && sb.sg.dhead && sb.sg.batch && sb.sg.tree_ptr &&
                                sb.sg.B > 0 && sb.sg.tree_status[0] && sb.sg.tree_status[1]),
                 "readout-gradient input needs the planned TD/BU pair");
  if (planned) {   // K1's plans: complete rows per chunk, long rows per block, no fixup
    const int64_t gplan = (capmax + kPlanGrid - 1) / kPlanGrid;   // K1's chunk grid
    const int64_t nchunk = (gplan + kRowsGroups - 1) / kRowsGroups;
    int nlongblk = int(std::min<int64_t>(256, std::max<int64_t>(1, capmax / (kPlanChunk + 1))));
    nlongblk += int((8 - (nchunk + nlongblk) % 8) % 8);   // gridDim.x % 8 == 0 (xcd_contig)
    if (sb.sg.sgn)
      hipLaunchKernelGGL(k_spmm_rows<true>, dim3(unsigned(nchunk + nlongblk), gy), dim3(kRowsThreads), 0, stream,
                         sb, nchunk, nlongblk);
    else
      hipLaunchKernelGGL(k_spmm_rows<false>, dim3(unsigned(nchunk + nlongblk), gy), dim3(kRowsThreads), 0,
                         stream, sb, nchunk, nlongblk);
  } else if (F == 64) {
    constexpr int L = 16;
    hipLaunchKernelGGL(k_spmm_narrow<L>, dim3(grid_for(gmax, 256 / L), gy), dim3(256), 0, stream, sb);
    BGCN_CHECK_LAUNCH();
    if (gmax > 1)
      hipLaunchKernelGGL(k_spmm_fixup_narrow<L>, dim3(grid_for(gmax - 1, 256 / L), gy), dim3(256), 0,
                         stream, sb);
  } else if (F == 128) {
    constexpr int L = 32;
    hipLaunchKernelGGL(k_spmm_narrow<L>, dim3(grid_for(gmax, 256 / L), gy), dim3(256), 0, stream, sb);
    BGCN_CHECK_LAUNCH();
    if (gmax > 1)
      hipLaunchKernelGGL(k_spmm_fixup_narrow<L>, dim3(grid_for(gmax - 1, 256 / L), gy), dim3(256), 0,
                         stream, sb);
  } else {
    const int ws = (F + 255) / 256;                 // 256-float slices per chunk
    const int64_t nblk = (gmax * ws + 3) / 4;
    BGCN_CHECK_ARG(nblk < (int64_t(1) << 31), "aggregation too large for one launch");
    hipLaunchKernelGGL(k_spmm_slice, dim3(unsigned(nblk), gy), dim3(kWaveBlock), 0, stream, sb, ws);
    BGCN_CHECK_LAUNCH();
    const unsigned slices = unsigned((F + kWideSlice - 1) / kWideSlice);
    if (gmax > 1)
      hipLaunchKernelGGL(k_spmm_fixup_wide, dim3(unsigned(gmax - 1), slices, gy), dim3(256), 0, stream, sb);
  }
  BGCN_CHECK_LAUNCH();
  return BGCN_OK;
}

int spmm_impl(const int32_t* ptr, const int32_t* row, const int32_t* col, const float* w,
              int64_t rows, int64_t capacity, const float* in, int64_t ld_in, float* out,
              int64_t ld_out, int32_t F, const float* bias, int epi, void* ws, size_t ws_bytes,
              hipStream_t stream) {
  BGCN_CHECK_ARG(rows > 0 && capacity >= rows, "bad rows/capacity");
  BGCN_CHECK_ARG(ws && ws_bytes >= spmm_ws_size(capacity, F), "workspace too small");
  SpmmBatch sb{};
  sb.rows = rows;
  sb.F = F;
  sb.epi = epi;
  sb.p[0] = SpmmProb{ptr, row, col, w, in, ld_in, out, ld_out, bias, static_cast<float*>(ws),
                     (capacity + npg_for(F) - 1) / npg_for(F), capacity};
  return spmm_batch_impl(sb, 1, stream);
}

int64_t spmm_groups(int64_t capacity, int32_t F) { return (capacity + npg_for(F) - 1) / npg_for(F); }

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

BT_READER(spmm)
