// Sparse-feature path of the fused BiGCN encoder.
//
// The reference's node features are bag-of-words counts (Process/getTwittergraph.py:
// 67-72: x[n, 5000] holds the "idx:count" pairs of one post, ~10-20 non-zeros) stored
// dense.  Every product with X or with the root-extended X[root] is exact when the
// zero entries are skipped (x * w == 0 for x == 0), so this path reads the dense X from
// HBM exactly once per step, compacts every row to an ELL list (col, val) of at most
// kCap entries, and evaluates
//   conv1        Z1[i]         = sum_s val_s * W1^T[col_s]                      (K2)
//   conv2        Z2_d[i]       = sum_{k<64} a_ik W2_d^T[k] + sum_{s in root(i)} a_is W2_d^T[64+col_s]
//   dW2 (root)   dW2_d[:,64+c] = sum_{b: c in root_b} 2 relu(x_rb,c) sum_{i in b} keep_i[64+c] dZ2_d[i]
//   dW1          dW1[:, c]     = sum_{i: x_ic != 0} x_ic dZ1[i]                 (K10)
// (a_ik = keep * 2 * relu(.)), every sum in a fixed order (deterministic).  dW1 and the
// dW2 root columns come out of one pass over the column-sorted (CSC) non-zeros of X.
// A row with more than kCap non-zeros sets a device flag that switches the whole batch
// to the dense MFMA path (identical results); every kernel of both paths checks the flag
// on the device, so the choice costs no host sync.
#include <cstdlib>
#include <cstring>



#include "bgcn_bwd.h"
#include "bgcn_drop_body.h"
#include "bgcn_graph_body.h"
#include "bgcn_internal.h"
#include "bgcn_sparse.h"
#include "bgcn_trace.h"

namespace bgcn {
namespace {

__device__ __forceinline__ bool use_sparse(const SparseState& S) { return S.mode != 1 && S.flags[0] == 0; }

// the prologue's clears when its launch is skipped (weight images current): the step's
// status word and the readout tickets, by conv1's block 0 (both are first used by the
// readout, two launches later)
__device__ __forceinline__ void conv1_clears(const SparseState& S) {
  if (!S.conv1_clears || blockIdx.x != 0) return;
  if (threadIdx.x == 0 && S.zero_word) *S.zero_word = 0;
  if (S.rtick)
    for (int64_t b = threadIdx.x; b < S.B; b += blockDim.x) S.rtick[b] = 0;
}

// ---------------------------------------------------------------- weight transposes
// W1T[c][d*64 + o] = W1_d[o][c] (c < F) and W2T_d[k][o] = W2_d[o][k] (k < 64+F):
// 32 x 32 tiles through LDS; blockIdx.z: 0/1 = W1 td/bu, 2/3 = W2 td/bu.
__device__ __forceinline__ void transpose_tile(const SparseState& S, int bx, int by, int z,
                                               const float* __restrict__ w1td,
                                               const float* __restrict__ w1bu,
                                               const float* __restrict__ w2td,
                                               const float* __restrict__ w2bu) {
  __shared__ float tile[32][33];
  const int64_t K = z < 2 ? S.F : S.F + H;
  const float* src = z == 0 ? w1td : z == 1 ? w1bu : z == 2 ? w2td : w2bu;
  const int64_t k0 = int64_t(bx) * 32;
  const int o0 = by * 32;
  if (k0 >= K) return;
  const int tx = threadIdx.x & 31, ty = threadIdx.x >> 5;  // 32 x 8
  for (int r = ty; r < 32; r += 8) {
    const int64_t k = k0 + tx;
    tile[r][tx] = k < K ? src[int64_t(o0 + r) * K + k] : 0.f;
  }
  __syncthreads();
  for (int r = ty; r < 32; r += 8) {
    const int64_t k = k0 + r;
    if (k >= K) continue;
    if (z < 2) S.w1t[k * (2 * H) + z * H + o0 + tx] = tile[tx][r];
    else S.w2t[(int64_t(z - 2) * K + k) * H + o0 + tx] = tile[tx][r];
  }
}

// Batch part of the prologue (block bid of blockDim threads): blocks [0, nR) the node ->
// root map (block 0 also resets the overflow flags), then the tree pointers (binary
// search in the sorted batch vector).
__device__ inline void prologue_batch_body(const SparseState& S, const int64_t* __restrict__ batch,
                                           const int64_t* __restrict__ rootindex,
                                           int32_t* __restrict__ node_root, int32_t* __restrict__ tree_ptr,
                                           int bid, int nR) {
  if (bid == 0 && nR > 0 && S.mode != 1 && threadIdx.x < 8) S.flags[threadIdx.x] = 0;
  if (bid < nR) {
    const int64_t i = int64_t(bid) * blockDim.x + threadIdx.x;
    if (i >= S.N) return;
    const int64_t b = batch[i];
    // a node in no tree would keep stale backward rows (the readout never visits it):
    // flagged as a bad index, which invalidates the step
    if ((b < 0 || b >= S.B) && S.bstatus) atomicOr(S.bstatus, 1);
    const int64_t bc = b < 0 ? 0 : (b >= S.B ? S.B - 1 : b);
    const int64_t r = rootindex[bc];
    node_root[i] = int32_t((b >= 0 && b < S.B && r >= 0 && r < S.N) ? r : 0);
    return;
  }
  const int64_t b = int64_t(bid - nR) * blockDim.x + threadIdx.x;
  if (b > S.B) return;
  int64_t lo = 0, hi = S.N;
  while (lo < hi) {
    const int64_t mid = (lo + hi) >> 1;
    if (batch[mid] < b) lo = mid + 1; else hi = mid;
  }
  tree_ptr[b] = int32_t(lo);
}

// W2_d[:, :64] split for the bf16 MFMA (kSplitBlocks 256-thread blocks per direction, one
// element per thread): conv2's image [3][o][k] and the middle launch's [3][c][o] (hi / mid /
// lo: both feed fp32-grade six-product MFMAs).
constexpr int kSplitBlocks = H * H / 256;
__device__ inline void split_w2_block(const SparseState& S, int sb, const float* __restrict__ w2td,
                                      const float* __restrict__ w2bu) {
  const int d = sb / kSplitBlocks;
  const float* W2 = d == 0 ? w2td : w2bu;
  const int64_t ld = S.F + H;
  __bf16* cs = S.w2s + int64_t(d) * 3 * H * kW2sLd;
  __bf16* ds = S.w2d + int64_t(d) * 3 * H * kW2dLd;
  {
    const int e = (sb % kSplitBlocks) * 256 + threadIdx.x;
    const int o = e >> 6, k = e & 63;
    __bf16 x, y, z;
    const float v = W2[int64_t(o) * ld + k];
    split3_bf16(v, x, y, z);
    cs[o * kW2sLd + k] = x;
    cs[H * kW2sLd + o * kW2sLd + k] = y;
    cs[2 * H * kW2sLd + o * kW2sLd + k] = z;
    split3_bf16(v, x, y, z);
    ds[k * kW2dLd + o] = x;
    ds[H * kW2dLd + k * kW2dLd + o] = y;
    ds[2 * H * kW2dLd + k * kW2dLd + o] = z;
  }
}

// Forward prologue, one launch: the weight transposes (sparse path), node -> root map,
// tree pointers (binary search in the sorted batch vector) and the overflow-flag reset.
// Block ranges: [0, nT) transposes, [nT, nT + nR) node_root, then tree_ptr.
__global__ __launch_bounds__(256) void k_prologue(SparseState S, const float* __restrict__ w1td,
                                                  const float* __restrict__ w1bu,
                                                  const float* __restrict__ w2td,
                                                  const float* __restrict__ w2bu,
                                                  const int64_t* __restrict__ batch,
                                                  const int64_t* __restrict__ rootindex,
                                                  int32_t* __restrict__ node_root,
                                                  int32_t* __restrict__ tree_ptr, int nTx, int nT,
                                                  int nR) {
  const int blk = blockIdx.x;
  if (blk == 0 && threadIdx.x == 0 && S.zero_word) *S.zero_word = 0;
  if (blk == 0 && S.rtick)
    for (int64_t b = threadIdx.x; b < S.B; b += blockDim.x) S.rtick[b] = 0;
  if (blk < nT) {
    if (S.mode == 1) return;
    transpose_tile(S, blk % nTx, (blk / nTx) % 2, blk / (2 * nTx), w1td, w1bu, w2td, w2bu);
    return;
  }
  const int nS = nT > 0 ? 2 * kSplitBlocks : 0;   // the split W2 images ride with the transposes
  if (blk < nT + nS) {
    split_w2_block(S, blk - nT, w2td, w2bu);
    return;
  }
  prologue_batch_body(S, batch, rootindex, node_root, tree_ptr, blk - nT - nS, nR);
}

// ---------------------------------------------------------------- X compaction + conv1
// One wave per row.  The whole row is requested up front (16-byte pieces per lane:
// 20 KiB of a 5000-wide row in flight per wave) so HBM sees deep, independent streams;
// then the non-zeros are compacted in ascending column order - a 16-byte piece that is
// all zero across the wave (the common case for bag-of-words rows) costs one ballot -
// and Z1[i] = sum val * W1T[col] with each lane owning 2 of the 128 outputs.
constexpr int kRowChunks = 20;  // float4 per lane per pass (F <= 5120 in one pass)

// Z1[i] += sum_s val_s * W1T[col_s] for the (col, val) pairs of lane-held lists: lane s
// (< cnt) holds pair s; the pairs reach the wave by scalar readlane, gathers unconditional
// (clamped column), 8 in flight.
__device__ __forceinline__ float2 conv1_row(const SparseState& S, int cnt, int32_t col_l, float val_l) {
  const int lane = threadIdx.x & 63;
  float2 acc = make_float2(0.f, 0.f);
  for (int s0 = 0; s0 < cnt; s0 += 8) {
    float2 w[8];
    float x[8];
#pragma unroll
    for (int u = 0; u < 8; ++u) {
      const int sl = s0 + u < cnt ? s0 + u : 0;                // wave-uniform
      const int32_t c = min(max(__builtin_amdgcn_readlane(col_l, sl), 0), int32_t(S.F - 1));
      x[u] = s0 + u < cnt ? __int_as_float(__builtin_amdgcn_readlane(__float_as_int(val_l), sl)) : 0.f;
      w[u] = *reinterpret_cast<const float2*>(S.w1t + int64_t(c) * (2 * H) + 2 * lane);
    }
#pragma unroll
    for (int u = 0; u < 8; ++u) {
      acc.x = fmaf(x[u], w[u].x, acc.x);
      acc.y = fmaf(x[u], w[u].y, acc.y);
    }
  }
  return acc;
}

// Row i of X -> its ELL list (+ conv1).  r: the row's 16-byte chunks (row_chunks<TX>()
// per lane: the whole row, F <= kSparseMaxF), already in flight.
static_assert(kRowChunks * 64 * 4 >= kSparseMaxF, "one pass per row");
template <class TX> constexpr int row_chunks() { return kRowChunks * 4 / XChunk<TX>::kElems; }
// Two ways to place a row's non-zeros in ascending column order.  Per element: a ballot
// per element position of the 16-byte piece, every lane counting the set lanes below it
// (E ballots per piece).  By prefix: each lane's non-zero mask, then the exclusive prefix
// of the per-lane counts - one ballot when no lane holds two non-zeros (the common case
// for bag-of-words rows), else by the counts' bit planes - and a loop over the lane's own
// non-zeros.  The prefix form halves the kernel's registers (205 -> 126-138) and moves bf16
// X at 5.9 instead of 4.3 TB/s alone on the GPU (a bf16 piece holds 8 elements: 8 ballots
// per piece).  Beside the training chain the faster pass costs the chain more: fp32 keeps
// the per-element form (twitter15 0.289 vs 0.298-0.316 ms per step), bf16 takes the
// prefix form paced at one block per CU (weibo_bf16 0.646 vs 0.669 ms, synth1024_bf16
// 0.793 vs 0.811: profiles/r02_compact_ab.txt).  BGCN_COMPACT_PREFIX: 1 bf16 only, 2 both.
#ifndef BGCN_COMPACT_PREFIX
#define BGCN_COMPACT_PREFIX 1
#endif
template <class TX> constexpr bool compact_by_prefix() {
  return BGCN_COMPACT_PREFIX >= 2 || (BGCN_COMPACT_PREFIX == 1 && sizeof(TX) == 2);
}
// Walk a row's non-zeros in ascending column order: emit(pos, col, val) for each, pos =
// its rank in the row (lanes below a lane contribute all their non-zeros first); returns
// the row's count (wave-uniform).
template <class TX, class Emit>
__device__ __forceinline__ int walk_row(const u32x4* r, Emit emit) {
  typedef XChunk<TX> XC;
  constexpr int E = XC::kElems;
  const int lane = threadIdx.x & 63;
  const uint64_t lt = (lane == 0) ? 0ull : (~0ull >> (64 - lane));
  int cnt = 0;
  if constexpr (!compact_by_prefix<TX>()) {
#pragma unroll
  for (int u = 0; u < row_chunks<TX>(); ++u) {
    const u32x4 ru = r[u];                           // past the row: 0 (range-checked load)
    if (__ballot(XC::any(ru)) == 0ull) continue;     // wave-uniform skip
    int pos = cnt;
#pragma unroll
    for (int c = 0; c < E; ++c) {
      const uint64_t m = __ballot(XC::nz(ru, c));
      pos += __popcll(m & lt);
      cnt += __popcll(m);
    }
    const int col0 = (u * 64 + lane) * E;
#pragma unroll
    for (int c = 0; c < E; ++c) {
      if (XC::nz(ru, c)) {
        emit(pos, col0 + c, XC::elem(ru, c));
        ++pos;
      }
    }
  }
  } else {
#pragma unroll
  for (int u = 0; u < row_chunks<TX>(); ++u) {
    const u32x4 ru = r[u];                           // past the row: 0 (range-checked load)
    uint32_t mb = 0;                                 // this lane's non-zero elements
#pragma unroll
    for (int c = 0; c < E; ++c) mb |= uint32_t(XC::nz(ru, c)) << c;
    const uint64_t any = __ballot(mb != 0u);
    if (any == 0ull) continue;                       // wave-uniform skip
    // the exclusive prefix of the per-lane counts, one ballot when no lane holds two (the
    // common case for bag-of-words rows), else by the counts' bit planes
    const int n = __popc(mb);
    int pos = cnt;
    if (__ballot(n > 1) == 0ull) {
      pos += __popcll(any & lt);
      cnt += __popcll(any);
    } else {
#pragma unroll
      for (int k = 0; k < 4; ++k) {                  // n <= 8
        const uint64_t bk = __ballot((n >> k) & 1);
        pos += __popcll(bk & lt) << k;
        cnt += __popcll(bk) << k;
      }
    }
    const int col0 = (u * 64 + lane) * E;
    while (mb) {
      const int c = __builtin_ctz(mb);
      mb &= mb - 1u;
      emit(pos, col0 + c, XC::elem(ru, c));
      ++pos;
    }
  }
  }
  return cnt;
}

// The entries past kCap of a long row -> dst[pos] (pos >= kCap), in column order.  The row
// is loaded again one 16-byte piece per lane at a time in a rolled loop: the rare branch
// must not add registers to the pass over X (an unrolled second walk took the fp32 form
// from 205 to 256 + AGPRs, half its occupancy).
template <class TX>
__device__ void spill_walk(__amdgpu_buffer_rsrc_t rs, uint2* dst) {
  typedef XChunk<TX> XC;
  constexpr int E = XC::kElems;
  const int lane = threadIdx.x & 63;
  const uint64_t lt = (lane == 0) ? 0ull : (~0ull >> (64 - lane));
  int cnt = 0;
  constexpr int kG = 5;                              // pieces in flight
  static_assert(row_chunks<TX>() % kG == 0, "spill walk groups");
#pragma unroll 1
  for (int u0 = 0; u0 < row_chunks<TX>(); u0 += kG) {
  u32x4 rg[kG];
#pragma unroll
  for (int v = 0; v < kG; ++v)
    rg[v] = __builtin_amdgcn_raw_buffer_load_b128(rs, ((u0 + v) * 64 + lane) * 16, 0, kAuxNT);
#pragma unroll
  for (int v = 0; v < kG; ++v) {
    const int u = u0 + v;
    const u32x4 ru = rg[v];
    uint32_t mb = 0;
#pragma unroll
    for (int c = 0; c < E; ++c) mb |= uint32_t(XC::nz(ru, c)) << c;
    const int n = __popc(mb);
    int pos = cnt;
#pragma unroll
    for (int k = 0; k < 4; ++k) {                    // n <= 8
      const uint64_t bk = __ballot((n >> k) & 1);
      pos += __popcll(bk & lt) << k;
      cnt += __popcll(bk) << k;
    }
    const int col0 = (u * 64 + lane) * E;
    while (mb) {
      const int c = __builtin_ctz(mb);
      mb &= mb - 1u;
      if (pos >= kCap) dst[pos] = make_uint2(uint32_t(col0 + c), __float_as_uint(XC::elem(ru, c)));
      ++pos;
    }
  }
  }
}

// Row i of X -> its ELL list, the entries past kCap to the spill pool (+ conv1 over both).
template <bool kConv1, class TX>
__device__ __forceinline__ void compact_row(const SparseState& S, int64_t i, const u32x4* r,
                                            __amdgpu_buffer_rsrc_t rs, int32_t* s_col, float* s_val,
                                            float* __restrict__ Z1) {
  const int lane = threadIdx.x & 63;
  const int cnt = walk_row<TX>(r, [&](int pos, int col, float v) {
    if (pos < kCap) {
      s_col[pos] = col;
      s_val[pos] = v;
    }
  });
  if (lane == 0) S.nnz[i] = cnt;
  const int nov = cnt > kCap ? cnt - kCap : 0;       // wave-uniform
  int off = 0;
  if (nov > 0) {
    // a row of more words than the ELL holds (the reference caps none, getTwittergraph.py:
    // 16-24): its tail goes to the batch's spill pool, in column order
    int o = 0;
    if (lane == 0) o = atomicAdd(&S.flags[1], nov);
    o = __builtin_amdgcn_readfirstlane(o);
    if (o < 0 || int64_t(o) + nov > S.ovf_cap) {     // pool full: the batch goes dense
      if (lane == 0) atomicOr(&S.flags[0], 1);
      return;
    }
    if (lane == 0) {
      S.ovf_off[i] = o;
      S.long_rows[atomicAdd(&S.flags[2], 1)] = int32_t(i);   // conv1's long-row blocks
    }
    uint2* dst = S.ovf + o - kCap;
    spill_walk<TX>(rs, dst);
    off = o;
  }
  const int ce = cnt < kCap ? cnt : kCap;
  __builtin_amdgcn_s_waitcnt(0xc07f);   // lgkmcnt(0): this wave's LDS writes have landed
  __builtin_amdgcn_wave_barrier();
  const int32_t col_l = lane < ce ? s_col[lane] : 0;
  const float val_l = lane < ce ? s_val[lane] : 0.f;
  if (lane < ce) {
    S.cols[i * kCap + lane] = col_l;
    S.vals[i * kCap + lane] = val_l;
  }
  if (kConv1) {
    float2 acc = conv1_row(S, ce, col_l, val_l);
    if (nov > 0) {   // the spilled entries, 64 at a time (this wave's own stores, read back)
      __builtin_amdgcn_fence(__ATOMIC_RELEASE, "workgroup");
      __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "workgroup");
      for (int k0 = 0; k0 < nov; k0 += 64) {
        const int n = min(64, nov - k0);
        const uint2 e = S.ovf[off + k0 + min(lane, n - 1)];
        const float2 p = conv1_row(S, n, int32_t(e.x), __uint_as_float(e.y));
        acc.x += p.x;
        acc.y += p.y;
      }
    }
    *reinterpret_cast<float2*>(Z1 + i * (2 * H) + 2 * lane) = acc;
  }
}

// kConv1 = true: compaction + conv1 in one pass (the encoder's forward); false: the ELL
// only (weight-independent batch preparation, bgcn_prepare_batch).  A wave keeps ~20 KB
// of X in flight: one fp32 row, or two bf16 rows (their loads issued together).
// Body: block bid of nblk 256-thread blocks (grid-stride over rows).
template <bool kConv1, class TX>
__device__ inline void compact_body(const SparseState& S, const TX* __restrict__ X, int64_t ldx,
                                    float* __restrict__ Z1, int bid, int nblk) {
  constexpr int kRows = sizeof(TX) == 2 ? 2 : 1;
  __shared__ int32_t s_col[4][kCap];
  __shared__ float s_val[4][kCap];
  if (S.mode == 1) return;
  const int wave = threadIdx.x >> 6, lane = threadIdx.x & 63;
  // grid-stride over rows (the preparation's grid covers every row once: one fp32 row or
  // two bf16 rows per wave; a capped grid strides)
  const int64_t stride = int64_t(nblk) * 4;
  for (int64_t i0 = int64_t(bid) * 4 + wave; i0 < S.N; i0 += stride * kRows) {
    u32x4 r[kRows][row_chunks<TX>()];
    __amdgpu_buffer_rsrc_t rs[kRows];
#pragma unroll
    for (int k = 0; k < kRows; ++k) {   // all loads in flight; a row past N reads nothing
      const int64_t ik = i0 + k * stride;
      rs[k] = row_rsrc(X + min<int64_t>(ik, S.N - 1) * ldx, ik < S.N ? uint32_t(S.F * sizeof(TX)) : 0u);
#pragma unroll
      for (int u = 0; u < row_chunks<TX>(); ++u)
        r[k][u] = __builtin_amdgcn_raw_buffer_load_b128(rs[k], (u * 64 + lane) * 16, 0, kAuxNT);
    }
#pragma unroll
    for (int k = 0; k < kRows; ++k) {
      const int64_t i = i0 + k * stride;
      if (i < S.N) compact_row<kConv1, TX>(S, i, r[k], rs[k], s_col[wave], s_val[wave], Z1);
    }
  }
}

// The host-fed input form (bgcn_batch.x_row_ptr / x_col / x_val): the rows arrive already
// compacted, in ascending column order, so the ELL list, the spill pool and the long-row
// list are filled from them with the contents compact_row writes from the dense row (the
// step computes the same bits either way).  One 32-lane half-wave per row (a BoW row holds
// ~12 entries), grid-stride; reads nnz x 8 bytes instead of N x F x 4.  The lists come
// from the host, so every row is checked first: a negative start or count, a column
// outside [0, F) or columns not strictly ascending set the batch status bit 0 (the step
// is then rejected like a bad edge index) and the row is written empty, so no later
// kernel indexes by a bad column.
__device__ inline void csr_ell_body(const SparseState& S, const int32_t* __restrict__ rp,
                                    const int32_t* __restrict__ rc, const float* __restrict__ rv, int bid,
                                    int nblk) {
  if (S.mode == 1) return;
  const int lane = threadIdx.x & 31;
  const int half = threadIdx.x & 32;
  const int64_t nhalf = int64_t(nblk) * (blockDim.x / 32);
  for (int64_t i = (int64_t(bid) * blockDim.x + threadIdx.x) / 32; i < S.N; i += nhalf) {
    const int32_t b = rp[i], cnt = rp[i + 1] - b;      // half-wave uniform
    bool bad = b < 0 || cnt < 0;
    int32_t c0 = 0;
    float v0 = 0.f;
    if (!bad) {
      bool lbad = false;
      int32_t prev = -1;
      for (int k0 = 0; k0 < cnt; k0 += 32) {
        const int k = k0 + lane;
        const int32_t c = rc[b + min(k, cnt - 1)];
        if (k0 == 0) {
          c0 = c;
          v0 = rv[b + min(k, cnt - 1)];
        }
        int32_t pc = __shfl_up(c, 1, 32);
        if (lane == 0) pc = prev;
        lbad = lbad || (k < cnt && (c < 0 || c >= S.F || c <= pc));
        prev = __shfl(c, 31, 32);                      // (a later chunk exists only if this one is full)
      }
      bad = ((__ballot(lbad) >> half) & 0xffffffffull) != 0ull;
    }
    if (bad) {
      if (lane == 0) {
        S.nnz[i] = 0;
        if (S.bstatus) atomicOr(S.bstatus, 1);
      }
      continue;
    }
    const int ce = cnt < kCap ? cnt : kCap;
    if (lane < ce) {
      S.cols[i * kCap + lane] = c0;
      S.vals[i * kCap + lane] = v0;
    }
    if (lane == 0) S.nnz[i] = cnt;
    if (cnt > kCap) {   // a long row: its tail to the spill pool, as compact_row does
      const int nov = cnt - kCap;
      int o = 0;
      if (lane == 0) o = atomicAdd(&S.flags[1], nov);
      o = __shfl(o, 0, 32);
      if (o < 0 || int64_t(o) + nov > S.ovf_cap) {     // pool full: results invalid (status bit 2)
        if (lane == 0) atomicOr(&S.flags[0], 1);
        continue;
      }
      if (lane == 0) {
        S.ovf_off[i] = o;
        S.long_rows[atomicAdd(&S.flags[2], 1)] = int32_t(i);
      }
      for (int k = lane; k < nov; k += 32)
        S.ovf[o + k] = make_uint2(uint32_t(rc[b + kCap + k]), __float_as_uint(rv[b + kCap + k]));
    }
  }
}

__global__ __launch_bounds__(256) void k_csr_ell(SparseState S, const int32_t* __restrict__ rp,
                                                 const int32_t* __restrict__ rc, const float* __restrict__ rv) {
  csr_ell_body(S, rp, rc, rv, int(blockIdx.x), int(gridDim.x));
}

// bgcn_csr_to_dense: one wave per row, the row assembled in LDS (zeros, then the row's
// entries) and written with 16-byte stores - every output element written once, in order.
template <class TX>
__global__ __launch_bounds__(128) void k_csr_dense(const int32_t* __restrict__ rp, const int32_t* __restrict__ rc,
                                                   const float* __restrict__ rv, int64_t N, int64_t F,
                                                   TX* __restrict__ X, int64_t ldx, int32_t* status) {
  extern __shared__ __attribute__((aligned(16))) float rowbuf[];
  const int wave = threadIdx.x >> 6, lane = threadIdx.x & 63;
  const int64_t Fp = (F + 3) / 4 * 4;
  float* row = rowbuf + wave * Fp;
  const int nw = int(blockDim.x) >> 6;
  for (int64_t i = int64_t(blockIdx.x) * nw + wave; i < N; i += int64_t(gridDim.x) * nw) {
    for (int64_t c = lane; c < Fp; c += 64) row[c] = 0.f;
    __builtin_amdgcn_wave_barrier();
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
    const int32_t b = rp[i], e = rp[i + 1];
    for (int32_t k = b + lane; k < e; k += 64) {
      const int32_t c = rc[k];
      if (c >= 0 && c < F) row[c] = rv[k];
      else if (status) atomicOr(status, 1);
    }
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
    __builtin_amdgcn_wave_barrier();
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
    TX* out = X + i * ldx;
    if constexpr (sizeof(TX) == 4) {
      for (int64_t c = int64_t(lane) * 4; c < F; c += 256)
        *reinterpret_cast<float4*>(out + c) = *reinterpret_cast<const float4*>(row + c);
    } else {   // round to nearest even (the host-fed values of a bf16 batch are bf16-exact)
      for (int64_t c = lane; c < F; c += 64) {
        const uint32_t u = __float_as_uint(row[c]);
        out[c] = TX((u + 0x7fffu + ((u >> 16) & 1u)) >> 16);
      }
    }
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
    __builtin_amdgcn_wave_barrier();
  }
}

template <bool kConv1, class TX>
__global__ __launch_bounds__(256) void k_compact_conv1(SparseState S, const TX* __restrict__ X,
                                                       int64_t ldx, float* __restrict__ Z1) {
  compact_body<kConv1, TX>(S, X, ldx, Z1, int(blockIdx.x), int(gridDim.x));
}

// conv1 lin from a prepared ELL of X (bgcn_prepare_batch): four rows per wave, one per
// 16-lane quarter, lane l of a quarter owning outputs [8l, 8l + 8) of the 128 (both
// directions).  The kernel is latency-bound (ELL load -> W1^T row gathers from L2 ->
// store per row), so a wave keeps four rows' gathers in flight instead of one
// (measured at Weibo size: 62 us for one row per wave, beside nothing).  Entry s of a
// row reaches its quarter by shuffle (entries s and s + 16 per lane); past a row's count
// the value is 0 and the (clamped) column still loads, so every load is unconditional.
constexpr int kC1Rows = 4;
#ifndef BGCN_C1_THREADS
#define BGCN_C1_THREADS 256
#endif
constexpr int kC1Threads = BGCN_C1_THREADS;   // threads per block
__global__ __launch_bounds__(kC1Threads) void k_conv1_gather(SparseState S, float* __restrict__ Z1) {
  BT_BEGIN
  conv1_clears(S);
  if (!use_sparse(S)) return;
  const int lane = threadIdx.x & 63, ql = lane & 15, qb = lane & 48;
  const int64_t i = (int64_t(blockIdx.x) * (kC1Threads / 64) + (threadIdx.x >> 6)) * kC1Rows + (lane >> 4);
  const bool live = i < S.N;
  const int64_t ic = live ? i : S.N - 1;
  const int nall = live ? S.nnz[ic] : 0;
  const int cnt = min(nall, kCap);
  const int32_t c0 = S.cols[ic * kCap + ql], c1 = S.cols[ic * kCap + 16 + ql];
  const float v0 = S.vals[ic * kCap + ql], v1 = S.vals[ic * kCap + 16 + ql];
  // the wave's longest row bounds the loop (uniform)
  int cmax = cnt;
  cmax = max(cmax, __shfl_xor(cmax, 16, 64));
  cmax = max(cmax, __shfl_xor(cmax, 32, 64));
  float4 a0 = f4zero(), a1 = f4zero();
  for (int s0 = 0; s0 < cmax; s0 += 8) {
    float4 w0[8], w1[8];
    float x[8];
#pragma unroll
    for (int u = 0; u < 8; ++u) {
      const int sl = s0 + u;                          // uniform
      const int src = qb + (sl & 15);
      const int32_t c = __shfl(sl < 16 ? c0 : c1, src, 64);
      const float v = __shfl(sl < 16 ? v0 : v1, src, 64);
      x[u] = sl < cnt ? v : 0.f;
      const int32_t cc = min(max(c, 0), int32_t(S.F - 1));
      const float* wr = S.w1t + int64_t(cc) * (2 * H) + 8 * ql;
      w0[u] = ld4(wr);
      w1[u] = ld4(wr + 4);
    }
#pragma unroll
    for (int u = 0; u < 8; ++u) {
      a0 = f4fma(x[u], w0[u], a0);
      a1 = f4fma(x[u], w1[u], a1);
    }
  }
  if (nall > kCap) {   // spilled entries of a long row (rare): one at a time
    const int64_t off = S.ovf_off[ic];
    for (int k = 0; k < nall - kCap; ++k) {
      const uint2 e = S.ovf[off + k];
      const float v = __uint_as_float(e.y);
      const float* wr = S.w1t + int64_t(min(max(int32_t(e.x), 0), int32_t(S.F - 1))) * (2 * H) + 8 * ql;
      a0 = f4fma(v, ld4(wr), a0);
      a1 = f4fma(v, ld4(wr + 4), a1);
    }
  }
  if (live) {
    st4_chain(Z1, i * (2 * H) + 8 * ql, a0);
    st4_chain(Z1, i * (2 * H) + 8 * ql + 4, a1);
  }
  BT_END(1);
}

// The same product with two rows per wave: half-wave h (32 lanes) owns row 2w + h, lane
// l of a half the outputs [4l, 4l + 4) - one 16-byte load per lane per entry, a wave
// instruction still moves 1 KiB (two 512-byte W1^T rows).  The loop runs to the longer
// of the two rows in steps of kStep entries (a wave-uniform bound), so a wave issues
// fewer padded gathers than with four rows, and holds fewer registers (more waves per
// SIMD).
#ifndef BGCN_C1_MODE
#define BGCN_C1_MODE 2   // 0: four rows per wave (k_conv1_gather); 1 / 2: two rows, steps of 8 / 4
#endif
// Long rows (more than kCap non-zeros: the ELL list + the spill pool) get a block each
// instead of a half-wave: a long row walked by one half-wave is a serial chain of gathers
// (270 entries: ~70 us at 4 in flight), so the block's four waves take a quarter of the
// entries each, 8 gathers in flight per wave, combined in wave order (deterministic).
// Blocks stride over the compaction's list of long rows; with none they exit at once.
constexpr int kLongRowBlocks = 256;
__device__ inline void conv1_long_rows(const SparseState& S, float* __restrict__ Z1, int bid, int nblk) {
  __shared__ float part[4][2 * H];
  const int n_long = S.flags[2];
  const int wv = threadIdx.x >> 6, lane = threadIdx.x & 63;
  for (int q = bid; q < n_long; q += nblk) {
    const int64_t i = S.long_rows[q];
    const int nall = S.nnz[i];
    const int64_t off = S.ovf_off[i];
    const int seg = (nall + 3) / 4;
    const int e0 = wv * seg, e1 = min(nall, e0 + seg);
    float2 acc = make_float2(0.f, 0.f);
    for (int k0 = e0; k0 < e1; k0 += 64) {
      const int n = min(64, e1 - k0);
      const int e = k0 + min(lane, n - 1);
      // ELL entry (e < kCap) or pool entry: both loaded from clamped indices, selected after
      const int32_t ce = S.cols[i * kCap + min(e, kCap - 1)];
      const float ve = S.vals[i * kCap + min(e, kCap - 1)];
      const uint2 pe = S.ovf[off + max(e - kCap, 0)];
      const float2 p = conv1_row(S, n, e < kCap ? ce : int32_t(pe.x), e < kCap ? ve : __uint_as_float(pe.y));
      acc.x += p.x;
      acc.y += p.y;
    }
    part[wv][2 * lane] = acc.x;
    part[wv][2 * lane + 1] = acc.y;
    __syncthreads();
    if (threadIdx.x < 2 * H)
      Z1[i * (2 * H) + threadIdx.x] = (part[0][threadIdx.x] + part[1][threadIdx.x]) +
                                     (part[2][threadIdx.x] + part[3][threadIdx.x]);
    __syncthreads();
  }
}

// Entries of two rows per wave (half h: row 2w + h) held by the half's lanes (cl, vl of
// lane hl: entry hl), cnt of this half, cmax the wave-uniform bound: acc += val * W1^T[col].
template <int kStep>
__device__ __forceinline__ float4 conv1_half_entries(const SparseState& S, int32_t cl, float vl, int cnt,
                                                     int cmax, float4 acc) {
  const int lane = threadIdx.x & 63, hl = lane & 31, hb = lane & 32;
  for (int s0 = 0; s0 < cmax; s0 += kStep) {
    float4 w[kStep];
    float x[kStep];
#pragma unroll
    for (int u = 0; u < kStep; ++u) {
      const int sl = s0 + u;                          // uniform, < kCap
      const int32_t c = __shfl(cl, hb + (sl & 31), 64);
      const float v = __shfl(vl, hb + (sl & 31), 64);
      x[u] = sl < cnt ? v : 0.f;
      const int32_t cc = min(max(c, 0), int32_t(S.F - 1));
      w[u] = ld4(S.w1t + int64_t(cc) * (2 * H) + 4 * hl);
    }
#pragma unroll
    for (int u = 0; u < kStep; ++u) acc = f4fma(x[u], w[u], acc);
  }
  return acc;
}
// conv2's root-slot B operand of tree b, direction d (SparseState::rimg): slot s of the
// root's ELL list holds 2 relu(x_root,col_s) W2_d^T[64 + col_s] at k = (s & 1) 16 + (s >> 1)
// of the image's 32-wide rows, split hi / mid / lo - the operand conv2's fill built per item
// from three dependent loads (item root -> its ELL slots -> W2^T rows); one block per (tree,
// direction) of conv1's launch, where the chain has the loads' latency to spare.
__device__ inline void root_image_block(const SparseState& S, const int64_t* __restrict__ rootindex, float sc,
                                        int blk) {
  const int b = blk >> 1, d = blk & 1;
  const int64_t r0 = rootindex[b];
  const int64_t r = r0 >= 0 && r0 < S.N ? r0 : 0;   // (a bad root id is flagged by the batch checks)
  const int rn_all = S.nnz[r];
  const int rn = min(rn_all, kCap);
  const float* w2t = S.w2t + int64_t(d) * (S.F + H) * H;
  __bf16* img = S.rimg + (int64_t(b) * 2 + d) * 3 * H * kCap;
  if (d == 0 && threadIdx.x < kCap)
    S.rcols[int64_t(b) * kCap + threadIdx.x] = threadIdx.x < rn ? uint32_t(H + S.cols[r * kCap + threadIdx.x]) : 0u;
  if (d == 0 && threadIdx.x == 0) S.rinfo[b] = rn_all;
  for (int e = threadIdx.x; e < kCap * (H / 4); e += int(blockDim.x)) {
    const int s = e >> 4, q = (e & 15) * 4;
    const int64_t slot = r * kCap + s;
    const int32_t col = min(max(S.cols[slot], 0), int32_t(S.F - 1));
    const float val = S.vals[slot];
    const float4 w = ld4(w2t + int64_t(H + col) * H + q);
    const float av = s < rn ? sc * fmaxf(val, 0.f) : 0.f;
    const float vv[4] = {av * w.x, av * w.y, av * w.z, av * w.w};
    const int k = (s & 1) * (kCap / 2) + (s >> 1);
#pragma unroll
    for (int u = 0; u < 4; ++u) {
      __bf16 x, y, z;
      split3_bf16(vv[u], x, y, z);
      const int64_t o = int64_t(q + u) * kCap + k;
      img[o] = x;
      img[H * kCap + o] = y;
      img[2 * H * kCap + o] = z;
    }
  }
}

// Blocks [0, nroot): conv2's root images (root_image_block, 2 per tree when the caller wants
// them, else none); then [nroot, nroot + kLongRowBlocks): the long rows (conv1_long_rows);
// then two rows per wave.
template <int kStep>
__global__ __launch_bounds__(256) void k_conv1_rows2(SparseState S, float* __restrict__ Z1,
                                                     const int64_t* __restrict__ rootindex, float sc, int nroot) {
  BT_BEGIN
  conv1_clears(S);
  if (!use_sparse(S)) return;
  if (int(blockIdx.x) < nroot) {
    root_image_block(S, rootindex, sc, int(blockIdx.x));
    return;
  }
  const int bx = int(blockIdx.x) - nroot;
  if (bx < kLongRowBlocks) {
    conv1_long_rows(S, Z1, bx, kLongRowBlocks);
    return;
  }
  const int lane = threadIdx.x & 63, hl = lane & 31;
  const int64_t i = (int64_t(bx - kLongRowBlocks) * 4 + (threadIdx.x >> 6)) * 2 + (lane >> 5);
  const bool live = i < S.N;
  const int64_t ic = live ? i : S.N - 1;
  const int nall = live ? S.nnz[ic] : 0;
  const int cnt = min(nall, kCap);
  const int32_t cl = S.cols[ic * kCap + hl];
  const float vl = S.vals[ic * kCap + hl];
  int cmax = max(cnt, __shfl_xor(cnt, 32, 64));
  cmax = __builtin_amdgcn_readfirstlane(cmax);
  const float4 acc = conv1_half_entries<kStep>(S, cl, vl, cnt, cmax, f4zero());
  if (live && nall <= kCap) st4_chain(Z1, i * (2 * H) + 4 * hl, acc);   // long rows: their block's
  BT_END(1);
}

// ---------------------------------------------------------------- conv2 forward
// conv2 lin on the sparse path, one work item (<= kChunk nodes of one tree) per block:
//   Z2_d[i] = [keep * 2 relu(H1_d[i]) | kept_d(i, s)] . [W2_d^T[0:64] ; Wr_b]
//   Wr_b[s] = 2 relu(x_root,col_s) W2_d^T[64 + col_s]      (s < nnz(root), else 0)
// i.e. one [nodes x (64 + nnz(root))] x [. x 64] product per item, with the dropout-masked
// relu(H1) and the per-node root keep bits (0/1) generated in registers and the block's B
// operand staged once in LDS.  The root keep masks are stored in S.rbits for the dW2 root
// columns of the backward.  Each wave stages its 32-row H1 tile through LDS (coalesced).
//
// The product runs on the bf16 MFMA in the fp32-grade split form (mfma_x6, bgcn_common.h):
// the f32-input MFMA issues at the FP32 vector rate and bounds this kernel at Weibo /
// 1024-node sizes; the three-product form (~1e-5 relative) flips relu'(H2) for entries
// near zero, hence six.  B is staged transposed and pre-split (hi / mid / lo bf16 [o][k]):
// k < 64 the H1 columns (W2^T rows), k in [64, 96) the root slots (slot 2j + h at
// 64 + 16h + j, value 2 relu(x_root) W2^T[64 + col]).  K order: lane half h owns H1
// columns [32h, 32h + 32) (k-step s: columns 32h + 8s + j) and root slots 2j + h (k-step
// t: slots 2(8t + j) + h), so each lane hashes only its own keep words and the steps past
// the root's non-zeros are skipped; the keep bits are exact in bf16 (three products).
#ifndef BGCN_C2_PREFETCH
#define BGCN_C2_PREFETCH 1   // 0: each H1 tile requested when it is staged (30 VGPRs fewer)
#endif
constexpr int kC2Ld = H + 1;             // f32 row stride of the staged H1 tiles
constexpr int kC2K = H + kCap;           // B rows: 64 H1 columns + 32 root slot positions
constexpr int kC2Ld16 = kC2K + 8;        // bf16 row stride of the split B (16-byte aligned)
__global__ __launch_bounds__(256) void k_conv2_sparse(SparseState S, const float* __restrict__ H1,
                                                      const int32_t* __restrict__ tree_ptr,
                                                      const int64_t* __restrict__ rootindex,
                                                      float* __restrict__ Z2, KeepSrc keep) {
  BT_BEGIN
  if (!use_sparse(S)) return;
  const int item = blockIdx.x;
  if (item >= S.tree_item0[S.B]) return;
  __shared__ __attribute__((aligned(16))) __bf16 Bs[3][H * kC2Ld16];   // hi, mid, lo
  __shared__ float Hs[4 * 32 * kC2Ld];
  __shared__ uint32_t rk[kCap];
  const int d = blockIdx.y;
  const int64_t beg = S.item_beg[item], end = S.item_end[item];
  const int wv = threadIdx.x >> 6, l = threadIdx.x & 63, r32 = l & 31, h = l >> 5;
  // the wave's first H1 tile is requested before the B fill's dependent chain (root ->
  // its ELL slots -> W2^T rows) starts, so its latency hides behind the fill; a tile past
  // the item loads (clamped) rows it then ignores - no load under a branch
  auto h1load = [&](int t, float4 (&hv)[8]) {   // coalesced: 8 x 1 KiB per wave
    const int64_t i0 = beg + 32 * t;
#pragma unroll
    for (int u = 0; u < 8; ++u) {
      const int e = l + 64 * u, rr = e >> 4, q = (e & 15) * 4;
      hv[u] = ld4(H1 + min<int64_t>(i0 + rr, end - 1) * (2 * H) + d * H + q);
    }
  };
  float4 hv[8];
  if (BGCN_C2_PREFETCH) h1load(wv, hv);
  const int64_t r = S.item_root[item];
  const int rn_all = S.nnz[r];
  const int rn = min(rn_all, kCap);   // root slots in the ELL (the rest spilled)
  const int mh = (rn + 1) / 2;   // root slot pairs (slot 2j + h, j < mh)
  const float sc = keep.scale();
  const int64_t K2 = S.F + H;
  const float* w2t = S.w2t + int64_t(d) * K2 * H;
  // B fill with unconditional loads (clamped slot / column; see k_dh1), selects after
  if (threadIdx.x < kCap)
    rk[threadIdx.x] = threadIdx.x < rn ? uint32_t(H + S.cols[r * kCap + threadIdx.x]) : 0u;
  {   // k < 64: the prologue's split image of W2_d[:, :64] (16-byte copies, 8 per row part)
    static_assert(kC2Ld16 == kW2sLd, "conv2's B rows are the prologue image's rows");
    const __bf16* src = S.w2s + int64_t(d) * 3 * H * kW2sLd;
    for (int e = threadIdx.x; e < 3 * H * 8; e += 256) {
      const int part = e / (H * 8), o = (e / 8) % H, q = (e % 8) * 8;
      *reinterpret_cast<uint4*>(&Bs[part][o * kC2Ld16 + q]) =
          *reinterpret_cast<const uint4*>(src + (int64_t(part) * H + o) * kW2sLd + q);
    }
  }
  for (int e = threadIdx.x; e < kCap * (H / 4); e += 256) {  // root slots (zero past rn)
    const int s = e >> 4, q = (e & 15) * 4;
    const int64_t slot = r * kCap + s;              // always inside the row's ELL list
    const int32_t col = min(max(S.cols[slot], 0), int32_t(S.F - 1));
    const float val = S.vals[slot];
    const float4 w = ld4(w2t + int64_t(H + col) * H + q);
    const float av = s < rn ? sc * fmaxf(val, 0.f) : 0.f;
    const float vv[4] = {av * w.x, av * w.y, av * w.z, av * w.w};
    const int k = H + (s & 1) * (kCap / 2) + (s >> 1);
#pragma unroll
    for (int u = 0; u < 4; ++u) {
      const int o = (q + u) * kC2Ld16 + k;
      split3_bf16(vv[u], Bs[0][o], Bs[1][o], Bs[2][o]);
    }
  }
  __syncthreads();
  BT_MARK(2, 0);

  float* hs = &Hs[wv * 32 * kC2Ld];   // this wave's staged 32 x 64 H1 tile
  auto h1stage = [&](const float4 (&hv)[8]) {
#pragma unroll
    for (int u = 0; u < 8; ++u) {
      const int e = l + 64 * u, rr = e >> 4, q = (e & 15) * 4;
      float* dst = &hs[rr * kC2Ld + q];
      dst[0] = hv[u].x; dst[1] = hv[u].y; dst[2] = hv[u].z; dst[3] = hv[u].w;
    }
    __builtin_amdgcn_s_waitcnt(0xc07f);   // lgkmcnt(0): the wave's LDS writes landed
    __builtin_amdgcn_wave_barrier();
  };
  // the main product of tile t (32 nodes of the item): H1 tile staged through LDS, the
  // dropout-masked relu(H1) and the root keep bits generated in registers, six-product
  // bf16 MFMAs; the root keep masks go to S.rbits
  // (the tile's H1 rows are in the wave's LDS tile already: h1stage)
  auto tile = [&](int t, f32x16& acc0, f32x16& acc1) {
    const int64_t i0 = beg + 32 * t;
    const int64_t i = i0 + r32;
    const bool ok = i < end;
    if (t == wv) BT_MARK(2, 1);
    const float* hrow = &hs[r32 * kC2Ld + 32 * h];
    const uint32_t ni = uint32_t(ok ? i : beg);
    const uint32_t kb = keep.base(ni);   // the node's hash base, shared by its words
    const uint32_t wd = keep.get_b(uint32_t(d), ni, kb, uint32_t(h));
    uint32_t m = 0;
#pragma unroll
    for (int j = 0; j < kCap / 2; ++j) {
      uint32_t bit = 0;
      if (j < mh) {
        const int sl = 2 * j + h;
        const uint32_t k = rk[sl];
        bit = sl < rn ? (keep.get_b(uint32_t(d), ni, kb, k >> 5) >> (k & 31)) & 1u : 0u;
      }
      m |= bit << (2 * j + h);
    }
    acc0 = f32x16{};
    acc1 = f32x16{};
#pragma unroll
    for (int s = 0; s < 4; ++s) {   // H1 columns 32h + 8s + j
      bf16x8 ah, am, al;
#pragma unroll
      for (int j = 0; j < 8; ++j) {
        const int kk = 8 * s + j;
        const float a = ((wd >> kk) & 1u) ? sc * fmaxf(hrow[kk], 0.f) : 0.f;
        __bf16 x, y, z;
        split3_bf16(a, x, y, z);
        ah[j] = x; am[j] = y; al[j] = z;
      }
      const int k = 32 * h + 8 * s;
#pragma unroll
      for (int half = 0; half < 2; ++half) {
        const int o = (32 * half + r32) * kC2Ld16 + k;
        const bf16x8 bh = *reinterpret_cast<const bf16x8*>(&Bs[0][o]);
        const bf16x8 bm = *reinterpret_cast<const bf16x8*>(&Bs[1][o]);
        const bf16x8 bl = *reinterpret_cast<const bf16x8*>(&Bs[2][o]);
        if (half == 0) acc0 = mfma_x6(ah, am, al, bh, bm, bl, acc0);
        else acc1 = mfma_x6(ah, am, al, bh, bm, bl, acc1);
      }
      __builtin_amdgcn_sched_barrier(0);
    }
#pragma unroll
    for (int tt = 0; tt < 2; ++tt) {   // root slots 2(8tt + j) + h
      if (8 * tt < mh) {
        bf16x8 ar;
#pragma unroll
        for (int j = 0; j < 8; ++j) ar[j] = __bf16(((m >> (2 * (8 * tt + j) + h)) & 1u) ? 1.f : 0.f);
        const int k = H + (kCap / 2) * h + 8 * tt;
#pragma unroll
        for (int half = 0; half < 2; ++half) {
          const int o = (32 * half + r32) * kC2Ld16 + k;
          f32x16 c = half == 0 ? acc0 : acc1;
          c = mfma_bf16(ar, *reinterpret_cast<const bf16x8*>(&Bs[2][o]), c);
          c = mfma_bf16(ar, *reinterpret_cast<const bf16x8*>(&Bs[1][o]), c);
          c = mfma_bf16(ar, *reinterpret_cast<const bf16x8*>(&Bs[0][o]), c);
          if (half == 0) acc0 = c; else acc1 = c;
        }
      }
    }
    m |= __shfl_xor(m, 32);
    if (h == 0 && ok) S.rbits[int64_t(d) * S.N + i] = m;
    if (t == wv) BT_MARK(2, 2);
  };
  auto store = [&](int t, const f32x16& acc0, const f32x16& acc1) {
    const int64_t i0 = beg + 32 * t;
#pragma unroll
    for (int q = 0; q < 16; ++q) {
      const int64_t ii = i0 + (q & 3) + 8 * (q >> 2) + 4 * h;
      if (ii < end) {
        Z2[ii * (2 * H) + d * H + r32] = acc0[q];
        Z2[ii * (2 * H) + d * H + 32 + r32] = acc1[q];
      }
    }
  };
  static_assert(kChunk / 32 == 8, "two tiles per wave");
  if (rn_all <= kCap) {
    // tile wv (its H1 rows requested at the start), then tile wv + 4, whose rows are
    // requested as soon as the first tile's are staged: in flight during its products
    if (beg + 32 * wv < end) {
      if (!BGCN_C2_PREFETCH) h1load(wv, hv);
      h1stage(hv);
      if (BGCN_C2_PREFETCH) h1load(wv + 4, hv);
      f32x16 acc0, acc1;
      tile(wv, acc0, acc1);
      store(wv, acc0, acc1);
      if (beg + 32 * (wv + 4) < end) {
        if (!BGCN_C2_PREFETCH) h1load(wv + 4, hv);
        h1stage(hv);
        tile(wv + 4, acc0, acc1);
        store(wv + 4, acc0, acc1);
      }
    }
  } else {
    // The root's spilled non-zeros (a root row of more than kCap words, rare): further
    // [nodes x 32] x [32 x 64] products of the same form as the root slots - A the exact
    // 0/1 keep bits, B = 2 relu(x_root,c) W2_d^T[64 + c] split three ways - 32 pool entries
    // per round, accumulated into the wave's two tiles held in registers (no Z2 round
    // trips), then stored.  Software-pipelined: the pool entries are loaded two rounds
    // ahead and the W2^T rows they select one round ahead, so a round's dependent loads
    // hide behind the previous round's products.
    f32x16 acc[2][2];
#pragma unroll
    for (int j = 0; j < 2; ++j)
      if (beg + 32 * (wv + 4 * j) < end) {
        if (j == 1 || !BGCN_C2_PREFETCH) h1load(wv + 4 * j, hv);
        h1stage(hv);
        tile(wv + 4 * j, acc[j][0], acc[j][1]);
      }
    const int64_t off = S.ovf_off[r];
    const int nsp = rn_all - kCap;
    const int sq0 = threadIdx.x >> 4, sq1 = (threadIdx.x + 256) >> 4, qq = (threadIdx.x & 15) * 4;
    auto ent_at = [&](int c0, int s_) { return S.ovf[off + min(c0 + s_, nsp - 1)]; };
    auto w_of = [&](uint2 e) {
      return ld4(w2t + int64_t(H + min(max(int32_t(e.x), 0), int32_t(S.F - 1))) * H + qq);
    };
    const int tk = min(int(threadIdx.x), kCap - 1);
    uint2 e0 = ent_at(0, sq0), e1 = ent_at(0, sq1), rkc = ent_at(0, tk);
    uint2 n0 = ent_at(kCap, sq0), n1 = ent_at(kCap, sq1), rkn = ent_at(kCap, tk);
    float4 w0 = w_of(e0), w1 = w_of(e1);
    for (int c0 = 0; c0 < nsp; c0 += kCap) {
      const int cn = min(kCap, nsp - c0);
      __syncthreads();   // every wave is done with Bs / rk
      if (threadIdx.x < kCap) rk[threadIdx.x] = uint32_t(H + min(max(int32_t(rkc.x), 0), int32_t(S.F - 1)));
#pragma unroll
      for (int j = 0; j < 2; ++j) {
        const int s_ = j == 0 ? sq0 : sq1;
        const uint2 ent = j == 0 ? e0 : e1;
        const float4 w = j == 0 ? w0 : w1;
        const float av = s_ < cn ? sc * fmaxf(__uint_as_float(ent.y), 0.f) : 0.f;
        const float vv[4] = {av * w.x, av * w.y, av * w.z, av * w.w};
        const int k = H + (s_ & 1) * (kCap / 2) + (s_ >> 1);
#pragma unroll
        for (int u = 0; u < 4; ++u) {
          const int o = (qq + u) * kC2Ld16 + k;
          split3_bf16(vv[u], Bs[0][o], Bs[1][o], Bs[2][o]);
        }
      }
      __syncthreads();
      // the next rounds' loads, in flight during this round's products
      e0 = n0; e1 = n1; rkc = rkn;
      n0 = ent_at(c0 + 2 * kCap, sq0); n1 = ent_at(c0 + 2 * kCap, sq1); rkn = ent_at(c0 + 2 * kCap, tk);
      w0 = w_of(e0); w1 = w_of(e1);
      const int mc = (cn + 1) / 2;
#pragma unroll
      for (int j = 0; j < 2; ++j) {
        const int64_t i0 = beg + 32 * (wv + 4 * j);
        if (i0 >= end) continue;
        const int64_t i = i0 + r32;
        const uint32_t ni = uint32_t(i < end ? i : beg);
        const uint32_t kb = keep.base(ni);
        uint32_t m = 0;
#pragma unroll
        for (int jj = 0; jj < kCap / 2; ++jj) {
          const int sl = 2 * jj + h;
          if (jj < mc && sl < cn) {
            const uint32_t k = rk[sl];
            m |= ((keep.get_b(uint32_t(d), ni, kb, k >> 5) >> (k & 31)) & 1u) << sl;
          }
        }
#pragma unroll
        for (int tt = 0; tt < 2; ++tt) {
          if (8 * tt < mc) {
            bf16x8 ar;
#pragma unroll
            for (int jj = 0; jj < 8; ++jj) ar[jj] = __bf16(((m >> (2 * (8 * tt + jj) + h)) & 1u) ? 1.f : 0.f);
            const int k = H + (kCap / 2) * h + 8 * tt;
#pragma unroll
            for (int half = 0; half < 2; ++half) {
              const int o = (32 * half + r32) * kC2Ld16 + k;
              f32x16 c = acc[j][half];
              c = mfma_bf16(ar, *reinterpret_cast<const bf16x8*>(&Bs[2][o]), c);
              c = mfma_bf16(ar, *reinterpret_cast<const bf16x8*>(&Bs[1][o]), c);
              acc[j][half] = mfma_bf16(ar, *reinterpret_cast<const bf16x8*>(&Bs[0][o]), c);
            }
          }
        }
      }
    }
#pragma unroll
    for (int j = 0; j < 2; ++j)
      if (beg + 32 * (wv + 4 * j) < end) store(wv + 4 * j, acc[j][0], acc[j][1]);
  }
  BT_END(2);
}


// The same conv2 with every wave on ONE 32-node tile: a block takes half a work item
// (tiles 4 half .. 4 half + 3; the second half of an item of <= 128 nodes exits at once), so
// no wave runs two tiles in series (the whole kernel was the fill plus two tiles' products
// on the items of 256 nodes), and each lane loads its H1 A-fragment (row r32, columns
// [32h, 32h + 32) of direction d: eight 16-byte loads, a 128-byte run) straight into
// registers at the kernel's start, under the B fill - no LDS staging of H1 (the block's LDS
// is the B operand only).  BGCN_C2_HALF=0 keeps k_conv2_sparse.
#ifndef BGCN_C2_HALF
#define BGCN_C2_HALF 1
#endif
// 1: conv2_half copies per-tree root images that extra blocks of conv1's launch build (one
// dependent level less in conv2's fill).  Measured (profiles/r05_pass_regs_ab.txt,
// r05_timeline_*_rimg.txt): conv1 alone 15.6 -> 19.5 us for its 2B extra blocks, conv2
// unchanged (20.6 -> 20.2), the step not faster - off.
#ifndef BGCN_C2H_WAVES
#define BGCN_C2H_WAVES 1   // min waves per SIMD (register budget: 5 -> <= 96, beside two waves of the pass)
#endif
#ifndef BGCN_C2H_PREFETCH
#define BGCN_C2H_PREFETCH 1
#endif
#ifndef BGCN_C2_RIMG
#define BGCN_C2_RIMG 0
#endif
__global__ __launch_bounds__(256, BGCN_C2H_WAVES) void k_conv2_half(SparseState S, const float* __restrict__ H1,
                                                    float* __restrict__ Z2, KeepSrc keep) {
  BT_BEGIN
  if (!use_sparse(S)) return;
  const int item = int(blockIdx.x >> 1), half = int(blockIdx.x & 1);
  if (item >= S.tree_item0[S.B]) return;
  __shared__ __attribute__((aligned(16))) __bf16 Bs[3][H * kC2Ld16];   // hi, mid, lo
  __shared__ uint32_t rk[kCap];
  const int d = blockIdx.y;
  const int64_t beg = S.item_beg[item], end = S.item_end[item];
  if (beg + 128 * half >= end) return;               // block-uniform: no tile in this half
  const int wv = threadIdx.x >> 6, l = threadIdx.x & 63, r32 = l & 31, h = l >> 5;
  const int t = 4 * half + wv;
  const int64_t i0 = beg + 32 * t;
  const int64_t i = i0 + r32;
  const bool ok = i < end;
  const bool live = i0 < end;                        // wave-uniform: the wave has a tile
  // this lane's A-fragment rows (clamped: a row past the item reads the item's last row and
  // is masked by `ok`), requested before the fill (BGCN_C2H_PREFETCH) or after it - the
  // latter keeps the 32 registers free during the fill: 114 -> ~84 per wave, so the kernel
  // fits beside two waves of the pass over X (2 x 208 + 96 <= 512) on every CU
  float4 hv[8];
  const float* hsrc = H1 + min<int64_t>(i, end - 1) * (2 * H) + d * H + 32 * h;
  if (BGCN_C2H_PREFETCH) {
#pragma unroll
    for (int u = 0; u < 8; ++u) hv[u] = ld4(hsrc + 4 * u);
  }
  const int64_t r = S.item_root[item];
  const float sc = keep.scale();
  const int64_t K2 = S.F + H;
  const float* w2t = S.w2t + int64_t(d) * K2 * H;
  {
    const __bf16* src = S.w2s + int64_t(d) * 3 * H * kW2sLd;
    for (int e = threadIdx.x; e < 3 * H * 8; e += 256) {
      const int part = e / (H * 8), o = (e / 8) % H, q = (e % 8) * 8;
      *reinterpret_cast<uint4*>(&Bs[part][o * kC2Ld16 + q]) =
          *reinterpret_cast<const uint4*>(src + (int64_t(part) * H + o) * kW2sLd + q);
    }
  }
  int rn_all;
  if (S.rimg_ready) {   // the tree's root image from conv1's launch: one dependent level
    const int b = S.item_tree[item];
    rn_all = S.rinfo[b];
    if (threadIdx.x < kCap) rk[threadIdx.x] = S.rcols[int64_t(b) * kCap + threadIdx.x];
    const __bf16* img = S.rimg + (int64_t(b) * 2 + d) * 3 * H * kCap;
    for (int e = threadIdx.x; e < 3 * H * (kCap / 8); e += 256) {   // 16-byte pieces: 4 per 32-wide row
      const int part = e / (H * 4), o = (e / 4) % H, q = (e % 4) * 8;
      *reinterpret_cast<uint4*>(&Bs[part][o * kC2Ld16 + H + q]) =
          *reinterpret_cast<const uint4*>(img + (int64_t(part) * H + o) * kCap + q);
    }
  } else {
    rn_all = S.nnz[r];
  }
  const int rn = min(rn_all, kCap);
  const int mh = (rn + 1) / 2;
  (void)mh;
  if (!S.rimg_ready && threadIdx.x < kCap)
    rk[threadIdx.x] = threadIdx.x < rn ? uint32_t(H + S.cols[r * kCap + threadIdx.x]) : 0u;
  for (int e = threadIdx.x; !S.rimg_ready && e < kCap * (H / 4); e += 256) {
    const int s = e >> 4, q = (e & 15) * 4;
    const int64_t slot = r * kCap + s;
    const int32_t col = min(max(S.cols[slot], 0), int32_t(S.F - 1));
    const float val = S.vals[slot];
    const float4 w = ld4(w2t + int64_t(H + col) * H + q);
    const float av = s < rn ? sc * fmaxf(val, 0.f) : 0.f;
    const float vv[4] = {av * w.x, av * w.y, av * w.z, av * w.w};
    const int k = H + (s & 1) * (kCap / 2) + (s >> 1);
#pragma unroll
    for (int u = 0; u < 4; ++u) {
      const int o = (q + u) * kC2Ld16 + k;
      split3_bf16(vv[u], Bs[0][o], Bs[1][o], Bs[2][o]);
    }
  }
  __syncthreads();
  BT_MARK(2, 0);
  if (!BGCN_C2H_PREFETCH) {
#pragma unroll
    for (int u = 0; u < 8; ++u) hv[u] = ld4(hsrc + 4 * u);
  }
  // a wave without a tile (the half's last tiles past a short item) computes nothing but
  // stays for the spill rounds' barriers
  const uint32_t ni = uint32_t(ok ? i : beg);
  const uint32_t kb = keep.base(ni);
  f32x16 acc0 = {}, acc1 = {};
  if (live) {
    const uint32_t wd = keep.get_b(uint32_t(d), ni, kb, uint32_t(h));
    const float hf[32] = {hv[0].x, hv[0].y, hv[0].z, hv[0].w, hv[1].x, hv[1].y, hv[1].z, hv[1].w,
                          hv[2].x, hv[2].y, hv[2].z, hv[2].w, hv[3].x, hv[3].y, hv[3].z, hv[3].w,
                          hv[4].x, hv[4].y, hv[4].z, hv[4].w, hv[5].x, hv[5].y, hv[5].z, hv[5].w,
                          hv[6].x, hv[6].y, hv[6].z, hv[6].w, hv[7].x, hv[7].y, hv[7].z, hv[7].w};
#pragma unroll
    for (int s = 0; s < 4; ++s) {   // H1 columns 32h + 8s + j
      bf16x8 ah, am, al;
#pragma unroll
      for (int j = 0; j < 8; ++j) {
        const int kk = 8 * s + j;
        const float a = ((wd >> kk) & 1u) ? sc * fmaxf(hf[kk], 0.f) : 0.f;
        __bf16 x, y, z;
        split3_bf16(a, x, y, z);
        ah[j] = x; am[j] = y; al[j] = z;
      }
      const int k = 32 * h + 8 * s;
#pragma unroll
      for (int hh = 0; hh < 2; ++hh) {
        const int o = (32 * hh + r32) * kC2Ld16 + k;
        const bf16x8 bh = *reinterpret_cast<const bf16x8*>(&Bs[0][o]);
        const bf16x8 bm = *reinterpret_cast<const bf16x8*>(&Bs[1][o]);
        const bf16x8 bl = *reinterpret_cast<const bf16x8*>(&Bs[2][o]);
        if (hh == 0) acc0 = mfma_x6(ah, am, al, bh, bm, bl, acc0);
        else acc1 = mfma_x6(ah, am, al, bh, bm, bl, acc1);
      }
      __builtin_amdgcn_sched_barrier(0);
    }
  }
  if (t == 4 * half) BT_MARK(2, 2);
  // the root slots (exact 0/1 keep bits times the staged root rows, three products); a root
  // row over the ELL cap continues from the spill pool in rounds of kCap entries
  const int64_t off = rn_all > kCap ? S.ovf_off[r] : 0;
  const int nsp = rn_all > kCap ? rn_all - kCap : 0;
  for (int c0 = -kCap; c0 < nsp; c0 += kCap) {
    const int cn = c0 < 0 ? rn : min(kCap, nsp - c0);
    if (c0 >= 0) {   // a spill round: the next kCap pool entries into the root slots
      __syncthreads();   // every wave is done with the previous round's slots (all waves loop alike)
      const int tk = min(int(threadIdx.x), kCap - 1);
      const uint2 ek = S.ovf[off + min(c0 + tk, nsp - 1)];
      if (threadIdx.x < kCap) rk[threadIdx.x] = uint32_t(H + min(max(int32_t(ek.x), 0), int32_t(S.F - 1)));
      for (int e = threadIdx.x; e < kCap * (H / 4); e += 256) {
        const int s = e >> 4, q = (e & 15) * 4;
        const uint2 ent = S.ovf[off + min(c0 + s, nsp - 1)];
        const float4 w = ld4(w2t + int64_t(H + min(max(int32_t(ent.x), 0), int32_t(S.F - 1))) * H + q);
        const float av = s < cn ? sc * fmaxf(__uint_as_float(ent.y), 0.f) : 0.f;
        const float vv[4] = {av * w.x, av * w.y, av * w.z, av * w.w};
        const int k = H + (s & 1) * (kCap / 2) + (s >> 1);
#pragma unroll
        for (int u = 0; u < 4; ++u) {
          const int o = (q + u) * kC2Ld16 + k;
          split3_bf16(vv[u], Bs[0][o], Bs[1][o], Bs[2][o]);
        }
      }
      __syncthreads();
    }
    const int mc = (cn + 1) / 2;
    uint32_t m = 0;
#pragma unroll
    for (int j = 0; j < kCap / 2; ++j) {
      const int sl = 2 * j + h;
      if (j < mc && sl < cn) {
        const uint32_t k = rk[sl];
        m |= ((keep.get_b(uint32_t(d), ni, kb, k >> 5) >> (k & 31)) & 1u) << sl;
      }
    }
#pragma unroll
    for (int tt = 0; tt < 2; ++tt) {
      if (live && 8 * tt < mc) {
        bf16x8 ar;
#pragma unroll
        for (int j = 0; j < 8; ++j) ar[j] = __bf16(((m >> (2 * (8 * tt + j) + h)) & 1u) ? 1.f : 0.f);
        const int k = H + (kCap / 2) * h + 8 * tt;
#pragma unroll
        for (int hh = 0; hh < 2; ++hh) {
          const int o = (32 * hh + r32) * kC2Ld16 + k;
          f32x16 c = hh == 0 ? acc0 : acc1;
          c = mfma_bf16(ar, *reinterpret_cast<const bf16x8*>(&Bs[2][o]), c);
          c = mfma_bf16(ar, *reinterpret_cast<const bf16x8*>(&Bs[1][o]), c);
          c = mfma_bf16(ar, *reinterpret_cast<const bf16x8*>(&Bs[0][o]), c);
          if (hh == 0) acc0 = c; else acc1 = c;
        }
      }
    }
    if (c0 < 0) {   // the ELL slots' keep mask, for the dW2 root columns of the backward
      m |= __shfl_xor(m, 32);
      if (h == 0 && ok) S.rbits[int64_t(d) * S.N + i] = m;
    }
  }
#pragma unroll
  for (int q = 0; q < 16; ++q) {
    const int64_t ii = i0 + (q & 3) + 8 * (q >> 2) + 4 * h;
    if (ii < end) {
      Z2[ii * (2 * H) + d * H + r32] = acc0[q];
      Z2[ii * (2 * H) + d * H + 32 + r32] = acc1[q];
    }
  }
  BT_END(2);
}

// ---------------------------------------------------------------- dW2 root columns, part 1
// Work item = (tree b, chunk of <= kChunk nodes of b), blockIdx.y = direction:
// part[d][item][s][o] = sum_{i in chunk} keep_i[64 + col_s] * dZ2_d[i][o] for the root's
// non-zeros s (the 2 relu(x) factor is applied in k_dw_cols).
// one block: items per tree = ceil(n_b / kChunk), exclusive scan over trees (1024 at a
// time with a carry), then every tree writes its item descriptors.
__device__ inline void items_body(const SparseState& S, const int32_t* __restrict__ tree_ptr,
                                  const int64_t* __restrict__ rootindex) {
  if (S.mode == 1) return;   // (not the overflow flag: the pass over X may run beside this)
  __shared__ int sh[1024];
  __shared__ int carry;
  const int nth = int(blockDim.x);
  if (threadIdx.x == 0) carry = 0;
  __syncthreads();
  for (int64_t b0 = 0; b0 < S.B; b0 += nth) {
    const int64_t b = b0 + threadIdx.x;
    const int t0 = b < S.B ? tree_ptr[b] : 0, t1 = b < S.B ? tree_ptr[b + 1] : 0;
    const int chunks = (t1 - t0 + kChunk - 1) / kChunk;
    sh[threadIdx.x] = chunks;
    __syncthreads();
    for (int o = 1; o < nth; o <<= 1) {
      const int v = threadIdx.x >= o ? sh[threadIdx.x - o] : 0;
      __syncthreads();
      sh[threadIdx.x] += v;
      __syncthreads();
    }
    const int first = carry + sh[threadIdx.x] - chunks;
    if (b < S.B) {
      S.tree_item0[b] = first < S.max_items ? first : S.max_items;
      // the item's node range and root stored with it: its readers skip the tree_ptr /
      // rootindex level of their dependent load chains
      const int64_t r = rootindex[b];
      const int32_t root = int32_t(r >= 0 && r < S.N ? r : 0);
      for (int q = 0; q < chunks && first + q < S.max_items; ++q) {
        S.item_tree[first + q] = int32_t(b);
        S.item_beg[first + q] = t0 + q * kChunk;
        S.item_end[first + q] = min(t0 + (q + 1) * kChunk, t1);
        S.item_root[first + q] = root;
      }
    }
    __syncthreads();
    if (threadIdx.x == nth - 1) carry += sh[nth - 1];
    __syncthreads();
  }
  if (threadIdx.x == 0) S.tree_item0[S.B] = carry < S.max_items ? carry : S.max_items;
}

__global__ __launch_bounds__(1024) void k_items(SparseState S, const int32_t* __restrict__ tree_ptr,
                                                const int64_t* __restrict__ rootindex) {
  items_body(S, tree_ptr, rootindex);
}

// dW2 root-column partials per work item (<= kChunk nodes of one tree), on the MFMA:
//   part[s][o] = sum_{i in item} kept_d(i, s) * dZ2_d[i][o]      (s < 32 root slots)
// a [32 x nodes] x [nodes x 64] product with the 0/1 keep masks of the forward (S.rbits)
// as A.  Each wave takes 64 of the item's nodes (lane half h owns 32 of them: permuted
// K); the four waves' partials are combined in a fixed order.
// Device body, 256 threads: work item `item` of direction d; smem: kRootPartSmem floats.
constexpr int kRootPartSmem = kChunk + 4 * kCap * H;
__device__ inline void root_part_body(const SparseState& S, const float* __restrict__ dZ2,
                                      const int32_t* __restrict__ tree_ptr, int item, int d,
                                      float* smem) {
  if (!use_sparse(S)) return;
  if (item >= S.tree_item0[S.B]) return;
  uint32_t* bits = reinterpret_cast<uint32_t*>(smem);
  float (*red)[kCap * H] = reinterpret_cast<float (*)[kCap * H]>(smem + kChunk);
  const int64_t beg = S.item_beg[item], end = S.item_end[item];
  for (int t = threadIdx.x; t < kChunk; t += 256) {
    const int64_t i = beg + t;
    bits[t] = i < end ? S.rbits[int64_t(d) * S.N + i] : 0u;
  }
  __syncthreads();
  const int wv = threadIdx.x >> 6, l = threadIdx.x & 63, r32 = l & 31, h = l >> 5;
  f32x16 acc0 = {}, acc1 = {};
  if (beg + wv * 64 < end) {
    // bf16 MFMA: A = the 0/1 keep bits (exact in bf16), B = dZ2 split hi + mid + lo
    // (three products: all 24 bits, the fp32-grade dW2 root columns); k-step s takes
    // nodes n0 + 16s + 8h + j
    const int64_t n0 = beg + wv * 64;
#pragma unroll
    for (int s = 0; s < 4; ++s) {
      bf16x8 a, b0h, b0m, b0l, b1h, b1m, b1l;
      float z0[8], z1[8];
#pragma unroll
      for (int j = 0; j < 8; ++j) {
        const int64_t node = n0 + 16 * s + 8 * h + j;
        const float* zr = dZ2 + (node < end ? node : beg) * (2 * H) + d * H;
        z0[j] = zr[r32];
        z1[j] = zr[32 + r32];
      }
#pragma unroll
      for (int j = 0; j < 8; ++j) {
        const int64_t node = n0 + 16 * s + 8 * h + j;
        const bool ok = node < end;
        a[j] = __bf16((ok && ((bits[node - beg] >> r32) & 1u)) ? 1.f : 0.f);
        __bf16 x, y, z;
        split3_bf16(ok ? z0[j] : 0.f, x, y, z);
        b0h[j] = x; b0m[j] = y; b0l[j] = z;
        split3_bf16(ok ? z1[j] : 0.f, x, y, z);
        b1h[j] = x; b1m[j] = y; b1l[j] = z;
      }
      acc0 = mfma_bf16(a, b0l, acc0);
      acc0 = mfma_bf16(a, b0m, acc0);
      acc0 = mfma_bf16(a, b0h, acc0);
      acc1 = mfma_bf16(a, b1l, acc1);
      acc1 = mfma_bf16(a, b1m, acc1);
      acc1 = mfma_bf16(a, b1h, acc1);
    }
  }
#pragma unroll
  for (int q = 0; q < 16; ++q) {
    const int sl = (q & 3) + 8 * (q >> 2) + 4 * h;
    red[wv][sl * H + r32] = acc0[q];
    red[wv][sl * H + 32 + r32] = acc1[q];
  }
  __syncthreads();
  float* out = S.root_part + (int64_t(d) * S.max_items + item) * (kCap * H);
  for (int e = threadIdx.x; e < kCap * H; e += 256)
    out[e] = (red[0][e] + red[1][e]) + (red[2][e] + red[3][e]);
}

// ---------------------------------------------------------------- CSC of X
// Stable counting sort of the non-zeros by column (rows stay in order inside a column):
//   k_csc_hist     per row block (kRowBlock rows, a thread per row): column histogram
//                  in LDS -> hist[r][c]
//   k_csc_prefix   per column: exclusive prefix over the row blocks, column totals
//   k_csc_colscan  one block: column starts/ends = exclusive scan of the totals
//   k_csc_place    per row block: start + the block's prefix, then the rows in order,
//                  32 at a time, rank inside the batch from per-column row bitmasks
// No float atomics, no general sort; deterministic.  Every global load is issued
// unconditionally (clamped index, select afterwards) so the loads of a thread overlap.
// (bodies: kRowBlock threads; hsm / psm = the launch's dynamic shared memory)
// Spilled entries of a group of rows, flattened over the block's threads: pre[r] = the
// group's entries before row r (pre[nrows] = total), off[r] = row r's first pool entry.
// f(r, entry) runs for every entry with four pool loads in flight per thread (a row's
// entries walked by one thread were a serial chain of dependent loads: a 270-word row
// cost the placement ~300 us).
__device__ __forceinline__ int spill_row_of(const int* pre, int nrows, int e) {
  int lo = 0, hi = nrows - 1;   // the last row r with pre[r] <= e (rows of no entries skipped)
  while (lo < hi) {
    const int mid = (lo + hi + 1) >> 1;
    if (pre[mid] <= e) lo = mid; else hi = mid - 1;
  }
  return lo;
}
template <class Fn>
__device__ __forceinline__ void for_spill(const SparseState& S, const int* pre, const int* off, int nrows,
                                          Fn f) {
  const int total = pre[nrows];
  for (int e0 = int(threadIdx.x); e0 < total; e0 += 4 * int(blockDim.x)) {
    int r[4];
    uint2 v[4];
#pragma unroll
    for (int u = 0; u < 4; ++u) {
      const int e = min(e0 + u * int(blockDim.x), total - 1);
      r[u] = spill_row_of(pre, nrows, e);
      v[u] = S.ovf[off[r[u]] + (e - pre[r[u]])];
    }
#pragma unroll
    for (int u = 0; u < 4; ++u)
      if (e0 + u * int(blockDim.x) < total) f(r[u], v[u]);
  }
}

__device__ inline void csc_hist_body(const SparseState& S, int bid, int32_t* hsm) {   // hsm [F]
  if (!use_sparse(S)) return;
  for (int64_t c = threadIdx.x; c < S.F; c += kRowBlock) hsm[c] = 0;
  const int64_t i = int64_t(bid) * kRowBlock + threadIdx.x;
  const int64_t ic = min<int64_t>(i, S.N - 1);
  const int nall = i < S.N ? S.nnz[ic] : 0;
  const int n = min(nall, kCap);
  int32_t cl[kCap];
#pragma unroll
  for (int q = 0; q < kCap / 4; ++q) {
    const int4 v = *reinterpret_cast<const int4*>(S.cols + ic * kCap + 4 * q);
    cl[4 * q] = v.x; cl[4 * q + 1] = v.y; cl[4 * q + 2] = v.z; cl[4 * q + 3] = v.w;
  }
  __syncthreads();
#pragma unroll
  for (int s = 0; s < kCap; ++s)
    if (s < n) atomicAdd(&hsm[cl[s]], 1);
  const int nsp = nall > kCap ? nall - kCap : 0;
  if (__syncthreads_or(nsp)) {   // the block's long rows (rare): their spilled entries
    __shared__ int pre[kRowBlock + 1], off[kRowBlock], wsum[kRowBlock / 64];
    const int lane = threadIdx.x & 63, wv = threadIdx.x >> 6;
    int x = nsp;
#pragma unroll
    for (int o = 1; o < 64; o <<= 1) {
      const int y = __shfl_up(x, o, 64);
      if (lane >= o) x += y;
    }
    if (lane == 63) wsum[wv] = x;
    __syncthreads();
    int base = 0, total = 0;
#pragma unroll
    for (int w = 0; w < kRowBlock / 64; ++w) {
      base += w < wv ? wsum[w] : 0;
      total += wsum[w];
    }
    pre[threadIdx.x] = base + x - nsp;
    off[threadIdx.x] = nsp ? S.ovf_off[ic] : 0;
    if (threadIdx.x == 0) pre[kRowBlock] = total;
    __syncthreads();
    for_spill(S, pre, off, kRowBlock, [&](int, uint2 v) { atomicAdd(&hsm[v.x], 1); });
  }
  __syncthreads();
  int32_t* out = S.hist + int64_t(bid) * S.F;
  for (int64_t c = threadIdx.x; c < S.F; c += kRowBlock) out[c] = hsm[c];
}
__global__ __launch_bounds__(kRowBlock) void k_csc_hist(SparseState S) {
  extern __shared__ __attribute__((aligned(16))) int32_t hsm[];
  csc_hist_body(S, int(blockIdx.x), hsm);
}

// 64 columns x 4 row-block quarters per block; hist[r][c] becomes the exclusive prefix
// of column c over row blocks < r.  Loads in groups of 8 (independent).
// per column: exclusive prefix of the row-block counts.  A 256-thread block takes
// kPrefixCols columns x kPrefixSegs segments of the row blocks (each segment summed, then
// rewritten as prefixes, eight loads in flight); the segment totals are combined in
// segment order.  16 x 16: a Weibo / 1024-node batch has 370-460 row blocks, and with 4
// segments of a column per thread the two passes took ~30 dependent load rounds.
constexpr int kPrefixCols = 16, kPrefixSegs = 256 / kPrefixCols;
__device__ inline void csc_prefix_body(const SparseState& S, int R, int bid) {
  if (!use_sparse(S)) return;
  __shared__ int32_t part[kPrefixSegs][kPrefixCols];
  const int cl = threadIdx.x % kPrefixCols, q = threadIdx.x / kPrefixCols;
  const int64_t c = min<int64_t>(int64_t(bid) * kPrefixCols + cl, S.F - 1);
  const bool live = int64_t(bid) * kPrefixCols + cl < S.F;
  const int rq = (R + kPrefixSegs - 1) / kPrefixSegs, rb = q * rq, re = min(R, rb + rq);
  int32_t sum = 0;
  for (int r0 = rb; r0 < re; r0 += 8) {
    int32_t v[8];
#pragma unroll
    for (int u = 0; u < 8; ++u) v[u] = S.hist[int64_t(max(min(r0 + u, re - 1), 0)) * S.F + c];
#pragma unroll
    for (int u = 0; u < 8; ++u) sum += r0 + u < re ? v[u] : 0;
  }
  part[q][cl] = sum;
  __syncthreads();
  int32_t run = 0;
  for (int qq = 0; qq < q; ++qq) run += part[qq][cl];
  for (int r0 = rb; r0 < re; r0 += 8) {
    int32_t v[8];
#pragma unroll
    for (int u = 0; u < 8; ++u) v[u] = S.hist[int64_t(max(min(r0 + u, re - 1), 0)) * S.F + c];
#pragma unroll
    for (int u = 0; u < 8; ++u) {
      if (live && r0 + u < re) S.hist[int64_t(r0 + u) * S.F + c] = run;
      run += r0 + u < re ? v[u] : 0;
    }
  }
  if (live && q == kPrefixSegs - 1) S.col_total[c] = run;
}
__global__ __launch_bounds__(256) void k_csc_prefix(SparseState S, int R) {
  csc_prefix_body(S, R, int(blockIdx.x));
}

// column starts: exclusive scan of col_total, one 1024-thread block (thread = run of
// consecutive columns, block scan of the run sums)
// (body: any block size >= 256)
__device__ inline void csc_colscan_body(const SparseState& S) {
  if (!use_sparse(S)) return;
  __shared__ int32_t wsum[1024];
  const int64_t F = S.F;
  const int nth = int(blockDim.x);
  const int64_t per = (F + nth - 1) / nth;
  const int64_t c0 = threadIdx.x * per;
  constexpr int kMaxPer = kSparseMaxF / 256;
  int32_t v[kMaxPer];
  int32_t local = 0;
#pragma unroll
  for (int k = 0; k < kMaxPer; ++k) {
    const int64_t c = c0 + k;
    v[k] = (k < per && c < F) ? S.col_total[min<int64_t>(c, F - 1)] : 0;
    local += v[k];
  }
  wsum[threadIdx.x] = local;
  __syncthreads();
  for (int o = 1; o < nth; o <<= 1) {
    const int32_t t = threadIdx.x >= o ? wsum[threadIdx.x - o] : 0;
    __syncthreads();
    wsum[threadIdx.x] += t;
    __syncthreads();
  }
  int32_t run = wsum[threadIdx.x] - local;
#pragma unroll
  for (int k = 0; k < kMaxPer; ++k) {
    const int64_t c = c0 + k;
    if (k < per && c < F) {
      S.col_start[c] = run;
      S.col_end[c] = run + v[k];
    }
    run += v[k];
  }
}

__global__ __launch_bounds__(1024) void k_csc_colscan(SparseState S) { csc_colscan_body(S); }

// Row block of a placement block: the blocks of one XCD (block ids equal mod 8 - the
// dispatcher hands blocks to the XCDs round-robin) take consecutive row blocks, whose
// entries of a column are adjacent in the CSC, so a line of it is mostly written from one
// XCD's L2 instead of from all eight (the placement's stores are scattered by column).
__device__ inline void csc_place_body(const SparseState& S, int bid, int32_t* psm) {
  if (!use_sparse(S)) return;   // psm: [F] counters, [F] row masks
  bid = xcd_contig(bid, int((S.N + kRowBlock - 1) / kRowBlock));
  int32_t* cnt = psm;
  uint32_t* rows = reinterpret_cast<uint32_t*>(psm + S.F);
  const int64_t F = S.F;
  const int32_t* pre = S.hist + int64_t(bid) * F;
  for (int64_t c0 = threadIdx.x; c0 < F; c0 += 4 * 256) {
    int32_t st[4], pr[4];
#pragma unroll
    for (int u = 0; u < 4; ++u) {
      const int64_t c = min<int64_t>(c0 + 256 * u, F - 1);
      st[u] = S.col_start[c];
      pr[u] = pre[c];
    }
#pragma unroll
    for (int u = 0; u < 4; ++u) {
      const int64_t c = c0 + 256 * u;
      if (c < F) {
        cnt[c] = st[u] + pr[u];
        rows[c] = 0u;
      }
    }
  }
  // all of the block's entries up front: thread t holds entries t + 256k (k < 32) of
  // the row block = slot t % 32 of rows (t / 32) + 8k
  const int64_t r0 = int64_t(bid) * kRowBlock;
  const int s = threadIdx.x % kCap;
  constexpr int kPer = kRowBlock * kCap / 256;   // 32
  int32_t col[kPer], nn[kPer];
  float val[kPer];
  uint32_t rootbits = 0u;   // bit k: row of entry k is a tree root
#pragma unroll
  for (int k = 0; k < kPer; ++k) {   // issue all loads first ...
    const int64_t ic = min<int64_t>(r0 + threadIdx.x / kCap + 8 * k, S.N - 1);
    nn[k] = S.nnz[ic];
    col[k] = S.cols[ic * kCap + s];
    val[k] = S.vals[ic * kCap + s];
    rootbits |= uint32_t(S.root_map[ic] == int32_t(ic)) << k;
  }
  uint32_t smask = 0u;   // bit bt: batch bt (rows 32bt .. 32bt + 31) holds a long row
#pragma unroll
  for (int k = 0; k < kPer; ++k) {   // ... then mask the padding slots
    const int64_t i = r0 + threadIdx.x / kCap + 8 * k;
    col[k] = (i < S.N && s < nn[k]) ? col[k] : -1;
    smask |= (i < S.N && nn[k] > kCap) ? (1u << (k / 4)) : 0u;
  }
  // The block's long rows (rare): their spilled entries are indexed once for the whole
  // block - rpre[t] = the block's spilled entries before row t (a block-wide scan), rslot /
  // roff per row - and staged in LDS (up to kPlaceStage of them; beyond, read from the pool
  // in place), so a batch's passes over them need no dependent global loads.
  constexpr int kPlaceStage = 1024;
  __shared__ int rpre[kRowBlock + 1], roff[kRowBlock], wsum[kRowBlock / 64];
  __shared__ uint32_t rslot[kRowBlock];
  __shared__ uint2 sbuf[kPlaceStage];
  __shared__ uint32_t smask_s;
  if (threadIdx.x == 0) smask_s = 0u;
  __syncthreads();
  if (smask) atomicOr(&smask_s, smask);
  __syncthreads();
  smask = smask_s;
  bool staged = true;
  if (smask) {
    const int t = threadIdx.x, lane = t & 63, wv = t >> 6;
    const int64_t i = r0 + t;
    const int na = i < S.N ? S.nnz[i] : 0;
    const int nsp = na > kCap ? na - kCap : 0;
    const int o = nsp ? S.ovf_off[i] : 0;
    const uint32_t sl = nsp ? (uint32_t(i * kCap) | kCscSpillFlag | (S.root_map[i] == int32_t(i) ? kCscRootFlag : 0u))
                            : 0u;
    int x = nsp;
#pragma unroll
    for (int d = 1; d < 64; d <<= 1) {
      const int y = __shfl_up(x, d, 64);
      if (lane >= d) x += y;
    }
    if (lane == 63) wsum[wv] = x;
    __syncthreads();
    int base = 0, total = 0;
#pragma unroll
    for (int w = 0; w < kRowBlock / 64; ++w) {
      base += w < wv ? wsum[w] : 0;
      total += wsum[w];
    }
    rpre[t] = base + x - nsp;
    roff[t] = o;
    rslot[t] = sl;
    if (t == 0) rpre[kRowBlock] = total;
    staged = total <= kPlaceStage;
    __syncthreads();
    if (staged) {
      for (int e0 = t; e0 < total; e0 += 4 * kRowBlock) {   // four pool loads in flight
        uint2 v[4];
#pragma unroll
        for (int u = 0; u < 4; ++u) {
          const int e = min(e0 + u * kRowBlock, total - 1);
          const int r = spill_row_of(rpre, kRowBlock, e);
          v[u] = S.ovf[roff[r] + (e - rpre[r])];
        }
#pragma unroll
        for (int u = 0; u < 4; ++u)
          if (e0 + u * kRowBlock < total) sbuf[e0 + u * kRowBlock] = v[u];
      }
    }
    __syncthreads();
  }
  // f(row within the batch, entry, block row) for every spilled entry of batch bt
  auto batch_spill = [&](int bt, auto f) {
    const int lo0 = bt * 32, e1 = rpre[lo0 + 32];
    for (int e = rpre[lo0] + int(threadIdx.x); e < e1; e += int(blockDim.x)) {
      int lo = lo0, hi = lo0 + 31;   // the last row with rpre <= e
      while (lo < hi) {
        const int mid = (lo + hi + 1) >> 1;
        if (rpre[mid] <= e) lo = mid; else hi = mid - 1;
      }
      const uint2 v = staged ? sbuf[e] : S.ovf[roff[lo] + (e - rpre[lo])];
      f(lo - lo0, v, lo);
    }
  };
  // rows of the block in order, 32 rows (= 1024 slots, 4 per thread) per batch.  The
  // columns of one row are distinct, so an entry's rank among the batch's entries of
  // its column = the number of earlier batch rows holding that column: an OR of row
  // bits per column (order-independent) + popcount.
  constexpr int kBatchRows = 32;
#pragma unroll
  for (int bt = 0; bt < kRowBlock / kBatchRows; ++bt) {
    int rr[4], rank[4];
    const bool spill = (smask >> bt) & 1u;
#pragma unroll
    for (int k = 0; k < 4; ++k) {
      rr[k] = threadIdx.x / kCap + 8 * k;   // row within the batch
      const int32_t cc = col[4 * bt + k];
      if (cc >= 0) atomicOr(&rows[cc], 1u << rr[k]);
    }
    // spilled entries of the batch's rows (their columns are distinct from the row's ELL
    // columns, so the same row-bit ranks hold), flattened over the block's threads
    if (spill) batch_spill(bt, [&](int r, uint2 v, int) { atomicOr(&rows[v.x], 1u << r); });
    __syncthreads();
#pragma unroll
    for (int k = 0; k < 4; ++k) {
      const int32_t cc = col[4 * bt + k];
      rank[k] = -1;
      if (cc >= 0) {
        const uint32_t m = rows[cc];
        rank[k] = __popc(m & ((1u << rr[k]) - 1u));
        const int64_t i = r0 + bt * kBatchRows + rr[k];
        const uint32_t flag = ((rootbits >> (4 * bt + k)) & 1u) ? kCscRootFlag : 0u;
        S.csc[cnt[cc] + rank[k]] = make_uint2(uint32_t(i * kCap + s) | flag, __float_as_uint(val[4 * bt + k]));
      }
    }
    if (spill)
      batch_spill(bt, [&](int r, uint2 v, int br) {
        S.csc[cnt[v.x] + __popc(rows[v.x] & ((1u << r) - 1u))] = make_uint2(rslot[br], v.y);
      });
    __syncthreads();
    if (!spill) {
#pragma unroll
      for (int k = 0; k < 4; ++k) {
        const int32_t cc = col[4 * bt + k];
        if (rank[k] == 0) {   // the batch's first entry of a column advances its counter
          cnt[cc] += __popc(rows[cc]);
          rows[cc] = 0u;
        }
      }
    } else {   // two phases: the counters (row bits read-only), then the clears
#pragma unroll
      for (int k = 0; k < 4; ++k)
        if (rank[k] == 0) cnt[col[4 * bt + k]] += __popc(rows[col[4 * bt + k]]);
      batch_spill(bt, [&](int r, uint2 v, int) {
        if ((rows[v.x] & ((1u << r) - 1u)) == 0u) cnt[v.x] += __popc(rows[v.x]);
      });
      __syncthreads();
#pragma unroll
      for (int k = 0; k < 4; ++k)
        if (rank[k] >= 0) rows[col[4 * bt + k]] = 0u;
      batch_spill(bt, [&](int, uint2 v, int) { rows[v.x] = 0u; });
    }
    __syncthreads();
  }
}
__global__ __launch_bounds__(256) void k_csc_place(SparseState S) {
  extern __shared__ __attribute__((aligned(16))) int32_t psm[];
  csc_place_body(S, int(blockIdx.x), psm);
}

// dW1 = [dZ1_td | dZ1_bu]^T X over the CSC of X: four waves per column (four columns per
// block), each lane owning 2 of the 128 outputs; wave k of a column takes the column's
// 64-entry batches k, k + 4, ... (slot and value loaded side by side: k_csc_place stores
// the value next to the slot), then issues the dZ1 row gathers kDw1Depth at a time with
// clamped indices; (row, value) reach the wave by scalar readlane.  The four partials are
// combined in LDS in wave order (deterministic).  One wave per column leaves the chip with
// F = 5000 waves, each walking its whole column serially: fine at Twitter size (~70
// entries per column; the split measured 14 us slower there), slow at Weibo size (~225).
constexpr int kDw1Depth = 16;
// Device body, 1024 threads, column block bid; smem: kDw1Smem floats.
constexpr int kDw1Smem = 2 * 2 * H * 17;   // dW1 and the dW2 root-column partials
// Spilled root entries (a root row of more than kCap words): their dW2 root-column
// partial is summed over the tree's nodes directly (no ELL slot, no item partial):
//   sum_{i in tree b} keep_d(i, 64 + c) * dZ2_d[i][o]
__device__ __forceinline__ void tree_range(const SparseState& S, int b, int64_t& nb, int64_t& ne) {
  const int it0 = S.tree_item0[b], it1 = S.tree_item0[b + 1];
  nb = it1 > it0 ? S.item_beg[it0] : 0;
  ne = it1 > it0 ? S.item_end[it1 - 1] : 0;
}

// kPart: 0 = dW1 and the dW2 root columns, 1 = the dW2 root columns only (no dZ1
// gathers, dW1 untouched: the deferred-dW1 step's tail A), 2 = dW1 only.
template <int kDw1Split, int kPart = 0>                       // waves per column (1 or 4)
__device__ inline void dw1_body(const SparseState& S, const float* __restrict__ dZ1,
                                float* __restrict__ dw1_td, float* __restrict__ dw1_bu,
                                const int64_t* __restrict__ batch, float* __restrict__ dw2_td,
                                float* __restrict__ dw2_bu, float scale, int bid, float* smem,
                                const float* __restrict__ dZ2, const KeepSrc& keep) {
  const int kDw1Cols = int(blockDim.x >> 6) / kDw1Split;   // columns per block
  if (!use_sparse(S)) return;
  float (*t1)[17] = reinterpret_cast<float (*)[17]>(smem);
  float (*t2)[17] = reinterpret_cast<float (*)[17]>(smem + 2 * H * 17);
  const int wave = threadIdx.x >> 6, lane = threadIdx.x & 63;
  const int part = wave % kDw1Split;
  const int64_t F = S.F;
  const int64_t c = int64_t(bid) * kDw1Cols + wave / kDw1Split;
  const int rd = lane >> 5, ro = (2 * lane) & (H - 1);   // this lane's (direction, output pair)
  float2 a1 = make_float2(0.f, 0.f), a2 = make_float2(0.f, 0.f);
  if (c < F) {
    const int64_t beg = S.col_start[c], end = S.col_end[c];
    for (int64_t u0 = beg + 64 * part; u0 < end; u0 += 64 * kDw1Split) {
      const int64_t u = min<int64_t>(u0 + lane, end - 1);   // clamped: duplicates, x masked
      const uint2 ent = S.csc[u];
      const uint32_t slot = ent.x & kCscSlotMask;
      const float xv = __uint_as_float(ent.y);
      const int n = int(min<int64_t>(64, end - u0));
      const float x_l = lane < n ? xv : 0.f;
      const int32_t i_l = int32_t(slot / kCap);
      for (int j0 = 0; j0 < (kPart == 1 ? 0 : n); j0 += kDw1Depth) {
        float2 gv[kDw1Depth];
        float x[kDw1Depth];
#pragma unroll
        for (int v = 0; v < kDw1Depth; ++v) {
          const int j = j0 + v < n ? j0 + v : n - 1;   // wave-uniform: scalar broadcast
          const int32_t i = __builtin_amdgcn_readlane(i_l, j);
          x[v] = j0 + v < n ? __int_as_float(__builtin_amdgcn_readlane(__float_as_int(x_l), j)) : 0.f;
          gv[v] = *reinterpret_cast<const float2*>(dZ1 + int64_t(i) * (2 * H) + 2 * lane);
        }
#pragma unroll
        for (int v = 0; v < kDw1Depth; ++v) {
          a1.x = fmaf(x[v], gv[v].x, a1.x);
          a1.y = fmaf(x[v], gv[v].y, a1.y);
        }
      }
      // dW2 root columns: dW2_d[:, 64 + c] = sum over the root rows holding column c (tree
      // order = CSC row order) of 2 relu(x) * sum_items root_part[d][item][slot] - the
      // root entries (rare) are flagged in the CSC record, so this pass over the column
      // finds them (a separate role re-read every column and gathered node_root per entry)
      uint64_t m = kPart == 2 ? 0ull : __ballot(lane < n && (ent.x & kCscRootFlag));
      while (m) {   // in row (= tree) order
        const int j = __builtin_ctzll(m);
        m &= m - 1;
        const int32_t i = __builtin_amdgcn_readlane(i_l, j);     // j is wave-uniform
        const int32_t sl = int32_t(__builtin_amdgcn_readlane(int32_t(slot), j) % kCap);
        const float f = scale * fmaxf(__int_as_float(__builtin_amdgcn_readlane(__float_as_int(x_l), j)), 0.f);
        const int b = int(batch[i]);
        float2 sum = make_float2(0.f, 0.f);
        if (__builtin_amdgcn_readlane(int32_t(ent.x), j) & int32_t(kCscSpillFlag)) {
          int64_t nb, ne;
          tree_range(S, b, nb, ne);
          const uint32_t k = uint32_t(H + c);
          for (int64_t n0 = nb; n0 < ne; n0 += 4) {   // four rows in flight, in node order
            float2 z[4];
            uint32_t kw[4];
#pragma unroll
            for (int u = 0; u < 4; ++u) {
              const int64_t nd = min(n0 + u, ne - 1);
              z[u] = *reinterpret_cast<const float2*>(dZ2 + nd * (2 * H) + rd * H + ro);
              kw[u] = keep.get(uint32_t(rd), uint32_t(nd), k >> 5);
            }
#pragma unroll
            for (int u = 0; u < 4; ++u)
              if (n0 + u < ne && ((kw[u] >> (k & 31)) & 1u)) {
                sum.x += z[u].x;
                sum.y += z[u].y;
              }
          }
          a2.x = fmaf(f, sum.x, a2.x);
          a2.y = fmaf(f, sum.y, a2.y);
          continue;
        }
        const int it0 = S.tree_item0[b], it1 = S.tree_item0[b + 1];
        for (int it = it0; it < it1; it += 4) {   // four item partials in flight, in item order
          float2 v[4];
#pragma unroll
          for (int q = 0; q < 4; ++q)
            v[q] = *reinterpret_cast<const float2*>(
                S.root_part + (int64_t(rd) * S.max_items + min(it + q, it1 - 1)) * (kCap * H) + sl * H + ro);
#pragma unroll
          for (int q = 0; q < 4; ++q)
            if (it + q < it1) {
              sum.x += v[q].x;
              sum.y += v[q].y;
            }
        }
        a2.x = fmaf(f, sum.x, a2.x);
        a2.y = fmaf(f, sum.y, a2.y);
      }
    }
  }
  t1[2 * lane][wave] = a1.x;
  t1[2 * lane + 1][wave] = a1.y;
  t2[2 * lane][wave] = a2.x;
  t2[2 * lane + 1][wave] = a2.y;
  __syncthreads();
  // combine the column's partials in wave order, then store (kDw1Cols consecutive columns
  // per output row); every root column is written (zero when no root holds it)
  const int tx = threadIdx.x % kDw1Cols;
  const int64_t cc = int64_t(bid) * kDw1Cols + tx;
  const int64_t K2 = F + H;
  for (int ty = threadIdx.x / kDw1Cols; ty < 2 * H && cc < F; ty += int(blockDim.x) / kDw1Cols) {
    float acc = t1[ty][tx * kDw1Split], acc2 = t2[ty][tx * kDw1Split];
#pragma unroll
    for (int k = 1; k < kDw1Split; ++k) {
      acc += t1[ty][tx * kDw1Split + k];
      acc2 += t2[ty][tx * kDw1Split + k];
    }
    float* dst = ty < H ? dw1_td + int64_t(ty) * F : dw1_bu + int64_t(ty - H) * F;
    if (kPart != 1) dst[cc] = acc;
    float* dst2 = ty < H ? dw2_td + int64_t(ty) * K2 : dw2_bu + int64_t(ty - H) * K2;
    if (kPart != 2) dst2[H + cc] = acc2;
  }
}

// dW1 by output slices, XCD-aware (the default form).  The 128-wide dZ1 row splits into
// kSlices slices of kSliceW outputs; the blocks of XCD x (blocks are dispatched to the
// XCDs round-robin: block b runs on XCD b % 8) take slice x % kSlices of every column of
// their column groups, so an XCD's L2 serves the gathers of ONE slice of dZ1 - N x 128 B
// (3.9 MB at Twitter size) instead of the whole 15.7 MB table, most of which the
// column-per-wave form fetched from the Infinity Cache (PMC: 140 MB per launch, the
// fabric-bound ~7 TB/s).  A wave takes one (column, slice): kSliceGroups entries per
// gather instruction (kSliceLanes lanes x 16 B per entry), kSliceDepth rounds in flight;
// the lane groups' partials are combined by a fixed xor-shuffle tree (deterministic).  The
// dW2 root columns ride along as in dw1_body (same per-output order, same values).
#ifndef BGCN_DW1_SLICES
#define BGCN_DW1_SLICES 4
#endif
#ifndef BGCN_DW1_DEPTH
#define BGCN_DW1_DEPTH 4
#endif
constexpr int kSlices = BGCN_DW1_SLICES;
constexpr int kSliceW = 2 * H / kSlices;          // outputs per slice
constexpr int kSliceLanes = kSliceW / 4;          // lanes per entry (one float4 each)
constexpr int kSliceGroups = 64 / kSliceLanes;    // entries per gather instruction
constexpr int kSliceDepth = BGCN_DW1_DEPTH;
#ifndef BGCN_DW1_CSC_PF
#define BGCN_DW1_CSC_PF 1
#endif
constexpr bool kDw1CscPf = BGCN_DW1_CSC_PF != 0;
static_assert(8 % kSlices == 0 && kSliceW <= H && kSliceLanes >= 1, "slices");
__device__ __forceinline__ float4 shfl4(float4 v, int src) {
  return make_float4(__shfl(v.x, src, 64), __shfl(v.y, src, 64), __shfl(v.z, src, 64), __shfl(v.w, src, 64));
}
__device__ __forceinline__ float4 shfl_xor4(float4 v, int m) {
  return make_float4(__shfl_xor(v.x, m, 64), __shfl_xor(v.y, m, 64), __shfl_xor(v.z, m, 64),
                     __shfl_xor(v.w, m, 64));
}
// blocks of the sliced form for F columns with W waves (= columns) per block
__host__ __device__ inline int dw1_sliced_blocks(int64_t F, int W) {
  const int64_t groups = (F + W - 1) / W, reps = 8 / kSlices;
  return int(8 * ((groups + reps - 1) / reps));
}
// rows in flight per lane group in the spilled-root sweep (rare): 1 keeps the launch at 64
// VGPRs, 8 dW1 waves per SIMD (4: 80 VGPRs, 6 waves; twitter15 +1 %,
// profiles/r03_tail_depth_ab.txt)
#ifndef BGCN_SPILL_DEPTH
#define BGCN_SPILL_DEPTH 1
#endif
constexpr int kSpillDepth = BGCN_SPILL_DEPTH;
template <int kPart = 0>   // 0: dW1 + the dW2 root columns, 2: dW1 only (see dw1_body)
__device__ inline void dw1_sliced_body(const SparseState& S, const float* __restrict__ dZ1,
                                       float* __restrict__ dw1_td, float* __restrict__ dw1_bu,
                                       const int64_t* __restrict__ batch, float* __restrict__ dw2_td,
                                       float* __restrict__ dw2_bu, float scale, int bid, float* smem,
                                       const float* __restrict__ dZ2, const KeepSrc& keep,
                                       const TailAdam* ad = nullptr) {
  if (!use_sparse(S)) return;
  const int W = int(blockDim.x >> 6);
  const int64_t F = S.F;
  const int x = bid & 7, sl_ = x % kSlices;
  const int64_t cg = int64_t(bid >> 3) * (8 / kSlices) + x / kSlices;
  const int wave = threadIdx.x >> 6, lane = threadIdx.x & 63;
  const int g = lane / kSliceLanes, q = lane % kSliceLanes;
  const int so = kSliceW * sl_, d = so / H, oo = so % H + 4 * q;   // slice start, direction, my outputs
  const int64_t c = cg * W + wave;
  // the fused optimiser step (TailAdam, kPart 0): this block's kSliceW outputs x W columns of
  // W1_d and of W2_d's root columns - their parameters and moments requested here, beside
  // the gathers, and updated with the finished gradients at the end
  const bool fa = kPart == 0 && ad && ad->on && int(threadIdx.x) < kSliceW * W && !ad->skip();
  const int ka1 = d == 0 ? 0 : 4, ka2 = d == 0 ? 2 : 6;
  const int a_ol = int(threadIdx.x) / W, a_tx = int(threadIdx.x) % W;
  const int64_t a_cc = min<int64_t>(cg * W + a_tx, F - 1);
  const int64_t ia1 = int64_t(so % H + a_ol) * F + a_cc, ia2 = int64_t(so % H + a_ol) * (F + H) + H + a_cc;
  float ap1 = 0.f, am1 = 0.f, av1 = 0.f, ap2 = 0.f, am2 = 0.f, av2 = 0.f;
  if (fa) {
    ap1 = ad->p[ka1][ia1]; am1 = ad->m[ka1][ia1]; av1 = ad->v[ka1][ia1];
    ap2 = ad->p[ka2][ia2]; am2 = ad->m[ka2][ia2]; av2 = ad->v[ka2][ia2];
  }
  float4 a1 = f4zero(), a2 = f4zero();
  bool spill_root = false;
  if (c < F) {
    const int64_t beg = S.col_start[c], end = S.col_end[c];
    // the next 64 CSC entries are requested before this chunk's gathers (BGCN_DW1_CSC_PF):
    // loads retire in order, so they cost no wait, and the chunk loop then takes one
    // dependent round trip less per 64 entries
    // (32-bit entry indices: the CSC holds fewer than 2^31 entries, kSparseMaxN)
    const int32_t be = int32_t(beg), en = int32_t(end);
    uint2 ent_nx = be < en ? S.csc[min(be + lane, en - 1)] : make_uint2(0u, 0u);
    for (int32_t u0 = be; u0 < en; u0 += 64) {
      uint2 ent;
      if constexpr (kDw1CscPf) {
        ent = ent_nx;
        if (u0 + 64 < en) ent_nx = S.csc[min(u0 + 64 + lane, en - 1)];
      } else {
        ent = S.csc[min(u0 + lane, en - 1)];   // clamped: duplicates, x masked
      }
      const uint32_t slot = ent.x & kCscSlotMask;
      const int n = min(64, en - u0);
      const float x_l = lane < n ? __uint_as_float(ent.y) : 0.f;
      const int32_t i_l = int32_t(slot / kCap);
      for (int j0 = 0; j0 < n; j0 += kSliceGroups * kSliceDepth) {
        float4 gv[kSliceDepth];
        float xx[kSliceDepth];
#pragma unroll
        for (int v = 0; v < kSliceDepth; ++v) {
          const int j = j0 + v * kSliceGroups + g;
          const int jc = j < n ? j : n - 1;
          const int32_t i = __shfl(i_l, jc, 64);
          const float xv = __shfl(x_l, jc, 64);
          xx[v] = j < n ? xv : 0.f;
          gv[v] = ld4(dZ1 + int64_t(i) * (2 * H) + so + 4 * q);
        }
#pragma unroll
        for (int v = 0; v < kSliceDepth; ++v) a1 = f4fma(xx[v], gv[v], a1);
      }
      uint64_t m = kPart == 2 ? 0ull : __ballot(lane < n && (ent.x & kCscRootFlag));
      while (m) {   // root entries, in row (= tree) order; lane group 0 holds the slice
        const int j = __builtin_ctzll(m);
        m &= m - 1;
        const int32_t i = __builtin_amdgcn_readlane(i_l, j);
        const int32_t sl = int32_t(__builtin_amdgcn_readlane(int32_t(slot), j) % kCap);
        const float f = scale * fmaxf(__int_as_float(__builtin_amdgcn_readlane(__float_as_int(x_l), j)), 0.f);
        if (__builtin_amdgcn_readlane(int32_t(ent.x), j) & int32_t(kCscSpillFlag)) {
          spill_root = true;   // summed after the column's main pass (its registers are free then)
          continue;
        }
        if (g != 0) continue;
        const int b = int(batch[i]);
        float4 sum = f4zero();
        const int it0 = S.tree_item0[b], it1 = S.tree_item0[b + 1];
        for (int it = it0; it < it1; it += 4) {   // four item partials in flight, in item order
          float4 v[4];
#pragma unroll
          for (int qq = 0; qq < 4; ++qq)
            v[qq] = ld4(S.root_part + (int64_t(d) * S.max_items + min(it + qq, it1 - 1)) * (kCap * H) + sl * H + oo);
#pragma unroll
          for (int qq = 0; qq < 4; ++qq)
            if (it + qq < it1) sum = f4add(sum, v[qq]);
        }
        a2 = f4fma(f, sum, a2);
      }
    }
    if (spill_root) {
      // the column's spilled root entries (a root row of more than kCap words, rare), in
      // row order: sum_{i in tree} keep_d(i, 64 + c) * dZ2_d[i] - lane group g takes the
      // tree's nodes g, g + 8, ..., the groups' partials combined by the fixed xor tree
      const uint32_t k = uint32_t(H + c);
      for (int64_t u0 = beg; u0 < end; u0 += 64) {
        const int64_t u = min<int64_t>(u0 + lane, end - 1);
        const uint2 ent = S.csc[u];
        const int n = int(min<int64_t>(64, end - u0));
        uint64_t m = __ballot(lane < n && (ent.x & kCscRootFlag) && (ent.x & kCscSpillFlag));
        while (m) {
          const int j = __builtin_ctzll(m);
          m &= m - 1;
          const int32_t i = int32_t((uint32_t(__builtin_amdgcn_readlane(int32_t(ent.x), j)) & kCscSlotMask) / kCap);
          const float f = scale * fmaxf(__int_as_float(__builtin_amdgcn_readlane(int32_t(ent.y), j)), 0.f);
          int64_t nb, ne;
          tree_range(S, int(batch[i]), nb, ne);
          float4 sum = f4zero();
          for (int64_t n0 = nb + g; n0 < ne; n0 += kSpillDepth * kSliceGroups) {   // rows in flight
            float4 z[kSpillDepth];
            uint32_t kw[kSpillDepth];
#pragma unroll
            for (int v = 0; v < kSpillDepth; ++v) {
              const int64_t nd = min(n0 + v * kSliceGroups, ne - 1);
              z[v] = ld4(dZ2 + nd * (2 * H) + d * H + oo);
              kw[v] = keep.get(uint32_t(d), uint32_t(nd), k >> 5);
            }
#pragma unroll
            for (int v = 0; v < kSpillDepth; ++v)
              if (n0 + v * kSliceGroups < ne && ((kw[v] >> (k & 31)) & 1u)) sum = f4add(sum, z[v]);
          }
#pragma unroll
          for (int off = kSliceLanes; off < 64; off <<= 1) sum = f4add(sum, shfl_xor4(sum, off));
          if (g == 0) a2 = f4fma(f, sum, a2);
        }
      }
    }
  }
#pragma unroll
  for (int off = kSliceLanes; off < 64; off <<= 1) a1 = f4add(a1, shfl_xor4(a1, off));
  float* t1 = smem;                                 // [kSliceW][W + 1]
  float* t2 = smem + kSliceW * (W + 1);
  if (g == 0) {
    const float v1[4] = {a1.x, a1.y, a1.z, a1.w}, v2[4] = {a2.x, a2.y, a2.z, a2.w};
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      t1[(4 * q + j) * (W + 1) + wave] = v1[j];
      t2[(4 * q + j) * (W + 1) + wave] = v2[j];
    }
  }
  __syncthreads();
  const int64_t K2 = F + H;
  float* w1 = d == 0 ? dw1_td : dw1_bu;
  float* w2 = d == 0 ? dw2_td : dw2_bu;
  for (int e = threadIdx.x; e < kSliceW * W; e += int(blockDim.x)) {
    const int ol = e / W, tx = e % W;
    const int64_t cc = cg * W + tx;
    if (cc >= F) continue;
    const int o = so % H + ol;
    const float g1 = t1[ol * (W + 1) + tx], g2 = t2[ol * (W + 1) + tx];
    w1[int64_t(o) * F + cc] = g1;
    if (kPart != 2) w2[int64_t(o) * K2 + H + cc] = g2;
    if (fa && e == int(threadIdx.x)) {   // (this thread's prefetched pair: a_ol == ol, a_cc == cc)
      adam_elem(ap1, g1, am1, av1, ad->c(ka1));
      ad->p[ka1][ia1] = ap1; ad->m[ka1][ia1] = am1; ad->v[ka1][ia1] = av1;
      adam_elem(ap2, g2, am2, av2, ad->c(ka2));
      ad->p[ka2][ia2] = ap2; ad->m[ka2][ia2] = am2; ad->v[ka2][ia2] = av2;
      if (ad->w1t) {
        ad->w1t[cc * (2 * H) + d * H + o] = ap1;                 // W1^T[c][d*64 + o]
        ad->w2t[(int64_t(d) * K2 + H + cc) * H + o] = ap2;       // W2^T_d[64 + c][o]
      }
    }
  }
}

// The fused optimiser step's parameters without a tail role of their own (b2: the middle
// launch's db2; the head's fc weight and bias), one extra block of the tail launch; it also
// counts a skipped update as k_adam does.
__device__ inline void tail_adam_block(const TailAdam& ad) {
  if (ad.skip()) {
    if (threadIdx.x == 0 && ad.skip_count) atomicAdd(ad.skip_count, 1);
    return;
  }
  const int ks[4] = {3, 7, 8, 9};
#pragma unroll
  for (int q = 0; q < 4; ++q) {
    const int k = ks[q];
    const AdamConst c = ad.c(k);
    for (int64_t e = threadIdx.x; e < ad.n[k]; e += blockDim.x) {
      float p = ad.p[k][e], m = ad.m[k][e], v = ad.v[k][e];
      adam_elem(p, ad.g[k][e], m, v, c);
      ad.p[k][e] = p;
      ad.m[k][e] = m;
      ad.v[k][e] = v;
    }
  }
}

// ---------------------------------------------------------------- batch preparation
// The fused step's weight-independent preparation of one batch (bgcn_prepare_batch /
// the next batch on the side lane) as six launches of 256-thread blocks, each carrying
// the independent steps of three chains side by side (a lone launch on a lane costs
// ~5 us however little it does):
//   A  zero the K1 counters | node -> root map, tree pointers, flag reset | DropEdge bounds
//   B  DropEdge select | tree work items | the pass over X (ELL compaction)
//   C  K1 count | CSC column histograms
//   D  K1 scan (decoupled look-back) | CSC per-column prefixes
//   E  K1 fill + self loops + D^-1/2 | CSC column starts
//   F  K1 normalisation + plans | CSC placement
struct PrepArgs {
  SparseState S;
  GraphBatch gb;
  DropList dl[2];
  const int64_t *batch, *rootindex;
  int32_t *node_root, *tree_ptr, *status;
  const void* X;
  int64_t ldx;
  const int32_t *xr_ptr, *xr_col;   // host-fed compacted features (X == nullptr), else null
  const float* xr_val;
  uint64_t* span;                   // device span stamps of the launch (timing class 7) or null
  int64_t* eptr;
  uint64_t seed;
  uint4* zero[2];
  int nzero[2];         // 16-byte words per zero range
  int nz, nRP, nR, nbd[2], lists;
  int nsel, ncomp;
  int nce, R;
  int ntile, nprefix;
  int ne, nn, np;
};

__global__ __launch_bounds__(256) void k_prep_a(PrepArgs a) {
  int b = int(blockIdx.x);
  if (b < a.nz) {   // 16 B per thread, 4 KB per block
    const int64_t w = int64_t(b) * 256 + threadIdx.x;
    const int64_t w0 = a.nzero[0];
    if (w < w0) a.zero[0][w] = make_uint4(0u, 0u, 0u, 0u);
    else if (w - w0 < a.nzero[1]) a.zero[1][w - w0] = make_uint4(0u, 0u, 0u, 0u);
    return;
  }
  b -= a.nz;
  if (b < a.nRP) {
    prologue_batch_body(a.S, a.batch, a.rootindex, a.node_root, a.tree_ptr, b, a.nR);
    return;
  }
  b -= a.nRP;
  const int d = b < a.nbd[0] ? 0 : 1;
  drop_bounds_body(a.dl[d], d, a.batch, a.S.N, a.S.B, a.eptr, a.status, d == 0 ? b : b - a.nbd[0]);
}

template <class TX>
__device__ inline void prep_b_body(const PrepArgs& a) {
  int b = int(blockIdx.x);
  if (b < a.nsel) {   // (tree, list) blocks first: they finish beside the pass over X
    const int d = b / int(a.S.B);
    drop_select_body(a.dl[d], d, int64_t(b % int(a.S.B)), a.batch, a.S.N, a.S.B, a.seed, a.eptr, 1,
                     nullptr, a.status);
    return;
  }
  b -= a.nsel;
  if (b == 0) {
    items_body(a.S, a.tree_ptr, a.rootindex);
    return;
  }
  if (a.xr_ptr) csr_ell_body(a.S, a.xr_ptr, a.xr_col, a.xr_val, b - 1, a.ncomp);
  else compact_body<false, TX>(a.S, static_cast<const TX*>(a.X), a.ldx, nullptr, b - 1, a.ncomp);
}

// a.span (the kernel-timing hook, class 7): every block min's its start and max's its end
// into the launch's wall-clock pair - the kernel's own span, as rocprofv3 reports it
// Register budget of the pass over X (min waves per SIMD of __launch_bounds__): with fp32
// X 1.5 blocks per CU run beside the training chain, and at the pass's natural 201 (-> 208)
// VGPRs the X-window kernels (conv2 116, the aggregations 88-116, the readout 106) fit only
// on the CUs holding ONE block of the pass: conv2's waves ran on 124 of 256 CUs and started
// up to 60 us late (profiles/r05_block_trace_instep.txt).  Capping the pass (3: 168 VGPRs,
// 4: 128, no spills) lets them in everywhere, but the step got SLOWER (twitter15 474k ->
// 453k / 445k, profiles/r05_pass_regs_ab.txt): the pass then ran 158 instead of 121 us
// beside a chain that was no faster - the X window is bound by the memory system, not by
// CU room, so the pass keeps its registers.
#ifndef BGCN_PREP_B_WAVES
#define BGCN_PREP_B_WAVES 2
#endif
template <class TX>
__global__ __launch_bounds__(256, BGCN_PREP_B_WAVES) void k_prep_b(PrepArgs a) {
  if (a.span && threadIdx.x == 0 && blockIdx.x < kSpanStarts)
    a.span[blockIdx.x] = uint64_t(wall_clock64());
  prep_b_body<TX>(a);
  if (a.span) {
    __syncthreads();
    if (threadIdx.x == 0)
      atomicMax(reinterpret_cast<unsigned long long*>(a.span) + kSpanStarts + blockIdx.x % kSpanEnds,
                static_cast<unsigned long long>(wall_clock64()));
  }
}

// The graph lane's launches of the two-lane preparation carry only their K1 / DropEdge
// roles, as kernels of their own: a merged launch is allocated the registers of its
// heaviest role (k_prep_b: the fp32 pass over X, 201 VGPRs; k_prep_f: the CSC placement,
// 234), so the DropEdge select's 256 blocks held 201 registers per wave for the ~90 us they
// run beside the pass - one block per CU that the chain's conv2 (236 registers) then could
// not share: conv2's waves started up to 60 us late in the X window
// (profiles/r05_block_trace_instep.txt).
__global__ __launch_bounds__(256) void k_prep_select(PrepArgs a) {
  const int b = int(blockIdx.x);
  if (b >= a.nsel) return;
  const int d = b / int(a.S.B);
  drop_select_body(a.dl[d], d, int64_t(b % int(a.S.B)), a.batch, a.S.N, a.S.B, a.seed, a.eptr, 1, nullptr,
                   a.status);
}

__global__ __launch_bounds__(256) void k_prep_f_graph(PrepArgs a) {
  const int per = a.ne + a.nn + a.np;
  const int b = int(blockIdx.x);
  if (b < 2 * per) graph_rank_norm_body(a.gb, a.gb.g[b / per], b % per, a.ne, a.nn);
}

__global__ __launch_bounds__(256) void k_prep_c(PrepArgs a) {
  extern __shared__ __attribute__((aligned(16))) int32_t dsm[];
  int b = int(blockIdx.x);
  if (b < 2 * a.nce) {
    graph_count_body(a.gb, a.gb.g[b / a.nce], b % a.nce);
    return;
  }
  csc_hist_body(a.S, b - 2 * a.nce, dsm);
}

__global__ __launch_bounds__(256) void k_prep_d(PrepArgs a) {
  int b = int(blockIdx.x);
  if (b < 2 * a.ntile) {
    graph_scan_body(a.gb, a.gb.g[b / a.ntile]);
    return;
  }
  csc_prefix_body(a.S, a.R, b - 2 * a.ntile);
}

__global__ __launch_bounds__(256) void k_prep_e(PrepArgs a) {
  int b = int(blockIdx.x);
  const int per = a.ne + a.nn;
  if (b < 2 * per) {
    graph_fill_nodes_body(a.gb, a.gb.g[b / per], b % per, a.ne);
    return;
  }
  csc_colscan_body(a.S);
}

#ifndef BGCN_PREP_F_WAVES
#define BGCN_PREP_F_WAVES 2   // (3 caps the CSC placement at 168 VGPRs with 85 spilled: not taken)
#endif
__global__ __launch_bounds__(256, BGCN_PREP_F_WAVES) void k_prep_f(PrepArgs a) {
  extern __shared__ __attribute__((aligned(16))) int32_t dsm[];
  int b = int(blockIdx.x);
  const int per = a.ne + a.nn + a.np;
  if (b < 2 * per) {
    graph_rank_norm_body(a.gb, a.gb.g[b / per], b % per, a.ne, a.nn);
    return;
  }
  csc_place_body(a.S, b - 2 * per, dsm);
}

// ---------------------------------------------------------------- merged backward launches
// middle (256 threads): dH1 (+ the relu(H1) block of dW2), db2 column sums, dW2 partials
// (dense path), dW2 root partials, the head's weight gradients;  tail (512 threads): dW1
// over the CSC, dW2 root columns, the dW2 partial reduction, db1 column sums.  Roles by
// block range, in that order.
// db2 from the readout's per-item positive-H2 counts (BwdMidArgs::db2_dhead): dH2 of a
// row is [H2 > 0] * dhead[b] / |tree b| (BiGCN_Twitter.py:57,65), so column c of db2 =
// sum_i dH2[i][c] = sum over items p of count[p][c] * dhead[tree(p)][hc] / |tree(p)|; one
// block per column, the fixed order of colsum_col_block (items past tree_item0[B]: none).
__device__ inline void db2_from_counts(const BwdMidArgs& a, int c, float* sm) {
  const int nit = a.S.tree_item0[a.S.B];
  const int hc = c < H ? 2 * H + c : c - H;   // head input = cat(BU, TD) (:128)
  const float* cnt = a.db2.part;
  float acc = 0.f;
  for (int p0 = 0; p0 < nit; p0 += 4 * 256) {   // 4 items per thread in flight
    int32_t b[4];
    float v[4];
#pragma unroll
    for (int u = 0; u < 4; ++u) {
      const int p = min(p0 + u * 256 + int(threadIdx.x), nit - 1);
      b[u] = a.S.item_tree[p];
      v[u] = cnt[int64_t(p) * 128 + c];
    }
#pragma unroll
    for (int u = 0; u < 4; ++u) {
      const int64_t bb = min<int64_t>(max<int64_t>(b[u], 0), a.S.B - 1);
      const float n = float(max(a.tree_ptr[bb + 1] - a.tree_ptr[bb], 1));
      const float g = a.db2_dhead[bb * kHeadIn + hc];
      if (p0 + u * 256 + int(threadIdx.x) < nit) acc += v[u] * (g / n);
    }
  }
#pragma unroll
  for (int m = 32; m >= 1; m >>= 1) acc += __shfl_xor(acc, m);
  if ((threadIdx.x & 63) == 0) sm[threadIdx.x >> 6] = acc;
  __syncthreads();
  if (threadIdx.x == 0) {
    const float s = ((sm[0] + sm[1]) + sm[2]) + sm[3];
    if (c < H) a.db2.out_td[c] = s; else a.db2.out_bu[c - H] = s;
  }
}

constexpr int cmax(int a, int b) { return a > b ? a : b; }
constexpr int kMidSmem = cmax(cmax(cmax(kDw2Smem, kRootPartSmem), cmax(kDh1Smem, kColsumSmem)), kHeadGradSmem);
template <class TX>
__global__ __launch_bounds__(256, 2) void k_bwd_mid(BwdMidArgs a) {   // LDS: two blocks per CU (dh1_body)
  __shared__ __attribute__((aligned(16))) float smem[kMidSmem];
  BT_BEGIN
  int b = int(blockIdx.x);
  if (b < 2 * a.nblk_h) {   // longest-lived role first
    // the relu(H1) block of dW2 rides along when the sparse path is the one running
    float* part = (a.S.mode != 1 && !dense_active(a.gate)) ? a.dw2_sparse.part : nullptr;
    dh1_body(a.dZ2, a.H1, a.W2td, a.W2bu, a.S.F + H, a.S.N, a.keep, a.dH1, a.colpart, a.rows_h, part,
             a.nblk_h, b % a.nblk_h, b / a.nblk_h, smem, a.S.mode != 1 ? a.S.w2d : nullptr);
    BT_END(72);
    return;
  }
  b -= 2 * a.nblk_h;
  if (b < kColsumColBlocks) {   // db2 before the short roles: not the launch's last blocks
    if (a.db2_dhead) db2_from_counts(a, b, smem);
    else colsum_col_block(a.db2, b, smem);
    BT_END(73);
    return;
  }
  b -= kColsumColBlocks;
  if (b < a.n_dw2) {
    dw2_body<TX>(static_cast<const TX*>(a.X), a.ldx, a.S.F, a.H1, a.dZ2, a.node_root, a.S.N, a.keep,
                 a.gate, a.dw2_dense, a.dw2_sparse, a.n_dw2_dense, b, smem);
    BT_END(70);
    return;
  }
  b -= a.n_dw2;
  if (b < a.n_root) {
    root_part_body(a.S, a.dZ2, a.tree_ptr, b % a.S.max_items, b / a.S.max_items, smem);
    BT_END(71);
    return;
  }
  head_grad_block(a.hg, b - a.n_root, smem);
}

constexpr int kTailSmem = cmax(cmax(kDw1Smem, kRedSmem), kColsumSmem);
#ifndef BGCN_TAIL_THREADS
#define BGCN_TAIL_THREADS 512   // 1024-thread blocks ran one per CU: dW1 in two rounds
#endif
constexpr int kTailThreads = BGCN_TAIL_THREADS;   // threads per block of the tail launch
// kPart (the deferred-dW1 step, bgcn_step_args.defer_dw1): 0 = every role; 1 = all but dW1
// (the dW2 root columns by one wave per column, dw1_body<1, 1>); 2 = dW1 only
template <int kDw1Split, int kPart = 0>   // kDw1Split 0: dw1_sliced_body, else dw1_body's waves per column
__global__ __launch_bounds__(kTailThreads) void k_bwd_tail(BwdTailArgs a) {
  __shared__ __attribute__((aligned(16))) float smem[kTailSmem];
  BT_BEGIN
  int b = int(blockIdx.x);
  if (b < a.n_dw1) {
    if constexpr (kPart == 1)
      dw1_body<1, 1>(a.S, a.dZ1, a.dw1_td, a.dw1_bu, a.batch, a.dw2_td, a.dw2_bu, a.keep_scale, b, smem,
                     a.dZ2, a.keep);
    else if constexpr (kDw1Split == 0)
      dw1_sliced_body<kPart>(a.S, a.dZ1, a.dw1_td, a.dw1_bu, a.batch, a.dw2_td, a.dw2_bu, a.keep_scale, b,
                             smem, a.dZ2, a.keep, &a.adam);
    else
      dw1_body<kDw1Split, kPart>(a.S, a.dZ1, a.dw1_td, a.dw1_bu, a.batch, a.dw2_td, a.dw2_bu, a.keep_scale, b,
                                 smem, a.dZ2, a.keep);
    BT_END(80);
    return;
  }
  if (kPart == 2) return;
  b -= a.n_dw1;
  if (b < a.red_dense.blocks + a.red_sparse.blocks) {
    reduce_dw2_body(a.dw2_part, a.S.F + H, a.dw2_td, a.dw2_bu, a.gate, a.red_dense, a.red_sparse, b, smem,
                    &a.adam);
    BT_END(82);
    return;
  }
  b -= a.red_dense.blocks + a.red_sparse.blocks;
  if (b < colsum_job_blocks(kTailThreads)) {
    colsum_job_block(a.db1, b, smem, &a.adam);
    BT_END(83);
    return;
  }
  if (a.adam.on) tail_adam_block(a.adam);   // the launch's last block
}

}  // namespace

// The dense feature mode's dW2 root columns for bf16 X (dw2_bf16_body) as a launch of its
// own: ~45 KB of LDS, three blocks per CU (inside the middle launch they ran at its two
// per CU).
// The H1 columns' blocks (dw2_body's column tile 0: f32 MFMA, a split's k-tiles in
// sequence, the launch's longest-lived blocks) go first, so they run beside the root
// columns instead of lengthening the middle launch.
constexpr int kDw2RootSmem = cmax(kDw2bSmem, kDw2Smem);
__global__ __launch_bounds__(256) void k_dw2_bf16(BwdMidArgs a) {
  __shared__ __attribute__((aligned(16))) float smem[kDw2RootSmem];
  int b = int(blockIdx.x);
  if (b < a.n_dw2h) {
    dw2_body<bf16_t>(static_cast<const bf16_t*>(a.X), a.ldx, a.S.F, a.H1, a.dZ2, a.node_root, a.S.N, a.keep,
                     a.gate, a.dw2_dense, a.dw2_sparse, a.n_dw2_dense, b, smem);
    return;
  }
  b -= a.n_dw2h;
  dw2_bf16_body(static_cast<const bf16_t*>(a.X), a.ldx, a.S.F, a.dZ2, a.node_root, a.S.N, a.keep, a.gate,
                a.dw2_dense, a.gxb, b, smem);
}

// ... and for fp32 X (dw2_root_body: k-tiles of one root's nodes, the root factor
// applied per tile in fp32), same LDS and block ids; TX = bf16_t: the same form for bf16 X
// (the default; BGCN_DW2_ROOT=0 keeps k_dw2_bf16).
#ifndef BGCN_DW2R_WPE
#define BGCN_DW2R_WPE 3   // three waves per SIMD (162 VGPRs at BGCN_DW2R_DEEP 1)
#endif
template <class TX>
__global__ __launch_bounds__(256) __attribute__((amdgpu_waves_per_eu(BGCN_DW2R_WPE))) void k_dw2_root(BwdMidArgs a) {
  __shared__ __attribute__((aligned(16))) float smem[kDw2RootSmem];
  int b = int(blockIdx.x);
  if (b < a.n_dw2h) {
    dw2_body<TX>(static_cast<const TX*>(a.X), a.ldx, a.S.F, a.H1, a.dZ2, a.node_root, a.S.N, a.keep,
                 a.gate, a.dw2_dense, a.dw2_sparse, a.n_dw2_dense, b, smem);
    return;
  }
  b -= a.n_dw2h;
  dw2_root_body<TX>(static_cast<const TX*>(a.X), a.ldx, a.S.F, a.dZ2, a.node_root, a.S.N, a.keep, a.gate,
                    a.dw2_dense, a.gxb, b, smem);
}

int dw2_bf16_launch(BwdMidArgs& a, hipStream_t s) {
  if (a.n_dw2b <= 0) return BGCN_OK;
  const unsigned n = unsigned(a.n_dw2b + a.n_dw2h);
  if (a.dw2b_f32 == 1)
    hipLaunchKernelGGL(k_dw2_root<float>, dim3(n), dim3(256), 0, s, a);
  else if (a.dw2b_f32 == 2)
    hipLaunchKernelGGL(k_dw2_root<bf16_t>, dim3(n), dim3(256), 0, s, a);
  else
    hipLaunchKernelGGL(k_dw2_bf16, dim3(n), dim3(256), 0, s, a);
  BGCN_CHECK_LAUNCH();
  return BGCN_OK;
}

// The dense feature mode's dW2 (fp32 X; dw2_body, f32 MFMA) as a launch of its own: inside
// the middle launch it ran at that launch's register budget (210 VGPRs since the fused
// dH1 + relu(H1)-dW2 role of round 3: two waves per SIMD) - 76.5 -> 64 TF/s.
__global__ __launch_bounds__(256) void k_dw2_f32(BwdMidArgs a) {
  __shared__ __attribute__((aligned(16))) float smem[kDw2Smem];
  dw2_body<float>(static_cast<const float*>(a.X), a.ldx, a.S.F, a.H1, a.dZ2, a.node_root, a.S.N, a.keep,
                  a.gate, a.dw2_dense, a.dw2_sparse, a.n_dw2_dense, int(blockIdx.x), smem);
}

int dw2_f32_launch(BwdMidArgs& a, hipStream_t s) {
  if (a.n_dw2f <= 0) return BGCN_OK;
  hipLaunchKernelGGL(k_dw2_f32, dim3(unsigned(a.n_dw2f)), dim3(256), 0, s, a);
  BGCN_CHECK_LAUNCH();
  return BGCN_OK;
}

int bwd_mid_launch(BwdMidArgs& a, int x_dtype, hipStream_t s) {
  a.n_root = (a.S.mode != 1) ? 2 * a.S.max_items : 0;
  const int n = a.n_dw2 + a.n_root + 2 * a.nblk_h + kColsumColBlocks + a.n_hg;
  if (x_dtype == BGCN_DTYPE_BF16)
    hipLaunchKernelGGL(k_bwd_mid<bf16_t>, dim3(unsigned(n)), dim3(256), 0, s, a);
  else
    hipLaunchKernelGGL(k_bwd_mid<float>, dim3(unsigned(n)), dim3(256), 0, s, a);
  BGCN_CHECK_LAUNCH();
  return BGCN_OK;
}

int bwd_tail_launch(BwdTailArgs& a, hipStream_t s, int part) {
  // one wave per column (with 1024-thread blocks, one per CU, four waves per column won
  // from 64k rows; with 512-thread blocks one wave wins at every size: synth1024_bf16
  // 0.839 vs 0.850-0.859 ms, weibo_bf16 0.690 vs 0.697, profiles/r02_split_ab.txt);
  // BGCN_DW1_SPLIT=1/4 forces either (read per call: tests compare both)
  // default: the XCD-aware output slices (dw1_sliced_body), BGCN_DW1_SPLIT=0
  const char* e = std::getenv("BGCN_DW1_SPLIT");
  const bool sparse = a.S.mode != 1;
  const int split = e ? atoi(e) : 0;
  constexpr int wpb = kTailThreads / 64;   // waves per block
  const int cols1 = split == 4 ? wpb / 4 : wpb;
  a.n_dw1 = !sparse ? 0 : split == 0 ? dw1_sliced_blocks(a.S.F, wpb) : int((a.S.F + cols1 - 1) / cols1);
  if (part == 1) a.n_dw1 = !sparse ? 0 : int((a.S.F + wpb - 1) / wpb);   // root columns: a wave per column
  a.n_rootcols = 0;   // the dW2 root columns ride with the dW1 waves (dw1_body)
  // the reduction configurations are sized in 1024-thread blocks (4 groups of 256)
  a.red_dense.blocks *= 1024 / kTailThreads;
  a.red_sparse.blocks *= 1024 / kTailThreads;
  if (part != 0 || split != 0) a.adam.on = 0;   // (bigcn_backward_impl only fuses into part 0's sliced form)
  const int n = part == 2 ? a.n_dw1
                          : a.n_dw1 + a.red_dense.blocks + a.red_sparse.blocks + colsum_job_blocks(kTailThreads) +
                                (a.adam.on ? 1 : 0);
  if (n == 0) return BGCN_OK;
  if (part == 1) {
    hipLaunchKernelGGL((k_bwd_tail<1, 1>), dim3(unsigned(n)), dim3(kTailThreads), 0, s, a);
    BGCN_CHECK_LAUNCH();
    return BGCN_OK;
  }
  if (part == 2) {
    if (split == 4)
      hipLaunchKernelGGL((k_bwd_tail<4, 2>), dim3(unsigned(n)), dim3(kTailThreads), 0, s, a);
    else if (split == 1)
      hipLaunchKernelGGL((k_bwd_tail<1, 2>), dim3(unsigned(n)), dim3(kTailThreads), 0, s, a);
    else
      hipLaunchKernelGGL((k_bwd_tail<0, 2>), dim3(unsigned(n)), dim3(kTailThreads), 0, s, a);
    BGCN_CHECK_LAUNCH();
    return BGCN_OK;
  }
  if (split == 4)
    hipLaunchKernelGGL(k_bwd_tail<4>, dim3(unsigned(n)), dim3(kTailThreads), 0, s, a);
  else if (split == 1)
    hipLaunchKernelGGL(k_bwd_tail<1>, dim3(unsigned(n)), dim3(kTailThreads), 0, s, a);
  else
    hipLaunchKernelGGL(k_bwd_tail<0>, dim3(unsigned(n)), dim3(kTailThreads), 0, s, a);
  BGCN_CHECK_LAUNCH();
  return BGCN_OK;
}

// ---------------------------------------------------------------- host side
size_t carve_images(Carve& c, int64_t F, WeightImages* im) {
  WeightImages t;
  t.w1t = c.take<float>(size_t(F) * 2 * H);
  t.w2t = c.take<float>(size_t(2) * (F + H) * H);
  t.w2s = c.take<__bf16>(size_t(2) * 3 * H * kW2sLd);
  t.w2d = c.take<__bf16>(size_t(2) * 3 * H * kW2dLd);
  if (im) *im = t;
  return c.off;
}

size_t carve_sparse(Carve& c, int64_t N, int64_t B, int64_t F, SparseState* S) {
  SparseState t{};
  t.N = N;
  t.F = F;
  t.B = B;
  t.max_items = int(N / kChunk + B + 1);
  t.w1t = c.take<float>(size_t(F) * 2 * H);
  t.w2t = c.take<float>(size_t(2) * (F + H) * H);
  t.w2s = c.take<__bf16>(size_t(2) * 3 * H * kW2sLd);
  t.w2d = c.take<__bf16>(size_t(2) * 3 * H * kW2dLd);
  t.item_tree = c.take<int32_t>(size_t(t.max_items));
  t.item_beg = c.take<int32_t>(size_t(t.max_items));
  t.item_end = c.take<int32_t>(size_t(t.max_items));
  t.item_root = c.take<int32_t>(size_t(t.max_items));
  t.tree_item0 = c.take<int32_t>(size_t(B + 1));
  t.root_part = c.take<float>(size_t(2) * t.max_items * kCap * H);
  const size_t slots = size_t(N) * kCap;
  const size_t R = size_t((N + kRowBlock - 1) / kRowBlock);
  t.hist = c.take<int32_t>(R * size_t(F));
  t.col_total = c.take<int32_t>(size_t(F));
  t.col_start = c.take<int32_t>(size_t(F));
  t.col_end = c.take<int32_t>(size_t(F));
  t.csc = c.take<uint2>(slots + size_t(N) * kSpillPerRow);
  t.rbits = c.take<uint32_t>(size_t(2) * N);
  t.ovf_off = c.take<int32_t>(size_t(N));   // the per-op encoder's spill pool (a prepared
  t.ovf_cap = N * kSpillPerRow;             // batch brings its own)
  t.ovf = c.take<uint2>(size_t(t.ovf_cap));
  t.long_rows = c.take<int32_t>(size_t(N));
  t.rimg = c.take<__bf16>(size_t(B) * 2 * 3 * H * kCap);
  t.rcols = c.take<uint32_t>(size_t(B) * kCap);
  t.rinfo = c.take<int32_t>(size_t(B));
  if (S) {
    t.mode = S->mode;
    t.flags = S->flags;
    t.nnz = S->nnz;
    t.cols = S->cols;
    t.vals = S->vals;
    *S = t;
  }
  return c.off;
}

int sparse_prologue(SparseState& S, const bgcn_bigcn_args* a, int32_t* node_root, hipStream_t s,
                    bool batch_part) {
  const int nTx = int((S.F + H + 31) / 32);
  const int nT = S.mode == 1 ? 0 : nTx * 2 * 4;
  const int nS = nT > 0 ? 2 * kSplitBlocks : 0;
  const int nR = batch_part ? int((S.N + 255) / 256) : 0;
  const int nP = batch_part ? int((S.B + 1 + 255) / 256) : 0;
  const int nZ = (nT + nR + nP == 0 && (S.zero_word || S.rtick)) ? 1 : 0;
  if (nT + nR + nP + nZ == 0) return BGCN_OK;
  hipLaunchKernelGGL(k_prologue, dim3(unsigned(nT + nS + nR + nP + nZ)), dim3(256), 0, s, S, a->td_w1, a->bu_w1,
                     a->td_w2, a->bu_w2, a->batch, a->rootindex, node_root, a->tree_ptr, nTx, nT, nR);
  BGCN_CHECK_LAUNCH();
  return BGCN_OK;
}

int sparse_compact_conv1(SparseState& S, const void* X, int xdt, int64_t ldx, float* Z1,
                         hipStream_t s) {
  if (xdt == BGCN_DTYPE_BF16)
    hipLaunchKernelGGL((k_compact_conv1<true, bf16_t>), dim3(grid_for(S.N, 4)), dim3(256), 0, s, S,
                       static_cast<const bf16_t*>(X), ldx, Z1);
  else
    hipLaunchKernelGGL((k_compact_conv1<true, float>), dim3(grid_for(S.N, 4)), dim3(256), 0, s, S,
                       static_cast<const float*>(X), ldx, Z1);
  BGCN_CHECK_LAUNCH();
  return BGCN_OK;
}

int sparse_items(SparseState& S, const int32_t* tree_ptr, const int64_t* rootindex, hipStream_t s) {
  hipLaunchKernelGGL(k_items, dim3(1), dim3(1024), 0, s, S, tree_ptr, rootindex);
  BGCN_CHECK_LAUNCH();
  return BGCN_OK;
}

int sparse_conv2(SparseState& S, const float* H1, const int32_t* tree_ptr, const int64_t* rootindex,
                 float* Z2, KeepSrc keep, hipStream_t s) {
  if (BGCN_C2_HALF)
    hipLaunchKernelGGL(k_conv2_half, dim3(unsigned(2 * S.max_items), 2), dim3(256), 0, s, S, H1, Z2, keep);
  else
    hipLaunchKernelGGL(k_conv2_sparse, dim3(unsigned(S.max_items), 2), dim3(256), 0, s, S, H1,
                       tree_ptr, rootindex, Z2, keep);
  BGCN_CHECK_LAUNCH();
  return BGCN_OK;
}


int sparse_csc(SparseState& S, hipStream_t s) {
  const int R = int((S.N + kRowBlock - 1) / kRowBlock);
  hipLaunchKernelGGL(k_csc_hist, dim3(unsigned(R)), dim3(kRowBlock), size_t(S.F) * sizeof(int32_t), s, S);
  BGCN_CHECK_LAUNCH();
  hipLaunchKernelGGL(k_csc_prefix, dim3(grid_for(S.F, kPrefixCols)), dim3(256), 0, s, S, R);
  BGCN_CHECK_LAUNCH();
  hipLaunchKernelGGL(k_csc_colscan, dim3(1), dim3(1024), 0, s, S);
  BGCN_CHECK_LAUNCH();
  hipLaunchKernelGGL(k_csc_place, dim3(unsigned(R)), dim3(256), size_t(2 * S.F) * sizeof(int32_t), s, S);
  BGCN_CHECK_LAUNCH();
  return BGCN_OK;
}

#ifndef BGCN_PREP_LANES_DEFAULT
#define BGCN_PREP_LANES_DEFAULT 2   // profiles/r03_chain_experiments_late.txt
#endif
// the sparse state of a prepared batch's buffers
static void prepared_state(const Prepared& p, int64_t N, int64_t B, int64_t F, int mode, SparseState& S) {
  S.mode = mode;
  S.N = N; S.F = F; S.B = B;
  S.max_items = int(N / kChunk + B + 1);
  S.flags = p.x_flags; S.nnz = p.x_nnz; S.cols = p.x_cols; S.vals = p.x_vals;
  S.item_tree = p.item_tree; S.tree_item0 = p.tree_item0;
  S.item_beg = p.item_beg; S.item_end = p.item_end; S.item_root = p.item_root;
  S.hist = p.hist; S.col_total = p.col_total; S.col_start = p.col_start; S.col_end = p.col_end;
  S.csc = p.csc;
  S.ovf_off = p.x_ovf_off; S.ovf = p.x_ovf; S.ovf_cap = p.ovf_cap; S.long_rows = p.x_long;
  S.root_map = p.node_root;
  S.bstatus = p.status;
}

int prep_pipeline(const Prepared& p, const bgcn_batch* bt, int64_t F, int degree_on, int mode,
                  hipStream_t s, bool x_part, int nlanes) {
  const int64_t N = bt->num_nodes, B = bt->num_graphs;
  BGCN_CHECK_HIP(hipMemsetAsync(p.status, 0, sizeof(int32_t), s));
  PrepArgs a{};
  SparseState& S = a.S;
  prepared_state(p, N, B, F, mode, S);
  a.batch = bt->batch; a.rootindex = bt->rootindex;
  a.node_root = p.node_root; a.tree_ptr = p.tree_ptr; a.status = p.status;
  a.X = bt->x; a.ldx = bt->ldx;
  if (!bt->x) { a.xr_ptr = bt->x_row_ptr; a.xr_col = bt->x_col; a.xr_val = bt->x_val; }
  // DropEdge (dataset.py:68-90) in the masked form: dropped edges become self loops, which
  // K1 removes - the graphs of the compacted lists, no kept count on the host
  const int64_t Etd = bt->td_num_edges, Ebu = bt->bu_num_edges;
  const bool drop = bt->td_droprate > 0.0 || bt->bu_droprate > 0.0;
  const int64_t* td = bt->td_edge_index;
  const int64_t* bu = bt->bu_edge_index;
  a.lists = drop ? 2 : 0;
  if (drop) {
    BGCN_CHECK_ARG(p.dws && p.dws_bytes >= drop_ws_size(B), "drop workspace too small");
    Carve c(p.dws, p.dws_bytes);
    a.eptr = c.take<int64_t>(size_t(2 * (B + 1)));
    a.dl[0] = DropList{td, Etd, p.td_drop, Etd, bt->td_droprate, 0u};
    a.dl[1] = DropList{bu, Ebu, p.bu_drop, Ebu, bt->bu_droprate, 1u};
    a.seed = bt->drop_seed;
    if (td) td = p.td_drop;
    if (bu) bu = p.bu_drop;
  }
  GraphArgs ga[2];
  graph_pair_args(td, Etd, bu, Ebu, &p.td, &p.bu, p.status, p.gws, p.gws_bytes, ga);
  size_t zb[2] = {0, 0};
  BGCN_TRY(graph_batch_setup(ga, 2, N, degree_on, &a.gb, zb, bt->batch));
  for (int k = 0; k < 2; ++k) {
    a.zero[k] = reinterpret_cast<uint4*>(a.gb.g[k].cnt_t);
    a.nzero[k] = int(zb[k] / 16);
    BGCN_CHECK_ARG(zb[k] % 16 == 0 && (reinterpret_cast<uintptr_t>(a.zero[k]) & 15) == 0, "zero range");
  }
  const bool sparse = mode != 1;
  const bool xp = sparse && x_part;   // the pass over X and the CSC of X in these launches
  const int64_t Emax = std::max(Etd, Ebu);
  a.nz = int((a.nzero[0] + a.nzero[1] + 255) / 256);
  a.nR = int((N + 255) / 256);
  a.nRP = a.nR + int((B + 1 + 255) / 256);
  a.nbd[0] = drop ? int(Etd / 256 + 1) : 0;
  a.nbd[1] = drop ? int(Ebu / 256 + 1) : 0;
  a.nsel = drop ? int(2 * B) : 0;
  {   // The pass over X is paced: with fp32 X 1.5 4-wave blocks per CU stride over the
      // rows (~30 MB of loads in flight, ~4.5 TB/s).  A wave per row over all rows drains
      // X at 5.5 TB/s but floods the memory queues with ~100 MB of requests, and every
      // load of the latency-bound training chain beside it then waits behind them:
      // measured 0.293-0.295 ms per step paced vs 0.303-0.306 unpaced (twitter15; 224-288
      // blocks within 1%, 512 worse than either).  With the shorter chain of 512-thread
      // aggregation / tail blocks, 384 blocks: 0.2964-0.2966 vs 0.304-0.308 at 256
      // (profiles/r02_pace_ab.txt).  bf16 X (the prefix compaction, compact_by_prefix):
      // one block per CU - 192 / 256 / 320 / 512 / 1024 blocks / the full grid: weibo_bf16
      // 0.667 / 0.646 / 0.661 / 0.709 / 0.688 / 0.697 ms (profiles/r02_compact_ab.txt).
      // BGCN_PREP_BLOCKS (read per call) overrides: 0 = full grid, n = n blocks.
    static const int ncu = [] {
      int dev = 0, n = 0;
      if (hipGetDevice(&dev) != hipSuccess ||
          hipDeviceGetAttribute(&n, hipDeviceAttributeMultiprocessorCount, dev) != hipSuccess)
        n = 256;
      return n > 0 ? n : 256;
    }();
    const bool bf = bt->x_dtype == BGCN_DTYPE_BF16;
    a.ncomp = xp ? int(grid_for(N, bf ? 8 : 4)) : 0;
    int cap = bf ? (compact_by_prefix<bf16_t>() ? ncu : 0) : ncu + ncu / 2;
    const char* e = std::getenv("BGCN_PREP_BLOCKS");
    if (e) cap = atoi(e);
    if (cap > 0) a.ncomp = std::min(a.ncomp, cap);
    // host-fed compacted rows: 8 rows per block over every row, nothing to pace (nnz x 8 B)
    if (a.xr_ptr && xp) a.ncomp = int(grid_for(N, 8));
  }
  a.nce = graph_edge_blocks(Emax);
  a.R = xp ? int((N + kRowBlock - 1) / kRowBlock) : 0;
  a.ntile = int(graph_scan_tiles(N));
  a.nprefix = xp ? int(grid_for(F, kPrefixCols)) : 0;
  a.ne = graph_edge_blocks(Emax);
  a.nn = graph_node_blocks(N);
  a.np = graph_pos_blocks(Emax, N);
  const dim3 blk(256);
  hipLaunchKernelGGL(k_prep_a, dim3(unsigned(a.nz + a.nRP + a.nbd[0] + a.nbd[1])), blk, 0, s, a);
  BGCN_CHECK_LAUNCH();
  const size_t hist_smem = xp ? size_t(F) * sizeof(int32_t) : 0;
  // Two lanes (the default; BGCN_PREP_LANES=1, read once, keeps one): DropEdge select + K1
  // run on a second lane beside the pass over X, and the CSC of X follows the pass on the
  // side lane - the roles of each merged launch split by chain.  K1's four latency-bound
  // launches then overlap the X window, where the chain is stalled anyway, instead of the
  // chain's second half: twitter15 0.2691-0.2724 vs 0.2732-0.2749 ms per step over five
  // interleaved rounds, synth1024_bf16 -0.7 %, weibo_bf16 within its noise (+0.5 %)
  static const int default_lanes = [] {
    const char* e = std::getenv("BGCN_PREP_LANES");
    return e ? atoi(e) : BGCN_PREP_LANES_DEFAULT;
  }();
  const int lanes = nlanes > 0 ? nlanes : default_lanes;
  if (lanes == 2 && xp) {
    hipStream_t g = s;
    BGCN_TRY(aux_fork(s, kLaneGraph, &g));
    PrepArgs ag = a;           // graph chain: DropEdge select, K1 count / scan / fill / norm
    ag.ncomp = 0; ag.R = 0; ag.nprefix = 0;
    PrepArgs ax = a;           // X chain: tree items, the pass over X, the CSC of X
    ax.nsel = 0; ax.nce = 0; ax.ntile = 0; ax.ne = 0; ax.nn = 0; ax.np = 0;
    if (ag.nsel > 0) {
      hipLaunchKernelGGL(k_prep_select, dim3(unsigned(ag.nsel)), blk, 0, g, ag);
      BGCN_CHECK_LAUNCH();
    }
    if (ag.nce > 0) hipLaunchKernelGGL(k_prep_c, dim3(unsigned(2 * ag.nce)), blk, 0, g, ag);
    if (ag.ntile > 0) hipLaunchKernelGGL(k_prep_d, dim3(unsigned(2 * ag.ntile)), blk, 0, g, ag);
    if (ag.ne + ag.nn > 0) hipLaunchKernelGGL(k_prep_e, dim3(unsigned(2 * (ag.ne + ag.nn))), blk, 0, g, ag);
    if (ag.ne + ag.nn + ag.np > 0)
      hipLaunchKernelGGL(k_prep_f_graph, dim3(unsigned(2 * (ag.ne + ag.nn + ag.np))), blk, 0, g, ag);
    BGCN_CHECK_LAUNCH();
    timing_begin(7, s);
    ax.span = span_slot(7);
    if (bt->x_dtype == BGCN_DTYPE_BF16) hipLaunchKernelGGL(k_prep_b<bf16_t>, dim3(unsigned(1 + ax.ncomp)), blk, 0, s, ax);
    else hipLaunchKernelGGL(k_prep_b<float>, dim3(unsigned(1 + ax.ncomp)), blk, 0, s, ax);
    BGCN_CHECK_LAUNCH();
    timing_end(7, s);
    hipLaunchKernelGGL(k_prep_c, dim3(unsigned(ax.R)), blk, hist_smem, s, ax);
    hipLaunchKernelGGL(k_prep_d, dim3(unsigned(ax.nprefix)), blk, 0, s, ax);
    hipLaunchKernelGGL(k_prep_e, dim3(1u), blk, 0, s, ax);
    hipLaunchKernelGGL(k_prep_f, dim3(unsigned(ax.R)), blk, 2 * hist_smem, s, ax);
    BGCN_CHECK_LAUNCH();
    BGCN_TRY(aux_join(s, kLaneGraph));
    return BGCN_OK;
  }
  timing_begin(7, s);
  a.span = span_slot(7);
  const unsigned nb = unsigned(a.nsel + 1 + a.ncomp);
  if (bt->x_dtype == BGCN_DTYPE_BF16) hipLaunchKernelGGL(k_prep_b<bf16_t>, dim3(nb), blk, 0, s, a);
  else hipLaunchKernelGGL(k_prep_b<float>, dim3(nb), blk, 0, s, a);
  BGCN_CHECK_LAUNCH();
  timing_end(7, s);
  if (2 * a.nce + a.R > 0) {
    hipLaunchKernelGGL(k_prep_c, dim3(unsigned(2 * a.nce + a.R)), blk, hist_smem, s, a);
    BGCN_CHECK_LAUNCH();
  }
  hipLaunchKernelGGL(k_prep_d, dim3(unsigned(2 * a.ntile + a.nprefix)), blk, 0, s, a);
  BGCN_CHECK_LAUNCH();
  hipLaunchKernelGGL(k_prep_e, dim3(unsigned(2 * (a.ne + a.nn) + (xp ? 1 : 0))), blk, 0, s, a);
  BGCN_CHECK_LAUNCH();
  hipLaunchKernelGGL(k_prep_f, dim3(unsigned(2 * (a.ne + a.nn + a.np) + a.R)), blk, 2 * hist_smem, s, a);
  BGCN_CHECK_LAUNCH();
  return BGCN_OK;
}

int sparse_prepare(const Prepared& p, int64_t N, int64_t B, int64_t F, int mode,
                   const int64_t* batch, const int64_t* rootindex, const void* X, int xdt, int64_t ldx,
                   hipStream_t s, int part, const bgcn_batch* csr) {
  SparseState S{};
  S.mode = mode;
  S.N = N; S.F = F; S.B = B;
  S.max_items = int(N / kChunk + B + 1);
  S.flags = p.x_flags; S.nnz = p.x_nnz; S.cols = p.x_cols; S.vals = p.x_vals;
  S.item_tree = p.item_tree; S.tree_item0 = p.tree_item0;
  S.item_beg = p.item_beg; S.item_end = p.item_end; S.item_root = p.item_root;
  S.hist = p.hist; S.col_total = p.col_total; S.col_start = p.col_start; S.col_end = p.col_end;
  S.csc = p.csc;
  S.ovf_off = p.x_ovf_off; S.ovf = p.x_ovf; S.ovf_cap = p.ovf_cap; S.long_rows = p.x_long;
  S.root_map = p.node_root;
  S.bstatus = p.status;
  if (!(part & 1)) return mode == 1 ? BGCN_OK : sparse_csc(S, s);
  const int nR = int((N + 255) / 256), nP = int((B + 1 + 255) / 256);
  hipLaunchKernelGGL(k_prologue, dim3(unsigned(nR + nP)), dim3(256), 0, s, S, nullptr, nullptr,
                     nullptr, nullptr, batch, rootindex, p.node_root, p.tree_ptr, 1, 0, nR);
  BGCN_CHECK_LAUNCH();
  if (mode == 1) return BGCN_OK;
  BGCN_TRY(sparse_items(S, p.tree_ptr, rootindex, s));
  timing_begin(7, s);
  const dim3 grid(grid_for(N, xdt == BGCN_DTYPE_BF16 ? 8 : 4));
  if (!X && csr)
    hipLaunchKernelGGL(k_csr_ell, dim3(grid_for(N, 8)), dim3(256), 0, s, S, csr->x_row_ptr, csr->x_col, csr->x_val);
  else if (xdt == BGCN_DTYPE_BF16)
    hipLaunchKernelGGL((k_compact_conv1<false, bf16_t>), grid, dim3(256), 0, s, S,
                       static_cast<const bf16_t*>(X), ldx, nullptr);
  else
    hipLaunchKernelGGL((k_compact_conv1<false, float>), grid, dim3(256), 0, s, S,
                       static_cast<const float*>(X), ldx, nullptr);
  timing_end(7, s);
  BGCN_CHECK_LAUNCH();
  return (part & 2) ? sparse_csc(S, s) : BGCN_OK;
}

int sparse_conv1_gather(SparseState& S, float* Z1, hipStream_t s, const int64_t* rootindex, float sc) {
  // conv2's root images ride in this launch (BGCN_C2_HALF, BGCN_C2_RIMG; rootindex given)
  const int nroot = (BGCN_C2_HALF && BGCN_C2_RIMG && rootindex) ? int(2 * S.B) : 0;
  S.rimg_ready = nroot > 0 ? 1 : 0;
#if BGCN_C1_MODE == 1
  hipLaunchKernelGGL(k_conv1_rows2<8>, dim3(nroot + kLongRowBlocks + grid_for(S.N, 8)), dim3(256), 0, s, S, Z1,
                     rootindex, sc, nroot);
#elif BGCN_C1_MODE == 2
  hipLaunchKernelGGL(k_conv1_rows2<4>, dim3(nroot + kLongRowBlocks + grid_for(S.N, 8)), dim3(256), 0, s, S, Z1,
                     rootindex, sc, nroot);
#else
  S.rimg_ready = 0;
  hipLaunchKernelGGL(k_conv1_gather, dim3(grid_for(S.N, (kC1Threads / 64) * kC1Rows)), dim3(kC1Threads), 0, s,
                     S, Z1);
#endif
  BGCN_CHECK_LAUNCH();
  return BGCN_OK;
}



}  // namespace bgcn

extern "C" size_t bgcn_weight_images_size(int64_t in_feats) {
  if (in_feats <= 0) return 0;
  bgcn::Carve c(nullptr, 0);
  return bgcn::carve_images(c, in_feats, nullptr) + 256;
}

BT_READER(sparse)

extern "C" int bgcn_csr_to_dense(const int32_t* x_row_ptr, const int32_t* x_col, const float* x_val,
                                 int64_t num_nodes, int64_t in_feats, void* x, int64_t ldx, int32_t x_dtype,
                                 int32_t* status, bgcn_stream_t stream) {
  using namespace bgcn;
  BGCN_CHECK_ARG(num_nodes > 0 && in_feats > 0 && in_feats % 4 == 0 && ldx >= in_feats && ldx % 4 == 0,
                 "bad sizes (in_feats and ldx: multiples of 4)");
  BGCN_CHECK_ARG(x_row_ptr && x_col && x_val && x, "null pointer");
  BGCN_CHECK_ARG((reinterpret_cast<uintptr_t>(x) & 15) == 0, "x must be 16-byte aligned");
  BGCN_CHECK_ARG(x_dtype == BGCN_DTYPE_F32 || x_dtype == BGCN_DTYPE_BF16, "bad x_dtype");
  BGCN_CHECK_ARG(in_feats <= 8192, "in_feats > 8192 (the row is assembled in LDS)");
  hipStream_t s = reinterpret_cast<hipStream_t>(stream);
  const size_t smem = size_t(2) * size_t((in_feats + 3) / 4 * 4) * sizeof(float);   // two waves' rows
  const dim3 grid(unsigned(std::min<int64_t>((num_nodes + 1) / 2, 8192)));
  if (x_dtype == BGCN_DTYPE_BF16)
    hipLaunchKernelGGL(k_csr_dense<bf16_t>, grid, dim3(128), smem, s, x_row_ptr, x_col, x_val, num_nodes, in_feats,
                       static_cast<bf16_t*>(x), ldx, status);
  else
    hipLaunchKernelGGL(k_csr_dense<float>, grid, dim3(128), smem, s, x_row_ptr, x_col, x_val, num_nodes, in_feats,
                       static_cast<float*>(x), ldx, status);
  BGCN_CHECK_LAUNCH();
  return BGCN_OK;
}
