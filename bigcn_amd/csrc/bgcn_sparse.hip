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
#include <cstring>



#include "bgcn_sparse.h"

namespace bgcn {
namespace {

constexpr int H = 64;

__device__ __forceinline__ bool use_sparse(const SparseState& S) { return S.mode != 1 && S.flags[0] == 0; }

// ---------------------------------------------------------------- weight transposes
// W1T[c][d*64 + o] = W1_d[o][c] (c < F) and W2T_d[k][o] = W2_d[o][k] (k < 64+F):
// 32 x 32 tiles through LDS; blockIdx.z: 0/1 = W1 td/bu, 2/3 = W2 td/bu.
__global__ __launch_bounds__(256) void k_transpose_weights(SparseState S, const float* __restrict__ w1td,
                                                           const float* __restrict__ w1bu,
                                                           const float* __restrict__ w2td,
                                                           const float* __restrict__ w2bu) {
  if (!use_sparse(S)) return;
  __shared__ float tile[32][33];
  const int z = blockIdx.z;
  const int64_t K = z < 2 ? S.F : S.F + H;
  const float* src = z == 0 ? w1td : z == 1 ? w1bu : z == 2 ? w2td : w2bu;
  const int64_t k0 = int64_t(blockIdx.x) * 32;
  const int o0 = blockIdx.y * 32;
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

// ---------------------------------------------------------------- X compaction + conv1
// One wave per row: stream the dense row (float4 per lane, 4 x 1 KiB in flight),
// compact the non-zeros in (chunk, component, lane) order, then
// Z1[i] = sum val * W1T[col] with each lane owning 2 of the 128 outputs.
__global__ __launch_bounds__(256) void k_compact_conv1(SparseState S, const float* __restrict__ X,
                                                       int64_t ldx, float* __restrict__ Z1) {
  __shared__ int32_t s_col[4][kCap];
  __shared__ float s_val[4][kCap];
  if (S.mode == 1) return;
  const int wave = threadIdx.x >> 6, lane = threadIdx.x & 63;
  const int64_t i = int64_t(blockIdx.x) * 4 + wave;
  if (i >= S.N) return;
  const float* row = X + i * ldx;
  const int nq = int(S.F / 4);   // float4 per row (F % 4 == 0)
  int cnt = 0;
  const uint64_t lt = (lane == 0) ? 0ull : (~0ull >> (64 - lane));
  for (int q0 = 0; q0 < nq; q0 += 4 * 64) {
    float4 v[4];
#pragma unroll
    for (int u = 0; u < 4; ++u) {
      const int q = q0 + u * 64 + lane;
      v[u] = q < nq ? ld4(row + int64_t(q) * 4) : f4zero();
    }
#pragma unroll
    for (int u = 0; u < 4; ++u) {
      const float e[4] = {v[u].x, v[u].y, v[u].z, v[u].w};
#pragma unroll
      for (int c = 0; c < 4; ++c) {
        const bool nz = e[c] != 0.f;
        const uint64_t m = __ballot(nz);
        const int pos = cnt + __popcll(m & lt);
        if (nz && pos < kCap) {
          s_col[wave][pos] = (q0 + u * 64 + lane) * 4 + c;
          s_val[wave][pos] = e[c];
        }
        cnt += __popcll(m);
      }
    }
  }
  if (lane == 0) S.nnz[i] = cnt;
  if (cnt > kCap) {
    if (lane == 0) atomicOr(&S.flags[0], 1);
    return;
  }
  __builtin_amdgcn_s_waitcnt(0xc07f);   // lgkmcnt(0): this wave's LDS writes have landed
  __builtin_amdgcn_wave_barrier();
  if (lane < cnt) {
    S.cols[i * kCap + lane] = s_col[wave][lane];
    S.vals[i * kCap + lane] = s_val[wave][lane];
  }
  float2 acc = make_float2(0.f, 0.f);
  for (int s0 = 0; s0 < cnt; s0 += 8) {
    float2 w[8];
    float x[8];
#pragma unroll
    for (int u = 0; u < 8; ++u) {
      const int s = s0 + u;
      const bool ok = s < cnt;
      x[u] = ok ? s_val[wave][s] : 0.f;
      w[u] = ok ? *reinterpret_cast<const float2*>(S.w1t + int64_t(s_col[wave][s]) * (2 * H) + 2 * lane)
                : make_float2(0.f, 0.f);
    }
#pragma unroll
    for (int u = 0; u < 8; ++u) {
      acc.x = fmaf(x[u], w[u].x, acc.x);
      acc.y = fmaf(x[u], w[u].y, acc.y);
    }
  }
  *reinterpret_cast<float2*>(Z1 + i * (2 * H) + 2 * lane) = acc;
}

// ---------------------------------------------------------------- conv2 forward
// conv2 lin on the sparse path, one work item (<= kChunk nodes of one tree) per block:
//   Z2_d[i] = [keep * 2 relu(H1_d[i]) | kept_d(i, s)] . [W2_d^T[0:64] ; Wr_b]
//   Wr_b[s] = 2 relu(x_root,col_s) W2_d^T[64 + col_s]      (s < nnz(root), else 0)
// i.e. one [nodes x 96] x [96 x 64] product on the fp32 MFMA per item, with the
// dropout-masked relu(H1) and the per-node root keep bits (0/1) generated in registers
// and the tree's root block of W2^T staged in LDS.  The root keep masks are stored in
// S.rbits for the dW2 root columns of the backward.  K order is permuted per lane half
// (half h owns k in [48h, 48h + 48)), B rows padded to 66 floats so the two halves read
// disjoint LDS banks.
constexpr int kC2K = 2 * H / 4 * 3;  // 96 = 64 relu(H1) columns + 32 root slots
constexpr int kC2Ld = H + 2;
__global__ __launch_bounds__(256) void k_conv2_sparse(SparseState S, const float* __restrict__ H1,
                                                      const int32_t* __restrict__ tree_ptr,
                                                      const int64_t* __restrict__ rootindex,
                                                      float* __restrict__ Z2, KeepSrc keep) {
  if (!use_sparse(S)) return;
  const int item = blockIdx.x;
  if (item >= S.tree_item0[S.B]) return;
  __shared__ float Bs[kC2K * kC2Ld];
  __shared__ uint32_t rk[kCap];
  const int d = blockIdx.y;
  const int b = S.item_tree[item];
  const int64_t beg = int64_t(tree_ptr[b]) + int64_t(S.item_chunk[item]) * kChunk;
  const int64_t end = min<int64_t>(beg + kChunk, int64_t(tree_ptr[b + 1]));
  const int64_t r = rootindex[b];
  const int rn = S.nnz[r];
  const float sc = keep.scale();
  const int64_t K2 = S.F + H;
  const float* w2t = S.w2t + int64_t(d) * K2 * H;
  if (threadIdx.x < kCap)
    rk[threadIdx.x] = threadIdx.x < rn ? uint32_t(H + S.cols[r * kCap + threadIdx.x]) : 0u;
  for (int e = threadIdx.x; e < H * (H / 4); e += 256) {
    const int k = e >> 4, q = (e & 15) * 4;
    const float4 v = ld4(w2t + int64_t(k) * H + q);
    float* dst = &Bs[k * kC2Ld + q];
    dst[0] = v.x; dst[1] = v.y; dst[2] = v.z; dst[3] = v.w;
  }
  for (int e = threadIdx.x; e < kCap * (H / 4); e += 256) {
    const int s = e >> 4, q = (e & 15) * 4;
    float4 v = f4zero();
    if (s < rn) {
      const float av = sc * fmaxf(S.vals[r * kCap + s], 0.f);
      const float4 w = ld4(w2t + int64_t(H + S.cols[r * kCap + s]) * H + q);
      v = make_float4(av * w.x, av * w.y, av * w.z, av * w.w);
    }
    float* dst = &Bs[(H + s) * kC2Ld + q];
    dst[0] = v.x; dst[1] = v.y; dst[2] = v.z; dst[3] = v.w;
  }
  __syncthreads();

  const int wv = threadIdx.x >> 6, l = threadIdx.x & 63, r32 = l & 31, h = l >> 5;
  for (int t = wv; t < kChunk / 32; t += 4) {
    const int64_t i0 = beg + 32 * t;
    if (i0 >= end) break;
    const int64_t i = i0 + r32;
    const bool ok = i < end;
    const float* hrow = H1 + (ok ? i : beg) * (2 * H) + d * H;
    const uint32_t w0 = ok ? keep.get(uint32_t(d), uint32_t(i), 0u) : 0u;
    const uint32_t w1 = ok ? keep.get(uint32_t(d), uint32_t(i), 1u) : 0u;
    float a[48];
    if (h == 0) {
#pragma unroll
      for (int q = 0; q < 12; ++q) {
        const float4 v = ld4(hrow + 4 * q);
        const float ve[4] = {v.x, v.y, v.z, v.w};
#pragma unroll
        for (int e = 0; e < 4; ++e) {
          const int k = 4 * q + e;
          const uint32_t bit = k < 32 ? (w0 >> k) & 1u : (w1 >> (k - 32)) & 1u;
          a[k] = bit ? sc * fmaxf(ve[e], 0.f) : 0.f;
        }
      }
    } else {
#pragma unroll
      for (int q = 0; q < 4; ++q) {
        const float4 v = ld4(hrow + 48 + 4 * q);
        const float ve[4] = {v.x, v.y, v.z, v.w};
#pragma unroll
        for (int e = 0; e < 4; ++e) {
          const int k = 48 + 4 * q + e;
          a[k - 48] = ((w1 >> (k - 32)) & 1u) ? sc * fmaxf(ve[e], 0.f) : 0.f;
        }
      }
      uint32_t m = 0;
#pragma unroll
      for (int s = 0; s < kCap; ++s) {
        uint32_t bit = 0;
        if (s < rn && ok) {
          const uint32_t k = rk[s];
          bit = (keep.get(uint32_t(d), uint32_t(i), k >> 5) >> (k & 31)) & 1u;
        }
        m |= bit << s;
        a[16 + s] = bit ? 1.f : 0.f;
      }
      if (ok) S.rbits[int64_t(d) * S.N + i] = m;
    }
    f32x16 acc0 = {}, acc1 = {};
    const float* bp = &Bs[(48 * h) * kC2Ld + r32];
#pragma unroll
    for (int kk = 0; kk < 48; ++kk) {
      acc0 = mfma32x32x2(a[kk], bp[kk * kC2Ld], acc0);
      acc1 = mfma32x32x2(a[kk], bp[kk * kC2Ld + 32], acc1);
    }
#pragma unroll
    for (int q = 0; q < 16; ++q) {
      const int64_t ii = i0 + (q & 3) + 8 * (q >> 2) + 4 * h;
      if (ii < end) {
        Z2[ii * (2 * H) + d * H + r32] = acc0[q];
        Z2[ii * (2 * H) + d * H + 32 + r32] = acc1[q];
      }
    }
  }
}


// ---------------------------------------------------------------- dW2 root columns, part 1
// Work item = (tree b, chunk of <= kChunk nodes of b), blockIdx.y = direction:
// part[d][item][s][o] = sum_{i in chunk} keep_i[64 + col_s] * dZ2_d[i][o] for the root's
// non-zeros s (the 2 relu(x) factor is applied in k_dw_cols).
// one block: items per tree = ceil(n_b / kChunk), exclusive scan over trees (1024 at a
// time with a carry), then every tree writes its item descriptors.
__global__ __launch_bounds__(1024) void k_items(SparseState S, const int32_t* __restrict__ tree_ptr) {
  if (!use_sparse(S)) return;
  __shared__ int sh[1024];
  __shared__ int carry;
  if (threadIdx.x == 0) carry = 0;
  __syncthreads();
  for (int64_t b0 = 0; b0 < S.B; b0 += 1024) {
    const int64_t b = b0 + threadIdx.x;
    const int chunks = b < S.B ? (tree_ptr[b + 1] - tree_ptr[b] + kChunk - 1) / kChunk : 0;
    sh[threadIdx.x] = chunks;
    __syncthreads();
    for (int o = 1; o < 1024; o <<= 1) {
      const int v = threadIdx.x >= o ? sh[threadIdx.x - o] : 0;
      __syncthreads();
      sh[threadIdx.x] += v;
      __syncthreads();
    }
    const int first = carry + sh[threadIdx.x] - chunks;
    if (b < S.B) {
      S.tree_item0[b] = first < S.max_items ? first : S.max_items;
      for (int q = 0; q < chunks && first + q < S.max_items; ++q) {
        S.item_tree[first + q] = int32_t(b);
        S.item_chunk[first + q] = q;
      }
    }
    __syncthreads();
    if (threadIdx.x == 1023) carry += sh[1023];
    __syncthreads();
  }
  if (threadIdx.x == 0) S.tree_item0[S.B] = carry < S.max_items ? carry : S.max_items;
}

__global__ __launch_bounds__(256) void k_dw2_root_part(SparseState S, const float* __restrict__ dZ2,
                                                       const int32_t* __restrict__ tree_ptr) {
  if (!use_sparse(S)) return;
  const int item = blockIdx.x;
  if (item >= S.tree_item0[S.B]) return;
  __shared__ uint32_t bits[kChunk];
  __shared__ float red[4][kCap][H];
  const int d = blockIdx.y;
  const int b = S.item_tree[item];
  const int64_t beg = int64_t(tree_ptr[b]) + int64_t(S.item_chunk[item]) * kChunk;
  const int64_t end = min<int64_t>(beg + kChunk, int64_t(tree_ptr[b + 1]));
  // root keep masks of the forward's conv2 (bit s = root non-zero s kept for node i)
  for (int t = threadIdx.x; t < kChunk; t += 256) {
    const int64_t i = beg + t;
    bits[t] = i < end ? S.rbits[int64_t(d) * S.N + i] : 0u;
  }
  __syncthreads();
  const int o = threadIdx.x & 63, sl = threadIdx.x >> 6;   // 64 outputs x 4 node slices
  float acc[kCap];
#pragma unroll
  for (int s = 0; s < kCap; ++s) acc[s] = 0.f;
  // eight independent dZ2 loads in flight per thread (a chunk row is 256 B apart)
  for (int64_t i0 = beg + sl; i0 < end; i0 += 32) {
    float g[8];
#pragma unroll
    for (int u = 0; u < 8; ++u) {
      const int64_t i = i0 + 4 * u;
      g[u] = i < end ? dZ2[i * (2 * H) + d * H + o] : 0.f;
    }
#pragma unroll
    for (int u = 0; u < 8; ++u) {
      const int64_t i = i0 + 4 * u;
      const uint32_t m = i < end ? bits[i - beg] : 0u;
#pragma unroll
      for (int s = 0; s < kCap; ++s) acc[s] += ((m >> s) & 1u) ? g[u] : 0.f;
    }
  }
#pragma unroll
  for (int s = 0; s < kCap; ++s) red[sl][s][o] = acc[s];
  __syncthreads();
  float* out = S.root_part + (int64_t(d) * S.max_items + item) * (kCap * H);
  for (int e = threadIdx.x; e < kCap * H; e += 256) {
    const int s = e / H, oo = e % H;
    out[e] = (red[0][s][oo] + red[1][s][oo]) + (red[2][s][oo] + red[3][s][oo]);
  }
}

// ---------------------------------------------------------------- CSC of X
// Stable counting sort of the non-zeros by column (rows stay in order inside a column):
//   k_csc_hist    per row block (kRowBlock rows): column histogram in LDS -> hist[r][c]
//   k_csc_prefix  per column: exclusive prefix over the row blocks, column totals
//   k_csc_place   per row block: column starts (LDS scan of the totals) + the block's
//                 prefix, then the rows in order, 8 at a time, rank inside the batch
// No float atomics, no general sort; deterministic.
__global__ __launch_bounds__(256) void k_csc_hist(SparseState S) {
  if (!use_sparse(S)) return;
  extern __shared__ __attribute__((aligned(16))) int32_t hsm[];   // [F]
  for (int64_t c = threadIdx.x; c < S.F; c += 256) hsm[c] = 0;
  __syncthreads();
  const int64_t r0 = int64_t(blockIdx.x) * kRowBlock;
  for (int t = threadIdx.x; t < kRowBlock * kCap; t += 256) {
    const int64_t i = r0 + t / kCap;
    const int s = t % kCap;
    if (i < S.N && s < S.nnz[i]) atomicAdd(&hsm[S.cols[i * kCap + s]], 1);
  }
  __syncthreads();
  int32_t* out = S.hist + int64_t(blockIdx.x) * S.F;
  for (int64_t c = threadIdx.x; c < S.F; c += 256) out[c] = hsm[c];
}

// 64 columns x 4 row-block quarters per block; hist[r][c] becomes the exclusive prefix
__global__ __launch_bounds__(256) void k_csc_prefix(SparseState S, int R) {
  if (!use_sparse(S)) return;
  __shared__ int32_t part[4][64];
  const int cl = threadIdx.x & 63, q = threadIdx.x >> 6;
  const int64_t c = int64_t(blockIdx.x) * 64 + cl;
  const int rq = (R + 3) / 4, rb = q * rq, re = min(R, rb + rq);
  int32_t sum = 0;
  if (c < S.F)
    for (int r = rb; r < re; ++r) sum += S.hist[int64_t(r) * S.F + c];
  part[q][cl] = sum;
  __syncthreads();
  int32_t run = 0;
  for (int qq = 0; qq < q; ++qq) run += part[qq][cl];
  if (c < S.F) {
    for (int r = rb; r < re; ++r) {
      const int32_t v = S.hist[int64_t(r) * S.F + c];
      S.hist[int64_t(r) * S.F + c] = run;
      run += v;
    }
    if (q == 3) S.col_total[c] = run;
  }
}

__global__ __launch_bounds__(256) void k_csc_place(SparseState S) {
  if (!use_sparse(S)) return;
  extern __shared__ __attribute__((aligned(16))) int32_t psm[];   // [F] counters, [F] row masks
  int32_t* cnt = psm;
  uint32_t* rows = reinterpret_cast<uint32_t*>(psm + S.F);
  __shared__ int32_t wsum[256];
  // column starts: exclusive scan of col_total (each thread a contiguous run of columns)
  const int64_t F = S.F;
  const int64_t per = (F + 255) / 256;
  const int64_t c0 = threadIdx.x * per, c1 = min<int64_t>(F, c0 + per);
  int32_t local = 0;
  for (int64_t c = c0; c < c1; ++c) local += S.col_total[c];
  wsum[threadIdx.x] = local;
  __syncthreads();
  for (int o = 1; o < 256; o <<= 1) {
    const int32_t v = threadIdx.x >= o ? wsum[threadIdx.x - o] : 0;
    __syncthreads();
    wsum[threadIdx.x] += v;
    __syncthreads();
  }
  int32_t run = wsum[threadIdx.x] - local;
  const int32_t* pre = S.hist + int64_t(blockIdx.x) * F;
  for (int64_t c = c0; c < c1; ++c) {
    const int32_t t = S.col_total[c];
    cnt[c] = run + pre[c];
    rows[c] = 0u;
    if (blockIdx.x == 0) { S.col_start[c] = run; S.col_end[c] = run + t; }
    run += t;
  }
  __syncthreads();
  // rows of the block in order, 32 rows (= 1024 slots, 4 per thread) per batch.  The
  // columns of one row are distinct, so an entry's rank among the batch's entries of
  // its column = the number of earlier batch rows holding that column: an OR of row bits
  // per column (order-independent) + popcount.
  const int64_t r0 = int64_t(blockIdx.x) * kRowBlock;
  constexpr int kBatchRows = 32;
  for (int b = 0; b < kRowBlock; b += kBatchRows) {
    int32_t col[4];
    int rr[4];
#pragma unroll
    for (int k = 0; k < 4; ++k) {
      const int t = threadIdx.x + 256 * k;
      rr[k] = t / kCap;
      const int64_t i = r0 + b + rr[k];
      const int s = t % kCap;
      col[k] = (i < S.N && s < S.nnz[i]) ? S.cols[i * kCap + s] : -1;
      if (col[k] >= 0) atomicOr(&rows[col[k]], 1u << rr[k]);
    }
    __syncthreads();
    int rank[4];
#pragma unroll
    for (int k = 0; k < 4; ++k) {
      rank[k] = -1;
      if (col[k] >= 0) {
        const uint32_t m = rows[col[k]];
        rank[k] = __popc(m & ((1u << rr[k]) - 1u));
        const int64_t i = r0 + b + rr[k];
        S.csc_slot[cnt[col[k]] + rank[k]] = uint32_t(i * kCap + (threadIdx.x + 256 * k) % kCap);
      }
    }
    __syncthreads();
#pragma unroll
    for (int k = 0; k < 4; ++k) {
      if (rank[k] == 0) {   // the batch's first entry of a column advances its counter
        cnt[col[k]] += __popc(rows[col[k]]);
        rows[col[k]] = 0u;
      }
    }
    __syncthreads();
  }
}

// ---------------------------------------------------------------- dW1 + dW2 root columns
// One wave per column c (16 columns per 1024-thread block), the column's non-zeros in
// row order, 64 at a time (lane l loads entry l), 8 dZ1 rows in flight:
//   dW1[:, c]       += x_ic * dZ1[i]                      (lane: outputs 2l, 2l+1)
//   dW2_d[:, 64+c]  += 2 relu(x_ic) * sum_items part_d    (i a root; lane: output l)
__global__ __launch_bounds__(1024) void k_dw_cols(SparseState S, const float* __restrict__ dZ1,
                                                  const int32_t* __restrict__ node_root,
                                                  const int64_t* __restrict__ batch,
                                                  float* __restrict__ dw1_td, float* __restrict__ dw1_bu,
                                                  float* __restrict__ dw2_td, float* __restrict__ dw2_bu,
                                                  float scale) {
  if (!use_sparse(S)) return;
  __shared__ float t1[2 * H][17];
  __shared__ float t2[2][H][17];
  const int wave = threadIdx.x >> 6, lane = threadIdx.x & 63;
  const int64_t c = int64_t(blockIdx.x) * 16 + wave;
  float2 a1 = make_float2(0.f, 0.f);
  float a2[2] = {0.f, 0.f};
  if (c < S.F) {
    const int64_t beg = S.col_start[c], end = S.col_end[c];
    for (int64_t u0 = beg; u0 < end; u0 += 64) {
      const int64_t u = u0 + lane;
      const bool ok = u < end;
      const uint32_t slot = ok ? S.csc_slot[u] : 0u;
      const float x_l = ok ? S.vals[slot] : 0.f;
      const int32_t i_l = int32_t(slot / kCap);
      const int32_t s_l = int32_t(slot % kCap);
      const bool root_l = ok && node_root[i_l] == i_l;
      const int n = int(min<int64_t>(64, end - u0));
      const uint64_t roots = __ballot(root_l);
      for (int j0 = 0; j0 < n; j0 += 8) {
        float2 g[8];
        float x[8];
#pragma unroll
        for (int v = 0; v < 8; ++v) {
          const int j = j0 + v;
          const int32_t i = __shfl(i_l, j < 64 ? j : 0, 64);
          x[v] = j < n ? __shfl(x_l, j < 64 ? j : 0, 64) : 0.f;
          g[v] = j < n ? *reinterpret_cast<const float2*>(dZ1 + int64_t(i) * (2 * H) + 2 * lane)
                       : make_float2(0.f, 0.f);
        }
#pragma unroll
        for (int v = 0; v < 8; ++v) {
          a1.x = fmaf(x[v], g[v].x, a1.x);
          a1.y = fmaf(x[v], g[v].y, a1.y);
        }
      }
      // root rows (rare): dW2 root columns, in row (= tree) order
      uint64_t m = roots;
      while (m) {
        const int j = __builtin_ctzll(m);
        m &= m - 1;
        const int32_t i = __shfl(i_l, j, 64);
        const int32_t s = __shfl(s_l, j, 64);
        const float xv = __shfl(x_l, j, 64);
        const int b = int(batch[i]);
        const float f = scale * fmaxf(xv, 0.f);
#pragma unroll
        for (int d = 0; d < 2; ++d) {
          float sum = 0.f;
          for (int it = S.tree_item0[b]; it < S.tree_item0[b + 1]; ++it)
            sum += S.root_part[(int64_t(d) * S.max_items + it) * (kCap * H) + s * H + lane];
          a2[d] = fmaf(f, sum, a2[d]);
        }
      }
    }
  }
  t1[2 * lane][wave] = a1.x;
  t1[2 * lane + 1][wave] = a1.y;
  t2[0][lane][wave] = a2[0];
  t2[1][lane][wave] = a2[1];
  __syncthreads();
  // coalesced stores: 16 consecutive columns per output row
  const int tx = threadIdx.x & 15, ty = threadIdx.x >> 4;   // 16 x 64
  const int64_t cc = int64_t(blockIdx.x) * 16 + tx;
  if (cc < S.F) {
    const int64_t K2 = S.F + H;
    for (int o = ty; o < 2 * H; o += 64) {
      float* dst = o < H ? dw1_td + int64_t(o) * S.F : dw1_bu + int64_t(o - H) * S.F;
      dst[cc] = t1[o][tx];
    }
    for (int o = ty; o < H; o += 64) {
      dw2_td[int64_t(o) * K2 + H + cc] = t2[0][o][tx];
      dw2_bu[int64_t(o) * K2 + H + cc] = t2[1][o][tx];
    }
  }
}

}  // namespace

// ---------------------------------------------------------------- host side
size_t carve_sparse(Carve& c, int64_t N, int64_t B, int64_t F, SparseState* S) {
  SparseState t{};
  t.N = N;
  t.F = F;
  t.B = B;
  t.max_items = int(N / kChunk + B + 1);
  t.w1t = c.take<float>(size_t(F) * 2 * H);
  t.w2t = c.take<float>(size_t(2) * (F + H) * H);
  t.item_tree = c.take<int32_t>(size_t(t.max_items));
  t.item_chunk = c.take<int32_t>(size_t(t.max_items));
  t.tree_item0 = c.take<int32_t>(size_t(B + 1));
  t.root_part = c.take<float>(size_t(2) * t.max_items * kCap * H);
  const size_t slots = size_t(N) * kCap;
  const size_t R = size_t((N + kRowBlock - 1) / kRowBlock);
  t.hist = c.take<int32_t>(R * size_t(F));
  t.col_total = c.take<int32_t>(size_t(F));
  t.col_start = c.take<int32_t>(size_t(F));
  t.col_end = c.take<int32_t>(size_t(F));
  t.csc_slot = c.take<uint32_t>(slots);
  t.rbits = c.take<uint32_t>(size_t(2) * N);
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

int sparse_transpose(SparseState& S, const bgcn_bigcn_args* a, hipStream_t s) {
  dim3 grid(unsigned((S.F + H + 31) / 32), 2, 4);
  hipLaunchKernelGGL(k_transpose_weights, grid, dim3(256), 0, s, S, a->td_w1, a->bu_w1, a->td_w2,
                     a->bu_w2);
  BGCN_CHECK_LAUNCH();
  return BGCN_OK;
}

int sparse_compact_conv1(SparseState& S, const float* X, int64_t ldx, float* Z1, hipStream_t s) {
  hipLaunchKernelGGL(k_compact_conv1, dim3(grid_for(S.N, 4)), dim3(256), 0, s, S, X, ldx, Z1);
  BGCN_CHECK_LAUNCH();
  return BGCN_OK;
}

int sparse_items(SparseState& S, const int32_t* tree_ptr, hipStream_t s) {
  hipLaunchKernelGGL(k_items, dim3(1), dim3(1024), 0, s, S, tree_ptr);
  BGCN_CHECK_LAUNCH();
  return BGCN_OK;
}

int sparse_conv2(SparseState& S, const float* H1, const int32_t* tree_ptr, const int64_t* rootindex,
                 float* Z2, KeepSrc keep, hipStream_t s) {
  hipLaunchKernelGGL(k_conv2_sparse, dim3(unsigned(S.max_items), 2), dim3(256), 0, s, S, H1,
                     tree_ptr, rootindex, Z2, keep);
  BGCN_CHECK_LAUNCH();
  return BGCN_OK;
}

int sparse_dw2_root_part(SparseState& S, const int32_t* tree_ptr, const float* dZ2, hipStream_t s) {
  hipLaunchKernelGGL(k_dw2_root_part, dim3(unsigned(S.max_items), 2), dim3(256), 0, s, S, dZ2,
                     tree_ptr);
  BGCN_CHECK_LAUNCH();
  return BGCN_OK;
}

int sparse_csc(SparseState& S, hipStream_t s) {
  const int R = int((S.N + kRowBlock - 1) / kRowBlock);
  hipLaunchKernelGGL(k_csc_hist, dim3(unsigned(R)), dim3(256), size_t(S.F) * sizeof(int32_t), s, S);
  BGCN_CHECK_LAUNCH();
  hipLaunchKernelGGL(k_csc_prefix, dim3(grid_for(S.F, 64)), dim3(256), 0, s, S, R);
  BGCN_CHECK_LAUNCH();
  hipLaunchKernelGGL(k_csc_place, dim3(unsigned(R)), dim3(256), size_t(2 * S.F) * sizeof(int32_t), s, S);
  BGCN_CHECK_LAUNCH();
  return BGCN_OK;
}

int sparse_dw_cols(SparseState& S, const bgcn_bigcn_args* a, const float* dZ1,
                   const int32_t* node_root, KeepSrc keep, hipStream_t s) {
  hipLaunchKernelGGL(k_dw_cols, dim3(unsigned((S.F + 15) / 16)), dim3(1024), 0, s, S, dZ1, node_root,
                     a->batch, a->td_dw1, a->bu_dw1, a->td_dw2, a->bu_dw2, keep.scale());
  BGCN_CHECK_LAUNCH();
  return BGCN_OK;
}

}  // namespace bgcn
