// Fused bidirectional BiGCN encoder (TDrumorGCN + BUrumorGCN) forward/backward.
//
// Reference: model/Twitter/BiGCN_Twitter.py:26-67 (TD), :77-114 (BU), :125-128
// (BU-first concat); identical math in model/Weibo/BiGCN_Weibo.py:22-44, :52-74.
//
// Per direction d (TD: edge_index, BU: BU_edge_index):
//   Z1 = X W1^T                      conv1 lin          (fused TD+BU: one pass over X)
//   H1 = A_d Z1 + b1                 conv1 propagate    (:42)
//   A2 = drop(relu([H1 | X[root]]))  root extend, cat, relu, dropout (:45-54) - never
//                                    materialised: generated inside the conv2 GEMM
//   Z2 = A2 W2^T ; H2 = A_d Z2 + b2  conv2 (:56)
//   out = mean_tree([relu(H2) | H1[root]])   (:57-65; H1[root] is the detached x2)
// Backward follows SURVEY.md 8(a) "Gradient dataflow": no gradient reaches conv1
// through the root-extended x2 (copy.copy makes a new leaf, :44).
#include "bgcn_bwd.h"
#include "bgcn_internal.h"
#include "bgcn_sparse.h"
#include "bgcn_trace.h"

namespace bgcn {

namespace {

// (tree_ptr / node_root are built by the forward prologue, k_prologue in bgcn_sparse.hip)

// ---------------------------------------------------------------- conv2 forward
// Z2[:, d*H:(d+1)*H] = A2_d . W2_d^T with A2_d[i][k] generated on the fly:
//   k <  H : keep * s * relu(H1[i][d*H + k])
//   k >= H : keep * s * relu(X[root(i)][k - H])
// Block tile 64 nodes x 64 outputs, waves 2 x 2 (32 x 32 each), blockIdx.y = d.
template <class TX>
__global__ __launch_bounds__(256) void k_conv2_fwd(const TX* __restrict__ X, int64_t ldx,
                                                   int64_t F, const float* __restrict__ H1,
                                                   const int32_t* __restrict__ node_root,
                                                   const float* __restrict__ W2td,
                                                   const float* __restrict__ W2bu,
                                                   float* __restrict__ Z2, int64_t N, KeepSrc keep,
                                                   const int32_t* __restrict__ gate) {
  if (gate_closed(gate)) return;
  constexpr int BM = 64, LS = BK + 1;
  __shared__ float As[2][BM * LS];
  __shared__ float Bs[2][H * LS];
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int wr = wave >> 1, wc = wave & 1;
  const int d = blockIdx.y;
  const float* W2 = d == 0 ? W2td : W2bu;
  const int64_t K2 = H + F, ldw = H + F;
  const int64_t m0 = int64_t(blockIdx.x) * BM;
  const float sc = keep.scale();

  // A generation map: node m = tid/4, 8 consecutive k at 8*(tid%4)
  const int gm = tid >> 2, gk = (tid & 3) * 8;
  const int64_t gi = m0 + gm;
  const bool gok = gi < N;
  const TX* xroot = X + int64_t(gok ? node_root[gi] : 0) * ldx;
  const float* h1row = H1 + (gok ? gi : 0) * (2 * H) + d * H;
  // B staging map: W2 row o = tid/8 + 32 i, k quad (tid%8)*4
  const int so = tid >> 3, sq = (tid & 7) * 4;

  float4 ga[2], rb[2];
  uint32_t gw = 0;
  auto gload = [&](int64_t k0) {
    int64_t k = k0 + gk;
    gw = gok ? keep.get(uint32_t(d), uint32_t(gi), uint32_t(k0 / 32)) : 0u;
#pragma unroll
    for (int j = 0; j < 2; ++j) {
      int64_t kk = k + 4 * j;
      float4 v = f4zero();
      if (gok) {
        if (kk < H) v = ld4(h1row + kk);
        else if (kk - H < F) v = xq(xroot + (kk - H));
      }
      ga[j] = v;
    }
#pragma unroll
    for (int i = 0; i < 2; ++i) {
      int64_t kk = k0 + sq;
      rb[i] = kk < K2 ? ld4(W2 + int64_t(so + 32 * i) * ldw + kk) : f4zero();
    }
  };
  auto sstore = [&](int buf) {
    float* a = &As[buf][gm * LS + gk];
#pragma unroll
    for (int j = 0; j < 2; ++j) {
      float v[4] = {ga[j].x, ga[j].y, ga[j].z, ga[j].w};
#pragma unroll
      for (int e = 0; e < 4; ++e) {
        int bit = gk + 4 * j + e;
        a[4 * j + e] = ((gw >> bit) & 1u) ? sc * fmaxf(v[e], 0.f) : 0.f;
      }
    }
#pragma unroll
    for (int i = 0; i < 2; ++i) {
      float* b = &Bs[buf][(so + 32 * i) * LS + sq];
      b[0] = rb[i].x; b[1] = rb[i].y; b[2] = rb[i].z; b[3] = rb[i].w;
    }
  };

  f32x16 acc = {0};
  const int h = lane >> 5, r32 = lane & 31;
  const int nk = int((K2 + BK - 1) / BK);
  gload(0);
  sstore(0);
  __syncthreads();
  for (int kt = 0; kt < nk; ++kt) {
    const int buf = kt & 1;
    if (kt + 1 < nk) gload(int64_t(kt + 1) * BK);
    const float* A = &As[buf][(wr * 32 + r32) * LS + h];
    const float* B = &Bs[buf][(wc * 32 + r32) * LS + h];
#pragma unroll
    for (int s = 0; s < BK / 2; ++s) acc = mfma32x32x2(A[2 * s], B[2 * s], acc);
    if (kt + 1 < nk) sstore(buf ^ 1);
    __syncthreads();
  }
#pragma unroll
  for (int r = 0; r < 16; ++r) {
    int64_t m = m0 + wr * 32 + acc_row(r, lane);
    if (m < N) Z2[m * (2 * H) + d * H + wc * 32 + r32] = acc[r];
  }
}

// The same conv2 for bf16 X on the bf16 MFMA (v_mfma_f32_32x32x16_bf16).  Block = 128 nodes
// x the 64 outputs of direction d = blockIdx.y; wave w takes nodes [32w, 32w + 32) and both
// 32-wide output tiles.  Lane map: lane (h = l >> 5, r = l & 31) supplies A[r][8h + j] and
// B[8h + j][r]; D register q is D[(q & 3) + 8 (q >> 2) + 4h][r].
//   k < 64, the H1 block: A = keep * s * relu(H1) is fp32 - each lane builds its fragments
//     straight from global memory (8 consecutive H1 values, its keep word) and from W2's
//     rows (8 consecutive k of output r), both split three ways: six products (mfma_x6),
//     fp32-grade (conv2's output feeds a relu).
//   k >= 64, the root block, in 32-wide k-tiles aligned to the keep words: A = keep * s *
//     relu(x_root) is exact in bf16 (bag-of-words counts, s = 2), so three products against
//     W2 split three ways.  A staged as 16-byte pieces of one node's row per lane on
//     consecutive nodes, B as one W2 row's 8 consecutive k per lane on consecutive rows
//     (row stride kC2fLd: conflict-free 16-byte LDS stores); the next tile's global loads
//     are in flight during the current tile's MFMAs.
constexpr int kC2fBK = 32, kC2fLd = kC2fBK + 8;
// The dense conv2's root block for fp32 X: every node of a tree reads the same root row, so
// s * relu(x_root) is split three ways once per tree (R[b][p][c], rows zero-padded to ldr,
// a multiple of the k-tile) and each node only masks the planes by its keep bits - the
// split was most of the kernel's VALU work (14 VALU instructions per MFMA, r04_dense_pmc).
__global__ __launch_bounds__(256) void k_root_split(const float* __restrict__ X, int64_t ldx, int64_t F,
                                                    const int64_t* __restrict__ rootindex, int64_t B, float sc,
                                                    uint16_t* __restrict__ R, int64_t ldr,
                                                    const int32_t* __restrict__ gate) {
  if (gate_closed(gate)) return;
  const int64_t b = blockIdx.y;
  const int64_t c = int64_t(blockIdx.x) * 256 + threadIdx.x;
  if (b >= B || c >= ldr) return;
  const int64_t root = rootindex[b];
  const float v = (c < F && root >= 0) ? sc * fmaxf(X[root * ldx + c], 0.f) : 0.f;
  __bf16 h, m, l;
  split3_bf16(v, h, m, l);
  uint16_t* r = R + b * 3 * ldr + c;
  r[0] = __builtin_bit_cast(uint16_t, h);
  r[ldr] = __builtin_bit_cast(uint16_t, m);
  r[2 * ldr] = __builtin_bit_cast(uint16_t, l);
}
template <class TX, bool kR = false>
__global__ __launch_bounds__(256) void k_conv2_fwd_bf16(const TX* __restrict__ X, int64_t ldx, int64_t F,
                                                        const float* __restrict__ H1,
                                                        const int32_t* __restrict__ node_root,
                                                        const float* __restrict__ W2td,
                                                        const float* __restrict__ W2bu,
                                                        float* __restrict__ Z2, int64_t N, KeepSrc keep,
                                                        const int32_t* __restrict__ gate,
                                                        const uint16_t* __restrict__ R = nullptr, int64_t ldr = 0,
                                                        const int64_t* __restrict__ batch = nullptr) {
  if (gate_closed(gate)) return;
  constexpr int BM = 128, PX = sizeof(TX) == 2 ? 1 : 3;   // A planes: bf16 X exact, fp32 X split
  __shared__ __attribute__((aligned(16))) __bf16 As[PX][BM * kC2fLd];
  __shared__ __attribute__((aligned(16))) __bf16 Bs[3][H * kC2fLd];
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int h = lane >> 5, r32 = lane & 31;
  const int d = blockIdx.y;
  const float* W2 = d == 0 ? W2td : W2bu;
  const int64_t ldw = H + F;
  const int64_t m0 = int64_t(blockIdx.x) * BM;
  const float sc = keep.scale();
  f32x16 acc[2] = {};

  {   // the H1 block (k < 64): fragments from global memory, six products
    const int64_t m = m0 + 32 * wave + r32;
    const bool mok = m < N;
    const float* hrow = H1 + (mok ? m : 0) * (2 * H) + d * H;
#pragma unroll
    for (int s = 0; s < H / 16; ++s) {
      const int k = 16 * s + 8 * h;
      const uint32_t wd = mok ? keep.get(uint32_t(d), uint32_t(m), uint32_t(k >> 5)) : 0u;
      const float4 x0 = ld4(hrow + k), x1 = ld4(hrow + k + 4);
      const float xa[8] = {x0.x, x0.y, x0.z, x0.w, x1.x, x1.y, x1.z, x1.w};
      bf16x8 ah, am, al;
#pragma unroll
      for (int j = 0; j < 8; ++j) {
        const float a = ((wd >> ((k + j) & 31)) & 1u) ? sc * fmaxf(xa[j], 0.f) : 0.f;
        __bf16 p, q, t;
        split3_bf16(a, p, q, t);
        ah[j] = p; am[j] = q; al[j] = t;
      }
#pragma unroll
      for (int c = 0; c < 2; ++c) {
        const float* wrow = W2 + int64_t(32 * c + r32) * ldw + k;
        const float4 w0 = ld4(wrow), w1 = ld4(wrow + 4);
        const float wa[8] = {w0.x, w0.y, w0.z, w0.w, w1.x, w1.y, w1.z, w1.w};
        bf16x8 bh, bm, bl;
#pragma unroll
        for (int j = 0; j < 8; ++j) {
          __bf16 p, q, t;
          split3_bf16(wa[j], p, q, t);
          bh[j] = p; bm[j] = q; bl[j] = t;
        }
        acc[c] = mfma_x6(ah, am, al, bh, bm, bl, acc[c]);
      }
    }
  }

  // the root block: k-tiles of 32 A2 columns (64 + 32t ..), keep word 2 + t
  const int ar = tid & (BM - 1), ak = (tid >> 7) * 16;         // A: node ar, columns ak .. ak + 15
  const int64_t am_ = m0 + ar;
  const bool aok = am_ < N;
  const TX* xrow = X + int64_t(aok ? node_root[am_] : 0) * ldx;
  const int br = tid & (H - 1), bk = (tid >> 6) * 8;           // B: W2 row br, k bk .. bk + 7
  const float* wrow = W2 + int64_t(br) * ldw + H;
  constexpr int kRA = 2 * sizeof(TX) / 2;   // 16-byte X pieces per thread (16 columns)
  constexpr int kPE = 8 / (sizeof(TX) / 2); // X elements per piece
  u32x4 ra[kR ? 6 : kRA];   // kR: the tree's split planes of s relu(x_root), 3 x 2 pieces
  uint32_t rw = 0;
  float4 rb[2];
  const uint16_t* rrow = nullptr;
  if constexpr (kR) rrow = R + (aok ? batch[am_] : 0) * 3 * ldr;
  auto gload = [&](int64_t c0) {   // c0: first X column of the tile
    rw = aok ? keep.get(uint32_t(d), uint32_t(am_), uint32_t((H + c0) >> 5)) : 0u;
    if constexpr (kR) {   // (R rows are zero-padded to ldr >= the last tile's end)
#pragma unroll
      for (int p = 0; p < 3; ++p)
#pragma unroll
        for (int i = 0; i < 2; ++i)
          ra[2 * p + i] = *reinterpret_cast<const u32x4*>(rrow + p * ldr + c0 + ak + 8 * i);
    } else {
#pragma unroll
      for (int i = 0; i < kRA; ++i) {
        const int64_t c = c0 + ak + kPE * i;
        const bool ok = aok && c < F;
        const u32x4 v = *reinterpret_cast<const u32x4*>(xrow + (ok ? c : 0));
        ra[i] = ok ? v : u32x4{0u, 0u, 0u, 0u};
      }
    }
#pragma unroll
    for (int i = 0; i < 2; ++i) {
      const int64_t c = c0 + bk + 4 * i;
      const bool ok = c < F;   // F % 4 == 0
      const float4 v = ld4(wrow + (ok ? c : 0));
      rb[i] = ok ? v : f4zero();
    }
  };
  auto sstore = [&]() {
    if constexpr (kR) {   // keep * (the tree's planes): a 16-bit mask per element, no split
#pragma unroll
      for (int i = 0; i < 2; ++i) {
        u32x4 m;
#pragma unroll
        for (int q = 0; q < 4; ++q) {
          const uint32_t bits = (rw >> (ak + 8 * i + 2 * q)) & 3u;
          m[q] = ((bits & 1u) ? 0x0000ffffu : 0u) | ((bits & 2u) ? 0xffff0000u : 0u);
        }
#pragma unroll
        for (int p = 0; p < 3; ++p) {
          const u32x4 v = ra[2 * p + i];
          *reinterpret_cast<u32x4*>(&As[p][ar * kC2fLd + ak + 8 * i]) =
              u32x4{v[0] & m[0], v[1] & m[1], v[2] & m[2], v[3] & m[3]};
        }
      }
    } else
#pragma unroll
    for (int i = 0; i < 2; ++i) {   // keep * s * relu(x): exact in bf16 for bf16 X (s is 1 or 2)
      bf16x8 v, vm, vl;
#pragma unroll
      for (int j = 0; j < 8; ++j) {
        float x;
        if constexpr (PX == 1) {
          const uint32_t wv = ra[i][j >> 1];
          x = __uint_as_float((j & 1) ? (wv & 0xffff0000u) : (wv << 16));
        } else {
          x = __uint_as_float(ra[2 * i + (j >> 2)][j & 3]);
        }
        const bool kept = (rw >> (ak + 8 * i + j)) & 1u;
        const float a = kept ? sc * fmaxf(x, 0.f) : 0.f;
        if constexpr (PX == 1) {
          v[j] = __bf16(a);
        } else {
          __bf16 p, q, t;
          split3_bf16(a, p, q, t);
          v[j] = p; vm[j] = q; vl[j] = t;
        }
      }
      *reinterpret_cast<bf16x8*>(&As[0][ar * kC2fLd + ak + 8 * i]) = v;
      if constexpr (PX == 3) {
        *reinterpret_cast<bf16x8*>(&As[PX - 2][ar * kC2fLd + ak + 8 * i]) = vm;
        *reinterpret_cast<bf16x8*>(&As[PX - 1][ar * kC2fLd + ak + 8 * i]) = vl;
      }
    }
    bf16x8 hv, mv, lv;
    const float wv[8] = {rb[0].x, rb[0].y, rb[0].z, rb[0].w, rb[1].x, rb[1].y, rb[1].z, rb[1].w};
#pragma unroll
    for (int j = 0; j < 8; ++j) {
      __bf16 p, q, t;
      split3_bf16(wv[j], p, q, t);
      hv[j] = p; mv[j] = q; lv[j] = t;
    }
    const int o = br * kC2fLd + bk;
    *reinterpret_cast<bf16x8*>(&Bs[0][o]) = hv;
    *reinterpret_cast<bf16x8*>(&Bs[1][o]) = mv;
    *reinterpret_cast<bf16x8*>(&Bs[2][o]) = lv;
  };
  const int nk = int((F + kC2fBK - 1) / kC2fBK);
  gload(0);
  sstore();
  __syncthreads();
  for (int kt = 0; kt < nk; ++kt) {
    if (kt + 1 < nk) gload(int64_t(kt + 1) * kC2fBK);
#pragma unroll
    for (int s = 0; s < kC2fBK / 16; ++s) {
      const int ko = 16 * s + 8 * h;
      bf16x8 a[PX];
#pragma unroll
      for (int p = 0; p < PX; ++p) a[p] = *reinterpret_cast<const bf16x8*>(&As[p][(32 * wave + r32) * kC2fLd + ko]);
#pragma unroll
      for (int c = 0; c < 2; ++c) {
        const int o = (32 * c + r32) * kC2fLd + ko;
        const bf16x8 b0 = *reinterpret_cast<const bf16x8*>(&Bs[0][o]);
        const bf16x8 b1 = *reinterpret_cast<const bf16x8*>(&Bs[1][o]);
        const bf16x8 b2 = *reinterpret_cast<const bf16x8*>(&Bs[2][o]);
        if constexpr (PX == 1) {
          f32x16 t = acc[c];
          t = mfma_bf16(a[0], b2, t);
          t = mfma_bf16(a[0], b1, t);
          acc[c] = mfma_bf16(a[0], b0, t);
        } else {
          acc[c] = mfma_x6(a[0], a[PX - 2], a[PX - 1], b0, b1, b2, acc[c]);
        }
      }
    }
    __syncthreads();
    if (kt + 1 < nk) {
      sstore();
      __syncthreads();
    }
  }
#pragma unroll
  for (int q = 0; q < 16; ++q) {
    const int64_t m = m0 + 32 * wave + acc_row(q, lane);
    if (m >= N) continue;
#pragma unroll
    for (int c = 0; c < 2; ++c) Z2[m * (2 * H) + d * H + 32 * c + r32] = acc[c][q];
  }
}

// ---------------------------------------------------------------- readout
// head_in[b] = [BU: mean(relu(H2_bu)) | H1_bu[root] , TD: mean(relu(H2_td)) | H1_td[root]]
// One 1024-thread block per tree: per direction 32 row slices x 16 lanes x float4, eight
// independent row loads in flight per slice, then a fixed-order two-level LDS reduction
// (deterministic).  The root half is the mean of identical copies, i.e. H1[root] itself
// (the reference's root_extend is a detached copy, BiGCN_Twitter.py:42-47, so it has no
// backward).  With hd.W set (bgcn_train_step) wave 0 then runs the classifier head on
// the tree's row (head_row): fc, log_softmax, NLL term, dz and dhead.
constexpr int kReadSlices = 32;
__global__ __launch_bounds__(1024) void k_readout_fwd(const float* __restrict__ H1,
                                                      const float* __restrict__ H2,
                                                      const int32_t* __restrict__ tree_ptr,
                                                      const int64_t* __restrict__ rootindex,
                                                      int64_t N, int64_t B, float* __restrict__ head,
                                                      HeadArgs hd) {
  BT_BEGIN
  __shared__ float4 red[2][kReadSlices][16];
  __shared__ float4 red2[2][4][16];
  __shared__ float4 hrow[4 * H / 4];
  const int b = blockIdx.x;
  const int d = threadIdx.x >> 9, t = threadIdx.x & 511;
  const int lane = t & 15, slice = t >> 4;
  const int64_t beg = tree_ptr[b], end = tree_ptr[b + 1];
  const float* src = H2 + d * H + lane * 4;
  float4 s = f4zero();
  int64_t i = beg + slice;
  for (; i + 7 * kReadSlices < end; i += 8 * kReadSlices) {
    float4 v[8];
#pragma unroll
    for (int u = 0; u < 8; ++u) v[u] = ld4(src + (i + u * kReadSlices) * (2 * H));
#pragma unroll
    for (int u = 0; u < 8; ++u) s = f4add(s, f4relu(v[u]));
  }
  for (; i < end; i += kReadSlices) s = f4add(s, f4relu(ld4(src + i * (2 * H))));
  red[d][slice][lane] = s;
  __syncthreads();
  if (t < 64) {
    const int g = t >> 4;
    float4 acc = red[d][g * 8][lane];
#pragma unroll
    for (int q = 1; q < 8; ++q) acc = f4add(acc, red[d][g * 8 + q][lane]);
    red2[d][g][lane] = acc;
  }
  __syncthreads();
  const int base = (d == 1 ? 0 : 2 * H) + lane * 4;  // BU first (:128)
  if (t < 16) {
    float4 acc = red2[d][0][lane];
#pragma unroll
    for (int q = 1; q < 4; ++q) acc = f4add(acc, red2[d][q][lane]);
    const float cnt = float(end - beg > 0 ? end - beg : 1);
    acc = make_float4(acc.x / cnt, acc.y / cnt, acc.z / cnt, acc.w / cnt);
    st4(head + int64_t(b) * (4 * H) + base, acc);
    hrow[base / 4] = acc;
  } else if (t < 32) {
    const int64_t root = rootindex[b];
    const float4 hr = (end > beg && root >= 0 && root < N)
                          ? ld4(H1 + root * (2 * H) + d * H + lane * 4) : f4zero();
    st4(head + int64_t(b) * (4 * H) + base + H, hr);
    hrow[(base + H) / 4] = hr;
  }
  if (hd.W == nullptr) return;
  __syncthreads();
  if (threadIdx.x < 64) head_row(hd, b, B, hrow[threadIdx.x]);
  BT_END(5);
}

// The same readout over tree work items (sparse path: S.item_* exist), so a large tree
// no longer bounds the launch.  Block = one item (<= kChunk nodes of one tree), 512
// threads = 2 directions x 16 row slices x 16 lanes x float4, eight row loads in flight
// per slice.  A tree of one item finishes in its block; otherwise every item stores its
// partial (rpart[item][2H]) and the tree's last arrival (rtick[b], zeroed by the
// prologue / conv1) adds the partials in item order: a fixed order whichever block arrives
// last (deterministic).  Blocks from max_items on cover trees without nodes (mean 0, root
// row 0, head on the bias).
//
// sgn != nullptr (the backward's readout-gradient aggregation follows, SpmmSign): every
// row's relu'(H2) as a sign word per direction (bit 16c + l = column 4l + c) and the item's
// positive counts per column (cnt[item][2H], padding items zero: db2 in the middle launch).
// The readout backward needs no hand-off inside this launch (dhead is read by later
// launches), so item blocks never wait for each other at any batch size.
constexpr int kRoSlices = 16;
// The end of an item block of the readout (k_readout_items): the per-slice
// sums (and sign-mode positive counts) reduced in slice order, the item's counts stored, and
// - when the item completes its tree - the tree's mean row, root half and head.  An item of
// a multi-item tree stores its partial; the tree's last arrival (rtick) adds the partials
// in item order (deterministic whichever block arrives last).
template <int MC, bool kSgn>
__device__ __forceinline__ void readout_item_finish(const SparseState& S, int blk, int64_t b, int item0, int nit,
                                                    float4 s, float4 pc, const int32_t* __restrict__ tree_ptr,
                                                    int64_t N, int64_t B, float* __restrict__ head,
                                                    float* __restrict__ rpart, const HeadArgs& hd,
                                                    float* __restrict__ cnt, const HeadRegs<MC>& hreg,
                                                    float4 hroot, int64_t root, float4 (*red)[kRoSlices][16],
                                                    float4 (*redc)[kRoSlices][16], float4* hrow) {
  const int d = threadIdx.x >> 8, t = threadIdx.x & 255;
  const int lane = t & 15, slice = t >> 4;
  const int dd = (threadIdx.x >> 4) & 1, ll = threadIdx.x & 15;   // wave 0: (dir, lane)
  red[d][slice][lane] = s;
  if (kSgn) redc[d][slice][lane] = pc;
  __syncthreads();
  if (kSgn && blk < S.max_items && slice == 0) {   // the item's counts, slices in order
    float4 acc = redc[d][0][lane];
#pragma unroll
    for (int q = 1; q < kRoSlices; ++q) acc = f4add(acc, redc[d][q][lane]);
    st4(cnt + int64_t(blk) * (2 * H) + d * H + lane * 4, acc);
  }
  if (threadIdx.x >= 64) return;   // wave 0 finishes the item (and the tree)
  bool last = true;
  float4 acc = f4zero();
  if (threadIdx.x < 32) {
    acc = red[dd][0][ll];
#pragma unroll
    for (int q = 1; q < kRoSlices; ++q) acc = f4add(acc, red[dd][q][ll]);
  }
  if (nit > 1) {
    // partials go out as agent-scope atomic stores (write-through past the XCD's L2) and
    // are read back by the last arrival with agent-scope atomic loads: no L2 write-back /
    // invalidate (a __threadfence per block cost the launch 13.7 -> 48 us)
    float* p = rpart + int64_t(blk) * (2 * H) + dd * H + ll * 4;
    if (threadIdx.x < 32) {
      __hip_atomic_store(p + 0, acc.x, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      __hip_atomic_store(p + 1, acc.y, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      __hip_atomic_store(p + 2, acc.z, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      __hip_atomic_store(p + 3, acc.w, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    }
    __atomic_signal_fence(__ATOMIC_SEQ_CST);
    __builtin_amdgcn_s_waitcnt(0);   // the stores are acknowledged before the ticket
    __atomic_signal_fence(__ATOMIC_SEQ_CST);
    int tk = 0;
    if (threadIdx.x == 0)
      tk = __hip_atomic_fetch_add(&S.rtick[b], 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    tk = __shfl(tk, 0, 64);
    last = tk == nit - 1;
    if (last && threadIdx.x < 32) {
      const float* q0 = rpart + int64_t(item0) * (2 * H) + dd * H + ll * 4;
      for (int q = 0; q < nit; ++q) {
        const float* pq = q0 + int64_t(q) * (2 * H);
        const float4 v = make_float4(__hip_atomic_load(pq + 0, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT),
                                     __hip_atomic_load(pq + 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT),
                                     __hip_atomic_load(pq + 2, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT),
                                     __hip_atomic_load(pq + 3, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT));
        acc = q == 0 ? v : f4add(acc, v);
      }
    }
  }
  if (last) {
    const int64_t t0 = tree_ptr[b], t1 = tree_ptr[b + 1];
    const int base = (dd == 1 ? 0 : 2 * H) + ll * 4;   // BU first (:128)
    if (threadIdx.x < 32) {
      const float n = float(t1 - t0 > 0 ? t1 - t0 : 1);
      acc = make_float4(acc.x / n, acc.y / n, acc.z / n, acc.w / n);
      st4(head + b * (4 * H) + base, acc);
      hrow[base / 4] = acc;
    } else {
      const float4 hr = (t1 > t0 && root >= 0 && root < N) ? hroot : f4zero();
      st4(head + b * (4 * H) + base + H, hr);
      hrow[(base + H) / 4] = hr;
    }
    if (hd.W != nullptr) {
      __builtin_amdgcn_s_waitcnt(0xc07f);   // lgkmcnt(0): wave 0's hrow writes have landed
      __builtin_amdgcn_wave_barrier();
      head_row(hd, b, B, hrow[threadIdx.x], hreg);
    }
  }
}

// kSgn = (sgn != nullptr), a template argument so no run-time test sits between the row
// loads and their use
template <int MC, bool kSgn>   // MC: classes of the head held in registers (HeadRegs)
__global__ __launch_bounds__(512, MC <= 4 ? 4 : 2) void k_readout_items(SparseState S, const float* __restrict__ H1,
                                                       const float* __restrict__ H2,
                                                       const int32_t* __restrict__ tree_ptr,
                                                       const int64_t* __restrict__ rootindex,
                                                       int64_t N, int64_t B, float* __restrict__ head,
                                                       float* __restrict__ rpart, HeadArgs hd,
                                                       float* __restrict__ cnt, uint64_t* __restrict__ sgn) {
  BT_BEGIN
  __shared__ float4 red[2][kRoSlices][16];
  __shared__ float4 redc[2][kRoSlices][16];
  __shared__ float4 hrow[4 * H / 4];
  const int blk = int(blockIdx.x);
  int64_t b, beg, end;
  int item0 = 0, nit = 1;
  if (blk < S.max_items) {
    if (blk >= S.tree_item0[S.B]) {
      if (kSgn && threadIdx.x < 2 * H) cnt[int64_t(blk) * (2 * H) + threadIdx.x] = 0.f;
      return;
    }
    b = S.item_tree[blk];
    beg = S.item_beg[blk];
    end = S.item_end[blk];
    item0 = S.tree_item0[b];
    nit = S.tree_item0[b + 1] - item0;
  } else {
    b = blk - S.max_items;
    if (b >= B || tree_ptr[b + 1] > tree_ptr[b]) return;   // trees with nodes have items
    beg = end = tree_ptr[b];
  }
  const int d = threadIdx.x >> 8, t = threadIdx.x & 255;
  const int lane = t & 15, slice = t >> 4;
  const int dd = (threadIdx.x >> 4) & 1, ll = threadIdx.x & 15;   // wave 0: (dir, lane)
  // wave 0 issues the tree's tail operands first (root row of H1, the head's W / bias /
  // label), so they arrive under the row loads instead of after them
  HeadRegs<MC> hreg;
  float4 hroot = f4zero();
  int64_t root = 0;
  if (threadIdx.x < 64) {
    if (hd.W != nullptr) head_load(hd, b, hreg);
    root = rootindex[b];
    hroot = ld4(H1 + (root >= 0 && root < N ? root : 0) * (2 * H) + dd * H + ll * 4);
  }
  const float* src = H2 + d * H + lane * 4;
  float4 s = f4zero();
  float4 pc = f4zero();   // sgn: positive-H2 counts of this thread's columns
  for (int64_t i = beg + slice; i < end; i += 8 * kRoSlices) {
    float4 v[8];
#pragma unroll
    for (int u = 0; u < 8; ++u) v[u] = ld4(src + min<int64_t>(i + u * kRoSlices, end - 1) * (2 * H));
#pragma unroll
    for (int u = 0; u < 8; ++u) {
      const bool ok = i + u * kRoSlices < end;
      if (ok) s = f4add(s, f4relu(v[u]));
      if constexpr (kSgn) {
        // the row's sign word from four ballots over the wave's 4 row slices x 16 lanes;
        // lane 0 of each slice stores its row's word
        const int sh = 16 * (slice & 3);
        const uint64_t b0 = (__ballot(ok && v[u].x > 0.f) >> sh) & 0xffffull;
        const uint64_t b1 = (__ballot(ok && v[u].y > 0.f) >> sh) & 0xffffull;
        const uint64_t b2 = (__ballot(ok && v[u].z > 0.f) >> sh) & 0xffffull;
        const uint64_t b3 = (__ballot(ok && v[u].w > 0.f) >> sh) & 0xffffull;
        if (ok && lane == 0) sgn[(i + u * kRoSlices) * 2 + d] = b0 | (b1 << 16) | (b2 << 32) | (b3 << 48);
        if (ok) pc = f4add(pc, make_float4(float(v[u].x > 0.f), float(v[u].y > 0.f), float(v[u].z > 0.f),
                                           float(v[u].w > 0.f)));
      }
    }
  }
  readout_item_finish<MC, kSgn>(S, blk, b, item0, nit, s, pc, tree_ptr, N, B, head, rpart, hd, cnt, hreg, hroot,
                                root, red, redc, hrow);
  BT_END(5);
}

// dH2[i][d*H + f] = dhead[b(i)][r1 block of d][f] / cnt_b * [H2 > 0]; block partial
// column sums -> colpart[blk][2H].  256 threads = 8 row phases x 32 lanes x float4; a
// block covers kReadBwdRows rows, every thread's rows are loaded before use.  Blocks
// from nblk on run the classifier head's weight gradients (hj, bgcn_train_step).
constexpr int kReadBwdRows = 64;
__global__ __launch_bounds__(256) void k_readout_bwd(const float* __restrict__ dhead,
                                                     const float* __restrict__ H2,
                                                     const int64_t* __restrict__ batch,
                                                     const int32_t* __restrict__ tree_ptr,
                                                     int64_t N, int64_t B,
                                                     float* __restrict__ dH2,
                                                     float* __restrict__ colpart,
                                                     int nblk, HeadGradJob hj) {
  BT_BEGIN
  if (int(blockIdx.x) >= nblk) {
    __shared__ __attribute__((aligned(16))) float hsm[kHeadGradSmem];
    head_grad_block(hj, int(blockIdx.x) - nblk, hsm);
    return;
  }
  constexpr int kPer = kReadBwdRows / 8;
  __shared__ float4 red[8][32];
  const int l = threadIdx.x & 31, ph = threadIdx.x >> 5;
  const int c = l * 4, d = c / H, f = c % H;
  const int hoff = (d == 1 ? 0 : 2 * H) + f;
  const int64_t r0 = int64_t(blockIdx.x) * kReadBwdRows;
  // unconditional loads from clamped rows / trees (see k_dh1), selects afterwards
  int64_t bt[kPer];
  float4 h2[kPer];
#pragma unroll
  for (int u = 0; u < kPer; ++u) {
    const int64_t i = min<int64_t>(r0 + ph + 8 * u, N - 1);
    bt[u] = batch[i];
    h2[u] = ld4(H2 + i * (2 * H) + c);
  }
  int32_t t0[kPer], t1[kPer];
  float4 dh[kPer];
#pragma unroll
  for (int u = 0; u < kPer; ++u) {
    const int64_t b = min<int64_t>(max<int64_t>(bt[u], 0), B - 1);
    t0[u] = tree_ptr[b];
    t1[u] = tree_ptr[b + 1];
    dh[u] = ld4(dhead + b * (4 * H) + hoff);
  }
  float4 cs = f4zero();
#pragma unroll
  for (int u = 0; u < kPer; ++u) {
    const int64_t i = r0 + ph + 8 * u;
    const bool ok = i < N && bt[u] >= 0 && bt[u] < B;
    const float cnt = float(max(t1[u] - t0[u], 1));
    float4 g;
    g.x = ok && h2[u].x > 0.f ? dh[u].x / cnt : 0.f;
    g.y = ok && h2[u].y > 0.f ? dh[u].y / cnt : 0.f;
    g.z = ok && h2[u].z > 0.f ? dh[u].z / cnt : 0.f;
    g.w = ok && h2[u].w > 0.f ? dh[u].w / cnt : 0.f;
    if (i < N) st4(dH2 + i * (2 * H) + c, g);
    cs = f4add(cs, g);
  }
  red[ph][l] = cs;
  __syncthreads();
  if (ph == 0) {
    float4 acc = red[0][l];
#pragma unroll
    for (int q = 1; q < 8; ++q) acc = f4add(acc, red[q][l]);
    st4(colpart + int64_t(blockIdx.x) * (2 * H) + c, acc);
  }
  BT_END(6);
}

// out_td[c] = sum_p colpart[p][c], out_bu[c] = sum_p colpart[p][H + c]: one block per
// column, strided partial sums + a fixed LDS tree (deterministic).
__global__ __launch_bounds__(256) void k_colsum_reduce(const float* __restrict__ colpart, int P,
                                                       float* __restrict__ out_td,
                                                       float* __restrict__ out_bu) {
  __shared__ float red[256];
  const int c = blockIdx.x;
  float acc = 0.f;
  for (int p = threadIdx.x; p < P; p += 256) acc += colpart[int64_t(p) * (2 * H) + c];
  red[threadIdx.x] = acc;
  __syncthreads();
  for (int o = 128; o > 0; o >>= 1) {
    if (threadIdx.x < o) red[threadIdx.x] += red[threadIdx.x + o];
    __syncthreads();
  }
  if (threadIdx.x == 0) {
    if (c < H) out_td[c] = red[0]; else out_bu[c - H] = red[0];
  }
}

__global__ void k_keep_words(uint64_t seed, int64_t N, int nw, uint32_t* __restrict__ words) {
  int64_t idx = int64_t(blockIdx.x) * blockDim.x + threadIdx.x;
  if (idx >= 2 * N * nw) return;
  int w = int(idx % nw);
  int64_t rest = idx / nw;
  int64_t node = rest % N;
  int d = int(rest / N);
  words[idx] = keep_word(seed, uint32_t(d), uint32_t(node), uint32_t(w));
}

// ---------------------------------------------------------------- workspace

struct FusedWs {
  int32_t* node_root;
  float *z1, *z2, *d2, *dz2, *dh1, *dz1;  // [N, 2H]
  float* colpart;                         // [nblk, 2H] db1 partials (k_dh1)
  float* colpart2;                        // [nblk, 2H] db2 partials (k_readout_bwd)
  float* rpart;                           // [max_items, 2H] readout partials (k_readout_items)
  int32_t* rtick;                         // [B] readout arrival counters
  float* spmm_ws; size_t spmm_bytes;
  float* dw2_part;                        // [2][S2][H][H+F]
  float* tn_ws; size_t tn_bytes;
  uint16_t* rplanes;                      // dense conv2, fp32 X: the trees' split root rows (k_root_split)
  int S2; int64_t kchunk2;
  int S2d; int64_t kchunk2d;              // the dense feature mode's dW2 node splits (more: shorter loops)
  int Sh; int64_t kchunkh;
  SpmmPlan plan[2][2];                    // [td, bu][forward, backward] (prepared batch) or null
  // [td, bu] status words of graph builds that checked tree-locality (the prepared batch's,
  // or bgcn_graph_view.tree_status); either null: the sign-word readout backward is off
  const int32_t* tree_status[2];
};

int dw2_splits(int64_t N, int64_t F) {
  int64_t tiles = 2 * ((H + F + 63) / 64);
  int64_t want = (5 * 256 + tiles - 1) / tiles;
  int64_t maxs = (N + BK - 1) / BK;
  int64_t s = want < maxs ? want : maxs;
  return int(s < 1 ? 1 : (s > 64 ? 64 : s));
}

size_t carve_fused(Carve& c, int64_t N, int64_t B, int64_t F, FusedWs* w) {
  FusedWs t;
  const size_t nm = size_t(N) * 2 * H;
  int64_t cap = 2 * N + 4;  // spmm capacity upper bound is set per call; see spmm_capacity
  (void)cap;
  t.node_root = c.take<int32_t>(size_t(N));
  t.z1 = c.take<float>(nm);
  t.z2 = c.take<float>(nm);
  t.d2 = c.take<float>(nm);
  t.dz2 = c.take<float>(nm);
  t.dh1 = c.take<float>(nm);
  t.dz1 = c.take<float>(nm);
  const int64_t nblk = std::max((N + kDh1Rows - 1) / kDh1Rows,
                                 (N + kReadBwdRows - 1) / kReadBwdRows);
  t.colpart = c.take<float>(size_t(nblk) * 2 * H);
  t.colpart2 = c.take<float>(size_t(std::max<int64_t>(nblk, N / kChunk + B + 1)) * 2 * H);   // (max_items)
  t.rpart = c.take<float>(size_t(N / kChunk + B + 1) * 2 * H);   // max_items (carve_sparse)
  t.rtick = c.take<int32_t>(size_t(B));
  t.S2 = dw2_splits(N, F);
  int64_t kc = (N + t.S2 - 1) / t.S2;
  kc = (kc + BK - 1) / BK * BK;
  if (kc == 0) kc = BK;
  t.kchunk2 = kc;
  t.S2 = int((N + kc - 1) / kc);
  if (t.S2 < 1) t.S2 = 1;
  // dense feature mode: node splits of >= 2048 nodes, at most 32 (its dW2 blocks loop over
  // a split's nodes: 8 splits left 400+ serial k-tiles per block at Weibo size)
  {
    static const int64_t kd_env = [] { const char* e = std::getenv("BGCN_DW2D_NODES"); return e ? int64_t(atol(e)) : 0; }();
    int64_t kd = kd_env > 0 ? kd_env : std::max<int64_t>(2048, (N + 31) / 32);   // (env: A/B runs)
    kd = (kd + 63) / 64 * 64;
    t.kchunk2d = kd;
    t.S2d = int(std::max<int64_t>(1, (N + kd - 1) / kd));
    if (t.S2d < t.S2) { t.S2d = t.S2; t.kchunk2d = t.kchunk2; }
  }
  // sparse path: relu(H1) block of dW2 over node splits of >= 128 nodes (partial rows of
  // 64), at most ~kDw2MaxSplits splits: every split writes a 2 x 64 x 64 partial that the
  // tail re-reads (118k nodes: 922 splits = 30 MB of partials at 128 nodes each)
#ifndef BGCN_DW2_MAX_SPLITS
#define BGCN_DW2_MAX_SPLITS 256
#endif
  // (whole 64-row dH1 tiles: the split's dH1 block forms its dW2 partial, bgcn_bwd.h)
  t.kchunkh = std::max<int64_t>(128, ((N + BGCN_DW2_MAX_SPLITS - 1) / BGCN_DW2_MAX_SPLITS + 63) / 64 * 64);
  t.Sh = int((N + t.kchunkh - 1) / t.kchunkh);
  if (t.Sh < 1) t.Sh = 1;
  const size_t dense_part = size_t(2) * std::max(t.S2, t.S2d) * H * (H + F), sparse_part = size_t(2) * t.Sh * H * H;
  t.dw2_part = c.take<float>(dense_part > sparse_part ? dense_part : sparse_part);
  t.tn_bytes = tn_ws_size(2 * H, F, N);
  t.tn_ws = c.take<float>(t.tn_bytes / sizeof(float) + 1);
  t.rplanes = c.take<uint16_t>(size_t(B) * 3 * size_t((F + kC2fBK - 1) / kC2fBK * kC2fBK));
  if (w) *w = t;
  return c.off;
}

// the spmm scratch depends on the graph capacity (E + N), carved after the fixed part
size_t fused_ws_fixed(int64_t N, int64_t B, int64_t F) {
  Carve c(nullptr, 0);
  carve_fused(c, N, B, F, nullptr);
  carve_sparse(c, N, B, F, nullptr);
  return c.off;
}

// prepared: the batch comes prepared (bgcn_train_step); under BGCN_FEAT_SPARSE its x is then
// never read and may be NULL (host-fed compacted features)
int check_args(const bgcn_bigcn_args* a, bool prepared = false) {
  const bool need_x = !(prepared && a->feat_mode == BGCN_FEAT_SPARSE);
  BGCN_CHECK_ARG(a, "null args");
  BGCN_CHECK_ARG(a->hid == H, "fused path requires hid == out == 64");
  BGCN_CHECK_ARG(a->num_nodes > 0 && a->num_graphs > 0 && a->in_feats > 0, "bad sizes");
  BGCN_CHECK_ARG(a->in_feats % 4 == 0 && a->ldx % 4 == 0 && a->ldx >= a->in_feats,
                 "in_feats and ldx must be multiples of 4");
  BGCN_CHECK_ARG((a->x || !need_x) && a->batch && a->rootindex && a->tree_ptr && a->h1 && a->h2,
                 "null pointer");
  BGCN_CHECK_ARG(a->x_dtype == BGCN_DTYPE_F32 || a->x_dtype == BGCN_DTYPE_BF16, "bad x_dtype");
  BGCN_CHECK_ARG((reinterpret_cast<uintptr_t>(a->x) & 15) == 0, "x must be 16-byte aligned");
  BGCN_CHECK_ARG(a->td.t_ptr && a->bu.t_ptr && a->td.s_ptr && a->bu.s_ptr, "null graph");
  BGCN_CHECK_ARG(a->feat_mode == BGCN_FEAT_AUTO || a->feat_mode == BGCN_FEAT_DENSE ||
                     a->feat_mode == BGCN_FEAT_SPARSE, "bad feat_mode");
  BGCN_CHECK_ARG(a->feat_mode != BGCN_FEAT_SPARSE || (a->in_feats <= kSparseMaxF && a->num_nodes <= kSparseMaxN),
                 "BGCN_FEAT_SPARSE needs in_feats <= 5120");
  return BGCN_OK;
}

KeepSrc make_keep(const bgcn_bigcn_args* a) {
  KeepSrc k;
  k.words = a->keep_words;
  k.seed = a->seed;
  k.num_nodes = a->num_nodes;
  k.nw = int32_t((a->hid + a->in_feats + 31) / 32);
  k.training = a->training ? 1 : 0;
  return k;
}

}  // namespace

size_t bigcn_ws_size(int64_t N, int64_t B, int64_t F, int64_t hid) {
  (void)hid;
  // spmm scratch sized for the largest possible graph of N nodes (a forest has at
  // most N - 1 edges; allow E <= 4N for general inputs)
  return fused_ws_fixed(N, B, F) + 256 + spmm_ws_size(5 * N + 64, 2 * H);
}

// TD (columns [0, H)) and BU (columns [H, 2H)) aggregations of one [N, 2H] matrix in
// one launch; `transposed` selects A^T (backward).
static SpmmBatch pair_batch(const bgcn_graph_view& td, const bgcn_graph_view& bu, bool transposed,
                            int64_t N, const float* in, float* out, const float* bias_td,
                            const float* bias_bu, int epi, FusedWs& w) {
  const size_t half = w.spmm_bytes / 2 / 256 * 256;
  SpmmBatch sb{};
  sb.rows = N;
  sb.F = H;
  sb.epi = epi;
  const bgcn_graph_view* g[2] = {&td, &bu};
  for (int d = 0; d < 2; ++d) {
    const bgcn_graph_view& v = *g[d];
    sb.p[d] = SpmmProb{transposed ? v.s_ptr : v.t_ptr, transposed ? v.s_row : v.t_row,
                       transposed ? v.s_col : v.t_col, transposed ? v.s_w : v.t_w,
                       in + d * H, 2 * H, out + d * H, 2 * H, d == 0 ? bias_td : bias_bu,
                       reinterpret_cast<float*>(reinterpret_cast<char*>(w.spmm_ws) + d * half),
                       spmm_groups(v.capacity, H), v.capacity, w.plan[d][transposed ? 1 : 0]};
  }
  return sb;
}

static int spmm_pair(const bgcn_graph_view& td, const bgcn_graph_view& bu, bool transposed,
                     int64_t N, const float* in, float* out, const float* bias_td,
                     const float* bias_bu, int epi, FusedWs& w, hipStream_t s,
                     const SpmmSign* sign = nullptr) {
  const size_t half = w.spmm_bytes / 2 / 256 * 256;
  BGCN_CHECK_ARG(spmm_ws_size(td.capacity, H) <= half && spmm_ws_size(bu.capacity, H) <= half,
                 "graph capacity exceeds workspace");
  SpmmBatch sb = pair_batch(td, bu, transposed, N, in, out, bias_td, bias_bu, epi, w);
  if (sign) sb.sg = *sign;
  return spmm_batch_impl(sb, 2, s);
}

// The sparse path's readout backward rides in the backward's first aggregation (dZ2 =
// A^T dH2 from the readout's H2 sign words, SpmmSign) whenever that aggregation takes K1's
// plans: no dH2 round trip, no k_readout_bwd launch.  The forward's readout then stores the
// sign words (in the dH2 buffer, unused on this path) and per-item positive counts (db2 =
// sum over items of count x dhead / tree size, the middle launch).  BGCN_READOUT_SIGN=0
// (read per call) keeps k_readout_bwd / the fused readout.
static bool readout_sign(const bgcn_bigcn_args* a, const SparseState& sp, FusedWs& w) {
  if (sp.mode == 1) return false;
  // the graphs' builds must have checked tree-locality (a cross-tree edge then switches the
  // aggregation to per-neighbour tree scales on the device); unchecked graphs keep
  // k_readout_bwd, which handles any edge set
  if (!w.tree_status[0] || !w.tree_status[1]) return false;
  const char* e = std::getenv("BGCN_READOUT_SIGN");
  if (e && atoi(e) == 0) return false;
  const SpmmBatch sb = pair_batch(a->td, a->bu, true, a->num_nodes, nullptr, nullptr, nullptr, nullptr,
                                  BGCN_EPI_NONE, w);
  return spmm_planned(sb, 2);
}

// Workspace + sparse state of one call.  The sparse path's per-row lists and its
// overflow flag live in caller-owned buffers (saved from forward to backward).
static int setup(const bgcn_bigcn_args* a, void* ws, size_t ws_bytes, FusedWs& w, SparseState& sp,
                 const int32_t*& gate, const Prepared* prep, const WeightImages* img) {
  const int64_t N = a->num_nodes, B = a->num_graphs, F = a->in_feats;
  BGCN_CHECK_ARG(ws && ws_bytes >= bigcn_ws_size(N, B, F, H), "workspace too small");
  BGCN_CHECK_ARG(a->feat_mode == BGCN_FEAT_DENSE ||
                     (a->x_flags && a->x_nnz && a->x_cols && a->x_vals),
                 "sparse feature buffers required unless feat_mode == BGCN_FEAT_DENSE");
  Carve c(ws, ws_bytes);
  carve_fused(c, N, B, F, &w);
  sp.mode = (a->feat_mode == BGCN_FEAT_DENSE || F > kSparseMaxF || N > kSparseMaxN) ? 1 : 0;
  sp.flags = a->x_flags;
  sp.nnz = a->x_nnz;
  sp.cols = a->x_cols;
  sp.vals = a->x_vals;
  carve_sparse(c, N, B, F, &sp);
  BGCN_CHECK_ARG(c.ok(), "workspace too small");
  if (img) {
    sp.w1t = img->w1t; sp.w2t = img->w2t; sp.w2s = img->w2s; sp.w2d = img->w2d;
  }
  if (sp.mode != 1) sp.rtick = w.rtick;   // item readout (tree items exist on the sparse path)
  w.spmm_bytes = ws_bytes - align_up(c.off, 256) - 256;
  w.spmm_ws = c.take<float>(1);
  for (int d = 0; d < 2; ++d)
    for (int o = 0; o < 2; ++o) {
      // the prepared batch's plans, else the ones the caller's graph views carry
      // (bgcn_graph_pair_plans), else none
      const bgcn_spmm_plan& vp = (d == 0 ? a->td : a->bu).plan[o];
      w.plan[d][o] = prep ? prep->plan[d][o]
                          : SpmmPlan{static_cast<const int2*>(vp.bnd), vp.longs, vp.nlong};
    }
  w.tree_status[0] = prep ? prep->status : a->td.tree_status;
  w.tree_status[1] = prep ? prep->status : a->bu.tree_status;
  if (prep) {   // the batch's weight-independent state lives in the prepared buffer
    w.node_root = prep->node_root;
    sp.item_tree = prep->item_tree; sp.tree_item0 = prep->tree_item0;
    sp.item_beg = prep->item_beg; sp.item_end = prep->item_end; sp.item_root = prep->item_root;
    sp.hist = prep->hist; sp.col_total = prep->col_total;
    sp.col_start = prep->col_start; sp.col_end = prep->col_end;
    sp.csc = prep->csc;
    sp.ovf_off = prep->x_ovf_off; sp.ovf = prep->x_ovf; sp.ovf_cap = prep->ovf_cap;
    sp.long_rows = prep->x_long;
  }
  // dense kernels run when feat_mode == dense (no gate) or when the sparse path overflowed
  // (auto); under BGCN_FEAT_SPARSE they are not launched (dense_launched)
  gate = sp.mode == 1 ? nullptr : a->x_flags;
  return BGCN_OK;
}

// the dense path's conv2 and dW2 root columns on the bf16 MFMA: bf16 X exact (BGCN_GEMM_BF16=0,
// read once, keeps the f32 MFMA forms), fp32 X split three ways, six products
// (BGCN_GEMM_X6=0, read once, keeps the f32 MFMA forms); 16-byte X rows and W2 rows
static bool bf16_mfma_ok(const bgcn_bigcn_args* a) {
  static const bool b16 = [] { const char* e = std::getenv("BGCN_GEMM_BF16"); return !(e && atoi(e) == 0); }();
  static const bool x6 = [] { const char* e = std::getenv("BGCN_GEMM_X6"); return !(e && atoi(e) == 0); }();
  return (a->x_dtype == BGCN_DTYPE_BF16 ? b16 : x6) && a->in_feats % 8 == 0 && a->ldx % 8 == 0 && (reinterpret_cast<uintptr_t>(a->x) & 15) == 0 &&
         (reinterpret_cast<uintptr_t>(a->td_w2) & 15) == 0 && (reinterpret_cast<uintptr_t>(a->bu_w2) & 15) == 0;
}

// whether the (gated) dense kernels are launched at all
static bool dense_launched(const bgcn_bigcn_args* a, const SparseState& sp) {
  return sp.mode == 1 || a->feat_mode != BGCN_FEAT_SPARSE;
}

// Forward.  Main stream: node maps, conv1 (sparse compaction + gather, or dense MFMA),
// propagate, conv2, propagate, readout.  When a backward follows, the CSC of X for dW1
// is built on the auxiliary lane right after conv1's lin, overlapped with the
// latency-bound second half of the forward, and joined before returning.  graph_lane
// >= 0: the caller is building the TD/BU graphs on that lane (bgcn_train_step), joined
// just before their first use.  head (bgcn_train_step): classifier head fused into the
// readout.
static int forward_tail(const bgcn_bigcn_args* a, FusedWs& w, SparseState& sp, KeepSrc keep,
                        const int32_t* gate, hipStream_t s, const HeadArgs* head, bool forked);

int bigcn_forward_impl(const bgcn_bigcn_args* a, void* ws, size_t ws_bytes, hipStream_t s,
                       int graph_lane, const HeadArgs* head, const Prepared* prep,
                       const WeightImages* img, bool img_current) {
  BGCN_TRY(check_args(a, prep != nullptr));
  BGCN_CHECK_ARG(a->head_in && a->td_w1 && a->bu_w1 && a->td_w2 && a->bu_w2, "null pointer");
  const int64_t N = a->num_nodes, F = a->in_feats;
  FusedWs w;
  SparseState sp{};
  const int32_t* gate = nullptr;
  BGCN_TRY(setup(a, ws, ws_bytes, w, sp, gate, prep, img));
  KeepSrc keep = make_keep(a);
  const bool sparse = sp.mode != 1;

  if (prep) {
    // prepared batch (bgcn_train_step): graphs, tree maps, items, ELL and CSC of X exist;
    // only the weight transposes and conv1's gather from the ELL remain (the prologue
    // also clears the step's status word, which the head ORs into)
    sp.zero_word = head ? head->status : nullptr;
    if (sparse && img && img_current)
      sp.conv1_clears = 1;   // nothing left for the prologue but its two clears
    else
      BGCN_TRY(sparse_prologue(sp, a, w.node_root, s, false));
    if (sparse) {
      timing_begin(0, s);
      BGCN_TRY(sparse_conv1_gather(sp, w.z1, s, a->rootindex, keep.scale()));
      timing_end(0, s);
    }
    if (dense_launched(a, sp))
      BGCN_TRY(gemm_xwt_x(a->x, a->x_dtype, a->ldx, a->td_w1, a->bu_w1, F, H, w.z1, 2 * H, N, 2 * H,
                          F, s, gate));
    if (graph_lane >= 0) BGCN_TRY(aux_join(s, graph_lane));   // K1 of a just-prepared batch
    return forward_tail(a, w, sp, keep, gate, s, head, false);
  }

  // one prologue launch: weight transposes, node -> root map, tree pointers, flag reset
  BGCN_TRY(sparse_prologue(sp, a, w.node_root, s));
  // tree work items (conv2 / dW2 root partials) on the side lane, beside the pass over X
  bool side_busy = graph_lane >= 0;
  if (sparse) {
    hipStream_t xi;
    BGCN_TRY(aux_fork(s, kLaneSide, &xi));
    BGCN_TRY(sparse_items(sp, a->tree_ptr, a->rootindex, xi));
    side_busy = side_busy || xi != s;
  }
  // conv1 lin, TD and BU in one pass over X: sparse (compaction + gather) or dense MFMA
  // (the conv1 of feat_mode dense; in auto mode a device-gated fallback)
  bool forked = false;
  if (sparse) {
    timing_begin(0, s);
    BGCN_TRY(sparse_compact_conv1(sp, a->x, a->x_dtype, a->ldx, w.z1, s));
    timing_end(0, s);
  }
  if (dense_launched(a, sp)) {
    timing_begin(sparse ? 4 : 0, s);
    BGCN_TRY(gemm_xwt_x(a->x, a->x_dtype, a->ldx, a->td_w1, a->bu_w1, F, H, w.z1, 2 * H, N, 2 * H, F,
                        s, gate));
    timing_end(sparse ? 4 : 0, s);
  }
  // the graphs (built on graph_lane by bgcn_train_step) and the items are needed from
  // here on; the join comes before the CSC fork so that it never waits for the CSC
  if (side_busy) BGCN_TRY(aux_join(s, kLaneSide));
  if (sparse && a->save_for_backward) {
    hipStream_t x;
    BGCN_TRY(aux_fork(s, kLaneSide, &x));
    sp.root_map = w.node_root;
    BGCN_TRY(sparse_csc(sp, x));
    forked = true;
  }
  return forward_tail(a, w, sp, keep, gate, s, head, forked);
}

// conv1 propagate -> conv2 -> conv2 propagate -> readout (+ head); joins the side lane
// when `forked`.
static int forward_tail(const bgcn_bigcn_args* a, FusedWs& w, SparseState& sp, KeepSrc keep,
                        const int32_t* gate, hipStream_t s, const HeadArgs* head, bool forked) {
  const int64_t N = a->num_nodes, B = a->num_graphs, F = a->in_feats;
  const bool sparse = sp.mode != 1;
  // conv1 propagate + bias (pre-relu h1 is saved: it is also the detached x2)
  BGCN_TRY(spmm_pair(a->td, a->bu, false, N, w.z1, a->h1, a->td_b1, a->bu_b1, BGCN_EPI_NONE, w, s));
  // conv2 lin with the root-extended, relu'd, dropped-out A operand generated in-kernel
  timing_begin(2, s);
  if (sparse) BGCN_TRY(sparse_conv2(sp, a->h1, a->tree_ptr, a->rootindex, w.z2, keep, s));
  if (dense_launched(a, sp)) {
    // bf16 X: the bf16 MFMA (BGCN_GEMM_BF16=0 keeps the f32 MFMA form)
    if (a->x_dtype == BGCN_DTYPE_BF16 && bf16_mfma_ok(a))
      hipLaunchKernelGGL(k_conv2_fwd_bf16<bf16_t>, dim3(grid_for(N, 128), 2), dim3(256), 0, s,
                         static_cast<const bf16_t*>(a->x), a->ldx, F, a->h1, w.node_root, a->td_w2,
                         a->bu_w2, w.z2, N, keep, gate);
    else if (a->x_dtype == BGCN_DTYPE_F32 && bf16_mfma_ok(a) && N >= kX6MinRows && N >= 32 * B) {
      // the trees' root planes once, then the conv2 that only masks them (trees of >= 32
      // nodes on average: PHEME's ~10-node trees share too little to pay the extra launch,
      // 34 -> 56 us at pheme768)
      const int64_t ldr = (F + kC2fBK - 1) / kC2fBK * kC2fBK;
      hipLaunchKernelGGL(k_root_split, dim3(grid_for(ldr, 256), unsigned(B)), dim3(256), 0, s,
                         static_cast<const float*>(a->x), a->ldx, F, a->rootindex, B, keep.scale(), w.rplanes,
                         ldr, gate);
      BGCN_CHECK_LAUNCH();
      hipLaunchKernelGGL((k_conv2_fwd_bf16<float, true>), dim3(grid_for(N, 128), 2), dim3(256), 0, s,
                         static_cast<const float*>(a->x), a->ldx, F, a->h1, w.node_root, a->td_w2,
                         a->bu_w2, w.z2, N, keep, gate, w.rplanes, ldr, a->batch);
    } else if (a->x_dtype == BGCN_DTYPE_F32 && bf16_mfma_ok(a) && N >= kX6MinRows)
      hipLaunchKernelGGL(k_conv2_fwd_bf16<float>, dim3(grid_for(N, 128), 2), dim3(256), 0, s,
                         static_cast<const float*>(a->x), a->ldx, F, a->h1, w.node_root, a->td_w2,
                         a->bu_w2, w.z2, N, keep, gate);
    else if (a->x_dtype == BGCN_DTYPE_BF16)
      hipLaunchKernelGGL(k_conv2_fwd<bf16_t>, dim3(grid_for(N, 64), 2), dim3(256), 0, s,
                         static_cast<const bf16_t*>(a->x), a->ldx, F, a->h1, w.node_root, a->td_w2,
                         a->bu_w2, w.z2, N, keep, gate);
    else
      hipLaunchKernelGGL(k_conv2_fwd<float>, dim3(grid_for(N, 64), 2), dim3(256), 0, s,
                         static_cast<const float*>(a->x), a->ldx, F, a->h1, w.node_root, a->td_w2,
                         a->bu_w2, w.z2, N, keep, gate);
    BGCN_CHECK_LAUNCH();
  }
  timing_end(2, s);
  BGCN_TRY(spmm_pair(a->td, a->bu, false, N, w.z2, a->h2, a->td_b2, a->bu_b2, BGCN_EPI_NONE, w, s));
  const HeadArgs no_head{};
  if (sparse) {
    const HeadArgs hd = head ? *head : no_head;
    uint64_t* sgn = readout_sign(a, sp, w) ? reinterpret_cast<uint64_t*>(w.d2) : nullptr;
    const dim3 g(unsigned(sp.max_items + B));
    if (hd.C <= 4 && sgn)
      hipLaunchKernelGGL((k_readout_items<4, true>), g, dim3(512), 0, s, sp, a->h1, a->h2, a->tree_ptr,
                         a->rootindex, N, B, a->head_in, w.rpart, hd, w.colpart2, sgn);
    else if (hd.C <= 4)
      hipLaunchKernelGGL((k_readout_items<4, false>), g, dim3(512), 0, s, sp, a->h1, a->h2, a->tree_ptr,
                         a->rootindex, N, B, a->head_in, w.rpart, hd, w.colpart2, sgn);
    else if (sgn)
      hipLaunchKernelGGL((k_readout_items<kMaxClasses, true>), g, dim3(512), 0, s, sp, a->h1, a->h2,
                         a->tree_ptr, a->rootindex, N, B, a->head_in, w.rpart, hd, w.colpart2, sgn);
    else
      hipLaunchKernelGGL((k_readout_items<kMaxClasses, false>), g, dim3(512), 0, s, sp, a->h1, a->h2,
                         a->tree_ptr, a->rootindex, N, B, a->head_in, w.rpart, hd, w.colpart2, sgn);
  }
  else
    hipLaunchKernelGGL(k_readout_fwd, dim3(unsigned(B)), dim3(1024), 0, s, a->h1, a->h2,
                       a->tree_ptr, a->rootindex, N, B, a->head_in, head ? *head : no_head);
  BGCN_CHECK_LAUNCH();
  if (forked) BGCN_TRY(aux_join(s, kLaneSide));
  return BGCN_OK;
}

// Backward, given the forward's workspace.  Main stream: readout' -> dZ2 -> dH1 -> dZ1
// -> dW1.  Side lane, forked as soon as its inputs exist: db2, the dW2 chain (relu(H1)
// block, root partials, root columns), db1 and the gated dense dW1; joined at the end.
int bigcn_backward_impl(const bgcn_bigcn_args* a, void* ws, size_t ws_bytes, hipStream_t s,
                        const Prepared* prep, bool side_busy, const HeadGradJob* head,
                        const WeightImages* img, bool defer_dw1, const TailAdam* adam, bool* adam_done) {
  if (adam_done) *adam_done = false;
  BGCN_TRY(check_args(a, prep != nullptr));
  BGCN_CHECK_ARG(a->dhead_in && a->td_dw1 && a->bu_dw1 && a->td_dw2 && a->bu_dw2 && a->td_db1 &&
                     a->bu_db1 && a->td_db2 && a->bu_db2,
                 "null gradient pointer");
  const int64_t N = a->num_nodes, B = a->num_graphs, F = a->in_feats;
  FusedWs w;
  SparseState sp{};
  const int32_t* gate = nullptr;
  BGCN_TRY(setup(a, ws, ws_bytes, w, sp, gate, prep, img));
  KeepSrc keep = make_keep(a);
  const bool sparse = sp.mode != 1;
  const bool have_csc = a->save_for_backward || prep != nullptr;
  hipStream_t x;

  // readout + relu' -> dH2: folded into the next aggregation on the sparse path (the
  // forward's readout left the H2 sign words and per-item counts, readout_sign; the head's
  // weight gradients then run in extra blocks of the middle launch), else k_readout_bwd
  // (+ the head's weight gradients in its extra blocks); db2 in the middle launch
  const int64_t nblk_r = (N + kReadBwdRows - 1) / kReadBwdRows;
  const HeadGradJob no_head{};
  const int nhead = head ? head->C + 1 : 0;
  const bool sign = readout_sign(a, sp, w);
  if (!sign) {
    hipLaunchKernelGGL(k_readout_bwd, dim3(unsigned(nblk_r + nhead)), dim3(256), 0, s, a->dhead_in, a->h2,
                       a->batch, a->tree_ptr, N, B, w.d2, w.colpart2, int(nblk_r), head ? *head : no_head);
    BGCN_CHECK_LAUNCH();
  }
  // dZ2 = A^T dH2 (sign: dH2 generated from the readout's H2 sign words)
  const SpmmSign sg{reinterpret_cast<const uint64_t*>(w.d2), a->dhead_in, a->batch, a->tree_ptr, B,
                    {w.tree_status[0], w.tree_status[1]}};
  BGCN_TRY(spmm_pair(a->td, a->bu, true, N, sign ? nullptr : w.d2, w.dz2, nullptr, nullptr, BGCN_EPI_NONE, w, s,
                     sign ? &sg : nullptr));
  // the CSC of X, when the forward did not leave one, is built on the side lane
  bool forked = false;
  if (sparse && !have_csc) {
    BGCN_TRY(aux_fork(s, kLaneSide, &x));
    sp.root_map = w.node_root;
    BGCN_TRY(sparse_csc(sp, x));
    forked = true;
  }

  // ---- middle launch: dW2 partials (the dense config, gated, and the sparse path's
  // relu(H1) block), the dW2 root-column partials, dH1 through dropout and relu (+ db1
  // partials) and the db2 column sums.  One dependent launch instead of four.
  const int64_t nblk_h = w.Sh;   // dH1 (+ relu(H1) dW2 partial) blocks: one per node split
  const int gxd = int(grid_for(H + F, 64));
  BwdMidArgs m{};
  m.S = sp;
  m.X = a->x; m.ldx = a->ldx; m.H1 = a->h1; m.dZ2 = w.dz2;
  m.node_root = w.node_root; m.tree_ptr = a->tree_ptr; m.gate = gate; m.keep = keep;
  // the dense feature mode takes its own (larger) node-split count; auto mode's gated
  // fallback keeps the small one (its blocks are launched every step and mostly exit)
  const int S2 = sp.mode == 1 ? w.S2d : w.S2;
  const int64_t kchunk2 = sp.mode == 1 ? w.kchunk2d : w.kchunk2;
  m.dw2_dense = Dw2Cfg{kchunk2, S2, gxd, 1, H + F, w.dw2_part};
  m.dw2_sparse = Dw2Cfg{w.kchunkh, w.Sh, 1, 0, int64_t(H), w.dw2_part};
  m.n_dw2_dense = dense_launched(a, sp) ? gxd * S2 * 2 : 0;
  // (fp32 X: the six-product form of k_dw2_bf16 measured 394 + 126 us against the f32
  // MFMA launch's 469 at the bench workload; k_dw2_root<float> takes the root factor out of
  // the MFMA operand instead, three products as for bf16 X.  BGCN_DW2_ROOT (read per call,
  // A/B runs and tests): 0 = k_dw2_f32 / k_dw2_bf16, 2 = the root form for any tree size)
  const char* root_env = std::getenv("BGCN_DW2_ROOT");
  const int root_mode = root_env ? atoi(root_env) : 1;
  const bool root_f32 = root_mode != 0;
  // (the tree-run tiles need trees of >= 32 nodes on average, as conv2's root planes do:
  // PHEME's ~10-node trees left 64-node tiles mostly empty, 15.6 -> 43.2 us)
  const bool big_trees = root_mode == 2 || N >= 32 * B;
  const bool dw2b = m.n_dw2_dense && sp.mode == 1 && bf16_mfma_ok(a) &&
                    (a->x_dtype == BGCN_DTYPE_BF16 || (a->x_dtype == BGCN_DTYPE_F32 && root_f32 && big_trees));
  if (dw2b) {
    // dense mode: the root columns on the bf16 MFMA (k_dw2_bf16 / k_dw2_root, a launch
    // of its own), dw2_body keeps column tile 0 (the H1 columns)
    // bf16 X takes the same form (weibo_bf16 dense 44.0k -> 48.1k trees/s against k_dw2_bf16,
    // whose operand carries keep x X; BGCN_DW2_ROOT=0: k_dw2_bf16)
    const bool root_bf16 = root_f32;
    m.dw2b_f32 = a->x_dtype == BGCN_DTYPE_F32 ? 1 : (root_bf16 && big_trees ? 2 : 0);
    m.gxb = int(grid_for(F, 128));
    m.n_dw2b = m.gxb * S2 * 2;
    m.dw2_dense.gx = 1;
    m.n_dw2_dense = S2 * 2;
  }
  // dense mode, fp32 X: the dW2 blocks as their own launch (k_dw2_f32: their register
  // budget, not the middle launch's); the middle launch then runs dH1, db2 and the head
  const bool dw2_own = m.n_dw2_dense && sp.mode == 1 && a->x_dtype == BGCN_DTYPE_F32 && !dw2b;
  if (dw2_own) {
    m.n_dw2f = m.n_dw2_dense;
  }
  m.n_dw2 = dw2_own ? 0 : m.n_dw2_dense;   // the sparse relu(H1) block is formed by the dH1 blocks
  // the H1 columns in the root columns' launch (its first blocks), not the middle launch's
  // (there their k-tiles in sequence made it 17 -> 124 us at twitter15 fp32).  BGCN_DW2_H_MID=1: the middle launch
  const char* h_env = std::getenv("BGCN_DW2_H_MID");
  const bool h_mid = h_env && atoi(h_env) == 1;
  if (dw2b && !h_mid) {
    m.n_dw2h = m.n_dw2_dense;
    m.n_dw2 = 0;
  }
  m.W2td = a->td_w2; m.W2bu = a->bu_w2; m.dH1 = w.dh1; m.colpart = w.colpart; m.nblk_h = int(nblk_h);
  m.rows_h = w.kchunkh;
  m.db2 = ColsumJob{w.colpart2, sign ? sp.max_items : int(nblk_r), a->td_db2, a->bu_db2};
  if (sign) {   // the partials are per-item positive counts, scaled by their tree's dhead
    m.db2_dhead = a->dhead_in;
  }
  if (sign && head) {   // the head's weight gradients (k_readout_bwd's extra blocks otherwise)
    m.hg = *head;
    m.n_hg = nhead;
  }
  timing_begin(3, s);
  BGCN_TRY(dw2_f32_launch(m, s));
  if (dw2_own) timing_end(3, s);   // class 3 = the dW2 GEMM alone in this form
  BGCN_TRY(dw2_bf16_launch(m, s));
  BGCN_TRY(bwd_mid_launch(m, a->x_dtype, s));
  if (!dw2_own) timing_end(3, s);

  // dZ1 = A^T dH1
  BGCN_TRY(spmm_pair(a->td, a->bu, true, N, w.dh1, w.dz1, nullptr, nullptr, BGCN_EPI_NONE, w, s));
  // dW1 by the dense MFMA GEMM: dense mode on main; the gated fallback of auto mode on
  // the side lane
  if (dense_launched(a, sp)) {
    if (sparse) {
      BGCN_TRY(aux_fork(s, kLaneSide, &x));
      forked = true;
    }
    BGCN_TRY(gemm_tn_x(w.dz1, 2 * H, a->x, a->x_dtype, a->ldx, a->td_dw1, a->bu_dw1, F, H, 2 * H, F,
                       N, w.tn_ws, w.tn_bytes, sparse ? x : s, sparse ? 6 : 1, gate));
  }
  if (sparse && !have_csc) {   // CSC built on the side (the join covers every branch so far)
    BGCN_TRY(aux_join(s, kLaneSide));
    forked = false;
  }

  // ---- tail launch: dW1 over the CSC of X (sparse), the dW2 root columns, the dW2
  // partial reductions and the db1 column sums
  BwdTailArgs t{};
  t.S = sp;
  t.dZ1 = w.dz1; t.dw1_td = a->td_dw1; t.dw1_bu = a->bu_dw1;
  t.node_root = w.node_root; t.batch = a->batch; t.dw2_td = a->td_dw2; t.dw2_bu = a->bu_dw2;
  t.keep_scale = keep.scale(); t.dw2_part = w.dw2_part; t.gate = gate;
  t.keep = keep; t.dZ2 = w.dz2;
  // 1024-thread blocks, 4 output tiles of 64 each
  t.red_dense = RedCfg{S2, H + F, 1,
                       dense_launched(a, sp) ? int(std::min<unsigned>(grid_for(2 * H * (H + F), 256), 256)) : 0};
  t.red_sparse = RedCfg{w.Sh, int64_t(H), 0, sparse ? int(grid_for(2 * H * H, 256)) : 0};
  t.db1 = ColsumJob{w.colpart, int(nblk_h), a->td_db1, a->bu_db1};
  timing_begin(5, s);
  // deferred dW1 (bgcn_train_step with defer_dw1): every gradient but dW1 is final when
  // this launch ends; bigcn_backward_dw1 runs the dW1 waves later
  // the step's optimiser step in the same launch (bgcn_step_args.adam): on the sparse path
  // with no dense kernel launched (the gated dense dW1 would arrive after the tail's blocks)
  if (adam && adam->on && sparse && !dense_launched(a, sp) && !defer_dw1) t.adam = *adam;
  BGCN_TRY(bwd_tail_launch(t, s, defer_dw1 ? 1 : 0));
  // (the launcher clears adam.on for a tail form that cannot carry it: BGCN_DW1_SPLIT != 0)
  if (adam_done) *adam_done = t.adam.on != 0;
  timing_end(5, s);
  (void)side_busy;
  timing_end(9, s);   // the main stream's own chain (span class, bgcn_train_step)
  // join only what this backward forked (a next-batch preparation on the side lane is
  // waited for by the next bgcn_train_step call instead)
  if (forked) BGCN_TRY(aux_join(s, kLaneSide));
  return BGCN_OK;
}

// The deferred dW1 of a backward that ran with defer_dw1 (same args, workspace, prepared
// batch): the tail's dW1 waves alone (the sparse path; the dense fallback's dW1 GEMM ran
// inside the backward).
int bigcn_backward_dw1(const bgcn_bigcn_args* a, void* ws, size_t ws_bytes, hipStream_t s, const Prepared* prep,
                       const WeightImages* img) {
  BGCN_TRY(check_args(a, prep != nullptr));
  BGCN_CHECK_ARG(a->td_dw1 && a->bu_dw1, "null gradient pointer");
  FusedWs w;
  SparseState sp{};
  const int32_t* gate = nullptr;
  BGCN_TRY(setup(a, ws, ws_bytes, w, sp, gate, prep, img));
  if (sp.mode == 1) return BGCN_OK;
  BwdTailArgs t{};
  t.S = sp;
  t.dZ1 = w.dz1; t.dw1_td = a->td_dw1; t.dw1_bu = a->bu_dw1;
  t.node_root = w.node_root; t.batch = a->batch; t.dw2_td = a->td_dw2; t.dw2_bu = a->bu_dw2;
  t.keep_scale = make_keep(a).scale(); t.gate = gate;
  timing_begin(11, s);
  BGCN_TRY(bwd_tail_launch(t, s, 2));
  timing_end(11, s);
  return BGCN_OK;
}

int keep_words_impl(uint64_t seed, int64_t N, int32_t nw, uint32_t* words, hipStream_t s) {
  BGCN_CHECK_ARG(N > 0 && nw > 0 && nw <= 256 && words, "bad arguments");
  hipLaunchKernelGGL(k_keep_words, dim3(grid_for(2 * N * nw, 256)), dim3(256), 0, s, seed, N, nw,
                     words);
  BGCN_CHECK_LAUNCH();
  return BGCN_OK;
}

}  // namespace bgcn

extern "C" size_t bgcn_bigcn_workspace_size(int64_t num_nodes, int64_t num_graphs,
                                            int64_t in_feats, int64_t hid) {
  return bgcn::bigcn_ws_size(num_nodes, num_graphs, in_feats, hid);
}
extern "C" int bgcn_bigcn_forward(const bgcn_bigcn_args* args, void* workspace,
                                  size_t workspace_bytes, bgcn_stream_t stream) {
  if (args && args->prepared)
    return bgcn::bigcn_prepared_call(args, workspace, workspace_bytes, reinterpret_cast<hipStream_t>(stream),
                                     false);
  return bgcn::bigcn_forward_impl(args, workspace, workspace_bytes,
                                  reinterpret_cast<hipStream_t>(stream), -1, nullptr, nullptr);
}
extern "C" int bgcn_bigcn_backward(const bgcn_bigcn_args* args, void* workspace,
                                   size_t workspace_bytes, bgcn_stream_t stream) {
  if (args && args->prepared)
    return bgcn::bigcn_prepared_call(args, workspace, workspace_bytes, reinterpret_cast<hipStream_t>(stream),
                                     true);
  return bgcn::bigcn_backward_impl(args, workspace, workspace_bytes,
                                   reinterpret_cast<hipStream_t>(stream), nullptr, false);
}
extern "C" int bgcn_keep_words(uint64_t seed, int64_t num_nodes, int32_t num_words,
                               uint32_t* words, bgcn_stream_t stream) {
  return bgcn::keep_words_impl(seed, num_nodes, num_words, words,
                               reinterpret_cast<hipStream_t>(stream));
}

BT_READER(bigcn)
