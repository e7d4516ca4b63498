// Device bodies of the backward's middle and tail launches (bgcn_sparse.hip defines the
// merged kernels): the dW2 relu(H1)-block / dense partials, their fixed-order reduction
// and dH1.  Each body takes its block id within its role and a slice of the launch's
// shared memory, so several roles share one launch (one dependent launch instead of
// four on the caller's stream).
#pragma once

#include "bgcn_internal.h"
#include "bgcn_sparse.h"

namespace bgcn {

constexpr int BK = 32;
constexpr int H = 64;  // hid = out = 64 (BiGCN_Twitter.py:144; the fused path is specialised)

__device__ __forceinline__ int acc_row(int r, int lane) { return (r & 3) + 8 * (r >> 2) + 4 * (lane >> 5); }

// ---------------------------------------------------------------- dW2
// part[d][s][o][c] = sum_{i in split s} dZ2[i][d*H+o] * A2_d[i][c]   (A2_d generated)
// Block tile 64 (o) x 64 (c), waves 2 x 2; grid (ceil((H+F)/64), S, 2).
// One launch configuration of k_dw2: a grid of gx column tiles x S node splits x 2
// directions over partial rows of ldp columns.

// Two configurations share one launch (blocks [0, nblk0) run cfg0, the rest cfg1): the
// dense path's full grid (all 64+F columns, few node splits; want_dense = 1) and the
// sparse path's relu(H1) block only (column tile 0, many node splits, ldp = 64;
// want_dense = 0).  Only the configuration of the path selected on the device works.
// Device body, 256 threads, block id `bid` of the role; smem: kDw2Smem floats.
constexpr int kDw2Smem = 4 * BK * H;
template <class TX>
__device__ inline void dw2_body(const TX* __restrict__ X, int64_t ldx, int64_t F,
                                const float* __restrict__ H1, const float* __restrict__ dZ2,
                                const int32_t* __restrict__ node_root, int64_t N, KeepSrc keep,
                                const int32_t* __restrict__ gate, const Dw2Cfg& cfg0,
                                const Dw2Cfg& cfg1, int nblk0, int bid, float* smem) {
  const bool second = bid >= nblk0;
  const Dw2Cfg& cfg = second ? cfg1 : cfg0;
  const int bl = second ? bid - nblk0 : bid;
  if (dense_active(gate) != (cfg.want_dense != 0)) return;
  const int64_t kchunk = cfg.kchunk, ldp = cfg.ldp;
  const int S = cfg.S;
  float* __restrict__ part = cfg.part;
  constexpr int BN = 64;
  float (*As)[BK * H] = reinterpret_cast<float (*)[BK * H]>(smem);              // [node][o]
  float (*Bs)[BK * BN] = reinterpret_cast<float (*)[BK * BN]>(smem + 2 * BK * H);  // [node][c]
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int wr = wave >> 1, wc = wave & 1;
  const int bx = bl % cfg.gx, split = (bl / cfg.gx) % S, d = bl / (cfg.gx * S);
  const int64_t K2 = H + F;
  const int64_t c0 = int64_t(bx) * BN;
  const int64_t kb = int64_t(split) * kchunk, ke = min<int64_t>(kb + kchunk, N);
  const float sc = keep.scale();

  // A staging: dZ2 tile 32 nodes x 64 -> node = tid/16 + 16 i, o quad (tid%16)*4
  const int an = tid >> 4, aq = (tid & 15) * 4;
  // B generation: node = tid/8, 8 columns at (tid%8)*8
  const int bn = tid >> 3, bc = (tid & 7) * 8;
  float4 ra[2], gb[2];
  uint32_t gw = 0;
  // unconditional loads from clamped nodes / columns, zeroed by select (see k_dh1)
  auto gload = [&](int64_t k0) {
#pragma unroll
    for (int i = 0; i < 2; ++i) {
      const int64_t node = k0 + an + 16 * i;
      const float4 v = ld4(dZ2 + min<int64_t>(node, ke - 1) * (2 * H) + d * H + aq);
      ra[i] = node < ke ? v : f4zero();
    }
    const int64_t node = k0 + bn;
    const bool ok = node < ke;
    const int64_t nc = min<int64_t>(node, ke - 1);
    const int64_t c = c0 + bc;
    gw = keep.get(uint32_t(d), uint32_t(nc), uint32_t(min<int64_t>(c / 32, keep.nw - 1)));   // (clamped: the last tile runs past K2)
    gw = ok ? gw : 0u;
    const int32_t root = node_root[nc];
    const TX* xr = X + int64_t(root < 0 ? 0 : root) * ldx;
    const float* h1 = H1 + nc * (2 * H) + d * H;
#pragma unroll
    for (int j = 0; j < 2; ++j) {
      const int64_t cc = min<int64_t>(c + 4 * j, K2 - 4);
      float4 v;
      if constexpr (sizeof(TX) == sizeof(float)) v = ld4(cc < H ? h1 + cc : xr + (cc - H));
      else v = cc < H ? ld4(h1 + cc) : xq(xr + (cc - H));
      gb[j] = (ok && c + 4 * j < K2) ? v : f4zero();
    }
  };
  auto sstore = [&](int buf) {
#pragma unroll
    for (int i = 0; i < 2; ++i) st4(&As[buf][(an + 16 * i) * H + aq], ra[i]);
    const int bit0 = int((c0 + bc) & 31);
#pragma unroll
    for (int j = 0; j < 2; ++j) {
      float v[4] = {gb[j].x, gb[j].y, gb[j].z, gb[j].w};
      float o[4];
#pragma unroll
      for (int e = 0; e < 4; ++e)
        o[e] = ((gw >> (bit0 + 4 * j + e)) & 1u) ? sc * fmaxf(v[e], 0.f) : 0.f;
      st4(&Bs[buf][bn * BN + bc + 4 * j], make_float4(o[0], o[1], o[2], o[3]));
    }
  };

  // Blocked accumulation: each 32-node k-tile sums into a fresh accumulator (16 MFMA
  // steps), which is then added to the running sum - one fp32 accumulator took ~1000
  // sequential MFMA adds per 2048-node split, and where the node terms cancel (a small
  // entry of a large sum) that left TD conv2's weight gradient 2.3e-5 off the fp64 oracle
  // elementwise (4.4x under the 1e-4 bar); the tile sums cut the
  // sequential depth to 16 + kchunk / 32.
  f32x16 acc = {0};
  const int h = lane >> 5, r32 = lane & 31;
  const int nk = int((ke - kb + BK - 1) / BK);
  if (nk > 0) {
    gload(kb);
    sstore(0);
  }
  __syncthreads();
  for (int kt = 0; kt < nk; ++kt) {
    const int buf = kt & 1;
    if (kt + 1 < nk) gload(kb + int64_t(kt + 1) * BK);
    const float* A = &As[buf][h * H + wr * 32 + r32];
    const float* B = &Bs[buf][h * BN + wc * 32 + r32];
#ifdef BGCN_DW2_ONE_ACC   // A/B build: the single running accumulator of round 5
#pragma unroll
    for (int s = 0; s < BK / 2; ++s) acc = mfma32x32x2(A[2 * s * H], B[2 * s * BN], acc);
#else
    f32x16 tile = {0};
#pragma unroll
    for (int s = 0; s < BK / 2; ++s) tile = mfma32x32x2(A[2 * s * H], B[2 * s * BN], tile);
#pragma unroll
    for (int r = 0; r < 16; ++r) acc[r] += tile[r];
#endif
    if (kt + 1 < nk) sstore(buf ^ 1);
    __syncthreads();
  }
  float* out = part + (int64_t(d) * S + split) * (H * ldp);
#pragma unroll
  for (int r = 0; r < 16; ++r) {
    int64_t c = c0 + wc * 32 + r32;
    int o = wr * 32 + acc_row(r, lane);
    if (c < ldp) out[int64_t(o) * ldp + c] = acc[r];
  }
}

// The dense config's root columns (c >= 64) for bf16 X on the bf16 MFMA:
//   part[d][s][o][64 + x] = sum_{i in split s} dZ2_d[i][o] * keep(d, i, 64 + x) * s * relu(X[root(i)][x])
// (the H1 columns c < 64 stay with dw2_body's column tile 0).  The A2 values are exact in
// bf16 (bag-of-words counts, s = 1 or 2) and dZ2 is split three ways: three products,
// fp32-grade.  Block tile 64 (o) x 128 (x) over 64-node k-tiles, 4 waves as 2 x 2 (wave
// tile 32 x 64).  Both operands are node-major in memory and staged transposed into
// node-contiguous LDS rows, each lane writing its row's contiguous nodes as 16-byte stores
// on consecutive rows (conflict-free); the tile's 64 x 4 keep words are hashed once (one per
// thread) and shared through LDS.  Block id: (column tile bx, split, direction) with gxb
// column tiles of 128.  smem: kDw2bSmem floats.
constexpr int kDw2bBK = 64, kDw2bLd = kDw2bBK + 8;
constexpr int kDw2bSmem = (3 * H * kDw2bLd + 128 * kDw2bLd) / 2 + kDw2bBK * 4;
__device__ inline void dw2_bf16_body(const bf16_t* __restrict__ X, int64_t ldx, int64_t F,
                                     const float* __restrict__ dZ2, const int32_t* __restrict__ node_root,
                                     int64_t N, KeepSrc keep, const int32_t* __restrict__ gate,
                                     const Dw2Cfg& cfg, int gxb, int bid, float* smem) {
  if (!dense_active(gate)) return;
  __bf16* As = reinterpret_cast<__bf16*>(smem);                 // [3][64 o][kDw2bLd]
  __bf16* Bs = As + 3 * H * kDw2bLd;                            // [128 x][kDw2bLd]
  uint32_t* kwl = reinterpret_cast<uint32_t*>(Bs + 128 * kDw2bLd);   // [64 nodes][4 words]
  const int S = cfg.S;
  const int bx = bid % gxb, split = (bid / gxb) % S, d = bid / (gxb * S);
  const int64_t n0 = int64_t(bx) * 128;                         // first X column of the tile
  const int64_t kb = int64_t(split) * cfg.kchunk, ke = min<int64_t>(kb + cfg.kchunk, N);
  const float sc = keep.scale();
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int wr = wave >> 1, wc = wave & 1, h = lane >> 5, r32 = lane & 31;
  constexpr int kGN = kDw2bBK / 4, kBN = kDw2bBK / 2;           // nodes per thread: dZ2 / A2
  const int go = tid & 63, gn = (tid >> 6) * kGN;               // dZ2: column o, kGN nodes
  const int bc = tid & 127, bn = (tid >> 7) * kBN;              // A2: column x, kBN nodes
  const bool cok = n0 + bc < F;
  const uint32_t w0 = uint32_t((H + n0) >> 5);                  // the tile's first keep word
  float rg[kGN];
  uint32_t rx[kBN / 2];   // two bf16 per word
  uint32_t rk = 0;
  auto gload = [&](int64_t k0) {
#pragma unroll
    for (int u = 0; u < kGN; ++u) {
      const int64_t k = k0 + gn + u;
      const float v = dZ2[min<int64_t>(k, ke - 1) * (2 * H) + d * H + go];
      rg[u] = k < ke ? v : 0.f;
    }
    // the nodes' root rows: a 32-node run inside one tree (the common case: trees are
    // contiguous and hundreds of nodes long) shares one root, so one X element per thread
    const int64_t kf = min<int64_t>(k0 + bn, ke - 1), kl = min<int64_t>(k0 + bn + kBN - 1, ke - 1);
    const int32_t rf = node_root[kf], rl = node_root[kl];
    if (rf == rl) {   // wave-uniform (the wave's threads share bn)
      const uint16_t v = X[int64_t(rf < 0 ? 0 : rf) * ldx + (cok ? n0 + bc : 0)];
      const uint32_t vv = cok ? uint32_t(v) : 0u;
#pragma unroll
      for (int u = 0; u < kBN; u += 2) {
        const bool ok0 = k0 + bn + u < ke, ok1 = k0 + bn + u + 1 < ke;
        rx[u >> 1] = (ok0 ? vv : 0u) | ((ok1 ? vv : 0u) << 16);
      }
    } else {
#pragma unroll
      for (int u = 0; u < kBN; u += 2) {
        uint32_t two = 0;
#pragma unroll
        for (int t = 0; t < 2; ++t) {
          const int64_t k = k0 + bn + u + t;
          const int32_t root = node_root[min<int64_t>(k, ke - 1)];
          const uint16_t v = X[int64_t(root < 0 ? 0 : root) * ldx + (cok ? n0 + bc : 0)];
          two |= uint32_t((k < ke && cok) ? v : uint16_t(0)) << (16 * t);
        }
        rx[u >> 1] = two;
      }
    }
    {
      const int64_t k = k0 + (tid >> 2);
      const uint32_t wd = keep.get(uint32_t(d), uint32_t(min<int64_t>(k, ke - 1)), min(w0 + uint32_t(tid & 3), uint32_t(keep.nw - 1)));
      rk = k < ke ? wd : 0u;
    }
  };
  auto sstore = [&]() {
    kwl[tid] = rk;
#pragma unroll
    for (int j = 0; j < kGN / 8; ++j) {
      bf16x8 hv, mv, lv;
#pragma unroll
      for (int u = 0; u < 8; ++u) {
        __bf16 x, y, z;
        split3_bf16(rg[8 * j + u], x, y, z);
        hv[u] = x; mv[u] = y; lv[u] = z;
      }
      const int oa = go * kDw2bLd + gn + 8 * j;
      *reinterpret_cast<bf16x8*>(&As[oa]) = hv;
      *reinterpret_cast<bf16x8*>(&As[H * kDw2bLd + oa]) = mv;
      *reinterpret_cast<bf16x8*>(&As[2 * H * kDw2bLd + oa]) = lv;
    }
    __syncthreads();   // kwl
    const int wsel = bc >> 5, bit = bc & 31;
#pragma unroll
    for (int j = 0; j < kBN / 8; ++j) {
      bf16x8 v;
#pragma unroll
      for (int e = 0; e < 8; ++e) {
        const int u = 8 * j + e;
        const bool kept = (kwl[(bn + u) * 4 + wsel] >> bit) & 1u;
        const float x = __uint_as_float((rx[u >> 1] >> (16 * (u & 1))) << 16);
        v[e] = __bf16(kept ? sc * fmaxf(x, 0.f) : 0.f);   // exact: s is 1 or 2
      }
      *reinterpret_cast<bf16x8*>(&Bs[bc * kDw2bLd + bn + 8 * j]) = v;
    }
  };
  f32x16 acc[2] = {};
  const int nk = int((ke - kb + kDw2bBK - 1) / kDw2bBK);
  if (nk > 0) {
    gload(kb);
    sstore();
  }
  __syncthreads();
  for (int kt = 0; kt < nk; ++kt) {
    if (kt + 1 < nk) gload(kb + int64_t(kt + 1) * kDw2bBK);
#pragma unroll
    for (int s = 0; s < kDw2bBK / 16; ++s) {
      const int ko = 16 * s + 8 * h;
      const int oa = (wr * 32 + r32) * kDw2bLd + ko;
      const bf16x8 a0 = *reinterpret_cast<const bf16x8*>(&As[oa]);
      const bf16x8 a1 = *reinterpret_cast<const bf16x8*>(&As[H * kDw2bLd + oa]);
      const bf16x8 a2 = *reinterpret_cast<const bf16x8*>(&As[2 * H * kDw2bLd + oa]);
#pragma unroll
      for (int ni = 0; ni < 2; ++ni) {
        const bf16x8 b = *reinterpret_cast<const bf16x8*>(&Bs[(wc * 64 + ni * 32 + r32) * kDw2bLd + ko]);
        f32x16 c = acc[ni];
        c = mfma_bf16(a2, b, c);
        c = mfma_bf16(a1, b, c);
        acc[ni] = mfma_bf16(a0, b, c);
      }
    }
    __syncthreads();
    if (kt + 1 < nk) {
      sstore();
      __syncthreads();
    }
  }
  float* out = cfg.part + (int64_t(d) * S + split) * (H * cfg.ldp) + H + n0;
#pragma unroll
  for (int q = 0; q < 16; ++q) {
    const int o = wr * 32 + acc_row(q, lane);
#pragma unroll
    for (int ni = 0; ni < 2; ++ni) {
      const int c = wc * 64 + ni * 32 + r32;
      if (n0 + c < F) out[int64_t(o) * cfg.ldp + c] = acc[ni][q];
    }
  }
}

// The dense config's root columns (fp32 and bf16 X; dw2_bf16_body above is the bf16
// form it replaced, kept behind BGCN_DW2_ROOT=0).  A node's root-column operand is
// keep(d, i, 64 + x) * s * relu(X[root(i)][x]); its second factor is the same for every node
// of one tree, so over k-tiles that are runs of one root's nodes (<= 64, trees are
// contiguous) the tile's product factors:
//   part[d][s][o][64 + x] = sum over tiles T of  s*relu(X[root_T][x]) * sum_{i in T} dZ2_d[i][o] keep(d, i, 64 + x)
// The inner sum runs on the bf16 MFMA with the keep bits as the exact 0/2 operand and dZ2
// split three ways (fp32-grade products, as dw2_bf16_body), into a fresh tile accumulator;
// the root factor is one fp32 FMA per output and tile (the lane's column is fixed, so one
// factor per lane and 32-column half).  Each tile's run is found by a ballot over its 64
// node_root entries (every wave computes the same run), so the next tile's start is known
// when its loads are issued.  Layout, block ids and smem as dw2_bf16_body.
#ifndef BGCN_DW2R_DEEP
#define BGCN_DW2R_DEEP 1   // tiles whose loads are in flight (2: +20 VGPRs, two waves per SIMD: 4 % slower)
#endif
__device__ __forceinline__ float x_elem(const float* p) { return *p; }
__device__ __forceinline__ float x_elem(const bf16_t* p) { return bf2f(*p); }
template <class TX>
__device__ inline void dw2_root_body(const TX* __restrict__ X, int64_t ldx, int64_t F,
                                     const float* __restrict__ dZ2, const int32_t* __restrict__ node_root,
                                     int64_t N, KeepSrc keep, const int32_t* __restrict__ gate,
                                     const Dw2Cfg& cfg, int gxb, int bid, float* smem) {
  if (!dense_active(gate)) return;
  __bf16* As = reinterpret_cast<__bf16*>(smem);                 // [3][64 o][kDw2bLd]
  __bf16* Bs = As + 3 * H * kDw2bLd;                            // [128 x][kDw2bLd]
  uint32_t* kwl = reinterpret_cast<uint32_t*>(Bs + 128 * kDw2bLd);   // [4 words][64 nodes]
  const int S = cfg.S;
  const int bx = bid % gxb, split = (bid / gxb) % S, d = bid / (gxb * S);
  const int64_t n0 = int64_t(bx) * 128;                         // first X column of the tile
  const int64_t kb = int64_t(split) * cfg.kchunk, ke = min<int64_t>(kb + cfg.kchunk, N);
  const float sc = keep.scale();
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int wr = wave >> 1, wc = wave & 1, h = lane >> 5, r32 = lane & 31;
  constexpr int kGN = kDw2bBK / 4, kBN = kDw2bBK / 2;           // nodes per thread: dZ2 / keep bits
  const int go = tid & 63, gn = (tid >> 6) * kGN;               // dZ2: column o, kGN nodes
  const int bc = tid & 127, bn = (tid >> 7) * kBN;              // keep bits: column x, kBN nodes
  const uint32_t w0 = uint32_t((H + n0) >> 5);                  // the tile's first keep word
  // this thread's keep word, clamped to the node's last (the last column tile's words past
  // F only feed output columns that are not stored; injected words must not be read past
  // the array's end)
  const uint32_t wk = min(w0 + uint32_t(tid & 3), uint32_t(keep.nw - 1));
  const uint32_t voff_g = uint32_t(gn * (2 * H) + go) * 4u;     // this thread's first dZ2 element in a tile
  const float hsc = 0.5f * sc;                                  // exact: sc is 1 or 2
  // one tile's loads in registers (BGCN_DW2R_DEEP 2 keeps two, issued two tiles before
  // their LDS staging; the default relies on three waves per SIMD instead)
  struct Stage {
    float rg[kGN];
    uint32_t rk;
    float vn[2];   // the tile's root factors for this lane's two output columns
    int run;       // the tile's nodes (>= 1)
  };
  auto gload = [&](Stage& st, int64_t t0) {
    const int32_t rl = node_root[min<int64_t>(t0 + lane, ke - 1)];
    const int32_t r0 = __builtin_amdgcn_readfirstlane(rl);
    const unsigned long long diff = __ballot(rl != r0 || t0 + lane >= ke);
    const int run = diff ? int(__builtin_ctzll(diff)) : kDw2bBK;
    st.run = run;
    // the run's dZ2 rows through a descriptor of run rows: rows past it read as zero
    const __amdgpu_buffer_rsrc_t rs = row_rsrc(dZ2 + t0 * (2 * H) + d * H, uint32_t(run) * (2 * H) * 4u);
#pragma unroll
    for (int u = 0; u < kGN; ++u)
      st.rg[u] = __uint_as_float(__builtin_amdgcn_raw_buffer_load_b32(rs, voff_g + uint32_t(u) * (2 * H) * 4u, 0, 0));
    {
      const int k = tid >> 2;
      const uint32_t wd = keep.get(uint32_t(d), uint32_t(min<int64_t>(t0 + k, ke - 1)), wk);
      st.rk = k < run ? wd : 0u;
    }
    const TX* xr = X + int64_t(r0) * ldx;
#pragma unroll
    for (int ni = 0; ni < 2; ++ni) {
      const int64_t c = n0 + wc * 64 + ni * 32 + r32;
      const float x = x_elem(xr + (c < F ? c : F - 1));
      st.vn[ni] = c < F ? hsc * fmaxf(x, 0.f) : 0.f;   // (the keep operand is 2 per kept bit)
    }
  };
  // dZ2 split exactly by truncation (x = hi + mid + lo, each a bf16: hi keeps x's top 8
  // significant bits, mid the next 8 of the remainder, lo the rest), two values per packed
  // word; the keep bits expanded to bf16 0 / 2 two nodes per word, from word-major kwl
  auto sstore = [&](const Stage& st) {
    kwl[(tid & 3) * kDw2bBK + (tid >> 2)] = st.rk;
#pragma unroll
    for (int j = 0; j < kGN / 8; ++j) {
      uint32_t hw[4], mw[4], lw[4];
#pragma unroll
      for (int p = 0; p < 4; ++p) {
        uint32_t xb[2], rb[2], lb[2];
#pragma unroll
        for (int e = 0; e < 2; ++e) {
          const float x = st.rg[8 * j + 2 * p + e];
          xb[e] = __float_as_uint(x);
          const float r = x - __uint_as_float(xb[e] & 0xffff0000u);
          rb[e] = __float_as_uint(r);
          lb[e] = __float_as_uint(r - __uint_as_float(rb[e] & 0xffff0000u));
        }
        hw[p] = __builtin_amdgcn_perm(xb[1], xb[0], 0x07060302u);   // upper halves: value 0 low
        mw[p] = __builtin_amdgcn_perm(rb[1], rb[0], 0x07060302u);
        lw[p] = __builtin_amdgcn_perm(lb[1], lb[0], 0x07060302u);
      }
      const int oa = go * kDw2bLd + gn + 8 * j;
      *reinterpret_cast<uint4*>(&As[oa]) = make_uint4(hw[0], hw[1], hw[2], hw[3]);
      *reinterpret_cast<uint4*>(&As[H * kDw2bLd + oa]) = make_uint4(mw[0], mw[1], mw[2], mw[3]);
      *reinterpret_cast<uint4*>(&As[2 * H * kDw2bLd + oa]) = make_uint4(lw[0], lw[1], lw[2], lw[3]);
    }
    __syncthreads();   // kwl
    const int wsel = bc >> 5, bit = bc & 31;
#pragma unroll
    for (int j = 0; j < kBN / 8; ++j) {
      const uint4 k0 = *reinterpret_cast<const uint4*>(&kwl[wsel * kDw2bBK + bn + 8 * j]);
      const uint4 k1 = *reinterpret_cast<const uint4*>(&kwl[wsel * kDw2bBK + bn + 8 * j + 4]);
      const uint32_t kw[8] = {k0.x, k0.y, k0.z, k0.w, k1.x, k1.y, k1.z, k1.w};
      uint32_t bw[4];   // bf16 2.0 = 0x4000: the bit moved to bit 14 of each half
#pragma unroll
      for (int p = 0; p < 4; ++p)
        bw[p] = ((__builtin_amdgcn_ubfe(kw[2 * p + 1], bit, 1) << 16) | __builtin_amdgcn_ubfe(kw[2 * p], bit, 1)) << 14;
      *reinterpret_cast<uint4*>(&Bs[bc * kDw2bLd + bn + 8 * j]) = make_uint4(bw[0], bw[1], bw[2], bw[3]);
    }
  };
  f32x16 acc[2] = {};
  int run = 0;
  float v0 = 0.f, v1 = 0.f;
  int64_t tn = ke;   // the start of the tile after the staged one
  // the staged tile times its root factors into acc: one 32-column half at a time (one
  // fresh tile accumulator live), the A operands re-read from LDS for the second half
  auto mul_tile = [&]() {
#pragma unroll
    for (int ni = 0; ni < 2; ++ni) {
      f32x16 tile = {};
      // (every k-step runs: the rows past the run are zero in A; skipping the empty steps
      // made the compiler predicate the MFMAs and select the accumulators)
#pragma unroll
      for (int s = 0; s < kDw2bBK / 16; ++s) {
        const int ko = 16 * s + 8 * h;
        const int oa = (wr * 32 + r32) * kDw2bLd + ko;
        const bf16x8 a0 = *reinterpret_cast<const bf16x8*>(&As[oa]);
        const bf16x8 a1 = *reinterpret_cast<const bf16x8*>(&As[H * kDw2bLd + oa]);
        const bf16x8 a2 = *reinterpret_cast<const bf16x8*>(&As[2 * H * kDw2bLd + oa]);
        const bf16x8 b = *reinterpret_cast<const bf16x8*>(&Bs[(wc * 64 + ni * 32 + r32) * kDw2bLd + ko]);
        tile = mfma_bf16(a2, b, tile);
        tile = mfma_bf16(a1, b, tile);
        tile = mfma_bf16(a0, b, tile);
      }
      const float vv = ni ? v1 : v0;
#pragma unroll
      for (int q = 0; q < 16; ++q) acc[ni][q] = fmaf(vv, tile[q], acc[ni][q]);
    }
  };
#if BGCN_DW2R_DEEP == 2
  // two tiles' loads in flight: the staged tile is multiplied while `nxt` holds the next
  // tile's loads (start tn) and the one after is loaded into `fre`
  auto step = [&](Stage& nxt, Stage& fre) -> bool {
    const int64_t tnn = tn < ke ? tn + nxt.run : ke;
    if (tnn < ke) gload(fre, tnn);
    mul_tile();
    __syncthreads();
    if (tn >= ke) return false;   // block-uniform
    sstore(nxt);
    __syncthreads();
    run = nxt.run;
    v0 = nxt.vn[0]; v1 = nxt.vn[1];
    tn = tnn;
    return true;
  };
  Stage sa, sb;
  if (kb < ke) {
    gload(sa, kb);
    sstore(sa);
    run = sa.run;
    v0 = sa.vn[0]; v1 = sa.vn[1];
    tn = kb + run;
    if (tn < ke) gload(sb, tn);
    __syncthreads();
    while (step(sb, sa) && step(sa, sb)) {
    }
  }
#else
  // one tile's loads in flight (the occupancy hides the rest)
  Stage st;
  if (kb < ke) {
    gload(st, kb);
    sstore(st);
    run = st.run;
    v0 = st.vn[0]; v1 = st.vn[1];
    tn = kb + run;
    __syncthreads();
    while (true) {   // block-uniform
      if (tn < ke) gload(st, tn);
      mul_tile();
      __syncthreads();
      if (tn >= ke) break;
      sstore(st);
      __syncthreads();
      run = st.run;
      v0 = st.vn[0]; v1 = st.vn[1];
      tn += run;
    }
  }
#endif
  float* out = cfg.part + (int64_t(d) * S + split) * (H * cfg.ldp) + H + n0;
#pragma unroll
  for (int q = 0; q < 16; ++q) {
    const int o = wr * 32 + acc_row(q, lane);
#pragma unroll
    for (int ni = 0; ni < 2; ++ni) {
      const int c = wc * 64 + ni * 32 + r32;
      if (n0 + c < F) out[int64_t(o) * cfg.ldp + c] = acc[ni][q];
    }
  }
}

// dW2_d[o][c] = sum_s part[d][s][o][c] (fixed order) for c < ldp; the dense config
// reduces all 64+F columns, the sparse config the relu(H1) block (the root columns come
// from the root-column body).  A 256-thread group owns 64 consecutive outputs (a tile);
// its 4 waves take splits s = q (mod 4), eight loads in flight each, combined in wave
// order: deterministic.  A 1024-thread block runs 4 groups on 4 consecutive tiles and
// strides over the tiles in step (every group passes the same barriers); `blocks` of
// the configuration share the tiles, so a small grid retires cheaply when the gate
// skips it.

constexpr int kRedSmem = 4 * 4 * 64;
// ad (the step's fused optimiser step, sparse config only): each finished W2_d[o][c < 64]
// gradient updates its parameter and writes the weight images (W2^T and the bf16 splits of
// W2[:, :64]) as bgcn_optim.hip's image tiles do.
__device__ inline void reduce_dw2_body(const float* __restrict__ part, int64_t K2,
                                       float* __restrict__ dw_td, float* __restrict__ dw_bu,
                                       const int32_t* __restrict__ gate, const RedCfg& c0,
                                       const RedCfg& c1, int bid, float* smem, const TailAdam* ad = nullptr) {
  const bool second = bid >= c0.blocks;
  const RedCfg& cfg = second ? c1 : c0;
  const int bl = second ? bid - c0.blocks : bid;
  if (dense_active(gate) != (cfg.want_dense != 0)) return;
  const int S = cfg.S;
  const int64_t ldp = cfg.ldp;
  const int grp = threadIdx.x >> 8, ngrp = int(blockDim.x >> 8);   // 256-thread groups
  float (*red)[64] = reinterpret_cast<float (*)[64]>(smem + grp * 4 * 64);
  const int64_t per = int64_t(H) * ldp;
  const int64_t ntiles = (2 * per + 63) / 64;
  const int q = (threadIdx.x >> 6) & 3, t = threadIdx.x & 63;
  for (int64_t base = int64_t(bl) * ngrp; base < ntiles; base += int64_t(cfg.blocks) * ngrp) {
    const int64_t tile = base + grp;
    const int64_t idx = tile * 64 + t;
    const bool valid = tile < ntiles && idx < 2 * per;
    const int d = valid ? int(idx / per) : 0;
    const int64_t e = valid ? idx % per : 0;
    const float* p = part + int64_t(d) * S * per + e;
    const int64_t o = e / ldp, cw = e % ldp;   // the gradient's W2_d[o][cw] (sparse config: cw < 64)
    const bool fa = ad && ad->on && !cfg.want_dense && q == 0 && valid && cw < H && !ad->skip();
    const int ka = d == 0 ? 2 : 6;
    const int64_t ia = o * K2 + cw;
    float ap = 0.f, am = 0.f, av = 0.f;
    if (fa) {   // requested before the split sums
      ap = ad->p[ka][ia];
      am = ad->m[ka][ia];
      av = ad->v[ka][ia];
    }
    float acc = 0.f;
    int s = q;
    if (valid) {
      for (; s + 28 < S; s += 32) {   // eight loads in flight, summed in split order
        float v[8];
#pragma unroll
        for (int u = 0; u < 8; ++u) v[u] = p[int64_t(s + 4 * u) * per];
#pragma unroll
        for (int u = 0; u < 8; ++u) acc += v[u];
      }
      for (; s < S; s += 4) acc += p[int64_t(s) * per];
    }
    red[q][t] = acc;
    __syncthreads();
    if (q == 0 && valid) {
      const float gsum = ((red[0][t] + red[1][t]) + red[2][t]) + red[3][t];
      (d == 0 ? dw_td : dw_bu)[(e / ldp) * K2 + e % ldp] = gsum;
      if (fa) {
        adam_elem(ap, gsum, am, av, ad->c(ka));
        ad->p[ka][ia] = ap;
        ad->m[ka][ia] = am;
        ad->v[ka][ia] = av;
        if (ad->w2t) {
          ad->w2t[(int64_t(d) * K2 + cw) * H + o] = ap;
          __bf16 x, y, z;
          split3_bf16(ap, x, y, z);
          __bf16* cs = ad->w2s + int64_t(d) * 3 * H * kW2sLd + o * kW2sLd + cw;   // conv2's [o][k]
          cs[0] = x;
          cs[H * kW2sLd] = y;
          cs[2 * H * kW2sLd] = z;
          __bf16* ds = ad->w2d + int64_t(d) * 3 * H * kW2dLd + cw * kW2dLd + o;   // the middle launch's [c][o]
          ds[0] = x;
          ds[H * kW2dLd] = y;
          ds[2 * H * kW2dLd] = z;
        }
      }
    }
    __syncthreads();
  }
}

// dH1[i][d*H + c] = (dZ2_d[i] . W2_d[:, c]) * keep(d,i,c) * s * [H1 > 0], c < H,
// + block partial column sums, over `rows` consecutive nodes (64-row tiles) of direction
// d per block.  A 64-row x 64-column tile per 256-thread block, four waves as 2 row halves
// x 2 column halves, on the bf16 MFMA in the fp32-grade six-product form (mfma_x6,
// bgcn_common.h): dH1 feeds A^T dH1, whose rows at star roots sum thousands of children
// with cancellation, so the three-product form's 2^-16 relative error per product grew to
// 1.2e-4 of max|dW1| at Weibo size (the fp32 reference path: 1e-6); with six products dW1
// is fp32-grade at every size (tests/test_gpu_fullsize.py).  The dZ2 tile is staged in LDS
// split three ways (hi / mid / lo, rows of 72 bf16 = 16-byte aligned, each element split
// once by the staging thread) and W2[:, :64]^T comes split three ways from the weight
// image, so every operand fragment is one 16-byte LDS read.  55 KB of LDS: two blocks per
// CU (splitting per fragment in registers instead fit three per CU in 45 KB but took
// longer: twitter15 0.280 vs 0.276 ms, the two column-half waves split every element
// twice; round 2's three-product form 0.273).
//
// dw2part != nullptr (the sparse path, gated off when the dense path runs): the same
// block also forms the relu(H1) block of dW2 over its rows,
//   part[d][bx][o][c] = sum_i dZ2_d[i][o] * keep(d,i,c) * s * relu(H1_d[i][c]),
// from the operands the dH1 tile already holds: each lane's 16 (row, c) values of H1 and
// of the keep words, in the accumulator row order acc_row(q, h), are its B fragments of
// two 32x32x16 k-steps (element j of step s: row 16s + 8(j>>2) + 4h + (j&3)); the dZ2^T
// fragments are read from the staged tile in that row order.  These products feed dW2
// directly (no fan-in amplification: 2e-5 elementwise at every size), so they keep the
// three-product split.  Two row-half waves are combined in LDS (fixed order).  One block
// per node split (the tail reduces the splits).
// Device body, 256 threads; smem: kDh1Smem floats.
#ifndef BGCN_DH1_X6
#define BGCN_DH1_X6 1   // 0: the three-product form (A/B only: not fp32-grade)
#endif
#ifndef BGCN_DW2P_X6
#define BGCN_DW2P_X6 1   // the relu(H1) block of dW2 in the six-product form (0: three products)
#endif
#ifndef BGCN_DH1_PREFETCH
#define BGCN_DH1_PREFETCH 1   // 0: the next tile's loads issued after the tile (A/B)
#endif
constexpr int kDh1Rows = 64;
constexpr int kDsLd = H + 8;   // bf16 row stride of the staged, split tiles
constexpr int kDh1Smem = (6 * kDh1Rows * kDsLd) / 2 + 2 * H;
// dH1[i][d*H + c] = (dZ2_d[i] . W2_d[:, c]) * keep(d,i,c) * s * [H1 > 0], c < H,
// + block partial column sums, over `rows` consecutive nodes (64-row tiles) of direction
// d per block.  A 64-row x 64-column tile per 256-thread block, four waves as 2 row halves
// x 2 column halves, on the bf16 MFMA in split form (mfma_x3, bgcn_common.h: this launch
// was bound by the f32-input MFMA, 64 cycles per 32x32x2).  The dZ2 tile and W2[:, :64]^T
// are staged in LDS already split (hi / lo bf16, rows of 72 = 16-byte aligned), so every
// operand fragment of dH1 is one 16-byte LDS read.
//
// dw2part != nullptr (the sparse path, gated off when the dense path runs): the same
// block also forms the relu(H1) block of dW2 over its rows,
//   part[d][bx][o][c] = sum_i dZ2_d[i][o] * keep(d,i,c) * s * relu(H1_d[i][c]),
// from the operands the dH1 tile already holds: each lane's 16 (row, c) values of H1 and
// of the keep words, in the accumulator row order acc_row(q, h), are its B fragments of
// two 32x32x16 k-steps (element j of step s: row 16s + 8(j>>2) + 4h + (j&3)); the dZ2^T
// fragments are read from the staged tile in that row order.  Two row-half waves are
// combined in LDS (fixed order).  One block per node split (the tail reduces the splits).
// Device body, 256 threads; smem: kDh1Smem floats.
__device__ inline void dh1_body(const float* __restrict__ dZ2, const float* __restrict__ H1,
                                const float* __restrict__ W2td, const float* __restrict__ W2bu,
                                int64_t ldw2, int64_t N, KeepSrc keep, float* __restrict__ dH1,
                                float* __restrict__ colpart, int64_t rows, float* __restrict__ dw2part,
                                int nsplit, int bx, int d, float* smem,
                                const __bf16* __restrict__ w2d = nullptr) {
  __bf16* Dh = reinterpret_cast<__bf16*>(smem);   // dZ2 tile [row][o], hi / mid / lo
  __bf16* Dm = Dh + kDh1Rows * kDsLd;
  __bf16* Dl = Dm + kDh1Rows * kDsLd;
  __bf16* Wh = Dl + kDh1Rows * kDsLd;             // W2[:, :64]^T [c][o], hi / mid / lo
  __bf16* Wm = Wh + H * kDsLd;
  __bf16* Wl = Wm + H * kDsLd;
  float (*red)[H] = reinterpret_cast<float (*)[H]>(smem + 3 * kDh1Rows * kDsLd);
  const float* W2 = d == 0 ? W2td : W2bu;
  const int wid = threadIdx.x >> 6, l = threadIdx.x & 63;
  const int rh = wid & 1, ch = wid >> 1;
  const int r = l & 31, h = l >> 5;
  const int c = ch * 32 + r;  // output column of this lane (within H)
  const int64_t beg = int64_t(bx) * rows, end = min<int64_t>(beg + rows, N);
  const int ntile = int((end - beg + kDh1Rows - 1) / kDh1Rows);
  const float sc = keep.scale();
  const bool want_dw2 = dw2part != nullptr;

  float4 dv[4];
  float hv[16];
  auto gload = [&](int64_t blk0) {   // one tile's dZ2 rows and this lane's H1 values
#pragma unroll
    for (int u = 0; u < 4; ++u) {    // element e = tid + 256u of a 64 x 16 float4 grid
      const int e = threadIdx.x + 256 * u, rr = e >> 4, q = (e & 15) * 4;
      dv[u] = ld4(dZ2 + min<int64_t>(blk0 + rr, N - 1) * (2 * H) + d * H + q);
    }
#pragma unroll
    for (int q = 0; q < 16; ++q) {
      const int64_t i = min<int64_t>(blk0 + rh * 32 + (q & 3) + 8 * (q >> 2) + 4 * h, N - 1);
      hv[q] = H1[i * (2 * H) + d * H + c];
    }
  };
  if (w2d) {   // the prologue's split image ([2][c][o], hi / lo): 16-byte copies
    
    const __bf16* src = w2d + int64_t(d) * 3 * H * kW2dLd;
    uint4 cv[6];
#pragma unroll
    for (int u = 0; u < 6; ++u) {
      const int e = threadIdx.x + 256 * u, part = e >> 9, c = (e >> 3) & 63, q = (e & 7) * 8;
      cv[u] = *reinterpret_cast<const uint4*>(src + (int64_t(part) * H + c) * kW2dLd + q);
    }
    gload(beg);
#pragma unroll
    for (int u = 0; u < 6; ++u) {
      const int e = threadIdx.x + 256 * u, part = e >> 9, c = (e >> 3) & 63, q = (e & 7) * 8;
      *reinterpret_cast<uint4*>(Wh + (int64_t(part) * H + c) * kDsLd + q) = cv[u];
    }
  } else {
    float4 wv[4];
#pragma unroll
    for (int u = 0; u < 4; ++u) {
      const int e = threadIdx.x + 256 * u, rr = e >> 4, q = (e & 15) * 4;
      wv[u] = ld4(W2 + int64_t(rr) * ldw2 + q);
    }
    gload(beg);
#pragma unroll
    for (int u = 0; u < 4; ++u) {     // W2[o = rr][c = q + t] -> W^T[c][o]
      const int e = threadIdx.x + 256 * u, rr = e >> 4, q = (e & 15) * 4;
      const float v[4] = {wv[u].x, wv[u].y, wv[u].z, wv[u].w};
#pragma unroll
      for (int t = 0; t < 4; ++t)
        split3_bf16(v[t], Wh[(q + t) * kDsLd + rr], Wm[(q + t) * kDsLd + rr], Wl[(q + t) * kDsLd + rr]);
    }
  }
  f32x16 pw0 = {}, pw1 = {};   // dW2 partial: o in [0, 32) / [32, 64), columns ch*32 + r
  float cs = 0.f;
  for (int t = 0; t < ntile; ++t) {
    const int64_t blk0 = beg + int64_t(t) * kDh1Rows;
    const int64_t row0 = blk0 + rh * 32;
#pragma unroll
    for (int u = 0; u < 4; ++u) {
      const int e = threadIdx.x + 256 * u, rr = e >> 4, q = (e & 15) * 4;
      const float v[4] = {dv[u].x, dv[u].y, dv[u].z, dv[u].w};
#pragma unroll
      for (int k = 0; k < 4; ++k) split3_bf16(v[k], Dh[rr * kDsLd + q + k], Dm[rr * kDsLd + q + k], Dl[rr * kDsLd + q + k]);
    }
    // this tile's per-lane operands: a2 = keep * s * relu(H1) split (dW2's B fragments in
    // accumulator row order), bit q of km = kept and H1 > 0 (dH1)
    bf16x8 a2h[2], a2l[2];
#if BGCN_DW2P_X6
    bf16x8 a2m[2];
#endif
    uint32_t km = 0;
#pragma unroll
    for (int q = 0; q < 16; ++q) {
      const int64_t i = row0 + (q & 3) + 8 * (q >> 2) + 4 * h;
      const uint32_t wd = keep.get(uint32_t(d), uint32_t(min<int64_t>(i, N - 1)), uint32_t(c >> 5));
      const bool kept = ((wd >> (c & 31)) & 1u) && i < N;
#if BGCN_DW2P_X6
      __bf16 x, y, z;
      split3_bf16(kept ? sc * fmaxf(hv[q], 0.f) : 0.f, x, y, z);
      a2h[q >> 3][q & 7] = x;
      a2m[q >> 3][q & 7] = y;
      a2l[q >> 3][q & 7] = z;
#else
      __bf16 x, y;
      split_bf16(kept ? sc * fmaxf(hv[q], 0.f) : 0.f, x, y);
      a2h[q >> 3][q & 7] = x;
      a2l[q >> 3][q & 7] = y;
#endif
      km |= uint32_t(kept && hv[q] > 0.f) << q;
      if ((q & 3) == 3) __builtin_amdgcn_sched_barrier(0);   // four keep hashes in flight
    }
    __syncthreads();
#if BGCN_DH1_PREFETCH
    // the next tile's dZ2 rows and H1 values are in flight during this tile's products
    // (dv / hv are consumed above: staged in LDS, folded into km and a2)
    if (t + 1 < ntile) gload(blk0 + kDh1Rows);
#endif
    // dH1: A = dZ2 rows (row rh*32 + r, o = 16s + 8h + j), B = W2^T (column c)
    f32x16 acc = {};
    const __bf16* ah = &Dh[(rh * 32 + r) * kDsLd + 8 * h];
    const __bf16* am = &Dm[(rh * 32 + r) * kDsLd + 8 * h];
    const __bf16* al = &Dl[(rh * 32 + r) * kDsLd + 8 * h];
    const __bf16* bh = &Wh[c * kDsLd + 8 * h];
    const __bf16* bm = &Wm[c * kDsLd + 8 * h];
    const __bf16* bl = &Wl[c * kDsLd + 8 * h];
#pragma unroll
    for (int s = 0; s < 4; ++s) {
#if BGCN_DH1_X6
      acc = mfma_x6(*reinterpret_cast<const bf16x8*>(ah + 16 * s), *reinterpret_cast<const bf16x8*>(am + 16 * s),
                    *reinterpret_cast<const bf16x8*>(al + 16 * s), *reinterpret_cast<const bf16x8*>(bh + 16 * s),
                    *reinterpret_cast<const bf16x8*>(bm + 16 * s), *reinterpret_cast<const bf16x8*>(bl + 16 * s),
                    acc);
#else   // A/B: the three-product form (hi + mid = the two-way split)
      (void)al; (void)bl;
      acc = mfma_x3(*reinterpret_cast<const bf16x8*>(ah + 16 * s), *reinterpret_cast<const bf16x8*>(am + 16 * s),
                    *reinterpret_cast<const bf16x8*>(bh + 16 * s), *reinterpret_cast<const bf16x8*>(bm + 16 * s), acc);
#endif
      __builtin_amdgcn_sched_barrier(0);   // one k-step's fragments live at a time
    }
    __builtin_amdgcn_sched_barrier(0);
#pragma unroll
    for (int q = 0; q < 16; ++q) {
      const int64_t i = row0 + (q & 3) + 8 * (q >> 2) + 4 * h;
      const float g = ((km >> q) & 1u) ? acc[q] * sc : 0.f;
      if (i < N) {
        dH1[i * (2 * H) + d * H + c] = g;
        cs += g;
      }
    }
    if (want_dw2) {
      // dW2: A = dZ2^T (o = r / 32 + r, rows in the a2 fragments' order), B = a2
#pragma unroll
      for (int s = 0; s < 2; ++s) {
#if BGCN_DW2P_X6
        // the fp32-grade six-product form (both operands split three ways, ~2^-24 relative):
        // the three-product form's ~1e-5 left the relu(H1) block of dW2 only 4-8x under
        // the 1e-4 bar at full size (profiles/r04_parity_*.json)
        bf16x8 z0h, z0m, z0l, z1h, z1m, z1l;
#pragma unroll
        for (int j = 0; j < 8; ++j) {
          const int k = rh * 32 + 16 * s + 8 * (j >> 2) + 4 * h + (j & 3);
          z0h[j] = Dh[k * kDsLd + r];
          z0m[j] = Dm[k * kDsLd + r];
          z0l[j] = Dl[k * kDsLd + r];
          z1h[j] = Dh[k * kDsLd + 32 + r];
          z1m[j] = Dm[k * kDsLd + 32 + r];
          z1l[j] = Dl[k * kDsLd + 32 + r];
        }
        pw0 = mfma_x6(z0h, z0m, z0l, a2h[s], a2m[s], a2l[s], pw0);
        pw1 = mfma_x6(z1h, z1m, z1l, a2h[s], a2m[s], a2l[s], pw1);
#else
        bf16x8 z0h, z0l, z1h, z1l;
#pragma unroll
        for (int j = 0; j < 8; ++j) {
          const int k = rh * 32 + 16 * s + 8 * (j >> 2) + 4 * h + (j & 3);
          z0h[j] = Dh[k * kDsLd + r];
          z0l[j] = Dm[k * kDsLd + r];
          z1h[j] = Dh[k * kDsLd + 32 + r];
          z1l[j] = Dm[k * kDsLd + 32 + r];
        }
        pw0 = mfma_x3(z0h, z0l, a2h[s], a2l[s], pw0);
        pw1 = mfma_x3(z1h, z1l, a2h[s], a2l[s], pw1);
#endif
        __builtin_amdgcn_sched_barrier(0);
      }
    }
    __syncthreads();   // the staged tile is rewritten by the next tile
#if !BGCN_DH1_PREFETCH
    if (t + 1 < ntile) gload(blk0 + kDh1Rows);
#endif
  }
  cs += __shfl_xor(cs, 32);
  if (h == 0) red[rh][c] = cs;
  __syncthreads();
  if (threadIdx.x < H)
    colpart[int64_t(bx) * (2 * H) + d * H + threadIdx.x] = red[0][threadIdx.x] + red[1][threadIdx.x];
  if (!want_dw2) return;
  // combine the two row halves: rh = 1 parks its partial in LDS, rh = 0 adds and stores
  float* P = smem;   // [64 o][64 c] over the staged tiles (free after the loop's barrier)
  if (rh == 1) {
#pragma unroll
    for (int q = 0; q < 16; ++q) {
      const int o = acc_row(q, l);
      P[o * H + c] = pw0[q];
      P[(32 + o) * H + c] = pw1[q];
    }
  }
  __syncthreads();
  if (rh == 0) {
    float* out = dw2part + (int64_t(d) * nsplit + bx) * (H * H);
#pragma unroll
    for (int q = 0; q < 16; ++q) {
      const int o = acc_row(q, l);
      out[o * H + c] = pw0[q] + P[o * H + c];
      out[(32 + o) * H + c] = pw1[q] + P[(32 + o) * H + c];
    }
  }
}



}  // namespace bgcn
