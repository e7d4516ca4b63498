// K2 / K10: the dense GEMMs of GCNConv.lin on MFMA (fp32 in, fp32 accumulate).
//
// The reference runs lin BEFORE propagate (PyG >= 2.0 GCNConv), so conv1 is the
// genuine dense (N x 5000) . (5000 x 64) product; its weight gradient is the
// (64 x N) . (N x 5000) product.  Both directions (TD, BU) read the same X, so the
// build fuses them: one pass over X against [W1_td ; W1_bu] (128 columns) forward
// and one pass over X for [dZ1_td | dZ1_bu]^T backward.
//
// gfx950 has exact f32-in MFMA (v_mfma_f32_32x32x2_f32, a k-ordered f32 fma chain,
// 64 FLOP/clk/SIMD = 157 TFLOP/s chip peak).  Tiles are staged global -> VGPR -> LDS
// (register staging, one LDS double buffer, one barrier per K step; the next tile's
// global loads are issued before the current tile's MFMAs).
//
// MFMA 32x32x2 f32 operand maps (cdna_hip_programming.md section 3): lane l supplies
// A[i = l&31][k = l>>5] and B[k = l>>5][j = l&31]; D register r of lane l is
// D[row = (r&3) + 8*(r>>2) + 4*(l>>5)][col = l&31].
#include <cstdlib>

#include "bgcn_internal.h"

namespace bgcn {

constexpr int BK = 32;

__device__ __forceinline__ int acc_row(int r, int lane) { return (r & 3) + 8 * (r >> 2) + 4 * (lane >> 5); }

// ============================================================================
// Y[M, Nc] = X[M, K] . W[Nc, K]^T.   Block tile 64 x 128, 4 waves as 2 x 2,
// wave tile 32 x 64 (two 32x32 accumulators).  LDS tiles are row-major with a
// 33-float stride (conflict-free ds_read_b32 for the column-of-rows read).
// ============================================================================
// BKM = false: W is [Nc, K] (Y = X W^T, GCNConv.lin forward);
// BKM = true : W is [K, Nc] (Y = X W, the input gradient dX = dZ W of GCNConv.lin),
//              staged k-major in LDS.  W1/split are ignored for BKM.
template <bool VEC, bool BKM, class TX = float>
__global__ __launch_bounds__(256) void k_gemm_xwt(const TX* __restrict__ X, int64_t ldx,
                                                  const float* __restrict__ W0,
                                                  const float* __restrict__ W1, int64_t ldw,
                                                  int64_t split, float* __restrict__ Y,
                                                  int64_t ldy, int64_t M, int64_t Nc, int64_t K,
                                                  const int32_t* __restrict__ gate) {
  if (gate_closed(gate)) return;
  constexpr int BM = 64, BN = 128, LS = BK + 1;
  __shared__ float As[2][BM * LS];
  __shared__ float Bs[2][BN * LS];  // BKM: [BK][BN] (fits: BK*BN <= BN*LS)
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int wr = wave >> 1, wc = wave & 1;
  const int64_t m0 = int64_t(blockIdx.x) * BM, n0 = int64_t(blockIdx.y) * BN;
  const int srow = tid >> 3, skq = (tid & 7) * 4;  // staging: row, k offset (float4)

  const TX* arow[2];
  bool aok[2];
#pragma unroll
  for (int i = 0; i < 2; ++i) {
    int64_t m = m0 + srow + 32 * i;
    aok[i] = m < M;
    arow[i] = X + (aok[i] ? m : 0) * ldx;
  }
  const float* brow[4];
  bool bok[4];
#pragma unroll
  for (int i = 0; i < 4; ++i) {
    int64_t n = n0 + srow + 32 * i;
    bok[i] = n < Nc;
    int64_t nn = bok[i] ? n : 0;
    brow[i] = nn < split ? W0 + nn * ldw : W1 + (nn - split) * ldw;
  }

  // BKM staging: k = tid/32 + 8 i, n quad (tid%32)*4
  const int bk_k = tid >> 5, bk_n = (tid & 31) * 4;
  float4 ra[2], rb[4];
  auto gload = [&](int64_t k0) {
    int64_t k = k0 + skq;
#pragma unroll
    for (int i = 0; i < 2; ++i) {
      if (VEC) {
        ra[i] = (aok[i] && k < K) ? xq(arow[i] + k) : f4zero();
      } else {
        float t[4];
#pragma unroll
        for (int j = 0; j < 4; ++j) t[j] = (aok[i] && k + j < K) ? xs(arow[i] + k + j) : 0.f;
        ra[i] = make_float4(t[0], t[1], t[2], t[3]);
      }
    }
    if constexpr (BKM) {
#pragma unroll
      for (int i = 0; i < 4; ++i) {
        int64_t kk = k0 + bk_k + 8 * i, n = n0 + bk_n;
        if (VEC) {
          rb[i] = (kk < K && n < Nc) ? ld4(W0 + kk * ldw + n) : f4zero();
        } else {
          float t[4];
#pragma unroll
          for (int j = 0; j < 4; ++j) t[j] = (kk < K && n + j < Nc) ? W0[kk * ldw + n + j] : 0.f;
          rb[i] = make_float4(t[0], t[1], t[2], t[3]);
        }
      }
    } else {
#pragma unroll
      for (int i = 0; i < 4; ++i) {
        if (VEC) {
          rb[i] = (bok[i] && k < K) ? ld4(brow[i] + k) : f4zero();
        } else {
          float t[4];
#pragma unroll
          for (int j = 0; j < 4; ++j) t[j] = (bok[i] && k + j < K) ? brow[i][k + j] : 0.f;
          rb[i] = make_float4(t[0], t[1], t[2], t[3]);
        }
      }
    }
  };
  auto sstore = [&](int buf) {
#pragma unroll
    for (int i = 0; i < 2; ++i) {
      float* d = &As[buf][(srow + 32 * i) * LS + skq];
      d[0] = ra[i].x; d[1] = ra[i].y; d[2] = ra[i].z; d[3] = ra[i].w;
    }
    if constexpr (BKM) {
#pragma unroll
      for (int i = 0; i < 4; ++i) st4(&Bs[buf][(bk_k + 8 * i) * BN + bk_n], rb[i]);
    } else {
#pragma unroll
      for (int i = 0; i < 4; ++i) {
        float* d = &Bs[buf][(srow + 32 * i) * LS + skq];
        d[0] = rb[i].x; d[1] = rb[i].y; d[2] = rb[i].z; d[3] = rb[i].w;
      }
    }
  };

  f32x16 acc0 = {0}, acc1 = {0};
  const int h = lane >> 5, r32 = lane & 31;
  const int nk = int((K + BK - 1) / BK);
  gload(0);
  sstore(0);
  __syncthreads();
  for (int kt = 0; kt < nk; ++kt) {
    const int buf = kt & 1;
    if (kt + 1 < nk) gload(int64_t(kt + 1) * BK);
    const float* A = &As[buf][(wr * 32 + r32) * LS + h];
    if constexpr (BKM) {
      const float* B0 = &Bs[buf][h * BN + wc * 64 + r32];
#pragma unroll
      for (int s = 0; s < BK / 2; ++s) {
        float a = A[2 * s], b0 = B0[2 * s * BN], b1 = B0[2 * s * BN + 32];
        acc0 = mfma32x32x2(a, b0, acc0);
        acc1 = mfma32x32x2(a, b1, acc1);
      }
    } else {
      const float* B0 = &Bs[buf][(wc * 64 + r32) * LS + h];
      const float* B1 = B0 + 32 * LS;
#pragma unroll
      for (int s = 0; s < BK / 2; ++s) {
        float a = A[2 * s], b0 = B0[2 * s], b1 = B1[2 * s];
        acc0 = mfma32x32x2(a, b0, acc0);
        acc1 = mfma32x32x2(a, b1, acc1);
      }
    }
    if (kt + 1 < nk) sstore(buf ^ 1);
    __syncthreads();
  }
#pragma unroll
  for (int r = 0; r < 16; ++r) {
    int64_t m = m0 + wr * 32 + acc_row(r, lane);
    if (m >= M) continue;
    int64_t n = n0 + wc * 64 + r32;
    if (n < Nc) Y[m * ldy + n] = acc0[r];
    if (n + 32 < Nc) Y[m * ldy + n + 32] = acc1[r];
  }
}

// ============================================================================
// Partial C_s[Mc, Nc] = G[Ks, Mc]^T . X[Ks, Nc] over the node chunk Ks of split s.
// Block tile 128 (Mc) x 64 (Nc), waves 2 x 2 -> wave tile 64 x 32.  Both operands
// are k-major in memory (rows = nodes) and staged k-major in LDS (no padding: the
// MFMA read is 32 consecutive floats per half-wave).
// ============================================================================
template <bool VEC, class TX = float>
__global__ __launch_bounds__(256) void k_gemm_tn(const float* __restrict__ G, int64_t ldg,
                                                 const TX* __restrict__ X, int64_t ldx,
                                                 float* __restrict__ part, int64_t Mc, int64_t Nc,
                                                 int64_t K, int64_t kchunk,
                                                 const int32_t* __restrict__ gate) {
  if (gate_closed(gate)) return;
  constexpr int BM = 128, BN = 64;
  __shared__ float Gs[2][BK * BM];
  __shared__ float Xs[2][BK * BN];
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int wr = wave >> 1, wc = wave & 1;
  const int64_t n0 = int64_t(blockIdx.x) * BN, m0 = int64_t(blockIdx.y) * BM;
  const int64_t kb = int64_t(blockIdx.z) * kchunk;
  const int64_t ke = min<int64_t>(kb + kchunk, K);
  float* out = part + int64_t(blockIdx.z) * Mc * Nc;

  // staging maps: G tile 32 nodes x 128 -> 4 float4/thread; X tile 32 x 64 -> 2 float4/thread
  const int g_node = tid >> 5, g_q = (tid & 31) * 4;
  const int x_node = tid >> 4, x_q = (tid & 15) * 4;
  float4 rg[4], rx[2];
  auto gload = [&](int64_t k0) {
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      int64_t k = k0 + g_node + 8 * i;
      int64_t m = m0 + g_q;
      if (VEC) {
        rg[i] = (k < ke && m < Mc) ? ld4(G + k * ldg + m) : f4zero();
      } else {
        float t[4];
#pragma unroll
        for (int j = 0; j < 4; ++j) t[j] = (k < ke && m + j < Mc) ? G[k * ldg + m + j] : 0.f;
        rg[i] = make_float4(t[0], t[1], t[2], t[3]);
      }
    }
#pragma unroll
    for (int i = 0; i < 2; ++i) {
      int64_t k = k0 + x_node + 16 * i;
      int64_t n = n0 + x_q;
      if (VEC) {
        rx[i] = (k < ke && n < Nc) ? xq(X + k * ldx + n) : f4zero();
      } else {
        float t[4];
#pragma unroll
        for (int j = 0; j < 4; ++j) t[j] = (k < ke && n + j < Nc) ? xs(X + k * ldx + n + j) : 0.f;
        rx[i] = make_float4(t[0], t[1], t[2], t[3]);
      }
    }
  };
  auto sstore = [&](int buf) {
#pragma unroll
    for (int i = 0; i < 4; ++i) st4(&Gs[buf][(g_node + 8 * i) * BM + g_q], rg[i]);
#pragma unroll
    for (int i = 0; i < 2; ++i) st4(&Xs[buf][(x_node + 16 * i) * BN + x_q], rx[i]);
  };

  f32x16 acc0 = {0}, acc1 = {0};
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
    const float* A0 = &Gs[buf][h * BM + wr * 64 + r32];
    const float* Bp = &Xs[buf][h * BN + wc * 32 + r32];
#pragma unroll
    for (int s = 0; s < BK / 2; ++s) {
      float a0 = A0[2 * s * BM], a1 = A0[2 * s * BM + 32], b = Bp[2 * s * BN];
      acc0 = mfma32x32x2(a0, b, acc0);
      acc1 = mfma32x32x2(a1, b, acc1);
    }
    if (kt + 1 < nk) sstore(buf ^ 1);
    __syncthreads();
  }
#pragma unroll
  for (int r = 0; r < 16; ++r) {
    int64_t n = n0 + wc * 32 + r32;
    if (n >= Nc) continue;
    int64_t m = m0 + wr * 64 + acc_row(r, lane);
    if (m < Mc) out[m * Nc + n] = acc0[r];
    if (m + 32 < Mc) out[(m + 32) * Nc + n] = acc1[r];
  }
}

// The same partials with a 64 x 64 wave tile (block 128 x 128, four accumulators per
// wave): one LDS operand read per f32 MFMA instead of 1.5, and a third less global
// traffic per flop; 64 KB of LDS, two blocks per CU.  Vector-aligned operands only.
#ifndef BGCN_TN_WIDE_BK
#define BGCN_TN_WIDE_BK 16   // k-tile depth (nodes; kchunk stays a multiple of BK = 32): 32 KB of LDS,
                             // four blocks per CU (32: 0.345 ms, 16: 0.322, 8: 0.327 at twitter15)
#endif
__global__ __launch_bounds__(256) void k_gemm_tn_w(const float* __restrict__ G, int64_t ldg,
                                                   const float* __restrict__ X, int64_t ldx,
                                                   float* __restrict__ part, int64_t Mc, int64_t Nc,
                                                   int64_t K, int64_t kchunk,
                                                   const int32_t* __restrict__ gate) {
  if (gate_closed(gate)) return;
  constexpr int BM = 128, BN = 128, TK = BGCN_TN_WIDE_BK;
  __shared__ float Gs[2][TK * BM];
  __shared__ float Xs[2][TK * BN];
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int wr = wave >> 1, wc = wave & 1;
  const int64_t n0 = int64_t(blockIdx.x) * BN, m0 = int64_t(blockIdx.y) * BM;
  const int64_t kb = int64_t(blockIdx.z) * kchunk;
  const int64_t ke = min<int64_t>(kb + kchunk, K);
  float* out = part + int64_t(blockIdx.z) * Mc * Nc;
  // staging maps: both tiles TK nodes x 128 -> TK / 8 float4 per thread each
  const int s_node = tid >> 5, s_q = (tid & 31) * 4;
  float4 rg[TK / 8], rx[TK / 8];
  auto gload = [&](int64_t k0) {
#pragma unroll
    for (int i = 0; i < TK / 8; ++i) {
      const int64_t k = k0 + s_node + 8 * i;
      const int64_t m = m0 + s_q, n = n0 + s_q;
      rg[i] = (k < ke && m < Mc) ? ld4(G + k * ldg + m) : f4zero();
      rx[i] = (k < ke && n < Nc) ? ld4(X + k * ldx + n) : f4zero();
    }
  };
  auto sstore = [&](int buf) {
#pragma unroll
    for (int i = 0; i < TK / 8; ++i) {
      st4(&Gs[buf][(s_node + 8 * i) * BM + s_q], rg[i]);
      st4(&Xs[buf][(s_node + 8 * i) * BN + s_q], rx[i]);
    }
  };
  f32x16 acc[2][2] = {};
  const int h = lane >> 5, r32 = lane & 31;
  const int nk = int((ke - kb + TK - 1) / TK);
  if (nk > 0) {
    gload(kb);
    sstore(0);
  }
  __syncthreads();
  for (int kt = 0; kt < nk; ++kt) {
    const int buf = kt & 1;
    if (kt + 1 < nk) gload(kb + int64_t(kt + 1) * TK);
    const float* A0 = &Gs[buf][h * BM + wr * 64 + r32];
    const float* B0 = &Xs[buf][h * BN + wc * 64 + r32];
#pragma unroll
    for (int s = 0; s < TK / 2; ++s) {
      const float a0 = A0[2 * s * BM], a1 = A0[2 * s * BM + 32];
      const float b0 = B0[2 * s * BN], b1 = B0[2 * s * BN + 32];
      acc[0][0] = mfma32x32x2(a0, b0, acc[0][0]);
      acc[0][1] = mfma32x32x2(a0, b1, acc[0][1]);
      acc[1][0] = mfma32x32x2(a1, b0, acc[1][0]);
      acc[1][1] = mfma32x32x2(a1, b1, acc[1][1]);
    }
    if (kt + 1 < nk) sstore(buf ^ 1);
    __syncthreads();
  }
#pragma unroll
  for (int r = 0; r < 16; ++r) {
#pragma unroll
    for (int j = 0; j < 2; ++j) {
      const int64_t n = n0 + wc * 64 + j * 32 + r32;
      if (n >= Nc) continue;
#pragma unroll
      for (int i = 0; i < 2; ++i) {
        const int64_t m = m0 + wr * 64 + i * 32 + acc_row(r, lane);
        if (m < Mc) out[m * Nc + n] = acc[i][j][r];
      }
    }
  }
}

// ============================================================================
// bf16 X on the bf16 MFMA (v_mfma_f32_32x32x16_bf16, 16x the k-depth of the f32 MFMA per
// instruction).  Bag-of-words X is exact in bf16; the fp32 operand (W, or dZ1) is split
// into hi + mid + lo bf16 parts (split3_bf16: all 24 mantissa bits), so each k-step takes
// three products (small terms first) and the result is fp32-grade - conv1's output feeds a
// relu, where a 1e-5 relative error flips relu' for entries near zero.  Both kernels stage
// k-contiguous bf16 rows in LDS (row stride kB16LD: 16-byte aligned ds_read_b128 per lane)
// through registers (next tile's global loads in flight during the current tile's MFMAs).
// Lane map of 32x32x16: lane (h = l >> 5, r = l & 31) supplies A[r][8h + j] and
// B[8h + j][r] (j < 8); D register q is D[(q & 3) + 8 (q >> 2) + 4h][r].
// ============================================================================
constexpr int kB16BK = 32, kB16LD = kB16BK + 8;   // (64-wide k-tiles measured slower: 0.67 / 0.87 ms)
typedef unsigned int u32x4v __attribute__((ext_vector_type(4)));

// X's bf16 planes: bf16 X is exact (one plane, three products per k-step); fp32 X is split
// three ways like the fp32 operand (three planes, mfma_x6: six products, fp32-grade) - the
// f32-input MFMA issues at 1/16 of the bf16 rate, so six bf16 products are still ~2.7x
// its throughput (BGCN_GEMM_X6=0, read once, keeps the f32 MFMA kernels for fp32 X)
template <class TX> struct XPlanes { static constexpr int P = sizeof(TX) == 2 ? 1 : 3; };
// the split planes of 8 consecutive X elements (16 B bf16 / 32 B fp32 in registers)
template <class TX> struct XPiece;
template <> struct XPiece<bf16_t> {
  u32x4v v;
  __device__ __forceinline__ void load(const bf16_t* p, bool ok) {
    const u32x4v t = *reinterpret_cast<const u32x4v*>(p);
    v = ok ? t : u32x4v{0u, 0u, 0u, 0u};
  }
  __device__ __forceinline__ void store(__bf16* const* planes, int o) const {
    *reinterpret_cast<u32x4v*>(planes[0] + o) = v;
  }
};
template <> struct XPiece<float> {
  float4 v[2];
  __device__ __forceinline__ void load(const float* p, bool ok) {
    const float4 a = ld4(p), b = ld4(p + 4);
    v[0] = ok ? a : f4zero();
    v[1] = ok ? b : f4zero();
  }
  __device__ __forceinline__ void store(__bf16* const* planes, int o) const {
    bf16x8 h, m, l;
    const float e[8] = {v[0].x, v[0].y, v[0].z, v[0].w, v[1].x, v[1].y, v[1].z, v[1].w};
#pragma unroll
    for (int j = 0; j < 8; ++j) {
      __bf16 x, y, z;
      split3_bf16(e[j], x, y, z);
      h[j] = x; m[j] = y; l[j] = z;
    }
    *reinterpret_cast<bf16x8*>(planes[0] + o) = h;
    *reinterpret_cast<bf16x8*>(planes[1] + o) = m;
    *reinterpret_cast<bf16x8*>(planes[2] + o) = l;
  }
};
// acc += a.b with a in PA planes and b in PB (one exact operand: three products; both split
// three ways: six, mfma_x6)
template <int PA, int PB>
__device__ __forceinline__ f32x16 mfma_planes(const bf16x8 (&a)[PA], const bf16x8 (&b)[PB], f32x16 c) {
  if constexpr (PA == 1) {
    c = mfma_bf16(a[0], b[2], c);
    c = mfma_bf16(a[0], b[1], c);
    return mfma_bf16(a[0], b[0], c);
  } else if constexpr (PB == 1) {
    c = mfma_bf16(a[2], b[0], c);
    c = mfma_bf16(a[1], b[0], c);
    return mfma_bf16(a[0], b[0], c);
  } else {
    return mfma_x6(a[0], a[1], a[2], b[0], b[1], b[2], c);
  }
}

// Y[M, Nc] = X[M, K] (bf16 or fp32) . W[Nc, K]^T (fp32; rows [0, split) from W0, the rest
// W1).  Block tile 128 x 128 (4 waves as 2 x 2, wave tile 64 x 64), K % 8 == 0, ldx % 8 == 0.
template <class TX>
__global__ __launch_bounds__(256) void k_gemm_xwt_bf16(const TX* __restrict__ X, int64_t ldx,
                                                       const float* __restrict__ W0,
                                                       const float* __restrict__ W1, int64_t ldw,
                                                       int64_t split, float* __restrict__ Y, int64_t ldy,
                                                       int64_t M, int64_t Nc, int64_t K,
                                                       const int32_t* __restrict__ gate) {
  if (gate_closed(gate)) return;
  constexpr int BM = 128, BN = 128, PX = XPlanes<TX>::P;
  __shared__ __attribute__((aligned(16))) __bf16 As[PX][BM * kB16LD];
  __shared__ __attribute__((aligned(16))) __bf16 Bs[3][BN * kB16LD];
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int wr = wave >> 1, wc = wave & 1, h = lane >> 5, r32 = lane & 31;
  const int64_t m0 = int64_t(blockIdx.x) * BM, n0 = int64_t(blockIdx.y) * BN;
  // staging: X rows tid / 4 + 64 i, 8 k at (tid % 4) * 8; W row tid % 128, 16 k at (tid / 128) * 16
  // (each lane writes its row's contiguous k-range per plane as 16-byte LDS stores on
  // consecutive rows across lanes, conflict-free; one 2-byte store per element per plane
  // kept the waves parked at the barriers)
  constexpr int kXR = BM * kB16BK / 8 / 256;   // 8-element X pieces per thread
  constexpr int kWK = kB16BK / 2;               // W elements per thread (one row, kWK consecutive k)
  const int xr = tid / (kB16BK / 8), xk = (tid % (kB16BK / 8)) * 8;
  const int wrow = tid & 127, wk = (tid >> 7) * kWK;
  const TX* xp[kXR];
  bool xok[kXR];
#pragma unroll
  for (int i = 0; i < kXR; ++i) {
    const int64_t m = m0 + xr + (256 / (kB16BK / 8)) * i;
    xok[i] = m < M;
    xp[i] = X + (xok[i] ? m : 0) * ldx;
  }
  const int64_t wn = n0 + wrow;
  const bool wok = wn < Nc;
  const float* wp = (wok ? wn : 0) < split ? W0 + (wok ? wn : 0) * ldw : W1 + ((wok ? wn : 0) - split) * ldw;
  XPiece<TX> ra[kXR];
  float4 rb[kWK / 4];
  __bf16* aplanes[PX];
#pragma unroll
  for (int p = 0; p < PX; ++p) aplanes[p] = As[p];
  auto gload = [&](int64_t k0) {
#pragma unroll
    for (int i = 0; i < kXR; ++i) {
      const int64_t k = k0 + xk;
      const bool ok = xok[i] && k < K;
      ra[i].load(xp[i] + (ok ? k : 0), ok);
    }
#pragma unroll
    for (int i = 0; i < kWK / 4; ++i) {
      const int64_t k = k0 + wk + 4 * i;
      const bool ok = wok && k < K;
      const float4 v = ld4(wp + (ok ? k : 0));
      rb[i] = ok ? v : f4zero();
    }
  };
  auto sstore = [&]() {
#pragma unroll
    for (int i = 0; i < kXR; ++i) ra[i].store(aplanes, (xr + (256 / (kB16BK / 8)) * i) * kB16LD + xk);
    bf16x8 hv[kWK / 8], mv[kWK / 8], lv[kWK / 8];
#pragma unroll
    for (int i = 0; i < kWK / 4; ++i) {
      const float v[4] = {rb[i].x, rb[i].y, rb[i].z, rb[i].w};
#pragma unroll
      for (int e = 0; e < 4; ++e) {
        __bf16 x, y, z;
        split3_bf16(v[e], x, y, z);
        hv[i >> 1][(i & 1) * 4 + e] = x;
        mv[i >> 1][(i & 1) * 4 + e] = y;
        lv[i >> 1][(i & 1) * 4 + e] = z;
      }
    }
    const int o = wrow * kB16LD + wk;
#pragma unroll
    for (int j = 0; j < kWK / 8; ++j) {
      *reinterpret_cast<bf16x8*>(&Bs[0][o + 8 * j]) = hv[j];
      *reinterpret_cast<bf16x8*>(&Bs[1][o + 8 * j]) = mv[j];
      *reinterpret_cast<bf16x8*>(&Bs[2][o + 8 * j]) = lv[j];
    }
  };
  f32x16 acc[2][2] = {};
  const int nk = int((K + kB16BK - 1) / kB16BK);
  gload(0);
  sstore();
  __syncthreads();
  for (int kt = 0; kt < nk; ++kt) {
    if (kt + 1 < nk) gload(int64_t(kt + 1) * kB16BK);
#pragma unroll
    for (int s = 0; s < kB16BK / 16; ++s) {
      const int ko = 16 * s + 8 * h;
      bf16x8 a[2][PX], b[2][3];
#pragma unroll
      for (int mi = 0; mi < 2; ++mi)
#pragma unroll
        for (int p = 0; p < PX; ++p)
          a[mi][p] = *reinterpret_cast<const bf16x8*>(&As[p][(wr * 64 + mi * 32 + r32) * kB16LD + ko]);
#pragma unroll
      for (int p = 0; p < 3; ++p)
#pragma unroll
        for (int ni = 0; ni < 2; ++ni)
          b[ni][p] = *reinterpret_cast<const bf16x8*>(&Bs[p][(wc * 64 + ni * 32 + r32) * kB16LD + ko]);
#pragma unroll
      for (int mi = 0; mi < 2; ++mi)
#pragma unroll
        for (int ni = 0; ni < 2; ++ni) acc[mi][ni] = mfma_planes<PX, 3>(a[mi], b[ni], acc[mi][ni]);
    }
    __syncthreads();
    if (kt + 1 < nk) {
      sstore();
      __syncthreads();
    }
  }
#pragma unroll
  for (int mi = 0; mi < 2; ++mi)
#pragma unroll
    for (int q = 0; q < 16; ++q) {
      const int64_t m = m0 + wr * 64 + mi * 32 + acc_row(q, lane);
      if (m >= M) continue;
#pragma unroll
      for (int ni = 0; ni < 2; ++ni) {
        const int64_t n = n0 + wc * 64 + ni * 32 + r32;
        if (n < Nc) Y[m * ldy + n] = acc[mi][ni][q];
      }
    }
}

// Partial C_s[Mc, Nc] = G[Ks, Mc]^T (fp32, split) . X[Ks, Nc] (bf16 or fp32, XPlanes) over
// the node chunk of split s.  Block tile 128 (Mc) x 128 (Nc), 4 waves as 2 x 2.  Both
// operands are k-major in memory (rows = nodes): staged transposed into k-contiguous LDS
// rows.  Nc % 8 == 0, ldx % 8 == 0, ldg % 4 == 0.
template <class TX>
__global__ __launch_bounds__(256) void k_gemm_tn_bf16(const float* __restrict__ G, int64_t ldg,
                                                      const TX* __restrict__ X, int64_t ldx,
                                                      float* __restrict__ part, int64_t Mc, int64_t Nc,
                                                      int64_t K, int64_t kchunk,
                                                      const int32_t* __restrict__ gate) {
  if (gate_closed(gate)) return;
  constexpr int BM = 128, BN = 128, PX = XPlanes<TX>::P;
  __shared__ __attribute__((aligned(16))) __bf16 As[3][BM * kB16LD];
  __shared__ __attribute__((aligned(16))) __bf16 Bs[PX][BN * kB16LD];
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int wr = wave >> 1, wc = wave & 1, h = lane >> 5, r32 = lane & 31;
  const int64_t n0 = int64_t(blockIdx.x) * BN, m0 = int64_t(blockIdx.y) * BM;
  const int64_t kb = int64_t(blockIdx.z) * kchunk;
  const int64_t ke = min<int64_t>(kb + kchunk, K);
  float* out = part + int64_t(blockIdx.z) * Mc * Nc;
  // staging, transposed into k-contiguous LDS rows: thread t takes column m = t % 128 of G
  // and column n = t % 128 of X over the 16 nodes (t / 128) * 16 ..: lanes load consecutive
  // columns (coalesced) and each writes its row's 32 contiguous bytes per plane as two
  // 16-byte LDS stores on consecutive rows across lanes, conflict-free (two nodes per 4-byte
  // store with lanes 8 rows apart hit 2 of 64 banks: 88 % of the LDS cycles were conflicts,
  // profiles/r03_dense_bf16_pmc.txt)
  constexpr int kNK = kB16BK / 2;   // nodes per thread
  const int sc_ = tid & 127, sk = (tid >> 7) * kNK;
  float rg[kNK];
  float rx[kNK];
  auto gload = [&](int64_t k0) {
    const int64_t m = m0 + sc_, n = n0 + sc_;
#pragma unroll
    for (int u = 0; u < kNK; ++u) {
      const int64_t k = k0 + sk + u;
      const bool okg = k < ke && m < Mc, okx = k < ke && n < Nc;
      const float g = G[(okg ? k : 0) * ldg + (okg ? m : 0)];
      const float x = xs(X + (okx ? k : 0) * ldx + (okx ? n : 0));
      rg[u] = okg ? g : 0.f;
      rx[u] = okx ? x : 0.f;
    }
  };
  auto split_store = [&](const float (&r)[kNK], __bf16* p0, __bf16* p1, __bf16* p2) {
    bf16x8 hv[kNK / 8], mv[kNK / 8], lv[kNK / 8];
#pragma unroll
    for (int u = 0; u < kNK; ++u) {
      __bf16 x, y, z;
      split3_bf16(r[u], x, y, z);
      hv[u >> 3][u & 7] = x;
      mv[u >> 3][u & 7] = y;
      lv[u >> 3][u & 7] = z;
    }
    const int o = sc_ * kB16LD + sk;
#pragma unroll
    for (int j = 0; j < kNK / 8; ++j) {
      *reinterpret_cast<bf16x8*>(p0 + o + 8 * j) = hv[j];
      if (p1) *reinterpret_cast<bf16x8*>(p1 + o + 8 * j) = mv[j];
      if (p2) *reinterpret_cast<bf16x8*>(p2 + o + 8 * j) = lv[j];
    }
  };
  auto sstore = [&]() {
    split_store(rg, As[0], As[1], As[2]);
    if constexpr (PX == 1)   // bf16 X: exact, one plane (the conversion back is exact)
      split_store(rx, Bs[0], nullptr, nullptr);
    else
      split_store(rx, Bs[0], Bs[PX > 1 ? 1 : 0], Bs[PX > 2 ? 2 : 0]);
  };
  f32x16 acc[2][2] = {};
  const int nk = int((ke - kb + kB16BK - 1) / kB16BK);
  if (nk > 0) {
    gload(kb);
    sstore();
  }
  __syncthreads();
  for (int kt = 0; kt < nk; ++kt) {
    if (kt + 1 < nk) gload(kb + int64_t(kt + 1) * kB16BK);
#pragma unroll
    for (int s = 0; s < kB16BK / 16; ++s) {
      const int ko = 16 * s + 8 * h;
      bf16x8 a[2][3], b[2][PX];
#pragma unroll
      for (int p = 0; p < 3; ++p)
#pragma unroll
        for (int mi = 0; mi < 2; ++mi)
          a[mi][p] = *reinterpret_cast<const bf16x8*>(&As[p][(wr * 64 + mi * 32 + r32) * kB16LD + ko]);
#pragma unroll
      for (int p = 0; p < PX; ++p)
#pragma unroll
        for (int ni = 0; ni < 2; ++ni)
          b[ni][p] = *reinterpret_cast<const bf16x8*>(&Bs[p][(wc * 64 + ni * 32 + r32) * kB16LD + ko]);
#pragma unroll
      for (int mi = 0; mi < 2; ++mi)
#pragma unroll
        for (int ni = 0; ni < 2; ++ni) acc[mi][ni] = mfma_planes<3, PX>(a[mi], b[ni], acc[mi][ni]);
    }
    __syncthreads();
    if (kt + 1 < nk) {
      sstore();
      __syncthreads();
    }
  }
#pragma unroll
  for (int mi = 0; mi < 2; ++mi)
#pragma unroll
    for (int q = 0; q < 16; ++q) {
      const int64_t m = m0 + wr * 64 + mi * 32 + acc_row(q, lane);
      if (m >= Mc) continue;
#pragma unroll
      for (int ni = 0; ni < 2; ++ni) {
        const int64_t n = n0 + wc * 64 + ni * 32 + r32;
        if (n < Nc) out[m * Nc + n] = acc[mi][ni][q];
      }
    }
}

// conv1 for fp32 X on the bf16 MFMA in the six-product form, with X read straight into
// the A fragments.  Each X element feeds exactly one wave (a wave owns 32 rows and all 128
// output columns of its block), so X never passes through LDS: lane (h, r) loads pieces i
// = 0..7 of row r of each 64-wide k-tile, floats 8i + 4h .. + 3 (one instruction moves 32
// contiguous bytes of each of 32 rows; consecutive instructions finish each 128-byte line),
// and splits them three ways in registers; k is permuted consistently on both operands
// (k-step s takes pieces 2s and 2s + 1; W's LDS rows hold the same k in that order), so
// the MFMA's sum is unchanged.  W (the 2.5 MB shared operand, L2-resident) is
// split once per block and k-tile into LDS planes (double buffer, one barrier per k-tile).
// X tiles are prefetched two k-tiles ahead (the tile about to be used is split into its
// bf16 fragments first, which frees its registers for the load two tiles on).  Block: 4
// waves = 128 rows x 128 columns; Nc % 128 == 0, K % 4 == 0, ldx % 4 == 0, 16-byte rows.
constexpr int kX6KT = 64, kX6LD = kX6KT + 8;   // k-tile, LDS row stride (144 B: conflict-free b128)
__global__ __launch_bounds__(256) void k_gemm_xwt_x6(const float* __restrict__ X, int64_t ldx,
                                                     const float* __restrict__ W0, const float* __restrict__ W1,
                                                     int64_t ldw, int64_t split, float* __restrict__ Y, int64_t ldy,
                                                     int64_t M, int64_t K, const int32_t* __restrict__ gate) {
  if (gate_closed(gate)) return;
  __shared__ __attribute__((aligned(16))) __bf16 Ws[2][3][128 * kX6LD];
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6, h = lane >> 5, r32 = lane & 31;
  const int64_t n0 = int64_t(blockIdx.y) * 128;
  const int64_t row = int64_t(blockIdx.x) * 128 + wave * 32 + r32;
  const bool rok = row < M;
  // range-checked buffer loads: the tile offset rides in the VGPR offset with the row (the
  // hardware range check covers voffset + the immediate, not the SGPR offset), so the ring's
  // prefetches past the last k-tile of the last row / W row read zeros; the piece is in the
  // immediate.  The host checks that M * ldx * 4 and the W rows fit 32-bit offsets
  const __amdgpu_buffer_rsrc_t xr = row_rsrc(X, uint32_t(M * ldx * 4));
  const uint32_t xo = rok ? uint32_t((row * ldx + 4 * h) * 4) : 0u;   // (rows past M: row 0, discarded)
  const int wcol = tid & 127, wkh = (tid >> 7) * 32;           // W staging: column, k-half
  const int64_t wn0 = n0 + (wcol & ~63);                        // the wave's 64 columns: one of W0 / W1
  const __amdgpu_buffer_rsrc_t wrs = row_rsrc(wn0 < split ? W0 + wn0 * ldw : W1 + (wn0 - split) * ldw,
                                              uint32_t(64 * ldw * 4));
  const uint32_t wo = uint32_t(((wcol & 63) * ldw + wkh) * 4);
  const int nk = int((K + kX6KT - 1) / kX6KT);

  float4 xa[2][8];    // X tiles in flight (ring of two)
  float4 wr[8];       // the next W tile
  bf16x8 af[4][3];    // the current X tile's fragments: k-step x plane
  f32x16 acc[4] = {};
  auto ld = [](__amdgpu_buffer_rsrc_t r, uint32_t vo, int so) {
    const u32x4 v = __builtin_amdgcn_raw_buffer_load_b128(r, vo, so, 0);
    return make_float4(__uint_as_float(v[0]), __uint_as_float(v[1]), __uint_as_float(v[2]), __uint_as_float(v[3]));
  };
  // (the k tail - the next row's data - is masked where the tile is consumed, so that no
  // instruction touches a load's registers before its phase)
  auto xload = [&](float4 (&d)[8], int kt) {   // piece i: k = 8i + 4h .. + 3 of the tile
#pragma unroll
    for (int i = 0; i < 8; ++i) d[i] = ld(xr, xo + uint32_t(kt * kX6KT * 4) + 32 * i, 0);
  };
  auto wload = [&](int kt) {
#pragma unroll
    for (int i = 0; i < 8; ++i) wr[i] = ld(wrs, wo + uint32_t(kt * kX6KT * 4) + 16 * i, 0);
  };
  // LDS position of tile k inside its 16-group: 8 ((k >> 2) & 1) + 4 (k >> 3) + (k & 3), so
  // that lane h's b128 at 16 s + 8 h holds k = 16 s + 4 h + (0..3) and 16 s + 8 + 4 h + (0..3),
  // the k of its two X pieces 2s and 2s + 1
  auto wstore = [&](int kt) {
    const int buf = kt & 1;
    const int64_t k0 = int64_t(kt) * kX6KT + wkh;
#pragma unroll
    for (int j = 0; j < 4; ++j) {   // 8 positions per 16-byte store: group j >> 1, half j & 1
      bf16x8 p0, p1, p2;
      const int g = j >> 1, hh = j & 1;   // positions 8 hh .. : k = 16 g + 4 hh + (0..3), 16 g + 8 + 4 hh + ..
      const float4 w0 = k0 + 16 * g + 4 * hh < K ? wr[4 * g + hh] : f4zero();
      const float4 w1 = k0 + 16 * g + 8 + 4 * hh < K ? wr[4 * g + 2 + hh] : f4zero();
      const float v[8] = {w0.x, w0.y, w0.z, w0.w, w1.x, w1.y, w1.z, w1.w};
#pragma unroll
      for (int e = 0; e < 8; ++e) {
        __bf16 a, b, c;
        split3_bf16(v[e], a, b, c);
        p0[e] = a; p1[e] = b; p2[e] = c;
      }
      const int o = wcol * kX6LD + wkh + 8 * j;
      *reinterpret_cast<bf16x8*>(&Ws[buf][0][o]) = p0;
      *reinterpret_cast<bf16x8*>(&Ws[buf][1][o]) = p1;
      *reinterpret_cast<bf16x8*>(&Ws[buf][2][o]) = p2;
    }
  };
  auto xsplit = [&](const float4 (&d)[8], int kt) {   // k-step s = pieces 2s, 2s + 1
    const int64_t k0 = int64_t(kt) * kX6KT + 4 * h;
#pragma unroll
    for (int st = 0; st < 4; ++st) {
      const float4 x0 = k0 + 16 * st < K ? d[2 * st] : f4zero();
      const float4 x1 = k0 + 16 * st + 8 < K ? d[2 * st + 1] : f4zero();
      const float v[8] = {x0.x, x0.y, x0.z, x0.w, x1.x, x1.y, x1.z, x1.w};
#pragma unroll
      for (int e = 0; e < 8; ++e) {
        __bf16 a, b, c;
        split3_bf16(v[e], a, b, c);
        af[st][0][e] = a; af[st][1][e] = b; af[st][2][e] = c;
      }
    }
  };
  auto mma = [&](int buf) {
#pragma unroll
    for (int st = 0; st < 4; ++st) {
#pragma unroll
      for (int ni = 0; ni < 4; ++ni) {
        const int o = (32 * ni + r32) * kX6LD + 16 * st + 8 * h;
        const bf16x8 b0 = *reinterpret_cast<const bf16x8*>(&Ws[buf][0][o]);
        const bf16x8 b1 = *reinterpret_cast<const bf16x8*>(&Ws[buf][1][o]);
        const bf16x8 b2 = *reinterpret_cast<const bf16x8*>(&Ws[buf][2][o]);
        acc[ni] = mfma_x6(af[st][0], af[st][1], af[st][2], b0, b1, b2, acc[ni]);
      }
    }
  };
  // one k-tile: split the current X tile, reuse its registers for the tile two on, MFMAs on
  // the W planes of this tile, then stage the next W tile into the other buffer
  // (no conditional loads in the loop: a load under a branch is waited for at the join, which
  // serialised every tile; tiles past K load zeros through the masks, and the tile count is
  // rounded up to even for the two-tile ring)
  // (scheduling barriers keep the phases in this order: the compiler otherwise hoists the W
  // split above the MFMAs and waits for its L2 loads right after issuing them)
  auto step = [&](float4 (&cur)[8], int kt) {
    wload(kt + 1);
    xsplit(cur, kt);
    xload(cur, kt + 2);
    __builtin_amdgcn_sched_barrier(0);
    mma(kt & 1);
    __builtin_amdgcn_sched_barrier(0);
    wstore(kt + 1);
    __syncthreads();
  };
  wload(0);
  wstore(0);
  xload(xa[0], 0);
  xload(xa[1], 1);
  __syncthreads();
  for (int kt = 0; kt < nk; kt += 2) {
    step(xa[0], kt);
    step(xa[1], kt + 1);
  }
#pragma unroll
  for (int ni = 0; ni < 4; ++ni)
#pragma unroll
    for (int q = 0; q < 16; ++q) {
      const int64_t m = int64_t(blockIdx.x) * 128 + wave * 32 + acc_row(q, lane);
      if (m < M) Y[m * ldy + n0 + 32 * ni + r32] = acc[ni][q];
    }
}

// The same conv1 with the split work spread between the MFMAs (one wave per SIMD hides up
// to ~5 single-issue instructions per 32-cycle MFMA gap: MI355X_MICROARCH.md), so the tile
// is MFMA-paced instead of MFMA phase + split phase.  A tile's 16 MFMA groups (k-step st x
// column tile ni, six products each) carry, in order: the split of the tile's own X piece 3
// (groups 0-3, while st = 0 runs), then the next tile's X pieces 0, 1, 2 into the fragment
// slots st = 0, 1, 2 free by then (groups 4-15), and the next tile's W split into the other
// LDS buffer (groups 4-11).  X tiles ride a ring of three register slots (the load of tile
// kt + 3 is issued as soon as tile kt's raw piece 3 is split), the next W tile is loaded at
// group 11 and written one tile later.  One barrier per k-tile.
__global__ __launch_bounds__(256) void k_gemm_xwt_x6p(const float* __restrict__ X, int64_t ldx,
                                                      const float* __restrict__ W0, const float* __restrict__ W1,
                                                      int64_t ldw, int64_t split, float* __restrict__ Y, int64_t ldy,
                                                      int64_t M, int64_t K, const int32_t* __restrict__ gate) {
  if (gate_closed(gate)) return;
  __shared__ __attribute__((aligned(16))) __bf16 Ws[2][3][128 * kX6LD];
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6, h = lane >> 5, r32 = lane & 31;
  const int64_t n0 = int64_t(blockIdx.y) * 128;
  const int64_t row = int64_t(blockIdx.x) * 128 + wave * 32 + r32;
  const bool rok = row < M;
  const __amdgpu_buffer_rsrc_t xr = row_rsrc(X, uint32_t(M * ldx * 4));
  const uint32_t xo = rok ? uint32_t((row * ldx + 4 * h) * 4) : 0u;   // (rows past M: row 0, discarded)
  const int wcol = tid & 127, wkh = (tid >> 7) * 32;
  const int64_t wn0 = n0 + (wcol & ~63);
  const __amdgpu_buffer_rsrc_t wrs = row_rsrc(wn0 < split ? W0 + wn0 * ldw : W1 + (wn0 - split) * ldw,
                                              uint32_t(64 * ldw * 4));
  const uint32_t wo = uint32_t(((wcol & 63) * ldw + wkh) * 4);
  const int nk = int((K + kX6KT - 1) / kX6KT);

  float4 x0[8], x1[8], x2[8];   // X tile ring
  float4 wr[8];                  // the next W tile (raw)
  bf16x8 af[4][3];               // fragments by k-step (rolling: see above)
  f32x16 acc[4] = {};
  auto ld = [](__amdgpu_buffer_rsrc_t r, uint32_t vo, int so) {
    const u32x4 v = __builtin_amdgcn_raw_buffer_load_b128(r, vo, so, 0);
    return make_float4(__uint_as_float(v[0]), __uint_as_float(v[1]), __uint_as_float(v[2]), __uint_as_float(v[3]));
  };
  auto xload = [&](float4 (&d)[8], int kt) {
#pragma unroll
    for (int i = 0; i < 8; ++i) d[i] = ld(xr, xo + uint32_t(kt * kX6KT * 4) + 32 * i, 0);
  };
  auto wload = [&](int kt) {
#pragma unroll
    for (int i = 0; i < 8; ++i) wr[i] = ld(wrs, wo + uint32_t(kt * kX6KT * 4) + 16 * i, 0);
  };
  // two elements (e, e + 1) of X piece st of tile kt into fragment slot st
  auto xpart = [&](const float4 (&d)[8], int kt, int st, int e) {
    const int64_t k = int64_t(kt) * kX6KT + 4 * h + 16 * st + (e < 4 ? 0 : 8);
    const float4 q = k < K ? d[2 * st + (e >> 2)] : f4zero();
    const float v0 = (e & 3) == 0 ? q.x : q.z, v1 = (e & 3) == 0 ? q.y : q.w;
    __bf16 a, b, c;
    split3_bf16(v0, a, b, c);
    af[st][0][e] = a; af[st][1][e] = b; af[st][2][e] = c;
    split3_bf16(v1, a, b, c);
    af[st][0][e + 1] = a; af[st][1][e + 1] = b; af[st][2][e + 1] = c;
  };
  // W chunk j (8 LDS positions of the 16-group permutation) of tile kt into buffer kt & 1
  auto wchunk = [&](int kt, int j) {
    const int buf = kt & 1;
    const int64_t k0 = int64_t(kt) * kX6KT + wkh;
    const int g = j >> 1, hh = j & 1;
    const float4 w0 = k0 + 16 * g + 4 * hh < K ? wr[4 * g + hh] : f4zero();
    const float4 w1 = k0 + 16 * g + 8 + 4 * hh < K ? wr[4 * g + 2 + hh] : f4zero();
    const float v[8] = {w0.x, w0.y, w0.z, w0.w, w1.x, w1.y, w1.z, w1.w};
    bf16x8 p0, p1, p2;
#pragma unroll
    for (int e = 0; e < 8; ++e) {
      __bf16 a, b, c;
      split3_bf16(v[e], a, b, c);
      p0[e] = a; p1[e] = b; p2[e] = c;
    }
    const int o = wcol * kX6LD + wkh + 8 * j;
    *reinterpret_cast<bf16x8*>(&Ws[buf][0][o]) = p0;
    *reinterpret_cast<bf16x8*>(&Ws[buf][1][o]) = p1;
    *reinterpret_cast<bf16x8*>(&Ws[buf][2][o]) = p2;
  };
  auto mg = [&](int buf, int st, int ni) {
    const int o = (32 * ni + r32) * kX6LD + 16 * st + 8 * h;
    const bf16x8 b0 = *reinterpret_cast<const bf16x8*>(&Ws[buf][0][o]);
    const bf16x8 b1 = *reinterpret_cast<const bf16x8*>(&Ws[buf][1][o]);
    const bf16x8 b2 = *reinterpret_cast<const bf16x8*>(&Ws[buf][2][o]);
    acc[ni] = mfma_x6(af[st][0], af[st][1], af[st][2], b0, b1, b2, acc[ni]);
  };
  // tile kt: A = X(kt) (piece 3 still raw), B = X(kt + 1), C = X(kt + 2) (in flight)
  auto tile = [&](int kt, float4 (&A)[8], float4 (&B)[8]) {
    const int buf = kt & 1;
#pragma unroll
    for (int ni = 0; ni < 4; ++ni) {
      mg(buf, 0, ni);
      xpart(A, kt, 3, 2 * ni);
    }
    xload(A, kt + 3);
#pragma unroll
    for (int ni = 0; ni < 4; ++ni) {
      mg(buf, 1, ni);
      xpart(B, kt + 1, 0, 2 * ni);
      if (ni & 1) wchunk(kt + 1, ni >> 1);
    }
#pragma unroll
    for (int ni = 0; ni < 4; ++ni) {
      mg(buf, 2, ni);
      xpart(B, kt + 1, 1, 2 * ni);
      if (ni & 1) wchunk(kt + 1, 2 + (ni >> 1));
    }
    wload(kt + 2);
#pragma unroll
    for (int ni = 0; ni < 4; ++ni) {
      mg(buf, 3, ni);
      xpart(B, kt + 1, 2, 2 * ni);
    }
    __syncthreads();
  };
  wload(0);
#pragma unroll
  for (int j = 0; j < 4; ++j) wchunk(0, j);
  xload(x0, 0);
  xload(x1, 1);
  xload(x2, 2);
  wload(1);
#pragma unroll
  for (int st = 0; st < 3; ++st)
#pragma unroll
    for (int e = 0; e < 8; e += 2) xpart(x0, 0, st, e);
  __syncthreads();
  for (int kt = 0; kt < nk; kt += 3) {
    tile(kt, x0, x1);
    tile(kt + 1, x1, x2);
    tile(kt + 2, x2, x0);
  }
#pragma unroll
  for (int ni = 0; ni < 4; ++ni)
#pragma unroll
    for (int q = 0; q < 16; ++q) {
      const int64_t m = int64_t(blockIdx.x) * 128 + wave * 32 + acc_row(q, lane);
      if (m < M) Y[m * ldy + n0 + 32 * ni + r32] = acc[ni][q];
    }
}

// C[m][n] = sum_s part[s][m][n] (fixed order), rows [0, split) -> C0, the rest -> C1.
__global__ __launch_bounds__(256) void k_reduce_splits(const float* __restrict__ part, int S,
                                                       int64_t Mc, int64_t Nc, float* __restrict__ C0,
                                                       float* __restrict__ C1, int64_t ldc,
                                                       int64_t split, const int32_t* __restrict__ gate) {
  if (gate_closed(gate)) return;
  const int64_t total = Mc * Nc;
  for (int64_t idx = int64_t(blockIdx.x) * blockDim.x + threadIdx.x; idx < total;
       idx += int64_t(gridDim.x) * blockDim.x) {
    float acc = part[idx];
    for (int s = 1; s < S; ++s) acc += part[int64_t(s) * total + idx];
    const int64_t m = idx / Nc, n = idx % Nc;
    if (m < split) C0[m * ldc + n] = acc;
    else C1[(m - split) * ldc + n] = acc;
  }
}

// ---------------------------------------------------------------- host side
int tn_splits(int64_t Mc, int64_t Nc, int64_t K) {
  // aim for ~5 blocks per CU over 256 CUs, never less than 32 nodes per split
  int64_t tiles = ((Nc + 63) / 64) * ((Mc + 127) / 128);
  int64_t want = (5 * 256 + tiles - 1) / tiles;
  int64_t maxs = (K + BK - 1) / BK;
  int64_t s = want < maxs ? want : maxs;
  return int(s < 1 ? 1 : (s > 64 ? 64 : s));
}

// k_gemm_tn_w (128 x 128 tiles): node splits for about BGCN_TN_WIDE_BLOCKS blocks (A/B
// knob, read once; default 1024)
int tn_splits_w(int64_t Mc, int64_t Nc, int64_t K) {
  static const int64_t target = [] { const char* e = std::getenv("BGCN_TN_WIDE_BLOCKS"); return e ? std::max<int64_t>(1, atol(e)) : int64_t(1024); }();
  const int64_t tiles = ((Nc + 127) / 128) * ((Mc + 127) / 128);
  const int64_t want = std::max<int64_t>(1, target / tiles);
  const int64_t maxs = (K + BK - 1) / BK;
  const int64_t s = want < maxs ? want : maxs;
  return int(s < 1 ? 1 : (s > 64 ? 64 : s));
}

size_t tn_ws_size(int64_t Mc, int64_t Nc, int64_t K) {
  const int S = std::max(tn_splits(Mc, Nc, K), tn_splits_w(Mc, Nc, K));
  return size_t(S) * size_t(Mc) * size_t(Nc) * sizeof(float) + 256;
}

static bool aligned16(const void* p) { return (reinterpret_cast<uintptr_t>(p) & 15) == 0; }

// whether X of this type takes the bf16 MFMA kernels: bf16 X (BGCN_GEMM_BF16=0 keeps the
// f32 MFMA) and fp32 X in the six-product form (BGCN_GEMM_X6=0 keeps the f32 MFMA); both
// read once
template <class TX>
static bool bf16_mfma_for() {
  static const bool on = [] {
    const char* e = std::getenv(sizeof(TX) == 2 ? "BGCN_GEMM_BF16" : "BGCN_GEMM_X6");
    return !(e && atoi(e) == 0);
  }();
  return on;
}

template <class TX>
static int gemm_xwt_t(const TX* X, int64_t ldx, const float* W0, const float* W1, int64_t ldw,
                      int64_t split, float* Y, int64_t ldy, int64_t M, int64_t Nc, int64_t K,
                      hipStream_t stream, const int32_t* gate) {
  BGCN_CHECK_ARG(X && W0 && Y, "null pointer");
  BGCN_CHECK_ARG(M >= 0 && Nc > 0 && K > 0, "bad shape");
  BGCN_CHECK_ARG(ldx >= K && ldw >= K && ldy >= Nc, "bad leading dimension");
  BGCN_CHECK_ARG(split >= Nc || W1, "W1 required when split < Nc");
  if (M == 0) return BGCN_OK;
  // the vector path loads 4 features at once (16 B fp32, 8 B bf16)
  const bool xal = (reinterpret_cast<uintptr_t>(X) & (4 * sizeof(TX) - 1)) == 0;
  bool vec = K % 4 == 0 && ldx % 4 == 0 && ldw % 4 == 0 && xal && aligned16(W0) &&
             (!W1 || aligned16(W1));
  // fp32 X: the six-product kernel with X straight into the A fragments
  if (sizeof(TX) == 4 && bf16_mfma_for<TX>() && M >= kX6MinRows && vec && Nc % 128 == 0 && split % 64 == 0 &&
      (reinterpret_cast<uintptr_t>(X) & 15) == 0 && M * ldx * 4 < (int64_t(1) << 32) - 16 &&
      64 * ldw * 4 < (int64_t(1) << 32)) {
    static const int pipe = [] { const char* e = std::getenv("BGCN_X6_PIPE"); return e ? atoi(e) : 1; }();
    if (pipe)
      hipLaunchKernelGGL(k_gemm_xwt_x6p, dim3(grid_for(M, 128), unsigned(Nc / 128)), dim3(256), 0, stream,
                         reinterpret_cast<const float*>(X), ldx, W0, W1, ldw, split, Y, ldy, M, K, gate);
    else
      hipLaunchKernelGGL(k_gemm_xwt_x6, dim3(grid_for(M, 128), unsigned(Nc / 128)), dim3(256), 0, stream,
                         reinterpret_cast<const float*>(X), ldx, W0, W1, ldw, split, Y, ldy, M, K, gate);
    BGCN_CHECK_LAUNCH();
    return BGCN_OK;
  }
  // bf16 X: the bf16 MFMA with W split three ways (fp32 X below kX6MinRows keeps the f32
  // MFMA: the XPlanes form of this kernel measured 466 us against its 377 at full size)
  if (sizeof(TX) == 2 && bf16_mfma_for<TX>() && vec && K % 8 == 0 && ldx % 8 == 0 &&
      (reinterpret_cast<uintptr_t>(X) & 15) == 0) {
    hipLaunchKernelGGL(k_gemm_xwt_bf16<TX>, dim3(grid_for(M, 128), grid_for(Nc, 128)), dim3(256), 0, stream,
                       X, ldx, W0, W1, ldw, split, Y, ldy, M, Nc, K, gate);
    BGCN_CHECK_LAUNCH();
    return BGCN_OK;
  }
  dim3 grid(grid_for(M, 64), grid_for(Nc, 128));
  if (vec)
    hipLaunchKernelGGL((k_gemm_xwt<true, false, TX>), grid, dim3(256), 0, stream, X, ldx, W0, W1,
                       ldw, split, Y, ldy, M, Nc, K, gate);
  else
    hipLaunchKernelGGL((k_gemm_xwt<false, false, TX>), grid, dim3(256), 0, stream, X, ldx, W0, W1,
                       ldw, split, Y, ldy, M, Nc, K, gate);
  BGCN_CHECK_LAUNCH();
  return BGCN_OK;
}

int gemm_xwt_impl(const float* X, int64_t ldx, const float* W0, const float* W1, int64_t ldw,
                  int64_t split, float* Y, int64_t ldy, int64_t M, int64_t Nc, int64_t K,
                  hipStream_t stream, const int32_t* gate) {
  return gemm_xwt_t(X, ldx, W0, W1, ldw, split, Y, ldy, M, Nc, K, stream, gate);
}

int gemm_xwt_x(const void* X, int xdt, int64_t ldx, const float* W0, const float* W1, int64_t ldw,
               int64_t split, float* Y, int64_t ldy, int64_t M, int64_t Nc, int64_t K,
               hipStream_t stream, const int32_t* gate) {
  if (xdt == BGCN_DTYPE_BF16)
    return gemm_xwt_t(static_cast<const bf16_t*>(X), ldx, W0, W1, ldw, split, Y, ldy, M, Nc, K,
                      stream, gate);
  return gemm_xwt_t(static_cast<const float*>(X), ldx, W0, W1, ldw, split, Y, ldy, M, Nc, K,
                    stream, gate);
}

int gemm_xw_impl(const float* X, int64_t ldx, const float* W, int64_t ldw, float* Y, int64_t ldy,
                 int64_t M, int64_t Nc, int64_t K, hipStream_t stream) {
  BGCN_CHECK_ARG(X && W && Y, "null pointer");
  BGCN_CHECK_ARG(M >= 0 && Nc > 0 && K > 0, "bad shape");
  BGCN_CHECK_ARG(ldx >= K && ldw >= Nc && ldy >= Nc, "bad leading dimension");
  if (M == 0) return BGCN_OK;
  bool vec = K % 4 == 0 && Nc % 4 == 0 && ldx % 4 == 0 && ldw % 4 == 0 && aligned16(X) &&
             aligned16(W);
  dim3 grid(grid_for(M, 64), grid_for(Nc, 128));
  if (vec)
    hipLaunchKernelGGL((k_gemm_xwt<true, true>), grid, dim3(256), 0, stream, X, ldx, W,
                       (const float*)nullptr, ldw, Nc, Y, ldy, M, Nc, K, (const int32_t*)nullptr);
  else
    hipLaunchKernelGGL((k_gemm_xwt<false, true>), grid, dim3(256), 0, stream, X, ldx, W,
                       (const float*)nullptr, ldw, Nc, Y, ldy, M, Nc, K, (const int32_t*)nullptr);
  BGCN_CHECK_LAUNCH();
  return BGCN_OK;
}

// ---------------------------------------------------------------- column sums
// out[c] = sum_r A[r][c]: bias gradients of the generic GCNConv backward
// (deterministic two-stage reduction).
constexpr int kColRows = 256;

__global__ __launch_bounds__(256) void k_colsum_part(const float* __restrict__ A, int64_t lda,
                                                     int64_t rows, int C,
                                                     float* __restrict__ part) {
  const int c = blockIdx.y * 256 + threadIdx.x;
  if (c >= C) return;
  const int64_t r0 = int64_t(blockIdx.x) * kColRows, r1 = min<int64_t>(r0 + kColRows, rows);
  float acc = 0.f;
  for (int64_t r = r0; r < r1; ++r) acc += A[r * lda + c];
  part[int64_t(blockIdx.x) * C + c] = acc;
}

__global__ void k_colsum_final(const float* __restrict__ part, int P, int C, float* __restrict__ out) {
  const int c = blockIdx.x * blockDim.x + threadIdx.x;
  if (c >= C) return;
  float acc = 0.f;
  for (int p = 0; p < P; ++p) acc += part[int64_t(p) * C + c];
  out[c] = acc;
}

size_t colsum_ws_size(int64_t rows, int32_t C) {
  int64_t P = (rows + kColRows - 1) / kColRows;
  return size_t(P > 0 ? P : 1) * size_t(C) * sizeof(float) + 256;
}

int colsum_impl(const float* A, int64_t lda, int64_t rows, int32_t C, float* out, void* ws,
                size_t ws_bytes, hipStream_t stream) {
  BGCN_CHECK_ARG(out && C > 0 && rows >= 0 && lda >= C && (rows == 0 || A), "bad arguments");
  BGCN_CHECK_ARG(ws && ws_bytes >= colsum_ws_size(rows, C), "workspace too small");
  float* part = static_cast<float*>(ws);
  int P = int((rows + kColRows - 1) / kColRows);
  if (P == 0) {
    BGCN_CHECK_HIP(hipMemsetAsync(out, 0, size_t(C) * sizeof(float), stream));
    return BGCN_OK;
  }
  hipLaunchKernelGGL(k_colsum_part, dim3(unsigned(P), unsigned((C + 255) / 256)), dim3(256), 0,
                     stream, A, lda, rows, C, part);
  BGCN_CHECK_LAUNCH();
  hipLaunchKernelGGL(k_colsum_final, dim3(grid_for(C, 256)), dim3(256), 0, stream, part, P, C,
                     out);
  BGCN_CHECK_LAUNCH();
  return BGCN_OK;
}

template <class TX>
static int gemm_tn_t(const float* G, int64_t ldg, const TX* X, int64_t ldx, float* C0, float* C1,
                     int64_t ldc, int64_t split, int64_t Mc, int64_t Nc, int64_t K, void* ws,
                     size_t ws_bytes, hipStream_t stream, int timing_cls, const int32_t* gate) {
  BGCN_CHECK_ARG(G && X && C0, "null pointer");
  BGCN_CHECK_ARG(Mc > 0 && Nc > 0 && K >= 0, "bad shape");
  BGCN_CHECK_ARG(ldg >= Mc && ldx >= Nc && ldc >= Nc, "bad leading dimension");
  BGCN_CHECK_ARG(split >= Mc || C1, "C1 required when split < Mc");
  BGCN_CHECK_ARG(ws && ws_bytes >= tn_ws_size(Mc, Nc, K), "workspace too small");
  const bool xal = (reinterpret_cast<uintptr_t>(X) & (4 * sizeof(TX) - 1)) == 0;
  bool vec = Mc % 4 == 0 && Nc % 4 == 0 && ldg % 4 == 0 && ldx % 4 == 0 && aligned16(G) && xal;
  // fp32 X: the 64 x 64 wave-tile kernel (BGCN_TN_WIDE=0 keeps k_gemm_tn)
  static const bool wide_on = [] { const char* e = std::getenv("BGCN_TN_WIDE"); return !(e && atoi(e) == 0); }();
  const bool wide = sizeof(TX) == 4 && vec && wide_on;
  int S = wide ? tn_splits_w(Mc, Nc, K) : tn_splits(Mc, Nc, K);
  int64_t kchunk = (K + S - 1) / S;
  kchunk = (kchunk + BK - 1) / BK * BK;
  if (kchunk == 0) kchunk = BK;
  S = int((K + kchunk - 1) / kchunk);
  if (S < 1) S = 1;
  float* part = static_cast<float*>(ws);
  timing_begin(timing_cls, stream);
  bool done = false;
  if constexpr (sizeof(TX) == 4) {
    if (wide) {
      hipLaunchKernelGGL(k_gemm_tn_w, dim3(grid_for(Nc, 128), grid_for(Mc, 128), S), dim3(256), 0, stream, G, ldg,
                         reinterpret_cast<const float*>(X), ldx, part, Mc, Nc, K, kchunk, gate);
      done = true;
    }
  }
  // bf16 X: the bf16 MFMA with G split three ways.  fp32 X keeps the f32 MFMA: the
  // six-product forms measured 385 us (k_gemm_tn_bf16<float>), 489 us (X read straight into
  // the B fragments) and 479 us (that kernel with its splits between the MFMAs) against
  // its 374-377 us at the bench workload
  if (sizeof(TX) == 2 && bf16_mfma_for<TX>() && vec && Nc % 8 == 0 && ldx % 8 == 0 && (reinterpret_cast<uintptr_t>(X) & 15) == 0) {
    hipLaunchKernelGGL(k_gemm_tn_bf16<TX>, dim3(grid_for(Nc, 128), grid_for(Mc, 128), S), dim3(256), 0, stream, G,
                       ldg, X, ldx, part, Mc, Nc, K, kchunk, gate);
    done = true;
  }
  dim3 grid(grid_for(Nc, 64), grid_for(Mc, 128), S);
  if (done) {
  } else if (vec)
    hipLaunchKernelGGL((k_gemm_tn<true, TX>), grid, dim3(256), 0, stream, G, ldg, X, ldx, part, Mc,
                       Nc, K, kchunk, gate);
  else
    hipLaunchKernelGGL((k_gemm_tn<false, TX>), grid, dim3(256), 0, stream, G, ldg, X, ldx, part, Mc,
                       Nc, K, kchunk, gate);
  BGCN_CHECK_LAUNCH();
  timing_end(timing_cls, stream);
  hipLaunchKernelGGL(k_reduce_splits, dim3(std::min<unsigned>(grid_for(Mc * Nc, 256), 1024)), dim3(256), 0, stream, part, S,
                     Mc, Nc, C0, C1, ldc, split, gate);
  BGCN_CHECK_LAUNCH();
  return BGCN_OK;
}

int gemm_tn_impl(const float* G, int64_t ldg, const float* X, int64_t ldx, float* C0, float* C1,
                 int64_t ldc, int64_t split, int64_t Mc, int64_t Nc, int64_t K, void* ws,
                 size_t ws_bytes, hipStream_t stream, int timing_cls, const int32_t* gate) {
  return gemm_tn_t(G, ldg, X, ldx, C0, C1, ldc, split, Mc, Nc, K, ws, ws_bytes, stream, timing_cls,
                   gate);
}

int gemm_tn_x(const float* G, int64_t ldg, const void* X, int xdt, int64_t ldx, float* C0,
              float* C1, int64_t ldc, int64_t split, int64_t Mc, int64_t Nc, int64_t K, void* ws,
              size_t ws_bytes, hipStream_t stream, int timing_cls, const int32_t* gate) {
  if (xdt == BGCN_DTYPE_BF16)
    return gemm_tn_t(G, ldg, static_cast<const bf16_t*>(X), ldx, C0, C1, ldc, split, Mc, Nc, K, ws,
                     ws_bytes, stream, timing_cls, gate);
  return gemm_tn_t(G, ldg, static_cast<const float*>(X), ldx, C0, C1, ldc, split, Mc, Nc, K, ws,
                   ws_bytes, stream, timing_cls, gate);
}

}  // namespace bgcn

extern "C" int bgcn_gemm_xwt(const float* X, int64_t ldx, const float* W0, const float* W1,
                             int64_t ldw, int64_t split, float* Y, int64_t ldy, int64_t M,
                             int64_t Nc, int64_t K, bgcn_stream_t stream) {
  return bgcn::gemm_xwt_impl(X, ldx, W0, W1, ldw, split, Y, ldy, M, Nc, K,
                             reinterpret_cast<hipStream_t>(stream), nullptr);
}

extern "C" int bgcn_gemm_xw(const float* X, int64_t ldx, const float* W, int64_t ldw, float* Y,
                            int64_t ldy, int64_t M, int64_t Nc, int64_t K, bgcn_stream_t stream) {
  return bgcn::gemm_xw_impl(X, ldx, W, ldw, Y, ldy, M, Nc, K,
                            reinterpret_cast<hipStream_t>(stream));
}

extern "C" size_t bgcn_colsum_workspace_size(int64_t rows, int32_t C) {
  return bgcn::colsum_ws_size(rows, C);
}

extern "C" int bgcn_colsum(const float* A, int64_t lda, int64_t rows, int32_t C, float* out,
                           void* workspace, size_t workspace_bytes, bgcn_stream_t stream) {
  return bgcn::colsum_impl(A, lda, rows, C, out, workspace, workspace_bytes,
                           reinterpret_cast<hipStream_t>(stream));
}

extern "C" size_t bgcn_gemm_tn_workspace_size(int64_t Mc, int64_t Nc, int64_t K) {
  return bgcn::tn_ws_size(Mc, Nc, K);
}

extern "C" int bgcn_gemm_tn(const float* G, int64_t ldg, const float* X, int64_t ldx, float* C0,
                            float* C1, int64_t ldc, int64_t split, int64_t Mc, int64_t Nc,
                            int64_t K, void* workspace, size_t workspace_bytes,
                            bgcn_stream_t stream) {
  return bgcn::gemm_tn_impl(G, ldg, X, ldx, C0, C1, ldc, split, Mc, Nc, K, workspace,
                            workspace_bytes, reinterpret_cast<hipStream_t>(stream), -1, nullptr);
}
