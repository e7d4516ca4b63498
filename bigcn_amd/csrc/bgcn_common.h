// Shared device helpers and host-side error plumbing for libbgcn (gfx950 only).
#pragma once

#include <hip/hip_runtime.h>
#include <stdint.h>

#include <algorithm>
#include <string>

#include "../../include/bgcn.h"

namespace bgcn {

// ---------------------------------------------------------------- host errors
void set_error(const std::string& msg);
int fail(int code, const std::string& msg);

#define BGCN_CHECK_ARG(cond, msg)                   \
  do {                                              \
    if (!(cond)) return ::bgcn::fail(BGCN_EINVAL, msg); \
  } while (0)

#define BGCN_CHECK_HIP(expr)                                                           \
  do {                                                                                 \
    hipError_t _e = (expr);                                                            \
    if (_e != hipSuccess)                                                              \
      return ::bgcn::fail(BGCN_EHIP, std::string(#expr ": ") + hipGetErrorString(_e)); \
  } while (0)

#define BGCN_CHECK_LAUNCH() BGCN_CHECK_HIP(hipGetLastError())

inline int propagate(int rc) { return rc; }
#define BGCN_TRY(expr)           \
  do {                           \
    int _rc = (expr);            \
    if (_rc != BGCN_OK) return _rc; \
  } while (0)

inline size_t align_up(size_t x, size_t a) { return (x + a - 1) / a * a; }

// Simple bump allocator over a caller-provided workspace.
// Blocks are dispatched to the 8 XCDs round-robin (block b of a 1-D grid runs on XCD b % 8).
// xcd_contig(b, R) renumbers blocks [0, R) so that each XCD takes a contiguous range of
// logical blocks (XCD x: [x q + min(x, r), ...), q = R / 8, r = R % 8): work items that
// share data (adjacent rows of one tree) then share one XCD's L2.  A 2-D grid keeps the
// mapping for every row when gridDim.x is a multiple of 8.
__host__ __device__ inline int xcd_contig(int b, int R) {
  const int q = R / 8, r = R % 8, x = b % 8, i = b / 8;
  return x * q + (x < r ? x : r) + i;
}

struct Carve {
  char* base;
  size_t cap;
  size_t off = 0;
  Carve(void* b, size_t c) : base(static_cast<char*>(b)), cap(c) {}
  template <class T>
  T* take(size_t count) {
    off = align_up(off, 256);
    T* p = reinterpret_cast<T*>(base ? base + off : nullptr);
    off += count * sizeof(T);
    return p;
  }
  bool ok() const { return off <= cap; }
};

// Auxiliary streams ("lanes") of the current device for independent branches of the
// fused step: aux_fork sets *branch to lane's stream after making it wait for the work
// queued on `main` so far; aux_join makes `main` wait for everything queued on the lane.
// On the legacy null stream (whose cross-stream waits synchronise the host) *branch =
// main and the branch runs inline.  The side lane carries every branch of the step; the
// graph lane (created on first use) only the next batch's DropEdge + K1 beside its pass over
// X (prep_pipeline).  HIP maps streams onto a few hardware queues (GPU_MAX_HW_QUEUES = 4):
// the graph lane's work ends inside the pass over X, long before any collective of the step
// is queued.
constexpr int kAuxLanes = 2;
constexpr int kLaneSide = 0;
constexpr int kLaneGraph = 1;   // the next batch's DropEdge + K1 beside its pass over X
int aux_fork(hipStream_t main, int lane, hipStream_t* branch);
int aux_join(hipStream_t main, int lane);
// the next-batch preparation of bgcn_train_step is not joined by its own call: its end is
// recorded (aux_prep_done) and the caller's stream waits for it at the start of the next
// call (aux_prep_wait) - no join at the end of a step
int aux_prep_done(hipStream_t main);
int aux_prep_wait(hipStream_t main);

// kernel timing hook (bench.py): record HIP events around a launch of a class
void timing_begin(int cls, hipStream_t s);
void timing_end(int cls, hipStream_t s);
// the span record of the next launch of a stamped class (nullptr: not timed): blocks
// b < kSpanStarts store their start time at [b], every block atomicMax's its end time into
// [kSpanStarts + b % kSpanEnds] (distinct addresses: no contention) - span_stamp_*
constexpr int kSpanStarts = 64, kSpanEnds = 8192, kSpanRecord = kSpanStarts + kSpanEnds;
uint64_t* span_slot(int cls);

constexpr int kWave = 64;
// status word bits: 1 bad edge index, 2 bad label, 4 over-full feature row (sparse
// mode), 8 an internal hand-off timed out (kStatusInternal; results invalid)
constexpr int32_t kStatusInternal = 8;

// ---------------------------------------------------------------- device
// Dropout keep word for (seed, direction, node, word): 32 keep bits covering
// columns [32*word, 32*word+32) of the [H + F] concat (F.dropout p = 0.5: every bit a fair
// coin).  Two rounds of a 32-bit mixer (lowbias32, Wellons: a bijection with full
// avalanche): a per-node base mix32(node ^ seed_lo), then per (word, direction) mix32(base ^
// ((2 word + dir) * golden + seed_hi)).  The base is shared by every word of a node, so a
// kernel that needs many words of one node (conv2's root slots: up to 17 per lane and
// tile) hoists it (KeepSrc::base / get_b): 32-bit multiplies only, against three 64-bit
// ones per word of the splitmix64 form this replaced (which dominated conv2's VALU time).
// The restatement (oracle/bigcn_oracle.py keep_word) is bit-exact (test_gpu_dropedge).
__device__ __forceinline__ uint32_t mix32(uint32_t x) {
  x ^= x >> 16;
  x *= 0x7feb352du;
  x ^= x >> 15;
  x *= 0x846ca68bu;
  x ^= x >> 16;
  return x;
}
__device__ __forceinline__ uint32_t keep_node_base(uint64_t seed, uint32_t node) {
  return mix32(node ^ uint32_t(seed));
}
__device__ __forceinline__ uint32_t keep_word_at(uint64_t seed, uint32_t base, uint32_t dir, uint32_t word) {
  return mix32(base ^ (((word << 1) | (dir & 1u)) * 0x9E3779B9u + uint32_t(seed >> 32)));
}
__device__ __forceinline__ uint32_t keep_word(uint64_t seed, uint32_t dir, uint32_t node,
                                              uint32_t word) {
  return keep_word_at(seed, keep_node_base(seed, node), dir, word);
}

// Keep word source used by the fused kernels.
struct KeepSrc {
  const uint32_t* words;  // injected [2][N][nw] or nullptr => generated
  uint64_t seed;
  int64_t num_nodes;
  int32_t nw;
  int32_t training;  // 0 => all kept, scale 1
  __device__ __forceinline__ uint32_t get(uint32_t dir, uint32_t node, uint32_t w) const {
    if (!training) return 0xffffffffu;
    if (words) return words[(size_t(dir) * size_t(num_nodes) + node) * size_t(nw) + w];
    return keep_word(seed, dir, node, w);
  }
  // the node's hash base (generated words only): get_b(dir, node, base(node), w) == get(dir, node, w)
  __device__ __forceinline__ uint32_t base(uint32_t node) const { return keep_node_base(seed, node); }
  __device__ __forceinline__ uint32_t get_b(uint32_t dir, uint32_t node, uint32_t b, uint32_t w) const {
    if (!training) return 0xffffffffu;
    if (words) return words[(size_t(dir) * size_t(num_nodes) + node) * size_t(nw) + w];
    return keep_word_at(seed, b, dir, w);
  }
  __host__ __device__ __forceinline__ float scale() const { return training ? 2.0f : 1.0f; }
};

typedef float f32x4 __attribute__((ext_vector_type(4)));
typedef float f32x16 __attribute__((ext_vector_type(16)));

__device__ __forceinline__ f32x16 mfma32x32x2(float a, float b, f32x16 c) {
  return __builtin_amdgcn_mfma_f32_32x32x2f32(a, b, c, 0, 0, 0);
}

// fp32 products on the bf16 MFMA.  The f32-input MFMA issues at the FP32 vector rate, 1/16
// of the bf16 one; x = hi + lo with hi = bf16(x), lo = bf16(x - hi) keeps 16 of x's 24
// mantissa bits, and a.b ~ ah.bh + ah.bl + al.bh (al.bl and the two residuals dropped,
// each <= 2^-18 |a b|): ~1e-5 relative per product, accumulated in fp32.  Used where the
// result feeds only linear steps (the backward's dH1 / dW2 products): a forward product
// that feeds a relu flips its sign for entries near zero (measured on conv2: not used).
// Lane map of 32x32x16: lane (h = l >> 5, r = l & 31) holds A[r][8h + j] and B[8h + j][r].
typedef __bf16 bf16x8 __attribute__((ext_vector_type(8)));
__device__ __forceinline__ f32x16 mfma_bf16(bf16x8 a, bf16x8 b, f32x16 c) {
  return __builtin_amdgcn_mfma_f32_32x32x16_bf16(a, b, c, 0, 0, 0);
}
__device__ __forceinline__ void split_bf16(float x, __bf16& hi, __bf16& lo) {
  hi = __bf16(x);
  lo = __bf16(x - float(hi));
}
// fp32-grade form (for products that feed a relu, where 1e-5 relative flips signs of
// entries near zero): x = hi + mid + lo keeps all 24 bits, and a.b takes the six products
// down to 2^-16 |a b| (al.bh, am.bm, ah.bl, am.bh, ah.bm, ah.bh, small terms first) - the
// dropped ones are below 2^-24 |a b|, fp32's own rounding.
__device__ __forceinline__ void split3_bf16(float x, __bf16& hi, __bf16& mid, __bf16& lo) {
  hi = __bf16(x);
  const float r = x - float(hi);
  mid = __bf16(r);
  lo = __bf16(r - float(mid));
}
__device__ __forceinline__ f32x16 mfma_x6(bf16x8 ah, bf16x8 am, bf16x8 al, bf16x8 bh, bf16x8 bm,
                                          bf16x8 bl, f32x16 c) {
  c = mfma_bf16(al, bh, c);
  c = mfma_bf16(am, bm, c);
  c = mfma_bf16(ah, bl, c);
  c = mfma_bf16(am, bh, c);
  c = mfma_bf16(ah, bm, c);
  return mfma_bf16(ah, bh, c);
}
// acc += a.b for split operands (three bf16 products, small terms first)
__device__ __forceinline__ f32x16 mfma_x3(bf16x8 ah, bf16x8 al, bf16x8 bh, bf16x8 bl, f32x16 c) {
  c = mfma_bf16(al, bh, c);
  c = mfma_bf16(ah, bl, c);
  return mfma_bf16(ah, bh, c);
}

__device__ __forceinline__ float4 ld4(const float* p) { return *reinterpret_cast<const float4*>(p); }
__device__ __forceinline__ void st4(float* p, float4 v) { *reinterpret_cast<float4*>(p) = v; }
// streaming (non-temporal) 16-byte load: data read once, kept out of the caches' LRU
__device__ __forceinline__ float4 ld4_nt(const float* p) {
  const f32x4 v = __builtin_nontemporal_load(reinterpret_cast<const f32x4*>(p));
  return make_float4(v.x, v.y, v.z, v.w);
}
// streaming (non-temporal) 16-byte store: output never re-read by the writer's kernel
__device__ __forceinline__ void st4_nt(float* p, float4 v) {
  f32x4 t;
  t.x = v.x; t.y = v.y; t.z = v.z; t.w = v.w;
  __builtin_nontemporal_store(t, reinterpret_cast<f32x4*>(p));
}
__device__ __forceinline__ float4 f4zero() { return make_float4(0.f, 0.f, 0.f, 0.f); }
__device__ __forceinline__ float4 f4fma(float a, float4 x, float4 acc) {
  acc.x = fmaf(a, x.x, acc.x);
  acc.y = fmaf(a, x.y, acc.y);
  acc.z = fmaf(a, x.z, acc.z);
  acc.w = fmaf(a, x.w, acc.w);
  return acc;
}
__device__ __forceinline__ float4 f4add(float4 a, float4 b) {
  return make_float4(a.x + b.x, a.y + b.y, a.z + b.z, a.w + b.w);
}
__device__ __forceinline__ float4 f4mul(float4 a, float4 b) {
  return make_float4(a.x * b.x, a.y * b.y, a.z * b.z, a.w * b.w);
}
__device__ __forceinline__ float4 f4relu(float4 a) {
  return make_float4(fmaxf(a.x, 0.f), fmaxf(a.y, 0.f), fmaxf(a.z, 0.f), fmaxf(a.w, 0.f));
}

inline unsigned grid_for(int64_t n, int block) { return unsigned((n + block - 1) / block); }

// Dense-path gate: the fused encoder runs the dense MFMA kernels only when the sparse
// feature path is off (gate == nullptr: always run) or has flagged an overflow row
// (*gate != 0).  Decided on the device, so no host sync.
// ---------------------------------------------------------------- node-feature loads
// X is fp32 or raw bfloat16 (uint16_t storage; bag-of-words counts are exact in bf16).
// xq: 4 consecutive features (ldx and the column are multiples of 4), xs: one feature;
// _nt: streaming.  Kernels reading X are templated on the element type.
typedef uint16_t bf16_t;
typedef unsigned int u32x2 __attribute__((ext_vector_type(2)));
__device__ __forceinline__ float bf2f(uint32_t bits16) { return __uint_as_float(bits16 << 16); }
__device__ __forceinline__ float4 bf4(uint32_t lo, uint32_t hi) {
  return make_float4(__uint_as_float(lo << 16), __uint_as_float(lo & 0xffff0000u),
                     __uint_as_float(hi << 16), __uint_as_float(hi & 0xffff0000u));
}
__device__ __forceinline__ float4 xq(const float* p) { return ld4(p); }
__device__ __forceinline__ float4 xq(const bf16_t* p) {
  const uint2 u = *reinterpret_cast<const uint2*>(p);
  return bf4(u.x, u.y);
}
__device__ __forceinline__ float4 xq_nt(const float* p) { return ld4_nt(p); }
__device__ __forceinline__ float4 xq_nt(const bf16_t* p) {
  const u32x2 u = __builtin_nontemporal_load(reinterpret_cast<const u32x2*>(p));
  return bf4(u.x, u.y);
}
// raw streaming loads of 4 features, converted later: a conversion right after its load
// would make the compiler wait for each load in turn instead of keeping all in flight
// Row loads go through a buffer descriptor of the row (wave-uniform base, 32-bit lane
// offsets + immediates, hardware range check: bytes past the row read as 0 - no clamped
// addresses held in registers), non-temporal.
typedef unsigned int u32x4 __attribute__((ext_vector_type(4)));
__device__ __forceinline__ __amdgpu_buffer_rsrc_t row_rsrc(const void* row, uint32_t bytes) {
  const uint64_t pa = reinterpret_cast<uint64_t>(row);
  const uint32_t lo = __builtin_amdgcn_readfirstlane(uint32_t(pa));
  const uint32_t hi = __builtin_amdgcn_readfirstlane(uint32_t(pa >> 32));
  void* base = reinterpret_cast<void*>(uint64_t(lo) | (uint64_t(hi) << 32));
  return __builtin_amdgcn_make_buffer_rsrc(base, 0, __builtin_amdgcn_readfirstlane(bytes), 0x00020000);
}
__device__ __forceinline__ void st4_chain(float* base, int64_t off, float4 v) {
#if BGCN_WT_OUT
  u32x4 d;
  d.x = __float_as_uint(v.x); d.y = __float_as_uint(v.y); d.z = __float_as_uint(v.z); d.w = __float_as_uint(v.w);
  __builtin_amdgcn_raw_buffer_store_b128(d, row_rsrc(base, 0xfffffff0u), uint32_t(off * 4), 0, 16);   // sc1
#else
  st4(base + off, v);
#endif
}
// The chain's [N, 128] activations (Z1, H1, dZ2, dZ1, ...) are read by the NEXT launch only:
// stored write-through (sc1), the producer's kernel boundary has no dirty lines left to write
// back (MI355X_MICROARCH.md price table, "boundary": + B / 6 TB/s for B dirty bytes, ~2.5 us
// per 15 MB matrix).  base: wave-uniform; off: elements (32-bit byte offsets).
#ifndef BGCN_WT_OUT
#define BGCN_WT_OUT 0   // A/B r04: chain alone 148-151 vs 147-154 us, step within noise
#endif
__device__ __forceinline__ void st4_chain(float* base, int64_t off, float4 v);
#ifndef BGCN_X_AUX
#define BGCN_X_AUX 2   // A/B: the cache-policy bits of the pass over X (sc0 = 1, nt = 2, sc1 = 16)
#endif
constexpr int kAuxNT = BGCN_X_AUX;   // buffer-load cache policy: non-temporal
// 16 B of an X row as one lane loads it: four fp32 or eight bf16 elements.  The zero
// tests work on the raw bits (magnitude bits only: -0 is zero, NaN is not, as `!= 0.f`),
// so a bf16 chunk costs the same instructions as an fp32 one for twice the elements.
template <class TX> struct XChunk;
template <> struct XChunk<float> {
  static constexpr int kElems = 4;
  __device__ static bool any(u32x4 r) { return ((r.x | r.y | r.z | r.w) & 0x7fffffffu) != 0; }
  __device__ static bool nz(u32x4 r, int c) { return (r[c] & 0x7fffffffu) != 0; }
  __device__ static float elem(u32x4 r, int c) { return __uint_as_float(r[c]); }
};
template <> struct XChunk<bf16_t> {
  static constexpr int kElems = 8;
  __device__ static bool any(u32x4 r) { return ((r.x | r.y | r.z | r.w) & 0x7fff7fffu) != 0; }
  __device__ static bool nz(u32x4 r, int c) {
    return (r[c >> 1] & ((c & 1) ? 0x7fff0000u : 0x00007fffu)) != 0;
  }
  __device__ static float elem(u32x4 r, int c) {   // element 2w is the low half of word w
    return __uint_as_float((c & 1) ? (r[c >> 1] & 0xffff0000u) : (r[c >> 1] << 16));
  }
};
__device__ __forceinline__ float xs(const float* p) { return *p; }
__device__ __forceinline__ float xs(const bf16_t* p) { return bf2f(*p); }

// Aggregation plan of one CSR orientation (built by K1 for the fused step, weight-
// independent): chunk g of the nominal kPlanChunk-entry grid covers the entries
// [bnd[g].x, bnd[g].y) - complete rows of <= kPlanChunk entries only (the boundary moves
// back to the row start; an empty or negative range means no work); the rows of more
// entries ("long rows", BU star roots) are listed in longs[0 .. *nlong) and aggregated by
// one block each.  No row is split, so no fixup pass follows.
constexpr int kPlanChunk = 16;
// The chunk grid itself is finer: chunk g owns the rows [row(g * kPlanGrid), row((g + 1) *
// kPlanGrid)), at most kPlanGrid + kPlanChunk - 1 entries, so a group's gathers mostly fit
// in one round of eight (a 16-entry grid took two dependent rounds per group).
#ifndef BGCN_PLAN_GRID
#define BGCN_PLAN_GRID 16
#endif
constexpr int kPlanGrid = BGCN_PLAN_GRID;
static_assert(kPlanGrid <= kPlanChunk, "a chunk holds at most 2 * 16 - 1 entries");
struct SpmmPlan {
  const int2* bnd;
  const int32_t* longs;
  const int32_t* nlong;
};

__device__ __forceinline__ bool gate_closed(const int32_t* gate) { return gate && *gate == 0; }
__device__ __forceinline__ bool dense_active(const int32_t* gate) { return !gate_closed(gate); }

}  // namespace bgcn
