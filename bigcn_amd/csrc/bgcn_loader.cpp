// Native host-fed loader: worker THREADS collate each batch of a
// TreeStore into a slot of a page-locked ring, the caller's thread issues one H2D copy per
// batch and gets the batch's layout back.  The role of the reference's
// DataLoader(traindata_list, batch_size=128, shuffle=True, num_workers=5) + Batch_data.to(device)
// (model/Twitter/BiGCN_Twitter.py:168,174-176) with the collation of feed.pack_batch
// (PyG Batch.from_data_list: "index" keys offset by the running node count, batch / ptr built,
// BU = the flipped TD list; Process/dataset.py:80-90) - byte for byte the same packed batch
// (tests/test_feed.py), with no per-batch Python: the torch DataLoader's main-process side
// (index queue, result unpickling, the sampler, the tensor bookkeeping of the copy) took
// ~170 us per batch, more than half the host-fed step.
//
// Slot life cycle: FREE -> packed by a worker -> READY -> copy issued by bgcn_loader_next
// (an event recorded after it on the copy stream) -> FREE again once the caller's thread
// sees that event completed (the worker packing batch seq + nslots into it waits for it).  Batches come out in
// sequence order; the permutation of each epoch is a Fisher-Yates shuffle from a
// counter-based generator of (seed, epoch), so a run is reproducible for a given seed.
#include <hip/hip_runtime.h>

#include <algorithm>
#include <chrono>
#include <cstdlib>
#include <atomic>
#include <condition_variable>
#include <cstring>
#include <mutex>
#include <new>
#include <thread>
#include <vector>

#include "bgcn.h"
#include "bgcn_common.h"

namespace bgcn {
namespace {

constexpr int64_t kAlign = 256;
inline int64_t pad(int64_t n) { return (n + kAlign - 1) / kAlign * kAlign; }

// the packed sections, in order (feed._SECTIONS): element sizes
constexpr int kSections = 9;
constexpr int kElem[kSections] = {4, 4, 4, 8, 8, 8, 8, 8, 8};

inline uint64_t splitmix(uint64_t& s) {
  uint64_t z = (s += 0x9E3779B97F4A7C15ull);
  z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ull;
  z = (z ^ (z >> 27)) * 0x94D049BB133111EBull;
  return z ^ (z >> 31);
}

// float -> bf16 -> float, round to nearest even (torch's .to(torch.bfloat16)); NaN kept quiet
inline float round_bf16(float v) {
  uint32_t u;
  std::memcpy(&u, &v, 4);
  if ((u & 0x7f800000u) == 0x7f800000u && (u & 0x007fffffu)) {
    u |= 0x00400000u;
    u &= 0xffff0000u;
  } else {
    u += 0x7fffu + ((u >> 16) & 1u);
    u &= 0xffff0000u;
  }
  float r;
  std::memcpy(&r, &u, 4);
  return r;
}

// k_slot_copy's default grid: 16 blocks keep ~256 KB of PCIe reads in flight (the copy runs at
// the 64-block rate, ~0.11 ms per 4.5 MB batch) and leave the step's kernels the other CUs -
// host-fed 476-488k vs 434-448k trees/s with 64 blocks (profiles/r06_slot_copy_blocks_ab.txt)
constexpr int kCopyBlocks = 16;

struct Slot {
  uint8_t* host = nullptr;       // page-locked (registered), or plain memory (host-only loader)
  const uint8_t* dev = nullptr;  // the same pages in the device's address space (pinned loader)
  int64_t next = 0;              // the batch it takes next (its index, then + nslots per use)
  int64_t seq = -1;              // the batch it holds / is being packed with
  int state = 0;                 // 0 free, 1 packing, 2 ready, 3 copy issued, 4 held (host-only)
  hipEvent_t copied = nullptr;   // recorded after the copy out of it
  bgcn_loader_batch meta{};
  std::vector<int64_t> trees;    // the batch's tree ids (store order)
};

struct Loader {
  bgcn_tree_store st{};
  std::vector<int64_t> indices;  // the dataset's trees (store ids)
  int64_t batch_size = 0;
  bool drop_last = true, shuffle = true, bf16 = false, pinned = true;
  uint64_t seed = 0;
  int64_t epochs = 1, per_epoch = 0, total = 0;
  int64_t slot_bytes = 0;
  std::vector<Slot> slots;
  std::vector<std::vector<int64_t>> perm;   // per epoch (built on first use)
  std::mutex mu;
  std::condition_variable cv;
  int64_t next_pack = 0;         // next batch a worker claims
  int64_t next_out = 0;          // next batch bgcn_loader_next returns
  Slot* held = nullptr;          // host-only use: the slot whose bytes the caller is reading
  bool stop = false;
  std::string error;
  std::vector<std::thread> workers;
  int device = 0;
  // time accounting (bgcn_loader_stats), under mu
  int64_t packs = 0;
  double pack_ms = 0, slot_wait_ms = 0, caller_wait_ms = 0;
  double copy_call_ms = 0, copy_call_ms_max = 0, record_call_ms_max = 0;   // host time in the copy calls
  // the H2D copy: k_slot_copy reading the mapped slot (default), or hipMemcpyAsync on the
  // DMA engine (BGCN_LOADER_COPY=sdma, A/B only: see k_slot_copy)
  bool sdma = false;
  int copy_blocks = kCopyBlocks;   // k_slot_copy's grid (BGCN_LOADER_COPY_BLOCKS, A/B)
};

inline double ms_since(std::chrono::steady_clock::time_point t0) {
  return std::chrono::duration<double, std::milli>(std::chrono::steady_clock::now() - t0).count();
}

const std::vector<int64_t>& epoch_perm(Loader& L, int64_t e) {   // under L.mu
  while (int64_t(L.perm.size()) <= e) {
    std::vector<int64_t> p(L.indices);
    if (L.shuffle) {
      uint64_t s = L.seed ^ (0xD1B54A32D192ED03ull * uint64_t(L.perm.size() + 1));
      for (int64_t i = int64_t(p.size()) - 1; i > 0; --i) {
        const int64_t j = int64_t(splitmix(s) % uint64_t(i + 1));
        std::swap(p[size_t(i)], p[size_t(j)]);
      }
    }
    L.perm.push_back(std::move(p));
  }
  return L.perm[size_t(e)];
}

// feed.pack_batch without host DropEdge: the same sections, offsets and values
bool pack(const Loader& L, const std::vector<int64_t>& t, uint8_t* out, int64_t cap, bgcn_loader_batch& m,
          std::string& err) {
  const bgcn_tree_store& s = L.st;
  const int64_t B = int64_t(t.size());
  int64_t N = 0, nnz = 0, E = 0;
  for (int64_t b = 0; b < B; ++b) {
    const int64_t k = t[size_t(b)];
    N += s.tree_node[k + 1] - s.tree_node[k];
    nnz += s.entry_off[k + 1] - s.entry_off[k];
    E += s.tree_edge[k + 1] - s.tree_edge[k];
  }
  const int64_t count[kSections] = {N + 1, nnz, nnz, 2 * E, 2 * E, N, B, B, B + 1};
  int64_t off = 0;
  for (int q = 0; q < kSections; ++q) {
    m.off[q] = off;
    off += pad(count[q] * kElem[q]);
  }
  if (off > cap) {
    err = "a batch does not fit the loader's slot";
    return false;
  }
  int32_t* rp = reinterpret_cast<int32_t*>(out + m.off[0]);
  int32_t* xc = reinterpret_cast<int32_t*>(out + m.off[1]);
  float* xv = reinterpret_cast<float*>(out + m.off[2]);
  int64_t* ei = reinterpret_cast<int64_t*>(out + m.off[3]);
  int64_t* bei = reinterpret_cast<int64_t*>(out + m.off[4]);
  int64_t* bt = reinterpret_cast<int64_t*>(out + m.off[5]);
  int64_t* ri = reinterpret_cast<int64_t*>(out + m.off[6]);
  int64_t* yy = reinterpret_cast<int64_t*>(out + m.off[7]);
  int64_t* pt = reinterpret_cast<int64_t*>(out + m.off[8]);
  int64_t n0 = 0, z0 = 0, e0 = 0, nnz_max = 0, spill = 0;
  bool bad = false;
  rp[0] = 0;
  for (int64_t b = 0; b < B; ++b) {
    const int64_t k = t[size_t(b)];
    const int64_t na = s.tree_node[k], nb = s.tree_node[k + 1];
    const int64_t za = s.entry_off[k], zb = s.entry_off[k + 1];
    const int64_t ea = s.tree_edge[k], eb = s.tree_edge[k + 1];
    pt[b] = n0;
    for (int64_t i = na; i < nb; ++i) {
      const int32_t c = s.node_nnz[i];
      rp[n0 + (i - na) + 1] = rp[n0 + (i - na)] + c;
      nnz_max = std::max<int64_t>(nnz_max, c);
      spill += std::max<int64_t>(int64_t(c) - BGCN_SPARSE_CAP, 0);
      bt[n0 + (i - na)] = b;
    }
    // the tree's non-zeros: plain copies (a column check pass the compiler vectorises)
    std::memcpy(xc + z0, s.cols + za, size_t(zb - za) * 4);
    if (L.bf16) {
      for (int64_t z = za; z < zb; ++z) xv[z0 + (z - za)] = round_bf16(s.vals[z]);
    } else {
      std::memcpy(xv + z0, s.vals + za, size_t(zb - za) * 4);
    }
    int32_t lo = 0, hi = 0;
    for (int64_t z = z0; z < z0 + (zb - za); ++z) {
      lo = std::min(lo, xc[z]);
      hi = std::max(hi, xc[z]);
    }
    bad |= lo < 0 || (zb > za && hi >= s.in_feats);
    for (int64_t e = ea; e < eb; ++e) {
      const int64_t p = int64_t(s.edges[e]) + n0, c = int64_t(s.edges[s.edges_ld + e]) + n0;
      ei[e0 + (e - ea)] = p;
      ei[E + e0 + (e - ea)] = c;
      bei[e0 + (e - ea)] = c;           // BU: the flipped TD list
      bei[E + e0 + (e - ea)] = p;
    }
    ri[b] = int64_t(s.rootindex[k]) + n0;
    yy[b] = s.y[k];
    n0 += nb - na;
    z0 += zb - za;
    e0 += eb - ea;
  }
  pt[B] = n0;
  if (bad) {
    err = "a feature column outside [0, in_feats) in the store";
    return false;
  }
  m.num_nodes = N;
  m.num_graphs = B;
  m.nnz = nnz;
  m.td_num_edges = m.bu_num_edges = E;
  m.nnz_max = nnz_max;
  m.spill = spill;
  m.bytes = off;
  return true;
}

// The H2D copy of a packed slot: a kernel reading the slot's page-locked pages through their
// device mapping (PCIe reads, 16 B per lane, four in flight; kCopyBlocks blocks), on the
// caller's copy stream.
// (Round 6: hipMemcpyAsync on the DMA engine stalled the issuing call by ~6.5 ms every few
// batches when copies came back to back - HSA_ENABLE_SDMA=0 removed the stalls - so the
// library issues its own copy; tools/loader_probe.py, profiles/r06_loader_probe*.json.)
typedef unsigned int copy4_t __attribute__((ext_vector_type(4)));
__global__ __launch_bounds__(256) void k_slot_copy(const copy4_t* __restrict__ src, copy4_t* __restrict__ dst,
                                                  int64_t n16) {
  const int64_t stride = int64_t(gridDim.x) * 1024;
  for (int64_t i = int64_t(blockIdx.x) * 1024 + threadIdx.x; i < n16; i += stride) {
    copy4_t v[4];
#pragma unroll
    for (int u = 0; u < 4; ++u) v[u] = __builtin_nontemporal_load(src + min<int64_t>(i + 256 * u, n16 - 1));
#pragma unroll
    for (int u = 0; u < 4; ++u)
      if (i + 256 * u < n16) __builtin_nontemporal_store(v[u], dst + i + 256 * u);
  }
}

// The caller's thread retires copied slots: a slot whose copy was issued (state 3) goes back
// to the workers (state 0) once its copy event has completed - polled with hipEventQuery,
// never waited for by a worker.  (Round 6: workers blocking in hipEventSynchronize on their
// slot's copy stalled the caller's next hipMemcpyAsync by ~6.5 ms every few batches when
// the copies ran back to back - tools/loader_probe.py, profiles/r06_loader_probe.json.)
// Under L->mu; true when a slot was retired.
bool retire_copied(Loader* L) {
  bool any = false;
  for (Slot& s : L->slots) {
    if (s.state == 3 && hipEventQuery(s.copied) == hipSuccess) {
      s.state = 0;
      any = true;
    }
  }
  return any;
}

// The caller waits (under lk) until batch `seq` is packed, retiring completed copies
// meanwhile so that workers waiting for those slots can go on.
void wait_packed(Loader* L, std::unique_lock<std::mutex>& lk, Slot& s, int64_t seq) {
  const auto tw = std::chrono::steady_clock::now();
  if (retire_copied(L)) L->cv.notify_all();
  while (!(s.state == 2 && s.seq == seq) && L->error.empty()) {
    L->cv.wait_for(lk, std::chrono::microseconds(50));
    if (retire_copied(L)) L->cv.notify_all();
  }
  L->caller_wait_ms += ms_since(tw);
}

void worker(Loader* L) {
  // (the workers make no HIP call: the caller's thread issues the copies and retires them)
  std::vector<int64_t> trees;
  for (;;) {
    int64_t seq;
    Slot* sl;
    {
      std::unique_lock<std::mutex> lk(L->mu);
      if (L->stop || L->next_pack >= L->total) return;
      seq = L->next_pack++;
      const auto tw = std::chrono::steady_clock::now();
      sl = &L->slots[size_t(seq % int64_t(L->slots.size()))];
      // the slot's turn: its previous batch (seq - nslots) handed out and its copy retired
      L->cv.wait(lk, [&] { return L->stop || (sl->next == seq && sl->state == 0); });
      if (L->stop) return;
      const std::vector<int64_t>& p = epoch_perm(*L, seq / L->per_epoch);
      const int64_t b0 = (seq % L->per_epoch) * L->batch_size;
      const int64_t b1 = std::min<int64_t>(b0 + L->batch_size, int64_t(p.size()));
      trees.assign(p.begin() + b0, p.begin() + b1);
      sl->state = 1;
      sl->seq = seq;
      L->slot_wait_ms += ms_since(tw);
    }
    bgcn_loader_batch m{};
    std::string err;
    const auto tp = std::chrono::steady_clock::now();
    const bool ok = pack(*L, trees, sl->host, L->slot_bytes, m, err);
    const double tpack = ms_since(tp);
    {
      std::lock_guard<std::mutex> lk(L->mu);
      L->pack_ms += tpack;
      ++L->packs;
      m.seq = seq;
      sl->meta = m;
      sl->trees = trees;
      sl->state = 2;
      if (!ok && L->error.empty()) L->error = err;
    }
    L->cv.notify_all();
  }
}

}  // namespace
}  // namespace bgcn

using namespace bgcn;

extern "C" {

int bgcn_loader_create(const bgcn_tree_store* st, const int64_t* indices, int64_t n, int64_t batch_size,
                       int drop_last, int shuffle, uint64_t seed, int64_t epochs, int num_threads, int nslots,
                       int bf16_values, int pinned, void** handle) {
  BGCN_CHECK_ARG(st && handle && batch_size > 0 && epochs > 0 && num_threads > 0 && nslots >= 2,
                 "bad loader arguments");
  BGCN_CHECK_ARG(st->num_trees >= 0 && st->in_feats > 0 && st->tree_node && st->node_nnz && st->entry_off &&
                     st->cols && st->vals && st->tree_edge && st->edges && st->rootindex && st->y,
                 "bad tree store");
  Loader* L = new (std::nothrow) Loader;
  BGCN_CHECK_ARG(L, "out of memory");
  L->st = *st;
  if (indices) {
    for (int64_t i = 0; i < n; ++i) {
      if (indices[i] < 0 || indices[i] >= st->num_trees) {
        delete L;
        return fail(BGCN_EINVAL, "a tree index outside the store");
      }
    }
    L->indices.assign(indices, indices + n);
  } else {
    L->indices.resize(size_t(st->num_trees));
    for (int64_t i = 0; i < st->num_trees; ++i) L->indices[size_t(i)] = i;
  }
  const int64_t cnt = int64_t(L->indices.size());
  L->batch_size = batch_size;
  L->drop_last = drop_last != 0;
  L->shuffle = shuffle != 0;
  L->seed = seed;
  L->epochs = epochs;
  L->bf16 = bf16_values != 0;
  L->pinned = pinned != 0;
  L->per_epoch = L->drop_last ? cnt / batch_size : (cnt + batch_size - 1) / batch_size;
  L->total = L->per_epoch * epochs;
  // slot size: the largest batch_size trees (bytes per tree as feed._per_tree_bytes) + padding
  std::vector<int64_t> per;
  per.reserve(L->indices.size());
  for (int64_t k : L->indices) {
    const int64_t nn = st->tree_node[k + 1] - st->tree_node[k];
    const int64_t nz = st->entry_off[k + 1] - st->entry_off[k];
    const int64_t ne = st->tree_edge[k + 1] - st->tree_edge[k];
    per.push_back(4 * nn + 8 * nz + 32 * ne + 8 * nn + 24);
  }
  std::sort(per.begin(), per.end(), std::greater<int64_t>());
  int64_t sb = 8 * (batch_size + 2) + kSections * kAlign + 4;
  for (int64_t i = 0; i < std::min<int64_t>(batch_size, int64_t(per.size())); ++i) sb += per[size_t(i)];
  L->slot_bytes = (sb + 4095) / 4096 * 4096;   // (page-aligned slots: aligned_alloc + register)
  L->slots.resize(size_t(nslots));
  for (int i = 0; i < nslots; ++i) L->slots[size_t(i)].next = i;
  if (L->pinned && hipGetDevice(&L->device) != hipSuccess) L->pinned = false;
  if (const char* e = std::getenv("BGCN_LOADER_COPY")) L->sdma = std::strcmp(e, "sdma") == 0;
  if (const char* e = std::getenv("BGCN_LOADER_COPY_BLOCKS")) L->copy_blocks = std::max(1, std::atoi(e));
  for (size_t k = 0; k < L->slots.size(); ++k) {
    Slot& s = L->slots[k];
    void* p = nullptr;
    bool ok;
    if (L->pinned) {
      // cached host pages, page-locked for the DMA (the packing threads write ~4.5 MB per
      // Twitter-sized batch; hipHostMalloc's default mapping made those writes slower), and
      // mapped into the device's address space for k_slot_copy
      p = std::aligned_alloc(4096, size_t(L->slot_bytes));
      ok = p != nullptr && hipHostRegister(p, size_t(L->slot_bytes), hipHostRegisterMapped) == hipSuccess;
      if (!ok && p) {
        std::free(p);
        p = nullptr;
      }
      void* dp = nullptr;
      ok = ok && hipHostGetDevicePointer(&dp, p, 0) == hipSuccess && dp != nullptr;
      s.dev = static_cast<const uint8_t*>(dp);
      ok = ok && hipEventCreateWithFlags(&s.copied, hipEventDisableTiming) == hipSuccess;
    } else {
      p = ::operator new(size_t(L->slot_bytes), std::nothrow);
      ok = p != nullptr;
    }
    // the pages faulted in here, not by the first packs (16 threads faulting 4 MB slots at
    // once serialise on the address space: 13-16 ms per first batch)
    if (ok) std::memset(p, 0, size_t(L->slot_bytes));
    s.host = static_cast<uint8_t*>(p);
    if (!ok) {
      bgcn_loader_destroy(L);
      return fail(BGCN_EHIP, "loader slot allocation failed");
    }
  }
  for (int i = 0; i < num_threads; ++i) L->workers.emplace_back(worker, L);
  *handle = L;
  return BGCN_OK;
}

int64_t bgcn_loader_slot_bytes(void* handle) {
  return handle ? static_cast<Loader*>(handle)->slot_bytes : 0;
}

int64_t bgcn_loader_len(void* handle) { return handle ? static_cast<Loader*>(handle)->total : 0; }

int bgcn_loader_next(void* handle, void* dst, size_t dst_bytes, bgcn_stream_t stream, bgcn_loader_batch* out,
                     int64_t* trees, int64_t trees_cap, const void** host_bytes) {
  Loader* L = static_cast<Loader*>(handle);
  BGCN_CHECK_ARG(L && out, "null loader / output");
  std::unique_lock<std::mutex> lk(L->mu);
  if (L->held) {   // host-only use: the previous call's slot goes back to the workers
    L->held->state = 0;
    L->held->next = L->held->seq + int64_t(L->slots.size());
    L->held = nullptr;
    L->cv.notify_all();
  }
  if (L->next_out >= L->total) return 1;   // the end of the data
  const int64_t seq = L->next_out;
  Slot& s = L->slots[size_t(seq % int64_t(L->slots.size()))];
  wait_packed(L, lk, s, seq);
  if (!L->error.empty()) return fail(BGCN_EINVAL, L->error.c_str());
  *out = s.meta;
  if (trees) {
    BGCN_CHECK_ARG(trees_cap >= int64_t(s.trees.size()), "tree list buffer too small");
    std::copy(s.trees.begin(), s.trees.end(), trees);
  }
  if (dst) {
    BGCN_CHECK_ARG(L->pinned, "a host-only loader copies nothing");
    BGCN_CHECK_ARG(dst_bytes >= size_t(s.meta.bytes), "device buffer too small for the batch");
    auto st = reinterpret_cast<hipStream_t>(stream);
    const auto tc = std::chrono::steady_clock::now();
    if (L->sdma) {
      BGCN_CHECK_HIP(hipMemcpyAsync(dst, s.host, size_t(s.meta.bytes), hipMemcpyHostToDevice, st));
    } else {
      BGCN_CHECK_ARG((reinterpret_cast<uintptr_t>(dst) & 15) == 0, "device buffer must be 16-byte aligned");
      const int64_t n16 = s.meta.bytes / 16;   // sections are 256-byte padded
      hipLaunchKernelGGL(k_slot_copy, dim3(unsigned(std::min<int64_t>(L->copy_blocks, (n16 + 1023) / 1024))),
                         dim3(256), 0, st, reinterpret_cast<const copy4_t*>(s.dev), static_cast<copy4_t*>(dst), n16);
      BGCN_CHECK_HIP(hipGetLastError());
    }
    const double tcall = ms_since(tc);
    const auto tr = std::chrono::steady_clock::now();
    BGCN_CHECK_HIP(hipEventRecord(s.copied, st));
    const double trec = ms_since(tr);
    L->copy_call_ms += tcall + trec;
    L->copy_call_ms_max = std::max(L->copy_call_ms_max, tcall);
    L->record_call_ms_max = std::max(L->record_call_ms_max, trec);
    s.state = 3;
    s.next = seq + int64_t(L->slots.size());
  } else {
    // host-only use (tests): the bytes stay readable until the next call
    if (host_bytes) *host_bytes = s.host;
    s.state = 4;
    L->held = &s;
  }
  ++L->next_out;
  lk.unlock();
  L->cv.notify_all();
  return BGCN_OK;
}

int bgcn_loader_wait(void* handle) {
  Loader* L = static_cast<Loader*>(handle);
  BGCN_CHECK_ARG(L, "null loader");
  std::unique_lock<std::mutex> lk(L->mu);
  if (L->next_out >= L->total) return 1;
  const int64_t seq = L->next_out;
  Slot& s = L->slots[size_t(seq % int64_t(L->slots.size()))];
  wait_packed(L, lk, s, seq);
  if (!L->error.empty()) return fail(BGCN_EINVAL, L->error.c_str());
  return BGCN_OK;
}

int bgcn_loader_get_stats(void* handle, bgcn_loader_stats* out, int reset) {
  Loader* L = static_cast<Loader*>(handle);
  BGCN_CHECK_ARG(L && out, "null loader / output");
  std::lock_guard<std::mutex> lk(L->mu);
  out->packs = L->packs;
  out->pack_ms = L->pack_ms;
  out->slot_wait_ms = L->slot_wait_ms;
  out->caller_wait_ms = L->caller_wait_ms;
  out->threads = int64_t(L->workers.size());
  out->copy_call_ms = L->copy_call_ms;
  out->copy_call_ms_max = L->copy_call_ms_max;
  out->record_call_ms_max = L->record_call_ms_max;
  if (reset) {
    L->packs = 0;
    L->pack_ms = L->slot_wait_ms = L->caller_wait_ms = L->copy_call_ms = L->copy_call_ms_max = L->record_call_ms_max = 0;
  }
  return BGCN_OK;
}

void bgcn_loader_destroy(void* handle) {
  Loader* L = static_cast<Loader*>(handle);
  if (!L) return;
  {
    std::lock_guard<std::mutex> lk(L->mu);
    L->stop = true;
  }
  L->cv.notify_all();
  for (std::thread& t : L->workers) t.join();
  for (Slot& s : L->slots) {
    if (L->pinned) {
      if (s.copied) {
        (void)hipEventSynchronize(s.copied);
        (void)hipEventDestroy(s.copied);
      }
      if (s.host) {
        (void)hipHostUnregister(s.host);
        std::free(s.host);
      }
    } else if (s.host) {
      ::operator delete(s.host);
    }
  }
  delete L;
}

}  // extern "C"
