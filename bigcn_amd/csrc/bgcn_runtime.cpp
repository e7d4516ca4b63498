// Host runtime of libbgcn: thread-local error string, ABI version, the per-device auxiliary
// streams ("lanes") of the fused step's independent branches, and the (process-global) kernel-timing
// hook bench.py uses to measure the dominant kernel with HIP events on the stream it is
// launched on.
#include <hip/hip_runtime.h>

#include <cstdlib>
#include <mutex>
#include <string>
#include <vector>

#include "bgcn_common.h"

namespace bgcn {

namespace {
constexpr int kTimingClasses = 12;
thread_local std::string g_err;

struct TimingState {
  bool enabled = false;
  unsigned mask = 0;  // bit c: class c is timed
  struct Pair { hipEvent_t a, b; };
  std::vector<Pair> pending[kTimingClasses];
  hipEvent_t open[kTimingClasses] = {};
  double total_ms[kTimingClasses] = {};
  int64_t count[kTimingClasses] = {};
  std::vector<hipEvent_t> free_events;  // recycled after readout: no create in the timed loop
};
// process-global: the fused backward runs on autograd's device thread, the forward on
// the caller's thread; both record into the same state
TimingState g_tm;
std::mutex g_tm_mu;

// Device-side spans (span_slot): one record per launch of a stamped kernel - the start
// times of its first kSpanStarts blocks and the end time of every block (slot b mod
// kSpanEnds), on the device's constant wall clock, written without contended atomics; the
// host takes min(start) and max(end).  Zeroed when timing is enabled.
constexpr int kSpanCap = 256;   // launches per timing session
struct SpanState {
  uint64_t* dev = nullptr;
  int next = 0;
  std::vector<int> slots[kTimingClasses];
};
SpanState g_span;

// auxiliary streams ("lanes") + fork/join events per device (created on first use)
constexpr int kMaxDevices = 64;
struct AuxState {
  hipStream_t stream[kAuxLanes] = {};
  hipEvent_t fork[kAuxLanes] = {}, join[kAuxLanes] = {};
  hipEvent_t prep = nullptr;   // end of the side lane's last next-batch preparation
  bool prep_pending = false;   // recorded, not yet waited for by the stream that queued it
  hipStream_t prep_owner = nullptr;   // the caller's stream whose step queued it
};
AuxState g_aux[kMaxDevices];
std::mutex g_aux_mu;

// Each lane of a device is created on its first use.
AuxState* aux_state(int lane) {
  int dev = 0;
  if (lane < 0 || lane >= kAuxLanes) return nullptr;
  if (hipGetDevice(&dev) != hipSuccess || dev < 0 || dev >= kMaxDevices) return nullptr;
  AuxState& a = g_aux[dev];
  if (!a.stream[lane]) {   // a lane's stream is created on its first use (an unused lane
                           // takes no hardware queue)
    for (int k = lane; k <= lane; ++k) {
      hipStream_t st;
      // BGCN_SIDE_CU_EVERY=k (A/B knob, read at lane creation): the lane may not use CU i
      // when i % k == k - 1, leaving those CUs to the caller's chain
      const char* ce = std::getenv("BGCN_SIDE_CU_EVERY");
      const int every = ce ? atoi(ce) : 0;
      if (every > 1) {
        hipDeviceProp_t prop;
        if (hipGetDeviceProperties(&prop, dev) != hipSuccess) return nullptr;
        const int ncu = prop.multiProcessorCount;
        std::vector<uint32_t> mask((ncu + 31) / 32, 0u);
        for (int i = 0; i < ncu; ++i)
          if (i % every != every - 1) mask[i / 32] |= 1u << (i % 32);
        if (hipExtStreamCreateWithCUMask(&st, uint32_t(mask.size()), mask.data()) != hipSuccess)
          return nullptr;
      } else if (hipStreamCreateWithFlags(&st, hipStreamNonBlocking) != hipSuccess) {
        return nullptr;
      }
      // fork / join events only order two streams of the same device: a device-scope
      // release suffices (what a kernel boundary on one stream gives).  The default
      // system-scope fence writes back and invalidates every XCD's L2 at each record
      // (measured ~6 us of device time per fork, and the next kernels start cold).
      constexpr unsigned kFlags = hipEventDisableTiming | hipEventDisableSystemFence;
      if (hipEventCreateWithFlags(&a.fork[k], kFlags) != hipSuccess ||
          hipEventCreateWithFlags(&a.join[k], kFlags) != hipSuccess)
        return nullptr;
      if (!a.prep && hipEventCreateWithFlags(&a.prep, kFlags) != hipSuccess) return nullptr;
      a.stream[k] = st;
    }
  }
  return &a;
}
}  // namespace

void set_error(const std::string& msg) { g_err = msg; }

int fail(int code, const std::string& msg) {
  g_err = msg;
  return code;
}

hipEvent_t take_event() {  // caller holds g_tm_mu
  if (!g_tm.free_events.empty()) {
    hipEvent_t e = g_tm.free_events.back();
    g_tm.free_events.pop_back();
    return e;
  }
  hipEvent_t e = nullptr;
  // timing only: no system-scope fence (no L2 writeback / invalidate that would perturb
  // the kernels being timed)
  return hipEventCreateWithFlags(&e, hipEventDisableSystemFence) == hipSuccess ? e : nullptr;
}

void timing_begin(int cls, hipStream_t s) {
  if (!g_tm.enabled || cls < 0 || cls >= kTimingClasses || !((g_tm.mask >> cls) & 1u)) return;
  std::lock_guard<std::mutex> lk(g_tm_mu);
  hipEvent_t e = take_event();
  if (!e) return;
  (void)hipEventRecord(e, s);
  g_tm.open[cls] = e;
}

uint64_t* span_slot(int cls) {
  if (!g_tm.enabled || cls < 0 || cls >= kTimingClasses || !((g_tm.mask >> cls) & 1u)) return nullptr;
  std::lock_guard<std::mutex> lk(g_tm_mu);
  if (!g_span.dev || g_span.next >= kSpanCap) return nullptr;
  const int i = g_span.next++;
  g_span.slots[cls].push_back(i);
  return g_span.dev + size_t(kSpanRecord) * i;
}

void timing_end(int cls, hipStream_t s) {
  if (!g_tm.enabled || cls < 0 || cls >= kTimingClasses || !((g_tm.mask >> cls) & 1u)) return;
  std::lock_guard<std::mutex> lk(g_tm_mu);
  if (!g_tm.open[cls]) return;
  hipEvent_t e = take_event();
  if (!e) return;
  (void)hipEventRecord(e, s);
  g_tm.pending[cls].push_back({g_tm.open[cls], e});
  g_tm.open[cls] = nullptr;
}

// BGCN_SERIAL=1 in the environment runs every branch inline (A/B measurements)
bool serial_branches() {
  static const bool v = [] {
    const char* e = std::getenv("BGCN_SERIAL");
    return e && e[0] == '1';
  }();
  return v;
}

int aux_fork(hipStream_t main, int lane, hipStream_t* branch) {
  *branch = main;
  if (!main || serial_branches()) return BGCN_OK;  // inline (see bgcn_common.h)
  std::lock_guard<std::mutex> lk(g_aux_mu);
  AuxState* a = aux_state(lane);
  if (!a) return fail(BGCN_EHIP, "auxiliary stream unavailable");
  BGCN_CHECK_HIP(hipEventRecord(a->fork[lane], main));
  BGCN_CHECK_HIP(hipStreamWaitEvent(a->stream[lane], a->fork[lane], 0));
  *branch = a->stream[lane];
  return BGCN_OK;
}

int aux_join(hipStream_t main, int lane) {
  if (!main || serial_branches()) return BGCN_OK;
  std::lock_guard<std::mutex> lk(g_aux_mu);
  AuxState* a = aux_state(lane);
  if (!a) return fail(BGCN_EHIP, "auxiliary stream unavailable");
  BGCN_CHECK_HIP(hipEventRecord(a->join[lane], a->stream[lane]));
  BGCN_CHECK_HIP(hipStreamWaitEvent(main, a->join[lane], 0));
  // everything queued on the lane is now ordered before `main` - but only the stream that
  // queued the preparation may stop waiting for it (another stream's join, e.g. an eval
  // forward, says nothing about the training stream)
  if (lane == kLaneSide && main == a->prep_owner) a->prep_pending = false;
  return BGCN_OK;
}

int aux_prep_done(hipStream_t main) {
  if (!main || serial_branches()) return BGCN_OK;
  std::lock_guard<std::mutex> lk(g_aux_mu);
  AuxState* a = aux_state(kLaneSide);
  if (!a) return fail(BGCN_EHIP, "auxiliary stream unavailable");
  BGCN_CHECK_HIP(hipEventRecord(a->prep, a->stream[kLaneSide]));
  a->prep_pending = true;
  a->prep_owner = main;
  return BGCN_OK;
}

int aux_prep_wait(hipStream_t main) {
  if (!main || serial_branches()) return BGCN_OK;
  std::lock_guard<std::mutex> lk(g_aux_mu);
  AuxState* a = aux_state(kLaneSide);
  if (!a) return fail(BGCN_EHIP, "auxiliary stream unavailable");
  if (!a->prep_pending) return BGCN_OK;
  BGCN_CHECK_HIP(hipStreamWaitEvent(main, a->prep, 0));
  if (main == a->prep_owner) a->prep_pending = false;   // other streams keep waiting too
  return BGCN_OK;
}

}  // namespace bgcn

extern "C" int bgcn_abi_version(void) { return BGCN_ABI_VERSION; }

extern "C" int bgcn_join_side(bgcn_stream_t stream) {
  return bgcn::aux_join(reinterpret_cast<hipStream_t>(stream), bgcn::kLaneSide);
}

extern "C" const char* bgcn_last_error(void) { return bgcn::g_err.c_str(); }

extern "C" int bgcn_set_kernel_timing(int enable) {
  std::lock_guard<std::mutex> lk(bgcn::g_tm_mu);
  auto& t = bgcn::g_tm;
  t.enabled = enable != 0;
  t.mask = unsigned(enable);
  for (int c = 0; c < bgcn::kTimingClasses; ++c) {
    t.total_ms[c] = 0;
    t.count[c] = 0;
    if (!t.enabled) continue;       // disabling keeps the pending events for readout
    for (auto& p : t.pending[c]) {  // enabling drops events of classes nobody read out
      (void)hipEventSynchronize(p.b);
      t.free_events.push_back(p.a);
      t.free_events.push_back(p.b);
    }
    t.pending[c].clear();
    if (t.open[c]) (void)hipEventSynchronize(t.open[c]), t.free_events.push_back(t.open[c]);
    t.open[c] = nullptr;
  }
  // the span array: (re)filled with {~0, 0} pairs when timing is enabled, synchronously
  // (outside any timed region); disabling keeps the recorded spans for bgcn_kernel_span
  auto& sp = bgcn::g_span;
  if (t.enabled) {
    for (auto& v : sp.slots) v.clear();
    sp.next = 0;
    const size_t bytes = sizeof(uint64_t) * size_t(bgcn::kSpanRecord) * bgcn::kSpanCap;
    if (!sp.dev && hipMalloc(reinterpret_cast<void**>(&sp.dev), bytes) != hipSuccess) sp.dev = nullptr;
    if (sp.dev && (hipMemset(sp.dev, 0, bytes) != hipSuccess || hipDeviceSynchronize() != hipSuccess))
      return bgcn::fail(BGCN_EHIP, "span array init failed");
  }
  // pre-create events so that the timed loop only records (hipEventCreate is not free)
  while (t.enabled && t.free_events.size() < 1024) {
    hipEvent_t e = nullptr;
    if (hipEventCreate(&e) != hipSuccess) break;
    t.free_events.push_back(e);
  }
  return BGCN_OK;
}

// Synchronises on the recorded events (call outside the timed region).
extern "C" int bgcn_kernel_timing(int kernel_class, float* total_ms, int64_t* launches) {
  std::lock_guard<std::mutex> lk(bgcn::g_tm_mu);
  auto& t = bgcn::g_tm;
  if (kernel_class < 0 || kernel_class >= bgcn::kTimingClasses) return bgcn::fail(BGCN_EINVAL, "bad kernel class");
  auto& v = t.pending[kernel_class];
  for (auto& p : v) {
    float ms = 0.f;
    if (hipEventSynchronize(p.b) != hipSuccess) return bgcn::fail(BGCN_EHIP, "event sync failed");
    if (hipEventElapsedTime(&ms, p.a, p.b) == hipSuccess) {
      t.total_ms[kernel_class] += ms;
      t.count[kernel_class] += 1;
    }
    t.free_events.push_back(p.a);
    t.free_events.push_back(p.b);
  }
  v.clear();
  if (total_ms) *total_ms = float(t.total_ms[kernel_class]);
  if (launches) *launches = t.count[kernel_class];
  return BGCN_OK;
}

// Synchronises (hipDeviceSynchronize, then one copy of the used pairs).
extern "C" int bgcn_kernel_span(int kernel_class, float* total_ms, int64_t* launches) {
  std::lock_guard<std::mutex> lk(bgcn::g_tm_mu);
  if (kernel_class < 0 || kernel_class >= bgcn::kTimingClasses) return bgcn::fail(BGCN_EINVAL, "bad kernel class");
  auto& sp = bgcn::g_span;
  double ms = 0.0;
  int64_t n = 0;
  if (sp.dev && !sp.slots[kernel_class].empty()) {
    BGCN_CHECK_HIP(hipDeviceSynchronize());
    std::vector<uint64_t> h(size_t(bgcn::kSpanRecord) * size_t(sp.next));
    BGCN_CHECK_HIP(hipMemcpy(h.data(), sp.dev, h.size() * sizeof(uint64_t), hipMemcpyDeviceToHost));
    int dev = 0, khz = 0;
    BGCN_CHECK_HIP(hipGetDevice(&dev));
    BGCN_CHECK_HIP(hipDeviceGetAttribute(&khz, hipDeviceAttributeWallClockRate, dev));
    if (khz <= 0) return bgcn::fail(BGCN_EHIP, "no wall clock rate");
    for (int i : sp.slots[kernel_class]) {
      const uint64_t* r = h.data() + size_t(bgcn::kSpanRecord) * i;
      uint64_t a = ~uint64_t(0), b = 0;
      for (int k = 0; k < bgcn::kSpanStarts; ++k)
        if (r[k]) a = r[k] < a ? r[k] : a;
      for (int k = bgcn::kSpanStarts; k < bgcn::kSpanRecord; ++k) b = r[k] > b ? r[k] : b;
      if (b >= a && a != ~uint64_t(0)) {
        ms += double(b - a) / double(khz);
        ++n;
      }
    }
  }
  if (total_ms) *total_ms = float(ms);
  if (launches) *launches = n;
  return BGCN_OK;
}
