// plan.hip — native step launcher: a recorded training step replayed from C++.
//
// The eager step of the executor (runtime/executor.py) is a fixed sequence of ~340 kernel launches
// on two streams (the high-priority critical-path stream and the weight-gradient side stream) plus
// the cross-stream event records / waits that order them. Issued from Python every launch costs
// ~19 us of host time (ctypes marshalling of the argument block, geometry keys, stream objects):
// 6.4 ms per ResNet-50 step, 3-5 ms per CIFAR step -- the host, not the GPU, bounds the CIFAR
// steps and any future faster ImageNet step. A HIP graph removes that cost but replays every
// branch from one normal-priority queue (ResNet-50: 10.4 vs 9.6 ms eager).
//
// A Plan keeps the eager structure and drops the Python: while the calling thread records
// (drn_plan_record_begin .. _end), every drn::launch of the library appends {kernel, grid, block,
// LDS, stream, by-value argument copy} instead of launching (drn_common.h), and the runtime adds
// event-record / stream-wait entries (drn_plan_event_record / drn_plan_stream_wait) where the
// Python step would have called torch's stream API. drn_plan_replay(begin, end) then re-issues
// entries [begin, end) with hipModuleLaunchKernel (function handles resolved at record time) /
// hipEventRecord / hipStreamWaitEvent: the same
// kernels, arguments, streams and priorities as the eager step, one host call per segment (the
// data-parallel step is cut at the points where a bucket collective is issued from Python).
// The equivalent of the reference's per-step `mon_sess.run(train_op)` executor call
// (resnet_cifar_main.py:320-321).
#include "drn_common.h"

#include <algorithm>
#include <atomic>
#include <condition_variable>
#include <memory>
#include <mutex>
#include <thread>
#include <vector>

#include <immintrin.h>

namespace drn {

thread_local Plan* g_plan_rec = nullptr;

struct PlanEntry {
  enum Kind : int { LAUNCH = 0, RECORD = 1, WAIT = 2 };
  int kind = LAUNCH;
  const void* fn = nullptr;
  hipFunction_t func = nullptr;  // resolved once at record time: replay skips the stub lookup
  dim3 grid, block;
  size_t shm = 0;
  hipStream_t stream = nullptr;
  void* blob = nullptr;
  void** argv = nullptr;
  void (*del)(void*) = nullptr;
  int ev = -1;
  // multi-lane replay: the entry's lane (one per stream) and, for event entries, the previous
  // entry on the same event (issued first when it lies in the replayed range)
  int lane = 0;
  int prev_ev = -1;
};

struct Plan {
  std::vector<PlanEntry> e;
  std::vector<hipEvent_t> events;
  std::vector<hipStream_t> lanes;          // distinct streams, in order of first use
  std::vector<int> last_ev_entry;          // per event: its latest entry so far (recording)
  std::vector<char> ev_waited;             // per event: some stream waits on it (else its records are dead)
  size_t analyzed_n = 0;
  int launches = 0;
  int device = 0;
  // ---- multi-lane replay (drn_plan_set_threads) ----
  int threads = 1;
  std::unique_ptr<std::atomic<uint64_t>[]> issued;  // per entry: epoch of its last issue
  size_t issued_n = 0;
  uint64_t epoch = 0;
  std::vector<std::thread> workers;
  std::mutex mu;
  std::condition_variable cv_go, cv_done;
  uint64_t job = 0;                        // generation of the published range
  int job_begin = 0, job_end = 0, job_lanes = 0;
  int done = 0;
  bool stop = false;
  std::atomic<int> err{0};
  ~Plan() {
    {
      std::lock_guard<std::mutex> g(mu);
      stop = true;
    }
    cv_go.notify_all();
    for (auto& t : workers) t.join();
    for (auto& x : e) {
      if (x.del != nullptr) x.del(x.blob);
      delete[] x.argv;
    }
    for (auto ev : events) (void)hipEventDestroy(ev);
  }
};

static int lane_of(Plan* p, hipStream_t s) {
  for (size_t i = 0; i < p->lanes.size(); ++i)
    if (p->lanes[i] == s) return (int)i;
  p->lanes.push_back(s);
  return (int)p->lanes.size() - 1;
}

void plan_add_launch(Plan* p, const void* fn, dim3 grid, dim3 block, size_t shm, hipStream_t s, void* blob,
                     void** argv, void (*del)(void*)) {
  PlanEntry x;
  x.kind = PlanEntry::LAUNCH;
  x.fn = fn;
  if (hipGetFuncBySymbol(&x.func, fn) != hipSuccess) x.func = nullptr;
  x.grid = grid;
  x.block = block;
  x.shm = shm;
  x.stream = s;
  x.blob = blob;
  x.argv = argv;
  x.del = del;
  x.lane = lane_of(p, s);
  p->e.push_back(x);
  ++p->launches;
}

static void add_event_entry(Plan* p, PlanEntry& x) {
  x.lane = lane_of(p, x.stream);
  x.prev_ev = p->last_ev_entry[x.ev];
  p->last_ev_entry[x.ev] = (int)p->e.size();
  p->e.push_back(x);
}

static hipError_t issue(const Plan* p, const PlanEntry& x) {
  switch (x.kind) {
    case PlanEntry::LAUNCH:
      return x.func != nullptr ? hipModuleLaunchKernel(x.func, x.grid.x, x.grid.y, x.grid.z, x.block.x, x.block.y,
                                                       x.block.z, (unsigned)x.shm, x.stream, x.argv, nullptr)
                               : hipLaunchKernel(x.fn, x.grid, x.block, x.argv, x.shm, x.stream);
    case PlanEntry::RECORD:  // (records nothing in the plan waits on -- most side-stream marks -- are skipped)
      return p->ev_waited[x.ev] ? hipEventRecord(p->events[x.ev], x.stream) : hipSuccess;
    default:
      return hipStreamWaitEvent(x.stream, p->events[x.ev], 0);
  }
}

// One lane of a multi-lane replay: the entries of one stream, in order. An event entry first
// waits (host-side) until the previous entry on its event -- on another lane -- has been issued
// in this replay, so every event sees its records and waits in the recorded order (a wait never
// observes a record of a later step: that could order a stream after its own future work).
static void run_lane(Plan* p, int lane, int begin, int end, uint64_t epoch) {
  for (int i = begin; i < end; ++i) {
    const PlanEntry& x = p->e[i];
    if (x.lane != lane) continue;
    if (x.kind != PlanEntry::LAUNCH && x.prev_ev >= begin && p->e[x.prev_ev].lane != lane) {
      while (p->issued[x.prev_ev].load(std::memory_order_acquire) != epoch) {
        if (p->err.load(std::memory_order_relaxed) != 0) return;
        _mm_pause();
      }
    }
    const hipError_t rc = issue(p, x);
    if (rc != hipSuccess) {
      int z = 0;
      p->err.compare_exchange_strong(z, (int)rc);
      return;
    }
    if (x.kind != PlanEntry::LAUNCH) p->issued[i].store(epoch, std::memory_order_release);
  }
}

static void worker_main(Plan* p, int lane, uint64_t seen) {
  (void)hipSetDevice(p->device);
  for (;;) {
    int b, e;
    uint64_t ep;
    {
      std::unique_lock<std::mutex> g(p->mu);
      p->cv_go.wait(g, [&] { return p->stop || p->job != seen; });
      if (p->stop) return;
      seen = p->job;
      b = p->job_begin;
      e = p->job_end;
      ep = p->epoch;
      if (lane >= p->job_lanes) b = e;  // this range has fewer streams
    }
    if (b < e) run_lane(p, lane, b, e, ep);
    {
      std::lock_guard<std::mutex> g(p->mu);
      ++p->done;
    }
    p->cv_done.notify_one();
  }
}

}  // namespace drn

using drn::Plan;
using drn::PlanEntry;

DRN_API void* drn_plan_create() { return new Plan(); }

DRN_API void drn_plan_destroy(void* p) { delete static_cast<Plan*>(p); }

// Start / stop recording the calling thread's launches into p (one plan per thread at a time).
DRN_API int drn_plan_record_begin(void* p) {
  if (p == nullptr || drn::g_plan_rec != nullptr) return (int)hipErrorInvalidValue;
  drn::g_plan_rec = static_cast<Plan*>(p);
  (void)hipGetDevice(&drn::g_plan_rec->device);
  return 0;
}

DRN_API int drn_plan_record_end() {
  if (drn::g_plan_rec == nullptr) return (int)hipErrorInvalidValue;
  drn::g_plan_rec = nullptr;
  return 0;
}

// A new (timing-disabled) event of the plan; returns its index.
DRN_API int drn_plan_new_event(void* pv) {
  Plan* p = static_cast<Plan*>(pv);
  hipEvent_t ev;
  const hipError_t rc = hipEventCreateWithFlags(&ev, hipEventDisableTiming);
  if (rc != hipSuccess) return -(int)rc;
  p->events.push_back(ev);
  p->last_ev_entry.push_back(-1);
  return (int)p->events.size() - 1;
}

DRN_API int drn_plan_event_record(void* pv, int ev, hipStream_t s) {
  Plan* p = static_cast<Plan*>(pv);
  if (ev < 0 || ev >= (int)p->events.size()) return (int)hipErrorInvalidValue;
  PlanEntry x;
  x.kind = PlanEntry::RECORD;
  x.ev = ev;
  x.stream = s;
  add_event_entry(p, x);
  return 0;
}

DRN_API int drn_plan_stream_wait(void* pv, hipStream_t s, int ev) {
  Plan* p = static_cast<Plan*>(pv);
  if (ev < 0 || ev >= (int)p->events.size()) return (int)hipErrorInvalidValue;
  PlanEntry x;
  x.kind = PlanEntry::WAIT;
  x.ev = ev;
  x.stream = s;
  add_event_entry(p, x);
  return 0;
}

// Entries recorded so far (segment boundaries are entry positions).
DRN_API int drn_plan_size(void* pv) { return (int)static_cast<Plan*>(pv)->e.size(); }

DRN_API int drn_plan_launches(void* pv) { return static_cast<Plan*>(pv)->launches; }

// Host threads issuing a replay (1: the calling thread issues every entry in recorded order;
// n > 1: one thread per stream of the replayed range, up to n -- the streams' launches are
// enqueued concurrently, cross-stream events in recorded order; ranges with more streams than
// threads replay serially).
DRN_API int drn_plan_set_threads(void* pv, int n) {
  Plan* p = static_cast<Plan*>(pv);
  if (n < 1 || n > 8) return (int)hipErrorInvalidValue;
  p->threads = n;
  return 0;
}

// Streams (lanes) the plan's entries use.
DRN_API int drn_plan_lanes(void* pv) { return (int)static_cast<Plan*>(pv)->lanes.size(); }

// Entries of one kind (0 launch, 1 event record, 2 stream wait).
DRN_API int drn_plan_count(void* pv, int kind) {
  int n = 0;
  for (const auto& x : static_cast<Plan*>(pv)->e) n += x.kind == kind;
  return n;
}

static void analyze(Plan* p) {
  if (p->analyzed_n == p->e.size()) return;
  p->ev_waited.assign(p->events.size(), 0);
  for (const auto& x : p->e)
    if (x.kind == PlanEntry::WAIT) p->ev_waited[x.ev] = 1;
  p->analyzed_n = p->e.size();
}

// Event records replay actually issues (records of events no entry waits on are skipped).
DRN_API int drn_plan_live_records(void* pv) {
  Plan* p = static_cast<Plan*>(pv);
  analyze(p);
  int n = 0;
  for (const auto& x : p->e) n += x.kind == PlanEntry::RECORD && p->ev_waited[x.ev];
  return n;
}

static int replay_serial(Plan* p, int begin, int end) {
  for (int i = begin; i < end; ++i) {
    const hipError_t rc = drn::issue(p, p->e[i]);
    if (rc != hipSuccess) return (int)rc;
  }
  return 0;
}

// Re-issue entries [begin, end); returns the first HIP error.
DRN_API int drn_plan_replay(void* pv, int begin, int end) {
  Plan* p = static_cast<Plan*>(pv);
  if (begin < 0 || end > (int)p->e.size() || begin > end) return (int)hipErrorInvalidValue;
  analyze(p);
  int nl = 0;
  for (int i = begin; i < end; ++i) nl = std::max(nl, p->e[i].lane + 1);
  bool null_stream = false;  // the legacy default stream orders against others by host order
  for (int l = 0; l < nl; ++l) null_stream |= p->lanes[l] == nullptr;
  if (p->threads <= 1 || nl <= 1 || nl > p->threads || null_stream) return replay_serial(p, begin, end);
  if (p->issued_n != p->e.size()) {
    p->issued.reset(new std::atomic<uint64_t>[p->e.size()]);
    for (size_t i = 0; i < p->e.size(); ++i) p->issued[i].store(0);
    p->issued_n = p->e.size();
  }
  while ((int)p->workers.size() < nl - 1)  // (a new worker starts at the current generation)
    p->workers.emplace_back(drn::worker_main, p, (int)p->workers.size() + 1, p->job);
  p->err.store(0);
  {
    std::lock_guard<std::mutex> g(p->mu);
    ++p->epoch;
    p->job_begin = begin;
    p->job_end = end;
    p->job_lanes = nl;
    p->done = 0;
    ++p->job;
  }
  p->cv_go.notify_all();
  drn::run_lane(p, 0, begin, end, p->epoch);
  {
    std::unique_lock<std::mutex> g(p->mu);
    p->cv_done.wait(g, [&] { return p->done == (int)p->workers.size(); });
  }
  return p->err.load();
}
