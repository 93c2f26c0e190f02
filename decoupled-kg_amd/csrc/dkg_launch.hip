// Host-side launcher of captured forward graphs on several streams at once (include/dkg.h
// "Launcher").  A hipGraphLaunch costs ~1 us of host time per kernel node plus a fixed ~9 us
// (DESIGN.md 6), and one thread launching the graphs of four streams one after the other keeps
// the last stream idle for the sum of the others' launches: a 20-forward run spent ~100 us of its
// ~335 us enqueuing.  Here every stream's graphs are launched by its own host thread (the caller
// takes stream 0), so the streams start together and the enqueue time is one stream's share.
//
// Workers are created once and wait on a generation counter: spinning (a few us to wake) while
// "armed", otherwise on a condition variable (no CPU burnt between calls).  Pure host code: no
// kernel in this translation unit.
#include <hip/hip_runtime.h>

#include <atomic>
#include <cstdarg>
#include <chrono>
#include <condition_variable>
#include <cstdio>
#include <mutex>
#include <new>
#include <thread>
#include <vector>

#include "dkg.h"
#include "dkg_kernels.h"

namespace dkg {

namespace {

int fail(int code, const char* fmt, ...) {
  char buf[256];
  va_list ap;
  va_start(ap, fmt);
  vsnprintf(buf, sizeof(buf), fmt, ap);
  va_end(ap);
  return report_error(code, buf);
}

struct Launcher {
  int nthreads = 1;  // including the caller
  std::vector<std::thread> workers;
  std::atomic<uint64_t> gen{0};
  std::atomic<int> pending{0};
  std::atomic<int> first_err{0};
  std::atomic<bool> quit{false};
  std::atomic<int64_t> spin_until_ns{0};
  std::mutex mu;
  std::condition_variable cv;
  // one dkg_launcher_graphs call at a time: the call's launch set lives in the fields below and the
  // workers' pending count is per call, so concurrent callers would overwrite each other's sets
  std::mutex call_mu;
  // the current call: stream s launches graphs[offs[s] .. offs[s+1]) on streams[s]; thread t takes the
  // streams s with s % nthreads == t
  int n_streams = 0;
  void* const* streams = nullptr;
  const int* offs = nullptr;
  void* const* graphs = nullptr;

  static int64_t now_ns() {
    return std::chrono::duration_cast<std::chrono::nanoseconds>(std::chrono::steady_clock::now().time_since_epoch())
        .count();
  }

  void run_share(int t) {
    for (int s = t; s < n_streams; s += nthreads) {
      // the stream's device current on this thread (a worker starts on device 0)
      hipDevice_t want = 0;
      int cur = -1;
      if (hipStreamGetDevice(reinterpret_cast<hipStream_t>(streams[s]), &want) == hipSuccess &&
          hipGetDevice(&cur) == hipSuccess && cur != (int)want)
        (void)hipSetDevice((int)want);
      for (int g = offs[s]; g < offs[s + 1]; ++g) {
        const hipError_t e = hipGraphLaunch(reinterpret_cast<hipGraphExec_t>(graphs[g]),
                                            reinterpret_cast<hipStream_t>(streams[s]));
        if (e != hipSuccess) {
          int zero = 0;
          first_err.compare_exchange_strong(zero, (int)e);
          return;
        }
      }
    }
  }

  void worker(int t) {
    uint64_t seen = 0;
    for (;;) {
      // spin while armed, else sleep until the generation moves
      while (gen.load(std::memory_order_acquire) == seen && !quit.load(std::memory_order_relaxed)) {
        if (now_ns() < spin_until_ns.load(std::memory_order_relaxed)) {
          __builtin_ia32_pause();
          continue;
        }
        std::unique_lock<std::mutex> lk(mu);
        cv.wait_for(lk, std::chrono::milliseconds(50), [&] {
          return gen.load(std::memory_order_acquire) != seen || quit.load(std::memory_order_relaxed) ||
                 now_ns() < spin_until_ns.load(std::memory_order_relaxed);
        });
      }
      if (quit.load(std::memory_order_relaxed)) return;
      seen = gen.load(std::memory_order_acquire);
      run_share(t);
      pending.fetch_sub(1, std::memory_order_acq_rel);
    }
  }
};

}  // namespace

}  // namespace dkg

using dkg::Launcher;

extern "C" {

int dkg_launcher_create(int threads, void** out) {
  if (!out) return dkg::fail(DKG_ERR_ARG, "NULL handle pointer");
  if (threads < 1 || threads > 64) return dkg::fail(DKG_ERR_ARG, "launcher threads=%d (1..64)", threads);
  Launcher* L = new (std::nothrow) Launcher();
  if (!L) return dkg::fail(DKG_ERR_HIP, "out of host memory");
  L->nthreads = threads;
  for (int t = 1; t < threads; ++t) L->workers.emplace_back([L, t] { L->worker(t); });
  *out = L;
  return DKG_OK;
}

int dkg_launcher_arm(void* h, double seconds) {
  Launcher* L = static_cast<Launcher*>(h);
  if (!L) return dkg::fail(DKG_ERR_ARG, "NULL launcher");
  const int64_t until = Launcher::now_ns() + (int64_t)(seconds > 0 ? seconds * 1e9 : 0);
  L->spin_until_ns.store(until, std::memory_order_relaxed);
  {
    std::lock_guard<std::mutex> lk(L->mu);
  }
  L->cv.notify_all();
  return DKG_OK;
}

int dkg_launcher_graphs(void* h, int n_streams, void* const* streams, const int* offs, void* const* graphs) {
  Launcher* L = static_cast<Launcher*>(h);
  if (!L) return dkg::fail(DKG_ERR_ARG, "NULL launcher");
  if (n_streams < 0 || (n_streams > 0 && (!streams || !offs || !graphs)))
    return dkg::fail(DKG_ERR_ARG, "bad launcher arguments");
  for (int s = 0; s < n_streams; ++s)
    if (offs[s + 1] < offs[s]) return dkg::fail(DKG_ERR_ARG, "graph offsets not increasing at stream %d", s);
  std::lock_guard<std::mutex> call(L->call_mu);
  L->n_streams = n_streams;
  L->streams = streams;
  L->offs = offs;
  L->graphs = graphs;
  L->first_err.store(0, std::memory_order_relaxed);
  const int nw = L->nthreads - 1;
  L->pending.store(nw, std::memory_order_relaxed);
  L->gen.fetch_add(1, std::memory_order_acq_rel);
  if (nw > 0 && Launcher::now_ns() >= L->spin_until_ns.load(std::memory_order_relaxed)) {
    std::lock_guard<std::mutex> lk(L->mu);
    L->cv.notify_all();
  }
  L->run_share(0);
  while (L->pending.load(std::memory_order_acquire) > 0) __builtin_ia32_pause();
  const int e = L->first_err.load(std::memory_order_relaxed);
  if (e) return dkg::fail(DKG_ERR_HIP, "hipGraphLaunch: %s", hipGetErrorString((hipError_t)e));
  return DKG_OK;
}

int dkg_launcher_destroy(void* h) {
  Launcher* L = static_cast<Launcher*>(h);
  if (!L) return DKG_OK;
  L->quit.store(true, std::memory_order_relaxed);
  {
    std::lock_guard<std::mutex> lk(L->mu);
  }
  L->cv.notify_all();
  for (auto& t : L->workers) t.join();
  delete L;
  return DKG_OK;
}

}  // extern "C"
