// Graph-launch probe: n captured HIP graphs (one per stream) launched from the calling thread one after
// another, or from n pre-started host threads at once.  Returns the host span of the launches (us) and
// each launch call's duration; the caller times the GPU side.  Built by tools/ubench/Makefile into
// libgraphpar.so (ctypes, tools/graph_launch_probe.py).
#include <hip/hip_runtime.h>

#include <atomic>
#include <chrono>
#include <thread>
#include <vector>

static double now_us() {
  return std::chrono::duration<double, std::micro>(std::chrono::steady_clock::now().time_since_epoch()).count();
}

extern "C" double graphpar_launch(void** execs, void** streams, int n, int parallel, double* call_us) {
  if (!parallel) {
    const double t0 = now_us();
    for (int i = 0; i < n; ++i) {
      const double a = now_us();
      (void)hipGraphLaunch((hipGraphExec_t)execs[i], (hipStream_t)streams[i]);
      call_us[i] = now_us() - a;
    }
    return now_us() - t0;
  }
  std::atomic<int> ready{0};
  std::atomic<bool> go{false};
  std::vector<double> ends(n, 0.0);
  std::vector<std::thread> th;
  for (int i = 0; i < n; ++i)
    th.emplace_back([&, i] {
      ready.fetch_add(1);
      while (!go.load(std::memory_order_acquire)) {
      }
      const double a = now_us();
      (void)hipGraphLaunch((hipGraphExec_t)execs[i], (hipStream_t)streams[i]);
      ends[i] = now_us();
      call_us[i] = ends[i] - a;
    });
  while (ready.load() < n) {
  }
  const double t0 = now_us();
  go.store(true, std::memory_order_release);
  for (auto& t : th) t.join();
  double e = t0;
  for (double v : ends) e = v > e ? v : e;
  return e - t0;
}
