// host_threads.h -- the host setup's fork-join helpers (nested dissection,
// tile plan, gather plan).  A process-wide budget of worker threads: the CPUs
// this process may run on, capped by ARSLAM_HOST_THREADS, else
// OMP_NUM_THREADS (the GPU box grants one GPU 16 of the node's cores and says
// so there), else 16.  A fork that finds no thread left runs inline, so
// nested forks never oversubscribe and every result is the one the serial
// order gives (callers combine the branches' outputs in a fixed order).
#pragma once

#include <sched.h>

#include <algorithm>
#include <atomic>
#include <cstdlib>
#include <exception>
#include <mutex>
#include <thread>
#include <vector>

namespace arslam {

inline int host_thread_cap() {
  static const int cap = [] {
    int n = 0;
    cpu_set_t set;
    if (sched_getaffinity(0, sizeof(set), &set) == 0) n = CPU_COUNT(&set);
    if (n <= 0) n = (int)std::max(1u, std::thread::hardware_concurrency());
    int lim = 16;
    for (const char *env : {"ARSLAM_HOST_THREADS", "OMP_NUM_THREADS"})
      if (const char *v = std::getenv(env)) {
        if (std::atoi(v) > 0) { lim = std::atoi(v); break; }
      }
    return std::max(1, std::min(n, lim));
  }();
  return cap;
}

// extra threads available beyond the caller's
inline std::atomic<int> &host_thread_pool() {
  static std::atomic<int> avail{host_thread_cap() - 1};
  return avail;
}

inline bool host_thread_take() {
  std::atomic<int> &a = host_thread_pool();
  int v = a.load(std::memory_order_relaxed);
  while (v > 0)
    if (a.compare_exchange_weak(v, v - 1, std::memory_order_acq_rel)) return true;
  return false;
}

inline void host_thread_give() { host_thread_pool().fetch_add(1, std::memory_order_acq_rel); }

// The first exception thrown by any branch of a fork (bad_alloc on a large
// graph, an ApiError), rethrown on the calling thread once every thread has
// joined -- an exception must not escape a std::thread (std::terminate), so
// it reaches the C-ABI's guard as an error code instead.
struct HostForkError {
  std::mutex m;
  std::exception_ptr e;
  template <class F>
  void run(F &&f) {
    try {
      f();
    } catch (...) {
      std::lock_guard<std::mutex> g(m);
      if (!e) e = std::current_exception();
    }
  }
  void rethrow() {
    if (e) std::rethrow_exception(e);
  }
};

// fn(i) for i in [0, n): on up to n threads (the caller's included) as the
// budget allows, each index run exactly once; blocks until all are done
template <class F>
void host_parallel_for(int n, F &&fn) {
  if (n <= 0) return;
  std::atomic<int> next{0};
  HostForkError err;
  auto work = [&] {
    err.run([&] {
      for (int i; (i = next.fetch_add(1, std::memory_order_relaxed)) < n;) fn(i);
    });
  };
  std::vector<std::thread> ts;
  for (int k = 1; k < n && host_thread_take(); ++k) ts.emplace_back(work);
  work();
  for (auto &t : ts) {
    t.join();
    host_thread_give();
  }
  err.rethrow();
}

// a() and b() concurrently when a thread is free (a on the new one), else in turn
template <class A, class B>
void host_fork2(bool worth_it, A &&a, B &&b) {
  if (worth_it && host_thread_take()) {
    HostForkError err;
    std::thread t([&] { err.run(a); });
    err.run(b);
    t.join();
    host_thread_give();
    err.rethrow();
  } else {
    a();
    b();
  }
}

}  // namespace arslam
