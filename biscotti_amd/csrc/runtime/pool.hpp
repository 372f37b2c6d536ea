// Persistent host thread pool and asynchronous job dispatcher of the runtime (used by the pybind11 bindings for
// the VRF, Schnorr and KZG batches).  Header-only so the native self-test can stress them under ThreadSanitizer
// (python -m biscotti_amd._build --tsan; csrc/selftest/selftest.cpp test_pool).
#pragma once
#include <pthread.h>

#include <algorithm>
#include <atomic>
#include <condition_variable>
#include <deque>
#include <functional>
#include <mutex>
#include <thread>
#include <vector>

namespace bsc {

// Persistent worker pool for host crypto of many local peers (VRF proofs, Schnorr signatures):
// threads are created once, each call hands out indices through an atomic counter.
class Pool {
  // Several jobs may run at once (background VRF proofs, round-wide Schnorr batches, the main
  // thread's calls): every run() registers its job, works on it itself, and the persistent
  // workers help whichever registered job still has items and is below its thread cap.
  struct Job {
    const std::function<void(size_t)>* f;
    size_t n;
    int cap;                          // pool workers allowed on this job (threads - 1)
    std::atomic<size_t> next{0};
    int active = 0;                   // workers inside the job (guarded by m_)
  };

 public:
  void run(size_t n, int threads, const std::function<void(size_t)>& f) {
    if (threads <= 1 || n <= 1) {
      for (size_t i = 0; i < n; ++i) f(i);
      return;
    }
    Job job;
    job.f = &f;
    job.n = n;
    job.cap = std::min<int>(threads, int(n)) - 1;
    {
      std::lock_guard<std::mutex> lk(m_);
      ensure(threads - 1);
      jobs_.push_back(&job);
    }
    cv_.notify_all();
    for (size_t i; (i = job.next.fetch_add(1)) < n;) f(i);
    std::unique_lock<std::mutex> lk(m_);
    jobs_.erase(std::find(jobs_.begin(), jobs_.end(), &job));  // no new helper can join
    done_cv_.wait(lk, [&] { return job.active == 0; });       // helpers still inside finish
  }
  ~Pool() {
    {
      std::lock_guard<std::mutex> lk(m_);
      stop_ = true;
    }
    cv_.notify_all();
    for (auto& t : workers_) t.join();
  }

 private:
  void ensure(int k) {  // caller holds m_
    while (int(workers_.size()) < k) workers_.emplace_back([this] { loop(); });
  }
  Job* pick() {  // caller holds m_
    for (Job* j : jobs_)
      if (j->active < j->cap && j->next.load() < j->n) return j;
    return nullptr;
  }
  void loop() {
    pthread_setname_np(pthread_self(), "bsc-pool");   // per-thread CPU attribution (utils/threadcpu.py)
    std::unique_lock<std::mutex> lk(m_);
    for (;;) {
      Job* j = nullptr;
      cv_.wait(lk, [&] { return stop_ || (j = pick()) != nullptr; });
      if (stop_) return;
      ++j->active;
      lk.unlock();
      for (size_t i; (i = j->next.fetch_add(1)) < j->n;) (*j->f)(i);
      lk.lock();
      if (--j->active == 0) done_cv_.notify_all();
    }
  }
  std::vector<std::thread> workers_;
  std::vector<Job*> jobs_;
  std::mutex m_;
  std::condition_variable cv_, done_cv_;
  bool stop_ = false;
};
inline Pool& pool() {
  static Pool* p = new Pool();  // intentionally leaked: no join at interpreter teardown
  return *p;
}
// Persistent threads for the asynchronous jobs (VRF batches, signature batches, KZG checks): a job
// is handed over through a queue instead of a fresh std::thread (~45 us of the submitting thread's
// time per creation on these hosts).  A thread is added only when every existing one is busy, so a
// job that waits on an earlier one (VrfJob::after) never waits behind work queued after it.
class Dispatcher {
 public:
  void submit(std::function<void()> f) {
    {
      std::lock_guard<std::mutex> lk(m_);
      q_.push_back(std::move(f));
      if (int(q_.size()) > idle_) std::thread([this] { loop(); }).detach();
    }
    cv_.notify_one();
  }

 private:
  void loop() {
    pthread_setname_np(pthread_self(), "bsc-job");
    std::unique_lock<std::mutex> lk(m_);
    for (;;) {
      ++idle_;
      cv_.wait(lk, [&] { return !q_.empty(); });
      --idle_;
      std::function<void()> f = std::move(q_.front());
      q_.pop_front();
      lk.unlock();
      f();
      lk.lock();
    }
  }
  std::deque<std::function<void()>> q_;
  std::mutex m_;
  std::condition_variable cv_;
  int idle_ = 0;
};
inline Dispatcher& dispatcher() {
  static Dispatcher* d = new Dispatcher();  // intentionally leaked, like the pool
  return *d;
}

template <class F>
inline void parallel_for(size_t n, int threads, F f) {
  std::function<void(size_t)> fn = f;
  pool().run(n, threads, fn);
}

}  // namespace bsc
