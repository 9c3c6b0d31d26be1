// util.cc -- worker threads standing in for DPDK lcores (rte_eal_remote_launch /
// rte_eal_wait_lcore, reference src/include/util.h:216-236).
#include "bitar/util.h"

#include <cerrno>
#include <condition_variable>
#include <map>
#include <mutex>
#include <thread>

namespace bitar {

namespace {

class Worker {
 public:
  Worker() : thread_([this] { Run(); }) {}
  ~Worker() {
    {
      std::lock_guard<std::mutex> lock(mu_);
      stop_ = true;
    }
    cv_.notify_all();
    thread_.join();
  }

  int Launch(internal::LcoreFunction fn, void* arg) {
    std::lock_guard<std::mutex> lock(mu_);
    if (fn_ != nullptr || running_) return -EBUSY;
    fn_ = fn;
    arg_ = arg;
    cv_.notify_all();
    return 0;
  }

  int Wait() {
    std::unique_lock<std::mutex> lock(mu_);
    done_cv_.wait(lock, [this] { return fn_ == nullptr && !running_; });
    const int r = result_;
    result_ = 0;
    return r;
  }

 private:
  void Run() {
    std::unique_lock<std::mutex> lock(mu_);
    for (;;) {
      cv_.wait(lock, [this] { return stop_ || fn_ != nullptr; });
      if (stop_ && fn_ == nullptr) return;
      auto fn = fn_;
      auto* arg = arg_;
      running_ = true;
      lock.unlock();
      const int r = fn(arg);
      lock.lock();
      result_ = r;
      running_ = false;
      fn_ = nullptr;
      done_cv_.notify_all();
    }
  }

  std::mutex mu_;
  std::condition_variable cv_, done_cv_;
  internal::LcoreFunction fn_ = nullptr;
  void* arg_ = nullptr;
  bool running_ = false;
  bool stop_ = false;
  int result_ = 0;
  std::thread thread_;
};

std::mutex g_mu;
std::map<std::uint32_t, std::unique_ptr<Worker>>& Workers() {
  static std::map<std::uint32_t, std::unique_ptr<Worker>> w;
  return w;
}

Worker* Get(std::uint32_t lcore_id) {
  std::lock_guard<std::mutex> lock(g_mu);
  auto& w = Workers()[lcore_id];
  if (!w) w = std::make_unique<Worker>();
  return w.get();
}

}  // namespace

namespace internal {

int RemoteLaunch(LcoreFunction fn, void* arg, std::uint32_t lcore_id) {
  return Get(lcore_id)->Launch(fn, arg);
}

}  // namespace internal

int WaitLcore(std::uint32_t lcore_id) { return Get(lcore_id)->Wait(); }

}  // namespace bitar
