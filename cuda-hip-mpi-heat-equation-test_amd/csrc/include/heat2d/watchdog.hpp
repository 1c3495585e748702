// Hang / failure watchdog for the communication path.
//
// The reference has none: a dead MPI peer leaves every other rank blocked in
// MPI_Sendrecv forever (fortran/hip/heat.F90:212-213). Here a background
// thread polls a progress source; when work is outstanding and nothing has
// completed for `timeout_s`, or the fabric reports an error, it fires once:
// calls on_fire(reason) (RCCL: ncclCommAbort, which makes the blocked RCCL
// kernels and host calls return) so that the rank fails loudly — with its
// rank, step and reason — instead of hanging.
#pragma once

#include <atomic>
#include <chrono>
#include <condition_variable>
#include <functional>
#include <mutex>
#include <string>
#include <thread>

namespace heat2d {

class Watchdog {
 public:
  enum Status { Idle = 0, Progress = 1, Pending = 2, Error = 3 };
  // poll(&detail) -> Idle (nothing outstanding), Progress (something completed
  // since the last poll), Pending (outstanding, nothing completed) or Error.
  using PollFn = std::function<Status(std::string*)>;
  using FireFn = std::function<void(const std::string&)>;

  Watchdog(double timeout_s, double period_s, PollFn poll, FireFn on_fire);
  ~Watchdog();
  Watchdog(const Watchdog&) = delete;
  Watchdog& operator=(const Watchdog&) = delete;

  bool fired() const { return fired_.load(); }
  std::string reason() const;
  double timeout_s() const { return timeout_; }

  // HEAT2D_COMM_TIMEOUT (seconds; 0 disables), default `dflt`
  static double env_timeout(double dflt);

 private:
  void loop();
  double timeout_, period_;
  PollFn poll_;
  FireFn fire_;
  std::atomic<bool> fired_{false};
  std::atomic<bool> stop_{false};
  mutable std::mutex mu_;
  std::condition_variable cv_;
  std::string reason_;
  std::thread th_;
};

}  // namespace heat2d
