// Communication watchdog (watchdog.hpp).
#include "heat2d/watchdog.hpp"

#include <cstdlib>

namespace heat2d {

Watchdog::Watchdog(double timeout_s, double period_s, PollFn poll, FireFn on_fire)
    : timeout_(timeout_s), period_(period_s), poll_(std::move(poll)), fire_(std::move(on_fire)) {
  if (timeout_ > 0) th_ = std::thread(&Watchdog::loop, this);
}

Watchdog::~Watchdog() {
  {
    std::lock_guard<std::mutex> g(mu_);
    stop_ = true;
  }
  cv_.notify_all();
  if (th_.joinable()) th_.join();
}

std::string Watchdog::reason() const {
  std::lock_guard<std::mutex> g(mu_);
  return reason_;
}

double Watchdog::env_timeout(double dflt) {
  if (const char* e = std::getenv("HEAT2D_COMM_TIMEOUT")) return std::atof(e);
  return dflt;
}

void Watchdog::loop() {
  using clk = std::chrono::steady_clock;
  auto last = clk::now();  // last progress (or start of the current wait)
  bool waiting = false;
  std::unique_lock<std::mutex> lk(mu_);
  while (!stop_) {
    cv_.wait_for(lk, std::chrono::duration<double>(period_));
    if (stop_) break;
    lk.unlock();
    std::string detail;
    const Status st = poll_(&detail);
    const auto now = clk::now();
    std::string why;
    if (st == Error) {
      why = "communication error: " + detail;
    } else if (st == Pending) {
      if (!waiting) {
        waiting = true;
        last = now;
      }
      const double idle = std::chrono::duration<double>(now - last).count();
      if (idle > timeout_)
        why = "no halo exchange completed for " + std::to_string((int)idle) + " s (timeout " +
              std::to_string(timeout_) + " s; HEAT2D_COMM_TIMEOUT): a peer rank is dead or hung" +
              (detail.empty() ? "" : " — " + detail);
    } else {
      waiting = st == Progress;
      last = now;
    }
    if (!why.empty()) {
      {
        std::lock_guard<std::mutex> g(mu_);
        reason_ = why;
      }
      fired_ = true;
      fire_(why);
      return;
    }
    lk.lock();
  }
}

}  // namespace heat2d
