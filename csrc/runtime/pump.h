// Event pump of the job manager (SURVEY G-10).
//
// Reference: DrMessagePump (GraphManager/kernel/DrMessagePump.h:20-295): listeners receive
// messages posted from any thread, immediately or after a delay (timers), and the job manager's
// state machine only ever runs in response to one.  Here the state machine (JobGraph) runs on the
// job manager's thread; everything that can change it - a vertex result arriving from a worker,
// a duplicate-check timer, a user cancel - is a message.  The manager blocks in wait() with the
// GIL released until the next message or the earliest timer is due: no polling interval, no
// sleep.
//
// A message is (kind, payload): small integers; the Python side keeps any object the payload
// refers to.  Delivery order: due timers by deadline then post order, immediate messages in post
// order.  close() wakes every waiter with no messages and makes later posts no-ops.
#pragma once

#include <chrono>
#include <condition_variable>
#include <cstdint>
#include <deque>
#include <mutex>
#include <queue>
#include <utility>
#include <vector>

namespace dryad {

class MessagePump {
 public:
  using Clock = std::chrono::steady_clock;
  struct Message {
    int32_t kind;
    int64_t payload;
  };

  void post(int32_t kind, int64_t payload) {
    std::lock_guard<std::mutex> lk(m_);
    if (closed_) return;
    q_.push_back({kind, payload});
    ++posted_;
    cv_.notify_one();
  }

  // Deliver (kind, payload) once delay_ms milliseconds have passed.
  void post_after(int64_t delay_ms, int32_t kind, int64_t payload) {
    std::lock_guard<std::mutex> lk(m_);
    if (closed_) return;
    timers_.push(Timer{Clock::now() + std::chrono::milliseconds(delay_ms < 0 ? 0 : delay_ms), seq_++, {kind, payload}});
    ++posted_;
    cv_.notify_one();
  }

  // Every message that is due, blocking until there is one: timeout_ms < 0 waits until a message
  // (or close()), 0 only collects what is due.  Returns an empty list on timeout or close.
  std::vector<Message> wait(int64_t timeout_ms) {
    std::unique_lock<std::mutex> lk(m_);
    const bool forever = timeout_ms < 0;
    const auto limit = Clock::now() + std::chrono::milliseconds(forever ? 0 : timeout_ms);
    for (;;) {
      std::vector<Message> out;
      const auto now = Clock::now();
      while (!timers_.empty() && timers_.top().due <= now) {
        out.push_back(timers_.top().msg);
        timers_.pop();
      }
      while (!q_.empty()) {
        out.push_back(q_.front());
        q_.pop_front();
      }
      if (!out.empty() || closed_) {
        delivered_ += out.size();
        return out;
      }
      if (!forever && now >= limit) return out;
      auto until = forever ? Clock::time_point::max() : limit;
      if (!timers_.empty() && timers_.top().due < until) until = timers_.top().due;
      if (until == Clock::time_point::max()) {
        cv_.wait(lk);
      } else {
        // timed wait against the system clock (pthread_cond_timedwait): the steady-clock overload
        // goes through pthread_cond_clockwait, which ThreadSanitizer (GCC 11) does not intercept;
        // the loop re-checks every deadline on the steady clock
        cv_.wait_until(lk, std::chrono::system_clock::now() +
                               std::chrono::duration_cast<std::chrono::system_clock::duration>(until - Clock::now()));
      }
    }
  }

  void close() {
    std::lock_guard<std::mutex> lk(m_);
    closed_ = true;
    cv_.notify_all();
  }

  size_t pending() const {
    std::lock_guard<std::mutex> lk(m_);
    return q_.size() + timers_.size();
  }
  uint64_t posted() const {
    std::lock_guard<std::mutex> lk(m_);
    return posted_;
  }
  uint64_t delivered() const {
    std::lock_guard<std::mutex> lk(m_);
    return delivered_;
  }

 private:
  struct Timer {
    Clock::time_point due;
    uint64_t seq;
    Message msg;
    bool operator>(const Timer& o) const { return due != o.due ? due > o.due : seq > o.seq; }
  };
  mutable std::mutex m_;
  std::condition_variable cv_;
  std::deque<Message> q_;
  std::priority_queue<Timer, std::vector<Timer>, std::greater<Timer>> timers_;
  uint64_t seq_ = 0, posted_ = 0, delivered_ = 0;
  bool closed_ = false;
};

}  // namespace dryad
