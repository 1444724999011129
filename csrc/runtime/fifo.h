// Bounded in-process FIFO channel of byte blocks (SURVEY C-5).
//
// Reference: the FIFO channel that joins the vertices of a subgraph vertex running in one process
// (DryadVertex/VertexHost/system/channel/include/channelfifo.h:27-241, channelfifo.cpp; used by
// DryadSubGraphVertex, subgraphvertex.h:20-202).  A writer blocks while the queued bytes exceed
// the capacity (back pressure), a reader blocks while the queue is empty; close() by the writer
// turns an empty queue into end-of-stream, abort() by either side fails both ends with the given
// error, as an upstream vertex failure does in the reference.
//
// Blocks are moved, never copied, between the two ends.  One block larger than the capacity is
// still admitted when the queue is empty (otherwise it could never pass).
#pragma once

#include <chrono>
#include <condition_variable>
#include <cstdint>
#include <deque>
#include <mutex>
#include <string>
#include <vector>

namespace dryad {

class BlockFifo {
 public:
  using Block = std::vector<uint8_t>;
  enum class Status { Ok = 0, Timeout = 1, Closed = 2, Aborted = 3 };

  explicit BlockFifo(uint64_t capacity_bytes) : cap_(capacity_bytes ? capacity_bytes : 1) {}

  // Blocks while full.  timeout_ms < 0 waits forever, 0 polls.
  Status put(Block&& b, int64_t timeout_ms) {
    std::unique_lock<std::mutex> lk(m_);
    auto room = [&] { return aborted_ || closed_ || q_.empty() || bytes_ + b.size() <= cap_; };
    if (!wait(lk, not_full_, room, timeout_ms)) return Status::Timeout;
    if (aborted_) return Status::Aborted;
    if (closed_) return Status::Closed;
    bytes_ += b.size();
    peak_ = bytes_ > peak_ ? bytes_ : peak_;
    q_.push_back(std::move(b));
    ++puts_;
    not_empty_.notify_one();
    return Status::Ok;
  }

  // Blocks while empty and open.  Closed = end of stream (queue drained).
  Status get(Block& out, int64_t timeout_ms) {
    std::unique_lock<std::mutex> lk(m_);
    auto ready = [&] { return aborted_ || closed_ || !q_.empty(); };
    if (!wait(lk, not_empty_, ready, timeout_ms)) return Status::Timeout;
    if (aborted_) return Status::Aborted;
    if (q_.empty()) return Status::Closed;
    out = std::move(q_.front());
    q_.pop_front();
    bytes_ -= out.size();
    not_full_.notify_one();
    return Status::Ok;
  }

  void close() {
    std::lock_guard<std::mutex> lk(m_);
    closed_ = true;
    not_empty_.notify_all();
    not_full_.notify_all();
  }

  void abort(const std::string& why) {
    std::lock_guard<std::mutex> lk(m_);
    if (!aborted_) error_ = why;
    aborted_ = true;
    not_empty_.notify_all();
    not_full_.notify_all();
  }

  std::string error() const { std::lock_guard<std::mutex> lk(m_); return error_; }
  uint64_t queued_bytes() const { std::lock_guard<std::mutex> lk(m_); return bytes_; }
  uint64_t queued_blocks() const { std::lock_guard<std::mutex> lk(m_); return q_.size(); }
  uint64_t peak_bytes() const { std::lock_guard<std::mutex> lk(m_); return peak_; }
  uint64_t blocks_written() const { std::lock_guard<std::mutex> lk(m_); return puts_; }
  uint64_t capacity() const { return cap_; }
  bool closed() const { std::lock_guard<std::mutex> lk(m_); return closed_; }

 private:
  template <typename Pred>
  static bool wait(std::unique_lock<std::mutex>& lk, std::condition_variable& cv, Pred pred, int64_t timeout_ms) {
    if (timeout_ms < 0) {
      cv.wait(lk, pred);
      return true;
    }
    return cv.wait_for(lk, std::chrono::milliseconds(timeout_ms), pred);
  }

  const uint64_t cap_;
  mutable std::mutex m_;
  std::condition_variable not_empty_, not_full_;
  std::deque<Block> q_;
  uint64_t bytes_ = 0, peak_ = 0, puts_ = 0;
  bool closed_ = false, aborted_ = false;
  std::string error_;
};

}  // namespace dryad
