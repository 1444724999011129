// WorkQueue: a fixed pool of worker threads (reference common/include/workqueue.h:20-73, an IOCP
// pool with numWorkerThreads / numConcurrentThreads).  Used by the vertex runtime for
// asynchronous channel I/O: reading input channel files and writing output channels overlap
// with operator execution on the Python side (the GIL is released while native I/O runs).
#pragma once
#include <atomic>
#include <condition_variable>
#include <cstdint>
#include <deque>
#include <functional>
#include <memory>
#include <mutex>
#include <string>
#include <thread>
#include <vector>

namespace dryad {

class WorkQueue {
 public:
  explicit WorkQueue(int threads);
  ~WorkQueue();
  void submit(std::function<void()> fn);
  void drain();   // wait until every submitted item has run
  int threads() const { return (int)pool_.size(); }

 private:
  void loop();
  std::vector<std::thread> pool_;
  std::deque<std::function<void()>> q_;
  std::mutex mu_;
  std::condition_variable cv_, idle_cv_;
  int inflight_ = 0;
  bool stop_ = false;
};

// A batch of file reads issued on a WorkQueue; results are fetched by index.
struct ReadBatch {
  std::vector<std::string> paths;
  std::vector<std::string> data;
  std::vector<std::string> errors;
  std::vector<uint8_t> done;
  std::mutex mu;
  std::condition_variable cv;
  int remaining = 0;
};

std::shared_ptr<ReadBatch> read_files_async(WorkQueue& q, const std::vector<std::string>& paths);
void wait_read(ReadBatch& b, size_t i);

// Write `data` to `path` atomically: write to path + ".partial", fsync optional, rename.
void write_file_atomic(const std::string& path, const uint8_t* data, size_t n);

}  // namespace dryad
