#include "workqueue.h"

#include <cstdio>
#include <stdexcept>

namespace dryad {

WorkQueue::WorkQueue(int threads) {
  if (threads < 1) threads = 1;
  for (int i = 0; i < threads; ++i) pool_.emplace_back([this] { loop(); });
}

WorkQueue::~WorkQueue() {
  {
    std::lock_guard<std::mutex> g(mu_);
    stop_ = true;
  }
  cv_.notify_all();
  for (auto& t : pool_) t.join();
}

void WorkQueue::submit(std::function<void()> fn) {
  {
    std::lock_guard<std::mutex> g(mu_);
    q_.push_back(std::move(fn));
    ++inflight_;
  }
  cv_.notify_one();
}

void WorkQueue::drain() {
  std::unique_lock<std::mutex> g(mu_);
  idle_cv_.wait(g, [this] { return inflight_ == 0; });
}

void WorkQueue::loop() {
  for (;;) {
    std::function<void()> fn;
    {
      std::unique_lock<std::mutex> g(mu_);
      cv_.wait(g, [this] { return stop_ || !q_.empty(); });
      if (stop_ && q_.empty()) return;
      fn = std::move(q_.front());
      q_.pop_front();
    }
    try {
      fn();
    } catch (...) {
    }
    {
      std::lock_guard<std::mutex> g(mu_);
      if (--inflight_ == 0) idle_cv_.notify_all();
    }
  }
}

static std::string slurp(const std::string& path) {
  FILE* f = fopen(path.c_str(), "rb");
  if (!f) throw std::runtime_error("cannot open " + path);
  std::string out;
  char buf[1 << 16];
  size_t n;
  while ((n = fread(buf, 1, sizeof buf, f)) > 0) out.append(buf, n);
  const bool err = ferror(f);
  fclose(f);
  if (err) throw std::runtime_error("read error on " + path);
  return out;
}

std::shared_ptr<ReadBatch> read_files_async(WorkQueue& q, const std::vector<std::string>& paths) {
  auto b = std::make_shared<ReadBatch>();
  b->paths = paths;
  b->data.resize(paths.size());
  b->errors.resize(paths.size());
  b->done.assign(paths.size(), 0);
  b->remaining = (int)paths.size();
  for (size_t i = 0; i < paths.size(); ++i) {
    q.submit([b, i] {
      std::string d, e;
      try {
        d = slurp(b->paths[i]);
      } catch (const std::exception& ex) {
        e = ex.what();
      }
      std::lock_guard<std::mutex> g(b->mu);
      b->data[i] = std::move(d);
      b->errors[i] = std::move(e);
      b->done[i] = 1;
      b->remaining--;
      b->cv.notify_all();
    });
  }
  return b;
}

void wait_read(ReadBatch& b, size_t i) {
  std::unique_lock<std::mutex> g(b.mu);
  b.cv.wait(g, [&] { return b.done[i] != 0; });
}

void write_file_atomic(const std::string& path, const uint8_t* data, size_t n) {
  const std::string tmp = path + ".partial";
  FILE* f = fopen(tmp.c_str(), "wb");
  if (!f) throw std::runtime_error("cannot create " + tmp);
  size_t w = n ? fwrite(data, 1, n, f) : 0;
  const bool err = (w != n) || ferror(f);
  fclose(f);
  if (err) {
    remove(tmp.c_str());
    throw std::runtime_error("write error on " + tmp);
  }
  if (rename(tmp.c_str(), path.c_str()) != 0) throw std::runtime_error("rename failed for " + path);
}

}  // namespace dryad
