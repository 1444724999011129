#include "partreader.h"

#include <fcntl.h>
#include <sys/stat.h>
#include <unistd.h>

#include <cerrno>
#include <chrono>
#include <cstring>
#include <stdexcept>

namespace dryad {

ChunkReader::ChunkReader(const std::string& path, int64_t offset, int64_t length, int64_t chunk_bytes,
                         const std::vector<std::pair<uint64_t, int64_t>>& bufs, int threads) {
  if (chunk_bytes <= 0 || bufs.empty()) throw std::invalid_argument("ChunkReader: chunk size / buffers");
  for (size_t i = 0; i < bufs.size(); ++i)
    if (bufs[i].first == 0 || bufs[i].second < chunk_bytes)
      throw std::invalid_argument("ChunkReader: buffer " + std::to_string(i) + " holds " +
                                  std::to_string(bufs[i].second) + " bytes, less than a " +
                                  std::to_string(chunk_bytes) + "-byte chunk");
  fd_ = ::open(path.c_str(), O_RDONLY | O_CLOEXEC);
  if (fd_ < 0) throw std::runtime_error("ChunkReader: cannot open " + path + ": " + std::strerror(errno));
  struct stat st;
  if (::fstat(fd_, &st) != 0) {
    ::close(fd_);
    throw std::runtime_error("ChunkReader: stat " + path);
  }
  offset_ = offset < 0 ? 0 : offset;
  const int64_t avail = (int64_t)st.st_size > offset_ ? (int64_t)st.st_size - offset_ : 0;
  length_ = length < 0 || length > avail ? avail : length;
  chunk_ = chunk_bytes;
  nchunks_ = (length_ + chunk_ - 1) / chunk_;
#ifdef POSIX_FADV_SEQUENTIAL
  ::posix_fadvise(fd_, offset_, length_, POSIX_FADV_SEQUENTIAL);
#endif
  for (size_t i = 0; i < bufs.size(); ++i) {
    bufs_.push_back(reinterpret_cast<uint8_t*>(bufs[i].first));
    free_.push_back((int)i);
  }
  const int nt = threads < 1 ? 1 : threads;
  for (int i = 0; i < nt; ++i) pool_.emplace_back([this] { run(); });
}

ChunkReader::~ChunkReader() {
  stop();
  if (fd_ >= 0) ::close(fd_);
}

void ChunkReader::stop() {
  {
    std::lock_guard<std::mutex> g(mu_);
    stop_ = true;
  }
  cv_free_.notify_all();
  cv_ready_.notify_all();
  for (auto& t : pool_)
    if (t.joinable()) t.join();
  pool_.clear();
}

void ChunkReader::run() {
  for (;;) {
    int slot;
    {
      std::unique_lock<std::mutex> lk(mu_);
      cv_free_.wait(lk, [this] { return stop_ || !free_.empty() || next_chunk_.load() >= nchunks_; });
      if (stop_ || next_chunk_.load() >= nchunks_) return;
      slot = free_.front();
      free_.pop_front();
    }
    const int64_t c = next_chunk_.fetch_add(1);
    if (c >= nchunks_) {
      std::lock_guard<std::mutex> g(mu_);
      free_.push_back(slot);
      cv_free_.notify_one();
      return;
    }
    const int64_t pos = offset_ + c * chunk_;
    const int64_t want = (c + 1) * chunk_ <= length_ ? chunk_ : length_ - c * chunk_;
    int64_t got = 0;
    std::string e;
    while (got < want) {
      const ssize_t r = ::pread(fd_, bufs_[slot] + got, (size_t)(want - got), (off_t)(pos + got));
      if (r < 0) {
        if (errno == EINTR) continue;
        e = std::string("pread: ") + std::strerror(errno);
        break;
      }
      if (r == 0) {
        e = "pread: unexpected end of file";
        break;
      }
      got += r;
    }
    {
      std::lock_guard<std::mutex> g(mu_);
      if (!e.empty() && err_.empty()) err_ = e;
      ReadyChunk rc;
      rc.slot = slot;
      rc.chunk = c;
      rc.bytes = got;
      ready_.push_back(rc);
    }
    cv_ready_.notify_one();
  }
}

bool ChunkReader::next(ReadyChunk* out, int64_t timeout_ms) {
  std::unique_lock<std::mutex> lk(mu_);
  if (handed_ >= nchunks_) return false;
  auto ok = [this] { return !ready_.empty() || !err_.empty() || stop_; };
  if (timeout_ms < 0) {
    cv_ready_.wait(lk, ok);
  } else if (!cv_ready_.wait_for(lk, std::chrono::milliseconds(timeout_ms), ok)) {
    out->slot = -1;
    return true;             // timed out: nothing ready yet (slot = -1)
  }
  if (!err_.empty() || ready_.empty()) return false;
  *out = ready_.front();
  ready_.pop_front();
  ++handed_;
  return true;
}

void ChunkReader::release(int slot) {
  {
    std::lock_guard<std::mutex> g(mu_);
    if (slot < 0 || slot >= (int)bufs_.size()) return;
    free_.push_back(slot);
  }
  cv_free_.notify_one();
}

std::string ChunkReader::error() {
  std::lock_guard<std::mutex> g(mu_);
  return err_;
}

}  // namespace dryad
