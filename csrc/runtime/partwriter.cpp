#include "partwriter.h"

#include <fcntl.h>
#include <sys/mman.h>
#include <sys/stat.h>
#include <unistd.h>

#include <cerrno>
#include <cstring>
#include <stdexcept>

namespace dryad {

#ifndef MADV_POPULATE_WRITE
#define MADV_POPULATE_WRITE 23
#endif

ChunkWriter::ChunkWriter(const std::string& path, const std::vector<uint64_t>& buf_ptrs, int threads,
                         int64_t extend_bytes, bool mapped)
    : extend_(extend_bytes > 0 ? extend_bytes : (256ll << 20)), mapped_(mapped) {
  if (buf_ptrs.empty()) throw std::invalid_argument("ChunkWriter: no buffers");
  paths_.push_back(path);
  for (size_t i = 0; i < buf_ptrs.size(); ++i) bufs_.push_back(reinterpret_cast<uint8_t*>(buf_ptrs[i]));
  start(threads);
}

ChunkWriter::ChunkWriter(const std::vector<std::string>& paths, const std::vector<uint64_t>& buf_ptrs, int threads,
                         int64_t extend_bytes, bool reuse)
    : extend_(extend_bytes > 0 ? extend_bytes : (256ll << 20)), reuse_(reuse) {
  if (buf_ptrs.empty()) throw std::invalid_argument("ChunkWriter: no buffers");
  if (paths.empty()) throw std::invalid_argument("ChunkWriter: no files");
  paths_ = paths;
  for (size_t i = 0; i < buf_ptrs.size(); ++i) bufs_.push_back(reinterpret_cast<uint8_t*>(buf_ptrs[i]));
  start(threads);
}

void ChunkWriter::start(int threads) {
  for (const auto& p : paths_) {
    // reuse_: an existing file (a recycled part of a replaced table) is overwritten in place, its
    // blocks and page-cache pages kept; finish() cuts it to the new size
    const int fd = ::open(p.c_str(), O_RDWR | O_CREAT | (reuse_ ? 0 : O_TRUNC) | O_CLOEXEC, 0644);
    if (fd < 0) {
      const std::string e = std::strerror(errno);
      for (int f : fds_) ::close(f);
      fds_.clear();
      throw std::runtime_error("ChunkWriter: cannot create " + p + ": " + e);
    }
    fds_.push_back(fd);
    off_t have = 0;
    if (reuse_) {
      struct stat st;
      if (::fstat(fd, &st) == 0) have = st.st_size;
    }
    allocated_.push_back((int64_t)have);
  }
  for (size_t i = 0; i < bufs_.size(); ++i) free_.push_back((int)i);
  const int nt = threads < 1 ? 1 : threads;
  for (int i = 0; i < nt; ++i) pool_.emplace_back([this] { run(); });
}

ChunkWriter::~ChunkWriter() {
  abort();
}

void ChunkWriter::abort() {
  {
    std::lock_guard<std::mutex> g(mu_);
    stop_ = true;
  }
  cv_job_.notify_all();
  cv_free_.notify_all();
  cv_idle_.notify_all();
  for (auto& t : pool_)
    if (t.joinable()) t.join();
  pool_.clear();
  for (int& fd : fds_)
    if (fd >= 0) {
      ::close(fd);
      fd = -1;
    }
}

// Reserve file blocks ahead of the writes (one metadata update per `extend` bytes instead of one
// per write); a file system without fallocate just skips it.  Mapped writes need the file to
// reach `end` before the mapping is touched, so there a failed fallocate becomes an ftruncate.
bool ChunkWriter::extend_to(int file, int64_t end) {
  std::lock_guard<std::mutex> g(ext_mu_);
  int64_t& allocated = allocated_[file];
  if (end <= allocated) return true;
  const int fd = fds_[file];
  const int64_t target = ((end + extend_ - 1) / extend_) * extend_;
  if (::posix_fallocate(fd, allocated, target - allocated) == 0) allocated = target;
  else if (!mapped_) allocated = end;         // not supported here: plain extending writes
  else if (::ftruncate(fd, (off_t)target) == 0) allocated = target;
  else return false;
  return true;
}

// One job through a MAP_SHARED window of the file: buffered pwrite()s to one file serialise on
// its inode lock (one thread copies into the page cache at a time, ~11-12 GB/s on the MI355X
// box), while page faults on distinct pages of a shared mapping run in parallel, so every writer
// thread copies at once.  Pages are pre-faulted writable in one call per job.  False when the
// window cannot be mapped (the caller then pwrite()s).
bool ChunkWriter::write_mapped(const Job& j) {
  const int64_t page = 4096, lo = j.off & ~(page - 1), len = j.off + j.bytes - lo;
  void* m = ::mmap(nullptr, (size_t)len, PROT_READ | PROT_WRITE, MAP_SHARED, fds_[j.file], (off_t)lo);
  if (m == MAP_FAILED) return false;
  ::madvise(m, (size_t)len, MADV_POPULATE_WRITE);           // best effort (kernels >= 5.14)
  std::memcpy(static_cast<uint8_t*>(m) + (j.off - lo), bufs_[j.slot], (size_t)j.bytes);
  ::munmap(m, (size_t)len);
  return true;
}

int ChunkWriter::acquire() {
  std::unique_lock<std::mutex> lk(mu_);
  cv_free_.wait(lk, [this] { return stop_ || !free_.empty() || !err_.empty(); });
  if (stop_ || !err_.empty()) return -1;
  const int s = free_.front();
  free_.pop_front();
  return s;
}

void ChunkWriter::submit(int slot, int64_t offset, int64_t bytes, int file) {
  if (file < 0 || file >= (int)fds_.size()) throw std::out_of_range("ChunkWriter: no such file");
  {
    std::lock_guard<std::mutex> g(mu_);
    jobs_.push_back(Job{slot, offset, bytes, file});
  }
  cv_job_.notify_one();
}

void ChunkWriter::run() {
  for (;;) {
    Job j;
    {
      std::unique_lock<std::mutex> lk(mu_);
      cv_job_.wait(lk, [this] { return stop_ || !jobs_.empty(); });
      if (jobs_.empty()) return;                // stop_ with nothing queued
      j = jobs_.front();
      jobs_.pop_front();
      ++active_;
    }
    std::string e;
    int64_t done = 0;
    if (!extend_to(j.file, j.off + j.bytes)) e = std::string("ftruncate: ") + std::strerror(errno);
    else if (mapped_ && write_mapped(j)) done = j.bytes;
    while (e.empty() && done < j.bytes) {
      const ssize_t r = ::pwrite(fds_[j.file], bufs_[j.slot] + done, (size_t)(j.bytes - done), (off_t)(j.off + done));
      if (r < 0) {
        if (errno == EINTR) continue;
        e = std::string("pwrite: ") + std::strerror(errno);
        break;
      }
      done += r;
    }
    {
      std::lock_guard<std::mutex> g(mu_);
      if (!e.empty() && err_.empty()) err_ = e;
      written_ += done;
      free_.push_back(j.slot);
      --active_;
    }
    cv_free_.notify_one();
    cv_idle_.notify_all();
  }
}

int64_t ChunkWriter::finish(int64_t final_size) {
  std::vector<int64_t> sizes(fds_.size(), 0);
  sizes[0] = final_size;
  return finish_all(sizes);
}

int64_t ChunkWriter::finish_all(const std::vector<int64_t>& sizes) {
  if (sizes.size() != fds_.size()) throw std::invalid_argument("ChunkWriter: one size per file");
  {
    std::unique_lock<std::mutex> lk(mu_);
    cv_idle_.wait(lk, [this] { return jobs_.empty() && active_ == 0; });
  }
  std::string e = error();
  for (size_t i = 0; i < fds_.size() && e.empty(); ++i)
    if (::ftruncate(fds_[i], (off_t)sizes[i]) != 0) e = std::string("ftruncate: ") + std::strerror(errno);
  const int64_t w = written_;
  abort();
  if (!e.empty()) throw std::runtime_error("ChunkWriter " + paths_[0] + ": " + e);
  return w;
}

std::string ChunkWriter::error() {
  std::lock_guard<std::mutex> g(mu_);
  return err_;
}

}  // namespace dryad
