// ChunkReader: a file read into a ring of caller-owned (page-locked) host buffers by a pool of
// reader threads, chunk by chunk, so the caller can DMA each chunk to HBM while the next ones are
// read.  The native side of the partfile -> HBM path (reference: the overlapped channel reader
// DryadVertex/VertexHost/system/channel/src/channelbuffernativereader.cpp, which keeps several
// 256 MB extents in flight).  The HIP copies stay on the Python side (the runtime module does not
// link HIP): the reader only fills host buffers.
//
//   reader threads  claim the next chunk index, wait for a free buffer slot, pread() the chunk
//                   into it, publish (slot, chunk, bytes)
//   next()          any ready chunk (not necessarily in file order), GIL released while waiting
//   release(slot)   the caller's DMA out of the slot has completed
//
// Where records start inside a variable-length record stream is not known per chunk; the block
// index the device decoder needs comes from the part's index sidecar (written with the part) or
// from scan_record_blocks (codec.h) over the whole buffer.
#pragma once
#include <atomic>
#include <condition_variable>
#include <cstdint>
#include <deque>
#include <mutex>
#include <string>
#include <thread>
#include <utility>
#include <vector>

namespace dryad {

struct ReadyChunk {
  int slot = -1;
  int64_t chunk = -1;     // chunk index (file offset = offset + chunk * chunk_bytes)
  int64_t bytes = 0;
};

class ChunkReader {
 public:
  // [offset, offset + length) of `path` (length < 0: to the end) in chunks of chunk_bytes, into
  // the buffers bufs[i] = (address, size in bytes), with `threads` reader threads.  Every buffer
  // must hold a whole chunk: a buffer smaller than chunk_bytes (or a null one) is refused with
  // std::invalid_argument before any thread starts, so no read can run past a buffer.
  ChunkReader(const std::string& path, int64_t offset, int64_t length, int64_t chunk_bytes,
              const std::vector<std::pair<uint64_t, int64_t>>& bufs, int threads);
  ~ChunkReader();
  int64_t size() const { return length_; }
  int64_t chunks() const { return nchunks_; }
  // Next ready chunk; returns false when every chunk has been handed out (or on error: check
  // error()).  timeout_ms < 0: wait indefinitely.
  bool next(ReadyChunk* out, int64_t timeout_ms);
  void release(int slot);
  std::string error();
  void stop();

 private:
  void run();
  int fd_ = -1;
  int64_t offset_ = 0, length_ = 0, chunk_ = 0, nchunks_ = 0;
  std::vector<uint8_t*> bufs_;
  std::vector<std::thread> pool_;
  std::mutex mu_;
  std::condition_variable cv_free_, cv_ready_;
  std::deque<int> free_;
  std::deque<ReadyChunk> ready_;
  std::atomic<int64_t> next_chunk_{0};
  int64_t handed_ = 0;
  bool stop_ = false;
  std::string err_;
};

}  // namespace dryad
