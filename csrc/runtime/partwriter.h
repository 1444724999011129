// ChunkWriter: a part file written from a ring of caller-owned (page-locked) host buffers by a
// pool of writer threads, so the caller can DMA the next chunk out of HBM while earlier ones are
// written.  The native side of the HBM -> partfile path (reference: the overlapped channel writer
// DryadVertex/VertexHost/system/channel/src/channelbuffernativewriter.cpp, which extends its file
// in 256 MB steps, s_fileExtendChunk at :35, and keeps several writes in flight).  The HIP copies
// stay on the Python side (io/writer.py): the writer only drains host buffers.
//
//   acquire()                 a free buffer slot (blocks while every slot is queued / writing)
//   submit(slot, off, bytes, file)  write the slot's first `bytes` bytes at offset `off` of file
//                             `file`; the file is pre-extended ahead of the writes in `extend` steps
//   finish(size)              wait for every write, cut the (first) file to `size`, close it
//   finish_all(sizes)         the same for every file
// Several files (one writer over the part files of a split partition): buffered writes to one
// file serialise on its inode lock (~12 GB/s on the MI355X box), writes to distinct files do not
// (40-93 GB/s with 4-12 threads, profiles/r4/filewrite_ab2.log), so the caller interleaves the
// chunks of the files.
// `reuse` (several files): existing files are overwritten in place instead of truncated (the
// parts of a replaced table recycled as the new table's part files: no page-cache pages freed and
// allocated again, io/partfile.py recycle pool).
// `mapped`: the threads copy into shared mappings of the file instead of pwrite()ing, so they
// fill the page cache in parallel (partwriter.cpp, write_mapped).
#pragma once
#include <condition_variable>
#include <cstdint>
#include <deque>
#include <mutex>
#include <string>
#include <thread>
#include <vector>

namespace dryad {

class ChunkWriter {
 public:
  ChunkWriter(const std::string& path, const std::vector<uint64_t>& buf_ptrs, int threads, int64_t extend_bytes,
              bool mapped = false);
  ChunkWriter(const std::vector<std::string>& paths, const std::vector<uint64_t>& buf_ptrs, int threads,
              int64_t extend_bytes, bool reuse = false);
  ~ChunkWriter();
  int acquire();                                   // -1 on error (see error())
  void submit(int slot, int64_t offset, int64_t bytes, int file = 0);
  int64_t finish(int64_t final_size);              // bytes written; throws on error
  int64_t finish_all(const std::vector<int64_t>& sizes);
  std::string error();
  void abort();                                    // stop the threads, close (the file stays)

 private:
  struct Job {
    int slot;
    int64_t off, bytes;
    int file;
  };
  void start(int threads);
  void run();
  bool extend_to(int file, int64_t end);
  bool write_mapped(const Job& j);
  std::vector<int> fds_;
  std::vector<std::string> paths_;
  std::vector<int64_t> allocated_;
  int64_t extend_ = 0, written_ = 0;
  std::vector<uint8_t*> bufs_;
  std::vector<std::thread> pool_;
  std::mutex mu_, ext_mu_;
  std::condition_variable cv_job_, cv_free_, cv_idle_;
  std::deque<int> free_;
  std::deque<Job> jobs_;
  int active_ = 0;
  bool stop_ = false, mapped_ = false, reuse_ = false;
  std::string err_;
};

}  // namespace dryad
