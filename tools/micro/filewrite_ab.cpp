// Page-cache write ceiling for one part file: N threads pwrite() 64 MB chunks into one file
// (buffered writes to one inode serialise on its lock) against N threads copying the same chunks
// into a shared MAP_SHARED mapping of the pre-sized file (page faults on distinct pages run in
// parallel), with and without MADV_POPULATE_WRITE pre-faulting each chunk; then the same bytes
// pwrite()n into one file per thread (is the ceiling per inode or global?) and O_DIRECT pwrite()s
// into one preallocated file (no page cache).
// Build: g++ -O3 -std=c++17 -pthread tools/micro/filewrite_ab.cpp -o tools/micro/bin/filewrite_ab
// Run:   filewrite_ab <dir> <GB> <threads...>
#ifndef _GNU_SOURCE
#define _GNU_SOURCE
#endif
#include <fcntl.h>
#include <sys/mman.h>
#include <unistd.h>

#include <atomic>
#include <chrono>
#include <cstdint>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <functional>
#include <string>
#include <thread>
#include <vector>

#ifndef MADV_POPULATE_WRITE
#define MADV_POPULATE_WRITE 23
#endif

namespace {
constexpr size_t kChunk = 64ull << 20;

double now() {
  return std::chrono::duration<double>(std::chrono::steady_clock::now().time_since_epoch()).count();
}

void run_threads(int nt, size_t chunks, const std::function<void(size_t)>& fn) {
  std::atomic<size_t> next{0};
  std::vector<std::thread> ts;
  for (int i = 0; i < nt; ++i)
    ts.emplace_back([&] {
      for (size_t c; (c = next.fetch_add(1)) < chunks;) fn(c);
    });
  for (auto& t : ts) t.join();
}
}  // namespace

int main(int argc, char** argv) {
  if (argc < 4) {
    std::fprintf(stderr, "usage: %s dir GB threads...\n", argv[0]);
    return 2;
  }
  const std::string dir = argv[1];
  const size_t bytes = (size_t)(std::atof(argv[2]) * 1e9) / kChunk * kChunk;
  const size_t chunks = bytes / kChunk;
  std::vector<uint8_t*> src(16);
  for (auto& p : src) {
    p = (uint8_t*)std::aligned_alloc(4096, kChunk);
    std::memset(p, 0x5a, kChunk);
  }
  const std::string path = dir + "/filewrite_ab.bin";
  for (int a = 3; a < argc; ++a) {
    const int nt = std::atoi(argv[a]);
    for (int mode = 0; mode < 5; ++mode) {
      ::unlink(path.c_str());
      if (mode == 3) {                       // one file per thread
        std::vector<int> fds(nt);
        for (int i = 0; i < nt; ++i) {
          fds[i] = ::open((path + "." + std::to_string(i)).c_str(), O_RDWR | O_CREAT | O_TRUNC, 0644);
          if (fds[i] < 0) { std::perror("open"); return 1; }
        }
        const double t0 = now();
        std::vector<std::thread> ts;
        for (int i = 0; i < nt; ++i)
          ts.emplace_back([&, i] {
            for (size_t c = i, k = 0; c < chunks; c += nt, ++k)
              if (::pwrite(fds[i], src[c % 16], kChunk, (off_t)(k * kChunk)) != (ssize_t)kChunk) std::abort();
          });
        for (auto& t : ts) t.join();
        const double t1 = now();
        for (int i = 0; i < nt; ++i) { ::close(fds[i]); ::unlink((path + "." + std::to_string(i)).c_str()); }
        std::printf("%-28s threads %2d  %.2f GB in %.3f s = %.2f GB/s\n", "pwrite (one file per thread)", nt,
                    bytes / 1e9, t1 - t0, bytes / 1e9 / (t1 - t0));
        std::fflush(stdout);
        continue;
      }
      const int fd = ::open(path.c_str(), O_RDWR | O_CREAT | O_TRUNC | (mode == 4 ? O_DIRECT : 0), 0644);
      if (fd < 0) {
        std::perror("open");
        return 1;
      }
      const double t0 = now();
      if (mode == 0 || mode == 4) {
        ::posix_fallocate(fd, 0, (off_t)bytes);
        run_threads(nt, chunks, [&](size_t c) {
          size_t done = 0;
          while (done < kChunk) {
            const ssize_t r = ::pwrite(fd, src[c % 16] + done, kChunk - done, (off_t)(c * kChunk + done));
            if (r <= 0) std::abort();
            done += (size_t)r;
          }
        });
      } else {
        if (::ftruncate(fd, (off_t)bytes) != 0) std::abort();
        ::posix_fallocate(fd, 0, (off_t)bytes);
        auto* map = (uint8_t*)::mmap(nullptr, bytes, PROT_READ | PROT_WRITE, MAP_SHARED, fd, 0);
        if (map == MAP_FAILED) {
          std::perror("mmap");
          return 1;
        }
        run_threads(nt, chunks, [&](size_t c) {
          uint8_t* d = map + c * kChunk;
          if (mode == 2) ::madvise(d, kChunk, MADV_POPULATE_WRITE);
          std::memcpy(d, src[c % 16], kChunk);
        });
        ::munmap(map, bytes);
      }
      const double t1 = now();
      ::close(fd);
      std::printf("%-28s threads %2d  %.2f GB in %.3f s = %.2f GB/s\n",
                  mode == 0 ? "pwrite (one file)" : mode == 1 ? "mmap memcpy" : mode == 2 ? "mmap populate+memcpy"
                                                                                       : "O_DIRECT pwrite (one file)", nt,
                  bytes / 1e9, t1 - t0, bytes / 1e9 / (t1 - t0));
      std::fflush(stdout);
    }
  }
  ::unlink(path.c_str());
  return 0;
}
