// Ceiling of the radix-scatter memory pattern without any ranking work: every workgroup reads a
// 64 KB tile contiguously and writes it as `bins` runs of 64 KB / bins bytes, run d of tile t
// landing right after run d of tile t - 1 in destination region d (what a radix pass with
// uniform digits writes).  Measures read + write TB/s for run sizes 128 B .. 8 KB (bins 512 .. 8)
// over 10 GB, against a plain contiguous copy.  If the 256-bin case sits near the radix passes'
// 3.4 TB/s, the pass is bound by this write pattern, not by its ranking.
// Build: hipcc --offload-arch=gfx950 -O3 -std=c++17 tools/micro/runwrite_ceiling.hip -o tools/micro/bin/runwrite_ceiling
#include <hip/hip_runtime.h>

#include <cstdint>
#include <cstdio>
#include <cstdlib>

namespace {
constexpr uint32_t kTileBytes = 64 * 1024;

__global__ __launch_bounds__(256) void runs(const uint4* __restrict__ in, uint4* __restrict__ out, uint64_t tiles,
                                            uint32_t bins, uint64_t region_pieces) {
  const uint32_t per_tile = kTileBytes / 16;             // 16-byte pieces per tile
  const uint32_t run = per_tile / bins;                  // pieces per run
  for (uint64_t t = blockIdx.x; t < tiles; t += gridDim.x) {
    const uint4* src = in + t * per_tile;
    for (uint32_t j = threadIdx.x; j < per_tile; j += blockDim.x) {
      const uint32_t d = j / run, k = j - d * run;
      out[(uint64_t)d * region_pieces + t * run + k] = src[j];
    }
  }
}

__global__ __launch_bounds__(256) void copy(const uint4* __restrict__ in, uint4* __restrict__ out, uint64_t pieces) {
  for (uint64_t i = blockIdx.x * (uint64_t)blockDim.x + threadIdx.x; i < pieces; i += (uint64_t)gridDim.x * blockDim.x)
    out[i] = in[i];
}
}  // namespace

#define HC(x)                                                      \
  do {                                                             \
    hipError_t e_ = (x);                                           \
    if (e_ != hipSuccess) {                                        \
      std::fprintf(stderr, "%s: %s\n", #x, hipGetErrorString(e_)); \
      std::exit(1);                                                \
    }                                                              \
  } while (0)

int main() {
  const uint64_t bytes = 10ull << 30;
  const uint64_t tiles = bytes / kTileBytes, pieces = bytes / 16;
  uint4 *in, *out;
  HC(hipMalloc(&in, bytes));
  HC(hipMalloc(&out, bytes));
  HC(hipMemset(in, 1, bytes));
  hipEvent_t a, b;
  HC(hipEventCreate(&a));
  HC(hipEventCreate(&b));
  auto timeit = [&](auto launch) {
    float best = 1e9f;
    for (int it = 0; it < 4; ++it) {
      HC(hipEventRecord(a));
      launch();
      HC(hipEventRecord(b));
      HC(hipEventSynchronize(b));
      float ms;
      HC(hipEventElapsedTime(&ms, a, b));
      if (it > 0 && ms < best) best = ms;
    }
    return best;
  };
  float ms = timeit([&] { copy<<<16384, 256>>>(in, out, pieces); });
  std::printf("contiguous copy        %.3f ms  %.2f TB/s (read + write)\n", ms, 2.0 * bytes / 1e12 / (ms / 1e3));
  for (uint32_t bins : {8u, 32u, 64u, 128u, 256u, 512u}) {
    const uint64_t region = tiles * (kTileBytes / 16 / bins);
    for (unsigned grid : {512u, 2048u}) {
      ms = timeit([&] { runs<<<grid, 256>>>(in, out, tiles, bins, region); });
      std::printf("runs of %5u B (%3u bins) grid %5u  %.3f ms  %.2f TB/s\n", kTileBytes / bins, bins, grid, ms,
                  2.0 * bytes / 1e12 / (ms / 1e3));
    }
  }
  std::fflush(stdout);
  return 0;
}
