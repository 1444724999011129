// Microbenchmark: HBM read cost of touching only the first 16 bytes of every 64-byte row vs the
// whole row (does the memory system fetch less than a full line / sector for a partial read?).
// Build: hipcc --offload-arch=gfx950 -O3 tools/micro/strided_read.hip -o build/strided_read
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdint>

__global__ void read_rows(const uint4* __restrict__ in, uint64_t rows, int pieces_per_row, int stride_pieces,
                          unsigned long long* __restrict__ sink) {
  uint32_t acc = 0;
  for (uint64_t r = blockIdx.x * (uint64_t)blockDim.x + threadIdx.x; r < rows; r += (uint64_t)gridDim.x * blockDim.x) {
    for (int p = 0; p < pieces_per_row; ++p) {
      const uint4 v = in[r * stride_pieces + p];
      acc ^= v.x ^ v.y ^ v.z ^ v.w;
    }
  }
  if (acc == 0x12345678u) atomicAdd(sink, 1ull);
}

int main() {
  const uint64_t bytes = 32ull << 30;              // 32 GB table of 64-byte rows
  uint4* buf;
  unsigned long long* sink;
  if (hipMalloc(&buf, bytes) != hipSuccess || hipMalloc(&sink, 8) != hipSuccess) return 1;
  hipMemset(buf, 1, bytes);
  hipEvent_t a, b;
  hipEventCreate(&a);
  hipEventCreate(&b);
  for (int cfg = 0; cfg < 6; ++cfg) {
    const int row_pieces = cfg < 3 ? 4 : 8;                    // 64- or 128-byte rows
    const int pieces = cfg < 3 ? (4 >> cfg) : (8 >> (cfg - 3));
    const uint64_t nr = bytes / (16 * row_pieces);
    float best = 1e9f;
    for (int it = 0; it < 4; ++it) {
      hipEventRecord(a);
      read_rows<<<8192, 256>>>(buf, nr, pieces, row_pieces, sink);
      hipEventRecord(b);
      hipEventSynchronize(b);
      float ms;
      hipEventElapsedTime(&ms, a, b);
      if (it && ms < best) best = ms;
    }
    printf("read %3d of %3d bytes per row: %.2f ms, %.0f GB/s of touched bytes, %.0f GB/s of table\n", 16 * pieces,
           16 * row_pieces, best, nr * 16.0 * pieces / best / 1e6, bytes / best / 1e6);
  }
  return 0;
}
