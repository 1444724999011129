// Exclusive scan of a device uint32 array (the count matrices of the radix and bucket passes):
// reduce per 4096-element chunk, scan the chunk totals in one workgroup, scan down.
#pragma once
#include "common.h"

namespace {

constexpr int kScanChunk = 4096;           // elements per scan workgroup (16 per thread)

// --- exclusive scan of a uint32 array of length M (M <= 256 * kScanChunk) ---
__global__ __launch_bounds__(256) void rs_scan_reduce(const uint32_t* __restrict__ a, uint32_t M,
                                                      uint32_t* __restrict__ partial) {
  __shared__ uint32_t sc[4];
  const uint32_t base = blockIdx.x * kScanChunk + threadIdx.x * 16;
  uint32_t s = 0;
#pragma unroll
  for (int k = 0; k < 16; ++k) s += (base + k < M) ? a[base + k] : 0u;
  uint32_t total;
  block_exclusive_scan256(s, sc, total);
  if (threadIdx.x == 0) partial[blockIdx.x] = total;
}

__global__ __launch_bounds__(256) void rs_scan_partials(uint32_t* __restrict__ partial, uint32_t S) {
  __shared__ uint32_t sc[4];
  const uint32_t t = threadIdx.x;
  uint32_t v = t < S ? partial[t] : 0u;
  uint32_t total;
  uint32_t ex = block_exclusive_scan256(v, sc, total);
  if (t < S) partial[t] = ex;
}

__global__ __launch_bounds__(256) void rs_scan_down(uint32_t* __restrict__ a, uint32_t M,
                                                    const uint32_t* __restrict__ partial) {
  __shared__ uint32_t sc[4];
  const uint32_t base = blockIdx.x * kScanChunk + threadIdx.x * 16;
  uint32_t v[16];
  uint32_t s = 0;
#pragma unroll
  for (int k = 0; k < 16; ++k) {
    v[k] = (base + k < M) ? a[base + k] : 0u;
    s += v[k];
  }
  uint32_t total;
  uint32_t run = block_exclusive_scan256(s, sc, total) + partial[blockIdx.x];
#pragma unroll
  for (int k = 0; k < 16; ++k) {
    if (base + k < M) a[base + k] = run;
    run += v[k];
  }
}

void scan_inplace(uint32_t* a, uint32_t M, uint32_t* partial, hipStream_t s) {
  const uint32_t S = (M + kScanChunk - 1) / kScanChunk;
  rs_scan_reduce<<<S, 256, 0, s>>>(a, M, partial);
  rs_scan_partials<<<1, 256, 0, s>>>(partial, S);
  rs_scan_down<<<S, 256, 0, s>>>(a, M, partial);
}

}  // namespace
