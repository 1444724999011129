// Per-rank data path of the multi-rank TeraSort around the all-to-all-v (ops/recordsort.py).
//
//   ts_sample_keys   the sampler's keys of a generated input (gen://terasort), generated at the
//                    sample positions only (a record is a pure function of its number)
//   extract64_tile   E64 entries of received 100-byte rows read as whole lines through LDS, with
//                    the window-digit histograms of the look-back sort fused in (the receive side
//                    of stored-row inputs; generated inputs take the fine-bucket exchange of
//                    tsmerge.hip)
//
// The reference's equivalent is the sampler + RangePartition vertex of CreateRangePartition
// (LinqToDryad/DryadLinqQueryGen.cs:2362-2474; DryadLinqVertex.cs:4909-5151) writing one file
// per destination, here a bucket-ordered HBM send buffer for RCCL.
#include "common.h"
#include "rowkey.h"
#include "terasort_gen.h"

namespace {

constexpr int kBins = 256;
__global__ __launch_bounds__(256) void ts_sample_keys_kernel(uint64_t first, uint64_t seed, uint64_t off,
                                                             uint64_t stride, uint64_t m, uint64_t lo_or,
                                                             E128* __restrict__ out) {
  for (uint64_t k = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; k < m; k += (uint64_t)gridDim.x * blockDim.x) {
    const uint64_t i = off + k * stride;
    uint64_t kA, kB;
    dr_ts::ts_key_words(seed, first + i, kA, kB);
    E128 e;
    e.hi = kA;
    e.lo = (kB & 0xFFFF000000000000ull) | lo_or | (uint32_t)i;
    out[k] = e;
  }
}

// E64 entries (key window << 32 | row) of `n` rows of `stride` bytes (4 <= stride <= 128, a
// multiple of 4), read a 256-row tile at a time as whole 16-byte chunks into LDS (the one-row-per-
// lane extract_keys64 issues three dword loads 100 bytes apart per row: 37 ms at 1.25e9 rows).
// hist_part (nullable): per-workgroup [4][256] histograms of the four window bytes, the producer
// histograms of dr_sort_u64_onesweep.
template <bool HIST>
__global__ __launch_bounds__(256) void extract64_tile_kernel(const uint8_t* __restrict__ rows, uint64_t n,
                                                             uint32_t stride, uint32_t key_off, uint32_t key_len,
                                                             uint32_t P, E64* __restrict__ out,
                                                             uint32_t* __restrict__ hist_part) {
  __shared__ __attribute__((aligned(16))) uint4 img[(256 * 128 + 32) / 16];
  __shared__ uint32_t hist[HIST ? 4 : 1][kBins];
  const int t = threadIdx.x;
  if constexpr (HIST) {
    hist[0][t] = 0; hist[1][t] = 0; hist[2][t] = 0; hist[3][t] = 0;
  }
  const uint8_t* lds = reinterpret_cast<const uint8_t*>(img);
  for (uint64_t row0 = (uint64_t)blockIdx.x * 256; row0 < n; row0 += (uint64_t)gridDim.x * 256) {
    const uint32_t nr = (uint32_t)((n - row0) < 256 ? (n - row0) : 256);
    const uintptr_t a = reinterpret_cast<uintptr_t>(rows + row0 * stride);
    const uint32_t shift = (uint32_t)(a & 15);
    const uint4* src = reinterpret_cast<const uint4*>(a - shift);
    const uint32_t chunks = (nr * stride + shift + 15) / 16;
    __syncthreads();                               // the previous tile's keys have been read
    for (uint32_t c = t; c < chunks; c += kBlock) img[c] = src[c];
    __syncthreads();
    if (t < nr) {
      const uint32_t o = shift + t * stride + key_off;
      uint64_t k0, k1;
      load_key128(lds + o, key_len, (o & 3) == 0, k0, k1);
      const uint32_t win = key_window(k0, k1, P);
      E64 e;
      e.v = ((uint64_t)win << 32) | (uint32_t)(row0 + t);
      out[row0 + t] = e;
      if constexpr (HIST) {
#pragma unroll
        for (int p = 0; p < 4; ++p) atomicAdd(&hist[p][(win >> (8 * p)) & 0xFF], 1u);
      }
    }
  }
  if constexpr (HIST) {
    __syncthreads();
#pragma unroll
    for (int p = 0; p < 4; ++p) hist_part[((uint64_t)blockIdx.x * 4 + p) * kBins + t] = hist[p][t];
  }
}

}  // namespace

// Sample keys of gen://terasort records first + off + k * stride (k < m) as E128 entries
// {hi = key bytes 0..7, lo = key bytes 8..9 << 48 | lo_or | slice offset}: the entries the
// multi-rank sort's sampler draws (ops/recordsort.choose_separators).
DR_API int dr_ts_sample_keys(uint64_t first, uint64_t seed, uint64_t off, uint64_t stride, uint64_t m,
                             uint64_t lo_or, E128* out, hipStream_t s) {
  if (m == 0) return 0;
  ts_sample_keys_kernel<<<grid_for(m, 256, 1024), 256, 0, s>>>(first, seed, off, stride, m, lo_or, out);
  DR_LAUNCH_CHECK();
  return 0;
}

DR_API uint32_t dr_extract_keys64_tile_parts(uint64_t n) { return grid_for(n, 256, 8192); }

// dr_extract_keys64 reading whole rows through LDS; hist_part (nullable) receives
// dr_extract_keys64_tile_parts(n) per-workgroup [4][256] window-byte histograms.
DR_API int dr_extract_keys64_tile(const uint8_t* rows, uint64_t n, uint32_t stride, uint32_t key_off,
                                  uint32_t key_len, uint32_t prefix_bits, E64* out, uint32_t* hist_part,
                                  hipStream_t s) {
  if (stride == 0 || (stride & 3) || stride > 128 || key_len == 0 || key_len > 16 || key_off + key_len > stride)
    return (int)hipErrorInvalidValue;
  if (n >= (1ull << 32)) return (int)hipErrorInvalidValue;
  if (n == 0) return 0;
  const unsigned g = dr_extract_keys64_tile_parts(n);
  if (hist_part)
    extract64_tile_kernel<true><<<g, 256, 0, s>>>(rows, n, stride, key_off, key_len, prefix_bits, out, hist_part);
  else
    extract64_tile_kernel<false><<<g, 256, 0, s>>>(rows, n, stride, key_off, key_len, prefix_bits, out, nullptr);
  DR_LAUNCH_CHECK();
  return 0;
}
