// Fine-bucket exchange of the multi-rank TeraSort (ops/recordsort.py, gen:// inputs).
//
// The send side sorts its records' E64 entries (key bytes 0..3 as the window) on the window, so
// its rows leave in key order, and the key ranges of the exchange are unions of FINE BUCKETS (the
// top `fb` key bits, fb >= 25: ~300 rows of the whole job per bucket).  Every source sends, next
// to its rows, its row count per fine bucket.  A received key range is then, per fine bucket, W
// contiguous slices (one per source) of rows that all share their top fb key bits, and the
// receive side orders each bucket on its own in LDS (ts_tile_merge): no entry extraction, no
// radix passes and no random row gather over the received block, one sequential read and one
// sequential write of the rows.
//   ts_fine_starts   starts[k] = first sorted entry with bucket >= k (k = 0 .. 2^fb)
//   ts_tile_merge    one workgroup per fine bucket: its slices staged in LDS at the 100-byte
//                    pitch, keys (bits fb..79 + tile index) bitonic-sorted in LDS, rows written
//                    back in key order
// Reference: the sampler + RangePartition + MergeSort stages of CreateRangePartition
// (LinqToDryad/DryadLinqQueryGen.cs:2362-2474); its merge of the sorted inputs becomes a
// per-bucket LDS sort because the buckets are small enough to hold.
#include "common.h"

namespace {

constexpr uint32_t kTmCap = 512;                   // rows of one bucket held in LDS (9 index bits)
constexpr uint32_t kTmMaxW = 64;                   // sources
constexpr uint32_t kTmWords = 25;                  // 100-byte rows

__global__ __launch_bounds__(256) void ts_fine_starts_kernel(const E64* __restrict__ ent, uint64_t n, uint32_t fb,
                                                             uint32_t* __restrict__ starts) {
  const uint32_t nb = 1u << fb;
  const int sh = 64 - (int)fb;
  for (uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (uint64_t)gridDim.x * blockDim.x) {
    const uint32_t b = (uint32_t)(ent[i].v >> sh);
    if (i == 0) {
      for (uint32_t k = 0; k <= b; ++k) starts[k] = 0;
    } else {
      const uint32_t pb = (uint32_t)(ent[i - 1].v >> sh);
      for (uint32_t k = pb + 1; k <= b; ++k) starts[k] = (uint32_t)i;
    }
    if (i == n - 1) {
      for (uint32_t k = b + 1; k <= nb; ++k) starts[k] = (uint32_t)n;
    }
  }
}

// pre[s * K + k] = row (of `rows`) where bucket k's slice from source s starts, cnt[s * K + k] its
// rows; bucket k's output rows start at out row outoff[k].  A bucket of more than kTmCap rows is
// skipped and flagged (*overflow); the caller orders that key range another way.
__global__ __launch_bounds__(256) void ts_tile_merge_kernel(const uint32_t* __restrict__ rows, uint32_t* __restrict__ out,
                                                            const int64_t* __restrict__ pre,
                                                            const int32_t* __restrict__ cnt,
                                                            const int64_t* __restrict__ outoff, uint32_t W, uint32_t K,
                                                            uint32_t fb, uint32_t* __restrict__ overflow) {
  __shared__ __attribute__((aligned(16))) uint32_t stage[kTmCap * kTmWords];
  __shared__ uint64_t key[kTmCap];
  __shared__ uint64_t srow[kTmCap];
  __shared__ int64_t sbase[kTmMaxW];
  __shared__ uint32_t spre[kTmMaxW + 1];
  const uint32_t t = threadIdx.x;
  for (uint32_t k = blockIdx.x; k < K; k += gridDim.x) {
    if (t < W) sbase[t] = pre[(uint64_t)t * K + k];
    if (t == 0) {
      uint32_t acc = 0;
      for (uint32_t s = 0; s < W; ++s) {
        spre[s] = acc;
        acc += (uint32_t)cnt[(uint64_t)s * K + k];
      }
      spre[W] = acc;
    }
    __syncthreads();
    const uint32_t nt = spre[W];
    if (nt == 0 || nt > kTmCap) {
      if (nt > kTmCap && t == 0) atomicOr(overflow, 1u);
      __syncthreads();
      continue;
    }
    for (uint32_t i = t; i < nt; i += kBlock) {     // source row of each tile row (source-major = stable)
      uint32_t s = 0;
      while (spre[s + 1] <= i) ++s;
      srow[i] = (uint64_t)(sbase[s] + (int64_t)(i - spre[s]));
    }
    __syncthreads();
    // the bucket's rows into LDS: W contiguous slices, every load of a batch in flight at once
    const uint32_t words = nt * kTmWords;
    for (uint32_t j0 = t; j0 < words; j0 += kBlock * 10) {
      uint32_t v[10];
#pragma unroll
      for (int q = 0; q < 10; ++q) {
        const uint32_t j = j0 + q * kBlock;
        if (j < words) {
          const uint32_t r = j / kTmWords, c = j - r * kTmWords;
          v[q] = rows[srow[r] * kTmWords + c];
        }
      }
#pragma unroll
      for (int q = 0; q < 10; ++q) {
        const uint32_t j = j0 + q * kBlock;
        if (j < words) stage[j] = v[q];
      }
    }
    __syncthreads();
    // sort keys: key bits [fb, 80) left-aligned (the top fb bits are the bucket), tile index below
    uint32_t P = 1;
    while (P < nt) P <<= 1;
    for (uint32_t i = t; i < P; i += kBlock) {
      uint64_t kv = ~0ull;
      if (i < nt) {
        const uint32_t* w = stage + i * kTmWords;
        const uint64_t k0 = ((uint64_t)bswap32(w[0]) << 32) | bswap32(w[1]);
        const uint64_t k1 = (uint64_t)(bswap32(w[2]) >> 16);          // key bytes 8, 9
        const uint64_t hi = (k0 << fb) | ((k1 << 48) >> (64 - fb));
        kv = (hi & ~(uint64_t)(kTmCap - 1)) | i;
      }
      key[i] = kv;
    }
    __syncthreads();
    for (uint32_t size = 2; size <= P; size <<= 1) {
      for (uint32_t stride = size >> 1; stride > 0; stride >>= 1) {
        for (uint32_t i = t; i < (P >> 1); i += kBlock) {
          const uint32_t lo = 2 * i - (i & (stride - 1)), hi = lo + stride;
          const bool asc = (lo & size) == 0;
          const uint64_t a = key[lo], b = key[hi];
          if ((a > b) == asc) {
            key[lo] = b;
            key[hi] = a;
          }
        }
        __syncthreads();
      }
    }
    uint32_t* o = out + (uint64_t)outoff[k] * kTmWords;
    for (uint32_t j = t; j < words; j += kBlock) {
      const uint32_t r = j / kTmWords, c = j - r * kTmWords;
      const uint32_t i = (uint32_t)(key[r] & (kTmCap - 1));
      __builtin_nontemporal_store(stage[i * kTmWords + c], o + j);
    }
    __syncthreads();
  }
}

}  // namespace

// starts: (1 << fb) + 1 uint32 = for each fine bucket k the first position of `ent` (sorted on
// at least the top fb window bits) whose bucket is >= k; starts[1 << fb] = n.
DR_API int dr_ts_fine_starts(const E64* ent, uint64_t n, uint32_t fb, uint32_t* starts, hipStream_t s) {
  if (fb == 0 || fb > 28 || n >= (1ull << 32)) return (int)hipErrorInvalidValue;
  if (n == 0) return (int)hipMemsetAsync(starts, 0, ((size_t(1) << fb) + 1) * sizeof(uint32_t), s);
  ts_fine_starts_kernel<<<grid_for(n, 256, 16384), 256, 0, s>>>(ent, n, fb, starts);
  DR_LAUNCH_CHECK();
  return 0;
}

DR_API uint32_t dr_ts_tile_cap() { return kTmCap; }

// rows / out: 100-byte rows (4-byte aligned); pre, cnt: [W][K]; outoff: [K]; 25 <= fb <= 32.
DR_API int dr_ts_tile_merge(const uint8_t* rows, uint8_t* out, const int64_t* pre, const int32_t* cnt,
                            const int64_t* outoff, uint32_t W, uint32_t K, uint32_t fb, uint32_t* overflow,
                            hipStream_t s) {
  if (W == 0 || W > kTmMaxW || fb < 25 || fb > 32) return (int)hipErrorInvalidValue;
  if ((reinterpret_cast<uintptr_t>(rows) | reinterpret_cast<uintptr_t>(out)) & 3) return (int)hipErrorInvalidValue;
  if (K == 0) return 0;
  const unsigned g = K < 65536u ? K : 65536u;
  ts_tile_merge_kernel<<<g, 256, 0, s>>>(reinterpret_cast<const uint32_t*>(rows), reinterpret_cast<uint32_t*>(out),
                                         pre, cnt, outoff, W, K, fb, overflow);
  DR_LAUNCH_CHECK();
  return 0;
}
