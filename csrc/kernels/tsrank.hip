// Per-rank data path of the multi-rank TeraSort around the all-to-all-v (ops/recordsort.py).
//
// Send side over a generated input (gen://terasort).  A record is a pure function of its number,
// so the range partition needs neither a stored input table nor per-record sort entries:
//   ts_sample_keys   the sampler's keys, generated at the sample positions only
//   ts_dest_count    every record's key (generator hash) -> key range by binary search of the
//                    separators (LDS) -> per-workgroup bucket histogram, bucket = round-major
//                    range id (round b of the pipelined exchange = every rank's b-th range)
//   ts_dest_scatter  the same keys again -> stable, LDS-ranked scatter of the 32-bit record
//                    offsets into bucket order: 5 GB at 1.25e9 records, where the entry path
//                    writes 20 GB of 16-byte entries, rewrites them (range destination) and
//                    reads them twice more (histogram + bucket scatter)
//   ts_gen_gather    record idx[p] generated into send row p, one exchange round at a time, so
//                    round 0 goes on the wire after ~1/B of the pack instead of all of it
// Receive side: extract64_tile (E64 entries of received 100-byte rows read as whole lines
// through LDS, with the window-digit histograms of the look-back sort fused in).
//
// The reference's equivalent is the sampler + RangePartition vertex of CreateRangePartition
// (LinqToDryad/DryadLinqQueryGen.cs:2362-2474; DryadLinqVertex.cs:4909-5151) writing one file
// per destination, here a bucket-ordered HBM send buffer for RCCL.
#include "common.h"
#include "rowkey.h"
#include "scan.h"
#include "terasort_gen.h"

namespace {

constexpr int kBins = 256;
constexpr int kDsItems = 8;                        // records per thread per tile of the scatter
constexpr int kDsTile = kBlock * kDsItems;         // 2048
constexpr uint32_t kMaxG = 1024;

struct Seps {
  const E128* seps;
  uint32_t nsep;       // <= 255
  uint64_t lo_or;      // OR-ed into a record's lo word (rank << 32 when ties are split by rank)
  uint64_t lo_mask;    // compared bits of lo
  uint32_t subs;       // key ranges per destination rank (pipelined exchange rounds)
  uint32_t ranks;
};

__device__ __forceinline__ void load_seps(const Seps& sp, uint64_t* shi, uint64_t* slo) {
  for (uint32_t k = threadIdx.x; k < sp.nsep; k += blockDim.x) {
    shi[k] = sp.seps[k].hi;
    slo[k] = sp.seps[k].lo & sp.lo_mask;
  }
}

// bucket of record `first + i` (i = offset in this rank's slice, also its tie-break row index)
__device__ __forceinline__ uint32_t ts_bucket(uint64_t seed, uint64_t first, uint64_t i, const Seps& sp,
                                              const uint64_t* shi, const uint64_t* slo) {
  uint64_t kA, kB;
  dr_ts::ts_key_words(seed, first + i, kA, kB);
  const uint64_t kh = kA, kl = ((kB & 0xFFFF000000000000ull) | sp.lo_or | (uint32_t)i) & sp.lo_mask;
  uint32_t lo = 0, hi = sp.nsep;
  while (lo < hi) {                                // count of separators below the key
    const uint32_t mid = (lo + hi) >> 1;
    const uint64_t sh = shi[mid], sl = slo[mid];
    const bool before = sh < kh || (sh == kh && sl < kl);
    lo = before ? mid + 1 : lo;
    hi = before ? hi : mid;
  }
  return sp.subs > 1 ? (lo % sp.subs) * sp.ranks + lo / sp.subs : lo;
}

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

__global__ __launch_bounds__(256) void ts_dest_count_kernel(uint64_t first, uint64_t seed, uint64_t n, Seps sp,
                                                            uint32_t* __restrict__ counts, uint32_t G,
                                                            uint64_t per_block) {
  __shared__ uint64_t shi[256], slo[256];
  __shared__ uint32_t hist[4][kBins];
  const int t = threadIdx.x, w = wave_id();
  load_seps(sp, shi, slo);
  hist[0][t] = 0; hist[1][t] = 0; hist[2][t] = 0; hist[3][t] = 0;
  __syncthreads();
  const uint64_t beg = (uint64_t)blockIdx.x * per_block;
  const uint64_t end = beg + per_block < n ? beg + per_block : n;
  for (uint64_t i = beg + t; i < end; i += kBlock) atomicAdd(&hist[w][ts_bucket(seed, first, i, sp, shi, slo)], 1u);
  __syncthreads();
  counts[(uint64_t)t * G + blockIdx.x] = hist[0][t] + hist[1][t] + hist[2][t] + hist[3][t];
}

// Stable scatter of the record offsets into bucket order (the radix scatter's wave multisplit
// through LDS lane masks, one tile of 2048 records at a time, each bucket's run of a tile
// written contiguously).
__global__ __launch_bounds__(256) void ts_dest_scatter_kernel(uint64_t first, uint64_t seed, uint64_t n, Seps sp,
                                                              const uint32_t* __restrict__ offsets, uint32_t G,
                                                              uint64_t per_block, uint32_t* __restrict__ idx) {
  __shared__ uint64_t shi[256], slo[256];
  __shared__ uint32_t stage[kDsTile];
  __shared__ uint8_t dslot[kDsTile];
  __shared__ uint32_t wcnt[4][kBins];
  __shared__ unsigned long long wmask[4][kBins];
  __shared__ uint32_t goff[kBins];
  __shared__ uint32_t bstart[kBins];
  __shared__ uint32_t sc[4];
  const int t = threadIdx.x, w = wave_id(), l = lane_id();
  load_seps(sp, shi, slo);
  goff[t] = offsets[(uint64_t)t * G + blockIdx.x];
  wmask[0][t] = 0ull; wmask[1][t] = 0ull; wmask[2][t] = 0ull; wmask[3][t] = 0ull;
  const uint64_t beg = (uint64_t)blockIdx.x * per_block;
  const uint64_t end = beg + per_block < n ? beg + per_block : n;
  const unsigned long long lanebit = 1ull << l;
  for (uint64_t base = beg; base < end; base += kDsTile) {
    const uint32_t cnt = (uint32_t)((end - base) < (uint64_t)kDsTile ? (end - base) : kDsTile);
    wcnt[0][t] = 0; wcnt[1][t] = 0; wcnt[2][t] = 0; wcnt[3][t] = 0;
    __syncthreads();
    uint32_t rk[kDsItems], dg[kDsItems];
#pragma unroll
    for (int r = 0; r < kDsItems; ++r) {
      const uint32_t pos = w * (kDsTile / 4) + r * 64 + l;
      const bool valid = pos < cnt;
      const uint32_t d = valid ? ts_bucket(seed, first, base + pos, sp, shi, slo) : 0u;
      if (valid) atomicOr(&wmask[w][d], lanebit);
      __builtin_amdgcn_wave_barrier();
      const unsigned long long peers = valid ? wmask[w][d] : 0ull;
      const uint32_t below = popc_below(peers);
      const uint32_t prior = wcnt[w][d];
      __builtin_amdgcn_wave_barrier();
      if (valid && below == 0) {
        wcnt[w][d] = prior + (uint32_t)__popcll(peers);
        wmask[w][d] = 0ull;
      }
      __builtin_amdgcn_wave_barrier();
      rk[r] = prior + below;
      dg[r] = d;
    }
    __syncthreads();
    const uint32_t c0 = wcnt[0][t], c1 = wcnt[1][t], c2 = wcnt[2][t], c3 = wcnt[3][t];
    const uint32_t tot = c0 + c1 + c2 + c3;
    wcnt[0][t] = 0; wcnt[1][t] = c0; wcnt[2][t] = c0 + c1; wcnt[3][t] = c0 + c1 + c2;
    uint32_t all;
    bstart[t] = block_exclusive_scan256(tot, sc, all);
    __syncthreads();
#pragma unroll
    for (int r = 0; r < kDsItems; ++r) {
      const uint32_t pos = w * (kDsTile / 4) + r * 64 + l;
      if (pos < cnt) {
        const uint32_t slot = bstart[dg[r]] + wcnt[w][dg[r]] + rk[r];
        stage[slot] = (uint32_t)(base + pos);
        dslot[slot] = (uint8_t)dg[r];
      }
    }
    __syncthreads();
    for (uint32_t j = t; j < cnt; j += kBlock) {
      const uint32_t d = dslot[j];
      idx[(uint64_t)goff[d] + (j - bstart[d])] = stage[j];
    }
    __syncthreads();
    goff[t] += tot;
  }
}

__global__ void ts_bucket_starts_kernel(const uint32_t* __restrict__ counts_scanned, uint32_t G, uint64_t n,
                                        uint64_t* __restrict__ starts) {
  const int t = threadIdx.x;
  starts[t] = counts_scanned[(uint64_t)t * G];
  if (t == 0) starts[kBins] = n;
}

inline void dest_geometry(uint64_t n, uint32_t& G, uint64_t& per_block) {
  uint64_t tiles = (n + kDsTile - 1) / kDsTile;
  if (tiles < 1) tiles = 1;
  G = (uint32_t)(tiles < kMaxG ? tiles : kMaxG);
  per_block = ((tiles + G - 1) / G) * kDsTile;
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

DR_API uint64_t dr_ts_dest_workspace(uint64_t n) {
  uint32_t G; uint64_t per_block;
  dest_geometry(n, G, per_block);
  return ((uint64_t)kBins * G + 1024) * sizeof(uint32_t);
}

// Bucket order of gen://terasort records first .. first + n - 1 (n < 2^32): idx (n uint32)
// receives the slice offsets grouped by bucket, stable; bucket_starts (kBins + 1 uint64, device)
// every bucket's start.  Bucket of a record = the count of separators (E128, ascending, nsep <= 255)
// below its key {hi, (lo | lo_or) & lo_mask}, renumbered (g % subs) * ranks + g / subs when subs > 1.
DR_API int dr_ts_dest_partition(uint64_t first, uint64_t seed, uint64_t n, const E128* seps, uint32_t nsep,
                                uint64_t lo_or, uint64_t lo_mask, uint32_t subs, uint32_t ranks, void* ws,
                                uint32_t* idx, uint64_t* bucket_starts, hipStream_t s) {
  if (nsep > 255 || n >= (1ull << 32)) return (int)hipErrorInvalidValue;
  if (subs > 1 && (uint64_t)subs * ranks != (uint64_t)nsep + 1) return (int)hipErrorInvalidValue;
  if (n == 0) {
    hipMemsetAsync(bucket_starts, 0, sizeof(uint64_t) * (kBins + 1), s);
    return 0;
  }
  uint32_t G; uint64_t per_block;
  dest_geometry(n, G, per_block);
  Seps sp{seps, nsep, lo_or, lo_mask, subs, ranks};
  uint32_t* counts = reinterpret_cast<uint32_t*>(ws);
  uint32_t* partial = counts + (uint64_t)kBins * G;
  ts_dest_count_kernel<<<G, 256, 0, s>>>(first, seed, n, sp, counts, G, per_block);
  scan_inplace(counts, kBins * G, partial, s);
  ts_bucket_starts_kernel<<<1, kBins, 0, s>>>(counts, G, n, bucket_starts);
  ts_dest_scatter_kernel<<<G, 256, 0, s>>>(first, seed, n, sp, counts, G, per_block, idx);
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
