// LSD radix sort of 128-bit (hi, lo) entries + key extraction + row gather, for gfx950.
//
// This is the engine behind OrderBy / Sort / MergeSort / RangePartition of the vertex operator
// library (reference: LinqToDryad/DryadLinqVertex.cs:293-423 `Sort`/`MergeSort`, and the threaded
// `ParallelSort` at :9321-9817 which sorts 2^21-element chunks and k-way merges them).  Instead of
// comparison sorting boxed records we sort compact 16-byte (key, row-index) entries with a stable
// reduce-then-scan LSD radix sort and then gather whole rows once (key-pointer sort).
//
// Per 8-bit pass:
//   rs_count   : G workgroups, each owns a contiguous range of 2048-entry tiles and builds a
//                256-bin LDS histogram (one sub-histogram per wave to cut LDS atomic contention)
//   rs_scan_*  : exclusive scan of the [digit][block] count matrix (3 tiny kernels)
//   rs_scatter : per tile, wave-level multi-split ranking with 64-bit ballots (8 ballots per
//                64-entry row), block-local reorder through LDS so that each digit's run is
//                written contiguously (coalesced 16-byte stores), stable across tiles/blocks.
#include "common.h"
#include "terasort_gen.h"
#include "scan.h"
#include "rowkey.h"

#include <cstdlib>

namespace {

constexpr int kRadixBits = 8;
constexpr int kBins = 1 << kRadixBits;
constexpr int kItems = 8;                  // default entries per thread per tile
constexpr int kTile = kBlock * kItems;     // 2048 entries per tile (default geometry)
constexpr int kMaxGrid = 1024;             // workgroups for count/scatter (4 per CU)

template <typename T>
__device__ __forceinline__ uint32_t digit_of(const T& e, int shift) {
  return shift >= 64 ? (uint32_t)((e.hi >> (shift - 64)) & 0xFF)
                     : (uint32_t)((e.lo >> shift) & 0xFF);
}

__device__ __forceinline__ uint32_t digit_of(const E64& e, int shift) {
  return (uint32_t)((e.v >> shift) & 0xFF);
}

template <typename T>
__global__ __launch_bounds__(256) void rs_count(const T* __restrict__ in, uint64_t n, int shift,
                                                uint32_t* __restrict__ counts, uint32_t G,
                                                uint64_t per_block) {
  __shared__ uint32_t hist[4][kBins];
  const int t = threadIdx.x, w = wave_id();
  for (int i = t; i < 4 * kBins; i += kBlock) (&hist[0][0])[i] = 0;
  __syncthreads();
  const bool use_hi = shift >= 64;
  const int s = use_hi ? shift - 64 : shift;
  constexpr int W = sizeof(T) / 8;   // 64-bit words per entry
  const uint64_t* src = reinterpret_cast<const uint64_t*>(in) + (use_hi ? 1 : 0);
  const uint64_t beg = (uint64_t)blockIdx.x * per_block;
  const uint64_t end = beg + per_block < n ? beg + per_block : n;
  uint64_t i = beg + t;
  // 8 independent loads in flight per thread before the LDS atomics.
  for (; i + 7 * kBlock < end; i += 8 * kBlock) {
    uint64_t v[8];
#pragma unroll
    for (int k = 0; k < 8; ++k) v[k] = src[W * (i + k * kBlock)];
#pragma unroll
    for (int k = 0; k < 8; ++k) atomicAdd(&hist[w][(v[k] >> s) & 0xFF], 1u);
  }
  for (; i < end; i += kBlock) atomicAdd(&hist[w][(src[W * i] >> s) & 0xFF], 1u);
  __syncthreads();
  const uint32_t c = hist[0][t] + hist[1][t] + hist[2][t] + hist[3][t];
  counts[(uint64_t)t * G + blockIdx.x] = c;
}

// v2: all of a tile's loads are issued back to back and the NEXT tile is prefetched into
// registers while the current one is ranked and staged (software pipelining across tiles), so a
// workgroup's global-load latency overlaps its LDS ranking / scatter work.
// EXPAND (T = E64 only): the pass writes 16-byte E128 entries {lo = row index, hi = window +
// bias} instead, so a compact sort of narrow integer keys hands consumers the usual E128 layout.
template <typename T, int ITEMS, bool EXPAND = false>
__global__ __launch_bounds__(256) void rs_scatter_v2(const T* __restrict__ in, T* __restrict__ out,
                                                     uint64_t n, int shift,
                                                     const uint32_t* __restrict__ offsets, uint32_t G,
                                                     uint64_t per_block, uint64_t bias = 0) {
  constexpr int kTile = kBlock * ITEMS;
  __shared__ T stage[kTile];
  __shared__ uint32_t wcnt[4][kBins];
  __shared__ uint32_t goff[kBins];
  __shared__ uint32_t bstart[kBins];
  __shared__ uint32_t sc[4];
  const int t = threadIdx.x, w = wave_id(), l = lane_id();
  goff[t] = offsets[(uint64_t)t * G + blockIdx.x];
  const uint64_t beg = (uint64_t)blockIdx.x * per_block;
  const uint64_t end = beg + per_block < n ? beg + per_block : n;
  T cur[ITEMS], nxt[ITEMS];
  auto load_tile = [&](uint64_t base, T* dst) {
    const uint32_t c = (uint32_t)((end - base) < (uint64_t)kTile ? (end - base) : kTile);
#pragma unroll
    for (int r = 0; r < ITEMS; ++r) {
      const uint32_t pos = w * (kTile / 4) + r * 64 + l;
      if (pos < c) dst[r] = in[base + pos];
    }
  };
  if (beg < end) load_tile(beg, cur);
  for (uint64_t base = beg; base < end; base += kTile) {
    const uint32_t cnt = (uint32_t)((end - base) < (uint64_t)kTile ? (end - base) : kTile);
    if (base + kTile < end) load_tile(base + kTile, nxt);
    wcnt[0][t] = 0; wcnt[1][t] = 0; wcnt[2][t] = 0; wcnt[3][t] = 0;
    __syncthreads();
    uint32_t rk[ITEMS], dg[ITEMS];
#pragma unroll
    for (int r = 0; r < ITEMS; ++r) {
      const uint32_t pos = w * (kTile / 4) + r * 64 + l;
      const bool valid = pos < cnt;
      const uint32_t d = valid ? digit_of(cur[r], shift) : 0u;
      uint64_t peers = ballot64(valid);
#pragma unroll
      for (int k = 0; k < kRadixBits; ++k) {
        const bool bit = (d >> k) & 1u;
        const uint64_t b = ballot64(bit);
        peers &= bit ? b : ~b;
      }
      const uint32_t below = popc_below(peers);
      const uint32_t prior = wcnt[w][d];
      __builtin_amdgcn_wave_barrier();
      if (valid && below == 0) wcnt[w][d] = prior + (uint32_t)__popcll(peers);
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
    for (int r = 0; r < ITEMS; ++r) {
      const uint32_t pos = w * (kTile / 4) + r * 64 + l;
      if (pos < cnt) stage[bstart[dg[r]] + wcnt[w][dg[r]] + rk[r]] = cur[r];
    }
    __syncthreads();
#pragma unroll 4
    for (uint32_t j = t; j < cnt; j += kBlock) {
      const T v = stage[j];
      const uint32_t d = digit_of(v, shift);
      if constexpr (EXPAND) {
        const uint64_t w = reinterpret_cast<const uint64_t&>(v);
        E128 x;
        x.lo = (uint32_t)w;
        x.hi = (w >> 32) + bias;
        reinterpret_cast<E128*>(out)[(uint64_t)goff[d] + (j - bstart[d])] = x;
      } else {
        out[(uint64_t)goff[d] + (j - bstart[d])] = v;
      }
    }
    __syncthreads();
    goff[t] += tot;
#pragma unroll
    for (int r = 0; r < ITEMS; ++r) cur[r] = nxt[r];
  }
}

// v3: the v2 pass with the wave multisplit done through LDS lane masks instead of one ballot per
// digit bit: every lane ORs its bit into the mask of its digit (ds_or_b64), reads the mask back
// (= its peers), and the first peer clears it.  ~10 instructions per entry instead of ~45 for the
// 8 ballots, which were half of the v2 pass's issue time (profiles/pmc_counters_r2.md).  LDS
// instructions of one wave execute in order, so no barrier separates the OR, the read and the
// clear.
template <typename T, int ITEMS>
__global__ __launch_bounds__(256) void rs_scatter_v3(const T* __restrict__ in, T* __restrict__ out,
                                                     uint64_t n, int shift,
                                                     const uint32_t* __restrict__ offsets, uint32_t G,
                                                     uint64_t per_block) {
  constexpr int kTile = kBlock * ITEMS;
  __shared__ T stage[kTile];
  __shared__ uint32_t wcnt[4][kBins];
  __shared__ unsigned long long wmask[4][kBins];
  __shared__ uint32_t goff[kBins];
  __shared__ uint32_t bstart[kBins];
  __shared__ uint32_t sc[4];
  const int t = threadIdx.x, w = wave_id(), l = lane_id();
  goff[t] = offsets[(uint64_t)t * G + blockIdx.x];
  wmask[0][t] = 0ull; wmask[1][t] = 0ull; wmask[2][t] = 0ull; wmask[3][t] = 0ull;
  const uint64_t beg = (uint64_t)blockIdx.x * per_block;
  const uint64_t end = beg + per_block < n ? beg + per_block : n;
  T cur[ITEMS], nxt[ITEMS];
  auto load_tile = [&](uint64_t base, T* dst) {
    const uint32_t c = (uint32_t)((end - base) < (uint64_t)kTile ? (end - base) : kTile);
#pragma unroll
    for (int r = 0; r < ITEMS; ++r) {
      const uint32_t pos = w * (kTile / 4) + r * 64 + l;
      if (pos < c) dst[r] = in[base + pos];
    }
  };
  if (beg < end) load_tile(beg, cur);
  const unsigned long long lanebit = 1ull << l;
  for (uint64_t base = beg; base < end; base += kTile) {
    const uint32_t cnt = (uint32_t)((end - base) < (uint64_t)kTile ? (end - base) : kTile);
    if (base + kTile < end) load_tile(base + kTile, nxt);
    wcnt[0][t] = 0; wcnt[1][t] = 0; wcnt[2][t] = 0; wcnt[3][t] = 0;
    __syncthreads();
    uint32_t rk[ITEMS], dg[ITEMS];
#pragma unroll
    for (int r = 0; r < ITEMS; ++r) {
      const uint32_t pos = w * (kTile / 4) + r * 64 + l;
      const bool valid = pos < cnt;
      const uint32_t d = valid ? digit_of(cur[r], shift) : 0u;
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
    for (int r = 0; r < ITEMS; ++r) {
      const uint32_t pos = w * (kTile / 4) + r * 64 + l;
      if (pos < cnt) stage[bstart[dg[r]] + wcnt[w][dg[r]] + rk[r]] = cur[r];
    }
    __syncthreads();
#pragma unroll 4
    for (uint32_t j = t; j < cnt; j += kBlock) {
      const T v = stage[j];
      const uint32_t d = digit_of(v, shift);
      out[(uint64_t)goff[d] + (j - bstart[d])] = v;
    }
    __syncthreads();
    goff[t] += tot;
#pragma unroll
    for (int r = 0; r < ITEMS; ++r) cur[r] = nxt[r];
  }
}


// Wide-workgroup pass for the count-matrix sorts: NT threads (NT / 64 waves, up to 16), ITEMS
// entries per thread, the per-wave digit masks aliasing the stage (written only after the
// ranking), digit-indexed work on threads < 256.  No register prefetch: the other waves' loads
// are in flight while some rank or store.
template <typename T, int ITEMS, int NT>
__global__ __launch_bounds__(NT) void rs_scatter_w(const T* __restrict__ in, T* __restrict__ out, uint64_t n,
                                                   int shift, const uint32_t* __restrict__ offsets, uint32_t G,
                                                   uint64_t per_block) {
  constexpr int kT = NT * ITEMS, kNW = NT / 64;
  static_assert(NT >= kBins && kNW * kBins * 8 <= kT * (int)sizeof(T), "bins on 256 threads; masks fit the stage");
  __shared__ T stage[kT];
  __shared__ uint32_t wcnt[kNW][kBins];
  __shared__ uint32_t goff[kBins];
  __shared__ uint32_t bstart[kBins];
  __shared__ uint32_t sc[4];
  unsigned long long* wmask = reinterpret_cast<unsigned long long*>(stage);   // [kNW][kBins]
  const int t = threadIdx.x, w = wave_id(), l = lane_id();
  const uint64_t beg = (uint64_t)blockIdx.x * per_block;
  const uint64_t end = beg + per_block < n ? beg + per_block : n;
  if (beg >= end) return;                                   // uniform
  if (t < kBins) goff[t] = offsets[(uint64_t)t * G + blockIdx.x];
  const unsigned long long lanebit = 1ull << l;
  for (uint64_t base = beg; base < end; base += kT) {
    const uint32_t cnt = (uint32_t)((end - base) < (uint64_t)kT ? (end - base) : kT);
    T cur[ITEMS];
#pragma unroll
    for (int r = 0; r < ITEMS; ++r) {
      const uint32_t pos = w * (kT / kNW) + r * 64 + l;
      if (pos < cnt) cur[r] = in[base + pos];
    }
    for (int i = t; i < kNW * kBins; i += NT) {
      wmask[i] = 0ull;
      (&wcnt[0][0])[i] = 0;
    }
    __syncthreads();
    uint32_t rk[ITEMS], dg[ITEMS];
#pragma unroll
    for (int r = 0; r < ITEMS; ++r) {
      const uint32_t pos = w * (kT / kNW) + r * 64 + l;
      const bool valid = pos < cnt;
      const uint32_t d = valid ? digit_of(cur[r], shift) : 0u;
      unsigned long long* wm = wmask + w * kBins;
      if (valid) atomicOr(&wm[d], lanebit);
      __builtin_amdgcn_wave_barrier();
      const unsigned long long peers = valid ? wm[d] : 0ull;
      const uint32_t below = popc_below(peers);
      const uint32_t prior = wcnt[w][d];
      __builtin_amdgcn_wave_barrier();
      if (valid && below == 0) {
        wcnt[w][d] = prior + (uint32_t)__popcll(peers);
        wm[d] = 0ull;
      }
      __builtin_amdgcn_wave_barrier();
      rk[r] = prior + below;
      dg[r] = d;
    }
    __syncthreads();
    uint32_t tot = 0;
    if (t < kBins) {
#pragma unroll
      for (int k = 0; k < kNW; ++k) {
        const uint32_t c = wcnt[k][t];
        wcnt[k][t] = tot;
        tot += c;
      }
    }
    {
      const uint32_t inc = wave_inclusive_scan(tot);
      if (l == 63 && w < 4) sc[w] = inc;
      __syncthreads();
      const uint32_t b = (w > 0 ? sc[0] : 0) + (w > 1 ? sc[1] : 0) + (w > 2 ? sc[2] : 0);
      if (t < kBins) bstart[t] = b + inc - tot;
      __syncthreads();
    }
#pragma unroll
    for (int r = 0; r < ITEMS; ++r) {
      const uint32_t pos = w * (kT / kNW) + r * 64 + l;
      if (pos < cnt) stage[bstart[dg[r]] + wcnt[w][dg[r]] + rk[r]] = cur[r];
    }
    __syncthreads();
#pragma unroll 4
    for (uint32_t j = t; j < cnt; j += NT) {
      const T v = stage[j];
      const uint32_t d = digit_of(v, shift);
      out[(uint64_t)goff[d] + (j - bstart[d])] = v;
    }
    __syncthreads();
    if (t < kBins) goff[t] += tot;
  }
}

// E128 count-matrix sort pass: 1024 threads x 8 entries (8192-entry, 128 KB tiles) measured 4.24 vs
// 5.72 ms per pass of 5e8 entries for rs_scatter_v2 at 256 x 8 (profiles/r6/kernels/sort_shape_ab.txt),
// but two of three GPU-suite runs with the wide sort passes on hit an illegal address in a streamed
// GroupBy (profiles/r6/gpu_suite_r6zh_fault.log, gpu_suite_r6zm_fault.log) and none with them off:
// every count-matrix sort stays on its 256-thread kernel until that is understood.
#ifndef DR_SORT_NT
#define DR_SORT_NT 256                         // 256: rs_scatter_v2; 1024 (DR_SORT_ITEMS 8): rs_scatter_w
#endif
#ifndef DR_SORT_ITEMS
#define DR_SORT_ITEMS 8
#endif
// E64 dr_sort_u64 pass: 512 threads x 16 (8192-entry tiles) measured 6.74 vs 7.48 ms per 10 GB pass
// for rs_scatter_v3 at 256 x 16 (1024 x 16 6.87, two VGPRs spill); off, as DR_SORT_NT
#ifndef DR_SORT64_NT
#define DR_SORT64_NT 256                       // 256: rs_scatter_v3 x 16 (and v2 in the expand sort)
#endif
constexpr uint64_t kSortTile = (uint64_t)DR_SORT_NT * DR_SORT_ITEMS;

inline void sort_geometry(uint64_t n, uint32_t& G, uint64_t& per_block) {
  const uint64_t tile = kSortTile;
  uint64_t tiles = (n + tile - 1) / tile;
  if (tiles < 1) tiles = 1;
  G = (uint32_t)(tiles < (uint64_t)kMaxGrid ? tiles : (uint64_t)kMaxGrid);
  per_block = ((tiles + G - 1) / G) * tile;
}

void launch_scatter(const E128* in, E128* out, uint64_t n, int shift, const uint32_t* offsets, uint32_t G,
                    uint64_t per_block, hipStream_t s) {
#if DR_SORT_NT == 256
  rs_scatter_v2<E128, kItems><<<G, 256, 0, s>>>(in, out, n, shift, offsets, G, per_block);
#else
  rs_scatter_w<E128, DR_SORT_ITEMS, DR_SORT_NT><<<G, DR_SORT_NT, 0, s>>>(in, out, n, shift, offsets, G, per_block);
#endif
}

}  // namespace

// Workspace needed by dr_sort_u128 (bytes).
// Sized for the finest workgroup geometry of any sort that takes this workspace: kTile (2048-entry)
// tiles, finer than dr_sort_u64_expand's 4096 and the E128 / E64 passes' 8192 (a workspace sized
// by the coarser sort_geometry let the expand sort's count matrix overrun it).
DR_API uint64_t dr_sort_u128_workspace(uint64_t n) {
  uint64_t tiles = (n + kTile - 1) / kTile;
  if (tiles < 1) tiles = 1;
  const uint64_t G = tiles < (uint64_t)kMaxGrid ? tiles : (uint64_t)kMaxGrid;
  return ((uint64_t)kBins * G + 1024) * sizeof(uint32_t);
}

// Stable LSD radix sort of `n` entries on composite key bits [begin_bit, end_bit) (multiples of 8;
// bit 0 = lsb of lo, bit 64 = lsb of hi).  Ping-pongs between `keys` and `tmp`; *result_in_tmp
// tells the caller where the sorted sequence ended up.  Returns a hipError_t.
DR_API int dr_sort_u128(E128* keys, E128* tmp, uint64_t n, int begin_bit, int end_bit, void* ws,
                        hipStream_t s, int* result_in_tmp) {
  *result_in_tmp = 0;
  if (n == 0 || begin_bit >= end_bit) return 0;
  // passes are 8-bit digits at begin_bit, begin_bit + 8, ...; a digit may not straddle lo/hi, so
  // unaligned ranges must lie inside hi (the caller guarantees the bits above end_bit are constant
  // when (end_bit - begin_bit) is not a multiple of 8 or end_bit is unaligned)
  if (end_bit > 128 || begin_bit < 0 || ((end_bit - begin_bit) & 7)) return (int)hipErrorInvalidValue;
  if ((begin_bit & 7) && begin_bit < 64) return (int)hipErrorInvalidValue;
  if (n >= (1ull << 32)) return (int)hipErrorInvalidValue;
  uint32_t G; uint64_t per_block;
  sort_geometry(n, G, per_block);
  uint32_t* counts = reinterpret_cast<uint32_t*>(ws);
  uint32_t* partial = counts + (uint64_t)kBins * G;
  E128* src = keys;
  E128* dst = tmp;
  int flips = 0;
  for (int shift = begin_bit; shift < end_bit; shift += kRadixBits) {
    rs_count<<<G, 256, 0, s>>>(src, n, shift, counts, G, per_block);
    scan_inplace(counts, kBins * G, partial, s);
    launch_scatter(src, dst, n, shift, counts, G, per_block, s);
    E128* x = src; src = dst; dst = x;
    flips ^= 1;
  }
  DR_LAUNCH_CHECK();
  *result_in_tmp = flips;
  return 0;
}

// Per-digit totals of one pass (used by partition ops that only need the histogram of a small
// digit, e.g. destination ids): writes kBins uint64 totals of digit at `shift`.
namespace {
__global__ void rs_digit_totals(const uint32_t* __restrict__ counts_scanned, uint32_t G, uint64_t n,
                                uint64_t* __restrict__ starts) {
  const int t = threadIdx.x;
  starts[t] = counts_scanned[(uint64_t)t * G];
  if (t == 0) starts[kBins] = n;
}
}  // namespace

// One stable counting-sort pass on the 8-bit digit at `shift`; additionally reports the start
// offset of every digit value in `digit_starts` (kBins + 1 uint64, device).  This is the
// partition primitive (hash / range partition by destination id).
DR_API int dr_partition_pass_u128(const E128* in, E128* out, uint64_t n, int shift, void* ws,
                                  uint64_t* digit_starts, hipStream_t s) {
  if (n >= (1ull << 32) || (shift & 7) || shift > 120) return (int)hipErrorInvalidValue;
  if (n == 0) {
    hipMemsetAsync(digit_starts, 0, sizeof(uint64_t) * (kBins + 1), s);
    return 0;
  }
  uint32_t G; uint64_t per_block;
  sort_geometry(n, G, per_block);
  uint32_t* counts = reinterpret_cast<uint32_t*>(ws);
  uint32_t* partial = counts + (uint64_t)kBins * G;
  rs_count<<<G, 256, 0, s>>>(in, n, shift, counts, G, per_block);
  scan_inplace(counts, kBins * G, partial, s);
  rs_digit_totals<<<1, kBins, 0, s>>>(counts, G, n, digit_starts);
  launch_scatter(in, out, n, shift, counts, G, per_block, s);
  DR_LAUNCH_CHECK();
  return 0;
}

// ---------------------------------------------------------------------------------------------
// Key extraction from fixed-width rows: key bytes [key_off, key_off + key_len), key_len <= 12,
// compared as unsigned big-endian bytes (memcmp order, = TeraSort / byte-string order).
//   hi = key bytes 0..7, lo = key bytes 8..11 in bits 63..32, row index (idx_base + i) in 31..0.
namespace {
__global__ __launch_bounds__(256) void extract_keys_kernel(const uint8_t* __restrict__ rows, uint64_t n,
                                                           uint32_t stride, uint32_t key_off,
                                                           uint32_t key_len, uint32_t idx_base,
                                                           E128* __restrict__ out) {
  for (uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n;
       i += (uint64_t)gridDim.x * blockDim.x) {
    const uint8_t* r = rows + i * stride + key_off;
    uint64_t hi = 0, lo = 0;
    if (((stride | key_off) & 3) == 0) {
      const uint32_t* w = reinterpret_cast<const uint32_t*>(r);
      uint32_t b[3] = {0, 0, 0};
      const uint32_t nw = (key_len + 3) >> 2;
      for (uint32_t k = 0; k < nw; ++k) b[k] = bswap32(w[k]);
      // mask bytes beyond key_len
      uint32_t full = key_len;
      for (int k = 0; k < 3; ++k) {
        const int bytes = (int)full - 4 * k;
        if (bytes <= 0) b[k] = 0;
        else if (bytes < 4) b[k] &= 0xFFFFFFFFu << (8 * (4 - bytes));
      }
      hi = ((uint64_t)b[0] << 32) | b[1];
      lo = (uint64_t)b[2] << 32;
    } else {
      for (uint32_t k = 0; k < key_len; ++k) {
        const uint64_t v = r[k];
        if (k < 8) hi |= v << (8 * (7 - k));
        else lo |= v << (8 * (11 - k) + 32);
      }
    }
    E128 e;
    e.hi = hi;
    e.lo = lo | (uint32_t)(idx_base + (uint32_t)i);
    out[i] = e;
  }
}

// Specialisation for the TeraSort record (stride 100, 10-byte key at offset 0): three dword loads.
__global__ __launch_bounds__(256) void extract_keys_ts(const uint32_t* __restrict__ rows, uint64_t n,
                                                       uint32_t idx_base, E128* __restrict__ out) {
  for (uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n;
       i += (uint64_t)gridDim.x * blockDim.x) {
    const uint32_t* r = rows + i * 25;
    const uint32_t w0 = r[0], w1 = r[1], w2 = r[2];
    E128 e;
    e.hi = ((uint64_t)bswap32(w0) << 32) | bswap32(w1);
    e.lo = ((uint64_t)(bswap32(w2) & 0xFFFF0000u) << 32) | (uint32_t)(idx_base + (uint32_t)i);
    out[i] = e;
  }
}
}  // namespace

DR_API int dr_extract_keys(const uint8_t* rows, uint64_t n, uint32_t stride, uint32_t key_off,
                           uint32_t key_len, uint32_t idx_base, E128* out, hipStream_t s) {
  if (key_len == 0 || key_len > 12) return (int)hipErrorInvalidValue;
  if (n == 0) return 0;
  const unsigned g = grid_for(n, 256, 16384);
  if (stride == 100 && key_off == 0 && key_len == 10)
    extract_keys_ts<<<g, 256, 0, s>>>(reinterpret_cast<const uint32_t*>(rows), n, idx_base, out);
  else
    extract_keys_kernel<<<g, 256, 0, s>>>(rows, n, stride, key_off, key_len, idx_base, out);
  DR_LAUNCH_CHECK();
  return 0;
}

// ---------------------------------------------------------------------------------------------
// Row gather: out[i] = rows[idx(i)] for fixed-width rows (stride multiple of 4 bytes), where
// idx(i) is the low 32 bits of entries[i].lo (key-pointer sort result) or an explicit int64 index.
// A workgroup handles 256 output rows: indices staged in LDS, then the 256*W output dwords are
// written fully coalesced; each 64-lane load instruction reads ~2.5 rows of contiguous bytes.
namespace {
template <int WCONST>
__global__ __launch_bounds__(256) void gather_rows_kernel(const uint32_t* __restrict__ in,
                                                          uint32_t* __restrict__ out,
                                                          const E128* __restrict__ ent,
                                                          const int64_t* __restrict__ idx64,
                                                          uint64_t n, uint32_t Wdyn) {
  const uint32_t W = WCONST > 0 ? (uint32_t)WCONST : Wdyn;
  __shared__ uint64_t sidx[256];
  const int t = threadIdx.x;
  for (uint64_t row0 = (uint64_t)blockIdx.x * 256; row0 < n; row0 += (uint64_t)gridDim.x * 256) {
    if (row0 + t < n) sidx[t] = ent ? (uint64_t)(uint32_t)ent[row0 + t].lo : (uint64_t)idx64[row0 + t];
    __syncthreads();
    const uint32_t rows = (uint32_t)((n - row0) < 256 ? (n - row0) : 256);
    const uint32_t words = rows * W;
    uint32_t* o = out + row0 * W;
    uint32_t j = t;
    for (; j + 3 * 256 < words; j += 4 * 256) {
      uint32_t v[4];
#pragma unroll
      for (int k = 0; k < 4; ++k) {
        const uint32_t jj = j + k * 256;
        const uint32_t r = jj / W, c = jj - r * W;
        v[k] = in[sidx[r] * W + c];
      }
#pragma unroll
      for (int k = 0; k < 4; ++k) o[j + k * 256] = v[k];
    }
    for (; j < words; j += 256) {
      const uint32_t r = j / W, c = j - r * W;
      o[j] = in[sidx[r] * W + c];
    }
    __syncthreads();
  }
}
}  // namespace

// 16-byte vectorised gather for a compile-time stride S (multiple of 4): each output uint4 chunk
// is read from one source row (or stitched from two adjacent output rows' sources) and written
// with one 16-byte store; ~4x fewer memory instructions than the dword path.
namespace {
__device__ __forceinline__ uint4 load16_a4(const uint8_t* p) {
  uint4 v;
  __builtin_memcpy(&v, __builtin_assume_aligned(p, 4), 16);
  return v;
}

template <int S>
__global__ __launch_bounds__(256) void gather_rows_v4_kernel(const uint8_t* __restrict__ in, uint8_t* __restrict__ out,
                                                             const E128* __restrict__ ent,
                                                             const int64_t* __restrict__ idx64, uint64_t n) {
  static_assert(S % 4 == 0, "stride must be a multiple of 4");
  __shared__ uint64_t sidx[257];
  const int t = threadIdx.x;
  for (uint64_t row0 = (uint64_t)blockIdx.x * 256; row0 < n; row0 += (uint64_t)gridDim.x * 256) {
    const uint32_t rows = (uint32_t)((n - row0) < 256 ? (n - row0) : 256);
    if (t < (int)rows) sidx[t] = ent ? (uint64_t)(uint32_t)ent[row0 + t].lo : (uint64_t)idx64[row0 + t];
    __syncthreads();
    if (rows == 256) {
      constexpr uint32_t chunks = 256 * S / 16;
      uint4* o = reinterpret_cast<uint4*>(out + row0 * S);
      for (uint32_t c = t; c < chunks; c += 256) {
        const uint32_t b = 16 * c;
        const uint32_t r = b / S, off = b - r * S;
        const uint8_t* src = in + sidx[r] * S + off;
        uint4 v;
        if (off + 16 <= S) {
          v = load16_a4(src);
        } else {
          uint32_t w[4];
          const uint32_t k1 = (S - off) / 4;
          const uint32_t* a = reinterpret_cast<const uint32_t*>(src);
          const uint32_t* bnext = reinterpret_cast<const uint32_t*>(in + sidx[r + 1] * S);
#pragma unroll
          for (uint32_t k = 0; k < 4; ++k) w[k] = k < k1 ? a[k] : bnext[k - k1];
          v = make_uint4(w[0], w[1], w[2], w[3]);
        }
        o[c] = v;
      }
    } else {
      const uint32_t W = S / 4;
      const uint32_t words = rows * W;
      const uint32_t* inw = reinterpret_cast<const uint32_t*>(in);
      uint32_t* o = reinterpret_cast<uint32_t*>(out) + row0 * W;
      for (uint32_t j = t; j < words; j += 256) {
        const uint32_t r = j / W, c = j - r * W;
        o[j] = inw[sidx[r] * W + c];
      }
    }
    __syncthreads();
  }
}

}  // namespace

DR_API int dr_gather_rows(const uint8_t* rows, uint8_t* out, const E128* entries, const int64_t* idx,
                          uint64_t n, uint32_t stride, hipStream_t s) {
  if (stride == 100 && n > 0 && (((uintptr_t)out) & 15) == 0) {
    gather_rows_v4_kernel<100><<<grid_for(n, 256, 16384), 256, 0, s>>>(rows, out, entries, idx, n);
    DR_LAUNCH_CHECK();
    return 0;
  }
  if (stride == 0 || (stride & 3)) return (int)hipErrorInvalidValue;
  if (n == 0) return 0;
  const uint32_t W = stride / 4;
  const unsigned g = grid_for(n, 256, 16384);
  const uint32_t* in = reinterpret_cast<const uint32_t*>(rows);
  uint32_t* o = reinterpret_cast<uint32_t*>(out);
  if (W == 25)
    gather_rows_kernel<25><<<g, 256, 0, s>>>(in, o, entries, idx, n, W);
  else
    gather_rows_kernel<0><<<g, 256, 0, s>>>(in, o, entries, idx, n, W);
  DR_LAUNCH_CHECK();
  return 0;
}

// ---------------------------------------------------------------------------------------------
// Range destination: for each entry, dest = #separators strictly below its key (ascending) or
// strictly above (descending).  Key = (hi, lo & lo_mask).  Separators live in LDS (<= 255).
// Writes (hi = dest, lo = original lo) to `out` (may alias `in`), ready for one partition pass
// at shift 64.  Mirrors DryadLinqVertex.RangePartition + DryadLinqUtil.BinarySearch
// (reference LinqToDryad/DryadLinqVertex.cs:4909-5151, DryadLinqUtil.cs:112-140).
namespace {
__global__ __launch_bounds__(256) void range_dest_kernel(const E128* __restrict__ in, E128* __restrict__ out,
                                                         uint64_t n, const E128* __restrict__ seps,
                                                         uint32_t nsep, uint64_t lo_mask, int desc,
                                                         uint32_t subs, uint32_t ranks) {
  __shared__ uint64_t shi[256], slo[256];
  for (uint32_t k = threadIdx.x; k < nsep; k += blockDim.x) {
    shi[k] = seps[k].hi;
    slo[k] = seps[k].lo & lo_mask;
  }
  __syncthreads();
  for (uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n;
       i += (uint64_t)gridDim.x * blockDim.x) {
    E128 e = in[i];
    const uint64_t kh = e.hi, kl = e.lo & lo_mask;
    // branchless binary search for the count of separators "before" the key
    uint32_t lo = 0, hi = nsep;
    while (lo < hi) {
      const uint32_t mid = (lo + hi) >> 1;
      const uint64_t sh = shi[mid], sl = slo[mid];
      const bool before = desc ? (sh > kh || (sh == kh && sl > kl)) : (sh < kh || (sh == kh && sl < kl));
      lo = before ? mid + 1 : lo;
      hi = before ? hi : mid;
    }
    // sub-range pipelining: key range g = rank * subs + sub is renumbered sub-major
    // (sub * ranks + rank) so that one partition pass lays out round `sub` of the exchange as one
    // contiguous destination-ordered block
    e.hi = subs > 1 ? (uint64_t)((lo % subs) * ranks + lo / subs) : (uint64_t)lo;
    out[i] = e;
  }
}
}  // namespace

DR_API int dr_range_dest_u128(const E128* in, E128* out, uint64_t n, const E128* seps, uint32_t nsep,
                              uint64_t lo_mask, int descending, uint32_t subs, uint32_t ranks,
                              hipStream_t s) {
  if (nsep > 255) return (int)hipErrorInvalidValue;
  if (subs > 1 && (uint64_t)subs * ranks != (uint64_t)nsep + 1) return (int)hipErrorInvalidValue;
  if (n == 0) return 0;
  range_dest_kernel<<<grid_for(n, 256, 16384), 256, 0, s>>>(in, out, n, seps, nsep, lo_mask, descending,
                                                            subs, ranks);
  DR_LAUNCH_CHECK();
  return 0;
}

// ---------------------------------------------------------------------------------------------
// Bucket scatter of whole rows (the send-buffer pack of a range / hash shuffle): rows[i] goes to
// its bucket's contiguous region, bucket = low byte of entries[i].hi (from dr_range_dest_u128 or
// a hash destination), stable within a bucket.  Replaces "partition the entries, then gather the
// rows through them": that gather reads every 100-byte row at a scattered address (the partition
// interleaves up to 256 streams); here each 512-row tile is read coalesced into LDS, ranked by
// bucket with the radix-scatter ballots, and each bucket's rows are written as one contiguous run.
namespace {
constexpr int kBsTile = 512;
constexpr int kBsMaxW = 32;   // dwords per row held in LDS (stride <= 128 bytes)

template <int WC>
__global__ __launch_bounds__(256) void bucket_scatter_rows_kernel(const E128* __restrict__ ent,
                                                                  const uint32_t* __restrict__ rows,
                                                                  uint32_t* __restrict__ out, uint64_t n,
                                                                  uint32_t Wdyn,
                                                                  const uint32_t* __restrict__ offsets,
                                                                  uint32_t G, uint64_t per_block) {
  constexpr int ITEMS = kBsTile / kBlock;
  constexpr int LW = WC > 0 ? WC : kBsMaxW;
  const uint32_t W = WC > 0 ? (uint32_t)WC : Wdyn;
  __shared__ uint32_t srow[kBsTile * LW];
  __shared__ uint16_t perm[kBsTile];
  __shared__ uint8_t dslot[kBsTile];
  __shared__ uint32_t wcnt[4][kBins];
  __shared__ uint32_t goff[kBins];
  __shared__ uint32_t bstart[kBins];
  __shared__ uint32_t sc[4];
  const int t = threadIdx.x, w = wave_id(), l = lane_id();
  goff[t] = offsets[(uint64_t)t * G + blockIdx.x];
  const uint64_t beg = (uint64_t)blockIdx.x * per_block;
  const uint64_t end = beg + per_block < n ? beg + per_block : n;
  for (uint64_t base = beg; base < end; base += kBsTile) {
    const uint32_t cnt = (uint32_t)((end - base) < (uint64_t)kBsTile ? (end - base) : kBsTile);
    const uint32_t words = cnt * W;
    const uint32_t* src = rows + base * W;
    for (uint32_t j = t; j < words; j += kBlock) srow[j] = src[j];
    wcnt[0][t] = 0; wcnt[1][t] = 0; wcnt[2][t] = 0; wcnt[3][t] = 0;
    __syncthreads();
    uint32_t rk[ITEMS], dg[ITEMS];
#pragma unroll
    for (int r = 0; r < ITEMS; ++r) {
      const uint32_t pos = w * (kBsTile / 4) + r * 64 + l;
      const bool valid = pos < cnt;
      const uint32_t d = valid ? (uint32_t)(ent[base + pos].hi & 0xFF) : 0u;
      uint64_t peers = ballot64(valid);
#pragma unroll
      for (int k = 0; k < kRadixBits; ++k) {
        const bool bit = (d >> k) & 1u;
        const uint64_t b = ballot64(bit);
        peers &= bit ? b : ~b;
      }
      const uint32_t below = popc_below(peers);
      const uint32_t prior = wcnt[w][d];
      __builtin_amdgcn_wave_barrier();
      if (valid && below == 0) wcnt[w][d] = prior + (uint32_t)__popcll(peers);
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
    for (int r = 0; r < ITEMS; ++r) {
      const uint32_t pos = w * (kBsTile / 4) + r * 64 + l;
      if (pos < cnt) {
        const uint32_t slot = bstart[dg[r]] + wcnt[w][dg[r]] + rk[r];
        perm[slot] = (uint16_t)pos;
        dslot[slot] = (uint8_t)dg[r];
      }
    }
    __syncthreads();
    // slot-major dword copy: consecutive lanes write consecutive dwords of consecutive slots, and
    // consecutive slots of one bucket are consecutive rows of the output
    for (uint32_t q = t; q < words; q += kBlock) {
      const uint32_t j = q / W, c = q - j * W;
      const uint32_t d = dslot[j];
      out[((uint64_t)goff[d] + (j - bstart[d])) * W + c] = srow[(uint32_t)perm[j] * W + c];
    }
    __syncthreads();
    goff[t] += tot;
  }
}
// 100-byte rows (TeraSort records): the same scatter with the tile moved as 16-byte pieces and
// the next tile's pieces and bucket bytes loaded into registers while the current tile is ranked
// and written (the dword-at-a-time load above exposes one HBM round trip per few dwords).
constexpr int kBs25Pieces = (kBsTile * 25 / 4 + kBlock - 1) / kBlock;   // 13 per thread

__global__ __launch_bounds__(256) void bucket_scatter_rows25_kernel(const E128* __restrict__ ent,
                                                                    const uint32_t* __restrict__ rows,
                                                                    uint32_t* __restrict__ out, uint64_t n,
                                                                    const uint32_t* __restrict__ offsets,
                                                                    uint32_t G, uint64_t per_block) {
  constexpr int ITEMS = kBsTile / kBlock;
  constexpr uint32_t W = 25;
  __shared__ __attribute__((aligned(16))) uint32_t srow[kBsTile * W];
  __shared__ uint16_t perm[kBsTile];
  __shared__ uint8_t dslot[kBsTile];
  __shared__ uint32_t wcnt[4][kBins];
  __shared__ uint32_t goff[kBins];
  __shared__ uint32_t bstart[kBins];
  __shared__ uint32_t sc[4];
  const int t = threadIdx.x, w = wave_id(), l = lane_id();
  goff[t] = offsets[(uint64_t)t * G + blockIdx.x];
  const uint64_t beg = (uint64_t)blockIdx.x * per_block;
  const uint64_t end = beg + per_block < n ? beg + per_block : n;
  static_assert(kBs25Pieces == 13 && ITEMS == 2, "13 named piece registers, 2 bucket bytes");
  // named registers (an array here was placed in scratch)
  uint4 p0, p1, p2, p3, p4, p5, p6, p7, p8, p9, p10, p11, p12;
  uint32_t dn0, dn1;
#define DR_BS25_ALL(M) M(0, p0) M(1, p1) M(2, p2) M(3, p3) M(4, p4) M(5, p5) M(6, p6) M(7, p7) M(8, p8) \
  M(9, p9) M(10, p10) M(11, p11) M(12, p12)
  // a macro, not a lambda: arrays captured by a lambda are placed in scratch
#define DR_BS25_LD(I, P) { const uint32_t q_ = t + (I) * kBlock; P = s4_[q_ < pcs_ ? q_ : lp_]; }
#define DR_BS25_ISSUE(BASE)                                                                   \
  {                                                                                           \
    const uint64_t b_ = (BASE);                                                               \
    const uint32_t c_ = (uint32_t)((end - b_) < (uint64_t)kBsTile ? (end - b_) : kBsTile);    \
    const uint32_t pcs_ = c_ * W / 4;                                                         \
    const uint4* s4_ = reinterpret_cast<const uint4*>(rows + b_ * W);                         \
    const uint32_t lp_ = pcs_ ? pcs_ - 1 : 0;                                                 \
    DR_BS25_ALL(DR_BS25_LD)                      /* clamped, unconditional */                 \
    const uint32_t pa_ = w * (kBsTile / 4) + l, pb_ = pa_ + 64;                               \
    dn0 = (uint32_t)(ent[b_ + (pa_ < c_ ? pa_ : c_ - 1)].hi & 0xFF);                          \
    dn1 = (uint32_t)(ent[b_ + (pb_ < c_ ? pb_ : c_ - 1)].hi & 0xFF);                          \
  }
  if (beg >= end) return;                         // uniform: the whole workgroup leaves
  DR_BS25_ISSUE(beg)
  for (uint64_t base = beg; base < end; base += kBsTile) {
    const uint32_t cnt = (uint32_t)((end - base) < (uint64_t)kBsTile ? (end - base) : kBsTile);
    const uint32_t words = cnt * W, pieces = words / 4;
    uint4* s4 = reinterpret_cast<uint4*>(srow);
#define DR_BS25_ST(I, P) { const uint32_t q = t + (I) * kBlock; if (q < pieces) s4[q] = P; }
    DR_BS25_ALL(DR_BS25_ST)
#undef DR_BS25_ST
    for (uint32_t j = pieces * 4 + t; j < words; j += kBlock) srow[j] = rows[base * W + j];   // <= 3 tail dwords
    uint32_t dg[ITEMS] = {dn0, dn1};
    // unconditional (the last tile re-reads itself): an array assigned under a branch in the
    // loop was placed in scratch
    DR_BS25_ISSUE(base + kBsTile < end ? base + kBsTile : base)
    wcnt[0][t] = 0; wcnt[1][t] = 0; wcnt[2][t] = 0; wcnt[3][t] = 0;
    __syncthreads();
    uint32_t rk[ITEMS];
#pragma unroll
    for (int r = 0; r < ITEMS; ++r) {
      const uint32_t pos = w * (kBsTile / 4) + r * 64 + l;
      const bool valid = pos < cnt;
      const uint32_t d = valid ? dg[r] : 0u;
      uint64_t peers = ballot64(valid);
#pragma unroll
      for (int k = 0; k < kRadixBits; ++k) {
        const bool bit = (d >> k) & 1u;
        const uint64_t b = ballot64(bit);
        peers &= bit ? b : ~b;
      }
      const uint32_t below = popc_below(peers);
      const uint32_t prior = wcnt[w][d];
      __builtin_amdgcn_wave_barrier();
      if (valid && below == 0) wcnt[w][d] = prior + (uint32_t)__popcll(peers);
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
    for (int r = 0; r < ITEMS; ++r) {
      const uint32_t pos = w * (kBsTile / 4) + r * 64 + l;
      if (pos < cnt) {
        const uint32_t slot = bstart[dg[r]] + wcnt[w][dg[r]] + rk[r];
        perm[slot] = (uint16_t)pos;
        dslot[slot] = (uint8_t)dg[r];
      }
    }
    __syncthreads();
    for (uint32_t q = t; q < words; q += kBlock) {
      const uint32_t j = q / W, c = q - j * W;
      const uint32_t d = dslot[j];
      out[((uint64_t)goff[d] + (j - bstart[d])) * W + c] = srow[(uint32_t)perm[j] * W + c];
    }
    __syncthreads();
    goff[t] += tot;
  }
#undef DR_BS25_ISSUE
#undef DR_BS25_LD
#undef DR_BS25_ALL
}
}  // namespace

// Stable bucket scatter of `n` fixed-width rows (stride % 4 == 0, stride <= 128) by the low byte
// of entries[i].hi; `bucket_starts` (kBins + 1 uint64, device) receives every bucket's offset.
DR_API int dr_bucket_scatter_rows(const E128* ent, const uint8_t* rows, uint8_t* out, uint64_t n,
                                  uint32_t stride, void* ws, uint64_t* bucket_starts, hipStream_t s) {
  if (stride == 0 || (stride & 3) || stride > 4 * kBsMaxW || n >= (1ull << 32)) return (int)hipErrorInvalidValue;
  if (n == 0) {
    hipMemsetAsync(bucket_starts, 0, sizeof(uint64_t) * (kBins + 1), s);
    return 0;
  }
  uint32_t G; uint64_t per_block;
  sort_geometry(n, G, per_block);
  uint32_t* counts = reinterpret_cast<uint32_t*>(ws);
  uint32_t* partial = counts + (uint64_t)kBins * G;
  rs_count<<<G, 256, 0, s>>>(ent, n, 64, counts, G, per_block);
  scan_inplace(counts, kBins * G, partial, s);
  rs_digit_totals<<<1, kBins, 0, s>>>(counts, G, n, bucket_starts);
  const uint32_t W = stride / 4;
  const uint32_t* in = reinterpret_cast<const uint32_t*>(rows);
  uint32_t* o = reinterpret_cast<uint32_t*>(out);
  if (W == 25 && (((uintptr_t)rows) & 15) == 0)
    bucket_scatter_rows25_kernel<<<G, 256, 0, s>>>(ent, in, o, n, counts, G, per_block);
  else if (W == 25)
    bucket_scatter_rows_kernel<25><<<G, 256, 0, s>>>(ent, in, o, n, W, counts, G, per_block);
  else
    bucket_scatter_rows_kernel<0><<<G, 256, 0, s>>>(ent, in, o, n, W, counts, G, per_block);
  DR_LAUNCH_CHECK();
  return 0;
}


// ---------------------------------------------------------------------------------------------
// Prefix sort + tie fix-up: after a stable sort on hi only (64 key bits), runs of equal hi are
// re-ordered by the full lo word (remaining key bytes, then row index = stable order) by one
// thread per run.  Random keys (TeraSort) have essentially no such runs, saving two radix passes
// for 10-byte keys; a run longer than `max_run` sets *overflow so the caller falls back to the
// full-width sort.
namespace {
__global__ __launch_bounds__(256) void tie_fixup_kernel(E128* __restrict__ e, uint64_t n, uint32_t max_run,
                                                        uint32_t* __restrict__ overflow) {
  for (uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; i + 1 < n;
       i += (uint64_t)gridDim.x * blockDim.x) {
    const uint64_t h = e[i].hi;
    if (e[i + 1].hi != h) continue;
    if (i > 0 && e[i - 1].hi == h) continue;   // not the run start
    uint64_t j = i + 1;
    while (j + 1 < n && e[j + 1].hi == h && j - i < max_run) ++j;
    if (j - i >= max_run) {
      atomicOr(overflow, 1u);
      continue;
    }
    for (uint64_t a = i + 1; a <= j; ++a) {   // insertion sort by lo
      const E128 x = e[a];
      uint64_t b = a;
      while (b > i && e[b - 1].lo > x.lo) {
        e[b] = e[b - 1];
        --b;
      }
      e[b] = x;
    }
  }
}
}  // namespace

DR_API int dr_tie_fixup(E128* e, uint64_t n, uint32_t max_run, uint32_t* overflow, hipStream_t s) {
  if (n < 2) return 0;
  tie_fixup_kernel<<<grid_for(n, 256, 16384), 256, 0, s>>>(e, n, max_run, overflow);
  DR_LAUNCH_CHECK();
  return 0;
}

// ---------------------------------------------------------------------------------------------
// Hybrid sort, phase 2: segmented in-LDS sort of runs.  After a stable LSD sort on only the top
// window of varying key bits (3 passes for ~1e9 uniform keys instead of 8-10), entries sharing
// those bits form short runs (expected n / 2^window ~ 75).  Each workgroup owns the runs that
// START in its 2048-entry core and reads up to 256 more entries so a run spilling past the core
// is finished by its owner; positions inside a run are permuted in place, which never changes the
// run-id bits other workgroups read.  Rank of x in its run = #(y < x) + #(y == x, y before x)
// on the masked key: a stable sort on [begin_bit, end_bit) whatever the unmasked bits hold.
// Lanes of a wave walk the same run in lockstep, so the LDS reads are mostly broadcasts.
// A run that does not end inside the window sets *overflow (caller falls back to full LSD).
namespace {
constexpr int kSegCore = 2048, kSegExt = 256, kSegWin = kSegCore + kSegExt, kSegPer = kSegWin / 256;  // 9

// Comparison keys: the run is fixed by masked hi >> B (B = run_shift), so only the 64 key bits
// right below the run bits, k = (hi << (64 - B)) | (lo >> B), plus (REST) the masked low B bits
// of lo when the key extends that far, decide the order inside a run; position breaks ties.
template <bool REST>
__global__ __launch_bounds__(256) void seg_sort_kernel(E128* __restrict__ e, uint64_t n, int run_shift,
                                                       uint64_t mh, uint64_t ml, uint32_t* __restrict__ overflow) {
  __shared__ __attribute__((aligned(16))) uint64_t kk[kSegWin];
  __shared__ uint64_t rest[REST ? kSegWin : 1];
  __shared__ uint32_t rid32[kSegWin];
  __shared__ uint16_t rid_of[kSegWin];
  __shared__ uint16_t rstart[kSegWin + 1];
  __shared__ uint32_t sc[4];
  const int t = threadIdx.x;
  const int B = run_shift;
  const uint64_t c0 = (uint64_t)blockIdx.x * kSegCore;
  if (c0 >= n) return;
  const uint32_t core = (uint32_t)((n - c0) < (uint64_t)kSegCore ? (n - c0) : kSegCore);
  const uint64_t wend = (c0 + kSegWin) < n ? c0 + kSegWin : n;
  const uint32_t L = (uint32_t)(wend - c0);
  const uint64_t rest_mask = B ? (ml & ((1ull << B) - 1)) : 0ull;
  auto key64 = [&](uint64_t hi, uint64_t lo) -> uint64_t {
    return B ? ((hi << (64 - B)) | (lo >> B)) : lo;
  };
  // thread t loads (and later ranks) positions t, t + 256, ...: the unmasked entries stay in
  // registers; LDS gets the comparison keys and the low 32 bits of the run id (the window is at
  // most 32 bits wide for n < 2^32, and every key shares the bits above it)
  E128 mine[kSegPer];
#pragma unroll
  for (int k = 0; k < kSegPer; ++k) {
    const uint32_t i = t + k * 256;
    if (i < L) {
      mine[k] = e[c0 + i];
      const uint64_t h = mine[k].hi & mh, lo = mine[k].lo & ml;
      kk[i] = key64(h, lo);
      if (REST) rest[i] = lo & rest_mask;
      rid32[i] = (uint32_t)(h >> B);
    }
  }
  const uint32_t prev_rid = (c0 > 0) ? (uint32_t)((e[c0 - 1].hi & mh) >> B) : 0u;
  __syncthreads();
  uint32_t f = 0;
#pragma unroll
  for (int k = 0; k < kSegPer; ++k) {
    const uint32_t p = t * kSegPer + k;
    if (p < L) {
      const uint32_t r = rid32[p];
      const bool start = (p == 0) ? (c0 == 0 || prev_rid != r) : (rid32[p - 1] != r);
      if (start) f |= 1u << k;
    }
  }
  uint32_t nruns;
  const uint32_t base = block_exclusive_scan256((uint32_t)__popc(f), sc, nruns);
  uint32_t id = base;
#pragma unroll
  for (int k = 0; k < kSegPer; ++k) {
    const uint32_t p = t * kSegPer + k;
    if (p < L) {
      if (f & (1u << k)) { rstart[id] = (uint16_t)p; ++id; }
      rid_of[p] = (uint16_t)(id - 1);   // 0xFFFF: run started before this window
    }
  }
  if (t == 0) rstart[nruns] = (uint16_t)L;
  __syncthreads();
  const bool open_end = wend < n;
#pragma unroll
  for (int k = 0; k < kSegPer; ++k) {
    const uint32_t p = t + k * 256;
    if (p >= L) continue;
    const uint32_t r = rid_of[p];
    if (r == 0xFFFFu) continue;
    const uint32_t rs = rstart[r];
    if (rs >= core) continue;                       // owned by the next workgroup
    if (open_end && r + 1 == nruns) {               // run may continue past the window
      atomicOr(overflow, 1u);
      continue;
    }
    const uint32_t re = rstart[r + 1];
    if (re - rs == 1) continue;
    const uint64_t kx = kk[p];
    const uint64_t rx = REST ? rest[p] : 0ull;
    // rank = #{y in run : (k_y, rest_y, j) < (k_x, rest_x, p)}
    uint32_t cnt = 0;
    uint32_t j = rs;
    if (!REST) {
      for (; j < (rs & ~1u) + 2 && j < re; ++j) cnt += (kk[j] < kx || (kk[j] == kx && j < p)) ? 1u : 0u;
      for (; j + 4 <= re; j += 4) {   // 16-byte aligned pairs: two ds_read_b128 per 4 keys
        const ulonglong2 y0 = *reinterpret_cast<const ulonglong2*>(&kk[j]);
        const ulonglong2 y1 = *reinterpret_cast<const ulonglong2*>(&kk[j + 2]);
        cnt += (y0.x < kx || (y0.x == kx && j < p)) ? 1u : 0u;
        cnt += (y0.y < kx || (y0.y == kx && j + 1 < p)) ? 1u : 0u;
        cnt += (y1.x < kx || (y1.x == kx && j + 2 < p)) ? 1u : 0u;
        cnt += (y1.y < kx || (y1.y == kx && j + 3 < p)) ? 1u : 0u;
      }
    }
    for (; j < re; ++j) {
      const uint64_t y = kk[j];
      const uint64_t ry = REST ? rest[j] : 0ull;
      cnt += (y < kx || (y == kx && (ry < rx || (ry == rx && j < p)))) ? 1u : 0u;
    }
    e[c0 + rs + cnt] = mine[k];
  }
}

// [min, max] of hi over all entries (the hybrid sort skips the common prefix of all keys).
__global__ __launch_bounds__(256) void hi_range_kernel(const E128* __restrict__ e, uint64_t n,
                                                       unsigned long long* __restrict__ range) {
  uint64_t mn = ~0ull, mx = 0;
  for (uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (uint64_t)gridDim.x * blockDim.x) {
    const uint64_t h = e[i].hi;
    mn = h < mn ? h : mn;
    mx = h > mx ? h : mx;
  }
#pragma unroll
  for (int m = 32; m >= 1; m >>= 1) {
    const uint64_t a = __shfl_xor(mn, m, 64), b = __shfl_xor(mx, m, 64);
    mn = a < mn ? a : mn;
    mx = b > mx ? b : mx;
  }
  if (lane_id() == 0) {
    atomicMin(range, (unsigned long long)mn);
    atomicMax(range + 1, (unsigned long long)mx);
  }
}
}  // namespace

DR_API int dr_seg_sort_runs(E128* e, uint64_t n, int run_shift, uint64_t mask_hi, uint64_t mask_lo,
                            uint32_t* overflow, hipStream_t s) {
  if (run_shift < 0 || run_shift > 63) return (int)hipErrorInvalidValue;
  if (n < 2) return 0;
  const uint64_t g = (n + kSegCore - 1) / kSegCore;
  const bool rest = run_shift > 0 && (mask_lo & ((1ull << run_shift) - 1)) != 0;
  if (rest)
    seg_sort_kernel<true><<<(unsigned)g, 256, 0, s>>>(e, n, run_shift, mask_hi, mask_lo, overflow);
  else
    seg_sort_kernel<false><<<(unsigned)g, 256, 0, s>>>(e, n, run_shift, mask_hi, mask_lo, overflow);
  DR_LAUNCH_CHECK();
  return 0;
}

// [min, max] of entries[].hi into range[0..1] (caller initialises to {~0, 0}).
DR_API int dr_hi_range(const E128* e, uint64_t n, uint64_t* range, hipStream_t s) {
  if (n == 0) return 0;
  hi_range_kernel<<<grid_for(n, 256 * 8, 4096), 256, 0, s>>>(e, n, reinterpret_cast<unsigned long long*>(range));
  DR_LAUNCH_CHECK();
  return 0;
}

// ---------------------------------------------------------------------------------------------
// Payload-carrying sort (32-byte E256 / 40-byte E320 entries).  A GroupBy whose aggregates fold
// at most three (four) 8-byte columns sorts the values WITH the key: 4 LSD passes move 2x the bytes of a key-pointer
// sort, but the segmented reduction afterwards streams the sorted array instead of gathering
// every value column through a random row permutation (which runs at the HBM line-rate limit:
// one 128-byte line per 8-byte value).
namespace {

template <typename T>
__global__ __launch_bounds__(256) void pack_wide_kernel(const int64_t* __restrict__ key, int64_t bias,
                                                        const uint64_t* __restrict__ v0, const uint64_t* __restrict__ v1,
                                                        const uint64_t* __restrict__ v2, const uint64_t* __restrict__ v3,
                                                        uint64_t n, T* __restrict__ out) {
  constexpr int W = sizeof(T) / 8;
  for (uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (uint64_t)gridDim.x * blockDim.x) {
    uint64_t w[W];
    w[1] = key ? (uint64_t)key[i] - (uint64_t)bias : 0ull;   // key - min: >= 0, unsigned order = signed order
    w[0] = v0 ? v0[i] : 0ull;
    w[2] = v1 ? v1[i] : 0ull;
    w[3] = v2 ? v2[i] : 0ull;
    if constexpr (W > 4) w[4] = v3 ? v3[i] : 0ull;
    uint64_t* o = reinterpret_cast<uint64_t*>(out + i);
#pragma unroll
    for (int k = 0; k < W; ++k) o[k] = w[k];
  }
}

// flags[i] = 1 where hi differs from the previous entry's (entries `words` 64-bit words apart)
__global__ __launch_bounds__(256) void hi_flags_kernel(const uint64_t* __restrict__ e, uint32_t words, uint64_t n,
                                                       int64_t* __restrict__ flags) {
  for (uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (uint64_t)gridDim.x * blockDim.x)
    flags[i] = (i == 0 || e[(i - 1) * words + 1] != e[i * words + 1]) ? 1 : 0;
}

}  // namespace

// Wide sort entries (words = 4: E256, 5: E320) from an int64 key column (hi = key - bias, bias =
// the column minimum; key == nullptr leaves hi zero: a row-major value buffer) and up to
// words - 1 8-byte value columns (nullptr = absent) in lo, p0, ...
DR_API int dr_pack_wide(int words, const int64_t* key, int64_t bias, const uint64_t* v0, const uint64_t* v1,
                        const uint64_t* v2, const uint64_t* v3, uint64_t n, void* out, hipStream_t s) {
  if (n == 0) return 0;
  const unsigned g = grid_for(n, 256, 16384);
  if (words == 4) pack_wide_kernel<E256><<<g, 256, 0, s>>>(key, bias, v0, v1, v2, nullptr, n, static_cast<E256*>(out));
  else if (words == 5) pack_wide_kernel<E320><<<g, 256, 0, s>>>(key, bias, v0, v1, v2, v3, n, static_cast<E320*>(out));
  else return (int)hipErrorInvalidValue;
  DR_LAUNCH_CHECK();
  return 0;
}

DR_API int dr_hi_flags(const uint64_t* entries, uint32_t words, uint64_t n, int64_t* flags, hipStream_t s) {
  if (n == 0) return 0;
  if (words < 2 || words > 5) return (int)hipErrorInvalidValue;
  hi_flags_kernel<<<grid_for(n, 256, 16384), 256, 0, s>>>(entries, words, n, flags);
  DR_LAUNCH_CHECK();
  return 0;
}

namespace {

// NT = 1024 (rs_scatter_w): one wide workgroup per CU with a 4096-entry E256 tile (128 KiB) or a
// 3072-entry E320 tile (120 KiB): E256 pass 3.21 vs 4.47 ms for rs_scatter_v2 at 256 threads x 8
// (2048-entry, 64 KiB tiles; profiles/r6/kernels/sortwide_ab.txt).  NT = 256 selects rs_scatter_v2.
// Off by default like DR_SORT_NT (256 threads x 8 E256 / x 4 E320 through rs_scatter_v2).
#ifndef DR_SORTW_NT
#define DR_SORTW_NT 256
#endif
#ifndef DR_SORTW_ITEMS256
#define DR_SORTW_ITEMS256 8
#endif
#ifndef DR_SORTW_ITEMS320
#define DR_SORTW_ITEMS320 4
#endif
template <typename T, int ITEMS, int NT>
int sort_wide(T* keys, T* tmp, uint64_t n, int begin_bit, int end_bit, void* ws, hipStream_t s, int* result_in_tmp) {
  const uint64_t tile = (uint64_t)NT * ITEMS;
  uint64_t tiles = (n + tile - 1) / tile;
  if (tiles < 1) tiles = 1;
  const uint32_t G = (uint32_t)(tiles < (uint64_t)kMaxGrid ? tiles : (uint64_t)kMaxGrid);
  const uint64_t per_block = ((tiles + G - 1) / G) * tile;
  uint32_t* counts = reinterpret_cast<uint32_t*>(ws);
  uint32_t* partial = counts + (uint64_t)kBins * G;
  T* src = keys;
  T* dst = tmp;
  int flips = 0;
  for (int shift = begin_bit; shift < end_bit; shift += kRadixBits) {
    rs_count<<<G, 256, 0, s>>>(src, n, shift, counts, G, per_block);
    scan_inplace(counts, kBins * G, partial, s);
    if constexpr (NT == 256)
      rs_scatter_v2<T, ITEMS><<<G, 256, 0, s>>>(src, dst, n, shift, counts, G, per_block);
    else
      rs_scatter_w<T, ITEMS, NT><<<G, NT, 0, s>>>(src, dst, n, shift, counts, G, per_block);
    T* x = src; src = dst; dst = x;
    flips ^= 1;
  }
  DR_LAUNCH_CHECK();
  *result_in_tmp = flips;
  return 0;
}

}  // namespace

// Stable LSD radix sort of wide entries (words = 4: E256, 5: E320) on composite key bits
// [begin_bit, end_bit) of (hi, lo); same contract as dr_sort_u128, workspace
// dr_sort_u256_workspace(n).
DR_API int dr_sort_wide(int words, void* keys, void* tmp, uint64_t n, int begin_bit, int end_bit, void* ws,
                        hipStream_t s, int* result_in_tmp) {
  *result_in_tmp = 0;
  if (n == 0 || begin_bit >= end_bit) return 0;
  if (end_bit > 128 || begin_bit < 0 || ((end_bit - begin_bit) & 7)) return (int)hipErrorInvalidValue;
  if ((begin_bit & 7) && begin_bit < 64) return (int)hipErrorInvalidValue;
  if (n >= (1ull << 32)) return (int)hipErrorInvalidValue;
  if (words == 4)
    return sort_wide<E256, DR_SORTW_ITEMS256, DR_SORTW_NT>(static_cast<E256*>(keys), static_cast<E256*>(tmp), n,
                                                           begin_bit, end_bit, ws, s, result_in_tmp);
  if (words == 5)
    return sort_wide<E320, DR_SORTW_ITEMS320, DR_SORTW_NT>(static_cast<E320*>(keys), static_cast<E320*>(tmp), n,
                                                           begin_bit, end_bit, ws, s, result_in_tmp);
  return (int)hipErrorInvalidValue;
}

DR_API uint64_t dr_sort_u256_workspace(uint64_t n) {
  (void)n;
  return ((uint64_t)kBins * kMaxGrid + 1024) * sizeof(uint32_t);
}

// ---------------------------------------------------------------------------------------------
// Compact row sort (fixed-width rows, byte-string key in memcmp order).
//
// The 16-byte key-pointer entries of the hybrid sort move 40 GB per LSD pass at 1.25e9 rows.  Here
// an entry is 8 bytes: the 32 key bits right below the common prefix of all keys (the "window")
// and the 32-bit row index.  A stable LSD sort over the window (4 passes at 1e9 rows, 20 GB each)
// leaves runs of equal windows (mean n / 2^32 ~ 0.3 extra entries per run for uniform keys); the
// row gather then finishes those runs itself: it reads the full keys of the rows of a
// multi-entry run (which it fetches anyway), ranks them in LDS and writes every row at its final
// position.  A run longer than the gather's LDS window sets *overflow (the caller falls back to
// the full-key hybrid sort).
namespace {

__global__ __launch_bounds__(256) void extract_keys64_kernel(const uint8_t* __restrict__ rows, uint64_t n,
                                                             uint32_t stride, uint32_t key_off, uint32_t key_len,
                                                             uint32_t P, uint32_t idx_base, E64* __restrict__ out) {
  const bool aligned = ((stride | key_off) & 3) == 0;
  for (uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (uint64_t)gridDim.x * blockDim.x) {
    uint64_t k0, k1;
    load_key128(rows + i * stride + key_off, key_len, aligned, k0, k1);
    E64 e;
    e.v = ((uint64_t)key_window(k0, k1, P) << 32) | (uint32_t)(idx_base + (uint32_t)i);
    out[i] = e;
  }
}

// ent[i] := (key bits [P, P + 32) of row (ent[i] & 0xFFFFFFFF)) << 32 | row: the next, more
// significant window of an LSD chain of compact sorts over a key longer than one window.
__global__ __launch_bounds__(256) void rekey64_kernel(const uint8_t* __restrict__ rows, uint32_t pitch,
                                                      uint32_t key_off, uint32_t key_len, uint32_t P,
                                                      E64* __restrict__ ent, uint64_t n) {
  const bool aligned = ((pitch | key_off) & 3) == 0;
  for (uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (uint64_t)gridDim.x * blockDim.x) {
    const uint32_t idx = (uint32_t)ent[i].v;
    uint64_t k0, k1;
    load_key128(rows + (uint64_t)idx * pitch + key_off, key_len, aligned, k0, k1);
    E64 e;
    e.v = ((uint64_t)key_window(k0, k1, P) << 32) | idx;
    ent[i] = e;
  }
}

// ent[i] := i << 32 | row: every entry its own run (the gather copies without a fix-up).
__global__ __launch_bounds__(256) void e64_position_window_kernel(E64* __restrict__ ent, uint64_t n) {
  for (uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (uint64_t)gridDim.x * blockDim.x) {
    E64 e;
    e.v = (i << 32) | (uint32_t)ent[i].v;
    ent[i] = e;
  }
}

constexpr int kGfCore = 256, kGfExt = 64, kGfWin = kGfCore + kGfExt;

// One workgroup per 256 output positions (grid-stride): owns the runs that START in its core and
// finishes them up to 64 positions past it; positions of a run started by the previous workgroup
// are left to that workgroup.  Rows are copied dword-wise, output-coalesced (gather_rows_kernel).
template <int WC, bool NT = false>
__global__ __launch_bounds__(256) void gather_fixup_kernel(const uint32_t* __restrict__ rows, uint32_t* __restrict__ out,
                                                           const E64* __restrict__ ent, uint64_t n, uint32_t Wdyn,
                                                           uint32_t key_off, uint32_t key_len, int run_shift,
                                                           uint32_t* __restrict__ overflow,
                                                           const int32_t* __restrict__ err) {
  if (err != nullptr && *err != 0) return;     // the look-back sort failed: the entries are no permutation
  const uint32_t W = WC > 0 ? (uint32_t)WC : Wdyn;
  const uint32_t Win = W;
  __shared__ uint32_t rid[kGfWin + 1];     // rid[p + 1] = run id of window position p; rid[0] = position -1
  __shared__ uint32_t idx[kGfWin];
  __shared__ uint32_t sidx[kGfWin];
  __shared__ uint64_t kk0[kGfWin], kk1[kGfWin];
  __shared__ uint32_t own[2];
  const int t = threadIdx.x;
  const uint8_t* rbytes = reinterpret_cast<const uint8_t*>(rows);
  const bool aligned = (((Win * 4) | key_off) & 3) == 0;
  for (uint64_t c0 = (uint64_t)blockIdx.x * kGfCore; c0 < n; c0 += (uint64_t)gridDim.x * kGfCore) {
    const uint32_t L = (uint32_t)((n - c0) < (uint64_t)kGfWin ? (n - c0) : kGfWin);
    const uint32_t core = L < (uint32_t)kGfCore ? L : (uint32_t)kGfCore;
    for (uint32_t p = t; p < L; p += kBlock) {
      const uint64_t v = ent[c0 + p].v;
      rid[p + 1] = (uint32_t)(v >> run_shift);
      uint32_t i = (uint32_t)v;
      if (i >= n) {                    // corrupt entries: never read past the rows (flag 2: redo)
        atomicOr(overflow, 2u);
        i = 0;
      }
      idx[p] = i;
    }
    if (t == 0) {
      rid[0] = c0 > 0 ? (uint32_t)(ent[c0 - 1].v >> run_shift) : 0u;
      own[0] = 0xFFFFFFFFu;
      own[1] = 0xFFFFFFFFu;
    }
    __syncthreads();
    for (uint32_t p = t; p < L; p += kBlock) {
      const bool start = (c0 + p == 0) || rid[p + 1] != rid[p];
      if (start) atomicMin(&own[p < core ? 0 : 1], p);
    }
    __syncthreads();
    const uint32_t ob = own[0];
    uint32_t oe = own[1];
    if (oe == 0xFFFFFFFFu && c0 + L == n) oe = L;
    if (ob == 0xFFFFFFFFu) {           // the whole core continues a run owned by a previous workgroup
      __syncthreads();
      continue;
    }
    if (oe == 0xFFFFFFFFu) {           // a run owned here does not end inside the window
      if (t == 0) atomicOr(overflow, 1u);
      __syncthreads();
      continue;
    }
    // phase A: keys of the rows in multi-entry runs
    for (uint32_t p = ob + t; p < oe; p += kBlock) {
      const bool multi = (p > ob && rid[p + 1] == rid[p]) || (p + 1 < oe && rid[p + 2] == rid[p + 1]);
      if (multi) {
        uint64_t k0, k1;
        load_key128(rbytes + (uint64_t)idx[p] * (Win * 4) + key_off, key_len, aligned, k0, k1);
        kk0[p] = k0;
        kk1[p] = k1;
      } else {
        sidx[p - ob] = idx[p];
      }
    }
    __syncthreads();
    // phase B: rank inside each run: (key, position) order = stable
    for (uint32_t p = ob + t; p < oe; p += kBlock) {
      const uint32_t r = rid[p + 1];
      const bool multi = (p > ob && rid[p] == r) || (p + 1 < oe && rid[p + 2] == r);
      if (!multi) continue;
      uint32_t rs = p, re = p + 1;
      while (rs > ob && rid[rs] == r) --rs;
      while (re < oe && rid[re + 1] == r) ++re;
      const uint64_t a0 = kk0[p], a1 = kk1[p];
      uint32_t cnt = 0;
      for (uint32_t q = rs; q < re; ++q) {
        const uint64_t b0 = kk0[q], b1 = kk1[q];
        cnt += (b0 < a0 || (b0 == a0 && (b1 < a1 || (b1 == a1 && q < p)))) ? 1u : 0u;
      }
      sidx[rs + cnt - ob] = idx[p];
    }
    __syncthreads();
    const uint32_t words = (oe - ob) * W;
    uint32_t* o = out + (c0 + ob) * W;
    uint32_t j = t;
    for (; j + 3 * kBlock < words; j += 4 * kBlock) {
      uint32_t v[4];
#pragma unroll
      for (int k = 0; k < 4; ++k) {
        const uint32_t jj = j + k * kBlock;
        const uint32_t r = jj / W, c = jj - r * W;
        v[k] = rows[(uint64_t)sidx[r] * Win + c];
      }
#pragma unroll
      for (int k = 0; k < 4; ++k) {
        if constexpr (NT) __builtin_nontemporal_store(v[k], o + j + k * kBlock);
        else o[j + k * kBlock] = v[k];
      }
    }
    for (; j < words; j += kBlock) {
      const uint32_t r = j / W, c = j - r * W;
      o[j] = rows[(uint64_t)sidx[r] * Win + c];
    }
    __syncthreads();
  }
}

// Row gather + run fix-up for 100-byte records stored at a 128-byte pitch, rows fetched FIRST:
// the window's rows [ob, oe) are requested in position order (8 lanes per aligned 128-byte line,
// 7 16-byte nontemporal loads hold the record, every load of the window in flight before any is
// used) and staged in LDS at the output's 100-byte pitch; runs of equal windows are then ranked
// from the staged keys (no second, dependent round trip to HBM for the keys of multi-entry
// runs), and the output is written from LDS in rank order as contiguous dwords.
// (1-GPU TeraSort step 103.5 -> 101.4 ms; the same staging of 100-byte-pitch rows with dword
// loads was slower than gather_fixup_kernel<25>: 84 -> 99-101 ms over 1.25e9 received rows.)
__global__ __launch_bounds__(256) void gather_fixup_staged_kernel(const uint32_t* __restrict__ rows,
                                                                  uint32_t* __restrict__ out,
                                                                  const E64* __restrict__ ent, uint64_t n,
                                                                  uint32_t key_off, uint32_t key_len, int run_shift,
                                                                  uint32_t* __restrict__ overflow,
                                                                  const int32_t* __restrict__ err) {
  if (err != nullptr && *err != 0) return;     // the look-back sort failed: the entries are no permutation
  constexpr uint32_t W = 25;
  __shared__ uint32_t rid[kGfWin + 1];     // rid[p + 1] = run id of window position p; rid[0] = position -1
  __shared__ uint32_t idx[kGfWin];
  __shared__ uint16_t slot[kGfWin];        // output position - ob -> staged row
  __shared__ __attribute__((aligned(16))) uint32_t stage[kGfWin * W];
  __shared__ uint32_t own[2];
  const int t = threadIdx.x;
  const uint8_t* sbytes = reinterpret_cast<const uint8_t*>(stage);
  const bool aligned = (key_off & 3) == 0;
  for (uint64_t c0 = (uint64_t)blockIdx.x * kGfCore; c0 < n; c0 += (uint64_t)gridDim.x * kGfCore) {
    const uint32_t L = (uint32_t)((n - c0) < (uint64_t)kGfWin ? (n - c0) : kGfWin);
    const uint32_t core = L < (uint32_t)kGfCore ? L : (uint32_t)kGfCore;
    for (uint32_t p = t; p < L; p += kBlock) {
      const uint64_t v = ent[c0 + p].v;
      rid[p + 1] = (uint32_t)(v >> run_shift);
      uint32_t i = (uint32_t)v;
      if (i >= n) {                    // corrupt entries: never read past the rows (flag 2: redo)
        atomicOr(overflow, 2u);
        i = 0;
      }
      idx[p] = i;
    }
    if (t == 0) {
      rid[0] = c0 > 0 ? (uint32_t)(ent[c0 - 1].v >> run_shift) : 0u;
      own[0] = 0xFFFFFFFFu;
      own[1] = 0xFFFFFFFFu;
    }
    __syncthreads();
    for (uint32_t p = t; p < L; p += kBlock) {
      const bool start = (c0 + p == 0) || rid[p + 1] != rid[p];
      if (start) atomicMin(&own[p < core ? 0 : 1], p);
    }
    __syncthreads();
    const uint32_t ob = own[0];
    uint32_t oe = own[1];
    if (oe == 0xFFFFFFFFu && c0 + L == n) oe = L;
    if (ob == 0xFFFFFFFFu) {           // the whole core continues a run owned by a previous workgroup
      __syncthreads();
      continue;
    }
    if (oe == 0xFFFFFFFFu) {           // a run owned here does not end inside the window
      if (t == 0) atomicOr(overflow, 1u);
      __syncthreads();
      continue;
    }
    const uint32_t nrows = oe - ob;
    // phase 1: fetch the rows in position order into the stage
    {
      constexpr int kRounds = kGfWin / 32;         // 32 rows per round (8 lanes each)
      const uint32_t g = t >> 3, sub = t & 7;
      const uint8_t* rb = reinterpret_cast<const uint8_t*>(rows);
      uint4 buf[kRounds];
#pragma unroll
      for (int k = 0; k < kRounds; ++k) {
        const uint32_t r = g + 32 * k;
        if (r < nrows && sub < 7) {
          const uint4* src = reinterpret_cast<const uint4*>(rb + (uint64_t)idx[ob + r] * 128 + sub * 16);
          buf[k].x = __builtin_nontemporal_load(&src->x);
          buf[k].y = __builtin_nontemporal_load(&src->y);
          buf[k].z = __builtin_nontemporal_load(&src->z);
          buf[k].w = __builtin_nontemporal_load(&src->w);
        }
      }
#pragma unroll
      for (int k = 0; k < kRounds; ++k) {
        const uint32_t r = g + 32 * k;
        if (r < nrows && sub < 7) {
          uint32_t* d = stage + r * W + sub * 4;
          d[0] = buf[k].x;
          if (sub < 6) {
            d[1] = buf[k].y;
            d[2] = buf[k].z;
            d[3] = buf[k].w;
          }
        }
      }
    }
    __syncthreads();
    // phase 2: rank inside each run of equal windows, (key, position) order = stable
    for (uint32_t p = ob + t; p < oe; p += kBlock) {
      const uint32_t r = rid[p + 1];
      const bool multi = (p > ob && rid[p] == r) || (p + 1 < oe && rid[p + 2] == r);
      if (!multi) {
        slot[p - ob] = (uint16_t)(p - ob);
        continue;
      }
      uint32_t rs = p, re = p + 1;
      while (rs > ob && rid[rs] == r) --rs;
      while (re < oe && rid[re + 1] == r) ++re;
      uint64_t a0, a1;
      load_key128(sbytes + (p - ob) * (W * 4) + key_off, key_len, aligned, a0, a1);
      uint32_t cnt = 0;
      for (uint32_t q = rs; q < re; ++q) {
        uint64_t b0, b1;
        load_key128(sbytes + (q - ob) * (W * 4) + key_off, key_len, aligned, b0, b1);
        cnt += (b0 < a0 || (b0 == a0 && (b1 < a1 || (b1 == a1 && q < p)))) ? 1u : 0u;
      }
      slot[rs + cnt - ob] = (uint16_t)(p - ob);
    }
    __syncthreads();
    // phase 3: the output rows from the stage in rank order
    const uint32_t words = nrows * W;
    uint32_t* o = out + (c0 + ob) * W;
    for (uint32_t j = t; j < words; j += kBlock) {
      const uint32_t r = j / W, c = j - r * W;
      __builtin_nontemporal_store(stage[(uint32_t)slot[r] * W + c], o + j);
    }
    __syncthreads();
  }
}

// Row gather + BUCKET sort for 100-byte records at a 128-byte pitch whose E64 entries are sorted
// on the top `win` window bits only (win = 64 - run_shift, e.g. 24 of the 32: one look-back radix
// pass fewer), so a run of equal run ids -- a key bucket -- averages tens of rows (~75 for 1.25e9
// rows at 24 bits) and is ordered here, in LDS, by the rest of its key (then by position: stable).
// A workgroup owns the runs that START in its kBkCore-position core and finishes them up to kBkExt
// positions past it (a longer run flags overflow bit 0 and the caller re-sorts).  Two windows in
// flight: while window j is ranked and stored from the LDS stage, the rows of window j + 1 are
// loading into registers (8 lanes per aligned 128-byte line) and the entries of window j + 2 too
// (the barriers wait on LDS traffic only).  Per window: the staged rows' 64 key bits after the run
// id become their sub-keys; an LDS counting sort on bin = ((run id - first) << 8 | next 8 key bits)
// >> bsh (bins ordered like the keys) places every row but the few sharing a bin, ranked by (run
// id, sub-key, full key, position); the window leaves in rank order as 16-byte stores.
constexpr uint32_t kBkCore = 352, kBkExt = 192, kBkWin = kBkCore + kBkExt, kBkThreads = 512;
constexpr uint32_t kBkBins = kBkThreads;
constexpr int kBkRounds = (kBkWin + 63) / 64;          // row-load rounds: 64 rows (8 lanes each) per round
static_assert(kBkWin <= 2 * kBkThreads, "two entries per thread");

__global__ __launch_bounds__(kBkThreads) __attribute__((amdgpu_waves_per_eu(4))) void gather_bucket_staged_kernel(
    const uint32_t* __restrict__ rows, uint32_t* __restrict__ out, const E64* __restrict__ ent, uint64_t n,
    uint32_t key_off, uint32_t key_len, int run_shift, uint32_t* __restrict__ overflow,
    const int32_t* __restrict__ err) {
  if (err != nullptr && *err != 0) return;     // the look-back sort failed: the entries are no permutation
  constexpr uint32_t W = 25;
  typedef uint32_t u32x4a __attribute__((ext_vector_type(4), aligned(4)));
  __shared__ uint32_t rid[2][kBkWin + 1];  // rid[b][p + 1] = run id of window position p; [b][0] = position -1
  __shared__ uint32_t idx[2][kBkWin];
  __shared__ uint64_t sk[kBkWin];          // staged row -> key bits [win, win + 64)
  __shared__ uint16_t slot[kBkWin];        // output position - ob -> staged row
  __shared__ uint16_t member[kBkWin];      // rows of bin b: member[bin start .. bin end)
  __shared__ uint32_t bcnt[kBkBins];
  __shared__ uint32_t bcur[kBkBins];
  __shared__ uint32_t wsum[kBkThreads / 64];
  __shared__ uint32_t own[2][2];
  __shared__ __attribute__((aligned(16))) uint32_t stage[kBkWin * W];
  const uint32_t t = threadIdx.x;
  const uint8_t* sbytes = reinterpret_cast<const uint8_t*>(stage);
  const uint8_t* rb8 = reinterpret_cast<const uint8_t*>(rows);
  const bool aligned = (key_off & 3) == 0;
  const int win = 64 - run_shift;
  const uint64_t step = (uint64_t)gridDim.x * kBkCore;
  const uint32_t g = t >> 3, sub = t & 7;

  uint64_t ev0 = 0, ev1 = 0, evp = 0;      // entries of the next window to publish (positions t, t + 512, -1)
  auto ent_load = [&](uint64_t c0) {
    if (c0 >= n) return;
    const uint64_t L = (n - c0) < (uint64_t)kBkWin ? (n - c0) : kBkWin;
    if (t < L) ev0 = ent[c0 + t].v;
    if (t + kBkThreads < L) ev1 = ent[c0 + t + kBkThreads].v;
    if (t == 0 && c0 > 0) evp = ent[c0 - 1].v;
  };
  // publish the loaded entries of the window at c0 into buffer b and find its owned range
  auto publish = [&](uint32_t b, uint64_t c0) {
    const uint32_t L = (uint32_t)((n - c0) < (uint64_t)kBkWin ? (n - c0) : kBkWin);
    if (t < L) {
      rid[b][t + 1] = (uint32_t)(ev0 >> run_shift);
      uint32_t i = (uint32_t)ev0;
      if (i >= n) {                    // corrupt entries: never read past the rows (flag 2: redo)
        atomicOr(overflow, 2u);
        i = 0;
      }
      idx[b][t] = i;
    }
    if (t + kBkThreads < L) {
      rid[b][t + kBkThreads + 1] = (uint32_t)(ev1 >> run_shift);
      uint32_t i = (uint32_t)ev1;
      if (i >= n) {
        atomicOr(overflow, 2u);
        i = 0;
      }
      idx[b][t + kBkThreads] = i;
    }
    if (t == 0) {
      rid[b][0] = c0 > 0 ? (uint32_t)(evp >> run_shift) : 0u;
      own[b][0] = 0xFFFFFFFFu;
      own[b][1] = 0xFFFFFFFFu;
    }
  };
  auto find_owned = [&](uint32_t b, uint64_t c0) {
    const uint32_t L = (uint32_t)((n - c0) < (uint64_t)kBkWin ? (n - c0) : kBkWin);
    const uint32_t core = L < kBkCore ? L : kBkCore;
    for (uint32_t p = t; p < L; p += kBkThreads) {
      const bool start = (c0 + p == 0) || rid[b][p + 1] != rid[b][p];
      if (start) atomicMin(&own[b][p < core ? 0 : 1], p);
    }
  };
  // owned range [ob, oe) of the published window (oe = ob: nothing to do; overflow flagged)
  auto owned = [&](uint32_t b, uint64_t c0, uint32_t& ob, uint32_t& oe) {
    const uint32_t L = (uint32_t)((n - c0) < (uint64_t)kBkWin ? (n - c0) : kBkWin);
    ob = own[b][0];
    oe = own[b][1];
    if (oe == 0xFFFFFFFFu && c0 + L == n) oe = L;
    if (ob == 0xFFFFFFFFu) {           // the whole core continues a run owned by a previous workgroup
      ob = oe = 0;
    } else if (oe == 0xFFFFFFFFu) {    // a run owned here does not end inside the window
      if (t == 0) atomicOr(overflow, 1u);
      ob = oe = 0;
    }
  };
  uint4 buf[kBkRounds];
  // every lane loads (rows past nrows re-read the last row's line, a cache hit): no branch around
  // the loads, so the compiler never has to wait for one load before issuing the next
  auto rows_load = [&](uint32_t b, uint32_t ob, uint32_t nrows) {
    const uint32_t last = nrows ? nrows - 1 : 0;
#pragma unroll
    for (int k = 0; k < kBkRounds; ++k) {
      const uint32_t r = g + 64 * k;
      const uint32_t i = idx[b][ob + (r < nrows ? r : last)];
      const uint4* src = reinterpret_cast<const uint4*>(rb8 + (uint64_t)i * 128 + sub * 16);
      buf[k].x = __builtin_nontemporal_load(&src->x);
      buf[k].y = __builtin_nontemporal_load(&src->y);
      buf[k].z = __builtin_nontemporal_load(&src->z);
      buf[k].w = __builtin_nontemporal_load(&src->w);
    }
  };

  // prologue: window 0 published and its rows loading, the entries of window 1 loading
  uint64_t c0 = (uint64_t)blockIdx.x * kBkCore;
  if (c0 >= n) return;
  ent_load(c0);
  publish(0, c0);
  __syncthreads();
  find_owned(0, c0);
  __syncthreads();
  uint32_t ob, oe;
  owned(0, c0, ob, oe);
  rows_load(0, ob, oe - ob);
  ent_load(c0 + step);
  for (uint32_t j = 0; c0 < n; ++j, c0 += step) {
    const uint32_t b = j & 1;
    const uint32_t nrows = oe - ob;
    const uint64_t c1 = c0 + step;
    // (1) this window's rows to the stage; the next window's entries published
#pragma unroll
    for (int k = 0; k < kBkRounds; ++k) {
      const uint32_t r = g + 64 * k;
      if (r < nrows && sub < 7) {
        uint32_t* d = stage + r * W + sub * 4;
        d[0] = buf[k].x;
        if (sub < 6) {
          d[1] = buf[k].y;
          d[2] = buf[k].z;
          d[3] = buf[k].w;
        }
      }
    }
    if (c1 < n) publish(b ^ 1, c1);
    bcnt[t] = 0;
    __syncthreads();
    // (2) sub-keys of the staged rows; the next window's owned range
    for (uint32_t r = t; r < nrows; r += kBkThreads) {
      uint64_t k0, k1;
      load_key128(sbytes + r * (W * 4) + key_off, key_len, aligned, k0, k1);
      sk[r] = (k0 << win) | (k1 >> (64 - win));
    }
    if (c1 < n) find_owned(b ^ 1, c1);
    __syncthreads();
    // (3) the next window's rows and the entries after it start loading
    uint32_t ob1 = 0, oe1 = 0;
    if (c1 < n) {
      owned(b ^ 1, c1, ob1, oe1);
      rows_load(b ^ 1, ob1, oe1 - ob1);
      ent_load(c1 + step);
    }
    // (4) this window: counting sort, in-bin rank, stores in rank order
    if (nrows > 0) {
      const uint32_t rid0 = rid[b][ob + 1];
      const uint64_t span = ((uint64_t)(rid[b][oe] - rid0) + 1) << 8;
      uint32_t bsh = 0;
      while ((span >> bsh) > kBkBins) ++bsh;
      auto bin_of = [&](uint32_t p) -> uint32_t {
        return (uint32_t)(((((uint64_t)(rid[b][p + 1] - rid0)) << 8) | (sk[p - ob] >> 56)) >> bsh);
      };
      for (uint32_t p = ob + t; p < oe; p += kBkThreads) atomicAdd(&bcnt[bin_of(p)], 1u);
      __syncthreads();
      {                                // exclusive scan of the kBkBins bins, one per lane
        const uint32_t c = bcnt[t];
        const uint32_t inc = wave_inclusive_scan(c);
        if (lane_id() == 63) wsum[wave_id()] = inc;
        __syncthreads();
        uint32_t run = inc - c;
        for (int w = 0; w < wave_id(); ++w) run += wsum[w];
        bcur[t] = run;
      }
      __syncthreads();
      for (uint32_t p = ob + t; p < oe; p += kBkThreads) member[atomicAdd(&bcur[bin_of(p)], 1u)] = (uint16_t)(p - ob);
      __syncthreads();
      for (uint32_t p = ob + t; p < oe; p += kBkThreads) {
        const uint32_t bn = bin_of(p), end = bcur[bn], beg = end - bcnt[bn];
        const uint32_t me = p - ob, ra = rid[b][p + 1];
        const uint64_t a = sk[me];
        uint32_t r = beg;
        bool full = false;
        uint64_t a0 = 0, a1 = 0;
        for (uint32_t m = beg; m < end; ++m) {
          const uint32_t x = member[m];
          if (x == me) continue;
          const uint32_t rbx = rid[b][x + ob + 1];
          const uint64_t bk = sk[x];
          if (rbx != ra || bk != a) {
            r += (rbx < ra || (rbx == ra && bk < a)) ? 1u : 0u;
            continue;
          }
          if (!full) {                 // equal sub-keys: the full key, then the position
            load_key128(sbytes + me * (W * 4) + key_off, key_len, aligned, a0, a1);
            full = true;
          }
          uint64_t b0, b1;
          load_key128(sbytes + x * (W * 4) + key_off, key_len, aligned, b0, b1);
          r += (b0 < a0 || (b0 == a0 && (b1 < a1 || (b1 == a1 && x < me)))) ? 1u : 0u;
        }
        slot[r] = (uint16_t)me;
      }
      __syncthreads();
      uint32_t* o = out + (c0 + ob) * W;
      for (uint32_t jj = g; jj < nrows; jj += kBkThreads / 8) {
        if (sub < 7) {
          const uint32_t* sr = stage + (uint32_t)slot[jj] * W + sub * 4;
          uint32_t* dst = o + jj * W + sub * 4;
          if (sub < 6) *reinterpret_cast<u32x4a*>(dst) = u32x4a{sr[0], sr[1], sr[2], sr[3]};
          else dst[0] = sr[0];
        }
      }
    }
    __syncthreads();
    ob = ob1;
    oe = oe1;
  }
}

}  // namespace

DR_API int dr_extract_keys64(const uint8_t* rows, uint64_t n, uint32_t stride, uint32_t key_off, uint32_t key_len,
                             uint32_t prefix_bits, uint32_t idx_base, E64* out, hipStream_t s) {
  if (key_len == 0 || key_len > 16 || key_off + key_len > stride) return (int)hipErrorInvalidValue;
  if (n == 0) return 0;
  if (n + idx_base > (1ull << 32)) return (int)hipErrorInvalidValue;
  extract_keys64_kernel<<<grid_for(n, 256, 16384), 256, 0, s>>>(rows, n, stride, key_off, key_len, prefix_bits,
                                                                idx_base, out);
  DR_LAUNCH_CHECK();
  return 0;
}

// Stable LSD radix sort of E64 entries on bits [begin_bit, end_bit) (multiples of 8, < 64 = the
// window); 16 entries per thread per tile (128 contiguous output bytes per digit run).
DR_API int dr_sort_u64(E64* keys, E64* tmp, uint64_t n, int begin_bit, int end_bit, void* ws, hipStream_t s,
                       int* result_in_tmp) {
  *result_in_tmp = 0;
  if (n == 0 || begin_bit >= end_bit) return 0;
  if (end_bit > 64 || begin_bit < 0 || (begin_bit & 7) || (end_bit & 7)) return (int)hipErrorInvalidValue;
  if (n >= (1ull << 32)) return (int)hipErrorInvalidValue;
  constexpr int ITEMS = 16;
  const uint64_t tile = (uint64_t)DR_SORT64_NT * ITEMS;
  uint64_t tiles = (n + tile - 1) / tile;
  if (tiles < 1) tiles = 1;
  const uint32_t G = (uint32_t)(tiles < (uint64_t)kMaxGrid ? tiles : (uint64_t)kMaxGrid);
  const uint64_t per_block = ((tiles + G - 1) / G) * tile;
  uint32_t* counts = reinterpret_cast<uint32_t*>(ws);
  uint32_t* partial = counts + (uint64_t)kBins * G;
  E64* src = keys;
  E64* dst = tmp;
  int flips = 0;
  for (int shift = begin_bit; shift < end_bit; shift += kRadixBits) {
    rs_count<<<G, 256, 0, s>>>(src, n, shift, counts, G, per_block);
    scan_inplace(counts, kBins * G, partial, s);
#if DR_SORT64_NT == 256
    rs_scatter_v3<E64, ITEMS><<<G, 256, 0, s>>>(src, dst, n, shift, counts, G, per_block);
#else
    rs_scatter_w<E64, ITEMS, DR_SORT64_NT><<<G, DR_SORT64_NT, 0, s>>>(src, dst, n, shift, counts, G, per_block);
#endif
    E64* x = src; src = dst; dst = x;
    flips ^= 1;
  }
  DR_LAUNCH_CHECK();
  *result_in_tmp = flips;
  return 0;
}

// Stable LSD sort of E64 entries on bits [begin_bit, end_bit) whose LAST pass writes E128 entries
// {lo = row index, hi = (entry >> 32) + bias} to `out` (n x 16 bytes, not aliasing keys/tmp): the
// sort of a narrow integer key (span < 2^32; entries = (norm key - norm min) << 32 | row) at half
// the traffic of the 16-byte sort, handing the E128 layout to segment / join consumers.
DR_API int dr_sort_u64_expand(E64* keys, E64* tmp, E128* out, uint64_t n, int begin_bit, int end_bit, uint64_t bias,
                              void* ws, hipStream_t s) {
  if (n == 0) return 0;
  if (end_bit > 64 || begin_bit < 32 || (begin_bit & 7) || (end_bit & 7) || begin_bit >= end_bit)
    return (int)hipErrorInvalidValue;
  if (n >= (1ull << 32)) return (int)hipErrorInvalidValue;
  constexpr int ITEMS = 16;
  // the dr_sort_u64 geometry (DR_SORT64_NT x 16 entries per tile); the last, expanding pass keeps
  // rs_scatter_v2 (256 threads walk the workgroup's slice in 4096-entry tiles)
  const uint64_t tile = (uint64_t)DR_SORT64_NT * ITEMS;
  uint64_t tiles = (n + tile - 1) / tile;
  if (tiles < 1) tiles = 1;
  const uint32_t G = (uint32_t)(tiles < (uint64_t)kMaxGrid ? tiles : (uint64_t)kMaxGrid);
  const uint64_t per_block = ((tiles + G - 1) / G) * tile;
  uint32_t* counts = reinterpret_cast<uint32_t*>(ws);
  uint32_t* partial = counts + (uint64_t)kBins * G;
  E64* src = keys;
  E64* dst = tmp;
  for (int shift = begin_bit; shift < end_bit; shift += kRadixBits) {
    rs_count<<<G, 256, 0, s>>>(src, n, shift, counts, G, per_block);
    scan_inplace(counts, kBins * G, partial, s);
    if (shift + kRadixBits >= end_bit) {
      rs_scatter_v2<E64, ITEMS, true><<<G, 256, 0, s>>>(src, reinterpret_cast<E64*>(out), n, shift, counts, G,
                                                        per_block, bias);
    } else {
#if DR_SORT64_NT == 256
      rs_scatter_v2<E64, ITEMS><<<G, 256, 0, s>>>(src, dst, n, shift, counts, G, per_block);
#else
      rs_scatter_w<E64, ITEMS, DR_SORT64_NT><<<G, DR_SORT64_NT, 0, s>>>(src, dst, n, shift, counts, G, per_block);
#endif
      E64* x = src; src = dst; dst = x;
    }
  }
  DR_LAUNCH_CHECK();
  return 0;
}

// ---------------------------------------------------------------------------------------------
// Single-histogram LSD sort of E64 entries with decoupled look-back ("onesweep").
//
// dr_sort_u64 reads the entries twice per pass: rs_count builds the per-workgroup digit counts of
// the pass, then rs_scatter_v3 moves them.  A digit's count over the whole array does not depend
// on the order, so here ONE read (os_hist_kernel) builds the histograms of every pass, and each
// scatter pass finds a tile's per-digit output offset from the tiles before it instead of from a
// count matrix:
//   * tiles (16384 entries) are claimed in order from a per-pass ticket counter, so every tile a
//     workgroup waits for belongs to a workgroup that is already running;
//   * a tile publishes its 256 digit counts as 8-byte {tag, value} granules (one agent-scope
//     atomic store each: the granule is its own flag), first tagged "aggregate of this tile", then,
//     once its prefix is known, "inclusive prefix up to this tile";
//   * digit d's thread walks back over the predecessors' granules, adding aggregates, until it
//     meets an inclusive prefix (tile 0 publishes its inclusive prefix at once).
// Tags are 2 * (pass + 1) + {0 aggregate, 1 inclusive}; the granules and tickets are zeroed by one
// memset per call, so a granule left by an earlier pass or call is never taken for this pass's.
// The ranking inside a tile and the LDS reorder are rs_scatter_v3's.  A spin that outlives
// kOsSpinLimit polls sets the error word and gives up (the prefix it has summed is a lower bound,
// so every store stays inside the output); the caller checks that word.
namespace {

#ifndef DR_OS_NT
#define DR_OS_NT 1024                          // look-back scatter workgroup: 16 waves, one per CU by LDS
#endif
#ifndef DR_OS_ITEMS
#define DR_OS_ITEMS 16                         // entries per thread: 16384-entry tiles (128 KB stage)
#endif
#ifndef DR_OS_LB
#define DR_OS_LB 4                             // look-back granules per round trip
#endif
// Tile shape A/B at 1.25e9 entries (profiles/r6/kernels/os_shape_ab.txt, per pass): 256 threads x 32
// 6.00 ms, 512 x 16 5.80, 512 x 32 6.12, 768 x 20 6.07, 1024 x 12 6.47, 1024 x 16 5.74 (LB 8: 5.86).
// Round 5's 256-thread sweep: 16 items 33.9 ms / 4 passes, 20: 32.7, 24: 29.3, 32: 25.1, 40: 34.6.
constexpr int kOsThreads = DR_OS_NT;
constexpr int kOsItems = DR_OS_ITEMS;
constexpr int kOsMaxPasses = 8;
constexpr uint32_t kOsHistGrid = 1024;
constexpr uint32_t kOsSpinLimit = 1u << 22;
constexpr uint64_t kOsHeader = 256;            // tickets[8] at 0, error word at 64
typedef __attribute__((address_space(1))) unsigned long long os_gu64;
typedef __attribute__((address_space(1))) unsigned int os_gu32;

inline uint64_t os_tiles(uint64_t n) {
  const uint64_t tile = (uint64_t)kOsThreads * kOsItems;
  return (n + tile - 1) / tile;
}

// workspace: [header | digit counts: 8 x 256 u32 | granules: tiles x 256 u64] (bytes), all zeroed
// per call
constexpr uint64_t kOsCounts = (uint64_t)kOsMaxPasses * kBins * 4;
inline uint64_t os_granule_bytes(uint64_t n) { return os_tiles(n) * kBins * 8; }
inline uint64_t os_workspace_bytes(uint64_t n) { return kOsHeader + kOsCounts + os_granule_bytes(n); }

// counts[p][d] += count of digit d of pass p (bits begin_bit + 8p ..) in this workgroup's slice
__global__ __launch_bounds__(256) void os_hist_kernel(const uint64_t* __restrict__ in, uint64_t n, int begin_bit,
                                                      int P, uint32_t* counts) {
  __shared__ uint32_t hist[4][kOsMaxPasses][kBins];
  const int t = threadIdx.x, w = wave_id();
  for (int i = t; i < 4 * kOsMaxPasses * kBins; i += kBlock) (&hist[0][0][0])[i] = 0;
  __syncthreads();
  const uint64_t per = (n + gridDim.x - 1) / gridDim.x;
  const uint64_t beg = (uint64_t)blockIdx.x * per;
  const uint64_t end = beg + per < n ? beg + per : n;
  uint64_t i = beg + t;
  for (; i + 7 * kBlock < end; i += 8 * kBlock) {
    uint64_t v[8];
#pragma unroll
    for (int k = 0; k < 8; ++k) v[k] = in[i + k * kBlock];
#pragma unroll
    for (int k = 0; k < 8; ++k) {
      const uint64_t x = v[k] >> begin_bit;
      for (int p = 0; p < P; ++p) atomicAdd(&hist[w][p][(x >> (8 * p)) & 0xFF], 1u);
    }
  }
  for (; i < end; i += kBlock) {
    const uint64_t x = in[i] >> begin_bit;
    for (int p = 0; p < P; ++p) atomicAdd(&hist[w][p][(x >> (8 * p)) & 0xFF], 1u);
  }
  __syncthreads();
  for (int p = 0; p < P; ++p) {
    const uint32_t c = hist[0][p][t] + hist[1][p][t] + hist[2][p][t] + hist[3][p][t];
    if (c) __hip_atomic_fetch_add((os_gu32*)(counts + p * kBins + t), c, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  }
}

// counts[p][d] += sum over a range of producer partials part[k][first + p][d] (k < parts; the
// partials cover the 4 digits of bits [32, 64), the sort the P = 4 - first digits from first)
__global__ __launch_bounds__(256) void os_hist_parts_kernel(const uint32_t* __restrict__ part, uint32_t parts,
                                                            int first, uint32_t* counts) {
  const int t = threadIdx.x;
  const uint32_t per = (parts + gridDim.x - 1) / gridDim.x;
  const uint32_t k0 = blockIdx.x * per, k1 = k0 + per < parts ? k0 + per : parts;
  uint32_t s[4] = {0, 0, 0, 0};
  for (uint32_t k = k0; k < k1; ++k) {
#pragma unroll
    for (int p = 0; p < 4; ++p) s[p] += p >= first ? part[((uint64_t)k * 4 + p) * kBins + t] : 0u;
  }
#pragma unroll
  for (int p = 0; p < 4; ++p)
    if (p >= first && s[p]) __hip_atomic_fetch_add((os_gu32*)(counts + (p - first) * kBins + t), s[p], __ATOMIC_RELAXED,
                                       __HIP_MEMORY_SCOPE_AGENT);
}

// counts[p][d] := exclusive prefix over the digits of pass p (one workgroup per pass).  A pass
// whose digits do not add up to n (producer histograms that belong to other entries) sets bit 1
// of *err: the scatter passes then store nothing (their offsets could leave the output).
__global__ __launch_bounds__(256) void os_hist_scan_kernel(uint32_t* __restrict__ counts, uint64_t n,
                                                           uint32_t* __restrict__ err) {
  __shared__ uint32_t sc[4];
  const int t = threadIdx.x, p = blockIdx.x;
  uint32_t total;
  const uint32_t ex = block_exclusive_scan256(counts[p * kBins + t], sc, total);
  counts[p * kBins + t] = ex;
  if (t == 0 && (uint64_t)total != n) atomicOr(err, 2u);
}

// One pass: NT threads (NT / 64 waves), ITEMS entries per thread, a tile of NT * ITEMS entries,
// each wave ranking a contiguous kTile / NW of them (stable).  16 waves over a 16384-entry tile:
// 64 entries (512 bytes) per digit per tile on average, and fewer serial ranking steps per wave
// than 4 waves over 8192 entries.  The per-wave digit masks alias the stage (written only after the
// ranking); digit-indexed work stays on threads < 256.
template <int ITEMS, int LB, int NT>
__global__ __launch_bounds__(NT) void os_scatter_kernel(const E64* __restrict__ in, E64* __restrict__ out,
                                                              uint64_t n, int shift, const uint32_t* __restrict__ gbase,
                                                              unsigned long long* granules, uint32_t* ticket,
                                                              uint32_t* err, uint32_t tag_agg, uint32_t tiles) {
  constexpr int kTile = NT * ITEMS, kNW = NT / 64;
  static_assert(NT >= kBins && kNW * kBins <= kTile, "bins on the first 256 threads; masks fit the stage");
  __shared__ E64 stage[kTile];
  __shared__ uint32_t wcnt[kNW][kBins];
  __shared__ uint32_t bstart[kBins];
  __shared__ uint32_t goff[kBins];
  __shared__ uint32_t sc[4];
  __shared__ uint32_t tile_sh;
  unsigned long long* wmask = reinterpret_cast<unsigned long long*>(stage);   // [kNW][kBins]
  const int t = threadIdx.x, w = wave_id(), l = lane_id();
  const unsigned long long tag_inc = tag_agg + 1u;
  if (*err & 2u) return;
  if (t == 0) tile_sh = __hip_atomic_fetch_add((os_gu32*)ticket, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  for (int i = t; i < kNW * kBins; i += NT) {
    wmask[i] = 0ull;
    (&wcnt[0][0])[i] = 0;
  }
  __syncthreads();
  const uint32_t tile = tile_sh;
  if (tile >= tiles) return;
  const uint64_t base = (uint64_t)tile * kTile;
  const uint32_t cnt = (uint32_t)((n - base) < (uint64_t)kTile ? (n - base) : kTile);
  E64 cur[ITEMS];
#pragma unroll
  for (int r = 0; r < ITEMS; ++r) {
    const uint32_t pos = w * (kTile / kNW) + r * 64 + l;
    if (pos < cnt) cur[r] = in[base + pos];
  }
  const unsigned long long lanebit = 1ull << l;
  uint32_t rk[ITEMS], dg[ITEMS];
#pragma unroll
  for (int r = 0; r < ITEMS; ++r) {
    const uint32_t pos = w * (kTile / kNW) + r * 64 + l;
    const bool valid = pos < cnt;
    const uint32_t d = valid ? digit_of(cur[r], shift) : 0u;
    unsigned long long* wm = wmask + w * kBins;
    if (valid) atomicOr(&wm[d], lanebit);
    __builtin_amdgcn_wave_barrier();
    const unsigned long long peers = valid ? wm[d] : 0ull;
    const uint32_t below = popc_below(peers);
    const uint32_t prior = wcnt[w][d];
    __builtin_amdgcn_wave_barrier();
    if (valid && below == 0) {
      wcnt[w][d] = prior + (uint32_t)__popcll(peers);
      wm[d] = 0ull;
    }
    __builtin_amdgcn_wave_barrier();
    rk[r] = prior + below;
    dg[r] = d;
  }
  __syncthreads();
  uint32_t tot = 0;
  os_gu64* mine = (os_gu64*)(granules + (uint64_t)tile * kBins + (t < kBins ? t : 0));
  if (t < kBins) {
#pragma unroll
    for (int k = 0; k < kNW; ++k) {
      const uint32_t c = wcnt[k][t];
      wcnt[k][t] = tot;
      tot += c;
    }
    __hip_atomic_store(mine, ((tile == 0 ? tag_inc : (unsigned long long)tag_agg) << 32) | tot, __ATOMIC_RELAXED,
                       __HIP_MEMORY_SCOPE_AGENT);
  }
  {
    // exclusive scan of the 256 digit totals (waves 0..3); the other waves only meet the barriers
    const uint32_t inc = wave_inclusive_scan(tot);
    if (l == 63 && w < 4) sc[w] = inc;
    __syncthreads();
    const uint32_t b = (w > 0 ? sc[0] : 0) + (w > 1 ? sc[1] : 0) + (w > 2 ? sc[2] : 0);
    if (t < kBins) bstart[t] = b + inc - tot;
    __syncthreads();
  }
#pragma unroll
  for (int r = 0; r < ITEMS; ++r) {
    const uint32_t pos = w * (kTile / kNW) + r * 64 + l;
    if (pos < cnt) stage[bstart[dg[r]] + wcnt[w][dg[r]] + rk[r]] = cur[r];
  }
  if (t < kBins) {
    uint32_t excl = 0;
    if (tile > 0) {
      uint64_t j = tile;
      uint32_t spins = 0;
      for (;;) {
        unsigned long long g[LB];
#pragma unroll
        for (int k = 0; k < LB; ++k)
          g[k] = j >= (uint64_t)k + 1
                     ? __hip_atomic_load((os_gu64*)(granules + (j - 1 - k) * kBins + t), __ATOMIC_RELAXED,
                                         __HIP_MEMORY_SCOPE_AGENT)
                     : 0ull;
        bool done = false;
        int used = 0;
#pragma unroll
        for (int k = 0; k < LB; ++k) {
          if (done || used < k) continue;
          const uint32_t tag = (uint32_t)(g[k] >> 32);
          if (tag == (uint32_t)tag_inc) {
            excl += (uint32_t)g[k];
            done = true;
          } else if (tag == tag_agg) {
            excl += (uint32_t)g[k];
            used = k + 1;
          }
        }
        if (done) break;
        j -= (uint64_t)used;
        if (used == 0) {
          if (++spins > kOsSpinLimit) {
            __hip_atomic_fetch_or((os_gu32*)err, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
            break;
          }
          __builtin_amdgcn_s_sleep(1);
        }
      }
      __hip_atomic_store(mine, (tag_inc << 32) | (excl + tot), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    }
    goff[t] = gbase[t] + excl;
  }
  __syncthreads();
#pragma unroll 4
  for (uint32_t j = t; j < cnt; j += NT) {
    const E64 v = stage[j];
    const uint32_t d = digit_of(v, shift);
    out[(uint64_t)goff[d] + (j - bstart[d])] = v;
  }
}

}  // namespace


DR_API uint64_t dr_sort_u64_onesweep_workspace(uint64_t n) { return os_workspace_bytes(n > 0 ? n : 1); }

// Stable LSD sort of E64 entries on bits [begin_bit, end_bit) (multiples of 8, <= 64 bits, at most
// 8 passes) through one histogram read and one look-back scatter per pass.  `ws` holds
// dr_sort_u64_onesweep_workspace(n) bytes.  err_out (device uint32, nullable = the word at byte
// 64 of ws, zeroed per call; otherwise never cleared here, so one flag can collect several calls):
// bit 0 = a look-back gave up, bit 1 = the histograms do not count n entries (nothing was moved).
// Either way the result is not sorted and the entries' order is lost; the caller rebuilds them
// and sorts with dr_sort_u64.
// hist_part (nullable; sorts of bits [32 + 8k, 64) only): `parts` per-workgroup [4][256]
// histograms of the digits of bits [32, 64) the producer of the entries wrote
// (dr_terasort_gen_keys64_pitch128), used instead of the histogram read.
DR_API int dr_sort_u64_onesweep(E64* keys, E64* tmp, uint64_t n, int begin_bit, int end_bit, void* ws,
                                uint64_t ws_bytes, const uint32_t* hist_part, uint32_t parts, uint32_t* err_out,
                                hipStream_t s, int* result_in_tmp) {
  *result_in_tmp = 0;
  if (n == 0 || begin_bit >= end_bit) return 0;
  if (end_bit > 64 || begin_bit < 0 || (begin_bit & 7) || (end_bit & 7)) return (int)hipErrorInvalidValue;
  if (n >= (1ull << 32) || ws_bytes < os_workspace_bytes(n)) return (int)hipErrorInvalidValue;
  const int P = (end_bit - begin_bit) / 8;
  const uint64_t tiles = os_tiles(n);
  if (tiles >= (1ull << 31)) return (int)hipErrorInvalidValue;
  uint8_t* w8 = reinterpret_cast<uint8_t*>(ws);
  uint32_t* tickets = reinterpret_cast<uint32_t*>(w8);
  uint32_t* err = err_out ? err_out : reinterpret_cast<uint32_t*>(w8 + 64);
  uint32_t* gbase = reinterpret_cast<uint32_t*>(w8 + kOsHeader);
  unsigned long long* granules = reinterpret_cast<unsigned long long*>(w8 + kOsHeader + kOsCounts);
  hipError_t e = hipMemsetAsync(w8, 0, kOsHeader + kOsCounts + os_tiles(n) * kBins * 8, s);
  if (e != hipSuccess) return (int)e;
  if (hist_part) {
    if (begin_bit < 32 || end_bit != 64 || parts == 0) return (int)hipErrorInvalidValue;
    os_hist_parts_kernel<<<parts < 256 ? parts : 256, 256, 0, s>>>(hist_part, parts, (begin_bit - 32) / 8, gbase);
  } else {
    const uint32_t G = (uint32_t)(tiles < kOsHistGrid ? tiles : kOsHistGrid);
    os_hist_kernel<<<G, 256, 0, s>>>(reinterpret_cast<const uint64_t*>(keys), n, begin_bit, P, gbase);
  }
  os_hist_scan_kernel<<<P, 256, 0, s>>>(gbase, n, err);
  E64* src = keys;
  E64* dst = tmp;
  int flips = 0;
  for (int p = 0; p < P; ++p) {
    os_scatter_kernel<kOsItems, DR_OS_LB, kOsThreads><<<(unsigned)tiles, kOsThreads, 0, s>>>(
        src, dst, n, begin_bit + 8 * p, gbase + p * kBins, granules, tickets + p, err, 2u * (p + 1), (uint32_t)tiles);
    E64* x = src; src = dst; dst = x;
    flips ^= 1;
  }
  DR_LAUNCH_CHECK();
  *result_in_tmp = flips;
  return 0;
}

// Row gather + run fix-up of the compact sort: out = rows in (window, full key, position) order.
// run_shift = 64 - (window bits the LSD sort covered).  stride % 4 == 0, key_len <= 16.
// err (nullable): the look-back sort's error word; when set nothing is read or written.  An entry
// naming a row >= n sets bit 1 of *overflow (the caller redoes the sort) instead of being read.
DR_API int dr_gather_fixup(const uint8_t* rows, uint8_t* out, const E64* ent, uint64_t n, uint32_t stride,
                           uint32_t key_off, uint32_t key_len, int run_shift, uint32_t* overflow, const int32_t* err,
                           hipStream_t s) {
  if (stride == 0 || (stride & 3) || key_len == 0 || key_len > 16 || key_off + key_len > stride) return (int)hipErrorInvalidValue;
  if (run_shift < 32 || run_shift > 63) return (int)hipErrorInvalidValue;
  if (n == 0) return 0;
  const unsigned g = grid_for(n, kGfCore, 16384);
  const uint32_t W = stride / 4;
  const uint32_t* in = reinterpret_cast<const uint32_t*>(rows);
  uint32_t* o = reinterpret_cast<uint32_t*>(out);
  if (W == 25)   // nontemporal output stores (-1.2% gather time at 1e9 rows)
    gather_fixup_kernel<25, true><<<g, 256, 0, s>>>(in, o, ent, n, W, key_off, key_len, run_shift, overflow, err);
  else
    gather_fixup_kernel<0><<<g, 256, 0, s>>>(in, o, ent, n, W, key_off, key_len, run_shift, overflow, err);
  DR_LAUNCH_CHECK();
  return 0;
}

// dr_gather_fixup from input rows stored at a 128-byte pitch (in: n x 128 bytes, the first
// `stride` bytes of each row are the record) into back-to-back rows of `stride` bytes.
DR_API int dr_gather_fixup_pitch128(const uint8_t* rows, uint8_t* out, const E64* ent, uint64_t n, uint32_t stride,
                                    uint32_t key_off, uint32_t key_len, int run_shift, uint32_t* overflow,
                                    const int32_t* err, hipStream_t s) {
  if (stride != 100 || key_len == 0 || key_len > 16 || key_off + key_len > stride) return (int)hipErrorInvalidValue;
  if (run_shift < 32 || run_shift > 63) return (int)hipErrorInvalidValue;
  if (n == 0) return 0;
  const unsigned g = grid_for(n, kGfCore, 16384);
  gather_fixup_staged_kernel<<<g, 256, 0, s>>>(reinterpret_cast<const uint32_t*>(rows),
                                                   reinterpret_cast<uint32_t*>(out), ent, n, key_off, key_len,
                                                   run_shift, overflow, err);
  DR_LAUNCH_CHECK();
  return 0;
}

// gather_bucket_staged_kernel: entries sorted on their top 64 - run_shift window bits (16..31 of
// them), key at most 16 bytes.  Overflow bit 0: a run longer than the kernel's window extension.
DR_API int dr_gather_bucket_pitch128(const uint8_t* rows, uint8_t* out, const E64* ent, uint64_t n, uint32_t key_off,
                                     uint32_t key_len, int run_shift, uint32_t* overflow, const int32_t* err,
                                     hipStream_t s) {
  if (key_len == 0 || key_len > 16 || key_off + key_len > 100) return (int)hipErrorInvalidValue;
  if (run_shift < 33 || run_shift > 48 || n >= (1ull << 32)) return (int)hipErrorInvalidValue;
  if ((reinterpret_cast<uintptr_t>(rows) & 15) || (reinterpret_cast<uintptr_t>(out) & 3)) return (int)hipErrorInvalidValue;
  if (n == 0) return 0;
  gather_bucket_staged_kernel<<<grid_for(n, kBkCore, 16384), kBkThreads, 0, s>>>(
      reinterpret_cast<const uint32_t*>(rows), reinterpret_cast<uint32_t*>(out), ent, n, key_off, key_len, run_shift,
      overflow, err);
  DR_LAUNCH_CHECK();
  return 0;
}

// Rows are `pitch` bytes apart (100 back to back, or 128 for the line-aligned layout).
DR_API int dr_rekey64(const uint8_t* rows, uint32_t pitch, uint32_t key_off, uint32_t key_len, uint32_t P, E64* ent,
                      uint64_t n, hipStream_t s) {
  if (key_len == 0 || key_len > 16 || key_off + key_len > pitch || n >= (1ull << 32)) return (int)hipErrorInvalidValue;
  if (n == 0) return 0;
  rekey64_kernel<<<grid_for(n, 256, 16384), 256, 0, s>>>(rows, pitch, key_off, key_len, P, ent, n);
  DR_LAUNCH_CHECK();
  return 0;
}

DR_API int dr_e64_position_window(E64* ent, uint64_t n, hipStream_t s) {
  if (n >= (1ull << 32)) return (int)hipErrorInvalidValue;
  if (n == 0) return 0;
  e64_position_window_kernel<<<grid_for(n, 256, 16384), 256, 0, s>>>(ent, n);
  DR_LAUNCH_CHECK();
  return 0;
}
