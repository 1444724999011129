// Synthetic TeraSort store (gensort-style 100-byte records) and valsort-style validation.
//
// The benchmark input of BASELINE.json ("1 TB TeraSort") is produced by a counter-based generator
// so every rank can materialise its slice of the global table directly in HBM: record g is a pure
// function of (seed, g), which is also what makes re-execution of a failed input vertex
// idempotent (the reference gets the same property from immutable partfiles).
//
// Record layout (100 bytes):
//   [0,10)   key: 10 pseudo-random bytes
//   [10,12)  0x00 0x11
//   [12,44)  record number as 32 upper-case hex digits
//   [44,48)  0x88 0x99 0xAA 0xBB
//   [48,96)  filler: 12 runs of 4 identical letters
//   [96,100) 0xCC 0xDD 0xEE 0xFF
#include "common.h"
#include "terasort_gen.h"

namespace {

using dr_ts::ts_record;

// One workgroup generates 256 consecutive records: each thread builds one record in LDS, then
// the block streams the 25.6 KB image out with coalesced 16-byte stores.  With KEYS the producer
// also emits the record's 16-byte sort entry (the extract_keys_ts layout: hi = key bytes 0..7,
// lo = key bytes 8..9 << 48 | row index) and folds [min, max] of hi into hi_range, so a sort
// that consumes the generated table skips its key-extraction pass (one 100-byte row read each).
// KEYS: 0 = rows only, 1 = E128 entries (full 80-bit key), 2 = E64 entries of the compact row
// sort (key bits 0..31 in the high word: the window for a zero common prefix).
// PITCH: 32-bit words per stored row: 25 (100-byte rows back to back) or 32 (one row per aligned
// 128-byte line, bytes 100..127 zero: the HBM line a random row read fetches holds exactly that row).
// HIST (KEYS == 2): also the histograms of the four window bytes (the digits of the compact sort's
// four LSD passes), one [4][256] partial per workgroup in hist_part, so that sort needs no
// histogram read of its own (dr_sort_u64_onesweep with hist_part).
template <int KEYS, bool ROWS = true, int PITCH = 25, bool HIST = false, bool NTS = false>
__global__ __launch_bounds__(256) void ts_gen_kernel(uint32_t* __restrict__ out, uint64_t n, uint64_t first,
                                                     uint64_t seed, void* __restrict__ keys, uint32_t idx_base,
                                                     unsigned long long* __restrict__ hi_range,
                                                     uint32_t* __restrict__ hist_part = nullptr) {
  __shared__ __attribute__((aligned(16))) uint32_t img[256 * 25];
  __shared__ uint32_t hist[HIST ? 4 : 1][256];
  if constexpr (HIST) {
#pragma unroll
    for (int p = 0; p < 4; ++p) hist[p][threadIdx.x] = 0;
    __syncthreads();
  }
  uint64_t mn = ~0ull, mx = 0;
  for (uint64_t row0 = (uint64_t)blockIdx.x * 256; row0 < n; row0 += (uint64_t)gridDim.x * 256) {
    const uint32_t rows = (uint32_t)((n - row0) < 256 ? (n - row0) : 256);
    if (threadIdx.x < rows) {
      uint32_t w[25];
      ts_record(seed, first + row0 + threadIdx.x, w);
      if (ROWS) {
#pragma unroll
        for (int k = 0; k < 25; ++k) img[threadIdx.x * 25 + k] = w[k];
      }
      if (KEYS) {
        const uint64_t hi = ((uint64_t)bswap32(w[0]) << 32) | bswap32(w[1]);
        const uint32_t idx = idx_base + (uint32_t)(row0 + threadIdx.x);
        if (KEYS == 1) {
          E128 e;
          e.hi = hi;
          e.lo = ((uint64_t)(bswap32(w[2]) & 0xFFFF0000u) << 32) | idx;
          static_cast<E128*>(keys)[row0 + threadIdx.x] = e;
        } else {
          static_cast<uint64_t*>(keys)[row0 + threadIdx.x] = (hi & 0xFFFFFFFF00000000ull) | idx;
          if constexpr (HIST) {
#pragma unroll
            for (int p = 0; p < 4; ++p) atomicAdd(&hist[p][(uint32_t)(hi >> (32 + 8 * p)) & 0xFF], 1u);
          }
        }
        mn = hi < mn ? hi : mn;
        mx = hi > mx ? hi : mx;
      }
    }
    if (!ROWS) continue;                       // keys only: no record image to store
    __syncthreads();
    if constexpr (PITCH == 32) {
      uint4* dst = reinterpret_cast<uint4*>(out + row0 * 32);
      for (uint32_t j = threadIdx.x; j < rows * 8; j += 256) {
        const uint32_t r = j >> 3, q = (j & 7) * 4;
        const uint32_t* src = img + r * 25 + q;
        uint4 v;
        v.x = q < 25 ? src[0] : 0u;
        v.y = q + 1 < 25 ? src[1] : 0u;
        v.z = q + 2 < 25 ? src[2] : 0u;
        v.w = q + 3 < 25 ? src[3] : 0u;
        if constexpr (NTS) {
          uint32_t* d = reinterpret_cast<uint32_t*>(dst + j);
          __builtin_nontemporal_store(v.x, d);
          __builtin_nontemporal_store(v.y, d + 1);
          __builtin_nontemporal_store(v.z, d + 2);
          __builtin_nontemporal_store(v.w, d + 3);
        } else {
          dst[j] = v;
        }
      }
      __syncthreads();
      continue;
    }
    uint32_t* o = out + row0 * 25;
    const uint32_t words = rows * 25;
    if (rows == 256) {
      const uint4* src = reinterpret_cast<const uint4*>(img);
      uint4* dst = reinterpret_cast<uint4*>(o);
      for (uint32_t j = threadIdx.x; j < 256 * 25 / 4; j += 256) dst[j] = src[j];
    } else {
      for (uint32_t j = threadIdx.x; j < words; j += 256) o[j] = img[j];
    }
    __syncthreads();
  }
  if constexpr (HIST) {
    __syncthreads();
#pragma unroll
    for (int p = 0; p < 4; ++p) hist_part[((uint64_t)blockIdx.x * 4 + p) * 256 + threadIdx.x] = hist[p][threadIdx.x];
  }
  if (KEYS && hi_range) {
#pragma unroll
    for (int m = 32; m >= 1; m >>= 1) {
      const uint64_t a = __shfl_xor(mn, m, 64), b = __shfl_xor(mx, m, 64);
      mn = a < mn ? a : mn;
      mx = b > mx ? b : mx;
    }
    if (lane_id() == 0) {
      atomicMin(hi_range, (unsigned long long)mn);
      atomicMax(hi_range + 1, (unsigned long long)mx);
    }
  }
}

__device__ __forceinline__ uint64_t rec_hash(const uint32_t* r) {
  uint64_t h = 0xCBF29CE484222325ull;
#pragma unroll
  for (int k = 0; k < 25; ++k) h = (h ^ r[k]) * 0x100000001B3ull;
  return mix64(h);
}

__device__ __forceinline__ void ts_key(const uint32_t* r, uint64_t& hi, uint32_t& lo) {
  hi = ((uint64_t)bswap32(r[0]) << 32) | bswap32(r[1]);
  lo = bswap32(r[2]) >> 16;
}

// out[0] += sum of record hashes (mod 2^64), out[1] += #i with key(i-1) > key(i).
template <bool DESC>
__global__ __launch_bounds__(256) void ts_check_kernel(const uint32_t* __restrict__ rows, uint64_t n,
                                                       unsigned long long* __restrict__ out) {
  uint64_t hsum = 0, bad = 0;
  for (uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n;
       i += (uint64_t)gridDim.x * blockDim.x) {
    const uint32_t* r = rows + i * 25;
    hsum += rec_hash(r);
    if (i > 0) {
      uint64_t h0, h1; uint32_t l0, l1;
      ts_key(r - 25, h0, l0);
      ts_key(r, h1, l1);
      if (DESC ? (h0 < h1 || (h0 == h1 && l0 < l1)) : (h0 > h1 || (h0 == h1 && l0 > l1))) ++bad;
    }
  }
  hsum = wave_sum64(hsum);
  bad = wave_sum64(bad);
  if (lane_id() == 0) {
    atomicAdd(&out[0], (unsigned long long)hsum);
    atomicAdd(&out[1], (unsigned long long)bad);
  }
}


// Records first + idx[p] generated into rows p of `out` (100-byte rows back to back, 4-byte
// aligned): the send-buffer pack of a distributed sort over gen://terasort (ops/recordsort.py),
// idx being the bucket-ordered record offsets of dr_ts_dest_partition.  Each workgroup builds 256
// records in LDS and streams them out with 16-byte nontemporal stores from the first 16-byte
// boundary on (dword stores for the few words before it and after the last full chunk).
// IS = idx stride in 32-bit words: 1 (int32 offsets) or 2 (the low words of sorted E64 entries).
// seg (nullable): nseg segments {out row, idx position}, ascending in out row, seg[0].out = 0:
// out row p takes idx position seg[s].idx + p - seg[s].out of the last segment starting at or
// before p (one launch packs a whole exchange round: one segment per destination).
template <int IS>
__global__ __launch_bounds__(256) void ts_gen_gather_kernel(uint32_t* __restrict__ out, const uint32_t* __restrict__ idx,
                                                            uint64_t n, uint64_t first, uint64_t seed,
                                                            const int64_t* __restrict__ seg = nullptr,
                                                            uint32_t nseg = 0) {
  __shared__ __attribute__((aligned(16))) uint32_t img[256 * 25];
  __shared__ int64_t sseg[64][2];
  const uint32_t t = threadIdx.x;
  if (nseg) {
    if (t < 2 * nseg) sseg[t >> 1][t & 1] = seg[t];
    __syncthreads();
  }
  for (uint64_t row0 = (uint64_t)blockIdx.x * 256; row0 < n; row0 += (uint64_t)gridDim.x * 256) {
    const uint32_t rows = (uint32_t)((n - row0) < 256 ? (n - row0) : 256);
    if (t < rows) {
      uint32_t w[25];
      uint64_t p = row0 + t;
      if (nseg) {
        uint32_t s = 0;
        while (s + 1 < nseg && (uint64_t)sseg[s + 1][0] <= p) ++s;
        p = (uint64_t)sseg[s][1] + (p - (uint64_t)sseg[s][0]);
      }
      ts_record(seed, first + idx[p * IS], w);
#pragma unroll
      for (int k = 0; k < 25; ++k) img[t * 25 + k] = w[k];
    }
    __syncthreads();
    uint32_t* o = out + row0 * 25;
    const uint32_t words = rows * 25;
    uint32_t head = (4u - (uint32_t)((reinterpret_cast<uintptr_t>(o) >> 2) & 3u)) & 3u;
    head = head < words ? head : words;
    if (t < head) o[t] = img[t];
    const uint32_t nch = (words - head) >> 2;
    for (uint32_t c = t; c < nch; c += 256) {
      const uint32_t q = head + 4 * c;
      uint32_t* d = o + q;
      __builtin_nontemporal_store(img[q], d);
      __builtin_nontemporal_store(img[q + 1], d + 1);
      __builtin_nontemporal_store(img[q + 2], d + 2);
      __builtin_nontemporal_store(img[q + 3], d + 3);
    }
    for (uint32_t q = head + 4 * nch + t; q < words; q += 256) o[q] = img[q];
    __syncthreads();
  }
}

}  // namespace

DR_API int dr_terasort_gen(uint8_t* out, uint64_t n, uint64_t first_index, uint64_t seed, hipStream_t s) {
  if (n == 0) return 0;
  ts_gen_kernel<0><<<grid_for(n, 256, 16384), 256, 0, s>>>(reinterpret_cast<uint32_t*>(out), n, first_index,
                                                           seed, nullptr, 0, nullptr);
  DR_LAUNCH_CHECK();
  return 0;
}

// Generator fused with key extraction: also writes n sort entries (row index idx_base + i) and,
// when hi_range is non-null, min/max of the entries' hi words (caller initialises {~0, 0}).
DR_API int dr_terasort_gen_keys(uint8_t* out, uint64_t n, uint64_t first_index, uint64_t seed, E128* keys,
                                uint32_t idx_base, uint64_t* hi_range, hipStream_t s) {
  if (n == 0) return 0;
  if (n + idx_base > (1ull << 32)) return (int)hipErrorInvalidValue;
  ts_gen_kernel<1><<<grid_for(n, 256, 16384), 256, 0, s>>>(reinterpret_cast<uint32_t*>(out), n, first_index,
                                                           seed, keys, idx_base,
                                                           reinterpret_cast<unsigned long long*>(hi_range));
  DR_LAUNCH_CHECK();
  return 0;
}

// Same, emitting the 8-byte entries of the compact row sort (dr_extract_keys64 with prefix 0).
DR_API int dr_terasort_gen_keys64(uint8_t* out, uint64_t n, uint64_t first_index, uint64_t seed, E64* keys,
                                  uint32_t idx_base, uint64_t* hi_range, hipStream_t s) {
  if (n == 0) return 0;
  if (n + idx_base > (1ull << 32)) return (int)hipErrorInvalidValue;
  ts_gen_kernel<2><<<grid_for(n, 256, 16384), 256, 0, s>>>(reinterpret_cast<uint32_t*>(out), n, first_index,
                                                           seed, keys, idx_base,
                                                           reinterpret_cast<unsigned long long*>(hi_range));
  DR_LAUNCH_CHECK();
  return 0;
}

// Same with the records at a 128-byte pitch (out: n x 128 bytes, bytes 100..127 of each row zero).
// hist_part (nullable): [dr_terasort_gen_hist_parts(n)][4][256] uint32 per-workgroup histograms of
// the four window bytes of the entries.
DR_API uint32_t dr_terasort_gen_hist_parts(uint64_t n) { return grid_for(n, 256, 16384); }

DR_API int dr_terasort_gen_keys64_pitch128(uint8_t* out, uint64_t n, uint64_t first_index, uint64_t seed, E64* keys,
                                           uint32_t idx_base, uint64_t* hi_range, uint32_t* hist_part, hipStream_t s) {
  if (n == 0) return 0;
  if (n + idx_base > (1ull << 32)) return (int)hipErrorInvalidValue;
  if (reinterpret_cast<uintptr_t>(out) & 15) return (int)hipErrorInvalidValue;
  const unsigned g = grid_for(n, 256, 16384);
  // nontemporal row stores (profiles/r3/ab_gen_nt.log: 105.8-106.2 -> 103.7-104.0 ms per step)
  if (hist_part)
    ts_gen_kernel<2, true, 32, true, true><<<g, 256, 0, s>>>(reinterpret_cast<uint32_t*>(out), n, first_index, seed,
                                                             keys, idx_base,
                                                             reinterpret_cast<unsigned long long*>(hi_range),
                                                             hist_part);
  else
    ts_gen_kernel<2, true, 32, false, true><<<g, 256, 0, s>>>(reinterpret_cast<uint32_t*>(out), n, first_index, seed,
                                                              keys, idx_base,
                                                              reinterpret_cast<unsigned long long*>(hi_range));
  DR_LAUNCH_CHECK();
  return 0;
}


// Send rows of a generated input: out row p = record first + idx[p] (see ts_gen_gather_kernel).
DR_API int dr_terasort_gen_gather(uint8_t* out, const uint32_t* idx, uint64_t n, uint64_t first, uint64_t seed,
                                  hipStream_t s) {
  if (n == 0) return 0;
  if (reinterpret_cast<uintptr_t>(out) & 3) return (int)hipErrorInvalidValue;
  ts_gen_gather_kernel<1><<<grid_for(n, 256, 16384), 256, 0, s>>>(reinterpret_cast<uint32_t*>(out), idx, n, first,
                                                                  seed);
  DR_LAUNCH_CHECK();
  return 0;
}

// Send rows of a generated input in the order of sorted E64 entries: out row p = record
// first + (uint32)ent[q(p)] (the fine-bucket send side of the multi-rank TeraSort,
// ops/recordsort.py), q(p) = p, or through nseg <= 64 segments {out row, entry} (device int64
// [nseg][2], see ts_gen_gather_kernel): one launch per exchange round.
DR_API int dr_terasort_gen_gather64(uint8_t* out, const E64* ent, uint64_t n, uint64_t first, uint64_t seed,
                                    const int64_t* seg, uint32_t nseg, hipStream_t s) {
  if (n == 0) return 0;
  if (reinterpret_cast<uintptr_t>(out) & 3) return (int)hipErrorInvalidValue;
  if (nseg > 64 || (nseg > 0 && seg == nullptr)) return (int)hipErrorInvalidValue;
  ts_gen_gather_kernel<2><<<grid_for(n, 256, 16384), 256, 0, s>>>(reinterpret_cast<uint32_t*>(out),
                                                                  reinterpret_cast<const uint32_t*>(ent), n, first,
                                                                  seed, seg, nseg);
  DR_LAUNCH_CHECK();
  return 0;
}

// E64 entries only (key bytes 0..3 << 32 | idx_base + i), no records: the send side of the
// multi-rank TeraSort sorts these before any record exists.  hist_part as in
// dr_terasort_gen_keys64_pitch128 ([dr_terasort_gen_hist_parts(n)][4][256], nullable).
DR_API int dr_terasort_gen_entries64(E64* keys, uint64_t n, uint64_t first_index, uint64_t seed, uint32_t idx_base,
                                     uint32_t* hist_part, hipStream_t s) {
  if (n == 0) return 0;
  if (n + idx_base > (1ull << 32)) return (int)hipErrorInvalidValue;
  const unsigned g = grid_for(n, 256, 16384);
  if (hist_part)
    ts_gen_kernel<2, false, 25, true><<<g, 256, 0, s>>>(nullptr, n, first_index, seed, keys, idx_base, nullptr,
                                                        hist_part);
  else
    ts_gen_kernel<2, false><<<g, 256, 0, s>>>(nullptr, n, first_index, seed, keys, idx_base, nullptr);
  DR_LAUNCH_CHECK();
  return 0;
}

// Accumulates [hash_sum, order_violations] into out2 (2 x uint64, device; caller zeroes it).
DR_API int dr_terasort_check(const uint8_t* rows, uint64_t n, uint64_t* out2, hipStream_t s) {
  if (n == 0) return 0;
  ts_check_kernel<false><<<grid_for(n, 256, 8192), 256, 0, s>>>(reinterpret_cast<const uint32_t*>(rows), n,
                                                                reinterpret_cast<unsigned long long*>(out2));
  DR_LAUNCH_CHECK();
  return 0;
}

// dr_terasort_check of a descending order (OrderByDescending output).
DR_API int dr_terasort_check_desc(const uint8_t* rows, uint64_t n, uint64_t* out2, hipStream_t s) {
  if (n == 0) return 0;
  ts_check_kernel<true><<<grid_for(n, 256, 8192), 256, 0, s>>>(reinterpret_cast<const uint32_t*>(rows), n,
                                                               reinterpret_cast<unsigned long long*>(out2));
  DR_LAUNCH_CHECK();
  return 0;
}
