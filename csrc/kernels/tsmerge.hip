// Fine-bucket exchange of the multi-rank TeraSort (ops/recordsort.py, gen:// inputs).
//
// The send side sorts its records' E64 entries (key bytes 0..3 as the window) on the top bits of
// the window, so its rows leave in bucket order, and the key ranges of the exchange are unions of
// FINE BUCKETS (the top `fb` key bits, 16 <= fb <= 24: ~600 rows of the whole job per bucket).  Every source sends, next
// to its rows, its row count per fine bucket.  A received key range is then, per fine bucket, W
// contiguous slices (one per source) of rows that all share their top fb key bits, and the
// receive side orders each bucket on its own (ts_tile_merge): no entry extraction, no radix
// passes and no random row gather over the received block, one read and one write of the rows.
//   ts_fine_starts   starts[k] = first sorted entry with bucket >= k (k = 0 .. 2^fb)
//   ts_tile_merge    one workgroup per fine bucket: its rows held in registers (two per lane),
//                    their keys ranked by an LDS counting sort, the rows stored to their slots
// Reference: the sampler + RangePartition + MergeSort stages of CreateRangePartition
// (LinqToDryad/DryadLinqQueryGen.cs:2362-2474); its merge of the sorted inputs becomes a
// per-bucket sort because the buckets are small enough to hold in one workgroup.
#include "common.h"

namespace {

constexpr uint32_t kTmCap = 1024;                  // rows of one bucket a workgroup orders
constexpr uint32_t kTmMaxW = 64;                   // sources
constexpr uint32_t kTmThreads = 512;
constexpr uint32_t kTmRows = kTmCap / kTmThreads;  // rows per lane, held in registers (2 x 25 dwords)
typedef uint32_t u32x4u __attribute__((ext_vector_type(4), aligned(4)));   // 16-byte access, 4-byte aligned
constexpr uint32_t kTmBins = 1024;                 // LDS counting-sort bins (next 10 key bits)

// Four entries per lane per step (two 16-byte loads; the entry before them comes from the lane
// below, or one cached load for lane 0 of a wave), every bucket boundary between consecutive
// entries written once.
template <bool PAIRS>
__global__ __launch_bounds__(256) void ts_fine_starts_kernel(const E64* __restrict__ ent, uint64_t n, uint32_t fb,
                                                             uint32_t* __restrict__ starts) {
  const uint32_t nb = 1u << fb;
  const int sh = 64 - (int)fb;
  const uint64_t groups = (n + 3) / 4;
  const uint64_t* e = reinterpret_cast<const uint64_t*>(ent);
  for (uint64_t g0 = (uint64_t)blockIdx.x * blockDim.x; g0 < groups; g0 += (uint64_t)gridDim.x * blockDim.x) {
    const uint64_t g = g0 + threadIdx.x;
    const uint64_t i0 = 4 * g;
    uint32_t b[4] = {0, 0, 0, 0};
    if (PAIRS && i0 + 3 < n) {
      const ulonglong2 a = *reinterpret_cast<const ulonglong2*>(e + i0);
      const ulonglong2 c = *reinterpret_cast<const ulonglong2*>(e + i0 + 2);
      b[0] = (uint32_t)(a.x >> sh); b[1] = (uint32_t)(a.y >> sh); b[2] = (uint32_t)(c.x >> sh); b[3] = (uint32_t)(c.y >> sh);
    } else {
      for (int k = 0; k < 4; ++k) b[k] = i0 + k < n ? (uint32_t)(e[i0 + k] >> sh) : 0u;
    }
    // the bucket of entry i0 - 1: the lane below's last, or a load at a wave's first lane
    uint32_t prev = __shfl_up(b[3], 1, 64);
    if (lane_id() == 0 && i0 > 0 && i0 - 1 < n) prev = (uint32_t)(e[i0 - 1] >> sh);
    if (i0 < n) {
#pragma unroll
      for (int k = 0; k < 4; ++k) {
        const uint64_t i = i0 + k;
        if (i >= n) break;
        const uint32_t pb = k == 0 ? prev : b[k - 1];
        if (i == 0) {
          for (uint32_t q = 0; q <= b[k]; ++q) starts[q] = 0;
        } else {
          for (uint32_t q = pb + 1; q <= b[k]; ++q) starts[q] = (uint32_t)i;
        }
        if (i == n - 1) {
          for (uint32_t q = b[k] + 1; q <= nb; ++q) starts[q] = (uint32_t)n;
        }
      }
    }
  }
}

// Key bits [fb, 80) of a row whose first 10 bytes are the key (fb >= 16: they fit 64 bits),
// left-aligned.
__device__ __forceinline__ uint64_t tm_key(uint32_t w0, uint32_t w1, uint32_t w2, uint32_t fb) {
  const uint64_t k0 = ((uint64_t)bswap32(w0) << 32) | bswap32(w1);
  const uint64_t k1 = (uint64_t)(bswap32(w2) >> 16);                  // key bytes 8, 9
  return (k0 << fb) | ((k1 << 48) >> (64 - fb));
}

// The same key for a row whose key is `klen` <= 10 bytes at byte `koff` (read byte by byte, the
// missing bytes zero: equal keys compare equal, so ties keep their (source, position) order), its
// bits inverted for a descending sort (`desc`): the order the window-sorted E64 entries and the fine
// buckets of an inverted key define.
__device__ __forceinline__ uint64_t tm_key_at(const uint8_t* r, uint32_t koff, uint32_t klen, bool desc, uint32_t fb) {
  uint64_t k0 = 0;
  uint32_t k1 = 0;
#pragma unroll
  for (uint32_t j = 0; j < 10; ++j) {
    uint32_t b = j < klen ? (uint32_t)r[koff + j] : 0u;
    if (desc && j < klen) b ^= 0xFFu;
    if (j < 8) k0 = (k0 << 8) | b;
    else k1 = (k1 << 8) | b;
  }
  return (k0 << fb) | (((uint64_t)k1 << 48) >> (64 - fb));
}

// Key of staged / loaded row `r`: the TeraSort layout (10-byte key at byte 0, ascending) from its
// first three words, any other key spec (kspec = koff | klen << 8 | desc << 16) byte by byte.
template <bool GEN>
__device__ __forceinline__ uint64_t tm_row_key(const uint32_t* r, uint32_t kspec, uint32_t fb) {
  if (!GEN) return tm_key(r[0], r[1], r[2], fb);
  return tm_key_at(reinterpret_cast<const uint8_t*>(r), kspec & 0xFFu, (kspec >> 8) & 0xFFu, (kspec >> 16) & 1u, fb);
}

// Rows of one bucket staged in LDS at the record pitch (100-byte rows: two workgroups per CU,
// 79.4 KB each; 128-byte rows: one, 99 KB).
constexpr uint32_t kTsStage = 736;
constexpr uint32_t kTsBins = 256;                  // staged path: next 8 key bits
constexpr uint32_t kTsPasses = (kTsStage + 63) / 64;

// pre[s * K + k] = row (of `rows`) where bucket k's slice from source s starts, cnt[s * K + k] its
// rows; bucket k's output rows start at out row outoff[k].  A workgroup orders buckets
// blockIdx.x, + gridDim.x, ... (a bucket averages ~600 rows; FINE_ROWS), two in flight: while it
// ranks and stores bucket j from the LDS stage, the rows of bucket j + 1 are already loading into
// registers (12 x 16 bytes per lane, issued right after bucket j was staged), and wave 0 holds
// the slice metadata of bucket j + 2 (the barriers wait on LDS traffic only, so the row loads stay
// in flight across them).  Per bucket of nt <= kTsStage rows:
//   * its W source slices, already in registers (8 lanes per row, 16-byte loads; a wave reads 8
//     consecutive rows of a slice, 800 contiguous bytes), are written to the stage at the 100-byte
//     pitch;
//   * an LDS counting sort on the next 8 key bits plus an in-bin rank by (key, tile index) gives
//     each output slot its tile row (source-major tile index = stable);
//   * the bucket leaves in OUTPUT order: a wave stores 8 consecutive output rows, 800 contiguous
//     bytes, every row read back from the stage.  Both HBM streams are contiguous.
// kTsStage < nt <= kTmCap (a rare large bucket): left to ts_tile_merge_big_kernel.  A bucket of
// more than kTmCap rows is skipped and flagged (*overflow); the caller orders that key range
// another way.
template <uint32_t RW, bool GEN>
__global__ __launch_bounds__(kTmThreads) __attribute__((amdgpu_waves_per_eu(RW <= 25 ? 4 : 2))) void ts_tile_merge_kernel(const uint32_t* __restrict__ rows,
                                                                   uint32_t* __restrict__ out,
                                                                   const int64_t* __restrict__ pre,
                                                                   const int32_t* __restrict__ cnt,
                                                                   const int64_t* __restrict__ outoff, uint32_t W,
                                                                   uint32_t K, uint32_t fb,
                                                                   uint32_t* __restrict__ overflow, uint32_t kspec) {
  constexpr uint32_t P = (RW + 3) / 4;              // 16-byte pieces per row (the last may be partial)
  constexpr uint32_t kPoolWords = kTsStage * RW + kTsStage + 2 * kTsBins;
  static_assert(P <= 8, "rows of at most 128 bytes");
  __shared__ __attribute__((aligned(16))) uint32_t pool[kPoolWords];
  __shared__ int64_t sbase[2][kTmMaxW];
  __shared__ uint32_t spre[2][kTmMaxW + 1];
  __shared__ int64_t sout[2];
  __shared__ uint32_t wtot[kTmThreads / 64];
  const uint32_t t = threadIdx.x;
  const uint32_t G = gridDim.x;
  uint32_t* stage = pool;
  uint16_t* member = reinterpret_cast<uint16_t*>(pool + kTsStage * RW);
  uint16_t* perm = member + kTsStage;
  uint32_t* bcnt = pool + kTsStage * RW + kTsStage;
  uint32_t* bcur = bcnt + kTsBins;
  const uint32_t g = t >> 3, sub = t & 7;

  // wave 0, lane s < W: source s's (slice start, rows) of a bucket; lane 0 also its output row
  int64_t nx_pre = 0, nx_out = 0;
  uint32_t nx_cnt = 0;
  auto meta_load = [&](uint32_t k) {
    nx_cnt = 0;
    if (t < W && k < K) {
      nx_pre = pre[(uint64_t)t * K + k];
      nx_cnt = (uint32_t)cnt[(uint64_t)t * K + k];
      if (t == 0) nx_out = outoff[k];
    }
  };
  auto meta_store = [&](uint32_t buf) {           // wave 0: slice starts within the tile, by scan
    const uint32_t c = t < W ? nx_cnt : 0u;
    const uint32_t inc = wave_inclusive_scan(c);
    if (t < W) {
      sbase[buf][t] = nx_pre;
      spre[buf][t] = inc - c;
    }
    if (t == 63) spre[buf][W] = inc;
    if (t == 0) sout[buf] = nx_out;
  };
  u32x4u v[kTsPasses];
  auto rows_load = [&](uint32_t buf, uint32_t nt) {
    uint32_t s = 0;
#pragma unroll
    for (uint32_t p = 0; p < kTsPasses; ++p) {
      const uint32_t i = g + 64 * p;
      if (i < nt && sub < P) {
        while (spre[buf][s + 1] <= i) ++s;
        const uint32_t* src = rows + (uint64_t)(sbase[buf][s] + (int64_t)(i - spre[buf][s])) * RW + sub * 4;
        if ((sub + 1) * 4 <= RW) {
          v[p] = *reinterpret_cast<const u32x4u*>(src);
        } else {                                   // the row's last, partial piece: never read past it
          v[p].x = src[0];
          if (RW % 4 > 1) v[p].y = src[1];
          if (RW % 4 > 2) v[p].z = src[2];
        }
      }
    }
  };

  uint32_t k = blockIdx.x;
  if (t < 64) {
    meta_load(k);
    meta_store(0);
    meta_load(k + G);
  }
  __syncthreads();
  uint32_t nt = spre[0][W];
  if (k < K && nt <= kTsStage) rows_load(0, nt);
  for (uint32_t j = 0; k < K; ++j, k += G) {
    const uint32_t b = j & 1;
    const int64_t ob = sout[b];
    if (t < 64) {
      meta_store(b ^ 1);                            // bucket k + G
      meta_load(k + 2 * G);
    }
    if (t < kTsBins) bcnt[t] = 0;
    const bool staged = nt > 0 && nt <= kTsStage;
    if (staged) {
#pragma unroll
      for (uint32_t p = 0; p < kTsPasses; ++p) {
        const uint32_t i = g + 64 * p;
        if (i < nt && sub < P) {
          uint32_t* d = stage + i * RW + sub * 4;
          d[0] = v[p].x;
          if ((sub + 1) * 4 <= RW) {
            d[1] = v[p].y;
            d[2] = v[p].z;
            d[3] = v[p].w;
          } else {
            if (RW % 4 > 1) d[1] = v[p].y;
            if (RW % 4 > 2) d[2] = v[p].z;
          }
        }
      }
    }
    __syncthreads();
    const uint32_t nt2 = spre[b ^ 1][W];
    if (k + G < K && nt2 <= kTsStage) rows_load(b ^ 1, nt2);     // in flight while bucket k is ordered
    if (nt > kTmCap && t == 0) atomicOr(overflow, 1u);
    if (staged) {
      uint32_t* o = out + (uint64_t)ob * RW;
      for (uint32_t i = t; i < nt; i += kTmThreads) {
        const uint32_t* r = stage + i * RW;
        atomicAdd(&bcnt[(uint32_t)(tm_row_key<GEN>(r, kspec, fb) >> 56)], 1u);
      }
      __syncthreads();
      uint32_t c = 0, inc = 0;
      if (t < kTsBins) {                          // exclusive scan of the 256 bins: waves 0..3
        c = bcnt[t];
        inc = wave_inclusive_scan(c);
        if (lane_id() == 63) wtot[wave_id()] = inc;
      }
      __syncthreads();
      if (t < kTsBins) {
        uint32_t run = inc - c;
        for (int w = 0; w < wave_id(); ++w) run += wtot[w];
        bcur[t] = run;
      }
      __syncthreads();
      for (uint32_t i = t; i < nt; i += kTmThreads) {
        const uint32_t* r = stage + i * RW;
        member[atomicAdd(&bcur[(uint32_t)(tm_row_key<GEN>(r, kspec, fb) >> 56)], 1u)] = (uint16_t)i;
      }
      __syncthreads();
      for (uint32_t i = t; i < nt; i += kTmThreads) {   // slot = bin start + smaller (key, index) in the bin
        const uint32_t* r = stage + i * RW;
        const uint64_t a = tm_row_key<GEN>(r, kspec, fb);
        const uint32_t d = (uint32_t)(a >> 56), end = bcur[d], beg = end - bcnt[d];
        uint32_t slot = beg;
        for (uint32_t m = beg; m < end; ++m) {
          const uint32_t x = member[m];
          const uint32_t* q = stage + x * RW;
          const uint64_t bb = tm_row_key<GEN>(q, kspec, fb);
          slot += (bb < a || (bb == a && x < i)) ? 1u : 0u;
        }
        perm[slot] = (uint16_t)i;
      }
      __syncthreads();
#pragma unroll 4
      for (uint32_t p = 0; p < kTsPasses; ++p) {
        const uint32_t jj = g + 64 * p;
        if (jj < nt && sub < P) {
          const uint32_t* sr = stage + (uint32_t)perm[jj] * RW + sub * 4;
          uint32_t* dst = o + jj * RW + sub * 4;
          // plain stores: the bucket's first and last lines are partial, completed in L2 by the
          // neighbouring buckets (nontemporal stores write partial lines through)
          if ((sub + 1) * 4 <= RW) {
            *reinterpret_cast<u32x4u*>(dst) = u32x4u{sr[0], sr[1], sr[2], sr[3]};
          } else {
            dst[0] = sr[0];
            if (RW % 4 > 1) dst[1] = sr[1];
            if (RW % 4 > 2) dst[2] = sr[2];
          }
        }
      }
    }
    __syncthreads();
    nt = nt2;
  }
}

// The buckets of kTsStage < nt <= kTmCap rows (rare: > 5 sigma above the ~600-row mean at
// FINE_ROWS) that ts_tile_merge_kernel leaves: each workgroup scans 512 buckets' sizes, lists the
// large ones in LDS and orders them with the register path -- lane t holds tile rows t and t + 512
// (6 x 16 + 4 bytes each), ranks by the next 10 key bits, rows stored to their slots.
template <uint32_t RW, bool GEN>
__global__ __launch_bounds__(kTmThreads) __attribute__((amdgpu_waves_per_eu(4))) void ts_tile_merge_big_kernel(
    const uint32_t* __restrict__ rows, uint32_t* __restrict__ out, const int64_t* __restrict__ pre,
    const int32_t* __restrict__ cnt, const int64_t* __restrict__ outoff, uint32_t W, uint32_t K, uint32_t fb,
    uint32_t kspec) {
  __shared__ uint64_t key[kTmCap];
  __shared__ uint16_t member[kTmCap];
  __shared__ uint16_t rnk[kTmCap];
  __shared__ uint32_t bcnt[kTmBins];
  __shared__ uint32_t bcur[kTmBins];
  __shared__ int64_t sbase[kTmMaxW];
  __shared__ uint32_t spre[kTmMaxW + 1];
  __shared__ uint32_t wtot[kTmThreads / 64];
  __shared__ uint32_t list[kTmThreads];
  __shared__ uint32_t nlist;
  const uint32_t t = threadIdx.x;
  if (t == 0) nlist = 0;
  __syncthreads();
  {
    const uint64_t kk = (uint64_t)blockIdx.x * kTmThreads + t;
    if (kk < K) {
      uint32_t nt = 0;
      for (uint32_t s = 0; s < W; ++s) nt += (uint32_t)cnt[(uint64_t)s * K + kk];
      if (nt > kTsStage && nt <= kTmCap) list[atomicAdd(&nlist, 1u)] = (uint32_t)kk;
    }
  }
  __syncthreads();
  const uint32_t nl = nlist;
  for (uint32_t li = 0; li < nl; ++li) {
    const uint32_t k = list[li];
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
    constexpr uint32_t F = RW / 4, T = RW % 4;       // full 16-byte pieces, tail words per row
    uint32_t* o = out + (uint64_t)outoff[k] * RW;
    bcnt[t] = 0;
    bcnt[t + kTmThreads] = 0;
    u32x4u v[kTmRows][F > 0 ? F : 1];
    uint32_t tail[kTmRows][T > 0 ? T : 1];
    uint64_t gkey[kTmRows];                          // GEN: the key read from the row in HBM
#pragma unroll
    for (uint32_t h = 0; h < kTmRows; ++h) {
      const uint32_t i = t + h * kTmThreads;        // tile row: source-major = stable
      if (i < nt) {
        uint32_t s = 0;
        while (spre[s + 1] <= i) ++s;
        const uint32_t* src = rows + (uint64_t)(sbase[s] + (int64_t)(i - spre[s])) * RW;
#pragma unroll
        for (uint32_t q = 0; q < F; ++q) v[h][q] = *reinterpret_cast<const u32x4u*>(src + 4 * q);
#pragma unroll
        for (uint32_t q = 0; q < T; ++q) tail[h][q] = src[4 * F + q];
        if (GEN) gkey[h] = tm_row_key<true>(src, kspec, fb);
      }
    }
    __syncthreads();
#pragma unroll
    for (uint32_t h = 0; h < kTmRows; ++h) {
      const uint32_t i = t + h * kTmThreads;
      if (i < nt) {
        const uint64_t kv = GEN ? gkey[h]                  // the top 10 bits pick the bin
                                : F > 0 ? tm_key(v[h][0].x, v[h][0].y, v[h][0].z, fb)
                                        : tm_key(tail[h][0], tail[h][T > 1 ? 1 : 0], tail[h][T > 2 ? 2 : 0], fb);
        key[i] = kv;
        atomicAdd(&bcnt[(uint32_t)(kv >> 54)], 1u);
      }
    }
    __syncthreads();
    {                                               // exclusive scan of the 1024 bins, 2 per lane
      const uint32_t c0 = bcnt[2 * t], c1 = bcnt[2 * t + 1];
      const uint32_t inc = wave_inclusive_scan(c0 + c1);
      if (lane_id() == 63) wtot[wave_id()] = inc;
      __syncthreads();
      uint32_t run = inc - c0 - c1;
      for (int w = 0; w < wave_id(); ++w) run += wtot[w];
      bcur[2 * t] = run;
      bcur[2 * t + 1] = run + c0;
    }
    __syncthreads();
    for (uint32_t i = t; i < nt; i += kTmThreads) member[atomicAdd(&bcur[(uint32_t)(key[i] >> 54)], 1u)] = (uint16_t)i;
    __syncthreads();
    for (uint32_t i = t; i < nt; i += kTmThreads) {   // rank = bin start + smaller (key, index) in the bin
      const uint64_t a = key[i];
      const uint32_t d = (uint32_t)(a >> 54), end = bcur[d], beg = end - bcnt[d];
      uint32_t r = beg;
      for (uint32_t m = beg; m < end; ++m) {
        const uint32_t x = member[m];
        const uint64_t b = key[x];
        r += (b < a || (b == a && x < i)) ? 1u : 0u;
      }
      rnk[i] = (uint16_t)r;
    }
    __syncthreads();
#pragma unroll
    for (uint32_t h = 0; h < kTmRows; ++h) {
      const uint32_t i = t + h * kTmThreads;
      if (i < nt) {
        uint32_t* dst = o + (uint32_t)rnk[i] * RW;
#pragma unroll
        for (uint32_t q = 0; q < F; ++q) *reinterpret_cast<u32x4u*>(dst + 4 * q) = v[h][q];
#pragma unroll
        for (uint32_t q = 0; q < T; ++q) dst[4 * F + q] = tail[h][q];
      }
    }
    __syncthreads();
  }
}

// Send side of the fine-bucket exchange over a MATERIALISED table (hbm:// / partfile:// rows or
// the generator's table): out row p (100-byte rows back to back) := input row (uint32)ent[q(p)],
// q(p) = seg[s].ent + p - seg[s].out for the last segment s starting at or before p (one segment
// per (round, destination): the send buffer is round-major, every piece in fine-bucket order).
// PW = input pitch in dwords: 32 (one aligned 128-byte line per row: every random row read is one
// HBM line) or 25 (rows back to back, 4-byte aligned).  One workgroup moves 256 rows per tile:
// their entry indices to LDS, then 8 lanes per row issue the row's 16-byte loads (7 per row, all
// 8 rows of a lane in flight before any is used) into an LDS stage at the output pitch, and the
// tile leaves as contiguous 16-byte nontemporal stores.  ``err`` (nullable): the look-back sort's
// error word; non-zero means the entries are not a permutation, and nothing is read.  An index
// past n_in (a broken caller) is not dereferenced: the row is zero-filled and *bad is set.
template <int PW, int OW>
__global__ __launch_bounds__(256) void ts_pack_rows_kernel(const uint32_t* __restrict__ rows, uint64_t n_in,
                                                           const E64* __restrict__ ent, uint64_t n,
                                                           const int64_t* __restrict__ seg, uint32_t nseg,
                                                           uint32_t* __restrict__ out, const int32_t* __restrict__ err,
                                                           uint32_t* __restrict__ bad) {
  constexpr uint32_t P = (OW + 3) / 4;             // 16-byte pieces per row (the last may be partial)
  static_assert(P <= 8 && PW >= OW, "rows of at most 128 bytes");
  __shared__ __attribute__((aligned(16))) uint32_t stage[256 * OW];
  __shared__ uint32_t sidx[256];
  __shared__ int64_t sseg[256][2];
  const uint32_t t = threadIdx.x;
  if (err != nullptr && *err != 0) return;
  for (uint32_t k = t; k < 2 * nseg; k += 256) sseg[k >> 1][k & 1] = seg[k];
  __syncthreads();
  for (uint64_t row0 = (uint64_t)blockIdx.x * 256; row0 < n; row0 += (uint64_t)gridDim.x * 256) {
    const uint32_t rows_here = (uint32_t)((n - row0) < 256 ? (n - row0) : 256);
    if (t < rows_here) {
      const uint64_t p = row0 + t;
      uint32_t lo = 0, hi = nseg;                  // last segment with out <= p
      while (hi - lo > 1) {
        const uint32_t mid = (lo + hi) >> 1;
        if ((uint64_t)sseg[mid][0] <= p) lo = mid; else hi = mid;
      }
      const uint64_t q = nseg ? (uint64_t)sseg[lo][1] + (p - (uint64_t)sseg[lo][0]) : p;
      uint32_t i = (uint32_t)ent[q].v;
      if (i >= n_in) {
        atomicOr(bad, 1u);
        i = 0xFFFFFFFFu;
      }
      sidx[t] = i;
    }
    __syncthreads();
    {
      const uint32_t g = t >> 3, sub = t & 7;
      u32x4u buf[8];
#pragma unroll
      for (int k = 0; k < 8; ++k) {
        const uint32_t r = g + 32 * k;
        buf[k] = u32x4u{0u, 0u, 0u, 0u};
        if (r < rows_here && sub < P && sidx[r] != 0xFFFFFFFFu) {
          const uint32_t* src = rows + (uint64_t)sidx[r] * PW + sub * 4;
          if (PW == 32) {                      // line-aligned input: whole 16-byte pieces are there
            const uint4* s4 = reinterpret_cast<const uint4*>(src);
            buf[k].x = __builtin_nontemporal_load(&s4->x);
            buf[k].y = __builtin_nontemporal_load(&s4->y);
            buf[k].z = __builtin_nontemporal_load(&s4->z);
            buf[k].w = __builtin_nontemporal_load(&s4->w);
          } else if ((sub + 1) * 4 <= (uint32_t)OW) {
            buf[k] = *reinterpret_cast<const u32x4u*>(src);
          } else {                             // the row's last, partial piece: never read past it
            buf[k].x = src[0];
            if (OW % 4 > 1) buf[k].y = src[1];
            if (OW % 4 > 2) buf[k].z = src[2];
          }
        }
      }
#pragma unroll
      for (int k = 0; k < 8; ++k) {
        const uint32_t r = g + 32 * k;
        if (r < rows_here && sub < P) {
          uint32_t* d = stage + r * OW + sub * 4;
          d[0] = buf[k].x;
          if ((sub + 1) * 4 <= (uint32_t)OW) {
            d[1] = buf[k].y;
            d[2] = buf[k].z;
            d[3] = buf[k].w;
          } else {
            if (OW % 4 > 1) d[1] = buf[k].y;
            if (OW % 4 > 2) d[2] = buf[k].z;
          }
        }
      }
    }
    __syncthreads();
    uint32_t* o = out + row0 * OW;
    const uint32_t words = rows_here * OW;
    uint32_t head = (4u - (uint32_t)((reinterpret_cast<uintptr_t>(o) >> 2) & 3u)) & 3u;
    head = head < words ? head : words;
    if (t < head) o[t] = stage[t];
    const uint32_t nch = (words - head) >> 2;
    if (head == 0) {                 // (a tile starts at a multiple of 256 rows: always, for an aligned out)
      typedef uint32_t u32x4n __attribute__((ext_vector_type(4)));
      for (uint32_t c = t; c < nch; c += 256) {  // one 16-byte nontemporal store per lane and chunk
        const u32x4n v = *reinterpret_cast<const u32x4n*>(stage + 4 * c);
        __builtin_nontemporal_store(v, reinterpret_cast<u32x4n*>(o + 4 * c));
      }
    } else {
      for (uint32_t c = t; c < nch; c += 256) {
        const uint32_t q = head + 4 * c;
        uint32_t* d = o + q;
        __builtin_nontemporal_store(stage[q], d);
        __builtin_nontemporal_store(stage[q + 1], d + 1);
        __builtin_nontemporal_store(stage[q + 2], d + 2);
        __builtin_nontemporal_store(stage[q + 3], d + 3);
      }
    }
    for (uint32_t q = head + 4 * nch + t; q < words; q += 256) o[q] = stage[q];
    __syncthreads();
  }
}

}  // namespace

// Send rows of a materialised table in the order of window-sorted E64 entries (see
// ts_pack_rows_kernel).  rows: n_in input rows at `pitch` bytes (100 or 128; 128 needs 16-byte
// alignment); out: n rows of 100 bytes; seg: nseg <= 256 segments {out row, entry} (device int64
// [nseg][2], seg[0].out = 0, ascending), or nseg = 0 for q(p) = p; err: look-back error word
// (nullable); bad: set when an entry's row index is out of range.
namespace {

// Rows of 4 * RW bytes, RW = 2 .. 32 (8-byte to 128-byte records), dispatched to their template.
#define DR_TS_WIDTHS(X) X(2) X(3) X(4) X(5) X(6) X(7) X(8) X(9) X(10) X(11) X(12) X(13) X(14) X(15) X(16) \
  X(17) X(18) X(19) X(20) X(21) X(22) X(23) X(24) X(25) X(26) X(27) X(28) X(29) X(30) X(31) X(32)

int pack_rows_w(const uint8_t* rows, uint64_t n_in, uint32_t pitch, const E64* ent, uint64_t n, const int64_t* seg,
                uint32_t nseg, uint8_t* out, uint32_t rec, const int32_t* err, uint32_t* bad, hipStream_t s) {
  if (n == 0) return 0;
  if (nseg > 256 || (nseg > 0 && seg == nullptr) || bad == nullptr) return (int)hipErrorInvalidValue;
  if ((reinterpret_cast<uintptr_t>(out) | reinterpret_cast<uintptr_t>(rows)) & 3) return (int)hipErrorInvalidValue;
  if (rec % 4 || rec < 8 || rec > 128 || (pitch != rec && pitch != 128)) return (int)hipErrorInvalidValue;
  if (pitch == 128 && (reinterpret_cast<uintptr_t>(rows) & 15)) return (int)hipErrorInvalidValue;
  const unsigned g = grid_for(n, 256, 32768);
  const uint32_t* in = reinterpret_cast<const uint32_t*>(rows);
  uint32_t* o = reinterpret_cast<uint32_t*>(out);
  const uint32_t ow = rec / 4;
#define DR_TS_PACK(w)                                                                             \
  if (ow == (w)) {                                                                                \
    if (pitch == 128) ts_pack_rows_kernel<32, (w)><<<g, 256, 0, s>>>(in, n_in, ent, n, seg, nseg, o, err, bad); \
    else ts_pack_rows_kernel<(w), (w)><<<g, 256, 0, s>>>(in, n_in, ent, n, seg, nseg, o, err, bad);            \
  }
  DR_TS_WIDTHS(DR_TS_PACK)
#undef DR_TS_PACK
  DR_LAUNCH_CHECK();
  return 0;
}

}  // namespace

DR_API int dr_ts_pack_rows(const uint8_t* rows, uint64_t n_in, uint32_t pitch, const E64* ent, uint64_t n,
                           const int64_t* seg, uint32_t nseg, uint8_t* out, const int32_t* err, uint32_t* bad,
                           hipStream_t s) {
  return pack_rows_w(rows, n_in, pitch, ent, n, seg, nseg, out, 100, err, bad, s);
}

// dr_ts_pack_rows for records of `rec` bytes (a multiple of 4, 8..128) at `pitch` (rec or 128).
DR_API int dr_ts_pack_rows_w(const uint8_t* rows, uint64_t n_in, uint32_t pitch, const E64* ent, uint64_t n,
                             const int64_t* seg, uint32_t nseg, uint8_t* out, uint32_t rec, const int32_t* err,
                             uint32_t* bad, hipStream_t s) {
  return pack_rows_w(rows, n_in, pitch, ent, n, seg, nseg, out, rec, err, bad, s);
}

// starts: (1 << fb) + 1 uint32 = for each fine bucket k the first position of `ent` (sorted on
// at least the top fb window bits) whose bucket is >= k; starts[1 << fb] = n.
DR_API int dr_ts_fine_starts(const E64* ent, uint64_t n, uint32_t fb, uint32_t* starts, hipStream_t s) {
  if (fb < 16 || fb > 24 || n >= (1ull << 32)) return (int)hipErrorInvalidValue;   // FINE_MIN/MAX_BITS
  if (n == 0) return (int)hipMemsetAsync(starts, 0, ((size_t(1) << fb) + 1) * sizeof(uint32_t), s);
  if (reinterpret_cast<uintptr_t>(ent) & 15)       // 16-byte pair loads need 16-byte aligned entries
    ts_fine_starts_kernel<false><<<grid_for((n + 3) / 4, 256, 16384), 256, 0, s>>>(ent, n, fb, starts);
  else
    ts_fine_starts_kernel<true><<<grid_for((n + 3) / 4, 256, 16384), 256, 0, s>>>(ent, n, fb, starts);
  DR_LAUNCH_CHECK();
  return 0;
}

DR_API uint32_t dr_ts_tile_cap() { return kTmCap; }

// rows / out: 100-byte rows (4-byte aligned); pre, cnt: [W][K]; outoff: [K]; 16 <= fb <= 24 (the
// caller's FINE_MIN_BITS..FINE_MAX_BITS).  A bucket past kTmCap rows is flagged, never ordered.
namespace {
// Fine buckets that each hold ONE key (every key bit is a bucket bit, e.g. a 2-byte key at
// fb >= 16): the merge is the W slices of a bucket copied in source order, at any bucket size
// (the LDS merge would flag a bucket past its 1024 rows).  One wave per bucket.
__global__ __launch_bounds__(256) void ts_bucket_copy_kernel(const uint8_t* __restrict__ rows,
                                                             uint8_t* __restrict__ out,
                                                             const int64_t* __restrict__ pre,
                                                             const int32_t* __restrict__ cnt,
                                                             const int64_t* __restrict__ outoff, uint32_t W,
                                                             uint32_t K, uint32_t rec) {
  const uint32_t lane = threadIdx.x & 63;
  const uint32_t wave = (blockIdx.x * blockDim.x + threadIdx.x) >> 6;
  const uint32_t waves = (gridDim.x * blockDim.x) >> 6;
  for (uint32_t k = wave; k < K; k += waves) {
    uint64_t dst = (uint64_t)outoff[k] * rec;
    for (uint32_t s = 0; s < W; ++s) {
      const int32_t c = cnt[(uint64_t)s * K + k];
      if (c <= 0) continue;
      const uint64_t src = (uint64_t)pre[(uint64_t)s * K + k] * rec;
      const uint64_t bytes = (uint64_t)c * rec;
      const uint8_t* a = rows + src;
      uint8_t* b = out + dst;
      if (((reinterpret_cast<uintptr_t>(a) | reinterpret_cast<uintptr_t>(b) | bytes) & 15) == 0) {
        const uint4* a4 = reinterpret_cast<const uint4*>(a);
        uint4* b4 = reinterpret_cast<uint4*>(b);
        for (uint64_t i = lane; i < bytes / 16; i += 64) b4[i] = a4[i];
      } else {
        const uint32_t* a1 = reinterpret_cast<const uint32_t*>(a);
        uint32_t* b1 = reinterpret_cast<uint32_t*>(b);
        for (uint64_t i = lane; i < bytes / 4; i += 64) b1[i] = a1[i];
      }
      dst += bytes;
    }
  }
}
}  // namespace

// The merge of fine buckets that each hold one key: bucket k's W slices rows[pre[s, k] ..
// + cnt[s, k]) copied in source order to out[outoff[k]:] (records of `rec` bytes, a multiple of 4).
DR_API int dr_ts_bucket_copy(const uint8_t* rows, uint8_t* out, const int64_t* pre, const int32_t* cnt,
                             const int64_t* outoff, uint32_t W, uint32_t K, uint32_t rec, hipStream_t s) {
  if (W == 0 || rec % 4 || rec == 0) return (int)hipErrorInvalidValue;
  if ((reinterpret_cast<uintptr_t>(rows) | reinterpret_cast<uintptr_t>(out)) & 3) return (int)hipErrorInvalidValue;
  if (K == 0) return 0;
  const unsigned g = (unsigned)((K + 3) / 4 < 65536 ? (K + 3) / 4 : 65536);
  ts_bucket_copy_kernel<<<g, 256, 0, s>>>(rows, out, pre, cnt, outoff, W, K, rec);
  DR_LAUNCH_CHECK();
  return 0;
}

// dr_ts_tile_merge for records of `rec` bytes (a multiple of 4, 12..128) ordered by the key of
// `key_len` <= 10 bytes at byte `key_off` (descending: `desc`).  The TeraSort layout (10-byte key
// at byte 0, ascending) reads the key as three words; any other as bytes.
DR_API int dr_ts_tile_merge_w(const uint8_t* rows, uint8_t* out, const int64_t* pre, const int32_t* cnt,
                              const int64_t* outoff, uint32_t W, uint32_t K, uint32_t fb, uint32_t* overflow,
                              uint32_t rec, uint32_t key_off, uint32_t key_len, uint32_t desc, hipStream_t s) {
  if (W == 0 || W > kTmMaxW || fb < 16 || fb > 24) return (int)hipErrorInvalidValue;
  if ((reinterpret_cast<uintptr_t>(rows) | reinterpret_cast<uintptr_t>(out)) & 3) return (int)hipErrorInvalidValue;
  if (rec % 4 || rec < 12 || rec > 128) return (int)hipErrorInvalidValue;
  if (key_len < 1 || key_len > 10 || key_off + key_len > rec) return (int)hipErrorInvalidValue;
  if (K == 0) return 0;
  const unsigned g = K < 65536u ? K : 65536u;
  const uint32_t* in = reinterpret_cast<const uint32_t*>(rows);
  uint32_t* o = reinterpret_cast<uint32_t*>(out);
  const uint32_t rw = rec / 4;
  const unsigned gb = (K + kTmThreads - 1) / kTmThreads;
  const bool gen = !(key_off == 0 && key_len == 10 && !desc);
  const uint32_t kspec = key_off | (key_len << 8) | ((desc ? 1u : 0u) << 16);
#define DR_TS_MERGE(w)                                                                               \
  if (rw == (w) && (w) >= 3) {                                                                       \
    constexpr uint32_t RWC = (w) >= 3 ? (w) : 3;                                                     \
    if (gen) {                                                                                       \
      ts_tile_merge_kernel<RWC, true><<<g, kTmThreads, 0, s>>>(in, o, pre, cnt, outoff, W, K, fb, overflow, kspec); \
      DR_LAUNCH_CHECK();                                                                             \
      ts_tile_merge_big_kernel<RWC, true><<<gb, kTmThreads, 0, s>>>(in, o, pre, cnt, outoff, W, K, fb, kspec);      \
    } else {                                                                                         \
      ts_tile_merge_kernel<RWC, false><<<g, kTmThreads, 0, s>>>(in, o, pre, cnt, outoff, W, K, fb, overflow, kspec); \
      DR_LAUNCH_CHECK();                                                                             \
      ts_tile_merge_big_kernel<RWC, false><<<gb, kTmThreads, 0, s>>>(in, o, pre, cnt, outoff, W, K, fb, kspec);     \
    }                                                                                                \
    DR_LAUNCH_CHECK();                                                                               \
  }
  DR_TS_WIDTHS(DR_TS_MERGE)
#undef DR_TS_MERGE
  return 0;
}

DR_API int dr_ts_tile_merge(const uint8_t* rows, uint8_t* out, const int64_t* pre, const int32_t* cnt,
                            const int64_t* outoff, uint32_t W, uint32_t K, uint32_t fb, uint32_t* overflow,
                            hipStream_t s) {
  return dr_ts_tile_merge_w(rows, out, pre, cnt, outoff, W, K, fb, overflow, 100, 0, 10, 0, s);
}
