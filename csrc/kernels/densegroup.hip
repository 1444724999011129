// Dense-key GroupBy aggregation: partition packed rows by key bits, then aggregate each
// partition in an LDS table addressed directly by the key's low bits (no sort, no hashing, no
// gather through a permutation).
//
// BASELINE config "GroupBy-Aggregate 10B x 64-byte records" with keys uniform over 2^30: almost
// every key is its own group (738M groups per 1.25e9 rows), so a partial aggregation shrinks
// nothing and the sort-based path pays 4 radix passes plus a random-row gather (45 ms of 32-byte
// reads through the permutation, profiles/r2_kernels_gb.csv).  The reference's ParallelHashGroupBy
// (DryadLinqVertex.cs:5342-6417) hashes every record into a per-thread dictionary; on MI355X the
// dictionary becomes a 2^12-slot LDS table per workgroup, reached after two stable partition
// passes over 16-byte rows:
//
//   row          key - kmin (kbits) | v0 - vmin0 | v1 - vmin1 | v2 - vmin2, bit-packed into 128 bits
//                (the caller derives the widths from column bounds: generator metadata or a pass)
//   pass 1       columns -> rows, stable partition by key bits [tb, tb + d1)     (dg_scatter<true>)
//   pass 2       rows -> rows, stable partition by key bits [tb + d1, kbits)    (dg_scatter<false>)
//                => rows ordered by key >> tb: every run of equal key >> tb is one LDS table
//   aggregate    every workgroup streams an equal slice of the rows (ends moved to run starts by
//                two 64-ary wave searches), folds each run into the table with LDS integer atomics
//                (count, sum / min / max of the offsets) and emits the occupied slots when the run
//                id changes (global output cursor)
//
// Each partition pass is count (per-workgroup histograms, bucket-major) + exclusive scan (host
// side, torch) + scatter: a workgroup ranks an 8192-row tile (4096 at 10-bit digits) by digit with
// wave64 multisplits, writes the rows into LDS in bucket order and stores every bucket's run
// contiguously.
#include "common.h"

namespace {
// Aggregate workgroups are kAgThreads (16 waves); partition passes see DgSc.  Scattered 16-byte
// rows (2048-row tiles into 1024 buckets) measured 2.5-2.8x the written bytes at the memory side,
// so a tile holds as many rows per bucket as the LDS allows.
constexpr int kDgThreads = 512;
constexpr int kDgWaves = kDgThreads / 64;
#ifndef DR_DG_WPE
#define DR_DG_WPE 4
#endif
#ifndef DR_DG_GMAX
#define DR_DG_GMAX 1536
#endif
#ifndef DR_DG_LDS_MATCH
#define DR_DG_LDS_MATCH 1     // in-wave digit match: 1 LDS atomicOr masks (~1 % faster per pass, profiles/r6/kernels/dg_ab_*), 0 ballots per digit bit
#endif
#ifndef DR_DG_BIG_TILE
#define DR_DG_BIG_TILE 8192   // rows per tile of the <= 9-bit-digit passes (profiles/r6/kernels/dg_tile8k_ab.txt)
#endif
// Partition-pass shape per digit width: <= 512 buckets stage 8192-row tiles (128 KB of LDS, one
// 1024-thread workgroup per CU, 16 rows = 256 bytes per bucket per tile on average); 1024 buckets
// keep 4096-row tiles in 512-thread workgroups (two per CU) for the LDS of their wave counts.
// Fewer, longer bucket runs per tile are fewer partial lines at the memory side: 8192-row tiles cut
// the two passes of the 2^30-key GroupBy from 16.5 + 12.7 to 15.0 + 11.2 ms.
template <int DB>
struct DgSc {
  static constexpr int tile = DB <= 9 ? DR_DG_BIG_TILE : 4096;
  static constexpr int threads = tile >= 8192 ? 1024 : 512;
  static constexpr int waves = threads / 64;
  static constexpr int items = tile / threads;     // rows per thread per tile
  static constexpr int wpe = DB <= 9 ? DR_DG_WPE : 2;  // 10-bit digits: one workgroup per CU by LDS
};
constexpr int kDgGridTile = DR_DG_BIG_TILE > 4096 ? DR_DG_BIG_TILE : 4096;  // per_block granule
constexpr int kDgMaxDigit = 10;               // digit bits per pass (1024 buckets)
constexpr int kDgTableBits = 12;              // LDS table slots per run: 4096
constexpr int kDgSlots = 1 << kDgTableBits;
constexpr int kDgMaxCols = 3;

typedef unsigned __int128 u128;

struct DgPack {
  const int64_t* key;
  const int64_t* col[kDgMaxCols];
  int64_t kmin;
  int64_t vmin[kDgMaxCols];
  uint32_t kbits;
  uint32_t vbits[kDgMaxCols];
  uint32_t ncols;
};

// Exclusive scan across a workgroup of NW waves; scratch holds NW words of LDS.
template <int NW = kDgWaves>
__device__ __forceinline__ uint32_t dg_block_scan(uint32_t v, uint32_t* scratch, uint32_t& total) {
  const int w = wave_id(), l = lane_id();
  const uint32_t inc = wave_inclusive_scan(v);
  if (l == 63) scratch[w] = inc;
  __syncthreads();
  uint32_t base = 0, tot = 0;
#pragma unroll
  for (int k = 0; k < NW; ++k) {
    const uint32_t x = scratch[k];
    base += k < w ? x : 0u;
    tot += x;
  }
  total = tot;
  __syncthreads();
  return base + inc - v;
}

__device__ __forceinline__ uint64_t dg_field(u128 r, uint32_t off, uint32_t bits) {
  const uint64_t v = (uint64_t)(r >> off);
  return bits >= 64 ? v : (v & ((1ull << bits) - 1));
}

// per-(bucket, workgroup) histogram of digit = (key offset >> shift) & (2^dbits - 1), either from
// the int64 key column (ROWS = false) or from the packed rows (ROWS = true)
// With ROWS and a non-null `joint`, also the size of every run (key offset >> table bits) of the
// final order: the rows come from the first pass, sorted by its digit (the low bits of the run id),
// so a workgroup's slice spans a few low-digit values: counted in an LDS window of kDgWin of them
// (x the 2^dbits high digits), rows outside it straight into `joint` (global atomics).
constexpr int kDgWin = 4;

template <bool ROWS>
__global__ __launch_bounds__(256) void dg_count_kernel(const int64_t* __restrict__ key, const uint4* __restrict__ rows,
                                                       uint64_t n, int64_t kmin, uint32_t kbits, uint32_t shift,
                                                       uint32_t dbits, uint32_t* __restrict__ counts, uint32_t G,
                                                       uint64_t per_block, uint32_t* __restrict__ joint,
                                                       uint32_t lo_bits) {
  __shared__ uint32_t hist[1 << kDgMaxDigit];
  __shared__ uint32_t jw[ROWS ? kDgWin << kDgMaxDigit : 1];
  const int t = threadIdx.x;
  const uint32_t nb = 1u << dbits, mask = nb - 1;
  const uint32_t lomask = (1u << lo_bits) - 1;
  for (uint32_t i = t; i < nb; i += kBlock) hist[i] = 0;
  if (ROWS && joint)
    for (uint32_t i = t; i < (uint32_t)kDgWin * nb; i += kBlock) jw[i] = 0;
  __syncthreads();
  const uint64_t beg = (uint64_t)blockIdx.x * per_block;
  const uint64_t end = beg + per_block < n ? beg + per_block : n;
  const uint64_t kmask = kbits >= 64 ? ~0ull : ((1ull << kbits) - 1);
  uint32_t lo0 = 0;
  if (ROWS && joint && beg < end) {
    const uint4 r = rows[beg];
    lo0 = (uint32_t)(((((uint64_t)r.y << 32) | r.x) & kmask) >> kDgTableBits) & lomask;
  }
  for (uint64_t i = beg + t; i < end; i += kBlock) {
    uint64_t ko;
    if constexpr (ROWS) {
      const uint4 r = rows[i];
      ko = (((uint64_t)r.y << 32) | r.x) & kmask;
    } else {
      ko = (uint64_t)(key[i] - kmin);
    }
    const uint32_t d = (uint32_t)((ko >> shift) & mask);
    atomicAdd(&hist[d], 1u);
    if (ROWS && joint) {
      const uint32_t lo = (uint32_t)(ko >> kDgTableBits) & lomask;
      if (lo - lo0 < (uint32_t)kDgWin) atomicAdd(&jw[d * kDgWin + (lo - lo0)], 1u);
      else atomicAdd(&joint[((uint64_t)d << lo_bits) | lo], 1u);
    }
  }
  __syncthreads();
  for (uint32_t i = t; i < nb; i += kBlock) counts[(uint64_t)i * G + blockIdx.x] = hist[i];
  if (ROWS && joint)
    for (uint32_t i = t; i < (uint32_t)kDgWin * nb; i += kBlock) {
      const uint32_t v = jw[i];
      const uint32_t lo = lo0 + i % kDgWin;
      if (v && lo <= lomask) atomicAdd(&joint[((uint64_t)(i / kDgWin) << lo_bits) | lo], v);
    }
}

// Stable partition of rows [beg, end) of each workgroup by digit; offsets[d * G + b] = first output
// row of workgroup b's bucket d (exclusive prefix of the bucket-major counts).
template <bool FROM_COLS, int DB>
__global__ __launch_bounds__(DgSc<DB>::threads) __attribute__((amdgpu_waves_per_eu(DgSc<DB>::wpe))) void dg_scatter_kernel(DgPack pk, const uint4* __restrict__ in, uint64_t n,
                                                         uint32_t shift, const int64_t* __restrict__ offsets, uint32_t G,
                                                         uint64_t per_block, uint4* __restrict__ out) {
  constexpr uint32_t nb = 1u << DB, mask = nb - 1;
  constexpr int kT = DgSc<DB>::tile, kTh = DgSc<DB>::threads, kNW = DgSc<DB>::waves, kIt = DgSc<DB>::items;
  constexpr int kPer = (nb + kTh - 1) / kTh;   // buckets per thread in the scans
  // 16-bit wave counts and bucket starts (<= kT) and no per-slot digit array (recomputed from
  // the staged row): 149 KB of LDS at DB = 9 (one workgroup per CU), 85 KB at DB = 10 (two)
  __shared__ uint4 tile[kT];
  __shared__ uint16_t wcnt[kNW][nb];
  __shared__ int64_t goff[nb];
  __shared__ uint16_t bstart[nb];
  __shared__ uint32_t sc[kNW];
  const int t = threadIdx.x, w = wave_id(), l = lane_id();
  const uint64_t beg = (uint64_t)blockIdx.x * per_block;
  const uint64_t end = beg + per_block < n ? beg + per_block : n;
  if (beg >= end) return;                              // uniform: the whole workgroup leaves
  const uint64_t kmask = pk.kbits >= 64 ? ~0ull : ((1ull << pk.kbits) - 1);
  for (uint32_t i = t; i < nb; i += kTh) goff[i] = offsets[(uint64_t)i * G + blockIdx.x];
  // raw inputs of one tile: the key and value columns (FROM_COLS) or the packed rows
  constexpr int kRaw = FROM_COLS ? 1 + kDgMaxCols : 1;
  int64_t rawc[FROM_COLS ? kIt : 1][kRaw];
  uint4 rawr[FROM_COLS ? 1 : kIt];
  auto load_raw = [&](uint64_t tb) {
#pragma unroll
    for (int r = 0; r < kIt; ++r) {
      const uint64_t i = tb + w * (kT / kNW) + r * 64 + l;
      const bool ok = i < end;
      if constexpr (FROM_COLS) {
        rawc[r][0] = ok ? pk.key[i] : pk.kmin;
#pragma unroll
        for (int j = 0; j < kDgMaxCols; ++j)
          rawc[r][1 + j] = (ok && j < (int)pk.ncols) ? pk.col[j][i] : pk.vmin[j];
      } else {
        rawr[r] = ok ? in[i] : make_uint4(0u, 0u, 0u, 0u);
      }
    }
  };
  for (uint64_t base = beg; base < end; base += kT) {
    const uint32_t cnt = (uint32_t)((end - base) < (uint64_t)kT ? (end - base) : kT);
    // 16 waves per CU either way: while some waves rank or store, others' loads are in flight (a
    // register prefetch of the next tile would need ~150-180 VGPRs)
    load_raw(base);
    for (uint32_t i = t; i < kNW * nb; i += kTh) (&wcnt[0][0])[i] = 0;
#if DR_DG_LDS_MATCH
    static_assert(kNW * nb * 8 <= kT * 16, "the digit masks fit the row stage");
    for (uint32_t i = t; i < kNW * nb; i += kTh) reinterpret_cast<unsigned long long*>(tile)[i] = 0ull;
#endif
    uint4 rv[kIt];
#pragma unroll
    for (int r = 0; r < kIt; ++r) {
      if constexpr (FROM_COLS) {
        u128 v = (u128)(uint64_t)(rawc[r][0] - pk.kmin);
        uint32_t off = pk.kbits;
#pragma unroll
        for (int j = 0; j < kDgMaxCols; ++j) {
          if (j < (int)pk.ncols) {
            v |= (u128)(uint64_t)(rawc[r][1 + j] - pk.vmin[j]) << off;
            off += pk.vbits[j];
          }
        }
        rv[r] = make_uint4((uint32_t)v, (uint32_t)(v >> 32), (uint32_t)(v >> 64), (uint32_t)(v >> 96));
      } else {
        rv[r] = rawr[r];
      }
    }
    __syncthreads();
    uint32_t rk[kIt], dg[kIt];
#pragma unroll
    for (int r = 0; r < kIt; ++r) {
      const uint32_t pos = w * (kT / kNW) + r * 64 + l;
      const bool valid = pos < cnt;
      const uint64_t ko = (((uint64_t)rv[r].y << 32) | rv[r].x) & kmask;
      const uint32_t d = valid ? (uint32_t)((ko >> shift) & mask) : 0u;
#if DR_DG_LDS_MATCH
      // wave64 multisplit by per-wave digit masks in LDS (aliasing the row stage, which is only
      // written after the ranking): one ds_or_b64 per lane, the mask read back, cleared by the leader
      unsigned long long* wm = reinterpret_cast<unsigned long long*>(tile) + (uint32_t)w * nb;
      if (valid) atomicOr(&wm[d], 1ull << l);
      __builtin_amdgcn_wave_barrier();
      const uint64_t peers = valid ? wm[d] : 0ull;
#else
      // wave64 multisplit: the lanes holding the same digit, by one ballot per digit bit
      uint64_t peers = ballot64(valid);
#pragma unroll
      for (int k = 0; k < DB; ++k) {
        const bool bit = (d >> k) & 1u;
        const uint64_t b = ballot64(bit);
        peers &= bit ? b : ~b;
      }
#endif
      const uint32_t below = popc_below(peers);
      const uint32_t prior = wcnt[w][d];
      __builtin_amdgcn_wave_barrier();
      if (valid && below == 0) {
        wcnt[w][d] = (uint16_t)(prior + (uint32_t)__popcll(peers));
#if DR_DG_LDS_MATCH
        wm[d] = 0ull;
#endif
      }
      __builtin_amdgcn_wave_barrier();
      rk[r] = prior + below;
      dg[r] = d;
    }
    __syncthreads();
    // bucket totals, wave offsets inside each bucket, and the bucket starts inside the tile
    uint32_t tot[kPer], run = 0;
#pragma unroll
    for (int q = 0; q < kPer; ++q) {
      const uint32_t b = t * kPer + q;
      tot[q] = 0;
      if (b < nb) {
        uint32_t acc = 0;
#pragma unroll
        for (int k = 0; k < kNW; ++k) {
          const uint32_t c = wcnt[k][b];
          wcnt[k][b] = (uint16_t)acc;
          acc += c;
        }
        tot[q] = acc;
      }
      run += tot[q];
    }
    uint32_t all;
    uint32_t pre = dg_block_scan<kNW>(run, sc, all);
#pragma unroll
    for (int q = 0; q < kPer; ++q) {
      const uint32_t b = t * kPer + q;
      if (b < nb) bstart[b] = (uint16_t)pre;
      pre += tot[q];
    }
    __syncthreads();
#pragma unroll
    for (int r = 0; r < kIt; ++r) {
      const uint32_t pos = w * (kT / kNW) + r * 64 + l;
      if (pos < cnt) {
        const uint32_t slot = (uint32_t)bstart[dg[r]] + wcnt[w][dg[r]] + rk[r];
        tile[slot] = rv[r];
      }
    }
    __syncthreads();
    // consecutive slots of one bucket are consecutive output rows
#pragma unroll 4
    for (uint32_t j = t; j < cnt; j += kTh) {
      const uint4 v = tile[j];
      const uint32_t d = (uint32_t)((((((uint64_t)v.y << 32) | v.x) & kmask) >> shift) & mask);
      out[goff[d] + (int64_t)(j - bstart[d])] = v;
    }
    __syncthreads();
#pragma unroll
    for (int q = 0; q < kPer; ++q) {
      const uint32_t b = t * kPer + q;
      if (b < nb) goff[b] += tot[q];
    }
  }
}

#ifndef DR_DG_AGG_NT
#define DR_DG_AGG_NT 1024     // 16 waves per CU: 9.86 vs 11.92 ms at 512 (profiles/r6/kernels/dg_agg_ab.txt)
#endif
#ifndef DR_DG_AGG_U
#define DR_DG_AGG_U 4
#endif
constexpr int kAgThreads = DR_DG_AGG_NT;      // aggregation workgroup (one per CU by its 112 KB table)
constexpr int kAgWaves = kAgThreads / 64;

struct DgAgg {
  uint32_t nacc;
  uint32_t pack;                 // PACK: the Sum accumulator that carries the count
  uint32_t op[kDgMaxCols];       // 0 = sum, 1 = min, 2 = max (of the column's offsets)
  uint32_t field_off[kDgMaxCols];
  uint32_t field_bits[kDgMaxCols];
  int64_t vmin[kDgMaxCols];
};

// The rows are sorted by run id (key offset >> table bits); rstart[r] .. rstart[r + 1] are run r's
// rows.  Workgroup b folds the runs [wrun[b], wrun[b + 1]) (equal row shares) into its LDS table,
// kU * kAgThreads rows per step with the next step's rows (possibly of the next run) in flight, and
// emits the table at the end of each run: no barrier inside a run.
//
// PACK (a Sum aggregate ag.pack of a field of <= 32 bits, runs of < 2^16 rows): the count rides
// in the top 16 bits of that sum's 64-bit slot, one LDS atomic per row fewer.
//
// Emission: slot q * kAgThreads + t is thread t's in round q.  Each wave compacts its occupied slots of a
// round with a ballot, so every wave store writes one contiguous range of each output column (the
// slot-major assignment wrote 8 scattered elements per thread and cost ~2.5x the bytes written).
template <bool PACK>
__device__ __forceinline__ void dg_agg_body(const uint4* __restrict__ rows, const int64_t* __restrict__ rstart,
                                            const int64_t* __restrict__ wrun, int64_t kmin, const DgAgg& ag,
                                            unsigned long long* __restrict__ head, int64_t* __restrict__ okey,
                                            int64_t* __restrict__ ocnt, int64_t* const* oacc, uint32_t* cnt,
                                            unsigned long long (*acc)[kDgSlots], uint32_t* wtot,
                                            unsigned long long* obase) {
  const int t = threadIdx.x, w = wave_id(), l = lane_id();
  constexpr int kRounds = kDgSlots / kAgThreads;
  constexpr int kU = DR_DG_AGG_U;                       // rows per thread per step
  constexpr uint64_t kStep = (uint64_t)kU * kAgThreads;
  constexpr unsigned long long kOne = 1ull << 48, kLow = kOne - 1;
  const int64_t r1 = wrun[blockIdx.x + 1];
  auto reset = [&](int sl) {
    if (!PACK) cnt[sl] = 0;
#pragma unroll
    for (int a = 0; a < kDgMaxCols; ++a)
      if (a < (int)ag.nacc) acc[a][sl] = ag.op[a] == 1 ? ~0ull : 0ull;
  };
  for (int q = 0; q < kRounds; ++q) reset(q * kAgThreads + t);
  auto emit = [&](uint64_t run) {
    uint32_t pos[kRounds];
    uint32_t mine = 0;
#pragma unroll
    for (int q = 0; q < kRounds; ++q) {
      const int sl = q * kAgThreads + t;
      const bool occ = PACK ? acc[ag.pack][sl] != 0ull : cnt[sl] != 0u;
      const uint64_t bal = ballot64(occ);
      pos[q] = popc_below(bal);
      mine |= (uint32_t)occ << q;
      if (l == 0) wtot[q * kAgWaves + w] = (uint32_t)__popcll(bal);
    }
    __syncthreads();
    static_assert(kRounds * kAgWaves <= 64, "one wave scans the per-(round, wave) counts");
    if (w == 0) {                        // exclusive scan of the (round, wave) counts, one lane each
      const uint32_t c = l < kRounds * kAgWaves ? wtot[l] : 0u;
      const uint32_t inc = wave_inclusive_scan(c);
      if (l < kRounds * kAgWaves) wtot[l] = inc - c;
      if (l == 63) *obase = atomicAdd(head, (unsigned long long)inc);
    }
    __syncthreads();
    uint64_t o = *obase;
#pragma unroll
    for (int q = 0; q < kRounds; ++q) {
      const uint32_t before = wtot[q * kAgWaves + w];
      if ((mine >> q) & 1u) {
        const int sl = q * kAgThreads + t;
        const uint64_t oo = o + before + pos[q];
        const uint32_t c = PACK ? (uint32_t)(acc[ag.pack][sl] >> 48) : cnt[sl];
        okey[oo] = kmin + (int64_t)((run << kDgTableBits) | (uint64_t)sl);
        ocnt[oo] = c;
#pragma unroll
        for (int a = 0; a < kDgMaxCols; ++a) {
          if (a < (int)ag.nacc) {
            const int64_t av = PACK && a == (int)ag.pack ? (int64_t)(acc[a][sl] & kLow) : (int64_t)acc[a][sl];
            oacc[a][oo] = ag.op[a] == 0 ? av + (int64_t)c * ag.vmin[a] : av + ag.vmin[a];
          }
        }
        reset(sl);
      }
    }
    __syncthreads();
  };
  auto advance = [&](int64_t& r, uint64_t& b, uint64_t& e) {
    if (b + kStep < e) { b += kStep; return true; }
    do {
      if (++r >= r1) return false;
      b = (uint64_t)rstart[r];
      e = (uint64_t)rstart[r + 1];
    } while (b == e);
    return true;
  };
  auto load = [&](uint64_t b, uint64_t e, uint4* dst) {
#pragma unroll
    for (int u = 0; u < kU; ++u) {
      const uint64_t i = b + (uint64_t)u * kAgThreads + t;
      dst[u] = i < e ? rows[i] : make_uint4(0u, 0u, 0u, 0u);
    }
  };
  int64_t r = wrun[blockIdx.x] - 1;
  uint64_t b = 0, e = 0;
  if (!advance(r, b, e)) return;                         // uniform: no non-empty run here
  uint4 buf[kU], nbuf[kU];
  load(b, e, buf);
  while (true) {
    int64_t nr = r;
    uint64_t nbg = b, ne = e;
    const bool more = advance(nr, nbg, ne);
    if (more) load(nbg, ne, nbuf);                       // the next step in flight
#pragma unroll
    for (int u = 0; u < kU; ++u) {
      const uint64_t i = b + (uint64_t)u * kAgThreads + t;
      if (i < e) {
        const uint4 rr = buf[u];
        const u128 v = (u128)rr.x | ((u128)rr.y << 32) | ((u128)rr.z << 64) | ((u128)rr.w << 96);
        const uint32_t sl = (uint32_t)((uint64_t)v & (kDgSlots - 1));
        if (!PACK) atomicAdd(&cnt[sl], 1u);
#pragma unroll
        for (int a = 0; a < kDgMaxCols; ++a) {
          if (a < (int)ag.nacc) {
            const unsigned long long f = dg_field(v, ag.field_off[a], ag.field_bits[a]);
            if (ag.op[a] == 0) atomicAdd(&acc[a][sl], PACK && a == (int)ag.pack ? (kOne | f) : f);
            else if (ag.op[a] == 1) atomicMin(&acc[a][sl], f);
            else atomicMax(&acc[a][sl], f);
          }
        }
      }
    }
    if (!more || nr != r) {                               // run r is complete
      __syncthreads();
      emit((uint64_t)r);
    }
    if (!more) break;
#pragma unroll
    for (int u = 0; u < kU; ++u) buf[u] = nbuf[u];
    r = nr;
    b = nbg;
    e = ne;
  }
}

__global__ __launch_bounds__(kAgThreads) void dg_agg_kernel(const uint4* __restrict__ rows,
                                                            const int64_t* __restrict__ rstart,
                                                            const int64_t* __restrict__ wrun, uint32_t kbits,
                                                            int64_t kmin, DgAgg ag, unsigned long long* __restrict__ head,
                                                            int64_t* __restrict__ okey, int64_t* __restrict__ ocnt,
                                                            int64_t* __restrict__ oacc0, int64_t* __restrict__ oacc1,
                                                            int64_t* __restrict__ oacc2, int pack) {
  __shared__ uint32_t cnt[kDgSlots];
  __shared__ unsigned long long acc[kDgMaxCols][kDgSlots];
  __shared__ uint32_t wtot[(kDgSlots / kAgThreads) * kAgWaves];
  __shared__ unsigned long long obase;
  int64_t* const oacc[3] = {oacc0, oacc1, oacc2};
  if (pack)
    dg_agg_body<true>(rows, rstart, wrun, kmin, ag, head, okey, ocnt, oacc, cnt, acc, wtot, &obase);
  else
    dg_agg_body<false>(rows, rstart, wrun, kmin, ag, head, okey, ocnt, oacc, cnt, acc, wtot, &obase);
}
}  // namespace

DR_API uint32_t dr_dg_table_bits() { return kDgTableBits; }
DR_API uint32_t dr_dg_max_digit() { return kDgMaxDigit; }

// Workgroups and rows per workgroup of a partition pass (counts are sized (1 << dbits) * G).
DR_API uint32_t dr_dg_grid(uint64_t n, uint64_t* per_block) {
  uint64_t tiles = (n + kDgGridTile - 1) / kDgGridTile;
  if (tiles < 1) tiles = 1;
  const uint64_t G = tiles < DR_DG_GMAX ? tiles : DR_DG_GMAX;
  *per_block = ((tiles + G - 1) / G) * kDgGridTile;
  return (uint32_t)G;
}

static int dg_pack_from(DgPack* p, const int64_t* key, const int64_t* const* cols, const int64_t* vmin,
                        const uint32_t* vbits, uint32_t ncols, int64_t kmin, uint32_t kbits) {
  if (ncols > (uint32_t)kDgMaxCols || kbits == 0 || kbits > 64) return 1;
  uint32_t tot = kbits;
  p->key = key;
  p->kmin = kmin;
  p->kbits = kbits;
  p->ncols = ncols;
  for (uint32_t j = 0; j < (uint32_t)kDgMaxCols; ++j) {
    p->col[j] = j < ncols ? cols[j] : nullptr;
    p->vmin[j] = j < ncols ? vmin[j] : 0;
    p->vbits[j] = j < ncols ? vbits[j] : 0;
    tot += p->vbits[j];
    if (j < ncols && (vbits[j] == 0 || vbits[j] > 64)) return 1;
  }
  return tot > 128 ? 1 : 0;
}

// rows == null: histogram of the key column; else of the packed rows.
// joint (rows only, may be null): u32 [2^(dbits + lo_bits)] zeroed by the caller, receives the
// size of every run id (digit << lo_bits | low digit) of the final order.
DR_API int dr_dg_count(const int64_t* key, const void* rows, uint64_t n, int64_t kmin, uint32_t kbits, uint32_t shift,
                       uint32_t dbits, uint32_t* counts, uint32_t G, uint64_t per_block, uint32_t* joint,
                       uint32_t lo_bits, hipStream_t s) {
  if (dbits == 0 || dbits > (uint32_t)kDgMaxDigit) return (int)hipErrorInvalidValue;
  if (n == 0) return 0;
  if (rows)
    dg_count_kernel<true><<<G, 256, 0, s>>>(nullptr, static_cast<const uint4*>(rows), n, kmin, kbits, shift, dbits,
                                             counts, G, per_block, joint, lo_bits);
  else
    dg_count_kernel<false><<<G, 256, 0, s>>>(key, nullptr, n, kmin, kbits, shift, dbits, counts, G, per_block,
                                              nullptr, 0);
  DR_LAUNCH_CHECK();
  return 0;
}

// in == null: rows packed from key + cols; else partition the packed rows `in`.
DR_API int dr_dg_scatter(const int64_t* key, const int64_t* const* cols, const int64_t* vmin, const uint32_t* vbits,
                         uint32_t ncols, int64_t kmin, uint32_t kbits, const void* in, uint64_t n, uint32_t shift,
                         uint32_t dbits, const int64_t* offsets, uint32_t G, uint64_t per_block, void* out,
                         hipStream_t s) {
  if (dbits == 0 || dbits > (uint32_t)kDgMaxDigit) return (int)hipErrorInvalidValue;
  DgPack p;
  if (dg_pack_from(&p, key, cols, vmin, vbits, ncols, kmin, kbits)) return (int)hipErrorInvalidValue;
  if (n == 0) return 0;
#define DG_SC(FC, DBV)                                                                                \
  dg_scatter_kernel<FC, DBV><<<G, DgSc<DBV>::threads, 0, s>>>(p, static_cast<const uint4*>(in), n, shift, offsets, G, per_block, \
                                               static_cast<uint4*>(out))
#define DG_SC_ALL(FC)                                                                                 \
  switch (dbits) {                                                                                    \
    case 1: DG_SC(FC, 1); break; case 2: DG_SC(FC, 2); break; case 3: DG_SC(FC, 3); break;            \
    case 4: DG_SC(FC, 4); break; case 5: DG_SC(FC, 5); break; case 6: DG_SC(FC, 6); break;            \
    case 7: DG_SC(FC, 7); break; case 8: DG_SC(FC, 8); break; case 9: DG_SC(FC, 9); break;            \
    default: DG_SC(FC, 10); break;                                                                            \
  }
  if (in) {
    DG_SC_ALL(false);
  } else {
    DG_SC_ALL(true);
  }
#undef DG_SC_ALL
#undef DG_SC
  DR_LAUNCH_CHECK();
  return 0;
}

// rows: packed rows sorted by run id (key offset >> table bits); rstart: int64 [runs + 1] row
// offsets of the runs; wrun: int64 [G + 1] run ranges of the G workgroups.  ops / off / bits / vmin:
// nacc accumulators over packed fields.  head (u64, zeroed) receives the group count; outputs are
// sized by the caller (>= the number of groups).  pack: 1 + the index of a Sum accumulator over a
// field of <= 32 bits when every run is shorter than 2^16 rows (the count then shares its LDS
// slot), else 0.
DR_API int dr_dg_aggregate(const void* rows, const int64_t* rstart, const int64_t* wrun, uint32_t G, uint32_t kbits,
                           int64_t kmin, uint32_t nacc, const uint32_t* ops, const uint32_t* off, const uint32_t* bits,
                           const int64_t* vmin, unsigned long long* head, int64_t* okey, int64_t* ocnt,
                           int64_t* const* oacc, int pack, hipStream_t s) {
  if (nacc > (uint32_t)kDgMaxCols) return (int)hipErrorInvalidValue;
  DgAgg ag;
  ag.nacc = nacc;
  for (uint32_t a = 0; a < (uint32_t)kDgMaxCols; ++a) {
    ag.op[a] = a < nacc ? ops[a] : 0;
    ag.field_off[a] = a < nacc ? off[a] : 0;
    ag.field_bits[a] = a < nacc ? bits[a] : 0;
    ag.vmin[a] = a < nacc ? vmin[a] : 0;
    if (a < nacc && (ag.op[a] > 2 || ag.field_bits[a] == 0 || ag.field_off[a] + ag.field_bits[a] > 128))
      return (int)hipErrorInvalidValue;
  }
  ag.pack = pack > 0 ? (uint32_t)(pack - 1) : 0;
  if (pack && (ag.pack >= nacc || ag.op[ag.pack] != 0 || ag.field_bits[ag.pack] > 32)) return (int)hipErrorInvalidValue;
  if (G == 0) return 0;
  dg_agg_kernel<<<G, kAgThreads, 0, s>>>(static_cast<const uint4*>(rows), rstart, wrun, kbits, kmin, ag, head, okey,
                                         ocnt, nacc > 0 ? oacc[0] : nullptr, nacc > 1 ? oacc[1] : nullptr,
                                         nacc > 2 ? oacc[2] : nullptr, pack);
  DR_LAUNCH_CHECK();
  return 0;
}

// ---------------------------------------------------------------------------------------------
// Dense running state of a streamed GroupBy (runtime/stream_agg.DenseState): one slot per key of
// the range [lo, lo + R), one array per accumulator.  A chunk's (partial) rows fold into it in ONE
// pass: per row the slot index, the occupancy byte, and every accumulator's atomic (count / add /
// min / max), instead of one library scatter kernel per accumulator re-reading the keys.
namespace {
constexpr int kDsMaxSpecs = 8;

struct DsSpecs {
  void* state[kDsMaxSpecs];
  const void* val[kDsMaxSpecs];
  uint32_t op[kDsMaxSpecs];      // 0 count (+1), 1 add, 2 min, 3 max
  uint32_t sdt[kDsMaxSpecs];     // state dtype: 0 int64, 1 float64 (add only)
  uint32_t vdt[kDsMaxSpecs];     // value dtype: 0 int64, 1 float64, 2 int32, 3 int8, 4 float32, 5 int16
  uint32_t nspec;
};

__device__ __forceinline__ int64_t ds_load_i(const void* p, uint32_t dt, uint64_t i) {
  switch (dt) {
    case 0: return static_cast<const int64_t*>(p)[i];
    case 2: return static_cast<const int32_t*>(p)[i];
    case 3: return static_cast<const int8_t*>(p)[i];
    case 5: return static_cast<const int16_t*>(p)[i];
    case 1: return (int64_t) static_cast<const double*>(p)[i];
    default: return (int64_t) static_cast<const float*>(p)[i];
  }
}

__device__ __forceinline__ double ds_load_f(const void* p, uint32_t dt, uint64_t i) {
  if (dt == 1) return static_cast<const double*>(p)[i];
  if (dt == 4) return (double)static_cast<const float*>(p)[i];
  return (double)ds_load_i(p, dt, i);
}

__global__ __launch_bounds__(256) void dense_state_update_kernel(const void* __restrict__ key, uint32_t kdt, uint64_t n,
                                                                 int64_t lo, uint64_t range, uint8_t* __restrict__ seen,
                                                                 DsSpecs sp, uint64_t stride, uint32_t* __restrict__ bad) {
  for (uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (uint64_t)gridDim.x * blockDim.x) {
    const uint64_t idx = (uint64_t)(ds_load_i(key, kdt, i) - lo);
    if (idx >= range) {                  // a key outside the state (a broken caller): not stored
      atomicOr(bad, 1u);
      continue;
    }
    if (seen != nullptr) seen[idx] = 1;
    const uint64_t slot = idx * stride;  // stride > 1: a key's accumulators side by side (one sector)
    for (uint32_t s = 0; s < sp.nspec; ++s) {
      const uint32_t op = sp.op[s];
      if (sp.sdt[s] == 1) {
        atomicAdd(static_cast<double*>(sp.state[s]) + slot, ds_load_f(sp.val[s], sp.vdt[s], i));
        continue;
      }
      long long* st = static_cast<long long*>(sp.state[s]) + slot;
      if (op == 0) {
        atomicAdd(reinterpret_cast<unsigned long long*>(st), 1ull);
      } else {
        const long long v = (long long)ds_load_i(sp.val[s], sp.vdt[s], i);
        if (op == 1) atomicAdd(reinterpret_cast<unsigned long long*>(st), (unsigned long long)v);
        else if (op == 2) atomicMin(st, v);
        else atomicMax(st, v);
      }
    }
  }
}
}  // namespace

// key: n keys of dtype kdt (0 int64, 2 int32, 5 int16, 3 int8); seen: `range` bytes (nullable: a
// count accumulator tells occupancy); state / val / op / sdt / vdt: nspec accumulators (see
// DsSpecs; val ignored for count), key k's slot of accumulator s at state[s][(k - lo) * stride]
// (stride = nspec: one row of 8-byte slots per key).  bad: set when a key falls outside the range.
DR_API int dr_dense_state_update(const void* key, uint32_t kdt, uint64_t n, int64_t lo, uint64_t range, uint8_t* seen,
                                 void* const* state, const void* const* val, const uint32_t* op, const uint32_t* sdt,
                                 const uint32_t* vdt, uint32_t nspec, uint64_t stride, uint32_t* bad, hipStream_t s) {
  if (stride == 0) return (int)hipErrorInvalidValue;
  if (nspec > (uint32_t)kDsMaxSpecs || (kdt != 0 && kdt != 2 && kdt != 3 && kdt != 5)) return (int)hipErrorInvalidValue;
  if (n == 0) return 0;
  DsSpecs sp;
  for (uint32_t k = 0; k < nspec; ++k) {
    if (op[k] > 3 || sdt[k] > 1 || vdt[k] > 5 || (sdt[k] == 1 && op[k] != 1) || (op[k] != 0 && val[k] == nullptr))
      return (int)hipErrorInvalidValue;
    sp.state[k] = state[k];
    sp.val[k] = val[k];
    sp.op[k] = op[k];
    sp.sdt[k] = sdt[k];
    sp.vdt[k] = vdt[k];
  }
  sp.nspec = nspec;
  dense_state_update_kernel<<<grid_for(n, 256, 16384), 256, 0, s>>>(key, kdt, n, lo, range, seen, sp, stride, bad);
  DR_LAUNCH_CHECK();
  return 0;
}
