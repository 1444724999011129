// Partitioned ("grace") hash join of fixed-width row tables for CDNA4 (gfx950).
//
// Reference: DryadLinqVertex.HashJoin / ParallelHashJoin (LinqToDryad/DryadLinqVertex.cs:852-897,
// 6703-7315) builds a hash lookup over the co-partitioned inner side and streams the outer side
// through it; the inputs of both sides were hash partitioned by the join key upstream
// (DryadLinqQueryGen.cs:1419-1609 VisitJoin).  Here the same two phases run on one GPU's HBM:
//
//   partition  rows -> bucket (or rank) by a 64-bit hash of the key bytes.  Per chunk: a count
//              pass (per-workgroup LDS histograms), a per-bucket scan that also advances the
//              bucket fill counters on the device, and a scatter pass that reads each tile of rows
//              coalesced into LDS, ranks it by bucket with wave ballots and writes every bucket's
//              rows as one contiguous run at that bucket's destination (an HBM bucket store, a
//              staging area that is then copied to pinned host DRAM, or an all-to-all send
//              buffer).  No intermediate key entries, no second gather of the rows.
//   join       per bucket pair: an open-addressing table (16-byte slots, linear probing, slots
//              claimed with one CAS on the row-index word) over the build side's keys, sized so a
//              bucket's table stays in the 256 MiB Infinity Cache; the probe side streams through
//              it and either aggregates on the fly (count + sums of one int64 column per side: any
//              linear result selector followed by Sum/Count) or emits (probe row, build row) pairs.
//
// Keys are compared as raw bytes (<= 12 bytes at a 4-byte aligned offset); both sides of a join
// hash identically, which is all a partitioned join needs.
#include "common.h"

namespace {

constexpr uint32_t kEmpty = 0xFFFFFFFFu;
constexpr uint32_t kGMax = 1024;          // count / scatter workgroups (4 per CU)
constexpr uint32_t kMaxBuckets = 256;
constexpr uint64_t kSlotMix = 0xA24BAED4963EE407ull;

struct __attribute__((aligned(16))) HSlot {
  uint64_t k0;
  uint32_t k1;
  uint32_t idx;
};

// Tile of up to 16 * 256 16-byte pieces into LDS: every load of the thread is issued before the
// first LDS store (one wait for all of them instead of one HBM round trip per piece).  idx(q) maps
// a piece to its global 16-byte index.
template <int N = 16, typename F>
__device__ __forceinline__ void tile_to_lds(uint4* __restrict__ lds, const uint4* __restrict__ src, uint32_t pieces,
                                            F idx) {
  uint4 v[N];
  const uint32_t last = pieces ? pieces - 1 : 0;   // clamped, unconditional loads: v stays in VGPRs
#pragma unroll
  for (int i = 0; i < N; ++i) {
    const uint32_t q = threadIdx.x + i * kBlock;
    v[i] = src[idx(q < pieces ? q : last)];
  }
#pragma unroll
  for (int i = 0; i < N; ++i) {
    const uint32_t q = threadIdx.x + i * kBlock;
    if (q < pieces) lds[q] = v[i];
  }
}

__device__ __forceinline__ uint32_t keep_mask(int bytes) {
  return bytes >= 4 ? 0xFFFFFFFFu : (bytes <= 0 ? 0u : ((1u << (8 * bytes)) - 1u));
}

// key bytes at r (4-byte aligned) -> (k0 = bytes 0..7, k1 = bytes 8..11), bytes past key_len zero
template <typename P>
__device__ __forceinline__ void row_key(const P* __restrict__ r, int key_len, uint64_t& k0, uint32_t& k1) {
  const uint32_t d0 = r[0] & keep_mask(key_len);
  const uint32_t d1 = key_len > 4 ? (r[1] & keep_mask(key_len - 4)) : 0u;
  k1 = key_len > 8 ? (r[2] & keep_mask(key_len - 8)) : 0u;
  k0 = (uint64_t)d0 | ((uint64_t)d1 << 32);
}

__device__ __forceinline__ uint64_t key_hash(uint64_t k0, uint32_t k1, uint64_t seed) {
  return mix64(k0 ^ mix64((uint64_t)k1 ^ seed));
}

// destination in [0, nb) from 32 hash bits at `shift` (fast range reduction: any nb)
__device__ __forceinline__ uint32_t dest_of(uint64_t h, int shift, uint32_t nb) {
  return (uint32_t)((((h >> shift) & 0xFFFFFFFFull) * (uint64_t)nb) >> 32);
}

void geometry(uint64_t n, uint32_t tile, uint32_t& G, uint64_t& per_block) {
  uint64_t tiles = (n + tile - 1) / tile;
  if (tiles < 1) tiles = 1;
  G = (uint32_t)(tiles < kGMax ? tiles : kGMax);
  per_block = ((tiles + G - 1) / G) * tile;
}

__global__ __launch_bounds__(256) void gp_count_kernel(const uint32_t* __restrict__ rows, uint64_t n, uint32_t W,
                                                       uint32_t kw, int key_len, uint64_t seed, int shift, uint32_t nb,
                                                       uint32_t* __restrict__ counts, uint32_t G, uint64_t per_block) {
  __shared__ uint32_t hist[4][kMaxBuckets];
  const int t = threadIdx.x, w = wave_id();
  for (int i = t; i < 4 * (int)kMaxBuckets; i += kBlock) (&hist[0][0])[i] = 0;
  __syncthreads();
  const uint64_t beg = (uint64_t)blockIdx.x * per_block;
  const uint64_t end = beg + per_block < n ? beg + per_block : n;
  for (uint64_t i = beg + t; i < end; i += 4 * kBlock) {
    uint64_t k0[4];
    uint32_t k1[4];
#pragma unroll
    for (int u = 0; u < 4; ++u) {
      const uint64_t r = i + (uint64_t)u * kBlock;
      if (r < end) row_key(rows + r * W + kw, key_len, k0[u], k1[u]);
    }
#pragma unroll
    for (int u = 0; u < 4; ++u)
      if (i + (uint64_t)u * kBlock < end) atomicAdd(&hist[w][dest_of(key_hash(k0[u], k1[u], seed), shift, nb)], 1u);
  }
  __syncthreads();
  for (uint32_t b = t; b < nb; b += kBlock)
    counts[(uint64_t)b * G + blockIdx.x] = hist[0][b] + hist[1][b] + hist[2][b] + hist[3][b];
}

// one workgroup per bucket: chunk total of the bucket
__global__ __launch_bounds__(256) void gp_totals_kernel(const uint32_t* __restrict__ counts, uint32_t G,
                                                        uint64_t* __restrict__ totals) {
  __shared__ uint32_t sc[4];
  const uint32_t b = blockIdx.x;
  uint32_t s = 0;
  for (uint32_t g = threadIdx.x; g < G; g += kBlock) s += counts[(uint64_t)b * G + g];
  uint32_t total;
  block_exclusive_scan256(s, sc, total);
  if (threadIdx.x == 0) totals[b] = total;
}

// one workgroup per bucket: exclusive scan of the bucket's per-workgroup counts (in place) and its
// destination base.  Buckets b >= contig_from are laid out back to back from row 0 of their
// pointer (send buffers, spill staging); the others append at their fill counter, which advances
// (a fill past cap is flagged in *overflow; the scatter drops those rows).
__global__ __launch_bounds__(256) void gp_offsets_kernel(uint32_t* __restrict__ counts, uint32_t G,
                                                         const uint64_t* __restrict__ totals,
                                                         int64_t* __restrict__ fill, const int64_t* __restrict__ cap,
                                                         uint32_t contig_from, int64_t* __restrict__ base_out,
                                                         int64_t* __restrict__ chunk_counts,
                                                         uint32_t* __restrict__ overflow) {
  __shared__ uint32_t sc[4];
  const uint32_t b = blockIdx.x, t = threadIdx.x;
  uint32_t v[4];
  uint32_t s = 0;
#pragma unroll
  for (int k = 0; k < 4; ++k) {
    const uint32_t g = 4 * t + k;
    v[k] = g < G ? counts[(uint64_t)b * G + g] : 0u;
    s += v[k];
  }
  uint32_t total;
  uint32_t run = block_exclusive_scan256(s, sc, total);
#pragma unroll
  for (int k = 0; k < 4; ++k) {
    const uint32_t g = 4 * t + k;
    if (g < G) counts[(uint64_t)b * G + g] = run;
    run += v[k];
  }
  if (t == 0) {
    int64_t base = 0;
    if (b >= contig_from) {
      for (uint32_t j = contig_from; j < b; ++j) base += (int64_t)totals[j];
    } else {
      base = fill[b];
      const int64_t nf = base + (int64_t)total;
      if (cap != nullptr && nf > cap[b]) atomicOr(overflow, 1u);
      fill[b] = nf;
    }
    base_out[b] = base;
    chunk_counts[b] = (int64_t)total;
  }
}

// Stable bucket scatter of rows.  ITEMS rows per thread per tile (tile = 256 * ITEMS rows of
// <= 64 KiB), WC = dwords per input row when known at compile time (0: runtime), VEC: 16-byte
// copies.  Projection: the destination rows are input dwords [PO, PO + OW) (column pruning before
// the shuffle: only the columns the join's key and result selector read travel), OWC = OW when
// known at compile time.
// STAGE_PROJ (VEC, OWC > 0, key inside the projection): the LDS image holds only the projected
// dwords of each row, so a 64 KiB tile carries 64 / OWC * 256 rows and each bucket's output run is
// that many times longer (16-byte rows of 64-byte inputs: 4096-row tiles, ~256-byte runs).
// ATOMIC (every destination appends at its fill counter, row order inside a destination free):
// no count pass; each tile reserves its rows per destination with one atomicAdd on the fill
// counter (a join's buckets do not need the input order).  Rows past cap are dropped and flagged.
template <int ITEMS, int WC, int OWC, bool VEC, bool STAGE_PROJ = false, bool ATOMIC = false, int LDSW = 16384,
          int NT = 256>
__global__ __launch_bounds__(NT) void gp_scatter_kernel(const uint32_t* __restrict__ rows, uint64_t n, uint32_t Wdyn,
                                                         uint32_t kw, int key_len, uint64_t seed, int shift, uint32_t nb,
                                                         const uint32_t* __restrict__ prefix,
                                                         const int64_t* __restrict__ base,
                                                         const uint64_t* __restrict__ dst_ptr,
                                                         const int64_t* __restrict__ cap, uint32_t contig_from,
                                                         uint32_t G, uint64_t per_block, uint32_t OWdyn, uint32_t PO,
                                                         int64_t* __restrict__ fill = nullptr,
                                                         uint32_t* __restrict__ overflow = nullptr) {
  constexpr int TILE = NT * ITEMS, NW = NT / 64;
  // projected tiles: one 16-byte piece per row (kGpProjNT x kGpProjItems rows); rows of 129..512
  // bytes: one row per thread in a 128 KiB tile (one workgroup per CU)
  constexpr int LDS_DW = STAGE_PROJ ? TILE * 4 : LDSW;
  static_assert(STAGE_PROJ || LDS_DW >= kBlock * ITEMS, "tile");
  static_assert(NT == kBlock || STAGE_PROJ, "wider workgroups stage projections only");
  static_assert(!STAGE_PROJ || OWC == 4, "staged projections are one 16-byte piece per row");
  const uint32_t W = WC > 0 ? (uint32_t)WC : Wdyn;
  const uint32_t OW = OWC > 0 ? (uint32_t)OWC : OWdyn;
  const uint32_t LW = STAGE_PROJ ? OW : W;            // dwords per row in the LDS image
  const uint32_t LPO = STAGE_PROJ ? 0u : PO;          // projection offset inside the LDS image
  const uint32_t lkw = STAGE_PROJ ? kw - PO : kw;     // key offset inside the LDS image
  __shared__ __attribute__((aligned(16))) uint32_t srow[LDS_DW];
  __shared__ uint16_t perm[TILE];
  __shared__ uint8_t dslot[TILE];
  __shared__ uint32_t wcnt[NW][kMaxBuckets];
  __shared__ int64_t goff[kMaxBuckets];
  __shared__ uint32_t bstart[kMaxBuckets];
  __shared__ uint64_t sptr[kMaxBuckets];
  __shared__ int64_t scap[kMaxBuckets];
  __shared__ uint32_t sc[4];
  const int t = threadIdx.x, w = wave_id(), l = lane_id();
  if ((uint32_t)t < nb) {
    goff[t] = ATOMIC ? 0 : base[t] + (int64_t)prefix[(uint64_t)t * G + blockIdx.x];
    sptr[t] = dst_ptr[t];
    scap[t] = (cap && (uint32_t)t < contig_from) ? cap[t] : (int64_t)0x7FFFFFFFFFFFFFFFll;
  }
  const uint64_t beg = (uint64_t)blockIdx.x * per_block;
  const uint64_t end = beg + per_block < n ? beg + per_block : n;
  // STAGE_PROJ: one 16-byte piece per row, ITEMS per thread, the next tile's loads in flight
  // while this tile is ranked and written out
  static_assert(!STAGE_PROJ || ITEMS <= 8, "staged projections: at most 8 pieces per thread");
  // STAGE_PROJ: the next tile's 8 pieces per thread in 8 named registers (an array is placed in
  // scratch), in flight while this tile is ranked and written out
  uint4 p0, p1, p2, p3, p4, p5, p6, p7;
  const uint32_t pC = W / 4, pP4 = PO / 4;
  auto issue = [&](uint64_t tb2) {
    const uint32_t pieces = (uint32_t)((end - tb2) < (uint64_t)TILE ? (end - tb2) : TILE);
    const uint32_t last = pieces ? pieces - 1 : 0;
    const uint4* src = reinterpret_cast<const uint4*>(rows + tb2 * W);
#define DR_GP_LD(I, P) if (ITEMS > (I)) { const uint32_t q = t + (I) * NT; P = src[(uint64_t)(q < pieces ? q : last) * pC + pP4]; }
    DR_GP_LD(0, p0) DR_GP_LD(1, p1) DR_GP_LD(2, p2) DR_GP_LD(3, p3)
    DR_GP_LD(4, p4) DR_GP_LD(5, p5) DR_GP_LD(6, p6) DR_GP_LD(7, p7)
#undef DR_GP_LD
  };
  if (STAGE_PROJ && beg < end) issue(beg);
  for (uint64_t tb = beg; tb < end; tb += TILE) {
    const uint32_t cnt = (uint32_t)((end - tb) < (uint64_t)TILE ? (end - tb) : TILE);
    if (STAGE_PROJ) {
      uint4* s4 = reinterpret_cast<uint4*>(srow);
#define DR_GP_ST(I, P) if (ITEMS > (I)) { const uint32_t q = t + (I) * NT; if (q < cnt) s4[q] = P; }
      DR_GP_ST(0, p0) DR_GP_ST(1, p1) DR_GP_ST(2, p2) DR_GP_ST(3, p3)
      DR_GP_ST(4, p4) DR_GP_ST(5, p5) DR_GP_ST(6, p6) DR_GP_ST(7, p7)
#undef DR_GP_ST
      if (tb + TILE < end) issue(tb + TILE);
    } else if (VEC) {
      tile_to_lds(reinterpret_cast<uint4*>(srow), reinterpret_cast<const uint4*>(rows + tb * W), cnt * W / 4,
                  [](uint32_t q) { return (uint64_t)q; });
    } else {
      const uint32_t words = cnt * W;
      const uint32_t* src = rows + tb * W;
      for (uint32_t j = t; j < words; j += NT) srow[j] = src[j];
    }
    for (int i = t; i < NW * kMaxBuckets; i += NT) (&wcnt[0][0])[i] = 0;
    __syncthreads();
    uint32_t rk[ITEMS], dg[ITEMS];
#pragma unroll
    for (int r = 0; r < ITEMS; ++r) {
      const uint32_t pos = w * (TILE / NW) + r * 64 + l;
      const bool valid = pos < cnt;
      uint32_t d = 0;
      if (valid) {
        uint64_t k0;
        uint32_t k1;
        row_key(srow + pos * LW + lkw, key_len, k0, k1);
        d = dest_of(key_hash(k0, k1, seed), shift, nb);
      }
      uint64_t peers = ballot64(valid);
#pragma unroll
      for (int k = 0; k < 8; ++k) {
        const bool bit = (d >> k) & 1u;
        const uint64_t bb = ballot64(bit);
        peers &= bit ? bb : ~bb;
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
    uint32_t tot = 0;
    if (t < kMaxBuckets) {
#pragma unroll
      for (int q = 0; q < NW; ++q) {
        const uint32_t c = wcnt[q][t];
        wcnt[q][t] = tot;
        tot += c;
      }
    }
    {
      // exclusive scan of the 256 bucket totals (waves 0..3; other waves only meet the barriers)
      const uint32_t inc = wave_inclusive_scan(tot);
      if (l == 63 && w < 4) sc[w] = inc;
      __syncthreads();
      const uint32_t b0 = (w > 0 ? sc[0] : 0) + (w > 1 ? sc[1] : 0) + (w > 2 ? sc[2] : 0);
      if (t < kMaxBuckets) bstart[t] = b0 + inc - tot;
      __syncthreads();
    }
    if (ATOMIC && (uint32_t)t < nb && tot)
      goff[t] = (int64_t)atomicAdd(reinterpret_cast<unsigned long long*>(fill + t), (unsigned long long)tot);
    __syncthreads();
#pragma unroll
    for (int r = 0; r < ITEMS; ++r) {
      const uint32_t pos = w * (TILE / NW) + r * 64 + l;
      if (pos < cnt) {
        const uint32_t slot = bstart[dg[r]] + wcnt[w][dg[r]] + rk[r];
        perm[slot] = (uint16_t)pos;
        dslot[slot] = (uint8_t)dg[r];
      }
    }
    if (ATOMIC && (uint32_t)t < nb && tot && goff[t] + (int64_t)tot > scap[t]) atomicOr(overflow, 1u);
    __syncthreads();
    // slot-major copy: consecutive lanes write consecutive pieces of consecutive slots, and the
    // slots of one bucket are consecutive rows of its destination
    if (VEC) {
      const uint32_t LC = LW / 4, OC = OW / 4, P4 = LPO / 4;
      const uint32_t chunks = cnt * OC;
      const uint4* s4 = reinterpret_cast<const uint4*>(srow);
      for (uint32_t q = t; q < chunks; q += NT) {
        const uint32_t j = q / OC, c = q - j * OC;
        const uint32_t d = dslot[j];
        const int64_t row = goff[d] + (int64_t)(j - bstart[d]);
        if (row < scap[d])
          reinterpret_cast<uint4*>(sptr[d])[(uint64_t)row * OC + c] = s4[(uint32_t)perm[j] * LC + P4 + c];
      }
    } else {
      const uint32_t words = cnt * OW;
      for (uint32_t q = t; q < words; q += NT) {
        const uint32_t j = q / OW, c = q - j * OW;
        const uint32_t d = dslot[j];
        const int64_t row = goff[d] + (int64_t)(j - bstart[d]);
        if (row < scap[d])
          reinterpret_cast<uint32_t*>(sptr[d])[(uint64_t)row * OW + c] = srow[(uint32_t)perm[j] * LW + LPO + c];
      }
    }
    __syncthreads();
    if (!ATOMIC && (uint32_t)t < nb) goff[t] += tot;
    __syncthreads();
  }
}

// ---------------------------------------------------------------------------------------------
// Open-addressing hash table over the build side's keys.
__device__ __forceinline__ uint64_t slot_of(uint64_t h, uint64_t mask) { return mix64(h ^ kSlotMix) & mask; }

__global__ __launch_bounds__(256) void ht_build_kernel(const uint32_t* __restrict__ rows, uint64_t n, uint32_t W,
                                                       uint32_t kw, int key_len, uint64_t seed, HSlot* __restrict__ table,
                                                       uint64_t mask) {
  const uint64_t stride = (uint64_t)gridDim.x * blockDim.x;
  for (uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += stride) {
    uint64_t k0;
    uint32_t k1;
    row_key(rows + i * W + kw, key_len, k0, k1);
    uint64_t s = slot_of(key_hash(k0, k1, seed), mask);
    for (uint64_t probe = 0; probe <= mask; ++probe) {
      if (atomicCAS(&table[s].idx, kEmpty, (uint32_t)i) == kEmpty) {
        table[s].k0 = k0;
        table[s].k1 = k1;
        break;
      }
      s = (s + 1) & mask;
    }
  }
}

// Probe + fused aggregate: partial[blockIdx] = (matches, sum of the probe rows' int64 column at
// byte col_p once per match, sum of the matched build rows' int64 column at col_b).  Partials are
// plain stores (a same-address atomic per wave serialises at the memory side); ht_sum_partials
// folds them into acc.
__global__ __launch_bounds__(256) void ht_probe_sum_kernel(const uint32_t* __restrict__ prow, uint64_t np, uint32_t Wp,
                                                           uint32_t kwp, int key_len, uint64_t seed,
                                                           const HSlot* __restrict__ table, uint64_t mask,
                                                           const uint8_t* __restrict__ brow, uint32_t stride_b,
                                                           uint32_t col_p, uint32_t col_b,
                                                           uint64_t* __restrict__ partial) {
  __shared__ uint64_t red[3][4];
  uint64_t cnt = 0, sp = 0, sb = 0;
  const uint64_t stride = (uint64_t)gridDim.x * blockDim.x;
  for (uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; i < np; i += stride) {
    const uint32_t* r = prow + i * Wp;
    uint64_t k0;
    uint32_t k1;
    row_key(r + kwp, key_len, k0, k1);
    const uint64_t vp = *reinterpret_cast<const uint64_t*>(reinterpret_cast<const uint8_t*>(r) + col_p);
    uint64_t s = slot_of(key_hash(k0, k1, seed), mask);
    for (uint64_t probe = 0; probe <= mask; ++probe) {
      const HSlot x = table[s];
      if (x.idx == kEmpty) break;
      if (x.k0 == k0 && x.k1 == k1) {
        ++cnt;
        sp += vp;
        sb += *reinterpret_cast<const uint64_t*>(brow + (uint64_t)x.idx * stride_b + col_b);
      }
      s = (s + 1) & mask;
    }
  }
  cnt = wave_sum64(cnt);
  sp = wave_sum64(sp);
  sb = wave_sum64(sb);
  const int w = wave_id();
  if (lane_id() == 0) {
    red[0][w] = cnt;
    red[1][w] = sp;
    red[2][w] = sb;
  }
  __syncthreads();
  if (threadIdx.x < 3) {
    const int k = threadIdx.x;
    partial[(uint64_t)blockIdx.x * 3 + k] = red[k][0] + red[k][1] + red[k][2] + red[k][3];
  }
}

__global__ __launch_bounds__(256) void ht_sum_partials(const uint64_t* __restrict__ partial, uint32_t G,
                                                       unsigned long long* __restrict__ acc) {
  __shared__ uint64_t red[3][4];
  uint64_t v[3] = {0, 0, 0};
  for (uint32_t g = threadIdx.x; g < G; g += blockDim.x)
    for (int k = 0; k < 3; ++k) v[k] += partial[(uint64_t)g * 3 + k];
  for (int k = 0; k < 3; ++k) v[k] = wave_sum64(v[k]);
  if (lane_id() == 0)
    for (int k = 0; k < 3; ++k) red[k][wave_id()] = v[k];
  __syncthreads();
  if (threadIdx.x < 3) {
    const int k = threadIdx.x;
    acc[k] += red[k][0] + red[k][1] + red[k][2] + red[k][3];
  }
}

// Probe emitting pairs: EMIT = false counts matches per probe row, EMIT = true writes
// (probe row, build row) pairs at offs[i].
template <bool EMIT>
__global__ __launch_bounds__(256) void ht_probe_pairs_kernel(const uint32_t* __restrict__ prow, uint64_t np, uint32_t Wp,
                                                             uint32_t kwp, int key_len, uint64_t seed,
                                                             const HSlot* __restrict__ table, uint64_t mask,
                                                             int64_t* __restrict__ count, const int64_t* __restrict__ offs,
                                                             int64_t* __restrict__ po, int64_t* __restrict__ bo) {
  const uint64_t stride = (uint64_t)gridDim.x * blockDim.x;
  for (uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; i < np; i += stride) {
    uint64_t k0;
    uint32_t k1;
    row_key(prow + i * Wp + kwp, key_len, k0, k1);
    uint64_t s = slot_of(key_hash(k0, k1, seed), mask);
    int64_t c = 0;
    const int64_t o = EMIT ? offs[i] : 0;
    for (uint64_t probe = 0; probe <= mask; ++probe) {
      const HSlot x = table[s];
      if (x.idx == kEmpty) break;
      if (x.k0 == k0 && x.k1 == k1) {
        if (EMIT) {
          po[o + c] = (int64_t)i;
          bo[o + c] = (int64_t)x.idx;
        }
        ++c;
      }
      s = (s + 1) & mask;
    }
    if (!EMIT) count[i] = c;
  }
}

bool key_ok(uint32_t stride, uint32_t key_off, uint32_t key_len) {
  return stride > 0 && (stride & 3) == 0 && (key_off & 3) == 0 && key_len >= 1 && key_len <= 12 &&
         key_off + key_len <= stride;
}

}  // namespace

// Staged 16-byte projections: workgroup threads x pieces per thread (tile rows = product).  512 x 8
// (4096-row 64 KiB tiles, one workgroup per CU) vs 256 x 8 (2048 rows, three per CU): 2.29 vs 2.64 ms
// per 130M-row chunk of the 2 x 100 GB join, 1024 x 4 2.32 (profiles/r6/kernels/gp_shape_ab.txt).
#ifndef DR_GP_PROJ_NT
#define DR_GP_PROJ_NT 512
#endif
#ifndef DR_GP_PROJ_ITEMS
#define DR_GP_PROJ_ITEMS 8
#endif
constexpr int kGpProjNT = DR_GP_PROJ_NT;
constexpr int kGpProjItems = DR_GP_PROJ_ITEMS;

// Rows up to this many bytes are partitioned (wide rows: one per thread, kWideLdsDw dwords of LDS).
constexpr uint32_t kMaxStride = 512;
constexpr int kWideLdsDw = 256 * (kMaxStride / 4);

// Workspace (bytes) of dr_grace_partition for n rows of `stride` bytes into nb destinations.
DR_API uint64_t dr_grace_workspace(uint64_t n, uint32_t stride, uint32_t nb) {
  uint32_t G; uint64_t per_block;
  geometry(n, stride <= 64 ? 1024 : stride <= 128 ? 512 : 256, G, per_block);   // the most workgroups any tile gives
  return (uint64_t)nb * G * 4 + (uint64_t)nb * 8 * 2 + 256;
}

// Partition `n` rows (stride % 4 == 0, <= kMaxStride bytes) by dest = fastrange(32 bits of hash(key) at
// `shift`, nb) into per-destination runs at dst_ptr[d] (device array of nb row pointers).  The
// destination rows are bytes [proj_off, proj_off + out_stride) of the input rows (out_stride =
// stride, proj_off = 0: whole rows).
// Destinations d < contig_from append at their device fill counter fill[d] (advanced by this call;
// rows past cap[d] are dropped and *overflow set); destinations d >= contig_from are laid out back
// to back from row 0 of dst_ptr[d].  chunk_counts[d] / bases[d] receive this call's rows and first
// row per destination.
DR_API int dr_grace_partition(const uint8_t* rows, uint64_t n, uint32_t stride, uint32_t key_off, uint32_t key_len,
                              uint64_t seed, int shift, uint32_t nb, const uint64_t* dst_ptr, int64_t* fill,
                              const int64_t* cap, uint32_t contig_from, int64_t* chunk_counts, int64_t* bases,
                              uint32_t* overflow, void* ws, uint32_t out_stride, uint32_t proj_off, int unordered,
                              hipStream_t s) {
  if (!key_ok(stride, key_off, key_len) || stride > kMaxStride || nb < 1 || nb > kMaxBuckets || n >= (1ull << 32) ||
      (shift != 0 && shift != 32))
    return (int)hipErrorInvalidValue;
  if (out_stride == 0 || (out_stride & 3) || (proj_off & 3) || proj_off + out_stride > stride)
    return (int)hipErrorInvalidValue;
  if (n == 0) {
    hipMemsetAsync(chunk_counts, 0, sizeof(int64_t) * nb, s);
    return 0;
  }
  const bool small = stride <= 64, wide = stride > 128;
  const bool vec0 = (stride & 15) == 0 && (out_stride & 15) == 0 && (proj_off & 15) == 0 &&
                    (((uintptr_t)rows) & 15) == 0;
  // 16-byte projection holding the key: stage only the projected slice (4096-row tiles)
  const bool stage_proj = vec0 && out_stride == 16 && stride > 16 && key_off >= proj_off &&
                          key_off + key_len <= proj_off + out_stride;
  uint32_t G; uint64_t per_block;
  geometry(n, stage_proj ? kGpProjNT * kGpProjItems : (small ? 1024 : wide ? 256 : 512), G, per_block);
  uint32_t* counts = reinterpret_cast<uint32_t*>(ws);
  uint64_t* totals = reinterpret_cast<uint64_t*>(reinterpret_cast<uint8_t*>(ws) + (((uint64_t)nb * G * 4 + 15) & ~15ull));
  const uint32_t W = stride / 4, kw = key_off / 4;
  const uint32_t* in = reinterpret_cast<const uint32_t*>(rows);
  if (unordered && stage_proj && contig_from >= nb) {
    // every destination appends at its fill counter: no count pass, one reservation per tile
    gp_scatter_kernel<kGpProjItems, 0, 4, true, true, true, 16384, kGpProjNT><<<G, kGpProjNT, 0, s>>>(
                                                                    in, n, W, kw, (int)key_len, seed, shift, nb,
                                                                    nullptr, nullptr, dst_ptr, cap, contig_from, G,
                                                                    per_block, out_stride / 4, proj_off / 4, fill,
                                                                    overflow);
    DR_LAUNCH_CHECK();
    return 0;
  }
  gp_count_kernel<<<G, 256, 0, s>>>(in, n, W, kw, (int)key_len, seed, shift, nb, counts, G, per_block);
  gp_totals_kernel<<<nb, 256, 0, s>>>(counts, G, totals);
  gp_offsets_kernel<<<nb, 256, 0, s>>>(counts, G, totals, fill, cap, contig_from, bases, chunk_counts, overflow);
  const bool vec = vec0;
  const uint32_t OW = out_stride / 4, PO = proj_off / 4;
#define DR_GP_SCATTER(IT, WCV, OWCV, VECV)                                                               \
  gp_scatter_kernel<IT, WCV, OWCV, VECV><<<G, 256, 0, s>>>(in, n, W, kw, (int)key_len, seed, shift, nb, counts, \
                                                           bases, dst_ptr, cap, contig_from, G, per_block, OW, PO)
  if (stage_proj) {
    gp_scatter_kernel<kGpProjItems, 0, 4, true, true, false, 16384, kGpProjNT><<<G, kGpProjNT, 0, s>>>(
                                                             in, n, W, kw, (int)key_len, seed, shift, nb, counts,
                                                             bases, dst_ptr, cap, contig_from, G, per_block, OW, PO);
  } else if (wide) {
    if (vec)
      gp_scatter_kernel<1, 0, 0, true, false, false, kWideLdsDw><<<G, 256, 0, s>>>(
          in, n, W, kw, (int)key_len, seed, shift, nb, counts, bases, dst_ptr, cap, contig_from, G, per_block, OW, PO);
    else
      gp_scatter_kernel<1, 0, 0, false, false, false, kWideLdsDw><<<G, 256, 0, s>>>(
          in, n, W, kw, (int)key_len, seed, shift, nb, counts, bases, dst_ptr, cap, contig_from, G, per_block, OW, PO);
  } else if (small) {
    if (stride == 64 && out_stride == 64 && vec) DR_GP_SCATTER(4, 16, 16, true);
    else if (vec) DR_GP_SCATTER(4, 0, 0, true);
    else DR_GP_SCATTER(4, 0, 0, false);
  } else {
    if (vec) DR_GP_SCATTER(2, 0, 0, true);
    else DR_GP_SCATTER(2, 0, 0, false);
  }
#undef DR_GP_SCATTER
  DR_LAUNCH_CHECK();
  return 0;
}

// Build: table (2^log_cap 16-byte slots) must be memset to 0xFF; n <= 0.9 * 2^log_cap.
DR_API int dr_ht_build(const uint8_t* rows, uint64_t n, uint32_t stride, uint32_t key_off, uint32_t key_len,
                       uint64_t seed, void* table, int log_cap, hipStream_t s) {
  if (!key_ok(stride, key_off, key_len) || log_cap < 4 || log_cap > 34 || n >= (1ull << 32) ||
      n * 10 > (9ull << log_cap))
    return (int)hipErrorInvalidValue;
  if (n == 0) return 0;
  ht_build_kernel<<<grid_for(n, 256, 16384), 256, 0, s>>>(reinterpret_cast<const uint32_t*>(rows), n, stride / 4,
                                                          key_off / 4, (int)key_len, seed,
                                                          reinterpret_cast<HSlot*>(table), (1ull << log_cap) - 1);
  DR_LAUNCH_CHECK();
  return 0;
}

// Probe + fused aggregate (acc: 3 int64, accumulated): see ht_probe_sum_kernel.  ws holds
// kProbeGrid * 3 uint64 partials.
constexpr unsigned kProbeGrid = 2048;
DR_API uint64_t dr_ht_probe_sum_workspace() { return (uint64_t)kProbeGrid * 3 * 8; }

DR_API int dr_ht_probe_sum(const uint8_t* prow, uint64_t np, uint32_t stride_p, uint32_t key_off_p, uint32_t key_len,
                           uint64_t seed, const void* table, int log_cap, const uint8_t* brow, uint32_t stride_b,
                           uint32_t col_p, uint32_t col_b, int64_t* acc, void* ws, hipStream_t s) {
  if (!key_ok(stride_p, key_off_p, key_len) || log_cap < 4 || log_cap > 34 || (stride_p & 7) || (stride_b & 7) ||
      (col_p & 7) || (col_b & 7) || col_p + 8 > stride_p || col_b + 8 > stride_b)
    return (int)hipErrorInvalidValue;
  if (np == 0) return 0;
  const unsigned g = grid_for(np, 256, kProbeGrid);
  uint64_t* partial = reinterpret_cast<uint64_t*>(ws);
  ht_probe_sum_kernel<<<g, 256, 0, s>>>(reinterpret_cast<const uint32_t*>(prow), np, stride_p / 4, key_off_p / 4,
                                        (int)key_len, seed, reinterpret_cast<const HSlot*>(table),
                                        (1ull << log_cap) - 1, brow, stride_b, col_p, col_b, partial);
  ht_sum_partials<<<1, 256, 0, s>>>(partial, g, reinterpret_cast<unsigned long long*>(acc));
  DR_LAUNCH_CHECK();
  return 0;
}

// Probe emitting pairs: emit = 0 -> count[i] = matches of probe row i; emit = 1 -> pairs at offs[i].
DR_API int dr_ht_probe_pairs(const uint8_t* prow, uint64_t np, uint32_t stride_p, uint32_t key_off_p, uint32_t key_len,
                             uint64_t seed, const void* table, int log_cap, int64_t* count, const int64_t* offs,
                             int64_t* po, int64_t* bo, int emit, hipStream_t s) {
  if (!key_ok(stride_p, key_off_p, key_len) || log_cap < 4 || log_cap > 34) return (int)hipErrorInvalidValue;
  if (np == 0) return 0;
  const unsigned g = grid_for(np, 256, 16384);
  const uint32_t* p = reinterpret_cast<const uint32_t*>(prow);
  const HSlot* tb = reinterpret_cast<const HSlot*>(table);
  if (emit)
    ht_probe_pairs_kernel<true><<<g, 256, 0, s>>>(p, np, stride_p / 4, key_off_p / 4, (int)key_len, seed, tb,
                                                  (1ull << log_cap) - 1, count, offs, po, bo);
  else
    ht_probe_pairs_kernel<false><<<g, 256, 0, s>>>(p, np, stride_p / 4, key_off_p / 4, (int)key_len, seed, tb,
                                                   (1ull << log_cap) - 1, count, offs, po, bo);
  DR_LAUNCH_CHECK();
  return 0;
}

// ---------------------------------------------------------------------------------------------
// Radix join: the bucket pairs of the grace partitioning are split further, by two more digits
// of the same key hash, into partitions whose build side fits an LDS hash table; every
// partition pair is then joined by one workgroup entirely in LDS (no global atomics, no random
// HBM / Infinity-Cache reads).  This is the radix-partitioned hash join of the main-memory join
// literature mapped onto CDNA4: partition until the working set is on-chip, then build + probe
// on-chip.  Rows are fixed-width (RW dwords, 16 or 32 bytes) with an 8-byte-or-shorter key.
//
//   rp_count   per tile (a tile never crosses a segment): digit histogram in LDS
//   rp_scan    per segment: digit totals, digit starts, per-tile destination offsets
//   rp_scatter per tile: rows staged in LDS, ranked by digit with wave ballots (stable), every
//              digit's rows written as one contiguous run
//   rj_join_sum per partition pair: LDS open-addressing table over the build rows (64-bit CAS),
//              probe rows streamed through it with the Count/Sum aggregate fused in; partitions
//              too large for the LDS table (key skew) are listed for the global-table path.
namespace {

// 64 KiB tiles (4096 16-byte rows) in 1024-thread workgroups: ~94 KiB of LDS, one workgroup of 16
// waves per CU, 32 rows per digit run at 7-bit digits.  Join step 190.3 vs 201.5 ms against 32 KiB
// tiles at three 256-thread workgroups per CU (rp_scatter 13.8 vs 15.1 ms per pass, fewer tiles
// for rp_scan: profiles/r6/kernels/rp_shape_ab.txt); a 64 KiB tile in ONE 256-thread workgroup
// per CU ran at half the rate (round 3): the 16 waves keep loads in flight while others rank.
#ifndef DR_RP_TILE_BYTES
#define DR_RP_TILE_BYTES 65536
#endif
#ifndef DR_RP_NT
#define DR_RP_NT 1024
#endif
constexpr uint32_t kRpTileBytes = DR_RP_TILE_BYTES;
constexpr uint32_t kRaTileBytes = 32768;          // radix-aggregation pass A (ra_cols_*): 256-thread
                                                  // workgroups, the next tile's columns in registers
constexpr int kRpThreads = DR_RP_NT;              // rp_scatter workgroup
constexpr uint64_t kRjEmpty = 0xFFFFFFFFFFFFFFFFull;
constexpr uint32_t kRjCap = 2048;                 // LDS slots (16 B each: 32 KiB, 4 workgroups per CU)
constexpr int kRjPer = 6;                         // rows per thread held in registers (1536 >= 0.75 cap)

__device__ __forceinline__ uint32_t rp_seg_of(const int64_t* __restrict__ tile_base, uint32_t nseg, uint64_t t) {
  uint32_t lo = 0, hi = nseg;                      // last s with tile_base[s] <= t
  while (hi - lo > 1) {
    const uint32_t mid = (lo + hi) >> 1;
    if ((uint64_t)tile_base[mid] <= t) lo = mid; else hi = mid;
  }
  return lo;
}

template <int RW>
__device__ __forceinline__ uint32_t rp_digit(const uint32_t* r, int key_len, uint64_t seed, int shift, uint32_t dmask) {
  uint64_t k0;
  uint32_t k1;
  row_key(r, key_len, k0, k1);
  return (uint32_t)(key_hash(k0, k1, seed) >> shift) & dmask;
}

template <int RW>
__global__ __launch_bounds__(256) void rp_count_kernel(const uint32_t* __restrict__ rows,
                                                       const int64_t* __restrict__ seg_begin,
                                                       const int64_t* __restrict__ seg_len,
                                                       const int64_t* __restrict__ tile_base, uint32_t nseg,
                                                       uint64_t ntiles, uint32_t kw, int key_len, uint64_t seed,
                                                       int shift, int bits, uint32_t* __restrict__ counts) {
  constexpr uint32_t TILE = kRpTileBytes / (4 * RW);
  const uint32_t D = 1u << bits, dmask = D - 1;
  __shared__ uint32_t hist[4][256];
  const int t = threadIdx.x, w = wave_id();
  for (uint64_t tile = blockIdx.x; tile < ntiles; tile += gridDim.x) {
    for (int i = t; i < 4 * 256; i += kBlock) (&hist[0][0])[i] = 0;
    __syncthreads();
    const uint32_t s = rp_seg_of(tile_base, nseg, tile);
    const uint64_t r0 = (tile - (uint64_t)tile_base[s]) * TILE;
    const uint64_t left = (uint64_t)seg_len[s] - r0;
    const uint32_t cnt = left < TILE ? (uint32_t)left : TILE;
    const uint32_t* base = rows + ((uint64_t)seg_begin[s] + r0) * RW;
    // every key word of the thread's rows in flight before the first digit (clamped,
    // unconditional loads: one HBM round trip per tile instead of one per row)
    constexpr int PER = TILE / kBlock;
    uint32_t k0[PER], k1[PER], k2[PER];
    const uint32_t last = cnt ? cnt - 1 : 0;
#pragma unroll
    for (int r = 0; r < PER; ++r) {
      const uint32_t i = t + r * kBlock;
      const uint32_t* q = base + (uint64_t)(i < cnt ? i : last) * RW + kw;
      k0[r] = q[0];
      k1[r] = key_len > 4 ? q[1] : 0u;
      k2[r] = key_len > 8 ? q[2] : 0u;
    }
#pragma unroll
    for (int r = 0; r < PER; ++r) {
      if (t + r * kBlock < cnt) {
        const uint32_t kk[3] = {k0[r], k1[r], k2[r]};
        atomicAdd(&hist[w][rp_digit<RW>(kk, key_len, seed, shift, dmask)], 1u);
      }
    }
    __syncthreads();
    for (uint32_t d = t; d < D; d += kBlock) counts[tile * D + d] = hist[0][d] + hist[1][d] + hist[2][d] + hist[3][d];
    __syncthreads();
  }
}

// one workgroup per segment, thread = digit: totals, digit starts (part_start / part_len of the
// segment's D partitions) and each tile's absolute destination row per digit (in place)
__global__ __launch_bounds__(256) void rp_scan_kernel(const int64_t* __restrict__ seg_begin,
                                                      const int64_t* __restrict__ tile_base, int bits,
                                                      uint32_t* __restrict__ counts, int64_t* __restrict__ part_start,
                                                      int64_t* __restrict__ part_len) {
  __shared__ uint32_t sc[4];
  const uint32_t s = blockIdx.x, d = threadIdx.x, D = 1u << bits;
  const uint64_t t0 = (uint64_t)tile_base[s], t1 = (uint64_t)tile_base[s + 1];
  uint64_t tot = 0;
  if (d < D)
    for (uint64_t t = t0; t < t1; ++t) tot += counts[t * D + d];
  uint32_t all;
  const uint32_t ex = block_exclusive_scan256((uint32_t)tot, sc, all);
  if (d < D) {
    uint64_t run = (uint64_t)seg_begin[s] + ex;
    part_start[(uint64_t)s * D + d] = (int64_t)run;
    part_len[(uint64_t)s * D + d] = (int64_t)tot;
    for (uint64_t t = t0; t < t1; ++t) {
      const uint32_t c = counts[t * D + d];
      counts[t * D + d] = (uint32_t)run;          // rows < 2^32 (checked by the launcher)
      run += c;
    }
  }
}

template <int RW>
__global__ __launch_bounds__(kRpThreads) void rp_scatter_kernel(const uint32_t* __restrict__ rows, uint32_t* __restrict__ out,
                                                         const int64_t* __restrict__ seg_begin,
                                                         const int64_t* __restrict__ seg_len,
                                                         const int64_t* __restrict__ tile_base, uint32_t nseg,
                                                         uint64_t ntiles, uint32_t kw, int key_len, uint64_t seed,
                                                         int shift, int bits, const uint32_t* __restrict__ offsets) {
  constexpr int NT = kRpThreads, NW = NT / 64;
  constexpr uint32_t TILE = kRpTileBytes / (4 * RW);
  constexpr int ITEMS = TILE / NT;
  constexpr uint32_t C = RW / 4;                    // 16-byte pieces per row
  constexpr int PIECES = TILE * C / NT;             // staged 16-byte pieces per thread
  static_assert(PIECES >= 1 && PIECES <= 8 && NT >= 256, "tile shape");
  const uint32_t D = 1u << bits, dmask = D - 1;
  __shared__ __attribute__((aligned(16))) uint4 srow[TILE * C];
  __shared__ uint16_t perm[TILE];
  __shared__ uint8_t dslot[TILE];
  __shared__ uint32_t wcnt[NW][256];
  __shared__ uint32_t bstart[256];
  __shared__ uint32_t goff[256];
  __shared__ uint32_t sc[4];
  const int t = threadIdx.x, w = wave_id(), l = lane_id();
  auto locate = [&](uint64_t tile, uint32_t& cnt) -> const uint4* {
    const uint32_t s = rp_seg_of(tile_base, nseg, tile);
    const uint64_t r0 = (tile - (uint64_t)tile_base[s]) * TILE;
    const uint64_t left = (uint64_t)seg_len[s] - r0;
    cnt = left < TILE ? (uint32_t)left : TILE;
    return reinterpret_cast<const uint4*>(rows + ((uint64_t)seg_begin[s] + r0) * RW);
  };
  // the next tile's pieces live in named registers across the loop (an array here was placed in
  // scratch)
  uint4 p0, p1, p2, p3, p4, p5, p6, p7;
  const uint4* nsrc = nullptr;
  uint32_t ncnt = 0;
  auto issue = [&](const uint4* src, uint32_t pieces) {
    const uint32_t last = pieces ? pieces - 1 : 0;
#define DR_RP_LD(I, P) if (PIECES > (I)) { const uint32_t q = t + (I) * NT; P = src[q < pieces ? q : last]; }
    DR_RP_LD(0, p0) DR_RP_LD(1, p1) DR_RP_LD(2, p2) DR_RP_LD(3, p3)
    DR_RP_LD(4, p4) DR_RP_LD(5, p5) DR_RP_LD(6, p6) DR_RP_LD(7, p7)
#undef DR_RP_LD
  };
  if ((uint64_t)blockIdx.x < ntiles) {
    nsrc = locate(blockIdx.x, ncnt);
    issue(nsrc, ncnt * C);
  }
  for (uint64_t tile = blockIdx.x; tile < ntiles; tile += gridDim.x) {
    const uint32_t cnt = ncnt;
    {
      const uint32_t pieces = cnt * C;
#define DR_RP_ST(I, P) if (PIECES > (I)) { const uint32_t q = t + (I) * NT; if (q < pieces) srow[q] = P; }
      DR_RP_ST(0, p0) DR_RP_ST(1, p1) DR_RP_ST(2, p2) DR_RP_ST(3, p3)
      DR_RP_ST(4, p4) DR_RP_ST(5, p5) DR_RP_ST(6, p6) DR_RP_ST(7, p7)
#undef DR_RP_ST
    }
    if (tile + gridDim.x < ntiles) {               // the next tile's rows are in flight from here on
      nsrc = locate(tile + gridDim.x, ncnt);
      issue(nsrc, ncnt * C);
    }
    for (int i = t; i < NW * 256; i += NT) (&wcnt[0][0])[i] = 0;
    if ((uint32_t)t < D) goff[t] = offsets[tile * D + t];
    __syncthreads();
    uint32_t rk[ITEMS], dg[ITEMS];
#pragma unroll
    for (int r = 0; r < ITEMS; ++r) {
      const uint32_t pos = w * (TILE / NW) + r * 64 + l;
      const bool valid = pos < cnt;
      const uint32_t d = valid ? rp_digit<RW>(reinterpret_cast<const uint32_t*>(srow) + pos * RW + kw, key_len, seed,
                                              shift, dmask)
                               : 0u;
      uint64_t peers = ballot64(valid);
      for (int k = 0; k < bits; ++k) {
        const bool bit = (d >> k) & 1u;
        const uint64_t bb = ballot64(bit);
        peers &= bit ? bb : ~bb;
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
    uint32_t tot = 0;
    if (t < 256) {
#pragma unroll
      for (int k = 0; k < NW; ++k) {
        const uint32_t c = wcnt[k][t];
        wcnt[k][t] = tot;
        tot += c;
      }
    }
    {
      // exclusive scan of the 256 digit totals (waves 0..3; the other waves meet the barriers)
      const uint32_t inc = wave_inclusive_scan(tot);
      if (l == 63 && w < 4) sc[w] = inc;
      __syncthreads();
      const uint32_t b = (w > 0 ? sc[0] : 0) + (w > 1 ? sc[1] : 0) + (w > 2 ? sc[2] : 0);
      if (t < 256) bstart[t] = b + inc - tot;
      __syncthreads();
    }
#pragma unroll
    for (int r = 0; r < ITEMS; ++r) {
      const uint32_t pos = w * (TILE / NW) + r * 64 + l;
      if (pos < cnt) {
        const uint32_t slot = bstart[dg[r]] + wcnt[w][dg[r]] + rk[r];
        perm[slot] = (uint16_t)pos;
        dslot[slot] = (uint8_t)dg[r];
      }
    }
    __syncthreads();
    uint4* o4 = reinterpret_cast<uint4*>(out);
    for (uint32_t q = t; q < cnt * C; q += NT) {
      const uint32_t j = q / C, c = q - j * C;
      const uint32_t d = dslot[j];
      o4[((uint64_t)goff[d] + (j - bstart[d])) * C + c] = srow[(uint32_t)perm[j] * C + c];
    }
    __syncthreads();
  }
}

__device__ __forceinline__ uint32_t dword_of(const uint4& x, uint32_t i) {
  return i == 0 ? x.x : (i == 1 ? x.y : (i == 2 ? x.z : x.w));
}

// key (<= 8 bytes at dword kw) and the int64 at dword vw of a 16-byte row held in registers
__device__ __forceinline__ void row16(const uint4& x, uint32_t kw, int key_len, uint32_t vw, uint64_t& k0,
                                      uint64_t& v) {
  const uint32_t d0 = dword_of(x, kw) & keep_mask(key_len);
  const uint32_t d1 = key_len > 4 ? (dword_of(x, kw + 1) & keep_mask(key_len - 4)) : 0u;
  k0 = (uint64_t)d0 | ((uint64_t)d1 << 32);
  v = (uint64_t)dword_of(x, vw) | ((uint64_t)dword_of(x, vw + 1) << 32);
}

// one workgroup per partition pair (grid-stride): LDS table over the build rows, probe, fused
// Count / Sum(probe int64 at byte col_p) / Sum(build int64 at byte col_b) per match.  16-byte rows
// (key <= 8 bytes): a partition's build rows and its first probe rows are loaded into registers in
// one batch before the table is built, so the two HBM round trips overlap.
__global__ __launch_bounds__(256) void rj_join_sum_kernel(const uint4* __restrict__ brows,
                                                          const int64_t* __restrict__ bstart,
                                                          const int64_t* __restrict__ blen,
                                                          const uint4* __restrict__ prows,
                                                          const int64_t* __restrict__ pstart,
                                                          const int64_t* __restrict__ plen, uint64_t nparts,
                                                          uint32_t kw, int key_len, uint64_t seed, uint32_t col_b,
                                                          uint32_t col_p, uint32_t* __restrict__ ovf_count,
                                                          uint32_t* __restrict__ ovf_list, uint64_t* __restrict__ partial) {
  __shared__ unsigned long long keys[kRjCap];
  __shared__ uint64_t vals[kRjCap];
  __shared__ uint32_t bad;
  __shared__ uint64_t red[3][4];
  const int t = threadIdx.x;
  const uint32_t vb = col_b / 4, vp = col_p / 4;
  uint64_t cnt = 0, sp = 0, sb = 0;
  auto probe = [&](const uint4& x, uint64_t mask) {
    uint64_t k0, v;
    row16(x, kw, key_len, vp, k0, v);
    uint64_t sl = slot_of(key_hash(k0, 0u, seed), mask);
    for (;;) {
      const uint64_t k = keys[sl];
      if (k == kRjEmpty) break;
      if (k == k0) {
        ++cnt;
        sp += v;
        sb += vals[sl];
      }
      sl = (sl + 1) & mask;
    }
  };
  for (uint64_t p = blockIdx.x; p < nparts; p += gridDim.x) {
    const uint64_t nb = (uint64_t)blen[p], np = (uint64_t)plen[p];
    if (nb == 0 || np == 0) continue;
    if (nb * 4 > (uint64_t)kRjCap * 3) {           // load > 0.75: the global-table path joins it
      if (t == 0) ovf_list[atomicAdd(ovf_count, 1u)] = (uint32_t)p;
      continue;
    }
    const uint4* b0 = brows + bstart[p];
    const uint4* p0 = prows + pstart[p];
    uint4 bx[kRjPer], px[kRjPer];
#pragma unroll
    for (int k = 0; k < kRjPer; ++k) {             // clamped, unconditional: registers, no scratch
      const uint64_t i = t + (uint64_t)k * kBlock;
      bx[k] = b0[i < nb ? i : nb - 1];
      px[k] = p0[i < np ? i : np - 1];
    }
    uint32_t cap = 64;                             // load <= 0.5 below kRjCap, <= 0.75 at it
    while (cap < 2 * nb && cap < kRjCap) cap <<= 1;
    const uint64_t mask = cap - 1;
    for (uint32_t i = t; i < cap; i += kBlock) keys[i] = kRjEmpty;
    if (t == 0) bad = 0;
    __syncthreads();
#pragma unroll
    for (int k = 0; k < kRjPer; ++k) {
      if (t + (uint64_t)k * kBlock >= nb) continue;
      uint64_t k0, v;
      row16(bx[k], kw, key_len, vb, k0, v);
      if (k0 == kRjEmpty) {
        bad = 1;
        continue;
      }
      uint64_t sl = slot_of(key_hash(k0, 0u, seed), mask);
      while (atomicCAS(&keys[sl], kRjEmpty, (unsigned long long)k0) != kRjEmpty) sl = (sl + 1) & mask;
      vals[sl] = v;
    }
    __syncthreads();
    if (bad) {                                     // the empty-slot sentinel is a real key here
      if (t == 0) ovf_list[atomicAdd(ovf_count, 1u)] = (uint32_t)p;
      __syncthreads();
      continue;
    }
#pragma unroll
    for (int k = 0; k < kRjPer; ++k)
      if (t + (uint64_t)k * kBlock < np) probe(px[k], mask);
    for (uint64_t j = t + (uint64_t)kRjPer * kBlock; j < np; j += kBlock) probe(p0[j], mask);
    __syncthreads();
  }
  cnt = wave_sum64(cnt);
  sp = wave_sum64(sp);
  sb = wave_sum64(sb);
  const int w = wave_id();
  if (lane_id() == 0) {
    red[0][w] = cnt;
    red[1][w] = sp;
    red[2][w] = sb;
  }
  __syncthreads();
  if (t < 3) partial[(uint64_t)blockIdx.x * 3 + t] = red[t][0] + red[t][1] + red[t][2] + red[t][3];
}

constexpr unsigned kRpGrid = 2048;
constexpr unsigned kRjGrid = 4096;

}  // namespace

// One stable radix-partition pass over segments of fixed-width rows (row_bytes 16 or 32, key <= 8
// bytes at a 4-aligned offset): segment s = rows [seg_begin[s], seg_begin[s] + seg_len[s]) of
// `rows` is split by digit d = (hash(key) >> shift) & (2^bits - 1) into `out` at the same
// segment position, digit-major; part_start / part_len (nseg * 2^bits) receive every new
// partition.  tile_base (nseg + 1, device) = exclusive scan of the segments' tile counts
// (dr_radix_tile_rows rows per tile); counts = ntiles * 2^bits uint32 of scratch.
DR_API uint32_t dr_radix_tile_rows(uint32_t row_bytes) { return kRpTileBytes / row_bytes; }

DR_API int dr_radix_partition(const uint8_t* rows, uint8_t* out, uint32_t row_bytes, uint32_t key_off, uint32_t key_len,
                              uint64_t seed, int shift, int bits, const int64_t* seg_begin, const int64_t* seg_len,
                              const int64_t* tile_base, uint32_t nseg, uint64_t ntiles, uint64_t total_rows,
                              uint32_t* counts, int64_t* part_start, int64_t* part_len, hipStream_t s) {
  if ((row_bytes != 16 && row_bytes != 32) || !key_ok(row_bytes, key_off, key_len) || key_len > 8 || bits < 1 ||
      bits > 8 || shift < 0 || shift + bits > 64 || total_rows >= (1ull << 32) || nseg == 0)
    return (int)hipErrorInvalidValue;
  if (ntiles == 0) {
    hipMemsetAsync(part_len, 0, sizeof(int64_t) * ((uint64_t)nseg << bits), s);
    rp_scan_kernel<<<nseg, 256, 0, s>>>(seg_begin, tile_base, bits, counts, part_start, part_len);
    return 0;
  }
  const uint32_t* in = reinterpret_cast<const uint32_t*>(rows);
  uint32_t* o = reinterpret_cast<uint32_t*>(out);
  const unsigned g = (unsigned)(ntiles < kRpGrid ? ntiles : kRpGrid);
  const uint32_t kw = key_off / 4;
  if (row_bytes == 16) {
    rp_count_kernel<4><<<g, 256, 0, s>>>(in, seg_begin, seg_len, tile_base, nseg, ntiles, kw, (int)key_len, seed,
                                         shift, bits, counts);
    rp_scan_kernel<<<nseg, 256, 0, s>>>(seg_begin, tile_base, bits, counts, part_start, part_len);
    rp_scatter_kernel<4><<<g, kRpThreads, 0, s>>>(in, o, seg_begin, seg_len, tile_base, nseg, ntiles, kw, (int)key_len, seed,
                                           shift, bits, counts);
  } else {
    rp_count_kernel<8><<<g, 256, 0, s>>>(in, seg_begin, seg_len, tile_base, nseg, ntiles, kw, (int)key_len, seed,
                                         shift, bits, counts);
    rp_scan_kernel<<<nseg, 256, 0, s>>>(seg_begin, tile_base, bits, counts, part_start, part_len);
    rp_scatter_kernel<8><<<g, kRpThreads, 0, s>>>(in, o, seg_begin, seg_len, tile_base, nseg, ntiles, kw, (int)key_len, seed,
                                           shift, bits, counts);
  }
  DR_LAUNCH_CHECK();
  return 0;
}

// Join of aligned partition pairs (build / probe partitions p from the same radix passes) in LDS;
// acc (3 int64) += (matches, sum of probe int64 at col_p per match, sum of build int64 at col_b
// per match).  Partitions the LDS table cannot take are appended to ovf_list (ovf_count, device)
// for the caller's global-table path.  ws = dr_radix_join_workspace() bytes.
DR_API uint64_t dr_radix_join_workspace() { return (uint64_t)kRjGrid * 3 * 8; }

DR_API int dr_radix_join_sum(const uint8_t* brows, const int64_t* bstart, const int64_t* blen, const uint8_t* prows,
                             const int64_t* pstart, const int64_t* plen, uint64_t nparts, uint32_t row_bytes,
                             uint32_t key_off, uint32_t key_len, uint64_t seed, uint32_t col_b, uint32_t col_p,
                             uint32_t* ovf_count, uint32_t* ovf_list, int64_t* acc, void* ws, hipStream_t s) {
  if (row_bytes != 16 || !key_ok(row_bytes, key_off, key_len) || key_len > 8 || (col_b & 7) || (col_p & 7) ||
      col_b + 8 > row_bytes || col_p + 8 > row_bytes || (((uintptr_t)brows | (uintptr_t)prows) & 15))
    return (int)hipErrorInvalidValue;
  if (nparts == 0) return 0;
  const unsigned g = (unsigned)(nparts < kRjGrid ? nparts : kRjGrid);
  uint64_t* partial = reinterpret_cast<uint64_t*>(ws);
  rj_join_sum_kernel<<<g, 256, 0, s>>>(reinterpret_cast<const uint4*>(brows), bstart, blen,
                                       reinterpret_cast<const uint4*>(prows), pstart, plen, nparts, key_off / 4,
                                       (int)key_len, seed, col_b, col_p, ovf_count, ovf_list, partial);
  ht_sum_partials<<<1, 256, 0, s>>>(partial, g, reinterpret_cast<unsigned long long*>(acc));
  DR_LAUNCH_CHECK();
  return 0;
}

// ---------------------------------------------------------------------------------------------
// Radix aggregation: high-cardinality GroupBy on one 8-byte key (K6; the reference's partial +
// final hash GroupBy vertices, DryadLinqVertex.cs:437-585, with the partitioning of
// DryadLinqQueryGen.cs:1638-1700).  The same plan as the radix join: split the rows by digits of
// the key hash until a partition's distinct keys fit an LDS table, then fold every partition on
// chip.  Per GroupBy:
//
//   ra_cols_count / ra_cols_scatter  pass A over the key and value COLUMNS: every row is packed
//              into a 16- or 32-byte row (key, up to three 8-byte values) while it is split by the
//              first digit, so packing costs no pass of its own
//   dr_radix_partition               passes B, C, ... (the join's segmented passes) on the rows
//   ra_agg     one workgroup per partition: LDS open-addressing table (64-bit CAS on the key,
//              ds atomics on a count and up to three accumulators), then the groups are written
//              to the shared output through chunk reservations (one global atomic per 16K groups;
//              a partition may straddle two chunks).  Only the last chunk of each workgroup can
//              end partly empty; the caller closes those holes by moving the tail groups in.
//              Partitions whose table fills (or that hold the empty-slot key) are listed for the
//              caller's fallback.  Group order is unspecified, as for the LDS hash-agg path.
namespace {

constexpr int kRaAcc = 3;
constexpr uint32_t kRaCap = 1024;          // 8 KB keys + 4 KB counts + 24 KB accumulators: 4 workgroups per CU
constexpr uint32_t kRaChunk = 16384;       // output groups per reservation
constexpr unsigned kRaGrid = 2048;         // 4 workgroups per CU (36 KB of LDS each)
constexpr unsigned long long kRaEmpty = 0x8000000000000000ull;
enum RaOp : int { RA_SUM_I = 0, RA_MIN_I = 1, RA_MAX_I = 2, RA_SUM_F = 4, RA_MIN_F = 5, RA_MAX_F = 6 };

struct RaCols {
  const uint64_t* key;
  const uint64_t* val[kRaAcc];
  int nval;
};

struct RaSpec {
  int nacc;
  int op[kRaAcc];
  int word[kRaAcc];        // 8-byte word of the packed row that holds the folded value (1..3)
};

struct RaOut {
  int64_t* key;
  int64_t* cnt;
  uint64_t* acc[kRaAcc];
};

__device__ __forceinline__ unsigned long long ra_identity(int op) {
  switch (op) {
    case RA_MIN_I: return 0x7FFFFFFFFFFFFFFFull;
    case RA_MAX_I: return 0x8000000000000000ull;
    case RA_MIN_F: return (unsigned long long)__double_as_longlong(__builtin_inf());
    case RA_MAX_F: return (unsigned long long)__double_as_longlong(-__builtin_inf());
    default: return 0ull;
  }
}

__device__ __noinline__ void ra_fminmax(unsigned long long* p, double v, bool is_min) {
  unsigned long long old = *p, assumed;
  do {
    assumed = old;
    const double cur = __longlong_as_double((long long)assumed);
    if (is_min ? !(v < cur) : !(v > cur)) break;
    old = atomicCAS(p, assumed, (unsigned long long)__double_as_longlong(v));
  } while (assumed != old);
}

__device__ __forceinline__ void ra_fold(unsigned long long* p, uint64_t v, int op) {
  switch (op) {
    case RA_SUM_I: atomicAdd(p, (unsigned long long)v); break;
    case RA_MIN_I: atomicMin(reinterpret_cast<long long*>(p), (long long)v); break;
    case RA_MAX_I: atomicMax(reinterpret_cast<long long*>(p), (long long)v); break;
    case RA_SUM_F: atomicAdd(reinterpret_cast<double*>(p), __longlong_as_double((long long)v)); break;
    case RA_MIN_F: ra_fminmax(p, __longlong_as_double((long long)v), true); break;
    default: ra_fminmax(p, __longlong_as_double((long long)v), false); break;
  }
}

// pass A histogram: the digit of every key of a tile (tiles of the packed row width)
template <int RW>
__global__ __launch_bounds__(256) void ra_cols_count_kernel(const uint64_t* __restrict__ key, uint64_t n,
                                                            uint64_t ntiles, uint64_t seed, int shift, int bits,
                                                            uint32_t* __restrict__ counts) {
  constexpr uint32_t TILE = kRaTileBytes / (4 * RW);
  const uint32_t D = 1u << bits, dmask = D - 1;
  __shared__ uint32_t hist[4][256];
  const int t = threadIdx.x, w = wave_id();
  const uint64_t hs = mix64(seed);               // key_hash(k, 0, seed) of the row passes
  // one histogram per workgroup over its contiguous tile range (ra_cols_scatter walks the same
  // range in order), so the digit scan runs over gridDim.x entries instead of every tile
  const uint64_t per = (ntiles + gridDim.x - 1) / gridDim.x;
  const uint64_t t0 = blockIdx.x * per, t1 = t0 + per < ntiles ? t0 + per : ntiles;
  for (int i = t; i < 4 * 256; i += kBlock) (&hist[0][0])[i] = 0;
  __syncthreads();
  const uint64_t r_end = t1 * TILE < n ? t1 * TILE : n;
  for (uint64_t i = t0 * TILE + t; i < r_end; i += kBlock)
    atomicAdd(&hist[w][(uint32_t)(mix64(key[i] ^ hs) >> shift) & dmask], 1u);
  __syncthreads();
  for (uint32_t d = t; d < D; d += kBlock)
    counts[(uint64_t)blockIdx.x * D + d] = hist[0][d] + hist[1][d] + hist[2][d] + hist[3][d];
}

// pass A scatter: a tile's key / value columns are loaded (the next tile's while this one is
// ranked and written), packed into LDS rows, ranked by digit with wave ballots (stable) and
// written digit-major at the offsets of rp_scan
template <int RW>
__global__ __launch_bounds__(256) void ra_cols_scatter_kernel(RaCols in, uint64_t n, uint64_t ntiles, uint64_t seed,
                                                              int shift, int bits, const uint32_t* __restrict__ offsets,
                                                              uint32_t* __restrict__ out) {
  constexpr uint32_t TILE = kRaTileBytes / (4 * RW);
  constexpr int ITEMS = TILE / kBlock;
  constexpr uint32_t C = RW / 4;
  const uint32_t D = 1u << bits, dmask = D - 1;
  __shared__ __attribute__((aligned(16))) uint4 srow[TILE * C];
  __shared__ uint16_t perm[TILE];
  __shared__ uint8_t dslot[TILE];
  __shared__ uint32_t wcnt[4][256];
  __shared__ uint32_t bstart[256];
  __shared__ uint32_t goff[256];
  __shared__ uint32_t sc[4];
  const int t = threadIdx.x, w = wave_id(), l = lane_id();
  const uint64_t hs = mix64(seed);
  uint64_t kr[ITEMS], v0[ITEMS], v1[ITEMS], v2[ITEMS];
#define DR_RA_ISSUE(TL)                                                                   \
  {                                                                                       \
    const uint64_t r0_ = (TL) * TILE;                                                     \
    _Pragma("unroll") for (int r = 0; r < ITEMS; ++r) {                                   \
      uint64_t i_ = r0_ + w * (TILE / 4) + r * 64 + l;                                    \
      i_ = i_ < n ? i_ : n - 1;                   /* clamped, unconditional */            \
      kr[r] = in.key[i_];                                                                 \
      v0[r] = in.nval > 0 ? in.val[0][i_] : 0ull;                                         \
      v1[r] = (RW == 8 && in.nval > 1) ? in.val[1][i_] : 0ull;                            \
      v2[r] = (RW == 8 && in.nval > 2) ? in.val[2][i_] : 0ull;                            \
    }                                                                                     \
  }
  const uint64_t per = (ntiles + gridDim.x - 1) / gridDim.x;
  const uint64_t t0 = blockIdx.x * per, t1 = t0 + per < ntiles ? t0 + per : ntiles;
  if ((uint32_t)t < D) goff[t] = offsets[(uint64_t)blockIdx.x * D + t];   // advanced tile by tile
  if (t0 < t1) DR_RA_ISSUE(t0)
  for (uint64_t tile = t0; tile < t1; ++tile) {
    const uint64_t r0 = tile * TILE;
    const uint32_t cnt = n - r0 < TILE ? (uint32_t)(n - r0) : TILE;
    uint32_t dg[ITEMS];
#pragma unroll
    for (int r = 0; r < ITEMS; ++r) {
      const uint32_t pos = w * (TILE / 4) + r * 64 + l;
      dg[r] = (uint32_t)(mix64(kr[r] ^ hs) >> shift) & dmask;
      if (pos < cnt) {
        srow[pos * C] = make_uint4((uint32_t)kr[r], (uint32_t)(kr[r] >> 32), (uint32_t)v0[r], (uint32_t)(v0[r] >> 32));
        if constexpr (C == 2)
          srow[pos * C + 1] = make_uint4((uint32_t)v1[r], (uint32_t)(v1[r] >> 32), (uint32_t)v2[r], (uint32_t)(v2[r] >> 32));
      }
    }
    if (tile + 1 < t1) DR_RA_ISSUE(tile + 1)
    wcnt[0][t] = 0; wcnt[1][t] = 0; wcnt[2][t] = 0; wcnt[3][t] = 0;
    __syncthreads();
    uint32_t rk[ITEMS];
#pragma unroll
    for (int r = 0; r < ITEMS; ++r) {
      const uint32_t pos = w * (TILE / 4) + r * 64 + l;
      const bool valid = pos < cnt;
      const uint32_t d = valid ? dg[r] : 0u;
      uint64_t peers = ballot64(valid);
      for (int k = 0; k < bits; ++k) {
        const bool bit = (d >> k) & 1u;
        const uint64_t bb = ballot64(bit);
        peers &= bit ? bb : ~bb;
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
    const uint32_t mine = c0 + c1 + c2 + c3;
    wcnt[0][t] = 0; wcnt[1][t] = c0; wcnt[2][t] = c0 + c1; wcnt[3][t] = c0 + c1 + c2;
    uint32_t all;
    bstart[t] = block_exclusive_scan256(mine, sc, all);
    __syncthreads();
#pragma unroll
    for (int r = 0; r < ITEMS; ++r) {
      const uint32_t pos = w * (TILE / 4) + r * 64 + l;
      if (pos < cnt) {
        const uint32_t slot = bstart[dg[r]] + wcnt[w][dg[r]] + rk[r];
        perm[slot] = (uint16_t)pos;
        dslot[slot] = (uint8_t)dg[r];
      }
    }
    __syncthreads();
    uint4* o4 = reinterpret_cast<uint4*>(out);
    for (uint32_t q = t; q < cnt * C; q += kBlock) {
      const uint32_t j = q / C, c = q - j * C;
      const uint32_t d = dslot[j];
      o4[((uint64_t)goff[d] + (j - bstart[d])) * C + c] = srow[(uint32_t)perm[j] * C + c];
    }
    __syncthreads();
    if ((uint32_t)t < D) goff[t] += mine;
  }
#undef DR_RA_ISSUE
}

__device__ __forceinline__ uint64_t ra_word(const uint4& a, const uint4& b, int wi) {
  switch (wi) {
    case 1: return (uint64_t)a.z | ((uint64_t)a.w << 32);
    case 2: return (uint64_t)b.x | ((uint64_t)b.y << 32);
    default: return (uint64_t)b.z | ((uint64_t)b.w << 32);
  }
}

// one workgroup per partition (grid-stride).  The table is sized to the partition (3 slots per
// row, multiple of 64, <= kRaCap; slot = fast range of a second hash), so a small partition clears
// and scans only its own slots.  A partition's first kRaPer * 256 rows are in registers before its
// table is built: they were loaded while the previous partition's groups were written out.
constexpr int kRaPer = 3;
#ifndef RA_SLOTS_PER_ROW
#define RA_SLOTS_PER_ROW 3          // table load <= 1/3 (all-distinct keys): ~1.2 probes per insert
#endif

template <int RW>
__global__ __launch_bounds__(256, 4) void ra_agg_kernel(const uint4* __restrict__ rows, const int64_t* __restrict__ pstart,
                                                        const int64_t* __restrict__ plen, uint64_t nparts,
                                                        uint64_t seed, RaSpec sp, RaOut o, uint64_t out_cap,
                                                        unsigned long long* __restrict__ head,
                                                        uint32_t* __restrict__ ovf_count, uint32_t* __restrict__ ovf_list,
                                                        unsigned long long* __restrict__ tails) {
  constexpr uint32_t C = RW / 4;
  __shared__ unsigned long long keys[kRaCap];
  __shared__ uint32_t cnts[kRaCap];
  __shared__ unsigned long long acc[kRaAcc][kRaCap];
  __shared__ uint32_t used, bad, lidx;
  __shared__ unsigned long long ccur, cend, s_first, s_second, s_rem;
  const int t = threadIdx.x, l = lane_id();
  const uint64_t hs = mix64(seed);
  if (t == 0) {
    ccur = 0;
    cend = 0;
  }
  uint4 ra[kRaPer], rb[kRaPer];
  // a macro, not a lambda: arrays captured by a lambda were placed in scratch
#define DR_RA_BATCH(P)                                                                    \
  {                                                                                       \
    const uint64_t len_ = (uint64_t)plen[P];                                              \
    /* an empty partition (a trailing one starts at n) reads row 0, never past the end */ \
    const uint4* base_ = len_ ? rows + (uint64_t)pstart[P] * C : rows;                    \
    const uint64_t last_ = len_ ? len_ - 1 : 0;                                           \
    _Pragma("unroll") for (int k = 0; k < kRaPer; ++k) { /* clamped, unconditional */     \
      uint64_t r_ = t + (uint64_t)k * kBlock;                                             \
      r_ = r_ < len_ ? r_ : last_;                                                        \
      ra[k] = base_[r_ * C];                                                              \
      rb[k] = C == 2 ? base_[r_ * C + 1] : make_uint4(0u, 0u, 0u, 0u);                    \
    }                                                                                     \
  }
  auto insert = [&](uint4 a, uint4 b, uint32_t cap) {
    const unsigned long long k = (unsigned long long)a.x | ((unsigned long long)a.y << 32);
    if (k == kRaEmpty) {
      bad = 1;
      return;
    }
    uint32_t sl = (uint32_t)((mix64(mix64(k ^ hs) ^ kSlotMix) >> 32) * (uint64_t)cap >> 32);
    bool ok = false;
    for (uint32_t probes = 0; probes < cap; ++probes) {
      const unsigned long long cur = keys[sl];
      if (cur == k) {
        ok = true;
        break;
      }
      if (cur == kRaEmpty) {
        const unsigned long long prev = atomicCAS(&keys[sl], kRaEmpty, k);
        if (prev == kRaEmpty) atomicAdd(&used, 1u);
        if (prev == kRaEmpty || prev == k) {
          ok = true;
          break;
        }
      }
      sl = sl + 1 == cap ? 0 : sl + 1;
    }
    if (!ok) {                                      // table full
      bad = 1;
      return;
    }
    atomicAdd(&cnts[sl], 1u);
#pragma unroll
    for (int j = 0; j < kRaAcc; ++j)
      if (j < sp.nacc) ra_fold(&acc[j][sl], ra_word(a, b, sp.word[j]), sp.op[j]);
  };
  if ((uint64_t)blockIdx.x < nparts) DR_RA_BATCH(blockIdx.x)
  for (uint64_t p = blockIdx.x; p < nparts; p += gridDim.x) {
    const uint64_t len = (uint64_t)plen[p];
    const uint4* base = rows + (uint64_t)pstart[p] * C;
    const uint64_t nxt = p + gridDim.x;
    if (len == 0) {
      if (nxt < nparts) DR_RA_BATCH(nxt)
      continue;
    }
    uint64_t c64 = ((RA_SLOTS_PER_ROW * len + 63) / 64) * 64;
    const uint32_t cap = c64 < kRaCap ? (uint32_t)c64 : kRaCap;
    for (uint32_t i = t; i < cap; i += kBlock) {
      keys[i] = kRaEmpty;
      cnts[i] = 0;
#pragma unroll
      for (int j = 0; j < kRaAcc; ++j)
        if (j < sp.nacc) acc[j][i] = ra_identity(sp.op[j]);
    }
    if (t == 0) {
      used = 0;
      bad = 0;
      lidx = 0;
    }
    __syncthreads();
    // unrolled: the batch's probe chains overlap (a rolled loop over a rotating register window
    // was 1.6x slower)
#pragma unroll
    for (int k = 0; k < kRaPer; ++k)
      if (t + (uint64_t)k * kBlock < len) insert(ra[k], rb[k], cap);
    for (uint64_t r = t + (uint64_t)kRaPer * kBlock; r < len; r += kBlock) {
      const uint4 a = base[r * C];
      uint4 b = make_uint4(0u, 0u, 0u, 0u);
      if constexpr (C == 2) b = base[r * C + 1];
      insert(a, b, cap);
    }
    __syncthreads();
    if (nxt < nparts) DR_RA_BATCH(nxt)             // the next partition's rows arrive meanwhile
    if (bad) {
      if (t == 0) ovf_list[atomicAdd(ovf_count, 1u)] = (uint32_t)p;
      __syncthreads();
      continue;
    }
    if (t == 0) {                                   // output space: rest of the chunk + a new one
      const unsigned long long ng = used, c = ccur, rem = cend - ccur;
      s_first = c;
      s_rem = rem;
      if (rem >= ng) {
        ccur = c + ng;
        s_second = 0;
      } else {
        const unsigned long long nb = atomicAdd(head, (unsigned long long)kRaChunk);
        s_second = nb;
        ccur = nb + (ng - rem);
        cend = nb + kRaChunk;
      }
    }
    __syncthreads();
    const unsigned long long first = s_first, second = s_second, rem = s_rem;
    for (uint32_t b0 = 0; b0 < cap; b0 += kBlock) {
      const uint32_t i = b0 + t;
      const unsigned long long k = i < cap ? keys[i] : kRaEmpty;
      const bool occ = k != kRaEmpty;
      const uint64_t m = ballot64(occ);
      uint32_t wb = 0;
      if (l == 0 && m) wb = atomicAdd(&lidx, (uint32_t)__popcll(m));
      wb = __shfl(wb, 0, 64);
      if (occ) {
        const unsigned long long li = wb + popc_below(m);
        const unsigned long long pos = li < rem ? first + li : second + (li - rem);
        if (pos < out_cap) {
          o.key[pos] = (int64_t)k;
          o.cnt[pos] = (int64_t)cnts[i];
#pragma unroll
          for (int j = 0; j < kRaAcc; ++j)
            if (j < sp.nacc) o.acc[j][pos] = acc[j][i];
        }
      }
    }
    __syncthreads();
  }
  if (t == 0) {
    tails[2 * (uint64_t)blockIdx.x] = ccur;
    tails[2 * (uint64_t)blockIdx.x + 1] = cend;
  }
#undef DR_RA_BATCH
}

}  // namespace

// Pass A of the radix aggregation: key column (int64) + nval <= 3 value columns (8-byte words)
// -> rows of row_bytes (16: key + 1 value, 32: key + 3 values; missing values zero) split by
// digit (hash(key) >> shift) & (2^bits - 1) into `out`; part_start / part_len (2^bits) receive the
// partitions.  counts: dr_radix_agg_pack_grid(n, row_bytes) * 2^bits uint32 of scratch;
// seg_tile (3 int64, device) = {0, 0, that grid}: rp_scan's segment begin and "tile" bases of the
// one input segment.
DR_API int dr_radix_agg_pack(const int64_t* key, const void* const* vals, int nval, uint64_t n, uint32_t row_bytes,
                             uint64_t seed, int shift, int bits, const int64_t* seg_tile, uint32_t* counts,
                             int64_t* part_start, int64_t* part_len, uint8_t* out, hipStream_t s) {
  if ((row_bytes != 16 && row_bytes != 32) || nval < 0 || nval > (row_bytes == 16 ? 1 : 3) || bits < 1 || bits > 8 ||
      shift < 0 || shift + bits > 64 || n == 0 || n >= (1ull << 32))
    return (int)hipErrorInvalidValue;
  RaCols in{};
  in.key = reinterpret_cast<const uint64_t*>(key);
  for (int j = 0; j < nval; ++j) in.val[j] = reinterpret_cast<const uint64_t*>(vals[j]);
  in.nval = nval;
  const uint32_t tile = kRaTileBytes / row_bytes;
  const uint64_t ntiles = (n + tile - 1) / tile;
  const unsigned g = (unsigned)(ntiles < kRpGrid ? ntiles : kRpGrid);
  // counts / offsets per workgroup (its contiguous tile range), so rp_scan's "tiles" are the g
  // workgroups: seg_tile = {seg_begin = 0, 0, g}
  if (row_bytes == 16) {
    ra_cols_count_kernel<4><<<g, 256, 0, s>>>(in.key, n, ntiles, seed, shift, bits, counts);
    rp_scan_kernel<<<1, 256, 0, s>>>(seg_tile, seg_tile + 1, bits, counts, part_start, part_len);
    ra_cols_scatter_kernel<4><<<g, 256, 0, s>>>(in, n, ntiles, seed, shift, bits, counts,
                                                reinterpret_cast<uint32_t*>(out));
  } else {
    ra_cols_count_kernel<8><<<g, 256, 0, s>>>(in.key, n, ntiles, seed, shift, bits, counts);
    rp_scan_kernel<<<1, 256, 0, s>>>(seg_tile, seg_tile + 1, bits, counts, part_start, part_len);
    ra_cols_scatter_kernel<8><<<g, 256, 0, s>>>(in, n, ntiles, seed, shift, bits, counts,
                                                reinterpret_cast<uint32_t*>(out));
  }
  DR_LAUNCH_CHECK();
  return 0;
}

DR_API uint32_t dr_radix_agg_pack_grid(uint64_t n, uint32_t row_bytes) {
  const uint64_t ntiles = (n + kRaTileBytes / row_bytes - 1) / (kRaTileBytes / row_bytes);
  return (uint32_t)(ntiles < kRpGrid ? (ntiles ? ntiles : 1) : kRpGrid);
}

DR_API uint32_t dr_radix_agg_grid(uint64_t nparts) { return (uint32_t)(nparts < kRaGrid ? (nparts ? nparts : 1) : kRaGrid); }
DR_API uint32_t dr_radix_agg_chunk() { return kRaChunk; }

// Fold of the final partitions: ops[j] (RaOp) of the 8-byte word words[j] (1..3) of each row,
// nacc <= 3, plus a count per group.  Groups go to okey / ocnt / oacc[j] at positions reserved
// from *head (zeroed by the caller) in chunks of dr_radix_agg_chunk(); tails (2 per workgroup of
// dr_radix_agg_grid(nparts)) receive each workgroup's unused chunk end [cur, end).  out_cap must
// be >= n + (grid + 1) * chunk.  Partitions the LDS table cannot hold go to ovf_list.
DR_API int dr_radix_agg(const uint8_t* rows, uint32_t row_bytes, const int64_t* pstart, const int64_t* plen,
                        uint64_t nparts, uint64_t seed, int nacc, const int* ops, const int* words,
                        unsigned long long* head, uint64_t out_cap, int64_t* okey, int64_t* ocnt, void* const* oacc,
                        uint32_t* ovf_count, uint32_t* ovf_list, unsigned long long* tails, hipStream_t s) {
  if ((row_bytes != 16 && row_bytes != 32) || nacc < 0 || nacc > kRaAcc || ((uintptr_t)rows & 15))
    return (int)hipErrorInvalidValue;
  RaSpec sp{};
  RaOut o{};
  sp.nacc = nacc;
  for (int j = 0; j < nacc; ++j) {
    if (words[j] < 1 || words[j] > (row_bytes == 16 ? 1 : 3) ||
        !(ops[j] == RA_SUM_I || ops[j] == RA_MIN_I || ops[j] == RA_MAX_I || ops[j] == RA_SUM_F ||
          ops[j] == RA_MIN_F || ops[j] == RA_MAX_F))
      return (int)hipErrorInvalidValue;
    sp.op[j] = ops[j];
    sp.word[j] = words[j];
    o.acc[j] = reinterpret_cast<uint64_t*>(oacc[j]);
  }
  o.key = okey;
  o.cnt = ocnt;
  if (nparts == 0) return 0;
  const unsigned g = dr_radix_agg_grid(nparts);
  const uint4* r4 = reinterpret_cast<const uint4*>(rows);
  if (row_bytes == 16)
    ra_agg_kernel<4><<<g, 256, 0, s>>>(r4, pstart, plen, nparts, seed, sp, o, out_cap, head, ovf_count, ovf_list, tails);
  else
    ra_agg_kernel<8><<<g, 256, 0, s>>>(r4, pstart, plen, nparts, seed, sp, o, out_cap, head, ovf_count, ovf_list, tails);
  DR_LAUNCH_CHECK();
  return 0;
}
