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
template <int ITEMS, int WC, int OWC, bool VEC, bool STAGE_PROJ = false>
__global__ __launch_bounds__(256) void gp_scatter_kernel(const uint32_t* __restrict__ rows, uint64_t n, uint32_t Wdyn,
                                                         uint32_t kw, int key_len, uint64_t seed, int shift, uint32_t nb,
                                                         const uint32_t* __restrict__ prefix,
                                                         const int64_t* __restrict__ base,
                                                         const uint64_t* __restrict__ dst_ptr,
                                                         const int64_t* __restrict__ cap, uint32_t contig_from,
                                                         uint32_t G, uint64_t per_block, uint32_t OWdyn, uint32_t PO) {
  constexpr int TILE = kBlock * ITEMS;
  const uint32_t W = WC > 0 ? (uint32_t)WC : Wdyn;
  const uint32_t OW = OWC > 0 ? (uint32_t)OWC : OWdyn;
  const uint32_t LW = STAGE_PROJ ? OW : W;            // dwords per row in the LDS image
  const uint32_t LPO = STAGE_PROJ ? 0u : PO;          // projection offset inside the LDS image
  const uint32_t lkw = STAGE_PROJ ? kw - PO : kw;     // key offset inside the LDS image
  __shared__ __attribute__((aligned(16))) uint32_t srow[16384];   // 64 KiB of rows
  __shared__ uint16_t perm[TILE];
  __shared__ uint8_t dslot[TILE];
  __shared__ uint32_t wcnt[4][kMaxBuckets];
  __shared__ int64_t goff[kMaxBuckets];
  __shared__ uint32_t bstart[kMaxBuckets];
  __shared__ uint64_t sptr[kMaxBuckets];
  __shared__ int64_t scap[kMaxBuckets];
  __shared__ uint32_t sc[4];
  const int t = threadIdx.x, w = wave_id(), l = lane_id();
  if ((uint32_t)t < nb) {
    goff[t] = base[t] + (int64_t)prefix[(uint64_t)t * G + blockIdx.x];
    sptr[t] = dst_ptr[t];
    scap[t] = (cap && (uint32_t)t < contig_from) ? cap[t] : (int64_t)0x7FFFFFFFFFFFFFFFll;
  }
  const uint64_t beg = (uint64_t)blockIdx.x * per_block;
  const uint64_t end = beg + per_block < n ? beg + per_block : n;
  for (uint64_t tb = beg; tb < end; tb += TILE) {
    const uint32_t cnt = (uint32_t)((end - tb) < (uint64_t)TILE ? (end - tb) : TILE);
    if (STAGE_PROJ) {
      const uint32_t C = W / 4, OC = OW / 4, P4 = PO / 4;
      const uint32_t chunks = cnt * OC;
      const uint4* src = reinterpret_cast<const uint4*>(rows + tb * W);
      uint4* dst = reinterpret_cast<uint4*>(srow);
      for (uint32_t q = t; q < chunks; q += kBlock) {
        const uint32_t j = q / OC, c = q - j * OC;
        dst[q] = src[(uint64_t)j * C + P4 + c];
      }
    } else if (VEC) {
      const uint32_t chunks = cnt * W / 4;
      const uint4* src = reinterpret_cast<const uint4*>(rows + tb * W);
      uint4* dst = reinterpret_cast<uint4*>(srow);
      for (uint32_t j = t; j < chunks; j += kBlock) dst[j] = src[j];
    } else {
      const uint32_t words = cnt * W;
      const uint32_t* src = rows + tb * W;
      for (uint32_t j = t; j < words; j += kBlock) srow[j] = src[j];
    }
    wcnt[0][t] = 0; wcnt[1][t] = 0; wcnt[2][t] = 0; wcnt[3][t] = 0;
    __syncthreads();
    uint32_t rk[ITEMS], dg[ITEMS];
#pragma unroll
    for (int r = 0; r < ITEMS; ++r) {
      const uint32_t pos = w * (TILE / 4) + r * 64 + l;
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
    const uint32_t c0 = wcnt[0][t], c1 = wcnt[1][t], c2 = wcnt[2][t], c3 = wcnt[3][t];
    const uint32_t tot = c0 + c1 + c2 + c3;
    wcnt[0][t] = 0; wcnt[1][t] = c0; wcnt[2][t] = c0 + c1; wcnt[3][t] = c0 + c1 + c2;
    uint32_t all;
    bstart[t] = block_exclusive_scan256(tot, sc, all);
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
    // slot-major copy: consecutive lanes write consecutive pieces of consecutive slots, and the
    // slots of one bucket are consecutive rows of its destination
    if (VEC) {
      const uint32_t LC = LW / 4, OC = OW / 4, P4 = LPO / 4;
      const uint32_t chunks = cnt * OC;
      const uint4* s4 = reinterpret_cast<const uint4*>(srow);
      for (uint32_t q = t; q < chunks; q += kBlock) {
        const uint32_t j = q / OC, c = q - j * OC;
        const uint32_t d = dslot[j];
        const int64_t row = goff[d] + (int64_t)(j - bstart[d]);
        if (row < scap[d])
          reinterpret_cast<uint4*>(sptr[d])[(uint64_t)row * OC + c] = s4[(uint32_t)perm[j] * LC + P4 + c];
      }
    } else {
      const uint32_t words = cnt * OW;
      for (uint32_t q = t; q < words; q += kBlock) {
        const uint32_t j = q / OW, c = q - j * OW;
        const uint32_t d = dslot[j];
        const int64_t row = goff[d] + (int64_t)(j - bstart[d]);
        if (row < scap[d])
          reinterpret_cast<uint32_t*>(sptr[d])[(uint64_t)row * OW + c] = srow[(uint32_t)perm[j] * LW + LPO + c];
      }
    }
    __syncthreads();
    if ((uint32_t)t < nb) goff[t] += tot;
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

// Workspace (bytes) of dr_grace_partition for n rows of `stride` bytes into nb destinations.
DR_API uint64_t dr_grace_workspace(uint64_t n, uint32_t stride, uint32_t nb) {
  uint32_t G; uint64_t per_block;
  geometry(n, stride <= 64 ? 1024 : 512, G, per_block);     // the most workgroups any tile size gives
  return (uint64_t)nb * G * 4 + (uint64_t)nb * 8 * 2 + 256;
}

// Partition `n` rows (stride % 4 == 0, <= 128 bytes) by dest = fastrange(32 bits of hash(key) at
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
                              uint32_t* overflow, void* ws, uint32_t out_stride, uint32_t proj_off, hipStream_t s) {
  if (!key_ok(stride, key_off, key_len) || stride > 128 || nb < 1 || nb > kMaxBuckets || n >= (1ull << 32) ||
      (shift != 0 && shift != 32))
    return (int)hipErrorInvalidValue;
  if (out_stride == 0 || (out_stride & 3) || (proj_off & 3) || proj_off + out_stride > stride)
    return (int)hipErrorInvalidValue;
  if (n == 0) {
    hipMemsetAsync(chunk_counts, 0, sizeof(int64_t) * nb, s);
    return 0;
  }
  const bool small = stride <= 64;
  const bool vec0 = (stride & 15) == 0 && (out_stride & 15) == 0 && (proj_off & 15) == 0 &&
                    (((uintptr_t)rows) & 15) == 0;
  // 16-byte projection holding the key: stage only the projected slice (4096-row tiles)
  const bool stage_proj = vec0 && out_stride == 16 && stride > 16 && key_off >= proj_off &&
                          key_off + key_len <= proj_off + out_stride;
  uint32_t G; uint64_t per_block;
  geometry(n, stage_proj ? 4096 : (small ? 1024 : 512), G, per_block);
  uint32_t* counts = reinterpret_cast<uint32_t*>(ws);
  uint64_t* totals = reinterpret_cast<uint64_t*>(reinterpret_cast<uint8_t*>(ws) + (((uint64_t)nb * G * 4 + 15) & ~15ull));
  const uint32_t W = stride / 4, kw = key_off / 4;
  const uint32_t* in = reinterpret_cast<const uint32_t*>(rows);
  gp_count_kernel<<<G, 256, 0, s>>>(in, n, W, kw, (int)key_len, seed, shift, nb, counts, G, per_block);
  gp_totals_kernel<<<nb, 256, 0, s>>>(counts, G, totals);
  gp_offsets_kernel<<<nb, 256, 0, s>>>(counts, G, totals, fill, cap, contig_from, bases, chunk_counts, overflow);
  const bool vec = vec0;
  const uint32_t OW = out_stride / 4, PO = proj_off / 4;
#define DR_GP_SCATTER(IT, WCV, OWCV, VECV)                                                               \
  gp_scatter_kernel<IT, WCV, OWCV, VECV><<<G, 256, 0, s>>>(in, n, W, kw, (int)key_len, seed, shift, nb, counts, \
                                                           bases, dst_ptr, cap, contig_from, G, per_block, OW, PO)
  if (stage_proj) {
    gp_scatter_kernel<16, 0, 4, true, true><<<G, 256, 0, s>>>(in, n, W, kw, (int)key_len, seed, shift, nb, counts,
                                                              bases, dst_ptr, cap, contig_from, G, per_block, OW, PO);
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
