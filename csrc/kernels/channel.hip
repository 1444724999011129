// Channel kernels: the send side of a hash / range shuffle between GPUs, for columnar tables.
//
// A Dryad CrossProduct channel (GraphBuilder.cs:481-504, DryadLinqVertex.cs:4788-4907
// HashPartition) becomes: destination of every record (stable_hash_dest / range_dest, one E128
// entry per row with the port in the low byte of .hi), then ONE pass that moves every column of
// the table into port-grouped order, then one RCCL all-to-all-v per column (parallel/exchange.py).
// The grouped table is both the local output ports and the send buffer: when the ports are
// numbered rank-major (the LUT below), the rows for destination rank r are one contiguous slice of
// every column, so nothing is packed again per destination.
//
//   pc_count_kernel    per-(bucket, workgroup) histogram of the (LUT-mapped) ports
//   pc_scatter_kernel  stable multi-column bucket scatter: each 512-row tile is ranked by bucket
//                      with wave64 ballot multisplits, then every column is staged through LDS
//                      (coalesced loads) and written as one contiguous run per bucket
//                      (pc_scatter_rows_kernel: <= 32 bytes of dword columns per row staged whole)
//   copy_segments      variable-length string bytes into a compact heap in row order (the string
//                      heap of the rows sent to each rank, sent by a second all-to-all-v)
#include "common.h"

namespace {
constexpr int kPcTile = 512;
constexpr int kPcItems = kPcTile / kBlock;   // rows ranked per thread per tile
constexpr int kPcMaxCols = 16;
constexpr int kPcChunk = 8;                  // dwords per row staged per column pass

struct PcCols {
  const uint8_t* in[kPcMaxCols];
  uint8_t* out[kPcMaxCols];
  uint32_t width[kPcMaxCols];   // bytes per row: 1, 2 or a multiple of 4
  uint32_t ncols;
};

// A row's bucket: the low byte of its E128 entry's hi word, or its byte of a uint8 port array
// (PORT8: the hash partitioner's compact form, 1 byte per row instead of 16).
template <bool PORT8>
__device__ __forceinline__ uint32_t pc_port(const void* __restrict__ ent, uint64_t i) {
  if constexpr (PORT8) return static_cast<const uint8_t*>(ent)[i];
  else return (uint32_t)(static_cast<const E128*>(ent)[i].hi & 0xFF);
}

template <bool PORT8>
__global__ __launch_bounds__(256) void pc_count_kernel(const void* __restrict__ ent, uint64_t n,
                                                       const uint8_t* __restrict__ lut, uint32_t* __restrict__ counts,
                                                       uint32_t G, uint64_t per_block) {
  __shared__ uint32_t hist[256];
  __shared__ uint8_t slut[256];
  const int t = threadIdx.x;
  hist[t] = 0;
  slut[t] = lut ? lut[t] : (uint8_t)t;
  __syncthreads();
  const uint64_t beg = (uint64_t)blockIdx.x * per_block;
  const uint64_t end = beg + per_block < n ? beg + per_block : n;
  for (uint64_t i = beg + t; i < end; i += kBlock) atomicAdd(&hist[slut[pc_port<PORT8>(ent, i)]], 1u);
  __syncthreads();
  counts[(uint64_t)t * G + blockIdx.x] = hist[t];
}

__device__ __forceinline__ uint32_t pc_load_narrow(const uint8_t* p, uint64_t row, uint32_t w) {
  return w == 1 ? (uint32_t)p[row] : (uint32_t)reinterpret_cast<const uint16_t*>(p)[row];
}

__device__ __forceinline__ void pc_store_narrow(uint8_t* p, uint64_t row, uint32_t w, uint32_t v) {
  if (w == 1) p[row] = (uint8_t)v;
  else reinterpret_cast<uint16_t*>(p)[row] = (uint16_t)v;
}

template <bool PORT8>
__global__ __launch_bounds__(256) void pc_scatter_kernel(const void* __restrict__ ent, uint64_t n,
                                                         const uint8_t* __restrict__ lut, PcCols cols,
                                                         const int64_t* __restrict__ offsets, uint32_t G,
                                                         uint64_t per_block) {
  __shared__ uint32_t buf[kPcTile * kPcChunk];
  __shared__ uint16_t perm[kPcTile];
  __shared__ uint8_t dslot[kPcTile];
  __shared__ uint32_t wcnt[4][256];
  __shared__ int64_t goff[256];
  __shared__ uint32_t bstart[256];
  __shared__ uint32_t sc[4];
  __shared__ uint8_t slut[256];
  const int t = threadIdx.x, w = wave_id(), l = lane_id();
  const uint64_t beg = (uint64_t)blockIdx.x * per_block;
  const uint64_t end = beg + per_block < n ? beg + per_block : n;
  if (beg >= end) return;                                    // uniform: the whole workgroup leaves
  slut[t] = lut ? lut[t] : (uint8_t)t;
  goff[t] = offsets[(uint64_t)t * G + blockIdx.x];
  __syncthreads();
  for (uint64_t base = beg; base < end; base += kPcTile) {
    const uint32_t cnt = (uint32_t)((end - base) < (uint64_t)kPcTile ? (end - base) : kPcTile);
    wcnt[0][t] = 0; wcnt[1][t] = 0; wcnt[2][t] = 0; wcnt[3][t] = 0;
    __syncthreads();
    uint32_t rk[kPcItems], dg[kPcItems];
#pragma unroll
    for (int r = 0; r < kPcItems; ++r) {
      const uint32_t pos = w * (kPcTile / 4) + r * 64 + l;
      const bool valid = pos < cnt;
      const uint32_t d = valid ? (uint32_t)slut[pc_port<PORT8>(ent, base + pos)] : 0u;
      uint64_t peers = ballot64(valid);
#pragma unroll
      for (int k = 0; k < 8; ++k) {
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
    for (int r = 0; r < kPcItems; ++r) {
      const uint32_t pos = w * (kPcTile / 4) + r * 64 + l;
      if (pos < cnt) {
        const uint32_t slot = bstart[dg[r]] + wcnt[w][dg[r]] + rk[r];
        perm[slot] = (uint16_t)pos;
        dslot[slot] = (uint8_t)dg[r];
      }
    }
    __syncthreads();
    // every column through LDS: coalesced tile loads, then slot-major stores (consecutive slots of
    // one bucket are consecutive output rows)
    for (uint32_t k = 0; k < cols.ncols; ++k) {
      const uint32_t wb = cols.width[k];
      const uint8_t* src = cols.in[k];
      uint8_t* dst = cols.out[k];
      if (wb < 4) {
        for (uint32_t j = t; j < cnt; j += kBlock) buf[j] = pc_load_narrow(src, base + j, wb);
        __syncthreads();
        for (uint32_t j = t; j < cnt; j += kBlock) {
          const uint32_t d = dslot[j];
          pc_store_narrow(dst, (uint64_t)(goff[d] + (int64_t)(j - bstart[d])), wb, buf[perm[j]]);
        }
        __syncthreads();
        continue;
      }
      const uint32_t wpr = wb >> 2;
      const uint32_t* s32 = reinterpret_cast<const uint32_t*>(src);
      uint32_t* d32 = reinterpret_cast<uint32_t*>(dst);
      for (uint32_t cw0 = 0; cw0 < wpr; cw0 += kPcChunk) {
        const uint32_t cw = wpr - cw0 < (uint32_t)kPcChunk ? wpr - cw0 : (uint32_t)kPcChunk;
        const uint32_t words = cnt * cw;
        if (cw == 1) {
          for (uint32_t q = t; q < words; q += kBlock) buf[q] = s32[(base + q) * wpr + cw0];
        } else if (cw == 2) {
          for (uint32_t q = t; q < words; q += kBlock) buf[q] = s32[(base + (q >> 1)) * wpr + cw0 + (q & 1)];
        } else {
          for (uint32_t q = t; q < words; q += kBlock) {
            const uint32_t r = q / cw, c = q - r * cw;
            buf[q] = s32[(base + r) * wpr + cw0 + c];
          }
        }
        __syncthreads();
        for (uint32_t q = t; q < words; q += kBlock) {
          const uint32_t j = cw == 1 ? q : (cw == 2 ? (q >> 1) : q / cw);
          const uint32_t c = q - j * cw;
          const uint32_t d = dslot[j];
          const uint64_t row = (uint64_t)(goff[d] + (int64_t)(j - bstart[d]));
          d32[row * wpr + cw0 + c] = buf[(uint32_t)perm[j] * cw + c];
        }
        __syncthreads();
      }
    }
    goff[t] += tot;
    __syncthreads();
  }
}

// pc_scatter_kernel for tables whose 4k-byte columns hold at most kPcChunk dwords per row in total
// (e.g. a key and three int64 values) plus at most kPcNarrow 1- or 2-byte columns (e.g. a count of
// int8 ones): every dword and narrow value of the tile's rows, over all columns, is loaded at once (kPcRowItems independent loads per lane, no branch around them: the
// lanes past the tile re-read its first row) and staged in LDS as whole rows, then stored slot by
// slot into every column.  Item i of lane t is dword c = i / 2 of tile row t + 256 (i % 2): the
// column of every load and store is a compile-time dword index, its pointer a scalar.  The
// per-column passes above keep one column's 4 KB per workgroup in flight between barriers (2.4 TB/s
// in the 8-rank GroupBy's hash partition).
constexpr int kPcRowItems = kPcTile * kPcChunk / kBlock;

// global (not flat) accesses through a generic pointer of global memory: flat loads and stores
// also count on the LDS wait counter, so every LDS wait would wait for them too
__device__ __forceinline__ uint32_t gload(const uint32_t* p, uint64_t i) {
  return reinterpret_cast<const __attribute__((address_space(1))) uint32_t*>(reinterpret_cast<uintptr_t>(p))[i];
}
__device__ __forceinline__ void gstore(uint32_t* p, uint64_t i, uint32_t v) {
  reinterpret_cast<__attribute__((address_space(1))) uint32_t*>(reinterpret_cast<uintptr_t>(p))[i] = v;
}
__device__ __forceinline__ uint32_t gload_narrow(const uint8_t* p, uint64_t row, uint32_t w) {
  const uintptr_t a = reinterpret_cast<uintptr_t>(p);
  return w == 1 ? (uint32_t)reinterpret_cast<const __attribute__((address_space(1))) uint8_t*>(a)[row]
                : (uint32_t)reinterpret_cast<const __attribute__((address_space(1))) uint16_t*>(a)[row];
}
__device__ __forceinline__ void gstore_narrow(uint8_t* p, uint64_t row, uint32_t w, uint32_t v) {
  const uintptr_t a = reinterpret_cast<uintptr_t>(p);
  if (w == 1) reinterpret_cast<__attribute__((address_space(1))) uint8_t*>(a)[row] = (uint8_t)v;
  else reinterpret_cast<__attribute__((address_space(1))) uint16_t*>(a)[row] = (uint16_t)v;
}
constexpr int kPcNarrow = 2;             // 1- / 2-byte columns the row kernel carries
static_assert(kPcRowItems == 2 * kPcChunk && kPcTile == 2 * kBlock, "item i: dword i / 2, row half i % 2");

template <bool PORT8>
__global__ __launch_bounds__(256) void pc_scatter_rows_kernel(const void* __restrict__ ent, uint64_t n,
                                                              const uint8_t* __restrict__ lut, PcCols cols,
                                                              const int64_t* __restrict__ offsets, uint32_t G,
                                                              uint64_t per_block) {
  __shared__ uint32_t buf[kPcTile * kPcChunk];
  __shared__ uint16_t nbuf[kPcNarrow][kPcTile];
  __shared__ uint16_t perm[kPcTile];
  __shared__ uint8_t dslot[kPcTile];
  __shared__ uint32_t wcnt[4][256];
  __shared__ int64_t goff[256];
  __shared__ uint32_t bstart[256];
  __shared__ uint32_t sc[4];
  __shared__ uint8_t slut[256];
  const int t = threadIdx.x, w = wave_id(), l = lane_id();
  const uint64_t beg = (uint64_t)blockIdx.x * per_block;
  const uint64_t end = beg + per_block < n ? beg + per_block : n;
  if (beg >= end) return;                                    // uniform: the whole workgroup leaves
  slut[t] = lut ? lut[t] : (uint8_t)t;
  goff[t] = offsets[(uint64_t)t * G + blockIdx.x];
  // row dword c -> its column's words, words per row and word index (all scalars)
  const uint32_t* cin[kPcChunk];
  uint32_t* cout[kPcChunk];
  uint32_t cwpr[kPcChunk], cwd[kPcChunk];
  uint32_t WT = 0;
#pragma unroll
  for (int c = 0; c < kPcChunk; ++c) {
    cin[c] = nullptr;
    cout[c] = nullptr;
    cwpr[c] = 1;
    cwd[c] = 0;
    uint32_t start = 0;
#pragma unroll
    for (int k = 0; k < kPcMaxCols; ++k) {
      const uint32_t wk = (uint32_t)k < cols.ncols && cols.width[k] >= 4 ? cols.width[k] >> 2 : 0u;
      if ((uint32_t)c >= start && (uint32_t)c < start + wk) {
        cin[c] = reinterpret_cast<const uint32_t*>(cols.in[k]);
        cout[c] = reinterpret_cast<uint32_t*>(cols.out[k]);
        cwpr[c] = wk;
        cwd[c] = (uint32_t)c - start;
      }
      start += wk;
    }
    if (c == kPcChunk - 1) WT = start;
  }
  // the 1- and 2-byte columns (at most kPcNarrow: the caller checks), loaded with the dwords
  const uint8_t* nin[kPcNarrow];
  uint8_t* nout[kPcNarrow];
  uint32_t nw[kPcNarrow];
#pragma unroll
  for (int m = 0; m < kPcNarrow; ++m) {
    nin[m] = nullptr;
    nout[m] = nullptr;
    nw[m] = 0;
    uint32_t seen = 0;
#pragma unroll
    for (int k = 0; k < kPcMaxCols; ++k) {
      const bool narrow = (uint32_t)k < cols.ncols && cols.width[k] < 4;
      if (narrow && seen == (uint32_t)m) {
        nin[m] = cols.in[k];
        nout[m] = cols.out[k];
        nw[m] = cols.width[k];
      }
      seen += narrow ? 1u : 0u;
    }
  }
  __syncthreads();
  // a tile's rows (every column) and ports, loaded at once with clamped rows (no branch around a
  // load); the next tile's loads are issued as soon as this tile is staged, so they are in flight
  // while it is ranked and stored
  uint32_t v[kPcRowItems];
  uint32_t nv[kPcNarrow][2];
  uint32_t pd[kPcItems];
  auto load_tile = [&](uint64_t b0, uint32_t cn) {
#pragma unroll
    for (int i = 0; i < kPcRowItems; ++i) {
      const int c = i >> 1;
      const uint32_t r = (uint32_t)t + (uint32_t)(i & 1) * kBlock;
      const bool use = (uint32_t)c < WT;
      v[i] = gload(use ? cin[c] : cin[0], (b0 + (r < cn ? r : 0u)) * (use ? cwpr[c] : 1u) + (use ? cwd[c] : 0u));
    }
#pragma unroll
    for (int m = 0; m < kPcNarrow; ++m)
#pragma unroll
      for (int h = 0; h < 2; ++h) {
        const uint32_t r = (uint32_t)t + (uint32_t)h * kBlock;
        nv[m][h] = gload_narrow(nw[m] ? nin[m] : reinterpret_cast<const uint8_t*>(cin[0]), b0 + (r < cn ? r : 0u),
                                nw[m] ? nw[m] : 1u);
      }
#pragma unroll
    for (int r = 0; r < kPcItems; ++r) {
      const uint32_t pos = w * (kPcTile / 4) + r * 64 + l;
      pd[r] = pc_port<PORT8>(ent, b0 + (pos < cn ? pos : 0u));
    }
  };
  auto tile_rows = [&](uint64_t b0) -> uint32_t {
    return (uint32_t)((end - b0) < (uint64_t)kPcTile ? (end - b0) : kPcTile);
  };
  load_tile(beg, tile_rows(beg));
  for (uint64_t base = beg; base < end; base += kPcTile) {
    const uint32_t cnt = tile_rows(base);
    wcnt[0][t] = 0; wcnt[1][t] = 0; wcnt[2][t] = 0; wcnt[3][t] = 0;
    __syncthreads();
    uint32_t rk[kPcItems], dg[kPcItems];
#pragma unroll
    for (int r = 0; r < kPcItems; ++r) {
      const uint32_t pos = w * (kPcTile / 4) + r * 64 + l;
      const bool valid = pos < cnt;
      const uint32_t d = valid ? (uint32_t)slut[pd[r]] : 0u;
      uint64_t peers = ballot64(valid);
#pragma unroll
      for (int k = 0; k < 8; ++k) {
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
#pragma unroll
    for (int i = 0; i < kPcRowItems; ++i) {
      const int c = i >> 1;
      const uint32_t r = (uint32_t)t + (uint32_t)(i & 1) * kBlock;
      if ((uint32_t)c < WT && r < cnt) buf[r * WT + c] = v[i];
    }
#pragma unroll
    for (int m = 0; m < kPcNarrow; ++m)
#pragma unroll
      for (int h = 0; h < 2; ++h) {
        const uint32_t r = (uint32_t)t + (uint32_t)h * kBlock;
        if (nw[m] && r < cnt) nbuf[m][r] = (uint16_t)nv[m][h];
      }
    if (base + kPcTile < end) load_tile(base + kPcTile, tile_rows(base + kPcTile));
    __syncthreads();
    const uint32_t c0 = wcnt[0][t], c1 = wcnt[1][t], c2 = wcnt[2][t], c3 = wcnt[3][t];
    const uint32_t tot = c0 + c1 + c2 + c3;
    wcnt[0][t] = 0; wcnt[1][t] = c0; wcnt[2][t] = c0 + c1; wcnt[3][t] = c0 + c1 + c2;
    uint32_t all;
    bstart[t] = block_exclusive_scan256(tot, sc, all);
    __syncthreads();
#pragma unroll
    for (int r = 0; r < kPcItems; ++r) {
      const uint32_t pos = w * (kPcTile / 4) + r * 64 + l;
      if (pos < cnt) {
        const uint32_t slot = bstart[dg[r]] + wcnt[w][dg[r]] + rk[r];
        perm[slot] = (uint16_t)pos;
        dslot[slot] = (uint8_t)dg[r];
      }
    }
    __syncthreads();
    // slot-major stores: consecutive slots of one bucket are consecutive output rows of a column
#pragma unroll
    for (int i = 0; i < kPcRowItems; ++i) {
      const int c = i >> 1;
      const uint32_t j = (uint32_t)t + (uint32_t)(i & 1) * kBlock;
      if ((uint32_t)c < WT && j < cnt) {
        const uint32_t d = dslot[j];
        const uint64_t row = (uint64_t)(goff[d] + (int64_t)(j - bstart[d]));
        gstore(cout[c], row * cwpr[c] + cwd[c], buf[(uint32_t)perm[j] * WT + c]);
      }
    }
#pragma unroll
    for (int m = 0; m < kPcNarrow; ++m)
#pragma unroll
      for (int h = 0; h < 2; ++h) {
        const uint32_t j = (uint32_t)t + (uint32_t)h * kBlock;
        if (nw[m] && j < cnt) {
          const uint32_t d = dslot[j];
          gstore_narrow(nout[m], (uint64_t)(goff[d] + (int64_t)(j - bstart[d])), nw[m], nbuf[m][perm[j]]);
        }
      }
    __syncthreads();                   // every store has read goff / bstart
    goff[t] += tot;
    __syncthreads();
  }
}

// One wave per 64 consecutive rows: the wave's strings form one destination range of T bytes
// (gaps between them allowed: bytes in a gap are not written); lane b copies bytes b, b+64, ...
// after a 6-step search of the row that holds it.
__global__ __launch_bounds__(256) void copy_segments_kernel(const uint8_t* __restrict__ src,
                                                            const int64_t* __restrict__ soff,
                                                            const int64_t* __restrict__ len,
                                                            const int64_t* __restrict__ doff, uint64_t n,
                                                            uint8_t* __restrict__ dst) {
  __shared__ int64_t ends[4][64];
  __shared__ int64_t begs[4][64];
  __shared__ int64_t srcs[4][64];
  const int w = wave_id(), l = lane_id();
  const uint64_t nwaves = (uint64_t)gridDim.x * 4;
  for (uint64_t g = (uint64_t)blockIdx.x * 4 + w; g * 64 < n; g += nwaves) {
    const uint64_t r0 = g * 64;
    const uint64_t rows = n - r0 < 64 ? n - r0 : 64;
    const int64_t base = doff[r0];
    int64_t e = 0, so = 0, st = 0;
    if ((uint64_t)l < rows) {
      st = doff[r0 + l] - base;
      e = st + len[r0 + l];
      so = soff[r0 + l] - st;          // source byte of destination byte b in this row: so + b
    } else {
      st = e = doff[r0 + rows - 1] - base + len[r0 + rows - 1];
    }
    ends[w][l] = e;
    begs[w][l] = st;
    srcs[w][l] = so;
    __builtin_amdgcn_wave_barrier();
    const int64_t T = __shfl(e, 63, 64);
    for (int64_t b = l; b < T; b += 64) {
      int lo = 0;
#pragma unroll
      for (int step = 32; step >= 1; step >>= 1)
        if (lo + step <= 63 && ends[w][lo + step - 1] <= b) lo += step;
      if (b >= begs[w][lo]) dst[base + b] = src[srcs[w][lo] + b];   // gaps between strings stay
    }
    __builtin_amdgcn_wave_barrier();
  }
}
// Bulk copy by the CUs (16-byte vector loads / stores, 4 in flight per lane, grid-stride).  Either
// side may be page-locked host memory mapped into the device address space: the CUs then move the
// bytes over PCIe themselves, without a DMA engine (a second path next to the copy engines when
// both directions stream at once).
__global__ __launch_bounds__(256) void copy_wide_kernel(const uint4* __restrict__ src, uint4* __restrict__ dst,
                                                        uint64_t n16) {
  const uint64_t stride = (uint64_t)gridDim.x * blockDim.x;
  uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
  for (; i + 3 * stride < n16; i += 4 * stride) {
    uint4 v[4];
#pragma unroll
    for (int k = 0; k < 4; ++k) v[k] = src[i + k * stride];
#pragma unroll
    for (int k = 0; k < 4; ++k) dst[i + k * stride] = v[k];
  }
  for (; i < n16; i += stride) dst[i] = src[i];
}

__global__ void copy_tail_kernel(const uint8_t* __restrict__ src, uint8_t* __restrict__ dst, uint32_t n) {
  const uint32_t i = threadIdx.x;
  if (i < n) dst[i] = src[i];
}
}  // namespace

// Geometry shared by the count and scatter launches (the caller sizes `counts` as 256 * G).
#ifndef DR_PC_GMAX
#define DR_PC_GMAX 16384
#endif
DR_API uint32_t dr_pc_grid(uint64_t n, uint64_t* per_block) {
  uint64_t tiles = (n + kPcTile - 1) / kPcTile;
  if (tiles < 1) tiles = 1;
  // up to DR_PC_GMAX workgroups of 4 waves: at 1024 (16 waves per CU, many tiles each) the row
  // scatter waited on memory; a few tiles per workgroup keeps more of them in flight
  // (tools/gpurun/r5c_pc_ab.sh, profiles/r5/pc_grid_ab.txt)
  const uint64_t G = tiles < DR_PC_GMAX ? tiles : DR_PC_GMAX;
  *per_block = ((tiles + G - 1) / G) * kPcTile;
  return (uint32_t)G;
}

// ent: E128 entries (port8 = 0) or a uint8 port per row (port8 = 1).
DR_API int dr_pc_count(const void* ent, uint64_t n, const uint8_t* lut, uint32_t* counts, uint32_t G,
                       uint64_t per_block, int port8, hipStream_t s) {
  if (n == 0) return 0;
  if (port8)
    pc_count_kernel<true><<<G, 256, 0, s>>>(ent, n, lut, counts, G, per_block);
  else
    pc_count_kernel<false><<<G, 256, 0, s>>>(ent, n, lut, counts, G, per_block);
  DR_LAUNCH_CHECK();
  return 0;
}

// offsets: int64 [256 * G], exclusive prefix of the bucket-major counts (destination row of each
// workgroup's first row of each bucket).  in/out/width: ncols (<= 16) device columns.
DR_API int dr_pc_scatter(const void* ent, uint64_t n, const uint8_t* lut, const void* const* in, void* const* out,
                         const uint32_t* width, uint32_t ncols, const int64_t* offsets, uint32_t G, uint64_t per_block,
                         int port8, hipStream_t s) {
  if (ncols > (uint32_t)kPcMaxCols || n >= (1ull << 40)) return (int)hipErrorInvalidValue;
  if (n == 0 || ncols == 0) return 0;
  PcCols c;
  for (uint32_t k = 0; k < ncols; ++k) {
    const uint32_t wb = width[k];
    if (wb == 0 || (wb > 2 && (wb & 3))) return (int)hipErrorInvalidValue;
    c.in[k] = static_cast<const uint8_t*>(in[k]);
    c.out[k] = static_cast<uint8_t*>(out[k]);
    c.width[k] = wb;
  }
  c.ncols = ncols;
  uint32_t wt = 0, narrow = 0;
  for (uint32_t k = 0; k < ncols; ++k) {
    wt += width[k] >= 4 ? width[k] >> 2 : 0u;
    narrow += width[k] < 4 ? 1u : 0u;
  }
  if (wt > 0 && wt <= (uint32_t)kPcChunk && narrow <= (uint32_t)kPcNarrow) {   // whole rows staged at once
    if (port8)
      pc_scatter_rows_kernel<true><<<G, 256, 0, s>>>(ent, n, lut, c, offsets, G, per_block);
    else
      pc_scatter_rows_kernel<false><<<G, 256, 0, s>>>(ent, n, lut, c, offsets, G, per_block);
  } else if (port8)
    pc_scatter_kernel<true><<<G, 256, 0, s>>>(ent, n, lut, c, offsets, G, per_block);
  else
    pc_scatter_kernel<false><<<G, 256, 0, s>>>(ent, n, lut, c, offsets, G, per_block);
  DR_LAUNCH_CHECK();
  return 0;
}

DR_API int dr_copy_segments(const uint8_t* src, const int64_t* soff, const int64_t* len, const int64_t* doff,
                            uint64_t n, uint8_t* dst, hipStream_t s) {
  if (n == 0) return 0;
  copy_segments_kernel<<<grid_for((n + 63) / 64, 4, 8192), 256, 0, s>>>(src, soff, len, doff, n, dst);
  DR_LAUNCH_CHECK();
  return 0;
}

// dst/src: device pointers (HBM, or page-locked host memory through its device mapping).
// grid: workgroups (0 = 1024).  Bytes past the last 16-byte block are copied by a second launch.
DR_API int dr_copy_wide(void* dst, const void* src, uint64_t nbytes, uint32_t grid, hipStream_t s) {
  if (nbytes == 0) return 0;
  if (((uintptr_t)dst | (uintptr_t)src) & 15) return (int)hipErrorInvalidValue;
  const uint64_t n16 = nbytes / 16;
  if (n16) {
    const uint64_t want = (n16 + 255) / 256;
    const uint32_t g = (uint32_t)(want < (grid ? grid : 1024u) ? want : (grid ? grid : 1024u));
    copy_wide_kernel<<<g, 256, 0, s>>>(static_cast<const uint4*>(src), static_cast<uint4*>(dst), n16);
  }
  const uint32_t tail = (uint32_t)(nbytes - n16 * 16);
  if (tail)
    copy_tail_kernel<<<1, 64, 0, s>>>(static_cast<const uint8_t*>(src) + n16 * 16, static_cast<uint8_t*>(dst) + n16 * 16,
                                      tail);
  DR_LAUNCH_CHECK();
  return 0;
}
