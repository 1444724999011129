// Record (de)serialisation on the device (K14): DryadLinqBinary fixed-width records <-> columns.
//
// A record type whose fields are all fixed-width primitives (no strings, no nullable fields)
// serialises as the little-endian fields back to back (reference DryadLinqBinaryWriter.cs
// WriteRawBytes of each primitive; DryadLinqCodeGen.cs:1041-1096 field order), so a partfile
// part of such records is an [n, width] byte matrix.  Decoding = scattering each field's bytes
// into its column (AoS -> SoA), encoding = the reverse: records of <= 128 bytes through LDS tiles
// (codec_tile_kernel), wider ones one thread per (record, field) with byte loads / stores
// (fields need not be aligned inside the record).
#include "common.h"

namespace {
constexpr int kMaxFields = 32;

struct FieldMap {
  uint32_t off[kMaxFields];
  uint32_t size[kMaxFields];
  uint8_t* col[kMaxFields];
};

template <bool DECODE>
__global__ __launch_bounds__(256) void codec_kernel(uint8_t* __restrict__ rows, uint64_t n, uint32_t width, int nf,
                                                    FieldMap m) {
  const uint64_t total = n * (uint64_t)nf;
  for (uint64_t t = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; t < total; t += (uint64_t)gridDim.x * blockDim.x) {
    const uint64_t r = t / nf;
    const int f = (int)(t % nf);
    const uint32_t sz = m.size[f];
    uint8_t* rp = rows + r * width + m.off[f];
    uint8_t* cp = m.col[f] + r * sz;
    if (DECODE) {
      for (uint32_t b = 0; b < sz; ++b) cp[b] = rp[b];
    } else {
      for (uint32_t b = 0; b < sz; ++b) rp[b] = cp[b];
    }
  }
}

// Tiled variant (records of <= 128 bytes): a 256-record tile moves between HBM and LDS as whole
// 16-byte chunks (coalesced, from the first 16-byte boundary of the tile on), and between LDS and
// the columns one element per thread (coalesced column access).  The per-(record, field) kernel
// above issues one byte load and one byte store per byte at a record stride.  Encode writes the
// tile's partial first / last chunks byte by byte (their other bytes belong to the neighbouring
// tiles).
__device__ __forceinline__ uint64_t lds_bytes(const uint8_t* p, uint32_t sz) {
  uint64_t v = 0;
  for (uint32_t b = 0; b < sz; ++b) v |= (uint64_t)p[b] << (8 * b);
  return v;
}

template <bool DECODE>
__global__ __launch_bounds__(256) void codec_tile_kernel(uint8_t* __restrict__ rows, uint64_t n, uint32_t width, int nf,
                                                         FieldMap m) {
  __shared__ uint4 img[(256 * 128 + 32) / 16];
  uint8_t* lds = reinterpret_cast<uint8_t*>(img);
  const uint32_t t = threadIdx.x;
  for (uint64_t row0 = (uint64_t)blockIdx.x * 256; row0 < n; row0 += (uint64_t)gridDim.x * 256) {
    const uint32_t nr = (uint32_t)((n - row0) < 256 ? (n - row0) : 256);
    uint8_t* a = rows + row0 * width;
    const uint32_t shift = (uint32_t)(reinterpret_cast<uintptr_t>(a) & 15);
    uint4* base = reinterpret_cast<uint4*>(a - shift);
    const uint32_t bytes = nr * width;
    const uint32_t chunks = (bytes + shift + 15) / 16;
    __syncthreads();                               // the previous tile is done with the LDS image
    if (DECODE) {
      for (uint32_t c = t; c < chunks; c += 256) img[c] = base[c];
      __syncthreads();
      for (int f = 0; f < nf; ++f) {
        const uint32_t sz = m.size[f];
        if (t < nr) {
          const uint8_t* src = lds + shift + t * width + m.off[f];
          uint8_t* dst = m.col[f] + (row0 + t) * sz;
          if (sz == 8) *reinterpret_cast<uint64_t*>(dst) = lds_bytes(src, 8);
          else if (sz == 4) *reinterpret_cast<uint32_t*>(dst) = (uint32_t)lds_bytes(src, 4);
          else if (sz == 2) *reinterpret_cast<uint16_t*>(dst) = (uint16_t)lds_bytes(src, 2);
          else for (uint32_t b = 0; b < sz; ++b) dst[b] = src[b];
        }
      }
    } else {
      for (int f = 0; f < nf; ++f) {
        const uint32_t sz = m.size[f];
        if (t < nr) {
          uint8_t* dst = lds + shift + t * width + m.off[f];
          const uint8_t* src = m.col[f] + (row0 + t) * sz;
          uint64_t v = 0;
          if (sz == 8) v = *reinterpret_cast<const uint64_t*>(src);
          else if (sz == 4) v = *reinterpret_cast<const uint32_t*>(src);
          else if (sz == 2) v = *reinterpret_cast<const uint16_t*>(src);
          if (sz == 8 || sz == 4 || sz == 2) {
            for (uint32_t b = 0; b < sz; ++b) dst[b] = (uint8_t)(v >> (8 * b));
          } else {
            for (uint32_t b = 0; b < sz; ++b) dst[b] = src[b];
          }
        }
      }
      __syncthreads();
      for (uint32_t c = t; c < chunks; c += 256) {
        const uint32_t c0 = c * 16;                 // chunk bytes [c0, c0 + 16) of the image
        if (c0 >= shift && c0 + 16 <= shift + bytes) {
          base[c] = img[c];
        } else {
          uint8_t* d = reinterpret_cast<uint8_t*>(base + c);
          for (uint32_t b = 0; b < 16; ++b)
            if (c0 + b >= shift && c0 + b < shift + bytes) d[b] = lds[c0 + b];
        }
      }
    }
  }
}
}  // namespace

// direction 0: rows -> columns (decode), 1: columns -> rows (encode).  offs/sizes/cols are host
// arrays of nf <= 32 entries (cols hold device pointers).
DR_API int dr_codec_fixed(uint8_t* rows, uint64_t n, uint32_t width, int nf, const uint32_t* offs,
                          const uint32_t* sizes, uint8_t* const* cols, int direction, hipStream_t s) {
  if (nf < 1 || nf > kMaxFields) return (int)hipErrorInvalidValue;
  if (n == 0) return 0;
  FieldMap m;
  for (int f = 0; f < nf; ++f) {
    m.off[f] = offs[f];
    m.size[f] = sizes[f];
    m.col[f] = cols[f];
    if (offs[f] + sizes[f] > width) return (int)hipErrorInvalidValue;
  }
  bool aligned_cols = true;                    // column element stores need natural alignment
  for (int f = 0; f < nf; ++f)
    if (reinterpret_cast<uintptr_t>(cols[f]) % (sizes[f] <= 8 ? sizes[f] : 1)) aligned_cols = false;
  if (width <= 128 && aligned_cols) {
    const unsigned g = grid_for(n, 256, 16384);
    if (direction == 0)
      codec_tile_kernel<true><<<g, 256, 0, s>>>(rows, n, width, nf, m);
    else
      codec_tile_kernel<false><<<g, 256, 0, s>>>(rows, n, width, nf, m);
    DR_LAUNCH_CHECK();
    return 0;
  }
  const unsigned g = grid_for(n * (uint64_t)nf, 256, 16384);
  if (direction == 0)
    codec_kernel<true><<<g, 256, 0, s>>>(rows, n, width, nf, m);
  else
    codec_kernel<false><<<g, 256, 0, s>>>(rows, n, width, nf, m);
  DR_LAUNCH_CHECK();
  return 0;
}

// ---------------------------------------------------------------------------------------------
// Variable-length records (fields: fixed-width primitives and strings; no nullable fields).
//
// A string field is compact(#UTF-16 code units) + compact(#UTF-8 bytes) + the bytes, with the
// second compact's width (1 or 4 bytes) taken from the maximum byte count (units + 1) * 3
// (reference DryadLinqBinaryWriter.cs:523-546, DryadLinqBinaryReader.cs:341-366, 628-632;
// compact = 1 byte below 0x80, else 4 bytes big-endian with the top bit set).  Where records
// start is only known by parsing from the stream's start, so decoding takes a block index
// (byte offset of every B-th record, written with the part or found by the host scan
// codec.cpp:scan_record_blocks): one thread per block parses its B records and writes the
// columns; string fields become (offset, length) pairs into the part's bytes, which stay the
// string heap.  Encoding: per record its size (string bytes are scanned for their UTF-16
// units), an exclusive scan on the host side, then one thread per record writes it.
namespace {
struct VarMap {
  uint32_t size[kMaxFields];      // bytes of a fixed field, 0 = string
  uint8_t* col[kMaxFields];       // fixed: the column; string: int64 byte offsets
  int64_t* len[kMaxFields];       // string: int64 byte lengths
  const uint8_t* heap[kMaxFields];// encode: the string field's heap
};

__device__ __forceinline__ uint32_t rd_compact(const uint8_t* p, uint64_t& pos, uint64_t end, bool& bad) {
  if (pos >= end) { bad = true; return 0; }
  const uint32_t b0 = p[pos];
  if (b0 < 0x80) { pos += 1; return b0; }
  if (pos + 4 > end) { bad = true; return 0; }
  const uint32_t v = ((b0 & 0x7Fu) << 24) | ((uint32_t)p[pos + 1] << 16) | ((uint32_t)p[pos + 2] << 8) | p[pos + 3];
  pos += 4;
  return v;
}

__global__ __launch_bounds__(256) void codec_var_decode(const uint8_t* __restrict__ buf, uint64_t nbytes,
                                                        const int64_t* __restrict__ block_off, uint64_t nblocks,
                                                        uint32_t B, uint64_t n, int nf, VarMap m,
                                                        uint32_t* __restrict__ err) {
  for (uint64_t b = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; b < nblocks;
       b += (uint64_t)gridDim.x * blockDim.x) {
    uint64_t pos = (uint64_t)block_off[b];
    uint64_t end = b + 1 < nblocks ? (uint64_t)block_off[b + 1] : nbytes;
    end = end < nbytes ? end : nbytes;             // a stale / corrupt index never reads past the part
    const uint64_t r0 = b * B, r1 = r0 + B < n ? r0 + B : n;
    bool bad = pos > end;
    for (uint64_t r = r0; r < r1 && !bad; ++r) {
      for (int f = 0; f < nf; ++f) {
        const uint32_t sz = m.size[f];
        if (sz) {
          if (pos + sz > end) { bad = true; break; }
          uint8_t* c = m.col[f] + r * sz;
          for (uint32_t k = 0; k < sz; ++k) c[k] = buf[pos + k];
          pos += sz;
        } else {
          rd_compact(buf, pos, end, bad);
          const uint32_t nb = rd_compact(buf, pos, end, bad);
          if (bad || pos + nb > end) { bad = true; break; }
          reinterpret_cast<int64_t*>(m.col[f])[r] = (int64_t)pos;
          m.len[f][r] = (int64_t)nb;
          pos += nb;
        }
      }
    }
    if (bad || pos != end) atomicOr(err, 1u);      // the index and the stream disagree
  }
}

__device__ __forceinline__ uint32_t utf16_units_dev(const uint8_t* s, uint64_t nb) {
  uint32_t u = 0;
  for (uint64_t i = 0; i < nb;) {
    const uint8_t c = s[i];
    if (c < 0x80) { i += 1; u += 1; }
    else if (c < 0xE0) { i += 2; u += 1; }
    else if (c < 0xF0) { i += 3; u += 1; }
    else { i += 4; u += 2; }
  }
  return u;
}

__device__ __forceinline__ uint32_t compact_size(uint32_t v) { return v < 0x80 ? 1u : 4u; }

// pass 1: record sizes (and the UTF-16 unit counts of every string field)
__global__ __launch_bounds__(256) void codec_var_sizes(uint64_t n, int nf, VarMap m, uint32_t* __restrict__ units,
                                                       int64_t* __restrict__ sizes) {
  for (uint64_t r = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; r < n; r += (uint64_t)gridDim.x * blockDim.x) {
    uint64_t sz = 0;
    int sf = 0;
    for (int f = 0; f < nf; ++f) {
      if (m.size[f]) {
        sz += m.size[f];
      } else {
        const int64_t off = reinterpret_cast<const int64_t*>(m.col[f])[r];
        const uint64_t nb = (uint64_t)m.len[f][r];
        const uint32_t u = utf16_units_dev(m.heap[f] + off, nb);
        units[(uint64_t)sf * n + r] = u;
        sz += compact_size(u) + compact_size((u + 1) * 3) + nb;
        ++sf;
      }
    }
    sizes[r] = (int64_t)sz;
  }
}

__device__ __forceinline__ void wr_compact(uint8_t* o, uint64_t& pos, uint32_t v, uint32_t width) {
  if (width == 1) {
    o[pos++] = (uint8_t)v;
  } else {
    o[pos] = (uint8_t)((v >> 24) | 0x80u);
    o[pos + 1] = (uint8_t)(v >> 16);
    o[pos + 2] = (uint8_t)(v >> 8);
    o[pos + 3] = (uint8_t)v;
    pos += 4;
  }
}

// pass 2: every record at its exclusive-scan offset
__global__ __launch_bounds__(256) void codec_var_encode(uint8_t* __restrict__ out, uint64_t n, int nf, VarMap m,
                                                        const uint32_t* __restrict__ units,
                                                        const int64_t* __restrict__ offs) {
  for (uint64_t r = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; r < n; r += (uint64_t)gridDim.x * blockDim.x) {
    uint64_t pos = (uint64_t)offs[r];
    int sf = 0;
    for (int f = 0; f < nf; ++f) {
      const uint32_t sz = m.size[f];
      if (sz) {
        const uint8_t* c = m.col[f] + r * sz;
        for (uint32_t k = 0; k < sz; ++k) out[pos + k] = c[k];
        pos += sz;
      } else {
        const int64_t off = reinterpret_cast<const int64_t*>(m.col[f])[r];
        const uint64_t nb = (uint64_t)m.len[f][r];
        const uint32_t u = units[(uint64_t)sf * n + r];
        wr_compact(out, pos, u, compact_size(u));
        wr_compact(out, pos, (uint32_t)nb, compact_size((u + 1) * 3));
        const uint8_t* s = m.heap[f] + off;
        for (uint64_t k = 0; k < nb; ++k) out[pos + k] = s[k];
        pos += nb;
        ++sf;
      }
    }
  }
}

int fill_varmap(VarMap* m, int nf, const uint32_t* sizes, uint8_t* const* cols, int64_t* const* lens,
                const uint8_t* const* heaps) {
  if (nf < 1 || nf > kMaxFields) return 1;
  for (int f = 0; f < nf; ++f) {
    m->size[f] = sizes[f];
    m->col[f] = cols[f];
    m->len[f] = sizes[f] ? nullptr : lens[f];
    m->heap[f] = (sizes[f] || !heaps) ? nullptr : heaps[f];
    if (!sizes[f] && !lens[f]) return 1;
  }
  return 0;
}
}  // namespace

// buf: nbytes of a record stream in HBM; block_off: nblocks int64 (device) offsets of records
// 0, B, 2B, ...; n records.  sizes[f] = bytes of fixed field f or 0 for a string field; cols[f]
// = the fixed column or the int64 offsets column; lens[f] = int64 lengths column (strings).
// *err (device u32, zeroed) is set when a block does not parse to the next block's offset.
DR_API int dr_codec_var_decode(const uint8_t* buf, uint64_t nbytes, const int64_t* block_off, uint64_t nblocks,
                               uint32_t B, uint64_t n, int nf, const uint32_t* sizes, uint8_t* const* cols,
                               int64_t* const* lens, uint32_t* err, hipStream_t s) {
  VarMap m;
  if (B == 0 || fill_varmap(&m, nf, sizes, cols, lens, nullptr)) return (int)hipErrorInvalidValue;
  if (nblocks == 0) return 0;
  codec_var_decode<<<grid_for(nblocks, 256, 8192), 256, 0, s>>>(buf, nbytes, block_off, nblocks, B, n, nf, m, err);
  DR_LAUNCH_CHECK();
  return 0;
}

// Pass 1 of the encoder: units (uint32 [#string fields][n]) and record sizes (int64 [n]).
DR_API int dr_codec_var_sizes(uint64_t n, int nf, const uint32_t* sizes, uint8_t* const* cols, int64_t* const* lens,
                              const uint8_t* const* heaps, uint32_t* units, int64_t* rec_sizes, hipStream_t s) {
  VarMap m;
  if (fill_varmap(&m, nf, sizes, cols, lens, heaps)) return (int)hipErrorInvalidValue;
  if (n == 0) return 0;
  codec_var_sizes<<<grid_for(n, 256, 16384), 256, 0, s>>>(n, nf, m, units, rec_sizes);
  DR_LAUNCH_CHECK();
  return 0;
}

// Pass 2: records written at offs (int64 [n], exclusive scan of the sizes) into out.
DR_API int dr_codec_var_encode(uint8_t* out, uint64_t n, int nf, const uint32_t* sizes, uint8_t* const* cols,
                               int64_t* const* lens, const uint8_t* const* heaps, const uint32_t* units,
                               const int64_t* offs, hipStream_t s) {
  VarMap m;
  if (fill_varmap(&m, nf, sizes, cols, lens, heaps)) return (int)hipErrorInvalidValue;
  if (n == 0) return 0;
  codec_var_encode<<<grid_for(n, 256, 16384), 256, 0, s>>>(out, n, nf, m, units, offs);
  DR_LAUNCH_CHECK();
  return 0;
}
