// Columns <-> fixed-width sort rows, for the fine-bucket exchange over columnar tables
// (ops/rowpack.py).  A columnar table sorted by a numeric key is packed into rows whose first bytes
// are the key in byte-comparable form (big-endian, the sign bit flipped; a float's bits fully
// inverted when negative), followed by the other columns' raw bytes; the rows then take the same
// path as any row table (ops/recordsort.distributed_sort_rows: E64 window entries, fine buckets,
// one RCCL all-to-all-v per round, the LDS tile merge), and the received rows are unpacked back
// into columns.  An integer key that is a table column travels only as its key bytes and is
// recovered from them.
//
// Both directions stage 256 rows per workgroup in LDS (<= 32 KB: rows of <= 128 bytes): the
// columns are read and written one element per lane (coalesced across the wave), the rows as
// whole 16-byte pieces of the contiguous row block.
//
// Reference: the reference sorts records of any type through its serialized form
// (DryadLinqVertex.cs:9330-9335, ParallelSort; DryadLinqBinaryWriter.cs record encoding); here
// the record's byte-comparable form is built on the device instead of compared field by field.
#include "common.h"

namespace {

constexpr uint32_t kRpRows = 256;
constexpr uint32_t kRpMaxRec = 128;

// One column of the row layout.  kind: 0 raw little-endian bytes, 1 signed integer as key bytes,
// 2 IEEE float as key bytes, 3 unsigned integer as key bytes.  A key part is its value's ordered
// unsigned form u (order-preserving), less the job-wide minimum `base`, shifted left by `shift`
// so its highest possibly set bit is bit 63, and stored as the top `kbytes` bytes (big-endian):
// the key's leading bytes then carry information (the fine buckets are its top 16..24 bits, which
// a small integer's or a float's raw bits would leave constant), and the part is no wider than
// its value range.  Unpack (flags bit 1) of a key part recovers the integer column from it.
struct RpCol {
  uint64_t ptr;
  uint64_t base;
  uint32_t width;    // 1, 2, 4 or 8 bytes (the column's element)
  uint32_t off;      // byte offset in the row
  uint32_t kind;
  uint32_t flags;    // bit 0: pack writes it; bit 1: unpack writes the column from it
  uint32_t shift;    // 0..63
  uint32_t kbytes;   // 1..8 key bytes
};

__device__ __forceinline__ uint64_t rp_load(const RpCol& c, uint64_t i) {
  const uint8_t* p = reinterpret_cast<const uint8_t*>(c.ptr);
  switch (c.width) {
    case 1: return p[i];
    case 2: return reinterpret_cast<const uint16_t*>(p)[i];
    case 4: return reinterpret_cast<const uint32_t*>(p)[i];
    default: return reinterpret_cast<const uint64_t*>(p)[i];
  }
}

__device__ __forceinline__ void rp_store(const RpCol& c, uint64_t i, uint64_t v) {
  uint8_t* p = reinterpret_cast<uint8_t*>(c.ptr);
  switch (c.width) {
    case 1: p[i] = (uint8_t)v; break;
    case 2: reinterpret_cast<uint16_t*>(p)[i] = (uint16_t)v; break;
    case 4: reinterpret_cast<uint32_t*>(p)[i] = (uint32_t)v; break;
    default: reinterpret_cast<uint64_t*>(p)[i] = v; break;
  }
}

// value (its `w` raw bytes) -> the ordered unsigned integer (same order as the values)
__device__ __forceinline__ uint64_t rp_norm(uint64_t v, uint32_t w, uint32_t kind) {
  const uint64_t sign = 1ull << (8 * w - 1);
  const uint64_t mask = w == 8 ? ~0ull : ((1ull << (8 * w)) - 1);
  v &= mask;
  if (kind == 1) return v ^ sign;
  if (kind == 2) {
    if (v == sign) v = 0;                                          // -0.0 orders as +0.0
    return ((v & sign) ? ~v : (v | sign)) & mask;
  }
  return v;
}

__device__ __forceinline__ uint64_t rp_denorm(uint64_t k, uint32_t w, uint32_t kind) {
  const uint64_t sign = 1ull << (8 * w - 1);
  const uint64_t mask = w == 8 ? ~0ull : ((1ull << (8 * w)) - 1);
  if (kind == 1) return (k ^ sign) & mask;
  if (kind == 2) return ((k & sign) ? (k & ~sign) : ~k) & mask;
  return k & mask;
}

__global__ __launch_bounds__(kRpRows) void rp_pack_kernel(const RpCol* __restrict__ cols, uint32_t ncols, uint64_t n,
                                                          uint32_t rec, uint8_t* __restrict__ out) {
  __shared__ __attribute__((aligned(16))) uint32_t img[kRpRows * kRpMaxRec / 4];
  uint8_t* bimg = reinterpret_cast<uint8_t*>(img);
  const uint32_t t = threadIdx.x;
  const uint32_t rw = rec / 4;
  for (uint64_t row0 = (uint64_t)blockIdx.x * kRpRows; row0 < n; row0 += (uint64_t)gridDim.x * kRpRows) {
    const uint32_t nr = (uint32_t)((n - row0) < kRpRows ? (n - row0) : kRpRows);
    __syncthreads();                               // the previous tile has been stored
    for (uint32_t w = t; w < nr * rw; w += kRpRows) img[w] = 0;       // padding bytes stay zero
    __syncthreads();
    if (t < nr) {
      uint8_t* r = bimg + t * rec;
      for (uint32_t c = 0; c < ncols; ++c) {
        const RpCol col = cols[c];
        if (!(col.flags & 1)) continue;
        const uint64_t v = rp_load(col, row0 + t);
        if (col.kind == 0) {
          for (uint32_t b = 0; b < col.width; ++b) r[col.off + b] = (uint8_t)(v >> (8 * b));
        } else {
          const uint64_t k = (rp_norm(v, col.width, col.kind) - col.base) << col.shift;
          for (uint32_t b = 0; b < col.kbytes; ++b) r[col.off + b] = (uint8_t)(k >> (56 - 8 * b));
        }
      }
    }
    __syncthreads();
    const uint32_t words = nr * rw;
    uint32_t* o = reinterpret_cast<uint32_t*>(out + row0 * rec);
    if ((reinterpret_cast<uintptr_t>(o) & 15) == 0) {
      const uint32_t q = words / 4;
      for (uint32_t i = t; i < q; i += kRpRows)
        reinterpret_cast<uint4*>(o)[i] = reinterpret_cast<const uint4*>(img)[i];
      for (uint32_t i = 4 * q + t; i < words; i += kRpRows) o[i] = img[i];
    } else {
      for (uint32_t i = t; i < words; i += kRpRows) o[i] = img[i];
    }
  }
}

__global__ __launch_bounds__(kRpRows) void rp_unpack_kernel(const uint8_t* __restrict__ rows, const RpCol* __restrict__ cols,
                                                            uint32_t ncols, uint64_t n, uint32_t rec) {
  __shared__ __attribute__((aligned(16))) uint32_t img[kRpRows * kRpMaxRec / 4];
  const uint8_t* bimg = reinterpret_cast<const uint8_t*>(img);
  const uint32_t t = threadIdx.x;
  const uint32_t rw = rec / 4;
  for (uint64_t row0 = (uint64_t)blockIdx.x * kRpRows; row0 < n; row0 += (uint64_t)gridDim.x * kRpRows) {
    const uint32_t nr = (uint32_t)((n - row0) < kRpRows ? (n - row0) : kRpRows);
    const uint32_t words = nr * rw;
    const uint32_t* s = reinterpret_cast<const uint32_t*>(rows + row0 * rec);
    __syncthreads();                               // the previous tile has been read
    if ((reinterpret_cast<uintptr_t>(s) & 15) == 0) {
      const uint32_t q = words / 4;
      for (uint32_t i = t; i < q; i += kRpRows)
        reinterpret_cast<uint4*>(img)[i] = reinterpret_cast<const uint4*>(s)[i];
      for (uint32_t i = 4 * q + t; i < words; i += kRpRows) img[i] = s[i];
    } else {
      for (uint32_t i = t; i < words; i += kRpRows) img[i] = s[i];
    }
    __syncthreads();
    if (t < nr) {
      const uint8_t* r = bimg + t * rec;
      for (uint32_t c = 0; c < ncols; ++c) {
        const RpCol col = cols[c];
        if (!(col.flags & 2)) continue;
        uint64_t v = 0;
        if (col.kind == 0) {
          for (uint32_t b = 0; b < col.width; ++b) v |= (uint64_t)r[col.off + b] << (8 * b);
        } else {
          uint64_t k = 0;
          for (uint32_t b = 0; b < col.kbytes; ++b) k |= (uint64_t)r[col.off + b] << (56 - 8 * b);
          v = rp_denorm((k >> col.shift) + col.base, col.width, col.kind);
        }
        rp_store(col, row0 + t, v);
      }
    }
  }
}

int rp_check(const void* cols, uint32_t ncols, uint32_t rec) {
  if (ncols == 0 || ncols > 64 || rec % 4 || rec < 4 || rec > kRpMaxRec || cols == nullptr)
    return (int)hipErrorInvalidValue;
  return 0;
}

}  // namespace

// Pack `n` rows of `rec` bytes (a multiple of 4, <= 128) into `out` from the columns `cols`
// (device array of RpCol, `ncols` <= 64; every column's bytes lie inside the row, checked by the
// caller, ops/rowpack.py).
DR_API int dr_rows_pack(const void* cols, uint32_t ncols, uint64_t n, uint32_t rec, uint8_t* out, hipStream_t s) {
  const RpCol* c = reinterpret_cast<const RpCol*>(cols);
  if (int e = rp_check(c, ncols, rec)) return e;
  if (n == 0) return 0;
  rp_pack_kernel<<<grid_for(n, kRpRows, 8192), kRpRows, 0, s>>>(c, ncols, n, rec, out);
  DR_LAUNCH_CHECK();
  return 0;
}

// Unpack `n` rows of `rec` bytes into the columns flagged for it.
DR_API int dr_rows_unpack(const uint8_t* rows, const void* cols, uint32_t ncols, uint64_t n, uint32_t rec,
                          hipStream_t s) {
  const RpCol* c = reinterpret_cast<const RpCol*>(cols);
  if (int e = rp_check(c, ncols, rec)) return e;
  if (n == 0) return 0;
  rp_unpack_kernel<<<grid_for(n, kRpRows, 8192), kRpRows, 0, s>>>(rows, c, ncols, n, rec);
  DR_LAUNCH_CHECK();
  return 0;
}
