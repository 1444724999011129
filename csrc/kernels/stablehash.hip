// Device image of the host partitioner hash (dryad_amd/runtime/vertex_ops.py stable_hash):
// HashPartition and every keyed shuffle must send a key to the same consumer whether the
// producing vertex ran on the device or fell back to the host, and whatever column width a
// partition inferred for itself (int32 vs int64, float32 vs float64).  So the device hashes the
// key VALUE exactly as the host does:
//
//   bool            -> 1 / 0
//   integer         -> fmix(two's-complement 64-bit image)   (any width: widened first)
//   float           -> integral and |v| < 2^63 ? fmix((int64)v) : FNV-1a-64 of the 8 LE bytes of
//                      the double (NaN canonicalised to 0x7FF8000000000000; -0.0 is integral 0)
//   bytes / string  -> FNV-1a-64 of the bytes (strings are UTF-8 in the heap)
//   tuple / record  -> h = 0x345678; h = (h ^ H(x)) * 1000003 for every field
//
// port = (h & 0x7FFFFFFF) % nparts  (reference DryadLinqVertex.cs:4788-4907).  The launcher
// writes E128 entries {lo = row index, hi = port} ready for the stable partition pass(es).
#include "common.h"

namespace {

enum HKind : int {
  H_U8 = 0, H_I8 = 1, H_BOOL = 2, H_I16 = 3, H_U16 = 4, H_I32 = 5, H_U32 = 6, H_I64 = 7, H_U64 = 8, H_F32 = 9,
  H_F64 = 10, H_BYTES = 20, H_STR = 21
};

constexpr uint64_t kFnvOff = 0xCBF29CE484222325ull;
constexpr uint64_t kFnvPrime = 0x100000001B3ull;
constexpr int kMaxHashCols = 8;

struct HashCol {
  const void* p;          // column data | rows base | string heap
  const int64_t* off;     // H_STR: byte offset per record
  const int64_t* len;     // H_STR: byte length per record
  uint32_t stride;        // H_BYTES: row stride
  uint32_t boff;          // H_BYTES: field offset in the row
  uint32_t blen;          // H_BYTES: field length
  int kind;
};

struct HashSpec {
  HashCol c[kMaxHashCols];
  int ncols;
  int tuple_form;         // 1: key is a tuple / record of the columns, 0: a single value
};

__device__ __forceinline__ uint64_t fmix_int(uint64_t x) {
  x ^= x >> 33;
  x *= 0xFF51AFD7ED558CCDull;
  x ^= x >> 33;
  return x;
}

__device__ __forceinline__ uint64_t fnv_u64le(uint64_t v) {
  uint64_t h = kFnvOff;
#pragma unroll
  for (int b = 0; b < 8; ++b) h = (h ^ ((v >> (8 * b)) & 0xFF)) * kFnvPrime;
  return h;
}

__device__ __forceinline__ uint64_t fnv_bytes(const uint8_t* p, uint64_t n) {
  uint64_t h = kFnvOff;
  for (uint64_t i = 0; i < n; ++i) h = (h ^ p[i]) * kFnvPrime;
  return h;
}

__device__ __forceinline__ uint64_t hash_double(double v) {
  if (v != v) return fnv_u64le(0x7FF8000000000000ull);
  if (__builtin_isfinite(v) && __builtin_fabs(v) < 9.2233720368547758e18 && v == __builtin_trunc(v))
    return fmix_int((uint64_t)(int64_t)v);
  return fnv_u64le((uint64_t)__double_as_longlong(v));
}

__device__ __forceinline__ uint64_t hash_one(const HashCol& c, uint64_t i) {
  switch (c.kind) {
    case H_BOOL: return ((const uint8_t*)c.p)[i] ? 1ull : 0ull;
    case H_U8: return fmix_int(((const uint8_t*)c.p)[i]);
    case H_I8: return fmix_int((uint64_t)(int64_t)((const int8_t*)c.p)[i]);
    case H_I16: return fmix_int((uint64_t)(int64_t)((const int16_t*)c.p)[i]);
    case H_U16: return fmix_int(((const uint16_t*)c.p)[i]);
    case H_I32: return fmix_int((uint64_t)(int64_t)((const int32_t*)c.p)[i]);
    case H_U32: return fmix_int(((const uint32_t*)c.p)[i]);
    case H_I64: case H_U64: return fmix_int(((const uint64_t*)c.p)[i]);
    case H_F32: return hash_double((double)((const float*)c.p)[i]);
    case H_F64: return hash_double(((const double*)c.p)[i]);
    case H_BYTES: return fnv_bytes((const uint8_t*)c.p + i * (uint64_t)c.stride + c.boff, c.blen);
    case H_STR: return fnv_bytes((const uint8_t*)c.p + c.off[i], (uint64_t)c.len[i]);
  }
  return 0;
}

__global__ __launch_bounds__(256) void stable_hash_dest_kernel(HashSpec spec, uint64_t n, uint32_t nparts,
                                                               E128* __restrict__ out, int64_t* __restrict__ hout,
                                                               uint8_t* __restrict__ pout) {
  for (uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (uint64_t)gridDim.x * blockDim.x) {
    uint64_t h;
    if (spec.tuple_form) {
      h = 0x345678ull;
      for (int c = 0; c < spec.ncols; ++c) h = (h ^ hash_one(spec.c[c], i)) * 1000003ull;
    } else {
      h = hash_one(spec.c[0], i);
    }
    if (hout) hout[i] = (int64_t)h;
    if (out) {
      E128 e;
      e.lo = i;
      e.hi = (nparts ? (h & 0x7FFFFFFFull) % nparts : 0);
      out[i] = e;
    }
    if (pout) pout[i] = (uint8_t)(nparts ? (h & 0x7FFFFFFFull) % nparts : 0);
  }
}

}  // namespace

// kinds/ptrs describe up to 8 key columns (see HashCol); nparts = 0 only returns the hashes.
// out: E128 {row, port} entries; pout (nparts <= 256): one port byte per row; either may be null.
DR_API int dr_stable_hash_dest(const int* kinds, const void* const* ptrs, const int64_t* const* offs,
                               const int64_t* const* lens, const uint32_t* strides, const uint32_t* boffs,
                               const uint32_t* blens, int ncols, int tuple_form, uint64_t n, uint32_t nparts,
                               E128* out, int64_t* hout, uint8_t* pout, hipStream_t s) {
  if (ncols < 1 || ncols > kMaxHashCols || (!tuple_form && ncols != 1)) return (int)hipErrorInvalidValue;
  if (pout && (nparts == 0 || nparts > 256)) return (int)hipErrorInvalidValue;
  if (nparts > 0x7FFFFFFFu) return (int)hipErrorInvalidValue;
  HashSpec spec{};
  for (int c = 0; c < ncols; ++c) {
    HashCol& h = spec.c[c];
    h.kind = kinds[c];
    h.p = ptrs[c];
    h.off = offs ? offs[c] : nullptr;
    h.len = lens ? lens[c] : nullptr;
    h.stride = strides ? strides[c] : 0;
    h.boff = boffs ? boffs[c] : 0;
    h.blen = blens ? blens[c] : 0;
    if (h.kind == H_STR && (!h.off || !h.len)) return (int)hipErrorInvalidValue;
    if (h.kind == H_BYTES && h.boff + h.blen > h.stride) return (int)hipErrorInvalidValue;
  }
  spec.ncols = ncols;
  spec.tuple_form = tuple_form;
  if (n == 0) return 0;
  stable_hash_dest_kernel<<<grid_for(n, 256, 16384), 256, 0, s>>>(spec, n, nparts, out, hout, pout);
  DR_LAUNCH_CHECK();
  return 0;
}
