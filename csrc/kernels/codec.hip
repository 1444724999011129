// Record (de)serialisation on the device (K14): DryadLinqBinary fixed-width records <-> columns.
//
// A record type whose fields are all fixed-width primitives (no strings, no nullable fields)
// serialises as the little-endian fields back to back (reference DryadLinqBinaryWriter.cs
// WriteRawBytes of each primitive; DryadLinqCodeGen.cs:1041-1096 field order), so a partfile
// part of such records is an [n, width] byte matrix.  Decoding = scattering each field's bytes
// into its column (AoS -> SoA), encoding = the reverse; one thread per (record, field).  Bytes
// are moved with byte loads/stores because fields need not be aligned inside the record.
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
  const unsigned g = grid_for(n * (uint64_t)nf, 256, 16384);
  if (direction == 0)
    codec_kernel<true><<<g, 256, 0, s>>>(rows, n, width, nf, m);
  else
    codec_kernel<false><<<g, 256, 0, s>>>(rows, n, width, nf, m);
  DR_LAUNCH_CHECK();
  return 0;
}
