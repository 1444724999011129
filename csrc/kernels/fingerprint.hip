// Rabin 64-bit fingerprints on the device.
//
// Reference: LinqToDryad/Hash64.cs:29-352 and classlib DrFPrint.cpp compute Rabin fingerprints
// over GF(2) with the DryadLINQ polynomial; the host twin is csrc/runtime/codec.cpp Rabin64.  The
// device kernels give bit-identical results to Rabin64::extend(empty, bytes):
//
//   dr_rabin_strings : one fingerprint per (heap, off, len) string (text lines, string fields)
//   dr_rabin_rows    : one fingerprint per fixed-width row slice rows[i, off:off+width]
//   dr_str_pairs_differ : 1 if any pair (A[ia[i]], B[ib[i]]) of strings differs — the collision
//                      check behind fingerprint grouping and joins
//
// The eight 256-entry slicing tables (16 KB) are staged in LDS once per workgroup; each lane
// folds eight bytes per step (tab[7..0] lookups, the word-wise identity of extend_u64), then the
// tail byte by byte with tab[0].  Lookups are data dependent so LDS bank conflicts are random;
// the kernels are bound by the scattered heap reads, not the table.
#include "common.h"

namespace {

constexpr int kTabWords = 8 * 256;

__device__ __forceinline__ void load_tables(const uint64_t* __restrict__ g, uint64_t* s) {
  for (int i = threadIdx.x; i < kTabWords; i += blockDim.x) s[i] = g[i];
  __syncthreads();
}

__device__ __forceinline__ uint64_t fold8(const uint64_t* __restrict__ tab, uint64_t fp, uint64_t v) {
  fp ^= v;
  uint64_t r = 0;
#pragma unroll
  for (int b = 0; b < 8; ++b) r ^= tab[(7 - b) * 256 + ((fp >> (8 * b)) & 0xFF)];
  return r;
}

__device__ __forceinline__ uint64_t load_le8(const uint8_t* p) {
  // unaligned little-endian 8-byte load assembled from bytes (heap offsets are arbitrary)
  uint64_t v = 0;
#pragma unroll
  for (int k = 0; k < 8; ++k) v |= (uint64_t)p[k] << (8 * k);
  return v;
}

__device__ __forceinline__ uint64_t rabin_bytes(const uint64_t* __restrict__ tab, uint64_t fp, const uint8_t* p,
                                                int64_t L) {
  int64_t k = 0;
  if ((((uintptr_t)p) & 7) == 0) {
    for (; k + 8 <= L; k += 8) fp = fold8(tab, fp, *reinterpret_cast<const uint64_t*>(p + k));
  } else {
    for (; k + 8 <= L; k += 8) fp = fold8(tab, fp, load_le8(p + k));
  }
  for (; k < L; ++k) fp = (fp >> 8) ^ tab[(fp & 0xFF) ^ p[k]];
  return fp;
}

__global__ __launch_bounds__(256) void rabin_strings_kernel(const uint8_t* __restrict__ heap,
                                                            const int64_t* __restrict__ off,
                                                            const int64_t* __restrict__ len, uint64_t n,
                                                            const uint64_t* __restrict__ gtab, uint64_t init,
                                                            int64_t* __restrict__ out) {
  __shared__ uint64_t tab[kTabWords];
  load_tables(gtab, tab);
  for (uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (uint64_t)gridDim.x * blockDim.x)
    out[i] = (int64_t)rabin_bytes(tab, init, heap + off[i], len[i]);
}

__global__ __launch_bounds__(256) void rabin_rows_kernel(const uint8_t* __restrict__ rows, uint64_t n, uint32_t stride,
                                                         uint32_t col, uint32_t width,
                                                         const uint64_t* __restrict__ gtab, uint64_t init,
                                                         int64_t* __restrict__ out) {
  __shared__ uint64_t tab[kTabWords];
  load_tables(gtab, tab);
  for (uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (uint64_t)gridDim.x * blockDim.x)
    out[i] = (int64_t)rabin_bytes(tab, init, rows + i * stride + col, width);
}

__global__ __launch_bounds__(256) void str_pairs_differ_kernel(
    const uint8_t* __restrict__ ha, const int64_t* __restrict__ offa, const int64_t* __restrict__ lena,
    const int64_t* __restrict__ ia, const uint8_t* __restrict__ hb, const int64_t* __restrict__ offb,
    const int64_t* __restrict__ lenb, const int64_t* __restrict__ ib, uint64_t n, int32_t* __restrict__ bad) {
  for (uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (uint64_t)gridDim.x * blockDim.x) {
    const int64_t a = ia ? ia[i] : (int64_t)i;
    const int64_t b = ib[i];
    if (ha == hb && offa == offb && a == b) continue;
    const int64_t L = lena[a];
    bool diff = lenb[b] != L;
    const uint8_t* pa = ha + offa[a];
    const uint8_t* pb = hb + offb[b];
    for (int64_t k = 0; !diff && k < L; ++k) diff = pa[k] != pb[k];
    if (diff) atomicOr(bad, 1);
  }
}

inline unsigned blocks_for(uint64_t n) {
  // grid-stride; the table load is amortised over many items per workgroup
  uint64_t b = (n + 255) / 256;
  return (unsigned)(b < 4096 ? (b ? b : 1) : 4096);
}

}  // namespace

DR_API int dr_rabin_strings(const uint8_t* heap, const int64_t* off, const int64_t* len, uint64_t n,
                            const uint64_t* tables, uint64_t init, int64_t* out, hipStream_t s) {
  if (n == 0) return 0;
  rabin_strings_kernel<<<blocks_for(n), 256, 0, s>>>(heap, off, len, n, tables, init, out);
  DR_LAUNCH_CHECK();
  return 0;
}

DR_API int dr_rabin_rows(const uint8_t* rows, uint64_t n, uint32_t stride, uint32_t col, uint32_t width,
                         const uint64_t* tables, uint64_t init, int64_t* out, hipStream_t s) {
  if (n == 0) return 0;
  rabin_rows_kernel<<<blocks_for(n), 256, 0, s>>>(rows, n, stride, col, width, tables, init, out);
  DR_LAUNCH_CHECK();
  return 0;
}

DR_API int dr_str_pairs_differ(const uint8_t* ha, const int64_t* offa, const int64_t* lena, const int64_t* ia,
                               const uint8_t* hb, const int64_t* offb, const int64_t* lenb, const int64_t* ib,
                               uint64_t n, int32_t* bad, hipStream_t s) {
  if (n == 0) return 0;
  str_pairs_differ_kernel<<<grid_for(n, 256, 16384), 256, 0, s>>>(ha, offa, lena, ia, hb, offb, lenb, ib, n, bad);
  DR_LAUNCH_CHECK();
  return 0;
}
