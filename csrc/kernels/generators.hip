// Synthetic columnar stores for the secondary BASELINE configs (GroupBy-Aggregate, hash join).
//
// gen://records64: 64-byte records = 8 int64 fields (Key, V1..V7), record i of a global table:
//   Key = mix64(seed ^ (i * G)) % nkeys            (uniform keys; nkeys sets the group count)
//   Vj  = mix64((seed + j * H) ^ i) >> 33           (non-negative 31-bit values: sums of 2^32
//                                                    records cannot overflow int64)
// gen://records64?...&mode=dim: a "dimension table" whose keys are a bijection of [0, nkeys)
//   Key = (i * A + seed) % nkeys   (A odd, coprime with nkeys — the caller picks it)
//   Vj  = mix64((seed + j * H) ^ Key) >> 33        (payload is a function of the key, so a join's
//                                                    expected result can be computed from the probe
//                                                    side alone)
// Counter based, so every rank materialises exactly its slice in HBM and a re-executed input
// vertex regenerates identical data.  models/records_cpu.py is the numpy twin.
#include "common.h"

namespace {
constexpr uint64_t kG = 0x9E3779B97F4A7C15ull;
constexpr uint64_t kH = 0xD1B54A32D192ED03ull;

__global__ __launch_bounds__(256) void gen_records64_kernel(int64_t* const* __restrict__ cols, int ncols, uint64_t n,
                                                            uint64_t first, uint64_t nkeys, uint64_t mkeys,
                                                            uint64_t seed, uint64_t dim_mult, bool wide) {
  for (uint64_t r = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; r < n; r += (uint64_t)gridDim.x * blockDim.x) {
    const uint64_t i = first + r;
    if (dim_mult) {
      const uint64_t key = wide ? (uint64_t)(((unsigned __int128)i * dim_mult + seed) % nkeys)
                                : fast_mod64(i * dim_mult + seed, nkeys, mkeys);
      cols[0][r] = (int64_t)key;
      for (int j = 1; j < ncols; ++j) cols[j][r] = (int64_t)(mix64((seed + (uint64_t)j * kH) ^ key) >> 33);
    } else {
      cols[0][r] = (int64_t)fast_mod64(mix64(seed ^ (i * kG)), nkeys, mkeys);
      for (int j = 1; j < ncols; ++j) cols[j][r] = (int64_t)(mix64((seed + (uint64_t)j * kH) ^ i) >> 33);
    }
  }
}

// Columns, two rows per lane (uniform-key mode): the column pointers are read once into
// registers, the field loop is unrolled (NC a template argument) and each lane writes one 16-byte
// nontemporal store per column (the one-row kernel above re-reads the pointer array and issues
// 8-byte stores in a runtime loop: ~3 TB/s on the GroupBy config's 40 GB).  Columns that are not
// 16-byte aligned take the one-row path (a uniform branch).
typedef unsigned long long u64x2 __attribute__((ext_vector_type(2)));
typedef __attribute__((address_space(1))) u64x2 gu64x2;   // global (not flat) stores
template <int NC>
__global__ __launch_bounds__(256) void gen_records64_pair_kernel(int64_t* const* __restrict__ cols, uint64_t n,
                                                                 uint64_t first, uint64_t nkeys, uint64_t mkeys,
                                                                 uint64_t seed) {
  int64_t* c[NC];
  bool aligned = true;
#pragma unroll
  for (int j = 0; j < NC; ++j) {
    c[j] = cols[j];
    aligned = aligned && ((((uintptr_t)c[j]) & 15) == 0);
  }
  const uint64_t stride = (uint64_t)gridDim.x * blockDim.x;
  const uint64_t t0 = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (!aligned) {
    for (uint64_t r = t0; r < n; r += stride) {
      const uint64_t i = first + r;
      c[0][r] = (int64_t)fast_mod64(mix64(seed ^ (i * kG)), nkeys, mkeys);
#pragma unroll
      for (int j = 1; j < NC; ++j) c[j][r] = (int64_t)(mix64((seed + (uint64_t)j * kH) ^ i) >> 33);
    }
    return;
  }
  const uint64_t pairs = n >> 1;
  for (uint64_t q = t0; q < pairs; q += stride) {
    const uint64_t i = first + 2 * q;
    u64x2 v;
    v.x = fast_mod64(mix64(seed ^ (i * kG)), nkeys, mkeys);
    v.y = fast_mod64(mix64(seed ^ ((i + 1) * kG)), nkeys, mkeys);
    __builtin_nontemporal_store(v, (gu64x2*)(c[0]) + q);
#pragma unroll
    for (int j = 1; j < NC; ++j) {
      const uint64_t h = seed + (uint64_t)j * kH;
      v.x = mix64(h ^ i) >> 33;
      v.y = mix64(h ^ (i + 1)) >> 33;
      __builtin_nontemporal_store(v, (gu64x2*)(c[j]) + q);
    }
  }
  if ((n & 1) && t0 == 0) {                         // the last row of an odd count
    const uint64_t r = n - 1, i = first + r;
    c[0][r] = (int64_t)fast_mod64(mix64(seed ^ (i * kG)), nkeys, mkeys);
#pragma unroll
    for (int j = 1; j < NC; ++j) c[j][r] = (int64_t)(mix64((seed + (uint64_t)j * kH) ^ i) >> 33);
  }
}

// Row-major twin: out[r * ncols + j] (a 64-byte row store when ncols = 8).  One lane per field,
// so a wave writes 8 consecutive 64-byte rows with coalesced 8-byte stores; the key modulo is a
// multiply-high reduction (fast_mod64) instead of a 64- or 128-bit software division.  WIDE: the
// dimension-table product i * dim_mult + seed may pass 2^64 (then 128-bit arithmetic is needed).
template <int NC, bool WIDE>
__global__ __launch_bounds__(256) void gen_records64_rows_kernel(int64_t* __restrict__ out, uint64_t n,
                                                                 uint64_t first, uint64_t nkeys, uint64_t mkeys,
                                                                 uint64_t seed, uint64_t dim_mult) {
  const uint64_t total = n * NC;
  for (uint64_t e = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; e < total; e += (uint64_t)gridDim.x * blockDim.x) {
    const uint64_t r = e / NC;
    const int j = (int)(e - r * NC);
    const uint64_t i = first + r;
    uint64_t v;
    if (dim_mult) {
      uint64_t key;
      if (WIDE) key = (uint64_t)(((unsigned __int128)i * dim_mult + seed) % nkeys);
      else key = fast_mod64(i * dim_mult + seed, nkeys, mkeys);
      v = j == 0 ? key : (mix64((seed + (uint64_t)j * kH) ^ key) >> 33);
    } else {
      v = j == 0 ? fast_mod64(mix64(seed ^ (i * kG)), nkeys, mkeys) : (mix64((seed + (uint64_t)j * kH) ^ i) >> 33);
    }
    out[e] = (int64_t)v;
  }
}
// One row per thread, staged: each thread computes its row's NC fields (the key once, not once
// per field lane) into an LDS image of 256 rows, which the block then streams out with 16-byte
// stores (the per-field-lane kernel above issues eight 8-byte stores per row and recomputes the
// dimension-table key in every lane).
template <int NC, bool WIDE>
__global__ __launch_bounds__(256) void gen_records64_rows_lds_kernel(int64_t* __restrict__ out, uint64_t n,
                                                                     uint64_t first, uint64_t nkeys, uint64_t mkeys,
                                                                     uint64_t seed, uint64_t dim_mult) {
  __shared__ __attribute__((aligned(16))) int64_t img[256 * NC];
  for (uint64_t row0 = (uint64_t)blockIdx.x * 256; row0 < n; row0 += (uint64_t)gridDim.x * 256) {
    const uint32_t rows = (uint32_t)((n - row0) < 256 ? (n - row0) : 256);
    if (threadIdx.x < rows) {
      const uint64_t i = first + row0 + threadIdx.x;
      uint64_t key;
      if (dim_mult) {
        if (WIDE) key = (uint64_t)(((unsigned __int128)i * dim_mult + seed) % nkeys);
        else key = fast_mod64(i * dim_mult + seed, nkeys, mkeys);
      } else {
        key = fast_mod64(mix64(seed ^ (i * kG)), nkeys, mkeys);
      }
      const uint64_t src = dim_mult ? key : i;
      img[threadIdx.x * NC] = (int64_t)key;
#pragma unroll
      for (int j = 1; j < NC; ++j) img[threadIdx.x * NC + j] = (int64_t)(mix64((seed + (uint64_t)j * kH) ^ src) >> 33);
    }
    __syncthreads();
    const uint32_t words = rows * NC;                // int64 words of this block's rows
    int64_t* o = out + row0 * NC;
    if ((words & 1) == 0 && (((uintptr_t)o) & 15) == 0) {
      const uint4* s4 = reinterpret_cast<const uint4*>(img);
      uint4* d4 = reinterpret_cast<uint4*>(o);
      for (uint32_t q = threadIdx.x; q < words / 2; q += 256) d4[q] = s4[q];
    } else {
      for (uint32_t q = threadIdx.x; q < words; q += 256) o[q] = img[q];
    }
    __syncthreads();
  }
}
}  // namespace

// cols: device array of ncols (<= 8) device pointers to int64 columns of length n.
// dim_mult != 0 selects the dimension-table mode (key = (i * dim_mult + seed) % nkeys).
DR_API int dr_gen_records64(int64_t* const* cols, int ncols, uint64_t n, uint64_t first, uint64_t nkeys,
                            uint64_t seed, uint64_t dim_mult, hipStream_t s) {
  if (ncols < 1 || ncols > 8 || nkeys == 0) return (int)hipErrorInvalidValue;
  if (n == 0) return 0;
  if (!dim_mult) {
    const unsigned g = grid_for((n + 1) / 2, 256, 16384);
    switch (ncols) {
#define DR_GEN_PAIR(NCV) \
  case NCV: gen_records64_pair_kernel<NCV><<<g, 256, 0, s>>>(cols, n, first, nkeys, ~0ull / nkeys, seed); break;
      DR_GEN_PAIR(1) DR_GEN_PAIR(2) DR_GEN_PAIR(3) DR_GEN_PAIR(4)
      DR_GEN_PAIR(5) DR_GEN_PAIR(6) DR_GEN_PAIR(7) DR_GEN_PAIR(8)
#undef DR_GEN_PAIR
    }
    DR_LAUNCH_CHECK();
    return 0;
  }
  const unsigned __int128 top = (unsigned __int128)(first + n) * dim_mult + seed;
  gen_records64_kernel<<<grid_for(n, 256, 16384), 256, 0, s>>>(cols, ncols, n, first, nkeys, ~0ull / nkeys, seed,
                                                               dim_mult, dim_mult && (top >> 64) != 0);
  DR_LAUNCH_CHECK();
  return 0;
}

DR_API int dr_gen_records64_rows(int64_t* out, int ncols, uint64_t n, uint64_t first, uint64_t nkeys, uint64_t seed,
                                 uint64_t dim_mult, hipStream_t s) {
  if (ncols < 1 || ncols > 8 || nkeys == 0) return (int)hipErrorInvalidValue;
  if (n == 0) return 0;
  const uint64_t m = ~0ull / nkeys;
  // the dimension-table key needs 128-bit arithmetic once (first + n) * dim_mult + seed can pass 2^64
  const unsigned __int128 top = (unsigned __int128)(first + n) * dim_mult + seed;
  const bool wide = dim_mult && (top >> 64) != 0;
  const bool staged = true;  // LDS-staged rows (the one-lane-per-field kernel is kept for reference)
  const unsigned g = staged ? grid_for(n, 256, 8192) : grid_for(n * (uint64_t)ncols, 256, 16384);
#define DR_GEN_ROWS(NCV)                                                                              \
  do {                                                                                                \
    if (staged) {                                                                                     \
      if (wide) gen_records64_rows_lds_kernel<NCV, true><<<g, 256, 0, s>>>(out, n, first, nkeys, m, seed, dim_mult); \
      else gen_records64_rows_lds_kernel<NCV, false><<<g, 256, 0, s>>>(out, n, first, nkeys, m, seed, dim_mult);    \
    } else if (wide) {                                                                                \
      gen_records64_rows_kernel<NCV, true><<<g, 256, 0, s>>>(out, n, first, nkeys, m, seed, dim_mult); \
    } else {                                                                                          \
      gen_records64_rows_kernel<NCV, false><<<g, 256, 0, s>>>(out, n, first, nkeys, m, seed, dim_mult); \
    }                                                                                                 \
  } while (0)
  switch (ncols) {
    case 1: DR_GEN_ROWS(1); break;
    case 2: DR_GEN_ROWS(2); break;
    case 3: DR_GEN_ROWS(3); break;
    case 4: DR_GEN_ROWS(4); break;
    case 5: DR_GEN_ROWS(5); break;
    case 6: DR_GEN_ROWS(6); break;
    case 7: DR_GEN_ROWS(7); break;
    default: DR_GEN_ROWS(8); break;
  }
#undef DR_GEN_ROWS
  DR_LAUNCH_CHECK();
  return 0;
}
