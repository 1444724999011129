// Shared device helpers for the Dryad-AMD CDNA4 (gfx950) kernel library.
//
// Every kernel in csrc/kernels is written for 64-lane wavefronts (CDNA4), 256-thread workgroups
// (4 waves, one per SIMD), and launched through an extern "C" launcher that takes raw device
// pointers plus a hipStream_t so the Python side (ctypes over torch tensors) can call it without
// any torch C++ dependency.
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

#define DR_API extern "C" __attribute__((visibility("default")))

// 128-bit sort entry: `hi` holds the most significant key bits, `lo` the rest of the key in its
// top bits and (usually) a 32-bit row index in its low bits.  The composite sort key is
// (hi << 64 | lo); radix digits are always byte aligned.
struct __attribute__((aligned(16))) E128 {
  uint64_t lo;
  uint64_t hi;
};

// 64-bit sort entry of the compact row sort: a 32-bit window of the key (the 32 key bits right
// below the common prefix of all keys) in the high word, a 32-bit row index in the low word.
struct __attribute__((aligned(8))) E64 {
  uint64_t v;
};

// 256-bit sort entry: an E128 key (same digit layout) carrying two more payload words, so a sort
// can move up to three 8-byte values with the key instead of leaving a row permutation to gather
// through (GroupBy with decomposable aggregates: sequential segmented reduction afterwards).
struct __attribute__((aligned(16))) E256 {
  uint64_t lo;
  uint64_t hi;
  uint64_t p0;
  uint64_t p1;
};

// 320-bit variant (four payload words) for the final stage of a distributed GroupBy, whose
// partial counts are one more column to fold.
struct __attribute__((aligned(8))) E320 {
  uint64_t lo;
  uint64_t hi;
  uint64_t p0;
  uint64_t p1;
  uint64_t p2;
};

static constexpr int kWave = 64;
static constexpr int kBlock = 256;

__device__ __forceinline__ int lane_id() { return threadIdx.x & 63; }
__device__ __forceinline__ int wave_id() { return threadIdx.x >> 6; }

// Number of set bits of `mask` in lanes strictly below the calling lane (v_mbcnt pair).
__device__ __forceinline__ uint32_t popc_below(uint64_t mask) {
  return __builtin_amdgcn_mbcnt_hi((uint32_t)(mask >> 32),
                                   __builtin_amdgcn_mbcnt_lo((uint32_t)mask, 0u));
}

__device__ __forceinline__ uint64_t ballot64(bool p) { return __ballot(p); }

// Inclusive wave-level scan (64 lanes) of a 32-bit value.
__device__ __forceinline__ uint32_t wave_inclusive_scan(uint32_t v) {
  const int l = lane_id();
#pragma unroll
  for (int d = 1; d < 64; d <<= 1) {
    uint32_t o = __shfl_up(v, d, 64);
    if (l >= d) v += o;
  }
  return v;
}

__device__ __forceinline__ uint64_t wave_inclusive_scan64(uint64_t v) {
  const int l = lane_id();
#pragma unroll
  for (int d = 1; d < 64; d <<= 1) {
    uint64_t o = __shfl_up(v, d, 64);
    if (l >= d) v += o;
  }
  return v;
}

__device__ __forceinline__ uint64_t wave_sum64(uint64_t v) {
#pragma unroll
  for (int d = 32; d >= 1; d >>= 1) v += __shfl_xor(v, d, 64);
  return v;
}

__device__ __forceinline__ uint32_t wave_sum32(uint32_t v) {
#pragma unroll
  for (int d = 32; d >= 1; d >>= 1) v += __shfl_xor(v, d, 64);
  return v;
}

// Exclusive scan across a 256-thread block. `scratch` must hold 4 words of LDS.
// Returns the exclusive prefix; `total` receives the block sum.
__device__ __forceinline__ uint32_t block_exclusive_scan256(uint32_t v, uint32_t* scratch,
                                                            uint32_t& total) {
  const int w = wave_id(), l = lane_id();
  uint32_t inc = wave_inclusive_scan(v);
  if (l == 63) scratch[w] = inc;
  __syncthreads();
  uint32_t w0 = scratch[0], w1 = scratch[1], w2 = scratch[2], w3 = scratch[3];
  uint32_t base = (w > 0 ? w0 : 0) + (w > 1 ? w1 : 0) + (w > 2 ? w2 : 0);
  total = w0 + w1 + w2 + w3;
  __syncthreads();
  return base + inc - v;
}

__device__ __forceinline__ uint32_t bswap32(uint32_t x) { return __builtin_bswap32(x); }

// splitmix64 finaliser: the counter-based generator used by synthetic stores.
__device__ __host__ __forceinline__ uint64_t mix64(uint64_t z) {
  z += 0x9E3779B97F4A7C15ull;
  z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ull;
  z = (z ^ (z >> 27)) * 0x94D049BB133111EBull;
  return z ^ (z >> 31);
}

// x mod d for any 64-bit x, given m = ~0ull / d (host-precomputed): q = mulhi(x, m) undershoots
// the true quotient by at most one, so a single correction makes the result exact.
__device__ __forceinline__ uint64_t fast_mod64(uint64_t x, uint64_t d, uint64_t m) {
  const uint64_t q = __umul64hi(x, m);
  const uint64_t r = x - q * d;
  return r >= d ? r - d : r;
}

// Grid sizing for streaming kernels: enough workgroups to fill 256 CUs several times over.
static inline unsigned grid_for(uint64_t work_items, unsigned per_block, unsigned cap = 8192) {
  uint64_t g = (work_items + per_block - 1) / per_block;
  if (g < 1) g = 1;
  if (g > cap) g = cap;
  return (unsigned)g;
}

#define DR_LAUNCH_CHECK()                                     \
  do {                                                        \
    hipError_t _e = hipGetLastError();                        \
    if (_e != hipSuccess) return (int)_e;                     \
  } while (0)
