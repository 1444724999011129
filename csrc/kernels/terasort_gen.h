// gensort-style TeraSort record generator shared by the generator / validation kernels
// (terasort.hip) and the generate-into-buckets scatter of the distributed sort (sort.hip).
#pragma once
#include "common.h"

namespace dr_ts {

__device__ __forceinline__ uint32_t hex_word(uint64_t g, uint32_t k) {
  // bytes 4k..4k+3 of the 32-hex-digit record number field starting at byte 12 (k in 7..10)
  uint32_t w = 0;
#pragma unroll
  for (int b = 0; b < 4; ++b) {
    const uint32_t q = 4 * k + b - 12;                    // digit index 16..31
    const uint32_t nib = (uint32_t)(g >> (4 * (31 - q))) & 0xF;
    w |= (nib < 10 ? '0' + nib : 'A' + nib - 10) << (8 * b);
  }
  return w;
}

// The two hash words behind record g's 10-byte key: key bytes 0..7 = kA (big-endian), bytes 8..9 =
// the top 16 bits of kB.
__device__ __forceinline__ void ts_key_words(uint64_t seed, uint64_t g, uint64_t& kA, uint64_t& kB) {
  kA = mix64(seed ^ mix64(g));
  kB = mix64(kA ^ 0xD1B54A32D192ED03ull);
}

// The 25 little-endian dwords of record g, computed directly (one hash triple per record).
__device__ __forceinline__ void ts_record(uint64_t seed, uint64_t g, uint32_t* w) {
  uint64_t kA, kB;
  ts_key_words(seed, g, kA, kB);
  const uint64_t fil = mix64(g ^ (seed * 0x2545F4914F6CDD1Dull) ^ 0xF00DF00DF00DF00Dull);
  w[0] = bswap32((uint32_t)(kA >> 32));
  w[1] = bswap32((uint32_t)kA);
  w[2] = (uint32_t)(kB >> 56) | (((uint32_t)(kB >> 48) & 0xFF) << 8) | (0x11u << 24);
  w[3] = w[4] = w[5] = w[6] = 0x30303030u;
#pragma unroll
  for (uint32_t k = 7; k < 11; ++k) w[k] = hex_word(g, k);
  w[11] = 0xBBAA9988u;
#pragma unroll
  for (uint32_t i = 0; i < 12; ++i) w[12 + i] = ('A' + (uint32_t)((fil >> (5 * i)) % 26)) * 0x01010101u;
  w[24] = 0xFFEEDDCCu;
}

}  // namespace dr_ts
