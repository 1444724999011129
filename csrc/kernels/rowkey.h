// Byte-string keys of fixed-width rows (memcmp order) as a 128-bit big-endian integer, and the
// 32-bit "window" of such a key below a common prefix (the compact sort's entry key).
#pragma once
#include "common.h"

namespace {

__device__ __forceinline__ void load_key128(const uint8_t* r, uint32_t key_len, bool aligned, uint64_t& k0,
                                            uint64_t& k1) {
  uint32_t b[4] = {0, 0, 0, 0};
  if (aligned) {
    const uint32_t* w = reinterpret_cast<const uint32_t*>(r);
    const uint32_t nw = (key_len + 3) >> 2;
    for (uint32_t k = 0; k < nw; ++k) b[k] = bswap32(w[k]);
  } else {
    for (uint32_t k = 0; k < key_len; ++k) b[k >> 2] |= (uint32_t)r[k] << (8 * (3 - (k & 3)));
  }
#pragma unroll
  for (int k = 0; k < 4; ++k) {
    const int bytes = (int)key_len - 4 * k;
    if (bytes <= 0) b[k] = 0;
    else if (bytes < 4) b[k] &= 0xFFFFFFFFu << (8 * (4 - bytes));
  }
  k0 = ((uint64_t)b[0] << 32) | b[1];
  k1 = ((uint64_t)b[2] << 32) | b[3];
}

// window = composite key bits [P, P + 32) counted from the most significant end
__device__ __forceinline__ uint32_t key_window(uint64_t k0, uint64_t k1, uint32_t P) {
  const unsigned __int128 k = ((unsigned __int128)k0 << 64) | k1;
  return P >= 128 ? 0u : (uint32_t)((k << P) >> 96);
}

}  // namespace
