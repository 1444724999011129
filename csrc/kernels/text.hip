// Text kernels: LineRecord splitting and WordCount tokenisation on the device (K15).
//
// Reference: LineRecord reading splits a byte stream at '\n' (DryadLinqTextReader, LineRecord.cs)
// and WordCount-style jobs tokenise with String.Split + GroupBy.  Here a partition's text is one
// byte heap in HBM; lines / tokens are (offset, length) pairs found by byte classification +
// stream compaction, and words are grouped by a 64-bit hash (radix sort) with a byte-exact
// collision check against each group's representative.
//   dr_text_marks     : per byte, bit0 = line start, bit1 = token start, bit2 = token end
//   dr_token_hash     : FNV-1a-64 then mix64 of each (off, len) token
//   dr_token_verify   : 1 where a token differs from its group's representative (hash collision)
#include "common.h"

namespace {

__device__ __forceinline__ bool is_space(uint8_t c) { return c == ' ' || c == '\t' || c == '\n' || c == '\r'; }

__global__ __launch_bounds__(256) void text_marks_kernel(const uint8_t* __restrict__ buf, uint64_t n,
                                                         uint8_t* __restrict__ marks) {
  for (uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (uint64_t)gridDim.x * blockDim.x) {
    const uint8_t c = buf[i];
    const uint8_t p = i ? buf[i - 1] : (uint8_t)'\n';
    const uint8_t q = (i + 1 < n) ? buf[i + 1] : (uint8_t)'\n';
    uint8_t m = 0;
    // a line starts at 0 and after every "\n", "\r\n" or lone "\r" (DryadLinqTextReader.cs:217-240)
    if (p == '\n' || (p == '\r' && c != '\n')) m |= 1;
    if (!is_space(c) && is_space(p)) m |= 2;
    if (!is_space(c) && is_space(q)) m |= 4;
    marks[i] = m;
  }
}

__global__ __launch_bounds__(256) void token_hash_kernel(const uint8_t* __restrict__ buf, const int64_t* __restrict__ off,
                                                         const int64_t* __restrict__ len, uint64_t nt,
                                                         int64_t* __restrict__ out) {
  for (uint64_t t = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; t < nt; t += (uint64_t)gridDim.x * blockDim.x) {
    const uint8_t* s = buf + off[t];
    const int64_t L = len[t];
    uint64_t h = 0xCBF29CE484222325ull;
    for (int64_t k = 0; k < L; ++k) h = (h ^ s[k]) * 0x100000001B3ull;
    out[t] = (int64_t)mix64(h ^ (uint64_t)L);
  }
}

// rep[t] = token index of t's group representative; out[t] = 1 if bytes differ
__global__ __launch_bounds__(256) void token_verify_kernel(const uint8_t* __restrict__ buf, const int64_t* __restrict__ off,
                                                           const int64_t* __restrict__ len, const int64_t* __restrict__ rep,
                                                           uint64_t nt, int32_t* __restrict__ bad) {
  for (uint64_t t = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; t < nt; t += (uint64_t)gridDim.x * blockDim.x) {
    const int64_t r = rep[t];
    if (r == (int64_t)t) continue;
    const int64_t L = len[t];
    bool diff = len[r] != L;
    for (int64_t k = 0; !diff && k < L; ++k) diff = buf[off[t] + k] != buf[off[r] + k];
    if (diff) atomicOr(bad, 1);
  }
}

// mode 0: s == pat, 1: s.startswith(pat), 2: s.endswith(pat), 3: pat in s (substring)
__global__ __launch_bounds__(256) void str_match_kernel(const uint8_t* __restrict__ heap, const int64_t* __restrict__ off,
                                                        const int64_t* __restrict__ len, uint64_t n,
                                                        const uint8_t* __restrict__ pat, int64_t plen, int mode,
                                                        bool* __restrict__ out) {
  for (uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (uint64_t)gridDim.x * blockDim.x) {
    const uint8_t* s = heap + off[i];
    const int64_t L = len[i];
    bool ok;
    if (mode == 0 || mode == 1 || mode == 2) {
      ok = (mode == 0) ? (L == plen) : (L >= plen);
      const int64_t base = (mode == 2) ? L - plen : 0;
      for (int64_t k = 0; ok && k < plen; ++k) ok = s[base + k] == pat[k];
    } else {
      ok = false;
      for (int64_t st = 0; !ok && st + plen <= L; ++st) {
        bool m = true;
        for (int64_t k = 0; m && k < plen; ++k) m = s[st + k] == pat[k];
        ok = m;
      }
    }
    out[i] = ok;
  }
}

}  // namespace

DR_API int dr_str_match(const uint8_t* heap, const int64_t* off, const int64_t* len, uint64_t n, const uint8_t* pat,
                        int64_t plen, int mode, bool* out, hipStream_t s) {
  if (n == 0) return 0;
  str_match_kernel<<<grid_for(n, 256, 16384), 256, 0, s>>>(heap, off, len, n, pat, plen, mode, out);
  DR_LAUNCH_CHECK();
  return 0;
}

DR_API int dr_text_marks(const uint8_t* buf, uint64_t n, uint8_t* marks, hipStream_t s) {
  if (n == 0) return 0;
  text_marks_kernel<<<grid_for(n, 256, 16384), 256, 0, s>>>(buf, n, marks);
  DR_LAUNCH_CHECK();
  return 0;
}

DR_API int dr_token_hash(const uint8_t* buf, const int64_t* off, const int64_t* len, uint64_t nt, int64_t* out,
                         hipStream_t s) {
  if (nt == 0) return 0;
  token_hash_kernel<<<grid_for(nt, 256, 16384), 256, 0, s>>>(buf, off, len, nt, out);
  DR_LAUNCH_CHECK();
  return 0;
}

DR_API int dr_token_verify(const uint8_t* buf, const int64_t* off, const int64_t* len, const int64_t* rep, uint64_t nt,
                           int32_t* bad, hipStream_t s) {
  if (nt == 0) return 0;
  token_verify_kernel<<<grid_for(nt, 256, 16384), 256, 0, s>>>(buf, off, len, rep, nt, bad);
  DR_LAUNCH_CHECK();
  return 0;
}

namespace {

// Strings laid inline into fixed-width rows (the grace join's packed rows, runtime/grace_stage.py):
// one wave per 64 rows, each lane copying one row's string byte by byte (strings are short: the
// caller caps them at max_len); the destination bytes past a string stay as they were (zero).
__global__ __launch_bounds__(256) void scatter_strings_kernel(const uint8_t* __restrict__ heap,
                                                              const int64_t* __restrict__ off,
                                                              const int64_t* __restrict__ len, uint64_t n,
                                                              uint8_t* __restrict__ dst, uint64_t stride,
                                                              uint32_t dst_off, uint32_t max_len,
                                                              uint32_t* __restrict__ overflow) {
  for (uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (uint64_t)gridDim.x * blockDim.x) {
    int64_t L = len[i];
    if (L < 0 || L > (int64_t)max_len) {
      atomicOr(overflow, 1u);
      L = L < 0 ? 0 : (int64_t)max_len;
    }
    const uint8_t* s = heap + off[i];
    uint8_t* d = dst + i * stride + dst_off;
    for (int64_t k = 0; k < L; ++k) d[k] = s[k];
  }
}

}  // namespace

// dst row i (stride bytes apart) gets string i's bytes at dst_off; lengths past max_len are cut
// and flag *overflow (the caller refuses the layout).
DR_API int dr_scatter_strings(const uint8_t* heap, const int64_t* off, const int64_t* len, uint64_t n, uint8_t* dst,
                              uint64_t stride, uint32_t dst_off, uint32_t max_len, uint32_t* overflow,
                              hipStream_t s) {
  if (n == 0) return 0;
  if (dst_off + max_len > stride || overflow == nullptr) return (int)hipErrorInvalidValue;
  scatter_strings_kernel<<<grid_for(n, 256, 16384), 256, 0, s>>>(heap, off, len, n, dst, stride, dst_off, max_len,
                                                                  overflow);
  DR_LAUNCH_CHECK();
  return 0;
}
