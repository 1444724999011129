// A/B of the row gather of 100-byte records (the receive side of the multi-rank TeraSort and any
// unpitched row table; csrc/kernels/sort.hip gather_fixup_kernel<25> copy phase): out[i] =
// rows[idx[i]] for a pseudo-random bijection idx, 1e9 rows (100 GB in, 100 GB out).
//   dword     lanes copy consecutive dwords of the 256 rows a workgroup owns (production);
//   aligned16 8 lanes per row load the 16-byte-aligned pieces that cover the row (7 or 8 loads,
//             every piece of the window requested before any is used), the row is shifted into
//             place in LDS at the output's 100-byte pitch, then stored as contiguous 16-byte words.
// Build: hipcc --offload-arch=gfx950 -O3 -std=c++17 -I csrc/kernels tools/micro/gather100_ab.hip -o tools/micro/bin/gather100_ab
#include <hip/hip_runtime.h>

#include <cstdio>
#include <cstdlib>

#include "common.h"

namespace {
constexpr uint32_t kRows = 256;
typedef uint32_t u32x4 __attribute__((ext_vector_type(4)));

__global__ void fill(uint32_t* rows, uint64_t words) {
  for (uint64_t i = blockIdx.x * (uint64_t)blockDim.x + threadIdx.x; i < words; i += (uint64_t)gridDim.x * blockDim.x)
    rows[i] = (uint32_t)mix64(i);
}

__global__ void make_idx(uint32_t* idx, uint64_t n, uint64_t a, uint64_t b) {
  for (uint64_t i = blockIdx.x * (uint64_t)blockDim.x + threadIdx.x; i < n; i += (uint64_t)gridDim.x * blockDim.x)
    idx[i] = (uint32_t)((i * a + b) % n);
}

__global__ __launch_bounds__(256) void g_dword(const uint32_t* __restrict__ rows, uint32_t* __restrict__ out,
                                               const uint32_t* __restrict__ idx, uint64_t n) {
  __shared__ uint32_t sidx[kRows];
  const int t = threadIdx.x;
  for (uint64_t c0 = (uint64_t)blockIdx.x * kRows; c0 < n; c0 += (uint64_t)gridDim.x * kRows) {
    const uint32_t L = (uint32_t)(n - c0 < kRows ? n - c0 : kRows);
    if (t < (int)L) sidx[t] = idx[c0 + t];
    __syncthreads();
    const uint32_t words = L * 25;
    uint32_t* o = out + c0 * 25;
    uint32_t j = t;
    for (; j + 3 * 256 < words; j += 4 * 256) {
      uint32_t v[4];
#pragma unroll
      for (int k = 0; k < 4; ++k) {
        const uint32_t jj = j + k * 256, r = jj / 25, c = jj - r * 25;
        v[k] = rows[(uint64_t)sidx[r] * 25 + c];
      }
#pragma unroll
      for (int k = 0; k < 4; ++k) __builtin_nontemporal_store(v[k], o + j + k * 256);
    }
    for (; j < words; j += 256) {
      const uint32_t r = j / 25, c = j - r * 25;
      o[j] = rows[(uint64_t)sidx[r] * 25 + c];
    }
    __syncthreads();
  }
}

__global__ __launch_bounds__(256) void g_aligned16(const uint32_t* __restrict__ rows, uint32_t* __restrict__ out,
                                                   const uint32_t* __restrict__ idx, uint64_t n, uint64_t words_total) {
  __shared__ uint32_t sidx[kRows];
  __shared__ __attribute__((aligned(16))) uint32_t stage[kRows * 25];
  const int t = threadIdx.x, sub = t & 7, grp = t >> 3;     // 32 rows per pass, 8 lanes per row
  const uint4* r4 = reinterpret_cast<const uint4*>(rows);
  const uint64_t pieces_total = (words_total + 3) / 4;
  for (uint64_t c0 = (uint64_t)blockIdx.x * kRows; c0 < n; c0 += (uint64_t)gridDim.x * kRows) {
    const uint32_t L = (uint32_t)(n - c0 < kRows ? n - c0 : kRows);
    if (t < (int)L) sidx[t] = idx[c0 + t];
    __syncthreads();
    // every lane requests its pieces of all 8 row groups first, then places them
    uint4 v[8];
#pragma unroll
    for (int k = 0; k < 8; ++k) {
      const uint32_t r = k * 32 + grp;
      v[k] = make_uint4(0, 0, 0, 0);
      if (r < L) {
        const uint64_t w0 = (uint64_t)sidx[r] * 25;            // first dword of the row
        const uint64_t p = (w0 >> 2) + sub;                      // 16-byte piece of this lane
        if (p * 4 < w0 + 25 && p < pieces_total) v[k] = r4[p];
      }
    }
#pragma unroll
    for (int k = 0; k < 8; ++k) {
      const uint32_t r = k * 32 + grp;
      if (r < L) {
        const uint64_t w0 = (uint64_t)sidx[r] * 25;
        const uint64_t p = (w0 >> 2) + sub;
        const uint32_t vv[4] = {v[k].x, v[k].y, v[k].z, v[k].w};
#pragma unroll
        for (int q = 0; q < 4; ++q) {
          const int64_t wi = (int64_t)(p * 4 + q) - (int64_t)w0;    // dword of the row
          if (wi >= 0 && wi < 25) stage[r * 25 + wi] = vv[q];
        }
      }
    }
    __syncthreads();
    u32x4* o4 = reinterpret_cast<u32x4*>(out + c0 * 25);
    const u32x4* s4 = reinterpret_cast<const u32x4*>(stage);
    const uint32_t pieces = L * 25 / 4;
    for (uint32_t j = t; j < pieces; j += 256) __builtin_nontemporal_store(s4[j], o4 + j);
    for (uint32_t j = pieces * 4 + t; j < L * 25; j += 256) out[c0 * 25 + j] = stage[j];
    __syncthreads();
  }
}

__global__ void diff(const uint32_t* a, const uint32_t* b, uint64_t words, unsigned long long* bad) {
  uint32_t k = 0;
  for (uint64_t i = blockIdx.x * (uint64_t)blockDim.x + threadIdx.x; i < words; i += (uint64_t)gridDim.x * blockDim.x)
    k += a[i] != b[i];
  if (k) atomicAdd(bad, (unsigned long long)k);
}
}  // namespace

#define HC(x)                                                      \
  do {                                                             \
    hipError_t e_ = (x);                                           \
    if (e_ != hipSuccess) {                                        \
      std::fprintf(stderr, "%s: %s\n", #x, hipGetErrorString(e_)); \
      std::exit(1);                                                \
    }                                                              \
  } while (0)

int main(int argc, char** argv) {
  const uint64_t n = argc > 1 ? std::strtoull(argv[1], nullptr, 10) : 1000000000ull;
  const uint64_t words = n * 25;
  uint32_t *rows, *o1, *o2, *idx;
  unsigned long long* bad;
  HC(hipMalloc(&rows, words * 4));
  HC(hipMalloc(&o1, words * 4));
  HC(hipMalloc(&o2, words * 4));
  HC(hipMalloc(&idx, n * 4));
  HC(hipMalloc(&bad, 8));
  fill<<<8192, 256>>>(rows, words);
  make_idx<<<8192, 256>>>(idx, n, 2654435761ull % n | 1, 12345);   // odd multiplier: a bijection when n is even
  HC(hipDeviceSynchronize());
  hipEvent_t a, b;
  HC(hipEventCreate(&a));
  HC(hipEventCreate(&b));
  const unsigned grid = 16384;
  for (int variant = 0; variant < 2; ++variant) {
    float best = 1e9f;
    for (int it = 0; it < 4; ++it) {
      HC(hipEventRecord(a));
      if (variant == 0)
        g_dword<<<grid, 256>>>(rows, o1, idx, n);
      else
        g_aligned16<<<grid, 256>>>(rows, o2, idx, n, words);
      HC(hipEventRecord(b));
      HC(hipEventSynchronize(b));
      float ms;
      HC(hipEventElapsedTime(&ms, a, b));
      if (it > 0 && ms < best) best = ms;
    }
    std::printf("%-10s %.3f ms  %.2f TB/s (in + out)\n", variant == 0 ? "dword" : "aligned16", best,
                2.0 * words * 4 / 1e12 / (best / 1e3));
  }
  HC(hipMemset(bad, 0, 8));
  diff<<<8192, 256>>>(o1, o2, words, bad);
  unsigned long long hb = 0;
  HC(hipMemcpy(&hb, bad, 8, hipMemcpyDeviceToHost));
  std::printf("mismatched words: %llu\n", hb);
  std::fflush(stdout);
  return hb != 0;
}
