// A/B of the look-back radix scatter pass (csrc/kernels/sort.hip os_scatter_kernel) on 1.25e9
// E64 entries: one 8-bit digit pass, the production tile geometry, two ways of ranking a wave's
// entries by digit:
//   lds     per item: LDS atomicOr of the lane bit into a per-(wave, digit) mask, read the mask
//           back (the digit's peers), leader updates the wave's digit counter (production);
//   ballot  per item: the peers mask from 8 ballots of the digit bits (no LDS atomics, no mask
//           reset), leader updates the counter.
// Reports ms per pass and the logical TB/s (8 B read + 8 B written per entry); checks that both
// variants produce the same permutation.
// Build: hipcc --offload-arch=gfx950 -O3 -std=c++17 -I csrc/kernels tools/micro/scatter_ab.hip -o tools/micro/bin/scatter_ab
#include <hip/hip_runtime.h>

#include <cstdio>
#include <cstdlib>
#include <vector>

#include "common.h"

namespace {
constexpr int kBins = 256;
typedef __attribute__((address_space(1))) unsigned long long gu64;
typedef __attribute__((address_space(1))) unsigned int gu32;

__device__ __forceinline__ uint32_t dig(const E64& e, int shift) { return (uint32_t)((e.v >> shift) & 0xFF); }

__global__ void fill(E64* x, uint64_t n) {
  for (uint64_t i = blockIdx.x * (uint64_t)blockDim.x + threadIdx.x; i < n; i += (uint64_t)gridDim.x * blockDim.x)
    x[i].v = (mix64(i * 0x9E37ull + 11) & ~0xFFFFFFFFull) | (uint32_t)i;
}

__global__ void hist(const E64* x, uint64_t n, int shift, uint32_t* counts) {
  __shared__ uint32_t h[kBins];
  h[threadIdx.x] = 0;
  __syncthreads();
  for (uint64_t i = blockIdx.x * (uint64_t)blockDim.x + threadIdx.x; i < n; i += (uint64_t)gridDim.x * blockDim.x)
    atomicAdd(&h[dig(x[i], shift)], 1u);
  __syncthreads();
  atomicAdd(&counts[threadIdx.x], h[threadIdx.x]);
}

__global__ void excl(uint32_t* c) {
  __shared__ uint32_t sc[4];
  uint32_t tot;
  c[threadIdx.x] = block_exclusive_scan256(c[threadIdx.x], sc, tot);
}

template <int ITEMS, bool BALLOT, bool DIRECT = false, int MODE = 0>
__global__ __launch_bounds__(256) void scatter(const E64* __restrict__ in, E64* __restrict__ out, uint64_t n, int shift,
                                               const uint32_t* __restrict__ gbase, unsigned long long* granules,
                                               uint32_t* ticket, uint32_t tiles, const uint32_t* toff = nullptr) {
  constexpr int kTile = kBlock * ITEMS;
  constexpr uint32_t tag_agg = 2, tag_inc = 3;
  __shared__ E64 stage[DIRECT ? 1 : kTile];
  __shared__ uint32_t wcnt[4][kBins];
  __shared__ unsigned long long wmask[BALLOT ? 1 : 4][kBins];
  __shared__ uint32_t bstart[kBins];
  __shared__ uint32_t goff[kBins];
  __shared__ uint32_t sc[4];
  __shared__ uint32_t tile_sh;
  const int t = threadIdx.x, w = wave_id(), l = lane_id();
  if (t == 0) tile_sh = __hip_atomic_fetch_add((gu32*)ticket, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  if constexpr (!BALLOT) {
    wmask[0][t] = 0ull; wmask[1][t] = 0ull; wmask[2][t] = 0ull; wmask[3][t] = 0ull;
  }
  wcnt[0][t] = 0; wcnt[1][t] = 0; wcnt[2][t] = 0; wcnt[3][t] = 0;
  __syncthreads();
  const uint32_t tile = tile_sh;
  if (tile >= tiles) return;
  const uint64_t base = (uint64_t)tile * kTile;
  const uint32_t cnt = (uint32_t)((n - base) < (uint64_t)kTile ? (n - base) : kTile);
  E64 cur[ITEMS];
#pragma unroll
  for (int r = 0; r < ITEMS; ++r) {
    const uint32_t pos = w * (kTile / 4) + r * 64 + l;
    if (pos < cnt) cur[r] = in[base + pos];
  }
  uint32_t rk[ITEMS], dg[ITEMS];
#pragma unroll
  for (int r = 0; r < ITEMS; ++r) {
    const uint32_t pos = w * (kTile / 4) + r * 64 + l;
    const bool valid = pos < cnt;
    const uint32_t d = valid ? dig(cur[r], shift) : 0u;
    unsigned long long peers;
    if constexpr (MODE == 1) {      // timing only: one returning LDS atomic per item (unstable order)
      rk[r] = valid ? atomicAdd(&wcnt[w][d], 1u) : 0u;
      dg[r] = d;
      continue;
    }
    if constexpr (BALLOT) {
      peers = __ballot(valid);
#pragma unroll
      for (int b = 0; b < 8; ++b) {
        const unsigned long long m = __ballot((d >> b) & 1u);
        peers &= ((d >> b) & 1u) ? m : ~m;
      }
      if (!valid) peers = 0ull;
    } else {
      if (valid) atomicOr(&wmask[w][d], 1ull << l);
      __builtin_amdgcn_wave_barrier();
      peers = valid ? wmask[w][d] : 0ull;
    }
    const uint32_t below = popc_below(peers);
    const uint32_t prior = wcnt[w][d];
    __builtin_amdgcn_wave_barrier();
    if (valid && below == 0) {
      wcnt[w][d] = prior + (uint32_t)__popcll(peers);
      if constexpr (!BALLOT) wmask[w][d] = 0ull;
    }
    __builtin_amdgcn_wave_barrier();
    rk[r] = prior + below;
    dg[r] = d;
  }
  __syncthreads();
  const uint32_t c0 = wcnt[0][t], c1 = wcnt[1][t], c2 = wcnt[2][t], c3 = wcnt[3][t];
  const uint32_t tot = c0 + c1 + c2 + c3;
  gu64* mine = (gu64*)(granules + (uint64_t)tile * kBins + t);
  __hip_atomic_store(mine, ((unsigned long long)(tile == 0 ? tag_inc : tag_agg) << 32) | tot, __ATOMIC_RELAXED,
                     __HIP_MEMORY_SCOPE_AGENT);
  unsigned long long pre[4] = {0ull, 0ull, 0ull, 0ull};
  if constexpr (MODE == 3) {                      // first look-back window in flight under the stage fill
#pragma unroll
    for (int k = 0; k < 4; ++k)
      if (tile >= (uint32_t)k + 1)
        pre[k] = __hip_atomic_load((gu64*)(granules + (uint64_t)(tile - 1 - k) * kBins + t), __ATOMIC_RELAXED,
                                   __HIP_MEMORY_SCOPE_AGENT);
  }
  wcnt[0][t] = 0; wcnt[1][t] = c0; wcnt[2][t] = c0 + c1; wcnt[3][t] = c0 + c1 + c2;
  uint32_t all;
  bstart[t] = block_exclusive_scan256(tot, sc, all);
  __syncthreads();
  if constexpr (!DIRECT) {
#pragma unroll
    for (int r = 0; r < ITEMS; ++r) {
      const uint32_t pos = w * (kTile / 4) + r * 64 + l;
      if (pos < cnt) stage[bstart[dg[r]] + wcnt[w][dg[r]] + rk[r]] = cur[r];
    }
  }
  uint32_t ex = 0;
  if (MODE == 2) {
    ex = toff[(uint64_t)tile * kBins + t];        // offsets computed beforehand: no look-back
  } else if (tile > 0) {
    uint64_t j = tile;
    bool first = MODE == 3;
    for (;;) {
      unsigned long long g[4];
#pragma unroll
      for (int k = 0; k < 4; ++k)
        g[k] = first ? pre[k]
                     : j >= (uint64_t)k + 1 ? __hip_atomic_load((gu64*)(granules + (j - 1 - k) * kBins + t),
                                                                __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT)
                                            : 0ull;
      first = false;
      bool done = false;
      int used = 0;
#pragma unroll
      for (int k = 0; k < 4; ++k) {
        if (done || used < k) continue;
        const uint32_t tag = (uint32_t)(g[k] >> 32);
        if (tag == tag_inc) {
          ex += (uint32_t)g[k];
          done = true;
        } else if (tag == tag_agg) {
          ex += (uint32_t)g[k];
          used = k + 1;
        }
      }
      if (done) break;
      j -= (uint64_t)used;
      if (used == 0) __builtin_amdgcn_s_sleep(1);
    }
    __hip_atomic_store(mine, ((unsigned long long)tag_inc << 32) | (ex + tot), __ATOMIC_RELAXED,
                       __HIP_MEMORY_SCOPE_AGENT);
  }
  goff[t] = gbase[t] + ex;
  __syncthreads();
  if constexpr (DIRECT) {
    // no LDS reorder: every entry stored from its register to its final place
#pragma unroll
    for (int r = 0; r < ITEMS; ++r) {
      const uint32_t pos = w * (kTile / 4) + r * 64 + l;
      if (pos < cnt) out[(uint64_t)goff[dg[r]] + wcnt[w][dg[r]] + rk[r]] = cur[r];
    }
  } else {
#pragma unroll 4
    for (uint32_t j = t; j < cnt; j += kBlock) {
      const E64 v = stage[j];
      const uint32_t d = dig(v, shift);
      out[(uint64_t)goff[d] + (j - bstart[d])] = v;
    }
  }
}

// Two independent ranking streams per wave: the first half of the wave's items ranked with the
// LDS lane-mask atomics, the second half with ballots, in the same loop iteration, so one
// stream's LDS latency overlaps the other's VALU/SALU work; the second half's ranks then add the
// first half's digit counts (the halves are contiguous, so the order stays stable).  The stage
// aliases the ranking state (both are dead outside their phase).
template <int ITEMS>
__global__ __launch_bounds__(256) void scatter_dual(const E64* __restrict__ in, E64* __restrict__ out, uint64_t n,
                                                    int shift, const uint32_t* __restrict__ gbase,
                                                    unsigned long long* granules, uint32_t* ticket, uint32_t tiles) {
  constexpr int kTile = kBlock * ITEMS, H = ITEMS / 2;
  constexpr uint32_t tag_agg = 2, tag_inc = 3;
  struct Rank {
    unsigned long long wmask[4][kBins];
    uint32_t wcntB[4][kBins];
  };
  __shared__ union U {
    E64 stage[kTile];
    Rank r;
  } u;
  __shared__ uint32_t wcnt[4][kBins];
  __shared__ uint32_t bstart[kBins];
  __shared__ uint32_t goff[kBins];
  __shared__ uint32_t sc[4];
  __shared__ uint32_t tile_sh;
  const int t = threadIdx.x, w = wave_id(), l = lane_id();
  if (t == 0) tile_sh = __hip_atomic_fetch_add((gu32*)ticket, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
#pragma unroll
  for (int k = 0; k < 4; ++k) {
    u.r.wmask[k][t] = 0ull;
    u.r.wcntB[k][t] = 0;
    wcnt[k][t] = 0;
  }
  __syncthreads();
  const uint32_t tile = tile_sh;
  if (tile >= tiles) return;
  const uint64_t base = (uint64_t)tile * kTile;
  const uint32_t cnt = (uint32_t)((n - base) < (uint64_t)kTile ? (n - base) : kTile);
  E64 cur[ITEMS];
#pragma unroll
  for (int r = 0; r < ITEMS; ++r) {
    const uint32_t pos = w * (kTile / 4) + r * 64 + l;
    if (pos < cnt) cur[r] = in[base + pos];
  }
  uint32_t rk[ITEMS], dg[ITEMS];
#pragma unroll
  for (int r = 0; r < H; ++r) {
    const uint32_t posA = w * (kTile / 4) + r * 64 + l, posB = posA + H * 64;
    const bool vA = posA < cnt, vB = posB < cnt;
    const uint32_t dA = vA ? dig(cur[r], shift) : 0u, dB = vB ? dig(cur[r + H], shift) : 0u;
    if (vA) atomicOr(&u.r.wmask[w][dA], 1ull << l);
    unsigned long long pB = __ballot(vB);
#pragma unroll
    for (int b = 0; b < 8; ++b) {
      const unsigned long long m = __ballot((dB >> b) & 1u);
      pB &= ((dB >> b) & 1u) ? m : ~m;
    }
    if (!vB) pB = 0ull;
    __builtin_amdgcn_wave_barrier();
    const unsigned long long pA = vA ? u.r.wmask[w][dA] : 0ull;
    const uint32_t bA = popc_below(pA), bB = popc_below(pB);
    const uint32_t prA = wcnt[w][dA], prB = u.r.wcntB[w][dB];
    __builtin_amdgcn_wave_barrier();
    if (vA && bA == 0) {
      wcnt[w][dA] = prA + (uint32_t)__popcll(pA);
      u.r.wmask[w][dA] = 0ull;
    }
    if (vB && bB == 0) u.r.wcntB[w][dB] = prB + (uint32_t)__popcll(pB);
    __builtin_amdgcn_wave_barrier();
    rk[r] = prA + bA;
    dg[r] = dA;
    rk[r + H] = prB + bB;
    dg[r + H] = dB;
  }
  __syncthreads();
  // the second half follows the first: its ranks start after the first half's digit counts
#pragma unroll
  for (int r = H; r < ITEMS; ++r) rk[r] += wcnt[w][dg[r]];
  uint32_t c[4];
#pragma unroll
  for (int k = 0; k < 4; ++k) c[k] = wcnt[k][t] + u.r.wcntB[k][t];
  __syncthreads();                                   // ranking state dead: the stage may reuse it
  const uint32_t tot = c[0] + c[1] + c[2] + c[3];
  gu64* mine = (gu64*)(granules + (uint64_t)tile * kBins + t);
  __hip_atomic_store(mine, ((unsigned long long)(tile == 0 ? tag_inc : tag_agg) << 32) | tot, __ATOMIC_RELAXED,
                     __HIP_MEMORY_SCOPE_AGENT);
  wcnt[0][t] = 0; wcnt[1][t] = c[0]; wcnt[2][t] = c[0] + c[1]; wcnt[3][t] = c[0] + c[1] + c[2];
  uint32_t all;
  bstart[t] = block_exclusive_scan256(tot, sc, all);
  __syncthreads();
#pragma unroll
  for (int r = 0; r < ITEMS; ++r) {
    const uint32_t pos = w * (kTile / 4) + r * 64 + l;
    if (pos < cnt) u.stage[bstart[dg[r]] + wcnt[w][dg[r]] + rk[r]] = cur[r];
  }
  uint32_t ex = 0;
  if (tile > 0) {
    uint64_t j = tile;
    for (;;) {
      unsigned long long g[4];
#pragma unroll
      for (int k = 0; k < 4; ++k)
        g[k] = j >= (uint64_t)k + 1 ? __hip_atomic_load((gu64*)(granules + (j - 1 - k) * kBins + t), __ATOMIC_RELAXED,
                                                        __HIP_MEMORY_SCOPE_AGENT)
                                    : 0ull;
      bool done = false;
      int used = 0;
#pragma unroll
      for (int k = 0; k < 4; ++k) {
        if (done || used < k) continue;
        const uint32_t tag = (uint32_t)(g[k] >> 32);
        if (tag == tag_inc) {
          ex += (uint32_t)g[k];
          done = true;
        } else if (tag == tag_agg) {
          ex += (uint32_t)g[k];
          used = k + 1;
        }
      }
      if (done) break;
      j -= (uint64_t)used;
      if (used == 0) __builtin_amdgcn_s_sleep(1);
    }
    __hip_atomic_store(mine, ((unsigned long long)tag_inc << 32) | (ex + tot), __ATOMIC_RELAXED,
                       __HIP_MEMORY_SCOPE_AGENT);
  }
  goff[t] = gbase[t] + ex;
  __syncthreads();
#pragma unroll 4
  for (uint32_t j = t; j < cnt; j += kBlock) {
    const E64 v = u.stage[j];
    const uint32_t d = dig(v, shift);
    out[(uint64_t)goff[d] + (j - bstart[d])] = v;
  }
}

// per-tile digit counts (8192-entry tiles) and their exclusive prefix over tiles, per digit
__global__ void tile_hist(const E64* x, uint64_t n, int shift, uint32_t* th) {
  __shared__ uint32_t h[kBins];
  h[threadIdx.x] = 0;
  __syncthreads();
  const uint64_t b0 = (uint64_t)blockIdx.x * 8192, b1 = b0 + 8192 < n ? b0 + 8192 : n;
  for (uint64_t i = b0 + threadIdx.x; i < b1; i += 256) atomicAdd(&h[dig(x[i], shift)], 1u);
  __syncthreads();
  th[(uint64_t)blockIdx.x * kBins + threadIdx.x] = h[threadIdx.x];
}

__global__ void tile_scan(uint32_t* th, uint64_t tiles) {       // one thread per digit
  uint32_t acc = 0;
  for (uint64_t t = 0; t < tiles; ++t) {
    const uint32_t v = th[t * kBins + threadIdx.x];
    th[t * kBins + threadIdx.x] = acc;
    acc += v;
  }
}

__global__ void diff(const E64* a, const E64* b, uint64_t n, unsigned long long* bad) {
  uint32_t k = 0;
  for (uint64_t i = blockIdx.x * (uint64_t)blockDim.x + threadIdx.x; i < n; i += (uint64_t)gridDim.x * blockDim.x)
    k += a[i].v != b[i].v;
  if (k) atomicAdd(bad, (unsigned long long)k);
}
}  // namespace

#define HC(x)                                                              \
  do {                                                                     \
    hipError_t e_ = (x);                                                   \
    if (e_ != hipSuccess) {                                                \
      std::fprintf(stderr, "%s: %s\n", #x, hipGetErrorString(e_));         \
      std::exit(1);                                                        \
    }                                                                      \
  } while (0)

template <int ITEMS, bool BALLOT, bool DIRECT = false>
static float run(const E64* in, E64* out, uint64_t n, int shift, const uint32_t* gbase, void* ws, size_t ws_bytes) {
  const uint64_t tile = 256ull * ITEMS, tiles = (n + tile - 1) / tile;
  float best = 1e9f;
  hipEvent_t a, b;
  HC(hipEventCreate(&a));
  HC(hipEventCreate(&b));
  for (int it = 0; it < 4; ++it) {
    HC(hipMemset(ws, 0, ws_bytes));
    HC(hipEventRecord(a));
    scatter<ITEMS, BALLOT, DIRECT><<<(unsigned)tiles, 256>>>(in, out, n, shift, gbase,
                                                     reinterpret_cast<unsigned long long*>((char*)ws + 256),
                                                     reinterpret_cast<uint32_t*>(ws), (uint32_t)tiles);
    HC(hipEventRecord(b));
    HC(hipEventSynchronize(b));
    float ms;
    HC(hipEventElapsedTime(&ms, a, b));
    if (it > 0 && ms < best) best = ms;
  }
  return best;
}

int main(int argc, char** argv) {
  const uint64_t n = argc > 1 ? std::strtoull(argv[1], nullptr, 10) : 1250000000ull;
  const int shift = 32;
  E64 *in, *o1, *o2;
  uint32_t* gbase;
  unsigned long long* bad;
  HC(hipMalloc(&in, n * 8));
  HC(hipMalloc(&o1, n * 8));
  HC(hipMalloc(&o2, n * 8));
  HC(hipMalloc(&gbase, kBins * 4));
  HC(hipMalloc(&bad, 8));
  const size_t ws_bytes = 256 + ((n + 4095) / 4096 + 1) * kBins * 8;
  void* ws;
  HC(hipMalloc(&ws, ws_bytes));
  fill<<<8192, 256>>>(in, n);
  HC(hipMemset(gbase, 0, kBins * 4));
  hist<<<4096, 256>>>(in, n, shift, gbase);
  excl<<<1, 256>>>(gbase);
  HC(hipDeviceSynchronize());
  const double gb = n * 16.0 / 1e9;
  float ms = run<32, false>(in, o1, n, shift, gbase, ws, ws_bytes);
  std::printf("lds    items=32: %.3f ms  %.2f TB/s\n", ms, gb / ms);
  ms = run<32, true>(in, o2, n, shift, gbase, ws, ws_bytes);
  std::printf("ballot items=32: %.3f ms  %.2f TB/s\n", ms, gb / ms);
  HC(hipMemset(bad, 0, 8));
  diff<<<4096, 256>>>(o1, o2, n, bad);
  unsigned long long hb = 0;
  HC(hipMemcpy(&hb, bad, 8, hipMemcpyDeviceToHost));
  std::printf("mismatches lds vs ballot: %llu\n", hb);
  {
    const uint64_t tl = 256ull * 32, tiles = (n + tl - 1) / tl;
    float best = 1e9f;
    hipEvent_t a, b;
    HC(hipEventCreate(&a));
    HC(hipEventCreate(&b));
    for (int it = 0; it < 4; ++it) {
      HC(hipMemset(ws, 0, ws_bytes));
      HC(hipEventRecord(a));
      scatter_dual<32><<<(unsigned)tiles, 256>>>(in, o2, n, shift, gbase,
                                                 reinterpret_cast<unsigned long long*>((char*)ws + 256),
                                                 reinterpret_cast<uint32_t*>(ws), (uint32_t)tiles);
      HC(hipEventRecord(b));
      HC(hipEventSynchronize(b));
      float t_;
      HC(hipEventElapsedTime(&t_, a, b));
      if (it > 0 && t_ < best) best = t_;
    }
    std::printf("dual-stream ranking items=32: %.3f ms  %.2f TB/s\n", best, gb / best);
    HC(hipMemset(bad, 0, 8));
    diff<<<4096, 256>>>(o1, o2, n, bad);
    HC(hipMemcpy(&hb, bad, 8, hipMemcpyDeviceToHost));
    std::printf("mismatches lds vs dual: %llu\n", hb);
  }
  {
    const uint64_t tl = 256ull * 32, tiles = (n + tl - 1) / tl;
    uint32_t* toff;
    HC(hipMalloc(&toff, tiles * kBins * 4));
    tile_hist<<<(unsigned)tiles, 256>>>(in, n, shift, toff);
    tile_scan<<<1, 256>>>(toff, tiles);
    HC(hipDeviceSynchronize());
    hipEvent_t a, b;
    HC(hipEventCreate(&a));
    HC(hipEventCreate(&b));
    for (int mode = 1; mode <= 3; ++mode) {
      float best = 1e9f;
      for (int it = 0; it < 4; ++it) {
        HC(hipMemset(ws, 0, ws_bytes));
        HC(hipEventRecord(a));
        auto* g = reinterpret_cast<unsigned long long*>((char*)ws + 256);
        auto* tk = reinterpret_cast<uint32_t*>(ws);
        if (mode == 1)
          scatter<32, false, false, 1><<<(unsigned)tiles, 256>>>(in, o2, n, shift, gbase, g, tk, (uint32_t)tiles, toff);
        else if (mode == 2)
          scatter<32, false, false, 2><<<(unsigned)tiles, 256>>>(in, o2, n, shift, gbase, g, tk, (uint32_t)tiles, toff);
        else
          scatter<32, false, false, 3><<<(unsigned)tiles, 256>>>(in, o2, n, shift, gbase, g, tk, (uint32_t)tiles, toff);
        HC(hipEventRecord(b));
        HC(hipEventSynchronize(b));
        float t_;
        HC(hipEventElapsedTime(&t_, a, b));
        if (it > 0 && t_ < best) best = t_;
      }
      std::printf("%s: %.3f ms  %.2f TB/s\n", mode == 1 ? "atomic ranks, unstable (timing only)" :
                  mode == 2 ? "offsets precomputed (no look-back)" : "look-back window prefetched under the stage fill",
                  best, gb / best);
      if (mode >= 2) {
        HC(hipMemset(bad, 0, 8));
        diff<<<4096, 256>>>(o1, o2, n, bad);
        HC(hipMemcpy(&hb, bad, 8, hipMemcpyDeviceToHost));
        std::printf("mismatches lds vs precomputed: %llu\n", hb);
      }
    }
  }
  ms = run<24, true>(in, o2, n, shift, gbase, ws, ws_bytes);
  std::printf("ballot items=24: %.3f ms  %.2f TB/s\n", ms, gb / ms);
  ms = run<16, true>(in, o2, n, shift, gbase, ws, ws_bytes);
  std::printf("ballot items=16: %.3f ms  %.2f TB/s\n", ms, gb / ms);
  std::fflush(stdout);
  return hb != 0;
}
