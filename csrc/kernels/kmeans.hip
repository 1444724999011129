// Fused k-means step on MFMA (gfx950): nearest-centroid assignment + per-centroid partial sums.
//
// BASELINE config "k-means on 1B x 128-dim points (Apply/Fork iterative DAG, MFMA reductions)".
// The reference expresses k-means as a DoWhile over Apply/Fork stages on the CPU; here the per-
// partition Apply body is one kernel:
//
//   dist(x, c) = ||c||^2 - 2 x.c     (||x||^2 is constant per point and dropped)
//
// x.c for a 32-point x 32-centroid tile is computed with the exact-f32 matrix core instruction
// v_mfma_f32_32x32x2_f32 (64 MFMAs over D = 128); the argmin over centroids is a 5-step lane
// butterfly; the assigned points' coordinates are added into an LDS-privatised [K][D] accumulator
// with ds_add_f32 (lanes = dimensions), flushed periodically to f64 global sums.  Points are read
// from HBM once per iteration (plus a dimension-sliced second pass when K is too large for an LDS
// slab).
//
// Operand layout (f32 32x32x2, lane l, r = l & 31, h = l >> 5): A[i = r][k = h], B[k = h][j = r].
// The D = 128 reduction is split as k-step kk in [0, 64) covering dims {kk, 64 + kk} for h = 0/1,
// so each lane keeps its point's half-row (64 consecutive floats) in registers and reads the
// centroid tile with 16-byte LDS loads.  C/D: col j = l & 31, row = (reg & 3) + 8 (reg >> 2) + 4 h.
#include "common.h"

namespace {

typedef float f32x16 __attribute__((ext_vector_type(16)));
constexpr int D = 128;
constexpr int CT = 32;            // centroids per MFMA tile
constexpr int LDW = D + 4;        // padded LDS row (132 floats = 528 B: b128 conflict-free)
constexpr int kWaves = 8;         // 512-thread workgroups: one per CU holds the whole LDS budget
constexpr int kPts = kWaves * 32; // points per workgroup tile
constexpr int kFlushTiles = 64;   // flush the f32 LDS slab to f64 every 64 tiles (16K points)
constexpr uint32_t kLdsBudget = 150 * 1024;

// Accumulation (SLAB): for each of its 32 points (uniform loop) a wave adds the point's row into
// slab[j][0..127] with lanes = dimensions: consecutive addresses, so every ds_add_f32 is
// bank-conflict-free no matter how many points share a centroid (a lane-per-point layout puts all
// 64 lanes on one bank).  The rows are re-read from L2 (the tile was loaded an instant ago).
template <bool CRES, bool SLAB>
__global__ __launch_bounds__(512) void kmeans_step_kernel(const float* __restrict__ X, uint64_t n,
                                                          const float* __restrict__ C, const float* __restrict__ cnorm,
                                                          int K, int32_t* __restrict__ assign,
                                                          double* __restrict__ gsum, unsigned long long* __restrict__ gcnt,
                                                          int dbg) {
  extern __shared__ __attribute__((aligned(16))) float smem[];
  const int Kc = CRES ? ((K + CT - 1) / CT) * CT : CT;
  float* ctile = smem;                              // [Kc][LDW]
  float* cn = ctile + Kc * LDW;                     // [Kc]
  int* bestj_db = reinterpret_cast<int*>(cn + Kc);  // [2][kPts] double-buffered by tile parity
  float* acc_s = reinterpret_cast<float*>(bestj_db + 2 * kPts);   // [K][D] (SLAB)
  unsigned int* cnt_s = reinterpret_cast<unsigned int*>(acc_s + (SLAB ? K * D : 0));

  const int t = threadIdx.x, w = t >> 6, l = t & 63;
  const int r = l & 31, h = l >> 5;
  auto stage = [&](int c0, int rows, float* dst, float* dn) {
    for (int i = t; i < rows * (D / 4); i += kWaves * 64) {
      const int j = i / (D / 4), q = i % (D / 4);
      float4 v = make_float4(0.f, 0.f, 0.f, 0.f);
      if (c0 + j < K) v = reinterpret_cast<const float4*>(C + (uint64_t)(c0 + j) * D)[q];
      *reinterpret_cast<float4*>(dst + j * LDW + 4 * q) = v;
    }
    for (int j = t; j < rows; j += kWaves * 64) dn[j] = (c0 + j < K) ? cnorm[c0 + j] : __builtin_inff();
  };
  auto flush = [&]() {
    for (int i = t; i < K * D; i += kWaves * 64) {
      const float v = acc_s[i];
      if (v != 0.f) { atomicAdd(gsum + i, (double)v); acc_s[i] = 0.f; }
    }
    for (int i = t; i < K; i += kWaves * 64)
      if (cnt_s[i]) { atomicAdd(gcnt + i, (unsigned long long)cnt_s[i]); cnt_s[i] = 0u; }
  };
  if (SLAB) {
    for (int i = t; i < K * D; i += kWaves * 64) acc_s[i] = 0.f;
    for (int i = t; i < K; i += kWaves * 64) cnt_s[i] = 0u;
  }
  if (CRES) stage(0, Kc, ctile, cn);
  __syncthreads();
  const uint64_t tiles = (n + kPts - 1) / kPts;
  int since_flush = 0;
  float sink = 0.f;
  float a[64];   // this lane's point (A operand): X[p][64h .. 64h + 63]
  auto load_a = [&](uint64_t tl, float* dst) {
    const uint64_t pp = tl * kPts + w * 32 + r;
    const bool ok = pp < n;
    const float4* src = reinterpret_cast<const float4*>(X + (ok ? pp : 0) * D + 64 * h);
#pragma unroll
    for (int q = 0; q < 16; ++q) {
      const float4 v = ok ? src[q] : make_float4(0.f, 0.f, 0.f, 0.f);
      dst[4 * q] = v.x; dst[4 * q + 1] = v.y; dst[4 * q + 2] = v.z; dst[4 * q + 3] = v.w;
    }
  };
  if (blockIdx.x < tiles) load_a(blockIdx.x, a);
  int parity = 0;
  for (uint64_t tile = blockIdx.x; tile < tiles; tile += gridDim.x, parity ^= 1) {
    // a wave may publish tile i+1's winners while slower waves still read tile i's
    int* bestj_s = bestj_db + parity * kPts;
    const uint64_t p0 = tile * kPts + w * 32;
    const uint64_t p = p0 + r;
    const bool pvalid = p < n;
    // D = C_tile x X^T: lane (r, h) receives the distances of point r to the 16 centroids
    // (g & 3) + 8 (g >> 2) + 4 h of the tile, so the argmin is in-lane VALU work; the two
    // halves are merged once per point tile.
    float bd = __builtin_inff();
    int bj = 0;
    for (int c0 = 0; c0 < ((dbg & 2) ? 0 : K); c0 += CT) {
      const float* tb = ctile;
      const float* tn = cn;
      if (CRES) {
        tb = ctile + c0 * LDW;
        tn = cn + c0;
      } else {
        __syncthreads();
        stage(c0, CT, ctile, cn);
        __syncthreads();
      }
      // two independent accumulation chains (even / odd k-steps) keep the matrix pipe busy
      // instead of serialising 64 dependent MFMAs on one accumulator
      f32x16 acc = {}, acc2 = {};
      const float* brow = tb + r * LDW + 64 * h;
#pragma unroll
      for (int q = 0; q < 16; ++q) {
        const float4 b = *reinterpret_cast<const float4*>(brow + 4 * q);
        acc = __builtin_amdgcn_mfma_f32_32x32x2f32(b.x, a[4 * q + 0], acc, 0, 0, 0);
        acc2 = __builtin_amdgcn_mfma_f32_32x32x2f32(b.y, a[4 * q + 1], acc2, 0, 0, 0);
        acc = __builtin_amdgcn_mfma_f32_32x32x2f32(b.z, a[4 * q + 2], acc, 0, 0, 0);
        acc2 = __builtin_amdgcn_mfma_f32_32x32x2f32(b.w, a[4 * q + 3], acc2, 0, 0, 0);
      }
      acc += acc2;
#pragma unroll
      for (int q4 = 0; q4 < 4; ++q4) {
        const float4 cv = *reinterpret_cast<const float4*>(tn + 8 * q4 + 4 * h);
        const float cc[4] = {cv.x, cv.y, cv.z, cv.w};
#pragma unroll
        for (int e = 0; e < 4; ++e) {
          const float d = cc[e] - 2.f * acc[4 * q4 + e];
          if (d < bd) { bd = d; bj = c0 + 8 * q4 + 4 * h + e; }
        }
      }
    }
    {
      const float od = __shfl_xor(bd, 32, 64);
      const int oj = __shfl_xor(bj, 32, 64);
      if (od < bd || (od == bd && oj < bj)) { bd = od; bj = oj; }
    }
    // prefetch the next tile's points while this tile is accumulated
    float an[64];
    const uint64_t nt = tile + gridDim.x;
    if (nt < tiles) load_a(nt, an);
    if (h == 0) bestj_s[w * 32 + r] = bj;
    __syncthreads();
    if (assign && pvalid && h == 0) assign[p] = bj;
    if (SLAB && !(dbg & 1)) {
      // Centroid j's slab row is owned by wave j % 8 of this workgroup: plain (non-atomic) LDS
      // read-modify-write, lanes = dimensions (LDS float atomics run ~40x slower than ds_read/
      // ds_write on gfx950).  Each wave picks its points of the 256-point tile with a ballot and
      // walks them 4 at a time so 8 row loads (L2 hits) are in flight per step.
      const uint64_t t0 = tile * kPts;
#pragma unroll 1
      for (int c = 0; c < kPts / 64; ++c) {
        const int jj = bestj_s[c * 64 + l];
        uint64_t m = ballot64((t0 + c * 64 + l < n) && ((jj & (kWaves - 1)) == w));
        while (m) {
          int bidx[4];
          int cntb = 0;
#pragma unroll
          for (int u = 0; u < 4; ++u) {
            bidx[u] = m ? (int)__builtin_ctzll(m) : -1;
            if (m) { m &= m - 1; ++cntb; }
          }
          float v0[4], v1[4];
          int jv[4];
#pragma unroll
          for (int u = 0; u < 4; ++u) {
            const int bb = bidx[u] < 0 ? bidx[0] : bidx[u];
            const float* xr = X + (t0 + c * 64 + bb) * D;
            v0[u] = (dbg & 8) ? 1.f : xr[l];
            v1[u] = (dbg & 8) ? 1.f : xr[64 + l];
            jv[u] = __builtin_amdgcn_readlane(jj, bb);
          }
#pragma unroll
          for (int u = 0; u < 4; ++u) {
            if (u < cntb) {
              if (dbg & 4) { sink += v0[u] + v1[u]; continue; }
              float* dst = acc_s + jv[u] * D;
              dst[l] += v0[u];
              dst[64 + l] += v1[u];
              if (l == 0) cnt_s[jv[u]] += 1u;
            }
          }
        }
      }
      if (++since_flush == kFlushTiles) {
        since_flush = 0;
        __syncthreads();
        flush();
      }
    }
#pragma unroll
    for (int i = 0; i < 64; ++i) a[i] = an[i];
  }
  if (SLAB) {
    __syncthreads();
    if (sink == 12345.f) acc_s[0] += 1.f;   // keeps the debug-only loads alive
    flush();
  }
}

// Large K: assignment-only pass above, then the sums by dimension slices of width SW so a
// [K][SW] slab fits LDS.  Lane = (point, dim) with 64 / SW points per wave instruction.
template <int SW>
__global__ __launch_bounds__(256) void kmeans_accum_kernel(const float* __restrict__ X, uint64_t n,
                                                           const int32_t* __restrict__ assign, int K,
                                                           double* __restrict__ gsum, unsigned long long* __restrict__ gcnt) {
  extern __shared__ __attribute__((aligned(16))) float slab[];   // [K][SW] + [K] counts
  unsigned int* cnt = reinterpret_cast<unsigned int*>(slab + K * SW);
  const int t = threadIdx.x;
  const int d0 = blockIdx.y * SW;
  for (int i = t; i < K * SW; i += 256) slab[i] = 0.f;
  for (int i = t; i < K; i += 256) cnt[i] = 0u;
  __syncthreads();
  constexpr int PPI = 256 / SW;   // points per block instruction
  const int pl = t / SW, d = t % SW;
  for (uint64_t q = (uint64_t)blockIdx.x * PPI; q < n; q += (uint64_t)gridDim.x * PPI) {
    const uint64_t p = q + pl;
    if (p < n) {
      const int j = assign[p];
      atomicAdd(slab + j * SW + d, X[p * D + d0 + d]);
      if (blockIdx.y == 0 && d == 0) atomicAdd(cnt + j, 1u);
    }
  }
  __syncthreads();
  for (int i = t; i < K * SW; i += 256) {
    const float v = slab[i];
    if (v != 0.f) atomicAdd(gsum + (uint64_t)(i / SW) * D + d0 + (i % SW), (double)v);
  }
  if (blockIdx.y == 0)
    for (int i = t; i < K; i += 256)
      if (cnt[i]) atomicAdd(gcnt + i, (unsigned long long)cnt[i]);
}

__global__ void sq_norms_kernel(const float* __restrict__ C, int K, float* __restrict__ out) {
  const int j = blockIdx.x;
  float s = 0.f;
  for (int d = threadIdx.x; d < D; d += 64) {
    const float v = C[(uint64_t)j * D + d];
    s += v * v;
  }
#pragma unroll
  for (int m = 32; m >= 1; m >>= 1) s += __shfl_xor(s, m, 64);
  if (threadIdx.x == 0) out[j] = s;
}

uint32_t step_smem(int K, bool cres, bool slab) {
  const int Kc = cres ? ((K + CT - 1) / CT) * CT : CT;
  return (uint32_t)((Kc * LDW + Kc + 2 * kPts) * 4 + (slab ? (uint32_t)K * D * 4 + (uint32_t)K * 4 : 0));
}

int g_num_cus = 0;

int num_cus() {
  if (g_num_cus == 0) {
    int dev = 0;
    hipGetDevice(&dev);
    hipDeviceGetAttribute(&g_num_cus, hipDeviceAttributeMultiprocessorCount, dev);
    if (g_num_cus <= 0) g_num_cus = 256;
  }
  return g_num_cus;
}

template <typename F>
void set_smem(F kern, uint32_t bytes) {
  hipFuncSetAttribute(reinterpret_cast<const void*>(kern), hipFuncAttributeMaxDynamicSharedMemorySize, (int)bytes);
}

}  // namespace

// Mode chosen for K (exposed for tests/benchmarks): 0 = centroids + slab resident,
// 1 = streamed centroid tiles + slab, 2 = assignment pass + sliced accumulation.
DR_API int dr_kmeans_mode(int K) {
  if (step_smem(K, true, true) <= kLdsBudget) return 0;
  if (step_smem(K, false, true) <= kLdsBudget) return 1;
  return 2;
}

// One k-means step over n points of dimension 128.  gsum (K*D f64) and gcnt (K u64) accumulate;
// the caller zeroes them.  assign (n int32) may be null unless K needs mode 2.
DR_API int dr_kmeans_step(const float* X, uint64_t n, int d, const float* C, int K, float* cnorm_ws,
                          int32_t* assign, double* gsum, unsigned long long* gcnt, hipStream_t s) {
  if (d != D || K < 1 || K > 4096) return (int)hipErrorInvalidValue;
  sq_norms_kernel<<<K, 64, 0, s>>>(C, K, cnorm_ws);
  if (n == 0) return 0;
  const int mode = dr_kmeans_mode(K);
  static int dbg = -1;   // DRYAD_KM_DEBUG: bit0 skip accumulation, bit1 skip distances (profiling only)
  if (dbg < 0) {
    const char* e = getenv("DRYAD_KM_DEBUG");
    dbg = e ? atoi(e) : 0;
  }
  const uint64_t tiles = (n + kPts - 1) / kPts;
  const uint64_t cap = (uint64_t)num_cus() * (mode == 2 ? 2 : 1);
  const unsigned grid = (unsigned)(tiles < cap ? tiles : cap);
  if (mode == 0) {
    const uint32_t sm = step_smem(K, true, true);
    set_smem(kmeans_step_kernel<true, true>, sm);
    kmeans_step_kernel<true, true><<<grid, kWaves * 64, sm, s>>>(X, n, C, cnorm_ws, K, assign, gsum, gcnt, dbg);
  } else if (mode == 1) {
    const uint32_t sm = step_smem(K, false, true);
    set_smem(kmeans_step_kernel<false, true>, sm);
    kmeans_step_kernel<false, true><<<grid, kWaves * 64, sm, s>>>(X, n, C, cnorm_ws, K, assign, gsum, gcnt, dbg);
  } else {
    if (!assign) return (int)hipErrorInvalidValue;
    const uint32_t sm = step_smem(K, false, false);
    kmeans_step_kernel<false, false><<<grid, kWaves * 64, sm, s>>>(X, n, C, cnorm_ws, K, assign, gsum, gcnt, dbg);
    const uint32_t per = 128 * 1024;
    const unsigned ag = (unsigned)num_cus();
#define DR_ACCUM(SWV)                                                                              \
    do {                                                                                           \
      const uint32_t sm2 = (uint32_t)K * (SWV + 1) * 4;                                            \
      set_smem(kmeans_accum_kernel<SWV>, sm2);                                                     \
      kmeans_accum_kernel<SWV><<<dim3(ag, D / SWV), 256, sm2, s>>>(X, n, assign, K, gsum, gcnt);   \
    } while (0)
    if ((uint32_t)K * 64 * 4 <= per) DR_ACCUM(64);
    else if ((uint32_t)K * 32 * 4 <= per) DR_ACCUM(32);
    else if ((uint32_t)K * 16 * 4 <= per) DR_ACCUM(16);
    else DR_ACCUM(8);
#undef DR_ACCUM
  }
  DR_LAUNCH_CHECK();
  return 0;
}

// Synthetic blob points (the k-means benchmark input, gen://points): point i belongs to blob
// (i * 2654435761) % blobs; coordinate d = centre(blob, d) + 0.2 * (u - 0.5) with centre in
// [-5, 5).  Every operation is explicitly rounded (no FMA contraction) so the numpy twin in
// models/kmeans_cpu.py reproduces it bit for bit.
namespace {
__device__ __forceinline__ float u01(uint64_t z) { return (float)(mix64(z) >> 40) * (1.0f / 16777216.0f); }

__global__ __launch_bounds__(256) void kmeans_gen_kernel(float* __restrict__ X, uint64_t n, uint64_t first,
                                                         int blobs, uint64_t seed) {
  for (uint64_t e = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; e < n * D; e += (uint64_t)gridDim.x * blockDim.x) {
    const uint64_t i = e / D + first;
    const uint64_t d = e % D;
    const uint64_t b = (i * 2654435761ull) % (uint64_t)blobs;
    const float centre = __fsub_rn(__fmul_rn(10.f, u01(seed ^ (b * 0x9E3779B97F4A7C15ull) ^ (d * 0x632BE59BD9B4E019ull))), 5.f);
    const float noise = __fsub_rn(u01(seed * 31 + i * 0xD1B54A32D192ED03ull + d), 0.5f);
    X[e] = __fadd_rn(centre, __fmul_rn(0.2f, noise));
  }
}
}  // namespace

DR_API int dr_kmeans_gen(float* X, uint64_t n, int d, uint64_t first, int blobs, uint64_t seed, hipStream_t s) {
  if (d != D) return (int)hipErrorInvalidValue;
  if (n == 0) return 0;
  kmeans_gen_kernel<<<grid_for(n * D, 256, 16384), 256, 0, s>>>(X, n, first, blobs, seed);
  DR_LAUNCH_CHECK();
  return 0;
}
