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
// butterfly; the assigned point's coordinates (still in registers: they are the MFMA A operand)
// are added into an LDS-privatised [K][D] accumulator with ds_add_f32, flushed once per workgroup
// to f64 global sums.  Points are read from HBM exactly once per iteration.
//
// Operand layout (f32 32x32x2, lane l, r = l & 31, h = l >> 5): A[i = r][k = h], B[k = h][j = r].
// The D = 128 reduction is split as k-step kk in [0, 64) covering dims {kk, 64 + kk} for h = 0/1,
// so each lane keeps its point's half-row (64 consecutive floats) in registers and reads the
// centroid tile with 16-byte LDS loads.  C/D: col j = l & 31, row = (reg & 3) + 8 (reg >> 2) + 4 h.
#include "common.h"

namespace {

typedef float f32x16 __attribute__((ext_vector_type(16)));
constexpr int D = 128;
constexpr int CT = 32;            // centroids per tile
constexpr int LDW = D + 4;        // padded LDS row (132 floats = 528 B: b128 conflict-free)

template <bool ACC_LDS>
__global__ __launch_bounds__(256) void kmeans_step_kernel(const float* __restrict__ X, uint64_t n,
                                                          const float* __restrict__ C, const float* __restrict__ cnorm,
                                                          int K, int32_t* __restrict__ assign,
                                                          double* __restrict__ gsum, unsigned long long* __restrict__ gcnt,
                                                          float* __restrict__ gsum_f32) {
  extern __shared__ __attribute__((aligned(16))) float smem[];
  float* ctile = smem;                              // [CT][LDW]
  float* cn = ctile + CT * LDW;                     // [CT]
  int* bestj_s = reinterpret_cast<int*>(cn + CT);   // [4 waves][32]
  float* acc_s = reinterpret_cast<float*>(bestj_s + 4 * 32);   // [K][D] (ACC_LDS)
  unsigned int* cnt_s = reinterpret_cast<unsigned int*>(acc_s + (ACC_LDS ? K * D : 0));

  const int t = threadIdx.x, w = wave_id(), l = lane_id();
  const int r = l & 31, h = l >> 5;
  if (ACC_LDS) {
    for (int i = t; i < K * D; i += 256) acc_s[i] = 0.f;
    for (int i = t; i < K; i += 256) cnt_s[i] = 0u;
  }
  const uint64_t tiles = (n + 127) / 128;
  for (uint64_t tile = blockIdx.x; tile < tiles; tile += gridDim.x) {
    const uint64_t p = tile * 128 + w * 32 + r;   // this lane's point (A-operand row)
    const bool pvalid = p < n;
    float a[64];
    {
      const float4* src = reinterpret_cast<const float4*>(X + (pvalid ? p : 0) * D + 64 * h);
#pragma unroll
      for (int q = 0; q < 16; ++q) {
        float4 v = pvalid ? src[q] : make_float4(0.f, 0.f, 0.f, 0.f);
        a[4 * q] = v.x; a[4 * q + 1] = v.y; a[4 * q + 2] = v.z; a[4 * q + 3] = v.w;
      }
    }
    float bestd[16];
    int bestj[16];
#pragma unroll
    for (int g = 0; g < 16; ++g) { bestd[g] = __builtin_inff(); bestj[g] = 0; }

    for (int c0 = 0; c0 < K; c0 += CT) {
      __syncthreads();
      // stage centroid tile [CT][D] -> LDS (padded rows); missing centroids -> +inf norm
      for (int i = t; i < CT * (D / 4); i += 256) {
        const int j = i / (D / 4), q = i % (D / 4);
        float4 v = make_float4(0.f, 0.f, 0.f, 0.f);
        if (c0 + j < K) v = reinterpret_cast<const float4*>(C + (uint64_t)(c0 + j) * D)[q];
        *reinterpret_cast<float4*>(ctile + j * LDW + 4 * q) = v;
      }
      if (t < CT) cn[t] = (c0 + t < K) ? cnorm[c0 + t] : __builtin_inff();
      __syncthreads();
      f32x16 acc = {};
      const float* brow = ctile + r * LDW + 64 * h;
#pragma unroll
      for (int q = 0; q < 16; ++q) {
        const float4 b = *reinterpret_cast<const float4*>(brow + 4 * q);
        acc = __builtin_amdgcn_mfma_f32_32x32x2f32(a[4 * q + 0], b.x, acc, 0, 0, 0);
        acc = __builtin_amdgcn_mfma_f32_32x32x2f32(a[4 * q + 1], b.y, acc, 0, 0, 0);
        acc = __builtin_amdgcn_mfma_f32_32x32x2f32(a[4 * q + 2], b.z, acc, 0, 0, 0);
        acc = __builtin_amdgcn_mfma_f32_32x32x2f32(a[4 * q + 3], b.w, acc, 0, 0, 0);
      }
      const float cj = cn[r];
      const int jj = c0 + r;
#pragma unroll
      for (int g = 0; g < 16; ++g) {
        float d = cj - 2.f * acc[g];
        int j = jj;
#pragma unroll
        for (int m = 1; m < 32; m <<= 1) {   // argmin across the 32 centroid lanes of this half
          const float od = __shfl_xor(d, m, 64);
          const int oj = __shfl_xor(j, m, 64);
          if (od < d || (od == d && oj < j)) { d = od; j = oj; }
        }
        if (d < bestd[g] || (d == bestd[g] && j < bestj[g])) { bestd[g] = d; bestj[g] = j; }
      }
    }
    // publish per-row winners: row = (g & 3) + 8 (g >> 2) + 4 h, held by every lane of the half
    if (r == 0) {
#pragma unroll
      for (int g = 0; g < 16; ++g) bestj_s[w * 32 + (g & 3) + 8 * (g >> 2) + 4 * h] = bestj[g];
    }
    __syncthreads();
    const int myj = bestj_s[w * 32 + r];
    if (pvalid) {
      if (h == 0) assign[p] = myj;
      if (ACC_LDS) {
        float* dst = acc_s + myj * D + 64 * h;
#pragma unroll
        for (int k = 0; k < 64; ++k) atomicAdd(dst + k, a[k]);
        if (h == 0) atomicAdd(cnt_s + myj, 1u);
      } else {
        float* dst = gsum_f32 + (uint64_t)myj * D + 64 * h;
#pragma unroll
        for (int k = 0; k < 64; ++k) atomicAdd(dst + k, a[k]);
        if (h == 0) atomicAdd(gcnt + myj, 1ull);
      }
    }
  }
  if (ACC_LDS) {
    __syncthreads();
    for (int i = t; i < K * D; i += 256) {
      const float v = acc_s[i];
      if (v != 0.f) atomicAdd(gsum + i, (double)v);
    }
    for (int i = t; i < K; i += 256)
      if (cnt_s[i]) atomicAdd(gcnt + i, (unsigned long long)cnt_s[i]);
  }
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

}  // namespace

DR_API uint64_t dr_kmeans_smem_bytes(int K, int acc_lds) {
  return (uint64_t)(CT * LDW + CT + 4 * 32) * 4 + (acc_lds ? (uint64_t)K * D * 4 + (uint64_t)K * 4 : 0);
}

// One k-means step over n points of dimension 128.  gsum (K*D f64) and gcnt (K u64) accumulate;
// the caller zeroes them.  gsum_f32 is scratch (K*D f32, zeroed) used only when K is too large
// for the LDS accumulator.
DR_API int dr_kmeans_step(const float* X, uint64_t n, int d, const float* C, int K, float* cnorm_ws,
                          int32_t* assign, double* gsum, unsigned long long* gcnt, float* gsum_f32, hipStream_t s) {
  if (d != D || K < 1) return (int)hipErrorInvalidValue;
  sq_norms_kernel<<<K, 64, 0, s>>>(C, K, cnorm_ws);
  if (n == 0) return 0;
  const bool lds = (uint64_t)K * D * 4 <= 64 * 1024;
  const uint64_t tiles = (n + 127) / 128;
  const unsigned grid = (unsigned)(tiles < 2048 ? tiles : 2048);
  const size_t smem = dr_kmeans_smem_bytes(K, lds ? 1 : 0);
  if (lds)
    kmeans_step_kernel<true><<<grid, 256, smem, s>>>(X, n, C, cnorm_ws, K, assign, gsum, gcnt, gsum_f32);
  else
    kmeans_step_kernel<false><<<grid, 256, smem, s>>>(X, n, C, cnorm_ws, K, assign, gsum, gcnt, gsum_f32);
  DR_LAUNCH_CHECK();
  return 0;
}

// Synthetic Gaussian-mixture points: point i belongs to blob (i * 2654435761) % K; coordinates
// = blob centre (deterministic from blob id) + small deterministic noise.
namespace {
__device__ __forceinline__ float u01(uint64_t z) { return (float)(mix64(z) >> 40) * (1.0f / 16777216.0f); }

__global__ __launch_bounds__(256) void kmeans_gen_kernel(float* __restrict__ X, uint64_t n, uint64_t first,
                                                         int blobs, uint64_t seed) {
  for (uint64_t e = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; e < n * D; e += (uint64_t)gridDim.x * blockDim.x) {
    const uint64_t i = e / D + first;
    const int d = (int)(e % D);
    const uint64_t b = (i * 2654435761ull) % (uint64_t)blobs;
    const float centre = 10.f * u01(seed ^ (b * 0x9E3779B97F4A7C15ull) ^ (uint64_t)d * 0x632BE59BD9B4E019ull) - 5.f;
    const float noise = u01(seed * 31 + i * 0xD1B54A32D192ED03ull + (uint64_t)d) - 0.5f;
    X[e] = centre + 0.2f * noise;
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
