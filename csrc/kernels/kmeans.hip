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

#include <cstdio>
#include <cstdlib>

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


// ---------------------------------------------------------------------------------------------
// K <= 64: the whole step on bf16 MFMA (mode 3).
//
// Distances.  x.c with x = xh + xm (+ 2^-16-relative rest), c = ch + cm split into bf16 parts:
// xh.ch + xh.cm + xm.ch = three v_mfma_f32_32x32x16_bf16 per 16 dims, 5.3x fewer matrix-core
// cycles than the exact-f32 v_mfma_f32_32x32x2_f32 path, with |error| <= ~1.1e-4 |x| max|c| on a
// distance.  Every point whose best and second-best estimates are closer than twice that bound
// is re-ranked with exact f32 dot products, so the assignment is the f32 nearest centroid.
//
// Sums.  S[c][d] += sum_p onehot[p][c] x[p][d] is a GEMM: A = one-hot (exact in bf16), B = the
// point tile split EXACTLY into three bf16 parts (x = xh + xm + xl), f32 accumulation in the
// matrix core's accumulators, flushed to the f64 global sums every `flush` tiles.  No LDS
// read-modify-write and no per-point serial loop.
//
// A wave owns 32-point tiles: it loads a tile (lane (r, h) = point r's dims 16s + 8h .. +7, the
// distance MFMA's B operand), prefetches the next one, stages the tile in LDS for the transposed
// (point-major) reads of the sum MFMA, and keeps the K x 128 sums in 8 accumulator tiles.
// Lane map (32x32x16 bf16): A[row r][k = 8h + j], B[k = 8h + j][col r], C col = l & 31,
// row = (g & 3) + 8 (g >> 2) + 4 h.
typedef __bf16 bf16x8 __attribute__((ext_vector_type(8)));
#ifndef DR_KM_CROW
#define DR_KM_CROW 144
#endif
// bf16 per centroid row in LDS: 288 B = 72 dwords, so the 16-byte fragment reads (lane (r, g) at
// row r, dims 32 s + 8 g) of every ds_read_b128 lane group hit 16 distinct 4-bank sets (136, the
// previous pitch: 2-way conflicts in each group, ~1e9 conflict cycles per assignment call)
constexpr int kCRow = DR_KM_CROW;
constexpr int kXRow = 132;   // floats per point row of the LDS tile
// |estimate - f32 distance| <= kKmTol |x| max|c|: bf16 split residuals 3 * 2^-16 plus f32
// accumulation over 384 products (2.3e-5), both relative to sum |x_i c_i| <= |x| |c|, doubled.
constexpr float kKmTol = 1.5e-4f;

// K <= 64 on 16x16x32 bf16 MFMA, two workgroups per CU (mode 3, default).
//
// (A 32x32x16 kernel that held a wave's whole K x 128 sum tile in registers, 496 VGPR+AGPR, and
// a 32-point LDS tile per wave ran one wave per SIMD, so its MFMA, VALU and HBM waits serialised.)  Here a workgroup steps over 64 points (16 per wave):
//   distances  each wave: its 16 points x 16-centroid tiles, 3 split-bf16 MFMAs per 32 dims, the
//              next step's loads issued per k-step as their registers free up; argmin + runner-up
//              merged over the 4 lanes that share a point; near ties flagged as before
//   sums       every wave: the block's 64 points (one-hot x exact 3-part bf16 split of x, K = 32
//              points per MFMA) for its own 32-dim slice, so a wave keeps K x 32 sums (32 registers)
// LDS: the block's 64 staged points (34 KB) + split centroids (35 KB at K = 64) -> two workgroups
// per CU, two waves per SIMD.  Lane map (16x16x32): A[row l&15][k = 8(l>>4) + j],
// B[k = 8(l>>4) + j][col l&15], C col = l&15, row = 4(l>>4) + reg.
typedef float f32x4 __attribute__((ext_vector_type(4)));
constexpr int kM16Pts = 64;         // points per workgroup step
// staged point rows: 130 floats, so the sum MFMAs' transposed reads (16 lanes = 16 consecutive
// dims of one point, 4 lane groups 8 points apart) hit 64 distinct banks; rows are 8-byte aligned,
// so staging uses 64-bit LDS writes (a 16-byte write off its alignment replays at 64 cycles)
constexpr int kXRow16 = 130;

template <int KT>
__global__ __launch_bounds__(256, 2) void kmeans_mfma16_kernel(const float* __restrict__ X, uint64_t n,
                                                               const float* __restrict__ C,
                                                               const float* __restrict__ cnorm, int K,
                                                               int32_t* __restrict__ assign, double* __restrict__ gsum,
                                                               unsigned long long* __restrict__ gcnt, int flush_steps) {
  constexpr int KP = 16 * KT;
  __shared__ __attribute__((aligned(16))) __bf16 chi[KP * kCRow];
  __shared__ __attribute__((aligned(16))) __bf16 cmd[KP * kCRow];
  __shared__ float cn[KP];
  __shared__ float cmax_s;
  __shared__ __attribute__((aligned(16))) float xs[kM16Pts * kXRow16];
  // one-hot assignment matrix [centroid][point] in bf16, kept in LDS: each point's owner lane sets
  // its single 1.0 and clears it again next step, so no lane compares every (centroid, point) pair.
  // 16-byte slots of a row are XOR-swizzled by (row >> 1) & 7: the A-fragment reads (16 rows x
  // 2 slots per lane group) then hit 16 distinct bank slots.
  __shared__ __attribute__((aligned(16))) __bf16 ohs[KP * kM16Pts];
  __shared__ unsigned int wcnt[KP];
  const int t = threadIdx.x, w = t >> 6, l = t & 63, r = l & 15, g = l >> 4;
  for (int i = t; i < KP * D; i += 256) {
    const int c = i / D, d = i % D;
    const float v = c < K ? C[(uint64_t)c * D + d] : 0.f;
    const __bf16 vh = (__bf16)v;
    chi[c * kCRow + d] = vh;
    cmd[c * kCRow + d] = (__bf16)(v - (float)vh);
  }
  for (int i = t; i < KP * kM16Pts; i += 256) ohs[i] = (__bf16)0.f;
  for (int c = t; c < KP; c += 256) {
    cn[c] = c < K ? cnorm[c] : __builtin_inff();
    wcnt[c] = 0u;
  }
  if (t == 0) {
    float m = 0.f;
    for (int c = 0; c < K; ++c) m = fmaxf(m, cnorm[c]);
    cmax_s = sqrtf(m);
  }
  __syncthreads();
  const float cmax = cmax_s;
  const uint64_t steps = (n + kM16Pts - 1) / kM16Pts;
  f32x4 S[KT][2];
#pragma unroll
  for (int ct = 0; ct < KT; ++ct) {
    S[ct][0] = f32x4{};
    S[ct][1] = f32x4{};
  }
  // lane (r, g) holds point r's dims 32 s + 8 g .. + 7, s < 4
  float xr[32];
  auto load_part = [&](uint64_t step, int s_, float* dst) {
    // clamped, unconditional: a point past n re-reads point n - 1 (its row is finite, it sets no
    // one-hot entry and writes no assignment), so no branch wraps the loads
    const uint64_t p = min(step * kM16Pts + 16 * w + r, n - 1);
    const float4* src = reinterpret_cast<const float4*>(X + p * D + 32 * s_ + 8 * g);
    const float4 a = src[0];
    const float4 b = src[1];
    dst[8 * s_ + 0] = a.x; dst[8 * s_ + 1] = a.y; dst[8 * s_ + 2] = a.z; dst[8 * s_ + 3] = a.w;
    dst[8 * s_ + 4] = b.x; dst[8 * s_ + 5] = b.y; dst[8 * s_ + 6] = b.z; dst[8 * s_ + 7] = b.w;
  };
  if ((uint64_t)blockIdx.x < steps) {
#pragma unroll
    for (int s_ = 0; s_ < 4; ++s_) load_part(blockIdx.x, s_, xr);
  }
  auto flush = [&]() {
#pragma unroll
    for (int ct = 0; ct < KT; ++ct)
#pragma unroll
      for (int dt = 0; dt < 2; ++dt) {
#pragma unroll
        for (int q = 0; q < 4; ++q) {
          const int c = ct * 16 + 4 * g + q;
          const float v = S[ct][dt][q];
          if (c < K && v != 0.f) atomicAdd(gsum + (uint64_t)c * D + 32 * w + 16 * dt + r, (double)v);
        }
        S[ct][dt] = f32x4{};
      }
  };
  auto oh_at = [](int c, int pt) { return c * kM16Pts + 8 * ((pt >> 3) ^ ((c >> 1) & 7)) + (pt & 7); };
  int since = 0, marked = -1;   // marked: the centroid whose one-hot entry this lane set last step
  for (uint64_t step = blockIdx.x; step < steps; step += gridDim.x) {
    const uint64_t p = step * kM16Pts + 16 * w + r;
    const bool pvalid = p < n;
    // stage the wave's 16 points for the sum MFMAs of every wave (point-major rows)
    float* xrow = xs + (16 * w + r) * kXRow16;
#pragma unroll
    for (int s_ = 0; s_ < 4; ++s_)
#pragma unroll
      for (int q = 0; q < 4; ++q)
        *reinterpret_cast<float2*>(xrow + 32 * s_ + 8 * g + 2 * q) = make_float2(xr[8 * s_ + 2 * q], xr[8 * s_ + 2 * q + 1]);
    f32x4 Dt[KT];
#pragma unroll
    for (int ct = 0; ct < KT; ++ct) Dt[ct] = f32x4{};
    float xx = 0.f;
#pragma unroll
    for (int s_ = 0; s_ < 4; ++s_) {
      bf16x8 xh, xm;
#pragma unroll
      for (int j = 0; j < 8; ++j) {
        const float v = xr[8 * s_ + j];
        xx = fmaf(v, v, xx);
        xh[j] = (__bf16)v;
        xm[j] = (__bf16)(v - (float)xh[j]);
      }
      load_part(step + gridDim.x, s_, xr);   // next step in flight; unconditional (clamped rows) so
                                             // the loaded registers need no loop-carried copy
      bf16x8 ah[KT], am[KT];                              // every fragment read before the MFMAs
#pragma unroll
      for (int ct = 0; ct < KT; ++ct) {
        ah[ct] = *reinterpret_cast<const bf16x8*>(chi + (ct * 16 + r) * kCRow + 32 * s_ + 8 * g);
        am[ct] = *reinterpret_cast<const bf16x8*>(cmd + (ct * 16 + r) * kCRow + 32 * s_ + 8 * g);
      }
#pragma unroll
      for (int ct = 0; ct < KT; ++ct) {
        Dt[ct] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(ah[ct], xh, Dt[ct], 0, 0, 0);
        Dt[ct] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(ah[ct], xm, Dt[ct], 0, 0, 0);
        Dt[ct] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(am[ct], xh, Dt[ct], 0, 0, 0);
      }
    }
    // argmin with the runner-up over this lane's 4 KT centroids, then over the 4 lanes of the point
    float bd = __builtin_inff(), sd = __builtin_inff();
    int bj = 0;
#pragma unroll
    for (int ct = 0; ct < KT; ++ct)
#pragma unroll
      for (int q = 0; q < 4; ++q) {
        const int c = ct * 16 + 4 * g + q;
        const float d = fmaf(-2.f, Dt[ct][q], cn[c]);
        sd = fminf(sd, fmaxf(bd, d));
        bj = d < bd ? c : bj;
        bd = fminf(bd, d);
      }
#pragma unroll
    for (int m = 16; m <= 32; m <<= 1) {
      const float obd = __shfl_xor(bd, m, 64), osd = __shfl_xor(sd, m, 64);
      const int obj = __shfl_xor(bj, m, 64);
      xx += __shfl_xor(xx, m, 64);
      if (obd < bd || (obd == bd && obj < bj)) {
        sd = fminf(bd, osd);
        bd = obd;
        bj = obj;
      } else {
        sd = fminf(sd, obd);
      }
    }
    const bool near = K > 1 && (sd - bd) <= 2.f * kKmTol * sqrtf(xx) * cmax;
    if (g == 0) {
      if (marked >= 0) ohs[oh_at(marked, 16 * w + r)] = (__bf16)0.f;
      marked = pvalid ? bj : -1;
      if (pvalid) {
        ohs[oh_at(bj, 16 * w + r)] = (__bf16)1.f;
        atomicAdd(&wcnt[bj], 1u);
        assign[p] = near ? (int32_t)((uint32_t)bj | 0x80000000u) : bj;
      }
    }
    __syncthreads();
    // sums over the block's 64 points for this wave's dims 32 w .. 32 w + 31
#pragma unroll
    for (int ks = 0; ks < 2; ++ks) {
      bf16x8 oh[KT];
#pragma unroll
      for (int ct = 0; ct < KT; ++ct) oh[ct] = *reinterpret_cast<const bf16x8*>(ohs + oh_at(ct * 16 + r, 32 * ks + 8 * g));
      float xv[2][8];                                     // both dim tiles' values read up front
#pragma unroll
      for (int dt = 0; dt < 2; ++dt)
#pragma unroll
        for (int j = 0; j < 8; ++j) xv[dt][j] = xs[(32 * ks + 8 * g + j) * kXRow16 + 32 * w + 16 * dt + r];
#pragma unroll
      for (int dt = 0; dt < 2; ++dt) {
        // x split EXACTLY into three bf16 parts (x = xh + xm + xl), so a cluster's sum carries
        // only the f32 accumulation rounding (this kernel is the fallback of the split-plane path
        // below, which reads the parts precomputed)
        bf16x8 ph, pm, pl;
#pragma unroll
        for (int j = 0; j < 8; ++j) {
          const float v = xv[dt][j];
          const __bf16 a0 = (__bf16)v;
          const float r1 = v - (float)a0;
          const __bf16 a1 = (__bf16)r1;
          ph[j] = a0;
          pm[j] = a1;
          pl[j] = (__bf16)(r1 - (float)a1);
        }
#pragma unroll
        for (int ct = 0; ct < KT; ++ct) {
          S[ct][dt] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(oh[ct], ph, S[ct][dt], 0, 0, 0);
          S[ct][dt] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(oh[ct], pm, S[ct][dt], 0, 0, 0);
          S[ct][dt] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(oh[ct], pl, S[ct][dt], 0, 0, 0);
        }
      }
    }
    __syncthreads();                          // xs / ohs are rewritten by the next step
    if (++since == flush_steps) {
      since = 0;
      flush();
    }
  }
  flush();
  __syncthreads();
  for (int c = t; c < K; c += 256)
    if (wcnt[c]) atomicAdd(gcnt + c, (unsigned long long)wcnt[c]);
}

// ---------------------------------------------------------------------------------------------
// K <= 64 on a precomputed bf16 plane with incrementally maintained sums (mode 3, default when
// the plane fits in HBM).
//
// The points of a k-means job are static across its iterations, so two things are done once per
// point table instead of once per iteration:
//   * the bf16 rounding xh of every coordinate and |x| per point (kmeans_hi_kernel), 256 + 4 bytes
//     per point: an iteration's assignment kernel reads half the bytes of the f32 rows and does
//     no conversion work;
//   * the per-cluster sums: S[c] = sum of x over the points assigned to c (f64) and the counts are
//     kept with the table; after an iteration's final assignment, kmeans_movers_kernel moves the
//     exact f32 row of every point whose cluster changed (all of them on the first iteration, a
//     few percent after that) from its old cluster's sums to its new one's.
// The step's result is therefore the exact sums of the f32 points of each cluster (f64
// accumulation of f32 values), as a from-scratch pass would compute them.
//
//   assignment  each wave independently: 16-point tiles, xh.ch + xh.cm on 16x16x32 bf16 MFMAs
//               (c = ch + cm split in LDS), argmin + runner-up merged over the 4 lanes of a point;
//               |estimate - f32 distance| <= kKmTolH |x| max|c| (xh's rounding 2^-9 |x|, cm's
//               residual 2^-17, f32 accumulation, doubled for d = |c|^2 - 2 x.c), so points whose
//               best two estimates are closer than twice that are flagged and re-ranked exactly
//               from the f32 row (kmeans_near_list + kmeans_rerank_kernel)
constexpr float kKmTolH = 4.0e-3f;
#ifndef DR_KM_DEPTH
#define DR_KM_DEPTH 2                               // (a build-time constant; tools/micro/km_depth_ab.py)
#endif
constexpr int kKmDepth = DR_KM_DEPTH;               // 16-point tiles in flight per wave
#ifndef DR_KM_WAVES
#define DR_KM_WAVES 8                               // waves per workgroup (they share the LDS fragments)
#endif
constexpr int kKmWaves = DR_KM_WAVES;
#ifndef DR_KM_CH_REGS
#define DR_KM_CH_REGS 0                             // ch fragments kept in registers (0: LDS per tile)
#endif

__global__ __launch_bounds__(256) void kmeans_hi_kernel(const float* __restrict__ X, uint64_t n,
                                                        __bf16* __restrict__ XH, float* __restrict__ xnorm) {
  // one wave per point, lane l: dims 2l, 2l + 1
  const int l = threadIdx.x & 63;
  const uint64_t nw = ((uint64_t)gridDim.x * blockDim.x) >> 6;
  for (uint64_t p = ((uint64_t)blockIdx.x * blockDim.x + threadIdx.x) >> 6; p < n; p += nw) {
    const float2 v = reinterpret_cast<const float2*>(X + p * D)[l];
    float ss = fmaf(v.x, v.x, v.y * v.y);
    XH[p * D + 2 * l] = (__bf16)v.x;
    XH[p * D + 2 * l + 1] = (__bf16)v.y;
#pragma unroll
    for (int m = 32; m >= 1; m >>= 1) ss += __shfl_xor(ss, m, 64);
    if (l == 0) xnorm[p] = sqrtf(ss);
  }
}

// The points stream through registers, KD 16-point tiles ahead of the one being assigned (the
// 32 GB plane is read once; only deep prefetch keeps enough bytes in flight per CU at two waves
// per SIMD).  The ch fragments (KT x 4 x 16 bytes per lane) are read from LDS once per wave and stay
// in registers, the cm fragments are read from LDS per tile (16 KB of LDS per tile and wave at
// KT = 4: a quarter of the fragment traffic of reading both per tile).
template <int KT, int KD>
__global__ __launch_bounds__(64 * kKmWaves) void kmeans_assign_kernel(const __bf16* __restrict__ XH,
                                                            const float* __restrict__ xnorm, uint64_t n,
                                                            const float* __restrict__ C,
                                                            const float* __restrict__ cnorm, int K,
                                                            int32_t* __restrict__ assign) {
  constexpr int KP = 16 * KT;
  __shared__ __attribute__((aligned(16))) __bf16 chi[KP * kCRow];
  __shared__ __attribute__((aligned(16))) __bf16 cmd[KP * kCRow];
  __shared__ float cn[KP];
  __shared__ float cmax_s;
  const int t = threadIdx.x, w = t >> 6, l = t & 63, r = l & 15, g = l >> 4;
  for (int i = t; i < KP * D; i += 64 * kKmWaves) {
    const int c = i / D, d = i % D;
    const float v = c < K ? C[(uint64_t)c * D + d] : 0.f;
    const __bf16 vh = (__bf16)v;
    chi[c * kCRow + d] = vh;
    cmd[c * kCRow + d] = (__bf16)(v - (float)vh);
  }
  for (int c = t; c < KP; c += 64 * kKmWaves) cn[c] = c < K ? cnorm[c] : __builtin_inff();
  if (t == 0) {
    float m = 0.f;
    for (int c = 0; c < K; ++c) m = fmaxf(m, cnorm[c]);
    cmax_s = sqrtf(m);
  }
  __syncthreads();
  const float cmax = cmax_s;
#if DR_KM_CH_REGS
  bf16x8 ch[KT][4];
#pragma unroll
  for (int ct = 0; ct < KT; ++ct)
#pragma unroll
    for (int s_ = 0; s_ < 4; ++s_)
      ch[ct][s_] = *reinterpret_cast<const bf16x8*>(chi + (ct * 16 + r) * kCRow + 32 * s_ + 8 * g);
#endif
  const uint64_t tiles = (n + 15) / 16;
  const uint64_t gw = (uint64_t)blockIdx.x * kKmWaves + w, GW = (uint64_t)gridDim.x * kKmWaves;
  // lane (r, g) holds dims 32 s + 8 g .. + 7 of point r of the tile, s < 4; clamped rows (a point
  // past n re-reads point n - 1 and writes nothing), so the loads need no branch
  struct Pts {
    bf16x8 x[4];
    float xn;
  };
  auto load = [&](uint64_t tile, Pts& d) {
    const uint64_t p = min(tile * 16 + r, n - 1);
#pragma unroll
    for (int s_ = 0; s_ < 4; ++s_) d.x[s_] = *reinterpret_cast<const bf16x8*>(XH + p * D + 32 * s_ + 8 * g);
    d.xn = xnorm[p];
  };
  Pts ring[KD];
#pragma unroll
  for (int j = 0; j < KD; ++j)
    if (gw + j * GW < tiles) load(gw + j * GW, ring[j]);
  for (uint64_t tile = gw; tile < tiles; tile += GW) {
    // compiler barrier: keeps the cm fragment reads below inside the loop (hoisted, they would
    // take 16 x KT more registers per lane than the prefetch ring they displace)
    asm volatile("" ::: "memory");
    const uint64_t p = tile * 16 + r;
    f32x4 Dt[KT];
#pragma unroll
    for (int ct = 0; ct < KT; ++ct) Dt[ct] = f32x4{};
    const Pts cur = ring[0];
#pragma unroll
    for (int j = 0; j + 1 < KD; ++j) ring[j] = ring[j + 1];
    const uint64_t nx = tile + KD * GW;
    load(nx < tiles ? nx : tile, ring[KD - 1]);       // KD tiles in flight under the MFMAs
#pragma unroll
    for (int s_ = 0; s_ < 4; ++s_) {
#pragma unroll
      for (int ct = 0; ct < KT; ++ct) {
        const bf16x8 am = *reinterpret_cast<const bf16x8*>(cmd + (ct * 16 + r) * kCRow + 32 * s_ + 8 * g);
#if DR_KM_CH_REGS
        const bf16x8 ah = ch[ct][s_];
#else
        const bf16x8 ah = *reinterpret_cast<const bf16x8*>(chi + (ct * 16 + r) * kCRow + 32 * s_ + 8 * g);
#endif
        Dt[ct] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(ah, cur.x[s_], Dt[ct], 0, 0, 0);
        Dt[ct] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(am, cur.x[s_], Dt[ct], 0, 0, 0);
      }
    }
    float bd = __builtin_inff(), sd = __builtin_inff();
    int bj = 0;
#pragma unroll
    for (int ct = 0; ct < KT; ++ct)
#pragma unroll
      for (int q = 0; q < 4; ++q) {
        const int c = ct * 16 + 4 * g + q;
        const float d = fmaf(-2.f, Dt[ct][q], cn[c]);
        sd = fminf(sd, fmaxf(bd, d));
        bj = d < bd ? c : bj;
        bd = fminf(bd, d);
      }
#pragma unroll
    for (int m = 16; m <= 32; m <<= 1) {
      const float obd = __shfl_xor(bd, m, 64), osd = __shfl_xor(sd, m, 64);
      const int obj = __shfl_xor(bj, m, 64);
      if (obd < bd || (obd == bd && obj < bj)) {
        sd = fminf(bd, osd);
        bd = obd;
        bj = obj;
      } else {
        sd = fminf(sd, obd);
      }
    }
    const bool near = K > 1 && (sd - bd) <= 2.f * kKmTolH * cur.xn * cmax;
    if (g == 0 && p < n) assign[p] = near ? (int32_t)((uint32_t)bj | 0x80000000u) : bj;
  }
}

// Moves every point whose final assignment changed since the previous step (prev < 0: never
// assigned) between the clusters' sums S (f64 [K][128]) and counts, and records the assignment.
// Centroid c's LDS row belongs to wave c & 3: plain read-modify-write of f64, lanes = dims l and
// 64 + l; each wave walks the block's 256-point batch by ballot and keeps 8 f32 rows in flight.
__global__ __launch_bounds__(256) void kmeans_movers_kernel(const float* __restrict__ X, uint64_t n,
                                                            const int32_t* __restrict__ assign,
                                                            int32_t* __restrict__ prev, int K,
                                                            double* __restrict__ S, long long* __restrict__ cnt) {
  __shared__ __attribute__((aligned(16))) double slab[64 * D];
  __shared__ int dcnt[64];
  __shared__ int cur_s[256], old_s[256];
  const int t = threadIdx.x, w = t >> 6, l = t & 63;
  for (int i = t; i < 64 * D; i += 256) slab[i] = 0.0;
  if (t < 64) dcnt[t] = 0;
  for (uint64_t b = (uint64_t)blockIdx.x * 256; b < n; b += (uint64_t)gridDim.x * 256) {
    const uint64_t p = b + t;
    int a = -1, o = -1;
    if (p < n) {
      a = assign[p];
      o = prev[p];
      if (a != o) prev[p] = a;
    }
    __syncthreads();   // the previous batch's readers are done with cur_s / old_s
    cur_s[t] = a;
    old_s[t] = o;
    __syncthreads();
#pragma unroll 1
    for (int c = 0; c < 4; ++c) {
      const int ca = cur_s[64 * c + l], co = old_s[64 * c + l];
      const bool mv = ca != co;
      // one entry per (point, row this wave owns): +x into row ca, -x from row co
      uint64_t madd = ballot64(mv && ca >= 0 && (ca & 3) == w);
      uint64_t msub = ballot64(mv && co >= 0 && (co & 3) == w);
      while (madd | msub) {
        int idx[8], crow[8];
        double sgn[8];
        int k8 = 0;
#pragma unroll
        for (int u = 0; u < 8; ++u) {
          idx[u] = 0;
          crow[u] = 0;
          sgn[u] = 0.0;
          if (madd) {
            const int k = __builtin_ctzll(madd);
            madd &= madd - 1;
            idx[u] = k; crow[u] = __builtin_amdgcn_readlane(ca, k); sgn[u] = 1.0; ++k8;
          } else if (msub) {
            const int k = __builtin_ctzll(msub);
            msub &= msub - 1;
            idx[u] = k; crow[u] = __builtin_amdgcn_readlane(co, k); sgn[u] = -1.0; ++k8;
          }
        }
        float v0[8], v1[8];
#pragma unroll
        for (int u = 0; u < 8; ++u) {
          const float* xr = X + (b + 64 * c + idx[u]) * D;
          v0[u] = xr[l];
          v1[u] = xr[64 + l];
        }
#pragma unroll
        for (int u = 0; u < 8; ++u) {
          if (u < k8) {
            double* dst = slab + crow[u] * D;
            dst[l] += sgn[u] * (double)v0[u];
            dst[64 + l] += sgn[u] * (double)v1[u];
            if (l == 0) dcnt[crow[u]] += sgn[u] > 0 ? 1 : -1;
          }
        }
      }
    }
  }
  __syncthreads();
  for (int i = t; i < K * D; i += 256) {
    const double v = slab[i];
    if (v != 0.0) atomicAdd(S + i, v);
  }
  if (t < K && dcnt[t]) atomicAdd(reinterpret_cast<unsigned long long*>(cnt + t), (unsigned long long)(long long)dcnt[t]);
}

// Compaction of the near-tie flags (bit 31 of assign) into (point, estimate) pairs; clears the flag.
// Zeroes the near-tie count + pad (4 words) before a step.  A kernel rather than a memset node so
// that a captured step (runtime/hipgraph.py) resets it on every replay like an eager run does.
__global__ void kmeans_near_reset(uint32_t* __restrict__ near_cnt) {
  if (threadIdx.x < 4) near_cnt[threadIdx.x] = 0u;
}

// Lists the points flagged near-tie by the step kernel (capacity n entries: each point is listed
// at most once per step; writes past it are dropped so a missed reset cannot overrun the list).
__global__ __launch_bounds__(256) void kmeans_near_list(int32_t* __restrict__ assign, uint64_t n,
                                                        uint32_t* __restrict__ near_cnt, uint32_t* __restrict__ near_list) {
  for (uint64_t b = (uint64_t)blockIdx.x * blockDim.x; b < n; b += (uint64_t)gridDim.x * blockDim.x) {
    const uint64_t p = b + threadIdx.x;
    const int32_t a = p < n ? assign[p] : 0;
    const bool near = a < 0;
    const uint64_t m = __ballot(near);
    if (m) {
      const int l = threadIdx.x & 63;
      const int first = __builtin_ctzll(m);
      uint32_t base = 0;
      if (l == first) base = atomicAdd(near_cnt, (uint32_t)__popcll(m));
      base = __shfl(base, first, 64);
      if (near) {
        const uint32_t o = base + popc_below(m);
        const uint32_t est = (uint32_t)a & 0x7FFFFFFFu;
        if (o < n) {
          near_list[2 * (uint64_t)o] = (uint32_t)p;
          near_list[2 * (uint64_t)o + 1] = est;
        }
        assign[p] = (int32_t)est;
      }
    }
  }
}

// Exact f32 re-rank of the near-tie points listed by kmeans_near_list: one wave per point, lane
// c computes the f32 distance to centroid c; if the estimate's choice was wrong the assignment is
// corrected and, when the step kernel accumulated sums (gsum != null), the point's row and count
// move to the right centroid.  The grid drains the device-side count.
__global__ __launch_bounds__(64) void kmeans_rerank_kernel(const float* __restrict__ X, const float* __restrict__ C,
                                                           const float* __restrict__ cnorm, int K,
                                                           const uint32_t* __restrict__ near_cnt,
                                                           const uint32_t* __restrict__ near_list,
                                                           int32_t* __restrict__ assign, double* __restrict__ gsum,
                                                           unsigned long long* __restrict__ gcnt, uint64_t n) {
  const uint32_t total = (uint64_t)*near_cnt < n ? *near_cnt : (uint32_t)n;
  const int l = threadIdx.x;
  for (uint32_t i = blockIdx.x; i < total; i += gridDim.x) {
    const uint64_t p = near_list[2 * (uint64_t)i];
    const int est = (int)near_list[2 * (uint64_t)i + 1];
    const float4* xr = reinterpret_cast<const float4*>(X + p * D);
    float d = __builtin_inff();
    if (l < K) {
      const float4* cr = reinterpret_cast<const float4*>(C + (uint64_t)l * D);
      float a0 = 0.f, a1 = 0.f;
      for (int k = 0; k < D / 4; k += 2) {
        const float4 x0 = xr[k], x1 = xr[k + 1], c0 = cr[k], c1 = cr[k + 1];
        a0 = fmaf(x0.x, c0.x, fmaf(x0.y, c0.y, fmaf(x0.z, c0.z, fmaf(x0.w, c0.w, a0))));
        a1 = fmaf(x1.x, c1.x, fmaf(x1.y, c1.y, fmaf(x1.z, c1.z, fmaf(x1.w, c1.w, a1))));
      }
      d = cnorm[l] - 2.f * (a0 + a1);
    }
    int bj = l;
#pragma unroll
    for (int m = 32; m >= 1; m >>= 1) {
      const float od = __shfl_xor(d, m, 64);
      const int oj = __shfl_xor(bj, m, 64);
      if (od < d || (od == d && oj < bj)) { d = od; bj = oj; }
    }
    if (bj == est) continue;
    if (gsum) {
      const float v0 = X[p * D + l], v1 = X[p * D + 64 + l];
      atomicAdd(gsum + (uint64_t)est * D + l, -(double)v0);
      atomicAdd(gsum + (uint64_t)est * D + 64 + l, -(double)v1);
      atomicAdd(gsum + (uint64_t)bj * D + l, (double)v0);
      atomicAdd(gsum + (uint64_t)bj * D + 64 + l, (double)v1);
      if (l == 0) {
        atomicAdd(gcnt + est, ~0ull);          // -1
        atomicAdd(gcnt + bj, 1ull);
      }
    }
    if (l == 0) assign[p] = bj;
  }
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
// 1 = streamed centroid tiles + slab, 2 = assignment pass + sliced accumulation,
// 3 = K <= 64 on bf16 MFMA (split-precision distances with exact re-rank, MFMA one-hot sums).
DR_API int dr_kmeans_mode(int K) {
  if (K <= 64) return 3;
  if (step_smem(K, true, true) <= kLdsBudget) return 0;
  if (step_smem(K, false, true) <= kLdsBudget) return 1;
  return 2;
}

// One k-means step over n points of dimension 128.  gsum (K*D f64) and gcnt (K u64) accumulate;
// the caller zeroes them.  assign (n int32) may be null unless K needs mode 2; near_ws (mode 3)
// holds dr_kmeans_near_workspace(n) bytes.
DR_API uint64_t dr_kmeans_near_workspace(uint64_t n) { return 8 * n + 16; }

DR_API int dr_kmeans_step(const float* X, uint64_t n, int d, const float* C, int K, float* cnorm_ws,
                          int32_t* assign, double* gsum, unsigned long long* gcnt, void* near_ws, hipStream_t s) {
  if (d != D || K < 1 || K > 4096) return (int)hipErrorInvalidValue;
  sq_norms_kernel<<<K, 64, 0, s>>>(C, K, cnorm_ws);
  if (n == 0) return 0;
  const int mode = dr_kmeans_mode(K);
  constexpr int dbg = 0;     // the kernels' phase-skip bits stay off in the library (no env knob)
  if (mode == 3) {
    // near_ws: [0] = count, then 2 words per listed point (point, estimated centroid); 8 n + 16
    // bytes (dr_kmeans_near_workspace)
    if (!near_ws || !assign) return (int)hipErrorInvalidValue;
    const uint64_t wt = (n + 31) / 32;
    const uint64_t blocks = (wt + 3) / 4;
    const unsigned g3 = (unsigned)(blocks < (uint64_t)num_cus() ? blocks : (uint64_t)num_cus());
    uint32_t* near_cnt = reinterpret_cast<uint32_t*>(near_ws);
    uint32_t* near_list = near_cnt + 4;
    kmeans_near_reset<<<1, 64, 0, s>>>(near_cnt);
    {
      const uint64_t st = (n + kM16Pts - 1) / kM16Pts;
      const uint64_t cap = 2 * (uint64_t)num_cus();
      const unsigned g16 = (unsigned)(st < cap ? st : cap);
#define DR_KM16(KTV) kmeans_mfma16_kernel<KTV><<<g16, 256, 0, s>>>(X, n, C, cnorm_ws, K, assign, gsum, gcnt, 128)
      if (K <= 16) DR_KM16(1);
      else if (K <= 32) DR_KM16(2);
      else if (K <= 48) DR_KM16(3);
      else DR_KM16(4);
#undef DR_KM16
    }
    kmeans_near_list<<<grid_for(n, 256, 4096), 256, 0, s>>>(assign, n, near_cnt, near_list);
    kmeans_rerank_kernel<<<1024, 64, 0, s>>>(X, C, cnorm_ws, K, near_cnt, near_list, assign, gsum, gcnt, n);
    DR_LAUNCH_CHECK();
    if (dbg & 8) {
      uint32_t v = 0;
      hipMemcpyAsync(&v, near_cnt, 4, hipMemcpyDeviceToHost, s);
      hipStreamSynchronize(s);
      fprintf(stderr, "[kmeans] near-tie points re-ranked: %u of %llu\n", v, (unsigned long long)n);
    }
    return 0;
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

// bf16 plane of n points (K <= 64 path): XH = n * 128 bf16, xnorm = n f32 (|x|).
DR_API int dr_kmeans_hi(const float* X, uint64_t n, __bf16* XH, float* xnorm, hipStream_t s) {
  if (n == 0) return 0;
  kmeans_hi_kernel<<<grid_for(n * 64, 256, 8192), 256, 0, s>>>(X, n, XH, xnorm);
  DR_LAUNCH_CHECK();
  return 0;
}

// One k-means step (K <= 64) on the bf16 plane with sums kept across steps.  assign (n) receives
// the final assignment; prev (n, -1 = none), S (K * 128 f64) and cnt (K i64) are the table's
// running per-cluster state: zero S / cnt and fill prev with -1 whenever K or the points change.
// After the call S / cnt hold the sums / counts of this step's assignment.
DR_API int dr_kmeans_step_hi(const __bf16* XH, const float* xnorm, const float* X, uint64_t n, const float* C, int K,
                             float* cnorm_ws, int32_t* assign, int32_t* prev, double* S, long long* cnt,
                             void* near_ws, hipStream_t s) {
  if (K < 1 || K > 64 || !assign || !prev || !S || !cnt || !near_ws) return (int)hipErrorInvalidValue;
  sq_norms_kernel<<<K, 64, 0, s>>>(C, K, cnorm_ws);
  if (n == 0) return 0;
  uint32_t* near_cnt = reinterpret_cast<uint32_t*>(near_ws);
  uint32_t* near_list = near_cnt + 4;
  kmeans_near_reset<<<1, 64, 0, s>>>(near_cnt);
  const uint64_t waves = (n + 15) / 16;
  const uint64_t cap = 32 / kKmWaves * (uint64_t)num_cus();
  const uint64_t wg = (waves + kKmWaves - 1) / kKmWaves;
  const unsigned ga = (unsigned)(wg < cap ? wg : cap);
#define DR_KMA(KTV) kmeans_assign_kernel<KTV, kKmDepth><<<ga, 64 * kKmWaves, 0, s>>>(XH, xnorm, n, C, cnorm_ws, K, assign)
  if (K <= 16) DR_KMA(1);
  else if (K <= 32) DR_KMA(2);
  else if (K <= 48) DR_KMA(3);
  else DR_KMA(4);
#undef DR_KMA
  kmeans_near_list<<<grid_for(n, 256, 4096), 256, 0, s>>>(assign, n, near_cnt, near_list);
  kmeans_rerank_kernel<<<1024, 64, 0, s>>>(X, C, cnorm_ws, K, near_cnt, near_list, assign, nullptr, nullptr, n);
  const uint64_t mb = (n + 255) / 256;
  const uint64_t mcap = 4 * (uint64_t)num_cus();
  kmeans_movers_kernel<<<(unsigned)(mb < mcap ? mb : mcap), 256, 0, s>>>(X, n, assign, prev, K, S, cnt);
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
