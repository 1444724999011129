// Whole-partition aggregates (K11) on CDNA4: Count/LongCount/Sum/Min/Max/Average/Any/All/
// Contains/First/Last/Single of one partition in ONE streaming pass over its columns.
//
// Reference: the partial stage of the two-stage aggregates (DryadLinqQueryGen.cs:3384-3395,
// DLinqBasicAggregateNode DryadLinqQueryNode.cs:2577) runs the per-partition operator of
// DryadLinqVertex.cs:1673-4697 (Count, Sum, Min, Max, Average, Any, All, First, Last, Single ...)
// as one C# loop per aggregate over the deserialised records.  Here every aggregate of a
// partition is one slot of a register accumulator array: each lane walks the columns with a
// grid-stride loop (8 consecutive rows per lane per trip: 16-byte vector loads), the wave folds its lanes
// with xor shuffles, the workgroup folds its 4 waves in LDS, and a second single-workgroup
// kernel folds the per-workgroup partials in a fixed order (bit-reproducible float sums for a
// given partition size, no float atomics).
//
// Slots: op SUM/MIN/MAX over a value column (int64 / int32 / uint8-bool accumulate in int64,
// float64 / float32 in double), COUNT of rows, FIRST / LAST = smallest / largest row index.
// Every slot takes an optional bool mask (the traced predicate); masked-out rows do not count.
#include "common.h"

namespace {

constexpr int kMaxAgg = 8;
constexpr unsigned kMaxBlocks = 2048;   // 8 workgroups per CU on 256 CUs
enum { R_SUM = 0, R_MIN = 1, R_MAX = 2, R_COUNT = 3, R_FIRST = 4, R_LAST = 5 };
enum { V_I64 = 0, V_F64 = 1, V_I32 = 2, V_F32 = 3, V_U8 = 4, V_NONE = 5 };

struct RedSpec {
  int m;
  int op[kMaxAgg];
  int vt[kMaxAgg];
  const void* val[kMaxAgg];
  const uint8_t* mask[kMaxAgg];
  int vsame[kMaxAgg];   // slot reads the same value column as the slot before it (reuse the registers)
  int msame[kMaxAgg];   // same mask as the slot before it
};

__device__ __forceinline__ bool is_f(int vt) { return vt == V_F64 || vt == V_F32; }
__device__ __forceinline__ double as_d(int64_t x) { return __longlong_as_double(x); }
__device__ __forceinline__ int64_t as_i(double x) { return __double_as_longlong(x); }

__device__ __forceinline__ int64_t identity(int op, bool f) {
  switch (op) {
    case R_MIN: return f ? as_i(__builtin_inf()) : INT64_MAX;
    case R_MAX: return f ? as_i(-__builtin_inf()) : INT64_MIN;
    case R_FIRST: return INT64_MAX;
    case R_LAST: return -1;
    default: return f && op == R_SUM ? as_i(0.0) : 0;
  }
}

__device__ __forceinline__ int64_t combine(int op, bool f, int64_t a, int64_t b) {
  switch (op) {
    case R_SUM: return f ? as_i(as_d(a) + as_d(b)) : a + b;
    case R_MIN: return f ? as_i(fmin(as_d(a), as_d(b))) : (b < a ? b : a);
    case R_MAX: return f ? as_i(fmax(as_d(a), as_d(b))) : (b > a ? b : a);
    case R_COUNT: return a + b;
    case R_FIRST: return b < a ? b : a;
    default: return b > a ? b : a;   // R_LAST
  }
}

__device__ __forceinline__ int64_t shfl_xor64(int64_t v, int d) {
  return (int64_t)__shfl_xor((long long)v, d, 64);
}

// The contribution of row i to a slot (value bits in the slot's accumulator domain).
__device__ __forceinline__ int64_t element(int op, int vt, const void* p, uint64_t i) {
  if (op == R_COUNT) return 1;
  if (op == R_FIRST || op == R_LAST) return (int64_t)i;
  switch (vt) {
    case V_I64: return static_cast<const int64_t*>(p)[i];
    case V_F64: return static_cast<const int64_t*>(p)[i];          // already double bits
    case V_I32: return (int64_t) static_cast<const int32_t*>(p)[i];
    case V_F32: return as_i((double) static_cast<const float*>(p)[i]);
    default: return (int64_t) static_cast<const uint8_t*>(p)[i];
  }
}

typedef long long ll2_t __attribute__((ext_vector_type(2)));
typedef int i4_t __attribute__((ext_vector_type(4)));
typedef float f4_t __attribute__((ext_vector_type(4)));

// Rows base..base+7 of one slot's value column with 16-byte vector loads (the caller guarantees
// 16-byte aligned columns and base % 8 == 0).
__device__ __forceinline__ void load8(int op, int vt, const void* p, uint64_t base, int64_t* x) {
  if (op == R_COUNT) {
#pragma unroll
    for (int k = 0; k < 8; ++k) x[k] = 1;
    return;
  }
  if (op == R_FIRST || op == R_LAST) {
#pragma unroll
    for (int k = 0; k < 8; ++k) x[k] = (int64_t)(base + k);
    return;
  }
  switch (vt) {
    case V_I64:
    case V_F64: {
      const ll2_t* q = reinterpret_cast<const ll2_t*>(static_cast<const int64_t*>(p) + base);
#pragma unroll
      for (int j = 0; j < 4; ++j) {
        const ll2_t v = q[j];
        x[2 * j] = v.x;
        x[2 * j + 1] = v.y;
      }
      break;
    }
    case V_I32: {
      const i4_t* q = reinterpret_cast<const i4_t*>(static_cast<const int32_t*>(p) + base);
#pragma unroll
      for (int j = 0; j < 2; ++j) {
        const i4_t v = q[j];
        x[4 * j] = v.x; x[4 * j + 1] = v.y; x[4 * j + 2] = v.z; x[4 * j + 3] = v.w;
      }
      break;
    }
    case V_F32: {
      const f4_t* q = reinterpret_cast<const f4_t*>(static_cast<const float*>(p) + base);
#pragma unroll
      for (int j = 0; j < 2; ++j) {
        const f4_t v = q[j];
        x[4 * j] = as_i((double)v.x); x[4 * j + 1] = as_i((double)v.y);
        x[4 * j + 2] = as_i((double)v.z); x[4 * j + 3] = as_i((double)v.w);
      }
      break;
    }
    default: {
      const uint64_t w = *reinterpret_cast<const uint64_t*>(static_cast<const uint8_t*>(p) + base);
#pragma unroll
      for (int k = 0; k < 8; ++k) x[k] = (int64_t)((w >> (8 * k)) & 0xFF);
    }
  }
}

template <int M>
__global__ __launch_bounds__(256) void reduce_partial_kernel(RedSpec s, uint64_t n, int64_t* __restrict__ part) {
  int64_t acc[M];
#pragma unroll
  for (int a = 0; a < M; ++a) acc[a] = identity(s.op[a], is_f(s.vt[a]));
  const uint64_t tid = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
  const uint64_t nthr = (uint64_t)gridDim.x * blockDim.x;
  const uint64_t n8 = n & ~7ull;
  // 8 consecutive rows per lane per trip: 16-byte loads of every slot's column, one 8-byte load
  // of its mask bytes
  // (Sum / Min / Max of one column, or several slots under one predicate, load it once)
  for (uint64_t base = tid * 8; base < n8; base += nthr * 8) {
    int64_t x[8];
    uint64_t mw = 0;
#pragma unroll
    for (int a = 0; a < M; ++a) {
      const int op = s.op[a];
      const bool f = is_f(s.vt[a]);
      if (!(a > 0 && s.vsame[a])) load8(op, s.vt[a], s.val[a], base, x);
      if (!(a > 0 && s.msame[a]))
        mw = s.mask[a] ? *reinterpret_cast<const uint64_t*>(s.mask[a] + base) : 0x0101010101010101ull;
#pragma unroll
      for (int k = 0; k < 8; ++k) {
        const int64_t c = combine(op, f, acc[a], x[k]);
        acc[a] = ((mw >> (8 * k)) & 0xFF) ? c : acc[a];
      }
    }
  }
  for (uint64_t i = n8 + tid; i < n; i += nthr) {
#pragma unroll
    for (int a = 0; a < M; ++a) {
      if (s.mask[a] != nullptr && s.mask[a][i] == 0) continue;
      acc[a] = combine(s.op[a], is_f(s.vt[a]), acc[a], element(s.op[a], s.vt[a], s.val[a], i));
    }
  }
  __shared__ int64_t red[4][M];
  const int w = wave_id(), l = lane_id();
#pragma unroll
  for (int a = 0; a < M; ++a) {
    const int op = s.op[a];
    const bool f = is_f(s.vt[a]);
    int64_t v = acc[a];
#pragma unroll
    for (int d = 32; d >= 1; d >>= 1) v = combine(op, f, v, shfl_xor64(v, d));
    if (l == 0) red[w][a] = v;
  }
  __syncthreads();
  if (threadIdx.x < M) {
    const int a = threadIdx.x;
    const int op = s.op[a];
    const bool f = is_f(s.vt[a]);
    int64_t v = red[0][a];
    for (int k = 1; k < 4; ++k) v = combine(op, f, v, red[k][a]);
    part[(uint64_t)blockIdx.x * kMaxAgg + a] = v;
  }
}

// One workgroup folds the per-workgroup partials (fixed order -> reproducible).
__global__ __launch_bounds__(256) void reduce_final_kernel(RedSpec s, unsigned nblocks, const int64_t* __restrict__ part,
                                                           int64_t* __restrict__ out) {
  __shared__ int64_t red[4][kMaxAgg];
  const int w = wave_id(), l = lane_id();
  for (int a = 0; a < s.m; ++a) {
    const int op = s.op[a];
    const bool f = is_f(s.vt[a]);
    int64_t v = identity(op, f);
    for (unsigned b = threadIdx.x; b < nblocks; b += blockDim.x) v = combine(op, f, v, part[(uint64_t)b * kMaxAgg + a]);
#pragma unroll
    for (int d = 32; d >= 1; d >>= 1) v = combine(op, f, v, shfl_xor64(v, d));
    if (l == 0) red[w][a] = v;
  }
  __syncthreads();
  if (threadIdx.x < (unsigned)s.m) {
    const int a = threadIdx.x;
    const int op = s.op[a];
    const bool f = is_f(s.vt[a]);
    int64_t v = red[0][a];
    for (int k = 1; k < 4; ++k) v = combine(op, f, v, red[k][a]);
    out[a] = v;
  }
}

template <int M>
void launch_partial(const RedSpec& s, uint64_t n, unsigned g, int64_t* part, hipStream_t st) {
  hipLaunchKernelGGL(reduce_partial_kernel<M>, dim3(g), dim3(kBlock), 0, st, s, n, part);
}

}  // namespace

DR_API uint64_t dr_reduce_workspace() { return (uint64_t)kMaxBlocks * kMaxAgg * sizeof(int64_t); }

// m (1..8) aggregate slots over n rows.  ops/vts/vals/masks: per slot.  out: int64[m] holding the
// result bits (double bits for float slots).  ws: dr_reduce_workspace() bytes of device memory.
DR_API int dr_reduce_multi(int m, const int* ops, const int* vts, const void* const* vals, const void* const* masks,
                           uint64_t n, int64_t* out, void* ws, hipStream_t st) {
  if (m < 1 || m > kMaxAgg) return (int)hipErrorInvalidValue;
  RedSpec s{};
  s.m = m;
  for (int a = 0; a < kMaxAgg; ++a) {
    const int b = a < m ? a : m - 1;      // pad unused slots with a copy (never read back)
    s.op[a] = ops[b];
    s.vt[a] = vts[b];
    s.val[a] = vals[b];
    s.mask[a] = static_cast<const uint8_t*>(masks[b]);
    if (s.op[a] < R_SUM || s.op[a] > R_LAST || s.vt[a] < V_I64 || s.vt[a] > V_NONE) return (int)hipErrorInvalidValue;
    if ((s.op[a] == R_SUM || s.op[a] == R_MIN || s.op[a] == R_MAX) && (s.vt[a] == V_NONE || s.val[a] == nullptr))
      return (int)hipErrorInvalidValue;
  }
  for (int a = 1; a < kMaxAgg; ++a) {
    const bool valued = s.op[a] == R_SUM || s.op[a] == R_MIN || s.op[a] == R_MAX;
    const bool pvalued = s.op[a - 1] == R_SUM || s.op[a - 1] == R_MIN || s.op[a - 1] == R_MAX;
    s.vsame[a] = (valued && pvalued && s.val[a] == s.val[a - 1] && s.vt[a] == s.vt[a - 1]) ||
                 (s.op[a] == s.op[a - 1] && !valued);
    s.msame[a] = s.mask[a] == s.mask[a - 1];
  }
  const unsigned g = grid_for(n, kBlock * 8, kMaxBlocks);
  int64_t* part = static_cast<int64_t*>(ws);
  switch (m) {
    case 1: launch_partial<1>(s, n, g, part, st); break;
    case 2: launch_partial<2>(s, n, g, part, st); break;
    case 3: launch_partial<3>(s, n, g, part, st); break;
    case 4: launch_partial<4>(s, n, g, part, st); break;
    default: launch_partial<8>(s, n, g, part, st); break;
  }
  DR_LAUNCH_CHECK();
  hipLaunchKernelGGL(reduce_final_kernel, dim3(1), dim3(kBlock), 0, st, s, g, part, out);
  DR_LAUNCH_CHECK();
  return 0;
}
