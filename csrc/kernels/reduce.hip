// Whole-partition aggregates (K11) on CDNA4: Count/LongCount/Sum/Min/Max/Average/Any/All/
// Contains/First/Last/Single of one partition in ONE streaming pass over its columns.
//
// Reference: the partial stage of the two-stage aggregates (DryadLinqQueryGen.cs:3384-3395,
// DLinqBasicAggregateNode DryadLinqQueryNode.cs:2577) runs the per-partition operator of
// DryadLinqVertex.cs:1673-4697 (Count, Sum, Min, Max, Average, Any, All, First, Last, Single ...)
// as one C# loop per aggregate over the deserialised records.  Here every aggregate of a
// partition is one slot of a register accumulator array: each lane walks the columns with a
// grid-stride loop (4 independent loads in flight per column per lane), the wave folds its lanes
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

template <int M>
__global__ __launch_bounds__(256) void reduce_partial_kernel(RedSpec s, uint64_t n, int64_t* __restrict__ part) {
  int64_t acc[M];
#pragma unroll
  for (int a = 0; a < M; ++a) acc[a] = identity(s.op[a], is_f(s.vt[a]));
  const uint64_t stride = (uint64_t)gridDim.x * blockDim.x;
  uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
  // 4 rows per lane per trip: independent loads keep HBM busy
  for (; i + 3 * stride < n; i += 4 * stride) {
#pragma unroll
    for (int a = 0; a < M; ++a) {
      const int op = s.op[a], vt = s.vt[a];
      const bool f = is_f(vt);
      int64_t x[4];
      bool ok[4];
#pragma unroll
      for (int k = 0; k < 4; ++k) {
        const uint64_t r = i + k * stride;
        ok[k] = s.mask[a] == nullptr || s.mask[a][r] != 0;
        x[k] = element(op, vt, s.val[a], r);
      }
#pragma unroll
      for (int k = 0; k < 4; ++k)
        if (ok[k]) acc[a] = combine(op, f, acc[a], x[k]);
    }
  }
  for (; i < n; i += stride) {
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
  const unsigned g = grid_for(n, kBlock * 4, kMaxBlocks);
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
