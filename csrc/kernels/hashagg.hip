// Hash aggregation for low-cardinality GroupBy (K6 "GPU hash aggregation, LDS pre-aggregation";
// reference DryadLinqVertex.cs:437-585 hash group-by with a 16411-entry table).
//
// Every workgroup streams a contiguous slice of the (key, value columns) in ONE coalesced pass and
// folds it into a private open-addressing table in LDS (64-bit ds CAS on the key, ds atomics on the
// accumulators).  At the end the LDS table is merged into a global HBM table with one atomic per
// (workgroup, distinct key).  Keys that find no LDS slot (table full) go straight to the global
// table.  The sort-based path (radix sort + segmented reduce) stays the choice for
// high-cardinality keys; the caller picks from a sampled distinct count.
#include "common.h"

namespace {
constexpr int kMaxAggs = 8;
constexpr int kLdsSlots = 1024;
constexpr unsigned long long kEmpty = 0x8000000000000000ull;   // INT64_MIN marks a free slot
enum Op : int { SUM_I = 0, MIN_I = 1, MAX_I = 2, COUNT = 3, SUM_F = 4, MIN_F = 5, MAX_F = 6 };

struct HSpec {
  int op[kMaxAggs];
  const uint64_t* vals[kMaxAggs];
  uint64_t* gacc[kMaxAggs];   // [capacity + 1]; slot `capacity` holds the key INT64_MIN
};

__device__ __forceinline__ uint64_t identity(int op) {
  switch (op) {
    case MIN_I: return 0x7FFFFFFFFFFFFFFFull;
    case MAX_I: return 0x8000000000000000ull;
    case MIN_F: return (uint64_t)__double_as_longlong(__builtin_inf());
    case MAX_F: return (uint64_t)__double_as_longlong(-__builtin_inf());
    default: return 0ull;
  }
}

__device__ __forceinline__ void fmin_max_atomic(unsigned long long* p, double v, bool is_min) {
  unsigned long long old = *p, assumed;
  do {
    assumed = old;
    const double cur = __longlong_as_double((long long)assumed);
    const double nv = is_min ? (v < cur ? v : cur) : (v > cur ? v : cur);
    if (nv == cur) break;
    old = atomicCAS(p, assumed, (unsigned long long)__double_as_longlong(nv));
  } while (assumed != old);
}

// works for LDS and global pointers (generic address space)
__device__ __forceinline__ void combine_atomic(uint64_t* p, uint64_t v, int op) {
  unsigned long long* q = reinterpret_cast<unsigned long long*>(p);
  switch (op) {
    case SUM_I: case COUNT: atomicAdd(q, (unsigned long long)v); break;
    case MIN_I: atomicMin(reinterpret_cast<long long*>(p), (long long)v); break;
    case MAX_I: atomicMax(reinterpret_cast<long long*>(p), (long long)v); break;
    case SUM_F: atomicAdd(reinterpret_cast<double*>(p), __longlong_as_double((long long)v)); break;
    case MIN_F: fmin_max_atomic(q, __longlong_as_double((long long)v), true); break;
    default: fmin_max_atomic(q, __longlong_as_double((long long)v), false); break;
  }
}

__device__ __forceinline__ uint32_t hslot(uint64_t k, uint64_t mask) { return (uint32_t)(mix64(k) & mask); }

// global insert: returns the slot of key k (capacity is a power of two, load factor <= 1/2)
__device__ __forceinline__ uint64_t global_slot(unsigned long long* gkeys, uint64_t cap, uint64_t k, uint32_t* overflow) {
  if (k == kEmpty) return cap;
  uint64_t h = mix64(k) & (cap - 1);
  for (uint64_t probe = 0; probe < cap; ++probe) {
    const unsigned long long cur = gkeys[h];
    if (cur == k) return h;
    if (cur == kEmpty) {
      const unsigned long long prev = atomicCAS(&gkeys[h], kEmpty, (unsigned long long)k);
      if (prev == kEmpty || prev == k) return h;
    }
    h = (h + 1) & (cap - 1);
  }
  atomicOr(overflow, 1u);
  return cap;
}

__global__ __launch_bounds__(256) void hashagg_kernel(const int64_t* __restrict__ keys, uint64_t n, int nagg, HSpec sp,
                                                      unsigned long long* __restrict__ gkeys, uint64_t cap,
                                                      uint32_t* __restrict__ overflow) {
  extern __shared__ __attribute__((aligned(16))) unsigned long long smem_u64[];
  unsigned long long* lkey = smem_u64;                                  // [kLdsSlots]
  uint64_t* lacc = reinterpret_cast<uint64_t*>(smem_u64 + kLdsSlots);   // [kLdsSlots][nagg]
  const int t = threadIdx.x;
  for (int i = t; i < kLdsSlots; i += 256) {
    lkey[i] = kEmpty;
    for (int a = 0; a < nagg; ++a) lacc[i * nagg + a] = identity(sp.op[a]);
  }
  __syncthreads();
  const uint64_t per = (n + gridDim.x - 1) / gridDim.x;
  const uint64_t beg = (uint64_t)blockIdx.x * per;
  const uint64_t end = beg + per < n ? beg + per : n;
  for (uint64_t i = beg + t; i < end; i += 256) {
    const uint64_t k = (uint64_t)keys[i];
    int slot = -1;
    if (k != kEmpty) {
      uint32_t h = hslot(k, kLdsSlots - 1);
      for (int probe = 0; probe < 32; ++probe) {          // bounded probing, then spill to HBM
        const unsigned long long cur = lkey[h];
        if (cur == k) { slot = (int)h; break; }
        if (cur == kEmpty) {
          const unsigned long long prev = atomicCAS(&lkey[h], kEmpty, (unsigned long long)k);
          if (prev == kEmpty || prev == k) { slot = (int)h; break; }
        }
        h = (h + 1) & (kLdsSlots - 1);
      }
    }
    if (slot >= 0) {
      for (int a = 0; a < nagg; ++a)
        combine_atomic(&lacc[slot * nagg + a], sp.op[a] == COUNT ? 1ull : sp.vals[a][i], sp.op[a]);
    } else {
      const uint64_t g = global_slot(gkeys, cap, k, overflow);
      for (int a = 0; a < nagg; ++a)
        combine_atomic(sp.gacc[a] + g, sp.op[a] == COUNT ? 1ull : sp.vals[a][i], sp.op[a]);
    }
  }
  __syncthreads();
  for (int s = t; s < kLdsSlots; s += 256) {
    const unsigned long long k = lkey[s];
    if (k == kEmpty) continue;
    const uint64_t g = global_slot(gkeys, cap, k, overflow);
    for (int a = 0; a < nagg; ++a) combine_atomic(sp.gacc[a] + g, lacc[s * nagg + a], sp.op[a]);
  }
}
}  // namespace

// keys: int64 [n]; vals[a]: 64-bit columns (ignored for COUNT); gkeys [cap] preset to INT64_MIN;
// gaccs[a] [cap + 1] preset to each op's identity.  *overflow set if the global table filled up.
DR_API int dr_hash_aggregate(const int64_t* keys, uint64_t n, int nagg, const int* ops, const void* const* vals,
                             void* const* gaccs, unsigned long long* gkeys, uint64_t cap, uint32_t* overflow,
                             hipStream_t s) {
  if (nagg < 1 || nagg > kMaxAggs || cap == 0 || (cap & (cap - 1))) return (int)hipErrorInvalidValue;
  if (n == 0) return 0;
  HSpec sp;
  for (int a = 0; a < nagg; ++a) {
    sp.op[a] = ops[a];
    sp.vals[a] = reinterpret_cast<const uint64_t*>(vals[a]);
    sp.gacc[a] = reinterpret_cast<uint64_t*>(gaccs[a]);
  }
  int dev = 0, cus = 256;
  hipGetDevice(&dev);
  hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev);
  uint64_t blocks = (uint64_t)cus * 4;
  if (blocks * 1024 > n) blocks = (n + 1023) / 1024;
  if (blocks < 1) blocks = 1;
  const size_t smem = (size_t)kLdsSlots * (1 + nagg) * sizeof(uint64_t);
  hipFuncSetAttribute(reinterpret_cast<const void*>(hashagg_kernel), hipFuncAttributeMaxDynamicSharedMemorySize,
                      (int)smem);
  hashagg_kernel<<<(unsigned)blocks, 256, smem, s>>>(keys, n, nagg, sp, gkeys, cap, overflow);
  DR_LAUNCH_CHECK();
  return 0;
}
