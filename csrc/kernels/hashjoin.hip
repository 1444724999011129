// Device hash join (K8) for CDNA4: a bucketed (CSR) hash table built over the inner side's
// key entries, probed by the outer side.
//
// Reference: DryadLinqVertex.HashJoin (DryadLinqVertex.cs:852-897) and ParallelHashJoin
// (:6703-7315) build a hash lookup of the (co-partitioned) inner records and stream the outer
// records through it, emitting resultSelector(outer, inner) for every match, outer order first.
//
// Build: no atomics on the table itself and a deterministic layout.
//   hj_slots   slot(key) = top log2(cap) bits of a 64-bit mix of the key (cap >= 2 * inner rows);
//              writes the entry (lo = inner position, hi = slot) and bumps a per-slot histogram
//   stable LSD radix sort of those entries on the slot bits                 [dr_sort_u128]
//   exclusive scan of the histogram = CSR bucket starts                     [dr_scan_i64]
//   hj_gather  bucket-ordered copy of the inner key entries, so a probe reads ONE contiguous run
//              (16-byte entries: the average bucket of <= 0.5 entries is one cache line)
// Probe: one lane per outer row hashes its key, reads starts[slot..slot+1] and compares the full
// key (hi, lo & mask) of every entry of the bucket.  Pass 1 counts matches, a scan turns the
// counts into output offsets, pass 2 writes (outer row, inner row) pairs.  Because the sort is
// stable, matches come out in outer row order and, per outer row, in inner row order — the LINQ
// Join order of the reference's LocalDebug path.
#include "common.h"

namespace {

__device__ __forceinline__ uint64_t key_hash(uint64_t hi, uint64_t lo) {
  return mix64(hi ^ mix64(lo ^ 0x5851F42D4C957F2Dull));
}

__device__ __forceinline__ uint64_t slot_of(uint64_t hi, uint64_t lo, int log_cap) {
  return key_hash(hi, lo) >> (64 - log_cap);
}

__global__ __launch_bounds__(256) void hj_slots_kernel(const E128* __restrict__ inner, uint64_t n, uint64_t lo_mask,
                                                       int log_cap, E128* __restrict__ out,
                                                       unsigned long long* __restrict__ hist) {
  const uint64_t stride = (uint64_t)gridDim.x * blockDim.x;
  for (uint64_t j = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; j < n; j += stride) {
    const E128 e = inner[j];
    const uint64_t s = slot_of(e.hi, e.lo & lo_mask, log_cap);
    E128 o;
    o.lo = j;
    o.hi = s;
    out[j] = o;
    atomicAdd(&hist[s], 1ull);
  }
}

__global__ __launch_bounds__(256) void hj_gather_kernel(const E128* __restrict__ sorted, uint64_t n,
                                                        const E128* __restrict__ inner, E128* __restrict__ keys) {
  const uint64_t stride = (uint64_t)gridDim.x * blockDim.x;
  for (uint64_t k = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; k < n; k += stride)
    keys[k] = inner[sorted[k].lo];
}

template <bool EMIT>
__global__ __launch_bounds__(256) void hj_probe_kernel(const E128* __restrict__ outer, uint64_t no,
                                                       const E128* __restrict__ keys,
                                                       const int64_t* __restrict__ starts, int log_cap,
                                                       uint64_t lo_mask, int64_t* __restrict__ count,
                                                       const int64_t* __restrict__ offs, int64_t* __restrict__ oo,
                                                       int64_t* __restrict__ ii) {
  const uint64_t stride = (uint64_t)gridDim.x * blockDim.x;
  for (uint64_t o = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; o < no; o += stride) {
    const E128 e = outer[o];
    const uint64_t klo = e.lo & lo_mask;
    const uint64_t s = slot_of(e.hi, klo, log_cap);
    const int64_t a = starts[s], b = starts[s + 1];
    const int64_t base = EMIT ? offs[o] : 0;
    const int64_t orow = (int64_t)(uint32_t)e.lo;
    int64_t c = 0;
    for (int64_t k = a; k < b; ++k) {
      const E128 x = keys[k];
      if (x.hi == e.hi && (x.lo & lo_mask) == klo) {
        if (EMIT) {
          oo[base + c] = orow;
          ii[base + c] = (int64_t)(uint32_t)x.lo;
        }
        ++c;
      }
    }
    if (!EMIT) count[o] = c;
  }
}

}  // namespace

// inner [n] E128 key entries (row index in the low 32 bits of lo) -> out [n] (lo = position,
// hi = slot); hist [2^log_cap + 1] zeroed by the caller.
DR_API int dr_hj_slots(const E128* inner, uint64_t n, uint64_t lo_mask, int log_cap, E128* out,
                       unsigned long long* hist, hipStream_t st) {
  if (log_cap < 1 || log_cap > 40) return (int)hipErrorInvalidValue;
  if (n == 0) return 0;
  hipLaunchKernelGGL(hj_slots_kernel, dim3(grid_for(n, kBlock * 4)), dim3(kBlock), 0, st, inner, n, lo_mask, log_cap,
                     out, hist);
  DR_LAUNCH_CHECK();
  return 0;
}

// keys[k] = inner[sorted[k].lo]
DR_API int dr_hj_gather(const E128* sorted, uint64_t n, const E128* inner, E128* keys, hipStream_t st) {
  if (n == 0) return 0;
  hipLaunchKernelGGL(hj_gather_kernel, dim3(grid_for(n, kBlock * 4)), dim3(kBlock), 0, st, sorted, n, inner, keys);
  DR_LAUNCH_CHECK();
  return 0;
}

// emit = 0: count[o] = number of inner matches of outer[o]; emit = 1: write the pairs at offs[o].
DR_API int dr_hj_probe(const E128* outer, uint64_t no, const E128* keys, const int64_t* starts, int log_cap,
                       uint64_t lo_mask, int64_t* count, const int64_t* offs, int64_t* oo, int64_t* ii, int emit,
                       hipStream_t st) {
  if (log_cap < 1 || log_cap > 40) return (int)hipErrorInvalidValue;
  if (no == 0) return 0;
  const unsigned g = grid_for(no, kBlock * 4);
  if (emit)
    hipLaunchKernelGGL(hj_probe_kernel<true>, dim3(g), dim3(kBlock), 0, st, outer, no, keys, starts, log_cap, lo_mask,
                       count, offs, oo, ii);
  else
    hipLaunchKernelGGL(hj_probe_kernel<false>, dim3(g), dim3(kBlock), 0, st, outer, no, keys, starts, log_cap,
                       lo_mask, count, offs, oo, ii);
  DR_LAUNCH_CHECK();
  return 0;
}
