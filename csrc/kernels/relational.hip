// Relational kernels for the GPU vertex operator library (gfx950).
//
//   dr_build_keys       : up to 4 typed key columns -> order-preserving 128-bit sort entries
//                         (normalised keys in the top bits, row index in the low 32 bits)
//   dr_hash_dest        : hash of the key bits -> destination partition in entry.hi (HashPartition,
//                         reference DryadLinqVertex.cs:4788-4907 port = hash % nPorts)
//   dr_segment_flags    : 1 where the key differs from the previous sorted entry (GroupBy /
//                         Distinct boundaries, ordered-GroupBy adjacent difference :586-760)
//   dr_seg_reduce       : segmented sum/min/max/count over rows in sorted order, wave-level
//                         segmented scan with 64-bit shuffles then one atomic per run tail
//   dr_join_ranges      : for each sorted outer key, [lower, upper) among sorted inner keys
//   dr_join_emit        : expand the ranges into (outer row, inner row) pairs (MergeJoin :898-1162)
//   dr_scan_i64         : exclusive prefix sum of int64 (any length, reduce-then-scan)
#include "common.h"

namespace {

enum KeyType : int {
  K_U8 = 0, K_I8 = 1, K_BOOL = 2, K_I16 = 3, K_U16 = 4, K_I32 = 5, K_U32 = 6, K_I64 = 7, K_U64 = 8, K_F32 = 9,
  K_F64 = 10
};

__device__ __forceinline__ int key_bits(int t) {
  switch (t) {
    case K_U8: case K_I8: case K_BOOL: return 8;
    case K_I16: case K_U16: return 16;
    case K_I32: case K_U32: case K_F32: return 32;
    default: return 64;
  }
}

// order-preserving unsigned image of one key value
__device__ __forceinline__ uint64_t norm_key(const void* col, uint64_t i, int t) {
  switch (t) {
    case K_U8: case K_BOOL: return ((const uint8_t*)col)[i];
    case K_I8: return (uint8_t)(((const int8_t*)col)[i]) ^ 0x80u;
    case K_I16: return (uint16_t)(((const int16_t*)col)[i]) ^ 0x8000u;
    case K_U16: return ((const uint16_t*)col)[i];
    case K_I32: return (uint32_t)(((const int32_t*)col)[i]) ^ 0x80000000u;
    case K_U32: return ((const uint32_t*)col)[i];
    case K_I64: return (uint64_t)(((const int64_t*)col)[i]) ^ 0x8000000000000000ull;
    case K_U64: return ((const uint64_t*)col)[i];
    // -0.0 folds into +0.0 and every NaN into one canonical NaN, so equality consumers
    // (GroupBy / Distinct / Join) see the host's notion of equal floats
    case K_F32: {
      uint32_t u = ((const uint32_t*)col)[i];
      if (u == 0x80000000u) u = 0;
      if ((u & 0x7F800000u) == 0x7F800000u && (u & 0x007FFFFFu)) u = 0x7FC00000u;
      return (u & 0x80000000u) ? (uint32_t)~u : (u | 0x80000000u);
    }
    case K_F64: {
      uint64_t u = ((const uint64_t*)col)[i];
      if (u == 0x8000000000000000ull) u = 0;
      if ((u & 0x7FF0000000000000ull) == 0x7FF0000000000000ull && (u & 0x000FFFFFFFFFFFFFull))
        u = 0x7FF8000000000000ull;
      return (u & 0x8000000000000000ull) ? ~u : (u | 0x8000000000000000ull);
    }
  }
  return 0;
}

struct KeyCols {
  const void* col[4];
  int type[4];
  int desc[4];
  int ncols;
};

__global__ __launch_bounds__(256) void build_keys_kernel(KeyCols kc, uint64_t n, uint32_t idx_base, int total_bits,
                                                         E128* __restrict__ out) {
  for (uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (uint64_t)gridDim.x * blockDim.x) {
    unsigned __int128 k = 0;
    for (int c = 0; c < kc.ncols; ++c) {
      const int b = key_bits(kc.type[c]);
      uint64_t v = norm_key(kc.col[c], i, kc.type[c]);
      if (kc.desc[c]) v = ~v & (b == 64 ? ~0ull : ((1ull << b) - 1));
      k = (k << b) | v;
    }
    k <<= (128 - total_bits);
    E128 e;
    e.hi = (uint64_t)(k >> 64);
    e.lo = (uint64_t)k | (uint32_t)(idx_base + (uint32_t)i);
    out[i] = e;
  }
}

__global__ __launch_bounds__(256) void hash_dest_kernel(E128* __restrict__ e, uint64_t n, uint64_t lo_mask,
                                                        uint32_t nparts) {
  for (uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (uint64_t)gridDim.x * blockDim.x) {
    E128 x = e[i];
    const uint64_t h = mix64(x.hi ^ mix64(x.lo & lo_mask));
    x.hi = (uint32_t)((h >> 32) % nparts);
    e[i] = x;
  }
}

__global__ __launch_bounds__(256) void segment_flags_kernel(const E128* __restrict__ e, uint64_t n, uint64_t lo_mask,
                                                            int64_t* __restrict__ flags) {
  for (uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (uint64_t)gridDim.x * blockDim.x) {
    int64_t f = 1;
    if (i > 0) {
      const E128 a = e[i - 1], b = e[i];
      f = (a.hi != b.hi || (a.lo & lo_mask) != (b.lo & lo_mask)) ? 1 : 0;
    }
    flags[i] = f;
  }
}

// ----- segmented reduction -------------------------------------------------------------------
template <typename T>
struct OpSum { __device__ static T f(T a, T b) { return a + b; } };
template <typename T>
struct OpMin { __device__ static T f(T a, T b) { return b < a ? b : a; } };
template <typename T>
struct OpMax { __device__ static T f(T a, T b) { return b > a ? b : a; } };

__device__ __forceinline__ void atomic_combine(int64_t* p, int64_t v, int op) {
  unsigned long long* q = reinterpret_cast<unsigned long long*>(p);
  if (op == 0 || op == 3) { atomicAdd(q, (unsigned long long)v); return; }
  if (op == 1) { atomicMin(reinterpret_cast<long long*>(p), (long long)v); return; }
  atomicMax(reinterpret_cast<long long*>(p), (long long)v);
}

__device__ __forceinline__ void atomic_combine(double* p, double v, int op) {
  if (op == 0 || op == 3) { atomicAdd(p, v); return; }
  unsigned long long* q = reinterpret_cast<unsigned long long*>(p);
  unsigned long long old = *q, assumed;
  do {
    assumed = old;
    const double cur = __longlong_as_double((long long)assumed);
    const double nv = (op == 1) ? (v < cur ? v : cur) : (v > cur ? v : cur);
    if (nv == cur) break;
    old = atomicCAS(q, assumed, (unsigned long long)__double_as_longlong(nv));
  } while (assumed != old);
}

template <typename T, typename Op>
__device__ __forceinline__ void seg_reduce_body(const T* __restrict__ vals, const E128* __restrict__ ent,
                                                const int64_t* __restrict__ seg, uint64_t n, T* __restrict__ out,
                                                int op, T ident) {
  const int lane = lane_id();
  const uint64_t waves = ((uint64_t)gridDim.x * blockDim.x) >> 6;
  const uint64_t w0 = (((uint64_t)blockIdx.x * blockDim.x) + threadIdx.x) >> 6;
  for (uint64_t base = w0 * 64; base < n; base += waves * 64) {
    const uint64_t i = base + lane;
    const bool valid = i < n;
    T v = ident;
    int64_t s = -1;
    if (valid) {
      const uint32_t row = ent ? (uint32_t)ent[i].lo : (uint32_t)i;
      v = (op == 3) ? (T)1 : vals[row];
      s = seg[i];
    }
#pragma unroll
    for (int d = 1; d < 64; d <<= 1) {
      const T o = __shfl_up(v, d, 64);
      const int64_t os = __shfl_up(s, d, 64);
      if (lane >= d && os == s) v = Op::f(v, o);
    }
    const int64_t ns = __shfl_down(s, 1, 64);
    const bool tail = valid && (lane == 63 || i + 1 >= n || ns != s);
    if (tail) atomic_combine(&out[s], v, op);
  }
}

template <typename T>
__global__ __launch_bounds__(256) void seg_reduce_kernel(const T* vals, const E128* ent, const int64_t* seg, uint64_t n,
                                                         T* out, int op, T ident) {
  if (op == 1) seg_reduce_body<T, OpMin<T>>(vals, ent, seg, n, out, op, ident);
  else if (op == 2) seg_reduce_body<T, OpMax<T>>(vals, ent, seg, n, out, op, ident);
  else seg_reduce_body<T, OpSum<T>>(vals, ent, seg, n, out, op, ident);
}

// ----- fused multi-aggregate segmented reduction ------------------------------------------------
// One pass over the sorted entries computes up to 8 aggregates (GroupBy's Count/Sum/Min/Max of
// several columns): the segmented-scan predicates are computed once per wave and shared by all
// aggregates, and a segment that starts and ends inside one wave (the common case: most groups
// are short) is written with a plain store; only segments crossing a wave boundary use atomics.
enum MultiOp : int { M_SUM_I = 0, M_MIN_I = 1, M_MAX_I = 2, M_COUNT = 3, M_SUM_F = 4, M_MIN_F = 5, M_MAX_F = 6 };
constexpr int kMaxAggs = 8;
struct AggSpecs {
  int op[kMaxAggs];
  const uint64_t* vals[kMaxAggs];
  uint64_t* out[kMaxAggs];
  uint32_t stride[kMaxAggs];   // elements between consecutive records (1 = column, k = AoS row)
  const uint64_t* rows;        // packed 32-byte rows shared by every value aggregate (or nullptr):
  uint32_t word[kMaxAggs];     // then aggregate a reads word[a] of row r, loaded as two 16-byte vectors
};

__device__ __forceinline__ uint64_t m_combine(uint64_t a, uint64_t b, int op) {
  switch (op) {
    case M_SUM_I: case M_COUNT: return a + b;
    case M_MIN_I: return (int64_t)b < (int64_t)a ? b : a;
    case M_MAX_I: return (int64_t)b > (int64_t)a ? b : a;
    case M_SUM_F: return (uint64_t)__double_as_longlong(__longlong_as_double((long long)a) + __longlong_as_double((long long)b));
    case M_MIN_F: {
      const double x = __longlong_as_double((long long)a), y = __longlong_as_double((long long)b);
      return y < x ? b : a;
    }
    default: {
      const double x = __longlong_as_double((long long)a), y = __longlong_as_double((long long)b);
      return y > x ? b : a;
    }
  }
}

__device__ __forceinline__ void m_atomic(uint64_t* p, uint64_t v, int op) {
  switch (op) {
    case M_SUM_I: case M_COUNT: atomicAdd(reinterpret_cast<unsigned long long*>(p), (unsigned long long)v); break;
    case M_MIN_I: atomicMin(reinterpret_cast<long long*>(p), (long long)v); break;
    case M_MAX_I: atomicMax(reinterpret_cast<long long*>(p), (long long)v); break;
    case M_SUM_F: atomicAdd(reinterpret_cast<double*>(p), __longlong_as_double((long long)v)); break;
    default: atomic_combine(reinterpret_cast<double*>(p), __longlong_as_double((long long)v), op == M_MIN_F ? 1 : 2);
  }
}


// Thread-serial variant: each lane reduces PER consecutive sorted elements on its own (segments
// that start and end inside the lane are written directly), and only the per-lane tail partials
// take part in a 64-lane segmented scan — 1/PER of the cross-lane traffic of the per-element
// scan above.  Segments touching the chunk boundary are combined with atomics.
// KEYS (fused segment ids): no segment-id array.  The entries are sorted E128 {lo = row, hi =
// key} (lo_mask 0, one 64-bit key word); a lane derives its elements' segment ids from key changes
// + a wave prefix of its start counts + chunk_base[chunk] (exclusive scan of
// dr_group_chunk_starts), and writes every group's key (hi ^ key_xor) at its start.
template <int PER, int NAGG, bool PACKED, bool KEYS = false>
__global__ __launch_bounds__(256) void seg_reduce_multi_serial(const E128* __restrict__ ent,
                                                               const int64_t* __restrict__ seg, uint64_t n,
                                                               AggSpecs sp,
                                                               const int64_t* __restrict__ chunk_base = nullptr,
                                                               uint64_t key_xor = 0,
                                                               uint64_t* __restrict__ keys_out = nullptr) {
  constexpr uint64_t kChunkElems = 64 * PER;
  const int lane = lane_id();
  const uint64_t waves = ((uint64_t)gridDim.x * blockDim.x) >> 6;
  const uint64_t w0 = (((uint64_t)blockIdx.x * blockDim.x) + threadIdx.x) >> 6;
  // KEYS: the next chunk's sorted entries are loaded while this chunk's permuted rows are in
  // flight (clamped, unconditional loads: an element past n re-reads entry n - 1 and is masked by
  // cnt), so a wave waits for one HBM round trip per chunk instead of two
  uint64_t pk[KEYS ? PER : 1];
  uint32_t pr[KEYS ? PER : 1];
  auto prefetch = [&](uint64_t cb) {
    if constexpr (KEYS) {
      const uint64_t f0 = cb + (uint64_t)lane * PER;
#pragma unroll
      for (int k = 0; k < PER; ++k) {
        const uint64_t i = f0 + k < n ? f0 + k : n - 1;
        const E128 x = ent[i];
        pk[k] = x.hi;
        pr[k] = (uint32_t)x.lo;
      }
    }
  };
  if (KEYS && n) prefetch(w0 * kChunkElems < n ? w0 * kChunkElems : 0);
  for (uint64_t cbase = w0 * kChunkElems; cbase < n; cbase += waves * kChunkElems) {
    const uint64_t first = cbase + (uint64_t)lane * PER;
    int64_t sid[PER];
    uint32_t row[PER];
    int cnt = 0;
    const uint64_t cend = (cbase + kChunkElems < n) ? cbase + kChunkElems : n;
    int64_t chunk_first, chunk_last;
    bool open_left, open_right;
    if constexpr (KEYS) {
      uint64_t kh[PER];
      uint32_t f[PER];
      cnt = first < n ? (int)((n - first) < (uint64_t)PER ? (n - first) : (uint64_t)PER) : 0;
#pragma unroll
      for (int k = 0; k < PER; ++k) {
        kh[k] = pk[k];
        row[k] = pr[k];
      }
      // key of the element before the lane's first: the previous lane's last (lane 0: a load)
      uint64_t prev = __shfl_up(kh[PER - 1], 1, 64);
      if (lane == 0 && first > 0) prev = ent[first - 1].hi;
      uint32_t c = 0;
#pragma unroll
      for (int k = 0; k < PER; ++k) {
        const uint64_t pk = k == 0 ? prev : kh[k - 1];
        f[k] = (k < cnt && (first + k == 0 || kh[k] != pk)) ? 1u : 0u;
        c += f[k];
      }
      const uint64_t incl = wave_inclusive_scan64((uint64_t)c);
      const int64_t b0 = chunk_base[cbase / kChunkElems] + (int64_t)(incl - c);
      uint32_t run = 0;
#pragma unroll
      for (int k = 0; k < PER; ++k) {
        run += f[k];
        if (k < cnt) {
          sid[k] = b0 + (int64_t)run - 1;
          if (f[k]) keys_out[sid[k]] = kh[k] ^ key_xor;
        } else {
          sid[k] = INT64_MIN + (int64_t)(lane * PER + k);   // unique, never matches
        }
      }
      const uint64_t total = __shfl(incl, 63, 64);
      chunk_first = __shfl(sid[0], 0, 64);
      chunk_last = chunk_base[cbase / kChunkElems] + (int64_t)total - 1;
      open_left = cbase > 0 && __shfl(f[0], 0, 64) == 0u;
      open_right = cend < n && ent[cend].hi == ent[cend - 1].hi;
    } else {
#pragma unroll
      for (int k = 0; k < PER; ++k) {
        const uint64_t i = first + k;
        if (i < n) {
          sid[k] = seg[i];
          row[k] = ent ? (uint32_t)ent[i].lo : (uint32_t)i;
          cnt = k + 1;
        } else {
          sid[k] = INT64_MIN + (int64_t)(lane * PER + k);   // unique, never matches
          row[k] = 0;
        }
      }
      // segments continuing across the chunk boundary must be combined atomically
      chunk_first = seg[cbase];
      chunk_last = seg[cend - 1];
      open_left = cbase > 0 && seg[cbase - 1] == chunk_first;
      open_right = cend < n && seg[cend] == chunk_last;
    }
    const int64_t head_id = sid[0], tail_id = sid[PER - 1];
    const int64_t prev_tail = __shfl_up(tail_id, 1, 64);
    const int64_t next_head = __shfl_down(head_id, 1, 64);
    const bool carry_in = lane > 0 && prev_tail == head_id;
    const bool tail_continues = (lane < 63) ? (next_head == tail_id) : false;
    // lane-level scan predicates (key equality of tail ids), shared by all aggregates
    uint32_t same = 0;
#pragma unroll
    for (int k = 0, d = 1; d < 64; d <<= 1, ++k) {
      const int64_t o = __shfl_up(tail_id, d, 64);
      if (lane >= d && o == tail_id) same |= 1u << k;
    }
    // every aggregate's permuted (random) loads are issued up front, PER x NAGG per lane in flight
    // (with packed rows the NAGG loads of one row hit the same 32-byte sector together)
    typedef unsigned long long u2_t __attribute__((ext_vector_type(2)));
    // PACKED: one 32-byte row per sorted entry, 2 vector loads instead of one load per aggregate;
    // else every aggregate's permuted loads.  Either way all loads are issued up front.
    u2_t r0[PACKED ? PER : 1], r1[PACKED ? PER : 1];
    uint64_t vv[PACKED ? 1 : NAGG][PER];
    if constexpr (PACKED) {
#pragma unroll
      for (int k = 0; k < PER; ++k) {
        if (k < cnt) {
          const u2_t* q = reinterpret_cast<const u2_t*>(sp.rows + (uint64_t)row[k] * 4);
          r0[k] = q[0];
          r1[k] = q[1];
        } else {
          r0[k] = u2_t{0ull, 0ull};
          r1[k] = u2_t{0ull, 0ull};
        }
      }
      if constexpr (KEYS) {
        const uint64_t nb = cbase + waves * kChunkElems;
        prefetch(nb < n ? nb : cbase);
      }
    } else {
#pragma unroll
      for (int a = 0; a < NAGG; ++a) {
        const int op = sp.op[a];
#pragma unroll
        for (int k = 0; k < PER; ++k)
          vv[a][k] = (k < cnt) ? ((op == M_COUNT) ? 1ull : sp.vals[a][(uint64_t)row[k] * sp.stride[a]]) : 0ull;
      }
    }
#pragma unroll
    for (int a = 0; a < NAGG; ++a) {
      const int op = sp.op[a];
      uint64_t v[PER];
      if constexpr (PACKED) {
        const uint32_t wd = sp.word[a];
#pragma unroll
        for (int k = 0; k < PER; ++k) {
          const uint64_t x = wd == 0 ? r0[k].x : wd == 1 ? r0[k].y : wd == 2 ? r1[k].x : r1[k].y;
          v[k] = (k < cnt) ? ((op == M_COUNT) ? 1ull : x) : 0ull;
        }
      } else {
#pragma unroll
        for (int k = 0; k < PER; ++k) v[k] = vv[a][k];
      }
      // serial pass over the lane's runs
      uint64_t acc = v[0];
      uint64_t head_val = 0;
      bool head_done = false;
#pragma unroll
      for (int k = 1; k < PER; ++k) {
        if (k < cnt && sid[k] == sid[k - 1]) {
          acc = m_combine(acc, v[k], op);
        } else {
          if (!head_done) {           // first run of the lane ends at k-1
            head_val = acc;
            head_done = true;
          } else if (k - 1 < cnt) {   // an interior run, entirely inside this lane
            const int64_t s_ = sid[k - 1];
            if ((s_ == chunk_first && open_left) || (s_ == chunk_last && open_right)) m_atomic(sp.out[a] + s_, acc, op);
            else sp.out[a][s_] = acc;
          }
          acc = v[k];
        }
      }
      const uint64_t tail_val = acc;   // last run of the lane (== first run if the lane has one run)
      // inclusive segmented scan of tail partials across lanes
      uint64_t S = tail_val;
#pragma unroll
      for (int k = 0, d = 1; d < 64; d <<= 1, ++k) {
        const uint64_t o = __shfl_up(S, d, 64);
        if (same & (1u << k)) S = m_combine(S, o, op);
      }
      const uint64_t carry = __shfl_up(S, 1, 64);
      if (cnt == 0) continue;
      if (head_done) {
        // the lane's first run ends inside the lane: carry (if any) + head partial
        const uint64_t hv = carry_in ? m_combine(carry, head_val, op) : head_val;
        if ((head_id == chunk_first && open_left) || (head_id == chunk_last && open_right)) m_atomic(sp.out[a] + head_id, hv, op);
        else sp.out[a][head_id] = hv;
      }
      // the lane's last run: written by the lane where the segment ends (S already includes
      // every earlier lane's share of it)
      // (a lane cut short by the end of the array already wrote all its runs in the serial pass)
      if (cnt == PER && !tail_continues) {
        const int64_t s_ = tail_id;
        if ((s_ == chunk_first && open_left) || (s_ == chunk_last && open_right)) m_atomic(sp.out[a] + s_, S, op);
        else sp.out[a][s_] = S;
      }
    }
  }
}

// ----- merge join ----------------------------------------------------------------------------
__device__ __forceinline__ bool key_less(const E128& a, const E128& b, uint64_t m) {
  return a.hi < b.hi || (a.hi == b.hi && (a.lo & m) < (b.lo & m));
}

__global__ __launch_bounds__(256) void join_ranges_kernel(const E128* __restrict__ outer, uint64_t no,
                                                          const E128* __restrict__ inner, uint64_t ni, uint64_t m,
                                                          int64_t* __restrict__ lower, int64_t* __restrict__ count) {
  for (uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; i < no; i += (uint64_t)gridDim.x * blockDim.x) {
    const E128 k = outer[i];
    uint64_t lo = 0, hi = ni;
    while (lo < hi) {   // lower bound
      const uint64_t mid = (lo + hi) >> 1;
      if (key_less(inner[mid], k, m)) lo = mid + 1; else hi = mid;
    }
    uint64_t lb = lo;
    hi = ni;
    while (lo < hi) {   // upper bound
      const uint64_t mid = (lo + hi) >> 1;
      if (!key_less(k, inner[mid], m)) lo = mid + 1; else hi = mid;
    }
    lower[i] = (int64_t)lb;
    count[i] = (int64_t)(lo - lb);
  }
}

__global__ __launch_bounds__(256) void join_emit_kernel(const E128* __restrict__ outer, const E128* __restrict__ inner,
                                                        uint64_t no, const int64_t* __restrict__ lower,
                                                        const int64_t* __restrict__ count,
                                                        const int64_t* __restrict__ offs,
                                                        int64_t* __restrict__ out_outer, int64_t* __restrict__ out_inner) {
  for (uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; i < no; i += (uint64_t)gridDim.x * blockDim.x) {
    const int64_t c = count[i], lb = lower[i], o = offs[i];
    const int64_t orow = (int64_t)(uint32_t)outer[i].lo;
    for (int64_t j = 0; j < c; ++j) {
      out_outer[o + j] = orow;
      out_inner[o + j] = (int64_t)(uint32_t)inner[lb + j].lo;
    }
  }
}

// ----- int64 exclusive scan ------------------------------------------------------------------
constexpr int kChunk = 4096;   // 256 threads x 16

__global__ __launch_bounds__(256) void scan_reduce_i64(const int64_t* __restrict__ a, uint64_t n,
                                                       int64_t* __restrict__ part) {
  __shared__ uint64_t sc[4];
  const uint64_t base = (uint64_t)blockIdx.x * kChunk + threadIdx.x * 16;
  int64_t s = 0;
#pragma unroll
  for (int k = 0; k < 16; ++k) s += (base + k < n) ? a[base + k] : 0;
  uint64_t w = wave_sum64((uint64_t)s);
  if (lane_id() == 0) sc[wave_id()] = w;
  __syncthreads();
  if (threadIdx.x == 0) part[blockIdx.x] = (int64_t)(sc[0] + sc[1] + sc[2] + sc[3]);
}

__global__ __launch_bounds__(256) void scan_down_i64(const int64_t* __restrict__ a, int64_t* __restrict__ out,
                                                     uint64_t n, const int64_t* __restrict__ part_ex) {
  __shared__ uint64_t sc[4];
  const uint64_t base = (uint64_t)blockIdx.x * kChunk + threadIdx.x * 16;
  int64_t v[16];
  int64_t s = 0;
#pragma unroll
  for (int k = 0; k < 16; ++k) {
    v[k] = (base + k < n) ? a[base + k] : 0;
    s += v[k];
  }
  const uint64_t inc = wave_inclusive_scan64((uint64_t)s);
  if (lane_id() == 63) sc[wave_id()] = inc;
  __syncthreads();
  const int w = wave_id();
  uint64_t pre = 0;
  for (int k = 0; k < w; ++k) pre += sc[k];
  int64_t run = (int64_t)(pre + inc) - s + part_ex[blockIdx.x];
#pragma unroll
  for (int k = 0; k < 16; ++k) {
    if (base + k < n) out[base + k] = run;
    run += v[k];
  }
}

}  // namespace

// ---------------------------------------------------------------------------------------------
// Returns the number of key bits (<= 96) or a negative hipError.
DR_API int dr_build_keys(const void* const* cols, const int* types, const int* desc, int ncols, uint64_t n,
                         uint32_t idx_base, E128* out, int* begin_bit, hipStream_t s) {
  if (ncols < 1 || ncols > 4) return (int)hipErrorInvalidValue;
  KeyCols kc{};
  int bits = 0;
  for (int c = 0; c < ncols; ++c) {
    kc.col[c] = cols[c];
    kc.type[c] = types[c];
    kc.desc[c] = desc ? desc[c] : 0;
    const int t = types[c];
    bits += (t <= K_BOOL) ? 8 : (t <= K_U16) ? 16 : (t <= K_U32 || t == K_F32) ? 32 : 64;
  }
  kc.ncols = ncols;
  if (bits > 96) return (int)hipErrorInvalidValue;
  *begin_bit = (128 - bits) & ~7;
  if (n == 0) return 0;
  build_keys_kernel<<<grid_for(n, 256, 16384), 256, 0, s>>>(kc, n, idx_base, bits, out);
  DR_LAUNCH_CHECK();
  return 0;
}

namespace {
// E64 entries of a narrow integer key: ((norm(key) - bias) << 32) | (idx_base + i); the caller
// guarantees norm(key) - bias < 2^32 for every row (bias = norm(min key)).
__global__ __launch_bounds__(256) void build_keys64_kernel(const void* __restrict__ col, int type, uint64_t n,
                                                           uint64_t bias, uint32_t idx_base, uint64_t* __restrict__ out) {
  for (uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (uint64_t)gridDim.x * blockDim.x)
    out[i] = ((norm_key(col, i, type) - bias) << 32) | (uint32_t)(idx_base + (uint32_t)i);
}
}  // namespace

DR_API int dr_build_keys64(const void* col, int type, uint64_t n, uint64_t bias, uint32_t idx_base, uint64_t* out,
                           hipStream_t s) {
  if (type < K_U8 || type > K_U64) return (int)hipErrorInvalidValue;   // integer keys only
  if (n == 0) return 0;
  if (n + idx_base > (1ull << 32)) return (int)hipErrorInvalidValue;
  build_keys64_kernel<<<grid_for(n, 256, 16384), 256, 0, s>>>(col, type, n, bias, idx_base, out);
  DR_LAUNCH_CHECK();
  return 0;
}

DR_API int dr_hash_dest(E128* e, uint64_t n, uint64_t lo_mask, uint32_t nparts, hipStream_t s) {
  if (nparts == 0 || nparts > 256) return (int)hipErrorInvalidValue;
  if (n == 0) return 0;
  hash_dest_kernel<<<grid_for(n, 256, 16384), 256, 0, s>>>(e, n, lo_mask, nparts);
  DR_LAUNCH_CHECK();
  return 0;
}

DR_API int dr_segment_flags(const E128* e, uint64_t n, uint64_t lo_mask, int64_t* flags, hipStream_t s) {
  if (n == 0) return 0;
  segment_flags_kernel<<<grid_for(n, 256, 16384), 256, 0, s>>>(e, n, lo_mask, flags);
  DR_LAUNCH_CHECK();
  return 0;
}

// op: 0 sum, 1 min, 2 max, 3 count; dtype: 0 int64, 1 float64.  `out` must be pre-initialised
// with the identity; `ent` (optional) maps sorted position -> row of `vals`.
DR_API int dr_seg_reduce(const void* vals, const E128* ent, const int64_t* seg, uint64_t n, void* out, int op,
                         int dtype, hipStream_t s) {
  if (n == 0) return 0;
  const unsigned g = grid_for(n, 256, 8192);
  if (dtype == 0) {
    const int64_t ident = op == 1 ? INT64_MAX : op == 2 ? INT64_MIN : 0;
    seg_reduce_kernel<int64_t><<<g, 256, 0, s>>>((const int64_t*)vals, ent, seg, n, (int64_t*)out, op, ident);
  } else {
    const double ident = op == 1 ? __builtin_inf() : op == 2 ? -__builtin_inf() : 0.0;
    seg_reduce_kernel<double><<<g, 256, 0, s>>>((const double*)vals, ent, seg, n, (double*)out, op, ident);
  }
  DR_LAUNCH_CHECK();
  return 0;
}

// Fused multi-aggregate segmented reduce (seg_reduce_multi_serial: one thread walks each chunk of rows).  ops/vals/outs: host
// arrays of nagg (<= 8) entries; outputs must be pre-filled with each op's identity.
// strides: host array of nagg element strides (nullptr = all 1); with ent == nullptr the values
// are already in sorted order (row = position).
DR_API int dr_seg_reduce_multi(const E128* ent, const int64_t* seg, uint64_t n, int nagg, const int* ops,
                               const void* const* vals, void* const* outs, const uint32_t* strides, hipStream_t s) {
  if (nagg < 1 || nagg > kMaxAggs) return (int)hipErrorInvalidValue;
  if (n == 0) return 0;
  AggSpecs sp;
  for (int a = 0; a < nagg; ++a) {
    sp.op[a] = ops[a];
    sp.vals[a] = reinterpret_cast<const uint64_t*>(vals[a]);
    sp.out[a] = reinterpret_cast<uint64_t*>(outs[a]);
    sp.stride[a] = strides ? strides[a] : 1u;
    // a missing output, or a value column missing for a value-reading op, would fault the device
    if (sp.out[a] == nullptr || (sp.op[a] != M_COUNT && sp.vals[a] == nullptr)) return (int)hipErrorInvalidValue;
  }
  // packed-row mode: every value aggregate reads a word of the same 16-byte-aligned 4-word rows
  sp.rows = nullptr;
  {
    uintptr_t base = UINTPTR_MAX;
    bool packed = ent != nullptr;
    int nval = 0;
    for (int a = 0; a < nagg; ++a) {
      if (sp.op[a] == M_COUNT) continue;
      ++nval;
      packed = packed && sp.stride[a] == 4;
      base = reinterpret_cast<uintptr_t>(sp.vals[a]) < base ? reinterpret_cast<uintptr_t>(sp.vals[a]) : base;
    }
    packed = packed && nval > 0 && (base & 15) == 0;
    for (int a = 0; a < nagg && packed; ++a) {
      sp.word[a] = 0;
      if (sp.op[a] == M_COUNT) continue;
      const uintptr_t d = reinterpret_cast<uintptr_t>(sp.vals[a]) - base;
      if (d % 8 != 0 || d / 8 > 3) packed = false;
      else sp.word[a] = (uint32_t)(d / 8);
    }
    if (packed) sp.rows = reinterpret_cast<const uint64_t*>(base);
  }
  {
    const unsigned g = grid_for(n, 256 * 8, 8192);
#define DR_SEGRED_CASE(N)                                                             \
      case N:                                                                          \
        if (sp.rows) seg_reduce_multi_serial<8, N, true><<<g, 256, 0, s>>>(ent, seg, n, sp);  \
        else seg_reduce_multi_serial<8, N, false><<<g, 256, 0, s>>>(ent, seg, n, sp);       \
        break;
    switch (nagg) {
      DR_SEGRED_CASE(1) DR_SEGRED_CASE(2) DR_SEGRED_CASE(3) DR_SEGRED_CASE(4)
      DR_SEGRED_CASE(5) DR_SEGRED_CASE(6) DR_SEGRED_CASE(7)
      default: DR_SEGRED_CASE(8)
    }
#undef DR_SEGRED_CASE
  }
  DR_LAUNCH_CHECK();
  return 0;
}

namespace {
// group starts per 512-entry wave chunk of sorted E128 entries keyed by hi alone (lo_mask 0)
__global__ __launch_bounds__(256) void group_chunk_starts_kernel(const E128* __restrict__ e, uint64_t n,
                                                                 int64_t* __restrict__ cnt) {
  constexpr int PER = 8;
  constexpr uint64_t kChunkElems = 64 * PER;
  const int lane = lane_id();
  const uint64_t waves = ((uint64_t)gridDim.x * blockDim.x) >> 6;
  const uint64_t w0 = (((uint64_t)blockIdx.x * blockDim.x) + threadIdx.x) >> 6;
  // lane-adjacent loads (element cbase + 64 k + lane): each load instruction covers 1 KB of
  // consecutive entries instead of one 16-byte word in each of 64 lines; the chunk (and so the
  // count) is the same 512 consecutive entries either way
  for (uint64_t cbase = w0 * kChunkElems; cbase < n; cbase += waves * kChunkElems) {
    uint64_t kh[PER];
#pragma unroll
    for (int k = 0; k < PER; ++k) {
      const uint64_t i = cbase + (uint64_t)(64 * k + lane);
      kh[k] = i < n ? e[i].hi : 0;
    }
    const uint64_t before = (lane == 0 && cbase > 0) ? e[cbase - 1].hi : 0;
    uint64_t c = 0;
#pragma unroll
    for (int k = 0; k < PER; ++k) {
      const uint64_t i = cbase + (uint64_t)(64 * k + lane);
      uint64_t prev = __shfl_up(kh[k], 1, 64);
      if (k > 0) {
        const uint64_t wrap = __shfl(kh[k > 0 ? k - 1 : 0], 63, 64);   // lane 63 of step k-1
        if (lane == 0) prev = wrap;
      } else if (lane == 0) {
        prev = before;
      }
      c += (i < n && (i == 0 || kh[k] != prev)) ? 1 : 0;
    }
    c = wave_sum64(c);
    if (lane == 0) cnt[cbase / kChunkElems] = (int64_t)c;
  }
}
}  // namespace

// Group starts per 512-entry chunk (cnt: ceil(n / 512) int64) of sorted {row, key} entries.
DR_API uint32_t dr_group_chunk_elems() { return 512; }

DR_API int dr_group_chunk_starts(const E128* e, uint64_t n, int64_t* cnt, hipStream_t s) {
  if (n == 0) return 0;
  group_chunk_starts_kernel<<<grid_for(n, 256 * 8, 8192), 256, 0, s>>>(e, n, cnt);
  DR_LAUNCH_CHECK();
  return 0;
}

// dr_seg_reduce_multi with fused segment ids (see seg_reduce_multi_serial KEYS): chunk_base =
// exclusive scan of dr_group_chunk_starts, keys_out[g] = hi ^ key_xor of group g.
DR_API int dr_seg_reduce_multi_keys(const E128* ent, uint64_t n, const int64_t* chunk_base, uint64_t key_xor,
                                    uint64_t* keys_out, int nagg, const int* ops, const void* const* vals,
                                    void* const* outs, const uint32_t* strides, hipStream_t s) {
  if (nagg < 1 || nagg > kMaxAggs || ent == nullptr || chunk_base == nullptr || keys_out == nullptr)
    return (int)hipErrorInvalidValue;
  if (n == 0) return 0;
  AggSpecs sp;
  for (int a = 0; a < nagg; ++a) {
    sp.op[a] = ops[a];
    sp.vals[a] = reinterpret_cast<const uint64_t*>(vals[a]);
    sp.out[a] = reinterpret_cast<uint64_t*>(outs[a]);
    sp.stride[a] = strides ? strides[a] : 1u;
    if (sp.out[a] == nullptr || (sp.op[a] != M_COUNT && sp.vals[a] == nullptr)) return (int)hipErrorInvalidValue;
  }
  sp.rows = nullptr;
  {
    uintptr_t base = UINTPTR_MAX;
    bool packed = true;
    int nval = 0;
    for (int a = 0; a < nagg; ++a) {
      if (sp.op[a] == M_COUNT) continue;
      ++nval;
      packed = packed && sp.stride[a] == 4;
      base = reinterpret_cast<uintptr_t>(sp.vals[a]) < base ? reinterpret_cast<uintptr_t>(sp.vals[a]) : base;
    }
    packed = packed && nval > 0 && (base & 15) == 0;
    for (int a = 0; a < nagg && packed; ++a) {
      sp.word[a] = 0;
      if (sp.op[a] == M_COUNT) continue;
      const uintptr_t d = reinterpret_cast<uintptr_t>(sp.vals[a]) - base;
      if (d % 8 != 0 || d / 8 > 3) packed = false;
      else sp.word[a] = (uint32_t)(d / 8);
    }
    if (packed) sp.rows = reinterpret_cast<const uint64_t*>(base);
  }
  const unsigned g = grid_for(n, 256 * 8, 8192);
#define DR_SEGRED_KCASE(N)                                                                                    \
  case N:                                                                                                     \
    if (sp.rows) seg_reduce_multi_serial<8, N, true, true><<<g, 256, 0, s>>>(ent, nullptr, n, sp, chunk_base, \
                                                                             key_xor, keys_out);             \
    else seg_reduce_multi_serial<8, N, false, true><<<g, 256, 0, s>>>(ent, nullptr, n, sp, chunk_base,        \
                                                                      key_xor, keys_out);                    \
    break;
  switch (nagg) {
    DR_SEGRED_KCASE(1) DR_SEGRED_KCASE(2) DR_SEGRED_KCASE(3) DR_SEGRED_KCASE(4)
    DR_SEGRED_KCASE(5) DR_SEGRED_KCASE(6) DR_SEGRED_KCASE(7)
    default: DR_SEGRED_KCASE(8)
  }
#undef DR_SEGRED_KCASE
  DR_LAUNCH_CHECK();
  return 0;
}

DR_API int dr_join_ranges(const E128* outer, uint64_t no, const E128* inner, uint64_t ni, uint64_t lo_mask,
                          int64_t* lower, int64_t* count, hipStream_t s) {
  if (no == 0) return 0;
  join_ranges_kernel<<<grid_for(no, 256, 16384), 256, 0, s>>>(outer, no, inner, ni, lo_mask, lower, count);
  DR_LAUNCH_CHECK();
  return 0;
}

DR_API int dr_join_emit(const E128* outer, const E128* inner, uint64_t no, const int64_t* lower, const int64_t* count,
                        const int64_t* offs, int64_t* out_outer, int64_t* out_inner, hipStream_t s) {
  if (no == 0) return 0;
  join_emit_kernel<<<grid_for(no, 256, 16384), 256, 0, s>>>(outer, inner, no, lower, count, offs, out_outer, out_inner);
  DR_LAUNCH_CHECK();
  return 0;
}

DR_API uint64_t dr_scan_i64_workspace(uint64_t n) {
  uint64_t total = 0;
  uint64_t m = n;
  while (m > 1) {
    m = (m + kChunk - 1) / kChunk;
    total += m;
  }
  return (total + 8) * sizeof(int64_t);
}

// out[i] = sum_{j<i} a[i]  (may alias a).  Recursive reduce-then-scan.
DR_API int dr_scan_i64(const int64_t* a, int64_t* out, uint64_t n, void* ws, hipStream_t s) {
  if (n == 0) return 0;
  int64_t* part = reinterpret_cast<int64_t*>(ws);
  const uint64_t nb = (n + kChunk - 1) / kChunk;
  if (nb == 1) {
    hipMemsetAsync(part, 0, sizeof(int64_t), s);
    scan_down_i64<<<1, 256, 0, s>>>(a, out, n, part);
    DR_LAUNCH_CHECK();
    return 0;
  }
  scan_reduce_i64<<<(unsigned)nb, 256, 0, s>>>(a, n, part);
  int rc = dr_scan_i64(part, part, nb, part + nb, s);
  if (rc) return rc;
  scan_down_i64<<<(unsigned)nb, 256, 0, s>>>(a, out, n, part);
  DR_LAUNCH_CHECK();
  return 0;
}

namespace {

// ----- fused segment ids -----------------------------------------------------------------------
// flag(i) = 1 where sorted entry i starts a new key (hi or masked lo differs from entry i - 1)
__device__ __forceinline__ int64_t seg_flag(const E128* __restrict__ e, uint64_t i, uint64_t lo_mask) {
  if (i == 0) return 1;
  const E128 a = e[i - 1], b = e[i];
  return (a.hi != b.hi || ((a.lo ^ b.lo) & lo_mask) != 0) ? 1 : 0;
}

__global__ __launch_bounds__(256) void seg_count_kernel(const E128* __restrict__ e, uint64_t n, uint64_t lo_mask,
                                                        int64_t* __restrict__ part) {
  __shared__ uint64_t sc[4];
  const uint64_t base = (uint64_t)blockIdx.x * kChunk + threadIdx.x * 16;
  int64_t s = 0;
#pragma unroll
  for (int k = 0; k < 16; ++k) s += (base + k < n) ? seg_flag(e, base + k, lo_mask) : 0;
  uint64_t w = wave_sum64((uint64_t)s);
  if (lane_id() == 0) sc[wave_id()] = w;
  __syncthreads();
  if (threadIdx.x == 0) part[blockIdx.x] = (int64_t)(sc[0] + sc[1] + sc[2] + sc[3]);
}

// ids[i] = (number of segment starts at or before i) - 1; starts[id] = i at every start
__global__ __launch_bounds__(256) void seg_ids_kernel(const E128* __restrict__ e, uint64_t n, uint64_t lo_mask,
                                                      const int64_t* __restrict__ part_ex, int64_t* __restrict__ ids,
                                                      int64_t* __restrict__ starts) {
  __shared__ uint64_t sc[4];
  const uint64_t base = (uint64_t)blockIdx.x * kChunk + threadIdx.x * 16;
  int64_t v[16];
  int64_t s = 0;
#pragma unroll
  for (int k = 0; k < 16; ++k) {
    v[k] = (base + k < n) ? seg_flag(e, base + k, lo_mask) : 0;
    s += v[k];
  }
  const uint64_t inc = wave_inclusive_scan64((uint64_t)s);
  if (lane_id() == 63) sc[wave_id()] = inc;
  __syncthreads();
  const int w = wave_id();
  uint64_t pre = 0;
  for (int k = 0; k < w; ++k) pre += sc[k];
  int64_t run = (int64_t)(pre + inc) - s + part_ex[blockIdx.x];
#pragma unroll
  for (int k = 0; k < 16; ++k) {
    run += v[k];
    if (base + k < n) {
      ids[base + k] = run - 1;
      if (v[k]) starts[run - 1] = (int64_t)(base + k);
    }
  }
}

}  // namespace

// Segment ids of sorted entries in two passes over the entries (no flag array): ids[i] = segment
// of entry i, starts[g] = first position of segment g (starts needs room for n values); the
// segment count is ids[n - 1] + 1.  ws: dr_scan_i64_workspace(n) bytes.
DR_API int dr_segment_ids(const E128* e, uint64_t n, uint64_t lo_mask, int64_t* ids, int64_t* starts, void* ws,
                          hipStream_t s) {
  if (n == 0) return 0;
  int64_t* part = reinterpret_cast<int64_t*>(ws);
  const uint64_t nb = (n + kChunk - 1) / kChunk;
  seg_count_kernel<<<(unsigned)nb, 256, 0, s>>>(e, n, lo_mask, part);
  int rc = dr_scan_i64(part, part, nb, part + nb, s);
  if (rc) return rc;
  seg_ids_kernel<<<(unsigned)nb, 256, 0, s>>>(e, n, lo_mask, part, ids, starts);
  DR_LAUNCH_CHECK();
  return 0;
}

