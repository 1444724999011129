// Record-boundary discovery for parts of variable-length DryadLinqBinary records (strings are a
// compact UTF-16 unit count, a compact byte count and the UTF-8 bytes; reference
// DryadLinqBinaryReader.cs:341-366 ReadCompactInt32, :628-632 ReadString), on the device and
// without an index sidecar.  A length-prefixed stream is only parseable from a known boundary,
// so the part is cut into C-byte chunks and parsed speculatively:
//
//   1. vs_chain   one lane per chunk parses from the chunk start as if it were a boundary
//                 (restarting a byte later until kLock records in a row parse) and sets a bit
//                 for every position it visits (the chunk's speculative chain), plus the first
//                 position it reaches past the chunk (its exit).
//   2. vs_walk    lane c walks on from its exit until it lands on a position some later chain
//                 visited (the sync point).  From there on the two parses coincide (the parse
//                 is a function of the position), so if chain c is right at its exit, the walk
//                 and then the later chain from the sync point are right too.  Chain 0 starts at
//                 offset 0, a true boundary, so the true boundaries are: chain 0, walk 0, the
//                 synced chain from its sync point, its walk, ... (a host pointer chase only when
//                 some walk does not sync in the very next chunk).
//   3. vs_fix     clears every chain bit before the chunk's true entry (all of them in a chunk no
//                 chain enters) and counts the rest; vs_walk_bits adds the walk positions.
//   4. vs_select  after an exclusive scan of the per-chunk counts, writes the byte offset of
//                 every B-th record: the block index codec_var_decode takes.
//
// Plausibility checks that every writer of the format satisfies (units <= bytes <= 3 units, the
// byte count's width fixed by the unit count, as DryadLinqBinaryWriter.cs:523-546 writes it) make
// wrong chains fail or re-synchronise quickly.  Anything irregular (a walk that never syncs, a
// chain that fails after its entry) is reported and the caller scans the part on the host.
#include "common.h"

namespace {
constexpr int kMaxF = 32;
constexpr uint64_t kBad = ~0ull;
constexpr uint64_t kGiveUp = ~0ull - 1;

struct VSchema {
  int nf;
  uint32_t size[kMaxF];   // bytes of a fixed field, 0 = string
};

__device__ __forceinline__ uint64_t vs_step(const uint8_t* __restrict__ b, uint64_t p, uint64_t n, const VSchema& s) {
  for (int f = 0; f < s.nf; ++f) {
    const uint32_t sz = s.size[f];
    if (sz) {
      p += sz;
      continue;
    }
    if (p >= n) return kBad;
    uint32_t u = b[p];
    if (u < 0x80) {
      p += 1;
    } else {
      if (p + 4 > n) return kBad;
      u = ((u & 0x7Fu) << 24) | ((uint32_t)b[p + 1] << 16) | ((uint32_t)b[p + 2] << 8) | b[p + 3];
      if (u < 0x80) return kBad;                     // never written in the wide form
      p += 4;
    }
    if (p >= n) return kBad;
    uint32_t nb = b[p];
    const bool wide = ((uint64_t)u + 1) * 3 >= 0x80;
    if (nb < 0x80) {
      if (wide) return kBad;
      p += 1;
    } else {
      if (!wide || p + 4 > n) return kBad;
      nb = ((nb & 0x7Fu) << 24) | ((uint32_t)b[p + 1] << 16) | ((uint32_t)b[p + 2] << 8) | b[p + 3];
      p += 4;
    }
    if (nb < u || (uint64_t)nb > 3ull * u) return kBad;
    p += nb;
  }
  return p <= n ? p : kBad;
}

__device__ __forceinline__ bool vs_bit(const uint32_t* __restrict__ bits, uint64_t p) {
  return (bits[p >> 5] >> (p & 31)) & 1u;
}

// A chain locks onto the stream once kLock records in a row parse, each shorter than the chunk;
// until then a failed (or implausibly long) parse restarts it one byte after the previous start
// (and forgets the positions of that attempt), so a chunk whose start is not a boundary still
// finds one and follows the stream from there (the exit walks of the previous chunk then meet it
// within the chunk).  The length bound matters in large parts: a misaligned 4-byte length there
// can land gigabytes ahead and still inside the part.  A locked chain that fails stops: it was
// not on the stream.  (A false lock only costs speed: the walks step over it.)
constexpr int kLock = 6;

__global__ __launch_bounds__(256) void vs_chain(const uint8_t* __restrict__ b, uint64_t n, uint32_t C, uint64_t nch,
                                                VSchema s, uint32_t* __restrict__ bits, int64_t* __restrict__ exitp) {
  for (uint64_t c = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; c < nch; c += (uint64_t)gridDim.x * blockDim.x) {
    const uint64_t s0 = c * C, s1 = s0 + C < n ? s0 + C : n;
    const uint64_t wend = (s1 + 31) >> 5;
    uint64_t cw = s0 >> 5, p = s0, start = s0;
    uint32_t acc = 0;
    uint64_t tent[kLock];
    int run = 0;
    bool locked = c == 0;                             // offset 0 is a boundary: chain 0 never restarts
    auto mark = [&](uint64_t q) {                     // positions arrive in increasing order
      const uint64_t w = q >> 5;
      while (cw < w) {
        bits[cw++] = acc;
        acc = 0;
      }
      acc |= 1u << (q & 31);
    };
    while (p < s1) {
      const uint64_t q = vs_step(b, p, n, s);
      if (q == kBad || (!locked && q - p > C)) {
        if (locked) break;
        run = 0;                                      // not a boundary after all: next start
        p = ++start;
        continue;
      }
      if (locked) {
        mark(p);
      } else {
        tent[run++] = p;
        if (run == kLock) {
          locked = true;
          for (int k = 0; k < kLock; ++k) mark(tent[k]);
        }
      }
      p = q;
    }
    if (!locked && run > 0 && p >= s1) {               // a short run that reached the chunk end
      for (int k = 0; k < run; ++k) mark(tent[k]);
      locked = true;
    }
    while (cw < wend) {
      bits[cw++] = acc;
      acc = 0;
    }
    exitp[c] = locked && p >= s1 ? (int64_t)p : -1;   // -1 = no run reached the chunk end
  }
}

__global__ __launch_bounds__(256) void vs_walk(const uint8_t* __restrict__ b, uint64_t n, uint64_t nch, VSchema s,
                                               const uint32_t* __restrict__ bits, const int64_t* __restrict__ exitp,
                                               int64_t* __restrict__ sync, uint32_t max_steps) {
  for (uint64_t c = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; c < nch; c += (uint64_t)gridDim.x * blockDim.x) {
    uint64_t p = (uint64_t)exitp[c];
    uint64_t y = kBad;
    for (uint32_t k = 0; p != kBad; ++k) {
      if (p >= n) {
        y = p == n ? n : kBad;                        // the stream ends exactly here
        break;
      }
      if (vs_bit(bits, p)) {
        y = p;
        break;
      }
      if (k >= max_steps) {
        y = kGiveUp;
        break;
      }
      p = vs_step(b, p, n, s);
    }
    sync[c] = (int64_t)y;
  }
}

// entry[j]: the first true boundary of chunk j (its start for chunk 0, a walk's sync point
// otherwise), -1 when no chain is entered in chunk j (its records, if any, come from a walk).
__global__ __launch_bounds__(256) void vs_fix(uint64_t n, uint32_t C, uint64_t nch, const int64_t* __restrict__ entry,
                                              uint32_t* __restrict__ bits, uint64_t* __restrict__ cnt) {
  for (uint64_t j = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; j < nch; j += (uint64_t)gridDim.x * blockDim.x) {
    const uint64_t s0 = j * C, s1 = s0 + C < n ? s0 + C : n;
    const int64_t e = entry[j];
    const uint64_t from = e < 0 ? s1 : (uint64_t)e;
    uint64_t k = 0;
    for (uint64_t w = s0 >> 5; w < (s1 + 31) >> 5; ++w) {
      const uint64_t wb = w << 5;
      uint32_t x = bits[w];
      if (wb + 32 <= from) {
        x = 0;
      } else if (wb < from) {
        x &= ~0u << (from - wb);
      }
      bits[w] = x;
      k += __popc(x);
    }
    cnt[j] = k;
  }
}

// The walks of the chunks on the true path (entry of the next entered chunk = their sync point):
// their positions are true boundaries (the chains there were cleared by vs_fix).
__global__ __launch_bounds__(256) void vs_walk_bits(const uint8_t* __restrict__ b, uint64_t n, uint32_t C,
                                                    uint64_t nch, VSchema s, const uint8_t* __restrict__ on_path,
                                                    const int64_t* __restrict__ exitp, const int64_t* __restrict__ sync,
                                                    uint32_t* __restrict__ bits, unsigned long long* __restrict__ cnt) {
  for (uint64_t c = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; c < nch; c += (uint64_t)gridDim.x * blockDim.x) {
    if (!on_path[c]) continue;
    uint64_t p = (uint64_t)exitp[c];
    const uint64_t y = (uint64_t)sync[c];
    uint64_t cur = kBad, k = 0;
    while (p < y) {
      const uint64_t j = p / C;
      if (j != cur) {
        if (k) atomicAdd(cnt + cur, (unsigned long long)k);
        cur = j;
        k = 0;
      }
      atomicOr(bits + (p >> 5), 1u << (p & 31));
      ++k;
      p = vs_step(b, p, n, s);
    }
    if (k) atomicAdd(cnt + cur, (unsigned long long)k);
  }
}

__global__ __launch_bounds__(256) void vs_select(uint64_t n, uint32_t C, uint64_t nch, const uint32_t* __restrict__ bits,
                                                 const int64_t* __restrict__ base, uint32_t B,
                                                 int64_t* __restrict__ block_off) {
  for (uint64_t j = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; j < nch; j += (uint64_t)gridDim.x * blockDim.x) {
    const uint64_t s0 = j * C, s1 = s0 + C < n ? s0 + C : n;
    uint64_t idx = (uint64_t)base[j];
    uint64_t next = (idx + B - 1) / B * B;            // the next record index that starts a block
    for (uint64_t w = s0 >> 5; w < (s1 + 31) >> 5; ++w) {
      uint32_t x = bits[w];
      const uint32_t pc = __popc(x);
      while (x && next < idx + pc) {
        // the (next - idx)-th set bit of x
        uint32_t y = x;
        for (uint64_t r = next - idx; r; --r) y &= y - 1;
        const uint32_t bit = __ffs(y) - 1;
        block_off[next / B] = (int64_t)((w << 5) + bit);
        next += B;
      }
      idx += pc;
    }
  }
}

int fill_schema(VSchema* s, int nf, const uint32_t* sizes) {
  if (nf < 1 || nf > kMaxF) return 1;
  s->nf = nf;
  for (int f = 0; f < nf; ++f) s->size[f] = sizes[f];
  return 0;
}
}  // namespace

// Pass 1+2: bits (u32 [ceil(n/32)]), exitp / sync (int64 [nch]); C a multiple of 32.
DR_API int dr_varscan_chains(const uint8_t* buf, uint64_t n, uint32_t C, int nf, const uint32_t* sizes,
                             uint32_t* bits, int64_t* exitp, int64_t* sync, uint32_t max_steps, hipStream_t st) {
  VSchema s;
  if (C == 0 || (C & 31) || fill_schema(&s, nf, sizes)) return (int)hipErrorInvalidValue;
  const uint64_t nch = (n + C - 1) / C;
  if (nch == 0) return 0;
  vs_chain<<<grid_for(nch, 256, 1u << 16), 256, 0, st>>>(buf, n, C, nch, s, bits, exitp);
  DR_LAUNCH_CHECK();
  vs_walk<<<grid_for(nch, 256, 1u << 16), 256, 0, st>>>(buf, n, nch, s, bits, exitp, sync, max_steps);
  DR_LAUNCH_CHECK();
  return 0;
}

// Pass 3: entry (int64 [nch], -1 = not entered), on_path (u8 [nch]): cnt (u64 [nch]) = the true
// boundaries per chunk, bits = exactly the true boundaries.
DR_API int dr_varscan_fix(const uint8_t* buf, uint64_t n, uint32_t C, int nf, const uint32_t* sizes,
                          const int64_t* entry, const uint8_t* on_path, const int64_t* exitp, const int64_t* sync,
                          uint32_t* bits, uint64_t* cnt, hipStream_t st) {
  VSchema s;
  if (C == 0 || (C & 31) || fill_schema(&s, nf, sizes)) return (int)hipErrorInvalidValue;
  const uint64_t nch = (n + C - 1) / C;
  if (nch == 0) return 0;
  vs_fix<<<grid_for(nch, 256, 1u << 16), 256, 0, st>>>(n, C, nch, entry, bits, cnt);
  DR_LAUNCH_CHECK();
  vs_walk_bits<<<grid_for(nch, 256, 1u << 16), 256, 0, st>>>(buf, n, C, nch, s, on_path, exitp, sync, bits,
                                                             reinterpret_cast<unsigned long long*>(cnt));
  DR_LAUNCH_CHECK();
  return 0;
}

// Pass 4: base (int64 [nch]) = exclusive scan of cnt; block_off (int64 [ceil(records / B)]).
DR_API int dr_varscan_select(uint64_t n, uint32_t C, const uint32_t* bits, const int64_t* base, uint32_t B,
                             int64_t* block_off, hipStream_t st) {
  if (C == 0 || (C & 31) || B == 0) return (int)hipErrorInvalidValue;
  const uint64_t nch = (n + C - 1) / C;
  if (nch == 0) return 0;
  vs_select<<<grid_for(nch, 256, 1u << 16), 256, 0, st>>>(n, C, nch, bits, base, B, block_off);
  DR_LAUNCH_CHECK();
  return 0;
}
