// bic_device.h -- device-side helpers shared by the HIP kernels (wave64 primitives, the
// Golomb k rule, the med residual word, chunk/row bookkeeping). Included by .hip files only.
#pragma once
#include "bic_internal.h"

#include <climits>

namespace bic {

#define BIC_MSB 0x8000000000000000ull
constexpr int kBlock = 256;   // 4 waves
constexpr int kWaves = kBlock / 64;
constexpr int kLdsWords = 1024;  // u32 staging words per wave in the emitter (32768 bits)

// ------------------------------------------------------------------------------------
// wave / block primitives (wave64)
// ------------------------------------------------------------------------------------
__device__ __forceinline__ int lane_id() { return threadIdx.x & 63; }
// wave-uniform copies (SGPRs): the compiler cannot always prove a value uniform (e.g. the result of
// a branchy index remap), and a uniform loop counter in VGPRs turns the loop into an exec-masked one
__device__ __forceinline__ uint32_t uni_u32(uint32_t v) { return (uint32_t)__builtin_amdgcn_readfirstlane((int)v); }
__device__ __forceinline__ uint64_t uni_u64(uint64_t v) {
  return ((uint64_t)uni_u32((uint32_t)(v >> 32)) << 32) | uni_u32((uint32_t)v);
}
// the wave's index in its workgroup as a wave-uniform value: the compiler takes threadIdx.x >> 6 for
// divergent, and every row / plane / offset derived from it (and every branch on those) would then be
// vector work under exec masks (C3 count pass: 2,530 -> 2,323 VALU instructions, 56 -> 50 VGPRs)
__device__ __forceinline__ uint32_t wave_id() { return uni_u32(threadIdx.x >> 6); }

__device__ __forceinline__ uint64_t shfl_u64(uint64_t v, int src) {
  const uint32_t lo = __shfl((unsigned)(v & 0xffffffffu), src);
  const uint32_t hi = __shfl((unsigned)(v >> 32), src);
  return ((uint64_t)hi << 32) | lo;
}

// ---- DPP primitives (every lane of the wave active) --------------------------------------
// Cross-lane steps through DPP (a few cycles each) instead of ds_bpermute (an LDS round trip,
// ~50+ cycles): the scans and reductions below are dependent chains, so their latency is what
// a row's wave waits for. CTRL: 0x111.. row_shr:n, 0x138 wave_shr:1, 0x140 row_mirror,
// 0x141 row_half_mirror, 0x142 row_bcast:15, 0x143 row_bcast:31, 0xB1 / 0x4E quad swaps.
template <int CTRL, int RM = 0xf>
__device__ __forceinline__ uint32_t dpp0(uint32_t v) {  // invalid source lanes / masked rows read 0
  return (uint32_t)__builtin_amdgcn_update_dpp(0, (int)v, CTRL, RM, 0xf, true);
}
template <int CTRL, int RM = 0xf>
__device__ __forceinline__ int dpp_or(int old, int v) {  // invalid source lanes / masked rows read old
  return __builtin_amdgcn_update_dpp(old, v, CTRL, RM, 0xf, false);
}
__device__ __forceinline__ uint32_t lane63_u32(uint32_t v) { return (uint32_t)__builtin_amdgcn_readlane((int)v, 63); }
__device__ __forceinline__ uint64_t lane63_u64(uint64_t v) {
  return ((uint64_t)lane63_u32((uint32_t)(v >> 32)) << 32) | lane63_u32((uint32_t)v);
}
// lane i gets lane i-d's value, lanes < d their own (__shfl_up semantics); d = 1 through DPP
__device__ __forceinline__ uint64_t shfl_up_u64(uint64_t v, int d) {
  if (d == 1) {
    const uint32_t lo = (uint32_t)dpp_or<0x138>((int)(uint32_t)v, (int)(uint32_t)v);
    const uint32_t hi = (uint32_t)dpp_or<0x138>((int)(uint32_t)(v >> 32), (int)(uint32_t)(v >> 32));
    return ((uint64_t)hi << 32) | lo;
  }
  const uint32_t lo = __shfl_up((unsigned)(v & 0xffffffffu), d);
  const uint32_t hi = __shfl_up((unsigned)(v >> 32), d);
  return ((uint64_t)hi << 32) | lo;
}

// inclusive scans: Hillis-Steele inside each 16-lane row (row_shr 1, 2, 4, 8), then the row
// totals carried into rows 1 and 3 (row_bcast:15) and into rows 2 and 3 (row_bcast:31)
__device__ __forceinline__ uint32_t wave_incl_sum_u32(uint32_t x) {
  x += dpp0<0x111>(x);
  x += dpp0<0x112>(x);
  x += dpp0<0x114>(x);
  x += dpp0<0x118>(x);
  x += dpp0<0x142, 0xA>(x);
  x += dpp0<0x143, 0xC>(x);
  return x;
}
template <int CTRL, int RM = 0xf>
__device__ __forceinline__ uint64_t dpp0_u64(uint64_t v) {
  return ((uint64_t)dpp0<CTRL, RM>((uint32_t)(v >> 32)) << 32) | dpp0<CTRL, RM>((uint32_t)v);
}
__device__ __forceinline__ uint64_t wave_incl_sum_u64(uint64_t x) {
  x += dpp0_u64<0x111>(x);
  x += dpp0_u64<0x112>(x);
  x += dpp0_u64<0x114>(x);
  x += dpp0_u64<0x118>(x);
  x += dpp0_u64<0x142, 0xA>(x);
  x += dpp0_u64<0x143, 0xC>(x);
  return x;
}
__device__ __forceinline__ int wave_incl_max(int x) {
  x = max(x, dpp_or<0x111>(INT_MIN, x));
  x = max(x, dpp_or<0x112>(INT_MIN, x));
  x = max(x, dpp_or<0x114>(INT_MIN, x));
  x = max(x, dpp_or<0x118>(INT_MIN, x));
  x = max(x, dpp_or<0x142, 0xA>(INT_MIN, x));
  x = max(x, dpp_or<0x143, 0xC>(INT_MIN, x));
  return x;
}
// (the old operand of every DPP step is the operation's identity, never x itself: with old = x the
// compiler keeps a v_mov_b32_dpp plus a copy of x per step instead of one v_max_i32_dpp)
// reductions (wave-uniform results): quad swaps and the two mirrors give every lane its row's
// total (wave_sum_u64: the four rows are combined from readlanes); the 32-bit ones carry the row
// totals into row 3 with row_bcast:15 / row_bcast:31 and read lane 63 once
__device__ __forceinline__ uint64_t wave_sum_u64(uint64_t x) {
  x += dpp0_u64<0xB1>(x);
  x += dpp0_u64<0x4E>(x);
  x += dpp0_u64<0x141>(x);
  x += dpp0_u64<0x140>(x);
  uint64_t s = 0;
#pragma unroll
  for (int r = 0; r < 64; r += 16)
    s += ((uint64_t)(uint32_t)__builtin_amdgcn_readlane((int)(uint32_t)(x >> 32), r) << 32) |
         (uint32_t)__builtin_amdgcn_readlane((int)(uint32_t)x, r);
  return s;
}
__device__ __forceinline__ uint32_t wave_sum_u32(uint32_t x) {
  x += dpp0<0xB1>(x);
  x += dpp0<0x4E>(x);
  x += dpp0<0x141>(x);
  x += dpp0<0x140>(x);
  x += dpp0<0x142, 0xA>(x);
  x += dpp0<0x143, 0xC>(x);
  return lane63_u32(x);
}
__device__ __forceinline__ int wave_max(int x) {
  x = max(x, dpp_or<0xB1>(INT_MIN, x));
  x = max(x, dpp_or<0x4E>(INT_MIN, x));
  x = max(x, dpp_or<0x141>(INT_MIN, x));
  x = max(x, dpp_or<0x140>(INT_MIN, x));
  x = max(x, dpp_or<0x142, 0xA>(INT_MIN, x));
  x = max(x, dpp_or<0x143, 0xC>(INT_MIN, x));
  return __builtin_amdgcn_readlane(x, 63);
}
__device__ __forceinline__ int wave_min(int x) {
  x = min(x, dpp_or<0xB1>(INT_MAX, x));
  x = min(x, dpp_or<0x4E>(INT_MAX, x));
  x = min(x, dpp_or<0x141>(INT_MAX, x));
  x = min(x, dpp_or<0x140>(INT_MAX, x));
  x = min(x, dpp_or<0x142, 0xA>(INT_MAX, x));
  x = min(x, dpp_or<0x143, 0xC>(INT_MAX, x));
  return __builtin_amdgcn_readlane(x, 63);
}

// DPP wave reductions: four in-row steps (quad swaps, half-row and row mirrors: a few cycles each,
// against ~50 for a ds_bpermute shuffle) leave every lane with its 16-lane row's total; the four row
// totals are combined from readlanes. The result is wave-uniform.
template <int CTRL>
__device__ __forceinline__ uint32_t dpp_u32(uint32_t v) {
  return (uint32_t)__builtin_amdgcn_update_dpp(0, (int)v, CTRL, 0xf, 0xf, false);
}
__device__ __forceinline__ uint32_t wave_total_u32(uint32_t v) {
  v += dpp_u32<0xB1>(v);   // quad_perm(1,0,3,2)
  v += dpp_u32<0x4E>(v);   // quad_perm(2,3,0,1)
  v += dpp_u32<0x141>(v);  // row_half_mirror
  v += dpp_u32<0x140>(v);  // row_mirror
  return (uint32_t)__builtin_amdgcn_readlane((int)v, 0) + (uint32_t)__builtin_amdgcn_readlane((int)v, 16) +
         (uint32_t)__builtin_amdgcn_readlane((int)v, 32) + (uint32_t)__builtin_amdgcn_readlane((int)v, 48);
}
template <int CTRL>
__device__ __forceinline__ unsigned long long dpp_min_step(unsigned long long v) {
  const uint32_t lo = dpp_u32<CTRL>((uint32_t)v), hi = dpp_u32<CTRL>((uint32_t)(v >> 32));
  const unsigned long long o = ((unsigned long long)hi << 32) | lo;
  return o < v ? o : v;
}
__device__ __forceinline__ unsigned long long wave_min_u64(unsigned long long v) {
  v = dpp_min_step<0xB1>(v);
  v = dpp_min_step<0x4E>(v);
  v = dpp_min_step<0x141>(v);
  v = dpp_min_step<0x140>(v);
  unsigned long long m = v;
#pragma unroll
  for (int r = 16; r < 64; r += 16) {
    const unsigned long long o = ((unsigned long long)(uint32_t)__builtin_amdgcn_readlane((int)(v >> 32), r) << 32) |
                                 (uint32_t)__builtin_amdgcn_readlane((int)(uint32_t)v, r);
    m = o < m ? o : m;
  }
  const unsigned long long m0 = ((unsigned long long)(uint32_t)__builtin_amdgcn_readlane((int)(v >> 32), 0) << 32) |
                                (uint32_t)__builtin_amdgcn_readlane((int)(uint32_t)v, 0);
  return m0 < m ? m0 : m;
}
// lane i receives lane i-1's value, lane 0 receives 0 (DPP wave_shr:1)
__device__ __forceinline__ uint64_t wave_shr1_u64(uint64_t v) {
  const uint32_t lo = (uint32_t)__builtin_amdgcn_update_dpp(0, (int)(uint32_t)v, 0x138, 0xf, 0xf, true);
  const uint32_t hi = (uint32_t)__builtin_amdgcn_update_dpp(0, (int)(uint32_t)(v >> 32), 0x138, 0xf, 0xf, true);
  return ((uint64_t)hi << 32) | lo;
}

// Exclusive block scan for blockDim.x <= 1024 (<= 16 waves). tmp: >= 17 entries of LDS.
template <typename T>
__device__ __forceinline__ T block_excl_scan(T x, T* tmp, T& total) {
  const int l = lane_id(), w = (int)wave_id(), nw = blockDim.x >> 6;
  T inc;
  if constexpr (sizeof(T) == 8) inc = wave_incl_sum_u64(x);
  else inc = wave_incl_sum_u32(x);
  if (l == 63) tmp[w] = inc;
  __syncthreads();
  if (w == 0) {
    const T v = l < nw ? tmp[l] : T(0);
    T vi;
    if constexpr (sizeof(T) == 8) vi = wave_incl_sum_u64(v);
    else vi = wave_incl_sum_u32(v);
    if (l < nw) tmp[l] = vi - v;
    if (l == nw - 1) tmp[16] = vi;
  }
  __syncthreads();
  const T res = tmp[w] + inc - x;
  total = tmp[16];
  __syncthreads();
  return res;
}

// ------------------------------------------------------------------------------------
// Decoupled look-back records (row encoder tiles, sample coder blocks): 8-byte {flag, value}
// granules written and polled with agent-scope relaxed atomics (cdna_hip_programming.md §6
// Guideline 16, R2). flag 0 = not yet published, kAgg = the unit's own total, kInc = inclusive
// prefix. A unit takes its index from a ticket counter, so every unit it waits on holds an earlier
// ticket and is already running or done.
// ------------------------------------------------------------------------------------
constexpr uint64_t kAgg = 1ull << 62, kInc = 2ull << 62, kValMask = (1ull << 62) - 1;

__device__ __forceinline__ void rec_store(uint64_t* p, uint64_t v) {
  __hip_atomic_store(p, v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}
__device__ __forceinline__ uint64_t rec_load(uint64_t* p) {
  return __hip_atomic_load(p, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}

// Exclusive prefix of the record values [base, me): decoupled look-back by one wave. Each probe
// reads 256 predecessors (4 per lane; position p = 4*lane + q counts back from me-1) and stops
// at the nearest inclusive record, so the inclusive front advances 256 tiles per round trip.
// Bounded spin.
__device__ __forceinline__ uint64_t lookback(uint64_t* recs, uint64_t base, uint64_t me, uint32_t* flags) {
  uint64_t excl = 0;
  int64_t pos = (int64_t)me - 1;
  const int lane = lane_id();
  uint32_t spins = 0;
  while (pos >= (int64_t)base) {
    uint64_t r[4];
    int stop = 256;
#pragma unroll
    for (int q = 0; q < 4; ++q) {  // all four loads in flight before any is used
      const int64_t idx = pos - (4 * lane + q);
      r[q] = rec_load(&recs[idx >= (int64_t)base ? idx : (int64_t)base]);
    }
#pragma unroll
    for (int q = 0; q < 4; ++q) {
      if (pos - (4 * lane + q) < (int64_t)base) r[q] = kInc;
      const uint64_t inc = __ballot((r[q] >> 62) == 2);
      if (inc) stop = min(stop, 4 * (int)__builtin_ctzll(inc) + q);
    }
    bool bad = false;
#pragma unroll
    for (int q = 0; q < 4; ++q) bad |= (4 * lane + q <= stop) && (r[q] >> 62) == 0;
    if (__ballot(bad)) {
      __builtin_amdgcn_s_sleep(2);
      if (++spins > (1u << 24)) {  // ~seconds: a record never arrived
        if (lane == 0) atomicOr(&flags[2], 1u);
        return excl;
      }
      continue;
    }
    uint64_t v = 0;
#pragma unroll
    for (int q = 0; q < 4; ++q) v += (4 * lane + q <= stop) ? (r[q] & kValMask) : 0;
    excl += wave_sum_u64(v);
    if (stop < 256) break;
    pos -= 256;
  }
  return excl;
}

// Bijective XCD-aware remap (cdna_hip_programming.md §5 "XCD swizzle must be bijective"):
// blocks that share an XCD (b % 8 equal) get a contiguous range of logical ids, so the
// chunks of consecutive rows -- which re-read each other as the row above -- share an L2.
__device__ __forceinline__ uint32_t xcd_remap(uint32_t b, uint32_t nb) {
  if (nb < 16) return b;
  const uint32_t q = nb / 8, r = nb % 8, x = b % 8;
  return (x < r ? x * (q + 1) : r * (q + 1) + (x - r) * q) + b / 8;
}

// GolombCoder.cpp:33 for n >= 1 samples with accumulated error A (A < 2^31):
// the smallest k >= 0 with (n << k) >= A, found from the two leading-one positions.
// (selects only, no branch: the per-codeword loops stay straight-line)
__device__ __forceinline__ uint32_t golomb_k(uint32_t n, uint32_t A) {
  const uint32_t k = (uint32_t)(__clz((int)n) - __clz((int)A));  // (meaningless when A <= n: unused)
  const uint32_t kk = k + ((n << (k & 31u)) < A ? 1u : 0u);
  return A <= n ? 0u : kk;
}
__device__ __forceinline__ uint32_t golomb_k_state(uint32_t n, uint32_t A) {
  const uint32_t k = golomb_k(n | (n == 0 ? 1u : 0u), A);  // (computed for every n: no branch)
  return n == 0 ? 1u : k;  // Golomb.h:18 -- a fresh coder starts at k = 1
}

__device__ __forceinline__ uint64_t bswap64(uint64_t x) { return __builtin_bswap64(x); }

// Bits of the Golomb codewords whose '1' lies in residual word w of a row (plus the end-of-row
// codeword when eol) -- the length the row encoder's emission produces for that word -- without
// forming any codeword. n = samples of the plane before the word's first 1, jp = column of the
// row's last 1 before the word (-1: none), arow = row * (cols + 1) (so A = arow + jp + 1 - n).
// When every codeword of the bits x has the same k (k bounds as in encode_word) and k <= 3, the
// sum of s >> k over the inner runs is counted word-parallel: an inner zero at column p adds one
// bit iff its index in its run is 2^k - 1 mod 2^k, i.e. iff p = j mod 2^k for the 1 at column j
// that opened the run. With the word bit-reversed (column b at significance b), the zeros following
// the 1s of one residue class c are Z & ~(Z + (E_c << 1)) (the carry of each E_c bit ripples
// through its run and stops at the next 1), so each class costs one add and a popcount
// (word_len_fast; x != 0, n >= 1; false when the bounds disagree or k > 3). Other words walk their
// codewords (GolombCoder.cpp:29-34 lengths), one per 1 and a branch-free step each (counting them byte
// by byte with per-byte bounds measured slower: C3 walk 19 -> 27 us, C2 31 -> 34 us).
// kor |= 1 << k for every k the codewords use (k capped at 31).
__device__ __forceinline__ bool word_len_fast(uint64_t x, uint32_t w, uint32_t n, int jp, uint32_t arow, bool eol,
                                              uint32_t cols, uint32_t& kor, uint32_t& len) {
  const uint32_t m = (uint32_t)__popcll(x);
  const uint32_t bf = (uint32_t)__builtin_clzll(x), bl = 63u - (uint32_t)__builtin_ctzll(x);
  const uint32_t pfirst = w * 64 + bf, plast = w * 64 + bl;
  const uint32_t khi = golomb_k(n, arow + plast - (n + m - 1));
  const uint32_t klo = golomb_k(n + m - 1 + (eol ? 1u : 0u), arow + (uint32_t)(jp + 1) - n);
  if (khi != klo || khi > 3) return false;
  const uint32_t k = khi;
  kor |= 1u << k;
  len = m * (k + 1) + ((pfirst - (uint32_t)(jp + 1)) >> k);
  if (eol) len += k + 1 + ((cols - 1 - plast) >> k);
  if (m > 1) {
    const uint64_t xr = __builtin_bitreverse64(x);
    const uint64_t between = ((1ull << bl) - 1ull) & ~((2ull << bf) - 1ull);  // bf < bl here
    const uint64_t Z = ~xr & between;
    if (k == 0) {
      len += (uint32_t)__popcll(Z);
    } else {
      const uint64_t pat = k == 1 ? 0x5555555555555555ull : (k == 2 ? 0x1111111111111111ull : 0x0101010101010101ull);
      const uint32_t ncls = 1u << k;
      uint64_t rest = Z;
      for (uint32_t c = 0; c + 1 < ncls; ++c) {
        const uint64_t P = pat << c;
        const uint64_t F = Z & ~(Z + ((xr & P) << 1));
        len += (uint32_t)__popcll(F & P);
        rest &= ~F;
      }
      len += (uint32_t)__popcll(rest & (pat << (ncls - 1)));
    }
  }
  return true;
}
__device__ __forceinline__ uint32_t word_len(uint64_t x, uint32_t w, uint32_t n, int jp, uint32_t arow, bool eol,
                                             uint32_t cols, uint32_t& kor) {
  if (!x && !eol) return 0;
  uint32_t len = 0;
  if (x && n && word_len_fast(x, w, n, jp, arow, eol, cols, kor, len)) return len;
  // one codeword at a time: A = arow + jp + 1 - n grows by each run (A' = A + s as n' = n + 1)
  uint32_t A = arow + (uint32_t)(jp + 1) - n;
  len = 0;
  while (x) {
    const int cz = __builtin_clzll(x);
    x ^= BIC_MSB >> cz;
    const int j = (int)(w * 64) + cz;
    const uint32_t s = (uint32_t)(j - jp - 1);
    const uint32_t k = golomb_k_state(n, A);
    kor |= 1u << min(k, 31u);
    len += k + 1 + (s >> k);
    A += s;
    ++n;
    jp = j;
  }
  if (eol) {  // the end-of-row codeword
    const uint32_t k = golomb_k_state(n, A);
    kor |= 1u << min(k, 31u);
    len += k + 1 + ((cols - 1 - (uint32_t)jp) >> k);
  }
  return len;
}

// word_len, also returning which codewords have k = 1: kt gets the bit of every 1 of x whose codeword
// has k = 1, keol (eol) the end-of-row codeword's k == 1 (the masks of bic_k1pi.h kmix_*)
__device__ __forceinline__ uint32_t word_len_kt(uint64_t x, uint32_t w, uint32_t n, int jp, uint32_t arow, bool eol,
                                                uint32_t cols, uint32_t& kor, uint64_t& kt, uint32_t& keol) {
  kt = 0;
  keol = 0;
  if (!x && !eol) return 0;
  uint32_t len = 0;
  if (x && n) {
    const uint32_t k0 = kor;
    kor = 0;
    if (word_len_fast(x, w, n, jp, arow, eol, cols, kor, len)) {
      kt = kor == 2u ? x : 0ull;  // (one k for the word's codewords, the end-of-row one included)
      keol = eol && kor == 2u ? 1u : 0u;
      kor |= k0;
      return len;
    }
    kor = k0;
  }
  uint32_t A = arow + (uint32_t)(jp + 1) - n;
  len = 0;
  while (x) {
    const int cz = __builtin_clzll(x);
    x ^= BIC_MSB >> cz;
    const int j = (int)(w * 64) + cz;
    const uint32_t s = (uint32_t)(j - jp - 1);
    const uint32_t k = golomb_k_state(n, A);
    kor |= 1u << min(k, 31u);
    kt |= k == 1 ? BIC_MSB >> cz : 0ull;
    len += k + 1 + (s >> k);
    A += s;
    ++n;
    jp = j;
  }
  if (eol) {
    const uint32_t k = golomb_k_state(n, A);
    kor |= 1u << min(k, 31u);
    keol = k == 1 ? 1u : 0u;
    len += k + 1 + ((cols - 1 - (uint32_t)jp) >> k);
  }
  return len;
}

// ------------------------------------------------------------------------------------
// residual word of a chunk step (med in word form), shared by every chunk kernel
// ------------------------------------------------------------------------------------
struct RowCtx {
  const uint64_t* cur;  // row i
  const uint64_t* up;   // row i-1 (nullptr for i = 0)
  uint64_t pcarry, ucarry;  // left neighbours of lane 0 for the next step
};

__device__ __forceinline__ RowCtx row_ctx(const uint64_t* planes, const Geom& g, uint32_t plane,
                                          uint32_t row, uint32_t c0) {
  RowCtx rc;
  rc.cur = planes + (uint64_t)plane * g.plane_words + (uint64_t)row * g.wpr;
  rc.up = row ? rc.cur - g.wpr : nullptr;
  rc.pcarry = c0 ? rc.cur[c0 - 1] : 0;
  rc.ucarry = (c0 && rc.up) ? rc.up[c0 - 1] : 0;
  return rc;
}

template <bool PREDICT>
__device__ __forceinline__ uint64_t resid_word(RowCtx& rc, const Geom& g, uint32_t row, uint32_t w) {
  const bool valid = w < g.used;
  const uint64_t p = valid ? rc.cur[w] : 0;
  uint64_t r;
  if constexpr (PREDICT) {
    const uint64_t u = (valid && rc.up) ? rc.up[w] : 0;
    uint64_t pl = shfl_up_u64(p, 1), ul = shfl_up_u64(u, 1);
    if (lane_id() == 0) { pl = rc.pcarry; ul = rc.ucarry; }
    rc.pcarry = lane63_u64(p);
    rc.ucarry = lane63_u64(u);
    r = p ^ u ^ ((p >> 1) | (pl << 63)) ^ ((u >> 1) | (ul << 63));
    if (row == 0 && w == 0) r &= ~BIC_MSB;  // pred.cpp never writes pP(0,0)
  } else {
    r = p;
  }
  if (w == g.used - 1) r &= g.trail;
  return valid ? r : 0;
}

// The residual words of one row for lane words w = t*64 + lane (t < WPL), zero past the row.
// Every load is issued before any is used (addresses clamped into the row), so the wave pays
// one memory latency, not WPL of them. With D = P ^ U the med residual is D ^ (D >> 1 | Dl << 63)
// (shifts distribute over XOR), one cross-lane shuffle per word.
template <int WPL, bool PREDICT>
__device__ __forceinline__ void resid_row(const uint64_t* planes, const Geom& g, uint32_t plane, uint32_t row,
                                          uint64_t (&r)[WPL], uint32_t c0 = 0) {
  const int lane = lane_id();
  const uint64_t* cur = planes + (uint64_t)plane * g.plane_words + (uint64_t)row * g.wpr;
  const uint64_t* up = row ? cur - g.wpr : cur;
  uint64_t p[WPL], u[WPL];
#pragma unroll
  for (int t = 0; t < WPL; ++t) {
    const uint32_t w = c0 + t * 64 + lane;
    const uint32_t wc = w < g.used ? w : g.used - 1;
    p[t] = cur[wc];
    if constexpr (PREDICT) u[t] = up[wc];
  }
  uint64_t carry = 0;  // D of the word left of the chunk (chunks after the first of a row)
  if (PREDICT && c0) carry = cur[c0 - 1] ^ (row ? up[c0 - 1] : 0);
#pragma unroll
  for (int t = 0; t < WPL; ++t) {
    const uint32_t w = c0 + t * 64 + lane;
    uint64_t d = p[t];
    if constexpr (PREDICT) {
      if (row) d ^= u[t];
      uint64_t dl = shfl_up_u64(d, 1);
      if (lane == 0) dl = carry;
      carry = lane63_u64(d);
      d ^= (d >> 1) | (dl << 63);
      if (row == 0 && w == 0) d &= ~BIC_MSB;  // pred.cpp never writes pP(0,0)
    }
    if (w == g.used - 1) d &= g.trail;
    r[t] = w < g.used ? d : 0;
  }
}

// resid_row (c0 = 0) split into its loads and its arithmetic, so a loop can have the next row's
// loads in flight while it works on this one.
template <int WPL, bool PREDICT>
__device__ __forceinline__ void row_load(const uint64_t* planes, const Geom& g, uint32_t plane, uint32_t row,
                                         uint64_t (&p)[WPL], uint64_t (&u)[WPL]) {
  const uint64_t* cur = planes + (uint64_t)plane * g.plane_words + (uint64_t)row * g.wpr;
  const uint64_t* up = row ? cur - g.wpr : cur;
#pragma unroll
  for (int t = 0; t < WPL; ++t) {
    const uint32_t w = t * 64 + lane_id();
    const uint32_t wc = w < g.used ? w : g.used - 1;
    p[t] = cur[wc];
    u[t] = PREDICT && row ? up[wc] : 0;
  }
}
template <int WPL, bool PREDICT>
__device__ __forceinline__ void row_resid(const Geom& g, uint32_t row, const uint64_t (&p)[WPL],
                                          const uint64_t (&u)[WPL], uint64_t (&r)[WPL]) {
  const int lane = lane_id();
  uint64_t carry = 0;
#pragma unroll
  for (int t = 0; t < WPL; ++t) {
    const uint32_t w = t * 64 + lane;
    uint64_t d = p[t];
    if constexpr (PREDICT) {
      d ^= u[t];
      uint64_t dl = shfl_up_u64(d, 1);
      if (lane == 0) dl = carry;
      carry = lane63_u64(d);
      d ^= (d >> 1) | (dl << 63);
      if (row == 0 && w == 0) d &= ~BIC_MSB;  // pred.cpp never writes pP(0,0)
    }
    if (w == g.used - 1) d &= g.trail;
    r[t] = w < g.used ? d : 0;
  }
}

struct ChunkId {
  uint32_t plane, row, c;
  uint64_t id;
  bool ok;
};
__device__ __forceinline__ ChunkId chunk_id(const Geom& g) {
  ChunkId ci;
  const uint32_t b = xcd_remap(blockIdx.x, gridDim.x);
  ci.id = (uint64_t)b * kWaves + wave_id();
  ci.ok = ci.id < g.nchunks;
  const uint64_t id = ci.ok ? ci.id : 0;
  ci.plane = (uint32_t)(id / g.chunks_per_plane);
  const uint64_t r = id % g.chunks_per_plane;
  ci.row = (uint32_t)(r / g.cpr);
  ci.c = (uint32_t)(r % g.cpr);
  return ci;
}

// ------------------------------------------------------------------------------------
// Shared per-step bookkeeping of the Golomb kernels: for the lane's word, the sample
// index of its first 1 and the column of the last 1 before it in the row.
// ------------------------------------------------------------------------------------
struct StepState {
  uint32_t n_carry;
  int jp_carry;
};

__device__ __forceinline__ void step_prefix(uint64_t r, uint32_t w, StepState& st, uint32_t& n_w,
                                            int& jp_w) {
  const uint32_t pc = (uint32_t)__popcll(r);
  const uint32_t inc = wave_incl_sum_u32(pc);
  n_w = st.n_carry + inc - pc;
  st.n_carry += lane63_u32(inc);
  const int lastc = r ? (int)(w * 64 + 63 - __builtin_ctzll(r)) : -1;
  const int mx = wave_incl_max(lastc);
  const int ex = dpp_or<0x138>(-1, mx);  // lane 0: -1
  jp_w = max(st.jp_carry, ex);
  st.jp_carry = max(st.jp_carry, (int)lane63_u32((uint32_t)mx));
}


// The column of the row's last 1 before the lane's word (-1: none), carried across steps.
__device__ __forceinline__ int step_jp(uint64_t r, uint32_t w, int& jp_carry) {
  const int lastc = r ? (int)(w * 64 + 63 - __builtin_ctzll(r)) : -1;
  const int mx = wave_incl_max(lastc);
  const int ex = dpp_or<0x138>(-1, mx);  // lane 0: -1
  const int jp = max(jp_carry, ex);
  jp_carry = max(jp_carry, (int)lane63_u32((uint32_t)mx));
  return jp;
}

// Codeword sinks: OR the bits of a codeword (k-bit binary part, then the '1' after the
// unary zeros) into an LDS image (u32 words) or into global big-endian 64-bit words.
struct LdsSink {
  uint32_t* buf;
  uint32_t idx, cur;
  __device__ __forceinline__ void flush() {
    if (cur) atomicOr(&buf[idx], cur);
    cur = 0;
  }
  __device__ __forceinline__ void orw(uint32_t i, uint32_t v) {
    if (i != idx) { flush(); idx = i; }
    cur |= v;
  }
  // nb <= 32 bits of v at local bit offset off (MSB-first)
  __device__ __forceinline__ void put(uint32_t off, uint32_t v, uint32_t nb) {
    const uint32_t i = off >> 5, sh = off & 31;
    if (sh + nb <= 32) {
      orw(i, v << (32 - sh - nb));
    } else {
      orw(i, v >> (sh + nb - 32));
      orw(i + 1, v << (64 - sh - nb));
    }
  }
  __device__ __forceinline__ void bit(uint32_t off) { orw(off >> 5, 0x80000000u >> (off & 31)); }
};

// (hi:lo) >> sh, low 64 bits, for sh in 0..63: two v_alignbit_b32 (a 64-bit funnel shift) when sh
// is wave-uniform, instead of two 64-bit shifts, an or and the sh == 0 select.
__device__ __forceinline__ uint64_t funnel64(uint64_t hi, uint64_t lo, uint32_t sh) {
  const uint32_t h1 = (uint32_t)(hi >> 32), h0 = (uint32_t)hi, l1 = (uint32_t)(lo >> 32), l0 = (uint32_t)lo;
  uint32_t r1, r0;
  if (sh < 32) {  // ({h0, l1, l0} >> sh)
    r1 = __builtin_amdgcn_alignbit(h0, l1, sh);
    r0 = __builtin_amdgcn_alignbit(l1, l0, sh);
  } else {  // ({h1, h0, l1} >> (sh - 32))
    r1 = __builtin_amdgcn_alignbit(h1, h0, sh - 32);
    r0 = __builtin_amdgcn_alignbit(h0, l1, sh - 32);
  }
  return ((uint64_t)r1 << 32) | r0;
}

// Zero a wave's 32-bit LDS row image (n16 16-byte units) before codewords are OR'd into it with 4-byte
// LDS atomics: the 16-byte zero stores are drained (s_waitcnt lgkmcnt(0)) before the first atomic issues,
// and the asm's "memory" clobber also keeps the compiler from moving any LDS access across it.
// Round 4's k_emit_k1 zeroed its 64-bit image with 16-byte stores and OR'd 8-byte atomics into it with
// neither; on the first encode of a process, with k_emit_rest's workgroups sharing the CUs, its k = 1 rows
// lost about a quarter of their 1 bits. Its ISA (profiles/r06/isa_67ba6e6_k_emit_k1.txt)
// has every ds_write_b128 of the zeroing before every ds_or_b64 of the row, over exactly the wave's own
// 684 words: neither a compiler reordering nor the extent. What measured clean is the same-width form:
// the 64-bit images zero with 8-byte stores of the atomics' own width and type (k1_rows, emit_known_row);
// this drain guards the mixed-width 32-bit images against the same hazard.
__device__ __forceinline__ void lds_image_zero32(uint32_t* img, uint32_t n16) {
  uint4* z = reinterpret_cast<uint4*>(img);
  for (uint32_t i = lane_id(); i < n16; i += 64) z[i] = make_uint4(0, 0, 0, 0);
  asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
}

// A row image of 64-bit LDS words (bit 64 i + b at significance 63 - b of word i), OR'd with
// ds_or_b64: a lane's string (<= 128 bits at any offset) lands in at most three words.
__device__ __forceinline__ void lds_or64(uint64_t* img, uint32_t i, uint64_t v) {
  if (v) atomicOr(reinterpret_cast<unsigned long long*>(img + i), (unsigned long long)v);
}
// write_row for a 64-bit LDS image (bic_fused.hip place128_64, bic_egad.hip): output word t of the row holds image bits
// [64 t - G % 64, 64 t - G % 64 + 64): two LDS words and a funnel shift.
__device__ __forceinline__ void write_row64(const uint64_t* img, uint64_t L, uint64_t G, uint64_t* out,
                                            uint64_t* frag) {
  const uint64_t w0 = G >> 6, w1 = (G + L - 1) >> 6;
  const uint32_t nw = (uint32_t)(w1 - w0 + 1), g = (uint32_t)(G & 63);
  const bool head_whole = g == 0, tail_whole = ((G + L) & 63) == 0;
  for (uint32_t t = lane_id(); t < nw; t += 64) {
    const uint64_t cur = img[t], prev = t ? img[t - 1] : 0ull;
    const uint64_t v = funnel64(prev, cur, g);
    const bool whole = (t != 0 || head_whole) && (t != nw - 1 || tail_whole);
    if (whole) out[w0 + t] = bswap64(v);
    else if (frag) frag[t == 0 ? 0 : 1] = v;
    else atomicOr(reinterpret_cast<unsigned long long*>(out + w0 + t), (unsigned long long)bswap64(v));  // zeroed shared word
  }
}

struct GlobalSink {
  unsigned long long* buf;  // big-endian 64-bit words
  uint64_t idx, cur;
  __device__ __forceinline__ void flush() {
    if (cur) atomicOr(&buf[idx], (unsigned long long)bswap64(cur));
    cur = 0;
  }
  __device__ __forceinline__ void orw(uint64_t i, uint64_t v) {
    if (i != idx) { flush(); idx = i; }
    cur |= v;
  }
  __device__ __forceinline__ void put(uint64_t off, uint32_t v, uint32_t nb) {
    const uint64_t i = off >> 6;
    const uint32_t sh = (uint32_t)(off & 63);
    if (sh + nb <= 64) {
      orw(i, (uint64_t)v << (64 - sh - nb));
    } else {
      orw(i, (uint64_t)v >> (sh + nb - 64));
      orw(i + 1, (uint64_t)v << (128 - sh - nb));
    }
  }
  __device__ __forceinline__ void bit(uint64_t off) { orw(off >> 6, BIC_MSB >> (off & 63)); }
};

template <typename Sink, typename Off>
__device__ __forceinline__ void emit_codeword(Sink& sk, Off off, uint32_t s, uint32_t k) {
  if (k) {
    const uint32_t bin = s & ((1u << k) - 1u);
    if (bin) sk.put(off, bin, k);
  }
  sk.bit(off + k + (s >> k));
}

}  // namespace bic
