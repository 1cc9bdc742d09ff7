// bic_fused.hip -- row encoders for rows of up to 256 words (16384 columns): med residual ->
// per-row runs -> Golomb stream and/or EG stream, one wavefront per row, 16-row tiles.
//
// Semantics are those of bic_kernels.hip (GolombCoder.cpp:13-34, eg.cpp:20-37, pred.cpp:3-15);
// the difference is the schedule. The default single kernel (k_encode_rows):
//  * tiles are claimed in order through an atomic ticket, so every tile a workgroup looks back
//    at was claimed earlier and is running or finished (no deadlock, whatever the dispatch order);
//  * the tile's 1-count is published at once and a decoupled look-back over the earlier tiles
//    of the plane yields the number of samples before each row (the Golomb coder state);
//  * every codeword is computed ONCE: each lane turns its word into a register string
//    (first codeword's binary part, its unary zeros, then <= 128 bits), or -- when the k
//    bounds prove k = 0 for every codeword of the word -- copies the word's bits (a k = 0
//    codeword is exactly the run's zeros and its 1); constant k = 1..3 words go byte by byte
//    through precomputed tables;
//  * lane strings are OR'd into an LDS row image; the tile's bit length is published and a
//    second look-back gives its offset; whole 64-bit words go to HBM with plain stores and
//    the (at most two) words shared with neighbouring rows go to a fragment table that the
//    fixup kernel combines (no atomics on the output, no pre-zeroing of the output).
// The two-pass option (k_len_rows, k_emit_rows) computes lengths and offsets first and then
// writes every row independently; same output, slower.
// Inter-workgroup records are 8-byte {flag, value} granules written and polled with
// agent-scope atomics (cdna_hip_programming.md §6 Guideline 16, R2), spins bounded.
#include "bic_device.h"
#include "bic_k1pi.h"  // the k = 1 rows' backward-parity encoder (host-compilable: tests/cpp/k1pi_check.cpp)
#include "bic_kstat.h"

#include <algorithm>

namespace bic {

#ifdef BIC_STAMPS  // diagnostic build only (make stamps): per-wave phase clocks, never in the product
__device__ unsigned long long g_stamps[1 << 22];
// BIC_KNOWN=1 (diagnostic): replay the tile prefixes recorded by the previous normal launch
// instead of looking them back, to measure what the look-back waits cost
__device__ unsigned long long g_known[2][1 << 17];
#define STAMP(slot)                                                                        \
  do {                                                                                     \
    const unsigned long long t_ = __builtin_amdgcn_s_memtime();                            \
    if (lane == 0 && (uint64_t)id * 8 + (slot) < (1u << 21)) g_stamps[(uint64_t)id * 8 + (slot)] = t_; \
  } while (0)
// k_row_walk's phases (slots 4-7 of the row: entry, residual word loaded, length walked, stored), on
// the 100 MHz clock every XCD shares (s_memrealtime), waiting for the phase's loads first
#define WSTAMP(slot)                                                                               \
  do {                                                                                             \
    asm volatile("s_waitcnt vmcnt(0) lgkmcnt(0)" ::: "memory");                                    \
    const unsigned long long t_ = __builtin_amdgcn_s_memrealtime();                                \
    if (threadIdx.x == 0 && (uint64_t)id * 8 + (slot) < (1u << 21)) g_stamps[(uint64_t)id * 8 + (slot)] = t_; \
  } while (0)
// k_scan_rows' phases per workgroup (slots of g_stamps from 1 << 21: ONES scan, then LEN scan)
#define SSTAMP(slot)                                                                              \
  do {                                                                                            \
    asm volatile("s_waitcnt vmcnt(0) lgkmcnt(0)" ::: "memory");                                   \
    const unsigned long long t_ = __builtin_amdgcn_s_memrealtime();                               \
    if (threadIdx.x == 0) g_stamps[(1u << 21) + (ONES ? 0u : 8192u) + blockIdx.x * 8u + (slot)] = t_; \
  } while (0)
// the class launch's phases (tools/k01_stamps.py), 4 slots per index: per kmix row (index 1 << 18 + its
// row id; slots 0-2: entry, loads done, stored), per wave of k_emit_k01 (index 1 << 19 + 8192 + its wave;
// slots 0-3: entry, k = 0 rows done (rest role: kmix rows done), -, exit)
#define XSTAMP(idx, slot)                                                                          \
  do {                                                                                             \
    asm volatile("s_waitcnt vmcnt(0) lgkmcnt(0)" ::: "memory");                                    \
    const unsigned long long t_ = __builtin_amdgcn_s_memrealtime();                                \
    if (lane_id() == 0 && (uint64_t)(idx) * 4 + (slot) < (1u << 22)) g_stamps[(uint64_t)(idx) * 4 + (slot)] = t_; \
  } while (0)
// (the same without draining the memory counters first: the instruction's issue time)
#define YSTAMP(idx, slot)                                                                          \
  do {                                                                                             \
    const unsigned long long t_ = __builtin_amdgcn_s_memrealtime();                                \
    if (lane_id() == 0 && (uint64_t)(idx) * 4 + (slot) < (1u << 22)) g_stamps[(uint64_t)(idx) * 4 + (slot)] = t_; \
  } while (0)
#else
#define XSTAMP(idx, slot) \
  do {                    \
  } while (0)
#define YSTAMP(idx, slot) \
  do {                    \
  } while (0)
#define STAMP(slot) \
  do {              \
  } while (0)
#define WSTAMP(slot) \
  do {               \
  } while (0)
#define SSTAMP(slot) \
  do {               \
  } while (0)
#endif

constexpr int kTileRows = 16;  // rows (= waves) per workgroup tile (C3: 666 us vs 677 at 8 rows)
constexpr int kGImg = 684;    // u32 words of Golomb row image per wave (21760 bits; with the EG image and
                              // the k = 1, 2 byte tables 4 workgroups (32 waves) fit one CU's LDS)
constexpr int kEImg = 520;    // u32 words of EG row image per wave (cols <= 16384)
constexpr int kPad = 4;       // zeroed words after an image's end (get64 reads ahead)
#ifndef BIC_K1_LC
#define BIC_K1_LC 1  // lane l holds the row's words l WPL .. (one wave scan per row, not per word group)
#endif
#ifndef BIC_K1_PI
#define BIC_K1_PI 1  // k = 1 rows by the backward parity (k1_pi, the [pi][byte] table); 0: encode_word_k1b
#endif
#if BIC_K1_PI && !BIC_K1_LC
#error "BIC_K1_PI needs BIC_K1_LC"
#endif
constexpr uint32_t kK1Table = BIC_K1_PI ? 512u : 0u;  // the k = 1 rows' table in the u32 byte tables
#ifndef BIC_KNOWN_PI
// k_emit_known's k = 1 rows (C4, C2, predict): 1 the backward parity, 0 encode_word_k1b (C4 0.268 ms
// against 0.283 with the parity's strided lanes)
#define BIC_KNOWN_PI 0
#endif
constexpr uint32_t kKnownTable = BIC_KNOWN_PI ? 512u : 0u;
#ifndef BIC_SLOW_REST
#define BIC_SLOW_REST 1  // class kernels' path: the slow rows by k_emit_rest (listed by the LEN scan), no k_rows_global
#endif
constexpr bool kSlowRest = BIC_SLOW_REST != 0;
#ifndef BIC_K01_REST
#define BIC_K01_REST 0
#endif
// the class kernels' path (EG source): the mixed-k and slow rows by k_emit_k01's own leading workgroups
// (rest_role: one CU slot each, beside the persistent class waves) instead of k_emit_rest on the second
// stream -- the emission is one launch, without the fork / join events
constexpr bool kK01Rest = BIC_K01_REST != 0;
#ifndef BIC_KMIX
#define BIC_KMIX 0
#endif
// the class kernels' path: rows mixing k = 0 and k = 1 by kmix_rows inside k_emit_k01 (the walk's k = 1
// masks, bic_k1pi.h kmix_*) instead of k_emit_rest's per-codeword encoder
constexpr bool kKMixRows = BIC_KMIX != 0;
#ifndef BIC_KNOWN_MIX
#define BIC_KNOWN_MIX 0
#endif
// k_emit_known (planes in, Golomb alone: C4's path): the walked rows mixing k = 0 and k = 1 written by the
// row's own wave from the walk's k = 1 masks (kmix_encode) instead of by k_emit_rest beside it
constexpr bool kKnownMix = BIC_KNOWN_MIX != 0;
#ifndef BIC_K01_RG
#define BIC_K01_RG 0  // (A/B: the rest role's workgroups; 0: one per CU, the persistent ones one fewer per CU)
#endif
constexpr uint32_t kK01Rg = BIC_K01_RG;
#ifndef BIC_K01_PRIO
#define BIC_K01_PRIO 0
#endif
#ifndef BIC_K01_RLAST
#define BIC_K01_RLAST 0
#endif
constexpr bool kK01Prio = BIC_K01_PRIO != 0, kK01RLast = BIC_K01_RLAST != 0;

// One lane's codewords for one residual word.
struct LaneEnc {
  uint32_t head, k0, z;  // first codeword: k0-bit binary part, then z unary zeros
  uint64_t t0, t1;       // the rest (starting with the first codeword's '1'), MSB-first
  uint32_t tlen;
  uint32_t len;          // total bits
  bool lng;              // rest longer than 128 bits: placed by re-iteration
#ifdef BIC_STAMPS
  uint32_t path;         // diagnostic: 1 copy mode, 2 byte table, 3 per-codeword loop
#endif
};

__device__ __forceinline__ void tail_put(LaneEnc& e, uint64_t cw, uint32_t nb) {  // nb 1..64
  const uint32_t pos = e.tlen;
  e.tlen = pos + nb;
  if (pos + nb > 128) { e.lng = true; return; }
  const uint32_t sh = 128 - pos - nb;
  if (sh >= 64) {
    e.t0 |= cw << (sh - 64);
  } else {
    e.t1 |= cw << sh;
    if (sh + nb > 64) e.t0 |= cw >> (64 - sh);
  }
}

// Byte tables for words whose codewords all share one k in 1..3 (built on the host,
// bic_kernels.hip build_byte_lut): for a byte v != 0, the codewords that lie wholly inside the
// byte (after its first 1) as one right-aligned pattern R of lr bits, plus the byte's leading (t)
// and trailing (tz) zeros. k = 1, 2: packed u32 R | lr << 21 | t << 26 | tz << 29, staged in LDS
// by the encoder; k = 3: u64 R | lr << 32 | t << 40 | tz << 44 from global memory.
struct ByteTables {
  const uint32_t* t12;  // [2][256]
  const uint64_t* t3;   // [256]
};
__device__ __forceinline__ void tail_put_n(LaneEnc& e, uint64_t cw, uint32_t nb) {
  if (nb) tail_put(e, cw, nb);
}

// STR = false computes only e.len (the length pass of the two-pass encoder).
template <bool STR = true>
__device__ __forceinline__ LaneEnc encode_word(uint64_t x, uint32_t w, uint32_t n, int jp, uint32_t arow,
                                               bool eol, uint32_t cols, ByteTables lut) {
  LaneEnc e{};
  if (!x && !eol) return e;
  if (x && n) {
    // A never decreases and n only grows along the word, so every codeword's k lies between
    // k(n_last, A_first) and k(n_first, A_last); when the two agree, k is the same throughout.
    const uint32_t m = (uint32_t)__popcll(x);
    const uint32_t plast = w * 64 + 63 - (uint32_t)__builtin_ctzll(x);
    const uint32_t aup = arow + plast - (n + m - 1);  // >= A of the last codeword (and = A of the EOL's)
    const uint32_t afirst = arow + (uint32_t)(jp + 1) - n;
    const uint32_t khi = golomb_k(n, aup);
    const uint32_t klo = golomb_k(n + m - 1 + (eol ? 1u : 0u), afirst);
    if (khi == klo && khi == 0) {
      // k = 0: a codeword is its run's zeros and the 1 -- the word's bits verbatim
      e.z = w * 64 - (uint32_t)(jp + 1);
      e.t0 = x;
      if (!eol) {
        e.tlen = plast - w * 64 + 1;
      } else {
        const uint32_t p = cols - w * 64;  // the EOL codeword's '1'
        if (p < 64) e.t0 |= BIC_MSB >> p; else e.t1 = BIC_MSB;
        e.tlen = p + 1;
      }
      e.len = e.z + e.tlen;
#ifdef BIC_STAMPS
      e.path = 1;
#endif
      return e;
    }
    if (khi == klo && khi <= 3) {
#ifdef BIC_STAMPS
      e.path = 2;
#endif
      const uint32_t k = khi, kmask = (1u << k) - 1u;
      uint32_t c = w * 64 - (uint32_t)(jp + 1);  // zeros of the open run
      bool first = true;
      const uint32_t* T = lut.t12 + (k - 1) * 256;
#pragma unroll
      for (int b = 0; b < 8; ++b) {
        const uint32_t v = (uint32_t)(x >> (56 - 8 * b)) & 0xffu;
        if (v) {
          uint32_t R, lr, t, tz;
          if (k <= 2) {
            const uint32_t en = T[v];
            R = en & 0x1fffffu;
            lr = (en >> 21) & 31u;
            t = (en >> 26) & 7u;
            tz = en >> 29;
          } else {
            const uint64_t en = lut.t3[v];
            R = (uint32_t)en;
            lr = (uint32_t)(en >> 32) & 63u;
            t = (uint32_t)(en >> 40) & 15u;
            tz = (uint32_t)(en >> 44) & 15u;
          }
          const uint32_t sr = c + t, q = sr >> k, bin = sr & kmask;
          if constexpr (STR) {
            if (first) {
              e.head = bin;
              e.k0 = k;
              e.z = q;
              tail_put(e, (1ull << lr) | R, 1 + lr);
              first = false;
            } else {
              const uint32_t nb = k + q + 1;  // sr <= 63 here
              if (nb + lr <= 64) {
                tail_put(e, ((((uint64_t)bin << (q + 1)) | 1ull) << lr) | R, nb + lr);
              } else {
                tail_put(e, ((uint64_t)bin << (q + 1)) | 1ull, nb);
                tail_put_n(e, R, lr);
              }
            }
          }
          e.len += k + q + 1 + lr;
          c = tz;
        } else {
          c += 8;
        }
      }
      if (eol) {  // the row's trailing zeros (pad columns excluded)
        const uint32_t sr = c - (w * 64 + 64 - cols), q = sr >> k;
        if constexpr (STR) tail_put(e, ((uint64_t)(sr & kmask) << (q + 1)) | 1ull, k + q + 1);
        e.len += k + q + 1;
      }
      return e;
    }
  }
  // k changes inside the word (or n = 0, the plane's first sample): one codeword at a time, the
  // word's first one (binary part and unary zeros cut off: head, z) peeled off the loop, and
  // A = arow + jp + 1 - n carried (A' = A + s as n' = n + 1). (Byte by byte with per-byte k bounds
  // measured slower.)
#ifdef BIC_STAMPS
  e.path = 3;
#endif
  uint32_t A = arow + (uint32_t)(jp + 1) - n;
  {
    uint32_t s;
    int j;
    if (x) {
      const int cz = __builtin_clzll(x);
      x ^= BIC_MSB >> cz;
      j = (int)(w * 64) + cz;
      s = (uint32_t)(j - jp - 1);
    } else {  // (eol: the row's end-of-row codeword alone)
      j = (int)cols;
      s = cols - 1 - (uint32_t)jp;
      eol = false;
    }
    const uint32_t k = golomb_k_state(n, A);
    const uint32_t q = s >> k;
    if constexpr (STR) {
      e.head = s & ((1u << k) - 1u);
      e.k0 = k;
      e.z = q;
      tail_put(e, 1, 1);
    }
    e.len += k + q + 1;
    A += s;
    ++n;
    jp = j;
  }
  while (x) {  // (n >= 1 from here; s <= 62: k + q + 1 <= 64)
    const int cz = __builtin_clzll(x);
    x ^= BIC_MSB >> cz;
    const int j = (int)(w * 64) + cz;
    const uint32_t s = (uint32_t)(j - jp - 1);
    const uint32_t k = golomb_k(n, A), q = s >> k;
    if constexpr (STR) tail_put(e, ((uint64_t)(s & ((1u << k) - 1u)) << (q + 1)) | 1ull, k + q + 1);
    e.len += k + q + 1;
    A += s;
    ++n;
    jp = j;
  }
  if (eol) {
    const uint32_t s = cols - 1 - (uint32_t)jp;
    const uint32_t k = golomb_k(n, A), q = s >> k;
    if constexpr (STR) tail_put(e, ((uint64_t)(s & ((1u << k) - 1u)) << (q + 1)) | 1ull, k + q + 1);
    e.len += k + q + 1;
  }
  return e;
}

// OR the nb (1..64) low bits of v into the 128-bit MSB-first string (t0, t1) at bit pos
// (pos + nb <= 128 whenever v != 0), branch-free.
__device__ __forceinline__ void or128(uint64_t& t0, uint64_t& t1, uint64_t v, uint32_t pos, uint32_t nb) {
  const uint32_t end = pos + nb;
  const uint64_t p0 = end <= 64 ? v << ((64 - end) & 63) : v >> ((end - 64) & 63);
  t0 |= pos < 64 ? p0 : 0ull;
  t1 |= end > 64 ? v << ((128 - end) & 63) : 0ull;
}

// encode_word for a row whose codewords all have k = 1 (kK1Row): no k bounds, no sample count, no
// divergent paths. The first codeword (binary part in head, its q zeros in z) is cut off as in
// encode_word; the rest goes byte by byte through the k = 1 table: byte i's first 1 closes the open
// run (c zeros before the byte + t): its binary bit, q zeros, then the table's '1' + R -- one
// pattern appended to a right-aligned 128-bit accumulator (two 64-bit shifts and an or); the word's
// first byte appends '1' + R only. <= 128 bits except through long runs (then lng: placed by
// emit_word_k1).
__device__ __forceinline__ void acc_put(uint64_t& hi, uint64_t& lo, uint64_t pat, uint32_t nb) {  // nb 1..63
  hi = (hi << nb) | (lo >> (64 - nb));
  lo = (lo << nb) | pat;
}
__device__ __forceinline__ void acc_zeros(uint64_t& hi, uint64_t& lo, uint32_t nb) {  // nb <= 128
  if (nb >= 64) {
    hi = lo;
    lo = 0;
    nb -= 64;
  }
  if (nb) {
    hi = (hi << nb) | (lo >> (64 - nb));
    lo <<= nb;
  }
}
// append bin, q zeros, then pat (np bits, 1..63): total 1 + q + np bits
__device__ __forceinline__ void acc_codeword(uint64_t& hi, uint64_t& lo, uint32_t& p, uint32_t bin, uint32_t q,
                                             uint64_t pat, uint32_t np) {
  const uint32_t nb = 1 + q + np;
  if (p + nb <= 128) {
    if (nb <= 63) {
      acc_put(hi, lo, ((uint64_t)bin << (nb - 1)) | pat, nb);
    } else {
      acc_put(hi, lo, bin, 1);
      acc_zeros(hi, lo, q);
      acc_put(hi, lo, pat, np);
    }
  }
  p += nb;
}

__device__ __forceinline__ LaneEnc encode_word_k1(uint64_t x, uint32_t w, int jp, bool eol, uint32_t cols,
                                                  const uint32_t* T1) {
  LaneEnc e{};
  e.k0 = 1;
  uint32_t c = w * 64 - (uint32_t)(jp + 1);  // zeros of the open run
  if (!x) {
    if (eol) {
      const uint32_t s = cols - 1 - (uint32_t)jp;
      e.head = s & 1u;
      e.z = s >> 1;
      e.t0 = BIC_MSB;
      e.tlen = 1;
      e.len = 2 + e.z;
    }
    return e;
  }
  const uint32_t bf = (uint32_t)__builtin_clzll(x);
  const uint32_t s1 = c + bf, fb = bf >> 3;
  e.head = s1 & 1u;
  e.z = s1 >> 1;
  uint64_t hi = 0, lo = 0;
  uint32_t p = 0;
#pragma unroll
  for (uint32_t i = 0; i < 8; ++i) {
    const uint32_t v = (uint32_t)(x >> (56 - 8 * i)) & 0xffu;
    if (v) {
      const uint32_t en = T1[v];
      const uint32_t R = en & 0x1fffffu, lr = (en >> 21) & 31u, t = (en >> 26) & 7u, tz = en >> 29;
      const uint64_t pat = (1ull << lr) | R;
      if (i == fb) {
        acc_put(hi, lo, pat, lr + 1);
        p += lr + 1;
      } else {
        const uint32_t s = c + t;
        acc_codeword(hi, lo, p, s & 1u, s >> 1, pat, lr + 1);
      }
      c = tz;
    } else {
      c += 8;
    }
  }
  if (eol) {  // the row's trailing zeros (pad columns excluded)
    const uint32_t s = c - (w * 64 + 64 - cols);
    acc_codeword(hi, lo, p, s & 1u, s >> 1, 1ull, 1);
  }
  e.tlen = p;
  e.len = 1 + e.z + p;
  e.lng = p > 128;
  if (!e.lng) {  // left-align the p-bit string
    const uint32_t sh = 128 - p;
    if (sh >= 64) {
      e.t0 = lo << (sh - 64);
      e.t1 = 0;
    } else if (sh) {
      e.t0 = (hi << sh) | (lo >> (64 - sh));
      e.t1 = lo << sh;
    } else {
      e.t0 = hi;
      e.t1 = lo;
    }
  }
  return e;
}

// encode_word_k1 without branches: every byte runs the same instructions (its codeword from the k = 1
// table whether or not it holds a 1, selected in or out), so a wave never executes divergent paths.
// Inside a word a run's zeros are < 64 + 7, so a byte's pattern (bin, q zeros, '1', R) is < 64 bits;
// out-of-range shift amounts of unselected bytes are clamped.
__device__ __forceinline__ LaneEnc encode_word_k1b(uint64_t x, uint32_t w, int jp, bool eol, uint32_t cols,
                                                   const uint32_t* T1) {
  LaneEnc e{};
  e.k0 = 1;
  uint32_t c = w * 64 - (uint32_t)(jp + 1);  // zeros of the open run
  if (!x) {
    if (eol) {
      const uint32_t s = cols - 1 - (uint32_t)jp;
      e.head = s & 1u;
      e.z = s >> 1;
      e.t0 = BIC_MSB;
      e.tlen = 1;
      e.len = 2 + e.z;
    }
    return e;
  }
  const uint32_t bf = (uint32_t)__builtin_clzll(x), fb = bf >> 3;
  const uint32_t s1 = c + bf;
  e.head = s1 & 1u;
  e.z = s1 >> 1;
  uint64_t hi = 0, lo = 0;
  uint32_t p = 0;
#pragma unroll
  for (uint32_t i = 0; i < 8; ++i) {
    const uint32_t v = (uint32_t)(x >> (56 - 8 * i)) & 0xffu;
    const uint32_t en = T1[v];
    const uint32_t R = en & 0x1fffffu, lr = (en >> 21) & 31u, t = (en >> 26) & 7u, tz = en >> 29;
    const uint32_t sr = c + t;
    const uint32_t q1 = min((sr >> 1) + 1u, 62u - lr);  // the '1' after q zeros, then R
    const uint64_t tail = (1ull << lr) | R;
    const bool first = i == fb;
    const uint64_t pat = first ? tail : ((uint64_t)(sr & 1u) << (q1 + lr)) | tail;
    const uint32_t nb = first ? lr + 1 : q1 + 1 + lr;  // 1..63
    const bool act = v != 0;
    const uint64_t nhi = (hi << nb) | (lo >> (64 - nb));
    const uint64_t nlo = (lo << nb) | pat;
    hi = act ? nhi : hi;
    lo = act ? nlo : lo;
    p += act ? nb : 0u;
    c = act ? tz : c + 8;
  }
  if (eol) {  // the row's trailing zeros (pad columns excluded): bin, q zeros, '1' (< 64 bits)
    const uint32_t sr = c - (w * 64 + 64 - cols), q1 = (sr >> 1) + 1;
    const uint32_t nb = q1 + 1;
    const uint64_t pat = ((uint64_t)(sr & 1u) << q1) | 1ull;
    hi = (hi << nb) | (lo >> (64 - nb));
    lo = (lo << nb) | pat;
    p += nb;
  }
  e.tlen = p;
  e.len = 1 + e.z + p;
  e.lng = p > 128;
  if (!e.lng) {  // left-align the p-bit string
    const uint32_t sh = 128 - p;
    if (sh >= 64) {
      e.t0 = lo << (sh - 64);
      e.t1 = 0;
    } else if (sh) {
      e.t0 = (hi << sh) | (lo >> (64 - sh));
      e.t1 = lo << sh;
    } else {
      e.t0 = hi;
      e.t1 = lo;
    }
  }
  return e;
}

__device__ __forceinline__ void place128_64(uint64_t* img, uint32_t off, uint64_t A, uint64_t B, uint32_t tlen) {
  if (!tlen) return;
  const uint32_t i = off >> 6, sh = off & 63;
  uint64_t D0 = A, D1 = B, D2 = 0;
  if (sh) {
    D0 = A >> sh;
    D1 = (A << (64 - sh)) | (B >> sh);
    D2 = B << (64 - sh);
  }
  const uint32_t nw = (sh + tlen + 63) >> 6;
  lds_or64(img, i, D0);
  if (nw > 1) lds_or64(img, i + 1, D1);
  if (nw > 2) lds_or64(img, i + 2, D2);
}
struct LdsSink64 {
  uint64_t* buf;
  uint32_t idx;
  uint64_t cur;
  __device__ __forceinline__ void flush() {
    if (cur) atomicOr(reinterpret_cast<unsigned long long*>(buf + idx), (unsigned long long)cur);
    cur = 0;
  }
  __device__ __forceinline__ void orw(uint32_t i, uint64_t v) {
    if (i != idx) {
      flush();
      idx = i;
    }
    cur |= v;
  }
  __device__ __forceinline__ void put(uint32_t off, uint32_t v, uint32_t nb) {  // nb <= 32
    const uint32_t i = off >> 6, sh = off & 63;
    if (sh + nb <= 64) {
      orw(i, (uint64_t)v << (64 - sh - nb));
    } else {
      orw(i, (uint64_t)v >> (sh + nb - 64));
      orw(i + 1, (uint64_t)v << (128 - sh - nb));
    }
  }
  __device__ __forceinline__ void bit(uint32_t off) { orw(off >> 6, BIC_MSB >> (off & 63)); }
};

// emit_word for k = 1 rows (the lng fallback of encode_word_k1).
template <typename Sink, typename Off>
__device__ __forceinline__ void emit_word_k1(Sink& sk, Off off, uint64_t x, uint32_t w, int jp, bool eol, uint32_t cols) {
  for (;;) {
    int j;
    uint32_t s;
    if (x) {
      const int cz = __builtin_clzll(x);
      x ^= BIC_MSB >> cz;
      j = (int)(w * 64) + cz;
      s = (uint32_t)(j - jp - 1);
    } else if (eol) {
      j = (int)cols;
      s = cols - 1 - (uint32_t)jp;
      eol = false;
    } else {
      break;
    }
    if (s & 1u) sk.put(off, 1u, 1);
    sk.bit(off + 1 + (s >> 1));
    off += 2 + (s >> 1);
    jp = j;
  }
}

// Emit one word's codewords through a sink at bit offset `off` (fallback paths).
template <typename Sink, typename Off>
__device__ __forceinline__ void emit_word(Sink& sk, Off off, uint64_t x, uint32_t w, uint32_t n, int jp,
                                          uint32_t arow, bool eol, uint32_t cols) {
  for (;;) {
    int j;
    uint32_t s;
    if (x) {
      const int cz = __builtin_clzll(x);
      x ^= BIC_MSB >> cz;
      j = (int)(w * 64) + cz;
      s = (uint32_t)(j - jp - 1);
    } else if (eol) {
      j = (int)cols;
      s = cols - 1 - (uint32_t)jp;
      eol = false;
    } else {
      break;
    }
    const uint32_t k = golomb_k_state(n, arow + (uint32_t)(jp + 1) - n);
    if (k) {
      const uint32_t bin = s & ((1u << k) - 1u);
      if (bin) sk.put(off, bin, k);
    }
    sk.bit(off + k + (s >> k));
    off += k + (s >> k) + 1;
    ++n;
    jp = j;
  }
}

__device__ __forceinline__ void lds_or(uint32_t* img, uint32_t i, uint32_t v) {
  if (v) atomicOr(&img[i], v);
}

// OR tlen (<= 128) bits (A:B, MSB-first) into the image at bit `off`.
__device__ __forceinline__ void place128(uint32_t* img, uint32_t off, uint64_t A, uint64_t B, uint32_t tlen) {
  if (!tlen) return;
  const uint32_t i = off >> 5, sh = off & 31;
  uint64_t D0 = A, D1 = B, D2 = 0;
  if (sh) {
    D0 = A >> sh;
    D1 = (A << (64 - sh)) | (B >> sh);
    D2 = B << (64 - sh);
  }
  const uint32_t nw = (sh + tlen + 31) >> 5;
  lds_or(img, i, (uint32_t)(D0 >> 32));
  if (nw > 1) lds_or(img, i + 1, (uint32_t)D0);
  if (nw > 2) lds_or(img, i + 2, (uint32_t)(D1 >> 32));
  if (nw > 3) lds_or(img, i + 3, (uint32_t)D1);
  if (nw > 4) lds_or(img, i + 4, (uint32_t)(D2 >> 32));
}

__device__ __forceinline__ void place_small(uint32_t* img, uint32_t off, uint32_t v, uint32_t nb) {
  if (!nb || !v) return;
  const uint32_t i = off >> 5, sh = off & 31;
  if (sh + nb <= 32) {
    lds_or(img, i, v << (32 - sh - nb));
  } else {
    lds_or(img, i, v >> (sh + nb - 32));
    lds_or(img, i + 1, v << (64 - sh - nb));
  }
}

// 64 image bits starting at bit a (a may be negative: leading zeros).
__device__ __forceinline__ uint64_t raw64(const uint32_t* img, int64_t a) {
  if (a <= -64) return 0;
  const int64_t b = a < 0 ? 0 : a;
  const uint32_t i = (uint32_t)(b >> 5), sh = (uint32_t)(b & 31);
  const uint64_t hi = ((uint64_t)img[i] << 32) | img[i + 1];
  const uint64_t v = sh ? (hi << sh) | (img[i + 2] >> (32 - sh)) : hi;
  return a < 0 ? v >> (-a) : v;
}

// Same, of the image with a '0' inserted at position ins (ins < 0: no insertion).
__device__ __forceinline__ uint64_t img64(const uint32_t* img, int64_t a, int64_t ins) {
  if (ins < 0 || ins >= a + 64) return raw64(img, a);
  const uint64_t Y = raw64(img, a - 1);
  if (ins < a) return Y;
  const uint32_t q = (uint32_t)(ins - a);
  const uint64_t X = raw64(img, a);
  const uint64_t hi = q ? ~(~0ull >> q) : 0ull;
  const uint64_t lo = q == 63 ? 0ull : (~0ull >> (q + 1));
  return (X & hi) | (Y & lo);
}

// Is output word w entirely inside the row's bit range [G, G+L)?
__device__ __forceinline__ bool word_complete(uint64_t w, uint64_t G, uint64_t L) {
  return w * 64 >= G && w * 64 + 64 <= G + L;
}

// A word the row shares with a neighbouring row: into the fragment table (k_fixup combines them).
__device__ __forceinline__ void put_shared(uint64_t* out, uint64_t wi, uint64_t* frag, int which, uint64_t v) {
  (void)out;
  (void)wi;
  frag[which] = v;
}

// Write a row image of L bits to absolute bit G of out (threads tid of nt: a wave's lanes by
// default): whole words with plain stores, the
// first/last word (when shared with another row) into frag[0]/frag[1]. Output word t of the row
// holds image bits [64t - G%64, 64t - G%64 + 64): the bit shift inside the image's u32 words is
// the same for every t, so the common case (no inserted bit) is three LDS reads and a funnel
// shift per word, branch-free and independent across iterations.
__device__ __forceinline__ void write_row(const uint32_t* img, uint64_t L, uint64_t G, int64_t ins,
                                          uint64_t* out, uint64_t* frag, uint32_t tid = lane_id(), uint32_t nt = 64) {
  const uint64_t w0 = G >> 6, w1 = (G + L - 1) >> 6, nw = w1 - w0 + 1;
  if (ins >= 0) {
    for (uint64_t t = tid; t < nw; t += nt) {
      const uint64_t wb = (w0 + t) * 64;
      const uint64_t v = img64(img, (int64_t)wb - (int64_t)G, ins);
      if (word_complete(w0 + t, G, L)) out[w0 + t] = bswap64(v);
      else put_shared(out, w0 + t, frag, t == 0 ? 0 : 1, v);
    }
    return;
  }
  const uint32_t g = (uint32_t)(G & 63);
  for (uint32_t t = tid; t < (uint32_t)nw; t += nt) {
    const int32_t a = (int32_t)(64 * t) - (int32_t)g;  // first image bit of output word t
    const uint32_t b = a < 0 ? 0u : (uint32_t)a;
    const uint32_t i = b >> 5, sh = b & 31;
    const uint64_t hi = ((uint64_t)img[i] << 32) | img[i + 1];
    uint64_t v = (hi << sh) | ((uint64_t)img[i + 2] >> (32 - sh));
    if (a < 0) v >>= -a;
    if (t != 0 && t != (uint32_t)nw - 1) out[w0 + t] = bswap64(v);
    else if (word_complete(w0 + t, G, L)) out[w0 + t] = bswap64(v);
    else put_shared(out, w0 + t, frag, t == 0 ? 0 : 1, v);
  }
}

// glen[] flags of the staged encoder (set by the prefix kernels, read-only afterwards: every
// consumer masks them off, so the two emission launches never write glen)
constexpr uint64_t kK0Row = 1ull << 63;  // every codeword of the row has k = 0
constexpr uint64_t kK1Row = 1ull << 62;  // every codeword of the row has k = 1
constexpr uint64_t kKMix = 1ull << 61;   // k = 0 and k = 1 mixed, masks stored (kmix_rows)
constexpr uint64_t kKEol1 = 1ull << 60;  // (kKMix) the end-of-row codeword has k = 1
constexpr uint64_t kLenMask = kKEol1 - 1;

struct FusedArgs {
  Geom g;
  const uint64_t* planes;
  const uint64_t* lut;  // byte tables (see ByteTables): [256] u64 for k = 3, then [2][256] u32
  uint32_t* counter;   // zeroed per launch
  uint64_t* ones_rec;  // zeroed per launch
  uint64_t* bits_rec;  // zeroed per launch
  uint64_t *gboff, *glen, *gfrag, *gslow;
  uint64_t *eboff, *elen, *efrag;
  uint32_t* row_o;     // two-pass / staged encoders: ones of the plane before each row
  uint32_t* sones;     // staged encoder: per (plane, row, strip) 1-counts and k statistics
  int4* krec;
  uint32_t* kpos;
  uint32_t ns;         // strips per row
  uint32_t* walk_ids;  // staged encoder: rows k_row_walk walks (count in counter[2])
  uint32_t* rest_ids;  // staged encoder: rows the REST emit launch writes (count in counter[3])
  uint32_t* slow_n;    // number of rows k_rows_global must write (zeroed per launch)
  uint64_t* slow_ids;  // their row ids
  uint64_t* out_g;
  uint64_t slot_g;
  uint64_t* bits_g;
  uint64_t* out_e;
  uint64_t slot_e;
  uint64_t* bits_e;
  uint32_t* flags;
  // packed output (FusedScratch::off_g / off_e): per-plane totals of residual 1s (ONES scan), the
  // planes' packed start words (k_plane_bases) and EG start bits; ebase null: slot mode
  uint64_t* pones;
  uint64_t* gbase;
  uint64_t* ebase;
  uint64_t* off_g;
  uint64_t* off_e;
  uint64_t* index;  // FusedScratch::index
  // bic_encode_gray without planes (FusedScratch::eg_src): the count pass wrote the EG stream in its
  // uniform layout and the residual rows are read back from it (null: residual from planes)
  const uint64_t* esrc;
  uint64_t* efix;
  uint64_t* cls;  // FusedScratch::cls (EG source: the class emission kernels' row lists, (id, offset)
                  // pairs; the class kernels store as unsigned long long, a type apart, so the compiler
                  // keeps these loads on the scalar cache: no wait on the vector memory counter)
  uint64_t* sink;     // FusedScratch::sink
  uint32_t* walk_o;   // FusedScratch::walk_o (the walked rows' row_o)
  uint32_t rgrid;     // k_emit_k01: its leading workgroups in the rest role (0: k_emit_rest writes those rows)
  // class kernels' path: per walked row (walk list index < kcap) the k = 1 masks of its words (kmix_rows),
  // and per kKMix row its walk list index
  uint64_t* kmask;
  uint32_t* row_wi;
  uint32_t kcap;
#ifdef BIC_STAMPS
  int known;
#endif
};

// A row's absolute Golomb bit offset: gboff holds it relative to the plane's slot start (LEN scan);
// packed output moves the plane to its packed start word gbase[plane]
__device__ __forceinline__ uint64_t gb_abs(const FusedArgs& a, uint64_t id, uint32_t plane) {
  const uint64_t G = a.gboff[id];
  return a.off_g ? G - (uint64_t)plane * a.slot_g * 64 + a.gbase[plane] * 64 : G;
}

// ---- residual rows read back from the EG stream (FusedArgs::esrc) ------------------------------
// bic_encode_gray without planes: the count pass (k_gray_strips, EGS) writes each plane's EG stream
// (eg.cpp:20-37 with the block size fixed at 1: per row ~R, then the end-of-row '1') in its uniform
// layout -- bit 0 a '1', row r at bit r (cols + 1) + 1 -- instead of storing R: that layout is the
// stream itself but for ONE bit, cleared after the emission (eg_fix_bit). Every reader of R takes
// the row from there: ~(64 stream bits at the row's offset + 64 w), a wave-uniform funnel shift.
__device__ __forceinline__ uint64_t eg_src_bit0(const Geom& g, uint32_t row) {
  return (uint64_t)row * (g.cols + 1) + 1;
}
// residual word w of a row (any lane pattern; two loads, the second one usually a cache hit)
__device__ __forceinline__ uint64_t eg_src_word(const uint64_t* eplane, const Geom& g, uint32_t row, uint32_t w) {
  if (w >= g.used) return 0;
  const uint64_t b = eg_src_bit0(g, row) + (uint64_t)w * 64;
  const uint64_t* p = eplane + (b >> 6);
  const uint32_t sh = (uint32_t)(b & 63);
  const uint64_t hi = bswap64(p[0]);
  const uint64_t x = sh ? funnel64(hi, bswap64(p[1]), 64 - sh) : hi;
  return ~x & (w == g.used - 1 ? g.trail : ~0ull);
}
// the row's words t * 64 + lane (t < WPL) as resid_row gives them: one load per word, lane l + 1's word
// through DPP (wave_shl:1), lane 63's from lane 0 of the next word group (the last: one uniform load)
// (as two halves, so that a wave can issue a row's loads one row ahead: eg_src_load, then
// eg_src_assemble when the words are needed)
template <int WPL>
__device__ __forceinline__ void eg_src_load(const uint64_t* eplane, const Geom& g, uint32_t row, uint64_t (&v)[WPL],
                                            uint64_t& last) {
  const int lane = lane_id();
  const uint64_t b = eg_src_bit0(g, row);
  const uint64_t* p = eplane + (b >> 6);
  const uint32_t nw = g.used;  // stream words used: nw (+ 1 when the row is not word-aligned)
#pragma unroll
  for (int t = 0; t < WPL; ++t) {  // (every lane loads, at a clamped index: eg_src_assemble masks)
    const uint32_t j = t * 64 + lane;
    v[t] = p[j < nw ? j : nw - 1];
  }
  last = p[(b & 63) ? nw : nw - 1];  // (uniform address; unused when the row is word-aligned)
}
template <int WPL>
__device__ __forceinline__ void eg_src_assemble(const Geom& g, uint32_t row, const uint64_t (&v)[WPL], uint64_t last,
                                                uint64_t (&r)[WPL]) {
  const int lane = lane_id();
  const uint32_t sh = (uint32_t)(eg_src_bit0(g, row) & 63);
  const uint32_t nw = g.used;
#pragma unroll
  for (int t = 0; t < WPL; ++t) {
    const uint32_t j = t * 64 + lane;
    const uint64_t hi = bswap64(v[t]);
    uint64_t nx = ((uint64_t)(uint32_t)__builtin_amdgcn_update_dpp(0, (int)(uint32_t)(v[t] >> 32), 0x130, 0xf, 0xf, true) << 32) |
                  (uint32_t)__builtin_amdgcn_update_dpp(0, (int)(uint32_t)v[t], 0x130, 0xf, 0xf, true);
    if (lane == 63) {
      if (t + 1 < WPL && (t + 1) * 64 < (int)nw)
        nx = ((uint64_t)(uint32_t)__builtin_amdgcn_readlane((int)(uint32_t)(v[t + 1 < WPL ? t + 1 : t] >> 32), 0) << 32) |
             (uint32_t)__builtin_amdgcn_readlane((int)(uint32_t)v[t + 1 < WPL ? t + 1 : t], 0);
      else
        nx = last;
    }
    // (lane j + 1's word is its clamped load when j + 1 >= nw: only its bits past the row are used)
    const uint64_t x = sh ? funnel64(hi, bswap64(nx), 64 - sh) : hi;
    r[t] = j < nw ? ~x & (j == nw - 1 ? g.trail : ~0ull) : 0;
  }
}
// the row's words t * 64 + lane (t < WPL) as resid_row gives them: one load per word, lane l + 1's word
// through DPP (wave_shl:1), lane 63's from lane 0 of the next word group (the last: one uniform load)
template <int WPL>
__device__ __forceinline__ void eg_src_row(const uint64_t* eplane, const Geom& g, uint32_t row, uint64_t (&r)[WPL]) {
  uint64_t v[WPL], last;
  eg_src_load<WPL>(eplane, g, row, v, last);
  eg_src_assemble<WPL>(g, row, v, last, r);
}

// The row's words with lane l holding words l WPL .. l WPL + WPL - 1 (consecutive: one prefix per
// lane over its own words, one wave scan per row instead of one per word group): WPL + 1 loads
// per lane, the last one lane l + 1's first (clamped: masked in the assembly)
template <int WPL>
__device__ __forceinline__ void eg_src_load_lc(const uint64_t* eplane, const Geom& g, uint32_t row,
                                               uint64_t (&v)[WPL + 1]) {
  const uint64_t b = eg_src_bit0(g, row);
  const uint64_t* p = eplane + (b >> 6);
  const uint32_t jmax = (b & 63) ? g.used : g.used - 1;
#pragma unroll
  for (int t = 0; t <= WPL; ++t) {
    const uint32_t j = (uint32_t)lane_id() * WPL + t;
    v[t] = p[j < jmax ? j : jmax];
  }
}
template <int WPL>
__device__ __forceinline__ void eg_src_assemble_lc(const Geom& g, uint32_t row, const uint64_t (&v)[WPL + 1],
                                                   uint64_t (&r)[WPL]) {
  const uint32_t sh = (uint32_t)(eg_src_bit0(g, row) & 63);
#pragma unroll
  for (int t = 0; t < WPL; ++t) {
    const uint32_t w = (uint32_t)lane_id() * WPL + t;
    const uint64_t hi = bswap64(v[t]);
    const uint64_t x = sh ? funnel64(hi, bswap64(v[t + 1]), 64 - sh) : hi;
    r[t] = w < g.used ? ~x & (w == g.used - 1 ? g.trail : ~0ull) : 0;
  }
}

// Global-memory emission for a row whose Golomb image does not fit the LDS window: codeword
// bits landing in the row's first/last output word are kept for the fragment table, the rest
// is OR'd into words this wave zeroed first.
struct FragSink {
  unsigned long long* out;
  uint64_t wh, wt;
  bool hpart, tpart;
  uint64_t acc_h, acc_t;
  uint64_t idx, cur;
  __device__ __forceinline__ void flush() {
    if (!cur) return;
    if (idx == wh && hpart) acc_h |= cur;
    else if (idx == wt && tpart) acc_t |= cur;
    else atomicOr(&out[idx], (unsigned long long)bswap64(cur));
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

// The residual word w of the row, read back from the EG image (~R, pad-masked): the image is
// written for every row, so the Golomb steps need no registers for the row.
__device__ __forceinline__ uint64_t img_resid(const uint32_t* eimg, const Geom& g, uint32_t w) {
  if (w >= g.used) return 0;
  const uint64_t v = ((uint64_t)eimg[2 * w] << 32) | eimg[2 * w + 1];
  return ~v & (w == g.used - 1 ? g.trail : ~0ull);
}

// Rows whose Golomb output exceeds the LDS window (a long dense stretch at large k): the main
// kernel records their offset and sample base and appends them to a list; k_rows_global (a small
// grid walking that list, one wave per row) recomputes each and writes it straight to global
// memory -- its inner words are zeroed and OR'd, the bits landing in its first/last (shared) word
// go to the fragment table.
// (row_global_at: the row's absolute offset G, length L and slow = its samples before + 1 given)
template <bool PREDICT>
__device__ __forceinline__ void row_global_at(const FusedArgs& a, uint64_t id, uint32_t plane, uint32_t row,
                                              uint64_t G, uint64_t L, uint64_t slow, int lane) {
  const Geom& g = a.g;
  uint64_t* frag = a.gfrag + 2 * id;
  const uint64_t wh = G >> 6, wt = (G + L - 1) >> 6;
  const bool hpart = !word_complete(wh, G, L);
  const bool tpart = !word_complete(wt, G, L);
  for (uint64_t i = wh + lane; i <= wt; i += 64)
    if (!((i == wh && hpart) || (i == wt && tpart))) a.out_g[i] = 0;
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  FragSink fs{reinterpret_cast<unsigned long long*>(a.out_g), wh, wt, hpart, tpart, 0, 0, 0, 0};
  StepState st{(uint32_t)(slow - 1), -1};
  const uint32_t arow = row * (g.cols + 1);
  RowCtx rc = row_ctx(a.planes, g, plane, row, 0);
  uint64_t carry = G;
  for (uint32_t w0 = 0; w0 < g.used; w0 += 64) {
    const uint32_t w = w0 + lane;
    const uint64_t x = (!PREDICT && a.esrc) ? eg_src_word(a.esrc + (uint64_t)plane * a.slot_e, g, row, w)
                                            : resid_word<PREDICT>(rc, g, row, w);
    uint32_t n;
    int jp;
    step_prefix(x, w, st, n, jp);
    const bool eol = w == g.used - 1;
    const LaneEnc e = encode_word<false>(x, w, n, jp, arow, eol, g.cols,
                                         ByteTables{reinterpret_cast<const uint32_t*>(a.lut + 256), a.lut});
    const uint32_t inc = wave_incl_sum_u32(e.len);
    const uint64_t off = carry + inc - e.len;
    carry += lane63_u32(inc);
    emit_word(fs, off, x, w, n, jp, arow, eol, g.cols);
  }
  fs.flush();
  uint64_t h = fs.acc_h, tl = fs.acc_t;
#pragma unroll
  for (int d = 32; d >= 1; d >>= 1) {
    h |= shfl_u64(h, lane ^ d);
    tl |= shfl_u64(tl, lane ^ d);
  }
  if (lane == 0) {
    if (hpart) put_shared(a.out_g, wh, frag, 0, h | (wh == wt ? tl : 0));
    if (tpart && wt != wh) put_shared(a.out_g, wt, frag, 1, tl);
  }
}
template <bool PREDICT>
__device__ __forceinline__ void row_global(const FusedArgs& a, uint64_t id, int lane) {
  const Geom& g = a.g;
  const uint32_t plane = (uint32_t)(id / g.rows), row = (uint32_t)(id % g.rows);
  row_global_at<PREDICT>(a, id, plane, row, gb_abs(a, id, plane), a.glen[id] & kLenMask, a.gslow[id], lane);
}

// EG source: after every reader of the residual rows, the one bit per plane in which the uniform
// layout differs from the EG stream (eg_src_junctions' ONES scan found it: the first 1's bit, or the
// layout's bit past the end of a plane without 1s) is cleared. The readers are the Golomb emission
// (k_emit_k01 / k_emit_known, k_emit_rest) and the slow rows (k_rows_global, or k_emit_rest's own
// loop on the class kernels' path), so with the Golomb stream requested the clear is k_fixup's (block
// 0, launched after both); without it nothing reads the rows and k_rows_global's one block does it.
__device__ __forceinline__ void eg_fix_bit(const uint64_t* efix, uint64_t* out_e, uint64_t slot_e, uint32_t nplanes) {
  if (!efix || blockIdx.x != 0 || threadIdx.x >= nplanes) return;
  const uint64_t P = efix[threadIdx.x];
  uint64_t* w = out_e + (uint64_t)threadIdx.x * slot_e + (P >> 6);
  *w &= ~bswap64(BIC_MSB >> (P & 63));
}

template <bool PREDICT>
__global__ __launch_bounds__(256) void k_rows_global(FusedArgs a) {
  const int lane = lane_id();
  if (!a.out_g) eg_fix_bit(a.esrc ? a.efix : nullptr, a.out_e, a.slot_e, a.g.nplanes);
  const uint32_t nslow = *a.slow_n;
  for (uint32_t li = blockIdx.x * 4 + wave_id(); li < nslow; li += gridDim.x * 4)
    row_global<PREDICT>(a, a.slow_ids[li], lane);
}

// One workgroup = one TILE of kTileRows consecutive rows of one plane (one wave per row). Tiles
// are claimed in order through one atomic ticket counter with the planes interleaved (tile t ->
// plane t % nplanes), so the planes' look-back chains advance side by side and any idle CU takes
// the oldest pending tile of any plane; one look-back per tile (by wave 0) serves its rows, which
// combine their counts through LDS. (Per-plane counters bound to blockIdx were measured slower:
// 793-918 us vs 682 us for C3, the claims themselves are not the limit.)
template <int WPL, bool PREDICT, bool DO_G, bool DO_E>
__global__ __launch_bounds__(64 * kTileRows, 8) void k_encode_rows(FusedArgs a) {
  __shared__ __attribute__((aligned(16))) uint32_t lds[kTileRows * (kGImg + kEImg)];
  __shared__ uint64_t sh_cnt[kTileRows], sh_len[kTileRows], sh_pre[2];
  __shared__ uint32_t sh_tile;
  __shared__ uint32_t s_lut[512];  // k = 1, 2 byte tables
  const Geom& g = a.g;
  // (the wave index left divergent here: as a scalar the compiler re-schedules this kernel's row loop
  // and C2 measured 0.032 -> 0.033-0.035 ms)
  const int lane = lane_id(), wave = threadIdx.x >> 6;
  uint32_t* gimg = lds + wave * (kGImg + kEImg);
  uint32_t* eimg = gimg + kGImg;
  const uint32_t tpp = (g.rows + kTileRows - 1) / kTileRows;  // tiles per plane
  if (threadIdx.x == 0) sh_tile = atomicAdd(a.counter, 1u);
  if (threadIdx.x < 512) s_lut[threadIdx.x] = reinterpret_cast<const uint32_t*>(a.lut + 256)[threadIdx.x];
  __syncthreads();
  const uint64_t tile = sh_tile;
  if (tile >= (uint64_t)tpp * g.nplanes) return;  // uniform over the workgroup
  const uint32_t plane = (uint32_t)(tile % g.nplanes), trow = (uint32_t)(tile / g.nplanes);
  const uint64_t rbase = (uint64_t)plane * tpp;  // this plane's first tile record
  const uint64_t rid = rbase + trow;             // this tile's record
  const uint32_t row = trow * kTileRows + wave;
  const bool valid = row < g.rows;
  const uint64_t id = (uint64_t)plane * g.rows + row;  // per-row output records
  STAMP(0);

  // ---- residual row -> EG image (~R, pad-masked, EOL '1'); 1-count; first 1 ----------------
  uint32_t ones = 0;
  int fcol = INT_MAX;
  if (valid) {
    if constexpr (DO_G) lds_image_zero32(gimg, kGImg / 4);  // the Golomb image (row loads in flight)
    uint64_t rr[WPL];
    resid_row<WPL, PREDICT>(a.planes, g, plane, row, rr);
#pragma unroll
    for (int t = 0; t < WPL; ++t) {
      const uint32_t w = t * 64 + lane;
      const uint64_t r = rr[t];
      ones += (uint32_t)__popcll(r);
      if (r && fcol == INT_MAX) fcol = (int)(w * 64 + __builtin_clzll(r));
      if (w < g.used) {
        const uint64_t v = ~r & (w == g.used - 1 ? g.trail : ~0ull);
        eimg[2 * w] = (uint32_t)(v >> 32);
        eimg[2 * w + 1] = (uint32_t)v;
      }
    }
    if (lane < kPad + 1) eimg[2 * g.used + lane] = 0;
    ones = wave_sum_u32(ones);
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
    __builtin_amdgcn_wave_barrier();
    if (lane == 0) eimg[g.cols >> 5] |= 0x80000000u >> (g.cols & 31);  // EOL '1'
  }
  STAMP(1);
  if (lane == 0) sh_cnt[wave] = ones;
  __syncthreads();

  // ---- samples before this row: ones of earlier rows (+ one EOL sample per row) ----
#ifdef BIC_STAMPS
  if (a.known) {
    if (threadIdx.x == 0) sh_pre[0] = g_known[0][rid];
  } else
#endif
  if (wave == 0) {
    uint64_t tile_ones = 0;
    for (int q = 0; q < kTileRows; ++q) tile_ones += sh_cnt[q];
    uint64_t O = 0;
    if (trow == 0) {
      if (lane == 0) rec_store(&a.ones_rec[rid], kInc | tile_ones);
    } else {
      if (lane == 0) rec_store(&a.ones_rec[rid], kAgg | tile_ones);
      O = lookback(a.ones_rec, rbase, rid, a.flags);
      if (lane == 0) rec_store(&a.ones_rec[rid], kInc | (O + tile_ones));
    }
    if (lane == 0) sh_pre[0] = O;
#ifdef BIC_STAMPS
    if (lane == 0 && rid < (1u << 17)) g_known[0][rid] = O;
#endif
  }
  __syncthreads();
  STAMP(2);
  uint64_t O = sh_pre[0];
  for (int q = 0; q < wave; ++q) O += sh_cnt[q];

  // ---- Golomb length of the row (word_len: no codewords formed), published for the tile at once:
  // the tiles after this one find its bit count before its codewords exist, so the bit-offset
  // look-back does not wait on any tile's emission. Wave 0 looks back while the others emit. ----
  uint64_t L = 0;
  if constexpr (DO_G) {
    if (valid) {
      StepState st{(uint32_t)(O + row), -1};
      const uint32_t arow = row * (g.cols + 1);
      uint32_t ll = 0;
      for (uint32_t w0 = 0; w0 < g.used; w0 += 64) {
        const uint32_t w = w0 + lane;
        const uint64_t x = img_resid(eimg, g, w);
        uint32_t n;
        int jp;
        step_prefix(x, w, st, n, jp);
        uint32_t kor = 0;
        ll += word_len(x, w, n, jp, arow, w == g.used - 1, g.cols, kor);
      }
      L = wave_sum_u32(ll);
    }
    if (lane == 0) sh_len[wave] = L;
    __syncthreads();
#ifdef BIC_STAMPS
    if (a.known) {
      if (threadIdx.x == 0) sh_pre[1] = g_known[1][rid];
    } else
#endif
    if (wave == 0) {
      uint64_t tile_bits = 0;
      for (int q = 0; q < kTileRows; ++q) tile_bits += sh_len[q];
      uint64_t Gt = 0;
      if (trow == 0) {
        if (lane == 0) rec_store(&a.bits_rec[rid], kInc | tile_bits);
      } else {
        if (lane == 0) rec_store(&a.bits_rec[rid], kAgg | tile_bits);
        Gt = lookback(a.bits_rec, rbase, rid, a.flags);
        if (lane == 0) rec_store(&a.bits_rec[rid], kInc | (Gt + tile_bits));
      }
      if (lane == 0) sh_pre[1] = Gt;
#ifdef BIC_STAMPS
      if (lane == 0 && rid < (1u << 17)) g_known[1][rid] = Gt;
#endif
    }
  }

  // ---- EG as written (eg.cpp:20-37): per row ~R then '1'; a '0' after the plane's first 1 ----
  if (DO_E && valid) {
    const bool f_here = O == 0 && ones > 0;
    fcol = wave_min(fcol);
    const uint64_t Le = (uint64_t)g.cols + 1 + (f_here ? 1 : 0);
    const uint64_t Ge_rel = (uint64_t)row * (g.cols + 1) + (O > 0 ? 1 : 0);
    const uint64_t cap = a.slot_e * 64;
    const uint64_t Ge = (uint64_t)plane * cap + Ge_rel;
    __builtin_amdgcn_fence(__ATOMIC_ACQ_REL, "wavefront");
    __builtin_amdgcn_wave_barrier();
    if (Ge_rel + Le <= cap) {
      write_row(eimg, Le, Ge, f_here ? (int64_t)fcol + 1 : -1, a.out_e, a.efrag + 2 * id);
      if (lane == 0) { a.eboff[id] = Ge; a.elen[id] = Le; }
    } else if (lane == 0) {
      a.eboff[id] = Ge;
      a.elen[id] = 0;  // overflowed: nothing written, fixup skips
      atomicOr(&a.flags[0], 1u);
    }
    if (lane == 0 && row == g.rows - 1) a.bits_e[plane] = Ge_rel + Le;
  }

  STAMP(3);
  // ---- Golomb codewords into the row image (rows longer than the LDS window: row_global_at below) ----
  if constexpr (DO_G) {
    constexpr uint32_t kCapBits = (kGImg - kPad) * 32;
    const bool fits = L <= kCapBits;
#ifdef BIC_STAMPS
    uint32_t dbg_slow = 0;
#endif
    if (valid && fits) {
      StepState st{(uint32_t)(O + row), -1};
      const uint32_t arow = row * (g.cols + 1);
      uint64_t loc = 0;
      for (uint32_t w0 = 0; w0 < g.used; w0 += 64) {
        const uint32_t w = w0 + lane;
        const uint64_t x = img_resid(eimg, g, w);
        uint32_t n;
        int jp;
        step_prefix(x, w, st, n, jp);
        const bool eol = w == g.used - 1;
        const LaneEnc e = encode_word(x, w, n, jp, arow, eol, g.cols, ByteTables{s_lut, a.lut});
#ifdef BIC_STAMPS
        dbg_slow += (e.path == 3 ? 1u : 0u) + (e.lng ? 1000u : 0u) + (e.path == 1 ? 1000000u : 0u);
#endif
        const uint32_t inc = wave_incl_sum_u32(e.len);
        const uint64_t off = loc + inc - e.len;
        loc += lane63_u32(inc);
        if (!e.lng) {
          place_small(gimg, (uint32_t)off, e.head, e.k0);
          place128(gimg, (uint32_t)(off + e.k0 + e.z), e.t0, e.t1, e.tlen);
        } else {
          LdsSink ls{gimg, 0, 0};
          emit_word(ls, (uint32_t)off, x, w, n, jp, arow, eol, g.cols);
          ls.flush();
        }
      }
      if (lane == 0 && loc != L) atomicOr(&a.flags[3], 1u);  // word_len disagrees with the emission
    }
    STAMP(4);
#ifdef BIC_STAMPS
    {
      const uint32_t tot = wave_sum_u32(dbg_slow);
      if (lane == 0 && (uint64_t)id * 8 + 7 < (1u << 21)) g_stamps[(uint64_t)id * 8 + 7] = tot;
    }
#endif
    __syncthreads();
    STAMP(5);
    if (valid) {
      uint64_t Grel = sh_pre[1];
      for (int q = 0; q < wave; ++q) Grel += sh_len[q];
      const uint64_t cap = a.slot_g * 64;
      const uint64_t G = (uint64_t)plane * cap + Grel;
      if (lane == 0 && row == g.rows - 1) a.bits_g[plane] = Grel + L;
      if (Grel + L <= cap) {
        if (fits) {
          __builtin_amdgcn_fence(__ATOMIC_ACQ_REL, "wavefront");
          __builtin_amdgcn_wave_barrier();
          write_row(gimg, L, G, -1, a.out_g, a.gfrag + 2 * id);
        }
        if (lane == 0) {
          a.gboff[id] = G;
          a.glen[id] = L;
          a.gslow[id] = 0;
        }
        // a row longer than the LDS window: written here, straight to global memory (no list, no
        // k_rows_global launch)
        if (!fits) row_global_at<PREDICT>(a, id, plane, row, G, L, O + row + 1, lane);
      } else if (lane == 0) {
        a.gboff[id] = G;
        a.glen[id] = 0;
        a.gslow[id] = 0;
        atomicOr(&a.flags[0], 1u);
      }
    }
    STAMP(6);
  }
}

// ==========================================================================================
// Two-pass encoder. Pass 1 (k_len_rows) runs the look-back chains with nothing but lengths:
// per 8-row tile the ones count, the ones prefix, each row's Golomb length (byte tables, no
// codeword strings) and the bits prefix; it stores, per row, the ones before it and both
// streams' bit offsets. Pass 2 (k_emit_rows) then writes every row independently -- no
// look-back, no workgroup barrier -- streaming each row's codewords through a small LDS window
// whose complete words go straight to HBM. A row's first and last word (shared with the
// neighbouring rows) go to the fragment table, as in the single-pass kernel.
// ==========================================================================================
constexpr int kWin = 1024;                      // u32 words of one wave's output window (also holds
                                                // the EG image of a plane's first-1 row)
constexpr uint32_t kIterCap = (kWin - 8) * 32 - 128;  // bits one 64-word step may emit

template <int WPL, bool PREDICT, bool DO_G, bool DO_E>
__global__ __launch_bounds__(64 * kTileRows, 8) void k_len_rows(FusedArgs a) {
  // (sh_len apart from sh_cnt: a wave that finishes its length early must not overwrite the 1-counts
  // a slower wave is still summing for its O -- one array for both raced: a wrong O, a wrong length,
  // about 1 in 15 two-pass calls, tools/dbg_twopass.py)
  __shared__ uint64_t sh_cnt[kTileRows], sh_len[kTileRows], sh_pre[2];
  __shared__ uint32_t sh_tile;
  __shared__ uint32_t s_lut[512];
  const Geom& g = a.g;
  const int lane = lane_id(), wave = (int)wave_id();
  const uint32_t tpp = (g.rows + kTileRows - 1) / kTileRows;
  if (threadIdx.x == 0) sh_tile = atomicAdd(a.counter, 1u);
  if (DO_G && threadIdx.x < 512) s_lut[threadIdx.x] = reinterpret_cast<const uint32_t*>(a.lut + 256)[threadIdx.x];
  __syncthreads();
  const uint64_t tile = sh_tile;
  if (tile >= (uint64_t)tpp * g.nplanes) return;  // uniform over the workgroup
  const uint32_t plane = (uint32_t)(tile % g.nplanes), trow = (uint32_t)(tile / g.nplanes);
  const uint64_t rbase = (uint64_t)plane * tpp, rid = rbase + trow;
  const uint32_t row = trow * kTileRows + wave;
  const bool valid = row < g.rows;
  const uint64_t id = (uint64_t)plane * g.rows + row;

  uint64_t rr[WPL];
  uint32_t ones = 0;
  if (valid) {
    resid_row<WPL, PREDICT>(a.planes, g, plane, row, rr);
#pragma unroll
    for (int t = 0; t < WPL; ++t) ones += (uint32_t)__popcll(rr[t]);
    ones = wave_sum_u32(ones);
  }
  if (lane == 0) sh_cnt[wave] = ones;
  __syncthreads();
  if (wave == 0) {
    uint64_t tile_ones = 0;
    for (int q = 0; q < kTileRows; ++q) tile_ones += sh_cnt[q];
    uint64_t O = 0;
    if (trow == 0) {
      if (lane == 0) rec_store(&a.ones_rec[rid], kInc | tile_ones);
    } else {
      if (lane == 0) rec_store(&a.ones_rec[rid], kAgg | tile_ones);
      O = lookback(a.ones_rec, rbase, rid, a.flags);
      if (lane == 0) rec_store(&a.ones_rec[rid], kInc | (O + tile_ones));
    }
    if (lane == 0) sh_pre[0] = O;
  }
  __syncthreads();
  uint64_t O = sh_pre[0];
  for (int q = 0; q < wave; ++q) O += sh_cnt[q];

  if (DO_E && valid && lane == 0) {  // EG as written: ~R then '1' per row; a '0' after the plane's first 1
    const uint64_t Le = (uint64_t)g.cols + 1 + ((O == 0 && ones > 0) ? 1 : 0);
    const uint64_t Ge_rel = (uint64_t)row * (g.cols + 1) + (O > 0 ? 1 : 0);
    const uint64_t cap = a.slot_e * 64;
    a.eboff[id] = (uint64_t)plane * cap + Ge_rel;
    if (Ge_rel + Le <= cap) {
      a.elen[id] = Le;
    } else {
      a.elen[id] = 0;
      atomicOr(&a.flags[0], 1u);
    }
    if (row == g.rows - 1) a.bits_e[plane] = Ge_rel + Le;
  }
  if (valid && lane == 0) a.row_o[id] = (uint32_t)O;

  if constexpr (DO_G) {
    uint64_t L = 0;
    uint32_t step_max = 0;
    if (valid) {
      StepState st{(uint32_t)(O + row), -1};
      const uint32_t arow = row * (g.cols + 1);
#pragma unroll
      for (int t = 0; t < WPL; ++t) {
        const uint32_t w = t * 64 + lane;
        if (t * 64 >= (int)g.used) break;
        uint32_t n;
        int jp;
        step_prefix(rr[t], w, st, n, jp);
        uint32_t kor = 0;
        const uint32_t tot = wave_sum_u32(word_len(rr[t], w, n, jp, arow, w == g.used - 1, g.cols, kor));
        L += tot;
        step_max = max(step_max, tot);
      }
    }
    if (lane == 0) sh_len[wave] = L;
    __syncthreads();
    if (wave == 0) {
      uint64_t tile_bits = 0;
      for (int q = 0; q < kTileRows; ++q) tile_bits += sh_len[q];
      uint64_t Gt = 0;
      if (trow == 0) {
        if (lane == 0) rec_store(&a.bits_rec[rid], kInc | tile_bits);
      } else {
        if (lane == 0) rec_store(&a.bits_rec[rid], kAgg | tile_bits);
        Gt = lookback(a.bits_rec, rbase, rid, a.flags);
        if (lane == 0) rec_store(&a.bits_rec[rid], kInc | (Gt + tile_bits));
      }
      if (lane == 0) sh_pre[1] = Gt;
    }
    __syncthreads();
    if (valid && lane == 0) {
      uint64_t Grel = sh_pre[1];
      for (int q = 0; q < wave; ++q) Grel += sh_len[q];
      const uint64_t cap = a.slot_g * 64;
      a.gboff[id] = (uint64_t)plane * cap + Grel;
      if (row == g.rows - 1) a.bits_g[plane] = Grel + L;
      if (Grel + L <= cap) {
        a.glen[id] = L;
        a.gslow[id] = step_max > kIterCap ? O + row + 1 : 0;  // k_rows_global writes such rows
        if (step_max > kIterCap) a.slow_ids[atomicAdd(a.slow_n, 1u)] = id;
      } else {
        a.glen[id] = 0;
        a.gslow[id] = 0;
        atomicOr(&a.flags[0], 1u);
      }
    }
  }
}

// EG row from registers: row bit b (b < cols) is ~R, bit cols is the end-of-row '1'; output word
// j of the row holds row bits [64j - g, 64j - g + 64) with g = Ge % 64. Lane l forms words
// j = 64t + l from its own row word and its left neighbour's (one shuffle per step).
// INV = false: the row bits are R itself (a Golomb row whose codewords all have k = 0).
template <int WPL, bool INV = true>
__device__ __forceinline__ void eg_row_regs(const uint64_t (&rr)[WPL], const Geom& g, uint64_t Ge, uint64_t Le,
                                            uint64_t* out, uint64_t* frag) {
  const int lane = lane_id();
  const uint32_t sh = (uint32_t)(Ge & 63);
  const uint64_t w0 = Ge >> 6, nw = ((Ge + Le - 1) >> 6) - w0 + 1;
  const uint32_t eolw = g.cols >> 6;
  const uint64_t eolbit = BIC_MSB >> (g.cols & 63);
  const bool head_whole = sh == 0, tail_whole = ((Ge + Le) & 63) == 0;  // (only the first / last word can be shared)
  uint64_t carry = 0;
#pragma unroll
  for (int t = 0; t <= WPL; ++t) {
    const uint32_t j = t * 64 + lane;
    if (t * 64 >= (int)nw) break;
    uint64_t X = 0;
    if (t < WPL && j < g.used) X = INV ? ~rr[t] & (j == g.used - 1 ? g.trail : ~0ull) : rr[t];
    if (j == eolw) X |= eolbit;
    uint64_t Xl = shfl_up_u64(X, 1);
    if (lane == 0) Xl = carry;
    carry = lane63_u64(X);
    const uint64_t v = funnel64(Xl, X, sh);
    if (j < nw) {
      const uint64_t wi = w0 + j;
      if ((j != 0 || head_whole) && (j != nw - 1 || tail_whole)) out[wi] = bswap64(v);
      else put_shared(out, wi, frag, j == 0 ? 0 : 1, v);
    }
  }
}

template <int WPL, bool PREDICT, bool DO_G, bool DO_E>
__global__ __launch_bounds__(64 * kTileRows, 8) void k_emit_rows(FusedArgs a) {
  __shared__ __attribute__((aligned(16))) uint32_t lds[kTileRows * kWin];
  __shared__ uint32_t s_lut[512];
  const Geom& g = a.g;
  const int lane = lane_id(), wave = (int)wave_id();
  uint32_t* win = lds + wave * kWin;
  if (DO_G && threadIdx.x < 512) s_lut[threadIdx.x] = reinterpret_cast<const uint32_t*>(a.lut + 256)[threadIdx.x];
  __syncthreads();  // the only workgroup barrier
  const uint64_t id = (uint64_t)blockIdx.x * kTileRows + wave;
  if (id >= (uint64_t)g.rows * g.nplanes) return;
  const uint32_t plane = (uint32_t)(id / g.rows), row = (uint32_t)(id % g.rows);
  const bool do_g = DO_G && a.glen[id] != 0 && a.gslow[id] == 0;
  const bool do_e = DO_E && a.elen[id] != 0;
  if (!do_g && !do_e) return;
  if (do_g) lds_image_zero32(win, kWin / 4);
  uint64_t rr[WPL];
  resid_row<WPL, PREDICT>(a.planes, g, plane, row, rr);
  const uint32_t O = a.row_o[id];

  if (do_e) {
    const uint64_t Ge = a.eboff[id], Le = a.elen[id];
    if (Le == (uint64_t)g.cols + 1) {
      eg_row_regs<WPL>(rr, g, Ge, Le, a.out_e, a.efrag + 2 * id);
    } else {
      // the plane's first 1 is in this row: EG image with the inserted '0' (once per plane)
      uint32_t* eimg = win;  // reused before the Golomb window is live
      int fcol = INT_MAX;
#pragma unroll
      for (int t = 0; t < WPL; ++t) {
        const uint32_t w = t * 64 + lane;
        if (rr[t] && fcol == INT_MAX) fcol = (int)(w * 64 + __builtin_clzll(rr[t]));
        if (w < g.used) {
          const uint64_t v = ~rr[t] & (w == g.used - 1 ? g.trail : ~0ull);
          eimg[2 * w] = (uint32_t)(v >> 32);
          eimg[2 * w + 1] = (uint32_t)v;
        }
      }
      if (lane < kPad + 1) eimg[2 * g.used + lane] = 0;
      fcol = wave_min(fcol);
      __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
      __builtin_amdgcn_wave_barrier();
      if (lane == 0) eimg[g.cols >> 5] |= 0x80000000u >> (g.cols & 31);
      __builtin_amdgcn_fence(__ATOMIC_ACQ_REL, "wavefront");
      __builtin_amdgcn_wave_barrier();
      write_row(eimg, Le, Ge, (int64_t)fcol + 1, a.out_e, a.efrag + 2 * id);
      __builtin_amdgcn_fence(__ATOMIC_ACQ_REL, "wavefront");
      __builtin_amdgcn_wave_barrier();
      if (do_g) {
        lds_image_zero32(win, kWin / 4);
        __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
        __builtin_amdgcn_wave_barrier();
      }
    }
  }

  if constexpr (DO_G) {
    if (!do_g) return;
    const uint64_t G = a.gboff[id], L = a.glen[id];
    uint64_t* out = a.out_g;
    uint64_t* frag = a.gfrag + 2 * id;
    uint64_t wbase = G & ~63ull;  // absolute bit of win[0]
    const uint64_t first_word = G >> 6;
    StepState st{O + row, -1};
    const uint32_t arow = row * (g.cols + 1);
    uint64_t loc = 0;  // row bits placed so far
#pragma unroll
    for (int t = 0; t < WPL; ++t) {
      const uint32_t w = t * 64 + lane;
      if (t * 64 >= (int)g.used) break;
      const uint64_t x = rr[t];
      uint32_t n;
      int jp;
      step_prefix(x, w, st, n, jp);
      const bool eol = w == g.used - 1;
      const LaneEnc e = encode_word<true>(x, w, n, jp, arow, eol, g.cols, ByteTables{s_lut, a.lut});
      const uint32_t inc = wave_incl_sum_u32(e.len);
      const uint32_t p = (uint32_t)(G + loc - wbase) + inc - e.len;  // window bit of this lane's string
      if (!e.lng) {
        place_small(win, p, e.head, e.k0);
        place128(win, p + e.k0 + e.z, e.t0, e.t1, e.tlen);
      } else {
        LdsSink ls{win, 0, 0};
        emit_word(ls, p, x, w, n, jp, arow, eol, g.cols);
        ls.flush();
      }
      loc += lane63_u32(inc);
      __builtin_amdgcn_fence(__ATOMIC_ACQ_REL, "wavefront");
      __builtin_amdgcn_wave_barrier();
      // flush the complete 64-bit words; the row's first word, if shared, is a fragment
      const uint32_t nfull = (uint32_t)((G + loc - wbase) >> 6);
      for (uint32_t q = lane; q < nfull; q += 64) {
        const uint64_t v = ((uint64_t)win[2 * q] << 32) | win[2 * q + 1];
        const uint64_t wi = (wbase >> 6) + q;
        if (wi == first_word && (G & 63)) frag[0] = v;
        else out[wi] = bswap64(v);
      }
      if (nfull) {  // carry the partial word to the front, clear the rest
        const uint32_t c0 = win[2 * nfull], c1 = win[2 * nfull + 1];
        __builtin_amdgcn_fence(__ATOMIC_ACQ_REL, "wavefront");
        __builtin_amdgcn_wave_barrier();
        for (uint32_t q = 2 + lane; q < 2 * nfull + 2; q += 64) win[q] = 0;
        if (lane == 0) { win[0] = c0; win[1] = c1; }
        wbase += 64ull * nfull;
        __builtin_amdgcn_fence(__ATOMIC_ACQ_REL, "wavefront");
        __builtin_amdgcn_wave_barrier();
      }
    }
    // the row's last word, if it ends inside one
    if ((G + L) & 63) {
      if (lane == 0) {
        const uint64_t v = ((uint64_t)win[0] << 32) | win[1];
        if ((wbase >> 6) == first_word) frag[0] = v;
        else frag[1] = v;
      }
    }
  }
}

// ==========================================================================================
// Staged encoder (default): every inter-row dependency is resolved by a kernel boundary instead of
// a decoupled look-back, so no workgroup ever waits on another (a cross-XCD look-back hop costs
// microseconds, MI355X_MICROARCH.md barrier-counter row, and a tile waiting on one holds its
// CU's waves idle). Stages: per-row residual 1-counts (k_med_rows<ROWS>) -> per-plane scan ->
// per-row Golomb lengths (word_len) -> per-plane scan of the lengths -> k_emit_known, where each
// wave walks its rows independently (persistent waves, static row order, no barriers).
// ==========================================================================================

// Golomb length of a row from its sample base O (ones of the plane before it): rows whose k
// statistics (bic_kstat.h) prove every codeword k = 0 (length cols + 1: the residual row and its
// end-of-row '1') or k = 1 (2n + (zeros - odd runs) / 2) get their length without being read;
// returns true for the others (k_row_walk walks them).
__device__ __forceinline__ bool row_class(const FusedArgs& a, uint64_t id, uint32_t row, uint32_t O, const RowK& rk) {
  const Geom& g = a.g;
  if (row == 0) return true;  // (the plane's first sample has k = 1 from the fresh state, Golomb.h:18)
  const int64_t N0 = (int64_t)O + row, A0 = (int64_t)row * g.cols - O;
  if (A0 - N0 + rk.q0 <= 0) {
    a.glen[id] = kK0Row | (g.cols + 1);
    return false;
  }
  if (A0 - 2 * N0 + rk.qh <= 0 && A0 - N0 + rk.ql > 0) {
    const uint64_t n = rk.ones + 1, zeros = g.cols - rk.ones, odd = n - rk.chg;
    a.glen[id] = kK1Row | (2 * n + (zeros - odd) / 2);
    return false;
  }
  return true;
}

// Packed output: the planes' start words in each coder's buffer (streams word-aligned, plane order:
// bic_pack_streams' layout) from the Golomb totals (LEN scan) and the EG lengths (rows (cols + 1), + 1
// when the plane holds a residual 1: eg.cpp's first-run bit), each capped at the slot size so that an
// overflowing plane (BIC_ENOSPC) cannot push a later one past the buffer. One workgroup.
__device__ __forceinline__ void plane_bases(const FusedArgs& a, uint64_t* tmp) {
  const Geom& g = a.g;
  uint64_t cg = 0, ce = 0;  // running bases (words)
  for (uint32_t q0 = 0; q0 < g.nplanes; q0 += 1024) {
    const uint32_t q = q0 + threadIdx.x;
    const bool in = q < g.nplanes;
    uint64_t gw = 0, ew = 0;
    if (in && a.off_g) gw = min((a.bits_g[q] + 63) / 64, a.slot_g);
    if (in && a.off_e) ew = min(((uint64_t)g.rows * (g.cols + 1) + (a.pones[q] ? 1 : 0) + 63) / 64, a.slot_e);
    uint64_t tg, te;
    const uint64_t pg = block_excl_scan<uint64_t>(gw, tmp, tg) + cg;
    const uint64_t pe = block_excl_scan<uint64_t>(ew, tmp, te) + ce;
    if (in && a.off_g) {
      a.off_g[q] = pg;
      a.gbase[q] = pg;
    }
    if (in && a.off_e) {
      a.off_e[q] = pe;
      a.ebase[q] = pe * 64;
    }
    cg += tg;
    ce += te;
  }
  if (threadIdx.x == 0) {
    if (a.off_g) a.off_g[g.nplanes] = cg;
    if (a.off_e) a.off_e[g.nplanes] = ce;
  }
}
// Exclusive per-plane scan of per-row values. Each 1024-thread workgroup owns kScanChunk rows of a
// plane (kScanPer consecutive rows per thread) and sums the plane's earlier rows itself (coalesced,
// at most rows / 1024 loads per thread), so no workgroup waits on another and a plane spreads over
// rows / kScanChunk CUs. ONES: the strips' 1-counts (sones) -> row_o[], the ones before each row;
// with CLASSIFY each row is also classified (row_class) and the rows to walk are appended to
// walk_ids. Otherwise: glen[] Golomb lengths -> gboff[] absolute bit offsets in the plane's slot,
// bits_g[] the plane's total; rows past the slot's end get glen = 0 and raise the overflow flag
// (a later chunk may then sum a zeroed length: its offsets stay inside the slot, and the call
// reports BIC_ENOSPC with the stream undefined).
#ifndef BIC_LEN_REV
#define BIC_LEN_REV 0
#endif
constexpr bool kLenRev = BIC_LEN_REV != 0;
constexpr uint32_t kScanPer = 1, kScanChunk = 1024 * kScanPer;  // (1024-row chunks: twice the workgroups of 2048, C3 prefix 51 -> 42 us)
template <bool ONES, bool CLASSIFY>
__global__ __launch_bounds__(1024) void k_scan_rows(FusedArgs a) {
  __shared__ uint64_t tmp[17];
  const Geom& g = a.g;
  const uint32_t nb = (g.rows + kScanChunk - 1) / kScanChunk;
  // (BIC_LEN_REV, the LEN scan: chunks dealt bottom row chunk first, planes interleaved, so the class
  // lists -- appended in about this order -- lead with the rows the count pass wrote last, the part of
  // the EG stream the Infinity Cache may still hold when the emission reads it)
  const bool rev = kLenRev && !ONES;
  const uint32_t plane = rev ? blockIdx.x % g.nplanes : blockIdx.x / nb;
  const uint32_t b = rev ? nb - 1 - blockIdx.x / g.nplanes : blockIdx.x % nb;
  const uint64_t base = (uint64_t)plane * g.rows;
  auto val = [&](uint32_t r) -> uint64_t {
    if constexpr (ONES) {
      uint64_t o = 0;
      for (uint32_t q = 0; q < a.ns; ++q) o += a.sones[(base + r) * a.ns + q];
      return o;
    } else {
      return a.glen[base + r] & kLenMask;
    }
  };
  SSTAMP(0);
  const uint32_t r0 = b * kScanChunk + threadIdx.x * kScanPer;
  uint64_t v[kScanPer], sum = 0;
#pragma unroll
  for (uint32_t i = 0; i < kScanPer; ++i) {
    v[i] = r0 + i < g.rows ? val(r0 + i) : 0;
    sum += v[i];
  }
  // (ONES + CLASSIFY: the rows' k statistics loaded now, their latency under the scans below)
  RowKRaw rks[kScanPer];
  if constexpr (ONES && CLASSIFY) {
#pragma unroll
    for (uint32_t i = 0; i < kScanPer; ++i) {
      const uint64_t id = base + (r0 + i < g.rows ? r0 + i : 0);
      rks[i] = row_kstats_load(a.krec + id * a.ns, a.kpos + id * a.ns, a.ns);
    }
  }
  SSTAMP(1);
  uint64_t before = 0;  // this thread's share of the plane's rows before the chunk
  const uint32_t lim = b * kScanChunk;
  if constexpr (ONES) {  // the records of those rows are one contiguous range
    const uint32_t* so = a.sones + base * a.ns;
    const uint64_t flat = (uint64_t)lim * a.ns;  // a multiple of 4 (lim is one of kScanChunk)
    if ((base * a.ns) % 4 == 0) {  // 16-byte loads
      const uint4* s4 = reinterpret_cast<const uint4*>(so);
#pragma unroll 8
      for (uint64_t i = threadIdx.x; i < flat / 4; i += 1024) {
        const uint4 q = s4[i];
        before += (uint64_t)q.x + q.y + q.z + q.w;
      }
    } else {
#pragma unroll 8
      for (uint64_t i = threadIdx.x; i < flat; i += 1024) before += so[i];
    }
  } else {
#pragma unroll 8
    for (uint32_t r = threadIdx.x; r < lim; r += 1024) before += val(r);
  }
  SSTAMP(2);
  uint64_t tot, btot;
  uint64_t pre = block_excl_scan<uint64_t>(sum, tmp, tot);
  (void)block_excl_scan<uint64_t>(before, tmp, btot);
  pre += btot;
  SSTAMP(3);
  if constexpr (ONES) {
    bool walks[kScanPer];  // classify every row of the thread first: their record loads overlap
    uint64_t p = pre;
#pragma unroll
    for (uint32_t i = 0; i < kScanPer; ++i) {
      const uint32_t r = r0 + i;
      if constexpr (CLASSIFY) walks[i] = r < g.rows && row_class(a, base + r, r, (uint32_t)p, row_kstats_combine(rks[i], g.cols));
      else walks[i] = false;
      p += v[i];
    }
#pragma unroll
    for (uint32_t i = 0; i < kScanPer; ++i) {
      const uint32_t r = r0 + i;
      const bool in = r < g.rows;
      if (in) a.row_o[base + r] = (uint32_t)pre;
      const bool walk = walks[i];
      if constexpr (CLASSIFY) {
        const uint64_t m = __ballot(walk);  // wave-aggregated append to the list of rows to walk
        if (m) {
          uint32_t wb = 0;
          const int leader = __builtin_ctzll(m);
          if (lane_id() == leader) wb = atomicAdd(a.counter + 2, (uint32_t)__popcll(m));
          wb = (uint32_t)__shfl((int)wb, leader);
          if (walk) {
            const uint32_t wi = wb + (uint32_t)__popcll(m & ((1ull << lane_id()) - 1ull));
            a.walk_ids[wi] = (uint32_t)(base + r);
            a.walk_o[wi] = (uint32_t)pre;
          }
        }
      }
      const bool first1 = in && pre == 0 && v[i] > 0;  // the row holding the plane's first 1
      if (a.esrc) {
        // EG source: the stream bit eg.cpp's first-run '0' makes differ from the uniform layout: the
        // first 1's own bit (the layout has a '1' there, the shifted ~R of the pixel before it)
        if (first1) {
          const uint32_t* so = a.sones + (base + r) * a.ns;
          const uint32_t* kp = a.kpos + (base + r) * a.ns;
          uint32_t j1 = 0;
          for (uint32_t q = 0; q < a.ns; ++q)
            if (so[q]) {
              j1 = kp[q] & 0xffffu;
              break;
            }
          a.efix[plane] = (uint64_t)r * (g.cols + 1) + j1;
        }
      } else if (first1 && !walk && a.out_e) {
        // (EG inserts a '0' after it): listed for REST here unless walked (k_row_walk's list)
        a.rest_ids[atomicAdd(a.counter + 3, 1u)] = (uint32_t)(base + r);
      }
      pre += v[i];
    }
    if (b == nb - 1 && threadIdx.x == 0) {
      const uint64_t po = btot + tot;
      a.pones[plane] = po;  // the plane's residual 1s
      if (a.esrc) {  // the EG length (eg.cpp: rows (cols + 1), + 1 for the first run's g = 1 bit)
        a.bits_e[plane] = (uint64_t)g.rows * (g.cols + 1) + (po ? 1 : 0);
        if (!po) a.efix[plane] = (uint64_t)g.rows * (g.cols + 1);  // no 1: the layout's last bit is past the end
      }
    }
  } else {
    const uint64_t cap = a.slot_g * 64;
    if (a.cls) {  // EG source: this chunk's k = 0 / k = 1 rows appended to the class lists
      static_assert(kScanPer == 1, "one row per thread");
      const uint32_t r = r0;
      const uint64_t f = r < g.rows ? a.glen[base + r] : 0;
      const bool ok = pre + v[0] <= cap && v[0] != 0;  // (an overflowing row is written by nobody)
      // a k = 1 or mixed row too long for an LDS row image is written by k_emit_rest's slow-row loop
      // (row_global; k = 0 rows are shifted copies, no image): the list is complete before the emission
      constexpr uint32_t kCapBitsRest = (kGImg - kPad) * 32;
      const bool big = v[0] > kCapBitsRest;
      const uint32_t c0 = ok && (f & kK0Row) ? 1u : 0u, c1 = ok && (f & kK1Row) && (!big || !kSlowRest) ? 1u : 0u;
      if (ok && !(f & kK0Row) && big && (kSlowRest || !(f & kK1Row))) {
        a.gslow[base + r] = a.row_o[base + r] + r + 1;
        a.slow_ids[atomicAdd(a.slow_n, 1u)] = base + r;
      }
      // the mixed rows that fit an LDS image: those with the walk's k = 1 masks (kKMix) listed for kmix_rows
      // (the class entries' third list, counter[8]), the others (a codeword with k >= 2) for k_emit_k01's
      // rest role (rest_ids, counter[6]). ~1 % of the rows: most waves append nothing.
      const bool cx = kK01Rest && ok && (f & kKMix) && !big;
      const bool cm = kK01Rest && ok && !(f & (kK0Row | kK1Row | kKMix)) && !big;
      const uint64_t mx = __ballot(cx), mm = __ballot(cm);
      if (mx) {
        const int leader = __builtin_ctzll(mx);
        uint32_t wb = 0;
        if (lane_id() == leader) wb = atomicAdd(a.counter + 8, (uint32_t)__popcll(mx));
        wb = (uint32_t)__shfl((int)wb, leader);
        if (cx) {
          const uint64_t e = 2 * (uint64_t)g.rows * g.nplanes + wb + (uint32_t)__popcll(mx & ((1ull << lane_id()) - 1ull));
          a.cls[2 * e] = (base + r) | ((v[0] & kLenMask) << 32);
          a.cls[2 * e + 1] = (uint64_t)plane * cap + pre;
        }
      }
      if (mm) {
        const int leader = __builtin_ctzll(mm);
        uint32_t wb = 0;
        if (lane_id() == leader) wb = atomicAdd(a.counter + 6, (uint32_t)__popcll(mm));
        wb = (uint32_t)__shfl((int)wb, leader);
        if (cm) a.rest_ids[wb + (uint32_t)__popcll(mm & ((1ull << lane_id()) - 1ull))] = (uint32_t)(base + r);
      }
      uint32_t t0, t1;
      const uint32_t x0 = block_excl_scan<uint32_t>(c0, reinterpret_cast<uint32_t*>(tmp), t0);
      const uint32_t x1 = block_excl_scan<uint32_t>(c1, reinterpret_cast<uint32_t*>(tmp), t1);
      __shared__ uint32_t lb[2];
      if (threadIdx.x == 0) {
        lb[0] = t0 ? atomicAdd(a.counter + 4, t0) : 0u;
        lb[1] = t1 ? atomicAdd(a.counter + 5, t1) : 0u;
      }
      __syncthreads();
      const uint64_t nrows = (uint64_t)g.rows * g.nplanes;
      const uint64_t G = (uint64_t)plane * cap + pre;  // (gboff's value, written below)
      if (c0) {
        a.cls[2 * (lb[0] + x0)] = (base + r) | ((uint64_t)plane << 32);  // id, plane (the length is cols + 1)
        a.cls[2 * (lb[0] + x0) + 1] = G;
      }
      if (c1) {
        a.cls[2 * (nrows + lb[1] + x1)] = (base + r) | (v[0] << 32);
        a.cls[2 * (nrows + lb[1] + x1) + 1] = G;
      }
    }
#pragma unroll
    for (uint32_t i = 0; i < kScanPer; ++i) {
      const uint32_t r = r0 + i;
      if (r < g.rows) {
        a.gboff[base + r] = (uint64_t)plane * cap + pre;
        if (a.index) {  // the decoders' row index (bic_row_index): slot-relative offset, 1s before the row
          a.index[2 * (base + r)] = pre;
          a.index[2 * (base + r) + 1] = a.row_o[base + r];
        }
        if (pre + v[i] > cap) {
          a.glen[base + r] = 0;  // overflowed: nothing written, fixup skips
          atomicOr(&a.flags[0], 1u);
        }
      }
      pre += v[i];
    }
    if (b == nb - 1 && threadIdx.x == 0) a.bits_g[plane] = btot + tot;
  }
  SSTAMP(4);
}

// One row across a workgroup of blockDim.x / 64 (<= 4) waves, lane = word 64 v + lane of wave v:
// the lane's sample base n (samples of the plane before its word's first 1, from nbase = the
// samples before the row) and jp (the row's last 1 before its word, -1: none), from wave scans
// and the earlier waves' totals exchanged through LDS (sh: 8 words); ones = the row's 1s.
struct WideRow {
  uint32_t n;
  int jp;
  uint32_t ones;
};
__device__ __forceinline__ WideRow wide_prefix(uint64_t x, uint32_t w, uint32_t nbase, uint32_t* sh) {
  const int lane = lane_id(), v = (int)wave_id(), nw = blockDim.x >> 6;
  const uint32_t pc = (uint32_t)__popcll(x), inc = wave_incl_sum_u32(pc);
  const int mx = wave_incl_max(x ? (int)(w * 64 + 63 - __builtin_ctzll(x)) : -1);
  if (lane == 63) {
    sh[v] = inc;
    sh[8 + v] = (uint32_t)mx;
  }
  __syncthreads();
  uint32_t nb = nbase, tot = 0;
  int jb = -1;
  for (int u = 0; u < nw; ++u) {
    const uint32_t c = sh[u];
    if (u < v) {
      nb += c;
      jb = max(jb, (int)sh[8 + u]);
    }
    tot += c;
  }
  __syncthreads();  // sh is reused
  return WideRow{nb + inc - pc, max(jb, dpp_or<0x138>(-1, mx)), tot};
}

// The listed rows' Golomb lengths (codeword walk, word_len), one workgroup per row and one HALF word
// per lane (lanes 2w and 2w + 1 share residual word w, each counting the codewords whose '1' lies in
// its 32 columns), so a row's serial codeword chain is at most 32 columns long; a fixed grid strides
// over the list, whose length k_scan_rows left in counter[2]. k_emit_rest takes the rows with mixed k,
// and the row holding the plane's first 1, from this same list. (One word per lane: C3 walk 17.4 us.)
constexpr uint32_t kWalkWaves = 8192;  // the walk grid in waves (32 per CU), whatever the row width
#ifndef BIC_WALK_SPLIT
#define BIC_WALK_SPLIT 2
#endif
constexpr uint32_t kWalkSplit = BIC_WALK_SPLIT;  // lanes per residual word (1 or 2)
// residual word w of a row on its own (the word left of it loaded too): no cross-lane exchange, so
// any lane layout can call it
template <bool PREDICT>
__device__ __forceinline__ uint64_t resid_word_at(const uint64_t* planes, const Geom& g, uint32_t plane, uint32_t row,
                                                  uint32_t w) {
  if (w >= g.used) return 0;
  const uint64_t* cur = planes + (uint64_t)plane * g.plane_words + (uint64_t)row * g.wpr;
  uint64_t d = cur[w];
  if constexpr (PREDICT) {
    const uint64_t* up = cur - g.wpr;
    if (row) d ^= up[w];
    const uint64_t dl = w ? cur[w - 1] ^ (row ? up[w - 1] : 0ull) : 0ull;
    d ^= (d >> 1) | (dl << 63);
    if (row == 0 && w == 0) d &= ~BIC_MSB;  // pred.cpp never writes pP(0,0)
  }
  return w == g.used - 1 ? d & g.trail : d;
}
template <bool PREDICT>
__global__ __launch_bounds__(512) void k_row_walk(FusedArgs a) {
  __shared__ uint32_t sh[16], sl[8], sk[8];
  const Geom& g = a.g;
  const int lane = lane_id(), v = (int)wave_id(), nw = blockDim.x >> 6;
  const uint32_t w = (64 * v + lane) / kWalkSplit, h = kWalkSplit == 1 ? 1u : (uint32_t)lane & 1u;
  const uint64_t hmask = kWalkSplit == 1 ? ~0ull : (h ? 0x00000000FFFFFFFFull : 0xFFFFFFFF00000000ull);
  const uint32_t nlist = __hip_atomic_load(a.counter + 2, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  // (the list entry -- row id and its row_o, side by side -- of the workgroup's next row is loaded
  // while this row is walked)
  uint32_t nid = blockIdx.x < nlist ? a.walk_ids[blockIdx.x] : 0u, nO = blockIdx.x < nlist ? a.walk_o[blockIdx.x] : 0u;
  for (uint32_t i = blockIdx.x; i < nlist; i += gridDim.x) {
    const uint64_t id = nid;
    const uint32_t O = nO;
    if (i + gridDim.x < nlist) {
      nid = a.walk_ids[i + gridDim.x];
      nO = a.walk_o[i + gridDim.x];
    }
    WSTAMP(4);
    const uint32_t plane = (uint32_t)(id / g.rows), row = (uint32_t)(id % g.rows);
    const uint64_t x = ((!PREDICT && a.esrc) ? eg_src_word(a.esrc + (uint64_t)plane * a.slot_e, g, row, w)
                                             : resid_word_at<PREDICT>(a.planes, g, plane, row, w)) & hmask;
    WSTAMP(5);
    const WideRow p = wide_prefix(x, w, O + row, sh);
    uint32_t kor = 0, keol = 0;
    uint64_t kt = 0;
    const bool eol = w == g.used - 1 && h == 1;
    uint32_t ll = (kKMixRows || kKnownMix) && a.kmask ? word_len_kt(x, w, p.n, p.jp, row * (g.cols + 1), eol, g.cols, kor, kt, keol)
                                       : word_len(x, w, p.n, p.jp, row * (g.cols + 1), eol, g.cols, kor);
    ll = wave_sum_u32(ll);
    WSTAMP(6);
    const uint64_t ks = __ballot(kor & ~1u), k1s = __ballot(kor & ~2u);  // some k != 0 / some k != 1
    const uint64_t kbig = __ballot(kor & ~3u), ke = __ballot(keol);     // some k >= 2 / the end-of-row k = 1
    if ((kKMixRows || kKnownMix) && a.kmask && i < a.kcap) {  // the word's k = 1 mask (its two halves' lanes combined) for kmix_row
      const uint64_t kw = kWalkSplit == 2 ? kt | shfl_u64(kt, lane ^ 1) : kt;
      if ((kWalkSplit == 1 || h == 0) && w < g.used) a.kmask[(uint64_t)i * g.used + w] = kw;
    }
    if (lane == 0) {
      sl[v] = ll;
      sk[v] = (ks ? 1u : 0u) | (k1s ? 2u : 0u) | (kbig ? 4u : 0u) | (ke ? 8u : 0u);
    }
    __syncthreads();
    if (threadIdx.x == 0) {
      uint32_t L = 0, kk = 0;
      for (int u = 0; u < nw; ++u) {
        L += sl[u];
        kk |= sk[u];
      }
      // (mixed-k rows and the plane's first-1 row are k_emit_rest's: it finds them in this list by
      // glen's flags and row_o, so no row is appended here -- thousands of same-address atomics
      // would serialise this kernel; on the class kernels' path the mixed rows whose codewords all have
      // k <= 1 and whose masks were stored are kmix_rows', flagged kKMix)
      const bool kmix = a.kmask && i < a.kcap && (kk & 3u) == 3u && !(kk & 4u);
      a.glen[id] = L | (!(kk & 1u) ? kK0Row : (!(kk & 2u) ? kK1Row : 0)) | (kmix ? kKMix : 0) |
                   (kmix && (kk & 8u) ? kKEol1 : 0);
      if (kmix) a.row_wi[id] = i;
    }
    WSTAMP(7);
    __syncthreads();
  }
}

// The rows with every prefix known. EG rows, and Golomb rows whose codewords all have k = 0 (the
// residual row and its '1'), are shifted copies formed in registers; Golomb rows whose codewords
// all have k = 1 go through an LDS row image (byte tables), written with plain stores. Rows whose
// image exceeds the LDS window go to the k_rows_global list; rows with mixed k and the EG row of
// the plane's first 1 are k_emit_rest's (their per-codeword path alone costs ~50 VGPRs, which
// would halve this kernel's occupancy). The words shared with neighbouring rows go to the fragment
// tables (k_fixup). One wave per row, persistent 4-wave workgroups, no barriers after the byte
// tables are staged (XCD-remapped block order: the waves of one XCD hold consecutive rows, the
// row above is an L2 hit).
constexpr int kEmitWaves = 4;
#ifndef BIC_REST_AUX
#define BIC_REST_AUX 1
#endif
constexpr bool kRestAux = BIC_REST_AUX != 0;
#ifndef BIC_REST_PRIO
#define BIC_REST_PRIO 0  // (A/B: k_emit_rest's waves at s_setprio(N) beside the class kernels)
#endif  // k_emit_rest on the context's second stream (beside k_emit_known)
#ifndef BIC_CLASS_NT
#define BIC_CLASS_NT 0
#endif
// the class kernels' output stores (typed unsigned long long; BIC_CLASS_NT: non-temporal)
__device__ __forceinline__ void class_store(uint64_t* dst, uint64_t v) {
  if constexpr (BIC_CLASS_NT) __builtin_nontemporal_store((unsigned long long)v, reinterpret_cast<unsigned long long*>(dst));
  else *reinterpret_cast<unsigned long long*>(dst) = v;
}
// write_row64 with a fixed number of store instructions (MAXT per lane, the idle lanes' to a.sink)
// and its stores typed unsigned long long (k_emit_k0)
template <int MAXT>
__device__ __forceinline__ void write_row64_fixed(const uint64_t* img, uint64_t L, uint64_t G, uint64_t* out,
                                                  uint64_t* frag, uint64_t* sink) {
  const int lane = lane_id();
  const uint64_t w0 = G >> 6, w1 = (G + L - 1) >> 6;
  const uint32_t nw = (uint32_t)(w1 - w0 + 1), g = (uint32_t)(G & 63);
  const bool head_whole = g == 0, tail_whole = ((G + L) & 63) == 0;
#pragma unroll
  for (int it = 0; it < MAXT; ++it) {
    const uint32_t t = it * 64 + lane;
    const bool in = t < nw;
    const uint32_t tc = in ? t : 0u;
    // (the image read as unsigned long long, the type its atomics write: ordered after them)
    const unsigned long long* im = reinterpret_cast<const unsigned long long*>(img);
    const uint64_t cur = im[tc], prev = tc ? im[tc - 1] : 0ull;
    const uint64_t v = funnel64(prev, cur, g);
    const bool whole = in && (t != 0 || head_whole) && (t != nw - 1 || tail_whole);
    uint64_t* dst = whole ? out + w0 + t : (in ? frag + (t == 0 ? 0 : 1) : sink + lane);
    class_store(dst, whole ? bswap64(v) : v);
  }
}

// Rows mixing k = 0 and k = 1 (the walk stored each word's k = 1 mask): the backward-parity rows of
// k1_rows with every column's k from the masks (bic_k1pi.h kmix_kk / kmix_word_*: a byte whose columns
// share one k through the k = 1 table or verbatim, a byte where k changes column by column).
// GolombCoder.cpp:13-34 per codeword. Lane l holds words t * 64 + l (one word group at a time: few
// registers). kmix_encode: the row's residual words rr and k = 1 masks ktw into the wave's LDS image
// gimg, then out (L bits at G; the words shared with neighbouring rows to the fragment table).
template <int WPL>
__device__ __forceinline__ void kmix_encode(const FusedArgs& a, const uint64_t (&rr)[WPL], const uint64_t (&ktw)[WPL],
                                            uint32_t keol, uint64_t id, uint64_t L, uint64_t G, uint32_t* gimg,
                                            const uint32_t* s_lut) {
  const Geom& g = a.g;
  const int lane = lane_id();
  constexpr uint32_t kCapBits = (kGImg - kPad) * 32;
  const uint32_t tail = g.cols & 63u;  // columns of the row's last word (0: a full word)
    unsigned long long* z = reinterpret_cast<unsigned long long*>(gimg);
    for (int j = lane; j < kGImg / 2; j += 64) z[j] = 0ull;
    uint64_t* img = reinterpret_cast<uint64_t*>(gimg);
    auto ws = [&](int t, uint64_t& xt, uint64_t& Z, uint64_t& kt) {
      const uint32_t w = (uint32_t)t * 64 + lane;
      const uint64_t valid = w < g.used ? (w == g.used - 1 ? g.trail : ~0ull) : 0ull;
      const uint64_t eb = (w == g.used - 1 && tail) ? (BIC_MSB >> tail) : 0ull;  // the end-of-row 1
      xt = rr[t] | eb;
      Z = ~xt & valid;
      kt = (ktw[t] & rr[t]) | (keol ? eb : 0ull);
    };
    // zeta (pi right of the word) and nk (the k of the first codeword ending after the word): from the
    // nearest lane to the right in the word's group holding a 1, else from the first such word of a
    // later group (carried), else the end of the row
    uint32_t zb = 0, kb = 0, zc = 0, kc = keol;
#pragma unroll
    for (int t = WPL - 1; t >= 0; --t) {
      uint64_t xt, Z, kt;
      ws(t, xt, Z, kt);
      const uint32_t cz = xt ? (uint32_t)__builtin_clzll(xt) : 0u;
      const uint32_t lead = cz & 1u, leadk = (uint32_t)(kt >> (63 - cz)) & 1u;
      const uint64_t m1 = __ballot(xt != 0);
      const uint64_t nm = m1 & ~((2ull << lane) - 1ull);
      const int src = nm ? (int)__builtin_ctzll(nm) : lane;
      const uint32_t ln = (uint32_t)__shfl((int)lead, src), lnk = (uint32_t)__shfl((int)leadk, src);
      zb |= (nm ? ln : zc) << t;
      kb |= (nm ? lnk : kc) << t;
      if (m1) {
        const int f = (int)__builtin_ctzll(m1);
        zc = (uint32_t)__builtin_amdgcn_readlane((int)lead, f);
        kc = (uint32_t)__builtin_amdgcn_readlane((int)leadk, f);
      }
    }
    const uint32_t kk0 = kc, lf = zc;  // the row's first codeword's k (its remainder bit leads), pi(-1)
    const uint32_t* T = s_lut;
    uint32_t loc = kk0;
#pragma unroll
    for (int t = 0; t < WPL; ++t) {
      if (t * 64 >= (int)g.used) break;
      const uint32_t w = (uint32_t)t * 64 + lane;
      uint64_t xt, Z, kt;
      ws(t, xt, Z, kt);
      const uint32_t zt = (zb >> t) & 1u, nt = (kb >> t) & 1u;
      const uint64_t Pi = k1_pi(xt, Z, zt), KK = kmix_kk(xt, Z, kt, nt);
      uint64_t hi = 0, lo = 0, A, B;
      uint32_t Lw = 0;
      if (w < g.used) {
        if (w == g.used - 1 && tail) Lw = kmix_word_last(rr[t], Pi, KK, nt, tail, hi, lo);
        else Lw = kmix_word_full2(rr[t], Pi, KK, nt, T, hi, lo);
      }
      left128(hi, lo, Lw ? Lw : 128u, A, B);
      const uint32_t inc = wave_incl_sum_u32(Lw);
      place128_64(img, loc + inc - Lw, A, B, Lw);
      loc += lane63_u32(inc);
    }
    const uint32_t tot = loc + (tail ? 0u : 1u);
    if (lane == 0) {
      if (kk0 && lf) lds_or64(img, 0, BIC_MSB);
      if (!tail) lds_or64(img, (tot - 1) >> 6, BIC_MSB >> ((tot - 1) & 63));  // the end-of-row '1'
      if (tot != L) atomicOr(&a.flags[3], 1u);  // the walk's length disagrees with the emission
    }
    write_row64_fixed<(kCapBits / 64 + 1 + 63) / 64>(img, L, G, a.out_g, a.gfrag + 2 * (uint64_t)id, a.sink);
}

// kmask / row_wi of a kKMix row: its words' k = 1 masks (word t * 64 + lane)
template <int WPL>
__device__ __forceinline__ void kmix_masks(const FusedArgs& a, uint64_t id, uint64_t (&ktw)[WPL]) {
  const uint64_t* km = a.kmask + (uint64_t)a.row_wi[id] * a.g.used;
#pragma unroll
  for (int t = 0; t < WPL; ++t) {
    const uint32_t w = (uint32_t)t * 64 + lane_id();
    ktw[t] = km[w < a.g.used ? w : a.g.used - 1];
  }
}

// One row of k_emit_known (rr: its residual words; O, Lf, Gb: its ones before, Golomb length + flags,
// absolute Golomb bit offset; Eb: its plane's EG start bit), by one wave with its LDS image gimg.
template <int WPL, bool PREDICT, bool DO_G, bool DO_E>
__device__ __forceinline__ void emit_known_row(const FusedArgs& a, uint64_t id, uint32_t plane, uint32_t row,
                                               const uint64_t (&rr)[WPL], uint32_t O, uint64_t Lf, uint64_t Gb,
                                               uint64_t Eb, uint32_t* gimg, const uint32_t* s_lut,
                                               const uint32_t* s_lut2 = nullptr) {
  const Geom& g = a.g;
  const int lane = lane_id();
  constexpr uint32_t kCapBits = (kGImg - kPad) * 32;
  const uint64_t L = Lf & kLenMask;
  const bool k0 = (Lf & kK0Row) != 0, k1 = (Lf & kK1Row) != 0, fits = L <= kCapBits;
  const bool gk1 = DO_G && L && k1 && fits;  // Golomb row through the LDS image (k = 1 byte tables)
  if (gk1) {  // zero the Golomb image: 8-byte stores of its atomics' type (see lds_image_zero32)
    unsigned long long* z = reinterpret_cast<unsigned long long*>(gimg);
    for (int i = lane; i < kGImg / 2; i += 64) z[i] = 0ull;
  }
  bool f_here = false;  // the plane's first 1 is in this row (k_emit_rest writes its EG row)
  if (DO_E && O == 0) {
    uint32_t ones = 0;
#pragma unroll
    for (int t = 0; t < WPL; ++t) ones += (uint32_t)__popcll(rr[t]);
    f_here = wave_sum_u32(ones) > 0;
  }
  if constexpr (DO_E) {  // EG as written (eg.cpp:20-37): per row ~R then '1'; a '0' after the plane's first 1
    const uint64_t Le = (uint64_t)g.cols + 1 + (f_here ? 1 : 0);
    const uint64_t Ge_rel = (uint64_t)row * (g.cols + 1) + (O > 0 ? 1 : 0);
    const uint64_t cap = a.slot_e * 64;
    const uint64_t Ge = Eb + Ge_rel;
    if (Ge_rel + Le <= cap) {
      if (!f_here) eg_row_regs<WPL>(rr, g, Ge, Le, a.out_e, a.efrag + 2 * id);
      if (lane == 0) {
        a.eboff[id] = Ge;
        a.elen[id] = Le;
      }
    } else if (lane == 0) {
      a.eboff[id] = Ge;
      a.elen[id] = 0;
      atomicOr(&a.flags[0], 1u);
    }
    if (lane == 0 && row == g.rows - 1) a.bits_e[plane] = Ge_rel + Le;
  }
  STAMP(1);
#ifdef BIC_STAMPS
  if (lane == 0) g_stamps[id * 8 + 3] = (k0 ? 1u : 0u) | (gk1 ? 2u : 0u) | ((uint64_t)blockIdx.x << 8) |
                                        ((uint64_t)wave_id() << 40);
#endif
  if constexpr (DO_G) {
    if (k0 && L) {
      eg_row_regs<WPL, false>(rr, g, Gb, L, a.out_g, a.gfrag + 2 * id);
    } else if (gk1) {  // every codeword k = 1: branch-free byte-table words into a 64-bit LDS image
      uint64_t* img = reinterpret_cast<uint64_t*>(gimg);
#if BIC_KNOWN_PI
      // the backward parity (k1_pi) over words t * 64 + lane: zeta of a word from the next word of the
      // row holding a 1 -- in its group t to the right (ballot, bpermute), else the first such word of a
      // later group (uniform)
      const uint32_t tail = g.cols & 63u;
      uint64_t xt[WPL], Zm[WPL];
      uint32_t lead[WPL];
      uint64_t m1[WPL];
#pragma unroll
      for (int t = 0; t < WPL; ++t) {
        const uint32_t w = t * 64 + lane;
        const uint64_t valid = w < g.used ? (w == g.used - 1 ? g.trail : ~0ull) : 0ull;
        xt[t] = rr[t] | ((w == g.used - 1 && tail) ? (BIC_MSB >> tail) : 0ull);
        Zm[t] = ~xt[t] & valid;
        lead[t] = xt[t] ? (uint32_t)__builtin_clzll(xt[t]) & 1u : 0u;
        m1[t] = __ballot(xt[t] != 0);
      }
      uint32_t carry = 0, first_r = 0;  // lead of the first word holding a 1 in the groups after t
      uint32_t zeta[WPL];
#pragma unroll
      for (int t = WPL - 1; t >= 0; --t) {
        const uint64_t nm = m1[t] & ~((2ull << lane) - 1ull);
        const uint32_t ln = (uint32_t)__shfl((int)lead[t], nm ? (int)__builtin_ctzll(nm) : lane);
        zeta[t] = nm ? ln : carry;
        if (m1[t]) carry = (uint32_t)__builtin_amdgcn_readlane((int)lead[t], (int)__builtin_ctzll(m1[t]));
      }
      first_r = carry;  // (the lead of the row's first word holding a 1; 0: none)
      const uint32_t* T = s_lut;
      uint32_t loc = 1;  // bit 0: the first run's remainder
#pragma unroll
      for (int t = 0; t < WPL; ++t) {
        if (t * 64 >= (int)g.used) break;
        const uint32_t w = t * 64 + lane;
        const uint64_t Pi = k1_pi(xt[t], Zm[t], zeta[t]);
        uint64_t hi = 0, lo = 0, A, B;
        uint32_t Lw = 0;
        if (w < g.used) {
          if (w == g.used - 1 && tail) Lw = k1_word_last(rr[t], Pi, tail, hi, lo);
          else Lw = k1_word_full(rr[t], Pi, T, hi, lo);
        }
        left128(hi, lo, Lw ? Lw : 128u, A, B);
        const uint32_t inc = wave_incl_sum_u32(Lw);
        place128_64(img, loc + inc - Lw, A, B, Lw);
        loc += lane63_u32(inc);
      }
      if (!tail) ++loc;  // the end-of-row '1' after the last word
      if (lane == 0) {
        if (first_r) lds_or64(img, 0, BIC_MSB);
        if (!tail) lds_or64(img, (loc - 1) >> 6, BIC_MSB >> ((loc - 1) & 63));
      }
#else
      int jpc = -1;
      uint32_t loc = 0;
#pragma unroll
      for (int t = 0; t < WPL; ++t) {
        if (t * 64 >= (int)g.used) break;
        const uint32_t w = t * 64 + lane;
        const uint64_t x = rr[t];
        const int jp = step_jp(x, w, jpc);
        const bool eol = w == g.used - 1;
        const LaneEnc e = encode_word_k1b(x, w, jp, eol, g.cols, s_lut);
        const uint32_t inc = wave_incl_sum_u32(e.len);
        const uint32_t off = loc + inc - e.len;
        loc += lane63_u32(inc);
        if (!e.lng) {
          if (e.head) lds_or64(img, off >> 6, BIC_MSB >> (off & 63));
          place128_64(img, off + 1 + e.z, e.t0, e.t1, e.tlen);
        } else {
          LdsSink64 ls{img, 0, 0};
          emit_word_k1(ls, off, x, w, jp, eol, g.cols);
          ls.flush();
        }
      }
#endif
      if (lane == 0 && loc != L) atomicOr(&a.flags[3], 1u);  // word_len disagrees with the emission
      __builtin_amdgcn_fence(__ATOMIC_ACQ_REL, "wavefront");
      __builtin_amdgcn_wave_barrier();
      write_row64(img, L, Gb, a.out_g, a.gfrag + 2 * id);
    } else if (kKnownMix && !DO_E && a.kmask && (Lf & kKMix) && L && fits) {  // k = 0 and k = 1 mixed
      uint64_t ktw[WPL];
      kmix_masks<WPL>(a, id, ktw);
      kmix_encode<WPL>(a, rr, ktw, (Lf & kKEol1) ? 1u : 0u, id, L, Gb, gimg, s_lut2);
    }
    if (lane == 0) {
      // glen keeps its flags: k_emit_rest (on the other stream) reads them too
      const bool slow = L && !k0 && !fits;
      a.gslow[id] = slow ? O + row + 1 : 0;  // k_rows_global writes the row
      if (slow) a.slow_ids[atomicAdd(a.slow_n, 1u)] = id;
    }
  }
}

#ifndef BIC_KNOWN_BATCH
#define BIC_KNOWN_BATCH 1  // (4: C4 0.272 -> 0.309 ms; kept as a build-time A/B knob)
#endif
template <int WPL>
constexpr int kKnownBatch = WPL == 1 ? BIC_KNOWN_BATCH : 1;
// ES: the residual rows from the EG stream the count pass wrote (FusedArgs::esrc; PREDICT false)
template <int WPL, bool PREDICT, bool DO_G, bool DO_E, bool ES = false>
#ifndef BIC_KNOWN_MINW
#define BIC_KNOWN_MINW 4  // (k_emit_known<1>: minimum waves per SIMD the compiler must fit)
#endif
__global__ __launch_bounds__(64 * kEmitWaves, WPL == 1 ? BIC_KNOWN_MINW : 4) void k_emit_known(FusedArgs a) {
  __shared__ __attribute__((aligned(16))) uint32_t lds[kEmitWaves * kGImg];
  __shared__ uint32_t s_lut[512];
  __shared__ uint32_t s_lut2[kKnownMix && DO_G && !DO_E ? 512 : 1];  // (kmix_encode: the k = 1 parity table)
  const Geom& g = a.g;
  [[maybe_unused]] const int lane = lane_id();
  const int wave = (int)wave_id();
  uint32_t* gimg = lds + wave * kGImg;
  if (DO_G)
    for (uint32_t i = threadIdx.x; i < 512; i += blockDim.x) s_lut[i] = reinterpret_cast<const uint32_t*>(a.lut + 256)[kKnownTable + i];
  if constexpr (kKnownMix && DO_G && !DO_E)
    for (uint32_t i = threadIdx.x; i < 512; i += blockDim.x) s_lut2[i] = reinterpret_cast<const uint32_t*>(a.lut + 256)[kK1Table + i];
  __syncthreads();  // the only workgroup barrier
  const uint64_t nrows = (uint64_t)g.rows * g.nplanes;
  // persistent waves: rows id, id + stride, ...
  const uint64_t stride = (uint64_t)gridDim.x * kEmitWaves;
  const uint64_t id0 = (uint64_t)xcd_remap(blockIdx.x, gridDim.x) * kEmitWaves +
                       (uint32_t)__builtin_amdgcn_readfirstlane(wave);  // (uniform, as the compiler sees it)
  if constexpr (!ES && kKnownBatch<WPL> > 1) {
    // one-word rows (WPL = 1: rows of <= 4096 columns, e.g. C4's frames) are latency-bound: a wave
    // loads kKnownBatch rows before it stores the first one's output (a wave that loaded after
    // storing would wait for its stores' acknowledgements every row: vmcnt counts both)
    constexpr int B = kKnownBatch<WPL>;
    for (uint64_t id = id0; id < nrows; id += stride * B) {
      uint64_t cp_[B][WPL], cu_[B][WPL];
      uint32_t O[B];
      uint64_t Lf[B], Gb[B];
#pragma unroll
      for (int u = 0; u < B; ++u) {
        const uint64_t iu = id + u * stride < nrows ? id + u * stride : id;
        const uint32_t plane = (uint32_t)(iu / g.rows), row = (uint32_t)(iu % g.rows);
        row_load<WPL, PREDICT>(a.planes, g, plane, row, cp_[u], cu_[u]);
        O[u] = a.row_o[iu];
        Lf[u] = DO_G ? a.glen[iu] : 0;
        Gb[u] = DO_G ? gb_abs(a, iu, plane) : 0;
      }
#pragma unroll
      for (int u = 0; u < B; ++u) {
        const uint64_t iu = id + u * stride;
        if (iu >= nrows) break;
        const uint32_t plane = (uint32_t)(iu / g.rows), row = (uint32_t)(iu % g.rows);
        uint64_t rr[WPL];
        row_resid<WPL, PREDICT>(g, row, cp_[u], cu_[u], rr);
        const uint64_t Eb = DO_E ? (a.ebase ? a.ebase[plane] : (uint64_t)plane * a.slot_e * 64) : 0;
        emit_known_row<WPL, PREDICT, DO_G, DO_E>(a, iu, plane, row, rr, O[u], Lf[u], Gb[u], Eb, gimg, s_lut, s_lut2);
        __builtin_amdgcn_fence(__ATOMIC_ACQ_REL, "wavefront");  // the next row reuses the LDS image
        __builtin_amdgcn_wave_barrier();
      }
    }
    return;
  }
  for (uint64_t id = id0; id < nrows; id += stride) {
    const uint32_t plane = (uint32_t)(id / g.rows), row = (uint32_t)(id % g.rows);
    STAMP(0);
    uint64_t rr[WPL];
    uint32_t O;
    uint64_t Lf, Gb;
    if constexpr (ES) {
      eg_src_row<WPL>(a.esrc + (uint64_t)plane * a.slot_e, g, row, rr);
      O = a.row_o[id];
      Lf = DO_G ? a.glen[id] : 0;
      Gb = DO_G ? gb_abs(a, id, plane) : 0;
    } else {
      uint64_t cp_[WPL], cu_[WPL];
      row_load<WPL, PREDICT>(a.planes, g, plane, row, cp_, cu_);
      O = a.row_o[id];
      Lf = DO_G ? a.glen[id] : 0;
      Gb = DO_G ? gb_abs(a, id, plane) : 0;  // loaded with the row, not after the branch that uses it
      row_resid<WPL, PREDICT>(g, row, cp_, cu_, rr);
    }
    const uint64_t Eb = DO_E ? (a.ebase ? a.ebase[plane] : (uint64_t)plane * a.slot_e * 64) : 0;
    emit_known_row<WPL, PREDICT, DO_G, DO_E>(a, id, plane, row, rr, O, Lf, Gb, Eb, gimg, s_lut, s_lut2);
    STAMP(2);
    __builtin_amdgcn_fence(__ATOMIC_ACQ_REL, "wavefront");  // the next row reuses the LDS image
    __builtin_amdgcn_wave_barrier();
  }
}

// ---- EG source: one light emission kernel per row class ------------------------------------------
// With the residual rows read back from the EG stream (FusedArgs::esrc) the Golomb emission is split
// by the class the prefix kernels proved for the row (the LEN scan's lists): rows whose codewords
// all have k = 0 are shifted copies of the EG stream, inverted (k_emit_k0, no LDS), rows whose
// codewords all have k = 1 go through the byte tables and an LDS row image (k_emit_k1); mixed rows
// stay k_emit_rest's. Persistent waves, one row at a time, in the list order i, i + nw, ...
//
// Both kernels keep the memory system busy the same way: the next row's source words are loaded
// before the current row's output is stored, into the other of two word buffers (ping-pong, no
// register copies). gfx9's vmcnt counts stores with loads: a wave that loaded after storing would
// wait for its stores' acknowledgements every row. With the loads first, every load and store issued
// unconditionally (clamped indices, idle lanes storing to a.sink), the list entries read through the
// scalar cache (the kernels' stores are typed unsigned long long, apart from the entries' u64, and
// they hold no fence or workgroup barrier, so the compiler proves the entries unclobbered), the
// compiler waits for the loads alone.
__device__ __forceinline__ uint64_t rl64(uint64_t v, uint32_t l) {
  return ((uint64_t)(uint32_t)__builtin_amdgcn_readlane((int)(uint32_t)(v >> 32), (int)l) << 32) |
         (uint32_t)__builtin_amdgcn_readlane((int)(uint32_t)v, (int)l);
}

__device__ __forceinline__ uint64_t cls_ld(const FusedArgs& a, uint64_t i) { return a.cls[i]; }

// k = 0: the row's Golomb bits are R then the end-of-row '1' (GolombCoder.cpp:13-34 with k = 0: each
// sample's zeros and its '1'), i.e. the EG row ~R '1' (eg.cpp:20-37) with its first cols bits inverted.
// Output word t of the row (at bit Gb) holds row bits [64 t - g, 64 t - g + 64), g = Gb % 64: the
// stream bits from Bsrc + 64 t - g (Bsrc: the row in the EG slot), one funnel shift per word.
#ifndef BIC_K0_W16
#define BIC_K0_W16 0
#endif
#ifndef BIC_K0_BATCH
// (8-byte lanes, pipelined batches of 3: C3 emission 162-165 -> 157-158 us; of 2: 159-162; of 4: 170-173.
// Batches of 2 keep k_emit_k01 at <= 128 VGPRs (113; batches of 3: 129), which its rest role needs
// (BIC_K01_REST: a fourth workgroup slot per CU beside three persistent ones). 16-byte lanes: 115 VGPRs
// at batches of 2). Round 6: batches of 2 with four workgroups per CU (BIC_K01_OCC 4, 113 VGPRs) --
// k_emit_k01 137 -> 132-137 us against 142-147 at batches of 3 and three per CU, same box
// (profiles/r06/ab_emission.txt gj25, gj26); the C3 step unchanged (k_emit_rest beside it takes the slack)
#define BIC_K0_BATCH 2
#endif
constexpr int kK0Batch = BIC_K0_BATCH;
#ifndef BIC_DIAG_K0
#define BIC_DIAG_K0 0
#endif
#ifndef BIC_K0_PLACE_AHEAD
#define BIC_K0_PLACE_AHEAD 0
#endif
#ifndef BIC_K0_PIPE
#define BIC_K0_PIPE 1
#endif
#ifndef BIC_K0_FAST
#define BIC_K0_FAST 1
#endif
// the k = 0 list's entries i0, i0 + nw, ... (one wave; i0 and nw wave-uniform)
template <int WPL, int BATCH = kK0Batch>
__device__ __forceinline__ void k0_rows(const FusedArgs& a, uint32_t i0, uint32_t nw) {
  const Geom& g = a.g;
  const int lane = lane_id();
  const uint32_t n = __hip_atomic_load(a.counter + 4, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  const uint64_t L = (uint64_t)g.cols + 1;
  const uint64_t* S = a.esrc;
  if (i0 >= n) return;
  const uint32_t R = (n - i0 + nw - 1) / nw;  // the wave's rows
  struct Row {
    uint32_t id;
    uint64_t G;
    int64_t si;
    uint32_t d;
  };
  // row k of the wave (list entry i0 + k nw): where its output and its source bits are
  auto place = [&](uint32_t k) {
    const uint64_t e = i0 + (uint64_t)k * nw;
    Row r;
    const uint64_t e0 = cls_ld(a, 2 * e);
    r.id = (uint32_t)e0;
    // (the k = 0 entries carry the plane where the k = 1 ones carry the length, which is cols + 1 here:
    // no division by rows on the scalar unit)
    const uint32_t plane = (uint32_t)(e0 >> 32), row = r.id - plane * g.rows;
    const uint64_t Gs = cls_ld(a, 2 * e + 1);
    r.G = a.off_g ? Gs - (uint64_t)plane * a.slot_g * 64 + a.gbase[plane] * 64 : Gs;
    // stream bit of output word t's first bit: Bsrc - G % 64 + 64 t (>= -63: floor below)
    const int64_t s0 = (int64_t)((uint64_t)plane * a.slot_e * 64 + eg_src_bit0(g, row)) - (int64_t)(r.G & 63);
    r.si = s0 >> 6;
    r.d = (uint32_t)(s0 & 63);
    return r;
  };
#if !BIC_K0_W16 && BIC_K0_FAST
  // Word groups 64 k .. 64 k + 63 of the output row. A group wholly inside the row (k >= 1 and before
  // the row's last word: C3's groups 1-3 of 5) needs no masks, clamps or fragment selects -- a uniform
  // branch on the row's scalar offsets -- and loads / stores through a scalar base plus the lane's
  // 32-bit offset: ~16 VALU per group instead of ~55 (the copies share each SIMD's VALU issue with the
  // k = 1 rows and k_emit_rest, and the younger waves wait for it: tools/k01_stamps.py)
  auto load = [&](const Row& r, uint64_t (&v)[WPL + 1]) {
    const int64_t jend = r.si + (int64_t)((r.d + (r.G & 63) + g.cols) >> 6);
    const uint64_t* sb = S + r.si;  // (r.si >= -1: only group 0 may start before the stream)
#pragma unroll
    for (int k = 0; k <= WPL; ++k) {
      if (k >= 1 && r.si + 64 * k + 63 <= jend) {
        v[k] = sb[64 * k + lane];
      } else {
        const int64_t j = r.si + 64 * k + lane;
        const int64_t jc = j > jend ? jend : j;
        v[k] = S[jc < 0 ? 0 : jc];
      }
    }
  };
  auto emit = [&](const Row& cur, uint64_t (&v)[WPL + 1]) {
    const uint32_t gs = (uint32_t)(cur.G & 63);
    const uint64_t w0 = cur.G >> 6, nwo = ((cur.G + L - 1) >> 6) - w0 + 1;  // output words (<= used + 2)
    const uint64_t eolw = (uint64_t)(g.cols + gs) >> 6, eolb = BIC_MSB >> ((g.cols + gs) & 63);
    const int64_t jend = cur.si + (int64_t)((cur.d + gs + g.cols) >> 6);
    unsigned long long* ob = reinterpret_cast<unsigned long long*>(a.out_g + w0);
#pragma unroll
    for (int k = 0; k <= WPL; ++k) {
      uint64_t nx = ((uint64_t)(uint32_t)__builtin_amdgcn_update_dpp(0, (int)(uint32_t)(v[k] >> 32), 0x130, 0xf, 0xf, true) << 32) |
                    (uint32_t)__builtin_amdgcn_update_dpp(0, (int)(uint32_t)v[k], 0x130, 0xf, 0xf, true);
      if (k < WPL) {
        const uint64_t n0 = rl64(v[k + 1 <= WPL ? k + 1 : k], 0);
        if (lane == 63) nx = n0;
      }
      if (k >= 1 && (uint64_t)(64 * k + 63) < nwo - 1) {  // interior group: a shifted, inverted copy
        const uint64_t x = ~(cur.d ? funnel64(bswap64(v[k]), bswap64(nx), 64 - cur.d) : bswap64(v[k]));
        class_store(reinterpret_cast<uint64_t*>(ob + 64 * k + lane), bswap64(x));
        continue;
      }
      const uint32_t t = 64 * k + lane;
      const int64_t j = cur.si + 64 * k + lane;
      const uint64_t vk = (j >= 0 && j <= jend) ? v[k] : 0ull;
      // (lane 63's next word: the next group's first, in range when that group is)
      const uint64_t hi = bswap64(vk);
      uint64_t x = ~(cur.d ? funnel64(hi, bswap64(nx), 64 - cur.d) : hi);
      // row bits outside [0, cols) are not the row's: before it (word 0's first gs bits) and from the
      // end-of-row '1' on
      if (t == 0) x &= ~0ull >> gs;
      if (t >= eolw) x = t == eolw ? (x & ~((eolb << 1) - 1)) | eolb : 0ull;
      const bool in = t < nwo;
      const bool whole = in && (t != 0 || gs == 0) && (t != nwo - 1 || ((cur.G + L) & 63) == 0);
      uint64_t* dst = whole ? a.out_g + w0 + t : (in ? a.gfrag + 2 * (uint64_t)cur.id + (t == 0 ? 0 : 1) : a.sink + lane);
      if (k < WPL || in) class_store(dst, whole ? bswap64(x) : x);
    }
  };
#elif !BIC_K0_W16
  // the row's source words (those holding its bits through its end-of-row '1'; the slot may end
  // there): every lane loads, at a clamped index, the words outside masked where used
  auto load = [&](const Row& r, uint64_t (&v)[WPL + 1]) {
    const int64_t jend = r.si + (int64_t)((r.d + (r.G & 63) + g.cols) >> 6);
#pragma unroll
    for (int k = 0; k <= WPL; ++k) {
      const int64_t j = r.si + 64 * k + lane;
      const int64_t jc = j > jend ? jend : j;
#if BIC_DIAG_K0 == 2  // diagnostic build only (wrong output): the copies' loads from one cached line
      v[k] = S[lane + (r.id & 1)];
      (void)jc;
#else
      v[k] = S[jc < 0 ? 0 : jc];
#endif
    }
  };
  auto emit = [&](const Row& cur, uint64_t (&v)[WPL + 1]) {
    const uint32_t gs = (uint32_t)(cur.G & 63);
    const uint64_t w0 = cur.G >> 6, nwo = ((cur.G + L - 1) >> 6) - w0 + 1;  // output words (<= used + 2)
    const uint64_t eolw = (uint64_t)(g.cols + gs) >> 6, eolb = BIC_MSB >> ((g.cols + gs) & 63);
    const int64_t jend = cur.si + (int64_t)((cur.d + gs + g.cols) >> 6);
#pragma unroll
    for (int k = 0; k <= WPL; ++k) {
      const int64_t j = cur.si + 64 * k + lane;
      v[k] &= 0ull - (uint64_t)((j >= 0) & (j <= jend));
    }
#pragma unroll
    for (int k = 0; k <= WPL; ++k) {
      const uint32_t t = 64 * k + lane;
      uint64_t nx = ((uint64_t)(uint32_t)__builtin_amdgcn_update_dpp(0, (int)(uint32_t)(v[k] >> 32), 0x130, 0xf, 0xf, true) << 32) |
                    (uint32_t)__builtin_amdgcn_update_dpp(0, (int)(uint32_t)v[k], 0x130, 0xf, 0xf, true);
      if (k < WPL) {
        const uint64_t n0 = rl64(v[k + 1 <= WPL ? k + 1 : k], 0);
        if (lane == 63) nx = n0;
      }
      const uint64_t hi = bswap64(v[k]);
      uint64_t x = ~(cur.d ? funnel64(hi, bswap64(nx), 64 - cur.d) : hi);
      // row bits outside [0, cols) are not the row's: before it (word 0's first gs bits) and from the
      // end-of-row '1' on
      if (t == 0) x &= ~0ull >> gs;
      if (t >= eolw) x = t == eolw ? (x & ~((eolb << 1) - 1)) | eolb : 0ull;
      const bool in = t < nwo;
      const bool whole = in && (t != 0 || gs == 0) && (t != nwo - 1 || ((cur.G + L) & 63) == 0);
      uint64_t* dst = whole ? a.out_g + w0 + t : (in ? a.gfrag + 2 * (uint64_t)cur.id + (t == 0 ? 0 : 1) : a.sink + lane);
#if BIC_DIAG_K0 == 1  // diagnostic build only (wrong output): the copies' stores all to the sink
      dst = a.sink + lane;
#endif
      // (unsigned long long: a type apart from the u64 loads, so no load is taken to depend on it)
      // Only the last word group has lanes past the row (the row's 257-258 words of C3): those store
      // nothing (exec-masked, the instruction count unchanged) instead of writing the sink (emission
      // 158-161 -> 155-160 us on one box)
      if (k < WPL || in) class_store(dst, whole ? bswap64(x) : x);
    }
  };
#else
  // 16 bytes per lane: lane q holds output words t0 = 128 k + 2 q - e and t0 + 1 (e = w0 & 1, so the
  // pair's store is 16-byte aligned) and loads the source words si + t0, si + t0 + 1 with one 16-byte
  // load (8-byte aligned: dword alignment is all global dwordx4 needs); si + t0 + 2 is lane q + 1's
  // first word (DPP), lane 63's from the next group's lane 0. Half the memory instructions of the
  // 8-byte form per row.
  constexpr int NG = (64 * WPL + 3 + 127) / 128;
  using V2 = HIP_vector_type<unsigned long long, 2>;
  auto load = [&](const Row& r, V2 (&v)[NG]) {
    const int64_t jend = r.si + (int64_t)((r.d + (r.G & 63) + g.cols) >> 6);
    const int64_t e = (int64_t)((r.G >> 6) & 1);
#pragma unroll
    for (int k = 0; k < NG; ++k) {
      const int64_t j = r.si - e + 128 * k + 2 * lane;
      int64_t jc = j > jend - 1 ? jend - 1 : j;
      jc = jc < 0 ? 0 : jc;
      v[k] = *reinterpret_cast<const V2*>(S + jc);
      // words outside [0, jend] read as 0, the clamped pairs realigned (j = jend: its first word is the
      // clamped pair's second; j = -1: its second word is the clamped pair's first)
      const unsigned long long lo = v[k].x, hi = v[k].y;
      v[k].x = (j >= 0 && j < jend) ? lo : (j == jend ? hi : 0ull);
      v[k].y = (j >= 0 && j + 1 <= jend) ? (j < jend ? hi : 0ull) : (j == -1 ? lo : 0ull);
    }
  };
  auto emit = [&](const Row& cur, V2 (&v)[NG]) {
    const uint32_t gs = (uint32_t)(cur.G & 63);
    const uint64_t w0 = cur.G >> 6;
    const int64_t nwo = (int64_t)(((cur.G + L - 1) >> 6) - w0 + 1);
    const int64_t eolw = (int64_t)((g.cols + gs) >> 6);
    const uint64_t eolb = BIC_MSB >> ((g.cols + gs) & 63);
    const int64_t e = (int64_t)(w0 & 1);
    const bool tail_whole = ((cur.G + L) & 63) == 0;
    auto fix = [&](uint64_t x, int64_t t) {
      if (t == 0) x &= ~0ull >> gs;
      if (t >= eolw) x = t == eolw ? (x & ~((eolb << 1) - 1)) | eolb : 0ull;
      return x;
    };
#pragma unroll
    for (int k = 0; k < NG; ++k) {
      const int64_t t0 = 128 * k + 2 * lane - e, t1 = t0 + 1;
      uint64_t n0 = ((uint64_t)(uint32_t)__builtin_amdgcn_update_dpp(0, (int)(uint32_t)(v[k].x >> 32), 0x130, 0xf, 0xf, true) << 32) |
                    (uint32_t)__builtin_amdgcn_update_dpp(0, (int)(uint32_t)v[k].x, 0x130, 0xf, 0xf, true);
      if (k + 1 < NG) {
        const uint64_t nn = rl64(v[k + 1 < NG ? k + 1 : k].x, 0);
        if (lane == 63) n0 = nn;
      }
      const uint64_t h0 = bswap64(v[k].x), h1 = bswap64(v[k].y), h2 = bswap64(n0);
      const uint64_t x0 = fix(~(cur.d ? funnel64(h0, h1, 64 - cur.d) : h0), t0);
      const uint64_t x1 = fix(~(cur.d ? funnel64(h1, h2, 64 - cur.d) : h1), t1);
      const bool in0 = t0 >= 0 && t0 < nwo, in1 = t1 >= 0 && t1 < nwo;
      const bool wh0 = in0 && (t0 != 0 || gs == 0) && (t0 != nwo - 1 || tail_whole);
      const bool wh1 = in1 && (t1 != 0 || gs == 0) && (t1 != nwo - 1 || tail_whole);
      if (wh0 && wh1) {
        V2 o;
        o.x = bswap64(x0);
        o.y = bswap64(x1);
        *reinterpret_cast<V2*>(a.out_g + w0 + t0) = o;
      } else {
        if (in0) class_store(wh0 ? a.out_g + w0 + t0 : a.gfrag + 2 * (uint64_t)cur.id + (t0 == 0 ? 0 : 1), wh0 ? bswap64(x0) : x0);
        if (in1) class_store(wh1 ? a.out_g + w0 + t1 : a.gfrag + 2 * (uint64_t)cur.id + (t1 == 0 ? 0 : 1), wh1 ? bswap64(x1) : x1);
      }
    }
  };
#define BIC_K0_VT V2
#define BIC_K0_VN NG
#endif
#if !BIC_K0_W16
#define BIC_K0_VT uint64_t
#define BIC_K0_VN WPL + 1
#endif
  // rows in batches of BATCH: every row's loads issued before the first row's stores, so a wave
  // waits for its previous stores once per batch
#if BIC_K0_PLACE_AHEAD
  // the next batch's list entries (scalar loads) are read while this batch is emitted, so a batch's
  // source loads never wait behind its own list entries
  Row rn[BATCH];
#pragma unroll
  for (int u = 0; u < BATCH; ++u) rn[u] = place((uint32_t)u < R ? (uint32_t)u : 0u);
  for (uint32_t k = 0; k < R; k += BATCH) {
    Row r[BATCH];
    BIC_K0_VT v[BATCH][BIC_K0_VN];
#pragma unroll
    for (int u = 0; u < BATCH; ++u) {
      r[u] = rn[u];
      load(r[u], v[u]);
    }
#pragma unroll
    for (int u = 0; u < BATCH; ++u) rn[u] = place(k + BATCH + u < R ? k + BATCH + u : k);
#pragma unroll
    for (int u = 0; u < BATCH; ++u)
      if (k + u < R) emit(r[u], v[u]);
  }
#elif BIC_K0_PIPE
  // software-pipelined: batch k + 1's loads issued before batch k's stores, so the wait for a batch's
  // loads never covers the previous batch's stores (vmcnt counts both, in order)
  Row ra[BATCH], rb[BATCH];
  BIC_K0_VT va[BATCH][BIC_K0_VN], vb[BATCH][BIC_K0_VN];
#pragma unroll
  for (int u = 0; u < BATCH; ++u) {
    ra[u] = place((uint32_t)u < R ? (uint32_t)u : 0u);
    load(ra[u], va[u]);
  }
  for (uint32_t k = 0; k < R; k += 2 * BATCH) {
#pragma unroll
    for (int u = 0; u < BATCH; ++u) {
      const uint32_t kk = k + BATCH + u;
      rb[u] = place(kk < R ? kk : k);
      load(rb[u], vb[u]);
    }
#pragma unroll
    for (int u = 0; u < BATCH; ++u)
      if (k + u < R) emit(ra[u], va[u]);
#pragma unroll
    for (int u = 0; u < BATCH; ++u) {
      const uint32_t kk = k + 2 * BATCH + u;
      ra[u] = place(kk < R ? kk : k);
      load(ra[u], va[u]);
    }
#pragma unroll
    for (int u = 0; u < BATCH; ++u)
      if (k + BATCH + u < R) emit(rb[u], vb[u]);
  }
#else
  for (uint32_t k = 0; k < R; k += BATCH) {
    Row r[BATCH];
    BIC_K0_VT v[BATCH][BIC_K0_VN];
#pragma unroll
    for (int u = 0; u < BATCH; ++u) {
      r[u] = place(k + u < R ? k + u : k);
      load(r[u], v[u]);
    }
#pragma unroll
    for (int u = 0; u < BATCH; ++u)
      if (k + u < R) emit(r[u], v[u]);
  }
#endif
}
#undef BIC_K0_VT
#undef BIC_K0_VN

// k = 1 rows: emit_known_row's byte-table path (encode_word_k1b into a 64-bit LDS row image, then
// write_row64_fixed); rows whose image exceeds the window are listed for k_rows_global.
#ifndef BIC_K1_BATCH
#define BIC_K1_BATCH 3
#endif
constexpr int kK1Batch = BIC_K1_BATCH;
#ifndef BIC_K1_DYN
#define BIC_K1_DYN 0  // (one ticket counter for every chunk of the ~32k k = 1 rows of C3: emission 157 -> 540 us;
                      // device-scope atomics on one word stall every wave and the memory channel holding it)
#endif
constexpr bool kK1Dyn = BIC_K1_DYN != 0;  // k1_rows: chunks claimed by ticket instead of a static share
// the k = 1 list's entries i0, i0 + nw, ... (one wave, with its LDS row image and the byte table)
template <int WPL>
__device__ __forceinline__ void k1_rows(const FusedArgs& a, uint32_t i0, uint32_t nw, uint32_t* gimg,
                                        const uint32_t* s_lut) {
  const Geom& g = a.g;
  const int lane = lane_id();
  constexpr uint32_t kCapBits = (kGImg - kPad) * 32;
  const uint64_t nrows = (uint64_t)g.rows * g.nplanes;
  const uint32_t n = __hip_atomic_load(a.counter + 5, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  if (i0 >= n) return;
  const uint32_t R = (n - i0 + nw - 1) / nw;
  struct Row {
    uint32_t id, plane, row;
    uint64_t G, L;
  };
  // (list entry e of the k = 1 list)
  auto place_e = [&](uint64_t e_rel) {
    const uint64_t e = nrows + e_rel;
    Row r;
    const uint64_t e0 = cls_ld(a, 2 * e);
    r.id = (uint32_t)e0;
    r.L = e0 >> 32;
    r.plane = r.id / g.rows;
    r.row = r.id % g.rows;
    const uint64_t Gs = cls_ld(a, 2 * e + 1);
    r.G = a.off_g ? Gs - (uint64_t)r.plane * a.slot_g * 64 + a.gbase[r.plane] * 64 : Gs;
    return r;
  };
  auto place = [&](uint32_t k) { return place_e(i0 + (uint64_t)k * nw); };  // the wave's k-th row
#if BIC_K1_LC
  constexpr int kV = WPL + 1;
  auto emit = [&](const Row& cur, const uint64_t (&v)[kV], uint64_t) {
    if (cur.L > kCapBits) {  // (the LEN scan lists such rows as slow, never here: a length disagreement)
      if (lane == 0) {
        if (kSlowRest) {
          atomicOr(&a.flags[3], 1u);
        } else {
          *reinterpret_cast<unsigned long long*>(a.gslow + cur.id) = a.row_o[cur.id] + cur.row + 1;
          *reinterpret_cast<unsigned long long*>(a.slow_ids + atomicAdd(a.slow_n, 1u)) = cur.id;
        }
      }
      return;
    }
    YSTAMP((1u << 18) + cur.id, 0);
    unsigned long long* z = reinterpret_cast<unsigned long long*>(gimg);
    for (int j = lane; j < kGImg / 2; j += 64) z[j] = 0ull;
    uint64_t rr[WPL];
    eg_src_assemble_lc<WPL>(g, cur.row, v, rr);
    YSTAMP((1u << 18) + cur.id, 1);
    uint64_t* img = reinterpret_cast<uint64_t*>(gimg);
#if BIC_K1_PI
    // the backward parity form (k1_pi): pi of each word's last column's right context (zeta) from the
    // next word holding a 1 -- in this lane, or the nearest lane to the right holding one (one ballot,
    // one bpermute); the row's first remainder bit from the first lane holding a 1
    const uint32_t tail = g.cols & 63u;  // columns of the row's last word (0: a full word)
    uint64_t xt[WPL], Zm[WPL];
    bool any = false;
    uint32_t lead = 0;
#pragma unroll
    for (int t = 0; t < WPL; ++t) {
      const uint32_t w = (uint32_t)lane * WPL + t;
      const uint64_t valid = w < g.used ? (w == g.used - 1 ? g.trail : ~0ull) : 0ull;
      xt[t] = rr[t] | ((w == g.used - 1 && tail) ? (BIC_MSB >> tail) : 0ull);  // + the end-of-row 1
      Zm[t] = ~xt[t] & valid;
    }
#pragma unroll
    for (int t = WPL - 1; t >= 0; --t)
      if (xt[t]) {
        lead = (uint32_t)__builtin_clzll(xt[t]) & 1u;
        any = true;
      }
    const uint64_t m1 = __ballot(any);
    const uint64_t nm = m1 & ~((2ull << lane) - 1ull);  // the lanes right of this one holding a 1
    const uint32_t ln = (uint32_t)__shfl((int)lead, nm ? (int)__builtin_ctzll(nm) : lane);
    const uint32_t lf = (uint32_t)__shfl((int)lead, m1 ? (int)__builtin_ctzll(m1) : 0);
    uint32_t zc = nm ? ln : 0u;  // (no 1 to the right: the end-of-row 1 follows the last word)
    uint32_t zeta[WPL];
#pragma unroll
    for (int t = WPL - 1; t >= 0; --t) {
      zeta[t] = zc;
      if (xt[t]) zc = (uint32_t)__builtin_clzll(xt[t]) & 1u;
    }
    const uint32_t* T = s_lut;
    uint64_t A[WPL], B[WPL];
    uint32_t lw[WPL], lsum = 0;
#pragma unroll
    for (int t = 0; t < WPL; ++t) {
      const uint32_t w = (uint32_t)lane * WPL + t;
      const uint64_t Pi = k1_pi(xt[t], Zm[t], zeta[t]);
      uint64_t hi = 0, lo = 0;
      uint32_t L = 0;
      if (w < g.used) {
        if (w == g.used - 1 && tail) L = k1_word_last(rr[t], Pi, tail, hi, lo);
        else L = k1_word_full(rr[t], Pi, T, hi, lo);
      }
      left128(hi, lo, L ? L : 128u, A[t], B[t]);
      lw[t] = L;
      lsum += L;
    }
    const uint32_t inc = wave_incl_sum_u32(lsum);
    uint32_t off = 1u + inc - lsum;  // (bit 0: the first run's remainder)
    const uint32_t tot = 1u + lane63_u32(inc) + (tail ? 0u : 1u);
#pragma unroll
    for (int t = 0; t < WPL; ++t) {
      place128_64(img, off, A[t], B[t], lw[t]);
      off += lw[t];
    }
    if (lane == 0) {
      if (lf && m1) lds_or64(img, 0, BIC_MSB);
      if (!tail) lds_or64(img, (tot - 1) >> 6, BIC_MSB >> ((tot - 1) & 63));  // the end-of-row '1'
      if (tot != cur.L) atomicOr(&a.flags[3], 1u);  // the closed-form length disagrees with the emission
    }
    YSTAMP((1u << 18) + cur.id, 2);
    write_row64_fixed<(kCapBits / 64 + 1 + 63) / 64>(img, cur.L, cur.G, a.out_g, a.gfrag + 2 * (uint64_t)cur.id,
                                                     a.sink);
    YSTAMP((1u << 18) + cur.id, 3);
#else
    // the lane's words l WPL + t: their last 1s, the wave's exclusive max of the lanes' last 1
    int lastc[WPL], mxl = -1;
#pragma unroll
    for (int t = 0; t < WPL; ++t) {
      const uint32_t w = (uint32_t)lane * WPL + t;
      lastc[t] = rr[t] ? (int)(w * 64 + 63 - __builtin_ctzll(rr[t])) : -1;
      mxl = max(mxl, lastc[t]);
    }
    int jp = dpp_or<0x138>(-1, wave_incl_max(mxl));  // lane 0: -1
    LaneEnc e[WPL];
    int jps[WPL];
    uint32_t lsum = 0;
#pragma unroll
    for (int t = 0; t < WPL; ++t) {
      const uint32_t w = (uint32_t)lane * WPL + t;
      jps[t] = jp;
      e[t] = encode_word_k1b(rr[t], w, jp, w == g.used - 1, g.cols, s_lut);
      lsum += e[t].len;
      jp = max(jp, lastc[t]);
    }
    const uint32_t inc = wave_incl_sum_u32(lsum);
    uint32_t off = inc - lsum;
    const uint32_t loc = lane63_u32(inc);
#pragma unroll
    for (int t = 0; t < WPL; ++t) {
      const uint32_t w = (uint32_t)lane * WPL + t;
      if (!e[t].lng) {
        if (e[t].head) lds_or64(img, off >> 6, BIC_MSB >> (off & 63));
        place128_64(img, off + 1 + e[t].z, e[t].t0, e[t].t1, e[t].tlen);
      } else {
        LdsSink64 ls{img, 0, 0};
        emit_word_k1(ls, off, rr[t], w, jps[t], w == g.used - 1, g.cols);
        ls.flush();
      }
      off += e[t].len;
    }
    if (lane == 0 && loc != cur.L) atomicOr(&a.flags[3], 1u);  // word_len disagrees with the emission
    write_row64_fixed<(kCapBits / 64 + 1 + 63) / 64>(img, cur.L, cur.G, a.out_g, a.gfrag + 2 * (uint64_t)cur.id,
                                                     a.sink);
#endif
  };
  auto load = [&](const Row& r, uint64_t (&v)[kV], uint64_t&) {
    eg_src_load_lc<WPL>(a.esrc + (uint64_t)r.plane * a.slot_e, g, r.row, v);
  };
#else
  auto emit = [&](const Row& cur, const uint64_t (&v)[WPL], uint64_t last) {
    if (cur.L > kCapBits) {  // (the LEN scan lists such rows as slow, never here: a length disagreement)
      if (lane == 0) {
        if (kSlowRest) {
          atomicOr(&a.flags[3], 1u);
        } else {
          *reinterpret_cast<unsigned long long*>(a.gslow + cur.id) = a.row_o[cur.id] + cur.row + 1;
          *reinterpret_cast<unsigned long long*>(a.slow_ids + atomicAdd(a.slow_n, 1u)) = cur.id;
        }
      }
      return;
    }
    // zeroed as unsigned long long, the type of the image's atomics (so ordered before them)
    unsigned long long* z = reinterpret_cast<unsigned long long*>(gimg);
    for (int j = lane; j < kGImg / 2; j += 64) z[j] = 0ull;
    uint64_t rr[WPL];
    eg_src_assemble<WPL>(g, cur.row, v, last, rr);
    uint64_t* img = reinterpret_cast<uint64_t*>(gimg);
    int jpc = -1;
    uint32_t loc = 0;
#pragma unroll
    for (int t = 0; t < WPL; ++t) {
      if (t * 64 >= (int)g.used) break;
      const uint32_t w = t * 64 + lane;
      const uint64_t x = rr[t];
      const int jp = step_jp(x, w, jpc);
      const bool eol = w == g.used - 1;
      const LaneEnc e = encode_word_k1b(x, w, jp, eol, g.cols, s_lut);
      const uint32_t inc = wave_incl_sum_u32(e.len);
      const uint32_t off = loc + inc - e.len;
      loc += lane63_u32(inc);
      if (!e.lng) {
        if (e.head) lds_or64(img, off >> 6, BIC_MSB >> (off & 63));
        place128_64(img, off + 1 + e.z, e.t0, e.t1, e.tlen);
      } else {
        LdsSink64 ls{img, 0, 0};
        emit_word_k1(ls, off, x, w, jp, eol, g.cols);
        ls.flush();
      }
    }
    if (lane == 0 && loc != cur.L) atomicOr(&a.flags[3], 1u);  // word_len disagrees with the emission
    // (no fence: the image's zeroing, atomics and reads are one wave's 8-byte LDS operations of one type --
    // the same width, which measured in order where a 16-byte zeroing did not (lds_image_zero32) -- and the
    // compiler keeps same-typed accesses in their order)
    // (rows up to kCapBits: at most (kCapBits + 63) / 64 + 1 output words)
    write_row64_fixed<(kCapBits / 64 + 1 + 63) / 64>(img, cur.L, cur.G, a.out_g, a.gfrag + 2 * (uint64_t)cur.id,
                                                     a.sink);
  };
  auto load = [&](const Row& r, uint64_t (&v)[WPL], uint64_t& last) {
    eg_src_load<WPL>(a.esrc + (uint64_t)r.plane * a.slot_e, g, r.row, v, last);
  };
  constexpr int kV = WPL;
#endif
  if constexpr (kK1Dyn) {
    // Chunks of kK1Batch consecutive list entries claimed by ticket (counter[10]; each wave comes here
    // when its k = 0 share is done, so the waves that finish it early -- the older ones, which win the
    // memory and issue arbitration -- take more of these rows). The next chunk is claimed after this
    // chunk's loads and before its stores: the wait for the ticket never covers this chunk's stores.
    (void)R;
    uint32_t tv = 0;
    if (lane == 0) tv = atomicAdd(a.counter + 10, 1u);
    for (;;) {
      const uint32_t c = uni_u32(tv) * (uint32_t)kK1Batch;
      if (c >= n) break;
      Row r[kK1Batch];
      uint64_t v[kK1Batch][kV], l[kK1Batch];
#pragma unroll
      for (int u = 0; u < kK1Batch; ++u) {
        r[u] = place_e(c + u < n ? c + u : c);
        load(r[u], v[u], l[u]);
      }
      if (lane == 0) tv = atomicAdd(a.counter + 10, 1u);
#pragma unroll
      for (int u = 0; u < kK1Batch; ++u)
        if (c + u < n) emit(r[u], v[u], l[u]);
    }
    return;
  }
  for (uint32_t k = 0; k < R; k += kK1Batch) {  // (batches as k_emit_k0)
    Row r[kK1Batch];
    uint64_t v[kK1Batch][kV], l[kK1Batch];
#pragma unroll
    for (int u = 0; u < kK1Batch; ++u) {
      r[u] = place(k + u < R ? k + u : k);
      load(r[u], v[u], l[u]);
    }
#pragma unroll
    for (int u = 0; u < kK1Batch; ++u)
      if (k + u < R) emit(r[u], v[u], l[u]);
  }
}

// The rows the prefix kernels leave to this launch: Golomb rows with mixed k (per-codeword k,
// encode_word; among the walked rows, counter[2]) and the EG row holding the plane's first 1 (with
// its inserted '0'; walked, or listed by k_scan_rows in counter[3]). One workgroup per row, one word
// per lane (wide_prefix), one LDS image per workgroup.
// One row of k_emit_rest (a whole workgroup, one word per lane; `walked`: an entry of the walk list,
// skipped unless mixed-k or its plane's first-1 row -- uniform over the workgroup). Ends with a
// workgroup barrier whenever it touched the images or sh (they are reused by the next row).
template <bool PREDICT, bool DO_G, bool DO_E>
__device__ __forceinline__ void rest_row(const FusedArgs& a, uint64_t id, bool walked, uint32_t* gimg, uint32_t* eimg,
                                         const uint32_t* s_lut, uint32_t* sh, int* sf) {
  const Geom& g = a.g;
  const int lane = lane_id(), v = (int)wave_id(), nw = blockDim.x >> 6;
  const uint32_t w = 64 * v + lane;
  constexpr uint32_t kCapBits = (kGImg - kPad) * 32;
  {
    const uint32_t plane = (uint32_t)(id / g.rows), row = (uint32_t)(id % g.rows);
    const uint32_t O = a.row_o[id];
    const uint64_t Lf = DO_G ? a.glen[id] : 0;
    const uint64_t L = Lf & kLenMask;
    const bool k0 = (Lf & kK0Row) != 0, k1 = (Lf & kK1Row) != 0;
    if (walked) {  // a walked row: skip it unless mixed or the first-1 row (uniform over the workgroup)
      const uint64_t onext = row + 1 < g.rows ? a.row_o[id + 1] : a.pones[plane];
      if (!(L && !k0 && !k1) && !(DO_E && O == 0 && onext > 0)) return;
      if (!DO_E && a.kmask && (Lf & kKMix) && L <= kCapBits) return;  // (k_emit_k01's kmix_rows writes it)
    }
    const bool gmix = DO_G && L && !k0 && !k1 && L <= kCapBits;
    uint64_t rr[1];
    if (!PREDICT && a.esrc) rr[0] = eg_src_word(a.esrc + (uint64_t)plane * a.slot_e, g, row, w);
    else resid_row<1, PREDICT>(a.planes, g, plane, row, rr, 64 * v);
    const uint64_t x = rr[0];
    const WideRow p = wide_prefix(x, w, O + row, sh);
    const bool f_here = DO_E && O == 0 && p.ones > 0;
    if (gmix) {
      uint4* z = reinterpret_cast<uint4*>(gimg);
      for (uint32_t j = threadIdx.x; j < kGImg / 4; j += blockDim.x) z[j] = make_uint4(0, 0, 0, 0);
    }
    if (f_here) {  // EG image (~R, pad-masked, EOL '1'); write_row inserts the '0' after the first 1
      const int fc = wave_min(x ? (int)(w * 64 + __builtin_clzll(x)) : INT_MAX);
      if (lane == 0) sf[v] = fc;
      if (w < g.used) {
        const uint64_t e = ~x & (w == g.used - 1 ? g.trail : ~0ull);
        eimg[2 * w] = (uint32_t)(e >> 32);
        eimg[2 * w + 1] = (uint32_t)e;
      }
      if (threadIdx.x < kPad + 1) eimg[2 * g.used + threadIdx.x] = 0;
    }
    __syncthreads();
    if (f_here) {
      if (threadIdx.x == 0) eimg[g.cols >> 5] |= 0x80000000u >> (g.cols & 31);  // EOL '1'
      __syncthreads();
      int fcol = INT_MAX;
      for (int u = 0; u < nw; ++u) fcol = min(fcol, sf[u]);
      const uint64_t Le = (uint64_t)g.cols + 2;
      const uint64_t Ge_rel = (uint64_t)row * (g.cols + 1);
      const uint64_t cap = a.slot_e * 64;
      if (Ge_rel + Le <= cap)
        write_row(eimg, Le, (a.ebase ? a.ebase[plane] : (uint64_t)plane * cap) + Ge_rel, (int64_t)fcol + 1, a.out_e,
                  a.efrag + 2 * id, threadIdx.x, blockDim.x);
    }
    if (gmix) {
      const uint32_t arow = row * (g.cols + 1);
      const bool eol = w == g.used - 1;
      const LaneEnc e = encode_word(x, w, p.n, p.jp, arow, eol, g.cols, ByteTables{s_lut, a.lut});
      const uint32_t inc = wave_incl_sum_u32(e.len);
      if (lane == 63) sh[v] = inc;
      __syncthreads();
      uint32_t wb = 0, tot = 0;
      for (int u = 0; u < nw; ++u) {
        if (u < v) wb += sh[u];
        tot += sh[u];
      }
      const uint32_t off = wb + inc - e.len;
      if (!e.lng) {
        place_small(gimg, off, e.head, e.k0);
        place128(gimg, off + e.k0 + e.z, e.t0, e.t1, e.tlen);
      } else {
        LdsSink ls{gimg, 0, 0};
        emit_word(ls, off, x, w, p.n, p.jp, arow, eol, g.cols);
        ls.flush();
      }
      __syncthreads();
      if (threadIdx.x == 0 && tot != L) atomicOr(&a.flags[3], 1u);  // word_len disagrees with the emission
      write_row(gimg, L, gb_abs(a, id, plane), -1, a.out_g, a.gfrag + 2 * id, threadIdx.x,
                blockDim.x);
    }
    __syncthreads();  // the images and sh are reused by the next row
  }
}

template <bool PREDICT, bool DO_G, bool DO_E>
__global__ __launch_bounds__(256) void k_emit_rest(FusedArgs a) {
  __shared__ __attribute__((aligned(16))) uint32_t gimg[kGImg];
  __shared__ __attribute__((aligned(16))) uint32_t eimg[kEImg];
  __shared__ uint32_t s_lut[512];
  __shared__ uint32_t sh[16];  // (wide_prefix: up to 8 waves)
  __shared__ int sf[4];
  const int lane = lane_id(), v = (int)wave_id(), nw = blockDim.x >> 6;
#if BIC_REST_PRIO
  __builtin_amdgcn_s_setprio(BIC_REST_PRIO);  // (A/B: the listed rows' waves ahead in the issue arbitration)
#endif
  if (DO_G)
    for (uint32_t i = threadIdx.x; i < 512; i += blockDim.x) s_lut[i] = reinterpret_cast<const uint32_t*>(a.lut + 256)[i];
  __syncthreads();
  // the scan's list (first-1 rows it did not walk), then the walked rows that are mixed-k or hold
  // their plane's first 1
  const uint32_t nrest = __hip_atomic_load(a.counter + 3, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  const uint32_t nwalk = DO_G ? __hip_atomic_load(a.counter + 2, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) : 0u;
  for (uint32_t i = blockIdx.x; i < nrest + nwalk; i += gridDim.x)
    rest_row<PREDICT, DO_G, DO_E>(a, i < nrest ? a.rest_ids[i] : a.walk_ids[i - nrest], i >= nrest, gimg, eimg, s_lut,
                                  sh, sf);
  // the class kernels' path (a.cls): the LEN scan listed every row too long for an LDS image, so the
  // slow rows are written here, one wave per row, overlapping the class kernels (no k_rows_global)
  if (DO_G && !PREDICT && kSlowRest && a.cls) {
    const uint32_t nslow = __hip_atomic_load(a.slow_n, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    for (uint32_t li = blockIdx.x * nw + v; li < nslow; li += gridDim.x * nw) row_global<false>(a, a.slow_ids[li], lane);
  }
}

// the class entries' third list (BIC_KMIX: k_emit_k01's rest role), residual rows from the EG stream
template <int WPL>
__device__ __forceinline__ void kmix_row(const FusedArgs& a, uint32_t i, uint32_t* gimg, const uint32_t* s_lut) {
  const Geom& g = a.g;
  const int lane = lane_id();
  constexpr uint32_t kCapBits = (kGImg - kPad) * 32;
  const uint64_t nrows = (uint64_t)g.rows * g.nplanes;
  const uint64_t e = 2 * nrows + i;
  const uint64_t e0 = cls_ld(a, 2 * e);
  const uint32_t id = (uint32_t)e0;
  const uint64_t L = e0 >> 32;
  const uint32_t plane = id / g.rows, row = id % g.rows;
  const uint64_t Gs = cls_ld(a, 2 * e + 1);
  const uint64_t G = a.off_g ? Gs - (uint64_t)plane * a.slot_g * 64 + a.gbase[plane] * 64 : Gs;
  XSTAMP((1u << 18) + id, 0);
  const uint32_t keol = (a.glen[id] & kKEol1) ? 1u : 0u;
  uint64_t rr[WPL], ktw[WPL];
  eg_src_row<WPL>(a.esrc + (uint64_t)plane * a.slot_e, g, row, rr);
  kmix_masks<WPL>(a, id, ktw);
  XSTAMP((1u << 18) + id, 1);
  if (L > kCapBits) {  // (the LEN scan lists such rows as slow, never here: a length disagreement)
    if (lane == 0) atomicOr(&a.flags[3], 1u);
    return;
  }
  kmix_encode<WPL>(a, rr, ktw, keol, id, L, G, gimg, s_lut);
  XSTAMP((1u << 18) + id, 2);
}

// The class launch's rest role (the FusedArgs::rgrid leading workgroups of k_emit_k01, dispatched first,
// one CU slot each beside the persistent class waves): the rows whose latency would otherwise be the
// persistent waves' tail. First the rows mixing k = 0 and k = 1 (kmix_row, one wave each, claimed by
// ticket: counter[9]); then, per workgroup, the mixed rows with a codeword of k >= 2 (rest_ids,
// counter[6]; k_emit_rest's rows, ticket counter[7]); then the slow rows, one wave each. This is
// k_emit_rest on a second stream without the stream: no fork / join events around the emission.
template <int WPL>
__device__ __forceinline__ void rest_role(const FusedArgs& a, uint32_t* lds, uint32_t* s_lut, uint32_t* s_lut2) {
  __shared__ uint32_t sh[16];
  __shared__ int sf[4];
  __shared__ uint32_t tk[2];
  for (uint32_t i = threadIdx.x; i < 512; i += blockDim.x) {
    s_lut[i] = reinterpret_cast<const uint32_t*>(a.lut + 256)[kK1Table + i];  // (kmix_row: the k = 1 table)
    s_lut2[i] = reinterpret_cast<const uint32_t*>(a.lut + 256)[i];            // (rest_row: encode_word's)
  }
  __syncthreads();
  if (a.kmask) {
    const uint32_t nx = __hip_atomic_load(a.counter + 8, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    uint32_t* gimg = lds + wave_id() * kGImg;
    for (;;) {
      uint32_t t = 0;
      if (lane_id() == 0) t = atomicAdd(a.counter + 9, 1u);
      t = uni_u32((uint32_t)__shfl((int)t, 0));
      if (t >= nx) break;
      kmix_row<WPL>(a, t, gimg, s_lut);
      __builtin_amdgcn_fence(__ATOMIC_ACQ_REL, "wavefront");  // the next row reuses the LDS image
      __builtin_amdgcn_wave_barrier();
    }
    XSTAMP((1u << 19) + 8192u + blockIdx.x * 4u + wave_id(), 1);
    __syncthreads();  // (the images are the workgroup's again)
  }
  const uint32_t n = __hip_atomic_load(a.counter + 6, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  for (uint32_t it = 0;; ++it) {
    // (two ticket slots: a thread still reading the last one is never overwritten)
    if (threadIdx.x == 0) tk[it & 1] = n ? atomicAdd(a.counter + 7, 1u) : 0u;
    __syncthreads();
    const uint32_t i = tk[it & 1];
    if (i >= n) break;
    rest_row<false, true, false>(a, a.rest_ids[i], false, lds, nullptr, s_lut2, sh, sf);
  }
  if (kSlowRest) {
    const uint32_t nslow = __hip_atomic_load(a.slow_n, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    for (uint32_t li = blockIdx.x * 4 + wave_id(); li < nslow; li += a.rgrid * 4) row_global<false>(a, a.slow_ids[li], lane_id());
  }
}

// Both classes in one launch: persistent waves take their share of each list, the k = 0 rows first.
// The waves reach the byte-table rows at different times, so the copies (memory-bound) and the
// byte-table rows (issue-bound) run side by side instead of one launch after the other. (Odd waves
// starting on the k = 1 rows measured 196-198 µs against 192-193, round 4.)
template <int WPL>
#ifndef BIC_K01_OCC
#define BIC_K01_OCC 4  // a minimum of workgroups (one wave per SIMD each) per CU for k_emit_k01 (0: none;
                       // the compiler then took 133 VGPRs, three per CU)
#endif
__global__ __launch_bounds__(256, BIC_K01_OCC ? BIC_K01_OCC : 1) void k_emit_k01(FusedArgs a) {
  __shared__ __attribute__((aligned(16))) uint32_t lds[4 * kGImg];
  __shared__ uint32_t s_lut[512];
  const int lane = lane_id();
  [[maybe_unused]] const uint32_t gwv = (1u << 19) + 8192u + blockIdx.x * 4u + wave_id();  // (XSTAMP index)
  XSTAMP(gwv, 0);
  // the rest role: the grid's first rgrid workgroups, or (BIC_K01_RLAST) its last ones -- dispatched after
  // the persistent ones, so its waves are the younger ones in the SIMDs' VALU arbitration
  const uint32_t pb = kK01RLast ? gridDim.x - a.rgrid : 0u;  // the rest role's first workgroup
  if constexpr (kK01Rest) {
    if (blockIdx.x >= pb && blockIdx.x < pb + a.rgrid) {  // the rest role (k_emit_rest's rows in this launch)
      __shared__ uint32_t s_lut2[512];
      rest_role<WPL>(a, lds, s_lut, s_lut2);
      XSTAMP(gwv, 3);
      return;
    }
  }
  // (BIC_K01_PRIO: the persistent waves' VALU ahead of the rest role's, whose per-codeword rows would
  // otherwise take issue slots from the copies)
  if constexpr (kK01Prio) __builtin_amdgcn_s_setprio(2);
  uint32_t* gimg = lds + wave_id() * kGImg;
  // every wave writes the whole table itself (the same values as the others): its own reads then
  // follow its own writes, and the kernel needs no workgroup barrier
  for (uint32_t i = lane; i < 512; i += 64) s_lut[i] = reinterpret_cast<const uint32_t*>(a.lut + 256)[kK1Table + i];
  const uint32_t nb = gridDim.x - a.rgrid, nw = nb * 4;
  // (the wave index through readfirstlane: the compiler then knows i0, and every branch on it, is uniform;
  // rgrid is a multiple of 8, so block b - rgrid keeps block b's XCD)
  const uint32_t i0 = xcd_remap(blockIdx.x - (kK01RLast ? 0u : a.rgrid), nb) * 4 + wave_id();
  k0_rows<WPL>(a, i0, nw);
  XSTAMP(gwv, 1);
  k1_rows<WPL>(a, i0, nw, gimg, s_lut);
  XSTAMP(gwv, 3);
}

__global__ __launch_bounds__(1024) void k_plane_bases(FusedArgs a) {
  __shared__ uint64_t tmp[17];
  plane_bases(a, tmp);
}

// Combine the fragments of the words rows share: the row holding a shared word's first bit
// owns it and ORs in the head fragments of the following rows that start inside that word.
__global__ __launch_bounds__(256) void k_fixup(const uint64_t* __restrict__ boff, const uint64_t* __restrict__ len,
                                               const uint64_t* __restrict__ frag, uint64_t* __restrict__ out,
                                               const uint64_t* __restrict__ boff2, const uint64_t* __restrict__ len2,
                                               const uint64_t* __restrict__ frag2, uint64_t* __restrict__ out2,
                                               uint32_t rows, uint64_t nrows, uint32_t second,
                                               const uint64_t* __restrict__ gbase = nullptr, uint64_t slot_bits = 0,
                                               const uint64_t* __restrict__ efix = nullptr, uint64_t* eout = nullptr,
                                               uint64_t eslot = 0, uint32_t enp = 0, uint32_t* zc = nullptr,
                                               uint64_t* zr = nullptr, uint64_t zn = 0) {
  eg_fix_bit(efix, eout, eslot, enp);  // (EG source: after every reader of the residual rows)
  if (zr) {  // single / two-pass encoder: its counters and 2 zn look-back records cleared for the next call
    const uint64_t zi = (uint64_t)blockIdx.x * 256 + threadIdx.x;
    if (zi < zn) {
      zr[zi] = 0;
      zr[zn + zi] = 0;
    }
    if (blockIdx.x == 0 && threadIdx.x < 64) zc[threadIdx.x] = 0;
  }
  // blocks [second, ...) serve the second stream (EG) when both streams are written
  if (blockIdx.x >= second) {
    boff = boff2;
    len = len2;
    frag = frag2;
    out = out2;
    gbase = nullptr;
  }
  const uint64_t id = (uint64_t)(blockIdx.x >= second ? blockIdx.x - second : blockIdx.x) * 256 + threadIdx.x;
  if (id >= nrows) return;
  const uint64_t pend = (id / rows + 1) * (uint64_t)rows;
  // gbase: the first stream's offsets are slot-relative, its planes packed from word gbase[plane]
  const uint64_t sft = gbase ? gbase[id / rows] * 64 - (id / rows) * slot_bits : 0;
  // every load this row usually needs is issued at once (the row, its two fragments, the next row's
  // offset, length and head fragment): one memory round trip instead of three dependent ones
  const bool nx = id + 1 < pend;
  const uint64_t G = boff[id] + sft, L = len[id] & kLenMask;  // (the staged encoder's glen carries row flags)
  const uint64_t f0 = frag[2 * id], f1 = frag[2 * id + 1];
  const uint64_t G1 = nx ? boff[id + 1] + sft : 0, L1 = nx ? len[id + 1] & kLenMask : 0, h1 = nx ? frag[2 * id + 2] : 0;
  if (L == 0) return;
  const uint64_t wt = (G + L - 1) >> 6, wh = G >> 6;
  const uint64_t wb = wt * 64;
  if (wb < G) return;                     // the word's first bit belongs to an earlier row
  if (wb + 64 <= G + L) return;           // a whole word of this row: already stored
  uint64_t v = (wh == wt) ? f0 : f1;
  if (!nx || L1 == 0 || G1 >= wb + 64) {
    out[wt] = bswap64(v);
    return;
  }
  v |= h1;
  for (uint64_t r2 = id + 2; r2 < pend; ++r2) {
    if ((len[r2] & kLenMask) == 0 || boff[r2] + sft >= wb + 64) break;
    v |= frag[2 * r2];
  }
  out[wt] = bswap64(v);
}

// the fixup of any row encoder that leaves its shared words as fragments (bic_egad.hip)
void launch_fixup_rows(hipStream_t s, const uint64_t* boff, const uint64_t* len, const uint64_t* frag, uint64_t* out,
                       uint32_t rows, uint64_t nrows) {
  const uint32_t grid = (uint32_t)((nrows + 255) / 256);
  k_fixup<<<grid, 256, 0, s>>>(boff, len, frag, out, boff, len, frag, out, rows, nrows, 0xffffffffu);
}

// ------------------------------------------------------------------------------------
// walked rows whose k = 1 masks the walk stores (kmix_rows; the others stay the rest role's): 4 Mi mask
// words, 32 MiB (C3: 16,384 rows, against ~1,400 walked)
static uint32_t kmask_rows(const Geom& g) {
  const uint64_t n = (uint64_t)g.rows * g.nplanes;
  return (uint32_t)std::min<uint64_t>(n, std::max<uint64_t>(64, (4ull << 20) / g.used));
}

size_t fused_scratch_bytes(const Geom& g) {
  const size_t n = (size_t)g.rows * g.nplanes;
  return 256 + n * 8 * 2 + n * 8 * 10 + n * kMaxStrips * (16 + 4 + 4) + n * 4 * 4 + 1024 + (size_t)g.nplanes * 8 * 4 + 64 +
         n * 16 * 3 + 64 + 512 +  // (cls: three lists, sink)
         n * 4 + (size_t)kmask_rows(g) * g.used * 8 + 64;  // (row_wi, kmask)
}

FusedScratch carve_fused_scratch(void* base, const Geom& g) {
  const size_t n = (size_t)g.rows * g.nplanes;
  char* p = reinterpret_cast<char*>(base);
  FusedScratch fs;
  fs.counter = reinterpret_cast<uint32_t*>(p);
  fs.ones_rec = reinterpret_cast<uint64_t*>(p + 256);
  fs.bits_rec = fs.ones_rec + n;
  fs.zero_bytes = 256 + n * 16;
  uint64_t* q = fs.bits_rec + n;
  fs.gboff = q; q += n;
  fs.glen = q; q += n;
  fs.gfrag = q; q += 2 * n;
  fs.gslow = q; q += n;
  fs.eboff = q; q += n;
  fs.elen = q; q += n;
  fs.efrag = q; q += 2 * n;
  fs.slow_ids = q; q += n;
  fs.krec = reinterpret_cast<int4*>(q);
  fs.kpos = reinterpret_cast<uint32_t*>(fs.krec + n * kMaxStrips);
  fs.sones = fs.kpos + n * kMaxStrips;
  fs.row_o = fs.sones + n * kMaxStrips;
  fs.walk_ids = fs.row_o + n;
  fs.rest_ids = fs.walk_ids + n;
  fs.walk_o = fs.rest_ids + n;
  {
    uintptr_t e = reinterpret_cast<uintptr_t>(fs.walk_o + n);
    e = (e + 7) & ~(uintptr_t)7;
    fs.pones = reinterpret_cast<uint64_t*>(e);
    fs.gbase = fs.pones + g.nplanes;
    fs.ebase = fs.gbase + g.nplanes;
    fs.efix = fs.ebase + g.nplanes;
    fs.cls = fs.efix + g.nplanes;
    fs.sink = fs.cls + 6 * n;
    fs.kmask = fs.sink + 64;
    fs.kcap = kmask_rows(g);
    fs.row_wi = reinterpret_cast<uint32_t*>(fs.kmask + (size_t)fs.kcap * g.used);
  }
  fs.ns = 1;
  fs.counted = false;
  fs.slow_n = fs.counter + 1;  // zeroed with the counter
  return fs;
}

bool fused_supported(const Geom& g) { return g.used <= 256; }

#ifdef BIC_STAMPS
int read_stamps(uint64_t* host, size_t n) {
  return hipMemcpyFromSymbol(host, HIP_SYMBOL(g_stamps), n * 8, 0, hipMemcpyDeviceToHost) == hipSuccess ? 0 : 3;
}
#endif

void launch_fused(hipStream_t s, const Geom& g, const uint64_t* planes, const uint64_t* lut, int predict,
                  const FusedScratch& fs,
                  uint64_t* out_g, uint64_t slot_g, uint64_t* bits_g, uint64_t* out_e, uint64_t slot_e,
                  uint64_t* bits_e, uint32_t* flags, int mode, int stage) {
  if (stage == kFusedPrep) {
    // the staged encoder's count pass zeroes its counters itself (kZeroWords, launch_row_ones /
    // launch_gray_rows)
    // (single / two-pass: not when the previous call's k_fixup left them zero)
    if (mode != kEncStaged && !fs.zero_ready) (void)launch_fill(s, fs.counter, 0, fs.zero_bytes);
    return;
  }
  const bool single_pass = mode == kEncSingle;
  FusedArgs a{g, planes, lut, fs.counter, fs.ones_rec, fs.bits_rec, fs.gboff, fs.glen, fs.gfrag, fs.gslow,
              fs.eboff, fs.elen, fs.efrag, fs.row_o, fs.sones, fs.krec, fs.kpos, fs.counted ? fs.ns : 1u, fs.walk_ids, fs.rest_ids, fs.slow_n, fs.slow_ids, out_g, slot_g, bits_g, out_e, slot_e,
              bits_e, flags};
  a.pones = fs.pones;
  a.walk_o = fs.walk_o;
  a.gbase = fs.gbase;
  a.off_g = out_g ? fs.off_g : nullptr;
  a.off_e = out_e ? fs.off_e : nullptr;
  a.ebase = a.off_e ? fs.ebase : nullptr;
  a.index = out_g ? fs.index : nullptr;
  // EG source (bic_encode_gray without planes): the count pass wrote the EG stream, the emission is
  // Golomb's alone and reads the residual rows from it
  const bool es = mode == kEncStaged && fs.eg_src && out_e && !a.off_e && !predict;
  a.esrc = es ? out_e : nullptr;
  a.efix = es ? fs.efix : nullptr;
  a.cls = es && out_g && !fs.eg_src_one ? fs.cls : nullptr;
  a.sink = fs.sink;
  // the walk stores the k = 1 masks of mixed rows for kmix_rows (class kernels' path only)
  // (k_emit_k01's rest role writes kKMix rows; or k_emit_known itself, planes in and Golomb alone)
  a.kmask = (a.cls && kKMixRows && kK01Rest) || (kKnownMix && !es && out_g && !out_e && mode == kEncStaged) ? fs.kmask
                                                                                                            : nullptr;
  a.row_wi = fs.row_wi;
  a.kcap = fs.kcap;
#ifdef BIC_STAMPS
  a.known = getenv("BIC_KNOWN") && getenv("BIC_KNOWN")[0] == '1';
#endif
  const uint64_t nrows = (uint64_t)g.rows * g.nplanes;
  const uint32_t grid = (uint32_t)((g.rows + kTileRows - 1) / kTileRows * (uint64_t)g.nplanes);  // one per tile
  const uint32_t egrid = (uint32_t)((nrows + kTileRows - 1) / kTileRows);                       // one per 8 rows
  const bool dg = out_g != nullptr, de = out_e != nullptr && !es;  // de: the emission writes EG
  const uint32_t fgrid = (uint32_t)((nrows + 255) / 256);
  if (stage == kFusedFinish) {
    // a fixed small grid walks the list of LDS-overflow rows (usually empty); block 0 also clears
    // the EG source's one bit per plane (eg_fix_bit)
    // (a.cls: k_emit_rest wrote the slow rows; single pass: k_encode_rows did)
    if ((dg && !single_pass && (!a.cls || !kSlowRest)) || (!dg && es)) {
      if (predict) k_rows_global<true><<<dg ? 256 : 1, 256, 0, s>>>(a);
      else k_rows_global<false><<<dg ? 256 : 1, 256, 0, s>>>(a);
    }
    if (!dg && !de) return;
    k_fixup<<<dg && de ? 2 * fgrid : fgrid, 256, 0, s>>>(dg ? fs.gboff : fs.eboff, dg ? fs.glen : fs.elen,
                                                        dg ? fs.gfrag : fs.efrag, dg ? out_g : out_e,
                                                        fs.eboff, fs.elen, fs.efrag, out_e, g.rows, nrows,
                                                        dg && de ? fgrid : 0xffffffffu,
                                                        dg && mode == kEncStaged ? a.off_g ? fs.gbase : nullptr : nullptr,
                                                        slot_g * 64, dg ? a.efix : nullptr, out_e, slot_e, g.nplanes,
                                                        fs.counter, mode != kEncStaged ? fs.ones_rec : nullptr, nrows);
    return;
  }
  const int wpl = g.used <= 64 ? 1 : (g.used <= 128 ? 2 : 4);
  if (mode == kEncStaged) {
    if (stage == kFusedPrefix) {
      if (!fs.counted) launch_row_ones(s, g, planes, predict, fs.sones, fs.krec, fs.kpos, fs.counter);
      const uint32_t sgrid = (g.rows + kScanChunk - 1) / kScanChunk * g.nplanes;
      if (dg) k_scan_rows<true, true><<<sgrid, 1024, 0, s>>>(a);
      else k_scan_rows<true, false><<<sgrid, 1024, 0, s>>>(a);
      if (dg) {
        const uint32_t wwv = (kWalkSplit * g.used + 63) / 64;  // k_row_walk: waves per row (<= 8)
        if (predict) k_row_walk<true><<<kWalkWaves / wwv, 64 * wwv, 0, s>>>(a);
        else k_row_walk<false><<<kWalkWaves / wwv, 64 * wwv, 0, s>>>(a);
        k_scan_rows<false, false><<<sgrid, 1024, 0, s>>>(a);  // (+ the row index)
      }
      // packed output: the planes' start words (the rows' Golomb offsets stay slot-relative: gb_abs)
      // -- as the LEN scan's last workgroup instead, its device-scope release fences (an L2 write-back
      // per workgroup) made C4's prefix 99 -> 153 us
      if (a.off_g || a.off_e) k_plane_bases<<<1, 1024, 0, s>>>(a);
      return;
    }
    if (!dg && !de) return;  // EG source without Golomb: the count pass and the ONES scan wrote it all
    // persistent grids (more rows per wave when the image is larger)
    static thread_local int cus = 0;
    if (!cus) {
      int dev = 0;
      (void)hipGetDevice(&dev);
      (void)hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev);
      if (cus <= 0) cus = 256;
    }
    // one resident wave set: as many workgroups per CU as the instance's registers and LDS allow
    // (WPL = 4: <= 128 VGPRs, 4; WPL = 1: 7), queried once per instance
    auto occ_of = [](const void* fn) {
      int occ = 0;
      if (hipOccupancyMaxActiveBlocksPerMultiprocessor(&occ, fn, 64 * kEmitWaves, 0) != hipSuccess || occ < 1) occ = 4;
      return std::min(occ, 8);
    };
    auto egrid_of = [&](int occ) {
      return (uint32_t)std::min<uint64_t>((nrows + kEmitWaves - 1) / kEmitWaves, (uint64_t)cus * (uint32_t)occ);
    };
    // k_emit_rest (listed rows, latency bound: few workgroups) first, on the aux stream when there
    // is one, so that it can overlap the main launch, which skips the listed rows' parts
    const uint32_t nwv = (g.used + 63) / 64;  // waves per row in k_emit_rest
    const uint32_t rgrid = (uint32_t)std::min<uint64_t>(nrows, (uint64_t)cus * 32 / nwv);  // 32 waves per CU (16: C4 +6 us; 4: C3 +30 us -- the listed rows are latency-bound)
    // (bic_prof_*: events around the main emission kernel alone, on its stream s -- the roofline kernel's
    // launch, without the fork / join of the second stream; null: not timed)
    auto main_ev = [&](hipEvent_t e) {
      if (e && hipEventRecord(e, s) == hipSuccess && e == fs.ev_main1 && fs.ev_main_rec) *fs.ev_main_rec = true;
    };
    // (the class kernels' path with the rest role inside k_emit_k01: one launch, no second stream)
    const bool one_launch = es && a.cls && kK01Rest;
    hipStream_t rs = s;
    if (!one_launch && kRestAux && fs.aux && fs.ev_fork && fs.ev_join && hipEventRecord(fs.ev_fork, s) == hipSuccess &&
        hipStreamWaitEvent(fs.aux, fs.ev_fork, 0) == hipSuccess)
      rs = fs.aux;
#define BIC_EMIT1(W, P, DG, DE, ES)                                                                    \
  {                                                                                                  \
    k_emit_rest<P, DG, DE><<<rgrid, 64 * nwv, 0, rs>>>(a);                                           \
    static const int occ_ = occ_of(reinterpret_cast<const void*>(&k_emit_known<W, P, DG, DE, ES>));  \
    main_ev(fs.ev_main0);                                                                            \
    k_emit_known<W, P, DG, DE, ES><<<egrid_of(occ_), 64 * kEmitWaves, 0, s>>>(a);                    \
    main_ev(fs.ev_main1);                                                                            \
  }
#define BIC_EMIT(W, P)                                                                                \
  if (dg && de) BIC_EMIT1(W, P, true, true, false) else if (dg) BIC_EMIT1(W, P, true, false, false) else BIC_EMIT1(W, P, false, true, false)
    if (predict) {
      if (wpl == 1) { BIC_EMIT(1, true); } else if (wpl == 2) { BIC_EMIT(2, true); } else { BIC_EMIT(4, true); }
    } else if (es && !a.cls) {  // Golomb alone, the residual rows from the EG stream, one kernel
      if (wpl == 1) { BIC_EMIT1(1, false, true, false, true); } else if (wpl == 2) { BIC_EMIT1(2, false, true, false, true); }
      else { BIC_EMIT1(4, false, true, false, true); }
    } else if (es) {  // Golomb alone, the residual rows from the EG stream: one kernel per row class
#define BIC_EMITC(W)                                                                                      \
  {                                                                                                    \
    static const int o_ = occ_of(reinterpret_cast<const void*>(&k_emit_k01<W>));                      \
    if (one_launch) {                                                                                  \
      a.rgrid = kK01Rg ? kK01Rg : std::max(8u, (uint32_t)cus / 8 * 8);                                 \
      main_ev(fs.ev_main0);                                                                            \
      const uint32_t pg = (uint32_t)std::min<uint64_t>((nrows + 3) / 4, kK01Rg ? (uint64_t)cus * o_ - a.rgrid   \
                                                                                 : (uint64_t)cus * std::max(1, o_ - 1)); \
      k_emit_k01<W><<<a.rgrid + pg, 256, 0, s>>>(a);                                                   \
      main_ev(fs.ev_main1);                                                                            \
    } else {                                                                                           \
      k_emit_rest<false, true, false><<<rgrid, 64 * nwv, 0, rs>>>(a);                                  \
      main_ev(fs.ev_main0);                                                                            \
      k_emit_k01<W><<<egrid_of(o_), 256, 0, s>>>(a);                                                   \
      main_ev(fs.ev_main1);                                                                            \
    }                                                                                                  \
  }
      if (wpl == 1) { BIC_EMITC(1); } else if (wpl == 2) { BIC_EMITC(2); } else { BIC_EMITC(4); }
#undef BIC_EMITC
    } else {
      if (wpl == 1) { BIC_EMIT(1, false); } else if (wpl == 2) { BIC_EMIT(2, false); } else { BIC_EMIT(4, false); }
    }
#undef BIC_EMIT
#undef BIC_EMIT1
    if (rs != s && (hipEventRecord(fs.ev_join, rs) != hipSuccess || hipStreamWaitEvent(s, fs.ev_join, 0) != hipSuccess))
      (void)hipStreamSynchronize(rs);  // no join event: wait on the host rather than race
    return;
  }
  if (stage == kFusedPrefix) return;
  const dim3 blk(64 * kTileRows);
#define BIC_PASSES(W, P, DG, DE)                                                        \
  if (single_pass) {                                                                    \
    k_encode_rows<W, P, DG, DE><<<grid, blk, 0, s>>>(a);                                \
  } else {                                                                              \
    k_len_rows<W, P, DG, DE><<<grid, blk, 0, s>>>(a);                                   \
    k_emit_rows<W, P, DG, DE><<<egrid, blk, 0, s>>>(a);                                 \
  }
#define BIC_CODERS(W, P)                                                                \
  if (dg && de) { BIC_PASSES(W, P, true, true) }                                        \
  else if (dg) { BIC_PASSES(W, P, true, false) }                                        \
  else { BIC_PASSES(W, P, false, true) }
  if (predict) {
    if (wpl == 1) { BIC_CODERS(1, true) } else if (wpl == 2) { BIC_CODERS(2, true) } else { BIC_CODERS(4, true) }
  } else {
    if (wpl == 1) { BIC_CODERS(1, false) } else if (wpl == 2) { BIC_CODERS(2, false) } else { BIC_CODERS(4, false) }
  }
#undef BIC_CODERS
#undef BIC_PASSES
}

}  // namespace bic
