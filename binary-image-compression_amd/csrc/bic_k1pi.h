// bic_k1pi.h -- the k = 1 rows' encoder by the backward parity (bic_fused.hip k1_rows), in plain
// integer code compilable for the host as well (tests/cpp/k1pi_check.cpp checks it against the oracle on
// the CPU). Table: bic_kernels.hip build_byte_lut, u32 entries [512 + pi * 256 + byte].
#pragma once
#include <cstdint>
#if defined(__HIPCC__)
#include <hip/hip_runtime.h>
#define BIC_HDI __host__ __device__ __attribute__((always_inline)) inline
#else
#define BIC_HDI __attribute__((always_inline)) inline
#endif
#if defined(__HIPCC__) || defined(__clang__)
#define BIC_UNROLL _Pragma("unroll")
#define BIC_NOUNROLL _Pragma("unroll 1")
#else
#define BIC_UNROLL _Pragma("GCC unroll 8")
#define BIC_NOUNROLL _Pragma("GCC unroll 1")
#endif

namespace bic {

// ---- k = 1 rows by the backward parity --------------------------------------------------------
// With every codeword at k = 1 a sample s is coded (GolombCoder.cpp:13-34, this build's bit order)
// as its remainder bit r = s & 1, then s >> 1 zeros, then '1'. Read right to left that is a two-state
// transducer without look-ahead: for column c let pi(c) be the parity of the zeros right of c up to
// the next 1 (the end of the row counting as a 1). Then a 1 at c emits '1' and pi(c) (its own
// terminator, then the remainder of the run that follows it), a zero with pi(c) = 1 emits '0' (one
// per pair of zeros), a zero with pi(c) = 0 nothing; the row's output is pi(-1) (the first run's
// remainder), those column outputs in order, and the end-of-row codeword's '1'. Within a byte every
// pi follows from the byte's bits and pi of its last column, so a byte's output is one table entry
// (k1pi_table, build_byte_lut: [pi][byte] -> bits | length << 16, <= 16 bits); pi over a whole word
// is bit-parallel (k1_pi).
constexpr uint64_t kEvenPos = 0x5555555555555555ull, kOddPos = 0xAAAAAAAAAAAAAAAAull;  // bit significance
// pi of every column of a word (MSB = its first column): xt its 1s (the row's end-of-row 1 included
// when it lies inside the word), Z its zeros (valid columns only), zeta = pi of its last column's right
// neighbour context: the parity of the zeros from the word's end up to the next 1 of the row.
// A zero preceding a 1 at bit p has (b - p - 1) zeros right of it: the zeros preceding the 1s of one
// significance class are Z & ~(Z + (those 1s << 1)) (the carry ripples through the run and stops at the
// previous 1).
BIC_HDI uint64_t k1_pi(uint64_t xt, uint64_t Z, uint32_t zeta) {
  const uint64_t FE = Z & ~(Z + ((xt & kEvenPos) << 1));
  const uint64_t FO = Z & ~(Z + ((xt & kOddPos) << 1));
  uint64_t PZ = (FE & kEvenPos) | (FO & kOddPos);
  const uint64_t T = Z & ((xt & (0ull - xt)) - 1ull);  // the zeros after the word's last 1 (all of Z: no 1)
  PZ |= T & (zeta ? kEvenPos : kOddPos);
  return PZ | (xt & ((Z & ~PZ) << 1)) | (xt & (uint64_t)zeta);
}
// The output of a full word (64 valid columns, no end-of-row 1 inside): eight table entries, joined
// pairwise (<= 32 bits), by four (<= 64) and into a right-aligned 128-bit (hi, lo); returns its length.
BIC_HDI uint32_t k1_word_full(uint64_t x, uint64_t Pi, const uint32_t* T, uint64_t& hi, uint64_t& lo) {
  uint64_t q[2];
  uint32_t lq[2];
BIC_UNROLL
  for (int h = 0; h < 2; ++h) {
    const uint32_t xv = (uint32_t)(x >> (32 - 32 * h)), pv = (uint32_t)(Pi >> (32 - 32 * h));
    uint32_t b[4], l[4];
BIC_UNROLL
    for (int j = 0; j < 4; ++j) {
      const uint32_t e = T[(((pv >> (24 - 8 * j)) & 1u) << 8) | ((xv >> (24 - 8 * j)) & 0xffu)];
      b[j] = e & 0xffffu;
      l[j] = e >> 16;
    }
    const uint32_t p0 = (b[0] << l[1]) | b[1], p1 = (b[2] << l[3]) | b[3];
    const uint32_t lp1 = l[2] + l[3];
    q[h] = ((uint64_t)p0 << lp1) | p1;
    lq[h] = l[0] + l[1] + lp1;
  }
  const uint32_t lb = lq[1];
  lo = lb >= 64 ? q[1] : (q[0] << lb) | q[1];
  hi = lb >= 64 ? q[0] : (lb ? q[0] >> (64 - lb) : 0ull);
  return lq[0] + lb;
}
// The same for a word holding the row's end (valid columns < 64 or the end-of-row 1 right after it),
// column by column (one word per row at most); includes the end-of-row '1'.
BIC_HDI uint32_t k1_word_last(uint64_t x, uint64_t Pi, uint32_t nvalid, uint64_t& hi, uint64_t& lo) {
  hi = lo = 0;
  uint32_t L = 0;
  auto put = [&](uint32_t v, uint32_t n) {
    hi = (hi << n) | (lo >> (64 - n));
    lo = (lo << n) | v;
    L += n;
  };
  for (uint32_t c = 0; c < nvalid; ++c) {
    const uint32_t xb = (uint32_t)(x >> (63 - c)) & 1u, pb = (uint32_t)(Pi >> (63 - c)) & 1u;
    if (xb) put(2u | pb, 2);
    else if (pb) put(0u, 1);
  }
  put(1u, 1);
  return L;
}
// ---- rows whose codewords mix k = 0 and k = 1 (the walked rows, k_row_walk's masks) ---------------
// With kk(c) the k of the codeword column c belongs to (a zero: the codeword its run ends in; a 1: its
// own; kk(cols) the end-of-row codeword's), the forward output is: pi(-1) first when kk(0) = 1; a 1
// at c emits '1', then pi(c) when kk(c + 1) = 1 (the next codeword's remainder); a zero emits '0'
// when kk(c) = 0, or when kk(c) = 1 and pi(c) = 1; then the end-of-row '1'. kk = 1 everywhere is the
// k = 1 transducer above, kk = 0 everywhere the residual row itself (k = 0: each run's zeros and its 1).
//
// KK, the kk of every column of a word (MSB = its first column): xt its 1s (the end-of-row 1 included
// when inside the word), Z its zeros, kt the 1s of xt whose codeword has k = 1, nk the k of the first
// codeword ending after the word. Zeros take the k of the 1 ending their run: the runs before the
// k = 1 1s are Z & ~(Z + (kt << 1)) (as in k1_pi), the run leaving the word takes nk.
BIC_HDI uint64_t kmix_kk(uint64_t xt, uint64_t Z, uint64_t kt, uint32_t nk) {
  const uint64_t F = Z & ~(Z + (kt << 1));
  const uint64_t T = Z & ((xt & (0ull - xt)) - 1ull);  // the zeros after the word's last 1
  return kt | F | (nk ? T : 0ull);
}
// one column's output appended to (bits, len) (len + 2 <= 64)
BIC_HDI void kmix_col(uint32_t xb, uint32_t pb, uint32_t kb, uint32_t kn, uint64_t& bits, uint32_t& len) {
  if (xb) {
    bits = (bits << 1) | 1u;
    ++len;
    if (kn) {
      bits = (bits << 1) | pb;
      ++len;
    }
  } else if (!kb || pb) {
    bits <<= 1;
    ++len;
  }
}
// a full word (64 valid columns, no end-of-row 1 inside): byte by byte, a byte whose columns and the
// column after it all have kk = 1 through the k = 1 table T, all kk = 0 verbatim, the others column by
// column; joined into a right-aligned 128-bit (hi, lo); kkn = kk of the column after the word
BIC_HDI uint32_t kmix_word_full(uint64_t x, uint64_t Pi, uint64_t KK, uint32_t kkn, const uint32_t* T, uint64_t& hi,
                                uint64_t& lo) {
  hi = lo = 0;
  uint32_t L = 0;
  // KK shifted one column left, the word's kkn after its last column: bit c of KN = kk(c + 1)
  const uint64_t KN = (KK << 1) | (uint64_t)kkn;
  // (a loop, not unrolled: these rows are rare, and eight unrolled three-way bytes cost the kernel
  // ~25 registers)
BIC_NOUNROLL
  for (int j = 0; j < 8; ++j) {
    const uint32_t sh = 56 - 8 * j;
    const uint32_t xb = (uint32_t)(x >> sh) & 0xffu, kb = (uint32_t)(KK >> sh) & 0xffu, kn = (uint32_t)(KN >> sh) & 0xffu;
    uint64_t b;
    uint32_t l;
    if (kb == 0xffu && kn == 0xffu) {
      const uint32_t e = T[(((uint32_t)(Pi >> sh) & 1u) << 8) | xb];
      b = e & 0xffffu;
      l = e >> 16;
    } else if (kb == 0 && kn == 0) {
      b = xb;
      l = 8;
    } else {
      b = 0;
      l = 0;
      const uint32_t pv = (uint32_t)(Pi >> sh) & 0xffu;
BIC_NOUNROLL
      for (int c = 7; c >= 0; --c)
        kmix_col((xb >> c) & 1u, (pv >> c) & 1u, (kb >> c) & 1u, (kn >> c) & 1u, b, l);
    }
    hi = l ? (hi << l) | (lo >> (64 - l)) : hi;
    lo = (lo << l) | b;
    L += l;
  }
  return L;
}
// The same, with the eight table reads issued together (one LDS round trip per word, as k1_word_full):
// every byte's entry is read, used when the byte and the column after it all have kk = 1; a byte with
// kk = 0 throughout is verbatim; the bytes where kk changes (a few per mixed row) go column by column.
BIC_HDI uint32_t kmix_word_full2(uint64_t x, uint64_t Pi, uint64_t KK, uint32_t kkn, const uint32_t* T, uint64_t& hi,
                                 uint64_t& lo) {
  const uint64_t KN = (KK << 1) | (uint64_t)kkn;
  uint32_t b[8], l[8];
  uint32_t mixed = 0;  // bit j: byte j goes column by column
BIC_UNROLL
  for (int j = 0; j < 8; ++j) {
    const uint32_t sh = 56 - 8 * j;
    const uint32_t xb = (uint32_t)(x >> sh) & 0xffu, kb = (uint32_t)(KK >> sh) & 0xffu, kn = (uint32_t)(KN >> sh) & 0xffu;
    const uint32_t e = T[(((uint32_t)(Pi >> sh) & 1u) << 8) | xb];
    const bool one = kb == 0xffu && kn == 0xffu, zero = kb == 0 && kn == 0;
    b[j] = one ? (e & 0xffffu) : xb;
    l[j] = one ? (e >> 16) : 8u;
    mixed |= (one || zero) ? 0u : (1u << j);
  }
  if (mixed) {
BIC_NOUNROLL
    for (int j = 0; j < 8; ++j) {
      if (!((mixed >> j) & 1u)) continue;
      const uint32_t sh = 56 - 8 * j;
      const uint32_t xb = (uint32_t)(x >> sh) & 0xffu, kb = (uint32_t)(KK >> sh) & 0xffu, kn = (uint32_t)(KN >> sh) & 0xffu;
      const uint32_t pv = (uint32_t)(Pi >> sh) & 0xffu;
      uint64_t bb = 0;
      uint32_t ll = 0;
BIC_NOUNROLL
      for (int c = 7; c >= 0; --c) kmix_col((xb >> c) & 1u, (pv >> c) & 1u, (kb >> c) & 1u, (kn >> c) & 1u, bb, ll);
      // (constant indices below: select the slot instead of indexing the arrays dynamically)
BIC_UNROLL
      for (int q = 0; q < 8; ++q)
        if (q == j) {
          b[q] = (uint32_t)bb;
          l[q] = ll;
        }
    }
  }
  // joined as k1_word_full: pairs (<= 32 bits), fours (<= 64), the two halves into 128 bits
  uint64_t q[2];
  uint32_t lq[2];
BIC_UNROLL
  for (int h = 0; h < 2; ++h) {
    const uint32_t* bh = b + 4 * h;
    const uint32_t* lh = l + 4 * h;
    const uint32_t p0 = (bh[0] << lh[1]) | bh[1], p1 = (bh[2] << lh[3]) | bh[3];
    const uint32_t lp1 = lh[2] + lh[3];
    q[h] = ((uint64_t)p0 << lp1) | p1;
    lq[h] = lh[0] + lh[1] + lp1;
  }
  const uint32_t lb = lq[1];
  lo = lb >= 64 ? q[1] : (q[0] << lb) | q[1];
  hi = lb >= 64 ? q[0] : (lb ? q[0] >> (64 - lb) : 0ull);
  return lq[0] + lb;
}
// the word holding the row's end (nvalid < 64 columns, or the end-of-row 1 right after it), column by
// column; includes the end-of-row '1' (KK's bit at column nvalid: the end-of-row codeword's k)
BIC_HDI uint32_t kmix_word_last(uint64_t x, uint64_t Pi, uint64_t KK, uint32_t kkn, uint32_t nvalid, uint64_t& hi,
                                uint64_t& lo) {
  hi = lo = 0;
  uint32_t L = 0;
  const uint64_t KN = (KK << 1) | (uint64_t)kkn;
  for (uint32_t c = 0; c < nvalid; ++c) {
    uint64_t b = 0;
    uint32_t l = 0;
    kmix_col((uint32_t)(x >> (63 - c)) & 1u, (uint32_t)(Pi >> (63 - c)) & 1u, (uint32_t)(KK >> (63 - c)) & 1u,
             (uint32_t)(KN >> (63 - c)) & 1u, b, l);
    hi = l ? (hi << l) | (lo >> (64 - l)) : hi;
    lo = (lo << l) | b;
    L += l;
  }
  hi = (hi << 1) | (lo >> 63);
  lo = (lo << 1) | 1u;
  return L + 1;
}

// the length kmix_word_full / kmix_word_last return, by popcounts (Z: the word's valid zeros; the
// end-of-row 1, when inside the word, neither in x nor in Z): 1s, the remainders after them, zeros
// with k = 0, zeros with k = 1 and pi = 1 (+ 1 for the end-of-row '1': eol)
BIC_HDI uint32_t kmix_word_len(uint64_t x, uint64_t Z, uint64_t Pi, uint64_t KK, uint32_t kkn, bool eol) {
  const uint64_t KN = (KK << 1) | (uint64_t)kkn;
  return (uint32_t)(__builtin_popcountll(x) + __builtin_popcountll(x & KN) + __builtin_popcountll(Z & ~KK) +
                    __builtin_popcountll(Z & KK & Pi)) + (eol ? 1u : 0u);
}

// left-align a right-aligned 128-bit string of L bits (place128_64's operands)
BIC_HDI void left128(uint64_t hi, uint64_t lo, uint32_t L, uint64_t& A, uint64_t& B) {
  const uint32_t sh = 128 - L;
  if (sh >= 64) {
    A = lo << (sh - 64);
    B = 0;
  } else if (sh) {
    A = (hi << sh) | (lo >> (64 - sh));
    B = lo << sh;
  } else {
    A = hi;
    B = lo;
  }
}

// the [pi][byte] table (host): bits (right-aligned, <= 16) | length << 16; pi = the parity of the zeros
// right of the byte's last column up to the next 1 (build_byte_lut stores it at u32 entry 512)
inline void k1pi_build_table(uint32_t* T) {
  for (unsigned pe = 0; pe < 2; ++pe)
    for (unsigned v = 0; v < 256; ++v) {
      unsigned pi[8], z = pe;
      for (int c = 7; c >= 0; --c) {
        pi[c] = z;
        z = ((v >> (7 - c)) & 1u) ? 0u : (z ^ 1u);
      }
      uint32_t bits = 0, len = 0;
      for (int c = 0; c < 8; ++c) {
        if ((v >> (7 - c)) & 1u) {
          bits = (bits << 2) | 2u | pi[c];
          len += 2;
        } else if (pi[c]) {
          bits <<= 1;
          len += 1;
        }
      }
      T[pe * 256 + v] = bits | (len << 16);
    }
}

}  // namespace bic
