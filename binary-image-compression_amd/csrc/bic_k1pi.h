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
#else
#define BIC_UNROLL _Pragma("GCC unroll 8")
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
