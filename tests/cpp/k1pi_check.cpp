// k1pi_check.cpp -- TEST (CPU): the k = 1 rows' backward-parity encoder of bic_fused.hip k1_rows
// (BIC_K1_PI), composed on the host exactly as the kernel composes it -- 64 lanes, lane l holding the
// row's words l*WPL .. l*WPL + WPL - 1, the ballot / nearest-right-lane exchange for zeta, the wave scan
// of the lanes' lengths, the words' 128-bit strings OR'd into a row image at their offsets -- over the
// helpers of csrc/bic_k1pi.h that the kernel uses. Reads rows of residual words from stdin, writes each
// row's bit string ('0'/'1' characters, one line per row): tests/test_k1pi_host.py compares them with
// the oracle's Golomb rows whose codewords all have k = 1.
//
// stdin: cols nrows, then nrows * ceil(cols / 64) words (hex); mode 'm' (rows mixing k = 0 and k = 1):
// each row's words, then its k = 1 masks (one per word, hex), then the end-of-row codeword's k.
#include <cstdint>
#include <cstdio>
#include <cstdlib>
#include <vector>

#include "bic_k1pi.h"

using namespace bic;

constexpr uint64_t kMsb = 1ull << 63;

// the strided layout of k_emit_known (emit_known_row): lane l holds words t * 64 + l
static std::vector<int> encode_row_strided(const std::vector<uint64_t>& row, uint32_t cols, const uint32_t* T) {
  const uint32_t used = (cols + 63) / 64;
  const int WPL = used <= 64 ? 1 : (used <= 128 ? 2 : 4);
  const uint32_t tail = cols & 63u;
  const uint64_t trail = ~0ull << (63 - (cols - 1) % 64);
  std::vector<uint64_t> xt(64 * WPL), Zm(64 * WPL), rr(64 * WPL);
  std::vector<uint32_t> lead(64 * WPL, 0);
  std::vector<uint64_t> m1(WPL, 0);
  for (int t = 0; t < WPL; ++t)
    for (int lane = 0; lane < 64; ++lane) {
      const uint32_t w = t * 64 + lane;
      const uint64_t valid = w < used ? (w == used - 1 ? trail : ~0ull) : 0ull;
      const uint64_t r = w < used ? row[w] & valid : 0ull;
      const int i = t * 64 + lane;
      rr[i] = r;
      xt[i] = r | ((w == used - 1 && tail) ? (kMsb >> tail) : 0ull);
      Zm[i] = ~xt[i] & valid;
      lead[i] = xt[i] ? (uint32_t)__builtin_clzll(xt[i]) & 1u : 0u;
      if (xt[i]) m1[t] |= 1ull << lane;
    }
  std::vector<uint32_t> zeta(64 * WPL);
  uint32_t carry = 0;
  for (int t = WPL - 1; t >= 0; --t) {
    for (int lane = 0; lane < 64; ++lane) {
      const uint64_t nm = m1[t] & ~((lane == 63 ? 0ull : (2ull << lane)) - 1ull);
      zeta[t * 64 + lane] = nm ? lead[t * 64 + __builtin_ctzll(nm)] : carry;
    }
    if (m1[t]) carry = lead[t * 64 + __builtin_ctzll(m1[t])];
  }
  const uint32_t first_r = carry;
  std::vector<int> bits(1, (int)first_r);
  for (int t = 0; t < WPL; ++t)
    for (int lane = 0; lane < 64; ++lane) {
      const uint32_t w = t * 64 + lane;
      if (w >= used) continue;
      const int i = t * 64 + lane;
      const uint64_t Pi = k1_pi(xt[i], Zm[i], zeta[i]);
      uint64_t hi = 0, lo = 0, A, B;
      const uint32_t L = (w == used - 1 && tail) ? k1_word_last(rr[i], Pi, tail, hi, lo) : k1_word_full(rr[i], Pi, T, hi, lo);
      left128(hi, lo, L ? L : 128u, A, B);
      for (uint32_t b = 0; b < L; ++b) bits.push_back((int)(((b < 64 ? A : B) >> (63 - (b & 63))) & 1u));
    }
  if (!tail) bits.push_back(1);
  return bits;
}

static std::vector<int> encode_row(const std::vector<uint64_t>& row, uint32_t cols, const uint32_t* T) {
  const uint32_t used = (cols + 63) / 64;
  const int WPL = used <= 64 ? 1 : (used <= 128 ? 2 : 4);
  const uint32_t tail = cols & 63u;
  const uint64_t trail = ~0ull << (63 - (cols - 1) % 64);
  // per lane state
  std::vector<uint64_t> xt(64 * WPL), Zm(64 * WPL), rr(64 * WPL);
  std::vector<uint32_t> lead(64, 0), anyl(64, 0);
  for (int lane = 0; lane < 64; ++lane)
    for (int t = 0; t < WPL; ++t) {
      const uint32_t w = (uint32_t)lane * WPL + t;
      const uint64_t valid = w < used ? (w == used - 1 ? trail : ~0ull) : 0ull;
      const uint64_t r = w < used ? row[w] & valid : 0ull;
      rr[lane * WPL + t] = r;
      xt[lane * WPL + t] = r | ((w == used - 1 && tail) ? (kMsb >> tail) : 0ull);
      Zm[lane * WPL + t] = ~xt[lane * WPL + t] & valid;
    }
  for (int lane = 0; lane < 64; ++lane)
    for (int t = WPL - 1; t >= 0; --t)
      if (xt[lane * WPL + t]) {
        lead[lane] = (uint32_t)__builtin_clzll(xt[lane * WPL + t]) & 1u;
        anyl[lane] = 1;
      }
  uint64_t m1 = 0;
  for (int lane = 0; lane < 64; ++lane) m1 |= (uint64_t)anyl[lane] << lane;
  const uint32_t lf = m1 ? lead[__builtin_ctzll(m1)] : 0u;
  std::vector<uint64_t> A(64 * WPL), B(64 * WPL);
  std::vector<uint32_t> lw(64 * WPL), lsum(64, 0);
  for (int lane = 0; lane < 64; ++lane) {
    const uint64_t nm = m1 & ~((lane == 63 ? 0ull : (2ull << lane)) - 1ull);
    uint32_t zc = nm ? lead[__builtin_ctzll(nm)] : 0u;
    std::vector<uint32_t> zeta(WPL);
    for (int t = WPL - 1; t >= 0; --t) {
      zeta[t] = zc;
      if (xt[lane * WPL + t]) zc = (uint32_t)__builtin_clzll(xt[lane * WPL + t]) & 1u;
    }
    for (int t = 0; t < WPL; ++t) {
      const uint32_t w = (uint32_t)lane * WPL + t;
      const uint64_t Pi = k1_pi(xt[lane * WPL + t], Zm[lane * WPL + t], zeta[t]);
      uint64_t hi = 0, lo = 0;
      uint32_t L = 0;
      if (w < used) {
        if (w == used - 1 && tail) L = k1_word_last(rr[lane * WPL + t], Pi, tail, hi, lo);
        else L = k1_word_full(rr[lane * WPL + t], Pi, T, hi, lo);
      }
      left128(hi, lo, L ? L : 128u, A[lane * WPL + t], B[lane * WPL + t]);
      lw[lane * WPL + t] = L;
      lsum[lane] += L;
    }
  }
  uint32_t total = 1;
  std::vector<uint32_t> lane_off(64);
  for (int lane = 0; lane < 64; ++lane) {
    lane_off[lane] = total;
    total += lsum[lane];
  }
  if (!tail) ++total;
  std::vector<int> bits(total, 0);
  bits[0] = (int)(lf && m1);
  for (int lane = 0; lane < 64; ++lane) {
    uint32_t off = lane_off[lane];
    for (int t = 0; t < WPL; ++t) {
      const uint32_t L = lw[lane * WPL + t];
      for (uint32_t i = 0; i < L; ++i) {
        const uint64_t word = i < 64 ? A[lane * WPL + t] : B[lane * WPL + t];
        bits[off + i] |= (int)((word >> (63 - (i & 63))) & 1u);
      }
      off += L;
    }
  }
  if (!tail) bits[total - 1] = 1;
  return bits;
}

// rows whose codewords mix k = 0 and k = 1 (bic_fused.hip kmix_rows): lane l holds words l*WPL ..,
// kt[w] the k = 1 1s of word w (the walk's masks), keol the end-of-row codeword's k
static std::vector<int> encode_row_mixed(const std::vector<uint64_t>& row, const std::vector<uint64_t>& ktw, uint32_t keol,
                                         uint32_t cols, const uint32_t* T) {
  const uint32_t used = (cols + 63) / 64;
  const int WPL = used <= 64 ? 1 : (used <= 128 ? 2 : 4);
  const uint32_t tail = cols & 63u;
  const uint64_t trail = ~0ull << (63 - (cols - 1) % 64);
  std::vector<uint64_t> xt(64 * WPL), Zm(64 * WPL), rr(64 * WPL), kt(64 * WPL);
  std::vector<uint32_t> lead(64, 0), leadk(64, 0), anyl(64, 0);
  for (int lane = 0; lane < 64; ++lane)
    for (int t = 0; t < WPL; ++t) {
      const uint32_t w = (uint32_t)lane * WPL + t;
      const uint64_t valid = w < used ? (w == used - 1 ? trail : ~0ull) : 0ull;
      const uint64_t r = w < used ? row[w] & valid : 0ull;
      const uint64_t eb = (w == used - 1 && tail) ? (kMsb >> tail) : 0ull;
      const int i = lane * WPL + t;
      rr[i] = r;
      xt[i] = r | eb;
      Zm[i] = ~xt[i] & valid;
      kt[i] = (w < used ? ktw[w] & r : 0ull) | (keol ? eb : 0ull);
    }
  for (int lane = 0; lane < 64; ++lane)
    for (int t = WPL - 1; t >= 0; --t)
      if (xt[lane * WPL + t]) {
        const int i = lane * WPL + t;
        const int cz = __builtin_clzll(xt[i]);
        lead[lane] = (uint32_t)cz & 1u;
        leadk[lane] = (uint32_t)(kt[i] >> (63 - cz)) & 1u;
        anyl[lane] = 1;
      }
  uint64_t m1 = 0;
  for (int lane = 0; lane < 64; ++lane) m1 |= (uint64_t)anyl[lane] << lane;
  const uint32_t lf = m1 ? lead[__builtin_ctzll(m1)] : 0u;
  const uint32_t kk0 = m1 ? leadk[__builtin_ctzll(m1)] : keol;
  std::vector<uint64_t> A(64 * WPL), B(64 * WPL);
  std::vector<uint32_t> lw(64 * WPL), lsum(64, 0);
  for (int lane = 0; lane < 64; ++lane) {
    const uint64_t nm = m1 & ~((lane == 63 ? 0ull : (2ull << lane)) - 1ull);
    uint32_t zc = nm ? lead[__builtin_ctzll(nm)] : 0u;
    uint32_t kc = nm ? leadk[__builtin_ctzll(nm)] : keol;
    std::vector<uint32_t> zeta(WPL), nk(WPL);
    for (int t = WPL - 1; t >= 0; --t) {
      zeta[t] = zc;
      nk[t] = kc;
      const int i = lane * WPL + t;
      if (xt[i]) {
        const int cz = __builtin_clzll(xt[i]);
        zc = (uint32_t)cz & 1u;
        kc = (uint32_t)(kt[i] >> (63 - cz)) & 1u;
      }
    }
    for (int t = 0; t < WPL; ++t) {
      const uint32_t w = (uint32_t)lane * WPL + t;
      const int i = lane * WPL + t;
      const uint64_t Pi = k1_pi(xt[i], Zm[i], zeta[t]);
      const uint64_t KK = kmix_kk(xt[i], Zm[i], kt[i], nk[t]);
      uint64_t hi = 0, lo = 0;
      uint32_t L = 0;
      if (w < used) {
        if (w == used - 1 && tail) L = kmix_word_last(rr[i], Pi, KK, nk[t], tail, hi, lo);
        else L = kmix_word_full(rr[i], Pi, KK, nk[t], T, hi, lo);
      }
      left128(hi, lo, L ? L : 128u, A[i], B[i]);
      lw[i] = L;
      lsum[lane] += L;
    }
  }
  uint32_t total = kk0;
  std::vector<uint32_t> lane_off(64);
  for (int lane = 0; lane < 64; ++lane) {
    lane_off[lane] = total;
    total += lsum[lane];
  }
  if (!tail) ++total;
  std::vector<int> bits(total, 0);
  if (kk0) bits[0] = (int)lf;
  for (int lane = 0; lane < 64; ++lane) {
    uint32_t off = lane_off[lane];
    for (int t = 0; t < WPL; ++t) {
      const uint32_t L = lw[lane * WPL + t];
      for (uint32_t i = 0; i < L; ++i) {
        const uint64_t word = i < 64 ? A[lane * WPL + t] : B[lane * WPL + t];
        bits[off + i] |= (int)((word >> (63 - (i & 63))) & 1u);
      }
      off += L;
    }
  }
  if (!tail) bits[total - 1] = 1;
  return bits;
}

// the same in bic_fused.hip kmix_rows' own layout: lane l holds words t * 64 + l, one word group at a
// time (zeta / nk from the nearest right lane of the group holding a 1, else carried from later groups)
static std::vector<int> encode_row_mixed_strided(const std::vector<uint64_t>& row, const std::vector<uint64_t>& ktw,
                                                 uint32_t keol, uint32_t cols, const uint32_t* T) {
  const uint32_t used = (cols + 63) / 64;
  const int WPL = used <= 64 ? 1 : (used <= 128 ? 2 : 4);
  const uint32_t tail = cols & 63u;
  const uint64_t trail = ~0ull << (63 - (cols - 1) % 64);
  auto ws = [&](uint32_t w, uint64_t& x, uint64_t& xt, uint64_t& Z, uint64_t& kt) {
    const uint64_t valid = w < used ? (w == used - 1 ? trail : ~0ull) : 0ull;
    const uint64_t eb = (w == used - 1 && tail) ? (kMsb >> tail) : 0ull;
    x = w < used ? row[w] & valid : 0ull;
    xt = x | eb;
    Z = ~xt & valid;
    kt = (w < used ? ktw[w] & x : 0ull) | (keol ? eb : 0ull);
  };
  std::vector<uint32_t> zb(64, 0), kb(64, 0);
  uint32_t zc = 0, kc = keol;
  for (int t = WPL - 1; t >= 0; --t) {
    uint32_t lead[64], leadk[64];
    uint64_t m1 = 0;
    for (int lane = 0; lane < 64; ++lane) {
      uint64_t x, xt, Z, kt;
      ws(t * 64 + lane, x, xt, Z, kt);
      const uint32_t cz = xt ? (uint32_t)__builtin_clzll(xt) : 0u;
      lead[lane] = cz & 1u;
      leadk[lane] = (uint32_t)(kt >> (63 - cz)) & 1u;
      if (xt) m1 |= 1ull << lane;
    }
    for (int lane = 0; lane < 64; ++lane) {
      const uint64_t nm = m1 & ~((lane == 63 ? 0ull : (2ull << lane)) - 1ull);
      zb[lane] |= (nm ? lead[__builtin_ctzll(nm)] : zc) << t;
      kb[lane] |= (nm ? leadk[__builtin_ctzll(nm)] : kc) << t;
    }
    if (m1) {
      zc = lead[__builtin_ctzll(m1)];
      kc = leadk[__builtin_ctzll(m1)];
    }
  }
  const uint32_t kk0 = kc, lf = zc;
  std::vector<int> bits;
  if (kk0) bits.push_back((int)lf);
  for (int t = 0; t < WPL; ++t)
    for (int lane = 0; lane < 64; ++lane) {
      const uint32_t w = t * 64 + lane;
      if (w >= used) continue;
      uint64_t x, xt, Z, kt;
      ws(w, x, xt, Z, kt);
      const uint32_t zt = (zb[lane] >> t) & 1u, nt = (kb[lane] >> t) & 1u;
      const uint64_t Pi = k1_pi(xt, Z, zt), KK = kmix_kk(xt, Z, kt, nt);
      uint64_t hi = 0, lo = 0, A, B;
      const bool last = w == used - 1 && tail;
      const uint32_t L = last ? kmix_word_last(x, Pi, KK, nt, tail, hi, lo) : kmix_word_full2(x, Pi, KK, nt, T, hi, lo);
      if (L != kmix_word_len(x, Z, Pi, KK, nt, last)) {
        fprintf(stderr, "kmix_word_len disagrees at word %u\n", w);
        exit(4);
      }
      left128(hi, lo, L ? L : 128u, A, B);
      for (uint32_t b = 0; b < L; ++b) bits.push_back((int)(((b < 64 ? A : B) >> (63 - (b & 63))) & 1u));
    }
  if (!tail) bits.push_back(1);
  return bits;
}

int main(int argc, char** argv) {
  const bool strided = argc > 1 && argv[1][0] == 's';
  const bool mixed = argc > 1 && (argv[1][0] == 'm' || argv[1][0] == 'n');  // each row: words, k = 1 masks, keol
  const bool mixed_strided = argc > 1 && argv[1][0] == 'n';
  uint32_t T[512];
  k1pi_build_table(T);
  unsigned cols = 0, nrows = 0;
  if (scanf("%u %u", &cols, &nrows) != 2) return 2;
  const uint32_t used = (cols + 63) / 64;
  std::vector<uint64_t> row(used);
  for (unsigned r = 0; r < nrows; ++r) {
    for (uint32_t w = 0; w < used; ++w) {
      unsigned long long v = 0;
      if (scanf("%llx", &v) != 1) return 3;
      row[w] = v;
    }
    std::vector<uint64_t> ktw(used, 0);
    unsigned keol = 0;
    if (mixed) {
      for (uint32_t w = 0; w < used; ++w) {
        unsigned long long v = 0;
        if (scanf("%llx", &v) != 1) return 3;
        ktw[w] = v;
      }
      if (scanf("%u", &keol) != 1) return 3;
    }
    const std::vector<int> b = mixed_strided ? encode_row_mixed_strided(row, ktw, keol, cols, T)
                               : mixed ? encode_row_mixed(row, ktw, keol, cols, T)
                                     : strided ? encode_row_strided(row, cols, T) : encode_row(row, cols, T);
    for (int x : b) putchar('0' + x);
    putchar('\n');
  }
  return 0;
}
