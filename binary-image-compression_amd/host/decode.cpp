// decode.cpp -- include/bic_decode.h.
#include "bic_decode.h"

#include "bic.h"

namespace bic {

unsigned GolombStreamDecoder::decodeSample() {
  const unsigned low = r_->bits(k);
  unsigned high = 0;
  while (!r_->bit()) {
    if (r_->overrun()) return 0;
    ++high;
  }
  const unsigned s = (high << k) | low;
  ++samples;
  accumulatedError += s;
  unsigned kk = 0;
  while ((samples << kk) < accumulatedError) ++kk;
  k = kk;
  return s;
}

int decode_plane(const uint8_t* stream, uint64_t bits, int coder, binary_matrix& R) {
  const idx_t rows = R.get_rows(), cols = R.get_cols();
  R.clear();
  BitReader in(stream, bits);
  if (coder == BIC_CODER_GOLOMB) {
    GolombStreamDecoder dec(&in);
    for (idx_t i = 0; i < rows; ++i) {
      idx_t j = 0;
      for (;;) {
        const idx_t s = dec.decodeSample();
        if (in.overrun() || j + s > cols) return -1;
        if (j + s == cols) break;  // end-of-row codeword
        R.set(i, j + s);
        j += s + 1;
      }
    }
  } else if (coder == BIC_CODER_EG) {
    bool first = true;
    for (idx_t i = 0; i < rows; ++i) {
      for (idx_t j = 0; j < cols; ++j) {
        if (in.bit()) continue;  // a zero pixel
        R.set(i, j);
        if (first) {  // the g = 1 remainder bit of the plane's first non-EOL run
          if (in.bit()) return -1;
          first = false;
        }
      }
      if (!in.bit()) return -1;  // end of row
    }
  } else if (coder == BIC_CODER_EG_ADAPTIVE) {
    // eg.cpp:41-55 (the #if 0 decoder): '1' = a full block (len += blockSize, incBlockSize), until
    // a '0' and the g-bit remainder (then decBlockSize) -- or until the blocks pass the columns left,
    // which is the end-of-row '1'. The index saturates at 31 as in the encoder (bic.h).
    static const unsigned J[32] = {0, 0, 0, 0, 1, 1, 1, 1, 2, 2, 2, 2, 3, 3, 3, 3,
                                   4, 4, 5, 5, 6, 6, 7, 7, 8, 9, 10, 11, 12, 13, 14, 15};
    int idx = 0;
    unsigned g = 1, bs = 1;  // eg.h:9
    for (idx_t i = 0; i < rows; ++i) {
      idx_t j = 0;
      for (;;) {
        const uint64_t maxlen = (uint64_t)(cols - j);
        uint64_t len = 0;
        bool eol = false;
        while (in.bit()) {
          if (in.overrun()) return -1;
          len += bs;
          if (len > maxlen) {
            eol = true;
            break;
          }
          if (idx < 31) ++idx;
          g = J[idx];
          bs = 1u << g;
        }
        if (eol) break;
        len += in.bits(g);
        if (idx > 0) --idx;
        g = J[idx];
        bs = 1u << g;
        if (in.overrun() || len >= maxlen) return -1;
        R.set(i, j + (idx_t)len);
        j += (idx_t)len + 1;
      }
    }
  } else {
    return -1;
  }
  return (in.overrun() || in.position() != bits) ? -1 : 0;
}

void unmed(const binary_matrix& R, bool p00, binary_matrix& P) {
  const idx_t rows = R.get_rows(), cols = R.get_cols(), wpr = R.get_blocks_per_row();
  if (rows == 0 || cols == 0) return;
  const block_t* r = R.raw_blocks();
  block_t* p = P.raw_blocks();
  const idx_t used = cols % 64;
  const block_t tail = used ? ~0ul << (64 - used) : ~0ul;
  for (idx_t i = 0; i < rows; ++i) {
    block_t carry = 0, up_prev = 0;  // P(i, column before this word), U(column before)
    for (idx_t w = 0; w < wpr; ++w) {
      const block_t m = w + 1 == wpr ? tail : ~0ul;
      const block_t u = i ? p[(i - 1) * wpr + w] : 0;
      // P(i,j) ^ P(i,j-1) = R(i,j) ^ U(j) ^ U(j-1) =: T(j); P is the running XOR of T
      block_t t = (r[i * wpr + w] & m) ^ u ^ ((u >> 1) | (up_prev << 63));
      if (i == 0 && w == 0) t = (t & ~(1ul << 63)) | ((block_t)p00 << 63);
      t ^= t >> 1;
      t ^= t >> 2;
      t ^= t >> 4;
      t ^= t >> 8;
      t ^= t >> 16;
      t ^= t >> 32;
      if (carry) t = ~t;
      t &= m;
      p[i * wpr + w] = t;
      carry = t & 1;
      up_prev = u;
    }
  }
}

}  // namespace bic
