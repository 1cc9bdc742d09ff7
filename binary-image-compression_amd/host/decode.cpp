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
