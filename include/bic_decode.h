// bic_decode.h -- decoders of this build's plane streams, used to prove that
// the GPU streams are decodable and lossless. Host code: decoding an adaptive Golomb stream is
// a serial walk by construction.
//
// Stream grammar (bic.h): for every row, in raster order, one codeword per 1-pixel (the zeros
// before it) and one end-of-row codeword (the trailing zeros, possibly 0).
//   Golomb: codeword = k-bit binary part, (s >> k) zeros, '1'; k from the state of Golomb.h
//           (read order of the reference decoder, GolombDecoder.cpp:15-23, unsigned samples).
//   EG (as written, eg.cpp:20-37 with block size fixed at 1): '1' per zero, then '1' at the end
//           of a row or '0' before a 1-pixel, followed by one more '0' at the plane's first 1.
// The med residual R(0,0) is always 0 (pred.cpp never writes it), so a predicted stream does
// not carry P(0,0): unmed() takes it as side information.
#ifndef BIC_DECODE_H
#define BIC_DECODE_H

#include <stdint.h>

#include "Golomb.h"
#include "binmat.h"

namespace bic {

class BitReader {
 public:
  BitReader(const uint8_t* bytes, uint64_t bits) : p_(bytes), bits_(bits), pos_(0) {}
  bool empty() const { return pos_ >= bits_; }
  uint64_t position() const { return pos_; }
  // next bit; reading past the end sets overrun() and returns 0
  int bit() {
    if (pos_ >= bits_) {
      over_ = true;
      return 0;
    }
    const int b = (p_[pos_ >> 3] >> (7 - (pos_ & 7))) & 1;
    ++pos_;
    return b;
  }
  uint32_t bits(unsigned k) {
    uint32_t v = 0;
    for (unsigned i = 0; i < k; ++i) v = (v << 1) | (uint32_t)bit();
    return v;
  }
  bool overrun() const { return over_; }

 private:
  const uint8_t* p_;
  uint64_t bits_, pos_;
  bool over_ = false;
};

// Inverse of GolombCoder::codeSample with the same state update.
class GolombStreamDecoder : public Golomb {
 public:
  explicit GolombStreamDecoder(BitReader* r) : Golomb(), r_(r) {}
  unsigned decodeSample();

 private:
  BitReader* r_;
};

// Residual plane of a stream into R (allocated rows x cols): coder = BIC_CODER_GOLOMB,
// BIC_CODER_EG or BIC_CODER_EG_ADAPTIVE. Returns 0, or -1 if the stream is malformed or its length is not `bits`.
int decode_plane(const uint8_t* stream, uint64_t bits, int coder, binary_matrix& R);

// P from its med residual R (pred.h) and P(0,0); P allocated like R.
void unmed(const binary_matrix& R, bool p00, binary_matrix& P);

}  // namespace bic

#endif
