// coders.cpp -- GolombCoder (GolombCoder.h) and EG / EGCoder (eg.h): the reference's per-sample
// state machines (GolombCoder.cpp:13-34, eg.cpp:2-37). They count bits like the reference; bit
// streams for whole planes come from the GPU encoder (bic_gpu.h).
#include <cassert>

#include "GolombCoder.h"
#include "eg.h"

void GolombCoder::binaryEncode(unsigned sample, unsigned kk) {
  assert(kk < sizeof(int) * 8);
  bitcount += kk + (sample >> kk) + 1;  // k-bit binary part, unary quotient, stop bit
}

void GolombCoder::codeSample(unsigned sample) {
  binaryEncode(sample, k);
  ++samples;
  accumulatedError += sample;
  // smallest k with n * 2^k >= A, in the coder's 32-bit arithmetic
  unsigned kk = 0;
  while ((samples << kk) < accumulatedError) ++kk;
  k = kk;
}

namespace {
// JPEG-LS run-length order table J[0..31] (ITU-T T.87 A.7.1.2), the reference's EGLUT
constexpr unsigned char kRunOrder[32] = {0, 0, 0, 0, 1, 1, 1, 1, 2, 2, 2,  2,  3,  3,  3,  3,
                                         4, 4, 5, 5, 6, 6, 7, 7, 8, 9, 10, 11, 12, 13, 14, 15};
}  // namespace

// The reference lets lutIndex reach 32 and then reads one entry past its table (eg.cpp:5-7);
// here the index saturates at the last entry.
void EG::incBlockSize() {
  if (lutIndex < 31) ++lutIndex;
  g = kRunOrder[lutIndex];
  blockSize = 1u << g;
}

void EG::decBlockSize() {
  if (lutIndex > 0) --lutIndex;
  g = kRunOrder[lutIndex];
  blockSize = 1u << g;
}

void EGCoder::codeRun(int len, bool eol) {
  // `len >= blockSize` compares as unsigned in the reference (eg.cpp:22)
  unsigned left = (unsigned)len;
  while (left >= blockSize) {  // one '1' per full block
    left -= blockSize;
    ++bitcount;
  }
  if (eol) {
    ++bitcount;  // '1': run ended by the end of the row
  } else {
    bitcount += g + 1;  // '0' + g-bit remainder
    decBlockSize();
  }
}
