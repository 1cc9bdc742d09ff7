// GolombCoder.h -- Golomb-power-of-two sample coder of the reference API (drop-in for
// /root/reference/src/GolombCoder.h). codeSample(s) costs k + (s >> k) + 1 bits: the k-bit
// binary part, s >> k zeros, a terminating '1' (the order GolombDecoder.cpp:17-21 reads).
// Like the reference, this class only counts bits; whole planes are coded to an actual bit
// stream on the GPU through bic_gpu.h, which also advances a coder's state.
#ifndef __compresoreeg__GolombCoder__
#define __compresoreeg__GolombCoder__

#include <cmath>

#include "Golomb.h"

using namespace std;  // the reference header exports it; kept for source compatibility

class GolombCoder : public Golomb {
 public:
  GolombCoder() : Golomb(), bitcount() {}
  void codeSample(unsigned);
  long bitcount;

 private:
  void binaryEncode(unsigned, unsigned);
};

#endif
