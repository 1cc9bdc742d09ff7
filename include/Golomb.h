// Golomb.h -- adaptive Golomb coder state of the reference API (drop-in for
// /root/reference/src/Golomb.h): a fresh coder has k = 1 and no history; after n samples with
// sum A, k = min{k >= 0 : n << k >= A} (32-bit unsigned arithmetic).
#ifndef Predictor_RLS_Golomb_h
#define Predictor_RLS_Golomb_h

namespace bic {
struct coder_state;  // GPU bridge (bic_gpu.h) reads and advances the state of whole planes
}

class Golomb {
 public:
  Golomb() : accumulatedError(0), samples(0), k(1) {}

 protected:
  unsigned accumulatedError;  // A: sum of the samples coded so far
  unsigned samples;           // n
  unsigned k;                 // parameter for the next sample
  friend struct bic::coder_state;
};

#endif
