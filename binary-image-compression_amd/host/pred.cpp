// pred.cpp -- med() of the reference API (include/pred.h; reference pred.cpp:3-15) on the GPU.
#include "pred.h"

#include <cstdio>
#include <cstdlib>

#include "bic_gpu.h"

void med(const binary_matrix& P, binary_matrix& pP) {
  const int rc = bic::default_device().med(P, pP);
  if (rc != BIC_OK) {
    std::fprintf(stderr, "med: %s\n", bic_strerror(rc));
    std::abort();
  }
}
