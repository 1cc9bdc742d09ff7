// coding.cpp -- include/coding.h (reference: coding.cpp:19-32).
#include "coding.h"

#include <cmath>

#include "bic.h"

double enumerative_codelength(const unsigned n, const unsigned r) { return bic_enum_codelength(n, r); }

double universal_codelength(const unsigned n, const unsigned r) {
  const double half_log = 0.5 * std::log2((double)n);
  if (r == 0 || r >= n) return half_log;
  const double p = (double)r / (double)n;
  return double(n) * (-p * std::log2(p) - (1.0 - p) * std::log2(1.0 - p)) + half_log;
}
