/* tests/cpp/gsl_shim/gsl/gsl_sf_gamma.h -- TEST INFRASTRUCTURE ONLY.
 *
 * GSL is not installed in this image. The reference's compress*_test.cpp drivers include this header
 * for one function, gsl_sf_lnchoose (compress7_test.cpp:7,25-28; compress_test.cpp:7,36-39). For the
 * drop-in build (tests/test_dropin_compress.py: the drivers compiled unchanged against include/ and
 * libbicpp.so) this header supplies that one function. It is used for this build's side only: no
 * reference build is made with it. The expected output is assembled from the reference's own loop
 * objects (oracle/ref_capi.cpp) with the same lnchoose, so both sides see the same enumL values.
 *
 * ln C(n, m) as a left-to-right sum of log((n - m + i) / i), i = 1..m. Only the symmetry step
 * m = min(m, n - m) matches GSL's gsl_sf_lnchoose_e; GSL itself takes differences of lnfact, so the two
 * can differ in the last ulps. The sum is reproducible from Python's math.log (libm's log), which
 * tests/test_dropin_compress.py uses for the expected lines. Parity of enumL with a GSL-linked build is
 * therefore unpinned: a last-ulp difference that flips a ceil in enumL would not be caught here. */
#ifndef BIC_TEST_GSL_SF_GAMMA_H
#define BIC_TEST_GSL_SF_GAMMA_H
#include <math.h>

static inline double gsl_sf_lnchoose(unsigned int n, unsigned int m) {
  if (m > n) return NAN; /* GSL: domain error */
  if (2 * m > n) m = n - m;
  double s = 0.0;
  for (unsigned int i = 1; i <= m; ++i) s += log((double)(n - m + i) / (double)i);
  return s;
}

#endif
