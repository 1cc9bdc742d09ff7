// coding.h -- code-length helpers of the reference API (drop-in for
// /root/reference/src/coding.h). enumerative_codelength is computed in closed form here
// (bic_enum_codelength), not through GSL's gsl_sf_lnchoose; see DESIGN.md for where the two can
// round differently.
#ifndef CODING_H
#define CODING_H

#include "binmat.h"

#define COSMOS_2E 5.436563656918090181591196596855297684669
#define COSMOS_2PI 6.283185307179586231995926937088370323181
#define COSMOS_2EPI 17.07946844534713193297648103907704353333
#define COSMOS_LOG2E 1.442695040888963387004650940070860087872
#define COSMOS_LOG2PI 1.651496129472318719066947778628673404455
#define COSMOS_LOG2EPI 4.0941911703612818840269937936682254076

// log2 C(n, r) bits; 0 for r = 0.
double enumerative_codelength(const unsigned n, const unsigned r);
// n H(r/n) + log2(n)/2 bits (the two-part universal code).
double universal_codelength(const unsigned n, const unsigned r);

#endif
