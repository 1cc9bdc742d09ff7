// pred.h -- the med ("3-neighbour XOR") predictor of the reference (pred.cpp:3-15; the same
// function is bilinear_predictor in coding.cpp:5-17 and a local med in compress7_test.cpp:44-56).
// The reference ships no header for it; callers declared it themselves.
#ifndef PRED_H
#define PRED_H

#include "binmat.h"

// pP(i,j) = P(i-1,j-1) ^ P(i,j-1) ^ P(i-1,j) ^ P(i,j) with out-of-range neighbours 0, except
// that pP(0,0) and the pad bits of pP are left as they were. Runs on the GPU (bic_med_residual);
// aborts with a message if no gfx950 device is available.
void med(const binary_matrix& P, binary_matrix& pP);

#endif
