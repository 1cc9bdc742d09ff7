// util.h -- helpers of the reference API (drop-in for /root/reference/src/util.h).
#ifndef UTIL_H
#define UTIL_H

#include <utility>

#include "binmat.h"

typedef std::pair<idx_t, idx_t> aux_t;

// Tiles the rows of D (each a vectorised sqrt(cols) x sqrt(cols) patch) into one PBM image.
void render_mosaic(const binary_matrix& D, const char* fname);
// Counting sort of s[0..n) by .first (small non-negative keys); equal keys end up in reverse
// input order, as in the reference.
void counting_sort(aux_t* s, idx_t n);
// Writes A as P4 to a file; -2 if it cannot be opened.
int write_pbm(binary_matrix& A, const char* fname);

#endif
