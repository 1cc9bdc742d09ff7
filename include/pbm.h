// pbm.h -- binary PBM (P4) I/O of the reference API (drop-in for /root/reference/src/pbm.h).
// Raster rows are ceil(cols/8) bytes, MSB = leftmost pixel, which is also the bit order of a
// binary_matrix word: read/write move whole bytes, not single pixels.
#ifndef PBM_H
#define PBM_H

#include <cstdio>

#include "binmat.h"

// Status codes, values as in the reference (pbm.h:8-16).
typedef enum error_code {
  PBM_OK = 0,
  PBM_READ_ERROR = 1,
  PBM_FILE_NOT_FOUND = 2,
  PBM_INVALID_HEADER = 3,
  PBM_INVALID_DATA = 4,
  PBM_WRITE_ERROR = 5,
  PBM_INVALID_FORMAT = 6
} ErrorCode;

// "P4", width, height; like the reference, the height is read with a trailing-whitespace
// pattern that also consumes whitespace-valued raster bytes (SURVEY.md §4 hazard 2).
ErrorCode read_pbm_header(FILE* fimg, idx_t& rows, idx_t& cols);
// Clears A, then fills its rows from the raster; PBM_INVALID_DATA on a short raster (the rows
// read so far are kept).
ErrorCode read_pbm_data(FILE* fimg, binary_matrix& A);
ErrorCode write_pbm(binary_matrix& A, FILE* fimg);

#endif
