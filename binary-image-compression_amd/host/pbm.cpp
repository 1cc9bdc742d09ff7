// pbm.cpp -- P4 I/O (include/pbm.h), following /root/reference/src/pbm.cpp:4-77 for what is
// read, what is returned and what ends up in the matrix. A raster row of ceil(cols/8) bytes has
// the bit order of the matrix words, so rows move as big-endian 8-byte groups.
#include "pbm.h"

#include <vector>

namespace {

inline block_t load_be(const unsigned char* p, size_t n) {  // n <= 8 bytes, missing bytes = 0
  block_t w = 0;
  for (size_t b = 0; b < 8; ++b) w = (w << 8) | (b < n ? p[b] : 0);
  return w;
}

inline void store_be(block_t w, unsigned char* p, size_t n) {
  for (size_t b = 0; b < n; ++b) p[b] = (unsigned char)(w >> (56 - 8 * b));
}

// mask of the bits of the last word of a row that hold pixels
inline block_t row_tail_mask(idx_t cols) {
  const idx_t used = cols % BITS_PER_BLOCK;
  return used ? ONES << (BITS_PER_BLOCK - used) : ONES;
}

}  // namespace

ErrorCode read_pbm_header(FILE* fimg, idx_t& rows, idx_t& cols) {
  if (fgetc(fimg) != 'P') return PBM_INVALID_HEADER;
  if (fgetc(fimg) != '4') return PBM_INVALID_HEADER;
  int width = 0, height = 0;
  int got = fscanf(fimg, " %d", &width);
  if (width == 0 || got == 0) return PBM_INVALID_HEADER;
  got = fscanf(fimg, " %d ", &height);  // the trailing ' ' skips ALL whitespace (hazard 2)
  if (height == 0 || got == 0) return PBM_INVALID_HEADER;
  rows = (idx_t)(long)height;
  cols = (idx_t)(long)width;
  return PBM_OK;
}

ErrorCode read_pbm_data(FILE* fimg, binary_matrix& A) {
  A.clear();
  const idx_t rows = A.get_rows(), cols = A.get_cols();
  if (rows == 0) return cols ? PBM_INVALID_DATA : PBM_OK;  // pbm.cpp:48 (no pixel was read)
  const size_t row_bytes = (cols + 7) / 8;
  const idx_t bpr = A.get_blocks_per_row();
  const block_t tail = row_tail_mask(cols);
  std::vector<unsigned char> buf(row_bytes);
  block_t* data = A.raw_blocks();
  for (idx_t i = 0; i < rows; ++i) {
    const size_t got = fread(buf.data(), 1, row_bytes, fimg);
    block_t* row = data + i * bpr;
    for (idx_t w = 0; w < bpr; ++w) {
      const size_t b0 = 8 * w;
      row[w] = b0 < got ? load_be(&buf[b0], got - b0 < 8 ? got - b0 : 8) : 0;
    }
    if (bpr) row[bpr - 1] &= tail;
    if (got < row_bytes) return PBM_INVALID_DATA;
  }
  return PBM_OK;
}

ErrorCode write_pbm(binary_matrix& A, FILE* fimg) {
  const idx_t rows = A.get_rows(), cols = A.get_cols();
  fprintf(fimg, "P4\n%lu %lu\n", cols, rows);
  const size_t row_bytes = (cols + 7) / 8;
  const idx_t bpr = A.get_blocks_per_row();
  const block_t tail = row_tail_mask(cols);
  std::vector<unsigned char> buf(row_bytes + 8);
  const block_t* data = A.raw_blocks();
  for (idx_t i = 0; i < rows; ++i) {
    const block_t* row = data + i * bpr;
    for (idx_t w = 0; w < bpr; ++w) store_be(w + 1 == bpr ? row[w] & tail : row[w], &buf[8 * w], 8);
    fwrite(buf.data(), 1, row_bytes, fimg);
  }
  return PBM_OK;
}
