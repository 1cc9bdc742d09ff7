// binmat.cpp -- binary_matrix (include/binmat.h), written word-at-a-time against the
// semantics of /root/reference/src/binmat.cpp. Behaviour that callers can observe is kept,
// including the reference's edge effects (tile reads that run into the next row, the stride of
// col_weight, the unimplemented A^t*B^t product). Where the reference is undefined (shifts by
// 64, reads past the buffer) this file defines the result; DESIGN.md lists each case.
#include "binmat.h"

#include <cassert>
#include <iomanip>

namespace {

constexpr idx_t kBits = BITS_PER_BLOCK;

inline idx_t popcount(block_t v) { return (idx_t)__builtin_popcountl(v); }
inline bool parity(block_t v) { return __builtin_parityl(v) != 0; }

// v << s for s in [0, 64]; 64 gives 0 (the reference's `x << (64 - 0)` is undefined)
inline block_t shl(block_t v, idx_t s) { return s >= kBits ? 0 : v << s; }

idx_t g_grid_width = 10;  // binmat.cpp:618

}  // namespace

void set_grid_width(idx_t g) { g_grid_width = g; }

// ---- construction ---------------------------------------------------------------------------

void binary_matrix::shape(idx_t r, idx_t c) {
  rows = r;
  cols = c;
  len = r * c;
  blocks_per_row = (c + kBits - 1) / kBits;
  data_blocks = blocks_per_row * r;
  last_bit_offset = (c - 1) % kBits;  // c = 0 wraps to 63, as in binmat.cpp:146
  trail_mask = ONES << (kBits - 1 - last_bit_offset);
  last_block = blocks_per_row - 1;
}

binary_matrix::binary_matrix(idx_t _rows, idx_t _cols) {
  shape(_rows, _cols);
  data = new block_t[data_blocks]();  // zeroed: the reference leaves it uninitialised
}

void binary_matrix::allocate(idx_t _rows, idx_t _cols) {
  shape(_rows, _cols);
  data = new block_t[data_blocks]();  // zeroed: the reference leaves it uninitialised
}

binary_matrix::binary_matrix(const binary_matrix& o)
    : rows(o.rows), cols(o.cols), len(o.len), last_bit_offset(o.last_bit_offset),
      data_blocks(o.data_blocks), blocks_per_row(o.blocks_per_row), last_block(o.last_block),
      data(new block_t[o.data_blocks]), trail_mask(o.trail_mask) {
  if (data_blocks) std::memcpy(data, o.data, data_blocks * sizeof(block_t));
}

binary_matrix& binary_matrix::operator=(const binary_matrix& A) {
  if (this == &A) return *this;
  delete[] data;
  rows = A.rows;
  cols = A.cols;
  len = A.len;
  last_bit_offset = A.last_bit_offset;
  data_blocks = A.data_blocks;
  blocks_per_row = A.blocks_per_row;
  last_block = A.last_block;
  data = A.data;  // shared, not copied (binmat.cpp:180-184)
  trail_mask = A.trail_mask;
  return *this;
}

binary_matrix binary_matrix::get_copy() const { return binary_matrix(*this); }

void binary_matrix::copy_to(binary_matrix& B) const {
  if (data_blocks) std::memcpy(B.data, data, data_blocks * sizeof(block_t));
}

// ---- fills ------------------------------------------------------------------------------------

void binary_matrix::clear() {
  if (rows * cols != 0) std::memset(data, 0x00, rows * blocks_per_row * sizeof(block_t));
}

void binary_matrix::set() {
  if (rows * cols != 0) std::memset(data, 0xff, rows * blocks_per_row * sizeof(block_t));
}

void binary_matrix::flip() {
  if (rows * cols == 0) return;
  for (idx_t k = 0; k < data_blocks; ++k) data[k] = ~data[k];
}

// ---- reductions -------------------------------------------------------------------------------

idx_t binary_matrix::weight() const {
  if (rows * cols == 0) return 0;
  idx_t w = 0;
  for (idx_t i = 0; i < rows; ++i) w += row_weight(i);
  return w;
}

idx_t binary_matrix::row_weight(idx_t i) const {
  assert(i < rows);
  if (rows == 0) return 0;
  const block_t* r = data + i * blocks_per_row;
  idx_t w = 0;
  for (idx_t j = 0; j + 1 < blocks_per_row; ++j) w += popcount(r[j]);
  if (blocks_per_row) w += popcount(r[last_block] & trail_mask);
  return w;
}

idx_t binary_matrix::col_weight(idx_t j) const {
  assert(j < cols);
  if (cols == 0) return 0;
  // as written (binmat.cpp:84-90): the row pointer advances by blocks_per_row words while the
  // loop index, compared against `rows`, advances by blocks_per_row too
  idx_t w = 0;
  for (idx_t r = 0; r * blocks_per_row < rows; ++r) w += (word(r, j) & bit(j)) ? 1 : 0;
  return w;
}

bool binary_matrix::sum() const {
  if (rows * cols == 0) return false;
  bool s = false;
  for (idx_t i = 0; i < rows; ++i) s ^= row_sum(i);
  return s;
}

bool binary_matrix::row_sum(idx_t i) const {
  assert(i < rows);
  if (cols == 0) return false;
  const block_t* r = data + i * blocks_per_row;
  block_t acc = r[last_block] & trail_mask;
  for (idx_t j = 0; j + 1 < blocks_per_row; ++j) acc ^= r[j];
  return parity(acc);
}

bool binary_matrix::col_sum(idx_t j) const {
  bool s = false;
  for (idx_t i = 0; i < rows; ++i) s ^= (word(i, j) & bit(j)) != 0;
  return s;
}

// ---- rows, columns, vectorisation -----------------------------------------------------------

binary_matrix binary_matrix::get_row(const idx_t i) const {
  assert(i < rows);
  binary_matrix r(1, cols);
  copy_row_to(i, r);
  return r;
}

void binary_matrix::copy_row_to(const idx_t i, binary_matrix& B) const {
  assert(i < rows);
  std::memcpy(B.data, data + i * blocks_per_row, blocks_per_row * sizeof(block_t));
}

void binary_matrix::set_row(const idx_t i, const binary_matrix& src) {
  assert(i < rows);
  std::memcpy(data + i * blocks_per_row, src.data, blocks_per_row * sizeof(block_t));
}

binary_matrix binary_matrix::get_col(const idx_t j) const {
  assert(j <= cols);
  binary_matrix c(1, rows);
  copy_col_to(j, c);
  return c;
}

void binary_matrix::copy_col_to(const idx_t j, binary_matrix& B) const {
  assert(j <= cols);
  B.clear();
  for (idx_t i = 0; i < rows; ++i)
    if (word(i, j) & bit(j)) B.data[i / kBits] |= bit(i);
}

void binary_matrix::set_col(const idx_t j, const binary_matrix& src) {
  assert(j <= cols);
  for (idx_t i = 0; i < rows; ++i) set(i, j, (src.data[i / kBits] & bit(i)) != 0);
}

binary_matrix binary_matrix::get_vectorized() const {
  binary_matrix v(1, rows * cols);
  copy_vectorized_to(v);
  return v;
}

// Row i lands at bit offset i*cols of the 1 x rows*cols vector (binmat.cpp:306-320).
void binary_matrix::copy_vectorized_to(binary_matrix& v) const {
  v.clear();
  for (idx_t i = 0; i < rows; ++i) {
    const idx_t start = cols * i;
    const idx_t sh = start % kBits;
    idx_t d = start / kBits;
    for (idx_t j = 0; j < blocks_per_row; ++j, ++d) {
      const block_t w = get_block(i, j);
      if (d < v.data_blocks) v.data[d] |= w >> sh;
      if (d + 1 < v.data_blocks) v.data[d + 1] = shl(w, kBits - sh);
    }
  }
}

// Inverse of copy_vectorized_to: destination row i takes bits [i*cols, i*cols + 64*bpr) of src,
// so the pad bits of each row receive the first bits of the next one (binmat.cpp:322-341).
void binary_matrix::set_vectorized(const binary_matrix& src) {
  clear();
  for (idx_t i = 0; i < rows; ++i) {
    const idx_t start = cols * i;
    const idx_t sh = start % kBits;
    idx_t s = start / kBits;
    for (idx_t j = 0; j < blocks_per_row; ++j, ++s) {
      block_t w = s < src.data_blocks ? src.data[s] << sh : 0;
      if (sh && s + 1 < src.data_blocks) w |= src.data[s + 1] >> (kBits - sh);
      data[i * blocks_per_row + j] |= w;
    }
  }
}

void binary_matrix::transpose_to(binary_matrix& B) const {
  assert(rows == B.cols);
  assert(cols == B.rows);
  for (idx_t j = 0; j < cols; ++j) {
    block_t* dst = B.data + j * B.blocks_per_row;
    std::memset(dst, 0, B.blocks_per_row * sizeof(block_t));
    for (idx_t i = 0; i < rows; ++i)
      if (word(i, j) & bit(j)) dst[i / kBits] |= bit(i);
  }
}

// The reference allocates rows x cols here and then asserts (binmat.cpp:210-214); that only
// works for square matrices, for which both agree.
binary_matrix binary_matrix::get_transposed() const {
  binary_matrix T(cols, rows);
  transpose_to(T);
  return T;
}

// ---- tiles ------------------------------------------------------------------------------------

binary_matrix binary_matrix::get_submatrix(const idx_t i0, const idx_t i1, const idx_t j0,
                                           const idx_t j1) const {
  assert(i0 < i1);
  assert(j0 < j1);
  binary_matrix B(i1 - i0, j1 - j0);
  copy_submatrix_to(i0, i1, j0, j1, B);
  return B;
}

// Destination word (di, dj) is read from the source at FLAT word index (i0+di)*bpr + j0/64 + dj
// (and the word after it when j0 is not word aligned); words past the buffer read as 0. A tile
// that extends past the right edge therefore continues into the next source row
// (binmat.cpp:267-298, SURVEY.md §4 hazard 3).
void binary_matrix::copy_submatrix_to(const idx_t i0, const idx_t i1, const idx_t j0, const idx_t j1,
                                      binary_matrix& B) const {
  assert(i0 < i1);
  assert(j0 < j1);
  const idx_t sh = j0 % kBits;
  auto src = [&](idx_t k) -> block_t { return k < data_blocks ? data[k] : 0; };
  for (idx_t di = 0; di < B.rows; ++di) {
    const idx_t base = (i0 + di) * blocks_per_row + j0 / kBits;
    for (idx_t dj = 0; dj < B.blocks_per_row; ++dj) {
      const block_t hi = src(base + dj);
      B.data[di * B.blocks_per_row + dj] = sh ? (hi << sh) | (src(base + dj + 1) >> (kBits - sh)) : hi;
    }
  }
}

// Writes src at (i0, j0), clipped to the rows of this matrix (binmat.cpp:373-414). Words are
// addressed as (row, word-column) pairs that may step one word past the end of a row, which
// then lands on the first word of the next row, exactly as the reference's arithmetic does.
void binary_matrix::set_submatrix(const idx_t i0, const idx_t j0, const binary_matrix& B) {
  const idx_t sh = j0 % kBits;
  const idx_t w0 = j0 / kBits;
  const idx_t end_bit = (sh + B.cols) % kBits;                  // bits used in the last word
  const idx_t span = (kBits - 1 + sh + B.cols) / kBits;         // destination words per row
  auto rd = [&](idx_t i, idx_t j) -> block_t {                  // get_block, guarded at the end
    const idx_t k = i * blocks_per_row + j;
    return k < data_blocks ? get_block(i, j) : 0;
  };
  auto wr = [&](idx_t i, idx_t j, block_t v) {
    const idx_t k = i * blocks_per_row + j;
    if (k < data_blocks) data[k] = v;
  };
  if (sh == 0 || span == 1) {
    // each source word maps onto one destination word
    const block_t from_sh = sh ? (ONES >> sh) : ONES;
    const block_t to_end = end_bit ? (ONES << (kBits - end_bit)) : ONES;
    const block_t m = from_sh & to_end;
    for (idx_t si = 0, di = i0; si < B.rows && di < rows; ++si, ++di) {
      idx_t sj = 0, dj = w0;
      for (; sj < B.last_block && dj < blocks_per_row; ++sj, ++dj) wr(di, dj, B.get_block(si, sj));
      wr(di, dj, (rd(di, dj) & ~m) | ((B.get_block(si, sj) >> sh) & m));
    }
    return;
  }
  // unaligned and spanning: each source word straddles two destination words
  const block_t top = ONES << (kBits - sh);   // the first sh bits of a word
  const block_t tail = end_bit ? (ONES << (kBits - end_bit)) : 0;
  for (idx_t si = 0, di = i0; si < B.rows && di < rows; ++si, ++di) {
    idx_t sj = 0, dj = w0;
    for (; sj < B.last_block && dj < last_block; ++sj, ++dj) {
      const block_t w = B.get_block(si, sj);
      wr(di, dj, (rd(di, dj) & top) | (w >> sh));
      wr(di, dj + 1, (rd(di, dj + 1) & ~top) | (w << (kBits - sh)));
    }
    const block_t w = B.get_block(si, sj);
    const block_t keep = dj <= last_block ? rd(di, dj) : 0;
    wr(di, dj, (keep & top) | (w >> sh));
    if (dj < last_block) wr(di, dj + 1, (rd(di, dj + 1) & ~tail) | ((w << (kBits - sh)) & tail));
  }
}

// ---- growth -----------------------------------------------------------------------------------

void binary_matrix::add_rows(idx_t nrows) {
  rows += nrows;
  const idx_t words = blocks_per_row * rows;
  block_t* grown = new block_t[words]();
  if (data_blocks) std::memcpy(grown, data, data_blocks * sizeof(block_t));
  delete[] data;
  data = grown;
  data_blocks = words;
}

void binary_matrix::remove_rows(idx_t nrows) {
  if (nrows < rows) {
    rows -= nrows;
    data_blocks -= blocks_per_row * nrows;
  } else {
    rows = 0;
    data_blocks = 0;
  }
}

// ---- algebra over GF(2) -------------------------------------------------------------------------

binary_matrix& add(const binary_matrix& A, const binary_matrix& B, binary_matrix& C) {
  assert(C.data != 0);
  assert(C.rows == A.rows && C.rows == B.rows);
  assert(C.cols == A.cols && C.cols == B.cols);
  for (idx_t i = 0; i < A.rows; ++i)
    for (idx_t j = 0; j < C.blocks_per_row; ++j) C.set_block(i, j, A.get_block(i, j) ^ B.get_block(i, j));
  return C;
}

binary_matrix& bool_and(const binary_matrix& A, const binary_matrix& B, binary_matrix& C) {
  assert(C.data != 0);
  assert(C.rows == A.rows && C.rows == B.rows);
  assert(C.cols == A.cols && C.cols == B.cols);
  for (idx_t i = 0; i < A.rows; ++i)
    for (idx_t j = 0; j < C.blocks_per_row; ++j) C.set_block(i, j, A.get_block(i, j) & B.get_block(i, j));
  return C;
}

idx_t dist(const binary_matrix& A, const binary_matrix& B) {
  assert(A.rows == B.rows);
  assert(A.cols == B.cols);
  idx_t w = 0;
  for (idx_t i = 0; i < A.rows; ++i)
    for (idx_t j = 0; j < A.blocks_per_row; ++j) w += popcount(A.get_block(i, j) ^ B.get_block(i, j));
  return w;
}

// C = A B: row i of C is the XOR of the rows k of B with A(i,k) = 1
binary_matrix& mul_AB(const binary_matrix& A, const binary_matrix& B, binary_matrix& C) {
  assert(C.data != 0);
  assert(C.rows == A.rows && C.cols == B.cols && A.cols == B.rows);
  C.clear();
  for (idx_t k = 0; k < B.rows; ++k)
    for (idx_t i = 0; i < A.rows; ++i)
      if (A.get_block(i, k / kBits) & binary_matrix::bit(k))
        for (idx_t j = 0; j < B.blocks_per_row; ++j) C.set_block(i, j, C.get_block(i, j) ^ B.get_block(k, j));
  return C;
}

// C = A^t B: row i of C is the XOR of the rows k of B with A(k,i) = 1
binary_matrix& mul_AtB(const binary_matrix& A, const binary_matrix& B, binary_matrix& C) {
  assert(C.data != 0);
  assert(C.rows == A.cols && C.cols == B.cols && A.rows == B.rows);
  C.clear();
  for (idx_t k = 0; k < A.rows; ++k)
    for (idx_t i = 0; i < A.cols; ++i)
      if (A.get_block(k, i / kBits) & binary_matrix::bit(i))
        for (idx_t j = 0; j < B.blocks_per_row; ++j) C.set_block(i, j, C.get_block(i, j) ^ B.get_block(k, j));
  return C;
}

// C = A B^t: C(i,j) = <row i of A, row j of B>. As written (binmat.cpp:584-592) j runs over
// B.cols, not B.rows: columns of C beyond B.cols keep their old value, and for B.cols > B.rows the
// extra rows of B read as 0 past the buffer and the writes past C's rows are dropped.
binary_matrix& mul_ABt(const binary_matrix& A, const binary_matrix& B, binary_matrix& C) {
  assert(C.data != 0);
  assert(C.rows == A.rows && C.cols == B.rows && A.cols == B.cols);
  for (idx_t i = 0; i < A.rows; ++i) {
    for (idx_t j = 0; j < B.cols; ++j) {
      block_t acc = 0;
      for (idx_t k = 0; k < A.blocks_per_row; ++k) {
        const idx_t kb = j * B.blocks_per_row + k;
        acc ^= A.get_block(i, k) & (kb < B.data_blocks ? B.get_block(j, k) : 0);
      }
      const idx_t kc = i * C.blocks_per_row + j / kBits;
      if (kc < C.data_blocks) C.set(i, j, parity(acc));
    }
  }
  return C;
}

// As written (binmat.cpp:596-604): not implemented, C is returned unchanged.
binary_matrix& mul_AtBt(const binary_matrix& A, const binary_matrix& B, binary_matrix& C) {
  assert(C.data != 0);
  assert(C.rows == A.cols && C.cols == B.rows && A.rows == B.cols);
  (void)A;
  (void)B;
  return C;
}

binary_matrix& mul(const binary_matrix& A, const bool At, const binary_matrix& B, const bool Bt,
                   binary_matrix& C) {
  if (At) return Bt ? mul_AtBt(A, B, C) : mul_AtB(A, B, C);
  return Bt ? mul_ABt(A, B, C) : mul_AB(A, B, C);
}

// ---- printing -----------------------------------------------------------------------------------

// Same text as binmat.cpp:624-644: a header line, a ruler with '|' every 64 columns, then one
// line per row with '#' for ones and '.' / '+' (grid crossings) for zeros.
std::ostream& operator<<(std::ostream& out, const binary_matrix& A) {
  out << "rows=" << A.rows << "\tcols=" << A.cols << "\tlen=" << A.len << "\tbpw=" << kBits
      << "\tdw=" << A.data_blocks << "\twpr=" << A.blocks_per_row << "\ttm=" << bm_bitset(A.trail_mask)
      << std::endl;
  std::string line = "       ";
  for (idx_t j = 0; j < A.cols; ++j) {
    line += (j % kBits) ? ' ' : '|';
    line += ' ';
  }
  out << line << std::endl;
  for (idx_t i = 0; i < A.rows; ++i) {
    out << std::setw(5) << i << "  ";
    line.clear();
    for (idx_t j = 0; j < A.cols; ++j) {
      const bool grid = (i % g_grid_width) == 0 && (j % g_grid_width) == 0;
      line += A.get(i, j) ? '#' : (grid ? '+' : '.');
      line += ' ';
    }
    out << line << std::endl;
  }
  return out;
}
