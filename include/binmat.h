// binmat.h -- bit-packed binary matrix of the reference API (drop-in for
// /root/reference/src/binmat.h). Host container; the GPU hot path that consumes it is in
// bic_gpu.h / bic.h. Storage is exactly the layout the HIP kernels read (bic.h header):
// rows x blocks_per_row 64-bit words, row-major, column j at bit 63 - j%64 of word j/64.
//
// Ownership follows the reference (binmat.h:47,178; binmat.cpp:180-184): no destructor;
// destroy() frees; operator= frees the target and then SHARES the source's buffer.
// Methods marked "as written" reproduce reference behaviour that looks unintended but is
// observable by its callers; DESIGN.md §"C++ API" lists them.
#ifndef BINMAT_H
#define BINMAT_H

#include <bitset>
#include <cstring>
#include <iostream>

typedef unsigned long idx_t;
typedef unsigned long block_t;

#define BITS_PER_BLOCK (sizeof(block_t) * 8)
#define ONES (~block_t(0))
#define ZEROES (block_t(0))
#define LSB block_t(1)
#define MSB (LSB << (BITS_PER_BLOCK - 1))
#define IMSB (ONES >> 1)
#define ILSB (ONES << 1)

// boolean exclusive or of two truth values (used by the reference's predictors)
#define XOR(a, b) ((!(a) && (b)) || ((a) && !(b)))

typedef std::bitset<BITS_PER_BLOCK> bm_bitset;

class binary_matrix {
 public:
  // -- construction / ownership ------------------------------------------------------------
  binary_matrix(idx_t _rows, idx_t _cols);       // storage zeroed (the reference leaves it uninitialised)
  binary_matrix() : rows(0), cols(0), len(0), last_bit_offset(0), data_blocks(0),
                    blocks_per_row(0), last_block(0), data(nullptr), trail_mask(0) {}
  binary_matrix(const binary_matrix& other);      // deep copy
  ~binary_matrix() {}                             // explicit destroy() only
  void allocate(idx_t _rows, idx_t _cols);
  void destroy() {
    delete[] data;
    reset();
  }
  binary_matrix& operator=(const binary_matrix& A);  // frees own buffer, shares A's

  // -- geometry ------------------------------------------------------------------------------
  inline idx_t get_rows() const { return rows; }
  inline idx_t get_cols() const { return cols; }
  inline idx_t get_len() const { return len; }

  // -- element access ------------------------------------------------------------------------
  inline bool get(const idx_t i, const idx_t j) const { return (word(i, j) & bit(j)) != 0; }
  inline void set(const idx_t i, const idx_t j) { word(i, j) |= bit(j); }
  inline void clear(const idx_t i, const idx_t j) { word(i, j) &= ~bit(j); }
  inline void flip(const idx_t i, const idx_t j) { word(i, j) ^= bit(j); }
  inline void set(const idx_t i, const idx_t j, const bool v) {
    if (v) set(i, j); else clear(i, j);
  }

  // -- whole-matrix fills ----------------------------------------------------------------------
  void clear();  // every word of every row, including the pad bits
  void set();
  void flip();

  // -- reductions --------------------------------------------------------------------------------
  idx_t weight() const;
  idx_t row_weight(idx_t i) const;
  idx_t col_weight(idx_t j) const;  // as written: samples rows 0, 1, ... while r*blocks_per_row < rows
  bool sum() const;
  bool row_sum(idx_t i) const;
  bool col_sum(idx_t j) const;

  // -- copies, views -------------------------------------------------------------------------------
  binary_matrix get_copy() const;
  binary_matrix get_vectorized() const;      // 1 x rows*cols
  binary_matrix get_col(const idx_t j) const;  // returned as a 1 x rows ROW vector
  binary_matrix get_row(const idx_t i) const;
  binary_matrix get_submatrix(const idx_t i0, const idx_t i1, const idx_t j0, const idx_t j1) const;
  binary_matrix get_transposed() const;
  void copy_to(binary_matrix& B) const;
  void copy_vectorized_to(binary_matrix& B) const;
  void copy_col_to(const idx_t j, binary_matrix& B) const;
  void copy_row_to(const idx_t i, binary_matrix& B) const;
  void copy_submatrix_to(const idx_t i0, const idx_t i1, const idx_t j0, const idx_t j1,
                         binary_matrix& B) const;
  void transpose_to(binary_matrix& B) const;

  void set_vectorized(const binary_matrix& src);
  void set_col(const idx_t j, const binary_matrix& src);
  void set_row(const idx_t i, const binary_matrix& src);
  void set_submatrix(const idx_t i0, const idx_t j0, const binary_matrix& src);

  void add_rows(idx_t nrows);     // new rows zeroed; as written, len is not updated
  void remove_rows(idx_t nrows);  // keeps the buffer

  // -- algebra over GF(2) -------------------------------------------------------------------------
  friend std::ostream& operator<<(std::ostream& out, const binary_matrix& A);
  friend binary_matrix& add(const binary_matrix& A, const binary_matrix& B, binary_matrix& C);
#define bool_xor add
  friend binary_matrix& bool_and(const binary_matrix& A, const binary_matrix& B, binary_matrix& C);
  friend binary_matrix& mul(const binary_matrix& A, const bool At, const binary_matrix& B,
                            const bool Bt, binary_matrix& C);
  friend idx_t dist(const binary_matrix& A, const binary_matrix& B);

  // -- raw storage (extension: what the GPU bridge hands to the C ABI) ---------------------------
  inline block_t* raw_blocks() { return data; }
  inline const block_t* raw_blocks() const { return data; }
  inline idx_t get_blocks_per_row() const { return blocks_per_row; }

 private:
  void reset() {
    rows = cols = len = last_bit_offset = data_blocks = blocks_per_row = last_block = 0;
    data = nullptr;
    trail_mask = 0;
  }
  void shape(idx_t r, idx_t c);
  inline block_t& word(idx_t i, idx_t j) const { return data[i * blocks_per_row + j / BITS_PER_BLOCK]; }
  static inline block_t bit(idx_t j) { return MSB >> (j % BITS_PER_BLOCK); }
  // word j of row i with the pad bits of the last word of a row cleared
  inline block_t get_block(const idx_t i, const idx_t j) const {
    const block_t w = data[i * blocks_per_row + j];
    return j < last_block ? w : (w & trail_mask);
  }
  inline void set_block(const idx_t i, const idx_t j, const block_t b) { data[i * blocks_per_row + j] = b; }

  friend binary_matrix& mul_AB(const binary_matrix&, const binary_matrix&, binary_matrix&);
  friend binary_matrix& mul_AtB(const binary_matrix&, const binary_matrix&, binary_matrix&);
  friend binary_matrix& mul_ABt(const binary_matrix&, const binary_matrix&, binary_matrix&);
  friend binary_matrix& mul_AtBt(const binary_matrix&, const binary_matrix&, binary_matrix&);

  idx_t rows;
  idx_t cols;
  idx_t len;              // rows*cols at allocation
  idx_t last_bit_offset;  // (cols-1) % 64
  idx_t data_blocks;      // words allocated (rows*blocks_per_row)
  idx_t blocks_per_row;   // ceil(cols/64)
  idx_t last_block;       // blocks_per_row - 1
  block_t* data;
  block_t trail_mask;     // valid bits of a row's last word
};

// Spacing of the '+' grid marks operator<< prints (default 10, binmat.cpp:618-620).
void set_grid_width(idx_t g);

#endif
