// bic_gf2.hip -- SURVEY.md §8 f4: the binary_matrix algebra over GF(2) on the device.
//
//  * binmat.cpp:516-542 mul_AB:   C = A B, row i of C = XOR of the rows k of B with A(i,k) = 1
//    (k < K = B.rows, whole words of B, C cleared first);
//  * binmat.cpp:545-572 mul_AtB:  C = A^t B, the same with A(k,i) (k < A.rows, i < A.cols);
//  * binmat.cpp:575-594 mul_ABt:  C(i,j) = parity of (row i of A AND row j of B) over A's whole
//    words, for j < B.cols as written (C has B.rows columns): bits j in [B.rows, B.cols) of a row
//    are written 0, bits past B.cols keep their value, writes past C's storage are dropped;
//  * binmat.cpp:596-604 mul_AtBt: not implemented, C unchanged;
//  * binmat.cpp:199-214 transpose_to (get_transposed): B(j,i) = A(i,j).
//
// Layout is the plane layout of every other kernel: rows x wpr u64 words, column j at bit 63 - j%64
// of word j/64. No MFMA: a GF(2) product is AND/XOR on bits, which the VALU does 64 at a time per
// lane; the products go through per-workgroup "four Russians" nibble tables in LDS.
#include "bic_device.h"

namespace bic {

// 64 x 64 bit block transpose per wave: lane l holds source row 64 rb + l, word wb; for each of
// the block's 64 columns one ballot gathers the column's bits over the 64 rows (bit l = row l, so
// the MSB-first output word is its bit reversal -- a scalar op: the ballot is wave-uniform), and
// lane b keeps column b's word. 64 ballots per 64 output words, no LDS.
// dst has ncols_out rows (source columns 0 .. ncols_out - 1; columns past the source's s_words
// words read 0) of d_words words at stride d_stride (source rows past s_rows read 0).
__global__ __launch_bounds__(256) void k_gf2_transpose(const uint64_t* __restrict__ src, uint32_t s_rows,
                                                       uint32_t s_stride, uint32_t s_words, uint32_t ncols_out,
                                                       uint64_t* __restrict__ dst, uint32_t d_stride,
                                                       uint32_t d_words) {
  const int lane = lane_id();
  const uint32_t wb = blockIdx.x;                            // source word column
  const uint32_t rb = blockIdx.y * 4 + wave_id();   // source row block = destination word
  if (rb >= d_words) return;                                    // wave-uniform
  const uint32_t r = rb * 64 + lane;
  const uint64_t x = (r < s_rows && wb < s_words) ? src[(uint64_t)r * s_stride + wb] : 0ull;
  uint64_t out = 0;
#pragma unroll 8
  for (int b = 0; b < 64; ++b) {
    const uint64_t m = __builtin_amdgcn_ballot_w64(((x >> (63 - b)) & 1ull) != 0);
    out = lane == b ? __builtin_bitreverse64(m) : out;
  }
  const uint32_t c = wb * 64 + lane;
  if (c < ncols_out) dst[(uint64_t)c * d_stride + rb] = out;
}

// C (M x 64 nw) = A (M x kbits) B (kbits x 64 nw) over GF(2), four Russians on nibbles:
// a workgroup owns 256 rows x 4 output words; for each 64-bit word of A it stages B's 64 rows of
// those 4 words, builds the 16 nibble tables (entry n of table t = XOR of the rows 4t + i with bit
// 3 - i of n set; 32 B per entry: the 4 words side by side) and every row XORs in 16 entries, one
// per nibble of its A word. LDS: 2 KiB of B + 8 KiB of tables.
// Store: bits c < nset of every row get the product; bits past nset keep C's old value (mul_ABt
// as written); nset = 64 nw replaces the whole row (mul_AB, mul_AtB). Words past nw are not touched.
constexpr int kGfRows = 256, kGfWords = 4;
__global__ __launch_bounds__(256) void k_gf2_ab(const uint64_t* __restrict__ A, uint32_t M, uint32_t a_stride,
                                                uint32_t kbits, const uint64_t* __restrict__ B, uint32_t b_stride,
                                                uint32_t nw, uint64_t* __restrict__ C, uint32_t c_stride,
                                                uint32_t nset) {
  __shared__ __attribute__((aligned(16))) uint64_t sb[64 * kGfWords];
  __shared__ __attribute__((aligned(16))) uint64_t tab[16 * 16 * kGfWords];
  const uint32_t t = threadIdx.x;
  const uint32_t j0 = blockIdx.x * kGfWords;
  const uint32_t row = blockIdx.y * kGfRows + t;
  const uint64_t* arow = A + (uint64_t)min(row, M - 1) * a_stride;
  uint64_t acc[kGfWords] = {0, 0, 0, 0};
  const uint32_t kw_n = (kbits + 63) / 64;
  for (uint32_t kw = 0; kw < kw_n; ++kw) {
    {  // stage B rows 64 kw .. 64 kw + 63, words j0 .. j0 + 3
      const uint32_t r = t >> 2, jj = t & 3, k = kw * 64 + r;
      sb[t] = (k < kbits && j0 + jj < nw) ? B[(uint64_t)k * b_stride + j0 + jj] : 0ull;
    }
    uint64_t a = arow[kw];  // issued before the barriers: its latency hides behind the table build
    const uint32_t rem = kbits - kw * 64;
    if (rem < 64) a &= ~0ull << (64 - rem);  // A's bits past kbits are not products
    __syncthreads();
#pragma unroll
    for (int q = 0; q < 4; ++q) {  // 1024 table words, 4 per thread
      const uint32_t e = t + 256 * q, jj = e & 3, n = (e >> 2) & 15, tb = e >> 6;
      uint64_t v = 0;
#pragma unroll
      for (int i = 0; i < 4; ++i) v ^= ((n >> (3 - i)) & 1u) ? sb[(tb * 4 + i) * kGfWords + jj] : 0ull;
      tab[e] = v;
    }
    __syncthreads();
#pragma unroll
    for (int tb = 0; tb < 16; ++tb) {
      const uint32_t n = (uint32_t)(a >> (60 - 4 * tb)) & 15u;
      const uint4* p = reinterpret_cast<const uint4*>(tab + (tb * 16 + n) * kGfWords);
      const uint4 lo = p[0], hi = p[1];
      acc[0] ^= ((uint64_t)lo.y << 32) | lo.x;
      acc[1] ^= ((uint64_t)lo.w << 32) | lo.z;
      acc[2] ^= ((uint64_t)hi.y << 32) | hi.x;
      acc[3] ^= ((uint64_t)hi.w << 32) | hi.z;
    }
    __syncthreads();  // the next word's staging overwrites sb / tab
  }
  if (row >= M) return;
#pragma unroll
  for (int jj = 0; jj < kGfWords; ++jj) {
    const uint32_t j = j0 + jj;
    if (j >= nw) break;
    uint64_t* dst = C + (uint64_t)row * c_stride + j;
    const uint32_t lo = j * 64;
    if (lo + 64 <= nset) {
      *dst = acc[jj];
    } else if (lo < nset) {
      const uint64_t m = ~0ull << (64 - (nset - lo));  // the first nset - lo bits
      *dst = (acc[jj] & m) | (*dst & ~m);
    }
  }
}

void launch_gf2_transpose(hipStream_t s, const uint64_t* src, uint32_t s_rows, uint32_t s_stride, uint32_t s_words,
                          uint32_t ncols_out, uint64_t* dst, uint32_t d_stride, uint32_t d_words) {
  const uint32_t gx = (ncols_out + 63) / 64, gy = (d_words + 3) / 4;
  if (gx && gy)
    k_gf2_transpose<<<dim3(gx, gy), 256, 0, s>>>(src, s_rows, s_stride, s_words, ncols_out, dst, d_stride, d_words);
}

void launch_gf2_ab(hipStream_t s, const uint64_t* A, uint32_t M, uint32_t a_stride, uint32_t kbits, const uint64_t* B,
                   uint32_t b_stride, uint32_t nw, uint64_t* C, uint32_t c_stride, uint32_t nset) {
  const uint32_t gx = (nw + kGfWords - 1) / kGfWords, gy = (M + kGfRows - 1) / kGfRows;
  if (gx && gy) k_gf2_ab<<<dim3(gx, gy), 256, 0, s>>>(A, M, a_stride, kbits, B, b_stride, nw, C, c_stride, nset);
}

}  // namespace bic
