/*
 * bic_oracle.h -- TEST INFRASTRUCTURE ONLY (the parity checker, never the product).
 *
 * A plain-C, bit-serial restatement of the reference's hot path
 * (nacho-pancho/binary-image-compression @ /root/reference/src):
 *
 *   bitplane extraction   bitplane_tool.cpp:24-30
 *   med predictor         pred.cpp:3-15  (== coding.cpp:5-17 bilinear_predictor)
 *   weight                binmat.cpp:57-67
 *   Golomb coder          Golomb.h:12-29, GolombCoder.cpp:13-34
 *   EG run coder          eg.h:7-27, eg.cpp:4-37
 *   tile path (R=0)       compress7_test.cpp:118-275 with the search window empty
 *   get_submatrix         binmat.cpp:259-298 (incl. the next-row wrap at the right edge)
 *   set_submatrix         binmat.cpp:373-414 (restated per bit)
 *
 * plus the build-defined parts the reference leaves open:
 * run extraction per row and the MSB-first bit writer.
 *
 * Parity pinning: tests/golden/ holds vectors produced by the reference's own
 * objects (oracle/_ref, built from /root/reference/src by oracle/Makefile) and
 * tests/test_oracle_golden.py checks this restatement against them.
 *
 * Only tests/, __graft_entry__.smoke() and bench.py's cpu_baseline leg may load
 * this library. The product (binary-image-compression_amd/) never links it.
 *
 * Plane layout (same as binary_matrix, binmat.h:114-141): rows x wpr uint64
 * words, row-major; column j lives in word j/64 at bit (63 - j%64).
 */
#ifndef BIC_ORACLE_H
#define BIC_ORACLE_H

#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

/* ---- synthetic inputs (SURVEY.md §8 d) ---------------------------------- */
uint64_t bo_splitmix64(uint64_t* state);
/* Bernoulli(p) plane: bit = (16-bit draw < round(p*65536)); four draws per
 * splitmix64 output, consumed MSB-first. Trailing bits past `cols` are zero. */
void bo_gen_plane(uint64_t seed, double p, size_t rows, size_t cols, size_t wpr,
                  uint64_t* plane);
/* n uniform bytes (one splitmix64 output per 8 bytes, little-endian order). */
void bo_gen_bytes(uint64_t seed, size_t n, uint8_t* out);

/* ---- bit access --------------------------------------------------------- */
int  bo_get(const uint64_t* P, size_t wpr, size_t i, size_t j);
void bo_set(uint64_t* P, size_t wpr, size_t i, size_t j, int v);

/* ---- L1/L3 ops ---------------------------------------------------------- */
/* bitplane_tool.cpp:24-30 -- plane bi holds (gray[i*cols+j] >> bi) & 1.
 * gray is 8-bit (bytes_per_px = 1) or 16-bit host-order (bytes_per_px = 2). */
void bo_bitplanes(const void* gray, int bytes_per_px, size_t rows, size_t cols,
                  int nplanes, uint64_t* planes, size_t wpr);
/* plane2pgm_tool.cpp:26-41 -- gray[li] |= 1 << b for every set bit of plane b (samples as the
 * tool's pixel_t, 32-bit; bits no plane covers are 0). */
void bo_planes_to_gray(const uint64_t* planes, int nplanes, size_t rows, size_t cols, size_t wpr,
                       uint32_t* gray);
/* number of planes bitplane_tool.cpp:24 extracts: #{bi : 2^bi < maxval} */
int bo_num_planes(int maxval);
/* pred.cpp:3-15, bit-serial. R(0,0) and the trailing pad bits are left 0
 * (the reference leaves them unwritten; observed 0 -- SURVEY.md §4 hazard 1). */
void bo_med(const uint64_t* P, uint64_t* R, size_t rows, size_t cols, size_t wpr);
/* binmat.cpp:57-67 (the last word of every row trail-masked). */
uint64_t bo_weight(const uint64_t* P, size_t rows, size_t cols, size_t wpr);

/* ---- bit writer (build-defined): MSB-first bytes ------- */
typedef struct {
    uint8_t* buf;     /* may be NULL: count only */
    size_t cap_bits;  /* capacity in bits */
    uint64_t pos;     /* bits written (counted even past capacity) */
    int overflow;
} bo_bw;
void bo_bw_init(bo_bw* bw, uint8_t* buf, size_t cap_bytes);
void bo_bw_put(bo_bw* bw, uint32_t value, unsigned nbits); /* nbits <= 32 */
void bo_bw_zeros(bo_bw* bw, uint64_t n);

/* ---- Golomb (Golomb.h:12-29, GolombCoder.cpp:13-34) --------------------- */
typedef struct {
    uint32_t accumulatedError;
    uint32_t samples;
    uint32_t k;
    int64_t bitcount;
} bo_golomb;
void bo_golomb_init(bo_golomb* g);
/* codes one sample: k-bit binary part (s mod 2^k, MSB-first), (s>>k) zeros,
 * then '1' (order of GolombCoder.cpp:22-25). Returns the codeword length. */
uint32_t bo_golomb_code(bo_golomb* g, uint32_t s, bo_bw* bw);

/* ---- EG (eg.h:7-27, eg.cpp:2-37) ----------------------------------------- */
typedef struct {
    uint32_t g, blockSize;
    int lutIndex;
    uint64_t bitcount;
    int adaptive; /* 0: as written (incBlockSize disabled, eg.cpp:25);
                     1: JPEG-LS run mode (incBlockSize per full block, lutIndex capped at 31) */
} bo_eg;
void bo_eg_init(bo_eg* e, int adaptive);
/* '1' per full block, then EOL -> '1', else '0' + g-bit remainder (eg.cpp:24-33) */
uint32_t bo_eg_code(bo_eg* e, int len, int eol, bo_bw* bw);

/* ---- plane encoders (run extraction) ------------------- */
/* Per row, raster order: for each 1 the count of 0s since the previous 1 (or the
 * row start) as a normal sample; at row end the trailing-zero count as the EOL
 * sample (emitted even when 0). One coder instance per plane.
 * coder: 0 = Golomb, 1 = EG as written, 2 = EG adaptive.
 * Writes MSB-first bytes into out (NULL = count only), zero-padded to a 64-bit
 * multiple. Returns the stream length in bits (before padding), or -1 when out
 * is non-NULL and too small. *nsamples (may be NULL) receives the sample count. */
int64_t bo_encode_plane(const uint64_t* plane, size_t rows, size_t cols, size_t wpr,
                        int predict, int coder, uint8_t* out, size_t cap_bytes,
                        uint64_t* nsamples);
/* The run samples themselves (s, eol) for a plane -- for tests. Returns count;
 * writes at most cap entries. */
size_t bo_plane_runs(const uint64_t* plane, size_t rows, size_t cols, size_t wpr,
                     uint32_t* runs, uint8_t* eols, size_t cap);
/* Golomb-code an arbitrary sample sequence starting from a fresh coder. */
int64_t bo_golomb_samples(const uint32_t* s, size_t n, uint8_t* out, size_t cap_bytes,
                          uint32_t* k_out, uint32_t* len_out);

/* ---- decoders (round-trip checks of the build-defined stream) ----------- */
/* Inverse of bo_encode_plane for coder 0 (Golomb). Rebuilds the residual (or the
 * plane when predict = 0); with predict = 1 it then inverts med, taking P(0,0)
 * from `corner` (the one bit med discards). Returns 0 on success. */
int bo_decode_plane_golomb(const uint8_t* stream, uint64_t nbits, size_t rows, size_t cols,
                           size_t wpr, int predict, int corner, uint64_t* plane);
/* EG over a run list (coder: 1 as written, 2 adaptive), MSB-first bits into out (nullable);
 * per-run bits into bits_out (nullable). Returns the total bits, -1 on overflow. */
int64_t bo_eg_runs(const int32_t* len, const uint8_t* eol, size_t n, int adaptive, uint8_t* out,
                   size_t cap_bytes, uint32_t* bits_out);
/* The decoders' row index (bic.h bic_row_index): per row, the Golomb stream's bit offset of
 * the row's first codeword and the residual 1s of the plane before the row. */
void bo_row_index(const uint64_t* plane, size_t rows, size_t cols, size_t wpr, int predict, uint64_t* index);
/* the adaptive EG coder's row index: per row the stream bits before it and the coder state (lutIndex,
 * 32 = fresh) at its start */
void bo_egad_row_index(const uint64_t* plane, size_t rows, size_t cols, size_t wpr, int predict, uint64_t* index);
/* inverse med with P(0,0) = corner */
void bo_unmed(const uint64_t* R, uint64_t* P, size_t rows, size_t cols, size_t wpr, int corner);

/* ---- tiles (compress7_test.cpp:118-275 with R=0) ---- */
/* get_submatrix(i0,i0+W,j0,j0+W) semantics of binmat.cpp:259-298, including the
 * read of the next row's first word at the right edge and 0 past the last word. */
void bo_get_submatrix(const uint64_t* I, size_t rows, size_t cols, size_t wpr,
                      size_t i0, size_t i1, size_t j0, size_t j1, uint64_t* B, size_t bwpr);
/* set_submatrix(i0,j0,B): bits of B written at (i0+r, j0+c), clipped to I. */
void bo_set_submatrix(uint64_t* I, size_t rows, size_t cols, size_t wpr,
                      size_t i0, size_t j0, const uint64_t* B, size_t brows, size_t bcols, size_t bwpr);
/* log2 C(n,r) (enumL, compress7_test.cpp:25-28) without GSL: exact integer
 * values at r in {0, 1, n-1, n} for power-of-two n, long-double lgamma otherwise. */
double bo_enumL(unsigned n, unsigned r);
/* The tile loop. lentab[w] = (uint64)(2 + enumL(W*W, w)) for w = 0..W*W.
 * I is modified in place (residual write-back, compress7_test.cpp:272).
 * Per tile (raster order): w_nonpred, w_pred, mode ('o' or 'O'), chosen length.
 * Returns the Golomb bitcount of the chosen weights; *L_out = sum of lengths. */
int64_t bo_patch_encode(uint64_t* I, size_t rows, size_t cols, size_t wpr, unsigned W,
                        const uint64_t* lentab, uint32_t* w_nonpred, uint32_t* w_pred,
                        char* modes, uint64_t* L_out, uint8_t* stream, size_t cap_bytes);

/* compress_test.cpp:73-111 (patch match search): for each W x W tile in raster order over
 * ceil(rows/W) x ceil(cols/W), the position (i2, j2) of the least Hamming distance over the
 * causal search region, first in scan order, exactly as the reference's two loops with their
 * early exit at a perfect match; (0, 0, W*W) when nothing beats W*W. */
void bo_patch_search(const uint64_t* I, size_t rows, size_t cols, size_t wpr, unsigned W,
                     uint32_t* besti, uint32_t* bestj, uint32_t* bestd);
/* The same search for the tiles of tile rows [tr0, tr1) only (every tile's search is independent
 * of the others' results), written at their raster indices of the full arrays: lets the tests
 * split the checker over host threads. */
void bo_patch_search_rows(const uint64_t* I, size_t rows, size_t cols, size_t wpr, unsigned W,
                          size_t tr0, size_t tr1, uint32_t* besti, uint32_t* bestj, uint32_t* bestd);

/* compress7_test.cpp:117-275 with search window R and match threshold T (rows, cols multiples
 * of W): per tile the causal search over the image as modified by the residual write-back of
 * every earlier tile, modes 'X' 'x' (match, predicted or not) 'O' 'o' (no match), the chosen
 * weight coded by golomb_match / golomb_nomatch, the residual written back into I (in place).
 * enumL[w] = enumL(W*W, w) for w = 0..W*W. Outputs per tile (each nullable): besti, bestj,
 * bestd (W*W+1 when the region is empty), weights, modes. stats (nullable) [4]: matches,
 * golomb_match bits, golomb_nomatch bits, sum of the chosen lengths (L before the bitcounts).
 * Streams (nullable, cap_bytes each) receive the two coders' codewords. Returns 0, -1 on a bad
 * argument or stream overflow. */
int bo_match_encode(uint64_t* I, size_t rows, size_t cols, size_t wpr, unsigned W, unsigned T, unsigned R,
                    const double* enumL, uint32_t* besti, uint32_t* bestj, uint32_t* bestd,
                    uint32_t* weights, char* modes, uint64_t* stats, uint8_t* stream_match,
                    uint8_t* stream_nomatch, size_t cap_bytes);
/* the same loop, invert = 1: compress8_test.cpp's variant (patch inversion, see bic_oracle.c);
 * inverted (nullable): per tile, whether the patch was flipped. */
int bo_match_encode_v(uint64_t* I, size_t rows, size_t cols, size_t wpr, unsigned W, unsigned T, unsigned R,
                      const double* enumL, uint32_t* besti, uint32_t* bestj, uint32_t* bestd,
                      uint32_t* weights, char* modes, uint64_t* stats, uint8_t* stream_match,
                      uint8_t* stream_nomatch, size_t cap_bytes, int invert, uint8_t* inverted);

/* the loops of compress4_test.cpp (variant 4), compress5_test.cpp (5), compress6_test.cpp (6):
 * no med, the residual written back on a match only; modes 'x' / 'o' (see bic_oracle.c). */
int bo_match_encode_var(uint64_t* I, size_t rows, size_t cols, size_t wpr, unsigned W, unsigned T, unsigned R,
                        const double* enumL, uint32_t* besti, uint32_t* bestj, uint32_t* bestd,
                        uint32_t* weights, char* modes, uint64_t* stats, uint8_t* stream_match,
                        uint8_t* stream_nomatch, size_t cap_bytes, int variant);

/* ---- binary_matrix algebra over GF(2) ----------------- */
/* Reference layout only: wpr = ceil(cols/64) for every operand (the loops index words flat).
 * bo_gf2_transpose: binmat.cpp:199-214 (copy_col_to + set_row): dst (cols x rows). bo_gf2_mul:
 * op 0 mul_AB binmat.cpp:516-542, 1 mul_AtB :545-572, 2 mul_ABt :575-594 (j < B.cols as written;
 * rows of B past B.rows read 0, writes past C dropped), 3 mul_AtBt :596-604 (C unchanged). C is
 * read (ABt keeps bits) and written in place. Returns 0, -1 on a shape the reference asserts. */
void bo_gf2_transpose(const uint64_t* src, size_t rows, size_t cols, uint64_t* dst);
int bo_gf2_mul(int op, const uint64_t* A, size_t a_rows, size_t a_cols, const uint64_t* B, size_t b_rows,
               size_t b_cols, uint64_t* C, size_t c_rows, size_t c_cols);

/* ---- CPU baseline (bench.py cpu_baseline leg) ---------------------------- */
/* med + Golomb + EG over nplanes planes, OpenMP over planes when built with it.
 * Returns total Golomb bits + EG bits; *threads_used receives the thread count. */
uint64_t bo_baseline_planes(const uint64_t* planes, int nplanes, size_t rows, size_t cols,
                            size_t wpr, int predict, int do_eg, int* threads_used);

#ifdef __cplusplus
}
#endif
#endif
