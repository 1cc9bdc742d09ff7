// ref_capi.cpp -- TEST INFRASTRUCTURE ONLY.
//
// A thin extern "C" harness over the REFERENCE's own objects, compiled from the
// read-only sources under /root/reference/src by oracle/Makefile into
// oracle/_ref/libref.so (git-ignored; kept off the GPU box by .gpurunignore). No reference
// source is copied here: this file only calls the reference's binary_matrix / med /
// GolombCoder / EGCoder / pbm / pnm.
//
// Used (1) by tests/golden/make_golden.py to produce the golden vectors that pin
// oracle/bic_oracle.c, (2) by the in-container cross-checks (tests/test_ref_crosscheck.py,
// tests/test_dropin_compress.py) and (3) by bench.py's cpu_baseline leg where it is present
// (kind "reference"; on the GPU box it is not, and the oracle port is timed).
#include "binmat.h"
#include "pbm.h"
#include "pnm.h"
#include "GolombCoder.h"
#include "eg.h"

#include <chrono>
#include <cstring>
#include <sstream>
#include <cstdint>
#include <cstdio>
#include <vector>
#include <omp.h>

void med(const binary_matrix& P, binary_matrix& pP);  // pred.cpp:3

namespace {

// GolombCoder keeps k protected (Golomb.h:20-24); a derived view reads it.
struct GolombProbe : public GolombCoder {
  unsigned current_k() const { return k; }
};

binary_matrix from_words(const uint64_t* P, size_t rows, size_t cols, size_t wpr) {
  binary_matrix A(rows, cols);
  A.clear();
  for (size_t i = 0; i < rows; ++i)
    for (size_t j = 0; j < cols; ++j)
      if (P[i * wpr + j / 64] & (0x8000000000000000ull >> (j % 64))) A.set(i, j);
  return A;
}

void to_words(const binary_matrix& A, uint64_t* P, size_t wpr) {
  const size_t rows = A.get_rows(), cols = A.get_cols();
  for (size_t i = 0; i < rows; ++i) {
    for (size_t w = 0; w < wpr; ++w) P[i * wpr + w] = 0;
    for (size_t j = 0; j < cols; ++j)
      if (A.get(i, j)) P[i * wpr + j / 64] |= 0x8000000000000000ull >> (j % 64);
  }
}

}  // namespace

extern "C" {

// med over a whole plane; the output matrix is cleared first so the bits the
// reference never writes (R(0,0), pad) read 0, as observed.
int ref_med(const uint64_t* P, uint64_t* R, size_t rows, size_t cols, size_t wpr) {
  binary_matrix A = from_words(P, rows, cols, wpr);
  binary_matrix B(rows, cols);
  B.clear();
  med(A, B);
  to_words(B, R, wpr);
  A.destroy();
  B.destroy();
  return 0;
}

// The same call pattern on the reference's own med (pred.cpp:3-15): n calls on separate W x W
// tiles, as compress7_test.cpp:205-206 makes them. Returns seconds per call.
double ref_med_calls(int n, int W) {
  binary_matrix P(W, W), R(W, W);
  P.clear();
  R.clear();
  uint64_t s = 0x5EED;
  const auto t0 = std::chrono::steady_clock::now();
  for (int t = 0; t < n; ++t) {
    for (int i = 0; i < W; ++i)
      for (int j = 0; j < W; ++j) {
        s = s * 6364136223846793005ull + 1442695040888963407ull;
        P.set(i, j, (s >> 62) & 1);
      }
    med(P, R);
  }
  const double dt = std::chrono::duration<double>(std::chrono::steady_clock::now() - t0).count();
  P.destroy();
  R.destroy();
  return dt / n;
}

uint64_t ref_weight(const uint64_t* P, size_t rows, size_t cols, size_t wpr) {
  binary_matrix A = from_words(P, rows, cols, wpr);
  const uint64_t w = A.weight();
  A.destroy();
  return w;
}

// Feeds samples to one GolombCoder; per sample reports the k used and the
// bitcount increment (the codeword length).
int64_t ref_golomb(const uint32_t* s, size_t n, uint32_t* k_out, uint32_t* len_out) {
  GolombProbe g;
  for (size_t i = 0; i < n; ++i) {
    const long before = g.bitcount;
    if (k_out) k_out[i] = g.current_k();
    g.codeSample(s[i]);
    if (len_out) len_out[i] = (uint32_t)(g.bitcount - before);
  }
  return g.bitcount;
}

uint64_t ref_eg(const int32_t* len, const uint8_t* eol, size_t n, uint32_t* bits_out) {
  EGCoder e;
  for (size_t i = 0; i < n; ++i) {
    const unsigned long before = e.bitcount;
    e.codeRun(len[i], eol[i] != 0);
    if (bits_out) bits_out[i] = (uint32_t)(e.bitcount - before);
  }
  return e.bitcount;
}

// eg.cpp:20-37 with line 25's incBlockSize() enabled (what the #if 0 decoder, eg.cpp:41-55, reads),
// stepped by the reference's own EG state machine (EG::incBlockSize / decBlockSize over EGLUT,
// eg.cpp:2-18); the writes of lines 24, 29, 32-33 as an MSB-first bit string. The index is not
// stepped past 31: there the reference's incBlockSize would read EGLUT[32], past the table.
uint64_t ref_eg_adaptive(const int32_t* len, const uint8_t* eol, size_t n, uint32_t* bits_out, uint8_t* out,
                         size_t cap_bytes) {
  EGCoder e;
  uint64_t pos = 0;
  auto put = [&](uint32_t v, unsigned nb) {
    for (unsigned b = nb; b-- > 0;) {
      if (out && (pos >> 3) < cap_bytes && ((v >> b) & 1u)) out[pos >> 3] |= (uint8_t)(0x80u >> (pos & 7));
      ++pos;
    }
  };
  for (size_t i = 0; i < n; ++i) {
    const uint64_t before = pos;
    int l = len[i];
    while (l >= (int)e.blockSize) {
      l -= (int)e.blockSize;
      put(1, 1);
      if (e.lutIndex < 31) e.incBlockSize();
    }
    if (eol[i]) {
      put(1, 1);
    } else {
      put(0, 1);
      put((uint32_t)l, e.g);
      e.decBlockSize();
    }
    if (bits_out) bits_out[i] = (uint32_t)(pos - before);
  }
  return pos;
}

// The reference's header readers on a file (pnm.cpp:20-42 read_pnm_header, pbm.cpp:4-27
// read_pbm_header) and where they leave the file position: the raster offset.
int ref_pnm_header(const char* path, int* type, long* rows, long* cols, int* maxval, long* offset) {
  FILE* f = fopen(path, "rb");
  if (!f) return -2;
  int c0 = fgetc(f), c1 = fgetc(f);
  rewind(f);
  int rc;
  if (c0 == 'P' && c1 == '4') {
    idx_t r = 0, c = 0;
    rc = read_pbm_header(f, r, c) == PBM_OK ? 0 : -1;
    *type = 4;
    *rows = (long)r;
    *cols = (long)c;
    *maxval = 1;
  } else {
    int t = 0, w = 0, h = 0, mv = 0;
    rc = read_pnm_header(f, t, w, h, mv);  // closes f on a bad magic
    if (rc) return rc;
    *type = t;
    *rows = h;
    *cols = w;
    *maxval = mv;
  }
  *offset = ftell(f);
  fclose(f);
  return rc;
}

int ref_get_submatrix(const uint64_t* I, size_t rows, size_t cols, size_t wpr, size_t i0,
                      size_t i1, size_t j0, size_t j1, uint64_t* B, size_t bwpr) {
  binary_matrix A = from_words(I, rows, cols, wpr);
  binary_matrix S = A.get_submatrix(i0, i1, j0, j1);
  to_words(S, B, bwpr);
  A.destroy();
  S.destroy();
  return 0;
}

int ref_set_submatrix(uint64_t* I, size_t rows, size_t cols, size_t wpr, size_t i0, size_t j0,
                      const uint64_t* B, size_t brows, size_t bcols, size_t bwpr) {
  binary_matrix A = from_words(I, rows, cols, wpr);
  binary_matrix S = from_words(B, brows, bcols, bwpr);
  A.set_submatrix(i0, j0, S);
  to_words(A, I, wpr);
  A.destroy();
  S.destroy();
  return 0;
}

// compress7_test.cpp:118-275 with R = 0 (no tile ever matches):
// reference get_submatrix / weight / med / GolombCoder / set_submatrix, the
// mode picked by the caller-supplied length table (lentab[w] = (idx_t)(2+enumL)).
int64_t ref_tile_loop(uint64_t* Iw, size_t rows, size_t cols, size_t wpr, unsigned W,
                      const uint64_t* lentab, uint32_t* w_nonpred, uint32_t* w_pred,
                      char* modes, uint64_t* L_out) {
  binary_matrix I = from_words(Iw, rows, cols, wpr);
  const size_t Ny = (W - 1 + rows) / W, Nx = (W - 1 + cols) / W;
  GolombCoder g;
  uint64_t L = 0;
  size_t t = 0;
  for (size_t i = 0; i < Ny; ++i)
    for (size_t j = 0; j < Nx; ++j, ++t) {
      const size_t i0 = i * W, j0 = j * W;
      binary_matrix P = I.get_submatrix(i0, i0 + W, j0, j0 + W);
      binary_matrix dP(W, W);
      dP.clear();
      med(P, dP);
      const uint64_t wo = P.weight(), wO = dP.weight();
      const bool pred = lentab[wo] > lentab[wO];
      const uint64_t w = pred ? wO : wo;
      L += lentab[w];
      g.codeSample((unsigned)w);
      I.set_submatrix(i0, j0, pred ? dP : P);
      if (w_nonpred) w_nonpred[t] = (uint32_t)wo;
      if (w_pred) w_pred[t] = (uint32_t)wO;
      if (modes) modes[t] = pred ? 'O' : 'o';
      P.destroy();
      dP.destroy();
    }
  to_words(I, Iw, wpr);
  I.destroy();
  if (L_out) *L_out = L;
  return g.bitcount;
}

// PBM round trip through read_pbm_header/read_pbm_data/write_pbm (pbm.cpp).
int ref_pbm_roundtrip(const char* in_path, const char* out_path, uint64_t* rows_cols) {
  FILE* f = fopen(in_path, "r");
  if (!f) return -1;
  idx_t rows = 0, cols = 0;
  const int rc = read_pbm_header(f, rows, cols);
  if (rc != PBM_OK) { fclose(f); return rc; }
  binary_matrix A(rows, cols);
  read_pbm_data(f, A);
  fclose(f);
  FILE* o = fopen(out_path, "w");
  if (!o) { A.destroy(); return -2; }
  write_pbm(A, o);
  fclose(o);
  A.destroy();
  rows_cols[0] = rows;
  rows_cols[1] = cols;
  return 0;
}

// Reads a PBM with the reference reader and returns its bits as words.
int ref_read_pbm(const char* path, uint64_t* P, size_t wpr, uint64_t* rows_cols) {
  FILE* f = fopen(path, "r");
  if (!f) return -1;
  idx_t rows = 0, cols = 0;
  const int rc = read_pbm_header(f, rows, cols);
  if (rc != PBM_OK) { fclose(f); return rc; }
  rows_cols[0] = rows;
  rows_cols[1] = cols;
  if (P) {
    binary_matrix A(rows, cols);
    read_pbm_data(f, A);
    to_words(A, P, wpr);
    A.destroy();
  }
  fclose(f);
  return 0;
}

// Reads a PGM header + data with the reference reader (pnm.cpp:20-89).
int ref_read_pgm(const char* path, int* hdr /*type,cols,rows,maxval*/, uint32_t* pixels) {
  FILE* f = fopen(path, "r");
  if (!f) return -1;
  int type, cols, rows, maxval;
  if (read_pnm_header(f, type, cols, rows, maxval) != 0) return -2;  // closes f on failure
  hdr[0] = type; hdr[1] = cols; hdr[2] = rows; hdr[3] = maxval;
  int rc = 0;
  if (pixels) rc = read_pgm_data(f, type, cols, rows, maxval, pixels);
  fclose(f);
  return rc;
}

// CPU baseline (bench.py, kind "reference"): the reference's bit-serial med,
// GolombCoder::codeSample and EGCoder::codeRun over per-row runs, OpenMP over
// independent planes (the reference has no OpenMP on this path, SURVEY.md §8 d).
// Returns elapsed seconds of the timed region; bits[0] = Golomb bits, bits[1] = EG bits.
double ref_baseline_planes(const uint64_t* planes, int nplanes, size_t rows, size_t cols,
                           size_t wpr, int predict, int do_eg, int threads, uint64_t* bits,
                           int* threads_used) {
  std::vector<binary_matrix> in(nplanes);
  for (int p = 0; p < nplanes; ++p) in[p] = from_words(planes + (size_t)p * rows * wpr, rows, cols, wpr);
  if (threads > 0) omp_set_num_threads(threads);
  uint64_t gbits = 0, ebits = 0;
  int used = 1;
  const double t0 = omp_get_wtime();
#pragma omp parallel for schedule(dynamic, 1) reduction(+ : gbits, ebits)
  for (int p = 0; p < nplanes; ++p) {
    if (omp_get_thread_num() == 0) used = omp_get_num_threads();
    binary_matrix R(rows, cols);
    const binary_matrix* src = &in[p];
    if (predict) { R.clear(); med(in[p], R); src = &R; }
    GolombCoder g;
    EGCoder e;
    for (size_t i = 0; i < rows; ++i) {
      long last = -1;
      for (size_t j = 0; j < cols; ++j)
        if (src->get(i, j)) {
          g.codeSample((unsigned)((long)j - last - 1));
          if (do_eg) e.codeRun((int)((long)j - last - 1), false);
          last = (long)j;
        }
      g.codeSample((unsigned)((long)cols - 1 - last));
      if (do_eg) e.codeRun((int)((long)cols - 1 - last), true);
    }
    gbits += (uint64_t)g.bitcount;
    ebits += (uint64_t)e.bitcount;
    R.destroy();
  }
  const double dt = omp_get_wtime() - t0;
  for (int p = 0; p < nplanes; ++p) in[p].destroy();
  bits[0] = gbits;
  bits[1] = ebits;
  if (threads_used) *threads_used = used;
  return dt;
}

}  // extern "C"

// compress_test.cpp:73-111's search on the reference's own binary_matrix (get_submatrix, dist)
// wP (nullable): per tile P.weight() (compress_test.cpp:119-120 prints lengths from it)
extern "C" int ref_patch_search_w(const uint64_t* I, size_t rows, size_t cols, size_t wpr, unsigned W,
                                  uint32_t* besti, uint32_t* bestj, uint32_t* bestd, uint32_t* wP) {
  binary_matrix A = from_words(I, rows, cols, wpr);
  const idx_t Ny = (W - 1 + rows) / W, Nx = (W - 1 + cols) / W;
  binary_matrix P, P2;
  idx_t li = 0;
  for (idx_t i = 0; i < Ny; i++)
    for (idx_t j = 0; j < Nx; j++, li++) {
      const idx_t i0 = i * W, j0 = j * W;
      P = A.get_submatrix(i0, i0 + W, j0, j0 + W);
      idx_t bi = 0, bj = 0, bd = (idx_t)W * W;
      int i2;
      bool perfect = false;
      for (i2 = 0; (i2 <= int(i0 - W)) && !perfect; i2++)
        for (int j2 = 0; j2 < int(cols); j2++) {
          P2 = A.get_submatrix(i2, i2 + W, j2, j2 + W);
          const idx_t d = dist(P, P2);
          if (d < bd) { bd = d; bi = i2; bj = j2; }
          if (bd == 0) { perfect = true; break; }
        }
      for (; (i2 <= int(i0)) && !perfect; i2++)
        for (int j2 = 0; j2 <= int(j0 - W); j2++) {
          P2 = A.get_submatrix(i2, i2 + W, j2, j2 + W);
          const idx_t d = dist(P, P2);
          if (d < bd) { bd = d; bi = i2; bj = j2; }
          if (bd == 0) { perfect = true; break; }
        }
      besti[li] = (uint32_t)bi;
      bestj[li] = (uint32_t)bj;
      bestd[li] = (uint32_t)bd;
      if (wP) wP[li] = (uint32_t)P.weight();
    }
  P.destroy();
  P2.destroy();
  A.destroy();
  return 0;
}

extern "C" int ref_patch_search(const uint64_t* I, size_t rows, size_t cols, size_t wpr, unsigned W,
                                uint32_t* besti, uint32_t* bestj, uint32_t* bestd) {
  return ref_patch_search_w(I, rows, cols, wpr, W, besti, bestj, bestd, nullptr);
}

// compress6_test.cpp:62-78 prints its M x M predictor matrices (D: ones on the diagonal and the first
// superdiagonal; iD: the upper triangle) through the reference's operator<< (binmat.cpp:624-644) before
// set_grid_width is called (so with the default grid width). Those lines, into buf (NUL-terminated);
// returns their length, or -1 when cap is too small.
extern "C" long ref_print_pred_matrices(unsigned M, char* buf, size_t cap) {
  binary_matrix D(M, M), iD(M, M);
  D.clear();
  iD.clear();
  for (idx_t i = 0; i < M; i++) {
    D.set(i, i);
    if (i > 0) D.set(i - 1, i);
    for (idx_t j = i; j < M; j++) iD.set(i, j);
  }
  set_grid_width(10);  // binmat.cpp:618's initial value, what the driver prints with
  std::ostringstream os;
  os << "D:<<" << D << std::endl;
  os << "iD:<<" << iD << std::endl;
  D.destroy();
  iD.destroy();
  const std::string t = os.str();
  if (t.size() + 1 > cap) return -1;
  std::memcpy(buf, t.c_str(), t.size() + 1);
  return (long)t.size();
}

// write_pbm (pbm.cpp) of a plane given as words: the file a driver writes for its final image.
extern "C" int ref_write_pbm(const uint64_t* P, size_t rows, size_t cols, size_t wpr, const char* path) {
  binary_matrix A = from_words(P, rows, cols, wpr);
  FILE* o = fopen(path, "w");
  if (!o) { A.destroy(); return -1; }
  write_pbm(A, o);
  fclose(o);
  A.destroy();
  return 0;
}

// compress7_test.cpp:117-275 with search window R and threshold T on the reference's own
// binary_matrix (get_submatrix, dist, add, weight, set_submatrix), med (pred.cpp:3, the same
// formula as compress7's local med) and two GolombCoders. enumL(W*W, w) comes from the caller
// (GSL is absent here). The length expressions are the driver's, evaluated in double and
// converted to idx_t the same way; only ceil(log2(search_win_size)) for a size <= 0 (an undefined
// conversion on x86-64: 2^63) is taken as "no match" directly. dP / dP3 are cleared first (the
// driver leaves their (0,0) uninitialised). stats [4]: matches, bits match, bits nomatch, L.
// w4 (nullable): per tile the four weights the driver prints (compress7_test.cpp:191-209):
// nonmatch/nonpred, nonmatch/pred, match/nonpred, match/pred.
extern "C" int ref_match_loop_w4(uint64_t* Iw, size_t rows, size_t cols, size_t wpr, unsigned W, unsigned T,
                                 unsigned R, const double* enuml, uint32_t* besti, uint32_t* bestj,
                                 uint32_t* bestd, uint32_t* weights, char* modes, uint64_t* stats, uint32_t* w4) {
  binary_matrix I = from_words(Iw, rows, cols, wpr);
  const int iW = (int)W, iR = (int)R;
  const idx_t M = (idx_t)W * W;
  const idx_t Ny = (W - 1 + rows) / W, Nx = (W - 1 + cols) / W;
  binary_matrix P, P2;
  binary_matrix P3(W, W);
  GolombCoder golomb_match, golomb_nomatch;
  uint64_t L = 0, matches = 0;
  idx_t li = 0;
  for (idx_t i = 0; i < Ny; i++)
    for (idx_t j = 0; j < Nx; j++, li++) {
      const int i0 = i * W, j0 = j * W;
      P = I.get_submatrix(i0, i0 + W, j0, j0 + W);
      idx_t bi = 0, bj = 0, bd = M + 1;
      int i2;
      bool perfect = false;
      const int mini = i0 > iR ? (i0 - iR) : 0;
      const int minj = (j0 > iR) ? (j0 - iR) : 0;
      const int maxj = ((j0 + iR) > (int(cols) - iW)) ? (cols - W) : (j0 + iR);
      const int mini2 = (i0 > iW) ? (i0 - iW) : 0;
      const int maxj2 = (j0 > iW) ? (j0 - iW) : 0;
      const int swin = (i0 - mini2) * (maxj2 - minj) + (mini2 - mini) * (maxj - minj);
      for (i2 = i0; (i2 >= mini2) && !perfect; i2--)
        for (int j2 = maxj2; j2 >= minj; j2--) {
          P2 = I.get_submatrix(i2, i2 + W, j2, j2 + W);
          const idx_t d = dist(P, P2);
          if (d < bd) { bd = d; bi = i2; bj = j2; }
          if (bd <= T) { perfect = true; break; }
        }
      for (i2 = i0 - iW; (i2 >= mini) && !perfect; i2--)
        for (int j2 = maxj; j2 >= minj; j2--) {
          P2 = I.get_submatrix(i2, i2 + W, j2, j2 + W);
          const idx_t d = dist(P, P2);
          if (d < bd) { bd = d; bi = i2; bj = j2; }
          if (bd <= T) { perfect = true; break; }
        }
      if (bd <= M) {
        P2 = I.get_submatrix(bi, bi + W, bj, bj + W);
        add(P, P2, P3);
      } else {
        P3 = P.get_copy();
      }
      const idx_t w_mn = P3.weight(), w_nn = P.weight();
      binary_matrix dP(W, W), dP3(W, W);
      dP.clear();
      dP3.clear();
      med(P, dP);
      med(P3, dP3);
      const idx_t w_mp = dP3.weight(), w_np = dP.weight();
      if (w4) {
        w4[4 * li] = (uint32_t)w_nn;
        w4[4 * li + 1] = (uint32_t)w_np;
        w4[4 * li + 2] = (uint32_t)w_mn;
        w4[4 * li + 3] = (uint32_t)w_mp;
      }
      const bool ok = swin > 0;
      const idx_t idx_len = ok ? (idx_t)ceil(log2(swin)) : 0;
      const idx_t nn_len = 1 + 1 + enuml[w_nn], np_len = 1 + 1 + enuml[w_np];
      const idx_t mn_len = ok ? (idx_t)(1 + 1 + idx_len + enuml[w_mn]) : ~(idx_t)0;
      const idx_t mp_len = ok ? (idx_t)(1 + 1 + idx_len + enuml[w_mp]) : ~(idx_t)0;
      const bool mpred = mn_len > mp_len, npred = nn_len > np_len;
      const idx_t match_len = mpred ? mp_len : mn_len, nomatch_len = npred ? np_len : nn_len;
      const bool take = nomatch_len > match_len;
      idx_t w;
      if (take) {
        w = mpred ? w_mp : w_mn;
        golomb_match.codeSample(w);
        matches++;
        L += match_len;
        I.set_submatrix(i0, j0, mpred ? dP3 : P3);
      } else {
        w = npred ? w_np : w_nn;
        golomb_nomatch.codeSample(w);
        L += nomatch_len;
        I.set_submatrix(i0, j0, npred ? dP : P);
      }
      if (besti) besti[li] = (uint32_t)bi;
      if (bestj) bestj[li] = (uint32_t)bj;
      if (bestd) bestd[li] = (uint32_t)bd;
      if (weights) weights[li] = (uint32_t)w;
      if (modes) modes[li] = take ? (mpred ? 'X' : 'x') : (npred ? 'O' : 'o');
      dP.destroy();
      dP3.destroy();
    }
  to_words(I, Iw, wpr);
  if (stats) {
    stats[0] = matches;
    stats[1] = (uint64_t)golomb_match.bitcount;
    stats[2] = (uint64_t)golomb_nomatch.bitcount;
    stats[3] = L;
  }
  P.destroy();
  P2.destroy();
  I.destroy();
  return 0;
}

extern "C" int ref_match_loop(uint64_t* Iw, size_t rows, size_t cols, size_t wpr, unsigned W, unsigned T,
                              unsigned R, const double* enuml, uint32_t* besti, uint32_t* bestj,
                              uint32_t* bestd, uint32_t* weights, char* modes, uint64_t* stats) {
  return ref_match_loop_w4(Iw, rows, cols, wpr, W, T, R, enuml, besti, bestj, bestd, weights, modes, stats, nullptr);
}

// The tile loops of compress4_test.cpp:89-170 (variant 4), compress5_test.cpp:89-170 (5) and
// compress6_test.cpp:111-208 (6) over the reference's own objects (get_submatrix, dist, add, weight,
// set_submatrix, GolombCoder), statement for statement; enumL from the caller (GSL is absent).
// modes: 'x' match, 'o' no match.
// w2 (nullable): per tile P.weight() and the match weight (the drivers print both, through their lengths
// or directly: compress6_test.cpp:189-190).
extern "C" int ref_match_loop_var_w2(uint64_t* Iw, size_t rows, size_t cols, size_t wpr, unsigned W, unsigned T,
                                     unsigned R, const double* enuml, uint32_t* besti, uint32_t* bestj,
                                     uint32_t* bestd, uint32_t* weights, char* modes, uint64_t* stats, int variant,
                                     uint32_t* w2) {
  if (variant < 4 || variant > 6) return -1;
  binary_matrix I = from_words(Iw, rows, cols, wpr);
  const int iW = (int)W, iR = (int)R;
  const idx_t M = (idx_t)W * W;
  const idx_t Ny = (W - 1 + rows) / W, Nx = (W - 1 + cols) / W;
  binary_matrix P, P2;
  binary_matrix P3(W, W);
  GolombCoder golomb_match, golomb_nomatch;
  uint64_t L = 0, matches = 0;
  idx_t li = 0;
  for (idx_t i = 0; i < Ny; i++)
    for (idx_t j = 0; j < Nx; j++, li++) {
      const int i0 = i * W, j0 = j * W;
      P = I.get_submatrix(i0, i0 + W, j0, j0 + W);
      const idx_t worstd = W * W / 2;
      idx_t bi = 0, bj = 0, bd = M + 1;
      int i2;
      bool perfect = false;
      const int mini = i0 > iR ? (i0 - iR) : 0;
      const int mini2 = (i0 > iW) ? (i0 - iW) : 0;
      const int minj = (j0 > iR) ? (j0 - iR) : 0;
      const int maxj = ((j0 + iR) > (int(cols) - iW)) ? (cols - W) : (j0 + iR);
      for (i2 = i0; (i2 >= mini2) && !perfect; i2--)
        for (int j2 = int(j0 - W); j2 >= minj; j2--) {
          P2 = I.get_submatrix(i2, i2 + W, j2, j2 + W);
          const idx_t d = dist(P, P2);
          if (variant == 5 ? ((d - worstd) > (bd - worstd)) : (d < bd)) { bd = d; bi = i2; bj = j2; }
          if (bd <= T) { perfect = true; break; }
        }
      for (i2 = i0 - iW; (i2 >= mini) && !perfect; i2--)
        for (int j2 = maxj; j2 >= minj; j2--) {
          P2 = I.get_submatrix(i2, i2 + W, j2, j2 + W);
          const idx_t d = dist(P, P2);
          if (variant == 5 ? ((d - worstd) > (bd - worstd)) : (d < bd)) { bd = d; bi = i2; bj = j2; }
          if (bd <= T) { perfect = true; break; }
        }
      idx_t match_len, nomatch_len, match_weight;
      const idx_t idx_len = ceil(log2(li));
      if (variant == 6) {  // compress6_test.cpp:166-194
        if (bd <= M) {
          P2 = I.get_submatrix(bi, bi + W, bj, bj + W);
          add(P, P2, P3);
        } else {
          P3 = P.get_copy();
        }
        match_weight = P3.weight();
        nomatch_len = 1 + enuml[P.weight()];
        match_len = 1 + idx_len + enuml[match_weight];
      } else {  // compress4_test.cpp:143-155
        P2 = I.get_submatrix(bi, bi + W, bj, bj + W);
        add(P, P2, P3);
        match_weight = bd;
        nomatch_len = 1 + enuml[P.weight()];
        match_len = (bd <= M) ? (idx_t)(1 + idx_len + enuml[bd]) : 100000;
      }
      const idx_t wP = P.weight();
      if (w2) {
        w2[2 * li] = (uint32_t)wP;
        w2[2 * li + 1] = (uint32_t)match_weight;
      }
      const bool take = nomatch_len > match_len;
      if (take) {
        golomb_match.codeSample(match_weight);
        matches++;
        L += match_len;
        I.set_submatrix(i0, j0, P3);
      } else {
        golomb_nomatch.codeSample(wP);
        L += nomatch_len;
      }
      if (besti) besti[li] = (uint32_t)bi;
      if (bestj) bestj[li] = (uint32_t)bj;
      if (bestd) bestd[li] = (uint32_t)bd;
      if (weights) weights[li] = (uint32_t)(take ? match_weight : wP);
      if (modes) modes[li] = take ? 'x' : 'o';
    }
  to_words(I, Iw, wpr);
  if (stats) {
    stats[0] = matches;
    stats[1] = (uint64_t)golomb_match.bitcount;
    stats[2] = (uint64_t)golomb_nomatch.bitcount;
    stats[3] = L;
  }
  P.destroy();
  P2.destroy();
  P3.destroy();
  I.destroy();
  return 0;
}

extern "C" int ref_match_loop_var(uint64_t* Iw, size_t rows, size_t cols, size_t wpr, unsigned W, unsigned T,
                                  unsigned R, const double* enuml, uint32_t* besti, uint32_t* bestj,
                                  uint32_t* bestd, uint32_t* weights, char* modes, uint64_t* stats, int variant) {
  return ref_match_loop_var_w2(Iw, rows, cols, wpr, W, T, R, enuml, besti, bestj, bestd, weights, modes, stats,
                               variant, nullptr);
}

// compress8_test.cpp:126-272's tile loop over the reference's own objects (get_submatrix, dist,
// flip, add, med, weight, set_submatrix, GolombCoder); enumL from the caller (GSL is absent). As
// written except that a window's `inv` (left uninitialised by the driver when the window is not
// inverted, :157) is false. inverted (nullable): bestinv per tile.
extern "C" int ref_match_loop8(uint64_t* Iw, size_t rows, size_t cols, size_t wpr, unsigned W, unsigned T,
                               unsigned R, const double* enuml, uint32_t* besti, uint32_t* bestj,
                               uint32_t* bestd, uint32_t* weights, char* modes, uint8_t* inverted,
                               uint64_t* stats) {
  binary_matrix I = from_words(Iw, rows, cols, wpr);
  const int iW = (int)W, iR = (int)R;
  const idx_t M = (idx_t)W * W;
  const idx_t Tt = T;
  const idx_t Ny = (W - 1 + rows) / W, Nx = (W - 1 + cols) / W;
  binary_matrix P, P2;
  binary_matrix P3(W, W);
  GolombCoder golomb_match, golomb_nomatch;
  uint64_t L = 0, matches = 0;
  idx_t li = 0;
  for (idx_t i = 0; i < Ny; i++)
    for (idx_t j = 0; j < Nx; j++, li++) {
      const int i0 = i * W, j0 = j * W;
      int i2;
      P = I.get_submatrix(i0, i0 + W, j0, j0 + W);
      idx_t bi = 0, bj = 0, bd = M + 1;
      bool bestinv = (P.weight() - M) < (P.weight());
      bool perfect = (P.weight() <= Tt) || (P.weight() >= (M - Tt));
      const int mini = i0 > iR ? (i0 - iR) : 0;
      const int minj = (j0 > iR) ? (j0 - iR) : 0;
      const int maxj = ((j0 + iR) > (int(cols) - iW)) ? (cols - W) : (j0 + iR);
      const int mini2 = (i0 > iW) ? (i0 - iW) : 0;
      const int maxj2 = (j0 > iW) ? (j0 - iW) : 0;
      const int swin = (i0 - mini2) * (maxj2 - minj) + (mini2 - mini) * (maxj - minj);
      for (int loop = 0; loop < 2; ++loop) {
        const int ihi = loop ? i0 - iW : i0, ilo = loop ? mini : mini2, jhi = loop ? maxj : maxj2;
        for (i2 = ihi; (i2 >= ilo) && !perfect; i2--)
          for (int j2 = jhi; j2 >= minj; j2--) {
            P2 = I.get_submatrix(i2, i2 + W, j2, j2 + W);
            idx_t d = dist(P, P2);
            bool inv = false;
            if ((M - d) < d) {
              inv = true;
              d = M - d;
            }
            if (d < bd) {
              bestinv = inv;
              bd = d;
              bi = i2;
              bj = j2;
              if (bd <= Tt) {
                perfect = true;
                break;
              }
            }
          }
      }
      if (bestinv) P.flip();
      if (bd <= M) {
        P2 = I.get_submatrix(bi, bi + W, bj, bj + W);
        add(P, P2, P3);
      } else {
        P3 = P.get_copy();
      }
      const idx_t w_mn = P3.weight(), w_nn = P.weight();
      binary_matrix dP(W, W), dP3(W, W);
      dP.clear();
      dP3.clear();
      med(P, dP);
      med(P3, dP3);
      const idx_t w_mp = dP3.weight(), w_np = dP.weight();
      const bool ok = swin > 0;
      const idx_t idx_len = ok ? (idx_t)ceil(log2(swin)) : 0;
      const idx_t nn_len = 2 + enuml[w_nn], np_len = 2 + enuml[w_np];
      const idx_t mn_len = ok ? (idx_t)(3 + idx_len + enuml[w_mn]) : ~(idx_t)0;
      const idx_t mp_len = ok ? (idx_t)(3 + idx_len + enuml[w_mp]) : ~(idx_t)0;
      const bool mpred = mn_len > mp_len, npred = nn_len > np_len;
      const idx_t match_len = mpred ? mp_len : mn_len, nomatch_len = npred ? np_len : nn_len;
      const bool take = nomatch_len > match_len;
      idx_t w;
      if (take) {
        w = mpred ? w_mp : w_mn;
        golomb_match.codeSample(w);
        matches++;
        L += match_len;
        I.set_submatrix(i0, j0, mpred ? dP3 : P3);
      } else {
        w = npred ? w_np : w_nn;
        golomb_nomatch.codeSample(w);
        L += nomatch_len;
        I.set_submatrix(i0, j0, npred ? dP : P);
      }
      if (besti) besti[li] = (uint32_t)bi;
      if (bestj) bestj[li] = (uint32_t)bj;
      if (bestd) bestd[li] = (uint32_t)bd;
      if (weights) weights[li] = (uint32_t)w;
      if (modes) modes[li] = take ? (mpred ? 'X' : 'x') : (npred ? 'O' : 'o');
      if (inverted) inverted[li] = bestinv ? 1 : 0;
      dP.destroy();
      dP3.destroy();
    }
  to_words(I, Iw, wpr);
  if (stats) {
    stats[0] = matches;
    stats[1] = (uint64_t)golomb_match.bitcount;
    stats[2] = (uint64_t)golomb_nomatch.bitcount;
    stats[3] = L;
  }
  P.destroy();
  P2.destroy();
  I.destroy();
  return 0;
}

// binary_matrix algebra on the reference's own objects (binmat.cpp:199-214, 516-616): C starts as
// Cin (mul_ABt keeps bits), words in the reference layout (wpr = ceil(cols/64), padding bits 0).
extern "C" int ref_gf2_mul(int op, const uint64_t* A, size_t a_rows, size_t a_cols, const uint64_t* B,
                           size_t b_rows, size_t b_cols, uint64_t* C, size_t c_rows, size_t c_cols) {
  binary_matrix Am = from_words(A, a_rows, a_cols, (a_cols + 63) / 64);
  binary_matrix Bm = from_words(B, b_rows, b_cols, (b_cols + 63) / 64);
  binary_matrix Cm = from_words(C, c_rows, c_cols, (c_cols + 63) / 64);
  // mul_ABt's block_sum XORs the word's bytes into one shared variable from an OpenMP parallel for
  // (binmat.cpp:48-52, a data race): with one thread it is the parity it is meant to be
  const int nt = omp_get_max_threads();
  omp_set_num_threads(1);
  mul(Am, op == 1 || op == 3, Bm, op == 2 || op == 3, Cm);
  omp_set_num_threads(nt);
  to_words(Cm, C, (c_cols + 63) / 64);
  return 0;
}

extern "C" int ref_gf2_transpose(const uint64_t* src, size_t rows, size_t cols, uint64_t* dst) {
  binary_matrix Am = from_words(src, rows, cols, (cols + 63) / 64);
  binary_matrix T(cols, rows);
  Am.transpose_to(T);
  to_words(T, dst, (rows + 63) / 64);
  return 0;
}
