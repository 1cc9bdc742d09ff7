// host_api_check.cpp -- test program for the C++ reference API (include/*.h, libbicpp.so),
// driven by tests/test_host_api.py. Written the way a reference user would write it: planes in
// binary_matrix, runs fed to GolombCoder::codeSample / EGCoder::codeRun, PBM/PGM through pbm.h /
// pnm.h. Modes:
//   kat                                  coder known answers (no device)
//   decode <coder> <rows> <cols> <bits> <stream> <out.pbm>     stream -> residual plane
//   unmed <resid.pbm> <p00> <out.pbm>    inverse predictor
//   gpu <in.pgm> <outdir>                GPU path: bitplanes, med, encode, tiles; self-checks
//                                        against the reference coders and the decoders, writes
//                                        planes and streams for the oracle comparison
#include <chrono>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <string>
#include <vector>

#include "GolombCoder.h"
#include "bic_decode.h"
#include "bic_gpu.h"
#include "coding.h"
#include "eg.h"
#include "pbm.h"
#include "pnm.h"
#include "pred.h"

namespace {

int failures = 0;

#define CHECK(cond, ...)                                   \
  do {                                                     \
    if (!(cond)) {                                         \
      std::printf("FAIL %s:%d: ", __FILE__, __LINE__);     \
      std::printf(__VA_ARGS__);                            \
      std::printf("\n");                                   \
      ++failures;                                          \
    }                                                      \
  } while (0)

// the runs of a plane, coded sample by sample with the reference-API coders
void code_runs(const binary_matrix& R, GolombCoder* g, EGCoder* e) {
  for (idx_t i = 0; i < R.get_rows(); ++i) {
    unsigned run = 0;
    for (idx_t j = 0; j < R.get_cols(); ++j) {
      if (!R.get(i, j)) {
        ++run;
        continue;
      }
      if (g) g->codeSample(run);
      if (e) e->codeRun((int)run, false);
      run = 0;
    }
    if (g) g->codeSample(run);
    if (e) e->codeRun((int)run, true);
  }
}

binary_matrix read_pbm_file(const char* path) {
  FILE* f = std::fopen(path, "r");
  if (!f) {
    std::printf("cannot open %s\n", path);
    std::exit(2);
  }
  idx_t rows = 0, cols = 0;
  if (read_pbm_header(f, rows, cols) != PBM_OK) std::exit(2);
  binary_matrix A(rows, cols);
  read_pbm_data(f, A);
  std::fclose(f);
  return A;
}

std::vector<uint8_t> read_file(const char* path) {
  std::vector<uint8_t> b;
  FILE* f = std::fopen(path, "rb");
  if (!f) return b;
  int c;
  while ((c = std::fgetc(f)) != EOF) b.push_back((uint8_t)c);
  std::fclose(f);
  return b;
}

void write_file(const std::string& path, const std::vector<uint8_t>& b) {
  FILE* f = std::fopen(path.c_str(), "wb");
  if (!b.empty()) std::fwrite(b.data(), 1, b.size(), f);
  std::fclose(f);
}

struct Probe : GolombCoder {  // exposes the protected state for the known-answer test
  unsigned kk() const { return k; }
};

int kat() {
  // SURVEY.md §8 c known answer: k sequence and lengths of GolombCoder on these samples
  const unsigned s[] = {0, 0, 0, 5, 3, 0, 12, 1, 100, 7, 0, 0, 1, 2, 3};
  const unsigned ks[] = {1, 0, 0, 0, 1, 1, 1, 2, 2, 4, 4, 4, 4, 4, 4};
  const unsigned len[] = {2, 1, 1, 6, 3, 2, 8, 3, 28, 5, 5, 5, 5, 5, 5};
  Probe g;
  long before = 0;
  for (int i = 0; i < 15; ++i) {
    CHECK(g.kk() == ks[i], "k[%d] = %u, expected %u", i, g.kk(), ks[i]);
    g.codeSample(s[i]);
    CHECK(g.bitcount - before == (long)len[i], "len[%d]", i);
    before = g.bitcount;
  }
  CHECK(g.bitcount == 84, "golomb total %ld", g.bitcount);
  EGCoder e;
  e.codeRun(3, false);
  e.codeRun(0, false);
  e.codeRun(7, true);
  e.codeRun(2, true);
  CHECK(e.bitcount == 17, "eg total %lu", e.bitcount);
  CHECK(e.g == 0 && e.blockSize == 1, "eg state");
  CHECK(enumerative_codelength(1024, 0) == 0.0, "enum r=0");
  CHECK(enumerative_codelength(1024, 1) == 10.0, "enum r=1");
  CHECK(bic::planes_for_maxval(255) == 8 && bic::planes_for_maxval(256) == 8 && bic::planes_for_maxval(257) == 9,
        "planes_for_maxval");
  std::printf("kat %s\n", failures ? "FAILED" : "ok");
  return failures ? 1 : 0;
}

int decode(int argc, char** argv) {
  if (argc < 8) return 2;
  const int coder = std::atoi(argv[2]);
  const idx_t rows = std::strtoul(argv[3], nullptr, 10), cols = std::strtoul(argv[4], nullptr, 10);
  const uint64_t bits = std::strtoull(argv[5], nullptr, 10);
  std::vector<uint8_t> s = read_file(argv[6]);
  binary_matrix R(rows, cols);
  const int rc = bic::decode_plane(s.data(), bits, coder, R);
  FILE* f = std::fopen(argv[7], "w");
  write_pbm(R, f);
  std::fclose(f);
  R.destroy();
  std::printf("decode rc=%d\n", rc);
  return rc ? 1 : 0;
}

int unmed_cmd(int argc, char** argv) {
  if (argc < 5) return 2;
  binary_matrix R = read_pbm_file(argv[2]);
  binary_matrix P(R.get_rows(), R.get_cols());
  bic::unmed(R, std::atoi(argv[3]) != 0, P);
  FILE* f = std::fopen(argv[4], "w");
  write_pbm(P, f);
  std::fclose(f);
  return 0;
}

int gpu(int argc, char** argv) {
  if (argc < 4) return 2;
  const std::string out = argv[3];
  FILE* f = std::fopen(argv[2], "r");
  int type = 0, rows = 0, cols = 0, maxval = 0;
  if (!f || read_pnm_header(f, type, cols, rows, maxval)) return 2;
  std::vector<pixel_t> gray((size_t)rows * cols);
  read_pgm_data(f, type, cols, rows, maxval, gray.data());
  std::fclose(f);
  const int np = bic::planes_for_maxval(maxval);

  bic::Device dev(0);
  CHECK(dev.status() == BIC_OK, "device: %s", bic_strerror(dev.status()));
  if (dev.status() != BIC_OK) return 1;

  // bitplanes on the device vs the reference's per-pixel loop (bitplane_tool.cpp:24-30)
  std::vector<binary_matrix> planes;
  planes.reserve(np);
  for (int p = 0; p < np; ++p) planes.emplace_back(rows, cols);
  CHECK(dev.bitplanes(gray.data(), rows, cols, np, planes.data()) == BIC_OK, "bitplanes");
  binary_matrix A(rows, cols);
  for (int p = 0, b = 1; p < np; ++p, b <<= 1) {
    for (int i = 0, li = 0; i < rows; ++i)
      for (int j = 0; j < cols; ++j, ++li) A.set(i, j, gray[li] & b);
    CHECK(dist(A, planes[p]) == 0, "plane %d differs from the per-pixel loop", p);
    char name[64];
    std::snprintf(name, sizeof(name), "/plane_%02d.pbm", p);
    FILE* pf = std::fopen((out + name).c_str(), "w");
    write_pbm(planes[p], pf);
    std::fclose(pf);
  }

  // med on the device: pP(0,0) and pad bits keep their old contents
  for (int p = 0; p < np; ++p) {
    binary_matrix R(rows, cols);
    R.set();
    med(planes[p], R);
    CHECK(R.get(0, 0), "med wrote pP(0,0)");
    idx_t w = 0;
    binary_matrix R2(rows, cols);
    R2.clear();
    CHECK(dev.med(planes[p], R2, &w) == BIC_OK, "Device::med");
    CHECK(R2.weight() == w, "med weight %lu vs %lu", R2.weight(), w);
    R.clear(0, 0);
    CHECK(dist(R, R2) == 0, "med residual differs between calls");
    // inverse predictor restores the plane
    binary_matrix back(rows, cols);
    bic::unmed(R2, planes[p].get(0, 0), back);
    CHECK(dist(back, planes[p]) == 0, "unmed(med(P)) != P for plane %d", p);
    R.destroy();
    R2.destroy();
    back.destroy();
  }

  // whole-plane encode vs the per-sample reference coders, both predict modes
  for (int predict = 0; predict < 2; ++predict) {
    std::vector<GolombCoder> g(np);
    std::vector<EGCoder> e(np);
    std::vector<bic::Stream> gs, es;
    CHECK(dev.encode(planes.data(), np, predict != 0, g.data(), &gs, e.data(), &es) == BIC_OK, "encode");
    for (int p = 0; p < np; ++p) {
      binary_matrix R(rows, cols);
      if (predict) {
        R.clear();
        med(planes[p], R);
      } else {
        planes[p].copy_to(R);
      }
      GolombCoder g_ref;
      EGCoder e_ref;
      code_runs(R, &g_ref, &e_ref);
      CHECK(g[p].bitcount == g_ref.bitcount, "golomb bits plane %d: %ld vs %ld", p, g[p].bitcount, g_ref.bitcount);
      CHECK(e[p].bitcount == e_ref.bitcount, "eg bits plane %d", p);
      CHECK((uint64_t)g[p].bitcount == gs[p].bits && e[p].bitcount == es[p].bits, "stream lengths");
      CHECK(bic::coder_state::k(g[p]) == bic::coder_state::k(g_ref) &&
                bic::coder_state::samples(g[p]) == bic::coder_state::samples(g_ref) &&
                bic::coder_state::accumulated(g[p]) == bic::coder_state::accumulated(g_ref),
            "golomb state plane %d", p);
      CHECK(e[p].g == e_ref.g && e[p].blockSize == e_ref.blockSize && e[p].lutIndex == e_ref.lutIndex,
            "eg state plane %d", p);
      for (int c = 0; c < 2; ++c) {
        const bic::Stream& s = c ? es[p] : gs[p];
        binary_matrix D(rows, cols);
        CHECK(bic::decode_plane(s.bytes.data(), s.bits, c, D) == 0, "decode plane %d coder %d", p, c);
        CHECK(dist(D, R) == 0, "decoded residual differs, plane %d coder %d", p, c);
        D.destroy();
        char name[64];
        std::snprintf(name, sizeof(name), "/stream_%c%d_%02d.bin", c ? 'e' : 'g', predict, p);
        write_file(out + name, s.bytes);
      }
      R.destroy();
    }
  }

  // the sample coder continues a coder's state exactly like repeated codeSample calls
  {
    std::vector<unsigned> s(5000);
    unsigned x = 12345;
    for (auto& v : s) {
      x = x * 1103515245u + 12345u;
      v = (x >> 16) % 37;
    }
    GolombCoder a, b;
    for (int i = 0; i < 100; ++i) a.codeSample(s[i]), b.codeSample(s[i]);
    bic::Stream st;
    CHECK(dev.code_samples(a, s.data() + 100, s.size() - 100, &st) == BIC_OK, "code_samples");
    for (size_t i = 100; i < s.size(); ++i) b.codeSample(s[i]);
    CHECK(a.bitcount == b.bitcount, "code_samples bits %ld vs %ld", a.bitcount, b.bitcount);
    CHECK(bic::coder_state::k(a) == bic::coder_state::k(b), "code_samples k");
  }

  // tiles (compress7 R = 0): chosen weights Golomb-coded like golomb_nomatch.codeSample
  if (rows % 8 == 0 && cols % 8 == 0) {
    bic::TileResult t;
    CHECK(dev.tiles(planes[0], 8, &t) == BIC_OK, "tiles");
    GolombCoder gt;
    for (size_t i = 0; i < t.weights.size(); ++i) {
      CHECK(t.weights[i] == (t.modes[i] == 'O' ? t.w_pred[i] : t.w_nonpred[i]), "tile %zu mode", i);
      gt.codeSample(t.weights[i]);
    }
    CHECK((uint64_t)gt.bitcount == t.stream.bits, "tile stream bits");
  }

  // compress_test.cpp's search, written with the reference API (get_submatrix, dist) as the
  // driver does, against the GPU search on plane 0
  {
    const unsigned W = 5;
    std::vector<uint32_t> bi, bj, bd;
    CHECK(dev.patch_search(planes[0], W, &bi, &bj, &bd) == BIC_OK, "patch_search");
    const idx_t Ny = (W - 1 + rows) / W, Nx = (W - 1 + cols) / W;
    binary_matrix P, P2;
    idx_t li = 0;
    const binary_matrix& I = planes[0];
    for (idx_t i = 0; i < Ny && li < 40; i++)
      for (idx_t j = 0; j < Nx && li < 40; j++, li++) {
        const idx_t i0 = i * W, j0 = j * W;
        P = I.get_submatrix(i0, i0 + W, j0, j0 + W);
        idx_t besti = 0, bestj = 0, bestd = W * W;
        int i2;
        bool perfect = false;
        for (i2 = 0; (i2 <= int(i0 - W)) && !perfect; i2++)
          for (int j2 = 0; j2 < int(cols); j2++) {
            P2 = I.get_submatrix(i2, i2 + W, j2, j2 + W);
            const idx_t d = dist(P, P2);
            if (d < bestd) { bestd = d; besti = i2; bestj = j2; }
            if (bestd == 0) { perfect = true; break; }
          }
        for (; (i2 <= int(i0)) && !perfect; i2++)
          for (int j2 = 0; j2 <= int(j0 - W); j2++) {
            P2 = I.get_submatrix(i2, i2 + W, j2, j2 + W);
            const idx_t d = dist(P, P2);
            if (d < bestd) { bestd = d; besti = i2; bestj = j2; }
            if (bestd == 0) { perfect = true; break; }
          }
        CHECK(bi[li] == besti && bj[li] == bestj && bd[li] == bestd, "patch search tile %lu", li);
      }
    P.destroy();
    P2.destroy();
  }

  // compress7_test.cpp's loop with a search window, written with this build's reference API as
  // the driver writes it (get_submatrix, dist, add, med, weight, set_submatrix, GolombCoder),
  // against bic::Device::match_encode on the top-left multiple-of-W part of plane np-1
  {
    const unsigned W = 8, T = 1, R = 24;
    const idx_t mr = rows / W * W, mc = cols / W * W;
    if (mr && mc) {
      binary_matrix I = planes[np - 1].get_submatrix(0, mr, 0, mc), I2 = I.get_copy();
      const idx_t M = W * W;
      std::vector<double> e(M + 1);
      for (idx_t w = 0; w <= M; ++w) e[w] = enumerative_codelength(M, w);
      bic::MatchResult res;
      GolombCoder gm_gpu, gn_gpu;
      CHECK(dev.match_encode(I2, W, T, R, &res, &gm_gpu, &gn_gpu, e.data()) == BIC_OK, "match_encode");
      GolombCoder golomb_match, golomb_nomatch;
      binary_matrix P, P2, P3(W, W);
      idx_t li = 0, matches = 0, L = 0;
      const int iW = W, iR = R;
      for (idx_t i = 0; i < mr / W; i++)
        for (idx_t j = 0; j < mc / W; j++, li++) {
          const int i0 = i * W, j0 = j * W;
          P = I.get_submatrix(i0, i0 + W, j0, j0 + W);
          idx_t besti = 0, bestj = 0, bestd = M + 1;
          int i2;
          bool perfect = false;
          const int mini = i0 > iR ? i0 - iR : 0, minj = j0 > iR ? j0 - iR : 0;
          const int maxj = (j0 + iR > int(mc) - iW) ? int(mc) - iW : j0 + iR;
          const int mini2 = i0 > iW ? i0 - iW : 0, maxj2 = j0 > iW ? j0 - iW : 0;
          const int swin = (i0 - mini2) * (maxj2 - minj) + (mini2 - mini) * (maxj - minj);
          for (i2 = i0; i2 >= mini2 && !perfect; i2--)
            for (int j2 = maxj2; j2 >= minj; j2--) {
              P2 = I.get_submatrix(i2, i2 + W, j2, j2 + W);
              const idx_t d = dist(P, P2);
              if (d < bestd) { bestd = d; besti = i2; bestj = j2; }
              if (bestd <= T) { perfect = true; break; }
            }
          for (i2 = i0 - iW; i2 >= mini && !perfect; i2--)
            for (int j2 = maxj; j2 >= minj; j2--) {
              P2 = I.get_submatrix(i2, i2 + W, j2, j2 + W);
              const idx_t d = dist(P, P2);
              if (d < bestd) { bestd = d; besti = i2; bestj = j2; }
              if (bestd <= T) { perfect = true; break; }
            }
          if (bestd <= M) {
            P2 = I.get_submatrix(besti, besti + W, bestj, bestj + W);
            add(P, P2, P3);
          } else {
            P3 = P.get_copy();
          }
          binary_matrix dP(W, W), dP3(W, W);
          med(P, dP);
          med(P3, dP3);
          const idx_t wmn = P3.weight(), wnn = P.weight(), wmp = dP3.weight(), wnp = dP.weight();
          const bool ok = swin > 0;
          const idx_t idx_len = ok ? (idx_t)ceil(log2(swin)) : 0;
          const idx_t nn = 1 + 1 + e[wnn], np_ = 1 + 1 + e[wnp];
          const idx_t mn = ok ? (idx_t)(1 + 1 + idx_len + e[wmn]) : ~(idx_t)0;
          const idx_t mp = ok ? (idx_t)(1 + 1 + idx_len + e[wmp]) : ~(idx_t)0;
          const bool mpred = mn > mp, npred = nn > np_;
          const idx_t mlen = mpred ? mp : mn, nlen = npred ? np_ : nn;
          const bool take = nlen > mlen;
          const idx_t w = take ? (mpred ? wmp : wmn) : (npred ? wnp : wnn);
          if (take) {
            golomb_match.codeSample(w);
            matches++;
            L += mlen;
            I.set_submatrix(i0, j0, mpred ? dP3 : P3);
          } else {
            golomb_nomatch.codeSample(w);
            L += nlen;
            I.set_submatrix(i0, j0, npred ? dP : P);
          }
          const char mode = take ? (mpred ? 'X' : 'x') : (npred ? 'O' : 'o');
          CHECK(res.besti[li] == besti && res.bestj[li] == bestj && res.bestd[li] == bestd && res.weights[li] == w &&
                    res.modes[li] == (uint8_t)mode, "match tile %lu", li);
          dP.destroy();
          dP3.destroy();
        }
      CHECK(dist(I, I2) == 0, "match residual image");
      CHECK(res.matches == matches && res.L == L, "match totals");
      CHECK(gm_gpu.bitcount == golomb_match.bitcount && gn_gpu.bitcount == golomb_nomatch.bitcount,
            "match coders: %ld %ld vs %ld %ld", gm_gpu.bitcount, gn_gpu.bitcount, golomb_match.bitcount,
            golomb_nomatch.bitcount);
      CHECK(bic::coder_state::k(gm_gpu) == bic::coder_state::k(golomb_match) &&
                bic::coder_state::k(gn_gpu) == bic::coder_state::k(golomb_nomatch),
            "match coder state");
      I.destroy();
      I2.destroy();
      P.destroy();
      P2.destroy();
    }
  }

  for (auto& p : planes) p.destroy();
  A.destroy();
  std::printf("gpu %s planes=%d\n", failures ? "FAILED" : "ok", np);
  return failures ? 1 : 0;
}

// The compress7_test.cpp:205-206 call pattern: med() on n separate W x W tiles, each call a full
// round trip to the device (copy in, kernel, copy out). Prints the time per call; checks the tiles
// against the word-form med restated here (the host never computes med for the product).
int medcalls(int argc, char** argv) {
  const int n = argc > 2 ? std::atoi(argv[2]) : 65536, W = argc > 3 ? std::atoi(argv[3]) : 32;
  binary_matrix P(W, W), R(W, W);
  uint64_t s = 0x5EED;
  auto rnd = [&]() {
    s += 0x9E3779B97F4A7C15ull;
    uint64_t z = s;
    z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ull;
    z = (z ^ (z >> 27)) * 0x94D049BB133111EBull;
    return z ^ (z >> 31);
  };
  long bad = 0;
  med(P, R);  // the first call pays the context creation
  const auto t0 = std::chrono::steady_clock::now();
  for (int t = 0; t < n; ++t) {
    block_t* p = P.raw_blocks();
    for (idx_t i = 0; i < (idx_t)W; ++i) p[i * P.get_blocks_per_row()] = rnd() & (W == 64 ? ~0ull : ~(~0ull >> W));
    med(P, R);
    if (t % 4096 == 0) {  // spot check: R(i,j) = P(i-1,j-1)^P(i,j-1)^P(i-1,j)^P(i,j), R(0,0) kept
      for (idx_t i = 0; i < (idx_t)W; ++i)
        for (idx_t j = 0; j < (idx_t)W; ++j) {
          if (i == 0 && j == 0) continue;
          int e = P.get(i, j);
          if (j) e ^= P.get(i, j - 1);
          if (i) e ^= P.get(i - 1, j);
          if (i && j) e ^= P.get(i - 1, j - 1);
          bad += e != R.get(i, j);
        }
    }
  }
  const double dt = std::chrono::duration<double>(std::chrono::steady_clock::now() - t0).count();
  std::printf("medcalls n=%d W=%d us_per_call=%.2f total_s=%.3f bad=%ld\n", n, W, dt / n * 1e6, dt, bad);
  P.destroy();
  R.destroy();
  return bad ? 1 : 0;
}

}  // namespace

int main(int argc, char** argv) {
  if (argc < 2) return 2;
  const std::string mode = argv[1];
  if (mode == "kat") return kat();
  if (mode == "decode") return decode(argc, argv);
  if (mode == "unmed") return unmed_cmd(argc, argv);
  if (mode == "gpu") return gpu(argc, argv);
  if (mode == "medcalls") return medcalls(argc, argv);
  return 2;
}
