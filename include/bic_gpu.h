// bic_gpu.h -- the reference C++ API's hot path on an MI355X: what bitplane_tool.cpp, pred.cpp
// and GolombCoder / EGCoder do pixel by pixel on the host, done for whole planes by the HIP
// kernels behind bic.h. Host matrices (binmat.h) are copied to the device as they are (their
// storage already is the kernels' plane layout), results are copied back.
//
// Every call returns a bic.h status code (BIC_OK = 0). A Device whose status() is not BIC_OK
// (no gfx950 GPU, no HIP runtime) fails every call with that code; nothing falls back to the CPU.
#ifndef BIC_GPU_H
#define BIC_GPU_H

#include <stdint.h>

#include <vector>

#include "GolombCoder.h"
#include "bic.h"
#include "binmat.h"
#include "eg.h"
#include "pnm.h"

namespace bic {

// One encoded stream: MSB-first bits, zero-padded to a whole byte.
struct Stream {
  std::vector<uint8_t> bytes;
  uint64_t bits = 0;
};

// Reads and advances the protected state of the reference coders (friend of Golomb and EG).
struct coder_state {
  static bool fresh(const GolombCoder& c) { return c.samples == 0 && c.accumulatedError == 0 && c.k == 1; }
  static bool fresh(const EGCoder& e) { return e.g == 1 && e.blockSize == 1 && e.lutIndex == 0; }
  static unsigned samples(const GolombCoder& c) { return c.samples; }
  static unsigned accumulated(const GolombCoder& c) { return c.accumulatedError; }
  static unsigned k(const GolombCoder& c) { return c.k; }
  // the state codeSample leaves after `n` more samples summing to `sum` that cost `bits` bits
  static void advance(GolombCoder& c, uint64_t n, uint64_t sum, uint64_t bits);
  // the state codeRun leaves after a plane: `ones` non-EOL runs, `bits` bits
  static void advance(EGCoder& e, uint64_t ones, uint64_t bits);
};

// Number of planes bitplane_tool.cpp:24 writes for a maxval: #{bi : 2^bi < maxval}.
int planes_for_maxval(int maxval);

// Result of the W x W tile path (compress7_test.cpp:184-275 with R = 0), one entry per tile in
// raster order.
struct TileResult {
  std::vector<uint32_t> weights;    // the weight that was Golomb-coded (w_pred if 'O' else w_nonpred)
  std::vector<uint32_t> w_nonpred;  // P.weight()
  std::vector<uint32_t> w_pred;     // med(P).weight()
  std::vector<uint8_t> modes;       // 'o' or 'O'
  Stream stream;                    // golomb_nomatch's codewords
  uint64_t L = 0;                   // sum of lentab[chosen weight]
};

// Result of compress7_test.cpp's tile loop with a search window (Device::match_encode), per tile
// in raster order, plus the state the driver's two GolombCoders end in.
struct MatchResult {
  std::vector<uint32_t> besti, bestj, bestd;  // the search (:184; bestd = W*W+1: empty region)
  std::vector<uint32_t> weights;              // the coded weight
  std::vector<uint8_t> modes;                 // 'X' 'x' (match) or 'O' 'o'
  Stream stream_match, stream_nomatch;        // golomb_match / golomb_nomatch codewords
  uint64_t matches = 0, L = 0;                // L: sum of the chosen lengths (before the bitcounts)
};

class Device {
 public:
  explicit Device(int ordinal = 0);
  ~Device();
  Device(const Device&) = delete;
  Device& operator=(const Device&) = delete;

  int status() const { return status_; }
  bic_ctx* ctx() { return ctx_; }

  // bitplane_tool.cpp:24-30: planes[bi](i,j) = (gray[i*cols+j] >> bi) & 1 for bi < nplanes
  // (1..32). Each planes[bi] must be allocated rows x cols.
  int bitplanes(const pixel_t* gray, idx_t rows, idx_t cols, int nplanes, binary_matrix* planes);

  // pred.cpp:3-15 into R (allocated like P); R(0,0) and R's pad bits keep their old values.
  // weight (nullable) receives the number of residual ones in R outside (0,0).
  int med(const binary_matrix& P, binary_matrix& R, idx_t* weight = nullptr);

  // Runs of every plane (one sample per 1-pixel and one end-of-row sample per row, raster
  // order) coded with a fresh coder per plane: GolombCoder::codeSample (golomb != nullptr) and/or
  // EGCoder::codeRun (eg != nullptr), of the med residual (predict) or of the plane itself.
  // golomb / eg point to nplanes coders that must be fresh; on return they hold the state and
  // bitcount the reference coders would have after coding the same runs. Streams are optional.
  int encode(const binary_matrix* planes, int nplanes, bool predict, GolombCoder* golomb,
             std::vector<Stream>* golomb_streams, EGCoder* eg, std::vector<Stream>* eg_streams);

  // GolombCoder::codeSample over samples[0..n), continuing from the coder's current state.
  int code_samples(GolombCoder& coder, const unsigned* samples, size_t n, Stream* stream = nullptr);

  // The tile path over I (rows and cols multiples of W, 1 <= W <= 64). lentab[w] =
  // (idx_t)(2 + enumL(W*W, w)); pass nullptr to use this build's (coding.h). resid (nullable,
  // allocated like I) receives the image after the residual write-back.
  int tiles(const binary_matrix& I, unsigned W, TileResult* out, const uint64_t* lentab = nullptr,
            binary_matrix* resid = nullptr);

  // compress_test.cpp:73-111: per W x W tile (raster order over ceil(rows/W) x ceil(cols/W)) the
  // least-distance window of the causal search region, first in the reference's scan order.
  int patch_search(const binary_matrix& I, unsigned W, std::vector<uint32_t>* besti,
                   std::vector<uint32_t>* bestj, std::vector<uint32_t>* bestd);

  // compress7_test.cpp:117-275 with W, T, R as its argv[2..4] (rows, cols multiples of W): I is
  // replaced by the image after the residual write-back; golomb_match / golomb_nomatch (fresh)
  // end in the state the driver's coders end in. enuml[w] = enumL(W*W, w) (nullptr: this build's).
  int match_encode(binary_matrix& I, unsigned W, unsigned T, unsigned R, MatchResult* out,
                   GolombCoder* golomb_match = nullptr, GolombCoder* golomb_nomatch = nullptr,
                   const double* enuml = nullptr);

 private:
  struct Buf {
    void* p = nullptr;
    size_t cap = 0;
  };
  int ensure(Buf& b, size_t bytes);
  int upload(const binary_matrix& M, uint64_t* dst);
  int download(uint64_t* src, binary_matrix& M);
  int fetch_stream(const uint64_t* slot, uint64_t bits, Stream* s);

  bic_ctx* ctx_ = nullptr;
  int status_ = BIC_ENODEV;
  Buf in_, out_a_, out_b_, small_, aux_;
};

// The process-wide device used by the free function med() (pred.h): device 0, created on
// first use. Aborts with a message if it is not usable.
Device& default_device();

}  // namespace bic

#endif
