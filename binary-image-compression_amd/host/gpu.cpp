// gpu.cpp -- bic::Device (include/bic_gpu.h): the reference C++ API's planes handed to the
// HIP kernels through the C ABI (bic.h). This file only moves data and bookkeeping; every
// pixel-level operation runs in the kernels.
#include "bic_gpu.h"

#include <cstdio>
#include <cstdlib>

namespace bic {

namespace {
constexpr uint64_t kDomain = 0x80000000ull;  // the reference coders' 32-bit state stays exact below 2^31

bool same_shape(const binary_matrix& a, const binary_matrix& b) {
  return a.get_rows() == b.get_rows() && a.get_cols() == b.get_cols() &&
         a.get_blocks_per_row() == b.get_blocks_per_row() && (a.raw_blocks() || !a.get_rows());
}
}  // namespace

void coder_state::advance(GolombCoder& c, uint64_t n, uint64_t sum, uint64_t bits) {
  c.bitcount += (long)bits;
  if (n == 0) return;  // codeSample was never called: k keeps its value
  c.samples += (unsigned)n;
  c.accumulatedError += (unsigned)sum;
  unsigned k = 0;
  while ((c.samples << k) < c.accumulatedError) ++k;
  c.k = k;
}

void coder_state::advance(EGCoder& e, uint64_t ones, uint64_t bits) {
  e.bitcount += bits;
  if (ones) e.decBlockSize();  // every non-EOL run calls it; from a fresh coder one call is the fixpoint
}

int planes_for_maxval(int maxval) {
  int n = 0;
  for (long b = 1; b < maxval; b <<= 1) ++n;
  return n;
}

Device::Device(int ordinal) { status_ = bic_ctx_create(ordinal, &ctx_); }

Device::~Device() {
  if (!ctx_) return;
  for (Buf* b : {&in_, &out_a_, &out_b_, &small_, &aux_}) bic_free(ctx_, b->p);
  bic_ctx_destroy(ctx_);
}

int Device::ensure(Buf& b, size_t bytes) {
  if (b.cap >= bytes) return BIC_OK;
  int rc = bic_free(ctx_, b.p);
  b.p = nullptr;
  b.cap = 0;
  if (rc) return rc;
  const size_t want = bytes + bytes / 4 + 256;
  if ((rc = bic_malloc(ctx_, want, &b.p))) return rc;
  b.cap = want;
  return BIC_OK;
}

int Device::upload(const binary_matrix& M, uint64_t* dst) {
  return bic_memcpy_h2d(ctx_, dst, M.raw_blocks(), M.get_rows() * M.get_blocks_per_row() * sizeof(uint64_t));
}

int Device::download(uint64_t* src, binary_matrix& M) {
  return bic_memcpy_d2h(ctx_, M.raw_blocks(), src, M.get_rows() * M.get_blocks_per_row() * sizeof(uint64_t));
}

int Device::fetch_stream(const uint64_t* slot, uint64_t bits, Stream* s) {
  s->bits = bits;
  s->bytes.assign((bits + 7) / 8, 0);
  // slots hold big-endian words, so device bytes are already the stream's bytes
  return bic_memcpy_d2h(ctx_, s->bytes.data(), slot, s->bytes.size());
}

#define BIC_TRY(x)            \
  do {                        \
    const int rc_ = (x);      \
    if (rc_) return rc_;      \
  } while (0)

int Device::bitplanes(const pixel_t* gray, idx_t rows, idx_t cols, int nplanes, binary_matrix* planes) {
  BIC_TRY(status_);
  if (nplanes < 1 || nplanes > 32 || !planes || (!gray && rows && cols)) return BIC_EINVAL;
  for (int p = 0; p < nplanes; ++p)
    if (planes[p].get_rows() != rows || planes[p].get_cols() != cols || (rows && !planes[p].raw_blocks()))
      return BIC_EINVAL;
  if (rows == 0 || cols == 0) return BIC_OK;
  const idx_t wpr = planes[0].get_blocks_per_row();
  const size_t pixels = rows * cols, plane_words = rows * wpr;
  BIC_TRY(ensure(in_, pixels));
  BIC_TRY(ensure(out_a_, 8 * plane_words * sizeof(uint64_t)));
  std::vector<uint8_t> bytes(pixels);
  // the kernel reads one byte per pixel: byte b of every pixel feeds planes 8b .. 8b+7
  for (int b = 0; 8 * b < nplanes; ++b) {
    const int nb = nplanes - 8 * b < 8 ? nplanes - 8 * b : 8;
    for (size_t i = 0; i < pixels; ++i) bytes[i] = (uint8_t)(gray[i] >> (8 * b));
    BIC_TRY(bic_memcpy_h2d(ctx_, in_.p, bytes.data(), pixels));
    uint64_t* dev = static_cast<uint64_t*>(out_a_.p);
    BIC_TRY(bic_bitplanes_u8(ctx_, static_cast<const uint8_t*>(in_.p), cols, rows, cols, nb, dev, wpr));
    BIC_TRY(bic_sync(ctx_));
    for (int q = 0; q < nb; ++q) BIC_TRY(download(dev + q * plane_words, planes[8 * b + q]));
  }
  return BIC_OK;
}

int Device::med(const binary_matrix& P, binary_matrix& R, idx_t* weight) {
  BIC_TRY(status_);
  if (!same_shape(P, R)) return BIC_EINVAL;
  const idx_t rows = P.get_rows(), cols = P.get_cols(), wpr = P.get_blocks_per_row();
  if (weight) *weight = 0;
  if (rows == 0 || cols == 0) return BIC_OK;
  const size_t words = rows * wpr;
  BIC_TRY(ensure(in_, words * 8));
  BIC_TRY(ensure(out_a_, words * 8));
  BIC_TRY(ensure(small_, 64));
  uint64_t* d_in = static_cast<uint64_t*>(in_.p);
  uint64_t* d_out = static_cast<uint64_t*>(out_a_.p);
  uint64_t* d_w = weight ? static_cast<uint64_t*>(small_.p) : nullptr;
  // one copy in, the kernel, one copy out: the copy back waits for the kernel (same stream) and
  // reports its errors, so a small call (compress7_test.cpp:205-206 calls med per tile) pays two
  // host round trips and no flag read (med raises none)
  BIC_TRY(upload(P, d_in));
  BIC_TRY(bic_med_residual(ctx_, d_in, 1, rows, cols, wpr, 1, d_out, d_w));
  // the reference writes neither R(0,0) nor R's pad bits (pred.cpp:5-13): keep R's
  const bool r00 = R.get(0, 0);
  std::vector<uint64_t> old_tail(rows);
  const idx_t used = cols % 64;
  const uint64_t pad = used ? ~(~0ull << (64 - used)) : 0;
  block_t* r = R.raw_blocks();
  for (idx_t i = 0; i < rows; ++i) old_tail[i] = r[i * wpr + wpr - 1] & pad;
  BIC_TRY(download(d_out, R));
  for (idx_t i = 0; i < rows; ++i) r[i * wpr + wpr - 1] = (r[i * wpr + wpr - 1] & ~pad) | old_tail[i];
  R.set(0, 0, r00);
  if (weight) {
    uint64_t w = 0;
    BIC_TRY(bic_memcpy_d2h(ctx_, &w, d_w, 8));
    *weight = w;
  }
  return BIC_OK;
}

int Device::encode(const binary_matrix* planes, int nplanes, bool predict, GolombCoder* golomb,
                   std::vector<Stream>* golomb_streams, EGCoder* eg, std::vector<Stream>* eg_streams) {
  BIC_TRY(status_);
  if (nplanes < 1 || !planes || (!golomb && !eg)) return BIC_EINVAL;
  for (int p = 0; p < nplanes; ++p) {
    if (!same_shape(planes[0], planes[p])) return BIC_EINVAL;
    if ((golomb && !coder_state::fresh(golomb[p])) || (eg && !coder_state::fresh(eg[p]))) return BIC_EINVAL;
  }
  const idx_t rows = planes[0].get_rows(), cols = planes[0].get_cols(), wpr = planes[0].get_blocks_per_row();
  if (golomb_streams) golomb_streams->assign(golomb ? nplanes : 0, Stream());
  if (eg_streams) eg_streams->assign(eg ? nplanes : 0, Stream());
  if (rows == 0 || cols == 0) return BIC_OK;
  const size_t plane_words = rows * wpr;
  const size_t slot_g = bic_encode_slot_words(rows, cols, BIC_CODER_GOLOMB);
  const size_t slot_e = bic_encode_slot_words(rows, cols, BIC_CODER_EG);
  BIC_TRY(ensure(in_, nplanes * plane_words * 8));
  if (golomb) BIC_TRY(ensure(out_a_, nplanes * slot_g * 8));
  if (eg) BIC_TRY(ensure(out_b_, nplanes * slot_e * 8));
  BIC_TRY(ensure(small_, 3 * nplanes * 8));
  uint64_t* d_in = static_cast<uint64_t*>(in_.p);
  uint64_t* d_bits = static_cast<uint64_t*>(small_.p);  // [golomb bits | eg bits | residual ones]
  for (int p = 0; p < nplanes; ++p) BIC_TRY(upload(planes[p], d_in + p * plane_words));
  uint64_t* d_g = golomb ? static_cast<uint64_t*>(out_a_.p) : nullptr;
  uint64_t* d_e = eg ? static_cast<uint64_t*>(out_b_.p) : nullptr;
  BIC_TRY(bic_encode_planes2(ctx_, d_in, nplanes, rows, cols, wpr, predict ? 1 : 0, d_g, slot_g,
                             golomb ? d_bits : nullptr, d_e, slot_e, eg ? d_bits + nplanes : nullptr));
  BIC_TRY(bic_med_residual(ctx_, d_in, nplanes, rows, cols, wpr, predict ? 1 : 0, nullptr, d_bits + 2 * nplanes));
  BIC_TRY(bic_sync(ctx_));
  std::vector<uint64_t> h(3 * nplanes);
  BIC_TRY(bic_memcpy_d2h(ctx_, h.data(), d_bits, h.size() * 8));
  for (int p = 0; p < nplanes; ++p) {
    const uint64_t ones = h[2 * nplanes + p];
    if (golomb) {
      // samples: one per 1 plus one per row; their sum is the number of zeros
      coder_state::advance(golomb[p], ones + rows, rows * cols - ones, h[p]);
      if (golomb_streams) BIC_TRY(fetch_stream(d_g + p * slot_g, h[p], &(*golomb_streams)[p]));
    }
    if (eg) {
      coder_state::advance(eg[p], ones, h[nplanes + p]);
      if (eg_streams) BIC_TRY(fetch_stream(d_e + p * slot_e, h[nplanes + p], &(*eg_streams)[p]));
    }
  }
  return BIC_OK;
}

int Device::code_samples(GolombCoder& coder, const unsigned* samples, size_t n, Stream* stream) {
  BIC_TRY(status_);
  if (!samples && n) return BIC_EINVAL;
  uint64_t total = 0;
  for (size_t i = 0; i < n; ++i) total += samples[i];
  const uint64_t n0 = coder_state::samples(coder), a0 = coder_state::accumulated(coder);
  if (n0 + n >= kDomain || a0 + total >= kDomain) return BIC_EINVAL;
  if (stream) *stream = Stream();
  if (n == 0) return BIC_OK;
  const size_t cap = (total + 33 * n + 63) / 64 + 1;  // k + 1 <= 33 and s >> k <= s per sample
  BIC_TRY(ensure(in_, n * 4));
  BIC_TRY(ensure(out_a_, cap * 8));
  BIC_TRY(ensure(small_, 16));
  uint64_t* d_bits = static_cast<uint64_t*>(small_.p);
  BIC_TRY(bic_memcpy_h2d(ctx_, in_.p, samples, n * 4));
  BIC_TRY(bic_golomb_encode_samples(ctx_, static_cast<const uint32_t*>(in_.p), n, n0, a0, 0,
                                    static_cast<uint64_t*>(out_a_.p), cap, d_bits));
  BIC_TRY(bic_sync(ctx_));
  uint64_t h[2];
  BIC_TRY(bic_memcpy_d2h(ctx_, h, d_bits, sizeof(h)));
  coder_state::advance(coder, n, h[1], h[0]);
  if (stream) BIC_TRY(fetch_stream(static_cast<uint64_t*>(out_a_.p), h[0], stream));
  return BIC_OK;
}

int Device::tiles(const binary_matrix& I, unsigned W, TileResult* out, const uint64_t* lentab,
                  binary_matrix* resid) {
  BIC_TRY(status_);
  const idx_t rows = I.get_rows(), cols = I.get_cols(), wpr = I.get_blocks_per_row();
  if (!out || W < 1 || W > 64 || rows % W || cols % W || (resid && !same_shape(I, *resid))) return BIC_EINVAL;
  std::vector<uint64_t> table;
  if (!lentab) {
    table.resize((size_t)W * W + 1);
    BIC_TRY(bic_tile_lentab(W, table.data()));
    lentab = table.data();
  }
  const size_t nt = (rows / W) * (cols / W);
  *out = TileResult();
  if (nt == 0) return BIC_OK;
  const size_t words = rows * wpr;
  const size_t cap = (rows * cols + 33 * nt + 63) / 64 + 1;  // chosen weights sum to <= rows*cols
  BIC_TRY(ensure(in_, words * 8));
  BIC_TRY(ensure(out_a_, cap * 8));
  BIC_TRY(ensure(out_b_, resid ? words * 8 : 8));
  BIC_TRY(ensure(aux_, nt * 13 + 64));
  BIC_TRY(ensure(small_, 24));
  uint32_t* d_w = static_cast<uint32_t*>(aux_.p);
  uint8_t* d_modes = reinterpret_cast<uint8_t*>(d_w + 3 * nt);
  uint64_t* d_stats = static_cast<uint64_t*>(small_.p);
  BIC_TRY(upload(I, static_cast<uint64_t*>(in_.p)));
  BIC_TRY(bic_patch_encode(ctx_, static_cast<const uint64_t*>(in_.p), rows, cols, wpr, W, lentab, d_w, d_w + nt,
                           d_w + 2 * nt, d_modes, resid ? static_cast<uint64_t*>(out_b_.p) : nullptr,
                           static_cast<uint64_t*>(out_a_.p), cap, d_stats));
  BIC_TRY(bic_sync(ctx_));
  uint64_t st[3];
  BIC_TRY(bic_memcpy_d2h(ctx_, st, d_stats, sizeof(st)));
  out->weights.resize(nt);
  out->w_nonpred.resize(nt);
  out->w_pred.resize(nt);
  out->modes.resize(nt);
  BIC_TRY(bic_memcpy_d2h(ctx_, out->weights.data(), d_w, nt * 4));
  BIC_TRY(bic_memcpy_d2h(ctx_, out->w_nonpred.data(), d_w + nt, nt * 4));
  BIC_TRY(bic_memcpy_d2h(ctx_, out->w_pred.data(), d_w + 2 * nt, nt * 4));
  BIC_TRY(bic_memcpy_d2h(ctx_, out->modes.data(), d_modes, nt));
  out->L = st[2];
  BIC_TRY(fetch_stream(static_cast<uint64_t*>(out_a_.p), st[0], &out->stream));
  if (resid) BIC_TRY(download(static_cast<uint64_t*>(out_b_.p), *resid));
  return BIC_OK;
}

int Device::patch_search(const binary_matrix& I, unsigned W, std::vector<uint32_t>* besti,
                         std::vector<uint32_t>* bestj, std::vector<uint32_t>* bestd) {
  BIC_TRY(status_);
  if (!besti || !bestj || !bestd || W < 1 || W > 64) return BIC_EINVAL;
  const idx_t rows = I.get_rows(), cols = I.get_cols(), wpr = I.get_blocks_per_row();
  const size_t nt = ((W - 1 + rows) / W) * ((W - 1 + cols) / W);
  besti->assign(nt, 0);
  bestj->assign(nt, 0);
  bestd->assign(nt, W * W);
  if (nt == 0) return BIC_OK;
  BIC_TRY(ensure(in_, rows * wpr * 8));
  BIC_TRY(ensure(aux_, 3 * nt * 4));
  uint32_t* d = static_cast<uint32_t*>(aux_.p);
  BIC_TRY(upload(I, static_cast<uint64_t*>(in_.p)));
  BIC_TRY(bic_patch_search(ctx_, static_cast<const uint64_t*>(in_.p), rows, cols, wpr, W, d, d + nt, d + 2 * nt));
  BIC_TRY(bic_sync(ctx_));
  BIC_TRY(bic_memcpy_d2h(ctx_, besti->data(), d, nt * 4));
  BIC_TRY(bic_memcpy_d2h(ctx_, bestj->data(), d + nt, nt * 4));
  BIC_TRY(bic_memcpy_d2h(ctx_, bestd->data(), d + 2 * nt, nt * 4));
  return BIC_OK;
}

int Device::match_encode(binary_matrix& I, unsigned W, unsigned T, unsigned R, MatchResult* out,
                         GolombCoder* golomb_match, GolombCoder* golomb_nomatch, const double* enuml) {
  BIC_TRY(status_);
  if (!out || W < 1 || W > 64) return BIC_EINVAL;
  if ((golomb_match && !coder_state::fresh(*golomb_match)) || (golomb_nomatch && !coder_state::fresh(*golomb_nomatch)))
    return BIC_EINVAL;
  const idx_t rows = I.get_rows(), cols = I.get_cols(), wpr = I.get_blocks_per_row();
  if (rows % W || cols % W) return BIC_EINVAL;
  const size_t nt = (rows / W) * (cols / W), M = (size_t)W * W;
  *out = MatchResult();
  if (nt == 0) return BIC_OK;
  std::vector<double> table;
  if (!enuml) {
    table.resize(M + 1);
    for (size_t w = 0; w <= M; ++w) table[w] = bic_enum_codelength((unsigned)M, (unsigned)w);
    enuml = table.data();
  }
  const size_t cap = (rows * cols + 33 * nt + 63) / 64 + 1;  // both streams, always enough
  const size_t tile_bytes = ((4 * 4 + 1) * nt + 255) & ~(size_t)255;
  BIC_TRY(ensure(in_, rows * wpr * 8));
  BIC_TRY(ensure(out_a_, 2 * cap * 8));
  BIC_TRY(ensure(aux_, tile_bytes));
  BIC_TRY(ensure(small_, 64));
  uint64_t* d_I = static_cast<uint64_t*>(in_.p);
  uint64_t* d_s = static_cast<uint64_t*>(out_a_.p);
  uint32_t* d_t = static_cast<uint32_t*>(aux_.p);
  uint64_t* d_st = static_cast<uint64_t*>(small_.p);
  BIC_TRY(upload(I, d_I));
  BIC_TRY(bic_match_encode(ctx_, d_I, rows, cols, wpr, W, T, R, enuml, d_t, d_t + nt, d_t + 2 * nt, d_t + 3 * nt,
                           reinterpret_cast<uint8_t*>(d_t + 4 * nt), d_I, d_s, d_s + cap, cap, d_st));
  BIC_TRY(bic_sync(ctx_));
  uint64_t st[4];
  BIC_TRY(bic_memcpy_d2h(ctx_, st, d_st, sizeof(st)));
  std::vector<uint32_t>* arrs[4] = {&out->besti, &out->bestj, &out->bestd, &out->weights};
  for (int k = 0; k < 4; ++k) {
    arrs[k]->resize(nt);
    BIC_TRY(bic_memcpy_d2h(ctx_, arrs[k]->data(), d_t + k * nt, nt * 4));
  }
  out->modes.resize(nt);
  BIC_TRY(bic_memcpy_d2h(ctx_, out->modes.data(), d_t + 4 * nt, nt));
  BIC_TRY(fetch_stream(d_s, st[1], &out->stream_match));
  BIC_TRY(fetch_stream(d_s + cap, st[2], &out->stream_nomatch));
  BIC_TRY(download(d_I, I));
  out->matches = st[0];
  out->L = st[3];
  // the coders' state: samples, their sum and bits per coder
  uint64_t n[2] = {0, 0}, sum[2] = {0, 0};
  for (size_t i = 0; i < nt; ++i) {
    const int c = (out->modes[i] == 'X' || out->modes[i] == 'x') ? 0 : 1;
    n[c] += 1;
    sum[c] += out->weights[i];
  }
  if (golomb_match) coder_state::advance(*golomb_match, n[0], sum[0], st[1]);
  if (golomb_nomatch) coder_state::advance(*golomb_nomatch, n[1], sum[1], st[2]);
  return BIC_OK;
}

Device& default_device() {
  static Device* dev = new Device(0);
  if (dev->status() != BIC_OK) {
    std::fprintf(stderr, "bic: no usable gfx950 device for the GPU hot path: %s\n", bic_strerror(dev->status()));
    std::abort();
  }
  return *dev;
}

}  // namespace bic
