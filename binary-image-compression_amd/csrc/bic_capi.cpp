// bic_capi.cpp -- the C ABI of include/bic.h: argument validation (the reference's asserts
// become BIC_EINVAL), the per-device context (stream, scratch arena, deferred-error flags)
// and the launch sequences. Compiled with hipcc for gfx950; no CPU fallback exists: without a
// gfx950 device every entry point fails with BIC_ENODEV.
#include "bic.h"
#include "bic_internal.h"

#include <algorithm>
#include <cctype>
#include <cmath>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <functional>
#include <map>
#include <new>
#include <string>
#include <vector>

#ifdef BIC_STAMPS
namespace bic {
int read_stamps(uint64_t* host, size_t n);
int read_match_stamps(uint64_t* host, size_t n);
}
#endif

struct bic_ctx {
  int device = 0;
  hipStream_t own = nullptr;
  hipStream_t cur = nullptr;
  hipStream_t aux = nullptr;      // the staged encoder's second stream (REST emit launch), made on first use
  hipEvent_t ev_fork = nullptr, ev_join = nullptr;
  void* scratch = nullptr;
  size_t scratch_bytes = 0;
  // bytes at the arena's start left zero by the last call (the single / two-pass encoder's k_fixup
  // clears its counter and look-back records for the next call); ensure_scratch hands the value to
  // its caller (scratch_zero_prev) and resets it, since any other user may dirty the arena
  size_t scratch_zero = 0, scratch_zero_prev = 0;
  // a call was enqueued under stream capture: graph replays then run work this bookkeeping never sees
  // (a captured call leaves nothing zeroed when enqueued, and a replay may dirty the arena between two
  // eager calls), so from then on every single / two-pass call clears the records itself
  bool captured = false;
  uint64_t* lut = nullptr;        // device [3][256] byte table of the fused encoder
  uint32_t* flags = nullptr;      // device [4]: overflow, domain, look-back timeout, internal length check
  uint64_t* lentab = nullptr;     // device copy of the tile length table
  size_t lentab_cap = 0;          // entries
  uint64_t* staging = nullptr;    // pinned host staging for lentab
  size_t staging_cap = 0;         // entries
  std::vector<uint64_t> lentab_host;  // what ctx->lentab holds
  double* enuml = nullptr;        // device copy of the match loop's enumL table
  double* enuml_staging = nullptr;  // pinned host staging for it
  size_t enuml_cap = 0;           // entries
  std::vector<double> enuml_host;  // what ctx->enuml holds
  uint64_t* rbuf = nullptr;       // bic_encode_gray* without planes: the count pass's residual planes
  size_t rbuf_bytes = 0;
  unsigned match_parts = 0;       // bic_set_match_parts: workgroups per tile (0 = by region size)
  // kernel timing (bic_prof_*): HIP events recorded on the launch stream around each kernel
  bool prof_on = false;
  std::string prof_only;  // bic_prof_only: bracket only launches of this name ("" = all)
  bool force_multipass = false;
  bool two_pass = false;       // BIC_OPT_TWO_PASS: the two-pass row encoder instead of the staged one
  bool single_kernel = false;  // BIC_OPT_SINGLE_KERNEL: the single kernel with decoupled look-backs
  bool force_staged = false;   // BIC_OPT_STAGED: the staged encoder whatever the batch size
  bool one_stream = false;     // BIC_OPT_ONE_STREAM: no second stream for the staged encoder's emission
  bool eg_src_off = false;     // BIC_OPT_EG_SOURCE = 0: bic_encode_gray* stores R instead of writing EG
  bool eg_src_one = false;     // BIC_OPT_EG_SOURCE = 2: one emission kernel for every row class
  struct Rec { std::string name; hipEvent_t a, b; };
  std::vector<Rec> recs;
  std::vector<hipEvent_t> pool;
};

namespace {

// A failing HIP call returns BIC_EDEVICE; with BIC_VERBOSE set in the environment it is also named on
// stderr (source line, call, HIP's error string)
void hip_fail(hipError_t e, int line, const char* what) {
  static const bool verbose = std::getenv("BIC_VERBOSE") != nullptr;
  if (verbose) std::fprintf(stderr, "bic_capi.cpp:%d: %s: %s\n", line, what, hipGetErrorString(e));
}
#define BIC_HIP(x)                                  \
  do {                                              \
    const hipError_t bic_e_ = (x);                  \
    if (bic_e_ != hipSuccess) {                     \
      hip_fail(bic_e_, __LINE__, #x);               \
      return BIC_EDEVICE;                           \
    }                                               \
  } while (0)
#ifndef BIC_PROF_EVENT_FLAGS
#define BIC_PROF_EVENT_FLAGS hipEventDisableSystemFence
#endif
constexpr unsigned kProfEventFlags = BIC_PROF_EVENT_FLAGS;

hipEvent_t take_event(bic_ctx* ctx) {
  if (!ctx->pool.empty()) {
    hipEvent_t e = ctx->pool.back();
    ctx->pool.pop_back();
    return e;
  }
  hipEvent_t e = nullptr;
  // device-scope timing events: a system-scope release at every record would write back L2 between
  // the launches it brackets
  if (hipEventCreateWithFlags(&e, kProfEventFlags) != hipSuccess) (void)hipEventCreate(&e);
  return e;
}

bool prof_wants(bic_ctx* ctx, const char* name) {
  return ctx->prof_on && (ctx->prof_only.empty() || ctx->prof_only == name);
}

// The staged encoder's emission stage: `name` times its main kernel alone (events the launch records
// on its own stream right around that kernel, FusedScratch::ev_main*: the roofline kernel's launch
// duration), "<name>_stage" the whole stage, the second stream's fork and join included.
template <typename F>
void timed_rows(bic_ctx* ctx, bic::FusedScratch& fs, const char* name, F&& launch) {
  const std::string stage_name = std::string(name) + "_stage";
  const bool k = prof_wants(ctx, name), st = prof_wants(ctx, stage_name.c_str());
  hipEvent_t a = nullptr, b = nullptr, sa = nullptr, sb = nullptr;
  bool main_rec = false;
  if (k) {
    a = take_event(ctx);
    b = take_event(ctx);
    // (recorded here too: a path without a separate main kernel -- the single and two-pass encoders --
    // then times the whole stage, b recorded below)
    (void)hipEventRecord(a, ctx->cur);
    fs.ev_main0 = a;
    fs.ev_main1 = b;
    fs.ev_main_rec = &main_rec;
  }
  if (st) {
    sa = take_event(ctx);
    sb = take_event(ctx);
    (void)hipEventRecord(sa, ctx->cur);
  }
  launch();
  // (an event never recorded would fail hipEventElapsedTime, and that error would stay pending for
  // the next call's hipGetLastError)
  if (k && !main_rec) (void)hipEventRecord(b, ctx->cur);
  if (st) {
    (void)hipEventRecord(sb, ctx->cur);
    ctx->recs.push_back({stage_name, sa, sb});
  }
  if (k) {
    fs.ev_main0 = fs.ev_main1 = nullptr;
    fs.ev_main_rec = nullptr;
    ctx->recs.push_back({name, a, b});
  }
}

// Runs one launch, bracketed by events when profiling is on.
template <typename F>
void timed(bic_ctx* ctx, const char* name, F&& launch) {
  if (!ctx->prof_on || (!ctx->prof_only.empty() && ctx->prof_only != name)) {
    launch();
    return;
  }
  hipEvent_t a = take_event(ctx), b = take_event(ctx);
  (void)hipEventRecord(a, ctx->cur);
  launch();
  (void)hipEventRecord(b, ctx->cur);
  ctx->recs.push_back({name, a, b});
}

int bind(bic_ctx* ctx) {
  if (!ctx) return BIC_EINVAL;
  BIC_HIP(hipSetDevice(ctx->device));
  return BIC_OK;
}

int ensure_scratch(bic_ctx* ctx, size_t bytes) {
  ctx->scratch_zero_prev = ctx->scratch_zero;
  ctx->scratch_zero = 0;
  if (bytes <= ctx->scratch_bytes) return BIC_OK;
  ctx->scratch_zero_prev = 0;
  BIC_HIP(hipStreamSynchronize(ctx->cur));  // earlier calls may still use the old arena
  if (ctx->scratch) (void)hipFree(ctx->scratch);
  ctx->scratch = nullptr;
  ctx->scratch_bytes = 0;
  const size_t want = bytes + bytes / 4 + 4096;
  if (hipMalloc(&ctx->scratch, want) != hipSuccess) {
    ctx->scratch = nullptr;
    return BIC_ENOMEM;
  }
  ctx->scratch_bytes = want;
  return BIC_OK;
}

// The staged encoder's second stream and its fork / join events, made on first use; left null
// (one stream) when HIP cannot make them. Work on it is always joined back into ctx->cur.
void set_aux(bic_ctx* ctx, bic::FusedScratch& fs) {
  if (ctx->one_stream) {
    fs.aux = nullptr;
    fs.ev_fork = fs.ev_join = nullptr;
    return;
  }
  if (!ctx->aux) {
    hipStream_t st = nullptr;
    hipEvent_t a = nullptr, b = nullptr;
    if (hipStreamCreateWithFlags(&st, hipStreamNonBlocking) != hipSuccess) return;
    // device-scope fork / join events: they order two streams of this device, and a system-scope
    // release would write back L2 at every fork (emission 167-170 vs 172-174 us, same box). Round 4 had
    // switched them to system scope over a first-encode failure that the scope did not cause: that
    // build's k_emit_k1 lost bits of k = 1 rows with either scope (6 of 6 fresh processes each), and
    // only its LDS image zeroing decided it; these kernels measured 0 of 8 with either.
#ifndef BIC_FORK_EVENT_FLAGS
#define BIC_FORK_EVENT_FLAGS (hipEventDisableTiming | hipEventDisableSystemFence)
#endif
    const unsigned fl = BIC_FORK_EVENT_FLAGS;
    if (hipEventCreateWithFlags(&a, fl) != hipSuccess || hipEventCreateWithFlags(&b, fl) != hipSuccess) {
      if (a) (void)hipEventDestroy(a);
      (void)hipStreamDestroy(st);
      return;
    }
    ctx->aux = st;
    ctx->ev_fork = a;
    ctx->ev_join = b;
  }
  fs.aux = ctx->aux;
  fs.ev_fork = ctx->ev_fork;
  fs.ev_join = ctx->ev_join;
}

// The staged encoder's ~8 dependent launches cost more than the single kernel's look-back waits
// on small batches (C2, one 4096^2 plane: 81 vs 45 us); from kStagedMinRows rows or kStagedMinWords
// plane words (all planes) on it is the faster one (C3: 131,072 rows; one 16384^2 plane, 16,384 rows
// of 256 words: 0.181 vs 0.252 ms). BIC_OPT_STAGED forces it.
constexpr uint64_t kStagedMinRows = 32768, kStagedMinWords = 1ull << 20;
bool staged_pays(const bic_ctx* ctx, const bic::Geom& g) {
  const uint64_t rows = (uint64_t)g.rows * g.nplanes;
  return ctx->force_staged || rows >= kStagedMinRows || rows * g.used >= kStagedMinWords;
}

bool geom_ok(size_t rows, size_t cols, size_t wpr) {
  if (cols == 0 || rows > 0x7fffffffu || cols > 0x7ffffffeu) return false;
  if (wpr < (cols + 63) / 64 || wpr > 0xffffffffu) return false;
  // the reference's 32-bit coder state (Golomb.h:21-24) is only defined while the sample
  // count and accumulated error stay below 2^31: both are bounded by rows*(cols+1).
  return (unsigned long long)rows * (cols + 1) < 0x80000000ull;
}

}  // namespace

extern "C" {

const char* bic_strerror(int code) {
  switch (code) {
    case BIC_OK: return "ok";
    case BIC_EINVAL: return "invalid argument";
    case BIC_ENOMEM: return "device allocation failed";
    case BIC_EDEVICE: return "HIP runtime error";
    case BIC_ENOSPC: return "output slot too small";
    case BIC_ENODEV: return "no gfx950 device";
    case BIC_EDATA: return "malformed stream";
    default: return "unknown error";
  }
}

int bic_device_count(int* n) {
  if (!n) return BIC_EINVAL;
  int c = 0;
  if (hipGetDeviceCount(&c) != hipSuccess) c = 0;
  *n = c;
  return BIC_OK;
}

int bic_ctx_create(int device, bic_ctx** out) {
  if (!out) return BIC_EINVAL;
  *out = nullptr;
  int n = 0;
  if (hipGetDeviceCount(&n) != hipSuccess || device < 0 || device >= n) return BIC_ENODEV;
  hipDeviceProp_t prop;
  if (hipGetDeviceProperties(&prop, device) != hipSuccess) return BIC_EDEVICE;
  if (std::strncmp(prop.gcnArchName, "gfx950", 6) != 0) return BIC_ENODEV;  // built for gfx950 only
  BIC_HIP(hipSetDevice(device));
  bic_ctx* ctx = new (std::nothrow) bic_ctx();
  if (!ctx) return BIC_ENOMEM;
  ctx->device = device;
  if (hipStreamCreateWithFlags(&ctx->own, hipStreamNonBlocking) != hipSuccess) {
    delete ctx;
    return BIC_EDEVICE;
  }
  ctx->cur = ctx->own;
  {
    uint64_t host_lut[bic::kLutWords];
    bic::build_byte_lut(host_lut);
    bic::egad_build_nib(host_lut + bic::kLutEgadNib);
    bic::egad_build_dec_nib(host_lut + bic::kLutEgadDec);
    if (hipMalloc(&ctx->lut, sizeof(host_lut)) != hipSuccess ||
        hipMemcpy(ctx->lut, host_lut, sizeof(host_lut), hipMemcpyHostToDevice) != hipSuccess) {
      (void)hipStreamDestroy(ctx->own);
      delete ctx;
      return BIC_ENOMEM;
    }
  }
  if (hipMalloc(&ctx->flags, 4 * sizeof(uint32_t)) != hipSuccess ||
      hipMemset(ctx->flags, 0, 4 * sizeof(uint32_t)) != hipSuccess) {
    (void)hipStreamDestroy(ctx->own);
    delete ctx;
    return BIC_ENOMEM;
  }
  *out = ctx;
  return BIC_OK;
}

int bic_ctx_destroy(bic_ctx* ctx) {
  if (!ctx) return BIC_EINVAL;
  (void)hipSetDevice(ctx->device);
  (void)hipStreamSynchronize(ctx->cur);
  for (auto& r : ctx->recs) { (void)hipEventDestroy(r.a); (void)hipEventDestroy(r.b); }
  for (auto e : ctx->pool) (void)hipEventDestroy(e);
  if (ctx->scratch) (void)hipFree(ctx->scratch);
  if (ctx->flags) (void)hipFree(ctx->flags);
  if (ctx->enuml) (void)hipFree(ctx->enuml);
  if (ctx->enuml_staging) (void)hipHostFree(ctx->enuml_staging);
  if (ctx->lut) (void)hipFree(ctx->lut);
  if (ctx->rbuf) (void)hipFree(ctx->rbuf);
  if (ctx->lentab) (void)hipFree(ctx->lentab);
  if (ctx->staging) (void)hipHostFree(ctx->staging);
  if (ctx->own) (void)hipStreamDestroy(ctx->own);
  if (ctx->aux) (void)hipStreamDestroy(ctx->aux);
  if (ctx->ev_fork) (void)hipEventDestroy(ctx->ev_fork);
  if (ctx->ev_join) (void)hipEventDestroy(ctx->ev_join);
  delete ctx;
  return BIC_OK;
}

int bic_ctx_set_stream(bic_ctx* ctx, void* hip_stream) {
  if (!ctx) return BIC_EINVAL;
  ctx->cur = reinterpret_cast<hipStream_t>(hip_stream);  // NULL = the HIP null stream
  return BIC_OK;
}

void* bic_ctx_own_stream(bic_ctx* ctx) { return ctx ? reinterpret_cast<void*>(ctx->own) : nullptr; }

void* bic_ctx_get_stream(bic_ctx* ctx) { return ctx ? reinterpret_cast<void*>(ctx->cur) : nullptr; }

int bic_sync(bic_ctx* ctx) {
  int rc = bind(ctx);
  if (rc) return rc;
  BIC_HIP(hipStreamSynchronize(ctx->cur));
  BIC_HIP(hipGetLastError());
  uint32_t f[4] = {0, 0, 0, 0};
  BIC_HIP(hipMemcpy(f, ctx->flags, sizeof(f), hipMemcpyDeviceToHost));
  if (f[0] || f[1] || f[2] || f[3]) BIC_HIP(hipMemset(ctx->flags, 0, sizeof(f)));
  if (f[2] || f[3]) hip_fail(hipSuccess, __LINE__, f[2] ? "look-back record flag" : "length disagreement flag");
  if (f[2]) return BIC_EDEVICE;  // a look-back record never arrived (should not happen)
  if (f[3]) return BIC_EDEVICE;  // the row encoder's length pass disagreed with its emission (a bug)
  if (f[1] & 2u) return BIC_EDATA;  // a decoder met a malformed stream
  if (f[1]) return BIC_EINVAL;
  if (f[0]) return BIC_ENOSPC;
  return BIC_OK;
}

int bic_reserve(bic_ctx* ctx, int nplanes, size_t rows, size_t cols) {
  int rc = bind(ctx);
  if (rc) return rc;
  if (nplanes < 1 || !geom_ok(rows, cols, (cols + 63) / 64)) return BIC_EINVAL;
  const bic::Geom g = bic::make_geom(rows, cols, (cols + 63) / 64, nplanes);
  return ensure_scratch(ctx, bic::chunk_scratch_bytes(g));
}

int bic_malloc(bic_ctx* ctx, size_t bytes, void** dptr) {
  if (!dptr) return BIC_EINVAL;
  *dptr = nullptr;
  int rc = bind(ctx);
  if (rc) return rc;
  if (bytes == 0) return BIC_OK;
  return hipMalloc(dptr, bytes) == hipSuccess ? BIC_OK : BIC_ENOMEM;
}

int bic_free(bic_ctx* ctx, void* dptr) {
  int rc = bind(ctx);
  if (rc) return rc;
  if (dptr) BIC_HIP(hipFree(dptr));
  return BIC_OK;
}

int bic_memcpy_h2d(bic_ctx* ctx, void* dst, const void* src, size_t bytes) {
  int rc = bind(ctx);
  if (rc) return rc;
  if (bytes == 0) return BIC_OK;
  if (!dst || !src) return BIC_EINVAL;
  BIC_HIP(hipMemcpyAsync(dst, src, bytes, hipMemcpyHostToDevice, ctx->cur));
  BIC_HIP(hipStreamSynchronize(ctx->cur));
  return BIC_OK;
}

int bic_memcpy_d2h(bic_ctx* ctx, void* dst, const void* src, size_t bytes) {
  int rc = bind(ctx);
  if (rc) return rc;
  if (bytes == 0) return BIC_OK;
  if (!dst || !src) return BIC_EINVAL;
  BIC_HIP(hipMemcpyAsync(dst, src, bytes, hipMemcpyDeviceToHost, ctx->cur));
  BIC_HIP(hipStreamSynchronize(ctx->cur));
  return BIC_OK;
}

int bic_memset(bic_ctx* ctx, void* dst, int value, size_t bytes) {
  int rc = bind(ctx);
  if (rc) return rc;
  if (bytes == 0) return BIC_OK;
  if (!dst) return BIC_EINVAL;
  BIC_HIP((bic::launch_fill(ctx->cur, dst, value, bytes), hipGetLastError()));
  return BIC_OK;
}

int bic_ctx_set_option(bic_ctx* ctx, int option, long value) {
  if (!ctx) return BIC_EINVAL;
  if (option == BIC_OPT_MULTIPASS) {
    ctx->force_multipass = value != 0;
    return BIC_OK;
  }
  if (option == BIC_OPT_TWO_PASS) {
    ctx->two_pass = value != 0;
    return BIC_OK;
  }
  if (option == BIC_OPT_SINGLE_KERNEL) {
    ctx->single_kernel = value != 0;
    return BIC_OK;
  }
  if (option == BIC_OPT_STAGED) {
    ctx->force_staged = value != 0;
    return BIC_OK;
  }
  if (option == BIC_OPT_ONE_STREAM) {
    ctx->one_stream = value != 0;
    return BIC_OK;
  }
  if (option == BIC_OPT_EG_SOURCE) {
    ctx->eg_src_off = value == 0;
    ctx->eg_src_one = value == 2;
    return BIC_OK;
  }
  return BIC_EINVAL;
}

int bic_bitplanes_u8_range(bic_ctx* ctx, const uint8_t* gray, size_t pitch, size_t rows, size_t cols, int plane0,
                           int nplanes, uint64_t* planes, size_t wpr) {
  int rc = bind(ctx);
  if (rc) return rc;
  if (plane0 < 0 || nplanes < 1 || plane0 + nplanes > 8 || pitch < cols || (rows && (!gray || !planes)))
    return BIC_EINVAL;
  if (!geom_ok(rows, cols, wpr)) return BIC_EINVAL;
  if (rows == 0) return BIC_OK;
  timed(ctx, "bitplanes_u8", [&] {
    bic::launch_bitplanes_u8(ctx->cur, gray, pitch, (uint32_t)rows, (uint32_t)cols, plane0, nplanes, planes,
                             (uint32_t)wpr);
  });
  BIC_HIP(hipGetLastError());
  return BIC_OK;
}

int bic_bitplanes_u8(bic_ctx* ctx, const uint8_t* gray, size_t pitch, size_t rows, size_t cols,
                     int nplanes, uint64_t* planes, size_t wpr) {
  return bic_bitplanes_u8_range(ctx, gray, pitch, rows, cols, 0, nplanes, planes, wpr);
}

int bic_med_residual(bic_ctx* ctx, const uint64_t* planes, int nplanes, size_t rows, size_t cols,
                     size_t wpr, int predict, uint64_t* resid, uint64_t* weight_out) {
  int rc = bind(ctx);
  if (rc) return rc;
  if (nplanes < 1 || !geom_ok(rows, cols, wpr) || (rows && !planes)) return BIC_EINVAL;
  if (weight_out) BIC_HIP((bic::launch_fill(ctx->cur, weight_out, 0, sizeof(uint64_t) * nplanes), hipGetLastError()));
  if (rows == 0) return BIC_OK;
  const bic::Geom g = bic::make_geom(rows, cols, wpr, nplanes);
  if ((rc = ensure_scratch(ctx, bic::chunk_scratch_bytes(g)))) return rc;
  const bic::ChunkScratch cs = bic::carve_chunk_scratch(ctx->scratch, g);
  if (bic::med_rows_supported(g, planes, resid)) {
    timed(ctx, "med_count", [&] {
      bic::launch_med_rows(ctx->cur, g, planes, predict ? 1 : 0, resid, cs.ones, weight_out);
    });
  } else {
    timed(ctx, "med_count", [&] { bic::launch_count(ctx->cur, g, planes, predict ? 1 : 0, cs, resid, weight_out); });
  }
  BIC_HIP(hipGetLastError());
  return BIC_OK;
}

size_t bic_encode_slot_words(size_t rows, size_t cols, int coder) {
  const unsigned long long base = (unsigned long long)rows * (cols + 1);
  if (coder == BIC_CODER_EG) return (size_t)((base + 1 + 63) / 64);
  return (size_t)((2 * base + 63) / 64 + 64);
}

namespace {
// Packed output where the encoder cannot write it in place (encoders other than the staged one, the
// multi-pass path): ONE encode of both coders into slots in stream-ordered temporaries, then
// bic_pack_streams' kernel once per coder.
int pack_after(bic_ctx* ctx, int nplanes, uint64_t* out_g, size_t slot_g, uint64_t* bits_g, uint64_t* off_g,
               uint64_t* out_e, size_t slot_e, uint64_t* bits_e, uint64_t* off_e,
               const std::function<int(uint64_t*, uint64_t*)>& encode) {
  uint64_t *tg = nullptr, *te = nullptr;
  if (out_g) BIC_HIP(hipMallocAsync(reinterpret_cast<void**>(&tg), (size_t)nplanes * slot_g * 8, ctx->cur));
  if (out_e && hipMallocAsync(reinterpret_cast<void**>(&te), (size_t)nplanes * slot_e * 8, ctx->cur) != hipSuccess) {
    if (tg) (void)hipFreeAsync(tg, ctx->cur);
    return BIC_EDEVICE;
  }
  const int rc = encode(tg, te);
  if (rc == BIC_OK && tg)
    timed(ctx, "pack", [&] { bic::launch_pack(ctx->cur, tg, nplanes, slot_g, bits_g, out_g, off_g); });
  if (rc == BIC_OK && te)
    timed(ctx, "pack", [&] { bic::launch_pack(ctx->cur, te, nplanes, slot_e, bits_e, out_e, off_e); });
  if (tg) (void)hipFreeAsync(tg, ctx->cur);
  if (te) (void)hipFreeAsync(te, ctx->cur);
  BIC_HIP(hipGetLastError());
  return rc;
}
}  // namespace

static int encode_planes_impl(bic_ctx* ctx, const uint64_t* planes, int nplanes, size_t rows, size_t cols,
                              size_t wpr, int predict, uint64_t* out_golomb, size_t slot_golomb,
                              uint64_t* bits_golomb, uint64_t* off_golomb, uint64_t* out_eg, size_t slot_eg,
                              uint64_t* bits_eg, uint64_t* off_eg, uint64_t* row_index = nullptr) {
  int rc = bind(ctx);
  if (rc) return rc;
  if (nplanes < 1 || !geom_ok(rows, cols, wpr)) return BIC_EINVAL;
  if (!out_golomb && !out_eg) return BIC_EINVAL;
  if (out_golomb && (!bits_golomb || slot_golomb == 0)) return BIC_EINVAL;
  if (out_eg && (!bits_eg || slot_eg == 0)) return BIC_EINVAL;
  if (rows && !planes) return BIC_EINVAL;
  if (rows == 0) {
    if (out_golomb) BIC_HIP((bic::launch_fill(ctx->cur, bits_golomb, 0, sizeof(uint64_t) * nplanes), hipGetLastError()));
    if (out_eg) BIC_HIP((bic::launch_fill(ctx->cur, bits_eg, 0, sizeof(uint64_t) * nplanes), hipGetLastError()));
    if (off_golomb) BIC_HIP((bic::launch_fill(ctx->cur, off_golomb, 0, sizeof(uint64_t) * (nplanes + 1)), hipGetLastError()));
    if (off_eg) BIC_HIP((bic::launch_fill(ctx->cur, off_eg, 0, sizeof(uint64_t) * (nplanes + 1)), hipGetLastError()));
    return BIC_OK;
  }
  const int pr = predict ? 1 : 0;
  const bic::Geom g = bic::make_geom(rows, cols, wpr, nplanes);
  if (bic::fused_supported(g) && !ctx->force_multipass) {
    // one pass: residual -> runs -> both streams (bic_fused.hip)
    if ((rc = ensure_scratch(ctx, bic::fused_scratch_bytes(g)))) return rc;
    bic::FusedScratch fs = bic::carve_fused_scratch(ctx->scratch, g);
    set_aux(ctx, fs);
    const int mode = ctx->two_pass ? bic::kEncTwoPass
                     : (ctx->single_kernel || !staged_pays(ctx, g) || !bic::med_rows_supported(g, planes, nullptr))
                         ? bic::kEncSingle
                                                                                            : bic::kEncStaged;
    if (row_index && (mode != bic::kEncStaged || !out_golomb)) {  // the index from the staged prefix kernels
      if ((rc = encode_planes_impl(ctx, planes, nplanes, rows, cols, wpr, predict, out_golomb, slot_golomb,
                                   bits_golomb, off_golomb, out_eg, slot_eg, bits_eg, off_eg)))
        return rc;
      return bic_row_index(ctx, planes, nplanes, rows, cols, wpr, predict, row_index);
    }
    if ((off_golomb || off_eg) && mode != bic::kEncStaged)  // packed output via slots + pack
      return pack_after(ctx, nplanes, out_golomb, slot_golomb, bits_golomb, off_golomb, out_eg, slot_eg, bits_eg,
                        off_eg, [&](uint64_t* tg, uint64_t* te) {
                          return encode_planes_impl(ctx, planes, nplanes, rows, cols, wpr, predict, tg, slot_golomb,
                                                    bits_golomb, nullptr, te, slot_eg, bits_eg, nullptr);
                        });
    fs.off_g = off_golomb;
    fs.off_e = off_eg;
    fs.index = row_index;
    // (no memset when the previous call's k_fixup left the counters and records zero: C2 0.036 ->
    // 0.032 ms. A call on another stream without synchronisation would share the arena anyway: calls
    // on one context are ordered by the caller)
    hipStreamCaptureStatus cst = hipStreamCaptureStatusNone;
    if (hipStreamIsCapturing(ctx->cur, &cst) == hipSuccess && cst != hipStreamCaptureStatusNone) ctx->captured = true;
    fs.zero_ready = mode != bic::kEncStaged && !ctx->captured && ctx->scratch_zero_prev >= fs.zero_bytes;
    auto stage = [&](int st) {
      bic::launch_fused(ctx->cur, g, planes, ctx->lut, pr, fs, out_golomb, slot_golomb, bits_golomb, out_eg, slot_eg,
                        bits_eg, ctx->flags, mode, st);
    };
    stage(bic::kFusedPrep);
    // staged encoder: per-row counts, scans and Golomb lengths (every row's offsets known up front)
    if (mode == bic::kEncStaged) timed(ctx, "encode_prefix", [&] { stage(bic::kFusedPrefix); });
    // the row kernel alone is timed under the encoder's name (bench.py's roofline kernel)
    timed_rows(ctx, fs, out_golomb ? (out_eg ? "encode_rows_golomb_eg" : "encode_rows_golomb") : "encode_rows_eg",
               [&] { stage(bic::kFusedRows); });
    timed(ctx, "encode_finish", [&] { stage(bic::kFusedFinish); });
    BIC_HIP(hipGetLastError());
    if (mode != bic::kEncStaged && !ctx->captured) ctx->scratch_zero = fs.zero_bytes;  // (k_fixup cleared them)
    return BIC_OK;
  }
  // rows wider than 16384 columns: multi-pass chunk kernels (bic_kernels.hip)
  if (row_index) return BIC_EINVAL;  // (the decoders take rows of up to 16384 columns)
  if (off_golomb || off_eg)  // packed output via slots + pack
    return pack_after(ctx, nplanes, out_golomb, slot_golomb, bits_golomb, off_golomb, out_eg, slot_eg, bits_eg, off_eg,
                      [&](uint64_t* tg, uint64_t* te) {
                        return encode_planes_impl(ctx, planes, nplanes, rows, cols, wpr, predict, tg, slot_golomb,
                                                  bits_golomb, nullptr, te, slot_eg, bits_eg, nullptr);
                      });
  if ((rc = ensure_scratch(ctx, bic::chunk_scratch_bytes(g)))) return rc;
  const bic::ChunkScratch cs = bic::carve_chunk_scratch(ctx->scratch, g);
  timed(ctx, "med_count", [&] { bic::launch_count(ctx->cur, g, planes, pr, cs, nullptr, nullptr); });
  timed(ctx, "scan_rows", [&] { bic::launch_scan_rows(ctx->cur, g, cs); });
  if (out_golomb) {
    timed(ctx, "golomb_bits", [&] { bic::launch_golomb_bits(ctx->cur, g, planes, pr, cs); });
    timed(ctx, "golomb_offsets", [&] {
      bic::launch_golomb_offsets(ctx->cur, g, cs, out_golomb, slot_golomb, bits_golomb, ctx->flags);
    });
    timed(ctx, "golomb_emit", [&] {
      bic::launch_golomb_emit(ctx->cur, g, planes, pr, cs, out_golomb, slot_golomb);
    });
  }
  if (out_eg) {
    timed(ctx, "eg_emit", [&] {
      bic::launch_eg_emit(ctx->cur, g, planes, pr, cs, out_eg, slot_eg, bits_eg, ctx->flags);
    });
  }
  BIC_HIP(hipGetLastError());
  return BIC_OK;
}

int bic_encode_planes2(bic_ctx* ctx, const uint64_t* planes, int nplanes, size_t rows, size_t cols,
                       size_t wpr, int predict, uint64_t* out_golomb, size_t slot_golomb,
                       uint64_t* bits_golomb, uint64_t* out_eg, size_t slot_eg, uint64_t* bits_eg) {
  return encode_planes_impl(ctx, planes, nplanes, rows, cols, wpr, predict, out_golomb, slot_golomb, bits_golomb,
                            nullptr, out_eg, slot_eg, bits_eg, nullptr);
}

int bic_encode_planes_packed(bic_ctx* ctx, const uint64_t* planes, int nplanes, size_t rows, size_t cols,
                             size_t wpr, int predict, uint64_t* out_golomb, size_t slot_golomb,
                             uint64_t* bits_golomb, uint64_t* off_golomb, uint64_t* out_eg, size_t slot_eg,
                             uint64_t* bits_eg, uint64_t* off_eg, uint64_t* row_index) {
  if ((out_golomb && !off_golomb) || (out_eg && !off_eg)) return BIC_EINVAL;
  return encode_planes_impl(ctx, planes, nplanes, rows, cols, wpr, predict, out_golomb, slot_golomb, bits_golomb,
                            off_golomb, out_eg, slot_eg, bits_eg, off_eg, row_index);
}

static int encode_gray_impl(bic_ctx* ctx, const uint8_t* gray, size_t pitch, size_t rows, size_t cols, int plane0,
                            int nplanes, uint64_t* planes, size_t wpr, int predict, uint64_t* out_golomb,
                            size_t slot_golomb, uint64_t* bits_golomb, uint64_t* off_golomb, uint64_t* out_eg,
                            size_t slot_eg, uint64_t* bits_eg, uint64_t* off_eg, uint64_t* row_index = nullptr) {
  int rc = bind(ctx);
  if (rc) return rc;
  if (plane0 < 0 || nplanes < 1 || plane0 + nplanes > 8 || pitch < cols || !geom_ok(rows, cols, wpr))
    return BIC_EINVAL;
  if (!out_golomb && !out_eg) return BIC_EINVAL;
  if (out_golomb && (!bits_golomb || slot_golomb == 0)) return BIC_EINVAL;
  if (out_eg && (!bits_eg || slot_eg == 0)) return BIC_EINVAL;
  if (rows && !gray) return BIC_EINVAL;
  const bic::Geom g = bic::make_geom(rows, cols, wpr, nplanes);
  // EG source: no bitplanes wanted and the EG stream into slots -- the count pass writes the EG
  // stream (its uniform layout) instead of the residual planes, and the Golomb kernels read the
  // residual rows back from it (bic_internal.h FusedScratch::eg_src): no residual buffer at all
  const uint64_t eg_words = ((uint64_t)rows * (cols + 1) + 1 + 63) / 64;
  const bool fuse = rows && bic::fused_supported(g) && !ctx->force_multipass && !ctx->two_pass && !ctx->single_kernel &&
                    staged_pays(ctx, g) && bic::med_rows_supported(g, planes, nullptr) &&
                    bic::gray_rows_supported(g, gray, pitch, planes);
  const bool eg_src = fuse && !planes && predict && out_eg && !off_eg && bic::gray_eg_supported(g) &&
                      eg_words <= slot_eg && (out_golomb || !row_index) && !ctx->eg_src_off;
  if (!planes && rows && !eg_src) {
    // no bitplanes wanted: the count pass stores the med residual planes into the context's buffer
    // (the same bytes the bitplanes would take) and the encoder reads them with prediction off --
    // no row above, no med in the emission. Same streams (predict off on R = med on P).
    const size_t need = (size_t)nplanes * rows * wpr * 8;
    if (ctx->rbuf_bytes < need) {
      BIC_HIP(hipStreamSynchronize(ctx->cur));
      if (ctx->rbuf) (void)hipFree(ctx->rbuf);
      ctx->rbuf = nullptr;
      ctx->rbuf_bytes = 0;
      if (hipMalloc(&ctx->rbuf, need) != hipSuccess) return BIC_ENOMEM;
      ctx->rbuf_bytes = need;
    }
  }
  const bool store_resid = !planes && predict;
  if (!planes && !eg_src) planes = ctx->rbuf;
  if (!fuse) {  // the same result through the two separate calls
    if ((rc = bic_bitplanes_u8_range(ctx, gray, pitch, rows, cols, plane0, nplanes, planes, wpr))) return rc;
    return encode_planes_impl(ctx, planes, nplanes, rows, cols, wpr, predict, out_golomb, slot_golomb, bits_golomb,
                              off_golomb, out_eg, slot_eg, bits_eg, off_eg, row_index);
  }
  const int pr = predict && !store_resid ? 1 : 0;  // R stored: the encoder codes it as given
  if ((rc = ensure_scratch(ctx, bic::fused_scratch_bytes(g)))) return rc;
  bic::FusedScratch fs = bic::carve_fused_scratch(ctx->scratch, g);
  fs.counted = true;
  fs.ns = bic::gray_strips(g);
  fs.off_g = off_golomb;
  fs.off_e = off_eg;
  fs.index = out_golomb ? row_index : nullptr;
  fs.eg_src = eg_src;
  fs.eg_src_one = ctx->eg_src_one;
  set_aux(ctx, fs);
  auto stage = [&](int st) {
    bic::launch_fused(ctx->cur, g, planes, ctx->lut, pr, fs, out_golomb, slot_golomb, bits_golomb, out_eg, slot_eg,
                      bits_eg, ctx->flags, bic::kEncStaged, st);
  };
  stage(bic::kFusedPrep);
  timed(ctx, "bitplanes_count", [&] {
    bic::launch_gray_rows(ctx->cur, gray, pitch, g, predict ? 1 : 0, plane0, planes, fs.sones, fs.krec, fs.kpos,
                          fs.counter, store_resid, eg_src ? out_eg : nullptr, slot_eg);
  });
  timed(ctx, "encode_prefix", [&] { stage(bic::kFusedPrefix); });
  // (EG source: the emission is Golomb's alone, reading the residual rows from the EG stream)
  timed_rows(ctx, fs, eg_src ? "encode_rows_golomb_egsrc"
                             : out_golomb ? (out_eg ? "encode_rows_golomb_eg" : "encode_rows_golomb") : "encode_rows_eg",
             [&] { stage(bic::kFusedRows); });
  timed(ctx, "encode_finish", [&] { stage(bic::kFusedFinish); });
  BIC_HIP(hipGetLastError());
  if (row_index && !out_golomb) return bic_row_index(ctx, planes, nplanes, rows, cols, wpr, pr, row_index);
  return BIC_OK;
}

int bic_encode_gray_range(bic_ctx* ctx, const uint8_t* gray, size_t pitch, size_t rows, size_t cols, int plane0,
                          int nplanes, uint64_t* planes, size_t wpr, int predict, uint64_t* out_golomb,
                          size_t slot_golomb, uint64_t* bits_golomb, uint64_t* out_eg, size_t slot_eg,
                          uint64_t* bits_eg) {
  return encode_gray_impl(ctx, gray, pitch, rows, cols, plane0, nplanes, planes, wpr, predict, out_golomb, slot_golomb,
                          bits_golomb, nullptr, out_eg, slot_eg, bits_eg, nullptr);
}

int bic_encode_gray_packed(bic_ctx* ctx, const uint8_t* gray, size_t pitch, size_t rows, size_t cols, int plane0,
                           int nplanes, uint64_t* planes, size_t wpr, int predict, uint64_t* out_golomb,
                           size_t slot_golomb, uint64_t* bits_golomb, uint64_t* off_golomb, uint64_t* out_eg,
                           size_t slot_eg, uint64_t* bits_eg, uint64_t* off_eg, uint64_t* row_index) {
  if ((out_golomb && !off_golomb) || (out_eg && !off_eg)) return BIC_EINVAL;
  return encode_gray_impl(ctx, gray, pitch, rows, cols, plane0, nplanes, planes, wpr, predict, out_golomb, slot_golomb,
                          bits_golomb, off_golomb, out_eg, slot_eg, bits_eg, off_eg, row_index);
}

int bic_row_index(bic_ctx* ctx, const uint64_t* planes, int nplanes, size_t rows, size_t cols, size_t wpr,
                  int predict, uint64_t* index) {
  int rc = bind(ctx);
  if (rc) return rc;
  if (nplanes < 1 || !geom_ok(rows, cols, wpr) || (rows && (!planes || !index))) return BIC_EINVAL;
  if (rows == 0) return BIC_OK;
  const bic::Geom g = bic::make_geom(rows, cols, wpr, nplanes);
  if (!bic::fused_supported(g)) return BIC_EINVAL;
  if (!bic::med_rows_supported(g, planes, nullptr)) {
    // the count kernel reads 16-byte pairs of words: an even-pitched, aligned copy of the planes
    const size_t wpr2 = (wpr + 1) & ~(size_t)1;
    uint64_t* tmp = nullptr;
    BIC_HIP(hipMallocAsync(reinterpret_cast<void**>(&tmp), (size_t)nplanes * rows * wpr2 * 8, ctx->cur));
    rc = BIC_OK;
    if (hipMemcpy2DAsync(tmp, wpr2 * 8, planes, wpr * 8, wpr * 8, (size_t)nplanes * rows, hipMemcpyDeviceToDevice,
                         ctx->cur) != hipSuccess)
      rc = BIC_EDEVICE;
    if (rc == BIC_OK) rc = bic_row_index(ctx, tmp, nplanes, rows, cols, wpr2, predict, index);
    (void)hipFreeAsync(tmp, ctx->cur);
    return rc;
  }
  if ((rc = ensure_scratch(ctx, bic::fused_scratch_bytes(g)))) return rc;
  bic::FusedScratch fs = bic::carve_fused_scratch(ctx->scratch, g);
  fs.index = index;
  const size_t slot = bic_encode_slot_words(rows, cols, BIC_CODER_GOLOMB);
  // the staged encoder's prefix kernels alone (counts, scans, the walk of mixed-k rows, the
  // length scan): they touch no output words, only the scratch, the per-plane totals (gbase) and
  // the index; `index` stands in for the Golomb output, which they never write
  timed(ctx, "row_index", [&] {
    bic::launch_fused(ctx->cur, g, planes, ctx->lut, predict ? 1 : 0, fs, index, slot, fs.gbase, nullptr, 0, nullptr,
                      ctx->flags, bic::kEncStaged, bic::kFusedPrefix);
  });
  BIC_HIP(hipGetLastError());
  return BIC_OK;
}

int bic_decode_planes(bic_ctx* ctx, int coder, const uint64_t* streams, size_t slot_words, const uint64_t* word_off,
                      const uint64_t* plane_bits, const uint64_t* index, int nplanes, size_t rows, size_t cols,
                      size_t wpr, int predict, const uint8_t* p00, uint64_t* planes) {
  int rc = bind(ctx);
  if (rc) return rc;
  if (coder != BIC_CODER_GOLOMB && coder != BIC_CODER_EG && coder != BIC_CODER_EG_ADAPTIVE) return BIC_EINVAL;
  if (nplanes < 1 || !geom_ok(rows, cols, wpr) || !bic::decode_supported((uint32_t)cols)) return BIC_EINVAL;
  if (rows == 0) return BIC_OK;
  if (!streams || !plane_bits || !planes || (slot_words == 0 && !word_off)) return BIC_EINVAL;
  if ((coder == BIC_CODER_GOLOMB || coder == BIC_CODER_EG_ADAPTIVE) && !index) return BIC_EINVAL;
  if ((rc = ensure_scratch(ctx, bic::decode_scratch_bytes((uint32_t)rows, (uint32_t)wpr, (uint32_t)nplanes)))) return rc;
  timed(ctx, "decode", [&] {
    bic::launch_decode(ctx->cur, coder == BIC_CODER_GOLOMB ? 0 : coder == BIC_CODER_EG ? 1 : 2, streams, slot_words, word_off, plane_bits, index,
                       p00, (uint32_t)rows, (uint32_t)cols, (uint32_t)wpr, (uint32_t)nplanes, predict ? 1 : 0, planes,
                       ctx->scratch, ctx->flags, ctx->lut + bic::kLutEgadDec);
  });
  BIC_HIP(hipGetLastError());
  return BIC_OK;
}

int bic_encode_gray(bic_ctx* ctx, const uint8_t* gray, size_t pitch, size_t rows, size_t cols, int nplanes,
                    uint64_t* planes, size_t wpr, int predict, uint64_t* out_golomb, size_t slot_golomb,
                    uint64_t* bits_golomb, uint64_t* out_eg, size_t slot_eg, uint64_t* bits_eg) {
  return bic_encode_gray_range(ctx, gray, pitch, rows, cols, 0, nplanes, planes, wpr, predict, out_golomb,
                               slot_golomb, bits_golomb, out_eg, slot_eg, bits_eg);
}

int bic_encode_planes(bic_ctx* ctx, const uint64_t* planes, int nplanes, size_t rows, size_t cols,
                      size_t wpr, int predict, int coder, uint64_t* out, size_t slot_words,
                      uint64_t* plane_bits) {
  if (coder == BIC_CODER_GOLOMB)
    return bic_encode_planes2(ctx, planes, nplanes, rows, cols, wpr, predict, out, slot_words, plane_bits,
                              nullptr, 0, nullptr);
  if (coder == BIC_CODER_EG)
    return bic_encode_planes2(ctx, planes, nplanes, rows, cols, wpr, predict, nullptr, 0, nullptr, out,
                              slot_words, plane_bits);
  if (coder == BIC_CODER_EG_ADAPTIVE) {  // bic_egad.hip
    int rc = bind(ctx);
    if (rc) return rc;
    if (nplanes < 1 || !geom_ok(rows, cols, wpr) || (rows && (!planes || !out || !plane_bits)) || slot_words == 0)
      return BIC_EINVAL;
    if (rows == 0) {
      BIC_HIP((bic::launch_fill(ctx->cur, plane_bits, 0, sizeof(uint64_t) * nplanes), hipGetLastError()));
      return BIC_OK;
    }
    if ((rc = ensure_scratch(ctx, bic::egad_scratch_bytes((uint64_t)rows * nplanes)))) return rc;
    timed(ctx, "encode_eg_adaptive", [&] {
      bic::launch_egad(ctx->cur, planes, (uint32_t)rows, (uint32_t)cols, (uint32_t)wpr, (uint32_t)nplanes,
                       predict ? 1 : 0, out, slot_words, plane_bits, ctx->scratch, ctx->flags, nullptr,
                       ctx->lut + bic::kLutEgadNib);
    });
    BIC_HIP(hipGetLastError());
    return BIC_OK;
  }
  return BIC_EINVAL;
}

int bic_egad_row_index(bic_ctx* ctx, const uint64_t* planes, int nplanes, size_t rows, size_t cols, size_t wpr,
                       int predict, uint64_t* index) {
  int rc = bind(ctx);
  if (rc) return rc;
  if (nplanes < 1 || !geom_ok(rows, cols, wpr) || (rows && (!planes || !index))) return BIC_EINVAL;
  if (rows == 0) return BIC_OK;
  const uint64_t n = (uint64_t)rows * nplanes;
  const size_t sb = (bic::egad_scratch_bytes(n) + 255) & ~(size_t)255;
  if ((rc = ensure_scratch(ctx, sb + (size_t)nplanes * 8))) return rc;
  // a slot no row can overflow: <= 17 bits per column and end-of-row (a '1' per zero or block, a
  // '0' and <= 15 remainder bits per 1)
  const uint64_t slot = ((uint64_t)rows * (cols + 1) * 17 + 63) / 64;
  uint64_t* bits = reinterpret_cast<uint64_t*>(static_cast<char*>(ctx->scratch) + sb);
  timed(ctx, "egad_row_index", [&] {
    bic::launch_egad(ctx->cur, planes, (uint32_t)rows, (uint32_t)cols, (uint32_t)wpr, (uint32_t)nplanes,
                     predict ? 1 : 0, nullptr, slot, bits, ctx->scratch, ctx->flags, index, ctx->lut + bic::kLutEgadNib);
  });
  BIC_HIP(hipGetLastError());
  return BIC_OK;
}

int bic_golomb_encode_samples(bic_ctx* ctx, const uint32_t* samples, size_t n, uint64_t n0,
                              uint64_t a0, unsigned bit0, uint64_t* out, size_t cap_words,
                              uint64_t* bits_out) {
  int rc = bind(ctx);
  if (rc) return rc;
  // out == NULL with cap_words == 0: the lengths only (bits_out), no stream written
  if ((!samples && n) || !bits_out || bit0 >= 64 || (out ? cap_words == 0 : cap_words != 0)) return BIC_EINVAL;
  if (n0 + n >= 0x80000000ull || a0 >= 0x80000000ull) return BIC_EINVAL;
  if ((rc = ensure_scratch(ctx, bic::sample_scratch_bytes(n)))) return rc;
  const bic::SampleScratch ss = bic::carve_sample_scratch(ctx->scratch, n);
  timed(ctx, "golomb_samples", [&] {
    bic::launch_golomb_samples(ctx->cur, samples, n, n0, a0, bit0, out, cap_words, bits_out, ss, ctx->flags);
  });
  BIC_HIP(hipGetLastError());
  return BIC_OK;
}

int bic_patch_encode(bic_ctx* ctx, const uint64_t* plane, size_t rows, size_t cols, size_t wpr,
                     unsigned W, const uint64_t* lentab, uint32_t* weights, uint32_t* w_nonpred,
                     uint32_t* w_pred, uint8_t* modes, uint64_t* resid, uint64_t* stream,
                     size_t cap_words, uint64_t* stats) {
  int rc = bind(ctx);
  if (rc) return rc;
  if (!plane || !lentab || !stream || !stats || cap_words == 0) return BIC_EINVAL;
  if (W < 1 || W > 64 || rows % W || cols % W || !geom_ok(rows, cols, wpr)) return BIC_EINVAL;
  const size_t M = (size_t)W * W;
  const size_t ntiles = (rows / W) * (cols / W);
  if (ntiles >= 0x80000000ull || (unsigned long long)ntiles * M >= 0x80000000ull) return BIC_EINVAL;
  // length table -> device (pinned staging; the previous copy must be done before reuse). A table
  // equal to the one already on the device (the usual case: one W per run) is not re-sent, so
  // repeated calls do not synchronise the host with the stream.
  if (ctx->lentab_host.size() != M + 1 ||
      std::memcmp(ctx->lentab_host.data(), lentab, (M + 1) * sizeof(uint64_t)) != 0) {
    if (ctx->staging_cap < M + 1) {
      BIC_HIP(hipStreamSynchronize(ctx->cur));
      if (ctx->staging) (void)hipHostFree(ctx->staging);
      if (ctx->lentab) (void)hipFree(ctx->lentab);
      ctx->staging = nullptr;
      ctx->lentab = nullptr;
      ctx->staging_cap = ctx->lentab_cap = 0;
      if (hipHostMalloc(&ctx->staging, (M + 1) * sizeof(uint64_t)) != hipSuccess) return BIC_ENOMEM;
      if (hipMalloc(&ctx->lentab, (M + 1) * sizeof(uint64_t)) != hipSuccess) return BIC_ENOMEM;
      ctx->staging_cap = ctx->lentab_cap = M + 1;
    } else {
      BIC_HIP(hipStreamSynchronize(ctx->cur));
    }
    std::memcpy(ctx->staging, lentab, (M + 1) * sizeof(uint64_t));
    BIC_HIP(hipMemcpyAsync(ctx->lentab, ctx->staging, (M + 1) * sizeof(uint64_t),
                           hipMemcpyHostToDevice, ctx->cur));
    ctx->lentab_host.assign(lentab, lentab + M + 1);
  }
  // per-tile chosen weights feed the sample coder: use the caller's array or scratch
  const size_t wbytes = ((ntiles * sizeof(uint32_t)) + 255) & ~(size_t)255;
  const uint32_t nsplit = bic::tiles_split_blocks((uint32_t)rows, (uint32_t)cols, W);
  const size_t lbytes = ((size_t)nsplit * 8 + 255) & ~(size_t)255;
  if ((rc = ensure_scratch(ctx, wbytes + lbytes + bic::sample_scratch_bytes(ntiles)))) return rc;
  uint32_t* wts = weights ? weights : reinterpret_cast<uint32_t*>(ctx->scratch);
  uint64_t* lpart = reinterpret_cast<uint64_t*>(reinterpret_cast<char*>(ctx->scratch) + wbytes);
  const bic::SampleScratch ss =
      bic::carve_sample_scratch(reinterpret_cast<char*>(ctx->scratch) + wbytes + lbytes, ntiles);
  if (nsplit) {
    // three launches: tiles (which zero the coder's scratch and leave per-block length sums), the
    // coder's scan and emit (stats[0..1] from the scan, stats[2] = the length sums, from the emit)
    timed(ctx, "tiles", [&] {
      bic::launch_tiles_split(ctx->cur, plane, (uint32_t)rows, (uint32_t)cols, (uint32_t)wpr, W, ctx->lentab, wts,
                              w_nonpred, w_pred, modes, resid, lpart, ss.counter, (uint32_t)(ss.zero_bytes / 4));
    });
    timed(ctx, "golomb_samples", [&] {
      bic::launch_golomb_samples(ctx->cur, wts, ntiles, 0, 0, 0, stream, cap_words, stats, ss, ctx->flags, true, lpart,
                                 nsplit, stats + 2);
    });
    BIC_HIP(hipGetLastError());
    return BIC_OK;
  }
  BIC_HIP((bic::launch_fill(ctx->cur, stats, 0, 3 * sizeof(uint64_t)), hipGetLastError()));
  timed(ctx, "tiles", [&] {
    bic::launch_tiles(ctx->cur, plane, (uint32_t)rows, (uint32_t)cols, (uint32_t)wpr, W, ctx->lentab, wts,
                      w_nonpred, w_pred, modes, resid, stats);
  });
  timed(ctx, "golomb_samples", [&] {
    bic::launch_golomb_samples(ctx->cur, wts, ntiles, 0, 0, 0, stream, cap_words, stats, ss, ctx->flags);
  });
  BIC_HIP(hipGetLastError());
  return BIC_OK;
}

int bic_pack_streams(bic_ctx* ctx, const uint64_t* slots, int nplanes, size_t slot_words,
                     const uint64_t* plane_bits, uint64_t* dst, uint64_t* word_off) {
  int rc = bind(ctx);
  if (rc) return rc;
  if (!slots || !plane_bits || !dst || !word_off || nplanes < 1 || nplanes > 65535 || slot_words == 0)
    return BIC_EINVAL;
  timed(ctx, "pack", [&] { bic::launch_pack(ctx->cur, slots, nplanes, slot_words, plane_bits, dst, word_off); });
  BIC_HIP(hipGetLastError());
  return BIC_OK;
}

int bic_patch_search(bic_ctx* ctx, const uint64_t* plane, size_t rows, size_t cols, size_t wpr, unsigned W,
                     uint32_t* besti, uint32_t* bestj, uint32_t* bestd) {
  int rc = bind(ctx);
  if (rc) return rc;
  if (W < 1 || W > 64 || !geom_ok(rows, cols, wpr) || rows > 0x7fffffffu) return BIC_EINVAL;
  const size_t ntiles = ((W - 1 + rows) / W) * ((W - 1 + cols) / W);
  if (ntiles && (!plane || !besti || !bestj || !bestd)) return BIC_EINVAL;
  if ((unsigned long long)rows * cols >= (1ull << 40)) return BIC_EINVAL;  // scan index field
  timed(ctx, "patch_search", [&] {
    bic::launch_patch_search(ctx->cur, plane, (uint32_t)rows, (uint32_t)cols, (uint32_t)wpr, W, besti, bestj, bestd);
  });
  BIC_HIP(hipGetLastError());
  return BIC_OK;
}

static int match_encode_impl(bic_ctx* ctx, const uint64_t* plane, size_t rows, size_t cols, size_t wpr, unsigned W,
                             unsigned T, unsigned R, const double* enuml, uint32_t* besti, uint32_t* bestj,
                             uint32_t* bestd, uint32_t* weights, uint8_t* modes, uint64_t* resid,
                             uint64_t* stream_match, uint64_t* stream_nomatch, size_t cap_words, uint64_t* stats,
                             int invert, uint8_t* inverted, int var = 0) {
  int rc = bind(ctx);
  if (rc) return rc;
  if (!plane || !resid || !enuml || !stream_match || !stream_nomatch || !stats || cap_words == 0)
    return BIC_EINVAL;
  if (W < 1 || W > 64 || rows % W || cols % W || !geom_ok(rows, cols, wpr)) return BIC_EINVAL;
  if (R > 32767 || T > 0x7fffffffu || rows > 0x3fffffffu || cols > 0x3fffffffu) return BIC_EINVAL;
  const size_t M = (size_t)W * W;
  const size_t ntiles = (rows / W) * (cols / W);
  if (ntiles >= 0x80000000ull / 64 || (unsigned long long)ntiles * M >= 0x80000000ull) return BIC_EINVAL;
  for (size_t w = 0; w <= M; ++w)
    if (!(enuml[w] >= 0.0 && enuml[w] < 1e15)) return BIC_EINVAL;  // lengths stay exact in double
  if (ctx->enuml_host.size() != M + 1 || std::memcmp(ctx->enuml_host.data(), enuml, (M + 1) * sizeof(double)) != 0) {
    BIC_HIP(hipStreamSynchronize(ctx->cur));  // the previous copy out of the staging buffer is done
    if (ctx->enuml_cap < M + 1) {
      if (ctx->enuml_staging) (void)hipHostFree(ctx->enuml_staging);
      if (ctx->enuml) (void)hipFree(ctx->enuml);
      ctx->enuml_staging = nullptr;
      ctx->enuml = nullptr;
      ctx->enuml_cap = 0;
      if (hipHostMalloc(&ctx->enuml_staging, (M + 1) * sizeof(double)) != hipSuccess) return BIC_ENOMEM;
      if (hipMalloc(&ctx->enuml, (M + 1) * sizeof(double)) != hipSuccess) return BIC_ENOMEM;
      ctx->enuml_cap = M + 1;
    }
    std::memcpy(ctx->enuml_staging, enuml, (M + 1) * sizeof(double));
    BIC_HIP(hipMemcpyAsync(ctx->enuml, ctx->enuml_staging, (M + 1) * sizeof(double), hipMemcpyHostToDevice,
                           ctx->cur));
    ctx->enuml_host.assign(enuml, enuml + M + 1);
  }
  if (ntiles == 0) {
    BIC_HIP((bic::launch_fill(ctx->cur, stats, 0, 4 * sizeof(uint64_t)), hipGetLastError()));
    return BIC_OK;
  }
  const bic::MatchSched sched = bic::match_schedule(W, R, (uint32_t)cols, ctx->match_parts, (uint32_t)var,
                                                    (uint32_t)rows);
  if ((rc = ensure_scratch(ctx, bic::match_scratch_bytes(ntiles, sched)))) return rc;
  if (resid != plane)
    BIC_HIP(hipMemcpyAsync(resid, plane, rows * wpr * sizeof(uint64_t), hipMemcpyDeviceToDevice, ctx->cur));
  bic::MatchArgs a{};
  a.I = resid;
  a.rows = (uint32_t)rows;
  a.cols = (uint32_t)cols;
  a.wpr = (uint32_t)wpr;
  a.used = (uint32_t)((cols + 63) / 64);
  a.W = W;
  a.nx = (uint32_t)(cols / W);
  a.ny = (uint32_t)(rows / W);
  a.T = T;
  a.R = (int)R;
  a.enuml = ctx->enuml;
  a.besti = besti;
  a.bestj = bestj;
  a.bestd = bestd;
  a.weights = weights;
  a.modes = modes;
  a.flags = ctx->flags;
  a.inv = invert ? 1u : 0u;
  a.inverted = inverted;
  a.var = (uint32_t)var;
  timed(ctx, "match_tiles", [&] { bic::launch_match_tiles(ctx->cur, a, sched, ctx->scratch); });
  timed(ctx, "match_code", [&] {
    bic::launch_match_code(ctx->cur, a, reinterpret_cast<unsigned long long*>(stream_match),
                           reinterpret_cast<unsigned long long*>(stream_nomatch), cap_words, stats);
  });
  BIC_HIP(hipGetLastError());
  return BIC_OK;
}

int bic_match_encode(bic_ctx* ctx, const uint64_t* plane, size_t rows, size_t cols, size_t wpr, unsigned W,
                     unsigned T, unsigned R, const double* enuml, uint32_t* besti, uint32_t* bestj,
                     uint32_t* bestd, uint32_t* weights, uint8_t* modes, uint64_t* resid,
                     uint64_t* stream_match, uint64_t* stream_nomatch, size_t cap_words, uint64_t* stats) {
  return match_encode_impl(ctx, plane, rows, cols, wpr, W, T, R, enuml, besti, bestj, bestd, weights, modes, resid,
                           stream_match, stream_nomatch, cap_words, stats, 0, nullptr);
}

int bic_match_encode_inv(bic_ctx* ctx, const uint64_t* plane, size_t rows, size_t cols, size_t wpr, unsigned W,
                         unsigned T, unsigned R, const double* enuml, uint32_t* besti, uint32_t* bestj,
                         uint32_t* bestd, uint32_t* weights, uint8_t* modes, uint8_t* inverted, uint64_t* resid,
                         uint64_t* stream_match, uint64_t* stream_nomatch, size_t cap_words, uint64_t* stats) {
  return match_encode_impl(ctx, plane, rows, cols, wpr, W, T, R, enuml, besti, bestj, bestd, weights, modes, resid,
                           stream_match, stream_nomatch, cap_words, stats, 1, inverted);
}

int bic_match_encode_var(bic_ctx* ctx, int variant, const uint64_t* plane, size_t rows, size_t cols, size_t wpr,
                         unsigned W, unsigned T, unsigned R, const double* enuml, uint32_t* besti, uint32_t* bestj,
                         uint32_t* bestd, uint32_t* weights, uint8_t* modes, uint64_t* resid, uint64_t* stream_match,
                         uint64_t* stream_nomatch, size_t cap_words, uint64_t* stats) {
  if (variant == 7 || variant == 8)
    return match_encode_impl(ctx, plane, rows, cols, wpr, W, T, R, enuml, besti, bestj, bestd, weights, modes, resid,
                             stream_match, stream_nomatch, cap_words, stats, variant == 8, nullptr);
  if (variant < 4 || variant > 6) return BIC_EINVAL;
  return match_encode_impl(ctx, plane, rows, cols, wpr, W, T, R, enuml, besti, bestj, bestd, weights, modes, resid,
                           stream_match, stream_nomatch, cap_words, stats, 0, nullptr, variant);
}

int bic_set_match_parts(bic_ctx* ctx, unsigned parts) {
  if (!ctx) return BIC_EINVAL;
  ctx->match_parts = parts;
  return BIC_OK;
}

int bic_pbm_unpack(bic_ctx* ctx, const uint8_t* raster, size_t rows, size_t cols, uint64_t* plane, size_t wpr) {
  int rc = bind(ctx);
  if (rc) return rc;
  if (!geom_ok(rows, cols, wpr) || (rows && (!raster || !plane))) return BIC_EINVAL;
  timed(ctx, "pbm_unpack", [&] {
    bic::launch_pbm(ctx->cur, false, raster, nullptr, nullptr, plane, (uint32_t)rows, (uint32_t)cols, (uint32_t)wpr);
  });
  BIC_HIP(hipGetLastError());
  return BIC_OK;
}

int bic_planes_to_gray(bic_ctx* ctx, const uint64_t* planes, int plane0, int nplanes, size_t rows, size_t cols,
                       size_t wpr, int sample_bytes, void* gray, size_t pitch) {
  int rc = bind(ctx);
  if (rc) return rc;
  if ((sample_bytes != 1 && sample_bytes != 2) || plane0 < 0 || nplanes < 1 || plane0 + nplanes > 8 * sample_bytes)
    return BIC_EINVAL;
  if (!geom_ok(rows, cols, wpr) || pitch < cols * (size_t)sample_bytes || (rows && (!planes || !gray)))
    return BIC_EINVAL;
  if (rows == 0) return BIC_OK;
  timed(ctx, "planes_to_gray", [&] {
    bic::launch_planes_gray(ctx->cur, planes, (uint32_t)rows, (uint32_t)cols, (uint32_t)wpr, plane0, nplanes,
                            sample_bytes, static_cast<uint8_t*>(gray), (uint64_t)pitch);
  });
  BIC_HIP(hipGetLastError());
  return BIC_OK;
}

int bic_pgm_bitplanes(bic_ctx* ctx, const uint8_t* raster, size_t rows, size_t cols, int maxval, int plane0,
                      int nplanes, uint64_t* planes, size_t wpr) {
  int rc = bind(ctx);
  if (rc) return rc;
  if (maxval < 1 || maxval > 65535 || plane0 < 0 || nplanes < 1 || plane0 + nplanes > (maxval < 256 ? 8 : 16))
    return BIC_EINVAL;
  if (!geom_ok(rows, cols, wpr) || (rows && (!raster || !planes))) return BIC_EINVAL;
  if (rows == 0) return BIC_OK;
  timed(ctx, "pgm_bitplanes", [&] {
    bic::launch_raster_planes(ctx->cur, raster, maxval < 256 ? 1 : 2, (uint32_t)rows, (uint32_t)cols, plane0, nplanes,
                              planes, (uint32_t)wpr);
  });
  BIC_HIP(hipGetLastError());
  return BIC_OK;
}

namespace {
// pnm.cpp:5-18 skip_comments on a byte buffer: whitespace, then a '#' line (fgets into a 100-byte
// buffer: at most 99 bytes, through the newline) and again
void pnm_skip_comments(const uint8_t* b, size_t n, size_t& i) {
  for (;;) {
    while (i < n && std::isspace(b[i])) ++i;
    if (i >= n || b[i] != '#') return;
    ++i;  // the '#' (fgetc), then fgets' at most 99 bytes
    size_t k = 0;
    while (i < n && k < 99) {
      const uint8_t c = b[i++];
      ++k;
      if (c == '\n') break;
    }
  }
}
// fscanf("%d"): leading whitespace, an optional sign, digits
bool pnm_int(const uint8_t* b, size_t n, size_t& i, long long& v) {
  while (i < n && std::isspace(b[i])) ++i;
  bool neg = false;
  if (i < n && (b[i] == '+' || b[i] == '-')) neg = b[i++] == '-';
  if (i >= n || !std::isdigit(b[i])) return false;
  v = 0;
  while (i < n && std::isdigit(b[i])) {
    v = v * 10 + (b[i++] - '0');
    if (v > 0x7fffffffLL) return false;
  }
  if (neg) v = -v;
  return true;
}
}  // namespace

int bic_pnm_parse_header(const uint8_t* bytes, size_t n, bic_pnm_info* info) {
  if (!bytes || !info || n < 2 || bytes[0] != 'P') return BIC_EINVAL;
  size_t i = 2;
  long long w = 0, h = 0, mv = 1;
  const int type = bytes[1] - '0';
  if (type == 4) {  // pbm.cpp:4-27: " %d" then " %d " (which also eats whitespace-valued raster bytes)
    if (!pnm_int(bytes, n, i, w) || !pnm_int(bytes, n, i, h) || w <= 0 || h <= 0) return BIC_EINVAL;
    while (i < n && std::isspace(bytes[i])) ++i;
  } else if (type == 2 || type == 5 || type == 6) {  // pnm.cpp:20-42
    pnm_skip_comments(bytes, n, i);
    if (!pnm_int(bytes, n, i, w)) return BIC_EINVAL;
    pnm_skip_comments(bytes, n, i);
    if (!pnm_int(bytes, n, i, h)) return BIC_EINVAL;
    pnm_skip_comments(bytes, n, i);
    if (!pnm_int(bytes, n, i, mv)) return BIC_EINVAL;
    if (w <= 0 || h <= 0 || mv <= 0 || mv > 65535) return BIC_EINVAL;
    ++i;  // the fgetc after maxval
  } else {
    return BIC_EINVAL;
  }
  if (i > n) return BIC_EINVAL;
  info->type = type;
  info->cols = (size_t)w;
  info->rows = (size_t)h;
  info->maxval = (int)mv;
  info->data_offset = i;
  return BIC_OK;
}

int bic_pbm_pack(bic_ctx* ctx, const uint64_t* plane, size_t rows, size_t cols, size_t wpr, uint8_t* raster) {
  int rc = bind(ctx);
  if (rc) return rc;
  if (!geom_ok(rows, cols, wpr) || (rows && (!raster || !plane))) return BIC_EINVAL;
  timed(ctx, "pbm_pack", [&] {
    bic::launch_pbm(ctx->cur, true, nullptr, raster, plane, nullptr, (uint32_t)rows, (uint32_t)cols, (uint32_t)wpr);
  });
  BIC_HIP(hipGetLastError());
  return BIC_OK;
}

// ---- f4: GF(2) algebra -----------------------------------------------------------------------
namespace {
bool gf2_geom(size_t rows, size_t cols, size_t wpr) {
  return rows <= 0x7fffffffu && cols <= 0x7fffff00u && wpr >= (cols + 63) / 64 && wpr <= 0xffffffffu;
}
}  // namespace

int bic_gf2_transpose(bic_ctx* ctx, const uint64_t* src, size_t rows, size_t cols, size_t wpr, uint64_t* dst,
                      size_t dst_wpr) {
  int rc = bind(ctx);
  if (rc) return rc;
  if (!gf2_geom(rows, cols, wpr) || !gf2_geom(cols, rows, dst_wpr)) return BIC_EINVAL;
  if (!rows || !cols) return BIC_OK;
  if (!src || !dst) return BIC_EINVAL;
  timed(ctx, "gf2_transpose", [&] {
    bic::launch_gf2_transpose(ctx->cur, src, (uint32_t)rows, (uint32_t)wpr, (uint32_t)((cols + 63) / 64),
                              (uint32_t)cols, dst, (uint32_t)dst_wpr, (uint32_t)((rows + 63) / 64));
  });
  BIC_HIP(hipGetLastError());
  return BIC_OK;
}

// mul_AB as the kernel; mul_AtB = transpose(A) then mul_AB; mul_ABt = A times the transpose of B's
// whole words (its loop runs over A's blocks, binmat.cpp:586-588), stored for j < B.cols.
int bic_gf2_mul(bic_ctx* ctx, int op, const uint64_t* A, size_t a_rows, size_t a_cols, size_t a_wpr,
                const uint64_t* B, size_t b_rows, size_t b_cols, size_t b_wpr, uint64_t* C, size_t c_rows,
                size_t c_cols, size_t c_wpr) {
  int rc = bind(ctx);
  if (rc) return rc;
  if (!gf2_geom(a_rows, a_cols, a_wpr) || !gf2_geom(b_rows, b_cols, b_wpr) || !gf2_geom(c_rows, c_cols, c_wpr))
    return BIC_EINVAL;
  const uint32_t cw = (uint32_t)((c_cols + 63) / 64);
  switch (op) {
    case BIC_GF2_AB:
      if (c_rows != a_rows || c_cols != b_cols || a_cols != b_rows) return BIC_EINVAL;
      break;
    case BIC_GF2_ATB:
      if (c_rows != a_cols || c_cols != b_cols || a_rows != b_rows) return BIC_EINVAL;
      break;
    case BIC_GF2_ABT:
      if (c_rows != a_rows || c_cols != b_rows || a_cols != b_cols) return BIC_EINVAL;
      break;
    case BIC_GF2_ATBT:
      if (c_rows != a_cols || c_cols != b_rows || a_rows != b_cols) return BIC_EINVAL;
      return BIC_OK;  // binmat.cpp:596-604: "FALTA!" -- C is returned unchanged
    default:
      return BIC_EINVAL;
  }
  if (!c_rows || !cw) return BIC_OK;
  if (!A || !B || !C) return BIC_EINVAL;
  if (op == BIC_GF2_AB) {
    timed(ctx, "gf2_mul", [&] {
      bic::launch_gf2_ab(ctx->cur, A, (uint32_t)a_rows, (uint32_t)a_wpr, (uint32_t)a_cols, B, (uint32_t)b_wpr, cw, C,
                         (uint32_t)c_wpr, cw * 64u);
    });
    BIC_HIP(hipGetLastError());
    return BIC_OK;
  }
  // the transposed operand: At (a_cols x a_rows) or B's whole words transposed (64 aw x b_rows)
  const bool atb = op == BIC_GF2_ATB;
  const uint32_t aw = (uint32_t)((a_cols + 63) / 64);
  const uint64_t t_rows = atb ? a_cols : 64ull * aw, t_src_rows = atb ? a_rows : b_rows;
  const uint32_t t_words = (uint32_t)((t_src_rows + 63) / 64);
  uint64_t* T = nullptr;
  if (t_rows && t_words) {
    BIC_HIP(hipMallocAsync(reinterpret_cast<void**>(&T), (size_t)t_rows * t_words * 8, ctx->cur));
    timed(ctx, "gf2_transpose", [&] {
      if (atb)
        bic::launch_gf2_transpose(ctx->cur, A, (uint32_t)a_rows, (uint32_t)a_wpr, aw, (uint32_t)a_cols, T, t_words,
                                  t_words);
      else
        bic::launch_gf2_transpose(ctx->cur, B, (uint32_t)b_rows, (uint32_t)b_wpr, aw, (uint32_t)t_rows, T, t_words,
                                  t_words);
    });
  }
  timed(ctx, "gf2_mul", [&] {
    if (atb)
      bic::launch_gf2_ab(ctx->cur, T, (uint32_t)a_cols, t_words, (uint32_t)a_rows, B, (uint32_t)b_wpr, cw, C,
                         (uint32_t)c_wpr, cw * 64u);
    else  // cw == t_words (c_cols == b_rows); bits j >= b_rows of the product are 0
      bic::launch_gf2_ab(ctx->cur, A, (uint32_t)a_rows, (uint32_t)a_wpr, (uint32_t)t_rows, T, t_words, cw, C,
                         (uint32_t)c_wpr, (uint32_t)std::min<size_t>(b_cols, 64ull * cw));
  });
  if (T) (void)hipFreeAsync(T, ctx->cur);
  BIC_HIP(hipGetLastError());
  return BIC_OK;
}

// log2 C(n, r): the reference's enumL / enumerative_codelength (coding.cpp:19-22,
// compress7_test.cpp:25-28) without GSL. Exact at r in {0, n} (0) and, for power-of-two n,
// at r in {1, n-1} (log2 n -- where GSL's last-ulp rounding is unpinned, SURVEY.md §8 c);
// long-double lgamma elsewhere.
double bic_enum_codelength(unsigned n, unsigned r) {
  if (r == 0 || r >= n) return 0.0;
  const unsigned m = r * 2 > n ? n - r : r;
  if (m == 1) {
    if ((n & (n - 1)) == 0) {
      unsigned e = 0;
      while ((1u << e) < n) ++e;
      return (double)e;
    }
    return (double)std::log2((long double)n);
  }
  const long double ln = std::lgamma((long double)n + 1.0L) - std::lgamma((long double)m + 1.0L) -
                         std::lgamma((long double)(n - m) + 1.0L);
  return (double)(ln * 1.442695040888963407359924681001892137L);
}

int bic_tile_lentab(unsigned W, uint64_t* lentab) {
  if (W < 1 || W > 64 || !lentab) return BIC_EINVAL;
  const unsigned M = W * W;
  for (unsigned w = 0; w <= M; ++w)  // compress7_test.cpp:220-221: (idx_t)(1 + 1 + enumL(M, w))
    lentab[w] = (uint64_t)(2.0 + bic_enum_codelength(M, w));
  return BIC_OK;
}

int bic_prof_enable(bic_ctx* ctx, int on) {
  if (!ctx) return BIC_EINVAL;
  ctx->prof_on = on != 0;
  return BIC_OK;
}

int bic_prof_only(bic_ctx* ctx, const char* name) {
  if (!ctx) return BIC_EINVAL;
  ctx->prof_only = name ? name : "";
  return BIC_OK;
}

int bic_prof_collect(bic_ctx* ctx, char* buf, size_t cap) {
  int rc = bind(ctx);
  if (rc) return rc;
  if (!buf || cap == 0) return BIC_EINVAL;
  BIC_HIP(hipStreamSynchronize(ctx->cur));
  std::map<std::string, std::pair<unsigned long, double>> agg;
  for (auto& r : ctx->recs) {
    float ms = 0.f;
    if (hipEventElapsedTime(&ms, r.a, r.b) != hipSuccess) ms = -1.f;
    auto& e = agg[r.name];
    e.first += 1;
    e.second += ms;
    ctx->pool.push_back(r.a);
    ctx->pool.push_back(r.b);
  }
  ctx->recs.clear();
  (void)hipGetLastError();  // a failed elapsed-time query (-1 above) must not fail the next call
  std::string outs;
  for (auto& kv : agg) {
    char line[160];
    std::snprintf(line, sizeof line, "%s %lu %.6f\n", kv.first.c_str(), kv.second.first, kv.second.second);
    outs += line;
  }
  std::snprintf(buf, cap, "%s", outs.c_str());
  return outs.size() < cap ? BIC_OK : BIC_ENOSPC;
}

#ifdef BIC_STAMPS
int bic_debug_stamps(uint64_t* host, size_t n) { return bic::read_stamps(host, n); }
int bic_debug_match_stamps(uint64_t* host, size_t n) { return bic::read_match_stamps(host, n); }
#endif

}  // extern "C"
