// bic_internal.h -- shared between the HIP kernels (bic_kernels.hip) and the C ABI
// (bic_capi.cpp). Not installed; the public surface is include/bic.h.
#pragma once
#include <hip/hip_runtime.h>
#include <stddef.h>
#include <stdint.h>

namespace bic {

// Geometry of one batch of planes as the chunk kernels see it. A "chunk" is the unit
// one wavefront processes: up to 64*WPL consecutive words of ONE row (lane l handles
// words c0 + 64*t + l for t < WPL, so every load instruction is 512 contiguous bytes).
struct Geom {
  uint32_t rows, cols, wpr;
  uint32_t used;  // ceil(cols/64): words that hold pixels
  uint32_t wpl;   // words per lane (1, 2 or 4)
  uint32_t wpc;   // words per chunk = 64*wpl
  uint32_t cpr;   // chunks per row = ceil(used/wpc)
  uint32_t nplanes;
  uint64_t trail;             // valid-bit mask of word used-1 (binmat.cpp:146-147)
  uint64_t plane_words;       // rows*wpr
  uint64_t chunks_per_plane;  // rows*cpr
  uint64_t nchunks;           // nplanes*chunks_per_plane
  uint64_t words_used;        // rows*used per plane (word_bits stride)
};

Geom make_geom(size_t rows, size_t cols, size_t wpr, int nplanes);

// Per-call device scratch carved from the context arena.
struct ChunkScratch {
  uint32_t* ones;      // [nchunks]
  int32_t* last;       // [nchunks] last 1-column in the chunk, -1 if none
  int32_t* first;      // [nchunks] first 1-column in the chunk, INT32_MAX if none
  uint32_t* nbase;     // [nchunks] global sample index of the chunk's first 1
  int32_t* jprev;      // [nchunks] column of the last 1 before the chunk in its row, -1
  uint64_t* bits;      // [nchunks] Golomb bits of the chunk
  uint64_t* boff;      // [nchunks] absolute bit offset of the chunk in `out`
  uint32_t* word_bits; // [nplanes*rows*used]
  uint64_t* plane_F;   // [nplanes] raster index of the plane's first residual 1 (~0 if none)
  uint64_t* plane_ones;// [nplanes]
};
size_t chunk_scratch_bytes(const Geom& g);
ChunkScratch carve_chunk_scratch(void* base, const Geom& g);

// Launchers (all asynchronous on `s`). flags[0] = overflow, flags[1] = domain error.
void launch_bitplanes_u8(hipStream_t s, const uint8_t* gray, size_t pitch, uint32_t rows,
                         uint32_t cols, int plane0, int nplanes, uint64_t* planes, uint32_t wpr);
void launch_count(hipStream_t s, const Geom& g, const uint64_t* planes, int predict,
                  const ChunkScratch& cs, uint64_t* resid, uint64_t* weight_out);
void launch_scan_rows(hipStream_t s, const Geom& g, const ChunkScratch& cs);
// bic_med_residual for rows of <= 256 words: RPW rows per wave, 16-byte loads; part = one u32 per
// wave (scratch, ceil(rows/8) per plane)
bool med_rows_supported(const Geom& g, const void* planes, const void* resid);
// a9 adaptive EG (bic_egad.hip)
size_t egad_scratch_bytes(uint64_t nrows);
// out null: no emission (index only); index (nullable): per row its first bit in the plane's stream and
// the coder state there (bic_egad_row_index)
// nib: egad_build_nib's table in device memory (the context's byte-table buffer, kLutEgadNib)
void launch_egad(hipStream_t s, const uint64_t* planes, uint32_t rows, uint32_t cols, uint32_t wpr, uint32_t nplanes,
                 int predict, uint64_t* out, uint64_t slot, uint64_t* bits, void* scratch, uint32_t* flags,
                 uint64_t* index, const uint64_t* nib);
// the adaptive EG coder's nibble table (976 u64 entries), built on the host
void egad_build_nib(uint64_t* T);
constexpr size_t kLutEgadNib = 3 * 256;         // its offset in the context's byte-table buffer (u64 words)
constexpr size_t kLutEgadDec = kLutEgadNib + 976;  // the decoder's table (992 u64 words)
constexpr size_t kLutWords = kLutEgadDec + 992;    // the whole buffer
// f1 decoders (bic_decode.hip)
bool decode_supported(uint32_t cols);
size_t decode_scratch_bytes(uint32_t rows, uint32_t wpr, uint32_t nplanes);
// egnib: egad_build_dec_nib's table in device memory (the context's byte-table buffer, kLutEgadDec)
void launch_decode(hipStream_t s, int coder, const uint64_t* streams, uint64_t slot, const uint64_t* word_off,
                   const uint64_t* plane_bits, const uint64_t* index, const uint8_t* p00, uint32_t rows,
                   uint32_t cols, uint32_t wpr, uint32_t nplanes, int predict, uint64_t* out, void* scratch,
                   uint32_t* flags, const uint64_t* egnib);
// the adaptive EG decoder's nibble table (62 states x 16 nibbles, u64), built on the host
void egad_build_dec_nib(uint64_t* T);
void launch_med_rows(hipStream_t s, const Geom& g, const uint64_t* planes, int predict, uint64_t* resid,
                     uint32_t* part, uint64_t* weight_out);
void launch_golomb_bits(hipStream_t s, const Geom& g, const uint64_t* planes, int predict,
                        const ChunkScratch& cs);
void launch_golomb_offsets(hipStream_t s, const Geom& g, const ChunkScratch& cs, uint64_t* out,
                           uint64_t slot_words, uint64_t* plane_bits, uint32_t* flags);
void launch_golomb_emit(hipStream_t s, const Geom& g, const uint64_t* planes, int predict,
                        const ChunkScratch& cs, uint64_t* out, uint64_t slot_words);
void launch_eg_emit(hipStream_t s, const Geom& g, const uint64_t* planes, int predict,
                    const ChunkScratch& cs, uint64_t* out, uint64_t slot_words,
                    uint64_t* plane_bits, uint32_t* flags);

// Sample coder (GolombCoder::codeSample over an array).
struct SampleScratch {
  uint32_t* counter;   // block tickets
  uint64_t* a_rec;     // [nblk] look-back records: sums of samples
  uint64_t* b_rec;     // [nblk] look-back records: codeword bits
  uint64_t* blk_A;     // [nblk] accumulated error before the block
  uint64_t* blk_off;   // [nblk] absolute bit offset of the block
  size_t zero_bytes;   // counter + records, zeroed per launch
};
size_t sample_scratch_bytes(size_t n);
SampleScratch carve_sample_scratch(void* base, size_t n);
// prezeroed: the scratch's counter and records are already 0 (k_tiles_split zeroes them); lpart
// (nullable): nlpart per-block sums added into *lout by the emit launch
void launch_golomb_samples(hipStream_t s, const uint32_t* samples, size_t n, uint64_t n0,
                           uint64_t a0, unsigned bit0, uint64_t* out, size_t cap_words,
                           uint64_t* bits_out, const SampleScratch& ss, uint32_t* flags, bool prezeroed = false,
                           const uint64_t* lpart = nullptr, uint32_t nlpart = 0, uint64_t* lout = nullptr);
// the aligned tile path split over 4 waves per strip (W in 8, 16, 32, 64; else 0 blocks)
uint32_t tiles_split_blocks(uint32_t rows, uint32_t cols, uint32_t W);
void launch_tiles_split(hipStream_t s, const uint64_t* plane, uint32_t rows, uint32_t cols, uint32_t wpr, uint32_t W,
                        const uint64_t* lentab_dev, uint32_t* weights, uint32_t* w_nonpred, uint32_t* w_pred,
                        uint8_t* modes, uint64_t* resid, uint64_t* lpart, uint32_t* zero, uint32_t nzero);

// Tiles (compress7 R = 0 path).
void launch_tiles(hipStream_t s, const uint64_t* plane, uint32_t rows, uint32_t cols,
                  uint32_t wpr, uint32_t W, const uint64_t* lentab_dev, uint32_t* weights,
                  uint32_t* w_nonpred, uint32_t* w_pred, uint8_t* modes, uint64_t* resid,
                  uint64_t* stats);

// Single-pass row encoder (bic_fused.hip), rows of at most 256 words.
struct FusedScratch {
  uint32_t* counter;
  uint64_t *ones_rec, *bits_rec;
  size_t zero_bytes;  // counter + records, zeroed per launch
  bool zero_ready = false;  // (single / two-pass) already zero: the previous call's k_fixup cleared them
  uint64_t *gboff, *glen, *gfrag, *gslow, *eboff, *elen, *efrag;
  uint32_t* row_o;   // ones of the plane before each row (two-pass / staged encoders)
  // staged encoder's count pass: per (plane, row, strip) the residual 1-count and the Golomb k
  // statistics record (bic_kstat.h); ns records per row
  uint32_t* sones;
  int4* krec;
  uint32_t* kpos;
  uint32_t ns;
  uint32_t* walk_ids;  // rows whose Golomb length is walked (k_row_walk)
  uint32_t* walk_o;    // their ones before (row_o), beside the id: the walk loads both at once
  uint32_t* rest_ids;  // rows the REST emit launch writes (mixed k, the plane's first 1; counter[3])
  // optional second stream for the REST launch (it then runs beside the main emit launch) and
  // the fork / join events; null: one stream
  hipStream_t aux = nullptr;
  hipEvent_t ev_fork = nullptr, ev_join = nullptr;
  // (bic_prof_*) recorded on the launch stream around the staged emission's main kernel alone
  hipEvent_t ev_main0 = nullptr, ev_main1 = nullptr;
  bool* ev_main_rec = nullptr;  // set true when ev_main1 was recorded (paths without a main kernel leave it)
  bool counted;      // the count pass already ran (bic_encode_gray's fused bitplane kernel)
  uint32_t* slow_n;
  uint64_t* slow_ids;
  // packed output (staged encoder): when off_g / off_e are set, each coder's streams are written
  // word-aligned back to back from word 0 of its buffer (what bic_pack_streams makes of slots) and
  // off_*[0..nplanes] receive the word offsets; pones / gbase / ebase: per-plane scratch
  uint64_t* off_g = nullptr;
  uint64_t* off_e = nullptr;
  uint64_t *pones, *gbase, *ebase;
  // row index for the decoders (bic_row_index): per row, the bit offset of its first Golomb
  // codeword in its plane's stream and the residual 1s of the plane before it; null: not written
  uint64_t* index = nullptr;
  // EG source (bic_encode_gray without planes, slot output): the count pass (launch_gray_rows with
  // out_e) wrote the EG stream in its uniform layout (row r at bit r (cols + 1) + 1) instead of the
  // residual planes; the Golomb kernels read the residual rows back from the stream, and one bit per
  // plane (efix, found by the ONES scan) is cleared after them (bic_fused.hip eg_fix_bit)
  bool eg_src = false;
  uint64_t* efix = nullptr;
  // EG source: the LEN scan lists the rows whose codewords all have k = 0 (entries [0 .. counter[4]))
  // and all k = 1 (entries [n ..], counter[5]) for the two class emission kernels (n = rows * planes),
  // each entry two u64 words: the row id | its Golomb length << 32, then its slot-relative Golomb bit
  // offset (gboff's value); a third list (entries [2n ..], counter[8]) holds the rows mixing k = 0 and
  // k = 1 whose per-codeword k the walk stored (kmask / row_wi, kcap walked rows): kmix_rows. The other
  // mixed rows (a codeword with k >= 2) stay the rest role's / k_emit_rest's
  uint64_t* cls = nullptr;
  uint64_t* sink = nullptr;   // 64 words the class kernels' idle lanes store to (a fixed store count)
  uint64_t* kmask = nullptr;  // per walked row (walk list index < kcap): its words' k = 1 masks
  uint32_t* row_wi = nullptr; // per kKMix row: its walk list index
  uint32_t kcap = 0;
  bool eg_src_one = false;  // (A/B: the one emission kernel k_emit_known for every class instead)
};
size_t fused_scratch_bytes(const Geom& g);
FusedScratch carve_fused_scratch(void* base, const Geom& g);
bool fused_supported(const Geom& g);
// host: the fused encoder's byte tables -- lut[0..255] 64-bit entries for k = 3, then (as u32)
// [2][256] packed entries for k = 1, 2 (bic_fused.hip encode_word); 4 KiB
void build_byte_lut(uint64_t* lut);
void launch_fused(hipStream_t s, const Geom& g, const uint64_t* planes, const uint64_t* lut, int predict,
                  const FusedScratch& fs,
                  uint64_t* out_g, uint64_t slot_g, uint64_t* bits_g, uint64_t* out_e, uint64_t slot_e,
                  uint64_t* bits_e, uint32_t* flags, int mode, int stage);
// launch_fused modes: the staged encoder (prefix kernels, then independent rows; planes 16-byte
// aligned with an even row pitch), the single kernel with decoupled look-backs, the two-pass one
constexpr int kEncStaged = 0, kEncSingle = 1, kEncTwoPass = 2;
// launch_fused stages: zero the tickets and records; the staged encoder's prefix kernels (counts,
// scans, lengths); the row kernel(s); the LDS-overflow rows and the words adjacent rows share
constexpr int kFusedPrep = 0, kFusedRows = 1, kFusedFinish = 2, kFusedPrefix = 3;
// the staged encoder's count passes also zero its kZeroWords counters (no separate fill launch)
constexpr uint32_t kZeroWords = 64;
void launch_row_ones(hipStream_t s, const Geom& g, const uint64_t* planes, int predict, uint32_t* sones,
                     int4* krec, uint32_t* kpos, uint32_t* zero);
// bitplanes + the count pass in one read of the gray image (bic_encode_gray); gray_strips(g)
// k statistics records per row (one per 64-word strip)
bool gray_rows_supported(const Geom& g, const void* gray, size_t pitch, const void* planes);
uint32_t gray_strips(const Geom& g);
// store_resid: the words stored are the med residual R (planes = the caller's bitplanes are not
// wanted; the encoder then reads R with predict off), not the bitplanes P. out_e (with predict, the
// bitplanes not wanted): the EG stream instead of R (FusedScratch::eg_src; slots of eg_stride
// words); planes is then unused
void launch_gray_rows(hipStream_t s, const uint8_t* gray, size_t pitch, const Geom& g, int predict, int plane0,
                      uint64_t* planes, uint32_t* sones, int4* krec, uint32_t* kpos, uint32_t* zero,
                      bool store_resid = false, uint64_t* out_e = nullptr, uint64_t eg_stride = 0);
// the count pass can write the EG stream (FusedScratch::eg_src): rows of whole 64-word strips only
bool gray_eg_supported(const Geom& g);

void launch_patch_search(hipStream_t s, const uint64_t* plane, uint32_t rows, uint32_t cols, uint32_t wpr,
                         uint32_t W, uint32_t* besti, uint32_t* bestj, uint32_t* bestd);

// compress7_test.cpp:117-275 with a search window (bic_match.hip). The plane I is modified in
// place. Per-tile outputs left null are carved from the scratch by launch_match_tiles.
struct MatchArgs {
  uint64_t* I;
  uint32_t rows, cols, wpr, used, W, nx, ny, T;
  int R;
  uint32_t G;                       // tile schedule: workgroups per tile
  uint32_t H, K;                    // team schedule: helpers per tile row; tiles of slack
  const double* enuml;              // device, W*W+1
  uint32_t* counter;                // scratch: ticket
  unsigned long long* key;          // scratch: per tile min key
  uint32_t* done;                   // scratch: per tile
  uint32_t* arrive;                 // scratch: per tile
  uint32_t* lens;                   // scratch: per tile chosen length
  uint32_t *besti, *bestj, *bestd, *weights;
  uint8_t* modes;
  uint32_t* flags;
  uint32_t inv;                     // compress8_test.cpp's patch inversion (0: compress7_test.cpp)
  uint8_t* inverted;                // per tile: the patch was flipped (nullable)
  // the loop of compress4_test.cpp (4), compress5_test.cpp (5), compress6_test.cpp (6); 0: compress7/8
  // (per-tile schedule only)
  uint32_t var;
  unsigned long long* key2;         // scratch, variant 5: per tile the first window with d < W*W/2
};
constexpr uint32_t kSchedTiles = 0, kSchedRows = 1, kSchedTeam = 2;
struct MatchSched {
  uint32_t kind, G, H, K;
};
// code: 0 auto; 1..256 workgroups per tile; 0x10000 | H a team of 1 + H workgroups per tile row;
// anything else: per-tile workgroups, count from W and R
// var (MatchArgs::var) != 0: per-tile workgroups only; rows bounds the region for the automatic count
MatchSched match_schedule(uint32_t W, uint32_t R, uint32_t cols, uint32_t code, uint32_t var = 0, uint32_t rows = 0);
size_t match_scratch_bytes(size_t ntiles, const MatchSched& m);
void launch_match_tiles(hipStream_t s, MatchArgs& a, const MatchSched& m, void* scratch);
void launch_match_code(hipStream_t s, const MatchArgs& a, unsigned long long* out_m, unsigned long long* out_n,
                       size_t cap_words, uint64_t* stats);
void launch_pbm(hipStream_t s, bool pack, const uint8_t* raster_in, uint8_t* raster_out, const uint64_t* plane_in,
                uint64_t* plane_out, uint32_t rows, uint32_t cols, uint32_t wpr);
// P5 samples (1 or 2 bytes, any alignment) -> planes plane0.. (bic_raster.hip)
void launch_raster_planes(hipStream_t s, const uint8_t* raster, int bpp, uint32_t rows, uint32_t cols, int plane0,
                          int nplanes, uint64_t* planes, uint32_t wpr);
void launch_planes_gray(hipStream_t s, const uint64_t* planes, uint32_t rows, uint32_t cols, uint32_t wpr, int plane0,
                        int nplanes, int bps, uint8_t* gray, uint64_t pitch);

// GF(2) algebra (bic_gf2.hip)
void launch_gf2_transpose(hipStream_t s, const uint64_t* src, uint32_t s_rows, uint32_t s_stride, uint32_t s_words,
                          uint32_t ncols_out, uint64_t* dst, uint32_t d_stride, uint32_t d_words);
void launch_gf2_ab(hipStream_t s, const uint64_t* A, uint32_t M, uint32_t a_stride, uint32_t kbits, const uint64_t* B,
                   uint32_t b_stride, uint32_t nw, uint64_t* C, uint32_t c_stride, uint32_t nset);

// Byte fill by a kernel (every device-side memset of the library): hipMemsetAsync enqueued under stream
// capture replays wrongly on this ROCm (the first captured memset of a process zeroed 800 of 1,280 bytes,
// tools/capture_memset_probe.py), and the encoders' calls are meant to be capturable
void launch_fill(hipStream_t s, void* dst, int value, size_t bytes);
void launch_pack(hipStream_t s, const uint64_t* slots, int nplanes, size_t slot_words,
                 const uint64_t* plane_bits, uint64_t* dst, uint64_t* word_off);

}  // namespace bic
