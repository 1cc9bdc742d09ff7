/*
 * bic.h -- C ABI of the MI355X (gfx950) hot path of nacho-pancho/binary-image-compression:
 *          bitplane extraction -> med (3-neighbour XOR) prediction -> per-row zero runs
 *          -> adaptive Golomb (GolombCoder) / "EG" run-length (EGCoder) coding.
 *
 * Plain pointers and sizes only; no C++ or torch types. Every bulk pointer is a DEVICE
 * pointer (hipMalloc'd or any device allocation of the caller); the caller allocates every
 * output (the reference's convention "C is assumed to have been allocated",
 * binmat.cpp:462). Calls enqueue on the context's stream and return immediately;
 * bic_sync() waits and reports deferred errors (e.g. an output slot that was too small).
 *
 * Plane layout = the reference's binary_matrix storage (binmat.h:8-19, 114-141): rows x wpr
 * uint64 words, row-major, column j in word j/64 at bit 63 - j%64 (MSB = leftmost pixel),
 * wpr >= ceil(cols/64). Bits past `cols` are ignored on input and written 0 on output.
 * Several planes are stored back to back (plane p at planes + p*rows*wpr).
 *
 * Encoded streams (build-defined container): one stream per plane, MSB-first
 * bit order, stored as big-endian 64-bit words (so the bytes in memory ARE the bit stream),
 * zero-padded to a 64-bit boundary. Plane p's stream starts at out + p*slot_words.
 *
 * Reference interface each entry replaces is cited per function (file:line under /root/reference/src).
 * Error codes: 0 = OK; never exceptions (style of pbm.h:8-16 ErrorCode).
 */
#ifndef BIC_H
#define BIC_H

#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

#define BIC_OK 0
#define BIC_EINVAL 1   /* bad argument (the reference asserts, e.g. binmat.cpp:465-469, GolombCoder.cpp:14) */
#define BIC_ENOMEM 2   /* device allocation failed */
#define BIC_EDEVICE 3  /* HIP runtime error */
#define BIC_ENOSPC 4   /* an output slot was too small (reported by bic_sync) */
#define BIC_ENODEV 5   /* no usable gfx950 device */
#define BIC_EDATA 6    /* a decoder met a malformed stream (reported by bic_sync) */

#define BIC_CODER_GOLOMB 0 /* GolombCoder::codeSample over the run samples (GolombCoder.cpp:29-34) */
#define BIC_CODER_EG 1     /* EGCoder::codeRun as written: incBlockSize disabled (eg.cpp:20-37) */
/* EGCoder::codeRun as intended: incBlockSize() per full block (eg.cpp:25 uncommented) -- the JPEG-LS
 * run mode the #if 0 decoder (eg.cpp:41-55) reads; EGLUT's index saturates at 31. bic_encode_planes
 * only (slots as for Golomb: bic_encode_slot_words). */
#define BIC_CODER_EG_ADAPTIVE 2

typedef struct bic_ctx bic_ctx;

/* ---- context ----------------------------------------------------------------------------- */
int bic_ctx_create(int device, bic_ctx** out);
int bic_ctx_destroy(bic_ctx* ctx);
/* Enqueue on an external hipStream_t (e.g. torch's current stream); NULL is the HIP null
 * (legacy default) stream. A new ctx enqueues on its own non-blocking stream, which
 * bic_ctx_own_stream returns. A ctx's scratch arena and residual buffer (bic_encode_gray) are
 * shared by all its calls, whatever stream is bound: calls enqueued on two different streams must
 * not run concurrently (use one ctx per stream). */
int bic_ctx_set_stream(bic_ctx* ctx, void* hip_stream);
void* bic_ctx_get_stream(bic_ctx* ctx);
void* bic_ctx_own_stream(bic_ctx* ctx);
/* Wait for all work enqueued by this ctx; returns BIC_ENOSPC if an encode since the last
 * sync overflowed its slot (that plane's stream is then incomplete), else BIC_OK/BIC_EDEVICE. */
int bic_sync(bic_ctx* ctx);
const char* bic_strerror(int code);
int bic_device_count(int* n);
/* Device memory for callers without a runtime of their own (the C++ reference-API layer,
 * ctypes/cgo bindings). bic_malloc/bic_free act on the ctx's device; the copies are ordered
 * on the ctx stream and return after the copy has completed (host buffers are pageable). */
int bic_malloc(bic_ctx* ctx, size_t bytes, void** dptr);
int bic_free(bic_ctx* ctx, void* dptr);
int bic_memcpy_h2d(bic_ctx* ctx, void* dst, const void* src, size_t bytes);
int bic_memcpy_d2h(bic_ctx* ctx, void* dst, const void* src, size_t bytes);
int bic_memset(bic_ctx* ctx, void* dst, int value, size_t bytes);
/* Pre-grow the ctx scratch so later calls do not allocate (needed before stream capture). */
int bic_reserve(bic_ctx* ctx, int nplanes, size_t rows, size_t cols);
/* Options: BIC_OPT_MULTIPASS = 1 forces the multi-pass chunk kernels for every geometry
 * (cross-checking the row encoders); 0 (default) picks a row encoder where it applies. */
#define BIC_OPT_MULTIPASS 1
/* Row encoders (same output; the alternatives are kept as cross-checks and for comparison).
 * Default: the staged encoder -- per-row sample counts, per-plane scans and per-row Golomb
 * lengths first, then every row written independently -- for batches of >= 32768 rows (all
 * planes; planes 16-byte aligned, even row pitch), the single kernel below that (fewer launches).
 * BIC_OPT_STAGED = 1: the staged encoder for every batch size. BIC_OPT_TWO_PASS = 1: lengths and
 * offsets found by decoupled look-backs, then every row written. BIC_OPT_SINGLE_KERNEL = 1: one
 * kernel, rows staged in LDS until decoupled look-backs give their offsets. */
#define BIC_OPT_TWO_PASS 2
#define BIC_OPT_SINGLE_KERNEL 3
#define BIC_OPT_STAGED 4
/* BIC_OPT_ONE_STREAM = 1: the staged encoder's two emission launches run one after the other on
 * the ctx stream instead of side by side on a second stream (same output; a test hook for the
 * launch ordering). */
#define BIC_OPT_ONE_STREAM 5
/* BIC_OPT_EG_SOURCE = 0: bic_encode_gray* without planes stores the med residual planes in a ctx
 * buffer for the encoder (the round-3 path) instead of writing the EG stream from the count pass
 * and reading the residual rows back from it (default 1, slot output with the EG coder; same
 * streams: a cross-check and A/B hook); 2: the EG source with one emission kernel for every row
 * class instead of one per class (A/B hook). */
#define BIC_OPT_EG_SOURCE 6
int bic_ctx_set_option(bic_ctx* ctx, int option, long value);

/* ---- a2: bitplane extraction (bitplane_tool.cpp:24-30) -----------------------------------
 * gray: rows x cols bytes with row pitch `pitch` (>= cols). Plane bi receives bit bi of every
 * pixel, LSB plane first; nplanes in 1..8 (bitplane_tool extracts #{bi : 2^bi < maxval}). */
int bic_bitplanes_u8(bic_ctx* ctx, const uint8_t* gray, size_t pitch, size_t rows, size_t cols,
                     int nplanes, uint64_t* planes, size_t wpr);
/* The planes plane0 .. plane0 + nplanes - 1 (plane0 + nplanes <= 8) only: output plane b is bit
 * plane0 + b of each pixel (bitplane_tool.cpp:24-30's plane index bi = plane0 + b). A rank of a
 * plane-sharded encode extracts its own share of one image this way. */
int bic_bitplanes_u8_range(bic_ctx* ctx, const uint8_t* gray, size_t pitch, size_t rows, size_t cols, int plane0,
                           int nplanes, uint64_t* planes, size_t wpr);

/* ---- a5/a6: med residual + weight (pred.cpp:3-15, binmat.cpp:57-67) -----------------------
 * resid (nullable): the med residual of each plane (R(0,0) = 0 and pad bits 0, which is what
 * the reference leaves/observes). weight_out (nullable, device, nplanes entries): popcount of the
 * residual (predict = 1) or of the plane itself (predict = 0). */
int bic_med_residual(bic_ctx* ctx, const uint64_t* planes, int nplanes, size_t rows, size_t cols,
                     size_t wpr, int predict, uint64_t* resid, uint64_t* weight_out);

/* ---- a7-a10: plane encoder ------------------------------------------------------------------
 * Runs per row in raster order: one sample per 1-pixel (zeros since the previous 1 or the row
 * start) and one EOL sample per row (the trailing zeros, also when 0); one coder per plane,
 * fresh state (Golomb.h:14-19 / eg.h:9). predict = 1 codes the med residual, 0 the plane.
 * out: nplanes slots of slot_words 64-bit words; plane_bits (device, nplanes): stream length
 * in bits. Domain: rows*(cols+1) < 2^31 (the reference's 32-bit coder state never wraps). */
int bic_encode_planes(bic_ctx* ctx, const uint64_t* planes, int nplanes, size_t rows, size_t cols,
                      size_t wpr, int predict, int coder, uint64_t* out, size_t slot_words,
                      uint64_t* plane_bits);
/* Both streams of the same planes in one pass (either output may be NULL, not both):
 * Golomb into out_golomb/slot_golomb/bits_golomb, EG into out_eg/slot_eg/bits_eg. Same layout
 * and semantics as two bic_encode_planes calls; rows of up to 16384 columns run as a single
 * fused kernel (plus a fixup of the words adjacent rows share). */
int bic_encode_planes2(bic_ctx* ctx, const uint64_t* planes, int nplanes, size_t rows, size_t cols,
                       size_t wpr, int predict, uint64_t* out_golomb, size_t slot_golomb,
                       uint64_t* bits_golomb, uint64_t* out_eg, size_t slot_eg, uint64_t* bits_eg);
/* a2 + a5-a10 in one call: bitplane_tool.cpp:24-30's planes of a gray image (as
 * bic_bitplanes_u8, into `planes`) and both streams of every plane (as bic_encode_planes2). Rows of
 * up to 16384 columns whose gray rows hold ceil(cols/64)*64 readable bytes (pitch >= that; any
 * alignment of gray and pitch, e.g. a P5 raster where it lies in its file's bytes) read the image
 * once: the bitplane kernel also produces the encoder's per-row counts. Otherwise the same result
 * through the two separate calls.
 * planes may be NULL (also in the _range / _packed forms below): the bitplanes are then formed in
 * registers only and not returned. With the EG stream requested into slots (out_eg, no packed EG
 * offsets) and predict = 1, the count pass writes the EG stream itself and the Golomb emission
 * reads each residual row back out of it (no further buffer). Otherwise the count pass stores each
 * plane's med residual in a buffer the context keeps (nplanes * rows * wpr words; it grows to the
 * largest call and lives until bic_ctx_destroy), from which the encoder writes the same streams
 * without recomputing med (no row above, no prediction in the emission).
 * Reads of a gray row whose address or pitch is not 16-byte aligned round out to the enclosing
 * aligned 16-byte chunks (never a chunk without one of the row's readable bytes, so never past the
 * last page of the buffer, but up to 15 bytes beyond the readable range). */
int bic_encode_gray(bic_ctx* ctx, const uint8_t* gray, size_t pitch, size_t rows, size_t cols, int nplanes,
                    uint64_t* planes, size_t wpr, int predict, uint64_t* out_golomb, size_t slot_golomb,
                    uint64_t* bits_golomb, uint64_t* out_eg, size_t slot_eg, uint64_t* bits_eg);
/* bic_encode_gray for the planes plane0 .. plane0 + nplanes - 1 of the image (plane0 + nplanes <= 8):
 * `planes`, the slots and bit counts hold those planes in order (plane0 first). The streams are
 * the ones bic_encode_gray produces for the same planes: each plane has its own coders. */
int bic_encode_gray_range(bic_ctx* ctx, const uint8_t* gray, size_t pitch, size_t rows, size_t cols, int plane0,
                          int nplanes, uint64_t* planes, size_t wpr, int predict, uint64_t* out_golomb,
                          size_t slot_golomb, uint64_t* bits_golomb, uint64_t* out_eg, size_t slot_eg,
                          uint64_t* bits_eg);
/* Packed output (what bic_pack_streams makes of the slots, without the copy): each coder's streams
 * are written word-aligned back to back from word 0 of out_golomb / out_eg (capacity nplanes *
 * slot words each, as for the slots), and off_golomb / off_eg (device, nplanes + 1 u64) receive
 * every plane's start word and the total. The multi-GPU gather sends these buffers as they are.
 * The staged encoder writes the packed positions directly; the other encoders go through slots
 * in a temporary and the pack kernel. off_* must be given for every coder that is written. */
int bic_encode_planes_packed(bic_ctx* ctx, const uint64_t* planes, int nplanes, size_t rows, size_t cols,
                             size_t wpr, int predict, uint64_t* out_golomb, size_t slot_golomb,
                             uint64_t* bits_golomb, uint64_t* off_golomb, uint64_t* out_eg, size_t slot_eg,
                             uint64_t* bits_eg, uint64_t* off_eg, uint64_t* row_index);
int bic_encode_gray_packed(bic_ctx* ctx, const uint8_t* gray, size_t pitch, size_t rows, size_t cols, int plane0,
                           int nplanes, uint64_t* planes, size_t wpr, int predict, uint64_t* out_golomb,
                           size_t slot_golomb, uint64_t* bits_golomb, uint64_t* off_golomb, uint64_t* out_eg,
                           size_t slot_eg, uint64_t* bits_eg, uint64_t* off_eg, uint64_t* row_index);

/* ---- f1: decoders on the device (GolombDecoder.cpp:15-23 read order, eg.cpp:20-37 as written) --
 * row_index (device, nplanes * rows * 2 u64; nullable in the encoders above): per row of each plane,
 * [2 (p rows + r)] = the bit offset of the row's first Golomb codeword in plane p's stream and
 * [2 (p rows + r) + 1] = the residual 1s of plane p before row r (the coder state at the row start:
 * N = ones + r, A = r cols - ones, Golomb.h:21-24). The staged encoder writes it from its scans;
 * bic_row_index computes it from planes (the encoder's prefix kernels alone; cols <= 16384, planes
 * 16-byte aligned). */
int bic_row_index(bic_ctx* ctx, const uint64_t* planes, int nplanes, size_t rows, size_t cols, size_t wpr,
                  int predict, uint64_t* index);
/* The row index of the adaptive EG coder (BIC_CODER_EG_ADAPTIVE; eg.cpp:20-37 with incBlockSize):
 * [2 (p rows + r)] = the bit offset of row r's first codeword in plane p's stream, [2 (p rows + r) + 1]
 * = the coder state there (eg.h's lutIndex, 0..31; 32 = a fresh coder, row 0: index 0, g = 1). From
 * the planes (the encoder's map / resolve / length passes, no stream written). */
int bic_egad_row_index(bic_ctx* ctx, const uint64_t* planes, int nplanes, size_t rows, size_t cols, size_t wpr,
                       int predict, uint64_t* index);
/* streams -> planes (device): slot_words > 0: plane p's stream at streams + p * slot_words;
 * slot_words == 0: packed, at streams + word_off[p], word_off[0..nplanes] as the packed encoders write
 * it (plane p owns words word_off[p] .. word_off[p + 1]). plane_bits: each stream's length; a length
 * past the plane's slot or packed words is malformed (nothing beyond them is read). Golomb needs
 * row_index (rows decode independently); EG finds the row of the plane's first 1 itself;
 * BIC_CODER_EG_ADAPTIVE needs bic_egad_row_index's index (eg.cpp:41-55's read order). predict:
 * the streams code the med residual; P(0, 0), which med discards, comes from p00 (device, one byte
 * per plane; nullable: 0). cols <= 16384. A malformed stream (bad codeword, wrong length, missing
 * end-of-row bit) is reported by bic_sync as BIC_EDATA; the planes are then undefined. */
int bic_decode_planes(bic_ctx* ctx, int coder, const uint64_t* streams, size_t slot_words, const uint64_t* word_off,
                      const uint64_t* plane_bits, const uint64_t* row_index, int nplanes, size_t rows, size_t cols,
                      size_t wpr, int predict, const uint8_t* p00, uint64_t* planes);
/* A slot size (64-bit words) that every plane of this geometry fits for EG (exact) and for
 * Golomb on any input this build has seen (2*rows*(cols+1) bits + 64 words); a larger input
 * still reports BIC_ENOSPC rather than writing out of bounds. */
size_t bic_encode_slot_words(size_t rows, size_t cols, int coder);

/* ---- GolombCoder::codeSample over an arbitrary sample array (GolombCoder.cpp:29-34) --------
 * Coder state on entry: n0 samples already coded with accumulated error a0 (n0 = a0 = 0 is a
 * fresh GolombCoder). The stream is written starting at bit `bit0` of out (0 <= bit0 < 64;
 * lets a shard start at its global bit alignment); out[0 .. cap_words) must be writable.
 * bits_out (device, 2 x u64): [0] = codeword bits (= GolombCoder::bitcount), [1] = sum of samples.
 * out = NULL with cap_words = 0 computes bits_out only (no stream): a shard learns its length
 * before its bit offset is known, then encodes once at that offset. */
int bic_golomb_encode_samples(bic_ctx* ctx, const uint32_t* samples, size_t n, uint64_t n0,
                              uint64_t a0, unsigned bit0, uint64_t* out, size_t cap_words,
                              uint64_t* bits_out);

/* ---- a11-a13: W x W tile path (compress7_test.cpp:118-275 with R = 0) ---------------------
 * Per tile in raster order: w_nonpred = weight(P), w_pred = weight(med(P)) (med inside the tile,
 * R(0,0) = 0); mode 'O' iff lentab[w_nonpred] > lentab[w_pred] else 'o'; the chosen weight is
 * Golomb-coded (golomb_nomatch.codeSample, compress7_test.cpp:270) and lentab[chosen] summed (L).
 * lentab: HOST array of W*W+1 entries, lentab[w] = (idx_t)(2 + enumL(W*W, w)) (see coding.h).
 * Requires 1 <= W <= 64, rows % W == 0, cols % W == 0 (no edge wrap).
 * Outputs (device, each nullable except stream): weights (chosen), w_nonpred, w_pred (u32 per
 * tile), modes (u8 per tile), resid (the image after the residual write-back of :266/:272),
 * stream (cap_words words) and stats (device u64[3]: Golomb bits, sum of chosen weights, L). */
int bic_patch_encode(bic_ctx* ctx, const uint64_t* plane, size_t rows, size_t cols, size_t wpr,
                     unsigned W, const uint64_t* lentab, uint32_t* weights, uint32_t* w_nonpred,
                     uint32_t* w_pred, uint8_t* modes, uint64_t* resid, uint64_t* stream,
                     size_t cap_words, uint64_t* stats);

/* ---- patch match search (compress_test.cpp:73-111) ----------------------------
 * For every W x W tile in raster order over ceil(rows/W) x ceil(cols/W) (1 <= W <= 64): the
 * position (besti, bestj) and distance bestd of the least Hamming distance between the tile and a
 * W x W window over the causal search region -- rows 0 .. i0-W at every column, then rows
 * i0-W+1 .. i0 at columns 0 .. j0-W -- first in the reference's scan order; (0, 0, W*W) when no
 * window beats W*W. Windows use get_submatrix's flat indexing (binmat.cpp:267-298: past the right
 * edge they continue in the next row). Outputs: device u32 arrays, one entry per tile. */
int bic_patch_search(bic_ctx* ctx, const uint64_t* plane, size_t rows, size_t cols, size_t wpr, unsigned W,
                     uint32_t* besti, uint32_t* bestj, uint32_t* bestd);

/* ---- compress7_test.cpp:117-275 with a search window --------------------------
 * The driver's whole tile loop with its arguments W (argv[2]), T (argv[3]) and R (argv[4]): per W x W
 * tile in raster order, the least-distance window of the causal search region of the image as the
 * residual write-back of every earlier tile left it (rows i0 .. i0-W at columns j0-W .. j0-R, then
 * rows i0-W .. i0-R at columns j0+R .. j0-R, scanned downwards, stopping at the first distance
 * <= T), the four candidate lengths (2 + enumL, plus ceil(log2(search_win_size)) for a match), the
 * mode 'X' / 'x' (match, med or not) or 'O' / 'o' (no match), the chosen weight coded by
 * golomb_match or golomb_nomatch, and the residual written back.
 *   plane: device, rows x wpr, not modified; resid: device, rows x wpr, receives the image after
 *   the loop (may equal plane). enuml: HOST array of W*W+1 doubles, enuml[w] = enumL(W*W, w)
 *   (bic_enum_codelength, or the caller's GSL values). Requires 1 <= W <= 64, rows % W == 0,
 *   cols % W == 0, R <= 32767. Per tile (device, each nullable): besti, bestj, bestd (W*W+1 when
 *   the region holds no window), weights (the coded weight), modes. stream_match / stream_nomatch:
 *   device, cap_words each, the two coders' codewords. stats: device u64[4]: matches, bits of
 *   golomb_match, bits of golomb_nomatch, sum of the chosen lengths (the driver's L before it adds
 *   the two bitcounts). A search_win_size <= 0 (whose log2 the driver converts with undefined
 *   behaviour; 2^63 on x86-64) makes a match impossible for that tile. */
int bic_match_encode(bic_ctx* ctx, const uint64_t* plane, size_t rows, size_t cols, size_t wpr, unsigned W,
                     unsigned T, unsigned R, const double* enuml, uint32_t* besti, uint32_t* bestj,
                     uint32_t* bestd, uint32_t* weights, uint8_t* modes, uint64_t* resid,
                     uint64_t* stream_match, uint64_t* stream_nomatch, size_t cap_words, uint64_t* stats);
/* compress8_test.cpp:126-272's loop (patch inversion), otherwise as bic_match_encode:
 *   - a window's distance d becomes M - d when (M - d) < d, the window then inverted (:156-161);
 *     bestd is that min(d, M - d);
 *   - before any search a tile of weight <= T or >= M - T is a perfect match (:137: no window);
 *   - bestinv starts as (P.weight() - M) < P.weight() (:136, idx_t: the tile is all 1s) and takes
 *     the inversion of each better window (:163); an inverted tile is flipped (P.flip(), :207-210)
 *     before P3 and all four weights are formed;
 *   - the match lengths are 3 + idx_len + enumL (one bit more, :250-251).
 * inverted (device, per tile, nullable): bestinv. The driver leaves a non-inverted window's `inv`
 * uninitialised (:157); here it is false. T is the caller's (the driver's default is its goodT, :73). */
int bic_match_encode_inv(bic_ctx* ctx, const uint64_t* plane, size_t rows, size_t cols, size_t wpr, unsigned W,
                         unsigned T, unsigned R, const double* enuml, uint32_t* besti, uint32_t* bestj,
                         uint32_t* bestd, uint32_t* weights, uint8_t* modes, uint8_t* inverted, uint64_t* resid,
                         uint64_t* stream_match, uint64_t* stream_nomatch, size_t cap_words, uint64_t* stats);
/* The tile loops of the other windowed-search drivers, otherwise as bic_match_encode (same
 * arguments and outputs; the driver's W, T, R; variant 7 = bic_match_encode, 8 = bic_match_encode_inv
 * without the per-tile inversion flags):
 *   4: compress4_test.cpp:89-170 -- no med: the first loop starts at column j0 - W (none at j0 = 0),
 *      idx_len = ceil(log2(li)) of the tile's raster index li (li = 0: 2^63, never a match),
 *      nomatch_len = 1 + enumL(M, P.weight()), match_len = 1 + idx_len + enumL(M, bestd) when bestd
 *      <= M, else 100000; a match codes bestd with golomb_match and writes P ^ window back, no match
 *      codes P.weight() with golomb_nomatch and leaves the tile; modes 'x' / 'o';
 *   5: compress5_test.cpp:89-170 -- 4 with a window kept when (d - worstd) > (bestd - worstd) in
 *      idx_t arithmetic, worstd = W*W/2 (:94, :109, :126);
 *   6: compress6_test.cpp:111-208 -- 4 with P3 = P when no window and match_len = 1 + idx_len +
 *      enumL(M, P3.weight()) (no 100000 guard); its D / iD matrices (:64-76) are built but unused
 *      (#if 0, :172-182).
 * Schedule: per-tile workgroups (bic_set_match_parts 1..256, or automatic). */
int bic_match_encode_var(bic_ctx* ctx, int variant, const uint64_t* plane, size_t rows, size_t cols, size_t wpr,
                         unsigned W, unsigned T, unsigned R, const double* enuml, uint32_t* besti, uint32_t* bestj,
                         uint32_t* bestd, uint32_t* weights, uint8_t* modes, uint64_t* resid, uint64_t* stream_match,
                         uint64_t* stream_nomatch, size_t cap_words, uint64_t* stats);
/* Schedule of bic_match_encode (every schedule gives the same result): 0 (default) = automatic;
 * N in 1..256 = N workgroups per tile, tiles in raster order with flags between them;
 * 0x10000 | H = one workgroup per tile row walking its tiles, plus H helper workgroups that search
 * ahead of it (W of 8, 16 or 32 and a band of (R + 2W) x (cols/32 + 2) 32-bit words <= 30 Ki; other
 * W: the row workgroup alone); other values: per-tile workgroups, count from W and R. */
int bic_set_match_parts(bic_ctx* ctx, unsigned parts);

/* log2 C(n, r) (enumerative_codelength, coding.cpp:19-22) computed without GSL, and the tile
 * length table lentab[w] = (uint64)(2 + log2 C(W*W, w)) for w = 0..W*W (host memory, W*W+1
 * entries) that bic_patch_encode takes. Host-side helpers; no device needed. */
double bic_enum_codelength(unsigned n, unsigned r);
int bic_tile_lentab(unsigned W, uint64_t* lentab);

/* ---- stream packing ---------------------------------------------------------------------------
 * Concatenates the nplanes slot streams (plane_bits from bic_encode_planes) word-aligned into
 * dst; word_off (device, nplanes+1): start word of each plane in dst, word_off[nplanes] = total. */
int bic_pack_streams(bic_ctx* ctx, const uint64_t* slots, int nplanes, size_t slot_words,
                     const uint64_t* plane_bits, uint64_t* dst, uint64_t* word_off);

/* ---- PBM (P4) rasters on the device (pbm.cpp:29-77) ------------------------------------------
 * A P4 raster is rows x ceil(cols/8) bytes, MSB = leftmost pixel, rows byte-aligned (device
 * memory, no header, any alignment: e.g. a file's bytes + data_offset). unpack: raster -> planes
 * (rows x wpr words; pad bits 0); pack: planes -> raster (pad bits of the last byte of a row 0), as
 * read_pbm_data / write_pbm do bit by bit. */
int bic_pbm_unpack(bic_ctx* ctx, const uint8_t* raster, size_t rows, size_t cols, uint64_t* plane, size_t wpr);
int bic_pbm_pack(bic_ctx* ctx, const uint64_t* plane, size_t rows, size_t cols, size_t wpr, uint8_t* raster);

/* ---- a1 / f3: PNM headers on the host, PGM samples on the device (pnm.cpp:5-89) -------------
 * bic_pnm_parse_header: the header of a P4 (pbm.cpp:4-27, " %d " swallowing whitespace after the
 * height, raster bytes included) or P2 / P5 / P6 file (pnm.cpp:20-42: '#' comment lines between
 * fields, one byte after maxval) from its first n bytes (host memory); data_offset = where the
 * raster starts. P4: maxval = 1. */
typedef struct {
  int type;            /* 4 = P4 (PBM); 2, 5 = PGM; 6 = PPM */
  size_t rows, cols;
  int maxval;
  size_t data_offset;
} bic_pnm_info;
int bic_pnm_parse_header(const uint8_t* bytes, size_t n, bic_pnm_info* info);
/* P5 samples on the device -> planes plane0 .. plane0 + nplanes - 1 (bitplane_tool.cpp:24-30):
 * raster = the first sample (device, any alignment, e.g. a file's bytes + data_offset), 1 byte per
 * sample when maxval < 256 else 2 bytes big-endian (pnm.cpp:71-74), rows of cols samples. */
int bic_pgm_bitplanes(bic_ctx* ctx, const uint8_t* raster, size_t rows, size_t cols, int maxval, int plane0,
                      int nplanes, uint64_t* planes, size_t wpr);
/* planes -> gray samples on the device (replaces plane2pgm_tool.cpp:33-52, the reassembly loop
 * `gray_img[li] |= mask` over planes 0, 1, ... with mask = 1 << plane): plane b sets bit plane0 + b
 * of each sample, bits no plane covers are 0. sample_bytes 1: one byte per sample (plane0 + nplanes
 * <= 8); 2: two bytes big-endian, the P5 raster write_p5_data writes for maxval >= 256
 * (pnm.cpp:111-124; plane0 + nplanes <= 16). gray: device, rows of `pitch` bytes (any alignment);
 * only the rows' first cols * sample_bytes bytes are written. The device round trip is then
 * gray -> bic_encode_gray_packed -> bic_decode_planes -> bic_planes_to_gray. */
int bic_planes_to_gray(bic_ctx* ctx, const uint64_t* planes, int plane0, int nplanes, size_t rows, size_t cols,
                       size_t wpr, int sample_bytes, void* gray, size_t pitch);

/* ---- f4: binary_matrix algebra over GF(2) (binmat.cpp:199-214, 516-616) ---------------------
 * Matrices are rows x cols bits in the plane layout (wpr >= ceil(cols/64) words per row, device
 * memory). bic_gf2_transpose replaces transpose_to / get_transposed: dst (cols x rows, dst_wpr >=
 * ceil(rows/64)) gets dst(j,i) = src(i,j); the ceil(rows/64) words of every dst row are written
 * (bits past rows 0). bic_gf2_mul replaces mul(A, At, B, Bt, C) (binmat.cpp:606-616) with op =
 * BIC_GF2_AB (mul_AB :516-542), BIC_GF2_ATB (mul_AtB :545-572), BIC_GF2_ABT (mul_ABt :575-594) or
 * BIC_GF2_ATBT (mul_AtBt :596-604, not implemented there: C unchanged); the reference's asserts on
 * the shapes become BIC_EINVAL. C's first ceil(c_cols/64) words per row are written; mul_ABt as
 * written sets only bits j < b_cols of a row (0 for j >= b_rows) and keeps the others. Products
 * over the whole words of their operands, as the reference's block loops (padding bits included
 * where its loops include them). Scratch for the transposed operand is stream-ordered. */
#define BIC_GF2_AB 0
#define BIC_GF2_ATB 1
#define BIC_GF2_ABT 2
#define BIC_GF2_ATBT 3
int bic_gf2_transpose(bic_ctx* ctx, const uint64_t* src, size_t rows, size_t cols, size_t wpr, uint64_t* dst,
                      size_t dst_wpr);
int bic_gf2_mul(bic_ctx* ctx, int op, const uint64_t* A, size_t a_rows, size_t a_cols, size_t a_wpr,
                const uint64_t* B, size_t b_rows, size_t b_cols, size_t b_wpr, uint64_t* C, size_t c_rows,
                size_t c_cols, size_t c_wpr);

/* ---- kernel timing ------------------------------------------------------------------------
 * When enabled, every kernel launch of this ctx is bracketed by HIP events on the launch stream.
 * bic_prof_collect syncs, writes one line per kernel name ("name launches total_ms\n") into buf
 * and clears the records. */
int bic_prof_enable(bic_ctx* ctx, int on);
int bic_prof_collect(bic_ctx* ctx, char* buf, size_t cap);
/* Restrict the bracketing to launches recorded under `name` (NULL or "" = every launch). Each
 * event pair costs the step a few microseconds of pipeline drain, so a timed region that needs
 * one kernel's duration brackets only that kernel. */
int bic_prof_only(bic_ctx* ctx, const char* name);

#ifdef __cplusplus
}
#endif
#endif
