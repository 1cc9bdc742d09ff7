// bic_decode.hip -- SURVEY.md §8 f1: decoders of this build's plane streams on the GPU, so that a
// full-size image round-trips on the device (stream -> residual -> unmed -> planes).
//
// The reference has no working decoder (GolombDecoder.cpp does not compile: BinaryFileReader.h is
// missing; eg.cpp:41-55 is under #if 0), so the read order is that of GolombDecoder.cpp:15-23
// (k-bit binary part, then the unary zeros up to the '1'; GolombCoder.cpp:29-34's state update,
// unsigned samples) and eg.cpp:20-37 as written (a '1' per zero, '0' before a 1-pixel, '1' at the
// end of a row, one extra '0' after the plane's first 1).
//
//  * Golomb: a stream is serial by construction (every codeword's k depends on all earlier
//    samples), so rows are decoded independently from a row index -- per row the bit offset of
//    its first codeword and the plane's residual 1s before it, which give the coder state at the
//    row start (N = ones + row, A = row * cols - ones: Golomb.h:21-24). The staged encoder writes
//    the index for free (bic_encode_*_packed), bic_row_index computes it from planes. One wave per
//    row: the row's stream bits are staged in LDS with coalesced loads, one lane walks the
//    codewords (the chain is serial), the wave writes the row.
//  * EG: every row is cols + 1 bits at an offset known in closed form once the row holding the
//    plane's first residual 1 is known (the first row that is not all '1's): word-parallel.
//  * unmed (pred.cpp:3-15 inverted): with D(i, j) = P(i, j) ^ P(i - 1, j), med is R(i, j) =
//    D(i, j) ^ D(i, j - 1), so D is the prefix XOR of R along the row (R(0, 0), which med never
//    writes, replaced by the caller's P(0, 0)) and P the prefix XOR of D down the columns: the row
//    kernels emit D, then a chunked column scan (chunk XORs, their exclusive scan, apply) gives P.
#include "bic_device.h"

namespace bic {

constexpr int kDecWaves = 4;
constexpr uint32_t kDecWin = 1024;  // u64 stream words staged per wave (65,536 bits)
constexpr uint32_t kDecRowWords = 256;  // cols <= 16384

struct DecArgs {
  uint32_t rows, cols, wpr, used, nplanes;
  uint64_t trail;
  const uint64_t* streams;
  uint64_t slot;              // > 0: plane p at streams + p * slot; 0: packed, plane p at word_off[p]
  const uint64_t* word_off;
  const uint64_t* plane_bits;
  const uint64_t* index;
  const uint8_t* p00;         // per plane P(0, 0) (nullable: 0)
  uint32_t* first_row;        // EG: per plane, the row holding the first residual 1 (rows: none)
  uint64_t* out;              // [nplanes][rows][wpr]
  uint32_t* flags;
  int predict;
};

__device__ __forceinline__ const uint64_t* plane_stream(const DecArgs& a, uint32_t plane) {
  return a.streams + (a.slot ? (uint64_t)plane * a.slot : a.word_off[plane]);
}

// The residual row (lane words w = 64 t + lane, t < 4) -> the row's output words: D (the prefix
// XOR along the row, P(0, 0) in place of R(0, 0) on row 0) when predicting, R itself otherwise.
__device__ __forceinline__ void store_row(const DecArgs& a, uint32_t plane, uint32_t row, uint64_t (&r)[4]) {
  const int lane = lane_id();
  uint64_t* dst = a.out + ((uint64_t)plane * a.rows + row) * a.wpr;
  uint32_t carry = 0;
#pragma unroll
  for (int t = 0; t < 4; ++t) {
    const uint32_t w = t * 64 + lane;
    if (t * 64 >= (int)a.used) break;
    uint64_t x = w < a.used ? r[t] & (w == a.used - 1 ? a.trail : ~0ull) : 0;
    if (a.predict) {
      if (row == 0 && w == 0) x = (x & ~BIC_MSB) | ((a.p00 && a.p00[plane]) ? BIC_MSB : 0ull);
      x ^= x >> 1;
      x ^= x >> 2;
      x ^= x >> 4;
      x ^= x >> 8;
      x ^= x >> 16;
      x ^= x >> 32;  // bit j = XOR of the word's bits 0..j (MSB-first)
      const uint64_t par = __ballot((x & 1ull) != 0);
      const uint32_t cin = (carry + (uint32_t)__popcll(par & ((1ull << lane) - 1ull))) & 1u;
      if (cin) x = ~x;
      carry = (carry + (uint32_t)__popcll(par)) & 1u;
      if (w < a.used) x &= (w == a.used - 1 ? a.trail : ~0ull);
    }
    if (w < a.used) dst[w] = x;
  }
  for (uint32_t w = a.used + lane; w < a.wpr; w += 64) dst[w] = 0;  // pad words
}

__global__ __launch_bounds__(64 * kDecWaves) void k_dec_golomb_rows(DecArgs a) {
  __shared__ uint64_t win[kDecWaves][kDecWin + 2];
  __shared__ uint64_t rowbuf[kDecWaves][kDecRowWords];
  const int lane = lane_id();
  const uint32_t wave = uni_u32(threadIdx.x >> 6);
  const uint64_t id = (uint64_t)blockIdx.x * kDecWaves + wave;
  if (id >= (uint64_t)a.rows * a.nplanes) return;  // whole wave
  const uint32_t plane = (uint32_t)(id / a.rows), row = (uint32_t)(id % a.rows);
  const uint64_t* st = plane_stream(a, plane);
  const uint64_t G = a.index[2 * id], O = a.index[2 * id + 1];
  const uint64_t E = row + 1 < a.rows ? a.index[2 * id + 2] : a.plane_bits[plane];
  uint64_t* W = win[wave];
  uint64_t* rb = rowbuf[wave];
  for (uint32_t w = lane; w < kDecRowWords; w += 64) rb[w] = 0;
  bool bad = E < G + 1;  // every row has at least its end-of-row codeword
  const uint64_t w0 = G >> 6, nw = bad ? 0 : ((E + 63) >> 6) - w0;
  const bool global = nw > kDecWin;  // (not reached for cols <= 16384 streams this build writes)
  if (!global) {
    for (uint64_t t = lane; t < nw; t += 64) W[t] = bswap64(st[w0 + t]);
    if (lane < 2) W[nw + lane] = 0;
  }
  __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
  __builtin_amdgcn_wave_barrier();
  __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
  if (lane == 0 && !bad) {
    auto word = [&](uint64_t i) -> uint64_t {
      if (!global) return W[i];
      return i < nw ? bswap64(st[w0 + i]) : 0ull;
    };
    auto get64 = [&](uint64_t p) -> uint64_t {
      const uint64_t i = p >> 6;
      const uint32_t sh = (uint32_t)(p & 63);
      const uint64_t hi = word(i);
      return sh ? (hi << sh) | (word(i + 1) >> (64 - sh)) : hi;
    };
    uint64_t pos = G & 63;
    const uint64_t end = pos + (E - G);
    uint32_t n = (uint32_t)(O + row), A = (uint32_t)((uint64_t)row * a.cols - O);
    uint32_t j = 0;
    for (;;) {
      const uint32_t k = golomb_k_state(n, A);
      const uint64_t x = get64(pos);
      const uint32_t low = k ? (uint32_t)(x >> (64 - k)) : 0u;
      const uint64_t y = k ? x << k : x;
      uint64_t z;
      if (y) {
        z = (uint64_t)__builtin_clzll(y);
      } else {  // a unary run past this window
        z = 64 - k;
        uint64_t p2 = pos + 64;
        for (;;) {
          if (p2 >= end) {
            bad = true;
            break;
          }
          const uint64_t x2 = get64(p2);
          if (x2) {
            z += (uint64_t)__builtin_clzll(x2);
            break;
          }
          z += 64;
          p2 += 64;
        }
        if (bad) break;
      }
      if (z > a.cols) {
        bad = true;
        break;
      }
      const uint32_t s = ((uint32_t)z << k) | low;
      pos += k + z + 1;
      if (pos > end || (uint64_t)j + s > a.cols) {
        bad = true;
        break;
      }
      ++n;
      A += s;
      if (j + s == a.cols) break;  // the end-of-row codeword
      rb[(j + s) >> 6] |= BIC_MSB >> ((j + s) & 63);
      j += s + 1;
    }
    if (pos != end) bad = true;
  }
  if (__ballot(bad)) {
    if (lane == 0) atomicOr(&a.flags[1], 2u);  // malformed stream (bic_sync: BIC_EDATA)
  }
  __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
  __builtin_amdgcn_wave_barrier();
  __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
  uint64_t r[4];
#pragma unroll
  for (int t = 0; t < 4; ++t) r[t] = rb[t * 64 + lane];
  store_row(a, plane, row, r);
}

// EG: the row holding each plane's first residual 1 = the first row whose cols + 1 bits at the
// unshifted offset row * (cols + 1) are not all '1' (rows before it are ~0 and their '1').
__global__ __launch_bounds__(256) void k_dec_eg_first(DecArgs a) {
  const uint64_t gw = (uint64_t)blockIdx.x * 4 + (threadIdx.x >> 6);
  if (gw >= (uint64_t)a.rows * a.nplanes) return;
  const uint32_t plane = (uint32_t)(gw / a.rows), row = (uint32_t)(gw % a.rows);
  const uint64_t* st = plane_stream(a, plane);
  const uint64_t off = (uint64_t)row * (a.cols + 1), bits = a.plane_bits[plane];
  const uint32_t nw = (a.cols + 1 + 63) / 64;
  bool ones = true;
  for (uint32_t t = lane_id(); t < nw; t += 64) {
    const uint64_t p = off + 64ull * t;
    const uint32_t nb = min(64u, a.cols + 1 - 64 * t);
    const uint64_t i = p >> 6;
    const uint32_t sh = (uint32_t)(p & 63);
    const uint64_t maxw = (bits + 63) >> 6;
    const uint64_t hi = i < maxw ? bswap64(st[i]) : 0ull;
    uint64_t v = hi << sh;
    if (sh) v |= (i + 1 < maxw ? bswap64(st[i + 1]) : 0ull) >> (64 - sh);
    const uint64_t m = nb == 64 ? ~0ull : ~(~0ull >> nb);
    if ((v & m) != m) ones = false;
  }
  if (__ballot(!ones) && lane_id() == 0) atomicMin(&a.first_row[plane], row);
}

__global__ __launch_bounds__(256) void k_dec_eg_rows(DecArgs a) {
  const int lane = lane_id();
  const uint64_t id = (uint64_t)blockIdx.x * 4 + (threadIdx.x >> 6);
  if (id >= (uint64_t)a.rows * a.nplanes) return;
  const uint32_t plane = (uint32_t)(id / a.rows), row = (uint32_t)(id % a.rows);
  const uint64_t* st = plane_stream(a, plane);
  const uint32_t f = a.first_row[plane];
  const uint64_t bits = a.plane_bits[plane], maxw = (bits + 63) >> 6;
  const uint64_t off = (uint64_t)row * (a.cols + 1) + (row > f ? 1 : 0);
  auto get64 = [&](uint64_t p) -> uint64_t {
    const uint64_t i = p >> 6;
    const uint32_t sh = (uint32_t)(p & 63);
    const uint64_t hi = i < maxw ? bswap64(st[i]) : 0ull;
    return sh ? (hi << sh) | ((i + 1 < maxw ? bswap64(st[i + 1]) : 0ull) >> (64 - sh)) : hi;
  };
  uint64_t x[4];
#pragma unroll
  for (int t = 0; t < 4; ++t) x[t] = (uint32_t)(t * 64 + lane) < a.used ? get64(off + 64ull * (t * 64 + lane)) : ~0ull;
  bool bad = false;
  uint64_t ins = ~0ull;  // row bit after which the stream carries the inserted '0'
  if (row == f) {  // first residual 1 of the plane: the first '0' of the row
    int fc = INT_MAX;
#pragma unroll
    for (int t = 0; t < 4; ++t) {
      const uint32_t w = t * 64 + lane;
      if (w < a.used) {
        const uint64_t r = ~x[t] & (w == a.used - 1 ? a.trail : ~0ull);
        if (r && fc == INT_MAX) fc = (int)(w * 64 + __builtin_clzll(r));
      }
    }
    fc = wave_min(fc);
    if (fc == INT_MAX) bad = true;
    else ins = (uint64_t)fc;
#pragma unroll
    for (int t = 0; t < 4; ++t) {  // words past the inserted bit come one bit later
      const uint64_t w = (uint64_t)t * 64 + lane;
      if (w >= a.used || ins == ~0ull) continue;
      const uint64_t b0 = w * 64;
      if (b0 > ins) {
        x[t] = get64(off + b0 + 1);
      } else if (b0 + 63 > ins) {  // the word holding bit ins + 1
        const uint32_t q = (uint32_t)(ins - b0);  // row bits 0..q of the word unshifted
        const uint64_t hi = ~(~0ull >> (q + 1));
        x[t] = (x[t] & hi) | (get64(off + b0 + 1) & ~hi);
      }
    }
    if (ins != ~0ull && (get64(off + ins + 1) >> 63) != 0) bad = true;  // the inserted bit is '0'
  }
  const uint64_t eol = off + a.cols + (row == f ? 1 : 0);  // the end-of-row '1'
  if ((get64(eol) >> 63) == 0) bad = true;
  if (row + 1 == a.rows && eol + 1 != bits) bad = true;
  if (__ballot(bad) && lane == 0) atomicOr(&a.flags[1], 2u);
  uint64_t r[4];
#pragma unroll
  for (int t = 0; t < 4; ++t) r[t] = ~x[t];
  store_row(a, plane, row, r);
}

// unmed, column part: P(i) = XOR of D(0..i) per word column, in chunks of kColChunk rows.
constexpr uint32_t kColChunk = 64;
__global__ __launch_bounds__(256) void k_col_chunks(const uint64_t* __restrict__ D, uint64_t* __restrict__ ctot,
                                                    uint32_t rows, uint32_t wpr, uint32_t nplanes) {
  const uint32_t nch = (rows + kColChunk - 1) / kColChunk;
  const uint64_t t = (uint64_t)blockIdx.x * 256 + threadIdx.x;
  if (t >= (uint64_t)nplanes * nch * wpr) return;
  const uint32_t w = (uint32_t)(t % wpr);
  const uint64_t pc = t / wpr;
  const uint32_t c = (uint32_t)(pc % nch), plane = (uint32_t)(pc / nch);
  const uint64_t* p = D + ((uint64_t)plane * rows + (uint64_t)c * kColChunk) * wpr + w;
  const uint32_t nr = min(kColChunk, rows - c * kColChunk);
  uint64_t acc = 0;
  for (uint32_t r = 0; r < nr; ++r) acc ^= p[(uint64_t)r * wpr];
  ctot[t] = acc;
}
__global__ __launch_bounds__(256) void k_col_scan(uint64_t* __restrict__ ctot, uint32_t rows, uint32_t wpr,
                                                  uint32_t nplanes) {
  const uint32_t nch = (rows + kColChunk - 1) / kColChunk;
  const uint64_t t = (uint64_t)blockIdx.x * 256 + threadIdx.x;
  if (t >= (uint64_t)nplanes * wpr) return;
  const uint32_t w = (uint32_t)(t % wpr), plane = (uint32_t)(t / wpr);
  uint64_t* p = ctot + (uint64_t)plane * nch * wpr + w;
  uint64_t acc = 0;
  for (uint32_t c = 0; c < nch; ++c) {  // exclusive
    const uint64_t v = p[(uint64_t)c * wpr];
    p[(uint64_t)c * wpr] = acc;
    acc ^= v;
  }
}
__global__ __launch_bounds__(256) void k_col_apply(uint64_t* __restrict__ D, const uint64_t* __restrict__ ctot,
                                                   uint32_t rows, uint32_t wpr, uint32_t nplanes) {
  const uint32_t nch = (rows + kColChunk - 1) / kColChunk;
  const uint64_t t = (uint64_t)blockIdx.x * 256 + threadIdx.x;
  if (t >= (uint64_t)nplanes * nch * wpr) return;
  const uint32_t w = (uint32_t)(t % wpr);
  const uint64_t pc = t / wpr;
  const uint32_t c = (uint32_t)(pc % nch), plane = (uint32_t)(pc / nch);
  uint64_t* p = D + ((uint64_t)plane * rows + (uint64_t)c * kColChunk) * wpr + w;
  const uint32_t nr = min(kColChunk, rows - c * kColChunk);
  uint64_t acc = ctot[t];
  for (uint32_t r = 0; r < nr; ++r) {
    acc ^= p[(uint64_t)r * wpr];
    p[(uint64_t)r * wpr] = acc;
  }
}

bool decode_supported(uint32_t cols) { return cols >= 1 && (cols + 63) / 64 <= kDecRowWords; }

size_t decode_scratch_bytes(uint32_t rows, uint32_t wpr, uint32_t nplanes) {
  const uint64_t nch = (rows + kColChunk - 1) / kColChunk;
  return (size_t)nplanes * nch * wpr * 8 + (size_t)nplanes * 4 + 256;
}

void launch_decode(hipStream_t s, int coder, const uint64_t* streams, uint64_t slot, const uint64_t* word_off,
                   const uint64_t* plane_bits, const uint64_t* index, const uint8_t* p00, uint32_t rows,
                   uint32_t cols, uint32_t wpr, uint32_t nplanes, int predict, uint64_t* out, void* scratch,
                   uint32_t* flags) {
  DecArgs a;
  a.rows = rows;
  a.cols = cols;
  a.wpr = wpr;
  a.used = (cols + 63) / 64;
  a.nplanes = nplanes;
  a.trail = cols % 64 ? ~(~0ull >> (cols % 64)) : ~0ull;
  a.streams = streams;
  a.slot = slot;
  a.word_off = word_off;
  a.plane_bits = plane_bits;
  a.index = index;
  a.p00 = p00;
  a.out = out;
  a.flags = flags;
  a.predict = predict;
  uint64_t* ctot = reinterpret_cast<uint64_t*>(scratch);
  const uint64_t nch = (rows + kColChunk - 1) / kColChunk;
  a.first_row = reinterpret_cast<uint32_t*>(ctot + (uint64_t)nplanes * nch * wpr);
  const uint64_t nrows = (uint64_t)rows * nplanes;
  const uint32_t grid = (uint32_t)((nrows + 3) / 4);
  if (coder == 0) {
    k_dec_golomb_rows<<<grid, 64 * kDecWaves, 0, s>>>(a);
  } else {
    (void)hipMemsetAsync(a.first_row, 0xff, (size_t)nplanes * 4, s);
    k_dec_eg_first<<<grid, 256, 0, s>>>(a);
    k_dec_eg_rows<<<grid, 256, 0, s>>>(a);
  }
  if (predict) {
    const uint64_t nt = (uint64_t)nplanes * nch * wpr;
    k_col_chunks<<<(uint32_t)((nt + 255) / 256), 256, 0, s>>>(out, ctot, rows, wpr, nplanes);
    k_col_scan<<<(uint32_t)(((uint64_t)nplanes * wpr + 255) / 256), 256, 0, s>>>(ctot, rows, wpr, nplanes);
    k_col_apply<<<(uint32_t)((nt + 255) / 256), 256, 0, s>>>(out, ctot, rows, wpr, nplanes);
  }
}

}  // namespace bic
