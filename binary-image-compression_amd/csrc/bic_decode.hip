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
//    the index for free (bic_encode_*_packed), bic_row_index computes it from planes. One lane per
//    row walks its codewords (the chain is serial; a wave runs 64 rows' chains side by side).
//  * EG: every row is cols + 1 bits at an offset known in closed form once the row holding the
//    plane's first residual 1 is known (the first row that is not all '1's): word-parallel.
//  * unmed (pred.cpp:3-15 inverted): with D(i, j) = P(i, j) ^ P(i - 1, j), med is R(i, j) =
//    D(i, j) ^ D(i, j - 1), so D is the prefix XOR of R along the row (R(0, 0), which med never
//    writes, replaced by the caller's P(0, 0)) and P the prefix XOR of D down the columns: the row
//    kernels emit D, then a chunked column scan (chunk XORs, their exclusive scan, apply) gives P.
#include "bic_device.h"

namespace bic {

constexpr uint32_t kDecRowWords = 256;  // cols <= 16384 (the EG row kernel's four words per lane)
constexpr uint32_t kColChunk = 64;       // unmed's column scan: rows per chunk

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
  // unmed's column chunk totals (k_col_chunks' output), formed by the Golomb row kernel itself when
  // a wave's 64 rows are one column chunk of one plane (rows % kColChunk == 0); null otherwise
  uint64_t* ctot;
  const uint64_t* egnib;  // egad_build_dec_nib's table (the adaptive EG decoder)
};

__device__ __forceinline__ const uint64_t* plane_stream(const DecArgs& a, uint32_t plane) {
  return a.streams + (a.slot ? (uint64_t)plane * a.slot : a.word_off[plane]);
}

// Words of plane p's stream the decoder may read: ceil(plane_bits / 64), capped at the plane's
// capacity (its slot, or word_off[p + 1] - word_off[p] when packed). A stated length past the
// capacity is a malformed stream (`over`): nothing past the plane's own words is ever read.
__device__ __forceinline__ uint64_t plane_words(const DecArgs& a, uint32_t plane, bool& over) {
  const uint64_t want = (a.plane_bits[plane] + 63) >> 6;
  const uint64_t lo = a.slot ? 0 : a.word_off[plane];
  const uint64_t cap = a.slot ? a.slot : (a.word_off[plane + 1] >= lo ? a.word_off[plane + 1] - lo : 0);
  over = want > cap;
  return over ? cap : want;
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

// Golomb: one LANE per row, so a wave decodes 64 rows side by side (each lane's codeword chain is
// serial, and 64 chains in lockstep keep the SIMD issuing). The lanes' stream words come through a
// per-lane ring in LDS, refilled on a uniform cadence: every kDecRefill codewords each lane issues
// the loads of its next kDecBatch words into registers and writes the batch loaded one cadence
// earlier into its ring. (Loading each word when a lane crosses into it would make the wave wait
// for the latest load into the same registers -- issued one codeword earlier by some other lane --
// at nearly every codeword: vmcnt is per wave and in order.) A lane that runs ahead of its ring
// (long codewords) reads the words it lacks directly. Each 1 of the residual row goes into an
// output word in a register; a word is stored when the next 1 lies beyond it -- as D (the row's
// prefix XOR, unmed's row part) when predicting, R otherwise.
constexpr uint32_t kDecRing = 32, kDecBatch = 8, kDecRefill = 16;
__global__ __launch_bounds__(256) void k_dec_golomb_lanes(DecArgs a) {
  __shared__ uint64_t ring[kDecRing * 256];  // [slot][thread]
  const uint64_t id = (uint64_t)blockIdx.x * 256 + threadIdx.x;
  if (id >= (uint64_t)a.rows * a.nplanes) return;
  const uint32_t plane = (uint32_t)(id / a.rows), row = (uint32_t)(id % a.rows);
  const uint64_t* st = plane_stream(a, plane);
  const uint64_t G = a.index[2 * id], O = a.index[2 * id + 1];
  const uint64_t E = row + 1 < a.rows ? a.index[2 * id + 2] : a.plane_bits[plane];
  bool over;
  const uint64_t maxw = plane_words(a, plane, over);  // words of this plane's stream
  uint64_t* dst = a.out + ((uint64_t)plane * a.rows + row) * a.wpr;
  bool bad = over || E < G + 1;  // every row has at least its end-of-row codeword
  const uint64_t len = bad ? 0 : E - G;
  auto ld = [&](uint64_t i) -> uint64_t { return i < maxw ? bswap64(st[i]) : 0ull; };
  uint64_t* my = ring + threadIdx.x;
  auto slot = [&](uint64_t i) -> uint64_t& { return my[(uint32_t)(i % kDecRing) * 256]; };
  // ring: words [wl - kDecRing, wr) readable from LDS; [wr, wl) in flight in pend[]
  uint64_t pend[kDecBatch];
  uint64_t wl = (G >> 6) & ~(uint64_t)(kDecBatch - 1), wr = wl;
  auto issue = [&]() {
#pragma unroll
    for (uint32_t q = 0; q < kDecBatch; ++q) pend[q] = wl + q < maxw ? st[wl + q] : 0ull;
    wl += kDecBatch;
  };
  auto commit = [&]() {  // the batch in pend[] -> its ring slots
#pragma unroll
    for (uint32_t q = 0; q < kDecBatch; ++q) slot(wr + q) = bswap64(pend[q]);
    wr += kDecBatch;
  };
  issue();
  commit();
  issue();
  uint64_t wi = G >> 6;
  auto get = [&](uint64_t i) -> uint64_t { return i < wr ? slot(i) : ld(i); };
  uint64_t w0 = get(wi), w1 = get(wi + 1);
  uint32_t b = (uint32_t)(G & 63);  // bit position in w0
  uint64_t used_bits = 0;           // stream bits consumed by the row so far
  auto peek = [&]() -> uint64_t { return b ? (w0 << b) | (w1 >> (64 - b)) : w0; };
  auto advance = [&](uint32_t nb) {  // nb <= 64
    used_bits += nb;
    b += nb;
    if (b >= 64) {
      b -= 64;
      w0 = w1;
      ++wi;
      w1 = get(wi + 1);
    }
  };
  auto refill = [&]() {  // every lane still decoding, at the same codeword count
    if (wl > wr) commit();
    if (wl + kDecBatch - wi <= kDecRing) issue();  // (the slots it will fill hold words < wi)
  };
  uint32_t it = 0;
  const bool pred = a.predict != 0;
  const uint64_t p00 = (pred && row == 0 && a.p00 && a.p00[plane]) ? BIC_MSB : 0ull;
  uint32_t ow = 0, carry = 0;  // output word being filled, the prefix-XOR carry into it
  uint64_t acc = 0;
  auto flush = [&]() {  // store word ow (then ow + 1 is the open one)
    uint64_t x = acc;
    if (pred) {
      if (row == 0 && ow == 0) x = (x & ~BIC_MSB) | p00;  // R(0, 0) -> P(0, 0)
      x ^= x >> 1;
      x ^= x >> 2;
      x ^= x >> 4;
      x ^= x >> 8;
      x ^= x >> 16;
      x ^= x >> 32;  // bit j (MSB-first) = XOR of the word's bits 0..j
      const uint32_t par = (uint32_t)(x & 1ull);
      if (carry) x = ~x;
      carry ^= par;
    }
    if (ow == a.used - 1) x &= a.trail;
    dst[ow] = x;
    ++ow;
    acc = 0;
  };
  uint32_t n = (uint32_t)(O + row), A = (uint32_t)((uint64_t)row * a.cols - O);
  uint32_t j = 0;  // the row's next column
  while (!bad) {
    if ((++it & (kDecRefill - 1)) == 0) refill();
    const uint32_t k = golomb_k_state(n, A);
    uint32_t low = 0;
    if (k) {
      low = (uint32_t)(peek() >> (64 - k));
      advance(k);
    }
    uint64_t z = 0;  // unary zeros up to the '1'
    for (;;) {
      const uint64_t y = peek();
      if (y) {
        const uint32_t c = (uint32_t)__builtin_clzll(y);
        z += c;
        advance(c + 1);
        break;
      }
      z += 64;
      advance(64);
      if (used_bits > len || z > a.cols) break;
    }
    if (used_bits > len || z > a.cols) {
      bad = true;
      break;
    }
    const uint32_t s = ((uint32_t)z << k) | low;
    if ((uint64_t)j + s > a.cols) {
      bad = true;
      break;
    }
    ++n;
    A += s;
    if (j + s == a.cols) break;  // the end-of-row codeword
    const uint32_t c = j + s;    // the 1 of this codeword's sample
    while ((c >> 6) > ow) flush();
    acc |= BIC_MSB >> (c & 63);
    j = c + 1;
  }
  if (used_bits != len) bad = true;
  while (ow < a.used) flush();
  for (uint32_t w = a.used; w < a.wpr; ++w) dst[w] = 0;  // pad words
  if (bad) atomicOr(&a.flags[1], 2u);                     // malformed stream (bic_sync: BIC_EDATA)
}

// EG adaptive (BIC_CODER_EG_ADAPTIVE: eg.cpp:20-37 with incBlockSize enabled) in the read order of the
// #if 0 decoder (eg.cpp:41-55): per run '1' = a full block (len += blockSize, then incBlockSize), until
// a '0' and the g-bit remainder (then decBlockSize) -- or until a block passes the columns left,
// which is the end-of-row '1' (no incBlockSize after it, as the encoder writes it). The lutIndex
// saturates at 31 as in the encoder. The coder state is serial across the plane, so rows are decoded
// independently from the egad row index (bic_egad_row_index: per row its first bit and the state
// there; 32 = a fresh coder: index 0 but g = 1, eg.h:9). One lane per row; the leading 1s of the
// next 64 stream bits are counted at once (the blocks), the remainder read as one field.
__host__ __device__ __forceinline__ uint32_t egad_j(uint32_t i) { return i < 16 ? i >> 2 : (i < 24 ? (i >> 1) - 4 : i - 16); }
// Nibble steps: while the index is <= 15 (blocks of <= 8 columns, remainders of <= 3 bits) and the row's
// end is more than 40 columns away, 4 stream bits at a time through a table over the decoder's state
// (i, phase: in a run's '1's (U) or its remainder (R) after k of its g bits, value v) -- 17 U and 45 R
// states: the columns they advance (<= 36), the 1s they place there and the state after. Other bits
// (higher indices, the row's last columns and its end-of-row '1') one at a time, checked.
constexpr uint32_t kFreshD = 32;
__host__ __device__ __forceinline__ uint32_t egad_dsidx(uint32_t i, uint32_t ph, uint32_t k, uint32_t v) {
  if (!ph) return i == kFreshD ? 16u : i;
  if (i == kFreshD) return 17u;
  if (i < 8) return 18u + (i - 4);
  if (i < 12) return 22u + (i - 8) * 3 + (k ? 1 + v : 0u);
  return 34u + (i - 12) * 7 + (k == 0 ? 0u : (k == 1 ? 1 + v : 3 + v));
}
// entry: the 1s (bit 39 - p: column col + p) | P << 40 | i << 46 (5 bits, 16: fresh) | ph << 51 | k << 52 |
// v << 54 | the state's own table row << 57; bit 63: escape
void egad_build_dec_nib(uint64_t* T) {
  for (uint32_t n = 0; n < 62 * 16; ++n) T[n] = 1ull << 63;
  auto fill = [&](uint32_t i0, uint32_t ph0, uint32_t k0, uint32_t v0) {
    for (uint32_t nib = 0; nib < 16; ++nib) {
      uint32_t i = i0, ph = ph0, k = k0, v = v0, P = 0;
      uint64_t m = 0;
      bool esc = false;
      for (int b = 3; b >= 0 && !esc; --b) {
        const uint32_t bit = (nib >> b) & 1u;
        const uint32_t g = i == kFreshD ? 1u : egad_j(i);
        if (!ph) {
          if (bit) {  // a full block of zeros, incBlockSize
            P += i == kFreshD ? 1u : 1u << g;
            i = i == kFreshD ? 1u : i + 1;
          } else if (g == 0) {  // '0' with no remainder: the run's 1
            m |= 1ull << (39 - P);
            ++P;
            i = (i == kFreshD || i == 0) ? 0u : i - 1;
          } else {
            ph = 1;
            k = 0;
            v = 0;
          }
        } else {
          v = 2 * v + bit;
          if (++k == g) {  // the remainder read: its zeros, then the run's 1
            P += v;
            m |= 1ull << (39 - P);
            ++P;
            i = (i == kFreshD || i == 0) ? 0u : i - 1;
            ph = 0;
            k = v = 0;
          }
        }
        esc = i != kFreshD && i >= 16;
      }
      if (!esc)
        T[egad_dsidx(i0, ph0, k0, v0) * 16 + nib] =
            m | ((uint64_t)P << 40) | ((uint64_t)(i == kFreshD ? 16u : i) << 46) | ((uint64_t)ph << 51) |
            ((uint64_t)k << 52) | ((uint64_t)v << 54) | ((uint64_t)egad_dsidx(i, ph, k, v) << 57);
    }
  };
  for (uint32_t i = 0; i < 16; ++i) fill(i, 0, 0, 0);
  fill(kFreshD, 0, 0, 0);
  fill(kFreshD, 1, 0, 0);
  for (uint32_t i = 4; i < 16; ++i) {
    const uint32_t g = egad_j(i);
    for (uint32_t k = 0; k < g; ++k)
      for (uint32_t v = 0; v < (1u << k); ++v) fill(i, 1, k, v);
  }
}
__global__ __launch_bounds__(256) void k_dec_egad(DecArgs a) {
  __shared__ uint64_t sT[62 * 16];
  for (uint32_t q = threadIdx.x; q < 62 * 16; q += 256) sT[q] = a.egnib[q];
  __syncthreads();
  const uint64_t id = (uint64_t)blockIdx.x * 256 + threadIdx.x;
  if (id >= (uint64_t)a.rows * a.nplanes) return;
  const uint32_t plane = (uint32_t)(id / a.rows), row = (uint32_t)(id % a.rows);
  const uint64_t* st = plane_stream(a, plane);
  const uint64_t G = a.index[2 * id], S0 = a.index[2 * id + 1];
  const uint64_t E = row + 1 < a.rows ? a.index[2 * id + 2] : a.plane_bits[plane];
  bool over;
  const uint64_t maxw = plane_words(a, plane, over);
  uint64_t* dst = a.out + ((uint64_t)plane * a.rows + row) * a.wpr;
  bool bad = over || E < G + 1 || S0 > 32;  // every row has at least its end-of-row '1'
  const uint64_t len = bad ? 0 : E - G;
  auto ld = [&](uint64_t i) -> uint64_t { return i < maxw ? bswap64(st[i]) : 0ull; };
  // the stream through a window of 4 + 4 words: the next four are loaded when the current four are
  // entered, some hundred runs before they are needed (one lane per row has no other latency cover;
  // a load per word read as it is reached: 12.9 ms per C3 image)
  uint64_t base = G >> 6, cur[4], nxt[4];
  uint32_t ci = 0;  // w0 = cur[ci]
  auto load4 = [&](uint64_t (&d)[4], uint64_t at) {
#pragma unroll
    for (int q = 0; q < 4; ++q) d[q] = bad ? 0ull : ld(at + q);
  };
  load4(cur, base);
  load4(nxt, base + 4);
  uint64_t w0 = cur[0], w1 = cur[1];
  uint32_t b = (uint32_t)(G & 63);
  uint64_t used_bits = 0;
  auto peek = [&]() -> uint64_t { return b ? (w0 << b) | (w1 >> (64 - b)) : w0; };
  auto advance = [&](uint32_t nb) {  // nb <= 64
    used_bits += nb;
    b += nb;
    if (b >= 64) {
      b -= 64;
      w0 = w1;
      if (++ci == 4) {
        ci = 0;
        base += 4;
#pragma unroll
        for (int q = 0; q < 4; ++q) cur[q] = nxt[q];
        load4(nxt, base + 4);
      }
      w1 = ci == 0 ? cur[1] : (ci == 1 ? cur[2] : (ci == 2 ? cur[3] : nxt[0]));
    }
  };
  const bool pred = a.predict != 0;
  const uint64_t p00 = (pred && row == 0 && a.p00 && a.p00[plane]) ? BIC_MSB : 0ull;
  uint32_t ow = 0, carry = 0;
  uint64_t acc = 0;
  auto flush = [&]() {  // store word ow (as D when predicting: the row's prefix XOR)
    uint64_t x = acc;
    if (pred) {
      if (row == 0 && ow == 0) x = (x & ~BIC_MSB) | p00;
      x ^= x >> 1;
      x ^= x >> 2;
      x ^= x >> 4;
      x ^= x >> 8;
      x ^= x >> 16;
      x ^= x >> 32;
      const uint32_t par = (uint32_t)(x & 1ull);
      if (carry) x = ~x;
      carry ^= par;
    }
    if (ow == a.used - 1) x &= a.trail;
    dst[ow] = x;
    ++ow;
    acc = 0;
  };
  // the coder state: index i (kFreshD: a fresh coder, index 0 with g = 1, eg.h:9), phase ph (0: a
  // run's '1's, 1: its remainder after k of its g bits, value v); col: the row's next column
  uint32_t i = S0 == 32 ? kFreshD : (uint32_t)S0, ph = 0, k = 0, v = 0, col = 0;
  uint32_t sid = (i < 16 || i == kFreshD) ? egad_dsidx(i, 0, 0, 0) : 64u;  // the state's table row (64: none)
  auto one = [&](uint32_t c) {  // the run's 1 at column c
    while ((c >> 6) > ow) flush();
    acc |= BIC_MSB >> (c & 63);
  };
  while (!bad) {
    if (used_bits > len) {
      bad = true;
      break;
    }
    while (sid < 64 && col + 40 <= a.cols && used_bits + 4 <= len) {  // table steps while they apply
      const uint64_t e = sT[sid * 16 + (uint32_t)(peek() >> 60)];
      if (e >> 63) break;  // (escape: this nibble bit by bit)
      {
        advance(4);
        const uint32_t P = (uint32_t)(e >> 40) & 63u;
        const uint64_t m = (e & 0xFFFFFFFFFFull) << 24;  // MSB-first: bit 63 is column col
        if (m) {
          while ((col >> 6) > ow) flush();
          const uint32_t o = col & 63u;
          acc |= m >> o;
          if (o + P > 64) {
            const uint64_t spill = m << (64 - o);
            flush();
            acc |= spill;
          }
        }
        col += P;
        i = (uint32_t)(e >> 46) & 31u;
        i = i == 16 ? kFreshD : i;
        ph = (uint32_t)(e >> 51) & 1u;
        k = (uint32_t)(e >> 52) & 3u;
        v = (uint32_t)(e >> 54) & 7u;
        sid = (uint32_t)(e >> 57) & 63u;
      }
    }
    if (used_bits > len) {
      bad = true;
      break;
    }
    const uint32_t bit = (uint32_t)(peek() >> 63);
    advance(1);
    const uint32_t g = i == kFreshD ? 1u : egad_j(i);
    if (!ph) {
      if (bit) {  // a full block -- or, passing the row's end, its end-of-row '1'
        const uint32_t z = i == kFreshD ? 1u : 1u << g;
        if ((uint64_t)col + z > a.cols) break;
        col += z;
        i = i == kFreshD ? 1u : (i < 31 ? i + 1 : 31u);
      } else if (g == 0) {
        if (col >= a.cols) {
          bad = true;
          break;
        }
        one(col++);
        i = i == 0 ? 0u : i - 1;
      } else {
        ph = 1;
        k = 0;
        v = 0;
      }
    } else {
      v = 2 * v + bit;
      if (++k == g) {
        col += v;
        if (col >= a.cols) {
          bad = true;
          break;
        }
        one(col++);
        i = (i == kFreshD || i == 0) ? 0u : i - 1;
        ph = 0;
      }
    }
    sid = (i < 16 || i == kFreshD) ? egad_dsidx(i, ph, k, v) : 64u;
  }
  if (used_bits != len) bad = true;
  while (ow < a.used) flush();
  for (uint32_t w = a.used; w < a.wpr; ++w) dst[w] = 0;  // pad words
  if (bad) atomicOr(&a.flags[1], 2u);                     // malformed stream (bic_sync: BIC_EDATA)
}

// Golomb, byte machine: still one lane per row, but every lane consumes its stream 8 bits per
// step from one table lookup, instead of a codeword's serial chain per codeword.
// The state between steps: the phase (S: at a codeword start, U0 / U1: inside the unary part of a
// k = 0 / k = 1 codeword, and LOW / UK: the binary / unary part of a k >= 2 codeword), the column
// j of the next residual bit, n (samples so far, Golomb.h's N) and x = A - n (A counted bit by bit:
// a unary '0' adds 2^k zero columns at once, a k = 1 low bit its value). While 0 < n and x + 16 <= n
// every codeword start in the next 8 bits has k = golomb_k(n, A) = [x > 0] (A <= 2 n), and x moves
// by at most +16 over them; the decisions inside 8 bits are the same for every x <= -5 and for every
// x >= 5 (checked exhaustively), so one table entry per (phase, x clamped to [-5, 5], byte) gives
// the step: the residual columns it produces (<= 16), dx and the phase after. Other steps (n = 0,
// k >= 2, the row's last columns) go bit by bit through the general machine.
// The stream is read in blocks of 4 x 64 bits per lane. When every lane of the wave can take table
// steps for the whole block (n > 0, x + 512 <= n), the wave runs the block's 32 steps without
// per-step tests: four steps' columns (<= 64) are gathered in one register and placed once, and
// the (at most one) word each placement finishes is kept for the next block, whose start stores
// them -- right after the block's loads were waited for at the previous block's end, so no wait
// ever covers a young store. A lane stops before the byte holding its row's last stream bit and
// reads that byte through the general machine, which ends the row exactly at its stream's end.
// Other blocks (a plane's first row, k >= 2) step with per-step tests and store words as they
// finish.
constexpr int kNibXLo = -5, kNibXN = 11;
constexpr uint32_t kStepBits = 8, kStepVals = 1u << kStepBits;
constexpr uint32_t kNibTab = 3 * kNibXN * kStepVals;
enum : uint32_t { kPhS = 0, kPhU0 = 1, kPhU1 = 2, kPhLow = 3, kPhUK = 4 };
constexpr int kBlkSteps = 32;  // 4 chunks of 8 steps

// (phase, x, byte) at index (phase * 11 + x + 5) * 256 + byte -> len | (dx + 8) << 6 | (phase' * 11) << 11 |
// columns << 16 (the step's residual bits, first in bit 31)
__device__ uint32_t nib_entry(uint32_t idx) {
  const uint32_t nib = idx % kStepVals, xi = (idx / kStepVals) % kNibXN;
  uint32_t ph = idx / kStepVals / kNibXN;
  int x = (int)xi + kNibXLo, dx = 0;
  uint32_t ob = 0, len = 0;
  for (int i = 0; i < (int)kStepBits; ++i) {
    const uint32_t bit = (nib >> (kStepBits - 1 - i)) & 1u;
    if (ph == kPhS) {
      if (x > 0) {  // k = 1: the low bit (its value in zero columns)
        len += bit;
        x += (int)bit;
        dx += (int)bit;
        ph = kPhU1;
        continue;
      }
      ph = kPhU0;
    }
    if (bit == 0) {
      const int z = ph == kPhU1 ? 2 : 1;
      len += (uint32_t)z;
      x += z;
      dx += z;
    } else {
      ob |= 0x8000u >> len;
      ++len;
      --x;
      --dx;
      ph = kPhS;
    }
  }
  return len | (uint32_t)(dx + 8) << 6 | (ph * kNibXN) << 11 | ob << 16;
}

#ifndef BIC_DEC_BLOCKS
#define BIC_DEC_BLOCKS 1
#endif
constexpr bool kDecBlocks = BIC_DEC_BLOCKS != 0;  // the all-lanes block path (else per-step tests always)
__global__ __launch_bounds__(256) void k_dec_golomb_nib(DecArgs a) {
  __shared__ uint32_t tab[kNibTab];
  __shared__ uint64_t csum[4][kDecRowWords];  // per wave: the XOR of its rows' D words (a.ctot)
  for (uint32_t i = threadIdx.x; i < kNibTab; i += blockDim.x) tab[i] = nib_entry(i);
  if (a.ctot)
    for (uint32_t i = threadIdx.x; i < 4 * kDecRowWords; i += blockDim.x) (&csum[0][0])[i] = 0;
  __syncthreads();
  uint64_t* cs = csum[wave_id()];
  const uint64_t id = (uint64_t)blockIdx.x * 256 + threadIdx.x;
  const bool inrow = id < (uint64_t)a.rows * a.nplanes;
  const uint32_t plane = inrow ? (uint32_t)(id / a.rows) : 0, row = inrow ? (uint32_t)(id % a.rows) : 0;
  const uint64_t* st = plane_stream(a, plane);
  bool over = false;
  const uint64_t maxw = inrow ? plane_words(a, plane, over) : 0;
  const uint64_t G = inrow ? a.index[2 * id] : 0, O = inrow ? a.index[2 * id + 1] : 0;
  const uint64_t E = !inrow ? 0 : row + 1 < a.rows ? a.index[2 * id + 2] : a.plane_bits[plane];
  uint64_t* dst = a.out + ((uint64_t)plane * a.rows + row) * a.wpr;
  bool bad = inrow && (over || E < G + 1);  // every row has at least its end-of-row codeword
  const uint64_t len = bad ? 0 : E - G;
  bool live = inrow && !bad;  // still decoding (false once the row ended or the stream is malformed)
  const uint32_t cols = a.cols;
  const bool pred = a.predict != 0;
  const uint64_t p00 = (pred && row == 0 && a.p00 && a.p00[plane]) ? BIC_MSB : 0ull;
  // stream: word q holds stream bits [64 q, 64 q + 64) of the plane; the row's chunk c is the 64
  // bits from G + 64 c. Raw words (byte-swapped and cut at the plane's end only when used); lanes
  // without a stream read word 0 of the buffer.
  const uint64_t q0 = G >> 6;
  const uint32_t off = (uint32_t)(G & 63);
  const uint64_t* sp = live && maxw ? st : a.streams;
  const uint64_t lastw = live && maxw ? maxw - 1 : 0;
  auto ld = [&](uint64_t i) -> uint64_t { return sp[min(i, lastw)]; };
  auto word = [&](uint64_t raw, uint64_t i) -> uint64_t { return i < maxw && live ? bswap64(raw) : 0ull; };
  // machine state
  uint32_t ph = kPhS, j = 0, n = (uint32_t)(O + row), kk = 0, r = 0, low = 0, z = 0;
  int x = (int)((uint64_t)row * cols - O) - (int)n;
  uint64_t acc = 0;            // output word j >> 6 being filled (residual bits, MSB-first)
  uint32_t ow = 0, carry = 0;  // its index; the prefix-XOR parity of the words before it
  uint32_t bitpos = 0;         // stream bits of the row consumed
  bool done = false;           // the end-of-row codeword was read and the row's words stored
  auto store_word = [&](uint64_t v, uint32_t w) {  // word w of the row, in order: as D when predicting
    if (pred) {
      if (row == 0 && w == 0) v = (v & ~BIC_MSB) | p00;  // R(0, 0) -> P(0, 0)
      v ^= v >> 1;
      v ^= v >> 2;
      v ^= v >> 4;
      v ^= v >> 8;
      v ^= v >> 16;
      v ^= v >> 32;  // bit j (MSB-first) = XOR of the word's bits 0..j
      const uint32_t par = (uint32_t)(v & 1ull);
      if (carry) v = ~v;
      carry ^= par;
    }
    if (w >= a.used) return;  // (a malformed stream's columns past the row)
    if (w == a.used - 1) v &= a.trail;
    dst[w] = v;
    if (a.ctot) __hip_atomic_fetch_xor(cs + w, v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WAVEFRONT);
  };
  auto finish_word = [&]() {  // word ow complete: stored now (the stepped path)
    if (ow < a.used) store_word(acc, ow);
    ++ow;
    acc = 0;
  };
  auto fail = [&]() {
    bad = true;
    live = false;
  };
  // the general machine, one stream bit
  auto slow_bit = [&](uint32_t bit) {
    ++bitpos;
    if (ph == kPhS) {
      const uint32_t k = golomb_k_state(n, (uint32_t)(x + (int)n));
      if (k == 1) {
        j += bit;
        x += (int)bit;
        ph = kPhU1;
        return;
      }
      if (k == 0) {
        ph = kPhU0;
      } else {
        kk = k;
        r = k;
        low = 0;
        ph = kPhLow;
      }
    }
    if (ph == kPhLow) {
      low = (low << 1) | bit;
      if (--r == 0) {
        ph = kPhUK;
        z = 0;
      }
      return;
    }
    if (bit == 0) {
      if (ph == kPhUK) {
        if (++z > cols) fail();
      } else {
        const uint32_t dz = ph == kPhU1 ? 2u : 1u;
        j += dz;
        x += (int)dz;
      }
      if (j > cols) fail();
      return;
    }
    // the codeword's '1': its residual 1 (or the end of the row) at column c
    uint32_t c = j;
    if (ph == kPhUK) {
      const uint64_t s = ((uint64_t)z << kk) | low;
      if (j + s > cols) {
        fail();
        return;
      }
      c = j + (uint32_t)s;
      x += (int)s;
    }
    ph = kPhS;
    ++n;
    --x;
    if (c == cols) {  // the end-of-row codeword: the row's last words
      live = false;
      if (bitpos != len) {
        bad = true;
        return;
      }
      while (ow < a.used) finish_word();
      done = true;
      return;
    }
    while ((c >> 6) > ow) finish_word();
    acc |= BIC_MSB >> (c & 63);
    j = c + 1;
  };
  auto tab_at = [&](uint32_t phk, int xv, uint32_t byte) -> uint32_t {  // phk = phase * 11
    const uint32_t xc = (uint32_t)(min(max(xv, kNibXLo), kNibXLo + kNibXN - 1) - kNibXLo);
    return tab[(phk + xc) * kStepVals + byte];
  };
  // one stepped-path step: a table step when this lane can take one, else 8 general steps
  auto careful_step = [&](uint32_t byte) {
    if (ph <= kPhU1 && n > 0 && x + 2 * (int)kStepBits <= (int)n && j + 2 * kStepBits <= cols) {
      const uint32_t e = tab_at(ph * kNibXN, x, byte);
      const uint32_t l = e & 31u;
      const uint64_t obw = (uint64_t)(e & 0xffff0000u) << 32;
      const uint32_t pos = j & 63;
      acc |= obw >> pos;
      if (pos + l >= 64) {
        const uint64_t spill = pos ? obw << (64 - pos) : 0ull;
        finish_word();
        acc = spill;
      }
      j += l;
      n += (uint32_t)__popc(e >> 16);
      x += (int)((e >> 6) & 31u) - 8;
      ph = (((e >> 11) & 31u) * 3) >> 5;  // (phase * 11) -> phase
      bitpos += kStepBits;
    } else {
#pragma unroll 1
      for (int b = kStepBits - 1; b >= 0; --b)
        if (live) slow_bit((byte >> b) & 1u);
    }
  };
  // stream ring: A0..A4 = words q0 + 4 b .. q0 + 4 b + 4 of block b; B0..B3 the next block's words
  // 5..8, loaded at the block start and moved into A at its end
  uint64_t A0 = ld(q0), A1 = ld(q0 + 1), A2 = ld(q0 + 2), A3 = ld(q0 + 3), A4 = ld(q0 + 4);
  uint64_t D0 = 0, D1 = 0, D2 = 0, D3 = 0, D4 = 0, D5 = 0, D6 = 0, D7 = 0;  // words a fast block finished
  uint32_t dflags = 0, dbase = 0;  // which of D0..D7 hold a word; the first one's index
  // the byte holding the row's last stream bit (its end-of-row '1'): the block steps stop before it
  // and the general machine reads it, so the row ends exactly where its stream does
  const uint32_t last_step = len ? (uint32_t)((len - 1) / kStepBits) : 0u;
  for (uint64_t blk = 0;; ++blk) {
    if (!__ballot(live)) break;
    if (live && dflags) {  // the previous block's finished words, in order
      uint32_t w = dbase;
      if (dflags & 1u) store_word(D0, w++);
      if (dflags & 2u) store_word(D1, w++);
      if (dflags & 4u) store_word(D2, w++);
      if (dflags & 8u) store_word(D3, w++);
      if (dflags & 16u) store_word(D4, w++);
      if (dflags & 32u) store_word(D5, w++);
      if (dflags & 64u) store_word(D6, w++);
      if (dflags & 128u) store_word(D7, w++);
    }
    dflags = 0;
    const uint64_t cb = q0 + 4 * blk;
    const uint64_t B0 = ld(cb + 5), B1 = ld(cb + 6), B2 = ld(cb + 7), B3 = ld(cb + 8);
    const uint64_t x0 = word(A0, cb), x1 = word(A1, cb + 1), x2 = word(A2, cb + 2), x3 = word(A3, cb + 3),
                   x4 = word(A4, cb + 4);
    auto chunk_bits = [&](uint64_t lo, uint64_t hi) -> uint64_t { return off ? (lo << off) | (hi >> (64 - off)) : lo; };
    const uint64_t v0 = chunk_bits(x0, x1), v1 = chunk_bits(x1, x2), v2 = chunk_bits(x2, x3), v3 = chunk_bits(x3, x4);
    // the block's steps before the row's last byte (kBlkSteps: none of it in this block)
    const uint64_t s0 = (uint64_t)kBlkSteps * blk;
    const uint32_t stop = !live ? (uint32_t)kBlkSteps
                                : last_step < s0 ? 0u : (uint32_t)min((uint64_t)kBlkSteps, (uint64_t)last_step - s0);
    const bool bfast = !live || (ph <= kPhU1 && n > 0 && x + 16 * kBlkSteps <= (int)n);
    if (kDecBlocks && __all(bfast)) {
      // every lane: 8 groups of 4 table steps; each group's columns (<= 64) gathered in Q, then
      // placed after acc (finishing at most one word: kept in D<g>). When a lane's last byte lies
      // in this block (some lane's stop < 32: a wave-uniform choice), its steps from there on are
      // void.
      const bool ends = !__all(stop == (uint32_t)kBlkSteps);
      uint32_t phk = ph * kNibXN;
      dbase = ow;
      auto group = [&](uint32_t half, uint64_t& Dg, uint32_t g) {
        uint64_t Q = 0;
        uint32_t m = 0;
#pragma unroll
        for (int k = 0; k < 4; ++k) {
          const uint32_t e = tab_at(phk, x, (half >> (24 - 8 * k)) & 255u);
          const bool act = !ends || 4 * g + k < stop;
          const uint64_t q = ((uint64_t)(e & 0xffff0000u) << 32) >> m;
          Q |= act ? q : 0ull;
          m += act ? e & 31u : 0u;
          x += act ? (int)((e >> 6) & 31u) - 8 : 0;
          phk = act ? (e >> 11) & 31u : phk;
        }
        const uint32_t pos = j & 63;
        const uint64_t filled = acc | (Q >> pos);
        const bool cross = pos + m >= 64;
        Dg = filled;
        dflags |= cross ? 1u << g : 0u;
        acc = cross ? (pos ? Q << (64 - pos) : 0ull) : filled;
        ow += cross ? 1u : 0u;
        j += m;
        n += (uint32_t)__popcll(Q);
      };
      group((uint32_t)(v0 >> 32), D0, 0);
      group((uint32_t)v0, D1, 1);
      group((uint32_t)(v1 >> 32), D2, 2);
      group((uint32_t)v1, D3, 3);
      group((uint32_t)(v2 >> 32), D4, 4);
      group((uint32_t)v2, D5, 5);
      group((uint32_t)(v3 >> 32), D6, 6);
      group((uint32_t)v3, D7, 7);
      ph = (phk * 3) >> 5;
      bitpos += kStepBits * stop;
      if (ends && live && stop < (uint32_t)kBlkSteps) {
        // the lanes whose row ends here: their words so far, then the last byte bit by bit
        uint32_t w = dbase;
        if (dflags & 1u) store_word(D0, w++);
        if (dflags & 2u) store_word(D1, w++);
        if (dflags & 4u) store_word(D2, w++);
        if (dflags & 8u) store_word(D3, w++);
        if (dflags & 16u) store_word(D4, w++);
        if (dflags & 32u) store_word(D5, w++);
        if (dflags & 64u) store_word(D6, w++);
        if (dflags & 128u) store_word(D7, w++);
        dflags = 0;
        const uint64_t vq = stop < 8 ? v0 : stop < 16 ? v1 : stop < 24 ? v2 : v3;
        const uint32_t byte = (uint32_t)(vq >> (56 - 8 * (stop & 7))) & 255u;
#pragma unroll 1
        for (int b = kStepBits - 1; b >= 0; --b)
          if (live) slow_bit((byte >> b) & 1u);
        if (live) fail();  // no end-of-row codeword where the stream ends
      }
      if (live && bitpos > len) fail();
    } else {
      const uint64_t vs[4] = {v0, v1, v2, v3};
#pragma unroll 1
      for (int i = 0; i < kBlkSteps; ++i)
        if (live) careful_step((uint32_t)(vs[i >> 3] >> (56 - 8 * (i & 7))) & 255u);
      if (live && bitpos > len) fail();
    }
    A0 = A4;
    A1 = B0;
    A2 = B1;
    A3 = B2;
    A4 = B3;
  }
  if (inrow) {
    if (!done)  // a malformed stream (flagged): the row's words are zeros
      for (uint32_t w = 0; w < a.used; ++w) dst[w] = 0;
    for (uint32_t w = a.used; w < a.wpr; ++w) dst[w] = 0;  // pad words
    if (bad) atomicOr(&a.flags[1], 2u);                     // malformed stream (bic_sync: BIC_EDATA)
  }
  if (a.ctot && __ballot(inrow)) {  // the wave's chunk totals (its rows are chunk row / kColChunk)
    __builtin_amdgcn_fence(__ATOMIC_ACQ_REL, "wavefront");
    __builtin_amdgcn_wave_barrier();
    const uint64_t wid = ((uint64_t)blockIdx.x * 256 + threadIdx.x) / 64 * 64;  // the wave's first row id
    const uint32_t wplane = (uint32_t)(wid / a.rows), chunk = (uint32_t)(wid % a.rows) / kColChunk;
    const uint32_t nch = a.rows / kColChunk;
    for (uint32_t w = lane_id(); w < a.wpr; w += 64)
      a.ctot[((uint64_t)wplane * nch + chunk) * a.wpr + w] = w < kDecRowWords ? cs[w] : 0ull;
  }
}

// EG: the row holding each plane's first residual 1 = the first row whose cols + 1 bits at the
// unshifted offset row * (cols + 1) are not all '1' (rows before it are ~0 and their '1').
__global__ __launch_bounds__(256) void k_dec_eg_first(DecArgs a) {
  const uint64_t gw = (uint64_t)blockIdx.x * 4 + wave_id();
  if (gw >= (uint64_t)a.rows * a.nplanes) return;
  const uint32_t plane = (uint32_t)(gw / a.rows), row = (uint32_t)(gw % a.rows);
  const uint64_t* st = plane_stream(a, plane);
  const uint64_t off = (uint64_t)row * (a.cols + 1);
  bool over;
  const uint64_t maxw = plane_words(a, plane, over);
  const uint32_t nw = (a.cols + 1 + 63) / 64;
  bool ones = true;
  for (uint32_t t = lane_id(); t < nw; t += 64) {
    const uint64_t p = off + 64ull * t;
    const uint32_t nb = min(64u, a.cols + 1 - 64 * t);
    const uint64_t i = p >> 6;
    const uint32_t sh = (uint32_t)(p & 63);
    const uint64_t hi = i < maxw ? bswap64(st[i]) : 0ull;
    uint64_t v = hi << sh;
    if (sh) v |= (i + 1 < maxw ? bswap64(st[i + 1]) : 0ull) >> (64 - sh);
    const uint64_t m = nb == 64 ? ~0ull : ~(~0ull >> nb);
    if ((v & m) != m) ones = false;
  }
  // (an atomic only below the current minimum: every row of a dense plane qualifies, and as many
  // same-address atomics would serialise the launch)
  if (__ballot(!ones) && lane_id() == 0 &&
      row < __hip_atomic_load(&a.first_row[plane], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT))
    atomicMin(&a.first_row[plane], row);
}

__global__ __launch_bounds__(256) void k_dec_eg_rows(DecArgs a) {
  const int lane = lane_id();
  const uint64_t id = (uint64_t)blockIdx.x * 4 + wave_id();
  if (id >= (uint64_t)a.rows * a.nplanes) return;
  const uint32_t plane = (uint32_t)(id / a.rows), row = (uint32_t)(id % a.rows);
  const uint64_t* st = plane_stream(a, plane);
  const uint32_t f = a.first_row[plane];
  const uint64_t bits = a.plane_bits[plane];
  bool over;
  const uint64_t maxw = plane_words(a, plane, over);
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
  bool bad = over;
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
// the exclusive XOR scan over one word column's chunk totals: one workgroup per (plane, word), the
// chunks 256 at a time (wave scans by shuffles, the waves' totals through LDS)
__global__ __launch_bounds__(256) void k_col_scan_par(uint64_t* __restrict__ ctot, uint32_t rows, uint32_t wpr) {
  __shared__ uint64_t wt[4];
  const uint32_t nch = (rows + kColChunk - 1) / kColChunk;
  const uint32_t w = blockIdx.x % wpr, plane = blockIdx.x / wpr;
  uint64_t* p = ctot + (uint64_t)plane * nch * wpr + w;
  const int lane = lane_id(), wv = (int)wave_id();
  uint64_t carry = 0;
  for (uint32_t c0 = 0; c0 < nch; c0 += 256) {
    const uint32_t c = c0 + threadIdx.x;
    const uint64_t v = c < nch ? p[(uint64_t)c * wpr] : 0ull;
    uint64_t x = v;  // inclusive XOR scan across the wave
#pragma unroll
    for (int d = 1; d < 64; d <<= 1) {
      const uint64_t y = shfl_up_u64(x, d);
      if (lane >= d) x ^= y;
    }
    if (lane == 63) wt[wv] = x;
    __syncthreads();
    uint64_t before = carry;
    for (int u = 0; u < wv; ++u) before ^= wt[u];
    const uint64_t all = wt[0] ^ wt[1] ^ wt[2] ^ wt[3];
    __syncthreads();
    if (c < nch) p[(uint64_t)c * wpr] = before ^ x ^ v;  // exclusive
    carry ^= all;
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
                   uint32_t* flags, const uint64_t* egnib) {
  DecArgs a;
  a.egnib = egnib;
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
  a.ctot = nullptr;
  const bool fused_chunks = coder == 0 && predict && rows % kColChunk == 0;
  if (coder == 0) {
    if (fused_chunks) a.ctot = ctot;
#ifdef BIC_DEC_LANES
    k_dec_golomb_lanes<<<(uint32_t)((nrows + 255) / 256), 256, 0, s>>>(a);
#else
    k_dec_golomb_nib<<<(uint32_t)((nrows + 255) / 256), 256, 0, s>>>(a);
#endif
  } else if (coder == 2) {
    k_dec_egad<<<(uint32_t)((nrows + 255) / 256), 256, 0, s>>>(a);
  } else {
    (void)launch_fill(s, a.first_row, 0xff, (size_t)nplanes * 4);
    k_dec_eg_first<<<grid, 256, 0, s>>>(a);
    k_dec_eg_rows<<<grid, 256, 0, s>>>(a);
  }
  if (predict) {
    const uint64_t nt = (uint64_t)nplanes * nch * wpr;
    if (!fused_chunks) k_col_chunks<<<(uint32_t)((nt + 255) / 256), 256, 0, s>>>(out, ctot, rows, wpr, nplanes);
    k_col_scan_par<<<nplanes * wpr, 256, 0, s>>>(ctot, rows, wpr);
    k_col_apply<<<(uint32_t)((nt + 255) / 256), 256, 0, s>>>(out, ctot, rows, wpr, nplanes);
  }
}

}  // namespace bic
