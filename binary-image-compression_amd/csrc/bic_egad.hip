// bic_egad.hip -- SURVEY.md §8 a9 / §7 K5: the EG coder as its author intended it -- eg.cpp:20-37
// with the commented-out incBlockSize() of line 25 enabled, the JPEG-LS run mode the #if 0 decoder
// (eg.cpp:41-55) reads: per run, a '1' per full block of 2^g zeros (the block size then grows
// along EGLUT = J[], eg.cpp:2-10, index saturating at 31 where the reference reads EGLUT[32] past
// the table), then '1' at an end of row, or '0' and the g-bit remainder followed by decBlockSize
// (eg.cpp:12-18). A fresh coder has lutIndex 0, block size 1 but g = 1 (eg.h:9): it steps like
// index 0 and spends one remainder bit until its first transition.
//
// The coder state (lutIndex, 32 values) is carried across every run of the plane. Per run the
// transition is monotone in the state (a higher index has larger blocks, so it ends at a
// higher-or-equal index), hence so is a row's composed map F_r, and F_r(0) = F_r(31) proves F_r
// constant. The passes:
//   map      thread per row: the row's runs from state 0 and from state 31 (they meet within a
//            few dozen runs of a dense row): F_r(0), F_r(31)
//   resolve  wave per plane: s_{r+1} = F_r(s_r) -- a lookup when F_r is constant or s_r is an
//            end point, otherwise a walk of the row (rows too sparse to meet: few runs)
//   length   thread per row: the row's bits from its start state; per-plane scan -> offsets
//   emit     thread per row: the row's codewords at its offset (inner words stored, the words
//            shared with neighbouring rows kept as fragments for the fixup kernel)
#include "bic_device.h"

#include <algorithm>

namespace bic {

// EGLUT = J[] (eg.cpp:2-10: 0,0,0,0,1,1,1,1,2,2,2,2,3,3,3,3,4,4,5,5,6,6,7,7,8,9,...,15) in closed
// form: a table indexed by a per-lane state would be a dependent memory load per block step
__device__ __forceinline__ uint32_t eg_j(uint32_t i) { return i < 16 ? i >> 2 : (i < 24 ? (i >> 1) - 4 : i - 16); }
constexpr uint32_t kFresh = 32;  // eg.h:9: index 0, block size 1, g = 1
constexpr uint32_t kIdent = 0xFF;  // a lane without runs: its map is the identity
constexpr uint32_t kUnk = 0xFE;    // a start state not known yet

struct EgadArgs {
  uint32_t rows, cols, wpr, used, nplanes;
  uint64_t trail;
  int predict;
  const uint64_t* planes;
  uint64_t plane_words;
  uint8_t* lo_end;   // F_r(0)
  uint8_t* hi_end;   // F_r(31)
  uint8_t* start;    // the state at each row start (kFresh for row 0)
  uint64_t* len;     // bits of each row
  uint64_t* boff;    // absolute bit offset of each row in out
  uint64_t* frag;    // [2] per row: its first / last output word when shared
  uint64_t* out;
  uint64_t slot;     // words per plane
  uint64_t* bits;    // per plane
  uint32_t* flags;
  // wave-per-row form (rows of <= 256 words): per (row, lane) the lane's state map at 0 and 31
  // (kIdent: the lane holds no run), its start state and its bits; the rows whose codewords do not
  // fit the LDS image are listed for the thread-per-row emission
  uint8_t* lane_lo;
  uint8_t* lane_hi;
  uint8_t* lane_st;
  uint32_t* lane_bits;
  uint32_t* slow_n;
  uint32_t* slow_ids;
  const uint64_t* nib;  // egad_build_nib's table (kNibTable entries)
  uint32_t* map_n;      // rows whose map k_egad_rmap could not prove constant (k_egad_lmap walks them)
  uint32_t* map_ids;
};

// One run from state i: bits of its codeword, the new state. (eg.cpp:20-37 with incBlockSize.)
// The blocks go band by band: states with one block size (0-3: 1, 4-7: 2, ..., 16-17: 16, ...,
// 24, 25, ...: one state each, 31 saturating) are crossed in one step of len >> J blocks, so a run
// costs one step per band it crosses instead of one per block.
__device__ __forceinline__ uint32_t eg_run(uint32_t i, uint32_t len, bool eol, uint32_t& nbits, uint32_t& m,
                                           uint32_t& g, uint32_t& rem) {
  m = 0;
  if (i == kFresh && len) {  // a fresh coder's block is 1 zero, after which it is at index 1
    --len;
    m = 1;
    i = 1;
  }
  if (i != kFresh) {
    for (;;) {
      const uint32_t j = eg_j(i);
      const uint32_t end = i < 16 ? (i | 3u) + 1 : (i < 24 ? (i | 1u) + 1 : i + 1);  // first state past the band
      const uint32_t q = len >> j;                                                     // blocks the run holds
      if (i == 31) {  // saturated: every block is 2^15
        m += q;
        len -= q << j;
        break;
      }
      const uint32_t room = end - i, k = min(q, room);
      m += k;
      len -= k << j;
      i += k;
      if (k < room) break;  // stopped inside the band: len < its block size
    }
  }
  g = i == kFresh ? 1u : eg_j(i);
  rem = len;
  nbits = m + 1 + (eol ? 0u : g);
  if (!eol) i = (i == kFresh || i == 0) ? 0u : i - 1;
  return i;
}

// The runs of one row: f(len, eol) per run, from the residual computed word by
// word (med of the row and the row above, pred.cpp:3-15); the next four words' loads are in flight
// while four are used (uniform across the wave: every lane's row has the same words).
template <typename F>
__device__ __forceinline__ void row_runs(const EgadArgs& a, uint32_t plane, uint32_t row, F&& f) {
  const uint64_t* cur = a.planes + (uint64_t)plane * a.plane_words + (uint64_t)row * a.wpr;
  const uint64_t* up = row ? cur - a.wpr : nullptr;
  uint64_t dcarry = 0;
  int64_t last = -1;
  uint64_t p[4], u[4];  // this group's words; the next group's loads are in flight while it is used
  auto load = [&](uint32_t w0, uint64_t (&pp)[4], uint64_t (&uu)[4]) {
#pragma unroll
    for (int q = 0; q < 4; ++q) {
      const uint32_t w = min(w0 + q, a.used - 1);
      pp[q] = cur[w];
      uu[q] = (a.predict && up) ? up[w] : 0;
    }
  };
  load(0, p, u);
  for (uint32_t w0 = 0; w0 < a.used; w0 += 4) {
    uint64_t np[4], nu[4];
    if (w0 + 4 < a.used) load(w0 + 4, np, nu);
#pragma unroll
    for (int q = 0; q < 4; ++q) {
      const uint32_t w = w0 + q;
      if (w >= a.used) break;
      uint64_t x = p[q];
      if (a.predict) {
        const uint64_t d = p[q] ^ u[q];
        x = d ^ ((d >> 1) | (dcarry << 63));
        dcarry = d & 1;
        if (row == 0 && w == 0) x &= ~BIC_MSB;
      }
      if (w == a.used - 1) x &= a.trail;
      while (x) {
        const int cz = __builtin_clzll(x);
        x &= ~(BIC_MSB >> cz);
        const int64_t j = (int64_t)w * 64 + cz;
        f((uint32_t)(j - last - 1), false);
        last = j;
      }
    }
#pragma unroll
    for (int q = 0; q < 4; ++q) {
      p[q] = np[q];
      u[q] = nu[q];
    }
  }
  f((uint32_t)((int64_t)a.cols - 1 - last), true);
}

__global__ __launch_bounds__(256) void k_egad_map(EgadArgs a) {
  const uint64_t id = (uint64_t)blockIdx.x * 256 + threadIdx.x;
  if (id >= (uint64_t)a.rows * a.nplanes) return;
  const uint32_t plane = (uint32_t)(id / a.rows), row = (uint32_t)(id % a.rows);
  uint32_t lo = 0, hi = 31;
  row_runs(a, plane, row, [&](uint32_t len, bool eol) {
    uint32_t nb, m, g, rem;
    const bool same = hi == lo;  // met: one trajectory from here on
    lo = eg_run(lo, len, eol, nb, m, g, rem);
    hi = same ? lo : eg_run(hi, len, eol, nb, m, g, rem);
  });
  a.lo_end[id] = (uint8_t)lo;
  a.hi_end[id] = (uint8_t)hi;
}

// One wave per plane: the row start states in order, 64 rows per step. Row q of a step starts at
// F_{q-1}'s constant end when that map is constant (every lane at once); the others, in order, from
// the row before's start (0 or 31: its map's ends; else a walk of that row, all lanes the same walk).
__device__ __forceinline__ uint32_t egad_apply(const EgadArgs& a, uint32_t plane, uint32_t row, uint32_t s, uint32_t lo,
                                               uint32_t hi) {
  if (lo == hi || s == 0 || s == kFresh) return lo;
  if (s == 31) return hi;
  uint32_t t = s;
  row_runs(a, plane, row, [&](uint32_t len, bool eol) {
    uint32_t nb, m, g, rem;
    t = eg_run(t, len, eol, nb, m, g, rem);
  });
  return t;
}
__global__ __launch_bounds__(64) void k_egad_resolve(EgadArgs a) {
  const uint32_t plane = blockIdx.x;
  const int lane = lane_id();
  const uint64_t base = (uint64_t)plane * a.rows;
  uint32_t s = kFresh;  // the start of the step's first row
  for (uint32_t r0 = 0; r0 < a.rows; r0 += 64) {
    const uint32_t r = r0 + lane;
    const bool in = r < a.rows;
    const uint32_t lo = in ? a.lo_end[base + r] : 0, hi = in ? a.hi_end[base + r] : 0;
    const uint32_t plo = (uint32_t)dpp_or<0x138>((int)kUnk, (int)(lo == hi ? lo : kUnk));  // row r - 1's constant end
    uint32_t st = lane == 0 ? s : plo;
    for (uint64_t unk = __ballot(in && st == kUnk); unk; unk = __ballot(in && st == kUnk)) {
      const int q = __builtin_ctzll(unk);  // rows before it are known
      const uint32_t ps = (uint32_t)__builtin_amdgcn_readlane((int)st, q - 1);
      const uint32_t pl = (uint32_t)__builtin_amdgcn_readlane((int)lo, q - 1);
      const uint32_t ph = (uint32_t)__builtin_amdgcn_readlane((int)hi, q - 1);
      const uint32_t v = egad_apply(a, plane, r0 + q - 1, ps, pl, ph);
      if (lane == q) st = v;
    }
    if (in) a.start[base + r] = (uint8_t)st;
    const uint32_t n = min(64u, a.rows - r0);
    const uint32_t ls = (uint32_t)__builtin_amdgcn_readlane((int)st, n - 1);
    const uint32_t ll = (uint32_t)__builtin_amdgcn_readlane((int)lo, n - 1);
    const uint32_t lh = (uint32_t)__builtin_amdgcn_readlane((int)hi, n - 1);
    s = egad_apply(a, plane, r0 + n - 1, ls, ll, lh);
  }
}

__global__ __launch_bounds__(256) void k_egad_len(EgadArgs a) {
  const uint64_t id = (uint64_t)blockIdx.x * 256 + threadIdx.x;
  if (id >= (uint64_t)a.rows * a.nplanes) return;
  const uint32_t plane = (uint32_t)(id / a.rows), row = (uint32_t)(id % a.rows);
  uint32_t s = a.start[id];
  uint64_t L = 0;
  row_runs(a, plane, row, [&](uint32_t len, bool eol) {
    uint32_t nb, m, g, rem;
    s = eg_run(s, len, eol, nb, m, g, rem);
    L += nb;
  });
  a.len[id] = L;
}

// Per plane (one 1024-thread workgroup): exclusive scan of the row lengths -> absolute offsets in
// the plane's slot, the plane's total; rows past the slot get length 0 (BIC_ENOSPC, never written).
__global__ __launch_bounds__(1024) void k_egad_scan(EgadArgs a) {
  __shared__ uint64_t tmp[17];
  const uint32_t plane = blockIdx.x;
  const uint64_t base = (uint64_t)plane * a.rows, cap = a.slot * 64;
  uint64_t carry = 0;
  bool over = false;
  for (uint32_t r0 = 0; r0 < a.rows; r0 += 1024) {
    const uint32_t r = r0 + threadIdx.x;
    const uint64_t v = r < a.rows ? a.len[base + r] : 0;
    uint64_t tot;
    const uint64_t pre = block_excl_scan<uint64_t>(v, tmp, tot) + carry;
    if (r < a.rows) {
      a.boff[base + r] = (uint64_t)plane * cap + pre;
      if (pre + v > cap) {
        a.len[base + r] = 0;
        over = true;
      }
    }
    carry += tot;
  }
  if (__syncthreads_or(over) && threadIdx.x == 0) atomicOr(&a.flags[0], 1u);
  if (threadIdx.x == 0) a.bits[plane] = carry;
}

__device__ void egad_emit_row(const EgadArgs& a, uint64_t id) {
  const uint64_t L = a.len[id];
  if (L == 0) return;
  const uint32_t plane = (uint32_t)(id / a.rows), row = (uint32_t)(id % a.rows);
  const uint64_t G = a.boff[id];
  const uint64_t first = G >> 6, lastw = (G + L - 1) >> 6;
  uint64_t* frag = a.frag + 2 * id;
  uint64_t cw = first, acc = 0;  // the output word being filled and its bits so far
  uint32_t fill = (uint32_t)(G & 63);
  auto flush = [&]() {
    const bool whole = (cw != first || (G & 63) == 0) && (cw != lastw || ((G + L) & 63) == 0);
    if (whole) a.out[cw] = bswap64(acc);
    else frag[cw == first ? 0 : 1] = acc;
  };
  auto put = [&](uint64_t v, uint32_t n) {  // the n (<= 64) low bits of v
    while (n) {
      const uint32_t take = min(n, 64 - fill);
      const uint64_t part = (v >> (n - take)) & (take == 64 ? ~0ull : ((1ull << take) - 1));
      acc |= part << (64 - fill - take);
      fill += take;
      n -= take;
      if (fill == 64) {
        flush();
        ++cw;
        acc = 0;
        fill = 0;
      }
    }
  };
  uint32_t s = a.start[id];
  row_runs(a, plane, row, [&](uint32_t len, bool eol) {
    uint32_t nb, m, g, rem;
    s = eg_run(s, len, eol, nb, m, g, rem);
    while (m >= 64) {
      put(~0ull, 64);
      m -= 64;
    }
    if (m) put(~0ull, m);          // a '1' per full block
    if (eol) put(1, 1);             // end of row
    else put((uint64_t)rem, 1 + g);  // '0' and the g-bit remainder
  });
  if (fill) flush();
}
__global__ __launch_bounds__(256) void k_egad_emit(EgadArgs a) {
  const uint64_t id = (uint64_t)blockIdx.x * 256 + threadIdx.x;
  if (id < (uint64_t)a.rows * a.nplanes) egad_emit_row(a, id);
}

// ------------------------------------------------------------------------------------------
// Wave-per-row form (rows of <= 256 words): lane l holds the WPL consecutive words l WPL .. and
// the runs whose 1 lies in them (plus the end-of-row run on the lane of the row's last word), so a
// lane's serial chain is ~WPL * 32 runs instead of the row's ~8,192. Each lane's map is walked from
// 0 and from 31; maps are monotone, so equal ends make it constant, and the lanes' start states
// follow from a few rounds of composition (a lane walks only when its map is not constant and its
// start is neither 0 nor 31). The rows' maps then feed the per-plane resolve as before.
constexpr uint32_t kEgImg = 384;   // u64 words of row image per wave (24,576 bits)

template <int WPL>
struct EgLane {
  uint64_t R[WPL];
  uint32_t w0;  // first word of the lane
  int jp;       // column of the row's last 1 before the lane's words (-1: none)
  bool eol;     // the lane holds the row's last word: it ends with the end-of-row run
};

template <int WPL>
__device__ __forceinline__ EgLane<WPL> eg_lane_load(const EgadArgs& a, uint32_t plane, uint32_t row) {
  EgLane<WPL> L;
  const int lane = lane_id();
  L.w0 = (uint32_t)lane * WPL;
  const uint64_t* cur = a.planes + (uint64_t)plane * a.plane_words + (uint64_t)row * a.wpr;
  const bool pr = a.predict && row;
  const uint64_t* up = pr ? cur - a.wpr : cur;  // (row 0: loaded and not used, so no load sits in a branch)
  uint64_t D[WPL], U[WPL];
#pragma unroll
  for (int i = 0; i < WPL; ++i) {
    const uint32_t w = L.w0 + i;
    const uint32_t wc = w < a.used ? w : a.used - 1;
    D[i] = cur[wc];
    U[i] = up[wc];
  }
#pragma unroll
  for (int i = 0; i < WPL; ++i) D[i] = pr ? D[i] ^ U[i] : D[i];
  const uint64_t dl = wave_shr1_u64(D[WPL - 1]);  // the D word left of the lane (lane 0: 0)
  int last = -1;
#pragma unroll
  for (int i = 0; i < WPL; ++i) {
    const uint32_t w = L.w0 + i;
    uint64_t x = D[i];
    if (a.predict) {
      x = D[i] ^ ((D[i] >> 1) | ((i ? D[i - 1] : dl) << 63));
      if (row == 0 && w == 0) x &= ~BIC_MSB;  // pred.cpp never writes pP(0,0)
    }
    x = w < a.used ? (w == a.used - 1 ? x & a.trail : x) : 0ull;
    L.R[i] = x;
    if (x) last = (int)(w * 64 + 63 - __builtin_ctzll(x));
  }
  L.jp = dpp_or<0x138>(-1, wave_incl_max(last));
  L.eol = (a.used - 1) / WPL == (uint32_t)lane;
  return L;
}

// f(len, eol) for every run of the lane, in order
template <int WPL, typename F>
__device__ __forceinline__ void eg_lane_runs(const EgLane<WPL>& L, uint32_t cols, F&& f) {
  int prev = L.jp;
#pragma unroll
  for (int i = 0; i < WPL; ++i) {
    uint64_t x = L.R[i];
    while (x) {
      const int cz = __builtin_clzll(x);
      x &= ~(BIC_MSB >> cz);
      const int j = (int)((L.w0 + i) * 64) + cz;
      f((uint32_t)(j - prev - 1), false);
      prev = j;
    }
  }
  if (L.eol) f((uint32_t)((int)cols - 1 - prev), true);
}


// ---- Nibble form of a lane's runs (the wave-per-row kernels) -------------------------------------
// The coder read pixel by pixel: a state (i, c) -- the EGLUT index and the zeros of the open block --
// where a zero completes the block when c + 1 = 2^J(i) ('1', incBlockSize) and a 1 emits '0' and c in
// J(i) bits (decBlockSize); the fresh coder (kFresh) has block size 1 and g = 1. For i <= 15 (block
// sizes 1..8) and the fresh coder there are 61 states (i, c), and a 4-pixel nibble maps each to a new
// state and <= 20 output bits: one entry of a 61 x 16 table (egad_build_nib, host; staged in LDS)
// replaces up to four run steps. Zero stretches (a word's leading zeros, whole zero words, the
// end-of-row run) advance block by block, and states above 15 (sparse rows) go pixel by pixel.
constexpr uint32_t kNibStates = 61, kNibTable = kNibStates * 16;  // u64 entries
static_assert(kNibTable == kLutEgadDec - kLutEgadNib, "the context's table buffer holds the nibble table");
__host__ __device__ __forceinline__ uint32_t nib_j(uint32_t i) { return i < 16 ? i >> 2 : (i < 24 ? (i >> 1) - 4 : i - 16); }
// (row of state (i, c), i <= 15: the band J = i / 4 starts at row 4 (2^J - 1) and holds 2^J rows per
// index: ((i % 4 + 4) << J) - 4 + c -- arithmetic, no branch)
__host__ __device__ __forceinline__ uint32_t nib_idx(uint32_t i, uint32_t c) {
  return i == kFresh ? 60u : ((((i & 3u) | 4u) << (i >> 2)) - 4u + c);
}
// A coder state as one word (the walks of k_egad_llen / k_egad_lemit): i | c << 8, and either its table
// row x 16 << 16 (i <= 15 or the fresh coder) or bit 31 (i > 15: no table row, pixel by pixel; c then
// up to 2^15 - 1, bits 8..22). Equal words are equal states.
__host__ __device__ __forceinline__ uint32_t nib_st(uint32_t i, uint32_t c) {
  return (i < 16 || i == kFresh) ? (i | c << 8 | nib_idx(i, c) * 16 << 16) : (i | c << 8 | 0x80000000u);
}
__device__ __forceinline__ uint32_t st_i(uint32_t st) { return st & 63u; }
__device__ __forceinline__ uint32_t st_c(uint32_t st) { return (st >> 8) & ((int32_t)st < 0 ? 0x7FFFu : 0xFFu); }
// entry: bits (right-aligned, <= 20) | count << 24 | nib_st(i', c') << 32 (c' <= 7: one nibble from a
// state of block size <= 8)
void egad_build_nib(uint64_t* T) {
  for (uint32_t i0 = 0; i0 <= kFresh; ++i0) {
    if (i0 >= 16 && i0 != kFresh) continue;
    const uint32_t nc = i0 == kFresh ? 1u : 1u << nib_j(i0);
    for (uint32_t c0 = 0; c0 < nc; ++c0)
      for (uint32_t nib = 0; nib < 16; ++nib) {
        uint32_t i = i0, c = c0, n = 0;
        uint64_t bits = 0;
        for (int b = 3; b >= 0; --b) {
          const uint32_t bs = i == kFresh ? 1u : 1u << nib_j(i), g = i == kFresh ? 1u : nib_j(i);
          if ((nib >> b) & 1u) {  // a 1: '0' then c in g bits, decBlockSize
            bits = (bits << (1 + g)) | c;
            n += 1 + g;
            i = (i == kFresh || i == 0) ? 0u : i - 1;
            c = 0;
          } else if (++c == bs) {  // a full block: '1', incBlockSize
            bits = (bits << 1) | 1u;
            n += 1;
            i = i == kFresh ? 1u : (i < 31 ? i + 1 : 31u);
            c = 0;
          }
        }
        T[nib_idx(i0, c0) * 16 + nib] = bits | ((uint64_t)n << 24) | ((uint64_t)nib_st(i, c) << 32);
      }
  }
}

// One coder (i, c) walking a lane; out(v, n) takes n (<= 32) right-aligned bits
struct NibCoder {
  uint32_t i, c;
  // z zeros: whole blocks ('1' each) then the open block's count
  template <typename OUT>
  __device__ __forceinline__ void zeros(uint32_t z, OUT&& out) {
    uint32_t m = 0;
    while (z) {
      if (i == kFresh) {
        --z;
        ++m;
        i = 1;
        continue;
      }
      const uint32_t bs = 1u << nib_j(i), need = bs - c;
      if (z < need) {
        c += z;
        break;
      }
      z -= need;
      ++m;
      c = 0;
      if (i < 31) ++i;
    }
    while (m >= 32) {
      out(0xFFFFFFFFu, 32);
      m -= 32;
    }
    if (m) out((1u << m) - 1u, m);
  }
  // the n (1..4) pixels at the top of the nibble, one at a time
  template <typename OUT>
  __device__ __forceinline__ void pixels(uint32_t nib, uint32_t n, OUT&& out) {
    for (uint32_t b = 0; b < n; ++b) {
      const uint32_t bs = i == kFresh ? 1u : 1u << nib_j(i), g = i == kFresh ? 1u : nib_j(i);
      if ((nib >> (3 - b)) & 1u) {
        out(c, 1 + g);
        i = (i == kFresh || i == 0) ? 0u : i - 1;
        c = 0;
      } else if (++c == bs) {
        out(1u, 1);
        i = i == kFresh ? 1u : (i < 31 ? i + 1 : 31u);
        c = 0;
      }
    }
  }
  template <typename OUT>
  __device__ __forceinline__ void nibble(uint32_t nib, uint32_t n, const uint64_t* T, OUT&& out) {
    if (n == 4 && (i < 16 || i == kFresh)) {
      const uint64_t e = T[nib_idx(i, c) * 16 + nib];
      const uint32_t cnt = (uint32_t)(e >> 24) & 31u;
      if (cnt) out((uint32_t)e & 0xFFFFFFu, cnt);
      i = (uint32_t)(e >> 32) & 63u;
      c = (uint32_t)(e >> 40) & 0xFFu;
    } else {
      pixels(nib, n, out);
    }
  }
};

// The lane's runs from state s (its first run's start, column jp + 1, has an empty block): every
// column from there through the lane's last 1 (and, on the row's last lane, through the row's end
// and the end-of-row '1'). Returns the state after them.
// (stop: return after the step that ends at that column -- a step boundary of this lane's walk, whose
// boundaries do not depend on the state: eg_lane_nib2c's meeting point)
template <int WPL, typename OUT>
__device__ __forceinline__ uint32_t eg_lane_nib(const EgLane<WPL>& L, uint32_t used, uint32_t cols, uint32_t s,
                                                const uint64_t* T, OUT&& out, uint32_t stop = 0xFFFFFFFFu) {
  NibCoder k{s, 0};
  uint32_t col = (uint32_t)(L.jp + 1);  // the next column to code
#pragma unroll
  for (int t = 0; t < WPL; ++t) {
    const uint32_t w = L.w0 + t;
    const uint64_t x = L.R[t];
    if (w >= used || !x) continue;  // (zeros: coded by the next stretch)
    const uint32_t f1 = w * 64 + (uint32_t)__builtin_clzll(x), l1 = w * 64 + 63 - (uint32_t)__builtin_ctzll(x);
    const uint32_t a = f1 & ~3u;  // the nibble holding the word's first 1
    if (a > col) {  // (a >= col: col follows a 1 of an earlier word, or the row start)
      k.zeros(a - col, out);
      if (a >= stop) return k.i;
    }
    for (uint32_t nb = a; nb <= l1; nb += 4) {
      const uint32_t n = nb + 3 <= l1 ? 4u : l1 - nb + 1;
      k.nibble((uint32_t)(x >> (60 - (nb - w * 64))) & 15u, n, T, out);
      if (nb + n >= stop) return k.i;
    }
    col = l1 + 1;
  }
  if (L.eol) {
    k.zeros(cols - col, out);
    if (cols >= stop) return k.i;
    out(1u, 1);  // end of row (eg.cpp:30-32: no decBlockSize)
  }
  return k.i;
}

// eg_lane_nib from 0 and from 31 at once (the lane's map ends, k_egad_lmap): the two coders step
// together until they hold the same (i, c), after which the second is a copy of the first -- in a
// dense row they meet within a few nibbles
// (COUNT: also the bits of the walk from 0 -- btot in all, bat of them before the meeting point X, the
// column after the step where the two walks first hold the same state; X = ~0: they never meet. A walk
// from any start lies between the two (each step is monotone in (i, c) ordered by i, then c), so it
// has met them by X too, and its bits after X are btot - bat.)
template <int WPL, bool COUNT = false>
__device__ __forceinline__ void eg_lane_nib2(const EgLane<WPL>& L, uint32_t used, uint32_t cols, const uint64_t* T,
                                             uint32_t& lo, uint32_t& hi, uint32_t* X = nullptr, uint32_t* btot = nullptr,
                                             uint32_t* bat = nullptr) {
  NibCoder k0{0, 0}, k1{31, 0};
  bool met = false;
  uint32_t nb0 = 0, mX = 0xFFFFFFFFu, mb = 0;
  auto cnt = [&](uint32_t, uint32_t n) {
    if constexpr (COUNT) nb0 += n;
  };
  auto none = [](uint32_t, uint32_t) {};
  auto check = [&](uint32_t pos) {
    if (!met && k0.i == k1.i && k0.c == k1.c) {
      met = true;
      mX = pos;
      mb = nb0;
    }
  };
  uint32_t col = (uint32_t)(L.jp + 1);
#pragma unroll
  for (int t = 0; t < WPL; ++t) {
    const uint32_t w = L.w0 + t;
    const uint64_t x = L.R[t];
    if (w >= used || !x) continue;
    const uint32_t f1 = w * 64 + (uint32_t)__builtin_clzll(x), l1 = w * 64 + 63 - (uint32_t)__builtin_ctzll(x);
    const uint32_t a = f1 & ~3u;
    if (a > col) {
      k0.zeros(a - col, cnt);
      if (!met) k1.zeros(a - col, none);
      check(a);
    }
    for (uint32_t nb = a; nb <= l1; nb += 4) {
      const uint32_t nib = (uint32_t)(x >> (60 - (nb - w * 64))) & 15u, n = nb + 3 <= l1 ? 4u : l1 - nb + 1;
      k0.nibble(nib, n, T, cnt);
      if (!met) {
        k1.nibble(nib, n, T, none);
        check(nb + n);
      }
    }
    col = l1 + 1;
  }
  if (L.eol) {
    k0.zeros(cols - col, cnt);
    if (!met) k1.zeros(cols - col, none);
    check(cols);
    cnt(1u, 1);
  }
  lo = k0.i;
  hi = met ? k0.i : k1.i;
  if constexpr (COUNT) {
    *X = mX;
    *btot = nb0;
    *bat = mb;
  }
}

// ---- The lane walk as a chain of table steps (k_egad_llen, k_egad_lemit, the lane chain) ------------
// The same coder over the same columns as eg_lane_nib, with other step boundaries: the zeros before the
// nibble of the lane's first 1, then EVERY nibble from there to the one before the nibble of its last 1
// -- whole nibbles, across its words and through zero words, so no per-word partial nibble and zero
// stretch -- then that last nibble's pixels, then (row's last lane) the zeros to the row end and the
// end-of-row '1'. A table step is one LDS read whose high half is the next state (nib_st), so a step
// costs a handful of VALU; states above 15 (sparse rows) take the pixel path for their nibble. The
// boundaries depend on the lane's pixels alone, so eg_lane_walk2's meeting point is a boundary of every
// walk of the lane. (bic_egad.hip, round 6: 2.97 ms -> see DESIGN.md §3.)
#ifndef BIC_EGAD_CHAIN
#define BIC_EGAD_CHAIN 1
#endif
constexpr bool kEgadChain = BIC_EGAD_CHAIN != 0;
template <int WPL>
struct LaneSpan {
  uint32_t f1, l1;  // the lane's first and last 1 (columns); any = a 1 in the lane
  bool any;
};
template <int WPL>
__device__ __forceinline__ LaneSpan<WPL> lane_span(const EgLane<WPL>& L) {
  LaneSpan<WPL> sp{0u, 0u, false};
#pragma unroll
  for (int t = WPL - 1; t >= 0; --t) {  // (backwards: the first nonzero word's f1 is the last written)
    const uint64_t x = L.R[t];
    if (x) {
      const uint32_t w = L.w0 + t;
      if (!sp.any) sp.l1 = w * 64 + 63 - (uint32_t)__builtin_ctzll(x);
      sp.f1 = w * 64 + (uint32_t)__builtin_clzll(x);
      sp.any = true;
    }
  }
  return sp;
}
// the lane's nibble k (0 .. 16 WPL - 1), k uniform or not
template <int WPL>
__device__ __forceinline__ uint32_t lane_nib(const EgLane<WPL>& L, uint32_t k) {
  uint64_t x = 0;
#pragma unroll
  for (int t = 0; t < WPL; ++t) x = (k >> 4) == (uint32_t)t ? L.R[t] : x;
  return (uint32_t)(x >> (60 - 4 * (k & 15))) & 15u;
}
// one step of state st over a whole nibble
template <typename OUT>
__device__ __forceinline__ uint32_t chain_step(uint32_t st, uint32_t nib, const uint64_t* T, OUT&& out) {
  if ((int32_t)st < 0) {  // i > 15: pixel by pixel
    NibCoder q{st_i(st), st_c(st)};
    q.pixels(nib, 4, out);
    return nib_st(q.i, q.c);
  }
  const uint64_t e = T[(st >> 16) + nib];
  const uint32_t n = (uint32_t)(e >> 24) & 31u;
  if (n) out((uint32_t)e & 0xFFFFFFu, n);
  return (uint32_t)(e >> 32);
}
// chain_step for a walk that writes nothing (the map walks): a state above 15 whose open block cannot
// fill within the nibble (c + 4 < 2^J(i), J >= 4) steps in closed form -- each 1 lowers i by one and
// the zeros after the last 1 open the next block (fewer than 4 < 8, the block size of any i' >= 12) --
// so the walk from 31 leaves the pixel path after its first run instead of at i = 15
__device__ __forceinline__ uint32_t chain_step_free(uint32_t st, uint32_t nib, const uint64_t* T) {
  if ((int32_t)st < 0) {
    const uint32_t i = st_i(st), c = st_c(st);
    if (c + 4 < (1u << nib_j(i))) return nib_st(i - (uint32_t)__popc(nib), nib ? (uint32_t)__builtin_ctz(nib) : c + 4);
  }
  return chain_step(st, nib, T, [](uint32_t, uint32_t) {});
}
// eg_lane_nib's contract: the state after the lane's columns from start s (returns i); stop: return after
// the step that ends at that column (one of this walk's boundaries). FREE: the walk writes nothing
template <int WPL, bool FREE = false, typename OUT>
__device__ __forceinline__ uint32_t eg_lane_walk(const EgLane<WPL>& L, uint32_t used, uint32_t cols, uint32_t s,
                                                 const uint64_t* T, OUT&& out, uint32_t stop = 0xFFFFFFFFu) {
  const LaneSpan<WPL> sp = lane_span(L);
  NibCoder k{s, 0};
  uint32_t col = (uint32_t)(L.jp + 1);
  if (sp.any) {
    const uint32_t a0 = sp.f1 & ~3u, base = L.w0 * 64;
    if (a0 > col) {
      k.zeros(a0 - col, out);
      if (a0 >= stop) return k.i;
    }
    const uint32_t kf = (a0 - base) >> 2, kl = (sp.l1 - base) >> 2;
    const bool cut = stop <= base + 4 * kl;  // stops after a whole nibble
    const uint32_t ke = cut ? (stop - base) >> 2 : kl;
    uint32_t st = nib_st(k.i, k.c);
#pragma unroll
    for (int t = 0; t < WPL; ++t) {
      uint64_t cur = L.R[t];
#pragma unroll 1
      for (uint32_t j = 0; j < 16; ++j, cur <<= 4) {
        const uint32_t kk = 16 * t + j;
        if (kk >= kf && kk < ke) {
          if constexpr (FREE) st = chain_step_free(st, (uint32_t)(cur >> 60), T);
          else st = chain_step(st, (uint32_t)(cur >> 60), T, out);
        }
      }
    }
    if (cut) return st_i(st);
    NibCoder q{st_i(st), st_c(st)};
    q.pixels(lane_nib(L, kl), (sp.l1 & 3u) + 1, out);
    k = q;
    col = sp.l1 + 1;
    if (col >= stop) return k.i;
  }
  if (L.eol) {
    k.zeros(cols - col, out);
    if (cols >= stop) return k.i;
    out(1u, 1);  // end of row (eg.cpp:30-32: no decBlockSize)
  }
  return k.i;
}
// eg_lane_nib2<WPL, true>'s contract over eg_lane_walk's boundaries: the walks from 0 and 31 together
// until they hold the same state (X: the boundary where they first do; ~0: never), the walk from 0
// counted (btot bits in all, bat before X)
template <int WPL>
__device__ __forceinline__ void eg_lane_walk2(const EgLane<WPL>& L, uint32_t used, uint32_t cols, const uint64_t* T,
                                              uint32_t& lo, uint32_t& hi, uint32_t& X, uint32_t& btot, uint32_t& bat) {
  const LaneSpan<WPL> sp = lane_span(L);
  NibCoder k0{0, 0}, k1{31, 0};
  bool met = false;
  uint32_t nb0 = 0, mX = 0xFFFFFFFFu, mb = 0;
  auto cnt = [&](uint32_t, uint32_t n) { nb0 += n; };
  auto none = [](uint32_t, uint32_t) {};
  auto check = [&](uint32_t pos, bool same) {
    if (!met && same) {
      met = true;
      mX = pos;
      mb = nb0;
    }
  };
  uint32_t col = (uint32_t)(L.jp + 1);
  if (sp.any) {
    const uint32_t a0 = sp.f1 & ~3u, base = L.w0 * 64;
    if (a0 > col) {
      k0.zeros(a0 - col, cnt);
      if (!met) k1.zeros(a0 - col, none);
      check(a0, k0.i == k1.i && k0.c == k1.c);
    }
    const uint32_t kf = (a0 - base) >> 2, kl = (sp.l1 - base) >> 2;
    uint32_t s0 = nib_st(k0.i, k0.c), s1 = nib_st(k1.i, k1.c);
#pragma unroll
    for (int t = 0; t < WPL; ++t) {
      uint64_t cur = L.R[t];
#pragma unroll 1
      for (uint32_t j = 0; j < 16; ++j, cur <<= 4) {
        const uint32_t kk = 16 * t + j;
        if (kk >= kf && kk < kl) {
          const uint32_t nib = (uint32_t)(cur >> 60);
          s0 = chain_step(s0, nib, T, cnt);
          if (!met) {
            s1 = chain_step_free(s1, nib, T);
            check(base + 4 * (kk + 1), s0 == s1);
          }
        }
      }
    }
    const uint32_t nib = lane_nib(L, kl), n = (sp.l1 & 3u) + 1;
    k0 = NibCoder{st_i(s0), st_c(s0)};
    k0.pixels(nib, n, cnt);
    k1 = NibCoder{st_i(s1), st_c(s1)};
    if (!met) k1.pixels(nib, n, none);
    col = sp.l1 + 1;
    check(col, k0.i == k1.i && k0.c == k1.c);
  }
  if (L.eol) {
    k0.zeros(cols - col, cnt);
    if (!met) k1.zeros(cols - col, none);
    check(cols, k0.i == k1.i && k0.c == k1.c);
    cnt(1u, 1);
  }
  lo = k0.i;
  hi = met ? k0.i : k1.i;
  X = mX;
  btot = nb0;
  bat = mb;
}

// Every lane's start state for the row start s0 (lane 0 starts at s0): constant maps are known at
// once; a round hands each known end to the next lane. Returns the lane's start; *end = its end.
template <int WPL>
__device__ __forceinline__ uint32_t eg_lane_chain(const EgLane<WPL>& L, uint32_t used, uint32_t cols, uint32_t lo,
                                                  uint32_t hi, uint32_t s0, const uint64_t* T, uint32_t* end) {
  const int lane = lane_id();
  const bool ident = lo == kIdent;
  bool done = !ident && lo == hi;
  uint32_t sout = done ? lo : kUnk;
  uint32_t sin = lane == 0 ? s0 : kUnk;
  for (;;) {
    if (!done && sin != kUnk) {
      if (ident) sout = sin;
      else if (sin == 0 || sin == kFresh) sout = lo;  // (a fresh coder steps like index 0)
      else if (sin == 31) sout = hi;
      else if constexpr (kEgadChain) sout = eg_lane_walk<WPL, true>(L, used, cols, sin, T, [](uint32_t, uint32_t) {});
      else sout = eg_lane_nib(L, used, cols, sin, T, [](uint32_t, uint32_t) {});
      done = true;
    }
    const uint32_t prev = (uint32_t)dpp_or<0x138>((int)kUnk, (int)(done ? sout : kUnk));
    if (lane > 0 && sin == kUnk) sin = prev;
    if (__ballot(!done || sin == kUnk) == 0) break;
  }
  *end = sout;
  return sin;
}

// the nibble table into the workgroup's LDS (before any wave leaves)
__device__ __forceinline__ void nib_stage(const EgadArgs& a, uint64_t* sT) {
  for (uint32_t i = threadIdx.x; i < kNibTable; i += blockDim.x) sT[i] = a.nib[i];
  __syncthreads();
}

// The lanes' maps and the row's map F_r(0), F_r(31) (lane 63 carries the row's end).
template <int WPL>
__device__ __forceinline__ void egad_lmap_row(const EgadArgs& a, uint64_t id, const uint64_t* sT) {
  const uint32_t plane = (uint32_t)(id / a.rows), row = (uint32_t)(id % a.rows);
  const EgLane<WPL> L = eg_lane_load<WPL>(a, plane, row);
  bool any = L.eol;
#pragma unroll
  for (int t = 0; t < WPL; ++t) any |= L.R[t] != 0;
  uint32_t lo = kIdent, hi = kIdent;
  if (any) {
    eg_lane_nib2(L, a.used, a.cols, sT, lo, hi);
  }
  uint32_t e0, e31;
  (void)eg_lane_chain(L, a.used, a.cols, lo, hi, 0, sT, &e0);
  (void)eg_lane_chain(L, a.used, a.cols, lo, hi, 31, sT, &e31);
  if (lane_id() == 63) {
    a.lo_end[id] = (uint8_t)e0;
    a.hi_end[id] = (uint8_t)e31;
  }
}

// The row's map from a window at its end (k_egad_rmap, thread per row): the walks from 0 and 31 begin
// after the first 1 of the row's last four words -- any state there lies between them -- and go to the
// row's end; if they meet, F_r is constant and that is its value. A row of <= 4 words is walked whole
// from its start (F_r(0) and F_r(31) exactly). Other rows (no 1 in the window, or the walks not met)
// are listed for k_egad_lmap, which walks every lane of the row.
__device__ __forceinline__ uint64_t egad_resid(const EgadArgs& a, uint32_t plane, uint32_t row, uint32_t w) {
  if (w >= a.used) return 0;
  const uint64_t* cur = a.planes + (uint64_t)plane * a.plane_words + (uint64_t)row * a.wpr;
  uint64_t x = cur[w];
  if (a.predict) {
    const uint64_t* up = cur - a.wpr;
    const uint64_t d = x ^ (row ? up[w] : 0ull);
    const uint64_t dl = w ? cur[w - 1] ^ (row ? up[w - 1] : 0ull) : 0ull;
    x = d ^ ((d >> 1) | (dl << 63));
    if (row == 0 && w == 0) x &= ~BIC_MSB;  // pred.cpp never writes pP(0,0)
  }
  return w == a.used - 1 ? x & a.trail : x;
}
__global__ __launch_bounds__(256) void k_egad_rmap(EgadArgs a) {
  __shared__ uint64_t sT[kNibTable];
  nib_stage(a, sT);
  const uint64_t id = (uint64_t)blockIdx.x * 256 + threadIdx.x;
  if (id >= (uint64_t)a.rows * a.nplanes) return;
  const uint32_t plane = (uint32_t)(id / a.rows), row = (uint32_t)(id % a.rows);
  constexpr int K = 4;
  EgLane<K> L;
  L.w0 = a.used > K ? a.used - K : 0u;
  L.eol = true;
  L.jp = -1;
#pragma unroll
  for (int t = 0; t < K; ++t) L.R[t] = egad_resid(a, plane, row, L.w0 + t);
  if (L.w0) {  // start after the window's first 1
    bool found = false;
#pragma unroll
    for (int t = 0; t < K; ++t) {
      if (!found && L.R[t]) {
        const uint32_t b = (uint32_t)__builtin_clzll(L.R[t]);
        L.jp = (int)((L.w0 + t) * 64 + b);
        L.R[t] &= b == 63 ? 0ull : ~0ull >> (b + 1);
        found = true;
      } else if (!found) {
        L.R[t] = 0;
      }
    }
    if (!found) {
      a.map_ids[atomicAdd(a.map_n, 1u)] = (uint32_t)id;
      return;
    }
  }
  uint32_t lo, hi;
  eg_lane_nib2(L, a.used, a.cols, sT, lo, hi);
  if (!L.w0 || lo == hi) {
    a.lo_end[id] = (uint8_t)lo;
    a.hi_end[id] = (uint8_t)hi;
  } else {
    a.map_ids[atomicAdd(a.map_n, 1u)] = (uint32_t)id;
  }
}

// (the rows k_egad_rmap listed, a wave each)
template <int WPL>
__global__ __launch_bounds__(256) void k_egad_lmap(EgadArgs a) {
  __shared__ uint64_t sT[kNibTable];
  nib_stage(a, sT);
  const uint32_t nl = __hip_atomic_load(a.map_n, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  for (uint32_t li = blockIdx.x * 4 + wave_id(); li < nl; li += gridDim.x * 4)
    egad_lmap_row<WPL>(a, a.map_ids[li], sT);
}

// The row's bits from its start state: per lane its start and bits, the row's total.
template <int WPL>
__global__ __launch_bounds__(256) void k_egad_llen(EgadArgs a) {
  __shared__ uint64_t sT[kNibTable];
  nib_stage(a, sT);
  const uint64_t id = (uint64_t)blockIdx.x * 4 + wave_id();
  if (id >= (uint64_t)a.rows * a.nplanes) return;
  const uint32_t plane = (uint32_t)(id / a.rows), row = (uint32_t)(id % a.rows);
  const EgLane<WPL> L = eg_lane_load<WPL>(a, plane, row);
  // the lane's map ends (walks from 0 and 31 together, the one from 0 counted), its start from the
  // row's, then its bits: a walk from the start up to the meeting point and the rest from the count
  bool any = L.eol;
#pragma unroll
  for (int t = 0; t < WPL; ++t) any |= L.R[t] != 0;
  uint32_t lo = kIdent, hi = kIdent, X = 0xFFFFFFFFu, btot = 0, bat = 0;
  if (any) {
    if constexpr (kEgadChain) eg_lane_walk2(L, a.used, a.cols, sT, lo, hi, X, btot, bat);
    else eg_lane_nib2<WPL, true>(L, a.used, a.cols, sT, lo, hi, &X, &btot, &bat);
  }
  a.lane_lo[id * 64 + lane_id()] = (uint8_t)lo;
  uint32_t end;
  const uint32_t s = eg_lane_chain(L, a.used, a.cols, lo, hi, a.start[id], sT, &end);
  uint32_t bits = 0;
  if (lo != kIdent) {
    if constexpr (kEgadChain) (void)eg_lane_walk(L, a.used, a.cols, s, sT, [&](uint32_t, uint32_t n) { bits += n; }, X);
    else (void)eg_lane_nib(L, a.used, a.cols, s, sT, [&](uint32_t, uint32_t n) { bits += n; }, X);
    if (X != 0xFFFFFFFFu) bits += btot - bat;
  }
  a.lane_st[id * 64 + lane_id()] = (uint8_t)s;
  a.lane_bits[id * 64 + lane_id()] = bits;
  const uint64_t tot = wave_sum_u64(bits);
  if (lane_id() == 0) a.len[id] = tot;
}

// Bits into a 64-bit LDS row image (MSB-first), words OR'd as a lane leaves them (lanes share at
// most their first and last word).
struct EgImgSink {
  uint64_t* img;
  uint32_t idx;
  uint64_t cur, nxt;  // image words idx and idx + 1 so far
  __device__ __forceinline__ void flush() {
    if (cur) lds_or64(img, idx, cur);
    if (nxt) lds_or64(img, idx + 1, nxt);
    cur = nxt = 0;
  }
  // the n (1..32) low bits of v at bit pos; pos never moves back and by at most 32 per call, so the
  // window only ever slides by one word (selects, one branch per 64 bits)
  __device__ __forceinline__ void put(uint32_t pos, uint64_t v, uint32_t n) {
    const uint32_t i = pos >> 6, e = (pos & 63) + n;
    if (i != idx) {
      if (cur) lds_or64(img, idx, cur);
      cur = i == idx + 1 ? nxt : 0ull;
      if (i != idx + 1 && nxt) lds_or64(img, idx + 1, nxt);
      nxt = 0;
      idx = i;
    }
    v &= (1ull << n) - 1ull;
    cur |= e <= 64 ? v << (64 - e) : v >> (e - 64);
    nxt |= e > 64 ? v << ((128 - e) & 63) : 0ull;
  }
};

template <int WPL>
__global__ __launch_bounds__(256) void k_egad_lemit(EgadArgs a) {
  __shared__ __attribute__((aligned(16))) uint64_t imgs[4][kEgImg];
  __shared__ uint64_t sT[kNibTable];
  nib_stage(a, sT);
  const uint64_t id = (uint64_t)blockIdx.x * 4 + wave_id();
  if (id >= (uint64_t)a.rows * a.nplanes) return;
  const uint64_t Ltot = a.len[id];
  if (Ltot == 0) return;  // past the slot (BIC_ENOSPC)
  const uint32_t plane = (uint32_t)(id / a.rows), row = (uint32_t)(id % a.rows);
  const uint64_t G = a.boff[id];
  if ((G & 63) + Ltot > (uint64_t)(kEgImg - 1) * 64) {  // too long for the image: the thread-per-row emission
    if (lane_id() == 0) a.slow_ids[atomicAdd(a.slow_n, 1u)] = (uint32_t)id;
    return;
  }
  uint64_t* img = imgs[wave_id()];
  for (uint32_t i = lane_id(); i < kEgImg; i += 64) img[i] = 0;
  __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
  __builtin_amdgcn_wave_barrier();
  __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
  const EgLane<WPL> L = eg_lane_load<WPL>(a, plane, row);
  const uint32_t bits = a.lane_bits[id * 64 + lane_id()];
  uint32_t pos = wave_incl_sum_u32(bits) - bits;  // the lane's first bit in the row
  uint32_t s = a.lane_st[id * 64 + lane_id()];
  EgImgSink k{img, 0, 0, 0};
  if (a.lane_lo[id * 64 + lane_id()] != kIdent) {
    if constexpr (kEgadChain) {
      // codewords gathered 32 bits at a time in a register (acc's low nacc bits, nacc < 32 between
      // calls), the image window touched once per 32 bits instead of once per codeword
      uint64_t acc = 0;
      uint32_t nacc = 0;
      (void)eg_lane_walk(L, a.used, a.cols, s, sT, [&](uint32_t v, uint32_t n) {  // n <= 32
        acc = (acc << n) | v;
        nacc += n;
        if (nacc >= 32) {
          nacc -= 32;
          k.put(pos, (uint32_t)(acc >> nacc), 32);
          pos += 32;
        }
      });
      if (nacc) k.put(pos, (uint32_t)acc, nacc);
    } else {
      (void)eg_lane_nib(L, a.used, a.cols, s, sT, [&](uint32_t v, uint32_t n) {
        k.put(pos, v, n);
        pos += n;
      });
    }
  }
  k.flush();
  __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
  __builtin_amdgcn_wave_barrier();
  __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
  // image bit b = row bit b; write_row64 wants the row at bit G % 64 of image word 0's frame
  write_row64(img, Ltot, G, a.out, a.frag + 2 * id);
}

// The rows too long for the LDS image, thread per row (k_egad_emit's body on a list).
__device__ void egad_emit_row(const EgadArgs& a, uint64_t id);
__global__ __launch_bounds__(256) void k_egad_emit_list(EgadArgs a) {
  const uint32_t n = __hip_atomic_load(a.slow_n, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  for (uint32_t i = blockIdx.x * 256 + threadIdx.x; i < n; i += gridDim.x * 256) egad_emit_row(a, a.slow_ids[i]);
}

void launch_fixup_rows(hipStream_t s, const uint64_t* boff, const uint64_t* len, const uint64_t* frag, uint64_t* out,
                       uint32_t rows, uint64_t nrows);

// The decoders' row index (bic_egad_row_index): per row its first bit in the plane's stream and the
// coder state there (eg.h's lutIndex, kFresh for a fresh coder)
__global__ __launch_bounds__(256) void k_egad_index(EgadArgs a, uint64_t* index) {
  const uint64_t id = (uint64_t)blockIdx.x * 256 + threadIdx.x;
  if (id >= (uint64_t)a.rows * a.nplanes) return;
  index[2 * id] = a.boff[id] - (id / a.rows) * a.slot * 64;
  index[2 * id + 1] = a.start[id];
}

// len, boff, frag[2] (u64), lo_end, hi_end, start (u8); per (row, lane): lane_lo, lane_hi, lane_st
// (u8), lane_bits (u32); the slow-row list and its count
size_t egad_scratch_bytes(uint64_t nrows) { return nrows * (3 + 8 * 4) + nrows * 64 * 7 + nrows * 4 * 2 + 512; }

void launch_egad(hipStream_t s, const uint64_t* planes, uint32_t rows, uint32_t cols, uint32_t wpr, uint32_t nplanes,
                 int predict, uint64_t* out, uint64_t slot, uint64_t* bits, void* scratch, uint32_t* flags,
                 uint64_t* index, const uint64_t* nib) {
  EgadArgs a;
  a.nib = nib;
  a.rows = rows;
  a.cols = cols;
  a.wpr = wpr;
  a.used = (cols + 63) / 64;
  a.nplanes = nplanes;
  a.trail = cols % 64 ? ~(~0ull >> (cols % 64)) : ~0ull;
  a.predict = predict;
  a.planes = planes;
  a.plane_words = (uint64_t)rows * wpr;
  const uint64_t n = (uint64_t)rows * nplanes;
  uint64_t* q = reinterpret_cast<uint64_t*>(scratch);
  a.len = q; q += n;
  a.boff = q; q += n;
  a.frag = q; q += 2 * n;
  uint8_t* b = reinterpret_cast<uint8_t*>(q);
  a.lo_end = b; b += n;
  a.hi_end = b; b += n;
  a.start = b; b += n;
  a.lane_lo = b; b += n * 64;
  a.lane_hi = b; b += n * 64;
  a.lane_st = b; b += n * 64;
  uintptr_t u = (reinterpret_cast<uintptr_t>(b) + 15) & ~(uintptr_t)15;
  a.lane_bits = reinterpret_cast<uint32_t*>(u);
  a.slow_ids = a.lane_bits + n * 64;
  a.slow_n = a.slow_ids + n;
  a.map_n = a.slow_n + 1;  // (zeroed with slow_n)
  a.map_ids = a.slow_n + 2;
  a.out = out;
  a.slot = slot;
  a.bits = bits;
  a.flags = flags;
  const uint32_t grid = (uint32_t)((n + 255) / 256);
  // out == NULL: the row index only (no emission)
  if (a.used > 256) {  // rows wider than 16384 columns: thread per row
    k_egad_map<<<grid, 256, 0, s>>>(a);
    k_egad_resolve<<<nplanes, 64, 0, s>>>(a);
    k_egad_len<<<grid, 256, 0, s>>>(a);
    k_egad_scan<<<nplanes, 1024, 0, s>>>(a);
    if (out) k_egad_emit<<<grid, 256, 0, s>>>(a);
  } else {  // wave per row (4 rows per workgroup)
    const uint32_t wgrid = (uint32_t)((n + 3) / 4);
    (void)launch_fill(s, a.slow_n, 0, 8);
    // row maps from windows (thread per row), the rows they cannot settle by their lanes (a wave each)
    const uint32_t lgrid = (uint32_t)std::min<uint64_t>(wgrid, 2048);
#define BIC_EGAD(W)                                   \
  k_egad_rmap<<<grid, 256, 0, s>>>(a);                \
  k_egad_lmap<W><<<lgrid, 256, 0, s>>>(a);            \
  k_egad_resolve<<<nplanes, 64, 0, s>>>(a);           \
  k_egad_llen<W><<<wgrid, 256, 0, s>>>(a);            \
  k_egad_scan<<<nplanes, 1024, 0, s>>>(a);            \
  if (out) {                                          \
    k_egad_lemit<W><<<wgrid, 256, 0, s>>>(a);         \
    k_egad_emit_list<<<256, 256, 0, s>>>(a);          \
  }
    if (a.used <= 64) { BIC_EGAD(1) } else if (a.used <= 128) { BIC_EGAD(2) } else { BIC_EGAD(4) }
#undef BIC_EGAD
  }
  if (index) k_egad_index<<<grid, 256, 0, s>>>(a, index);
  if (out) launch_fixup_rows(s, a.boff, a.len, a.frag, out, rows, n);
}

}  // namespace bic
