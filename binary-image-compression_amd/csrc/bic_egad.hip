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

namespace bic {

// EGLUT = J[] (eg.cpp:2-10: 0,0,0,0,1,1,1,1,2,2,2,2,3,3,3,3,4,4,5,5,6,6,7,7,8,9,...,15) in closed
// form: a table indexed by a per-lane state would be a dependent memory load per block step
__device__ __forceinline__ uint32_t eg_j(uint32_t i) { return i < 16 ? i >> 2 : (i < 24 ? (i >> 1) - 4 : i - 16); }
constexpr uint32_t kFresh = 32;  // eg.h:9: index 0, block size 1, g = 1

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
};

// One run from state i: bits of its codeword, the new state. (eg.cpp:20-37 with incBlockSize.)
__device__ __forceinline__ uint32_t eg_run(uint32_t i, uint32_t len, bool eol, uint32_t& nbits, uint32_t& m,
                                           uint32_t& g, uint32_t& rem) {
  m = 0;
  for (;;) {
    const uint32_t B = i == kFresh ? 1u : 1u << eg_j(i);
    if (len < B) break;
    len -= B;
    ++m;
    i = i == kFresh ? 1u : (i < 31 ? i + 1 : 31u);
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
    lo = eg_run(lo, len, eol, nb, m, g, rem);
    if (hi != lo) hi = eg_run(hi, len, eol, nb, m, g, rem);
  });
  a.lo_end[id] = (uint8_t)lo;
  a.hi_end[id] = (uint8_t)hi;
}

// One wave per plane: the row start states in order, 64 rows' end points loaded at a time.
__global__ __launch_bounds__(64) void k_egad_resolve(EgadArgs a) {
  const uint32_t plane = blockIdx.x;
  const int lane = lane_id();
  const uint64_t base = (uint64_t)plane * a.rows;
  uint32_t s = 0;  // the map state of the row start (a fresh coder steps like index 0)
  for (uint32_t r0 = 0; r0 < a.rows; r0 += 64) {
    const uint32_t r = r0 + lane;
    const uint32_t lo = r < a.rows ? a.lo_end[base + r] : 0, hi = r < a.rows ? a.hi_end[base + r] : 0;
    const uint32_t n = min(64u, a.rows - r0);
    for (uint32_t q = 0; q < n; ++q) {
      const uint32_t row = r0 + q;
      if (lane == 0) a.start[base + row] = row == 0 ? (uint8_t)kFresh : (uint8_t)s;
      const uint32_t l = (uint32_t)__shfl((int)lo, (int)q), h = (uint32_t)__shfl((int)hi, (int)q);
      if (l == h || s == 0) {
        s = l;
      } else if (s == 31) {
        s = h;
      } else {  // F_r is not constant here: walk the row from s (all lanes, the same walk)
        uint32_t t = s;
        row_runs(a, plane, row, [&](uint32_t len, bool eol) {
          uint32_t nb, m, g, rem;
          t = eg_run(t, len, eol, nb, m, g, rem);
        });
        s = t;
      }
    }
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

__global__ __launch_bounds__(256) void k_egad_emit(EgadArgs a) {
  const uint64_t id = (uint64_t)blockIdx.x * 256 + threadIdx.x;
  if (id >= (uint64_t)a.rows * a.nplanes) return;
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

void launch_fixup_rows(hipStream_t s, const uint64_t* boff, const uint64_t* len, const uint64_t* frag, uint64_t* out,
                       uint32_t rows, uint64_t nrows);

size_t egad_scratch_bytes(uint64_t nrows) { return nrows * (3 + 8 * 4) + 256; }

void launch_egad(hipStream_t s, const uint64_t* planes, uint32_t rows, uint32_t cols, uint32_t wpr, uint32_t nplanes,
                 int predict, uint64_t* out, uint64_t slot, uint64_t* bits, void* scratch, uint32_t* flags) {
  EgadArgs a;
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
  a.start = b;
  a.out = out;
  a.slot = slot;
  a.bits = bits;
  a.flags = flags;
  const uint32_t grid = (uint32_t)((n + 255) / 256);
  k_egad_map<<<grid, 256, 0, s>>>(a);
  k_egad_resolve<<<nplanes, 64, 0, s>>>(a);
  k_egad_len<<<grid, 256, 0, s>>>(a);
  k_egad_scan<<<nplanes, 1024, 0, s>>>(a);
  k_egad_emit<<<grid, 256, 0, s>>>(a);
  launch_fixup_rows(s, a.boff, a.len, a.frag, out, rows, n);
}

}  // namespace bic
