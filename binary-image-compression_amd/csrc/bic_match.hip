// bic_match.hip -- compress7_test.cpp:117-275 with a search window R and a match threshold T
//  on one plane.
//
// Every tile searches the image as the residual write-back of all earlier tiles left it
// (:266, :272), so tiles are causally ordered. The region of tile (i, j) reaches W rows into its
// own tile row (columns left of it) and R rows up to column j0 + R + W - 1, so it depends on
// tile (i, j-1) and on tile (i-1, jd), jd = (maxj + W - 1) / W -- everything else it reads is
// covered transitively. Tiles run as a wavefront inside one launch:
//
//   * G workgroups per tile take tickets in raster order (ticket q -> tile q / G, part q % G), so a
//     workgroup only ever waits for tiles of lower tickets, which are already resident;
//   * each waits for its two predecessors' done flags (agent-scope acquire), stages the search
//     region in LDS and scans its share of the windows in the reference's scan order, in chunks,
//     stopping once a window with distance <= T is found (the reference's early exit);
//   * keys (d <= T ? 0 : d, scan index, d) are min-reduced per tile with a 64-bit atomicMin; the
//     last workgroup to arrive finishes the tile -- modes, lengths, residual write-back -- and
//     releases the tile's done flag.
//
// A second single-workgroup kernel codes the chosen weights with the two GolombCoders
// (golomb_match / golomb_nomatch, :256 / :269) in raster order.
#include "bic_device.h"

#include <algorithm>

namespace bic {

#ifdef BIC_STAMPS  // diagnostic build only (make stamps): per-tile phase clocks of the row workgroup
__device__ unsigned long long g_mstamps[1 << 20];
#define MSTAMP(tile, slot)                                                                   \
  do {                                                                                      \
    const unsigned long long t_ = __builtin_amdgcn_s_memtime();                             \
    if ((uint64_t)(tile) * 16 + (slot) < (1u << 20)) g_mstamps[(uint64_t)(tile) * 16 + (slot)] = t_; \
  } while (0)
int read_match_stamps(uint64_t* host, size_t n) {
  return hipMemcpyFromSymbol(host, HIP_SYMBOL(g_mstamps), n * 8, 0, hipMemcpyDeviceToHost) == hipSuccess ? 0 : 3;
}
#else
#define MSTAMP(tile, slot) \
  do {                     \
  } while (0)
#endif

namespace {

constexpr int kMB = 256;                 // threads per workgroup
constexpr int kPerThread = 4;            // windows per thread per chunk
constexpr uint32_t kChunk = kMB * kPerThread;
constexpr uint32_t kRegionWords = 4096;  // LDS image of the search region (32 KiB)
// A window's place in the reference's scan order is pos = loop << 32 | a << 16 | c (loop 0 or 1,
// a = rows down from the loop's first row, c = columns left of its first column): increasing pos is
// the scan order, and pos decodes to the window without a division. Keys order windows for the
// reduction: (d <= T ? 0 : d) << 51 | pos << 13 | d.
constexpr int kIdxShift = 13, kDpShift = 51;
constexpr uint64_t kIdxMask = (1ull << 38) - 1;

__device__ __forceinline__ uint64_t scan_pos(uint32_t loop, uint32_t a, uint32_t c) {
  return ((uint64_t)loop << 32) | ((uint64_t)a << 16) | c;
}
__device__ __forceinline__ unsigned long long make_key(uint32_t d, uint32_t T, uint64_t pos) {
  return ((unsigned long long)(d <= T ? 0u : d) << kDpShift) | ((unsigned long long)pos << kIdxShift) | d;
}
__device__ __forceinline__ uint64_t key_pos(unsigned long long key) { return (key >> kIdxShift) & kIdxMask; }
// compress8_test.cpp:156-161: with inversion a window's distance is min(d, M - d) (M - d taken when
// strictly smaller: that window is inverted). The distance field keeps d (13 bits) or, inverted
// mode, min(d, M - d) <= M / 2 <= 2048 in 12 bits and the window's inversion in bit 12 (the field
// is below the scan index: it never decides between keys).
__device__ __forceinline__ unsigned long long win_key(uint32_t d, uint32_t T, uint64_t pos, uint32_t M, uint32_t inv) {
  if (!inv) return make_key(d, T, pos);
  const bool f = M - d < d;
  const uint32_t e = f ? M - d : d;
  return ((unsigned long long)(e <= T ? 0u : e) << kDpShift) | ((unsigned long long)pos << kIdxShift) | e |
         (f ? 0x1000ull : 0ull);
}
__device__ __forceinline__ uint32_t key_dist(unsigned long long key, uint32_t inv) {
  return (uint32_t)(key & (inv ? 0xfffu : 0x1fffu));
}
__device__ __forceinline__ int key_flip(unsigned long long key, uint32_t inv) { return inv ? (int)((key >> 12) & 1) : 0; }
// compress5_test.cpp:94,109,126: a window replaces the best when (d - worstd) > (bestd - worstd) in idx_t
// (worstd = W*W/2, bestd from W*W+1): every d < worstd beats every d >= worstd and the initial value,
// and among those a larger d wins (ties: the earlier window). Two keys per window: the ranking one
// (worstd - 1 - d, never for d >= worstd) and the first window with d < worstd, whose distance decides
// whether the search ends there (the replacements only grow d, so bestd <= T can only hold after the
// first one: if it does not, no window ever ends the search).
constexpr uint32_t kRankNone = 0x1fffu;
__device__ __forceinline__ unsigned long long win_key5(uint32_t d, uint32_t worstd, uint64_t pos) {
  const uint32_t rank = d < worstd ? worstd - 1 - d : kRankNone;
  return ((unsigned long long)rank << kDpShift) | ((unsigned long long)pos << kIdxShift) | d;
}
__device__ __forceinline__ unsigned long long win_key5_first(uint32_t d, uint32_t worstd, uint64_t pos) {
  return ((unsigned long long)(d < worstd ? 0u : 1u) << kDpShift) | ((unsigned long long)pos << kIdxShift) | d;
}
// compress8_test.cpp:137: a tile of weight <= T or >= M - T (idx_t arithmetic) is a "perfect match"
// before any window is searched
__device__ __forceinline__ bool perfect_before(const MatchArgs& a, uint32_t w0) {
  const uint64_t M = (uint64_t)a.W * a.W;
  return a.inv && (w0 <= a.T || (uint64_t)w0 >= M - (uint64_t)a.T);
}

struct Region {
  int i0, j0, mini, minj, maxj, mini2, maxj2;
  int rlo, wlo;                 // first staged row and word column
  uint32_t nrows, stride;       // staged rows; words per staged row (+1 zero word)
  uint32_t n1c, n2c;
  uint64_t n1, n;               // windows of the first loop; of both loops
  int64_t swin;                 // search_win_size (:131)
};

__device__ __forceinline__ Region make_region(const MatchArgs& a, uint32_t t) {
  Region g;
  const int W = (int)a.W, R = a.R, cols = (int)a.cols;
  g.i0 = (int)(t / a.nx) * W;
  g.j0 = (int)(t % a.nx) * W;
  g.mini = g.i0 > R ? g.i0 - R : 0;                               // :125-130
  g.minj = g.j0 > R ? g.j0 - R : 0;
  g.maxj = (g.j0 + R > cols - W) ? cols - W : g.j0 + R;
  g.mini2 = g.i0 > W ? g.i0 - W : 0;
  // compress4/5/6_test.cpp start the first loop at int(j0 - W) (none at j0 = 0; :104 / :105 / :126)
  g.maxj2 = a.var ? g.j0 - W : (g.j0 > W ? g.j0 - W : 0);
  g.swin = (int64_t)(g.i0 - g.mini2) * (g.maxj2 - g.minj) + (int64_t)(g.mini2 - g.mini) * (g.maxj - g.minj);
  const int n1r = g.i0 - g.mini2 + 1, n1c = g.maxj2 - g.minj + 1;
  const int n2r = g.i0 - W - g.mini + 1, n2c = g.maxj - g.minj + 1;
  g.n1c = n1c > 0 ? (uint32_t)n1c : 0;
  g.n2c = n2c > 0 ? (uint32_t)n2c : 0;
  g.n1 = (uint64_t)n1r * g.n1c;
  g.n = g.n1 + (n2r > 0 ? (uint64_t)n2r * g.n2c : 0);
  g.rlo = min(g.mini, g.mini2);
  g.wlo = g.minj >> 6;
  g.nrows = (uint32_t)(g.i0 + W - g.rlo);
  g.stride = (uint32_t)(((g.maxj + W - 1) >> 6) - g.wlo + 2);
  return g;
}

// Loop 1 walks i2 = i0 .. mini2 and j2 = maxj2 .. minj, loop 2 i2 = i0-W .. mini and
// j2 = maxj .. minj (:138-174). Flat scan index -> position (the per-tile schedule splits flat ranges).
__device__ __forceinline__ uint64_t flat_pos(const Region& g, uint32_t idx) {
  if (idx < g.n1) {
    const uint32_t q = idx / g.n1c;
    return scan_pos(0, q, idx - q * g.n1c);
  }
  idx -= (uint32_t)g.n1;
  const uint32_t q = idx / g.n2c;
  return scan_pos(1, q, idx - q * g.n2c);
}
__device__ __forceinline__ void pos_window(const Region& g, int W, uint64_t pos, int& i2, int& j2) {
  const int a = (int)((pos >> 16) & 0xffff), c = (int)(pos & 0xffff);
  if (pos >> 32) {
    i2 = g.i0 - W - a;
    j2 = g.maxj - c;
  } else {
    i2 = g.i0 - a;
    j2 = g.maxj2 - c;
  }
}

// Cross-workgroup hand-offs without cache maintenance. An agent-scope release / acquire costs an L2
// write-back (buffer_wbl2) / invalidation (buffer_inv) of the whole XCD per hand-off -- microseconds,
// and under the feet of every other workgroup on it. Instead everything one workgroup writes for
// another (image words, flags, progress) is stored with agent-scope atomic stores, which go to the
// coherence point (sc1), and read with agent-scope atomic loads, which do not hit stale lines; a
// producer waits for its stores to be acknowledged (s_waitcnt vmcnt(0)) before it raises a flag, and
// a consumer issues its data loads only after it has seen the flag.
__device__ __forceinline__ uint32_t ld_relaxed(const uint32_t* p) {
  return __hip_atomic_load(p, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}
__device__ __forceinline__ uint64_t ld_word(const uint64_t* p) {
  return __hip_atomic_load(p, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}
__device__ __forceinline__ void st_word(uint64_t* p, uint64_t v) {
  __hip_atomic_store(p, v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}
__device__ __forceinline__ void stores_done() { __builtin_amdgcn_s_waitcnt(0); }
__device__ __forceinline__ void raise_flag(uint32_t* p, uint32_t v) {
  __hip_atomic_store(p, v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}

// W bits of row `row` from column `col`, MSB-aligned, from the LDS image or the plane
template <bool LDS>
__device__ __forceinline__ uint64_t row_bits(const MatchArgs& a, const Region& g, const uint64_t* S, int row,
                                             int col) {
  if constexpr (LDS) {
    const uint32_t c = (uint32_t)(col - g.wlo * 64), w = c >> 6, sh = c & 63;
    const uint64_t* p = S + (uint32_t)(row - g.rlo) * g.stride + w;
    return (p[0] << sh) | ((p[1] >> 1) >> (63 - sh));
  } else {
    const uint32_t w = (uint32_t)col >> 6, sh = (uint32_t)col & 63;
    const uint64_t* p = a.I + (uint64_t)row * a.wpr + w;
    const uint64_t hi = ld_word(p);
    const uint64_t lo = (sh && w + 1 < a.used) ? ld_word(p + 1) : 0;
    return (hi << sh) | ((lo >> 1) >> (63 - sh));
  }
}


// The tile's decision (:184-272), one lane per tile row r (lanes r >= W pass p = b = 0): p = tile
// row, b = row of the best window (0 when the region is empty), both MSB-aligned W bits. Writes the
// per-tile outputs and returns the row of the residual that is written back.
// flip: the best window's inversion, -1 without a window (compress8: bestinv then stays
// (P.weight() - M) < P.weight(), :136: the tile is all 1s); always -1 / ignored without inversion.
__device__ uint64_t decide_tile(const MatchArgs& a, const double* enuml, const Region& g, uint32_t t, int bi,
                                int bj, uint32_t bd, int flip, uint64_t p, uint64_t b, int r) {
  const int W = (int)a.W;
  const uint64_t topW = W >= 64 ? ~0ull : ~(~0ull >> W);
  if (a.var) {  // compress4_test.cpp:143-168, compress5_test.cpp:144-169, compress6_test.cpp:166-207
    const uint32_t M = (uint32_t)(W * W);
    const uint64_t p3 = p ^ b;  // (b = 0 without a window: compress6's P3 = P)
    const uint32_t s0 = wave_total_u32((uint32_t)__popcll(p) | (uint32_t)__popcll(p3) << 16);
    const uint32_t wP = s0 & 0xffff, w3 = s0 >> 16;
    // ceil(log2(li)) of the tile's raster index: li = 0 gives -inf, 2^63 as idx_t on x86-64
    const uint64_t idx_len = t == 0 ? (1ull << 63) : t == 1 ? 0 : 64 - (uint64_t)__clzll((unsigned long long)(t - 1));
    const uint64_t nomatch_len = (uint64_t)(1.0 + enuml[wP]);
    uint64_t match_len;
    uint32_t mw;
    if (a.var == 6) {
      match_len = (uint64_t)((double)(1 + idx_len) + enuml[w3]);
      mw = w3;
    } else {
      match_len = bd <= M ? (uint64_t)((double)(1 + idx_len) + enuml[bd]) : 100000;
      mw = bd;
    }
    const bool take = nomatch_len > match_len;
    if (r == 0) {
      a.besti[t] = (uint32_t)bi;
      a.bestj[t] = (uint32_t)bj;
      a.bestd[t] = bd;
      a.weights[t] = take ? mw : wP;
      a.lens[t] = (uint32_t)(take ? match_len : nomatch_len);
      a.modes[t] = take ? 'x' : 'o';
    }
    return take ? p3 : p;  // (the tile is written back unchanged without a match)
  }
  bool inv = false;
  if (a.inv) {  // compress8_test.cpp:136, :163, :207-210
    inv = flip >= 0 ? flip != 0 : wave_total_u32((uint32_t)__popcll(p)) == (uint32_t)(W * W);
    if (inv && r < W) p = ~p & topW;
  }
  const uint64_t p3 = p ^ b;
  // med inside the tile (compress7_test.cpp:43-55; (0,0) is never written: 0 here)
  const uint64_t pu = wave_shr1_u64(p), p3u = wave_shr1_u64(p3);  // the row above (0 for row 0)
  const uint64_t D = p ^ pu, D3 = p3 ^ p3u;
  const uint64_t lane_mask = r < W ? topW & (r == 0 ? ~BIC_MSB : ~0ull) : 0ull;
  const uint64_t dp = (D ^ (D >> 1)) & lane_mask, dp3 = (D3 ^ (D3 >> 1)) & lane_mask;
  // the four weights in 16-bit fields (each <= 64 * 64), two DPP reductions
  const uint32_t s0 = wave_total_u32((uint32_t)__popcll(p) | (uint32_t)__popcll(p3) << 16);
  const uint32_t s1 = wave_total_u32((uint32_t)__popcll(dp) | (uint32_t)__popcll(dp3) << 16);
  const uint32_t w_nn = s0 & 0xffff, w_mn = s0 >> 16, w_np = s1 & 0xffff, w_mp = s1 >> 16;
  // lengths (:212-221) in double, converted to idx_t like the driver
  const uint64_t nn_len = (uint64_t)(2.0 + enuml[w_nn]), np_len = (uint64_t)(2.0 + enuml[w_np]);
  uint64_t mn_len = ~0ull, mp_len = ~0ull;  // search_win_size <= 0: log2 -> 2^63, never a match
  if (g.swin >= 1) {
    const uint64_t idx_len = g.swin == 1 ? 0 : 64 - (uint64_t)__clzll((unsigned long long)(g.swin - 1));
    const uint64_t fixed = a.inv ? 3 : 2;  // compress8_test.cpp:250-251: one more bit (invert / not)
    mn_len = (uint64_t)((double)(fixed + idx_len) + enuml[w_mn]);
    mp_len = (uint64_t)((double)(fixed + idx_len) + enuml[w_mp]);
  }
  const bool mpred = mn_len > mp_len, npred = nn_len > np_len;  // :232, :243
  const uint64_t match_len = mpred ? mp_len : mn_len, nomatch_len = npred ? np_len : nn_len;
  const bool take = nomatch_len > match_len;                   // :255
  if (r == 0) {
    a.besti[t] = (uint32_t)bi;
    a.bestj[t] = (uint32_t)bj;
    a.bestd[t] = bd;
    a.weights[t] = take ? (mpred ? w_mp : w_mn) : (npred ? w_np : w_nn);
    a.lens[t] = (uint32_t)(take ? match_len : nomatch_len);
    a.modes[t] = take ? (mpred ? 'X' : 'x') : (npred ? 'O' : 'o');
    if (a.inverted) a.inverted[t] = inv ? 1 : 0;
  }
  return take ? (mpred ? dp3 : p3) : (npred ? dp : p);
}

template <bool LDS>
__device__ void match_tile(const MatchArgs& a, const Region& g, uint32_t t, uint32_t part, uint64_t* S,
                           uint64_t* Pl) {
  __shared__ unsigned long long red[kMB / 64], redA[kMB / 64];
  __shared__ int sh_last;
  const int W = (int)a.W;
  const uint32_t tid = threadIdx.x;
  const uint64_t topW = W >= 64 ? ~0ull : ~(~0ull >> W);

  if constexpr (LDS) {
    const uint32_t nw = g.nrows * g.stride;
    for (uint32_t e = tid; e < nw; e += kMB) {
      const uint32_t r = e / g.stride, c = e - r * g.stride;
      const uint32_t wc = (uint32_t)g.wlo + c;
      S[e] = (c + 1 < g.stride && wc < a.used) ? ld_word(a.I + (uint64_t)(g.rlo + (int)r) * a.wpr + wc) : 0ull;
    }
    __syncthreads();
  }
  if (tid < (uint32_t)W) Pl[tid] = row_bits<LDS>(a, g, S, g.i0 + (int)tid, g.j0) & topW;
  __syncthreads();
  bool skip = false;
  if (a.inv) {  // compress8_test.cpp:137: no search at all for a nearly empty / full tile
    uint32_t w0 = 0;
    for (int r = 0; r < W; ++r) w0 += (uint32_t)__popcll(Pl[r]);
    skip = perfect_before(a, w0);
  }
  const uint32_t M = (uint32_t)(W * W);
  const bool v5 = a.var == 5;
  const uint32_t worstd = M / 2;

  // this part's share of the scan, in chunks; a window at distance <= T ends the search (variant 5:
  // every window is scanned and the first-window rule applied by the tile's finish)
  const uint64_t lo = part * g.n / a.G, hi = skip ? lo : (part + 1) * g.n / a.G;
  unsigned long long best = ~0ull, bestA = ~0ull;
  uint32_t chunk = 0;
  for (uint64_t base = lo; base < hi; base += kChunk, ++chunk) {
#pragma unroll
    for (int q = 0; q < kPerThread; ++q) {
      const uint64_t idx = base + (uint32_t)q * kMB + tid;
      if (idx < hi) {
        int i2, j2;
        const uint64_t pos = flat_pos(g, (uint32_t)idx);
        pos_window(g, W, pos, i2, j2);
        uint32_t d = 0;
        for (int r = 0; r < W; ++r) d += (uint32_t)__popcll((row_bits<LDS>(a, g, S, i2 + r, j2) ^ Pl[r]) & topW);
        if (v5) {
          const unsigned long long ka = win_key5_first(d, worstd, pos), kb = win_key5(d, worstd, pos);
          bestA = ka < bestA ? ka : bestA;
          best = kb < best ? kb : best;
        } else {
          const unsigned long long key = win_key(d, a.T, pos, M, a.inv);
          best = key < best ? key : best;
        }
      }
    }
    int stop = !v5 && (best >> kDpShift) == 0;
    if (!v5 && (chunk & 7) == 7 && tid == 0 && !stop) {  // a lower part already found one
      const unsigned long long k = __hip_atomic_load(&a.key[t], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      stop = (k >> kDpShift) == 0 && key_pos(k) < flat_pos(g, (uint32_t)base);
    }
    if (__syncthreads_or(stop)) break;
  }
  best = wave_min_u64(best);
  if (lane_id() == 0) red[tid >> 6] = best;
  if (v5) {
    bestA = wave_min_u64(bestA);
    if (lane_id() == 0) redA[tid >> 6] = bestA;
  }
  __syncthreads();
  if (tid == 0) {
    for (int w = 1; w < kMB / 64; ++w) best = red[w] < best ? red[w] : best;
    best = red[0] < best ? red[0] : best;
    if (best != ~0ull) atomicMin(&a.key[t], best);
    if (v5) {
      for (int w = 0; w < kMB / 64; ++w) bestA = redA[w] < bestA ? redA[w] : bestA;
      if (bestA != ~0ull) atomicMin(&a.key2[t], bestA);
    }
    stores_done();
    const uint32_t old = atomicAdd(&a.arrive[t], 1u);
    sh_last = old + 1 == a.G;
  }
  __syncthreads();
  if (!sh_last || tid >= 64) return;

  // ---- the last workgroup finishes the tile (one lane per tile row) ----
  unsigned long long key = __hip_atomic_load(&a.key[t], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  if (v5) {  // compress5_test.cpp:104-136 (see win_key5)
    const unsigned long long kA = __hip_atomic_load(&a.key2[t], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    const bool firstA = kA != ~0ull && (kA >> kDpShift) == 0;  // some window with d < worstd
    unsigned long long ch = ~0ull;
    if (a.T > M) {  // bestd <= T after the first window: it alone decides (replacing W*W+1 or not)
      if (firstA && key_pos(kA) == flat_pos(g, 0)) ch = kA;
    } else if (firstA && key_dist(kA, 0) <= a.T) {
      ch = kA;
    } else if (key != ~0ull && (key >> kDpShift) != kRankNone) {
      ch = key;
    }
    key = ch;
  }
  const int r = (int)tid;
  uint32_t bd = M + 1;
  int bi = 0, bj = 0, flip = -1;
  if (key != ~0ull) {  // :184-189 (any window at all beats M + 1)
    bd = key_dist(key, a.inv);
    flip = key_flip(key, a.inv);
    pos_window(g, W, key_pos(key), bi, bj);
  }
  const uint64_t p = r < W ? Pl[r] : 0ull;
  const uint64_t b = (key != ~0ull && r < W) ? (row_bits<LDS>(a, g, S, bi + r, bj) & topW) : 0ull;
  const uint64_t res = decide_tile(a, a.enuml, g, t, bi, bj, bd, flip, p, b, r);
  // residual write-back (:266 / :272): W bits at (i0 + r, j0), one or two words
  if (r < W) {
    uint64_t* row = a.I + (uint64_t)(g.i0 + r) * a.wpr + (g.j0 >> 6);
    const uint32_t sh = (uint32_t)g.j0 & 63;
    st_word(row, (ld_word(row) & ~(topW >> sh)) | (res >> sh));
    if (sh + (uint32_t)W > 64) st_word(row + 1, (ld_word(row + 1) & ~(topW << (64 - sh))) | (res << (64 - sh)));
  }
  stores_done();
  if (r == 0) raise_flag(&a.done[t], 1u);
}

__global__ __launch_bounds__(kMB) void k_match_tiles(MatchArgs a) {
  __shared__ uint64_t S[kRegionWords];
  __shared__ uint64_t Pl[64];
  __shared__ uint32_t sh_q;
  if (threadIdx.x == 0) {
    const uint32_t q = atomicAdd(a.counter, 1u);
    sh_q = q;
    const uint32_t t = q / a.G;
    // predecessors: (i, j-1) and (i-1, jd)
    const Region g = make_region(a, t);
    const uint32_t ti = t / a.nx, tj = t % a.nx;
    uint32_t dep[2];
    int nd = 0;
    if (tj > 0) dep[nd++] = t - 1;
    if (ti > 0) {
      uint32_t jd = (uint32_t)(g.maxj + (int)a.W - 1) / a.W;
      if (jd >= a.nx) jd = a.nx - 1;
      dep[nd++] = (ti - 1) * a.nx + jd;
    }
    for (int k = 0; k < nd; ++k) {
      uint32_t spins = 0;
      while (ld_relaxed(&a.done[dep[k]]) == 0) {
        __builtin_amdgcn_s_sleep(2);
        if (++spins > (1u << 24)) {  // ~seconds: a predecessor never finished
          atomicOr(&a.flags[2], 1u);
          break;
        }
      }
    }
  }
  __syncthreads();
  const uint32_t t = sh_q / a.G, part = sh_q % a.G;
  const Region g = make_region(a, t);
  if (g.nrows * g.stride <= kRegionWords)
    match_tile<true>(a, g, t, part, S, Pl);
  else
    match_tile<false>(a, g, t, part, S, Pl);
}

// ---- one workgroup per tile row ----------------------------------------------------------
// The row's tiles run in order inside one 1024-thread workgroup, so the dependency on the tile to
// the left never leaves the CU; only the one on the row above crosses workgroups (a progress
// counter per tile row, polled once per tile). The band of rows a tile row searches -- R rows
// above it and its own W rows -- is kept in LDS at full width as 32-bit words (MSB = leftmost
// pixel, one spare zero word per row): the row's own band is loaded once and updated by its own
// write-backs; the rows above are (re)loaded column by column as the row above completes them.
constexpr int kRB = 1024;
constexpr uint32_t kRowLds = 30 * 1024;  // u32 words of the band image (120 KiB)

struct Band {
  int i0, lo;            // first tile row pixel, first band row
  uint32_t nr, pitch;    // band rows, u32 words per LDS row
};

__device__ __forceinline__ uint32_t band_word(const uint32_t* L, const Band& b, int row, uint32_t w) {
  return L[(uint32_t)(row - b.lo) * b.pitch + w];
}

// 64 bits of band row `row` from column `col`, MSB-aligned (reads three words; the pitch keeps
// two zero words past the last column)
__device__ __forceinline__ uint64_t band_bits64(const uint32_t* L, const Band& b, int row, int col) {
  const uint32_t* q = L + (uint32_t)(row - b.lo) * b.pitch + ((uint32_t)col >> 5);
  const uint32_t sh = (uint32_t)col & 31;
  const uint64_t x = ((uint64_t)q[0] << 32) | q[1];
  return (x << sh) | (((uint64_t)q[2] << sh) >> 32);
}

// KW bits (KW <= 32) of band row `row` from column `col`, in the low bits
template <int KW>
__device__ __forceinline__ uint32_t band_bits(const uint32_t* L, const Band& b, int row, int col) {
  const uint32_t* q = L + (uint32_t)(row - b.lo) * b.pitch + ((uint32_t)col >> 5);
  const uint64_t x = ((uint64_t)q[0] << 32) | q[1];
  const uint32_t v = (uint32_t)(x >> (64 - KW - ((uint32_t)col & 31)));
  return KW == 32 ? v : v & ((1u << KW) - 1u);
}

// load columns [w0, w1) (u32 words) of band rows [r0, r1) from the plane
__device__ __forceinline__ void band_load(uint32_t* L, const Band& b, const MatchArgs& a, int r0, int r1,
                                          uint32_t w0, uint32_t w1) {
  if (r1 <= r0 || w1 <= w0) return;
  const uint32_t nw = w1 - w0, n = (uint32_t)(r1 - r0) * nw;
  const uint32_t* I32 = reinterpret_cast<const uint32_t*>(a.I);  // other workgroups' stores: atomic loads
  for (uint32_t e = threadIdx.x; e < n; e += kRB) {
    const uint32_t rr = e / nw, w = w0 + (e - rr * nw);
    const int row = r0 + (int)rr;
    // u32 column w is the high (even w) or low half of u64 word w/2 (little-endian in memory)
    L[(uint32_t)(row - b.lo) * b.pitch + w] =
        ld_relaxed(I32 + ((uint64_t)row * a.wpr + (w >> 1)) * 2 + ((w & 1) ^ 1));
  }
}

// Tasks [t0, t1) of one search loop of the reference (i2 = i_top - a for a < nrows, j2 = j_top - c for
// c < ncols, position scan_pos(loop, a, c)). Task t = (g, c) = (t / ncols, t % ncols) covers
// the kGK windows a = g*kGK .. g*kGK+kGK-1 down one column, whose kGK + KW - 1 rows are extracted once
// into registers. Tasks with g*kGK < skip_a and c < skip_c are left out (another workgroup's share).
// Chunks of kRB tasks; the scan stops once the best key has distance <= T and a scan index below
// every window left (every window a later call of this workgroup scans has a larger index).
template <int KW, int kGK>
__device__ __forceinline__ void scan_tasks(const uint32_t* L, const Band& bd, const uint32_t* PW, uint32_t T,
                                           uint32_t inv, int i_top, uint32_t nrows, int j_top, uint32_t ncols,
                                           uint32_t loop, uint32_t t0, uint32_t t1, uint32_t skip_a, uint32_t skip_c,
                                           unsigned long long& best, bool& stop) {
  // 32/KW consecutive rows of KW bits share one 32-bit word, so a window's distance is KW/(32/KW)
  // xor + popcount pairs (PW: the tile's rows packed the same way)
  constexpr int kPack = 32 / KW, kNW = KW / kPack, kNE = kGK + KW - 1, kNP = kNE - kPack + 1;
  if (stop || t1 <= t0 || ncols == 0) return;
  constexpr bool kHoist = kNW <= 8;  // packed tile rows in registers, else read from LDS (broadcast)
  uint32_t Pr[kHoist ? kNW : 1];
  if constexpr (kHoist) {
#pragma unroll
    for (int r = 0; r < kNW; ++r) Pr[r] = PW[r];
  }
  for (uint32_t base = t0; base < t1; base += kRB) {
    const uint32_t task = base + threadIdx.x;
    if (task < t1) {
      const uint32_t g = task / ncols, c = task - g * ncols;
      const uint32_t a0 = g * kGK;
      if (!(a0 < skip_a && c < skip_c)) {
        const int j2 = j_top - (int)c;
        const uint32_t kk = min((uint32_t)kGK, nrows - a0);
        const int ybase = i_top - (int)a0 - (kGK - 1);  // band row of e[0]
        uint32_t e[kNE];
#pragma unroll
        for (int m = 0; m < kNE; ++m) {
          const int y = ybase + m;
          e[m] = y >= bd.lo ? band_bits<KW>(L, bd, y, j2) : 0u;
        }
        uint32_t pk[kNP];
#pragma unroll
        for (int m = 0; m < kNP; ++m) {
          uint32_t v = 0;
#pragma unroll
          for (int q = 0; q < kPack; ++q) v |= e[m + q] << (32 - KW * (q + 1));
          pk[m] = v;
        }
#pragma unroll
        for (int u = 0; u < kGK; ++u) {
          if ((uint32_t)u < kk) {
            uint32_t d = 0;
#pragma unroll
            for (int r = 0; r < kNW; ++r)
              d += (uint32_t)__popc(pk[kGK - 1 - u + r * kPack] ^ (kHoist ? Pr[kHoist ? r : 0] : PW[r]));
            const unsigned long long key = win_key(d, T, scan_pos(loop, a0 + (uint32_t)u, c), KW * KW, inv);
            best = key < best ? key : best;
          }
        }
      }
    }
    const uint32_t nt = base + kRB;
    bool s = (best >> kDpShift) == 0;
    if (s && nt < t1) {  // the first task left bounds the index of every window left
      const uint32_t g2 = nt / ncols, c2 = nt - g2 * ncols;
      s = key_pos(best) < scan_pos(loop, g2 * kGK, c2);
    }
    if (__syncthreads_or(s)) {
      stop = true;
      return;
    }
  }
}

// any W <= 64: one window per task
__device__ __forceinline__ void scan_loop_any(const uint32_t* L, const Band& bd, const uint64_t* P, int W,
                                              int i_top, uint32_t nrows, int j_top, uint32_t ncols, uint32_t loop,
                                              uint32_t T, uint32_t inv, unsigned long long& best, bool& stop) {
  if (stop || nrows == 0 || ncols == 0) return;
  const uint64_t topW = W >= 64 ? ~0ull : ~(~0ull >> W);
  const uint32_t n = nrows * ncols;
  for (uint32_t base = 0; base < n; base += kRB) {
    const uint32_t i = base + threadIdx.x;
    if (i < n) {
      const uint32_t q = i / ncols;
      const int i2 = i_top - (int)q, j2 = j_top - (int)(i - q * ncols);
      uint32_t d = 0;
      for (int r = 0; r < W; ++r) d += (uint32_t)__popcll((band_bits64(L, bd, i2 + r, j2) ^ P[r]) & topW);
      const unsigned long long key = win_key(d, T, scan_pos(loop, q, i - q * ncols), (uint32_t)(W * W), inv);
      best = key < best ? key : best;
    }
    const uint32_t nt = base + kRB;
    const bool s = (best >> kDpShift) == 0 && (nt >= n || key_pos(best) < scan_pos(loop, nt / ncols, nt % ncols));
    if (__syncthreads_or(s)) {
      stop = true;
      return;
    }
  }
}

__global__ __launch_bounds__(kRB) void k_match_rows(MatchArgs a, uint32_t* progress) {
  __shared__ uint32_t L[kRowLds];
  __shared__ uint64_t P64[64];
  __shared__ unsigned long long red[kRB / 64];
  __shared__ uint32_t sh_row;
  const int W = (int)a.W;
  const uint32_t tid = threadIdx.x;
  const uint64_t topW = W >= 64 ? ~0ull : ~(~0ull >> W);
  if (tid == 0) sh_row = atomicAdd(a.counter, 1u);
  __syncthreads();
  const uint32_t ti = sh_row;
  Band bd;
  bd.i0 = (int)ti * W;
  {
    const int mini = bd.i0 > a.R ? bd.i0 - a.R : 0, mini2 = bd.i0 > W ? bd.i0 - W : 0;
    bd.lo = min(mini, mini2);
  }
  bd.nr = (uint32_t)(bd.i0 + W - bd.lo);
  bd.pitch = (a.cols + 31) / 32 + 2;
  const uint32_t used32 = (a.cols + 31) / 32;
  // the row's own band (original pixels: nothing else writes it), pad words zero
  for (uint32_t e = tid; e < bd.nr * bd.pitch; e += kRB) L[e] = 0;
  __syncthreads();
  band_load(L, bd, a, bd.i0, bd.i0 + W, 0, used32);
  int final_col = -1;  // the rows above are loaded and final up to this column
  for (uint32_t tj = 0; tj < a.nx; ++tj) {
    const uint32_t t = ti * a.nx + tj;
    const Region g = make_region(a, t);
    // the row above must have finished every tile the region reads (tile (i-1, jd))
    const int cmax = g.maxj + W - 1;
    if (ti > 0 && cmax > final_col) {
      if (tid == 0) {
        uint32_t jd = (uint32_t)(g.maxj + W - 1) / (uint32_t)W;
        if (jd >= a.nx) jd = a.nx - 1;
        uint32_t spins = 0;
        while (__hip_atomic_load(&progress[ti - 1], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) < jd + 1) {
          __builtin_amdgcn_s_sleep(1);
          if (++spins > (1u << 24)) {
            atomicOr(&a.flags[2], 1u);
            break;
          }
        }
      }
      __syncthreads();
      // the word holding column final_col + 1 may have been loaded before it was final: reload it
      band_load(L, bd, a, bd.lo, bd.i0, (uint32_t)(final_col + 1) >> 5, ((uint32_t)cmax >> 5) + 1);
      final_col = cmax;
    }
    __syncthreads();
    if (tid < (uint32_t)W) {
      const uint64_t pr = band_bits64(L, bd, bd.i0 + (int)tid, g.j0) & topW;
      P64[tid] = pr;
    }
    __syncthreads();
    unsigned long long best = ~0ull;
    bool stop = false;
    if (a.inv) {  // compress8_test.cpp:137
      uint32_t w0 = 0;
      for (int r = 0; r < W; ++r) w0 += (uint32_t)__popcll(P64[r]);
      stop = perfect_before(a, w0);
    }
    // loop 1: i2 = i0 .. mini2, j2 = maxj2 .. minj; loop 2: i2 = i0-W .. mini, j2 = maxj .. minj
    const uint32_t n1r = (uint32_t)(g.i0 - g.mini2 + 1);
    const int n2r_ = g.i0 - W - g.mini + 1;
    const uint32_t n2r = n2r_ > 0 ? (uint32_t)n2r_ : 0;
    scan_loop_any(L, bd, P64, W, g.i0, n1r, g.maxj2, g.n1c, 0, a.T, a.inv, best, stop);
    scan_loop_any(L, bd, P64, W, g.i0 - W, n2r, g.maxj, g.n2c, 1, a.T, a.inv, best, stop);
    best = wave_min_u64(best);
    if (lane_id() == 0) red[tid >> 6] = best;
    __syncthreads();
    if (tid < 64) {
      unsigned long long key = red[0];
      for (int w = 1; w < kRB / 64; ++w) key = red[w] < key ? red[w] : key;
      const int r = (int)tid;
      uint32_t bdist = (uint32_t)(W * W) + 1;
      int bi = 0, bj = 0, flip = -1;
      if (key != ~0ull) {
        bdist = key_dist(key, a.inv);
        flip = key_flip(key, a.inv);
        pos_window(g, W, key_pos(key), bi, bj);
      }
      const uint64_t p = r < W ? P64[r] : 0ull;
      const uint64_t b = (key != ~0ull && r < W) ? (band_bits64(L, bd, bi + r, bj) & topW) : 0ull;
      const uint64_t res = decide_tile(a, a.enuml, g, t, bi, bj, bdist, flip, p, b, r);
      if (r < W) {
        // write-back: the plane (for the rows below) and the band image (for the tiles to the right)
        uint64_t* row = a.I + (uint64_t)(g.i0 + r) * a.wpr + (g.j0 >> 6);
        const uint32_t sh = (uint32_t)g.j0 & 63;
        st_word(row, (ld_word(row) & ~(topW >> sh)) | (res >> sh));
        if (sh + (uint32_t)W > 64) st_word(row + 1, (ld_word(row + 1) & ~(topW << (64 - sh))) | (res << (64 - sh)));
        uint32_t* q = L + (uint32_t)(g.i0 + r - bd.lo) * bd.pitch + ((uint32_t)g.j0 >> 5);
        const int s32 = g.j0 & 31;
#pragma unroll
        for (int k = 0; k < 3; ++k) {
          const int off = 32 * k - s32;  // column of word k relative to j0
          if (off >= W) break;
          const uint64_t part_v = off >= 0 ? res << off : res >> -off;
          const uint64_t part_m = off >= 0 ? topW << off : topW >> -off;
          const uint32_t v = (uint32_t)(part_v >> 32), m = (uint32_t)(part_m >> 32);
          q[k] = (q[k] & ~m) | v;
        }
      }
      stores_done();
      if (r == 0) raise_flag(&progress[ti], tj + 1);
    }
    __syncthreads();
  }
}

// ---- a team of workgroups per tile row --------------------------------------------------------
// One main workgroup walks the row's tiles as above; H helper workgroups search, ahead of it, every
// window of tile j that does not overlap the K tiles to its left (loop 1 windows with a >= W or
// c >= K*W, and all of loop 2), each a contiguous share of those tasks, once the main has finished
// tile j-K-1. Their best keys land in slots[t * H + h] (bit 63 = written). The main searches only
// the K*W x W windows over the recent tiles, combines the keys -- without waiting when its own
// key already has distance <= T below every helper window's scan index -- and decides the tile
// from LDS: the length table and the band image are both there, and the write-back goes to the
// plane from the band image without reading it. It publishes its progress one tile late, after
// the stores of the previous tile had the search time to land.
constexpr unsigned long long kSlotSet = 1ull << 63;

template <int KW>
__global__ __launch_bounds__(kRB) void k_match_team(MatchArgs a, uint32_t* progress, unsigned long long* slots) {
  constexpr int W = KW;
  constexpr int kGK = 4;  // windows per helper task
  constexpr uint64_t topW = ~(~0ull >> W);
  __shared__ uint32_t L[kRowLds];
  __shared__ double E[KW * KW + 1];
  __shared__ uint64_t P64[KW];
  __shared__ uint32_t P32[KW];
  __shared__ uint32_t PW[KW];
  __shared__ unsigned long long red[kRB / 64];
  __shared__ uint32_t sh_q;
  const uint32_t tid = threadIdx.x, H = a.H, KWc = a.K * W;
  if (tid == 0) sh_q = atomicAdd(a.counter, 1u);
  __syncthreads();
  const uint32_t ti = sh_q / (H + 1), role = sh_q % (H + 1);
  Band bd;
  bd.i0 = (int)ti * W;
  {
    const int mini = bd.i0 > a.R ? bd.i0 - a.R : 0, mini2 = bd.i0 > W ? bd.i0 - W : 0;
    bd.lo = min(mini, mini2);
  }
  bd.nr = (uint32_t)(bd.i0 + W - bd.lo);
  bd.pitch = (a.cols + 31) / 32 + 2;
  const uint32_t used32 = (a.cols + 31) / 32;
  for (uint32_t e = tid; e < bd.nr * bd.pitch; e += kRB) L[e] = 0;
  if (role == 0)
    for (uint32_t e = tid; e <= (uint32_t)(W * W); e += kRB) E[e] = a.enuml[e];
  __syncthreads();
  band_load(L, bd, a, bd.i0, bd.i0 + W, 0, used32);  // the row's own band, original pixels
  int final_col = -1;   // rows above: loaded and final up to this column
  int final_band = -1;  // helpers: the row's own band holds the main's residuals up to this column
  for (uint32_t tj = 0; tj < a.nx; ++tj) {
    const uint32_t t = ti * a.nx + tj;
    const Region g = make_region(a, t);
    const int cmax = g.maxj + W - 1;
    if (role == 0 && tid == 0) MSTAMP(t, 0);
    const bool need_above = ti > 0 && cmax > final_col;
    const uint32_t need_main = (role > 0 && tj > a.K) ? tj - a.K : 0;  // tiles the main must have done
    const int cb = (int)need_main * W - 1;
    const bool need_band = role > 0 && cb > final_band;
    if (need_above || need_band) {
      if (tid == 0) {
        uint32_t spins = 0;
        if (need_above) {
          uint32_t jd = (uint32_t)cmax / (uint32_t)W;
          if (jd >= a.nx) jd = a.nx - 1;
          while (__hip_atomic_load(&progress[ti - 1], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) < jd + 1) {
            __builtin_amdgcn_s_sleep(1);
            if (++spins > (1u << 24)) {
              atomicOr(&a.flags[2], 1u);
              break;
            }
          }
        }
        if (need_band) {
          while (__hip_atomic_load(&progress[ti], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) < need_main) {
            __builtin_amdgcn_s_sleep(1);
            if (++spins > (1u << 24)) {
              atomicOr(&a.flags[2], 1u);
              break;
            }
          }
        }
      }
      __syncthreads();
      if (need_above) {
        band_load(L, bd, a, bd.lo, bd.i0, (uint32_t)(final_col + 1) >> 5, ((uint32_t)cmax >> 5) + 1);
        final_col = cmax;
      }
      if (need_band) {
        band_load(L, bd, a, bd.i0, bd.i0 + W, (uint32_t)(final_band + 1) >> 5, ((uint32_t)cb >> 5) + 1);
        final_band = cb;
      }
    }
    __syncthreads();
    if (role == 0 && tid == 0) MSTAMP(t, 1);
    if (tid < (uint32_t)W) {
      const uint64_t pr = band_bits64(L, bd, bd.i0 + (int)tid, g.j0) & topW;
      P64[tid] = pr;
      P32[tid] = (uint32_t)(pr >> 32);  // rows packed 32/W per word, first row at the top
    }
    __syncthreads();
    if (tid < (uint32_t)(W * W / 32)) {
      uint32_t v = 0;
#pragma unroll
      for (int q = 0; q < 32 / W; ++q) v |= P32[tid * (32 / W) + q] >> (W * q);
      PW[tid] = v;
    }
    __syncthreads();
    if (role == 0 && tid == 0) MSTAMP(t, 2);
    if (role == 0 && tid < 64 && tj > 0) {  // publish the previous tile
      stores_done();
      if (tid == 0) raise_flag(&progress[ti], tj);
    }
    if (role == 0 && tid == 0) MSTAMP(t, 3);
    unsigned long long best = ~0ull;
    bool stop = false;
    if (a.inv) {  // compress8_test.cpp:137 (main and helpers alike: no window is searched)
      uint32_t w0 = 0;
#pragma unroll
      for (int r = 0; r < W; ++r) w0 += (uint32_t)__popcll(P64[r]);
      stop = perfect_before(a, w0);
    }
    const uint32_t n1r = (uint32_t)(g.i0 - g.mini2 + 1);
    const int n2r_ = g.i0 - W - g.mini + 1;
    const uint32_t n2r = n2r_ > 0 ? (uint32_t)n2r_ : 0;
    const uint32_t N1 = (n1r + kGK - 1) / kGK * g.n1c, N2 = (n2r + kGK - 1) / kGK * g.n2c;
    if (role == 0) {
      if (H == 0) {
        scan_tasks<KW, kGK>(L, bd, PW, a.T, a.inv, g.i0, n1r, g.maxj2, g.n1c, 0, 0, N1, 0, 0, best, stop);
        scan_tasks<KW, kGK>(L, bd, PW, a.T, a.inv, g.i0 - W, n2r, g.maxj, g.n2c, 1, 0, N2, 0, 0, best, stop);
      } else {  // the windows over the K tiles to the left (loop 1, a < W, c < K*W), one per thread
        const uint32_t fa = min(n1r, (uint32_t)W), fc = min(g.n1c, KWc);
        if (tid == 0) MSTAMP(t, 8);
        scan_tasks<KW, 4>(L, bd, PW, a.T, a.inv, g.i0, fa, g.maxj2, fc, 0, 0, (fa + 3) / 4 * fc, 0, 0, best, stop);
        if (tid == 0) MSTAMP(t, 9);
      }
    } else {
      const uint32_t h = role - 1, N = N1 + N2;
      const uint32_t lo = (uint32_t)((uint64_t)h * N / H), hi = (uint32_t)((uint64_t)(h + 1) * N / H);
      scan_tasks<KW, kGK>(L, bd, PW, a.T, a.inv, g.i0, n1r, g.maxj2, g.n1c, 0, lo, min(hi, N1), W, KWc, best, stop);
      scan_tasks<KW, kGK>(L, bd, PW, a.T, a.inv, g.i0 - W, n2r, g.maxj, g.n2c, 1, max(lo, N1) - N1,
                          hi > N1 ? hi - N1 : 0, 0, 0, best, stop);
    }
    best = wave_min_u64(best);
    if (role == 0 && tid == 0) MSTAMP(t, 10);
    if (lane_id() == 0) red[tid >> 6] = best;
    __syncthreads();
    if (role == 0 && tid == 0) MSTAMP(t, 4);
    if (tid < 64) {
      unsigned long long key = red[0];
      for (int w = 1; w < kRB / 64; ++w) key = red[w] < key ? red[w] : key;
      if (role > 0) {
        if (tid == 0)
          __hip_atomic_store(&slots[(uint64_t)t * H + (role - 1)], key | kSlotSet, __ATOMIC_RELAXED,
                             __HIP_MEMORY_SCOPE_AGENT);
      } else {
        const int r = (int)tid;
        // the helpers' windows start at (loop 1, a = 0, c = K*W), (loop 1, a = W) or loop 2
        const uint64_t hmin = g.n1c > KWc ? scan_pos(0, 0, KWc) : (n1r > (uint32_t)W ? scan_pos(0, W, 0) : scan_pos(1, 0, 0));
        if (H > 0 && !((key >> kDpShift) == 0 && key_pos(key) < hmin)) {
          unsigned long long v = ~0ull;  // lanes without a helper: no window
          if (r < (int)H) {
            const unsigned long long* sl = &slots[(uint64_t)t * H + r];
            uint32_t spins = 0;
            while (((v = __hip_atomic_load(sl, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT)) & kSlotSet) == 0) {
              __builtin_amdgcn_s_sleep(1);
              if (++spins > (1u << 24)) {
                atomicOr(&a.flags[2], 1u);
                break;
              }
            }
          }
          v = v == ~0ull ? ~0ull : (v & ~kSlotSet);  // ~0: that helper had no window
          v = wave_min_u64(v);
          key = v < key ? v : key;
        }
        if (tid == 0) MSTAMP(t, 5);
        uint32_t bdist = (uint32_t)(W * W) + 1;
        int bi = 0, bj = 0, flip = -1;
        if (key != ~0ull) {
          bdist = key_dist(key, a.inv);
          flip = key_flip(key, a.inv);
          pos_window(g, W, key_pos(key), bi, bj);
        }
        const uint64_t p = r < W ? P64[r] : 0ull;
        const uint64_t b = (key != ~0ull && r < W) ? (band_bits64(L, bd, bi + r, bj) & topW) : 0ull;
        const uint64_t res = decide_tile(a, E, g, t, bi, bj, bdist, flip, p, b, r);
        if (r < W) {
          uint32_t* q = L + (uint32_t)(g.i0 + r - bd.lo) * bd.pitch + ((uint32_t)g.j0 >> 5);
          const int s32 = g.j0 & 31;
#pragma unroll
          for (int k = 0; k < 3; ++k) {
            const int off = 32 * k - s32;  // column of word k relative to j0
            if (off >= W) break;
            const uint64_t part_v = off >= 0 ? res << off : res >> -off;
            const uint64_t part_m = off >= 0 ? topW << off : topW >> -off;
            const uint32_t v = (uint32_t)(part_v >> 32), m = (uint32_t)(part_m >> 32);
            q[k] = (q[k] & ~m) | v;
          }
          // the plane's words of this tile row, from the band image (no read of the plane)
          const uint32_t w0 = (uint32_t)g.j0 >> 6, w1 = (uint32_t)(g.j0 + W - 1) >> 6;
          const uint32_t* lr = L + (uint32_t)(g.i0 + r - bd.lo) * bd.pitch;
          for (uint32_t w = w0; w <= w1; ++w)
            st_word(a.I + (uint64_t)(g.i0 + r) * a.wpr + w, ((uint64_t)lr[2 * w] << 32) | lr[2 * w + 1]);
        }
        if (tid == 0) MSTAMP(t, 6);
      }
    }
    __syncthreads();
    if (role == 0 && tid == 0) MSTAMP(t, 7);
  }
  if (role == 0 && tid < 64) {
    stores_done();
    if (tid == 0) raise_flag(&progress[ti], a.nx);
  }
}

// GolombCoder::codeSample of the chosen weights, raster order, split by coder (matched tiles ->
// golomb_match, the others -> golomb_nomatch). One workgroup walks the tiles in blocks of
// kMB * 8; codewords are OR'd into words this workgroup zeroed first. stats: [0] matches,
// [1] bits match, [2] bits nomatch, [3] sum of lengths.
__global__ __launch_bounds__(kMB) void k_match_code(const uint32_t* __restrict__ weights,
                                                    const uint8_t* __restrict__ modes,
                                                    const uint32_t* __restrict__ lens, uint32_t ntiles,
                                                    unsigned long long* out_m, unsigned long long* out_n,
                                                    size_t cap_words, uint64_t* stats, uint32_t* flags) {
  constexpr int kI = 8;
  __shared__ uint64_t tmp[17];
  uint64_t n_s[2] = {0, 0}, A_s[2] = {0, 0}, B_s[2] = {0, 0}, L = 0;  // running coder state
  bool ok[2] = {true, true};
  unsigned long long* outs[2] = {out_m, out_n};
  for (uint32_t base = 0; base < ntiles; base += kMB * kI) {
    const uint32_t t0 = base + threadIdx.x * kI;
    uint32_t v[kI];
    uint32_t which = 0;  // bit i: tile t0+i uses golomb_match
    uint32_t valid = 0;
    uint64_t cnt[2] = {0, 0}, sum[2] = {0, 0};
#pragma unroll
    for (int i = 0; i < kI; ++i) {
      v[i] = 0;
      if (t0 + i < ntiles) {
        valid |= 1u << i;
        v[i] = weights[t0 + i];
        const uint8_t m = modes[t0 + i];
        const int s = (m == 'X' || m == 'x') ? 0 : 1;
        if (s == 0) which |= 1u << i;
        cnt[s] += 1;
        sum[s] += v[i];
        L += lens[t0 + i];
      }
    }
    uint64_t ex_n[2], ex_a[2], tot_n[2], tot_a[2];
#pragma unroll
    for (int s = 0; s < 2; ++s) {
      ex_n[s] = block_excl_scan<uint64_t>(cnt[s], tmp, tot_n[s]);
      ex_a[s] = block_excl_scan<uint64_t>(sum[s], tmp, tot_a[s]);
    }
    // codeword lengths, then bit offsets
    uint64_t bits[2] = {0, 0};
    {
      uint64_t nn[2] = {n_s[0] + ex_n[0], n_s[1] + ex_n[1]}, AA[2] = {A_s[0] + ex_a[0], A_s[1] + ex_a[1]};
#pragma unroll
      for (int i = 0; i < kI; ++i) {
        if (valid >> i & 1) {
          const int s = (which >> i & 1) ? 0 : 1;
          const uint32_t k = golomb_k_state((uint32_t)nn[s], (uint32_t)AA[s]);
          bits[s] += k + (v[i] >> k) + 1;
          nn[s] += 1;
          AA[s] += v[i];
        }
      }
    }
    uint64_t ex_b[2], tot_b[2];
#pragma unroll
    for (int s = 0; s < 2; ++s) {
      ex_b[s] = block_excl_scan<uint64_t>(bits[s], tmp, tot_b[s]);
      // zero the words this block writes (the one it shares with the previous block is kept)
      const uint64_t b0 = B_s[s], b1 = B_s[s] + tot_b[s];
      if ((b1 + 63) / 64 > cap_words) ok[s] = false;
      if (ok[s]) {
        const uint64_t w_lo = base == 0 ? 0 : (b0 + 63) / 64, w_hi = (b1 + 63) / 64;
        for (uint64_t w = w_lo + threadIdx.x; w < w_hi; w += kMB) outs[s][w] = 0;
      }
    }
    __syncthreads();
    {
      uint64_t nn[2] = {n_s[0] + ex_n[0], n_s[1] + ex_n[1]}, AA[2] = {A_s[0] + ex_a[0], A_s[1] + ex_a[1]};
      uint64_t off[2] = {B_s[0] + ex_b[0], B_s[1] + ex_b[1]};
      GlobalSink gs[2] = {{out_m, 0, 0}, {out_n, 0, 0}};
#pragma unroll
      for (int i = 0; i < kI; ++i) {
        if (valid >> i & 1) {
          const int s = (which >> i & 1) ? 0 : 1;
          const uint32_t k = golomb_k_state((uint32_t)nn[s], (uint32_t)AA[s]);
          if (ok[s]) emit_codeword(gs[s], off[s], v[i], k);
          off[s] += k + (v[i] >> k) + 1;
          nn[s] += 1;
          AA[s] += v[i];
        }
      }
      gs[0].flush();
      gs[1].flush();
    }
    __syncthreads();
#pragma unroll
    for (int s = 0; s < 2; ++s) {
      n_s[s] += tot_n[s];
      A_s[s] += tot_a[s];
      B_s[s] += tot_b[s];
    }
  }
  uint64_t Ltot;
  block_excl_scan<uint64_t>(L, tmp, Ltot);
  if (threadIdx.x == 0) {
    stats[0] = n_s[0];
    stats[1] = B_s[0];
    stats[2] = B_s[1];
    stats[3] = Ltot;
    if (!ok[0] || !ok[1]) atomicOr(&flags[0], 1u);
    if (n_s[0] >= 0x80000000ull || n_s[1] >= 0x80000000ull || A_s[0] >= 0x80000000ull ||
        A_s[1] >= 0x80000000ull)
      atomicOr(&flags[1], 1u);
  }
}

}  // namespace

bool match_rows_fit(uint32_t W, uint32_t R, uint32_t cols) {
  const uint64_t nr = (uint64_t)R + 2 * W;  // band rows: R (or W) above plus the tile row
  return nr * ((cols + 31) / 32 + 2) <= kRowLds;
}

MatchSched match_schedule(uint32_t W, uint32_t R, uint32_t cols, uint32_t code, uint32_t var, uint32_t rows) {
  MatchSched m{};
  if (var) {  // compress4/5/6 loops: per-tile workgroups (k_match_tiles); R bounded by the image
    if (code >= 1 && code <= 256) {
      m.kind = kSchedTiles;
      m.G = code;
      return m;
    }
    const uint64_t Rr = std::min<uint64_t>(R, std::max<uint64_t>(rows, cols));
    const uint64_t r1 = Rr >= W ? Rr - W + 1 : 0;
    const uint64_t nmax = r1 * std::min<uint64_t>(2 * Rr + 1, cols) + (uint64_t)(W + 1) * (r1 + 1);
    const uint64_t g = (nmax + 2 * kChunk - 1) / (2 * kChunk);
    m.kind = kSchedTiles;
    m.G = (uint32_t)(g < 1 ? 1 : g > 64 ? 64 : g);
    return m;
  }
  // windows of the largest region: (R-W+1) rows above at 2R+1 columns, W+1 rows at R-W+1 columns
  const uint64_t r1 = R >= W ? (uint64_t)(R - W + 1) : 0;
  const uint64_t nmax = r1 * (2ull * R + 1) + (uint64_t)(W + 1) * (r1 + 1);
  const bool fit = match_rows_fit(W, R, cols), team_w = W == 8 || W == 16 || W == 32;
  if (code >= 1 && code <= 256) {
    m.kind = kSchedTiles;
    m.G = code;
    return m;
  }
  if (code == 0 || (code & 0xffff0000u) == 0x10000u) {
    if (fit && team_w) {
      m.kind = kSchedTeam;
      const uint64_t h = (nmax + 2047) / 2048;  // helpers: ~2K windows (a couple of tasks per thread) each
      m.H = code ? (code & 0xffffu) : (uint32_t)(h < 1 ? 1 : h > 16 ? 16 : h);
      if (m.H > 64) m.H = 64;
      m.K = W == 8 ? 4 : W == 16 ? 3 : 2;
      return m;
    }
    if (fit) {
      m.kind = kSchedRows;
      return m;
    }
  }
  m.kind = kSchedTiles;  // auto count of workgroups per tile
  const uint64_t g = (nmax + 2 * kChunk - 1) / (2 * kChunk);
  m.G = (uint32_t)(g < 1 ? 1 : g > 64 ? 64 : g);
  return m;
}

size_t match_scratch_bytes(size_t ntiles, const MatchSched& m) {
  return 512 + ntiles * (8 + 4 * 7 + 1) + ntiles * (size_t)m.H * 8 + 256 + ntiles * 8 + 256;  // (+ key2)
}

void launch_match_tiles(hipStream_t s, MatchArgs& a, const MatchSched& m, void* scratch) {
  const uint32_t ntiles = a.nx * a.ny;
  char* c = reinterpret_cast<char*>(scratch);
  a.counter = reinterpret_cast<uint32_t*>(c);
  a.key = reinterpret_cast<unsigned long long*>(c + 256);
  a.done = reinterpret_cast<uint32_t*>(a.key + ntiles);
  a.arrive = a.done + ntiles;
  a.lens = a.arrive + ntiles;
  uint32_t* spare = a.lens + ntiles;
  if (!a.besti) a.besti = spare;
  if (!a.bestj) a.bestj = spare + ntiles;
  if (!a.bestd) a.bestd = spare + 2 * ntiles;
  if (!a.weights) a.weights = spare + 3 * ntiles;
  if (!a.modes) a.modes = reinterpret_cast<uint8_t*>(spare + 4 * ntiles);
  unsigned long long* slots = reinterpret_cast<unsigned long long*>(
      (reinterpret_cast<uintptr_t>(spare + 4 * ntiles) + ntiles + 255) & ~(uintptr_t)255);
  a.key2 = reinterpret_cast<unsigned long long*>(
      (reinterpret_cast<uintptr_t>(slots + (size_t)ntiles * m.H) + 255) & ~(uintptr_t)255);
  a.G = m.G;
  a.H = m.H;
  a.K = m.K;
  (void)launch_fill(s, a.counter, 0, 4);
  (void)launch_fill(s, a.key, 0xff, (size_t)ntiles * 8);
  if (a.var == 5) (void)launch_fill(s, a.key2, 0xff, (size_t)ntiles * 8);
  (void)launch_fill(s, a.done, 0, (size_t)ntiles * 8);  // done + arrive (row schedules: progress)
  uint32_t* progress = a.done;
  switch (m.kind) {
    case kSchedTeam:
      if (m.H) (void)launch_fill(s, slots, 0, (size_t)ntiles * m.H * 8);
      if (a.W == 8) k_match_team<8><<<a.ny * (m.H + 1), kRB, 0, s>>>(a, progress, slots);
      else if (a.W == 16) k_match_team<16><<<a.ny * (m.H + 1), kRB, 0, s>>>(a, progress, slots);
      else k_match_team<32><<<a.ny * (m.H + 1), kRB, 0, s>>>(a, progress, slots);
      break;
    case kSchedRows:
      k_match_rows<<<a.ny, kRB, 0, s>>>(a, progress);
      break;
    default:
      k_match_tiles<<<ntiles * a.G, kMB, 0, s>>>(a);
  }
}

void launch_match_code(hipStream_t s, const MatchArgs& a, unsigned long long* out_m, unsigned long long* out_n,
                       size_t cap_words, uint64_t* stats) {
  k_match_code<<<1, kMB, 0, s>>>(a.weights, a.modes, a.lens, a.nx * a.ny, out_m, out_n, cap_words, stats, a.flags);
}

}  // namespace bic
