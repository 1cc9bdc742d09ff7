// bic_kstat.h -- Golomb k statistics of row strips: the staged row encoder's count pass
// (bic_kernels.hip k_med_kstat, k_gray_strips) writes one record per (plane, row, strip);
// k_scan_rows (bic_fused.hip) combines a row's records (row_kstats) and, from the coder state at the
// row's start, proves that every codeword of the row has k = 0 or k = 1, whose lengths then have
// closed forms (no per-codeword walk). Included by .hip files only (after bic_device.h).
//
// For the row's samples t (its 1s at columns p_u, u = 0..ones-1, then the end-of-row sample at
// column cols; p_{-1} = -1) and the state (N0, A0) before the row, N_t = N0 + t and
// A_t = A0 + p_{t-1} + 1 - t (GolombCoder.cpp:29-34); k_t = 0 iff A_t <= N_t, and k_t = 1 iff
// N_t < A_t <= 2 N_t (GolombCoder.cpp:33). Relative to the start state, A_t - N_t - (A0 - N0) is 0
// at t = 0 and p_u - 2u - 1 at t = u + 1; A_t - 2 N_t - (A0 - 2 N0) is 0 and p_u - 3u - 2. A word of
// m 1s spanning columns pf..pl, with ob 1s of the strip before it, has its j-th 1 in
// [pf + j, pl - (m - 1 - j)], which bounds those by q0 = pl - m - 2 ob (max), ql = pf - 2 ob - m
// (min) and qh = pl - m - 3 ob - 1 (max). chg counts consecutive samples whose columns differ in
// parity: a run s_t = p_t - p_{t-1} - 1 is odd iff the two parities agree, so a row whose
// codewords all have k = 1 is sum(2 + s_t >> 1) = 2n + (zeros - odd runs) / 2 bits long
// (n = ones + 1 samples, zeros = cols - ones).
#pragma once
#include "bic_device.h"

namespace bic {

constexpr int32_t kNoOnes = 1 << 30;
constexpr uint32_t kMaxStrips = 4;  // records per row: k_med_kstat covers whole rows (1), k_gray_strips
                                    // one per 64-word strip (<= 4 for rows of <= 256 words)

// Parity changes between consecutive 1s inside a word: with columns MSB-first a 1's predecessor
// sits at a higher bit; adding S << 1 to ~x ripples each carry up through the zeros and stops at
// the predecessor, so (~x + (S << 1)) & x are the predecessors of S's 1s (a carry out of bit 63
// belongs to a 1 whose predecessor lies in an earlier word).
__device__ __forceinline__ uint32_t parity_changes(uint64_t x) {
  constexpr uint64_t kEven = 0xAAAAAAAAAAAAAAAAull;  // bits 63, 61, ...: even columns
  const uint64_t E = x & kEven, O = x & ~kEven;
  const uint64_t pe = (~x + (E << 1)) & x, po = (~x + (O << 1)) & x;
  return (uint32_t)__popcll(pe & O) + (uint32_t)__popcll(po & E);
}

// A lane's statistics over its consecutive residual words, fed in column order (lanek_word); ones
// counts the lane's 1s so far (the words' bounds are lane-local and rebased in lanek_store).
struct LaneK {
  uint32_t ones = 0, chg = 0;
  int32_t q0 = -kNoOnes, qh = -kNoOnes, ql = kNoOnes, first = -1, last = -1;
};
__device__ __forceinline__ void lanek_word(LaneK& k, uint64_t x, int32_t c0) {
  if (!x) return;
  const int32_t m = __popcll(x), o = (int32_t)k.ones;
  const int32_t pl = c0 + 63 - __builtin_ctzll(x), pf = c0 + __builtin_clzll(x);
  k.q0 = max(k.q0, pl - m - 2 * o);
  k.qh = max(k.qh, pl - m - 3 * o - 1);
  k.ql = min(k.ql, pf - 2 * o - m);
  k.chg += parity_changes(x) + (k.last >= 0 ? (uint32_t)((k.last ^ pf) & 1) : 0u);
  if (k.first < 0) k.first = pf;
  k.last = pl;
  k.ones += m;
}

// The record of the strip the wave's lanes cover (lanes in column order): one scan of the lanes' 1
// counts rebases their bounds, one max-scan of their last 1s links each lane's first 1 to its
// predecessor. Record {q0, qh, ql, ones | chg << 16} and {first | last << 16} (columns < 2^15,
// -1 = none); lane 0 stores them and the strip's 1-count.
__device__ __forceinline__ void lanek_store(const LaneK& k, int4* rec, uint32_t* pos, uint32_t* sones) {
  if (__ballot(k.ones != 0) == ~0ull) {
    // Every lane holds a 1 (the common case unless the strip is sparse): a lane's predecessor 1 is
    // lane l - 1's last and the strip's first / last 1 are lane 0's / lane 63's, so one scan of
    // (ones | chg << 16) (both <= 16384 per strip) and three reductions finish the record.
    const int32_t before = dpp_or<0x138>(-1, k.last);
    const uint32_t chg = k.chg + (before >= 0 ? (uint32_t)((before ^ k.first) & 1) : 0u);
    const uint32_t inc = wave_incl_sum_u32(k.ones | (chg << 16));
    const int32_t base = (int32_t)((inc & 0xffffu) - k.ones);
    const int32_t q0 = wave_max(k.q0 - 2 * base);
    const int32_t qh = wave_max(k.qh - 3 * base);
    const int32_t ql = wave_min(k.ql - 2 * base);
    const uint32_t t = lane63_u32(inc), tot = t & 0xffffu;
    const uint32_t f = (uint32_t)__builtin_amdgcn_readlane(k.first, 0);
    const uint32_t last = lane63_u32((uint32_t)k.last);
    if (lane_id() == 0) {
      *rec = make_int4(q0, qh, ql, (int32_t)(tot | (t >> 16 << 16)));
      *pos = (f & 0xffffu) | (last << 16);
      *sones = tot;
    }
    return;
  }
  const uint32_t inc = wave_incl_sum_u32(k.ones);
  const int32_t base = (int32_t)(inc - k.ones);
  const int mx = wave_incl_max(k.last);
  const int32_t before = dpp_or<0x138>(-1, mx);  // the last 1 of the lanes before (-1: none)
  uint32_t chg = k.chg;
  int32_t first = -1;
  if (k.ones) {
    if (before >= 0) chg += (uint32_t)((before ^ k.first) & 1);
    else first = k.first;
  }
  const int32_t q0 = wave_max(k.ones ? k.q0 - 2 * base : -kNoOnes);
  const int32_t qh = wave_max(k.ones ? k.qh - 3 * base : -kNoOnes);
  const int32_t ql = wave_min(k.ones ? k.ql - 2 * base : kNoOnes);
  const uint32_t c = wave_sum_u32(chg);
  const int32_t f = wave_max(first);
  const uint32_t tot = lane63_u32(inc);
  const uint32_t last = lane63_u32((uint32_t)mx);
  if (lane_id() == 0) {
    *rec = make_int4(q0, qh, ql, (int32_t)(tot | (c << 16)));
    *pos = ((uint32_t)f & 0xffffu) | (last << 16);
    *sones = tot;
  }
}

// A row's statistics from its ns strip records (the strips' local 1 counts rebased).
struct RowK {
  int32_t q0, qh, ql;
  uint32_t ones, chg;
};
__device__ __forceinline__ RowK row_kstats(const int4* rec, const uint32_t* pos, uint32_t ns, uint32_t cols) {
  RowK r{0, 0, 0, 0, 0};
  int32_t last = -1;
  for (uint32_t s = 0; s < ns; ++s) {
    const int4 v = rec[s];
    const uint32_t o = (uint32_t)v.w & 0xffffu;
    if (!o) continue;
    const uint32_t p = pos[s];
    r.q0 = max(r.q0, v.x - 2 * (int32_t)r.ones);
    r.qh = max(r.qh, v.y - 3 * (int32_t)r.ones);
    r.ql = min(r.ql, v.z - 2 * (int32_t)r.ones);
    r.chg += ((uint32_t)v.w >> 16) + (uint32_t)((last ^ (int32_t)(int16_t)(p & 0xffffu)) & 1);
    r.ones += o;
    last = (int16_t)(p >> 16);
  }
  r.chg += (uint32_t)((last ^ (int32_t)cols) & 1);  // the end-of-row sample at column cols
  return r;
}

}  // namespace bic
