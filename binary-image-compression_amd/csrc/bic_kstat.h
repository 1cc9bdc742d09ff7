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

// The strip records of up to 8 planes at once, for waves whose lanes hold ONE residual word per
// plane (k_gray_strips): strip_word_put leaves lane l's (m | chg << 8, pf | pl << 16) of plane b
// in the wave's LDS table t (1024 words); after a wave fence, strip_records lets lane
// L = 8 p + j combine lanes 8j..8j+7 of plane p in column order, then the eight parts of a plane
// are combined with 8-lane DPP scans (ones before the part, last 1 before it) and reductions;
// lane 8p stores plane p's record (the same record lanek_word + lanek_store make). One transposed
// pass instead of eight wave-wide scan-and-reduce chains.
__device__ __forceinline__ void strip_word_put(uint32_t* t, int b, uint64_t x, int32_t c0) {
  const int lane = lane_id();
  // branch-free: x = 0 gives m = 0 (strip_records then ignores c)
  const uint32_t m = (uint32_t)__popcll(x) | (parity_changes(x) << 8);
  // first / last 1 from the raw find-first-bit instructions (-1 for a zero half, so min() picks the
  // other half); an all-zero word gives garbage here, which strip_records ignores (m = 0). Four
  // instructions fewer per plane than clz / ffs with their zero cases
  uint32_t hh, hl, lh, ll;
  const uint32_t xh = (uint32_t)(x >> 32), xl = (uint32_t)x;
  asm volatile("v_ffbh_u32 %0, %1" : "=v"(hh) : "v"(xh));
  asm volatile("v_ffbh_u32 %0, %1" : "=v"(hl) : "v"(xl));
  asm volatile("v_ffbl_b32 %0, %1" : "=v"(lh) : "v"(xh));
  asm volatile("v_ffbl_b32 %0, %1" : "=v"(ll) : "v"(xl));
  const uint32_t lz = min(hh, hl + 32u), tz = min(ll, lh + 32u);
  const uint32_t c = ((uint32_t)c0 + lz) | (((uint32_t)c0 + 63u - tz) << 16);
  // lane l's value is value i = l & 7 of part 8b + (l >> 3): stored at word (i >> 2) * 256 +
  // 4 * part + (i & 3), so that strip_records' 16-byte reads (lane L: words 4L..4L+3 of each
  // quarter) are bank-conflict free
  const uint32_t idx = ((uint32_t)(lane & 7) >> 2) * 256 + 32 * b + 4 * (lane >> 3) + (lane & 3);
  t[idx] = m;
  t[512 + idx] = c;
}
template <int CTRL>
__device__ __forceinline__ int dpp_same(int v) {  // every source lane valid (quad perms, mirrors)
  // no old operand (bound_ctrl): the step folds into the max / min / add that uses it
  return __builtin_amdgcn_mov_dpp(v, CTRL, 0xf, 0xf, true);
}
__device__ __forceinline__ void strip_records(const uint32_t* t, int np, int4* krec, uint32_t* kpos, uint32_t* sones,
                                              uint64_t id0, uint64_t pstride) {
  const int L = lane_id(), p = L >> 3, j = L & 7;
  const uint4 a0 = *reinterpret_cast<const uint4*>(t + 4 * L);
  const uint4 a1 = *reinterpret_cast<const uint4*>(t + 256 + 4 * L);
  const uint4 c0 = *reinterpret_cast<const uint4*>(t + 512 + 4 * L);
  const uint4 c1 = *reinterpret_cast<const uint4*>(t + 768 + 4 * L);
  const uint32_t av[8] = {a0.x, a0.y, a0.z, a0.w, a1.x, a1.y, a1.z, a1.w};
  const uint32_t cv[8] = {c0.x, c0.y, c0.z, c0.w, c1.x, c1.y, c1.z, c1.w};
  uint32_t ones = 0, chg = 0;
  int32_t first = -1, last = -1, q0 = -kNoOnes, qh = -kNoOnes, ql = kNoOnes;
#pragma unroll
  for (int i = 0; i < 8; ++i) {
    const int32_t m = (int32_t)(av[i] & 0xffu);
    if (m) {
      const int32_t pf = (int32_t)(cv[i] & 0xffffu), pl = (int32_t)(cv[i] >> 16), o = (int32_t)ones;
      chg += (av[i] >> 8) + (last >= 0 ? (uint32_t)((last ^ pf) & 1) : 0u);
      q0 = max(q0, pl - m - 2 * o);
      qh = max(qh, pl - m - 1 - 3 * o);
      ql = min(ql, pf - m - 2 * o);
      if (first < 0) first = pf;
      last = pl;
      ones += (uint32_t)m;
    }
  }
  // inclusive 8-lane scans (row_shr inside the 16-lane row, masked to the part's group)
  uint32_t inc = ones;
  int32_t lmax = last;
#pragma unroll
  for (int d = 1; d < 8; d <<= 1) {
    const uint32_t o = d == 1 ? (uint32_t)dpp_or<0x111>(0, (int)inc) : d == 2 ? (uint32_t)dpp_or<0x112>(0, (int)inc)
                                                                             : (uint32_t)dpp_or<0x114>(0, (int)inc);
    const int32_t lm = d == 1 ? dpp_or<0x111>(-1, lmax) : d == 2 ? dpp_or<0x112>(-1, lmax) : dpp_or<0x114>(-1, lmax);
    if (j >= d) {
      inc += o;
      lmax = max(lmax, lm);
    }
  }
  const int32_t lprev = dpp_or<0x111>(-1, lmax);  // DPP outside any branch: every source lane active
  const int32_t before = j ? lprev : -1;           // the last 1 of the parts before
  const int32_t B = (int32_t)(inc - ones);
  if (ones) {
    if (before >= 0) chg += (uint32_t)((before ^ first) & 1);
    q0 -= 2 * B;
    qh -= 3 * B;
    ql -= 2 * B;
  }
  int32_t f = ones ? first : INT_MAX;
  uint32_t tot = ones;
  // 8-lane reductions: quad swaps, then the half-row mirror pairs the group's two quads
#define BIC_RED8(CTRL)                          \
  q0 = max(q0, dpp_same<CTRL>(q0));             \
  qh = max(qh, dpp_same<CTRL>(qh));             \
  ql = min(ql, dpp_same<CTRL>(ql));             \
  f = min(f, dpp_same<CTRL>(f));                \
  last = max(last, dpp_same<CTRL>(last));       \
  chg += (uint32_t)dpp_same<CTRL>((int)chg);    \
  tot += (uint32_t)dpp_same<CTRL>((int)tot);
  BIC_RED8(0xB1)
  BIC_RED8(0x4E)
  BIC_RED8(0x141)
#undef BIC_RED8
  if (j == 0 && p < np) {
    const uint64_t id = id0 + (uint64_t)p * pstride;
    krec[id] = make_int4(q0, qh, ql, (int32_t)(tot | (chg << 16)));
    kpos[id] = ((uint32_t)(f == INT_MAX ? -1 : f) & 0xffffu) | ((uint32_t)last << 16);
    sones[id] = tot;
  }
}

// A row's statistics from its ns (<= kMaxStrips) strip records (the strips' local 1 counts
// rebased). Every record is loaded before any is used.
struct RowK {
  int32_t q0, qh, ql;
  uint32_t ones, chg;
};
// (in two halves -- the strips' records loaded, then combined -- so a caller can keep the loads in
// flight across other work)
struct RowKRaw {
  int4 v[kMaxStrips];
  uint32_t pp[kMaxStrips];
};
__device__ __forceinline__ RowKRaw row_kstats_load(const int4* rec, const uint32_t* pos, uint32_t ns) {
  RowKRaw q;
#pragma unroll
  for (uint32_t s = 0; s < kMaxStrips; ++s) {
    q.v[s] = s < ns ? rec[s] : make_int4(0, 0, 0, 0);
    q.pp[s] = s < ns ? pos[s] : 0u;
  }
  return q;
}
__device__ __forceinline__ RowK row_kstats_combine(const RowKRaw& q, uint32_t cols) {
  const int4* v = q.v;
  const uint32_t* pp = q.pp;
  RowK r{0, 0, 0, 0, 0};
  int32_t last = -1;
#pragma unroll
  for (uint32_t s = 0; s < kMaxStrips; ++s) {
    const uint32_t o = (uint32_t)v[s].w & 0xffffu;
    if (!o) continue;
    r.q0 = max(r.q0, v[s].x - 2 * (int32_t)r.ones);
    r.qh = max(r.qh, v[s].y - 3 * (int32_t)r.ones);
    r.ql = min(r.ql, v[s].z - 2 * (int32_t)r.ones);
    r.chg += ((uint32_t)v[s].w >> 16) + (uint32_t)((last ^ (int32_t)(int16_t)(pp[s] & 0xffffu)) & 1);
    r.ones += o;
    last = (int16_t)(pp[s] >> 16);
  }
  r.chg += (uint32_t)((last ^ (int32_t)cols) & 1);  // the end-of-row sample at column cols
  return r;
}
__device__ __forceinline__ RowK row_kstats(const int4* rec, const uint32_t* pos, uint32_t ns, uint32_t cols) {
  return row_kstats_combine(row_kstats_load(rec, pos, ns), cols);
}

}  // namespace bic
