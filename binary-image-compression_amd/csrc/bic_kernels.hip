// bic_kernels.hip -- hand-written gfx950 (CDNA4) kernels for the hot path of
// nacho-pancho/binary-image-compression. Integer/bitwise only: no MFMA. Every kernel
// is HBM- or VALU-bound; loads are laid out so one wave instruction moves 512
// contiguous bytes, and chunk kernels remap blockIdx so neighbouring rows (which
// re-read each other as the "row above") stay on one XCD's L2.
//
// Reference semantics restated here (file:line under /root/reference/src):
//   med (pred.cpp:3-15)         word form: R = P ^ U ^ (P>>1|Pl<<63) ^ (U>>1|Ul<<63),
//                               R(0,0) = 0, pad bits 0
//   GolombCoder (GolombCoder.cpp:13-34, Golomb.h:14-19)
//                               k_0 = 1; after n samples with sum A: k = min{k : n<<k >= A}
//   EGCoder as written (eg.cpp:20-37)  len+1 bits per run, +1 on the first non-EOL run
//   bitplanes (bitplane_tool.cpp:24-30)
//   tile path (compress7_test.cpp:184-275 with R = 0)
#include "bic_device.h"
#include "bic_k1pi.h"
#include "bic_kstat.h"

namespace bic {

// ------------------------------------------------------------------------------------
// K1: bitplanes (bitplane_tool.cpp:24-30). Lane l of a wave owns output word l of a row: it
// loads its 64 pixels (four 16-byte loads), turns each group of 8 pixels into one byte per plane
// with an 8x8 bit transpose (MSB = leftmost pixel) and stores one 64-bit word per plane; 64 lanes
// store 512 contiguous bytes of each plane row. No LDS, no barrier.
// ------------------------------------------------------------------------------------
__device__ __forceinline__ uint64_t transpose8x8(uint64_t x) {
  uint64_t t;
  t = (x ^ (x >> 7)) & 0x00AA00AA00AA00AAull;
  x = x ^ t ^ (t << 7);
  t = (x ^ (x >> 14)) & 0x0000CCCC0000CCCCull;
  x = x ^ t ^ (t << 14);
  t = (x ^ (x >> 28)) & 0x00000000F0F0F0F0ull;
  x = x ^ t ^ (t << 28);
  return x;
}

template <bool VEC>
__global__ __launch_bounds__(kBlock) void k_bitplanes_u8(const uint8_t* __restrict__ gray, size_t pitch,
                                                         uint32_t rows, uint32_t cols, uint32_t used,
                                                         int plane0, int nplanes, uint64_t* __restrict__ planes,
                                                         uint32_t wpr) {
  const uint32_t groups = (used + 63) / 64;  // 64-word groups per row
  const uint64_t gw = (uint64_t)blockIdx.x * kWaves + wave_id();
  if (gw >= (uint64_t)rows * groups) return;
  const uint32_t row = (uint32_t)(gw / groups), w = (uint32_t)(gw % groups) * 64 + lane_id();
  if (w >= used) return;
  const uint8_t* src = gray + (uint64_t)row * pitch + (uint64_t)w * 64;
  uint64_t px[8];  // 8 groups of 8 pixels, little-endian bytes
  if (VEC && (uint64_t)w * 64 + 64 <= cols) {
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      const uint4 v = *reinterpret_cast<const uint4*>(src + 16 * i);
      px[2 * i] = (uint64_t)v.x | ((uint64_t)v.y << 32);
      px[2 * i + 1] = (uint64_t)v.z | ((uint64_t)v.w << 32);
    }
  } else {
#pragma unroll
    for (int g8 = 0; g8 < 8; ++g8) {
      uint64_t v = 0;
      for (int x = 0; x < 8; ++x) {
        const uint32_t j = w * 64 + g8 * 8 + x;
        if (j < cols) v |= (uint64_t)src[g8 * 8 + x] << (8 * x);
      }
      px[g8] = v;
    }
  }
  uint64_t T[8];
#pragma unroll
  for (int g8 = 0; g8 < 8; ++g8) T[g8] = transpose8x8(bswap64(px[g8]));  // byte b = plane b's 8 bits
  const uint64_t plane_words = (uint64_t)rows * wpr;
  uint64_t* dst = planes + (uint64_t)row * wpr + w;
#pragma unroll
  for (int b = 0; b < 8; ++b) {
    if (b >= nplanes) break;
    const int sb = 8 * (b + plane0);  // output plane b = bit plane0 + b of the gray value
    uint64_t v = 0;
#pragma unroll
    for (int g8 = 0; g8 < 8; ++g8) v |= ((T[g8] >> sb) & 0xffull) << (56 - 8 * g8);
    dst[b * plane_words] = v;
  }
}

void launch_bitplanes_u8(hipStream_t s, const uint8_t* gray, size_t pitch, uint32_t rows,
                         uint32_t cols, int plane0, int nplanes, uint64_t* planes, uint32_t wpr) {
  const uint32_t used = (cols + 63) / 64;
  const uint64_t waves = (uint64_t)rows * ((used + 63) / 64);
  const uint32_t grid = (uint32_t)((waves + kWaves - 1) / kWaves);
  const bool vec = (pitch % 16 == 0) && (((uintptr_t)gray) % 16 == 0);
  if (vec)
    k_bitplanes_u8<true><<<grid, kBlock, 0, s>>>(gray, pitch, rows, cols, used, plane0, nplanes, planes, wpr);
  else
    k_bitplanes_u8<false><<<grid, kBlock, 0, s>>>(gray, pitch, rows, cols, used, plane0, nplanes, planes, wpr);
}

// ------------------------------------------------------------------------------------
// K2: count pass -- med residual per chunk: popcount, first/last 1-column, optional
// residual store and per-plane weight (binmat.cpp:57-67).
// ------------------------------------------------------------------------------------
template <int WPL, bool PREDICT>
__global__ __launch_bounds__(kBlock) void k_count(Geom g, const uint64_t* __restrict__ planes,
                                                  ChunkScratch cs, uint64_t* __restrict__ resid) {
  const ChunkId ci = chunk_id(g);
  if (!ci.ok) return;  // whole wave uniform
  const uint32_t c0 = ci.c * g.wpc;
  const int lane = lane_id();
  uint64_t rr[WPL];
  resid_row<WPL, PREDICT>(planes, g, ci.plane, ci.row, rr, c0);
  uint32_t ones = 0;
  int last = -1, first = INT_MAX;
#pragma unroll
  for (int t = 0; t < WPL; ++t) {
    const uint32_t w = c0 + t * 64 + lane;
    const uint64_t r = rr[t];
    if (resid && w < g.wpr && w < c0 + g.wpc)
      resid[(uint64_t)ci.plane * g.plane_words + (uint64_t)ci.row * g.wpr + w] = r;
    ones += (uint32_t)__popcll(r);
    if (r) {
      last = (int)(w * 64 + 63 - __builtin_ctzll(r));
      if (first == INT_MAX) first = (int)(w * 64 + __builtin_clzll(r));
    }
  }
  ones = wave_sum_u32(ones);
  last = wave_max(last);
  first = wave_min(first);
  if (lane == 0) {
    cs.ones[ci.id] = ones;
    cs.last[ci.id] = last;
    cs.first[ci.id] = first;
  }
}

// per-plane weight (binmat.cpp:57-67) from the chunks' 1-counts: one workgroup per plane
__global__ __launch_bounds__(1024) void k_plane_weight(const uint32_t* __restrict__ ones, uint64_t chunks_per_plane,
                                                       uint64_t* weight_out) {
  __shared__ uint64_t tmp[17];
  const uint32_t* o = ones + (uint64_t)blockIdx.x * chunks_per_plane;
  uint64_t a = 0;
  for (uint64_t i = threadIdx.x; i < chunks_per_plane; i += 1024) a += o[i];
  uint64_t tot;
  block_excl_scan<uint64_t>(a, tmp, tot);
  if (threadIdx.x == 0) weight_out[blockIdx.x] = tot;
}

// K2b: bic_med_residual for rows of up to 256 words (even row pitch, 16-byte aligned planes):
// one wave walks RPW consecutive rows of a plane, keeping the row above in registers, with
// 16-byte loads (lane l holds words 2l, 2l+1 of each 128-word half). Writes the residual if
// asked and one 1-count per wave (k_plane_weight adds those up per plane).
template <int NP, int RPW, bool PREDICT>
__global__ __launch_bounds__(kBlock) void k_med_rows(Geom g, const uint64_t* __restrict__ planes,
                                                     uint64_t* __restrict__ resid, uint32_t* __restrict__ part) {
  const int lane = lane_id();
  const uint32_t wpp = (g.rows + RPW - 1) / RPW;  // waves per plane
  const uint64_t gw = (uint64_t)xcd_remap(blockIdx.x, gridDim.x) * kWaves + wave_id();
  if (gw >= (uint64_t)wpp * g.nplanes) return;
  const uint32_t plane = (uint32_t)(gw / wpp), r0 = (uint32_t)(gw % wpp) * RPW;
  const uint64_t* pl = planes + (uint64_t)plane * g.plane_words;
  uint64_t up0[NP], up1[NP];
#pragma unroll
  for (int t = 0; t < NP; ++t) {
    up0[t] = up1[t] = 0;
    if (PREDICT && r0) {
      const uint32_t w = t * 128 + 2 * lane;
      if (w < g.used) {
        const ulonglong2 v = *reinterpret_cast<const ulonglong2*>(pl + (uint64_t)(r0 - 1) * g.wpr + w);
        up0[t] = v.x;
        up1[t] = v.y;
      }
    }
  }
  uint32_t ones = 0;
  const uint32_t nr = min((uint32_t)RPW, g.rows - r0);
  uint64_t p0[NP], p1[NP];  // current row; the next one is loaded before this one is used
  auto load_row = [&](uint32_t row, uint64_t (&a)[NP], uint64_t (&b)[NP]) {
#pragma unroll
    for (int t = 0; t < NP; ++t) {
      const uint32_t w = t * 128 + 2 * lane;
      const ulonglong2 v = *reinterpret_cast<const ulonglong2*>(pl + (uint64_t)row * g.wpr + (w < g.used ? w : 0));
      a[t] = v.x;
      b[t] = v.y;
    }
  };
  load_row(r0, p0, p1);
  for (uint32_t i = 0; i < nr; ++i) {
    const uint32_t row = r0 + i;
    uint64_t q0[NP], q1[NP];
    if (i + 1 < nr) load_row(row + 1, q0, q1);
    uint64_t carry = 0;
#pragma unroll
    for (int t = 0; t < NP; ++t) {
      const uint32_t w = t * 128 + 2 * lane;
      uint64_t R0 = p0[t], R1 = p1[t];
      if constexpr (PREDICT) {
        const uint64_t D0 = p0[t] ^ up0[t], D1 = p1[t] ^ up1[t];
        uint64_t Dl = shfl_up_u64(D1, 1);
        if (lane == 0) Dl = carry;
        carry = lane63_u64(D1);
        R0 = D0 ^ ((D0 >> 1) | (Dl << 63));
        R1 = D1 ^ ((D1 >> 1) | (D0 << 63));
        if (row == 0 && w == 0) R0 &= ~BIC_MSB;  // pred.cpp never writes pP(0,0)
        up0[t] = p0[t];
        up1[t] = p1[t];
      }
      if (w >= g.used) R0 = 0;
      if (w + 1 >= g.used) R1 = 0;
      if (w == g.used - 1) R0 &= g.trail;
      if (w + 1 == g.used - 1) R1 &= g.trail;
      ones += (uint32_t)__popcll(R0) + (uint32_t)__popcll(R1);
      if (resid && w < g.wpr) {
        uint64_t* dst = resid + (uint64_t)plane * g.plane_words + (uint64_t)row * g.wpr + w;
        *reinterpret_cast<ulonglong2*>(dst) = make_ulonglong2(R0, R1);
      }
    }
#pragma unroll
    for (int t = 0; t < NP; ++t) {
      p0[t] = q0[t];
      p1[t] = q1[t];
    }
  }
  ones = wave_sum_u32(ones);
  if (lane == 0) part[gw] = ones;
}

// ------------------------------------------------------------------------------------
// The staged encoder's count pass (bic_kstat.h): per row of every plane its residual 1-count and k
// statistics record. Each wave walks rows whole, lane l owning the LW consecutive words
// LW*l .. LW*l + LW - 1 (64 * LW >= the row's words), so the k statistics accumulate inside the
// lane and one scan pair and one set of reductions per (plane, row) finish them (lanek_store).
// ------------------------------------------------------------------------------------
// From the planes (planes 16-byte aligned, even row pitch; med_rows_supported): RPW rows of one
// plane per wave, the row above kept in registers, the next row's loads in flight while this one is
// used.
template <int LW, int RPW, bool PREDICT>
__global__ __launch_bounds__(kBlock) void k_med_kstat(Geom g, const uint64_t* __restrict__ planes,
                                                      uint32_t* __restrict__ sones, int4* __restrict__ krec,
                                                      uint32_t* __restrict__ kpos, uint32_t* __restrict__ zero) {
  if (blockIdx.x == 0 && threadIdx.x < kZeroWords) zero[threadIdx.x] = 0;  // the encoder's counters
  const int lane = lane_id();
  const uint32_t wpp = (g.rows + RPW - 1) / RPW;  // waves per plane
  const uint64_t gw = (uint64_t)xcd_remap(blockIdx.x, gridDim.x) * kWaves + wave_id();
  if (gw >= (uint64_t)wpp * g.nplanes) return;  // whole wave
  const uint32_t plane = (uint32_t)(gw / wpp), r0 = (uint32_t)(gw % wpp) * RPW;
  const uint64_t* pl = planes + (uint64_t)plane * g.plane_words;
  const uint32_t w0 = LW * lane;
  auto load = [&](uint32_t row, uint64_t (&v)[LW]) {
    const uint64_t* src = pl + (uint64_t)row * g.wpr + w0;
    if constexpr (LW == 1) {
      v[0] = w0 < g.used ? src[0] : 0;
    } else {
#pragma unroll
      for (int i = 0; i < LW; i += 2) {  // pairs below `used` lie inside the (even) row pitch
        ulonglong2 t = make_ulonglong2(0, 0);
        if (w0 + i < g.used) t = *reinterpret_cast<const ulonglong2*>(src + i);
        v[i] = t.x;
        v[i + 1] = t.y;
      }
    }
  };
  uint64_t up[LW], cur[LW];
#pragma unroll
  for (int i = 0; i < LW; ++i) up[i] = 0;
  if (PREDICT && r0) load(r0 - 1, up);
  load(r0, cur);
  const uint32_t nr = min((uint32_t)RPW, g.rows - r0);
  for (uint32_t r = 0; r < nr; ++r) {
    const uint32_t row = r0 + r;
    uint64_t nxt[LW];
    if (r + 1 < nr) load(row + 1, nxt);
    LaneK k;
    uint64_t D[LW];
#pragma unroll
    for (int i = 0; i < LW; ++i) D[i] = PREDICT ? cur[i] ^ up[i] : cur[i];
    const uint64_t dl = wave_shr1_u64(D[LW - 1]);  // word LW*l - 1 (lane l - 1's last; lane 0: 0)
#pragma unroll
    for (int i = 0; i < LW; ++i) {
      const uint32_t w = w0 + i;
      uint64_t R = D[i];
      if constexpr (PREDICT) {
        R = D[i] ^ ((D[i] >> 1) | ((i ? D[i - 1] : dl) << 63));
        if (row == 0 && w == 0) R &= ~BIC_MSB;  // pred.cpp never writes pP(0,0)
      }
      R = w < g.used ? (w == g.used - 1 ? R & g.trail : R) : 0;
      lanek_word(k, R, (int32_t)(w * 64));
      up[i] = cur[i];
    }
    const uint64_t id = (uint64_t)plane * g.rows + row;
    lanek_store(k, krec + id, kpos + id, sones + id);
#pragma unroll
    for (int i = 0; i < LW; ++i) cur[i] = nxt[i];
  }
}

// Rows of <= 64 words (C4: 4096 columns): four rows per wave, one per 16-lane DPP row, lane q of a
// group owning words 4q .. 4q + 3. The row's scans and reductions then run inside a DPP row (4
// steps instead of 6, and one pass for four rows): ~4x fewer instructions per row than one row per
// wave with one word per lane, where the record's scan and reductions dominate.
template <int CTRL>
__device__ __forceinline__ int dpp16(int old, int v) {  // inside a 16-lane row; invalid sources read old
  return __builtin_amdgcn_update_dpp(old, v, CTRL, 0xf, 0xf, false);
}
__device__ __forceinline__ uint32_t row16_incl_sum(uint32_t x) {
  x += (uint32_t)dpp16<0x111>(0, (int)x);
  x += (uint32_t)dpp16<0x112>(0, (int)x);
  x += (uint32_t)dpp16<0x114>(0, (int)x);
  x += (uint32_t)dpp16<0x118>(0, (int)x);
  return x;
}
__device__ __forceinline__ int row16_incl_max(int x) {
  x = max(x, dpp16<0x111>(INT_MIN, x));
  x = max(x, dpp16<0x112>(INT_MIN, x));
  x = max(x, dpp16<0x114>(INT_MIN, x));
  x = max(x, dpp16<0x118>(INT_MIN, x));
  return x;
}
// every lane of the 16-lane row gets the row's max / min / sum (quad swaps, half mirror, mirror)
__device__ __forceinline__ int row16_max(int x) {
  x = max(x, dpp16<0xB1>(x, x));
  x = max(x, dpp16<0x4E>(x, x));
  x = max(x, dpp16<0x141>(x, x));
  x = max(x, dpp16<0x140>(x, x));
  return x;
}
__device__ __forceinline__ int row16_min(int x) {
  x = min(x, dpp16<0xB1>(x, x));
  x = min(x, dpp16<0x4E>(x, x));
  x = min(x, dpp16<0x141>(x, x));
  x = min(x, dpp16<0x140>(x, x));
  return x;
}
__device__ __forceinline__ uint32_t row16_sum(uint32_t x) {
  x += (uint32_t)dpp16<0xB1>(0, (int)x);
  x += (uint32_t)dpp16<0x4E>(0, (int)x);
  x += (uint32_t)dpp16<0x141>(0, (int)x);
  x += (uint32_t)dpp16<0x140>(0, (int)x);
  return x;
}

template <int RPW, bool PREDICT, bool V16>
__global__ __launch_bounds__(kBlock) void k_med_kstat16(Geom g, const uint64_t* __restrict__ planes,
                                                        uint32_t* __restrict__ sones, int4* __restrict__ krec,
                                                        uint32_t* __restrict__ kpos, uint32_t* __restrict__ zero) {
  if (blockIdx.x == 0 && threadIdx.x < kZeroWords) zero[threadIdx.x] = 0;  // the encoder's counters
  const int lane = lane_id(), q = lane & 15, grp = lane >> 4;
  const uint32_t wpp = (g.rows + RPW - 1) / RPW;  // waves per plane
  const uint64_t gw = (uint64_t)xcd_remap(blockIdx.x, gridDim.x) * kWaves + wave_id();
  if (gw >= (uint64_t)wpp * g.nplanes) return;  // whole wave
  const uint32_t plane = (uint32_t)(gw / wpp), r0 = (uint32_t)(gw % wpp) * RPW;
  const uint64_t* pl = planes + (uint64_t)plane * g.plane_words;
  const uint32_t w0 = 4 * (uint32_t)q;
  const uint32_t nr = min((uint32_t)RPW, g.rows - r0);
  // the group's row and the row above; the next four rows' loads are in flight while these are used
  auto load = [&](uint32_t rb, uint64_t (&P)[4], uint64_t (&U)[4]) {
    const uint32_t rr = rb + (uint32_t)grp < nr ? r0 + rb + (uint32_t)grp : r0;
    if constexpr (V16) {  // 16-byte aligned rows holding whole lanes: two 16-byte loads per row
      const uint32_t wc = w0 < g.used ? w0 : 0;
      const ulonglong2* p2 = reinterpret_cast<const ulonglong2*>(pl + (uint64_t)rr * g.wpr + wc);
      const ulonglong2 a = p2[0], b = p2[1];
      P[0] = a.x; P[1] = a.y; P[2] = b.x; P[3] = b.y;
      if (PREDICT && rr) {
        const ulonglong2* u2 = reinterpret_cast<const ulonglong2*>(pl + (uint64_t)(rr - 1) * g.wpr + wc);
        const ulonglong2 c = u2[0], d = u2[1];
        U[0] = c.x; U[1] = c.y; U[2] = d.x; U[3] = d.y;
      } else {
        U[0] = U[1] = U[2] = U[3] = 0;
      }
      return;
    }
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      const uint32_t w = w0 + i, wc = w < g.used ? w : g.used - 1;
      P[i] = pl[(uint64_t)rr * g.wpr + wc];
      U[i] = (PREDICT && rr) ? pl[(uint64_t)(rr - 1) * g.wpr + wc] : 0ull;
    }
  };
  uint64_t P[4], U[4];
  load(0, P, U);
  for (uint32_t rb = 0; rb < nr; rb += 4) {
    const uint32_t row = r0 + rb + (uint32_t)grp;
    const bool in = rb + (uint32_t)grp < nr;
    const uint32_t rr = in ? row : r0;  // (out-of-range groups recompute a valid row, store nothing)
    uint64_t NP[4], NU[4];
    if (rb + 4 < nr) load(rb + 4, NP, NU);
    uint64_t D[4];
#pragma unroll
    for (int i = 0; i < 4; ++i) D[i] = P[i] ^ U[i];
    // D word left of the lane: lane q - 1's last (q = 0: 0), inside the 16-lane row
    const uint64_t dl = ((uint64_t)(uint32_t)dpp16<0x111>(0, (int)(uint32_t)(D[3] >> 32)) << 32) |
                        (uint32_t)dpp16<0x111>(0, (int)(uint32_t)D[3]);
    LaneK k;
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      const uint32_t w = w0 + i;
      uint64_t R = D[i];
      if constexpr (PREDICT) {
        R = D[i] ^ ((D[i] >> 1) | ((i ? D[i - 1] : dl) << 63));
        if (rr == 0 && w == 0) R &= ~BIC_MSB;  // pred.cpp never writes pP(0,0)
      }
      R = w < g.used ? (w == g.used - 1 ? R & g.trail : R) : 0;
      lanek_word(k, R, (int32_t)(w * 64));
    }
    // the row's record (lanek_store inside the 16-lane row)
    const uint32_t inc = row16_incl_sum(k.ones);
    const int32_t base = (int32_t)(inc - k.ones);
    const int mx = row16_incl_max(k.last);
    const int32_t before = dpp16<0x111>(-1, mx);  // the last 1 of the lanes before (-1: none)
    uint32_t chg = k.chg;
    int32_t first = -1;
    if (k.ones) {
      if (before >= 0) chg += (uint32_t)((before ^ k.first) & 1);
      else first = k.first;
    }
    const int32_t q0 = row16_max(k.ones ? k.q0 - 2 * base : -kNoOnes);
    const int32_t qh = row16_max(k.ones ? k.qh - 3 * base : -kNoOnes);
    const int32_t ql = row16_min(k.ones ? k.ql - 2 * base : kNoOnes);
    const uint32_t c = row16_sum(chg);
    const int32_t f = row16_max(first);
    const uint32_t tot = row16_sum(k.ones);
    const int32_t last = row16_max(k.last);
    if (q == 0 && in) {
      const uint64_t id = (uint64_t)plane * g.rows + row;
      krec[id] = make_int4(q0, qh, ql, (int32_t)(tot | (c << 16)));
      kpos[id] = ((uint32_t)f & 0xffffu) | ((uint32_t)last << 16);
      sones[id] = tot;
    }
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      P[i] = NP[i];
      U[i] = NU[i];
    }
  }
}

void launch_row_ones(hipStream_t s, const Geom& g, const uint64_t* planes, int predict, uint32_t* sones,
                     int4* krec, uint32_t* kpos, uint32_t* zero) {
  constexpr int RPW = 8;
  const uint32_t wpp = (g.rows + RPW - 1) / RPW;
  const uint32_t grid = (uint32_t)(((uint64_t)wpp * g.nplanes + kWaves - 1) / kWaves);
#define BIC_KST(LW, P) k_med_kstat<LW, RPW, P><<<grid, kBlock, 0, s>>>(g, planes, sones, krec, kpos, zero)
  if (g.used <= 64) {  // four rows per wave
    constexpr int R16 = 16;
    const uint32_t wpp16 = (g.rows + R16 - 1) / R16;
    const uint32_t grid16 = (uint32_t)(((uint64_t)wpp16 * g.nplanes + kWaves - 1) / kWaves);
    // 16-byte loads when every lane's four words lie inside the row pitch at 16-byte alignment
    const bool v16 = g.wpr % 4 == 0 && g.used % 4 == 0 && reinterpret_cast<uintptr_t>(planes) % 16 == 0;
#define BIC_K16(P, V) k_med_kstat16<R16, P, V><<<grid16, kBlock, 0, s>>>(g, planes, sones, krec, kpos, zero)
    if (predict) { if (v16) BIC_K16(true, true); else BIC_K16(true, false); }
    else { if (v16) BIC_K16(false, true); else BIC_K16(false, false); }
#undef BIC_K16
  }
  else if (g.used <= 128) { if (predict) BIC_KST(2, true); else BIC_KST(2, false); }
  else { if (predict) BIC_KST(4, true); else BIC_KST(4, false); }
#undef BIC_KST
}

// From the gray image (bic_encode_gray: bitplane_tool.cpp:24-30 and the count pass in one read):
// one wave per strip of 64 plane words (4096 columns) and gray_rows_per_wave() rows; lane l owns word
// 64 s + l of strip s: four 16-byte loads give its 64 pixels (load64_mis when the rows are not
// 16-byte aligned), K1's 8x8 transposes one word per plane. The med residual (pred.cpp:3-15) needs
// the row above and the pixel left of the word (lane l - 1's last; lane 0 of strip s > 0 loads the
// byte before the strip): with prediction and planes = NULL it is formed on the bytes (BYTEMED, one
// row per wave, the residual planes stored); with the planes returned, from the plane words (four
// rows per wave, the row above's words carried, the next row's loads in flight); without prediction
// R = P. One k statistics record per (plane, row,
// strip) (all planes' records in one transposed pass, strip_records; row_kstats combines a row's
// strips). The gray rows must hold used * 64 readable bytes (pitch >= used * 64; gray_rows_supported).
#ifndef BIC_GRAY_ROWS
#define BIC_GRAY_ROWS 4
#endif
// rows per wave: the plane-word form carries the row above's plane words from row to row (four rows,
// one transpose of the row above per wave); the byte-domain med (BYTEMED below) needs only the row
// above's bytes, so one row per wave (53 VGPRs, up to 8 waves per SIMD: C3 count pass 150 -> 135 us)
#ifndef BIC_GRAY_ROWS_BM
#define BIC_GRAY_ROWS_BM 1
#endif
constexpr int kGrayRowsP = BIC_GRAY_ROWS, kGrayRowsBM = BIC_GRAY_ROWS_BM;
uint32_t gray_strips(const Geom& g) { return (g.used + 63) / 64; }

// out[b] = bytes b of w0..w3, w0's in the most significant byte (a 4x4 byte transpose)
__device__ __forceinline__ void perm_t4(uint32_t w0, uint32_t w1, uint32_t w2, uint32_t w3, uint32_t (&out)[4]) {
  const uint32_t a01 = __builtin_amdgcn_perm(w0, w1, 0x04000501u), b01 = __builtin_amdgcn_perm(w0, w1, 0x06020703u);
  const uint32_t a23 = __builtin_amdgcn_perm(w2, w3, 0x04000501u), b23 = __builtin_amdgcn_perm(w2, w3, 0x06020703u);
  out[0] = __builtin_amdgcn_perm(a01, a23, 0x07060302u);
  out[1] = __builtin_amdgcn_perm(a01, a23, 0x05040100u);
  out[2] = __builtin_amdgcn_perm(b01, b23, 0x07060302u);
  out[3] = __builtin_amdgcn_perm(b01, b23, 0x05040100u);
}

// transpose8x8 of bswap64(x1 << 32 | x0) on 32-bit halves with v_bitop3 (gfx950): the first two
// stages stay inside each half, the third moves nibbles between them; 21 VALU + 2 v_perm instead of
// the 64-bit form's ~29 (whose last stage the compiler turns into a 64-bit multiply).
__device__ __forceinline__ uint64_t transpose8x8_bs(uint32_t x0, uint32_t x1) {
  uint32_t hi = __builtin_bswap32(x0), lo = __builtin_bswap32(x1);
  uint32_t t;
  t = __builtin_amdgcn_bitop3_b32(lo, lo >> 7, 0x00AA00AAu, 0x28);  // (a ^ b) & c
  lo = __builtin_amdgcn_bitop3_b32(lo, t, t << 7, 0x96);           // a ^ b ^ c
  t = __builtin_amdgcn_bitop3_b32(hi, hi >> 7, 0x00AA00AAu, 0x28);
  hi = __builtin_amdgcn_bitop3_b32(hi, t, t << 7, 0x96);
  t = __builtin_amdgcn_bitop3_b32(lo, lo >> 14, 0x0000CCCCu, 0x28);
  lo = __builtin_amdgcn_bitop3_b32(lo, t, t << 14, 0x96);
  t = __builtin_amdgcn_bitop3_b32(hi, hi >> 14, 0x0000CCCCu, 0x28);
  hi = __builtin_amdgcn_bitop3_b32(hi, t, t << 14, 0x96);
  t = __builtin_amdgcn_bitop3_b32(lo, hi << 4, 0xF0F0F0F0u, 0x28);
  lo ^= t;
  hi ^= t >> 4;
  return ((uint64_t)hi << 32) | lo;
}

// FULL: every lane's word lies inside the row and the row has no pad bits (no mask)
template <bool FULL = false>
__device__ __forceinline__ void gray_to_planes(const uint4 (&v)[4], uint64_t (&pw)[8], uint64_t mask) {
  uint64_t T[8];
#pragma unroll
  for (int i = 0; i < 4; ++i) {
    T[2 * i] = transpose8x8_bs(v[i].x, v[i].y);
    T[2 * i + 1] = transpose8x8_bs(v[i].z, v[i].w);
  }
  // byte b of T[g8] -> byte 7 - g8 of pw[b]: four 4x4 byte transposes, 8 v_perm_b32 each
  uint32_t XL[4], YL[4], XH[4], YH[4];
  perm_t4((uint32_t)T[0], (uint32_t)T[1], (uint32_t)T[2], (uint32_t)T[3], XL);
  perm_t4((uint32_t)T[4], (uint32_t)T[5], (uint32_t)T[6], (uint32_t)T[7], YL);
  perm_t4((uint32_t)(T[0] >> 32), (uint32_t)(T[1] >> 32), (uint32_t)(T[2] >> 32), (uint32_t)(T[3] >> 32), XH);
  perm_t4((uint32_t)(T[4] >> 32), (uint32_t)(T[5] >> 32), (uint32_t)(T[6] >> 32), (uint32_t)(T[7] >> 32), YH);
#pragma unroll
  for (int b = 0; b < 4; ++b) {
    pw[b] = ((uint64_t)XL[b] << 32) | YL[b];
    pw[4 + b] = ((uint64_t)XH[b] << 32) | YH[b];
    if constexpr (!FULL) {
      pw[b] &= mask;
      pw[4 + b] &= mask;
    }
  }
}

// NP8: every plane of the image (no plane-count tests in the row loop)
#ifndef BIC_DIAG_GS
#define BIC_DIAG_GS 0
#endif
#ifndef BIC_GS_NT
#define BIC_GS_NT 0  // the count pass's EG words: 1 = non-temporal stores
#endif
__device__ __forceinline__ void eg_store(uint64_t* p, uint64_t v) {
  if constexpr (BIC_GS_NT) __builtin_nontemporal_store(v, p);
  else *p = v;
}
#ifndef BIC_GRAY_PREFETCH
#define BIC_GRAY_PREFETCH 1
#endif
constexpr bool kGrayPrefetch = BIC_GRAY_PREFETCH != 0;  // the next row's pixels loaded during this row
// BYTEMED (residual planes stored, planes = NULL in bic_encode_gray): bitplane extraction is linear over
// XOR, so the med residual is formed on the gray bytes -- G = row ^ row above, H = G ^ (G one pixel to
// the left) -- and ONE transpose of H gives every plane's R (pred.cpp:3-15: R = P ^ up ^ left ^ up-left).
// The row above is kept as bytes (no transpose of it, also none for the row above the wave's first row).
#ifndef BIC_GRAY_BYTEMED
#define BIC_GRAY_BYTEMED 1
#endif
constexpr bool kGrayByteMed = BIC_GRAY_BYTEMED != 0;
// EGS (FULL strips of rows of whole strips, BM): the EG stream instead of R (eg.cpp:20-37 with the
// block size fixed at 1: per row ~R then the end-of-row '1'), in the uniform layout -- bit 0 a '1', row
// r at bit r (cols + 1) + 1 of plane b's slot (word b * eg_stride) -- which is the stream but for one
// bit (bic_fused.hip eg_fix_bit). With the strip's first bit at offset e of a word, lane l stores the
// word that starts inside its own row word: its bits and lane l + 1's; lane 63's word crosses the
// strip's end, so the wave also forms the first word of what follows -- the next strip's, or after
// the row's '1' the next row's -- from one pixel per lane of that segment (two byte loads, the med on
// the bytes, one ballot per plane): every stream word is stored whole, by exactly one wave, and the
// wave of row 0's first strip also stores word 0 (the stream's first bit, then the row's first bits).
template <bool PREDICT, bool STORE_R>
constexpr int gray_rows_per_wave() { return kGrayByteMed && PREDICT && STORE_R ? kGrayRowsBM : kGrayRowsP; }
// 64 bytes from src at any alignment (MIS: src not 16-byte aligned): the aligned 16-byte chunks that
// hold them (never a chunk without one of them: no read past the buffer's last page), realigned by
// the offset (the same for every lane of a wave: w * 64 is a multiple of 16)
__device__ __forceinline__ void load64_mis(const uint8_t* src, uint4 (&v)[4]) {
  const uintptr_t a = reinterpret_cast<uintptr_t>(src);
  const uint32_t mis = (uint32_t)(a & 15), bs = mis & 3, dq = mis >> 2;
  const uint4* b = reinterpret_cast<const uint4*>(src - mis);  // (pointer arithmetic: stays a global load)
  uint32_t in[20];
#pragma unroll
  for (int q = 0; q < 4; ++q) {
    const uint4 x = b[q];
    in[4 * q] = x.x;
    in[4 * q + 1] = x.y;
    in[4 * q + 2] = x.z;
    in[4 * q + 3] = x.w;
  }
  const uint4 x4 = mis ? b[4] : make_uint4(0, 0, 0, 0);
  in[16] = x4.x;
  in[17] = x4.y;
  in[18] = x4.z;
  in[19] = x4.w;
  // out dword d = bytes 4 (d + dq) + bs ..: one wave-uniform case per dword offset (static indices)
#define BIC_MIS_CASE(DQ)                                                                                    \
  case DQ:                                                                                                  \
    _Pragma("unroll") for (int q = 0; q < 4; ++q) v[q] =                                                    \
        make_uint4(__builtin_amdgcn_alignbyte(in[4 * q + DQ + 1], in[4 * q + DQ], bs),                     \
                   __builtin_amdgcn_alignbyte(in[4 * q + DQ + 2], in[4 * q + DQ + 1], bs),                 \
                   __builtin_amdgcn_alignbyte(in[4 * q + DQ + 3], in[4 * q + DQ + 2], bs),                 \
                   __builtin_amdgcn_alignbyte(in[4 * q + DQ + 4], in[4 * q + DQ + 3], bs));                \
    break;
  switch (dq) {
    BIC_MIS_CASE(0)
    BIC_MIS_CASE(1)
    BIC_MIS_CASE(2)
    default: BIC_MIS_CASE(3)
  }
#undef BIC_MIS_CASE
}

template <bool PREDICT, bool FULL, bool STORE_R, bool NP8, bool EGS, bool MIS = false>
__device__ __forceinline__ void gray_strip_rows(const uint8_t* __restrict__ gray, size_t pitch, const Geom& g,
                                                uint32_t ns, uint32_t s, uint32_t r0, uint32_t plane0,
                                                uint64_t* __restrict__ planes, uint32_t* __restrict__ sones,
                                                int4* __restrict__ krec, uint32_t* __restrict__ kpos, uint32_t* tw,
                                                uint64_t* __restrict__ out_e, uint64_t eg_stride) {
  const int lane = lane_id();
  const int np = NP8 ? 8 : (int)g.nplanes;
  const uint32_t w = s * 64 + lane;
  const bool in = FULL || w < g.used;
  const uint64_t mask = FULL ? ~0ull : in ? (w == g.used - 1 ? g.trail : ~0ull) : 0ull;
  // the word's 64 pixels, and (lane 0 of strips s > 0) the pixel before the strip
  auto load = [&](uint32_t row, uint4 (&v)[4], uint32_t& lb) {
    const uint8_t* src = gray + (uint64_t)row * pitch + (uint64_t)w * 64;
    if constexpr (MIS) {
      if (in) load64_mis(src, v);
      else
#pragma unroll
        for (int q = 0; q < 4; ++q) v[q] = make_uint4(0, 0, 0, 0);
    } else {
#pragma unroll
      for (int q = 0; q < 4; ++q) v[q] = in ? reinterpret_cast<const uint4*>(src)[q] : make_uint4(0, 0, 0, 0);
    }
    lb = (lane == 0 && s > 0) ? (uint32_t)src[-1] : 0u;
    if (plane0) {  // planes plane0.. of the range: every pixel's bits shifted down (a wave-uniform branch)
      const uint32_t m = 0x01010101u * (0xffu >> plane0);
#pragma unroll
      for (int q = 0; q < 4; ++q) v[q] = make_uint4((v[q].x >> plane0) & m, (v[q].y >> plane0) & m,
                                                    (v[q].z >> plane0) & m, (v[q].w >> plane0) & m);
      lb >>= plane0;
    }
  };
  constexpr bool BM = kGrayByteMed && PREDICT && STORE_R;
  uint64_t up[8];
#pragma unroll
  for (int b = 0; b < 8; ++b) up[b] = 0;
  uint32_t ulast = 0, ulb = 0;  // the row above's last pixel of the word / pixel before the strip
  uint4 cur[4], upb[4];         // (BM: the row above's bytes)
#pragma unroll
  for (int q = 0; q < 4; ++q) upb[q] = make_uint4(0, 0, 0, 0);
  uint32_t clb;
  if (PREDICT && r0) {
    load(r0 - 1, cur, ulb);
    if constexpr (BM) {
#pragma unroll
      for (int q = 0; q < 4; ++q) upb[q] = cur[q];
    } else {
      gray_to_planes<FULL>(cur, up, mask);
      ulast = cur[3].w >> 24;
    }
  }
  load(r0, cur, clb);
  const uint32_t nr = min((uint32_t)gray_rows_per_wave<PREDICT, STORE_R>(), g.rows - r0);
  for (uint32_t r = 0; r < nr; ++r) {
    const uint32_t row = r0 + r;
    uint4 nxt[4];
    uint32_t nlb = 0;
    if (kGrayPrefetch && r + 1 < nr) load(row + 1, nxt, nlb);
    // EGS: the D byte of pixel `lane` of the segment after this strip (the next strip of the row, or
    // the next row's first pixels; none after the last row)
    const bool lastS = s + 1 == ns;
    const uint32_t rn = lastS ? row + 1 : row;
    uint32_t gn = 0;
    if (EGS && FULL && rn < g.rows) {
      const uint8_t* cp = gray + (uint64_t)rn * pitch + (lastS ? 0u : (s + 1) * 4096u) + lane;
      uint32_t cb = cp[0], ub = rn ? cp[-(int64_t)pitch] : 0u;
      gn = (cb ^ ub) >> plane0;
    }
    // D bits (8 planes per byte) of the pixel left of the word: lane l - 1's last, or the strip's
    // preceding pixel for lane 0 (0 at column 0)
    uint64_t pw[8];
    uint32_t left = 0;
    if constexpr (BM) {
      // G = D bytes (8 planes per byte), H = G ^ G one pixel left: H's planes are R
      uint32_t gd[16];
#pragma unroll
      for (int q = 0; q < 4; ++q) {
        gd[4 * q] = cur[q].x ^ upb[q].x;
        gd[4 * q + 1] = cur[q].y ^ upb[q].y;
        gd[4 * q + 2] = cur[q].z ^ upb[q].z;
        gd[4 * q + 3] = cur[q].w ^ upb[q].w;
      }
      uint32_t gl = (uint32_t)__builtin_amdgcn_update_dpp(0, (int)(gd[15] >> 24), 0x138, 0xf, 0xf, true);
      if (lane == 0) gl = clb ^ ulb;  // the D byte before the strip (0 at column 0)
      uint32_t hd[16];
      hd[0] = gd[0] ^ __builtin_amdgcn_alignbyte(gd[0], gl << 24, 3);
#pragma unroll
      for (int d = 1; d < 16; ++d) hd[d] = gd[d] ^ __builtin_amdgcn_alignbyte(gd[d], gd[d - 1], 3);
      if (row == 0 && w == 0) hd[0] &= ~0xffu;  // pred.cpp never writes pP(0,0)
      if constexpr (EGS && FULL) {  // the next segment's residual bytes: left of its first pixel this
                                    // strip's last one (same row), or none (a row's first pixel)
        uint32_t gl2 = (uint32_t)__builtin_amdgcn_update_dpp(0, (int)gn, 0x138, 0xf, 0xf, true);
        if (lane == 0) gl2 = lastS ? 0u : (uint32_t)__builtin_amdgcn_readlane((int)gd[15], 63) >> 24;
        gn = (gn ^ gl2) & 0xffu;
      }
      uint4 hv[4];
#pragma unroll
      for (int q = 0; q < 4; ++q) hv[q] = make_uint4(hd[4 * q], hd[4 * q + 1], hd[4 * q + 2], hd[4 * q + 3]);
      gray_to_planes<FULL>(hv, pw, mask);
#pragma unroll
      for (int q = 0; q < 4; ++q) upb[q] = cur[q];
      ulb = clb;
    } else {
      const uint32_t cl = cur[3].w >> 24;
      const uint32_t dl = (PREDICT && row) ? cl ^ ulast : cl;
      left = (uint32_t)__builtin_amdgcn_update_dpp(0, (int)dl, 0x138, 0xf, 0xf, true);
      if (lane == 0) left = (PREDICT && row) ? clb ^ ulb : clb;
      ulast = cl;
      ulb = clb;
      gray_to_planes<FULL>(cur, pw, mask);
    }
    uint32_t* tb = tw;
    // EG: the strip's first row bit (wave-uniform shift; lane l's word starts 64 l bits later)
    const uint64_t ep = (uint64_t)row * (g.cols + 1) + 1 + (uint64_t)s * 4096;
    const uint32_t esh = (uint32_t)(ep & 63);
    uint64_t* eo = out_e + (ep >> 6) + lane;
#pragma unroll
    for (int b = 0; b < 8; ++b) {
      if (!NP8 && b >= np) break;
      if (!STORE_R && in) planes[(uint64_t)b * g.plane_words + (uint64_t)row * g.wpr + w] = pw[b];
      uint64_t R = pw[b];
      if constexpr (PREDICT && !BM) {
        const uint64_t D = pw[b] ^ up[b];
        R = D ^ ((D >> 1) | ((uint64_t)((left >> b) & 1u) << 63));
        if constexpr (!FULL) R &= mask;
        if (row == 0 && w == 0) R &= ~BIC_MSB;  // pred.cpp never writes pP(0,0)
        up[b] = pw[b];
      }
      if (!EGS && STORE_R && in) planes[(uint64_t)b * g.plane_words + (uint64_t)row * g.wpr + w] = R;
      if constexpr (EGS && FULL) {
        const uint64_t E = ~R;
        // the 64 stream bits after this strip's: the next strip's first word, or the row's '1' and the
        // next row's first 63 bits (the '1' alone after the last row)
        uint64_t N = ~__builtin_bitreverse64(__ballot((gn >> b) & 1u));
        if (lastS) N = BIC_MSB | (rn < g.rows ? N >> 1 : 0ull);
        uint64_t* eb = eo + (uint64_t)b * eg_stride;
#if BIC_DIAG_GS == 1  // diagnostic build only (wrong output): every wave's EG words to one 1 KB block
        eb = out_e + (uint64_t)b * 128 + lane;
#endif
        if (esh == 0) {
          eg_store(eb, bswap64(E));
          if (lastS && lane == 63) eb[1] = bswap64(N);  // the word the '1' opens (the next row's first)
        } else {
          uint64_t En = ((uint64_t)(uint32_t)__builtin_amdgcn_update_dpp(0, (int)(E >> 32), 0x130, 0xf, 0xf, true) << 32) |
                        (uint32_t)__builtin_amdgcn_update_dpp(0, (int)(uint32_t)E, 0x130, 0xf, 0xf, true);
          if (lane == 63) En = N;
          eg_store(eb + 1, bswap64(funnel64(E, En, esh)));
          if (row == 0 && s == 0 && lane == 0) eb[0] = bswap64(BIC_MSB | (E >> 1));  // stream bit 0, row 0
        }
      }
      strip_word_put(tb, b, R, (int32_t)(w * 64));
    }
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
    __builtin_amdgcn_wave_barrier();
    strip_records(tw, np, krec, kpos, sones, (uint64_t)row * ns + s, (uint64_t)g.rows * ns);
    __builtin_amdgcn_fence(__ATOMIC_ACQ_REL, "wavefront");  // the next row rewrites the table
    __builtin_amdgcn_wave_barrier();
    if constexpr (kGrayPrefetch) {
#pragma unroll
      for (int q = 0; q < 4; ++q) cur[q] = nxt[q];
      clb = nlb;
    } else if (r + 1 < nr) {
      load(row + 1, cur, clb);
    }
  }
}

#ifndef BIC_GRAY_WAVES
#define BIC_GRAY_WAVES 4
#endif
template <bool PREDICT, bool STORE_R, bool EGS, bool MIS = false>
__global__ __launch_bounds__(kBlock, BIC_GRAY_WAVES) void k_gray_strips(const uint8_t* __restrict__ gray, size_t pitch, Geom g,
                                                        uint32_t ns, uint32_t plane0, uint64_t* __restrict__ planes,
                                                        uint32_t* __restrict__ sones, int4* __restrict__ krec,
                                                        uint32_t* __restrict__ kpos, uint32_t* __restrict__ zero,
                                                        uint64_t* __restrict__ out_e, uint64_t eg_stride) {
  __shared__ __attribute__((aligned(16))) uint32_t tab[kWaves][1024];  // strip_word_put tables
  if (blockIdx.x == 0 && threadIdx.x < kZeroWords) zero[threadIdx.x] = 0;  // the encoder's counters
  // the wave's index as a scalar: its strip, rows, stream offsets and branches are then wave-uniform
  // values in SGPRs (scalar branches, no exec-mask juggling around the EG stores)
  const uint32_t wv = wave_id();
  uint32_t* tw = tab[wv];
  const uint64_t gw = (uint64_t)xcd_remap(blockIdx.x, gridDim.x) * kWaves + wv;
  const uint32_t s = (uint32_t)(gw % ns);  // the strips of one row block are neighbouring waves
  const uint32_t r0 = (uint32_t)(gw / ns) * gray_rows_per_wave<PREDICT, STORE_R>();
  if (r0 >= g.rows) return;  // whole wave
  // strips wholly inside a row without pad bits (every strip of C3) drop the masks and the lane tests
  if ((s + 1) * 64 <= g.used && g.trail == ~0ull && g.nplanes == 8)
    gray_strip_rows<PREDICT, true, STORE_R, true, EGS, MIS>(gray, pitch, g, ns, s, r0, plane0, planes, sones, krec, kpos,
                                                            tw, out_e, eg_stride);
  else if ((s + 1) * 64 <= g.used && g.trail == ~0ull)
    gray_strip_rows<PREDICT, true, STORE_R, false, EGS, MIS>(gray, pitch, g, ns, s, r0, plane0, planes, sones, krec, kpos,
                                                             tw, out_e, eg_stride);
  else if constexpr (!EGS)  // (EGS launches have whole strips only: gray_eg_supported)
    gray_strip_rows<PREDICT, false, STORE_R, false, false, MIS>(gray, pitch, g, ns, s, r0, plane0, planes, sones, krec,
                                                                kpos, tw, nullptr, 0);
}

bool gray_eg_supported(const Geom& g) { return g.trail == ~0ull && g.used % 64 == 0 && g.used / 64 <= kMaxStrips; }

// any gray alignment and pitch (rows not 16-byte aligned: load64_mis); every row must hold used * 64
// readable bytes
bool gray_rows_supported(const Geom& g, const void* gray, size_t pitch, const void* planes) {
  (void)gray;
  return g.used <= 256 && pitch >= (size_t)g.used * 64 && reinterpret_cast<uintptr_t>(planes) % 8 == 0;
}

void launch_gray_rows(hipStream_t s, const uint8_t* gray, size_t pitch, const Geom& g, int predict, int plane0,
                      uint64_t* planes, uint32_t* sones, int4* krec, uint32_t* kpos, uint32_t* zero, bool store_resid,
                      uint64_t* out_e, uint64_t eg_stride) {
  const uint32_t ns = gray_strips(g);
  const uint32_t rpw = predict && store_resid ? gray_rows_per_wave<true, true>() : gray_rows_per_wave<true, false>();
  const uint64_t units = (uint64_t)(g.rows + rpw - 1) / rpw;  // row groups per strip
  const uint32_t grid = (uint32_t)((units * ns + kWaves - 1) / kWaves);
  const bool mis = pitch % 16 != 0 || reinterpret_cast<uintptr_t>(gray) % 16 != 0;  // e.g. a P5 raster in its file
  const bool egs = out_e && predict && store_resid && gray_eg_supported(g);
#define BIC_GS(P, R, E, M) \
  k_gray_strips<P, R, E, M><<<grid, kBlock, 0, s>>>(gray, pitch, g, ns, (uint32_t)plane0, planes, sones, krec, kpos, \
                                                    zero, out_e, eg_stride)
#define BIC_GS2(P, R) { if (mis) BIC_GS(P, R, false, true); else BIC_GS(P, R, false, false); }
  if (egs) { if (mis) BIC_GS(true, true, true, true); else BIC_GS(true, true, true, false); }
  else if (predict) { if (store_resid) BIC_GS2(true, true) else BIC_GS2(true, false) }
  else BIC_GS2(false, false)  // without prediction R = P
#undef BIC_GS2
#undef BIC_GS
}

void launch_med_rows(hipStream_t s, const Geom& g, const uint64_t* planes, int predict, uint64_t* resid,
                     uint32_t* part, uint64_t* weight_out) {
  constexpr int RPW = 8;
  const uint32_t wpp = (g.rows + RPW - 1) / RPW;
  const uint32_t grid = (uint32_t)(((uint64_t)wpp * g.nplanes + kWaves - 1) / kWaves);
#define BIC_MED(NP, P) k_med_rows<NP, RPW, P><<<grid, kBlock, 0, s>>>(g, planes, resid, part)
  if (g.used <= 128) { if (predict) BIC_MED(1, true); else BIC_MED(1, false); }
  else { if (predict) BIC_MED(2, true); else BIC_MED(2, false); }
#undef BIC_MED
  if (weight_out) k_plane_weight<<<g.nplanes, 1024, 0, s>>>(part, wpp, weight_out);
}

bool med_rows_supported(const Geom& g, const void* planes, const void* resid) {
  return g.used <= 256 && (g.wpr % 2) == 0 && (reinterpret_cast<uintptr_t>(planes) % 16) == 0 &&
         (reinterpret_cast<uintptr_t>(resid) % 16) == 0;
}

template <int WPL>
static void launch_count_t(hipStream_t s, const Geom& g, const uint64_t* planes, int predict,
                           const ChunkScratch& cs, uint64_t* resid, uint64_t* weight_out) {
  const uint32_t grid = (uint32_t)((g.nchunks + kWaves - 1) / kWaves);
  if (predict) k_count<WPL, true><<<grid, kBlock, 0, s>>>(g, planes, cs, resid);
  else k_count<WPL, false><<<grid, kBlock, 0, s>>>(g, planes, cs, resid);
  if (weight_out) k_plane_weight<<<g.nplanes, 1024, 0, s>>>(cs.ones, g.chunks_per_plane, weight_out);
}

void launch_count(hipStream_t s, const Geom& g, const uint64_t* planes, int predict,
                  const ChunkScratch& cs, uint64_t* resid, uint64_t* weight_out) {
  if (g.wpl == 1) launch_count_t<1>(s, g, planes, predict, cs, resid, weight_out);
  else if (g.wpl == 2) launch_count_t<2>(s, g, planes, predict, cs, resid, weight_out);
  else launch_count_t<4>(s, g, planes, predict, cs, resid, weight_out);
}

// ------------------------------------------------------------------------------------
// K3: per-plane row scan -- sample index of each chunk's first 1 (ones before it + one
// EOL sample per earlier row), the last 1 before each chunk in its row, the plane's
// first residual 1 (for EG) and its ones total. One 1024-thread workgroup per plane,
// one thread per row.
// ------------------------------------------------------------------------------------
__global__ __launch_bounds__(1024) void k_scan_rows(Geom g, ChunkScratch cs) {
  __shared__ uint32_t tmp[17];
  __shared__ unsigned long long fmin;
  const uint32_t plane = blockIdx.x;
  const uint64_t cbase = (uint64_t)plane * g.chunks_per_plane;
  if (threadIdx.x == 0) fmin = ~0ull;
  uint32_t carry = 0;
  for (uint32_t r0 = 0; r0 < g.rows; r0 += blockDim.x) {
    const uint32_t row = r0 + threadIdx.x;
    uint32_t row_ones = 0;
    if (row < g.rows)
      for (uint32_t c = 0; c < g.cpr; ++c) row_ones += cs.ones[cbase + (uint64_t)row * g.cpr + c];
    uint32_t tot;
    const uint32_t before = block_excl_scan<uint32_t>(row_ones, tmp, tot) + carry;
    if (row < g.rows) {
      uint32_t n = before + row;  // ones before the row + one EOL sample per earlier row
      int jp = -1;
      bool seen = false;
      for (uint32_t c = 0; c < g.cpr; ++c) {
        const uint64_t id = cbase + (uint64_t)row * g.cpr + c;
        cs.nbase[id] = n;
        cs.jprev[id] = jp;
        const uint32_t o = cs.ones[id];
        n += o;
        if (o) {
          if (!seen) {
            atomicMin(&fmin, (unsigned long long)row * g.cols + (uint64_t)cs.first[id]);
            seen = true;
          }
          jp = cs.last[id];
        }
      }
    }
    carry += tot;
  }
  __syncthreads();
  if (threadIdx.x == 0) {
    cs.plane_F[plane] = fmin;
    cs.plane_ones[plane] = carry;
  }
}

void launch_scan_rows(hipStream_t s, const Geom& g, const ChunkScratch& cs) {
  k_scan_rows<<<g.nplanes, 1024, 0, s>>>(g, cs);
}

// ------------------------------------------------------------------------------------
// K4: Golomb bit lengths per word (and per chunk).
// ------------------------------------------------------------------------------------
template <int WPL, bool PREDICT>
__global__ __launch_bounds__(kBlock) void k_golomb_bits(Geom g, const uint64_t* __restrict__ planes,
                                                        ChunkScratch cs) {
  const ChunkId ci = chunk_id(g);
  if (!ci.ok) return;
  const uint32_t c0 = ci.c * g.wpc;
  RowCtx rc = row_ctx(planes, g, ci.plane, ci.row, c0);
  const int lane = lane_id();
  StepState st{cs.nbase[ci.id], cs.jprev[ci.id]};
  const uint32_t arow = ci.row * (g.cols + 1);  // A = row*(C+1) + jp + 1 - n
  uint64_t total = 0;
  uint32_t* wb = cs.word_bits + (uint64_t)ci.plane * g.words_used + (uint64_t)ci.row * g.used;
#pragma unroll
  for (int t = 0; t < WPL; ++t) {
    const uint32_t w = c0 + t * 64 + lane;
    uint64_t x = resid_word<PREDICT>(rc, g, ci.row, w);
    uint32_t n;
    int jp;
    step_prefix(x, w, st, n, jp);
    uint32_t bits = 0;
    while (x) {
      const int cz = __builtin_clzll(x);
      x ^= BIC_MSB >> cz;
      const int j = (int)(w * 64) + cz;
      const uint32_t s = (uint32_t)(j - jp - 1);
      const uint32_t k = golomb_k_state(n, arow + (uint32_t)(jp + 1) - n);
      bits += k + (s >> k) + 1;
      ++n;
      jp = j;
    }
    if (w == g.used - 1) {  // EOL sample: the row's trailing zeros
      const uint32_t s = (uint32_t)((int)g.cols - 1 - jp);
      const uint32_t k = golomb_k_state(n, arow + (uint32_t)(jp + 1) - n);
      bits += k + (s >> k) + 1;
    }
    if (w < g.used) wb[w] = bits;
    total += bits;
  }
  total = wave_sum_u64(total);
  if (lane == 0) cs.bits[ci.id] = total;
}

void launch_golomb_bits(hipStream_t s, const Geom& g, const uint64_t* planes, int predict,
                        const ChunkScratch& cs) {
  const uint32_t grid = (uint32_t)((g.nchunks + kWaves - 1) / kWaves);
#define BIC_GB(W)                                                                     \
  if (predict) k_golomb_bits<W, true><<<grid, kBlock, 0, s>>>(g, planes, cs);         \
  else k_golomb_bits<W, false><<<grid, kBlock, 0, s>>>(g, planes, cs);
  if (g.wpl == 1) { BIC_GB(1) }
  else if (g.wpl == 2) { BIC_GB(2) }
  else { BIC_GB(4) }
#undef BIC_GB
}

// ------------------------------------------------------------------------------------
// K5: chunk bit offsets per plane (exclusive scan), plane totals, overflow check, and
// zeroing of every chunk's first/last output word (the only words two chunks share;
// the emitter ORs into them and plain-stores everything in between).
// ------------------------------------------------------------------------------------
__global__ __launch_bounds__(1024) void k_golomb_offsets(Geom g, ChunkScratch cs, uint64_t* out,
                                                         uint64_t slot_words, uint64_t* plane_bits,
                                                         uint32_t* flags) {
  __shared__ uint64_t tmp[17];
  const uint32_t plane = blockIdx.x;
  const uint64_t cbase = (uint64_t)plane * g.chunks_per_plane;
  const uint64_t slot0 = (uint64_t)plane * slot_words * 64;
  const uint64_t cap = slot_words * 64;
  uint64_t carry = 0;
  for (uint64_t i0 = 0; i0 < g.chunks_per_plane; i0 += blockDim.x) {
    const uint64_t i = i0 + threadIdx.x;
    const uint64_t b = i < g.chunks_per_plane ? cs.bits[cbase + i] : 0;
    uint64_t tot;
    const uint64_t rel = block_excl_scan<uint64_t>(b, tmp, tot) + carry;
    if (i < g.chunks_per_plane) {
      cs.boff[cbase + i] = slot0 + rel;
      if (b && rel + b <= cap) {
        out[(slot0 + rel) / 64] = 0;
        out[(slot0 + rel + b - 1) / 64] = 0;
      }
    }
    carry += tot;
  }
  if (threadIdx.x == 0) {
    plane_bits[plane] = carry;
    if (carry > cap) atomicOr(&flags[0], 1u);
  }
}

void launch_golomb_offsets(hipStream_t s, const Geom& g, const ChunkScratch& cs, uint64_t* out,
                           uint64_t slot_words, uint64_t* plane_bits, uint32_t* flags) {
  k_golomb_offsets<<<g.nplanes, 1024, 0, s>>>(g, cs, out, slot_words, plane_bits, flags);
}

// ------------------------------------------------------------------------------------
// K6: Golomb emitter. Codeword = k-bit binary part (s mod 2^k, MSB-first), (s>>k) zeros,
// '1' (GolombCoder.cpp:22-25). The output is zero except for the binary parts and the
// terminators, so each lane ORs only those bits. A chunk whose output span fits the wave's
// 4 KB LDS window assembles it there (u32 LDS ORs, one per touched word per lane) and
// writes it out with coalesced stores; longer spans (very long zero runs) OR straight
// into global memory.
// ------------------------------------------------------------------------------------
template <int WPL, bool PREDICT, bool STAGED>
__device__ __forceinline__ void emit_chunk(const Geom& g, const uint64_t* planes, const ChunkScratch& cs,
                                           const ChunkId& ci, uint64_t cb, uint32_t* lds,
                                           unsigned long long* gout) {
  const uint32_t c0 = ci.c * g.wpc;
  RowCtx rc = row_ctx(planes, g, ci.plane, ci.row, c0);
  const int lane = lane_id();
  StepState st{cs.nbase[ci.id], cs.jprev[ci.id]};
  const uint32_t arow = ci.row * (g.cols + 1);
  const uint32_t* wb = cs.word_bits + (uint64_t)ci.plane * g.words_used + (uint64_t)ci.row * g.used;
  const uint64_t gbase = (cb >> 6) << 6;  // bit index of LDS word 0
  uint64_t off_carry = cb;
  LdsSink ls{lds, 0, 0};
  GlobalSink gs{gout, 0, 0};
#pragma unroll
  for (int t = 0; t < WPL; ++t) {
    const uint32_t w = c0 + t * 64 + lane;
    uint64_t x = resid_word<PREDICT>(rc, g, ci.row, w);
    uint32_t n;
    int jp;
    step_prefix(x, w, st, n, jp);
    const uint32_t bits = w < g.used ? wb[w] : 0;
    const uint32_t binc = wave_incl_sum_u32(bits);
    uint64_t off = off_carry + binc - bits;
    off_carry += lane63_u32(binc);
    const bool eol = (w == g.used - 1);
    while (x || eol) {
      int j;
      uint32_t s;
      if (x) {
        const int cz = __builtin_clzll(x);
        x ^= BIC_MSB >> cz;
        j = (int)(w * 64) + cz;
        s = (uint32_t)(j - jp - 1);
      } else {
        j = (int)g.cols;  // EOL: the row's trailing zeros
        s = (uint32_t)((int)g.cols - 1 - jp);
      }
      const uint32_t k = golomb_k_state(n, arow + (uint32_t)(jp + 1) - n);
      if constexpr (STAGED) emit_codeword(ls, (uint32_t)(off - gbase), s, k);
      else emit_codeword(gs, off, s, k);
      off += k + (s >> k) + 1;
      ++n;
      jp = j;
      if (j == (int)g.cols) break;
    }
  }
  if constexpr (STAGED) ls.flush();
  else gs.flush();
}

template <int WPL, bool PREDICT>
__global__ __launch_bounds__(kBlock) void k_golomb_emit(Geom g, const uint64_t* __restrict__ planes,
                                                        ChunkScratch cs, uint64_t* __restrict__ out,
                                                        uint64_t slot_words) {
  __shared__ __attribute__((aligned(16))) uint32_t lds_all[kWaves * kLdsWords];
  const ChunkId ci = chunk_id(g);
  if (!ci.ok) return;
  const int lane = lane_id();
  uint32_t* lds = lds_all + wave_id() * kLdsWords;
  const uint64_t L = cs.bits[ci.id];
  const uint64_t cb = cs.boff[ci.id];
  const uint64_t slot_end = ((uint64_t)ci.plane + 1) * slot_words * 64;
  if (L == 0 || cb + L > slot_end) return;  // empty chunk, or the plane overflowed its slot
  const uint64_t w_first = cb >> 6, w_last = (cb + L - 1) >> 6;
  const uint64_t span_words = w_last - w_first + 1;  // 64-bit words
  auto* gout = reinterpret_cast<unsigned long long*>(out);
  if (span_words * 2 <= (uint64_t)kLdsWords) {
    for (uint32_t i = lane; i < span_words * 2; i += 64) lds[i] = 0;
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
    __builtin_amdgcn_wave_barrier();
    emit_chunk<WPL, PREDICT, true>(g, planes, cs, ci, cb, lds, gout);
    __builtin_amdgcn_fence(__ATOMIC_ACQ_REL, "wavefront");
    __builtin_amdgcn_wave_barrier();
    for (uint32_t i = lane; i < span_words; i += 64) {
      const uint64_t v = ((uint64_t)lds[2 * i] << 32) | lds[2 * i + 1];
      const uint64_t be = bswap64(v);
      if (i == 0 || i == span_words - 1) {
        if (v) atomicOr(&gout[w_first + i], (unsigned long long)be);
      } else {
        out[w_first + i] = be;
      }
    }
  } else {
    for (uint64_t i = w_first + 1 + lane; i < w_last; i += 64) out[i] = 0;
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    emit_chunk<WPL, PREDICT, false>(g, planes, cs, ci, cb, lds, gout);
  }
}

void launch_golomb_emit(hipStream_t s, const Geom& g, const uint64_t* planes, int predict,
                        const ChunkScratch& cs, uint64_t* out, uint64_t slot_words) {
  const uint32_t grid = (uint32_t)((g.nchunks + kWaves - 1) / kWaves);
#define BIC_GE(W)                                                                               \
  if (predict) k_golomb_emit<W, true><<<grid, kBlock, 0, s>>>(g, planes, cs, out, slot_words); \
  else k_golomb_emit<W, false><<<grid, kBlock, 0, s>>>(g, planes, cs, out, slot_words);
  if (g.wpl == 1) { BIC_GE(1) }
  else if (g.wpl == 2) { BIC_GE(2) }
  else { BIC_GE(4) }
#undef BIC_GE
}

// ------------------------------------------------------------------------------------
// K7: EG as written (eg.cpp:20-37 with incBlockSize disabled): blockSize stays 1, so a run
// of len zeros costs len '1' bits, then '1' at EOL or '0' (+ one g=1 bit '0' on the plane's
// first non-EOL run, after which g = 0). The stream is therefore, per row, the complement of
// the residual row followed by '1', with a single '0' inserted after the plane's first
// residual 1. One thread per output word; no atomics, no pre-zeroing.
// ------------------------------------------------------------------------------------
template <bool PREDICT>
__device__ __forceinline__ uint64_t resid_word_at(const uint64_t* plane, const Geom& g, uint32_t i,
                                                  uint32_t w) {
  if (w >= g.used) return 0;
  const uint64_t* cur = plane + (uint64_t)i * g.wpr;
  uint64_t r = cur[w];
  if constexpr (PREDICT) {
    const uint64_t pl = w ? cur[w - 1] : 0;
    uint64_t u = 0, ul = 0;
    if (i) {
      u = (cur - g.wpr)[w];
      ul = w ? (cur - g.wpr)[w - 1] : 0;
    }
    r = r ^ u ^ ((r >> 1) | (pl << 63)) ^ ((u >> 1) | (ul << 63));
    if (i == 0 && w == 0) r &= ~BIC_MSB;
  }
  if (w == g.used - 1) r &= g.trail;
  return r;
}

// 64 bits of the complemented residual row i starting at column j (left-aligned).
template <bool PREDICT>
__device__ __forceinline__ uint64_t notresid_bits(const uint64_t* plane, const Geom& g, uint32_t i,
                                                  uint32_t j) {
  const uint32_t w = j >> 6, sh = j & 63;
  uint64_t v = resid_word_at<PREDICT>(plane, g, i, w) << sh;
  if (sh) v |= resid_word_at<PREDICT>(plane, g, i, w + 1) >> (64 - sh);
  return ~v;
}

// 64 bits of the base stream S0 (rows of cols+1 bits: ~R row then '1') from bit a.
template <bool PREDICT>
__device__ __forceinline__ uint64_t eg_window(const uint64_t* plane, const Geom& g, uint64_t a) {
  const uint64_t rowlen = (uint64_t)g.cols + 1;
  uint64_t i = a / rowlen;
  uint32_t j = (uint32_t)(a % rowlen);
  uint64_t out = 0;
  uint32_t filled = 0;
  while (filled < 64 && i < g.rows) {
    if (j < g.cols) {
      const uint32_t take = min(64u - filled, g.cols - j);
      uint64_t v = notresid_bits<PREDICT>(plane, g, (uint32_t)i, j);
      if (take < 64) v &= ~(~0ull >> take);
      out |= v >> filled;
      filled += take;
      j += take;
    }
    if (filled < 64 && j == g.cols) {
      out |= BIC_MSB >> filled;
      ++filled;
      ++i;
      j = 0;
    }
  }
  return out;
}

template <bool PREDICT>
__global__ __launch_bounds__(kBlock) void k_eg_emit(Geom g, const uint64_t* __restrict__ planes,
                                                    ChunkScratch cs, uint64_t* __restrict__ out,
                                                    uint64_t slot_words, uint64_t words_per_plane,
                                                    uint64_t* plane_bits, uint32_t* flags) {
  const uint64_t tid = (uint64_t)blockIdx.x * kBlock + threadIdx.x;
  const uint32_t plane = (uint32_t)(tid / words_per_plane);
  if (plane >= g.nplanes) return;
  const uint64_t o = tid % words_per_plane;
  const uint64_t F = cs.plane_F[plane];
  const bool hasF = F != ~0ull;
  const uint64_t bits = (uint64_t)g.rows * (g.cols + 1) + (hasF ? 1 : 0);
  const uint64_t nw = (bits + 63) / 64;
  if (o == 0) {
    plane_bits[plane] = bits;
    if (nw > slot_words) atomicOr(&flags[0], 1u);
  }
  if (nw > slot_words || o >= nw) return;
  const uint64_t* P = planes + (uint64_t)plane * g.plane_words;
  const uint64_t b0 = o * 64;
  uint64_t v;
  if (!hasF) {
    v = eg_window<PREDICT>(P, g, b0);
  } else {
    const uint64_t f0 = (F / g.cols) * ((uint64_t)g.cols + 1) + F % g.cols;  // S0 index of F
    if (b0 + 63 <= f0) {
      v = eg_window<PREDICT>(P, g, b0);
    } else if (b0 >= f0 + 1) {
      v = eg_window<PREDICT>(P, g, b0 - 1);
      if (b0 == f0 + 1) v &= ~BIC_MSB;  // the inserted '0'
    } else {
      const uint32_t q = (uint32_t)(f0 + 1 - b0);  // 1..63: position of the inserted '0'
      const uint64_t X = eg_window<PREDICT>(P, g, b0);
      // Y bit t = S0[b0 - 1 + t]; only bits t >= q+1 >= 2 are used, so at b0 = 0 X >> 1 serves
      const uint64_t Y = b0 ? eg_window<PREDICT>(P, g, b0 - 1) : (X >> 1);
      const uint64_t hi = ~(~0ull >> q);
      const uint64_t lo = (q == 63) ? 0ull : (~0ull >> (q + 1));
      v = (X & hi) | (Y & lo);
    }
  }
  // pad bits after the stream end are zero
  if (o == nw - 1 && (bits & 63)) v &= ~(~0ull >> (bits & 63));
  out[(uint64_t)plane * slot_words + o] = bswap64(v);
}

void launch_eg_emit(hipStream_t s, const Geom& g, const uint64_t* planes, int predict,
                    const ChunkScratch& cs, uint64_t* out, uint64_t slot_words,
                    uint64_t* plane_bits, uint32_t* flags) {
  const uint64_t wpp = ((uint64_t)g.rows * (g.cols + 1) + 1 + 63) / 64;
  const uint64_t total = wpp * g.nplanes;
  const uint32_t grid = (uint32_t)((total + kBlock - 1) / kBlock);
  if (predict)
    k_eg_emit<true><<<grid, kBlock, 0, s>>>(g, planes, cs, out, slot_words, wpp, plane_bits, flags);
  else
    k_eg_emit<false><<<grid, kBlock, 0, s>>>(g, planes, cs, out, slot_words, wpp, plane_bits, flags);
}

// ------------------------------------------------------------------------------------
// Sample coder: GolombCoder::codeSample over an array. Blocks of kSampPerBlk samples take a
// ticket; a first kernel runs two decoupled look-backs per block -- the sum of the samples
// before it (the coder's accumulated error A) and, once its lengths are known, its bit offset
// -- and zeroes the block's output words; a second kernel writes the codewords.
// ------------------------------------------------------------------------------------
#ifndef BIC_SAMP_ITEMS
#define BIC_SAMP_ITEMS 4  // C5 (65,536 samples): 4 per thread 13 us for both launches, 8: 15.5, 16: 20.5
#endif
constexpr int kItems = BIC_SAMP_ITEMS;
constexpr uint32_t kSampPerBlk = kBlock * kItems;

__global__ __launch_bounds__(kBlock) void k_samp_scan(const uint32_t* __restrict__ s, size_t n, uint64_t n0,
                                                      uint64_t a0, unsigned bit0, SampleScratch ss,
                                                      uint64_t* out, size_t cap_words, uint64_t* bits_out,
                                                      uint32_t* flags, uint32_t nblk) {
  __shared__ uint64_t tmp[17];
  __shared__ uint64_t sh[2];
  __shared__ uint32_t sh_blk;
  if (threadIdx.x == 0) sh_blk = atomicAdd(ss.counter, 1u);
  __syncthreads();
  const uint32_t blk = sh_blk;
  const uint64_t base = (uint64_t)blk * kSampPerBlk + (uint64_t)threadIdx.x * kItems;
  uint32_t v[kItems];
  uint64_t a = 0;
#pragma unroll
  for (int i = 0; i < kItems; ++i) {
    v[i] = base + i < n ? s[base + i] : 0;
    a += v[i];
  }
  uint64_t tot_a;
  const uint64_t ea = block_excl_scan<uint64_t>(a, tmp, tot_a);
  if (threadIdx.x < 64) {  // A before this block
    uint64_t A0 = a0;
    if (blk == 0) {
      if (threadIdx.x == 0) rec_store(&ss.a_rec[0], kInc | (a0 + tot_a));
    } else {
      if (threadIdx.x == 0) rec_store(&ss.a_rec[blk], kAgg | tot_a);
      A0 = lookback(ss.a_rec, 0, blk, flags);  // inclusive records carry a0
      if (threadIdx.x == 0) rec_store(&ss.a_rec[blk], kInc | (A0 + tot_a));
    }
    if (threadIdx.x == 0) sh[0] = A0;
  }
  __syncthreads();
  const uint64_t Ablk = sh[0];
  uint64_t AA = Ablk + ea, bits = 0;
#pragma unroll
  for (int i = 0; i < kItems; ++i) {
    if (base + i < n) {
      const uint64_t nn = n0 + base + i;
      if (nn >= 0x80000000ull || AA >= 0x80000000ull) atomicOr(&flags[1], 1u);
      const uint32_t k = golomb_k_state((uint32_t)nn, (uint32_t)AA);
      bits += k + (v[i] >> k) + 1;
      AA += v[i];
    }
  }
  uint64_t tot_b;
  block_excl_scan<uint64_t>(bits, tmp, tot_b);
  if (threadIdx.x < 64) {  // bit offset of this block (the stream starts at bit0)
    uint64_t B0 = bit0;
    if (blk == 0) {
      if (threadIdx.x == 0) rec_store(&ss.b_rec[0], kInc | (bit0 + tot_b));
    } else {
      if (threadIdx.x == 0) rec_store(&ss.b_rec[blk], kAgg | tot_b);
      B0 = lookback(ss.b_rec, 0, blk, flags);  // inclusive records carry bit0
      if (threadIdx.x == 0) rec_store(&ss.b_rec[blk], kInc | (B0 + tot_b));
    }
    if (threadIdx.x == 0) {
      sh[1] = B0;
      ss.blk_A[blk] = Ablk;
      ss.blk_off[blk] = B0;
      if (blk == nblk - 1) {
        bits_out[0] = B0 + tot_b - bit0;
        bits_out[1] = Ablk + tot_a - a0;
      }
    }
  }
  __syncthreads();
  // zero the words this block's codewords touch (within the caller's capacity); the words it
  // shares with its neighbours may be zeroed by either -- all of it before any codeword is OR'd
  if (!out) return;  // lengths only (bic_golomb_encode_samples with no output)
  const uint64_t B0 = sh[1];
  const uint64_t w_lo = blk == 0 ? 0 : B0 / 64, w_hi = (B0 + tot_b + 63) / 64;
  if (w_hi > cap_words && threadIdx.x == 0) atomicOr(&flags[0], 1u);
  for (uint64_t w = w_lo + threadIdx.x; w < w_hi && w < cap_words; w += kBlock) out[w] = 0;
}

__global__ __launch_bounds__(kBlock) void k_samp_emit(const uint32_t* __restrict__ s, size_t n, uint64_t n0,
                                                      SampleScratch ss, uint64_t* out, const uint64_t* total_bits,
                                                      unsigned bit0, size_t cap_words, const uint64_t* lpart,
                                                      uint32_t nlpart, uint64_t* lout) {
  __shared__ uint64_t tmp[17];
  if (lpart && blockIdx.x == 0) {  // the tile kernel's per-block length sums (bic_patch_encode stats[2])
    uint64_t l = 0;
    for (uint32_t i = threadIdx.x; i < nlpart; i += kBlock) l += lpart[i];
    uint64_t tot;
    block_excl_scan<uint64_t>(l, tmp, tot);
    if (threadIdx.x == 0) *lout = tot;
    __syncthreads();  // tmp is reused below
  }
  if ((bit0 + *total_bits + 63) / 64 > cap_words) return;  // overflow: write nothing (flagged)
  const uint32_t blk = blockIdx.x;
  const uint64_t base = (uint64_t)blk * kSampPerBlk + (uint64_t)threadIdx.x * kItems;
  uint32_t v[kItems];
  uint64_t a = 0;
#pragma unroll
  for (int i = 0; i < kItems; ++i) {
    v[i] = base + i < n ? s[base + i] : 0;
    a += v[i];
  }
  uint64_t tot;
  uint64_t A = ss.blk_A[blk] + block_excl_scan<uint64_t>(a, tmp, tot);
  uint64_t bits = 0;
  {
    uint64_t AA = A;
#pragma unroll
    for (int i = 0; i < kItems; ++i) {
      if (base + i < n) {
        const uint32_t k = golomb_k_state((uint32_t)(n0 + base + i), (uint32_t)AA);
        bits += k + (v[i] >> k) + 1;
        AA += v[i];
      }
    }
  }
  uint64_t off = ss.blk_off[blk] + block_excl_scan<uint64_t>(bits, tmp, tot);
  GlobalSink gs{reinterpret_cast<unsigned long long*>(out), 0, 0};
#pragma unroll
  for (int i = 0; i < kItems; ++i) {
    if (base + i < n) {
      const uint32_t k = golomb_k_state((uint32_t)(n0 + base + i), (uint32_t)A);
      emit_codeword(gs, off, v[i], k);
      off += k + (v[i] >> k) + 1;
      A += v[i];
    }
  }
  gs.flush();
}

size_t sample_scratch_bytes(size_t n) {
  const size_t nblk = (n + kSampPerBlk - 1) / kSampPerBlk + 1;
  return 256 + 4 * nblk * sizeof(uint64_t) + 256;
}
SampleScratch carve_sample_scratch(void* base, size_t n) {
  const size_t nblk = (n + kSampPerBlk - 1) / kSampPerBlk + 1;
  char* c = reinterpret_cast<char*>(base);
  uint64_t* p = reinterpret_cast<uint64_t*>(c + 256);
  SampleScratch ss;
  ss.counter = reinterpret_cast<uint32_t*>(c);
  ss.a_rec = p;
  ss.b_rec = p + nblk;
  ss.blk_A = p + 2 * nblk;
  ss.blk_off = p + 3 * nblk;
  ss.zero_bytes = 256 + 2 * nblk * sizeof(uint64_t);
  return ss;
}

void launch_golomb_samples(hipStream_t s, const uint32_t* samples, size_t n, uint64_t n0,
                           uint64_t a0, unsigned bit0, uint64_t* out, size_t cap_words,
                           uint64_t* bits_out, const SampleScratch& ss, uint32_t* flags, bool prezeroed,
                           const uint64_t* lpart, uint32_t nlpart, uint64_t* lout) {
  const uint32_t nblk = (uint32_t)((n + kSampPerBlk - 1) / kSampPerBlk);
  if (nblk == 0) {
    (void)launch_fill(s, bits_out, 0, 2 * sizeof(uint64_t));
    if (lpart) (void)launch_fill(s, lout, 0, sizeof(uint64_t));
    return;
  }
  if (!prezeroed) (void)launch_fill(s, ss.counter, 0, ss.zero_bytes);
  k_samp_scan<<<nblk, kBlock, 0, s>>>(samples, n, n0, a0, bit0, ss, out, cap_words, bits_out, flags, nblk);
  if (out) k_samp_emit<<<nblk, kBlock, 0, s>>>(samples, n, n0, ss, out, bits_out, bit0, cap_words, lpart, nlpart, lout);
}

// ------------------------------------------------------------------------------------
// K8: W x W tiles (compress7_test.cpp:184-275, R = 0). One lane per tile row, floor(64/W)
// tiles per wave; med inside the tile (out-of-tile neighbours 0, R(0,0) = 0).
// ------------------------------------------------------------------------------------
__global__ __launch_bounds__(kBlock) void k_tiles(const uint64_t* __restrict__ plane, uint32_t rows,
                                                  uint32_t cols, uint32_t wpr, uint32_t W, uint32_t nx,
                                                  uint32_t ntiles, const uint64_t* __restrict__ lentab,
                                                  uint32_t* weights, uint32_t* w_nonpred, uint32_t* w_pred,
                                                  uint8_t* modes, unsigned long long* resid,
                                                  unsigned long long* stats) {
  __shared__ uint32_t pc_o[kBlock], pc_O[kBlock];
  __shared__ uint8_t sel[kBlock];
  __shared__ uint64_t red[2][kWaves];
  const int lane = lane_id(), wave = (int)wave_id();
  const uint32_t tpw = 64 / W;
  const uint64_t gw = (uint64_t)blockIdx.x * kWaves + wave;
  const uint32_t tloc = lane / W, r = lane % W;
  const uint64_t tile = gw * tpw + tloc;
  const bool active = tloc < tpw && tile < ntiles;
  const uint64_t topW = W == 64 ? ~0ull : ~(~0ull >> W);
  uint64_t x = 0;
  uint32_t i = 0, j0 = 0;
  if (active) {
    const uint32_t ti = (uint32_t)(tile / nx), tj = (uint32_t)(tile % nx);
    i = ti * W + r;
    j0 = tj * W;
    const uint64_t* row = plane + (uint64_t)i * wpr;
    const uint32_t w = j0 >> 6, sh = j0 & 63;
    x = row[w] << sh;
    if (sh && sh + W > 64) x |= row[w + 1] >> (64 - sh);
    x &= topW;
  }
  uint64_t up = shfl_up_u64(x, 1);
  if (r == 0) up = 0;
  uint64_t R = (x ^ (x >> 1) ^ up ^ (up >> 1)) & topW;
  if (r == 0) R &= ~BIC_MSB;
  pc_o[threadIdx.x] = (uint32_t)__popcll(x);
  pc_O[threadIdx.x] = (uint32_t)__popcll(R);
  __syncthreads();
  uint64_t myL = 0, myW = 0;
  if (active && r == 0) {
    uint32_t wo = 0, wO = 0;
    for (uint32_t q = 0; q < W; ++q) {
      wo += pc_o[threadIdx.x + q];
      wO += pc_O[threadIdx.x + q];
    }
    const bool pred = lentab[wo] > lentab[wO];  // compress7_test.cpp:248
    const uint32_t wc = pred ? wO : wo;
    if (weights) weights[tile] = wc;
    if (w_nonpred) w_nonpred[tile] = wo;
    if (w_pred) w_pred[tile] = wO;
    if (modes) modes[tile] = pred ? 'O' : 'o';
    sel[threadIdx.x] = pred;
    myL = lentab[wc];
    myW = wc;
  }
  __syncthreads();
  if (resid && active) {
    const uint64_t v = sel[threadIdx.x - r] ? R : x;
    if (v) {
      const uint32_t w = j0 >> 6, sh = j0 & 63;
      unsigned long long* row = resid + (uint64_t)i * wpr;
      atomicOr(&row[w], (unsigned long long)(v >> sh));
      if (sh && sh + W > 64) atomicOr(&row[w + 1], (unsigned long long)(v << (64 - sh)));
    }
  }
  myL = wave_sum_u64(myL);
  myW = wave_sum_u64(myW);
  if (lane == 0) { red[0][wave] = myL; red[1][wave] = myW; }
  __syncthreads();
  if (threadIdx.x == 0) {
    uint64_t a = 0, b = 0;
    for (int q = 0; q < kWaves; ++q) { a += red[0][q]; b += red[1][q]; }
    if (a) atomicAdd(&stats[2], (unsigned long long)a);
    (void)b;
  }
}

// K8a: W x W tiles for W in {8, 16, 32, 64} (W divides 64, so no tile straddles a word). One
// wave covers a strip of W rows x 64 words: lane l owns word column l, i.e. 64/W tiles side by
// side, and walks the W rows with coalesced 512-byte loads (the row above stays in a register).
// The med inside a tile (out-of-tile neighbours 0, R(0,0) = 0) is R = D ^ (D >> 1 & ~F) with
// D = row ^ row-above and F the tiles' first-column bits. A second walk (cache-resident) writes
// the residual image word by word -- every word exactly once: no pre-zeroing, no atomics.
template <int W>
__global__ __launch_bounds__(kBlock) void k_tiles_aligned(const uint64_t* __restrict__ plane, uint32_t rows,
                                                          uint32_t cols, uint32_t wpr, uint32_t used, uint32_t nx,
                                                          const uint64_t* __restrict__ lentab, uint32_t* weights,
                                                          uint32_t* w_nonpred, uint32_t* w_pred, uint8_t* modes,
                                                          uint64_t* resid, unsigned long long* stats) {
  constexpr int T = 64 / W;
  const int lane = lane_id();
  const uint64_t gw = (uint64_t)blockIdx.x * kWaves + wave_id();
  const uint32_t groups = (used + 63) / 64;
  const uint32_t ty = (uint32_t)(gw / groups), w = (uint32_t)(gw % groups) * 64 + lane;
  if (ty >= rows / W) return;  // wave-uniform
  const bool act = w < used;
  uint64_t F = 0;  // first column of every tile in the word
#pragma unroll
  for (int j = 0; j < T; ++j) F |= BIC_MSB >> (j * W);
  const uint64_t* src = plane + (uint64_t)ty * W * wpr + (act ? w : 0);
  uint32_t co[T], cO[T];
#pragma unroll
  for (int j = 0; j < T; ++j) co[j] = cO[j] = 0;
  uint64_t up = 0;
#pragma unroll 8
  for (int r = 0; r < W; ++r) {
    const uint64_t x = act ? src[(uint64_t)r * wpr] : 0;
    const uint64_t d = x ^ up;
    uint64_t R = d ^ ((d >> 1) & ~F);
    if (r == 0) R &= ~F;  // compress7's med never writes a tile's R(0,0)
#pragma unroll
    for (int j = 0; j < T; ++j) {
      const uint64_t m = (W == 64) ? ~0ull : (((1ull << W) - 1) << (64 - W * (j + 1)));
      co[j] += (uint32_t)__popcll(x & m);
      cO[j] += (uint32_t)__popcll(R & m);
    }
    up = x;
  }
  uint64_t L = 0, keepR = 0;  // keepR: word mask of the tiles coded as residuals ('O')
#pragma unroll
  for (int j = 0; j < T; ++j) {
    const uint32_t col0 = w * 64 + j * W;
    if (!act || col0 >= cols) continue;
    const uint64_t tile = (uint64_t)ty * nx + col0 / W;
    const bool pred = lentab[co[j]] > lentab[cO[j]];  // compress7_test.cpp:248
    const uint32_t wc = pred ? cO[j] : co[j];
    if (weights) weights[tile] = wc;
    if (w_nonpred) w_nonpred[tile] = co[j];
    if (w_pred) w_pred[tile] = cO[j];
    if (modes) modes[tile] = pred ? 'O' : 'o';
    L += lentab[wc];
    if (pred) keepR |= (W == 64) ? ~0ull : (((1ull << W) - 1) << (64 - W * (j + 1)));
  }
  if (resid && act) {
    uint64_t* dst = resid + (uint64_t)ty * W * wpr + w;
    const uint64_t valid = w == used - 1 && (cols & 63) ? ~(~0ull >> (cols & 63)) : ~0ull;
    up = 0;
#pragma unroll 8
    for (int r = 0; r < W; ++r) {
      const uint64_t x = src[(uint64_t)r * wpr];
      const uint64_t d = x ^ up;
      uint64_t R = d ^ ((d >> 1) & ~F);
      if (r == 0) R &= ~F;
      dst[(uint64_t)r * wpr] = ((R & keepR) | (x & ~keepR)) & valid;
      up = x;
    }
  }
  L = wave_sum_u64(L);
  if (lane == 0 && L) atomicAdd(&stats[2], (unsigned long long)L);
}

// K8c: the aligned tile path with a strip of W rows split over a workgroup's 4 waves (W / 4 rows
// each, kept in registers), so a launch has 4x the waves of k_tiles_aligned (C5, 8192^2 at W = 32:
// 2048 waves instead of 512; the strip's serial row loads were its latency): per-wave partial tile
// counts meet in LDS, every wave takes the totals for its lanes' tiles and writes its rows of the
// residual image from registers. The tile length sum goes to lpart[block] (no atomics, no zeroed
// stats: the sample coder adds the parts); the first blocks zero the sample coder's scratch
// (`zero`, nzero words), so its launch needs no fill before it.
template <int W>
__global__ __launch_bounds__(256) void k_tiles_split(const uint64_t* __restrict__ plane, uint32_t rows, uint32_t cols,
                                                     uint32_t wpr, uint32_t used, uint32_t nx,
                                                     const uint64_t* __restrict__ lentab, uint32_t* weights,
                                                     uint32_t* w_nonpred, uint32_t* w_pred, uint8_t* modes,
                                                     uint64_t* resid, uint64_t* lpart, uint32_t* zero, uint32_t nzero) {
  constexpr int T = 64 / W, RW = W / 4;
  __shared__ uint32_t part[4][T][2][64];
  const int lane = lane_id(), v = (int)wave_id();
  for (uint32_t i = blockIdx.x * 256 + threadIdx.x; i < nzero; i += gridDim.x * 256) zero[i] = 0;
  const uint32_t groups = (used + 63) / 64;
  const uint32_t ty = blockIdx.x / groups, w = (blockIdx.x % groups) * 64 + lane;
  const bool act = w < used;
  uint64_t F = 0;  // first column of every tile in the word
#pragma unroll
  for (int j = 0; j < T; ++j) F |= BIC_MSB >> (j * W);
  const uint32_t r0 = v * RW;  // this wave's first row inside the tile
  const uint64_t* src = plane + (uint64_t)ty * W * wpr + (act ? w : 0);
  uint64_t x[RW];
#pragma unroll
  for (int r = 0; r < RW; ++r) x[r] = act ? src[(uint64_t)(r0 + r) * wpr] : 0;
  const uint64_t above = (act && r0) ? src[(uint64_t)(r0 - 1) * wpr] : 0;  // the row above (inside the tile)
  uint32_t co[T], cO[T];
#pragma unroll
  for (int j = 0; j < T; ++j) co[j] = cO[j] = 0;
  uint64_t up = above;
#pragma unroll
  for (int r = 0; r < RW; ++r) {
    const uint64_t d = x[r] ^ up;
    uint64_t R = d ^ ((d >> 1) & ~F);
    if (r0 + r == 0) R &= ~F;  // compress7's med never writes a tile's R(0,0)
#pragma unroll
    for (int j = 0; j < T; ++j) {
      const uint64_t m = (W == 64) ? ~0ull : (((1ull << W) - 1) << (64 - W * (j + 1)));
      co[j] += (uint32_t)__popcll(x[r] & m);
      cO[j] += (uint32_t)__popcll(R & m);
    }
    up = x[r];
  }
#pragma unroll
  for (int j = 0; j < T; ++j) {
    part[v][j][0][lane] = co[j];
    part[v][j][1][lane] = cO[j];
  }
  __syncthreads();
  uint64_t L = 0, keepR = 0;  // keepR: word mask of the tiles coded as residuals ('O')
#pragma unroll
  for (int j = 0; j < T; ++j) {
    const uint32_t to = part[0][j][0][lane] + part[1][j][0][lane] + part[2][j][0][lane] + part[3][j][0][lane];
    const uint32_t tO = part[0][j][1][lane] + part[1][j][1][lane] + part[2][j][1][lane] + part[3][j][1][lane];
    const uint32_t col0 = w * 64 + j * W;
    if (!act || col0 >= cols) continue;
    const bool pred = lentab[to] > lentab[tO];  // compress7_test.cpp:248
    const uint32_t wc = pred ? tO : to;
    if (pred) keepR |= (W == 64) ? ~0ull : (((1ull << W) - 1) << (64 - W * (j + 1)));
    if (v == 0) {
      const uint64_t tile = (uint64_t)ty * nx + col0 / W;
      if (weights) weights[tile] = wc;
      if (w_nonpred) w_nonpred[tile] = to;
      if (w_pred) w_pred[tile] = tO;
      if (modes) modes[tile] = pred ? 'O' : 'o';
      L += lentab[wc];
    }
  }
  if (resid && act) {
    uint64_t* dst = resid + (uint64_t)ty * W * wpr + w;
    const uint64_t valid = w == used - 1 && (cols & 63) ? ~(~0ull >> (cols & 63)) : ~0ull;
    up = above;
#pragma unroll
    for (int r = 0; r < RW; ++r) {
      const uint64_t d = x[r] ^ up;
      uint64_t R = d ^ ((d >> 1) & ~F);
      if (r0 + r == 0) R &= ~F;
      dst[(uint64_t)(r0 + r) * wpr] = ((R & keepR) | (x[r] & ~keepR)) & valid;
      up = x[r];
    }
  }
  if (v == 0) {
    L = wave_sum_u64(L);
    if (lane == 0) lpart[blockIdx.x] = L;
  }
}

uint32_t tiles_split_blocks(uint32_t rows, uint32_t cols, uint32_t W) {
  if (W != 8 && W != 16 && W != 32 && W != 64) return 0;
  return rows / W * (((cols + 63) / 64 + 63) / 64);
}

void launch_tiles_split(hipStream_t s, const uint64_t* plane, uint32_t rows, uint32_t cols, uint32_t wpr, uint32_t W,
                        const uint64_t* lentab_dev, uint32_t* weights, uint32_t* w_nonpred, uint32_t* w_pred,
                        uint8_t* modes, uint64_t* resid, uint64_t* lpart, uint32_t* zero, uint32_t nzero) {
  const uint32_t nx = cols / W, used = (cols + 63) / 64;
  const uint32_t grid = tiles_split_blocks(rows, cols, W);
  if (resid && wpr > used) (void)launch_fill(s, resid, 0, (size_t)rows * wpr * sizeof(uint64_t));
#define BIC_TS(WW) k_tiles_split<WW><<<grid, 256, 0, s>>>(plane, rows, cols, wpr, used, nx, lentab_dev, weights, \
                                                       w_nonpred, w_pred, modes, resid, lpart, zero, nzero)
  if (W == 8) BIC_TS(8);
  else if (W == 16) BIC_TS(16);
  else if (W == 32) BIC_TS(32);
  else BIC_TS(64);
#undef BIC_TS
}

void launch_tiles(hipStream_t s, const uint64_t* plane, uint32_t rows, uint32_t cols, uint32_t wpr,
                  uint32_t W, const uint64_t* lentab_dev, uint32_t* weights, uint32_t* w_nonpred,
                  uint32_t* w_pred, uint8_t* modes, uint64_t* resid, uint64_t* stats) {
  const uint32_t nx = cols / W, ny = rows / W;
  const uint32_t ntiles = nx * ny;
  const uint32_t used = (cols + 63) / 64;
  unsigned long long* st = reinterpret_cast<unsigned long long*>(stats);
  if (W == 8 || W == 16 || W == 32 || W == 64) {
    // words past `used` in a row (wpr > used) are the only ones the kernel does not write
    if (resid && wpr > used) (void)launch_fill(s, resid, 0, (size_t)rows * wpr * sizeof(uint64_t));
    const uint64_t waves = (uint64_t)ny * ((used + 63) / 64);
    const uint32_t grid = (uint32_t)((waves + kWaves - 1) / kWaves);
#define BIC_TILES(WW) \
    k_tiles_aligned<WW><<<grid, kBlock, 0, s>>>(plane, rows, cols, wpr, used, nx, lentab_dev, weights, w_nonpred, \
                                               w_pred, modes, resid, st)
    if (W == 8) BIC_TILES(8);
    else if (W == 16) BIC_TILES(16);
    else if (W == 32) BIC_TILES(32);
    else BIC_TILES(64);
#undef BIC_TILES
    return;
  }
  if (resid) (void)launch_fill(s, resid, 0, (size_t)rows * wpr * sizeof(uint64_t));
  const uint32_t tpw = 64 / W;
  const uint64_t waves = (ntiles + tpw - 1) / tpw;
  const uint32_t grid = (uint32_t)((waves + kWaves - 1) / kWaves);
  k_tiles<<<grid, kBlock, 0, s>>>(plane, rows, cols, wpr, W, nx, ntiles, lentab_dev, weights, w_nonpred,
                                  w_pred, modes, reinterpret_cast<unsigned long long*>(resid), st);
}

// ------------------------------------------------------------------------------------
// stream packing: plane p's words go to dst + sum_{q<p} ceil(bits_q/64)
// ------------------------------------------------------------------------------------
__global__ __launch_bounds__(kBlock) void k_pack(const uint64_t* __restrict__ slots, int nplanes,
                                                 uint64_t slot_words, const uint64_t* __restrict__ plane_bits,
                                                 uint64_t* __restrict__ dst, uint64_t* word_off) {
  __shared__ uint64_t sh_off, sh_nw;
  const int p = blockIdx.y;
  if (threadIdx.x < 64) {  // this plane's start word: one wave sums the earlier planes' sizes
    uint64_t part = 0;
    for (int q = threadIdx.x; q < p; q += 64) part += (plane_bits[q] + 63) / 64;
    part = wave_sum_u64(part);
    if (threadIdx.x == 0) {
      sh_off = part;
      sh_nw = (plane_bits[p] + 63) / 64;
    }
  }
  __syncthreads();
  const uint64_t off = sh_off, nw = sh_nw;
  if (blockIdx.x == 0 && threadIdx.x == 0) {
    word_off[p] = off;
    if (p == nplanes - 1) word_off[nplanes] = off + nw;
  }
  if (nw > slot_words) return;
  const uint64_t* src = slots + (uint64_t)p * slot_words;
  for (uint64_t i = (uint64_t)blockIdx.x * kBlock + threadIdx.x; i < nw; i += (uint64_t)gridDim.x * kBlock)
    dst[off + i] = src[i];
}

// launch_fill: 16-byte stores over the aligned middle, single bytes at the unaligned ends
__global__ __launch_bounds__(kBlock) void k_fill(uint8_t* __restrict__ dst, uint32_t v4, size_t head, size_t n16,
                                                 size_t bytes) {
  const size_t i = (size_t)blockIdx.x * kBlock + threadIdx.x, stride = (size_t)gridDim.x * kBlock;
  uint4* m = reinterpret_cast<uint4*>(dst + head);
  for (size_t j = i; j < n16; j += stride) m[j] = make_uint4(v4, v4, v4, v4);
  const size_t tail0 = head + n16 * 16;
  for (size_t j = i; j < head + (bytes - tail0); j += stride) {
    const size_t b = j < head ? j : tail0 + (j - head);
    dst[b] = (uint8_t)v4;
  }
}
void launch_fill(hipStream_t s, void* dst, int value, size_t bytes) {
  if (!bytes) return;
  uint8_t* d = reinterpret_cast<uint8_t*>(dst);
  const size_t mis = reinterpret_cast<uintptr_t>(d) & 15;
  const size_t head = mis ? std::min<size_t>(16 - mis, bytes) : 0;
  const size_t n16 = (bytes - head) / 16;
  const uint32_t v4 = 0x01010101u * (uint32_t)(uint8_t)value;
  const size_t work = std::max<size_t>(n16, bytes - n16 * 16);
  const uint32_t grid = (uint32_t)std::min<size_t>((work + kBlock - 1) / kBlock, 4096);
  k_fill<<<grid ? grid : 1, kBlock, 0, s>>>(d, v4, head, n16, bytes);
}

void launch_pack(hipStream_t s, const uint64_t* slots, int nplanes, size_t slot_words,
                 const uint64_t* plane_bits, uint64_t* dst, uint64_t* word_off) {
  // ~4 words per thread per plane: enough blocks in flight without re-summing the prefix often
  uint32_t gx = (uint32_t)((slot_words / 2 + 4 * kBlock - 1) / (4 * kBlock));
  if (gx > 256) gx = 256;
  if (gx == 0) gx = 1;
  k_pack<<<dim3(gx, nplanes), kBlock, 0, s>>>(slots, nplanes, slot_words, plane_bits, dst, word_off);
}

// ------------------------------------------------------------------------------------
// K9: patch match search (compress_test.cpp:73-111). One workgroup per W x W tile; every
// candidate position of the causal search region gets its Hamming distance; the result is the
// first position in the reference's scan order with the least distance (its early exit at a
// perfect match finds exactly that), or (0, 0, W*W) when nothing beats W*W. Tiles and candidates
// are read with get_submatrix's flat word indexing (binmat.cpp:267-298): a window running past
// the right edge continues in the next row, past the last row it reads 0.
// ------------------------------------------------------------------------------------
struct FlatImage {
  const uint64_t* I;
  uint32_t rows, used, wpr;
  // 64 bits of row i starting at column j (j < 64 * used)
  __device__ __forceinline__ uint64_t window(uint32_t i, uint32_t j) const {
    if (i >= rows) return 0;
    const uint32_t w = j >> 6, sh = j & 63;
    const uint64_t a = I[(uint64_t)i * wpr + w];
    if (!sh) return a;
    uint64_t b = 0;
    if (w + 1 < used) b = I[(uint64_t)i * wpr + w + 1];
    else if (i + 1 < rows) b = I[(uint64_t)(i + 1) * wpr];
    return (a << sh) | (b >> (64 - sh));
  }
  // the first 32 of those bits (window(i, j) >> 32): the next word is read only when they cross
  // into it (sh > 32)
  __device__ __forceinline__ uint32_t window32(uint32_t i, uint32_t j) const {
    if (i >= rows) return 0;
    const uint32_t w = j >> 6, sh = j & 63;
    const uint64_t a = I[(uint64_t)i * wpr + w];
    if (sh <= 32) return (uint32_t)(a >> (32 - sh));
    uint64_t b = 0;
    if (w + 1 < used) b = I[(uint64_t)i * wpr + w + 1];
    else if (i + 1 < rows) b = I[(uint64_t)(i + 1) * wpr];
    return __builtin_amdgcn_alignbit((uint32_t)a, (uint32_t)(b >> 32), 64 - sh);
  }
};

__global__ __launch_bounds__(kBlock) void k_patch_search(FlatImage img, uint32_t cols, uint32_t W, uint32_t nx,
                                                         uint32_t* besti, uint32_t* bestj, uint32_t* bestd) {
  __shared__ uint64_t P[64];
  __shared__ unsigned long long red[kWaves];
  const uint32_t tile = blockIdx.x, ti = tile / nx, tj = tile % nx;
  const uint32_t i0 = ti * W, j0 = tj * W;
  const uint64_t topW = W >= 64 ? ~0ull : ~(~0ull >> W);
  if (threadIdx.x < W) P[threadIdx.x] = img.window(i0 + threadIdx.x, j0) & topW;
  __syncthreads();
  // the reference's loop bounds: int(i0 - W) and int(j0 - W) of unsigned differences
  const int lim1 = (int)(i0 - W), lim2 = (int)(j0 - W);
  const uint32_t rows1 = lim1 >= 0 ? (uint32_t)lim1 + 1 : 0;  // region 1: rows [0, rows1), all columns
  const uint32_t ncol2 = lim2 >= 0 ? (uint32_t)lim2 + 1 : 0;  // region 2: rows [rows1, i0], columns [0, ncol2)
  const uint64_t n1 = (uint64_t)rows1 * cols;
  unsigned long long best = ~0ull;  // (distance << 40) | scan index
  auto visit = [&](uint32_t i2, uint32_t j2, uint64_t idx) {
    uint32_t d = 0;
    for (uint32_t r = 0; r < W; ++r) d += (uint32_t)__popcll((P[r] ^ img.window(i2 + r, j2)) & topW);
    const unsigned long long key = ((unsigned long long)d << 40) | idx;
    best = key < best ? key : best;
  };
  for (uint32_t i2 = 0; i2 < rows1; ++i2)
    for (uint32_t j2 = threadIdx.x; j2 < cols; j2 += kBlock) visit(i2, j2, (uint64_t)i2 * cols + j2);
  if (ncol2)
    for (uint32_t i2 = rows1; i2 <= i0; ++i2)
      for (uint32_t j2 = threadIdx.x; j2 < ncol2; j2 += kBlock)
        visit(i2, j2, n1 + (uint64_t)(i2 - rows1) * ncol2 + j2);
#pragma unroll
  for (int dd = 32; dd >= 1; dd >>= 1) {
    const unsigned long long o = shfl_u64(best, lane_id() ^ dd);
    best = o < best ? o : best;
  }
  if (lane_id() == 0) red[wave_id()] = best;
  __syncthreads();
  if (threadIdx.x == 0) {
    for (int q = 1; q < kWaves; ++q) best = red[q] < best ? red[q] : best;
    best = red[0] < best ? red[0] : best;
    uint32_t bi = 0, bj = 0, bd = W * W;
    if (best != ~0ull && (uint32_t)(best >> 40) < W * W) {
      const uint64_t idx = best & ((1ull << 40) - 1);
      bd = (uint32_t)(best >> 40);
      if (idx < n1) {
        bi = (uint32_t)(idx / cols);
        bj = (uint32_t)(idx % cols);
      } else {
        bi = rows1 + (uint32_t)((idx - n1) / ncol2);
        bj = (uint32_t)((idx - n1) % ncol2);
      }
    }
    besti[tile] = bi;
    bestj[tile] = bj;
    bestd[tile] = bd;
  }
}

// k_patch_search for W <= 8: a thread owns columns j2 and slides down them, so each window costs
// ONE new row word (its W rows in registers, shifted by one per step) instead of W; the same
// windows, keys and reduction.
template <int WT>
__global__ __launch_bounds__(kBlock) void k_patch_search_w(FlatImage img, uint32_t cols, uint32_t nx,
                                                           uint32_t* besti, uint32_t* bestj, uint32_t* bestd) {
  __shared__ unsigned long long red[kWaves];
  constexpr uint32_t W = WT;
  const uint32_t tile = blockIdx.x, ti = tile / nx, tj = tile % nx;
  const uint32_t i0 = ti * W, j0 = tj * W;
  const uint32_t topW = ~(~0u >> W);  // W <= 8: the window's bits are the top of window32
  uint32_t p[WT];
#pragma unroll
  for (int r = 0; r < WT; ++r) p[r] = img.window32(i0 + r, j0) & topW;
  const int lim1 = (int)(i0 - W), lim2 = (int)(j0 - W);
  const uint32_t rows1 = lim1 >= 0 ? (uint32_t)lim1 + 1 : 0;
  const uint32_t ncol2 = lim2 >= 0 ? (uint32_t)lim2 + 1 : 0;
  const uint64_t n1 = (uint64_t)rows1 * cols;
  unsigned long long best = ~0ull;  // (distance << 40) | scan index
  // rows [ra, rb) of column j2, scan index base + (i2 - ra) * stride + j2
  auto column = [&](uint32_t j2, uint32_t ra, uint32_t rb, uint64_t base, uint64_t stride) {
    uint32_t win[WT];
#pragma unroll
    for (int r = 0; r < WT - 1; ++r) win[r] = img.window32(ra + r, j2);
    for (uint32_t i2 = ra; i2 < rb; ++i2) {
      win[WT - 1] = img.window32(i2 + W - 1, j2);
      uint32_t d = 0;
#pragma unroll
      for (int r = 0; r < WT; ++r) d += (uint32_t)__popc((p[r] ^ win[r]) & topW);
      const unsigned long long key = ((unsigned long long)d << 40) | (base + (uint64_t)(i2 - ra) * stride + j2);
      best = key < best ? key : best;
#pragma unroll
      for (int r = 0; r < WT - 1; ++r) win[r] = win[r + 1];
    }
  };
  if (rows1)
    for (uint32_t j2 = threadIdx.x; j2 < cols; j2 += kBlock) column(j2, 0, rows1, 0, cols);
  if (ncol2)
    for (uint32_t j2 = threadIdx.x; j2 < ncol2; j2 += kBlock) column(j2, rows1, i0 + 1, n1, ncol2);
#pragma unroll
  for (int dd = 32; dd >= 1; dd >>= 1) {
    const unsigned long long o = shfl_u64(best, lane_id() ^ dd);
    best = o < best ? o : best;
  }
  if (lane_id() == 0) red[wave_id()] = best;
  __syncthreads();
  if (threadIdx.x == 0) {
    for (int q = 0; q < kWaves; ++q) best = red[q] < best ? red[q] : best;
    uint32_t bi = 0, bj = 0, bd = W * W;
    if (best != ~0ull && (uint32_t)(best >> 40) < W * W) {
      const uint64_t idx = best & ((1ull << 40) - 1);
      bd = (uint32_t)(best >> 40);
      if (idx < n1) {
        bi = (uint32_t)(idx / cols);
        bj = (uint32_t)(idx % cols);
      } else {
        bi = rows1 + (uint32_t)((idx - n1) / ncol2);
        bj = (uint32_t)((idx - n1) % ncol2);
      }
    }
    besti[tile] = bi;
    bestj[tile] = bj;
    bestd[tile] = bd;
  }
}

void launch_patch_search(hipStream_t s, const uint64_t* plane, uint32_t rows, uint32_t cols, uint32_t wpr,
                         uint32_t W, uint32_t* besti, uint32_t* bestj, uint32_t* bestd) {
  const uint32_t nx = (W - 1 + cols) / W, ny = (W - 1 + rows) / W;
  if (!nx || !ny) return;
  FlatImage img{plane, rows, (cols + 63) / 64, wpr};
  const uint32_t g = nx * ny;
  switch (W) {
#define BIC_PSW(N) \
  case N: k_patch_search_w<N><<<g, kBlock, 0, s>>>(img, cols, nx, besti, bestj, bestd); return;
    BIC_PSW(1) BIC_PSW(2) BIC_PSW(3) BIC_PSW(4) BIC_PSW(5) BIC_PSW(6) BIC_PSW(7) BIC_PSW(8)
#undef BIC_PSW
    default:
      k_patch_search<<<g, kBlock, 0, s>>>(img, cols, W, nx, besti, bestj, bestd);
  }
}

// ------------------------------------------------------------------------------------
// Host: the fused encoder's byte table (bic_fused.hip encode_word). For k in 1..3 and byte v
// (MSB = first pixel), the codewords of the runs that start AND end inside v -- between its
// first and last 1 -- as one MSB-first pattern, with the byte's leading and trailing zeros.
void build_byte_lut(uint64_t* lut) {
  uint32_t* lut32 = reinterpret_cast<uint32_t*>(lut + 256);
  for (unsigned k = 1; k <= 3; ++k)
    for (unsigned v = 0; v < 256; ++v) {
      if (!v) {  // never read: the encoder skips zero bytes
        if (k == 3) lut[v] = 0;
        else lut32[(k - 1) * 256 + v] = 0;
        continue;
      }
      int pos[8], m = 0;
      for (int b = 0; b < 8; ++b)
        if ((v >> (7 - b)) & 1u) pos[m++] = b;
      uint64_t R = 0;
      unsigned lr = 0;
      for (int i = 1; i < m; ++i) {
        const unsigned s = (unsigned)(pos[i] - pos[i - 1] - 1);
        R = (R << k) | (s & ((1u << k) - 1u));  // binary part
        R <<= (s >> k);                          // unary zeros
        R = (R << 1) | 1u;                       // terminator
        lr += k + (s >> k) + 1;
      }
      const unsigned t = (unsigned)pos[0], tz = (unsigned)(7 - pos[m - 1]);
      if (k == 3)  // R up to 28 bits: 64-bit entry
        lut[v] = R | ((uint64_t)lr << 32) | ((uint64_t)t << 40) | ((uint64_t)tz << 44);
      else         // R up to 21 bits: R | lr << 21 | t << 26 | tz << 29
        lut32[(k - 1) * 256 + v] = (uint32_t)R | (lr << 21) | (t << 26) | (tz << 29);
    }
  k1pi_build_table(lut32 + 512);  // k = 1 rows by the backward parity (bic_k1pi.h)
}

Geom make_geom(size_t rows, size_t cols, size_t wpr, int nplanes) {
  Geom g{};
  g.rows = (uint32_t)rows;
  g.cols = (uint32_t)cols;
  g.wpr = (uint32_t)wpr;
  g.used = (uint32_t)((cols + 63) / 64);
  g.wpl = g.used <= 64 ? 1 : (g.used <= 128 ? 2 : 4);
  g.wpc = 64 * g.wpl;
  g.cpr = (g.used + g.wpc - 1) / g.wpc;
  g.nplanes = (uint32_t)nplanes;
  g.trail = ~0ull << (63 - (cols - 1) % 64);
  g.plane_words = (uint64_t)rows * wpr;
  g.chunks_per_plane = (uint64_t)rows * g.cpr;
  g.nchunks = g.chunks_per_plane * (uint64_t)nplanes;
  g.words_used = (uint64_t)rows * g.used;
  return g;
}

static size_t al(size_t x) { return (x + 255) & ~(size_t)255; }

size_t chunk_scratch_bytes(const Geom& g) {
  const size_t n = g.nchunks;
  return al(n * 4) * 5 + al(n * 8) * 2 + al(g.words_used * g.nplanes * 4) + al(g.nplanes * 8) * 2 + 256;
}

ChunkScratch carve_chunk_scratch(void* base, const Geom& g) {
  char* p = reinterpret_cast<char*>(base);
  const size_t n = g.nchunks;
  ChunkScratch cs;
  cs.ones = reinterpret_cast<uint32_t*>(p); p += al(n * 4);
  cs.last = reinterpret_cast<int32_t*>(p); p += al(n * 4);
  cs.first = reinterpret_cast<int32_t*>(p); p += al(n * 4);
  cs.nbase = reinterpret_cast<uint32_t*>(p); p += al(n * 4);
  cs.jprev = reinterpret_cast<int32_t*>(p); p += al(n * 4);
  cs.bits = reinterpret_cast<uint64_t*>(p); p += al(n * 8);
  cs.boff = reinterpret_cast<uint64_t*>(p); p += al(n * 8);
  cs.word_bits = reinterpret_cast<uint32_t*>(p); p += al(g.words_used * g.nplanes * 4);
  cs.plane_F = reinterpret_cast<uint64_t*>(p); p += al(g.nplanes * 8);
  cs.plane_ones = reinterpret_cast<uint64_t*>(p);
  return cs;
}

}  // namespace bic
