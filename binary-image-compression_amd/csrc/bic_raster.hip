// bic_raster.hip -- SURVEY.md §8 f3: PBM / PGM rasters on the device, read straight out of a file's
// bytes (any alignment: a raster starts after a header of any length), so a whole file -> streams
// path runs on the GPU with only the header parsed on the host (bic_pnm_parse_header).
//
//  * pbm.cpp:29-77 (read_pbm_data / write_pbm): P4 rows of ceil(cols / 8) bytes, MSB = leftmost
//    pixel, rows byte-aligned -- plane word w of row i is the big-endian value of the row's bytes
//    8w .. 8w + 7 (bytes past the row's end and pad bits 0).
//  * pnm.cpp:54-89 (read_pgm_p5_data) + bitplane_tool.cpp:24-30: P5 samples of 1 byte (maxval
//    < 256) or 2 bytes big-endian ((hi << 8) + lo, pnm.cpp:71-74), row-major, no row padding;
//    plane b = bit b of each sample.
// Each lane assembles its bytes from aligned 8-byte loads shifted by the raster's misalignment
// (neighbouring lanes share the loads' cache lines: 64 lanes read one contiguous span), and never
// touches an aligned word that holds no raster byte (no read past the buffer's last page).
#include "bic_device.h"

namespace bic {

// 8 raster bytes starting at byte p (little-endian u64: byte p in bits 0-7), p < end; words past
// end read as 0
__device__ __forceinline__ uint64_t bytes8(const uint8_t* base, uint64_t p, uint64_t end) {
  const uint64_t a = p >> 3, last = (end - 1) >> 3;
  const uint32_t s = (uint32_t)(p & 7);
  const uint64_t* W = reinterpret_cast<const uint64_t*>(base);
  const uint64_t lo = a <= last ? W[a] : 0ull;
  if (!s) return lo;
  const uint64_t hi = a + 1 <= last ? W[a + 1] : 0ull;
  return (lo >> (8 * s)) | (hi << (64 - 8 * s));
}

__device__ __forceinline__ uint64_t transpose8x8_r(uint64_t x) {
  uint64_t t;
  t = (x ^ (x >> 7)) & 0x00AA00AA00AA00AAull;
  x = x ^ t ^ (t << 7);
  t = (x ^ (x >> 14)) & 0x0000CCCC0000CCCCull;
  x = x ^ t ^ (t << 14);
  t = (x ^ (x >> 28)) & 0x00000000F0F0F0F0ull;
  x = x ^ t ^ (t << 28);
  return x;
}

// P4 raster -> plane. Thread per plane word. `base` is the raster's 8-aligned floor (off = the
// raster's byte offset in it), so every load is aligned.
__global__ __launch_bounds__(256) void k_pbm_unpack2(const uint8_t* __restrict__ base, uint32_t off, uint32_t rows,
                                                     uint32_t cols, uint32_t wpr, uint64_t* __restrict__ plane) {
  const uint64_t i = (uint64_t)blockIdx.x * 256 + threadIdx.x;
  const uint32_t used = (cols + 63) / 64, nb = (cols + 7) / 8;
  if (i >= (uint64_t)rows * wpr) return;
  const uint32_t row = (uint32_t)(i / wpr), w = (uint32_t)(i % wpr);
  uint64_t v = 0;
  if (w < used) {
    const uint64_t end = off + (uint64_t)rows * nb;
    v = bswap64(bytes8(base, off + (uint64_t)row * nb + 8ull * w, end));  // byte 0 = MSB
    const uint32_t valid = min(64u, cols - 64 * w);                         // pixels of this word
    if (valid < 64) v &= ~(~0ull >> valid);
  }
  plane[i] = v;
}

// plane -> P4 raster (8-aligned raster, rows a multiple of 8 bytes: one 8-byte store per word);
// otherwise byte stores.
__global__ __launch_bounds__(256) void k_pbm_pack2(const uint64_t* __restrict__ plane, uint32_t rows, uint32_t cols,
                                                   uint32_t wpr, uint8_t* __restrict__ raster, int vec) {
  const uint64_t i = (uint64_t)blockIdx.x * 256 + threadIdx.x;
  const uint32_t used = (cols + 63) / 64, nb = (cols + 7) / 8;
  if (i >= (uint64_t)rows * used) return;
  const uint32_t row = (uint32_t)(i / used), w = (uint32_t)(i % used);
  uint64_t v = plane[(uint64_t)row * wpr + w];
  if (w == used - 1 && (cols & 63)) v &= ~(~0ull >> (cols & 63));
  if (vec) {
    reinterpret_cast<uint64_t*>(raster)[((uint64_t)row * nb >> 3) + w] = bswap64(v);
    return;
  }
  uint8_t* dst = raster + (uint64_t)row * nb + 8ull * w;
#pragma unroll
  for (int b = 0; b < 8; ++b)
    if (8 * w + b < nb) dst[b] = (uint8_t)(v >> (56 - 8 * b));
}

// P5 samples (BPP = 1 or 2 bytes) -> planes plane0 .. plane0 + nplanes - 1. Lane = output word w
// of a row (64 samples); 16 (BPP 1) or 32 (BPP 2) aligned loads, the 8 x 8 bit transposes of
// k_bitplanes_u8 per byte column.
template <int BPP>
__global__ __launch_bounds__(256) void k_raster_planes(const uint8_t* __restrict__ base, uint32_t off, uint32_t rows,
                                                       uint32_t cols, int plane0, int nplanes,
                                                       uint64_t* __restrict__ planes, uint32_t wpr) {
  const uint32_t groups = (cols + 4095) / 4096;  // 64-word groups per row
  const uint64_t gw = (uint64_t)blockIdx.x * 4 + wave_id();
  if (gw >= (uint64_t)rows * groups) return;
  const uint32_t row = (uint32_t)(gw / groups), w = (uint32_t)(gw % groups) * 64 + lane_id();
  const uint32_t used = (cols + 63) / 64;
  if (w >= used) return;
  const uint64_t end = off + (uint64_t)rows * cols * BPP;
  const uint64_t p0 = off + ((uint64_t)row * cols + 64ull * w) * BPP;
  uint64_t lo8[8], hi8[8];  // per group of 8 samples: the low / high bytes, little-endian
#pragma unroll
  for (int g = 0; g < 8; ++g) {
    if constexpr (BPP == 1) {
      lo8[g] = bytes8(base, p0 + 8 * g, end);
      hi8[g] = 0;
    } else {
      const uint64_t a = bytes8(base, p0 + 16 * g, end), b = bytes8(base, p0 + 16 * g + 8, end);
      // sample = (byte 2k << 8) + byte 2k+1 (pnm.cpp:73): odd bytes are the low ones
      lo8[g] = ((uint64_t)__builtin_amdgcn_perm((uint32_t)(b >> 32), (uint32_t)b, 0x07050301u) << 32) |
               __builtin_amdgcn_perm((uint32_t)(a >> 32), (uint32_t)a, 0x07050301u);
      hi8[g] = ((uint64_t)__builtin_amdgcn_perm((uint32_t)(b >> 32), (uint32_t)b, 0x06040200u) << 32) |
               __builtin_amdgcn_perm((uint32_t)(a >> 32), (uint32_t)a, 0x06040200u);
    }
  }
  const uint32_t valid = min(64u, cols - 64 * w);
  const uint64_t mask = valid < 64 ? ~(~0ull >> valid) : ~0ull;  // samples past the row's end
  uint64_t TL[8], TH[8];
#pragma unroll
  for (int g = 0; g < 8; ++g) {
    TL[g] = transpose8x8_r(bswap64(lo8[g]));  // byte b = plane b's 8 bits of the group
    TH[g] = BPP == 2 ? transpose8x8_r(bswap64(hi8[g])) : 0;
  }
  const uint64_t plane_words = (uint64_t)rows * wpr;
  uint64_t* dst = planes + (uint64_t)row * wpr + w;
  for (int b = 0; b < nplanes; ++b) {
    const int sb = b + plane0;
    uint64_t v = 0;
#pragma unroll
    for (int g = 0; g < 8; ++g) v |= (((sb < 8 ? TL[g] : TH[g]) >> (8 * (sb & 7))) & 0xffull) << (56 - 8 * g);
    dst[b * plane_words] = v & mask;
  }
  if (w == used - 1)
    for (int b = 0; b < nplanes; ++b)
      for (uint32_t q = used; q < wpr; ++q) planes[b * plane_words + (uint64_t)row * wpr + q] = 0;  // pad words
}

// planes plane0 .. plane0 + nplanes - 1 -> gray samples (plane2pgm_tool.cpp:33-52: sample |= mask
// for every set bit of plane b, mask = 1 << b; bits no plane covers are 0). Lane = word w of a row
// (64 samples): byte (plane0 + b) & 7 of each group's 8x8 block holds plane b's byte, the 8x8 bit
// transpose (an involution) turns it back into 8 samples' bytes. BPS 1: one byte per sample; BPS 2:
// two bytes big-endian (the P5 layout write_p5_data uses for maxval >= 256, pnm.cpp:111-124).
// 16-byte stores when the row's bytes are 16-byte aligned (VEC), byte stores otherwise.
template <int BPS, bool VEC>
__global__ __launch_bounds__(256) void k_planes_gray(const uint64_t* __restrict__ planes, uint32_t rows, uint32_t cols,
                                                     uint32_t wpr, int plane0, int nplanes, uint8_t* __restrict__ gray,
                                                     uint64_t pitch) {
  const uint32_t groups = (cols + 4095) / 4096;
  const uint64_t gw = (uint64_t)blockIdx.x * 4 + wave_id();
  if (gw >= (uint64_t)rows * groups) return;
  const uint32_t row = (uint32_t)(gw / groups), w = (uint32_t)(gw % groups) * 64 + lane_id();
  const uint32_t used = (cols + 63) / 64;
  if (w >= used) return;
  const uint64_t plane_words = (uint64_t)rows * wpr;
  const uint64_t* src = planes + (uint64_t)row * wpr + w;
  uint64_t TL[8], TH[8];
#pragma unroll
  for (int g = 0; g < 8; ++g) TL[g] = TH[g] = 0;
  for (int b = 0; b < nplanes; ++b) {
    const uint64_t v = src[b * plane_words];
    const int sb = b + plane0;
#pragma unroll
    for (int g = 0; g < 8; ++g) {
      const uint64_t byte = ((v >> (56 - 8 * g)) & 0xffull) << (8 * (sb & 7));
      if (sb < 8) TL[g] |= byte;
      else TH[g] |= byte;
    }
  }
  uint32_t out[BPS * 16];  // the 64 samples' bytes in file order
#pragma unroll
  for (int g = 0; g < 8; ++g) {
    const uint64_t lo = bswap64(transpose8x8_r(TL[g]));  // byte k = sample 8g + k's low byte
    if constexpr (BPS == 1) {
      out[2 * g] = (uint32_t)lo;
      out[2 * g + 1] = (uint32_t)(lo >> 32);
    } else {
      const uint64_t hi = bswap64(transpose8x8_r(TH[g]));
      // big-endian samples: hi0 lo0 hi1 lo1 ...
      const uint32_t l0 = (uint32_t)lo, l1 = (uint32_t)(lo >> 32), h0 = (uint32_t)hi, h1 = (uint32_t)(hi >> 32);
      out[4 * g] = __builtin_amdgcn_perm(l0, h0, 0x05010400u);
      out[4 * g + 1] = __builtin_amdgcn_perm(l0, h0, 0x07030602u);
      out[4 * g + 2] = __builtin_amdgcn_perm(l1, h1, 0x05010400u);
      out[4 * g + 3] = __builtin_amdgcn_perm(l1, h1, 0x07030602u);
    }
  }
  uint8_t* dst = gray + (uint64_t)row * pitch + (uint64_t)w * 64 * BPS;
  const uint32_t valid = min(64u, cols - 64 * w);
  if (VEC && valid == 64) {
#pragma unroll
    for (int q = 0; q < BPS * 4; ++q)
      reinterpret_cast<uint4*>(dst)[q] = make_uint4(out[4 * q], out[4 * q + 1], out[4 * q + 2], out[4 * q + 3]);
    return;
  }
  for (uint32_t i = 0; i < valid * BPS; ++i) dst[i] = (uint8_t)(out[i >> 2] >> (8 * (i & 3)));
}

void launch_planes_gray(hipStream_t s, const uint64_t* planes, uint32_t rows, uint32_t cols, uint32_t wpr, int plane0,
                        int nplanes, int bps, uint8_t* gray, uint64_t pitch) {
  const uint64_t waves = (uint64_t)rows * ((cols + 4095) / 4096);
  const uint32_t grid = (uint32_t)((waves + 3) / 4);
  if (!grid) return;
  const bool vec = reinterpret_cast<uintptr_t>(gray) % 16 == 0 && pitch % 16 == 0;
#define BIC_PG(B, V) k_planes_gray<B, V><<<grid, 256, 0, s>>>(planes, rows, cols, wpr, plane0, nplanes, gray, pitch)
  if (bps == 1) { if (vec) BIC_PG(1, true); else BIC_PG(1, false); }
  else { if (vec) BIC_PG(2, true); else BIC_PG(2, false); }
#undef BIC_PG
}

void launch_pbm(hipStream_t s, bool pack, const uint8_t* raster_in, uint8_t* raster_out, const uint64_t* plane_in,
                uint64_t* plane_out, uint32_t rows, uint32_t cols, uint32_t wpr) {
  if (!pack) {
    const uint64_t n = (uint64_t)rows * wpr;
    const uintptr_t r = reinterpret_cast<uintptr_t>(raster_in);
    const uint8_t* base = reinterpret_cast<const uint8_t*>(r & ~(uintptr_t)7);
    if (n) k_pbm_unpack2<<<(uint32_t)((n + 255) / 256), 256, 0, s>>>(base, (uint32_t)(r & 7), rows, cols, wpr, plane_out);
    return;
  }
  const uint64_t n = (uint64_t)rows * ((cols + 63) / 64);
  const int vec = (reinterpret_cast<uintptr_t>(raster_out) % 8 == 0) && ((cols + 7) / 8) % 8 == 0;
  if (n) k_pbm_pack2<<<(uint32_t)((n + 255) / 256), 256, 0, s>>>(plane_in, rows, cols, wpr, raster_out, vec);
}

void launch_raster_planes(hipStream_t s, const uint8_t* raster, int bpp, uint32_t rows, uint32_t cols, int plane0,
                          int nplanes, uint64_t* planes, uint32_t wpr) {
  const uintptr_t r = reinterpret_cast<uintptr_t>(raster);
  const uint8_t* base = reinterpret_cast<const uint8_t*>(r & ~(uintptr_t)7);
  const uint64_t waves = (uint64_t)rows * ((cols + 4095) / 4096);
  const uint32_t grid = (uint32_t)((waves + 3) / 4);
  if (!grid) return;
  if (bpp == 1) k_raster_planes<1><<<grid, 256, 0, s>>>(base, (uint32_t)(r & 7), rows, cols, plane0, nplanes, planes, wpr);
  else k_raster_planes<2><<<grid, 256, 0, s>>>(base, (uint32_t)(r & 7), rows, cols, plane0, nplanes, planes, wpr);
}

}  // namespace bic
