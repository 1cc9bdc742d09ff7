// Microbenchmark (diagnostic, not product): the emission kernel's skeleton -- load a plane row and
// the row above, med residual, write the row's EG copy (~R and '1' at bit offset row*(cols+1)+1) --
// in several schedules, to see which shape reaches the HBM rate: C3 geometry (8 x 16384 rows of
// 256 words). Build: hipcc --offload-arch=gfx950 -O3 -o emit_skel emit_skel.hip
#include <hip/hip_runtime.h>

#include <cstdint>
#include <cstdio>

#define MSB 0x8000000000000000ull
constexpr uint32_t ROWS = 16384, USED = 256, PLANES = 8, COLS = 16384;
constexpr uint64_t NROWS = (uint64_t)ROWS * PLANES;
constexpr uint64_t SLOT = ((uint64_t)ROWS * (COLS + 1) + 1 + 63) / 64 + 1;

__device__ __forceinline__ int lane_id() { return threadIdx.x & 63; }
__device__ __forceinline__ uint64_t shr1(uint64_t v) {  // lane i gets lane i-1's value (wave_shr:1), lane 0 its own
  const uint32_t lo = (uint32_t)__builtin_amdgcn_update_dpp((int)(uint32_t)v, (int)(uint32_t)v, 0x138, 0xf, 0xf, false);
  const uint32_t hi = (uint32_t)__builtin_amdgcn_update_dpp((int)(uint32_t)(v >> 32), (int)(uint32_t)(v >> 32), 0x138, 0xf, 0xf, false);
  return ((uint64_t)hi << 32) | lo;
}
__device__ __forceinline__ uint64_t rl63(uint64_t v) {
  return ((uint64_t)(uint32_t)__builtin_amdgcn_readlane((int)(uint32_t)(v >> 32), 63) << 32) |
         (uint32_t)__builtin_amdgcn_readlane((int)(uint32_t)v, 63);
}

// strided layout (lane holds words 64 t + lane), as k_emit_known
__device__ __forceinline__ void row_strided(const uint64_t* planes, uint64_t id, uint64_t* out, bool load_only = false) {
  const uint32_t plane = (uint32_t)(id / ROWS), row = (uint32_t)(id % ROWS);
  const uint64_t* cur = planes + ((uint64_t)plane * ROWS + row) * USED;
  const uint64_t* up = row ? cur - USED : cur;
  const int lane = lane_id();
  uint64_t p[4], u[4], r[4];
#pragma unroll
  for (int t = 0; t < 4; ++t) {
    p[t] = cur[t * 64 + lane];
    u[t] = row ? up[t * 64 + lane] : 0;
  }
  uint64_t carry = 0;
#pragma unroll
  for (int t = 0; t < 4; ++t) {
    uint64_t d = p[t] ^ u[t];
    uint64_t dl = shr1(d);
    if (lane == 0) dl = carry;
    carry = rl63(d);
    r[t] = d ^ ((d >> 1) | (dl << 63));
  }
  const uint64_t Ge = (uint64_t)plane * SLOT * 64 + (uint64_t)row * (COLS + 1) + 1;
  const uint32_t sh = (uint32_t)(Ge & 63);
  const uint64_t w0 = Ge >> 6;
  uint64_t c2 = 0;
#pragma unroll
  for (int t = 0; t <= 4; ++t) {
    const uint32_t j = t * 64 + lane;
    uint64_t X = t < 4 ? ~r[t] : 0;
    if (j == COLS / 64) X |= MSB;
    uint64_t Xl = shr1(X);
    if (lane == 0) Xl = c2;
    c2 = rl63(X);
    const uint64_t v = sh ? (Xl << (64 - sh)) | (X >> sh) : X;
    if (j <= USED) out[w0 + j] = __builtin_bswap64(v);
  }
}

// A: persistent waves, rows id, id + stride (k_emit_known's schedule)
__global__ __launch_bounds__(256, 4) void k_a(const uint64_t* planes, uint64_t* out) {
  const uint64_t stride = (uint64_t)gridDim.x * 4;
  for (uint64_t id = (uint64_t)blockIdx.x * 4 + (threadIdx.x >> 6); id < NROWS; id += stride) row_strided(planes, id, out);
}
// C: one row per wave, no loop
__global__ __launch_bounds__(256) void k_c(const uint64_t* planes, uint64_t* out) {
  const uint64_t id = (uint64_t)blockIdx.x * 4 + (threadIdx.x >> 6);
  if (id < NROWS) row_strided(planes, id, out);
}

// C4: C limited to 4 waves per SIMD (the real kernel's occupancy at ~114 VGPRs)
__global__ __launch_bounds__(256) __attribute__((amdgpu_waves_per_eu(4, 4))) void k_c4(const uint64_t* planes, uint64_t* out) {
  const uint64_t id = (uint64_t)blockIdx.x * 4 + (threadIdx.x >> 6);
  if (id < NROWS) row_strided(planes, id, out);
}
// C2: C limited to 2 waves per SIMD
__global__ __launch_bounds__(256) __attribute__((amdgpu_waves_per_eu(2, 2))) void k_c2(const uint64_t* planes, uint64_t* out) {
  const uint64_t id = (uint64_t)blockIdx.x * 4 + (threadIdx.x >> 6);
  if (id < NROWS) row_strided(planes, id, out);
}
// A2: persistent, two rows per iteration (both rows' loads issued before either is used)
__global__ __launch_bounds__(256, 4) void k_a2(const uint64_t* planes, uint64_t* out) {
  const uint64_t stride = (uint64_t)gridDim.x * 4;
  for (uint64_t id = (uint64_t)blockIdx.x * 4 + (threadIdx.x >> 6); id < NROWS; id += 2 * stride) {
    row_strided(planes, id, out);
    if (id + stride < NROWS) row_strided(planes, id + stride, out);
  }
}

// D: consecutive layout (lane holds words 4 l .. 4 l + 3: two 16-byte loads per row), one row per wave
__global__ __launch_bounds__(256) void k_d(const uint64_t* planes, uint64_t* out) {
  const uint64_t id = (uint64_t)blockIdx.x * 4 + (threadIdx.x >> 6);
  if (id >= NROWS) return;
  const uint32_t plane = (uint32_t)(id / ROWS), row = (uint32_t)(id % ROWS);
  const int lane = lane_id();
  const uint64_t* cur = planes + ((uint64_t)plane * ROWS + row) * USED + 4 * lane;
  const ulonglong2* c2p = reinterpret_cast<const ulonglong2*>(cur);
  ulonglong2 pa = c2p[0], pb = c2p[1];
  ulonglong2 ua = make_ulonglong2(0, 0), ub = ua;
  if (row) {
    const ulonglong2* u2p = reinterpret_cast<const ulonglong2*>(cur - USED);
    ua = u2p[0];
    ub = u2p[1];
  }
  uint64_t d[4] = {pa.x ^ ua.x, pa.y ^ ua.y, pb.x ^ ub.x, pb.y ^ ub.y};
  uint64_t left = shr1(d[3]);
  if (lane == 0) left = 0;
  uint64_t r[4];
  r[0] = d[0] ^ ((d[0] >> 1) | (left << 63));
  r[1] = d[1] ^ ((d[1] >> 1) | (d[0] << 63));
  r[2] = d[2] ^ ((d[2] >> 1) | (d[1] << 63));
  r[3] = d[3] ^ ((d[3] >> 1) | (d[2] << 63));
  const uint64_t Ge = (uint64_t)plane * SLOT * 64 + (uint64_t)row * (COLS + 1) + 1;
  const uint32_t sh = (uint32_t)(Ge & 63);
  const uint64_t w0 = Ge >> 6;
  uint64_t X[4] = {~r[0], ~r[1], ~r[2], ~r[3]};
  uint64_t Xl = shr1(X[3]);
  if (lane == 0) Xl = 0;
  uint64_t v[4];
  v[0] = sh ? (Xl << (64 - sh)) | (X[0] >> sh) : X[0];
  v[1] = sh ? (X[0] << (64 - sh)) | (X[1] >> sh) : X[1];
  v[2] = sh ? (X[1] << (64 - sh)) | (X[2] >> sh) : X[2];
  v[3] = sh ? (X[2] << (64 - sh)) | (X[3] >> sh) : X[3];
  uint64_t* o = out + w0 + 4 * lane;
#pragma unroll
  for (int q = 0; q < 4; ++q) o[q] = __builtin_bswap64(v[q]);
  if (lane == 63) out[w0 + 256] = __builtin_bswap64((X[3] << (64 - sh)) | (MSB >> sh));
}

// E: consecutive layout, persistent with prefetch of the next row
__global__ __launch_bounds__(256, 4) void k_e(const uint64_t* planes, uint64_t* out) {
  const uint64_t stride = (uint64_t)gridDim.x * 4;
  const int lane = lane_id();
  uint64_t id = (uint64_t)blockIdx.x * 4 + (threadIdx.x >> 6);
  ulonglong2 pa, pb, ua, ub;
  auto load = [&](uint64_t i) {
    const uint32_t plane = (uint32_t)(i / ROWS), row = (uint32_t)(i % ROWS);
    const uint64_t* cur = planes + ((uint64_t)plane * ROWS + row) * USED + 4 * lane;
    pa = reinterpret_cast<const ulonglong2*>(cur)[0];
    pb = reinterpret_cast<const ulonglong2*>(cur)[1];
    if (row) {
      ua = reinterpret_cast<const ulonglong2*>(cur - USED)[0];
      ub = reinterpret_cast<const ulonglong2*>(cur - USED)[1];
    } else {
      ua = ub = make_ulonglong2(0, 0);
    }
  };
  if (id < NROWS) load(id);
  for (; id < NROWS; id += stride) {
    const uint32_t plane = (uint32_t)(id / ROWS), row = (uint32_t)(id % ROWS);
    uint64_t d[4] = {pa.x ^ ua.x, pa.y ^ ua.y, pb.x ^ ub.x, pb.y ^ ub.y};
    if (id + stride < NROWS) load(id + stride);
    uint64_t left = shr1(d[3]);
    if (lane == 0) left = 0;
    uint64_t r[4];
    r[0] = d[0] ^ ((d[0] >> 1) | (left << 63));
    r[1] = d[1] ^ ((d[1] >> 1) | (d[0] << 63));
    r[2] = d[2] ^ ((d[2] >> 1) | (d[1] << 63));
    r[3] = d[3] ^ ((d[3] >> 1) | (d[2] << 63));
    const uint64_t Ge = (uint64_t)plane * SLOT * 64 + (uint64_t)row * (COLS + 1) + 1;
    const uint32_t sh = (uint32_t)(Ge & 63);
    const uint64_t w0 = Ge >> 6;
    uint64_t X[4] = {~r[0], ~r[1], ~r[2], ~r[3]};
    uint64_t Xl = shr1(X[3]);
    if (lane == 0) Xl = 0;
    uint64_t v[4];
    v[0] = sh ? (Xl << (64 - sh)) | (X[0] >> sh) : X[0];
    v[1] = sh ? (X[0] << (64 - sh)) | (X[1] >> sh) : X[1];
    v[2] = sh ? (X[1] << (64 - sh)) | (X[2] >> sh) : X[2];
    v[3] = sh ? (X[2] << (64 - sh)) | (X[3] >> sh) : X[3];
    uint64_t* o = out + w0 + 4 * lane;
#pragma unroll
    for (int q = 0; q < 4; ++q) o[q] = __builtin_bswap64(v[q]);
    if (lane == 63) out[w0 + 256] = __builtin_bswap64((X[3] << (64 - sh)) | (MSB >> sh));
  }
}

// R: read-only reference (sum of the row words)
__global__ __launch_bounds__(256) void k_read(const uint64_t* planes, uint64_t* out) {
  const uint64_t i = (uint64_t)blockIdx.x * 256 + threadIdx.x;
  const ulonglong2* p = reinterpret_cast<const ulonglong2*>(planes);
  ulonglong2 a = p[i];
  if ((a.x ^ a.y) == 0x1234) out[0] = 1;
}
// W: copy reference (planes -> out, 16-byte)
__global__ __launch_bounds__(256) void k_copy(const uint64_t* planes, uint64_t* out) {
  const uint64_t i = (uint64_t)blockIdx.x * 256 + threadIdx.x;
  reinterpret_cast<ulonglong2*>(out)[i] = reinterpret_cast<const ulonglong2*>(planes)[i];
}

int main() {
  const size_t pw = NROWS * USED;
  uint64_t *planes[2], *out;
  for (int i = 0; i < 2; ++i) {
    (void)hipMalloc(&planes[i], pw * 8);
    (void)hipMemset(planes[i], 0x5a + i, pw * 8);
  }
  (void)hipMalloc(&out, (PLANES * SLOT + 1024) * 8);
  hipEvent_t a, b;
  (void)hipEventCreate(&a);
  (void)hipEventCreate(&b);
  int cus = 256;
  (void)hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, 0);
  const double bytes = 2.0 * pw * 8;  // read planes + write the EG copy
  auto run = [&](const char* name, auto launch) {
    for (int w = 0; w < 3; ++w) launch(planes[w & 1]);
    (void)hipDeviceSynchronize();
    (void)hipEventRecord(a);
    const int reps = 20;
    for (int r = 0; r < reps; ++r) launch(planes[r & 1]);
    (void)hipEventRecord(b);
    (void)hipEventSynchronize(b);
    float ms = 0;
    (void)hipEventElapsedTime(&ms, a, b);
    const double us = ms * 1e3 / reps;
    printf("%-48s %8.1f us  %6.2f TB/s (read+write)\n", name, us, bytes / (us * 1e-6) / 1e12);
  };
  run("A persistent strided (k_emit_known shape)", [&](uint64_t* p) { k_a<<<cus * 4, 256>>>(p, out); });
  run("A persistent strided, 8 WG/CU", [&](uint64_t* p) { k_a<<<cus * 8, 256>>>(p, out); });
  run("C one row per wave, strided", [&](uint64_t* p) { k_c<<<(uint32_t)(NROWS / 4), 256>>>(p, out); });
  run("C4 one row per wave, 4 waves/SIMD max", [&](uint64_t* p) { k_c4<<<(uint32_t)(NROWS / 4), 256>>>(p, out); });
  run("C2 one row per wave, 2 waves/SIMD max", [&](uint64_t* p) { k_c2<<<(uint32_t)(NROWS / 4), 256>>>(p, out); });
  run("A persistent strided, 2 WG/CU", [&](uint64_t* p) { k_a<<<cus * 2, 256>>>(p, out); });
  run("A persistent strided, 16 WG/CU", [&](uint64_t* p) { k_a<<<cus * 16, 256>>>(p, out); });
  run("A persistent strided, 32 WG/CU", [&](uint64_t* p) { k_a<<<cus * 32, 256>>>(p, out); });
  run("D one row per wave, consecutive words", [&](uint64_t* p) { k_d<<<(uint32_t)(NROWS / 4), 256>>>(p, out); });
  run("E persistent consecutive + prefetch (4 WG/CU)", [&](uint64_t* p) { k_e<<<cus * 4, 256>>>(p, out); });
  run("E persistent consecutive + prefetch (8 WG/CU)", [&](uint64_t* p) { k_e<<<cus * 8, 256>>>(p, out); });
  run("copy planes -> out (16-byte)", [&](uint64_t* p) { k_copy<<<(uint32_t)(pw / 2 / 256), 256>>>(p, out); });
  run("read planes only (x2 bytes counted)", [&](uint64_t* p) { k_read<<<(uint32_t)(pw / 2 / 256), 256>>>(p, out); });
  return 0;
}
