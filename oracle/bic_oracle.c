/*
 * bic_oracle.c -- TEST INFRASTRUCTURE ONLY. See bic_oracle.h for scope and the
 * reference file:line each function restates. Deliberately bit-serial and
 * simple: this is the checker the HIP path is compared against, not a fast path.
 */
#include "bic_oracle.h"

#include <assert.h>
#include <math.h>
#include <stdlib.h>
#include <string.h>
#ifdef _OPENMP
#include <omp.h>
#endif

#define BO_MSB 0x8000000000000000ull

/* ------------------------------------------------------------------------- */
uint64_t bo_splitmix64(uint64_t* state) {
    uint64_t z = (*state += 0x9E3779B97F4A7C15ull);
    z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ull;
    z = (z ^ (z >> 27)) * 0x94D049BB133111EBull;
    return z ^ (z >> 31);
}

void bo_gen_plane(uint64_t seed, double p, size_t rows, size_t cols, size_t wpr,
                  uint64_t* plane) {
    uint64_t st = seed;
    const uint32_t thr = (uint32_t)llround(p * 65536.0);
    const size_t used = (cols + 63) / 64;
    for (size_t i = 0; i < rows; ++i) {
        for (size_t w = 0; w < wpr; ++w) {
            uint64_t word = 0;
            if (w < used) {
                for (int q = 0; q < 16; ++q) {
                    const uint64_t x = bo_splitmix64(&st);
                    for (int d = 0; d < 4; ++d) {
                        const uint32_t draw = (uint32_t)(x >> (48 - 16 * d)) & 0xFFFFu;
                        word = (word << 1) | (draw < thr ? 1u : 0u);
                    }
                }
                if (w == used - 1 && (cols & 63)) word &= ~0ull << (64 - (cols & 63));
            }
            plane[i * wpr + w] = word;
        }
    }
}

void bo_gen_bytes(uint64_t seed, size_t n, uint8_t* out) {
    uint64_t st = seed;
    for (size_t i = 0; i < n; i += 8) {
        const uint64_t x = bo_splitmix64(&st);
        for (size_t b = 0; b < 8 && i + b < n; ++b) out[i + b] = (uint8_t)(x >> (8 * b));
    }
}

/* ------------------------------------------------------------------------- */
int bo_get(const uint64_t* P, size_t wpr, size_t i, size_t j) {
    return (P[i * wpr + j / 64] & (BO_MSB >> (j % 64))) != 0;
}

void bo_set(uint64_t* P, size_t wpr, size_t i, size_t j, int v) {
    uint64_t* w = &P[i * wpr + j / 64];
    const uint64_t m = BO_MSB >> (j % 64);
    if (v) *w |= m; else *w &= ~m;
}

int bo_num_planes(int maxval) {
    int n = 0;
    for (long b = 1; b < maxval; b <<= 1) ++n; /* bitplane_tool.cpp:24 */
    return n;
}

void bo_bitplanes(const void* gray, int bytes_per_px, size_t rows, size_t cols,
                  int nplanes, uint64_t* planes, size_t wpr) {
    const uint8_t* g8 = (const uint8_t*)gray;
    const uint16_t* g16 = (const uint16_t*)gray;
    memset(planes, 0, sizeof(uint64_t) * (size_t)nplanes * rows * wpr);
    for (int bi = 0; bi < nplanes; ++bi) {
        uint64_t* A = planes + (size_t)bi * rows * wpr;
        for (size_t i = 0, li = 0; i < rows; ++i)
            for (size_t j = 0; j < cols; ++j, ++li) {
                const unsigned px = bytes_per_px == 1 ? g8[li] : g16[li];
                bo_set(A, wpr, i, j, (px >> bi) & 1u);
            }
    }
}

void bo_planes_to_gray(const uint64_t* planes, int nplanes, size_t rows, size_t cols, size_t wpr,
                       uint32_t* gray) {
    memset(gray, 0, sizeof(uint32_t) * rows * cols);       /* plane2pgm_tool.cpp:27 */
    unsigned mask = 0x01;                                    /* plane2pgm_tool.cpp:32 */
    for (int b = 0; b < nplanes; ++b, mask <<= 1) {         /* :33-50, one plane per pass */
        const uint64_t* A = planes + (size_t)b * rows * wpr;
        for (size_t i = 0, li = 0; i < rows; ++i)            /* :35-41 */
            for (size_t j = 0; j < cols; ++j, ++li)
                if (bo_get(A, wpr, i, j)) gray[li] |= mask;
    }
}

void bo_med(const uint64_t* P, uint64_t* R, size_t rows, size_t cols, size_t wpr) {
    memset(R, 0, sizeof(uint64_t) * rows * wpr);
    if (rows == 0 || cols == 0) return;
    for (size_t j = 1; j < cols; ++j)                 /* pred.cpp:5-7 */
        bo_set(R, wpr, 0, j, bo_get(P, wpr, 0, j - 1) ^ bo_get(P, wpr, 0, j));
    for (size_t i = 1; i < rows; ++i) {                /* pred.cpp:8-13 */
        bo_set(R, wpr, i, 0, bo_get(P, wpr, i - 1, 0) ^ bo_get(P, wpr, i, 0));
        for (size_t j = 1; j < cols; ++j)
            bo_set(R, wpr, i, j,
                   bo_get(P, wpr, i - 1, j - 1) ^ bo_get(P, wpr, i, j - 1) ^
                   bo_get(P, wpr, i - 1, j) ^ bo_get(P, wpr, i, j));
    }
}

static int bo_popcount64(uint64_t x) {
    int c = 0;
    while (x) { x &= x - 1; ++c; }
    return c;
}

uint64_t bo_weight(const uint64_t* P, size_t rows, size_t cols, size_t wpr) {
    if (rows * cols == 0) return 0;
    const size_t bpr = (cols + 63) / 64;
    const uint64_t trail = ~0ull << (63 - (cols - 1) % 64); /* binmat.cpp:147 */
    uint64_t w = 0;
    for (size_t i = 0; i < rows; ++i)
        for (size_t j = 0; j < bpr; ++j) {
            uint64_t b = P[i * wpr + j];
            if (j == bpr - 1) b &= trail;                   /* binmat.h:188-190 */
            w += (uint64_t)bo_popcount64(b);
        }
    return w;
}

/* ------------------------------------------------------------------------- */
void bo_bw_init(bo_bw* bw, uint8_t* buf, size_t cap_bytes) {
    bw->buf = buf;
    bw->cap_bits = buf ? cap_bytes * 8 : 0;
    bw->pos = 0;
    bw->overflow = 0;
    if (buf) memset(buf, 0, cap_bytes);
}

static void bo_bw_bit1(bo_bw* bw, uint64_t at) {
    if (!bw->buf) return;
    if (at >= bw->cap_bits) { bw->overflow = 1; return; }
    bw->buf[at >> 3] |= (uint8_t)(0x80u >> (at & 7));
}

void bo_bw_put(bo_bw* bw, uint32_t value, unsigned nbits) {
    for (unsigned b = 0; b < nbits; ++b)
        if ((value >> (nbits - 1 - b)) & 1u) bo_bw_bit1(bw, bw->pos + b);
    bw->pos += nbits;
    if (bw->buf && bw->pos > bw->cap_bits) bw->overflow = 1;
}

void bo_bw_zeros(bo_bw* bw, uint64_t n) {
    bw->pos += n;
    if (bw->buf && bw->pos > bw->cap_bits) bw->overflow = 1;
}

/* ------------------------------------------------------------------------- */
void bo_golomb_init(bo_golomb* g) {  /* Golomb.h:14-19 */
    g->accumulatedError = 0;
    g->samples = 0;
    g->k = 1;
    g->bitcount = 0;
}

uint32_t bo_golomb_code(bo_golomb* g, uint32_t s, bo_bw* bw) {
    const uint32_t k = g->k;
    assert(k < 32);                                   /* GolombCoder.cpp:14 */
    const uint32_t unary = s >> k;                    /* GolombCoder.cpp:19 */
    if (bw) {
        bo_bw_put(bw, k ? (s & ((1u << k) - 1u)) : 0u, k); /* binary part */
        bo_bw_zeros(bw, unary);                            /* unary zeros */
        bo_bw_put(bw, 1u, 1);                              /* terminator  */
    }
    const uint32_t len = k + unary + 1;
    g->bitcount += len;                               /* GolombCoder.cpp:26 */
    g->samples++;                                     /* GolombCoder.cpp:31-33 */
    g->accumulatedError += s;
    uint32_t nk = 0;
    /* the domain the reference is defined on: samples << k never wraps before
     * reaching accumulatedError (guaranteed when accumulatedError < 2^31). */
    while (nk < 31 && (g->samples << nk) < g->accumulatedError) ++nk;
    g->k = nk;
    return len;
}

/* JPEG-LS run-length order table J[0..31] (ITU-T T.87 A.7.1.2), which the
 * reference's EGLUT (eg.cpp:2) is. */
static const unsigned char bo_J[32] = {0, 0, 0, 0, 1, 1, 1,  1,  2,  2,  2,  2,  3,  3,  3,  3,
                                       4, 4, 5, 5, 6, 6, 7,  7,  8,  9,  10, 11, 12, 13, 14, 15};

void bo_eg_init(bo_eg* e, int adaptive) {  /* eg.h:9 */
    e->g = 1;
    e->blockSize = 1;
    e->lutIndex = 0;
    e->bitcount = 0;
    e->adaptive = adaptive;
}

static void bo_eg_inc(bo_eg* e) {  /* eg.cpp:4-10, index capped at 31 */
    if (e->lutIndex < 31) e->lutIndex++;
    e->g = bo_J[e->lutIndex];
    e->blockSize = 1u << e->g;
}

static void bo_eg_dec(bo_eg* e) {  /* eg.cpp:12-18 */
    if (e->lutIndex > 0) e->lutIndex--;
    e->g = bo_J[e->lutIndex];
    e->blockSize = 1u << e->g;
}

uint32_t bo_eg_code(bo_eg* e, int len, int eol, bo_bw* bw) {
    uint32_t bits = 0;
    while ((unsigned)len >= e->blockSize) {          /* eg.cpp:22-27 */
        len -= (int)e->blockSize;
        if (bw) bo_bw_put(bw, 1u, 1);
        ++bits;
        if (e->adaptive) bo_eg_inc(e);
    }
    if (eol) {                                        /* eg.cpp:28-30 */
        if (bw) bo_bw_put(bw, 1u, 1);
        bits += 1;
    } else {                                          /* eg.cpp:31-35 */
        if (bw) { bo_bw_put(bw, 0u, 1); bo_bw_put(bw, (uint32_t)len, e->g); }
        bits += e->g + 1;
        bo_eg_dec(e);
    }
    e->bitcount += bits;
    return bits;
}

/* ------------------------------------------------------------------------- */
typedef struct {
    int coder;
    bo_golomb gol;
    bo_eg eg;
    bo_bw* bw;
    uint64_t nsamples;
} bo_sink;

static void bo_sink_run(bo_sink* s, uint32_t len, int eol) {
    if (s->coder == 0) bo_golomb_code(&s->gol, len, s->bw);
    else bo_eg_code(&s->eg, (int)len, eol, s->bw);
    s->nsamples++;
}

/* Run extraction, SURVEY.md §8 a7 (build-defined; shape from eg.h:23). */
static void bo_scan_runs(const uint64_t* src, size_t rows, size_t cols, size_t wpr, bo_sink* s) {
    for (size_t i = 0; i < rows; ++i) {
        long last = -1;
        for (size_t j = 0; j < cols; ++j) {
            if (bo_get(src, wpr, i, j)) {
                bo_sink_run(s, (uint32_t)((long)j - last - 1), 0);
                last = (long)j;
            }
        }
        bo_sink_run(s, (uint32_t)((long)cols - 1 - last), 1);
    }
}

int64_t bo_encode_plane(const uint64_t* plane, size_t rows, size_t cols, size_t wpr,
                        int predict, int coder, uint8_t* out, size_t cap_bytes,
                        uint64_t* nsamples) {
    const uint64_t* src = plane;
    uint64_t* R = NULL;
    if (predict) {
        R = (uint64_t*)malloc(sizeof(uint64_t) * rows * wpr + 8);
        bo_med(plane, R, rows, cols, wpr);
        src = R;
    }
    bo_bw bw;
    bo_bw_init(&bw, out, cap_bytes);
    bo_sink s;
    s.coder = coder == 0 ? 0 : 1;
    bo_golomb_init(&s.gol);
    bo_eg_init(&s.eg, coder == 2);
    s.bw = &bw;
    s.nsamples = 0;
    bo_scan_runs(src, rows, cols, wpr, &s);
    free(R);
    if (nsamples) *nsamples = s.nsamples;
    if (out && (bw.overflow || ((bw.pos + 63) / 64) * 8 > cap_bytes)) return -1;
    return (int64_t)bw.pos;
}

int64_t bo_eg_runs(const int32_t* len, const uint8_t* eol, size_t n, int adaptive, uint8_t* out,
                   size_t cap_bytes, uint32_t* bits_out) {
    bo_bw bw;
    bo_bw_init(&bw, out, cap_bytes);
    bo_eg e;
    bo_eg_init(&e, adaptive);
    for (size_t i = 0; i < n; ++i) {
        const uint32_t b = bo_eg_code(&e, len[i], eol[i], out ? &bw : NULL);
        if (bits_out) bits_out[i] = b;
    }
    if (out && bw.overflow) return -1;
    return (int64_t)e.bitcount;
}

/* bo_scan_runs with the coder state recorded at every row start (GolombCoder.cpp:29-34 lengths) */
void bo_row_index(const uint64_t* plane, size_t rows, size_t cols, size_t wpr, int predict, uint64_t* index) {
    const uint64_t* src = plane;
    uint64_t* R = NULL;
    if (predict) {
        R = (uint64_t*)malloc(sizeof(uint64_t) * rows * wpr + 8);
        bo_med(plane, R, rows, cols, wpr);
        src = R;
    }
    bo_golomb g;
    bo_golomb_init(&g);
    uint64_t ones = 0;
    for (size_t i = 0; i < rows; ++i) {
        index[2 * i] = (uint64_t)g.bitcount;
        index[2 * i + 1] = ones;
        long last = -1;
        for (size_t j = 0; j < cols; ++j)
            if (bo_get(src, wpr, i, j)) {
                bo_golomb_code(&g, (uint32_t)((long)j - last - 1), NULL);
                last = (long)j;
                ++ones;
            }
        bo_golomb_code(&g, (uint32_t)((long)cols - 1 - last), NULL);
    }
    free(R);
}

/* The adaptive EG coder (coder 2) with its state recorded at every row start: [2 i] = the stream bits
 * before row i, [2 i + 1] = eg.h's lutIndex there, 32 for a fresh coder (lutIndex 0 with g = 1, eg.h:9). */
void bo_egad_row_index(const uint64_t* plane, size_t rows, size_t cols, size_t wpr, int predict, uint64_t* index) {
    const uint64_t* src = plane;
    uint64_t* R = NULL;
    if (predict) {
        R = (uint64_t*)malloc(sizeof(uint64_t) * rows * wpr + 8);
        bo_med(plane, R, rows, cols, wpr);
        src = R;
    }
    bo_eg e;
    bo_eg_init(&e, 1);
    for (size_t i = 0; i < rows; ++i) {
        index[2 * i] = e.bitcount;
        index[2 * i + 1] = (e.lutIndex == 0 && e.g == 1) ? 32u : (uint64_t)e.lutIndex;
        long last = -1;
        for (size_t j = 0; j < cols; ++j)
            if (bo_get(src, wpr, i, j)) {
                bo_eg_code(&e, (int)((long)j - last - 1), 0, NULL);
                last = (long)j;
            }
        bo_eg_code(&e, (int)((long)cols - 1 - last), 1, NULL);
    }
    free(R);
}

size_t bo_plane_runs(const uint64_t* plane, size_t rows, size_t cols, size_t wpr,
                     uint32_t* runs, uint8_t* eols, size_t cap) {
    size_t n = 0;
    for (size_t i = 0; i < rows; ++i) {
        long last = -1;
        for (size_t j = 0; j < cols; ++j)
            if (bo_get(plane, wpr, i, j)) {
                if (n < cap) { runs[n] = (uint32_t)((long)j - last - 1); eols[n] = 0; }
                ++n;
                last = (long)j;
            }
        if (n < cap) { runs[n] = (uint32_t)((long)cols - 1 - last); eols[n] = 1; }
        ++n;
    }
    return n;
}

int64_t bo_golomb_samples(const uint32_t* s, size_t n, uint8_t* out, size_t cap_bytes,
                          uint32_t* k_out, uint32_t* len_out) {
    bo_bw bw;
    bo_bw_init(&bw, out, cap_bytes);
    bo_golomb g;
    bo_golomb_init(&g);
    for (size_t i = 0; i < n; ++i) {
        if (k_out) k_out[i] = g.k;
        const uint32_t len = bo_golomb_code(&g, s[i], &bw);
        if (len_out) len_out[i] = len;
    }
    if (out && (bw.overflow || ((bw.pos + 63) / 64) * 8 > cap_bytes)) return -1;
    return g.bitcount;
}

/* ------------------------------------------------------------------------- */
typedef struct {
    const uint8_t* buf;
    uint64_t nbits, pos;
} bo_br;

static int bo_br_bit(bo_br* r) {
    if (r->pos >= r->nbits) return -1;
    const int b = (r->buf[r->pos >> 3] >> (7 - (r->pos & 7))) & 1;
    r->pos++;
    return b;
}

void bo_unmed(const uint64_t* R, uint64_t* P, size_t rows, size_t cols, size_t wpr, int corner) {
    memset(P, 0, sizeof(uint64_t) * rows * wpr);
    for (size_t i = 0; i < rows; ++i)
        for (size_t j = 0; j < cols; ++j) {
            int v;
            if (i == 0 && j == 0) v = corner & 1;
            else {
                v = bo_get(R, wpr, i, j);
                if (j > 0) v ^= bo_get(P, wpr, i, j - 1);
                if (i > 0) v ^= bo_get(P, wpr, i - 1, j);
                if (i > 0 && j > 0) v ^= bo_get(P, wpr, i - 1, j - 1);
            }
            bo_set(P, wpr, i, j, v);
        }
}

/* Read order of GolombDecoder.cpp:17-21: k-bit binary, count zeros, the '1'. */
int bo_decode_plane_golomb(const uint8_t* stream, uint64_t nbits, size_t rows, size_t cols,
                           size_t wpr, int predict, int corner, uint64_t* plane) {
    uint64_t* dst = plane;
    uint64_t* R = NULL;
    if (predict) { R = (uint64_t*)malloc(sizeof(uint64_t) * rows * wpr + 8); dst = R; }
    memset(dst, 0, sizeof(uint64_t) * rows * wpr);
    bo_br br = {stream, nbits, 0};
    bo_golomb g;
    bo_golomb_init(&g);
    int rc = 0;
    for (size_t i = 0; i < rows && !rc; ++i) {
        size_t j = 0;
        for (;;) {
            uint32_t bin = 0;
            for (uint32_t b = 0; b < g.k; ++b) {
                const int v = bo_br_bit(&br);
                if (v < 0) { rc = 1; break; }
                bin = (bin << 1) | (uint32_t)v;
            }
            if (rc) break;
            uint64_t unary = 0;
            int v;
            while ((v = bo_br_bit(&br)) == 0) ++unary;
            if (v < 0) { rc = 1; break; }
            const uint64_t s64 = (unary << g.k) | bin;
            if (j + s64 > cols) { rc = 2; break; }
            bo_golomb_code(&g, (uint32_t)s64, NULL);
            const size_t pos = j + (size_t)s64;
            if (pos == cols) break;  /* EOL sample */
            bo_set(dst, wpr, i, pos, 1);
            j = pos + 1;
        }
    }
    if (!rc && predict) bo_unmed(R, plane, rows, cols, wpr, corner);
    free(R);
    return rc;
}

/* ------------------------------------------------------------------------- */
/* binmat.cpp:267-298: word-level extraction with the reference's compact block
 * indexing (k over rows*blocks_per_row), so a right-edge tile reads the first
 * word of the next row and anything past the last block reads 0. */
static uint64_t bo_block_at(const uint64_t* I, size_t bpr, size_t wpr, size_t data_blocks, size_t k) {
    if (k >= data_blocks) return 0;
    return I[(k / bpr) * wpr + k % bpr];
}

void bo_get_submatrix(const uint64_t* I, size_t rows, size_t cols, size_t wpr,
                      size_t i0, size_t i1, size_t j0, size_t j1, uint64_t* B, size_t bwpr) {
    const size_t bpr = (cols + 63) / 64;
    const size_t data_blocks = rows * bpr;
    const size_t brows = i1 - i0, bbpr = (j1 - j0 + 63) / 64;
    const size_t boff = j0 % 64;
    const size_t doff = j0 / 64 + i0 * bpr;
    for (size_t di = 0; di < brows; ++di)
        for (size_t dj = 0; dj < bbpr; ++dj) {
            const size_t k1 = doff + di * bpr + dj;
            uint64_t v;
            if (boff == 0) v = bo_block_at(I, bpr, wpr, data_blocks, k1);
            else
                v = (bo_block_at(I, bpr, wpr, data_blocks, k1) << boff) |
                    (bo_block_at(I, bpr, wpr, data_blocks, k1 + 1) >> (64 - boff));
            B[di * bwpr + dj] = v;
        }
}

/* binmat.cpp:373-414 for a source of at most 64 columns (one block per row),
 * which is every use on the path. Returns without effect for wider sources. */
void bo_set_submatrix(uint64_t* I, size_t rows, size_t cols, size_t wpr,
                      size_t i0, size_t j0, const uint64_t* B, size_t brows, size_t bcols, size_t bwpr) {
    if (bcols == 0 || bcols > 64) return;
    const size_t bpr = (cols + 63) / 64, last = bpr - 1;
    const uint64_t itrail = ~0ull << (63 - (cols - 1) % 64);
    const uint64_t btrail = ~0ull << (63 - (bcols - 1) % 64);
    const size_t boff = j0 % 64;
    const size_t lastoff = (boff + bcols) % 64;
    const size_t spanned = (63 + boff + bcols) / 64;
    for (size_t si = 0, di = i0; si < brows && di < rows; ++si, ++di) {
        const uint64_t sb = B[si * bwpr] & btrail;  /* B.get_block(si,0) */
        uint64_t* row = I + di * wpr;
        const size_t dj = j0 / 64;
        if (boff == 0 || spanned == 1) {
            const uint64_t mr = boff ? (~0ull >> boff) : ~0ull;
            const uint64_t ml = lastoff ? (~0ull << (64 - lastoff)) : ~0ull;
            const uint64_t m = mr & ml;
            uint64_t cur = row[dj];
            if (dj == last) cur &= itrail;           /* get_block trail mask */
            row[dj] = (cur & ~m) | ((sb >> boff) & m);
        } else {
            const uint64_t hi = ~0ull << (64 - boff);      /* bits kept in word dj */
            const uint64_t m3 = ~0ull << (64 - lastoff);   /* bits set in word dj+1 */
            uint64_t cur = row[dj];
            if (dj == last) cur &= itrail;
            row[dj] = (cur & hi) | (sb >> boff);
            if (dj < last) {
                uint64_t nxt = row[dj + 1];
                if (dj + 1 == last) nxt &= itrail;
                row[dj + 1] = (nxt & ~m3) | ((sb << (64 - boff)) & m3);
            }
        }
    }
}

double bo_enumL(unsigned n, unsigned r) {
    if (r == 0 || r >= n) return 0.0;  /* C(n,0) = C(n,n) = 1 */
    unsigned m = r * 2 > n ? n - r : r;
    if (m == 1) {
        /* log2 n; exact for powers of two (GSL's rounding here is what SURVEY
         * §8 c calls "parity unpinned at w in {1, M-1}") */
        if ((n & (n - 1)) == 0) {
            double e = 0;
            while ((1u << (unsigned)e) < n) e += 1.0;
            return e;
        }
        return (double)(log2l((long double)n));
    }
    const long double ln = lgammal((long double)n + 1.0L) - lgammal((long double)m + 1.0L) -
                           lgammal((long double)(n - m) + 1.0L);
    return (double)(ln * 1.442695040888963407359924681001892137L);
}

int64_t bo_patch_encode(uint64_t* I, size_t rows, size_t cols, size_t wpr, unsigned W,
                        const uint64_t* lentab, uint32_t* w_nonpred, uint32_t* w_pred,
                        char* modes, uint64_t* L_out, uint8_t* stream, size_t cap_bytes) {
    if (W == 0 || W > 64) return -1;
    const size_t Ny = (W - 1 + rows) / W, Nx = (W - 1 + cols) / W;
    uint64_t P[64], dP[64];
    bo_bw bw;
    bo_bw_init(&bw, stream, cap_bytes);
    bo_golomb g;
    bo_golomb_init(&g);
    uint64_t L = 0;
    size_t t = 0;
    for (size_t ti = 0; ti < Ny; ++ti)
        for (size_t tj = 0; tj < Nx; ++tj, ++t) {
            const size_t i0 = ti * W, j0 = tj * W;
            bo_get_submatrix(I, rows, cols, wpr, i0, i0 + W, j0, j0 + W, P, 1);
            const uint64_t wo = bo_weight(P, W, W, 1);
            bo_med(P, dP, W, W, 1);
            const uint64_t wO = bo_weight(dP, W, W, 1);
            const int pred = lentab[wo] > lentab[wO];     /* compress7_test.cpp:248 */
            const uint64_t w = pred ? wO : wo;
            L += lentab[w];
            if (w_nonpred) w_nonpred[t] = (uint32_t)wo;
            if (w_pred) w_pred[t] = (uint32_t)wO;
            if (modes) modes[t] = pred ? 'O' : 'o';
            bo_golomb_code(&g, (uint32_t)w, &bw);          /* compress7_test.cpp:270 */
            bo_set_submatrix(I, rows, cols, wpr, i0, j0, pred ? dP : P, W, W, 1); /* :272 */
        }
    if (L_out) *L_out = L;
    if (stream && bw.overflow) return -1;
    return g.bitcount;
}

/* ------------------------------------------------------------------------- */
uint64_t bo_baseline_planes(const uint64_t* planes, int nplanes, size_t rows, size_t cols,
                            size_t wpr, int predict, int do_eg, int* threads_used) {
    uint64_t total = 0;
    int nt = 1;
#ifdef _OPENMP
    nt = omp_get_max_threads();
#pragma omp parallel for schedule(dynamic, 1) reduction(+ : total)
#endif
    for (int p = 0; p < nplanes; ++p) {
        const uint64_t* P = planes + (size_t)p * rows * wpr;
        const size_t cap = (size_t)(2.5 * (double)rows * (double)(cols + 1) / 8.0) + 64;
        uint8_t* buf = (uint8_t*)malloc(cap);
        int64_t b = bo_encode_plane(P, rows, cols, wpr, predict, 0, buf, cap, NULL);
        if (b > 0) total += (uint64_t)b;
        if (do_eg) {
            b = bo_encode_plane(P, rows, cols, wpr, predict, 1, buf, cap, NULL);
            if (b > 0) total += (uint64_t)b;
        }
        free(buf);
    }
    if (threads_used) *threads_used = nt;
    return total;
}

/* compress_test.cpp:73-111, loop for loop (int conversions included: int(i0 - W) of an
 * unsigned difference is negative for i0 < W, so the first loop is skipped). */
void bo_patch_search(const uint64_t* I, size_t rows, size_t cols, size_t wpr, unsigned W,
                     uint32_t* besti, uint32_t* bestj, uint32_t* bestd) {
    bo_patch_search_rows(I, rows, cols, wpr, W, 0, (W - 1 + rows) / W, besti, bestj, bestd);
}

void bo_patch_search_rows(const uint64_t* I, size_t rows, size_t cols, size_t wpr, unsigned W,
                          size_t tr0, size_t tr1, uint32_t* besti, uint32_t* bestj, uint32_t* bestd) {
    const size_t Ny = (W - 1 + rows) / W, Nx = (W - 1 + cols) / W;
    const uint64_t topW = W >= 64 ? ~0ull : ~(~0ull >> W);
    uint64_t P[64], P2[64];
    if (tr1 > Ny) tr1 = Ny;
    size_t li = tr0 * Nx;
    for (size_t i = tr0; i < tr1; i++)
        for (size_t j = 0; j < Nx; j++, li++) {
            const size_t i0 = i * W, j0 = j * W;
            bo_get_submatrix(I, rows, cols, wpr, i0, i0 + W, j0, j0 + W, P, 1);
            size_t bi = 0, bj = 0, bd = (size_t)W * W;
            int i2;
            int perfect = 0;
            for (i2 = 0; (i2 <= (int)(i0 - W)) && !perfect; i2++) {
                for (int j2 = 0; j2 < (int)cols; j2++) {
                    bo_get_submatrix(I, rows, cols, wpr, (size_t)i2, (size_t)i2 + W, (size_t)j2, (size_t)j2 + W, P2, 1);
                    size_t d = 0;
                    for (unsigned r = 0; r < W; r++) d += (size_t)__builtin_popcountll((P[r] ^ P2[r]) & topW);
                    if (d < bd) { bd = d; bi = (size_t)i2; bj = (size_t)j2; }
                    if (bd == 0) { perfect = 1; break; }
                }
            }
            for (; (i2 <= (int)i0) && !perfect; i2++) {
                for (int j2 = 0; j2 <= (int)(j0 - W); j2++) {
                    bo_get_submatrix(I, rows, cols, wpr, (size_t)i2, (size_t)i2 + W, (size_t)j2, (size_t)j2 + W, P2, 1);
                    size_t d = 0;
                    for (unsigned r = 0; r < W; r++) d += (size_t)__builtin_popcountll((P[r] ^ P2[r]) & topW);
                    if (d < bd) { bd = d; bi = (size_t)i2; bj = (size_t)j2; }
                    if (bd == 0) { perfect = 1; break; }
                }
            }
            besti[li] = (uint32_t)bi;
            bestj[li] = (uint32_t)bj;
            bestd[li] = (uint32_t)bd;
        }
}

/* compress7_test.cpp:117-275 with a search window R and a match threshold T, loop for loop.
 * Search region of tile (i0, j0) (:127-174): rows i0 .. mini2 at columns maxj2 .. minj, then rows
 * i0-W .. mini at columns maxj .. minj, both scanned downwards, stopping at the first window with
 * distance <= T. The image is read as it stands after the residual write-back of every earlier
 * tile (:266, :272), so the search sees residuals, and at j0 = 0 its first window is the tile
 * itself. Lengths follow :218-221 in double: nomatch 2 + enumL[w], match (2 + idx_len) + enumL[w]
 * with idx_len = ceil(log2(search_win_size)); a search_win_size <= 0 (log2 of 0 or of a negative
 * number, converted to idx_t: 2^63 on x86-64) makes the match length huge, so such a tile never
 * takes the match branch. bestd = W*W+1 when the region holds no window (:124). */
int bo_match_encode(uint64_t* I, size_t rows, size_t cols, size_t wpr, unsigned W, unsigned T, unsigned R,
                    const double* enumL, uint32_t* besti, uint32_t* bestj, uint32_t* bestd,
                    uint32_t* weights, char* modes, uint64_t* stats, uint8_t* stream_match,
                    uint8_t* stream_nomatch, size_t cap_bytes) {
    return bo_match_encode_v(I, rows, cols, wpr, W, T, R, enumL, besti, bestj, bestd, weights, modes, stats,
                             stream_match, stream_nomatch, cap_bytes, 0, NULL);
}

/* invert = 0: compress7_test.cpp:117-275; invert = 1: compress8_test.cpp:126-272, which differs in
 *  - bestinv = (P.weight() - M) < P.weight() (:136; idx_t arithmetic: true iff the tile is all 1s);
 *  - perfect_match = P.weight() <= T || P.weight() >= M - T before any search (:137);
 *  - per window d = dist(P, P2) replaced by M - d when (M - d) < d, that window's inv = true (:156-161;
 *    the driver leaves inv uninitialised otherwise: defined here as false) and bestinv = inv with
 *    every improvement (:163);
 *  - P.flip() when bestinv (:207-210) before P3 and both weights are formed;
 *  - the match lengths carry one more bit (3 + idx_len + enumL, :250-251).
 * inverted (nullable): bestinv per tile. */
int bo_match_encode_v(uint64_t* I, size_t rows, size_t cols, size_t wpr, unsigned W, unsigned T, unsigned R,
                      const double* enumL, uint32_t* besti, uint32_t* bestj, uint32_t* bestd,
                      uint32_t* weights, char* modes, uint64_t* stats, uint8_t* stream_match,
                      uint8_t* stream_nomatch, size_t cap_bytes, int invert, uint8_t* inverted) {
    if (W == 0 || W > 64 || rows % W || cols % W) return -1;
    const size_t Ny = rows / W, Nx = cols / W, M = (size_t)W * W;
    const uint64_t topW = W >= 64 ? ~0ull : ~(~0ull >> W);
    uint64_t P[64], P2[64], P3[64], dP[64], dP3[64];
    bo_bw bwm, bwn;
    bo_bw_init(&bwm, stream_match, cap_bytes);
    bo_bw_init(&bwn, stream_nomatch, cap_bytes);
    bo_golomb gm, gn;
    bo_golomb_init(&gm);
    bo_golomb_init(&gn);
    uint64_t L = 0, matches = 0;
    size_t li = 0;
    const int iW = (int)W, iR = (int)R, icols = (int)cols;
    for (size_t i = 0; i < Ny; i++)
        for (size_t j = 0; j < Nx; j++, li++) {
            const int i0 = (int)(i * W), j0 = (int)(j * W);
            bo_get_submatrix(I, rows, cols, wpr, (size_t)i0, (size_t)i0 + W, (size_t)j0, (size_t)j0 + W, P, 1);
            size_t bi = 0, bj = 0, bd = M + 1;
            int perfect = 0, bestinv = 0;
            if (invert) {                                                /* compress8_test.cpp:136-137 */
                const uint64_t w0 = bo_weight(P, W, W, 1);
                bestinv = (uint64_t)(w0 - M) < w0;
                perfect = w0 <= T || w0 >= (uint64_t)M - (uint64_t)T;
            }
            const int mini = i0 > iR ? i0 - iR : 0;
            const int minj = j0 > iR ? j0 - iR : 0;
            const int maxj = (j0 + iR > icols - iW) ? icols - iW : j0 + iR;
            const int mini2 = i0 > iW ? i0 - iW : 0;
            const int maxj2 = j0 > iW ? j0 - iW : 0;
            const int64_t swin = (int64_t)(i0 - mini2) * (maxj2 - minj) + (int64_t)(mini2 - mini) * (maxj - minj);
            for (int pass = 0; pass < 2 && !perfect; pass++) {
                const int ihi = pass ? i0 - iW : i0, ilo = pass ? mini : mini2, jhi = pass ? maxj : maxj2;
                for (int i2 = ihi; i2 >= ilo && !perfect; i2--)
                    for (int j2 = jhi; j2 >= minj; j2--) {
                        bo_get_submatrix(I, rows, cols, wpr, (size_t)i2, (size_t)i2 + W, (size_t)j2, (size_t)j2 + W, P2, 1);
                        size_t d = 0;
                        for (unsigned r = 0; r < W; r++) d += (size_t)__builtin_popcountll((P[r] ^ P2[r]) & topW);
                        int inv = 0;
                        if (invert && M - d < d) { inv = 1; d = M - d; }    /* compress8_test.cpp:156-161 */
                        if (d < bd) { bd = d; bi = (size_t)i2; bj = (size_t)j2; bestinv = inv; }
                        if (bd <= T) { perfect = 1; break; }
                    }
            }
            if (bestinv)                                                 /* compress8_test.cpp:207-210 */
                for (unsigned r = 0; r < W; r++) P[r] = ~P[r];
            if (bd <= M) {                                               /* :185-190 */
                bo_get_submatrix(I, rows, cols, wpr, bi, bi + W, bj, bj + W, P2, 1);
                for (unsigned r = 0; r < W; r++) P3[r] = (P[r] ^ P2[r]) & topW;
            } else {
                for (unsigned r = 0; r < W; r++) P3[r] = P[r] & topW;
            }
            for (unsigned r = 0; r < W; r++) P[r] &= topW;
            bo_med(P, dP, W, W, 1);
            bo_med(P3, dP3, W, W, 1);
            const uint64_t w_mn = bo_weight(P3, W, W, 1), w_nn = bo_weight(P, W, W, 1);
            const uint64_t w_mp = bo_weight(dP3, W, W, 1), w_np = bo_weight(dP, W, W, 1);
            uint64_t idx_len = 0x8000000000000000ull;                     /* :212 */
            if (swin >= 1) idx_len = swin == 1 ? 0 : 64 - (uint64_t)__builtin_clzll((uint64_t)(swin - 1));
            const uint64_t nn_len = (uint64_t)(2.0 + enumL[w_nn]), np_len = (uint64_t)(2.0 + enumL[w_np]);
            uint64_t mn_len = ~0ull, mp_len = ~0ull;
            if (swin >= 1) {  /* compress8_test.cpp:250-251: one more bit (invert / not) */
                mn_len = (uint64_t)((double)(2 + (invert ? 1 : 0) + idx_len) + enumL[w_mn]);
                mp_len = (uint64_t)((double)(2 + (invert ? 1 : 0) + idx_len) + enumL[w_mp]);
            }
            const int mpred = mn_len > mp_len, npred = nn_len > np_len;  /* :232, :243 */
            const uint64_t match_len = mpred ? mp_len : mn_len, match_w = mpred ? w_mp : w_mn;
            const uint64_t nomatch_len = npred ? np_len : nn_len, nomatch_w = npred ? w_np : w_nn;
            const int take = nomatch_len > match_len;                   /* :255 */
            const uint64_t* res = take ? (mpred ? dP3 : P3) : (npred ? dP : P);
            const uint64_t w = take ? match_w : nomatch_w;
            if (take) {
                bo_golomb_code(&gm, (uint32_t)w, &bwm);
                matches++;
                L += match_len;
            } else {
                bo_golomb_code(&gn, (uint32_t)w, &bwn);
                L += nomatch_len;
            }
            bo_set_submatrix(I, rows, cols, wpr, (size_t)i0, (size_t)j0, res, W, W, 1);
            if (besti) besti[li] = (uint32_t)bi;
            if (bestj) bestj[li] = (uint32_t)bj;
            if (bestd) bestd[li] = (uint32_t)bd;
            if (weights) weights[li] = (uint32_t)w;
            if (modes) modes[li] = take ? (mpred ? 'X' : 'x') : (npred ? 'O' : 'o');
            if (inverted) inverted[li] = (uint8_t)bestinv;
        }
    if (stats) {
        stats[0] = matches;
        stats[1] = (uint64_t)gm.bitcount;
        stats[2] = (uint64_t)gn.bitcount;
        stats[3] = L;
    }
    if ((stream_match && bwm.overflow) || (stream_nomatch && bwn.overflow)) return -1;
    return 0;
}

/* The loops of compress4_test.cpp:89-170 (variant 4), compress5_test.cpp:89-170 (5) and
 * compress6_test.cpp:111-208 (6): no med, one coder decision, the residual written back only on a
 * match. Against compress7_test.cpp (bo_match_encode_v) they differ in
 *  - the first loop's columns j2 = j0 - W .. minj (int(j0-W), :104 / :104 / :126: none at j0 = 0);
 *  - idx_len = ceil(log2(li)) of the tile's raster index (:147 / :148 / :187; li = 0: log2(0) = -inf,
 *    converted to idx_t: 2^63 on x86-64, so the first tile never matches);
 *  - nomatch_len = 1 + enumL(M, P.weight()); variants 4/5: match_len = 1 + idx_len + enumL(M, bestd)
 *    when bestd <= M, else 100000 (:154 / :155); variant 6: match_len = 1 + idx_len + enumL(M,
 *    P3.weight()) with P3 = P ^ best window, or P itself when no window (:166-194);
 *  - a match codes bestd (4/5) / P3.weight() (6) with golomb_match and writes P3 back (:164 / :165 /
 *    :203); otherwise P.weight() with golomb_nomatch and the tile is left as it is;
 *  - variant 5 keeps a window when (d - worstd) > (bestd - worstd) in idx_t arithmetic, worstd =
 *    W*W/2 (compress5_test.cpp:94,109,126): unsigned wrap makes every d < worstd beat every d >= worstd
 *    and the initial W*W+1, and among those the larger d win.
 * modes: 'x' match, 'o' no match. Returns 0, -1 on a bad argument or stream overflow. */
int bo_match_encode_var(uint64_t* I, size_t rows, size_t cols, size_t wpr, unsigned W, unsigned T, unsigned R,
                        const double* enumL, uint32_t* besti, uint32_t* bestj, uint32_t* bestd,
                        uint32_t* weights, char* modes, uint64_t* stats, uint8_t* stream_match,
                        uint8_t* stream_nomatch, size_t cap_bytes, int variant) {
    if (W == 0 || W > 64 || rows % W || cols % W || variant < 4 || variant > 6) return -1;
    const size_t Ny = rows / W, Nx = cols / W, M = (size_t)W * W;
    const uint64_t worstd = (uint64_t)(W * W / 2);
    const uint64_t topW = W >= 64 ? ~0ull : ~(~0ull >> W);
    uint64_t P[64], P2[64], P3[64];
    bo_bw bwm, bwn;
    bo_bw_init(&bwm, stream_match, cap_bytes);
    bo_bw_init(&bwn, stream_nomatch, cap_bytes);
    bo_golomb gm, gn;
    bo_golomb_init(&gm);
    bo_golomb_init(&gn);
    uint64_t L = 0, matches = 0;
    size_t li = 0;
    const int iW = (int)W, iR = (int)R, icols = (int)cols;
    for (size_t i = 0; i < Ny; i++)
        for (size_t j = 0; j < Nx; j++, li++) {
            const int i0 = (int)(i * W), j0 = (int)(j * W);
            bo_get_submatrix(I, rows, cols, wpr, (size_t)i0, (size_t)i0 + W, (size_t)j0, (size_t)j0 + W, P, 1);
            for (unsigned r = 0; r < W; r++) P[r] &= topW;
            uint64_t bi = 0, bj = 0, bd = M + 1;
            int perfect = 0;
            const int mini = i0 > iR ? i0 - iR : 0;
            const int mini2 = i0 > iW ? i0 - iW : 0;
            const int minj = j0 > iR ? j0 - iR : 0;
            const int maxj = (j0 + iR > icols - iW) ? icols - iW : j0 + iR;
            for (int pass = 0; pass < 2 && !perfect; pass++) {
                const int ihi = pass ? i0 - iW : i0, ilo = pass ? mini : mini2, jhi = pass ? maxj : j0 - iW;
                for (int i2 = ihi; i2 >= ilo && !perfect; i2--)
                    for (int j2 = jhi; j2 >= minj; j2--) {
                        bo_get_submatrix(I, rows, cols, wpr, (size_t)i2, (size_t)i2 + W, (size_t)j2, (size_t)j2 + W, P2, 1);
                        uint64_t d = 0;
                        for (unsigned r = 0; r < W; r++) d += (uint64_t)__builtin_popcountll((P[r] ^ P2[r]) & topW);
                        const int better = variant == 5 ? (d - worstd) > (bd - worstd) : d < bd;
                        if (better) { bd = d; bi = (uint64_t)i2; bj = (uint64_t)j2; }
                        if (bd <= T) { perfect = 1; break; }
                    }
            }
            if (variant == 6 && bd > M) {
                for (unsigned r = 0; r < W; r++) P3[r] = P[r];
            } else {
                bo_get_submatrix(I, rows, cols, wpr, bi, bi + W, bj, bj + W, P2, 1);
                for (unsigned r = 0; r < W; r++) P3[r] = (P[r] ^ P2[r]) & topW;
            }
            const uint64_t wP = bo_weight(P, W, W, 1), w3 = bo_weight(P3, W, W, 1);
            const uint64_t idx_len = li == 0 ? 0x8000000000000000ull : li == 1 ? 0 : 64 - (uint64_t)__builtin_clzll((uint64_t)(li - 1));
            const uint64_t nomatch_len = (uint64_t)(1.0 + enumL[wP]);
            uint64_t match_len, match_w;
            if (variant == 6) {
                match_len = (uint64_t)((double)(1 + idx_len) + enumL[w3]);
                match_w = w3;
            } else {
                match_len = bd <= M ? (uint64_t)((double)(1 + idx_len) + enumL[bd]) : 100000;
                match_w = bd;
            }
            const int take = nomatch_len > match_len;
            if (take) {
                bo_golomb_code(&gm, (uint32_t)match_w, &bwm);
                matches++;
                L += match_len;
                bo_set_submatrix(I, rows, cols, wpr, (size_t)i0, (size_t)j0, P3, W, W, 1);
            } else {
                bo_golomb_code(&gn, (uint32_t)wP, &bwn);
                L += nomatch_len;
            }
            if (besti) besti[li] = (uint32_t)bi;
            if (bestj) bestj[li] = (uint32_t)bj;
            if (bestd) bestd[li] = (uint32_t)bd;
            if (weights) weights[li] = (uint32_t)(take ? match_w : wP);
            if (modes) modes[li] = take ? 'x' : 'o';
        }
    if (stats) {
        stats[0] = matches;
        stats[1] = (uint64_t)gm.bitcount;
        stats[2] = (uint64_t)gn.bitcount;
        stats[3] = L;
    }
    if ((stream_match && bwm.overflow) || (stream_nomatch && bwn.overflow)) return -1;
    return 0;
}

/* ---- binary_matrix algebra over GF(2) ---------------------------------------------------- */

static int gf2_bit(const uint64_t* M, size_t wpr, size_t i, size_t j) {
    return (int)((M[i * wpr + j / 64] >> (63 - j % 64)) & 1u);
}

/* binmat.cpp:199-214: for every column j, copy_col_to (col cleared, bit i = A(i, j)) then set_row */
void bo_gf2_transpose(const uint64_t* src, size_t rows, size_t cols, uint64_t* dst) {
    const size_t swpr = (cols + 63) / 64, dwpr = (rows + 63) / 64;
    for (size_t j = 0; j < cols; ++j) {
        uint64_t* d = dst + j * dwpr;
        for (size_t q = 0; q < dwpr; ++q) d[q] = 0;
        for (size_t i = 0; i < rows; ++i)
            if (gf2_bit(src, swpr, i, j)) d[i / 64] |= 0x8000000000000000ull >> (i % 64);
    }
}

int bo_gf2_mul(int op, const uint64_t* A, size_t a_rows, size_t a_cols, const uint64_t* B, size_t b_rows,
               size_t b_cols, uint64_t* C, size_t c_rows, size_t c_cols) {
    const size_t aw = (a_cols + 63) / 64, bw = (b_cols + 63) / 64, cw = (c_cols + 63) / 64;
    if (op == 0) {  /* mul_AB: C.clear(); for k, for i: if A(i,k) row i of C ^= row k of B */
        if (c_rows != a_rows || c_cols != b_cols || a_cols != b_rows) return -1;
        for (size_t q = 0; q < c_rows * cw; ++q) C[q] = 0;
        for (size_t k = 0; k < b_rows; ++k)
            for (size_t i = 0; i < a_rows; ++i)
                if (gf2_bit(A, aw, i, k))
                    for (size_t j = 0; j < bw; ++j) C[i * cw + j] ^= B[k * bw + j];
        return 0;
    }
    if (op == 1) {  /* mul_AtB: for k < A.rows, for i < A.cols: if A(k,i) row i of C ^= row k of B */
        if (c_rows != a_cols || c_cols != b_cols || a_rows != b_rows) return -1;
        for (size_t q = 0; q < c_rows * cw; ++q) C[q] = 0;
        for (size_t k = 0; k < a_rows; ++k)
            for (size_t i = 0; i < a_cols; ++i)
                if (gf2_bit(A, aw, k, i))
                    for (size_t j = 0; j < bw; ++j) C[i * cw + j] ^= B[k * bw + j];
        return 0;
    }
    if (op == 2) {  /* mul_ABt: C(i,j) = parity of XOR over A's blocks of A_ik & B_jk, j < B.cols */
        if (c_rows != a_rows || c_cols != b_rows || a_cols != b_cols) return -1;
        for (size_t i = 0; i < a_rows; ++i)
            for (size_t j = 0; j < b_cols; ++j) {
                uint64_t acc = 0;
                for (size_t k = 0; k < aw; ++k) acc ^= A[i * aw + k] & (j < b_rows ? B[j * bw + k] : 0ull);
                const size_t kc = i * cw + j / 64;
                if (kc >= c_rows * cw) continue;  /* C.set past the storage: dropped */
                const uint64_t m = 0x8000000000000000ull >> (j % 64);
                if (__builtin_parityll(acc)) C[kc] |= m; else C[kc] &= ~m;
            }
        return 0;
    }
    if (op == 3) {  /* mul_AtBt: "FALTA!" */
        if (c_rows != a_cols || c_cols != b_rows || a_rows != b_cols) return -1;
        return 0;
    }
    return -1;
}
