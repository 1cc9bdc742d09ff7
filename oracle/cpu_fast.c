/* cpu_fast.c -- TEST / BENCH INFRASTRUCTURE ONLY (bench.py's "strong CPU" baseline line; never
 * linked into the product). A word-parallel CPU encoder of the same streams the GPU writes:
 *   med in word form (pred.cpp:3-15: R = D ^ (D >> 1 | Dl << 63), D = P ^ U, R(0,0) = 0),
 *   runs by count-leading-zeros over residual words,
 *   Golomb codewords (GolombCoder.cpp:13-34: k from (N, A), k-bit binary part, unary zeros, '1')
 *   through a 64-bit accumulator, EG as written (eg.cpp:20-37: ~R of the row and '1'; one extra
 *   '0' after the plane's first 1) as word copies.
 * OpenMP over planes (each plane's coder is serial). Checked against the oracle's streams by
 * tests/test_oracle_golden.py::test_cpu_fast_matches_oracle. */
#include <stdint.h>
#include <stdlib.h>
#include <string.h>
#ifdef _OPENMP
#include <omp.h>
#endif

typedef struct {
    uint64_t* out; /* big-endian words; NULL = count only */
    uint64_t cap, pos, acc;
} fw;

static inline void fw_flush_word(fw* w) {
    const uint64_t i = (w->pos >> 6) - 1;
    if (w->out && i < w->cap) w->out[i] = __builtin_bswap64(w->acc);
    w->acc = 0;
}
/* append the n (<= 64) low bits of v */
static inline void fw_put(fw* w, uint64_t v, unsigned n) {
    if (!n) return;
    const unsigned fill = (unsigned)(w->pos & 63), room = 64 - fill;
    if (n < room) {
        w->acc |= v << (room - n);
        w->pos += n;
    } else {
        w->acc |= n == room ? v & (room == 64 ? ~0ull : ((1ull << room) - 1)) : v >> (n - room);
        w->pos += room;
        fw_flush_word(w);
        const unsigned rest = n - room;
        if (rest) {
            w->acc = v << (64 - rest);
            w->pos += rest;
        }
    }
}
static inline void fw_zeros(fw* w, uint64_t n) {
    while (n) {
        const unsigned take = n > 64 ? 64 : (unsigned)n;
        fw_put(w, 0, take);
        n -= take;
    }
}
static inline void fw_end(fw* w) {
    if (w->pos & 63) {
        const uint64_t i = w->pos >> 6;
        if (w->out && i < w->cap) w->out[i] = __builtin_bswap64(w->acc);
    }
}

static inline unsigned gk(uint32_t n, uint32_t A) { /* GolombCoder.cpp:33, Golomb.h:18 */
    if (n == 0) return 1;
    unsigned k = 0;
    while (k < 31 && (n << k) < A) ++k;
    return k;
}

/* one plane: Golomb and (do_eg) EG streams; returns the Golomb bits, *eg_bits the EG bits */
static uint64_t fast_plane(const uint64_t* P, size_t rows, size_t cols, size_t wpr, int predict, int do_eg,
                           uint64_t* gout, uint64_t gcap, uint64_t* eout, uint64_t ecap, uint64_t* eg_bits) {
    const size_t used = (cols + 63) / 64;
    const uint64_t trail = cols % 64 ? ~(~0ull >> (cols % 64)) : ~0ull;
    uint64_t* R = (uint64_t*)malloc(sizeof(uint64_t) * (used + 1));
    fw g = {gout, gcap, 0, 0}, e = {eout, ecap, 0, 0};
    uint32_t n = 0, A = 0;
    int seen = 0;
    for (size_t i = 0; i < rows; ++i) {
        const uint64_t* cur = P + i * wpr;
        const uint64_t* up = i ? cur - wpr : NULL;
        uint64_t carry = 0;
        for (size_t w = 0; w < used; ++w) {
            uint64_t d = cur[w];
            if (predict) {
                if (up) d ^= up[w];
                const uint64_t r = d ^ ((d >> 1) | (carry << 63));
                carry = d & 1;
                d = r;
                if (i == 0 && w == 0) d &= ~(1ull << 63);
            }
            if (w == used - 1) d &= trail;
            R[w] = d;
        }
        /* Golomb: runs by clz */
        long last = -1;
        for (size_t w = 0; w < used; ++w) {
            uint64_t x = R[w];
            while (x) {
                const int cz = __builtin_clzll(x);
                x &= ~(1ull << (63 - cz));
                const long j = (long)(w * 64) + cz;
                const uint32_t s = (uint32_t)(j - last - 1);
                const unsigned k = gk(n, A);
                if (k) fw_put(&g, s & ((1u << k) - 1u), k);
                fw_zeros(&g, s >> k);
                fw_put(&g, 1, 1);
                ++n;
                A += s;
                last = j;
            }
        }
        {
            const uint32_t s = (uint32_t)((long)cols - 1 - last);
            const unsigned k = gk(n, A);
            if (k) fw_put(&g, s & ((1u << k) - 1u), k);
            fw_zeros(&g, s >> k);
            fw_put(&g, 1, 1);
            ++n;
            A += s;
        }
        if (do_eg) { /* ~R and '1'; a '0' after the plane's first 1 */
            for (size_t w = 0; w < used; ++w) {
                const unsigned nb = w == used - 1 ? (unsigned)(cols - 64 * w) : 64;
                const uint64_t v = ~R[w] >> (64 - nb);
                if (!seen && R[w]) {
                    const unsigned f = (unsigned)__builtin_clzll(R[w]) + 1; /* bits up to the first 1 */
                    fw_put(&e, v >> (nb - f), f);
                    fw_put(&e, 0, 1);
                    fw_put(&e, f == nb ? 0 : v & ((1ull << (nb - f)) - 1ull), nb - f);
                    seen = 1;
                } else {
                    fw_put(&e, v, nb);
                }
            }
            fw_put(&e, 1, 1);
        }
    }
    fw_end(&g);
    fw_end(&e);
    free(R);
    if (eg_bits) *eg_bits = e.pos;
    return g.pos;
}

/* Golomb (+ EG) streams of every plane, OpenMP over planes; returns the total bits. When gout /
 * eout are given, plane p's streams go to gout + p * gslot / eout + p * eslot (words). */
uint64_t cf_encode_planes(const uint64_t* planes, int nplanes, size_t rows, size_t cols, size_t wpr, int predict,
                          int do_eg, uint64_t* gout, uint64_t gslot, uint64_t* eout, uint64_t eslot,
                          uint64_t* gbits, uint64_t* ebits, int* threads_used) {
    uint64_t total = 0;
    int nt = 1;
#ifdef _OPENMP
    nt = omp_get_max_threads();
    if (nt > nplanes) nt = nplanes;
#pragma omp parallel for schedule(dynamic, 1) reduction(+ : total) num_threads(nt)
#endif
    for (int p = 0; p < nplanes; ++p) {
        uint64_t* go = gout ? gout + (size_t)p * gslot : NULL;
        uint64_t* eo = eout ? eout + (size_t)p * eslot : NULL;
        const uint64_t gcap = gout ? gslot : 0;
        const uint64_t ecap = eout ? eslot : 0;
        uint64_t eb = 0;
        const uint64_t b = fast_plane(planes + (size_t)p * rows * wpr, rows, cols, wpr, predict, do_eg, go, gcap, eo,
                                      ecap, &eb);
        if (gbits) gbits[p] = b;
        if (ebits) ebits[p] = eb;
        total += b + eb;
    }
    if (threads_used) *threads_used = nt;
    return total;
}
