/* oracle_san.c -- the oracle (oracle/bic_oracle.c) and the strong-CPU encoder (oracle/cpu_fast.c)
 * under AddressSanitizer + UndefinedBehaviorSanitizer (oracle/Makefile san, tests/test_sanitize.py):
 * every entry point on ragged shapes, with round-trip self-checks. Exit 0 = clean. */
#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>

#include "../../oracle/bic_oracle.h"

uint64_t cf_encode_planes(const uint64_t* planes, int nplanes, size_t rows, size_t cols, size_t wpr, int predict,
                          int do_eg, uint64_t* gout, uint64_t gslot, uint64_t* eout, uint64_t eslot,
                          uint64_t* gbits, uint64_t* ebits, int* threads_used);

static int fails = 0;
#define CHECK(c)                                                   \
    do {                                                           \
        if (!(c)) {                                                \
            printf("FAIL %s:%d %s\n", __FILE__, __LINE__, #c);     \
            ++fails;                                               \
        }                                                          \
    } while (0)

static void planes_case(size_t rows, size_t cols, double p, int predict) {
    const size_t wpr = (cols + 63) / 64;
    uint64_t* P = calloc(rows * wpr, 8);
    uint64_t* Q = calloc(rows * wpr, 8);
    bo_gen_plane(0x5EED + rows + cols, p, rows, cols, wpr, P);
    const size_t cap = 2 * rows * (cols + 1) / 8 + 4096;
    uint8_t* buf = malloc(cap);
    for (int coder = 0; coder < 3; ++coder) {
        const int64_t b = bo_encode_plane(P, rows, cols, wpr, predict, coder, buf, cap, NULL);
        CHECK(b >= 0);
        if (coder == 0 && b >= 0) {
            CHECK(bo_decode_plane_golomb(buf, (uint64_t)b, rows, cols, wpr, predict,
                                         rows && cols ? (int)(P[0] >> 63) : 0, Q) == 0);
            CHECK(memcmp(P, Q, rows * wpr * 8) == 0);
        }
    }
    uint64_t* idx = calloc(2 * rows + 2, 8);
    bo_row_index(P, rows, cols, wpr, predict, idx);
    const uint64_t gslot = 2 * rows * (cols + 1) / 64 + 64, eslot = (rows * (cols + 1) + 64) / 64 + 1;
    uint64_t* G = calloc(gslot, 8);
    uint64_t* E = calloc(eslot, 8);
    uint64_t gb = 0, eb = 0;
    int nt = 0;
    cf_encode_planes(P, 1, rows, cols, wpr, predict, 1, G, gslot, E, eslot, &gb, &eb, &nt);
    const int64_t b0 = bo_encode_plane(P, rows, cols, wpr, predict, 0, buf, cap, NULL);
    CHECK((int64_t)gb == b0);
    CHECK(memcmp(G, buf, (size_t)((b0 + 63) / 64) * 8) == 0);
    CHECK(bo_weight(P, rows, cols, wpr) <= rows * cols);
    free(P), free(Q), free(buf), free(idx), free(G), free(E);
}

static void tiles_case(size_t rows, size_t cols, unsigned W) {
    const size_t wpr = (cols + 63) / 64, nt = (rows / W) * (cols / W);
    uint64_t* I = calloc(rows * wpr, 8);
    bo_gen_plane(0xABC + W, 0.1, rows, cols, wpr, I);
    uint64_t* lt = calloc(W * W + 1, 8);
    for (unsigned w = 0; w <= W * W; ++w) lt[w] = (uint64_t)(2 + bo_enumL(W * W, w));
    uint32_t* a = calloc(nt + 1, 4);
    uint32_t* b = calloc(nt + 1, 4);
    char* modes = calloc(nt + 1, 1);
    uint64_t L = 0;
    uint8_t* st = calloc(rows * cols / 2 + 4096, 1);
    CHECK(bo_patch_encode(I, rows, cols, wpr, W, lt, a, b, modes, &L, st, rows * cols / 2 + 4096) >= 0);
    double* en = calloc(W * W + 1, 8);
    for (unsigned w = 0; w <= W * W; ++w) en[w] = bo_enumL(W * W, w);
    uint32_t *bi = calloc(nt + 1, 4), *bj = calloc(nt + 1, 4), *bd = calloc(nt + 1, 4), *wt = calloc(nt + 1, 4);
    uint64_t stats[4];
    bo_gen_plane(0xDEF + W, 0.3, rows, cols, wpr, I);
    CHECK(bo_match_encode(I, rows, cols, wpr, W, 0, 2 * W, en, bi, bj, bd, wt, modes, stats, st, st,
                          rows * cols / 2 + 4096) == 0);
    const size_t ny = (rows + W - 1) / W, nx = (cols + W - 1) / W;
    uint32_t *si = calloc(ny * nx, 4), *sj = calloc(ny * nx, 4), *sd = calloc(ny * nx, 4);
    bo_patch_search(I, rows, cols, wpr, W, si, sj, sd);
    free(I), free(lt), free(a), free(b), free(modes), free(st), free(en), free(bi), free(bj), free(bd), free(wt);
    free(si), free(sj), free(sd);
}

int main(void) {
    const size_t shapes[][2] = {{1, 1}, {3, 64}, {7, 65}, {40, 1000}, {17, 4096}, {9, 130}, {2, 16384}};
    for (size_t i = 0; i < sizeof(shapes) / sizeof(shapes[0]); ++i)
        for (int pred = 0; pred < 2; ++pred) {
            planes_case(shapes[i][0], shapes[i][1], 0.5, pred);
            planes_case(shapes[i][0], shapes[i][1], 0.03, pred);
        }
    tiles_case(64, 128, 8);
    tiles_case(96, 96, 16);
    tiles_case(60, 75, 5);
    uint8_t gray[12 * 20];
    bo_gen_bytes(7, sizeof(gray), gray);
    uint64_t pl[8 * 12];
    bo_bitplanes(gray, 1, 12, 20, 8, pl, 1);
    printf("oracle_san: %d failures\n", fails);
    return fails ? 1 : 0;
}
