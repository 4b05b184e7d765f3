/*
 * host_asan.c -- the host C of libdmx under AddressSanitizer + UBSan (the
 * reference had only -Wall -g; its own inflate overran buffers).  Built by tests/c/Makefile
 * from dmx_host.c, dmx_inflate.c and dmx_gen.c compiled with -fsanitize=address,undefined,
 * linked with the HIP layer's objects; runs without a GPU:
 *   - deflate_decompress on every stream given on the command line, on every truncation of
 *     it and on single-bit flips at a stride: each call returns 0 or -E_*, never faults;
 *   - dmx_adler32_combine against a direct Adler-32 over split buffers;
 *   - dmx_gen_text / dmx_gen_random determinism;
 *   - dmx_refest_* (the reference's stats estimates) over 200 000 pseudo-random tokens of
 *     every kind (literals, lengths 3..258, distances 1..32768, all 30 distance codes, so
 *     the last split of a full alphabet is exercised) and its invalid-token error;
 *   - the boundary's error paths: deflate_compress without a GPU (-E_NEXIST), sw out of
 *     range (-E_RANGE), spawn / init / deinit.
 * Exit status 0 = no failed check (the sanitizers abort on their own findings).
 */
#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>
#include <unistd.h>

#include "dmx.h"

static uint32_t adler(const uint8_t* d, size_t n) {
    uint32_t a = 1, b = 0;
    for (size_t i = 0; i < n; i++) {
        a = (a + d[i]) % 65521u;
        b = (b + a) % 65521u;
    }
    return (b << 16) | a;
}

static int inflate_all(const uint8_t* z, size_t zn, long* ok, long* bad) {
    struct string_len in = {(unsigned char*)z, zn}, out = {NULL, 0};
    const int r = deflate_decompress(&out, &in, DEFLATE_NULLTERM);
    if (r == 0) {
        if (!out.str || out.str[out.len] != 0) return 1;   /* NULLTERM promise */
        ++*ok;
    } else {
        if (r > 0) return 1;
        ++*bad;
    }
    free(out.str);
    return 0;
}

int main(int argc, char** argv) {
    int fails = 0;
    long ok = 0, bad = 0;
    for (int a = 1; a < argc; a++) {
        FILE* f = fopen(argv[a], "rb");
        if (!f) { fprintf(stderr, "cannot open %s\n", argv[a]); return 2; }
        fseek(f, 0, SEEK_END);
        const long n = ftell(f);
        fseek(f, 0, SEEK_SET);
        uint8_t* z = (uint8_t*)malloc(n > 0 ? (size_t)n : 1);
        if (fread(z, 1, (size_t)n, f) != (size_t)n) return 2;
        fclose(f);
        /* exact copies of each length (every length up to 600, then 300 spread over the rest):
         * ASan sees any read past the end */
        const long tstep = n > 600 ? (n - 600) / 300 + 1 : 1;
        for (long t = 0; t <= n; t = t < 600 ? t + 1 : (t + tstep > n && t < n ? n : t + tstep)) {
            uint8_t* c = (uint8_t*)malloc(t ? (size_t)t : 1);
            memcpy(c, z, (size_t)t);
            fails += inflate_all(c, (size_t)t, &ok, &bad);
            free(c);
        }
        const long stride = n / 48 + 1;
        for (long p = 0; p < n; p += stride)
            for (int bit = 0; bit < 8; bit++) {
                uint8_t* c = (uint8_t*)malloc((size_t)n);
                memcpy(c, z, (size_t)n);
                c[p] ^= (uint8_t)(1u << bit);
                fails += inflate_all(c, (size_t)n, &ok, &bad);
                free(c);
            }
        free(z);
    }
    /* Adler-32 combine */
    uint8_t* buf = (uint8_t*)malloc(200000);
    dmx_gen_text(buf, 200000, 5);
    for (size_t cut = 0; cut <= 200000; cut += 9973) {
        const uint32_t c = dmx_adler32_combine(adler(buf, cut), adler(buf + cut, 200000 - cut), 200000 - cut);
        if (c != adler(buf, 200000)) { fprintf(stderr, "adler combine wrong at %zu\n", cut); fails++; }
    }
    uint8_t* b2 = (uint8_t*)malloc(200000);
    dmx_gen_text(b2, 200000, 5);
    if (memcmp(buf, b2, 200000)) { fprintf(stderr, "gen_text not deterministic\n"); fails++; }
    dmx_gen_random(buf, 99999, 7);
    dmx_gen_random(b2, 99999, 7);
    if (memcmp(buf, b2, 99999)) { fprintf(stderr, "gen_random not deterministic\n"); fails++; }
    {
        enum { NT = 200000 };
        uint32_t* tk = (uint32_t*)malloc(sizeof(uint32_t) * NT);
        struct compress_stats* rc = (struct compress_stats*)calloc(NT, sizeof(struct compress_stats));
        uint64_t x = 0x9E3779B97F4A7C15ull;
        for (int k = 0; k < NT; k++) {
            x ^= x << 13; x ^= x >> 7; x ^= x << 17;
            const uint32_t len = 3 + (uint32_t)(x % 256), dist = 1 + (uint32_t)((x >> 20) % 32768);
            tk[k] = (x >> 60) < 9 ? (uint32_t)((x >> 8) & 0xFF) : (dist << 9) | len;
        }
        dmx_refest* e = dmx_refest_create();
        uint32_t nf = 0;
        if (!e || dmx_refest_feed(e, tk, NT, rc, &nf) != 0 || nf != NT || rc[NT - 1].ll_bits <= 0 ||
            rc[NT - 1].d_bits <= 0 || rc[NT - 1].tree_bits <= 0) {
            fprintf(stderr, "refest feed\n");
            fails++;
        }
        tk[0] = (40000u << 9) | 5u;
        if (dmx_refest_feed(e, tk, 1, rc, &nf) != -E_RANGE || nf != 0) { fprintf(stderr, "refest range\n"); fails++; }
        dmx_refest_destroy(e);
        free(tk);
        free(rc);
    }
    free(buf);
    free(b2);
    /* boundary error paths without a GPU */
    int p[2];
    if (pipe(p) == 0) {
        if (write(p[1], "abcabcabc", 9) != 9) fails++;
        close(p[1]);
        const int r = deflate_compress(p[0], -1, -1, 32768, 0);
        if (r != -E_NEXIST && r != 0) { fprintf(stderr, "deflate_compress without a GPU: %d\n", r); fails++; }
        close(p[0]);
    }
    if (deflate_compress(0, -1, -1, 40000 & 0xFFFF, 0) != -E_RANGE) { fprintf(stderr, "sw range\n"); fails++; }
    deflate_compr_t* com = spawn_deflate_compr_t();
    deflate_compr_init(com, 0, 1, -1, 32768);
    deflate_compr_deinit(com);
    free(com);
    printf("host_asan: %ld streams inflated, %ld rejected with -E_*, %d failed checks\n", ok, bad, fails);
    return fails ? 1 : 0;
}
