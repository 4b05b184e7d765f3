/*
 * dmx_inflate.c -- RFC 1950/1951 inflate behind the reference's
 * deflate_decompress() signature (src/include/deflate_ext.h:16).
 *
 * The reference implementation (src/deflate_decompress.c:371-409) does not compile
 * and decodes incorrectly (dangling else at :247-250, reverse_bits
 * off by 2x, Adler-32 read little-endian at :402, 256 garbage prefix bytes at
 * :382-384).  This is a fresh decoder with the same contract:
 *   - zlib header checks as deflate_decompress_header (:347-368): CM = 8, CINFO <= 7,
 *     FCHECK, no preset dictionary;
 *   - blocks until BFINAL (:391-397): stored (:303-314), fixed (:325-334), dynamic
 *     (form_d1/form_d2 :164-235);
 *   - Adler-32 trailer verified MSB-first (RFC 1950 §2.2);
 *   - output malloc'd into decompr_dat (caller frees), '\0' appended with
 *     DEFLATE_NULLTERM (:399).
 * Returns 0 or -E_*.  Decoding is canonical-Huffman by code-length counts (one bit
 * per step), with a 9-bit first-level lookup table for the common short codes.
 */
#include <pthread.h>
#include <stdint.h>
#include <stdlib.h>
#include <string.h>

#include "../../include/dmx.h"

#define MAXBITS 15
#define FAST 9

typedef struct {
    const uint8_t* in;
    size_t n, pos;   /* byte position */
    uint64_t bitbuf;
    int bitcnt;
    uint8_t* out;
    size_t olen, ocap;
    int err;
} ist;

typedef struct {
    uint16_t count[MAXBITS + 1];
    uint16_t symbol[320];
    uint16_t fast[1 << FAST]; /* (len << 12) | sym, 0 = slow path */
} huff;

static inline int need(ist* s, int k) {
    while (s->bitcnt < k) {
        if (s->pos >= s->n) return 0;
        s->bitbuf |= (uint64_t)s->in[s->pos++] << s->bitcnt;
        s->bitcnt += 8;
    }
    return 1;
}

static inline int bits(ist* s, int k) {
    if (k == 0) return 0;
    if (!need(s, k)) { s->err = -E_LEN; return 0; }
    int v = (int)(s->bitbuf & ((1ull << k) - 1));
    s->bitbuf >>= k;
    s->bitcnt -= k;
    return v;
}

static int put(ist* s, uint8_t c) {
    if (s->olen == s->ocap) {
        size_t nc = s->ocap ? s->ocap * 2 : 1 << 16;
        uint8_t* no = (uint8_t*)realloc(s->out, nc + 1);
        if (!no) return -E_MALLOC;
        s->out = no;
        s->ocap = nc;
    }
    s->out[s->olen++] = c;
    return 0;
}

/* build a canonical decoder; returns 0 complete, >0 incomplete, <0 over-subscribed */
static int build(huff* h, const uint8_t* len, int n) {
    memset(h->count, 0, sizeof(h->count));
    for (int s = 0; s < n; s++) h->count[len[s]]++;
    if (h->count[0] == n) { memset(h->fast, 0, sizeof(h->fast)); return 0; }
    int left = 1;
    for (int l = 1; l <= MAXBITS; l++) {
        left <<= 1;
        left -= h->count[l];
        if (left < 0) return left;
    }
    uint16_t offs[MAXBITS + 1];
    offs[1] = 0;
    for (int l = 1; l < MAXBITS; l++) offs[l + 1] = offs[l] + h->count[l];
    for (int s = 0; s < n; s++)
        if (len[s]) h->symbol[offs[len[s]]++] = (uint16_t)s;
    /* first-level table: reversed canonical codes of length <= FAST */
    memset(h->fast, 0, sizeof(h->fast));
    int code = 0, idx = 0;
    for (int l = 1; l <= FAST; l++) {
        for (int k = 0; k < h->count[l]; k++, code++, idx++) {
            int r = 0;
            for (int b = 0; b < l; b++) r |= ((code >> b) & 1) << (l - 1 - b);
            for (int fill = r; fill < (1 << FAST); fill += 1 << l)
                h->fast[fill] = (uint16_t)((l << 12) | h->symbol[idx]);
        }
        code <<= 1;
    }
    return left;
}

/* Slow path: the canonical-code walk by per-length counts (first code / count / index per
 * length, one bit at a time) is the well-known loop of Mark Adler's puff.c (zlib
 * contrib/puff, zlib licence); restated here, it is not from the reference. */
static int decode(ist* s, const huff* h) {
    need(s, FAST);  /* may be short at the very end; the slow path copes */
    if (s->bitcnt >= FAST) {
        uint16_t e = h->fast[s->bitbuf & ((1u << FAST) - 1)];
        if (e) {
            int l = e >> 12;
            s->bitbuf >>= l;
            s->bitcnt -= l;
            return e & 0xFFF;
        }
    }
    int code = 0, first = 0, index = 0;
    for (int l = 1; l <= MAXBITS; l++) {
        code |= bits(s, 1);
        if (s->err) return -1;
        int count = h->count[l];
        if (code - count < first) return h->symbol[index + (code - first)];
        index += count;
        first += count;
        first <<= 1;
        code <<= 1;
    }
    s->err = -(int)E_HUFINV;
    return -1;
}

static const uint16_t lbase[29] = {3, 4, 5, 6, 7, 8, 9, 10, 11, 13, 15, 17, 19, 23, 27, 31,
                                   35, 43, 51, 59, 67, 83, 99, 115, 131, 163, 195, 227, 258};
static const uint8_t lext[29] = {0, 0, 0, 0, 0, 0, 0, 0, 1, 1, 1, 1, 2, 2, 2, 2, 3, 3, 3, 3, 4, 4, 4, 4, 5, 5, 5, 5, 0};
static const uint16_t dbase[30] = {1, 2, 3, 4, 5, 7, 9, 13, 17, 25, 33, 49, 65, 97, 129, 193, 257, 385,
                                   513, 769, 1025, 1537, 2049, 3073, 4097, 6145, 8193, 12289, 16385, 24577};
static const uint8_t dext[30] = {0, 0, 0, 0, 1, 1, 2, 2, 3, 3, 4, 4, 5, 5, 6, 6, 7, 7, 8, 8, 9, 9, 10, 10, 11, 11, 12, 12, 13, 13};

static int codes(ist* s, const huff* lh, const huff* dh) {
    for (;;) {
        int sym = decode(s, lh);
        if (s->err) return s->err;
        if (sym < 256) {
            int r = put(s, (uint8_t)sym);
            if (r) return r;
        } else if (sym == 256) {
            return 0;
        } else {
            sym -= 257;
            if (sym >= 29) return -(int)E_HUFVAL;
            int len = lbase[sym] + bits(s, lext[sym]);
            int ds = decode(s, dh);
            if (s->err) return s->err;
            if (ds < 0 || ds >= 30) return -(int)E_HUFVAL;
            size_t dist = (size_t)dbase[ds] + (size_t)bits(s, dext[ds]);
            if (s->err) return s->err;
            if (dist > s->olen) return -(int)E_HUFDIS;
            for (int k = 0; k < len; k++) {
                int r = put(s, s->out[s->olen - dist]);
                if (r) return r;
            }
        }
    }
}

static int stored(ist* s) {
    s->bitbuf >>= s->bitcnt & 7;  /* to a byte boundary */
    s->bitcnt -= s->bitcnt & 7;
    int len = bits(s, 16), nlen = bits(s, 16);
    if (s->err) return s->err;
    if (len != (~nlen & 0xFFFF)) return -(int)E_ZNLEN;
    for (int k = 0; k < len; k++) {
        int c = bits(s, 8);
        if (s->err) return s->err;
        int r = put(s, (uint8_t)c);
        if (r) return r;
    }
    return 0;
}

/* The fixed-code tables (RFC 1951 §3.2.6), built once: pthread_once makes concurrent
 * callers of deflate_decompress wait for the complete tables instead of reading a table
 * another thread is still writing. */
static huff fixed_lh, fixed_dh;
static pthread_once_t fixed_once = PTHREAD_ONCE_INIT;
static void fixed_build(void) {
    uint8_t l[288];
    for (int k = 0; k < 288; k++) l[k] = k < 144 ? 8 : k < 256 ? 9 : k < 280 ? 7 : 8;
    build(&fixed_lh, l, 288);
    for (int k = 0; k < 30; k++) l[k] = 5;
    build(&fixed_dh, l, 30);
}

static int fixed(ist* s) {
    pthread_once(&fixed_once, fixed_build);
    return codes(s, &fixed_lh, &fixed_dh);
}

static int dynamic(ist* s) {
    static const uint8_t order[19] = {16, 17, 18, 0, 8, 7, 9, 6, 10, 5, 11, 4, 12, 3, 13, 2, 14, 1, 15};
    uint8_t len[320];
    huff lh, dh;
    int nlen = bits(s, 5) + 257, ndist = bits(s, 5) + 1, ncode = bits(s, 4) + 4;
    if (s->err) return s->err;
    if (nlen > 286 || ndist > 30) return -(int)E_ZINV;
    memset(len, 0, sizeof(len));
    for (int k = 0; k < ncode; k++) len[order[k]] = (uint8_t)bits(s, 3);
    if (s->err) return s->err;
    if (build(&lh, len, 19) != 0) return -(int)E_HUFAMB;
    int idx = 0;
    while (idx < nlen + ndist) {
        int sym = decode(s, &lh);
        if (s->err) return s->err;
        if (sym < 16) {
            len[idx++] = (uint8_t)sym;
        } else {
            int v = 0, rep;
            if (sym == 16) {
                if (idx == 0) return -(int)E_ZINV;
                v = len[idx - 1];
                rep = 3 + bits(s, 2);
            } else if (sym == 17) {
                rep = 3 + bits(s, 3);
            } else {
                rep = 11 + bits(s, 7);
            }
            if (s->err) return s->err;
            if (idx + rep > nlen + ndist) return -(int)E_ZINV;
            while (rep--) len[idx++] = (uint8_t)v;
        }
    }
    if (len[256] == 0) return -(int)E_ZINV;
    int e = build(&lh, len, nlen);
    if (e < 0 || (e > 0 && nlen - lh.count[0] != 1)) return -(int)E_HUFAMB;
    e = build(&dh, len + nlen, ndist);
    if (e < 0 || (e > 0 && ndist - dh.count[0] != 1)) return -(int)E_HUFAMB;
    return codes(s, &lh, &dh);
}

static uint32_t adler32(const uint8_t* d, size_t n) {
    uint32_t a = 1, b = 0;
    while (n) {
        size_t k = n < 5552 ? n : 5552;
        n -= k;
        while (k--) { a += *d++; b += a; }
        a %= 65521u;
        b %= 65521u;
    }
    return (b << 16) | a;
}

int deflate_decompress(struct string_len* decompr_dat, struct string_len* compr_dat, int ops) {
    if (!decompr_dat || !compr_dat || (!compr_dat->str && compr_dat->len)) return -E_INVAL;
    ist s;
    memset(&s, 0, sizeof(s));
    s.in = compr_dat->str;
    s.n = compr_dat->len;
    decompr_dat->str = NULL;
    decompr_dat->len = 0;
    if (s.n < 2) return -(int)E_ZHEAD;
    const int cmf = s.in[0], flg = s.in[1];
    if ((cmf & 0x0F) != 8) return -(int)E_ZCMPMT;
    if ((cmf >> 4) > 7) return -(int)E_ZSLWIN;
    if (((cmf << 8) | flg) % 31) return -(int)E_ZFCHCK;
    if (flg & 0x20) return -(int)E_ZPDICT;
    s.pos = 2;
    int last, r = 0;
    do {
        last = bits(&s, 1);
        int type = bits(&s, 2);
        if (s.err) { r = s.err; break; }
        if (type == 0) r = stored(&s);
        else if (type == 1) r = fixed(&s);
        else if (type == 2) r = dynamic(&s);
        else r = -(int)E_ZBTYPE;
        if (r) break;
    } while (!last);
    if (!r) {
        /* drop the partial byte, then the big-endian Adler-32 */
        s.bitbuf >>= s.bitcnt & 7;
        s.bitcnt -= s.bitcnt & 7;
        uint32_t want = 0;
        for (int k = 0; k < 4; k++) want = (want << 8) | (uint32_t)bits(&s, 8);
        if (s.err) r = -(int)E_ZADL32;
        else if (want != adler32(s.out, s.olen)) r = -(int)E_ZADL32;
    }
    if (r) {
        free(s.out);
        return r;
    }
    if (!s.out) {
        s.out = (uint8_t*)malloc(1);
        if (!s.out) return -E_MALLOC;
    }
    if (ops & DEFLATE_NULLTERM) s.out[s.olen] = 0;  /* buffer always has one spare byte */
    decompr_dat->str = s.out;
    decompr_dat->len = s.olen;
    return 0;
}
