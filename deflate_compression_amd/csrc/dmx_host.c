/*
 * dmx_host.c -- host C side of libdmx: the reference's public codec API
 * (src/include/deflate_ext.h) on top of the HIP layer (dmx_kernels.hip).
 *
 *   deflate_compress(fd_in, fd_out, fd_stats, sw, ops)   deflate_compress.c:362-376
 *   spawn_deflate_compr_t / deflate_compr_init / _deinit  deflate_compress.c:83-112
 *   struct compress_stats stream                         deflate_compress.c:290-309
 *
 * Errors are returned as -E_* (global_errors.h / deflate_errors.h codes); nothing
 * longjmps.  There is no CPU encode path: the encode runs on the GPU or fails.
 */
#include <errno.h>
#include <limits.h>
#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>
#include <unistd.h>

#include "../../include/dmx.h"
#include "dmx_internal.h"

/* from dmx_kernels.hip */
dmx_ctx* dmx_cached_ctx(int device, uint64_t max_input, int* err);
void dmx_cached_lock(void);
void dmx_cached_unlock(void);

struct deflate_compr {
    int fd_in, fd_out, fd_stats;
    swi sw;
};

deflate_compr_t* spawn_deflate_compr_t(void) { return (deflate_compr_t*)calloc(1, sizeof(deflate_compr_t)); }

void deflate_compr_init(deflate_compr_t* com, int fd_in, int fd_out, int fd_stats, swi sw) {
    if (!com) return;
    com->fd_in = fd_in;
    com->fd_out = fd_out;
    com->fd_stats = fd_stats;
    com->sw = sw;
}

void deflate_compr_deinit(deflate_compr_t* com) {
    if (com) memset(com, 0, sizeof(*com));
}

static int read_all(int fd, uint8_t** buf, uint64_t* n) {
    uint64_t cap = 1 << 20, len = 0;
    uint8_t* b = (uint8_t*)malloc(cap);
    if (!b) return -E_MALLOC;
    for (;;) {
        if (len == cap) {
            uint8_t* nb = (uint8_t*)realloc(b, cap * 2);
            if (!nb) { free(b); return -E_MALLOC; }
            b = nb;
            cap *= 2;
        }
        ssize_t r = read(fd, b + len, cap - len);
        if (r < 0) {
            if (errno == EINTR) continue;
            free(b);
            return -E_NEXIST;
        }
        if (r == 0) break;
        len += (uint64_t)r;
    }
    *buf = b;
    *n = len;
    return 0;
}

static int write_all(int fd, const void* p, uint64_t n) {
    const uint8_t* c = (const uint8_t*)p;
    while (n) {
        ssize_t w = write(fd, c, n);
        if (w < 0) {
            if (errno == EINTR) continue;
            return -E_PIPE;
        }
        c += w;
        n -= (uint64_t)w;
    }
    return 0;
}

/* RFC 1951 §3.2.5 symbol + extra bits (host copy, used only to format stats) */
static void h_len_sym(int len, int* sym, int* eb) {
    static const int base[] = {11, 13, 15, 17, 19, 23, 27, 31, 35, 43, 51, 59, 67, 83, 99, 115, 131, 163, 195, 227};
    if (len == 258) { *sym = 285; *eb = 0; return; }
    if (len <= 10) { *sym = 254 + len; *eb = 0; return; }
    int k = 19;
    while (base[k] > len) k--;
    *sym = 265 + k;
    *eb = 1 + k / 4;
}
static void h_dist_sym(int dist, int* sym, int* eb) {
    int x = dist - 1, e = 0;
    if (x < 4) { *sym = x; *eb = 0; return; }
    while ((x >> (e + 1)) != 0) e++;
    *sym = 2 * e + ((x >> (e - 1)) & 1);
    *eb = e - 1;
}

/* One compress_stats record per token (deflate_compress.c:290-309): bytes = 1 + the token's
 * input offset, ll / d = the token.  The *_bits fields (DMX_STATS, include/dmx.h):
 *   "ref" (default): the reference's estimates -- its adaptive-Huffman scores ll_aht.score /
 *       d_aht.score (:297-298, aht.c:239-277) and the cost of describing the current codes
 *       (h_tree_d_lens + the code-length tree, :292-295), restated in dmx_refstats.c and
 *       running over the whole stream as the reference's trees do;
 *   "exact": this stream's exact costs, over the whole stream --
 *       tree_bits = header bits of every DEFLATE block begun so far (its own included:
 *                   BFINAL / BTYPE, and for dynamic blocks the code-length and code
 *                   descriptions; with DMX_F_SPLIT an sw block holds up to four),
 *       ll_bits   = lit/len code bits + length extra bits of every token so far (stored
 *                   blocks: 8 per byte),
 *       d_bits    = distance code bits + distance extra bits of every match so far.
 * The fields are int (deflate_ext.h:19-31).  A record whose bytes or *_bits would exceed
 * INT_MAX is never written: the records before it are, and the call returns -E_RANGE. */
static int write_stats(dmx_ctx* c, int fd, uint64_t n, int sw) {
    const uint32_t nblk = (uint32_t)((n + (uint64_t)sw - 1) / (uint64_t)sw);
    if (!nblk) return 0;
    const char* mode = getenv("DMX_STATS");
    const int exact = mode && strcmp(mode, "exact") == 0;
    if (mode && *mode && !exact && strcmp(mode, "ref") != 0) return -E_INVAL;
    uint32_t* tok = (uint32_t*)malloc(sizeof(uint32_t) * DMX_BLK);
    struct compress_stats* rec = (struct compress_stats*)malloc(sizeof(struct compress_stats) * DMX_BLK);
    dmx_refest* est = exact ? NULL : dmx_refest_create();
    int r = 0;
    long long tree_bits = 0, ll_bits = 0, d_bits = 0;   /* exact: over the whole stream */
    if (!tok || !rec || (!exact && !est)) r = -E_MALLOC;
    for (uint32_t b = 0; !r && b < nblk; b++) {
        int nt = dmx_last_tokens(c, b, tok, DMX_BLK);
        if (nt < 0) { r = nt; break; }
        uint32_t lim = (uint32_t)nt;   /* records of this block that fit the int fields */
        uint64_t pos = (uint64_t)b * (uint64_t)sw;
        for (uint32_t k = 0; k < (uint32_t)nt; k++) {
            const uint32_t t = tok[k];
            if (pos + 1 > (uint64_t)INT_MAX) { lim = k; break; }
            rec[k].bytes = (int)(pos + 1);
            if ((t >> 9) == 0) {
                rec[k].ll = (int)(t & 0xFF);
                rec[k].d = 0;
                pos += 1;
            } else {
                rec[k].ll = (int)(t & 0x1FF);
                rec[k].d = (int)(t >> 9);
                pos += t & 0x1FF;
            }
        }
        if (!exact) {
            uint32_t nf = 0;
            const int e = dmx_refest_feed(est, tok, lim, rec, &nf);
            if (e && e != -E_RANGE) { r = e; break; }
            lim = nf;
        } else {
            int nsub = 1;
            for (int sb = 0; !r && sb < nsub; sb++) {
                uint8_t lens[316];
                uint32_t range[2], bt = 0, hb = 0;
                nsub = dmx_last_subblock(c, b, (uint32_t)sb, range, &bt, &hb, lens);
                if (nsub < 0) { r = nsub; break; }
                tree_bits += bt == 2 ? (long long)hb : 3;
                for (uint32_t k = range[0]; k < range[1] && k < lim; k++) {
                    const uint32_t t = tok[k];
                    if ((t >> 9) == 0) {
                        ll_bits += bt == 0 ? 8 : (long long)lens[t & 0xFF];
                    } else {
                        const int len = (int)(t & 0x1FF), dist = (int)(t >> 9);
                        int sy, eb;
                        if (bt == 0) {          /* stored block: the bytes themselves */
                            ll_bits += 8 * len;
                        } else {
                            h_len_sym(len, &sy, &eb);
                            ll_bits += lens[sy] + eb;
                            h_dist_sym(dist, &sy, &eb);
                            d_bits += lens[DMX_DIST0 + sy] + eb;
                        }
                    }
                    if (tree_bits > INT_MAX || ll_bits > INT_MAX || d_bits > INT_MAX) { lim = k; break; }
                    rec[k].tree_bits = (int)tree_bits;
                    rec[k].ll_bits = (int)ll_bits;
                    rec[k].d_bits = (int)d_bits;
                }
            }
            if (r) break;
        }
        r = write_all(fd, rec, sizeof(struct compress_stats) * (uint64_t)lim);
        if (!r && lim < (uint32_t)nt) r = -E_RANGE;
    }
    free(tok); free(rec);
    dmx_refest_destroy(est);
    return r;
}

int deflate_compress(int fd_in, int fd_out, int fd_stats, swi sw, int ops) {
    (void)ops; /* unused by the reference's compress too */
    int swv = sw == 0 ? DMX_BLK : (int)sw;
    if (swv > DMX_BLK) return -E_RANGE;
    if (fd_stats >= 0) {   /* an unknown DMX_STATS mode fails before anything is encoded or written */
        const char* mode = getenv("DMX_STATS");
        if (mode && *mode && strcmp(mode, "exact") != 0 && strcmp(mode, "ref") != 0) return -E_INVAL;
    }
    const char* mc = getenv("DMX_MAX_CHAIN");
    dmx_opts o;
    o.sw = swv;
    o.max_chain = mc ? atoi(mc) : 0;
    o.flags = DMX_ZLIB;
    const char* lz = getenv("DMX_LAZY");   /* 1 = lazy evaluation (DMX_F_LAZY); default greedy */
    if (lz && atoi(lz) > 0) o.flags |= DMX_F_LAZY;
    const char* sp = getenv("DMX_SPLIT");  /* 1 = adaptive block splitting (DMX_F_SPLIT) */
    if (sp && atoi(sp) > 0) o.flags |= DMX_F_SPLIT;
    const char* dc = getenv("DMX_DICT");   /* 1 = cross-block dictionary (DMX_F_DICT) */
    if (dc && atoi(dc) > 0) o.flags |= DMX_F_DICT;
    const char* sc = getenv("DMX_STORE_CHECK");   /* 1 = noise blocks stored unparsed (§4.7);
                                                   * not with fd_stats: such blocks have no tokens */
    if (sc && atoi(sc) > 0 && fd_stats < 0) o.flags |= DMX_F_STORE_CHECK;
    const char* dp = getenv("DMX_DEEP");   /* 1 = adaptive chain depth (DMX_F_DEEP, bounded mode) */
    if (dp && atoi(dp) > 0) o.flags |= DMX_F_DEEP;
    o.reserved = 0;
    o.dict = NULL;
    o.dict_len = 0;
    if (fd_stats < 0) {   /* streaming: chunks of DMX_CHUNK_MB MiB (default 16) through pinned buffers */
        const char* cm = getenv("DMX_CHUNK_MB");
        const uint64_t mb = cm && atoi(cm) > 0 ? (uint64_t)atoi(cm) : 16u;
        int devs[64];
        const int nd = dmx_devices_from_env(devs, 64);   /* DMX_DEVICES: one host thread per GPU */
        if (nd < 0) return nd;
        if (nd > 0) return dmx_encode_fd_multi(fd_in, fd_out, &o, mb << 20, devs, nd);
        return dmx_encode_fd(fd_in, fd_out, &o, mb << 20);
    }
    uint8_t* in = NULL;
    uint64_t n = 0;
    int r = read_all(fd_in, &in, &n);
    if (r) return r;
    uint64_t cap = dmx_max_compressed(n, swv);
    uint8_t* out = (uint8_t*)malloc(cap);
    if (!out) { free(in); return -E_MALLOC; }
    uint64_t out_len = 0;
    dmx_cached_lock();   /* the stats read this encode's tokens back from the cached context */
    r = dmx_encode_host(in, n, out, cap, &out_len, &o);
    if (!r && fd_out >= 0) r = write_all(fd_out, out, out_len);
    if (!r && fd_stats >= 0) {
        const char* dev_s = getenv("DMX_DEVICE");
        int err = 0;
        dmx_ctx* c = dmx_cached_ctx(dev_s ? atoi(dev_s) : 0, n, &err);
        r = c ? write_stats(c, fd_stats, n, swv) : err;
    }
    dmx_cached_unlock();
    free(in);
    free(out);
    return r;
}

/* Adler-32 of A||B from adler(A), adler(B) and len(B) (RFC 1950 §8.2 arithmetic). */
uint32_t dmx_adler32_combine(uint32_t a, uint32_t b, uint64_t len_b) {
    const uint64_t M = 65521;
    const uint64_t rem = len_b % M;
    uint64_t s1 = a & 0xFFFF, s2 = (rem * s1) % M;
    s1 = (s1 + (b & 0xFFFF) + M - 1) % M;
    s2 = (s2 + ((a >> 16) & 0xFFFF) + ((b >> 16) & 0xFFFF) + M - rem) % M;
    return (uint32_t)(s1 | (s2 << 16));
}
