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
int dmx_encode_fd_cb(int fd_in, int fd_out, const dmx_opts* opts, uint64_t chunk,
                     int (*cb)(void* user, dmx_ctx* c, uint64_t chunk_bytes, uint64_t chunk_off), void* user);

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
 * INT_MAX is never written: the records before it are, and the call returns -E_RANGE.
 * The records are written chunk by chunk as the stream is encoded (dmx_encode_fd_cb): the
 * state (the estimator's trees, the exact running sums) carries over the chunks. */
typedef struct {
    int fd, exact, sw, range;   /* range: a record did not fit; none after it */
    dmx_refest* est;
    uint32_t* tok;
    struct compress_stats* rec;
    long long tree_bits, ll_bits, d_bits;
} stats_writer;

static int stats_chunk(void* user, dmx_ctx* c, uint64_t n, uint64_t base) {
    stats_writer* W = (stats_writer*)user;
    const int sw = W->sw;
    const uint32_t nblk = (uint32_t)((n + (uint64_t)sw - 1) / (uint64_t)sw);
    uint32_t* tok = W->tok;
    struct compress_stats* rec = W->rec;
    for (uint32_t b = 0; !W->range && b < nblk; b++) {
        int nt = dmx_last_tokens(c, b, tok, DMX_BLK);
        if (nt < 0) return nt;
        uint32_t lim = (uint32_t)nt;   /* records of this block that fit the int fields */
        uint64_t pos = base + (uint64_t)b * (uint64_t)sw;
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
        if (!W->exact) {
            uint32_t nf = 0;
            const int e = dmx_refest_feed(W->est, tok, lim, rec, &nf);
            if (e && e != -E_RANGE) return e;
            lim = nf;
        } else {
            int nsub = 1;
            for (int sb = 0; sb < nsub; sb++) {
                uint8_t lens[316];
                uint32_t range[2], bt = 0, hb = 0;
                nsub = dmx_last_subblock(c, b, (uint32_t)sb, range, &bt, &hb, lens);
                if (nsub < 0) return nsub;
                W->tree_bits += bt == 2 ? (long long)hb : 3;
                for (uint32_t k = range[0]; k < range[1] && k < lim; k++) {
                    const uint32_t t = tok[k];
                    if ((t >> 9) == 0) {
                        W->ll_bits += bt == 0 ? 8 : (long long)lens[t & 0xFF];
                    } else {
                        const int len = (int)(t & 0x1FF), dist = (int)(t >> 9);
                        int sy, eb;
                        if (bt == 0) {          /* stored block: the bytes themselves */
                            W->ll_bits += 8 * len;
                        } else {
                            h_len_sym(len, &sy, &eb);
                            W->ll_bits += lens[sy] + eb;
                            h_dist_sym(dist, &sy, &eb);
                            W->d_bits += lens[DMX_DIST0 + sy] + eb;
                        }
                    }
                    if (W->tree_bits > INT_MAX || W->ll_bits > INT_MAX || W->d_bits > INT_MAX) { lim = k; break; }
                    rec[k].tree_bits = (int)W->tree_bits;
                    rec[k].ll_bits = (int)W->ll_bits;
                    rec[k].d_bits = (int)W->d_bits;
                }
            }
        }
        const int e = write_all(W->fd, rec, sizeof(struct compress_stats) * (uint64_t)lim);
        if (e) return e;
        if (lim < (uint32_t)nt) W->range = 1;   /* the stream goes on; no more records */
    }
    return 0;
}

int deflate_compress(int fd_in, int fd_out, int fd_stats, swi sw, int ops) {
    (void)ops; /* unused by the reference's compress too */
    int swv = sw == 0 ? DMX_BLK : (int)sw;
    if (swv > DMX_BLK) return -E_RANGE;
    int exact = 0;
    if (fd_stats >= 0) {   /* an unknown DMX_STATS mode fails before anything is encoded or written */
        const char* mode = getenv("DMX_STATS");
        if (mode && *mode && strcmp(mode, "exact") != 0 && strcmp(mode, "ref") != 0) return -E_INVAL;
        exact = mode && strcmp(mode, "exact") == 0;
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
    const char* dd = getenv("DMX_DEEP_CHAIN");   /* DMX_F_DEEP depth (0 / unset = DMX_DEEP_CHAIN, 32) */
    o.deep_chain = dd ? atoi(dd) : 0;
    o.dict = NULL;
    o.dict_len = 0;
    /* streaming: chunks of DMX_CHUNK_MB MiB (default 16) through pinned buffers; each chunk a
     * shard of one zlib stream (DESIGN.md §6 framing), so any input size streams */
    const char* cm = getenv("DMX_CHUNK_MB");
    const uint64_t mb = cm && atoi(cm) > 0 ? (uint64_t)atoi(cm) : 16u;
    if (fd_stats < 0) {
        int devs[64];
        const int nd = dmx_devices_from_env(devs, 64);   /* DMX_DEVICES: one host thread per GPU */
        if (nd < 0) return nd;
        if (nd > 0) return dmx_encode_fd_multi(fd_in, fd_out, &o, mb << 20, devs, nd);
        return dmx_encode_fd(fd_in, fd_out, &o, mb << 20);
    }
    /* with the records: each chunk's tokens become records before the next chunk encodes */
    stats_writer W;
    memset(&W, 0, sizeof(W));
    W.fd = fd_stats;
    W.exact = exact;
    W.sw = swv;
    W.tok = (uint32_t*)malloc(sizeof(uint32_t) * DMX_BLK);
    W.rec = (struct compress_stats*)malloc(sizeof(struct compress_stats) * DMX_BLK);
    W.est = exact ? NULL : dmx_refest_create();
    int r = (!W.tok || !W.rec || (!exact && !W.est)) ? -E_MALLOC : 0;
    if (!r) r = dmx_encode_fd_cb(fd_in, fd_out, &o, mb << 20, stats_chunk, &W);
    if (!r && W.range) r = -E_RANGE;
    free(W.tok);
    free(W.rec);
    dmx_refest_destroy(W.est);
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
