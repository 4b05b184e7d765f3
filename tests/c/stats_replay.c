/*
 * stats_replay.c -- a C caller of the drop-in boundary, built the way a user of the
 * reference would build theirs: #include "dmx.h" (for the reference's deflate_ext.h) and link
 * -ldmx.  It automates the contract of the reference's own harness, tests/check_lld.c
 * (:20-39 replays each compress_stats record into the output, :56-79 runs the encoder on a
 * file and reads the records back), which only printed and does not compile:
 *
 *   stats_replay IN [SW]
 *     deflate_compress(fd_in, fd_out, fd_stats, SW, 0)   -> 0
 *     replay every record (d == 0: literal ll; else copy ll bytes from d back) block by block
 *     (every SW bytes the window restarts) and compare with IN;
 *     records: bytes == 1 + token start, running sums never decrease;
 *     deflate_decompress(the stream) == IN.
 *   Exit status 0 = all checks passed; the first failure is printed.
 */
#include <fcntl.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>
#include <unistd.h>

#include "dmx.h"

static unsigned char* slurp(const char* path, size_t* n) {
    FILE* f = fopen(path, "rb");
    if (!f) return NULL;
    fseek(f, 0, SEEK_END);
    long sz = ftell(f);
    fseek(f, 0, SEEK_SET);
    unsigned char* b = (unsigned char*)malloc(sz > 0 ? (size_t)sz : 1);
    *n = b && sz > 0 ? fread(b, 1, (size_t)sz, f) : 0;
    fclose(f);
    return b;
}

#define FAIL(...) do { fprintf(stderr, "stats_replay: " __VA_ARGS__); fputc('\n', stderr); return 1; } while (0)

int main(int argc, char** argv) {
    if (argc < 2) FAIL("usage: stats_replay IN [SW]");
    const int sw = argc > 2 ? atoi(argv[2]) : 32768;
    size_t n = 0;
    unsigned char* in = slurp(argv[1], &n);
    if (!in) FAIL("cannot read %s", argv[1]);
    char zpath[] = "/tmp/stats_replay_zXXXXXX", spath[] = "/tmp/stats_replay_sXXXXXX";
    const int fo = mkstemp(zpath), fs = mkstemp(spath);
    const int fi = open(argv[1], O_RDONLY);
    if (fo < 0 || fs < 0 || fi < 0) FAIL("cannot open files");
    const int rc = deflate_compress(fi, fo, fs, (swi)sw, 0);
    close(fi);
    close(fo);
    close(fs);
    if (rc != 0) FAIL("deflate_compress returned %d", rc);
    size_t zn = 0, sn = 0;
    unsigned char* z = slurp(zpath, &zn);
    unsigned char* st = slurp(spath, &sn);
    unlink(zpath);
    unlink(spath);
    if (!z || sn % sizeof(struct compress_stats)) FAIL("bad outputs (%zu stats bytes)", sn);
    const struct compress_stats* cs = (const struct compress_stats*)st;
    const size_t nrec = sn / sizeof(struct compress_stats);
    unsigned char* out = (unsigned char*)malloc(n + 1);
    size_t o = 0;
    long long prev_tree = 0, prev_ll = 0, prev_d = 0;
    /* DMX_STATS=exact: all three fields are running sums.  Default (the reference's
     * estimates): ll_bits / d_bits are adaptive-tree scores, which only grow; tree_bits is
     * the cost of describing the current codes, which may shrink. */
    const char* mode = getenv("DMX_STATS");
    const int exact = mode && strcmp(mode, "exact") == 0;
    for (size_t k = 0; k < nrec; k++) {   /* check_lld.c:20-39: rebuild the input token by token */
        if (cs[k].bytes != (int)o + 1) FAIL("record %zu: bytes %d, token starts at %zu", k, cs[k].bytes, o);
        if ((exact && cs[k].tree_bits < prev_tree) || cs[k].tree_bits < 0 || cs[k].ll_bits < prev_ll ||
            cs[k].d_bits < prev_d)
            FAIL("record %zu: running sums decrease", k);
        prev_tree = cs[k].tree_bits;
        prev_ll = cs[k].ll_bits;
        prev_d = cs[k].d_bits;
        if (cs[k].d == 0) {
            if (o >= n) FAIL("record %zu: past the input", k);
            out[o++] = (unsigned char)cs[k].ll;
        } else {
            const size_t blk0 = o - o % (size_t)sw;   /* a block's matches stay inside it */
            if (cs[k].ll < 3 || cs[k].ll > 258 || (size_t)cs[k].d > o - blk0 || o + (size_t)cs[k].ll > n)
                FAIL("record %zu: bad match (%d, %d) at %zu", k, cs[k].ll, cs[k].d, o);
            for (int j = 0; j < cs[k].ll; j++, o++) out[o] = out[o - (size_t)cs[k].d];
        }
    }
    if (o != n || memcmp(out, in, n) != 0) FAIL("replay differs from the input (%zu of %zu bytes)", o, n);
    struct string_len zin = {z, zn}, zout = {NULL, 0};
    const int dr = deflate_decompress(&zout, &zin, 0);
    if (dr != 0) FAIL("deflate_decompress returned %d", dr);
    if (zout.len != n || memcmp(zout.str, in, n) != 0) FAIL("inflated stream differs from the input");
    printf("stats_replay ok: %zu bytes, %zu records, %zu stream bytes, rate %.4f bits/byte\n", n, nrec, zn,
           nrec ? (double)(prev_tree + prev_ll + prev_d) / (double)n : 0.0);
    free(zout.str);
    free(out);
    free(in);
    free(z);
    free(st);
    return 0;
}
