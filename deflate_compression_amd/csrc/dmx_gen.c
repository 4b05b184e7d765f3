/*
 * dmx_gen.c -- seeded synthetic inputs for the bench and tests.
 * enwik8/enwik9 are not available offline, so C3/C5 use an enwik-style generator:
 * MediaWiki XML pages (<page>/<title>/<id>/<revision>/<text>) whose article text is
 * drawn from a Zipf-distributed vocabulary of pseudo-words, with wiki markup
 * ([[links]], '''bold''', ==headings==, {{templates}}, dates, numbers, lists).
 * C4 uses splitmix64 bytes (seed 0x5EED) in place of /dev/urandom.
 * Deterministic for a given (n, seed); independent of thread count.
 */
#include <math.h>
#include <stdint.h>
#include <stdlib.h>
#include <string.h>

#include "../../include/dmx.h"

static inline uint64_t splitmix64(uint64_t* x) {
    uint64_t z = (*x += 0x9E3779B97F4A7C15ull);
    z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ull;
    z = (z ^ (z >> 27)) * 0x94D049BB133111EBull;
    return z ^ (z >> 31);
}

void dmx_gen_random(uint8_t* buf, uint64_t n, uint64_t seed) {
    uint64_t x = seed;
    uint64_t i = 0;
    for (; i + 8 <= n; i += 8) {
        uint64_t v = splitmix64(&x);
        memcpy(buf + i, &v, 8);
    }
    if (i < n) {
        uint64_t v = splitmix64(&x);
        memcpy(buf + i, &v, n - i);
    }
}

#define NWORDS 24000
#define MAXW 16

typedef struct {
    uint64_t rng;
    char words[NWORDS][MAXW];
    uint8_t wlen[NWORDS];
    double* cdf;
    uint8_t* out;
    uint64_t n, pos;
} gen;

static inline double urand(gen* g) { return (double)(splitmix64(&g->rng) >> 11) * (1.0 / 9007199254740992.0); }
static inline uint32_t irand(gen* g, uint32_t m) { return (uint32_t)((splitmix64(&g->rng) >> 33) % m); }

static void emit(gen* g, const char* s, size_t k) {
    if (g->pos >= g->n) return;
    if (k > g->n - g->pos) k = (size_t)(g->n - g->pos);
    memcpy(g->out + g->pos, s, k);
    g->pos += k;
}
static void emits(gen* g, const char* s) { emit(g, s, strlen(s)); }

static uint32_t zipf_word(gen* g) {
    double u = urand(g);
    uint32_t lo = 0, hi = NWORDS - 1;
    while (lo < hi) {
        uint32_t mid = (lo + hi) >> 1;
        if (g->cdf[mid] < u) lo = mid + 1; else hi = mid;
    }
    return lo;
}

static void emit_word(gen* g, uint32_t w, int cap) {
    char tmp[MAXW];
    memcpy(tmp, g->words[w], g->wlen[w]);
    if (cap && tmp[0] >= 'a' && tmp[0] <= 'z') tmp[0] = (char)(tmp[0] - 32);
    emit(g, tmp, g->wlen[w]);
}

static void emit_num(gen* g, uint32_t v) {
    char t[16];
    int k = 0;
    do { t[15 - k++] = (char)('0' + v % 10); v /= 10; } while (v);
    emit(g, t + 16 - k, (size_t)k);
}

static void sentence(gen* g) {
    int nw = 6 + (int)irand(g, 20);
    for (int k = 0; k < nw && g->pos < g->n; k++) {
        if (k) emits(g, " ");
        double r = urand(g);
        uint32_t w = zipf_word(g);
        if (r < 0.045) {
            emits(g, "[[");
            emit_word(g, w, 1);
            if (urand(g) < 0.3) { emits(g, " "); emit_word(g, zipf_word(g), 0); }
            if (urand(g) < 0.2) { emits(g, "|"); emit_word(g, zipf_word(g), 0); }
            emits(g, "]]");
        } else if (r < 0.055) {
            emits(g, "'''");
            emit_word(g, w, 1);
            emits(g, "'''");
        } else if (r < 0.075) {
            emit_num(g, irand(g, 3000));
        } else {
            emit_word(g, w, k == 0);
        }
        if (k + 1 < nw && urand(g) < 0.06) emits(g, ",");
    }
    emits(g, urand(g) < 0.9 ? ". " : "; ");
}

static void page(gen* g, uint32_t id) {
    emits(g, "  <page>\n    <title>");
    emit_word(g, zipf_word(g) % 4000, 1);
    if (urand(g) < 0.5) { emits(g, " "); emit_word(g, zipf_word(g), 1); }
    emits(g, "</title>\n    <id>");
    emit_num(g, id);
    emits(g, "</id>\n    <revision>\n      <id>");
    emit_num(g, 15898900 + irand(g, 900000));
    emits(g, "</id>\n      <timestamp>200");
    emit_num(g, 2 + irand(g, 5));
    emits(g, "-0");
    emit_num(g, 1 + irand(g, 9));
    emits(g, "-1");
    emit_num(g, irand(g, 10));
    emits(g, "T0");
    emit_num(g, irand(g, 10));
    emits(g, ":2");
    emit_num(g, irand(g, 10));
    emits(g, ":4");
    emit_num(g, irand(g, 10));
    emits(g, "Z</timestamp>\n      <contributor>\n        <username>");
    emit_word(g, zipf_word(g) % 3000, 1);
    emits(g, "</username>\n        <id>");
    emit_num(g, irand(g, 400000));
    emits(g, "</id>\n      </contributor>\n      <text xml:space=\"preserve\">");
    if (urand(g) < 0.3) {
        emits(g, "{{Infobox ");
        emit_word(g, zipf_word(g) % 500, 0);
        emits(g, "\n| name = ");
        emit_word(g, zipf_word(g), 1);
        emits(g, "\n| image = ");
        emit_word(g, zipf_word(g), 0);
        emits(g, ".jpg\n}}\n");
    }
    int npar = 2 + (int)irand(g, 9);
    for (int p = 0; p < npar && g->pos < g->n; p++) {
        if (p && urand(g) < 0.35) {
            emits(g, "\n== ");
            emit_word(g, zipf_word(g) % 2000, 1);
            emits(g, " ==\n");
        }
        if (urand(g) < 0.15) {
            int ni = 2 + (int)irand(g, 6);
            for (int k = 0; k < ni; k++) {
                emits(g, "* [[");
                emit_word(g, zipf_word(g), 1);
                emits(g, "]]\n");
            }
        }
        int ns = 2 + (int)irand(g, 7);
        for (int s = 0; s < ns; s++) sentence(g);
        emits(g, "\n\n");
    }
    emits(g, "[[Category:");
    emit_word(g, zipf_word(g) % 1000, 1);
    emits(g, "]]</text>\n    </revision>\n  </page>\n");
}

void dmx_gen_text(uint8_t* buf, uint64_t n, uint64_t seed) {
    static const char* syl[] = {"a", "e", "i", "o", "u", "an", "en", "in", "on", "ar", "er", "or", "al", "el",
                                "th", "st", "re", "ti", "ca", "co", "de", "di", "ma", "mi", "na", "ne", "ra",
                                "ro", "sa", "se", "ta", "te", "to", "la", "le", "li", "lo", "pa", "pe", "po",
                                "ve", "ri", "ni", "mo", "ba", "be", "ge", "ha", "he", "ho", "ki", "ly", "ch",
                                "sh", "ph", "tion", "ing", "ed", "es", "ous", "ment", "ic", "ist", "ia", "us"};
    const int nsyl = (int)(sizeof(syl) / sizeof(syl[0]));
    gen* g = (gen*)calloc(1, sizeof(gen));
    if (!g) return;
    g->rng = seed ^ 0xD1B54A32D192ED03ull;
    g->out = buf;
    g->n = n;
    static const char* common[] = {"the", "of", "and", "in", "to", "a", "is", "was", "for", "as", "by",
                                   "with", "on", "that", "from", "his", "at", "he", "it", "an", "are",
                                   "which", "were", "or", "be", "first", "also", "this", "its", "has"};
    const int ncommon = (int)(sizeof(common) / sizeof(common[0]));
    for (int w = 0; w < NWORDS; w++) {
        char t[MAXW];
        int k = 0;
        if (w < ncommon) {
            k = (int)strlen(common[w]);
            memcpy(t, common[w], (size_t)k);
        } else {
            int ns = 1 + (int)irand(g, 3) + (w > 2000) + (w > 8000);
            for (int s = 0; s < ns; s++) {
                const char* y = syl[irand(g, (uint32_t)nsyl)];
                int yl = (int)strlen(y);
                if (k + yl >= MAXW) break;
                memcpy(t + k, y, (size_t)yl);
                k += yl;
            }
        }
        memcpy(g->words[w], t, (size_t)k);
        g->wlen[w] = (uint8_t)k;
    }
    g->cdf = (double*)malloc(sizeof(double) * NWORDS);
    double z = 0;
    for (int w = 0; w < NWORDS; w++) z += 1.0 / pow((double)(w + 1), 1.05);
    double acc = 0;
    for (int w = 0; w < NWORDS; w++) {
        acc += 1.0 / pow((double)(w + 1), 1.05) / z;
        g->cdf[w] = acc;
    }
    g->cdf[NWORDS - 1] = 1.0;
    emits(g, "<mediawiki xmlns=\"http://www.mediawiki.org/xml/export-0.3/\" version=\"0.3\" xml:lang=\"en\">\n");
    uint32_t id = 1;
    while (g->pos < g->n) page(g, id++);
    free(g->cdf);
    free(g);
}
