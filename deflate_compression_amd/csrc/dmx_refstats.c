/*
 * dmx_refstats.c -- the reference's estimate fields of struct compress_stats, restated for
 * the fd_stats channel of deflate_compress (host C, part of libdmx).
 *
 * In the reference every emitted token updates two adaptive Huffman trees (lit/len and
 * distance, src/aht.c:239-277) and then prices the current code description
 * (src/h_tree.c:75-148 + :242-302); the record of the token carries
 *     tree_bits = h_tree_d_lens(...) + h_tree_builder_score(...)   deflate_compress.c:292-295
 *     ll_bits   = ll_aht.score,  d_bits = d_aht.score               deflate_compress.c:297-298
 * (score = sum over the tree's leaves of weight x depth).  These numbers depend on the exact
 * update order of the reference's tree, so this file performs the same steps:
 *
 *   - an array-backed tree per alphabet: slots 0..n-1 are the symbols' leaves, internal
 *     nodes are handed out from slot n upwards as new symbols arrive (the current NYT,
 *     "not yet transmitted", slot is split into an internal node, the new leaf on its
 *     right and a fresh NYT on its left -- aht.c:243-263);
 *   - a doubly linked order list over the nodes (light to heavy, leaves before internal
 *     nodes of equal weight); a block is a run of equal weight and equal class;
 *   - an update promotes the leaf to its block leader (swap, aht.c:214-219), then walks to
 *     the root: a node slides past the next block when Vitter's invariant requires it
 *     (a leaf of weight w past internal nodes of weight w, an internal node of weight w
 *     past leaves of weight w + 1; aht.c:64-139), then its weight grows by one.  Depth
 *     changes are pushed through the moved subtrees and charged to the score as they
 *     happen (aht.c:42-62), in the reference's order: the scores are running sums of
 *     those charges, not a recount;
 *   - the code-length description: HLIT / HDIST from the trailing zero depths, the RFC
 *     1951 §3.2.7 run-length coding of the concatenated depth sequence with the
 *     reference's rules (zero runs: 18 while >= 11 remain, then ONE 17 for any rest > 1 --
 *     a rest of 2 included, which the RFC does not allow -- else a single 0; other runs:
 *     the value, 16 while >= 3 remain, then singles), 14 + 12 bits plus 3 per further
 *     code-length code down to the last used one in the RFC order (h_tree.c:137-146);
 *   - a two-queue Huffman build over the 19 code-length frequencies sorted by (weight,
 *     symbol) where a leaf is taken only when strictly lighter than the node-queue head
 *     (h_tree.c:242-280), priced as sum of weight x depth (h_tree.c:282-302).
 *
 * Depths of 19 or more (never seen on the golden inputs) would index past the reference's
 * 19-entry frequency array (undefined behaviour there); here they are counted in a wider
 * array and left out of the builder.  The single-used-code-length-symbol case, a TODO in
 * the reference (h_tree.c:257-259), cannot occur: symbol 256 is always present, so a zero
 * run and a non-zero depth are always both coded.
 *
 * Pinned record by record against the reference's own stats streams (tests/golden/
 * ref_stats.npz, written by the reference's own encoder -- tools/make_golden.py; tests/test_refstats.py).
 */
#include <limits.h>
#include <stdint.h>
#include <stdlib.h>
#include <string.h>

#include "../../include/dmx.h"

#define RS_LL 286   /* NUM_LITLEN_CODES, deflate.h:5 */
#define RS_D 30     /* NUM_DIST_CODES, deflate.h:6 */
#define RS_SLOTS (2 * RS_LL + 1)   /* leaves + internal nodes (+1: the last split of a full alphabet) */

typedef struct {
    uint32_t w[RS_SLOTS];     /* weight */
    int16_t dep[RS_SLOTS];    /* depth below the root */
    int16_t up[RS_SLOTS];     /* parent, -1 at the root */
    int16_t c0[RS_SLOTS];     /* left child, -1 for a leaf */
    int16_t c1[RS_SLOTS];     /* right child */
    int16_t nx[RS_SLOTS];     /* next node in the order list (heavier side), -1 at the end */
    int16_t pv[RS_SLOTS];     /* previous node in the order list */
    uint32_t score;           /* sum of weight x depth over the leaves, maintained incrementally */
    int dirty;                /* a leaf's depth changed (or a leaf appeared) since tree_bits was priced */
    int nsym;
    int nyt;                  /* slot of the current NYT leaf */
} rs_tree;

struct dmx_refest {
    rs_tree ll, d;
    uint32_t tree_bits;   /* the last price: unchanged while no leaf depth changes */
};

static void rs_init(rs_tree* t, int nsym) {
    memset(t, 0, sizeof(*t));
    t->nsym = nsym;
    t->nyt = nsym;
    t->up[nsym] = t->c0[nsym] = t->c1[nsym] = t->nx[nsym] = t->pv[nsym] = -1;
}

static inline int rs_leaf(const rs_tree* t, int x) { return t->c0[x] < 0; }

/* last node of x's block: follow the order list while weight and class stay the same */
static int rs_leader(const rs_tree* t, int x) {
    while (t->nx[x] >= 0) {
        const int y = t->nx[x];
        if (t->w[y] != t->w[x] || rs_leaf(t, x) != rs_leaf(t, y)) break;
        x = y;
    }
    return x;
}

/* give the subtree at x the depth d (its children d + 1, ...), charging the leaves' change */
static void rs_redepth(rs_tree* t, int x, int d) {
    for (;;) {
        if (rs_leaf(t, x)) {
            t->score += (uint32_t)(d - t->dep[x]) * t->w[x];
            t->dirty |= t->dep[x] != d;
            t->dep[x] = (int16_t)d;
            return;
        }
        t->dep[x] = (int16_t)d;
        rs_redepth(t, t->c0[x], d + 1);
        x = t->c1[x];
        d += 1;
    }
}

static inline void rs_repoint(rs_tree* t, int par, int from, int to) {
    if (t->c1[par] == from) t->c1[par] = (int16_t)to;
    else t->c0[par] = (int16_t)to;
}

/* Move x to just after b in the order list; every node between them (b included) takes the
 * tree position of the node before it, and x takes b's (aht.c:64-113). */
static void rs_slide(rs_tree* t, int x, int b) {
    const int bpar = t->up[b];
    if (t->pv[x] >= 0) t->nx[t->pv[x]] = t->nx[x];
    t->pv[t->nx[x]] = t->pv[x];
    int par = t->up[x];           /* owner of the slot the next node moves into */
    for (int cur = x; cur != b;) {
        const int m = t->nx[cur];
        rs_repoint(t, par, cur, m);
        if (t->dep[m] != t->dep[par] + 1) rs_redepth(t, m, t->dep[par] + 1);
        const int old = t->up[m];
        t->up[m] = (int16_t)par;
        par = old;
        cur = m;
    }
    rs_repoint(t, bpar, b, x);
    if (t->dep[x] != t->dep[bpar] + 1) rs_redepth(t, x, t->dep[bpar] + 1);
    t->up[x] = (int16_t)bpar;
    if (t->nx[b] >= 0) t->pv[t->nx[b]] = (int16_t)x;
    t->nx[x] = t->nx[b];
    t->pv[x] = (int16_t)b;
    t->nx[b] = (int16_t)x;
}

/* One step of the walk to the root (aht.c:115-139): slide when the invariant needs it, charge
 * a leaf's new unit of weight at its depth, bump the weight.  Returns the next node to
 * update (a leaf: its parent after the slide; an internal node: its parent before it) or -1
 * after the root. */
static int rs_bump(rs_tree* t, int p) {
    const uint32_t wt = t->w[p];
    int next = t->up[p];
    const int lead = rs_leader(t, p);
    if (t->nx[lead] >= 0) {
        const int b = t->nx[lead];
        const int pl = rs_leaf(t, p), bl = rs_leaf(t, b);
        if ((pl && !bl && t->w[b] == wt) || (!pl && bl && t->w[b] == wt + 1)) rs_slide(t, p, rs_leader(t, b));
        if (pl) {
            t->score += (uint32_t)t->dep[p];
            next = t->up[p];
        }
    } else {
        next = -1;
    }
    t->w[p] += 1;
    return next;
}

/* Exchange a with b (b later in the order list, same weight): order list and tree slots
 * (aht.c:141-212). */
static void rs_swap(rs_tree* t, int a, int b) {
    const int adj = t->nx[a] == b;
    const int a_nx = t->nx[a], a_pv = t->pv[a];
    t->nx[a] = t->nx[b];
    if (a_pv >= 0) t->nx[a_pv] = (int16_t)b;
    if (adj) {
        t->nx[b] = (int16_t)a;
    } else {
        t->nx[b] = (int16_t)a_nx;
        t->nx[t->pv[b]] = (int16_t)a;
    }
    t->pv[t->nx[a]] = (int16_t)a;
    t->pv[a] = adj ? (int16_t)b : t->pv[b];
    t->pv[b] = (int16_t)a_pv;
    if (!adj) t->pv[t->nx[b]] = (int16_t)b;
    const int pa = t->up[a], pb = t->up[b];
    if (pa == pb) {
        const int16_t c = t->c0[pa];
        t->c0[pa] = t->c1[pa];
        t->c1[pa] = c;
    } else {
        rs_repoint(t, pa, a, b);
        rs_repoint(t, pb, b, a);
        t->up[a] = (int16_t)pb;
        t->up[b] = (int16_t)pa;
    }
    if (t->dep[a] != t->dep[b]) {
        t->dirty = 1;
        t->score += (uint32_t)(t->dep[a] - t->dep[b]) * (t->w[b] - t->w[a]);
        const int16_t d = t->dep[a];
        t->dep[a] = t->dep[b];
        t->dep[b] = d;
    }
}

static inline int rs_sibling(const rs_tree* t, int x) {
    const int p = t->up[x];
    if (p < 0) return -1;
    return t->c0[p] == x ? t->c1[p] : t->c0[p];
}

/* One occurrence of symbol c (aht.c:239-277). */
static void rs_insert(rs_tree* t, int c) {
    int q, tail = -1;   /* tail: a leaf whose own bump comes after the walk */
    if (t->w[c] == 0) {  /* first occurrence: split the NYT slot */
        q = t->nyt;
        const int z = t->nyt + 1;   /* the new NYT */
        t->c1[q] = (int16_t)c;
        t->pv[q] = (int16_t)c;
        t->dep[c] = (int16_t)(t->dep[q] + 1);
        t->up[c] = (int16_t)q;
        t->c0[c] = t->c1[c] = -1;
        t->nx[c] = (int16_t)q;
        t->pv[c] = (int16_t)z;
        t->c0[q] = (int16_t)z;
        t->w[z] = 0;
        t->dep[z] = (int16_t)(t->dep[q] + 1);
        t->up[z] = (int16_t)q;
        t->c0[z] = t->c1[z] = -1;
        t->nx[z] = (int16_t)c;
        t->pv[z] = -1;
        t->nyt = z;
        t->dirty = 1;
        tail = c;
    } else {
        const int lead = rs_leader(t, c);
        if (lead != c) rs_swap(t, c, lead);
        q = c;
        if (rs_sibling(t, c) == t->nyt) {
            tail = c;
            q = t->up[c];
        }
    }
    while (q >= 0) q = rs_bump(t, q);
    if (tail >= 0) rs_bump(t, tail);
}

/* RFC 1951 §3.2.5 codes (the reference's get_len_code / get_dist_code, deflate_compress.c:182-217,
 * whose code outputs are correct for every length and distance) */
static int rs_len_code(int len) {
    static const uint16_t base[] = {3, 4, 5, 6, 7, 8, 9, 10, 11, 13, 15, 17, 19, 23, 27, 31, 35, 43, 51, 59,
                                    67, 83, 99, 115, 131, 163, 195, 227, 258};
    int k = 28;
    while (base[k] > len) k--;
    return 257 + k;
}
static int rs_dist_code(int dist) {
    const int x = dist - 1;
    if (x < 4) return x;
    int e = 31 - __builtin_clz((unsigned)x);   /* x in [2^e, 2^(e+1)) */
    return 2 * e + ((x >> (e - 1)) & 1);
}

/* tree_bits of one record: the code-length description's cost (h_tree.c:75-148) plus the
 * weighted depth of the code-length code built over its frequencies (h_tree.c:242-302) */
static uint32_t rs_tree_bits(const rs_tree* ll, const rs_tree* d) {
    static const uint8_t order[19] = {16, 17, 18, 0, 8, 7, 9, 6, 10, 5, 11, 4, 12, 3, 13, 2, 14, 1, 15};
    uint32_t f[RS_SLOTS];     /* code-length symbol frequencies (index = depth for 0..) */
    int16_t seq[RS_LL + RS_D];
    memset(f, 0, sizeof(f));
    int hd = RS_D - 1;
    while (hd >= 1 && d->dep[hd] == 0) hd--;
    int hl = RS_LL - 1;
    while (hl >= 257 && ll->dep[hl] == 0) hl--;
    const int nl = hl + 1, L = nl + hd + 1;
    memcpy(seq, ll->dep, sizeof(int16_t) * (size_t)nl);
    memcpy(seq + nl, d->dep, sizeof(int16_t) * (size_t)(hd + 1));
    int bits = 5 + 5 + 4 + 4 * 3;
    for (int i = 0; i < L;) {
        const int v = seq[i];
        int j = i + 1;
        while (j < L && seq[j] == v) j++;
        int run = j - i;
        if (v == 0 && run >= 3) {
            while (run >= 11) {
                run -= run < 138 ? run : 138;
                f[18]++;
                bits += 7;
            }
            if (run > 1) {
                f[17]++;
                bits += 3;
            } else if (run == 1) {
                f[0]++;
            }
        } else {
            f[v]++;
            run--;
            while (run >= 3) {
                run -= run < 6 ? run : 6;
                f[16]++;
                bits += 2;
            }
            f[v] += (uint32_t)run;
        }
        i = j;
    }
    int k = 15;   /* code-length codes sent beyond the first four */
    while (k > 4 && f[order[3 + k]] == 0) k--;
    bits += 3 * k;

    /* the 19 (weight, symbol) pairs in ascending order; weights are u16 in the reference */
    uint32_t key[19];
    int nk = 0;
    for (int s = 0; s < 19; s++) {
        const uint32_t kv = ((f[s] & 0xFFFFu) << 5) | (uint32_t)s;
        int p = nk++;
        while (p > 0 && key[p - 1] > kv) { key[p] = key[p - 1]; p--; }
        key[p] = kv;
    }
    uint32_t lw[19];
    int nlf = 0;
    for (int s = 0; s < 19; s++)
        if (key[s] >> 5) lw[nlf++] = key[s] >> 5;
    /* two queues: leaves lw[h0..), internal nodes iw[h1..t1); a child < 0 is leaf ~idx */
    uint32_t iw[19];
    int ch[19][2];
    int h0 = 0, h1 = 0, t1 = 0;
    const uint32_t EMPTY = 0xFFFFFFFFu;
    for (;;) {
        uint32_t p0 = h0 < nlf ? lw[h0] : EMPTY, p1 = h1 < t1 ? iw[h1] : EMPTY;
        int a, b;
        uint32_t wsum;
        if (p0 < p1) {
            a = ~h0;
            wsum = lw[h0++];
            p0 = h0 < nlf ? lw[h0] : EMPTY;
            if (p0 < p1) {
                b = ~h0;
                wsum += lw[h0++];
            } else if (p1 == EMPTY) {   /* one leaf only: unreachable (see the header) */
                b = a;
                wsum += 0;
            } else {
                b = h1;
                wsum += iw[h1++];
            }
        } else {
            a = h1;
            wsum = iw[h1++];
            p1 = h1 < t1 ? iw[h1] : EMPTY;
            if (p0 < p1) {
                b = ~h0;
                wsum += lw[h0++];
            } else {
                if (p1 == EMPTY) break;
                b = h1;
                wsum += iw[h1++];
            }
        }
        ch[t1][0] = a;
        ch[t1][1] = b;
        iw[t1++] = wsum;
    }
    uint32_t score = 0;
    if (t1 > 0) {
        int dep[19];
        dep[t1 - 1] = 1;   /* the root's children sit at depth 1 */
        for (int x = t1 - 1; x >= 0; x--)
            for (int s = 0; s < 2; s++) {
                const int c = ch[x][s];
                if (c < 0) score += lw[~c] * (uint32_t)dep[x];
                else dep[c] = dep[x] + 1;
            }
    }
    return (uint32_t)bits + score;
}

dmx_refest* dmx_refest_create(void) {
    dmx_refest* e = (dmx_refest*)malloc(sizeof(dmx_refest));
    if (!e) return NULL;
    rs_init(&e->ll, RS_LL);
    rs_init(&e->d, RS_D);
    rs_insert(&e->ll, 256);   /* the end-of-block code, counted once up front (deflate_compress.c:234) */
    e->tree_bits = 0;
    e->ll.dirty = 1;
    return e;
}

void dmx_refest_destroy(dmx_refest* e) { free(e); }

int dmx_refest_feed(dmx_refest* e, const uint32_t* tok, uint32_t ntok, struct compress_stats* rec,
                    uint32_t* nfilled) {
    if (nfilled) *nfilled = 0;
    if (!e || (ntok && (!tok || !rec))) return -E_INVAL;
    for (uint32_t k = 0; k < ntok; k++) {
        const uint32_t t = tok[k];
        if ((t >> 9) == 0) {
            rs_insert(&e->ll, (int)(t & 0xFF));
        } else {
            const int len = (int)(t & 0x1FF), dist = (int)(t >> 9);
            if (len < 3 || len > 258 || dist < 1 || dist > 32768) return -E_RANGE;
            rs_insert(&e->ll, rs_len_code(len));
            rs_insert(&e->d, rs_dist_code(dist));
        }
        if (e->ll.dirty || e->d.dirty) {   /* the price depends on the leaves' depths only */
            e->tree_bits = rs_tree_bits(&e->ll, &e->d);
            e->ll.dirty = e->d.dirty = 0;
        }
        const uint32_t tb = e->tree_bits;
        if (tb > INT_MAX || e->ll.score > INT_MAX || e->d.score > INT_MAX) return -E_RANGE;
        rec[k].tree_bits = (int)tb;
        rec[k].ll_bits = (int)e->ll.score;
        rec[k].d_bits = (int)e->d.score;
        if (nfilled) *nfilled = k + 1;
    }
    return 0;
}
