// dmx_kernels.hip -- the MI355X (gfx950 / CDNA4) hot path of the DEFLATE encoder.
//
// The input is cut into independent sw-byte blocks (sw <= 32768 = the window).
// Per encode, four launches on one HIP stream:
//   K1  dmx_match_kernel  one 1024-thread workgroup per block, block staged in LDS.
//                         P0: the reference's hash chains (deflate_compress.c:312-319,
//                         every position at the head of its bucket) as bucket-sorted
//                         position arrays, by a two-pass LDS radix sort;
//                         P1: the longest match of EVERY position (chain walk of
//                         :243-264, newest first, strict >) -- one lane per entry,
//                         candidates shifted through registers with DPP;
//                         P2: the greedy path 0 -> i + max(len,1) (:265-288) by
//                         speculative 32-position segments + two fix-up levels
//                         (optionally lazy evaluation first, DMX_F_LAZY);
//                         P3: token compaction (block scan) and lit/len + dist
//                         histograms.  Tokens -> HBM.
//   K2  dmx_huff_kernel   one wave per block: length-limited canonical Huffman
//                         codes, RFC 1951 §3.2.7 header, exact stored/fixed/
//                         dynamic cost, BTYPE choice (replaces the reference's
//                         per-token estimators aht.c / h_tree.c).
//   K3  dmx_scan_kernel   one workgroup: bit offsets of all blocks (a scan over an
//                         associative "stored blocks re-align" monoid), Adler-32
//                         combine, zlib header / flush / trailer, boundary words.
//   K4  dmx_pack_kernel   one 256-thread workgroup per block: bit-packs header +
//                         tokens (or the stored bytes) at the block's absolute bit
//                         offset in LDS, then coalesced 32-bit stores to HBM.
// Token encoding: t = byte (literal) | (dist << 9) | len  (DESIGN.md §2).
#include <hip/hip_runtime.h>
#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>

#include "dmx_internal.h"
#include "../../include/dmx.h"

#define MAXLEN 258

// ------------------------------------------------------------------------------------
// small device helpers
// ------------------------------------------------------------------------------------

__device__ __forceinline__ uint32_t dmx_hash(uint32_t tri) { return (tri * 0x9E3779B1u) >> DMX_HASH_SHIFT; }
// The order of the bucket-sorted array S: (bucket of the trigram in the low 3 bytes of w,
// position p < 32768) as one integer, so that adjacent entries are checked with one compare.
// Wave index as a scalar (wave-uniform: the SGPR keeps wave-derived LDS offsets out of
// the vector registers of the match kernel, which otherwise spills them).
__device__ __forceinline__ uint32_t wave_of(uint32_t tid) { return (uint32_t)__builtin_amdgcn_readfirstlane((int)(tid >> 6)); }
__device__ __forceinline__ uint32_t sort_key(uint32_t w, uint32_t p) { return (dmx_hash(w & 0xFFFFFFu) << 15) | p; }
// NB-byte chains (the exhaustive parse, NB = 4 or 5; 3 = the trigram chains): the bucket of
// the first NB bytes of w (position order, byte 0 in the low byte)
__device__ __forceinline__ uint32_t dmx_hash4(uint32_t w) { return (w * 0x9E3779B1u) >> DMX_HASH_SHIFT; }
template <int NB>
__device__ __forceinline__ uint32_t bucket_of(uint64_t w) {
    if (NB == 3) return dmx_hash((uint32_t)w & 0xFFFFFFu);
    if (NB == 4) return dmx_hash4((uint32_t)w);
    return (uint32_t)(((w & 0xFFFFFFFFFFull) * 0x9E3779B97F4A7C15ull) >> (64 - 13));
}
template <int NB>
__device__ __forceinline__ uint32_t sort_key_h(uint64_t w, uint32_t p) { return (bucket_of<NB>(w) << 15) | p; }
// the first NB bytes at p (NB <= 4: one dword)
template <int NB>
__device__ __forceinline__ uint64_t ldg(const uint32_t* W, uint32_t p);

// RFC 1951 §3.2.5 length -> symbol 257..285, extra-bit count, extra value
__device__ __forceinline__ void len_sym(uint32_t len, uint32_t& sym, uint32_t& eb, uint32_t& ev) {
    if (len == 258) { sym = 285; eb = 0; ev = 0; }
    else if (len <= 10) { sym = 254 + len; eb = 0; ev = 0; }
    else {
        uint32_t l = len - 3;
        uint32_t e = 31 - __clz(l) - 2;
        sym = 261 + 4 * e + ((l >> e) - 4);
        eb = e;
        ev = l & ((1u << e) - 1);
    }
}

// RFC 1951 §3.2.5 distance -> symbol 0..29, extra-bit count, extra value
__device__ __forceinline__ void dist_sym(uint32_t dist, uint32_t& sym, uint32_t& eb, uint32_t& ev) {
    uint32_t x = dist - 1;
    if (x < 4) { sym = x; eb = 0; ev = 0; }
    else {
        uint32_t e = 31 - __clz(x);
        eb = e - 1;
        sym = 2 * e + ((x >> (e - 1)) & 1);
        ev = x & ((1u << eb) - 1);
    }
}

__device__ __forceinline__ uint32_t len_eb_of_sym(uint32_t s) {  // s in 257..285
    return (s >= 265 && s < 285) ? (s - 261) / 4 : 0;
}
__device__ __forceinline__ uint32_t dist_eb_of_sym(uint32_t s) { return s < 4 ? 0 : s / 2 - 1; }
__device__ __forceinline__ uint32_t fixed_len(uint32_t s) { return s < 144 ? 8 : s < 256 ? 9 : s < 280 ? 7 : 8; }

// Wave sums by DPP row shifts (lane 15 of each row of 16 ends with the row's sum) and four
// readlanes; the result is uniform.  All 64 lanes must be active.  (__shfl_xor lowers to
// ds_bpermute with per-lane index registers that the compiler keeps live, and spills, across
// the match kernel.)
#define DMX_DPP_SHR(x, n) ((uint32_t)__builtin_amdgcn_update_dpp(0, (int)(x), 0x110 + (n), 0xF, 0xF, true))
__device__ __forceinline__ uint32_t wave_sum_u32(uint32_t v) {
    v += DMX_DPP_SHR(v, 1);
    v += DMX_DPP_SHR(v, 2);
    v += DMX_DPP_SHR(v, 4);
    v += DMX_DPP_SHR(v, 8);
    return __builtin_amdgcn_readlane(v, 15) + __builtin_amdgcn_readlane(v, 31) + __builtin_amdgcn_readlane(v, 47) +
           __builtin_amdgcn_readlane(v, 63);
}
__device__ __forceinline__ uint64_t dpp_shr64(uint64_t v, int n) {
    const uint32_t lo = (uint32_t)v, hi = (uint32_t)(v >> 32);
    uint32_t a, b;
    switch (n) {
        case 1: a = DMX_DPP_SHR(lo, 1); b = DMX_DPP_SHR(hi, 1); break;
        case 2: a = DMX_DPP_SHR(lo, 2); b = DMX_DPP_SHR(hi, 2); break;
        case 4: a = DMX_DPP_SHR(lo, 4); b = DMX_DPP_SHR(hi, 4); break;
        default: a = DMX_DPP_SHR(lo, 8); b = DMX_DPP_SHR(hi, 8); break;
    }
    return (uint64_t)a | ((uint64_t)b << 32);
}
__device__ __forceinline__ uint64_t readlane64(uint64_t v, int l) {
    return (uint64_t)(uint32_t)__builtin_amdgcn_readlane((int)(uint32_t)v, l) |
           ((uint64_t)(uint32_t)__builtin_amdgcn_readlane((int)(uint32_t)(v >> 32), l) << 32);
}
// A wave's next work item from a workgroup counter in LDS, called by all 64 lanes: each adds 1
// (one LDS add of 64 after the atomic optimizer) and (old value) / 64 is the item, the same in
// every lane.  Not `if (lane == 0) x = atomicAdd(..)`: the compiler threaded that branch into
// the previous iteration's lane-0 branches and made gram_pass's walk loop exit lane by lane --
// lanes 1..63 then spun on item 0, a GPU hang (round 4); a lane-0-only add value (1 : 0) takes
// the optimizer's 64-step iterative scan instead.
// Every caller runs it with all 64 lanes active (the counter then moves by 64 a claim);
// DMX_CHECK_CLAIM builds trap on a partial exec mask instead of handing out a wrong item.
__device__ __forceinline__ uint32_t wave_claim(uint32_t* ctr) {
#ifdef DMX_CHECK_CLAIM
    if (__builtin_amdgcn_read_exec() != ~0ull) __builtin_trap();
#endif
    return atomicAdd(ctr, 1u) >> 6;
}
__device__ __forceinline__ uint64_t wave_sum_u64(uint64_t v) {
    v += dpp_shr64(v, 1);
    v += dpp_shr64(v, 2);
    v += dpp_shr64(v, 4);
    v += dpp_shr64(v, 8);
    return readlane64(v, 15) + readlane64(v, 31) + readlane64(v, 47) + readlane64(v, 63);
}

// ------------------------------------------------------------------------------------
// K1: bucket-sorted chains + longest match of every position + greedy path + compaction
// ------------------------------------------------------------------------------------

#define MT 1024
#define MW (MT / 64)
#define DMX_STAMPS 16   // diagnostic u64 stamps per block (DMX_STAMPS=1 in the environment)
#define DATA_WORDS 8272   // 32 KiB + slack: 32-byte extension reads past the end (zeroed); the
                          // history kernel keeps the first bytes of the block there (>= 258 + 40)

struct __attribute__((aligned(16))) MatchLDS {
    uint32_t data[DATA_WORDS];    // the block, zero padded
    uint16_t sorted[DMX_BLK];     // positions sorted by (bucket, position) (P0); after the search: best distances
    uint16_t bstart[DMX_NBUCKET]; // start of every bucket in `sorted`
    uint8_t len8[DMX_BLK];        // best length - 3 (matches)
    uint32_t lit[DMX_BLK / 32];   // 1 = literal at that position
    uint32_t tsm[DMX_BLK / 32];   // token starts, 32 positions per word
    uint32_t exitp[DMX_BLK / 32];
    uint32_t hist[DMX_HIST];
    uint32_t wexit[MW];
    uint32_t wsum[MW];
    uint32_t ntok;
    uint32_t sortbad;   // the search saw two entries of one bucket out of position order
    unsigned long long adl_s, adl_t;
};

// Byte-granular reads of the LDS block built from ALIGNED reads + funnel shifts:
// an unaligned ds_read costs ~8x an aligned one on gfx950 (tools/ldsbench.hip:
// ~1000 vs ~130-220 cycles per wave-instruction with 16 waves resident).
__device__ __forceinline__ uint64_t fsh64(uint64_t lo, uint64_t hi, uint32_t sh) {   // sh in [0, 64)
    return sh ? ((lo >> sh) | (hi << (64 - sh))) : lo;
}
__device__ __forceinline__ uint64_t ld8(const uint32_t* W, uint32_t p) {   // bytes p..p+7
    // three aligned dwords + two v_alignbyte (ds_read2_b32 + ds_read_b32: 6 LDS cycles and 2
    // VALU; two 8-byte words + 64-bit shifts took ds_read2_b64, 8 cycles, and 6 VALU)
    const uint32_t a = p >> 2, sh = p & 3;
    const uint32_t w0 = W[a], w1 = W[a + 1], w2 = W[a + 2];
    return (uint64_t)__builtin_amdgcn_alignbyte(w1, w0, sh) | ((uint64_t)__builtin_amdgcn_alignbyte(w2, w1, sh) << 32);
}
__device__ __forceinline__ uint32_t ld4(const uint32_t* W, uint32_t p) {   // bytes p..p+3
    return __builtin_amdgcn_alignbyte(W[(p >> 2) + 1], W[p >> 2], p & 3);
}
template <int NB>
__device__ __forceinline__ uint64_t ldg(const uint32_t* W, uint32_t p) { return NB > 4 ? ld8(W, p) : (uint64_t)ld4(W, p); }
// A seed in 16 bits: the nearest earlier position q with the same first NG bytes (NG = 3 or
// 4, bit 15 = NG == 4), 0xFFFF = none (q <= bn - 3 < 0x7FFF); decoded into the search's key
// form NG << 15 | q, 0 = none.
template <int NG>
__device__ __forceinline__ uint16_t seed_enc(uint32_t q) {
    return q != 0xFFFFu ? (uint16_t)((NG == 4 ? 0x8000u : 0u) | q) : (uint16_t)0xFFFFu;
}
__device__ __forceinline__ uint32_t seed_dec(uint32_t s) {
    return s == 0xFFFFu ? 0u : ((3u + (s >> 15)) << 15) | (s & 0x7FFFu);
}
// bytes p..p+11 from four aligned dwords (two ds_read2_b32; ld8 + ld4 issued a fifth read)
__device__ __forceinline__ void ld12(const uint32_t* W, uint32_t p, uint32_t& x0, uint32_t& x1, uint32_t& x2) {
    const uint32_t a = p >> 2, sh = p & 3;
    const uint32_t w0 = W[a], w1 = W[a + 1], w2 = W[a + 2], w3 = W[a + 3];
    x0 = __builtin_amdgcn_alignbyte(w1, w0, sh);
    x1 = __builtin_amdgcn_alignbyte(w2, w1, sh);
    x2 = __builtin_amdgcn_alignbyte(w3, w2, sh);
}

__device__ __forceinline__ uint32_t adv_of(const MatchLDS& L, uint32_t p) {
    return ((L.lit[p >> 5] >> (p & 31)) & 1u) ? 1u : (uint32_t)L.len8[p] + 3u;
}

// Longest match (>= 3, ties to the nearest) of every position, deflate_compress.c:243-264.
// Work unit = one entry k of the bucket-sorted array S (position i = S[k]); a wave takes
// 64 consecutive entries (lane = entry), waves take chunks round-robin.  The chain of
// entry k is S[k-1], S[k-2], ..., S[start(bucket)] (newest first, P0), capped at K.
// Candidate j of lane l is entry k-j -- the entry j lanes below -- so every lane loads
// only its OWN position and first 16 bytes once, and the wave shifts (position, 16 bytes)
// down one lane per step with DPP wave_shr:1; lane 0 is fed from a halo of the KD
// entries below the chunk.  Each step compares 64 candidates with ~20 VALU instructions
// and no LDS traffic: 16 bytes give the exact length of any match < 16 (the usual case);
// longer candidates extend from LDS.  Chains longer than KD (exhaustive mode): the W0
// nearest candidates in registers, then windows of KD steps that stream only positions and
// test the bytes a longer match needs (the byte-at-best filter).  The kept key is len << 15 | q:
// longest, then nearest (largest q) -- the reference's newest-first walk with strict >
// (:249-263).  A lane stops comparing once its best is the longest possible length.
#define KD 32
#define W0 8    // long chains: candidates of the first window, compared in registers (the rest filtered)
#ifndef DMX_W0H4
#define DMX_W0H4 8   // the same on the exhaustive parse's 4-byte chains
#endif
#define CB 12   // bytes compared in registers per candidate step; longer matches extend from LDS
#define KE 8    // chains up to KE candidates use chunks with the halo embedded (64-K owned entries)
#ifndef XU
#define XU 4    // exhaustive later windows: filter steps whose LDS reads are in flight together
#endif
#define JR 8    // Jacobi rounds of the walk before the serial fallback
#define WALK_SERIAL 1024   // fallback: at most this many tokens (approximate path) -> one-lane token walk
#define TPMAX (DMX_NBUCKET)   // token positions listed in bstart (u16) for the token-major compaction
#define HSTR (DMX_HIST + 1)   // stride of the 4 histogram copies of the compaction
__device__ __forceinline__ uint32_t ffbl(uint32_t x) {   // lowest set bit, ~0 for 0 (v_ffbl_b32)
    return x ? (uint32_t)__builtin_ctz(x) : 0xFFFFFFFFu;
}
// v_ffbl_b32 as the hardware defines it (lowest set bit, ~0 for 0), opaque to the
// optimizer so it does not re-derive the zero case with compares and selects.
__device__ __forceinline__ uint32_t ffbl_hw(uint32_t x) {
    uint32_t r;
    asm("v_ffbl_b32 %0, %1" : "=v"(r) : "v"(x));
    return r;
}
__device__ __forceinline__ uint32_t match_bytes(uint64_t x) {   // equal leading bytes of an 8-byte xor
    return x ? ((uint32_t)__builtin_ctzll(x) >> 3) : 8u;
}
__device__ __forceinline__ uint32_t wshr(uint32_t v, uint32_t lane0) {   // lane l <- lane l-1; lane 0 <- lane0
    return (uint32_t)__builtin_amdgcn_update_dpp((int)lane0, (int)v, 0x138, 0xF, 0xF, false);
}
// Length of a candidate known to match bytes [0, kk): 24 bytes in the first LDS round trip
// (most extensions end there), then 32 per round trip.
// Each side is read as 9 aligned words and realigned with v_alignbyte (one VALU per 4
// bytes); the first differing word comes from a mask of non-zero xors.
#ifndef EXT_W2
#define EXT_W2 8   // words compared in each later round (reads reach 4 EXT_W2 + 4 bytes past kk)
#endif
#ifndef EXT_W1
#define EXT_W1 6   // words compared in the first round (24 bytes; 16 took 1.202 ms of K1 on C3, 24 1.185)
#endif
__device__ __forceinline__ uint32_t ext_len2(const uint32_t* A, uint32_t i, const uint32_t* B, uint32_t q, uint32_t kk,
                                             uint32_t lim) {
    {   // first round: 4 EXT_W1 bytes (EXT_W1 + 1 aligned words per side)
        const uint32_t a = (i + kk) >> 2, sa = (i + kk) & 3, c = (q + kk) >> 2, sc = (q + kk) & 3;
        uint32_t wa[EXT_W1 + 1], wc[EXT_W1 + 1];
#pragma unroll
        for (int t = 0; t < EXT_W1 + 1; t++) { wa[t] = A[a + t]; wc[t] = B[c + t]; }
        uint32_t x[EXT_W1], nz = 0;
#pragma unroll
        for (int t = 0; t < EXT_W1; t++) {
            x[t] = __builtin_amdgcn_alignbyte(wa[t + 1], wa[t], sa) ^ __builtin_amdgcn_alignbyte(wc[t + 1], wc[t], sc);
            nz |= (x[t] != 0 ? 1u : 0u) << t;
        }
        if (nz) {
            const uint32_t t0 = (uint32_t)__builtin_ctz(nz);
            uint32_t xv = x[0];
#pragma unroll
            for (int t = 1; t < EXT_W1; t++) xv = (t0 == (uint32_t)t) ? x[t] : xv;
            return kk + 4 * t0 + ((uint32_t)__builtin_ctz(xv) >> 3);
        }
        kk += 4 * EXT_W1;
        if (kk >= lim) return kk;
    }
    for (;;) {
        const uint32_t a = (i + kk) >> 2, sa = (i + kk) & 3, c = (q + kk) >> 2, sc = (q + kk) & 3;
        uint32_t wa[EXT_W2 + 1], wc[EXT_W2 + 1];
#pragma unroll
        for (int t = 0; t < EXT_W2 + 1; t++) { wa[t] = A[a + t]; wc[t] = B[c + t]; }
        uint32_t x[EXT_W2], nz = 0;
#pragma unroll
        for (int t = 0; t < EXT_W2; t++) {
            x[t] = __builtin_amdgcn_alignbyte(wa[t + 1], wa[t], sa) ^ __builtin_amdgcn_alignbyte(wc[t + 1], wc[t], sc);
            nz |= (x[t] != 0 ? 1u : 0u) << t;
        }
        if (nz) {
            const uint32_t t0 = (uint32_t)__builtin_ctz(nz);
            uint32_t xv = x[0];
#pragma unroll
            for (int t = 1; t < EXT_W2; t++) xv = (t0 == (uint32_t)t) ? x[t] : xv;
            return kk + 4 * t0 + ((uint32_t)__builtin_ctz(xv) >> 3);
        }
        kk += 4 * EXT_W2;
        if (kk >= lim) return kk;
    }
}
// (both sides in the block)
__device__ __forceinline__ uint32_t ext_len(const MatchLDS& L, uint32_t i, uint32_t q, uint32_t kk, uint32_t lim) {
    return ext_len2(L.data, i, L.data, q, kk, lim);
}
// Change bitmap (bounded mode with a short chain, K <= KE: the walk's exit array is free
// during the search): bit p = data[p] != data[p+1] (set for p >= bn - 1).  Built at the
// start of the search (search_positions); gives a distance-1 candidate's exact length in a
// few word reads.
__device__ __forceinline__ uint32_t* chg_bits(MatchLDS& L) { return L.exitp; }
__device__ __forceinline__ uint32_t* chg_bits(const MatchLDS& L) { return const_cast<uint32_t*>(L.exitp); }
// Winner of every entry of S in the short-chain mode (K <= KE), 4 bits per entry in bucket
// order, in bstart (bucket starts are not needed there): 0 = no match, j = 1..KE = chain
// candidate j (entry k - j of S), 15 = the history match (DMX_F_DICT).  After the search
// the distance of entry k is S[k] - S[k - j]: no distance staging buffer in HBM.
#define NIB_HIST 15u
__device__ __forceinline__ uint32_t* nib_words(MatchLDS& L) { return reinterpret_cast<uint32_t*>(L.bstart); }
// Length of the match at i against i - 1 (>= 1 known equal bytes), capped at lim: the first
// change at or after i - 1 ends it.
__device__ __forceinline__ uint32_t run_len(const MatchLDS& L, uint32_t i, uint32_t lim) {
    const uint32_t* C = chg_bits(L);
    const uint32_t x = i - 1u, a = x >> 5;   // lim <= 258: a change at x + lim - 1 <= 32a + 288 decides
    uint32_t r = 0xFFFFFFFFu;
#pragma unroll
    for (int t0 = 0; t0 < 10; t0 += 5) {   // 5 independent reads per round; most runs end in the first
        if (r != 0xFFFFFFFFu) break;
        uint32_t w[5];
#pragma unroll
        for (int t = 0; t < 5; t++) w[t] = C[min(a + (uint32_t)(t0 + t), (uint32_t)(DMX_BLK / 32 - 1))];
        if (t0 == 0) w[0] &= ~0u << (x & 31);
#pragma unroll
        for (int t = 4; t >= 0; t--) r = w[t] ? ((a + (uint32_t)(t0 + t)) << 5) + (uint32_t)__builtin_ctz(w[t]) : r;
    }
    return r == 0xFFFFFFFFu ? lim : min(r - x, lim);
}

// Builds the change bitmap (bounded mode, K <= KE, after P0: bstart is free) and returns
// whether the block is run-dominated: at least a quarter of its 32-byte segments hold fewer
// than 8 byte changes.  Such blocks search with run_len (search_positions<.., true>).
__device__ __forceinline__ bool build_chg(MatchLDS& L, uint32_t bn, uint32_t tid) {
    const uint32_t lo = tid << 5;
    const uint4 v0 = *reinterpret_cast<const uint4*>(&L.data[lo >> 2]);
    const uint4 v1 = *reinterpret_cast<const uint4*>(&L.data[(lo >> 2) + 4]);
    const uint32_t w[9] = {v0.x, v0.y, v0.z, v0.w, v1.x, v1.y, v1.z, v1.w, L.data[(lo >> 2) + 8]};
    uint32_t m = 0;
#pragma unroll
    for (int t = 0; t < 8; t++) {   // byte b of word t vs the byte after it
        const uint32_t nx = __builtin_amdgcn_alignbyte(w[t + 1], w[t], 1);
        const uint32_t x = w[t] ^ nx;
#pragma unroll
        for (int bb = 0; bb < 4; bb++) m |= (((x >> (8 * bb)) & 0xFFu) != 0u ? 1u : 0u) << (4 * t + bb);
    }
    const uint32_t last = bn ? bn - 1u : 0u;   // positions >= bn - 1 end every run
    if (lo + 32 > last) m |= lo >= last ? 0xFFFFFFFFu : ~((1u << (last - lo)) - 1u);
    chg_bits(L)[tid] = m;
    return __syncthreads_count(lo < bn && __popc(m) < 8) * 4 >= (int)((bn + 31) >> 5);
}

// Could candidate q (known to match [0, 16)) be strictly longer than best (>= 16)? Only if
// it also matches the byte at offset best.
__device__ __forceinline__ bool may_beat(const MatchLDS& L, uint32_t i, uint32_t q, uint32_t best) {
    const uint8_t* D8 = reinterpret_cast<const uint8_t*>(L.data);
    return D8[q + best] == D8[i + best];
}

// DPP row_shr:n (n = 1, 2, 4, 8) in VALU; lanes without a source read 0.  (__shfl_* lowers
// to ds_bpermute_b32, an LDS round trip.)
__device__ __forceinline__ uint32_t dpp_shr(uint32_t v, int n) {
    switch (n) {
        case 1: return (uint32_t)__builtin_amdgcn_update_dpp(0, (int)v, 0x111, 0xF, 0xF, true);
        case 2: return (uint32_t)__builtin_amdgcn_update_dpp(0, (int)v, 0x112, 0xF, 0xF, true);
        case 4: return (uint32_t)__builtin_amdgcn_update_dpp(0, (int)v, 0x114, 0xF, 0xF, true);
        default: return (uint32_t)__builtin_amdgcn_update_dpp(0, (int)v, 0x118, 0xF, 0xF, true);
    }
}

// LDS word accesses shared between lanes of one wave: relaxed workgroup-scope atomics keep
// them as plain ds_read/ds_write and stop the compiler from caching or reordering them
// (a volatile cast would drop the LDS address space and go through flat memory).
__device__ __forceinline__ uint32_t lds_ld(uint32_t* p) {
    return __hip_atomic_load(p, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
}
__device__ __forceinline__ void lds_st(uint32_t* p, uint32_t v) {
    __hip_atomic_store(p, v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
}

// Inclusive prefix sum over the wave: DPP row shifts inside each row of 16, row totals by readlane.
__device__ __forceinline__ uint32_t wave_incl_scan(uint32_t x) {
    const uint32_t r = threadIdx.x & 15, row = (threadIdx.x & 63) >> 4;
    uint32_t y;
    y = dpp_shr(x, 1); if (r >= 1) x += y;
    y = dpp_shr(x, 2); if (r >= 2) x += y;
    y = dpp_shr(x, 4); if (r >= 4) x += y;
    y = dpp_shr(x, 8); if (r >= 8) x += y;
    const uint32_t t0 = __builtin_amdgcn_readlane(x, 15), t1 = __builtin_amdgcn_readlane(x, 31),
                   t2 = __builtin_amdgcn_readlane(x, 47);
    return x + (row >= 1 ? t0 : 0u) + (row >= 2 ? t1 : 0u) + (row >= 3 ? t2 : 0u);
}

// The candidate steps of one chunk.  Step j: every register stream moves down one lane
// (lane 0 takes halo entry j-1), so lane l holds entry k-j, its j-th chain candidate.
// Key = (equal bytes, max 8) << 8 | (255 - j): the max over j is the longest match, then
// the smallest j = the nearest (positions increase along a bucket).  No per-step validity
// test: an entry before the bucket start has another bucket, hence another trigram, so it
// never reaches 3 equal bytes, and candidates < 3 bytes are discarded once after the max.
// Only the first chunk of the block (GUARD) has halo lanes without entries.
template <bool GUARD>
__device__ __forceinline__ void cand_step(uint32_t j, uint32_t& x0, uint32_t& x1, uint32_t& x2, uint32_t i0, uint32_t i1,
                                          uint32_t i2, uint32_t h0, uint32_t h1, uint32_t h2, uint32_t nc,
                                          uint32_t lim_eff, uint32_t& jkey, uint32_t& full) {
    const int src = (int)j - 1;
    x0 = wshr(x0, __builtin_amdgcn_readlane(h0, src));
    x1 = wshr(x1, __builtin_amdgcn_readlane(h1, src));
    x2 = wshr(x2, __builtin_amdgcn_readlane(h2, src));
    // equal leading bits of the 12-byte window, 96 = all: opaque v_ffbl (~0 for 0), two
    // saturating adds, v_min3, and the cap
    const uint32_t mb = min(min(min(ffbl_hw(i0 ^ x0), __builtin_elementwise_add_sat(ffbl_hw(i1 ^ x1), 32u)),
                                __builtin_elementwise_add_sat(ffbl_hw(i2 ^ x2), 64u)),
                            96u);
    uint32_t m = min(mb >> 3, lim_eff);
    bool fl = mb == 96u;
    if (GUARD) {
        m = j <= nc ? m : 0u;
        fl = fl && j <= nc;
    }
    jkey = max(jkey, (m << 8) | (255u - j));
    full |= fl ? (1u << src) : 0u;
}
template <bool GUARD>
__device__ __forceinline__ void cand_steps(uint32_t jmax, uint32_t& x0, uint32_t& x1, uint32_t& x2, uint32_t i0,
                                           uint32_t i1, uint32_t i2, uint32_t h0, uint32_t h1, uint32_t h2, uint32_t nc,
                                           uint32_t lim_eff, uint32_t& jkey, uint32_t& full) {
    uint32_t y0, y1, y2;
    uint32_t j = 1;
    for (; j + 1 <= jmax; j += 2) {   // two steps per trip, alternating registers (no copies)
        y0 = x0; y1 = x1; y2 = x2;
        cand_step<GUARD>(j, y0, y1, y2, i0, i1, i2, h0, h1, h2, nc, lim_eff, jkey, full);
        x0 = y0; x1 = y1; x2 = y2;
        cand_step<GUARD>(j + 1, x0, x1, x2, i0, i1, i2, h0, h1, h2, nc, lim_eff, jkey, full);
    }
    if (j <= jmax) cand_step<GUARD>(j, x0, x1, x2, i0, i1, i2, h0, h1, h2, nc, lim_eff, jkey, full);
}

// Candidates matching all CB register bytes (any of them beats every key found in
// registers): exact length from LDS.  Round 1: each lane's nearest one; a lane whose best
// is then the longest possible is done (runs end here).  The rest are spread over the
// wave's lanes through an LDS queue (one round for typical text instead of max-popcount
// rounds) and merged with atomicMax on the key, which orders longest, then nearest.
// kb = entry of lane 0 of the chunk (owner lane o has entry kb + o).
template <bool SHORT, bool RUNS>
__device__ __forceinline__ uint32_t resolve_full(MatchLDS& L, uint32_t bn, uint32_t lane, uint32_t wave, uint32_t k,
                                                 uint32_t i, uint32_t lim_eff, uint32_t bestkey, uint32_t full,
                                                 uint32_t kb) {
    if (__ballot(full != 0) == 0) return bestkey;
    if (full) {
        const uint32_t j = (uint32_t)__builtin_ctz(full) + 1u;
        full &= full - 1u;
        const uint32_t q = L.sorted[k - j];
        // distance 1 (runs): the length is where the run ends, from the change bitmap
        const uint32_t len = min(q + 1u == i && SHORT && RUNS ? run_len(L, i, lim_eff) : ext_len(L, i, q, CB, lim_eff),
                                 lim_eff);
        bestkey = max(bestkey, (len << 15) | q);
    }
    if ((bestkey >> 15) >= lim_eff) full = 0;
    if (SHORT) {   // chains <= 8: filter the rest in place, extend the (rare) survivors per lane
        const uint32_t bl = bestkey >> 15;
        const uint8_t* D8 = reinterpret_cast<const uint8_t*>(L.data);
        uint32_t surv = 0;
        if (full) {
            const uint32_t ib = D8[i + bl];
#pragma unroll
            for (uint32_t j = 1; j <= KE; j++)
                if ((full >> (j - 1)) & 1u) surv |= (D8[(uint32_t)L.sorted[k - j] + bl] == ib ? 1u : 0u) << (j - 1);
        }
        while (__ballot(surv != 0)) {
            if (surv) {
                const uint32_t j = (uint32_t)__builtin_ctz(surv) + 1u;
                surv &= surv - 1u;
                const uint32_t q = L.sorted[k - j];
                const uint32_t len = min(ext_len(L, i, q, CB, lim_eff), lim_eff);
                bestkey = max(bestkey, (len << 15) | q);
            }
        }
        return bestkey;
    }
    const uint32_t cnt = __popc(full);
    const uint32_t incl = wave_incl_scan(cnt);
    const uint32_t T = __builtin_amdgcn_readlane(incl, 63);
    uint32_t* Q = L.tsm + (wave << 6);     // P2 arrays, free during the search
    uint32_t* B = L.exitp + (wave << 6);
    for (uint32_t base = 0; base < T; base += 64) {
        lds_st(&B[lane], bestkey);   // owners' best so far: filters the queued candidates
        uint32_t f = full, idx = incl - cnt;
        while (f) {
            const uint32_t j = (uint32_t)__builtin_ctz(f) + 1u;
            f &= f - 1u;
            if (idx >= base && idx < base + 64) lds_st(&Q[idx - base], (k - j) | (lane << 16));
            idx++;
        }
        __builtin_amdgcn_wave_barrier();
        if (base + lane < T) {
            const uint32_t it = lds_ld(&Q[lane]), o = it >> 16;
            const uint32_t q = L.sorted[it & 0xFFFFu], ii = L.sorted[kb + o];
            const uint32_t lo = min(bn - ii, (uint32_t)MAXLEN);
            const uint32_t bl = lds_ld(&B[o]) >> 15;   // >= CB: the owner's round-1 length
            // only a candidate that also matches byte bl can be strictly longer
            if (bl < lo && may_beat(L, ii, q, bl)) {
                const uint32_t len = min(ext_len(L, ii, q, CB, lo), lo);
                __hip_atomic_fetch_max(&B[o], (len << 15) | q, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
            }
        }
        __builtin_amdgcn_wave_barrier();
        bestkey = max(bestkey, lds_ld(&B[lane]));
        __builtin_amdgcn_wave_barrier();
    }
    return bestkey;
}

// Result of one position: length (len8, literal bit) in position order, distance in bucket
// order -- one coalesced 128-byte store per wave (a store to pg[i] would scatter 2-byte
// partial-line writes over the block).
// DMX_F_DICT: hbk = the history kernel's result of entry k (len << 16 | dist, 0 = none, in
// the same bucket order); the history is older than the whole block, so it replaces the
// block's own match only when strictly longer.
template <bool DICT>
__device__ __forceinline__ void store_result(MatchLDS& L, uint16_t* __restrict__ pg, uint32_t k, uint32_t i,
                                             uint32_t bestkey, const uint32_t* __restrict__ hbk) {
    uint32_t len = bestkey >> 15, dist = bestkey ? i - (bestkey & 0x7FFFu) : 0u;
    if (DICT) {
        const uint32_t hw = hbk[k];
        if ((hw >> 16) > len) { len = hw >> 16; dist = hw & 0xFFFFu; }
    }
    if (len == 0) {
        atomicOr(&L.lit[i >> 5], 1u << (i & 31));
        L.len8[i] = 0;
    } else {
        L.len8[i] = (uint8_t)(len - 3);
    }
    pg[k] = (uint16_t)dist;
}

// Candidate steps with the halo embedded in the chunk (K <= KE): lanes 0..K-1 hold the K
// entries before the chunk's owned entries, so a plain wave_shr feeds every owned lane.
// The short-chain search compares CBS = 8 bytes in registers (two streams, 10 VALU per
// step): only 8 % of text entries have a candidate equal in all 8 (4.6 % in 12), and those
// go to the extension queue, which extends 64 of them at a time.
// Key = (equal bits rounded down to bytes) | (8 - j): one v_and_or, 8 * bytes in the high
// part, then the nearest (smallest j) -- K <= 8, so 8 - j fits the 3 low bits.  A key >= 64
// means some candidate equals all CBS bytes; the queue finds which ones from LDS.
#define CBS 8
template <bool GUARD, bool CLAMP>
__device__ __forceinline__ void cand_step_emb(uint32_t j, uint32_t& x0, uint32_t& x1, uint32_t i0, uint32_t i1,
                                              uint32_t nc, uint32_t lim_eff, uint32_t& jkey) {
    x0 = (uint32_t)__builtin_amdgcn_update_dpp(0, (int)x0, 0x138, 0xF, 0xF, true);
    x1 = (uint32_t)__builtin_amdgcn_update_dpp(0, (int)x1, 0x138, 0xF, 0xF, true);
    // equal leading bits, 64 = all CBS bytes: ffbl(0) = ~0 and the saturating add keeps it
    // there; one min3 caps at 64 (v_add_u32 clamp + v_min3_u32)
    const uint32_t mb = min(min(ffbl_hw(i0 ^ x0), __builtin_elementwise_add_sat(ffbl_hw(i1 ^ x1), 32u)), 64u);
    uint32_t key;
    if (CLAMP) key = (min(mb >> 3, lim_eff) << 3) | (8u - j);   // only chunks holding one of the last CBS-1 positions
    else key = (mb & ~7u) | (8u - j);
    if (GUARD) key = j <= nc ? key : 0u;
    jkey = max(jkey, key);
}
template <bool GUARD, bool CLAMP>
__device__ __forceinline__ void cand_steps_emb(uint32_t K, uint32_t i0, uint32_t i1, uint32_t nc, uint32_t lim_eff,
                                               uint32_t& jkey) {
    uint32_t x0 = i0, x1 = i1;
    for (uint32_t j = 1; j <= K; j++) cand_step_emb<GUARD, CLAMP>(j, x0, x1, i0, i1, nc, lim_eff, jkey);
}
// The common chunk (no guard, no clamp) with K known at compile time: fully unrolled, so the
// step's 8 - j is an inline constant and the key is one v_and_or_b32 (the compiler would
// narrow the -8 mask to a non-inline 0x78 and split it); keys of two steps fold into one
// v_max3.  10 VALU per step, no loop SALU.
template <int SJ>
__device__ __forceinline__ uint32_t step_key_c(uint32_t i0, uint32_t i1, uint32_t& x0, uint32_t& x1) {
    x0 = (uint32_t)__builtin_amdgcn_update_dpp(0, (int)x0, 0x138, 0xF, 0xF, true);
    x1 = (uint32_t)__builtin_amdgcn_update_dpp(0, (int)x1, 0x138, 0xF, 0xF, true);
    const uint32_t mb = min(min(ffbl_hw(i0 ^ x0), __builtin_elementwise_add_sat(ffbl_hw(i1 ^ x1), 32u)), 64u);
    uint32_t key;
    asm("v_and_or_b32 %0, %1, -8, %2" : "=v"(key) : "v"(mb), "n"(SJ));
    return key;
}
template <int J, int KK>
__device__ __forceinline__ void steps_from(uint32_t i0, uint32_t i1, uint32_t& x0, uint32_t& x1, uint32_t& jkey) {
    if constexpr (J <= KK) {
        const uint32_t ka = step_key_c<8 - J>(i0, i1, x0, x1);
        if constexpr (J + 1 <= KK) {
            const uint32_t kb = step_key_c<7 - J>(i0, i1, x0, x1);
            jkey = max(jkey, max(ka, kb));
        } else {
            jkey = max(jkey, ka);
        }
        steps_from<J + 2, KK>(i0, i1, x0, x1, jkey);
    }
}
template <int KK>
__device__ __forceinline__ void cand_steps_fixed(uint32_t i0, uint32_t i1, uint32_t& jkey) {
    uint32_t x0 = i0, x1 = i1;
    steps_from<1, KK>(i0, i1, x0, x1, jkey);
}

// Result of entry k (position i) in the short-chain mode: length (0 = none) and winner j
// (chain candidate, 1..KE).  The length goes to len8 / lit in position order, the winner to
// the entry's nibble; the distance is recovered after the search (nibble_dists).
// DMX_F_DICT: the history kernel's result of entry k (len << 16 | dist, 0 = none, bucket
// order) replaces the block's own match only when strictly longer.
template <bool DICT>
__device__ __forceinline__ void store_short(MatchLDS& L, uint32_t k, uint32_t i, uint32_t len, uint32_t j,
                                            const uint32_t* __restrict__ hbk) {
    if (DICT) {
        const uint32_t hw = hbk[k];
        if ((hw >> 16) > len) { len = hw >> 16; j = NIB_HIST; }
    }
    if (len == 0) {
        atomicOr(&L.lit[i >> 5], 1u << (i & 31));
        L.len8[i] = 0;
    } else {
        L.len8[i] = (uint8_t)(len - 3);
        atomicOr(&nib_words(L)[k >> 3], j << ((k & 7u) << 2));
    }
}

// The queued entries of one wave (qn <= 64, items k | jw << 15: entry k, whose nearest
// candidate equal in all CBS register bytes is chain candidate jw): lane l takes item l and
// extends jw from LDS.  A farther candidate must be strictly longer, so it must equal the
// CBS bytes and the byte at the best length: that byte is tested first (one read), the
// CBS bytes only for the rare survivors.  Then the entry's result is stored.
template <bool DICT, bool RUNS>
__device__ __forceinline__ void ext_queue(MatchLDS& L, uint32_t bn, uint32_t K, uint32_t* Qw, uint32_t qn,
                                          uint32_t lane, const uint32_t* __restrict__ hbk, uint32_t head = 0,
                                          uint32_t qmask = 63) {
    __builtin_amdgcn_wave_barrier();
    if (lane < qn) {
        const uint32_t it = lds_ld(&Qw[(head + lane) & qmask]);   // (items head .. head + qn - 1 of a ring)
        const uint32_t k = it & 0x7FFFu, nc = min(k, K);
        uint32_t bj = it >> 15;
        const uint32_t i = L.sorted[k];
        const uint32_t lim = min(bn - i, (uint32_t)MAXLEN);
        const uint8_t* D8 = reinterpret_cast<const uint8_t*>(L.data);
        const uint32_t q = L.sorted[k - bj];
        // distance 1 (runs): the length is where the run ends, from the change bitmap
        uint32_t bl = min(q + 1u == i && RUNS ? run_len(L, i, lim) : ext_len(L, i, q, CBS, lim), lim);
        if (bl < lim) {
            // the byte test of every farther candidate at once (independent LDS reads)
            const uint32_t ib = D8[i + bl], j0 = bj + 1u;
            uint32_t surv = 0;
#pragma unroll
            for (uint32_t t = 0; t < KE - 1; t++) {
                const uint32_t j = j0 + t;
                const uint32_t qj = L.sorted[k - min(j, nc)];
                surv |= (j <= nc && D8[qj + bl] == ib) ? 1u << t : 0u;
            }
            while (surv && bl < lim) {   // rare: test the CBS bytes, then extend
                const uint32_t j = j0 + (uint32_t)__builtin_ctz(surv);
                surv &= surv - 1u;
                const uint32_t qj = L.sorted[k - j];
                if (D8[qj + bl] != D8[i + bl] || ld8(L.data, qj) != ld8(L.data, i)) continue;
                const uint32_t len = min(ext_len(L, i, qj, CBS, lim), lim);
                if (len > bl) { bl = len; bj = j; }
            }
        }
        store_short<DICT>(L, k, i, bl, bj, hbk);
    }
    __builtin_amdgcn_wave_barrier();
}

// ---- Short chains K = 6..8 (the bench's parse), two entries per lane ----------------------
// Lane l holds the consecutive entries A = 2l' and B = 2l' + 1 of S (l' = l - HL); lanes below
// HL = ceil(K/2) are the halo.  Candidate j of A is B of lane l - (j+1)/2 (j odd) or A of lane
// l - j/2 (j even); of B, A of lane l - (j-1)/2 (j odd) or B of lane l - j/2 (j even).  So the
// wave shifts SA_s = A shifted down s lanes and SB_s serve both entries: per step pair one
// shift of each stream and four compares -- one DPP move per compare instead of two, half the
// halo lanes (HL of 64 instead of K), and the chunk's bookkeeping spread over 2 (64 - HL)
// entries instead of 64 - K.  Same keys and results as the one-entry-per-lane path.
#define PSHR(x) ((uint32_t)__builtin_amdgcn_update_dpp(0, (int)(x), 0x138, 0xF, 0xF, true))   // wave_shr:1
template <int SJ>
__device__ __forceinline__ uint32_t pkey(uint32_t e0, uint32_t e1, uint32_t c0, uint32_t c1) {
    const uint32_t mb = min(min(ffbl_hw(e0 ^ c0), __builtin_elementwise_add_sat(ffbl_hw(e1 ^ c1), 32u)), 64u);
    uint32_t key;
    asm("v_and_or_b32 %0, %1, -8, %2" : "=v"(key) : "v"(mb), "n"(SJ));
    return key;
}
// the first chunk (GUARD: candidates below entry 0) and chunks holding one of the last CBS - 1
// positions (CLAMP: lengths capped at the block end), per entry
template <bool GUARD, bool CLAMP>
__device__ __forceinline__ uint32_t pkey_g(uint32_t e0, uint32_t e1, uint32_t c0, uint32_t c1, uint32_t j, uint32_t nc,
                                           uint32_t lim) {
    const uint32_t mb = min(min(ffbl_hw(e0 ^ c0), __builtin_elementwise_add_sat(ffbl_hw(e1 ^ c1), 32u)), 64u);
    uint32_t key = CLAMP ? ((min(mb >> 3, lim) << 3) | (8u - j)) : ((mb & ~7u) | (8u - j));
    if (GUARD) key = j <= nc ? key : 0u;
    return key;
}
// step pair s (template recursion: the keys' 8 - j are inline constants); on entry pa = SA_{s-1},
// sb = SB_{s-1}
template <int KK, int S, bool GEN, bool GUARD, bool CLAMP>
__device__ __forceinline__ void pair_from(uint32_t a0, uint32_t a1, uint32_t b0, uint32_t b1, uint32_t& pa0,
                                          uint32_t& pa1, uint32_t& sb0, uint32_t& sb1, uint32_t& ka, uint32_t& kb,
                                          uint32_t nca, uint32_t ncb, uint32_t lima, uint32_t limb) {
    if constexpr (2 * S - 1 <= KK) {
        constexpr int J1 = 2 * S - 1, J2 = 2 * S;
        sb0 = PSHR(sb0);
        sb1 = PSHR(sb1);   // SB_S
        uint32_t ta, tb;
        if constexpr (GEN) {
            ta = pkey_g<GUARD, CLAMP>(a0, a1, sb0, sb1, J1, nca, lima);   // A vs B of lane l - S
            tb = pkey_g<GUARD, CLAMP>(b0, b1, pa0, pa1, J1, ncb, limb);   // B vs A of lane l - S + 1
        } else {
            ta = pkey<8 - J1>(a0, a1, sb0, sb1);
            tb = pkey<8 - J1>(b0, b1, pa0, pa1);
        }
        if constexpr (J2 <= KK) {
            pa0 = PSHR(pa0);
            pa1 = PSHR(pa1);   // SA_S
            uint32_t ua, ub;
            if constexpr (GEN) {
                ua = pkey_g<GUARD, CLAMP>(a0, a1, pa0, pa1, J2, nca, lima);   // A vs A of lane l - S
                ub = pkey_g<GUARD, CLAMP>(b0, b1, sb0, sb1, J2, ncb, limb);   // B vs B of lane l - S
            } else {
                ua = pkey<8 - J2>(a0, a1, pa0, pa1);
                ub = pkey<8 - J2>(b0, b1, sb0, sb1);
            }
            ka = max(ka, max(ta, ua));
            kb = max(kb, max(tb, ub));
        } else {
            ka = max(ka, ta);
            kb = max(kb, tb);
        }
        pair_from<KK, S + 1, GEN, GUARD, CLAMP>(a0, a1, b0, b1, pa0, pa1, sb0, sb1, ka, kb, nca, ncb, lima, limb);
    }
}
// Result of entry k at position i without a queued extension (store_short's, returning the
// winner nibble instead of storing it: both entries of a lane share one nibble word).
template <bool DICT>
__device__ __forceinline__ uint32_t short_result(MatchLDS& L, uint32_t k, uint32_t i, uint32_t jkey,
                                                 const uint32_t* __restrict__ hbk) {
    const uint32_t m = jkey >> 3;
    uint32_t len = m >= 3 ? m : 0u, j = m >= 3 ? 8u - (jkey & 7u) : 0u;
    if (DICT) {
        const uint32_t hw = hbk[k];
        if ((hw >> 16) > len) { len = hw >> 16; j = NIB_HIST; }
    }
    if (len == 0) {
        atomicOr(&L.lit[i >> 5], 1u << (i & 31));
        L.len8[i] = 0;
        return 0;
    }
    L.len8[i] = (uint8_t)(len - 3);
    return j;
}
template <bool DICT, int KK>
__device__ __forceinline__ uint32_t search_pairs(MatchLDS& L, uint32_t bn, uint32_t tid, bool stamp, uint64_t& tdef,
                                                 const uint32_t* __restrict__ hbk) {
    constexpr uint32_t HL = (KK + 1) / 2, OWN = 2 * (64 - HL);
    const uint32_t lane = tid & 63, wave = wave_of(tid);
    const uint32_t nvalid = bn > 2 ? bn - 2 : 0;
    uint32_t* Qw = L.tsm + (wave << 6);   // the extension queue (P2 arrays are free during the search)
    const uint64_t lt = (1ull << lane) - 1ull;
    uint32_t qn = 0, iters = 0;
    // chunks are taken from a workgroup counter (L.ntok, zeroed before the search), the next
    // one fetched a chunk ahead: the waves finish together whatever their queues cost
    uint32_t cnext = wave_claim(&L.ntok);
    for (;;) {
        const uint32_t base = (uint32_t)__builtin_amdgcn_readfirstlane((int)cnext) * OWN;
        const bool more = base < nvalid;   // wave-uniform
        if (more) cnext = wave_claim(&L.ntok);
        const int ea = (int)base + 2 * ((int)lane - (int)HL);
        const uint32_t ka = (uint32_t)ea, kb = ka + 1;
        const bool own = lane >= HL;
        const bool actA = more && own && ka < nvalid, actB = more && own && kb < nvalid;
        uint32_t jA = 0, jB = 0, limA = 0, limB = 0, iA = 0, iB = 0;
        if (more) {
            uint32_t a0 = 0, a1 = 0, b0 = 0, b1 = 0;
            if (ea >= 0 && ka < nvalid) {   // both positions in one aligned LDS word
                const uint32_t pr = reinterpret_cast<const uint32_t*>(L.sorted)[ka >> 1];
                iA = pr & 0xFFFFu;
                const uint64_t va = ld8(L.data, iA);
                a0 = (uint32_t)va;
                a1 = (uint32_t)(va >> 32);
                if (kb < nvalid) {
                    iB = pr >> 16;
                    const uint64_t vb = ld8(L.data, iB);
                    b0 = (uint32_t)vb;
                    b1 = (uint32_t)(vb >> 32);
                }
            }
            if (actA) limA = (bn - iA) < MAXLEN ? (bn - iA) : MAXLEN;
            if (actB) limB = (bn - iB) < MAXLEN ? (bn - iB) : MAXLEN;
            iters += 2 * KK;
            {   // sort check: A after B of the lane below, B after A
                const uint32_t skA = sort_key(a0, iA), skB = sort_key(b0, iB);
                const uint32_t pk = PSHR(skB);
                if (__ballot((actA && ka >= 1 && pk > skA) || (actB && skA > skB))) L.sortbad = 1;
            }
            uint32_t pa0 = a0, pa1 = a1, sb0 = b0, sb1 = b1;
            if (base == 0)
                pair_from<KK, 1, true, true, true>(a0, a1, b0, b1, pa0, pa1, sb0, sb1, jA, jB, min(ka, (uint32_t)KK),
                                                   min(kb, (uint32_t)KK), limA, limB);
            else if (__ballot((actA && limA < CBS) || (actB && limB < CBS)))
                pair_from<KK, 1, true, false, true>(a0, a1, b0, b1, pa0, pa1, sb0, sb1, jA, jB, KK, KK, limA, limB);
            else
                pair_from<KK, 1, false, false, false>(a0, a1, b0, b1, pa0, pa1, sb0, sb1, jA, jB, 0, 0, 0, 0);
        }
        // a candidate equal in all CBS bytes (key >= 64): the entry is queued for the LDS
        // extension (unless the block end caps it there); A's items, then B's
        const bool pushA = actA && jA >= (CBS << 3) && limA > CBS, pushB = actB && jB >= (CBS << 3) && limB > CBS;
        const uint64_t pmA = __ballot(pushA), pmB = __ballot(pushB);
#pragma nounroll
        for (uint32_t h = 0; h < 2; h++) {   // (one call site of ext_queue)
            const uint64_t pm = h ? pmB : pmA;
            const uint32_t npx = (uint32_t)__popcll(pm);
            if (qn + npx > 64 || (!more && qn)) {
                const uint64_t td0 = stamp ? __builtin_amdgcn_s_memtime() : 0;
                ext_queue<DICT, false>(L, bn, KK, Qw, qn, lane, hbk);
                if (stamp) tdef += __builtin_amdgcn_s_memtime() - td0;
                qn = 0;
            }
            if (!more) break;
            const bool p = h ? pushB : pushA;
            if (p) lds_st(&Qw[qn + (uint32_t)__popcll(pm & lt)], (h ? kb : ka) | ((8u - ((h ? jB : jA) & 7u)) << 15));
            qn += npx;
        }
        if (!more) break;
        uint32_t nib = 0;
        if (actA && !pushA) nib |= short_result<DICT>(L, ka, iA, jA, hbk) << ((ka & 7u) << 2);
        if (actB && !pushB) nib |= short_result<DICT>(L, kb, iB, jB, hbk) << ((kb & 7u) << 2);
        if (nib) atomicOr(&nib_words(L)[ka >> 3], nib);
    }
    return iters;
}

// ---- Short chains K = 6..8, four entries per lane (round 6) --------------------------------
// Lane l holds the consecutive entries E_r = 4l' + r (r = 0..3, l' = l - HQ) of S; the HQ = 2
// lanes below the owned ones are the halo (8 entries: K <= 8).  Candidate j of E_r is E_r' of
// lane l - s with 4s + r - r' = j: s = 0 (r' < r: the same lane, no move), s = 1 (every stream
// moved down one lane) and s = 2 (the streams r' >= 8 - K moved a second lane).  Per chunk
// 4 (64 - HQ) = 248 entries: half the stream moves per compare of the two-entry path (one DPP
// move per two compares), and the chunk's bookkeeping (claim, loads, sort check, limits, queue)
// spread over twice the entries.  Same keys, queue and results as search_pairs.
#define HQ 2
template <int KK, int S, int R, int RP, bool GEN, bool GUARD, bool CLAMP>
__device__ __forceinline__ void qcmp(const uint32_t (&e)[8], const uint32_t (&c)[8], uint32_t (&key)[4],
                                     const uint32_t (&nc)[4], const uint32_t (&lim)[4]) {
    constexpr int J = 4 * S + R - RP;
    if constexpr (J >= 1 && J <= KK) {
        uint32_t t;
        if constexpr (GEN) t = pkey_g<GUARD, CLAMP>(e[2 * R], e[2 * R + 1], c[2 * RP], c[2 * RP + 1], J, nc[R], lim[R]);
        else t = pkey<8 - J>(e[2 * R], e[2 * R + 1], c[2 * RP], c[2 * RP + 1]);
        key[R] = max(key[R], t);
    }
}
template <int KK, int S, int I, bool GEN, bool GUARD, bool CLAMP>
__device__ __forceinline__ void qrow(const uint32_t (&e)[8], const uint32_t (&c)[8], uint32_t (&key)[4],
                                     const uint32_t (&nc)[4], const uint32_t (&lim)[4]) {
    if constexpr (I < 16) {
        qcmp<KK, S, I / 4, I % 4, GEN, GUARD, CLAMP>(e, c, key, nc, lim);
        qrow<KK, S, I + 1, GEN, GUARD, CLAMP>(e, c, key, nc, lim);
    }
}
template <int KK, bool GEN, bool GUARD, bool CLAMP>
__device__ __forceinline__ void quad_steps(const uint32_t (&e)[8], uint32_t (&key)[4], const uint32_t (&nc)[4],
                                           const uint32_t (&lim)[4]) {
    qrow<KK, 0, 0, GEN, GUARD, CLAMP>(e, e, key, nc, lim);   // s = 0: the lane's own earlier entries
    uint32_t c[8];
#pragma unroll
    for (int q = 0; q < 8; q++) c[q] = PSHR(e[q]);
    qrow<KK, 1, 0, GEN, GUARD, CLAMP>(e, c, key, nc, lim);
#pragma unroll
    for (int q = 2 * (8 - KK); q < 8; q++) c[q] = PSHR(c[q]);   // (streams r' < 8 - K are not used at s = 2)
    qrow<KK, 2, 0, GEN, GUARD, CLAMP>(e, c, key, nc, lim);
}
template <bool DICT, int KK>
__device__ __forceinline__ uint32_t search_quads(MatchLDS& L, uint32_t bn, uint32_t tid, bool stamp, uint64_t& tdef,
                                                 const uint32_t* __restrict__ hbk) {
    static_assert(KK >= 5 && KK <= 8, "four entries per lane with a halo of two lanes: K = 5..8");
    constexpr uint32_t OWN = 4 * (64 - HQ);
    const uint32_t lane = tid & 63, wave = wave_of(tid);
    const uint32_t nvalid = bn > 2 ? bn - 2 : 0;
#ifndef DMX_QSLOTS
    // the extension queue: a ring of 128 items per wave over tsm + exitp (both free during the
    // search, adjacent in MatchLDS): a chunk's items go in at once, batches of 64 come out
    uint32_t* Qw = L.tsm + (wave << 7);
    uint32_t qh = 0;   // ring head (wave-uniform)
#else
    uint32_t* Qw = L.tsm + (wave << 6);   // the extension queue (P2 arrays are free during the search)
#endif
    const uint64_t lt = (1ull << lane) - 1ull;
    uint32_t qn = 0, iters = 0;
    uint32_t cnext = wave_claim(&L.ntok);   // chunks from the workgroup counter, one ahead (search_pairs)
    for (;;) {
        const uint32_t base = (uint32_t)__builtin_amdgcn_readfirstlane((int)cnext) * OWN;
        const bool more = base < nvalid;   // wave-uniform
        if (more) cnext = wave_claim(&L.ntok);
        const int ea = (int)base + 4 * ((int)lane - (int)HQ);
        const uint32_t k0 = (uint32_t)ea;
        const bool own = lane >= HQ;
        bool act[4];
#pragma unroll
        for (int r = 0; r < 4; r++) act[r] = more && own && k0 + (uint32_t)r < nvalid;
        uint32_t key[4] = {0, 0, 0, 0}, lim[4] = {0, 0, 0, 0}, pos[4] = {0, 0, 0, 0};
        if (more) {
            uint32_t e[8];
            {   // the four positions in one aligned 8-byte LDS word, then their first 8 bytes
                uint2 pr = make_uint2(0, 0);
                if (ea >= 0 && k0 < nvalid) pr = reinterpret_cast<const uint2*>(L.sorted)[k0 >> 2];
                pos[0] = pr.x & 0xFFFFu; pos[1] = pr.x >> 16; pos[2] = pr.y & 0xFFFFu; pos[3] = pr.y >> 16;
#pragma unroll
                for (int r = 0; r < 4; r++) {
                    if (!(k0 + (uint32_t)r < nvalid)) pos[r] = 0;   // (past the last entry: never a candidate)
                    const uint64_t v = ld8(L.data, pos[r]);
                    e[2 * r] = (uint32_t)v;
                    e[2 * r + 1] = (uint32_t)(v >> 32);
                }
            }
#pragma unroll
            for (int r = 0; r < 4; r++)
                if (act[r]) lim[r] = (bn - pos[r]) < MAXLEN ? (bn - pos[r]) : MAXLEN;
            iters += 4 * KK;
            {   // sort check: E_0 after E_3 of the lane below, E_r after E_(r-1)
                uint32_t sk[4];
#pragma unroll
                for (int r = 0; r < 4; r++) sk[r] = sort_key(e[2 * r], pos[r]);
                const uint32_t pk = PSHR(sk[3]);
                bool bad = act[0] && k0 >= 1 && pk > sk[0];
#pragma unroll
                for (int r = 1; r < 4; r++) bad = bad || (act[r] && sk[r - 1] > sk[r]);
#ifndef DMX_KO_SORTCHK   // timing knockout: no sort check
                if (__ballot(bad)) L.sortbad = 1;
#else
                (void)bad;
#endif
            }
            if (base == 0) {
                uint32_t nc[4];
#pragma unroll
                for (int r = 0; r < 4; r++) nc[r] = min(k0 + (uint32_t)r, (uint32_t)KK);
                quad_steps<KK, true, true, true>(e, key, nc, lim);
            } else if (__ballot((act[0] && lim[0] < CBS) || (act[1] && lim[1] < CBS) || (act[2] && lim[2] < CBS) ||
                                (act[3] && lim[3] < CBS))) {
                const uint32_t nc[4] = {KK, KK, KK, KK};
                quad_steps<KK, true, false, true>(e, key, nc, lim);
            } else {
                const uint32_t nc[4] = {0, 0, 0, 0};
                quad_steps<KK, false, false, false>(e, key, nc, lim);
            }
        }
        // a candidate equal in all CBS bytes (key >= 64): the entry is queued for the LDS
        // extension (unless the block end caps it there); E_0's items, then E_1's, ...
#ifndef DMX_QSLOTS
        bool push[4];
        uint64_t pmv[4];
        uint32_t npr[4];
#pragma unroll
        for (int r = 0; r < 4; r++) {
#ifdef DMX_KO_QUEUE   // timing knockout (wrong output): no queued extension
            push[r] = false;
#else
            push[r] = act[r] && key[r] >= (CBS << 3) && lim[r] > CBS;
#endif
            pmv[r] = __ballot(push[r]);
            npr[r] = (uint32_t)__popcll(pmv[r]);
        }
        const uint32_t npt = npr[0] + npr[1] + npr[2] + npr[3];
        // appends: all four slots at once when they fit the ring (the usual case), else one slot
        // at a time; batches of 64 leave whenever 64 are in (all of them at the end).  One call
        // site of ext_queue (code size, registers)
        uint32_t rs = (qn + npt <= 128u) ? 4u : 0u;   // next append: slot rs, 4 = all, 5 = done
        if (npt || (!more && qn)) {
#pragma nounroll
            for (;;) {
                const uint32_t want = rs == 4u ? npt : rs < 4u ? (rs == 0 ? npr[0] : rs == 1 ? npr[1] : rs == 2 ? npr[2] : npr[3]) : 0u;
                if (qn >= 64u || (qn && (!more || qn + want > 128u))) {
                    const uint32_t nq = qn < 64u ? qn : 64u;
                    const uint64_t td0 = stamp ? __builtin_amdgcn_s_memtime() : 0;
                    ext_queue<DICT, false>(L, bn, KK, Qw, nq, lane, hbk, qh, 127u);
                    if (stamp) tdef += __builtin_amdgcn_s_memtime() - td0;
                    qh += nq;
                    qn -= nq;
                    continue;
                }
                if (!more || rs == 5u) break;
                uint32_t off = 0;
#pragma unroll
                for (uint32_t r = 0; r < 4; r++) {
                    if (rs == 4u || rs == r) {
                        if (push[r])
                            lds_st(&Qw[(qh + qn + off + (uint32_t)__popcll(pmv[r] & lt)) & 127u],
                                   (k0 + r) | ((8u - (key[r] & 7u)) << 15));
                        off += npr[r];
                    }
                }
                qn += want;
                rs = rs >= 3u ? 5u : rs + 1u;
            }
        }
#else
        bool push[4];
        uint64_t pmv[4];
        uint32_t pbits = 0, jbits = 0;   // per slot r: push flag (bit r), the key's 8 - j (bits 3r + 2 .. 3r)
#pragma unroll
        for (int r = 0; r < 4; r++) {
#ifdef DMX_KO_QUEUE   // timing knockout (wrong output): no queued extension
            push[r] = false;
#else
            push[r] = act[r] && key[r] >= (CBS << 3) && lim[r] > CBS;
#endif
            pmv[r] = __ballot(push[r]);
            pbits |= push[r] ? 1u << r : 0u;
            jbits |= (key[r] & 7u) << (3 * r);
        }
        const uint32_t npt = (uint32_t)(__popcll(pmv[0]) + __popcll(pmv[1]) + __popcll(pmv[2]) + __popcll(pmv[3]));
        if (npt || (!more && qn)) {
#pragma nounroll
            for (uint32_t h = 0; h < 4; h++) {   // (one call site of ext_queue)
                const uint64_t pm = h == 0 ? pmv[0] : h == 1 ? pmv[1] : h == 2 ? pmv[2] : pmv[3];   // (scalar selects)
                const uint32_t npx = (uint32_t)__popcll(pm);
                if (qn + npx > 64 || (!more && qn)) {
                    const uint64_t td0 = stamp ? __builtin_amdgcn_s_memtime() : 0;
                    ext_queue<DICT, false>(L, bn, KK, Qw, qn, lane, hbk);
                    if (stamp) tdef += __builtin_amdgcn_s_memtime() - td0;
                    qn = 0;
                }
                if (!more) break;
                if ((pbits >> h) & 1u)
                    lds_st(&Qw[qn + (uint32_t)__popcll(pm & lt)], (k0 + h) | ((8u - ((jbits >> (3 * h)) & 7u)) << 15));
                qn += npx;
            }
        }
#endif
        if (!more) break;
        uint32_t nib = 0;
#pragma unroll
        for (int r = 0; r < 4; r++)
            if (act[r] && !push[r])
                nib |= short_result<DICT>(L, k0 + (uint32_t)r, pos[r], key[r], hbk) << (((k0 + (uint32_t)r) & 7u) << 2);
        if (nib) atomicOr(&nib_words(L)[k0 >> 3], nib);
    }
    return iters;
}

template <bool DICT, bool RUNS, int NB = 3>
__device__ __forceinline__ uint32_t search_positions(MatchLDS& L, uint32_t bn, int32_t max_chain, uint16_t* __restrict__ pg,
                                     uint32_t tid, bool stamp, uint64_t& tdef, const uint32_t* __restrict__ hbk,
                                     const uint16_t* __restrict__ seeds = nullptr) {
    constexpr bool H4 = NB > 3;   // NB-byte chains seeded with the shorter matches (P0')
    const uint32_t lane = tid & 63, wave = wave_of(tid);
    const uint32_t K = max_chain > 0 ? (uint32_t)max_chain : 0xFFFFFFFFu;
    const uint32_t nvalid = bn > 2 ? bn - 2 : 0;   // positions with a full trigram = entries of S
    uint32_t iters = 0;
    if (RUNS) build_chg(L, bn, tid);
#ifndef DMX_NO_PAIRS
    if (!RUNS && NB == 3 && K >= 6 && K <= 8) {
#ifndef DMX_PAIRS   // four entries per lane (search_quads; DMX_PAIRS: the round-5 two-entry path)
        iters = K == 8 ? search_quads<DICT, 8>(L, bn, tid, stamp, tdef, hbk)
              : K == 7 ? search_quads<DICT, 7>(L, bn, tid, stamp, tdef, hbk)
                       : search_quads<DICT, 6>(L, bn, tid, stamp, tdef, hbk);
#else   // two entries per lane (search_pairs)
        iters = K == 8 ? search_pairs<DICT, 8>(L, bn, tid, stamp, tdef, hbk)
              : K == 7 ? search_pairs<DICT, 7>(L, bn, tid, stamp, tdef, hbk)
                       : search_pairs<DICT, 6>(L, bn, tid, stamp, tdef, hbk);
#endif
    } else
#endif
    if (K <= KE) {
        // bounded mode with a short chain: chunks of 64-K owned entries, halo embedded.
        // Entries with a candidate equal in all CBS register bytes need the LDS extension; they
        // go to a per-wave queue (up to 64, in tsm) that is extended with all 64 lanes at once
        // when the next chunk would overflow it, instead of a few lanes of every chunk.
        uint32_t* Qw = L.tsm + (wave << 6);
        const uint64_t lt = (1ull << lane) - 1ull;
        uint32_t qn = 0;   // queued entries (wave-uniform)
        const uint32_t own = 64 - K;
        // one call site of ext_queue (code size, registers): the pass after the last chunk
        // only flushes the queue
        // chunks from the workgroup counter (L.ntok, zeroed before the search), as search_pairs
        uint32_t cnext = wave_claim(&L.ntok);
        for (;;) {
            const uint32_t base = (uint32_t)__builtin_amdgcn_readfirstlane((int)cnext) * own;
            const bool more = base < nvalid;   // wave-uniform
            if (more) cnext = wave_claim(&L.ntok);
            const int ei = (int)(base + lane) - (int)K;   // entry of this lane
            const uint32_t k = (uint32_t)ei;
            const bool act = more && lane >= K && k < nvalid;
            uint32_t i = 0, lim_eff = 0, jkey = 0;
            bool done = false;   // result already stored (runs)
            if (more) {
                const bool load = ei >= 0 && k < nvalid;
                uint32_t nc = 0;
                uint64_t iv0 = 0;
                if (load) {
                    i = L.sorted[k];
                    iv0 = ld8(L.data, i);
                }
                if (act) {
                    nc = min(k, K);
                    lim_eff = (bn - i) < MAXLEN ? (bn - i) : MAXLEN;
                }
                iters += K;
                const uint32_t i0 = (uint32_t)iv0, i1 = (uint32_t)(iv0 >> 32);
                {   // sort check: the predecessor entry (lane - 1) has a smaller (bucket, position)
                    const uint32_t sk = sort_key(i0, i);
                    const uint32_t pk = (uint32_t)__builtin_amdgcn_update_dpp(0, (int)sk, 0x138, 0xF, 0xF, true);
                    if (__ballot(act && ei >= 1 && pk > sk)) L.sortbad = 1;
                }
                bool skip = false;
                if (RUNS) {
                    // inside a run: when the distance-1 match already has the longest possible
                    // length, it is the answer (entry k-1 is position i-1 -- same trigram, so the
                    // same bucket, and no position lies between them -- and nearest wins ties).
                    // A chunk whose lanes all end here skips the candidate steps.
                    const bool rdone = act && i >= 1 && run_len(L, i, lim_eff) >= lim_eff;
                    if (__ballot(act && !rdone) == 0) {
                        if (act) store_short<DICT>(L, k, i, lim_eff, 1u, hbk);
                        done = true;
                        skip = true;
                    }
                }
                if (!skip) {
                    if (base == 0) cand_steps_emb<true, true>(K, i0, i1, nc, lim_eff, jkey);
                    else if (__ballot(act && lim_eff < CBS)) cand_steps_emb<false, true>(K, i0, i1, nc, lim_eff, jkey);
                    else if (K == 6) cand_steps_fixed<6>(i0, i1, jkey);
                    else if (K == 8) cand_steps_fixed<8>(i0, i1, jkey);
                    else if (K == 7) cand_steps_fixed<7>(i0, i1, jkey);
                    else if (K == 4) cand_steps_fixed<4>(i0, i1, jkey);
                    else cand_steps_emb<false, false>(K, i0, i1, nc, lim_eff, jkey);
                }
            }
            // a candidate equal in all CBS bytes (key >= 64) is the register best: the entry
            // is queued for the LDS extension (unless the block end caps it there)
            const bool push = act && !done && jkey >= (CBS << 3) && lim_eff > CBS;
            const uint64_t pm = __ballot(push);
            const uint32_t np = (uint32_t)__popcll(pm);
            if (qn + np > 64 || (!more && qn)) {
                const uint64_t td0 = stamp ? __builtin_amdgcn_s_memtime() : 0;
                ext_queue<DICT, RUNS>(L, bn, K, Qw, qn, lane, hbk);
                if (stamp) tdef += __builtin_amdgcn_s_memtime() - td0;
                qn = 0;
            }
            if (!more) break;
            if (push) lds_st(&Qw[qn + (uint32_t)__popcll(pm & lt)], k | ((8u - (jkey & 7u)) << 15));
            qn += np;
            if (act && !push && !done) {
                const uint32_t m = jkey >> 3;
                store_short<DICT>(L, k, i, m >= 3 ? m : 0u, m >= 3 ? 8u - (jkey & 7u) : 0u, hbk);
            }
        }
    } else
    // Longer chains (K > KE, exhaustive mode): chunks of 64 entries; lane 0 is fed from a halo
    // of the entries below the window (lane l holds entry k0 - 1 - jb - l), reloaded per
    // window.  Window 0 (the W0 = 8 nearest candidates; all of them for a bounded K <= KD):
    // 12-byte register streams, the window's best into the position-form key (len << 15 | q:
    // longest, then nearest), and its candidates equal in all 12 register bytes extended from
    // LDS (resolve_full).  Later windows of KD = 32 candidates: the byte-at-best filter below.
    // A lane needs more windows while its chain goes on and its best is short of
    // min(258, bn - i); the wave stops when no lane does.
    {
    // H4: the seeds (HBM) of the wave's next chunk are loaded one chunk ahead
    // chunks of 64 entries from the workgroup counter (L.ntok, zeroed before the search): a
    // chunk's chains cost anything from one window to hundreds, so a fixed share per wave left
    // the waves idling at the end of the phase; the next chunk (and its seeds) is fetched a
    // chunk ahead
    uint32_t cnx = wave_claim(&L.ntok);
    uint32_t c0 = (uint32_t)__builtin_amdgcn_readfirstlane((int)cnx);
    uint32_t snext = 0xFFFFu;   // (a 16-bit seed: none)
    if (H4 && (c0 << 6) + lane < nvalid) snext = seeds[L.sorted[(c0 << 6) + lane]];   // (raw: decoded at use)
    for (;;) {
        const uint32_t k0 = c0 << 6;
        if (k0 >= nvalid) break;
        cnx = wave_claim(&L.ntok);
        const uint32_t c1 = (uint32_t)__builtin_amdgcn_readfirstlane((int)cnx);
        const uint32_t k = k0 + lane;
        const bool act = k < nvalid;
        uint32_t i = 0, nc = 0, lim = 0;
        uint32_t seed = 0;
        if (H4) {
            seed = seed_dec(snext);
            if ((c1 << 6) + lane < nvalid) snext = seeds[L.sorted[(c1 << 6) + lane]];
        }
        uint64_t iv0 = 0;
        uint32_t i2 = 0;
        if (act) {
            i = L.sorted[k];
            uint32_t a0, a1;
            ld12(L.data, i, a0, a1, i2);
            iv0 = (uint64_t)a0 | ((uint64_t)a1 << 32);
            // bounded mode (K <= KD) needs no bucket rank: the K entries below k are examined
            // and those of other buckets never reach 3 equal bytes (cand_steps); only the
            // first K entries of the block lack K predecessors.  Longer chains need the rank.
            nc = K <= KD ? min(k, K) : min(k - (uint32_t)L.bstart[bucket_of<NB>(iv0)], K);
            lim = (bn - i) < MAXLEN ? (bn - i) : MAXLEN;
        }
        const uint32_t i0 = (uint32_t)iv0, i1 = (uint32_t)(iv0 >> 32);
        const uint32_t lim_eff = act ? lim : 0;
        const uint8_t* D8 = reinterpret_cast<const uint8_t*>(L.data);
        uint32_t bestkey = 0;
        if (H4 && act) bestkey = seed;   // the best match shorter than NB (P0', in HBM)
        constexpr uint32_t W0X = H4 ? DMX_W0H4 : W0;
        for (uint32_t jb = 0, wl = K <= KD ? KD : W0X;; jb += wl, wl = KD) {   // (bounded K <= KD: all in registers)
            // lanes that still need candidates jb + 1 ...: wave-uniform window length (window
            // 0: the W0 nearest candidates, by the register compare; then windows of KD)
            uint32_t need = (act && nc > jb && (bestkey >> 15) < lim) ? min(nc - jb, wl) : 0u;
            need = max(need, dpp_shr(need, 1));
            need = max(need, dpp_shr(need, 2));
            need = max(need, dpp_shr(need, 4));
            need = max(need, dpp_shr(need, 8));
            const uint32_t jmax = max(max(__builtin_amdgcn_readlane(need, 15), __builtin_amdgcn_readlane(need, 31)),
                                      max(__builtin_amdgcn_readlane(need, 47), __builtin_amdgcn_readlane(need, 63)));
            if (jmax == 0) break;
            iters += jmax;
            // halo of this window: lane l < KD holds entry k0 - 1 - jb - l (its bytes too in window 0)
            uint32_t hq = 0;
            uint64_t hv0 = 0;
            uint32_t h2 = 0;
            if (lane < KD && k0 >= jb + lane + 1) {
                hq = L.sorted[k0 - 1 - jb - lane];
                if (jb == 0) {
                    uint32_t a0, a1;
                    ld12(L.data, hq, a0, a1, h2);
                    hv0 = (uint64_t)a0 | ((uint64_t)a1 << 32);
                }
            }
            // lanes without a candidate j of this window: halo lanes before the block start
            // (k0 < jb + wl), or a bounded chain ending inside a later window (a bounded
            // K <= KD has a single window, at most K steps long, and needs no mask)
            const uint32_t ncw = nc > jb ? nc - jb : 0u;
            // H4: an entry before the bucket start can still share the trigram (3 bytes, from
            // any position, later ones too), so 4-byte chains are always masked at their end
            const bool guard = H4 || k0 < jb + wl || (K > W0 && K < jb + wl);
            if (jb == 0) {
                const uint32_t h0 = (uint32_t)hv0, h1 = (uint32_t)(hv0 >> 32);
                {   // sort check: the predecessor (lane - 1, lane 0: halo 0) has a smaller (bucket, position)
                    const uint32_t sk = sort_key_h<NB>(iv0, i);
                    const uint32_t pk = wshr(sk, __builtin_amdgcn_readlane(sort_key_h<NB>(hv0, hq), 0));
                    if (__ballot(act && k >= 1 && pk > sk)) L.sortbad = 1;
                }
                uint32_t x0 = i0, x1 = i1, x2 = i2;   // the candidate streams
                uint32_t jkey = 0, full = 0;   // full: bit j-1 = candidate j matches all CB bytes
                if (guard) cand_steps<true>(jmax, x0, x1, x2, i0, i1, i2, h0, h1, h2, ncw, lim_eff, jkey, full);
                else cand_steps<false>(jmax, x0, x1, x2, i0, i1, i2, h0, h1, h2, ncw, lim_eff, jkey, full);
                if (lim_eff <= CB) full = 0;
                // the window's register best in position form
                if (act && (jkey >> 8) >= 3)
                    bestkey = max(bestkey, ((jkey >> 8) << 15) | (uint32_t)L.sorted[k - (255u - (jkey & 255u))]);
                const uint64_t td0 = stamp ? __builtin_amdgcn_s_memtime() : 0;
                bestkey = resolve_full<false, false>(L, bn, lane, wave, k, i, lim_eff, bestkey, full, k0);
                if (stamp) tdef += __builtin_amdgcn_s_memtime() - td0;
            } else {
                // Later windows: a candidate farther than all those seen can only win if it is
                // strictly longer than the current best b, so it must equal bytes [0, b] -- in
                // particular the four ending at offset b (the first three while b < 3).  Only
                // the candidates' positions stream through the lanes (the halo holds positions
                // only); each step reads those four bytes of every lane's candidate from LDS
                // (two aligned dwords), and the rare survivors (1 % on text with two bytes, 5 %
                // with one) are kept in a mask and get their exact length from LDS after the
                // window, nearest first.
                const uint32_t bl0 = bestkey >> 15;
                const bool live = act && nc > jb && bl0 < lim;
                // bytes [s, s + 4), s = max(b, 3) - 3, must match (byte s + 3 only when b >= 3)
                const uint32_t s0 = max(bl0, 3u) - 3u, msk = bl0 >= 3 ? 0xFFFFFFFFu : 0x00FFFFFFu;
                const uint32_t ob = live ? ld4(L.data, i + s0) & msk : 0xFFFFFFFFu;
                const uint32_t omsk = live ? msk : 0u;   // lanes without work never survive
                uint32_t xp = (uint32_t)L.sorted[k - min(jb, k)];          // lane l: entry k - jb
                uint32_t surv = 0;
                // XU steps at a time: the positions by XU wave shifts, then all their LDS reads
                // in flight before the compares (one step at a time waited on every read)
                const uint32_t jlim = guard ? 0u : 0xFFFFFFFFu;   // guard: j <= ncw
                for (uint32_t j = 1; j <= jmax; j += XU) {
                    uint32_t xs[XU], v[XU];
#pragma unroll
                    for (uint32_t u = 0; u < XU; u++) {
                        xp = wshr(xp, __builtin_amdgcn_readlane(hq, (int)min(j + u - 1, (uint32_t)KD - 1)));
                        xs[u] = xp + s0;
                    }
#pragma unroll
                    for (uint32_t u = 0; u < XU; u++) v[u] = ld4(L.data, xs[u]);
#pragma unroll
                    for (uint32_t u = 0; u < XU; u++) {
                        const uint32_t jj = j + u;
                        surv |= ((v[u] & omsk) == ob && jj <= jmax && jj <= max(ncw, jlim)) ? 1u << (jj - 1) : 0u;
                    }
                }
                const uint64_t td0 = stamp ? __builtin_amdgcn_s_memtime() : 0;
                while (surv) {   // nearest first; a candidate of another bucket cannot reach 3 bytes
                    const uint32_t j = (uint32_t)__builtin_ctz(surv) + 1u;
                    surv &= surv - 1u;
                    const uint32_t bl = bestkey >> 15;
                    if (bl >= lim) break;
                    const uint32_t q = L.sorted[k - jb - j], tt = max(bl, 2u);
                    if (D8[q + tt] != D8[i + tt]) continue;
                    const uint32_t len = min(ext_len(L, i, q, 0, lim), lim);
                    if (len >= 3) bestkey = max(bestkey, (len << 15) | q);
                }
                if (stamp) tdef += __builtin_amdgcn_s_memtime() - td0;
            }
        }
        if (act) store_result<DICT>(L, pg, k, i, bestkey, hbk);
        c0 = c1;
    }
    }
    // the last two positions have no trigram: literals
    if (tid < 2 && bn >= 1 + tid) {
        const uint32_t p = bn - 1 - tid;
        atomicOr(&L.lit[p >> 5], 1u << (p & 31));
        L.len8[p] = 0;
    }
    return iters;
}

// Resolve segment s (positions [32s, 32s+32)) for a path entering at e >= 32s, against the
// path word m of that segment: if the walk from e meets one of m's positions the rest
// coincides (the next-function is deterministic).  Scalar code: every input is uniform.
__device__ __forceinline__ uint32_t resolve_word(const MatchLDS& L, uint32_t lo, uint32_t e, uint32_t bn, uint32_t m,
                                                 uint32_t lw, uint32_t x, uint32_t& nm_out, bool& merged) {
    merged = false;
    if (e >= lo + 32 || e >= bn) { nm_out = 0; return e; }
    uint32_t nm = 0, p = e;
    while (p < lo + 32 && p < bn) {
#ifndef DMX_WALK_STEP
        // a run of literals in one step (their bits in lw, up to the segment end or bn): every
        // position of it is a token start; no LDS read
        const uint32_t sh = p - lo;
        const uint32_t run = min(ffbl_hw(~(lw >> sh)), min(lo + 32u, bn) - p);   // (lit bits past bn may be set by P1b)
        if (run) {
            const uint32_t rm = (run >= 32u ? ~0u : ((1u << run) - 1u)) << sh;
            if (m & rm) {
                const uint32_t bb = ffbl_hw(m & rm), below = (1u << bb) - 1u;   // the first shared position
                nm_out = nm | (rm & below) | (m & ~below);
                merged = true;
                return x;
            }
            nm |= rm;
            p += run;
            continue;
        }
        const uint32_t bit = 1u << sh;
        if (m & bit) { nm_out = nm | (m & ~(bit - 1u)); merged = true; return x; }
        nm |= bit;
        p += (uint32_t)L.len8[p] + 3u;
#else
        const uint32_t bit = 1u << (p - lo);
        if (m & bit) { nm_out = nm | (m & ~(bit - 1u)); merged = true; return x; }
        nm |= bit;
        p += ((lw >> (p - lo)) & 1u) ? 1u : (uint32_t)L.len8[p] + 3u;
#endif
    }
    nm_out = nm;
    return p;
}

// Lanes of the wave holding the same value v as this lane (among the valid lanes): every
// lane ORs its bit into the wave's slot G[v] and reads the slot back (LDS executes a wave's
// instructions in order, so the read sees all ORs), then the slot is cleared for reuse.
// 3 LDS instructions instead of one ballot per bit of v.
__device__ __forceinline__ uint64_t group_of(unsigned long long* G, uint32_t v, bool valid) {
    const uint64_t vm = __ballot(valid);
    if (vm == 0) return 0;
    const uint32_t v0 = __builtin_amdgcn_readlane(v, (int)__builtin_ctzll(vm));
    if (__ballot(valid && v != v0) == 0) return valid ? vm : 0;   // one group (runs): no LDS traffic
    uint64_t eq = 0;
    if (valid) {
        __hip_atomic_fetch_or(&G[v], 1ull << (threadIdx.x & 63), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
        eq = __hip_atomic_load(&G[v], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
        __hip_atomic_store(&G[v], 0ull, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
    }
    return eq;
}

// T[v] += 1 for every valid lane (pair16: T holds two u16 counters per word); a single
// add when the valid lanes share v (runs), instead of a 64-way conflicting LDS atomic.
template <bool RUNCHK = true>
__device__ __forceinline__ void count_add(uint32_t* T, uint32_t v, bool valid, bool pair16) {
    if (!RUNCHK) {   // blocks that are not run-dominated: lanes rarely share v
        if (valid) {
            if (pair16) atomicAdd(&T[v >> 1], 1u << (16 * (v & 1)));
            else atomicAdd(&T[v], 1u);
        }
        return;
    }
    const uint64_t vm = __ballot(valid);
    if (vm == 0) return;
    const uint32_t first = (uint32_t)__builtin_ctzll(vm);
    const uint32_t v0 = __builtin_amdgcn_readlane(v, (int)first);
    if (__ballot(valid && v != v0) == 0) {
        if ((threadIdx.x & 63) == first) {
            const uint32_t c = (uint32_t)__popcll(vm);
            if (pair16) atomicAdd(&T[v0 >> 1], c << (16 * (v0 & 1)));
            else atomicAdd(&T[v0], c);
        }
    } else if (valid) {
        if (pair16) atomicAdd(&T[v >> 1], 1u << (16 * (v & 1)));
        else atomicAdd(&T[v], 1u);
    }
}

// Stable rank in T[v] (a running destination): the old value of an LDS atomicAdd, which
// same-address lanes of one instruction get in lane order on gfx950 (verified at run time
// by the search, see sort_positions).  A step whose valid lanes share v (runs) takes one
// add of the group size instead of a 64-way conflicting atomic.
template <bool RUNCHK = true>
__device__ __forceinline__ uint32_t atomic_rank(uint32_t* T, uint32_t v, bool valid, uint64_t lt) {
    if (!RUNCHK) return valid ? atomicAdd(&T[v], 1u) : 0u;
    const uint64_t vm = __ballot(valid);
    if (vm == 0) return 0;
    const uint32_t first = (uint32_t)__builtin_ctzll(vm);
    const uint32_t v0 = __builtin_amdgcn_readlane(v, (int)first);
    if (__ballot(valid && v != v0) == 0) {
        uint32_t base = 0;
        if ((threadIdx.x & 63) == first) base = atomicAdd(&T[v0], (uint32_t)__popcll(vm));
        return __builtin_amdgcn_readlane(base, (int)first) + (uint32_t)__popcll(vm & lt);
    }
    return valid ? atomicAdd(&T[v], 1u) : 0u;
}

// Exclusive prefix sum over the 1024 threads of the workgroup (all threads call it).
__device__ __forceinline__ uint32_t block_excl_scan(MatchLDS& L, uint32_t v, uint32_t tid) {
    const uint32_t incl = wave_incl_scan(v);
    if ((tid & 63) == 63) L.wsum[tid >> 6] = incl;
    __syncthreads();
    uint32_t base = 0;
    for (uint32_t w = 0; w < (tid >> 6); w++) base += L.wsum[w];
    __syncthreads();
    return base + incl - v;
}

// Rank in the 16-bit field at bit sh of T[v] (a pair of counters per word): the old field of
// an LDS atomicAdd of 1 << sh, which same-address lanes of one instruction get in lane order
// (checked at run time, see count_sort_positions).  A step whose valid lanes share v (runs)
// takes one add of the group size instead of a 64-way same-address atomic.
template <bool RUNCHK>
__device__ __forceinline__ uint32_t atomic_rank16(uint32_t* T, uint32_t v, bool valid, uint64_t lt, uint32_t sh) {
    if (RUNCHK) {
        const uint64_t vm = __ballot(valid);
        if (vm == 0) return 0;
        const uint32_t first = (uint32_t)__builtin_ctzll(vm);
        const uint32_t v0 = __builtin_amdgcn_readlane(v, (int)first);
        if (__ballot(valid && v != v0) == 0) {
            uint32_t base = 0;
            if ((threadIdx.x & 63) == first) base = atomicAdd(&T[v0], (uint32_t)__popcll(vm) << sh);
            return ((__builtin_amdgcn_readlane(base, (int)first) >> sh) & 0xFFFFu) + (uint32_t)__popcll(vm & lt);
        }
    }
    // every lane adds (0 when invalid; v = 0 then): no exec-masked branch per step, so the
    // 32 steps of a round issue their atomics back to back instead of one round trip each
    return (atomicAdd(&T[v], valid ? 1u << sh : 0u) >> sh) & 0xFFFFu;
}

// Bucket-sorted positions S (stable by position inside a bucket) by ONE counting pass over
// the 13-bit bucket (round 5; the two-pass LSD sort below stays as the checked fallback).
// The block's positions form four groups of 8192 (g = w >> 2 for wave w; round 6: two groups
// of 16384 until round 5, -DDMX_SORT_G2); T[h] (in len8) holds the counts of bucket h of groups
// 0 and 1 in its low and high 16 bits, T2[h] (in S's first half, free until the scatter)
// those of groups 2 and 3.
//  1. every wave hashes its 2048 positions [2048w, 2048w + 2048) into registers;
//  2. four rounds, one wave of each group per round (wave w in round w & 3), separated by
//     barriers: the wave adds 1 << 16 (g & 1) to its group's word of bucket h for its 32
//     steps of 64 positions and keeps the old field as the entry's rank.  Inside a round a
//     wave's LDS instructions execute in order and same-address lanes of one instruction in
//     lane order; the rounds run in position order, so the rank of every entry is the number
//     of earlier positions of its bucket in its group -- the stable order (four waves at a
//     time: half the rounds and barriers of two groups, the same atomics);
//  3. one scan over the 8192 buckets: each group's field := the first slot of its run
//     (start(h), + count0, + count1, + count2; start(h) is the bucket start long chains need);
//  4. every wave reads its entries' destinations (field + rank), a barrier (S's first half
//     held counters), then stores them, no atomics.
// One rank atomic per entry instead of the LSD sort's two (plus its second count), and the
// scatter is plain stores.  The search checks every adjacent pair of S (sortbad), so a lane
// order violation can never go unnoticed: the block then re-sorts with the match-any path.
template <bool RUNCHK, int NB>
__device__ __forceinline__ void count_sort_positions(MatchLDS& L, uint32_t bn, int32_t max_chain, uint32_t tid,
                                                     bool stamp, uint64_t* tp0) {
    const uint32_t lane = tid & 63, wave = wave_of(tid);
    const uint32_t nvalid = bn > 2 ? bn - 2 : 0;   // positions with a full trigram
    const bool need_starts = max_chain <= 0 || max_chain > KD;
    uint32_t* T = reinterpret_cast<uint32_t*>(L.len8);   // 8192 counter pairs (len8 is free in P0)
    const uint4 z4 = make_uint4(0, 0, 0, 0);
    reinterpret_cast<uint4*>(T)[tid] = z4;
    reinterpret_cast<uint4*>(T)[tid + MT] = z4;
#ifndef DMX_SORT_G2
    // four groups of four waves: groups 2 and 3 count in the first half of S (free until the
    // scatter), four ordered rounds of four waves instead of eight of two
    uint32_t* T2 = reinterpret_cast<uint32_t*>(L.sorted);
    reinterpret_cast<uint4*>(T2)[tid] = z4;
    reinterpret_cast<uint4*>(T2)[tid + MT] = z4;
    constexpr uint32_t NR = 4;
    uint32_t* Tg = (wave >> 3) ? T2 : T;
    const uint32_t sh = ((wave >> 2) & 1) << 4;   // this wave's group field
#else
    constexpr uint32_t NR = 8;
    uint32_t* Tg = T;
    const uint32_t sh = (wave >> 3) << 4;   // this wave's group field
#endif
    __syncthreads();   // (also: the staged block, for callers without a barrier after staging)
    const uint64_t lt = (1ull << lane) - 1ull;
    uint32_t x0l = (wave << 11) + lane, nvl = nvalid;
    uint32_t hh[16];   // bucket of each of this lane's 32 entries, two per register
    asm volatile("" : "+v"(x0l), "+v"(nvl));
#pragma unroll
    for (int st = 0; st < 32; st += 2) {
        const uint32_t xa = x0l + ((uint32_t)st << 6), xb = xa + 64;
        const uint32_t ha = xa < nvl ? bucket_of<NB>(ldg<NB>(L.data, xa)) : 0u;
        const uint32_t hb = xb < nvl ? bucket_of<NB>(ldg<NB>(L.data, xb)) : 0u;
        hh[st >> 1] = ha | (hb << 16);
        if ((st & 7) == 6) __builtin_amdgcn_sched_barrier(0);   // 8 loads in flight per group
    }
    if (stamp && tid == 0) tp0[0] = __builtin_amdgcn_s_memtime();
    uint32_t rk[16];                        // rank of each entry, two per register
#pragma unroll
    for (int j = 0; j < 16; j++) rk[j] = 0;
    for (uint32_t r = 0; r < NR; r++) {
        if (r == (wave & (NR - 1))) {
            asm volatile("" : "+v"(x0l), "+v"(nvl));
            if (RUNCHK) {
#pragma unroll
                for (int st = 0; st < 32; st++) {
                    const uint32_t x = x0l + ((uint32_t)st << 6);
                    const uint32_t h = (hh[st >> 1] >> (16 * (st & 1))) & 0xFFFFu;
                    const uint32_t rr = atomic_rank16<true>(Tg, h, x < nvl, lt, sh);
                    rk[st >> 1] |= rr << (16 * (st & 1));
                }
            } else {
                // 16 atomics in flight, then their ranks: the compiler keeps an atomic's use
                // next to it (one LDS round trip per step) unless the uses come after the batch
#pragma unroll
                for (int hb = 0; hb < 32; hb += 16) {
                    uint32_t old[16];
#pragma unroll
                    for (int q = 0; q < 16; q++) {
                        const int st = hb + q;
                        const uint32_t x = x0l + ((uint32_t)st << 6);
                        const uint32_t h = (hh[st >> 1] >> (16 * (st & 1))) & 0xFFFFu;
                        old[q] = atomicAdd(&Tg[h], x < nvl ? 1u << sh : 0u);
                    }
#pragma unroll
                    for (int q = 0; q < 16; q++) {
                        const int st = hb + q;
                        rk[st >> 1] |= ((old[q] >> sh) & 0xFFFFu) << (16 * (st & 1));
                    }
                }
            }
        }
        __syncthreads();
    }
    if (stamp && tid == 0) tp0[1] = __builtin_amdgcn_s_memtime();
    {   // bucket starts: thread t scans buckets 8t .. 8t + 7
        const uint4 a = reinterpret_cast<const uint4*>(T)[2 * tid], c = reinterpret_cast<const uint4*>(T)[2 * tid + 1];
        uint32_t w[8] = {a.x, a.y, a.z, a.w, c.x, c.y, c.z, c.w}, pre[8], s = 0;
#ifndef DMX_SORT_G2
        const uint4 a2 = reinterpret_cast<const uint4*>(T2)[2 * tid], c2 = reinterpret_cast<const uint4*>(T2)[2 * tid + 1];
        uint32_t w2[8] = {a2.x, a2.y, a2.z, a2.w, c2.x, c2.y, c2.z, c2.w};
#endif
#pragma unroll
        for (int j = 0; j < 8; j++) {
            pre[j] = s;
            s += (w[j] & 0xFFFFu) + (w[j] >> 16);
#ifndef DMX_SORT_G2
            s += (w2[j] & 0xFFFFu) + (w2[j] >> 16);
#endif
        }
        const uint32_t base = block_excl_scan(L, s, tid);
#pragma unroll
        for (int j = 0; j < 8; j++) {
            const uint32_t st0 = base + pre[j];
            pre[j] = st0;
#ifndef DMX_SORT_G2
            const uint32_t s1 = st0 + (w[j] & 0xFFFFu), s2 = s1 + (w[j] >> 16);
            w[j] = st0 | (s1 << 16);
            w2[j] = s2 | ((s2 + (w2[j] & 0xFFFFu)) << 16);
#else
            w[j] = st0 | ((st0 + (w[j] & 0xFFFFu)) << 16);
#endif
        }
        reinterpret_cast<uint4*>(T)[2 * tid] = make_uint4(w[0], w[1], w[2], w[3]);
        reinterpret_cast<uint4*>(T)[2 * tid + 1] = make_uint4(w[4], w[5], w[6], w[7]);
#ifndef DMX_SORT_G2
        reinterpret_cast<uint4*>(T2)[2 * tid] = make_uint4(w2[0], w2[1], w2[2], w2[3]);
        reinterpret_cast<uint4*>(T2)[2 * tid + 1] = make_uint4(w2[4], w2[5], w2[6], w2[7]);
#endif
        if (need_starts)
            reinterpret_cast<uint4*>(L.bstart)[tid] = make_uint4(pre[0] | (pre[1] << 16), pre[2] | (pre[3] << 16),
                                                                 pre[4] | (pre[5] << 16), pre[6] | (pre[7] << 16));
    }
    __syncthreads();
    asm volatile("" : "+v"(x0l), "+v"(nvl));
#ifndef DMX_SORT_G2
    // the destinations first (groups 2 and 3 read theirs from S's first half), then the stores
#pragma unroll
    for (int st = 0; st < 32; st++) {
        const uint32_t h = (hh[st >> 1] >> (16 * (st & 1))) & 0xFFFFu;
        const uint32_t rr = (rk[st >> 1] >> (16 * (st & 1))) & 0xFFFFu;
        const uint32_t dst = ((Tg[h] >> sh) & 0xFFFFu) + rr;
        rk[st >> 1] = (rk[st >> 1] & (0xFFFF0000u >> (16 * (st & 1)))) | ((dst & 0xFFFFu) << (16 * (st & 1)));
        if ((st & 7) == 7) __builtin_amdgcn_sched_barrier(0);
    }
    __syncthreads();
#pragma unroll
    for (int st = 0; st < 32; st++) {
        const uint32_t x = x0l + ((uint32_t)st << 6);
        if (x < nvl) L.sorted[(rk[st >> 1] >> (16 * (st & 1))) & 0xFFFFu] = (uint16_t)x;
    }
#else
#pragma unroll
    for (int st = 0; st < 32; st++) {
        const uint32_t x = x0l + ((uint32_t)st << 6);
        const uint32_t h = (hh[st >> 1] >> (16 * (st & 1))) & 0xFFFFu;
        const uint32_t rr = (rk[st >> 1] >> (16 * (st & 1))) & 0xFFFFu;
        if (x < nvl) L.sorted[((T[h] >> sh) & 0xFFFFu) + rr] = (uint16_t)x;
        if ((st & 7) == 7) __builtin_amdgcn_sched_barrier(0);
    }
#endif
    __syncthreads();
    if (stamp && tid == 0) tp0[2] = __builtin_amdgcn_s_memtime();
}

// Bucket-sorted positions S (stable by position inside a bucket), built here instead of
// by a separate chain pass: a two-pass LSD radix sort of the positions by bucket,
// digit 1 = bucket & 127, digit 2 = bucket >> 7.  Wave w owns the 2048 entries
// [2048w, 2048w+2048) of a pass.  Pass 1: sweep A counts (digit, wave) with LDS atomics
// (order-free), an exclusive scan (digit-major) turns counts into destinations, sweep B
// walks the entries again 64 per step, groups lanes with equal digits (LDS match-any,
// stable in lane order) and writes entry -> destination + earlier lanes of its group.
// Sweep B also stores each entry's digit 2 at its destination and counts pass 2's
// (digit, wave) totals, so pass 2 is a sequential read, one scan and the scatter; it
// reads its source into registers first, so it can write S in place.  Chains longer
// than KD need bucket starts: found afterwards where the bucket changes along S.
// Ranks inside a (digit, wave) group: EXACT = LDS match-any (order by construction); else
// the return value of an LDS atomicAdd per lane, which gfx950 serves in lane order for
// same-address lanes of one instruction (tools/atomic_order.hip: 0 of ~5e9 pairs out of
// order).  That order is not a documented guarantee, so the search verifies the result
// (every entry against its predecessor, sortbad) and the block falls back to EXACT.
// RUNCHK: count_add / atomic_rank first test whether all lanes of a step share one digit
// (runs), which turns a 64-way same-address atomic into one add; blocks that are not
// run-dominated (counted while staging) skip that test (correct either way).
template <bool EXACT, bool RUNCHK = true, int NB = 3>
__device__ __forceinline__ void sort_positions(MatchLDS& L, uint32_t bn, int32_t max_chain, uint32_t tid, bool stamp,
                                               uint64_t* tp0) {
#ifndef DMX_OLD_SORT
    if constexpr (!EXACT) {
        count_sort_positions<RUNCHK, NB>(L, bn, max_chain, tid, stamp, tp0);
        return;
    }
#endif
    const uint32_t lane = tid & 63, wave = wave_of(tid);
    const uint32_t nvalid = bn > 2 ? bn - 2 : 0;   // positions with a full trigram
    const bool need_starts = max_chain <= 0 || max_chain > KD;
    uint32_t* C = L.tsm;                                   // 16 x 128 pass-1 counters (tsm + exitp)
    uint32_t* C2 = L.lit;                                  // 16 x 64 pass-2 counters (lit: zeroed after P0)
    uint8_t* D2 = reinterpret_cast<uint8_t*>(L.bstart);    // digit 2 per pass-1 entry (bstart + len8[0, 16K))
    unsigned long long* G = reinterpret_cast<unsigned long long*>(L.len8 + DMX_BLK / 2);   // 16 x 128 lane masks
    unsigned long long* Gw = G + (wave << 7);
    for (uint32_t k = tid; k < 2 * (DMX_BLK / 32); k += MT) C[k] = 0;
    for (uint32_t k = tid; k < DMX_BLK / 32; k += MT) C2[k] = 0;
    for (uint32_t k = tid; k < 16 * 128; k += MT) G[k] = 0;
    __syncthreads();
    if (stamp && tid == 0) tp0[0] = __builtin_amdgcn_s_memtime();
    const uint64_t lt = (1ull << lane) - 1ull;
    const uint32_t x0 = (wave << 11) + lane;
    // per-sweep copies, laundered through an empty asm: the compiler otherwise keeps the
    // 32 step addresses and validity masks of one sweep live into the next (spills)
    uint32_t x0l = x0, nvl = nvalid;
    // bucket of each of this lane's 32 entries, two 13-bit values per register
    uint32_t hh[16];
    asm volatile("" : "+v"(x0l), "+v"(nvl));
#pragma unroll
    for (int st = 0; st < 32; st += 2) {
        const uint32_t xa = x0l + ((uint32_t)st << 6), xb = xa + 64;
        const uint32_t ha = xa < nvl ? bucket_of<NB>(ldg<NB>(L.data, xa)) : 0u;
        const uint32_t hb = xb < nvl ? bucket_of<NB>(ldg<NB>(L.data, xb)) : 0u;
        hh[st >> 1] = ha | (hb << 16);
        if ((st & 7) == 6) __builtin_amdgcn_sched_barrier(0);   // 8 loads in flight per group
    }
    // ---- pass 1: position order, digit = bucket & 127
    asm volatile("" : "+v"(x0l), "+v"(nvl));
#pragma unroll
    for (int st = 0; st < 32; st++) {
        const uint32_t x = x0l + ((uint32_t)st << 6);
        const uint32_t h = (hh[st >> 1] >> (16 * (st & 1))) & 0xFFFFu;
        count_add<RUNCHK>(C + (wave << 7), h & 127u, x < nvl, false);
    }
    __syncthreads();
    {   // destinations, digit-major: entry (dg, w) at order 16*dg + w; two per thread
        const uint32_t o0 = tid * 2, o1 = o0 + 1;
        const uint32_t i0 = ((o0 & 15) << 7) + (o0 >> 4), i1 = ((o1 & 15) << 7) + (o1 >> 4);
        const uint32_t v0 = C[i0], v1 = C[i1];
        const uint32_t ex = block_excl_scan(L, v0 + v1, tid);
        C[i0] = ex;
        C[i1] = ex + v0;
    }
    __syncthreads();
    asm volatile("" : "+v"(x0l), "+v"(nvl));
#pragma unroll
    for (int st = 0; st < 32; st++) {
        const uint32_t x = x0l + ((uint32_t)st << 6);
        const bool valid = x < nvl;
        const uint32_t h = (hh[st >> 1] >> (16 * (st & 1))) & 0xFFFFu;
        const uint32_t dg = h & 127u;
        uint32_t dst = 0;
        if (EXACT) {   // rank = destination + earlier lanes of the same digit (LDS match-any)
            const uint32_t c = valid ? C[(wave << 7) + dg] : 0u;
            const uint64_t eq = group_of(Gw, dg, valid);
            dst = c + (uint32_t)__popcll(eq & lt);
            if (valid && (eq >> lane) == 1ull) C[(wave << 7) + dg] = c + (uint32_t)__popcll(eq);
        } else {   // same-address LDS atomics return in lane order (checked, see above)
            dst = atomic_rank<RUNCHK>(&C[wave << 7], dg, valid, lt);
        }
        if (valid) {
            L.sorted[dst] = (uint16_t)x;
            D2[dst] = (uint8_t)(h >> 7);
        }
        count_add<RUNCHK>(C2, ((dst >> 11) << 6) | (h >> 7), valid, false);   // pass 2: (wave, digit)
        __builtin_amdgcn_sched_barrier(0);   // keep the unrolled steps apart (register pressure)
    }
    __syncthreads();
    if (stamp && tid == 0) tp0[1] = __builtin_amdgcn_s_memtime();
    // ---- pass 2: pass-1 order, digit = bucket >> 7
    uint32_t pk[16], dk[8];   // this lane's 32 source entries (u16 pairs) and digits (u8 quads)
    asm volatile("" : "+v"(x0l), "+v"(nvl));
#pragma unroll
    for (int st = 0; st < 32; st += 2) {
        const uint32_t xa = x0l + ((uint32_t)st << 6), xb = xa + 64;
        const uint32_t pa = xa < nvl ? (uint32_t)L.sorted[xa] : 0u;
        const uint32_t pb = xb < nvl ? (uint32_t)L.sorted[xb] : 0u;
        const uint32_t da = xa < nvl ? (uint32_t)D2[xa] : 0u;
        const uint32_t db = xb < nvl ? (uint32_t)D2[xb] : 0u;
        pk[st >> 1] = pa | (pb << 16);
        if ((st & 3) == 0) dk[st >> 2] = da | (db << 8);
        else dk[st >> 2] |= (da << 16) | (db << 24);
        if ((st & 7) == 6) __builtin_amdgcn_sched_barrier(0);
    }
    {   // destinations (dg, w) at order 16*dg + w, one per thread
        const uint32_t i0 = ((tid & 15) << 6) + (tid >> 4);
        const uint32_t v0 = C2[i0];
        const uint32_t ex = block_excl_scan(L, v0, tid);   // (its barriers also order the reads above)
        C2[i0] = ex;
    }
    __syncthreads();
    asm volatile("" : "+v"(x0l), "+v"(nvl));
#pragma unroll
    for (int st = 0; st < 32; st++) {
        const uint32_t x = x0l + ((uint32_t)st << 6);
        const bool valid = x < nvl;
        const uint32_t p = (pk[st >> 1] >> (16 * (st & 1))) & 0xFFFFu;
        const uint32_t dg = (dk[st >> 2] >> (8 * (st & 3))) & 0xFFu;
        if (EXACT) {
            const uint32_t c = valid ? C2[(wave << 6) + dg] : 0u;
            const uint64_t eq = group_of(Gw, dg, valid);
            if (valid) {
                L.sorted[c + (uint32_t)__popcll(eq & lt)] = (uint16_t)p;
                if ((eq >> lane) == 1ull) C2[(wave << 6) + dg] = c + (uint32_t)__popcll(eq);
            }
        } else {
            const uint32_t dst = atomic_rank<RUNCHK>(&C2[wave << 6], dg, valid, lt);
            if (valid) L.sorted[dst] = (uint16_t)p;
        }
        __builtin_amdgcn_sched_barrier(0);
    }
    __syncthreads();
    for (uint32_t k = tid; k < DMX_BLK / 32; k += MT) L.lit[k] = 0;
    if (need_starts) {   // bucket starts: entries whose bucket differs from the previous one
        for (uint32_t k = tid; k < nvalid; k += MT) {
            const uint32_t h = bucket_of<NB>(ldg<NB>(L.data, L.sorted[k]));
            const uint32_t hp = k ? bucket_of<NB>(ldg<NB>(L.data, L.sorted[k - 1])) : 0xFFFFFFFFu;
            if (h != hp) L.bstart[h] = (uint16_t)k;
        }
    }
    __syncthreads();
    if (stamp && tid == 0) tp0[2] = __builtin_amdgcn_s_memtime();
}


// P0' (the exhaustive parse on NB-byte chains): with S sorted by NG-byte buckets, the nearest
// earlier position with the same first NG bytes of every entry (NG < NB), as a seed key
// NG << 15 | q (NG = 3 writes every seed, 0 = none; NG = 4 only the entries it finds, whose
// keys beat the 3-byte ones).  Entries k - 1 .. k - PW stream through the lanes (wave
// shifts; lane 0 from a halo of the PW entries below the chunk); entries whose bucket goes on
// past PW colliding entries (a rare gram in a bucket it shares with a common one) are listed
// and walked afterwards a wave per entry, 64 entries a step.  Returns this thread's
// sort-order check (an entry before its predecessor).
template <int NG>
__device__ __forceinline__ uint32_t gram_pass(MatchLDS& L, uint32_t nv, uint32_t tid, uint16_t* __restrict__ seeds,
                                              uint32_t& ndefer, uint64_t& tsweep) {
#ifndef DMX_GRAM_PW
    constexpr uint32_t PW = 9;
#else
    constexpr uint32_t PW = DMX_GRAM_PW;   // (diagnostic builds)
#endif
    constexpr uint32_t GM = NG == 3 ? 0xFFFFFFu : 0xFFFFFFFFu;
    const uint32_t lane = tid & 63;
    uint32_t* UL = L.tsm;   // tsm + exitp: 2048 slots, free until the next sort
    uint32_t bad = 0;
    if (tid == 0) { L.ntok = 0; L.wsum[0] = 0; L.wsum[1] = 0; }   // list length, chunk and walk counters
    __syncthreads();
    uint32_t cnx = wave_claim(&L.wsum[0]);
    for (;;) {   // chunks of 64 entries from the workgroup counter, the next fetched a chunk ahead
        const uint32_t kb = (uint32_t)__builtin_amdgcn_readfirstlane((int)cnx) << 6;
        if (kb >= nv) break;
        cnx = wave_claim(&L.wsum[0]);
        const uint32_t k = kb + lane;
        const bool act = k < nv;
        const uint32_t i = act ? (uint32_t)L.sorted[k] : 0u, w = act ? ld4(L.data, i) : 0u;
        const uint32_t t = w & GM, hb = bucket_of<NG>(t);
        uint32_t hi = 0xFFFFu, hw = 0;   // halo: lane l < PW holds entry kb - 1 - l
        if (lane < PW && kb >= lane + 1) { hi = L.sorted[kb - 1 - lane]; hw = ld4(L.data, hi); }
        uint32_t ip = i, wp = w, q = 0xFFFFu;
        bool open = act && k > 0;   // still looking
        for (uint32_t st = 1; st <= PW; st++) {
            if (st > 1 && !__ballot(open)) break;   // most chunks: every lane found at step 1
            ip = wshr(ip, __builtin_amdgcn_readlane(hi, (int)st - 1));
            wp = wshr(wp, __builtin_amdgcn_readlane(hw, (int)st - 1));
            if (st == 1 && open && sort_key_h<NG>(wp, ip) > sort_key_h<NG>(w, i)) bad = 1;
            if (open && k >= st) {
                if ((wp & GM) == t) { q = ip; open = false; }
                else if (bucket_of<NG>(wp & GM) != hb) open = false;   // the bucket start is passed
            } else {
                open = false;
            }
        }
        if (open && k > PW) {   // more of the bucket to walk: later, a wave per entry
            const uint32_t u = atomicAdd(&L.ntok, 1u);
            if (u < 2 * (DMX_BLK / 32)) {
                UL[u] = ((k - PW) << 16) | k;
            } else {   // (the list is full) walk down to the bucket's first entry here
                for (uint32_t j = k - PW; j > 0; j--) {
                    const uint32_t c = L.sorted[j - 1], wc = ld4(L.data, c) & GM;
                    if (wc == t) { q = c; break; }
                    if (bucket_of<NG>(wc) != hb) break;
                }
            }
        }
        // (a gram that runs past the block's end is a match of fewer bytes: the 3-byte seed stays)
#ifndef DMX_H4_NOSTORE
        if (act && (NG == 3 || (q != 0xFFFFu && i + NG <= nv + 2))) seeds[i] = seed_enc<NG>(q);
#else
        if (act && q == 0x1234u) seeds[i] = (uint16_t)q;   // (diagnostic timing builds: the output is wrong)
#endif
    }
    __syncthreads();
    tsweep += __builtin_amdgcn_s_memtime();   // (diagnostic stamps: the sweep's end)
    const uint32_t nul = min(L.ntok, 2u * (DMX_BLK / 32));
    ndefer += L.ntok;
    for (;;) {   // listed entries from the workgroup counter (their walks differ in length)
        const uint32_t un = wave_claim(&L.wsum[1]);
        const uint32_t u = (uint32_t)__builtin_amdgcn_readfirstlane((int)un);
        if (u >= nul) break;
        const uint32_t e = (uint32_t)__builtin_amdgcn_readfirstlane((int)UL[u]);
        const uint32_t k = e & 0xFFFFu, i = L.sorted[k], t = ld4(L.data, i) & GM;
        const uint32_t hb = bucket_of<NG>(t);
        uint32_t q = 0xFFFFu;
        // down the bucket, 64 entries a step, to its first entry (where the bucket changes;
        // the sort computes no bucket starts for this pass)
        for (int jb = (int)(e >> 16); jb > 0; jb -= 64) {
            const int j = jb - 1 - (int)lane;
            const uint32_t c = j >= 0 ? (uint32_t)L.sorted[j] : 0u, wc = ld4(L.data, c) & GM;
            const bool inb = j >= 0 && bucket_of<NG>(wc) == hb;
            const uint64_t m = __ballot(inb && wc == t), x = __ballot(!inb);
            const uint64_t below = x ? ((1ull << __builtin_ctzll(x)) - 1ull) : ~0ull;   // lanes before the bucket's end
            if (m & below) {   // the lowest lane holds the nearest
                q = (uint32_t)__builtin_amdgcn_readlane((int)c, (int)__builtin_ctzll(m & below));
                break;
            }
            if (x) break;
        }
        if (lane == 0 && (NG == 3 || (q != 0xFFFFu && i + NG <= nv + 2))) seeds[i] = seed_enc<NG>(q);
    }
    // every store complete (in L2) before the caller's barrier: the search's loads of the
    // seeds come from other waves, and a workgroup barrier alone does not wait for stores
    __builtin_amdgcn_s_waitcnt(0);
    return bad;
}

// ------------------------------------------------------------------------------------
// K0 (DMX_F_DICT): the cross-block dictionary, DESIGN.md §4.6.  For every
// position i of block b, the longest match against the history (the previous sw block;
// block 0: the caller's dict bytes):
//   candidates = the K newest history positions q of i's bucket (all for K = 0) whose
//                trigram lies inside the history (q + 2 < hn), with distance
//                hn - q + i <= 32768; newest first, strict > (ties to the nearest);
//   bytes are compared across the boundary (the source runs from the history into the
//   block itself), up to min(258, bn - i).
// Two launches before the match kernel:
//   K0a dmx_chain_kernel  the bucket-sorted chains of every block (and of the dict), the
//                         match kernel's own sort, exported: S (positions by (bucket,
//                         position)) and the bucket ends.  The match kernel then loads
//                         its S instead of sorting (each block is sorted once).
//   K0b dmx_hist_kernel   the history search in the block's bucket order: lanes of one
//                         bucket share their candidates (the history's bucket tail), so
//                         their LDS reads are broadcasts.  Result per entry k of S:
//                         len << 16 | dist (0 = none) into the block's token slots, which
//                         the match kernel merges as it stores its own result
//                         (store_result) and overwrites with tokens in P3.
// Chain slots: slot 0 = the dict (block "-1"), slot b + 1 = block b.
// ------------------------------------------------------------------------------------
#define TB8(W, i) (reinterpret_cast<const uint8_t*>(W)[i])

// Stage bytes src[0, len) at LDS word array W (16-byte chunks, zero padded to nwords).
__device__ __forceinline__ void stage_bytes(uint32_t* W, uint32_t nwords, const uint8_t* src, uint32_t len,
                                            const uint8_t* src2, uint32_t len2, uint32_t tid) {
    // bytes [0, len) from src, then [len, len + len2) from src2, then zeros
    const bool al = ((reinterpret_cast<uintptr_t>(src) & 15) == 0);
    for (uint32_t k = tid; k < nwords / 4; k += MT) {
        const uint32_t p = k << 4;
        uint4 v;
        if (al && p + 16 <= len) {
            v = *reinterpret_cast<const uint4*>(src + p);
        } else {
            uint32_t w[4] = {0, 0, 0, 0};
            for (uint32_t j = 0; j < 16; j++) {
                const uint32_t x = p + j;
                const uint32_t c = x < len ? src[x] : (x - len < len2 ? src2[x - len] : 0u);
                w[j >> 2] |= c << (8 * (j & 3));
            }
            v = make_uint4(w[0], w[1], w[2], w[3]);
        }
        *reinterpret_cast<uint4*>(&W[k << 2]) = v;
    }
}

// History of block b: its bytes and length (0 = none).
__device__ __forceinline__ const uint8_t* hist_of(const uint8_t* in, uint32_t sw, uint32_t b, const uint8_t* pre,
                                                  uint32_t npre, uint32_t& hn) {
    if (b > 0) { hn = sw; return in + (uint64_t)(b - 1) * sw; }
    hn = (pre && npre) ? (npre < sw ? npre : sw) : 0u;
    return hn ? pre + (npre - hn) : nullptr;
}

__global__ __launch_bounds__(MT) void dmx_chain_kernel(const uint8_t* __restrict__ in, uint64_t n, uint32_t sw,
                                                       const uint8_t* __restrict__ pre, uint32_t npre,
                                                       uint16_t* __restrict__ chs, uint16_t* __restrict__ che,
                                                       uint32_t* __restrict__ nfallback) {
    __shared__ MatchLDS L;
    __shared__ uint64_t tp0[3];
    const uint32_t tid = threadIdx.x;
    const uint32_t slot = blockIdx.x;
    const uint8_t* src;
    uint32_t len;
    if (slot == 0) {
        src = hist_of(in, sw, 0, pre, npre, len);
    } else {
        const uint64_t off = (uint64_t)(slot - 1) * sw;
        len = (uint32_t)((n - off) < sw ? (n - off) : sw);
        src = in + off;
    }
    if (len < 3) return;   // no entries (slot 0 without a dict)
    stage_bytes(L.data, DATA_WORDS, src, len, nullptr, 0, tid);
    const uint32_t nv = len - 2;
    uint16_t* S = chs + (uint64_t)slot * DMX_BLK;
    uint16_t* E = che + (uint64_t)slot * DMX_NBUCKET;
    // run-dominated blocks (a quarter of the 16-byte chunks one repeated byte, as K1 counts them)
    // take the run-aware ranks; the others batch their rank atomics
    __shared__ uint32_t nruns;
    if (tid == 0) nruns = 0;
    __syncthreads();
    uint32_t runny = 0;
    for (uint32_t k = tid; k < (len + 15) / 16; k += MT) {
        const uint4 v = reinterpret_cast<const uint4*>(L.data)[k];
        runny += (k * 16 + 16 <= len && v.x == v.y && v.y == v.z && v.z == v.w && v.x == (v.x & 0xFFu) * 0x01010101u) ? 1u : 0u;
    }
    if (runny) atomicAdd(&nruns, runny);
    __syncthreads();
    const bool runs = nruns * 4u >= (len + 15) / 16;
    for (uint32_t attempt = 0;; attempt++) {
        if (attempt == 0 && runs) sort_positions<false, true>(L, len, 1, tid, false, tp0);
        else if (attempt == 0) sort_positions<false, false>(L, len, 1, tid, false, tp0);
        else sort_positions<true>(L, len, 1, tid, false, tp0);
        for (uint32_t k = tid; k < DMX_NBUCKET; k += MT) L.bstart[k] = 0;
        __syncthreads();
        bool bad = false;   // the lane-ordered atomic ranks are verified here, as in the search:
                            // every adjacent pair ascends by (bucket, position), so S is sorted
        for (uint32_t k = tid; k < nv; k += MT) {
            const uint32_t q = L.sorted[k];
            const uint32_t h = dmx_hash(ld4(L.data, q) & 0xFFFFFFu);
            if (k + 1 < nv) {
                const uint32_t q1 = L.sorted[k + 1];
                const uint32_t h1 = dmx_hash(ld4(L.data, q1) & 0xFFFFFFu);
                if (h1 != h) L.bstart[h] = (uint16_t)(k + 1);
                if (((h1 << 15) | q1) < ((h << 15) | q)) bad = true;
            } else {
                L.bstart[h] = (uint16_t)(k + 1);
            }
        }
        if (!__syncthreads_or(bad) || attempt) break;
        if (tid == 0) atomicAdd(nfallback, 1u);
    }
    for (uint32_t k = tid; k < (nv + 7) / 8; k += MT)   // 8 entries per 16-byte store
        reinterpret_cast<uint4*>(S)[k] = reinterpret_cast<const uint4*>(L.sorted)[k];
    for (uint32_t k = tid; k < DMX_NBUCKET / 8; k += MT)
        reinterpret_cast<uint4*>(E)[k] = reinterpret_cast<const uint4*>(L.bstart)[k];
}

// 146 KB, one workgroup per CU: the history, the block and the history's chains (S and the
// bucket ends) all in LDS, so the candidate loop has no global-memory latency (with S and
// the bucket ends read through the caches, two 66 KB workgroups per CU spent ~340 K cycles
// per block waiting on three dependent L2 reads per entry)
struct __attribute__((aligned(16))) HistLDS {
    uint32_t data[DATA_WORDS];        // the history, then the block's first bytes (sources crossing over)
    uint32_t cur[DMX_BLK / 4 + 80];   // the block (targets), zero padded
    uint16_t sp[DMX_BLK];             // the history's entries in bucket order (its S)
    uint16_t ep[DMX_NBUCKET];         // the history's bucket ends
    uint32_t qd[MW][64][2];           // per wave: entries waiting for the LDS extension
};

// One group of HG history candidates of entry i (target bytes t0..t2, bucket h): entries
// x, x - 1, ... of the history's S, the cnt-th candidate onwards.  Updates the best (longest,
// then nearest); returns whether the walk may stop (an entry past the distance limit or, in
// the exhaustive walk, of another bucket).  ONE: K <= HG, the only group (no walk state).
template <int HG, bool ONE, bool DEFER = false>
__device__ __forceinline__ bool hist_group(const HistLDS& L, int32_t x, uint32_t cnt, uint32_t K, uint32_t h,
                                           uint32_t t0, uint32_t t1, uint32_t t2, uint32_t i, uint32_t lim,
                                           int32_t minq, uint32_t& best, uint32_t& bq, uint32_t* fullp = nullptr) {
    const uint16_t* Sp = L.sp;
    uint32_t q[HG], s0[HG], s1[HG], s2[HG];
#pragma unroll
    for (int g = 0; g < HG; g++) q[g] = (x - g >= 0 && (!ONE || (uint32_t)g < K)) ? (uint32_t)Sp[x - g] : 0u;
#pragma unroll
    for (int g = 0; g < HG; g++) ld12(L.data, q[g], s0[g], s1[g], s2[g]);
    uint32_t key = 0, full = 0;
    bool left = false;
#pragma unroll
    for (int g = 0; g < HG; g++) {
        if (ONE && (uint32_t)g >= K) break;   // uniform
        const bool ok = x - g >= 0 && (ONE || cnt + (uint32_t)g < K) && (int32_t)q[g] >= minq;
        const uint32_t mb = min(min(ffbl_hw(t0 ^ s0[g]), __builtin_elementwise_add_sat(ffbl_hw(t1 ^ s1[g]), 32u)),
                                min(ffbl_hw(t2 ^ s2[g]), 32u) + 64u);
        const uint32_t m = ok ? min(mb >> 3, lim) : 0u;
        key = max(key, (m << 8) | (255u - (uint32_t)g));
        full |= (ok && mb == 96u && lim > CB) ? (1u << g) : 0u;
        if (!ONE) {
            left = left || (x - g >= 0 && (int32_t)q[g] < minq);
            if (K == 0xFFFFFFFFu)   // exhaustive: the walk ends at the bucket's start
                left = left || (x - g >= 0 && dmx_hash(s0[g] & 0xFFFFFFu) != h);
        }
    }
    if ((key >> 8) > best) { best = key >> 8; bq = q[255u - (key & 255u)]; }
    if (DEFER) {   // the extension waits in the wave's queue (hist_flush)
        *fullp = full;
        return false;
    }
    while (full) {   // nearest first; a farther one must be strictly longer
        const uint32_t g = (uint32_t)__builtin_ctz(full);
        full &= full - 1u;
        if (best >= lim) break;
        uint32_t qg = q[0];
#pragma unroll
        for (int gg = 1; gg < HG; gg++) qg = (uint32_t)gg == g ? q[gg] : qg;
        if (best > CB && TB8(L.data, qg + best) != TB8(L.cur, i + best)) continue;
        const uint32_t kk = min(ext_len2(L.cur, i, L.data, qg, CB, lim), lim);   // 16, then 32 B per round
        if (kk > best) { best = kk; bq = qg; }
    }
    return left;
}

// The queued entries of one wave (qn <= 64; items k | full << 16 and x | i << 16: entry k at
// position i, its group of candidates from entry x of the history's S, full = those equal in
// all CB register bytes): lane l extends item l's full candidates from LDS, nearest first,
// a farther one only if it also matches the byte at the best length, and stores the result.
// Extensions spread over all 64 lanes instead of the few lanes of each entry round that need one.
__device__ __forceinline__ void hist_flush(const HistLDS& L, uint32_t wave, uint32_t qn, uint32_t lane, uint32_t hn,
                                           uint32_t bn, uint32_t* __restrict__ hb) {
    __builtin_amdgcn_wave_barrier();
    if (lane < qn) {
        const uint32_t w0 = lds_ld(const_cast<uint32_t*>(&L.qd[wave][lane][0]));
        const uint32_t w1 = lds_ld(const_cast<uint32_t*>(&L.qd[wave][lane][1]));
        const uint32_t k = w0 & 0xFFFFu, i = w1 >> 16;
        const int32_t x = (int32_t)(w1 & 0xFFFFu);
        uint32_t full = w0 >> 16;
        const uint32_t lim = min(bn - i, (uint32_t)MAXLEN);
        uint32_t best = CB, bq = L.sp[x - (int32_t)__builtin_ctz(full)];   // the nearest full one
        while (full && best < lim) {
            const uint32_t g = (uint32_t)__builtin_ctz(full);
            full &= full - 1u;
            const uint32_t qg = L.sp[x - (int32_t)g];
            if (best > CB && TB8(L.data, qg + best) != TB8(L.cur, i + best)) continue;
            const uint32_t kk = min(ext_len2(L.cur, i, L.data, qg, CB, lim), lim);
            if (kk > best) { best = kk; bq = qg; }
        }
        hb[k] = (best << 16) | (hn - bq + i);
    }
    __builtin_amdgcn_wave_barrier();
}

// HG = history candidates per group: 6 for K <= 6, 7 for K = 7 (the bench default), 8 otherwise
// (K > 8 in groups of 8).
template <int HG>
__global__ __launch_bounds__(MT) void dmx_hist_kernel_t(const uint8_t* __restrict__ in, uint64_t n, uint32_t sw,
                                                      int32_t max_chain, const uint8_t* __restrict__ pre, uint32_t npre,
                                                      const uint16_t* __restrict__ chs, const uint16_t* __restrict__ che,
                                                      uint32_t* __restrict__ hb_g, uint64_t* __restrict__ dbg) {
    __shared__ HistLDS L;
    const uint32_t tid = threadIdx.x;
    const uint32_t b = blockIdx.x;
    const uint64_t off = (uint64_t)b * sw;
    const uint32_t bn = (uint32_t)((n - off) < sw ? (n - off) : sw);
    const uint8_t* cur = in + off;
    uint32_t hn;
    const uint8_t* hs = hist_of(in, sw, b, pre, npre, hn);
    uint32_t* hb = hb_g + (uint64_t)b * DMX_BLK;
    const uint32_t nvalid = bn > 2 ? bn - 2 : 0;
    if (hn < 3) {   // no history entries
        for (uint32_t k = tid; k < nvalid; k += MT) hb[k] = 0;
        return;
    }
    const uint64_t tbeg = dbg ? __builtin_amdgcn_s_memtime() : 0;
    stage_bytes(L.data, DATA_WORDS, hs, hn, cur, bn, tid);
    stage_bytes(L.cur, DMX_BLK / 4 + 80, cur, bn, nullptr, 0, tid);
    {   // the history's chains: S (hn - 2 entries, 8 per 16-byte load) and the bucket ends
        const uint4* Sg = reinterpret_cast<const uint4*>(chs + (uint64_t)b * DMX_BLK);
        const uint4* Eg = reinterpret_cast<const uint4*>(che + (uint64_t)b * DMX_NBUCKET);
        for (uint32_t k = tid; k < (hn - 2 + 7) / 8; k += MT) reinterpret_cast<uint4*>(L.sp)[k] = Sg[k];
        for (uint32_t k = tid; k < DMX_NBUCKET / 8; k += MT) reinterpret_cast<uint4*>(L.ep)[k] = Eg[k];
    }
    __syncthreads();
    const uint64_t ts0 = dbg ? __builtin_amdgcn_s_memtime() : 0;
    const uint16_t* Sc = chs + (uint64_t)(b + 1) * DMX_BLK;   // the block's entries in bucket order
    const uint16_t* Ep = L.ep;                                // the history's bucket ends (LDS)
    const uint32_t K = max_chain > 0 ? (uint32_t)max_chain : 0xFFFFFFFFu;
    const uint32_t lane = tid & 63, wave = wave_of(tid);
    const uint64_t lt = (1ull << lane) - 1ull;
    uint32_t qn = 0;   // queued entries of this wave (K <= HG)
    uint32_t inext = tid < nvalid ? (uint32_t)Sc[tid] : 0u;
    // wave-uniform trip count (every lane runs the queue code); lanes past nvalid idle
    for (uint32_t k0 = tid - lane; k0 < nvalid; k0 += MT) {
        const uint32_t k = k0 + lane;
        const bool act = k < nvalid;
        const uint32_t i = inext;
        if (k + MT < nvalid) inext = Sc[k + MT];   // next entry in flight during this one
        uint32_t best = 0, bq = 0, full = 0;
        int32_t x0 = -1;
        if (act) {
            uint32_t t0, t1, t2;
            ld12(L.cur, i, t0, t1, t2);
            const uint32_t h = dmx_hash(t0 & 0xFFFFFFu);
            const uint32_t lim = min(bn - i, (uint32_t)MAXLEN);
            const int32_t minq = (int32_t)(hn + i) - 32768;   // distance <= 32768
            // Candidates newest first in groups of HG, loaded together and compared
            // branch-free in registers on 12 bytes (longest, then nearest); only candidates
            // equal in all 12 are extended, those farther than the best so far only if they
            // match its last byte.  An entry older than the distance limit, or of another
            // bucket, can never win (a bucket's older entries are farther still; another bucket
            // is another trigram), so it is masked, and the walk ends after its group; the
            // exhaustive walk also ends where the bucket does.
            x0 = (int32_t)Ep[h] - 1;
            if (K <= (uint32_t)HG) {   // bounded (the bench's K = 7): one group, extensions queued
                hist_group<HG, true, true>(L, x0, 0, K, h, t0, t1, t2, i, lim, minq, best, bq, &full);
            } else {
                uint32_t cnt = 0;
                for (int32_t x = x0; x >= 0 && cnt < K && best < lim; x -= HG, cnt += HG)
                    if (hist_group<HG, false>(L, x, cnt, K, h, t0, t1, t2, i, lim, minq, best, bq)) break;
            }
        }
        const bool push = full != 0;
        const uint64_t pm = __ballot(push);
        const uint32_t np = (uint32_t)__popcll(pm);
        if (qn + np > 64) {
            hist_flush(L, wave, qn, lane, hn, bn, hb);
            qn = 0;
        }
        if (push) {
            const uint32_t slot = qn + (uint32_t)__popcll(pm & lt);
            lds_st(&L.qd[wave][slot][0], k | (full << 16));
            lds_st(&L.qd[wave][slot][1], (uint32_t)x0 | (i << 16));
        } else if (act) {
            hb[k] = best >= 3 ? (best << 16) | (hn - bq + i) : 0u;
        }
        qn += np;
    }
    if (qn) hist_flush(L, wave, qn, lane, hn, bn, hb);
    if (dbg) {   // stamps 12..15: staged, searched
        __syncthreads();
        if (tid == 0) {
            dbg[(uint64_t)b * DMX_STAMPS + 12] = ts0 - tbeg;
            dbg[(uint64_t)b * DMX_STAMPS + 13] = __builtin_amdgcn_s_memtime() - tbeg;
        }
    }
}

// K0 (DMX_F_STORE_CHECK): the noise check of every block, so that noise
// blocks skip the parse and go out stored.  One 256-thread workgroup per block.
//   pass 0: the 8 bit-plane counts of the first 4096 bytes (one 16-byte load per thread,
//           v_bcnt on masked words).  Text, runs and 7-bit data fail here and leave, having
//           read an eighth of the block.
//   pass 1: the whole block into registers (8 loads per thread in flight), Adler-32
//           partial sums (v_sad_u8, v_dot4_u32_u8).
//   pass 2 (noise-like blocks only; full blocks from the registers of pass 1): byte
//           histogram of every s-th position (s = 8 for full blocks: 4096 samples) and
//           17-bit presence bitmap of the 4-grams sampled by content (bits 11..13 of their
//           hash clear: an eighth), LDS atomics (17 KB: 8 workgroups per CU).  The
//           atomics bound this pass: round 2 sampled every other position and half the
//           4-grams (32 K atomics per block, 0.53 ms per GiB); now 8 K.
// A block that passes gets its whole record here (stored, no tokens); the match kernel then
// skips it and the Huffman kernels leave it alone.  Same integer rule as
// dmx_oracle_store_check.
#define SCT 256
#define SC_PLANE 4096   // bytes of the bit-plane test (SCT x 16: one load per thread)
__device__ __forceinline__ void sc_load(const uint8_t* d, uint32_t p, uint32_t bn, bool aligned16, uint32_t w[5]) {
    if (aligned16 && p + 20 <= bn) {
        const uint4 v = *reinterpret_cast<const uint4*>(d + p);
        w[0] = v.x; w[1] = v.y; w[2] = v.z; w[3] = v.w;
        w[4] = *reinterpret_cast<const uint32_t*>(d + p + 16);
    } else {   // block tail (or unaligned input): bytes past bn read as 0
#pragma unroll
        for (int j = 0; j < 5; j++) w[j] = 0;
        for (uint32_t j = 0; j < 20; j++)
            if (p + j < bn) w[j >> 2] |= (uint32_t)d[p + j] << (8 * (j & 3));
    }
}

// The parse of a block of bn copies of byte c in closed form (what the search + walk give
// for it, greedy or lazy, any chain bound, no dictionary): a literal, then q = (bn - 1) / 258
// distance-1 matches of 258, then the rest r = (bn - 1) % 258 as one distance-1 match when
// r >= 3, else r literals.  Tokens are written by the threads in parallel; thread 0 adds the
// histogram counts to H (zeroed, DMX_HIST entries).  Returns the token count.
__device__ __forceinline__ uint32_t uniform_parse(uint32_t bn, uint32_t c, uint32_t* __restrict__ tb, uint32_t* H,
                                                  uint32_t tid, uint32_t nthr) {
    const uint32_t R = bn ? bn - 1 : 0, q = R / MAXLEN, r = R % MAXLEN;
    const uint32_t ntok = bn ? 1 + q + (r >= 3 ? 1 : r) : 0;
    for (uint32_t k = tid; k < ntok; k += nthr) {
        uint32_t t = c;
        if (k >= 1 && k <= q) t = (1u << 9) | MAXLEN;
        else if (k == q + 1 && r >= 3) t = (1u << 9) | r;
        tb[k] = t;
    }
    if (tid == 0 && bn) {
        uint32_t sy, eb, ev;
        H[c] += 1 + (r >= 3 ? 0 : r);
        if (q) {
            len_sym(MAXLEN, sy, eb, ev);
            H[sy] += q;
        }
        if (r >= 3) {
            len_sym(r, sy, eb, ev);
            H[sy] += 1;
        }
        if (q + (r >= 3 ? 1 : 0)) {
            dist_sym(1u, sy, eb, ev);
            H[DMX_DIST0 + sy] += q + (r >= 3 ? 1 : 0);
        }
    }
    return ntok;
}

// Work lists (DMX_F_STORE_CHECK, round 5), so that a stored block costs no workgroup in K1,
// K2 or K4 (C4: 32 768 stored blocks).  dmx_worklist_kernel (one workgroup, after K0) builds
// them from K0's prestored values; dmx_ctx::wl (u32) holds counters, then three lists of
// cap_blocks entries each:
//   L1 = wl + WL_HDR             blocks K1 parses (prestored 0)
//   L2 = L1 + cap                blocks K2 codes (prestored 0 and 2)
//   L4 = L2 + cap                blocks K4 packs, appended by the scan's apply launch
// WL_M = the first block that K0 did not store and copy whole (prestored != 3).  Blocks
// 1 <= b < min(M, nblk - 1) form a prefix of stored blocks at their speculative offsets
// (every block before them is stored too): K0 wrote every byte of them and K4 never sees
// them.  (A first version appended to the lists from K0 with device atomics: 3 052 text
// blocks took 0.11 ms, 32 768 blocks of zeros 0.79 ms -- same-address atomics from every
// XCD serialise.)
// The hint (words WL_HINT, WL_HINT + 1: a host-mapped pinned address, set at allocation):
// {nblk, |L1|, |L2|, |L4|, dedupe candidates} of the latest encode, written by the list
// builder and K4 -- or, when that encode ran without the lists (every shape per block, no
// dedupe: text), by the scan kernel from K0's block kinds -- read by the host at the next
// encode to choose the launch shapes (wl_shape).  Only the shape depends on it -- every
// shape writes the same stream.
#define WL_N1 0
#define WL_C1 1
#define WL_N2 2
#define WL_N4 3
#define WL_M 5
#define WL_N5 6
#define WL_HINT 8
#define WL_HDR 16
// Uniform-block dedupe (round 5, the worklist kernel's `dedupe`): full blocks of one repeated
// byte c (prestored 2, 1 <= b <= nblk - 2) all encode to the same bit string, so only the
// first of them per byte value (its representative) is coded by K2 and packed by K4; the
// others (the dups, list L5 = L4 + cap, rep index per block in D = L5 + cap, ~0 = not a dup)
// take the representative's block record in the scan's tile pass and have its bits copied
// to their offsets by dmx_dup_copy_kernel after K4.
__host__ __device__ __forceinline__ const uint32_t* wl_dup(const uint32_t* wl, uint64_t cap) { return wl + WL_HDR + 4 * cap; }
// block b is a dup (the worklist kernel set bit 3 of its code; its representative is in D)
__device__ __forceinline__ bool is_dup(const uint16_t* codes, uint32_t b) { return codes && (codes[b] & 8u); }
// The code per block (u16, after D; K0 writes its prestored there, the worklist kernel adds
// the dup bit):
// prestored in bits 1:0, bit 2 = a full uniform block with 1 <= b <= nblk - 2 (a dedupe
// candidate), its byte value in 15:8, bit 3 = a dup
__host__ __device__ __forceinline__ uint16_t* wl_codes(uint32_t* wl, uint64_t cap) {
    return reinterpret_cast<uint16_t*>(wl + ((WL_HDR + 5 * cap + 3) & ~3ull));   // 16-byte aligned
}
__host__ __device__ __forceinline__ const uint16_t* wl_codes(const uint32_t* wl, uint64_t cap) {
    return reinterpret_cast<const uint16_t*>(wl + ((WL_HDR + 5 * cap + 3) & ~3ull));
}
__device__ __forceinline__ void wl_hint_put(const uint32_t* __restrict__ wl, int k, uint32_t v) {
    uint32_t* h = reinterpret_cast<uint32_t*>((uint64_t)wl[WL_HINT] | ((uint64_t)wl[WL_HINT + 1] << 32));
    if (h) __hip_atomic_store(&h[k], v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
}
// K4 never sees block x: a stored block of the whole-copy prefix (above)
__device__ __forceinline__ bool wl_skip(uint32_t x, uint32_t M, uint32_t nblk) {
    return x >= 1 && x < M && x + 1 < nblk;
}
// The bytes [A, P) of the stream that the skipped blocks 1 .. R - 1 (R = min(M, nblk - 1))
// occupy, at their speculative offsets (the true ones inside the stored prefix); empty when
// there are none.  Nothing after K0 may write there: the apply launch zeroes the words the
// other blocks share around that range byte by byte (zero_word_keep).
__device__ __forceinline__ uint64_t spec_stored_bit(uint32_t b, uint32_t sw, uint32_t flags);
__device__ __forceinline__ void wl_prefix_bytes(uint32_t M, uint32_t nblk, uint32_t sw, uint32_t flags,
                                                uint64_t& A, uint64_t& P) {
    const uint32_t R = M < nblk - 1 ? M : nblk - 1;
    A = P = 0;
    if (nblk >= 1 && R >= 2) { A = spec_stored_bit(1, sw, flags) >> 3; P = spec_stored_bit(R, sw, flags) >> 3; }
}
// zero output word w except its bytes in [A, P)
__device__ __forceinline__ void zero_word_keep(uint32_t* out32, uint64_t w, uint64_t A, uint64_t P) {
    const uint64_t q0 = 4 * w;
    if (q0 + 4 <= A || q0 >= P) { out32[w] = 0; return; }
    uint8_t* o8 = reinterpret_cast<uint8_t*>(out32);
    for (uint32_t i = 0; i < 4; i++)
        if (q0 + i < A || q0 + i >= P) o8[q0 + i] = 0;
}

// prestored: 0 = parse in K1; 1 = stored by the noise check; 2 = a block of one repeated
// byte, parsed here in closed form (K1 skips it, the Huffman kernels code it); 3 = stored,
// and its interior already written to the stream at the offset it has when every block
// before it is stored too (below; the pack kernel then writes only the rest).
//
// The speculative copy: block b of a stream whose blocks 0..b-1 are all stored starts at bit
// start + 8 b (sw + 5) (each stored block: one header byte with its 3 bits, LEN/NLEN, sw data
// bytes).  A stored block copies itself there -- the whole 16-byte output quads the pack
// kernel would copy (dmx_pack_kernel's stored path, same quads, same condition) -- while its
// input is still in L2 from the check, so on noise the input crosses HBM once and the pack
// kernel only writes the edges.  If an earlier block is not stored, the scan gives this block
// another offset; the pack kernel then writes the whole block and every other block writes
// all of its words, so a misplaced quad inside the stream is overwritten (words shared
// between blocks are zeroed by the scan first), and one past the stream's end is outside it.
__device__ __forceinline__ uint64_t spec_stored_bit(uint32_t b, uint32_t sw, uint32_t flags) {
    return ((flags & DMX_F_HEADER) ? 16ull : 0ull) + 8ull * (uint64_t)b * ((uint64_t)sw + 5);
}
// the stored block's 16-byte output quads with a whole 20-byte input window (the pack
// kernel's fast path); calls f(k, o0) for every such quad: output word gw0 + k, input offset o0
template <typename F>
__device__ __forceinline__ void stored_quads(uint64_t O, uint32_t bn, bool dal, uint32_t tid, uint32_t nthr, F f) {
    const uint32_t s0 = (uint32_t)(O & 31);
    const uint32_t P = (s0 + 3 + 7) & ~7u, B0 = (P + 32) >> 3;   // as the pack kernel: LEN/NLEN at P / 8, data at B0
    const uint32_t nwords = (uint32_t)(((uint64_t)P + 32 + 8ull * bn + 31) >> 5);   // (s0 + len_bits + 31) / 32
    const uint64_t gw0 = O >> 5;
    const uint32_t ks = 4 - (uint32_t)(gw0 & 3);
    const uint32_t nq = (dal && nwords > ks + 1) ? (nwords - 1 - ks) >> 2 : 0;
    for (uint32_t j = tid; j < nq; j += nthr) {
        const uint32_t k = ks + 4 * j;
        const int64_t o0 = (int64_t)(4 * k) - (int64_t)B0;
        if (o0 >= 0 && (uint64_t)((o0 & ~3ll) + 20) <= bn) f(k, o0);
    }
}
// The rest of a stored block at its speculative offset O (bit, byte-aligned) beyond K0's
// 16-byte quads (stored_quads): the header byte (BFINAL 0, BTYPE 00), LEN / NLEN, the words
// before and after the quads, any of the first two and last two quads that did not take the
// 20-byte fast path (as the pack kernel's stored path builds them); its two edge words by
// byte stores of its own bytes (a neighbour's bytes share them).  Threads r0, r0 + rstep, ...
// src(j) = data byte j of the block.
template <typename Src>
__device__ __forceinline__ void stored_rest(Src src, bool dal, uint32_t bn, uint64_t O,
                                            uint32_t r0, uint32_t rstep, uint32_t* __restrict__ out32) {
    const uint32_t s0 = (uint32_t)(O & 31), P = (s0 + 3 + 7) & ~7u, B0 = (P + 32) >> 3;
    const uint32_t nwords = (uint32_t)(((uint64_t)P + 32 + 8ull * bn + 31) >> 5);
    const uint32_t ebyte = B0 + bn;   // the block's end, in bytes from word O >> 5
    const uint64_t gw0 = O >> 5;
    const uint32_t ks = 4 - (uint32_t)(gw0 & 3);
    const uint32_t nq = (dal && nwords > ks + 1) ? (nwords - 1 - ks) >> 2 : 0;   // K0's quads (as its copy)
    const uint32_t lenw = (bn & 0xFFFFu) | ((~bn & 0xFFFFu) << 16);
    auto gen_byte = [&](uint32_t q) -> uint32_t {
        if (q >= B0) return (q - B0) < bn ? src(q - B0) : 0u;
        if (q >= (P >> 3)) return (lenw >> (8 * (q - (P >> 3)))) & 0xFFu;
        return 0u;   // the header byte (and the previous block's bytes below it: not written)
    };
    uint8_t* out8 = reinterpret_cast<uint8_t*>(out32 + gw0);
    auto put_word = [&](uint32_t k) {
        if (k == 0 || k == nwords - 1) {
            for (uint32_t q = 4 * k; q < 4 * k + 4; q++)
                if (q >= (s0 >> 3) && q < ebyte) out8[q] = (uint8_t)gen_byte(q);
        } else {
            uint32_t v = 0;
            for (uint32_t i = 0; i < 4; i++) v |= gen_byte(4 * k + i) << (8 * i);
            out32[gw0 + k] = v;
        }
    };
    auto fast = [&](uint32_t j) {
        const int64_t o0 = (int64_t)(4 * (ks + 4 * j)) - (int64_t)B0;
        return o0 >= 0 && (uint64_t)((o0 & ~3ll) + 20) <= bn;
    };
    const uint32_t kq = nq ? ks + 4 * nq : 0;
    const uint32_t nrest = nq ? ks + (nwords - kq) : nwords;   // words outside the quads
    for (uint32_t r = r0; r < nrest + 16; r += rstep) {
        if (r < nrest) {
            put_word(nq ? (r < ks ? r : kq + (r - ks)) : r);
        } else if (nq >= 4) {   // quads 0, 1, nq - 2, nq - 1 that are not fast
            const uint32_t t = r - nrest, qi = t >> 2;
            const uint32_t j = qi < 2 ? qi : nq - 4 + qi;
            if (!fast(j)) put_word(ks + 4 * j + (t & 3));
        }
    }
}

__device__ __forceinline__ void stored_rest(const uint8_t* __restrict__ d, uint32_t bn, uint64_t O,
                                            uint32_t r0, uint32_t rstep, uint32_t* __restrict__ out32) {
    stored_rest([&](uint32_t j) -> uint32_t { return d[j]; }, (reinterpret_cast<uintptr_t>(d) & 3) == 0, bn, O, r0,
                rstep, out32);
}
// SPEC (work-list mode, when most blocks were stored in the previous encode): a full block's
// eight chunks per thread are loaded before pass 0 decides anything, so the block's whole
// input is in flight during pass 0's test and barriers; otherwise (text: pass 0 rejects the
// block) they are loaded only for blocks that pass it.
template <bool SPEC>
__device__ __forceinline__ uint32_t store_check_block(const uint8_t* __restrict__ in, uint64_t n, uint32_t sw,
                                                      dmx_blkinfo* __restrict__ info, uint32_t* __restrict__ tok_g,
                                                      uint32_t* __restrict__ hist_g, uint32_t uni_ok, uint32_t flags,
                                                      uint32_t* __restrict__ out32, uint64_t out_cap) {
    __shared__ uint32_t bm[1u << 12];   // the 17-bit presence bitmap (16 KB: 8 workgroups per CU)
    __shared__ uint32_t hist[256];
    __shared__ uint64_t red[10][SCT / 64];
    __shared__ uint32_t pass_s;
    const uint32_t tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
    const uint32_t b = blockIdx.x;
    const uint64_t off = (uint64_t)b * sw;
    const uint32_t bn = (uint32_t)((n - off) < sw ? (n - off) : sw);
    const uint8_t* d = in + off;
    const uint32_t nblk = gridDim.x;
    if (bn < 4096) {
        if (tid == 0) info[b].prestored = 0;
        return 0u;
    }
    const bool aligned16 = ((reinterpret_cast<uintptr_t>(d) & 15) == 0);
    const bool full = aligned16 && bn == SCT * 16 * 8;
    uint4 v[8];
    // the 4 bytes after chunk i (for the 4-grams that straddle it) are the next lane's v[i].x
    // (DPP), except on lane 63, whose eight are held by lanes 0 .. 7 of nx63 (7 VGPRs fewer)
    uint32_t nx63 = 0;
    auto load_full = [&]() {
#pragma unroll
        for (int i = 0; i < 8; i++) v[i] = *reinterpret_cast<const uint4*>(d + ((tid + i * SCT) << 4));
        const uint32_t p63 = (((tid | 63u) + lane * SCT) << 4) + 16;
        nx63 = lane < 8 && p63 < bn ? *reinterpret_cast<const uint32_t*>(d + p63) : 0u;
    };
    auto next4 = [&](int i) -> uint32_t {
        const uint32_t nl = (uint32_t)__builtin_amdgcn_update_dpp(0, (int)v[i].x, 0x130, 0xF, 0xF, false);
        return lane == 63 ? (uint32_t)__builtin_amdgcn_readlane((int)nx63, i) : nl;
    };
    if (SPEC && full) load_full();
    // ---- pass 0: bit planes of the first 4096 bytes, one 16-byte load per thread ----
    {
        uint32_t w[5];
        if (SPEC && full) {   // chunk tid is v[0]
            w[0] = v[0].x; w[1] = v[0].y; w[2] = v[0].z; w[3] = v[0].w; w[4] = 0;   // (w[4] unused here)
        } else {
            sc_load(d, tid << 4, bn, aligned16, w);
        }
        uint32_t ones[8];
#pragma unroll
        for (int k = 0; k < 8; k++) {
            ones[k] = 0;
#pragma unroll
            for (int q = 0; q < 4; q++) ones[k] += __builtin_popcount(w[q] & (0x01010101u << k));
            ones[k] = wave_sum_u32(ones[k]);
        }
        if (lane == 0) {
#pragma unroll
            for (int k = 0; k < 8; k++) red[k][wave] = ones[k];
        }
        const uint32_t c4 = (uint32_t)d[0] * 0x01010101u;
        const bool u0 = w[0] == c4 && w[1] == c4 && w[2] == c4 && w[3] == c4;
        const bool uni4k = __syncthreads_and(u0) != 0;   // (also publishes red[])
        if (tid == 0) {
            bool ok = true;
            for (int k = 0; k < 8; k++) {
                int64_t o = 0;
#pragma unroll
                for (int w2 = 0; w2 < SCT / 64; w2++) o += (int64_t)red[k][w2];
                const int64_t dv = 2 * o - (int64_t)SC_PLANE;
                ok = ok && 8 * (dv < 0 ? -dv : dv) <= (int64_t)SC_PLANE;
            }
            pass_s = ok ? 1u : 0u;
            if (!ok) info[b].prestored = 0;
        }
        __syncthreads();
        if (!pass_s) {
            if (!uni_ok || !uni4k) return 0u;
            // the first 4 KiB are one repeated byte: is the whole block?  Then its parse has
            // a closed form (as in K1's uniform path; no dictionary): a literal, distance-1
            // matches of min(258, bytes left) while >= 3 bytes are left, then literals.
            bool u = true;
            for (uint32_t p = (tid + SCT) << 4; p < bn; p += SCT << 4) {
                uint32_t x[5];
                sc_load(d, p, bn, aligned16, x);
                const uint32_t nb = bn - p < 16 ? bn - p : 16;
#pragma unroll
                for (int q = 0; q < 4; q++) {
                    const uint32_t m = 4 * q + 4 <= (int)nb ? 0xFFFFFFFFu : (4 * q >= nb ? 0u : (1u << (8 * (nb - 4 * q))) - 1u);
                    u = u && ((x[q] ^ c4) & m) == 0;
                }
            }
            if (!__syncthreads_and(u)) return 0u;
            uint32_t* H = bm;   // the 320-entry histogram (bm is free here)
            for (uint32_t k = tid; k < DMX_HIST; k += SCT) H[k] = 0;
            __syncthreads();
            const uint32_t c = c4 & 0xFFu;
            const uint32_t nt = uniform_parse(bn, c, tok_g + (uint64_t)b * DMX_BLK, H, tid, SCT);
            if (tid == 0) {
                const uint64_t S = (uint64_t)c * bn, T = (uint64_t)c * ((uint64_t)bn * (bn - 1) / 2);
                info[b].ntok = nt;
                info[b].n = bn;
                info[b].adl_s = S;
                info[b].adl_w = (uint64_t)bn * S - T;
                // 2, and for a full block that is neither the first nor the last (a dedupe
                // candidate, the work lists) bit 2 and its byte value in bits 15:8
                info[b].prestored = 2u | ((bn == sw && b >= 1 && b + 2 <= nblk) ? 4u | (c << 8) : 0u);
            }
            __syncthreads();
            for (uint32_t k = tid; k < DMX_HIST; k += SCT) hist_g[(uint64_t)b * DMX_HIST + k] = H[k];
            return 2u | ((bn == sw && b >= 1 && b + 2 <= nblk) ? 4u | (c << 8) : 0u);
        }
    }
    // ---- pass 1: Adler sums (the block's data into registers for pass 2) ----
    uint64_t s = 0, t = 0;
    auto chunk1 = [&](uint32_t p, const uint32_t* w) {   // 16 bytes at block offset p
        uint32_t ts = 0, tt = 0;
#pragma unroll
        for (int q = 0; q < 4; q++) {
            ts = __builtin_amdgcn_sad_u8(w[q], 0u, ts);                                  // sum of bytes
            tt = __builtin_amdgcn_udot4(w[q], 0x03020100u + 0x04040404u * q, tt, false);  // sum of j * byte
        }
        s += ts;
        t += (uint64_t)p * ts + tt;
    };
    // full 32 KiB block: all loads in flight at once, and the data stays in registers for
    // pass 2 (w4: the 4 bytes after each chunk, for the 4-grams that straddle it)
    if (full) {
        if (!SPEC) load_full();
#pragma unroll
        for (int i = 0; i < 8; i++) {
            const uint32_t w[4] = {v[i].x, v[i].y, v[i].z, v[i].w};
            chunk1((tid + i * SCT) << 4, w);
        }

    } else {
        for (uint32_t p = tid << 4; p < bn; p += SCT << 4) {
            uint32_t w[5];
            sc_load(d, p, bn, aligned16, w);
            chunk1(p, w);
        }
    }
    s = wave_sum_u64(s);
    t = wave_sum_u64(t);
    if (lane == 0) {
        red[8][wave] = s;
        red[9][wave] = t;
    }
    // ---- pass 2: byte histogram + 4-gram bitmap ----
    for (uint32_t k = tid; k < (1u << 12) / 4; k += SCT) reinterpret_cast<uint4*>(bm)[k] = make_uint4(0, 0, 0, 0);
    hist[tid] = 0;   // (8 padded sub-histograms by lane & 7 measured slower: 0.59 -> 0.77 ms per GiB)
    __syncthreads();
    uint32_t qn = 0;   // sampled 4-grams of this thread
    // histogram stride s = 8 / 4 / 2 / 1 for blocks of >= 32768 / 16384 / 8192 / 4096 bytes
    const uint32_t smask = bn >= 32768 ? 7u : bn >= 16384 ? 3u : bn >= 8192 ? 1u : 0u;
    // (a per-lane loop over only the sampled positions -- about 6 ds_or per chunk for the wave
    // instead of 16 masked ones -- measured slower: 79 VGPRs, 510 -> 745 us on C4)
    auto chunk2 = [&](uint32_t p, const uint32_t* w) {   // 16 positions at block offset p (w[4]: next 4 bytes)
#pragma unroll
        for (int j = 0; j < 16; j++) {
            const uint32_t lo = w[j >> 2], hi = w[(j >> 2) + 1];
            const uint32_t g4 = (j & 3) ? __builtin_amdgcn_alignbyte(hi, lo, (uint32_t)(j & 3)) : lo;
            if (((uint32_t)j & smask) == 0 && p + j < bn) atomicAdd(&hist[(lo >> (8 * (j & 3))) & 0xFFu], 1u);
            const uint32_t x = g4 * 0x9E3779B1u;
            if (p + j + 4 <= bn && !(x & (7u << 11))) {   // sampled by content
                qn++;
                atomicOr(&bm[x >> 20], 1u << ((x >> 15) & 31));
            }
        }
    };
    if (full) {
#ifndef DMX_K0_NOPASS2   // (timing knockout, tools/build_var.sh)
#pragma unroll
        for (int i = 0; i < 8; i++) {
            const uint32_t w[5] = {v[i].x, v[i].y, v[i].z, v[i].w, next4(i)};
            chunk2((tid + i * SCT) << 4, w);
        }
#endif
    } else {
        for (uint32_t p = tid << 4; p < bn; p += SCT << 4) {
            uint32_t w[5];
            sc_load(d, p, bn, aligned16, w);
            chunk2(p, w);
        }
    }
    __syncthreads();
    uint64_t distinct = 0;
    for (uint32_t k = tid; k < (1u << 12); k += SCT) distinct += __builtin_popcount(bm[k]);
    const uint64_t hc = hist[tid];
    uint64_t s2 = hc * hc;
    distinct = wave_sum_u64(distinct);
    s2 = wave_sum_u64(s2);
    const uint64_t qw = wave_sum_u64((uint64_t)qn);
    __syncthreads();   // red[] reused
    if (lane == 0) { red[0][wave] = distinct; red[1][wave] = s2; red[2][wave] = qw; }
    __syncthreads();
    if (tid == 0) {
        uint64_t S = 0, T = 0, Dn = 0, S2 = 0, Q = 0;
#pragma unroll 1   // (one wave's partials at a time: all 20 u64 at once spilled at 64 VGPRs)
        for (int w = 0; w < SCT / 64; w++) {
            S += red[8][w]; T += red[9][w]; Dn += red[0][w]; S2 += red[1][w]; Q += red[2][w];
        }
        const uint64_t m = ((uint64_t)bn + smask) / (smask + 1), m2 = m * m;
        const uint64_t coll = Q - Dn;
#ifdef DMX_K0_NOPASS2
        const bool sto = (S2 | coll | m2 | 1) != 0;
#else
        const bool sto = 256 * S2 <= m2 + (m2 >> 4) + 256 * m && 16 * Q >= (uint64_t)bn && 64 * coll <= 4 * Q;
#endif
        // the speculative copy (above) when the whole block fits the output at that offset
        const bool spec = sto && (spec_stored_bit(b, sw, flags) >> 3) + (uint64_t)bn + 16 <= out_cap;
        info[b].prestored = sto ? (spec ? 3u : 1u) : 0u;
        pass_s = spec ? 1u : 0u;
#ifdef DMX_K0_NOCOPY
        pass_s = 0;
#endif
        if (sto) {
            info[b].ntok = 0;
            info[b].n = bn;
            info[b].adl_s = S;
            info[b].adl_w = (uint64_t)bn * S - T;
            info[b].btype = 0;
            info[b].hdr_bits = 3;
            info[b].body_bits = 0;
            info[b].nsub = 1;
        }
    }
    __syncthreads();
    if (pass_s && full) {
        // full block: the quads from pass 1's registers.  Quad j (output word gw0 + ks + 4 j)
        // holds input bytes [o0, o0 + 16), o0 = 16 j + R: chunk c = j (R >= 0) or j - 1 (R < 0)
        // and the next chunk, which the next lane holds (DPP); lane 63's next chunk is in
        // another wave, so its quads re-read the input (L2) as the general path does.
        const uint64_t O = spec_stored_bit(b, sw, flags);
        const uint32_t s0 = (uint32_t)(O & 31), P = (s0 + 3 + 7) & ~7u, B0 = (P + 32) >> 3;
        const uint32_t nwords = (uint32_t)(((uint64_t)P + 32 + 8ull * bn + 31) >> 5);
        const uint64_t gw0 = O >> 5;
        const uint32_t ks = 4 - (uint32_t)(gw0 & 3);
        const uint32_t nq = nwords > ks + 1 ? (nwords - 1 - ks) >> 2 : 0;
        const int32_t R = (int32_t)(4 * ks) - (int32_t)B0;
        const uint32_t r = (uint32_t)(R & 15), a4 = r >> 2, sh = r & 3, jadd = R < 0 ? 1u : 0u;
#pragma unroll
        for (int i = 0; i < 8; i++) {
            const uint32_t c = tid + (uint32_t)i * SCT, j = c + jadd;
            const int64_t o0 = 16 * (int64_t)j + R;
            const uint32_t n0 = (uint32_t)__builtin_amdgcn_update_dpp(0, (int)v[i].x, 0x130, 0xF, 0xF, false);
            const uint32_t n1 = (uint32_t)__builtin_amdgcn_update_dpp(0, (int)v[i].y, 0x130, 0xF, 0xF, false);
            const uint32_t n2 = (uint32_t)__builtin_amdgcn_update_dpp(0, (int)v[i].z, 0x130, 0xF, 0xF, false);
            const uint32_t n3 = (uint32_t)__builtin_amdgcn_update_dpp(0, (int)v[i].w, 0x130, 0xF, 0xF, false);
            if (j >= nq || o0 < 0 || (uint64_t)((o0 & ~3ll) + 20) > bn) continue;   // not one of the quads
            uint32_t w[5];
            if (lane != 63) {
                const uint32_t e8[8] = {v[i].x, v[i].y, v[i].z, v[i].w, n0, n1, n2, n3};
#pragma unroll
                for (int q = 0; q < 5; q++) w[q] = a4 == 0 ? e8[q] : a4 == 1 ? e8[q + 1] : a4 == 2 ? e8[q + 2] : e8[q + 3];
            } else {
                const uint32_t* p32 = reinterpret_cast<const uint32_t*>(d + (o0 & ~3ll));
#pragma unroll
                for (int q = 0; q < 5; q++) w[q] = p32[q];
            }
            uint4 o;
            o.x = sh ? __builtin_amdgcn_alignbyte(w[1], w[0], sh) : w[0];
            o.y = sh ? __builtin_amdgcn_alignbyte(w[2], w[1], sh) : w[1];
            o.z = sh ? __builtin_amdgcn_alignbyte(w[3], w[2], sh) : w[2];
            o.w = sh ? __builtin_amdgcn_alignbyte(w[4], w[3], sh) : w[3];
            *reinterpret_cast<uint4*>(&out32[gw0 + ks + 4 * j]) = o;
        }
        // The rest of the block (what stored_rest writes; then a block of the stored prefix
        // is complete, and at any other offset the scan's edge zeroing and K4 overwrite it),
        // from registers: wave 0 the words before the quads (header byte, LEN / NLEN, the first
        // data bytes) and quads 0, 1 if not fast; the last wave quads nq - 2, nq - 1 if not fast
        // and the words after them.  Source words by ds_bpermute from the wave's lanes (chunks
        // base .. base + 63 in slot I).  (Staged through LDS after a barrier it cost 20 us on
        // C4, with global byte loads 42 us; the fill kernel that did it took 10.5 us.)
#ifndef DMX_K0_NOREST   // (A/B knockout: the fill kernel then writes the rest)
        if (wave == 0 || wave == SCT / 64 - 1) {
            const bool front = wave == 0;
            const uint4 vv = front ? v[0] : v[7];
            const int32_t base = (int32_t)(wave * 64 + (front ? 0 : 7) * SCT);
            auto dword = [&](int32_t iw) -> uint32_t {   // input word iw, 0 outside the wave's chunks
                const int32_t src = (iw >> 2) - base;
                const bool ok = iw >= 0 && src >= 0 && src < 64 && 4 * iw < (int32_t)bn;
                const int a = (ok ? src : 0) << 2;
                const uint32_t x = (uint32_t)__builtin_amdgcn_ds_bpermute(a, (int)vv.x);
                const uint32_t y = (uint32_t)__builtin_amdgcn_ds_bpermute(a, (int)vv.y);
                const uint32_t z = (uint32_t)__builtin_amdgcn_ds_bpermute(a, (int)vv.z);
                const uint32_t w = (uint32_t)__builtin_amdgcn_ds_bpermute(a, (int)vv.w);
                const uint32_t c = (uint32_t)iw & 3u;
                return ok ? (c == 0 ? x : c == 1 ? y : c == 2 ? z : w) : 0u;
            };
            auto fastq = [&](uint32_t jq) {
                const int64_t q0 = (int64_t)(4 * (ks + 4 * jq)) - (int64_t)B0;
                return q0 >= 0 && (uint64_t)((q0 & ~3ll) + 20) <= bn;
            };
            uint32_t k;
            bool want;
            if (front) {
                k = lane;
                want = lane < ks || (lane < ks + 8 && !fastq((lane - ks) >> 2));
            } else {
                k = ks + 4 * (nq - 2) + lane;
                want = lane < 8 ? !fastq(nq - 2 + (lane >> 2)) : k < nwords;
            }
            const int32_t off = (int32_t)(4 * k) - (int32_t)B0;   // the word's first byte in the block's data
            const int32_t iw = off >> 2;                           // (floor)
            const uint32_t d0 = dword(iw), d1 = dword(iw + 1), sh2 = (uint32_t)off & 3u;
            uint32_t val = sh2 ? __builtin_amdgcn_alignbyte(d1, d0, sh2) : d0;
            const uint32_t lenw = (bn & 0xFFFFu) | ((~bn & 0xFFFFu) << 16);
            if (off < 0) {   // bytes below B0: the header byte (0) and LEN / NLEN
#pragma unroll
                for (uint32_t i = 0; i < 4; i++) {
                    const uint32_t q = 4 * k + i;
                    if (q < B0) {
                        const uint32_t hb = q >= (P >> 3) ? (lenw >> (8 * (q - (P >> 3)))) & 0xFFu : 0u;
                        val = (val & ~(0xFFu << (8 * i))) | (hb << (8 * i));
                    }
                }
            }
            if (want && nq >= 4) {
                if (k == 0 || k == nwords - 1) {   // edge words: this block's bytes only
                    uint8_t* o8 = reinterpret_cast<uint8_t*>(out32 + gw0);
                    const uint32_t ebyte = B0 + bn;
#pragma unroll
                    for (uint32_t i = 0; i < 4; i++) {
                        const uint32_t q = 4 * k + i;
                        if (q >= (s0 >> 3) && q < ebyte) o8[q] = (uint8_t)(val >> (8 * i));
                    }
                } else {
                    out32[gw0 + k] = val;
                }
            }
        }
#endif
    } else if (pass_s) {
        const uint64_t O = spec_stored_bit(b, sw, flags);
        const bool dal = (reinterpret_cast<uintptr_t>(d) & 3) == 0;
        stored_quads(O, bn, dal, tid, SCT, [&](uint32_t k, int64_t o0) {
            const uint32_t* p32 = reinterpret_cast<const uint32_t*>(d + (o0 & ~3ll));
            const uint32_t w0 = p32[0], w1 = p32[1], w2 = p32[2], w3 = p32[3], w4 = p32[4];
            const uint32_t sh = (uint32_t)(o0 & 3);
            uint4 v;
            v.x = sh ? __builtin_amdgcn_alignbyte(w1, w0, sh) : w0;
            v.y = sh ? __builtin_amdgcn_alignbyte(w2, w1, sh) : w1;
            v.z = sh ? __builtin_amdgcn_alignbyte(w3, w2, sh) : w2;
            v.w = sh ? __builtin_amdgcn_alignbyte(w4, w3, sh) : w3;
            *reinterpret_cast<uint4*>(&out32[(O >> 5) + k]) = v;
        });
    }
    return info[b].prestored;   // (the caller stores thread 0's)
}

// K0 (DMX_F_STORE_CHECK): the noise check of one block (store_check_block); with the work
// lists, thread 0 also writes the block's code (its prestored) to the list builder's array --
// in one place after the body, where its address costs no register through the body.
template <bool SPEC>
__global__ __launch_bounds__(SCT) void dmx_store_check_kernel(const uint8_t* __restrict__ in, uint64_t n, uint32_t sw,
                                                              dmx_blkinfo* __restrict__ info, uint32_t* __restrict__ tok_g,
                                                              uint32_t* __restrict__ hist_g, uint32_t uni_ok, uint32_t flags,
                                                              uint32_t* __restrict__ out32, uint64_t out_cap,
                                                              uint16_t* __restrict__ codes) {
    const uint32_t code = store_check_block<SPEC>(in, n, sw, info, tok_g, hist_g, uni_ok, flags, out32, out_cap);
    if (codes && threadIdx.x == 0) codes[blockIdx.x] = (uint16_t)code;
}

// The work lists from K0's prestored values: one launch, a workgroup per tile of WLC x WLT
// blocks.  Deterministic block order without a chip-wide scan: the workgroup of tile t first
// counts the kinds of every block before its tile (codes [0, t TS), u16 x 8 per load, at most
// nblk codes -- 64 KB at 1 GiB -- all loads in flight), which gives its lists' offsets, then
// writes its tile's entries in block order (ballot ranks per (step, wave), a scan of those
// counts).  The last tile's workgroup has then seen every block: it writes the list header
// (counts, M, K1's claim counter and K4's list zeroed) and the hint.  (Round 5's first builder
// was one workgroup sweeping every block twice: 21 us at 32 768 blocks, latency-bound; this
// one reads each code at most once per workgroup and its workgroups run side by side.)
// The prefix sweeps add up to ntile^2 / 2 x 8 KB of (L2 / MALL) reads: nothing at 1 GiB (8
// tiles), 64 MB at 16 GiB (128 tiles), ~20 GB at 288 GB -- small against those encodes'
// own traffic; the last tile's sweep is ~275 rounds of 4 x 16-byte loads per thread there.
// Dedupe: each byte value's representative is its first full uniform block in the stream, so
// for a tile it is either before the tile (the prefix sweep sees it) or inside it; the dups
// before the tile number (candidates before it) - (byte values among them).
#define WLT 1024
#define WLC 4
__global__ __launch_bounds__(WLT) void dmx_worklist_kernel(uint32_t nblk, uint32_t* __restrict__ wl, uint64_t cap,
                                                           uint32_t dedupe) {
    constexpr uint32_t TS = WLC * WLT;
    __shared__ uint32_t cnt[3][WLC * (WLT / 64)];   // per (j, wave) of the tile: list entries, then their offsets
    __shared__ uint32_t wsum[3], rep[256], red[4], mmin, tot[3];
    const uint32_t tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
    const uint64_t lt = (1ull << lane) - 1ull;
    const uint32_t t0 = blockIdx.x * TS;
    const bool last = blockIdx.x + 1 == gridDim.x;
    if (tid < 256) rep[tid] = 0xFFFFFFFFu;
    if (tid < 4) red[tid] = 0;
    if (tid == 0) mmin = nblk;
    __syncthreads();
    uint16_t* K = wl_codes(wl, cap);
    uint32_t* L1 = wl + WL_HDR;
    uint32_t* L2 = L1 + cap;
    uint32_t* L5 = L1 + 3 * cap;
    uint32_t* Dp = L1 + 4 * cap;
    // the prefix sweep (blocks [0, t0)): prestored-0 and -2 counts, candidates, their byte
    // values (rep: the first candidate per value), the first block that is not prestored 3
    uint32_t a0 = 0, a2 = 0, ac = 0, m = nblk, lastc = 0xFFFFFFFFu;
    auto see = [&](uint32_t k, uint32_t b) {
        const uint32_t ps = k & 3u;
        a0 += ps == 0;
        a2 += ps == 2;
        if (ps != 3u) m = min(m, b);
        if (k & 4u) {
            ac++;
            // a thread's blocks ascend: its first block of a byte value is its candidate
            if (dedupe && (k >> 8) != lastc) atomicMin(&rep[k >> 8], b);
            lastc = k >> 8;
        }
    };
    {
        const uint4* K8 = reinterpret_cast<const uint4*>(K);   // (16-byte aligned, t0 a multiple of 8)
        const uint32_t nq = t0 >> 3;
        for (uint32_t q0 = 0; q0 < nq; q0 += 4 * WLT) {
            uint4 v[4];
#pragma unroll
            for (uint32_t i = 0; i < 4; i++) {
                const uint32_t q = q0 + i * WLT + tid;
                v[i] = q < nq ? K8[q] : make_uint4(0x00030003u, 0x00030003u, 0x00030003u, 0x00030003u);
            }
#pragma unroll
            for (uint32_t i = 0; i < 4; i++) {
                const uint32_t bb = (q0 + i * WLT + tid) << 3;
                const uint32_t w[4] = {v[i].x, v[i].y, v[i].z, v[i].w};
#pragma unroll
                for (uint32_t e = 0; e < 4; e++) {   // two codes per word, counted in bit-parallel
                    const uint32_t x = w[e] & 0x00070007u;
                    const uint32_t z0 = ~(x | (x >> 1)) & 0x00010001u, z2 = (x >> 1) & ~x & 0x00010001u;
                    const uint32_t n3 = ~(x & (x >> 1)) & 0x00010001u, zc = (x >> 2) & 0x00010001u;
                    a0 += __builtin_popcount(z0);
                    a2 += __builtin_popcount(z2);
                    ac += __builtin_popcount(zc);
                    if (n3 && m == nblk) m = bb + 2 * e + ((n3 & 1u) ? 0u : 1u);   // (this thread's blocks ascend)
                    if (dedupe && zc) {
#pragma unroll
                        for (uint32_t h = 0; h < 2; h++) {
                            const uint32_t k = (w[e] >> (16 * h)) & 0xFFFFu;
                            if ((k & 4u) && (k >> 8) != lastc) atomicMin(&rep[k >> 8], bb + 2 * e + h);
                            if (k & 4u) lastc = k >> 8;
                        }
                    }
                }
            }
        }
    }
    const uint32_t p0 = a0, p2 = a2, pc = ac;   // this thread's prefix counts
    // the tile's codes (block b = t0 + j WLT + tid): they add to rep and (last tile) the totals
    uint32_t kc[WLC];   // code in bits 15:0, its kind (1 | 2 | 4) in bits 18:16
#pragma unroll
    for (uint32_t j = 0; j < WLC; j++) {
        const uint32_t b = t0 + j * WLT + tid;
        kc[j] = b < nblk ? (uint32_t)K[b] : 3u;
    }
    lastc = 0xFFFFFFFFu;
#pragma unroll
    for (uint32_t j = 0; j < WLC; j++) see(kc[j], t0 + j * WLT + tid);
    {
        const uint32_t s0 = wave_sum_u32(p0), s2 = wave_sum_u32(p2), sc = wave_sum_u32(pc), sa = wave_sum_u32(ac);
        if (lane == 0) {
            if (s0) atomicAdd(&red[0], s0);
            if (s2) atomicAdd(&red[1], s2);
            if (sc) atomicAdd(&red[2], sc);
            if (sa) atomicAdd(&red[3], sa);
        }
        if (m < nblk) atomicMin(&mmin, m);
    }
    __syncthreads();
    if (wave == 0) {   // the byte values with a candidate before the tile, and the list offsets
        uint32_t dv = 0;
#pragma unroll
        for (uint32_t q = 0; q < 4; q++) dv += (uint32_t)__popcll(__ballot(rep[q * 64 + lane] < t0));
        if (lane == 0) {
            const uint32_t dups = dedupe ? red[2] - dv : 0u;
            tot[0] = red[0];
            tot[1] = red[0] + red[1] - dups;
            tot[2] = dups;
        }
    }
    // per block: 1 = K1 parses it, 2 = K2 codes it, 4 = a dup (of r)
    auto kind = [&](uint32_t k, uint32_t b, uint32_t& r) -> uint32_t {
        r = 0xFFFFFFFFu;
        const uint32_t ps = k & 3u;
        if (ps == 0) return 3u;
        if (ps != 2) return 0u;
        if (dedupe && (k & 4u)) {
            const uint32_t rr = rep[k >> 8];
            if (rr != b) { r = rr; return 4u; }
        }
        return 2u;
    };
#pragma unroll
    for (uint32_t j = 0; j < WLC; j++) {
        const uint32_t b = t0 + j * WLT + tid;
        uint32_t r;
        const uint32_t t = b < nblk ? kind(kc[j], b, r) : 0u;
        kc[j] |= t << 16;
        const uint64_t m1 = __ballot(t & 1u), m2 = __ballot(t & 2u), m5 = __ballot(t & 4u);
        if (lane == 0) {
            cnt[0][j * (WLT / 64) + wave] = (uint32_t)__popcll(m1);
            cnt[1][j * (WLT / 64) + wave] = (uint32_t)__popcll(m2);
            cnt[2][j * (WLT / 64) + wave] = (uint32_t)__popcll(m5);
        }
    }
    __syncthreads();
    // exclusive scans of the three count tables (WLC x 16 entries each, j-major), by waves
    // 0 .. 2: WLC / 4 entries per lane
    if (wave < 3) {
        uint32_t* T = cnt[wave];
        uint32_t v[WLC / 4], sum = 0;
#pragma unroll
        for (uint32_t q = 0; q < WLC / 4; q++) { v[q] = T[lane * (WLC / 4) + q]; sum += v[q]; }
        const uint32_t incl = wave_incl_scan(sum);
        uint32_t run = tot[wave] + incl - sum;
#pragma unroll
        for (uint32_t q = 0; q < WLC / 4; q++) { T[lane * (WLC / 4) + q] = run; run += v[q]; }
        if (lane == 63) wsum[wave] = tot[wave] + incl;
    }
    __syncthreads();
#pragma unroll
    for (uint32_t j = 0; j < WLC; j++) {
        const uint32_t b = t0 + j * WLT + tid;
        const uint32_t t = kc[j] >> 16;
        const uint64_t m1 = __ballot(t & 1u), m2 = __ballot(t & 2u), m5 = __ballot(t & 4u);
        if (t & 1u) L1[cnt[0][j * (WLT / 64) + wave] + (uint32_t)__popcll(m1 & lt)] = b;
        if (t & 2u) L2[cnt[1][j * (WLT / 64) + wave] + (uint32_t)__popcll(m2 & lt)] = b;
        if (t & 4u) {   // a dup: its representative, and bit 3 of its code (what the kernels test)
            L5[cnt[2][j * (WLT / 64) + wave] + (uint32_t)__popcll(m5 & lt)] = b;
            uint32_t r;
            kind(kc[j] & 0xFFFFu, b, r);
            Dp[b] = r;
            K[b] = (uint16_t)((kc[j] & 0xFFFFu) | 8u);
        }
    }
    if (last && tid == 0) {   // every block seen: the header and the hint
        wl[WL_N1] = wsum[0];
        wl[WL_C1] = 0;
        wl[WL_N2] = wsum[1];
        wl[WL_N4] = 0;
        wl[WL_M] = mmin;
        wl[WL_N5] = wsum[2];
        wl_hint_put(wl, 0, nblk);
        wl_hint_put(wl, 1, wsum[0]);
        wl_hint_put(wl, 2, wsum[1]);
        wl_hint_put(wl, 4, red[3]);
    }
}

// After K4 (work-list mode), the blocks K4 skipped (a wave per 4 blocks), launched only when
// there are such blocks that K0 did not complete:
//  * a block of the stored prefix (wl_skip) that is not a full 16-byte aligned block gets the
//    bytes K0's speculative copy left out (stored_rest; K0 writes a full block's rest itself);
//  * a dup (uniform-block dedupe) gets its representative's bit string: output word k of the
//    dup holds the representative's bits shifted by the two offsets' difference, masked to
//    the dup's own bits (its two edge words, shared with its neighbours and zeroed by the
//    apply launch, by atomicOr).  The representative is complete: K4 packed it.
__global__ __launch_bounds__(256) void dmx_fill_kernel(const uint8_t* __restrict__ in, uint32_t sw, uint32_t flags,
                                                       const dmx_blkinfo* __restrict__ info,
                                                       const uint32_t* __restrict__ wl, uint64_t cap, uint32_t nblk,
                                                       uint32_t* __restrict__ out32, const dmx_result* __restrict__ res,
                                                       uint32_t dedupe) {
    if (res->status) return;
    // a wave covers the 4 blocks b0 .. b0 + 3
    const uint32_t lane = threadIdx.x & 63, b0 = (blockIdx.x * 4 + (threadIdx.x >> 6)) * 4;
    {   // a block of the stored prefix that K0 did not complete (not a full 16-byte aligned
        // block: K0 writes the rest of those itself), at its speculative offset: 16 lanes
        const uint32_t b = b0 + (lane >> 4);
        const uint8_t* d = in + (uint64_t)b * sw;
#ifdef DMX_K0_NOREST
        if (b < nblk && wl_skip(b, wl[WL_M], nblk))
#else
        if (b < nblk && wl_skip(b, wl[WL_M], nblk) && !(sw == SCT * 16 * 8 && (reinterpret_cast<uintptr_t>(d) & 15) == 0))
#endif
            stored_rest(d, sw, spec_stored_bit(b, sw, flags), lane & 15, 16, out32);
    }
    if (!dedupe) return;
    for (uint32_t i = 0; i < 4; i++) {   // dups: the whole wave per block
        const uint32_t b = b0 + i;
        if (b >= nblk || !(wl_codes(wl, cap)[b] & 8u)) continue;
        const uint32_t r = wl_dup(wl, cap)[b];
        const uint64_t Ob = info[b].off_bits, Or = info[r].off_bits, Lb = info[b].len_bits;
        const uint64_t gw0 = Ob >> 5;
        const uint32_t nwords = (uint32_t)(((Ob & 31) + Lb + 31) >> 5);
        for (uint32_t k = lane; k < nwords; k += 64) {
            const uint64_t lo = 32 * (gw0 + k), hi = lo + 32;                         // the word's bits
            const uint64_t a = lo > Ob ? lo : Ob, e = hi < Ob + Lb ? hi : Ob + Lb;   // its bits of the dup
            const uint64_t q = a - Ob + Or;                                            // their source bit
            const uint64_t qw = q >> 5;
            const uint32_t sh = (uint32_t)(q & 31);
            const uint64_t src = (uint64_t)out32[qw] | ((uint64_t)out32[qw + 1] << 32);
            const uint32_t nb = (uint32_t)(e - a);
            const uint64_t bits = (src >> sh) & ((1ull << nb) - 1ull);
            const uint32_t v = (uint32_t)(bits << (a - lo));
            if (nb == 32) out32[gw0 + k] = v;
            else atomicOr(&out32[gw0 + k], v);
        }
    }
}

// Diagnostic (a library variant built with -DDMX_DEBUG_STOP=1|2|3, never the product library): end the block after P0 (sort),
// P1 (search) or P2 (walk), recording it as an empty block, so that SQ counters of the
// truncated kernel give the instruction count of each phase by difference.  The stream
// of such an encode is not the input's.
__device__ __forceinline__ bool dbg_stop(uint32_t mflags, uint32_t phase, dmx_blkinfo* info, uint32_t* hist_g,
                                         uint32_t b, uint32_t bn, uint32_t tid) {
    if (((mflags >> 8) & 3u) != phase) return false;
    for (uint32_t k = tid; k < DMX_HIST; k += MT) hist_g[(uint64_t)b * DMX_HIST + k] = 0;
    if (tid == 0) {
        info[b].ntok = 0;
        info[b].n = bn;
        info[b].adl_s = 0;
        info[b].adl_w = 0;
        info[b].prestored = 0;
    }
    return true;
}

// DMX_F_DEEP (mflags & 8): the block's own chain depth, dmx_oracle_block_chain's rule --
// DMX_DEEP_CHAIN when 4 D < samples, D = the distinct buckets of the sampled positions
// p < bn - 2 with p mod 2048 < 256 (4 096 in a full block: 16 runs of 256).  Called by all
// threads after the staging barrier; L.hist (zero until P3) holds the 8192-bit bucket set
// and is zeroed again, L.ntok (zero until the walk) the count.  Two barriers.
__device__ __forceinline__ int32_t block_chain(MatchLDS& L, uint32_t bn, int32_t max_chain, uint32_t mflags,
                                               uint32_t tid) {
    const int32_t dk = (mflags >> 16) & 0xFFu ? (int32_t)((mflags >> 16) & 0xFFu) : (int32_t)DMX_DEEP_CHAIN;
    if (!(mflags & 8u) || max_chain <= 0 || max_chain >= dk) return max_chain;
    const uint32_t nvalid = bn > 2 ? bn - 2 : 0;
    uint32_t* SB = L.hist;
#pragma unroll
    for (uint32_t j = 0; j < 4; j++) {
        const uint32_t p = (((tid >> 8) + 4 * j) << 11) | (tid & 255u);
        if (p < nvalid) {
            const uint32_t h = dmx_hash(ld4(L.data, p) & 0xFFFFFFu);
            atomicOr(&SB[h >> 5], 1u << (h & 31));
        }
    }
    __syncthreads();
    if (tid < DMX_NBUCKET / 32) {
        const uint32_t c = wave_sum_u32((uint32_t)__popc(SB[tid]));
        SB[tid] = 0;
        if ((tid & 63) == 0) atomicAdd(&L.ntok, c);
    }
    __syncthreads();
    uint32_t ns = 0;
    for (uint32_t s = 0; s < 16; s++) {
        const uint32_t lo = s << 11;
        ns += nvalid > lo ? min(nvalid - lo, 256u) : 0u;
    }
    return 4 * L.ntok < ns ? dk : max_chain;
}

// NBX > 3: the exhaustive parse without a dictionary (max_chain = 0) on NBX-byte chains
// (P0'); a separate instantiation, so the bounded modes' code and registers are untouched
#ifndef DMX_NBX
#define DMX_NBX 4   // the exhaustive parse's chain length in bytes (4; 5 measured slower: a second gram pass and sort)
#endif
// 16 bytes of a block from HBM for the staging (bytes past bn are zero)
__device__ __forceinline__ uint4 stage16(const uint8_t* __restrict__ d, uint32_t p, uint32_t bn, bool aligned16) {
    if (aligned16 && p + 16 <= bn) return *reinterpret_cast<const uint4*>(d + p);
    uint32_t w[4] = {0, 0, 0, 0};
    for (uint32_t j = 0; j < 16; j++)
        if (p + j < bn) w[j >> 2] |= (uint32_t)d[p + j] << (8 * (j & 3));
    return make_uint4(w[0], w[1], w[2], w[3]);
}
template <bool DICT, int NBX, bool LOOP = false>
__device__ __forceinline__ void match_block(const uint32_t b, const uint8_t* __restrict__ in, uint64_t n, uint32_t sw,
                                            int32_t max_chain, uint32_t mflags, uint16_t* __restrict__ dist_g,
                                            const uint16_t* __restrict__ chs, uint32_t* __restrict__ tok_g,
                                            uint32_t* __restrict__ hist_g,
                                            dmx_blkinfo* __restrict__ info, uint64_t* __restrict__ dbg,
                                            uint32_t* __restrict__ nfallback) {
    __shared__ MatchLDS L;
    __shared__ uint64_t st_search, st_iters, st_w1, st_w23, st_def, tp0[3], st_rounds, st_p3a, st_h4[3], st_lz, st_w1w;
    uint32_t tid = threadIdx.x;
    // in the work-list loop the thread index goes through an empty asm: everything derived
    // from it is then computed per block, not hoisted out of the loop and kept live (spilled)
    // across the whole block
    if (LOOP) asm volatile("" : "+v"(tid));
    const uint32_t lane = tid & 63, wave = wave_of(tid);
    const uint64_t off = (uint64_t)b * sw;
    const uint32_t bn = (uint32_t)((n - off) < sw ? (n - off) : sw);
    const uint8_t* d = in + off;
    const bool aligned16 = ((reinterpret_cast<uintptr_t>(d) & 15) == 0);
    // a workgroup per block: the block's bytes (the 2 MT chunks below DMX_BLK) are requested
    // right after the noise check's record, so the two HBM latencies overlap (a stored
    // block's are wasted: such blocks take the work-list loop when they are most of the input)
    const uint32_t pst = info[b].prestored;   // (read unconditionally: a conditional read is waited for at once)
#ifndef DMX_LATE_STAGE   // (A/B build: the loads after the check, in the staging loop)
    constexpr bool early = !LOOP;
#else
    constexpr bool early = false;
#endif
    uint4 v0 = make_uint4(0, 0, 0, 0), v1 = v0;
    if (early) {
        v0 = stage16(d, tid << 4, bn, aligned16);
        v1 = stage16(d, (tid + MT) << 4, bn, aligned16);
    }
    if ((mflags & 4u) && pst) return;   // stored by the noise check (K0)
    uint16_t* pg = dist_g + (uint64_t)b * DMX_BLK;   // best distances, bucket order (staging)
    uint8_t* D8 = reinterpret_cast<uint8_t*>(L.data);

    // ---- P0: stage the block, the bucket starts and the bucket-sorted positions in LDS ----
    const uint64_t tbeg = dbg ? __builtin_amdgcn_s_memtime() : 0;
    if (tid == 0) { L.adl_s = 0; L.adl_t = 0; L.sortbad = (mflags & 2u) ? 1u : 0u; L.ntok = 0; }   // 2: test hook
    if (dbg && tid == 0) { st_search = 0; st_iters = 0; st_def = 0; st_p3a = 0; }
    for (uint32_t k = tid; k < DMX_HIST; k += MT) L.hist[k] = 0;
    for (uint32_t k = tid; k < DMX_BLK / 32; k += MT) L.lit[k] = 0;
#ifdef DMX_PF
    // L2 prefetch of the block DMX_PF blocks ahead (the one that takes this CU's slot next when
    // the blocks take about the same time; same XCD: DMX_PF is a multiple of 8): one dword per
    // 128-byte line, its value consumed after P0 so the load never stalls the staging
    uint32_t pfv = 0;
    if (!LOOP && tid < 256) {
        const uint64_t po = (uint64_t)(b + DMX_PF) * sw + (uint64_t)tid * 128;
        if (po < n) pfv = *reinterpret_cast<const uint32_t*>(in + (po & ~3ull));
    }
#endif
    uint32_t runny = 0;   // 16-byte chunks of one repeated byte (run-dominated blocks)
    // a block of one repeated byte: every chunk of this thread is one repeated byte, the same
    // byte cb in all of them (0x100: none yet), and (below, after the barrier) cb is byte 0
    // -- no separate load of byte 0
    bool uni = true;
    uint32_t cb = 0x100u;
    for (uint32_t k = tid; k < DATA_WORDS / 4; k += MT) {   // 16-byte chunks
        const uint32_t p = k << 4;
        uint4 v;
        if (early && k < 2 * MT) v = k < MT ? v0 : v1;
        else v = stage16(d, p, bn, aligned16);
        *reinterpret_cast<uint4*>(&L.data[k << 2]) = v;
        // run-dominated blocks take the run_len search (search_positions<.., true>): count the
        // 16-byte chunks that are one repeated byte
        const bool rep = v.x == v.y && v.y == v.z && v.z == v.w && v.x == (v.x & 0xFFu) * 0x01010101u;
        runny += (p < bn && rep) ? 1u : 0u;
        if (p + 16 <= bn) {
            uni = uni && rep && (cb == 0x100u || cb == (v.x & 0xFFu));
            cb = v.x & 0xFFu;
        } else if (p < bn) {   // the tail chunk: its bytes below bn
            const uint32_t w4[4] = {v.x, v.y, v.z, v.w};
            const uint32_t c0 = cb == 0x100u ? (v.x & 0xFFu) : cb;
            for (uint32_t j = 0; j < bn - p; j++) uni = uni && ((w4[j >> 2] >> (8 * (j & 3))) & 0xFFu) == c0;
            cb = c0;
        }
    }
    runny = wave_sum_u32(runny);
    if (lane == 0) L.wexit[wave] = runny;   // free until the walk; published by the barriers below
    // DMX_F_DICT: the chain kernel already sorted this block; the history kernel's
    // results (bucket order) wait in the block's token slots until P3
    const uint32_t* hbk = DICT ? tok_g + (uint64_t)b * DMX_BLK : nullptr;
    int32_t kb = max_chain;   // this block's chain depth (DMX_F_DEEP: block_chain)
    if (DICT) {
        const uint32_t nv = bn > 2 ? bn - 2 : 0;
        const uint16_t* Sg = chs + (uint64_t)(b + 1) * DMX_BLK;
        for (uint32_t k = tid; k < (nv + 7) / 8; k += MT)
            reinterpret_cast<uint4*>(L.sorted)[k] = reinterpret_cast<const uint4*>(Sg)[k];
        for (uint32_t k = tid; k < DMX_BLK / 32; k += MT) L.lit[k] = 0;
        __syncthreads();
        kb = block_chain(L, bn, max_chain, mflags, tid);
        if (kb <= 0 || kb > KD) {   // bucket starts, as sort_positions finds them
            for (uint32_t k = tid; k < nv; k += MT) {
                const uint32_t h = dmx_hash(ld4(L.data, L.sorted[k]) & 0xFFFFFFu);
                const uint32_t hp = k ? dmx_hash(ld4(L.data, L.sorted[k - 1]) & 0xFFFFFFu) : 0xFFFFFFFFu;
                if (h != hp) L.bstart[h] = (uint16_t)k;
            }
        }
        __syncthreads();
    } else {
        // a block of one repeated byte (no dictionary): the parse is known in closed form --
        // a literal, then distance-1 matches of min(258, bytes left) while >= 3 bytes are
        // left, then literals -- which is exactly what the search + walk would produce
        // (position i's nearest candidate is i - 1, matching to the block's end; lazy
        // evaluation never defers: i + 1 is never longer).  Tokens, histograms and the
        // block record are written directly.
        if (__syncthreads_and(uni) && __syncthreads_and(cb == 0x100u || cb == (uint32_t)D8[0])) {   // (also publishes the waves' run counts)
            const uint32_t c = D8[0];
            const uint32_t nt = uniform_parse(bn, c, tok_g + (uint64_t)b * DMX_BLK, L.hist, tid, MT);
            if (tid == 0) {
                const uint64_t S = (uint64_t)c * bn, T = (uint64_t)c * ((uint64_t)bn * (bn - 1) / 2);
                info[b].ntok = nt;
                info[b].n = bn;
                info[b].adl_s = S;
                info[b].adl_w = (uint64_t)bn * S - T;
                info[b].prestored = 0;
            }
            __syncthreads();
            for (uint32_t k = tid; k < DMX_HIST; k += MT) hist_g[(uint64_t)b * DMX_HIST + k] = L.hist[k];
            return;
        }
        uint32_t nrun0 = 0;
#pragma unroll
        for (int w = 0; w < MW; w++) nrun0 += L.wexit[w];
        // the exhaustive parse's first sort (trigram chains for the gram pass) needs no bucket
        // starts: the 4-byte sort makes the search's (max_chain 1 here only skips them)
        kb = block_chain(L, bn, max_chain, mflags, tid);
        const int32_t mc0 = (NBX > 3 && !DICT) ? 1 : kb;
        if (nrun0 * 4 >= ((bn + 15) >> 4)) sort_positions<false, true>(L, bn, mc0, tid, dbg != nullptr, tp0);
        else sort_positions<false, false>(L, bn, mc0, tid, dbg != nullptr, tp0);
    }

    if (dbg_stop(mflags, 1, info, hist_g, b, bn, tid)) return;
#ifdef DMX_PF
    asm volatile("" ::"v"(pfv));
#endif
    {   // Adler-32 partial sums of this block
        uint64_t s = 0, t = 0;
        const uint32_t lo = tid << 5;   // 32 bytes per thread, read as two 16-byte vectors
        const uint4 v0 = *reinterpret_cast<const uint4*>(&L.data[lo >> 2]);
        const uint4 v1 = *reinterpret_cast<const uint4*>(&L.data[(lo >> 2) + 4]);
        const uint32_t w[8] = {v0.x, v0.y, v0.z, v0.w, v1.x, v1.y, v1.z, v1.w};
#pragma unroll
        for (uint32_t j = 0; j < 32; j++) {   // bytes past bn are zero in LDS
            const uint32_t c = (w[j >> 2] >> (8 * (j & 3))) & 0xFFu;
            s += c;
            t += (uint64_t)(lo + j) * c;
        }
        s = wave_sum_u64(s);
        t = wave_sum_u64(t);
        if (lane == 0) { atomicAdd(&L.adl_s, (unsigned long long)s); atomicAdd(&L.adl_t, (unsigned long long)t); }
    }

    // ---- P0' (the exhaustive parse, no dictionary): 4-byte chains.  Every match of 4 or
    // more bytes is between positions with the same first 4 bytes, so the exhaustive search
    // runs over the chains of a second sort by a hash of 4 bytes (text: 17 candidates per
    // position on average instead of 39).  A match of exactly 3 is then the nearest earlier
    // position with the same trigram: read from the 3-byte sort first (the nearest entry of
    // the trigram's bucket with equal bytes; hash collisions are skipped) and kept in HBM,
    // in this block's token slots, until the search merges it (longest, then nearest).
    constexpr bool h4 = NBX > 3 && !DICT;   // launched only with max_chain == 0
    // this block's token slots (free until P3), as 16-bit seeds: 64 KB per block, so the seeds of
    // the 32 blocks of an XCD (2 MB) stay in its 4 MB L2 between the gram pass and the search
    uint16_t* seeds = reinterpret_cast<uint16_t*>(tok_g + (uint64_t)b * DMX_BLK);
    if constexpr (h4) {
        const uint32_t nv = bn > 2 ? bn - 2 : 0;
        const uint32_t hook = L.sortbad;   // the exact-sort test hook (mflags & 2)
        uint32_t npass = 0, ndefer = 0;
        uint64_t tsw = 0;
        for (uint32_t pass = 0;; pass++) {   // 3-byte grams from P0's sort (checked here)
            npass++;
            if (!__syncthreads_or(gram_pass<3>(L, nv, tid, seeds, ndefer, tsw)) || pass) break;
            if (tid == 0) atomicAdd(nfallback, 1u);   // counted in dmx_result.nsortfallback
            sort_positions<true>(L, bn, 1, tid, false, tp0);   // never observed on gfx950 (no starts, as above)
        }
        if constexpr (NBX > 4) {   // 4-byte grams from a 4-byte sort
            for (uint32_t pass = 0;; pass++) {
                npass++;
                if (hook || pass) sort_positions<true, true, 4>(L, bn, max_chain, tid, false, tp0);
                else sort_positions<false, true, 4>(L, bn, max_chain, tid, false, tp0);
                if (!__syncthreads_or(gram_pass<4>(L, nv, tid, seeds, ndefer, tsw)) || pass || hook) break;
                if (tid == 0) atomicAdd(nfallback, 1u);
            }
        }
        if (dbg && tid == 0) st_h4[0] = (__builtin_amdgcn_s_memtime() - tbeg) | ((uint64_t)npass << 48);
        if (dbg && tid == 0) st_h4[2] = tsw - tbeg;   // the 3-byte sweep's end (before its listed walks)
        uint32_t nr4 = 0;   // run-dominated blocks (counted while staging) take the run-aware ranks
#pragma unroll
        for (int w = 0; w < MW; w++) nr4 += L.wexit[w];
        if (hook) sort_positions<true, true, NBX>(L, bn, max_chain, tid, false, tp0);
        else if (nr4 * 4 >= ((bn + 15) >> 4)) sort_positions<false, true, NBX>(L, bn, max_chain, tid, false, tp0);
        else sort_positions<false, false, NBX>(L, bn, max_chain, tid, false, tp0);
        if (dbg && tid == 0) st_h4[1] = (__builtin_amdgcn_s_memtime() - tbeg) | ((uint64_t)min(ndefer, 65535u) << 48);
    }

    // ---- P1: longest match of every position ----
    const uint64_t t0 = dbg ? __builtin_amdgcn_s_memtime() : 0;
    uint64_t tdef = 0;
    for (uint32_t attempt = 0;; attempt++) {
        // run-dominated blocks (zeros, long runs) search with the change bitmap; a separate
        // instantiation keeps its registers out of the common path
        // (counted per wave while staging; the sort's barriers published the counts)
        uint32_t nrun = 0;
#pragma unroll
        for (int w = 0; w < MW; w++) nrun += L.wexit[w];
        const bool runs = kb > 0 && kb <= KE && nrun * 4 >= ((bn + 15) >> 4);
        if (kb > 0 && kb <= KE) {   // the winners' nibbles (bstart is free after P0)
            uint32_t z = 0;
            asm volatile("" : "+v"(z));   // (else the compiler keeps a zero quad in a scratch slot)
            reinterpret_cast<uint4*>(nib_words(L))[tid] = make_uint4(z, z, z, z);
        }
        if (tid == 0) L.ntok = 0;   // the search's chunk counter
        __syncthreads();
        const uint32_t its = runs ? search_positions<DICT, true>(L, bn, kb, pg, tid, dbg != nullptr, tdef, hbk)
                             : h4 ? search_positions<DICT, false, (h4 ? NBX : 3)>(L, bn, kb, pg, tid, dbg != nullptr, tdef, hbk, seeds)
                                  : search_positions<DICT, false>(L, bn, kb, pg, tid, dbg != nullptr, tdef, hbk);
        if (dbg && lane == 0 && attempt == 0) {
            atomicAdd((unsigned long long*)&st_iters, (unsigned long long)its);
            atomicMax((unsigned long long*)&st_search, (unsigned long long)(__builtin_amdgcn_s_memtime() - t0));
            atomicMax((unsigned long long*)&st_def, (unsigned long long)tdef);
        }
        __syncthreads();
        if (!L.sortbad || attempt) break;
        // never observed on gfx950: redo the block with the match-any sort (stable by construction);
        // counted (dmx_result.nsortfallback) so that every run shows it did not happen
        if (tid == 0) atomicAdd(nfallback, 1u);
        if (h4) sort_positions<true, true, (h4 ? NBX : 3)>(L, bn, kb, tid, dbg != nullptr, tp0);
        else sort_positions<true>(L, bn, kb, tid, dbg != nullptr, tp0);
    }
    const uint64_t t1 = dbg ? __builtin_amdgcn_s_memtime() : 0;
    if (dbg_stop(mflags, 2, info, hist_g, b, bn, tid)) return;

    // ---- P1b (DMX_F_LAZY): lazy evaluation as a per-position rule on the search results.
    // Position p (a match) becomes a literal when p+1 holds a strictly longer match; the
    // walk below then emits the literal and re-decides at p+1 -- exactly the sequential
    // sequential rule (bounded/lazy modes).  Each thread owns one literal word.
    if (mflags & 1u) {   // DMX_F_LAZY
        const uint32_t lw = L.lit[tid];
        const uint32_t nb0 = (tid + 1 < DMX_BLK / 32) ? (L.lit[tid + 1] & 1u) : 1u;
        const uint32_t* l32 = reinterpret_cast<const uint32_t*>(L.len8);
        uint32_t lv[9];
#pragma unroll
        for (int j = 0; j < 8; j++) lv[j] = l32[tid * 8 + j];
        lv[8] = (tid + 1 < DMX_BLK / 32) ? l32[tid * 8 + 8] : 0u;
        const uint32_t litn = (lw >> 1) | (nb0 << 31);   // literal bit of p+1
        uint32_t longer = 0;                              // len(p+1) > len(p)
#pragma unroll
        for (int bb = 0; bb < 32; bb++) {
            const uint32_t cur = (lv[bb >> 2] >> (8 * (bb & 3))) & 0xFFu;
            const uint32_t nxt = (lv[(bb + 1) >> 2] >> (8 * ((bb + 1) & 3))) & 0xFFu;
            longer |= (nxt > cur ? 1u : 0u) << bb;
        }
        __syncthreads();
        L.lit[tid] = lw | (~lw & ~litn & longer);
        __syncthreads();
    }
    if (dbg && tid == 0) st_lz = __builtin_amdgcn_s_memtime() - t1;

    // ---- P2: greedy path ----
    {   // W1: speculative walk of every 32-position segment from its start
        const uint32_t lo = tid << 5, lw = L.lit[tid];   // the segment's literal bits: one read
        uint32_t m = 0, p = lo;
        while (p < lo + 32 && p < bn) {
#ifndef DMX_WALK_STEP
            // a run of literals in one step (resolve_word); a match reads its length
            const uint32_t sh = p - lo;
            const uint32_t run = min(ffbl_hw(~(lw >> sh)), min(lo + 32u, bn) - p);   // (lit bits past bn may be set by P1b)
            if (run) {
                m |= (run >= 32u ? ~0u : ((1u << run) - 1u)) << sh;
                p += run;
                continue;
            }
            m |= 1u << sh;
            p += (uint32_t)L.len8[p] + 3u;
#else
            m |= 1u << (p - lo);
            p += ((lw >> (p - lo)) & 1u) ? 1u : (uint32_t)L.len8[p] + 3u;
#endif
        }
        L.tsm[tid] = m;
        L.exitp[tid] = p;
    }
    {   // the sorted positions are dead: permute the best distances (bucket order) into
        // position order in the same LDS slots, through registers (32 per thread).  Short
        // chains (K <= KE): distance = S[k] - S[k - j] from the winner nibble j of entry k (the
        // history's from its result); longer chains staged the distances in pg (HBM).
        __syncthreads();
        if (dbg && tid == 0) st_w1w = __builtin_amdgcn_s_memtime() - t1;
        const uint32_t nvalid = bn > 2 ? bn - 2 : 0;
        uint4 dv[4], pv[4];
        if (kb > 0 && kb <= KE) {
            const uint32_t* NW = nib_words(L);
#pragma unroll
            for (int j = 0; j < 4; j++) {
                const uint32_t c = tid + (uint32_t)j * MT;   // 8 entries per 16-byte chunk
                const bool in = c * 8 < nvalid;
                pv[j] = in ? reinterpret_cast<const uint4*>(L.sorted)[c] : make_uint4(0, 0, 0, 0);
                const uint32_t nw = in ? NW[c] : 0u;
                const uint32_t pw[4] = {pv[j].x, pv[j].y, pv[j].z, pv[j].w};
                uint32_t dw[4] = {0, 0, 0, 0};
#pragma unroll
                for (int e = 0; e < 8; e++) {
                    const uint32_t jj = (nw >> (4 * e)) & 15u, kk = c * 8 + (uint32_t)e;
                    uint32_t dist = 0;
                    if (jj == NIB_HIST) dist = DICT ? (hbk[kk] & 0xFFFFu) : 0u;
                    else if (jj) dist = ((pw[e >> 1] >> (16 * (e & 1))) & 0xFFFFu) - (uint32_t)L.sorted[kk - jj];
                    dw[e >> 1] |= dist << (16 * (e & 1));
                }
                dv[j] = make_uint4(dw[0], dw[1], dw[2], dw[3]);
            }
        } else {
#pragma unroll
            for (int j = 0; j < 4; j++) {
                const uint32_t c = tid + (uint32_t)j * MT;   // 8 entries per 16-byte chunk
                const bool in = c * 8 < nvalid;
                dv[j] = in ? reinterpret_cast<const uint4*>(pg)[c] : make_uint4(0, 0, 0, 0);
                pv[j] = in ? reinterpret_cast<const uint4*>(L.sorted)[c] : make_uint4(0, 0, 0, 0);
            }
        }
        __syncthreads();
#pragma unroll
        for (int j = 0; j < 4; j++) {
            const uint32_t dw[4] = {dv[j].x, dv[j].y, dv[j].z, dv[j].w}, pw[4] = {pv[j].x, pv[j].y, pv[j].z, pv[j].w};
#pragma unroll
            for (int e = 0; e < 8; e++) {
                // only matches (distance > 0): P3 reads S[p] for match tokens alone, so a
                // literal position keeps whatever the slot held
                const uint32_t kk = (tid + (uint32_t)j * MT) * 8 + (uint32_t)e;
                const uint32_t d16 = (dw[e >> 1] >> (16 * (e & 1))) & 0xFFFFu;
                if (kk < nvalid && d16 != 0) L.sorted[(pw[e >> 1] >> (16 * (e & 1))) & 0xFFFFu] = (uint16_t)d16;
            }
        }
    }
    if (dbg && tid == 0) st_w1 = __builtin_amdgcn_s_memtime() - t1;
    // W2 (parallel): Jacobi rounds.  Every segment takes the exit of its predecessor's
    // current path as its entry and, if that changed, re-walks from it until it meets its
    // own current path (the rest then coincides: the next-function is deterministic) or
    // leaves the segment.  A round where no entry changes is a fixed point, i.e. the
    // sequential path.  Typical text converges in a few rounds; a run of long matches moves
    // the true entry one segment per round, so after JR rounds the serial resolution below
    // finishes from the current (valid) segment paths.
    bool conv = false, serial = false;
    if (tid == 0) L.ntok = 0;
    {
        uint32_t entry = tid << 5;   // what W1 assumed
        uint32_t r = 0;
        for (; r < JR; r++) {
            if (r == 3) {   // not converged yet: few tokens (runs of long matches) -> serial walk below
                const uint32_t pc = wave_sum_u32((uint32_t)__popc(L.tsm[tid]));
                if (lane == 0) atomicAdd(&L.ntok, pc);
                __syncthreads();
                if (L.ntok <= WALK_SERIAL) { serial = true; break; }
            }
            const uint32_t e = tid == 0 ? 0u : L.exitp[tid - 1];
            __syncthreads();
            const bool ch = (tid << 5) < bn && e != entry;   // segments past the block end stay empty
            if (ch) {
                uint32_t nm;
                bool mg;
                const uint32_t x = resolve_word(L, tid << 5, e, bn, L.tsm[tid], L.lit[tid], L.exitp[tid], nm, mg);
                L.tsm[tid] = nm;
                L.exitp[tid] = x;
                entry = e;
            }
            if (!__syncthreads_or(ch)) { conv = true; break; }
        }
        if (dbg && tid == 0) st_rounds = r;
    }
    if (serial) {   // few tokens (runs of long matches): one lane walks the path token by token
        {
            conv = true;
            L.tsm[tid] = 0;
            __syncthreads();
            if (tid == 0) {
                uint32_t p = 0, wi = 0, cw = 0;
                while (p < bn) {
                    if ((p >> 5) != wi) { L.tsm[wi] = cw; cw = 0; wi = p >> 5; }
                    cw |= 1u << (p & 31);
                    p += adv_of(L, p);
                }
                L.tsm[wi] = cw;
            }
            __syncthreads();
        }
    }
    if (!conv) {
        {   // W2: each wave resolves its 64 segments assuming it is entered at 2048*wave.
            // Segment words live one per lane; the serial loop runs on uniform values.
            uint32_t myw = L.tsm[tid];
            const uint32_t myx = L.exitp[tid], myl = L.lit[tid];
            uint32_t e = wave << 11;
            for (uint32_t j = 0; j < 64; j++) {
                const uint32_t m = __builtin_amdgcn_readlane(myw, (int)j), x = __builtin_amdgcn_readlane(myx, (int)j),
                               lw = __builtin_amdgcn_readlane(myl, (int)j);
                uint32_t nm;
                bool mg;
                e = resolve_word(L, ((wave << 6) + j) << 5, e, bn, m, lw, x, nm, mg);
                if (lane == j) myw = nm;
            }
            L.tsm[tid] = myw;
            if (lane == 0) L.wexit[wave] = e;
        }
        __syncthreads();
        if (tid == 0) {   // W3: fix the waves whose true entry differs, until the paths merge
            uint32_t E = L.wexit[0];
            for (uint32_t w = 1; w < MW; w++) {
                if (E == (w << 11)) { E = L.wexit[w]; continue; }
                uint32_t e = E;
                for (uint32_t s = w << 6; s < (w << 6) + 64; s++) {
                    uint32_t nm;
                    bool mg;
                    e = resolve_word(L, s << 5, e, bn, L.tsm[s], L.lit[s], 0, nm, mg);
                    L.tsm[s] = nm;
                    if (mg) { e = L.wexit[w]; break; }
                }
                E = e;
            }
        }
        __syncthreads();
    }
    if (dbg && tid == 0) st_w23 = __builtin_amdgcn_s_memtime() - t1;
    if (dbg_stop(mflags, 3, info, hist_g, b, bn, tid)) return;
    // ---- P3: compaction + histograms ----
    {
        const uint32_t m = L.tsm[tid];
        const uint32_t cnt = __popc(m);
        const uint32_t x = wave_incl_scan(cnt);
        if (lane == 63) L.wsum[wave] = x;
        __syncthreads();
        if (wave == 0) {
            const uint32_t v = lane < MW ? L.wsum[lane] : 0, z = wave_incl_scan(v);
            if (lane < MW) L.wsum[lane] = z - v;
            if (lane == MW - 1) L.ntok = z;
        }
        __syncthreads();
        uint32_t k = L.wsum[wave] + x - cnt;
        uint32_t* tb = tok_g + (uint64_t)b * DMX_BLK;
        const uint32_t ntok = L.ntok;   // uniform (published by the barrier above)
        // Token-major: every thread lists its segment's token positions in token order (a
        // cheap serial loop), then each thread builds tokens t = tid, tid + 1024, ...: the work
        // is balanced over the lanes (segments hold 0..32 tokens) and the token stores are
        // coalesced.  The list lives in bstart (free after the permute), TPMAX tokens per round.
        uint16_t* TP = reinterpret_cast<uint16_t*>(L.bstart);
        // histograms in 4 copies (lane & 3; stride 321 words, so a symbol's copies sit in
        // different banks): a quarter of the same-address atomics of popular symbols.  tsm +
        // exitp (free now: the token words are in registers) hold them; summed into hist at the end.
        uint32_t* HS = L.tsm;
        for (uint32_t q = tid; q < 4 * HSTR; q += MT) HS[q] = 0;
        uint32_t* hl = HS + (lane & 3u) * HSTR;
        for (uint32_t r0 = 0; r0 < ntok; r0 += TPMAX) {
            const uint32_t r1 = min(r0 + TPMAX, ntok);
            if (r0) __syncthreads();   // the previous round's readers are done with the list
            uint32_t kk = k;
            for (uint32_t mm = m; mm && kk < r1; mm &= mm - 1u, kk++)
                if (kk >= r0) TP[kk - r0] = (uint16_t)((tid << 5) + (uint32_t)__builtin_ctz(mm));
            __syncthreads();
            if (dbg && tid == 0 && r0 == 0) st_p3a = __builtin_amdgcn_s_memtime() - t1;   // first list built
#ifdef DMX_P3_BATCH
            constexpr bool p3batch = true;
#else
            constexpr bool p3batch = h4;   // (batched loads: the exhaustive parse +0.6 %; K = 7 48.8 -> 50.1 K cycles to P3's end, round 6)
#endif
            if constexpr (!p3batch) {
#ifndef DMX_P3_BRANCHY
            for (uint32_t t = r0 + tid; t < r1; t += MT) {
                // one path for both token kinds: the byte, length and distance slots are read
                // together, the lit/len symbol is the byte or the length's (RFC 1951 3.2.5 by
                // formula: l = len - 3, e = max(floor(log2 l), 2) - 2, 257 + 4e + (l >> e), 258
                // -> 285), and only a match adds its distance symbol
                const uint32_t p = TP[t - r0];
                const bool lit = (L.lit[p >> 5] >> (p & 31)) & 1u;
                const uint32_t c = D8[p], len = (uint32_t)L.len8[p] + 3u, dist = L.sorted[p];
                const uint32_t l = len - 3u, e = max(31u - __clz(l | 1u), 2u) - 2u;
                const uint32_t sl = len == 258u ? 285u : 257u + 4u * e + (l >> e);
                atomicAdd(&hl[lit ? c : sl], 1u);
                if (!lit) {
                    const uint32_t x = dist - 1u, ed = 31u - __clz(x | 2u);
                    atomicAdd(&hl[DMX_DIST0 + (x < 2u ? x : 2u * ed + ((x >> (ed - 1u)) & 1u))], 1u);
                }
                tb[t] = lit ? c : (dist << 9) | len;
            }
#else
            for (uint32_t t = r0 + tid; t < r1; t += MT) {
                const uint32_t p = TP[t - r0];
                uint32_t tk;
                if ((L.lit[p >> 5] >> (p & 31)) & 1u) {
                    tk = D8[p];
                    atomicAdd(&hl[tk], 1u);
                } else {
                    const uint32_t len = (uint32_t)L.len8[p] + 3u, dist = L.sorted[p];
                    tk = (dist << 9) | len;
                    uint32_t sy, eb, ev;
                    len_sym(len, sy, eb, ev);
                    atomicAdd(&hl[sy], 1u);
                    dist_sym(dist, sy, eb, ev);
                    atomicAdd(&hl[DMX_DIST0 + sy], 1u);
                }
                tb[t] = tk;
            }
#endif
            } else {
            // DMX_P3_BATCH (and the exhaustive parse): P3B tokens per thread at a time, their LDS reads issued together (token position,
            // literal word, then byte, length and distance of each, whichever it is): three
            // rounds of latency for the batch instead of three per token
            constexpr uint32_t P3B = 8;
            for (uint32_t t0 = r0 + tid; t0 < r1; t0 += P3B * MT) {
                uint32_t pp[P3B], lw8[P3B], cb[P3B], l8[P3B], ds[P3B];
#pragma unroll
                for (uint32_t j = 0; j < P3B; j++) pp[j] = t0 + j * MT < r1 ? (uint32_t)TP[t0 + j * MT - r0] : 0u;
#pragma unroll
                for (uint32_t j = 0; j < P3B; j++) lw8[j] = L.lit[pp[j] >> 5];
#pragma unroll
                for (uint32_t j = 0; j < P3B; j++) {
                    cb[j] = D8[pp[j]];
                    l8[j] = L.len8[pp[j]];
                    ds[j] = L.sorted[pp[j]];
                }
#pragma unroll
                for (uint32_t j = 0; j < P3B; j++) {
                    const uint32_t t = t0 + j * MT;
                    if (t >= r1) break;
                    uint32_t tk;
                    if ((lw8[j] >> (pp[j] & 31)) & 1u) {
                        tk = cb[j];
                        atomicAdd(&hl[tk], 1u);
                    } else {
                        const uint32_t len = l8[j] + 3u, dist = ds[j];
                        tk = (dist << 9) | len;
                        uint32_t sy, eb, ev;
                        len_sym(len, sy, eb, ev);
                        atomicAdd(&hl[sy], 1u);
                        dist_sym(dist, sy, eb, ev);
                        atomicAdd(&hl[DMX_DIST0 + sy], 1u);
                    }
                    tb[t] = tk;
                }
            }
            }
        }
        __syncthreads();
        for (uint32_t q = tid; q < DMX_HIST; q += MT) L.hist[q] += HS[q] + HS[HSTR + q] + HS[2 * HSTR + q] + HS[3 * HSTR + q];
    }
    __syncthreads();
    const uint64_t p3b = dbg ? __builtin_amdgcn_s_memtime() - t1 : 0;
    for (uint32_t k = tid; k < DMX_HIST; k += MT) hist_g[(uint64_t)b * DMX_HIST + k] = L.hist[k];
    if (dbg && tid == 0) {
        dbg[(uint64_t)b * DMX_STAMPS + 0] = t0 - tbeg;
        dbg[(uint64_t)b * DMX_STAMPS + 1] = st_search;
        dbg[(uint64_t)b * DMX_STAMPS + 2] = __builtin_amdgcn_s_memtime() - t1;
        dbg[(uint64_t)b * DMX_STAMPS + 3] = st_def;
        dbg[(uint64_t)b * DMX_STAMPS + 4] = st_iters;
        dbg[(uint64_t)b * DMX_STAMPS + 5] = st_w1;
        dbg[(uint64_t)b * DMX_STAMPS + 6] = st_w23;
        dbg[(uint64_t)b * DMX_STAMPS + 7] = __builtin_amdgcn_s_memtime() - tbeg;
        dbg[(uint64_t)b * DMX_STAMPS + 8] = tp0[0] - tbeg;   // P0 sub-phases: block staged
        dbg[(uint64_t)b * DMX_STAMPS + 9] = tp0[1] - tbeg;   //   pass 1 done
        dbg[(uint64_t)b * DMX_STAMPS + 10] = tp0[2] - tbeg;  //   pass 2 done
        dbg[(uint64_t)b * DMX_STAMPS + 11] = st_rounds;      // walk: Jacobi rounds (JR = not converged)
        if (!DICT) {   // (12, 13 are the history kernel's with DMX_F_DICT)
            dbg[(uint64_t)b * DMX_STAMPS + 12] = h4 ? st_h4[2] : st_p3a;   // P3: token list built (exhaustive: sweep end)
            dbg[(uint64_t)b * DMX_STAMPS + 13] = p3b;        // P3: tokens and histograms done
            dbg[(uint64_t)b * DMX_STAMPS + 14] = h4 ? st_h4[0] : st_lz;    // exhaustive: nearest-trigram pass done; else P1b done
            dbg[(uint64_t)b * DMX_STAMPS + 15] = h4 ? st_h4[1] : st_w1w;   //   4-byte sort done; else W1's walk done
        }
    }
    if (tid == 0) {
        info[b].ntok = L.ntok;
        info[b].n = bn;
        info[b].adl_s = L.adl_s;
        info[b].adl_w = (uint64_t)bn * L.adl_s - L.adl_t;
        info[b].prestored = 0;
    }
}

// K1.  LOOP = false: one workgroup per block (blockIdx.x).  LOOP = true (DMX_F_STORE_CHECK,
// when most blocks were stored in the context's previous encode: dmx_encode_async's hint) a
// persistent grid of one workgroup per CU takes the blocks of the work list L1 from a device
// counter, the next one claimed while the current one runs; the index goes through LDS, so
// every wave leaves the loop together.  Stored blocks then cost nothing here (a workgroup per
// block: 32 768 workgroups of 161 KB that return at once, 0.07-0.16 ms for 1 GiB of noise);
// the loop's code is 2.5-4 % slower on text (its register allocation), hence the choice.
struct MatchArgs {   // dmx_match_kernel's arguments, one struct (read back per block in the loop)
    const uint8_t* in;
    uint64_t n;
    uint32_t sw;
    int32_t max_chain;
    uint32_t mflags;
    uint16_t* dist_g;
    const uint16_t* chs;
    uint32_t* tok_g;
    uint32_t* hist_g;
    dmx_blkinfo* info;
    uint64_t* dbg;
    uint32_t* nfallback;
    uint32_t* wl;
};
template <bool DICT, int NBX = 3, bool LOOP = false>
__global__ __launch_bounds__(MT) void dmx_match_kernel(const MatchArgs args) {
    if constexpr (!LOOP) {   // one workgroup per block (stored blocks return at once)
        match_block<DICT, NBX>(blockIdx.x, args.in, args.n, args.sw, args.max_chain, args.mflags, args.dist_g, args.chs,
                               args.tok_g, args.hist_g, args.info, args.dbg, args.nfallback);
        return;
    }
    uint32_t* const wl = args.wl;
    __shared__ uint32_t nb_s;
    uint32_t nx = 0;   // thread 0: the list index claimed for the next block
    if (wl && threadIdx.x == 0) nx = atomicAdd(&wl[WL_C1], 1u);
    for (uint32_t it = 0;; it++) {
        uint32_t b;
        if (!wl) {
            if (it) break;
            b = blockIdx.x;
        } else {
            if (threadIdx.x == 0) {
                uint32_t v = 0xFFFFFFFFu;
                if (nx < wl[WL_N1]) {
                    v = wl[WL_HDR + nx];
                    nx = atomicAdd(&wl[WL_C1], 1u);
                }
                nb_s = v;
            }
            __syncthreads();
            b = nb_s;
            __syncthreads();   // every thread has the index before thread 0 may write the next
            if (b == 0xFFFFFFFFu) break;
        }
        // the arguments through a pointer the compiler cannot follow across iterations: loaded
        // where the block needs them, as in a kernel without the loop, instead of hoisted and
        // kept live (spilled) through the whole block
        typedef const __attribute__((address_space(4))) MatchArgs* KArgs;   // constant memory: rematerialisable loads
        KArgs A = (KArgs)__builtin_amdgcn_kernarg_segment_ptr();
        asm volatile("" : "+s"(A));
        match_block<DICT, NBX, true>(b, A->in, A->n, A->sw, A->max_chain, A->mflags, A->dist_g, A->chs, A->tok_g,
                                     A->hist_g, A->info, A->dbg, A->nfallback);
    }
}

// ------------------------------------------------------------------------------------
// K2: Huffman codes + block type (one wave per block)
// ------------------------------------------------------------------------------------

struct K2LDS {   // 16-bit weights (a block has at most 32 769 symbols): 5.0 KB, 32 one-wave workgroups per CU
    union {
        struct {   // the frequencies (dead once huff_plan has the body costs)
            uint16_t fll[288];
            uint16_t fd[32];
        };
        struct {   // run-length coding of the code lengths (RFC 1951 §3.2.7), huff_cl onwards
            uint8_t rle_sym[320];
            uint8_t rle_ext[320];
        };
    };
    uint32_t fcl[20];     // (LDS atomics: 32-bit)
    uint8_t lll[288];
    uint8_t ld[32];
    uint8_t lcl[20];
    // Huffman construction (one alphabet at a time)
    // (at most 286 used symbols, 285 internal nodes)
    uint16_t fs[288];     // used symbols' weights sorted by (weight, symbol)
    uint16_t sym[288];    //   and their symbols
    union {
        uint16_t nodew[288];            // internal node weights, in creation order (huff_lengths)
        uint32_t hdr[DMX_HDR_WORDS];    // the header bits (huff_emit, after every huff_lengths)
    };
    uint16_t lpar[288];   // sorted leaf -> parent node
    union {
        uint32_t keys[288];   // the used symbols' sort keys (weight << 9 | symbol), before the merge
        struct {
            uint16_t up[288];     // node -> ancestor (pointer jumping)
            uint16_t dd[288];     // node -> distance to that ancestor (-> depth)
        };
    };
    int32_t blc[32];      // leaves per code length (a depth > 31 needs a total weight > 32 769)
    int32_t lstart[16];   // first sorted index that gets length d
    int32_t cnt[16];      // canonical codes: codes handed out per length so far
    uint32_t next[16];    // canonical codes: first code of each length
    uint32_t ccode[20];   // code-length codes, same packing
    int32_t rle_n, hlit, hdist, hclen;
};

// K2 helpers run on one wave (one wave per alphabet / per split group), so they
// synchronise the wave, never the workgroup: LDS writes of this wave done, then a
// compiler barrier.
__device__ __forceinline__ void wsync() {
    __builtin_amdgcn_fence(__ATOMIC_SEQ_CST, "workgroup");
    __builtin_amdgcn_wave_barrier();
}

__constant__ uint8_t c_clorder[19] = {16, 17, 18, 0, 8, 7, 9, 6, 10, 5, 11, 4, 12, 3, 13, 2, 14, 1, 15};

// Diagnostic builds (-DDMX_K2_STAMPS): cycles per K2 phase summed over the launch's blocks
// (dmx_k2_stamps): 0 rank sort, 1 two-queue merge, 2 depths + lengths, 3 canonical codes,
// 4 run-length coding, 5 header emission, 6 the rest, 7 blocks.
#ifdef DMX_K2_STAMPS
__device__ unsigned long long dmx_k2_st[16];
#define K2T() __builtin_amdgcn_s_memtime()
#define K2ST(k, t0) do { const uint64_t t1_ = K2T(); if ((threadIdx.x & 63) == 0) atomicAdd(&dmx_k2_st[k], (unsigned long long)(t1_ - (t0))); t0 = t1_; } while (0)
extern "C" int dmx_k2_stamps(unsigned long long* host, int reset) {
    if (hipMemcpyFromSymbol(host, HIP_SYMBOL(dmx_k2_st), sizeof(unsigned long long) * 16, 0, hipMemcpyDeviceToHost) != hipSuccess) return -1;
    if (reset) {
        unsigned long long z[16] = {};
        if (hipMemcpyToSymbol(HIP_SYMBOL(dmx_k2_st), z, sizeof(z), 0, hipMemcpyHostToDevice) != hipSuccess) return -1;
    }
    return 0;
}
#else
#define K2T() 0ull
#define K2ST(k, t0) ((void)(t0))
#endif
__constant__ uint8_t c_cl_eb[19] = {0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 2, 3, 7};

// Exclusive prefix sum over one wave (64 lanes).
__device__ __forceinline__ uint32_t wave_excl_scan(uint32_t v) { return wave_incl_scan(v) - v; }

// Code lengths for the weights f[0..n) limited to maxbits:
// used symbols sorted by (weight, symbol);
// two-queue merge (ties take the leaf); depths; overflow redistribution; the longest
// lengths to the least frequent symbols.  One wave; NR = symbol registers (64 each).
// Sorting, depths and the length assignment are lane-parallel; only the merge is serial
// (lane 0, one LDS round trip per node: both heads of both queues are read together).
template <int NR, typename F>
__device__ void huff_lengths(K2LDS& S, const F* f, int n, int maxbits, uint8_t* len, uint32_t lane) {
    [[maybe_unused]] uint64_t kt = K2T();
    uint32_t key[NR];
    uint32_t m = 0;
#pragma unroll
    for (int r = 0; r < NR; r++) {
        const int s = r * 64 + (int)lane;
        const uint32_t fv = s < n ? f[s] : 0u;
        key[r] = fv ? ((fv << 9) | (uint32_t)s) : 0xFFFFFFFFu;
        if (s < n) len[s] = 0;
        m += (uint32_t)__popcll(__ballot(fv != 0));
    }
    wsync();
    if (m == 0) return;
    if (m == 1) {   // one used symbol: one more code of length 1 (RFC 1951 allows it)
#pragma unroll
        for (int r = 0; r < NR; r++)
            if (key[r] != 0xFFFFFFFFu) {
                const uint32_t s0 = key[r] & 511u;
                len[s0] = 1;
                len[s0 == 0 ? 1 : 0] = 1;
            }
        wsync();
        return;
    }
    // rank among the used symbols: the used keys are compacted first (into S.keys, free until
    // the merge), so the broadcast loop runs over the m used keys only, not all n slots
    const uint32_t nru = (m + 63) >> 6;   // registers holding used keys
    {
        uint32_t base = 0;
#pragma unroll
        for (int r = 0; r < NR; r++) {
            const bool u = key[r] != 0xFFFFFFFFu;
            const uint64_t um = __ballot(u);
            if (u) S.keys[base + (uint32_t)__popcll(um & ((1ull << lane) - 1ull))] = key[r];
            base += (uint32_t)__popcll(um);
        }
    }
    wsync();
    uint32_t ck[NR], rk[NR];
#pragma unroll
    for (int r = 0; r < NR; r++) {
        const uint32_t i = (uint32_t)r * 64 + lane;
        ck[r] = i < m ? S.keys[i] : 0xFFFFFFFFu;
        rk[r] = 0;
    }
#pragma unroll
    for (int r2 = 0; r2 < NR; r2++) {
        if ((uint32_t)r2 >= nru) break;
        const uint32_t cnt2 = min(m - 64u * (uint32_t)r2, 64u);
        for (uint32_t l2 = 0; l2 < cnt2; l2++) {
            const uint32_t k2 = __builtin_amdgcn_readlane(ck[r2], (int)l2);
#pragma unroll
            for (int r = 0; r < NR; r++)
                rk[r] += k2 < ck[r] ? 1u : 0u;   // (registers past nru hold 0xFFFFFFFF: counted, never scattered)
        }
    }
#pragma unroll
    for (int r = 0; r < NR; r++)
        if (ck[r] != 0xFFFFFFFFu) {
            S.fs[rk[r]] = (uint16_t)(ck[r] >> 9);
            S.sym[rk[r]] = (uint16_t)(ck[r] & 511u);
        }
    if (lane < 32) S.blc[lane] = 0;
#ifndef DMX_MERGE_BRANCHY
    // sentinels for the merge: no leaf past the last (two reads ahead), no node not yet made
    // (a weight is at most 32 770, so 0xFFFF is above every real one)
    if (lane < 2) S.fs[m + lane] = 0xFFFFu;
#pragma unroll
    for (int r = 0; r < 5; r++)
        if (r * 64 + (int)lane < 288) S.nodew[r * 64 + lane] = 0xFFFFu;
#endif
    wsync();
    K2ST(0, kt);
    const int mm = (int)m, nn = mm - 1, root = nn - 1;
    if (lane == 0) {   // two-queue merge
        int li = 0, ni = 0;
#ifndef DMX_MERGE_BRANCHY
        // branch-free (the sentinels stand for an empty queue: of two items left at least one
        // is real, so a sentinel never wins a compare it should lose): four unconditional
        // reads, selects for the picks and the two parent slots -- no exec-mask changes in
        // the loop, about half the instructions of the branchy form (K2 is half VALU-bound)
        uint16_t* const H = reinterpret_cast<uint16_t*>(&S);   // the parent slots as one u16 space
        constexpr uint32_t OL = offsetof(K2LDS, lpar) / 2, OU = offsetof(K2LDS, up) / 2;
        uint32_t ul = 0;   // leaves taken; nodes taken = 2k - ul (a node takes two items)
        for (uint32_t k = 0; k < (uint32_t)nn; k++) {
            const uint32_t un = 2 * k - ul;
            uint32_t a0 = S.fs[ul], a1 = S.fs[ul + 1], b0 = S.nodew[un], b1 = S.nodew[un + 1];
            asm volatile("" : "+v"(a0), "+v"(a1), "+v"(b0), "+v"(b1));   // (all four read, none sunk into a branch)
            const uint32_t l1 = a0 <= b0 ? 1u : 0u;
            const uint32_t q1 = l1 ? OL + ul : OU + un;
            const uint32_t w1 = l1 ? a0 : b0, A = l1 ? a1 : a0, B = l1 ? b0 : b1;
            const uint32_t ul1 = ul + l1;
            const uint32_t l2 = A <= B ? 1u : 0u;
            const uint32_t q2 = l2 ? OL + ul1 : OU + (2 * k + 1 - ul1);
            ul = ul1 + l2;
            H[q1] = (uint16_t)k;
            H[q2] = (uint16_t)k;
            S.nodew[k] = (uint16_t)(w1 + (l2 ? A : B));
        }
        (void)li;
        (void)ni;
#else
        for (int k = 0; k < nn; k++) {
            const uint32_t a0 = li < mm ? S.fs[li] : 0xFFFFFFFFu, a1 = li + 1 < mm ? S.fs[li + 1] : 0xFFFFFFFFu;
            const uint32_t b0 = ni < k ? S.nodew[ni] : 0xFFFFFFFFu, b1 = ni + 1 < k ? S.nodew[ni + 1] : 0xFFFFFFFFu;
            uint32_t w;
            uint32_t A, B;
            if (li < mm && a0 <= b0) { w = a0; S.lpar[li++] = (uint16_t)k; A = a1; B = b0; }
            else { w = b0; S.up[ni++] = (uint16_t)k; A = a0; B = b1; }
            if (li < mm && A <= B) { w += A; S.lpar[li++] = (uint16_t)k; }
            else { w += B; S.up[ni++] = (uint16_t)k; }
            S.nodew[k] = (uint16_t)w;
        }
#endif
        S.up[root] = (uint16_t)root;
    }
    wsync();
    K2ST(1, kt);
    // node depths by pointer jumping: dd = distance to up, up = an ancestor, doubling
    uint32_t u[NR], d[NR];   // (nodes < NR x 64: n <= 64 NR)
#pragma unroll
    for (int r = 0; r < NR; r++) {
        const int j = r * 64 + (int)lane;
        u[r] = j < nn ? S.up[j] : 0u;
        d[r] = (j < nn && j != root) ? 1u : 0u;
        if (j < nn) S.dd[j] = (uint16_t)d[r];
    }
    wsync();
    for (int round = 0; round < 9; round++) {   // 2^9 > 320 nodes
        uint32_t du[NR], uu[NR];
#pragma unroll
        for (int r = 0; r < NR; r++) {
            const int j = r * 64 + (int)lane;
            du[r] = j < nn ? S.dd[u[r]] : 0u;
            uu[r] = j < nn ? S.up[u[r]] : 0u;
        }
        wsync();
        bool open = false;   // a node whose ancestor is not the root yet
#pragma unroll
        for (int r = 0; r < NR; r++) {
            const int j = r * 64 + (int)lane;
            d[r] += du[r];
            u[r] = uu[r];
            if (j < nn) { S.dd[j] = (uint16_t)d[r]; S.up[j] = (uint16_t)u[r]; }
            open = open || (j < nn && u[r] != (uint32_t)root);
        }
        wsync();
        if (!__ballot(open)) break;   // every node points at the root: the depths are final (text: 5 of 9 rounds)
    }
    // leaf depths -> leaves per length
    uint32_t maxd = 0;
#pragma unroll
    for (int r = 0; r < NR; r++) {
        const int i = r * 64 + (int)lane;
        if (i < mm) {
            const uint32_t dl = S.dd[S.lpar[i]] + 1u;
            atomicAdd(&S.blc[dl], 1);
            maxd = max(maxd, dl);
        }
    }
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) maxd = max(maxd, (uint32_t)__shfl_xor((int)maxd, o));
    wsync();
    if (lane == 0) {
        if ((int)maxd > maxbits) {   // overflow redistribution (miniz style)
            for (int e = maxbits + 1; e <= (int)maxd; e++) { S.blc[maxbits] += S.blc[e]; S.blc[e] = 0; }
            uint32_t total = 0;
            for (int e = 1; e <= maxbits; e++) total += (uint32_t)S.blc[e] << (maxbits - e);
            while (total != (1u << maxbits)) {
                S.blc[maxbits]--;
                for (int e = maxbits - 1; e >= 1; e--) {
                    if (S.blc[e]) { S.blc[e]--; S.blc[e + 1] += 2; break; }
                }
                total--;
            }
        }
        int k = 0;   // sorted index where length e starts: longest lengths first
        for (int e = maxbits; e >= 1; e--) { S.lstart[e] = k; k += S.blc[e]; }
    }
    wsync();
    // sorted index i gets the first length e (from maxbits down) whose range ends past i, i.e.
    // maxbits minus the lengths 2..maxbits whose range ends at or before i: the range ends
    // from one LDS read per lane, then broadcasts (the loop over e was a chain of dependent
    // LDS reads per symbol register)
#ifdef DMX_LEN_LOOP   // (A/B build: the loop over e per symbol register)
#pragma unroll
    for (int r = 0; r < 5; r++) {
        const int i = r * 64 + (int)lane;
        if (i < mm) {
            int e = maxbits;
            while (e > 1 && i >= S.lstart[e] + S.blc[e]) e--;
            len[S.sym[i]] = (uint8_t)e;
        }
    }
#else
    const int32_t endv = (lane >= 2 && (int)lane <= maxbits) ? S.lstart[lane] + S.blc[lane] : 0x7FFFFFFF;
    int32_t cnt[NR] = {};
#pragma unroll
    for (int e = 2; e <= 15; e++) {
        const int32_t x = __builtin_amdgcn_readlane(endv, e);
#pragma unroll
        for (int r = 0; r < NR; r++) cnt[r] += (r * 64 + (int)lane) >= x ? 1 : 0;
    }
#pragma unroll
    for (int r = 0; r < NR; r++) {
        const int i = r * 64 + (int)lane;
        if (i < mm) len[S.sym[i]] = (uint8_t)(maxbits - cnt[r]);
    }
#endif
    wsync();
    K2ST(2, kt);
}

// Canonical codes (RFC 1951 §3.2.2), bit-reversed, packed code | len << 16.  Lane-parallel:
// a symbol's code = first code of its length + number of earlier symbols of that length.
template <int NR>
__device__ void canon_codes(K2LDS& S, const uint8_t* len, int n, uint32_t* out, uint32_t lane) {
    if (lane < 16) S.cnt[lane] = 0;
    wsync();
#pragma unroll
    for (int r = 0; r < NR; r++) {
        const int s = r * 64 + (int)lane;
        if (s < n && len[s]) atomicAdd(&S.cnt[len[s]], 1);
    }
    wsync();
    if (lane == 0) {
        uint32_t c = 0;
        for (int b2 = 1; b2 < 16; b2++) { c = (c + (b2 > 1 ? (uint32_t)S.cnt[b2 - 1] : 0u)) << 1; S.next[b2] = c; }
        for (int b2 = 0; b2 < 16; b2++) S.cnt[b2] = 0;
    }
    wsync();
    const uint64_t lt = (1ull << lane) - 1ull;
#pragma unroll
    for (int r = 0; r < NR; r++) {
        const int s = r * 64 + (int)lane;
        const uint32_t l = s < n ? len[s] : 0u;
        uint64_t eq = __ballot(l != 0);
#pragma unroll
        for (int bit = 0; bit < 4; bit++) {
            const bool hb = (l >> bit) & 1u;
            const uint64_t mk = __ballot(hb);
            eq &= hb ? mk : ~mk;
        }
        if (l) {
            const uint32_t base = (uint32_t)S.cnt[l];
            const uint32_t v = S.next[l] + base + (uint32_t)__popcll(eq & lt);
            out[s] = (__brev(v) >> (32 - l)) | (l << 16);
            if ((eq >> lane) == 1ull) S.cnt[l] = (int32_t)(base + (uint32_t)__popcll(eq));
        } else if (s < n) {
            out[s] = 0;
        }
        wsync();
    }
}

// Run-length coding of the concatenated lit/len + distance code lengths:
// runs are found lane-parallel, every run's symbol count has a
// closed form, and a prefix sum places each run's symbols.
__device__ void rle_lengths(K2LDS& S, uint32_t lane) {
    const int hl = S.hlit, ns = hl + S.hdist;
    uint32_t v[5];
    uint64_t sm[5];
#pragma unroll
    for (int r = 0; r < 5; r++) {
        const int k = r * 64 + (int)lane;
        v[r] = k < ns ? (k < hl ? S.lll[k] : S.ld[k - hl]) : 0xFFu;
        const uint32_t pv = (k >= 1 && k - 1 < ns) ? (k - 1 < hl ? S.lll[k - 1] : S.ld[k - 1 - hl]) : 0x1FFu;
        sm[r] = __ballot(k < ns && v[r] != pv);
    }
    uint32_t cntr[5], runl[5];
#pragma unroll
    for (int r = 0; r < 5; r++) {
        const int k = r * 64 + (int)lane;
        cntr[r] = 0;
        runl[r] = 0;
        if ((sm[r] >> lane) & 1ull) {
            int nx = ns;   // next run start
            const uint64_t above = lane == 63 ? 0ull : (sm[r] & ~((2ull << lane) - 1ull));
            if (above) nx = r * 64 + (int)__builtin_ctzll(above);
            else {
#pragma unroll
                for (int r2 = r + 1; r2 < 5; r2++)
                    if (nx == ns && sm[r2]) nx = r2 * 64 + (int)__builtin_ctzll(sm[r2]);
            }
            const uint32_t R = (uint32_t)(nx - k);
            runl[r] = R;
            if (v[r] == 0) {
                uint32_t n18 = R / 138, rem = R % 138;
                if (rem >= 11) { n18++; rem = 0; }
                cntr[r] = n18 + (rem >= 3 ? 1u : rem);
            } else {
                uint32_t rr = R - 1, n16 = rr / 6, rem = rr % 6;
                if (rem >= 3) { n16++; rem = 0; }
                cntr[r] = 1 + n16 + rem;
            }
        }
    }
    uint32_t carry = 0;
#pragma unroll
    for (int r = 0; r < 5; r++) {
        const uint32_t incl = wave_incl_scan(cntr[r]);
        uint32_t o = carry + incl - cntr[r];
        carry += __builtin_amdgcn_readlane(incl, 63);
        if (cntr[r]) {   // emit this run's symbols exactly as the sequential rule does
            uint32_t rr = runl[r];
            const uint32_t val = v[r];
            if (val == 0) {
                while (rr >= 11) { const uint32_t c = rr < 138 ? rr : 138; S.rle_sym[o] = 18; S.rle_ext[o] = (uint8_t)(c - 11); o++; rr -= c; }
                if (rr >= 3) { S.rle_sym[o] = 17; S.rle_ext[o] = (uint8_t)(rr - 3); o++; rr = 0; }
                while (rr > 0) { S.rle_sym[o] = 0; S.rle_ext[o] = 0; o++; rr--; }
            } else {
                S.rle_sym[o] = (uint8_t)val; S.rle_ext[o] = 0; o++;
                rr--;
                while (rr >= 3) { const uint32_t c = rr < 6 ? rr : 6; S.rle_sym[o] = 16; S.rle_ext[o] = (uint8_t)(c - 3); o++; rr -= c; }
                while (rr > 0) { S.rle_sym[o] = (uint8_t)val; S.rle_ext[o] = 0; o++; rr--; }
            }
        }
    }
    if (lane < 20) S.fcl[lane] = 0;
    wsync();
    if (lane == 0) S.rle_n = (int32_t)carry;
    for (uint32_t t = lane; t < carry; t += 64) atomicAdd(&S.fcl[S.rle_sym[t]], 1u);
    wsync();
}

struct HuffRes {
    uint32_t bt, hbits;
    uint64_t body, cost;
};

// The code-length alphabet of a block whose lit/len and distance lengths and HLIT / HDIST
// are in S: the run-length coding of the lengths, its Huffman lengths, HCLEN.  One wave.
__device__ void huff_cl(K2LDS& S, uint32_t lane) {
    [[maybe_unused]] uint64_t kt = K2T();
    rle_lengths(S, lane);
    K2ST(4, kt);
    huff_lengths<1>(S, S.fcl, 19, 7, S.lcl, lane);
    const uint64_t nzc = __ballot(lane < 19 && S.lcl[c_clorder[lane < 19 ? lane : 0]] != 0);
    if (lane == 0) S.hclen = nzc ? max(4, 64 - (int)__builtin_clzll(nzc)) : 4;
    wsync();
}

// Plan one DEFLATE block from the frequencies in S.fll / S.fd (EOB included): code
// lengths, exact stored / fixed / dynamic costs, the type (the cheapest; stored only if
// allow_stored) and the header's bit count.  S keeps the lengths for huff_emit.  One wave.
__device__ HuffRes huff_plan(K2LDS& S, uint32_t bn, bool allow_stored, uint32_t lane) {
    // lit/len and distance code lengths
    huff_lengths<5>(S, S.fll, 286, 15, S.lll, lane);
    huff_lengths<1>(S, S.fd, 30, 15, S.ld, lane);
    {
        const uint64_t anyd = __ballot(lane < 30 && S.ld[lane] != 0);
        if (anyd == 0 && lane < 2) S.ld[lane] = 1;   // no matches: two 1-bit codes
        // HLIT / HDIST: trailing zero lengths dropped (>= 257 / >= 1)
        int hl = 257;
#pragma unroll
        for (int r = 0; r < 5; r++) {
            const int s = r * 64 + (int)lane;
            const uint64_t nz = __ballot(s < 286 && S.lll[s] != 0);
            if (nz) hl = max(hl, r * 64 + 64 - (int)__builtin_clzll(nz));
        }
        const uint64_t nzd = __ballot(lane < 30 && S.ld[lane] != 0);
        if (lane == 0) {
            S.hlit = hl;
            S.hdist = nzd ? max(1, 64 - (int)__builtin_clzll(nzd)) : 1;
        }
        wsync();
    }
    // exact costs: the bodies first -- the frequencies share their LDS with
    // the run-length coding of the lengths (huff_cl)
    uint64_t dyn_body = 0, fix_body = 0, extra = 0;
    for (int s = (int)lane; s < 286; s += 64) {
        const uint64_t f = S.fll[s];
        dyn_body += f * S.lll[s];
        fix_body += f * fixed_len((uint32_t)s);
        if (s >= 257) extra += f * len_eb_of_sym((uint32_t)s);
    }
    if (lane < 30) {
        const uint64_t f = S.fd[lane];
        dyn_body += f * S.ld[lane];
        fix_body += f * 5;
        extra += f * dist_eb_of_sym(lane);
    }
    wsync();
    huff_cl(S, lane);
    uint64_t hdr_rle = 0;
    for (int k = (int)lane; k < S.rle_n; k += 64) hdr_rle += S.lcl[S.rle_sym[k]] + c_cl_eb[S.rle_sym[k]];
    dyn_body = wave_sum_u64(dyn_body);
    fix_body = wave_sum_u64(fix_body);
    extra = wave_sum_u64(extra);
    hdr_rle = wave_sum_u64(hdr_rle);
    const uint64_t dyn_hdr = 3 + 5 + 5 + 4 + 3 * (uint64_t)S.hclen + hdr_rle;
    const uint64_t dyn_bits = dyn_hdr + dyn_body + extra;
    const uint64_t fix_bits = 3 + fix_body + extra;
    const uint64_t sto_bits = 3 + 7 + 32 + 8 * (uint64_t)bn;
    uint32_t bt = 2;
    uint64_t best = dyn_bits;
    if (fix_bits <= best) { best = fix_bits; bt = 1; }
    if (allow_stored && sto_bits < best) { best = sto_bits; bt = 0; }
    HuffRes h;
    h.bt = bt;
    h.hbits = bt == 2 ? (uint32_t)dyn_hdr : 3u;   // = the header items huff_emit places
    h.body = (bt == 2 ? dyn_body : fix_body) + extra;
    h.cost = best;
    return h;
}

// The planned block's canonical codes into codes_out (global; fixed codes for BTYPE 1) and its
// header bits (BFINAL/BTYPE + trees) into S.hdr; returns their count.  S holds huff_plan's
// (or huff_cl's) state.  One wave.
__device__ uint32_t huff_emit(K2LDS& S, uint32_t final_bit, uint32_t bt, uint32_t lane, uint32_t* __restrict__ codes_out) {
    for (int k = (int)lane; k < DMX_HDR_WORDS; k += 64) S.hdr[k] = 0;
    wsync();
    // code table for the packer (fixed codes for BTYPE 1)
    if (bt == 1) {
        for (int s = (int)lane; s < 288; s += 64) S.lll[s] = (uint8_t)fixed_len((uint32_t)s);
        for (int s = (int)lane; s < 30; s += 64) S.ld[s] = 5;
        wsync();
    }
    // fixed codes: the canonical assignment counts all 288 lit/len lengths (RFC 1951
    // 3.2.6: 280..287 are 8-bit codes, so the 9-bit codes of 144..255 start after them);
    // slots 286/287 are overwritten by the distance codes next (never emitted)
    [[maybe_unused]] uint64_t kt = K2T();
    canon_codes<5>(S, S.lll, bt == 1 ? 288 : 286, codes_out, lane);
    canon_codes<1>(S, S.ld, 30, codes_out + DMX_DIST0, lane);
    wsync();
    K2ST(3, kt);

    // header bits: items (value, bits) placed by a prefix sum over their bit counts
    uint32_t nitems = 1;
    if (bt == 2) {
        canon_codes<1>(S, S.lcl, 19, S.ccode, lane);   // code-length codes
        nitems = 4 + (uint32_t)S.hclen + (uint32_t)S.rle_n;
    }
    uint32_t carry = 0;
    for (uint32_t base = 0; base < nitems; base += 64) {
        const uint32_t it = base + lane;
        uint32_t val = 0, nb = 0;
        if (it < nitems) {
            if (it == 0) { val = final_bit | (bt << 1); nb = 3; }
            else if (it == 1) { val = (uint32_t)(S.hlit - 257); nb = 5; }
            else if (it == 2) { val = (uint32_t)(S.hdist - 1); nb = 5; }
            else if (it == 3) { val = (uint32_t)(S.hclen - 4); nb = 4; }
            else if (it < 4 + (uint32_t)S.hclen) { val = S.lcl[c_clorder[it - 4]]; nb = 3; }
            else {
                const uint32_t t = it - 4 - (uint32_t)S.hclen, sy = S.rle_sym[t], cw = S.ccode[sy];
                const uint32_t cl = cw >> 16;
                val = (cw & 0xFFFFu) | ((uint32_t)S.rle_ext[t] << cl);
                nb = cl + c_cl_eb[sy];
            }
        }
        const uint32_t incl = wave_incl_scan(nb);
        const uint32_t pos = carry + incl - nb;
        carry += __builtin_amdgcn_readlane(incl, 63);
        if (nb) {
            const uint32_t w = pos >> 5, sh = pos & 31;
            atomicOr(&S.hdr[w], val << sh);
            if (sh + nb > 32) atomicOr(&S.hdr[w + 1], val >> (32 - sh));
        }
    }
    wsync();
    K2ST(5, kt);
    return carry;
}

__device__ __forceinline__ void huff_one(const uint32_t b, const uint32_t* __restrict__ hist_g, dmx_blkinfo* __restrict__ info,
                                         uint32_t* __restrict__ codes_g, uint32_t* __restrict__ hdr_g,
                                         dmx_subinfo* __restrict__ sub_g, uint32_t nblk, uint32_t flags) {
    __shared__ K2LDS S;
    const uint32_t lane = threadIdx.x;
    const uint32_t* hg = hist_g + (uint64_t)b * DMX_HIST;
    if (info[b].prestored & 1u) return;   // K0 wrote the stored record (1, 3)
    const uint32_t bn = info[b].n;
    const uint32_t final_bit = ((flags & DMX_F_FINAL) && b == nblk - 1) ? 1u : 0u;

    [[maybe_unused]] uint64_t kt0 = K2T();
    for (int s = (int)lane; s < 288; s += 64) S.fll[s] = s < 286 ? (s == 256 ? 1u : hg[s]) : 0u;   // + end of block
    for (int s = (int)lane; s < 32; s += 64) S.fd[s] = s < 30 ? hg[DMX_DIST0 + s] : 0u;
    wsync();
    [[maybe_unused]] uint64_t kt1 = kt0;
    K2ST(8, kt1);
    uint32_t* cg = codes_g + (uint64_t)b * DMX_NSUB * DMX_HIST;
    HuffRes h = huff_plan(S, bn, true, lane);
    K2ST(9, kt1);
    h.hbits = huff_emit(S, final_bit, h.bt, lane, cg);
    K2ST(10, kt1);
#ifdef DMX_K2_STAMPS
    if (lane == 0) { atomicAdd(&dmx_k2_st[6], (unsigned long long)(K2T() - kt0)); atomicAdd(&dmx_k2_st[7], 1ull); }
#endif
    uint32_t* hgout = hdr_g + (uint64_t)b * DMX_NSUB * DMX_HDR_WORDS;
    for (uint32_t k = lane; k < (h.hbits + 31) / 32; k += 64) hgout[k] = S.hdr[k];
    if (lane == 0) {
        info[b].btype = h.bt;
        info[b].hdr_bits = h.hbits;
        info[b].body_bits = h.body;
        info[b].nsub = 1;
        dmx_subinfo si;
        si.t0 = 0;
        si.t1 = info[b].ntok;
        si.btype = h.bt;
        si.hdr_bits = h.hbits;
        si.body_bits = h.body;
        sub_g[(uint64_t)b * DMX_NSUB] = si;
    }
}

// K2: one wave per block (wl == nullptr), or a grid that strides over K0's list L2
// (DMX_F_STORE_CHECK: the blocks parsed by K1 or in closed form by K0).
__global__ __launch_bounds__(64) __attribute__((amdgpu_waves_per_eu(8))) void dmx_huff_kernel(const uint32_t* __restrict__ hist_g, dmx_blkinfo* __restrict__ info,
                                                      uint32_t* __restrict__ codes_g, uint32_t* __restrict__ hdr_g,
                                                      dmx_subinfo* __restrict__ sub_g, uint32_t nblk, uint32_t flags,
                                                      const uint32_t* __restrict__ wl, const uint32_t* __restrict__ L2,
                                                      const uint16_t* __restrict__ codes) {
    if (!L2) {   // a workgroup per block; dups (uniform-block dedupe) take their representative's coding
        if (is_dup(codes, blockIdx.x)) return;
        huff_one(blockIdx.x, hist_g, info, codes_g, hdr_g, sub_g, nblk, flags);
        return;
    }
    const uint32_t cnt = wl[WL_N2];
    for (uint32_t i = blockIdx.x; i < cnt; i += gridDim.x) {
        wsync();   // the previous block's LDS reads are done
        huff_one(L2[i], hist_g, info, codes_g, hdr_g, sub_g, nblk, flags);
    }
}

// K2s (DMX_F_SPLIT): adaptive block splitting, DESIGN.md §4.5.  Quarter k of
// a block holds the tokens whose start lies in [(k*bn)>>2, ((k+1)*bn)>>2).  Three launches,
// so that the ten latency-bound Huffman plans per block run as separate small workgroups
// (up to 16 per CU) instead of ten waves of one 105 KB workgroup (one per CU):
//   dmx_split_hist_kernel    per block: per-quarter histograms and quarter token bounds,
//                            rebuilt from the tokens (a prefix sum of token lengths gives
//                            their starts) -> HBM scratch;
//   dmx_split_plan_kernel    per (block, group): group g is one of the 10 contiguous runs of
//                            quarters, planned with huff_block (fixed or dynamic; only the
//                            whole block keeps the stored option) -> cost, codes, header;
//   dmx_split_choose_kernel  per block: the cheapest of the 8 cut masks (ties: fewer blocks,
//                            then the smaller mask; no empty group); the chosen groups'
//                            codes, headers and token ranges into the sub-block slots.
#define SPW 10
__constant__ uint8_t c_gi[SPW] = {0, 1, 2, 3, 0, 1, 2, 0, 1, 0};
__constant__ uint8_t c_gj[SPW] = {0, 1, 2, 3, 1, 2, 3, 2, 3, 3};

struct SplitGroup {
    uint32_t bt, hbits, empty, hl;   // hl: HLIT | HDIST << 16
    uint64_t body, cost;
};
struct SplitScratch {   // per block, in HBM (dmx_ctx.split)
    uint32_t qh[4][DMX_HIST];
    uint32_t qt[8];
    SplitGroup g[SPW];
    uint8_t lens[SPW][320];   // lit/len lengths 0..287, distance lengths 288..319 (huff_plan's)
};

__device__ __forceinline__ uint32_t grp_of(uint32_t i, uint32_t j) {   // inverse of c_gi / c_gj
    const uint32_t len = j - i;   // 0: 0..3, 1: 4..6, 2: 7..8, 3: 9
    return (len == 0 ? 0u : len == 1 ? 4u : len == 2 ? 7u : 9u) + i;
}

#define SHT 640
__global__ __launch_bounds__(SHT) void dmx_split_hist_kernel(const uint32_t* __restrict__ tok_g,
                                                             const dmx_blkinfo* __restrict__ info,
                                                             SplitScratch* __restrict__ sp) {
    __shared__ uint32_t qh[4][DMX_HIST];
    __shared__ uint32_t qt[5], wsum[SHT / 64];
    const uint32_t tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
    const uint32_t b = blockIdx.x;
    if (info[b].prestored & 1u) return;   // K0 wrote the stored record (1, 3)
    const uint32_t ntok = info[b].ntok, bn = info[b].n;
    for (uint32_t k = tid; k < 4 * DMX_HIST; k += SHT) (&qh[0][0])[k] = 0;
    if (tid < 5) qt[tid] = tid == 4 ? ntok : 0u;
    __syncthreads();
    const uint32_t B1 = bn >> 2, B2 = (2 * bn) >> 2, B3 = (3 * bn) >> 2;
    const uint32_t* tb = tok_g + (uint64_t)b * DMX_BLK;
    uint32_t carry = 0, c1 = 0, c2 = 0, c3 = 0;
    for (uint32_t base = 0; base < ntok; base += SHT) {
        const uint32_t t = base + tid;
        const uint32_t tk = t < ntok ? tb[t] : 0u;
        const uint32_t adv = t < ntok ? ((tk >> 9) == 0 ? 1u : (tk & 0x1FFu)) : 0u;
        const uint32_t incl = wave_incl_scan(adv);
        if (lane == 63) wsum[wave] = incl;
        __syncthreads();
        uint32_t wbase = 0, tot = 0;
#pragma unroll
        for (uint32_t w = 0; w < SHT / 64; w++) {
            const uint32_t x = wsum[w];
            if (w < wave) wbase += x;
            tot += x;
        }
        if (t < ntok) {
            const uint32_t st = carry + wbase + incl - adv;
            const uint32_t q = (st >= B1) + (st >= B2) + (st >= B3);
            c1 += st < B1;
            c2 += st < B2;
            c3 += st < B3;
            if ((tk >> 9) == 0) {
                atomicAdd(&qh[q][tk], 1u);
            } else {
                uint32_t sy, eb, ev;
                len_sym(tk & 0x1FFu, sy, eb, ev);
                atomicAdd(&qh[q][sy], 1u);
                dist_sym(tk >> 9, sy, eb, ev);
                atomicAdd(&qh[q][DMX_DIST0 + sy], 1u);
            }
        }
        carry += tot;
        __syncthreads();
    }
    c1 = wave_sum_u32(c1);
    c2 = wave_sum_u32(c2);
    c3 = wave_sum_u32(c3);
    if (lane == 0) {
        atomicAdd(&qt[1], c1);
        atomicAdd(&qt[2], c2);
        atomicAdd(&qt[3], c3);
    }
    __syncthreads();
    SplitScratch& o = sp[b];
    for (uint32_t k = tid; k < 4 * DMX_HIST; k += SHT) (&o.qh[0][0])[k] = (&qh[0][0])[k];
    if (tid < 5) o.qt[tid] = qt[tid];
}

__global__ __launch_bounds__(64) __attribute__((amdgpu_waves_per_eu(8))) void dmx_split_plan_kernel(SplitScratch* __restrict__ sp,
                                                            const dmx_blkinfo* __restrict__ info, uint32_t nblk,
                                                            uint32_t flags) {
    __shared__ K2LDS S;
    const uint32_t lane = threadIdx.x;
    const uint32_t b = blockIdx.x / SPW, g = blockIdx.x % SPW;
    SplitScratch& o = sp[b];
    if (info[b].prestored & 1u) return;
    const uint32_t bn = info[b].n;
    const uint32_t i = c_gi[g], j = c_gj[g];
    for (int s = (int)lane; s < 288; s += 64) {
        uint32_t f = 0;
        if (s == 256) f = 1;   // end of block
        else if (s < 286)
            for (uint32_t q = i; q <= j; q++) f += o.qh[q][s];
        S.fll[s] = f;
    }
    for (int s = (int)lane; s < 32; s += 64) {
        uint32_t f = 0;
        if (s < 30)
            for (uint32_t q = i; q <= j; q++) f += o.qh[q][DMX_DIST0 + s];
        S.fd[s] = f;
    }
    wsync();
    // costs only: the codes and header of the (few) chosen groups are built by the choose kernel
    const HuffRes h = huff_plan(S, bn, g == SPW - 1, lane);
    for (uint32_t k = lane; k < 80; k += 64)
        reinterpret_cast<uint32_t*>(o.lens[g])[k] = k < 72 ? reinterpret_cast<const uint32_t*>(S.lll)[k]
                                                           : reinterpret_cast<const uint32_t*>(S.ld)[k - 72];
    if (lane == 0) {
        SplitGroup r;
        r.bt = h.bt;
        r.hbits = h.hbits;
        r.empty = o.qt[j + 1] == o.qt[i];
        r.hl = (uint32_t)S.hlit | ((uint32_t)S.hdist << 16);
        r.body = h.body;
        r.cost = h.cost;
        o.g[g] = r;
    }
}

__global__ __launch_bounds__(64) void dmx_split_choose_kernel(const SplitScratch* __restrict__ sp,
                                                              dmx_blkinfo* __restrict__ info,
                                                              uint32_t* __restrict__ codes_g,
                                                              uint32_t* __restrict__ hdr_g,
                                                              dmx_subinfo* __restrict__ sub_g, uint32_t nblk,
                                                              uint32_t flags) {
    __shared__ uint32_t sg[DMX_NSUB], nsub_s;
    __shared__ K2LDS S;
    const uint32_t lane = threadIdx.x;
    const uint32_t b = blockIdx.x;
    const SplitScratch& o = sp[b];
    if (info[b].prestored & 1u) return;
    if (lane == 0) {   // cheapest cut mask: bit k = a cut after quarter k
        int best = -1;
        uint64_t bestc = 0;
        for (uint32_t c = 0; c < 8; c++) {
            uint64_t tot = 0;
            bool ok = true;
            uint32_t start = 0;
            for (uint32_t k = 0; k < 4; k++)
                if (k == 3 || ((c >> k) & 1u)) {
                    const uint32_t g = grp_of(start, k);
                    if (o.g[g].empty) ok = false;
                    tot += o.g[g].cost;
                    start = k + 1;
                }
            if (!ok) continue;
            if (best < 0 || tot < bestc || (tot == bestc && __popc(c) < __popc((uint32_t)best))) {
                best = (int)c;
                bestc = tot;
            }
        }
        uint32_t ns = 0, start = 0;
        uint32_t hb = 0, bt = 1;
        uint64_t body = 0;
        for (uint32_t k = 0; k < 4; k++)
            if (k == 3 || (((uint32_t)best >> k) & 1u)) {
                const uint32_t g = grp_of(start, k);
                sg[ns++] = g;
                hb += o.g[g].hbits;
                body += o.g[g].body;
                if (o.g[g].bt == 2) bt = 2;
                start = k + 1;
            }
        nsub_s = ns;
        info[b].btype = ns == 1 ? o.g[sg[0]].bt : bt;
        info[b].hdr_bits = hb;
        info[b].body_bits = body;
        info[b].nsub = ns;
    }
    wsync();
    const uint32_t nsub = nsub_s;
    for (uint32_t s = 0; s < nsub; s++) {
        const uint32_t g = sg[s];
        const uint64_t slot = (uint64_t)b * DMX_NSUB + s;
        // the group's codes and header from its planned lengths (as huff_block would emit them)
        for (uint32_t k = lane; k < 80; k += 64) {
            const uint32_t w = reinterpret_cast<const uint32_t*>(o.lens[g])[k];
            if (k < 72) reinterpret_cast<uint32_t*>(S.lll)[k] = w;
            else reinterpret_cast<uint32_t*>(S.ld)[k - 72] = w;
        }
        if (lane == 0) {
            S.hlit = (int32_t)(o.g[g].hl & 0xFFFFu);
            S.hdist = (int32_t)(o.g[g].hl >> 16);
        }
        wsync();
        if (o.g[g].bt == 2) huff_cl(S, lane);
        const uint32_t final_bit = ((flags & DMX_F_FINAL) && b == nblk - 1 && c_gj[g] == 3) ? 1u : 0u;
        const uint32_t hbits = huff_emit(S, final_bit, o.g[g].bt, lane, codes_g + slot * DMX_HIST);
        uint32_t* hg = hdr_g + slot * DMX_HDR_WORDS;
        for (uint32_t k = lane; k < (hbits + 31) / 32; k += 64) hg[k] = S.hdr[k];
        if (lane == 0) {
            dmx_subinfo si;
            si.t0 = o.qt[c_gi[g]];
            si.t1 = o.qt[c_gj[g] + 1];
            si.btype = o.g[g].bt;
            si.hdr_bits = o.g[g].hbits;
            si.body_bits = o.g[g].body;
            sub_g[slot] = si;
        }
    }
}

// ------------------------------------------------------------------------------------
// K3: block offsets (scan), Adler-32, framing
// ------------------------------------------------------------------------------------

// x -> s ? align8(x + a) + c : x + c   (stored blocks re-align; composable)
struct Mono {
    uint32_t s;
    uint64_t a, c;
};
__device__ __forceinline__ uint64_t align8(uint64_t x) { return (x + 7) & ~7ull; }
__device__ __forceinline__ Mono mcompose(const Mono& f, const Mono& g) {  // f first, then g
    Mono r;
    if (!g.s) { r.s = f.s; r.a = f.a; r.c = f.c + g.c; }
    else if (!f.s) { r.s = 1; r.a = f.c + g.a; r.c = g.c; }
    else { r.s = 1; r.a = f.a; r.c = align8(f.c + g.a) + g.c; }
    return r;
}
__device__ __forceinline__ uint64_t mapply(const Mono& f, uint64_t x) { return f.s ? align8(x + f.a) + f.c : x + f.c; }
__device__ __forceinline__ Mono mshfl_up(const Mono& v, int o) {
    Mono r;
    r.s = __shfl_up(v.s, o);
    r.a = __shfl_up(v.a, o);
    r.c = __shfl_up(v.c, o);
    return r;
}

__device__ __forceinline__ void gor_bits(uint32_t* out32, uint64_t pos, uint32_t v, uint32_t nb) {
    if (!nb) return;
    const uint64_t w = pos >> 5;
    const uint32_t sh = (uint32_t)(pos & 31);
    atomicOr(&out32[w], v << sh);
    if (sh + nb > 32) atomicOr(&out32[w + 1], v >> (32 - sh));
}

// zlib header (bits 0..15), the sync flush after a non-final shard's last block, the
// Adler-32 trailer; T = end of the last block, end = byte-aligned end of the DEFLATE data.
__device__ __forceinline__ void stream_framing(uint32_t* out32, uint32_t flags, uint32_t nblk, uint64_t T,
                                               uint64_t end, uint32_t adler) {
    const uint64_t start = (flags & DMX_F_HEADER) ? 16 : 0;
    if (flags & DMX_F_HEADER) gor_bits(out32, 0, 0x9C78u, 16);
    if (nblk == 0 && (flags & DMX_F_FINAL)) gor_bits(out32, start, 3u, 3);  // BFINAL=1, BTYPE=01, EOB=0000000
    if (!(flags & DMX_F_FINAL) && nblk > 0) gor_bits(out32, align8(T + 3) + 16, 0xFFFFu, 16);  // sync flush
    if (flags & DMX_F_TRAILER) {
        const uint32_t a = adler;
        const uint32_t be = (a >> 24) | ((a >> 8) & 0xFF00u) | ((a << 8) & 0xFF0000u) | (a << 24);
        gor_bits(out32, end, be, 32);
    }
}

#define ST 1024
#define ADL_MOD 65521u
#define SCAN_TILE 256

// K3, the stream layout, in three launches so that the per-block records are read by many
// CUs (one workgroup reading 32 768 records of 64 B was 0.2 ms):
//   dmx_scan_tile_kernel   per tile of 256 blocks: the blocks' layout elements (Mono: bits,
//                          or "align then bits" for stored blocks) scanned in the tile; each
//                          block's tile-local exclusive prefix parked in its off_bits/len_bits,
//                          the tile aggregate and the Adler/token/type partial sums -> tiles[];
//   dmx_scan_kernel        one workgroup: the tile aggregates -> tile prefixes, stream end,
//                          Adler-32, out_len, status (dmx_result); zeroes the words past the
//                          last block; an empty input gets its whole stream here;
//   dmx_scan_apply_kernel  per tile: absolute offsets, and zero the words each block shares
//                          with a neighbour (the pack kernel ORs those).
// The zlib header, sync flush and trailer are ORed by the pack kernel (first/last block).
struct ScanTile {
    uint64_t a, c, s;                      // aggregate Mono (s: has a stored block)
    uint64_t ps, pa, pc;                   // exclusive prefix over the tiles before
    uint64_t adl_s1, adl_s2, ntok, nsto, nfix;
    uint64_t kinds;   // K0's block kinds in the tile (16-bit fields: prestored 0, 2, 3, dedupe candidates)
    uint64_t pad_[4];
};

__device__ __forceinline__ Mono blk_elem(const dmx_blkinfo& bi) {
    Mono e = {0, 0, 0};
    if (bi.btype == 0) { e.s = 1; e.a = 3; e.c = 32 + 8 * (uint64_t)bi.n; }
    else { e.c = bi.hdr_bits + bi.body_bits; }
    return e;
}

__global__ __launch_bounds__(SCAN_TILE) void dmx_scan_tile_kernel(dmx_blkinfo* __restrict__ info, uint32_t nblk,
                                                                 uint64_t n, uint32_t sw, ScanTile* __restrict__ tiles,
                                                                 const uint16_t* __restrict__ codes,
                                                                 const uint32_t* __restrict__ dup,
                                                                 dmx_subinfo* __restrict__ sub_g) {
    __shared__ Mono wtot[SCAN_TILE / 64];
    __shared__ uint64_t red[SCAN_TILE / 64][6];
    const uint32_t tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
    const uint32_t b = blockIdx.x * SCAN_TILE + tid;
    Mono e = {0, 0, 0};
    uint64_t s1 = 0, s2 = 0, nt = 0, ns = 0, nf = 0, kd = 0;
    if (b < nblk) {
        dmx_blkinfo bi = info[b];
        {   // (the launch-shape hint: what K0 decided, DMX_F_STORE_CHECK)
            const uint32_t ps = bi.prestored;
            kd = (ps & 3u) == 0 ? 1ull : (ps & 3u) == 2 ? (1ull << 16) | ((ps & 4u) ? 1ull << 48 : 0ull)
                                       : (ps & 3u) == 3 ? 1ull << 32 : 0ull;
        }
        if (is_dup(codes, b)) {   // a dup (uniform-block dedupe): the representative's coding
            const uint32_t r = dup[b];
            const dmx_blkinfo ri = info[r];
            bi.btype = ri.btype;
            bi.hdr_bits = ri.hdr_bits;
            bi.body_bits = ri.body_bits;
            bi.nsub = ri.nsub;
            info[b].btype = ri.btype;
            info[b].hdr_bits = ri.hdr_bits;
            info[b].body_bits = ri.body_bits;
            info[b].nsub = ri.nsub;
            sub_g[(uint64_t)b * DMX_NSUB] = sub_g[(uint64_t)r * DMX_NSUB];
        }
        e = blk_elem(bi);
        const uint64_t end_b = (uint64_t)b * sw + bi.n;
        s1 = bi.adl_s % ADL_MOD;
        s2 = (bi.adl_w % ADL_MOD + ((n - end_b) % ADL_MOD) * s1) % ADL_MOD;
        nt = bi.ntok;
        ns = bi.btype == 0;
        nf = bi.btype == 1;
    }
    Mono x = e;
#pragma unroll
    for (int o = 1; o < 64; o <<= 1) {
        const Mono y = mshfl_up(x, o);
        if (lane >= (uint32_t)o) x = mcompose(y, x);
    }
    const Mono before = mshfl_up(x, 1);
    if (lane == 63) wtot[wave] = x;
    s1 = wave_sum_u64(s1);
    s2 = wave_sum_u64(s2);
    nt = wave_sum_u64(nt);
    ns = wave_sum_u64(ns);
    nf = wave_sum_u64(nf);
    kd = wave_sum_u64(kd);
    if (lane == 0) { red[wave][0] = s1; red[wave][1] = s2; red[wave][2] = nt; red[wave][3] = ns; red[wave][4] = nf; red[wave][5] = kd; }
    __syncthreads();
    Mono pre = {0, 0, 0};
    for (uint32_t w = 0; w < wave; w++) pre = mcompose(pre, wtot[w]);
    if (lane) pre = mcompose(pre, before);
    if (b < nblk) {   // tile-local exclusive prefix, finished by dmx_scan_apply_kernel
        info[b].off_bits = pre.c;
        info[b].len_bits = ((uint64_t)pre.s << 32) | pre.a;
    }
    if (tid == 0) {
        Mono agg = {0, 0, 0};
        uint64_t a1 = 0, a2 = 0, t2 = 0, t3 = 0, t4 = 0, t5 = 0;
        for (int w = 0; w < SCAN_TILE / 64; w++) {
            agg = mcompose(agg, wtot[w]);
            a1 += red[w][0]; a2 += red[w][1]; t2 += red[w][2]; t3 += red[w][3]; t4 += red[w][4]; t5 += red[w][5];
        }
        ScanTile& T = tiles[blockIdx.x];
        T.a = agg.a; T.c = agg.c; T.s = agg.s;
        T.adl_s1 = a1 % ADL_MOD; T.adl_s2 = a2 % ADL_MOD; T.ntok = t2; T.nsto = t3; T.nfix = t4; T.kinds = t5;
    }
}

__global__ __launch_bounds__(ST) void dmx_scan_kernel(ScanTile* __restrict__ tiles, uint32_t nblk, uint64_t n,
                                                      uint32_t flags, uint64_t out_cap,
                                                      uint32_t* __restrict__ out32, dmx_result* __restrict__ res,
                                                      uint32_t* __restrict__ nfallback, uint32_t* __restrict__ hint) {
    __shared__ Mono wtot[ST / 64];
    __shared__ uint32_t kcnt[4];
    __shared__ Mono carry_s;
    __shared__ uint64_t red[ST / 64][5];
    const uint32_t tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
    const uint64_t start = (flags & DMX_F_HEADER) ? 16 : 0;
    const uint32_t ntile = (nblk + SCAN_TILE - 1) / SCAN_TILE;
    uint64_t adl_s1 = 0, adl_s2 = 0, ntok = 0, nsto = 0, nfix = 0;
    uint32_t k0 = 0, k2 = 0, k3 = 0, ku = 0;
    if (tid < 4) kcnt[tid] = 0;
    // thread t owns tiles [t C, t C + C)
    const uint32_t C = (ntile + ST - 1) / ST;
    const uint32_t t0 = tid * C < ntile ? tid * C : ntile, t1 = t0 + C < ntile ? t0 + C : ntile;
    Mono agg = {0, 0, 0};
    for (uint32_t t = t0; t < t1; t++) {
        const ScanTile T = tiles[t];
        Mono e;
        e.s = (uint32_t)T.s; e.a = T.a; e.c = T.c;
        agg = mcompose(agg, e);
        adl_s1 = (adl_s1 + T.adl_s1) % ADL_MOD;
        adl_s2 = (adl_s2 + T.adl_s2) % ADL_MOD;
        ntok += T.ntok;
        nsto += T.nsto;
        nfix += T.nfix;
        k0 += (uint32_t)(T.kinds & 0xFFFFu);
        k2 += (uint32_t)((T.kinds >> 16) & 0xFFFFu);
        k3 += (uint32_t)((T.kinds >> 32) & 0xFFFFu);
        ku += (uint32_t)(T.kinds >> 48);
    }
    Mono x = agg;  // inclusive scan in the wave
#pragma unroll
    for (int o = 1; o < 64; o <<= 1) {
        const Mono y = mshfl_up(x, o);
        if (lane >= (uint32_t)o) x = mcompose(y, x);
    }
    if (lane == 63) wtot[wave] = x;
    __syncthreads();   // (kcnt zeroed)
    if (hint) {   // the launch-shape hint of an encode without the work lists (wl_shape)
        if (k0) atomicAdd(&kcnt[0], k0);
        if (k2) atomicAdd(&kcnt[1], k2);
        if (k3) atomicAdd(&kcnt[2], k3);
        if (ku) atomicAdd(&kcnt[3], ku);
    }
    if (tid == 0) {   // exclusive prefix over waves
        Mono acc = {0, 0, 0};
        for (int w = 0; w < ST / 64; w++) {
            const Mono t = wtot[w];
            wtot[w] = acc;
            acc = mcompose(acc, t);
        }
        carry_s = acc;
    }
    __syncthreads();
    {
        const Mono before = mshfl_up(x, 1);
        Mono pre = (lane == 0) ? wtot[wave] : mcompose(wtot[wave], before);
        for (uint32_t t = t0; t < t1; t++) {
            tiles[t].ps = pre.s; tiles[t].pa = pre.a; tiles[t].pc = pre.c;
            Mono e;
            e.s = (uint32_t)tiles[t].s; e.a = tiles[t].a; e.c = tiles[t].c;
            pre = mcompose(pre, e);
        }
    }
    // reductions
    adl_s1 = wave_sum_u64(adl_s1 % ADL_MOD);
    adl_s2 = wave_sum_u64(adl_s2 % ADL_MOD);
    ntok = wave_sum_u64(ntok);
    nsto = wave_sum_u64(nsto);
    nfix = wave_sum_u64(nfix);
    if (lane == 0) { red[wave][0] = adl_s1; red[wave][1] = adl_s2; red[wave][2] = ntok; red[wave][3] = nsto; red[wave][4] = nfix; }
    __syncthreads();
    __shared__ uint64_t s_end, s_T;
    __shared__ uint32_t s_adler;
    __shared__ int32_t s_status;
    if (tid == 0) {
        uint64_t s1 = 0, s2 = 0, nt = 0, ns = 0, nf = 0;
        for (int w = 0; w < ST / 64; w++) { s1 += red[w][0]; s2 += red[w][1]; nt += red[w][2]; ns += red[w][3]; nf += red[w][4]; }
        s1 = (1 + s1) % ADL_MOD;
        s2 = (n % ADL_MOD + s2) % ADL_MOD;
        const uint32_t adler = (uint32_t)((s2 << 16) | s1);
        uint64_t T = mapply(carry_s, start);
        if (nblk == 0 && (flags & DMX_F_FINAL)) T = start + 10;   // empty input: fixed block, EOB only
        uint64_t end = (flags & DMX_F_FINAL) ? align8(T) : (nblk == 0 ? align8(T) : align8(T + 3) + 32);
        uint64_t out_len = end / 8 + ((flags & DMX_F_TRAILER) ? 4 : 0);
        int32_t status = 0;
        if (((out_len + 3) & ~3ull) > out_cap) status = -(int32_t)E_SZ;
        res->out_len = out_len;
        res->end_bits = T;
        res->n = n;
        res->ntokens = nt;
        res->adler = adler;
        res->status = status;
        res->nblocks = nblk;
        res->nstored = (uint32_t)ns;
        res->nfixed = (uint32_t)nf;
        res->ndynamic = nblk - (uint32_t)ns - (uint32_t)nf;
        res->nsortfallback = nfallback[0];   // this encode's sort fallbacks; zeroed for the next
        nfallback[1] += nfallback[0];       // and the context's running total
        res->nsortfallback_total = nfallback[1];
        nfallback[0] = 0;
        if (hint) {   // {nblk, |L1|, |L2|, |L4| (the blocks K4 would take), dedupe candidates}
            __hip_atomic_store(&hint[0], nblk, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
            __hip_atomic_store(&hint[1], kcnt[0], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
            __hip_atomic_store(&hint[2], kcnt[0] + kcnt[1], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
            __hip_atomic_store(&hint[3], nblk - kcnt[2], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
            __hip_atomic_store(&hint[4], kcnt[3], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
        }
        s_end = end;
        s_T = T;
        s_adler = adler;
        s_status = status;
    }
    __syncthreads();
    if (s_status) return;
    // zero the words past the last block (the framing goes there)
    const uint64_t T = s_T, end = s_end;
    const uint64_t tail_end = end + ((flags & DMX_F_TRAILER) ? 32 : 0);
    // (word T >> 5, when the last block ends inside it, is that block's last word: the apply
    // launch zeroes it, keeping any bytes of the whole-copy prefix it holds)
    const uint64_t tw0 = nblk ? (T + 31) >> 5 : T >> 5;
    for (uint64_t w = tw0 + tid; w < ((tail_end + 31) >> 5); w += ST) out32[w] = 0;
    if (nblk == 0) {   // no pack launch: the whole stream is written here
        if (tid == 0 && start) out32[0] = 0;
        __syncthreads();
        if (tid == 0) stream_framing(out32, flags, 0, T, end, s_adler);
    }
}

__global__ __launch_bounds__(SCAN_TILE) void dmx_scan_apply_kernel(dmx_blkinfo* __restrict__ info, uint32_t nblk,
                                                                  uint32_t flags, uint32_t sw, const ScanTile* __restrict__ tiles,
                                                                  uint32_t* __restrict__ out32,
                                                                  const dmx_result* __restrict__ res,
                                                                  uint32_t* __restrict__ wl, uint32_t* __restrict__ L4,
                                                                  const uint16_t* __restrict__ codes) {
    if (res->status) return;
    const uint32_t b = blockIdx.x * SCAN_TILE + threadIdx.x;
    if (b >= nblk) return;
    const uint64_t start = (flags & DMX_F_HEADER) ? 16 : 0;
    const ScanTile& T = tiles[blockIdx.x];
    Mono tp, lp;
    tp.s = (uint32_t)T.ps; tp.a = T.pa; tp.c = T.pc;
    const dmx_blkinfo bi = info[b];
    lp.c = bi.off_bits; lp.s = (uint32_t)(bi.len_bits >> 32); lp.a = bi.len_bits & 0xFFFFFFFFu;
    const Mono pre = mcompose(tp, lp);
    const uint64_t o = mapply(pre, start);
    const uint64_t l = mapply(blk_elem(bi), o) - o;
    info[b].off_bits = o;
    info[b].len_bits = l;
    if (!wl) {
        out32[o >> 5] = 0;            // shared with the block before (or the zlib header)
        out32[(o + l - 1) >> 5] = 0;  // shared with the block after (or the framing)
        return;
    }
    // work lists: a block of the whole-copy prefix has its quads from K0 and gets the rest of
    // its bytes from K0 too (or the fill kernel: stored_rest, byte stores): nothing to zero; every other block zeroes its edge words -- only its own bytes where the neighbour is a
    // whole-copy block (that boundary is a byte boundary: both sides are stored blocks at their
    // speculative offsets) -- and goes on K4's list
    const uint32_t M = wl[WL_M];
    if (wl_skip(b, M, nblk)) return;
    uint64_t A, P;
    wl_prefix_bytes(M, nblk, sw, flags, A, P);
    const uint64_t w0 = o >> 5, w1 = (o + l - 1) >> 5;
    zero_word_keep(out32, w0, A, P);
    if (w1 != w0) zero_word_keep(out32, w1, A, P);
    if (is_dup(codes, b)) return;   // packed by dmx_dup_copy_kernel
    L4[atomicAdd(&wl[WL_N4], 1u)] = b;
}

// K3 in two launches when the stream has at most SA1_MAXT tiles (8 GiB of 32 KiB blocks):
// dmx_scan_tile_kernel as above, then this kernel, a workgroup per tile, which composes the
// tile aggregates itself (at most 4 per thread) -- its tile's prefix and the stream's total,
// hence the status every workgroup needs before it writes -- instead of a one-workgroup
// dmx_scan_kernel launch between the two.  The last tile's workgroup also does what that
// launch did once: Adler-32, the dmx_result record, the fallback counters, the hint and the
// words past the last block.  Then each block: as dmx_scan_apply_kernel.
#define SA1_MAXT (4 * SCAN_TILE)
__global__ __launch_bounds__(SCAN_TILE) void dmx_scan_apply1_kernel(dmx_blkinfo* __restrict__ info, uint32_t nblk, uint64_t n,
                                                                   uint32_t flags, uint64_t out_cap, uint32_t sw,
                                                                   const ScanTile* __restrict__ tiles,
                                                                   uint32_t* __restrict__ out32, dmx_result* __restrict__ res,
                                                                   uint32_t* __restrict__ nfallback, uint32_t* __restrict__ hint,
                                                                   uint32_t* __restrict__ wl, uint32_t* __restrict__ L4,
                                                                   const uint16_t* __restrict__ codes) {
    __shared__ Mono wt[SCAN_TILE / 64];
    __shared__ Mono s_pre;
    __shared__ uint64_t red[SCAN_TILE / 64][9];
    const uint32_t tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
    const uint32_t ntile = (nblk + SCAN_TILE - 1) / SCAN_TILE, tt = blockIdx.x;
    const bool lastwg = tt + 1 == ntile;
    const uint64_t start = (flags & DMX_F_HEADER) ? 16 : 0;
    // thread i composes tiles [i C, i C + C) in order; the one holding tile tt notes the part before it
    const uint32_t C = (ntile + SCAN_TILE - 1) / SCAN_TILE;
    const uint32_t t0 = tid * C < ntile ? tid * C : ntile, t1 = t0 + C < ntile ? t0 + C : ntile;
    Mono agg = {0, 0, 0}, part = {0, 0, 0};
    bool mine = false;
    uint64_t s1 = 0, s2 = 0, nt = 0, ns = 0, nf = 0, k0 = 0, k2 = 0, k3 = 0, ku = 0;
    for (uint32_t u = t0; u < t1; u++) {
        const ScanTile T = tiles[u];
        if (u == tt) { part = agg; mine = true; }
        Mono e;
        e.s = (uint32_t)T.s; e.a = T.a; e.c = T.c;
        agg = mcompose(agg, e);
        if (lastwg) {
            s1 = (s1 + T.adl_s1) % ADL_MOD;
            s2 = (s2 + T.adl_s2) % ADL_MOD;
            nt += T.ntok; ns += T.nsto; nf += T.nfix;
            k0 += T.kinds & 0xFFFFu; k2 += (T.kinds >> 16) & 0xFFFFu; k3 += (T.kinds >> 32) & 0xFFFFu; ku += T.kinds >> 48;
        }
    }
    Mono x = agg;   // inclusive scan over the threads' ranges
#pragma unroll
    for (int o = 1; o < 64; o <<= 1) {
        const Mono y = mshfl_up(x, o);
        if (lane >= (uint32_t)o) x = mcompose(y, x);
    }
    const Mono before = mshfl_up(x, 1);
    if (lane == 63) wt[wave] = x;
    if (lastwg) {
        s1 = wave_sum_u64(s1); s2 = wave_sum_u64(s2); nt = wave_sum_u64(nt);
        ns = wave_sum_u64(ns); nf = wave_sum_u64(nf);
        k0 = wave_sum_u64(k0); k2 = wave_sum_u64(k2); k3 = wave_sum_u64(k3); ku = wave_sum_u64(ku);
        if (lane == 0) {
            red[wave][0] = s1; red[wave][1] = s2; red[wave][2] = nt; red[wave][3] = ns; red[wave][4] = nf;
            red[wave][5] = k0; red[wave][6] = k2; red[wave][7] = k3; red[wave][8] = ku;
        }
    }
    __syncthreads();
    Mono tot = {0, 0, 0}, wpre = {0, 0, 0};
#pragma unroll
    for (int w = 0; w < SCAN_TILE / 64; w++) {
        if (w == (int)wave) wpre = tot;
        tot = mcompose(tot, wt[w]);
    }
    if (mine) s_pre = mcompose(lane ? mcompose(wpre, before) : wpre, part);
    // the stream's end and status (every workgroup: nothing is written past out_cap)
    const uint64_t T = mapply(tot, start);
    const uint64_t end = (flags & DMX_F_FINAL) ? align8(T) : align8(T + 3) + 32;
    const uint64_t out_len = end / 8 + ((flags & DMX_F_TRAILER) ? 4 : 0);
    const int32_t status = (((out_len + 3) & ~3ull) > out_cap) ? -(int32_t)E_SZ : 0;
    if (lastwg && tid == 0) {
        uint64_t a1 = 0, a2 = 0, ntk = 0, nst = 0, nfx = 0, q0 = 0, q2 = 0, q3 = 0, qu = 0;
        for (int w = 0; w < SCAN_TILE / 64; w++) {
            a1 += red[w][0]; a2 += red[w][1]; ntk += red[w][2]; nst += red[w][3]; nfx += red[w][4];
            q0 += red[w][5]; q2 += red[w][6]; q3 += red[w][7]; qu += red[w][8];
        }
        a1 = (1 + a1) % ADL_MOD;
        a2 = (n % ADL_MOD + a2) % ADL_MOD;
        res->out_len = out_len;
        res->end_bits = T;
        res->n = n;
        res->ntokens = ntk;
        res->adler = (uint32_t)((a2 << 16) | a1);
        res->status = status;
        res->nblocks = nblk;
        res->nstored = (uint32_t)nst;
        res->nfixed = (uint32_t)nfx;
        res->ndynamic = nblk - (uint32_t)nst - (uint32_t)nfx;
        res->nsortfallback = nfallback[0];
        nfallback[1] += nfallback[0];
        res->nsortfallback_total = nfallback[1];
        nfallback[0] = 0;
        if (hint) {   // as dmx_scan_kernel
            __hip_atomic_store(&hint[0], nblk, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
            __hip_atomic_store(&hint[1], (uint32_t)q0, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
            __hip_atomic_store(&hint[2], (uint32_t)(q0 + q2), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
            __hip_atomic_store(&hint[3], nblk - (uint32_t)q3, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
            __hip_atomic_store(&hint[4], (uint32_t)qu, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
        }
    }
    if (status) return;
    if (lastwg) {   // zero the words past the last block (the framing goes there)
        const uint64_t tail_end = end + ((flags & DMX_F_TRAILER) ? 32 : 0);
        for (uint64_t w = ((T + 31) >> 5) + tid; w < ((tail_end + 31) >> 5); w += SCAN_TILE) out32[w] = 0;   // (as dmx_scan_kernel)
    }
    __syncthreads();   // (s_pre)
    const uint32_t b = tt * SCAN_TILE + tid;
    if (b >= nblk) return;
    const Mono tp = s_pre;
    Mono lp;
    const dmx_blkinfo bi = info[b];
    lp.c = bi.off_bits; lp.s = (uint32_t)(bi.len_bits >> 32); lp.a = bi.len_bits & 0xFFFFFFFFu;
    const Mono pre = mcompose(tp, lp);
    const uint64_t o = mapply(pre, start);
    const uint64_t l = mapply(blk_elem(bi), o) - o;
    info[b].off_bits = o;
    info[b].len_bits = l;
    if (!wl) {
        out32[o >> 5] = 0;
        out32[(o + l - 1) >> 5] = 0;
        return;
    }
    const uint32_t M = wl[WL_M];
    if (wl_skip(b, M, nblk)) return;
    uint64_t A, P;
    wl_prefix_bytes(M, nblk, sw, flags, A, P);
    const uint64_t w0 = o >> 5, w1 = (o + l - 1) >> 5;
    zero_word_keep(out32, w0, A, P);
    if (w1 != w0) zero_word_keep(out32, w1, A, P);
    if (is_dup(codes, b)) return;
    L4[atomicAdd(&wl[WL_N4], 1u)] = b;
}

// ------------------------------------------------------------------------------------
// K4: bit packing
// ------------------------------------------------------------------------------------

#ifndef PT
#define PT 256
#endif
#ifndef TPT
#define TPT 4   // tokens per thread per packing round (8: 0.087 ms on C3, 4: 0.080)
#endif
#ifndef PK_RING
#define PK_RING 2048   // pack ring words: > 1 + max(160 header words, PT x TPT tokens x 48 bits / 32) + 1
#endif
static_assert(PK_RING > 2 + (PT * TPT * 48) / 32 && PK_RING > 162, "pack ring too small for a round");

// A workgroup barrier that orders LDS only: global loads in flight (the next round's tokens)
// stay in flight across it (__syncthreads() also waits for every outstanding global access).
__device__ __forceinline__ void lds_barrier() {
    asm volatile("s_waitcnt lgkmcnt(0)\n\ts_barrier" ::: "memory");
}

__device__ __forceinline__ void st_or64(uint32_t* st, uint32_t pos, uint64_t v, uint32_t nb) {
    if (!nb) return;
    const uint32_t w = pos >> 5, sh = pos & 31;
    const uint64_t a = v << sh;
    atomicOr(&st[w], (uint32_t)a);
    if (sh + nb > 32) atomicOr(&st[w + 1], (uint32_t)(a >> 32));
    if (sh + nb > 64) atomicOr(&st[w + 2], (uint32_t)(v >> (64 - sh)));
}

// The first block ORs the zlib header, the last one the sync flush / trailer (the scan
// zeroed those words; every write into them is an atomicOr).
__device__ __forceinline__ void pack_framing(uint32_t* out32, uint32_t flags, uint32_t nblk, uint32_t b,
                                             const dmx_result* res) {
    if (b == 0 && (flags & DMX_F_HEADER)) gor_bits(out32, 0, 0x9C78u, 16);
    if (b == nblk - 1) {
        const uint64_t T = res->end_bits;
        const uint64_t end = (flags & DMX_F_FINAL) ? align8(T) : align8(T + 3) + 32;
        stream_framing(out32, flags & ~DMX_F_HEADER, nblk, T, end, res->adler);
    }
}

__device__ __forceinline__ void pack_one(const uint32_t b, const uint8_t* __restrict__ in, uint32_t sw,
                                         const uint32_t* __restrict__ tok_g, const uint32_t* __restrict__ codes_g,
                                         const uint32_t* __restrict__ hdr_g, const dmx_blkinfo* __restrict__ info,
                                         const dmx_subinfo* __restrict__ sub_g,
                                         uint32_t nblk, uint32_t flags, uint32_t* __restrict__ out32,
                                         dmx_result* __restrict__ res) {
    __shared__ uint32_t stage[PK_RING];
    __shared__ uint32_t code[DMX_HIST];
#ifndef DMX_PACK_OLD
    // one entry per first piece of a token, value | bits << 24: literals 0..255, then the
    // lengths 3..258 with their extra bits appended (the length symbol, its code and its extra
    // bits in one read instead of len_sym arithmetic and a branch per token)
    __shared__ uint32_t ptab[512];
#endif
    __shared__ uint32_t wsum[PT / 64];
    const uint32_t tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
    const dmx_blkinfo bi = info[b];   // in flight with the status load (a stored block's WG is
    if (res->status) return;          // a chain of dependent loads: C4 launches 32 768 of them)
    const uint64_t O = bi.off_bits, Lb = bi.len_bits;
    const uint32_t s0 = (uint32_t)(O & 31);
    const uint32_t nwords = (uint32_t)((s0 + Lb + 31) >> 5);
    const uint32_t final_bit = ((flags & DMX_F_FINAL) && b == nblk - 1) ? 1u : 0u;
    if (bi.btype == 0) {
        // stored block straight from the input to the output, no LDS: the 3 header bits at s0,
        // LEN/NLEN at byte P/8, the data from byte B0 (bit offsets relative to word O >> 5).
        // Whole output quads (16-byte aligned in the stream) come from one 20-byte read of
        // the block and byte alignment in registers; the first word, the ragged ends and
        // unaligned blocks take the bytewise path.  The first and last words are shared
        // with the neighbouring blocks (zeroed by the scan kernel): atomicOr there.
        const uint8_t* d = in + (uint64_t)b * sw;
        const uint32_t bn = bi.n;
        const uint32_t P = (s0 + 3 + 7) & ~7u, B0 = (P + 32) >> 3;
        const uint32_t lenw = (bn & 0xFFFFu) | ((~bn & 0xFFFFu) << 16);
        const uint64_t gw0 = O >> 5;
        auto gen_word = [&](uint32_t k) -> uint32_t {
            uint32_t v = 0;
#pragma unroll
            for (uint32_t i = 0; i < 4; i++) {
                const uint32_t q = 4 * k + i;
                uint32_t by;
                if (q >= B0) by = (q - B0) < bn ? d[q - B0] : 0u;
                else if (q >= (P >> 3)) by = (lenw >> (8 * (q - (P >> 3)))) & 0xFFu;
                else by = (uint32_t)((((uint64_t)final_bit << s0) >> (8 * q)) & 0xFFu);
                v |= by << (8 * i);
            }
            return v;
        };
        auto put_word = [&](uint32_t k, uint32_t v) {
            if ((k == 0 && s0 != 0) || (k == nwords - 1 && ((s0 + Lb) & 31) != 0)) atomicOr(&out32[gw0 + k], v);
            else out32[gw0 + k] = v;
        };
        const bool dal = (reinterpret_cast<uintptr_t>(d) & 3) == 0;
        // K0's speculative copy landed where the scan put the block: its quads are written
        const bool spec = bi.prestored == 3 && O == spec_stored_bit(b, sw, flags);
        const uint32_t ks = 4 - (uint32_t)(gw0 & 3);                      // first quad: (gw0 + ks) % 4 == 0, ks >= 1
        const uint32_t nq = (dal && nwords > ks + 1) ? (nwords - 1 - ks) >> 2 : 0;   // quads short of the last word
        // With the copy in place only the first two and the last two quads can need words of
        // their own: quad j >= 2 starts at byte >= 36 > B0 (<= 9), and quad j <= nq - 3 ends
        // >= 44 bytes before the block's end, so both take the fast path, which K0 wrote.
        const uint32_t nqv = spec ? (nq < 4 ? nq : 4u) : nq;
        for (uint32_t t = tid; t < nqv; t += PT) {
            const uint32_t j = (spec && t >= 2) ? nq - (nqv - t) : t;
            const uint32_t k = ks + 4 * j;
            const int64_t o0 = (int64_t)(4 * k) - (int64_t)B0;
            if (o0 >= 0 && (uint64_t)((o0 & ~3ll) + 20) <= bn) {
                if (spec) continue;
                const uint32_t* p32 = reinterpret_cast<const uint32_t*>(d + (o0 & ~3ll));
                const uint32_t w0 = p32[0], w1 = p32[1], w2 = p32[2], w3 = p32[3], w4 = p32[4];
                const uint32_t sh = (uint32_t)(o0 & 3);
                uint4 v;
                v.x = sh ? __builtin_amdgcn_alignbyte(w1, w0, sh) : w0;
                v.y = sh ? __builtin_amdgcn_alignbyte(w2, w1, sh) : w1;
                v.z = sh ? __builtin_amdgcn_alignbyte(w3, w2, sh) : w2;
                v.w = sh ? __builtin_amdgcn_alignbyte(w4, w3, sh) : w3;
                *reinterpret_cast<uint4*>(&out32[gw0 + k]) = v;   // never word 0 or the last word
            } else {
#pragma unroll
                for (uint32_t i = 0; i < 4; i++) out32[gw0 + k + i] = gen_word(k + i);
            }
        }
        // the words outside the quads: [0, ks) and [ks + 4 nq, nwords)
        const uint32_t kq = nq ? ks + 4 * nq : 0;
        const uint32_t nrest = nq ? ks + (nwords - kq) : nwords;
        for (uint32_t r = tid; r < nrest; r += PT) {
            const uint32_t k = nq ? (r < ks ? r : kq + (r - ks)) : r;
            put_word(k, gen_word(k));
        }
        if (tid == 0 && (b == 0 || b == nblk - 1)) pack_framing(out32, flags, nblk, b, res);
        return;
    }
    // coded blocks: the bits go through an 8 KB LDS ring (PK_RING words) that is flushed to
    // the stream before every header and every round of PT x TPT tokens (<= 1 536 words per
    // round, <= 160 header words), so the LDS per workgroup is ~10 KB instead of one 33 KB
    // buffer for the whole block (4 per CU).  `base` = block word held in stage[0];
    // ring positions are block bit positions minus 32 * base.
    const uint64_t gw0 = O >> 5;
    const bool first_partial = s0 != 0;
    const bool last_partial = ((s0 + Lb) & 31) != 0;
    uint32_t base = 0;
    auto out_word = [&](uint32_t k, uint32_t v) {   // block word k (shared edge words: atomicOr)
        if ((k == 0 && first_partial) || (k == nwords - 1 && last_partial)) atomicOr(&out32[gw0 + k], v);
        else out32[gw0 + k] = v;
    };
    // write the ring's complete words below block bit `pos`; the partial word moves to stage[0]
    auto flush = [&](uint32_t pos) {
        lds_barrier();
        const uint32_t done = (pos >> 5) - base;
        for (uint32_t k = tid; k < done; k += PT) out_word(base + k, stage[k]);
        const uint32_t part = stage[done];
        lds_barrier();
        for (uint32_t k = tid; k <= done; k += PT) stage[k] = k == 0 ? part : 0u;
        base += done;
        lds_barrier();
    };
    const uint32_t* tb = tok_g + (uint64_t)b * DMX_BLK;
    // the first round's tokens, loaded before anything else (each round prefetches the next):
    // the rounds of a block no longer wait on a global load each
    uint32_t nxt[TPT];
    const uint32_t si0_t0 = bi.nsub > 1 ? sub_g[(uint64_t)b * DMX_NSUB].t0 : 0u;
#pragma unroll
    for (int t = 0; t < TPT; t++) nxt[t] = tb[min(si0_t0 + tid * TPT + (uint32_t)t, (uint32_t)DMX_BLK - 1)];
    for (uint32_t k = tid; k < PK_RING; k += PT) stage[k] = 0;
    for (uint32_t k = tid; k < 316; k += PT) code[k] = codes_g[(uint64_t)b * DMX_NSUB * DMX_HIST + k];
    __syncthreads();
#ifndef DMX_PACK_OLD
    auto build_ptab = [&]() {   // (after code[] is complete; a barrier follows)
        for (uint32_t k = tid; k < 512; k += PT) {
            uint32_t e;
            if (k < 256) {
                const uint32_t cw = code[k];
                e = (cw & 0xFFFFu) | ((cw >> 16) << 24);
            } else {
                uint32_t sy, eb, ev;
                len_sym(k - 253, sy, eb, ev);   // length k - 256 + 3
                const uint32_t cw = code[sy];
                e = ((cw & 0xFFFFu) | (ev << (cw >> 16))) | (((cw >> 16) + eb) << 24);
            }
            ptab[k] = e;
        }
    };
    build_ptab();
    __syncthreads();
#endif
    {   // (stored blocks left above)
        // one or more DEFLATE blocks (f3 split): header, tokens [t0, t1), end of block
        uint32_t pos = s0;   // block bit position
        for (uint32_t sb = 0; sb < bi.nsub; sb++) {
            const uint64_t slot = (uint64_t)b * DMX_NSUB + sb;
            const dmx_subinfo si = sub_g[slot];
            if (sb) {   // this block's codes (every thread is done with the previous ones)
                __syncthreads();
                for (uint32_t k = tid; k < 316; k += PT) code[k] = codes_g[slot * DMX_HIST + k];
#pragma unroll
                for (int t = 0; t < TPT; t++) nxt[t] = tb[min(si.t0 + tid * TPT + (uint32_t)t, (uint32_t)DMX_BLK - 1)];
                __syncthreads();
#ifndef DMX_PACK_OLD
                build_ptab();
                __syncthreads();
#endif
            }
            flush(pos);
            const uint32_t* hg = hdr_g + slot * DMX_HDR_WORDS;
            const uint32_t hb = si.hdr_bits;
            for (uint32_t k = tid; k < (hb + 31) / 32; k += PT) {
                const uint32_t nb = (hb - 32 * k) < 32 ? (hb - 32 * k) : 32;
                st_or64(stage, pos - 32 * base + 32 * k, hg[k], nb);
            }
            pos += hb;
            // tokens: TPT consecutive tokens per thread; a per-thread bit accumulator flushes
            // whole words into the zeroed ring, every one by atomicOr (the first and last are
            // shared with the neighbours; one unconditional ds_or instead of a nested branch
            // per piece: 0.0855 vs 0.087 ms at TPT 8, 0.080 at TPT 4, profiles/r04_pk)
            for (uint32_t c = si.t0; c < si.t1; c += PT * TPT) {
                flush(pos);
                const uint32_t j0 = c + tid * TPT;
                uint32_t cur[TPT];
    #pragma unroll
                for (int t = 0; t < TPT; t++) cur[t] = nxt[t];
                if (c + PT * TPT < si.t1) {   // the next round's tokens, in flight during this one
    #pragma unroll
                    for (int t = 0; t < TPT; t++) nxt[t] = tb[min(j0 + PT * TPT + (uint32_t)t, (uint32_t)DMX_BLK - 1)];
                }
                uint32_t pv[2 * TPT], pb[2 * TPT];   // up to two pieces per token, <= 28 bits each
                uint32_t mybits = 0;
    #pragma unroll
                for (int t = 0; t < TPT; t++) {
#ifndef DMX_PACK_OLD
                    {   // both pieces without a branch: the first from ptab, the distance's computed
                        // for every token and dropped for a literal; slots past the sub-block's
                        // last token (the last round) get no bits
                        const uint32_t tk = cur[t];
                        const bool ok = j0 + t < si.t1, lit = (tk >> 9) == 0;
                        const uint32_t e1 = ptab[lit ? tk : min(253u + (tk & 0x1FFu), 511u)];
                        // RFC 1951 3.2.5 distance symbol of x = distance - 1 without a branch:
                        // e = floor(log2(x | 2)), the symbol 2e + the bit below the top one
                        // (x < 2: the symbol is x; both have no extra bits)
                        const uint32_t x = lit ? 0u : (tk >> 9) - 1u;
                        const uint32_t e = 31u - __clz(x | 2u), eb = e - 1u;
                        const uint32_t sy = min(x < 2u ? x : 2u * e + ((x >> eb) & 1u), 29u);
                        const uint32_t cw = code[DMX_DIST0 + sy];
                        const bool dd = ok && !lit;
                        pv[2 * t] = ok ? (e1 & 0xFFFFFFu) : 0u;
                        pb[2 * t] = ok ? e1 >> 24 : 0u;
                        pv[2 * t + 1] = dd ? (cw & 0xFFFFu) | ((x & ((1u << eb) - 1u)) << (cw >> 16)) : 0u;
                        pb[2 * t + 1] = dd ? (cw >> 16) + eb : 0u;
                        mybits += pb[2 * t] + pb[2 * t + 1];
                    }
#else
                    pv[2 * t] = pb[2 * t] = pv[2 * t + 1] = pb[2 * t + 1] = 0;
                    if (j0 + t < si.t1) {
                        const uint32_t tk = cur[t];
                        if ((tk >> 9) == 0) {
                            const uint32_t cw = code[tk];
                            pv[2 * t] = cw & 0xFFFFu;
                            pb[2 * t] = cw >> 16;
                        } else {
                            uint32_t sy, eb, ev;
                            len_sym(tk & 0x1FFu, sy, eb, ev);
                            uint32_t cw = code[sy];
                            pv[2 * t] = (cw & 0xFFFFu) | (ev << (cw >> 16));
                            pb[2 * t] = (cw >> 16) + eb;
                            dist_sym(tk >> 9, sy, eb, ev);
                            cw = code[DMX_DIST0 + sy];
                            pv[2 * t + 1] = (cw & 0xFFFFu) | (ev << (cw >> 16));
                            pb[2 * t + 1] = (cw >> 16) + eb;
                        }
                        mybits += pb[2 * t] + pb[2 * t + 1];
                    }
#endif
                }
                // exclusive scan of the threads' bit counts over the workgroup
                const uint32_t incl = wave_incl_scan(mybits);
                if (lane == 63) wsum[wave] = incl;
                lds_barrier();
                uint32_t wbase = 0, tot = 0;
    #pragma unroll
                for (int w = 0; w < PT / 64; w++) {
                    const uint32_t t = wsum[w];
                    if ((uint32_t)w < wave) wbase += t;
                    tot += t;
                }
                if (mybits) {
                    const uint32_t p0 = pos - 32 * base + wbase + incl - mybits;
                    uint32_t w = p0 >> 5, ab = p0 & 31;
                    uint64_t acc = 0;
    #pragma unroll
                    for (int q = 0; q < 2 * TPT; q++) {
                        acc |= (uint64_t)pv[q] << ab;
                        ab += pb[q];
                        if (ab >= 32) {
                            atomicOr(&stage[w], (uint32_t)acc);
                            acc >>= 32;
                            ab -= 32;
                            w++;
                        }
                    }
                    if (ab) atomicOr(&stage[w], (uint32_t)acc);   // shared with the next thread
                }
                pos += tot;
                lds_barrier();
            }
            const uint32_t cw = code[256];
            if (tid == 0) st_or64(stage, pos - 32 * base, cw & 0xFFFFu, cw >> 16);
            pos += cw >> 16;
        }
    }
    __syncthreads();
    for (uint32_t k = tid; base + k < nwords; k += PT) out_word(base + k, stage[k]);
    if (tid == 0 && (b == 0 || b == nblk - 1)) pack_framing(out32, flags, nblk, b, res);
}

// K4: one workgroup per block (wl == nullptr), or a grid that strides over the apply
// launch's list L4 (DMX_F_STORE_CHECK: every block but the whole-copy prefix).
__global__ __launch_bounds__(PT) void dmx_pack_kernel(const uint8_t* __restrict__ in, uint32_t sw,
                                                      const uint32_t* __restrict__ tok_g, const uint32_t* __restrict__ codes_g,
                                                      const uint32_t* __restrict__ hdr_g, const dmx_blkinfo* __restrict__ info,
                                                      const dmx_subinfo* __restrict__ sub_g,
                                                      uint32_t nblk, uint32_t flags, uint32_t* __restrict__ out32,
                                                      dmx_result* __restrict__ res,
                                                      const uint32_t* __restrict__ wl, const uint32_t* __restrict__ L4,
                                                      const uint16_t* __restrict__ codes) {
    if (!L4) {   // a workgroup per block; with work lists, the whole-copy prefix returns at once
        if (wl && wl_skip(blockIdx.x, wl[WL_M], nblk)) return;
        if (is_dup(codes, blockIdx.x)) return;   // dmx_dup_copy_kernel's
        pack_one(blockIdx.x, in, sw, tok_g, codes_g, hdr_g, info, sub_g, nblk, flags, out32, res);
        if (wl && blockIdx.x == 0 && threadIdx.x == 0) wl_hint_put(wl, 3, wl[WL_N4]);
        return;
    }
    const uint32_t cnt = wl[WL_N4];
    if (blockIdx.x == 0 && threadIdx.x == 0) wl_hint_put(wl, 3, cnt);
    for (uint32_t i = blockIdx.x; i < cnt; i += gridDim.x) {
        __syncthreads();   // the previous block's LDS reads are done
        pack_one(L4[i], in, sw, tok_g, codes_g, hdr_g, info, sub_g, nblk, flags, out32, res);
    }
}

// ------------------------------------------------------------------------------------
// host side of the HIP layer (C ABI)
// ------------------------------------------------------------------------------------

#include "dmx_ctx.h"


// ---- fault injection (tests): DMX_FAULT="malloc:N" makes the N-th device / pinned allocation
// from now fail, "launch:N" the N-th encode launch check; dmx_fault_set() sets it at run time.
// Every error path must then return -E_* and leave nothing allocated that the context does
// not own (global_errors.h:60-81 is the reference's checkpoint mechanism).
#include <pthread.h>
static pthread_mutex_t g_fault_mu = PTHREAD_MUTEX_INITIALIZER;
static int g_fault_kind = 0;   // 1 = allocation, 2 = launch
static long g_fault_left = 0;
extern "C" int dmx_fault_set(const char* spec) {
    int kind = 0;
    long n = 0;
    if (spec && *spec) {
        if (!strncmp(spec, "malloc:", 7)) { kind = 1; n = atol(spec + 7); }
        else if (!strncmp(spec, "launch:", 7)) { kind = 2; n = atol(spec + 7); }
        else return -(int)E_INVAL;
        if (n <= 0) return -(int)E_RANGE;
    }
    pthread_mutex_lock(&g_fault_mu);
    g_fault_left = n;
    __atomic_store_n(&g_fault_kind, kind, __ATOMIC_RELEASE);
    pthread_mutex_unlock(&g_fault_mu);
    return 0;
}
__attribute__((constructor)) static void dmx_fault_env(void) { (void)dmx_fault_set(getenv("DMX_FAULT")); }
bool fault_hit(int kind) {
    // several host threads allocate and launch at once (dmx_encode_fd_multi): the unlocked
    // fast-path read is atomic, the update under the lock
    if (!__atomic_load_n(&g_fault_kind, __ATOMIC_ACQUIRE)) return false;
    pthread_mutex_lock(&g_fault_mu);
    bool hit = false;
    if (g_fault_kind == kind && g_fault_left > 0 && --g_fault_left == 0) {
        hit = true;
        __atomic_store_n(&g_fault_kind, 0, __ATOMIC_RELEASE);
    }
    pthread_mutex_unlock(&g_fault_mu);
    return hit;
}
hipError_t dmx_malloc(void** p, size_t n) {
    if (fault_hit(1)) { *p = NULL; return hipErrorOutOfMemory; }
    return hipMalloc(p, n);
}
hipError_t dmx_host_malloc(void** p, size_t n) {
    if (fault_hit(1)) { *p = NULL; return hipErrorOutOfMemory; }
    return hipHostMalloc(p, n, 0);
}

int hip_fail(hipError_t e, const char* what) {
    if (e != hipSuccess) {
        fprintf(stderr, "dmx: %s failed: %s\n", what, hipGetErrorString(e));
        return 1;
    }
    return 0;
}

extern "C" uint64_t dmx_max_compressed(uint64_t n, int32_t sw) {
    if (sw <= 0 || sw > DMX_BLK) sw = DMX_BLK;
    const uint64_t nblk = (n + (uint64_t)sw - 1) / (uint64_t)sw;
    return ((n + 5 * nblk + 2 + 4 + 5 + 16) + 3) & ~3ull;
}

static void ctx_free_ws(dmx_ctx* c) {
    if (c->dist) (void)hipFree(c->dist);
    if (c->tok) (void)hipFree(c->tok);
    if (c->hist) (void)hipFree(c->hist);
    if (c->codes) (void)hipFree(c->codes);
    if (c->hdr) (void)hipFree(c->hdr);
    if (c->sub) (void)hipFree(c->sub);
    if (c->info) (void)hipFree(c->info);
    if (c->tiles) (void)hipFree(c->tiles);
    if (c->wl) (void)hipFree(c->wl);
    c->dist = NULL; c->tok = NULL; c->hist = NULL; c->codes = NULL; c->hdr = NULL; c->sub = NULL; c->info = NULL;
    c->tiles = NULL;
    c->wl = NULL;
    c->cap_blocks = 0;
}

// Scratch of the block options, sized to the block capacity: split plans (DMX_F_SPLIT), the
// exported chains of every block + the dict (DMX_F_DICT), and the diagnostic stamps.
static int ctx_reserve_scratch(dmx_ctx* c) {
    const uint64_t cb = c->cap_blocks;
    if ((c->want & DMX_F_SPLIT) && c->cap_split < cb) {
        if (c->split) (void)hipFree(c->split);
        c->split = NULL;
        c->cap_split = 0;
        HIPCHK(dmx_malloc(&c->split, cb * sizeof(SplitScratch)));
        c->cap_split = cb;
    }
    if ((c->want & DMX_F_DICT) && c->cap_chain < cb + 1) {
        if (c->chs) (void)hipFree(c->chs);
        if (c->che) (void)hipFree(c->che);
        c->chs = NULL;
        c->che = NULL;
        c->cap_chain = 0;
        HIPCHK(dmx_malloc(&c->chs, (cb + 1) * DMX_BLK * sizeof(uint16_t)));
        HIPCHK(dmx_malloc(&c->che, (cb + 1) * DMX_NBUCKET * sizeof(uint16_t)));
        c->cap_chain = cb + 1;
    }
    if (getenv("DMX_STAMPS") && c->dbg_cap < cb) {
        if (c->dbg) (void)hipFree(c->dbg);
        c->dbg = NULL;
        c->dbg_cap = 0;
        HIPCHK(dmx_malloc(&c->dbg, cb * DMX_STAMPS * sizeof(uint64_t)));
        c->dbg_cap = cb;
    }
    return 0;
}

static int ctx_reserve(dmx_ctx* c, uint64_t nblk) {
    if (nblk <= c->cap_blocks) return ctx_reserve_scratch(c);
    ctx_free_ws(c);
    const uint64_t cb = nblk < 1 ? 1 : nblk;
    HIPCHK(dmx_malloc(&c->dist, cb * DMX_BLK * sizeof(uint16_t)));
    HIPCHK(dmx_malloc(&c->tok, cb * DMX_BLK * sizeof(uint32_t)));
    HIPCHK(dmx_malloc(&c->hist, cb * DMX_HIST * sizeof(uint32_t)));
    HIPCHK(dmx_malloc(&c->codes, cb * DMX_NSUB * DMX_HIST * sizeof(uint32_t)));
    HIPCHK(dmx_malloc(&c->hdr, cb * DMX_NSUB * DMX_HDR_WORDS * sizeof(uint32_t)));
    HIPCHK(dmx_malloc(&c->sub, cb * DMX_NSUB * sizeof(dmx_subinfo)));
    HIPCHK(dmx_malloc(&c->info, cb * sizeof(dmx_blkinfo)));
    HIPCHK(dmx_malloc(&c->tiles, (cb / SCAN_TILE + 1) * sizeof(ScanTile)));
    HIPCHK(dmx_malloc(&c->wl, (WL_HDR + 5 * cb + 4 + (cb + 16) / 2) * sizeof(uint32_t)));
    {   // the hint's device address in the list header
        uint64_t hp = 0;
        void* dp = NULL;
        if (c->whint && hipHostGetDevicePointer(&dp, (void*)c->whint, 0) == hipSuccess) hp = (uint64_t)(uintptr_t)dp;
        const uint32_t hw[2] = {(uint32_t)hp, (uint32_t)(hp >> 32)};
        HIPCHK(hipMemcpy(c->wl + WL_HINT, hw, sizeof(hw), hipMemcpyHostToDevice));
    }
    c->cap_blocks = cb;
    return ctx_reserve_scratch(c);
}

extern "C" int dmx_ctx_create(int device, uint64_t max_input, dmx_ctx** out) {
    *out = NULL;
    int ndev = 0;
    if (hipGetDeviceCount(&ndev) != hipSuccess || ndev <= 0) {
        fprintf(stderr, "dmx: no HIP device available (the encoder has no CPU fallback)\n");
        return -(int)E_NEXIST;
    }
    if (device < 0 || device >= ndev) return -(int)E_RANGE;
    HIPCHK(hipSetDevice(device));
    dmx_ctx* c = (dmx_ctx*)calloc(1, sizeof(dmx_ctx));
    if (!c) return -(int)E_MALLOC;
    c->device = device;
    {   // the test hooks' defaults: the environment, once per context (never per encode)
        const char* e = getenv("DMX_WORKLIST");
        c->hk_wl = !e ? -1 : !strcmp(e, "0") ? 0 : !strcmp(e, "list") ? 1 : !strcmp(e, "plain") ? 2 : -1;
        const char* dd = getenv("DMX_DEDUPE");
        c->hk_dedupe = dd ? (atoi(dd) > 0 ? 1 : 0) : -1;
        const char* s3 = getenv("DMX_SCAN3");
        c->hk_scan3 = s3 && !strcmp(s3, "1");
    }
    int ncu = 0;
    c->ncu = hipDeviceGetAttribute(&ncu, hipDeviceAttributeMultiprocessorCount, device) == hipSuccess && ncu > 0
                 ? (uint32_t)ncu : 256u;
    {   // the launch-shape hint (WL_HINT): zero = no encode yet; without it every shape is per block
        void* hp = NULL;
        if (hipHostMalloc(&hp, 32, hipHostMallocMapped | hipHostMallocCoherent) == hipSuccess) {
            memset(hp, 0, 32);
            c->whint = (volatile uint32_t*)hp;
            void* dp = NULL;
            if (hipHostGetDevicePointer(&dp, hp, 0) == hipSuccess) c->whint_dev = (uint32_t*)dp;
        }
    }
    if (hip_fail(hipStreamCreateWithFlags(&c->stream, hipStreamNonBlocking), "hipStreamCreate")) { c->stream = NULL; dmx_ctx_destroy(c); return -(int)E_DEVICE; }
    if (hip_fail(dmx_malloc(&c->res, sizeof(dmx_result)), "hipMalloc(res)")) { dmx_ctx_destroy(c); return -(int)E_DEVICE; }
    if (hip_fail(dmx_malloc(&c->nfb, 16), "hipMalloc(nfb)") || hip_fail(hipMemset(c->nfb, 0, 16), "hipMemset(nfb)")) {
        dmx_ctx_destroy(c);
        return -(int)E_DEVICE;
    }
    for (int j = 0; j < DMX_EV_RING; j++)
        for (int k = 0; k < 6; k++) (void)hipEventCreate(&c->ev[j][k]);
    const uint64_t nb = (max_input + DMX_BLK - 1) / DMX_BLK;
    const int r = ctx_reserve(c, nb);
    if (r) { dmx_ctx_destroy(c); return r; }
    *out = c;
    return 0;
}

extern "C" int dmx_ctx_reserve_flags(dmx_ctx* c, uint64_t n, int32_t sw, uint32_t flags) {
    if (!c) return -(int)E_INVAL;
    if (sw == 0) sw = DMX_BLK;
    if (sw < 1 || sw > DMX_BLK) return -(int)E_RANGE;
    const uint64_t nblk = (n + (uint64_t)sw - 1) / (uint64_t)sw;
    const uint32_t want = c->want | (flags & (DMX_F_SPLIT | DMX_F_DICT));
    const bool stamps = getenv("DMX_STAMPS") != NULL;
    const uint64_t cb = nblk > c->cap_blocks ? nblk : c->cap_blocks;
    if (nblk <= c->cap_blocks && want == c->want && (!(want & DMX_F_SPLIT) || c->cap_split >= cb) &&
        (!(want & DMX_F_DICT) || c->cap_chain >= cb + 1) && (!stamps || c->dbg_cap >= cb))
        return 0;   // nothing to do: no synchronisation
    HIPCHK(hipSetDevice(c->device));
    HIPCHK(hipStreamSynchronize(c->stream));
    HIPCHK(hipDeviceSynchronize());
    c->want = want;
    return ctx_reserve(c, nblk);
}

extern "C" int dmx_ctx_reserve(dmx_ctx* c, uint64_t n, int32_t sw) { return dmx_ctx_reserve_flags(c, n, sw, 0); }

extern "C" void dmx_ctx_destroy(dmx_ctx* c) {
    if (!c) return;
    (void)hipSetDevice(c->device);
    (void)hipStreamSynchronize(c->stream);
    ctx_free_ws(c);
    if (c->res) (void)hipFree(c->res);
    if (c->nfb) (void)hipFree(c->nfb);
    if (c->dbg) (void)hipFree(c->dbg);
    if (c->d_in) (void)hipFree(c->d_in);
    if (c->d_out) (void)hipFree(c->d_out);
    if (c->d_dict) (void)hipFree(c->d_dict);
    for (int k = 0; k < 2; k++) {
        if (c->fd_hin[k]) (void)hipHostFree(c->fd_hin[k]);
        if (c->fd_hout[k]) (void)hipHostFree(c->fd_hout[k]);
        if (c->fd_din[k]) (void)hipFree(c->fd_din[k]);
    }
    for (int k = 0; k < 2; k++) {
        if (c->fd_dout[k]) (void)hipFree(c->fd_dout[k]);
        if (c->fd_hres[k]) (void)hipHostFree(c->fd_hres[k]);
        if (c->fd_ev[k]) (void)hipEventDestroy(c->fd_ev[k]);
    }
    if (c->fd_cs) (void)hipStreamDestroy(c->fd_cs);
    fdp_free(c->fdp);
    if (c->whint) (void)hipHostFree((void*)c->whint);
    if (c->chs) (void)hipFree(c->chs);
    if (c->che) (void)hipFree(c->che);
    if (c->split) (void)hipFree(c->split);
    for (int j = 0; j < DMX_EV_RING; j++)
        for (int k = 0; k < 6; k++) if (c->ev[j][k]) (void)hipEventDestroy(c->ev[j][k]);
    if (c->stream) (void)hipStreamDestroy(c->stream);
    free(c);
}

// stage times per encode: [chain, match, huff, scan, pack] + the whole encode
static void ctx_collect_set(dmx_ctx* c, int j) {
    if (!c->ev_used[j]) return;
    c->ev_used[j] = 0;
    const int m = c->timing;
    int last = 5;
    while (last > 0 && !((m >> last) & 1)) last--;
    if (hipEventSynchronize(c->ev[j][last]) != hipSuccess) return;
    for (int k = 0; k < 5; k++) {
        float ms = 0.f;
        if (((m >> k) & 3) == 3 && hipEventElapsedTime(&ms, c->ev[j][k], c->ev[j][k + 1]) == hipSuccess) c->stage_ms[k] += ms;
    }
    float tot = 0.f;
    if ((m & 0x21) == 0x21 && hipEventElapsedTime(&tot, c->ev[j][0], c->ev[j][5]) == hipSuccess) c->stage_ms[5] += tot;
    c->stage_n++;
}

// Launch shapes of the work-list mode: the persistent K1 over L1, K2 over L2, K4 over L4 when
// the context's previous encode (WL_HINT) listed fewer than half of its blocks there, else a
// workgroup per block.  DMX_WORKLIST=list / plain forces one shape (tests), =0 turns the
// work lists off (one workgroup per block, no list builder, no whole copies in K0).
struct WlShape { bool loop1, list2, list4, dedupe; uint32_t n2, n4; };
// a list kernel's grid: the previous encode's list length (a guess: the kernels stride over
// the list whatever its length), within [lo, hi] and at most nblk
static uint32_t list_grid(uint32_t nblk, uint32_t prev, uint32_t lo, uint32_t hi) {
    uint32_t g = prev < lo ? lo : (prev > hi ? hi : prev);
    return g < nblk ? g : nblk;
}
static WlShape wl_shape(const dmx_ctx* c) {
    WlShape w = {false, false, false, false, ~0u, ~0u};
    if (c->hk_wl == 1) w = WlShape{true, true, true, false, ~0u, ~0u};
    else if (c->hk_wl != 2 && c->whint && c->whint[0]) {
        const uint32_t nb = c->whint[0];
        w.n2 = c->whint[2];   // the list grids are sized by the previous encode's lists
        w.n4 = c->whint[3];
        w.loop1 = 2 * c->whint[1] < nb;
        w.list2 = 2 * c->whint[2] < nb;
        w.list4 = 2 * c->whint[3] < nb;
        w.dedupe = 4 * c->whint[4] >= nb;   // a quarter of the blocks were full uniform blocks
    }
    if (c->hk_dedupe >= 0) w.dedupe = c->hk_dedupe > 0;
    return w;
}

extern "C" int dmx_ctx_set_hook(dmx_ctx* c, int hook, int value) {
    if (!c) return -(int)E_INVAL;
    switch (hook) {
        case DMX_HOOK_WORKLIST:
            if (value < -1 || value > 2) return -(int)E_RANGE;
            c->hk_wl = value;
            return 0;
        case DMX_HOOK_DEDUPE:
            if (value < -1 || value > 1) return -(int)E_RANGE;
            c->hk_dedupe = value;
            return 0;
        case DMX_HOOK_SCAN3:
            if (value < 0 || value > 1) return -(int)E_RANGE;
            c->hk_scan3 = value;
            return 0;
        default:
            return -(int)E_INVAL;
    }
}

extern "C" int dmx_encode_async(dmx_ctx* c, const void* d_in, uint64_t n, void* d_out, uint64_t out_cap,
                                const dmx_opts* opts, void* stream) {
    if (!c || !d_out || (!d_in && n)) return -(int)E_INVAL;
    dmx_opts o = {0, 0, DMX_ZLIB, 0, NULL, 0};
    if (opts) o = *opts;
    if (o.sw == 0) o.sw = DMX_BLK;
    if (o.sw < 1 || o.sw > DMX_BLK) return -(int)E_RANGE;
    if (o.max_chain < 0) return -(int)E_RANGE;
    if (o.deep_chain < 0 || o.deep_chain > 255) return -(int)E_RANGE;
    if ((reinterpret_cast<uintptr_t>(d_out) & 3) != 0) return -(int)E_INVAL;
    uint32_t dict_len = 0;   // DMX_F_DICT: history of block 0 (the last sw bytes are used)
    if ((o.flags & DMX_F_DICT) && o.dict && o.dict_len) {
        dict_len = o.dict_len < (uint64_t)o.sw ? (uint32_t)o.dict_len : (uint32_t)o.sw;
        o.dict = (const uint8_t*)o.dict + (o.dict_len - dict_len);
    }
    const uint64_t nblk64 = (n + (uint64_t)o.sw - 1) / (uint64_t)o.sw;
    if (nblk64 > c->cap_blocks || nblk64 > 0x7FFFFFFFull) return -(int)E_SZ;
    const uint32_t nblk = (uint32_t)nblk64;
    HIPCHK(hipSetDevice(c->device));
    // no allocation here (graph-capturable, no device-wide sync): the split / dictionary
    // scratch comes from dmx_ctx_reserve_flags
    if ((o.flags & DMX_F_SPLIT) && c->cap_split < nblk) return -(int)E_SZ;
    if ((o.flags & DMX_F_DICT) && c->cap_chain < (uint64_t)nblk + 1) return -(int)E_SZ;
    hipStream_t s = stream ? (hipStream_t)stream : c->stream;
    // DMX_F_STORE_CHECK: the work lists (WL_* above) and their launch shapes (wl_shape)
    const WlShape wsh = wl_shape(c);
    // an encode whose shapes are all per block and without the dedupe runs without the lists
    // (no list builder, no fill kernel); its scan kernel writes the hint instead
    const bool anyl = wsh.loop1 || wsh.list2 || wsh.list4 || wsh.dedupe;
    uint32_t* wl = ((o.flags & DMX_F_STORE_CHECK) && anyl && c->hk_wl != 0) ? c->wl : NULL;
    // the uniform-block dedupe's rep index per block (NULL: no dedupe in this encode)
    const bool dedupe = wl && wsh.dedupe && !(o.flags & DMX_F_SPLIT);
    const uint16_t* dupk = dedupe ? wl_codes((const uint32_t*)wl, c->cap_blocks) : NULL;   // dup bits (bit 3)
    const uint32_t* dupa = dedupe ? wl_dup(wl, c->cap_blocks) : NULL;                      // their representatives
    hipEvent_t* ev = NULL;
    if (c->timing && (c->ev_every <= 1 || c->ev_count++ % c->ev_every == 0)) {
        const int j = (int)(c->ev_next++ % DMX_EV_RING);
        ctx_collect_set(c, j);
        ev = c->ev[j];
        c->ev_used[j] = 1;
        if (c->timing & 1) (void)hipEventRecord(ev[0], s);
    }
    if (nblk) {
        // diagnostic phase stamps (DMX_STAMPS=1 when the context was reserved)
        uint64_t* dbg = c->dbg_cap >= nblk ? c->dbg : NULL;
        // stage 0 "dict" (DMX_F_DICT only): the chain kernel (every block's sorted chains, and
        // the dict's) and the history search; otherwise the match kernel sorts its own block
        if (o.flags & DMX_F_DICT) {
            hipLaunchKernelGGL(dmx_chain_kernel, dim3(nblk + 1), dim3(MT), 0, s, (const uint8_t*)d_in, n,
                               (uint32_t)o.sw, (const uint8_t*)o.dict, dict_len, c->chs, c->che, c->nfb);
            hipLaunchKernelGGL((o.max_chain >= 1 && o.max_chain <= 6) ? dmx_hist_kernel_t<6>
                               : o.max_chain == 7 ? dmx_hist_kernel_t<7> : dmx_hist_kernel_t<8>,
                               dim3(nblk), dim3(MT), 0, s, (const uint8_t*)d_in, n, (uint32_t)o.sw,
                               o.max_chain, (const uint8_t*)o.dict, dict_len, c->chs, c->che, c->tok, dbg);
        }
        // stage 0 also holds K0, the noise check (DMX_F_STORE_CHECK)
        if (o.flags & DMX_F_STORE_CHECK)
            hipLaunchKernelGGL(wl && wsh.loop1 ? dmx_store_check_kernel<true> : dmx_store_check_kernel<false>, dim3(nblk),
                               dim3(SCT), 0, s, (const uint8_t*)d_in, n,
                               (uint32_t)o.sw, c->info, c->tok, c->hist, (o.flags & DMX_F_DICT) ? 0u : 1u, o.flags,
                               (uint32_t*)d_out, out_cap, wl ? wl_codes(wl, c->cap_blocks) : NULL);
        if (ev && ((c->timing >> 1) & 1)) (void)hipEventRecord(ev[1], s);   // (the list builder counts to "match")
        if (wl) {
            hipLaunchKernelGGL(dmx_worklist_kernel, dim3((nblk + WLC * WLT - 1) / (WLC * WLT)), dim3(WLT), 0, s, nblk, wl,
                               (uint64_t)c->cap_blocks,
                               dupa ? 1u : 0u);
        }
#ifdef DMX_DEBUG_STOP   // diagnostic library variants only (tools/build_var.sh NAME -DDMX_DEBUG_STOP=1|2|3, dbg_stop)
        const uint32_t dstop = (uint32_t)(DMX_DEBUG_STOP) & 3u;
#else
        const uint32_t dstop = 0;
#endif
        const uint32_t mfl = ((o.flags & DMX_F_LAZY) ? 1u : 0u) | ((o.flags & DMX_F_EXACT_SORT) ? 2u : 0u) |
                             ((o.flags & DMX_F_STORE_CHECK) ? 4u : 0u) | ((o.flags & DMX_F_DEEP) ? 8u : 0u) | (dstop << 8) |
                             ((uint32_t)o.deep_chain << 16);   // DMX_F_DEEP depth (0 = DMX_DEEP_CHAIN)
        // work lists: the persistent K1 over L1 when the previous encode left most blocks
        // stored (wl_shape), else a workgroup per block
        const bool loop1 = wl && wsh.loop1;
        const dim3 g1(loop1 ? (nblk < c->ncu ? nblk : c->ncu) : nblk);
        const MatchArgs ma = {(const uint8_t*)d_in, n, (uint32_t)o.sw, o.max_chain, mfl, c->dist, c->chs, c->tok,
                              c->hist, c->info, dbg, c->nfb, loop1 ? wl : NULL};
        if (o.flags & DMX_F_DICT) {
            if (loop1) hipLaunchKernelGGL((dmx_match_kernel<true, 3, true>), g1, dim3(MT), 0, s, ma);
            else hipLaunchKernelGGL((dmx_match_kernel<true, 3, false>), g1, dim3(MT), 0, s, ma);
        } else if (o.max_chain == 0) {
            if (loop1) hipLaunchKernelGGL((dmx_match_kernel<false, DMX_NBX, true>), g1, dim3(MT), 0, s, ma);
            else hipLaunchKernelGGL((dmx_match_kernel<false, DMX_NBX, false>), g1, dim3(MT), 0, s, ma);
        } else {
            if (loop1) hipLaunchKernelGGL((dmx_match_kernel<false, 3, true>), g1, dim3(MT), 0, s, ma);
            else hipLaunchKernelGGL((dmx_match_kernel<false, 3, false>), g1, dim3(MT), 0, s, ma);
        }
        if (ev && ((c->timing >> 2) & 1)) (void)hipEventRecord(ev[2], s);
        if (o.flags & DMX_F_SPLIT)
            {
                hipLaunchKernelGGL(dmx_split_hist_kernel, dim3(nblk), dim3(SHT), 0, s, c->tok, c->info,
                                   (SplitScratch*)c->split);
                hipLaunchKernelGGL(dmx_split_plan_kernel, dim3(nblk * SPW), dim3(64), 0, s, (SplitScratch*)c->split,
                                   c->info, nblk, o.flags);
                hipLaunchKernelGGL(dmx_split_choose_kernel, dim3(nblk), dim3(64), 0, s, (const SplitScratch*)c->split,
                                   c->info, c->codes, c->hdr, c->sub, nblk, o.flags);
            }
        else
            hipLaunchKernelGGL(dmx_huff_kernel, dim3(wl && wsh.list2 ? list_grid(nblk, wsh.n2, 2 * c->ncu, 32 * c->ncu) : nblk),
                               dim3(64), 0, s, c->hist, c->info, c->codes, c->hdr, c->sub, nblk, o.flags,
                               wl && wsh.list2 ? wl : NULL, wl && wsh.list2 ? wl + WL_HDR + c->cap_blocks : NULL, dupk);
        if (ev && ((c->timing >> 3) & 1)) (void)hipEventRecord(ev[3], s);
    } else if (ev) {
        for (int k = 1; k <= 3; k++)
            if ((c->timing >> k) & 1) (void)hipEventRecord(ev[k], s);
    }
    const uint32_t ntile = (nblk + SCAN_TILE - 1) / SCAN_TILE;
    if (nblk)
        hipLaunchKernelGGL(dmx_scan_tile_kernel, dim3(ntile), dim3(SCAN_TILE), 0, s, c->info, nblk, n, (uint32_t)o.sw,
                           c->tiles, dupk, dupa, c->sub);
    uint32_t* L4 = wl ? wl + WL_HDR + 2 * c->cap_blocks : NULL;
    uint32_t* hintp = (!wl && (o.flags & DMX_F_STORE_CHECK)) ? c->whint_dev : NULL;
    if (nblk && ntile <= SA1_MAXT && !c->hk_scan3) {   // (hk_scan3: the three-launch scan at any size, tests)
        hipLaunchKernelGGL(dmx_scan_apply1_kernel, dim3(ntile), dim3(SCAN_TILE), 0, s, c->info, nblk, n, o.flags, out_cap,
                           (uint32_t)o.sw, (const ScanTile*)c->tiles, (uint32_t*)d_out, c->res, c->nfb, hintp, wl, L4, dupk);
    } else {
        hipLaunchKernelGGL(dmx_scan_kernel, dim3(1), dim3(ST), 0, s, c->tiles, nblk, n, o.flags, out_cap,
                           (uint32_t*)d_out, c->res, c->nfb, hintp);
        if (nblk)
            hipLaunchKernelGGL(dmx_scan_apply_kernel, dim3(ntile), dim3(SCAN_TILE), 0, s, c->info, nblk, o.flags, (uint32_t)o.sw, c->tiles,
                               (uint32_t*)d_out, (const dmx_result*)c->res, wl, L4, dupk);
    }
    if (ev && ((c->timing >> 4) & 1)) (void)hipEventRecord(ev[4], s);
    if (nblk)
        hipLaunchKernelGGL(dmx_pack_kernel, dim3(wl && wsh.list4 ? list_grid(nblk, wsh.n4, 2 * c->ncu, 16 * c->ncu) : nblk),
                           dim3(PT), 0, s, (const uint8_t*)d_in, (uint32_t)o.sw, c->tok, c->codes, c->hdr, c->info, c->sub,
                           nblk, o.flags, (uint32_t*)d_out, c->res, wl, wl && wsh.list4 ? L4 : NULL, dupk);
    // the blocks K4 skipped that K0 did not complete: dups, and the stored prefix unless every
    // block is a full 16-byte aligned one (a wave per 4 blocks)
#ifdef DMX_K0_NOREST
    const bool k0rest = false;
#else
    const bool k0rest = o.sw == SCT * 16 * 8 && (reinterpret_cast<uintptr_t>(d_in) & 15) == 0;
#endif
    if (nblk && wl && (dupa || !k0rest))
        hipLaunchKernelGGL(dmx_fill_kernel, dim3((nblk + 15) / 16), dim3(256), 0, s, (const uint8_t*)d_in, (uint32_t)o.sw,
                           o.flags, (const dmx_blkinfo*)c->info, (const uint32_t*)wl, (uint64_t)c->cap_blocks, nblk,
                           (uint32_t*)d_out, (const dmx_result*)c->res, dupa ? 1u : 0u);
    if (ev && ((c->timing >> 5) & 1)) (void)hipEventRecord(ev[5], s);
    HIPCHK(fault_hit(2) ? hipErrorLaunchFailure : hipGetLastError());
    c->last_nblk = nblk;
    c->last_sw = (uint32_t)o.sw;
    return 0;
}

extern "C" int dmx_encode_result_async(dmx_ctx* c, dmx_result* r, void* stream) {
    if (!c || !r) return -(int)E_INVAL;
    HIPCHK(hipSetDevice(c->device));
    hipStream_t s = stream ? (hipStream_t)stream : c->stream;
    HIPCHK(hipMemcpyAsync(r, c->res, sizeof(dmx_result), hipMemcpyDeviceToHost, s));
    return 0;
}

extern "C" int dmx_encode_result(dmx_ctx* c, dmx_result* r, void* stream) {
    HIPCHK(hipSetDevice(c->device));
    hipStream_t s = stream ? (hipStream_t)stream : c->stream;
    HIPCHK(hipMemcpyAsync(r, c->res, sizeof(dmx_result), hipMemcpyDeviceToHost, s));
    HIPCHK(hipStreamSynchronize(s));
    return 0;
}

extern "C" int dmx_ctx_set_timing(dmx_ctx* c, int enable) {
    (void)hipSetDevice(c->device);
    for (int j = 0; j < DMX_EV_RING; j++) c->ev_used[j] = 0;
    // 1: every stage boundary; 0x100 | s: only stage s's two events (s = 0 .. 4), so a timed
    // loop pays two event records per encode (each one a gap of a few us between kernels)
    c->timing = enable == 1 ? 0x3F : (enable & 0x100) ? 3 << (enable & 7) : 0;
    // 0x100 | s | every << 12: events on every `every`-th encode only (sampling the stage
    // inside a timed loop at a fraction of the event records' idle)
    c->ev_every = (enable & 0x100) ? ((uint32_t)enable >> 12) & 0xFFu : 0u;
    c->ev_count = 0;
    for (int k = 0; k < 6; k++) c->stage_ms[k] = 0;
    c->stage_n = 0;
    return 0;
}

extern "C" int dmx_ctx_stage_times(dmx_ctx* c, double* ms6, uint32_t* count) {
    (void)hipSetDevice(c->device);
    for (int j = 0; j < DMX_EV_RING; j++) ctx_collect_set(c, j);
    for (int k = 0; k < 6; k++) ms6[k] = c->stage_n ? c->stage_ms[k] / c->stage_n : 0.0;
    *count = c->stage_n;
    return 0;
}

__global__ void dmx_index_kernel(const dmx_blkinfo* __restrict__ info, uint32_t nblk, uint32_t sw,
                                 dmx_iblock* __restrict__ ix) {
    const uint32_t b = blockIdx.x * blockDim.x + threadIdx.x;
    if (b >= nblk) return;
    dmx_iblock e;
    e.bit = info[b].off_bits;
    e.out_off = (uint64_t)b * sw;
    e.out_len = info[b].n;
    e.reserved = 0;
    ix[b] = e;
}

extern "C" int dmx_block_index(dmx_ctx* c, dmx_iblock* d_index, uint32_t cap, void* stream) {
    if (!c || !d_index) return -(int)E_INVAL;
    if (cap < c->last_nblk) return -(int)E_RANGE;
    if (!c->last_nblk) return 0;
    HIPCHK(hipSetDevice(c->device));
    hipStream_t s = stream ? (hipStream_t)stream : c->stream;
    hipLaunchKernelGGL(dmx_index_kernel, dim3((c->last_nblk + 255) / 256), dim3(256), 0, s, c->info, c->last_nblk,
                       c->last_sw, d_index);
    HIPCHK(hipGetLastError());
    return (int)c->last_nblk;
}

extern "C" int dmx_last_blocks(dmx_ctx* c, uint32_t* ntok, uint8_t* btype, uint32_t* hdr_bits, uint32_t cap) {
    const uint32_t nb = c->last_nblk < cap ? c->last_nblk : cap;
    if (!nb) return 0;
    HIPCHK(hipSetDevice(c->device));
    HIPCHK(hipStreamSynchronize(c->stream));
    HIPCHK(hipDeviceSynchronize());
    dmx_blkinfo* h = (dmx_blkinfo*)malloc(sizeof(dmx_blkinfo) * nb);
    if (!h) return -(int)E_MALLOC;
    if (hip_fail(hipMemcpy(h, c->info, sizeof(dmx_blkinfo) * nb, hipMemcpyDeviceToHost), "hipMemcpy")) { free(h); return -(int)E_DEVICE; }
    for (uint32_t b = 0; b < nb; b++) {
        if (ntok) ntok[b] = h[b].ntok;
        if (btype) btype[b] = (uint8_t)h[b].btype;
        if (hdr_bits) hdr_bits[b] = h[b].hdr_bits;
    }
    free(h);
    return (int)nb;
}

extern "C" int dmx_last_tokens(dmx_ctx* c, uint32_t blk, uint32_t* tok, uint32_t cap) {
    if (blk >= c->last_nblk) return -(int)E_RANGE;
    HIPCHK(hipSetDevice(c->device));
    HIPCHK(hipDeviceSynchronize());
    dmx_blkinfo bi;
    HIPCHK(hipMemcpy(&bi, c->info + blk, sizeof(bi), hipMemcpyDeviceToHost));
    const uint32_t nt = bi.ntok < cap ? bi.ntok : cap;
    if (nt) HIPCHK(hipMemcpy(tok, c->tok + (uint64_t)blk * DMX_BLK, nt * sizeof(uint32_t), hipMemcpyDeviceToHost));
    return (int)bi.ntok;
}

extern "C" int dmx_last_code_lengths(dmx_ctx* c, uint32_t blk, uint8_t* lens316) {
    if (blk >= c->last_nblk) return -(int)E_RANGE;
    HIPCHK(hipSetDevice(c->device));
    HIPCHK(hipDeviceSynchronize());
    uint32_t cw[316];
    HIPCHK(hipMemcpy(cw, c->codes + (uint64_t)blk * DMX_NSUB * DMX_HIST, sizeof(cw), hipMemcpyDeviceToHost));
    for (int s = 0; s < 316; s++) lens316[s] = (uint8_t)(cw[s] >> 16);
    return 0;
}

extern "C" int dmx_last_subblock(dmx_ctx* c, uint32_t blk, uint32_t sub, uint32_t* tok_range, uint32_t* btype,
                                 uint32_t* hdr_bits, uint8_t* lens316) {
    if (blk >= c->last_nblk || sub >= DMX_NSUB) return -(int)E_RANGE;
    HIPCHK(hipSetDevice(c->device));
    HIPCHK(hipDeviceSynchronize());
    dmx_blkinfo bi;
    HIPCHK(hipMemcpy(&bi, c->info + blk, sizeof(bi), hipMemcpyDeviceToHost));
    if (sub >= bi.nsub) return -(int)E_RANGE;
    const uint64_t slot = (uint64_t)blk * DMX_NSUB + sub;
    dmx_subinfo si;
    HIPCHK(hipMemcpy(&si, c->sub + slot, sizeof(si), hipMemcpyDeviceToHost));
    if (tok_range) { tok_range[0] = si.t0; tok_range[1] = si.t1; }
    if (btype) *btype = si.btype;
    if (hdr_bits) *hdr_bits = si.hdr_bits;
    if (lens316) {
        uint32_t cw[316];
        HIPCHK(hipMemcpy(cw, c->codes + slot * DMX_HIST, sizeof(cw), hipMemcpyDeviceToHost));
        for (int k = 0; k < 316; k++) lens316[k] = (uint8_t)(cw[k] >> 16);
    }
    return (int)bi.nsub;
}

