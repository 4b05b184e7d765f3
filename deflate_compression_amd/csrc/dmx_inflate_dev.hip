// dmx_inflate_dev.hip -- RFC 1950/1951 inflate on the MI355X.
//
// Two kernels over one decoder:
//   * indexed (dmx_inflate_index_kernel): one single-wave workgroup per sw block listed in a
//     block index {start bit, output offset, output length}; it decodes DEFLATE blocks until
//     the sw block's output is complete (one, or up to four with DMX_F_SPLIT).  Blocks of a dmx stream
//     never reference earlier blocks (every sw-sized block is its own window),
//     so all blocks decode in parallel; the encoder exports the index (dmx_block_index).
//   * stream (dmx_inflate_stream_kernel): one workgroup decodes a whole zlib stream
//     (header, blocks until BFINAL, Adler-32 check) -- any RFC 1950 stream, e.g. PNG IDAT.
//
// The decoder is wave-uniform: the 64-bit bit buffer, the stream word index and the output
// position are SGPRs; the compressed stream is staged in two VGPRs (one dword per lane, the
// next 256 bytes prefetched), so a refill is a v_readlane.  The common path of the symbol loop
// is hand-scheduled (isym_run): the literal/length and distance tables live in VGPRs during it
// (a v_readlane under the VGPR index mode per lookup, no LDS round trip), each entry carries its base
// and is the s_bfe control of its own extra bits, a literal is one LDS byte store, and a match
// is copied by the whole wave, 64 bytes a round (periodic sources by residue; sources older
// than the ring from the output already flushed to HBM).  Output is assembled in an LDS ring
// and written to HBM in 16-byte-per-lane coalesced stores every half ring (indexed mode: an
// 8 KiB ring; stream mode: the 32 KiB window, folding the Adler-32 sums into the same pass).
// Tables: 10-bit first level, built lane-parallel (ballot counts and ranks) into a per-
// workgroup area of HBM and loaded into VGPRs by the symbol loop, so that LDS holds only the
// ring (12 workgroups per CU); longer codes take a canonical slow path (first code / count /
// offset per length, in LDS).
#include <hip/hip_runtime.h>
#include <pthread.h>
#include <stdint.h>
#include <type_traits>
#include <stdio.h>
#include <string.h>

#include "../../include/dmx.h"

#define IW 32768          // window = LDS ring (stream mode; the indexed mode's ring is IWX)
#ifndef DMX_IWX
#define DMX_IWX 8192      // indexed mode: an 8 KiB ring, older sources read back from HBM
#endif
#define IWX DMX_IWX
#define IWC 4096          // chained decode: a ring of 4 096 cells (8 KiB)
#define IFB 10            // first-level table bits
#define ITAB_WORDS 2048   // a workgroup's first-level tables in HBM: literal/length, then distance
#define IFLUSH 16384      // stream mode: flush to HBM every IFLUSH bytes (half the ring)

// The first-level entries (1 << IFB words per table, format "Table entries" below) live in
// HBM, ITAB_WORDS per workgroup: the symbol loop holds them in VGPRs and reloads them at each
// entry (agent-scope loads, L2), so LDS keeps only the ring and these small arrays -- 10 KB
// a workgroup, and all 3 052 blocks of 100 MB resident at once (12 per CU, the VGPR limit)
// instead of 2 048 (8 per CU with the tables in LDS).
struct ITable {
    uint16_t first[16];        // first canonical code of each length
    uint16_t cnt[16];
    uint16_t offs[16];         // index into sym[] of the first symbol of each length
    uint16_t sym[288];         // symbols sorted by (length, symbol)
};

// T = uint8_t: the output bytes; T = uint16_t: cells of the chained decode (a byte value, or
// 0x100 + b - 1 for the byte b positions before the sw block's first output byte, resolved
// afterwards: dmx_inflate_chained_async)
template <uint32_t W, typename T = uint8_t>
struct InfLDS {
    T win[W];
    ITable lt, dt;
    uint8_t len[320];
    uint8_t seq[320];
};

__device__ __forceinline__ uint32_t rfl(uint32_t v) { return __builtin_amdgcn_readfirstlane(v); }
__device__ __forceinline__ uint64_t rfl64(uint64_t v) {
    return ((uint64_t)rfl((uint32_t)(v >> 32)) << 32) | rfl((uint32_t)v);
}

// ---------------------------------------------------------------------------------------
// Bit reader.  Coordinates are relative to the dword-aligned address at or below z.  The
// stream is staged in two VGPRs, one dword per lane: vcur holds words wb + lane, vnxt words
// wb + 64 + lane, so a refill is one v_readlane; when the reader passes into vnxt the pair
// advances and the load of the next 256 bytes is issued, 64 refills before it is needed.
// Words that are not wholly inside the stream are assembled from bytes (zeros past the end).
// ---------------------------------------------------------------------------------------
// global-space views: plain loads, not flat ones (a flat load counts in lgkmcnt too, so every
// LDS wait would also wait for the stream prefetch)
typedef __attribute__((address_space(1))) const uint8_t gu8;
typedef __attribute__((address_space(1))) const uint32_t gu32;

struct IBits {
    gu8* zb;               // aligned base as bytes
    uint32_t lo, hi;       // valid byte range [lo, hi) relative to zb
    uint32_t wfast;        // words < wfast are wholly inside the stream
    uint32_t wb;           // word index of vcur's lane 0 (a multiple of 64)
    uint32_t vcur, vnxt;   // per lane: word wb + lane, word wb + 64 + lane
    uint32_t wi;           // next word
    uint32_t bc;
    uint64_t bb;
};

__device__ __forceinline__ uint32_t ib_vload(const IBits& r, uint32_t w0) {   // word w0 + lane
    const uint32_t wi = w0 + __lane_id();
    if (wi < r.wfast) return reinterpret_cast<gu32*>(r.zb)[wi];
    uint32_t v = 0;
    for (uint32_t j = 0; j < 4; j++) {
        const uint32_t b = wi * 4 + j;
        if (b >= r.lo && b < r.hi) v |= (uint32_t)r.zb[b] << (8 * j);
    }
    return v;
}
__device__ __forceinline__ uint32_t ib_word(IBits& r, uint32_t wi) {   // wi: sequential from the seek
    uint32_t k = wi - r.wb;
    if (k >= 64) {
        r.vcur = r.vnxt;
        r.wb += 64;
        r.vnxt = ib_vload(r, r.wb + 64);
        k -= 64;
    }
    return __builtin_amdgcn_readlane(r.vcur, k);
}
__device__ __forceinline__ void ib_refill(IBits& r) {   // afterwards bc >= 32
    if (r.bc <= 32) {
        r.bb |= (uint64_t)ib_word(r, r.wi) << r.bc;
        r.wi++;
        r.bc += 32;
    }
}
// a word read that starts 8 or more bytes past the end of the stream (word wi - 1 was the last read)
__device__ __forceinline__ bool ib_over(const IBits& r) { return (uint64_t)r.wi * 4 >= (uint64_t)r.hi + 12; }
__device__ __forceinline__ void ib_seek(IBits& r, uint64_t bit) {   // bit: relative to z
    const uint64_t ab = bit + (uint64_t)r.lo * 8;
    r.wi = (uint32_t)(ab >> 5);
    r.wb = r.wi & ~63u;
    r.vcur = ib_vload(r, r.wb);
    r.vnxt = ib_vload(r, r.wb + 64);
    r.bb = (uint64_t)ib_word(r, r.wi) >> (ab & 31);
    r.bc = 32 - (uint32_t)(ab & 31);
    r.wi++;
}
__device__ __forceinline__ void ib_init(IBits& r, const uint8_t* z, uint64_t zbytes) {
    const uintptr_t a = (uintptr_t)z;
    r.zb = (gu8*)(a & ~(uintptr_t)3);
    r.lo = (uint32_t)(a & 3);
    r.hi = r.lo + (uint32_t)zbytes;
    r.wfast = r.hi >> 2;
    r.wi = r.wb = 0;
    r.vcur = r.vnxt = 0;
    r.bb = 0;
    r.bc = 0;
}
__device__ __forceinline__ uint32_t ib_peek(const IBits& r, uint32_t n) { return (uint32_t)r.bb & ((1u << n) - 1); }
__device__ __forceinline__ void ib_drop(IBits& r, uint32_t n) {
    r.bb >>= n;
    r.bc -= n;
}
__device__ __forceinline__ uint32_t ib_bits(IBits& r, uint32_t n) {   // n <= 32
    ib_refill(r);
    const uint32_t v = n ? ib_peek(r, n) : 0;
    ib_drop(r, n);
    return v;
}
__device__ __forceinline__ uint64_t ib_bytepos(const IBits& r) {   // after ib_align; relative to z
    return (uint64_t)r.wi * 4 - r.bc / 8 - r.lo;
}

#define ISLOW 0xFFFFu

// DEFLATE length / distance bases by arithmetic (RFC 1951 3.2.5), no table loads.
__device__ __forceinline__ uint32_t len_extra(uint32_t li) { return li < 8 || li == 28 ? 0 : (li - 4) >> 2; }
__device__ __forceinline__ uint32_t len_base(uint32_t li) {
    return li < 8 ? li + 3 : li == 28 ? 258 : ((4 + (li & 3)) << ((li - 4) >> 2)) + 3;
}
__device__ __forceinline__ uint32_t dist_extra(uint32_t d) { return d < 4 ? 0 : (d - 2) >> 1; }
__device__ __forceinline__ uint32_t dist_base(uint32_t d) { return d < 4 ? d + 1 : ((2 + (d & 1)) << ((d - 2) >> 1)) + 1; }

// Table entries (32-bit).  The symbol loop looks its codes up in 1024-entry tables held in 16
// VGPRs (entry x in lane x & 63 of register x >> 6: a v_readlane under the index mode, no LDS round
// trip).  A length or distance entry is laid out so that it is itself the s_bfe control that
// extracts its extra bits from the bit buffer: bits [4:0] the code length (the field's offset),
// [22:16] the extra-bit count (its width); [12:8] code + extra bits (the bits to drop).
//   literal/length: literal  sym << 16 | clen                      (bit 15 clear)
//                   length   base << 23 | extra << 16 | 0x8000 | (clen + extra) << 8 | clen
//                   EOB      0xC000 | clen;  invalid (286, 287) 0xE000 | clen  (bit 14 set)
//   distance:       m << 28 | extra << 16 | (clen + extra) << 8 | clen, where base - 1 = m << extra
//                   (m = code for codes 0..3, 2 + (code & 1) above);  IVBAD invalid (30, 31)
//   both:           IVSLOW: a code longer than IFB bits (or none) -- the canonical slow path
#define IVSLOW 0xFFFFFFFFu
#define IVBAD 0xFFFFFFFEu
__device__ __forceinline__ uint32_t iv_ll(uint32_t e) {   // from a sym << 4 | clen entry
    if (e == ISLOW) return IVSLOW;
    const uint32_t sym = e >> 4, l = e & 15u;
    if (sym < 256) return (sym << 16) | l;
    if (sym == 256) return 0xC000u | l;
    const uint32_t li = sym - 257;
    if (li >= 29) return 0xE000u | l;
    const uint32_t x = len_extra(li);
    return (len_base(li) << 23) | (x << 16) | 0x8000u | ((l + x) << 8) | l;
}
__device__ __forceinline__ uint32_t iv_d(uint32_t e) {
    if (e == ISLOW) return IVSLOW;
    const uint32_t ds = e >> 4, l = e & 15u;
    if (ds >= 30) return IVBAD;
    const uint32_t x = dist_extra(ds), m = ds < 4 ? ds : 2 + (ds & 1);
    return (m << 28) | (x << 16) | ((l + x) << 8) | l;
}
// the value of a length / distance entry's field (its extra bits at the reader) and its base
__device__ __forceinline__ uint32_t iv_extra(uint64_t bb, uint32_t e) {
    return (uint32_t)(bb >> (e & 31u)) & ((1u << ((e >> 16) & 15u)) - 1);
}
__device__ __forceinline__ uint32_t iv_dbase(uint32_t e) { return ((e >> 28) << ((e >> 16) & 15u)) + 1; }

// ---------------------------------------------------------------------------------------
// Huffman tables, lane-parallel over symbols (lane t holds symbols t, t + 64, ...): counts per
// code length by ballots, the canonical first codes and offsets (uniform), then each symbol's
// rank among the symbols of its length (mbcnt of the same ballots) gives its code and its slot
// in the length-sorted list; every lane then fills its symbol's first-level entries at once,
// in the 32-bit format above (DIST: a distance table; otherwise literal/length, which also
// serves the code length code: its symbols 0..18 take the literal form).  IVSLOW marks a code
// longer than IFB bits (or no code).  Returns 0 complete, 1 incomplete, -1 over-subscribed.
// ---------------------------------------------------------------------------------------
// agent-scope load of a table word (to L2, past the vector L1, which may hold the words of the
// previous block's table)
__device__ __forceinline__ uint32_t gtab_ld(const uint32_t* p) {
    return __hip_atomic_load((const __attribute__((address_space(1))) uint32_t*)p, __ATOMIC_RELAXED,
                             __HIP_MEMORY_SCOPE_AGENT);
}

template <bool DIST, uint32_t W, typename TW>
__device__ __forceinline__ int itable_build(InfLDS<W, TW>& S, ITable& T, uint32_t* __restrict__ fast, int n,
                                            uint32_t lane) {
    const int nc = (n + 63) >> 6;   // symbol chunks, <= 5
    uint32_t lc[5];
#pragma unroll
    for (int c = 0; c < 5; c++) {
        const int s = c * 64 + (int)lane;
        lc[c] = (c < nc && s < n) ? S.len[s] : 0u;
    }
    for (int k = (int)lane; k < (1 << IFB); k += 64) fast[k] = IVSLOW;
    uint32_t cnt[16], first[16], offs[16];
#pragma unroll
    for (int l = 1; l < 16; l++) {
        uint32_t t = 0;
#pragma unroll
        for (int c = 0; c < 5; c++)
            if (c < nc) t += (uint32_t)__popcll(__ballot(lc[c] == (uint32_t)l));
        cnt[l] = t;
    }
    // Kraft check, first codes and offsets (uniform)
    int left = 1, res = 0;
    uint32_t code = 0, off = 0, cprev = 0;
#pragma unroll
    for (int l = 1; l < 16; l++) {
        left = 2 * left - (int)cnt[l];
        if (left < 0) res = -1;
        code = (code + cprev) << 1;
        first[l] = code;
        offs[l] = off;
        if (lane == 0) {
            T.first[l] = (uint16_t)code;
            T.cnt[l] = (uint16_t)cnt[l];
            T.offs[l] = (uint16_t)off;
        }
        off += cnt[l];
        cprev = cnt[l];
    }
    if (res == 0 && left > 0) res = 1;
    if (off == 0) res = 1;   // no codes at all
    if (res >= 0) {
        uint32_t run[16];
#pragma unroll
        for (int l = 1; l < 16; l++) run[l] = 0;
#pragma unroll
        for (int c = 0; c < 5; c++) {
            if (c >= nc) break;
            const uint32_t l0 = lc[c];
            uint32_t mycode = 0, myoff = 0;
#pragma unroll
            for (int l = 1; l < 16; l++) {
                const uint64_t m = __ballot(l0 == (uint32_t)l);
                const uint32_t below = __builtin_amdgcn_mbcnt_hi((uint32_t)(m >> 32), __builtin_amdgcn_mbcnt_lo((uint32_t)m, 0u));
                if (l0 == (uint32_t)l) {
                    mycode = first[l] + run[l] + below;
                    myoff = offs[l] + run[l] + below;
                }
                run[l] += (uint32_t)__popcll(m);
            }
            if (l0) {
                const uint32_t s = c * 64 + lane;
                T.sym[myoff] = (uint16_t)s;
                if (l0 <= IFB) {
                    const uint32_t rv = __brev(mycode) >> (32 - l0);
                    const uint32_t e16 = (s << 4) | l0;
                    const uint32_t e = DIST ? iv_d(e16) : iv_ll(e16);
                    for (uint32_t j = 0; j < (1u << (IFB - l0)); j++) fast[rv | (j << l0)] = e;
                }
            }
        }
    }
    __builtin_amdgcn_s_waitcnt(0);   // the table stores are done before anyone loads them
    __syncthreads();
    return res;
}

// Entry for the code at the reader (caller refilled: bc >= 15): the first-level entry, or
// for longer codes the canonical decode; ISLOW = no valid code.
__device__ __forceinline__ uint32_t ientry_slow(const IBits& r, const ITable& T) {
    const uint32_t cr = __brev((uint32_t)r.bb);   // next bits, first bit in the MSB
    for (uint32_t l = IFB + 1; l < 16; l++) {
        const uint32_t code = cr >> (32 - l);
        const uint32_t d = code - rfl(T.first[l]);
        if (d < rfl(T.cnt[l])) return (rfl(T.sym[rfl(T.offs[l]) + d]) << 4) | l;
    }
    return ISLOW;
}
// the code length code (symbols 0..18, in the literal form): sym << 4 | len, or ISLOW
__device__ __forceinline__ uint32_t ientry_cl(const IBits& r, const ITable& T, const uint32_t* fast) {
    const uint32_t e = rfl(gtab_ld(fast + ib_peek(r, IFB)));
    return e != IVSLOW ? (((e >> 16) & 0xFFu) << 4) | (e & 15u) : ientry_slow(r, T);
}

__constant__ uint8_t c_iclorder[19] = {16, 17, 18, 0, 8, 7, 9, 6, 10, 5, 11, 4, 12, 3, 13, 2, 14, 1, 15};

// ---------------------------------------------------------------------------------------
// Output.  Positions are 32-bit and relative to ob (a multiple of IW, so the window index
// of a position is pos & IM); stream mode moves ob forward as it flushes.
// ---------------------------------------------------------------------------------------
// DMX_INF_STAMPS (diagnostic builds only): per-workgroup cycle totals of the decode phases
#ifdef DMX_INF_STAMPS
#define INF_NST 16
__device__ unsigned long long dmx_inf_st[1 << 16][INF_NST];
#define IST_NOW() __builtin_amdgcn_s_memtime()
#define IST_ADD(o, k, v) ((o).st[k] += (v))
#else
#define IST_NOW() 0ull
#define IST_ADD(o, k, v) ((void)0)
#endif

struct IOut {
#ifdef DMX_INF_STAMPS
    unsigned long long st[INF_NST];   // 0 header + tables, 1 symbol loop, 2 flushes, 3 matches, 4 far matches, 5 asm runs,
                                      // 6 blocks, 7 code length table, 8 code lengths, 9 literal/length table,
                                      // 10 distance table, 11..15 asm-run exits IX_SYM .. IX_MATCH
#endif
    uint8_t* out;     // + base + ob = position 0
    uint64_t base, ob, cap;   // cap: absolute output capacity
    uint32_t op, fl;  // produced / flushed (relative)
    uint32_t a, b;    // stream mode: Adler-32 of everything flushed
};
#define IRENORM (1u << 30)

__device__ __forceinline__ uint32_t io_caprel(const IOut& o) {
    const uint64_t c = o.cap - o.ob;
    return c > 0x80000000ull ? 0x80000000u : (uint32_t)c;
}

__device__ __forceinline__ uint64_t wave_sum64(uint64_t v) {
    for (int s = 32; s >= 1; s >>= 1) v += __shfl_xor(v, s, 64);
    return v;
}

// Write window bytes [fl, upto) to HBM (upto - fl <= W).  ADLER: fold them into (a, b).
// Cells: window positions [fl, upto) to the cell buffer (2 bytes a position), 8 cells (16
// bytes) per lane where the destination is 16-byte aligned.
template <uint32_t W>
__device__ __forceinline__ void io_flush_cells(InfLDS<W, uint16_t>& S, IOut& o, uint32_t upto, uint32_t lane) {
    constexpr uint32_t IM = W - 1;
    __syncthreads();
    uint16_t* dst = reinterpret_cast<uint16_t*>(o.out) + o.base + o.ob;
    uint32_t p = o.fl;
    const uint32_t head = min(upto - p, (uint32_t)(((16 - (((uintptr_t)(dst + p)) & 15)) & 15) >> 1));
    if (lane < head) dst[p + lane] = S.win[(p + lane) & IM];
    p += head;
    for (; p + 8 <= upto; p += 512) {
        const uint32_t q = p + lane * 8;
        if (q + 8 <= upto) {
            uint32_t w[4];
#pragma unroll
            for (int k = 0; k < 4; k++)
                w[k] = (uint32_t)S.win[(q + 2 * k) & IM] | ((uint32_t)S.win[(q + 2 * k + 1) & IM] << 16);
            *(uint4*)&dst[q] = make_uint4(w[0], w[1], w[2], w[3]);
        } else if (q < upto) {
            for (uint32_t t = q; t < upto; t++) dst[t] = S.win[t & IM];
        }
    }
    if (p < upto && lane == 0)
        for (uint32_t t = p; t < upto; t++) dst[t] = S.win[t & IM];
    o.fl = upto;
    __builtin_amdgcn_s_waitcnt(0);   // the stores are done: far-match reads see them
    if (o.fl >= IRENORM) {
        o.ob += IRENORM;
        o.op -= IRENORM;
        o.fl -= IRENORM;
    }
    __syncthreads();
}

template <bool ADLER, uint32_t W, typename TW>
__device__ __forceinline__ void io_flush(InfLDS<W, TW>& S, IOut& o, uint32_t upto, uint32_t lane) {
    if constexpr (sizeof(TW) == 2) {
        io_flush_cells<W>(S, o, upto, lane);
        return;
    } else {
    constexpr uint32_t IM = W - 1;
    [[maybe_unused]] const unsigned long long ts0 = IST_NOW();
    __syncthreads();
    uint8_t* dst = o.out + o.base + o.ob;
    const uint32_t n = upto - o.fl;
    uint64_t ss = 0, tt = 0;
    uint32_t p = o.fl;
    // byte head up to a 16-byte aligned destination
    const uint32_t head = min(n, (uint32_t)((16 - (((uintptr_t)dst + p) & 15)) & 15));
    if (lane < head) {
        const uint32_t x = S.win[(p + lane) & IM];
        dst[p + lane] = (uint8_t)x;
        if (ADLER) { ss += x; tt += (uint64_t)(n - lane) * x; }
    }
    p += head;
    // 16 bytes per lane
    for (; p + 16 <= upto; p += 1024) {
        const uint32_t q = p + lane * 16;
        if (q + 16 <= upto) {
            uint32_t w[4];
            const uint32_t wp = q & IM;
            if ((wp & 15) == 0) {
                const uint4 v = *(const uint4*)&S.win[wp];
                w[0] = v.x; w[1] = v.y; w[2] = v.z; w[3] = v.w;
            } else {
                for (int k = 0; k < 4; k++) {
                    uint32_t x = 0;
                    for (int j = 0; j < 4; j++) x |= (uint32_t)S.win[(q + 4 * k + j) & IM] << (8 * j);
                    w[k] = x;
                }
            }
            *(uint4*)&dst[q] = make_uint4(w[0], w[1], w[2], w[3]);
            if (ADLER) {
                const uint32_t rem = upto - q;   // weight of the first byte
                for (int k = 0; k < 16; k++) {
                    const uint32_t x = (w[k >> 2] >> (8 * (k & 3))) & 0xFFu;
                    ss += x;
                    tt += (uint64_t)(rem - k) * x;
                }
            }
        } else if (q < upto) {   // the last partial stride: bytes
            for (uint32_t t = q; t < upto; t++) {
                const uint32_t x = S.win[t & IM];
                dst[t] = (uint8_t)x;
                if (ADLER) { ss += x; tt += (uint64_t)(upto - t) * x; }
            }
        }
    }
    if (p < upto && lane == 0) {   // fewer than 16 bytes left after the loop
        for (uint32_t t = p; t < upto; t++) {
            const uint32_t x = S.win[t & IM];
            dst[t] = (uint8_t)x;
            if (ADLER) { ss += x; tt += (uint64_t)(upto - t) * x; }
        }
    }
    if (ADLER) {
        ss = wave_sum64(ss);
        tt = wave_sum64(tt);
        // a' = a + S; b' = b + n * a + T  (mod 65521)
        const uint64_t b2 = (o.b + (uint64_t)(n % 65521) * o.a + tt % 65521) % 65521;
        o.a = rfl((uint32_t)((o.a + ss % 65521) % 65521));
        o.b = rfl((uint32_t)b2);
    }
    o.fl = upto;
    __builtin_amdgcn_s_waitcnt(0);   // the stores are done: far-match reads see them
    if (o.fl >= IRENORM) {   // keep relative positions small (ob stays a multiple of W)
        o.ob += IRENORM;
        o.op -= IRENORM;
        o.fl -= IRENORM;
    }
    __syncthreads();
    IST_ADD(o, 2, IST_NOW() - ts0);
    }
}

// LDS byte address of a __shared__ object (ds_* instructions address LDS from 0)
__device__ __forceinline__ uint32_t lds_addr(const void* p) {
    return (uint32_t)(uintptr_t)(const __attribute__((address_space(3))) void*)p;
}

// ---------------------------------------------------------------------------------------
// The symbol loop's common path, hand-scheduled.  Compiled code for this state machine spent
// ~100 instructions a token (the structurizer's branch flags, copies of the stream registers
// that waited for their prefetch); this one spends ~20 on a literal and ~60 on a match.
// In SGPRs: the 64-bit bit buffer (s[94:95]), bc, wi, op; the two tables come from HBM (the
// workgroup's table area, agent-scope loads) into v64..v79 (literal/length) and v80..v95
// (distance, bases in v96..v111) and are read by
// v_readlane under s_set_gpr_idx_on.  A literal is one ds_write_b8 (every lane stores the same
// byte); a match is 64 bytes a round (lane t: byte src + t, read before the round's writes,
// when distance >= length or >= 64; byte src + t mod distance for a shorter period; a
// source older than the ring from the flushed output in HBM).  Returns at the first event it
// leaves to the caller, with nothing of the current token consumed unless noted:
//   IX_SYM   a long, end-of-block or invalid literal/length code
//   IX_SEG   a refill at a token start that needs a stream segment it does not rotate into
//            (the segment after next is not wholly inside the stream)
//   IX_LIM   op >= lim at a literal or a length (a flush the run does not do itself, or the
//            capacity), or a length that does not fit the capacity
//   IX_DIST  length decoded into len; the distance code is long or invalid
//   IX_MATCH len and dist decoded: a distance before the output
// Hazards: a lane select written by SALU is 4+ instructions old at each v_readlane (s_nop 3
// where it is not); the stream prefetch is waited for before it is read and before return;
// m0 (written by s_set_gpr_idx_on) is restored.
// ---------------------------------------------------------------------------------------
// diagnostic timing builds only (the output is wrong): DMX_INF_NOFAR copies far sources from
// the ring instead of HBM, DMX_INF_NOWAIT writes a copy round without waiting for its reads
#ifdef DMX_INF_NOFAR
#define IFAR_BRANCH "s_cbranch_scc1 L_cp%=\n"
#else
#define IFAR_BRANCH "s_cbranch_scc1 L_far%=\n"
#endif
#ifdef DMX_INF_NOWAIT
#define ICOPY_WAIT
#else
#define ICOPY_WAIT "s_waitcnt lgkmcnt(0)\n"
#endif
// table lookups: lane s94 & 63 of register v64 + (s94 >> 6 & 15) (v80 + for distances, their
// bases at v96 +), read by v_readlane under the index mode: the mode indexes the readlane's
// VGPR source too (tools/gpridx_test.hip checks it on the device), so a lookup is s_bfe,
// s_set_gpr_idx_on, v_readlane, s_set_gpr_idx_off -- no VGPR copy of the indexed register
#define ILOOK_LL "s_set_gpr_idx_on s98, gpr_idx(SRC0)\n" "v_readlane_b32 s99, v64, s94\n" "s_set_gpr_idx_off\n"
#define ILOOK_D "s_set_gpr_idx_on s98, gpr_idx(SRC0)\n" "v_readlane_b32 s99, v80, s94\n" \
                "v_readlane_b32 s90, v96, s94\n" "s_set_gpr_idx_off\n"
// A copy of one round (length <= 64) is left pending: its LDS read (or HBM load, for a source
// older than the ring) is issued and the wave goes on decoding the next token while it is in
// flight; the write (lanes in s[84:85], data v116 >> v118, address v117) is issued before
// the next read of the ring, the next copy, or the return.  Literal stores in between touch
// other positions.
#define IFLUSH_PENDING(N) \
    "s_cmp_eq_u64 s[84:85], 0\n" \
    "s_cbranch_scc1 L_nf" #N "%=\n" \
    "s_waitcnt vmcnt(0) lgkmcnt(0)\n" \
    "s_mov_b64 exec, s[84:85]\n" \
    "v_lshrrev_b32 v116, v118, v116\n" \
    IWR " v117, v116\n" \
    "s_mov_b64 exec, s[86:87]\n" \
    "s_mov_b64 s[84:85], 0\n" \
    "L_nf" #N "%=:\n"
#define IX_SYM 1u
#define IX_SEG 2u
#define IX_LIM 3u
#define IX_DIST 4u
#define IX_MATCH 5u

template <uint32_t W, bool CELL>
__device__ __forceinline__ uint32_t isym_run(IBits& r, uint32_t& op, uint32_t& lim, uint32_t& fl, uint32_t capr,
                                             uint32_t fok, uint64_t gfl, uint32_t dfl, uint32_t lta,
                                             uint64_t tgl, uint64_t tgd, uint32_t toff, uint32_t lane, uint64_t gpos0,
                                             uint32_t& len, uint32_t& dist) {
    uint32_t ex;
    const uint64_t galn = gpos0 & ~3ull;   // output position 0 in HBM, as an aligned base + 0..3
    const uint32_t gmis = (uint32_t)gpos0 & 3u;
    const int32_t wrl = (int32_t)r.wfast - 192;   // rotate while the new segment is wholly inside
    const uint64_t zb = (uint64_t)(uintptr_t)r.zb;
    if constexpr (!CELL) {
#define ISYM_CELL 0
#include "dmx_isym.inc"
#undef ISYM_CELL
    } else {
#define ISYM_CELL 1
#include "dmx_isym.inc"
#undef ISYM_CELL
    }
    return ex;
}

// ---------------------------------------------------------------------------------------
// One DEFLATE block at the reader.  Returns 0 / -E_*; last = BFINAL.
// ---------------------------------------------------------------------------------------
// RING: flush to HBM every half ring (ADLER: folding the Adler-32 sums; the stream mode);
// otherwise the whole output stays in the window.  W < 32 KiB: matches farther than the ring
// read their source from the output already flushed to HBM.
// CELL: the chained decode of dictionary streams -- the window and the output hold 16-bit
// cells; a match reaching before the sw block's first byte writes reference cells there.
template <bool RING, bool ADLER, uint32_t W, bool CELL = false>
__device__ __forceinline__ int iblock(InfLDS<W, typename std::conditional<CELL, uint16_t, uint8_t>::type>& S, IBits& r,
                                      IOut& o, uint32_t* __restrict__ gt, uint32_t lane, bool& last) {
    constexpr uint32_t IM = W - 1, FL = W / 2;
    constexpr uint32_t CS = CELL ? 2 : 1;   // bytes per output position
    [[maybe_unused]] const unsigned long long ts0 = IST_NOW();
    IST_ADD(o, 6, 1);
    last = ib_bits(r, 1) != 0;
    const uint32_t bt = ib_bits(r, 2);
    if (bt == 0) {   // stored
        ib_drop(r, r.bc & 7);
        const uint32_t len = ib_bits(r, 16), nlen = ib_bits(r, 16);
        if (len != (~nlen & 0xFFFFu)) return -(int)E_ZNLEN;
        if (len > io_caprel(o) - o.op) return -(int)E_SZ;
        const uint64_t src = ib_bytepos(r);   // relative to z
        if (src + len + r.lo > r.hi) return -(int)E_LEN;
        gu8* zs = r.zb + r.lo + src;
        for (uint32_t c0 = 0; c0 < len; c0 += FL) {   // pieces the ring can hold
            if (RING && o.op - o.fl > W - FL) io_flush<ADLER>(S, o, o.op, lane);
            const uint32_t ce = min(len, c0 + FL);
            for (uint32_t j = c0 + lane; j < ce; j += 64) S.win[(o.op + (j - c0)) & IM] = zs[j];
            o.op += ce - c0;
        }
        __syncthreads();
        ib_seek(r, (src + len) * 8);
        return 0;
    }
    if (bt == 3) return -(int)E_ZBTYPE;
    int nlen = 288, ndist = 30;
    if (bt == 1) {   // fixed codes
        for (int s = (int)lane; s < 320; s += 64)
            S.seq[s] = (uint8_t)(s < 144 ? 8 : s < 256 ? 9 : s < 280 ? 7 : s < 288 ? 8 : 5);
    } else {
        nlen = (int)ib_bits(r, 5) + 257;
        ndist = (int)ib_bits(r, 5) + 1;
        const int ncode = (int)ib_bits(r, 4) + 4;
        if (nlen > 286 || ndist > 30) return -(int)E_ZINV;
        if (lane < 19) S.len[lane] = 0;
        __syncthreads();
        for (int k = 0; k < ncode; k++) {
            const uint32_t v = ib_bits(r, 3);
            if (lane == 0) S.len[c_iclorder[k]] = (uint8_t)v;
        }
        __syncthreads();
        [[maybe_unused]] const unsigned long long tc0 = IST_NOW();
        if (itable_build<false>(S, S.lt, gt, 19, lane) != 0) return -(int)E_HUFAMB;
        [[maybe_unused]] const unsigned long long tc1 = IST_NOW();
        IST_ADD(o, 7, tc1 - tc0);
        uint32_t prev = 0;
        int idx = 0, err = 0;
        while (idx < nlen + ndist) {
            ib_refill(r);
            const uint32_t e = ientry_cl(r, S.lt, gt);
            if (e == ISLOW) { err = -(int)E_HUFINV; break; }
            ib_drop(r, e & 15u);
            const uint32_t sy = e >> 4;
            if (sy < 16) {
                if (lane == 0) S.seq[idx] = (uint8_t)sy;
                prev = sy;
                idx++;
            } else {
                uint32_t rep, v = 0;
                if (sy == 16) {
                    if (idx == 0) { err = -(int)E_ZINV; break; }
                    v = prev;
                    rep = 3 + ib_bits(r, 2);
                } else if (sy == 17) {
                    rep = 3 + ib_bits(r, 3);
                } else {
                    rep = 11 + ib_bits(r, 7);
                }
                if (idx + (int)rep > nlen + ndist) { err = -(int)E_ZINV; break; }
                for (uint32_t q = lane; q < rep; q += 64) S.seq[idx + q] = (uint8_t)v;
                prev = v;
                idx += (int)rep;
            }
        }
        if (err) return err;
        __syncthreads();
        if (rfl(S.seq[256]) == 0) return -(int)E_ZINV;
    }
    // literal/length table from seq[0, nlen), distance table from seq[nlen, nlen + ndist)
    for (int s = (int)lane; s < 288; s += 64) S.len[s] = s < nlen ? S.seq[s] : 0;
    __syncthreads();
    [[maybe_unused]] const unsigned long long tl0 = IST_NOW();
    IST_ADD(o, 8, tl0 - ts0);
    int e = itable_build<false>(S, S.lt, gt, nlen, lane);
    [[maybe_unused]] const unsigned long long tl1 = IST_NOW();
    IST_ADD(o, 9, tl1 - tl0);
    if (e < 0 || (e > 0 && bt == 2 && rfl(S.lt.offs[15] + S.lt.cnt[15]) != 1)) return -(int)E_HUFAMB;
    for (int s = (int)lane; s < 32; s += 64) S.len[s] = s < ndist ? S.seq[nlen + s] : 0;
    __syncthreads();
    e = itable_build<true>(S, S.dt, gt + (1u << IFB), ndist, lane);
    IST_ADD(o, 10, IST_NOW() - tl1);
    if (e < 0 || (e > 0 && bt == 2 && rfl(S.dt.offs[15] + S.dt.cnt[15]) > 1)) return -(int)E_HUFAMB;

    // symbols: the common path in isym_run (literals, lengths and distances with table codes,
    // matches inside the ring without overlap or with a period >= 64); the rest here.
    uint32_t op = o.op;
    uint32_t capr = io_caprel(o);
    int err = 0;
    [[maybe_unused]] const unsigned long long ts1 = IST_NOW();
    IST_ADD(o, 0, ts1 - ts0);
    if (lds_addr(S.win) != 0) return -(int)E_RANGE;   // isym_run addresses the ring from LDS 0
    const uint64_t tgl = (uint64_t)(uintptr_t)gt, tgd = tgl + 4 * (1u << IFB);   // the tables' words, 4 bytes a lane
    const uint32_t dfl = o.ob != 0 ? 0x40000000u : 0u;   // stream mode: sources before ob exist
    const uint64_t gpos0 = (uint64_t)(uintptr_t)(o.out + CS * (o.base + o.ob));
    // the run flushes half rings itself (no Adler sums; a 16-byte aligned output)
    const uint32_t fok = (uint32_t)__builtin_amdgcn_readfirstlane((RING && !ADLER && (gpos0 & 15) == 0) ? 1 : 0);
    // the literal/length table's canonical arrays (long codes inside the run; 16-byte aligned:
    // the ring before them is W positions)
    const uint32_t lta = (uint32_t)__builtin_amdgcn_readfirstlane((int)lds_addr(&S.lt));
    static_assert((W * CS) % 16 == 0 && sizeof(ITable) == 672, "the run's ITable offsets (dmx_isym.inc)");
    for (;;) {
        uint32_t lim = RING ? min(capr, o.fl + FL) : capr, fl = o.fl;
        uint32_t len, dist;
        const uint32_t ex = isym_run<W, CELL>(r, op, lim, fl, capr, fok, gpos0, dfl, lta, tgl, tgd, lane * 4, lane, gpos0,
                                              len, dist);
        o.fl = fl;
        IST_ADD(o, 5, 1);
        IST_ADD(o, 11, ex == IX_SYM ? 1 : 0);
        IST_ADD(o, 12, ex == IX_SEG ? 1 : 0);
        IST_ADD(o, 13, ex == IX_LIM ? 1 : 0);
        IST_ADD(o, 14, ex == IX_DIST ? 1 : 0);
        IST_ADD(o, 15, ex == IX_MATCH ? 1 : 0);
        if (ex == IX_SEG) {   // a refill at a token start that the run does not rotate into
            ib_refill(r);
            continue;
        }
        if (ex == IX_LIM && RING && op - o.fl >= FL) {
            o.op = op;
            io_flush<ADLER>(S, o, o.fl + FL, lane);
            op = o.op;
            capr = io_caprel(o);
            continue;
        }
        uint32_t en = 0;
        if (ex == IX_SYM || ex == IX_LIM) {   // one symbol the general way (nothing consumed)
            ib_refill(r);
            en = rfl(gtab_ld(gt + ib_peek(r, IFB)));
            if (en == IVSLOW) {
                const uint32_t e16 = ientry_slow(r, S.lt);
                if (e16 == ISLOW) { err = -(int)E_HUFINV; break; }
                en = iv_ll(e16);
            }
            if (!(en & 0x8000u)) {   // a literal: at the capacity limit, or a long code
                ib_drop(r, en & 31u);
                if (op >= capr) { err = -(int)E_SZ; break; }
                S.win[op & IM] = (uint8_t)(en >> 16);   // (a byte value in a cell, too)
                op++;
                continue;
            }
            if (en & 0x4000u) {
                ib_drop(r, en & 31u);
                if (en & 0x2000u) err = -(int)E_HUFVAL;
                break;   // end of block
            }
            len = (en >> 23) + iv_extra(r.bb, en);
            ib_drop(r, (en >> 8) & 31u);
        }
        if (ex != IX_MATCH) {   // the distance the general way
            ib_refill(r);
            uint32_t ed = rfl(gtab_ld(gt + (1u << IFB) + ib_peek(r, IFB)));
            if (ed >= IVBAD) {
                const uint32_t e16 = ed == IVSLOW ? ientry_slow(r, S.dt) : ISLOW;
                ed = e16 == ISLOW ? IVBAD : iv_d(e16);
                if (ed == IVBAD) { err = -(int)E_HUFVAL; break; }
            }
            dist = iv_dbase(ed) + iv_extra(r.bb, ed);
            ib_drop(r, (ed >> 8) & 31u);
        }
        if (o.ob == 0 && dist > op && (!CELL || dist - op > o.base)) { err = -(int)E_HUFDIS; break; }
        if (len > capr - op) { err = -(int)E_SZ; break; }
        if (RING && op - o.fl >= FL) {   // half the ring is due before this match
            o.op = op;
            io_flush<ADLER>(S, o, o.fl + FL, lane);
            op = o.op;
            capr = io_caprel(o);
        }
        const uint32_t src = op - dist;
        IST_ADD(o, 3, 1);
        if (CELL && dist > op) {   // (o.ob == 0 here) from before the sw block: reference cells
            const uintptr_t g = (uintptr_t)(o.out + CS * o.base);
            auto cell_at = [&](uint32_t t) -> uint32_t {   // output position op + t
                const int32_t sp = (int32_t)op - (int32_t)dist + (int32_t)t;
                if (sp < 0) return 0xFFu + (uint32_t)(-sp);   // 0x100 + (back - 1)
                if (t >= dist) return S.win[(op + t - dist) & IM];   // this match's own output
                if (W < IW && dist > W) {   // flushed: from the cell buffer
                    const uintptr_t a = g + CS * (uintptr_t)sp;
                    const uint32_t w = __hip_atomic_load((gu32*)(a & ~(uintptr_t)3), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
                    return (w >> (8 * (a & 3))) & 0xFFFFu;
                }
                return S.win[(uint32_t)sp & IM];
            };
            if (len <= dist) {
                for (uint32_t t = lane; t < len; t += 64) S.win[(op + t) & IM] = cell_at(t);
            } else {   // the match overlaps itself (rare): in order, one lane
                if (lane == 0)
                    for (uint32_t t = 0; t < len; t++) S.win[(op + t) & IM] = cell_at(t);
            }
            __syncthreads();
        } else if (W < IW && dist > W) {
            IST_ADD(o, 4, 1);
            // older than the ring: from the output in HBM, flushed before this match (op - fl
            // stays below W / 2 + 258, so every source byte lies below fl).  Agent-scope loads
            // go to L2, past any vector-L1 copy of a line that was flushed in two pieces.
            const uintptr_t g = (uintptr_t)(o.out + CS * (o.base + o.ob));
            for (uint32_t t = lane; t < len; t += 64) {
                const uintptr_t a = g + CS * (uintptr_t)(src + t);
                const uint32_t w = __hip_atomic_load((gu32*)(a & ~(uintptr_t)3), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
                S.win[(op + t) & IM] = CELL ? (w >> (8 * (a & 3))) & 0xFFFFu : (w >> (8 * (a & 3))) & 0xFFu;
            }
        } else if (dist >= 64 || dist >= len) {   // every read is of bytes written before its round
            for (uint32_t t = lane; t < len; t += 64) S.win[(op + t) & IM] = S.win[(src + t) & IM];
        } else {   // short period: byte t repeats byte t mod dist
            const float inv = 1.0f / (float)dist;
            for (uint32_t t = lane; t < len; t += 64) {
                int q = (int)((float)t * inv);
                int rm = (int)t - q * (int)dist;
                if (rm >= (int)dist) rm -= (int)dist;
                if (rm < 0) rm += (int)dist;
                S.win[(op + t) & IM] = S.win[(src + (uint32_t)rm) & IM];
            }
        }
        op += len;
    }
    o.op = op;
    IST_ADD(o, 1, IST_NOW() - ts1);
    if (err) return err;
    if (ib_over(r)) return -(int)E_LEN;
    return 0;
}

// CELL: out is the cell buffer (2 bytes a position), out_cap in positions
template <bool CELL>
__global__ __launch_bounds__(64) void dmx_inflate_index_kernel(const uint8_t* __restrict__ z, uint64_t zbytes,
                                                               const dmx_iblock* __restrict__ index,
                                                               uint8_t* __restrict__ out, uint64_t out_cap,
                                                               uint32_t* __restrict__ gtab,
                                                               dmx_inflate_status* __restrict__ st) {
    // bytes: an 8 KiB ring, 10 KiB of LDS; cells: 4 096 cells, the same 10 KiB.  12 workgroups
    // per CU (151 VGPRs: 3 waves per SIMD), so 3 072 blocks decode at once
    constexpr uint32_t WR = CELL ? IWC : IWX;
    __shared__ InfLDS<WR, typename std::conditional<CELL, uint16_t, uint8_t>::type> S;
    uint32_t* gt = gtab + (uint64_t)blockIdx.x * ITAB_WORDS;
    const uint32_t lane = threadIdx.x;
    IBits r;
    ib_init(r, z, zbytes);
    const uint64_t bit = rfl64(index[blockIdx.x].bit);
    const uint64_t off = rfl64(index[blockIdx.x].out_off);
    const uint32_t olen = rfl(index[blockIdx.x].out_len);
    IOut o;
#ifdef DMX_INF_STAMPS
    for (int k = 0; k < INF_NST; k++) o.st[k] = 0;
#endif
    o.out = out;
    o.base = off;
    o.ob = 0;
    o.cap = olen;
    o.op = 0;
    o.fl = 0;
    o.a = 1;
    o.b = 0;
    int err = 0;
    if (olen > IW || off + olen > out_cap || (bit >> 3) >= zbytes) err = -(int)E_RANGE;
    if (!err) {
        ib_seek(r, bit);
        bool last = false;
        do {   // one sw block may be several DEFLATE blocks (DMX_F_SPLIT)
            err = iblock<true, false, WR, CELL>(S, r, o, gt, lane, last);
        } while (!err && o.op < olen && !last);
        if (!err && o.op != olen) err = -(int)E_SZ;
        if (!err) io_flush<false>(S, o, o.op, lane);
    }
    if (lane == 0 && err) atomicCAS(&st->status, 0, err);
    if (lane == 0 && !err) atomicAdd((unsigned long long*)&st->out_len, (unsigned long long)o.op);
#ifdef DMX_INF_STAMPS
    if (lane < INF_NST && blockIdx.x < (1u << 16)) dmx_inf_st[blockIdx.x][lane] = o.st[lane];
#endif
}

__global__ __launch_bounds__(64) void dmx_inflate_stream_kernel(const uint8_t* __restrict__ z, uint64_t zbytes,
                                                                uint8_t* __restrict__ out, uint64_t out_cap,
                                                                uint32_t* __restrict__ gtab,
                                                                dmx_inflate_status* __restrict__ st) {
    __shared__ InfLDS<IW> S;
    const uint32_t lane = threadIdx.x;
    IBits r;
    ib_init(r, z, zbytes);
    IOut o;
#ifdef DMX_INF_STAMPS
    for (int k = 0; k < INF_NST; k++) o.st[k] = 0;
#endif
    o.out = out;
    o.base = 0;
    o.ob = 0;
    o.cap = out_cap;
    o.op = 0;
    o.fl = 0;
    o.a = 1;
    o.b = 0;
    int err = 0;
    if (zbytes < 6) err = -(int)E_ZHEAD;
    if (!err) {
        const uint32_t cmf = z[0], flg = z[1];
        if ((cmf & 0x0F) != 8) err = -(int)E_ZCMPMT;
        else if ((cmf >> 4) > 7) err = -(int)E_ZSLWIN;
        else if (((cmf << 8) | flg) % 31) err = -(int)E_ZFCHCK;
        else if (flg & 0x20) err = -(int)E_ZPDICT;
    }
    if (!err) {
        ib_seek(r, 16);
        bool last = false;
        while (!err && !last) err = iblock<true, true, IW>(S, r, o, gtab, lane, last);
    }
    if (!err) {
        io_flush<true>(S, o, o.op, lane);
        ib_drop(r, r.bc & 7);   // Adler-32 trailer, MSB first
        uint32_t want = 0;
        for (int k = 0; k < 4; k++) want = (want << 8) | ib_bits(r, 8);
        if (ib_over(r)) err = -(int)E_LEN;
        else if (((o.b << 16) | o.a) != want) err = -(int)E_ZADL32;
    }
    if (lane == 0) {
        if (err) atomicCAS(&st->status, 0, err);
        else st->out_len = o.ob + o.op;
    }
}

// ------------------------------------------------------------------------------------
// C ABI
// ------------------------------------------------------------------------------------

// Table scratch of dmx_inflate_async: a stream-ordered allocation from a private memory pool
// per device, freed on the same stream after the launch.  The pool keeps what it was given
// (release threshold = no limit), so a steady stream of decodes allocates from the pool's
// reserve, not from the driver, and any number of streams (created and destroyed per
// request, or the per-thread default stream) is safe: no buffer is shared between calls.
// (Round 4 cached one buffer per (device, stream handle): it failed past 64 streams, never
// released a slot, and a reused handle shared a buffer with a destroyed stream's work.)
#define ITAB_DEVS 64
static hipMemPool_t g_itab_pool[ITAB_DEVS];
static pthread_mutex_t g_itab_mu = PTHREAD_MUTEX_INITIALIZER;
static hipMemPool_t itab_pool(int dev) {
    if (dev < 0 || dev >= ITAB_DEVS) return nullptr;
    pthread_mutex_lock(&g_itab_mu);
    if (!g_itab_pool[dev]) {
        hipMemPoolProps pp;
        memset(&pp, 0, sizeof(pp));
        pp.allocType = hipMemAllocationTypePinned;
        pp.handleTypes = hipMemHandleTypeNone;
        pp.location.type = hipMemLocationTypeDevice;
        pp.location.id = dev;
        hipMemPool_t p = nullptr;
        if (hipMemPoolCreate(&p, &pp) == hipSuccess) {
            uint64_t keep = ~0ull;
            (void)hipMemPoolSetAttribute(p, hipMemPoolAttrReleaseThreshold, &keep);
            g_itab_pool[dev] = p;
        }
    }
    hipMemPool_t r = g_itab_pool[dev];
    pthread_mutex_unlock(&g_itab_mu);
    return r;
}
static uint32_t* itab_scratch(hipStream_t s, uint64_t bytes) {
    int dev = 0;
    if (hipGetDevice(&dev) != hipSuccess) return nullptr;
    void* p = nullptr;
    hipMemPool_t pool = itab_pool(dev);
    if (pool ? hipMallocFromPoolAsync(&p, bytes, pool, s) != hipSuccess : hipMallocAsync(&p, bytes, s) != hipSuccess)
        return nullptr;
    return (uint32_t*)p;
}

extern "C" int dmx_inflate_async(const void* d_z, uint64_t zbytes, const dmx_iblock* d_index, uint32_t nblk,
                                 void* d_out, uint64_t out_cap, dmx_inflate_status* d_status, void* stream) {
    if (!d_z || !d_out || !d_status || (d_index && !nblk)) return -(int)E_INVAL;
    if (zbytes > 0xFFFFFFF0ull) return -(int)E_RANGE;   // reader word indices are 32-bit
    hipStream_t s = (hipStream_t)stream;
    if (hipMemsetAsync(d_status, 0, sizeof(dmx_inflate_status), s) != hipSuccess) return -(int)E_DEVICE;
    // the workgroups' first-level tables: scratch from the per-device stream-ordered pool
    // (hipMallocFromPoolAsync here, hipFreeAsync on the same stream after the launch)
    const uint64_t tb = (uint64_t)(d_index ? nblk : 1) * ITAB_WORDS * 4;
    uint32_t* gtab = itab_scratch(s, tb);
    if (!gtab) return -(int)E_MALLOC;
    if (d_index)
        hipLaunchKernelGGL(dmx_inflate_index_kernel<false>, dim3(nblk), dim3(64), 0, s, (const uint8_t*)d_z, zbytes,
                           d_index, (uint8_t*)d_out, out_cap, gtab, d_status);
    else
        hipLaunchKernelGGL(dmx_inflate_stream_kernel, dim3(1), dim3(64), 0, s, (const uint8_t*)d_z, zbytes,
                           (uint8_t*)d_out, out_cap, gtab, d_status);
    const hipError_t le = hipGetLastError();
    (void)hipFreeAsync(gtab, s);   // stream-ordered: after the decode
    if (le != hipSuccess) return -(int)E_DEVICE;
    return 0;
}

// ------------------------------------------------------------------------------------
// Chained decode (dictionary streams, DMX_F_DICT: a block's matches may reach into the block
// before it).  Three steps, all blocks in parallel:
//   1. dmx_inflate_index_kernel<true>: every sw block decodes on its own into 16-bit cells; a
//      byte it cannot know yet (a match source before the block's first output byte, or a
//      copy of such a cell) becomes a reference cell 0x100 + b - 1 = the byte b positions
//      before the block's start.  Copies inside the block copy cells, so a reference always
//      names a byte of an EARLIER block.
//   2. dmx_cells_prep_kernel: each reference becomes an absolute source position s; a source
//      that is already a byte is copied at once, otherwise P[j] = s, the cell is marked
//      unresolved (0xFFFF) and j goes on its block's list (as a 16-bit offset in the block).  The lists are per block -- block
//      b's entries sit in [out_off, out_off + count) of a list buffer, so a workgroup appends
//      with one LDS atomic per wave and no global atomic at all.
//      dmx_cells_jump_kernel, about log2(nblk) + 2 launches of one workgroup per block, each
//      over the list the one before it left: an unresolved j looks at s = P[j]: a resolved
//      cell is copied; otherwise it follows up to CHAIN_HOPS - 1 more links s <- P[s] in the
//      same launch, and if none reaches a byte, P[j] = P[s] and j goes on the next list (pointer jumping:
//      chains of references through many blocks -- a run carried across every block, say --
//      halve each launch).  In place: a stale read only delays resolution, never changes the
//      value (P moves along the chain, a resolved cell stays).  A block whose list is empty
//      returns at once.
//   3. dmx_cells_final_kernel: cells -> bytes; any cell still unresolved is an error.
// ------------------------------------------------------------------------------------
#define CHAIN_ROUNDS_MAX 40
#define CHAIN_WG 1024   // threads per block in prep and jump: a block's list is latency-bound
#ifndef CHAIN_HOPS
#define CHAIN_HOPS 3    // links followed per list entry and jump launch (1: 16.1, 2: 18.1, 3: 18.4, 4: 18.2 GB/s, `profiles/r03_h`)
#endif
#ifndef CHAIN_ILP
#define CHAIN_ILP 2     // list entries per jump thread in flight (two links each: 2 beat 4, `profiles/r03_d3`)
#endif

// Appends v at list[*lds_cnt ...] for every lane with want set; the whole wave calls it.
__device__ inline void chain_push(bool want, uint32_t v, uint16_t* __restrict__ list, uint32_t* lds_cnt) {
    const uint64_t m = __ballot(want);
    if (!m) return;
    const int lead = __ffsll((unsigned long long)m) - 1;
    const uint32_t lane = threadIdx.x & 63;
    uint32_t base = 0;
    if ((int)lane == lead) base = atomicAdd(lds_cnt, (uint32_t)__popcll(m));
    base = __shfl(base, lead);
    if (want) list[base + __popcll(m & ((1ull << lane) - 1))] = (uint16_t)v;
}

__global__ __launch_bounds__(CHAIN_WG) void dmx_cells_prep_kernel(const dmx_iblock* __restrict__ index, uint16_t* cells,
                                                            uint32_t* P, uint16_t* __restrict__ list,
                                                            uint32_t* __restrict__ count, uint32_t* __restrict__ total,
                                                            uint64_t cap, dmx_inflate_status* __restrict__ st) {
    __shared__ uint32_t nl;
    const uint64_t off = index[blockIdx.x].out_off;
    const uint32_t len = index[blockIdx.x].out_len;
    if (off > cap || len > cap - off || len > IW) {   // the decode already failed this index; read nothing
        if (threadIdx.x == 0) {
            count[blockIdx.x] = 0;
            atomicCAS(&st->status, 0, -(int32_t)E_RANGE);
        }
        return;
    }
    if (threadIdx.x == 0) nl = 0;
    __syncthreads();
    bool bad = false;
    for (uint32_t j0 = 0; j0 < len; j0 += CHAIN_WG) {   // uniform trip count: chain_push needs the whole wave
        const uint32_t j = j0 + threadIdx.x;
        bool want = false;
        if (j < len) {
            const uint32_t c = cells[off + j];
            if (c >= 0x100u) {
                const uint64_t back = (uint64_t)(c - 0xFFu) + j;   // positions before j
                if (back > off + j) {
                    bad = true;
                } else {
                    const uint32_t sp = (uint32_t)(off + j - back);
                    // a byte cell never changes; a reference (raw or already marked) waits
                    const uint16_t cs = cells[sp];
                    if (cs < 0x100u) {
                        cells[off + j] = cs;
                    } else {
                        P[off + j] = sp;
                        cells[off + j] = 0xFFFFu;
                        want = true;
                    }
                }
            }
        }
        chain_push(want, j, list + off, &nl);   // block-relative: 2 bytes an entry
    }
    __syncthreads();
    if (threadIdx.x == 0) {
        count[blockIdx.x] = nl;
        if (nl) atomicAdd(total, nl);
    }
    if (bad) atomicCAS(&st->status, 0, -(int32_t)E_HUFDIS);
}

__global__ __launch_bounds__(CHAIN_WG) void dmx_cells_jump_kernel(const dmx_iblock* __restrict__ index, uint16_t* cells,
                                                                 uint32_t* P, const uint16_t* __restrict__ lin,
                                                                 uint16_t* __restrict__ lout, const uint32_t* __restrict__ cin,
                                                                 uint32_t* __restrict__ cout, uint32_t* __restrict__ total) {
    __shared__ uint32_t nl;
    const uint32_t cnt = cin[blockIdx.x];
    if (cnt == 0) {
        if (threadIdx.x == 0) cout[blockIdx.x] = 0;
        return;
    }
    const uint64_t off = index[blockIdx.x].out_off;
    if (threadIdx.x == 0) nl = 0;
    __syncthreads();
    // CHAIN_ILP entries per thread, their dependent loads (list, P, cell, P) interleaved
    for (uint32_t u0 = 0; u0 < cnt; u0 += CHAIN_ILP * CHAIN_WG) {
        uint32_t j[CHAIN_ILP], sp[CHAIN_ILP];
        uint16_t cs[CHAIN_ILP];
        bool act[CHAIN_ILP], want[CHAIN_ILP];
#pragma unroll
        for (int k = 0; k < CHAIN_ILP; k++) {
            const uint32_t u = u0 + k * CHAIN_WG + threadIdx.x;
            act[k] = u < cnt;
            j[k] = act[k] ? (uint32_t)(off + lin[off + u]) : 0;
        }
#pragma unroll
        for (int k = 0; k < CHAIN_ILP; k++) {
            sp[k] = act[k] ? P[j[k]] : 0;
            act[k] = act[k] && sp[k] < j[k];   // never otherwise from a well-formed prep: stays unresolved
        }
#pragma unroll
        for (int k = 0; k < CHAIN_ILP; k++)
            cs[k] = act[k] ? cells[sp[k]] : 0;   // (plain loads: a stale copy is an older link of the chain)
#if CHAIN_HOPS > 1
        // more links in the same launch: while the source is unresolved, step to its own source
        // (P[s] < s on a well-formed chain); a byte found resolves j now, otherwise j jumps to
        // the last source's P (CHAIN_HOPS links a launch)
        uint32_t cur[CHAIN_ILP];
        bool ok[CHAIN_ILP];
#pragma unroll
        for (int k = 0; k < CHAIN_ILP; k++) { cur[k] = sp[k]; ok[k] = true; }
#pragma unroll
        for (int h = 1; h < CHAIN_HOPS; h++) {
            uint32_t nx[CHAIN_ILP];
#pragma unroll
            for (int k = 0; k < CHAIN_ILP; k++) {
                nx[k] = (act[k] && ok[k] && cs[k] == 0xFFFFu) ? P[cur[k]] : 0u;
                if (act[k] && ok[k] && cs[k] == 0xFFFFu && nx[k] >= cur[k]) ok[k] = false;   // (malformed: stays)
            }
#pragma unroll
            for (int k = 0; k < CHAIN_ILP; k++)
                if (act[k] && ok[k] && cs[k] == 0xFFFFu) { cs[k] = cells[nx[k]]; cur[k] = nx[k]; }
        }
#pragma unroll
        for (int k = 0; k < CHAIN_ILP; k++) {
            want[k] = false;
            if (act[k]) {
                if (cs[k] != 0xFFFFu) {
                    cells[j[k]] = cs[k];
                } else {
                    P[j[k]] = ok[k] ? P[cur[k]] : cur[k];
                    want[k] = true;
                }
            }
        }
#else
#pragma unroll
        for (int k = 0; k < CHAIN_ILP; k++) {
            want[k] = false;
            if (act[k]) {
                if (cs[k] != 0xFFFFu) {
                    cells[j[k]] = cs[k];
                } else {
                    P[j[k]] = P[sp[k]];
                    want[k] = true;
                }
            }
        }
#endif
#pragma unroll
        for (int k = 0; k < CHAIN_ILP; k++) chain_push(want[k], (uint32_t)(j[k] - off), lout + off, &nl);
    }
    __syncthreads();
    if (threadIdx.x == 0) {
        cout[blockIdx.x] = nl;
        if (nl) atomicAdd(total, nl);
    }
}

// One workgroup per sw block: its own output range [out_off, out_off + out_len) of the index,
// cells -> bytes.  Positions of d_out the index does not cover are neither read nor written
// (out_cap is a capacity: the cell scratch past the decoded bytes was never initialised).
__global__ __launch_bounds__(256) void dmx_cells_final_kernel(const dmx_iblock* __restrict__ index,
                                                             const uint16_t* __restrict__ cells, uint8_t* __restrict__ out,
                                                             uint64_t cap, dmx_inflate_status* __restrict__ st) {
    const uint64_t off = index[blockIdx.x].out_off;
    const uint32_t len = index[blockIdx.x].out_len;
    if (off > cap || len > cap - off || len > IW) return;   // the decode already failed this index
    const uint64_t n = off + len;
    bool bad = false;
    // 16 positions per thread and step; the range's unaligned head and tail byte by byte
    const uint64_t a0 = min((off + 15) & ~15ull, n), a1 = max(a0, n & ~15ull);
    for (uint64_t j = off + threadIdx.x; j < a0; j += 256) {
        bad = bad || cells[j] > 0xFFu;
        out[j] = (uint8_t)cells[j];
    }
    for (uint64_t j = a1 + threadIdx.x; j < n; j += 256) {
        bad = bad || cells[j] > 0xFFu;
        out[j] = (uint8_t)cells[j];
    }
    if (((uintptr_t)out & 15) == 0) {
        for (uint64_t j0 = a0 + (uint64_t)threadIdx.x * 16; j0 < a1; j0 += 256 * 16) {
            const uint4 a = *reinterpret_cast<const uint4*>(cells + j0), b = *reinterpret_cast<const uint4*>(cells + j0 + 8);
            const uint32_t w[8] = {a.x, a.y, a.z, a.w, b.x, b.y, b.z, b.w};
            uint32_t o[4];
#pragma unroll
            for (int k = 0; k < 4; k++) {
                const uint32_t lo = w[2 * k], hi = w[2 * k + 1];
                bad = bad || ((lo | hi) & 0xFF00FF00u) != 0;
                o[k] = (lo & 0xFFu) | ((lo >> 8) & 0xFF00u) | ((hi & 0xFFu) << 16) | ((hi << 8) & 0xFF000000u);
            }
            *reinterpret_cast<uint4*>(out + j0) = make_uint4(o[0], o[1], o[2], o[3]);
        }
    } else {
        for (uint64_t j = a0 + threadIdx.x; j < a1; j += 256) {
            bad = bad || cells[j] > 0xFFu;
            out[j] = (uint8_t)cells[j];
        }
    }
    if (bad) atomicCAS(&st->status, 0, -(int32_t)E_HUFDIS);
}

// work layout: [list totals per round, 256 B][list lengths 2 x nblk, 256-aligned][tables ITAB_WORDS x nblk]
// [cells 2*cap, 256-aligned][P 4*cap][list A 2*cap][list B 2*cap] (list entries: 16-bit block-relative)
static inline uint64_t chain_a256(uint64_t x) { return (x + 255) & ~255ull; }

extern "C" uint64_t dmx_inflate_chained_work(uint64_t out_cap, uint32_t nblk) {
    return 256 + chain_a256(8ull * nblk) + 4ull * ITAB_WORDS * nblk + chain_a256(2 * out_cap) + 8 * out_cap;
}

// The reference lists' total lengths of the last chained decode on this work buffer: [0] after
// the prep kernel, [r + 1] after jump launch r (a diagnostic: how fast the chains resolve).
extern "C" int dmx_inflate_chained_lists(const void* d_work, uint32_t* host, uint32_t n, void* stream) {
    if (!d_work || !host || n > CHAIN_ROUNDS_MAX + 1) return -(int)E_INVAL;
    if (hipMemcpyAsync(host, d_work, 4ull * n, hipMemcpyDeviceToHost, (hipStream_t)stream) != hipSuccess ||
        hipStreamSynchronize((hipStream_t)stream) != hipSuccess)
        return -(int)E_DEVICE;
    return 0;
}

extern "C" int dmx_inflate_chained_async(const void* d_z, uint64_t zbytes, const dmx_iblock* d_index, uint32_t nblk,
                                         void* d_out, uint64_t out_cap, void* d_work, uint64_t work_bytes,
                                         dmx_inflate_status* d_status, void* stream) {
    if (!d_z || !d_out || !d_status || !d_index || !nblk || !d_work) return -(int)E_INVAL;
    if (zbytes > 0xFFFFFFF0ull || out_cap > 0xFFFFFFF0ull) return -(int)E_RANGE;   // 32-bit positions
    if (work_bytes < dmx_inflate_chained_work(out_cap, nblk) || ((uintptr_t)d_work & 255)) return -(int)E_SZ;
    hipStream_t s = (hipStream_t)stream;
    uint32_t* T = (uint32_t*)d_work;   // list totals per round
    uint32_t* C[2] = {T + 64, T + 64 + nblk};
    uint32_t* gtab = (uint32_t*)((uint8_t*)d_work + 256 + chain_a256(8ull * nblk));
    uint16_t* cells = (uint16_t*)(gtab + (uint64_t)ITAB_WORDS * nblk);
    uint32_t* P = (uint32_t*)((uint8_t*)cells + chain_a256(2 * out_cap));
    uint16_t* L[2] = {(uint16_t*)(P + out_cap), (uint16_t*)(P + out_cap) + out_cap};
    if (hipMemsetAsync(d_status, 0, sizeof(dmx_inflate_status), s) != hipSuccess) return -(int)E_DEVICE;
    if (hipMemsetAsync(T, 0, 256, s) != hipSuccess) return -(int)E_DEVICE;
    hipLaunchKernelGGL(dmx_inflate_index_kernel<true>, dim3(nblk), dim3(64), 0, s, (const uint8_t*)d_z, zbytes, d_index,
                       (uint8_t*)cells, out_cap, gtab, d_status);
    hipLaunchKernelGGL(dmx_cells_prep_kernel, dim3(nblk), dim3(CHAIN_WG), 0, s, d_index, cells, P, L[0], C[0], T, out_cap, d_status);
    uint32_t rounds = 2;   // pointer jumping: a chain through k blocks takes ~log2(k) + 1 rounds
    while ((1ull << (rounds - 2)) < (uint64_t)nblk && rounds < CHAIN_ROUNDS_MAX) rounds++;
    for (uint32_t rd = 0; rd < rounds; rd++)
        hipLaunchKernelGGL(dmx_cells_jump_kernel, dim3(nblk), dim3(CHAIN_WG), 0, s, d_index, cells, P, L[rd & 1],
                           L[(rd + 1) & 1], C[rd & 1], C[(rd + 1) & 1], T + rd + 1);
    hipLaunchKernelGGL(dmx_cells_final_kernel, dim3(nblk), dim3(256), 0, s, d_index, cells, (uint8_t*)d_out, out_cap,
                       d_status);
    if (hipGetLastError() != hipSuccess) return -(int)E_DEVICE;
    return 0;
}

#ifdef DMX_INF_STAMPS
// diagnostic builds: copy the per-workgroup phase totals of the last indexed launch
extern "C" int dmx_inflate_stamps(void* host, uint64_t bytes) {
    if (bytes > sizeof(dmx_inf_st)) bytes = sizeof(dmx_inf_st);
    return hipMemcpyFromSymbol(host, HIP_SYMBOL(dmx_inf_st), bytes, 0, hipMemcpyDeviceToHost) == hipSuccess ? 0 : -1;
}
#endif
