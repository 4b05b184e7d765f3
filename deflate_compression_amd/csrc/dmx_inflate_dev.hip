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
// The decoder is wave-uniform and lives in scalar registers: the 64-bit bit buffer, the
// stream word index and the output position are SGPRs (table entries come back through
// readfirstlane), the stream is read with scalar loads, and the whole decode is one inlined
// loop -- no calls, no scratch.  Lane 0 stores literals; a match is copied by the whole wave
// from the periodic extension of its source (byte i of a match at distance d is the byte at
// op - d + i mod d), so every lane reads data that existed before the match and a match of
// up to 258 bytes is at most five independent LDS read/write rounds.  Output is assembled
// in a 32 KiB LDS window and written to HBM in 16-byte-per-lane coalesced stores (stream
// mode flushes every 16 KiB and folds the Adler-32 sums into the same pass).
// Tables: 10-bit first-level lookup of 16-bit entries (symbol << 4 | code length); codes
// longer than 10 bits take a canonical slow path (first code / count / offset per length).
#include <hip/hip_runtime.h>
#include <stdint.h>
#include <stdio.h>

#include "../../include/dmx.h"

#define IW 32768          // window = LDS ring
#define IM (IW - 1)
#define IFB 10            // first-level table bits
#define IFLUSH 16384      // stream mode: flush to HBM every IFLUSH bytes

struct ITable {
    uint16_t fast[1 << IFB];   // sym << 4 | len; ISLOW = code longer than IFB (or none)
    uint16_t first[16];        // first canonical code of each length
    uint16_t cnt[16];
    uint16_t offs[16];         // index into sym[] of the first symbol of each length
    uint16_t sym[288];         // symbols sorted by (length, symbol)
};

struct InfLDS {
    uint8_t win[IW];
    ITable lt, dt;
    uint8_t len[320];
    uint8_t seq[320];
};

__device__ __forceinline__ uint32_t rfl(uint32_t v) { return __builtin_amdgcn_readfirstlane(v); }
__device__ __forceinline__ uint64_t rfl64(uint64_t v) {
    return ((uint64_t)rfl((uint32_t)(v >> 32)) << 32) | rfl((uint32_t)v);
}

// ---------------------------------------------------------------------------------------
// Bit reader.  Coordinates are relative to the dword-aligned address at or below z, so the
// fast refill is one aligned scalar dword load; words that are not wholly inside the
// stream go through the byte path (zeros past the end, counted as overrun).
// ---------------------------------------------------------------------------------------
typedef __attribute__((address_space(4))) const uint32_t cu32;   // constant space: scalar loads

struct IBits {
    cu32* w;
    const uint8_t* zb;     // aligned base as bytes
    uint32_t lo, hi;       // valid byte range [lo, hi) relative to zb
    uint32_t wi, wfast;    // next word; words < wfast are wholly inside the stream
    uint32_t bc;
    uint64_t bb;
    bool over;
};

__device__ __forceinline__ uint32_t ib_word(IBits& r, uint32_t wi) {
    if (wi < r.wfast) return r.w[wi];
    uint32_t v = 0;
    for (uint32_t j = 0; j < 4; j++) {
        const uint32_t b = wi * 4 + j;
        if (b >= r.lo && b < r.hi) v |= (uint32_t)r.zb[b] << (8 * j);
    }
    if (wi * 4 >= r.hi + 8) r.over = true;
    return rfl(v);
}
__device__ __forceinline__ void ib_refill(IBits& r) {   // afterwards bc >= 32
    if (r.bc <= 32) {
        r.bb |= (uint64_t)ib_word(r, r.wi) << r.bc;
        r.wi++;
        r.bc += 32;
    }
}
__device__ __forceinline__ void ib_seek(IBits& r, uint64_t bit) {   // bit: relative to z
    const uint64_t ab = bit + (uint64_t)r.lo * 8;
    r.wi = (uint32_t)(ab >> 5);
    r.bb = (uint64_t)ib_word(r, r.wi) >> (ab & 31);
    r.bc = 32 - (uint32_t)(ab & 31);
    r.wi++;
}
__device__ __forceinline__ void ib_init(IBits& r, const uint8_t* z, uint64_t zbytes) {
    const uintptr_t a = (uintptr_t)z;
    r.zb = (const uint8_t*)(a & ~(uintptr_t)3);
    r.w = (cu32*)r.zb;
    r.lo = (uint32_t)(a & 3);
    r.hi = r.lo + (uint32_t)zbytes;
    r.wfast = r.hi >> 2;
    r.over = false;
    r.wi = 0;
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

// ---------------------------------------------------------------------------------------
// Huffman tables.  Lane l (1..15) owns code length l: it counts its symbols, then assigns
// their canonical codes in symbol order and fills their first-level entries.  Entries are
// sym << 4 | len; ISLOW marks a code longer than IFB bits (or no code), so "literal" is the
// single test e < 256 << 4.  Returns 0 complete, 1 incomplete, -1 over-subscribed.
// ---------------------------------------------------------------------------------------
#define ISLOW 0xFFFFu
#define ILIT (256u << 4)

__device__ __forceinline__ int itable_build(InfLDS& S, ITable& T, int n, uint32_t lane) {
    for (int k = (int)lane; k < (1 << IFB); k += 64) T.fast[k] = (uint16_t)ISLOW;
    uint32_t c = 0;
    if (lane >= 1 && lane < 16)
        for (int s = 0; s < n; s++) c += S.len[s] == lane;
    // Kraft check, first codes and offsets (uniform, unrolled)
    int left = 1, res = 0;
    uint32_t code = 0, off = 0, firstl = 0, offl = 0, cprev = 0;
    for (int l = 1; l < 16; l++) {
        const uint32_t cl = rfl(__builtin_amdgcn_readlane(c, l));
        left = 2 * left - (int)cl;
        if (left < 0) res = -1;
        code = (code + cprev) << 1;
        if ((uint32_t)l == lane) { firstl = code; offl = off; }
        if (lane == 0) {
            T.first[l] = (uint16_t)code;
            T.cnt[l] = (uint16_t)cl;
            T.offs[l] = (uint16_t)off;
        }
        off += cl;
        cprev = cl;
    }
    if (res == 0 && left > 0) res = 1;
    if (off == 0) res = 1;   // no codes at all
    __syncthreads();
    if (res >= 0 && lane >= 1 && lane < 16 && c) {
        uint32_t k = 0;
        for (int s = 0; s < n; s++) {
            if (S.len[s] != lane) continue;
            T.sym[offl + k] = (uint16_t)s;
            if (lane <= IFB) {
                const uint32_t rv = __brev(firstl + k) >> (32 - lane);
                const uint16_t e = (uint16_t)((s << 4) | lane);
                for (uint32_t j = 0; j < (1u << (IFB - lane)); j++) T.fast[rv | (j << lane)] = e;
            }
            k++;
        }
    }
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
__device__ __forceinline__ uint32_t ientry(const IBits& r, const ITable& T) {
    const uint32_t e = rfl(T.fast[ib_peek(r, IFB)]);
    return e != ISLOW ? e : ientry_slow(r, T);
}

// DEFLATE length / distance bases by arithmetic (RFC 1951 3.2.5), no table loads.
__device__ __forceinline__ uint32_t len_extra(uint32_t li) { return li < 8 || li == 28 ? 0 : (li - 4) >> 2; }
__device__ __forceinline__ uint32_t len_base(uint32_t li) {
    return li < 8 ? li + 3 : li == 28 ? 258 : ((4 + (li & 3)) << ((li - 4) >> 2)) + 3;
}
__device__ __forceinline__ uint32_t dist_extra(uint32_t d) { return d < 4 ? 0 : (d - 2) >> 1; }
__device__ __forceinline__ uint32_t dist_base(uint32_t d) { return d < 4 ? d + 1 : ((2 + (d & 1)) << ((d - 2) >> 1)) + 1; }

__constant__ uint8_t c_iclorder[19] = {16, 17, 18, 0, 8, 7, 9, 6, 10, 5, 11, 4, 12, 3, 13, 2, 14, 1, 15};

// ---------------------------------------------------------------------------------------
// Output.  Positions are 32-bit and relative to ob (a multiple of IW, so the window index
// of a position is pos & IM); stream mode moves ob forward as it flushes.
// ---------------------------------------------------------------------------------------
struct IOut {
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

// Write window bytes [fl, upto) to HBM (upto - fl <= IW).  ADLER: fold them into (a, b).
template <bool ADLER>
__device__ __forceinline__ void io_flush(InfLDS& S, IOut& o, uint32_t upto, uint32_t lane) {
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
    if (o.fl >= IRENORM) {   // keep relative positions small (ob stays a multiple of IW)
        o.ob += IRENORM;
        o.op -= IRENORM;
        o.fl -= IRENORM;
    }
    __syncthreads();
}

// ---------------------------------------------------------------------------------------
// One DEFLATE block at the reader.  Returns 0 / -E_*; last = BFINAL.
// ---------------------------------------------------------------------------------------
template <bool RING>
__device__ __forceinline__ int iblock(InfLDS& S, IBits& r, IOut& o, uint32_t lane, bool& last) {
    last = ib_bits(r, 1) != 0;
    const uint32_t bt = ib_bits(r, 2);
    if (bt == 0) {   // stored
        ib_drop(r, r.bc & 7);
        const uint32_t len = ib_bits(r, 16), nlen = ib_bits(r, 16);
        if (len != (~nlen & 0xFFFFu)) return -(int)E_ZNLEN;
        if (len > io_caprel(o) - o.op) return -(int)E_SZ;
        const uint64_t src = ib_bytepos(r);   // relative to z
        if (src + len + r.lo > r.hi) return -(int)E_LEN;
        const uint8_t* zs = r.zb + r.lo + src;
        for (uint32_t c0 = 0; c0 < len; c0 += IFLUSH) {   // pieces the ring can hold
            if (RING && o.op - o.fl > IW - IFLUSH) io_flush<true>(S, o, o.op, lane);
            const uint32_t ce = min(len, c0 + (uint32_t)IFLUSH);
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
        if (itable_build(S, S.lt, 19, lane) != 0) return -(int)E_HUFAMB;
        uint32_t prev = 0;
        int idx = 0, err = 0;
        while (idx < nlen + ndist) {
            ib_refill(r);
            const uint32_t e = ientry(r, S.lt);
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
    int e = itable_build(S, S.lt, nlen, lane);
    if (e < 0 || (e > 0 && bt == 2 && rfl(S.lt.offs[15] + S.lt.cnt[15]) != 1)) return -(int)E_HUFAMB;
    for (int s = (int)lane; s < 32; s += 64) S.len[s] = s < ndist ? S.seq[nlen + s] : 0;
    __syncthreads();
    e = itable_build(S, S.dt, ndist, lane);
    if (e < 0 || (e > 0 && bt == 2 && rfl(S.dt.offs[15] + S.dt.cnt[15]) > 1)) return -(int)E_HUFAMB;

    // symbols.  The inner loop is the literal run: one lookup, one compare, one byte store.
    uint32_t op = o.op;
    uint32_t capr = io_caprel(o);
    int err = 0;
    for (;;) {
        const uint32_t lim = RING ? min(capr, o.fl + IFLUSH) : capr;
        uint32_t en;
        for (;;) {
            ib_refill(r);
            en = rfl(S.lt.fast[ib_peek(r, IFB)]);
            if (en >= ILIT || op >= lim) break;
            ib_drop(r, en & 15u);
            if (lane == 0) S.win[op & IM] = (uint8_t)(en >> 4);
            op++;
        }
        if (RING && op - o.fl >= IFLUSH) {
            o.op = op;
            io_flush<true>(S, o, o.fl + IFLUSH, lane);
            op = o.op;
            capr = io_caprel(o);
            continue;
        }
        if (en == ISLOW) en = ientry_slow(r, S.lt);
        if (en == ISLOW) { err = -(int)E_HUFINV; break; }
        ib_drop(r, en & 15u);
        const uint32_t sy = en >> 4;
        if (sy < 256) {   // a literal at the capacity limit
            if (op >= capr) { err = -(int)E_SZ; break; }
            if (lane == 0) S.win[op & IM] = (uint8_t)sy;
            op++;
            continue;
        }
        if (sy == 256) break;
        const uint32_t li = sy - 257;
        if (li >= 29) { err = -(int)E_HUFVAL; break; }
        const uint32_t len = len_base(li) + ib_bits(r, len_extra(li));
        ib_refill(r);
        const uint32_t ed = ientry(r, S.dt);
        const uint32_t ds = ed >> 4;
        if (ed == ISLOW || ds >= 30) { err = -(int)E_HUFVAL; break; }
        ib_drop(r, ed & 15u);
        const uint32_t dist = dist_base(ds) + ib_bits(r, dist_extra(ds));
        if (o.ob == 0 && dist > op) { err = -(int)E_HUFDIS; break; }
        if (len > capr - op) { err = -(int)E_SZ; break; }
        const uint32_t src = op - dist;
        if (dist >= 64 || dist >= len) {   // every read is of bytes written before its round
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
    if (err) return err;
    if (r.over) return -(int)E_LEN;
    return 0;
}

__global__ __launch_bounds__(64) void dmx_inflate_index_kernel(const uint8_t* __restrict__ z, uint64_t zbytes,
                                                               const dmx_iblock* __restrict__ index,
                                                               uint8_t* __restrict__ out, uint64_t out_cap,
                                                               dmx_inflate_status* __restrict__ st) {
    __shared__ InfLDS S;
    const uint32_t lane = threadIdx.x;
    IBits r;
    ib_init(r, z, zbytes);
    const uint64_t bit = rfl64(index[blockIdx.x].bit);
    const uint64_t off = rfl64(index[blockIdx.x].out_off);
    const uint32_t olen = rfl(index[blockIdx.x].out_len);
    IOut o;
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
            err = iblock<false>(S, r, o, lane, last);
        } while (!err && o.op < olen && !last);
        if (!err && o.op != olen) err = -(int)E_SZ;
        if (!err) io_flush<false>(S, o, o.op, lane);
    }
    if (lane == 0 && err) atomicCAS(&st->status, 0, err);
    if (lane == 0 && !err) atomicAdd((unsigned long long*)&st->out_len, (unsigned long long)o.op);
}

__global__ __launch_bounds__(64) void dmx_inflate_stream_kernel(const uint8_t* __restrict__ z, uint64_t zbytes,
                                                                uint8_t* __restrict__ out, uint64_t out_cap,
                                                                dmx_inflate_status* __restrict__ st) {
    __shared__ InfLDS S;
    const uint32_t lane = threadIdx.x;
    IBits r;
    ib_init(r, z, zbytes);
    IOut o;
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
        while (!err && !last) err = iblock<true>(S, r, o, lane, last);
    }
    if (!err) {
        io_flush<true>(S, o, o.op, lane);
        ib_drop(r, r.bc & 7);   // Adler-32 trailer, MSB first
        uint32_t want = 0;
        for (int k = 0; k < 4; k++) want = (want << 8) | ib_bits(r, 8);
        if (r.over) err = -(int)E_LEN;
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

extern "C" int dmx_inflate_async(const void* d_z, uint64_t zbytes, const dmx_iblock* d_index, uint32_t nblk,
                                 void* d_out, uint64_t out_cap, dmx_inflate_status* d_status, void* stream) {
    if (!d_z || !d_out || !d_status || (d_index && !nblk)) return -(int)E_INVAL;
    if (zbytes > 0xFFFFFFF0ull) return -(int)E_RANGE;   // reader word indices are 32-bit
    hipStream_t s = (hipStream_t)stream;
    if (hipMemsetAsync(d_status, 0, sizeof(dmx_inflate_status), s) != hipSuccess) return -(int)E_DEVICE;
    if (d_index)
        hipLaunchKernelGGL(dmx_inflate_index_kernel, dim3(nblk), dim3(64), 0, s, (const uint8_t*)d_z, zbytes,
                           d_index, (uint8_t*)d_out, out_cap, d_status);
    else
        hipLaunchKernelGGL(dmx_inflate_stream_kernel, dim3(1), dim3(64), 0, s, (const uint8_t*)d_z, zbytes,
                           (uint8_t*)d_out, out_cap, d_status);
    if (hipGetLastError() != hipSuccess) return -(int)E_DEVICE;
    return 0;
}
