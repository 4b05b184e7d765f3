// dmx_inflate_dev.hip -- RFC 1950/1951 inflate on the MI355X.
//
// Two modes, one kernel:
//   * indexed: one workgroup (one wave) per DEFLATE block listed in a block index
//     {start bit, output offset, output length}.  Blocks of a dmx stream never reference
//     earlier blocks (every sw-sized block is its own window), so all blocks
//     decode in parallel; the encoder exports the index (dmx_block_index).
//   * stream: index == NULL, one workgroup decodes a whole zlib stream (header, blocks
//     until BFINAL, Adler-32 check) sequentially -- any RFC 1950 stream, e.g. PNG IDAT.
// Decoding is wave-uniform: every lane runs the same bit reader and table lookups, lane 0
// stores literals, the whole wave copies matches (rounds of min(dist, 64) bytes, so an
// overlapping source is always already written).  Output is assembled in a 32 KiB LDS
// window and written to HBM in coalesced chunks.  Tables: a 10-bit first-level lookup
// (len << 12 | sym) plus canonical counts for longer codes.
#include <hip/hip_runtime.h>
#include <stdint.h>
#include <stdio.h>

#include "../../include/dmx.h"

#define IW 32768          // window = LDS ring
#define IFB 10            // first-level table bits
#define IFLUSH 16384      // stream mode: flush to HBM every IFLUSH bytes

struct ITable {
    uint16_t fast[1 << IFB];   // (len << 12) | sym, 0 = longer than IFB
    uint16_t count[16];
    uint16_t sym[320];         // symbols sorted by (length, symbol)
};

struct InfLDS {
    uint8_t win[IW];
    ITable lt, dt;
    uint8_t len[320];
    uint16_t rev[320];
};

struct IBits {   // wave-uniform bit reader over the stream in global memory
    const uint8_t* z;
    uint64_t zbytes, pos;   // next byte to load
    uint64_t bb;
    uint32_t bc;
    bool over;
};

__device__ __forceinline__ void ib_refill(IBits& r) {
    while (r.bc <= 32) {
        uint32_t w;
        if (r.pos + 4 <= r.zbytes) {
            __builtin_memcpy(&w, r.z + r.pos, 4);
        } else {
            w = 0;
            for (uint32_t j = 0; j < 4; j++)
                if (r.pos + j < r.zbytes) w |= (uint32_t)r.z[r.pos + j] << (8 * j);
            if (r.pos + 4 > r.zbytes + 8) r.over = true;   // far past the end: corrupt stream
        }
        r.bb |= (uint64_t)w << r.bc;
        r.pos += 4;
        r.bc += 32;
    }
}
__device__ __forceinline__ uint32_t ib_bits(IBits& r, uint32_t n) {   // n <= 32
    if (n == 0) return 0;
    ib_refill(r);
    const uint32_t v = (uint32_t)(r.bb & ((1ull << n) - 1));
    r.bb >>= n;
    r.bc -= n;
    return v;
}
__device__ __forceinline__ void ib_align(IBits& r) {   // to a byte boundary
    const uint32_t d = r.bc & 7;
    r.bb >>= d;
    r.bc -= d;
}
__device__ __forceinline__ uint64_t ib_bitpos(const IBits& r) { return r.pos * 8 - r.bc; }

// Build a table from len[0..n): lane 0 sorts (counts, offsets, canonical codes), all
// lanes fill the first-level entries.  Returns 0 ok, <0 over-subscribed, >0 incomplete.
__device__ int itable_build(InfLDS& S, ITable& T, int n, uint32_t lane) {
    __shared__ int res;
    for (int k = (int)lane; k < (1 << IFB); k += 64) T.fast[k] = 0;
    if (lane == 0) {
        uint16_t offs[16];
        for (int l = 0; l < 16; l++) T.count[l] = 0;
        for (int s = 0; s < n; s++) T.count[S.len[s]]++;
        int left = 1, r = 0;
        for (int l = 1; l < 16; l++) {
            left <<= 1;
            left -= T.count[l];
            if (left < 0) { r = -1; break; }
        }
        if (r == 0) r = left;   // > 0: incomplete
        offs[1] = 0;
        for (int l = 1; l < 15; l++) offs[l + 1] = offs[l] + T.count[l];
        uint32_t code = 0;
        uint32_t next[16];
        for (int l = 1; l < 16; l++) { code = (code + (l > 1 ? T.count[l - 1] : 0)) << 1; next[l] = code; }
        for (int s = 0; s < n; s++) {
            const int l = S.len[s];
            if (!l) continue;
            T.sym[offs[l]++] = (uint16_t)s;
            const uint32_t c = next[l]++;
            S.rev[s] = (uint16_t)(__brev(c) >> (32 - l));
        }
        res = T.count[0] == n ? 0 : r;
    }
    __syncthreads();
    for (int s = (int)lane; s < n; s += 64) {
        const int l = S.len[s];
        if (l == 0 || l > IFB) continue;
        const uint32_t rv = S.rev[s];
        for (uint32_t k = 0; k < (1u << (IFB - l)); k++) T.fast[rv | (k << l)] = (uint16_t)((l << 12) | s);
    }
    __syncthreads();
    return res;
}

// One symbol (wave-uniform).  -1: invalid code.
__device__ __forceinline__ int isym(IBits& r, const ITable& T) {
    ib_refill(r);
    const uint32_t e = T.fast[r.bb & ((1u << IFB) - 1)];
    if (e) {
        const uint32_t l = e >> 12;
        r.bb >>= l;
        r.bc -= l;
        return (int)(e & 0xFFFu);
    }
    // canonical decode, one bit at a time (codes longer than IFB; rare)
    int code = 0, first = 0, index = 0;
    for (int l = 1; l < 16; l++) {
        code |= (int)(r.bb & 1u);
        r.bb >>= 1;
        r.bc -= 1;
        const int c = T.count[l];
        if (code - c < first) return T.sym[index + (code - first)];
        index += c;
        first += c;
        first <<= 1;
        code <<= 1;
    }
    return -1;
}

__constant__ uint16_t c_lbase[29] = {3, 4, 5, 6, 7, 8, 9, 10, 11, 13, 15, 17, 19, 23, 27, 31,
                                     35, 43, 51, 59, 67, 83, 99, 115, 131, 163, 195, 227, 258};
__constant__ uint8_t c_lext[29] = {0, 0, 0, 0, 0, 0, 0, 0, 1, 1, 1, 1, 2, 2, 2, 2, 3, 3, 3, 3, 4, 4, 4, 4, 5, 5, 5, 5, 0};
__constant__ uint16_t c_dbase[30] = {1, 2, 3, 4, 5, 7, 9, 13, 17, 25, 33, 49, 65, 97, 129, 193, 257, 385,
                                     513, 769, 1025, 1537, 2049, 3073, 4097, 6145, 8193, 12289, 16385, 24577};
__constant__ uint8_t c_dext[30] = {0, 0, 0, 0, 1, 1, 2, 2, 3, 3, 4, 4, 5, 5, 6, 6, 7, 7, 8, 8, 9, 9, 10, 10, 11, 11, 12, 12, 13, 13};
__constant__ uint8_t c_iclorder[19] = {16, 17, 18, 0, 8, 7, 9, 6, 10, 5, 11, 4, 12, 3, 13, 2, 14, 1, 15};

// Output state of one workgroup: op = bytes produced (absolute), fl = bytes flushed to HBM.
struct IOut {
    uint8_t* out;
    uint64_t base, cap, op, fl;
    bool ring;   // stream mode: the window wraps and is flushed as it fills
};

__device__ __forceinline__ void io_flush(InfLDS& S, IOut& o, uint64_t upto, uint32_t lane) {
    for (uint64_t p = o.fl + lane; p < upto; p += 64) o.out[o.base + p] = S.win[p & (IW - 1)];
    o.fl = upto;
    __syncthreads();
}

// Decode the symbols of one Huffman block.  Returns 0 or -E_*.
__device__ int icodes(InfLDS& S, IBits& r, IOut& o, uint32_t lane, bool fixed_dist) {
    for (;;) {
        const int sy = isym(r, S.lt);
        if (sy < 0) return -(int)E_HUFINV;
        if (sy < 256) {
            if (o.op >= o.cap) return -(int)E_SZ;
            if (lane == 0) S.win[o.op & (IW - 1)] = (uint8_t)sy;
            o.op++;
        } else if (sy == 256) {
            return 0;
        } else {
            const int li = sy - 257;
            if (li >= 29) return -(int)E_HUFVAL;
            const uint32_t len = c_lbase[li] + ib_bits(r, c_lext[li]);
            int ds;
            if (fixed_dist) ds = (int)(__brev(ib_bits(r, 5)) >> 27);
            else ds = isym(r, S.dt);
            if (ds < 0 || ds >= 30) return -(int)E_HUFVAL;
            const uint32_t dist = c_dbase[ds] + ib_bits(r, c_dext[ds]);
            if (dist > o.op || dist > IW) return -(int)E_HUFDIS;
            if (o.op + len > o.cap) return -(int)E_SZ;
            const uint32_t step = dist < 64 ? dist : 64;
            __builtin_amdgcn_wave_barrier();
            for (uint32_t t = 0; t < len; t += step) {
                const uint32_t m = min(step, len - t);
                if (lane < m) {
                    const uint64_t d = o.op + t + lane;
                    S.win[d & (IW - 1)] = S.win[(d - dist) & (IW - 1)];
                }
                __builtin_amdgcn_wave_barrier();
            }
            o.op += len;
        }
        if (o.ring && o.op - o.fl >= IFLUSH) io_flush(S, o, o.fl + IFLUSH, lane);
        if (r.over) return -(int)E_LEN;
    }
}

// One DEFLATE block at the reader.  Returns 0 / -E_*; *last = BFINAL.
__device__ int iblock(InfLDS& S, IBits& r, IOut& o, uint32_t lane, bool* last) {
    *last = ib_bits(r, 1) != 0;
    const uint32_t bt = ib_bits(r, 2);
    if (bt == 0) {   // stored
        ib_align(r);
        const uint32_t len = ib_bits(r, 16), nlen = ib_bits(r, 16);
        if (len != (~nlen & 0xFFFFu)) return -(int)E_ZNLEN;
        if (o.op + len > o.cap) return -(int)E_SZ;
        // bytes still in the bit buffer first, then straight from the stream
        uint32_t k = 0;
        while (k < len && r.bc >= 8) {
            if (lane == 0) S.win[(o.op + k) & (IW - 1)] = (uint8_t)(r.bb & 0xFFu);
            r.bb >>= 8;
            r.bc -= 8;
            k++;
        }
        __builtin_amdgcn_wave_barrier();
        if (k < len) {   // the bit buffer is empty now: copy the rest from memory
            const uint64_t src = r.pos;
            if (src + (len - k) > r.zbytes) return -(int)E_LEN;
            for (uint32_t c0 = k; c0 < len; c0 += IFLUSH) {   // pieces the ring can hold
                if (o.ring) io_flush(S, o, o.op + c0, lane);
                const uint32_t ce = min(len, c0 + (uint32_t)IFLUSH);
                for (uint32_t j = c0 + lane; j < ce; j += 64) S.win[(o.op + j) & (IW - 1)] = r.z[src + (j - k)];
                __syncthreads();
            }
            r.pos = src + (len - k);
            r.bb = 0;
            r.bc = 0;
        }
        o.op += len;
        return 0;
    }
    if (bt == 1) {   // fixed codes
        for (int s = (int)lane; s < 288; s += 64) S.len[s] = (uint8_t)(s < 144 ? 8 : s < 256 ? 9 : s < 280 ? 7 : 8);
        __syncthreads();
        itable_build(S, S.lt, 288, lane);
        return icodes(S, r, o, lane, true);
    }
    if (bt != 2) return -(int)E_ZBTYPE;
    const int nlen = (int)ib_bits(r, 5) + 257, ndist = (int)ib_bits(r, 5) + 1, ncode = (int)ib_bits(r, 4) + 4;
    if (nlen > 286 || ndist > 30) return -(int)E_ZINV;
    for (int s = (int)lane; s < 19; s += 64) S.len[s] = 0;
    __syncthreads();
    uint32_t clv[19];
    for (int k = 0; k < ncode; k++) clv[k] = ib_bits(r, 3);
    if (lane == 0)
        for (int k = 0; k < ncode; k++) S.len[c_iclorder[k]] = (uint8_t)clv[k];
    __syncthreads();
    if (itable_build(S, S.lt, 19, lane) != 0) return -(int)E_HUFAMB;
    // code lengths with runs (wave-uniform decode, lane 0 stores)
    uint8_t lens_prev = 0;
    int idx = 0;
    __shared__ uint8_t seq[320];
    while (idx < nlen + ndist) {
        const int sy = isym(r, S.lt);
        if (sy < 0) return -(int)E_HUFINV;
        if (sy < 16) {
            if (lane == 0) seq[idx] = (uint8_t)sy;
            lens_prev = (uint8_t)sy;
            idx++;
        } else {
            uint32_t rep;
            uint8_t v = 0;
            if (sy == 16) {
                if (idx == 0) return -(int)E_ZINV;
                v = lens_prev;
                rep = 3 + ib_bits(r, 2);
            } else if (sy == 17) {
                rep = 3 + ib_bits(r, 3);
            } else {
                rep = 11 + ib_bits(r, 7);
            }
            if (idx + (int)rep > nlen + ndist) return -(int)E_ZINV;
            for (uint32_t q = lane; q < rep; q += 64) seq[idx + q] = v;
            lens_prev = v;
            idx += (int)rep;
        }
        __builtin_amdgcn_wave_barrier();
    }
    __syncthreads();
    for (int s = (int)lane; s < 288; s += 64) S.len[s] = s < nlen ? seq[s] : 0;
    __syncthreads();
    if (S.len[256] == 0) return -(int)E_ZINV;
    int e = itable_build(S, S.lt, nlen, lane);
    if (e < 0 || (e > 0 && nlen - S.lt.count[0] != 1)) return -(int)E_HUFAMB;
    for (int s = (int)lane; s < 30; s += 64) S.len[s] = s < ndist ? seq[nlen + s] : 0;
    __syncthreads();
    e = itable_build(S, S.dt, ndist, lane);
    if (e < 0 || (e > 0 && ndist - S.dt.count[0] != 1)) return -(int)E_HUFAMB;
    return icodes(S, r, o, lane, false);
}

__global__ __launch_bounds__(64) void dmx_inflate_kernel(const uint8_t* __restrict__ z, uint64_t zbytes,
                                                         const dmx_iblock* __restrict__ index, uint32_t nblk,
                                                         uint8_t* __restrict__ out, uint64_t out_cap,
                                                         dmx_inflate_status* __restrict__ st) {
    __shared__ InfLDS S;
    const uint32_t lane = threadIdx.x;
    IBits r;
    r.z = z;
    r.zbytes = zbytes;
    r.bb = 0;
    r.bc = 0;
    r.over = false;
    IOut o;
    o.out = out;
    o.op = 0;
    o.fl = 0;
    int err = 0;
    if (index) {   // one DEFLATE block per workgroup, no history
        const dmx_iblock ix = index[blockIdx.x];
        if (ix.out_len > IW || ix.out_off + ix.out_len > out_cap) err = -(int)E_RANGE;
        r.pos = ix.bit >> 3;
        o.base = ix.out_off;
        o.cap = ix.out_len;
        o.ring = false;
        if (!err) {
            ib_bits(r, (uint32_t)(ix.bit & 7));
            bool last;
            err = iblock(S, r, o, lane, &last);
            if (!err && o.op != ix.out_len) err = -(int)E_SZ;
            if (!err) io_flush(S, o, o.op, lane);
        }
        if (lane == 0 && err) atomicCAS(&st->status, 0, err);
        if (lane == 0 && !err) atomicAdd((unsigned long long*)&st->out_len, (unsigned long long)o.op);
        return;
    }
    // whole zlib stream in this workgroup
    o.base = 0;
    o.cap = out_cap;
    o.ring = true;
    r.pos = 0;
    if (zbytes < 6) err = -(int)E_ZHEAD;
    if (!err) {
        const uint32_t cmf = z[0], flg = z[1];
        if ((cmf & 0x0F) != 8) err = -(int)E_ZCMPMT;
        else if ((cmf >> 4) > 7) err = -(int)E_ZSLWIN;
        else if (((cmf << 8) | flg) % 31) err = -(int)E_ZFCHCK;
        else if (flg & 0x20) err = -(int)E_ZPDICT;
    }
    r.pos = 2;
    bool last = false;
    while (!err && !last) err = iblock(S, r, o, lane, &last);
    if (!err) io_flush(S, o, o.op, lane);
    if (!err) {   // Adler-32 trailer (RFC 1950, MSB first) over the output in HBM
        ib_align(r);
        uint32_t want = 0;
        for (int k = 0; k < 4; k++) want = (want << 8) | ib_bits(r, 8);
        // per-lane sums over interleaved 4 KiB pieces, combined in order by lane 0
        __shared__ unsigned long long ps[64], pt[64];
        const uint64_t n = o.op;
        const uint64_t piece = 4096;
        uint32_t a = 1, bsum = 0;
        for (uint64_t p0 = 0; p0 < n; p0 += 64 * piece) {
            const uint64_t lo = p0 + lane * piece, hi = min(n, lo + piece);
            uint64_t s = 0, t = 0;
            for (uint64_t p = lo; p < hi; p++) { s += out[p]; t += (uint64_t)(hi - p) * out[p]; }
            ps[lane] = s;
            pt[lane] = t;
            __syncthreads();
            if (lane == 0) {
                for (uint32_t l = 0; l < 64; l++) {
                    const uint64_t plo = p0 + l * piece, phi = min(n, plo + piece);
                    if (plo >= n) break;
                    const uint64_t len = phi - plo;
                    // a' = a + s, b' = b + len * a + t   (mod 65521)
                    bsum = (uint32_t)((bsum + (len % 65521) * a + (pt[l] % 65521)) % 65521);
                    a = (uint32_t)((a + ps[l] % 65521) % 65521);
                }
            }
            __syncthreads();
        }
        if (lane == 0 && ((bsum << 16) | a) != want) err = -(int)E_ZADL32;
    }
    if (lane == 0) {
        if (err) atomicCAS(&st->status, 0, err);
        else st->out_len = o.op;
    }
}

// ------------------------------------------------------------------------------------
// C ABI
// ------------------------------------------------------------------------------------

extern "C" int dmx_inflate_async(const void* d_z, uint64_t zbytes, const dmx_iblock* d_index, uint32_t nblk,
                                 void* d_out, uint64_t out_cap, dmx_inflate_status* d_status, void* stream) {
    if (!d_z || !d_out || !d_status || (d_index && !nblk)) return -(int)E_INVAL;
    hipStream_t s = (hipStream_t)stream;
    if (hipMemsetAsync(d_status, 0, sizeof(dmx_inflate_status), s) != hipSuccess) return -(int)E_DEVICE;
    const uint32_t grid = d_index ? nblk : 1u;
    hipLaunchKernelGGL(dmx_inflate_kernel, dim3(grid), dim3(64), 0, s, (const uint8_t*)d_z, zbytes, d_index, nblk,
                       (uint8_t*)d_out, out_cap, d_status);
    if (hipGetLastError() != hipSuccess) return -(int)E_DEVICE;
    return 0;
}
