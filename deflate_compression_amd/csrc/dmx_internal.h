/* dmx_internal.h -- layouts shared by the HIP layer (dmx_kernels.hip) and the C host
 * code (dmx_host.c).  See DESIGN.md §2 for the HBM layout. */
#ifndef DMX_INTERNAL_H
#define DMX_INTERNAL_H

#include <stdint.h>

#define DMX_BLK 32768          /* max block size = LZ77 window (RFC 1951 §2) */
#define DMX_HASH_SHIFT 19      /* 13-bit bucket: (trigram * 0x9E3779B1) >> 19 */
#define DMX_NBUCKET 8192
#define DMX_NONE16 0xFFFFu     /* end of a hash chain */
#define DMX_HIST 320           /* per-block histogram stride: 286 lit/len + 30 dist (+pad) */
#define DMX_DIST0 286          /* first distance slot in hist / code tables */
#define DMX_HDR_WORDS 160      /* per-block header bit buffer (<= 4.5 kbit dynamic header) */
#define DMX_STAGE_WORDS 8224   /* pack staging: 32768*8+42+81 bits rounded up, in u32 */

/* Per-block record, one per sw-sized input block (64 B). */
typedef struct {
    uint32_t ntok;      /* match kernel: tokens in the block */
    uint32_t n;         /* block length in bytes */
    uint64_t adl_s;     /* sum of bytes */
    uint64_t adl_w;     /* sum of (n - k) * byte[k] */
    uint32_t btype;     /* huff kernel: 0 stored, 1 fixed, 2 dynamic */
    uint32_t hdr_bits;  /* bits of the block header (3-bit BFINAL/BTYPE + dynamic trees) */
    uint64_t body_bits; /* bits of the coded tokens + EOB (fixed/dynamic) */
    uint64_t off_bits;  /* scan kernel: absolute bit offset of the block in the output */
    uint64_t len_bits;  /* scan kernel: bits the block occupies (stored: incl. padding) */
    uint32_t nsub;      /* huff kernel: DEFLATE blocks emitted for this block (1..4, f3 split) */
    uint32_t prestored; /* store-check kernel (DMX_F_STORE_CHECK): 1 = stored without a parse,
                         * 2 = one repeated byte, parsed in closed form; 0 = parsed by K1 */
} dmx_blkinfo;

/* One emitted DEFLATE block inside an sw block (DMX_NSUB per block; f3 split). */
#define DMX_NSUB 4
typedef struct {
    uint32_t t0, t1;    /* token range [t0, t1) */
    uint32_t btype;     /* 1 fixed, 2 dynamic (a stored block is never split) */
    uint32_t hdr_bits;  /* header bits incl. the 3-bit BFINAL/BTYPE */
    uint64_t body_bits; /* coded tokens + extra bits + EOB */
} dmx_subinfo;

/* DMX_DEVICES parsed ("0,1,2,3" or "all"): entries written to devs, 0 if unset, -E_INVAL. */
#ifdef __cplusplus
extern "C" {
#endif
int dmx_devices_from_env(int* devs, int cap);
#ifdef __cplusplus
}
#endif

#endif
