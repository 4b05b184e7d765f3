// dmx_ctx.h -- the encoder context (dmx_ctx) and the host helpers shared by the HIP layer
// (dmx_kernels.hip: kernels, launches, context management) and its host-only pipeline code
// (dmx_fd.cpp: the cached per-device contexts, dmx_encode_host, the fd streaming paths).
// C++ only, internal.
#ifndef DMX_CTX_H
#define DMX_CTX_H

#include <hip/hip_runtime_api.h>
#include <stddef.h>
#include <stdint.h>

#include "dmx_internal.h"
#include "../../include/dmx.h"

#ifndef DMX_STAMPS
#define DMX_STAMPS 16   // diagnostic u64 stamps per block (DMX_STAMPS=1 in the environment)
#endif

struct ScanTile;   // (dmx_kernels.hip)
struct FdPipe;     // (dmx_fd.cpp)

#define DMX_EV_RING 32

struct dmx_ctx {
    int device;
    hipStream_t stream;
    uint64_t cap_blocks;
    uint16_t* dist;   // cap_blocks * DMX_BLK: best distances in bucket order (match kernel staging)
    uint32_t* tok;    // cap_blocks * DMX_BLK
    uint32_t* hist;   // cap_blocks * DMX_HIST
    uint32_t* codes;  // cap_blocks * DMX_HIST
    uint32_t* hdr;    // cap_blocks * DMX_NSUB * DMX_HDR_WORDS
    dmx_subinfo* sub; // cap_blocks * DMX_NSUB
    dmx_blkinfo* info;
    ScanTile* tiles;  // cap_blocks / SCAN_TILE + 1: per-tile aggregates and prefixes (scan)
    uint32_t* wl;     // WL_HDR + 3 cap_blocks: the work lists of DMX_F_STORE_CHECK (WL_* comment)
    volatile uint32_t* whint;   // host-mapped pinned {nblk, |L1|, |L2|, |L4|, uniform full blocks} of the latest encode (WL_HINT)
    uint32_t* whint_dev;        // its device address (the scan kernel writes it when an encode runs without the lists)
    uint32_t ncu;     // compute units (the persistent K1 grid of the work-list mode)
    dmx_result* res;
    uint32_t* nfb;        // [0] sort fallbacks of the encode in flight (kernels add, K3's scan reads and zeroes), [1] total
    uint64_t* dbg;        // optional per-block phase stamps (DMX_STAMPS=1)
    uint64_t dbg_cap;
    // last encode (introspection)
    uint32_t last_nblk;
    uint32_t last_sw;
    // host staging for dmx_encode_host
    void* d_in;
    uint64_t d_in_cap;
    void* d_out;
    uint64_t d_out_cap;
    void* d_dict;         // DMX_F_DICT history of block 0 (DMX_BLK bytes)
    // dmx_encode_fd streaming buffers, kept across calls (pinning ~100 MB costs ms)
    uint8_t* fd_hin[2];   // pinned input chunks
    uint8_t* fd_hout[2];  // pinned output chunks
    void* fd_din[2];      // device input chunks (the previous one is the next chunk's history);
                          // DMX_BLK bytes in front of the chunk hold a multi-GPU worker's history
    void* fd_dout[2];     // device output chunks (a multi-GPU worker copies one while encoding into the other)
    dmx_result* fd_hres[2];  // pinned
    hipStream_t fd_cs;    // multi-GPU worker: D2H copies beside the next encode
    hipEvent_t fd_ev[2];  // multi-GPU worker: encode i done
    uint64_t fd_chunk, fd_ocap;
    struct FdPipe* fdp;   // dmx_encode_fd's pipeline buffers (single device)
    uint16_t* chs;        // DMX_F_DICT: (cap_chain) x DMX_BLK bucket-sorted positions per block (+ the dict)
    uint16_t* che;        // DMX_F_DICT: (cap_chain) x DMX_NBUCKET bucket ends
    uint64_t cap_chain;
    void* split;          // DMX_F_SPLIT: cap_split x SplitScratch (per-block plans of the 10 groups)
    uint64_t cap_split;
    uint32_t want;        // DMX_F_SPLIT / DMX_F_DICT: scratch kept reserved with the workspace
    // timing: a ring of event sets so timed encodes never block the host
    int timing;       // bit k: record event k (set_timing: 1 = all six, 0x100 | s = stage s's two)
    hipEvent_t ev[DMX_EV_RING][6];
    int ev_used[DMX_EV_RING];
    uint32_t ev_next;
    uint32_t ev_every, ev_count;   // with a one-stage mask: events on every ev_every-th encode only
    double stage_ms[6];
    uint32_t stage_n;
    // test hooks (dmx_ctx_set_hook; defaults from the environment, read once at creation):
    int hk_wl;       // -1 adaptive launch shapes, 0 no work lists, 1 list shapes, 2 per-block shapes (DMX_WORKLIST)
    int hk_dedupe;   // -1 adaptive, 0 / 1 the uniform-block dedupe forced off / on (DMX_DEDUPE)
    int hk_scan3;    // 1: K3 in three launches at any size (DMX_SCAN3)
};

#define DMX_HIDDEN __attribute__((visibility("hidden")))
// device / pinned allocations through the fault injection of dmx_fault_set (dmx_kernels.hip)
DMX_HIDDEN bool fault_hit(int kind);
DMX_HIDDEN hipError_t dmx_malloc(void** p, size_t n);
DMX_HIDDEN hipError_t dmx_host_malloc(void** p, size_t n);
template <typename T>
static inline hipError_t dmx_malloc(T** p, size_t n) { return dmx_malloc(reinterpret_cast<void**>(p), n); }
// prints the failing call and returns 1 on an error
DMX_HIDDEN int hip_fail(hipError_t e, const char* what);
#define HIPCHK(x) do { if (hip_fail((x), #x)) return -(int)E_DEVICE; } while (0)
// the fd pipeline's buffers of a context (dmx_fd.cpp), freed with the context
DMX_HIDDEN void fdp_free(FdPipe* P);

#endif
