// dmx_fd.cpp -- host-only part of the HIP layer (C ABI): the cached per-device contexts,
// dmx_encode_host (host buffers through HBM), the single-device fd pipeline of
// deflate_compress (dmx_encode_fd / dmx_encode_fd_cb), the multi-GPU fd path
// (dmx_encode_fd_multi, §6) and dmx_debug_stamps.  No device code: built with the host
// compiler against the HIP runtime API (and into the ASan/UBSan host build, tests/c).
#include <pthread.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>

#include "dmx_ctx.h"

// --- host-buffer convenience on a cached context per device ---

#include <pthread.h>
// Guards the cached per-device contexts (dmx_encode_host, dmx_encode_fd, the fd API).
// Recursive: deflate_compress with fd_stats holds it across the encode and the token
// introspection that follows (dmx_cached_lock / dmx_cached_unlock), so no other caller's
// encode lands in between.
static pthread_mutex_t g_mu = PTHREAD_RECURSIVE_MUTEX_INITIALIZER_NP;
extern "C" void dmx_cached_lock(void) { pthread_mutex_lock(&g_mu); }
extern "C" void dmx_cached_unlock(void) { pthread_mutex_unlock(&g_mu); }
static dmx_ctx* g_ctx[64];

extern "C" dmx_ctx* dmx_cached_ctx(int device, uint64_t max_input, int* err) {
    *err = 0;
    if (device < 0 || device >= 64) { *err = -(int)E_RANGE; return NULL; }
    if (!g_ctx[device]) {
        int r = dmx_ctx_create(device, max_input, &g_ctx[device]);
        if (r) { *err = r; return NULL; }
    }
    return g_ctx[device];
}

static int ensure_buf(void** p, uint64_t* cap, uint64_t need) {
    if (*cap >= need && *p) return 0;
    if (*p) (void)hipFree(*p);
    *p = NULL;
    *cap = 0;
    HIPCHK(dmx_malloc(p, need ? need : 16));
    *cap = need;
    return 0;
}

extern "C" int dmx_encode_host(const uint8_t* in, uint64_t n, uint8_t* out, uint64_t out_cap, uint64_t* out_len,
                               const dmx_opts* opts) {
    dmx_opts o = {0, 0, DMX_ZLIB, 0, NULL, 0};
    if (opts) o = *opts;
    if (o.sw == 0) o.sw = DMX_BLK;
    if (o.sw < 1 || o.sw > DMX_BLK) return -(int)E_RANGE;
    const char* dev_s = getenv("DMX_DEVICE");
    const int dev = dev_s ? atoi(dev_s) : 0;
    pthread_mutex_lock(&g_mu);
    int err = 0;
    dmx_ctx* c = dmx_cached_ctx(dev, n, &err);
    int r = err;
    if (!r) {
        r = dmx_ctx_reserve_flags(c, n, o.sw, o.flags);
    }
    const uint64_t dcap = dmx_max_compressed(n, o.sw);
    if (!r) r = ensure_buf(&c->d_in, &c->d_in_cap, n + 16);
    if (!r) r = ensure_buf(&c->d_out, &c->d_out_cap, dcap);
    if (!r && hip_fail(hipSetDevice(c->device), "hipSetDevice")) r = -(int)E_DEVICE;
    if (!r && n && hip_fail(hipMemcpyAsync(c->d_in, in, n, hipMemcpyHostToDevice, c->stream), "H2D")) r = -(int)E_DEVICE;
    if (!r && (o.flags & DMX_F_DICT) && o.dict && o.dict_len) {   // host dictionary -> device
        const uint64_t dl = o.dict_len < (uint64_t)o.sw ? o.dict_len : (uint64_t)o.sw;
        if (!c->d_dict && hip_fail(dmx_malloc(&c->d_dict, DMX_BLK), "hipMalloc(dict)")) r = -(int)E_DEVICE;
        if (!r && hip_fail(hipMemcpyAsync(c->d_dict, (const uint8_t*)o.dict + (o.dict_len - dl), dl,
                                          hipMemcpyHostToDevice, c->stream), "H2D(dict)")) r = -(int)E_DEVICE;
        o.dict = c->d_dict;
        o.dict_len = dl;
    }
    if (!r) r = dmx_encode_async(c, c->d_in, n, c->d_out, c->d_out_cap, &o, NULL);
    dmx_result res;
    if (!r) r = dmx_encode_result(c, &res, NULL);
    if (!r && res.status) r = res.status;
    if (!r && res.out_len > out_cap) r = -(int)E_SZ;
    if (!r && hip_fail(hipMemcpy(out, c->d_out, res.out_len, hipMemcpyDeviceToHost), "D2H")) r = -(int)E_DEVICE;
    if (!r) *out_len = res.out_len;
    pthread_mutex_unlock(&g_mu);
    return r;
}

// --- streaming file-in/file-out (the fd API without per-token stats) ---
// The input is read in chunks of `chunk` bytes (a multiple of sw) straight into pinned
// buffers; chunk i is copied to the device and encoded while the host reads chunk i+1
// (several pread threads when fd_in is a regular file) and a writer thread writes chunk
// i-1's stream (writes stay in order: writer i starts after writer i-1 has ended).  Every
// chunk is a shard of one zlib stream (DESIGN.md §6 framing): the header on the first, a
// sync flush after every chunk that is not known to be the last (the file size, or a
// one-byte lookahead on pipes, tells), BFINAL on the last, and the Adler-32 combined on the
// host.  With DMX_F_DICT the previous chunk's last sw bytes (still in HBM) are the history
// of each chunk's first block, so the parse equals the one-shot parse.  One chunk:
// byte-identical to dmx_encode_host.  Pinned and device buffers live in the cached context.
#include <unistd.h>
#include <errno.h>
#include <sys/stat.h>
#include <time.h>
static int64_t read_full(int fd, uint8_t* b, uint64_t cap) {
    uint64_t len = 0;
    while (len < cap) {
        const ssize_t r = read(fd, b + len, cap - len);
        if (r < 0) {
            if (errno == EINTR) continue;
            return -(int64_t)E_NEXIST;
        }
        if (r == 0) break;
        len += (uint64_t)r;
    }
    return (int64_t)len;
}
static int write_full(int fd, const uint8_t* p, uint64_t n) {
    while (n) {
        const ssize_t w = write(fd, p, n);
        if (w < 0) {
            if (errno == EINTR) continue;
            return -(int)E_PIPE;
        }
        p += w;
        n -= (uint64_t)w;
    }
    return 0;
}

// Reader: a regular file of known size is read with FD_READERS parallel preads per chunk;
// anything else (pipes) with read() and a one-byte lookahead.
#define FD_READERS 8
struct FdReader {
    int fd;
    bool seekable;
    uint64_t off, size;   // seekable: next file offset, file size
    int carry;            // pipes: the lookahead byte (-1: none)
    bool eof;             // no byte after the chunk just read
};
struct PreadJob {
    int fd;
    uint8_t* b;
    uint64_t off, len;
    int rc;
};
static void* pread_job(void* a) {
    PreadJob* j = (PreadJob*)a;
    uint64_t done = 0;
    j->rc = 0;
    while (done < j->len) {
        const ssize_t r = pread(j->fd, j->b + done, j->len - done, (off_t)(j->off + done));
        if (r < 0) {
            if (errno == EINTR) continue;
            j->rc = -(int)E_NEXIST;
            return NULL;
        }
        if (r == 0) break;
        done += (uint64_t)r;
    }
    if (done < j->len) j->rc = -(int)E_NEXIST;   // the file shrank under us
    return NULL;
}
// The reader's pread helpers: FD_READERS - 1 threads started once per process (on the first
// chunk read) and woken per chunk, instead of FD_READERS - 1 pthread_create / join per chunk.
// Used by one reader at a time (dmx_encode_fd's, under g_mu).
struct PreadPool {
    pthread_mutex_t mu = PTHREAD_MUTEX_INITIALIZER;
    pthread_cond_t work = PTHREAD_COND_INITIALIZER, done = PTHREAD_COND_INITIALIZER;
    uint64_t gen = 0;
    int pending = 0, nth = 0;
    PreadJob* jobs = nullptr;
    int njobs = 0;
};
static PreadPool g_pp;
struct PreadWorker { int idx; };
static PreadWorker g_ppw[FD_READERS];
static void* pread_worker(void* a) {
    const int idx = ((PreadWorker*)a)->idx;
    uint64_t seen = 0;
    for (;;) {
        pthread_mutex_lock(&g_pp.mu);
        while (g_pp.gen == seen) pthread_cond_wait(&g_pp.work, &g_pp.mu);
        seen = g_pp.gen;
        PreadJob* j = idx < g_pp.njobs ? &g_pp.jobs[idx] : nullptr;
        pthread_mutex_unlock(&g_pp.mu);
        if (j) pread_job(j);
        pthread_mutex_lock(&g_pp.mu);
        if (--g_pp.pending == 0) pthread_cond_signal(&g_pp.done);
        pthread_mutex_unlock(&g_pp.mu);
    }
    return NULL;
}
// a forked child has none of the pool's threads: it starts its own on its first read
static void pread_pool_atfork_child() {
    pthread_mutex_init(&g_pp.mu, NULL);
    pthread_cond_init(&g_pp.work, NULL);
    pthread_cond_init(&g_pp.done, NULL);
    g_pp.gen = 0;
    g_pp.pending = 0;
    g_pp.nth = 0;
}
// jobs[0] runs on the calling thread, jobs[1..nj) on the pool (inline where it has no thread)
static void pread_run(PreadJob* jobs, int nj) {
    static bool atfork = false;
    if (!atfork) atfork = pthread_atfork(NULL, NULL, pread_pool_atfork_child) == 0;
    if (g_pp.nth == 0) {   // start the pool (threads that fail to start leave their jobs inline)
        for (int k = 1; k < FD_READERS; k++) {
            g_ppw[k].idx = k;
            pthread_t t;
            pthread_attr_t at;
            pthread_attr_init(&at);
            pthread_attr_setdetachstate(&at, PTHREAD_CREATE_DETACHED);
            const bool ok = pthread_create(&t, &at, pread_worker, &g_ppw[k]) == 0;
            pthread_attr_destroy(&at);
            if (!ok) break;
            g_pp.nth = k;
        }
        if (g_pp.nth == 0) g_pp.nth = -1;   // no threads: everything inline
    }
    const int nth = g_pp.nth > 0 ? g_pp.nth : 0;   // workers 1..nth
    if (nth) {
        pthread_mutex_lock(&g_pp.mu);
        g_pp.jobs = jobs;
        g_pp.njobs = nj < nth + 1 ? nj : nth + 1;
        g_pp.pending = nth;
        g_pp.gen++;
        pthread_cond_broadcast(&g_pp.work);
        pthread_mutex_unlock(&g_pp.mu);
    }
    if (nj > 0) pread_job(&jobs[0]);
    for (int k = nth + 1; k < nj; k++) pread_job(&jobs[k]);   // jobs without a worker
    if (nth) {
        pthread_mutex_lock(&g_pp.mu);
        while (g_pp.pending > 0) pthread_cond_wait(&g_pp.done, &g_pp.mu);
        pthread_mutex_unlock(&g_pp.mu);
    }
}

static int64_t fd_read_chunk(FdReader* R, uint8_t* b, uint64_t chunk) {
    if (R->seekable) {
        const uint64_t left = R->size - R->off, len = left < chunk ? left : chunk;
        const uint64_t piece = ((len + FD_READERS - 1) / FD_READERS + 4095) & ~4095ull;
        PreadJob jobs[FD_READERS];
        int nj = 0;
        for (uint64_t o = 0; o < len; o += piece, nj++)
            jobs[nj] = {R->fd, b + o, R->off + o, (len - o) < piece ? (len - o) : piece, 0};
#ifdef DMX_FD_SPAWN   // (A/B build: a thread per piece per chunk, as before round 5)
        pthread_t th[FD_READERS];
        bool started[FD_READERS] = {};
        for (int k = 1; k < nj; k++) {
            if (pthread_create(&th[k], NULL, pread_job, &jobs[k]) == 0) started[k] = true;
            else pread_job(&jobs[k]);
        }
        if (nj > 0) pread_job(&jobs[0]);
        for (int k = 1; k < nj; k++)
            if (started[k]) pthread_join(th[k], NULL);
#else
        pread_run(jobs, nj);
#endif
        int rc = 0;
        for (int k = 0; k < nj; k++)
            if (jobs[k].rc) rc = jobs[k].rc;
        if (rc) return rc;
        R->off += len;
        R->eof = R->off >= R->size;
        return (int64_t)len;
    }
    uint64_t off = 0;
    if (R->carry >= 0) b[off++] = (uint8_t)R->carry;
    const int64_t r = read_full(R->fd, b + off, chunk - off);
    if (r < 0) return r;
    const uint64_t len = off + (uint64_t)r;
    R->carry = -1;
    R->eof = true;
    if (len == chunk) {
        uint8_t nb;
        const int64_t q = read_full(R->fd, &nb, 1);
        if (q < 0) return q;
        if (q == 1) {
            R->carry = nb;
            R->eof = false;
        }
    }
    return (int64_t)len;
}

static int fd_buffers(dmx_ctx* c, uint64_t chunk, uint64_t ocap) {
    if (c->fd_chunk >= chunk && c->fd_ocap >= ocap) return 0;
    for (int k = 0; k < 2; k++) {
        if (c->fd_hin[k]) (void)hipHostFree(c->fd_hin[k]);
        if (c->fd_hout[k]) (void)hipHostFree(c->fd_hout[k]);
        if (c->fd_din[k]) (void)hipFree(c->fd_din[k]);
        if (c->fd_dout[k]) (void)hipFree(c->fd_dout[k]);
        c->fd_hin[k] = c->fd_hout[k] = NULL;
        c->fd_din[k] = c->fd_dout[k] = NULL;
    }
    c->fd_chunk = c->fd_ocap = 0;
    for (int k = 0; k < 2; k++) {   // input buffers: DMX_BLK bytes of history room + the chunk
        if (hip_fail(dmx_host_malloc((void**)&c->fd_hin[k], chunk + DMX_BLK + 16), "hipHostMalloc")) return -(int)E_MALLOC;
        if (hip_fail(dmx_host_malloc((void**)&c->fd_hout[k], ocap), "hipHostMalloc")) return -(int)E_MALLOC;
        if (hip_fail(dmx_malloc(&c->fd_din[k], chunk + DMX_BLK + 16), "hipMalloc")) return -(int)E_DEVICE;
        if (hip_fail(dmx_malloc(&c->fd_dout[k], ocap), "hipMalloc")) return -(int)E_DEVICE;
        if (!c->fd_hres[k] && hip_fail(dmx_host_malloc((void**)&c->fd_hres[k], sizeof(dmx_result)), "hipHostMalloc"))
            return -(int)E_MALLOC;
        if (!c->fd_ev[k] && hip_fail(hipEventCreateWithFlags(&c->fd_ev[k], hipEventDisableTiming), "hipEventCreate")) {
            c->fd_ev[k] = NULL;
            return -(int)E_DEVICE;
        }
    }
    if (!c->fd_cs && hip_fail(hipStreamCreateWithFlags(&c->fd_cs, hipStreamNonBlocking), "hipStreamCreate")) {
        c->fd_cs = NULL;
        return -(int)E_DEVICE;
    }
    c->fd_chunk = chunk;
    c->fd_ocap = ocap;
    return 0;
}

// --- the single-device fd path (dmx_encode_fd): a five-stage pipeline ---
// reader thread   chunk j of fd_in -> pinned input slot j % nin (FD_READERS parallel preads
//                 on a regular file), running ahead of the device;
// H2D stream      slot -> device input j % FDP_NDIN;
// encode stream   the context's stream: encode j (its history, with DMX_F_DICT, is the previous
//                 device input's tail) -> device output j % 2, result -> pinned record j % 2;
// D2H stream      device output -> pinned output slot j % nout, as soon as the host has
//                 read the chunk's length (the next chunk is already encoding);
// writer thread   slots to fd_out in order.
// The chunks are shards of one zlib stream (header on the first, a sync flush after every
// chunk but the last, BFINAL on the last; Adler-32 combined here), so the stream is
// byte-identical to the sequential loop's.  A chunk callback (the compress_stats writer)
// makes the loop serial: chunk j's tokens are read from the context before j + 1 encodes.
#define FDP_NIN 3
#define FDP_NOUT 3
#define FDP_NDIN 3
// Pinned host memory: (nin + nout) x chunk, 6 x DMX_CHUNK_MB at most.  Chunks above
// FDP_BIG_CHUNK take 2 + 2 slots, and when pinning 3 + 3 fails the pipeline retries with
// 2 + 2 (the round-3 footprint) before reporting -E_MALLOC.
#define FDP_BIG_CHUNK (256ull << 20)
struct FdPipe {
    uint64_t chunk, ocap;
    int nin, nout;              // pinned slots in use (FDP_NIN / FDP_NOUT, or 2 each, fdp_get)
    uint8_t* hin[FDP_NIN];      // pinned input slots
    uint8_t* hout[FDP_NOUT];    // pinned output slots
    void* din[FDP_NDIN];        // device input chunks
    void* dout[2];              // device output chunks
    dmx_result* hres[2];        // pinned result records
    hipStream_t sh, sd;         // H2D and D2H streams
    hipEvent_t evh[FDP_NIN];    // H2D from input slot k done
    hipEvent_t eve[2];          // encode j (and its result copy) done
    hipEvent_t evd[2];          // D2H from device output k done
    hipEvent_t evo[FDP_NOUT];   // D2H into output slot k done
    hipEvent_t th[FDP_NIN], te[2], td[FDP_NOUT];   // stage timing: H2D / encode / D2H begins
};

void fdp_free(FdPipe* P) {
    if (!P) return;
    for (int k = 0; k < FDP_NIN; k++) {
        if (P->hin[k]) (void)hipHostFree(P->hin[k]);
        if (P->evh[k]) (void)hipEventDestroy(P->evh[k]);
        if (P->th[k]) (void)hipEventDestroy(P->th[k]);
    }
    for (int k = 0; k < FDP_NOUT; k++) {
        if (P->hout[k]) (void)hipHostFree(P->hout[k]);
        if (P->evo[k]) (void)hipEventDestroy(P->evo[k]);
        if (P->td[k]) (void)hipEventDestroy(P->td[k]);
    }
    for (int k = 0; k < FDP_NDIN; k++)
        if (P->din[k]) (void)hipFree(P->din[k]);
    for (int k = 0; k < 2; k++) {
        if (P->dout[k]) (void)hipFree(P->dout[k]);
        if (P->hres[k]) (void)hipHostFree(P->hres[k]);
        if (P->eve[k]) (void)hipEventDestroy(P->eve[k]);
        if (P->evd[k]) (void)hipEventDestroy(P->evd[k]);
        if (P->te[k]) (void)hipEventDestroy(P->te[k]);
    }
    if (P->sh) (void)hipStreamDestroy(P->sh);
    if (P->sd) (void)hipStreamDestroy(P->sd);
    free(P);
}

// The context's pipeline buffers for chunks of `chunk` bytes (kept across calls: pinning
// ~100 MB costs milliseconds).
static int fdp_try(uint64_t chunk, uint64_t ocap, int nslot, FdPipe** out) {
    FdPipe* P = (FdPipe*)calloc(1, sizeof(FdPipe));
    if (!P) return -(int)E_MALLOC;
    P->nin = P->nout = nslot;
    int r = 0;
    for (int k = 0; !r && k < P->nin; k++) {
        if (hip_fail(dmx_host_malloc((void**)&P->hin[k], chunk + 16), "hipHostMalloc")) r = -(int)E_MALLOC;
        else if (hip_fail(hipEventCreate(&P->evh[k]), "hipEventCreate") || hip_fail(hipEventCreate(&P->th[k]), "hipEventCreate"))
            r = -(int)E_DEVICE;
    }
    for (int k = 0; !r && k < P->nout; k++) {
        if (hip_fail(dmx_host_malloc((void**)&P->hout[k], ocap), "hipHostMalloc")) r = -(int)E_MALLOC;
        else if (hip_fail(hipEventCreate(&P->evo[k]), "hipEventCreate") || hip_fail(hipEventCreate(&P->td[k]), "hipEventCreate"))
            r = -(int)E_DEVICE;
    }
    for (int k = 0; !r && k < FDP_NDIN; k++)
        if (hip_fail(dmx_malloc(&P->din[k], chunk + 16), "hipMalloc")) r = -(int)E_DEVICE;
    for (int k = 0; !r && k < 2; k++) {
        if (hip_fail(dmx_malloc(&P->dout[k], ocap), "hipMalloc")) r = -(int)E_DEVICE;
        else if (hip_fail(dmx_host_malloc((void**)&P->hres[k], sizeof(dmx_result)), "hipHostMalloc")) r = -(int)E_MALLOC;
        else if (hip_fail(hipEventCreate(&P->eve[k]), "hipEventCreate") || hip_fail(hipEventCreate(&P->te[k]), "hipEventCreate") ||
                 hip_fail(hipEventCreateWithFlags(&P->evd[k], hipEventDisableTiming), "hipEventCreate"))
            r = -(int)E_DEVICE;
    }
    if (!r && (hip_fail(hipStreamCreateWithFlags(&P->sh, hipStreamNonBlocking), "hipStreamCreate") ||
               hip_fail(hipStreamCreateWithFlags(&P->sd, hipStreamNonBlocking), "hipStreamCreate")))
        r = -(int)E_DEVICE;
    if (r) { fdp_free(P); return r; }
    P->chunk = chunk;
    P->ocap = ocap;
    *out = P;
    return 0;
}

// The context's pipeline buffers for chunks of `chunk` bytes (kept across calls: pinning
// ~100 MB costs milliseconds).
static int fdp_get(dmx_ctx* c, uint64_t chunk, uint64_t ocap, FdPipe** out) {
    if (c->fdp && c->fdp->chunk >= chunk && c->fdp->ocap >= ocap) { *out = c->fdp; return 0; }
    fdp_free(c->fdp);
    c->fdp = NULL;
    FdPipe* P = NULL;
    int r = fdp_try(chunk, ocap, chunk > FDP_BIG_CHUNK ? 2 : FDP_NIN, &P);
    if (r == -(int)E_MALLOC && chunk <= FDP_BIG_CHUNK) r = fdp_try(chunk, ocap, 2, &P);   // less pinned memory
    if (r) return r;
    c->fdp = P;
    *out = P;
    return 0;
}

// Host-side hand-off between the main loop and its reader / writer threads.
struct FdSync {
    pthread_mutex_t mu;
    pthread_cond_t cv;
    int err;                 // first error (any thread); stops everything
    uint64_t nread;          // chunks read (slots filled)
    uint64_t h2d_issued;     // chunks whose H2D was enqueued (evh recorded)
    uint64_t nposted;        // chunks handed to the writer
    uint64_t nwritten;       // chunks written
    int64_t len[FDP_NIN];    // bytes in input slot k
    bool eof[FDP_NIN];       // nothing after the chunk in slot k
    uint64_t olen[FDP_NOUT]; // stream bytes in output slot k
    bool done_reading;
    double read_ms, write_ms, d2h_ms;   // reader / writer thread busy time, D2H event time
};
static double fd_now_ms() {
    struct timespec ts;
    clock_gettime(CLOCK_MONOTONIC, &ts);
    return ts.tv_sec * 1e3 + ts.tv_nsec * 1e-6;
}
static dmx_fd_stats g_fd_last;
static bool g_fd_last_ok = false;
static pthread_mutex_t g_fd_last_mu = PTHREAD_MUTEX_INITIALIZER;
extern "C" int dmx_fd_last_stats(dmx_fd_stats* out) {
    if (!out) return -(int)E_INVAL;
    pthread_mutex_lock(&g_fd_last_mu);
    const bool ok = g_fd_last_ok;
    if (ok) *out = g_fd_last;
    pthread_mutex_unlock(&g_fd_last_mu);
    return ok ? 0 : -(int)E_INVAL;
}
struct FdReadJob { FdSync* S; FdReader* R; FdPipe* P; uint64_t chunk; };
struct FdWriteJob { FdSync* S; FdPipe* P; int fd; };

static void fds_fail(FdSync* S, int r) {
    pthread_mutex_lock(&S->mu);
    if (!S->err) S->err = r;
    pthread_cond_broadcast(&S->cv);
    pthread_mutex_unlock(&S->mu);
}

static void* fdp_reader(void* a) {
    FdReadJob* J = (FdReadJob*)a;
    FdSync* S = J->S;
    for (uint64_t j = 0;; j++) {
        const uint64_t nin = (uint64_t)J->P->nin;
        const int k = (int)(j % nin);
        pthread_mutex_lock(&S->mu);   // slot k is free once chunk j - nin's H2D was enqueued...
        while (!S->err && j >= nin && S->h2d_issued < j - nin + 1) pthread_cond_wait(&S->cv, &S->mu);
        const bool stop = S->err != 0;
        pthread_mutex_unlock(&S->mu);
        if (stop) break;
        // ...and has completed
        if (j >= nin && hip_fail(hipEventSynchronize(J->P->evh[k]), "hipEventSynchronize")) {
            fds_fail(S, -(int)E_DEVICE);
            break;
        }
        const double t0 = fd_now_ms();
        const int64_t len = fd_read_chunk(J->R, J->P->hin[k], J->chunk);
        const double t1 = fd_now_ms();
        if (len < 0) { fds_fail(S, (int)len); break; }
        pthread_mutex_lock(&S->mu);
        S->read_ms += t1 - t0;
        S->len[k] = len;
        S->eof[k] = J->R->eof;
        S->nread = j + 1;
        pthread_cond_broadcast(&S->cv);
        pthread_mutex_unlock(&S->mu);
        if (J->R->eof) break;
    }
    return NULL;
}

static void* fdp_writer(void* a) {
    FdWriteJob* J = (FdWriteJob*)a;
    FdSync* S = J->S;
    for (uint64_t j = 0;; j++) {
        const int k = (int)(j % (uint64_t)J->P->nout);
        pthread_mutex_lock(&S->mu);
        while (!S->err && S->nposted <= j && !(S->done_reading && S->nposted == j)) pthread_cond_wait(&S->cv, &S->mu);
        const bool stop = S->err != 0 || S->nposted <= j;   // an error, or every posted chunk written
        const uint64_t olen = S->olen[k];
        pthread_mutex_unlock(&S->mu);
        if (stop) break;
        if (hip_fail(hipEventSynchronize(J->P->evo[k]), "hipEventSynchronize")) { fds_fail(S, -(int)E_DEVICE); break; }
        float dms = 0.f;
        if (olen && hipEventElapsedTime(&dms, J->P->td[k], J->P->evo[k]) != hipSuccess) dms = 0.f;
        const double t0 = fd_now_ms();
        const int r = J->fd >= 0 ? write_full(J->fd, J->P->hout[k], olen) : 0;
        const double t1 = fd_now_ms();
        if (r) { fds_fail(S, r); break; }
        pthread_mutex_lock(&S->mu);
        S->write_ms += t1 - t0;
        S->d2h_ms += dms;
        S->nwritten = j + 1;
        pthread_cond_broadcast(&S->cv);
        pthread_mutex_unlock(&S->mu);
    }
    return NULL;
}

typedef int (*dmx_fd_chunk_cb)(void* user, dmx_ctx* c, uint64_t chunk_bytes, uint64_t chunk_off);
static int encode_fd_on(int device, int fd_in, int fd_out, const dmx_opts* opts, uint64_t chunk,
                        dmx_fd_chunk_cb cb, void* user);

extern "C" int dmx_encode_fd(int fd_in, int fd_out, const dmx_opts* opts, uint64_t chunk) {
    const char* dev_s = getenv("DMX_DEVICE");
    return encode_fd_on(dev_s ? atoi(dev_s) : 0, fd_in, fd_out, opts, chunk, NULL, NULL);
}
// The same with a callback after every chunk's encode (dmx_host.c: the compress_stats records,
// from the context's tokens of that chunk); the chunks are then encoded one at a time.
extern "C" int dmx_encode_fd_cb(int fd_in, int fd_out, const dmx_opts* opts, uint64_t chunk, dmx_fd_chunk_cb cb,
                                void* user) {
    const char* dev_s = getenv("DMX_DEVICE");
    return encode_fd_on(dev_s ? atoi(dev_s) : 0, fd_in, fd_out, opts, chunk, cb, user);
}

static int encode_fd_on(int device, int fd_in, int fd_out, const dmx_opts* opts, uint64_t chunk,
                        dmx_fd_chunk_cb cb, void* user) {
    dmx_opts o = {0, 0, DMX_ZLIB, 0, NULL, 0};
    if (opts) o = *opts;
    if (o.sw == 0) o.sw = DMX_BLK;
    if (o.sw < 1 || o.sw > DMX_BLK) return -(int)E_RANGE;
    const uint64_t sw = (uint64_t)o.sw;
    if (chunk < sw) chunk = sw;
    chunk -= chunk % sw;
    const uint32_t pflags = o.flags & (DMX_F_LAZY | DMX_F_SPLIT | DMX_F_DICT | DMX_F_EXACT_SORT | DMX_F_STORE_CHECK |
                                       DMX_F_DEEP);
    FdReader R = {fd_in, false, 0, 0, -1, true};
    {   // a regular file of known size from the current offset: parallel preads
        struct stat st;
        const off_t cur = lseek(fd_in, 0, SEEK_CUR);
        if (cur >= 0 && fstat(fd_in, &st) == 0 && S_ISREG(st.st_mode) && (uint64_t)st.st_size >= (uint64_t)cur) {
            R.seekable = true;
            R.off = (uint64_t)cur;
            R.size = (uint64_t)st.st_size;
        }
    }
    pthread_mutex_lock(&g_mu);
    int err = 0;
    dmx_ctx* c = dmx_cached_ctx(device, chunk, &err);
    int r = err;
    const uint64_t ocap = dmx_max_compressed(chunk, o.sw);
    FdPipe* P = NULL;
    if (!r) r = dmx_ctx_reserve_flags(c, chunk, (int32_t)sw, pflags);
    if (!r && hip_fail(hipSetDevice(c->device), "hipSetDevice")) r = -(int)E_DEVICE;
    if (!r) r = fdp_get(c, chunk, ocap, &P);
    if (r) {
        pthread_mutex_unlock(&g_mu);
        return r;
    }
    hipStream_t s = c->stream;
    FdSync S;
    memset(&S, 0, sizeof(S));
    pthread_mutex_init(&S.mu, NULL);
    pthread_cond_init(&S.cv, NULL);
    FdReadJob rj = {&S, &R, P, chunk};
    FdWriteJob wj = {&S, P, fd_out};
    pthread_t rt, wt;
    const bool rstarted = pthread_create(&rt, NULL, fdp_reader, &rj) == 0;
    if (!rstarted) fds_fail(&S, -(int)E_MALLOC);
    const bool wstarted = pthread_create(&wt, NULL, fdp_writer, &wj) == 0;
    if (!wstarted) fds_fail(&S, -(int)E_MALLOC);
    uint32_t adler = 1;
    uint64_t off = 0;   // offset of the chunk being finished in the bytes read (callback)
    uint64_t clen[2] = {0, 0};
    int cin[2] = {0, 0};   // the input slot of the chunk in device output k2 (its H2D events)
    double enc_ms = 0, h2d_ms = 0;
    uint64_t nchunks = 0, nin_total = 0, nout_total = 0;
    const double t_begin = fd_now_ms();
    // chunk j - 1's result: its length, Adler-32, the callback; then its D2H and the writer
    auto finish = [&](uint64_t j) -> int {
        const int k2 = (int)(j & 1), ko = (int)(j % (uint64_t)P->nout);
        if (hip_fail(hipEventSynchronize(P->eve[k2]), "hipEventSynchronize")) return -(int)E_DEVICE;
        if (P->hres[k2]->status) return P->hres[k2]->status;
        const uint64_t olen = P->hres[k2]->out_len;
        float ems = 0.f, hms = 0.f;   // this chunk's encode and H2D (done before its encode began)
        if (hipEventElapsedTime(&ems, P->te[k2], P->eve[k2]) == hipSuccess) enc_ms += ems;
        if (clen[k2] && hipEventElapsedTime(&hms, P->th[cin[k2]], P->evh[cin[k2]]) == hipSuccess) h2d_ms += hms;
        nout_total += olen;
        adler = dmx_adler32_combine(adler, P->hres[k2]->adler, clen[k2]);
        if (cb) {
            const int e = cb(user, c, clen[k2], off);
            if (e) return e;
        }
        off += clen[k2];
        pthread_mutex_lock(&S.mu);   // output slot ko: chunk j - nout written
        while (!S.err && j >= (uint64_t)P->nout && S.nwritten < j - (uint64_t)P->nout + 1) pthread_cond_wait(&S.cv, &S.mu);
        const int e = S.err;
        pthread_mutex_unlock(&S.mu);
        if (e) return e;
        if (hip_fail(hipEventRecord(P->td[ko], P->sd), "hipEventRecord")) return -(int)E_DEVICE;
        if (olen && hip_fail(hipMemcpyAsync(P->hout[ko], P->dout[k2], olen, hipMemcpyDeviceToHost, P->sd), "D2H"))
            return -(int)E_DEVICE;
        if (hip_fail(hipEventRecord(P->evd[k2], P->sd), "hipEventRecord") ||
            hip_fail(hipEventRecord(P->evo[ko], P->sd), "hipEventRecord"))
            return -(int)E_DEVICE;
        pthread_mutex_lock(&S.mu);
        S.olen[ko] = olen;
        S.nposted = j + 1;
        pthread_cond_broadcast(&S.cv);
        pthread_mutex_unlock(&S.mu);
        return 0;
    };
    bool have_prev = false;
    for (uint64_t i = 0; !r; i++) {
        const int ki = (int)(i % (uint64_t)P->nin), kd = (int)(i % FDP_NDIN), k2 = (int)(i & 1);
        pthread_mutex_lock(&S.mu);
        while (!S.err && S.nread <= i) pthread_cond_wait(&S.cv, &S.mu);
        r = S.err;
        const int64_t len = r ? 0 : S.len[ki];
        const bool last = r ? true : S.eof[ki];
        pthread_mutex_unlock(&S.mu);
        if (r) break;
        // H2D into device input kd: encode i - FDP_NDIN read it, encode i - FDP_NDIN + 1 its tail
        // (history); the latter is ordered after the former on the encode stream, and the host
        // has already waited for it (finish(i - 2) ran in the previous iteration, or earlier with
        // a callback), so the copy stream needs no wait packet before the copy
#ifdef DMX_FD_WAIT   // (A/B build: the stream wait as before)
        if (i >= FDP_NDIN - 1 && hip_fail(hipStreamWaitEvent(P->sh, P->eve[(i - (FDP_NDIN - 1)) & 1], 0), "wait"))
            r = -(int)E_DEVICE;
#endif
        if (!r && hip_fail(hipEventRecord(P->th[ki], P->sh), "hipEventRecord")) r = -(int)E_DEVICE;
        if (!r && len && hip_fail(hipMemcpyAsync(P->din[kd], P->hin[ki], (size_t)len, hipMemcpyHostToDevice, P->sh), "H2D"))
            r = -(int)E_DEVICE;
        if (!r && hip_fail(hipEventRecord(P->evh[ki], P->sh), "hipEventRecord")) r = -(int)E_DEVICE;
        pthread_mutex_lock(&S.mu);
        S.h2d_issued = i + 1;
        pthread_cond_broadcast(&S.cv);
        pthread_mutex_unlock(&S.mu);
        // the encode: after its H2D, and after the D2H that last read device output k2
        if (!r && hip_fail(hipStreamWaitEvent(s, P->evh[ki], 0), "wait")) r = -(int)E_DEVICE;
        if (!r && i >= 2 && hipEventQuery(P->evd[k2]) != hipSuccess &&   // (no wait packet when the D2H is done)
            hip_fail(hipStreamWaitEvent(s, P->evd[k2], 0), "wait"))
            r = -(int)E_DEVICE;
        dmx_opts oc = o;
        oc.flags = pflags | (i == 0 ? DMX_F_HEADER : 0u) | (last ? DMX_F_FINAL : 0u);
        oc.dict = NULL;
        oc.dict_len = 0;
        if ((pflags & DMX_F_DICT) && i > 0) {   // the previous chunk's tail, still on the device
            oc.dict = (const uint8_t*)P->din[(i - 1) % FDP_NDIN] + (chunk - sw);
            oc.dict_len = sw;
        }
        if (!r && hip_fail(hipEventRecord(P->te[k2], s), "hipEventRecord")) r = -(int)E_DEVICE;
        if (!r) r = dmx_encode_async(c, P->din[kd], (uint64_t)len, P->dout[k2], ocap, &oc, s);
        if (!r) r = dmx_encode_result_async(c, P->hres[k2], s);
        if (!r && hip_fail(hipEventRecord(P->eve[k2], s), "hipEventRecord")) r = -(int)E_DEVICE;
        clen[k2] = (uint64_t)len;
        cin[k2] = ki;
        nchunks++;
        nin_total += (uint64_t)len;
        // the previous chunk finishes while this one encodes (a callback needs the context's
        // tokens of its own chunk: then each chunk finishes before the next encodes)
        if (!r && cb) r = finish(i);
        else if (!r && have_prev) r = finish(i - 1);
        have_prev = !cb;
        if (!r && last) {
            if (!cb) r = finish(i);
            break;
        }
    }
    if (r) fds_fail(&S, r);
    pthread_mutex_lock(&S.mu);
    S.done_reading = true;
    pthread_cond_broadcast(&S.cv);
    pthread_mutex_unlock(&S.mu);
    if (rstarted) pthread_join(rt, NULL);
    if (wstarted) pthread_join(wt, NULL);
    if (!r) r = S.err;
    if (!r && fd_out >= 0) {
        const uint8_t tail[4] = {(uint8_t)(adler >> 24), (uint8_t)(adler >> 16), (uint8_t)(adler >> 8), (uint8_t)adler};
        r = write_full(fd_out, tail, 4);
    }
    if (R.seekable) (void)lseek(fd_in, (off_t)R.off, SEEK_SET);   // consumed, as read() would leave it
    // nothing may still run on the cached buffers when the lock is released
    (void)hipStreamSynchronize(P->sh);
    (void)hipStreamSynchronize(s);
    (void)hipStreamSynchronize(P->sd);
    if (!r) {
        pthread_mutex_lock(&g_fd_last_mu);
        g_fd_last.chunks = nchunks;
        g_fd_last.bytes_in = nin_total;
        g_fd_last.bytes_out = nout_total + 4;
        g_fd_last.wall_ms = fd_now_ms() - t_begin;
        g_fd_last.read_ms = S.read_ms;
        g_fd_last.h2d_ms = h2d_ms;
        g_fd_last.encode_ms = enc_ms;
        g_fd_last.d2h_ms = S.d2h_ms;
        g_fd_last.write_ms = S.write_ms;
        g_fd_last_ok = true;
        pthread_mutex_unlock(&g_fd_last_mu);
    }
    pthread_cond_destroy(&S.cv);
    pthread_mutex_destroy(&S.mu);
    pthread_mutex_unlock(&g_mu);
    return r;
}

// --- the fd path over several GPUs (dmx_encode_fd_multi, DMX_DEVICES) ---
// One host thread per listed device, each with its own context and pinned buffers (cached per
// list position).  Worker w takes chunks w, w + ndev, ...: pread from the file, H2D, encode,
// D2H, then waits for its turn and writes the chunk in file order; the Adler-32 values are
// combined in the same order.  The framing and the parse are dmx_encode_fd's, so the stream
// is byte-identical to it with the same chunk size.
static dmx_ctx* g_wctx[64];

struct MultiJob {
    int fd_in, fd_out;
    uint64_t off0, size, chunk, nchunks, sw;
    dmx_opts o;
    uint32_t pflags;
    int ndev;
    pthread_mutex_t mu;
    pthread_cond_t cv;
    uint64_t next;   // next chunk to write
    uint32_t adler;
    int err;
};
struct MultiWorker {
    MultiJob* J;
    dmx_ctx* c;
    int w;
};

static int pread_full(int fd, uint8_t* b, uint64_t len, uint64_t off) {
    uint64_t done = 0;
    while (done < len) {
        const ssize_t r = pread(fd, b + done, len - done, (off_t)(off + done));
        if (r < 0) {
            if (errno == EINTR) continue;
            return -(int)E_NEXIST;
        }
        if (r == 0) return -(int)E_NEXIST;   // the file shrank under us
        done += (uint64_t)r;
    }
    return 0;
}

static void multi_fail(MultiJob* J, int r) {
    pthread_mutex_lock(&J->mu);
    if (!J->err) J->err = r;
    pthread_cond_broadcast(&J->cv);
    pthread_mutex_unlock(&J->mu);
}

// Worker pipeline over its chunks t = 0, 1, ... (file chunks w, w + ndev, ...), two of
// everything: while the device encodes chunk t + 1 (input slot and output slot (t + 1) & 1),
// the host copies chunk t back on the copy stream, waits for its turn and writes it, and
// reads chunk t + 2 from the file.  With DMX_F_DICT each pread also takes the sw bytes before
// the chunk (the first block's history) into the slot's front, one H2D for both.
static int multi_enqueue(MultiJob* J, dmx_ctx* c, uint64_t i, uint64_t len, int k, uint64_t ocap) {
    dmx_opts oc = J->o;
    oc.flags = J->pflags | (i == 0 ? DMX_F_HEADER : 0u) | (i + 1 == J->nchunks ? DMX_F_FINAL : 0u);
    const bool hist = (J->pflags & DMX_F_DICT) && i > 0;
    const uint64_t front = hist ? J->sw : 0;
    oc.dict = hist ? (const uint8_t*)c->fd_din[k] + (DMX_BLK - front) : NULL;
    oc.dict_len = front;
    hipStream_t s = c->stream;
    if ((len || front) &&
        hip_fail(hipMemcpyAsync((uint8_t*)c->fd_din[k] + (DMX_BLK - front), c->fd_hin[k] + (DMX_BLK - front),
                                (size_t)(front + len), hipMemcpyHostToDevice, s), "H2D"))
        return -(int)E_DEVICE;
    int r = dmx_encode_async(c, (const uint8_t*)c->fd_din[k] + DMX_BLK, len, c->fd_dout[k], ocap, &oc, s);
    if (!r) r = dmx_encode_result_async(c, c->fd_hres[k], s);
    if (!r && hip_fail(hipEventRecord(c->fd_ev[k], s), "hipEventRecord")) r = -(int)E_DEVICE;
    return r;
}

static int multi_read(MultiJob* J, dmx_ctx* c, uint64_t i, uint64_t len, int k) {
    const uint64_t front = ((J->pflags & DMX_F_DICT) && i > 0) ? J->sw : 0;
    if (!len && !front) return 0;
    return pread_full(J->fd_in, c->fd_hin[k] + (DMX_BLK - front), front + len, J->off0 + i * J->chunk - front);
}

static void* multi_worker(void* a) {
    MultiWorker* W = (MultiWorker*)a;
    MultiJob* J = W->J;
    dmx_ctx* c = W->c;
    if (hip_fail(hipSetDevice(c->device), "hipSetDevice")) { multi_fail(J, -(int)E_DEVICE); return NULL; }
    const uint64_t ocap = dmx_max_compressed(J->chunk, (int32_t)J->sw);
    const uint64_t step = (uint64_t)J->ndev;
    auto chunk_len = [&](uint64_t i) {
        const uint64_t lo = i * J->chunk, left = J->size - J->off0 - lo;
        return left < J->chunk ? left : J->chunk;
    };
    uint64_t i = (uint64_t)W->w;
    int r = 0;
    if (i < J->nchunks) {
        r = multi_read(J, c, i, chunk_len(i), 0);
        if (!r) r = multi_enqueue(J, c, i, chunk_len(i), 0, ocap);
    }
    for (int k = 0; !r && i < J->nchunks; i += step, k ^= 1) {
        if (__atomic_load_n(&J->err, __ATOMIC_RELAXED)) break;
        const uint64_t len = chunk_len(i), in = i + step;
        const bool more = in < J->nchunks;
        if (more) r = multi_read(J, c, in, chunk_len(in), k ^ 1);   // beside the device's work on chunk i
        if (!r && hip_fail(hipEventSynchronize(c->fd_ev[k]), "hipEventSynchronize")) r = -(int)E_DEVICE;
        if (!r && c->fd_hres[k]->status) r = c->fd_hres[k]->status;
        const uint64_t olen = r ? 0 : c->fd_hres[k]->out_len;
        const uint32_t cadl = r ? 0 : c->fd_hres[k]->adler;
        if (!r && more) r = multi_enqueue(J, c, in, chunk_len(in), k ^ 1, ocap);   // the device goes on
        if (!r && (hip_fail(hipMemcpyAsync(c->fd_hout[k], c->fd_dout[k], olen, hipMemcpyDeviceToHost, c->fd_cs), "D2H") ||
                   hip_fail(hipStreamSynchronize(c->fd_cs), "hipStreamSynchronize")))
            r = -(int)E_DEVICE;
        if (r) break;
        pthread_mutex_lock(&J->mu);   // in order: chunk i after chunk i - 1
        while (J->next != i && !J->err) pthread_cond_wait(&J->cv, &J->mu);
        if (!J->err) {
            if (J->fd_out >= 0) r = write_full(J->fd_out, c->fd_hout[k], olen);
            J->adler = dmx_adler32_combine(J->adler, cadl, len);
            if (r) J->err = r;
            J->next = i + 1;
        }
        pthread_cond_broadcast(&J->cv);
        pthread_mutex_unlock(&J->mu);
    }
    if (r) multi_fail(J, r);
    (void)hipStreamSynchronize(c->stream);   // nothing of this call left in flight
    return NULL;
}

// DMX_DEVICES: "0,1,2,3" (a device may repeat: one context each) or "all"; the number of
// entries written to devs, 0 when unset or empty; -E_INVAL for a malformed list, -E_RANGE
// for more than cap entries, -E_NEXIST when "all" finds no device.
extern "C" int dmx_devices_from_env(int* devs, int cap) {
    const char* e = getenv("DMX_DEVICES");
    if (!e || !*e) return 0;
    if (!strcmp(e, "all")) {
        int nd = 0;
        if (hipGetDeviceCount(&nd) != hipSuccess || nd <= 0) return -(int)E_NEXIST;
        if (nd > cap) return -(int)E_RANGE;
        for (int k = 0; k < nd; k++) devs[k] = k;
        return nd;
    }
    int n = 0;
    for (const char* p = e; *p;) {
        char* end = NULL;
        const long v = strtol(p, &end, 10);
        if (end == p) return -(int)E_INVAL;
        if (n == cap) return -(int)E_RANGE;
        devs[n++] = (int)v;
        p = *end == ',' ? end + 1 : end;
        if (*end && *end != ',') return -(int)E_INVAL;
    }
    return n;
}

extern "C" int dmx_encode_fd_multi(int fd_in, int fd_out, const dmx_opts* opts, uint64_t chunk, const int* devices,
                                   int ndev) {
    if (!devices || ndev < 1 || ndev > 64) return -(int)E_RANGE;
    int nd = 0;   // every listed device must exist, whether or not the input reaches it
    if (hipGetDeviceCount(&nd) != hipSuccess || nd <= 0) return -(int)E_NEXIST;
    for (int w = 0; w < ndev; w++)
        if (devices[w] < 0 || devices[w] >= nd) return -(int)E_RANGE;
    // one device: the single-device streaming path (read-ahead and writer threads overlap
    // the encode), not one worker doing every step in turn
    if (ndev == 1) return encode_fd_on(devices[0], fd_in, fd_out, opts, chunk, NULL, NULL);
    dmx_opts o = {0, 0, DMX_ZLIB, 0, NULL, 0};
    if (opts) o = *opts;
    if (o.sw == 0) o.sw = DMX_BLK;
    if (o.sw < 1 || o.sw > DMX_BLK) return -(int)E_RANGE;
    const uint64_t sw = (uint64_t)o.sw;
    if (chunk < sw) chunk = sw;
    chunk -= chunk % sw;
    struct stat st;
    const off_t cur = lseek(fd_in, 0, SEEK_CUR);
    if (cur < 0 || fstat(fd_in, &st) != 0 || !S_ISREG(st.st_mode) || (uint64_t)st.st_size < (uint64_t)cur)
        return encode_fd_on(devices[0], fd_in, fd_out, opts, chunk, NULL, NULL);   // a pipe: one device, one reader
    MultiJob J;
    J.fd_in = fd_in;
    J.fd_out = fd_out;
    J.off0 = (uint64_t)cur;
    J.size = (uint64_t)st.st_size;
    J.chunk = chunk;
    J.sw = sw;
    J.nchunks = (J.size - J.off0 + chunk - 1) / chunk;
    if (J.nchunks == 0) J.nchunks = 1;   // an empty input is one empty chunk (header, EOB block, trailer)
    J.o = o;
    J.pflags = o.flags & (DMX_F_LAZY | DMX_F_SPLIT | DMX_F_DICT | DMX_F_EXACT_SORT | DMX_F_STORE_CHECK | DMX_F_DEEP);
    J.ndev = ndev < (int)J.nchunks ? ndev : (int)J.nchunks;
    pthread_mutex_init(&J.mu, NULL);
    pthread_cond_init(&J.cv, NULL);
    J.next = 0;
    J.adler = 1;
    J.err = 0;
    pthread_mutex_lock(&g_mu);
    int r = 0;
    MultiWorker W[64];
    const uint64_t ocap = dmx_max_compressed(chunk, o.sw);
    for (int w = 0; w < J.ndev && !r; w++) {   // the workers' contexts (cached per list position)
        if (g_wctx[w] && g_wctx[w]->device != devices[w]) {
            dmx_ctx_destroy(g_wctx[w]);
            g_wctx[w] = NULL;
        }
        if (!g_wctx[w]) r = dmx_ctx_create(devices[w], chunk, &g_wctx[w]);
        if (!r) r = dmx_ctx_reserve_flags(g_wctx[w], chunk, o.sw, J.pflags);
        if (!r && hip_fail(hipSetDevice(g_wctx[w]->device), "hipSetDevice")) r = -(int)E_DEVICE;
        if (!r) r = fd_buffers(g_wctx[w], chunk, ocap);
        W[w] = {&J, g_wctx[w], w};
    }
    pthread_t th[64];
    bool started[64] = {false};
    for (int w = 0; w < J.ndev && !r; w++) {
        if (pthread_create(&th[w], NULL, multi_worker, &W[w]) == 0) started[w] = true;
        else { multi_fail(&J, -(int)E_FORK); r = -(int)E_FORK; }
    }
    for (int w = 0; w < J.ndev; w++)
        if (started[w]) pthread_join(th[w], NULL);
    if (!r) r = J.err;
    if (!r && fd_out >= 0) {
        const uint32_t ad = J.adler;
        const uint8_t tail[4] = {(uint8_t)(ad >> 24), (uint8_t)(ad >> 16), (uint8_t)(ad >> 8), (uint8_t)ad};
        r = write_full(fd_out, tail, 4);
    }
    if (!r) (void)lseek(fd_in, (off_t)J.size, SEEK_SET);   // consumed, as read() would leave it
    for (int w = 0; w < J.ndev; w++)   // an error may have left copies in flight from the cached buffers
        if (r && g_wctx[w]) { (void)hipSetDevice(g_wctx[w]->device); (void)hipStreamSynchronize(g_wctx[w]->stream); }
    pthread_mutex_unlock(&g_mu);
    pthread_mutex_destroy(&J.mu);
    pthread_cond_destroy(&J.cv);
    return r;
}

// Per-block match-kernel phase stamps of the last encode (DMX_STAMPS=1): for each block
// {cycles to build the chains (wave 0), cycles until the last wave finished searching,
//  cycles of walk + compaction, tokens}.  Diagnostic only.
extern "C" int dmx_debug_stamps(dmx_ctx* c, uint64_t* out, uint32_t nblk) {
    if (!c->dbg || nblk > c->dbg_cap || nblk > c->last_nblk) return -(int)E_RANGE;
    HIPCHK(hipSetDevice(c->device));
    HIPCHK(hipDeviceSynchronize());
    HIPCHK(hipMemcpy(out, c->dbg, (uint64_t)nblk * DMX_STAMPS * sizeof(uint64_t), hipMemcpyDeviceToHost));
    return 0;
}
