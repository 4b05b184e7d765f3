/*
 * dmx.h -- C-ABI of libdmx, the MI355X-native DEFLATE encoder.
 *
 * Part 1 is the drop-in boundary: the exact entry points of the reference's public
 * codec API, src/include/deflate_ext.h of mparker97/deflate_compression, so a C
 * caller of the reference links against libdmx.so unchanged.
 * Part 2 is the device layer those entry points call: device-resident buffers,
 * explicit HIP streams, no allocation inside an encode (graph-capturable).
 *
 * All signatures are plain C types; no torch types cross this boundary.
 */
#ifndef DMX_H
#define DMX_H

#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

/* ======================= Part 1: reference API (deflate_ext.h) ======================= */

/* deflate_ext.h:6 -- deflate_decompress option: append a '\0' after the output */
#define DEFLATE_NULLTERM 1

/* deflate_ext.h:8 -- sliding-window index / window size type */
typedef unsigned short swi;

/* globals.h:42-46 -- byte string with explicit length */
struct string_len {
    unsigned char* str;
    size_t len;
};

/* deflate_ext.h:10-14 -- opaque compressor state + spawn/init/deinit.
 * Replaces struct deflate_compr (deflate_compress.c:69-81) and SPAWNABLE
 * (globals.h:20-29).  init never longjmps; errors surface from deflate_compress. */
typedef struct deflate_compr deflate_compr_t;
deflate_compr_t* spawn_deflate_compr_t(void);
void deflate_compr_init(deflate_compr_t* com, int fd_in, int fd_out, int fd_stats, swi sw);
void deflate_compr_deinit(deflate_compr_t* com);

/* deflate_ext.h:17, impl deflate_compress.c:362-376.
 * Reads fd_in to EOF, writes a zlib stream (RFC 1950/1951) to fd_out, and if
 * fd_stats >= 0 one 24-byte struct compress_stats per token.  sw = block size /
 * window (1..32768; 0 means 32768).  ops is unused (as in the reference).
 * The parse is the reference's: exhaustive hash-chain search, greedy, longest
 * match >= 3, ties to the nearest (DMX_MAX_CHAIN=K in the environment selects the
 * bounded fast mode).  Returns 0, or -E_* on error (the reference returned
 * nothing).  The encode runs on the MI355X (device DMX_DEVICE, default 0); there is
 * no CPU fallback: without a usable GPU it fails with -E_NEXIST. */
int deflate_compress(int fd_in, int fd_out, int fd_stats, swi sw, int ops);

/* deflate_ext.h:16, impl deflate_decompress.c:371-409 (that implementation does not
 * compile; this one is a fresh RFC 1950/1951 inflate).
 * Inflates compr_dat (zlib stream) into a malloc'd decompr_dat->str that the
 * caller frees.  ops & DEFLATE_NULLTERM appends a '\0' (not counted in len).
 * Returns 0 or -E_*. */
int deflate_decompress(struct string_len* decompr_dat, struct string_len* compr_dat, int ops);

/* deflate_ext.h:19-31 -- per-token record written to fd_stats.
 * bytes = 1 + input offset of the token; ll/d = literal byte (d == 0) or length/
 * distance.  The *_bits fields depend on DMX_STATS in the environment:
 *   unset / "ref"  the reference's own estimates (deflate_compress.c:290-298): tree_bits =
 *                  the code-length description cost of its adaptive Huffman trees
 *                  (h_tree.c:75-148) + the code-length code's weighted depth (:242-302),
 *                  ll_bits / d_bits = the adaptive trees' scores after this token
 *                  (aht.c:239-277), running over the whole stream as in the reference.
 *                  Same records as the reference for the same tokens (dmx_refest_*).
 *                  Parity unpinned past one window: the reference itself is only correct
 *                  for its first 32 KiB window, so records of later blocks
 *                  are checked against this host restatement fed the oracle's tokens, not
 *                  against the reference's own output.
 *   "exact"        exact costs of this stream, running over the whole stream: tree_bits =
 *                  header bits of every DEFLATE block begun so far (its own included;
 *                  the empty stored blocks that end each DMX_CHUNK_MB chunk but the last
 *                  are framing, not coding, and are not counted),
 *                  ll_bits = lit/len code + length extra bits of every token so far (8 per
 *                  byte in stored blocks), d_bits = distance code + extra bits so far.
 * The fields are int, as in the reference: deflate_compress returns -E_RANGE, after the
 * complete stream to fd_out and every record before it, at the first record whose bytes
 * or *_bits would exceed INT_MAX (inputs past 2 GiB, or about 2^31 bits of running sum). */
struct compress_stats {
    int bytes;
    int tree_bits;
    int ll_bits;
    int d_bits;
    int ll;
    int d;
};

/* Error codes: src/include/global_errors.h:24-35 and src/include/deflate_errors.h:9-22 (returned negated). */
#define E_LEN 1
#define E_MALLOC 2
#define E_FORK 3
#define E_PIPE 4
#define E_CRC 5
#define E_SZ 6
#define E_EXIST 7
#define E_NEXIST 8
#define E_NONULL 9
#define E_RANGE 10
#define E_INVAL 11
#define E_RESERV 12
#define DEFLATE_ERROR_MASK (1U << 24)
#define E_HUFAMB (DEFLATE_ERROR_MASK + 1)
#define E_HUFINV (DEFLATE_ERROR_MASK + 2)
#define E_HUFVAL (DEFLATE_ERROR_MASK + 3)
#define E_HUFDIS (DEFLATE_ERROR_MASK + 4)
#define E_ZADL32 (DEFLATE_ERROR_MASK + 5)
#define E_ZHEAD (DEFLATE_ERROR_MASK + 6)
#define E_ZFCHCK (DEFLATE_ERROR_MASK + 7)
#define E_ZCMPMT (DEFLATE_ERROR_MASK + 8)
#define E_ZSLWIN (DEFLATE_ERROR_MASK + 9)
#define E_ZPDICT (DEFLATE_ERROR_MASK + 10)
#define E_ZBSZ (DEFLATE_ERROR_MASK + 11)
#define E_ZNLEN (DEFLATE_ERROR_MASK + 12)
#define E_ZINV (DEFLATE_ERROR_MASK + 13)
#define E_ZBTYPE (DEFLATE_ERROR_MASK + 14)
/* dmx additions (outside both reference ranges) */
#define E_DEVICE (DEFLATE_ERROR_MASK + 64) /* HIP runtime / launch failure */

/* ============================ Part 2: device layer ============================ */

/* Stream framing flags (dmx_opts.flags). DMX_ZLIB = a complete zlib stream. */
#define DMX_F_HEADER 1u  /* write the 2-byte zlib header 78 9C */
#define DMX_F_TRAILER 2u /* write the Adler-32 trailer (big-endian) */
#define DMX_F_FINAL 4u   /* last block carries BFINAL; otherwise the stream ends with
                            an empty stored block (sync flush) so it is byte-aligned
                            and another shard can be appended */
#define DMX_ZLIB (DMX_F_HEADER | DMX_F_TRAILER | DMX_F_FINAL)
#define DMX_F_EXACT_SORT 16u  /* test hook: sort positions with the match-any grouping instead
                                of lane-ordered LDS atomics (same result; used by the tests) */
#define DMX_F_LAZY 8u    /* parse option: lazy evaluation, one position of
                            lookahead -- a match at i becomes a literal when the match at
                            i+1 is strictly longer.  Off = the reference's greedy parse. */
#define DMX_F_SPLIT 32u  /* block option: an sw block may be emitted as up to
                            four DEFLATE blocks cut at the token boundaries of its quarters,
                            each with its own codes, when that is smaller */

#define DMX_F_DICT 64u   /* parse option: cross-block dictionary -- every block
                            also searches the previous sw block (the K newest entries of its
                            hash chain, distance <= 32768); a history match is taken only when
                            strictly longer than the block's own.  Block 0
                            uses dmx_opts.dict when given.  Blocks then depend on their
                            predecessor: inflate with the stream mode, not the block index. */
#define DMX_F_STORE_CHECK 128u  /* block option: a block whose bytes pass an
                                 * integer noise check (flat byte histogram, few 4-byte
                                 * repeats) is emitted stored without a parse -- the stored
                                 * path runs at HBM speed instead of the match kernel's.  An
                                 * encoder policy of our own (the reference always parses);
                                 * the oracle applies the same rule.  Such blocks have no
                                 * tokens (no compress_stats records). */
#define DMX_F_DEEP 256u  /* parse option: adaptive chain depth for bounded
                            K < 64 -- a block whose trigrams are few (D distinct 13-bit
                            buckets among its positions p mod 2048 < 256, 4 D < samples:
                            small alphabets such as binary digits, hex, DNA) searches its
                            own chains 32 deep instead of K (dmx_opts.deep_chain sets
                            another depth; 32 is the cheapest depth that keeps every
                            reference-held text file within 2 % of the reference parse).  Text never qualifies. */
#define DMX_DEEP_CHAIN 32

typedef struct {
    int32_t sw;        /* block size 1..32768 (0 = 32768) */
    int32_t max_chain; /* 0 = exhaustive (reference semantics); K > 0 = the K newest chain entries */
    uint32_t flags;    /* DMX_F_* */
    int32_t deep_chain; /* DMX_F_DEEP: the chain depth of a small-alphabet block, 0..255
                           (0 = DMX_DEEP_CHAIN); values outside 0..255 return -E_RANGE, and a
                           depth <= max_chain has no effect (the block keeps K).  (This
                           field was `reserved`, always 0, before round 5.) */
    const void* dict;  /* DMX_F_DICT: the bytes just before the input (device memory for
                          dmx_encode_async, host memory for dmx_encode_host), history of
                          block 0; the last min(dict_len, sw) bytes are used.  NULL: none */
    uint64_t dict_len;
} dmx_opts;

/* Result of one encode, filled on the device, fetched by dmx_encode_result(). */
typedef struct {
    uint64_t out_len;   /* bytes written to d_out */
    uint64_t end_bits;  /* bit position after the last block (before flush/trailer) */
    uint64_t n;         /* input bytes */
    uint64_t ntokens;   /* tokens over all blocks */
    uint32_t adler;     /* Adler-32 of this input (RFC 1950 §8.2) */
    int32_t status;     /* 0 or -E_* */
    uint32_t nblocks;
    uint32_t nstored, nfixed, ndynamic;
    uint32_t nsortfallback; /* blocks of this encode whose lane-ordered radix sort failed its
                               order check and were re-sorted with the match-any grouping
                               (DESIGN.md §3); the DMX_F_EXACT_SORT test hook forces one per
                               searched block */
    uint32_t nsortfallback_total; /* the same, summed over every encode of the context */
} dmx_result;

typedef struct dmx_ctx dmx_ctx;

/* Allocate a device context (own HIP stream + workspace) for inputs up to max_input. */
int dmx_ctx_create(int device, uint64_t max_input, dmx_ctx** out);
void dmx_ctx_destroy(dmx_ctx* ctx);
/* Grow the workspace (synchronising) so that n bytes with block size sw fit. */
int dmx_ctx_reserve(dmx_ctx* ctx, uint64_t n, int32_t sw);
/* The same, plus the scratch the block options need from then on: DMX_F_SPLIT (split plans)
 * and DMX_F_DICT (every block's exported chains).  dmx_encode_async never allocates: with
 * those flags on a context not reserved for them it returns -E_SZ.  Synchronises only when
 * it allocates. */
int dmx_ctx_reserve_flags(dmx_ctx* ctx, uint64_t n, int32_t sw, uint32_t flags);
/* Worst-case output bytes for n input bytes with block size sw. */
uint64_t dmx_max_compressed(uint64_t n, int32_t sw);

/* Enqueue the whole encode of device buffer d_in[0..n) into d_out (capacity
 * out_cap) on `stream` (hipStream_t; NULL = the context's stream).  No host
 * synchronisation, no allocation (graph-capturable).  Returns 0 or -E_* for argument
 * errors: -E_SZ when n needs more blocks than the context holds, or DMX_F_SPLIT /
 * DMX_F_DICT on a context not reserved for them (dmx_ctx_reserve_flags).  With
 * DMX_F_STORE_CHECK, bytes of d_out past the final out_len (inside out_cap) may be
 * overwritten: a noise block is copied speculatively to the offset it would have if every
 * block before it were stored. */
int dmx_encode_async(dmx_ctx* ctx, const void* d_in, uint64_t n, void* d_out, uint64_t out_cap,
                     const dmx_opts* opts, void* stream);
/* Wait for the last encode on `stream` and copy its dmx_result to the host. */
int dmx_encode_result(dmx_ctx* ctx, dmx_result* r, void* stream);
/* Enqueue the copy of the last encode's dmx_result into r (pinned host memory for a truly
 * asynchronous copy) on `stream`, without waiting: the caller waits on the stream or on an
 * event recorded after this call.  Lets a pipeline (bench.py, N > 1) learn chunk i's length
 * while encode i + 1 runs. */
int dmx_encode_result_async(dmx_ctx* ctx, dmx_result* r, void* stream);

/* Host-buffer convenience (H2D, encode, D2H) on a cached per-device context.
 * *out_len receives the stream length; out must hold dmx_max_compressed(n, sw). */
int dmx_encode_host(const uint8_t* in, uint64_t n, uint8_t* out, uint64_t out_cap,
                    uint64_t* out_len, const dmx_opts* opts);

/* Streaming file-in/file-out encode (deflate_compress without fd_stats): reads fd_in in
 * chunks of `chunk` bytes (rounded down to a multiple of sw; 0 = sw) into pinned memory,
 * encodes chunk i on the device while reading chunk i+1, writes one zlib stream to fd_out
 * (chunks joined by sync flushes, Adler-32 combined on the host; DMX_F_DICT carries the
 * history across chunks).  opts->flags: the parse/block options (DMX_F_LAZY, _SPLIT, _DICT);
 * the framing is its own.  Returns 0 or -E_*. */
int dmx_encode_fd(int fd_in, int fd_out, const dmx_opts* opts, uint64_t chunk);

/* Where the last single-device dmx_encode_fd call (or deflate_compress without fd_stats)
 * spent its time, per stage of its pipeline: wall time of the call; the
 * reader thread's time in read()/pread(); the H2D copies, encodes and D2H copies on the
 * device (HIP event times, summed over chunks); the writer thread's time in write().  The
 * stages overlap, so the largest of them bounds the call.  Returns 0, or -E_INVAL when no
 * such call has finished in this process. */
typedef struct {
    uint64_t chunks, bytes_in, bytes_out;
    double wall_ms, read_ms, h2d_ms, encode_ms, d2h_ms, write_ms;
} dmx_fd_stats;
int dmx_fd_last_stats(dmx_fd_stats* out);

/* The same stream as dmx_encode_fd with the chunks spread over several GPUs: chunk i is
 * read (pread), encoded and copied back by the host thread of devices[i % ndev], and the
 * chunks are written to fd_out in order (one host thread per GPU).  Needs a
 * regular file as fd_in (a pipe falls back to dmx_encode_fd on devices[0]).  A device may
 * be listed more than once (one context per entry).  deflate_compress uses it when
 * DMX_DEVICES lists more than one device ("0,1,2,3" or "all").  Returns 0 or -E_*. */
int dmx_encode_fd_multi(int fd_in, int fd_out, const dmx_opts* opts, uint64_t chunk, const int* devices, int ndev);

/* Test hook (fault injection): "malloc:N" makes the N-th device or pinned
 * allocation of the library from now fail, "launch:N" the N-th encode's launch check;
 * NULL or "" turns it off.  Also read from DMX_FAULT when the library loads.  The failing
 * call returns -E_DEVICE (or -E_MALLOC for pinned memory) and leaves no allocation behind
 * that its context does not own.  Returns 0, or -E_INVAL / -E_RANGE for a bad spec. */
int dmx_fault_set(const char* spec);

/* Test hooks of one context: launch shapes that every encode must turn into the same stream
 * (DESIGN.md §3.3).  Their defaults come from the environment, read once when the context is
 * created (DMX_WORKLIST = 0 | list | plain, DMX_DEDUPE = 0 | 1, DMX_SCAN3 = 1); an encode
 * never reads the environment.  Values: DMX_HOOK_WORKLIST -1 adaptive (default), 0 no work
 * lists, 1 the list shapes, 2 a workgroup per block; DMX_HOOK_DEDUPE -1 adaptive, 0 off,
 * 1 on; DMX_HOOK_SCAN3 0 / 1 (K3 in three launches at any size).  Set them between encodes
 * on the context's own thread.  Returns 0, -E_INVAL (unknown hook) or -E_RANGE. */
#define DMX_HOOK_WORKLIST 1
#define DMX_HOOK_DEDUPE 2
#define DMX_HOOK_SCAN3 3
int dmx_ctx_set_hook(dmx_ctx* ctx, int hook, int value);

/* ---- GPU inflate, csrc/dmx_inflate_dev.hip ---- */
/* One entry per independently decodable DEFLATE block: start bit in the stream, output
 * offset and length.  Blocks of a dmx stream never reference earlier blocks. */
typedef struct {
    uint64_t bit;
    uint64_t out_off;
    uint32_t out_len;
    uint32_t reserved;
} dmx_iblock;
typedef struct {
    int32_t status;     /* 0 or -E_* (first error) */
    uint32_t reserved;
    uint64_t out_len;   /* bytes produced */
} dmx_inflate_status;
/* Device block index of the last encode of ctx (nblk entries into d_index, on stream). */
int dmx_block_index(dmx_ctx* ctx, dmx_iblock* d_index, uint32_t cap, void* stream);
/* Inflate on the GPU.  d_index != NULL: decode the nblk listed blocks in parallel (one
 * wave each) into d_out + out_off.  d_index == NULL: decode the whole zlib stream d_z
 * (header, blocks until BFINAL, Adler-32 check) in one workgroup.  Status in the device
 * record d_status.  The first-level tables live in device scratch taken from a per-device
 * stream-ordered pool on every call (hipMallocFromPoolAsync before the launch, hipFreeAsync
 * after it on the same stream).  Returns 0 or -E_*: -E_MALLOC when that scratch cannot be
 * allocated, -E_DEVICE for launch errors. */
int dmx_inflate_async(const void* d_z, uint64_t zbytes, const dmx_iblock* d_index, uint32_t nblk, void* d_out,
                      uint64_t out_cap, dmx_inflate_status* d_status, void* stream);

/* Chained GPU inflate: the blocks listed in d_index decoded in parallel although a block's
 * matches may reach into the blocks before it (DMX_F_DICT streams; any stream cut at block
 * starts).  Each block decodes into 16-bit cells -- a byte, or a reference to a position
 * before the block -- and pointer jumping over the references, about log2(nblk) + 2 short
 * launches, resolves them; then the cells become bytes in d_out.  d_work: device scratch of
 * dmx_inflate_chained_work(out_cap, nblk) bytes (about 10 per output byte), 256-byte aligned.  Status in d_status (out_len =
 * bytes decoded; a reference before the output start is -E_HUFDIS).  out_cap is a capacity:
 * only the ranges the index lists are written.  Returns 0 or -E_*. */
uint64_t dmx_inflate_chained_work(uint64_t out_cap, uint32_t nblk);
int dmx_inflate_chained_async(const void* d_z, uint64_t zbytes, const dmx_iblock* d_index, uint32_t nblk, void* d_out,
                              uint64_t out_cap, void* d_work, uint64_t work_bytes, dmx_inflate_status* d_status,
                              void* stream);
/* Diagnostic: the total length of the reference lists of the last chained decode that used
 * d_work -- host[0] after the prep kernel, host[r + 1] after jump launch r (n <= 41 entries;
 * synchronizes the stream).  Returns 0 or -E_*. */
int dmx_inflate_chained_lists(const void* d_work, uint32_t* host, uint32_t n, void* stream);

/* Introspection of the last encode of ctx (tests / fd_stats): per-block token
 * counts and the token stream (t = byte | dist << 9 | len),
 * per-block BTYPE, and the lit/len + distance code lengths (286 + 30 per block). */
int dmx_last_blocks(dmx_ctx* ctx, uint32_t* ntok, uint8_t* btype, uint32_t* hdr_bits,
                    uint32_t nblk_cap);
int dmx_last_tokens(dmx_ctx* ctx, uint32_t blk, uint32_t* tok, uint32_t cap);
int dmx_last_code_lengths(dmx_ctx* ctx, uint32_t blk, uint8_t* lens316);
/* DEFLATE block `sub` of sw block `blk` (DMX_F_SPLIT emits up to 4 per sw block):
 * token range [tok_range[0], tok_range[1]), BTYPE, header bits, and its 286 + 30 code
 * lengths.  Returns the number of DEFLATE blocks of `blk`, or -E_RANGE. */
int dmx_last_subblock(dmx_ctx* ctx, uint32_t blk, uint32_t sub, uint32_t* tok_range, uint32_t* btype,
                      uint32_t* hdr_bits, uint8_t* lens316);

/* Per-kernel HIP-event timing of subsequent encodes on the context's launches
 * (bench): enable, then read the mean milliseconds per launch of each stage
 * {chain, match, huff, scan, pack} and of the whole encode, and the number of timed encodes.
 * enable: 0 off, 1 every stage boundary, 0x100 | s only stage s's two events (s = 0..4; the
 * other stages and the whole encode read 0), and with | every << 12 (every = 2..255) on
 * every `every`-th encode only.  Each event record costs a few microseconds of idle
 * between kernels. */
int dmx_ctx_set_timing(dmx_ctx* ctx, int enable);
int dmx_ctx_stage_times(dmx_ctx* ctx, double* ms6, uint32_t* count);

/* Diagnostic: per-block match-kernel phase stamps (cycles) of the last encode, when the
 * process runs with DMX_STAMPS=1: 16 x u64 per block (see dmx_kernels.hip). */
int dmx_debug_stamps(dmx_ctx* ctx, uint64_t* out16, uint32_t nblk);

/* The reference's estimate fields of struct compress_stats (DMX_STATS=ref, the default of
 * deflate_compress's fd_stats channel): a host restatement of its two adaptive Huffman trees
 * and code-length pricing (csrc/dmx_refstats.c).  create() starts a stream (the end-of-block
 * code counted once, deflate_compress.c:234); feed() takes tokens in stream order (t = byte,
 * or dist << 9 | len) and fills rec[k].tree_bits / ll_bits / d_bits after token k (the other
 * fields untouched).  Returns 0, -E_INVAL, or -E_RANGE at the first token whose fields would
 * exceed INT_MAX or that is not a valid token; *nfilled = records filled.  Host only. */
typedef struct dmx_refest dmx_refest;
dmx_refest* dmx_refest_create(void);
void dmx_refest_destroy(dmx_refest* e);
int dmx_refest_feed(dmx_refest* e, const uint32_t* tok, uint32_t ntok, struct compress_stats* rec,
                    uint32_t* nfilled);

/* Adler-32 combine (RFC 1950 math): adler of A||B from adler(A), adler(B), len(B). */
uint32_t dmx_adler32_combine(uint32_t a, uint32_t b, uint64_t len_b);

/* Seeded synthetic inputs for the bench/tests (host, deterministic). */
void dmx_gen_text(uint8_t* buf, uint64_t n, uint64_t seed);    /* enwik-style wiki text */
void dmx_gen_random(uint8_t* buf, uint64_t n, uint64_t seed);  /* splitmix64 bytes */

#ifdef __cplusplus
}
#endif
#endif /* DMX_H */
