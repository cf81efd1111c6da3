/*
 * storb_rs.h -- C ABI of the MI355X-native Storb Reed-Solomon path.
 *
 * This is the drop-in boundary for the chunk->shard erasure stage of
 * crates/storb_base (reference @2025-08-01). Storb calls the external crate
 * zfec-rs @3f3a3720 through exactly three entry points:
 *
 *   zfec_rs::Fec::new(k, m)           crates/storb_base/src/piece.rs:328,383
 *   zfec_rs::Fec::encode(&[u8])       crates/storb_base/src/piece.rs:329
 *   zfec_rs::Fec::decode(&Vec<Chunk>, padlen)
 *                                     crates/storb_base/src/piece.rs:384-386
 *   zfec_rs::Chunk::new(data, index)  crates/storb_base/src/piece.rs:375,378
 *
 * A zfec-rs-compatible Rust shim patched in through the
 * workspace [patch] table maps those onto the functions below, so piece.rs,
 * storb_validator and storb_miner compile unchanged. The storb sizing
 * helpers (piece.rs:292-317) are exported too so every binding computes
 * (k, m, B) identically.
 *
 * Notation: n = total share count = Storb's `m` (EncodedChunk.m, "Total
 * blocks (data + parity)", piece.rs:190-191); n - k = parity shares. The
 * headline "RS(k=4, m=2)" is k = 4, n = 6.
 *
 * Conventions: plain C types only; the caller owns every buffer; nothing
 * here allocates or frees caller memory. Functions are thread-safe; a
 * context serialises the calls made on it (use one context per thread for
 * concurrency). Device pointers are HIP device memory of the context's GPU.
 */
#ifndef STORB_RS_H
#define STORB_RS_H

#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

/* Error codes. zfec-rs returns Err(..) that the reference `.expect()`s
 * (piece.rs:328-329,383-386): a shim maps any nonzero code to Err. */
#define STORB_RS_OK 0
#define STORB_RS_EINVAL 1     /* k < 1, k > n, n > 256, len == 0, bad index */
#define STORB_RS_ENOTENOUGH 2 /* fewer than k distinct shares */
#define STORB_RS_EDEVICE 3    /* HIP runtime failure (see storb_rs_last_error) */
#define STORB_RS_ENOMEM 4     /* device or pinned allocation failed */
#define STORB_RS_ENODEV 5     /* no usable gfx950 device */
#define STORB_RS_EAGAIN 6     /* storb_rs_op_test: the op's device work is still running */
#define STORB_RS_EBUSY 7      /* 64 unfinished async ops on the context already */
#define STORB_RS_ECLOSED 8    /* the async op's context was destroyed before storb_rs_op_finish */

#define STORB_RS_MAX_SHARES 256 /* zfec: n <= 256 */

typedef struct storb_rs_ctx storb_rs_ctx;

/* ---- library / context --------------------------------------------- */
const char *storb_rs_version(void);
const char *storb_rs_strerror(int code);
/* Number of HIP devices visible (0 when none; never an error). */
int storb_rs_device_count(void);
/* NUMA node of the host socket device `device` hangs off (sysfs), -1 if
 * unknown. A caller's thread on another node pays the socket link on every
 * pageable single call (host copies into the page-locked staging, which the
 * runtime places near the device): pin upload / download tasks there. */
int storb_rs_device_numa_node(int device);
/* device_ordinal >= 0 pins the context to that GPU; -1 picks devices
 * round-robin across contexts (objects partition across GPUs), among the GPUs
 * on the calling thread's NUMA node when it has any (storb_rs_select_device;
 * STORB_RS_NUMA_PICK=0 deals out all GPUs regardless of node). */
int storb_rs_ctx_create(int device_ordinal, storb_rs_ctx **out);
/* The rule storb_rs_ctx_create(-1) applies, as a pure function (no device
 * access; bindings and tests call it with any topology): the device that the
 * `ticket`-th context of a thread on `caller_node` gets, given each device's
 * node in device_nodes[0..ndev). Round-robin over the devices on caller_node;
 * over all devices when the caller's node is unknown (< 0) or has none.
 * -1 when ndev <= 0. */
int storb_rs_select_device(int caller_node, const int *device_nodes, int ndev,
                           uint64_t ticket);
/* Waits for everything the context queued, returns its device memory
 * (stream-ordered pool memory included) and frees it. Async ops started on
 * it and not yet finished are waited for and detached: storb_rs_op_test and
 * storb_rs_op_finish on them return STORB_RS_ECLOSED without touching the
 * destroyed context (finish still frees the op; outputs staged for finish
 * are not written). */
void storb_rs_ctx_destroy(storb_rs_ctx *ctx);
int storb_rs_ctx_device(const storb_rs_ctx *ctx);
/* Detail of the last failure on this context ("" if none). */
const char *storb_rs_last_error(const storb_rs_ctx *ctx);
/* Counters of a context (diagnostics, tests). */
typedef struct {
  uint64_t streamed_calls;   /* single calls completed on the streamed path */
  uint64_t stream_fallbacks; /* streamed attempts a workgroup gave up on (redone sliced) */
  uint64_t sliced_calls;     /* single calls on the column-sliced path */
  uint64_t live_ops;         /* async ops started and not finished */
  uint64_t tables;           /* cached coefficient tables */
  uint64_t device_syncs;     /* device-wide syncs the stream-ordering fallbacks took (rare) */
  int32_t caller_node;       /* NUMA node of the thread that created the context, -1 unknown */
  int32_t device_node;       /* NUMA node of the context's GPU, -1 unknown */
} storb_rs_ctx_stats_t;
int storb_rs_ctx_stats(const storb_rs_ctx *ctx, storb_rs_ctx_stats_t *out);
/* Bytes in use / reserved in the device's default stream-ordered memory pool
 * (where the contexts' coefficient tables live, hipMallocAsync): a destroyed
 * context leaves "used" where it found it. */
int storb_rs_device_pool_stats(int device, uint64_t *used, uint64_t *reserved);

/* ---- code parameters (host only, no GPU needed) ----------------------- */
/* zfec-rs Fec::new validation: STORB_RS_OK or STORB_RS_EINVAL. */
int storb_rs_check_params(uint32_t k, uint32_t n);
/* The n*k systematic generator (rows 0..k-1 identity), row-major. */
int storb_rs_enc_matrix(uint32_t k, uint32_t n, uint8_t *out_nk);
/* Shard size zfec uses for a chunk of len bytes: ceil(len / k). */
size_t storb_rs_block_size(uint32_t k, size_t len);
/* piece.rs:292-303 piece_length(); min_size/max_size 0 = the constants
 * of crates/storb_base/src/constants.rs:5-6 (16 KiB, 256 MiB). */
uint64_t storb_piece_length(uint64_t content_length, uint64_t min_size,
                            uint64_t max_size);
/* piece.rs:307-317 get_k_and_m(): k data shares, m TOTAL shares. */
void storb_get_k_and_m(uint64_t chunk_size, uint64_t *k, uint64_t *m);

/* ---- host-in / host-out (zfec-rs Fec::encode / Fec::decode) ----------- */
/* Encode one chunk: B = ceil(len/k), padlen = k*B - len. Writes the n-k
 * parity shares (B bytes each) to parity_out[0..n-k). Data shares are the
 * caller's own slices data[i*B, (i+1)*B) zero-padded (systematic code), so
 * only parity crosses back. block_out / padlen_out may be NULL. */
int storb_rs_encode(storb_rs_ctx *ctx, uint32_t k, uint32_t n,
                    const uint8_t *data, size_t len,
                    uint8_t *const *parity_out, size_t *block_out,
                    size_t *padlen_out);
/* zfec-rs Fec::encode's full result (piece.rs:329: all m shares in index
 * order): shares_out[0..k) receive the data shares (B bytes each, the last
 * zero-padded), shares_out[k..n) the parity. The data shares are copied by
 * the host copy pool while the kernel computes the parity, so a shim that
 * must return every share pays no serial copy of its own. */
int storb_rs_encode_shares(storb_rs_ctx *ctx, uint32_t k, uint32_t n,
                           const uint8_t *data, size_t len,
                           uint8_t *const *shares_out, size_t *block_out,
                           size_t *padlen_out);
/* Decode one chunk from nshares >= k shares (any order). Selection follows
 * decode_chunk (piece.rs:368-381): sort by index, keep the first k. Writes
 * k*block - padlen bytes to out. */
int storb_rs_decode(storb_rs_ctx *ctx, uint32_t k, uint32_t n,
                    const uint8_t *const *shares, const uint32_t *share_idx,
                    uint32_t nshares, size_t block, size_t padlen,
                    uint8_t *out);

/* Host-in/host-out repair of one stripe: shares[i] (block bytes) is share
 * share_idx[i]; share targets[r] is written to out[r] (block bytes). */
int storb_rs_repair(storb_rs_ctx *ctx, uint32_t k, uint32_t n,
                    const uint8_t *const *shares, const uint32_t *share_idx,
                    uint32_t nshares, size_t block, const uint32_t *targets,
                    uint32_t ntargets, uint8_t *const *out);

/* Pipelined host batch: nchunks equal-length chunks laid out back to back
 * in host memory (chunk c at data + c*chunk_len). Parity of chunk c, share
 * p lands at parity_out + (c*(n-k) + p)*B. Uses pinned staging and
 * overlapped H2D / kernel / D2H on the context's streams. */
int storb_rs_encode_chunks(storb_rs_ctx *ctx, uint32_t k, uint32_t n,
                           const uint8_t *data, size_t chunk_len,
                           uint32_t nchunks, uint8_t *parity_out);
/* Same, plus every share's blake3 piece id (upload.rs:623) computed on the
 * GPU where the shares already are: hashes_out + (c*n + i)*32 receives the
 * digest of share i (data i < k, parity i >= k) of chunk c. Data shares
 * never travel back over PCIe; only their 32-byte ids do. */
int storb_rs_encode_chunks_hashed(storb_rs_ctx *ctx, uint32_t k, uint32_t n,
                                  const uint8_t *data, size_t chunk_len,
                                  uint32_t nchunks, uint8_t *parity_out,
                                  uint8_t *hashes_out);

/* Pipelined host batch decode, the download side (download.rs:453-465
 * reconstructs one chunk after another): nchunks chunks of one (k, n, block,
 * padlen), e.g. an object's full-size chunks. Chunk c offers nshares[c]
 * shares: shares[o_c + i] is share share_idx[o_c + i], o_c = nshares[0] +
 * ... + nshares[c-1]. Per chunk the first k by index are used (decode_chunk,
 * piece.rs:368-381); its k*block - padlen bytes land at out + c*out_stride
 * (out_stride 0 = packed). ENOTENOUGH if any chunk has fewer than k
 * distinct shares (reconstruct_chunk's Err, piece.rs:462-473); nothing is
 * guaranteed written then. */
int storb_rs_decode_chunks(storb_rs_ctx *ctx, uint32_t k, uint32_t n,
                           size_t block, size_t padlen, uint32_t nchunks,
                           const uint8_t *const *shares,
                           const uint32_t *share_idx, const uint32_t *nshares,
                           uint8_t *out, size_t out_stride);

/* ---- page-locked host memory ------------------------------------------ */
/* Storb fills a chunk buffer from the upload body (upload.rs:333-383) and
 * hands it to encode_chunk (upload.rs:420). When that buffer -- and the
 * buffer parity lands in -- is page-locked, storb_rs_encode_chunks DMAs it
 * directly (no staging copy through the context's own pinned buffers).
 * Memory from storb_rs_host_alloc, or a caller range made page-locked with
 * storb_rs_host_register, qualifies; the check is by address range. */
int storb_rs_host_alloc(size_t len, void **out);
/* storb_rs_host_free / _unregister wait for every device of the process
 * before the range is unmapped (a kernel may still be reading it). */
int storb_rs_host_free(void *p); /* only pointers from storb_rs_host_alloc */
int storb_rs_host_register(void *p, size_t len);
int storb_rs_host_unregister(void *p);
/* 1 if [p, p+len) lies inside one range above, else 0. */
int storb_rs_host_is_pinned(const void *p, size_t len);

/* ---- device-resident batched variants -------------------------------- */
/* Stripe s, data share j lives at d_data + s*data_stride + j*block; parity
 * share p at d_parity + s*parity_stride + p*block. Strides of 0 mean the
 * packed defaults k*block and (n-k)*block. Asynchronous on `hip_stream`
 * (a hipStream_t; NULL = the HIP null stream, which orders with the
 * device's legacy default stream). The context records an order event on
 * `hip_stream` only now and then (every few calls), never on a stream it is
 * not being called with: a caller may destroy its stream once the work on it
 * has completed, and a context resource last used there is then reclaimed
 * after a device synchronisation. */
int storb_rs_encode_batch_dev(storb_rs_ctx *ctx, uint32_t k, uint32_t n,
                              size_t block, uint32_t nstripes,
                              const uint8_t *d_data, size_t data_stride,
                              uint8_t *d_parity, size_t parity_stride,
                              void *hip_stream);
/* Reconstruct the data shares of nstripes stripes that all lost the same
 * shares. share_idx lists the nshares >= k surviving share indices (first k
 * by index are used). Survivor i < k is read from the data region, i >= k
 * from the parity region. Only the missing data rows are computed (zfec).
 * They are written into d_out (same layout as d_data, stride out_stride);
 * when d_out != d_data the surviving data shares are copied there as well,
 * when d_out == d_data the reconstruction is in place. */
int storb_rs_decode_batch_dev(storb_rs_ctx *ctx, uint32_t k, uint32_t n,
                              size_t block, uint32_t nstripes,
                              const uint32_t *share_idx, uint32_t nshares,
                              const uint8_t *d_data, size_t data_stride,
                              const uint8_t *d_parity, size_t parity_stride,
                              uint8_t *d_out, size_t out_stride,
                              void *hip_stream);
/* Reconstruct nstripes stripes that each lost different shares -- Storb's
 * download: per chunk the first k + 1 pieces to ARRIVE from 10 fetch threads
 * are kept (crates/storb_validator/src/download.rs:363-451), then
 * decode_chunk sorts them and uses the first k by index (piece.rs:368-381),
 * so the survivor set varies from chunk to chunk. Stripe s offers nshares[s]
 * shares, share_idx[o_s .. o_s + nshares[s]) with o_s = nshares[0] + ... +
 * nshares[s-1]. Layout and d_out semantics as storb_rs_decode_batch_dev.
 * One launch over every stripe that lost up to 4 data shares (each workgroup
 * reads its own stripe's pattern and runs the tile of its own row count),
 * plus one per larger missing-row count -- never one per pattern.
 * ENOTENOUGH names the stripe. */
int storb_rs_decode_stripes_dev(storb_rs_ctx *ctx, uint32_t k, uint32_t n,
                                size_t block, uint32_t nstripes,
                                const uint32_t *share_idx, const uint32_t *nshares,
                                const uint8_t *d_data, size_t data_stride,
                                const uint8_t *d_parity, size_t parity_stride,
                                uint8_t *d_out, size_t out_stride,
                                void *hip_stream);
/* Decode-based repair. Storb's repair today re-fetches a
 * lost piece from another replica (crates/storb_validator/src/repair.rs:
 * 44-277); with RS it can instead regenerate any share row -- data or
 * parity -- from the first k surviving shares by index (the same survivor
 * rule as decode_chunk, piece.rs:368-381). Layout as decode_batch_dev; the
 * ntargets shares in targets[] are written in place into their own region.
 * EINVAL if a target is >= n, repeated, or one of the k shares read. */
int storb_rs_repair_batch_dev(storb_rs_ctx *ctx, uint32_t k, uint32_t n,
                              size_t block, uint32_t nstripes,
                              const uint32_t *share_idx, uint32_t nshares,
                              const uint32_t *targets, uint32_t ntargets,
                              uint8_t *d_data, size_t data_stride,
                              uint8_t *d_parity, size_t parity_stride,
                              void *hip_stream);
/* The primitive under both: out_r = XOR_j coef[r*k + j] * in_j over GF(2^8)
 * for r < rows, for every stripe (shard s of slot j at d_in[j] +
 * s*in_stride[j]). Serves repair (regenerate any share row). */
int storb_rs_apply_dev(storb_rs_ctx *ctx, uint32_t k, uint32_t rows,
                       const uint8_t *coef, const uint8_t *const *d_in,
                       const size_t *in_stride, uint8_t *const *d_out,
                       const size_t *out_stride, size_t block,
                       uint32_t nstripes, void *hip_stream);

/* ---- shard identity: BLAKE3 (hash mode, 32-byte digest) --------------- */
/* Storb names every shard by blake3(shard bytes): upload.rs:623,
 * crates/storb_miner/src/lib.rs:265-283, download.rs:158-161 (crate blake3
 * 1.8.2, reference Cargo.lock:1099). Host one-shot hash: */
void storb_blake3(const uint8_t *data, size_t len, uint8_t out[32]);
/* Device batch: message i = len bytes at d_in + i*stride (i < count); digest
 * i -> d_out + 32*i (device memory). len <= 16 MiB. Hashes the shards where
 * the encode kernel left them: data shares of N packed stripes are
 * (d_data, B, N*k, stride B), parity shares (d_parity, B, N*(n-k), B). */
int storb_rs_blake3_batch_dev(storb_rs_ctx *ctx, const uint8_t *d_in, size_t len,
                              uint32_t count, size_t stride, uint8_t *d_out,
                              void *hip_stream);

/* Encode with the piece ids (upload.rs:623 hashes every piece
 * right after encode_chunk): layout as storb_rs_encode_batch_dev, and the
 * blake3 digest of share t of stripe s (t < k data, then parity) at
 * d_hashes + (s*n + t)*32. (k, n) = (2, 3) / (4, 6) with block a multiple of
 * 1 KiB up to 256 KiB and 16-B aligned pointers run one kernel that hashes
 * every share while it encodes (each byte crosses HBM once); other
 * geometries run the encode kernel, then the hash kernel. */
int storb_rs_encode_hashed_dev(storb_rs_ctx *ctx, uint32_t k, uint32_t n,
                               size_t block, uint32_t nstripes,
                               const uint8_t *d_data, size_t data_stride,
                               uint8_t *d_parity, size_t parity_stride,
                               uint8_t *d_hashes, void *hip_stream);

/* ---- synthetic input (benchmarks / tests) ----------------------------- */
/* Object o (o < nobj) at d + o*obj_stride gets obj_len bytes of the
 * little-endian splitmix64 stream seeded with seed_base + o. */
int storb_rs_fill_splitmix_dev(storb_rs_ctx *ctx, uint8_t *d, size_t obj_len,
                               uint32_t nobj, size_t obj_stride,
                               uint64_t seed_base, void *hip_stream);

/* Which kernel variant the calls launch. AUTO (default): encodes of
 * (k, n) = (16, 24) and (32, 48) -- Storb's geometry for 8-32 MiB chunks --
 * run the bit-sliced encoder with the generator compiled in, everything else
 * the register-table kernel. PERM / LDS force that table kernel for every
 * call (benchmarks and the identical-output tests use them). */
#define STORB_RS_KERNEL_AUTO 0
#define STORB_RS_KERNEL_PERM 1 /* nibble tables in registers, v_perm_b32 */
#define STORB_RS_KERNEL_LDS 2  /* 256-B product tables staged in LDS */
int storb_rs_set_kernel(storb_rs_ctx *ctx, int variant);

/* Run-time-compiled bit-sliced kernels. Decode and repair apply rows of the
 * inverted survivor matrix, known only when the erasure pattern is. Under
 * AUTO, a matrix the table kernel is measured slower on (k >= 12 with >= 2
 * rows, k = 8..11 with >= 6, k <= 64, up to 32 rows as launches of <= 16;
 * batches >= 4 MiB)
 * gets its own bit-sliced kernel, compiled with hipRTC on a background thread
 * once the same matrix has been asked for twice, and cached; calls made
 * before or while it compiles run the table kernel. STORB_RS_JIT=0 disables,
 * =sync compiles before the first launch; STORB_RS_JIT_MAX caps the kernels
 * loaded at once (default 256; past it the least recently used idle one is
 * unloaded). storb_rs_decode_stripes_dev / decode_chunks with mixed patterns
 * use the per-stripe table kernel and compile nothing. */
typedef struct {
  uint64_t compiled;  /* kernels compiled and cached */
  uint64_t failed;    /* compiles that failed (those matrices use the table kernel) */
  uint64_t pending;   /* compiles queued or running */
  uint64_t launches;  /* launches of compiled kernels */
  uint64_t fallbacks; /* wanted a compiled kernel, ran the table kernel */
  double compile_ms;  /* total compile wall time */
  uint64_t evicted;   /* kernels unloaded to make room (LRU, idle ones only) */
  uint64_t loaded;    /* kernels currently cached (<= STORB_RS_JIT_MAX) */
  uint64_t refused;   /* compiled, but refused before loading: the code object
                       * makes a function call (storb_rs_code_object_calls);
                       * counted in `failed` too, so those matrices use the
                       * table kernel */
} storb_rs_jit_stats_t;
int storb_rs_jit_stats(storb_rs_jit_stats_t *out);
/* Whether a gfx950 code object (a raw ELF, as hipRTC returns it) has a kernel
 * that makes a function call: 1 (why[] names it), 0 none, -1 unreadable. The
 * library runs it on every run-time compiled kernel before loading it; an
 * out-of-line call is how a round-4 decode kernel hung.
 * Needs no device. */
int storb_rs_code_object_calls(const void *code, size_t len, char *why, size_t why_len);
/* Block until no compile is pending (benchmarks and tests). */
int storb_rs_jit_wait(void);
/* Ahead of the calls: queue (wait != 0: finish) the compile of the decode
 * kernel for one erasure pattern -- the shares offered, first k by index as
 * in decode_batch_dev; assemble != 0 for a decode into a separate chunk
 * buffer, 0 for in place. Only matrices the policy above wants are compiled
 * (the call is a no-op otherwise). Needs no GPU. EDEVICE if the compile
 * failed. */
int storb_rs_jit_prepare_decode(uint32_t k, uint32_t n, const uint32_t *share_idx,
                                uint32_t nshares, int assemble, int wait);

/* Asynchronous single-chunk calls. The reference calls encode_chunk /
 * decode_chunk synchronously inside async tasks (upload.rs:418-420,
 * download.rs:464; SURVEY 8(b) names an async variant as the next step); these
 * let an integration await the GPU instead of blocking a worker thread.
 * Arguments and results are those of storb_rs_encode / storb_rs_decode. The
 * call validates, copies the input into page-locked staging of the op's own
 * (the caller may reuse `data` / `shares` as soon as it returns), queues the
 * kernel on a stream of the op's own and returns; block_out / padlen_out are
 * set at once. The output buffers must stay valid until storb_rs_op_finish.
 * notify(user), if not NULL, is called exactly once when the op's device work
 * is done -- from a HIP runtime thread (it must only wake a waiter: no calls
 * into this library or HIP), or before the call returns when there is no
 * device work (k = 1, nothing missing). storb_rs_op_test polls (STORB_RS_OK
 * when done, STORB_RS_EAGAIN while running); storb_rs_op_finish waits if
 * needed, writes the outputs, frees the op and returns its result. Finish
 * every op exactly once, before destroying its context (an op outliving its
 * context finishes with STORB_RS_ECLOSED, see storb_rs_ctx_destroy). Ops of a context run
 * concurrently (one stream and staging slot each, reused after finish); with
 * 64 unfinished the call returns STORB_RS_EBUSY. On any error no op is
 * returned. */
typedef struct storb_rs_op storb_rs_op;
typedef void (*storb_rs_notify_fn)(void *user);
int storb_rs_encode_async(storb_rs_ctx *ctx, uint32_t k, uint32_t n, const uint8_t *data,
                          size_t len, uint8_t *const *parity_out, size_t *block_out,
                          size_t *padlen_out, storb_rs_notify_fn notify, void *user,
                          storb_rs_op **op);
int storb_rs_decode_async(storb_rs_ctx *ctx, uint32_t k, uint32_t n,
                          const uint8_t *const *shares, const uint32_t *share_idx,
                          uint32_t nshares, size_t block, size_t padlen, uint8_t *out,
                          storb_rs_notify_fn notify, void *user, storb_rs_op **op);
int storb_rs_op_test(const storb_rs_op *op);
int storb_rs_op_finish(storb_rs_op *op);
/* A notify function for the calls above that only wakes a waiter: writes an
 * 8-byte 1 to the eventfd (or pipe) whose descriptor is user, cast from
 * intptr_t. An event loop polls the descriptor (tokio AsyncFd, Python
 * selectors) instead of running code on the HIP runtime thread. */
void storb_rs_notify_fd(void *user);

/* Synchronise the context's own streams and the HIP null stream of its
 * device (where device calls given hip_stream = NULL run). Work the caller
 * queued on streams of its own is the caller's to synchronise. */
int storb_rs_sync(storb_rs_ctx *ctx);

#ifdef __cplusplus
}
#endif
#endif /* STORB_RS_H */
