/*
 * callfs_rs.h — C ABI of the MI355X-native Reed-Solomon erasure-coding path for CallFS.
 *
 * Drop-in boundary for erasure/codec.go: the Go package keeps its API
 * (NewCodec/Encode/Decode, codec.go:15,21,45) and a cgo shim
 * (erasure/codec_rocm.go, //go:build rocm && cgo — see INTEGRATION.md) binds the
 * functions below. All GF(2^8) arithmetic that the reference delegates to
 * github.com/klauspost/reedsolomon v1.13.3 (go.mod:13) runs here as hand-written
 * HIP kernels for gfx950.
 *
 * Conventions
 *  - Every function returns RS_OK (0) or a negative RS_E_* code.
 *  - No pointer passed in is retained after return (cgo pointer rules).
 *  - Host-memory entry points are synchronous (return after the D2H copy lands).
 *  - All entry points are thread-safe; one rs_ctx may be shared by every request
 *    goroutine, like the shared *Codec at erasure/manager.go:60.
 *  - There is no CPU compute fallback: without a usable HIP device rs_init fails
 *    with RS_E_HIP. Profiles with k+m > 256 (upstream switches to Leopard GF(2^16)
 *    in reedsolomon.New, codec.go:26) return RS_E_UNSUPPORTED and the Go shim keeps
 *    the CPU codec for them.
 */
#ifndef CALLFS_RS_H
#define CALLFS_RS_H

#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

#define RS_ABI_VERSION 1

/* ---- error codes (mapped to Go errors by the shim) ---- */
#define RS_OK                 0
#define RS_E_INVALID_PROFILE (-1)  /* erasure.ErrInvalidProfile (errors.go:9; codec.go:22-24,46-48) */
#define RS_E_SHORT_DATA      (-2)  /* reedsolomon.ErrShortData from Split (codec.go:31-34) */
#define RS_E_TOO_FEW_SHARDS  (-3)  /* reedsolomon.ErrTooFewShards from Reconstruct (codec.go:55) */
#define RS_E_SHARD_SIZE      (-4)  /* reedsolomon.ErrShardSize */
#define RS_E_NO_DATA         (-5)  /* reedsolomon.ErrShardNoData */
#define RS_E_CORRUPT         (-6)  /* erasure.ErrShardCorrupted (errors.go:8; codec.go:63-65) */
#define RS_E_INSUFFICIENT    (-7)  /* erasure.ErrInsufficientShards (errors.go:7; codec.go:73-75) */
#define RS_E_UNSUPPORTED     (-8)  /* k+m > 256: Leopard GF(2^16) path, not implemented on GPU */
#define RS_E_HIP             (-9)  /* HIP runtime failure / no device */
#define RS_E_ARG             (-10) /* NULL pointer, short buffer, bad count */
#define RS_E_SINGULAR        (-11) /* reedsolomon.ErrSingular (cannot happen for valid profiles) */
#define RS_E_NOMEM           (-12) /* host or device allocation failed */

typedef struct rs_ctx rs_ctx;
typedef struct rs_plan rs_plan;

/* ---- lifetime ---------------------------------------------------------------------
 * Replaces NewCodec (erasure/codec.go:15-17). device_mask: bit d selects HIP device d;
 * 0 selects every visible device. Host-memory calls are spread over the selected
 * devices (one per call, round-robin). */
int  rs_init(rs_ctx** out, unsigned device_mask);
void rs_shutdown(rs_ctx* ctx);
int  rs_device_count(const rs_ctx* ctx);
int  rs_abi_version(void);
const char* rs_strerror(int code);

/* ---- host-side helpers (no device needed) -------------------------------------------
 * rs_shard_size: S = ceil(len/k) as upstream Split computes it (codec.go:31).
 * rs_encode_matrix: E = V . inv(V[0:k]), (k+m) x k row-major (upstream buildMatrix,
 *   reached via reedsolomon.New at codec.go:26).
 * rs_decode_rows: for a presence mask over n = k+m shards, the first k present
 *   indices (valid), the missing indices, and the rows over the valid shards that
 *   produce every missing shard (data rows of inv(E[valid]); parity rows
 *   P[j].inv(E[valid])), as upstream Reconstruct computes them (codec.go:55).
 *   valid_out: k ints; missing_out: n ints; rows_out: n*k bytes (n_missing*k used). */
int rs_shard_size(int k, int m, int64_t len, int64_t* shard_size);
int rs_encode_matrix(int k, int m, uint8_t* out);
int rs_decode_rows(int k, int m, const uint8_t* present, int* valid_out, int* missing_out,
                   int* n_missing, uint8_t* rows_out);

/* ---- Codec-level, host memory (the cgo shim's two calls) ----------------------------
 * rs_codec_encode replaces Codec.Encode (erasure/codec.go:21-41): Split + Encode.
 *   Writes n = k+m shards of S = ceil(len/k) bytes back to back into shards_out
 *   (shard i at offset i*S; needs out_cap >= n*S). *shard_size receives S.
 *   len == 0 -> RS_E_SHORT_DATA (upstream Split).
 * rs_codec_decode replaces Codec.Decode (erasure/codec.go:45-78): Reconstruct + Verify
 *   + join + trim. shards[i] points to a buffer of at least S bytes for every i;
 *   lens[i] is that shard's length, 0 meaning missing (nil in Go). Missing shards are
 *   reconstructed INTO shards[i] and lens[i] is set to S (Decode mutates its shards
 *   argument in Go). out receives original_size bytes.
 *   Error precedence follows codec.go: profile, shard count/size, too few, corrupt,
 *   insufficient. */
int rs_codec_encode(rs_ctx* ctx, int k, int m, const uint8_t* data, size_t len,
                    uint8_t* shards_out, size_t out_cap, size_t* shard_size);
int rs_codec_decode(rs_ctx* ctx, int k, int m, uint8_t* const* shards, size_t* lens,
                    uint8_t* out, int64_t original_size);

/* ---- pinned host buffers: zero-copy staging -----------------------------------------
 * rs_host_alloc returns `bytes` of page-locked host memory (page-aligned) that the
 * host-memory entry points above and below DMA from and to directly. When every shard
 * buffer of a call (and, for rs_codec_decode, `out`) lies inside such allocations, the
 * call skips the library's CPU copy through its own pinned staging: H2D, kernels and
 * D2H run on the caller's bytes, and the CPU only enqueues. A server reads request
 * bodies and backend shards straight into these buffers. Calls with any
 * other buffer use the copy-pool staging path as before. Free with rs_host_free
 * (RS_E_ARG for a pointer rs_host_alloc did not return or that was already freed).
 * Freed buffers are kept by the context for reuse: fresh buffers are allocated in 2 MiB
 * granules, and a later rs_host_alloc returns the smallest kept buffer that fits without
 * wasting more than a quarter of it, both sides counted in granules (so a 4 KiB body
 * freed by one request serves the next), without page-locking new memory; a server may
 * allocate a body per request (CALLFS_RS_HOST_POOL_BYTES caps the idle bytes kept,
 * default 4 GiB, 0 = keep none; rs_shutdown releases them). No reference equivalent: Go's
 * io.ReadAll allocations (post_file_enhanced.go:127, manager.go:473,530) are what it
 * replaces on a ROCm build. */
int rs_host_alloc(rs_ctx* ctx, size_t bytes, void** out);
int rs_host_free(rs_ctx* ctx, void* p);

/* ---- Encoder-level, host memory (reedsolomon.Encoder methods used by codec.go) -----
 * rs_encode:      enc.Encode(shards)      (codec.go:36)  data: k ptrs, parity: m ptrs, S bytes each
 * rs_reconstruct: enc.Reconstruct(shards) (codec.go:55)  same buffer/lens contract as rs_codec_decode
 * rs_verify:      enc.Verify(shards)      (codec.go:59)  *ok = 1 when parity matches */
int rs_encode(rs_ctx* ctx, int k, int m, size_t S, const uint8_t* const* data,
              uint8_t* const* parity);
int rs_reconstruct(rs_ctx* ctx, int k, int m, uint8_t* const* shards, size_t* lens);
int rs_verify(rs_ctx* ctx, int k, int m, const uint8_t* const* shards, const size_t* lens,
              int* ok);

/* ---- Batched, host memory (many independent stripes per call) ----------------------
 * Not in the reference API: for callers holding many objects at once (repair of every
 * object that lost one shard, bulk re-encode, a server batching small uploads). Stripes
 * are grouped by (S, presence) and each group runs one pipeline in which small stripes
 * are packed many per H2D / launch / D2H, so a batch of 4 KiB objects costs a few round
 * trips instead of one per object.
 * rs_encode_batch: stripe b has sizes[b]-byte shards, data[b*k + i] / parity[b*m + j]
 *   (= rs_encode per stripe, codec.go:36). sizes[b] == 0 -> status[b] = RS_E_NO_DATA.
 * rs_reconstruct_batch: shards[b*n + i] / lens[b*n + i] with rs_reconstruct's contract
 *   per stripe (codec.go:55); verify != 0 also re-checks the present parity beyond the
 *   first k (codec.go:59) -> status[b] = RS_E_CORRUPT for that stripe alone.
 * status[b] receives each stripe's code (RS_OK, RS_E_NO_DATA, RS_E_SHARD_SIZE,
 * RS_E_TOO_FEW_SHARDS, RS_E_ARG, RS_E_CORRUPT). Returns RS_OK when every stripe is OK,
 * else the first nonzero status in stripe order; a call-level error (RS_E_ARG,
 * RS_E_INVALID_PROFILE, RS_E_HIP, RS_E_NOMEM) is returned directly with status[]
 * unspecified. */
int rs_encode_batch(rs_ctx* ctx, int k, int m, int batch, const size_t* sizes,
                    const uint8_t* const* data, uint8_t* const* parity, int* status);
int rs_reconstruct_batch(rs_ctx* ctx, int k, int m, int batch, uint8_t* const* shards,
                         size_t* lens, int verify, int* status);

/* ---- device-resident plans (batched stripes, graph-capturable launches) -------------
 * A plan fixes (k, m, S, batch, presence mask) and the device pointers of every
 * stripe's n shards: shards[b*n + i] is shard i of stripe b (device memory, S bytes).
 * present == NULL means "encode" (data present, parity missing). Launching a plan
 * computes every missing shard of every stripe from the first k present ones and
 * re-checks the remaining present parity (the Verify of codec.go:59), OR-ing 1 into
 * the plan's device status word on mismatch. rs_plan_launch only enqueues work on
 * `stream` (a hipStream_t; NULL = the null stream) — no allocation, no sync.
 * rs_plan_status synchronises `stream`, sets *corrupt when any stripe's verify rows
 * mismatched since the last status call, and clears the flags;
 * rs_plan_stripe_status does the same per stripe (flags: `batch` ints, nonzero =
 * that object is corrupt — ErrShardCorrupted for it alone). rs_plan_bytes: algorithmic
 * HBM bytes one launch moves (reads of the k+verify inputs + writes of the missing
 * shards). */
int  rs_plan_create(rs_ctx* ctx, int device, int k, int m, size_t S, int batch,
                    const uint8_t* present, uint8_t* const* shards, rs_plan** out);
int  rs_plan_launch(rs_plan* plan, void* stream);
int  rs_plan_status(rs_plan* plan, void* stream, int* corrupt);
int  rs_plan_stripe_status(rs_plan* plan, void* stream, int* flags);
/* rs_plan_launch that also times its kernels (measurement; no upstream counterpart):
 * start_event / stop_event (hipEvent_t, created by the caller, either may be NULL) are
 * recorded by the launch's first kernel dispatch when it starts and by its last when it
 * ends (hipExtLaunchKernel), so hipEventElapsedTime gives the kernels' own time, without
 * the stream's gap before the first and after the last (what rocprofv3's kernel trace
 * reports). */
int  rs_plan_launch_timed(rs_plan* plan, void* stream, void* start_event, void* stop_event);
uint64_t rs_plan_bytes(const rs_plan* plan);
void rs_plan_destroy(rs_plan* plan);

/* Tile-order tuning (no upstream counterpart; an autotuner for repeated launches).
 * Which order of column tiles HBM serves best for a shape varies between MI355X boxes
 * by 1-2 %. rs_plan_tune warms the device up in the rule's order (~150 ms
 * of launches), then times each launch group of the plan in every
 * tile order its kernel offers (`reps` launches per order, three rounds) and keeps the
 * fastest for later rs_plan_launch calls; the measured rule's order stays unless another
 * is > 1 % faster. Synchronous on `stream`; RS_E_ARG while `stream` is capturing. The
 * tuning launches recompute the plan's outputs from its inputs (same bytes; Verify rows
 * may flag status exactly as rs_plan_launch would). orders (NULL when max_groups == 0):
 * the chosen order per launch group, up to max_groups entries (RS_ORDER_* or -1 = the
 * launch has no choice). */
#define RS_ORDER_CONSECUTIVE 0
#define RS_ORDER_GROUP8 1
#define RS_ORDER_GROUP2 2
#define RS_ORDER_SEG8 3
#define RS_ORDER_SEG16 4
/* consecutive tiles, J = 8 / 32 of them per XCD in turn */
#define RS_ORDER_XCD8 5
#define RS_ORDER_XCD32 6
/* misaligned shards (upstream Split layout at odd S): the kernel that realigns loads and
 * parity stores in registers, RS_ORDER_REALIGN + the tile order it runs in (consecutive,
 * XCD8 or XCD32); on such launches RS_ORDER_0..6 name the plain kernel with unaligned
 * 16-B accesses in that tile order */
#define RS_ORDER_REALIGN 32
/* the launch group's bit-sliced kernel: an XOR network over bit planes
 * generated for the group's coefficient block and compiled at plan time (hiprtc; cached on
 * disk; past 2,048 coefficients per plan the blocks compile in the background while the plan
 * runs the nibble-table kernels), RS_ORDER_BITSLICE + the tile order it runs in (RS_ORDER_0..6);
 * pinning one waits for its compile */
#define RS_ORDER_BITSLICE 256
int  rs_plan_tune(rs_plan* plan, void* stream, int reps, int* orders, int max_groups);
/* Sets the tile order of launch groups 0..n-1 (the others: the rule) to orders[i], as
 * rs_plan_tune would: RS_ORDER_* that the group's kernel has an instance of (what
 * rs_plan_tune times, and XCD8 / XCD32 on aligned shards), or -1 for the rule. RS_E_ARG if any entry is not offered or n
 * exceeds rs_plan_groups; the plan is then unchanged. For orders tuned once and kept. */
int  rs_plan_set_orders(rs_plan* plan, const int* orders, int n);
/* The kernel form each launch group of the next rs_plan_launch runs, up to max_groups
 * entries: the pinned or tuned order, else the rule's (RS_ORDER_BITSLICE + its tile order
 * where the rule gives the group the bit-sliced kernel; the codes rs_plan_tune reports).
 * Returns the number of launch groups, or RS_E_ARG. */
int  rs_plan_forms(const rs_plan* plan, int* forms, int max_groups);
/* The tune table: every rs_plan_tune records its choice per launch shape
 * (device, k, rows, tiles-per-stripe bucket, address alignment, written / compared rows,
 * misalignment), and launches with no order of their own -- untuned plans, the host-memory
 * calls -- take the recorded form for their shape before the built-in rule. With
 * CALLFS_RS_TUNE_TABLE=<file> the table is read from and written back to that file, so a
 * box is tuned once. rs_tune_table_reset forgets every entry and binds the table to `path`
 * (NULL: CALLFS_RS_TUNE_TABLE, or memory only); rs_tune_table_entries counts them. */
int  rs_tune_table_reset(const char* path);
int  rs_tune_table_entries(void);
/* Measurement only (no upstream counterpart): enqueues the plan's launch groups as a
 * traffic ceiling of the same shape, on the production grid, tile order and slicing, for
 * a roofline denominator measured in the same process (bench.py):
 *   RS_CEIL_READ      the plan's read streams alone (k inputs + compared rows);
 *   RS_CEIL_WRITE     its write streams alone (leaves junk in the written shards:
 *                     relaunch the plan before relying on them).
 * Any other mode returns RS_E_ARG. (The development tools' A/B build, built on demand with
 * `python callfs_amd/build.py --ab`, adds the kernel's no-lookup form and aligned-window
 * probes: tools/callfs_rs_ab.h.) */
#define RS_CEIL_READ 1
#define RS_CEIL_WRITE 2
int  rs_plan_launch_ceiling(rs_plan* plan, void* stream, int mode);
/* The same, with its kernels timed as rs_plan_launch_timed times the plan's. */
int  rs_plan_launch_ceiling_timed(rs_plan* plan, void* stream, int mode, void* start_event,
                                  void* stop_event);
/* Launch groups of a plan (the `orders` entries rs_plan_tune can fill): one per up to 16
 * written or compared rows; 0 for a NULL plan. */
int  rs_plan_groups(const rs_plan* plan);

/* One-shot device-resident calls (build + launch + free; tables cached per profile).
 * Same pointer layout as rs_plan_create; synchronous on `stream`. rs_decode_dev
 * returns RS_E_CORRUPT when the verify rows mismatch. */
int rs_encode_dev(rs_ctx* ctx, int device, int k, int m, size_t S, int batch,
                  uint8_t* const* shards, void* stream);
int rs_decode_dev(rs_ctx* ctx, int device, int k, int m, size_t S, int batch,
                  const uint8_t* present, uint8_t* const* shards, void* stream);

/* ---- ShardChecksum on device-resident shards (codec.go:81-84; §8(f) of SURVEY.md) ----
 * SHA-256 of `count` messages already in HBM, one digest per message written to
 * `digests` (device memory, 32*count bytes, FIPS 180-4 byte order — hex-encode it for
 * the Go string). msgs/lens are HOST arrays of device pointers and byte lengths.
 * SHA-256 is serial within a message, so this pays off only in batches of many shards
 * (scrub, device-resident pipelines); a single request's checksums stay on the CPU.
 * rs_sha256_plan_* upload the message table once; rs_sha256_dev is the one-shot form
 * (synchronous on `stream`). */
typedef struct rs_hash_plan rs_hash_plan;
int  rs_sha256_plan_create(rs_ctx* ctx, int device, const uint8_t* const* msgs,
                           const uint64_t* lens, int count, rs_hash_plan** out);
int  rs_sha256_plan_launch(rs_hash_plan* plan, uint8_t* digests, void* stream);
void rs_sha256_plan_destroy(rs_hash_plan* plan);
int  rs_sha256_dev(rs_ctx* ctx, int device, const uint8_t* const* msgs, const uint64_t* lens,
                   int count, uint8_t* digests, void* stream);

#ifdef __cplusplus
}
#endif
#endif /* CALLFS_RS_H */
