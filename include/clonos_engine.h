/*
 * clonos_engine.h -- C-ABI of the MI355X causal-log engine (libclonos_engine.so).
 *
 * This is the drop-in boundary a JNI layer binds.  Plain
 * pointers and sizes only; no exceptions cross it; every entry point returns an
 * int status (CLG_OK == 0).  clg_last_error() gives a thread-local message.
 *
 * Reference interfaces replaced (R/ = /root/reference/flink-runtime/src/main/java/
 * org/apache/flink/runtime/causal/):
 *   ThreadCausalLog      R/log/thread/ThreadCausalLog.java:33-96  (impl :51-527)
 *   JobCausalLog         R/log/job/JobCausalLog.java:50-78        (impl JobCausalLogImpl.java:71-300)
 *   DeterminantEncoder   R/determinant/DeterminantEncoder.java:28-65 (decode side; impl
 *                        SimpleDeterminantEncoder.java:78-342)
 *   DeterminantResponseEvent.merge  R/DeterminantResponseEvent.java:128-148
 *
 * Memory model: log bytes live in HBM in fixed-size segments (= Netty components of
 * determinantBufferSize bytes, NettyConfig.java:86-89); log metadata (epoch start
 * offsets, consumer offsets, visible writer index) lives in the host engine and is
 * updated with exactly the reference's semantics.  Outputs go to caller-allocated
 * buffers, either host (CLG_MEM_HOST) or device (CLG_MEM_DEVICE, a hipMalloc'd pointer
 * on the engine's device).  Entry points are safe to call from any thread.  Per-log calls
 * (append, hasDelta, offset, a slice served from the host tail, logLength, a host-input
 * upstream delta) take only their log's lock stripe; GPU and multi-log calls take the
 * engine lock and every stripe.  GPU work runs on the engine stream, apart from device
 * slices with CLG_F_ASYNC_SLICE, which run on a second (gather) stream.
 */
#ifndef CLONOS_ENGINE_H
#define CLONOS_ENGINE_H

#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

#define CLG_ABI_VERSION 6

/* ---- status codes ---------------------------------------------------------- */
enum {
  CLG_OK = 0,
  CLG_E_INVALID_ARG = -1,
  CLG_E_CORRUPT_TAG = -2,        /* CorruptDeterminantArrayException(tag)  SimpleDeterminantEncoder.java:92 */
  CLG_E_TRUNCATED = -3,          /* record runs past the span (ByteBuf IndexOutOfBounds) */
  CLG_E_BAD_ENUM = -4,           /* Type.values()[ord] / CheckpointType.values()[ord] out of range (:231, :285) */
  CLG_E_NEG_LEN = -5,            /* negative name / reference length (NegativeArraySizeException, :235, :282) */
  CLG_E_BAD_SERIAL = -6,         /* malformed Java serialization stream (type 3, :333-341) */
  CLG_E_CONSUMER_BACKWARDS = -7, /* "Consumer went backwards"  ThreadCausalLogImpl.java:215-218 */
  CLG_E_NO_CONSUMER = -8,        /* getOffset/getDelta before hasDelta (NPE at :245 / :256) */
  CLG_E_GAP = -9,                /* upstream delta leaves a gap (delta.readerIndex(<0) at :143) */
  CLG_E_NOSPACE = -10,           /* segment pool exhausted (Java side blocks: requestBufferBlocking :444) */
  CLG_E_CAPACITY = -11,          /* caller output buffer too small; required size reported */
  CLG_E_STATE = -12,             /* inconsistent log state (index out of bounds) */
  CLG_E_DEVICE = -13,            /* HIP runtime error */
  CLG_E_NO_LOG = -14,            /* unknown / closed log handle */
  CLG_E_NOT_BUFFER_BUILT = -15,  /* subpartition recovery buffer holds another determinant
                                    (RuntimeException, ReplayingState.java:172-177) */
  CLG_E_EPOCH_GAP = -16          /* in-flight replay reaches an epoch with no buffers (the reference's
                                    ReplayIterator NPEs at logToReplay.get(++currentKey), :133) */
};

/* CLG_MEM_MAPPED: host memory registered with clg_host_register.  For decode outputs
 * (clg_decoded.out_kind) the single-launch small decode writes it straight from the GPU (no
 * staging copy); every other path treats it as CLG_MEM_HOST. */
enum { CLG_MEM_HOST = 0, CLG_MEM_DEVICE = 1, CLG_MEM_MAPPED = 2 };

/* Pin and map [p, p + bytes) of host memory for the device (hipHostRegister, mapped); a
 * caller that keeps its output buffers across decodes registers them once.  Unregister
 * before the memory is freed. */
int clg_host_register(void* p, uint64_t bytes);
int clg_host_unregister(void* p);

/* Determinant tags (Determinant.java:23-34). */
enum {
  CLG_TAG_ORDER = 0, CLG_TAG_TIMESTAMP = 1, CLG_TAG_RNG = 2, CLG_TAG_SERIALIZABLE = 3,
  CLG_TAG_TIMER_TRIGGER = 4, CLG_TAG_SOURCE_CHECKPOINT = 5, CLG_TAG_IGNORE_CHECKPOINT = 6,
  CLG_TAG_BUFFER_BUILT = 7
};

#define CLG_FULL_SHARING (-1) /* ExecutionConfig.determinantSharingDepth default */

/* ---- identities ---------------------------------------------------------------- */
/* InputChannelID (an AbstractID: lower/upper longs). */
typedef struct clg_channel_id { uint64_t lo, hi; } clg_channel_id;

/* CausalLogID (CausalLogID.java:38-198): main-thread log of a vertex, or a
 * subpartition log {vertex, intermediate result partition (lower, upper), index}. */
typedef struct clg_causal_log_id {
  int16_t vertex_id;
  uint8_t is_main;
  int8_t subpartition;
  uint32_t reserved;
  int64_t irp_lower;
  int64_t irp_upper;
} clg_causal_log_id;

typedef struct clg_config {
  uint32_t segment_bytes;  /* determinantBufferSize (NettyConfig.java:86-89); 16384 by default */
  uint32_t pool_segments;  /* segments preallocated in HBM (pool = segment_bytes * pool_segments);
                              beside it, for segments up to 64 KiB, the Serializable records' positions
                              per segment (segment_bytes / 16 + 8 bytes each, ~6 %; none if HBM is short) */
  int32_t device;          /* HIP device ordinal */
  int32_t sharing_depth;   /* determinantSharingDepth (-1 = full sharing, 0 = logging off) */
  uint32_t flags;          /* CLG_F_* */
  uint32_t host_tail_bytes; /* flushed bytes of each log's tail also kept in host memory (16384 by
                               default): host-output slices / getDeterminants inside the tail are
                               served by memcpy, without a GPU round trip; 0: every slice gathers */
  /* The in-flight (data) log's own HBM pool (InMemorySubpartitionInFlightLogger keeps the
   * network buffers it was given; here their bytes are copied into this pool, apart from
   * the determinant segments so that data volume never starves appendDeterminant).  0:
   * defaults (32 KiB segments = Flink's memory segment size, 4096 of them). */
  uint32_t ifl_segment_bytes;
  uint32_t ifl_pool_segments;
} clg_config;

#define CLG_F_TIMING 1u        /* record per-kernel HIP event timings (clg_kernel_stats) */
#define CLG_F_ROBUST_DECODE 2u /* skip the fast three-pass decode; always use the robust
                                  multi-pass pipeline (the fallback the fused kernel aborts to) */
#define CLG_F_NO_SMALL_DECODE 8u /* batches up to 1 MiB also take the three-pass decode, not the
                                   single-launch small-batch one (tests of the three-pass path) */
#define CLG_F_ASYNC_SLICE 4u   /* slices into device memory (clg_slice_batch, CLG_MEM_DEVICE)
                                  return once queued on the engine's gather stream and overlap
                                  later decodes; the output is ready after clg_sync or once
                                  clg_gather_stream's work completes.  Default: synchronous */

typedef struct clg_engine clg_engine;

/* ---- engine ---------------------------------------------------------------------- */
void clg_config_default(clg_config* cfg);
int clg_engine_create(const clg_config* cfg, clg_engine** out);
void clg_engine_destroy(clg_engine* e);
const char* clg_last_error(void);
int clg_abi_version(void);
/* The HIP stream (hipStream_t) all engine work is issued on. */
void* clg_engine_stream(clg_engine* e);
/* The stream CLG_F_ASYNC_SLICE gathers run on (hipStream_t). */
void* clg_gather_stream(clg_engine* e);
/* Flush staged appends to HBM and wait for all queued GPU work. */
int clg_sync(clg_engine* e);
/* Segments in use / free in the HBM pool. */
int clg_pool_stats(clg_engine* e, uint32_t* used, uint32_t* free_segments);
/* Segments in use / free in the in-flight log's pool. */
int clg_ifl_pool_stats(clg_engine* e, uint32_t* used, uint32_t* free_segments);

/* ---- JobCausalLog scope ------------------------------------------------------------
 * One JobCausalLogImpl per job per TaskManager (JobCausalLogFactory.java:56-67,
 * JobCausalLogImpl.java:71-122): a job owns its thread logs, its sharing depth
 * (ExecutionConfig.determinantSharingDepth) and its latestCompletedCheckpoint.  Job 0 is
 * the engine's default job (sharing depth from clg_config); clg_job_open adds others, so
 * that several jobs on one TaskManager share an engine without sharing log identities or
 * checkpoint CAS state.  Log handles are global to the engine. */
int clg_job_open(clg_engine* e, uint64_t job_lo, uint64_t job_hi, int32_t sharing_depth, uint32_t* job);
/* Closes every log of the job (JobCausalLogImpl.close :277-283); job 0 stays open. */
int clg_job_close(clg_engine* e, uint32_t job);

/* ---- ThreadCausalLog --------------------------------------------------------------- */
/* Opens a log of `job` (ThreadCausalLogImpl ctor :94-112): one empty component is allocated. */
int clg_log_open(clg_engine* e, uint32_t job, const clg_causal_log_id* id, uint32_t* handle);
/* close() :317-328 (the engine does not wait for consumers; caller guarantees drain). */
int clg_log_close(clg_engine* e, uint32_t log);
int clg_log_find(clg_engine* e, uint32_t job, const clg_causal_log_id* id, uint32_t* handle);
/* The CausalLogID and job of an open log (e.g. one clg_process_delta opened). */
int clg_log_get_id(clg_engine* e, uint32_t log, clg_causal_log_id* id, uint32_t* job);
/* appendDeterminant :158-177.  `rec` holds ONE encoded determinant (encodeTo bytes;
 * n == getEncodedSizeInBytes).  Staged on the host, flushed to HBM in batches.  When the
 * append crosses the log's staging bound it also flushes; CLG_E_DEVICE from that flush
 * means the record WAS logged (staged) and only the write-behind failed. */
int clg_append(clg_engine* e, uint32_t log, int64_t epoch, const uint8_t* rec, uint32_t n);
/* Many appends at once: rec i = bytes[off[i], off[i]+len[i]) for log[i] in epoch[i]. */
int clg_append_batch(clg_engine* e, const uint32_t* log, const int64_t* epoch, const uint64_t* off,
                     const uint32_t* len, uint32_t n, const uint8_t* bytes);
/* processUpstreamDelta :117-154 (dedup by offsetFromEpoch, append the new suffix). */
int clg_upstream_delta(clg_engine* e, uint32_t log, int64_t epoch, int32_t offset_from_epoch,
                       const uint8_t* delta, uint32_t n);
/* Batched processUpstreamDelta over one buffer (host or device memory): delta i is
 * bytes[src_off, src_off + len) for log `log`; per-request status.  Device input (an
 * RCCL receive buffer) is scattered into the log segments without a host round trip. */
typedef struct clg_delta_req {
  uint32_t log;
  int32_t offset_from_epoch;
  int64_t epoch;
  uint64_t src_off;
  uint32_t len;
  int32_t status; /* out */
} clg_delta_req;
int clg_upstream_delta_batch(clg_engine* e, clg_delta_req* reqs, uint32_t n, const uint8_t* bytes,
                             uint32_t in_kind);
int clg_log_length(clg_engine* e, uint32_t log, int32_t* out);                                /* :180-192 */
/* logLength of n logs at once (out[i] for log[i]); *total = their sum (either may be NULL). */
int clg_log_length_batch(clg_engine* e, const uint32_t* log, uint32_t n, int32_t* out, uint64_t* total);
int clg_has_delta(clg_engine* e, uint32_t log, clg_channel_id c, int64_t epoch, int32_t* out); /* :196-240 */
int clg_offset_from_epoch(clg_engine* e, uint32_t log, clg_channel_id c, int32_t* out);       /* :243-246 */
/* getDeltaForConsumer :249-277: bytes copied into `out` (host or device).  With
 * CLG_E_CAPACITY, *n is the required size and the consumer has not advanced. */
int clg_get_delta(clg_engine* e, uint32_t log, clg_channel_id c, int64_t epoch, void* out,
                  uint32_t cap, uint32_t out_kind, uint32_t* n);
/* getDeterminants(startEpoch) :285-313 (CLG_E_CAPACITY: *n = required size). */
int clg_get_determinants(clg_engine* e, uint32_t log, int64_t start_epoch, void* out, uint32_t cap,
                         uint32_t out_kind, uint32_t* n);
int clg_notify_checkpoint_complete(clg_engine* e, uint32_t log, int64_t checkpoint_id); /* :398-435 */
int clg_unregister_consumer(clg_engine* e, uint32_t log, clg_channel_id c);              /* :331-336 */

/* State introspection (for parity tests and the JNI safety assertions). */
typedef struct clg_log_state {
  int32_t writer;        /* visibleWriterIndex */
  int32_t capacity;      /* composite capacity = components * segment_bytes */
  int32_t n_components;
  int32_t n_epochs;
} clg_log_state;
int clg_log_get_state(clg_engine* e, uint32_t log, clg_log_state* st, int64_t* epoch_ids,
                      int32_t* epoch_offsets, int32_t cap_epochs);
int clg_consumer_state(clg_engine* e, uint32_t log, clg_channel_id c, int32_t* exists,
                       int64_t* epoch, int32_t* offset);
/* Raw physical bytes of the log's composite (reads HBM). */
int clg_log_read_phys(clg_engine* e, uint32_t log, int32_t phys, uint32_t n, uint8_t* host_out);

/* ---- batched delta slicing (serializeThreadDelta loop, Flat/Grouping serde) ------------
 * For each request, in order: hasDeltaForConsumer; if true, getOffsetFromEpochForConsumer
 * then getDeltaForConsumer.  All deltas are gathered by ONE kernel into `out`
 * (packed in request order).  res[i].status != 0 reports a per-request error
 * (e.g. CLG_E_CONSUMER_BACKWARDS) without aborting the batch. */
typedef struct clg_slice_req {
  uint32_t log;
  uint32_t reserved;
  clg_channel_id consumer;
  int64_t epoch;
} clg_slice_req;
typedef struct clg_slice_res {
  int32_t status;
  int32_t has_delta;
  int32_t offset_from_epoch;
  int32_t len;
  uint64_t out_off;
} clg_slice_res;
int clg_slice_batch(clg_engine* e, const clg_slice_req* reqs, uint32_t n, clg_slice_res* res,
                    void* out, uint64_t cap, uint32_t out_kind, uint64_t* total);
/* Consumer offsets set directly (used to position consumers mid-epoch in benchmarks and
 * when a standby takes over a channel); epoch must exist. */
int clg_consumer_seek(clg_engine* e, uint32_t log, clg_channel_id c, int64_t epoch, int32_t offset);
/* Batched form: consumer reqs[i] of log reqs[i].log positioned at offsets[i] of epoch
 * reqs[i].epoch (stops at the first failing entry). */
int clg_consumer_seek_batch(clg_engine* e, const clg_slice_req* reqs, const int32_t* offsets, uint32_t n);

/* ---- checkpoint completion fan-out (JobCausalLogImpl.notifyCheckpointComplete :230-246) --
 * CAS on the job's latestCompletedCheckpoint; if newer, truncates every open log of that
 * job (other jobs' logs are untouched).  Queued asynchronous decodes (clg_decode_logs_async)
 * whose start epochs are all >= checkpoint_id stay queued: the truncation drops only bytes
 * below the checkpoint, and the segments it frees return to the pool once those decodes are
 * waited for.  A queued decode from an earlier epoch (or appends not yet flushed) is
 * completed first, as by any other call that needs the engine exclusively. */
int clg_truncate_all(clg_engine* e, uint32_t job, int64_t checkpoint_id, int32_t* applied);

/* ---- batched decode (SimpleDeterminantEncoder.decodeNext over whole spans) -------------
 * Output is a dense SoA over all spans (span order, record order):
 *   off[i]  byte offset of record i inside its span;  tag[i];  v0[i] =
 *   ORDER channel (sign-extended byte) | TIMESTAMP ts | RNG number | BUFFER_BUILT bytes |
 *   TIMER_TRIGGER timestamp | SOURCE_CHECKPOINT checkpointID | IGNORE_CHECKPOINT
 *   checkpointID | SERIALIZABLE java-stream length.
 * Wide records (tags 3,4,5,6) also get a side-table row:
 *   w_idx (global record index), w_rc (recordCount), w_v1 (SourceCheckpoint timestamp),
 *   w_var_off/w_var_len (name, storage reference or java stream, span-relative),
 *   w_sub (TimerTrigger type ordinal; SourceCheckpoint type | hasRef<<7). */
typedef struct clg_decoded {
  uint32_t* off;
  uint8_t* tag;
  int64_t* v0;
  uint32_t* w_idx;
  int32_t* w_rc;
  int64_t* w_v1;
  uint32_t* w_var_off;
  uint32_t* w_var_len;
  uint8_t* w_sub;
  uint64_t cap;       /* capacity of the record arrays */
  uint64_t wcap;      /* capacity of the side-table arrays */
  uint32_t out_kind;  /* CLG_MEM_HOST / CLG_MEM_DEVICE */
  uint32_t reserved;
  /* results */
  uint64_t n_rec;
  uint64_t n_wide;
  int32_t err_status; /* first decode error (lowest span), CLG_OK if none */
  uint32_t err_span;
  int64_t err_off;    /* span-relative offset of the failing record */
  int32_t err_tag;
  uint32_t reserved2;
} clg_decoded;

/* Decode spans of host memory: span i = bytes[span_off[i], span_off[i]+span_len[i]).
 * span_rec_base (optional, n+1 entries) receives each span's first record index. */
int clg_decode_host(clg_engine* e, const uint8_t* bytes, const uint64_t* span_off,
                    const uint64_t* span_len, uint32_t n, clg_decoded* out, uint64_t* span_rec_base);
/* Decode logs resident in HBM: span i = getDeterminants(start_epoch[i]) of log[i]
 * (no copy: kernels read the segments in place). */
int clg_decode_logs(clg_engine* e, const uint32_t* log, const int64_t* start_epoch, uint32_t n,
                    clg_decoded* out, uint64_t* span_rec_base);
/* Asynchronous clg_decode_logs: returns once the decode is queued on the engine stream, so
 * the caller can plan and queue other work (e.g. the slices of the same step, or the next
 * batch's decode) while it runs.  `out`, its arrays and span_rec_base must stay valid, and
 * are not to be read, until the clg_decode_wait that pairs with this call returns, which
 * completes the decode (fallback paths included) and returns its status.  Every other call
 * that needs the engine exclusively completes the pending decodes first (their statuses are
 * kept for clg_decode_wait); clg_slice_batch into device memory with CLG_F_ASYNC_SLICE, the
 * consumer seeks, and clg_truncate_all at or below every start epoch leave them pending.
 * Up to CLG_DECODE_MAX_INFLIGHT decodes may be queued before the first is waited for, so the
 * GPU runs decode i+1 while the host completes decode i; give each its own output arrays.
 * One more is CLG_E_STATE (no decode's status is ever dropped). */
#define CLG_DECODE_MAX_INFLIGHT 2
int clg_decode_logs_async(clg_engine* e, const uint32_t* log, const int64_t* start_epoch, uint32_t n,
                          clg_decoded* out, uint64_t* span_rec_base);
/* Completes the OLDEST decode clg_decode_logs_async queued and not yet waited for, and
 * returns ITS status (FIFO: one wait per queued decode, in queue order).  A later decode
 * still running on the GPU is not waited for.  With nothing queued: CLG_OK. */
int clg_decode_wait(clg_engine* e);

/* ---- replay-prep (DeterminantResponseEvent.merge + LogReplayer decode) ----------------
 * `n` candidate copies of logs (e.g. one per responding GPU / downstream):
 * copy i is (key[i], bytes[off[i], off[i]+len[i])).  For every distinct key the LONGEST
 * copy wins, ties going to the later copy (merge :137-146, v2 on ties).  winner[k] and
 * the number of keys are returned; the winners are then decoded in one batch. */
int clg_replay_prep(clg_engine* e, const uint64_t* key, const uint8_t* bytes, const uint64_t* off,
                    const uint64_t* len, uint32_t n, uint32_t* winner, uint32_t* n_keys,
                    clg_decoded* out, uint64_t* span_rec_base);

/* ---- piggybacked deltas (AbstractDeltaSerializerDeserializer.java:89-163) -----------------
 * enrichWithCausalLogDelta for a batch of outgoing buffers.  Request i covers entries
 * [first, first + count) of log[] / flags[]: the logs the reference's strategy visits for
 * that channel, in its iteration order, after the strategy's pre-hasDelta filters:
 *   CLG_DELTA_FLAT          FlatDeltaSerializerDeserializer.serializeDataStrategy :57-90
 *   CLG_DELTA_HIERARCHICAL  GroupingDeltaSerializerDeserializer.serializeDataStrategy
 *                           :91-165 (vertex-major: the vertex's main log first, then its
 *                           partitions' subpartition logs, each partition contiguous)
 * hasDeltaForConsumer is called on every entry (with its side effects); the delta is sent
 * when it has bytes and the entry's CLG_DE_SEND flag is set (the Grouping strategy's
 * post-hasDelta subpartition filter, :148-151).  Output per request at out_off: the delta
 * header ([size i32][epoch i64] + strategy records, :93-103) then the deltas back to back;
 * out_len = header + deltas.  CLG_E_CAPACITY: *total = required, no consumer moved. */
#define CLG_DELTA_FLAT 0u
#define CLG_DELTA_HIERARCHICAL 1u
#define CLG_DE_SEND 1u

typedef struct clg_enrich_req {
  clg_channel_id consumer;
  int64_t epoch;
  uint32_t first;
  uint32_t count;
  int32_t status;        /* out */
  uint32_t header_bytes; /* out */
  uint64_t out_off;      /* out */
  uint64_t out_len;      /* out */
} clg_enrich_req;

int clg_enrich_batch(clg_engine* e, uint32_t strategy, clg_enrich_req* reqs, uint32_t n, const uint32_t* log,
                     const uint8_t* flags, void* out, uint64_t cap, uint32_t out_kind, uint64_t* total);

/* processCausalLogDelta (:117-163) + insertNewUpstreamLog (:165-194): parse one header +
 * deltas (msg, host or device) and apply processUpstreamDelta to every log it names,
 * opening the logs not seen before (in `job`).  *epoch = the header's epoch; handles[] receives the
 * logs in header order (*n_logs, up to cap); *consumed = header + delta bytes. */
int clg_process_delta(clg_engine* e, uint32_t job, uint32_t strategy, const uint8_t* msg, uint64_t n,
                      uint32_t in_kind, int64_t* epoch, uint32_t* handles, uint32_t cap, uint32_t* n_logs,
                      uint64_t* consumed);

/* ---- batched encode (SimpleDeterminantEncoder.encodeTo :56-75, writers :124-323) ---------
 * The inverse of the decode: records given in the decode's SoA layout (tag, v0; a
 * side-table row per wide record, rows in record order and w_idx naming the record;
 * w_var_off indexes `var`, the payload bytes: TimerTrigger names, storage references,
 * Serializable streams) are written back to back in record order -- exactly the bytes
 * the reference's appendDeterminant sequence would produce.  *n_out = bytes (also on
 * CLG_E_CAPACITY).  A record with tag > 7 or a side row naming another record:
 * CLG_E_INVALID_ARG with the record index in *bad_index. */
typedef struct clg_encode_in {
  const uint8_t* tag;
  const int64_t* v0;
  uint64_t n;
  const uint32_t* w_idx;
  const int32_t* w_rc;
  const int64_t* w_v1;
  const uint32_t* w_var_off;
  const uint32_t* w_var_len;
  const uint8_t* w_sub;
  uint64_t n_wide;
  const uint8_t* var;
  uint64_t var_len;
  uint32_t in_kind; /* CLG_MEM_HOST / CLG_MEM_DEVICE (all input arrays) */
  uint32_t reserved;
} clg_encode_in;

int clg_encode_batch(clg_engine* e, const clg_encode_in* in, void* out, uint64_t cap, uint32_t out_kind,
                     uint64_t* n_out, uint64_t* bad_index);

/* ---- DeterminantResponseEvent (DeterminantResponseEvent.java:36-148) ---------------------
 * The event's map CausalLogID -> log bytes is held as an entry array in the iteration
 * order of the reference's java.util.HashMap (JDK 8: 2^k buckets from 16, load factor
 * 0.75, bins keep insertion order); `table_cap` is that map's bucket count.  Entries
 * point at caller memory (clg_response_read: into the wire bytes).  A zeroed struct with
 * entries/cap set is an empty map. */
typedef struct clg_response_entry {
  clg_causal_log_id id;
  const uint8_t* bytes;
  uint64_t len;
} clg_response_entry;

typedef struct clg_response {
  int32_t found;
  int16_t vertex_id;
  int16_t reserved;
  int64_t correlation_id;
  uint32_t n;          /* entries, map iteration order */
  uint32_t cap;        /* capacity of `entries` */
  uint32_t table_cap;  /* HashMap bucket count (0: fresh map, 16) */
  uint32_t reserved2;
  clg_response_entry* entries;
} clg_response;

/* HashMap.put (:54-63 constructors, JobCausalLogImpl.java:197-199): insert or replace. */
int clg_response_put(clg_response* r, const clg_causal_log_id* id, const uint8_t* bytes, uint64_t len);
/* n puts in order (one call for a response of many logs, e.g. a cross-GPU merge's winners). */
int clg_response_put_batch(clg_response* r, const clg_causal_log_id* ids, const uint8_t* const* bytes,
                           const uint64_t* lens, uint32_t n);
/* write (:93-107).  *n_out = wire size (also on CLG_E_CAPACITY). */
int clg_response_write(const clg_response* r, uint8_t* out, uint64_t cap, uint64_t* n_out);
/* read (:109-125).  The count byte is signed: 128..255 entries read back as none, like the
 * reference.  *consumed = bytes read.  Truncated input: CLG_E_TRUNCATED. */
int clg_response_read(const uint8_t* in, uint64_t n, clg_response* r, uint64_t* consumed);
/* acc.merge(other) (:128-148): nothing if neither is found; per CausalLogID the longer
 * buffer wins, ties -> other's (v2). */
int clg_response_merge(clg_response* acc, const clg_response* other);
/* CausalLogID.hashCode (:151-163), for callers keeping their own maps. */
int32_t clg_causal_log_id_hash(const clg_causal_log_id* id);

/* ---- replay preparation (ReplayingState.java:58-214, LogReplayerImpl.java:51-158) --------
 * For each failed vertex v: its merged response (WaitingDeterminantsState.java:57,102 --
 * start from found=true and clg_response_merge every response in arrival order) and the
 * task's subpartition table.  One batch on the GPU:
 *   main logs  -- CausalLogID(v) of each vertex (absent: empty span), batched decode into
 *                 `main` (span v; LogReplayerImpl replays that record sequence);
 *   subpartition buffers -- for table entry j the response's log (absent: EMPTY_BUFFER),
 *                 BufferBuilt sizes into buffer_sizes[sizes_base[j] ...]
 *                 (SubpartitionRecoveryThread.run :161-188); sub_status[j] is CLG_OK or the
 *                 error that thread hits first (decode error of the record at sub_err_off,
 *                 or CLG_E_NOT_BUFFER_BUILT); sizes before the error are valid and
 *                 sub_count[j] gives their number.  Entries are global over all vertices, in
 *                 vertex order then table order. */
typedef struct clg_replay_vertex {
  const clg_response* acc;
  const clg_causal_log_id* subpartitions;
  uint32_t n_subpartitions;
  int16_t vertex_id;
  int16_t reserved;
} clg_replay_vertex;

typedef struct clg_replay_out {
  clg_decoded* main;          /* host output (out_kind CLG_MEM_HOST) */
  uint64_t* main_rec_base;    /* n_vertices + 1 */
  int32_t* buffer_sizes;      /* capacity sizes_cap */
  uint64_t sizes_cap;
  uint64_t* sizes_base;       /* n_subpartitions_total + 1 */
  uint64_t* sub_count;
  int32_t* sub_status;
  int64_t* sub_err_off;
  int32_t* sub_err_tag;
} clg_replay_out;

int clg_replay_prepare(clg_engine* e, const clg_replay_vertex* v, uint32_t n, clg_replay_out* out);
/* The same with every response entry's bytes in device memory on the engine's device (e.g.
 * the winners of a cross-GPU merge in an RCCL receive buffer): they are gathered into the
 * engine's staging area on the GPU, never through the host.  The gather reads whole aligned
 * 16-byte words, so each range needs 16 readable bytes before and after it inside its
 * allocation. */
int clg_replay_prepare_device(clg_engine* e, const clg_replay_vertex* v, uint32_t n, clg_replay_out* out);

/* getDeterminants(start_epoch[i]) of log[i] (:285-313) for n logs -- the copies
 * respondToDeterminantRequest answers with (JobCausalLogImpl.java:188-204) -- gathered by ONE
 * kernel back to back in request order into `out` (host or device); len[i] and out_off[i]
 * (optional) give each copy's size and place.  out == NULL: sizes only (*total = bytes
 * needed); cap < *total: CLG_E_CAPACITY. */
int clg_get_determinants_batch(clg_engine* e, const uint32_t* log, const int64_t* start_epoch, uint32_t n,
                               void* out, uint64_t cap, uint32_t out_kind, uint64_t* out_off, uint32_t* len,
                               uint64_t* total);

/* ---- in-flight (data) log (RT/inflightlogging/, I/ below) -------------------------------------
 * InFlightLog I/InFlightLog.java:32-55, two implementations (I/InFlightLogConfig.java:44 picks
 * one by taskmanager.inflight.type, default "spillable"):
 *   CLG_IFL_IN_MEMORY  InMemorySubpartitionInFlightLogger I/InMemorySubpartitionInFlightLogger.java:28-207
 *   CLG_IFL_SPILLABLE  SpillableSubpartitionInFlightLogger I/SpillableSubpartitionInFlightLogger.java:45-341
 *                      with SpilledReplayIterator I/SpilledReplayIterator.java:60-401 (replay semantics;
 *                      the spill files are not modelled -- every buffer stays in HBM, i.e. no spill
 *                      has completed, which is the deterministic case of the reference)
 * Per subpartition, the data buffers sent in each epoch, kept in HBM (the engine's in-flight pool,
 * clg_config.ifl_*; a buffer spans ceil(len / ifl_segment_bytes) segments) until a checkpoint
 * completes.  The Java side keeps refcounts; the engine owns the bytes.  A full pool is
 * CLG_E_NOSPACE with nothing logged: the caller applies backpressure (waits for a checkpoint to
 * free epochs) and retries. */
#define CLG_IFL_IN_MEMORY 0u
#define CLG_IFL_SPILLABLE 1u
int clg_ifl_open(clg_engine* e, uint32_t* handle); /* CLG_IFL_IN_MEMORY */
int clg_ifl_open_typed(clg_engine* e, uint32_t type, uint32_t* handle);
/* close() (in-memory :90-94, spillable :151-157): all buffers released. */
int clg_ifl_close(clg_engine* e, uint32_t ifl);
/* log(buffer, epochID, isFinished) (in-memory :44-48, spillable :84-103), batched: buffer i =
 * bytes[off[i], off[i] + len[i]) appended to ifl[i] in epoch[i], in order (host or device input).
 * Spillable: a buffer logged while the log is replaying (between getInFlightIterator and the
 * drain of its last buffer) reaches the live iterator (notifyNewBufferAdded,
 * SpilledReplayIterator.java:262-277).  When the log is replaying but getInFlightIterator has
 * never returned an iterator (its first call found nothing, :132-135), the reference's log()
 * throws a NullPointerException after appending (:98-99): every buffer is appended and the
 * status is CLG_E_STATE. */
int clg_ifl_log_batch(clg_engine* e, const uint32_t* ifl, const int64_t* epoch, const uint64_t* off,
                      const uint32_t* len, uint32_t n, const uint8_t* bytes, uint32_t in_kind);
/* notifyCheckpointComplete (in-memory :51-70, spillable :106-123): epochs < checkpoint_id are
 * dropped, their segments freed. */
int clg_ifl_notify_checkpoint_complete(clg_engine* e, uint32_t ifl, int64_t checkpoint_id);
/* Epochs and buffer counts (ascending epoch), for parity tests. */
int clg_ifl_state(clg_engine* e, uint32_t ifl, int64_t* epoch_ids, uint32_t* n_buffers, uint32_t cap,
                  uint32_t* n_epochs);
/* getInFlightIterator(startEpochID, ignoreBuffers) + draining the iterator, batched: for request
 * i the buffers the iterator yields after skipping ignore_buffers are gathered by one kernel,
 * back to back in request order, into `out` at out_off (len bytes); their sizes go to
 * sizes[sizes_off ...] (n_buffers entries).  remaining = the iterator's numberRemaining() after
 * the skip.  epochs (optional, indexed like sizes) receives each buffer's epoch: the iterator's
 * getEpoch() right before the next() that returns it, which
 * PipelinedSubpartition.getReplayedBufferUnsafe (:306-320) stamps on the BufferAndBacklog;
 * end_epoch is getEpoch() after the last buffer was taken (or after the skip when none is).
 * CLG_E_CAPACITY (bytes or sizes): *total / *total_buffers hold the required sizes, no bytes are
 * gathered and no iterator state changes.
 *
 * In-memory (ReplayIterator :107-201): the buffers of every epoch >= start when start itself holds
 * buffers, else nothing (:121-127: a start epoch that is absent, e.g. already truncated, yields
 * nothing).  An epoch without buffers between start and the last epoch (K buffers before it):
 * next() advances past each returned buffer (:156) and throws at the gap (:133), so the K-th
 * buffer is never delivered -- buffers [ignore_buffers, K-1) are gathered and status is
 * CLG_E_EPOCH_GAP.  A skip that throws inside getInFlightIterator (:78-79) -- ignore_buffers >= K
 * at a gap, beyond the buffers available without one, or any skip when start is absent -- is
 * CLG_E_STATE, nothing gathered.
 *
 * Spillable (getInFlightIterator :126-142, SpilledReplayIterator, EpochCursor :306-394): the
 * iterator covers tailMap(start) -- the epochs >= start, from the first one present.  Empty (or a
 * closed log): no iterator (res.flags CLG_IFL_NULL_ITERATOR, nothing gathered).  Its cursors step
 * epoch IDs one by one, so an epoch missing between the first and the last makes the iterator
 * throw: a skip reaching past it is CLG_E_STATE (inside the constructor); otherwise the prefetch
 * cursor stops at it in the constructor and the consumer's first next() throws (no buffer is
 * delivered, CLG_E_EPOCH_GAP).  The iterator stays the log's current one: max_buffers (0: all)
 * bounds how many are taken per request, and a request with CLG_IFL_CONTINUE takes the next
 * buffers of the current iterator (start and ignore_buffers unused), including buffers logged
 * since.  Taking its last buffer ends the replay (res.flags loses CLG_IFL_REPLAYING).
 * max_buffers and CLG_IFL_CONTINUE are spillable-only (CLG_E_INVALID_ARG otherwise). */
#define CLG_IFL_CONTINUE 1u       /* clg_ifl_replay_req.flags: continue the current iterator */
#define CLG_IFL_NULL_ITERATOR 1u  /* clg_ifl_replay_res.flags: getInFlightIterator returned null */
#define CLG_IFL_REPLAYING 2u      /* clg_ifl_replay_res.flags: the log is replaying after the call */
typedef struct clg_ifl_replay_req {
  uint32_t ifl;
  uint32_t ignore_buffers;
  int64_t start_epoch;
  uint32_t max_buffers; /* spillable: at most this many buffers taken (0: all) */
  uint32_t flags;       /* CLG_IFL_CONTINUE */
} clg_ifl_replay_req;
typedef struct clg_ifl_replay_res {
  int32_t status;
  uint32_t n_buffers;
  uint32_t remaining;
  uint32_t flags; /* CLG_IFL_NULL_ITERATOR | CLG_IFL_REPLAYING */
  uint64_t out_off;
  uint64_t len;
  uint64_t sizes_off;
  int64_t end_epoch;
} clg_ifl_replay_res;
int clg_ifl_replay_batch(clg_engine* e, const clg_ifl_replay_req* reqs, uint32_t n, clg_ifl_replay_res* res,
                         void* out, uint64_t cap, uint32_t out_kind, uint32_t* sizes, int64_t* epochs,
                         uint64_t sizes_cap, uint64_t* total, uint64_t* total_buffers);

/* ---- instrumentation ---------------------------------------------------------------- */
typedef struct clg_kernel_stat {
  char name[32];
  uint64_t launches;
  double total_ms;
  uint64_t bytes; /* algorithmic bytes attributed to the kernel */
} clg_kernel_stat;
int clg_kernel_stats(clg_engine* e, clg_kernel_stat* out, uint32_t cap, uint32_t* n);
int clg_kernel_stats_reset(clg_engine* e);

#ifdef __cplusplus
}
#endif
#endif /* CLONOS_ENGINE_H */
