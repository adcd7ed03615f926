/*
 * clonos_oracle.h -- CPU ORACLE (test infrastructure only).
 *
 * This is NOT product code.  It is a sequential C++ restatement of the reference
 * Java algorithms on the causal-log hot path, used exclusively as the checker by
 * tests/, __graft_entry__.smoke() and bench.py's cpu_baseline leg.  Nothing in
 * clonos_amd/ links or calls it.
 *
 * Reference files restated (paths relative to
 * /root/reference/flink-runtime/src/main/java/org/apache/flink/runtime/causal/):
 *   determinant/SimpleDeterminantEncoder.java:32-342   (encode/decodeNext)
 *   determinant/<Type>Determinant.java                  (record sizes)
 *   log/thread/ThreadCausalLogImpl.java:51-527           (log state machine)
 *   DeterminantResponseEvent.java:128-148                (merge, longest wins)
 * Third-party semantics restated (absent from /root/reference):
 *   Netty 4.1.24.Final CompositeByteBuf.discardReadComponents  (pinned by
 *     flink-runtime/src/test/.../causal/NettyTests.java:144-186)
 *   JDK 8 java.io.ObjectInputStream stream grammar (Java Object Serialization
 *     Specification, section 6.4) -- PARITY UNPINNED: no reference test covers it.
 *
 * Status codes are numerically identical to include/clonos_engine.h.
 */
#ifndef CLONOS_ORACLE_H
#define CLONOS_ORACLE_H

#include <stdint.h>
#include <stddef.h>

#ifdef __cplusplus
extern "C" {
#endif

enum {
  ORC_OK = 0,
  ORC_E_INVALID_ARG = -1,
  ORC_E_CORRUPT_TAG = -2,
  ORC_E_TRUNCATED = -3,
  ORC_E_BAD_ENUM = -4,
  ORC_E_NEG_LEN = -5,
  ORC_E_BAD_SERIAL = -6,
  ORC_E_CONSUMER_BACKWARDS = -7,
  ORC_E_NO_CONSUMER = -8,
  ORC_E_GAP = -9,
  ORC_E_CAPACITY = -11,
  ORC_E_STATE = -12,
};

/* One decoded determinant in the build's SoA layout (see include/clonos_engine.h). */
typedef struct orc_det {
  uint8_t tag;        /* 0..7, Determinant.java:23-34 */
  int64_t v0;         /* channel / timestamp / number / bytes / ts / checkpointID / java-stream length */
  int32_t record_count;
  int64_t v1;         /* SourceCheckpoint checkpointTimestamp */
  uint8_t sub;        /* TimerTrigger type ordinal; SourceCheckpoint cpType | hasRef<<7 */
  const uint8_t* var; /* name / storage reference / java stream bytes */
  uint32_t var_len;
} orc_det;

/* Encode one determinant exactly as SimpleDeterminantEncoder.encodeTo does.
 * For tag 3 `var` must already hold a complete Java serialization stream.
 * Returns encoded size, or ORC_E_CAPACITY / ORC_E_INVALID_ARG. */
int64_t orc_encode(const orc_det* d, uint8_t* out, size_t cap);

/* Length of one Java serialization stream (magic+version+one object), or <0. */
int64_t orc_jser_len(const uint8_t* p, size_t avail);

/* Sequential decodeNext loop over one contiguous span (SimpleDeterminantEncoder:78-93).
 * Writes up to `cap` records / `wcap` wide rows.  On a decode error returns the
 * status, *err_off = record start offset, *err_tag = tag byte; records before the
 * failing one are still written and counted. */
int orc_decode_span(const uint8_t* buf, size_t len,
                    uint32_t* off, uint8_t* tag, int64_t* v0,
                    uint32_t* w_idx, int32_t* w_rc, int64_t* w_v1,
                    uint32_t* w_var_off, uint32_t* w_var_len, uint8_t* w_sub,
                    size_t cap, size_t wcap, size_t* n_rec, size_t* n_wide,
                    int64_t* err_off, int32_t* err_tag);

/* Count-only decode (used by the CPU baseline to avoid allocation noise). */
int orc_decode_count(const uint8_t* buf, size_t len, size_t* n_rec, size_t* n_wide);

/* ---------------- ThreadCausalLogImpl model ---------------- */
typedef struct orc_log orc_log;
orc_log* orc_log_new(uint32_t component_bytes, int32_t sharing_depth);
void orc_log_free(orc_log*);
int orc_log_append(orc_log*, int64_t epoch, const uint8_t* bytes, uint32_t n);          /* appendDeterminant :158-177 */
int orc_log_upstream(orc_log*, const uint8_t* delta, uint32_t n, int32_t off_from_epoch, int64_t epoch); /* :117-154 */
int orc_log_has_delta(orc_log*, uint64_t ch_lo, uint64_t ch_hi, int64_t epoch, int* out); /* :196-240 */
int orc_log_offset(orc_log*, uint64_t ch_lo, uint64_t ch_hi, int32_t* out);               /* :243-246 */
int orc_log_get_delta(orc_log*, uint64_t ch_lo, uint64_t ch_hi, int64_t epoch,
                      uint8_t* out, uint32_t cap, uint32_t* n);                          /* :249-277 */
int orc_log_get_determinants(orc_log*, int64_t start_epoch, uint8_t* out, uint32_t cap, uint32_t* n); /* :285-313 */
int orc_log_length(orc_log*, int32_t* out);                                               /* :180-192 */
int orc_log_checkpoint_complete(orc_log*, int64_t cp);                                    /* :398-435 */
int orc_log_unregister(orc_log*, uint64_t ch_lo, uint64_t ch_hi);                         /* :331-336 */
/* State snapshot: writer (visibleWriterIndex), capacity (composite capacity),
 * n_components, epochs (id, offset) sorted by id. */
int orc_log_state(orc_log*, int32_t* writer, int32_t* capacity, int32_t* n_components,
                  int64_t* epoch_ids, int32_t* epoch_offs, int32_t cap_epochs, int32_t* n_epochs);
/* Consumer state: epoch id and logical offset (ConsumerOffset :495-526); *exists=0 if absent. */
int orc_log_consumer(orc_log*, uint64_t ch_lo, uint64_t ch_hi, int* exists, int64_t* epoch, int32_t* offset);
/* Raw physical bytes [phys, phys+n) of the composite (for state parity). */
int orc_log_read_phys(orc_log*, int32_t phys, uint32_t n, uint8_t* out);

/* ---------------- CPU baseline helpers ---------------- */
/* Decode `n_spans` spans of a packed buffer with `threads` std::threads (one span per task).
 * Returns total records; used by bench.py cpu_baseline. */
int64_t orc_bench_decode(const uint8_t* buf, const uint64_t* span_off, const uint64_t* span_len,
                         uint32_t n_spans, uint32_t threads);
/* Slice (memcpy) `n_req` ranges out of `buf` into `out` with `threads` threads. */
int64_t orc_bench_slice(const uint8_t* buf, const uint64_t* src_off, const uint64_t* len,
                        const uint64_t* dst_off, uint32_t n_req, uint8_t* out, uint32_t threads);

#ifdef __cplusplus
}
#endif
#endif
