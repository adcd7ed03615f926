/*
 * clonos_jni.c -- JNI shim: org.apache.flink.runtime.causal.engine.ClonosEngine natives
 * onto the C-ABI in include/clonos_engine.h.  No logic lives here: argument unpacking,
 * direct-buffer addresses (GetDirectBufferAddress, no copies), status passthrough.
 *
 * Build (on a host with a JDK; not possible in this container, which has no jni.h):
 *   cc -O2 -fPIC -shared -I$JAVA_HOME/include -I$JAVA_HOME/include/linux -Iinclude \
 *      jni/clonos_jni.c -Lclonos_amd -lclonos_engine -o libclonos_jni.so
 */
#include <jni.h>
#include <stdlib.h>
#include <string.h>

#include "clonos_engine.h"

#define ENG(h) ((clg_engine*)(intptr_t)(h))
#define FN(name) Java_org_apache_flink_runtime_causal_engine_ClonosEngine_##name

static void put_int(JNIEnv* env, jintArray a, jint v) { (*env)->SetIntArrayRegion(env, a, 0, 1, &v); }

static uint8_t* addr(JNIEnv* env, jobject buf, jint off) {
  if (!buf) return NULL;
  uint8_t* p = (uint8_t*)(*env)->GetDirectBufferAddress(env, buf);
  return p ? p + off : NULL;
}
static uint32_t cap(JNIEnv* env, jobject buf) {
  return buf ? (uint32_t)(*env)->GetDirectBufferCapacity(env, buf) : 0u;
}
static clg_channel_id ch(jlong lo, jlong hi) {
  clg_channel_id c = {(uint64_t)lo, (uint64_t)hi};
  return c;
}

JNIEXPORT jint JNICALL FN(nCreate)(JNIEnv* env, jclass cls, jint seg, jint pool, jint dev, jint depth,
                                   jint ifl_seg, jint ifl_pool, jlongArray out) {
  (void)cls;
  clg_config cfg;
  clg_config_default(&cfg);
  cfg.segment_bytes = (uint32_t)seg;
  cfg.pool_segments = (uint32_t)pool;
  cfg.ifl_segment_bytes = (uint32_t)ifl_seg;
  cfg.ifl_pool_segments = (uint32_t)ifl_pool;
  cfg.device = dev;
  cfg.sharing_depth = depth;
  clg_engine* e = NULL;
  int st = clg_engine_create(&cfg, &e);
  jlong h = (jlong)(intptr_t)e;
  (*env)->SetLongArrayRegion(env, out, 0, 1, &h);
  return st;
}

JNIEXPORT void JNICALL FN(nDestroy)(JNIEnv* env, jclass cls, jlong e) {
  (void)env;
  (void)cls;
  clg_engine_destroy(ENG(e));
}

JNIEXPORT jstring JNICALL FN(nLastError)(JNIEnv* env, jclass cls) {
  (void)cls;
  return (*env)->NewStringUTF(env, clg_last_error());
}

JNIEXPORT jint JNICALL FN(nJobOpen)(JNIEnv* env, jclass cls, jlong e, jlong job_lo, jlong job_hi, jint depth,
                                    jintArray out) {
  (void)cls;
  uint32_t j = 0;
  int st = clg_job_open(ENG(e), (uint64_t)job_lo, (uint64_t)job_hi, depth, &j);
  put_int(env, out, (jint)j);
  return st;
}

JNIEXPORT jint JNICALL FN(nJobClose)(JNIEnv* env, jclass cls, jlong e, jint job) {
  (void)env;
  (void)cls;
  return clg_job_close(ENG(e), (uint32_t)job);
}

JNIEXPORT jint JNICALL FN(nLogOpen)(JNIEnv* env, jclass cls, jlong e, jint job, jshort vid, jboolean is_main,
                                    jlong lo, jlong hi, jbyte sub, jintArray out) {
  (void)cls;
  clg_causal_log_id id;
  memset(&id, 0, sizeof id);
  id.vertex_id = vid;
  id.is_main = is_main ? 1 : 0;
  id.irp_lower = lo;
  id.irp_upper = hi;
  id.subpartition = sub;
  uint32_t h = 0;
  int st = clg_log_open(ENG(e), (uint32_t)job, &id, &h);
  put_int(env, out, (jint)h);
  return st;
}

JNIEXPORT jint JNICALL FN(nLogClose)(JNIEnv* env, jclass cls, jlong e, jint log) {
  (void)env;
  (void)cls;
  return clg_log_close(ENG(e), (uint32_t)log);
}

JNIEXPORT jint JNICALL FN(nAppend)(JNIEnv* env, jclass cls, jlong e, jint log, jlong epoch, jobject buf, jint off,
                                   jint len) {
  (void)cls;
  return clg_append(ENG(e), (uint32_t)log, epoch, addr(env, buf, off), (uint32_t)len);
}

JNIEXPORT jint JNICALL FN(nUpstreamDelta)(JNIEnv* env, jclass cls, jlong e, jint log, jlong epoch, jint ofe,
                                          jobject buf, jint off, jint len) {
  (void)cls;
  return clg_upstream_delta(ENG(e), (uint32_t)log, epoch, ofe, addr(env, buf, off), (uint32_t)len);
}

JNIEXPORT jint JNICALL FN(nLogLength)(JNIEnv* env, jclass cls, jlong e, jint log, jintArray out) {
  (void)cls;
  int32_t n = 0;
  int st = clg_log_length(ENG(e), (uint32_t)log, &n);
  put_int(env, out, n);
  return st;
}

JNIEXPORT jint JNICALL FN(nHasDelta)(JNIEnv* env, jclass cls, jlong e, jint log, jlong lo, jlong hi, jlong epoch,
                                     jintArray out) {
  (void)cls;
  int32_t has = 0;
  int st = clg_has_delta(ENG(e), (uint32_t)log, ch(lo, hi), epoch, &has);
  put_int(env, out, has);
  return st;
}

JNIEXPORT jint JNICALL FN(nOffsetFromEpoch)(JNIEnv* env, jclass cls, jlong e, jint log, jlong lo, jlong hi,
                                            jintArray out) {
  (void)cls;
  int32_t v = 0;
  int st = clg_offset_from_epoch(ENG(e), (uint32_t)log, ch(lo, hi), &v);
  put_int(env, out, v);
  return st;
}

JNIEXPORT jint JNICALL FN(nGetDelta)(JNIEnv* env, jclass cls, jlong e, jint log, jlong lo, jlong hi, jlong epoch,
                                     jobject buf, jintArray out) {
  (void)cls;
  uint32_t n = 0;
  int st = clg_get_delta(ENG(e), (uint32_t)log, ch(lo, hi), epoch, addr(env, buf, 0), cap(env, buf), CLG_MEM_HOST, &n);
  put_int(env, out, (jint)n);
  return st;
}

JNIEXPORT jint JNICALL FN(nGetDeterminants)(JNIEnv* env, jclass cls, jlong e, jint log, jlong start, jobject buf,
                                            jintArray out) {
  (void)cls;
  uint32_t n = 0;
  int st = clg_get_determinants(ENG(e), (uint32_t)log, start, addr(env, buf, 0), cap(env, buf), CLG_MEM_HOST, &n);
  put_int(env, out, (jint)n);
  return st;
}

JNIEXPORT jint JNICALL FN(nNotifyCheckpointComplete)(JNIEnv* env, jclass cls, jlong e, jint log, jlong cp) {
  (void)env;
  (void)cls;
  return clg_notify_checkpoint_complete(ENG(e), (uint32_t)log, cp);
}

JNIEXPORT jint JNICALL FN(nUnregisterConsumer)(JNIEnv* env, jclass cls, jlong e, jint log, jlong lo, jlong hi) {
  (void)env;
  (void)cls;
  return clg_unregister_consumer(ENG(e), (uint32_t)log, ch(lo, hi));
}

JNIEXPORT jint JNICALL FN(nTruncateAll)(JNIEnv* env, jclass cls, jlong e, jint job, jlong cp, jintArray applied) {
  (void)cls;
  int32_t a = 0;
  int st = clg_truncate_all(ENG(e), (uint32_t)job, cp, &a);
  put_int(env, applied, a);
  return st;
}

/* ---- batched paths ----------------------------------------------------------------
 * Arrays of handles / ids come in as Java primitive arrays (copied by the JVM), bulk data
 * as direct ByteBuffers (no copies).  Result words go back through long[] arrays. */

/* clg_decode_logs: SoA into direct buffers; res = {n_rec, n_wide, err_status, err_span,
 * err_off, err_tag}; spanRecBase has n + 1 entries. */
JNIEXPORT jint JNICALL FN(nDecodeLogs)(JNIEnv* env, jclass cls, jlong e, jintArray logs, jlongArray starts,
                                       jobject off, jobject tag, jobject v0, jobject w_idx, jobject w_rc, jobject w_v1,
                                       jobject w_var_off, jobject w_var_len, jobject w_sub, jlongArray res,
                                       jlongArray span_rec_base) {
  (void)cls;
  const jsize n = (*env)->GetArrayLength(env, logs);
  jint* lg = (*env)->GetIntArrayElements(env, logs, NULL);
  jlong* st = (*env)->GetLongArrayElements(env, starts, NULL);
  jlong* base = (*env)->GetLongArrayElements(env, span_rec_base, NULL);
  clg_decoded d;
  memset(&d, 0, sizeof d);
  d.off = (uint32_t*)addr(env, off, 0);
  d.tag = addr(env, tag, 0);
  d.v0 = (int64_t*)addr(env, v0, 0);
  d.w_idx = (uint32_t*)addr(env, w_idx, 0);
  d.w_rc = (int32_t*)addr(env, w_rc, 0);
  d.w_v1 = (int64_t*)addr(env, w_v1, 0);
  d.w_var_off = (uint32_t*)addr(env, w_var_off, 0);
  d.w_var_len = (uint32_t*)addr(env, w_var_len, 0);
  d.w_sub = addr(env, w_sub, 0);
  d.cap = cap(env, tag);
  d.wcap = cap(env, w_sub);
  d.out_kind = CLG_MEM_HOST;
  int s = clg_decode_logs(ENG(e), (const uint32_t*)lg, (const int64_t*)st, (uint32_t)n, &d, (uint64_t*)base);
  jlong r[6] = {(jlong)d.n_rec, (jlong)d.n_wide, d.err_status, d.err_span, d.err_off, d.err_tag};
  (*env)->SetLongArrayRegion(env, res, 0, 6, r);
  (*env)->ReleaseLongArrayElements(env, span_rec_base, base, 0);
  (*env)->ReleaseLongArrayElements(env, starts, st, JNI_ABORT);
  (*env)->ReleaseIntArrayElements(env, logs, lg, JNI_ABORT);
  return s;
}

/* clg_decode_logs_async: the decode is queued; ctx[0] receives a handle that nDecodeWait
 * completes and frees (the output ByteBuffers must stay reachable until then). */
typedef struct {
  clg_decoded d;
  uint64_t* base;
  jsize n;
} async_decode;

JNIEXPORT jint JNICALL FN(nDecodeLogsAsync)(JNIEnv* env, jclass cls, jlong e, jintArray logs, jlongArray starts,
                                            jobject off, jobject tag, jobject v0, jobject w_idx, jobject w_rc,
                                            jobject w_v1, jobject w_var_off, jobject w_var_len, jobject w_sub,
                                            jlongArray ctx) {
  (void)cls;
  const jsize n = (*env)->GetArrayLength(env, logs);
  async_decode* a = (async_decode*)calloc(1, sizeof(async_decode));
  if (!a) return CLG_E_INVALID_ARG;
  a->base = (uint64_t*)calloc((size_t)n + 1, sizeof(uint64_t));
  a->n = n;
  a->d.off = (uint32_t*)addr(env, off, 0);
  a->d.tag = addr(env, tag, 0);
  a->d.v0 = (int64_t*)addr(env, v0, 0);
  a->d.w_idx = (uint32_t*)addr(env, w_idx, 0);
  a->d.w_rc = (int32_t*)addr(env, w_rc, 0);
  a->d.w_v1 = (int64_t*)addr(env, w_v1, 0);
  a->d.w_var_off = (uint32_t*)addr(env, w_var_off, 0);
  a->d.w_var_len = (uint32_t*)addr(env, w_var_len, 0);
  a->d.w_sub = addr(env, w_sub, 0);
  a->d.cap = cap(env, tag);
  a->d.wcap = cap(env, w_sub);
  a->d.out_kind = CLG_MEM_HOST;
  jint* lg = (*env)->GetIntArrayElements(env, logs, NULL);
  jlong* st = (*env)->GetLongArrayElements(env, starts, NULL);
  int s = clg_decode_logs_async(ENG(e), (const uint32_t*)lg, (const int64_t*)st, (uint32_t)n, &a->d, a->base);
  (*env)->ReleaseLongArrayElements(env, starts, st, JNI_ABORT);
  (*env)->ReleaseIntArrayElements(env, logs, lg, JNI_ABORT);
  if (s != CLG_OK) {
    free(a->base);
    free(a);
    return s;
  }
  jlong h = (jlong)(intptr_t)a;
  (*env)->SetLongArrayRegion(env, ctx, 0, 1, &h);
  return s;
}

/* clg_decode_wait for the decode nDecodeLogsAsync queued: results as nDecodeLogs. */
JNIEXPORT jint JNICALL FN(nDecodeWait)(JNIEnv* env, jclass cls, jlong e, jlong ctx, jlongArray res,
                                       jlongArray span_rec_base) {
  (void)cls;
  async_decode* a = (async_decode*)(intptr_t)ctx;
  int s = clg_decode_wait(ENG(e));
  if (!a) return s;
  jlong r[6] = {(jlong)a->d.n_rec, (jlong)a->d.n_wide, a->d.err_status, a->d.err_span, a->d.err_off, a->d.err_tag};
  (*env)->SetLongArrayRegion(env, res, 0, 6, r);
  (*env)->SetLongArrayRegion(env, span_rec_base, 0, a->n + 1, (const jlong*)a->base);
  free(a->base);
  free(a);
  return s;
}

/* clg_decode_host over bytes[off, off + len): one span; results as nDecodeLogs. */
JNIEXPORT jint JNICALL FN(nDecodeHost)(JNIEnv* env, jclass cls, jlong e, jobject bytes, jint off, jint len, jobject o_off,
                                       jobject tag, jobject v0, jobject w_idx, jobject w_rc, jobject w_v1,
                                       jobject w_var_off, jobject w_var_len, jobject w_sub, jlongArray res) {
  (void)cls;
  clg_decoded d;
  memset(&d, 0, sizeof d);
  d.off = (uint32_t*)addr(env, o_off, 0);
  d.tag = addr(env, tag, 0);
  d.v0 = (int64_t*)addr(env, v0, 0);
  d.w_idx = (uint32_t*)addr(env, w_idx, 0);
  d.w_rc = (int32_t*)addr(env, w_rc, 0);
  d.w_v1 = (int64_t*)addr(env, w_v1, 0);
  d.w_var_off = (uint32_t*)addr(env, w_var_off, 0);
  d.w_var_len = (uint32_t*)addr(env, w_var_len, 0);
  d.w_sub = addr(env, w_sub, 0);
  d.cap = cap(env, tag);
  d.wcap = cap(env, w_sub);
  d.out_kind = CLG_MEM_HOST;
  uint64_t so = 0, sl = (uint64_t)len;
  uint64_t base[2] = {0, 0};
  int s = clg_decode_host(ENG(e), addr(env, bytes, off), &so, &sl, 1, &d, base);
  jlong r[6] = {(jlong)d.n_rec, (jlong)d.n_wide, d.err_status, d.err_span, d.err_off, d.err_tag};
  (*env)->SetLongArrayRegion(env, res, 0, 6, r);
  return s;
}

/* clg_log_get_id: out = {vertexId, isMain, irpLower, irpUpper, subpartition, job}. */
JNIEXPORT jint JNICALL FN(nLogGetId)(JNIEnv* env, jclass cls, jlong e, jint log, jlongArray out) {
  (void)cls;
  clg_causal_log_id id;
  uint32_t job = 0;
  memset(&id, 0, sizeof id);
  int s = clg_log_get_id(ENG(e), (uint32_t)log, &id, &job);
  jlong w[6] = {id.vertex_id, id.is_main, id.irp_lower, id.irp_upper, id.subpartition, (jlong)job};
  (*env)->SetLongArrayRegion(env, out, 0, 6, w);
  return s;
}

/* clg_enrich_batch: reqs packed as 5 longs per request {chLo, chHi, epoch, first, count};
 * res gets 4 longs per request {status, headerBytes, outOff, outLen}. */
JNIEXPORT jint JNICALL FN(nEnrichBatch)(JNIEnv* env, jclass cls, jlong e, jint strategy, jlongArray reqs,
                                        jintArray logs, jbyteArray flags, jobject out, jlongArray res,
                                        jlongArray total) {
  (void)cls;
  const jsize n = (*env)->GetArrayLength(env, reqs) / 5;
  jlong* rq = (*env)->GetLongArrayElements(env, reqs, NULL);
  jint* lg = (*env)->GetIntArrayElements(env, logs, NULL);
  jbyte* fl = (*env)->GetByteArrayElements(env, flags, NULL);
  clg_enrich_req* r = (clg_enrich_req*)calloc(n ? (size_t)n : 1u, sizeof(clg_enrich_req));
  for (jsize i = 0; i < n; ++i) {
    r[i].consumer = ch(rq[5 * i], rq[5 * i + 1]);
    r[i].epoch = rq[5 * i + 2];
    r[i].first = (uint32_t)rq[5 * i + 3];
    r[i].count = (uint32_t)rq[5 * i + 4];
  }
  uint64_t t = 0;
  int s = clg_enrich_batch(ENG(e), (uint32_t)strategy, r, (uint32_t)n, (const uint32_t*)lg, (const uint8_t*)fl,
                           addr(env, out, 0), cap(env, out), CLG_MEM_HOST, &t);
  for (jsize i = 0; i < n; ++i) {
    jlong w[4] = {r[i].status, (jlong)r[i].header_bytes, (jlong)r[i].out_off, (jlong)r[i].out_len};
    (*env)->SetLongArrayRegion(env, res, 4 * i, 4, w);
  }
  jlong tt = (jlong)t;
  (*env)->SetLongArrayRegion(env, total, 0, 1, &tt);
  free(r);
  (*env)->ReleaseByteArrayElements(env, flags, fl, JNI_ABORT);
  (*env)->ReleaseIntArrayElements(env, logs, lg, JNI_ABORT);
  (*env)->ReleaseLongArrayElements(env, reqs, rq, JNI_ABORT);
  return s;
}

/* clg_process_delta on msg[off, off + len); res = {epoch, nLogs, consumed}. */
JNIEXPORT jint JNICALL FN(nProcessDelta)(JNIEnv* env, jclass cls, jlong e, jint job, jint strategy, jobject msg,
                                         jint off, jint len, jintArray handles, jlongArray res) {
  (void)cls;
  int64_t ep = 0;
  uint32_t nl = 0;
  uint64_t used = 0;
  const jsize hc = (*env)->GetArrayLength(env, handles);
  jint* hs = (*env)->GetIntArrayElements(env, handles, NULL);
  int s = clg_process_delta(ENG(e), (uint32_t)job, (uint32_t)strategy, addr(env, msg, off), (uint64_t)len, CLG_MEM_HOST, &ep,
                            (uint32_t*)hs, (uint32_t)hc, &nl, &used);
  (*env)->ReleaseIntArrayElements(env, handles, hs, 0);
  jlong r[3] = {ep, (jlong)nl, (jlong)used};
  (*env)->SetLongArrayRegion(env, res, 0, 3, r);
  return s;
}

/* ReplayingState for one failed vertex: the merged DeterminantResponseEvent as written by
 * its write() (DeterminantResponseEvent.java:93-107) in `event`, the subpartition table as
 * 3 longs per entry {irpLower, irpUpper, index}.  Main-log SoA as in nDecodeLogs (res:
 * 6 longs); per subpartition 4 longs {count, status, errOff, errTag} in subRes and the
 * BufferBuilt sizes back to back in `sizes` (int32, native order). */
/* ReplayingState for one failed task (ReplayingState.java:67-70, :108-214) in one call:
 * bufs[0] = its main log's bytes (null: absent), bufs[1 + j] = subpartition j's recovery
 * buffer (null: absent, i.e. EMPTY_BUFFER), each a direct buffer holding lens[i] bytes;
 * subparts = (irpLower, irpUpper, index) per subpartition in the task's table order.
 * res = (n_rec, n_wide, err_status, err_span, err_off, err_tag) of the main-log decode;
 * sub_res = (count, status, err_off, err_tag, sizes_base) per subpartition. */
JNIEXPORT jint JNICALL FN(nReplayPrepare)(JNIEnv* env, jclass cls, jlong e, jshort vertex, jobjectArray bufs,
                                          jintArray lens, jlongArray subparts, jobject off, jobject tag, jobject v0,
                                          jobject w_idx, jobject w_rc, jobject w_v1, jobject w_var_off,
                                          jobject w_var_len, jobject w_sub, jlongArray res, jobject sizes,
                                          jlongArray sub_res) {
  (void)cls;
  const jsize ns = (*env)->GetArrayLength(env, subparts) / 3;
  jlong* sp = (*env)->GetLongArrayElements(env, subparts, NULL);
  jint* ln = (*env)->GetIntArrayElements(env, lens, NULL);
  clg_response_entry* ents = (clg_response_entry*)calloc((size_t)ns + 1u, sizeof(clg_response_entry));
  clg_causal_log_id* ids = (clg_causal_log_id*)calloc((size_t)ns + 1u, sizeof(clg_causal_log_id));
  uint64_t* sbase = (uint64_t*)calloc((size_t)ns + 1u, 8);
  uint64_t* cnt = (uint64_t*)calloc((size_t)ns + 1u, 8);
  int32_t* sst = (int32_t*)calloc((size_t)ns + 1u, 4);
  int64_t* soff = (int64_t*)calloc((size_t)ns + 1u, 8);
  int32_t* stg = (int32_t*)calloc((size_t)ns + 1u, 4);
  clg_response acc;
  memset(&acc, 0, sizeof acc);
  acc.found = 1;
  acc.vertex_id = vertex;
  acc.entries = ents;
  acc.cap = (uint32_t)ns + 1u;
  int s = CLG_OK;
  for (jsize i = 0; i <= ns && s == CLG_OK; ++i) {
    jobject b = (*env)->GetObjectArrayElement(env, bufs, i);
    clg_causal_log_id id;
    memset(&id, 0, sizeof id);
    id.vertex_id = vertex;
    id.is_main = i == 0;
    if (i > 0) {
      id.irp_lower = sp[3 * (i - 1)];
      id.irp_upper = sp[3 * (i - 1) + 1];
      id.subpartition = (int8_t)sp[3 * (i - 1) + 2];
      ids[i - 1] = id;
    }
    if (b) {
      s = clg_response_put(&acc, &id, addr(env, b, 0), (uint64_t)(uint32_t)ln[i]);
      (*env)->DeleteLocalRef(env, b);
    }
  }
  clg_decoded d;
  memset(&d, 0, sizeof d);
  d.off = (uint32_t*)addr(env, off, 0);
  d.tag = addr(env, tag, 0);
  d.v0 = (int64_t*)addr(env, v0, 0);
  d.w_idx = (uint32_t*)addr(env, w_idx, 0);
  d.w_rc = (int32_t*)addr(env, w_rc, 0);
  d.w_v1 = (int64_t*)addr(env, w_v1, 0);
  d.w_var_off = (uint32_t*)addr(env, w_var_off, 0);
  d.w_var_len = (uint32_t*)addr(env, w_var_len, 0);
  d.w_sub = addr(env, w_sub, 0);
  d.cap = cap(env, tag);
  d.wcap = cap(env, w_sub);
  d.out_kind = CLG_MEM_HOST;
  uint64_t main_base[2] = {0, 0};
  if (s == CLG_OK) {
    clg_replay_vertex v;
    memset(&v, 0, sizeof v);
    v.acc = &acc;
    v.subpartitions = ids;
    v.n_subpartitions = (uint32_t)ns;
    v.vertex_id = vertex;
    clg_replay_out o;
    memset(&o, 0, sizeof o);
    o.main = &d;
    o.main_rec_base = main_base;
    o.buffer_sizes = (int32_t*)addr(env, sizes, 0);
    o.sizes_cap = cap(env, sizes) / 4u;
    o.sizes_base = sbase;
    o.sub_count = cnt;
    o.sub_status = sst;
    o.sub_err_off = soff;
    o.sub_err_tag = stg;
    s = clg_replay_prepare(ENG(e), &v, 1, &o);
  }
  jlong r[6] = {(jlong)d.n_rec, (jlong)d.n_wide, d.err_status, d.err_span, d.err_off, d.err_tag};
  (*env)->SetLongArrayRegion(env, res, 0, 6, r);
  for (jsize i = 0; i < ns; ++i) {
    jlong w[5] = {(jlong)cnt[i], sst[i], soff[i], stg[i], (jlong)sbase[i]};
    (*env)->SetLongArrayRegion(env, sub_res, 5 * i, 5, w);
  }
  (*env)->ReleaseLongArrayElements(env, subparts, sp, JNI_ABORT);
  (*env)->ReleaseIntArrayElements(env, lens, ln, JNI_ABORT);
  free(ids), free(sbase), free(cnt), free(sst), free(soff), free(stg), free(ents);
  return s;
}

/* ---- in-flight (data) log: InMemorySubpartitionInFlightLogger (inflightlogging/, :28-207) or
 * SpillableSubpartitionInFlightLogger (:45-341), by type (CLG_IFL_IN_MEMORY / CLG_IFL_SPILLABLE) ---- */
JNIEXPORT jint JNICALL FN(nIflOpen)(JNIEnv* env, jclass cls, jlong e, jint type, jintArray out) {
  (void)cls;
  uint32_t h = 0;
  int s = clg_ifl_open_typed(ENG(e), (uint32_t)type, &h);
  put_int(env, out, (jint)h);
  return s;
}

JNIEXPORT jint JNICALL FN(nIflClose)(JNIEnv* env, jclass cls, jlong e, jint ifl) {
  (void)env;
  (void)cls;
  return clg_ifl_close(ENG(e), (uint32_t)ifl);
}

/* log(buffer, epochID, isFinished) :44-48 -- the buffer's readable bytes, copied to HBM. */
JNIEXPORT jint JNICALL FN(nIflLog)(JNIEnv* env, jclass cls, jlong e, jint ifl, jlong epoch, jobject buf, jint off,
                                   jint len) {
  (void)cls;
  const uint8_t* p = addr(env, buf, off);
  if (!p) return CLG_E_INVALID_ARG;
  uint32_t h = (uint32_t)ifl;
  int64_t ep = epoch;
  uint64_t o = 0;
  uint32_t n = (uint32_t)len;
  return clg_ifl_log_batch(ENG(e), &h, &ep, &o, &n, 1, p, CLG_MEM_HOST);
}

/* n buffers of one in-flight log, staged back to back in `buf`: lens[i] bytes each, epochs[i]. */
JNIEXPORT jint JNICALL FN(nIflLogBatch)(JNIEnv* env, jclass cls, jlong e, jint ifl, jlongArray epochs, jintArray lens,
                                        jobject buf, jint n) {
  (void)cls;
  if (n <= 0) return CLG_OK;
  const uint8_t* p = addr(env, buf, 0);
  if (!p) return CLG_E_INVALID_ARG;
  jlong* ep = (*env)->GetLongArrayElements(env, epochs, NULL);
  jint* ln = (*env)->GetIntArrayElements(env, lens, NULL);
  uint32_t* h = (uint32_t*)malloc(sizeof(uint32_t) * (size_t)n);
  uint64_t* off = (uint64_t*)malloc(sizeof(uint64_t) * (size_t)n);
  int st = CLG_E_INVALID_ARG;
  if (h && off) {
    uint64_t o = 0;
    for (jint i = 0; i < n; ++i) {
      h[i] = (uint32_t)ifl;
      off[i] = o;
      o += (uint32_t)ln[i];
    }
    st = clg_ifl_log_batch(ENG(e), h, (const int64_t*)ep, off, (const uint32_t*)ln, (uint32_t)n, p, CLG_MEM_HOST);
  }
  free(h);
  free(off);
  (*env)->ReleaseIntArrayElements(env, lens, ln, JNI_ABORT);
  (*env)->ReleaseLongArrayElements(env, epochs, ep, JNI_ABORT);
  return st;
}

JNIEXPORT jint JNICALL FN(nIflNotifyCheckpointComplete)(JNIEnv* env, jclass cls, jlong e, jint ifl, jlong cp) {
  (void)env;
  (void)cls;
  return clg_ifl_notify_checkpoint_complete(ENG(e), (uint32_t)ifl, cp);
}

/* getInFlightIterator(epoch, ignoreBuffers) drained into `out` (buffers back to back) and
 * `sizes` (i32 per buffer), at most maxBuffers (0: all; spillable only), or the next buffers of
 * the current iterator (flags CLG_IFL_CONTINUE, spillable only).  res = {status, buffers,
 * numberRemaining, bytes, required bytes, required buffers, end epoch, result flags}; the
 * call's status is CLG_E_CAPACITY when out/sizes are short (nothing taken then). */
JNIEXPORT jint JNICALL FN(nIflReplay)(JNIEnv* env, jclass cls, jlong e, jint ifl, jlong start, jint ignore,
                                      jint maxBuffers, jint flags, jobject out, jobject sizes, jobject epochs,
                                      jlongArray res) {
  (void)cls;
  clg_ifl_replay_req q;
  memset(&q, 0, sizeof q);
  q.ifl = (uint32_t)ifl;
  q.ignore_buffers = (uint32_t)ignore;
  q.start_epoch = start;
  q.max_buffers = (uint32_t)maxBuffers;
  q.flags = (uint32_t)flags;
  clg_ifl_replay_res r;
  memset(&r, 0, sizeof r);
  uint64_t total = 0, nbuf = 0;
  /* sizes (i32) and epochs (i64) are sized for the same number of buffers */
  uint64_t n_sizes = cap(env, sizes) / 4u;
  if (epochs && cap(env, epochs) / 8u < n_sizes) n_sizes = cap(env, epochs) / 8u;
  int s = clg_ifl_replay_batch(ENG(e), &q, 1, &r, addr(env, out, 0), cap(env, out), CLG_MEM_HOST,
                               (uint32_t*)addr(env, sizes, 0), (int64_t*)addr(env, epochs, 0), n_sizes, &total,
                               &nbuf);
  jlong w[8] = {r.status, (jlong)r.n_buffers, (jlong)r.remaining, (jlong)r.len, (jlong)total, (jlong)nbuf,
                (jlong)r.end_epoch, (jlong)r.flags};
  (*env)->SetLongArrayRegion(env, res, 0, 8, w);
  return s;
}
