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
                                   jlongArray out) {
  (void)cls;
  clg_config cfg;
  clg_config_default(&cfg);
  cfg.segment_bytes = (uint32_t)seg;
  cfg.pool_segments = (uint32_t)pool;
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

JNIEXPORT jint JNICALL FN(nLogOpen)(JNIEnv* env, jclass cls, jlong e, jshort vid, jboolean is_main, jlong lo,
                                    jlong hi, jbyte sub, jintArray out) {
  (void)cls;
  clg_causal_log_id id;
  memset(&id, 0, sizeof id);
  id.vertex_id = vid;
  id.is_main = is_main ? 1 : 0;
  id.irp_lower = lo;
  id.irp_upper = hi;
  id.subpartition = sub;
  uint32_t h = 0;
  int st = clg_log_open(ENG(e), &id, &h);
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

JNIEXPORT jint JNICALL FN(nTruncateAll)(JNIEnv* env, jclass cls, jlong e, jlong cp, jintArray applied) {
  (void)cls;
  int32_t a = 0;
  int st = clg_truncate_all(ENG(e), cp, &a);
  put_int(env, applied, a);
  return st;
}
