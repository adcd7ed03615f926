/* TEST INFRASTRUCTURE (CPU, no JVM, no GPU): drives the JNI shim's nReplayPrepare
 * (jni/clonos_jni.c) through a fake JNIEnv built on tests/jni_stub/jni.h.  The response is
 * accumulated by the real clg_response_put (libclonos_engine.so); clg_replay_prepare is
 * replaced by a recorder defined here (an executable's definition interposes on the
 * library's), which checks what the shim hands the engine and writes known outputs, so the
 * test sees exactly how the shim unpacks Java arrays and direct buffers and packs res /
 * subRes back (EngineReplayPreparation.java's layout).  Prints "OK" and exits 0, or names
 * the first mismatch and exits 1.  Built and run by tests/test_jni_shim.py. */
#include <stdio.h>
#include <stdlib.h>
#include <string.h>

#include "../jni/clonos_jni.c"

enum { K_BUF = 1, K_INT, K_LONG, K_OBJ };
typedef struct Obj {
  int kind;
  void* data;  /* buffer bytes / jint[] / jlong[] / jobject[] */
  jlong len;   /* bytes for a buffer, elements otherwise */
  int released, pinned;
} Obj;

static int fails = 0;
#define CHECK(c, ...)                     \
  do {                                    \
    if (!(c)) {                           \
      printf("FAIL %s:%d: ", __FILE__, __LINE__); \
      printf(__VA_ARGS__);                \
      printf("\n");                       \
      ++fails;                            \
    }                                     \
  } while (0)

static jsize f_len(JNIEnv* e, jarray a) { (void)e; return (jsize)((Obj*)a)->len; }
static jint* f_ints(JNIEnv* e, jintArray a, jboolean* c) {
  (void)e; (void)c; ((Obj*)a)->pinned++;
  return (jint*)((Obj*)a)->data;
}
static jlong* f_longs(JNIEnv* e, jlongArray a, jboolean* c) {
  (void)e; (void)c; ((Obj*)a)->pinned++;
  return (jlong*)((Obj*)a)->data;
}
static void f_rel_ints(JNIEnv* e, jintArray a, jint* p, jint mode) {
  (void)e; (void)p; (void)mode; ((Obj*)a)->released++;
}
static void f_rel_longs(JNIEnv* e, jlongArray a, jlong* p, jint mode) {
  (void)e; (void)p; (void)mode; ((Obj*)a)->released++;
}
static void f_set_longs(JNIEnv* e, jlongArray a, jsize at, jsize n, const jlong* v) {
  (void)e;
  Obj* o = (Obj*)a;
  CHECK(at >= 0 && at + n <= o->len, "SetLongArrayRegion [%d, %d) past %lld", at, at + n, (long long)o->len);
  if (at >= 0 && at + n <= o->len) memcpy((jlong*)o->data + at, v, (size_t)n * 8);
}
static void f_set_ints(JNIEnv* e, jintArray a, jsize at, jsize n, const jint* v) {
  (void)e;
  Obj* o = (Obj*)a;
  if (at >= 0 && at + n <= o->len) memcpy((jint*)o->data + at, v, (size_t)n * 4);
}
static void* f_addr(JNIEnv* e, jobject b) { (void)e; return ((Obj*)b)->kind == K_BUF ? ((Obj*)b)->data : NULL; }
static jlong f_cap(JNIEnv* e, jobject b) { (void)e; return ((Obj*)b)->kind == K_BUF ? ((Obj*)b)->len : -1; }
static jobject f_elem(JNIEnv* e, jobjectArray a, jsize i) { (void)e; return ((jobject*)((Obj*)a)->data)[i]; }
static int local_refs_deleted = 0;
static void f_del(JNIEnv* e, jobject o) { (void)e; (void)o; ++local_refs_deleted; }

static const struct JNINativeInterface_ kEnvTable = {
    NULL, f_len, f_ints, f_longs, NULL, f_rel_ints, f_rel_longs, NULL, f_set_ints, f_set_longs,
    f_addr, f_cap, f_elem, f_del};

/* ---- the recorder standing in for the engine ---- */
static const char* kMain = "main-log-bytes";
static const char* kSub0 = "sub0";
static const char* kSub2 = "subpartition-two";
static int calls = 0, ret_status = CLG_OK;

int clg_replay_prepare(clg_engine* e, const clg_replay_vertex* v, uint32_t n, clg_replay_out* o) {
  ++calls;
  CHECK((intptr_t)e == 0x1234, "engine handle %p", (void*)e);
  CHECK(n == 1, "n_vertices %u", n);
  CHECK(v->vertex_id == 7 && v->n_subpartitions == 3, "vertex %d, %u subpartitions", v->vertex_id,
        v->n_subpartitions);
  /* the table: (irpLower, irpUpper, index) per entry, in order */
  for (uint32_t j = 0; j < 3; ++j) {
    const clg_causal_log_id* id = &v->subpartitions[j];
    CHECK(!id->is_main && id->vertex_id == 7 && id->irp_lower == (int64_t)(100 + j) &&
              id->irp_upper == (int64_t)(200 + j) && id->subpartition == (int8_t)j,
          "subpartition %u id", j);
  }
  /* the response: the main log and subpartitions 0 and 2 (1 is absent) */
  const clg_response* r = v->acc;
  CHECK(r->found == 1 && r->vertex_id == 7 && r->n == 3, "response found %d vertex %d n %u", r->found, r->vertex_id, r->n);
  int seen = 0;
  for (uint32_t i = 0; i < r->n; ++i) {
    const clg_response_entry* en = &r->entries[i];
    const char* want = en->id.is_main ? kMain : (en->id.subpartition == 0 ? kSub0 : kSub2);
    CHECK(!en->id.is_main || en->id.irp_lower == 0, "main id");
    CHECK(en->id.is_main || en->id.subpartition == 0 || en->id.subpartition == 2, "entry %u subpartition %d", i,
          en->id.subpartition);
    CHECK(en->len == strlen(want) && memcmp(en->bytes, want, en->len) == 0, "entry %u bytes", i);
    seen |= en->id.is_main ? 1 : (en->id.subpartition == 0 ? 2 : 4);
  }
  CHECK(seen == 7, "entries seen %d", seen);
  /* outputs: the main SoA and per-subpartition results */
  clg_decoded* d = o->main;
  CHECK(d->out_kind == CLG_MEM_HOST && d->cap == 16 && d->wcap == 4, "main out kind %u cap %llu wcap %llu",
        d->out_kind, (unsigned long long)d->cap, (unsigned long long)d->wcap);
  for (uint32_t i = 0; i < 3; ++i) {
    d->off[i] = 10 * i;
    d->tag[i] = (uint8_t)(i + 1);
    d->v0[i] = -(int64_t)i;
  }
  d->w_idx[0] = 2;
  d->w_rc[0] = 5;
  d->w_v1[0] = 99;
  d->w_var_off[0] = 3;
  d->w_var_len[0] = 4;
  d->w_sub[0] = 1;
  d->n_rec = 3;
  d->n_wide = 1;
  d->err_status = ret_status;
  d->err_span = ret_status ? 0u : 0xFFFFFFFFu;  /* (unsigned: the shim widens it as is) */
  d->err_off = ret_status ? 11 : -1;
  d->err_tag = ret_status ? 9 : -1;
  o->main_rec_base[0] = 0;
  o->main_rec_base[1] = 3;
  CHECK(o->sizes_cap == 8, "sizes_cap %llu", (unsigned long long)o->sizes_cap);
  for (uint32_t j = 0; j < 3; ++j) {
    o->sub_count[j] = j == 1 ? 0 : j + 2;
    o->sub_status[j] = j == 2 ? CLG_E_CORRUPT_TAG : CLG_OK;
    o->sub_err_off[j] = j == 2 ? 33 : -1;
    o->sub_err_tag[j] = j == 2 ? 8 : -1;
    o->sizes_base[j] = j == 0 ? 0 : 2;
  }
  o->sizes_base[3] = 6;
  for (int k = 0; k < 6; ++k) o->buffer_sizes[k] = 1000 + k;
  return ret_status;
}

static Obj buf(const char* s) {
  Obj o = {K_BUF, (void*)s, (jlong)strlen(s), 0, 0};
  return o;
}

static int run(int status) {
  ret_status = status;
  JNIEnv env = &kEnvTable;
  Obj bm = buf(kMain), b0 = buf(kSub0), b2 = buf(kSub2);
  jobject bobjs[4] = {&bm, &b0, NULL, &b2};
  Obj bufs = {K_OBJ, bobjs, 4, 0, 0};
  jint lv[4] = {(jint)strlen(kMain), (jint)strlen(kSub0), 0, (jint)strlen(kSub2)};
  Obj lens = {K_INT, lv, 4, 0, 0};
  jlong sv[9] = {100, 200, 0, 101, 201, 1, 102, 202, 2};
  Obj subs = {K_LONG, sv, 9, 0, 0};
  uint32_t off[16], wi[4], wvo[4], wvl[4];
  uint8_t tag[16], ws[4];
  int64_t v0[16], wv1[4];
  int32_t wrc[4], sizes[8];
  memset(off, 0xEE, sizeof off);
  Obj o_off = {K_BUF, off, sizeof off, 0, 0}, o_tag = {K_BUF, tag, sizeof tag, 0, 0}, o_v0 = {K_BUF, v0, sizeof v0, 0, 0};
  Obj o_wi = {K_BUF, wi, sizeof wi, 0, 0}, o_wrc = {K_BUF, wrc, sizeof wrc, 0, 0}, o_wv1 = {K_BUF, wv1, sizeof wv1, 0, 0};
  Obj o_wvo = {K_BUF, wvo, sizeof wvo, 0, 0}, o_wvl = {K_BUF, wvl, sizeof wvl, 0, 0}, o_ws = {K_BUF, ws, sizeof ws, 0, 0};
  Obj o_sizes = {K_BUF, sizes, sizeof sizes, 0, 0};
  jlong rv[6], srv[15];
  memset(rv, 0x55, sizeof rv);
  memset(srv, 0x55, sizeof srv);
  Obj res = {K_LONG, rv, 6, 0, 0}, sres = {K_LONG, srv, 15, 0, 0};
  local_refs_deleted = 0;
  const int c0 = calls;
  const jint st = FN(nReplayPrepare)(&env, NULL, (jlong)0x1234, (jshort)7, &bufs, &lens, &subs, &o_off, &o_tag, &o_v0,
                                     &o_wi, &o_wrc, &o_wv1, &o_wvo, &o_wvl, &o_ws, &res, &o_sizes, &sres);
  CHECK(calls == c0 + 1, "clg_replay_prepare calls %d", calls - c0);
  CHECK(st == status, "status %d, want %d", st, status);
  /* res = (n_rec, n_wide, err_status, err_span, err_off, err_tag) */
  const jlong want_res[6] = {3, 1, status, status ? 0 : 0xFFFFFFFFll, status ? 11 : -1, status ? 9 : -1};
  for (int i = 0; i < 6; ++i) CHECK(rv[i] == want_res[i], "res[%d] = %lld, want %lld", i, (long long)rv[i], (long long)want_res[i]);
  /* subRes = (count, status, err_off, err_tag, sizes_base) per subpartition */
  const jlong want_sub[15] = {2, CLG_OK, -1, -1, 0, 0, CLG_OK, -1, -1, 2, 4, CLG_E_CORRUPT_TAG, 33, 8, 2};
  for (int i = 0; i < 15; ++i)
    CHECK(srv[i] == want_sub[i], "subRes[%d] = %lld, want %lld", i, (long long)srv[i], (long long)want_sub[i]);
  /* the outputs landed in the direct buffers themselves (no copies) */
  CHECK(off[0] == 0 && off[1] == 10 && off[2] == 20 && tag[2] == 3 && v0[1] == -1, "main SoA");
  CHECK(wi[0] == 2 && wrc[0] == 5 && wv1[0] == 99 && wvo[0] == 3 && wvl[0] == 4 && ws[0] == 1, "wide SoA");
  CHECK(sizes[0] == 1000 && sizes[5] == 1005, "buffer sizes");
  /* every pinned array released, every non-null element's local ref deleted */
  CHECK(subs.pinned == subs.released && lens.pinned == lens.released, "pins %d/%d, %d/%d", subs.pinned,
        subs.released, lens.pinned, lens.released);
  CHECK(local_refs_deleted == 3, "local refs deleted %d", local_refs_deleted);
  return 0;
}

int main(void) {
  run(CLG_OK);
  run(CLG_E_CORRUPT_TAG);  /* an engine error: the status and res still come back */
  if (fails) return 1;
  printf("OK\n");
  return 0;
}
