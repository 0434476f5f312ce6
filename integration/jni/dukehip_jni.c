/* dukehip_jni.c -- JNI glue between io.sesam.dukemicroservice.gpu.DukeHip (Java 8) and the C-ABI
 * of libdukehip.so (include/dukehip.h).  Java arrays are pinned for the call (Get*ArrayElements
 * / GetPrimitiveArrayCritical is avoided: dk_* calls block on the GPU), strings cross as char[]
 * = UTF-16 code units = width-2 dk_column.  A negative DK_E* return becomes
 * RuntimeException(dk_last_error()).
 *
 * Build (next to libdukehip.so; needs a JDK, which this image does not have):
 *   gcc -std=c99 -O2 -shared -fPIC -I$JAVA_HOME/include -I$JAVA_HOME/include/linux -Iinclude \
 *       integration/jni/dukehip_jni.c -Lsesam-duke-microservice_amd/build -ldukehip \
 *       -o libdukehip_jni.so
 */
#include <jni.h>
#include <stdint.h>
#include <stdlib.h>
#include <string.h>

#include "dukehip.h"

#define JFN(name) JNICALL Java_io_sesam_dukemicroservice_gpu_DukeHip_##name

static int throw_dk(JNIEnv* env, int rc) {
  if (rc >= 0) return 0;
  jclass ex = (*env)->FindClass(env, "java/lang/RuntimeException");
  (*env)->ThrowNew(env, ex, dk_last_error());
  return 1;
}

static void throw_msg(JNIEnv* env, const char* msg) {
  (*env)->ThrowNew(env, (*env)->FindClass(env, "java/lang/RuntimeException"), msg);
}

JNIEXPORT jlong JFN(create)(JNIEnv* env, jclass cls, jintArray cmp, jintArray q, jintArray formula,
                            jintArray tok, jdoubleArray low, jdoubleArray high, jdoubleArray minRatio,
                            jdouble threshold, jdouble maybe, jint mode, jint nkeys, jint device) {
  (void)cls;
  const jsize n = (*env)->GetArrayLength(env, cmp);
  if (n > 16) {
    throw_msg(env, "more than 16 properties");
    return 0;
  }
  dk_property props[16];
  jint *c = (*env)->GetIntArrayElements(env, cmp, NULL), *qq = (*env)->GetIntArrayElements(env, q, NULL);
  jint *f = (*env)->GetIntArrayElements(env, formula, NULL), *t = (*env)->GetIntArrayElements(env, tok, NULL);
  jdouble *lo = (*env)->GetDoubleArrayElements(env, low, NULL), *hi = (*env)->GetDoubleArrayElements(env, high, NULL);
  jdouble* mr = (*env)->GetDoubleArrayElements(env, minRatio, NULL);
  for (jsize i = 0; i < n; ++i) {
    props[i].comparator = c[i];
    props[i].qgram_q = qq[i];
    props[i].qgram_formula = f[i];
    props[i].qgram_tokenizer = t[i];
    props[i].low = lo[i];
    props[i].high = hi[i];
    props[i].min_ratio = mr[i];
  }
  (*env)->ReleaseIntArrayElements(env, cmp, c, JNI_ABORT);
  (*env)->ReleaseIntArrayElements(env, q, qq, JNI_ABORT);
  (*env)->ReleaseIntArrayElements(env, formula, f, JNI_ABORT);
  (*env)->ReleaseIntArrayElements(env, tok, t, JNI_ABORT);
  (*env)->ReleaseDoubleArrayElements(env, low, lo, JNI_ABORT);
  (*env)->ReleaseDoubleArrayElements(env, high, hi, JNI_ABORT);
  (*env)->ReleaseDoubleArrayElements(env, minRatio, mr, JNI_ABORT);
  dk_schema s;
  memset(&s, 0, sizeof s);
  s.nprops = (int32_t)n;
  s.props = props;
  s.threshold = threshold;
  s.maybe_threshold = maybe;
  s.mode = mode;
  s.nkeys = nkeys;
  dk_ctx* ctx = NULL;
  if (throw_dk(env, dk_create(&s, device, &ctx))) return 0;
  return (jlong)(intptr_t)ctx;
}

JNIEXPORT void JFN(destroy)(JNIEnv* env, jclass cls, jlong ctx) {
  (void)env;
  (void)cls;
  dk_destroy((dk_ctx*)(intptr_t)ctx);
}

/* the pinned pieces of one width-2 column */
typedef struct {
  jintArray joff;
  jcharArray junits;
  jbyteArray jpresent;
  jint* off;
  jchar* units;
  jbyte* present;
} Pinned;

static dk_column pin_column(JNIEnv* env, jintArray off, jcharArray units, jbyteArray present, Pinned* P) {
  P->joff = off;
  P->junits = units;
  P->jpresent = present;
  P->off = (*env)->GetIntArrayElements(env, off, NULL);
  P->units = (*env)->GetCharArrayElements(env, units, NULL);
  P->present = present ? (*env)->GetByteArrayElements(env, present, NULL) : NULL;
  dk_column c;
  c.offsets = (const uint32_t*)P->off;
  c.units = P->units;
  c.width = 2;
  c.present = (const uint8_t*)P->present;
  return c;
}

static void unpin_column(JNIEnv* env, Pinned* P) {
  (*env)->ReleaseIntArrayElements(env, P->joff, P->off, JNI_ABORT);
  (*env)->ReleaseCharArrayElements(env, P->junits, P->units, JNI_ABORT);
  if (P->present) (*env)->ReleaseByteArrayElements(env, P->jpresent, P->present, JNI_ABORT);
}

JNIEXPORT jintArray JFN(upsert)(JNIEnv* env, jclass cls, jlong ctx, jboolean transient_, jint n,
                                jlongArray ident, jbyteArray group, jbyteArray deleted,
                                jobjectArray offsets, jobjectArray units, jobjectArray present,
                                jobjectArray keyOffsets, jobjectArray keyUnits) {
  (void)cls;
  const jsize np = (*env)->GetArrayLength(env, offsets);
  const jsize nk = keyOffsets ? (*env)->GetArrayLength(env, keyOffsets) : 0;
  if (np > 16 || nk > 8) {
    throw_msg(env, "too many properties / key functions");
    return NULL;
  }
  dk_column cols[16], kcols[8];
  Pinned pc[16], pk[8];
  for (jsize p = 0; p < np; ++p)
    cols[p] = pin_column(env, (jintArray)(*env)->GetObjectArrayElement(env, offsets, p),
                         (jcharArray)(*env)->GetObjectArrayElement(env, units, p),
                         (jbyteArray)(*env)->GetObjectArrayElement(env, present, p), &pc[p]);
  for (jsize k = 0; k < nk; ++k)
    kcols[k] = pin_column(env, (jintArray)(*env)->GetObjectArrayElement(env, keyOffsets, k),
                          (jcharArray)(*env)->GetObjectArrayElement(env, keyUnits, k), NULL, &pk[k]);
  jlong* id = (*env)->GetLongArrayElements(env, ident, NULL);
  jbyte* g = group ? (*env)->GetByteArrayElements(env, group, NULL) : NULL;
  jbyte* d = deleted ? (*env)->GetByteArrayElements(env, deleted, NULL) : NULL;
  dk_batch b;
  memset(&b, 0, sizeof b);
  b.n = (uint64_t)n;
  b.ident = (const uint64_t*)id;
  b.group = (const uint8_t*)g;
  b.deleted = (const uint8_t*)d;
  b.columns = cols;
  b.key_columns = nk ? kcols : NULL;
  uint32_t* rows = (uint32_t*)malloc((size_t)n * 4 + 4);
  const int rc = transient_ ? dk_upsert_transient((dk_ctx*)(intptr_t)ctx, &b, rows)
                            : dk_upsert((dk_ctx*)(intptr_t)ctx, &b, rows);
  for (jsize p = 0; p < np; ++p) unpin_column(env, &pc[p]);
  for (jsize k = 0; k < nk; ++k) unpin_column(env, &pk[k]);
  (*env)->ReleaseLongArrayElements(env, ident, id, JNI_ABORT);
  if (g) (*env)->ReleaseByteArrayElements(env, group, g, JNI_ABORT);
  if (d) (*env)->ReleaseByteArrayElements(env, deleted, d, JNI_ABORT);
  jintArray out = NULL;
  if (!throw_dk(env, rc)) {
    out = (*env)->NewIntArray(env, n);
    (*env)->SetIntArrayRegion(env, out, 0, n, (const jint*)rows);
  }
  free(rows);
  return out;
}

JNIEXPORT void JFN(dropTransient)(JNIEnv* env, jclass cls, jlong ctx) {
  (void)cls;
  throw_dk(env, dk_drop_transient((dk_ctx*)(intptr_t)ctx));
}

JNIEXPORT void JFN(setOverwrite)(JNIEnv* env, jclass cls, jlong ctx, jboolean on) {
  (void)cls;
  throw_dk(env, dk_set_overwrite((dk_ctx*)(intptr_t)ctx, on ? 1 : 0));
}

JNIEXPORT jlong JFN(match)(JNIEnv* env, jclass cls, jlong ctx, jintArray rows) {
  (void)cls;
  const jsize n = (*env)->GetArrayLength(env, rows);
  jint* q = (*env)->GetIntArrayElements(env, rows, NULL);
  dk_result* res = NULL;
  const int rc = dk_match((dk_ctx*)(intptr_t)ctx, (const uint32_t*)q, (uint64_t)n, DK_MATCH_HOST, &res);
  (*env)->ReleaseIntArrayElements(env, rows, q, JNI_ABORT);
  if (throw_dk(env, rc)) return 0;
  return (jlong)(intptr_t)res;
}

JNIEXPORT jlongArray JFN(resultFirst)(JNIEnv* env, jclass cls, jlong result) {
  (void)cls;
  const dk_result* r = (const dk_result*)(intptr_t)result;
  jlongArray out = (*env)->NewLongArray(env, (jsize)(r->nqueries + 1));
  (*env)->SetLongArrayRegion(env, out, 0, (jsize)(r->nqueries + 1), (const jlong*)r->first);
  return out;
}

JNIEXPORT jintArray JFN(resultCandidate)(JNIEnv* env, jclass cls, jlong result) {
  (void)cls;
  const dk_result* r = (const dk_result*)(intptr_t)result;
  jintArray out = (*env)->NewIntArray(env, (jsize)r->n);
  if (r->n) (*env)->SetIntArrayRegion(env, out, 0, (jsize)r->n, (const jint*)r->candidate);
  return out;
}

JNIEXPORT jdoubleArray JFN(resultProb)(JNIEnv* env, jclass cls, jlong result) {
  (void)cls;
  const dk_result* r = (const dk_result*)(intptr_t)result;
  jdoubleArray out = (*env)->NewDoubleArray(env, (jsize)r->n);
  if (r->n) (*env)->SetDoubleArrayRegion(env, out, 0, (jsize)r->n, r->prob);
  return out;
}

JNIEXPORT jbyteArray JFN(resultKind)(JNIEnv* env, jclass cls, jlong result) {
  (void)cls;
  const dk_result* r = (const dk_result*)(intptr_t)result;
  jbyteArray out = (*env)->NewByteArray(env, (jsize)r->n);
  if (r->n) (*env)->SetByteArrayRegion(env, out, 0, (jsize)r->n, (const jbyte*)r->kind);
  return out;
}

JNIEXPORT jlong JFN(resultPairsScored)(JNIEnv* env, jclass cls, jlong result) {
  (void)env;
  (void)cls;
  return (jlong)((const dk_result*)(intptr_t)result)->pairs_scored;
}

JNIEXPORT void JFN(freeResult)(JNIEnv* env, jclass cls, jlong result) {
  (void)env;
  (void)cls;
  dk_free_result((dk_result*)(intptr_t)result);
}

JNIEXPORT jdouble JFN(compareRows)(JNIEnv* env, jclass cls, jlong ctx, jint r1, jint r2) {
  (void)cls;
  double p = 0.0;
  throw_dk(env, dk_compare_rows((dk_ctx*)(intptr_t)ctx, (uint32_t)r1, (uint32_t)r2, &p));
  return p;
}

JNIEXPORT jdouble JFN(compareValues)(JNIEnv* env, jclass cls, jlong ctx, jobjectArray a, jobjectArray b) {
  (void)cls;
  const jsize np = (*env)->GetArrayLength(env, a);
  if (np > 16) {
    throw_msg(env, "more than 16 properties");
    return 0.0;
  }
  /* one width-2 column per property holding the two records' values */
  dk_column cols[16];
  uint32_t off[16][3];
  uint8_t present[16][2];
  jchar* units[16];
  for (jsize p = 0; p < np; ++p) {
    jstring s[2] = {(jstring)(*env)->GetObjectArrayElement(env, a, p),
                    (jstring)(*env)->GetObjectArrayElement(env, b, p)};
    jsize len[2];
    for (int r = 0; r < 2; ++r) len[r] = s[r] ? (*env)->GetStringLength(env, s[r]) : 0;
    units[p] = (jchar*)malloc(((size_t)len[0] + len[1] + 1) * sizeof(jchar));
    off[p][0] = 0;
    off[p][1] = (uint32_t)len[0];
    off[p][2] = (uint32_t)(len[0] + len[1]);
    for (int r = 0; r < 2; ++r) {
      present[p][r] = s[r] != NULL;
      if (s[r]) (*env)->GetStringRegion(env, s[r], 0, len[r], units[p] + off[p][r]);
    }
    cols[p].offsets = off[p];
    cols[p].units = units[p];
    cols[p].width = 2;
    cols[p].present = present[p];
  }
  const uint64_t ident[2] = {0, 1};
  dk_batch pair;
  memset(&pair, 0, sizeof pair);
  pair.n = 2;
  pair.ident = ident;
  pair.columns = cols;
  double prob = 0.0;
  const int rc = dk_compare_values((dk_ctx*)(intptr_t)ctx, &pair, &prob);
  for (jsize p = 0; p < np; ++p) free(units[p]);
  throw_dk(env, rc);
  return prob;
}

JNIEXPORT void JFN(setProfiling)(JNIEnv* env, jclass cls, jlong ctx, jboolean on) {
  (void)cls;
  throw_dk(env, dk_set_profiling((dk_ctx*)(intptr_t)ctx, on ? 1 : 0));
}

JNIEXPORT void JFN(setResultRegion)(JNIEnv* env, jclass cls, jlong ctx, jobject region, jlong maxQueries) {
  (void)cls;
  void* base = region ? (*env)->GetDirectBufferAddress(env, region) : NULL;
  const jlong bytes = region ? (*env)->GetDirectBufferCapacity(env, region) : 0;
  throw_dk(env, dk_set_result_region((dk_ctx*)(intptr_t)ctx, base, (uint64_t)bytes, (uint64_t)maxQueries));
}
