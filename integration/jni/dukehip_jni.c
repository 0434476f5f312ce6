/* dukehip_jni.c -- JNI glue between io.sesam.dukemicroservice.gpu.DukeHip (Java 8) and the C-ABI
 * of libdukehip.so (include/dukehip.h).  Java arrays are pinned for the call (Get*ArrayElements
 * / GetPrimitiveArrayCritical is avoided: dk_* calls block on the GPU), strings cross as char[]
 * = UTF-16 code units = width-2 dk_column.  A negative DK_E* return becomes
 * DukeHipException(code, dk_last_error()).
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
#define CTX(h) ((dk_ctx*)(intptr_t)(h))

static void throw_msg(JNIEnv* env, const char* msg) {
  (*env)->ThrowNew(env, (*env)->FindClass(env, "java/lang/RuntimeException"), msg);
}

/* DukeHipException(code, dk_last_error()); if that class, its constructor or the object
 * cannot be made, the pending NoClassDefFoundError / OutOfMemoryError is cleared (no JNI call
 * but a few may run with an exception pending) and a RuntimeException carries the message. */
static int throw_dk(JNIEnv* env, int rc) {
  if (rc >= 0) return 0;
  const char* text = dk_last_error();
  jclass ex = (*env)->FindClass(env, "io/sesam/dukemicroservice/gpu/DukeHipException");
  jmethodID init = NULL;
  jstring msg = NULL;
  jobject e = NULL;
  if (ex && !(*env)->ExceptionCheck(env))
    init = (*env)->GetMethodID(env, ex, "<init>", "(ILjava/lang/String;)V");
  if (init && !(*env)->ExceptionCheck(env)) msg = (*env)->NewStringUTF(env, text);
  if (msg && !(*env)->ExceptionCheck(env)) e = (*env)->NewObject(env, ex, init, (jint)rc, msg);
  if (e && !(*env)->ExceptionCheck(env)) {
    (*env)->Throw(env, (jthrowable)e);
  } else {
    (*env)->ExceptionClear(env);
    throw_msg(env, text);
  }
  return 1;
}

/* ---- pipeline ctx --------------------------------------------------------------------- */

JNIEXPORT jlong JFN(create)(JNIEnv* env, jclass cls, jintArray cmp, jintArray q, jintArray formula,
                            jintArray tok, jdoubleArray low, jdoubleArray high, jdoubleArray minRatio,
                            jdouble threshold, jdouble maybe, jint mode, jint nkeys,
                            jintArray lookupProps, jint maxSearchHits, jfloat minRelevance,
                            jintArray devices, jintArray orders) {
  (void)cls;
  const jsize n = (*env)->GetArrayLength(env, cmp);
  const jsize no = orders ? (*env)->GetArrayLength(env, orders) : 0;
  if (no % (n ? n : 1) != 0 || no > DK_MAX_ORDER_CLASSES * 16) {
    throw_msg(env, "orders must hold norders x nprops entries (norders <= DK_MAX_ORDER_CLASSES)");
    return 0;
  }
  const jsize nl = lookupProps ? (*env)->GetArrayLength(env, lookupProps) : 0;
  const jsize nd = devices ? (*env)->GetArrayLength(env, devices) : 0;
  if (n > 16 || nl > 16 || nd > 64) {
    throw_msg(env, "more than 16 properties / lookup properties, or 64 devices");
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
  int32_t ord[DK_MAX_ORDER_CLASSES * 16];
  if (no) {  /* Processor.compare's HashMap order classes */
    (*env)->GetIntArrayRegion(env, orders, 0, no, (jint*)ord);
    s.norders = (int32_t)(no / (n ? n : 1));
    s.orders = ord;
  }
  int32_t lookup[16];
  dk_lucene luc;
  if (lookupProps) {  /* IncrementalLuceneDatabase semantics on the device */
    (*env)->GetIntArrayRegion(env, lookupProps, 0, nl, (jint*)lookup);
    memset(&luc, 0, sizeof luc);
    luc.nlookup = (int32_t)nl;
    luc.lookup_prop = lookup;
    luc.max_hits = maxSearchHits;
    luc.min_relevance = minRelevance;
    s.lucene = &luc;
  }
  int dev[64];
  int ndev = 1;
  dev[0] = 0;
  if (nd > 0) {
    (*env)->GetIntArrayRegion(env, devices, 0, nd, (jint*)dev);
    ndev = (int)nd;
  }
  dk_ctx* ctx = NULL;
  if (throw_dk(env, ndev > 1 ? dk_create_multi(&s, dev, ndev, &ctx) : dk_create(&s, dev[0], &ctx))) return 0;
  return (jlong)(intptr_t)ctx;
}

JNIEXPORT void JFN(destroy)(JNIEnv* env, jclass cls, jlong ctx) {
  (void)env;
  (void)cls;
  dk_destroy(CTX(ctx));
}

JNIEXPORT jint JFN(numDevices)(JNIEnv* env, jclass cls, jlong ctx) {
  (void)env;
  (void)cls;
  return (jint)dk_num_devices(CTX(ctx));
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

static jintArray rows_array(JNIEnv* env, const uint32_t* rows, uint64_t n) {
  jintArray out = (*env)->NewIntArray(env, (jsize)n);
  if (out && n) (*env)->SetIntArrayRegion(env, out, 0, (jsize)n, (const jint*)rows);
  return out;
}

JNIEXPORT jintArray JFN(upsert)(JNIEnv* env, jclass cls, jlong ctx, jboolean transient_, jint n,
                                jlongArray ident, jbyteArray group, jbyteArray deleted,
                                jobjectArray offsets, jobjectArray units, jobjectArray present,
                                jobjectArray keyOffsets, jobjectArray keyUnits, jbyteArray orderClass) {
  (void)cls;
  const jsize np = (*env)->GetArrayLength(env, offsets);
  if (orderClass && (*env)->GetArrayLength(env, orderClass) != n) {
    throw_msg(env, "orderClass must hold one class per record");
    return NULL;
  }
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
  jbyte* oc = orderClass ? (*env)->GetByteArrayElements(env, orderClass, NULL) : NULL;
  dk_batch b;
  memset(&b, 0, sizeof b);
  b.n = (uint64_t)n;
  b.ident = (const uint64_t*)id;
  b.group = (const uint8_t*)g;
  b.deleted = (const uint8_t*)d;
  b.columns = cols;
  b.key_columns = nk ? kcols : NULL;
  b.order_class = (const uint8_t*)oc;
  uint32_t* rows = (uint32_t*)malloc((size_t)n * 4 + 4);
  const int rc = transient_ ? dk_upsert_transient(CTX(ctx), &b, rows) : dk_upsert(CTX(ctx), &b, rows);
  if (oc) (*env)->ReleaseByteArrayElements(env, orderClass, oc, JNI_ABORT);
  for (jsize p = 0; p < np; ++p) unpin_column(env, &pc[p]);
  for (jsize k = 0; k < nk; ++k) unpin_column(env, &pk[k]);
  (*env)->ReleaseLongArrayElements(env, ident, id, JNI_ABORT);
  if (g) (*env)->ReleaseByteArrayElements(env, group, g, JNI_ABORT);
  if (d) (*env)->ReleaseByteArrayElements(env, deleted, d, JNI_ABORT);
  jintArray out = NULL;
  if (!throw_dk(env, rc)) out = rows_array(env, rows, (uint64_t)n);
  free(rows);
  return out;
}

JNIEXPORT void JFN(dropTransient)(JNIEnv* env, jclass cls, jlong ctx) {
  (void)cls;
  throw_dk(env, dk_drop_transient(CTX(ctx)));
}

JNIEXPORT void JFN(luceneSetStats)(JNIEnv* env, jclass cls, jlong ctx, jint mode) {
  (void)cls;
  throw_dk(env, dk_lucene_set_stats(CTX(ctx), (int)mode));
}

JNIEXPORT void JFN(luceneMerge)(JNIEnv* env, jclass cls, jlong ctx) {
  (void)cls;
  throw_dk(env, dk_lucene_merge(CTX(ctx)));
}

JNIEXPORT void JFN(setOverwrite)(JNIEnv* env, jclass cls, jlong ctx, jboolean on) {
  (void)cls;
  throw_dk(env, dk_set_overwrite(CTX(ctx), on ? 1 : 0));
}

JNIEXPORT jlong JFN(numRows)(JNIEnv* env, jclass cls, jlong ctx) {
  (void)env;
  (void)cls;
  return (jlong)dk_num_rows(CTX(ctx));
}

JNIEXPORT jint JFN(rowOfIdent)(JNIEnv* env, jclass cls, jlong ctx, jlong ident) {
  (void)env;
  (void)cls;
  uint32_t row = 0;
  return dk_row_of_ident(CTX(ctx), (uint64_t)ident, &row) == DK_OK ? (jint)row : -1;
}

JNIEXPORT jlong JFN(match)(JNIEnv* env, jclass cls, jlong ctx, jintArray rows) {
  (void)cls;
  const jsize n = (*env)->GetArrayLength(env, rows);
  jint* q = (*env)->GetIntArrayElements(env, rows, NULL);
  dk_result* res = NULL;
  const int rc = dk_match(CTX(ctx), (const uint32_t*)q, (uint64_t)n, DK_MATCH_HOST, &res);
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
  return rows_array(env, r->candidate, r->n);
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
  throw_dk(env, dk_compare_rows(CTX(ctx), (uint32_t)r1, (uint32_t)r2, &p));
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
  const int rc = dk_compare_values(CTX(ctx), &pair, &prob);
  for (jsize p = 0; p < np; ++p) free(units[p]);
  throw_dk(env, rc);
  return prob;
}

JNIEXPORT void JFN(setProfiling)(JNIEnv* env, jclass cls, jlong ctx, jboolean on) {
  (void)cls;
  throw_dk(env, dk_set_profiling(CTX(ctx), on ? 1 : 0));
}

JNIEXPORT void JFN(setResultRegion)(JNIEnv* env, jclass cls, jlong ctx, jobject region, jlong maxQueries) {
  (void)cls;
  void* base = region ? (*env)->GetDirectBufferAddress(env, region) : NULL;
  const jlong bytes = region ? (*env)->GetDirectBufferCapacity(env, region) : 0;
  throw_dk(env, dk_set_result_region(CTX(ctx), base, (uint64_t)bytes, (uint64_t)maxQueries));
}

/* ---- record-ID interner ----------------------------------------------------------------- */

JNIEXPORT jlong JFN(internerCreate)(JNIEnv* env, jclass cls) {
  (void)cls;
  dk_interner* ids = NULL;
  if (throw_dk(env, dk_interner_create(&ids))) return 0;
  return (jlong)(intptr_t)ids;
}

JNIEXPORT void JFN(internerDestroy)(JNIEnv* env, jclass cls, jlong ids) {
  (void)env;
  (void)cls;
  dk_interner_destroy((dk_interner*)(intptr_t)ids);
}

JNIEXPORT jlongArray JFN(internerIntern)(JNIEnv* env, jclass cls, jlong ids, jintArray offsets, jcharArray units) {
  (void)cls;
  const jsize n = (*env)->GetArrayLength(env, offsets) - 1;
  if (n < 0) {
    throw_msg(env, "offsets must hold n + 1 entries");
    return NULL;
  }
  Pinned P;
  dk_column col = pin_column(env, offsets, units, NULL, &P);
  uint64_t* out = (uint64_t*)malloc((size_t)n * 8 + 8);
  const int rc = dk_interner_intern((dk_interner*)(intptr_t)ids, &col, (uint64_t)n, out);
  unpin_column(env, &P);
  jlongArray res = NULL;
  if (!throw_dk(env, rc)) {
    res = (*env)->NewLongArray(env, n);
    if (n) (*env)->SetLongArrayRegion(env, res, 0, n, (const jlong*)out);
  }
  free(out);
  return res;
}

JNIEXPORT jlong JFN(internerFind)(JNIEnv* env, jclass cls, jlong ids, jstring id) {
  (void)cls;
  const jsize n = (*env)->GetStringLength(env, id);
  const jchar* u = (*env)->GetStringChars(env, id, NULL);
  uint64_t v = 0;
  const int rc = dk_interner_find((const dk_interner*)(intptr_t)ids, (const uint16_t*)u, (uint64_t)n, &v);
  (*env)->ReleaseStringChars(env, id, u);
  return rc == DK_OK ? (jlong)v : -1;
}

static jstring units_string(JNIEnv* env, const void* units, int width, uint64_t a, uint64_t n) {
  if (width == 2) return (*env)->NewString(env, (const jchar*)units + a, (jsize)n);
  jchar* w = (jchar*)malloc(n * sizeof(jchar) + 2);
  for (uint64_t i = 0; i < n; ++i) w[i] = ((const uint8_t*)units)[a + i];
  jstring s = (*env)->NewString(env, w, (jsize)n);
  free(w);
  return s;
}

JNIEXPORT jstring JFN(internerString)(JNIEnv* env, jclass cls, jlong ids, jlong id) {
  (void)cls;
  const uint16_t* u = NULL;
  uint64_t n = 0;
  if (throw_dk(env, dk_interner_string((const dk_interner*)(intptr_t)ids, (uint64_t)id, &u, &n))) return NULL;
  return units_string(env, u, 2, 0, n);
}

/* ---- native ingestion --------------------------------------------------------------------- */

JNIEXPORT jlong JFN(packJson)(JNIEnv* env, jclass cls, jlong ids, jbyteArray body, jstring datasetId,
                              jint groupNo, jobjectArray columnNames, jintArray columnProp,
                              jintArray columnCleaner, jint nprops, jobjectArray keyParts) {
  (void)cls;
  const jsize nc = (*env)->GetArrayLength(env, columnNames);
  const jsize nk = keyParts ? (*env)->GetArrayLength(env, keyParts) : 0;
  if (nk > 8) {
    throw_msg(env, "more than 8 key functions");
    return 0;
  }
  dk_source_column* cols = (dk_source_column*)calloc((size_t)nc + 1, sizeof(dk_source_column));
  jstring* jnames = (jstring*)calloc((size_t)nc + 1, sizeof(jstring));
  jint* prop = (*env)->GetIntArrayElements(env, columnProp, NULL);
  jint* clean = (*env)->GetIntArrayElements(env, columnCleaner, NULL);
  for (jsize i = 0; i < nc; ++i) {
    jnames[i] = (jstring)(*env)->GetObjectArrayElement(env, columnNames, i);
    cols[i].name = (*env)->GetStringUTFChars(env, jnames[i], NULL);  /* the attribute as given */
    cols[i].prop = prop[i];
    cols[i].cleaner = clean[i];
  }
  dk_key_function kf[8];
  dk_key_part* parts[8];
  for (jsize k = 0; k < nk; ++k) {
    jintArray jp = (jintArray)(*env)->GetObjectArrayElement(env, keyParts, k);
    const jsize m = (*env)->GetArrayLength(env, jp) / 4;
    parts[k] = (dk_key_part*)malloc((size_t)m * sizeof(dk_key_part) + sizeof(dk_key_part));
    (*env)->GetIntArrayRegion(env, jp, 0, m * 4, (jint*)parts[k]);  /* (prop, token, start, end)* */
    kf[k].nparts = (int32_t)m;
    kf[k].parts = parts[k];
  }
  const char* ds = (*env)->GetStringUTFChars(env, datasetId, NULL);
  dk_source src;
  memset(&src, 0, sizeof src);
  src.dataset_id = ds;
  src.group_no = groupNo;
  src.ncolumns = (int32_t)nc;
  src.columns = cols;
  src.nprops = nprops;
  src.nkeys = (int32_t)nk;
  src.keys = nk ? kf : NULL;
  const jsize len = (*env)->GetArrayLength(env, body);
  jbyte* json = (*env)->GetByteArrayElements(env, body, NULL);
  dk_packed* packed = NULL;
  const int rc = dk_pack_json(&src, (const char*)json, (uint64_t)len, (dk_interner*)(intptr_t)ids, &packed);
  (*env)->ReleaseByteArrayElements(env, body, json, JNI_ABORT);
  (*env)->ReleaseStringUTFChars(env, datasetId, ds);
  for (jsize i = 0; i < nc; ++i) (*env)->ReleaseStringUTFChars(env, jnames[i], cols[i].name);
  (*env)->ReleaseIntArrayElements(env, columnProp, prop, JNI_ABORT);
  (*env)->ReleaseIntArrayElements(env, columnCleaner, clean, JNI_ABORT);
  for (jsize k = 0; k < nk; ++k) free(parts[k]);
  free(cols);
  free(jnames);
  if (throw_dk(env, rc)) return 0;
  return (jlong)(intptr_t)packed;
}

#define PACKED(h) ((const dk_packed*)(intptr_t)(h))

JNIEXPORT jint JFN(packedSize)(JNIEnv* env, jclass cls, jlong packed) {
  (void)env;
  (void)cls;
  return (jint)PACKED(packed)->n;
}

JNIEXPORT jlongArray JFN(packedIdent)(JNIEnv* env, jclass cls, jlong packed) {
  (void)cls;
  const dk_packed* P = PACKED(packed);
  jlongArray out = (*env)->NewLongArray(env, (jsize)P->n);
  if (P->n) (*env)->SetLongArrayRegion(env, out, 0, (jsize)P->n, (const jlong*)P->ident);
  return out;
}

JNIEXPORT jbyteArray JFN(packedDeleted)(JNIEnv* env, jclass cls, jlong packed) {
  (void)cls;
  const dk_packed* P = PACKED(packed);
  jbyteArray out = (*env)->NewByteArray(env, (jsize)P->n);
  if (P->n && P->deleted) (*env)->SetByteArrayRegion(env, out, 0, (jsize)P->n, (const jbyte*)P->deleted);
  return out;
}

static jobjectArray column_strings(JNIEnv* env, const dk_column* c, uint64_t n) {
  jobjectArray out = (*env)->NewObjectArray(env, (jsize)n, (*env)->FindClass(env, "java/lang/String"), NULL);
  for (uint64_t i = 0; i < n && out; ++i) {
    if (c->present && !c->present[i]) continue;  /* no value: null */
    jstring s = units_string(env, c->units, c->width, c->offsets[i], c->offsets[i + 1] - c->offsets[i]);
    (*env)->SetObjectArrayElement(env, out, (jsize)i, s);
    (*env)->DeleteLocalRef(env, s);
  }
  return out;
}

JNIEXPORT jobjectArray JFN(packedValues)(JNIEnv* env, jclass cls, jlong packed, jint p) {
  (void)cls;
  return column_strings(env, &PACKED(packed)->columns[p], PACKED(packed)->n);
}

JNIEXPORT jobjectArray JFN(packedIds)(JNIEnv* env, jclass cls, jlong packed) {
  (void)cls;
  return column_strings(env, &PACKED(packed)->id, PACKED(packed)->n);
}

JNIEXPORT jobjectArray JFN(packedEntityIds)(JNIEnv* env, jclass cls, jlong packed) {
  (void)cls;
  return column_strings(env, &PACKED(packed)->entity_id, PACKED(packed)->n);
}

JNIEXPORT jintArray JFN(upsertPacked)(JNIEnv* env, jclass cls, jlong ctx, jlong packed, jboolean transient_) {
  (void)cls;
  const dk_packed* P = PACKED(packed);
  dk_batch b;
  memset(&b, 0, sizeof b);
  b.n = P->n;
  b.ident = P->ident;
  b.group = P->group;
  b.deleted = P->deleted;
  b.columns = P->columns;
  b.key_columns = P->key_columns;
  uint32_t* rows = (uint32_t*)malloc(P->n * 4 + 4);
  const int rc = transient_ ? dk_upsert_transient(CTX(ctx), &b, rows) : dk_upsert(CTX(ctx), &b, rows);
  jintArray out = NULL;
  if (!throw_dk(env, rc)) out = rows_array(env, rows, P->n);
  free(rows);
  return out;
}

JNIEXPORT void JFN(freePacked)(JNIEnv* env, jclass cls, jlong packed) {
  (void)env;
  (void)cls;
  dk_free_packed((dk_packed*)(intptr_t)packed);
}

/* ---- link sink ------------------------------------------------------------------------- */

JNIEXPORT jlong JFN(linkdbCreate)(JNIEnv* env, jclass cls, jlong ids) {
  (void)cls;
  dk_linkdb* db = NULL;
  if (throw_dk(env, dk_linkdb_create((const dk_interner*)(intptr_t)ids, &db))) return 0;
  return (jlong)(intptr_t)db;
}

JNIEXPORT void JFN(linkdbDestroy)(JNIEnv* env, jclass cls, jlong db) {
  (void)env;
  (void)cls;
  dk_linkdb_destroy((dk_linkdb*)(intptr_t)db);
}

JNIEXPORT jlongArray JFN(linkdbApply)(JNIEnv* env, jclass cls, jlong db, jlongArray queryIdent,
                                      jlongArray first, jlongArray candidateIdent, jdoubleArray prob,
                                      jbyteArray kind, jlong timestamp) {
  (void)cls;
  /* the C-ABI trusts these sizes: first[] holds nqueries + 1 non-decreasing offsets into the
   * candidate arrays, which all have one length */
  const jsize nq = (*env)->GetArrayLength(env, queryIdent);
  const jsize nc = (*env)->GetArrayLength(env, candidateIdent);
  if ((*env)->GetArrayLength(env, first) != nq + 1 || (*env)->GetArrayLength(env, prob) != nc ||
      (*env)->GetArrayLength(env, kind) != nc) {
    throw_msg(env, "linkdbApply: first must hold queryIdent.length + 1 entries and prob / kind "
                   "candidateIdent.length");
    return NULL;
  }
  {
    jlong f0 = 0, fl = 0;
    (*env)->GetLongArrayRegion(env, first, 0, 1, &f0);
    (*env)->GetLongArrayRegion(env, first, nq, 1, &fl);
    if (f0 != 0 || fl < 0 || fl > (jlong)nc) {
      throw_msg(env, "linkdbApply: first[0] must be 0 and first[queryIdent.length] at most "
                     "candidateIdent.length");
      return NULL;
    }
  }
  jlong* qi = (*env)->GetLongArrayElements(env, queryIdent, NULL);
  jlong* fi = (*env)->GetLongArrayElements(env, first, NULL);
  jlong* ci = (*env)->GetLongArrayElements(env, candidateIdent, NULL);
  jdouble* pr = (*env)->GetDoubleArrayElements(env, prob, NULL);
  jbyte* kd = (*env)->GetByteArrayElements(env, kind, NULL);
  dk_link_batch b;
  b.nqueries = (uint64_t)nq;
  b.query_ident = (const uint64_t*)qi;
  b.first = (const uint64_t*)fi;
  b.candidate_ident = (const uint64_t*)ci;
  b.prob = pr;
  b.kind = (const uint8_t*)kd;
  dk_link_stats st;
  memset(&st, 0, sizeof st);
  const int rc = dk_linkdb_apply((dk_linkdb*)(intptr_t)db, &b, (int64_t)timestamp, &st);
  (*env)->ReleaseLongArrayElements(env, queryIdent, qi, JNI_ABORT);
  (*env)->ReleaseLongArrayElements(env, first, fi, JNI_ABORT);
  (*env)->ReleaseLongArrayElements(env, candidateIdent, ci, JNI_ABORT);
  (*env)->ReleaseDoubleArrayElements(env, prob, pr, JNI_ABORT);
  (*env)->ReleaseByteArrayElements(env, kind, kd, JNI_ABORT);
  if (throw_dk(env, rc)) return NULL;
  const jlong s3[3] = {(jlong)st.asserted, (jlong)st.unchanged, (jlong)st.retracted};
  jlongArray out = (*env)->NewLongArray(env, 3);
  (*env)->SetLongArrayRegion(env, out, 0, 3, s3);
  return out;
}

JNIEXPORT jlong JFN(linkdbChangesSince)(JNIEnv* env, jclass cls, jlong db, jlong since) {
  (void)cls;
  dk_link_list* l = NULL;
  if (throw_dk(env, dk_linkdb_changes_since((const dk_linkdb*)(intptr_t)db, (int64_t)since, &l))) return 0;
  return (jlong)(intptr_t)l;
}

JNIEXPORT jlong JFN(linkdbLinksFor)(JNIEnv* env, jclass cls, jlong db, jlong ident) {
  (void)cls;
  dk_link_list* l = NULL;
  if (throw_dk(env, dk_linkdb_links_for((const dk_linkdb*)(intptr_t)db, (uint64_t)ident, &l))) return 0;
  return (jlong)(intptr_t)l;
}

JNIEXPORT jlong JFN(linkdbRetract)(JNIEnv* env, jclass cls, jlong db, jlong ident, jlong other, jlong timestamp) {
  (void)cls;
  uint64_t n = 0;
  throw_dk(env, dk_linkdb_retract((dk_linkdb*)(intptr_t)db, (uint64_t)ident, other < 0 ? UINT64_MAX : (uint64_t)other,
                                  (int64_t)timestamp, &n));
  return (jlong)n;
}

#define LIST(h) ((const dk_link_list*)(intptr_t)(h))

JNIEXPORT jlongArray JFN(linkListId1)(JNIEnv* env, jclass cls, jlong list) {
  (void)cls;
  jlongArray out = (*env)->NewLongArray(env, (jsize)LIST(list)->n);
  if (LIST(list)->n) (*env)->SetLongArrayRegion(env, out, 0, (jsize)LIST(list)->n, (const jlong*)LIST(list)->id1);
  return out;
}

JNIEXPORT jlongArray JFN(linkListId2)(JNIEnv* env, jclass cls, jlong list) {
  (void)cls;
  jlongArray out = (*env)->NewLongArray(env, (jsize)LIST(list)->n);
  if (LIST(list)->n) (*env)->SetLongArrayRegion(env, out, 0, (jsize)LIST(list)->n, (const jlong*)LIST(list)->id2);
  return out;
}

JNIEXPORT jbyteArray JFN(linkListStatus)(JNIEnv* env, jclass cls, jlong list) {
  (void)cls;
  jbyteArray out = (*env)->NewByteArray(env, (jsize)LIST(list)->n);
  if (LIST(list)->n) (*env)->SetByteArrayRegion(env, out, 0, (jsize)LIST(list)->n, (const jbyte*)LIST(list)->status);
  return out;
}

JNIEXPORT jbyteArray JFN(linkListKind)(JNIEnv* env, jclass cls, jlong list) {
  (void)cls;
  jbyteArray out = (*env)->NewByteArray(env, (jsize)LIST(list)->n);
  if (LIST(list)->n) (*env)->SetByteArrayRegion(env, out, 0, (jsize)LIST(list)->n, (const jbyte*)LIST(list)->kind);
  return out;
}

JNIEXPORT jdoubleArray JFN(linkListConfidence)(JNIEnv* env, jclass cls, jlong list) {
  (void)cls;
  jdoubleArray out = (*env)->NewDoubleArray(env, (jsize)LIST(list)->n);
  if (LIST(list)->n) (*env)->SetDoubleArrayRegion(env, out, 0, (jsize)LIST(list)->n, LIST(list)->confidence);
  return out;
}

JNIEXPORT jlongArray JFN(linkListTimestamp)(JNIEnv* env, jclass cls, jlong list) {
  (void)cls;
  jlongArray out = (*env)->NewLongArray(env, (jsize)LIST(list)->n);
  if (LIST(list)->n)
    (*env)->SetLongArrayRegion(env, out, 0, (jsize)LIST(list)->n, (const jlong*)LIST(list)->timestamp);
  return out;
}

JNIEXPORT void JFN(freeLinkList)(JNIEnv* env, jclass cls, jlong list) {
  (void)env;
  (void)cls;
  dk_free_link_list((dk_link_list*)(intptr_t)list);
}
