/*
 * JNI shim: org.apache.mahout.cf.taste.impl.similarity.CosineCMGpu -> the C
 * ABI of libmahout_cms.so (include/mahout_cms.h).
 *
 * Built only where a JDK provides jni.h (not in this image):
 *   cc -O2 -fPIC -shared -I$JAVA_HOME/include -I$JAVA_HOME/include/linux \
 *      -I../../include mahout_cms_jni.c -L../../mahout_amd -lmahout_cms \
 *      -Wl,-rpath,'$ORIGIN' -o libmahout_cms_jni.so
 *
 * Status codes map to the reference's exceptions: CMS_E_NO_SUCH_ID ->
 * NoSuchUserException / NoSuchItemException (GenericDataModel.java:210-215),
 * CMS_E_PARAM / CMS_E_SHAPE -> IllegalArgumentException
 * (AbstractCountMinSketch CMException / DoubleCountMinSketch checkArgument),
 * anything else -> TasteException.  NaN similarities are values, not errors.
 * The DataModel arrays are copied out with Get*ArrayRegion before the library
 * call (no critical region spans GPU work); small query arrays are pinned
 * only around a host-side copy.  The library never retains host pointers.
 * frac_bits < 0 from the Java side selects fp64 counters (CMS_COUNTER_F64).
 */
#include <jni.h>
#include <stdint.h>
#include <stdlib.h>

#include "mahout_cms.h"

#define CLS "org/apache/mahout/cf/taste/"

static void throw_named(JNIEnv* env, const char* cls, const char* msg) {
  jclass ex = (*env)->FindClass(env, cls);
  if (ex) (*env)->ThrowNew(env, ex, msg);
}

static int fail(JNIEnv* env, int rc, int item_ids) {
  if (rc == CMS_OK) return 0;
  const char* cls = CLS "common/TasteException";
  if (rc == CMS_E_NO_SUCH_ID) cls = item_ids ? CLS "common/NoSuchItemException" : CLS "common/NoSuchUserException";
  else if (rc == CMS_E_PARAM || rc == CMS_E_SHAPE) cls = "java/lang/IllegalArgumentException";
  jclass ex = (*env)->FindClass(env, cls);
  if (ex) (*env)->ThrowNew(env, ex, cms_last_error());
  return 1;
}

/* The shim is compiled against one cms_stats / cms_params layout: refuse a
   libmahout_cms.so of another ABI (System.loadLibrary then throws
   UnsatisfiedLinkError) instead of reading its structs with the wrong shape. */
JNIEXPORT jint JNICALL JNI_OnLoad(JavaVM* vm, void* reserved) {
  (void)vm;
  (void)reserved;
  return cms_abi_version() == CMS_ABI_VERSION ? JNI_VERSION_1_6 : JNI_ERR;
}

#define H(x) ((cms_handle*)(intptr_t)(x))
#define JFN(name) Java_org_apache_mahout_cf_taste_impl_similarity_CosineCMGpu_##name

JNIEXPORT jlong JNICALL JFN(nativeCreate)(JNIEnv* env, jclass c, jint depth, jint width, jlong seed, jlong n,
                                          jboolean weighted, jint device, jint frac_bits) {
  (void)c;
  cms_params p;
  cms_params_init(&p);
  p.depth = depth;
  p.width = width;
  p.seed = seed;
  p.num_owners = n;
  p.weighting = weighted ? CMS_WEIGHTED : CMS_UNWEIGHTED;
  p.device = device;
  /* frac_bits < 0: the preferences need DoubleCountMinSketch's fp64 counters
     (negative, non-dyadic, or masses a u32 counter cannot hold) */
  p.counter_type = frac_bits < 0 ? CMS_COUNTER_F64 : CMS_COUNTER_U32;
  p.frac_bits = frac_bits < 0 ? 0 : frac_bits;
  cms_handle* h = NULL;
  if (fail(env, cms_create(&p, &h), 0)) return 0;
  return (jlong)(intptr_t)h;
}

JNIEXPORT jlong JNICALL JFN(nativeCreatePerOwner)(JNIEnv* env, jclass c, jlong seed, jlong n, jboolean weighted,
                                                  jint device, jint frac_bits) {
  (void)c;
  cms_params p;
  cms_params_init(&p);
  p.seed = seed;
  p.num_owners = n;
  p.weighting = weighted ? CMS_WEIGHTED : CMS_UNWEIGHTED;
  p.device = device;
  p.counter_type = frac_bits < 0 ? CMS_COUNTER_F64 : CMS_COUNTER_U32;
  p.frac_bits = frac_bits < 0 ? 0 : frac_bits;
  cms_handle* h = NULL;
  if (fail(env, cms_create_per_owner(&p, &h), 0)) return 0;
  return (jlong)(intptr_t)h;
}

JNIEXPORT void JNICALL JFN(nativeConfigureOwnerShapes)(JNIEnv* env, jclass c, jlong h, jdouble q, jlong num_keys) {
  (void)c;
  fail(env, cms_configure_owner_shapes(H(h), q, num_keys), 0);
}

JNIEXPORT void JNICALL JFN(nativeSetOwnerDeltaEpsilon)(JNIEnv* env, jclass c, jlong h, jdoubleArray delta,
                                                       jdoubleArray epsilon) {
  (void)c;
  jdouble* pd = (*env)->GetPrimitiveArrayCritical(env, delta, NULL);
  jdouble* pe = (*env)->GetPrimitiveArrayCritical(env, epsilon, NULL);
  int rc = cms_set_owner_delta_epsilon(H(h), (const double*)pd, (const double*)pe);
  (*env)->ReleasePrimitiveArrayCritical(env, epsilon, pe, JNI_ABORT);
  (*env)->ReleasePrimitiveArrayCritical(env, delta, pd, JNI_ABORT);
  fail(env, rc, 0);
}

JNIEXPORT void JNICALL JFN(nativeSetOwnerIds)(JNIEnv* env, jclass c, jlong h, jlongArray ids) {
  (void)c;
  jsize n = (*env)->GetArrayLength(env, ids);
  jlong* p = (*env)->GetPrimitiveArrayCritical(env, ids, NULL);
  int rc = cms_set_owner_ids(H(h), (const int64_t*)p, n);
  (*env)->ReleasePrimitiveArrayCritical(env, ids, p, JNI_ABORT);
  fail(env, rc, 0);
}

/* The arrays are copied out with Get*ArrayRegion before the library call (which
   takes the handle's mutex and runs kernels): no critical region, and so no GC
   stall, spans GPU work.  offsets must hold num_owners + 1 entries and
   offsets[num_owners] must not run past the keys (or the values). */
JNIEXPORT void JNICALL JFN(nativeIngestCsr)(JNIEnv* env, jclass c, jlong h, jlongArray off, jlongArray keys,
                                            jfloatArray vals) {
  (void)c;
  if (!off || !keys) {
    throw_named(env, "java/lang/IllegalArgumentException", "null offsets or keys");
    return;
  }
  cms_stats st;
  st.struct_size = (uint32_t)sizeof st;
  if (fail(env, cms_get_stats(H(h), &st), 0)) return;
  const jsize no = (*env)->GetArrayLength(env, off);
  const jsize nk = (*env)->GetArrayLength(env, keys);
  if ((int64_t)no != st.num_owners + 1) {
    throw_named(env, "java/lang/IllegalArgumentException", "offsets must hold num_owners + 1 entries");
    return;
  }
  int64_t* po = (int64_t*)malloc(sizeof(int64_t) * (size_t)no);
  int64_t* pk = (int64_t*)malloc(sizeof(int64_t) * (size_t)(nk ? nk : 1));
  float* pv = vals ? (float*)malloc(sizeof(float) * (size_t)(nk ? nk : 1)) : NULL;
  if (!po || !pk || (vals && !pv)) {
    free(po);
    free(pk);
    free(pv);
    throw_named(env, "java/lang/OutOfMemoryError", "host staging for the DataModel");
    return;
  }
  (*env)->GetLongArrayRegion(env, off, 0, no, (jlong*)po);
  (*env)->GetLongArrayRegion(env, keys, 0, nk, (jlong*)pk);
  const char* bad = NULL;
  if (po[no - 1] > (int64_t)nk) bad = "offsets[num_owners] runs past the keys";
  if (vals && !bad) {
    if ((*env)->GetArrayLength(env, vals) < nk) bad = "fewer values than keys";
    else (*env)->GetFloatArrayRegion(env, vals, 0, nk, pv);
  }
  int rc = bad ? CMS_OK : cms_ingest_csr(H(h), po, pk, pv);
  free(po);
  free(pk);
  free(pv);
  if (bad) throw_named(env, "java/lang/IllegalArgumentException", bad);
  else fail(env, rc, 0);
}

JNIEXPORT void JNICALL JFN(nativeFinalize)(JNIEnv* env, jclass c, jlong h) {
  (void)c;
  fail(env, cms_finalize(H(h)), 0);
}

JNIEXPORT jdouble JNICALL JFN(nativeSimilarity)(JNIEnv* env, jclass c, jlong h, jlong a, jlong b, jboolean items) {
  (void)c;
  double out = 0.0;
  fail(env, cms_similarity(H(h), a, b, &out), items);
  return out;
}

JNIEXPORT jdoubleArray JNICALL JFN(nativeSimilarities)(JNIEnv* env, jclass c, jlong h, jlong a, jlongArray ids) {
  (void)c;
  jsize n = (*env)->GetArrayLength(env, ids);
  jdoubleArray res = (*env)->NewDoubleArray(env, n);
  if (!res) return NULL;
  int64_t* tmp_ids = (int64_t*)malloc(sizeof(int64_t) * (n ? n : 1));
  double* tmp_out = (double*)malloc(sizeof(double) * (n ? n : 1));
  (*env)->GetLongArrayRegion(env, ids, 0, n, (jlong*)tmp_ids);
  int rc = cms_similarities(H(h), a, tmp_ids, n, tmp_out);
  if (rc == CMS_OK) (*env)->SetDoubleArrayRegion(env, res, 0, n, tmp_out);
  free(tmp_ids);
  free(tmp_out);
  return fail(env, rc, 1) ? NULL : res;
}

JNIEXPORT jlongArray JNICALL JFN(nativeMostSimilar)(JNIEnv* env, jclass c, jlong h, jlong id, jint k) {
  (void)c;
  int64_t* ids = (int64_t*)malloc(sizeof(int64_t) * (k > 0 ? k : 1));
  double* sc = (double*)malloc(sizeof(double) * (k > 0 ? k : 1));
  int32_t cnt = 0;
  int rc = cms_most_similar(H(h), id, k, ids, sc, &cnt);
  jlongArray res = NULL;
  if (rc == CMS_OK) {
    res = (*env)->NewLongArray(env, cnt);
    if (res) (*env)->SetLongArrayRegion(env, res, 0, cnt, (const jlong*)ids);
  }
  free(ids);
  free(sc);
  return fail(env, rc, 0) ? NULL : res;
}

JNIEXPORT jdouble JNICALL JFN(nativePointQuery)(JNIEnv* env, jclass c, jlong h, jlong id, jlong key) {
  (void)c;
  double out = 0.0;
  fail(env, cms_point_query(H(h), id, key, &out), 0);
  return out;
}

JNIEXPORT jfloatArray JNICALL JFN(nativeEstimatePreferences)(JNIEnv* env, jclass c, jlong h, jlong user,
                                                               jlongArray nbs, jlongArray items, jfloat cap_min,
                                                               jfloat cap_max) {
  (void)c;
  jsize m = (*env)->GetArrayLength(env, nbs);
  jsize q = (*env)->GetArrayLength(env, items);
  int64_t* nb = (int64_t*)malloc(sizeof(int64_t) * (m ? m : 1));
  int64_t* it = (int64_t*)malloc(sizeof(int64_t) * (q ? q : 1));
  float* out = (float*)malloc(sizeof(float) * (q ? q : 1));
  (*env)->GetLongArrayRegion(env, nbs, 0, m, (jlong*)nb);
  (*env)->GetLongArrayRegion(env, items, 0, q, (jlong*)it);
  const int use_capper = !(cap_min != cap_min && cap_max != cap_max);  /* both NaN: no capper (:209-216) */
  int rc = cms_estimate_preferences(H(h), user, nb, m, it, q, use_capper, cap_min, cap_max, out);
  jfloatArray res = NULL;
  if (rc == CMS_OK) {
    res = (*env)->NewFloatArray(env, q);
    if (res) (*env)->SetFloatArrayRegion(env, res, 0, q, out);
  }
  free(nb);
  free(it);
  free(out);
  return fail(env, rc, 0) ? NULL : res;
}

/* GenericUserBasedRecommender.recommend for many users (cms_recommend_batch);
 * the outputs are Java arrays the caller sized: counts[n], items/values
 * [n * howMany]. */
static int64_t* longs_of(JNIEnv* env, jlongArray a, jsize* len) {
  *len = a ? (*env)->GetArrayLength(env, a) : 0;
  int64_t* p = (int64_t*)malloc(sizeof(int64_t) * (size_t)(*len ? *len : 1));
  if (p && *len) (*env)->GetLongArrayRegion(env, a, 0, *len, (jlong*)p);
  return p;
}

JNIEXPORT void JNICALL JFN(nativeRecommendBatch)(JNIEnv* env, jclass c, jlong h, jlongArray users, jlongArray nbo,
                                                 jlongArray nbs, jlongArray mids, jlongArray po, jlongArray pi,
                                                 jint how_many, jboolean include_known, jfloat cap_min,
                                                 jfloat cap_max, jintArray out_counts, jlongArray out_items,
                                                 jfloatArray out_values) {
  (void)c;
  jsize n, n_nbo, n_nb, n_m, n_po, n_pi;
  int64_t* u = longs_of(env, users, &n);
  int64_t* o = longs_of(env, nbo, &n_nbo);
  int64_t* nb = longs_of(env, nbs, &n_nb);
  int64_t* m = longs_of(env, mids, &n_m);
  int64_t* p_off = longs_of(env, po, &n_po);
  int64_t* p_it = longs_of(env, pi, &n_pi);
  const size_t outn = (size_t)n * (size_t)(how_many > 0 ? how_many : 1);
  int32_t* cnt = (int32_t*)malloc(sizeof(int32_t) * (size_t)(n ? n : 1));
  int64_t* it = (int64_t*)malloc(sizeof(int64_t) * (outn ? outn : 1));
  float* val = (float*)malloc(sizeof(float) * (outn ? outn : 1));
  int rc = CMS_E_OOM;
  /* the offsets must describe exactly the arrays handed over */
  if (u && o && nb && m && p_off && p_it && cnt && it && val) {
    rc = (n_nbo != n + 1 || o[0] != 0 || o[n] != n_nb || n_po != n_m + 1 || p_off[0] != 0 || p_off[n_m] != n_pi)
             ? CMS_E_PARAM
             : cms_recommend_batch(H(h), n, u, o, nb, n_m, m, p_off, p_it, how_many, include_known,
                                   !(cap_min != cap_min && cap_max != cap_max), cap_min, cap_max, cnt, it, val);
  }
  if (rc == CMS_OK) {
    (*env)->SetIntArrayRegion(env, out_counts, 0, n, (const jint*)cnt);
    (*env)->SetLongArrayRegion(env, out_items, 0, (jsize)outn, (const jlong*)it);
    (*env)->SetFloatArrayRegion(env, out_values, 0, (jsize)outn, val);
  }
  free(u);
  free(o);
  free(nb);
  free(m);
  free(p_off);
  free(p_it);
  free(cnt);
  free(it);
  free(val);
  fail(env, rc, 0);
}

typedef int (*top_k_fn)(cms_handle*, int32_t, int64_t*, double*, int32_t*);

static jobjectArray top_k_lists(JNIEnv* env, jlong h, jint k, top_k_fn fn) {
  cms_stats st;
  st.struct_size = (uint32_t)sizeof st;
  st.pairs_ingested = 0;
  if (fail(env, cms_get_stats(H(h), &st), 0)) return NULL;
  const int64_t n = st.num_owners;
  int64_t* ids = (int64_t*)malloc(sizeof(int64_t) * (size_t)n * (k > 0 ? k : 1));
  int32_t* cnt = (int32_t*)malloc(sizeof(int32_t) * (size_t)(n ? n : 1));
  int rc = fn(H(h), k, ids, NULL, cnt);
  jobjectArray res = NULL;
  if (rc == CMS_OK) {
    jclass longArr = (*env)->FindClass(env, "[J");
    res = longArr ? (*env)->NewObjectArray(env, (jsize)n, longArr, NULL) : NULL;
    for (int64_t r = 0; res && r < n; ++r) {
      jlongArray row = (*env)->NewLongArray(env, cnt[r]);
      if (!row) { res = NULL; break; }
      (*env)->SetLongArrayRegion(env, row, 0, cnt[r], (const jlong*)(ids + r * k));
      (*env)->SetObjectArrayElement(env, res, (jsize)r, row);
      (*env)->DeleteLocalRef(env, row);
    }
  }
  free(ids);
  free(cnt);
  return fail(env, rc, 0) ? NULL : res;
}

JNIEXPORT jobjectArray JNICALL JFN(nativeTopKAll)(JNIEnv* env, jclass c, jlong h, jint k) {
  (void)c;
  return top_k_lists(env, h, k, cms_top_k_all);
}

/* The periodic refresh of a streaming table (cms_top_k_refresh): the same
 * lists, recomputing only the pairs of owners touched since the last call. */
JNIEXPORT jobjectArray JNICALL JFN(nativeTopKRefresh)(JNIEnv* env, jclass c, jlong h, jint k) {
  (void)c;
  return top_k_lists(env, h, k, cms_top_k_refresh);
}

/* HashFunctionBuilder's drawn parameters (HashFunctionParams.draw) installed
   before the first ingest: the GPU hashes with the caller's own builder. */
JNIEXPORT void JNICALL JFN(nativeSetHashParams)(JNIEnv* env, jclass c, jlong h, jlongArray a, jlongArray b) {
  (void)c;
  const jsize n = (*env)->GetArrayLength(env, a);
  if ((*env)->GetArrayLength(env, b) != n) {
    throw_named(env, "java/lang/IllegalArgumentException", "a and b differ in length");
    return;
  }
  int64_t* pa = (int64_t*)malloc(sizeof(int64_t) * (size_t)(n > 0 ? n : 1));
  int64_t* pb = (int64_t*)malloc(sizeof(int64_t) * (size_t)(n > 0 ? n : 1));
  if (!pa || !pb) {
    free(pa);
    free(pb);
    throw_named(env, "java/lang/OutOfMemoryError", "hash parameters");
    return;
  }
  (*env)->GetLongArrayRegion(env, a, 0, n, (jlong*)pa);
  (*env)->GetLongArrayRegion(env, b, 0, n, (jlong*)pb);
  int rc = cms_set_hash_params(H(h), pa, pb, (int32_t)n);
  free(pa);
  free(pb);
  fail(env, rc, 0);
}

/* {width, depth} of an owner's own sketch (per-owner handle; cms_read_owner_sketch
   with out = NULL): the shape new DoubleCountMinSketch(delta, epsilon, ...) gives it. */
JNIEXPORT jintArray JNICALL JFN(nativeOwnerShape)(JNIEnv* env, jclass c, jlong h, jlong id) {
  (void)c;
  int32_t w = 0, d = 0;
  if (fail(env, cms_read_owner_sketch(H(h), id, NULL, 0, &w, &d), 0)) return NULL;
  jintArray out = (*env)->NewIntArray(env, 2);
  if (!out) return NULL;
  jint v[2] = {w, d};
  (*env)->SetIntArrayRegion(env, out, 0, 2, v);
  return out;
}

/* getExportedCMProfile(id)'s counters, [depth][width] row-major as
   DoubleCountMinSketch.count holds them (DoubleCountMinSketch.java:62-64). */
JNIEXPORT jdoubleArray JNICALL JFN(nativeReadOwnerSketch)(JNIEnv* env, jclass c, jlong h, jlong id) {
  (void)c;
  int32_t w = 0, d = 0;
  if (fail(env, cms_read_owner_sketch(H(h), id, NULL, 0, &w, &d), 0)) return NULL;
  const int64_t cells = (int64_t)w * d;
  double* buf = (double*)malloc(sizeof(double) * (size_t)(cells > 0 ? cells : 1));
  if (!buf) {
    throw_named(env, "java/lang/OutOfMemoryError", "owner sketch");
    return NULL;
  }
  int rc = cms_read_owner_sketch(H(h), id, buf, cells, &w, &d);
  if (fail(env, rc, 0)) {
    free(buf);
    return NULL;
  }
  jdoubleArray out = (*env)->NewDoubleArray(env, (jsize)cells);
  if (out) (*env)->SetDoubleArrayRegion(env, out, 0, (jsize)cells, buf);
  free(buf);
  return out;
}

JNIEXPORT void JNICALL JFN(nativeDestroy)(JNIEnv* env, jclass c, jlong h) {
  (void)env;
  (void)c;
  cms_destroy(H(h));
}
