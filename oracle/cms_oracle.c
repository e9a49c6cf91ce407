/*
 * cms_oracle.c -- CPU restatement of the reference CosineCM / DoubleCountMinSketch
 * path.  TEST INFRASTRUCTURE ONLY (see cms_oracle.h): the checker, never the
 * thing measured or shipped.  Compile with -ffp-contract=off: the reference's
 * fp64 sums are plain multiply-then-add (no FMA contraction in Java).
 *
 * "T/" = /root/reference/mr/src/main/java/org/apache/mahout/cf/taste/
 */
#define _GNU_SOURCE 1 /* qsort_r */
#include "cms_oracle.h"

#include <float.h>
#include <math.h>
#include <stdlib.h>
#include <string.h>

/* ------------------------------------------------------------------------ */
/* java.util.Random: 48-bit LCG, multiplier 0x5DEECE66D, addend 0xB.          */
/* Restated from the JDK's published algorithm (third-party, not under        */
/* /root/reference; used at T/impl/common/HashFunctionBuilder.java:27,46-47). */
/* ------------------------------------------------------------------------ */
#define JR_MULT 0x5DEECE66DULL
#define JR_ADD 0xBULL
#define JR_MASK ((1ULL << 48) - 1)

void orc_jrandom_init(orc_jrandom* r, int64_t seed) {
  r->seed = ((uint64_t)seed ^ JR_MULT) & JR_MASK; /* initialScramble */
}

static int32_t jr_next(orc_jrandom* r, int bits) {
  r->seed = (r->seed * JR_MULT + JR_ADD) & JR_MASK;
  return (int32_t)(uint32_t)(r->seed >> (48 - bits));
}

int32_t orc_jrandom_next_int(orc_jrandom* r) { return jr_next(r, 32); }

int64_t orc_jrandom_next_long(orc_jrandom* r) {
  /* ((long)next(32) << 32) + next(32); the second term is a sign-extended int */
  int64_t hi = (int64_t)jr_next(r, 32);
  int64_t lo = (int64_t)jr_next(r, 32);
  return (int64_t)((uint64_t)hi << 32) + lo;
}

/* Math.abs(long): Long.MIN_VALUE stays negative */
static int64_t java_abs_long(int64_t v) { return v < 0 ? (int64_t)(0 - (uint64_t)v) : v; }

/* HashFunctionBuilder(seed) + getHashFunction(i, w) for i = 0..d-1:
 * T/impl/common/HashFunctionBuilder.java:23-29 (Random(seed)), :42-56 (lazy
 * (a_i, b_i) = (abs(nextLong), abs(nextLong)) in row order).  The parameters
 * depend only on the row index (w enters at hash time, :93). */
void orc_hash_params(int64_t seed, int32_t depth, int64_t* a, int64_t* b) {
  orc_jrandom r;
  orc_jrandom_init(&r, seed);
  for (int32_t i = 0; i < depth; i++) {
    a[i] = java_abs_long(orc_jrandom_next_long(&r));
    b[i] = java_abs_long(orc_jrandom_next_long(&r));
  }
}

/* HashFunction.hash (T/impl/common/HashFunction.java:31-34):
 * a.multiply(k).add(b).mod(p).mod(w).intValue(), p = 2^63-25
 * (HashFunctionBuilder.java:24).  BigInteger.mod is non-negative. */
#define ORC_PRIME 9223372036854775783LL
int32_t orc_hash(int64_t a, int64_t b, int32_t width, int64_t key) {
  __int128 x = (__int128)a * (__int128)key + (__int128)b;
  __int128 r = x % (__int128)ORC_PRIME;
  if (r < 0) r += ORC_PRIME;
  return (int32_t)(r % (__int128)width);
}

void orc_hash_many(const int64_t* a, const int64_t* b, int32_t depth, int32_t width,
                   const int64_t* keys, int64_t n, int32_t* out) {
  for (int64_t i = 0; i < n; i++)
    for (int32_t r = 0; r < depth; r++) out[i * depth + r] = orc_hash(a[r], b[r], width, keys[i]);
}

/* AbstractCountMinSketch(delta, epsilon) (T/impl/common/AbstractCountMinSketch.java:69-83) */
int orc_shape_from_delta_epsilon(double delta, double epsilon, int32_t* width, int32_t* depth) {
  if (delta <= 0 || delta > exp(-1.0)) return -1;
  if (epsilon <= 0 || epsilon > exp(1.0)) return -1;
  *width = (int32_t)ceil(exp(1.0) / epsilon);
  *depth = (int32_t)ceil(log(1.0 / delta));
  return 0;
}

/* DoubleCountMinSketch.update (T/impl/common/DoubleCountMinSketch.java:72-80):
 * for i < d: j = h_i(key); count[j + i*w] += inc (inc = (double) float pref). */
void orc_sketch_build(double* table, int64_t rows, int32_t depth, int32_t width,
                      const int64_t* a, const int64_t* b,
                      const int64_t* owner_row, const int64_t* key, const float* val, int64_t n) {
  (void)rows;
  const int64_t stride = (int64_t)depth * width;
  for (int64_t t = 0; t < n; t++) {
    double inc = val ? (double)val[t] : 1.0;
    double* sk = table + owner_row[t] * stride;
    for (int32_t i = 0; i < depth; i++) {
      int32_t j = orc_hash(a[i], b[i], width, key[t]);
      double value = sk[j + (int64_t)i * width];
      sk[j + (int64_t)i * width] = value + inc;
    }
  }
}

/* DoubleCountMinSketch.get(long key) (:94-103): min over rows from Double.MAX_VALUE */
double orc_sketch_get(const double* sk, int32_t depth, int32_t width,
                      const int64_t* a, const int64_t* b, int64_t key) {
  double estimate = DBL_MAX;
  for (int32_t i = 0; i < depth; i++) {
    int32_t j = orc_hash(a[i], b[i], width, key);
    double value = sk[j + (int64_t)i * width];
    if (value < estimate) estimate = value;
  }
  return estimate;
}

/* java.lang.Math.min(double, double) */
static double java_min(double a, double b) {
  if (a != a) return a;
  if (a == 0.0 && b == 0.0 && signbit(b)) return b;
  return (a <= b) ? a : b;
}

/* DoubleCountMinSketch.cosine (:114-149) */
double orc_sketch_cosine(const double* sa, const double* sb, int32_t depth, int32_t width) {
  double minCosine = DBL_MAX;
  for (int32_t i = 0; i < depth; i++) {
    double valueA = 0.0, valueB = 0.0, valueAB = 0.0;
    const double* ra = sa + (int64_t)i * width;
    const double* rb = sb + (int64_t)i * width;
    for (int32_t j = 0; j < width; j++) {
      double xa = ra[j], xb = rb[j];
      valueA += xa * xa;
      valueB += xb * xb;
      valueAB += xa * xb;
    }
    double denominator = sqrt(valueA) * sqrt(valueB);
    if (denominator != 0) {
      double currentCosine = valueAB / denominator;
      minCosine = java_min(minCosine, currentCosine);
    }
  }
  if (minCosine == DBL_MAX) return NAN;
  return minCosine;
}

/* AbstractSimilarity.normalizeWeightResult (T/impl/similarity/AbstractSimilarity.java:313-330) */
double orc_normalize_weight_result(double result, int count, int num, int weighted) {
  double r = result;
  if (weighted) {
    double scaleFactor = 1.0 - (double)count / (double)(num + 1);
    if (r < 0.0) r = -1.0 + scaleFactor * (1.0 + r);
    else r = 1.0 - scaleFactor * (1.0 - r);
  }
  if (r < -1.0) r = -1.0;
  else if (r > 1.0) r = 1.0;
  return r;
}

/* CosineCM.userSimilarity (T/impl/similarity/CosineCM.java:83-96) */
double orc_cosine_cm(const double* sa, const double* sb, int32_t depth, int32_t width, int weighted) {
  double r = orc_sketch_cosine(sa, sb, depth, width);
  if (!isnan(r)) r = orc_normalize_weight_result(r, 1, 0, weighted);
  return r;
}

void orc_similarities_row(const double* table, int64_t rows, int32_t depth, int32_t width,
                          int64_t q, int weighted, double* out) {
  const int64_t stride = (int64_t)depth * width;
  for (int64_t j = 0; j < rows; j++) {
    if (j == q) { out[j] = NAN; continue; } /* MostSimilarEstimator self -> NaN */
    out[j] = orc_cosine_cm(table + q * stride, table + j * stride, depth, width, weighted);
  }
}

/* userSimilarity(q, p) (CosineCM.java:83-96) of Q query owners -- their
 * dense sketches qsk [Q][d][w], e.g. from orc_sketch_build -- against EVERY
 * owner p of a CSR (off[n + 1], keys, vals or NULL = 1.0), each p's sketch
 * rows taken from its own keys instead of a dense table (1M x d x w doubles
 * do not fit): in row i, B_j = sum of p's increments hashed to j, added in key
 * order as update (DoubleCountMinSketch.java:72-80) adds them, and cosine's
 * sums (:128-134) visit the buckets with B_j != 0 in ascending j.  The terms
 * skipped are products with xb = 0.0, and a partial sum that starts at +0.0
 * never becomes -0.0 (x + (-x) rounds to +0.0), so adding them back (x + 0.0
 * or x + -0.0) changes nothing: the result is orc_cosine_cm's on the dense
 * rows, bit for bit.  out[q * n + p]; OpenMP over the owners. */
void orc_cosine_queries_csr(const double* qsk, int64_t Q, const int64_t* off, const int64_t* keys, const float* vals,
                            int64_t n, int32_t depth, int32_t width, const int64_t* a, const int64_t* b,
                            int weighted, int32_t threads, double* out) {
  const int64_t dw = (int64_t)depth * width;
  const int32_t words = (width + 63) / 64;
  double* qa = (double*)malloc(sizeof(double) * (size_t)(Q * depth)); /* valueA of every query row */
  for (int64_t q = 0; q < Q; q++)
    for (int32_t i = 0; i < depth; i++) {
      double v = 0.0;
      const double* r = qsk + q * dw + (int64_t)i * width;
      for (int32_t j = 0; j < width; j++) v += r[j] * r[j];
      qa[q * depth + i] = v;
    }
#pragma omp parallel num_threads(threads > 0 ? threads : 1)
  {
    double* cnt = (double*)malloc(sizeof(double) * (size_t)width);
    uint64_t* bits = (uint64_t*)calloc((size_t)words, sizeof(uint64_t));
    double* ab = (double*)malloc(sizeof(double) * (size_t)Q);
    double* mins = (double*)malloc(sizeof(double) * (size_t)Q);
#pragma omp for schedule(dynamic, 64)
    for (int64_t p = 0; p < n; p++) {
      for (int64_t q = 0; q < Q; q++) mins[q] = DBL_MAX;
      for (int32_t i = 0; i < depth; i++) {
        for (int64_t t = off[p]; t < off[p + 1]; t++) {
          const double inc = vals ? (double)vals[t] : 1.0;
          const int32_t j = orc_hash(a[i], b[i], width, keys[t]);
          if (bits[j >> 6] >> (j & 63) & 1ULL) {
            cnt[j] = cnt[j] + inc;
          } else {
            bits[j >> 6] |= 1ULL << (j & 63);
            cnt[j] = 0.0 + inc;
          }
        }
        double vb = 0.0;
        for (int64_t q = 0; q < Q; q++) ab[q] = 0.0;
        for (int32_t wd = 0; wd < words; wd++) {
          uint64_t m = bits[wd];
          bits[wd] = 0;
          while (m) {
            const int32_t j = wd * 64 + __builtin_ctzll(m);
            m &= m - 1;
            const double xb = cnt[j];
            vb += xb * xb;
            for (int64_t q = 0; q < Q; q++) ab[q] += qsk[q * dw + (int64_t)i * width + j] * xb;
          }
        }
        for (int64_t q = 0; q < Q; q++) {
          const double den = sqrt(qa[q * depth + i]) * sqrt(vb);
          if (den != 0) mins[q] = java_min(mins[q], ab[q] / den);
        }
      }
      for (int64_t q = 0; q < Q; q++) {
        double r = mins[q] == DBL_MAX ? NAN : mins[q];
        if (!isnan(r)) r = orc_normalize_weight_result(r, 1, 0, weighted);
        out[q * n + p] = r;
      }
    }
    free(cnt);
    free(bits);
    free(ab);
    free(mins);
  }
  free(qa);
}

float orc_estimate_preference(const double* table, int32_t depth, int32_t width, const int64_t* a, const int64_t* b,
                              int64_t user_row, const int64_t* nb_rows, int64_t m, int64_t item_key, int weighted,
                              int use_capper, float cap_min, float cap_max) {
  const int64_t stride = (int64_t)depth * width;
  if (m == 0) return NAN;
  double preference = 0.0, total = 0.0;
  int count = 0;
  for (int64_t i = 0; i < m; i++) {
    const int64_t r = nb_rows[i];
    if (r == user_row) continue;
    const float pref = (float)orc_sketch_get(table + r * stride, depth, width, a, b, item_key);
    if (pref == 0.0f) continue; /* no data point */
    const double s = orc_cosine_cm(table + user_row * stride, table + r * stride, depth, width, weighted);
    if (isnan(s)) continue;
    preference += s * (double)pref;
    total += s;
    count++;
  }
  if (count <= 1) return NAN;
  float estimate = (float)(preference / total);
  if (use_capper) {
    if (estimate > cap_max) estimate = cap_max;
    else if (estimate < cap_min) estimate = cap_min;
  }
  return estimate;
}

/* SimilarUser.compareTo (T/impl/recommender/SimilarUser.java:62-78): similarity
 * desc, then ID asc.  Returns <0 if x sorts before y. */
static int su_cmp(int64_t xid, double xs, int64_t yid, double ys) {
  if (xs > ys) return -1;
  if (xs < ys) return 1;
  if (xid < yid) return -1;
  if (xid > yid) return 1;
  return 0;
}

/* TopItems.getTopUsers (T/impl/recommender/TopItems.java:91-136): a
 * PriorityQueue in reverse SimilarUser order (head = worst member), insertion
 * only while not full or when strictly better than the head's similarity. */
int32_t orc_top_users(const int64_t* ids, const double* scores, int64_t n, int32_t k,
                      int64_t* out_ids, double* out_scores) {
  int64_t* qid = (int64_t*)malloc(sizeof(int64_t) * (size_t)(k + 1));
  double* qs = (double*)malloc(sizeof(double) * (size_t)(k + 1));
  int32_t size = 0;
  int full = 0;
  double lowest = -INFINITY;
  for (int64_t t = 0; t < n; t++) {
    double s = scores[t];
    if (isnan(s)) continue;
    if (full && !(s > lowest)) continue;
    qid[size] = ids[t];
    qs[size] = s;
    size++;
    if (full || size > k) {
      /* poll(): remove the head = the member sorting LAST under compareTo */
      int32_t w = 0;
      for (int32_t m = 1; m < size; m++)
        if (su_cmp(qid[m], qs[m], qid[w], qs[w]) > 0) w = m;
      qid[w] = qid[size - 1];
      qs[w] = qs[size - 1];
      size--;
      full = 1;
    }
    /* lowestTopValue = topUsers.peek().getSimilarity() */
    int32_t h = 0;
    for (int32_t m = 1; m < size; m++)
      if (su_cmp(qid[m], qs[m], qid[h], qs[h]) > 0) h = m;
    lowest = qs[h];
  }
  /* Collections.sort(sorted) by compareTo (insertion sort: k is small) */
  for (int32_t x = 1; x < size; x++) {
    int64_t id = qid[x];
    double s = qs[x];
    int32_t y = x - 1;
    while (y >= 0 && su_cmp(qid[y], qs[y], id, s) > 0) {
      qid[y + 1] = qid[y];
      qs[y + 1] = qs[y];
      y--;
    }
    qid[y + 1] = id;
    qs[y + 1] = s;
  }
  for (int32_t x = 0; x < size; x++) {
    out_ids[x] = qid[x];
    if (out_scores) out_scores[x] = qs[x];
  }
  free(qid);
  free(qs);
  return size;
}

/* CountMinSketchConfig.probaInserted (T/impl/common/CountMinSketchConfig.java:170-178) */
double orc_proba_inserted(int32_t w, int32_t d, int32_t n, int32_t u) {
  double W = w, D = d, N = n, U = u;
  double falseP = pow(1 - pow(1 - 1 / W, N), D);
  return N / (N + falseP * (U - N));
}

/* probaNotExactRetrieve (:190-196) */
double orc_proba_not_exact_retrieve(int32_t w, int32_t d, int32_t n) {
  double W = w, D = d, N = n;
  return pow(1 - pow(1 - 1 / W, N), D);
}

/* Fmeasure (:210-219) */
double orc_fmeasure(int32_t w, int32_t d, int32_t n, int32_t u, double q) {
  double beta = 1 - orc_proba_not_exact_retrieve(w, d, n);
  double p = 1 - orc_proba_inserted(w, d, n, u);
  if (beta == 0 || p == 0) return 0;
  double q2 = pow(q, 2);
  return (1 + 2) * beta * p / (q2 * beta + p);
}

/* computeConfig inner search for one owner (:120-158): d in [1,25), w in [d,n],
 * ties to the LAST maximiser (>=). */
int orc_compute_config(int32_t n, int32_t u, double q, int32_t* best_w, int32_t* best_d,
                       double* delta, double* epsilon) {
  int32_t bestWidth = 0, bestDepth = 0;
  double bestMax = 0;
  for (int32_t d = 1; d < 25; d++)
    for (int32_t w = d; w <= n; w++) {
      double x = orc_fmeasure(w, d, n, u, q);
      if (x >= bestMax) {
        bestWidth = w;
        bestDepth = d;
        bestMax = x;
      }
    }
  if (bestWidth == 0 && bestDepth == 0) return -1;
  *best_w = bestWidth;
  *best_d = bestDepth;
  *epsilon = exp(1.0) / (double)bestWidth;
  *delta = exp(-(double)bestDepth);
  return 0;
}

/* Faithful cost model of CosineCM.userSimilarity over a pair list: the first
 * owner's sketch is rebuilt on every call (exportProfile, CosineCM.java:41-58,86),
 * the second comes from a lazily filled cache (getExportedCMProfile :60-67). */
static void build_one(double* sk, int32_t depth, int32_t width, const int64_t* a, const int64_t* b,
                      const int64_t* keys, const float* vals, int64_t lo, int64_t hi) {
  memset(sk, 0, sizeof(double) * (size_t)depth * (size_t)width);
  for (int64_t t = lo; t < hi; t++) {
    double inc = vals ? (double)vals[t] : 1.0;
    for (int32_t i = 0; i < depth; i++) {
      int32_t j = orc_hash(a[i], b[i], width, keys[t]);
      sk[j + (int64_t)i * width] += inc;
    }
  }
}

int64_t orc_faithful_pairs(const int64_t* offsets, const int64_t* keys, const float* vals,
                           int64_t rows, int32_t depth, int32_t width,
                           const int64_t* a, const int64_t* b,
                           const int64_t* pair_i, const int64_t* pair_j, int64_t npairs,
                           double* out) {
  const size_t stride = (size_t)depth * (size_t)width;
  double* fresh = (double*)malloc(sizeof(double) * stride);
  double** cache = (double**)calloc((size_t)rows, sizeof(double*));
  for (int64_t p = 0; p < npairs; p++) {
    int64_t i = pair_i[p], j = pair_j[p];
    build_one(fresh, depth, width, a, b, keys, vals, offsets[i], offsets[i + 1]);
    if (!cache[j]) {
      cache[j] = (double*)malloc(sizeof(double) * stride);
      build_one(cache[j], depth, width, a, b, keys, vals, offsets[j], offsets[j + 1]);
    }
    out[p] = orc_cosine_cm(fresh, cache[j], depth, width, 0);
  }
  for (int64_t r = 0; r < rows; r++) free(cache[r]);
  free(cache);
  free(fresh);
  return npairs;
}

int64_t orc_build_rows_reuse(const int64_t* offsets, const int64_t* keys, const float* vals,
                             int64_t row_lo, int64_t row_hi, int32_t depth, int32_t width,
                             const int64_t* a, const int64_t* b, double* checksum) {
  const size_t stride = (size_t)depth * (size_t)width;
  double* sk = (double*)malloc(sizeof(double) * stride);
  double acc = 0.0;
  int64_t updates = 0;
  for (int64_t r = row_lo; r < row_hi; r++) {
    build_one(sk, depth, width, a, b, keys, vals, offsets[r], offsets[r + 1]);
    updates += offsets[r + 1] - offsets[r];
    if (offsets[r + 1] > offsets[r]) acc += orc_sketch_get(sk, depth, width, a, b, keys[offsets[r]]);
  }
  free(sk);
  if (checksum) *checksum = acc;
  return updates;
}

/* ---- per-owner shapes at scale (CosineCM.userSimilarity, CosineCM.java:83-96) ----
 * userSimilarity(u1, u2) for Q query owners u1 against EVERY owner u2 of a
 * CSR with unit increments (vals NULL): u1's sketch built at u2's (w, d)
 * (exportProfile with u2's delta/epsilon, :41-58) against u2's own sketch.
 * Both rows are taken sparsely, as (bucket, count) runs in ascending bucket
 * order: the dense sums of orc_sketch_cosine add +0.0 for every other bucket,
 * which changes no partial sum (see orc_cosine_queries_csr), so the result is
 * orc_cosine_cm's on the dense rows bit for bit -- without materialising
 * rows of up to millions of counters per pair.  The owners are grouped by
 * shape so each query is hashed once per (w, d) class.  w[u2] == 0 (no
 * configuration) gives NaN.  out[q * n + u2]; OpenMP over the classes. */
typedef struct { int32_t bucket; int32_t count; } orc_run;

static int cmp_i32(const void* x, const void* y) {
  const int32_t a = *(const int32_t*)x, b = *(const int32_t*)y;
  return a < b ? -1 : a > b;
}

/* sorted runs of the buckets of keys[0..m) in sketch row (a, b, w); returns the run count */
static int64_t sparse_row(const int64_t* keys, int64_t m, int64_t a, int64_t b, int32_t w, int32_t* scratch,
                          orc_run* runs) {
  for (int64_t i = 0; i < m; i++) scratch[i] = orc_hash(a, b, w, keys[i]);
  qsort(scratch, (size_t)m, sizeof(int32_t), cmp_i32);
  int64_t nr = 0;
  for (int64_t i = 0; i < m; i++) {
    if (nr > 0 && runs[nr - 1].bucket == scratch[i]) runs[nr - 1].count++;
    else { runs[nr].bucket = scratch[i]; runs[nr].count = 1; nr++; }
  }
  return nr;
}

static int cmp_shape_idx(const void* x, const void* y, void* ctx) {
  const int32_t* w = ((const int32_t**)ctx)[0];
  const int32_t* d = ((const int32_t**)ctx)[1];
  const int64_t i = *(const int64_t*)x, j = *(const int64_t*)y;
  if (w[i] != w[j]) return w[i] < w[j] ? -1 : 1;
  if (d[i] != d[j]) return d[i] < d[j] ? -1 : 1;
  return i < j ? -1 : i > j;
}

void orc_per_owner_rows_csr(const int64_t* off, const int64_t* keys, int64_t n, const int32_t* shape_w,
                            const int32_t* shape_d, const int64_t* a, const int64_t* b, const int64_t* queries,
                            int64_t Q, int32_t threads, double* out) {
  int64_t* order = (int64_t*)malloc(sizeof(int64_t) * (size_t)(n > 0 ? n : 1));
  for (int64_t i = 0; i < n; i++) order[i] = i;
  const int32_t* ctx[2] = {shape_w, shape_d};
  qsort_r(order, (size_t)n, sizeof(int64_t), cmp_shape_idx, ctx);
  /* class boundaries */
  int64_t* cls = (int64_t*)malloc(sizeof(int64_t) * (size_t)(n + 1));
  int64_t nc = 0;
  for (int64_t i = 0; i < n; i++)
    if (i == 0 || shape_w[order[i]] != shape_w[order[i - 1]] || shape_d[order[i]] != shape_d[order[i - 1]])
      cls[nc++] = i;
  cls[nc] = n;
  int64_t qmax = 1, mmax = 1;
  for (int64_t q = 0; q < Q; q++) {
    const int64_t m = off[queries[q] + 1] - off[queries[q]];
    if (m > qmax) qmax = m;
  }
  for (int64_t i = 0; i < n; i++)
    if (off[i + 1] - off[i] > mmax) mmax = off[i + 1] - off[i];
#pragma omp parallel num_threads(threads > 0 ? threads : 1)
  {
    const int64_t big = qmax > mmax ? qmax : mmax;
    int32_t* scratch = (int32_t*)malloc(sizeof(int32_t) * (size_t)big);
    orc_run* mr = (orc_run*)malloc(sizeof(orc_run) * (size_t)mmax);
    /* each query's runs for every sketch row of the class: [Q][d][qmax] */
    orc_run* qr = NULL;
    int64_t* qn = NULL;
    double* qa = NULL;
    int32_t qd_cap = 0;
#pragma omp for schedule(dynamic, 1)
    for (int64_t c = 0; c < nc; c++) {
      const int64_t first = order[cls[c]];
      const int32_t w = shape_w[first], d = shape_d[first];
      if (w <= 0 || d <= 0) {
        for (int64_t t = cls[c]; t < cls[c + 1]; t++)
          for (int64_t q = 0; q < Q; q++) out[q * n + order[t]] = NAN;
        continue;
      }
      if (d > qd_cap) {
        free(qr);
        free(qn);
        free(qa);
        qd_cap = d;
        qr = (orc_run*)malloc(sizeof(orc_run) * (size_t)(Q * d * qmax));
        qn = (int64_t*)malloc(sizeof(int64_t) * (size_t)(Q * d));
        qa = (double*)malloc(sizeof(double) * (size_t)(Q * d));
      }
      for (int64_t q = 0; q < Q; q++) {
        const int64_t u1 = queries[q];
        for (int32_t r = 0; r < d; r++) {
          orc_run* runs = qr + (q * d + r) * qmax;
          const int64_t nr = sparse_row(keys + off[u1], off[u1 + 1] - off[u1], a[r], b[r], w, scratch, runs);
          qn[q * d + r] = nr;
          double v = 0.0;
          for (int64_t t = 0; t < nr; t++) v += (double)runs[t].count * (double)runs[t].count;
          qa[q * d + r] = v;
        }
      }
      for (int64_t t = cls[c]; t < cls[c + 1]; t++) {
        const int64_t u2 = order[t];
        double mins[64];
        for (int64_t q = 0; q < Q && q < 64; q++) mins[q] = DBL_MAX;
        for (int32_t r = 0; r < d; r++) {
          const int64_t nr = sparse_row(keys + off[u2], off[u2 + 1] - off[u2], a[r], b[r], w, scratch, mr);
          double vb = 0.0;
          for (int64_t s = 0; s < nr; s++) vb += (double)mr[s].count * (double)mr[s].count;
          for (int64_t q = 0; q < Q && q < 64; q++) {
            const orc_run* ra = qr + (q * d + r) * qmax;
            const int64_t na = qn[q * d + r];
            double ab = 0.0;
            int64_t i = 0, j = 0;
            while (i < na && j < nr) {
              if (ra[i].bucket < mr[j].bucket) i++;
              else if (ra[i].bucket > mr[j].bucket) j++;
              else {
                ab += (double)ra[i].count * (double)mr[j].count;
                i++;
                j++;
              }
            }
            const double den = sqrt(qa[q * d + r]) * sqrt(vb);
            if (den != 0) mins[q] = java_min(mins[q], ab / den);
          }
        }
        for (int64_t q = 0; q < Q && q < 64; q++) {
          double res = mins[q] == DBL_MAX ? NAN : mins[q];
          if (!isnan(res)) res = orc_normalize_weight_result(res, 1, 0, 0);
          out[q * n + u2] = res;
        }
      }
    }
    free(scratch);
    free(mr);
    free(qr);
    free(qn);
    free(qa);
  }
  free(order);
  free(cls);
}
