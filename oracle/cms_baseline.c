/*
 * cms_baseline.c -- the CPU baselines bench.py times beside the GPU (SURVEY.md
 * §8(d) "CPU baseline"): the reference path restated in C, in two modes, on
 * one core or on all the host cores the run may use (OpenMP).  TEST / BENCH
 * INFRASTRUCTURE ONLY, like the rest of oracle/: nothing in mahout_amd/ links
 * it.  The reference JVM path itself cannot run here (no JDK).
 *
 *   faithful   -- the reference's cost model: per owner a fresh fp64
 *                 DoubleCountMinSketch (d*w zero fill) and d hashes per update
 *                 computed like BigInteger ((a*k + b) mod p) mod w with a
 *                 128-bit division (HashFunction.java:31-34,
 *                 DoubleCountMinSketch.java:72-80); for similarities u1's
 *                 sketch is rebuilt on every call and u2's comes from a cache
 *                 (CosineCM.java:41-67,83-96).  Faster than the JVM (no
 *                 BigInteger allocation, no log.debug varargs boxing, no
 *                 TDoubleArrayList growth), so it flatters the reference.
 *   efficient  -- what a careful CPU implementation would do: u32 counters in
 *                 one shared table and the exact hash by folding 2^63 = 25
 *                 (mod p) instead of a division; for similarities every sketch
 *                 prebuilt once, per-(owner, row) norms computed once, one fp64
 *                 dot per row pair, four partners per pass over the query row.
 *
 * Parallel runs split owners (ingest) or query rows (similarity) across
 * threads with a dynamic schedule; every mode returns a checksum so the work
 * cannot be optimised away.
 */
#include <math.h>
#include <omp.h>
#include <stdint.h>
#include <stdlib.h>
#include <string.h>

#include "cms_oracle.h"

#define P63 9223372036854775783ULL /* 2^63 - 25 */
#define M63 ((1ULL << 63) - 1)

/* x mod p for x < 2^127, by folding 2^63 = 25 (mod p) twice */
static inline uint64_t fold_mod_p(unsigned __int128 x) {
  unsigned __int128 y = (x >> 63) * 25u + (x & M63);
  uint64_t z = (uint64_t)((y >> 63) * 25u) + (uint64_t)(y & M63);
  while (z >= P63) z -= P63;
  return z;
}

static inline uint64_t key_mod_p(int64_t k) {
  /* BigInteger semantics: the non-negative residue of a signed key */
  int64_t r = k % (int64_t)P63;
  return (uint64_t)(r < 0 ? r + (int64_t)P63 : r);
}

/* HashFunction.hash without a division: a, b, k reduced mod p */
static inline uint32_t fast_hash(uint64_t ap, uint64_t bp, uint64_t kp, uint32_t w, uint32_t wmask) {
  uint64_t h = fold_mod_p((unsigned __int128)ap * kp);
  h += bp;
  if (h >= P63) h -= P63;
  return wmask ? (uint32_t)(h & wmask) : (uint32_t)(h % w);
}

static int use_threads(int32_t nthreads) { return nthreads > 0 ? nthreads : omp_get_max_threads(); }

/* faithful ingest: owners [lo, hi) each into a fresh fp64 sketch */
int64_t orc_ingest_faithful_par(const int64_t* offsets, const int64_t* keys, const float* vals, int64_t row_lo,
                                int64_t row_hi, int32_t depth, int32_t width, const int64_t* a, const int64_t* b,
                                int32_t nthreads, double* checksum) {
  const size_t stride = (size_t)depth * (size_t)width;
  double acc = 0.0;
  int64_t updates = 0;
#pragma omp parallel num_threads(use_threads(nthreads)) reduction(+ : acc, updates)
  {
    double* sk = (double*)malloc(sizeof(double) * stride);
#pragma omp for schedule(dynamic, 16)
    for (int64_t r = row_lo; r < row_hi; r++) {
      memset(sk, 0, sizeof(double) * stride);
      for (int64_t t = offsets[r]; t < offsets[r + 1]; t++) {
        const double inc = vals ? (double)vals[t] : 1.0;
        for (int32_t i = 0; i < depth; i++) sk[orc_hash(a[i], b[i], width, keys[t]) + (int64_t)i * width] += inc;
      }
      updates += offsets[r + 1] - offsets[r];
      if (offsets[r + 1] > offsets[r]) acc += orc_sketch_get(sk, depth, width, a, b, keys[offsets[r]]);
    }
    free(sk);
  }
  if (checksum) *checksum = acc;
  return updates;
}

/* efficient ingest: owners [lo, hi) into a shared u32 table [hi-lo][d][w] */
int64_t orc_ingest_efficient_par(const int64_t* offsets, const int64_t* keys, const float* vals, int64_t row_lo,
                                 int64_t row_hi, int32_t depth, int32_t width, const int64_t* a, const int64_t* b,
                                 int32_t nthreads, uint32_t* table, double* checksum) {
  const size_t stride = (size_t)depth * (size_t)width;
  uint64_t ap[32], bp[32];
  for (int32_t i = 0; i < depth && i < 32; i++) {
    ap[i] = key_mod_p(a[i]);
    bp[i] = key_mod_p(b[i]);
  }
  const uint32_t wmask = (width & (width - 1)) == 0 ? (uint32_t)width - 1u : 0u;
  double acc = 0.0;
  int64_t updates = 0;
#pragma omp parallel for num_threads(use_threads(nthreads)) schedule(dynamic, 16) reduction(+ : acc, updates)
  for (int64_t r = row_lo; r < row_hi; r++) {
    uint32_t* sk = table + (size_t)(r - row_lo) * stride;
    memset(sk, 0, sizeof(uint32_t) * stride);
    for (int64_t t = offsets[r]; t < offsets[r + 1]; t++) {
      const uint32_t inc = vals ? (uint32_t)vals[t] : 1u;
      const uint64_t kp = key_mod_p(keys[t]);
      for (int32_t i = 0; i < depth; i++) sk[fast_hash(ap[i], bp[i], kp, (uint32_t)width, wmask) + (size_t)i * width] += inc;
    }
    updates += offsets[r + 1] - offsets[r];
    if (offsets[r + 1] > offsets[r]) acc += sk[fast_hash(ap[0], bp[0], key_mod_p(keys[offsets[r]]), width, wmask)];
  }
  if (checksum) *checksum = acc;
  return updates;
}

/* faithful similarities: pairs (pi[p], pj[p]); u2 sketches prebuilt for every
 * owner of the sample (the CosineCM cache, filled once), u1 rebuilt per call */
int64_t orc_faithful_pairs_par(const int64_t* offsets, const int64_t* keys, const float* vals, int64_t rows,
                               int32_t depth, int32_t width, const int64_t* a, const int64_t* b, const int64_t* pi,
                               const int64_t* pj, int64_t npairs, int32_t nthreads, double* checksum) {
  const size_t stride = (size_t)depth * (size_t)width;
  double* cache = (double*)malloc(sizeof(double) * stride * (size_t)rows);
  double acc = 0.0;
  const int nt = use_threads(nthreads);
#pragma omp parallel for num_threads(nt) schedule(dynamic, 4)
  for (int64_t r = 0; r < rows; r++) {
    double* sk = cache + (size_t)r * stride;
    memset(sk, 0, sizeof(double) * stride);
    for (int64_t t = offsets[r]; t < offsets[r + 1]; t++) {
      const double inc = vals ? (double)vals[t] : 1.0;
      for (int32_t i = 0; i < depth; i++) sk[orc_hash(a[i], b[i], width, keys[t]) + (int64_t)i * width] += inc;
    }
  }
#pragma omp parallel num_threads(nt) reduction(+ : acc)
  {
    double* fresh = (double*)malloc(sizeof(double) * stride);
#pragma omp for schedule(dynamic, 64)
    for (int64_t p = 0; p < npairs; p++) {
      const int64_t i = pi[p];
      memset(fresh, 0, sizeof(double) * stride);
      for (int64_t t = offsets[i]; t < offsets[i + 1]; t++) {
        const double inc = vals ? (double)vals[t] : 1.0;
        for (int32_t r = 0; r < depth; r++) fresh[orc_hash(a[r], b[r], width, keys[t]) + (int64_t)r * width] += inc;
      }
      const double s = orc_cosine_cm(fresh, cache + (size_t)pj[p] * stride, depth, width, 0);
      if (s == s) acc += s;
    }
    free(fresh);
  }
  free(cache);
  if (checksum) *checksum = acc;
  return npairs;
}

/* efficient similarities over prebuilt fp64 sketches [rows][d][w]: every
 * unordered pair (i, j), i in [i_lo, i_hi), j > i; norms once per (owner, row),
 * four partners per sweep of the query row */
int64_t orc_allpairs_efficient_par(const double* table, int64_t rows, int32_t depth, int32_t width, int64_t i_lo,
                                   int64_t i_hi, int32_t nthreads, double* checksum) {
  const size_t stride = (size_t)depth * (size_t)width;
  double* nrm = (double*)malloc(sizeof(double) * (size_t)rows * (size_t)depth);
  const int nt = use_threads(nthreads);
#pragma omp parallel for num_threads(nt) schedule(static)
  for (int64_t r = 0; r < rows; r++)
    for (int32_t i = 0; i < depth; i++) {
      const double* x = table + (size_t)r * stride + (size_t)i * width;
      double s = 0.0;
      for (int32_t j = 0; j < width; j++) s += x[j] * x[j];
      nrm[r * depth + i] = sqrt(s);
    }
  double acc = 0.0;
  int64_t pairs = 0;
#pragma omp parallel for num_threads(nt) schedule(dynamic, 1) reduction(+ : acc, pairs)
  for (int64_t q = i_lo; q < i_hi; q++) {
    const double* A = table + (size_t)q * stride;
    for (int64_t j0 = q + 1; j0 < rows; j0 += 4) {
      const int nj = rows - j0 < 4 ? (int)(rows - j0) : 4;
      double mn[4] = {INFINITY, INFINITY, INFINITY, INFINITY};
      for (int32_t i = 0; i < depth; i++) {
        const double* x = A + (size_t)i * width;
        double ab[4] = {0, 0, 0, 0};
        const double* y[4];
        for (int c = 0; c < 4; c++) y[c] = table + (size_t)(j0 + (c < nj ? c : 0)) * stride + (size_t)i * width;
        for (int32_t j = 0; j < width; j++) {
          const double xv = x[j];
          ab[0] += xv * y[0][j];
          ab[1] += xv * y[1][j];
          ab[2] += xv * y[2][j];
          ab[3] += xv * y[3][j];
        }
        for (int c = 0; c < nj; c++) {
          const double den = nrm[q * depth + i] * nrm[(j0 + c) * depth + i];
          if (den != 0) {
            const double v = ab[c] / den;
            if (v < mn[c]) mn[c] = v;
          }
        }
      }
      for (int c = 0; c < nj; c++) {
        if (mn[c] != INFINITY) acc += mn[c];
        pairs++;
      }
    }
  }
  free(nrm);
  if (checksum) *checksum = acc;
  return pairs;
}

/* GenericUserBasedRecommender.recommend (T/impl/recommender/
 * GenericUserBasedRecommender.java:84-105) with NearestNUserNeighborhood(nn)
 * (T/impl/neighborhood/NearestNUserNeighborhood.java:84-95) and the CosineCM
 * point-query estimate (:134-184), for users [u_lo, u_hi) of a user-owner
 * model over prebuilt fp64 sketches [rows][d][w] (efficient mode): per user
 * the similarity to every other user (min over rows of AB / (|A| |B|),
 * clamped as normalizeWeightResult), the first nn under (similarity desc,
 * ID = row asc), the neighbours' items minus the user's own (item indices
 * into item_keys; off/items: the model's CSR of item indices), each
 * candidate's estimate, and the how_many best values.  Returns the
 * estimates computed; *checksum sums the recommended values. */
int64_t orc_recommend_par(const double* table, int64_t rows, int32_t depth, int32_t width, const int64_t* a,
                          const int64_t* b, const int64_t* off, const int32_t* items, const int64_t* item_keys,
                          int64_t n_items, int32_t nn, int32_t how_many, int32_t use_capper, float cap_min,
                          float cap_max, int64_t u_lo, int64_t u_hi, int32_t nthreads, double* checksum) {
  const size_t stride = (size_t)depth * (size_t)width;
  double* nrm = (double*)malloc(sizeof(double) * (size_t)rows * (size_t)depth);
  uint64_t ap[64], bp[64];
  for (int i = 0; i < depth; i++) {
    ap[i] = key_mod_p(a[i]);
    bp[i] = key_mod_p(b[i]);
  }
  const uint32_t wmask = (width & (width - 1)) == 0 ? (uint32_t)width - 1u : 0u;
  const int nt = use_threads(nthreads);
#pragma omp parallel for num_threads(nt) schedule(static)
  for (int64_t r = 0; r < rows; r++)
    for (int32_t i = 0; i < depth; i++) {
      const double* x = table + (size_t)r * stride + (size_t)i * width;
      double s = 0.0;
      for (int32_t j = 0; j < width; j++) s += x[j] * x[j];
      nrm[r * depth + i] = sqrt(s);
    }
  double acc = 0.0;
  int64_t nest = 0;
#pragma omp parallel num_threads(nt) reduction(+ : acc, nest)
  {
    double* sims = (double*)malloc(sizeof(double) * (size_t)rows);
    int64_t* ids = (int64_t*)malloc(sizeof(int64_t) * (size_t)rows);
    int64_t* nb = (int64_t*)malloc(sizeof(int64_t) * (size_t)(nn > 0 ? nn : 1));
    double* nbs = (double*)malloc(sizeof(double) * (size_t)(nn > 0 ? nn : 1));
    uint8_t* mark = (uint8_t*)calloc((size_t)n_items, 1);
    int32_t* cand = (int32_t*)malloc(sizeof(int32_t) * (size_t)n_items);
    float* best = (float*)malloc(sizeof(float) * (size_t)(how_many + 1));
    for (int64_t r = 0; r < rows; r++) ids[r] = r;
#pragma omp for schedule(dynamic, 4)
    for (int64_t u = u_lo; u < u_hi; u++) {
      const double* A = table + (size_t)u * stride;
      for (int64_t v = 0; v < rows; v++) {
        if (v == u) {
          sims[v] = NAN;  /* the user itself is never a neighbour */
          continue;
        }
        const double* B = table + (size_t)v * stride;
        double mn = INFINITY;
        for (int32_t i = 0; i < depth; i++) {
          const double* x = A + (size_t)i * width;
          const double* y = B + (size_t)i * width;
          double ab = 0.0;
          for (int32_t j = 0; j < width; j++) ab += x[j] * y[j];
          const double den = nrm[u * depth + i] * nrm[v * depth + i];
          if (den != 0) {
            const double c = ab / den;
            if (c < mn) mn = c;
          }
        }
        sims[v] = mn == INFINITY ? NAN : (mn > 1.0 ? 1.0 : mn < -1.0 ? -1.0 : mn);
      }
      const int32_t m = orc_top_users(ids, sims, rows, nn, nb, nbs);
      int32_t nc = 0;
      for (int32_t t = 0; t < m; t++)
        for (int64_t k = off[nb[t]]; k < off[nb[t] + 1]; k++)
          if (!mark[items[k]]) {
            mark[items[k]] = 1;
            cand[nc++] = items[k];
          }
      for (int64_t k = off[u]; k < off[u + 1]; k++) mark[items[k]] = 2;  /* the user's own items */
      int32_t nbest = 0;
      for (int32_t c = 0; c < nc; c++) {
        const int32_t it = cand[c];
        if (mark[it] == 2) continue;
        uint32_t bk[64];
        const uint64_t kp = key_mod_p(item_keys[it]);
        for (int i = 0; i < depth; i++) bk[i] = (uint32_t)i * (uint32_t)width + fast_hash(ap[i], bp[i], kp, (uint32_t)width, wmask);
        double preference = 0.0, total = 0.0;
        int count = 0;
        for (int32_t t = 0; t < m; t++) {
          const double* S = table + (size_t)nb[t] * stride;
          double est = 1.7976931348623157e308;
          for (int i = 0; i < depth; i++)
            if (S[bk[i]] < est) est = S[bk[i]];
          const float pref = (float)est;
          if (pref == 0.0f || isnan(nbs[t])) continue;
          preference += nbs[t] * (double)pref;
          total += nbs[t];
          count++;
        }
        nest++;
        if (count <= 1) continue;
        float e = (float)(preference / total);
        if (use_capper) e = e > cap_max ? cap_max : e < cap_min ? cap_min : e;
        /* keep the how_many largest (insertion into a short sorted array) */
        int32_t p;
        if (nbest < how_many) {
          p = nbest++;
        } else {
          if (!(e > best[how_many - 1])) continue;
          p = how_many - 1;
        }
        while (p > 0 && best[p - 1] < e) {
          best[p] = best[p - 1];
          p--;
        }
        best[p] = e;
      }
      for (int32_t t = 0; t < nbest; t++) acc += best[t];
      for (int32_t c = 0; c < nc; c++) mark[cand[c]] = 0;
      for (int64_t k = off[u]; k < off[u + 1]; k++) mark[items[k]] = 0;
    }
    free(sims);
    free(ids);
    free(nb);
    free(nbs);
    free(mark);
    free(cand);
    free(best);
  }
  free(nrm);
  if (checksum) *checksum = acc;
  return nest;
}

int32_t orc_max_threads(void) { return omp_get_max_threads(); }
