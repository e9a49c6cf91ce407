// cms_query.hip -- sketch-cosine queries on gfx950.
//
// cosine (T/impl/common/DoubleCountMinSketch.java:114-149): for each sketch
// row i, valueA = sum xa^2, valueB = sum xb^2, valueAB = sum xa*xb (fp64, j
// ascending); den = sqrt(valueA)*sqrt(valueB); if den != 0 the row cosine
// valueAB/den enters a Math.min; NaN if no row qualified.  Then CosineCM
// applies normalizeWeightResult(r, 1, 0) (AbstractSimilarity.java:313-330).
//
// With u32 counters every product and partial sum is an integer; when a
// row's sum of squares is < 2^53 every fp64 partial sum of the reference is
// exact, so the integer dot product (u64) converted to double IS the
// reference's valueAB bit for bit, and sqrt/mul/div below are the same
// correctly rounded IEEE operations Java performs.  Rows whose norm reaches
// 2^53 take a sequential fp64 loop in the reference's exact order.
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cfloat>

#include "cms_device.h"
#include "cms_internal.h"

namespace cms {

__device__ __forceinline__ uint64_t wave_sum_u64(uint64_t v) {
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) v += __shfl_xor(v, o, 64);
  return v;
}

// Reference-order sequential fp64 sums for one sketch row (inexact regime).
__device__ void seq_row_sums(const TableView& tv, int64_t ra, int64_t rb, int64_t c0, int w, double& A, double& B,
                             double& AB) {
  A = 0.0;
  B = 0.0;
  AB = 0.0;
  for (int j = 0; j < w; ++j) {
    double xa = (double)tv.get(ra, c0 + j), xb = (double)tv.get(rb, c0 + j);
    A = __dadd_rn(A, __dmul_rn(xa, xa));
    B = __dadd_rn(B, __dmul_rn(xb, xb));
    AB = __dadd_rn(AB, __dmul_rn(xa, xb));
  }
}

// One workgroup (256 threads) per (query, target) pair.
__global__ __launch_bounds__(256) void k_pair_cosine(TableView tv, const uint64_t* norm, const double* nsqrt,
                                                     HashParams hp, int64_t q_row0, const int64_t* q_rows,
                                                     const int64_t* rows, int64_t m, int64_t nrows, int weighted,
                                                     double* out) {
  __shared__ uint64_t red[4];
  extern __shared__ uint32_t lc[];  // [w / 4]: a list query row's sketch row as u8 counters (list x list pairs)
  const int64_t t = blockIdx.x;
  if (t >= m) return;
  const int64_t r2 = rows[t];
  const int64_t q_row = q_rows ? q_rows[t] : q_row0;  // one query row, or one per pair (batched estimates)
  if (r2 < 0 || r2 >= nrows || q_row < 0 || q_row >= nrows) {
    if (threadIdx.x == 0) out[t] = __builtin_nan("");
    return;
  }
  const int w = (int)hp.width;
  double minc = DBL_MAX;
  for (int d = 0; d < hp.depth; ++d) {
    const int64_t c0 = (int64_t)d * w;
    const uint64_t Na = norm[q_row * hp.depth + d], Nb = norm[r2 * hp.depth + d];
    const bool exact = Na < (1ULL << 53) && Nb < (1ULL << 53);
    double valueAB, den;
    if (exact) {
      uint64_t dot = 0;
      const bool la = tv.hidx[q_row] == kFormList, lb = tv.hidx[r2] == kFormList;
      if (la && lb) {  // the query's row counted in LDS, summed at the other list's entries
        const uint32_t qm = tv.list_m(q_row), lm = tv.list_m(r2);
        const uint16_t* qe = tv.list_row(q_row, d, qm);
        const uint16_t* e = tv.list_row(r2, d, lm);
        for (int j = threadIdx.x; j < (w >> 2); j += 256) lc[j] = 0u;
        __syncthreads();
        for (uint32_t t = threadIdx.x; t < qm; t += 256) atomicAdd(&lc[qe[t] >> 2], 1u << ((qe[t] & 3u) * 8u));
        __syncthreads();
        const uint8_t* c8 = reinterpret_cast<const uint8_t*>(lc);
        for (uint32_t t = threadIdx.x; t < lm; t += 256) dot += c8[e[t]];
        __syncthreads();  // read before the next sketch row zeroes the counts
      } else if (la || lb) {  // valueAB = sum over a list row's entries of the other row's counter (update is linear)
        const int64_t lr = lb ? r2 : q_row, other = lb ? q_row : r2;
        const uint32_t lm = tv.list_m(lr);
        const uint16_t* e = tv.list_row(lr, d, lm);
        for (uint32_t t = threadIdx.x; t < lm; t += 256) dot += tv.get(other, c0 + e[t]);
      } else if ((w & 3) == 0) {
        for (int j = threadIdx.x; j < (w >> 2); j += 256) {
          const uint4 x = tv.get4(q_row, c0 + 4 * j), y = tv.get4(r2, c0 + 4 * j);
          dot += (uint64_t)x.x * y.x + (uint64_t)x.y * y.y + (uint64_t)x.z * y.z + (uint64_t)x.w * y.w;
        }
      } else {
        for (int j = threadIdx.x; j < w; j += 256) dot += (uint64_t)tv.get(q_row, c0 + j) * tv.get(r2, c0 + j);
      }
      dot = wave_sum_u64(dot);
      if ((threadIdx.x & 63) == 0) red[threadIdx.x >> 6] = dot;
      __syncthreads();
      dot = red[0] + red[1] + red[2] + red[3];
      __syncthreads();
      valueAB = (double)dot;
      den = __dmul_rn(nsqrt[q_row * hp.depth + d], nsqrt[r2 * hp.depth + d]);
    } else {
      double A, B;
      seq_row_sums(tv, q_row, r2, c0, w, A, B, valueAB);  // every thread (uniform result)
      den = __dmul_rn(__dsqrt_rn(A), __dsqrt_rn(B));
    }
    if (den != 0.0) minc = java_min(minc, __ddiv_rn(valueAB, den));
  }
  if (threadIdx.x == 0) {
    double r = (minc == DBL_MAX) ? __builtin_nan("") : minc;
    if (r == r) r = normalize_weight(r, weighted);
    out[t] = r;
  }
}

int pair_cosines(cms_handle* h, int64_t q_row, const int64_t* d_rows, int64_t m, double* d_out, hipStream_t s) {
  if (m <= 0) return CMS_OK;
  if (h->f64) return f64_pair_cosines(h, q_row, d_rows, m, d_out, s);
  TimedScope ts(h, "pair_cosine", s == nullptr);
  hipLaunchKernelGGL(k_pair_cosine, dim3((unsigned)m), dim3(256), (size_t)h->p.width, s ? s : h->stream, h->tview(), h->d_norm,
                     h->d_norm_sqrt, h->hp, q_row, (const int64_t*)nullptr, d_rows, m, h->n, (int)h->p.weighting,
                     d_out);
  CMS_HIP(hipGetLastError());
  return CMS_OK;
}

// cos(q_rows[t], rows[t]) for t < m: one launch for the (user, neighbour)
// pairs of many users (u32 counters).
int pair_cosines_many(cms_handle* h, const int64_t* d_qrows, const int64_t* d_rows, int64_t m, double* d_out,
                      hipStream_t s) {
  if (m <= 0) return CMS_OK;
  TimedScope ts(h, "pair_cosine", s == nullptr);
  hipLaunchKernelGGL(k_pair_cosine, dim3((unsigned)m), dim3(256), (size_t)h->p.width, s ? s : h->stream, h->tview(),
                     h->d_norm, h->d_norm_sqrt, h->hp, (int64_t)0, d_qrows, d_rows, m, h->n, (int)h->p.weighting,
                     d_out);
  CMS_HIP(hipGetLastError());
  return CMS_OK;
}

// DoubleCountMinSketch.get(key) (:94-103): min over rows, from Double.MAX_VALUE.
__global__ void k_point_query(TableView tv, HashParams hp, int64_t row, const int64_t* keys, int64_t m,
                              double* out) {
  for (int64_t i = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; i < m; i += (int64_t)gridDim.x * blockDim.x) {
    uint64_t kp = reduce_key(keys[i]);
    double est = DBL_MAX;
    for (int d = 0; d < hp.depth; ++d) {
      double v = (double)tv.get(row, (int64_t)d * hp.width + bucket(hp, d, kp));
      if (v < est) est = v;
    }
    out[i] = ldexp(est, -hp.frac_bits);
  }
}

// GenericUserBasedRecommender.doEstimatePreference with the CosineCM point
// query (GenericUserBasedRecommender.java:134-184), one thread per item, the
// neighbourhood walked in the caller's order so the fp64 sums round as in Java:
// pref = (float) get(item) of the neighbour's sketch (0 -> no data point),
// sim = userSimilarity(user, neighbour) (NaN skipped), preference += sim*pref,
// total += sim; < 2 points -> NaN; (float)(preference/total); then the
// EstimatedPreferenceCapper clamp when enabled.
__global__ void k_estimate(TableView tv, HashParams hp, int64_t user_row, const int64_t* nb_rows,
                           const double* sims, int64_t m, const int64_t* items, int64_t q, int use_capper, float lo,
                           float hi, float* out) {
  for (int64_t i = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; i < q; i += (int64_t)gridDim.x * blockDim.x) {
    const uint64_t kp = reduce_key(items[i]);
    uint32_t bk[CMS_MAX_DEPTH];
    for (int d = 0; d < hp.depth; ++d) bk[d] = (uint32_t)d * hp.width + bucket(hp, d, kp);
    double preference = 0.0, total = 0.0;
    int count = 0;
    for (int64_t j = 0; j < m; ++j) {
      const int64_t r = nb_rows[j];
      if (r == user_row) continue;
      double est = DBL_MAX;
      for (int d = 0; d < hp.depth; ++d) {
        const double v = (double)tv.get(r, bk[d]);
        if (v < est) est = v;
      }
      const float pref = (float)ldexp(est, -hp.frac_bits);
      if (pref == 0.0f) continue;
      const double s = sims[j];
      if (s != s) continue;
      preference = __dadd_rn(preference, __dmul_rn(s, (double)pref));
      total = __dadd_rn(total, s);
      ++count;
    }
    float e = __builtin_nanf("");
    if (count > 1) {
      e = (float)__ddiv_rn(preference, total);
      if (use_capper) {
        if (e > hi) e = hi;
        else if (e < lo) e = lo;
      }
    }
    out[i] = e;
  }
}

int estimate_preferences(cms_handle* h, int64_t user_row, const int64_t* d_nb_rows, const double* d_sims, int64_t m,
                         const int64_t* d_items, int64_t q, int use_capper, float lo, float hi, float* d_out,
                         hipStream_t s) {
  if (q <= 0) return CMS_OK;
  if (h->f64)
    return f64_estimate_preferences(h, user_row, d_nb_rows, d_sims, m, d_items, q, use_capper, lo, hi, d_out, s);
  unsigned grid = (unsigned)std::min<int64_t>((q + 255) / 256, 4096);
  hipLaunchKernelGGL(k_estimate, dim3(grid), dim3(256), 0, s ? s : h->stream, h->tview(), h->hp, user_row, d_nb_rows, d_sims,
                     m, d_items, q, use_capper, lo, hi, d_out);
  CMS_HIP(hipGetLastError());
  return CMS_OK;
}

// k_estimate for many users in one launch: candidate i belongs to user
// item_user[i], whose neighbourhood (rows and similarities, in the caller's
// order) is nb_rows / sims [nb_off[u], nb_off[u + 1]).  Each candidate's
// arithmetic is exactly k_estimate's.
__global__ void k_estimate_batch(TableView tv, HashParams hp, const int64_t* user_rows, const int64_t* nb_off,
                                 const int64_t* nb_rows, const double* sims, const int32_t* item_user,
                                 const int64_t* items, int64_t q, int use_capper, float lo, float hi, float* out) {
  for (int64_t i = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; i < q; i += (int64_t)gridDim.x * blockDim.x) {
    const int32_t u = item_user[i];
    const int64_t user_row = user_rows[u];
    const uint64_t kp = reduce_key(items[i]);
    uint32_t bk[CMS_MAX_DEPTH];
    for (int d = 0; d < hp.depth; ++d) bk[d] = (uint32_t)d * hp.width + bucket(hp, d, kp);
    double preference = 0.0, total = 0.0;
    int count = 0;
    for (int64_t j = nb_off[u]; j < nb_off[u + 1]; ++j) {
      const int64_t r = nb_rows[j];
      if (r == user_row) continue;
      double est = DBL_MAX;
      for (int d = 0; d < hp.depth; ++d) {
        const double v = (double)tv.get(r, bk[d]);
        if (v < est) est = v;
      }
      const float pref = (float)ldexp(est, -hp.frac_bits);
      if (pref == 0.0f) continue;
      const double s = sims[j];
      if (s != s) continue;
      preference = __dadd_rn(preference, __dmul_rn(s, (double)pref));
      total = __dadd_rn(total, s);
      ++count;
    }
    float e = __builtin_nanf("");
    if (count > 1) {
      e = (float)__ddiv_rn(preference, total);
      if (use_capper) {
        if (e > hi) e = hi;
        else if (e < lo) e = lo;
      }
    }
    out[i] = e;
  }
}

int estimate_preferences_batch(cms_handle* h, const int64_t* d_user_rows, const int64_t* d_nb_off,
                               const int64_t* d_nb_rows, const double* d_sims, const int32_t* d_item_user,
                               const int64_t* d_items, int64_t q, int use_capper, float lo, float hi, float* d_out,
                               hipStream_t s) {
  if (q <= 0) return CMS_OK;
  unsigned grid = (unsigned)std::min<int64_t>((q + 255) / 256, 8192);
  hipLaunchKernelGGL(k_estimate_batch, dim3(grid), dim3(256), 0, s ? s : h->stream, h->tview(), h->hp, d_user_rows,
                     d_nb_off, d_nb_rows, d_sims, d_item_user, d_items, q, use_capper, lo, hi, d_out);
  CMS_HIP(hipGetLastError());
  return CMS_OK;
}

int point_queries(cms_handle* h, int64_t row, const int64_t* d_keys, int64_t m, double* d_out, hipStream_t s) {
  if (m <= 0) return CMS_OK;
  if (h->f64) return f64_point_queries(h, row, d_keys, m, d_out, s);
  unsigned grid = (unsigned)std::min<int64_t>((m + 255) / 256, 4096);
  hipLaunchKernelGGL(k_point_query, dim3(grid), dim3(256), 0, s ? s : h->stream, h->tview(), h->hp, row, d_keys, m, d_out);
  CMS_HIP(hipGetLastError());
  return CMS_OK;
}

}  // namespace cms
