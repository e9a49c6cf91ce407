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

#include "cms_internal.h"

namespace cms {

__device__ __forceinline__ double java_min(double a, double b) {
  if (a != a) return a;
  if (a == 0.0 && b == 0.0 && signbit(b)) return b;
  return (a <= b) ? a : b;
}

// normalizeWeightResult(result, count=1, num=0)
__device__ __forceinline__ double normalize_weight(double r, int weighted) {
  if (weighted) {
    const double scale = __dsub_rn(1.0, 1.0 / 1.0);  // 1 - count/(num+1) = 0
    if (r < 0.0) r = __dadd_rn(-1.0, __dmul_rn(scale, __dadd_rn(1.0, r)));
    else r = __dsub_rn(1.0, __dmul_rn(scale, __dsub_rn(1.0, r)));
  }
  if (r < -1.0) r = -1.0;
  else if (r > 1.0) r = 1.0;
  return r;
}

__device__ __forceinline__ uint64_t wave_sum_u64(uint64_t v) {
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) v += __shfl_xor(v, o, 64);
  return v;
}

// Reference-order sequential fp64 sums for one sketch row (inexact regime).
__device__ void seq_row_sums(const uint32_t* a, const uint32_t* b, int w, double& A, double& B, double& AB) {
  A = 0.0;
  B = 0.0;
  AB = 0.0;
  for (int j = 0; j < w; ++j) {
    double xa = (double)a[j], xb = (double)b[j];
    A = __dadd_rn(A, __dmul_rn(xa, xa));
    B = __dadd_rn(B, __dmul_rn(xb, xb));
    AB = __dadd_rn(AB, __dmul_rn(xa, xb));
  }
}

// One workgroup (256 threads) per (query, target) pair.
__global__ __launch_bounds__(256) void k_pair_cosine(const uint32_t* table, const uint64_t* norm, const double* nsqrt,
                                                     HashParams hp, int64_t q_row, const int64_t* rows, int64_t m,
                                                     int64_t nrows, int weighted, double* out) {
  __shared__ uint64_t red[4];
  const int64_t t = blockIdx.x;
  if (t >= m) return;
  const int64_t r2 = rows[t];
  if (r2 < 0 || r2 >= nrows) {
    if (threadIdx.x == 0) out[t] = __builtin_nan("");
    return;
  }
  const int w = (int)hp.width;
  const int64_t dw = (int64_t)hp.depth * w;
  const uint32_t* pa = table + q_row * dw;
  const uint32_t* pb = table + r2 * dw;
  double minc = DBL_MAX;
  for (int d = 0; d < hp.depth; ++d) {
    const uint32_t* ra = pa + (int64_t)d * w;
    const uint32_t* rb = pb + (int64_t)d * w;
    const uint64_t Na = norm[q_row * hp.depth + d], Nb = norm[r2 * hp.depth + d];
    const bool exact = Na < (1ULL << 53) && Nb < (1ULL << 53);
    double valueAB, den;
    if (exact) {
      uint64_t dot = 0;
      if ((w & 3) == 0) {
        const uint4* a4 = reinterpret_cast<const uint4*>(ra);
        const uint4* b4 = reinterpret_cast<const uint4*>(rb);
        for (int j = threadIdx.x; j < (w >> 2); j += 256) {
          uint4 x = a4[j], y = b4[j];
          dot += (uint64_t)x.x * y.x + (uint64_t)x.y * y.y + (uint64_t)x.z * y.z + (uint64_t)x.w * y.w;
        }
      } else {
        for (int j = threadIdx.x; j < w; j += 256) dot += (uint64_t)ra[j] * rb[j];
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
      seq_row_sums(ra, rb, w, A, B, valueAB);  // every thread (uniform result)
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

int pair_cosines(cms_handle* h, int64_t q_row, const int64_t* d_rows, int64_t m, double* d_out) {
  if (m <= 0) return CMS_OK;
  TimedScope ts(h, "pair_cosine");
  hipLaunchKernelGGL(k_pair_cosine, dim3((unsigned)m), dim3(256), 0, h->stream, h->d_table, h->d_norm,
                     h->d_norm_sqrt, h->hp, q_row, d_rows, m, h->n, (int)h->p.weighting, d_out);
  CMS_HIP(hipGetLastError());
  return CMS_OK;
}

// DoubleCountMinSketch.get(key) (:94-103): min over rows, from Double.MAX_VALUE.
__global__ void k_point_query(const uint32_t* table, HashParams hp, int64_t row, const int64_t* keys, int64_t m,
                              double* out) {
  const int64_t dw = (int64_t)hp.depth * hp.width;
  for (int64_t i = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; i < m; i += (int64_t)gridDim.x * blockDim.x) {
    uint64_t kp = reduce_key(keys[i]);
    double est = DBL_MAX;
    for (int d = 0; d < hp.depth; ++d) {
      double v = (double)table[row * dw + (int64_t)d * hp.width + bucket(hp, d, kp)];
      if (v < est) est = v;
    }
    out[i] = est;
  }
}

int point_queries(cms_handle* h, int64_t row, const int64_t* d_keys, int64_t m, double* d_out) {
  if (m <= 0) return CMS_OK;
  unsigned grid = (unsigned)std::min<int64_t>((m + 255) / 256, 4096);
  hipLaunchKernelGGL(k_point_query, dim3(grid), dim3(256), 0, h->stream, h->d_table, h->hp, row, d_keys, m, d_out);
  CMS_HIP(hipGetLastError());
  return CMS_OK;
}

// ------------------------------------------------------------- top-k ----
// TopItems.getTopUsers (T/impl/recommender/TopItems.java:91-136) over
// candidates in ascending ID order, NaN skipped, ordered by SimilarUser
// (similarity desc, ID asc): the first k of that total order.  One
// workgroup per query: radix-select the k-th largest score key (8 x 8-bit
// digits), take every candidate above it plus the lowest-index ties, then a
// bitonic sort of <= 1024 survivors in LDS.

constexpr int kTopThreads = 1024;
constexpr int kTopMax = 1024;

__device__ __forceinline__ uint64_t score_key(double s) {
  if (s == 0.0) s = 0.0;  // -0.0 == +0.0 for SimilarUser.compareTo
  uint64_t u = (uint64_t)__double_as_longlong(s);
  return (u >> 63) ? ~u : (u | (1ULL << 63));
}

__global__ __launch_bounds__(kTopThreads) void k_top_k(const double* scores, int64_t ld, int64_t n, int32_t k,
                                                        int64_t row_begin, const int64_t* owner_ids, int64_t* out_ids,
                                                        double* out_scores, int32_t* counts) {
  __shared__ uint32_t hist[256];
  __shared__ uint64_t s_prefix;
  __shared__ uint32_t s_need;
  __shared__ uint64_t ckey[kTopMax];
  __shared__ int64_t cidx[kTopMax];
  __shared__ uint32_t s_cnt, s_ties_taken;
  __shared__ uint32_t wsum[kTopThreads / 64];

  const int64_t q = blockIdx.x;
  const double* sc = scores + q * ld;
  const int64_t self = row_begin + q;

  // count non-NaN candidates (self excluded: MostSimilarEstimator -> NaN)
  if (threadIdx.x == 0) {
    s_prefix = 0;
    s_cnt = 0;
    s_ties_taken = 0;
  }
  uint32_t valid = 0;
  for (int64_t j = threadIdx.x; j < n; j += kTopThreads) {
    double s = sc[j];
    valid += (j != self && s == s);
  }
  for (int o = 32; o > 0; o >>= 1) valid += __shfl_xor(valid, o, 64);
  if ((threadIdx.x & 63) == 0) wsum[threadIdx.x >> 6] = valid;
  __syncthreads();
  uint32_t nvalid = 0;
  for (int i = 0; i < kTopThreads / 64; ++i) nvalid += wsum[i];
  const uint32_t kk = (uint32_t)min<int64_t>(k, nvalid);
  if (threadIdx.x == 0) s_need = kk;  // rank (1-based) of the threshold among the largest
  __syncthreads();
  if (kk == 0) {
    if (threadIdx.x == 0) counts[q] = 0;
    return;
  }
  // radix select: find T = kk-th largest key, and how many keys are > T
  for (int shift = 56; shift >= 0; shift -= 8) {
    for (int i = threadIdx.x; i < 256; i += kTopThreads) hist[i] = 0;
    __syncthreads();
    const uint64_t pre = s_prefix;
    const uint64_t hmask = shift == 56 ? 0ULL : (~0ULL << (shift + 8));
    for (int64_t j = threadIdx.x; j < n; j += kTopThreads) {
      double s = sc[j];
      if (j == self || s != s) continue;
      uint64_t key = score_key(s);
      if ((key & hmask) == pre) atomicAdd(&hist[(key >> shift) & 255u], 1u);
    }
    __syncthreads();
    if (threadIdx.x == 0) {
      uint32_t need = s_need;
      int digit = 255;
      for (; digit > 0; --digit) {
        if (hist[digit] >= need) break;
        need -= hist[digit];
      }
      s_need = need;
      s_prefix = pre | ((uint64_t)digit << shift);
    }
    __syncthreads();
  }
  const uint64_t T = s_prefix;
  const uint32_t ties_needed = s_need;  // how many keys == T to take (lowest index first)
  // collect keys > T (fewer than kk), and the first ties_needed ties in index order
  for (int64_t base = 0; base < n; base += kTopThreads) {
    int64_t j = base + threadIdx.x;
    bool gt = false, tie = false;
    uint64_t key = 0;
    if (j < n) {
      double s = sc[j];
      if (j != self && s == s) {
        key = score_key(s);
        gt = key > T;
        tie = key == T;
      }
    }
    if (gt) {
      uint32_t pos = atomicAdd(&s_cnt, 1u);
      ckey[pos] = key;
      cidx[pos] = j;
    }
    // ordered tie compaction
    uint64_t bal = __ballot(tie);
    uint32_t lane_rank = __popcll(bal & ((1ULL << (threadIdx.x & 63)) - 1ULL));
    if ((threadIdx.x & 63) == 0) wsum[threadIdx.x >> 6] = __popcll(bal);
    __syncthreads();
    uint32_t before = s_ties_taken;
    for (int i = 0; i < (int)(threadIdx.x >> 6); ++i) before += wsum[i];
    if (tie && before + lane_rank < ties_needed) {
      uint32_t pos = atomicAdd(&s_cnt, 1u);
      ckey[pos] = key;
      cidx[pos] = j;
    }
    __syncthreads();
    if (threadIdx.x == 0) {
      uint32_t t = 0;
      for (int i = 0; i < kTopThreads / 64; ++i) t += wsum[i];
      s_ties_taken += t;
    }
    __syncthreads();
  }
  // bitonic sort of kk entries by (key desc, index asc), padded to pow2
  uint32_t P = 1;
  while (P < kk) P <<= 1;
  for (uint32_t i = kk + threadIdx.x; i < P; i += kTopThreads) {
    ckey[i] = 0;
    cidx[i] = INT64_MAX;
  }
  __syncthreads();
  for (uint32_t size = 2; size <= P; size <<= 1) {
    for (uint32_t stride = size >> 1; stride > 0; stride >>= 1) {
      for (uint32_t i = threadIdx.x; i < P; i += kTopThreads) {
        uint32_t jx = i ^ stride;
        if (jx > i) {
          bool up = ((i & size) == 0);
          // "before" = key larger, or equal key and smaller index
          bool i_before = ckey[i] > ckey[jx] || (ckey[i] == ckey[jx] && cidx[i] < cidx[jx]);
          if (up != i_before) {
            uint64_t tk = ckey[i];
            ckey[i] = ckey[jx];
            ckey[jx] = tk;
            int64_t ti = cidx[i];
            cidx[i] = cidx[jx];
            cidx[jx] = ti;
          }
        }
      }
      __syncthreads();
    }
  }
  for (uint32_t i = threadIdx.x; i < kk; i += kTopThreads) {
    int64_t j = cidx[i];
    out_ids[q * k + i] = owner_ids ? owner_ids[j] : j;
    out_scores[q * k + i] = sc[j];
  }
  if (threadIdx.x == 0) counts[q] = (int32_t)kk;
}

int top_k_slab(cms_handle* h, const double* slab, int64_t ld, int64_t first_row, int64_t count, int32_t k,
               int64_t* d_ids, double* d_scores, int32_t* d_counts) {
  TimedScope ts(h, "top_k");
  hipLaunchKernelGGL(k_top_k, dim3((unsigned)count), dim3(kTopThreads), 0, h->stream, slab, ld, h->n, k, first_row,
                     h->d_owner_ids, d_ids, d_scores, d_counts);
  CMS_HIP(hipGetLastError());
  return CMS_OK;
}

int top_k_rows(cms_handle* h, int64_t row_begin, int64_t row_count, int32_t k, int64_t* d_ids, double* d_scores,
               int32_t* d_counts) {
  if (k < 1 || k > kTopMax) return set_error(CMS_E_PARAM, "k must be in [1, %d]", kTopMax);
  const int64_t n = h->n;
  int rc = CMS_OK;
  if (mfma_eligible(h) && (rc = cosine_prepare(h))) return rc;
  if (mfma_eligible(h) && h->n_inexact_rows == 0) {
    // all-pairs MFMA slab for 128-aligned query blocks, then top-k per row
    const int64_t a0 = row_begin / 128 * 128, a1 = row_begin + row_count;
    const int64_t qb = std::max<int64_t>(128, ((int64_t(1) << 28) / std::max<int64_t>(1, n)) / 128 * 128);
    CMS_HIP(h->ws_slab.ensure(sizeof(double) * (size_t)(std::min(qb, a1 - a0) * n)));
    for (int64_t q0 = a0; q0 < a1; q0 += qb) {
      const int64_t qc = std::min(qb, a1 - q0);
      rc = cosine_slab(h, q0, qc, h->ws_slab.as<double>());
      if (rc) return rc;
      const int64_t f0 = std::max(q0, row_begin), f1 = std::min(q0 + qc, a1);
      rc = top_k_slab(h, h->ws_slab.as<double>() + (f0 - q0) * n, n, f0, f1 - f0, k, d_ids + (f0 - row_begin) * k,
                      d_scores + (f0 - row_begin) * k, d_counts + (f0 - row_begin));
      if (rc) return rc;
    }
    return CMS_OK;
  }
  // rows of the score slab per batch, bounded to ~1 GiB of fp64 scores
  int64_t qb = std::max<int64_t>(1, std::min<int64_t>(row_count, (int64_t(1) << 27) / std::max<int64_t>(1, n)));
  CMS_HIP(h->ws_out.ensure(sizeof(double) * (size_t)(qb * n)));
  CMS_HIP(h->ws_query.ensure(sizeof(int64_t) * (size_t)n));
  // target rows 0..n-1
  {
    std::vector<int64_t> all(n);
    for (int64_t i = 0; i < n; ++i) all[i] = i;
    CMS_HIP(hipMemcpyAsync(h->ws_query.ptr, all.data(), sizeof(int64_t) * n, hipMemcpyHostToDevice, h->stream));
    CMS_HIP(hipStreamSynchronize(h->stream));
  }
  for (int64_t r0 = 0; r0 < row_count; r0 += qb) {
    int64_t rc = std::min(qb, row_count - r0);
    for (int64_t q = 0; q < rc; ++q) {
      int e = pair_cosines(h, row_begin + r0 + q, h->ws_query.as<int64_t>(), n, h->ws_out.as<double>() + q * n);
      if (e) return e;
    }
    TimedScope ts(h, "top_k");
    hipLaunchKernelGGL(k_top_k, dim3((unsigned)rc), dim3(kTopThreads), 0, h->stream, h->ws_out.as<double>(), n, n, k,
                       row_begin + r0, h->d_owner_ids, d_ids + r0 * k, d_scores + r0 * k, d_counts + r0);
    CMS_HIP(hipGetLastError());
  }
  return CMS_OK;
}

}  // namespace cms
