// cms_f64.hip -- fp64 counters (CMS_COUNTER_F64): the reference's own counter
// type for arbitrary float preferences, negative and non-dyadic ones included.
//
// DoubleCountMinSketch keeps fp64 counters and adds (double) float prefs in
// the order its PreferenceArray hands them over (T/impl/common/
// DoubleCountMinSketch.java:72-80, fed by CosineCM.exportProfile :41-58, i.e.
// the DataModel's per-owner order).  fp64 addition is not associative, so this
// mode reproduces that order exactly instead of the integer fast paths:
//   - the row build walks each owner's keys in CSR order; in LDS every bucket
//     has exactly one owning thread, which applies that bucket's increments in
//     key order (count[j] += inc, one rounding per update, as in Java);
//   - valueA = sum_j x_j^2 per (owner, sketch row) is one sequential fp64 chain
//     in j order (DoubleCountMinSketch.cosine :131-138), kept as Math.sqrt(valueA);
//   - valueAB is the same sequential chain per pair and row, then the epilogue
//     den = sqrt(A) * sqrt(B), AB / den, Math.min over rows (NaN and -0.0 rules
//     included), normalizeWeightResult -- every operation IEEE round-to-nearest,
//     no FMA contraction (-ffp-contract=off), as the JVM computes it.
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cfloat>
#include <vector>

#include "cms_device.h"
#include "cms_internal.h"

namespace cms {

constexpr int kF64Threads = 256;
constexpr int kF64Chunk = 2048;  // keys staged per LDS round

// One workgroup per owner row.  LDS: the current sketch row [w] fp64, plus a
// staged chunk of (bucket, increment) pairs.  Thread t owns buckets j with
// j % 256 == t and walks the chunk in key order, so each counter receives its
// increments in exactly the reference's order.  Rows wider than the LDS holds
// (in_lds == 0: w > 16384) are updated in place in the table: the owning
// thread's loads and stores of a bucket are in program order, so the order of
// the adds -- and every rounding -- is the same.
__global__ __launch_bounds__(kF64Threads) void k_f64_build(const int64_t* off, const int64_t* keys, const float* vals,
                                                           int64_t nrows, HashParams hp, int accumulate, int in_lds,
                                                           double* tab) {
  extern __shared__ __align__(16) unsigned char smem[];
  const int w = (int)hp.width;
  double* lrow = reinterpret_cast<double*>(smem);                      // [w] (in_lds)
  double* cv = lrow + (in_lds ? w : 0);                                // [kF64Chunk]
  uint32_t* cb = reinterpret_cast<uint32_t*>(cv + kF64Chunk);         // [kF64Chunk]
  const int tid = threadIdx.x;
  for (int64_t r = blockIdx.x; r < nrows; r += gridDim.x) {
    const int64_t lo = off[r], hi = off[r + 1];
    if (hi <= lo && accumulate) continue;  // nothing to add to this owner
    double* dst = tab + r * (int64_t)hp.depth * w;
    for (int d = 0; d < hp.depth; ++d) {
      double* row = in_lds ? lrow : dst + (int64_t)d * w;
      if (in_lds)
        for (int j = tid; j < w; j += kF64Threads) row[j] = accumulate ? dst[(int64_t)d * w + j] : 0.0;
      for (int64_t c0 = lo; c0 < hi; c0 += kF64Chunk) {
        const int cnt = (int)min<int64_t>(kF64Chunk, hi - c0);
        __syncthreads();  // the previous chunk is consumed
        for (int i = tid; i < cnt; i += kF64Threads) {
          cb[i] = bucket(hp, d, reduce_key(keys[c0 + i]));
          cv[i] = vals ? (double)vals[c0 + i] : 1.0;
        }
        __syncthreads();
        for (int i = 0; i < cnt; ++i) {
          const uint32_t b = cb[i];  // uniform across the workgroup: an LDS broadcast
          if ((int)(b % kF64Threads) == tid) row[b] = __dadd_rn(row[b], cv[i]);
        }
      }
      __syncthreads();
      if (in_lds)
        for (int j = tid; j < w; j += kF64Threads) dst[(int64_t)d * w + j] = row[j];
      __syncthreads();
    }
  }
}

// Math.sqrt of the sequential valueA of every (owner, sketch row).
__global__ void k_f64_norms(const double* tab, int64_t cells, int w, double* nsqrt) {
  for (int64_t c = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; c < cells; c += (int64_t)gridDim.x * blockDim.x) {
    const double* x = tab + c * w;
    double a = 0.0;
    for (int j = 0; j < w; ++j) a = __dadd_rn(a, __dmul_rn(x[j], x[j]));
    nsqrt[c] = __dsqrt_rn(a);
  }
}

// CosineCM.userSimilarity of owner rows (qa, qb): the reference's loop.
__device__ double f64_cosine_cm(const double* tab, const double* nsqrt, int64_t qa, int64_t qb, int depth, int w,
                                int weighted) {
  const int64_t dw = (int64_t)depth * w;
  double minc = DBL_MAX;
  for (int d = 0; d < depth; ++d) {
    const double* xa = tab + qa * dw + (int64_t)d * w;
    const double* xb = tab + qb * dw + (int64_t)d * w;
    double ab = 0.0;
    for (int j = 0; j < w; ++j) ab = __dadd_rn(ab, __dmul_rn(xa[j], xb[j]));
    const double den = __dmul_rn(nsqrt[qa * depth + d], nsqrt[qb * depth + d]);
    if (den != 0.0) minc = java_min(minc, __ddiv_rn(ab, den));
  }
  double r = minc == DBL_MAX ? __builtin_nan("") : minc;
  if (r == r) r = normalize_weight(r, weighted);
  return r;
}

// similarities of (q_row, rows[i]) into out[i]; an unknown row gives NaN
__global__ void k_f64_pairs(const double* tab, const double* nsqrt, int depth, int w, int64_t q_row,
                            const int64_t* rows, int64_t m, int64_t nrows, int weighted, double* out) {
  for (int64_t i = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; i < m; i += (int64_t)gridDim.x * blockDim.x) {
    const int64_t r = rows[i];
    out[i] = (r < 0 || r >= nrows) ? __builtin_nan("") : f64_cosine_cm(tab, nsqrt, q_row, r, depth, w, weighted);
  }
}

// slab[q][c] = similarity(q0 + q, c) for q < qc, every owner c
__global__ void k_f64_slab(const double* tab, const double* nsqrt, int depth, int w, int64_t q0, int64_t qc,
                           int64_t n, int weighted, double* slab) {
  const int64_t total = qc * n;
  for (int64_t i = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; i < total; i += (int64_t)gridDim.x * blockDim.x) {
    const int64_t q = i / n, c = i - q * n;
    slab[i] = f64_cosine_cm(tab, nsqrt, q0 + q, c, depth, w, weighted);
  }
}

// DoubleCountMinSketch.get(key) (:94-103) on fp64 counters
__global__ void k_f64_point(const double* tab, HashParams hp, int64_t row, const int64_t* keys, int64_t m,
                            double* out) {
  const int64_t dw = (int64_t)hp.depth * hp.width;
  for (int64_t i = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; i < m; i += (int64_t)gridDim.x * blockDim.x) {
    const uint64_t kp = reduce_key(keys[i]);
    double est = DBL_MAX;
    for (int d = 0; d < hp.depth; ++d) {
      const double v = tab[row * dw + (int64_t)d * hp.width + bucket(hp, d, kp)];
      if (v < est) est = v;
    }
    out[i] = est;
  }
}

// doEstimatePreference (GenericUserBasedRecommender.java:134-184) on fp64
// counters: the k_estimate loop with the point query read as doubles
__global__ void k_f64_estimate(const double* tab, HashParams hp, int64_t user_row, const int64_t* nb_rows,
                               const double* sims, int64_t m, const int64_t* items, int64_t q, int use_capper,
                               float lo, float hi, float* out) {
  const int64_t dw = (int64_t)hp.depth * hp.width;
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
        const double v = tab[r * dw + bk[d]];
        if (v < est) est = v;
      }
      const float pref = (float)est;
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

// ---------------------------------------------- per-owner shapes, fp64 --
// CosineCM with CountMinSketchConfig (cms_create_per_owner) on fp64 counters:
// the DataModel stays resident as (key mod p, (double) pref) in CSR order.

__global__ void k_po_prep64(const int64_t* key, const float* val, int64_t np, uint64_t* kp, double* v64) {
  for (int64_t i = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; i < np; i += (int64_t)gridDim.x * blockDim.x) {
    kp[i] = reduce_key(key[i]);
    v64[i] = val ? (double)val[i] : 1.0;
  }
}

// Sketch row d of owner u's preferences [k0, k1) at shape (w, barrett) added
// into row[] (global or LDS) in key order: bucket b belongs to thread b % 256.
__device__ void f64_row_updates(const uint64_t* kp, const double* v64, int64_t k0, int64_t k1, HashParams hp, int d,
                                uint32_t w, uint64_t barrett, double* row, uint32_t* cb, double* cv) {
  const int tid = threadIdx.x;
  for (int64_t c0 = k0; c0 < k1; c0 += kF64Chunk) {
    const int cnt = (int)min<int64_t>(kF64Chunk, k1 - c0);
    __syncthreads();
    for (int i = tid; i < cnt; i += kF64Threads) {
      cb[i] = bucket_wb(hp, d, kp[c0 + i], w, barrett);
      cv[i] = v64[c0 + i];
    }
    __syncthreads();
    for (int i = 0; i < cnt; ++i) {
      const uint32_t b = cb[i];
      if ((int)(b % kF64Threads) == tid) row[b] = __dadd_rn(row[b], cv[i]);
    }
  }
  __syncthreads();
}

// own sketches (getExportedCMProfile, CosineCM.java:60-67) into the zeroed
// ragged fp64 array, and Math.sqrt of each row's sequential valueB
__global__ __launch_bounds__(kF64Threads) void k_po_f64_build(const int64_t* off, const uint64_t* kp, const double* v64,
                                                              const PoShape* shp, HashParams hp, int64_t n,
                                                              double* sk, double* nsq) {
  __shared__ uint32_t cb[kF64Chunk];
  __shared__ double cv[kF64Chunk];
  for (int64_t r = blockIdx.x; r < n; r += gridDim.x) {
    const PoShape s = shp[r];
    if (s.w <= 0) continue;
    for (int d = 0; d < s.d; ++d) {
      double* row = sk + s.soff + (int64_t)d * s.w;
      f64_row_updates(kp, v64, off[r], off[r + 1], hp, d, (uint32_t)s.w, s.barrett, row, cb, cv);
      if (threadIdx.x == 0) {
        __threadfence_block();
        double a = 0.0;
        for (int j = 0; j < s.w; ++j) a = __dadd_rn(a, __dmul_rn(row[j], row[j]));
        nsq[s.roff + d] = __dsqrt_rn(a);
      }
      __syncthreads();
    }
  }
}

// userSimilarity(u1 = qrows[t / m], u2 = crows[t % m]) on fp64 counters: u1's
// sketch built at u2's shape (exportProfile, CosineCM.java:41-58,86) one row at
// a time in a zeroed scratch row, then the reference's sequential loop.
__global__ __launch_bounds__(kF64Threads) void k_po_f64_pairs(const int64_t* off, const uint64_t* kp, const double* v64,
                                                              const PoShape* shp, const double* sk, const double* nsq,
                                                              HashParams hp, const int64_t* qrows, int64_t nq,
                                                              const int64_t* crows, int64_t m, double* scratch,
                                                              int64_t scratch_w, int weighted, double* out) {
  __shared__ uint32_t cb[kF64Chunk];
  __shared__ double cv[kF64Chunk];
  __shared__ double s_min;
  double* row = scratch + (int64_t)blockIdx.x * scratch_w;
  const int64_t total = nq * m;
  for (int64_t t = blockIdx.x; t < total; t += gridDim.x) {
    const int64_t u1 = qrows[t / m];
    const int64_t c = t % m;
    const int64_t u2 = crows ? crows[c] : c;
    const PoShape s = shp[u2];
    if (threadIdx.x == 0) s_min = DBL_MAX;
    for (int d = 0; d < s.d; ++d) {
      for (int j = threadIdx.x; j < s.w; j += kF64Threads) row[j] = 0.0;
      f64_row_updates(kp, v64, off[u1], off[u1 + 1], hp, d, (uint32_t)s.w, s.barrett, row, cb, cv);
      if (threadIdx.x == 0) {
        __threadfence_block();
        const double* xb = sk + s.soff + (int64_t)d * s.w;
        double A = 0.0, AB = 0.0;
        for (int j = 0; j < s.w; ++j) {
          A = __dadd_rn(A, __dmul_rn(row[j], row[j]));
          AB = __dadd_rn(AB, __dmul_rn(row[j], xb[j]));
        }
        const double den = __dmul_rn(__dsqrt_rn(A), nsq[s.roff + d]);
        if (den != 0.0) s_min = java_min(s_min, __ddiv_rn(AB, den));
      }
      __syncthreads();
    }
    if (threadIdx.x == 0) {
      double r = s_min == DBL_MAX ? __builtin_nan("") : s_min;
      if (r == r) r = normalize_weight(r, weighted);
      out[t] = r;
    }
    __syncthreads();
  }
}

__global__ void k_po_f64_point(const PoShape* shp, const double* sk, HashParams hp, int64_t row, const int64_t* keys,
                               int64_t m, double* out) {
  const PoShape s = shp[row];
  for (int64_t i = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; i < m; i += (int64_t)gridDim.x * blockDim.x) {
    const uint64_t kp = reduce_key(keys[i]);
    double est = DBL_MAX;
    for (int d = 0; d < s.d; ++d) {
      const double v = sk[s.soff + (int64_t)d * s.w + bucket_wb(hp, d, kp, (uint32_t)s.w, s.barrett)];
      if (v < est) est = v;
    }
    out[i] = est;
  }
}

__global__ void k_po_f64_estimate(const PoShape* shp, const double* sk, HashParams hp, int64_t user_row,
                                  const int64_t* nb_rows, const double* sims, int64_t m, const int64_t* items,
                                  int64_t q, int use_capper, float lo, float hi, float* out) {
  for (int64_t i = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; i < q; i += (int64_t)gridDim.x * blockDim.x) {
    const uint64_t kp = reduce_key(items[i]);
    double preference = 0.0, total = 0.0;
    int count = 0;
    for (int64_t j = 0; j < m; ++j) {
      const int64_t r = nb_rows[j];
      if (r == user_row) continue;
      const PoShape s = shp[r];
      double est = DBL_MAX;
      for (int d = 0; d < s.d; ++d) {
        const double v = sk[s.soff + (int64_t)d * s.w + bucket_wb(hp, d, kp, (uint32_t)s.w, s.barrett)];
        if (v < est) est = v;
      }
      const float pref = (float)est;
      if (pref == 0.0f) continue;
      const double sim = sims[j];
      if (sim != sim) continue;
      preference = __dadd_rn(preference, __dmul_rn(sim, (double)pref));
      total = __dadd_rn(total, sim);
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

static unsigned grid_for(int64_t work) {
  return (unsigned)std::max<int64_t>(1, std::min<int64_t>((work + 255) / 256, 8192));
}

int f64_ingest_csr(cms_handle* h, const int64_t* d_off, const int64_t* d_key, const float* d_val) {
  const int accumulate = h->empty ? 0 : 1;
  const size_t chunk_lds = (sizeof(double) + sizeof(uint32_t)) * kF64Chunk;
  const int in_lds = sizeof(double) * (size_t)h->p.width + chunk_lds <= 160 * 1024 ? 1 : 0;
  const size_t lds = (in_lds ? sizeof(double) * (size_t)h->p.width : 0) + chunk_lds;
  static bool attr = [] {
    (void)hipFuncSetAttribute((const void*)k_f64_build, hipFuncAttributeMaxDynamicSharedMemorySize, 160 * 1024);
    return true;
  }();
  (void)attr;
  if (h->empty) {
    CMS_HIP(hipMemsetAsync(h->d_t64, 0, sizeof(double) * (size_t)h->n * (size_t)h->dw, h->stream));
  }
  TimedScope ts(h, "build_rows");
  hipLaunchKernelGGL(k_f64_build, dim3((unsigned)std::min<int64_t>(h->n, 65536)), dim3(kF64Threads), lds, h->stream,
                     d_off, d_key, d_val, h->n, h->hp, 1, in_lds, h->d_t64);
  (void)accumulate;  // the table was zeroed above, so every build accumulates
  CMS_HIP(hipGetLastError());
  h->empty = false;
  h->norms_valid = false;
  return CMS_OK;
}

// COO pairs from host memory, owners by ID: grouped by owner on the host,
// stable, so each owner's increments keep the stream order (all-or-nothing:
// an unknown owner rejects the batch before the table is touched).
int f64_ingest_coo_host(cms_handle* h, const int64_t* owner, const int64_t* key, const float* val, int64_t np) {
  const int64_t n = h->n;
  std::vector<int64_t> rows(np);
  const bool by_id = !h->h_owner_ids.empty();
  for (int64_t i = 0; i < np; ++i) {
    int64_t r = owner[i];
    if (by_id) {
      auto it = std::lower_bound(h->h_owner_ids.begin(), h->h_owner_ids.end(), owner[i]);
      if (it == h->h_owner_ids.end() || *it != owner[i])
        return set_error(CMS_E_NO_SUCH_ID, "no such owner ID %lld", (long long)owner[i]);
      r = it - h->h_owner_ids.begin();
    } else if (r < 0 || r >= n) {
      return set_error(CMS_E_PARAM, "owner row outside [0, num_owners)");
    }
    rows[i] = r;
  }
  std::vector<int64_t> off(n + 1, 0), ck(np);
  std::vector<float> cv(val ? np : 0);
  for (int64_t i = 0; i < np; ++i) ++off[rows[i] + 1];
  for (int64_t r = 0; r < n; ++r) off[r + 1] += off[r];
  std::vector<int64_t> cur(off.begin(), off.end() - 1);
  for (int64_t i = 0; i < np; ++i) {
    const int64_t p = cur[rows[i]]++;
    ck[p] = key[i];
    if (val) cv[p] = val[i];
  }
  CMS_HIP(h->ws_in_row.ensure(sizeof(int64_t) * (size_t)(n + 1)));
  CMS_HIP(h->ws_in_key.ensure(sizeof(int64_t) * (size_t)np));
  if (val) CMS_HIP(h->ws_in_val.ensure(sizeof(float) * (size_t)np));
  CMS_HIP(hipMemcpyAsync(h->ws_in_row.ptr, off.data(), sizeof(int64_t) * (n + 1), hipMemcpyHostToDevice, h->stream));
  CMS_HIP(hipMemcpyAsync(h->ws_in_key.ptr, ck.data(), sizeof(int64_t) * np, hipMemcpyHostToDevice, h->stream));
  if (val) CMS_HIP(hipMemcpyAsync(h->ws_in_val.ptr, cv.data(), sizeof(float) * np, hipMemcpyHostToDevice, h->stream));
  int rc = f64_ingest_csr(h, h->ws_in_row.as<int64_t>(), h->ws_in_key.as<int64_t>(),
                          val ? h->ws_in_val.as<float>() : nullptr);
  if (rc) return rc;
  CMS_HIP(hipStreamSynchronize(h->stream));  // the host staging vectors die on return
  h->finalized = false;
  h->pairs_ingested += np;
  return CMS_OK;
}

int f64_norms(cms_handle* h) {
  const int64_t cells = h->n * h->p.depth;
  TimedScope ts(h, "norms");
  hipLaunchKernelGGL(k_f64_norms, dim3(grid_for(cells)), dim3(256), 0, h->stream, h->d_t64, cells, h->p.width,
                     h->d_norm_sqrt);
  CMS_HIP(hipGetLastError());
  h->norms_valid = true;
  return CMS_OK;
}

int f64_pair_cosines(cms_handle* h, int64_t q_row, const int64_t* d_rows, int64_t m, double* d_out, hipStream_t s) {
  if (m <= 0) return CMS_OK;
  TimedScope ts(h, "pair_cosine", s == nullptr);
  hipLaunchKernelGGL(k_f64_pairs, dim3(grid_for(m)), dim3(256), 0, s ? s : h->stream, h->d_t64, h->d_norm_sqrt, h->p.depth,
                     h->p.width, q_row, d_rows, m, h->n, (int)h->p.weighting, d_out);
  CMS_HIP(hipGetLastError());
  return CMS_OK;
}

int f64_slab(cms_handle* h, int64_t q0, int64_t qc, double* d_slab) {
  if (qc <= 0) return CMS_OK;
  TimedScope ts(h, "pair_cosine");
  hipLaunchKernelGGL(k_f64_slab, dim3(grid_for(qc * h->n)), dim3(256), 0, h->stream, h->d_t64, h->d_norm_sqrt,
                     h->p.depth, h->p.width, q0, qc, h->n, (int)h->p.weighting, d_slab);
  CMS_HIP(hipGetLastError());
  return CMS_OK;
}

int f64_point_queries(cms_handle* h, int64_t row, const int64_t* d_keys, int64_t m, double* d_out, hipStream_t s) {
  if (m <= 0) return CMS_OK;
  hipLaunchKernelGGL(k_f64_point, dim3(grid_for(m)), dim3(256), 0, s ? s : h->stream, h->d_t64, h->hp, row, d_keys, m, d_out);
  CMS_HIP(hipGetLastError());
  return CMS_OK;
}

int f64_estimate_preferences(cms_handle* h, int64_t user_row, const int64_t* d_nb_rows, const double* d_sims,
                             int64_t m, const int64_t* d_items, int64_t q, int use_capper, float lo, float hi,
                             float* d_out, hipStream_t s) {
  if (q <= 0) return CMS_OK;
  hipLaunchKernelGGL(k_f64_estimate, dim3(grid_for(q)), dim3(256), 0, s ? s : h->stream, h->d_t64, h->hp, user_row, d_nb_rows,
                     d_sims, m, d_items, q, use_capper, lo, hi, d_out);
  CMS_HIP(hipGetLastError());
  return CMS_OK;
}

}  // namespace cms

namespace cms {

// pair-kernel workgroups, each with a scratch row of po_max_w doubles (at most 2 GiB of scratch)
static int64_t po_f64_grid(cms_handle* h) {
  const int64_t w = std::max(1, h->po_max_w);
  return std::max<int64_t>(1, std::min<int64_t>(4096, (int64_t(1) << 31) / (8 * w)));
}

int po_f64_load(cms_handle* h, const int64_t* d_key, const float* d_val, int64_t npairs) {
  CMS_HIP(h->po_kp.ensure(sizeof(uint64_t) * std::max<int64_t>(npairs, 1)));
  CMS_HIP(h->po_v64.ensure(sizeof(double) * std::max<int64_t>(npairs, 1)));
  if (npairs > 0)
    hipLaunchKernelGGL(k_po_prep64, dim3(grid_for(npairs)), dim3(256), 0, h->stream, d_key, d_val, npairs,
                       h->po_kp.as<uint64_t>(), h->po_v64.as<double>());
  CMS_HIP(hipGetLastError());
  return CMS_OK;
}

int po_f64_finalize(cms_handle* h, int64_t total_counters, int64_t total_rows) {
  CMS_HIP(h->po_sk.ensure(sizeof(double) * std::max<int64_t>(total_counters, 1)));
  CMS_HIP(h->po_nsq.ensure(sizeof(double) * std::max<int64_t>(total_rows, 1)));
  CMS_HIP(hipMemsetAsync(h->po_sk.ptr, 0, sizeof(double) * std::max<int64_t>(total_counters, 1), h->stream));
  TimedScope ts(h, "po_build");
  hipLaunchKernelGGL(k_po_f64_build, dim3((unsigned)std::max<int64_t>(1, std::min<int64_t>(h->n, 65536))),
                     dim3(kF64Threads), 0, h->stream, h->po_off.as<int64_t>(), h->po_kp.as<uint64_t>(),
                     h->po_v64.as<double>(), h->po_shape.as<PoShape>(), h->hp, h->n, h->po_sk.as<double>(),
                     h->po_nsq.as<double>());
  CMS_HIP(hipGetLastError());
  CMS_HIP(h->po_scratch.ensure(sizeof(double) * (size_t)po_f64_grid(h) * (size_t)std::max(1, h->po_max_w)));
  return CMS_OK;
}

int po_f64_pair_cosines(cms_handle* h, const int64_t* d_qrows, int64_t nq, const int64_t* d_crows, int64_t m,
                        double* d_out, hipStream_t s) {
  (void)s;  // exclusive callers only: the workgroups' scratch rows belong to the handle
  TimedScope ts(h, "po_pair_cosine");
  const unsigned grid = (unsigned)std::max<int64_t>(1, std::min<int64_t>(nq * m, po_f64_grid(h)));
  hipLaunchKernelGGL(k_po_f64_pairs, dim3(grid), dim3(kF64Threads), 0, h->stream, h->po_off.as<int64_t>(),
                     h->po_kp.as<uint64_t>(), h->po_v64.as<double>(), h->po_shape.as<PoShape>(), h->po_sk.as<double>(),
                     h->po_nsq.as<double>(), h->hp, d_qrows, nq, d_crows, m, h->po_scratch.as<double>(),
                     (int64_t)std::max(1, h->po_max_w), (int)(h->p.weighting == CMS_WEIGHTED), d_out);
  CMS_HIP(hipGetLastError());
  return CMS_OK;
}

int po_f64_point_queries(cms_handle* h, int64_t row, const int64_t* d_keys, int64_t m, double* d_out, hipStream_t s) {
  hipLaunchKernelGGL(k_po_f64_point, dim3(grid_for(m)), dim3(256), 0, s ? s : h->stream, h->po_shape.as<PoShape>(),
                     h->po_sk.as<double>(), h->hp, row, d_keys, m, d_out);
  CMS_HIP(hipGetLastError());
  return CMS_OK;
}

int po_f64_estimate_preferences(cms_handle* h, int64_t user_row, const int64_t* d_nb_rows, const double* d_sims,
                                int64_t m, const int64_t* d_items, int64_t q, int use_capper, float lo, float hi,
                                float* d_out, hipStream_t s) {
  hipLaunchKernelGGL(k_po_f64_estimate, dim3(grid_for(q)), dim3(256), 0, s ? s : h->stream, h->po_shape.as<PoShape>(),
                     h->po_sk.as<double>(), h->hp, user_row, d_nb_rows, d_sims, m, d_items, q, use_capper, lo, hi,
                     d_out);
  CMS_HIP(hipGetLastError());
  return CMS_OK;
}

}  // namespace cms
