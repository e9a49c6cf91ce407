// cms_topk.hip -- per-owner top-k over a similarity slab on gfx950.
//
// TopItems.getTopUsers (T/impl/recommender/TopItems.java:91-136) iterates the
// candidate owners in ascending ID order, skips NaN (self included, via
// MostSimilarEstimator, GenericUserBasedRecommender.java:231-247) and keeps
// the first k of the total order SimilarUser.compareTo defines
// (T/impl/recommender/SimilarUser.java:62-78): similarity descending, ID
// ascending.  One workgroup per query row:
//   1. radix select (8 x 8-bit digits) of the k-th largest similarity key;
//   2. when more candidates tie at that key than are needed, a second radix
//      select over the OWNER ROW of the tied candidates (the slab columns may
//      be permuted, so column order is not ID order);
//   3. gather the survivors into LDS and bitonic-sort them by (key desc, row asc).
#include <hip/hip_runtime.h>

#include <algorithm>
#include <vector>

#include "cms_internal.h"

namespace cms {

constexpr int kTopThreads = 1024;
constexpr int kTopMax = 1024;

__device__ __forceinline__ uint64_t score_key(double s) {
  if (s == 0.0) s = 0.0;  // -0.0 == +0.0 under SimilarUser.compareTo
  uint64_t u = (uint64_t)__double_as_longlong(s);
  return (u >> 63) ? ~u : (u | (1ULL << 63));
}


__device__ __forceinline__ uint32_t block_count(uint32_t v, uint32_t* wsum) {
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) v += __shfl_xor(v, o, 64);
  __syncthreads();
  if ((threadIdx.x & 63) == 0) wsum[threadIdx.x >> 6] = v;
  __syncthreads();
  uint32_t t = 0;
  for (int i = 0; i < kTopThreads / 64; ++i) t += wsum[i];
  return t;
}

__global__ __launch_bounds__(kTopThreads) void k_top_k(const double* slab, int64_t ld, int64_t n, int32_t k,
                                                        const TopQuery* queries, const int64_t* perm,
                                                        const int64_t* owner_ids, int64_t* out_ids,
                                                        double* out_scores, int32_t* counts) {
  __shared__ uint32_t hist[256];
  __shared__ uint64_t s_prefix;
  __shared__ uint32_t s_need, s_tied;
  __shared__ uint64_t ckey[kTopMax];
  __shared__ int64_t crow[kTopMax];
  __shared__ int64_t ccol[kTopMax];
  __shared__ uint32_t s_cnt;
  __shared__ uint32_t wsum[kTopThreads / 64];

  const TopQuery Q = queries[blockIdx.x];
  const double* sc = slab + Q.slab_row * ld;
  const int tid = threadIdx.x;
  auto row_of = [&](int64_t j) -> int64_t { return perm ? perm[j] : j; };

  uint32_t valid = 0;
  for (int64_t j = tid; j < n; j += kTopThreads) {
    const double s = sc[j];
    valid += (j != Q.self_col && s == s);
  }
  const uint32_t nvalid = block_count(valid, wsum);
  const uint32_t kk = (uint32_t)min<int64_t>(k, nvalid);
  if (kk == 0) {
    if (tid == 0) counts[Q.out_pos] = 0;
    return;
  }
  if (tid == 0) {
    s_prefix = 0;
    s_need = kk;
    s_cnt = 0;
  }
  __syncthreads();
  // ---- 1. k-th largest key T; s_need = how many keys == T to take ----
  for (int shift = 56; shift >= 0; shift -= 8) {
    for (int i = tid; i < 256; i += kTopThreads) hist[i] = 0;
    __syncthreads();
    const uint64_t pre = s_prefix;
    const uint64_t hmask = shift == 56 ? 0ULL : (~0ULL << (shift + 8));
    for (int64_t j = tid; j < n; j += kTopThreads) {
      const double s = sc[j];
      if (j == Q.self_col || s != s) continue;
      const uint64_t key = score_key(s);
      if ((key & hmask) == pre) atomicAdd(&hist[(key >> shift) & 255u], 1u);
    }
    __syncthreads();
    if (tid == 0) {
      uint32_t need = s_need;
      int digit = 255;
      for (; digit > 0; --digit) {
        if (hist[digit] >= need) break;
        need -= hist[digit];
      }
      s_need = need;
      s_prefix = pre | ((uint64_t)digit << shift);
      if (shift == 0) s_tied = hist[digit];
    }
    __syncthreads();
  }
  const uint64_t T = s_prefix;
  const uint32_t ties_needed = s_need;
  const uint32_t ties_total = s_tied;
  __syncthreads();  // every thread holds T before step 2 reuses s_prefix / s_need
  // ---- 2. among keys == T, the ties_needed-th smallest owner row R ----
  uint64_t R = ~0ULL;
  if (ties_needed < ties_total) {
    if (tid == 0) s_prefix = 0;
    __syncthreads();
    for (int shift = 56; shift >= 0; shift -= 8) {
      for (int i = tid; i < 256; i += kTopThreads) hist[i] = 0;
      __syncthreads();
      const uint64_t pre = s_prefix;
      const uint64_t hmask = shift == 56 ? 0ULL : (~0ULL << (shift + 8));
      for (int64_t j = tid; j < n; j += kTopThreads) {
        const double s = sc[j];
        if (j == Q.self_col || s != s || score_key(s) != T) continue;
        const uint64_t rk = (uint64_t)row_of(j);
        if ((rk & hmask) == pre) atomicAdd(&hist[(rk >> shift) & 255u], 1u);
      }
      __syncthreads();
      if (tid == 0) {
        uint32_t need = s_need;  // smallest-first: walk digits upward
        int digit = 0;
        for (; digit < 255; ++digit) {
          if (hist[digit] >= need) break;
          need -= hist[digit];
        }
        s_need = need;
        s_prefix = pre | ((uint64_t)digit << shift);
      }
      __syncthreads();
    }
    R = s_prefix;
  }
  // ---- 3. gather: keys > T, and ties with owner row <= R ----
  for (int64_t j = tid; j < n; j += kTopThreads) {
    const double s = sc[j];
    if (j == Q.self_col || s != s) continue;
    const uint64_t key = score_key(s);
    if (key < T) continue;
    const int64_t rw = row_of(j);
    if (key == T && (uint64_t)rw > R) continue;
    const uint32_t pos = atomicAdd(&s_cnt, 1u);
    if (pos < kTopMax) {
      ckey[pos] = key;
      crow[pos] = rw;
      ccol[pos] = j;
    }
  }
  __syncthreads();
  uint32_t P = 1;
  while (P < kk) P <<= 1;
  for (uint32_t i = kk + tid; i < P; i += kTopThreads) {
    ckey[i] = 0;
    crow[i] = INT64_MAX;
  }
  __syncthreads();
  for (uint32_t size = 2; size <= P; size <<= 1) {
    for (uint32_t stride = size >> 1; stride > 0; stride >>= 1) {
      for (uint32_t i = tid; i < P; i += kTopThreads) {
        const uint32_t jx = i ^ stride;
        if (jx > i) {
          const bool up = (i & size) == 0;
          const bool i_first = ckey[i] > ckey[jx] || (ckey[i] == ckey[jx] && crow[i] < crow[jx]);
          if (up != i_first) {
            uint64_t tk = ckey[i];
            ckey[i] = ckey[jx];
            ckey[jx] = tk;
            int64_t tr = crow[i];
            crow[i] = crow[jx];
            crow[jx] = tr;
            int64_t tc = ccol[i];
            ccol[i] = ccol[jx];
            ccol[jx] = tc;
          }
        }
      }
      __syncthreads();
    }
  }
  for (uint32_t i = tid; i < kk; i += kTopThreads) {
    out_ids[Q.out_pos * k + i] = owner_ids ? owner_ids[crow[i]] : crow[i];
    out_scores[Q.out_pos * k + i] = sc[ccol[i]];
  }
  if (tid == 0) counts[Q.out_pos] = (int32_t)kk;
}

// ---- one-pass top-k: sampled threshold, candidate gather, LDS sort ----
// bucket(s) is monotone in s, so every score in a bucket >= t outranks every
// score below it: the first k of the candidates with bucket >= t (sorted by
// the same total order) are the first k of the row whenever at least k
// candidates exist.  t comes from a 1/32 sample of the row, aiming at ~2k+64
// candidates; rows where the guess misses (fewer than k, or more than
// kCand) are flagged with count -1 and redone by k_top_k.
constexpr int kBins = 4096;
constexpr int kCand = 2048;
constexpr int kSampleSeg = 256;  // sample = one 256-column segment in every 32

__device__ __forceinline__ int score_bucket(double s) {
  const int b = (int)((s + 1.0) * (kBins / 2));
  return b < 0 ? 0 : (b >= kBins ? kBins - 1 : b);
}

__global__ __launch_bounds__(kTopThreads) void k_top_k_fast(const double* slab, int64_t ld, int64_t n, int32_t k,
                                                             const TopQuery* queries, const int64_t* perm,
                                                             const int64_t* owner_ids, int64_t* out_ids,
                                                             double* out_scores, int32_t* counts) {
  __shared__ uint32_t hist[kBins];
  __shared__ uint64_t ckey[kCand];
  __shared__ uint32_t crow[kCand];
  __shared__ uint32_t ccol[kCand];
  __shared__ uint32_t wsum[kTopThreads / 64];
  __shared__ uint32_t s_cnt;
  __shared__ int s_t;

  const TopQuery Q = queries[blockIdx.x];
  const double* sc = slab + Q.slab_row * ld;
  const int tid = threadIdx.x;
  for (int i = tid; i < kBins; i += kTopThreads) hist[i] = 0;
  if (tid == 0) s_cnt = 0;
  __syncthreads();
  // 1. sample histogram
  const int64_t nseg = (n + kSampleSeg - 1) / kSampleSeg;
  uint32_t sampled = 0;
  for (int64_t base = 0; base < nseg; base += 32 * (kTopThreads / kSampleSeg)) {
    const int64_t sg = base + 32 * (tid / kSampleSeg);  // every 32nd segment, 4 per pass
    const int64_t j = sg * kSampleSeg + (tid & (kSampleSeg - 1));
    if (sg >= nseg || j >= n) continue;
    const double s = sc[j];
    if (j == Q.self_col || s != s) continue;
    atomicAdd(&hist[score_bucket(s)], 1u);
    ++sampled;
  }
  const uint32_t nsample = block_count(sampled, wsum);
  // 2. threshold bucket: highest t whose sampled tail, scaled up, reaches 2k + 64
  if (tid == 0) {
    const double scale = (double)n / (double)max<int64_t>(1, min<int64_t>(n, ((nseg + 31) / 32) * kSampleSeg));
    const double want = 2.0 * k + 64.0;
    uint32_t tail = 0;
    int t = kBins - 1;
    for (; t > 0; --t) {
      tail += hist[t];
      if ((double)tail * scale >= want) break;
    }
    s_t = nsample == 0 ? 0 : t;
  }
  __syncthreads();
  const int t = s_t;
  // 3. one pass over the row: count valid, gather candidates with bucket >= t
  uint32_t valid = 0;
  for (int64_t j0 = 0; j0 < n; j0 += 4 * kTopThreads) {
    double v[4];
#pragma unroll
    for (int u = 0; u < 4; ++u) {
      const int64_t j = j0 + u * kTopThreads + tid;
      v[u] = j < n ? sc[j] : __builtin_nan("");
    }
#pragma unroll
    for (int u = 0; u < 4; ++u) {
      const int64_t j = j0 + u * kTopThreads + tid;
      const double s = v[u];
      if (j == Q.self_col || s != s) continue;
      ++valid;
      if (score_bucket(s) < t) continue;
      const uint32_t pos = atomicAdd(&s_cnt, 1u);
      if (pos < kCand) {
        ckey[pos] = score_key(s);
        crow[pos] = (uint32_t)(perm ? perm[j] : j);
        ccol[pos] = (uint32_t)j;
      }
    }
  }
  const uint32_t nvalid = block_count(valid, wsum);
  uint32_t cnt = s_cnt;
  const uint32_t kk = (uint32_t)min<int64_t>(k, nvalid);
  if (kk == 0) {
    if (tid == 0) counts[Q.out_pos] = 0;
    return;
  }
  if (cnt < kk || cnt > (uint32_t)kCand) {
    // The sampled guess missed.  Histogram the side of t that holds the k-th
    // score (below t when too few candidates, at/above t when too many),
    // place the exact threshold bucket, and gather again.
    const bool below = cnt < kk;
    for (int i = tid; i < kBins; i += kTopThreads) hist[i] = 0;
    __syncthreads();
    for (int64_t j = tid; j < n; j += kTopThreads) {
      const double s = sc[j];
      if (j == Q.self_col || s != s) continue;
      const int b = score_bucket(s);
      if ((b < t) == below) atomicAdd(&hist[b], 1u);
    }
    __syncthreads();
    if (tid == 0) {
      uint32_t tail = below ? cnt : 0;
      int b = below ? t - 1 : kBins - 1;
      for (; b > 0; --b) {
        tail += hist[b];
        if (tail >= kk) break;
      }
      if (b == 0 && tail < kk) tail += hist[0];
      s_t = b;
      s_cnt = 0;
      wsum[0] = tail;  // candidates at bucket >= b
    }
    __syncthreads();
    const int t2 = s_t;
    const uint32_t need = wsum[0];
    __syncthreads();
    if (need > (uint32_t)kCand) {  // one bucket too dense to hold: radix select redo
      if (tid == 0) counts[Q.out_pos] = -1;
      return;
    }
    for (int64_t j = tid; j < n; j += kTopThreads) {
      const double s = sc[j];
      if (j == Q.self_col || s != s || score_bucket(s) < t2) continue;
      const uint32_t pos = atomicAdd(&s_cnt, 1u);
      if (pos < kCand) {
        ckey[pos] = score_key(s);
        crow[pos] = (uint32_t)(perm ? perm[j] : j);
        ccol[pos] = (uint32_t)j;
      }
    }
    __syncthreads();
    cnt = s_cnt;
  }
  // 4. bitonic sort of the candidates by (key desc, row asc)
  uint32_t P = 1;
  while (P < cnt) P <<= 1;
  for (uint32_t i = cnt + tid; i < P; i += kTopThreads) {
    ckey[i] = 0;
    crow[i] = 0xFFFFFFFFu;
  }
  __syncthreads();
  for (uint32_t size = 2; size <= P; size <<= 1) {
    for (uint32_t stride = size >> 1; stride > 0; stride >>= 1) {
      for (uint32_t i = tid; i < P; i += kTopThreads) {
        const uint32_t jx = i ^ stride;
        if (jx > i) {
          const bool up = (i & size) == 0;
          const bool i_first = ckey[i] > ckey[jx] || (ckey[i] == ckey[jx] && crow[i] < crow[jx]);
          if (up != i_first) {
            const uint64_t tk = ckey[i];
            ckey[i] = ckey[jx];
            ckey[jx] = tk;
            const uint32_t tr = crow[i];
            crow[i] = crow[jx];
            crow[jx] = tr;
            const uint32_t tc = ccol[i];
            ccol[i] = ccol[jx];
            ccol[jx] = tc;
          }
        }
      }
      __syncthreads();
    }
  }
  for (uint32_t i = tid; i < kk; i += kTopThreads) {
    out_ids[Q.out_pos * k + i] = owner_ids ? owner_ids[crow[i]] : (int64_t)crow[i];
    out_scores[Q.out_pos * k + i] = sc[ccol[i]];
  }
  if (tid == 0) counts[Q.out_pos] = (int32_t)kk;
}

int launch_top_k(cms_handle* h, const double* slab, const std::vector<TopQuery>& qs, int32_t k,
                        const int64_t* d_perm, int64_t* d_ids, double* d_scores, int32_t* d_counts) {
  if (qs.empty()) return CMS_OK;
  CMS_HIP(h->ws_topq.ensure(sizeof(TopQuery) * qs.size()));
  CMS_HIP(hipMemcpyAsync(h->ws_topq.ptr, qs.data(), sizeof(TopQuery) * qs.size(), hipMemcpyHostToDevice, h->stream));
  const bool fast = h->n < (int64_t(1) << 32);  // candidate rows/columns held as u32
  {
    TimedScope ts(h, "top_k");
    if (fast)
      hipLaunchKernelGGL(k_top_k_fast, dim3((unsigned)qs.size()), dim3(kTopThreads), 0, h->stream, slab, h->n, h->n,
                         k, h->ws_topq.as<TopQuery>(), d_perm, h->d_owner_ids, d_ids, d_scores, d_counts);
    else
      hipLaunchKernelGGL(k_top_k, dim3((unsigned)qs.size()), dim3(kTopThreads), 0, h->stream, slab, h->n, h->n, k,
                         h->ws_topq.as<TopQuery>(), d_perm, h->d_owner_ids, d_ids, d_scores, d_counts);
    CMS_HIP(hipGetLastError());
  }
  if (fast) {  // rows the sampled threshold missed go through the radix select
    std::vector<TopQuery> redo;
    // counts are indexed by out_pos; gather them per query
    std::vector<int32_t> all;
    int64_t maxpos = 0;
    for (const TopQuery& q : qs) maxpos = std::max(maxpos, q.out_pos);
    all.resize(maxpos + 1);
    CMS_HIP(hipMemcpyAsync(all.data(), d_counts, sizeof(int32_t) * (maxpos + 1), hipMemcpyDeviceToHost, h->stream));
    CMS_HIP(hipStreamSynchronize(h->stream));
    for (const TopQuery& q : qs)
      if (all[q.out_pos] < 0) redo.push_back(q);
    h->topk_redo += (int64_t)redo.size();
    if (!redo.empty()) {
      CMS_HIP(hipMemcpyAsync(h->ws_topq.ptr, redo.data(), sizeof(TopQuery) * redo.size(), hipMemcpyHostToDevice,
                             h->stream));
      TimedScope ts(h, "top_k");
      hipLaunchKernelGGL(k_top_k, dim3((unsigned)redo.size()), dim3(kTopThreads), 0, h->stream, slab, h->n, h->n, k,
                         h->ws_topq.as<TopQuery>(), d_perm, h->d_owner_ids, d_ids, d_scores, d_counts);
      CMS_HIP(hipGetLastError());
    }
  }
  CMS_HIP(hipStreamSynchronize(h->stream));  // host query list and ws reuse
  return CMS_OK;
}

// ---- candidate lists of the streaming all-pairs top-k (cosine_mfma: top_k_all) ----
// Rows whose list holds more than `limit` entries, appended to `list`.
__global__ void k_cand_select(const uint32_t* ccnt, int64_t p0, int64_t np, uint32_t limit, uint32_t* list,
                              uint32_t* list_n) {
  for (int64_t i = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; i < np; i += (int64_t)gridDim.x * blockDim.x)
    if (ccnt[p0 + i] > limit) list[atomicAdd(list_n, 1u)] = (uint32_t)(p0 + i);
}

constexpr int kCandThreads = 256;

// Shrink each listed row to its first k candidates under (score desc, owner
// row asc) -- the SimilarUser order -- and raise its admission threshold to
// the k-th score.  A list that overflowed its capacity is flagged (its row is
// recomputed exactly afterwards); the threshold stays a valid lower bound.
__device__ __forceinline__ double key_score(uint64_t key) {  // inverse of score_key
  return __longlong_as_double((long long)((key >> 63) ? (key & ~(1ULL << 63)) : ~key));
}

// sorted == 0 (a pass's compaction): the first k are SELECTED (radix select
// of the k-th key, then of the owner row among its ties -- the same total
// order) and kept unordered; only the final compaction (sorted == 1) sorts
// them for the emit.  A full bitonic sort of a 2048-entry list per owner was
// 0.3 s of the config-4 job at the first compactions after the multi-limb rows.
__global__ __launch_bounds__(kCandThreads) void k_cand_compact(const uint32_t* list, const uint32_t* list_n,
                                                               uint32_t* ccnt, uint32_t* cidx, double* cval,
                                                               int32_t cap, int32_t k, const int64_t* perm,
                                                               double* thr, uint32_t* ovf, int sorted) {
  static_assert(kCandThreads == 256, "one histogram bin per thread");
  __shared__ uint64_t key[kCandCapSym];
  __shared__ uint32_t row[kCandCapSym];
  __shared__ uint32_t pid[kCandCapSym];
  __shared__ double val[kCandCapSym];
  __shared__ uint32_t hist[256];
  __shared__ uint64_t s_prefix;
  __shared__ uint32_t s_need, s_tied, s_rprefix, s_out;
  const uint32_t nl = *list_n;
  const int tid = threadIdx.x;
  for (uint32_t e = blockIdx.x; e < nl; e += gridDim.x) {
    const int64_t p = list[e];
    const uint32_t c = ccnt[p];
    const uint32_t m = min(c, (uint32_t)cap);
    if (tid == 0 && c > (uint32_t)cap) ovf[p] = 1u;
    uint32_t P = 1;
    while (P < m) P <<= 1;
    for (uint32_t i = tid; i < P; i += kCandThreads) {
      if (i < m) {
        const uint32_t o = cidx[p * cap + i];
        const double v = cval[p * cap + i];
        key[i] = score_key(v);
        row[i] = (uint32_t)perm[o];
        pid[i] = o;
        val[i] = v;
      } else {
        key[i] = 0;
        row[i] = 0xFFFFFFFFu;
      }
    }
    __syncthreads();
    if (!sorted) {
      if (m >= (uint32_t)k) {
        if (tid == 0) {
          s_prefix = 0;
          s_need = (uint32_t)k;
        }
        __syncthreads();
        for (int shift = 56; shift >= 0; shift -= 8) {  // the k-th largest key T
          hist[tid] = 0;
          __syncthreads();
          const uint64_t pre = s_prefix;
          const uint64_t hmask = shift == 56 ? 0ULL : (~0ULL << (shift + 8));
          for (uint32_t i = tid; i < m; i += kCandThreads)
            if ((key[i] & hmask) == pre) atomicAdd(&hist[(key[i] >> shift) & 255u], 1u);
          __syncthreads();
          if (tid == 0) {
            uint32_t need = s_need;
            int digit = 255;
            for (; digit > 0; --digit) {
              if (hist[digit] >= need) break;
              need -= hist[digit];
            }
            s_need = need;
            s_prefix = pre | ((uint64_t)digit << shift);
            if (shift == 0) s_tied = hist[digit];
          }
          __syncthreads();
        }
        const uint64_t T = s_prefix;
        uint32_t R = 0xFFFFFFFFu;
        if (s_need < s_tied) {  // among keys == T, the s_need-th smallest owner row R
          if (tid == 0) s_rprefix = 0;
          __syncthreads();
          for (int shift = 24; shift >= 0; shift -= 8) {
            hist[tid] = 0;
            __syncthreads();
            const uint32_t pre = s_rprefix;
            const uint32_t hmask = shift == 24 ? 0u : (~0u << (shift + 8));
            for (uint32_t i = tid; i < m; i += kCandThreads)
              if (key[i] == T && (row[i] & hmask) == pre) atomicAdd(&hist[(row[i] >> shift) & 255u], 1u);
            __syncthreads();
            if (tid == 0) {
              uint32_t need = s_need;
              int digit = 0;
              for (; digit < 255; ++digit) {
                if (hist[digit] >= need) break;
                need -= hist[digit];
              }
              s_need = need;
              s_rprefix = pre | ((uint32_t)digit << shift);
            }
            __syncthreads();
          }
          R = s_rprefix;
        }
        if (tid == 0) s_out = 0;
        __syncthreads();
        for (uint32_t i = tid; i < m; i += kCandThreads) {
          if (key[i] > T || (key[i] == T && row[i] <= R)) {
            const uint32_t o = atomicAdd(&s_out, 1u);
            cidx[p * cap + o] = pid[i];
            cval[p * cap + o] = val[i];
          }
        }
        if (tid == 0) {
          ccnt[p] = (uint32_t)k;
          thr[p] = key_score(T);
        }
      }
      __syncthreads();
      continue;
    }
    for (uint32_t size = 2; size <= P; size <<= 1) {
      for (uint32_t stride = size >> 1; stride > 0; stride >>= 1) {
        for (uint32_t i = tid; i < P; i += kCandThreads) {
          const uint32_t jx = i ^ stride;
          if (jx > i) {
            const bool up = (i & size) == 0;
            const bool i_first = key[i] > key[jx] || (key[i] == key[jx] && row[i] < row[jx]);
            if (up != i_first) {
              const uint64_t tk = key[i];
              key[i] = key[jx];
              key[jx] = tk;
              const uint32_t tr = row[i];
              row[i] = row[jx];
              row[jx] = tr;
              const uint32_t tp = pid[i];
              pid[i] = pid[jx];
              pid[jx] = tp;
              const double tv = val[i];
              val[i] = val[jx];
              val[jx] = tv;
            }
          }
        }
        __syncthreads();
      }
    }
    const uint32_t kk = min(m, (uint32_t)k);
    for (uint32_t i = tid; i < kk; i += kCandThreads) {
      cidx[p * cap + i] = pid[i];
      cval[p * cap + i] = val[i];
    }
    if (tid == 0) {
      ccnt[p] = kk;
      if (kk == (uint32_t)k) thr[p] = val[k - 1];
    }
    __syncthreads();
  }
}

// Final lists -> outputs indexed by owner row (IDs through owner_ids).
__global__ void k_cand_emit(const uint32_t* ccnt, const uint32_t* cidx, const double* cval, int32_t cap, int32_t k,
                            int64_t p0, int64_t np, const int64_t* perm, const int64_t* owner_ids, int64_t* ids,
                            double* scores, int32_t* counts) {
  for (int64_t i = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; i < np; i += (int64_t)gridDim.x * blockDim.x) {
    const int64_t p = p0 + i;
    const int64_t orow = perm[p];
    const uint32_t c = min(ccnt[p], (uint32_t)k);
    counts[orow] = (int32_t)c;
    for (uint32_t t = 0; t < c; ++t) {
      const int64_t r = perm[cidx[p * cap + t]];
      ids[orow * k + t] = owner_ids ? owner_ids[r] : r;
      scores[orow * k + t] = cval[p * cap + t];
    }
  }
}

// Union of nparts partial lists per owner -> the first k under (score desc,
// ID asc).  Owner IDs ascend with owner rows, so ID order is the
// SimilarUser tie order; an ID offered by two parts (a row recomputed whole
// after an overflow) is kept once.
__global__ __launch_bounds__(kCandThreads) void k_topk_merge(int32_t nparts, int32_t k, int64_t n, const int64_t* ids,
                                                             const double* sc, const int32_t* cnt, int64_t* out_ids,
                                                             double* out_sc, int32_t* out_cnt) {
  __shared__ uint64_t key[kCandCap];
  __shared__ int64_t oid[kCandCap];
  __shared__ double val[kCandCap];
  __shared__ uint32_t s_m;
  const int tid = threadIdx.x;
  for (int64_t r = blockIdx.x; r < n; r += gridDim.x) {
    if (tid == 0) s_m = 0;
    __syncthreads();
    for (int32_t p = 0; p < nparts; ++p) {
      const int32_t c = min(cnt[(int64_t)p * n + r], k);
      for (int32_t i = tid; i < c; i += kCandThreads) {
        const uint32_t pos = atomicAdd(&s_m, 1u);
        const int64_t src = ((int64_t)p * n + r) * k + i;
        key[pos] = score_key(sc[src]);
        oid[pos] = ids[src];
        val[pos] = sc[src];
      }
    }
    __syncthreads();
    const uint32_t m = s_m;
    uint32_t P = 1;
    while (P < m) P <<= 1;
    for (uint32_t i = m + tid; i < P; i += kCandThreads) {
      key[i] = 0;
      oid[i] = INT64_MAX;
    }
    __syncthreads();
    for (uint32_t size = 2; size <= P; size <<= 1) {
      for (uint32_t stride = size >> 1; stride > 0; stride >>= 1) {
        for (uint32_t i = tid; i < P; i += kCandThreads) {
          const uint32_t jx = i ^ stride;
          if (jx > i) {
            const bool up = (i & size) == 0;
            const bool i_first = key[i] > key[jx] || (key[i] == key[jx] && oid[i] < oid[jx]);
            if (up != i_first) {
              const uint64_t tk = key[i];
              key[i] = key[jx];
              key[jx] = tk;
              const int64_t to = oid[i];
              oid[i] = oid[jx];
              oid[jx] = to;
              const double tv = val[i];
              val[i] = val[jx];
              val[jx] = tv;
            }
          }
        }
        __syncthreads();
      }
    }
    if (tid == 0) {  // sequential: drop adjacent duplicates, keep the first k
      int32_t c = 0;
      for (uint32_t i = 0; i < m && c < k; ++i) {
        if (i > 0 && oid[i] == oid[i - 1] && key[i] == key[i - 1]) continue;
        out_ids[r * k + c] = oid[i];
        out_sc[r * k + c] = val[i];
        ++c;
      }
      out_cnt[r] = c;
    }
    __syncthreads();
  }
}

int top_k_merge(cms_handle* h, int32_t k, int32_t nparts, const int64_t* d_ids, const double* d_scores,
                const int32_t* d_counts, int64_t* d_out_ids, double* d_out_scores, int32_t* d_out_counts) {
  if (k < 1 || k > kCandCap / 2) return set_error(CMS_E_PARAM, "k must be in [1, %d]", kCandCap / 2);
  TimedScope ts(h, "topk_merge");
  const int64_t n = h->n;
  const unsigned grid = (unsigned)std::min<int64_t>(n, 8192);
  // A merge workgroup holds kCandCap candidates in LDS, so more than
  // kCandCap / k lists merge in rounds: groups of g lists -> one list each.
  // Exact: the first k of a union under the (score desc, ID asc) total order
  // are the first k of the union of each group's first k (the shards' pair
  // sets are disjoint, so no owner appears twice).
  const int32_t g = kCandCap / k;
  DevBuf tmp[2];
  int cur = -1;
  while (nparts > g) {
    const int32_t groups = (nparts + g - 1) / g;
    DevBuf& o = tmp[(cur + 1) & 1];
    CMS_HIP(o.ensure((sizeof(int64_t) + sizeof(double)) * (size_t)groups * n * k + sizeof(int32_t) * (size_t)groups * n));
    int64_t* oi = o.as<int64_t>();
    double* os = reinterpret_cast<double*>(oi + (size_t)groups * n * k);
    int32_t* oc = reinterpret_cast<int32_t*>(os + (size_t)groups * n * k);
    for (int32_t q = 0; q < groups; ++q) {
      const int64_t p0 = (int64_t)q * g;
      const int32_t np = (int32_t)std::min<int64_t>(g, nparts - p0);
      hipLaunchKernelGGL(k_topk_merge, dim3(grid), dim3(kCandThreads), 0, h->stream, np, k, n, d_ids + p0 * n * k,
                         d_scores + p0 * n * k, d_counts + p0 * n, oi + (int64_t)q * n * k, os + (int64_t)q * n * k,
                         oc + (int64_t)q * n);
    }
    CMS_HIP(hipGetLastError());
    d_ids = oi;
    d_scores = os;
    d_counts = oc;
    nparts = groups;
    cur = (cur + 1) & 1;
  }
  hipLaunchKernelGGL(k_topk_merge, dim3(grid), dim3(kCandThreads), 0, h->stream, nparts, k, n, d_ids, d_scores,
                     d_counts, d_out_ids, d_out_scores, d_out_counts);
  CMS_HIP(hipGetLastError());
  if (cur >= 0) CMS_HIP(hipStreamSynchronize(h->stream));  // the round buffers free on return
  return CMS_OK;
}

int cand_compact(cms_handle* h, const CandBufs& cb, int64_t p0, int64_t np, uint32_t limit, int32_t k) {
  if (np <= 0) return CMS_OK;
  CMS_HIP(hipMemsetAsync(cb.list_n, 0, sizeof(uint32_t), h->stream));
  const unsigned g1 = (unsigned)std::min<int64_t>((np + 255) / 256, 4096);
  hipLaunchKernelGGL(k_cand_select, dim3(g1), dim3(256), 0, h->stream, cb.ccnt, p0, np, limit, cb.list, cb.list_n);
  hipLaunchKernelGGL(k_cand_compact, dim3(4096), dim3(kCandThreads), 0, h->stream, cb.list, cb.list_n, cb.ccnt,
                     cb.cidx, cb.cval, cb.cap, k, cosine_perm_device(h), cb.thr, cb.ovf,
                     limit == 0 ? 1 : 0);  // only the final compaction sorts
  CMS_HIP(hipGetLastError());
  return CMS_OK;
}

int cand_emit(cms_handle* h, const CandBufs& cb, int64_t p0, int64_t np, int32_t k, int64_t* d_ids, double* d_scores,
              int32_t* d_counts) {
  if (np <= 0) return CMS_OK;
  const unsigned g1 = (unsigned)std::min<int64_t>((np + 255) / 256, 8192);
  hipLaunchKernelGGL(k_cand_emit, dim3(g1), dim3(256), 0, h->stream, cb.ccnt, cb.cidx, cb.cval, cb.cap, k, p0, np,
                     cosine_perm_device(h), h->d_owner_ids, d_ids, d_scores, d_counts);
  CMS_HIP(hipGetLastError());
  return CMS_OK;
}

// Offer the similarities of slab rows (positions [m0, m0+qc)) to the lists
// of the columns [c0, c1): one thread per column walks the slab rows in order
// (no contention: a list has one writer here).
__global__ void k_slab_offer(const double* __restrict__ slab, int64_t ld, int64_t m0, int64_t qc, int64_t c0, int64_t c1,
                             const double* __restrict__ thr, uint32_t* __restrict__ ccnt, uint32_t* __restrict__ cidx,
                             double* __restrict__ cval, int32_t cap) {
  for (int64_t c = c0 + blockIdx.x * (int64_t)blockDim.x + threadIdx.x; c < c1; c += (int64_t)gridDim.x * blockDim.x) {
    const double t = thr[c];
    uint32_t cnt = ccnt[c];
    auto offer = [&](int64_t m, double v) {
      if (v != v || v < t || m0 + m == c) return;
      if (cnt < (uint32_t)cap) {
        cidx[c * cap + cnt] = (uint32_t)(m0 + m);
        cval[c * cap + cnt] = v;
      }
      ++cnt;
    };
    int64_t m = 0;
    for (; m + 8 <= qc; m += 8) {  // eight rows' loads in flight per thread
      double v[8];
#pragma unroll
      for (int u = 0; u < 8; ++u) v[u] = slab[(m + u) * ld + c];
#pragma unroll
      for (int u = 0; u < 8; ++u) offer(m + u, v[u]);
    }
    for (; m < qc; ++m) offer(m, slab[m * ld + c]);
    ccnt[c] = cnt;
  }
}

int multi_rows_slab_offer(cms_handle* h, const CandBufs& cb, int64_t m0, int64_t qc, int64_t c0, int64_t c1, int32_t k,
                          int64_t* d_ids, double* d_scores, int32_t* d_counts,
                          const std::vector<std::pair<int64_t, int64_t>>* cols) {
  const int64_t n = h->n;
  int rc;
  CMS_HIP(h->ws_slab.ensure(sizeof(double) * (size_t)(qc * n)));
  double* slab = h->ws_slab.as<double>();
  if (cols) {
    // a refresh's untouched multi-limb rows: only the pairs with a touched
    // owner changed, so only those columns are computed; the rest of the
    // slab stays NaN (never a candidate).  Columns a range rounds in are
    // current values too, which the fold accepts (k_rf_fold drops pairs both
    // lists hold).
    CMS_HIP(hipMemsetAsync(slab, 0xFF, sizeof(double) * (size_t)(qc * n), h->stream));
    h->slab_cols = *cols;
    rc = cosine_slab(h, m0, qc, slab);
    h->slab_cols.clear();
    if (rc) return rc;
  } else if ((rc = cosine_slab(h, m0, qc, slab))) {
    return rc;
  }
  // exact top-k of the slab rows
  std::vector<TopQuery> qs;
  for (int64_t p = m0; p < m0 + qc; ++p) qs.push_back(TopQuery{p - m0, p, h->h_perm[p]});
  if ((rc = launch_top_k(h, slab, qs, k, cosine_perm_device(h), d_ids, d_scores, d_counts))) return rc;
  // and the same similarities for the columns' lists, cap/2 slab rows at a
  // time: each part offers at most that many entries to a list compacted to
  // cap - part first (a slab may hold more rows than a list has room for);
  // with column ranges, only the single-limb columns inside them
  std::vector<std::pair<int64_t, int64_t>> offer;
  if (cols) {
    for (const auto& cr : *cols) {
      const int64_t lo = std::max(cr.first, c0), hi = std::min(cr.second, c1);
      if (lo < hi) offer.push_back({lo, hi});
    }
  } else if (c1 > c0) {
    offer.push_back({c0, c1});
  }
  for (const auto& oc : offer) {
    const int64_t part = std::max<int64_t>(1, cb.cap / 2);
    for (int64_t s0 = 0; s0 < qc;) {
      const int64_t pc = std::min(part, qc - s0);
      if ((rc = cand_compact(h, cb, oc.first, oc.second - oc.first, (uint32_t)(cb.cap - pc), k))) return rc;
      const unsigned g1 = (unsigned)std::min<int64_t>((oc.second - oc.first + 255) / 256, 8192);
      hipLaunchKernelGGL(k_slab_offer, dim3(g1), dim3(256), 0, h->stream, slab + s0 * n, n, m0 + s0, pc, oc.first,
                         oc.second, cb.thr, cb.ccnt, cb.cidx, cb.cval, cb.cap);
      CMS_HIP(hipGetLastError());
      s0 += pc;
    }
  }
  return CMS_OK;
}

// Slab rows for the multi-limb rows of the all-pairs job: each chunk streams
// the whole single-limb image once, so as many rows as memory allows -- up to
// 4096 at 1M owners (32 GiB), never fewer than the general slab budget, and
// leaving 6 GiB of the device free.
int64_t multi_slab_rows(cms_handle* h, int64_t n) {
  const int64_t base = slab_rows_for(n);
  size_t free_b = 0, total_b = 0;
  if (hipMemGetInfo(&free_b, &total_b) != hipSuccess) return base;
  const double have = (double)free_b + (double)h->ws_slab.bytes - 6.0 * (double)(1ULL << 30);
  int64_t rows = (int64_t)(have / (8.0 * (double)std::max<int64_t>(1, n)));
  rows = std::min<int64_t>(rows, ((int64_t(1) << 32) / std::max<int64_t>(1, n)));
#ifdef CMS_MULTI_SLAB_GIB  // A/B builds: a smaller slab (fewer bytes in the first job's allocations)
  rows = std::min<int64_t>(rows, ((int64_t)CMS_MULTI_SLAB_GIB << 27) / std::max<int64_t>(1, n));
#endif
  rows = rows / 128 * 128;
  return std::max(base, rows);
}

// slab budget: 2^30 fp64 similarities (8 GiB) -- 1,024 query rows at 1M owners
int64_t slab_rows_for(int64_t n) {
  return std::max<int64_t>(128, ((int64_t(1) << 30) / std::max<int64_t>(1, n)) / 128 * 128);
}

int slab_top_k_positions(cms_handle* h, const std::vector<int64_t>& pos, const std::vector<int64_t>& out_pos,
                         int32_t k, int64_t* d_ids, double* d_scores, int32_t* d_counts) {
  // MFMA slabs over the PERMUTED 128-row query tiles that hold a requested position
  const int64_t n = h->n;
  int rc = CMS_OK;
  if (pos.empty()) return CMS_OK;
  const int64_t slab_rows = slab_rows_for(n);
  std::vector<int64_t> tiles;
  for (int64_t p : pos) tiles.push_back(p / 128);
  std::sort(tiles.begin(), tiles.end());
  tiles.erase(std::unique(tiles.begin(), tiles.end()), tiles.end());
  // a run of consecutive tiles below never exceeds slab_rows rows (nor the tiles present)
  const int64_t max_run = std::min<int64_t>(slab_rows, (int64_t)tiles.size() * 128);
  CMS_HIP(h->ws_slab.ensure(sizeof(double) * (size_t)(max_run * n)));
  std::vector<std::pair<int64_t, int64_t>> q(pos.size());
  for (size_t i = 0; i < pos.size(); ++i) q[i] = {pos[i], out_pos[i]};
  std::sort(q.begin(), q.end());
  size_t ti = 0, qi = 0;
  while (ti < tiles.size()) {
    // a run of consecutive tiles, at most slab_rows rows
    size_t tj = ti + 1;
    while (tj < tiles.size() && tiles[tj] == tiles[tj - 1] + 1 && (int64_t)(tj - ti + 1) * 128 <= slab_rows) ++tj;
    const int64_t q0 = tiles[ti] * 128;
    const int64_t qc = std::min<int64_t>(n - q0, (int64_t)(tj - ti) * 128);
    if ((rc = cosine_slab(h, q0, qc, h->ws_slab.as<double>()))) return rc;
    std::vector<TopQuery> qs;
    for (; qi < q.size() && q[qi].first < q0 + qc; ++qi) qs.push_back(TopQuery{q[qi].first - q0, q[qi].first, q[qi].second});
    if ((rc = launch_top_k(h, h->ws_slab.as<double>(), qs, k, cosine_perm_device(h), d_ids, d_scores, d_counts)))
      return rc;
    ti = tj;
  }
  return CMS_OK;
}

// ---- incremental refresh of the all-pairs top-k (cms_top_k_refresh) ----
// A refresh recomputes only the pairs with a touched owner; every other pair's
// similarity is unchanged (cos(u, v) reads only u's and v's sketches and
// norms).  An untouched owner u keeps an exact list of depth D >= k from the
// last job.  Its new list is the first D of (the new job's list of u, which
// holds every touched candidate that can matter) + (the kept entries whose
// candidate is untouched).  Every untouched candidate missing from both is
// ordered after the kept list's last entry B (it was not in the kept list),
// so the merged entries ordered at or before B are exact; a list left with
// fewer than k such entries is recomputed whole.  A kept list that held every
// candidate (fewer than D) has no B: the merge is exact throughout.

__global__ void k_rf_mark(const int64_t* row, int64_t np, int64_t n, uint8_t* touch) {
  for (int64_t i = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; i < np; i += (int64_t)gridDim.x * blockDim.x) {
    const int64_t r = row[i];
    if (r >= 0 && r < n) touch[r] = 1;
  }
}

int refresh_mark(cms_handle* h, const int64_t* d_row, int64_t npairs) {
  const unsigned g = (unsigned)std::min<int64_t>((npairs + 255) / 256, 8192);
  hipLaunchKernelGGL(k_rf_mark, dim3(g), dim3(256), 0, h->stream, d_row, npairs, h->n, h->rf_touch.as<uint8_t>());
  CMS_HIP(hipGetLastError());
  return CMS_OK;
}

constexpr int kRfMax = 2 * (kCandCap / 2);  // new + kept entries of one row (depth <= kCandCap / 2)

__global__ __launch_bounds__(kCandThreads) void k_rf_fold(int64_t n, int32_t D, int32_t k, const uint8_t* touch,
                                                          const int64_t* nid, const double* nsc, const int32_t* ncnt,
                                                          int64_t* kid, double* ksc, int32_t* kcnt, uint8_t* kfull,
                                                          uint32_t* redo) {
  __shared__ uint64_t key[kRfMax];
  __shared__ int64_t rid[kRfMax];
  __shared__ double val[kRfMax];
  __shared__ uint32_t s_m;
  const int tid = threadIdx.x;
  for (int64_t r = blockIdx.x; r < n; r += gridDim.x) {
    const int32_t cn = min(ncnt[r], D);
    const int64_t base = r * D;
    if (touch[r]) {  // every pair of a touched owner was recomputed: its new list is exact
      for (int32_t i = tid; i < cn; i += kCandThreads) {
        kid[base + i] = nid[base + i];
        ksc[base + i] = nsc[base + i];
      }
      if (tid == 0) {
        kcnt[r] = cn;
        kfull[r] = cn < D ? 1 : 0;
      }
      continue;
    }
    const int32_t co = kcnt[r];
    const bool full = kfull[r] != 0;
    uint64_t bkey = 0;
    int64_t brow = -1;
    if (co > 0) {
      bkey = score_key(ksc[base + co - 1]);
      brow = kid[base + co - 1];
    }
    if (tid == 0) s_m = 0;
    __syncthreads();
    for (int32_t i = tid; i < cn; i += kCandThreads) {
      const uint32_t p = atomicAdd(&s_m, 1u);
      key[p] = score_key(nsc[base + i]);
      rid[p] = nid[base + i];
      val[p] = nsc[base + i];
    }
    for (int32_t i = tid; i < co; i += kCandThreads) {
      const int64_t c = kid[base + i];
      if (touch[c]) continue;  // stale: the new list carries its current score
      const uint32_t p = atomicAdd(&s_m, 1u);
      key[p] = score_key(ksc[base + i]);
      rid[p] = c;
      val[p] = ksc[base + i];
    }
    __syncthreads();
    const uint32_t m = s_m;
    uint32_t P = 1;
    while (P < m) P <<= 1;
    for (uint32_t i = m + tid; i < P; i += kCandThreads) {
      key[i] = 0;
      rid[i] = INT64_MAX;
    }
    __syncthreads();
    for (uint32_t size = 2; size <= P; size <<= 1) {
      for (uint32_t stride = size >> 1; stride > 0; stride >>= 1) {
        for (uint32_t i = tid; i < P; i += kCandThreads) {
          const uint32_t jx = i ^ stride;
          if (jx > i) {
            const bool up = (i & size) == 0;
            const bool i_first = key[i] > key[jx] || (key[i] == key[jx] && rid[i] < rid[jx]);
            if (up != i_first) {
              const uint64_t tk = key[i];
              key[i] = key[jx];
              key[jx] = tk;
              const int64_t tr = rid[i];
              rid[i] = rid[jx];
              rid[jx] = tr;
              const double tv = val[i];
              val[i] = val[jx];
              val[jx] = tv;
            }
          }
        }
        __syncthreads();
      }
    }
    if (tid == 0) {  // sequential: drop duplicates (an untouched pair both lists hold), keep the first D
      int32_t c = 0, valid = 0;
      for (uint32_t i = 0; i < m && c < D; ++i) {
        if (i > 0 && rid[i] == rid[i - 1] && key[i] == key[i - 1]) continue;
        kid[base + c] = rid[i];
        ksc[base + c] = val[i];
        ++c;
        if (full || key[i] > bkey || (key[i] == bkey && rid[i] <= brow)) valid = c;
      }
      kcnt[r] = full ? c : valid;
      kfull[r] = (full && c < D) ? 1 : 0;
      if (!full && valid < k) redo[1 + atomicAdd(redo, 1u)] = (uint32_t)r;
    }
    __syncthreads();
  }
}

int refresh_fold(cms_handle* h, const int64_t* d_new_ids, const double* d_new_sc, const int32_t* d_new_cnt, int32_t k,
                 uint32_t* d_redo) {
  if (h->rf_depth > kCandCap / 2) return set_error(CMS_E_PARAM, "refresh depth %d", h->rf_depth);
  CMS_HIP(hipMemsetAsync(d_redo, 0, sizeof(uint32_t), h->stream));
  const unsigned grid = (unsigned)std::min<int64_t>(h->n, 8192);
  hipLaunchKernelGGL(k_rf_fold, dim3(grid), dim3(kCandThreads), 0, h->stream, h->n, h->rf_depth, k,
                     h->rf_touch.as<uint8_t>(), d_new_ids, d_new_sc, d_new_cnt, h->rf_ids.as<int64_t>(),
                     h->rf_sc.as<double>(), h->rf_cnt.as<int32_t>(), h->rf_full.as<uint8_t>(), d_redo);
  CMS_HIP(hipGetLastError());
  return CMS_OK;
}

__global__ void k_rf_set_full(const int32_t* cnt, int64_t n, int32_t D, uint8_t* full) {
  for (int64_t r = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; r < n; r += (int64_t)gridDim.x * blockDim.x)
    full[r] = cnt[r] < D ? 1 : 0;
}

__global__ void k_rf_set_full_list(const int32_t* cnt, const uint32_t* list, int32_t D, uint8_t* full) {
  const uint32_t m = list[0];
  for (uint32_t i = blockIdx.x * blockDim.x + threadIdx.x; i < m; i += gridDim.x * blockDim.x) {
    const uint32_t r = list[1 + i];
    full[r] = cnt[r] < D ? 1 : 0;
  }
}

int refresh_set_full_list(cms_handle* h, const uint32_t* d_list, int64_t m) {
  if (m <= 0) return CMS_OK;
  const unsigned g = (unsigned)std::min<int64_t>((m + 255) / 256, 8192);
  hipLaunchKernelGGL(k_rf_set_full_list, dim3(g), dim3(256), 0, h->stream, h->rf_cnt.as<int32_t>(), d_list,
                     h->rf_depth, h->rf_full.as<uint8_t>());
  CMS_HIP(hipGetLastError());
  return CMS_OK;
}

int refresh_set_full(cms_handle* h) {
  const unsigned g = (unsigned)std::min<int64_t>((h->n + 255) / 256, 8192);
  hipLaunchKernelGGL(k_rf_set_full, dim3(g), dim3(256), 0, h->stream, h->rf_cnt.as<int32_t>(), h->n, h->rf_depth,
                     h->rf_full.as<uint8_t>());
  CMS_HIP(hipGetLastError());
  return CMS_OK;
}

__global__ void k_rf_emit(int64_t n, int32_t D, int32_t k, const int64_t* kid, const double* ksc, const int32_t* kcnt,
                          const int64_t* owner_ids, int64_t* ids, double* scores, int32_t* counts) {
  for (int64_t r = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; r < n; r += (int64_t)gridDim.x * blockDim.x) {
    const int32_t c = min(kcnt[r], k);
    counts[r] = c;
    for (int32_t t = 0; t < c; ++t) {
      const int64_t o = kid[r * D + t];
      ids[r * k + t] = owner_ids ? owner_ids[o] : o;
      scores[r * k + t] = ksc[r * D + t];
    }
  }
}

int refresh_emit(cms_handle* h, int32_t k, int64_t* d_ids, double* d_scores, int32_t* d_counts) {
  const unsigned g = (unsigned)std::min<int64_t>((h->n + 255) / 256, 8192);
  hipLaunchKernelGGL(k_rf_emit, dim3(g), dim3(256), 0, h->stream, h->n, h->rf_depth, k, h->rf_ids.as<int64_t>(),
                     h->rf_sc.as<double>(), h->rf_cnt.as<int32_t>(), h->d_owner_ids, d_ids, d_scores, d_counts);
  CMS_HIP(hipGetLastError());
  return CMS_OK;
}

int top_k_rows(cms_handle* h, int64_t row_begin, int64_t row_count, int32_t k, int64_t* d_ids, double* d_scores,
               int32_t* d_counts) {
  if (k < 1 || k > kTopMax) return set_error(CMS_E_PARAM, "k must be in [1, %d]", kTopMax);
  if (h->per_owner) return po_top_k_rows(h, row_begin, row_count, k, d_ids, d_scores, d_counts);
  const int64_t n = h->n;
  int rc = CMS_OK;
  if (mfma_eligible(h) && (rc = cosine_prepare(h))) return rc;
  const int64_t slab_rows = slab_rows_for(n);
  if (mfma_eligible(h) && h->n_inexact_rows == 0) {
    std::vector<int64_t> pos(row_count), outp(row_count);
    for (int64_t r = row_begin; r < row_begin + row_count; ++r) {
      pos[r - row_begin] = h->h_inv[r];
      outp[r - row_begin] = r - row_begin;
    }
    return slab_top_k_positions(h, pos, outp, k, d_ids, d_scores, d_counts);
  }
  // exact pair kernel per query row (widths not a multiple of 128, or owners
  // whose norms left the exact fp64 regime)
  const int64_t qb = std::min<int64_t>(row_count, slab_rows);
  CMS_HIP(h->ws_slab.ensure(sizeof(double) * (size_t)(qb * n)));
  CMS_HIP(h->ws_query.ensure(sizeof(int64_t) * (size_t)n));
  {
    std::vector<int64_t> all(n);
    for (int64_t i = 0; i < n; ++i) all[i] = i;
    CMS_HIP(hipMemcpyAsync(h->ws_query.ptr, all.data(), sizeof(int64_t) * n, hipMemcpyHostToDevice, h->stream));
    CMS_HIP(hipStreamSynchronize(h->stream));
  }
  for (int64_t r0 = 0; r0 < row_count; r0 += qb) {
    const int64_t rcnt = std::min(qb, row_count - r0);
    std::vector<TopQuery> qs;
    if (h->f64 && (rc = f64_slab(h, row_begin + r0, rcnt, h->ws_slab.as<double>()))) return rc;
    for (int64_t q = 0; q < rcnt; ++q) {
      const int64_t row = row_begin + r0 + q;
      if (!h->f64 && (rc = pair_cosines(h, row, h->ws_query.as<int64_t>(), n, h->ws_slab.as<double>() + q * n)))
        return rc;
      qs.push_back(TopQuery{q, row, r0 + q});
    }
    if ((rc = launch_top_k(h, h->ws_slab.as<double>(), qs, k, nullptr, d_ids, d_scores, d_counts))) return rc;
  }
  return CMS_OK;
}

}  // namespace cms
