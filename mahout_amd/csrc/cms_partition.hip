// cms_partition.hip -- unordered COO stream -> CSR keys grouped by owner row.
//
// The reference never sees an unordered stream: its DataModel hands CosineCM
// one PreferenceArray per owner (T/impl/similarity/CosineCM.java:49-56).  A
// streaming ingest has to group the pairs itself before the LDS row build
// (cms_build.hip).  Two MSD passes, fan-out <= 4096 each:
//   pass 1: coarse bin = row >> s2   (writes key + u16 fine index)
//   pass 2: fine bin   = row & (2^s2 - 1), segmented per coarse bin
//           (writes the key at its final CSR position; the scan of pass 2 also
//            yields the CSR row offsets)
// Each scatter stages a 4096-pair tile in LDS sorted by bin and writes it out
// as contiguous per-bin runs, so global writes coalesce instead of landing as
// isolated 8-byte stores.  Counts come from per-block LDS histograms and a
// device-wide scan -- no global atomics on hot rows.
#include <hip/hip_runtime.h>

#include <algorithm>

#include "cms_device.h"
#include "cms_internal.h"

namespace cms {

constexpr int kPartThreads = 512;
constexpr int kPartPer = 8;
constexpr int kPartTile = kPartThreads * kPartPer;  // pairs staged per tile
constexpr int kMaxBins = 4096;

__global__ __launch_bounds__(256) void k_p1_hist(const int64_t* row, int64_t n, int64_t chunk, int s2, int P1,
                                                 int64_t nrows, uint32_t* H1, int NB, uint32_t* flags) {
  extern __shared__ uint32_t lh[];
  for (int b = threadIdx.x; b < P1; b += blockDim.x) lh[b] = 0;
  __syncthreads();
  int64_t lo = (int64_t)blockIdx.x * chunk, hi = min(n, lo + chunk);
  bool bad = false;
  // two rows per 16-byte load
  const int64_t lo2 = (lo + 1) & ~int64_t(1);
  if (lo2 > lo && threadIdx.x == 0 && lo < hi) {
    int64_t r = row[lo];
    if (r < 0 || r >= nrows) bad = true;
    else atomicAdd(&lh[(uint32_t)(r >> s2)], 1u);
  }
  const int64_t npair = (hi - lo2) / 2;
  const longlong2* r2 = reinterpret_cast<const longlong2*>(row + lo2);
  for (int64_t i = threadIdx.x; i < npair; i += blockDim.x) {
    longlong2 v = r2[i];
    if (v.x < 0 || v.x >= nrows) bad = true;
    else atomicAdd(&lh[(uint32_t)(v.x >> s2)], 1u);
    if (v.y < 0 || v.y >= nrows) bad = true;
    else atomicAdd(&lh[(uint32_t)(v.y >> s2)], 1u);
  }
  if (threadIdx.x == 0 && lo2 + 2 * npair < hi) {
    int64_t r = row[hi - 1];
    if (r < 0 || r >= nrows) bad = true;
    else atomicAdd(&lh[(uint32_t)(r >> s2)], 1u);
  }
  if (bad) atomicOr(flags, kFlagBadRow);
  __syncthreads();
  for (int b = threadIdx.x; b < P1; b += blockDim.x) H1[(int64_t)b * NB + blockIdx.x] = lh[b];
}

// Exclusive scan of hist[0..P) into off[] by the whole block (P <= 4096).
__device__ __forceinline__ uint32_t scan_bins(const uint32_t* hist, uint32_t* off, int P, uint32_t* scr) {
  const int per = (P + kPartThreads - 1) / kPartThreads;
  const int b0 = threadIdx.x * per, b1 = min(P, b0 + per);
  uint32_t s = 0;
  for (int b = b0; b < b1; ++b) s += hist[b];
  uint32_t tot;
  uint32_t o = block_excl_scan_u32(s, scr, &tot);
  for (int b = b0; b < b1; ++b) {
    off[b] = o;
    o += hist[b];
  }
  return tot;
}

struct TileLds {
  int64_t* key;
  float* val;
  uint16_t* fine;
  uint16_t* bin;
  uint32_t* cursor;
  uint32_t* hist;
  uint32_t* off;
  uint32_t* scr;
};

__device__ __forceinline__ TileLds carve(unsigned char* smem, int P) {
  TileLds t;
  t.key = reinterpret_cast<int64_t*>(smem);
  t.val = reinterpret_cast<float*>(t.key + kPartTile);
  t.fine = reinterpret_cast<uint16_t*>(t.val + kPartTile);
  t.bin = t.fine + kPartTile;
  t.cursor = reinterpret_cast<uint32_t*>(t.bin + kPartTile);
  t.hist = t.cursor + P;
  t.off = t.hist + P;
  t.scr = t.off + P;
  return t;
}

static size_t tile_lds_bytes(int P) {
  return (size_t)kPartTile * (8 + 4 + 2 + 2) + (size_t)3 * P * 4 + 64 * 4;
}

// Pass 1: block b owns stream chunk [b*chunk, (b+1)*chunk); output region of
// (coarse bin, block) starts at O1[bin*NB + b].
__global__ __launch_bounds__(kPartThreads) void k_p1_scatter(const int64_t* row, const int64_t* key, const float* val,
                                                             int64_t n, int64_t chunk, int s2, int P1, int64_t nrows,
                                                             const uint32_t* O1, int NB, uint16_t* ofine,
                                                             int64_t* okey, float* oval) {
  extern __shared__ __align__(16) unsigned char smem[];
  TileLds L = carve(smem, P1);
  const int tid = threadIdx.x;
  for (int b = tid; b < P1; b += kPartThreads) L.cursor[b] = O1[(int64_t)b * NB + blockIdx.x];
  const int64_t lo = (int64_t)blockIdx.x * chunk, hi = min(n, lo + chunk);
  const uint32_t fmask = (1u << s2) - 1u;
  for (int64_t tb = lo; tb < hi; tb += kPartTile) {
    for (int b = tid; b < P1; b += kPartThreads) L.hist[b] = 0;
    __syncthreads();
    int64_t kk[kPartPer];
    float vv[kPartPer];
    uint32_t bb[kPartPer], rk[kPartPer];
#pragma unroll
    for (int u = 0; u < kPartPer; ++u) {
      int64_t e = tb + tid + (int64_t)u * kPartThreads;
      rk[u] = 0xFFFFFFFFu;
      if (e < hi) {
        int64_t r = row[e];
        kk[u] = key[e];
        vv[u] = val ? val[e] : 0.f;
        if (r >= 0 && r < nrows) {
          bb[u] = (uint32_t)r;
          rk[u] = atomicAdd(&L.hist[(uint32_t)(r >> s2)], 1u);
        }
      }
    }
    __syncthreads();
    const uint32_t cnt = scan_bins(L.hist, L.off, P1, L.scr);
    __syncthreads();
#pragma unroll
    for (int u = 0; u < kPartPer; ++u) {
      if (rk[u] != 0xFFFFFFFFu) {
        uint32_t bin = bb[u] >> s2;
        uint32_t p = L.off[bin] + rk[u];
        L.key[p] = kk[u];
        L.val[p] = vv[u];
        L.fine[p] = (uint16_t)(bb[u] & fmask);
        L.bin[p] = (uint16_t)bin;
      }
    }
    __syncthreads();
    for (uint32_t i = tid; i < cnt; i += kPartThreads) {
      uint32_t bin = L.bin[i];
      uint32_t g = L.cursor[bin] + (i - L.off[bin]);
      okey[g] = L.key[i];
      ofine[g] = L.fine[i];
      if (oval) oval[g] = L.val[i];
    }
    __syncthreads();
    for (int b = tid; b < P1; b += kPartThreads) L.cursor[b] += L.hist[b];
    __syncthreads();
  }
}

// binStart[b] = O1[b*NB] (exclusive, bin-major), binStart[P1] = total;
// blkStart = exclusive scan of ceil(size_b / CH2).  One block.
__global__ __launch_bounds__(1024) void k_p2_plan(const uint32_t* O1, const uint32_t* H1, int NB, int P1,
                                                  int64_t CH2, uint32_t* binStart, uint32_t* blkStart) {
  __shared__ uint32_t sc[1024 / 64 + 1];
  const uint32_t total = O1[(int64_t)(P1 - 1) * NB + NB - 1] + H1[(int64_t)(P1 - 1) * NB + NB - 1];
  int per = (P1 + 1023) / 1024;
  int lo = threadIdx.x * per, hi = min(P1, lo + per);
  uint32_t s = 0;
  for (int b = lo; b < hi; ++b) {
    uint32_t start = O1[(int64_t)b * NB];
    uint32_t end = (b + 1 < P1) ? O1[(int64_t)(b + 1) * NB] : total;
    binStart[b] = start;
    s += (uint32_t)((end - start + CH2 - 1) / CH2);
  }
  uint32_t tot;
  uint32_t off = block_excl_scan_u32(s, sc, &tot);
  for (int b = lo; b < hi; ++b) {
    uint32_t start = O1[(int64_t)b * NB];
    uint32_t end = (b + 1 < P1) ? O1[(int64_t)(b + 1) * NB] : total;
    blkStart[b] = off;
    off += (uint32_t)((end - start + CH2 - 1) / CH2);
  }
  if (threadIdx.x == 0) {
    blkStart[P1] = tot;
    binStart[P1] = total;
  }
}

__device__ __forceinline__ int find_bin(const uint32_t* blkStart, int P1, uint32_t x) {
  int lo = 0, hi = P1;  // last b with blkStart[b] <= x
  while (lo < hi) {
    int mid = (lo + hi) >> 1;
    if (blkStart[mid] <= x) lo = mid + 1;
    else hi = mid;
  }
  return lo - 1;
}

__global__ __launch_bounds__(256) void k_p2_hist(const uint16_t* fine, const uint32_t* binStart,
                                                 const uint32_t* blkStart, int P1, int64_t CH2, int P2,
                                                 uint32_t* H2) {
  extern __shared__ uint32_t lh[];
  uint32_t nblk = blkStart[P1];
  if (blockIdx.x >= nblk) return;
  int b = find_bin(blkStart, P1, blockIdx.x);
  for (int f = threadIdx.x; f < P2; f += blockDim.x) lh[f] = 0;
  __syncthreads();
  int64_t lo = binStart[b] + (int64_t)(blockIdx.x - blkStart[b]) * CH2;
  int64_t hi = min((int64_t)binStart[b + 1], lo + CH2);
  for (int64_t i = lo + threadIdx.x; i < hi; i += blockDim.x) atomicAdd(&lh[fine[i]], 1u);
  __syncthreads();
  for (int f = threadIdx.x; f < P2; f += blockDim.x) H2[(int64_t)blockIdx.x * P2 + f] = lh[f];
}

// One block per coarse bin: offsets of (block, fine bin) and the CSR row
// starts of the bin's rows.
__global__ __launch_bounds__(1024) void k_p2_scan(const uint32_t* H2, const uint32_t* binStart,
                                                  const uint32_t* blkStart, int P1, int P2, int64_t nrows,
                                                  uint32_t* O2, int64_t* row_start) {
  __shared__ uint32_t sc[1024 / 64 + 1];
  __shared__ uint32_t tots[kMaxBins];
  const int b = blockIdx.x;
  const uint32_t k0 = blkStart[b], k1 = blkStart[b + 1];
  for (int f = threadIdx.x; f < P2; f += blockDim.x) {
    uint32_t T = 0;
#pragma unroll 8
    for (uint32_t k = k0; k < k1; ++k) T += H2[(int64_t)k * P2 + f];
    tots[f] = T;
  }
  __syncthreads();
  // exclusive scan of tots over f (each thread a contiguous run)
  const int per = (P2 + 1023) / 1024;
  const int f0 = threadIdx.x * per, f1 = min(P2, f0 + per);
  uint32_t s = 0;
  for (int f = f0; f < f1; ++f) s += tots[f];
  uint32_t ex = block_excl_scan_u32(s, sc, nullptr);
  for (int f = f0; f < f1; ++f) {
    uint32_t t = tots[f];
    tots[f] = ex;
    ex += t;
  }
  __syncthreads();
  for (int f = threadIdx.x; f < P2; f += blockDim.x) {
    uint32_t base = binStart[b] + tots[f];
    int64_t r = (int64_t)b * P2 + f;
    if (r < nrows) row_start[r] = base;
    uint32_t run = base;
    // the counts were read above; batch the loads so they are in flight together
    uint32_t k = k0;
    for (; k + 8 <= k1; k += 8) {
      uint32_t c[8];
#pragma unroll
      for (int u = 0; u < 8; ++u) c[u] = H2[(int64_t)(k + u) * P2 + f];
#pragma unroll
      for (int u = 0; u < 8; ++u) {
        O2[(int64_t)(k + u) * P2 + f] = run;
        run += c[u];
      }
    }
    for (; k < k1; ++k) {
      uint32_t c = H2[(int64_t)k * P2 + f];
      O2[(int64_t)k * P2 + f] = run;
      run += c;
    }
  }
  if (b == P1 - 1 && threadIdx.x == 0) row_start[nrows] = binStart[P1];
}

__global__ __launch_bounds__(kPartThreads) void k_p2_scatter(const uint16_t* fine, const int64_t* key1,
                                                             const float* val1, const uint32_t* binStart,
                                                             const uint32_t* blkStart, int P1, int64_t CH2, int P2,
                                                             const uint32_t* O2, int64_t* okey, float* oval,
                                                             int32_t* orow) {
  extern __shared__ __align__(16) unsigned char smem[];
  uint32_t nblk = blkStart[P1];
  if (blockIdx.x >= nblk) return;
  TileLds L = carve(smem, P2);
  const int tid = threadIdx.x;
  const int b = find_bin(blkStart, P1, blockIdx.x);
  for (int f = tid; f < P2; f += kPartThreads) L.cursor[f] = O2[(int64_t)blockIdx.x * P2 + f];
  const int64_t lo = binStart[b] + (int64_t)(blockIdx.x - blkStart[b]) * CH2;
  const int64_t hi = min((int64_t)binStart[b + 1], lo + CH2);
  for (int64_t tb = lo; tb < hi; tb += kPartTile) {
    for (int f = tid; f < P2; f += kPartThreads) L.hist[f] = 0;
    __syncthreads();
    int64_t kk[kPartPer];
    float vv[kPartPer];
    uint32_t ff[kPartPer], rk[kPartPer];
#pragma unroll
    for (int u = 0; u < kPartPer; ++u) {
      int64_t e = tb + tid + (int64_t)u * kPartThreads;
      rk[u] = 0xFFFFFFFFu;
      if (e < hi) {
        ff[u] = fine[e];
        kk[u] = key1[e];
        vv[u] = val1 ? val1[e] : 0.f;
        rk[u] = atomicAdd(&L.hist[ff[u]], 1u);
      }
    }
    __syncthreads();
    const uint32_t cnt = scan_bins(L.hist, L.off, P2, L.scr);
    __syncthreads();
#pragma unroll
    for (int u = 0; u < kPartPer; ++u) {
      if (rk[u] != 0xFFFFFFFFu) {
        uint32_t p = L.off[ff[u]] + rk[u];
        L.key[p] = kk[u];
        L.val[p] = vv[u];
        L.bin[p] = (uint16_t)ff[u];
      }
    }
    __syncthreads();
    for (uint32_t i = tid; i < cnt; i += kPartThreads) {
      uint32_t f = L.bin[i];
      uint32_t g = L.cursor[f] + (i - L.off[f]);
      okey[g] = L.key[i];
      if (oval) oval[g] = L.val[i];
      if (orow) orow[g] = b * P2 + (int32_t)f;
    }
    __syncthreads();
    for (int f = tid; f < P2; f += kPartThreads) L.cursor[f] += L.hist[f];
    __syncthreads();
  }
}

static int ceil_log2(int64_t v) {
  int b = 0;
  while ((int64_t(1) << b) < v) ++b;
  return b;
}

int partition_to_csr(cms_handle* h, const int64_t* d_row, const int64_t* d_key, const float* d_val, int64_t npairs,
                     int64_t** out_off, int64_t** out_key, float** out_val, int32_t* out_rows) {
  const int64_t n = h->n;
  const int B = std::max(1, ceil_log2(n));
  int s2 = std::min(B, 10);
  if (B - s2 > 12) s2 = B - 12;
  const int P2 = 1 << s2;
  const int P1 = (int)((n + P2 - 1) / P2);
  if (P1 > kMaxBins || P2 > kMaxBins)
    return set_error(CMS_E_PARAM, "num_owners %lld too large for the partition", (long long)n);
  const int64_t chunk1 = std::max<int64_t>(4 * kPartTile, (npairs + 2047) / 2048);
  const int NB = (int)((npairs + chunk1 - 1) / chunk1);
  const int64_t CH2 = 4 * kPartTile;
  const int64_t nb2max = npairs / CH2 + P1 + 1;

  CMS_HIP(h->ws_p1_row.ensure(sizeof(uint16_t) * (size_t)npairs));
  CMS_HIP(h->ws_p1_key.ensure(sizeof(int64_t) * (size_t)npairs));
  if (d_val) CMS_HIP(h->ws_p1_val.ensure(sizeof(float) * (size_t)npairs));
  CMS_HIP(h->ws_csr_key.ensure(sizeof(int64_t) * (size_t)npairs));
  if (d_val) CMS_HIP(h->ws_csr_val.ensure(sizeof(float) * (size_t)npairs));
  CMS_HIP(h->ws_csr_off.ensure(sizeof(int64_t) * (size_t)(n + 1)));
  const int64_t L1 = (int64_t)P1 * NB, L2 = nb2max * P2;
  const int64_t nbs = (L1 + 4095) / 4096 + 1;
  const size_t hist_words = (size_t)(2 * L1 + 2 * L2 + nbs + 2 * (P1 + 1) + 64);
  CMS_HIP(h->ws_hist.ensure(sizeof(uint32_t) * hist_words));
  uint32_t* H1 = h->ws_hist.as<uint32_t>();
  uint32_t* O1 = H1 + L1;
  uint32_t* H2 = O1 + L1;
  uint32_t* O2 = H2 + L2;
  uint32_t* bsum = O2 + L2;
  uint32_t* binStart = bsum + nbs;
  uint32_t* blkStart = binStart + (P1 + 1);

  uint16_t* fine = h->ws_p1_row.as<uint16_t>();
  int64_t* key1 = h->ws_p1_key.as<int64_t>();
  float* val1 = d_val ? h->ws_p1_val.as<float>() : nullptr;
  int64_t* ckey = h->ws_csr_key.as<int64_t>();
  float* cval = d_val ? h->ws_csr_val.as<float>() : nullptr;
  int64_t* coff = h->ws_csr_off.as<int64_t>();
  static bool lds_attr = [] {
    (void)hipFuncSetAttribute((const void*)k_p1_scatter, hipFuncAttributeMaxDynamicSharedMemorySize, 160 * 1024);
    (void)hipFuncSetAttribute((const void*)k_p2_scatter, hipFuncAttributeMaxDynamicSharedMemorySize, 160 * 1024);
    return true;
  }();
  (void)lds_attr;
  {
    TimedScope ts(h, "partition");
    hipLaunchKernelGGL(k_p1_hist, dim3(NB), dim3(256), sizeof(uint32_t) * P1, h->stream, d_row, npairs, chunk1, s2,
                       P1, n, H1, NB, h->d_flags);
    int rc = scan_exclusive_u32(h, H1, O1, L1, bsum);
    if (rc) return rc;
    hipLaunchKernelGGL(k_p1_scatter, dim3(NB), dim3(kPartThreads), tile_lds_bytes(P1), h->stream, d_row, d_key,
                       d_val, npairs, chunk1, s2, P1, n, O1, NB, fine, key1, val1);
    hipLaunchKernelGGL(k_p2_plan, dim3(1), dim3(1024), 0, h->stream, O1, H1, NB, P1, CH2, binStart, blkStart);
    hipLaunchKernelGGL(k_p2_hist, dim3((unsigned)nb2max), dim3(256), sizeof(uint32_t) * P2, h->stream, fine,
                       binStart, blkStart, P1, CH2, P2, H2);
    hipLaunchKernelGGL(k_p2_scan, dim3(P1), dim3(1024), 0, h->stream, H2, binStart, blkStart, P1, P2, n, O2, coff);
    hipLaunchKernelGGL(k_p2_scatter, dim3((unsigned)nb2max), dim3(kPartThreads), tile_lds_bytes(P2), h->stream, fine,
                       key1, val1, binStart, blkStart, P1, CH2, P2, O2, ckey, cval, out_rows);
    CMS_HIP(hipGetLastError());
  }
  *out_off = coff;
  *out_key = ckey;
  *out_val = cval;
  return CMS_OK;
}

}  // namespace cms
