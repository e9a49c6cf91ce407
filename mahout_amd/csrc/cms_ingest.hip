// cms_ingest.hip -- sketch-update path on gfx950.
//
// Reference semantics: DoubleCountMinSketch.update(key, inc)
// (T/impl/common/DoubleCountMinSketch.java:72-80) applied for every
// (owner, key, value) of the stream: for each sketch row i < d,
// count[owner][i][h_i(key)] += inc.  Counters here are u32 (exact for the
// integer increments of implicit/rating streams, so the summation order the
// reference uses cannot change any value).
//
// Data path for a bulk build (table empty):
//   COO pairs --(2-pass MSD partition by owner row)--> CSR keys grouped by row
//   CSR --(k_build_rows: one workgroup per row or per SLICE of a hot row,
//          each sketch row staged in LDS, LDS atomics for the increments,
//          sum-of-squares fused, one coalesced write of the finished row)--> table
//   hot-row partial slices --(k_reduce_hot)--> table
// so every table byte is written exactly once (the zero fill is fused) and
// the stream is read a small constant number of times.  Small batches into a
// non-empty table use k_ingest_atomic (global atomics, exact for u32).
#include <hip/hip_runtime.h>

#include <algorithm>

#include "cms_internal.h"

namespace cms {

// ---------------------------------------------------------------- helpers --

__device__ __forceinline__ bool load_inc(const float* val, int64_t i, uint32_t& inc) {
  if (val == nullptr) {
    inc = 1u;
    return true;
  }
  float v = val[i];
  if (!(v >= 0.0f) || v != floorf(v) || v >= 4294967296.0f) {
    inc = 0u;
    return false;
  }
  inc = (uint32_t)v;
  return true;
}

__device__ __forceinline__ uint64_t sat_add(uint64_t a, uint64_t b) {
  uint64_t s = a + b;
  return s < a ? ~0ULL : s;
}

__device__ __forceinline__ uint32_t wave_incl_scan_u32(uint32_t v) {
  const int lane = threadIdx.x & 63;
#pragma unroll
  for (int o = 1; o < 64; o <<= 1) {
    uint32_t t = __shfl_up(v, o, 64);
    if (lane >= o) v += t;
  }
  return v;
}

__device__ __forceinline__ uint64_t wave_sum_u64_sat(uint64_t v) {
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) v = sat_add(v, __shfl_xor(v, o, 64));
  return v;
}

// Exclusive scan across the block; scratch needs (blockDim/64 + 1) words.
__device__ uint32_t block_excl_scan_u32(uint32_t v, uint32_t* scratch, uint32_t* total) {
  const int lane = threadIdx.x & 63, wid = threadIdx.x >> 6, nw = blockDim.x >> 6;
  uint32_t inc = wave_incl_scan_u32(v);
  if (lane == 63) scratch[wid] = inc;
  __syncthreads();
  if (threadIdx.x == 0) {
    uint32_t s = 0;
    for (int i = 0; i < nw; ++i) {
      uint32_t t = scratch[i];
      scratch[i] = s;
      s += t;
    }
    scratch[nw] = s;
  }
  __syncthreads();
  uint32_t res = inc - v + scratch[wid];
  if (total) *total = scratch[nw];
  __syncthreads();
  return res;
}

// Block-wide saturating u64 sum; returns the sum in every thread.
__device__ uint64_t block_sum_u64_sat(uint64_t v, uint64_t* scratch) {
  const int lane = threadIdx.x & 63, wid = threadIdx.x >> 6, nw = blockDim.x >> 6;
  v = wave_sum_u64_sat(v);
  if (lane == 0) scratch[wid] = v;
  __syncthreads();
  uint64_t s = 0;
  for (int i = 0; i < nw; ++i) s = sat_add(s, scratch[i]);
  __syncthreads();
  return s;
}

// ------------------------------------------------------- device-wide scan --
// Exclusive scan of u32[L] (L * max element < 2^32), 3 launches.
constexpr int kScanThreads = 256;
constexpr int kScanPer = 16;
constexpr int kScanTile = kScanThreads * kScanPer;

__global__ __launch_bounds__(kScanThreads) void k_scan_reduce(const uint32_t* in, int64_t L, uint32_t* bsum) {
  __shared__ uint32_t sc[kScanThreads / 64 + 1];
  int64_t base = (int64_t)blockIdx.x * kScanTile;
  uint32_t s = 0;
  for (int k = 0; k < kScanPer; ++k) {
    int64_t i = base + (int64_t)k * kScanThreads + threadIdx.x;
    if (i < L) s += in[i];
  }
  uint32_t tot;
  block_excl_scan_u32(s, sc, &tot);
  if (threadIdx.x == 0) bsum[blockIdx.x] = tot;
}

__global__ __launch_bounds__(1024) void k_scan_bsum(uint32_t* bsum, int64_t nb) {
  __shared__ uint32_t sc[1024 / 64 + 1];
  // each thread owns a contiguous run of ceil(nb/1024) entries
  int64_t per = (nb + 1023) / 1024;
  int64_t lo = (int64_t)threadIdx.x * per, hi = min(nb, lo + per);
  uint32_t s = 0;
  for (int64_t i = lo; i < hi; ++i) s += bsum[i];
  uint32_t off = block_excl_scan_u32(s, sc, nullptr);
  for (int64_t i = lo; i < hi; ++i) {
    uint32_t t = bsum[i];
    bsum[i] = off;
    off += t;
  }
}

__global__ __launch_bounds__(kScanThreads) void k_scan_down(const uint32_t* in, int64_t L, const uint32_t* bsum,
                                                             uint32_t* out) {
  __shared__ uint32_t sc[kScanThreads / 64 + 1];
  int64_t base = (int64_t)blockIdx.x * kScanTile;
  uint32_t carry = bsum[blockIdx.x];
  for (int k = 0; k < kScanPer; ++k) {
    int64_t i = base + (int64_t)k * kScanThreads + threadIdx.x;
    uint32_t v = i < L ? in[i] : 0u;
    uint32_t tot;
    uint32_t ex = block_excl_scan_u32(v, sc, &tot);
    if (i < L) out[i] = carry + ex;
    carry += tot;
  }
}

static int scan_exclusive_u32(cms_handle* h, const uint32_t* in, uint32_t* out, int64_t L, uint32_t* bsum) {
  if (L <= 0) return CMS_OK;
  int64_t nb = (L + kScanTile - 1) / kScanTile;
  hipLaunchKernelGGL(k_scan_reduce, dim3((unsigned)nb), dim3(kScanThreads), 0, h->stream, in, L, bsum);
  hipLaunchKernelGGL(k_scan_bsum, dim3(1), dim3(1024), 0, h->stream, bsum, nb);
  hipLaunchKernelGGL(k_scan_down, dim3((unsigned)nb), dim3(kScanThreads), 0, h->stream, in, L, bsum, out);
  CMS_HIP(hipGetLastError());
  return CMS_OK;
}

// ------------------------------------------------------------ hash probe --

__global__ void k_hash_keys(const int64_t* keys, int64_t n, HashParams hp, int32_t* out) {
  for (int64_t i = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; i < n; i += (int64_t)gridDim.x * blockDim.x) {
    uint64_t kp = reduce_key(keys[i]);
    for (int r = 0; r < hp.depth; ++r) out[i * hp.depth + r] = (int32_t)bucket(hp, r, kp);
  }
}

int hash_keys_device(cms_handle* h, const int64_t* d_keys, int64_t n, int32_t* d_out) {
  if (n <= 0) return CMS_OK;
  unsigned grid = (unsigned)std::min<int64_t>((n + 255) / 256, 4096);
  hipLaunchKernelGGL(k_hash_keys, dim3(grid), dim3(256), 0, h->stream, d_keys, n, h->hp, d_out);
  CMS_HIP(hipGetLastError());
  return CMS_OK;
}

// ----------------------------------------------------- owner ID -> row --

__global__ void k_map_ids(const int64_t* ids, int64_t n, const int64_t* sorted, int64_t nrows, int64_t* rows,
                          uint32_t* flags) {
  for (int64_t i = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; i < n; i += (int64_t)gridDim.x * blockDim.x) {
    int64_t id = ids[i];
    int64_t lo = 0, hi = nrows;
    while (lo < hi) {
      int64_t mid = (lo + hi) >> 1;
      if (sorted[mid] < id) lo = mid + 1;
      else hi = mid;
    }
    bool found = lo < nrows && sorted[lo] == id;
    rows[i] = found ? lo : -1;
    if (!found) atomicOr(flags, kFlagBadRow);
  }
}

// Pre-ingest validation of host-supplied batches (all-or-nothing ingest).
__global__ void k_validate(const int64_t* rows, const float* val, int64_t n, int64_t nrows, uint32_t* flags) {
  uint32_t f = 0;
  for (int64_t i = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; i < n; i += (int64_t)gridDim.x * blockDim.x) {
    if (rows) {
      int64_t r = rows[i];
      if (r < 0 || r >= nrows) f |= kFlagBadRow;
    }
    uint32_t inc;
    if (val && !load_inc(val, i, inc)) f |= kFlagBadValue;
  }
  if (f) atomicOr(flags, f);
}

int validate_batch(cms_handle* h, const int64_t* d_rows, const float* d_val, int64_t n) {
  if (n <= 0 || (!d_rows && !d_val)) return CMS_OK;
  unsigned grid = (unsigned)std::min<int64_t>((n + 255) / 256, 8192);
  hipLaunchKernelGGL(k_validate, dim3(grid), dim3(256), 0, h->stream, d_rows, d_val, n, h->n, h->d_flags);
  CMS_HIP(hipGetLastError());
  return CMS_OK;
}

int map_owner_ids(cms_handle* h, const int64_t* d_ids, int64_t n, int64_t* d_rows) {
  if (n <= 0) return CMS_OK;
  unsigned grid = (unsigned)std::min<int64_t>((n + 255) / 256, 8192);
  hipLaunchKernelGGL(k_map_ids, dim3(grid), dim3(256), 0, h->stream, d_ids, n, h->d_owner_ids, h->n, d_rows,
                     h->d_flags);
  CMS_HIP(hipGetLastError());
  return CMS_OK;
}

// ------------------------------------------------ small-batch atomic path --

__global__ void k_ingest_atomic(const int64_t* row, const int64_t* key, const float* val, int64_t n, int64_t nrows,
                                HashParams hp, uint32_t* table, uint64_t* row_mass, uint32_t* flags) {
  const int64_t dw = (int64_t)hp.depth * hp.width;
  for (int64_t i = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; i < n; i += (int64_t)gridDim.x * blockDim.x) {
    int64_t r = row[i];
    if (r < 0 || r >= nrows) {
      atomicOr(flags, kFlagBadRow);
      continue;
    }
    uint32_t inc;
    if (!load_inc(val, i, inc)) {
      atomicOr(flags, kFlagBadValue);
      continue;
    }
    if (inc == 0) continue;
    uint64_t kp = reduce_key(key[i]);
    uint32_t* sk = table + r * dw;
    for (int d = 0; d < hp.depth; ++d) atomicAdd(sk + (int64_t)d * hp.width + bucket(hp, d, kp), inc);
    unsigned long long old = atomicAdd((unsigned long long*)&row_mass[r], (unsigned long long)inc);
    if (old + inc >= (1ULL << 32)) atomicOr(flags, kFlagOverflow);
  }
}

// ------------------------------------------- COO -> CSR (MSD partition) --
// pass 1: coarse bin = row >> s2 (P1 bins), pass 2: fine bin = row & (P2-1).

__global__ __launch_bounds__(256) void k_p1_hist(const int64_t* row, int64_t n, int64_t chunk, int s2, int P1,
                                                 int64_t nrows, uint32_t* H1, int NB, uint32_t* flags) {
  extern __shared__ uint32_t lh[];
  for (int b = threadIdx.x; b < P1; b += blockDim.x) lh[b] = 0;
  __syncthreads();
  int64_t lo = (int64_t)blockIdx.x * chunk, hi = min(n, lo + chunk);
  bool bad = false;
  for (int64_t i = lo + threadIdx.x; i < hi; i += blockDim.x) {
    int64_t r = row[i];
    if (r < 0 || r >= nrows) {
      bad = true;
      continue;
    }
    atomicAdd(&lh[(uint32_t)(r >> s2)], 1u);
  }
  if (bad) atomicOr(flags, kFlagBadRow);
  __syncthreads();
  for (int b = threadIdx.x; b < P1; b += blockDim.x) H1[(int64_t)b * NB + blockIdx.x] = lh[b];
}

__global__ __launch_bounds__(256) void k_p1_scatter(const int64_t* row, const int64_t* key, const float* val,
                                                    int64_t n, int64_t chunk, int s2, int P1, int64_t nrows,
                                                    const uint32_t* O1, int NB, uint32_t* orow, int64_t* okey,
                                                    float* oval) {
  extern __shared__ uint32_t cur[];
  for (int b = threadIdx.x; b < P1; b += blockDim.x) cur[b] = O1[(int64_t)b * NB + blockIdx.x];
  __syncthreads();
  int64_t lo = (int64_t)blockIdx.x * chunk, hi = min(n, lo + chunk);
  for (int64_t i = lo + threadIdx.x; i < hi; i += blockDim.x) {
    int64_t r = row[i];
    if (r < 0 || r >= nrows) continue;
    uint32_t pos = atomicAdd(&cur[(uint32_t)(r >> s2)], 1u);
    orow[pos] = (uint32_t)r;
    okey[pos] = key[i];
    if (val) oval[pos] = val[i];
  }
}

// binStart[b] = O1[b*NB] (exclusive, bin-major), binStart[P1] = total;
// blkStart = exclusive scan of ceil(size_b / CH2).  One block.
__global__ __launch_bounds__(1024) void k_p2_plan(const uint32_t* O1, const uint32_t* H1, int NB, int P1,
                                                  int64_t CH2, uint32_t* binStart, uint32_t* blkStart) {
  __shared__ uint32_t sc[1024 / 64 + 1];
  int per = (P1 + 1023) / 1024;
  int lo = threadIdx.x * per, hi = min(P1, lo + per);
  uint32_t s = 0;
  for (int b = lo; b < hi; ++b) {
    uint32_t start = O1[(int64_t)b * NB];
    uint32_t end = (b + 1 < P1) ? O1[(int64_t)(b + 1) * NB]
                                : O1[(int64_t)(P1 - 1) * NB + NB - 1] + H1[(int64_t)(P1 - 1) * NB + NB - 1];
    binStart[b] = start;
    if (b == P1 - 1) binStart[P1] = end;
    s += (uint32_t)((end - start + CH2 - 1) / CH2);
  }
  uint32_t tot;
  uint32_t off = block_excl_scan_u32(s, sc, &tot);
  for (int b = lo; b < hi; ++b) {
    uint32_t start = binStart[b];
    uint32_t end = (b + 1 < P1) ? O1[(int64_t)(b + 1) * NB]
                                : O1[(int64_t)(P1 - 1) * NB + NB - 1] + H1[(int64_t)(P1 - 1) * NB + NB - 1];
    blkStart[b] = off;
    off += (uint32_t)((end - start + CH2 - 1) / CH2);
  }
  if (threadIdx.x == 0) blkStart[P1] = tot;
}

__device__ __forceinline__ int find_bin(const uint32_t* blkStart, int P1, uint32_t x) {
  int lo = 0, hi = P1;  // upper_bound over blkStart[0..P1) then -1
  while (lo < hi) {
    int mid = (lo + hi) >> 1;
    if (blkStart[mid] <= x) lo = mid + 1;
    else hi = mid;
  }
  return lo - 1;
}

__global__ __launch_bounds__(256) void k_p2_hist(const uint32_t* row32, const uint32_t* binStart,
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
  const uint32_t mask = (uint32_t)P2 - 1u;
  for (int64_t i = lo + threadIdx.x; i < hi; i += blockDim.x) atomicAdd(&lh[row32[i] & mask], 1u);
  __syncthreads();
  for (int f = threadIdx.x; f < P2; f += blockDim.x) H2[(int64_t)blockIdx.x * P2 + f] = lh[f];
}

// One block per coarse bin, P2 threads: offsets of (block, fine bin) and the
// CSR row starts of the bin's rows.
__global__ __launch_bounds__(1024) void k_p2_scan(const uint32_t* H2, const uint32_t* binStart,
                                                  const uint32_t* blkStart, int P1, int P2, int64_t nrows,
                                                  uint32_t* O2, int64_t* row_start) {
  __shared__ uint32_t sc[1024 / 64 + 1];
  const int b = blockIdx.x;
  const int f = threadIdx.x;
  const uint32_t k0 = blkStart[b], k1 = blkStart[b + 1];
  uint32_t T = 0;
  if (f < P2)
    for (uint32_t k = k0; k < k1; ++k) T += H2[(int64_t)k * P2 + f];
  uint32_t ex = block_excl_scan_u32(f < P2 ? T : 0u, sc, nullptr);
  if (f < P2) {
    uint32_t base = binStart[b] + ex;
    int64_t r = (int64_t)b * P2 + f;
    if (r < nrows) row_start[r] = base;
    uint32_t run = base;
    for (uint32_t k = k0; k < k1; ++k) {
      uint32_t c = H2[(int64_t)k * P2 + f];
      O2[(int64_t)k * P2 + f] = run;
      run += c;
    }
  }
  if (b == P1 - 1 && f == 0) row_start[nrows] = binStart[P1];
}

__global__ __launch_bounds__(256) void k_p2_scatter(const uint32_t* row32, const int64_t* key1, const float* val1,
                                                    const uint32_t* binStart, const uint32_t* blkStart, int P1,
                                                    int64_t CH2, int P2, const uint32_t* O2, int64_t* okey,
                                                    float* oval) {
  extern __shared__ uint32_t cur[];
  uint32_t nblk = blkStart[P1];
  if (blockIdx.x >= nblk) return;
  int b = find_bin(blkStart, P1, blockIdx.x);
  for (int f = threadIdx.x; f < P2; f += blockDim.x) cur[f] = O2[(int64_t)blockIdx.x * P2 + f];
  __syncthreads();
  int64_t lo = binStart[b] + (int64_t)(blockIdx.x - blkStart[b]) * CH2;
  int64_t hi = min((int64_t)binStart[b + 1], lo + CH2);
  const uint32_t mask = (uint32_t)P2 - 1u;
  for (int64_t i = lo + threadIdx.x; i < hi; i += blockDim.x) {
    uint32_t pos = atomicAdd(&cur[row32[i] & mask], 1u);
    okey[pos] = key1[i];
    if (val1) oval[pos] = val1[i];
  }
}

// --------------------------------------------------------- row build ----

struct HotInfo {
  int64_t row;
  int32_t nslices;
  int32_t slot0;  // first partial slot
};

// Hot rows (more than kSlice pairs) are split into slices built by separate
// workgroups into partial rows, summed by k_reduce_hot.
__global__ void k_build_plan(const int64_t* off, int64_t nrows, int64_t slice, int32_t* row_hot, HotInfo* hot,
                             int2* extra_map, uint32_t* counters /* [0]=hot [1]=slots [2]=extras */,
                             uint64_t* norm, int depth) {
  for (int64_t r = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; r < nrows; r += (int64_t)gridDim.x * blockDim.x) {
    int64_t c = off[r + 1] - off[r];
    if (c <= slice) {
      row_hot[r] = -1;
      continue;
    }
    int32_t ns = (int32_t)((c + slice - 1) / slice);
    uint32_t hidx = atomicAdd(&counters[0], 1u);
    uint32_t slot0 = atomicAdd(&counters[1], (uint32_t)ns);
    uint32_t e0 = atomicAdd(&counters[2], (uint32_t)(ns - 1));
    hot[hidx] = HotInfo{r, ns, (int32_t)slot0};
    row_hot[r] = (int32_t)hidx;
    for (int32_t s = 1; s < ns; ++s) extra_map[e0 + s - 1] = make_int2((int)hidx, s);
    for (int d = 0; d < depth; ++d) norm[r * depth + d] = 0;
  }
}

// grid = emax + nrows.  blocks [0, emax): extra slices of hot rows;
// blocks [emax, emax+nrows): one per row (slice 0 of a hot row).
__global__ __launch_bounds__(kBuildThreads) void k_build_rows(
    const int64_t* off, const int64_t* keys, const float* vals, int64_t nrows, HashParams hp, int64_t slice,
    const int32_t* row_hot, const HotInfo* hot, const int2* extra_map, const uint32_t* counters, int64_t emax,
    uint32_t* table, uint32_t* partials, uint64_t* row_mass, uint64_t* norm, uint32_t* flags, int accumulate) {
  extern __shared__ __align__(16) uint32_t lds[];  // [w] counters + reduce scratch
  uint64_t* red = reinterpret_cast<uint64_t*>(lds + ((hp.width + 3) & ~3));
  const int64_t dw = (int64_t)hp.depth * hp.width;
  const int w = (int)hp.width;

  int64_t row, lo, hi;
  uint32_t* dst;
  bool final_row;
  if (blockIdx.x < emax) {
    if (blockIdx.x >= counters[2]) return;
    int2 m = extra_map[blockIdx.x];
    HotInfo hi_ = hot[m.x];
    row = hi_.row;
    lo = off[row] + (int64_t)m.y * slice;
    hi = min(off[row + 1], lo + slice);
    dst = partials + (int64_t)(hi_.slot0 + m.y) * dw;
    final_row = false;
  } else {
    row = (int64_t)blockIdx.x - emax;
    lo = off[row];
    int32_t hidx = row_hot[row];
    if (hidx >= 0) {
      hi = lo + slice;
      dst = partials + (int64_t)hot[hidx].slot0 * dw;
      final_row = false;
    } else {
      hi = off[row + 1];
      dst = table + row * dw;
      final_row = true;
    }
  }

  uint64_t mass = 0;
  bool badv = false;
  for (int d = 0; d < hp.depth; ++d) {
    uint32_t* dst_d = dst + (int64_t)d * w;
    const bool load_old = final_row && accumulate;
    if ((w & 3) == 0) {
      uint4* l4 = reinterpret_cast<uint4*>(lds);
      const uint4* s4 = reinterpret_cast<const uint4*>(dst_d);
      for (int j = threadIdx.x; j < (w >> 2); j += blockDim.x) l4[j] = load_old ? s4[j] : make_uint4(0, 0, 0, 0);
    } else {
      for (int j = threadIdx.x; j < w; j += blockDim.x) lds[j] = load_old ? dst_d[j] : 0u;
    }
    __syncthreads();
    for (int64_t i = lo + threadIdx.x; i < hi; i += blockDim.x) {
      uint32_t inc;
      if (!load_inc(vals, i, inc)) {
        badv = true;
        continue;
      }
      if (d == 0) mass += inc;
      if (inc == 0) continue;
      uint64_t kp = reduce_key(keys[i]);
      atomicAdd(&lds[bucket(hp, d, kp)], inc);
    }
    __syncthreads();
    uint64_t sq = 0;
    if ((w & 3) == 0) {
      const uint4* l4 = reinterpret_cast<const uint4*>(lds);
      uint4* d4 = reinterpret_cast<uint4*>(dst_d);
      for (int j = threadIdx.x; j < (w >> 2); j += blockDim.x) {
        uint4 v = l4[j];
        d4[j] = v;
        if (final_row) {
          sq = sat_add(sq, (uint64_t)v.x * v.x);
          sq = sat_add(sq, (uint64_t)v.y * v.y);
          sq = sat_add(sq, (uint64_t)v.z * v.z);
          sq = sat_add(sq, (uint64_t)v.w * v.w);
        }
      }
    } else {
      for (int j = threadIdx.x; j < w; j += blockDim.x) {
        uint32_t v = lds[j];
        dst_d[j] = v;
        if (final_row) sq = sat_add(sq, (uint64_t)v * v);
      }
    }
    if (final_row) {
      uint64_t tot = block_sum_u64_sat(sq, red);
      if (threadIdx.x == 0) norm[row * hp.depth + d] = tot;
    }
    __syncthreads();
  }
  if (badv) atomicOr(flags, kFlagBadValue);
  uint64_t tm = block_sum_u64_sat(mass, red);
  if (threadIdx.x == 0) {
    if (final_row) {
      uint64_t m = accumulate ? row_mass[row] + tm : tm;
      row_mass[row] = m;
      if (m >= (1ULL << 32)) atomicOr(flags, kFlagOverflow);
    } else {
      unsigned long long old = atomicAdd((unsigned long long*)&row_mass[row], (unsigned long long)tm);
      if (old + tm >= (1ULL << 32)) atomicOr(flags, kFlagOverflow);
    }
  }
}

// Sum the partial slices of every hot row (plus the old row when
// accumulating) into the table; sums of squares by atomics into norm.
// grid = (chunks of 1024 counters per sketch row, depth, hot rows)
__global__ __launch_bounds__(256) void k_reduce_hot(const HotInfo* hot, const uint32_t* counters, HashParams hp,
                                                    const uint32_t* partials, uint32_t* table, uint64_t* norm,
                                                    int accumulate) {
  __shared__ uint64_t red[4];
  if (blockIdx.z >= counters[0]) return;
  HotInfo hi = hot[blockIdx.z];
  const int d = blockIdx.y;
  const int64_t dw = (int64_t)hp.depth * hp.width;
  const int w = (int)hp.width;
  uint64_t sq = 0;
  for (int j = blockIdx.x * 1024 + threadIdx.x; j < min(w, (int)(blockIdx.x + 1) * 1024); j += 256) {
    int64_t o = (int64_t)d * w + j;
    uint32_t s = accumulate ? table[hi.row * dw + o] : 0u;
    for (int k = 0; k < hi.nslices; ++k) s += partials[(int64_t)(hi.slot0 + k) * dw + o];
    table[hi.row * dw + o] = s;
    sq = sat_add(sq, (uint64_t)s * s);
  }
  uint64_t tot = block_sum_u64_sat(sq, red);
  if (threadIdx.x == 0) atomicAdd((unsigned long long*)&norm[hi.row * hp.depth + d], (unsigned long long)tot);
}

// --------------------------------------------------------- norms pass ----

__global__ __launch_bounds__(256) void k_norms(const uint32_t* table, int64_t nrows, HashParams hp, uint64_t* norm) {
  __shared__ uint64_t red[4];
  const int64_t dw = (int64_t)hp.depth * hp.width;
  const int w = (int)hp.width;
  for (int64_t row = blockIdx.x; row < nrows; row += gridDim.x) {
    for (int d = 0; d < hp.depth; ++d) {
      const uint32_t* p = table + row * dw + (int64_t)d * w;
      uint64_t sq = 0;
      if ((w & 3) == 0) {
        const uint4* p4 = reinterpret_cast<const uint4*>(p);
        for (int j = threadIdx.x; j < (w >> 2); j += blockDim.x) {
          uint4 v = p4[j];
          sq = sat_add(sq, (uint64_t)v.x * v.x);
          sq = sat_add(sq, (uint64_t)v.y * v.y);
          sq = sat_add(sq, (uint64_t)v.z * v.z);
          sq = sat_add(sq, (uint64_t)v.w * v.w);
        }
      } else {
        for (int j = threadIdx.x; j < w; j += blockDim.x) sq = sat_add(sq, (uint64_t)p[j] * p[j]);
      }
      uint64_t tot = block_sum_u64_sat(sq, red);
      if (threadIdx.x == 0) norm[row * hp.depth + d] = tot;
    }
  }
}

// sqrt of every norm (Math.sqrt(valueA), DoubleCountMinSketch.java:143);
// counts (row,d) cells whose norm is not exactly representable in fp64.
__global__ void k_norm_sqrt(const uint64_t* norm, int64_t cells, double* out, uint32_t* inexact) {
  for (int64_t i = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; i < cells; i += (int64_t)gridDim.x * blockDim.x) {
    uint64_t v = norm[i];
    if (v >= (1ULL << 53)) atomicAdd(inexact, 1u);
    out[i] = __dsqrt_rn((double)v);
  }
}

int compute_norms(cms_handle* h) {
  TimedScope ts(h, "norms");
  if (!h->norms_valid) {
    unsigned grid = (unsigned)std::min<int64_t>(h->n, 65536);
    if (grid > 0) hipLaunchKernelGGL(k_norms, dim3(grid), dim3(256), 0, h->stream, h->d_table, h->n, h->hp, h->d_norm);
    CMS_HIP(hipGetLastError());
    h->norms_valid = true;
  }
  int64_t cells = h->n * h->p.depth;
  CMS_HIP(hipMemsetAsync(h->d_flags + 1, 0, sizeof(uint32_t), h->stream));
  if (cells > 0) {
    unsigned grid = (unsigned)std::min<int64_t>((cells + 255) / 256, 8192);
    hipLaunchKernelGGL(k_norm_sqrt, dim3(grid), dim3(256), 0, h->stream, h->d_norm, cells, h->d_norm_sqrt,
                       h->d_flags + 1);
  }
  CMS_HIP(hipGetLastError());
  return CMS_OK;
}

// -------------------------------------------------------------- drivers --

static int ceil_log2(int64_t v) {
  int b = 0;
  while ((int64_t(1) << b) < v) ++b;
  return b;
}

int ingest_csr_device(cms_handle* h, const int64_t* d_off, const int64_t* d_key, const float* d_val, int64_t npairs) {
  const int64_t n = h->n;
  const int64_t dw = h->dw;
  const int accumulate = h->empty ? 0 : 1;
  // scratch: row_hot[n] i32, hot[n] HotInfo (bounded by npairs/slice), extra_map, counters
  int64_t max_hot = std::min<int64_t>(n, npairs / kSlice + 1);
  int64_t emax = npairs / kSlice + 1;
  size_t sz_rowhot = sizeof(int32_t) * (size_t)n;
  size_t sz_hot = sizeof(HotInfo) * (size_t)max_hot;
  size_t sz_extra = sizeof(int2) * (size_t)emax;
  size_t need = sz_rowhot + sz_hot + sz_extra + 64;
  CMS_HIP(h->ws_hot.ensure(need));
  char* base = h->ws_hot.as<char>();
  int32_t* row_hot = reinterpret_cast<int32_t*>(base);
  HotInfo* hot = reinterpret_cast<HotInfo*>(base + ((sz_rowhot + 15) & ~size_t(15)));
  int2* extra_map = reinterpret_cast<int2*>(reinterpret_cast<char*>(hot) + ((sz_hot + 15) & ~size_t(15)));
  uint32_t* counters = h->d_flags + 4;  // [4..7]
  CMS_HIP(hipMemsetAsync(counters, 0, 4 * sizeof(uint32_t), h->stream));
  {
    TimedScope ts(h, "build_plan");
    unsigned grid = (unsigned)std::max<int64_t>(1, std::min<int64_t>((n + 255) / 256, 4096));
    hipLaunchKernelGGL(k_build_plan, dim3(grid), dim3(256), 0, h->stream, d_off, n, kSlice, row_hot, hot, extra_map,
                       counters, h->d_norm, h->p.depth);
    CMS_HIP(hipGetLastError());
  }
  // partial slots <= npairs/slice + hot rows
  int64_t max_slots = npairs / kSlice + max_hot;
  CMS_HIP(h->ws_partials.ensure(sizeof(uint32_t) * (size_t)std::max<int64_t>(1, max_slots) * (size_t)dw));
  size_t lds = sizeof(uint32_t) * (size_t)((h->p.width + 3) & ~3) + 8 * sizeof(uint64_t);
  {
    TimedScope ts(h, "build_rows");
    hipLaunchKernelGGL(k_build_rows, dim3((unsigned)(emax + n)), dim3(kBuildThreads), lds, h->stream, d_off, d_key,
                       d_val, n, h->hp, kSlice, row_hot, hot, extra_map, counters, emax, h->d_table,
                       h->ws_partials.as<uint32_t>(), h->d_row_mass, h->d_norm, h->d_flags, accumulate);
    CMS_HIP(hipGetLastError());
  }
  {
    TimedScope ts(h, "reduce_hot");
    dim3 grid((unsigned)((h->p.width + 1023) / 1024), (unsigned)h->p.depth, (unsigned)std::max<int64_t>(1, max_hot));
    hipLaunchKernelGGL(k_reduce_hot, grid, dim3(256), 0, h->stream, hot, counters, h->hp,
                       h->ws_partials.as<uint32_t>(), h->d_table, h->d_norm, accumulate);
    CMS_HIP(hipGetLastError());
  }
  h->empty = false;
  h->norms_valid = true;  // build_rows + reduce_hot wrote the norm of every row
  return CMS_OK;
}

int ingest_coo_device(cms_handle* h, const int64_t* d_row, const int64_t* d_key, const float* d_val, int64_t npairs) {
  if (npairs <= 0) return CMS_OK;
  const int64_t n = h->n;
  // Small batch into a live table: exact global atomics.
  const bool small = npairs < 262144 || npairs * 8 < n;
  if (small || npairs >= (int64_t(1) << 31)) {
    if (npairs >= (int64_t(1) << 31)) {
      // split very large batches into partition-sized pieces
      const int64_t piece = int64_t(1) << 30;
      for (int64_t o = 0; o < npairs; o += piece) {
        int rc = ingest_coo_device(h, d_row + o, d_key + o, d_val ? d_val + o : nullptr, std::min(piece, npairs - o));
        if (rc) return rc;
      }
      return CMS_OK;
    }
    TimedScope ts(h, "ingest_atomic");
    if (h->empty) {
      CMS_HIP(hipMemsetAsync(h->d_table, 0, sizeof(uint32_t) * (size_t)(n * h->dw), h->stream));
      CMS_HIP(hipMemsetAsync(h->d_row_mass, 0, sizeof(uint64_t) * (size_t)n, h->stream));
    }
    unsigned grid = (unsigned)std::min<int64_t>((npairs + 255) / 256, 16384);
    hipLaunchKernelGGL(k_ingest_atomic, dim3(grid), dim3(256), 0, h->stream, d_row, d_key, d_val, npairs, n, h->hp,
                       h->d_table, h->d_row_mass, h->d_flags);
    CMS_HIP(hipGetLastError());
    h->empty = false;
    h->norms_valid = false;
    return CMS_OK;
  }

  // ---- partition into CSR ----
  const int B = std::max(1, ceil_log2(n));
  const int s2 = std::min(B, 10);
  const int P2 = 1 << s2;
  const int P1 = (int)((n + P2 - 1) / P2);
  if (P1 > 16384) return set_error(CMS_E_PARAM, "num_owners %lld too large for the partition", (long long)n);
  const int64_t chunk1 = std::max<int64_t>(16384, (npairs + 2047) / 2048);
  const int NB = (int)((npairs + chunk1 - 1) / chunk1);
  const int64_t CH2 = 16384;
  const int64_t nb2max = npairs / CH2 + P1 + 1;

  CMS_HIP(h->ws_p1_row.ensure(sizeof(uint32_t) * (size_t)npairs));
  CMS_HIP(h->ws_p1_key.ensure(sizeof(int64_t) * (size_t)npairs));
  if (d_val) CMS_HIP(h->ws_p1_val.ensure(sizeof(float) * (size_t)npairs));
  CMS_HIP(h->ws_csr_key.ensure(sizeof(int64_t) * (size_t)npairs));
  if (d_val) CMS_HIP(h->ws_csr_val.ensure(sizeof(float) * (size_t)npairs));
  CMS_HIP(h->ws_csr_off.ensure(sizeof(int64_t) * (size_t)(n + 1)));
  // hist area: H1 + O1 [P1*NB], H2 + O2 [nb2max*P2], bsum, binStart, blkStart
  const int64_t L1 = (int64_t)P1 * NB, L2 = nb2max * P2;
  const int64_t nbs = (std::max(L1, L2) + kScanTile - 1) / kScanTile + 1;
  size_t hist_words = (size_t)(2 * L1 + 2 * L2 + nbs + 2 * (P1 + 1) + 64);
  CMS_HIP(h->ws_hist.ensure(sizeof(uint32_t) * hist_words));
  uint32_t* H1 = h->ws_hist.as<uint32_t>();
  uint32_t* O1 = H1 + L1;
  uint32_t* H2 = O1 + L1;
  uint32_t* O2 = H2 + L2;
  uint32_t* bsum = O2 + L2;
  uint32_t* binStart = bsum + nbs;
  uint32_t* blkStart = binStart + (P1 + 1);

  uint32_t* row32 = h->ws_p1_row.as<uint32_t>();
  int64_t* key1 = h->ws_p1_key.as<int64_t>();
  float* val1 = d_val ? h->ws_p1_val.as<float>() : nullptr;
  int64_t* ckey = h->ws_csr_key.as<int64_t>();
  float* cval = d_val ? h->ws_csr_val.as<float>() : nullptr;
  int64_t* coff = h->ws_csr_off.as<int64_t>();
  {
    TimedScope ts(h, "partition");
    hipLaunchKernelGGL(k_p1_hist, dim3(NB), dim3(256), sizeof(uint32_t) * P1, h->stream, d_row, npairs, chunk1, s2,
                       P1, n, H1, NB, h->d_flags);
    int rc = scan_exclusive_u32(h, H1, O1, L1, bsum);
    if (rc) return rc;
    hipLaunchKernelGGL(k_p1_scatter, dim3(NB), dim3(256), sizeof(uint32_t) * P1, h->stream, d_row, d_key, d_val,
                       npairs, chunk1, s2, P1, n, O1, NB, row32, key1, val1);
    hipLaunchKernelGGL(k_p2_plan, dim3(1), dim3(1024), 0, h->stream, O1, H1, NB, P1, CH2, binStart, blkStart);
    hipLaunchKernelGGL(k_p2_hist, dim3((unsigned)nb2max), dim3(256), sizeof(uint32_t) * P2, h->stream, row32,
                       binStart, blkStart, P1, CH2, P2, H2);
    hipLaunchKernelGGL(k_p2_scan, dim3(P1), dim3(std::max(64, P2)), 0, h->stream, H2, binStart, blkStart, P1, P2, n,
                       O2, coff);
    hipLaunchKernelGGL(k_p2_scatter, dim3((unsigned)nb2max), dim3(256), sizeof(uint32_t) * P2, h->stream, row32,
                       key1, val1, binStart, blkStart, P1, CH2, P2, O2, ckey, cval);
    CMS_HIP(hipGetLastError());
  }
  return ingest_csr_device(h, coff, ckey, cval, npairs);
}

}  // namespace cms
