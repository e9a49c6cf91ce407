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
//   (k_build_rows lives in cms_build.hip)
// so every table byte is written exactly once (the zero fill is fused) and
// the stream is read a small constant number of times.  Small batches into a
// non-empty table use k_ingest_atomic (global atomics, exact for u32).
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cstdint>
#include <cstdlib>

#include "cms_device.h"
#include "cms_internal.h"

namespace cms {

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

int scan_exclusive_u32(cms_handle* h, const uint32_t* in, uint32_t* out, int64_t L, uint32_t* bsum) {
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
__global__ void k_validate(const int64_t* rows, const float* val, int64_t n, int64_t nrows, int fb, uint32_t* flags) {
  uint32_t f = 0;
  for (int64_t i = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; i < n; i += (int64_t)gridDim.x * blockDim.x) {
    if (rows) {
      int64_t r = rows[i];
      if (r < 0 || r >= nrows) f |= kFlagBadRow;
    }
    uint32_t inc;
    if (val && !load_inc(val, i, inc, fb)) f |= kFlagBadValue;
  }
  if (f) atomicOr(flags, f);
}

// CSR offsets from the caller: offsets[0] == 0 and non-decreasing, so every
// owner's range lies inside [0, offsets[n]).
__global__ void k_check_offsets(const int64_t* off, int64_t n, uint32_t* flags) {
  for (int64_t r = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; r < n; r += (int64_t)gridDim.x * blockDim.x) {
    if ((r == 0 && off[0] != 0) || off[r + 1] < off[r]) {
      atomicOr(flags, kFlagBadRow);
      return;
    }
  }
}

int check_offsets_device(cms_handle* h, const int64_t* d_off) {
  const unsigned grid = (unsigned)std::max<int64_t>(1, std::min<int64_t>((h->n + 255) / 256, 4096));
  hipLaunchKernelGGL(k_check_offsets, dim3(grid), dim3(256), 0, h->stream, d_off, h->n, h->d_flags);
  CMS_HIP(hipGetLastError());
  return CMS_OK;
}

int validate_batch(cms_handle* h, const int64_t* d_rows, const float* d_val, int64_t n) {
  if (n <= 0 || (!d_rows && !d_val)) return CMS_OK;
  unsigned grid = (unsigned)std::min<int64_t>((n + 255) / 256, 8192);
  hipLaunchKernelGGL(k_validate, dim3(grid), dim3(256), 0, h->stream, d_rows, d_val, n, h->n, h->hp.frac_bits, h->d_flags);
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

// counter c of row r += inc; returns the old value.  Narrow rows add into
// their half of the aligned 32-bit word: promote_rows guarantees the row's
// bound stays < 2^16, so no carry reaches the neighbouring half.
// u8 / 4-bit / 2-bit / 1-bit rows add into their byte / nibble / bits of the aligned word the same
// way: widen_rows ran first, so the row's counter bound stays within its form.
__device__ __forceinline__ uint32_t table_add(const TableView& tv, int64_t r, int64_t c, uint32_t inc) {
  const int32_t s = tv.hidx[r];
  if (s >= 0) return atomicAdd(tv.hot + (int64_t)s * tv.dw + c, inc);
  if (s == kFormU16) {
    const int64_t g = tv.base(r) + c;  // (the row's base is even: 64-B aligned)
    const uint32_t sh = (uint32_t)(g & 1) << 4;
    const uint32_t old = atomicAdd(reinterpret_cast<uint32_t*>(tv.t16) + (g >> 1), inc << sh);
    return (old >> sh) & 0xffffu;
  }
  if (s == kFormList) return tv.get(r, c);  // only inc == 0 reaches a list row (any mass widens it first)
  uint32_t* w32 = reinterpret_cast<uint32_t*>(tv.row16(r));  // slot start: 64-B aligned
  if (s == kFormU8) {
    const uint32_t sh = (uint32_t)(c & 3) << 3;
    return (atomicAdd(w32 + (c >> 2), inc << sh) >> sh) & 0xffu;
  }
  if (s == kFormU2) {
    const uint32_t sh = (uint32_t)(c & 15) << 1;
    return (atomicAdd(w32 + (c >> 4), inc << sh) >> sh) & 0x3u;
  }
  if (s == kFormU1) {
    const uint32_t sh = (uint32_t)(c & 31);
    return (atomicAdd(w32 + (c >> 5), inc << sh) >> sh) & 0x1u;
  }
  const uint32_t sh = (uint32_t)(c & 7) << 2;
  return (atomicAdd(w32 + (c >> 3), inc << sh) >> sh) & 0xfu;
}

// batch mass per row (counter units) for the promotion check of unsorted batches
__global__ void k_batch_mass(const int64_t* row, const float* val, int64_t n, int64_t nrows, int fb, uint64_t* delta) {
  for (int64_t i = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; i < n; i += (int64_t)gridDim.x * blockDim.x) {
    const int64_t r = row[i];
    uint32_t inc;
    if (r < 0 || r >= nrows || !load_inc(val, i, inc, fb) || inc == 0) continue;
    atomicAdd((unsigned long long*)&delta[r], (unsigned long long)inc);
  }
}

__global__ void k_bound_from_delta(const uint64_t* delta, const uint64_t* mass, int64_t n, uint64_t* bound) {
  for (int64_t r = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; r < n; r += (int64_t)gridDim.x * blockDim.x)
    bound[r] = delta[r] ? sat_add(delta[r], mass[r]) : 0ULL;
}

// With `track`, the norms and row maxima stay current: a counter moving from
// c to c+inc adds 2*c*inc + inc^2 to its sum of squares, and the per-update
// deltas telescope to the exact new sum whatever the atomic order.  A norm
// reaching 2^53 (inexact fp64 regime) raises flags[2] so finalize recomputes.
__global__ void k_ingest_atomic(const int64_t* row, const int64_t* key, const float* val, int64_t n, int64_t nrows,
                                HashParams hp, TableView tv, uint64_t* row_mass, uint64_t* norm, uint32_t* rowmax,
                                int track, uint32_t* flags) {
  for (int64_t i = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; i < n; i += (int64_t)gridDim.x * blockDim.x) {
    int64_t r = row[i];
    if (r < 0 || r >= nrows) {
      atomicOr(flags, kFlagBadRow);
      continue;
    }
    uint32_t inc;
    if (!load_inc(val, i, inc, hp.frac_bits)) {
      atomicOr(flags, kFlagBadValue);
      continue;
    }
    if (inc == 0) continue;
    uint64_t kp = reduce_key(key[i]);
    uint32_t cmax = 0;
    for (int d = 0; d < hp.depth; ++d) {
      uint32_t c = table_add(tv, r, (int64_t)d * hp.width + bucket(hp, d, kp), inc);
      if (track) {
        uint64_t delta = 2ULL * c * inc + (uint64_t)inc * inc;
        unsigned long long o = atomicAdd((unsigned long long*)&norm[r * hp.depth + d], (unsigned long long)delta);
        if (o + delta >= (1ULL << 53)) atomicOr(flags + 2, 1u);
        cmax = max(cmax, c + inc);
      }
    }
    if (track) atomicMax(&rowmax[r], cmax);
    unsigned long long old = atomicAdd((unsigned long long*)&row_mass[r], (unsigned long long)inc);
    if (old + inc >= (1ULL << 32)) atomicOr(flags, kFlagOverflow);
  }
}

// Incremental batch already grouped by owner (partition_to_csr with per-pair
// rows): the same exact counter atomics, but the norm / row-max / mass updates
// of the lanes of one owner are reduced inside the wave first (rows are
// non-decreasing along the lanes, so each owner is one contiguous lane run),
// so a hot owner costs one atomic per wave instead of one per pair.
__device__ __forceinline__ uint64_t seg_suffix_sum(uint64_t v, int32_t r, int lane) {
#pragma unroll
  for (int o = 1; o < 64; o <<= 1) {
    uint64_t ov = __shfl_down(v, o, 64);
    int32_t orr = __shfl_down(r, o, 64);
    if (lane + o < 64 && orr == r) v += ov;
  }
  return v;
}

__global__ __launch_bounds__(256) void k_ingest_sorted(const int32_t* rows, Keys keys, const float* val,
                                                        const int64_t* count, HashParams hp, TableView tv,
                                                        uint64_t* row_mass, uint64_t* norm, uint32_t* rowmax,
                                                        uint32_t* flags) {
  const int64_t n = *count;  // pairs that survived the partition's row check
  const int lane = threadIdx.x & 63;
  for (int64_t base = (int64_t)blockIdx.x * blockDim.x; base < n; base += (int64_t)gridDim.x * blockDim.x) {
    const int64_t i = base + threadIdx.x;
    int32_t r = -1;
    uint32_t inc = 0;
    uint64_t kp = 0;
    if (i < n) {
      r = rows[i];
      if (!load_inc(val, i, inc, hp.frac_bits)) {
        atomicOr(flags, kFlagBadValue);
        inc = 0;
      }
      kp = keys.at(i);
    }
    const int32_t rprev = __shfl_up(r, 1, 64);
    const bool head = r >= 0 && (lane == 0 || rprev != r);
    uint32_t cmax = 0;
    for (int d = 0; d < hp.depth; ++d) {
      uint64_t delta = 0;
      if (inc) {
        uint32_t c = table_add(tv, r, (int64_t)d * hp.width + bucket(hp, d, kp), inc);
        delta = 2ULL * c * inc + (uint64_t)inc * inc;
        cmax = max(cmax, c + inc);
      }
      delta = seg_suffix_sum(delta, r, lane);
      if (head && delta) {
        unsigned long long o = atomicAdd((unsigned long long*)&norm[(int64_t)r * hp.depth + d], (unsigned long long)delta);
        if (o + delta >= (1ULL << 53)) atomicOr(flags + 2, 1u);
      }
    }
    uint64_t mass = seg_suffix_sum((uint64_t)inc, r, lane);
#pragma unroll
    for (int o = 1; o < 64; o <<= 1) {
      uint32_t om = (uint32_t)__shfl_down((int)cmax, o, 64);
      int32_t orr = __shfl_down(r, o, 64);
      if (lane + o < 64 && orr == r) cmax = max(cmax, om);
    }
    if (head && mass) {
      atomicMax(&rowmax[r], cmax);
      unsigned long long old = atomicAdd((unsigned long long*)&row_mass[r], (unsigned long long)mass);
      if (old + mass >= (1ULL << 32)) atomicOr(flags, kFlagOverflow);
    }
  }
}

// --------------------------------------------------------- norms pass ----

__global__ __launch_bounds__(256) void k_norms(TableView tv, int64_t nrows, HashParams hp, uint64_t* norm,
                                               uint32_t* rowmax) {
  __shared__ uint64_t red[4];
  __shared__ uint32_t smax[4];
  extern __shared__ uint32_t lc[];  // [w / 4]: a list row's sketch row as u8 counters
  const int w = (int)hp.width;
  for (int64_t row = blockIdx.x; row < nrows; row += gridDim.x) {
    uint32_t vmax = 0;
    const bool list = tv.hidx[row] == kFormList;
    const uint32_t lm = list ? tv.list_m(row) : 0u;
    for (int d = 0; d < hp.depth; ++d) {
      const int64_t c0 = (int64_t)d * w;
      uint64_t sq = 0;
      if (list) {  // the sketch row counted in LDS (u8 counters, four per word: a list row's are < 2^8)
        const uint16_t* e = tv.list_row(row, d, lm);
        for (int j = threadIdx.x; j < (w >> 2); j += blockDim.x) lc[j] = 0u;
        __syncthreads();
        for (uint32_t t = threadIdx.x; t < lm; t += blockDim.x) atomicAdd(&lc[e[t] >> 2], 1u << ((e[t] & 3u) * 8u));
        __syncthreads();
        for (int j = threadIdx.x; j < (w >> 2); j += blockDim.x) {
          const uint32_t v = lc[j];
          sq += __builtin_amdgcn_udot4(v, v, 0u, false);
          vmax = max(vmax, max(max(v & 255u, (v >> 8) & 255u), max((v >> 16) & 255u, v >> 24)));
        }
        __syncthreads();
      } else if ((w & 3) == 0) {
        for (int j = threadIdx.x; j < (w >> 2); j += blockDim.x) {
          const uint4 v = tv.get4(row, c0 + 4 * j);
          vmax = max(vmax, max(max(v.x, v.y), max(v.z, v.w)));
          sq = sat_add(sq, (uint64_t)v.x * v.x);
          sq = sat_add(sq, (uint64_t)v.y * v.y);
          sq = sat_add(sq, (uint64_t)v.z * v.z);
          sq = sat_add(sq, (uint64_t)v.w * v.w);
        }
      } else {
        for (int j = threadIdx.x; j < w; j += blockDim.x) {
          const uint32_t v = tv.get(row, c0 + j);
          sq = sat_add(sq, (uint64_t)v * v);
          vmax = max(vmax, v);
        }
      }
      uint64_t tot = block_sum_u64_sat(sq, red);
      if (threadIdx.x == 0) norm[row * hp.depth + d] = tot;
    }
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) vmax = max(vmax, (uint32_t)__shfl_xor((int)vmax, o, 64));
    if ((threadIdx.x & 63) == 0) smax[threadIdx.x >> 6] = vmax;
    __syncthreads();
    if (threadIdx.x == 0) rowmax[row] = max(max(smax[0], smax[1]), max(smax[2], smax[3]));
    __syncthreads();
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

int local_norms(cms_handle* h) {
  const unsigned grid = (unsigned)std::min<int64_t>(h->n, 65536);
  if (grid > 0)
    hipLaunchKernelGGL(k_norms, dim3(grid), dim3(256), (size_t)h->p.width, h->stream, h->tview(), h->n, h->hp, h->d_norm,
                       h->d_rowmax);
  CMS_HIP(hipGetLastError());
  h->norms_valid = true;
  return CMS_OK;
}

int compute_norms(cms_handle* h) {
  TimedScope ts(h, "norms");
  if (h->stale_possible && h->norms_valid) {  // an incremental norm may have reached the inexact regime
    CMS_HIP(hipMemcpyAsync(h->h_pin + 2, h->d_flags + 2, sizeof(uint32_t), hipMemcpyDeviceToHost, h->stream));
    CMS_HIP(hipStreamSynchronize(h->stream));
    if (h->h_pin[2]) h->norms_valid = false;
  }
  h->stale_possible = false;
  if (!h->norms_valid) {
    CMS_HIP(hipMemsetAsync(h->d_flags + 2, 0, sizeof(uint32_t), h->stream));
    unsigned grid = (unsigned)std::min<int64_t>(h->n, 65536);
    if (grid > 0) hipLaunchKernelGGL(k_norms, dim3(grid), dim3(256), (size_t)h->p.width, h->stream, h->tview(), h->n,
                                     h->hp, h->d_norm, h->d_rowmax);
    CMS_HIP(hipGetLastError());
    h->norms_valid = true;
  }
  int64_t cells = h->n * h->p.depth;
  if (!h->inexact_zero) CMS_HIP(hipMemsetAsync(h->d_flags + 1, 0, sizeof(uint32_t), h->stream));
  h->inexact_zero = false;  // until a read-back sees 0
  if (cells > 0) {
    unsigned grid = (unsigned)std::min<int64_t>((cells + 255) / 256, 8192);
    hipLaunchKernelGGL(k_norm_sqrt, dim3(grid), dim3(256), 0, h->stream, h->d_norm, cells, h->d_norm_sqrt,
                       h->d_flags + 1);
  }
  CMS_HIP(hipGetLastError());
  return CMS_OK;
}

// -------------------------------------------------------------- drivers --

int ingest_coo_device(cms_handle* h, const int64_t* d_row, const int64_t* d_key, const float* d_val, int64_t npairs) {
  if (npairs <= 0) return CMS_OK;
  const int64_t n = h->n;
  if (h->rf_valid) {  // kept refresh lists: the batch's owners are recomputed by the next refresh
    if (int rc = refresh_mark(h, d_row, npairs)) return rc;
  }
  // Global atomics for a small batch, and for any batch into a live table
  // unless its atomic traffic (~d sector RMWs per pair) exceeds the
  // accumulate build's full-table read + write.
  const double table_bytes = 4.0 * (double)n * (double)h->dw;
  const bool small = npairs < 262144 || npairs * 8 < n ||
                     (!h->empty && (double)npairs * h->p.depth * 128.0 < 2.0 * table_bytes);
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
    if (!h->empty && h->norms_valid && npairs >= 32768 && n < (int64_t(1) << 31)) {
      // live table with current norms: group by owner, then wave-reduced atomics
      int64_t* coff;
      uint32_t* ctok;
      float* cval;
      CMS_HIP(h->ws_srow.ensure(sizeof(int32_t) * (size_t)npairs));
      int rc = partition_to_csr(h, d_row, d_key, d_val, npairs, &coff, &ctok, &cval, h->ws_srow.as<int32_t>());
      if (rc) return rc;
      {  // rows this batch could lift to 2^16 move to u32 slots first
        DevBuf& bound = h->ws_bound;
        DevBuf& force = h->ws_force;
        CMS_HIP(bound.ensure(sizeof(uint64_t) * (size_t)n));
        CMS_HIP(force.ensure((size_t)n));
        if ((rc = row_bounds(h, coff, coff + 1, cval, h->d_row_mass, INT64_MAX, bound.as<uint64_t>(),
                             force.as<uint8_t>())))
          return rc;
        if ((rc = promote_rows(h, bound.as<uint64_t>(), nullptr, true))) return rc;
        // u8 / nibble rows the batch could push past their form become u16
        if ((rc = widen_rows(h, bound.as<uint64_t>(), h->d_row_mass, false))) return rc;
      }
      TimedScope ts(h, "ingest_sorted");
      h->stale_possible = true;
      unsigned grid = (unsigned)std::min<int64_t>((npairs + 255) / 256, 16384);
      hipLaunchKernelGGL(k_ingest_sorted, dim3(grid), dim3(256), 0, h->stream, h->ws_srow.as<int32_t>(), Keys{d_key, ctok}, cval,
                         coff + n, h->hp, h->tview(), h->d_row_mass, h->d_norm, h->d_rowmax, h->d_flags);
      CMS_HIP(hipGetLastError());
      return CMS_OK;
    }
    TimedScope ts(h, "ingest_atomic");
    if (h->empty) {
      int rc = reset_rows_zero(h);
      if (rc) return rc;
      CMS_HIP(hipMemsetAsync(h->d_row_mass, 0, sizeof(uint64_t) * (size_t)n, h->stream));
      CMS_HIP(hipMemsetAsync(h->d_norm, 0, sizeof(uint64_t) * (size_t)(n * h->p.depth), h->stream));
      CMS_HIP(hipMemsetAsync(h->d_rowmax, 0, sizeof(uint32_t) * (size_t)n, h->stream));
      h->norms_valid = true;
    }
    {  // rows this batch could lift to 2^16 move to u32 slots first
      DevBuf& delta = h->ws_partials;  // scratch reused: [n] batch masses
      DevBuf& bound = h->ws_bound;
      CMS_HIP(delta.ensure(sizeof(uint64_t) * (size_t)n));
      CMS_HIP(bound.ensure(sizeof(uint64_t) * (size_t)n));
      CMS_HIP(hipMemsetAsync(delta.ptr, 0, sizeof(uint64_t) * (size_t)n, h->stream));
      const unsigned gp = (unsigned)std::min<int64_t>((npairs + 255) / 256, 16384);
      const unsigned gn = (unsigned)std::max<int64_t>(1, std::min<int64_t>((n + 255) / 256, 8192));
      hipLaunchKernelGGL(k_batch_mass, dim3(gp), dim3(256), 0, h->stream, d_row, d_val, npairs, n, h->hp.frac_bits,
                         delta.as<uint64_t>());
      hipLaunchKernelGGL(k_bound_from_delta, dim3(gn), dim3(256), 0, h->stream, delta.as<uint64_t>(), h->d_row_mass, n,
                         bound.as<uint64_t>());
      CMS_HIP(hipGetLastError());
      int rc = promote_rows(h, bound.as<uint64_t>(), nullptr, true);
      if (rc) return rc;
      if ((rc = widen_rows(h, bound.as<uint64_t>(), h->d_row_mass, false))) return rc;
    }
    const int track = h->norms_valid ? 1 : 0;
    h->stale_possible = true;
    unsigned grid = (unsigned)std::min<int64_t>((npairs + 255) / 256, 16384);
    hipLaunchKernelGGL(k_ingest_atomic, dim3(grid), dim3(256), 0, h->stream, d_row, d_key, d_val, npairs, n, h->hp,
                       h->tview(), h->d_row_mass, h->d_norm, h->d_rowmax, track, h->d_flags);
    CMS_HIP(hipGetLastError());
    h->empty = false;
    return CMS_OK;
  }

  // ---- group by owner (cms_partition.hip), then the LDS row build ----
  int64_t *clo, *chi;
  uint32_t* ctok;
  float* cval;
  int rc = kNoSpans;
  // the partition marks its spans ready before its last scatter, and the
  // build plan (which needs only the spans) runs beside that scatter
  h->plan_side_request = h->tune.plan_side != 0;
  h->spans_event = false;
  if (h->tune.hot_routing) rc = partition_to_spans(h, d_row, d_key, d_val, npairs, &clo, &chi, &ctok, &cval);
  if (rc == kNoSpans) {
    rc = partition_to_csr(h, d_row, d_key, d_val, npairs, &clo, &ctok, &cval);
    chi = clo + 1;
  }
  h->plan_side_request = false;
  if (rc) {
    h->spans_event = false;
    return rc;
  }
  rc = ingest_spans_device(h, clo, chi, d_key, ctok, cval, npairs);
  h->spans_event = false;
  return rc;
}

}  // namespace cms
