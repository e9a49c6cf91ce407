// cms_build.hip -- LDS-staged sketch-row build (the sketch-update hot kernel).
//
// Input: CSR keys grouped by owner row (the DataModel layout, or the output of
// the COO partition in cms_ingest.hip).  One workgroup builds one owner's
// d x w sketch one sketch row at a time in LDS:
//   - the owner's keys are read once (cached in registers across the d sketch
//     rows when the owner has <= 1024 keys, otherwise streamed in batches of
//     four loads per thread) and reduced mod p once;
//   - every update of sketch row r is an LDS atomic add at h_r(key)
//     (DoubleCountMinSketch.update, T/impl/common/DoubleCountMinSketch.java:72-80);
//   - the finished row leaves LDS as 16-byte coalesced stores, the same pass
//     zeroes the LDS slot for row r+1 and accumulates sum(c^2) (the valueA of
//     DoubleCountMinSketch.cosine :131-138) -- so the table is written exactly
//     once, zero fill included, and the norms cost no extra HBM pass.
// Hot owners (more than kSlice keys) are split into slices built by separate
// workgroups; a slice adds its LDS row into the (pre-zeroed) table row with
// 256-byte coalesced atomics and a small pass derives the hot rows' norms.
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cstdlib>

#include "cms_device.h"
#include "cms_internal.h"

namespace cms {

#ifdef CMS_BUILD_CHEAPHASH  // bound analysis only: a trivial hash instead of the exact mod-p one
#define bucket(hp, d, kp) ((uint32_t)(((kp) >> (d)) & (hp).wmask))
#endif
#ifdef CMS_BUILD_GATHERHASH  // bound analysis only: the row's bucket gathered from a per-key table
#define bucket(hp, d, kp) \
  ((uint32_t)(((&(hp).gtab[(kp) & 0xFFFFFFu].x)[((d) >> 1) & 3] >> (((d) & 1) << 4)) & (hp).wmask))
#endif

struct HotInfo {
  int64_t row;
  int32_t nslices;
  int32_t e0;  // first extra slice (extra_map index) of the row
};

#ifndef CMS_KEY_REGS
#define CMS_KEY_REGS 4
#endif
constexpr int kKeyRegs = CMS_KEY_REGS;

typedef unsigned short u16x2 __attribute__((ext_vector_type(2)));  // keys cached per thread: owners up to 1024 keys are read once

// 8 byte counters (each < 16) of two words -> 8 nibbles, counter k in bits 4k:
// x | x >> 4 puts counters 0|1 in byte 0 and 2|3 in byte 2; one v_perm_b32
// gathers bytes 0 and 2 of both words.
__device__ __forceinline__ uint32_t nibbles8(uint32_t lo, uint32_t hi) {
  return __builtin_amdgcn_perm(hi | (hi >> 4), lo | (lo >> 4), 0x06040200u);
}

// Rows with more than `split` keys are hot (u32 slot, built in slices of
// `slice` keys); slices [first, ns) of each are listed in extra_map (first =
// 1: slice 0 is built by the row's own k_build_rows block; first = 0: every
// slice by k_build_slices).
__global__ void k_build_plan(const int64_t* lo_, const int64_t* hi_, int64_t nrows, int64_t split, int64_t slice,
                             int first, int32_t* row_hot, HotInfo* hot, int2* extra_map,
                             uint32_t* counters /* [0]=hot rows [1]=mapped slices */, uint64_t* norm, uint32_t* rowmax,
                             int depth, const uint8_t* early) {
  const int lane = (int)__lane_id();
  for (int64_t base = blockIdx.x * (int64_t)blockDim.x; base < nrows; base += (int64_t)gridDim.x * blockDim.x) {
    const int64_t r = base + threadIdx.x;
    const int64_t c = r < nrows ? hi_[r] - lo_[r] : 0;
    const bool is_hot = c > split && !(early && early[r]);  // (an early row is built already: k_early_plan)
    if (r < nrows && !is_hot) row_hot[r] = -1;
    int32_t ns = 0;
    uint32_t hidx = 0, e0 = 0;
    if (is_hot) {
      ns = (int32_t)((c + slice - 1) / slice);
      // one 64-bit atomic claims the hot index (low word) and the mapped slices (high word)
      const unsigned long long old =
          atomicAdd(reinterpret_cast<unsigned long long*>(counters), ((unsigned long long)(ns - first) << 32) | 1ULL);
      hidx = (uint32_t)old;
      e0 = (uint32_t)(old >> 32);
      hot[hidx] = HotInfo{r, ns, (int32_t)e0};
      row_hot[r] = (int32_t)hidx;
      for (int d = 0; d < depth; ++d) norm[r * depth + d] = 0;
      rowmax[r] = 0;
    }
    // the wave writes each hot row's slice map together (a Zipf head row has
    // hundreds of slices)
    unsigned long long m = __ballot(is_hot);
    while (m) {
      const int l = __builtin_ctzll(m);
      m &= m - 1;
      const int32_t nsl = __builtin_amdgcn_readlane(ns, l);
      const uint32_t hl = (uint32_t)__builtin_amdgcn_readlane((int)hidx, l);
      const uint32_t el = (uint32_t)__builtin_amdgcn_readlane((int)e0, l);
      for (int32_t sl = first + lane; sl < nsl; sl += 64) extra_map[el + sl - first] = make_int2((int)hl, sl);
    }
  }
}

// Upper bound of every counter of each row after the coming build (the row's
// mass in counter units, old mass included when accumulating), and the rows
// whose keys are split over several workgroups (their slices add with u32
// atomics): both need a hot slot before the launch.
__global__ void k_row_bound_implicit(const int64_t* lo_, const int64_t* hi_, int64_t nrows, int fb, int64_t slice, const uint64_t* old_mass,
                                     uint64_t* bound, uint8_t* force) {
  for (int64_t r = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; r < nrows; r += (int64_t)gridDim.x * blockDim.x) {
    const int64_t c = hi_[r] - lo_[r];
    bound[r] = ((uint64_t)c << fb) + (old_mass ? old_mass[r] : 0ULL);
    force[r] = c > slice ? 1 : 0;
  }
}

__global__ __launch_bounds__(256) void k_row_bound_values(const int64_t* lo_, const int64_t* hi_, const float* vals, int64_t nrows, int fb,
                                                          int64_t slice, const uint64_t* old_mass, uint64_t* bound,
                                                          uint8_t* force) {
  __shared__ uint64_t red[4];
  for (int64_t r = blockIdx.x; r < nrows; r += gridDim.x) {
    uint64_t s = 0;
    for (int64_t i = lo_[r] + threadIdx.x; i < hi_[r]; i += 256) {
      uint32_t inc;
      if (load_inc(vals, i, inc, fb)) s += inc;  // bad values are flagged by the build itself
    }
    s = block_sum_u64_sat(s, red);
    if (threadIdx.x == 0) {
      bound[r] = sat_add(s, old_mass ? old_mass[r] : 0ULL);
      force[r] = (hi_[r] - lo_[r]) > slice ? 1 : 0;
    }
  }
}

// An owner of a fresh build whose every counter is provably below 2^8 (its
// mass bound) and whose keys fit the register cache: built whole in LDS by
// k_build_nibbles / k_build_bytes (not by k_build_rows).
constexpr int64_t kByteKeys = 64 * kKeyRegs;  // one wave's register cache (k_build_nibbles)
__device__ __forceinline__ bool byte_class(int32_t slot, int64_t nkeys, uint64_t bound) {
  return slot < 0 && nkeys <= kByteKeys && bound < 256;
}

// grid = emax + nrows: blocks [0, emax) build extra slices of hot owners (heavy
// work first), blocks [emax, emax + nrows) one owner each (slice 0 if hot).
// Store form of the narrow rows' write-out: 0 = 8-B stores (4 counters per
// lane), 1 = 16-B stores (8 counters per lane), 2 = 16-B non-temporal stores.
typedef uint32_t u32x4_t __attribute__((ext_vector_type(4)));
__device__ __forceinline__ void store_row(uint4* p, uint4 v, int sv) {
  if (sv == 2) {
    const u32x4_t x = {v.x, v.y, v.z, v.w};
    __builtin_nontemporal_store(x, reinterpret_cast<u32x4_t*>(p));
  } else {
    *p = v;
  }
}

#ifdef CMS_NO_SLICE_PAIRS
constexpr bool kNoSlicePairs = true;
#else
constexpr bool kNoSlicePairs = false;
#endif
constexpr int kBuildStoreForm = 2;
constexpr size_t kFormLdsMax = 64 * 1024;  // byte-form owners: [d][w] bytes of LDS per workgroup  // 16-B non-temporal: config-3 build 20.4 -> 19.4 ms, config 2 ~1% (scripts/store_ab.sh)

// waves per SIMD the row and mid builds are compiled for: 6 (up to 80 VGPRs,
// no spills) -- at 8 (64 VGPRs) both spilled a few registers and the config-3
// build scope took 7.21-7.25 ms against 6.80-6.82 ms at 6 (6.88-6.94 at 7)
#ifndef CMS_BUILD_WAVES
#define CMS_BUILD_WAVES 6
#endif
template <int SV>
__global__ __launch_bounds__(kBuildThreads) __attribute__((amdgpu_waves_per_eu(CMS_BUILD_WAVES, 8))) void k_build_rows(
    const int64_t* lo_, const int64_t* hi_, Keys keys, const float* vals, int64_t nrows, HashParams hp,
    int64_t slice,
    const int32_t* row_hot, const HotInfo* hot, const int2* extra_map, const uint32_t* counters, int64_t emax,
    TableView tv, uint64_t* row_mass, uint64_t* norm, uint32_t* rowmax, uint32_t* flags, int accumulate,
    int slices_done, const uint64_t* bound, int forms, int skip_untouched, int32_t* hidx_w, uint32_t* cbound,
    const int32_t* rows_list, const uint32_t* rows_cnt) {
  extern __shared__ __align__(16) uint32_t lds[];  // one sketch row [w] u32, or a byte-form owner's [d][w] u8
  __shared__ unsigned long long s_norm[CMS_MAX_DEPTH];
  __shared__ unsigned long long s_mass;
  __shared__ uint32_t s_max;  // largest counter of the row (limb count of the all-pairs operands)
  const int w = (int)hp.width;
  const int64_t dw = (int64_t)hp.depth * w;
  const int tid = threadIdx.x;

  int64_t row, lo, hi;
  bool atomic_mode;
  if (blockIdx.x < emax) {
    if (slices_done || blockIdx.x >= counters[1]) return;  // slices_done: k_build_slices built them
#ifdef CMS_BUILD_NOSLICES  // bound analysis only: hot rows' extra slices skipped
    return;
#endif
    int2 m = extra_map[blockIdx.x];
    row = hot[m.x].row;
    lo = lo_[row] + (int64_t)m.y * slice;
    hi = min(hi_[row], lo + slice);
    atomic_mode = true;
  } else {
    row = (int64_t)blockIdx.x - emax;
    if (rows_list) {  // only the listed rows (the slot rows; the others have kernels of their own)
      if (row >= (int64_t)*rows_cnt) return;
      row = rows_list[row];
    }
    lo = lo_[row];
    atomic_mode = row_hot[row] >= 0;
    if (atomic_mode && slices_done) return;  // a split row: all its slices ran in k_build_slices
    hi = atomic_mode ? lo + slice : hi_[row];
    // accumulating into a live table with current norms: a row without keys
    // keeps its counters, norms and form (a form row may only be touched
    // after widen_rows made it u16)
    if (skip_untouched && hi_[row] == lo) return;
  }
#ifdef CMS_BUILD_NOKEYS  // bound analysis only: the write path alone
  hi = lo;
#endif
  // a hot row (slot) is u32, any other row u16 (promote_rows ran before the launch)
  const int32_t slot = tv.hidx[row];
  uint32_t* dst = slot >= 0 ? tv.hot + (int64_t)slot * dw : nullptr;
  uint16_t* dst16 = tv.row16(row);
  const bool load_old = accumulate && !atomic_mode;
  if (tid < CMS_MAX_DEPTH) s_norm[tid] = 0ULL;
  if (tid == 0) {
    s_mass = 0ULL;
    s_max = 0u;
  }
  uint32_t vmax = 0;

  // keys of small owners: read and reduced once for all d sketch rows
  const bool cached = (hi - lo) <= (int64_t)kBuildThreads * kKeyRegs;
  // Byte forms: a fresh narrow owner whose mass (so every counter) stays
  // below 2^8 is built by k_build_nibbles (4-bit rows) or, when a counter
  // reaches 16, by k_build_bytes (u8 rows) -- both launched after this kernel.
  if (forms && !atomic_mode && !load_old && byte_class(slot, hi - lo, bound[row])) return;
  uint64_t kp[kKeyRegs];
  uint32_t ik[kKeyRegs];
  uint64_t mass = 0;
  bool badv = false;
  if (cached) {
#pragma unroll
    for (int k = 0; k < kKeyRegs; ++k) {
      int64_t i = lo + tid + (int64_t)k * kBuildThreads;
      kp[k] = 0;
      ik[k] = 0;
      if (i < hi) {
        uint32_t inc;
        if (!load_inc(vals, i, inc, hp.frac_bits)) {
          badv = true;
          inc = 0;
        }
        kp[k] = keys.at(i);
        ik[k] = inc;
        mass += inc;
      }
    }
  }
  {
  // LDS slot for sketch row 0 (the old counters when accumulating)
  for (int j = tid; j < w; j += kBuildThreads) lds[j] = load_old ? (dst ? dst[j] : (uint32_t)dst16[j]) : 0u;
  __syncthreads();

  // Narrow rows of a fresh build pair their sketch rows: every counter of such
  // a row is below 2^16 (promote_rows guarantees it), so row d counts in the
  // low and row d+1 in the high half of the same LDS word without a carry
  // between them -- d = 5 takes three update/write-out phases instead of five.
  // A slice of a split (hot) row with unit increments counts at most
  // slice << frac_bits < 2^16 per bucket, so it pairs its sketch rows the same
  // way and walks its (uncached) keys ceil(d/2) times instead of d times.
  const bool slice_pairs = atomic_mode && !vals && (slice << hp.frac_bits) < 65536 && !kNoSlicePairs;
  const bool pair_rows = ((!dst && !load_old && !atomic_mode) || slice_pairs) && (w & 3) == 0;
  for (int d = 0; d < hp.depth;) {
    const bool two = pair_rows && d + 1 < hp.depth;
    // ---- updates of sketch row d (and d+1) ----
    if (cached) {
#pragma unroll
      for (int k = 0; k < kKeyRegs; ++k)
        if (ik[k]) {
          atomicAdd(&lds[bucket(hp, d, kp[k])], ik[k]);
          if (two) atomicAdd(&lds[bucket(hp, d + 1, kp[k])], ik[k] << 16);
        }
    } else {
      for (int64_t base = lo; base < hi; base += 4 * kBuildThreads) {
        uint64_t kk[4];
        uint32_t inc4[4];
#pragma unroll
        for (int u = 0; u < 4; ++u) {
          int64_t i = base + tid + (int64_t)u * kBuildThreads;
          kk[u] = i < hi ? keys.at(i) : 0;
          inc4[u] = 0;
          if (i < hi) {
            uint32_t inc;
            if (!load_inc(vals, i, inc, hp.frac_bits)) {
              badv = true;
              inc = 0;
            }
            inc4[u] = inc;
          }
        }
#pragma unroll
        for (int u = 0; u < 4; ++u) {
          if (inc4[u]) {
            const uint64_t kr = kk[u];
            atomicAdd(&lds[bucket(hp, d, kr)], inc4[u]);
            if (two) atomicAdd(&lds[bucket(hp, d + 1, kr)], inc4[u] << 16);
          }
          if (d == 0) mass += inc4[u];
        }
      }
    }
    lds_barrier();  // LDS order only: the write-out stores stay in flight
    // ---- write-out of row d, zero/load the slot for row d+1, sum of squares ----
    const int64_t rofs = (int64_t)d * w;
    const bool more = load_old && d + 1 < hp.depth;
    if (atomic_mode && two) {  // paired slice rows: low halves row d, high halves row d + 1
      for (int j = tid; j < w; j += kBuildThreads) {
        const uint32_t v = lds[j];
        lds[j] = 0u;
        if (v & 0xFFFFu) atomicAdd(dst + rofs + j, v & 0xFFFFu);
        if (v >> 16) atomicAdd(dst + rofs + w + j, v >> 16);
      }
    } else if (atomic_mode) {  // slices of a split row: always a hot (u32) row
      for (int j = tid; j < w; j += kBuildThreads) {
        uint32_t v = lds[j];
        lds[j] = 0u;
#ifdef CMS_BUILD_NOSLICEADD  // bound analysis only: the slices' global atomics skipped
        if (v == 0xFFFFFFFFu)
#endif
        if (v) atomicAdd(dst + rofs + j, v);
      }
    } else if (two && SV > 0 && (w & 7) == 0) {
      // as below, 8 counters (16 B) per lane and row per store
      uint4* l4 = reinterpret_cast<uint4*>(lds);
      uint4* da = reinterpret_cast<uint4*>(dst16 + rofs);
      uint4* db = reinterpret_cast<uint4*>(dst16 + rofs + w);
      uint32_t sqa = 0, sqb = 0;
      u16x2 pm = {0, 0};
      for (int j = tid; j < (w >> 3); j += kBuildThreads) {
        const uint4 v = l4[2 * j], u = l4[2 * j + 1];
        l4[2 * j] = make_uint4(0, 0, 0, 0);
        l4[2 * j + 1] = make_uint4(0, 0, 0, 0);
        const uint32_t a0 = __builtin_amdgcn_perm(v.y, v.x, 0x05040100u), a1 = __builtin_amdgcn_perm(v.w, v.z, 0x05040100u);
        const uint32_t a2 = __builtin_amdgcn_perm(u.y, u.x, 0x05040100u), a3 = __builtin_amdgcn_perm(u.w, u.z, 0x05040100u);
        const uint32_t b0 = __builtin_amdgcn_perm(v.y, v.x, 0x07060302u), b1 = __builtin_amdgcn_perm(v.w, v.z, 0x07060302u);
        const uint32_t b2 = __builtin_amdgcn_perm(u.y, u.x, 0x07060302u), b3 = __builtin_amdgcn_perm(u.w, u.z, 0x07060302u);
        store_row(da + j, make_uint4(a0, a1, a2, a3), SV);
        store_row(db + j, make_uint4(b0, b1, b2, b3), SV);
        const u16x2 pa0 = __builtin_bit_cast(u16x2, a0), pa1 = __builtin_bit_cast(u16x2, a1);
        const u16x2 pa2 = __builtin_bit_cast(u16x2, a2), pa3 = __builtin_bit_cast(u16x2, a3);
        const u16x2 pb0 = __builtin_bit_cast(u16x2, b0), pb1 = __builtin_bit_cast(u16x2, b1);
        const u16x2 pb2 = __builtin_bit_cast(u16x2, b2), pb3 = __builtin_bit_cast(u16x2, b3);
        sqa = __builtin_amdgcn_udot2(pa0, pa0, sqa, false);
        sqa = __builtin_amdgcn_udot2(pa1, pa1, sqa, false);
        sqa = __builtin_amdgcn_udot2(pa2, pa2, sqa, false);
        sqa = __builtin_amdgcn_udot2(pa3, pa3, sqa, false);
        sqb = __builtin_amdgcn_udot2(pb0, pb0, sqb, false);
        sqb = __builtin_amdgcn_udot2(pb1, pb1, sqb, false);
        sqb = __builtin_amdgcn_udot2(pb2, pb2, sqb, false);
        sqb = __builtin_amdgcn_udot2(pb3, pb3, sqb, false);
        const u16x2 ma = __builtin_elementwise_max(__builtin_elementwise_max(pa0, pa1), __builtin_elementwise_max(pa2, pa3));
        const u16x2 mb = __builtin_elementwise_max(__builtin_elementwise_max(pb0, pb1), __builtin_elementwise_max(pb2, pb3));
        pm = __builtin_elementwise_max(pm, __builtin_elementwise_max(ma, mb));
      }
      vmax = max(vmax, max((uint32_t)pm.x, (uint32_t)pm.y));
      sqa = wave_sum_u32(sqa);
      sqb = wave_sum_u32(sqb);
      if ((tid & 63) == 0) {
        atomicAdd(&s_norm[d], (unsigned long long)sqa);
        atomicAdd(&s_norm[d + 1], (unsigned long long)sqb);
      }
    } else if (two) {
      // rows d and d+1 leave LDS together; squares by v_dot2_u32_u16 on the
      // packed store words: a narrow row's sum of squares is at most
      // mass * max < 2^32, so u32 partial sums are exact
      uint4* l4 = reinterpret_cast<uint4*>(lds);
      uint2* da = reinterpret_cast<uint2*>(dst16 + rofs);
      uint2* db = reinterpret_cast<uint2*>(dst16 + rofs + w);
      uint32_t sqa = 0, sqb = 0;
      u16x2 pm = {0, 0};
      for (int j = tid; j < (w >> 2); j += kBuildThreads) {
        const uint4 v = l4[j];
        l4[j] = make_uint4(0, 0, 0, 0);
        const uint32_t a0 = __builtin_amdgcn_perm(v.y, v.x, 0x05040100u), a1 = __builtin_amdgcn_perm(v.w, v.z, 0x05040100u);
        const uint32_t b0 = __builtin_amdgcn_perm(v.y, v.x, 0x07060302u), b1 = __builtin_amdgcn_perm(v.w, v.z, 0x07060302u);
        da[j] = make_uint2(a0, a1);
        db[j] = make_uint2(b0, b1);
        const u16x2 pa0 = __builtin_bit_cast(u16x2, a0), pa1 = __builtin_bit_cast(u16x2, a1);
        const u16x2 pb0 = __builtin_bit_cast(u16x2, b0), pb1 = __builtin_bit_cast(u16x2, b1);
        sqa = __builtin_amdgcn_udot2(pa0, pa0, sqa, false);
        sqa = __builtin_amdgcn_udot2(pa1, pa1, sqa, false);
        sqb = __builtin_amdgcn_udot2(pb0, pb0, sqb, false);
        sqb = __builtin_amdgcn_udot2(pb1, pb1, sqb, false);
        pm = __builtin_elementwise_max(pm, __builtin_elementwise_max(__builtin_elementwise_max(pa0, pa1),
                                                                     __builtin_elementwise_max(pb0, pb1)));
      }
      vmax = max(vmax, max((uint32_t)pm.x, (uint32_t)pm.y));
      sqa = wave_sum_u32(sqa);
      sqb = wave_sum_u32(sqb);
      if ((tid & 63) == 0) {
        atomicAdd(&s_norm[d], (unsigned long long)sqa);
        atomicAdd(&s_norm[d + 1], (unsigned long long)sqb);
      }
    } else {
      uint64_t sq = 0;
      // 16-B u32 stores for slots, 8-B u16 stores for narrow rows (when the
      // row offset keeps them aligned); the next sketch row's old counters
      // are loaded into the slot as it is drained
      const bool vec = (w & 3) == 0 && (dst != nullptr || (tv.base(row) & 3) == 0);
      if (vec && !dst && !more && SV > 0 && (w & 7) == 0 && (tv.base(row) & 7) == 0) {
        // narrow row, fresh build, 16-B stores (8 counters per lane)
        uint4* l4 = reinterpret_cast<uint4*>(lds);
        uint4* d4 = reinterpret_cast<uint4*>(dst16 + rofs);
        uint32_t sq32 = 0;
        u16x2 pm = {0, 0};
        for (int j = tid; j < (w >> 3); j += kBuildThreads) {
          const uint4 v = l4[2 * j], u = l4[2 * j + 1];
          l4[2 * j] = make_uint4(0, 0, 0, 0);
          l4[2 * j + 1] = make_uint4(0, 0, 0, 0);
          const uint32_t a0 = __builtin_amdgcn_perm(v.y, v.x, 0x05040100u), a1 = __builtin_amdgcn_perm(v.w, v.z, 0x05040100u);
          const uint32_t a2 = __builtin_amdgcn_perm(u.y, u.x, 0x05040100u), a3 = __builtin_amdgcn_perm(u.w, u.z, 0x05040100u);
          store_row(d4 + j, make_uint4(a0, a1, a2, a3), SV);
          const u16x2 pa0 = __builtin_bit_cast(u16x2, a0), pa1 = __builtin_bit_cast(u16x2, a1);
          const u16x2 pa2 = __builtin_bit_cast(u16x2, a2), pa3 = __builtin_bit_cast(u16x2, a3);
          sq32 = __builtin_amdgcn_udot2(pa0, pa0, sq32, false);
          sq32 = __builtin_amdgcn_udot2(pa1, pa1, sq32, false);
          sq32 = __builtin_amdgcn_udot2(pa2, pa2, sq32, false);
          sq32 = __builtin_amdgcn_udot2(pa3, pa3, sq32, false);
          pm = __builtin_elementwise_max(pm, __builtin_elementwise_max(__builtin_elementwise_max(pa0, pa1),
                                                                       __builtin_elementwise_max(pa2, pa3)));
        }
        vmax = max(vmax, max((uint32_t)pm.x, (uint32_t)pm.y));
        sq = sq32;
      } else if (vec && !dst && !more) {
        // narrow row, fresh build (the common case): every counter < 2^16, so
        // the squares are full-rate 24-bit products and no sum can saturate
        uint4* l4 = reinterpret_cast<uint4*>(lds);
        uint2* d2 = reinterpret_cast<uint2*>(dst16 + rofs);
        uint32_t sq32 = 0;  // < 2^32: see the paired write-out
        u16x2 pm = {0, 0};
        for (int j = tid; j < (w >> 2); j += kBuildThreads) {
          const uint4 v = l4[j];
          l4[j] = make_uint4(0, 0, 0, 0);
          const uint32_t a0 = __builtin_amdgcn_perm(v.y, v.x, 0x05040100u), a1 = __builtin_amdgcn_perm(v.w, v.z, 0x05040100u);
#ifdef CMS_BUILD_NOWRITE  // bound analysis only: no table stores
          if (v.x == 0xFFFFFFFFu)
#endif
          d2[j] = make_uint2(a0, a1);
          const u16x2 pa0 = __builtin_bit_cast(u16x2, a0), pa1 = __builtin_bit_cast(u16x2, a1);
          sq32 = __builtin_amdgcn_udot2(pa0, pa0, sq32, false);
          sq32 = __builtin_amdgcn_udot2(pa1, pa1, sq32, false);
          pm = __builtin_elementwise_max(pm, __builtin_elementwise_max(pa0, pa1));
        }
        vmax = max(vmax, max((uint32_t)pm.x, (uint32_t)pm.y));
        sq = sq32;
      } else if (vec) {
        uint4* l4 = reinterpret_cast<uint4*>(lds);
        for (int j = tid; j < (w >> 2); j += kBuildThreads) {
          const uint4 v = l4[j];
          uint4 nv = make_uint4(0, 0, 0, 0);
          if (more) {
            if (dst) {
              nv = reinterpret_cast<const uint4*>(dst + rofs + w)[j];
            } else {
              const ushort4 o = reinterpret_cast<const ushort4*>(dst16 + rofs + w)[j];
              nv = make_uint4(o.x, o.y, o.z, o.w);
            }
          }
          l4[j] = nv;
#ifdef CMS_BUILD_NOWRITE  // bound analysis only: no table stores
          if (v.x == 0xFFFFFFFFu)
#endif
          if (dst) reinterpret_cast<uint4*>(dst + rofs)[j] = v;
          else reinterpret_cast<ushort4*>(dst16 + rofs)[j] = make_ushort4((unsigned short)v.x, (unsigned short)v.y,
                                                                          (unsigned short)v.z, (unsigned short)v.w);
          vmax = max(vmax, max(max(v.x, v.y), max(v.z, v.w)));
          sq = sat_add(sq, (uint64_t)v.x * v.x);
          sq = sat_add(sq, (uint64_t)v.y * v.y);
          sq = sat_add(sq, (uint64_t)v.z * v.z);
          sq = sat_add(sq, (uint64_t)v.w * v.w);
        }
      } else {
        for (int j = tid; j < w; j += kBuildThreads) {
          const uint32_t v = lds[j];
          lds[j] = more ? (dst ? dst[rofs + w + j] : (uint32_t)dst16[rofs + w + j]) : 0u;
          if (dst) dst[rofs + j] = v;
          else dst16[rofs + j] = (uint16_t)v;
          vmax = max(vmax, v);
          sq = sat_add(sq, (uint64_t)v * v);
        }
      }
      // per-thread sums stay far below 2^64 for counters < 2^26; anything at or
      // above 2^53 only has to stay >= 2^53 (inexact regime), so clamp.
      sq = wave_sum_u64_sat(sq);
      if (sq > (1ULL << 60)) sq = 1ULL << 60;
      if ((tid & 63) == 0) atomicAdd(&s_norm[d], (unsigned long long)sq);
    }
    lds_barrier();  // LDS order only: the write-out stores stay in flight
    d += two ? 2 : 1;
  }
  }  // sketch-row loop

  if (badv) atomicOr(flags, kFlagBadValue);
  mass = wave_sum_u64_sat(mass);
  if ((tid & 63) == 0 && mass) atomicAdd(&s_mass, (unsigned long long)mass);
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) vmax = max(vmax, (uint32_t)__shfl_xor((int)vmax, o, 64));
  if ((tid & 63) == 0 && vmax) atomicMax(&s_max, vmax);
  __syncthreads();
  if (!atomic_mode && tid < hp.depth) norm[row * hp.depth + tid] = s_norm[tid];
  if (!atomic_mode && tid == 0) rowmax[row] = s_max;
  if (tid == 0) {
    uint64_t tm = s_mass;
    if (!atomic_mode) {
      uint64_t m = accumulate ? row_mass[row] + tm : tm;
      row_mass[row] = m;
      if (m >= (1ULL << 32)) atomicOr(flags, kFlagOverflow);
    } else if (tm) {
      unsigned long long old = atomicAdd((unsigned long long*)&row_mass[row], (unsigned long long)tm);
      if (old + tm >= (1ULL << 32)) atomicOr(flags, kFlagOverflow);
    }
  }
}

// Owner classes of a fresh build with forms: rows holding a u32 slot (split
// owners and masses >= 2^16: k_build_rows), byte-class rows (k_build_nibbles
// finds them itself) and the rest, the mid class (k_build_mid).  Each wave
// appends its rows with one atomic per list.
// Rows of chunks of kClassChunk owners per workgroup: the class lists are
// gathered in LDS (wave-aggregated LDS counters) and reserved with one global
// atomic per chunk and list -- with one atomic per wave the two list counters
// took ~200 us of contention at 1M owners.
constexpr int kClassChunk = 4096;
__global__ __launch_bounds__(256) void k_build_classes(const int64_t* lo_, const int64_t* hi_, int64_t nrows,
                                                       const int32_t* hidx, const uint64_t* bound, int32_t* slot_list,
                                                       int32_t* mid_list, uint32_t* cnt /* [0] slot, [1] mid */,
                                                       const uint8_t* early) {
  __shared__ int32_t s_slot[kClassChunk], s_mid[kClassChunk];
  __shared__ uint32_t s_n[2], s_b[2];
  const int lane = (int)__lane_id();
  const int tid = threadIdx.x;
  const unsigned long long below = (1ULL << lane) - 1ULL;
  for (int64_t r0 = (int64_t)blockIdx.x * kClassChunk; r0 < nrows; r0 += (int64_t)gridDim.x * kClassChunk) {
    if (tid < 2) s_n[tid] = 0;
    __syncthreads();
    for (int64_t r = r0 + tid; r < r0 + kClassChunk; r += 256) {  // (whole waves: the ballots)
      bool is_slot = false, is_mid = false;
      if (r < nrows && !(early && early[r])) {  // (an early row is built already)
        const int32_t sl = hidx[r];
        is_slot = sl >= 0;
        is_mid = !is_slot && !byte_class(sl, hi_[r] - lo_[r], bound[r]);
      }
      const unsigned long long ms = __ballot(is_slot), mm = __ballot(is_mid);
      uint32_t b0 = 0, b1 = 0;
      if (lane == 0) {
        if (ms) b0 = atomicAdd(&s_n[0], (uint32_t)__popcll(ms));
        if (mm) b1 = atomicAdd(&s_n[1], (uint32_t)__popcll(mm));
      }
      b0 = (uint32_t)__shfl((int)b0, 0, 64);
      b1 = (uint32_t)__shfl((int)b1, 0, 64);
      if (is_slot) s_slot[b0 + __popcll(ms & below)] = (int32_t)r;
      if (is_mid) s_mid[b1 + __popcll(mm & below)] = (int32_t)r;
    }
    __syncthreads();
    if (tid < 2) s_b[tid] = s_n[tid] ? atomicAdd(&cnt[tid], s_n[tid]) : 0u;
    __syncthreads();
    for (uint32_t i = tid; i < s_n[0]; i += 256) slot_list[s_b[0] + i] = s_slot[i];
    for (uint32_t i = tid; i < s_n[1]; i += 256) mid_list[s_b[1] + i] = s_mid[i];
    __syncthreads();
  }
}

// Mid-class owners (narrow, more than 256 keys or a mass >= 256): one
// workgroup per owner, in the narrowest form that holds it -- 4-bit first,
// u8 when a counter reaches 16, u16 when one reaches 256 (each escalation
// restarts the owner; the wider layout overwrites every byte the narrower one
// wrote).  The 4-bit attempt counts ALL d sketch rows at once in a [d][w]
// 4-bit LDS image (d*w/2 bytes, 20 KB at config 3), so each key is read and
// hashed once; its sums of squares come from reading the image back (v_dot4
// of the nibbles) as it is stored.  The u8 / u16 attempts go one sketch row
// at a time (a w- or 2w-byte image), the returning LDS adds giving each
// row's sum of squares.  A persistent grid walks the device-side list.
// mid owners of up to this many keys (the register-cached ones) may be list rows
#ifndef CMS_MID_LIST_KEYS
#define CMS_MID_LIST_KEYS (kBuildThreads * kKeyRegs)
#endif
constexpr int kMidListKeys = CMS_MID_LIST_KEYS;
// the row passes of owners past the register cache prefetch their keys a step
// ahead (measured slower: build scope 5.32 vs 5.11 ms, profiles/r06/ab)
#ifndef CMS_MID_ROW_PREFETCH
#define CMS_MID_ROW_PREFETCH 0
#endif
// keys per thread in flight per step of an uncached owner's row pass
#ifndef CMS_MID_ROW_KEYS
#define CMS_MID_ROW_KEYS 4
#endif
// byte-class list owners of <= 64 keys clear the words they added into after
// each sketch row instead of zeroing the wave's whole 4-bit row
#ifndef CMS_NIB_CLEAR1
#define CMS_NIB_CLEAR1 0
#endif
// byte-class list owners take their LDS adds back after each sketch row
// instead of zeroing the wave's 4-bit row before the next one
#ifndef CMS_NIB_UNADD
#define CMS_NIB_UNADD 0
#endif
// register-cached owners keep their keys' d buckets (u16 pairs) from one
// all-rows hash, so the u8 / u16 row passes (an escalation from 4-bit, or an
// owner starting at u8) do not hash again
#ifndef CMS_MID_BKT_CACHE
#define CMS_MID_BKT_CACHE 0
#endif
template <int SV, int D, int MT>
// 4 waves per SIMD: the key prefetch needs more than the 80 VGPRs of 6
// (it spilled there); the build measured the same (profiles/r04/ab_*_s5)
__global__ __launch_bounds__(MT) __attribute__((amdgpu_waves_per_eu(4, 8))) void k_build_mid(
    const int64_t* lo_, const int64_t* hi_, Keys keys, const float* vals, HashParams hp,
    const int32_t* list, const uint32_t* list_cnt, TableView tv, int32_t* hidx_w, uint32_t* cbound,
    uint64_t* row_mass, uint64_t* norm, uint32_t* rowmax, uint32_t* flags, int list_keys, int u4_keys, int u8_keys,
    int u8img) {
  constexpr int MTH = MT;                   // threads per owner (a workgroup)
  constexpr int MKR = kKeyRegs * 256 / MT;  // key registers per thread: 1024 keys cached per owner
  constexpr bool kBc = CMS_MID_BKT_CACHE && D > 0 && MKR <= 4;  // cached buckets (w <= 65536: u16)
  constexpr int RK = CMS_MID_ROW_PREFETCH ? 4 : CMS_MID_ROW_KEYS;  // keys per thread per step of an uncached row pass
  constexpr int kBcW = kBc ? (D + 1) / 2 : 1;                   // u16 pairs per key
  extern __shared__ __align__(16) uint32_t lds[];  // one sketch row of up to w u16 counters, or the [d][w] 4-bit image
  __shared__ unsigned long long s_norm[CMS_MAX_DEPTH];
  __shared__ unsigned long long s_mass;
  __shared__ uint32_t s_max, s_ovf;
  const int tid = threadIdx.x;
  const int w = (int)hp.width;
  const uint32_t count = *list_cnt;
  for (uint32_t li = blockIdx.x; li < count; li += gridDim.x) {
    const int64_t row = list[li];
    const int64_t lo = lo_[row], hi = hi_[row];
    const bool cached = (hi - lo) <= (int64_t)MTH * MKR;
    uint64_t kp[MKR];
    uint32_t ik[MKR];
    uint32_t bc[MKR][kBcW];  // kBc: key k's bucket in sketch row r at bits 16 (r & 1) of bc[k][r / 2]
    bool have_bc = false;
    uint64_t mass = 0;
    bool badv = false;
    if (cached) {
#pragma unroll
      for (int k = 0; k < MKR; ++k) {
        const int64_t i = lo + tid + (int64_t)k * MTH;
        kp[k] = 0;
        ik[k] = 0;
        if (i < hi) {
          uint32_t inc;
          if (!load_inc(vals, i, inc, hp.frac_bits)) {
            badv = true;
            inc = 0;
          }
          kp[k] = keys.at(i);
          ik[k] = inc;
          mass += inc;
        }
      }
    }
    uint4* d4 = reinterpret_cast<uint4*>(tv.row16(row));  // the row's slot (64-B aligned)
    // a LIST row (cms_internal.h kFormList) when the owner's keys sit in
    // registers, increments are units, and the list beats even the 4-bit row:
    // the counting below then only yields the norms and the maximum, and the
    // keys' buckets leave instead of the image (u16 counters -- a count past
    // 255 -- keep the dense row)
    const int64_t m = hi - lo;
    const bool as_list = cached && m <= list_keys && vals == nullptr && hp.frac_bits == 0 &&
                         (int64_t)hp.depth * m <= 8192 && 2 + 2 * (int64_t)hp.depth * m < (int64_t)hp.depth * w / 2;
    uint16_t* lst = tv.row16(row);
    int level = -1;  // the form that holds the owner: 0 4-bit, 1 u8, 2 u16 (the class bound keeps every counter < 2^16)
    uint32_t vmax = 0;
    // the first form tried (Tunables::mid_u4_keys / mid_u8_keys); a list row
    // leaves its entries in the 4-bit pass, so it always takes that pass
    const int start = as_list || m <= u4_keys ? 0 : m <= u8_keys ? 1 : 2;
    bool mass_pending = !cached;  // uncached keys: the mass is summed by the first pass over them
    // ALL sketch rows in one key pass in a [d][w] 4-bit image.  (A [d][w] u8
    // image after a 4-bit overflow -- a Zipf key set repeats its popular keys,
    // and config 3 has 40K u8 owners -- measured slower: its 40 KB per
    // workgroup halve the owners in flight, build 6.55 -> 7.01 ms.)
    if (start == 0) {
      constexpr int ab = 4;
      const int lga = 3;  // log2(counters per word)
      const uint32_t capa = (1u << ab) - 1u;
      const int nq_all = (int)((int64_t)hp.depth * w * ab >> 7);  // uint4 of the [d][w] image
      uint4* l4 = reinterpret_cast<uint4*>(lds);
      for (int j = tid; j < nq_all; j += MTH) l4[j] = make_uint4(0, 0, 0, 0);
      if (tid < CMS_MAX_DEPTH) s_norm[tid] = 0ULL;
      if (tid == 0) {
        s_max = 0u;
        s_ovf = 0u;
        s_mass = 0ULL;
      }
      __syncthreads();
      bool ovf = false;
      vmax = 0;
      // a list row at an unrolled depth takes its sums of squares from the
      // adds (2 c inc + inc^2 per update, telescoping to sum c^2) instead of
      // reading the image back: nothing of it is stored
      constexpr int kSq = D > 0 ? D : 1;
      uint32_t sqr[kSq];
#pragma unroll
      for (int d = 0; d < kSq; ++d) sqr[d] = 0u;
      const bool tele = D > 0 && as_list;
      // lt >= 0: the key's list index -- a list row's entries leave during
      // the count (a count past 255 later rewrites the slot as u16 rows)
      auto add_all = [&](uint64_t kr, uint32_t inc, int64_t lt, uint32_t* bcache) {
        each_bucket<D>(hp, kr, [&](int d, uint32_t bk) {
          if (kBc && bcache) bcache[d >> 1] = (d & 1) ? (bcache[d >> 1] | bk << 16) : bk;
          if (lt >= 0) lst[1 + (int64_t)d * m + lt] = (uint16_t)bk;
          const uint32_t c = (uint32_t)d * (uint32_t)w + bk;
          const uint32_t sh = (c & ((1u << lga) - 1u)) * (uint32_t)ab;
          const uint32_t old = (atomicAdd(&lds[c >> lga], inc << sh) >> sh) & capa;
          const uint32_t nv = old + inc;
          ovf |= nv > capa || inc > capa;  // carried into the next counter: a wider form
          vmax = max(vmax, nv);
          if (D > 0) sqr[D > 0 ? d : 0] += (2u * old + inc) * inc;
        });
      };
      if (cached) {
#pragma unroll
        for (int k = 0; k < MKR; ++k)
          if (ik[k]) add_all(kp[k], ik[k], as_list ? (int64_t)(tid + k * MTH) : int64_t(-1), kBc ? bc[k] : nullptr);
        have_bc = kBc;
      } else {
        // the next step's key loads go out before this step's keys are added
        constexpr int64_t kStep = 4 * MTH;
        uint64_t nx[4];
        auto fetch = [&](int64_t base) {
#pragma unroll
          for (int u = 0; u < 4; ++u) {
            const int64_t i = base + tid + (int64_t)u * MTH;
            nx[u] = i < hi ? keys.raw(i) : 0ULL;
          }
        };
        fetch(lo);
        for (int64_t base = lo; base < hi; base += kStep) {
          uint64_t kk[4];
          uint32_t inc4[4];
#pragma unroll
          for (int u = 0; u < 4; ++u) {
            kk[u] = nx[u];
            const int64_t i = base + tid + (int64_t)u * MTH;
            inc4[u] = 0;
            if (i < hi) {
              uint32_t inc;
              if (!load_inc(vals, i, inc, hp.frac_bits)) {
                badv = true;
                inc = 0;
              }
              inc4[u] = inc;
            }
          }
          if (base + kStep < hi) fetch(base + kStep);
#pragma unroll
          for (int u = 0; u < 4; ++u) {
            if (inc4[u]) add_all(keys.resolve(kk[u]), inc4[u], -1, nullptr);
            mass += inc4[u];
          }
        }
        mass_pending = false;
      }
      if (__ballot(ovf) && (tid & 63) == 0) s_ovf = 1u;
      __syncthreads();
      const bool fits = s_ovf == 0u;
      __syncthreads();  // every thread has read s_ovf before the row passes reset it
      if (fits) level = 0;
      if (fits && tele) {
#pragma unroll
        for (int d = 0; d < kSq; ++d) {
          const uint32_t sq = wave_sum_u32(sqr[d]);
          if ((tid & 63) == 0 && sq) atomicAdd(&s_norm[d], (unsigned long long)sq);
        }
        level = 3;  // a list row, norms done: no read-back
      }
    }
    if (level == 3) level = 0;
    else if (level == 0) {
      // read the image back: each sketch row's sum of squares (v_dot4 of its
      // low and high nibbles) as its rows leave for the slot
      const uint4* l4 = reinterpret_cast<const uint4*>(lds);
      const int nq = w >> 5;  // uint4 per 4-bit sketch row
      for (int d = 0; d < hp.depth; ++d) {
        uint32_t sq = 0;  // <= row mass * max counter < 2^32
        for (int j = tid; j < nq; j += MTH) {
          const uint4 v = l4[d * nq + j];
          const uint32_t x[4] = {v.x, v.y, v.z, v.w};
#pragma unroll
          for (int q = 0; q < 4; ++q) {
            const uint32_t lo4 = x[q] & 0x0F0F0F0Fu, hi4 = (x[q] >> 4) & 0x0F0F0F0Fu;
            sq = __builtin_amdgcn_udot4(lo4, lo4, sq, false);
            sq = __builtin_amdgcn_udot4(hi4, hi4, sq, false);
          }
#ifdef CMS_BUILD_NOWRITE  // bound analysis only: no table stores
          if (false)
#endif
          if (!as_list) store_row(d4 + d * nq + j, v, SV);
        }
        sq = wave_sum_u32(sq);
        if ((tid & 63) == 0 && sq) atomicAdd(&s_norm[d], (unsigned long long)sq);
      }
    }
    // owners that start at u8 (u8img): ALL sketch rows in one key pass in a
    // [d][w] u8 image (d*w bytes of LDS), each key read and hashed once
    // instead of once per sketch row; a counter past 255 goes on to u16 rows
    bool u8_failed = false;
    if (start == 1 && u8img) {
      const int nq_all = (int)(((int64_t)hp.depth * w) >> 4);  // uint4 of the [d][w] byte image
      uint4* l4 = reinterpret_cast<uint4*>(lds);
      for (int j = tid; j < nq_all; j += MTH) l4[j] = make_uint4(0, 0, 0, 0);
      if (tid < CMS_MAX_DEPTH) s_norm[tid] = 0ULL;
      if (tid == 0) {
        s_max = 0u;
        s_ovf = 0u;
        s_mass = 0ULL;
      }
      __syncthreads();
      bool ovf = false;
      vmax = 0;
      auto add_all8 = [&](uint64_t kr, uint32_t inc) {
        each_bucket<D>(hp, kr, [&](int d, uint32_t bk) {
          const uint32_t c = (uint32_t)d * (uint32_t)w + bk;
          const uint32_t sh = (c & 3u) << 3;
          const uint32_t old = (atomicAdd(&lds[c >> 2], inc << sh) >> sh) & 255u;
          const uint32_t nv = old + inc;
          ovf |= nv > 255u || inc > 255u;  // carried into the next counter: u16 rows
          vmax = max(vmax, nv);
        });
      };
      if (cached) {
#pragma unroll
        for (int k = 0; k < MKR; ++k)
          if (ik[k]) add_all8(kp[k], ik[k]);
      } else {
        constexpr int64_t kStep = 4 * MTH;
        uint64_t nx[4];
        auto fetch = [&](int64_t base) {
#pragma unroll
          for (int u = 0; u < 4; ++u) {
            const int64_t i = base + tid + (int64_t)u * MTH;
            nx[u] = i < hi ? keys.raw(i) : 0ULL;
          }
        };
        fetch(lo);
        for (int64_t base = lo; base < hi; base += kStep) {
          uint64_t kk[4];
          uint32_t inc4[4];
#pragma unroll
          for (int u = 0; u < 4; ++u) {
            kk[u] = nx[u];
            const int64_t i = base + tid + (int64_t)u * MTH;
            inc4[u] = 0;
            if (i < hi) {
              uint32_t inc;
              if (!load_inc(vals, i, inc, hp.frac_bits)) {
                badv = true;
                inc = 0;
              }
              inc4[u] = inc;
            }
          }
          if (base + kStep < hi) fetch(base + kStep);
#pragma unroll
          for (int u = 0; u < 4; ++u) {
            if (inc4[u]) add_all8(keys.resolve(kk[u]), inc4[u]);
            mass += inc4[u];
          }
        }
        mass_pending = false;
      }
      if (__ballot(ovf) && (tid & 63) == 0) s_ovf = 1u;
      __syncthreads();
      const bool fits = s_ovf == 0u;
      __syncthreads();  // every thread has read s_ovf before the row passes reset it
      if (fits) {
        level = 1;
        const uint4* r4 = reinterpret_cast<const uint4*>(lds);
        const int nq = w >> 4;  // uint4 per u8 sketch row
        for (int d = 0; d < hp.depth; ++d) {
          uint32_t sq = 0;  // <= row mass * max counter < 2^32
          for (int j = tid; j < nq; j += MTH) {
            const uint4 v = r4[d * nq + j];
            sq = __builtin_amdgcn_udot4(v.x, v.x, sq, false);
            sq = __builtin_amdgcn_udot4(v.y, v.y, sq, false);
            sq = __builtin_amdgcn_udot4(v.z, v.z, sq, false);
            sq = __builtin_amdgcn_udot4(v.w, v.w, sq, false);
#ifdef CMS_BUILD_NOWRITE  // bound analysis only: no table stores
            if (false)
#endif
            store_row(d4 + d * nq + j, v, SV);
          }
          sq = wave_sum_u32(sq);
          if ((tid & 63) == 0 && sq) atomicAdd(&s_norm[d], (unsigned long long)sq);
        }
      } else {
        u8_failed = true;
      }
    }
    // the 4-bit image overflowed (or was skipped): one sketch row at a time, u8 then u16
    if (level < 0) level = start > 1 || u8_failed ? 2 : 1;
    else level = -level - 1;  // done: mark so the row passes are skipped
    if (kBc && cached && level >= 0 && !have_bc) {  // all d buckets of the cached keys, once
#pragma unroll
      for (int k = 0; k < MKR; ++k)
        if (ik[k])
          each_bucket<D>(hp, kp[k], [&](int d, uint32_t bk) {
            bc[k][d >> 1] = (d & 1) ? (bc[k][d >> 1] | bk << 16) : bk;
          });
      have_bc = true;
    }
    for (;;) {
      if (level < 0) break;  // an all-rows image held every counter
      const int bits = 4 << level;
      const int lg = 3 - level;          // log2(counters per word)
      const uint32_t cap = (1u << bits) - 1u;
      const int nq = (w * bits) >> 7;    // uint4 per sketch row (w % 32 == 0)
      uint4* l4 = reinterpret_cast<uint4*>(lds);
      if (tid < CMS_MAX_DEPTH) s_norm[tid] = 0ULL;
      if (tid == 0) {
        s_max = 0u;
        s_ovf = 0u;
        s_mass = 0ULL;  // (added once, after the last pass; the 4-bit pass may not have run)
      }
      vmax = 0;
      for (int d = 0; d < hp.depth; ++d) {
        for (int j = tid; j < nq; j += MTH) l4[j] = make_uint4(0, 0, 0, 0);
        __syncthreads();
        uint64_t sq = 0;
        bool ovf = false;
        auto add = [&](uint64_t kr, uint32_t inc, const uint32_t* bcache) {
          uint32_t c;
          if (kBc && bcache) {  // the cached pair of row d: a select chain (d is not a compile-time index here)
            const uint32_t pr = d < 2 ? bcache[0] : (d < 4 || kBcW < 3) ? bcache[kBcW > 1 ? 1 : 0] : bcache[kBcW - 1];
            c = (pr >> ((d & 1) << 4)) & 0xFFFFu;
          } else {
            c = bucket(hp, d, kr);
          }
          const uint32_t sh = (c & ((1u << lg) - 1u)) * (uint32_t)bits;
          const uint32_t old = (atomicAdd(&lds[c >> lg], inc << sh) >> sh) & cap;
          const uint32_t nv = old + inc;
          ovf |= nv > cap || inc > cap;  // carried into the next counter: a wider form
          sq += (uint64_t)(2u * old + inc) * inc;
          vmax = max(vmax, nv);
        };
        if (cached) {
#pragma unroll
          for (int k = 0; k < MKR; ++k)
            if (ik[k]) add(kp[k], ik[k], kBc && have_bc ? bc[k] : nullptr);
        } else {
#if CMS_MID_ROW_PREFETCH
          // the next step's key loads go out before this step's keys are
          // added (the 4-bit pass's scheme; every row pass re-reads the keys)
          constexpr int64_t kStep = 4 * MTH;
          uint64_t nx[4];
          auto fetch = [&](int64_t base) {
#pragma unroll
            for (int u = 0; u < 4; ++u) {
              const int64_t i = base + tid + (int64_t)u * MTH;
              nx[u] = i < hi ? keys.raw(i) : 0ULL;
            }
          };
          fetch(lo);
#endif
          for (int64_t base = lo; base < hi; base += RK * MTH) {
            uint64_t kk[RK];
            uint32_t inc4[RK];
#if CMS_MID_ROW_PREFETCH
            uint64_t raw[4];
#pragma unroll
            for (int u = 0; u < 4; ++u) raw[u] = nx[u];
            if (base + kStep < hi) fetch(base + kStep);
#endif
#pragma unroll
            for (int u = 0; u < RK; ++u) {
              const int64_t i = base + tid + (int64_t)u * MTH;
#if CMS_MID_ROW_PREFETCH
              kk[u] = i < hi ? keys.resolve(raw[u]) : 0;
#else
              kk[u] = i < hi ? keys.at(i) : 0;
#endif
              inc4[u] = 0;
              if (i < hi) {
                uint32_t inc;
                if (!load_inc(vals, i, inc, hp.frac_bits)) {
                  badv = true;
                  inc = 0;
                }
                inc4[u] = inc;
              }
            }
#pragma unroll
            for (int u = 0; u < RK; ++u) {
              if (inc4[u]) add(kk[u], inc4[u], nullptr);
              if (mass_pending) mass += inc4[u];
            }
          }
          mass_pending = false;  // summed once, by row 0 of the first pass
        }
        sq = wave_sum_u64_sat(sq);
        if ((tid & 63) == 0 && sq) atomicAdd(&s_norm[d], (unsigned long long)sq);
        if (__ballot(ovf) && (tid & 63) == 0) s_ovf = 1u;
        __syncthreads();
        if (s_ovf) break;  // uniform: escalate
#ifdef CMS_BUILD_NOWRITE  // bound analysis only: no table stores
        if (false)
#endif
        if (!(as_list && level == 1))  // a list row's entries left in the 4-bit pass
          for (int j = tid; j < nq; j += MTH) store_row(d4 + d * nq + j, l4[j], SV);
        __syncthreads();  // the image is read out before the next sketch row zeroes it
      }
      if (!s_ovf || level == 2) break;
      __syncthreads();
      ++level;
    }
    if (level < 0) level = -level - 1;
    if (badv) atomicOr(flags, kFlagBadValue);
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) vmax = max(vmax, (uint32_t)__shfl_xor((int)vmax, o, 64));
    if ((tid & 63) == 0 && vmax) atomicMax(&s_max, vmax);
    mass = wave_sum_u64_sat(mass);
    if ((tid & 63) == 0 && mass) atomicAdd(&s_mass, (unsigned long long)mass);
    __syncthreads();
    if (tid < hp.depth) norm[row * hp.depth + tid] = s_norm[tid];
    const bool listed = as_list && level <= 1;
    if (tid == 0) {
      rowmax[row] = s_max;
      row_mass[row] = s_mass;
      if (s_mass >= (1ULL << 32)) atomicOr(flags, kFlagOverflow);
      if (listed) lst[0] = (uint16_t)m;
      hidx_w[row] = listed ? kFormList : level == 0 ? kFormU4 : level == 1 ? kFormU8 : kFormU16;
      cbound[row] = s_max;
    }
    __syncthreads();  // shared sums consumed before the next owner
  }
}

// Mid-class owners, one WAVE per owner (Tunables::mid_waves; unit
// increments): k_build_nibbles' scheme at the mid class's sizes.  Each wave
// counts one sketch row at a time in its own w-byte LDS slot -- 4-bit
// counters first for owners of <= mid_u4_keys keys (and list-row owners),
// else u8 -- with the returning LDS adds giving each row's sum of squares
// and maximum, and stores the row as it finishes.  No workgroup barrier: a
// wave's LDS operations execute in program order, so the waves of a
// workgroup never wait on each other (k_build_mid's 256-thread owners pass
// ~15 barriers per owner).  Keys are streamed per sketch row (L2-resident
// after the first), the next loads in flight; hashes take bucket_q's route
// (power-of-two widths), and an owner with a reduced key >= 2^32 goes to
// k_build_mid.  A counter past 15 restarts the
// owner at u8; past 255 (or more than mid_u8_keys keys) the owner is queued
// for k_build_mid's u16 rows (redo list).
template <int SV, int D>
__global__ __launch_bounds__(256) void k_build_mid_waves(
    const int64_t* lo_, const int64_t* hi_, Keys keys, HashParams hp, const int32_t* list, const uint32_t* list_cnt,
    TableView tv, int32_t* hidx_w, uint32_t* cbound, uint64_t* row_mass, uint64_t* norm, uint32_t* rowmax,
    int list_keys, int u4_keys, int u8_keys, int32_t* redo, uint32_t* redo_cnt) {
  extern __shared__ __align__(16) uint32_t lds[];  // [4][w / 4] words: one u8 (or 4-bit) sketch row per wave
  const int lane = threadIdx.x & 63;
  const int wv = threadIdx.x >> 6;
  const int w = (int)hp.width;
  const int depth = D > 0 ? D : hp.depth;
  const int64_t dw = (int64_t)depth * w;
  uint32_t* slot = lds + wv * (w >> 2);
  uint4* slot4 = reinterpret_cast<uint4*>(slot);
  const uint32_t count = *list_cnt;
  const uint32_t nwv = gridDim.x * 4u;
  for (uint32_t li = blockIdx.x * 4u + (uint32_t)wv; li < count; li += nwv) {
    const int64_t row = list[li];
    const int64_t lo = lo_[row], hi = hi_[row];
    const int64_t m = hi - lo;
    if (m > u8_keys) {  // starts at u16: k_build_mid
      if (lane == 0) redo[atomicAdd(redo_cnt, 1u)] = (int32_t)row;
      continue;
    }
    const bool as_list = m <= list_keys && (int64_t)depth * m <= 8192 && 2 + 2 * (int64_t)depth * m < dw / 2;
    uint16_t* lst = tv.row16(row);  // list row: [0] = m, then [d][m] buckets
    uint4* d4 = reinterpret_cast<uint4*>(tv.row16(row));
    int bits = (as_list || m <= u4_keys) ? 4 : 8;
    uint32_t vmax = 0;
    bool ovf = false, slow = false;  // slow: a reduced key >= 2^32 (bucket_q's route does not take it)
    for (;;) {
      const int lg = bits == 4 ? 3 : 2;  // log2(counters per word)
      const uint32_t cap = (1u << bits) - 1u;
      const int nq = (w * bits) >> 7;  // uint4 per sketch row
      vmax = 0;
      ovf = false;
      for (int r = 0; r < depth; ++r) {
        for (int j = lane; j < nq; j += 64) slot4[j] = make_uint4(0, 0, 0, 0);
        uint32_t sq = 0;  // <= m * 255 < 2^22
        // the owner's keys, 4 per lane per step, the next step's loads in
        // flight (re-read per sketch row: an owner's tokens stay in L2)
        constexpr int kAhead = 4;
        uint64_t nx[kAhead];
        auto fetch = [&](int64_t base) {
#pragma unroll
          for (int u = 0; u < kAhead; ++u) {
            const int64_t i = base + lane + (int64_t)u * 64;
            nx[u] = i < hi ? keys.raw(i) : 0ULL;
          }
        };
        fetch(lo);
        for (int64_t base = lo; base < hi; base += 64 * kAhead) {
          uint64_t kk[kAhead];
#pragma unroll
          for (int u = 0; u < kAhead; ++u) kk[u] = nx[u];
          if (base + 64 * kAhead < hi) fetch(base + 64 * kAhead);
#pragma unroll
          for (int u = 0; u < kAhead; ++u) {
            const int64_t i = base + lane + (int64_t)u * 64;
            const uint64_t kp = keys.resolve(kk[u]);
            slow |= i < hi && (kp >> 32) != 0;
            if (i < hi && (kp >> 32) == 0) {
              const uint32_t c = bucket_q(hp, r, kp, (double)(uint32_t)kp, (uint32_t)kp & hp.wmask);
              const uint32_t sh = (c & ((1u << lg) - 1u)) * (uint32_t)bits;
              const uint32_t old = (atomicAdd(&slot[c >> lg], 1u << sh) >> sh) & cap;
              ovf |= old == cap;  // the add carried into the next counter: a wider form
              sq += 2u * old + 1u;
              vmax = max(vmax, old + 1u);
              if (as_list) lst[1 + (int64_t)r * m + (i - lo)] = (uint16_t)c;
            }
          }
        }
        if (__ballot(ovf | slow)) break;  // uniform: escalate (or hand the owner to k_build_mid)
        sq = wave_sum_u32(sq);
#ifdef CMS_BUILD_NOWRITE  // bound analysis only: no table stores
        if (false)
#endif
        if (!as_list)
          for (int j = lane; j < nq; j += 64) store_row(d4 + r * nq + j, slot4[j], SV);
        if (lane == 0) norm[row * depth + r] = sq;
      }
      if (!__ballot(ovf) || bits == 8 || __ballot(slow)) break;
      bits = 8;
    }
    if (__ballot(ovf | slow)) {  // a counter past 255 (u16 rows) or a key the quotient route does not take
      if (lane == 0) redo[atomicAdd(redo_cnt, 1u)] = (int32_t)row;
      continue;
    }
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) vmax = max(vmax, (uint32_t)__shfl_xor((int)vmax, o, 64));
    if (lane == 0) {
      if (as_list) lst[0] = (uint16_t)m;
      rowmax[row] = vmax;
      row_mass[row] = (uint64_t)m;
      hidx_w[row] = as_list ? kFormList : bits == 4 ? kFormU4 : kFormU8;
      cbound[row] = vmax;
    }
  }
}

// Mid-class owners through ONE key pass (Tunables::mid_image, when the
// [d][w] u16 image fits 80 KB): k_build_slices' scheme -- every sketch row
// counted at once in a [d][w] u16 LDS image (no carry: a mid owner's mass,
// hence every counter, stays below 2^16) with non-returning LDS adds -- then
// one read-back pass that finds the largest counter and each row's sum of
// squares, and a store pass that packs the image into the narrowest form
// that holds it (4-bit, u8, u16; or the list row whose entries the key pass
// wrote).  No escalation passes, no per-row reloads of the keys.
constexpr int kImgThreads = 512;
template <int SV, int D>
__global__ __launch_bounds__(kImgThreads) void k_build_image(
    const int64_t* lo_, const int64_t* hi_, Keys keys, const float* vals, HashParams hp, const int32_t* list,
    const uint32_t* list_cnt, TableView tv, int32_t* hidx_w, uint32_t* cbound, uint64_t* row_mass, uint64_t* norm,
    uint32_t* rowmax, uint32_t* flags, int list_keys) {
  extern __shared__ __align__(16) uint32_t lds[];  // [d][w] u16 counters, two per word
  __shared__ unsigned long long s_norm[CMS_MAX_DEPTH];
  __shared__ unsigned long long s_mass;
  __shared__ uint32_t s_max;
  const int tid = threadIdx.x;
  const int w = (int)hp.width;
  const int64_t dw = (int64_t)hp.depth * w;
  const int words = (int)(dw >> 1);
  uint4* l4 = reinterpret_cast<uint4*>(lds);
  const uint32_t count = *list_cnt;
  for (uint32_t li = blockIdx.x; li < count; li += gridDim.x) {
    const int64_t row = list[li];
    const int64_t lo = lo_[row], hi = hi_[row];
    const int64_t m = hi - lo;
    for (int j = tid; j < (words >> 2); j += kImgThreads) l4[j] = make_uint4(0, 0, 0, 0);
    if (tid < CMS_MAX_DEPTH) s_norm[tid] = 0ULL;
    if (tid == 0) {
      s_mass = 0ULL;
      s_max = 0u;
    }
    __syncthreads();
    // a LIST row when the increments are units and the list beats the 4-bit
    // row (its entries leave during the key pass; a counter past 255 makes
    // the owner a dense u16 row instead, which overwrites them)
    const bool as_list = m <= list_keys && vals == nullptr && hp.frac_bits == 0 && (int64_t)hp.depth * m <= 8192 &&
                         2 + 2 * (int64_t)hp.depth * m < (int64_t)hp.depth * w / 2;
    uint16_t* lst = tv.row16(row);
    uint64_t mass = 0;
    bool badv = false;
    constexpr int kPer = 4;
    constexpr int64_t kStep = kPer * kImgThreads;
    uint64_t nx[kPer];
    auto fetch = [&](int64_t base) {
#pragma unroll
      for (int u = 0; u < kPer; ++u) {
        const int64_t i = base + tid + (int64_t)u * kImgThreads;
        nx[u] = i < hi ? keys.raw(i) : 0ULL;
      }
    };
    if (lo < hi) fetch(lo);
    for (int64_t base = lo; base < hi; base += kStep) {
      uint64_t kk[kPer];
#pragma unroll
      for (int u = 0; u < kPer; ++u) kk[u] = nx[u];
      if (base + kStep < hi) fetch(base + kStep);
#pragma unroll
      for (int u = 0; u < kPer; ++u) {
        const int64_t i = base + tid + (int64_t)u * kImgThreads;
        if (i >= hi) continue;
        uint32_t inc;
        if (!load_inc(vals, i, inc, hp.frac_bits)) {
          badv = true;
          inc = 0;
        }
        mass += inc;
        if (!inc) continue;
        const uint64_t kp = keys.resolve(kk[u]);
        const int64_t t = i - lo;
        each_bucket<D>(hp, kp, [&](int r, uint32_t bk) {
          if (as_list) lst[1 + (int64_t)r * m + t] = (uint16_t)bk;
          const uint32_t c = (uint32_t)r * (uint32_t)w + bk;
          atomicAdd(&lds[c >> 1], inc << ((c & 1u) << 4));
        });
      }
    }
    __syncthreads();
    // read-back: largest counter and each sketch row's sum of squares (a row
    // of w counters is w/8 uint4; w % 32 == 0 for forms)
    {
      const int q_row = w >> 3;
      uint32_t vmax = 0;
      for (int d = 0; d < hp.depth; ++d) {
        uint32_t sq = 0;  // <= row mass * max counter < 2^32
        for (int j = tid; j < q_row; j += kImgThreads) {
          const uint4 v = l4[d * q_row + j];
          const uint32_t x[4] = {v.x, v.y, v.z, v.w};
#pragma unroll
          for (int q = 0; q < 4; ++q) {
            const u16x2 p = __builtin_bit_cast(u16x2, x[q]);
            sq = __builtin_amdgcn_udot2(p, p, sq, false);
            vmax = max(vmax, max(x[q] & 0xFFFFu, x[q] >> 16));
          }
        }
        sq = wave_sum_u32(sq);
        if ((tid & 63) == 0 && sq) atomicAdd(&s_norm[d], (unsigned long long)sq);
      }
#pragma unroll
      for (int o = 32; o > 0; o >>= 1) vmax = max(vmax, (uint32_t)__shfl_xor((int)vmax, o, 64));
      if ((tid & 63) == 0 && vmax) atomicMax(&s_max, vmax);
      mass = wave_sum_u64_sat(mass);
      if ((tid & 63) == 0 && mass) atomicAdd(&s_mass, (unsigned long long)mass);
    }
    __syncthreads();
    const uint32_t vmax = s_max;
    const bool listed = as_list && vmax <= 255u;
    const int level = vmax <= 15u ? 0 : vmax <= 255u ? 1 : 2;  // 4-bit, u8, u16
    uint4* d4 = reinterpret_cast<uint4*>(lst);
    if (!listed) {
      // 32 counters (4 uint4 of the image) per step: one uint4 of 4-bit,
      // two of u8 or four of u16 counters
      const int steps = (int)(dw >> 5);
      for (int s = tid; s < steps; s += kImgThreads) {
        const uint4 a = l4[4 * s], b = l4[4 * s + 1], c = l4[4 * s + 2], e = l4[4 * s + 3];
        const uint32_t x[16] = {a.x, a.y, a.z, a.w, b.x, b.y, b.z, b.w, c.x, c.y, c.z, c.w, e.x, e.y, e.z, e.w};
        if (level == 2) {
#ifdef CMS_BUILD_NOWRITE  // bound analysis only: no table stores
          if (false)
#endif
          {
            store_row(d4 + 4 * s, a, SV);
            store_row(d4 + 4 * s + 1, b, SV);
            store_row(d4 + 4 * s + 2, c, SV);
            store_row(d4 + 4 * s + 3, e, SV);
          }
        } else if (level == 1) {
          uint32_t y[8];
#pragma unroll
          for (int q = 0; q < 8; ++q) y[q] = __builtin_amdgcn_perm(x[2 * q + 1], x[2 * q], 0x06040200u);  // bytes 0, 2 of each
#ifdef CMS_BUILD_NOWRITE
          if (false)
#endif
          {
            store_row(d4 + 2 * s, make_uint4(y[0], y[1], y[2], y[3]), SV);
            store_row(d4 + 2 * s + 1, make_uint4(y[4], y[5], y[6], y[7]), SV);
          }
        } else {
          uint32_t y[4];
#pragma unroll
          for (int q = 0; q < 4; ++q) {
            // 8 counters < 16: x[4q..4q+3] hold two each in their u16 halves
            const uint32_t b0 = __builtin_amdgcn_perm(x[4 * q + 1], x[4 * q], 0x06040200u);
            const uint32_t b1 = __builtin_amdgcn_perm(x[4 * q + 3], x[4 * q + 2], 0x06040200u);
            y[q] = nibbles8(b0, b1);
          }
#ifdef CMS_BUILD_NOWRITE
          if (false)
#endif
          store_row(d4 + s, make_uint4(y[0], y[1], y[2], y[3]), SV);
        }
      }
    }
    if (badv) atomicOr(flags, kFlagBadValue);
    if (tid < hp.depth) norm[row * hp.depth + tid] = s_norm[tid];
    if (tid == 0) {
      rowmax[row] = vmax;
      row_mass[row] = s_mass;
      if (s_mass >= (1ULL << 32)) atomicOr(flags, kFlagOverflow);
      if (listed) lst[0] = (uint16_t)m;
      hidx_w[row] = listed ? kFormList : level == 0 ? kFormU4 : level == 1 ? kFormU8 : kFormU16;
      cbound[row] = vmax;
    }
    __syncthreads();  // image and shared sums consumed before the next owner
  }
}

// Byte-class owners (byte_class): ONE WAVE per owner, four owners per
// workgroup, each wave with its own w/2-byte LDS slot (4 KB at w = 8192).  The
// owner's keys are read once into registers; each sketch row in turn is
// counted in the slot as 1-, 2- or 4-bit counters (the narrowest form the
// owner's key count suggests, widened on overflow) and leaves as 16-B
// non-temporal stores of the slot itself (no packing).  The LDS adds
// return the old counter, so each sketch row's sum of squares (2 c inc +
// inc^2 per update, telescoping to the exact sum) and the row maximum come out
// of the update pass.  With 4 KB per owner 32 owners are in flight per CU
// (the wave limit), against 8 with a whole-sketch 20 KB image per workgroup
// (config 3: 5.1 ms for this kernel with 4-bit rows only, 3.1 ms with 1- and
// 2-bit rows, which halve and quarter the row bytes).  A counter that would pass 15 (a
// repeated key, a collision, an increment >= 16) is detected by its add; the
// owner is queued for k_build_bytes, which rewrites its whole slot, norms and
// maximum as a u8 row.  Waves never wait on each other (no workgroup barrier):
// one wave's LDS operations execute in program order.
#ifndef CMS_MID_GRID_PER_CU  // persistent k_build_mid workgroups per CU
#define CMS_MID_GRID_PER_CU 8
#endif
#ifndef CMS_NIB_WAVES
#define CMS_NIB_WAVES 4
#endif

constexpr int kNibWaves = CMS_NIB_WAVES;
// owners with at most Tunables::bit_keys (64) keys try 1-bit rows first, with
// at most crumb_keys (256) 2-bit rows
// A byte-class owner's first form: 1-bit rows up to bit_keys keys, 2-bit up
// to crumb_keys, else 4-bit
__host__ __device__ __forceinline__ int nib_first_bits(int64_t m, int w, int bit_keys, int crumb_keys) {
  return (m <= bit_keys && (w & 127) == 0) ? 1 : (m <= crumb_keys && (w & 63) == 0) ? 2 : 4;
}
// ... stored as a list row: unit increments, at most list_keys keys, and the
// list (2 + 2 d m bytes) no larger than the dense row it would take first
__host__ __device__ __forceinline__ bool nib_list_row(int64_t m, int w, int d, bool weighted, int frac_bits,
                                                      int bit_keys, int crumb_keys, int list_keys) {
  return m <= list_keys && !weighted && frac_bits == 0 &&
         2 + 2 * (int64_t)d * m <= ((int64_t)d * w * nib_first_bits(m, w, bit_keys, crumb_keys)) / 8;
}

// Compact layout of a fresh build (row_layout): each row's arena capacity in
// 128-B units, by what its class's kernel can store -- a hot row nothing (its
// counters are u32 slot rows), a byte-class row its list entries or its u8
// image (k_build_nibbles' forms up to k_build_bytes' u8 rows), any other row
// (the mid class, or every row without forms) a whole u16 slot (kCapU16).
__global__ void k_row_caps(const int64_t* lo_, const int64_t* hi_, int64_t n, const uint64_t* bound,
                           const int32_t* hidx, int forms, int weighted, int frac_bits, int d, int w, int bit_keys,
                           int crumb_keys, int list_keys, uint32_t* caps) {
  const int64_t dw = (int64_t)d * w;
  const uint32_t full = (uint32_t)(slot_units(dw) / kRowAlign);
  for (int64_t r = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; r < n; r += (int64_t)gridDim.x * blockDim.x) {
    const int32_t s = hidx[r];
    const int64_t m = hi_[r] - lo_[r];
    uint32_t c = full;
    if (s >= 0) {
      c = 0;
    } else if (forms && byte_class(s, m, bound[r])) {
      const int64_t u16s = nib_list_row(m, w, d, weighted != 0, frac_bits, bit_keys, crumb_keys, list_keys)
                               ? 1 + (int64_t)d * m  // [0] = m, then the d x m entries
                               : dw / 2;             // the u8 image
      c = (uint32_t)((u16s + kRowAlign - 1) / kRowAlign);
    }
    caps[r] = c;
  }
}

// One byte-class owner by one wave (k_build_nibbles).  D > 0 (the handle's
// depth is 4 or 5): every key's d buckets are hashed up front, as d
// independent chains (an owner here has one key or a few per lane, so one
// row at a time left the wave waiting on each hash's fp64 dependency chain),
// kept in registers through the row passes and the form escalations.
template <int SV, int D>
__device__ __forceinline__ void nib_owner(
    int64_t row, uint32_t* lds, const int64_t* lo_, const int64_t* hi_, const Keys& keys, const float* vals,
    const HashParams& hp, const int32_t* row_hot, const uint64_t* bound, const TableView& tv, int32_t* hidx_w,
    uint32_t* cbound, uint64_t* row_mass, uint64_t* norm, uint32_t* rowmax, uint32_t* flags, int32_t* redo,
    uint32_t* redo_cnt, int bit_keys, int crumb_keys, int list_keys) {
  const int lane = threadIdx.x & 63;
  const int wv = threadIdx.x >> 6;
  const int64_t lo = lo_[row], hi = hi_[row];
  if (row_hot[row] >= 0 || !byte_class(tv.hidx[row], hi - lo, bound[row])) return;
  const int w = (int)hp.width;
  uint64_t kp[kKeyRegs];
  uint32_t ik[kKeyRegs];
  uint32_t mass = 0;
  bool badv = false;
#pragma unroll
  for (int k = 0; k < kKeyRegs; ++k) {
    const int64_t i = lo + lane + (int64_t)k * 64;
    kp[k] = 0;
    ik[k] = 0;
    if (i < hi) {
      uint32_t inc;
      if (!load_inc(vals, i, inc, hp.frac_bits)) {
        badv = true;
        inc = 0;
      }
      kp[k] = keys.at(i);
      ik[k] = inc;
      mass += inc;
    }
  }
  // 1-bit counters first for owners of <= bit_keys keys, 2-bit for <=
  // crumb_keys (most byte-class owners: no counter reaches 4), 4-bit for the
  // rest; an add that overflows the form restarts the owner one form wider
  // (the wider rows overwrite every byte the narrower ones wrote), and past 15
  // the owner goes to k_build_bytes (u8)
  const int64_t m = hi - lo;
  // list rows (cms_internal.h kFormList): unit increments, at most list_keys
  // keys; counted as 4-bit in LDS for the norms and the maximum only, the
  // entries leave as the owner's buckets (nib_first_bits / nib_list_row: the
  // compact layout sizes the row by the same rule, k_row_caps)
  int bits = nib_first_bits(m, w, bit_keys, crumb_keys);
  const bool as_list = nib_list_row(m, w, hp.depth, vals != nullptr, hp.frac_bits, bit_keys, crumb_keys, list_keys);
  if (as_list) bits = 4;
  uint16_t* lst = tv.row16(row);  // list row: [0] = m, then [d][m] buckets
  uint4* slot4 = reinterpret_cast<uint4*>(lds) + wv * (w >> 5);  // w/2 bytes per wave (the 4-bit row)
  uint32_t* slot = lds + wv * (w >> 3);
  uint4* d4 = reinterpret_cast<uint4*>(tv.row16(row));  // the row's u16 slot (64-B aligned)
  uint32_t vmax = 0;
  bool ovf = false;
  // D > 0: the first register slot's key (an owner of <= 64 keys: its only
  // one) has its d buckets hashed up front; a row pass picks its bucket by a
  // select chain (the row index is not a compile-time constant there)
  uint32_t b0 = 0, b1 = 0, b2 = 0, b3 = 0, b4 = 0;
  if (D > 0 && ik[0])
    each_bucket<D>(hp, kp[0], [&](int r, uint32_t c) {
      if (r == 0) b0 = c;
      else if (r == 1) b1 = c;
      else if (r == 2) b2 = c;
      else if (r == 3) b3 = c;
      else b4 = c;
    });
  for (;;) {
    const int lg = bits == 1 ? 5 : bits == 2 ? 4 : 3;  // log2(counters per 32-bit word)
    const uint32_t cap = (1u << bits) - 1u;
    const int nq = (w * bits) >> 7;   // uint4 per sketch row
    vmax = 0;
    ovf = false;
    // a list row's counts leave nothing behind: its adds are taken back after
    // each sketch row (CMS_NIB_UNADD), so only the first row zeroes the slot
    const bool unadd = CMS_NIB_UNADD && as_list;
    // a list owner of <= 64 keys (one per lane) clears the words its adds
    // touched instead of zeroing the whole 4-bit row before the next sketch row
    const bool clear1 = CMS_NIB_CLEAR1 && as_list && m <= 64;
    uint32_t c0 = 0;
    for (int d = 0; d < hp.depth; ++d) {
      if ((!unadd && !clear1) || d == 0)
        for (int j = lane; j < nq; j += 64) slot4[j] = make_uint4(0, 0, 0, 0);
      uint32_t sq = 0;
#pragma unroll
      for (int k = 0; k < kKeyRegs; ++k)
        if (ik[k]) {
          const uint32_t c = (D > 0 && k == 0)
                                 ? (d == 0 ? b0 : d == 1 ? b1 : d == 2 ? b2 : d == 3 ? b3 : b4)
                                 : bucket(hp, d, kp[k]);
          if (k == 0) c0 = c;
          const uint32_t sh = (c & ((1u << lg) - 1u)) * (uint32_t)bits;
          const uint32_t old = (atomicAdd(&slot[c >> lg], ik[k] << sh) >> sh) & cap;
          const uint32_t nv = old + ik[k];
          ovf |= nv > cap || ik[k] > cap;  // the add carried into the next counter: a wider form
          sq += (2u * old + ik[k]) * ik[k];
          vmax = max(vmax, nv);
          if (as_list) lst[1 + (int64_t)d * m + lane + 64 * k] = (uint16_t)c;
        }
      if (__ballot(ovf)) break;  // uniform: escalate (the slot is zeroed by the next owner's first row)
      // every nonzero nibble sits in a word some lane added into: those words
      // back to zero (after all the row's adds: one wave's LDS operations
      // execute in program order)
      if (clear1 && ik[0]) slot[c0 >> lg] = 0u;
      if (unadd) {  // no counter carried (checked above), so each subtraction only removes its own add
#pragma unroll
        for (int k = 0; k < kKeyRegs; ++k)
          if (ik[k]) {  // (the bucket read back from the entry this lane just wrote: no registers held)
            const uint32_t c = lst[1 + (int64_t)d * m + lane + 64 * k];
            atomicSub(&slot[c >> lg], ik[k] << ((c & ((1u << lg) - 1u)) * (uint32_t)bits));
          }
      }
      sq = wave_sum_u32(sq);  // <= mass * 15
#ifdef CMS_BUILD_NOWRITE  // bound analysis only: no table stores
      if (false)
#endif
      if (!as_list)
        for (int j = lane; j < nq; j += 64) store_row(d4 + d * nq + j, slot4[j], SV);
      if (lane == 0) norm[row * hp.depth + d] = sq;
    }
    if (!__ballot(ovf) || bits == 4) break;
    bits *= 2;
  }
  if (as_list && lane == 0) lst[0] = (uint16_t)m;
  if (badv) atomicOr(flags, kFlagBadValue);
  if (__ballot(ovf)) {  // to k_build_bytes; a list row (~row) stays one there: its counters are < 2^8 (m < 2^8)
    if (lane == 0) redo[atomicAdd(redo_cnt, 1u)] = as_list ? ~(int32_t)row : (int32_t)row;
    return;
  }
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) vmax = max(vmax, (uint32_t)__shfl_xor((int)vmax, o, 64));
  mass = wave_sum_u32(mass);  // < 2^8 (byte class)
  if (lane == 0) {
    rowmax[row] = vmax;
    row_mass[row] = mass;
    hidx_w[row] = as_list ? kFormList : bits == 1 ? kFormU1 : bits == 2 ? kFormU2 : kFormU4;
    cbound[row] = vmax;
  }
}


// Grid: one owner per wave, or (Tunables::nib_persist) persistent waves that
// take owners gw, gw + nw, ... -- a quarter of a million four-wave workgroups
// of a few thousand cycles each can be bound by the workgroup dispatch rate.
template <int SV, int D>
__global__ __launch_bounds__(64 * kNibWaves) __attribute__((amdgpu_waves_per_eu(8, 8))) void k_build_nibbles(
    const int64_t* lo_, const int64_t* hi_, Keys keys, const float* vals, int64_t nrows, HashParams hp,
    const int32_t* row_hot, const uint64_t* bound, TableView tv, int32_t* hidx_w, uint32_t* cbound, uint64_t* row_mass,
    uint64_t* norm, uint32_t* rowmax, uint32_t* flags, int32_t* redo, uint32_t* redo_cnt, int bit_keys,
    int crumb_keys, int list_keys) {
  extern __shared__ __align__(16) uint32_t lds[];  // [kNibWaves][w / 8] words: one sketch row of nibbles per wave
  const int64_t nw = (int64_t)gridDim.x * kNibWaves;
  for (int64_t row = (int64_t)blockIdx.x * kNibWaves + (threadIdx.x >> 6); row < nrows; row += nw)
    nib_owner<SV, D>(row, lds, lo_, hi_, keys, vals, hp, row_hot, bound, tv, hidx_w, cbound, row_mass, norm, rowmax, flags,
                  redo, redo_cnt, bit_keys, crumb_keys, list_keys);
}

// The byte-class owners a counter >= 16 sent back from k_build_nibbles: the
// same one-pass build on a [d][w] u8 image (dw bytes of LDS), stored as u8
// rows -- or, for a list row (listed as ~row), its entries written whole and
// the list kept (the compact layout sized it as a list; a list holds any
// counter below 2^8).  A persistent grid walks the device-side list (no host
// count).
template <int SV>
__global__ __launch_bounds__(kBuildThreads) void k_build_bytes(
    const int64_t* lo_, const int64_t* hi_, Keys keys, const float* vals, HashParams hp,
    const int32_t* list, const uint32_t* list_cnt, TableView tv, int32_t* hidx_w, uint32_t* cbound,
    uint64_t* row_mass, uint64_t* norm, uint32_t* rowmax, uint32_t* flags) {
  extern __shared__ __align__(16) uint32_t lds[];  // [d][w] bytes
  __shared__ unsigned long long s_norm[CMS_MAX_DEPTH];
  __shared__ uint32_t s_max, s_mass;
  const int tid = threadIdx.x;
  const int w = (int)hp.width;
  const int64_t dw = (int64_t)hp.depth * w;
  const uint32_t count = *list_cnt;
  for (uint32_t li = blockIdx.x; li < count; li += gridDim.x) {
    const bool keep_list = list[li] < 0;
    const int64_t row = keep_list ? ~(int64_t)list[li] : (int64_t)list[li];
    const int64_t lo = lo_[row], hi = hi_[row];
    uint16_t* lst = tv.row16(row);  // list row: [0] = m (k_build_nibbles wrote it), then [d][m] buckets
    if (tid < CMS_MAX_DEPTH) s_norm[tid] = 0ULL;
    if (tid == 0) {
      s_max = 0u;
      s_mass = 0u;
    }
    uint64_t kp[kKeyRegs];
    uint32_t ik[kKeyRegs];
    uint32_t mass = 0;
    bool badv = false;
#pragma unroll
    for (int k = 0; k < kKeyRegs; ++k) {
      const int64_t i = lo + tid + (int64_t)k * kBuildThreads;
      kp[k] = 0;
      ik[k] = 0;
      if (i < hi) {
        uint32_t inc;
        if (!load_inc(vals, i, inc, hp.frac_bits)) {
          badv = true;
          inc = 0;
        }
        kp[k] = keys.at(i);
        ik[k] = inc;
        mass += inc;
      }
    }
    const int nq = (int)(dw >> 4);  // uint4 words of the byte image
    uint4* l4 = reinterpret_cast<uint4*>(lds);
    for (int j = tid; j < nq; j += kBuildThreads) l4[j] = make_uint4(0, 0, 0, 0);
    __syncthreads();
    uint32_t vmax = 0;
    for (int d = 0; d < hp.depth; ++d) {
      uint32_t sq = 0;
#pragma unroll
      for (int k = 0; k < kKeyRegs; ++k)
        if (ik[k]) {
          const uint32_t bk = bucket(hp, d, kp[k]);
          const uint32_t c = (uint32_t)d * (uint32_t)w + bk;
          if (keep_list) lst[1 + (int64_t)d * (hi - lo) + tid + (int64_t)k * kBuildThreads] = (uint16_t)bk;
          const uint32_t sh = (c & 3u) << 3;
          const uint32_t old = (atomicAdd(&lds[c >> 2], ik[k] << sh) >> sh) & 255u;  // < 2^8: no carry
          sq += (2u * old + ik[k]) * ik[k];
          vmax = max(vmax, old + ik[k]);
        }
      sq = wave_sum_u32(sq);  // <= mass * 255 < 2^16
      if ((tid & 63) == 0 && sq) atomicAdd(&s_norm[d], (unsigned long long)sq);
    }
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) vmax = max(vmax, (uint32_t)__shfl_xor((int)vmax, o, 64));
    if ((tid & 63) == 0 && vmax) atomicMax(&s_max, vmax);
    mass = wave_sum_u32(mass);
    if ((tid & 63) == 0 && mass) atomicAdd(&s_mass, mass);
    __syncthreads();
    uint4* d4 = reinterpret_cast<uint4*>(lst);
#ifdef CMS_BUILD_NOWRITE  // bound analysis only: no table stores
    if (false)
#endif
    if (!keep_list)
      for (int j = tid; j < nq; j += kBuildThreads) store_row(d4 + j, l4[j], SV);
    if (badv) atomicOr(flags, kFlagBadValue);
    if (tid < hp.depth) norm[row * hp.depth + tid] = s_norm[tid];
    if (tid == 0) {
      rowmax[row] = s_max;
      row_mass[row] = s_mass;
      hidx_w[row] = keep_list ? kFormList : kFormU8;
      cbound[row] = s_max;
    }
    __syncthreads();  // the image and the shared sums are consumed before the next owner
  }
}

// Hot (split) owners with unit increments: one workgroup per SLICE of up to
// kHotSlice keys, all d sketch rows counted at once in an LDS image of u16
// counters ([d][w] u16: a slice of < 2^16 >> frac_bits unit increments cannot
// carry out of one), so each key is read and hashed ONCE (k_build_rows walks
// a slice's keys once per pair of sketch rows).  The image is added into the
// owner's u32 slot row (zeroed by promote_rows, or the old counters of an
// accumulating build) with 64-bit global atomics, two adjacent counters per
// add: a counter stays below its row mass < 2^32, so the low half never
// carries into the high one.  Bigger slices than k_build_rows' mean fewer
// dense slice images added into the slots.  No static LDS: two 80 KB images
// share a CU at d = 5, w = 8192.
constexpr int kSliceThreads = 512;
// a fresh build's single-slice owners store their slot rows whole (no slot
// zeroing, no 64-bit slot atomics; norms from the same pass)
#ifndef CMS_WHOLE_SLICES
#define CMS_WHOLE_SLICES 1
#endif
constexpr int64_t kHotSlice = 65535;  // keys per slice (u16 image, frac_bits 0)
// D: the depth when it is 4 or 5 (rows unrolled, each_bucket), else 0
template <int D>
__global__ __launch_bounds__(kSliceThreads) void k_build_slices(const int64_t* lo_, const int64_t* hi_, Keys keys,
                                                                HashParams hp, int64_t slice, const HotInfo* hot,
                                                                const int2* smap, const uint32_t* counters,
                                                                TableView tv, uint64_t* row_mass, uint32_t* flags,
                                                                uint16_t* img_out, int whole, uint64_t* norm,
                                                                uint32_t* rowmax) {
  extern __shared__ __align__(16) uint32_t lds[];  // [d * w / 2] words, two u16 counters each
  const uint32_t nsl = counters[1];
  if (blockIdx.x >= nsl) return;
  const int tid = threadIdx.x;
  // a Zipf head owner has hundreds of slices, adjacent in smap: workgroups
  // take the slices in a strided order (a prime stride is a bijection unless
  // it divides the count) so the ones running together belong to many owners
  // and their row adds do not all land on one 160 KB slot row at once
  const uint32_t stride = (nsl % 7919u) ? 7919u : 7907u;
  const uint32_t sidx = (uint32_t)(((uint64_t)blockIdx.x * stride) % nsl);  // the mapped slice (its image index)
  const int2 m = smap[sidx];
  const int64_t row = hot[m.x].row;
  const int64_t lo = lo_[row] + (int64_t)m.y * slice;
  const int64_t end = min(hi_[row], lo + slice);
  const int w = (int)hp.width;
  const int64_t dw = (int64_t)hp.depth * w;
  const int words = (int)(dw >> 1);
  uint4* l4 = reinterpret_cast<uint4*>(lds);
  for (int j = tid; j < (words >> 2); j += kSliceThreads) l4[j] = make_uint4(0, 0, 0, 0);
  for (int j = (words & ~3) + tid; j < words; j += kSliceThreads) lds[j] = 0u;
  __syncthreads();
  const uint32_t one = 1u << hp.frac_bits;
  // eight keys per thread per step; the next step's eight loads are issued
  // before this step's keys are hashed, so a key load's latency is hidden
  // behind the previous keys' d x 8 hashes and LDS adds
  constexpr int kPer = 8;  // (4: the same time, profiles/r04/ab_*_s5)
  constexpr int64_t kStep = kPer * kSliceThreads;
  uint64_t nx[kPer];
  auto fetch = [&](int64_t base) {
#pragma unroll
    for (int u = 0; u < kPer; ++u) {
      const int64_t i = base + tid + (int64_t)u * kSliceThreads;
      nx[u] = i < end ? keys.raw(i) : 0ULL;
    }
  };
  if (lo < end) fetch(lo);
  for (int64_t base = lo; base < end; base += kStep) {
    uint64_t kk[kPer];
#pragma unroll
    for (int u = 0; u < kPer; ++u) kk[u] = nx[u];
    if (base + kStep < end) fetch(base + kStep);
#pragma unroll
    for (int u = 0; u < kPer; ++u) {
      if (base + tid + (int64_t)u * kSliceThreads >= end) continue;  // (a raw key may be any 64-bit value)
      const uint64_t kp = keys.resolve(kk[u]);
      each_bucket<D>(hp, kp, [&](int r, uint32_t bk) {
        const uint32_t c = (uint32_t)r * (uint32_t)w + bk;
#ifdef CMS_BUILD_NOLDSADD  // bound analysis only: hashes kept live, no LDS adds
        if (c == 0xFFFFFFFFu)
#endif
        atomicAdd(&lds[c >> 1], one << ((c & 1u) << 4));
      });
    }
  }
  __syncthreads();
  if (whole && hot[m.x].nslices == 1) {
    // the owner's only slice, in a fresh build: its slot row is the image
    // itself (the slot was not zeroed), stored whole as u32 counters with
    // 16-B non-temporal stores; its sums of squares and largest counter come
    // from the same pass (k_hot_norms skips it)
    u32x4_t* o4 = reinterpret_cast<u32x4_t*>(tv.hot + (int64_t)tv.hidx[row] * dw);
    const uint2* s2 = reinterpret_cast<const uint2*>(lds);
    uint32_t vmax = 0;
    for (int r = 0; r < hp.depth; ++r) {
      uint64_t sq = 0;
      const int q0 = r * (w >> 2), q1 = q0 + (w >> 2);  // uint4 of u32 counters (4 per) of sketch row r
      for (int q = q0 + tid; q < q1; q += kSliceThreads) {
        const uint2 v = s2[q];  // four u16 counters
        const uint32_t c0 = v.x & 0xFFFFu, c1 = v.x >> 16, c2 = v.y & 0xFFFFu, c3 = v.y >> 16;
        sq += (uint64_t)c0 * c0 + (uint64_t)c1 * c1 + (uint64_t)c2 * c2 + (uint64_t)c3 * c3;
        vmax = max(max(vmax, max(c0, c1)), max(c2, c3));
        const u32x4_t x = {c0, c1, c2, c3};
        __builtin_nontemporal_store(x, o4 + q);
      }
      sq = wave_sum_u64_sat(sq);  // (no static LDS: two 80 KB images share a CU)
      if ((tid & 63) == 0 && sq) atomicAdd((unsigned long long*)&norm[row * hp.depth + r], (unsigned long long)sq);
    }
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) vmax = max(vmax, (uint32_t)__shfl_xor((int)vmax, o, 64));
    if ((tid & 63) == 0 && vmax) atomicMax(&rowmax[row], vmax);
  } else if (img_out) {
    // the slice's image leaves whole, as u16 counters with 16-B non-temporal
    // stores; k_slice_reduce sums an owner's images into its slot row (no
    // global atomics here)
    u32x4_t* o4 = reinterpret_cast<u32x4_t*>(img_out + (int64_t)sidx * dw);
    const uint4* s4 = reinterpret_cast<const uint4*>(lds);
    for (int j = tid; j < (words >> 2); j += kSliceThreads) {
      const uint4 v = s4[j];
      const u32x4_t x = {v.x, v.y, v.z, v.w};
      __builtin_nontemporal_store(x, o4 + j);
    }
  } else {
  unsigned long long* dst = reinterpret_cast<unsigned long long*>(tv.hot + (int64_t)tv.hidx[row] * dw);
  // the slices of one owner start their sweep at different 512-B-aligned
  // offsets of the slot row (same-address atomics from many workgroups queue)
  const int units = (words + 63) >> 6;
  const int rot = (int)(((uint32_t)m.y * 2654435761u >> 8) % (uint32_t)units) << 6;
  for (int jj = tid; jj < words; jj += kSliceThreads) {
    const int j = jj + rot < words ? jj + rot : jj + rot - words;
    const uint32_t v = lds[j];
#ifdef CMS_BUILD_NOSLICEADD  // bound analysis only: the slices' global atomics skipped
    if (v == 0xFFFFFFFFu)
#endif
    if (v) atomicAdd(dst + j, (unsigned long long)(v & 0xFFFFu) | ((unsigned long long)(v >> 16) << 32));
  }
  }
  if (tid == 0) {
    const uint64_t tm = (uint64_t)(end - lo) * one;
    const unsigned long long old = atomicAdd((unsigned long long*)&row_mass[row], (unsigned long long)tm);
    if (old + tm >= (1ULL << 32)) atomicOr(flags, kFlagOverflow);
  }
}

// Sum of squares of the hot rows after every slice landed; grid (<= 256, depth,
// chunks of 1024), blocks striding over the hot rows the plan counted (the
// host's bound on them is loose, and empty blocks still cost launch time).
// Norms and maxima of the hot (u32 slot) rows: one workgroup per (row,
// sketch row) at a time, the whole w counters in 16-byte loads (eight in
// flight per thread at w = 8192), one block reduction per sketch row.
// done_ns > 0: rows of at most done_ns slices already have their norms
// (k_slice_reduce stored them whole) and are skipped.
__global__ __launch_bounds__(256) void k_hot_norms(const HotInfo* hot, const uint32_t* counters, HashParams hp,
                                                   TableView tv, uint64_t* norm, uint32_t* rowmax, int done_ns) {
  __shared__ uint64_t red[4];
  const uint32_t nhot = counters[0];
  const int d = blockIdx.y;
  const int w = (int)hp.width;
  for (uint32_t hb = blockIdx.x; hb < nhot; hb += gridDim.x) {
    if (hot[hb].nslices <= done_ns) continue;  // (uniform per block)
    const int64_t row = hot[hb].row;
    const uint32_t* p = tv.hot + (int64_t)tv.hidx[row] * tv.dw + (int64_t)d * w;  // split rows are slots
    uint64_t sq = 0;
    uint32_t vmax = 0;
    if ((w & 3) == 0 && (((uintptr_t)p) & 15) == 0) {
      const uint4* p4 = reinterpret_cast<const uint4*>(p);
      for (int j = threadIdx.x; j < (w >> 2); j += 256) {
        const uint4 v = p4[j];
        sq = sat_add(sq, (uint64_t)v.x * v.x + (uint64_t)v.y * v.y);
        sq = sat_add(sq, (uint64_t)v.z * v.z + (uint64_t)v.w * v.w);
        vmax = max(vmax, max(max(v.x, v.y), max(v.z, v.w)));
      }
    } else {
      for (int j = threadIdx.x; j < w; j += 256) {
        sq = sat_add(sq, (uint64_t)p[j] * p[j]);
        vmax = max(vmax, p[j]);
      }
    }
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) vmax = max(vmax, (uint32_t)__shfl_xor((int)vmax, o, 64));
    if ((threadIdx.x & 63) == 0 && vmax) atomicMax(&rowmax[row], vmax);
    uint64_t tot = block_sum_u64_sat(sq, red);
    if (tot > (1ULL << 60)) tot = 1ULL << 60;
    if (threadIdx.x == 0) atomicAdd((unsigned long long*)&norm[row * hp.depth + d], (unsigned long long)tot);
  }
}

// The split owners' slot rows from their slices' u16 images (k_build_slices
// with img_out; Tunables::slice_reduce).  Task = (group of kRedGroup slices of
// one owner, chunk of 2048 counters): thread t sums 8 counters (one 16-B load
// per slice, four in flight) over the group's slices.  An owner of at most
// kRedGroup slices (nearly all: a split owner has a few) is one group per
// chunk, so its counters are stored whole -- the old ones added when
// accumulating -- and the same pass derives its rows' sums of squares and
// largest counter (k_hot_norms then skips it).  A Zipf head owner (hundreds of
// slices) has many groups, each adding its sums into the pre-zeroed (or old)
// slot with 64-bit atomics, two counters per add (no carry: every sum stays
// below the row mass < 2^32); k_hot_norms derives those rows' norms.
constexpr int kRedGroup = 16, kRedChunk = 2048;
__global__ __launch_bounds__(256) void k_slice_reduce(const HotInfo* hot, const int2* smap, const uint32_t* counters,
                                                      const uint16_t* img, HashParams hp, TableView tv, int accumulate,
                                                      uint64_t* norm, uint32_t* rowmax) {
  const uint32_t nsl = counters[1];
  const int64_t dw = tv.dw;
  const int w = (int)hp.width;
  const int nchunk = (int)((dw + kRedChunk - 1) / kRedChunk);
  const int lane = threadIdx.x & 63;
  for (int64_t t = blockIdx.x; t < (int64_t)nsl * nchunk; t += gridDim.x) {
    const uint32_t e = (uint32_t)(t / nchunk);
    const int ch = (int)(t - (int64_t)e * nchunk);
    const int2 m = smap[e];
    if (m.y % kRedGroup) continue;  // not a group's first slice (uniform per block)
    const HotInfo hi = hot[m.x];
    const int s1 = min(hi.nslices, m.y + kRedGroup);
    const int64_t j0 = (int64_t)ch * kRedChunk + (int64_t)threadIdx.x * 8;  // this thread's 8 counters
    const bool in = j0 < dw;
    uint32_t s[8] = {0, 0, 0, 0, 0, 0, 0, 0};
    auto add = [&](const u32x4_t v) {
      const uint32_t x[4] = {v.x, v.y, v.z, v.w};
#pragma unroll
      for (int c = 0; c < 4; ++c) {
        s[2 * c] += x[c] & 0xFFFFu;
        s[2 * c + 1] += x[c] >> 16;
      }
    };
    if (in) {
      const uint16_t* base = img + (int64_t)hi.e0 * dw + j0;
      auto src = [&](int sl) { return reinterpret_cast<const u32x4_t*>(base + (int64_t)sl * dw); };
      int sl = m.y;
      for (; sl + 3 < s1; sl += 4) {
        const u32x4_t a = __builtin_nontemporal_load(src(sl)), b = __builtin_nontemporal_load(src(sl + 1));
        const u32x4_t c = __builtin_nontemporal_load(src(sl + 2)), f = __builtin_nontemporal_load(src(sl + 3));
        add(a);
        add(b);
        add(c);
        add(f);
      }
      for (; sl < s1; ++sl) add(__builtin_nontemporal_load(src(sl)));
    }
    uint32_t* dst = tv.hot + (int64_t)tv.hidx[hi.row] * dw + j0;
    if (hi.nslices > kRedGroup) {  // several groups: add into the slot
      if (in) {
        unsigned long long* d2 = reinterpret_cast<unsigned long long*>(dst);
#pragma unroll
        for (int c = 0; c < 4; ++c)
          if (s[2 * c] | s[2 * c + 1])
            atomicAdd(d2 + c, (unsigned long long)s[2 * c] | ((unsigned long long)s[2 * c + 1] << 32));
      }
      continue;
    }
    uint64_t sq = 0;
    uint32_t vmax = 0;
    if (in) {
      uint4* d4 = reinterpret_cast<uint4*>(dst);
      if (accumulate) {
        const uint4 a = d4[0], b = d4[1];
        s[0] += a.x; s[1] += a.y; s[2] += a.z; s[3] += a.w;
        s[4] += b.x; s[5] += b.y; s[6] += b.z; s[7] += b.w;
      }
      d4[0] = make_uint4(s[0], s[1], s[2], s[3]);
      d4[1] = make_uint4(s[4], s[5], s[6], s[7]);
#pragma unroll
      for (int c = 0; c < 8; ++c) {
        sq = sat_add(sq, (uint64_t)s[c] * s[c]);
        vmax = max(vmax, s[c]);
      }
    }
    // the wave's 512 counters lie in one sketch row when w is a multiple of
    // 512 (config 3); otherwise each lane adds its own (w % 8 == 0: a
    // thread's 8 counters never straddle two rows)
    const int r = in ? (int)(j0 / w) : -1;
    const int r0 = __builtin_amdgcn_readfirstlane(r);
    if (__ballot(r != r0) == 0ULL) {
#pragma unroll
      for (int o = 32; o > 0; o >>= 1) vmax = max(vmax, (uint32_t)__shfl_xor((int)vmax, o, 64));
      sq = wave_sum_u64_sat(sq);
      if (lane == 0 && r0 >= 0) {
        if (vmax) atomicMax(&rowmax[hi.row], vmax);
        if (sq) atomicAdd((unsigned long long*)&norm[hi.row * hp.depth + r0], (unsigned long long)(sq > (1ULL << 60) ? (1ULL << 60) : sq));
      }
    } else if (in) {
      if (vmax) atomicMax(&rowmax[hi.row], vmax);
      if (sq) atomicAdd((unsigned long long*)&norm[hi.row * hp.depth + r], (unsigned long long)(sq > (1ULL << 60) ? (1ULL << 60) : sq));
    }
  }
}

// Early slices (Tunables::early_slices): the hot-routed owners of more than
// `split` keys, whose keys pass 1 of the partition already placed, claim hot
// slot base + t (t: their routing slot), their spans and slice map, with
// their norms and maxima zeroed -- one thread per routing slot, the slice map
// written by the row's own thread (a Zipf head owner: ~1000 slices).
__global__ void k_early_plan(const unsigned long long* slotkey, const uint32_t* bs1, int P1, int nslots,
                             int64_t split, int64_t slice, int64_t base, int32_t* hidx, uint8_t* early, int64_t* elo,
                             int64_t* ehi, HotInfo* hot, int2* extra_map, uint32_t* counters, uint64_t* norm,
                             uint32_t* rowmax, int depth) {
  const int t = blockIdx.x * blockDim.x + threadIdx.x;
  if (t >= nslots) return;
  const uint32_t o1 = (uint32_t)slotkey[t];
  if (o1 == 0) return;
  const int64_t row = (int64_t)o1 - 1;
  const int64_t lo = bs1[P1 + t], hi = bs1[P1 + t + 1];
  if (hi - lo <= split) return;  // built with the other rows after pass 2
  const int32_t ns = (int32_t)((hi - lo + slice - 1) / slice);
  const unsigned long long old = atomicAdd(reinterpret_cast<unsigned long long*>(counters), ((unsigned long long)ns << 32) | 1ULL);
  const uint32_t hx = (uint32_t)old, e0 = (uint32_t)(old >> 32);
  hot[hx] = HotInfo{row, ns, (int32_t)e0};
  for (int32_t sl = 0; sl < ns; ++sl) extra_map[e0 + sl] = make_int2((int)hx, sl);
  early[row] = 1;
  elo[row] = lo;
  ehi[row] = hi;
  hidx[row] = (int32_t)(base + t);
  for (int d = 0; d < depth; ++d) norm[row * depth + d] = 0;
  rowmax[row] = 0;
}

// ... and the slots of the early rows built by more than one slice (their
// slices add into the slot) are zeroed; a single slice stores its row whole.
__global__ __launch_bounds__(256) void k_early_zero(const HotInfo* hot, const uint32_t* counters, TableView tv) {
  const uint32_t nh = counters[0];
  for (uint32_t i = blockIdx.x; i < nh; i += gridDim.x) {
    if (hot[i].nslices <= 1) continue;
    uint4* dst = reinterpret_cast<uint4*>(tv.hot + (int64_t)tv.hidx[hot[i].row] * tv.dw);
    for (int64_t j = threadIdx.x; j < (tv.dw >> 2); j += 256) dst[j] = make_uint4(0, 0, 0, 0);
  }
}

int row_bounds(cms_handle* h, const int64_t* d_lo, const int64_t* d_hi, const float* d_val, const uint64_t* old_mass,
               int64_t slice, uint64_t* bound, uint8_t* force) {
  const int64_t n = h->n;
  if (d_val)
    hipLaunchKernelGGL(k_row_bound_values, dim3((unsigned)std::max<int64_t>(1, std::min<int64_t>(n, 65536))),
                       dim3(256), 0, h->stream, d_lo, d_hi, d_val, n, h->hp.frac_bits, slice, old_mass, bound, force);
  else
    hipLaunchKernelGGL(k_row_bound_implicit, dim3((unsigned)std::max<int64_t>(1, std::min<int64_t>((n + 255) / 256, 4096))),
                       dim3(256), 0, h->stream, d_lo, d_hi, n, h->hp.frac_bits, slice, old_mass, bound, force);
  CMS_HIP(hipGetLastError());
  return CMS_OK;
}

int ingest_csr_device(cms_handle* h, const int64_t* d_off, const int64_t* d_key, const float* d_val, int64_t npairs) {
  h->rf_valid = false;  // CSR batches do not mark touched owners: the next refresh is a full job
  return ingest_spans_device(h, d_off, d_off + 1, d_key, nullptr, d_val, npairs);
}

int ingest_spans_device(cms_handle* h, const int64_t* d_lo, const int64_t* d_hi, const int64_t* d_key,
                        const uint32_t* d_tok, const float* d_val, int64_t npairs) {
  const Keys keys{d_key, d_tok};
  const int64_t n = h->n;
  int rc0;
  const int accumulate = h->empty ? 0 : 1;
  // Rows with more than kSplit keys are hot: a u32 slot, built in slices.
  // kSplit: 8192 keys, or 16384 for rows of 8192+ counters (config 3: build
  // 19.4 -> 18.5 ms; config 2 prefers 8192).
  int64_t kSplit = cms::kSlice;
  if (h->p.width >= 8192) kSplit *= 2;
  if (h->tune.split_keys > 0) kSplit = h->tune.split_keys;
  // Unit increments whose [d][w] u16 image fits a workgroup's LDS: the
  // slices (every one, slice 0 included) run on k_build_slices, kHotSlice
  // keys each, one key pass.  Otherwise (weighted increments, wide shapes)
  // k_build_rows builds slices of kSplit keys, a pass per pair of sketch rows.
  const size_t img_lds = (size_t)h->dw * 2;
  const bool fast_slices = !d_val && (h->dw % 8) == 0 && img_lds <= 80 * 1024 && h->hp.frac_bits < 16;
  const int64_t kSliceKeys = fast_slices ? (kHotSlice >> h->hp.frac_bits) : kSplit;
  // a fresh build: single-slice owners store their slot rows whole
  // (k_build_slices), so their slots are not zeroed by the promotion
  const int whole_slices =
      CMS_WHOLE_SLICES && fast_slices && !accumulate && !h->tune.slice_reduce && (h->p.width % 4) == 0 ? 1 : 0;
  const int64_t max_hot = std::min<int64_t>(n, npairs / kSplit + 1);
  const int64_t emax = npairs / kSliceKeys + max_hot + 1;  // mapped slices
  const size_t sz_rowhot = (sizeof(int32_t) * (size_t)n + 15) & ~size_t(15);
  const size_t sz_hot = (sizeof(HotInfo) * (size_t)max_hot + 15) & ~size_t(15);
  const size_t sz_extra = sizeof(int2) * (size_t)emax;
  CMS_HIP(h->ws_hot.ensure(sz_rowhot + sz_hot + sz_extra + 64));
  char* base = h->ws_hot.as<char>();
  int32_t* row_hot = reinterpret_cast<int32_t*>(base);
  HotInfo* hot = reinterpret_cast<HotInfo*>(base + sz_rowhot);
  int2* extra_map = reinterpret_cast<int2*>(base + sz_rowhot + sz_hot);
  uint32_t* counters = h->d_flags + 4;  // [4..7]: hot rows, mapped slices (one u64 atomic), spare
  // Early slices (Tunables::early_slices): the hot-routed owners of more than
  // kSplit keys are final after pass 1 of the partition, so their rows are
  // claimed and built on side_stream3 beside pass 2 (k_early_plan,
  // k_early_zero, k_build_slices, k_hot_norms); the plan below skips them
  // (early flags) and the build joins them at its end.
  auto slices_kernel = [&]() {
    static bool attr = [] {
      for (const void* f : {(const void*)k_build_slices<0>, (const void*)k_build_slices<4>,
                            (const void*)k_build_slices<5>})
        (void)hipFuncSetAttribute(f, hipFuncAttributeMaxDynamicSharedMemorySize, 80 * 1024);
      return true;
    }();
    (void)attr;
    return h->p.depth == 5 ? k_build_slices<5> : h->p.depth == 4 ? k_build_slices<4> : k_build_slices<0>;
  };
  const uint8_t* eflag = nullptr;
  struct EarlyJoin {
    cms_handle* h;
    bool on = false;
    void end() {
      if (!on) return;
      on = false;
      (void)hipStreamWaitEvent(h->stream, h->ev_early, 0);
    }
    ~EarlyJoin() { end(); }
  } early_join{h};
  if (h->p1_event && !accumulate && fast_slices && whole_slices && h->forms_ok && (size_t)h->dw <= kFormLdsMax &&
      !h->plan_side_active) {
    h->p1_event = false;
    const hipStream_t s3 = h->side_stream3;
    const int nslots = h->p1_nslots;
    const int64_t emax_e = npairs / kSliceKeys + nslots + 1;
    const size_t sz_span = sizeof(int64_t) * (size_t)n;
    const size_t sz_flag = ((size_t)n + 15) & ~size_t(15);
    const size_t sz_ehot = (sizeof(HotInfo) * (size_t)nslots + 15) & ~size_t(15);
    CMS_HIP(h->ws_early.ensure(2 * sz_span + sz_flag + sz_ehot + sizeof(int2) * (size_t)emax_e + 64));
    char* eb = h->ws_early.as<char>();
    int64_t* elo = reinterpret_cast<int64_t*>(eb);
    int64_t* ehi = reinterpret_cast<int64_t*>(eb + sz_span);
    uint8_t* ef = reinterpret_cast<uint8_t*>(eb + 2 * sz_span);
    HotInfo* ehot = reinterpret_cast<HotInfo*>(eb + 2 * sz_span + sz_flag);
    int2* emap = reinterpret_cast<int2*>(eb + 2 * sz_span + sz_flag + sz_ehot);
    uint32_t* ecnt = h->d_flags + 12;  // [12..13]: early hot rows, mapped slices (one u64 atomic)
    // the table layout restarts here (the plan's own reset is skipped)
    CMS_HIP(hipStreamWaitEvent(s3, h->ev_p1, 0));
    CMS_HIP(hipMemsetAsync(h->d_hidx, 0xff, sizeof(int32_t) * (size_t)n, s3));
    h->hot_used = 0;
    int64_t ebase = 0;
    if ((rc0 = reserve_hot_slots(h, nslots, &ebase))) return rc0;
    CMS_HIP(hipMemsetAsync(ef, 0, (size_t)n, s3));
    CMS_HIP(hipMemsetAsync(ecnt, 0, 2 * sizeof(uint32_t), s3));
    hipLaunchKernelGGL(k_early_plan, dim3((unsigned)((nslots + 255) / 256)), dim3(256), 0, s3, h->p1_slotkey,
                       h->p1_bs1, h->p1_P1, nslots, kSplit, kSliceKeys, ebase, h->d_hidx, ef, elo, ehi, ehot, emap,
                       ecnt, h->d_norm, h->d_rowmax, h->p.depth);
    CMS_HIP(hipEventRecord(h->ev_e1, s3));  // rows claimed: the plan may read hidx and the flags
    hipLaunchKernelGGL(k_early_zero, dim3((unsigned)std::min(nslots, 1024)), dim3(256), 0, s3, ehot, ecnt, h->tview());
    hipLaunchKernelGGL(slices_kernel(), dim3((unsigned)emax_e), dim3(kSliceThreads), img_lds, s3, elo, ehi, keys,
                       h->hp, kSliceKeys, ehot, emap, ecnt, h->tview(), h->d_row_mass, h->d_flags, (uint16_t*)nullptr,
                       1, h->d_norm, h->d_rowmax);
    hipLaunchKernelGGL(k_hot_norms, dim3((unsigned)std::min(nslots, 1024), (unsigned)h->p.depth), dim3(256), 0, s3,
                       ehot, ecnt, h->hp, h->tview(), h->d_norm, h->d_rowmax, 1);
    CMS_HIP(hipGetLastError());
    CMS_HIP(hipEventRecord(h->ev_early, s3));
    early_join.on = true;
    eflag = ef;
  }
  h->p1_event = false;
  // A fresh unit-increment build right after a partition that marked its
  // spans (ingest_coo): the plan below needs only the spans, so it runs on
  // the side stream beside the partition's last scatter (h->stream swapped
  // for the section; joined back before the build reads the keys).
  struct PlanSide {
    cms_handle* h;
    bool on = false;
    void end() {
      if (!on) return;
      on = false;
      std::swap(h->stream, h->side_stream);
      h->plan_side_active = false;
      if (hipEventRecord(h->ev_plan, h->side_stream) == hipSuccess) (void)hipStreamWaitEvent(h->stream, h->ev_plan, 0);
    }
    ~PlanSide() { end(); }
  } plan_side{h};
  if (h->spans_event && !accumulate && !d_val && h->side_stream) {
    h->spans_event = false;
    CMS_HIP(hipStreamWaitEvent(h->side_stream, h->ev_spans, 0));
    std::swap(h->stream, h->side_stream);
    h->plan_side_active = true;  // nothing in the section may launch on h->side_stream (it is the main stream now)
    plan_side.on = true;
  }
  if (eflag) CMS_HIP(hipStreamWaitEvent(h->stream, h->ev_e1, 0));  // the early rows' claims first
  CMS_HIP(hipMemsetAsync(counters, 0, 4 * sizeof(uint32_t), h->stream));
  // table layout: rows that could reach 2^16, and split rows, get u32 slots
  {
    TimedScope ts(h, "build_plan");
    if (!accumulate && !eflag && (rc0 = reset_table_layout(h))) return rc0;
    DevBuf& bound = h->ws_bound;
    DevBuf& force = h->ws_force;
    CMS_HIP(bound.ensure(sizeof(uint64_t) * (size_t)std::max<int64_t>(n, 1)));
    CMS_HIP(force.ensure((size_t)std::max<int64_t>(n, 1)));
    if ((rc0 = row_bounds(h, d_lo, d_hi, d_val, accumulate ? h->d_row_mass : nullptr, kSplit, bound.as<uint64_t>(),
                          force.as<uint8_t>())))
      return rc0;
    // A fresh build with implicit (unit) increments: a row needs a slot when
    // it is split (more than kSplit keys: at most npairs / (kSplit + 1) rows)
    // or its mass reaches 2^16 (at most total / 2^16 rows; with
    // 2^(16 - s) > kSplit keys such a row is split anyway) -- a bound the host
    // knows without reading anything back.  Reserving costs slot memory, so
    // only a bound worth at most 2 GB of slots takes this path; a larger job
    // reads the count back.
    int64_t max_new = -1;
    if (!accumulate && !d_val && h->hp.frac_bits < 16) {
      const int64_t split = npairs / (kSplit + 1) + 1;
      const int64_t heavy = (int64_t)(((uint64_t)npairs << h->hp.frac_bits) / kNarrowLimit);
      const int64_t slots = (int64_t(1) << (16 - h->hp.frac_bits)) > kSplit ? split : split + heavy;
      if ((double)slots * (double)h->dw * 4.0 <= 2.0e9) max_new = slots;
    }
    // a fresh build's single-slice owners store their slot rows whole
    // (k_build_slices): their slots are not zeroed first
    const uint64_t whole_bound = whole_slices ? (uint64_t)kSliceKeys << h->hp.frac_bits : 0;
    if ((rc0 = promote_rows(h, bound.as<uint64_t>(), force.as<uint8_t>(), accumulate != 0, max_new, whole_bound)))
      return rc0;
    // accumulating: every touched u8 / nibble row becomes u16 first (the build
    // adds into u16 or u32 rows); untouched rows are skipped by the build when
    // their norms are current, otherwise every form row is widened
    if (accumulate &&
        (rc0 = widen_rows(h, h->norms_valid ? bound.as<uint64_t>() : nullptr, h->d_row_mass, true, d_lo, d_hi)))
      return rc0;
  }
  {
    TimedScope ts(h, "build_plan");
    unsigned grid = (unsigned)std::max<int64_t>(1, std::min<int64_t>((n + 255) / 256, 4096));
    hipLaunchKernelGGL(k_build_plan, dim3(grid), dim3(256), 0, h->stream, d_lo, d_hi, n, kSplit, kSliceKeys,
                       fast_slices ? 0 : 1, row_hot, hot, extra_map, counters, h->d_norm, h->d_rowmax, h->p.depth,
                       eflag);
    CMS_HIP(hipGetLastError());
  }
  // fresh builds may store byte forms: the whole [d][w] byte image in LDS
  const int forms = h->forms_ok && !accumulate && (size_t)h->dw <= kFormLdsMax ? 1 : 0;
  if (h->compact && !accumulate) {
    // the compact layout: capacities by class, their scan, the arena sized
    // (the one read-back of the build; beside the last scatter when the
    // plan runs on the side stream)
    TimedScope ts(h, "build_plan");
    CMS_HIP(h->ws_layout.ensure(sizeof(uint32_t) * (size_t)(2 * n + n / 4096 + 16)));
    uint32_t* caps = h->ws_layout.as<uint32_t>();
    const unsigned grid = (unsigned)std::max<int64_t>(1, std::min<int64_t>((n + 255) / 256, 4096));
    hipLaunchKernelGGL(k_row_caps, dim3(grid), dim3(256), 0, h->stream, d_lo, d_hi, n, h->ws_bound.as<uint64_t>(),
                       h->d_hidx, forms, d_val ? 1 : 0, h->hp.frac_bits, h->p.depth, h->p.width, h->tune.bit_keys,
                       h->tune.crumb_keys, lists_allowed(h) ? h->tune.list_keys : 0, caps);
    CMS_HIP(hipGetLastError());
    if ((rc0 = row_layout(h, caps, caps + n))) return rc0;
  }
  plan_side.end();
  const int skip_untouched = accumulate && h->norms_valid ? 1 : 0;
  const size_t lds = sizeof(uint32_t) * (size_t)((h->p.width + 3) & ~3);
  // k_build_rows: with fast slices it builds only the unsplit slot rows
  const int64_t row_emax = fast_slices ? 0 : emax;
  const int slices_done = fast_slices ? 1 : 0;
  bool hot_norms_done = false;
  // slice images summed by k_slice_reduce instead of global slot atomics
  // (Tunables::slice_reduce): emax images of d*w u16 counters
  const bool sreduce = fast_slices && h->tune.slice_reduce && (h->p.width % 8) == 0;
  uint16_t* simg = nullptr;
  if (sreduce) {
    CMS_HIP(h->ws_slicepart.ensure(sizeof(uint16_t) * (size_t)emax * (size_t)h->dw));
    simg = h->ws_slicepart.as<uint16_t>();
  }
  auto launch_hot_norms = [&]() -> int {
    TimedScope ts(h, "hot_norms");
    dim3 grid((unsigned)std::max<int64_t>(1, std::min<int64_t>(max_hot, 1024)), (unsigned)h->p.depth);
    hipLaunchKernelGGL(k_hot_norms, grid, dim3(256), 0, h->stream, hot, counters, h->hp, h->tview(), h->d_norm,
                       h->d_rowmax, sreduce ? kRedGroup : whole_slices);
    CMS_HIP(hipGetLastError());
    hot_norms_done = true;
    return CMS_OK;
  };
  {
    TimedScope ts(h, "build_rows");
    auto kern = k_build_rows<kBuildStoreForm>;
    // the split owners' slices, on the handle's stream (after the side stream
    // forks, so they overlap the byte and mid classes)
    auto launch_slices = [&]() -> int {
      if (!fast_slices) return CMS_OK;
#ifdef CMS_BUILD_SKIP_SLICES  // bound analysis only: the split owners' slices not built (wrong table)
      return CMS_OK;
#endif
      auto kslices = slices_kernel();
      hipLaunchKernelGGL(kslices, dim3((unsigned)emax), dim3(kSliceThreads), img_lds, h->stream, d_lo, d_hi,
                         keys, h->hp, kSliceKeys, hot, extra_map, counters, h->tview(), h->d_row_mass, h->d_flags,
                         simg, whole_slices, h->d_norm, h->d_rowmax);
      CMS_HIP(hipGetLastError());
      if (sreduce) {
        TimedScope ts(h, "slice_reduce");
        hipLaunchKernelGGL(k_slice_reduce, dim3((unsigned)((int64_t)h->num_cus * 8)), dim3(256), 0, h->stream, hot,
                           extra_map, counters, simg, h->hp, h->tview(), accumulate, h->d_norm, h->d_rowmax);
        CMS_HIP(hipGetLastError());
      }
      return CMS_OK;
    };
    if (forms) {
      // owner classes: slot rows -> k_build_slices / k_build_rows (the
      // handle's stream), byte rows -> k_build_nibbles (+ k_build_bytes for
      // the ones a counter >= 16 sends back) and mid rows -> k_build_mid on the
      // side stream, so the classes' kernels overlap (their tails no longer
      // leave CUs idle)
      CMS_HIP(h->ws_blist.ensure(sizeof(int32_t) * (size_t)(3 * n + 4)));
      int32_t* slot_list = h->ws_blist.as<int32_t>();
      int32_t* mid_list = slot_list + n;
      uint32_t* lcnt = reinterpret_cast<uint32_t*>(mid_list + n);  // [0] slot rows, [1] mid rows, [2] mid redo
      int32_t* mid_redo = mid_list + n + 4;                         // k_build_mid_waves -> k_build_mid (u16)
      CMS_HIP(h->ws_plist.ensure(sizeof(int32_t) * (size_t)(n + 1)));
      int32_t* redo = h->ws_plist.as<int32_t>();
      uint32_t* redo_cnt = reinterpret_cast<uint32_t*>(redo + n);
      CMS_HIP(hipMemsetAsync(lcnt, 0, 3 * sizeof(uint32_t), h->stream));
      CMS_HIP(hipMemsetAsync(redo_cnt, 0, sizeof(uint32_t), h->stream));
      hipLaunchKernelGGL(k_build_classes,
                         dim3((unsigned)std::max<int64_t>(1, std::min<int64_t>((n + kClassChunk - 1) / kClassChunk, 1024))),
                         dim3(256), 0, h->stream, d_lo, d_hi, n, h->d_hidx, h->ws_bound.as<uint64_t>(), slot_list,
                         mid_list, lcnt, eflag);
      CMS_HIP(hipGetLastError());
      if (h->plan_side_active) return set_error(CMS_E_STATE, "internal: side stream used while swapped for the plan");
      hipStream_t side = h->side_stream ? h->side_stream : h->stream;
#ifdef CMS_BUILD_SERIAL  // bound analysis only: the classes' kernels one after another (isolated durations)
      side = h->stream;
#endif
      // once the side stream has forked, every exit (error returns included)
      // joins it back: the caller's next work on h->stream may reuse or free
      // the buffers the side kernels are still writing
      // the mid class on a third stream (Tunables::build_streams == 3)
      const hipStream_t side2 = side != h->stream && h->tune.build_streams >= 3 ? h->side_stream2 : side;
      struct SideJoin {
        cms_handle* h;
        hipStream_t side, side2;
        bool armed = false;
        ~SideJoin() {
          if (armed && hipEventRecord(h->ev_join2, side) == hipSuccess)
            (void)hipStreamWaitEvent(h->stream, h->ev_join2, 0);
          if (armed && side2 != side && hipEventRecord(h->ev_join3, side2) == hipSuccess)
            (void)hipStreamWaitEvent(h->stream, h->ev_join3, 0);
        }
      } join{h, side, side2};
      if (side != h->stream) {
        CMS_HIP(hipEventRecord(h->ev_fork2, h->stream));
        CMS_HIP(hipStreamWaitEvent(side, h->ev_fork2, 0));
        if (side2 != side) CMS_HIP(hipStreamWaitEvent(side2, h->ev_fork2, 0));
        join.armed = true;
      }
      const int64_t nib_blocks = (n + kNibWaves - 1) / kNibWaves;
      auto knib = h->tune.nib_rows_once && h->p.depth == 5   ? k_build_nibbles<kBuildStoreForm, 5>
                  : h->tune.nib_rows_once && h->p.depth == 4 ? k_build_nibbles<kBuildStoreForm, 4>
                                                             : k_build_nibbles<kBuildStoreForm, 0>;
      hipLaunchKernelGGL(knib,
                         dim3((unsigned)(h->tune.nib_persist ? std::min<int64_t>(nib_blocks, (int64_t)h->num_cus * 8)
                                                             : nib_blocks)),
                         dim3(64 * kNibWaves), (size_t)kNibWaves * (size_t)h->p.width / 2, side, d_lo, d_hi, keys,
                         d_val, n, h->hp, row_hot, h->ws_bound.as<uint64_t>(), h->tview(), h->d_hidx, h->d_cbound,
                         h->d_row_mass, h->d_norm, h->d_rowmax, h->d_flags, redo, redo_cnt, h->tune.bit_keys,
                         h->tune.crumb_keys, lists_allowed(h) ? h->tune.list_keys : 0);
      // the u8 all-rows image (Tunables::mid_u8_image) when a [d][w] byte image fits 64 KB (config 3: 40 KB)
      const int u8img = h->tune.mid_u8_image && h->dw <= 64 * 1024 ? 1 : 0;
      const size_t mid_lds = std::max<size_t>((size_t)h->p.width * 2, u8img ? (size_t)h->dw : (size_t)h->dw / 2);
      const bool mid128 = h->tune.mid_threads == 128;
      auto kmid = h->p.depth == 5   ? (mid128 ? k_build_mid<kBuildStoreForm, 5, 128> : k_build_mid<kBuildStoreForm, 5, 256>)
                  : h->p.depth == 4 ? (mid128 ? k_build_mid<kBuildStoreForm, 4, 128> : k_build_mid<kBuildStoreForm, 4, 256>)
                                    : (mid128 ? k_build_mid<kBuildStoreForm, 0, 128> : k_build_mid<kBuildStoreForm, 0, 256>);
      const int mid_nt = mid128 ? 128 : 256;
      // the one-pass image build when the [d][w] u16 image fits 80 KB and the
      // row width packs into whole 4-bit words (Tunables::mid_image)
      const bool img = h->tune.mid_image && h->dw * 2 <= 80 * 1024 && (h->dw % 32) == 0;
      if (img) {
        static bool attr = [] {
          for (const void* f : {(const void*)k_build_image<kBuildStoreForm, 0>, (const void*)k_build_image<kBuildStoreForm, 4>,
                                (const void*)k_build_image<kBuildStoreForm, 5>})
            (void)hipFuncSetAttribute(f, hipFuncAttributeMaxDynamicSharedMemorySize, 80 * 1024);
          return true;
        }();
        (void)attr;
        auto kimg = h->p.depth == 5   ? k_build_image<kBuildStoreForm, 5>
                    : h->p.depth == 4 ? k_build_image<kBuildStoreForm, 4>
                                      : k_build_image<kBuildStoreForm, 0>;
        hipLaunchKernelGGL(kimg, dim3((unsigned)std::min<int64_t>(n, (int64_t)h->num_cus * 2)), dim3(kImgThreads),
                           (size_t)h->dw * 2, side, d_lo, d_hi, keys, d_val, h->hp, (const int32_t*)mid_list,
                           (const uint32_t*)(lcnt + 1), h->tview(), h->d_hidx, h->d_cbound, h->d_row_mass, h->d_norm,
                           h->d_rowmax, h->d_flags, lists_allowed(h) ? kMidListKeys : 0);
      } else if (h->tune.mid_waves && !d_val && h->hp.frac_bits == 0 && h->hp.fastq && (h->p.width % 32) == 0 &&
                 (size_t)h->p.width * 4 <= 64 * 1024) {
        // one wave per mid owner (4-bit / u8 rows), then k_build_mid for the
        // owners that need u16 rows
        auto kmw = h->p.depth == 5   ? k_build_mid_waves<kBuildStoreForm, 5>
                   : h->p.depth == 4 ? k_build_mid_waves<kBuildStoreForm, 4>
                                     : k_build_mid_waves<kBuildStoreForm, 0>;
        hipLaunchKernelGGL(kmw, dim3((unsigned)std::min<int64_t>((n + 3) / 4, (int64_t)h->num_cus * h->tune.mid_waves)),
                           dim3(256), (size_t)h->p.width * 4, side2, d_lo, d_hi, keys, h->hp, (const int32_t*)mid_list,
                           (const uint32_t*)(lcnt + 1), h->tview(), h->d_hidx, h->d_cbound, h->d_row_mass, h->d_norm,
                           h->d_rowmax, lists_allowed(h) ? kMidListKeys : 0, h->tune.mid_u4_keys,
                           h->tune.mid_u8_keys, mid_redo, lcnt + 2);
        hipLaunchKernelGGL(kmid, dim3((unsigned)std::min<int64_t>(n, (int64_t)h->num_cus * 2)), dim3(mid_nt),
                           mid_lds, side2, d_lo, d_hi, keys, d_val, h->hp, (const int32_t*)mid_redo,
                           (const uint32_t*)(lcnt + 2), h->tview(), h->d_hidx, h->d_cbound, h->d_row_mass, h->d_norm,
                           h->d_rowmax, h->d_flags, lists_allowed(h) ? kMidListKeys : 0, 0, 0, 0);
      } else
      hipLaunchKernelGGL(kmid, dim3((unsigned)std::min<int64_t>(n, (int64_t)h->num_cus * CMS_MID_GRID_PER_CU *
                                                                 (mid128 ? 2 : 1))),
                         dim3(mid_nt), mid_lds, side2, d_lo, d_hi, keys, d_val, h->hp, (const int32_t*)mid_list,
                         (const uint32_t*)(lcnt + 1), h->tview(), h->d_hidx, h->d_cbound, h->d_row_mass, h->d_norm,
                         h->d_rowmax, h->d_flags, lists_allowed(h) ? kMidListKeys : 0, h->tune.mid_u4_keys,
                         h->tune.mid_u8_keys, u8img);
      hipLaunchKernelGGL(k_build_bytes<kBuildStoreForm>, dim3((unsigned)std::min<int64_t>(n, (int64_t)h->num_cus * 2)),
                         dim3(kBuildThreads), (size_t)h->dw, side, d_lo, d_hi, keys, d_val, h->hp, redo, redo_cnt,
                         h->tview(), h->d_hidx, h->d_cbound, h->d_row_mass, h->d_norm, h->d_rowmax, h->d_flags);
      CMS_HIP(hipGetLastError());
      if ((rc0 = launch_slices())) return rc0;
      // slot rows: at most the slots in use (host-known), plus the mapped slices
      const int64_t nslot = std::min<int64_t>(n, h->hot_used);
      hipLaunchKernelGGL(kern, dim3((unsigned)(row_emax + nslot)), dim3(kBuildThreads), lds, h->stream, d_lo, d_hi,
                         keys, d_val, n, h->hp, kSliceKeys, row_hot, hot, extra_map, counters, row_emax, h->tview(),
                         h->d_row_mass, h->d_norm, h->d_rowmax, h->d_flags, accumulate, slices_done,
                         h->ws_bound.as<uint64_t>(), forms, skip_untouched, h->d_hidx, h->d_cbound,
                         (const int32_t*)slot_list, (const uint32_t*)lcnt);
      CMS_HIP(hipGetLastError());
      // (k_hot_norms here, overlapping the side streams' tail, measured no
      // faster: it competes with them for the CUs)
      if (join.armed) {
        join.armed = false;
        CMS_HIP(hipEventRecord(h->ev_join2, side));
        CMS_HIP(hipStreamWaitEvent(h->stream, h->ev_join2, 0));
        if (side2 != side) {
          CMS_HIP(hipEventRecord(h->ev_join3, side2));
          CMS_HIP(hipStreamWaitEvent(h->stream, h->ev_join3, 0));
        }
      }
    } else {
      if ((rc0 = launch_slices())) return rc0;
      hipLaunchKernelGGL(kern, dim3((unsigned)(row_emax + n)), dim3(kBuildThreads), lds, h->stream, d_lo, d_hi, keys,
                         d_val, n, h->hp, kSliceKeys, row_hot, hot, extra_map, counters, row_emax, h->tview(),
                         h->d_row_mass, h->d_norm, h->d_rowmax, h->d_flags, accumulate, slices_done,
                         h->ws_bound.as<uint64_t>(), forms, skip_untouched, h->d_hidx, h->d_cbound,
                         (const int32_t*)nullptr, (const uint32_t*)nullptr);
      CMS_HIP(hipGetLastError());
    }
  }
  if (!hot_norms_done && (rc0 = launch_hot_norms())) return rc0;
  early_join.end();  // the early rows' build joins the handle's stream
  h->empty = false;
  h->norms_valid = true;  // build_rows + hot_norms wrote the norm of every row
  return CMS_OK;
}

}  // namespace cms
