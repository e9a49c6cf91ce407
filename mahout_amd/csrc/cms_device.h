// cms_device.h -- wave64 / workgroup helpers shared by the gfx950 kernels.
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

#include "cms_hash.h"

namespace cms {

// Increment of pair i in counter units: 1 << fb for implicit streams, else the
// float preference scaled by 2^fb (the handle's frac_bits), which u32 counters
// accept only as a non-negative integer < 2^32.  Scaling by a power of two is
// exact, and every fp64 quantity the reference derives from such counters
// (sums of products, sqrt, products, quotients) scales exactly with it, so the
// similarities are the reference's bit for bit and point queries are the
// counter times 2^-fb.
__device__ __forceinline__ bool load_inc(const float* val, int64_t i, uint32_t& inc, int fb) {
  if (val == nullptr) {
    inc = 1u << fb;
    return true;
  }
  float v = ldexpf(val[i], fb);
  if (!(v >= 0.0f) || v != floorf(v) || v >= 4294967296.0f) {
    inc = 0u;
    return false;
  }
  inc = (uint32_t)v;
  return true;
}

// Keys of a grouped batch.  CSR ingests hand the build the caller's int64
// keys; the COO partition (cms_partition.hip) writes each key as a u32 TOKEN
// instead, halving the bytes the partition moves and the build reads: a key in
// [0, 2^31) is its own token, any other key travels as kTokEscape | i, its
// index in the batch's key array (batches are < 2^31 pairs), and is read from
// there.  at(i) is key i reduced mod p (the hash's input).
constexpr uint32_t kTokEscape = 0x80000000u;
__device__ __forceinline__ uint32_t make_token(int64_t key, int64_t idx) {
  return (uint64_t)key < (uint64_t)kTokEscape ? (uint32_t)key : (kTokEscape | (uint32_t)idx);
}
struct Keys {
  const int64_t* key;   // CSR keys (tok == null), or the batch's keys (escaped tokens index them)
  const uint32_t* tok;  // partition output tokens, or null
  __device__ __forceinline__ uint64_t at(int64_t i) const { return resolve(raw(i)); }
  // at(i) in two steps, so a loop can keep the next keys' loads in flight:
  // raw(i) is the one load (the token, or the key itself), resolve() the rest
  __device__ __forceinline__ uint64_t raw(int64_t i) const { return tok ? (uint64_t)tok[i] : (uint64_t)key[i]; }
  __device__ __forceinline__ uint64_t resolve(uint64_t r) const {
    if (tok) return r < kTokEscape ? r : reduce_key(key[r & (kTokEscape - 1u)]);
    return reduce_key((int64_t)r);
  }
};

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

__device__ __forceinline__ uint32_t wave_sum_u32(uint32_t v) {
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) v += __shfl_xor(v, o, 64);
  return v;
}

// Exclusive scan across the block; scratch needs (blockDim/64 + 1) words.
__device__ __forceinline__ uint32_t block_excl_scan_u32(uint32_t v, uint32_t* scratch, uint32_t* total) {
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
__device__ __forceinline__ uint64_t block_sum_u64_sat(uint64_t v, uint64_t* scratch) {
  const int lane = threadIdx.x & 63, wid = threadIdx.x >> 6, nw = blockDim.x >> 6;
  v = wave_sum_u64_sat(v);
  if (lane == 0) scratch[wid] = v;
  __syncthreads();
  uint64_t s = 0;
  for (int i = 0; i < nw; ++i) s = sat_add(s, scratch[i]);
  __syncthreads();
  return s;
}

// Math.min(a, b) for doubles (NaN wins; -0.0 < +0.0).
__device__ __forceinline__ double java_min(double a, double b) {
  if (a != a) return a;
  if (a == 0.0 && b == 0.0 && signbit(b)) return b;
  return (a <= b) ? a : b;
}

// normalizeWeightResult(result, count=1, num=0) (AbstractSimilarity.java:313-330):
// WEIGHTED scales by 1 - count/(num+1) = 0, i.e. +-1; then the clamp to [-1, 1].
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

// Workgroup barrier that orders LDS only: global loads and stores issued
// before it stay in flight (__syncthreads would drain them with its vmcnt(0)).
__device__ __forceinline__ void lds_barrier() {
  asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
  __builtin_amdgcn_s_barrier();
  asm volatile("" ::: "memory");
}

}  // namespace cms
