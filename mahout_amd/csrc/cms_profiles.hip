// cms_profiles.hip -- CosineCM with per-owner sketch shapes on gfx950.
//
// The reference sizes every owner's sketch on its own.  CountMinSketchConfig
// (T/impl/common/CountMinSketchConfig.java:120-158) picks (d, w) per owner by
// maximising Fmeasure (:210-219) and stores delta = exp(-d), epsilon = e/w;
// CosineCM.userSimilarity(u1, u2) (T/impl/similarity/CosineCM.java:83-96)
// then builds u1's sketch with u2's (delta, epsilon) (exportProfile :41-58),
// takes u2's own sketch from its cache (getExportedCMProfile :60-67) and
// returns the min-over-rows cosine (DoubleCountMinSketch.java:114-149).
//
// Here the DataModel stays resident in HBM as CSR (keys reduced mod p once,
// u32 increments).  Own sketches are built once at finalize into one ragged
// u32 array with exact u64 row norms.  A similarity never materialises u1's
// sketch in HBM: one wave per (u1, u2) pair hashes u1's preferences at u2's
// shape into an LDS bucket row (global scratch past kPoHist), and per sketch
// row forms
//   valueAB = sum_k v_k * B[h(k)]   (exact: u64, every term an integer)
//   valueA  = sum_j A[j]^2          (the LDS row; exact while < 2^53)
// -- the integers the reference's fp64 loops produce bit for bit while the
// sums stay below 2^53; past that the wave replays the reference's
// sequential fp64 loop in j order.  The epilogue is the same correctly
// rounded sqrt / mul / div and Math.min as the fixed-shape kernels.
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cfloat>
#include <cmath>
#include <vector>

#include "cms_device.h"
#include "cms_internal.h"

namespace cms {

constexpr int kPoThreads = 64;     // one wave per (u1, u2) pair
constexpr int kPoBigThreadsPair = 256;  // listed pairs of a big u1: four waves per pair
#ifndef CMS_PO_BIGROW
#define CMS_PO_BIGROW 16384
#endif
constexpr int kPoBigRow = CMS_PO_BIGROW;  // their LDS bucket row (64 KiB)
constexpr int kPoHist = 4096;      // LDS bucket row (u32); wider shapes use global scratch
constexpr int kPoGrid = 8192;      // pair-kernel blocks with LDS rows
constexpr int kPoGridWide = 1024;  // pair-kernel blocks when some width exceeds kPoHist
constexpr int kPoGridList = 32768; // pair-kernel blocks for a listed batch that needs no global rows
constexpr int kCfgThreads = 256;

// ------------------------------------------------ CountMinSketchConfig --

// Fmeasure(w, d, n, u, q) (:210-219) with probaNotExactRetrieve (:190-196)
// and probaInserted (:170-178) written out as the reference evaluates them.
__device__ __forceinline__ double po_fmeasure(int w, int d, int n, int u, double q2) {
  const double W = (double)w, D = (double)d, N = (double)n, U = (double)u;
  const double falseP = pow(1.0 - pow(1.0 - 1.0 / W, N), D);
  const double beta = 1.0 - falseP;
  const double p = 1.0 - N / (N + falseP * (U - N));
  if (beta == 0.0 || p == 0.0) return 0.0;
  return 3.0 * beta * p / (q2 * beta + p);
}

// computeConfig (:120-158), one workgroup per owner: every (d, w) with d in
// [1, 25) and w in [d, n] is scored; the loop keeps the LAST position whose
// score is >= the running best (which starts at 0), i.e. the last maximiser
// among scores >= 0 -- reduced here as max over (score, position).
__global__ __launch_bounds__(kCfgThreads) void k_po_config(const int64_t* off, int64_t n_owners, int32_t u,
                                                           double q2, int32_t* best_w, int32_t* best_d) {
  __shared__ double sf[kCfgThreads / 64];
  __shared__ uint64_t si[kCfgThreads / 64];
  for (int64_t r = blockIdx.x; r < n_owners; r += gridDim.x) {
    const int64_t len = off[r + 1] - off[r];
    const int nn = (int)std::min<int64_t>(len, 0x7fffffff);
    double bf = -1.0;  // no candidate yet
    uint64_t bi = 0;
    for (int d = 1; d < 25; ++d)
      for (int w = d + (int)threadIdx.x; w <= nn; w += kCfgThreads) {
        const double x = po_fmeasure(w, d, nn, u, q2);
        const uint64_t idx = ((uint64_t)d << 32) | (uint32_t)w;
        if (x >= 0.0 && (x > bf || (x == bf && idx > bi))) {
          bf = x;
          bi = idx;
        }
      }
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) {
      const double of = __shfl_xor(bf, o, 64);
      const uint64_t oi = __shfl_xor(bi, o, 64);
      if (of > bf || (of == bf && oi > bi)) {
        bf = of;
        bi = oi;
      }
    }
    if ((threadIdx.x & 63) == 0) {
      sf[threadIdx.x >> 6] = bf;
      si[threadIdx.x >> 6] = bi;
    }
    __syncthreads();
    if (threadIdx.x == 0) {
      for (int i = 1; i < kCfgThreads / 64; ++i)
        if (sf[i] > bf || (sf[i] == bf && si[i] > bi)) {
          bf = sf[i];
          bi = si[i];
        }
      best_w[r] = bf < 0.0 ? 0 : (int32_t)(uint32_t)bi;
      best_d[r] = bf < 0.0 ? 0 : (int32_t)(bi >> 32);
    }
    __syncthreads();
  }
}

// ------------------------------------------------------------ DataModel --

__global__ void k_po_prep(const int64_t* key, const float* val, int64_t np, int fb, uint64_t* kp, uint32_t* inc,
                          uint32_t* flags) {
  for (int64_t i = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; i < np; i += (int64_t)gridDim.x * blockDim.x) {
    kp[i] = reduce_key(key[i]);
    uint32_t v;
    if (!load_inc(val, i, v, fb)) atomicOr(flags, kFlagBadValue);
    inc[i] = v;
  }
}

// An owner's total mass bounds every counter of its sketch at any shape.
__global__ __launch_bounds__(256) void k_po_mass(const int64_t* off, int64_t n, const uint32_t* inc,
                                                 uint32_t* flags) {
  __shared__ uint64_t red[4];
  for (int64_t r = blockIdx.x; r < n; r += gridDim.x) {
    uint64_t s = 0;
    for (int64_t i = off[r] + threadIdx.x; i < off[r + 1]; i += 256) s += inc[i];
    s = block_sum_u64_sat(s, red);
    if (threadIdx.x == 0 && s >= (1ULL << 32)) atomicOr(flags, kFlagOverflow);
  }
}

// ----------------------------------------------------------- own sketches --

// getExportedCMProfile(u) for every owner: update(key, inc) at the owner's own
// shape (DoubleCountMinSketch.update :72-80), exact u32 global atomics.
__global__ __launch_bounds__(256) void k_po_build(const int64_t* off, const uint64_t* kp, const uint32_t* inc,
                                                  const PoShape* shp, HashParams hp, int64_t n, uint32_t* sk) {
  for (int64_t r = blockIdx.x; r < n; r += gridDim.x) {
    const PoShape s = shp[r];
    if (s.w <= 0) continue;
    for (int64_t i = off[r] + threadIdx.x; i < off[r + 1]; i += 256) {
      const uint64_t k = kp[i];
      const uint32_t v = inc[i];
      for (int d = 0; d < s.d; ++d)
        atomicAdd(&sk[s.soff + (int64_t)d * s.w + bucket_wbq(hp, d, k, (uint32_t)s.w, s.barrett)], v);
    }
  }
}

// Exact per-(owner, row) sum of squares and Math.sqrt of the reference's
// valueB: the integer sum below 2^53, else the sequential fp64 sum in j order.
__global__ __launch_bounds__(256) void k_po_norms(const PoShape* shp, int64_t n, const uint32_t* sk, uint64_t* norm,
                                                  double* nsq) {
  __shared__ uint64_t red[4];
  for (int64_t r = blockIdx.x; r < n; r += gridDim.x) {
    const PoShape s = shp[r];
    for (int d = 0; d < s.d; ++d) {
      const uint32_t* row = sk + s.soff + (int64_t)d * s.w;
      uint64_t q = 0;
      for (int j = threadIdx.x; j < s.w; j += 256) q = sat_add(q, (uint64_t)row[j] * row[j]);
      q = block_sum_u64_sat(q, red);
      if (threadIdx.x == 0) {
        double v;
        if (q < (1ULL << 53)) {
          v = (double)q;
        } else {
          v = 0.0;
          for (int j = 0; j < s.w; ++j) {
            const double x = (double)row[j];
            v = __dadd_rn(v, __dmul_rn(x, x));
          }
        }
        norm[s.roff + d] = q;
        nsq[s.roff + d] = __dsqrt_rn(v);
      }
    }
  }
}

// ------------------------------------------------------------ similarity --

struct PoPairArgs {
  const int64_t* off;
  const uint64_t* kp;
  const uint32_t* inc;
  const PoShape* shp;
  const uint32_t* sk;
  const uint64_t* norm;
  const double* nsq;
  const int64_t* qrows;  // [nq]
  const int64_t* crows;  // [m] or null (identity)
  int64_t nq, m;
  uint32_t* scratch;     // [gridDim][max_w] zeroed u32 rows (widths > kPoHist)
  int64_t scratch_w;
  double* out;           // [nq][m], or with ldo > 0 a slab [nq][ldo] at column u2
  int64_t ldo;
  int32_t weighted;
  // list mode: the pairs (u1 << 32) | u2 of plist[0, nq) into slab row u1 - q0
  const unsigned long long* plist = nullptr;
  int64_t q0 = 0;
  uint32_t* no_rows = nullptr;  // pairs that needed a global bucket row without scratch (a host error)
};

__device__ __forceinline__ uint64_t po_wave_sum(uint64_t v) {
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) v = sat_add(v, __shfl_xor(v, o, 64));
  return v;
}

// Open-addressed LDS table of at most 256 distinct buckets: keys (bucket + 1)
// at lds[0, kPoTab), counts at lds[kPoTab, 2 kPoTab); the slot of bucket j.
constexpr int kPoTab = 512;
__device__ __forceinline__ uint32_t po_tab_insert(uint32_t* lds, uint32_t j) {
  uint32_t slot = (j * 2654435761u) >> 23;  // 9 bits
  for (;;) {
    const uint32_t prev = atomicCAS(&lds[slot], 0u, j + 1u);
    if (prev == 0u || prev == j + 1u) return slot;
    slot = (slot + 1u) & (kPoTab - 1);
  }
}

// Sum over the NT threads of a block (every thread gets it).
template <int NT>
__device__ __forceinline__ uint64_t po_block_sum(uint64_t v, unsigned long long* red) {
  v = po_wave_sum(v);
  if (NT == 64) return v;
  if ((threadIdx.x & 63) == 0) red[threadIdx.x >> 6] = v;
  __syncthreads();
  uint64_t t = 0;
#pragma unroll
  for (int i = 0; i < NT / 64; ++i) t = sat_add(t, red[i]);
  __syncthreads();
  return t;
}

// userSimilarity(u1 = qrows[t / m], u2 = crows[t % m]): one block of NT
// threads per pair (one wave; four for listed pairs whose u1 has more than
// kPoBigQuery preferences).
template <int NT>
__global__ __launch_bounds__(NT) void k_po_pairs(PoPairArgs a, HashParams hp) {
  constexpr int kPoThreads = NT;  // (the body's stride)
  // the four-wave blocks (a big u1) keep rows of up to kPoBigRow counters in
  // LDS and take valueAB / valueA from one sweep over the row instead of a
  // second hashing pass (u1's buckets outnumber or rival the row's width)
  constexpr int kRow = NT > 64 ? kPoBigRow : kPoHist;
  __shared__ uint32_t lds[kRow];
  __shared__ unsigned long long red[NT / 64];
  const int lane = threadIdx.x;
  for (int j = lane; j < kRow; j += kPoThreads) lds[j] = 0u;
  __syncthreads();
  uint32_t* gsc = a.scratch ? a.scratch + (int64_t)blockIdx.x * a.scratch_w : nullptr;
  const int64_t total = a.plist ? a.nq : a.nq * a.m;
  for (int64_t t = blockIdx.x; t < total; t += gridDim.x) {
    int64_t u1, u2;
    if (a.plist) {
      const unsigned long long e = a.plist[t];
      u1 = (int64_t)(e >> 32);
      u2 = (int64_t)(e & 0xFFFFFFFFu);
    } else {
      u1 = a.qrows[t / a.m];
      const int64_t c = t % a.m;
      u2 = a.crows ? a.crows[c] : c;
    }
    const PoShape s = a.shp[u2];
    const uint32_t w = (uint32_t)s.w;
    uint32_t* hist = (w <= (uint32_t)kRow) ? lds : gsc;
    const bool sweep = NT > 64 && w <= (uint32_t)kRow;
    const int64_t k0 = a.off[u1], k1 = a.off[u1 + 1];
    double minc = DBL_MAX;
    // u1's counters at u2's shape: pass 1 adds every preference into the
    // bucket row; pass 2 takes each bucket back to zero with an exchange, so the
    // first key of a bucket collects its whole count c (c^2 into valueA) and
    // the row is clean for the next pair -- O(#preferences), not O(w)
    auto add_pass = [&](int d, uint64_t* ab, const uint32_t* brow) {
      for (int64_t i = k0 + lane; i < k1; i += kPoThreads) {
        const uint32_t j = bucket_wbq(hp, d, a.kp[i], w, s.barrett);
        const uint32_t v = a.inc[i];
        atomicAdd(&hist[j], v);
        if (ab) *ab = sat_add(*ab, (uint64_t)v * brow[j]);
      }
      __syncthreads();
    };
    auto clear_pass = [&](int d) {
      uint64_t a2 = 0;
      for (int64_t i = k0 + lane; i < k1; i += kPoThreads) {
        const uint32_t c = atomicExch(&hist[bucket_wbq(hp, d, a.kp[i], w, s.barrett)], 0u);
        a2 = sat_add(a2, (uint64_t)c * c);
      }
      __syncthreads();
      return a2;
    };
    // u1 with at most 4 preferences per lane: keys, increments and each
    // row's buckets stay in registers (one load per pair, one hash per key
    // and row; the exchange pass reuses the buckets)
    const bool cached = NT == 64 && k1 - k0 <= 4 * kPoThreads;
    // a cached u1 against a width past the LDS row: its (at most 256) buckets
    // go into an LDS hash table instead of a global bucket row
    const bool tab = cached && w > (uint32_t)kPoHist;
    if (hist == nullptr && !tab) {  // (uniform) a launch without scratch got a pair that needs it
      if (lane == 0) atomicAdd(a.no_rows, 1u);
      continue;
    }
    uint64_t ck[4];
    uint32_t cv[4], cj[4];
    if (cached) {
#pragma unroll
      for (int u = 0; u < 4; ++u) {
        const int64_t i = k0 + lane + (int64_t)u * kPoThreads;
        ck[u] = i < k1 ? a.kp[i] : 0ULL;
        cv[u] = i < k1 ? a.inc[i] : 0u;
      }
    }
    for (int d = 0; d < s.d; ++d) {
      const uint32_t* brow = a.sk + s.soff + (int64_t)d * w;
      uint64_t ab = 0;
      uint64_t a2p = 0;
      if (cached) {
        uint32_t bv[4], sl[4];
#pragma unroll
        for (int u = 0; u < 4; ++u) {
          cj[u] = cv[u] ? bucket_wbq(hp, d, ck[u], w, s.barrett) : 0u;
          bv[u] = cv[u] ? brow[cj[u]] : 0u;  // the gathers of all four keys in flight together
        }
#pragma unroll
        for (int u = 0; u < 4; ++u)
          if (cv[u]) {
            if (tab) {
              sl[u] = po_tab_insert(lds, cj[u]);
              atomicAdd(&lds[kPoTab + sl[u]], cv[u]);
            } else {
              atomicAdd(&hist[cj[u]], cv[u]);
            }
          }
#pragma unroll
        for (int u = 0; u < 4; ++u) ab = sat_add(ab, (uint64_t)cv[u] * bv[u]);
        __syncthreads();
#pragma unroll
        for (int u = 0; u < 4; ++u)
          if (cv[u]) {
            const uint32_t c = atomicExch(tab ? &lds[kPoTab + sl[u]] : &hist[cj[u]], 0u);
            a2p = sat_add(a2p, (uint64_t)c * c);
          }
        __syncthreads();
        if (tab) {  // every count is collected: the keys may go
#pragma unroll
          for (int u = 0; u < 4; ++u)
            if (cv[u]) lds[sl[u]] = 0u;
          __syncthreads();
        }
      } else if (sweep) {
        for (int64_t i = k0 + lane; i < k1; i += kPoThreads)
          atomicAdd(&hist[bucket_wbq(hp, d, a.kp[i], w, s.barrett)], a.inc[i]);
        __syncthreads();
        for (uint32_t j = lane; j < w; j += kPoThreads) {
          const uint32_t c = hist[j];
          if (c) {
            ab = sat_add(ab, (uint64_t)c * brow[j]);
            a2p = sat_add(a2p, (uint64_t)c * c);
            hist[j] = 0u;
          }
        }
        __syncthreads();
      } else {
        add_pass(d, &ab, brow);
        a2p = clear_pass(d);
      }
      const uint64_t a2 = po_block_sum<NT>(a2p, red);
      ab = po_block_sum<NT>(ab, red);
      const uint64_t b2 = a.norm[s.roff + d];
      double valueAB, den;
      if (a2 < (1ULL << 53) && b2 < (1ULL << 53)) {
        valueAB = (double)ab;  // ab <= sqrt(a2 * b2) < 2^53: exact
        den = __dmul_rn(__dsqrt_rn((double)a2), a.nsq[s.roff + d]);
      } else {  // the reference's sequential fp64 loop (:128-134) over the rebuilt row, every lane alike
        if (hist == nullptr) {  // (uniform) as above
          if (lane == 0) atomicAdd(a.no_rows, 1u);
          break;
        }
        add_pass(d, nullptr, brow);
        double A = 0.0, B = 0.0, AB = 0.0;
        for (uint32_t j = 0; j < w; ++j) {
          const double xa = (double)hist[j], xb = (double)brow[j];
          A = __dadd_rn(A, __dmul_rn(xa, xa));
          B = __dadd_rn(B, __dmul_rn(xb, xb));
          AB = __dadd_rn(AB, __dmul_rn(xa, xb));
        }
        valueAB = AB;
        den = __dmul_rn(__dsqrt_rn(A), __dsqrt_rn(B));
        __syncthreads();
        (void)clear_pass(d);
      }
      if (den != 0.0) minc = java_min(minc, __ddiv_rn(valueAB, den));
    }
    if (lane == 0) {
      double r = (minc == DBL_MAX) ? __builtin_nan("") : minc;
      if (r == r) r = normalize_weight(r, a.weighted);
      a.out[a.plist ? (u1 - a.q0) * a.ldo + u2 : a.ldo > 0 ? (t / a.m) * a.ldo + u2 : t] = r;
    }
  }
}

// ------------------------------------------- all-pairs slabs by shape class --
// userSimilarity(u1, u2) for a block of query rows against every candidate,
// the candidates grouped by their shape class (w, d): every member of a class
// hashes u1's preferences identically (CosineCM.java:86 builds u1 at u2's
// (delta, epsilon)), so a group of up to 64 members of one class (one lane
// each) shares the hashing, and each wave of a workgroup takes one query at
// a time.  The members' own sketches are read from the class's transposed
// image po_skT ([d w][members]: lane m's counter t at t * cnt + m, so a
// wave's 64 member loads are one contiguous 256-byte read, L2-resident while
// the workgroups of one XCD work through the same group); LDS holds only each
// wave's bucket row.  Per sketch row, u1's preferences are hashed ONCE into
// the wave's bucket row -- u1's sketch row at the class shape -- and then,
// whichever is less work:
//   dense (w <= nnz(u1); CMS_PO_DENSE_X4 / 4 x nnz): lane m forms valueAB = sum_j U1[j] * S_m[j] over
//     the w buckets (U1[j] a broadcast LDS read), valueA from one sweep over
//     the row, which also zeroes it;
//   sparse: 64 preferences at a time are parked as (bucket, increment) and
//     lane m gathers its member's counters at them; the row is cleared by an
//     exchange pass that yields valueA (k_po_pairs' scheme).
// Every sum is an exact integer in fp64 while both norms are below 2^53;
// pairs past that are listed for k_po_pairs' sequential replay.
constexpr int64_t kPoBigQuery = 4096;       // queries past this many preferences: k_po_bigq
constexpr int64_t kPoBigMaxDW = 38 * 1024;  // k_po_bigq: u1's [d][w] u32 image in LDS (152 KiB)
constexpr int kPoGroupMax = 64;            // members per narrow group: one lane each
constexpr int kPoGroupHistW = 2048;        // narrow classes: one LDS bucket row per wave
constexpr int kPoGroupWaves = 8;
constexpr int64_t kPoQueryChunk = 64;      // query rows per workgroup
constexpr int kPoSmallHist = 512;          // narrow groups launched by width: rows of 512, 1024, 2048 counters
constexpr int kPoHistParts = 3;            // (less LDS per workgroup for the narrower ones: more of them per CU)
__host__ __device__ constexpr int po_hist_part(int w) { return w <= kPoSmallHist ? 0 : w <= 2 * kPoSmallHist ? 1 : 2; }

struct PoAllArgs {
  const int64_t* off;
  const uint64_t* kp;
  const uint32_t* inc;
  const PoShape* shp;
  const uint32_t* sk;
  const uint64_t* norm;
  const double* nsq;
  const PoGroup* groups;   // narrow groups: pad = class index
  const PoGroup* classes;  // m0 = the class's first member in cmem
  const int64_t* toff;     // [nclasses] class offsets in skT
  const uint32_t* skT;
  const int64_t* cmem;
  int64_t g0, ngroups, nchunks, per_xcd;  // groups [g0, g0 + ngroups) of this launch
  int32_t hist_w;          // LDS bucket row stride per wave
  int32_t dense_x4;        // dense dots when 4 w <= dense_x4 nnz(u1)
  int64_t q0, qc, n;
  double* slab;  // [qc][n], column = candidate row
  unsigned long long* redo;  // (u1 << 32) | u2 of pairs past the exact regime
  uint32_t* redo_cnt;
  uint32_t redo_cap;
  int32_t weighted;
  int64_t big_skip;  // queries with more preferences than this are k_po_bigq's
};

// LDS of a group workgroup: bucket rows [waves][hist_w] u32, parked
// (bucket, increment) [waves][64] x 2 u32
__host__ __device__ constexpr size_t po_group_lds(int hist_w) {
  return (size_t)kPoGroupWaves * ((size_t)hist_w + 128) * 4;
}

__global__ __launch_bounds__(64 * kPoGroupWaves) void k_po_group_pairs(PoAllArgs a, HashParams hp) {
  extern __shared__ __align__(16) uint32_t lds[];
  // XCD-aware order: workgroups are dealt to the 8 XCDs round-robin, so the
  // (group, query chunk) tiles are numbered per XCD -- each XCD works through
  // consecutive groups, all query chunks of one group back to back, and the
  // group's member image stays in that XCD's L2
  const int64_t c = (int64_t)(blockIdx.x & 7) * a.per_xcd + (blockIdx.x >> 3);
  if (c >= a.ngroups * a.nchunks) return;
  const PoGroup g = a.groups[a.g0 + c / a.nchunks];
  const int64_t chunk = c % a.nchunks;
  const PoGroup cl = a.classes[g.pad];
  const int w = g.w, d = g.d, cnt = g.cnt;
  const int tid = threadIdx.x, lane = tid & 63;
  const int wv = __builtin_amdgcn_readfirstlane(tid >> 6);
  uint32_t* hist = lds + wv * (a.hist_w + 128);  // this wave's bucket row
  uint32_t* pj = hist + a.hist_w;                // parked buckets [64], increments [64]
  uint32_t* pv = pj + 64;
  for (int j = lane; j < w; j += 64) hist[j] = 0u;
  const bool member = lane < cnt;
  const int64_t u2 = member ? a.cmem[g.m0 + lane] : 0;
  const int64_t roff = member ? a.shp[u2].roff : 0;
  const int64_t ccnt = cl.cnt;  // member stride of the class image
  const uint32_t* T = a.skT + a.toff[g.pad] + (g.m0 - cl.m0) + (member ? lane : 0);
  const int64_t qa = chunk * kPoQueryChunk, qb = min(a.qc, qa + kPoQueryChunk);
  for (int64_t q = qa + wv; q < qb; q += kPoGroupWaves) {
    const int64_t u1 = a.q0 + q;
    const int64_t k0 = a.off[u1], k1 = a.off[u1 + 1];
    if (k1 - k0 > a.big_skip && w * d <= kPoBigMaxDW) continue;  // k_po_bigq builds this query once per class
    const bool dense = 4 * (int64_t)w <= a.dense_x4 * (k1 - k0);
    double minc = DBL_MAX;  // lane m < cnt: member m's running Math.min
    bool inexact = false;
    for (int r = 0; r < d; ++r) {
      double acc = 0.0;
      uint64_t a2 = 0;
      const uint32_t* trow = T + (int64_t)r * w * ccnt;
      if (dense) {
        for (int64_t i = k0 + lane; i < k1; i += 64)
          atomicAdd(&hist[bucket_wbq(hp, r, a.kp[i], (uint32_t)w, g.barrett)], a.inc[i]);
        // (a wave's LDS operations execute in order: the row is complete below)
        if (member) {
          int j = 0;
          for (; j + 8 <= w; j += 8) {
            uint32_t t8[8];
#pragma unroll
            for (int u = 0; u < 8; ++u) t8[u] = trow[(int64_t)(j + u) * ccnt];
#pragma unroll
            for (int u = 0; u < 8; ++u) acc = __fma_rn((double)hist[j + u], (double)t8[u], acc);
          }
          for (; j < w; ++j) acc = __fma_rn((double)hist[j], (double)trow[(int64_t)j * ccnt], acc);
        }
        for (int j = lane; j < w; j += 64) {
          const uint32_t cc = hist[j];
          a2 = sat_add(a2, (uint64_t)cc * cc);
          hist[j] = 0u;
        }
      } else {
        for (int64_t base = k0; base < k1; base += 64) {
          const int64_t i = base + lane;
          uint32_t j = 0, v = 0;
          if (i < k1) {
            j = bucket_wbq(hp, r, a.kp[i], (uint32_t)w, g.barrett);
            v = a.inc[i];
            atomicAdd(&hist[j], v);
          }
          pj[lane] = j;
          pv[lane] = v;  // read back below by every lane (in-order LDS)
          const int nt = (int)min<int64_t>(64, k1 - base);
          if (member) {
            int t = 0;
            for (; t + 8 <= nt; t += 8) {
              uint32_t t8[8];
#pragma unroll
              for (int u = 0; u < 8; ++u) t8[u] = trow[(int64_t)pj[t + u] * ccnt];
#pragma unroll
              for (int u = 0; u < 8; ++u) acc = __fma_rn((double)pv[t + u], (double)t8[u], acc);
            }
            for (; t < nt; ++t) acc = __fma_rn((double)pv[t], (double)trow[(int64_t)pj[t] * ccnt], acc);
          }
        }
        asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");  // the wave's adds land before its exchanges
        for (int64_t i = k0 + lane; i < k1; i += 64) {
          const uint32_t cc = atomicExch(&hist[bucket_wbq(hp, r, a.kp[i], (uint32_t)w, g.barrett)], 0u);
          a2 = sat_add(a2, (uint64_t)cc * cc);
        }
      }
      a2 = po_wave_sum(a2);
      if (member) {
        if (a2 < (1ULL << 53) && a.norm[roff + r] < (1ULL << 53)) {
          const double den = __dmul_rn(__dsqrt_rn((double)a2), a.nsq[roff + r]);
          if (den != 0.0) minc = java_min(minc, __ddiv_rn(acc, den));
        } else {
          inexact = true;
        }
      }
    }
    if (member) {
      double res = minc == DBL_MAX ? __builtin_nan("") : minc;
      if (res == res) res = normalize_weight(res, a.weighted);
      if (inexact) {  // k_po_pairs replays the reference's sequential loop
        res = __builtin_nan("");
        const uint32_t slot = atomicAdd(a.redo_cnt, 1u);
        if (slot < a.redo_cap) a.redo[slot] = ((unsigned long long)u1 << 32) | (unsigned long long)u2;
      }
      a.slab[q * a.n + u2] = res;
    }
  }
}

// Queries with many preferences (more than kPoBigQuery): hashing u1 once
// per group of 64 candidates would cost nnz(u1) x d per group -- the bulk of
// the whole job at config 2, where the head items hold millions of
// preferences.  Here u1's sketch at a narrow class's shape is built ONCE per
// class by a whole workgroup in LDS, and every member of the class takes its
// dense dot from the transposed member image po_skT (thread = member, so the
// loads coalesce).  Same exact arithmetic and epilogue as k_po_group_pairs.
constexpr int kPoBigThreads = 256;
struct PoBigArgs {
  const int64_t* off;
  const uint64_t* kp;
  const uint32_t* inc;
  const PoShape* shp;
  const uint64_t* norm;
  const double* nsq;
  const PoGroup* classes;   // m0: first member in cmem, pad: offset of the class in skT (in counters / 64)
  const int64_t* cmem;
  const uint32_t* skT;
  const int64_t* toff;      // [nclasses] offset of each class in skT
  const int64_t* bigq;      // [nbig] slab rows (0-based within the block) of the big queries
  int64_t q0, n;
  double* slab;
  unsigned long long* redo;
  uint32_t* redo_cnt;
  uint32_t redo_cap;
  int32_t weighted;
};

__global__ __launch_bounds__(kPoBigThreads) void k_po_bigq(PoBigArgs a, HashParams hp) {
  extern __shared__ __align__(16) uint32_t lds[];  // u1 at the class shape [d][w] u32
  __shared__ unsigned long long s_a2[CMS_MAX_DEPTH];
  const PoGroup c = a.classes[blockIdx.x];
  const int64_t q = a.bigq[blockIdx.y];
  const int64_t u1 = a.q0 + q;
  const int w = c.w, d = c.d, dw = w * d;
  if (dw > kPoBigMaxDW) return;  // (uniform) the group kernel keeps this class's big queries
  const int tid = threadIdx.x;
  for (int j = tid; j < dw; j += kPoBigThreads) lds[j] = 0u;
  if (tid < CMS_MAX_DEPTH) s_a2[tid] = 0ULL;
  __syncthreads();
  const int64_t k0 = a.off[u1], k1 = a.off[u1 + 1];
  for (int64_t i = k0 + tid; i < k1; i += kPoBigThreads) {
    const uint64_t kp = a.kp[i];
    const uint32_t v = a.inc[i];
    for (int r = 0; r < d; ++r) atomicAdd(&lds[r * w + bucket_wbq(hp, r, kp, (uint32_t)w, c.barrett)], v);
  }
  __syncthreads();
  for (int r = 0; r < d; ++r) {  // valueA of every row
    uint64_t a2 = 0;
    for (int j = tid; j < w; j += kPoBigThreads) {
      const uint32_t x = lds[r * w + j];
      a2 = sat_add(a2, (uint64_t)x * x);
    }
    a2 = po_wave_sum(a2);
    if ((tid & 63) == 0 && a2) atomicAdd(&s_a2[r], (unsigned long long)a2);
  }
  __syncthreads();
  const uint32_t* T = a.skT + a.toff[blockIdx.x];
  // `parts` threads per member (a power of two up to a wave) split each dot
  // over j; classes of 64+ members take one thread per member
  int parts = 1;
  while (parts < 64 && parts * 2 * c.cnt <= kPoBigThreads) parts *= 2;
  const int part = tid & (parts - 1);
  for (int m0 = tid / parts; m0 < ((c.cnt + (kPoBigThreads / parts) - 1) / (kPoBigThreads / parts)) * (kPoBigThreads / parts);
       m0 += kPoBigThreads / parts) {
    const int m = m0;
    const bool live = m < c.cnt;
    const int64_t u2 = live ? a.cmem[c.m0 + m] : 0;
    const PoShape s2 = a.shp[u2];
    double minc = DBL_MAX;
    bool inexact = false;
    for (int r = 0; r < d; ++r) {
      double acc = 0.0;
      if (live) {
        const uint32_t* tr = T + (int64_t)r * w * c.cnt + m;
#pragma unroll 4
        for (int j = part; j < w; j += parts) acc = __fma_rn((double)lds[r * w + j], (double)tr[(int64_t)j * c.cnt], acc);
      }
      for (int o = 1; o < parts; o <<= 1) acc += __shfl_xor(acc, o, 64);  // exact: integers below 2^53
      const uint64_t a2 = s_a2[r];
      if (live && a2 < (1ULL << 53) && a.norm[s2.roff + r] < (1ULL << 53)) {
        const double den = __dmul_rn(__dsqrt_rn((double)a2), a.nsq[s2.roff + r]);
        if (den != 0.0) minc = java_min(minc, __ddiv_rn(acc, den));
      } else {
        inexact = true;
      }
    }
    if (!live || part != 0) continue;
    double res = minc == DBL_MAX ? __builtin_nan("") : minc;
    if (res == res) res = normalize_weight(res, a.weighted);
    if (inexact) {
      res = __builtin_nan("");
      const uint32_t slot = atomicAdd(a.redo_cnt, 1u);
      if (slot < a.redo_cap) a.redo[slot] = ((unsigned long long)u1 << 32) | (unsigned long long)u2;
    }
    a.slab[q * a.n + u2] = res;
  }
}

// po_skT[toff[c] + t * cnt_c + m] = member m's counter t (t < d w), every
// narrow class c; one workgroup per (class, member)
__global__ __launch_bounds__(256) void k_po_transpose(const PoGroup* classes, const int64_t* cmem, const int64_t* toff,
                                                      const PoShape* shp, const uint32_t* sk, uint32_t* skT) {
  const PoGroup c = classes[blockIdx.x];
  for (int m = blockIdx.y; m < c.cnt; m += gridDim.y) {
    const PoShape s = shp[cmem[c.m0 + m]];
    const int dw = c.w * c.d;
    uint32_t* T = skT + toff[blockIdx.x] + m;
    for (int t = threadIdx.x; t < dw; t += 256) T[(int64_t)t * c.cnt] = sk[s.soff + t];
  }
}

// ------------------------------------------ wide candidates: row-0 bound --
// A wide owner u2 (its sketch too large for a group's LDS) against a query u1
// costs nnz(u1) x d2 hashes and gathers per pair, and config 2 has 1,289 of
// them against 100K queries (2.1e11 key-rows).  mostSimilar only keeps the
// top k, so each pair first gets a cheap UPPER bound from sketch row 0:
//   userSimilarity = normalize(min over rows r with den != 0 of AB_r / den_r)
//                 <= normalize(AB_0 / (sqrt(valueA_0 lower bound) * sqrt(B_0)))
// (valueA_0 = sum_j U1_0[j]^2 >= max(sum_k v_k^2, (sum_k v_k)^2 / w2) because
// the increments are non-negative; every fp64 step is correctly rounded and monotone, and
// normalize is non-decreasing).  A pair whose bound is below the query's
// current k-th best score (the narrow candidates' top k, computed first) can
// not enter the list and is written NaN, which TopItems skips; every other
// pair is listed for k_po_pairs' exact computation.  The bound applies only
// while the exact regime holds (sum v < 2^26 so every valueA < 2^53, and
// B_r < 2^53): row r's value is then the same exact expression with the true
// valueA_r.  With h->tune.po_bound_rows = 2 (CMS_PO_BOUND_ROWS) the bound is
// the smaller of rows 0 and 1.  The residues (a_r k + b_r) mod p of those
// rows are precomputed per preference (po_s0), so a key costs a Barrett
// reduction by u2's width and one gather per row.  Lane = wide owner (sorted
// by width), wave = query: the keys are wave-uniform (scalar loads), no
// reductions.
constexpr int kPoBoundWaves = 4;
constexpr int kPoBoundMaxRows = 2;
struct PoBoundArgs {
  const int64_t* off;
  const uint32_t* inc;
  const uint64_t* s0;    // [rows][np] residues (a_r k + b_r) mod p of every preference
  int64_t np;
  const PoShape* shp;
  const uint32_t* sk;
  const uint64_t* norm;
  const double* nsq;
  const int64_t* wrows;  // [nwide] bounded candidate rows (wide owners, the widest narrow part)
  int64_t nwide;
  int64_t big_skip;      // k_po_bigq's queries (more preferences than this) skip narrow candidates
  const double* tsc;     // [qc][k] the narrow candidates' top-k scores
  const int32_t* tcnt;   // [qc] their list lengths
  int32_t k;
  int64_t q0, qc, n;
  double* slab;
  // surviving pairs (u1 << 32) | u2: list 0 for k_po_pairs' LDS paths, list 1
  // for pairs that need its global bucket rows (w > kPoHist, nnz(u1) > 256),
  // list 2 for a u1 of more than kPoBigQuery preferences (four waves a pair)
  unsigned long long* surv[3];
  uint32_t* surv_cnt;    // [3]
  int32_t weighted;
};

// s mod w (s < 2^63, w < 2^30) by the Barrett constant floor((2^64-1)/w):
// the quotient estimate is q - 2 .. q, so the remainder is below 3w < 2^32
// and its low 32 bits are the whole of it; two branch-free corrections
__device__ __forceinline__ uint32_t po_mod_w(uint64_t s, uint32_t w, uint64_t barrett) {
  const uint64_t qq = (uint64_t)(((unsigned __int128)s * barrett) >> 64);
  uint32_t rem = (uint32_t)s - (uint32_t)qq * w;
  rem = rem >= w ? rem - w : rem;
  rem = rem >= w ? rem - w : rem;
  return rem;
}

__global__ __launch_bounds__(256) void k_po_s0(const uint64_t* kp, int64_t np, int rows, HashParams hp, uint64_t* s0) {
  for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < np; i += (int64_t)gridDim.x * blockDim.x) {
    const uint64_t k = kp[i];
    for (int r = 0; r < rows; ++r) s0[r * np + i] = residue_wbq(hp, r, k);
  }
}

__global__ __launch_bounds__(256) void k_po_nanfill(double* slab, int64_t n, const int64_t* wrows, int64_t nwide) {
  double* row = slab + (int64_t)blockIdx.x * n;
  for (int64_t m = threadIdx.x; m < nwide; m += blockDim.x) row[wrows[m]] = __builtin_nan("");
}

// wave-aggregated append of this lane's pair to list l when `keep`
__device__ __forceinline__ void po_append(const PoBoundArgs& a, int l, bool keep, unsigned long long e) {
  const int lane = threadIdx.x & 63;
  const uint64_t mask = __ballot(keep);
  if (mask == 0) return;
  const int first = __builtin_ctzll(mask);
  uint32_t base = 0;
  if (lane == first) base = atomicAdd(&a.surv_cnt[l], (uint32_t)__builtin_popcountll(mask));
  base = __shfl(base, first, 64);
  if (keep) a.surv[l][base + (uint32_t)__builtin_popcountll(mask & ((1ULL << lane) - 1ULL))] = e;
}

template <int R>
__global__ __launch_bounds__(64 * kPoBoundWaves) void k_po_wide_bound(PoBoundArgs a) {
  const int lane = threadIdx.x & 63;
  const int wv = __builtin_amdgcn_readfirstlane((int)(threadIdx.x >> 6));
  const int64_t q = (int64_t)blockIdx.y * kPoBoundWaves + wv;
  if (q >= a.qc) return;  // wave-uniform
  const int64_t m = (int64_t)blockIdx.x * 64 + lane;
  const int64_t u2 = a.wrows[m < a.nwide ? m : 0];
  const PoShape s = a.shp[u2];
  const uint32_t w = (uint32_t)s.w;
  // rows past u2's depth read row 0 (in bounds; left out of the bound below)
  const uint32_t* rowp[R];
#pragma unroll
  for (int r = 0; r < R; ++r) rowp[r] = a.sk + s.soff + (int64_t)(r < s.d ? r : 0) * w;
  const int64_t u1 = a.q0 + q;
  const int64_t k0 = a.off[u1], k1 = a.off[u1 + 1];
  // a narrow candidate of a big query is k_po_bigq's (exact already)
  const bool live = m < a.nwide && !(k1 - k0 > a.big_skip && w <= (uint32_t)kPoGroupHistW && s.w * s.d <= kPoBigMaxDW);
  uint64_t ab[R], a2 = 0, as = 0;
#pragma unroll
  for (int r = 0; r < R; ++r) ab[r] = 0;
  int64_t i = k0;
  constexpr int U = 8 / R;
  for (; i + U <= k1; i += U) {  // the keys' scalar loads together, then the gathers in flight
    uint64_t sv[R][U];
    uint32_t v[U], c[R][U];
#pragma unroll
    for (int u = 0; u < U; ++u) {
      v[u] = a.inc[i + u];
#pragma unroll
      for (int r = 0; r < R; ++r) sv[r][u] = a.s0[r * a.np + i + u];
    }
#pragma unroll
    for (int r = 0; r < R; ++r)
#pragma unroll
      for (int u = 0; u < U; ++u) c[r][u] = rowp[r][po_mod_w(sv[r][u], w, s.barrett)];
#pragma unroll
    for (int u = 0; u < U; ++u) {
#pragma unroll
      for (int r = 0; r < R; ++r) ab[r] += (uint64_t)v[u] * c[r][u];
      a2 += (uint64_t)v[u] * v[u];
      as += v[u];
    }
  }
  for (; i < k1; ++i) {
    const uint32_t v = a.inc[i];
#pragma unroll
    for (int r = 0; r < R; ++r) ab[r] += (uint64_t)v * rowp[r][po_mod_w(a.s0[r * a.np + i], w, s.barrett)];
    a2 += (uint64_t)v * v;
    as += v;
  }
  // (sums wrap only past sum v >= 2^26, where no pair is pruned)
  bool prune = false;
  if (live && a.tcnt[q] >= a.k && as < (1ULL << 26) && a2 != 0) {
    // valueA_r >= (sum_j U1_r[j])^2 / w as well (Cauchy-Schwarz over the w
    // buckets): the tighter of the two when u1 has many more preferences than
    // u2 has buckets
    const uint64_t spread = (as * as + w - 1) / w;
    if (spread > a2) a2 = spread;
    const double sa = __dsqrt_rn((double)a2);
    double ub = DBL_MAX;
#pragma unroll
    for (int r = 0; r < R; ++r) {
      if (r >= s.d) break;  // (that row's sums hashed row r against row 0's counters: no bound)
      const double sb = a.nsq[s.roff + r];
      if (a.norm[s.roff + r] < (1ULL << 53) && sb != 0.0) ub = java_min(ub, __ddiv_rn((double)ab[r], __dmul_rn(sa, sb)));
    }
    if (ub != DBL_MAX) prune = normalize_weight(ub, a.weighted) < a.tsc[q * a.k + a.k - 1];
  }
  if (live && prune) a.slab[q * a.n + u2] = __builtin_nan("");
  const bool keep = live && !prune;
  // k_po_pairs needs a global bucket row for u1 past its register cache, or
  // for the sequential replay of a pair past the exact regime
  bool norms_ok = as < (1ULL << 26);
  for (int r = 0; r < s.d && norms_ok; ++r) norms_ok = a.norm[s.roff + r] < (1ULL << 53);
  const bool global_rows = w > (uint32_t)kPoHist && (k1 - k0 > 4 * kPoThreads || !norms_ok);
  const unsigned long long e = ((unsigned long long)u1 << 32) | (unsigned long long)u2;
  const bool big = k1 - k0 > kPoBigQuery;  // (wave-uniform)
  if (big) {
    po_append(a, 2, keep, e);
  } else {
    po_append(a, 0, keep && !global_rows, e);
    po_append(a, 1, keep && global_rows, e);
  }
}

// DoubleCountMinSketch.get(key) (:94-103) of the owner's own sketch.
__global__ void k_po_point(const PoShape* shp, const uint32_t* sk, HashParams hp, int64_t row, const int64_t* keys,
                           int64_t m, double* out) {
  const PoShape s = shp[row];
  for (int64_t i = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; i < m; i += (int64_t)gridDim.x * blockDim.x) {
    const uint64_t kp = reduce_key(keys[i]);
    double est = DBL_MAX;
    for (int d = 0; d < s.d; ++d) {
      const double v = (double)sk[s.soff + (int64_t)d * s.w + bucket_wbq(hp, d, kp, (uint32_t)s.w, s.barrett)];
      if (v < est) est = v;
    }
    out[i] = ldexp(est, -hp.frac_bits);
  }
}

// doEstimatePreference with the point query of each neighbour's own sketch
// (GenericUserBasedRecommender.java:134-184), as k_estimate for fixed shapes.
__global__ void k_po_estimate(const PoShape* shp, const uint32_t* sk, HashParams hp, int64_t user_row,
                              const int64_t* nb_rows, const double* sims, int64_t m, const int64_t* items, int64_t q,
                              int use_capper, float lo, float hi, float* out) {
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
        const double v = (double)sk[s.soff + (int64_t)d * s.w + bucket_wbq(hp, d, kp, (uint32_t)s.w, s.barrett)];
        if (v < est) est = v;
      }
      const float pref = (float)ldexp(est, -hp.frac_bits);
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

// ---------------------------------------------------------------- host --

static unsigned grid_for(int64_t work, int64_t cap) {
  return (unsigned)std::max<int64_t>(1, std::min<int64_t>(work, cap));
}

int po_load_csr(cms_handle* h, const int64_t* d_off, const int64_t* d_key, const float* d_val, int64_t npairs,
                const int64_t* h_off) {
  const int64_t n = h->n;
  CMS_HIP(h->po_off.ensure(sizeof(int64_t) * (n + 1)));
  CMS_HIP(h->po_kp.ensure(sizeof(uint64_t) * std::max<int64_t>(npairs, 1)));
  CMS_HIP(h->po_inc.ensure(sizeof(uint32_t) * std::max<int64_t>(npairs, 1)));
  CMS_HIP(hipMemcpyAsync(h->po_off.ptr, d_off, sizeof(int64_t) * (n + 1), hipMemcpyDeviceToDevice, h->stream));
  if (h->f64) {  // fp64 counters: (double) preferences, any value
    if (int rc = po_f64_load(h, d_key, d_val, npairs)) return rc;
    h->h_po_off.assign(h_off, h_off + n + 1);
    h->po_npairs = npairs;
    h->po_loaded = true;
    h->finalized = false;
    return CMS_OK;
  }
  if (npairs > 0)
    hipLaunchKernelGGL(k_po_prep, dim3(grid_for((npairs + 255) / 256, 8192)), dim3(256), 0, h->stream, d_key, d_val,
                       npairs, h->hp.frac_bits, h->po_kp.as<uint64_t>(), h->po_inc.as<uint32_t>(), h->d_flags);
  hipLaunchKernelGGL(k_po_mass, dim3(grid_for(n, 65536)), dim3(256), 0, h->stream, h->po_off.as<int64_t>(), n,
                     h->po_inc.as<uint32_t>(), h->d_flags);
  CMS_HIP(hipGetLastError());
  h->h_po_off.assign(h_off, h_off + n + 1);
  h->po_npairs = npairs;
  h->po_loaded = true;
  h->finalized = false;
  return CMS_OK;
}

// shapes from (delta, epsilon) as new DoubleCountMinSketch(delta, epsilon, hfb)
// derives them (AbstractCountMinSketch.java:69-83); 0 marks a CMException
static int po_set_config(cms_handle* h, const double* delta, const double* eps) {
  const int64_t n = h->n;
  std::vector<int32_t> W(n), D(n);
  for (int64_t r = 0; r < n; ++r) {
    int32_t w = 0, d = 0;
    const double de = delta[r], ep = eps[r];
    const bool ok = !(de <= 0 || de > std::exp(-1.0)) && !(ep <= 0 || ep > std::exp(1.0));
    if (ok) {
      const double wf = std::ceil(std::exp(1.0) / ep), df = std::ceil(std::log(1.0 / de));
      if (!(wf <= (double)(1 << 24)) || !(df <= (double)CMS_MAX_DEPTH))
        return set_error(CMS_E_PARAM,
                         "owner row %lld: sketch shape %.0f x %.0f exceeds this build (width <= 2^24, depth <= %d)",
                         (long long)r, wf, df, CMS_MAX_DEPTH);
      w = (int32_t)wf;
      d = (int32_t)df;
    }
    W[r] = w;
    D[r] = d;
  }
  std::vector<PoShape> shp(n);
  int64_t so = 0, ro = 0;
  int32_t mw = 0, md = 0;
  for (int64_t r = 0; r < n; ++r) {
    shp[r].soff = so;
    shp[r].roff = ro;
    shp[r].w = W[r];
    shp[r].d = D[r];
    shp[r].barrett = W[r] > 0 ? (~0ULL) / (uint64_t)W[r] : 0;
    so += (int64_t)W[r] * D[r];
    ro += D[r];
    mw = std::max(mw, W[r]);
    md = std::max(md, D[r]);
  }
  CMS_HIP(h->po_shape.ensure(sizeof(PoShape) * n));
  CMS_HIP(hipMemcpyAsync(h->po_shape.ptr, shp.data(), sizeof(PoShape) * n, hipMemcpyHostToDevice, h->stream));
  CMS_HIP(hipStreamSynchronize(h->stream));
  h->h_po_delta.assign(delta, delta + n);
  h->h_po_eps.assign(eps, eps + n);
  h->h_po_w.swap(W);
  h->h_po_d.swap(D);
  h->po_max_w = mw;
  h->po_max_d = md;
  h->po_configured = true;
  h->finalized = false;
  return CMS_OK;
}

bool po_shared_scratch(cms_handle* h) { return h->per_owner && (h->f64 || h->po_max_w > kPoHist); }

int po_require_shapes(cms_handle* h, const int64_t* rows, int64_t m) {
  const int64_t cnt = rows ? m : h->n;
  for (int64_t i = 0; i < cnt; ++i) {
    const int64_t r = rows ? rows[i] : i;
    if (h->h_po_w[r] <= 0)
      return set_error(CMS_E_SKETCH,
                       "CountMinSketch error: delta/epsilon of owner %lld outside (0, e^-1] x (0, e] (CMException)",
                       (long long)(h->h_owner_ids.empty() ? r : h->h_owner_ids[r]));
  }
  return CMS_OK;
}

// Candidate groups of the all-pairs slabs: owners sorted by shape class
// (d, w); a class whose bucket row fits a wave's LDS row (narrow) is cut into
// groups of up to kPoGroupMax members, every other owner (wide) is its own
// group for k_po_pairs.  Narrow groups first.  The narrow classes whole, with
// their members' sketches transposed (po_skT), are the operand of both the
// group kernel and k_po_bigq.
static int po_build_groups(cms_handle* h) {
  const int64_t n = h->n;
  std::vector<int64_t> ord;
  ord.reserve(n);
  for (int64_t r = 0; r < n; ++r)
    if (h->h_po_w[r] > 0) ord.push_back(r);
  std::stable_sort(ord.begin(), ord.end(), [&](int64_t x, int64_t y) {
    return h->h_po_d[x] != h->h_po_d[y] ? h->h_po_d[x] < h->h_po_d[y] : h->h_po_w[x] < h->h_po_w[y];
  });
  std::vector<PoGroup> narrow, classes;
  std::vector<int64_t> cmem_n, cmem_w, toff;
  int32_t hist_w = 1, maxdw = 0;
  int64_t tot = 0;
  for (size_t i = 0; i < ord.size();) {
    const int32_t w = h->h_po_w[ord[i]], d = h->h_po_d[ord[i]];
    size_t e = i;
    while (e < ord.size() && h->h_po_w[ord[e]] == w && h->h_po_d[ord[e]] == d) ++e;
    if (w <= kPoGroupHistW) {
      PoGroup c{};
      c.w = w;
      c.d = d;
      c.barrett = (~0ULL) / (uint64_t)w;
      c.m0 = (int32_t)cmem_n.size();
      c.cnt = (int32_t)(e - i);
      const int32_t ci = (int32_t)classes.size();
      classes.push_back(c);
      toff.push_back(tot);
      tot += (int64_t)c.cnt * w * d;
      maxdw = std::max<int32_t>(maxdw, w * d);
      hist_w = std::max(hist_w, w);
      for (size_t m = i; m < e; m += kPoGroupMax) {
        PoGroup g = c;
        g.m0 = (int32_t)cmem_n.size();
        g.cnt = (int)std::min<size_t>(kPoGroupMax, e - m);
        g.pad = ci;
        for (int q = 0; q < g.cnt; ++q) cmem_n.push_back(ord[m + q]);
        narrow.push_back(g);
      }
    } else {
      for (size_t m = i; m < e; ++m) cmem_w.push_back(ord[m]);
    }
    i = e;
  }
  // narrow groups by width part (each part's launch takes only the LDS its
  // widest row needs, so more workgroups share a CU); class order kept within
  std::stable_sort(narrow.begin(), narrow.end(), [](const PoGroup& x, const PoGroup& y) {
    return po_hist_part(x.w) < po_hist_part(y.w);
  });
  int64_t nsmall[kPoHistParts] = {};
  for (const PoGroup& g : narrow) ++nsmall[po_hist_part(g.w)];
  std::vector<PoGroup> groups(narrow);
  std::vector<int64_t> cmem(cmem_n);
  cmem.insert(cmem.end(), cmem_w.begin(), cmem_w.end());
  for (size_t m = 0; m < cmem_w.size(); ++m) {  // wide owners: one group each (members at the end of cmem)
    PoGroup g{};
    g.w = h->h_po_w[cmem_w[m]];
    g.d = h->h_po_d[cmem_w[m]];
    g.barrett = (~0ULL) / (uint64_t)g.w;
    g.m0 = (int32_t)(cmem_n.size() + m);
    g.cnt = 1;
    g.wide = 1;
    groups.push_back(g);
  }
  CMS_HIP(h->po_groups.ensure(sizeof(PoGroup) * std::max<size_t>(1, groups.size())));
  CMS_HIP(h->po_cmem.ensure(sizeof(int64_t) * std::max<size_t>(1, cmem.size())));
  if (!groups.empty())
    CMS_HIP(hipMemcpyAsync(h->po_groups.ptr, groups.data(), sizeof(PoGroup) * groups.size(), hipMemcpyHostToDevice,
                           h->stream));
  if (!cmem.empty())
    CMS_HIP(hipMemcpyAsync(h->po_cmem.ptr, cmem.data(), sizeof(int64_t) * cmem.size(), hipMemcpyHostToDevice,
                           h->stream));
  h->po_nclasses = (int64_t)classes.size();
  h->po_class_maxdw = maxdw;
  if (!classes.empty()) {
    CMS_HIP(h->po_classes.ensure(sizeof(PoGroup) * classes.size() + sizeof(int64_t) * toff.size()));
    CMS_HIP(hipMemcpyAsync(h->po_classes.ptr, classes.data(), sizeof(PoGroup) * classes.size(), hipMemcpyHostToDevice,
                           h->stream));
    CMS_HIP(hipMemcpyAsync(h->po_classes.as<char>() + sizeof(PoGroup) * classes.size(), toff.data(),
                           sizeof(int64_t) * toff.size(), hipMemcpyHostToDevice, h->stream));
    CMS_HIP(h->po_skT.ensure(sizeof(uint32_t) * (size_t)std::max<int64_t>(tot, 1)));
    int32_t maxcnt = 1;
    for (const PoGroup& c : classes) maxcnt = std::max(maxcnt, c.cnt);
    hipLaunchKernelGGL(k_po_transpose, dim3((unsigned)classes.size(), (unsigned)std::min(maxcnt, 256)), dim3(256), 0,
                       h->stream, h->po_classes.as<PoGroup>(), h->po_cmem.as<int64_t>(),
                       reinterpret_cast<const int64_t*>(h->po_classes.as<char>() + sizeof(PoGroup) * classes.size()),
                       h->po_shape.as<PoShape>(), h->po_sk.as<uint32_t>(), h->po_skT.as<uint32_t>());
    CMS_HIP(hipGetLastError());
  }
  // k_po_wide_bound's candidates by width (lanes of a wave alike): the wide
  // owners, and the narrow ones of the widest part (their member images are
  // the group kernel's costliest) unless h->tune.po_bound_part2 is off
  std::vector<int64_t> wrows(cmem_w);
  h->po_nbound_narrow = 0;
  if (h->tune.po_bound_part2)
    for (const PoGroup& g : narrow)
      if (po_hist_part(g.w) == kPoHistParts - 1) {
        for (int q = 0; q < g.cnt; ++q) wrows.push_back(cmem_n[g.m0 + q]);
        h->po_nbound_narrow += g.cnt;
      }
  std::stable_sort(wrows.begin(), wrows.end(), [&](int64_t x, int64_t y) { return h->h_po_w[x] < h->h_po_w[y]; });
  h->po_nbound = (int64_t)wrows.size();
  if (!wrows.empty()) {
    CMS_HIP(h->po_wrows.ensure(sizeof(int64_t) * wrows.size()));
    CMS_HIP(hipMemcpyAsync(h->po_wrows.ptr, wrows.data(), sizeof(int64_t) * wrows.size(), hipMemcpyHostToDevice,
                           h->stream));
  }
  CMS_HIP(hipStreamSynchronize(h->stream));  // the host vectors die on return
  h->po_ngroups = (int64_t)groups.size();
  h->po_nnarrow = (int64_t)narrow.size();
  h->po_wide0 = (int64_t)cmem_n.size();
  h->po_hist_w = hist_w;
  for (int i = 0; i < kPoHistParts; ++i) h->po_nnarrow_part[i] = nsmall[i];
  h->po_gmax_lds = (int32_t)po_group_lds(hist_w);
  return CMS_OK;
}

int po_finalize(cms_handle* h) {
  if (!h->po_loaded) return set_error(CMS_E_STATE, "per-owner mode: ingest the DataModel (CSR) first");
  if (!h->po_configured)
    return set_error(CMS_E_STATE, "delta is null, call configure method first (cms_configure_owner_shapes)");
  const int64_t n = h->n;
  int64_t total = 0, rtot = 0;
  for (int64_t r = 0; r < n; ++r) {
    total += (int64_t)h->h_po_w[r] * h->h_po_d[r];
    rtot += h->h_po_d[r];
  }
  if (h->f64) {
    if (int rc = po_f64_finalize(h, total, rtot)) return rc;
    CMS_HIP(hipStreamSynchronize(h->stream));
    return CMS_OK;
  }
  CMS_HIP(h->po_sk.ensure(sizeof(uint32_t) * std::max<int64_t>(total, 1)));
  CMS_HIP(h->po_norm.ensure(sizeof(uint64_t) * std::max<int64_t>(rtot, 1)));
  CMS_HIP(h->po_nsq.ensure(sizeof(double) * std::max<int64_t>(rtot, 1)));
  CMS_HIP(hipMemsetAsync(h->po_sk.ptr, 0, sizeof(uint32_t) * std::max<int64_t>(total, 1), h->stream));
  {
    TimedScope ts(h, "po_build");
    hipLaunchKernelGGL(k_po_build, dim3(grid_for(n, 65536)), dim3(256), 0, h->stream, h->po_off.as<int64_t>(),
                       h->po_kp.as<uint64_t>(), h->po_inc.as<uint32_t>(), h->po_shape.as<PoShape>(), h->hp, n,
                       h->po_sk.as<uint32_t>());
    hipLaunchKernelGGL(k_po_norms, dim3(grid_for(n, 65536)), dim3(256), 0, h->stream, h->po_shape.as<PoShape>(), n,
                       h->po_sk.as<uint32_t>(), h->po_norm.as<uint64_t>(), h->po_nsq.as<double>());
    CMS_HIP(hipGetLastError());
  }
  if (h->po_max_w > kPoHist) {
    const size_t need = sizeof(uint32_t) * (size_t)kPoGridWide * (size_t)h->po_max_w;
    if (h->po_scratch.bytes < need) {
      CMS_HIP(h->po_scratch.ensure(need));
      CMS_HIP(hipMemsetAsync(h->po_scratch.ptr, 0, h->po_scratch.bytes, h->stream));
    }
  }
  h->po_s0_rows = std::max(1, std::min(std::min(h->tune.po_bound_rows, kPoBoundMaxRows), (int)h->hp.depth));
  CMS_HIP(h->po_s0.ensure(sizeof(uint64_t) * (size_t)h->po_s0_rows * (size_t)std::max<int64_t>(h->po_npairs, 1)));
  if (h->po_npairs > 0) {
    hipLaunchKernelGGL(k_po_s0, dim3(grid_for((h->po_npairs + 255) / 256, 16384)), dim3(256), 0, h->stream,
                       h->po_kp.as<uint64_t>(), h->po_npairs, h->po_s0_rows, h->hp, h->po_s0.as<uint64_t>());
    CMS_HIP(hipGetLastError());
  }
  if (int rc = po_build_groups(h)) return rc;
  CMS_HIP(hipStreamSynchronize(h->stream));
  return CMS_OK;
}

int po_pair_cosines(cms_handle* h, const int64_t* d_qrows, int64_t nq, const int64_t* d_crows, int64_t m,
                    double* d_out, hipStream_t s) {
  if (nq <= 0 || m <= 0) return CMS_OK;
  if (h->f64) return po_f64_pair_cosines(h, d_qrows, nq, d_crows, m, d_out, s);
  PoPairArgs a;
  a.off = h->po_off.as<int64_t>();
  a.kp = h->po_kp.as<uint64_t>();
  a.inc = h->po_inc.as<uint32_t>();
  a.shp = h->po_shape.as<PoShape>();
  a.sk = h->po_sk.as<uint32_t>();
  a.norm = h->po_norm.as<uint64_t>();
  a.nsq = h->po_nsq.as<double>();
  a.qrows = d_qrows;
  a.crows = d_crows;
  a.nq = nq;
  a.m = m;
  const bool wide = h->po_max_w > kPoHist;
  a.scratch = wide ? h->po_scratch.as<uint32_t>() : nullptr;
  a.scratch_w = wide ? h->po_max_w : 0;
  a.out = d_out;
  a.ldo = 0;
  a.weighted = h->p.weighting == CMS_WEIGHTED;
  TimedScope ts(h, "po_pair_cosine", s == nullptr);
  hipLaunchKernelGGL(k_po_pairs<kPoThreads>, dim3(grid_for(nq * m, wide ? kPoGridWide : kPoGrid)), dim3(kPoThreads), 0,
                     s ? s : h->stream, a, h->hp);
  CMS_HIP(hipGetLastError());
  return CMS_OK;
}

int po_point_queries(cms_handle* h, int64_t row, const int64_t* d_keys, int64_t m, double* d_out, hipStream_t s) {
  if (m <= 0) return CMS_OK;
  if (h->f64) return po_f64_point_queries(h, row, d_keys, m, d_out, s);
  hipLaunchKernelGGL(k_po_point, dim3(grid_for((m + 255) / 256, 4096)), dim3(256), 0, s ? s : h->stream,
                     h->po_shape.as<PoShape>(), h->po_sk.as<uint32_t>(), h->hp, row, d_keys, m, d_out);
  CMS_HIP(hipGetLastError());
  return CMS_OK;
}

int po_estimate_preferences(cms_handle* h, int64_t user_row, const int64_t* d_nb_rows, const double* d_sims, int64_t m,
                            const int64_t* d_items, int64_t q, int use_capper, float lo, float hi, float* d_out,
                            hipStream_t s) {
  if (q <= 0) return CMS_OK;
  if (h->f64)
    return po_f64_estimate_preferences(h, user_row, d_nb_rows, d_sims, m, d_items, q, use_capper, lo, hi, d_out, s);
  hipLaunchKernelGGL(k_po_estimate, dim3(grid_for((q + 255) / 256, 4096)), dim3(256), 0, s ? s : h->stream,
                     h->po_shape.as<PoShape>(), h->po_sk.as<uint32_t>(), h->hp, user_row, d_nb_rows, d_sims, m,
                     d_items, q, use_capper, lo, hi, d_out);
  CMS_HIP(hipGetLastError());
  return CMS_OK;
}

// slab[q][c] = userSimilarity(q0 + q, c) for q < qc and every candidate c
// (d_qrows: the rows q0 .. q0 + qc - 1 on the device): the narrow groups on
// k_po_group_pairs (big queries on k_po_bigq), the wide owners and any pair
// past the exact regime on k_po_pairs (scattered into the slab's columns).
// prune_k > 0: the slab feeds a top-prune_k selection, and wide pairs whose
// row-0 bound (k_po_wide_bound) cannot reach a query's list are NaN instead.
static int po_allpairs_slab(cms_handle* h, int64_t q0, int64_t qc, const int64_t* d_qrows, double* slab,
                            int32_t prune_k) {
  const int64_t n = h->n;
  PoAllArgs a{};
  a.off = h->po_off.as<int64_t>();
  a.kp = h->po_kp.as<uint64_t>();
  a.inc = h->po_inc.as<uint32_t>();
  a.shp = h->po_shape.as<PoShape>();
  a.sk = h->po_sk.as<uint32_t>();
  a.norm = h->po_norm.as<uint64_t>();
  a.nsq = h->po_nsq.as<double>();
  a.groups = h->po_groups.as<PoGroup>();
  a.cmem = h->po_cmem.as<int64_t>();
  a.q0 = q0;
  a.qc = qc;
  a.n = n;
  a.slab = slab;
  a.weighted = h->p.weighting == CMS_WEIGHTED;
  constexpr uint32_t kRedoCap = 1u << 16;
  CMS_HIP(h->po_redo.ensure(sizeof(unsigned long long) * kRedoCap + 16));
  a.redo = h->po_redo.as<unsigned long long>();
  a.redo_cnt = reinterpret_cast<uint32_t*>(a.redo + kRedoCap);
  a.redo_cap = kRedoCap;
  CMS_HIP(hipMemsetAsync(a.redo_cnt, 0, sizeof(uint32_t), h->stream));
  const int64_t nwide = h->po_ngroups - h->po_nnarrow;
  const bool prune = prune_k > 0 && !h->tune.po_no_prune && h->po_nbound > 0;
  // pruning: the bounded candidates' columns start NaN (the narrow top k
  // below is taken without them; k_po_bigq's big queries overwrite theirs)
  if (prune) {
    hipLaunchKernelGGL(k_po_nanfill, dim3((unsigned)qc), dim3(256), 0, h->stream, slab, n, h->po_wrows.as<int64_t>(),
                       h->po_nbound);
    CMS_HIP(hipGetLastError());
  }
  // queries of more than kPoBigQuery preferences take the narrow classes
  // through k_po_bigq (u1 hashed once per class); the group kernel skips them
  std::vector<int64_t> bigq;
  if (h->po_nclasses > 0 && !h->tune.po_no_bigq)
    for (int64_t q = 0; q < qc; ++q)
      if (h->h_po_off[q0 + q + 1] - h->h_po_off[q0 + q] > kPoBigQuery) bigq.push_back(q);
  a.big_skip = bigq.empty() ? INT64_MAX : kPoBigQuery;
  if (!bigq.empty()) {
    TimedScope ts(h, "po_bigq");
    CMS_HIP(h->ws_query2.ensure(sizeof(int64_t) * bigq.size()));
    CMS_HIP(hipMemcpyAsync(h->ws_query2.ptr, bigq.data(), sizeof(int64_t) * bigq.size(), hipMemcpyHostToDevice,
                           h->stream));
    PoBigArgs b{};
    b.off = a.off;
    b.kp = a.kp;
    b.inc = a.inc;
    b.shp = a.shp;
    b.norm = a.norm;
    b.nsq = a.nsq;
    b.classes = h->po_classes.as<PoGroup>();
    b.cmem = a.cmem;
    b.skT = h->po_skT.as<uint32_t>();
    b.toff = reinterpret_cast<const int64_t*>(h->po_classes.as<char>() + sizeof(PoGroup) * h->po_nclasses);
    b.bigq = h->ws_query2.as<int64_t>();
    b.q0 = q0;
    b.n = n;
    b.slab = slab;
    b.redo = a.redo;
    b.redo_cnt = a.redo_cnt;
    b.redo_cap = a.redo_cap;
    b.weighted = a.weighted;
    static bool battr = [] {
      // the dynamic image only: the static s_a2 counts against the same 160 KiB
      (void)hipFuncSetAttribute((const void*)k_po_bigq, hipFuncAttributeMaxDynamicSharedMemorySize,
                                (int)(sizeof(uint32_t) * kPoBigMaxDW));
      return true;
    }();
    (void)battr;
    hipLaunchKernelGGL(k_po_bigq, dim3((unsigned)h->po_nclasses, (unsigned)bigq.size()), dim3(kPoBigThreads),
                       sizeof(uint32_t) * (size_t)std::min<int64_t>(h->po_class_maxdw, kPoBigMaxDW), h->stream, b,
                       h->hp);
    CMS_HIP(hipGetLastError());
  }
  if (h->po_nnarrow > 0) {
    TimedScope ts(h, "po_group_pairs");
    static bool attr = [] {
      (void)hipFuncSetAttribute((const void*)k_po_group_pairs, hipFuncAttributeMaxDynamicSharedMemorySize,
                                (int)po_group_lds(kPoGroupHistW));
      return true;
    }();
    (void)attr;
    a.classes = h->po_classes.as<PoGroup>();
    a.toff = reinterpret_cast<const int64_t*>(h->po_classes.as<char>() + sizeof(PoGroup) * h->po_nclasses);
    a.skT = h->po_skT.as<uint32_t>();
    a.nchunks = (qc + kPoQueryChunk - 1) / kPoQueryChunk;
    a.dense_x4 = h->tune.po_dense_x4;
    int64_t g0 = 0;
    // (pruning with the widest part bounded: that part is k_po_wide_bound's)
    const int nparts = prune && h->po_nbound_narrow > 0 ? kPoHistParts - 1 : kPoHistParts;
    for (int pi = 0; pi < nparts; ++pi) {
      a.g0 = g0;
      a.ngroups = h->po_nnarrow_part[pi];
      g0 += a.ngroups;
      if (a.ngroups <= 0) continue;
      a.per_xcd = (a.ngroups * a.nchunks + 7) / 8;
      a.hist_w = std::min<int32_t>(kPoSmallHist << pi, h->po_hist_w);
      hipLaunchKernelGGL(k_po_group_pairs, dim3((unsigned)(8 * a.per_xcd)), dim3(64 * kPoGroupWaves),
                         po_group_lds(a.hist_w), h->stream, a, h->hp);
      CMS_HIP(hipGetLastError());
    }
  }
  if (nwide > 0 || prune) {  // wide candidates: one wave per pair, columns scattered into the slab
    PoPairArgs p{};
    p.off = a.off;
    p.kp = a.kp;
    p.inc = a.inc;
    p.shp = a.shp;
    p.sk = a.sk;
    p.norm = a.norm;
    p.nsq = a.nsq;
    p.qrows = d_qrows;
    p.crows = a.cmem + h->po_wide0;  // the wide owners close po_cmem
    p.nq = qc;
    p.m = nwide;
    const bool wide = h->po_max_w > kPoHist;
    p.scratch = wide ? h->po_scratch.as<uint32_t>() : nullptr;
    p.scratch_w = wide ? h->po_max_w : 0;
    p.out = slab;
    p.ldo = n;
    p.weighted = a.weighted;
    const int64_t nb = prune ? h->po_nbound : nwide;
    const int64_t npairs = qc * nb;
    if (prune) {
      // the narrow candidates' top k of every query (wide columns NaN), then
      // the row-0 bound against its k-th score; survivors listed
      const int32_t k = prune_k;
      const size_t ids_b = sizeof(int64_t) * (size_t)(qc * k), sc_b = sizeof(double) * (size_t)(qc * k);
      CMS_HIP(h->ws_pothr.ensure(ids_b + sc_b + sizeof(int32_t) * (size_t)qc));
      int64_t* tids = h->ws_pothr.as<int64_t>();
      double* tsc = reinterpret_cast<double*>(h->ws_pothr.as<char>() + ids_b);
      int32_t* tcnt = reinterpret_cast<int32_t*>(h->ws_pothr.as<char>() + ids_b + sc_b);
      CMS_HIP(h->ws_posurv.ensure(sizeof(unsigned long long) * 3 * (size_t)npairs + 16));
      unsigned long long* surv = h->ws_posurv.as<unsigned long long>();
      uint32_t* surv_cnt = reinterpret_cast<uint32_t*>(surv + 3 * npairs);  // [0..2] the lists; [3] no_rows
      CMS_HIP(hipMemsetAsync(surv_cnt, 0, 4 * sizeof(uint32_t), h->stream));
      std::vector<TopQuery> tq(qc);
      for (int64_t q = 0; q < qc; ++q) tq[q] = TopQuery{q, q0 + q, q};
      if (int rc = launch_top_k(h, slab, tq, k, nullptr, tids, tsc, tcnt)) return rc;
      PoBoundArgs b{};
      b.off = a.off;
      b.inc = a.inc;
      b.s0 = h->po_s0.as<uint64_t>();
      b.np = h->po_npairs;
      b.shp = a.shp;
      b.sk = a.sk;
      b.norm = a.norm;
      b.nsq = a.nsq;
      b.wrows = h->po_wrows.as<int64_t>();
      b.nwide = nb;
      b.big_skip = a.big_skip;
      b.tsc = tsc;
      b.tcnt = tcnt;
      b.k = k;
      b.q0 = q0;
      b.qc = qc;
      b.n = n;
      b.slab = slab;
      b.surv[0] = surv;
      b.surv[1] = surv + npairs;
      b.surv[2] = surv + 2 * npairs;
      b.surv_cnt = surv_cnt;
      b.weighted = a.weighted;
      {
        TimedScope ts(h, "po_wide_bound");
        // (an XCD-ordered 1-D tiling measured 8 % slower: the gathers are not L2-bound)
        const dim3 grid((unsigned)((nb + 63) / 64), (unsigned)((qc + kPoBoundWaves - 1) / kPoBoundWaves));
        if (h->po_s0_rows >= 2)
          hipLaunchKernelGGL(k_po_wide_bound<2>, grid, dim3(64 * kPoBoundWaves), 0, h->stream, b);
        else
          hipLaunchKernelGGL(k_po_wide_bound<1>, grid, dim3(64 * kPoBoundWaves), 0, h->stream, b);
        CMS_HIP(hipGetLastError());
      }
      uint32_t ns[3] = {0, 0, 0};
      CMS_HIP(hipMemcpyAsync(ns, surv_cnt, sizeof ns, hipMemcpyDeviceToHost, h->stream));
      CMS_HIP(hipStreamSynchronize(h->stream));
      h->po_wide_pairs += npairs;
      h->po_wide_exact += ns[0] + ns[1] + ns[2];
      p.q0 = q0;
      p.m = 1;
      p.no_rows = surv_cnt + 3;
      TimedScope ts(h, "po_pair_cosine");
      if (ns[0] > 0) {  // LDS bucket rows or tables only: a full grid of one-wave blocks
        p.plist = surv;
        p.nq = ns[0];
        p.scratch = nullptr;
        p.scratch_w = 0;
        hipLaunchKernelGGL(k_po_pairs<kPoThreads>, dim3(grid_for(ns[0], kPoGridList)), dim3(kPoThreads), 0, h->stream, p, h->hp);
        CMS_HIP(hipGetLastError());
      }
      if (ns[1] > 0) {  // global bucket rows: the scratch's blocks
        p.plist = surv + npairs;
        p.nq = ns[1];
        p.scratch = wide ? h->po_scratch.as<uint32_t>() : nullptr;
        p.scratch_w = wide ? h->po_max_w : 0;
        hipLaunchKernelGGL(k_po_pairs<kPoThreads>, dim3(grid_for(ns[1], wide ? kPoGridWide : kPoGrid)), dim3(kPoThreads), 0,
                           h->stream, p, h->hp);
        CMS_HIP(hipGetLastError());
      }
      if (ns[2] > 0) {  // big u1: four waves per pair, the scratch's blocks
        p.plist = surv + 2 * npairs;
        p.nq = ns[2];
        p.scratch = wide ? h->po_scratch.as<uint32_t>() : nullptr;
        p.scratch_w = wide ? h->po_max_w : 0;
        hipLaunchKernelGGL(k_po_pairs<kPoBigThreadsPair>, dim3(grid_for(ns[2], wide ? kPoGridWide : kPoGrid)),
                           dim3(kPoBigThreadsPair), 0, h->stream, p, h->hp);
        CMS_HIP(hipGetLastError());
      }
      uint32_t bad = 0;
      CMS_HIP(hipMemcpyAsync(&bad, surv_cnt + 3, sizeof bad, hipMemcpyDeviceToHost, h->stream));
      CMS_HIP(hipStreamSynchronize(h->stream));
      if (bad) return set_error(CMS_E_STATE, "per-owner all-pairs: %u listed pairs needed a global bucket row", bad);
    } else {
      TimedScope ts(h, "po_pair_cosine");
      hipLaunchKernelGGL(k_po_pairs<kPoThreads>, dim3(grid_for(npairs, wide ? kPoGridWide : kPoGrid)), dim3(kPoThreads), 0,
                         h->stream, p, h->hp);
      CMS_HIP(hipGetLastError());
    }
  }
  uint32_t nredo = 0;
  CMS_HIP(hipMemcpyAsync(&nredo, a.redo_cnt, sizeof(uint32_t), hipMemcpyDeviceToHost, h->stream));
  CMS_HIP(hipStreamSynchronize(h->stream));
  if (nredo > kRedoCap) return set_error(CMS_E_OVERFLOW, "per-owner all-pairs: %u pairs past the exact regime", nredo);
  if (nredo > 0) {  // the reference's sequential fp64 loop for these pairs (k_po_pairs)
    std::vector<unsigned long long> redo(nredo);
    CMS_HIP(hipMemcpy(redo.data(), a.redo, sizeof(unsigned long long) * nredo, hipMemcpyDeviceToHost));
    DevBuf rows;
    CMS_HIP(rows.ensure(sizeof(int64_t) * 2 * nredo));
    std::vector<int64_t> hr(2 * nredo);
    for (uint32_t i = 0; i < nredo; ++i) {
      hr[2 * i] = (int64_t)(redo[i] >> 32);
      hr[2 * i + 1] = (int64_t)(redo[i] & 0xFFFFFFFFu);
    }
    CMS_HIP(hipMemcpy(rows.ptr, hr.data(), sizeof(int64_t) * 2 * nredo, hipMemcpyHostToDevice));
    for (uint32_t i = 0; i < nredo; ++i) {
      const int64_t* pr = rows.as<int64_t>() + 2 * i;
      if (int rc = po_pair_cosines(h, pr, 1, pr + 1, 1, slab + (hr[2 * i] - q0) * n + hr[2 * i + 1])) return rc;
    }
    CMS_HIP(hipStreamSynchronize(h->stream));
  }
  return CMS_OK;
}

// mostSimilar for query rows [row_begin, row_begin + row_count): a slab of
// userSimilarity(query, candidate) over every candidate (the MostSimilarEstimator
// argument order, GenericUserBasedRecommender.java:231-247), then the shared
// TopItems.getTopUsers selection (cms_topk.hip).
int po_top_k_rows(cms_handle* h, int64_t row_begin, int64_t row_count, int32_t k, int64_t* d_ids, double* d_scores,
                  int32_t* d_counts) {
  if (k < 1 || k > 1024) return set_error(CMS_E_PARAM, "k must be in [1, 1024]");
  int rc = po_require_shapes(h, nullptr, 0);
  if (rc) return rc;
  const int64_t n = h->n;
  const int64_t qb = std::min<int64_t>(row_count, slab_rows_for(n));
  CMS_HIP(h->ws_slab.ensure(sizeof(double) * (size_t)(qb * n)));
  CMS_HIP(h->ws_query.ensure(sizeof(int64_t) * (size_t)qb));
  std::vector<int64_t> qrows(qb);
  for (int64_t r0 = 0; r0 < row_count; r0 += qb) {
    const int64_t rcnt = std::min(qb, row_count - r0);
    std::vector<TopQuery> qs;
    for (int64_t q = 0; q < rcnt; ++q) {
      qrows[q] = row_begin + r0 + q;
      qs.push_back(TopQuery{q, row_begin + r0 + q, r0 + q});
    }
    CMS_HIP(hipMemcpyAsync(h->ws_query.ptr, qrows.data(), sizeof(int64_t) * rcnt, hipMemcpyHostToDevice, h->stream));
    if (h->f64) {
      if ((rc = po_pair_cosines(h, h->ws_query.as<int64_t>(), rcnt, nullptr, n, h->ws_slab.as<double>()))) return rc;
    } else if ((rc = po_allpairs_slab(h, row_begin + r0, rcnt, h->ws_query.as<int64_t>(), h->ws_slab.as<double>(),
                                      k))) {
      return rc;
    }
    if ((rc = launch_top_k(h, h->ws_slab.as<double>(), qs, k, nullptr, d_ids, d_scores, d_counts))) return rc;
  }
  return CMS_OK;
}

}  // namespace cms

using namespace cms;

extern "C" {

int cms_configure_owner_shapes(cms_handle* h, double q, int64_t num_keys) {
  if (!h) return set_error(CMS_E_PARAM, "null handle");
  if (!h->per_owner) return set_error(CMS_E_STATE, "fixed-shape handle: shapes come from cms_params");
  if (num_keys < 0 || num_keys > 0x7fffffff) return set_error(CMS_E_PARAM, "num_keys must be an int (getNumItems)");
  std::lock_guard<std::shared_mutex> g(h->mu);
  (void)hipSetDevice(h->device);
  if (!h->po_loaded) return set_error(CMS_E_STATE, "per-owner mode: ingest the DataModel (CSR) first");
  const int64_t n = h->n;
  DevBuf bw, bd;
  CMS_HIP(bw.ensure(sizeof(int32_t) * n));
  CMS_HIP(bd.ensure(sizeof(int32_t) * n));
  {
    TimedScope ts(h, "po_config");
    hipLaunchKernelGGL(k_po_config, dim3(grid_for(n, 65536)), dim3(kCfgThreads), 0, h->stream,
                       h->po_off.as<int64_t>(), n, (int32_t)num_keys, std::pow(q, 2.0), bw.as<int32_t>(),
                       bd.as<int32_t>());
    CMS_HIP(hipGetLastError());
  }
  std::vector<int32_t> W(n), D(n);
  CMS_HIP(hipMemcpyAsync(W.data(), bw.ptr, sizeof(int32_t) * n, hipMemcpyDeviceToHost, h->stream));
  CMS_HIP(hipMemcpyAsync(D.data(), bd.ptr, sizeof(int32_t) * n, hipMemcpyDeviceToHost, h->stream));
  CMS_HIP(hipStreamSynchronize(h->stream));
  bw.release();
  bd.release();
  std::vector<double> delta(n), eps(n);
  for (int64_t r = 0; r < n; ++r) {
    if (W[r] == 0 && D[r] == 0)  // CountMinSketchConfig.java:145-147
      return set_error(CMS_E_SKETCH, "No solution found (this should not happen) (w=0 and d=0) for owner %lld",
                       (long long)(h->h_owner_ids.empty() ? r : h->h_owner_ids[r]));
    eps[r] = std::exp(1.0) / (double)W[r];
    delta[r] = std::exp(-(double)D[r]);
  }
  return po_set_config(h, delta.data(), eps.data());
}

int cms_set_owner_delta_epsilon(cms_handle* h, const double* delta, const double* epsilon) {
  if (!h || !delta || !epsilon) return set_error(CMS_E_PARAM, "null argument");
  if (!h->per_owner) return set_error(CMS_E_STATE, "fixed-shape handle: shapes come from cms_params");
  std::lock_guard<std::shared_mutex> g(h->mu);
  (void)hipSetDevice(h->device);
  return po_set_config(h, delta, epsilon);
}

int cms_get_owner_shapes(cms_handle* h, double* delta, double* epsilon, int32_t* width, int32_t* depth) {
  if (!h) return set_error(CMS_E_PARAM, "null handle");
  if (!h->per_owner) return set_error(CMS_E_STATE, "fixed-shape handle: shapes come from cms_params");
  std::lock_guard<std::shared_mutex> g(h->mu);
  if (!h->po_configured)
    return set_error(CMS_E_STATE, "delta is null, call configure method first (cms_configure_owner_shapes)");
  const size_t n = (size_t)h->n;
  if (delta) std::copy(h->h_po_delta.begin(), h->h_po_delta.begin() + n, delta);
  if (epsilon) std::copy(h->h_po_eps.begin(), h->h_po_eps.begin() + n, epsilon);
  if (width) std::copy(h->h_po_w.begin(), h->h_po_w.begin() + n, width);
  if (depth) std::copy(h->h_po_d.begin(), h->h_po_d.begin() + n, depth);
  return CMS_OK;
}

}  // extern "C"
