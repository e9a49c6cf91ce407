// cms_cosine_mfma.hip -- all-pairs sketch cosine on the gfx950 matrix cores.
//
// The table is a dense [n][d*w] matrix; DoubleCountMinSketch.cosine
// (T/impl/common/DoubleCountMinSketch.java:114-149) needs, per sketch row r,
// the dot product of two owners' w counters.  Those are d GEMMs with K = w,
// run here as ONE MFMA pipeline whose K loop walks the d segments and runs an
// fp64 epilogue at every segment boundary (den = sqrt(A)*sqrt(B), AB/den,
// Math.min over rows, NaN when no row qualifies, normalizeWeightResult).
//
// Exactness: counters are split into 7-bit limbs (c = sum_k c_k 128^k), so
// every product is an int8 x int8 MFMA with exact i32 accumulation
// (127^2 * 32768 < 2^31).  Owners whose counters all fit one limb (almost
// every owner of a Zipf stream) need one v_mfma_i32_32x32x32_i8 pass; tiles
// touching multi-limb owners run the MULTI variant, which folds each limb
// pair into an exact int64 dot.  The integer dot converted to double equals
// the reference's fp64 valueAB whenever the norms are < 2^53, and the
// epilogue performs the same correctly rounded IEEE operations as Java, so
// the similarities are bit-identical.
//
// Tile: 128 x 128 outputs per 256-thread workgroup (2 x 2 waves, each 64 x 64
// = 2 x 2 MFMA 32x32 tiles), K staged 128 bytes per row per stage through a
// double-buffered, XOR-swizzled LDS image (conflict-free ds_read_b128).
#include <hip/hip_fp16.h>
#include <hip/hip_runtime.h>

#include <algorithm>
#include <type_traits>
#include <cfloat>
#include <cstdlib>
#include <vector>

#include "cms_device.h"
#include "cms_internal.h"
#include "cms_mfma.h"

namespace cms {

constexpr int kTile = 128;      // output rows/cols per workgroup
constexpr int kBK = 128;        // K bytes per stage
constexpr int kMaxLimbs = 5;    // 35 bits >= any u32 counter
constexpr uint32_t kF4Max = 4;  // owners whose counters are all <= this also get an fp4 (e2m1) image

// ------------------------------------------------------------ preparation --

// Per owner row: limb count (from the largest counter, which the norm
// passes record), multi-limb flags (L > 1, L > 2), inexact-norm count and
// the count of owners needing all 5 limbs.
__global__ __launch_bounds__(256) void k_limb_count(const uint32_t* rowmax, int64_t nrows, const uint64_t* norm,
                                                    int depth, int fp4_ok, uint8_t* rowL, uint32_t* multi_flag,
                                                    uint32_t* deep_flag, uint32_t* f4_flag, uint32_t* inexact_rows) {
  const int64_t row = blockIdx.x * (int64_t)blockDim.x + threadIdx.x;
  if (row >= nrows) return;
  const uint32_t mx = rowmax[row];
  int L = 1;
  while (L < kMaxLimbs && (mx >> (7 * L)) != 0) ++L;
  rowL[row] = (uint8_t)L;
  multi_flag[row] = L > 1 ? 1u : 0u;
  deep_flag[row] = L > 2 ? 1u : 0u;
  f4_flag[row] = (fp4_ok && mx <= kF4Max) ? 1u : 0u;
  if (L == kMaxLimbs) atomicAdd(inexact_rows + 1, 1u);
  bool inexact = false;
  for (int d = 0; d < depth; ++d) inexact |= norm[row * depth + d] >= (1ULL << 53);
  if (inexact) atomicAdd(inexact_rows, 1u);
}

// Stable permutation: owners with 3+ limbs, then 2 limbs, then single-limb
// owners with a counter above kF4Max, then the fp4 class (every counter
// <= kF4Max), each class in row order (exclusive scans of the class flags).
// For an incremental refresh (tpos non-null) the touched owners of every
// class come first within their class, so the touched rows are four position
// ranges: whole symmetric-wave blocks of untouched single-limb rows can be
// skipped, and untouched multi-limb rows need only their touched columns.
// tpos: [0] int8, [1] fp4, [2] 3+ limbs, [3] 2 limbs (exclusive scans of the
// touched flags, n each); nt: their totals.
__global__ void k_limb_perm(const uint32_t* mpos, const uint32_t* multi_flag, const uint32_t* dpos,
                            const uint32_t* deep_flag, const uint32_t* fpos, const uint32_t* f4_flag,
                            const uint8_t* rowL, int64_t nrows, int64_t n_deep, int64_t n_multi, int64_t n_s8,
                            const uint8_t* touch, const uint32_t* tpos, int64_t nt8, int64_t nt4, int64_t ntd,
                            int64_t ntm, int64_t* perm, int64_t* inv, uint8_t* rowLp) {
  // rank q within a class of nt touched owners, touched first
  auto place = [&](int64_t r, int64_t q, const uint32_t* tp, int64_t nt) {
    return !tpos ? q : touch[r] ? (int64_t)tp[r] : nt + q - (int64_t)tp[r];
  };
  const uint32_t* tpos8 = tpos;
  const uint32_t* tpos4 = tpos ? tpos + nrows : nullptr;
  const uint32_t* tposd = tpos ? tpos + 2 * nrows : nullptr;
  const uint32_t* tposm = tpos ? tpos + 3 * nrows : nullptr;
  for (int64_t r = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; r < nrows; r += (int64_t)gridDim.x * blockDim.x) {
    int64_t p;
    if (deep_flag[r]) {
      p = place(r, (int64_t)dpos[r], tposd, ntd);
    } else if (multi_flag[r]) {
      p = n_deep + place(r, (int64_t)mpos[r] - (int64_t)dpos[r], tposm, ntm);
    } else if (f4_flag[r]) {
      p = n_multi + n_s8 + place(r, (int64_t)fpos[r], tpos4, nt4);  // rank in the fp4 class
    } else {
      p = n_multi + place(r, r - (int64_t)mpos[r] - (int64_t)fpos[r], tpos8, nt8);  // rank in the int8 class
    }
    perm[p] = r;
    inv[r] = p;
    rowLp[p] = rowL[r];
  }
}

// refresh: touched flags per class, [0] int8, [1] fp4, [2] 3+ limbs, [3] 2 limbs (n each)
__global__ void k_touch_class(const uint8_t* touch, const uint32_t* multi_flag, const uint32_t* deep_flag,
                              const uint32_t* f4_flag, int64_t n, uint32_t* tf) {
  for (int64_t r = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; r < n; r += (int64_t)gridDim.x * blockDim.x) {
    const bool t = touch[r] != 0, m = multi_flag[r] != 0, dp = deep_flag[r] != 0, f = f4_flag[r] != 0;
    tf[r] = (t && !m && !f) ? 1u : 0u;
    tf[n + r] = (t && !m && f) ? 1u : 0u;
    tf[2 * n + r] = (t && dp) ? 1u : 0u;
    tf[3 * n + r] = (t && m && !dp) ? 1u : 0u;
  }
}

// Limb images in permuted order: limb0[p] = c & 127 for every owner;
// hl[p][k-1] = (c >> 7k) & 127 for the multi-limb prefix p < n_multi.
// A list row (kFormList) is expanded one sketch row at a time: its entries
// are counted into w u8 counters (a list row's counters are < 2^8, four per
// LDS word, no carry), which then leave like any other row's.  Returns after
// fn(r, lc) ran for every sketch row r with the row's counters in lc.
template <class F>
__device__ __forceinline__ void expand_list_rows(const TableView& tv, int64_t row, int64_t dw, uint32_t* lc, F fn) {
  const uint32_t m = tv.list_m(row);
  const int w = tv.w, wq = w >> 2;
  for (int64_t r = 0; r * w < dw; ++r) {
    for (int j = threadIdx.x; j < wq; j += blockDim.x) lc[j] = 0u;
    __syncthreads();
    const uint16_t* e = tv.list_row(row, r, m);
    for (uint32_t t = threadIdx.x; t < m; t += blockDim.x) atomicAdd(&lc[e[t] >> 2], 1u << ((e[t] & 3u) * 8u));
    __syncthreads();
    fn(r, lc);
    __syncthreads();
  }
}

__global__ __launch_bounds__(256) void k_limb_write(TableView tv, int64_t dw, const int64_t* perm,
                                                    const uint8_t* rowLp, int64_t n_multi, int8_t* limb0, int8_t* hl) {
  extern __shared__ uint32_t lc[];  // [w / 4]: a list row's sketch row as u8 counters
  const int64_t p = blockIdx.x;
  const int64_t row = perm[p];
  int8_t* dst = limb0 + p * dw;
  const int L = p < n_multi ? rowLp[p] : 1;
  if (tv.hidx[row] == kFormList) {  // counters < 2^8: limb 0 = c & 127, limb 1 = c >> 7
    expand_list_rows(tv, row, dw, lc, [&](int64_t r, const uint32_t* c4) {
      for (int j = threadIdx.x; j < (tv.w >> 2); j += blockDim.x) {
        const uint32_t v = c4[j];
        const int64_t o = r * tv.w + 4 * j;
        *reinterpret_cast<uint32_t*>(dst + o) = v & 0x7F7F7F7Fu;
        if (L > 1) *reinterpret_cast<uint32_t*>(hl + p * (kMaxLimbs - 1) * dw + o) = (v >> 7) & 0x01010101u;
      }
    });
    return;
  }
  for (int64_t j = threadIdx.x * 4; j < dw; j += 256 * 4) {
    const uint4 v = tv.get4(row, j);
    *reinterpret_cast<char4*>(dst + j) = make_char4((signed char)(v.x & 127u), (signed char)(v.y & 127u),
                                                    (signed char)(v.z & 127u), (signed char)(v.w & 127u));
    for (int k = 1; k < L; ++k) {
      const int sh = 7 * k;
      *reinterpret_cast<char4*>(hl + (p * (kMaxLimbs - 1) + (k - 1)) * dw + j) =
          make_char4((signed char)((v.x >> sh) & 127u), (signed char)((v.y >> sh) & 127u),
                     (signed char)((v.z >> sh) & 127u), (signed char)((v.w >> sh) & 127u));
    }
  }
}

// fp4 (e2m1) image of positions [f0, n): two counters per byte, low nibble
// first.  Every counter is <= kF4Max, and 0..4 are exact e2m1 codes.
//
__global__ __launch_bounds__(256) void k_f4_write(TableView tv, int64_t dw, const int64_t* perm, int64_t f0,
                                                  uint8_t* f4, int sw) {
  extern __shared__ uint32_t lc[];  // [w / 4]: a list row's sketch row as u8 counters
  const int64_t p = f0 + blockIdx.x;
  const int64_t row = perm[p];
  const int64_t rs = dw / 2;
  // e2m1: 0 -> 0x0, 1 -> 0x2 (1.0), 2 -> 0x4 (2.0), 3 -> 0x5 (3.0), 4 -> 0x6 (4.0)
  constexpr uint32_t kCode = 0x65420u;  // nibble c = code of value c
  if (tv.hidx[row] == kFormList) {
    expand_list_rows(tv, row, dw, lc, [&](int64_t r, const uint32_t* c4) {
      for (int j = threadIdx.x; j < (tv.w >> 3); j += blockDim.x) {
        const uint32_t lo = c4[2 * j], hi = c4[2 * j + 1];
        uint32_t packed = 0;
#pragma unroll
        for (int q = 0; q < 8; ++q) packed |= ((kCode >> (4 * (((q < 4 ? lo : hi) >> (8 * (q & 3))) & 255u))) & 15u) << (4 * q);
        *reinterpret_cast<uint32_t*>(f4 + blk_off(blockIdx.x, (r * tv.w + 8 * j) / 2, rs, sw)) = packed;
      }
    });
    return;
  }
  for (int64_t j = threadIdx.x * 8; j < dw; j += 256 * 8) {
    const uint4 v0 = tv.get4(row, j);
    const uint4 v1 = tv.get4(row, j + 4);
    auto code = [&](uint32_t c) { return (kCode >> (4 * c)) & 15u; };
    const uint32_t packed = code(v0.x) | code(v0.y) << 4 | code(v0.z) << 8 | code(v0.w) << 12 | code(v1.x) << 16 |
                            code(v1.y) << 20 | code(v1.z) << 24 | code(v1.w) << 28;
    *reinterpret_cast<uint32_t*>(f4 + blk_off(blockIdx.x, j / 2, rs, sw)) = packed;
  }
}

// int8 limb-0 image of positions [p0, p0 + rows) in the K-blocked layout of
// the fp4 image (blk_off): the symmetric int8 waves' operands, so a stage of
// a 128-row block is one contiguous 16 KiB run instead of 128 lines a row
// stride apart.  The last block's padding rows are zero.
__global__ __launch_bounds__(256) void k_i8blk_write(const int8_t* limb0, int64_t dw, int64_t p0, int64_t rows,
                                                     int8_t* img, int sw) {
  const int64_t r = blockIdx.x;  // image row (whole blocks: padding rows write zeros)
  const int8_t* src = r < rows ? limb0 + (p0 + r) * dw : nullptr;
  for (int64_t j = threadIdx.x * 16; j < dw; j += 256 * 16) {
    const int4 v = src ? *reinterpret_cast<const int4*>(src + j) : make_int4(0, 0, 0, 0);
    *reinterpret_cast<int4*>(img + blk_off(r, j, dw, sw)) = v;
  }
}

// sqrt norms in PERMUTED order, row-major by sketch row: nsq_t[r][p] =
// nsqrt[perm[p]][r], so a panel's norms are one contiguous run per row.
__global__ void k_perm_norms(const double* nsqrt, const int64_t* perm, int64_t n, int depth, double* nsq_t) {
  for (int64_t p = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; p < n; p += (int64_t)gridDim.x * blockDim.x) {
    const int64_t o = perm[p];
    for (int r = 0; r < depth; ++r) nsq_t[(int64_t)r * n + p] = nsqrt[o * depth + r];
  }
}

__global__ void k_tile_limbs(const uint8_t* rowL, int64_t nrows, uint8_t* tileL) {
  const int64_t t = blockIdx.x * (int64_t)blockDim.x + threadIdx.x;
  const int64_t r0 = t * kTile;
  if (r0 >= nrows) return;
  uint8_t m = 1;
  for (int64_t r = r0; r < min(nrows, r0 + kTile); ++r) m = max(m, rowL[r]);
  tileL[t] = m;
}

// ------------------------------------------------------------- the kernel --

__device__ __forceinline__ double java_min_d(double a, double b) {
  if (a != a) return a;
  if (a == 0.0 && b == 0.0 && signbit(b)) return b;
  return (a <= b) ? a : b;
}

// LDS image of one 128 x 128-byte operand tile: row-major rows of 128 B, the
// 16-B chunk index XOR-swizzled with (row >> 1) & 7 so that every
// ds_read_b128 lane group of the fragment reads hits 16 distinct slots.
__device__ __forceinline__ int lds_off(int row, int ch) { return row * kBK + ((ch ^ ((row >> 1) & 7)) << 4); }

// Operands live in PERMUTED order: multi-limb owners first (positions
// [0, n_multi)), then the single-limb ones, each group in row order, so the
// multi-limb tiles are the first ceil(n_multi/128) row/column tiles only.
struct CosArgs {
  const int8_t* limb0;      // [n][dw]   limb 0 of perm[p]
  const int8_t* hl;         // [n_multi][kMaxLimbs-1][dw]  limbs 1.. of perm[p]
  const int64_t* perm;      // [n] permuted position -> owner row
  const uint8_t* rowL;      // [n] limb count of perm[p]
  const uint8_t* tileL;     // [ceil(n/128)] max limb count of a permuted tile
  const double* nsqrt;      // [n][d] by owner row
  int64_t n_multi;
  int64_t n;
  int64_t dw;
  int32_t w;
  int32_t depth;
  int64_t q0;               // first query row of the slab
  int64_t qcount;           // slab rows
  int64_t ldo;              // slab row stride (= n)
  double* out;              // [qcount][ldo]
  int32_t weighted;
  int32_t tiles_x;          // column tiles
};

__device__ int8_t g_zero16[16];  // source of the zero rows (past n, missing limbs)
#ifdef CMS_SCREEN_PROBE  // bound analysis only: waves / workgroups with every pair screened out, per row boundary
__device__ unsigned long long g_probe[4][32][2];  // [fmt*2 + wg][row][any alive]
#endif

// One stage of one operand (128 rows x 128 B = 16 KiB) by direct global->LDS
// loads: wave v, instruction u fills the 1 KiB (8 rows) at block 4v+u; lane i
// lands at byte 16 i of it, i.e. row 8(4v+u) + i/8, slot i%8, so it fetches
// chunk (i%8) ^ swz(row) -- the XOR swizzle lives on the source address and
// the LDS image stays lane-linear (glds writes base + 16 * lane).
__device__ __forceinline__ void stage_glds(const CosArgs& a, int64_t row0, int limb, int64_t koff,
                                           unsigned char* buf) {
  const int lane = threadIdx.x & 63, wv = threadIdx.x >> 6;
#pragma unroll
  for (int u = 0; u < 4; ++u) {
    const int blk = wv * 4 + u;
    const int row = blk * 8 + (lane >> 3);
    const int ch = (lane & 7) ^ ((row >> 1) & 7);
    const int64_t grow = row0 + row;
    const int8_t* src = g_zero16;
    if (grow < a.n) {
      if (limb == 0) src = a.limb0 + grow * a.dw + koff + ch * 16;
      else if (grow < a.n_multi && a.rowL[grow] > limb)
        src = a.hl + (grow * (kMaxLimbs - 1) + (limb - 1)) * a.dw + koff + ch * 16;
    }
    __builtin_amdgcn_global_load_lds((const __attribute__((address_space(1))) void*)src,
                                     (__attribute__((address_space(3))) void*)(buf + blk * 1024), 16, 0, 0);
  }
}

// Single-limb operand stage through a per-tile buffer descriptor: SGPR base
// (the tile's first row), 32-bit lane offsets, K offset in soffset; rows past
// n fall outside num_records and land as zeros.
struct TileSrc {
  __amdgpu_buffer_rsrc_t rsrc;
  int32_t voff[4];
};

__device__ __forceinline__ TileSrc tile_src(const CosArgs& a, int64_t row0) {
  TileSrc t;
  const int64_t rows = max<int64_t>(0, min<int64_t>(kTile, a.n - row0));
  const int8_t* base = a.limb0 + row0 * a.dw;
  t.rsrc = __builtin_amdgcn_make_buffer_rsrc((void*)base, (short)0, (int)(rows * a.dw), 0x00020000);
  const int lane = threadIdx.x & 63, wv = threadIdx.x >> 6;
#pragma unroll
  for (int u = 0; u < 4; ++u) {
    const int row = (wv * 4 + u) * 8 + (lane >> 3);
    const int ch = (lane & 7) ^ ((row >> 1) & 7);
    t.voff[u] = (int32_t)(row * a.dw) + ch * 16;
  }
  return t;
}

__device__ __forceinline__ void stage_buf(const TileSrc& t, int32_t koff, unsigned char* buf) {
  const int wv = threadIdx.x >> 6;
#pragma unroll
  for (int u = 0; u < 4; ++u)
    __builtin_amdgcn_raw_ptr_buffer_load_lds(t.rsrc, (__attribute__((address_space(3))) void*)(buf + (wv * 4 + u) * 1024),
                                             16, t.voff[u], koff, 0, 0);
}

template <bool MULTI>
__global__ __launch_bounds__(256, MULTI ? 1 : 2) void k_cosine_tile(CosArgs a, const int2* tile_list,
                                                                   int32_t tile_count) {
  extern __shared__ __align__(16) unsigned char lds[];  // [2 buffers][A 16K | B 16K] + sqrt norms
  double* s_sa = reinterpret_cast<double*>(lds + 4 * kTile * kBK);
  double* s_sb = s_sa + kTile;
  int64_t trow, tcol;
  if (tile_list) {
    if ((int)blockIdx.x >= tile_count) return;
    int2 t = tile_list[blockIdx.x];
    trow = t.y;
    tcol = t.x;
  } else {
    tcol = blockIdx.x;
    trow = blockIdx.y;
  }
  const int64_t row0 = a.q0 + trow * kTile;  // A rows (queries)
  const int64_t col0 = tcol * kTile;         // B rows (candidates)
  // an unaligned query start makes the row tile straddle two permuted tiles
  const int64_t tlast = min<int64_t>((row0 + kTile - 1) / kTile, a.tiles_x - 1);
  const int LA = MULTI ? max(a.tileL[row0 / kTile], a.tileL[tlast]) : 1;
  const int LB = MULTI ? a.tileL[col0 / kTile] : 1;
  if (!MULTI && !tile_list && (a.tileL[row0 / kTile] > 1 || a.tileL[col0 / kTile] > 1)) return;  // MULTI's job

  const int lane = threadIdx.x & 63, wid = threadIdx.x >> 6;
  const int wr = wid >> 1, wc = wid & 1;
  const int w = a.w;
  const int cstages = w / kBK;
  const int npairs = LA * LB;
  const int total = a.depth * npairs * cstages;

  i32x16 acc[2][2];
  int64_t dot[MULTI ? 2 : 1][MULTI ? 2 : 1][MULTI ? 16 : 1];
  double mn[2][2][16];
#pragma unroll
  for (int i = 0; i < 2; ++i)
#pragma unroll
    for (int j = 0; j < 2; ++j) {
#pragma unroll
      for (int e = 0; e < 16; ++e) {
        acc[i][j][e] = 0;
        mn[i][j][e] = DBL_MAX;
      }
    }
  if constexpr (MULTI) {
#pragma unroll
    for (int i = 0; i < 2; ++i)
#pragma unroll
      for (int j = 0; j < 2; ++j)
#pragma unroll
        for (int e = 0; e < 16; ++e) dot[i][j][e] = 0;
  }

  auto decode = [&](int s, int& r, int& la, int& lb, int& cs) {
    cs = s % cstages;
    int t = s / cstages;
    int p = t % npairs;
    r = t / npairs;
    la = p / LB;
    lb = p % LB;
  };

  TileSrc srcA, srcB;
  if constexpr (!MULTI) {
    srcA = tile_src(a, row0);
    srcB = tile_src(a, col0);
  }
  auto stage = [&](int s_, unsigned char* dstbuf) {
    int r_, la_, lb_, cs_;
    decode(s_, r_, la_, lb_, cs_);
    const int32_t koff = r_ * w + cs_ * kBK;
    if constexpr (MULTI) {
      stage_glds(a, row0, la_, koff, dstbuf);
      stage_glds(a, col0, lb_, koff, dstbuf + kTile * kBK);
    } else {
      stage_buf(srcA, koff, dstbuf);
      stage_buf(srcB, koff, dstbuf + kTile * kBK);
    }
  };
  stage(0, lds);
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  __syncthreads();

  for (int s = 0; s < total; ++s) {
    const int buf = s & 1;
    unsigned char* A = lds + buf * (2 * kTile * kBK);
    unsigned char* B = A + kTile * kBK;
    int r, la, lb, cs;
    decode(s, r, la, lb, cs);
    if (s + 1 < total) stage(s + 1, lds + (buf ^ 1) * (2 * kTile * kBK));  // prefetch into the free buffer
    // ---- 4 K-steps of 32 bytes, 2 x 2 MFMA tiles per wave ----
#pragma unroll
    for (int ks = 0; ks < 4; ++ks) {
      const int ch = 2 * ks + (lane >> 5);
      i8x16 fa[2], fb[2];
#pragma unroll
      for (int i = 0; i < 2; ++i) {
        const int row = wr * 64 + i * 32 + (lane & 31);
        fa[i] = *reinterpret_cast<const i8x16*>(A + lds_off(row, ch));
      }
#pragma unroll
      for (int j = 0; j < 2; ++j) {
        const int col = wc * 64 + j * 32 + (lane & 31);
        fb[j] = *reinterpret_cast<const i8x16*>(B + lds_off(col, ch));
      }
#pragma unroll
      for (int i = 0; i < 2; ++i)
#pragma unroll
        for (int j = 0; j < 2; ++j) acc[i][j] = __builtin_amdgcn_mfma_i32_32x32x32_i8(fa[i], fb[j], acc[i][j], 0, 0, 0);
    }
    const bool epilogue = cs == cstages - 1 && la == LA - 1 && lb == LB - 1;
    if (epilogue) {  // sqrt norms of this tile's rows/cols for sketch row r
      const int t = threadIdx.x & (kTile - 1);
      const int64_t g = (threadIdx.x < kTile ? row0 : col0) + t;
      const double v = g < a.n ? a.nsqrt[a.perm[g] * a.depth + r] : 0.0;
      (threadIdx.x < kTile ? s_sa : s_sb)[t] = v;
    }
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");  // stage s+1 landed (LDS-DMA counts on vmcnt)
    __syncthreads();

    if (cs == cstages - 1) {
      if constexpr (MULTI) {
        const int sh = 7 * (la + lb);
#pragma unroll
        for (int i = 0; i < 2; ++i)
#pragma unroll
          for (int j = 0; j < 2; ++j)
#pragma unroll
            for (int e = 0; e < 16; ++e) {
              dot[i][j][e] += (int64_t)acc[i][j][e] << sh;
              acc[i][j][e] = 0;
            }
      }
      if (la == LA - 1 && lb == LB - 1) {
        // ---- fp64 epilogue of sketch row r (DoubleCountMinSketch.java:143-147) ----
#pragma unroll
        for (int j = 0; j < 2; ++j) {
          const double sb = s_sb[wc * 64 + j * 32 + (lane & 31)];
#pragma unroll
          for (int i = 0; i < 2; ++i) {
#pragma unroll
            for (int e = 0; e < 16; ++e) {
              const double sa = s_sa[wr * 64 + i * 32 + (e & 3) + 8 * (e >> 2) + 4 * (lane >> 5)];
              double valueAB;
              if constexpr (MULTI) {
                valueAB = (double)dot[i][j][e];
                dot[i][j][e] = 0;
              } else {
                valueAB = (double)acc[i][j][e];
                acc[i][j][e] = 0;
              }
              const double den = __dmul_rn(sa, sb);
              if (den != 0.0) mn[i][j][e] = java_min_d(mn[i][j][e], __ddiv_rn(valueAB, den));
            }
          }
        }
      }
    }
  }

  // ---- write the slab: NaN when no row qualified, then normalizeWeightResult ----
#pragma unroll
  for (int i = 0; i < 2; ++i)
#pragma unroll
    for (int j = 0; j < 2; ++j) {
      const int64_t gcol = col0 + wc * 64 + j * 32 + (lane & 31);
#pragma unroll
      for (int e = 0; e < 16; ++e) {
        const int64_t grow = row0 + wr * 64 + i * 32 + (e & 3) + 8 * (e >> 2) + 4 * (lane >> 5);
        if (grow >= a.q0 + a.qcount || gcol >= a.n) continue;
        double rr = mn[i][j][e] == DBL_MAX ? __builtin_nan("") : mn[i][j][e];
        if (rr == rr) {
          if (a.weighted) rr = rr < 0.0 ? -1.0 : 1.0;  // scaleFactor 1 - 1/(0+1) = 0
          if (rr < -1.0) rr = -1.0;
          else if (rr > 1.0) rr = 1.0;
        }
        a.out[(grow - a.q0) * a.ldo + gcol] = rr;
      }
    }
}

// --------------------------------------------------------- 256 x 128 tile --
// 8 waves (4 x 2), each 64 x 64 MFMA outputs.  A = 256 operand rows, B = 128.
// NSTAGE-deep LDS ring of 48 KiB stages filled by buffer LDS-DMA; a raw
// s_barrier behind a counted vmcnt keeps the next stage in flight across it.
// The workgroups an XCD runs at once share one A panel (XCD-aware map).
//
// LS = limb slots per A owner.  LS = 1: A rows are owners (single-limb
// limb0 image).  LS = 2 / 4: A rows are the "virtual limb rows" of the
// multi-limb owners (ws_vl): within each 32-row MFMA block, row 8g + i holds
// limb g % LS of owner (g / LS) * 8 + i, so the LS limbs of an owner land in
// accumulator elements e, e+4, ... of ONE lane and fold exactly in registers
// (dot = sum_l acc_l << 7l) -- multi-limb x single-limb costs LS passes of
// A rows instead of a separate int64 kernel.  TRANS writes the transposed
// slab entries (query = B row), which is how single-limb queries meet
// multi-limb candidates: cosine(a, b) == cosine(b, a) bit for bit.
constexpr int kTA = 256, kTB = 128;

struct BigArgs {
  const int8_t* A;      // operand rows (limb0 image or ws_vl), first row of this launch
  int64_t a_vrows;      // operand rows available from A
  int64_t a_pos0;       // permuted position of A's first owner
  int64_t a_owners;     // owners covered from a_pos0
  const int8_t* B;      // candidate rows (limb0 image)
  int64_t b_pos0;       // permuted position of B's first row
  int64_t b_rows;       // candidates covered
  const int64_t* perm;  // permuted position -> owner row
  const double* nsq_t;  // [d][n] sqrt norms by PERMUTED position (row stride n)
  int64_t n;
  double* out;          // slab [qcount][ldo]
  int64_t ldo;
  int64_t q0, qcount;   // slab rows = permuted positions [q0, q0 + qcount)
  int64_t dw;
  int32_t w, depth;
  int32_t weighted, trans;
  int32_t tilesB, nblk;
  int32_t mode;  // CMS_BOUND_ANALYSIS builds only: bit0 skip loads, bit1 skip MFMA, bit2 skip epilogue
  // ---- candidate (streaming top-k) mode: cval != nullptr ----
  // Instead of the slab, every similarity v of a pair (a, b) is offered to
  // row a's candidate list when append_a and v >= thr[a], and to row b's when
  // append_b and v >= thr[b] (NaN never).  Lists hold (position, v).
  const double* thr;    // [n] per-position admission threshold (-inf: admit all)
  uint32_t* ccnt;       // [n] list lengths
  uint32_t* cidx;       // [n][cap] partner positions
  double* cval;         // [n][cap] similarities
  int32_t cap, append_a, append_b;
  // ---- symmetric wave: unordered 256-row block pairs {I, (I + wave) % nb} ----
  int32_t sym, wave, nb;  // sym: block I = positions [s0 + 256 I, ...) of the s_rows region
  int32_t band;           // sym: waves [wave, wave + band) in one launch
  int64_t s0, s_rows;
  // operand images: row stride rs bytes, kw bytes per sketch row (i8: dw, w;
  // fp4: dw/2, w/2); sym mode reads rows at (position - img0) * rs
  int64_t rs, img0;
  int32_t kw;
  // sym, fsel != 0: only the block pairs with a block below fblk0 (grid of
  // 2 * fblk0 block slots instead of nb)
  int32_t fblk0, fsel;
  // sym, rect != 0: the band's (I, J) pairs enumerated by si x sj rectangles
  // of blocks (njc J-chunks per I-block), so the ~32 workgroups an XCD runs
  // together share si A panels and sj B blocks instead of 1 and 16-32
  int32_t rect, si, sj, njc;
  int32_t noscreen;  // 1: exact epilogue for every pair (A/B of the screening)
  int32_t blk;       // int8 operands from a K-blocked image (k_i8blk_write); fp4 images always are
};

template <int NSTAGE, int LS, int BK, int FMT = 0>
__global__ __launch_bounds__(512, 1) void k_cosine_big(BigArgs g) {
  static_assert(BK == 128 || BK == 64, "stage depth");
  static_assert(FMT == 0 || LS == 1, "fp4 operands are single-limb owners");
  using AccT = typename AccOf<FMT>::type;
  constexpr int OA = kTA / LS;  // owners per A panel
  constexpr int OG = 4 / LS;    // owner groups per 32-row block in one lane
  constexpr int kStageA = kTA * BK, kStageB = kTB * BK, kStage = kStageA + kStageB;
  constexpr int RPI = 1024 / BK;            // rows per 1-KiB LDS-DMA instruction
  constexpr int OPA = kTA / RPI / 8;        // A instructions per wave per stage
  constexpr int OPB = kTB / RPI / 8;        // B instructions per wave per stage
  constexpr int OPS = OPA + OPB;
  extern __shared__ __align__(16) unsigned char lds[];
  const int depth = g.depth;
  double* s_sa = reinterpret_cast<double*>(lds + NSTAGE * kStage);  // [depth][256] (OA used)
  double* s_sb = s_sa + depth * kTA;                                 // [depth][128]
  // candidate mode: the panels' admission thresholds as fp16 rounded toward
  // -inf ([256] A owners, [128] B rows), for the fp32 screening epilogue
  __half* s_ta = reinterpret_cast<__half*>(s_sb + depth * kTB);
  __half* s_tb = s_ta + kTA;
  const int nblk = g.nblk;
  const int bx = blockIdx.x, xcd = bx & 7, q8 = nblk >> 3, r8 = nblk & 7;
  const int lin = (xcd < r8 ? xcd * (q8 + 1) : r8 * (q8 + 1) + (xcd - r8) * q8) + (bx >> 3);
  const int8_t* gA = g.A;
  const int8_t* gB = g.B;
  int64_t a_pos0 = g.a_pos0, a_owners = g.a_owners, a_vrows = g.a_vrows, b_pos0 = g.b_pos0, b_rows = g.b_rows;
  int64_t vrow0, own0, bcol0;
  bool diag = false;  // symmetric diagonal block: only pairs a < b
  if (g.sym) {
    // A band of waves: block I meets J = I + wave + t (t < band), both
    // 128-column halves.  Consecutive workgroups share I (its panel stays in
    // the XCD's L2 for 2*band workgroups) and neighbouring I share most J.
    int c, half, wv;
    if (g.rect) {
      const int per = 2 * g.si * g.sj;
      const int blk = lin / per, loc = lin - blk * per;
      const int ib = blk / g.njc, jc = blk - ib * g.njc;
      half = loc & 1;
      const int li = (loc >> 1) / g.sj, lj = (loc >> 1) - li * g.sj;
      c = ib * g.si + li;
      if (c >= g.nb) return;
      wv = ib * g.si + g.wave + jc * g.sj + lj - c;  // unwrapped J' - I
      if (wv < g.wave || wv >= g.wave + g.band) return;
    } else {
      const int per = 2 * g.band;
      c = lin / per;
      const int rem = lin - c * per;
      half = rem & 1;
      wv = g.wave + (rem >> 1);
    }
    int I = c;
    if (g.fsel) {
      // only the pairs with a block below fblk0: c < fblk0 is that block as I,
      // c >= fblk0 enumerates J = c - fblk0 < fblk0 with I >= fblk0
      if (c >= g.fblk0) {
        I = ((c - g.fblk0 - wv) % g.nb + g.nb) % g.nb;
        if (I < g.fblk0) return;  // already the first run's pair
      }
    }
    if ((g.nb & 1) == 0 && 2 * wv == g.nb && 2 * I >= g.nb) return;  // {I, I + nb/2} once
    const int J = (I + wv) % g.nb;
    diag = I == J;
    a_pos0 = g.s0 + (int64_t)I * kTA;
    a_owners = a_vrows = min<int64_t>(kTA, g.s_rows - (int64_t)I * kTA);
    b_pos0 = g.s0 + (int64_t)J * kTA + half * kTB;
    b_rows = min<int64_t>(kTB, g.s_rows - (int64_t)J * kTA - half * kTB);
    if (b_rows <= 0) return;  // the whole workgroup leaves before any barrier
    gA = g.A + (a_pos0 - g.img0) * g.rs;
    gB = g.B + (b_pos0 - g.img0) * g.rs;
    vrow0 = own0 = bcol0 = 0;
  } else {
    // A panel fastest: an XCD's co-resident workgroups cover a few candidate
    // tiles x every query panel, so both operands mostly hit the XCD's L2 and
    // each candidate tile leaves HBM once per launch.
    const int tilesA = g.nblk / g.tilesB;
    const int ta = lin % tilesA, tb = lin / tilesA;
    vrow0 = (int64_t)ta * kTA;  // first operand row of the A panel
    own0 = (int64_t)ta * OA;    // first owner (relative to a_pos0)
    bcol0 = (int64_t)tb * kTB;
  }

  const int tid = threadIdx.x, lane = tid & 63, wid = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int wr = wid >> 1, wc = wid & 1;
  const int kw = g.kw;  // bytes per sketch row in the operand image
  const int64_t rs = g.rs;
  const int cstages = kw / BK;
#ifdef CMS_BOUND_ANALYSIS
  const int kMode = g.mode;  // bit0 skip loads, bit1 skip MFMA, bit2 skip epilogue
#else
  constexpr int kMode = 0;
#endif
  const int total = depth * cstages;

  // sqrt norms of the panel's owners, straight into LDS by LDS-DMA (256 B
  // per instruction, past-the-end owners land as zeros).  Issued before the
  // first stages, so the stage-0 vmcnt wait covers them, and the first
  // epilogue runs behind at least one barrier.
  for (int k = wid; k < 12 * depth; k += 8) {
    const int r = k / 12, part = k % 12;  // parts 0..7: A (8 x 32 owners), 8..11: B (4 x 32)
    const bool isA = part < 8;
    const int64_t first = isA ? own0 + part * 32 : bcol0 + (part - 8) * 32;
    const int64_t lim = isA ? min<int64_t>(a_owners, own0 + OA) : b_rows;
    const int64_t cnt = max<int64_t>(0, min<int64_t>(32, lim - first));
    const double* src = g.nsq_t + (int64_t)r * g.n + (isA ? a_pos0 : b_pos0) + first;
    const __amdgpu_buffer_rsrc_t rs =
        __builtin_amdgcn_make_buffer_rsrc((void*)src, (short)0, (int)(cnt * 8), 0x00020000);
    double* dst = isA ? s_sa + r * kTA + part * 32 : s_sb + r * kTB + (part - 8) * 32;
    __builtin_amdgcn_raw_ptr_buffer_load_lds(rs, (__attribute__((address_space(3))) void*)dst, 4, lane * 4, 0, 0, 0);
  }

  // Screening (candidate mode, unweighted, single-limb): once a pair's fp32
  // estimate of one row cosine is below both owners' thresholds by more than
  // its error bound, min over rows can only be lower, so the pair can never
  // be admitted and its exact fp64 epilogue is skipped; a wave runs the exact
  // epilogue only while one of its pairs is still alive.
  const bool screen = g.cval != nullptr && !g.weighted && LS == 1 && !g.noscreen;
  if (screen) {
    for (int i = tid; i < kTA + kTB; i += 512) {
      const bool isA = i < kTA;
      const int64_t o = isA ? own0 + i : bcol0 + (i - kTA);
      const int64_t lim = isA ? a_owners : b_rows;
      const double t = o < lim ? g.thr[(isA ? a_pos0 : b_pos0) + o] : __builtin_inf();
      (isA ? s_ta : s_tb - kTA)[i] = __float2half_rd(__double2float_rd(t));  // never above the threshold
    }
  }

  // buffer descriptors bound the panel: rows past the end land as zeros.
  // fp4 operands use the K-blocked image (k_f4_write; sym panels start on a
  // block): a panel's rows past the end inside its last block are the
  // image's zero padding, the rows beyond that block fall outside the bound.
  const bool BLK = FMT == 1 || g.blk != 0;
  const int64_t rowsA = max<int64_t>(0, min<int64_t>(kTA, a_vrows - vrow0));
  const int64_t rowsB = max<int64_t>(0, min<int64_t>(kTB, b_rows - bcol0));
  const int64_t recA = BLK ? (rowsA + kImgBlk - 1) / kImgBlk * kImgBlk * rs : rowsA * rs;
  const int64_t recB = BLK ? (rowsB + kImgBlk - 1) / kImgBlk * kImgBlk * rs : rowsB * rs;
  const __amdgpu_buffer_rsrc_t rsA =
      __builtin_amdgcn_make_buffer_rsrc((void*)(gA + vrow0 * rs), (short)0, (int)recA, 0x00020000);
  const __amdgpu_buffer_rsrc_t rsB =
      __builtin_amdgcn_make_buffer_rsrc((void*)(gB + bcol0 * rs), (short)0, (int)recB, 0x00020000);
  // Instruction u of wave wid fills LDS rows [(wid + 8u) * RPI, +RPI); lane
  // i lands at byte 16 i, i.e. row (wid + 8u) * RPI + i / (BK/16), slot
  // i % (BK/16), and fetches the chunk the swizzle puts there.  The 8*RPI-row
  // step leaves the swizzle unchanged, so one voffset per lane serves every
  // instruction and the row step is a constant add.
  constexpr int CPR = BK / 16;  // 16-B chunks per row
  const int srow = wid * RPI + lane / CPR;
  const int slot = lane % CPR;
  const int32_t chunk = (BK == 128 ? (slot ^ ((srow >> 1) & 7)) : (slot ^ ((srow >> 2) & 3))) << 4;
  // row-major image: row r at r * rs; K-blocked image (BLK, slices of BK
  // bytes): row r at (r / 128) * 128 * rs + (r % 128) * BK, K slice s at
  // s * 128 * BK; instruction u's rows start at 8 u RPI (block, row in block)
  const int32_t rstep = 8 * RPI * (int32_t)rs;
  const int32_t bstep = kImgBlk * (int32_t)rs;
  const int32_t vo = BLK ? (srow / kImgBlk) * bstep + (srow % kImgBlk) * BK + chunk : (int32_t)(srow * rs) + chunk;
#define UOFF(u) \
  (BLK ? vo + ((8 * (u) * RPI) / kImgBlk) * bstep + ((8 * (u) * RPI) % kImgBlk) * BK : vo + (u) * rstep)
  auto issue = [&](int s) {
    if (kMode & 1) return;
    const int r = s / cstages, cs = s - r * cstages;
    const int32_t koff = BLK ? s * (kImgBlk * BK) : r * kw + cs * BK;
    unsigned char* st = lds + (s % NSTAGE) * kStage;
#pragma unroll
    for (int u = 0; u < OPA; ++u)
      __builtin_amdgcn_raw_ptr_buffer_load_lds(rsA, (__attribute__((address_space(3))) void*)(st + (wid + 8 * u) * 1024),
                                               16, UOFF(u), koff, 0, 0);
#pragma unroll
    for (int u = 0; u < OPB; ++u)
      __builtin_amdgcn_raw_ptr_buffer_load_lds(
          rsB, (__attribute__((address_space(3))) void*)(st + kStageA + (wid + 8 * u) * 1024), 16, UOFF(u),
          koff, 0, 0);
  };
#undef UOFF

  AccT acc[2][2];
  // running Math.min of each pair.  Single-limb rows keep the fp64 value.
  // Multi-limb rows keep (exact dot << 5 | sketch row) of the row holding it
  // (k_cosine_sym's packed state, 64-bit: dots < 2^53): rows are compared by
  // fp32 estimates, exactly only inside a 2^-17 margin, and the value is
  // divided out once, exactly, at the end.
  constexpr bool kPacked = LS > 1;
  using StT = typename std::conditional<kPacked, uint64_t, double>::type;
  constexpr StT kEmptySt = kPacked ? (StT)~0ULL : (StT)DBL_MAX;
  StT mn[2][2][4 * OG];
  uint64_t alive = ~0ULL;  // bit (i*2+j)*16 + og*4 + q: the pair may still be admitted
#pragma unroll
  for (int i = 0; i < 2; ++i)
#pragma unroll
    for (int j = 0; j < 2; ++j) {
#pragma unroll
      for (int e = 0; e < 16; ++e) acc[i][j][e] = 0;
#pragma unroll
      for (int e = 0; e < 4 * OG; ++e) mn[i][j][e] = kEmptySt;
    }

#pragma unroll
  for (int s = 0; s < NSTAGE - 1; ++s)
    if (s < total) issue(s);

  for (int s = 0; s < total; ++s) {
    // stage s landed: at most the (NSTAGE-2) younger stages (OPS ops each) stay in flight
    asm volatile("" ::: "memory");
    if (s + NSTAGE - 2 < total) wait_vmcnt<OPS * (NSTAGE - 2)>();
    else wait_vmcnt<0>();
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
    __builtin_amdgcn_s_barrier();
    asm volatile("" ::: "memory");
    if (s + NSTAGE - 1 < total) issue(s + NSTAGE - 1);  // refill the slot read in iteration s-1
    const unsigned char* A = lds + (s % NSTAGE) * kStage;
    const unsigned char* B = A + kStageA;
#pragma unroll
    for (int ks = 0; ks < BK / 32; ++ks) {
      if (kMode & 2) break;
      const int ch = 2 * ks + (lane >> 5);
      i8x16 fa[2], fb[2];
#pragma unroll
      for (int i = 0; i < 2; ++i)
        fa[i] = *reinterpret_cast<const i8x16*>(A + lds_off_bk<BK>(wr * 64 + i * 32 + (lane & 31), ch));
#pragma unroll
      for (int j = 0; j < 2; ++j)
        fb[j] = *reinterpret_cast<const i8x16*>(B + lds_off_bk<BK>(wc * 64 + j * 32 + (lane & 31), ch));
#pragma unroll
      for (int i = 0; i < 2; ++i)
#pragma unroll
        for (int j = 0; j < 2; ++j) acc[i][j] = mfma_step<FMT>(fa[i], fb[j], acc[i][j]);
    }
    const int r = s / cstages;
    if (s - r * cstages == cstages - 1 && !(kMode & 4)) {
      // ---- fp64 epilogue of sketch row r (DoubleCountMinSketch.java:143-147) ----
      // Branch-free: every term is AB / (sqrtA * sqrtB) with AB >= 0 and a
      // finite den, so no NaN or -0.0 reaches Math.min and it is a plain
      // "smaller wins"; den == 0 rows are masked out.  Each sqrtA serves
      // both column fragments.
      double sb[2];
#pragma unroll
      for (int j = 0; j < 2; ++j) sb[j] = s_sb[r * kTB + wc * 64 + j * 32 + (lane & 31)];
      if (screen) {
        // fp32 estimate AB / (sa * sb): relative error < 2^-20 (exact AB < 2^27
        // and two conversions, one v_rcp_f32 (1 ulp) and two products)
        float rb[2], tb[2];
#pragma unroll
        for (int j = 0; j < 2; ++j) {
          rb[j] = __builtin_amdgcn_rcpf((float)sb[j]);
          tb[j] = __half2float(s_tb[wc * 64 + j * 32 + (lane & 31)]);
        }
#pragma unroll
        for (int i = 0; i < 2; ++i)
#pragma unroll
          for (int og = 0; og < OG; ++og)
#pragma unroll
            for (int q = 0; q < 4; ++q) {
              const int ol = (wr * 64 + i * 32) / LS + og * 8 + q + 4 * (lane >> 5);
              const float sa = (float)s_sa[r * kTA + ol];
              const float ra = __builtin_amdgcn_rcpf(sa);
              const float ta = __half2float(s_ta[ol]);
#pragma unroll
              for (int j = 0; j < 2; ++j) {
                const int bit = (i * 2 + j) * 16 + og * 4 + q;
                const float est = (float)acc[i][j][q + 4 * og] * ra * rb[j];
                const bool dead = sa != 0.0f && (float)sb[j] != 0.0f && est < fminf(ta, tb[j]) - 4e-6f;
                if (dead) alive &= ~(1ULL << bit);
              }
            }
      }
#ifdef CMS_SCREEN_PROBE
      if (screen) {
        __shared__ int s_probe[32];
        const bool wa = __any(alive != 0ULL);
        if (lane == 0) atomicAdd(&g_probe[FMT * 2][r][wa ? 1 : 0], 1ull);
        if (tid < 32 && s - r * cstages == cstages - 1 && r == 0) s_probe[tid] = 0;
        __syncthreads();
        if (lane == 0 && wa) atomicOr(&s_probe[r], 1);
        __syncthreads();
        if (tid == 0) atomicAdd(&g_probe[FMT * 2 + 1][r][s_probe[r] ? 1 : 0], 1ull);
      }
#endif
      if (!screen || __any(alive != 0ULL)) {
#pragma unroll
      for (int i = 0; i < 2; ++i) {
#pragma unroll
        for (int og = 0; og < OG; ++og)
#pragma unroll
          for (int q = 0; q < 4; ++q) {
            const int ol = (wr * 64 + i * 32) / LS + og * 8 + q + 4 * (lane >> 5);
            const double sa = s_sa[r * kTA + ol];
            if constexpr (!kPacked) {
#pragma unroll
              for (int j = 0; j < 2; ++j) {
                if (screen && !((alive >> ((i * 2 + j) * 16 + og * 4 + q)) & 1ULL)) continue;
                const double den = __dmul_rn(sa, sb[j]);
                const double v = __ddiv_rn((double)acc[i][j][q + 4 * og], den);
                StT& m = mn[i][j][og * 4 + q];
                m = (den != 0.0 && v < m) ? v : m;
              }
            } else {
            if (sa == 0.0) continue;  // den == 0: this sketch row does not qualify
            const float ra = __builtin_amdgcn_rcpf((float)sa);
#pragma unroll
            for (int j = 0; j < 2; ++j) {
              if (screen && !((alive >> ((i * 2 + j) * 16 + og * 4 + q)) & 1ULL)) continue;
              if (sb[j] == 0.0) continue;
              int64_t dot = 0;
#pragma unroll
              for (int l = 0; l < LS; ++l) dot += (int64_t)acc[i][j][q + 4 * (og * LS + l)] << (7 * l);
              StT& m = mn[i][j][og * 4 + q];
              bool take = m == kEmptySt;
              if (!take) {
                const int col = wc * 64 + j * 32 + (lane & 31);
                const int r0 = (int)(m & 31ULL);
                const int64_t d0 = (int64_t)(m >> 5);
                const double sa0 = s_sa[r0 * kTA + ol], sb0 = s_sb[r0 * kTB + col];
                const float est = (float)dot * ra * __builtin_amdgcn_rcpf((float)sb[j]);
                const float est0 = (float)d0 * __builtin_amdgcn_rcpf((float)sa0) * __builtin_amdgcn_rcpf((float)sb0);
                if (est < est0 * (1.0f - 0x1p-17f)) {
                  take = true;
                } else if (est <= est0 * (1.0f + 0x1p-17f)) {  // too close for fp32: the exact values
                  take = __ddiv_rn((double)dot, __dmul_rn(sa, sb[j])) < __ddiv_rn((double)d0, __dmul_rn(sa0, sb0));
                }
              }
              if (take) m = ((uint64_t)dot << 5) | (uint64_t)r;
            }
            }
          }
      }
      }
#pragma unroll
      for (int i = 0; i < 2; ++i)
#pragma unroll
        for (int j = 0; j < 2; ++j)
#pragma unroll
          for (int e = 0; e < 16; ++e) acc[i][j][e] = 0;
    }
  }

  // ---- NaN when no row qualified, then normalizeWeightResult; slab or lists ----
#pragma unroll
  for (int i = 0; i < 2; ++i)
#pragma unroll
    for (int j = 0; j < 2; ++j) {
      const int64_t bi = bcol0 + wc * 64 + j * 32 + (lane & 31);
      const int64_t bp = b_pos0 + bi;
      const double tb_ = (g.cval && g.append_b && bi < b_rows) ? g.thr[bp] : 0.0;
#pragma unroll
      for (int og = 0; og < OG; ++og)
#pragma unroll
        for (int q = 0; q < 4; ++q) {
          const int64_t ai = own0 + (wr * 64 + i * 32) / LS + og * 8 + q + 4 * (lane >> 5);
          if (ai >= a_owners || bi >= b_rows) continue;
          if (screen && !((alive >> ((i * 2 + j) * 16 + og * 4 + q)) & 1ULL)) continue;  // never admitted
          const int64_t ap = a_pos0 + ai;
          const StT m = mn[i][j][og * 4 + q];
          double rr = __builtin_nan("");
          if constexpr (kPacked) {
            if (m != kEmptySt) {
              const int r0 = (int)(m & 31ULL);
              const int ol = (wr * 64 + i * 32) / LS + og * 8 + q + 4 * (lane >> 5);
              rr = __ddiv_rn((double)(int64_t)(m >> 5),
                             __dmul_rn(s_sa[r0 * kTA + ol], s_sb[r0 * kTB + wc * 64 + j * 32 + (lane & 31)]));
            }
          } else {
            rr = m == kEmptySt ? rr : m;
          }
          if (rr == rr) {
            if (g.weighted) rr = rr < 0.0 ? -1.0 : 1.0;  // scaleFactor 1 - 1/(0+1) = 0
            if (rr < -1.0) rr = -1.0;
            else if (rr > 1.0) rr = 1.0;
          }
          if (g.cval) {
            if (rr != rr || ap == bp || (diag && ap > bp)) continue;
            if (g.append_a && rr >= g.thr[ap]) {
              const uint32_t slot = atomicAdd(&g.ccnt[ap], 1u);
              if (slot < (uint32_t)g.cap) {
                g.cidx[ap * g.cap + slot] = (uint32_t)bp;
                g.cval[ap * g.cap + slot] = rr;
              }
            }
            if (g.append_b && rr >= tb_) {
              const uint32_t slot = atomicAdd(&g.ccnt[bp], 1u);
              if (slot < (uint32_t)g.cap) {
                g.cidx[bp * g.cap + slot] = (uint32_t)ap;
                g.cval[bp * g.cap + slot] = rr;
              }
            }
            continue;
          }
          const int64_t orow = g.trans ? bp : ap, ocol = g.trans ? ap : bp;
          if (orow < g.q0 || orow >= g.q0 + g.qcount) continue;
          g.out[(orow - g.q0) * g.ldo + ocol] = rr;
        }
    }
}

// Virtual limb rows of the multi-limb owners at positions [o0, o1) for the
// LS-slot layout above; missing limbs and the tail are zero rows.
__global__ __launch_bounds__(256) void k_vl_build(const int8_t* limb0, const int8_t* hl, const uint8_t* rowLp,
                                                  int64_t o0, int64_t o1, int64_t dw, int LS, int8_t* vl) {
  const int64_t v = blockIdx.x;
  const int rr = (int)(v & 31), grp = rr >> 3;
  const int limb = grp % LS;
  const int64_t o = o0 + (v >> 5) * (32 / LS) + (grp / LS) * 8 + (rr & 7);
  const int8_t* src = nullptr;
  if (o < o1) {
    if (limb == 0) src = limb0 + o * dw;
    else if (limb < rowLp[o]) src = hl + (o * (kMaxLimbs - 1) + (limb - 1)) * dw;
  }
  int4* dst = reinterpret_cast<int4*>(vl + v * dw);
  for (int64_t j = threadIdx.x; j < dw / 16; j += 256)
    dst[j] = src ? reinterpret_cast<const int4*>(src)[j] : make_int4(0, 0, 0, 0);
}

// ---------------------------------------------------------------- driver --

int cosine_prepare(cms_handle* h) {
  if (h->mfma_ready) return CMS_OK;
  const int64_t n = h->n, dw = h->dw;
  const int64_t ntiles = (n + kTile - 1) / kTile;
  CMS_HIP(h->ws_limb0.ensure((size_t)n * (size_t)dw));
  // meta: perm[n] i64 | inv[n] i64 | multi_flag[n] u32 | mpos[n] u32 | bsum | rowL[n] | rowLp[n] | tileL[ntiles]
  //       | deep_flag[n] u32 | dpos[n] u32 | f4_flag[n] u32 | fpos[n] u32
  const int64_t nbs = (n + 4095) / 4096 + 1;
  CMS_HIP(h->ws_limbmeta.ensure((size_t)n * (8 + 8 + 4 + 4 + 1 + 1 + 4 + 4 + 4 + 4) + 4 * (size_t)nbs +
                                (size_t)ntiles + 64));
  int64_t* perm = h->ws_limbmeta.as<int64_t>();
  int64_t* inv = perm + n;
  uint32_t* mflag = reinterpret_cast<uint32_t*>(inv + n);
  uint32_t* mpos = mflag + n;
  uint32_t* bsum = mpos + n;
  uint8_t* rowL = reinterpret_cast<uint8_t*>(bsum + nbs);
  uint8_t* rowLp = rowL + n;
  uint8_t* tileL = rowLp + n;
  uint32_t* dflag = reinterpret_cast<uint32_t*>((reinterpret_cast<uintptr_t>(tileL + ntiles) + 15) & ~uintptr_t(15));
  uint32_t* dpos = dflag + n;
  uint32_t* fflag = dpos + n;
  uint32_t* fpos = fflag + n;
  uint32_t* cnt = h->d_flags + 8;  // [8] inexact owners, [9] 5-limb owners
  CMS_HIP(hipMemsetAsync(cnt, 0, 2 * sizeof(uint32_t), h->stream));
  // fp4 operands need whole 128-B stages of packed counters (256 per stage)
  int fp4_ok = (h->p.width % 256) == 0 ? 1 : 0;
  // stage depth of the symmetric waves = K slice width of their blocked images
  h->sym_sw = sym_stage_bytes();
  if (!h->tune.fp4) fp4_ok = 0;
  uint32_t host[8];
  {
    TimedScope ts(h, "limb_prep");
    hipLaunchKernelGGL(k_limb_count, dim3((unsigned)((n + 255) / 256)), dim3(256), 0, h->stream, h->d_rowmax, n,
                       h->d_norm, h->p.depth, fp4_ok, rowL, mflag, dflag, fflag, cnt);
    int rc = scan_exclusive_u32(h, mflag, mpos, n, bsum);
    if (rc) return rc;
    CMS_HIP(hipMemcpyAsync(&host[0], mpos + n - 1, 4, hipMemcpyDeviceToHost, h->stream));
    CMS_HIP(hipMemcpyAsync(&host[1], mflag + n - 1, 4, hipMemcpyDeviceToHost, h->stream));
    rc = scan_exclusive_u32(h, dflag, dpos, n, bsum);
    if (rc) return rc;
    CMS_HIP(hipGetLastError());
    CMS_HIP(hipMemcpyAsync(&host[2], cnt, 8, hipMemcpyDeviceToHost, h->stream));
    CMS_HIP(hipMemcpyAsync(&host[4], dpos + n - 1, 4, hipMemcpyDeviceToHost, h->stream));
    CMS_HIP(hipMemcpyAsync(&host[5], dflag + n - 1, 4, hipMemcpyDeviceToHost, h->stream));
    rc = scan_exclusive_u32(h, fflag, fpos, n, bsum);
    if (rc) return rc;
    CMS_HIP(hipMemcpyAsync(&host[6], fpos + n - 1, 4, hipMemcpyDeviceToHost, h->stream));
    CMS_HIP(hipMemcpyAsync(&host[7], fflag + n - 1, 4, hipMemcpyDeviceToHost, h->stream));
    CMS_HIP(hipStreamSynchronize(h->stream));
  }
  const int64_t n_multi = (int64_t)host[0] + host[1];
  const int64_t n_deep = (int64_t)host[4] + host[5];
  const int64_t n_f4 = (int64_t)host[6] + host[7];
  const int64_t n_s8 = n - n_multi - n_f4;
  // fp4 image from the first 768-row block of the single-limb region that
  // holds fp4 owners only (symmetric-wave blocks start at n_multi)
  const int64_t f0 = std::min<int64_t>(n, n_multi + (n_s8 + kSymBlk - 1) / kSymBlk * kSymBlk);
  h->n_f4 = n_f4;
  h->f4_pos0 = f0;
  h->n_hot_limb = (uint32_t)n_multi;
  h->n_inexact_rows = host[2];
  const uint32_t n_five = host[3];
  CMS_HIP(h->ws_limbhot.ensure((size_t)std::max<int64_t>(1, n_multi) * (kMaxLimbs - 1) * (size_t)dw));
  // incremental refresh: touched owners first within their class
  const uint8_t* touch = nullptr;
  uint32_t* tpos = nullptr;
  int64_t nt[4] = {0, 0, 0, 0};  // touched int8, fp4, 3+ limb, 2-limb owners
  if (h->rf_restrict) {
    CMS_HIP(h->rf_perm.ensure(sizeof(uint32_t) * 8 * (size_t)n));
    uint32_t* tf = h->rf_perm.as<uint32_t>();
    tpos = tf + 4 * n;
    touch = h->rf_touch.as<uint8_t>();
    TimedScope ts(h, "limb_prep");
    const unsigned grid = (unsigned)std::min<int64_t>((n + 255) / 256, 4096);
    hipLaunchKernelGGL(k_touch_class, dim3(grid), dim3(256), 0, h->stream, touch, mflag, dflag, fflag, n, tf);
    CMS_HIP(hipGetLastError());
    uint32_t th[8];
    for (int c = 0; c < 4; ++c) {
      int rc = scan_exclusive_u32(h, tf + c * n, tpos + c * n, n, bsum);
      if (rc) return rc;
      CMS_HIP(hipMemcpyAsync(&th[2 * c], tpos + c * n + n - 1, 4, hipMemcpyDeviceToHost, h->stream));
      CMS_HIP(hipMemcpyAsync(&th[2 * c + 1], tf + c * n + n - 1, 4, hipMemcpyDeviceToHost, h->stream));
    }
    CMS_HIP(hipStreamSynchronize(h->stream));
    for (int c = 0; c < 4; ++c) nt[c] = (int64_t)th[2 * c] + th[2 * c + 1];
  }
  const int64_t nt8 = nt[0], nt4 = nt[1];
  h->rf_td = nt[2];
  h->rf_tm = nt[3];
  h->rf_nd = n_deep;
  h->rf_t8 = nt8;
  h->rf_t4 = nt4;
  h->rf_s8 = n_s8;
  {
    TimedScope ts(h, "limb_prep");
    unsigned grid = (unsigned)std::min<int64_t>((n + 255) / 256, 4096);
    hipLaunchKernelGGL(k_limb_perm, dim3(grid), dim3(256), 0, h->stream, mpos, mflag, dpos, dflag, fpos, fflag, rowL,
                       n, n_deep, n_multi, n_s8, touch, tpos, nt8, nt4, nt[2], nt[3], perm, inv, rowLp);
    hipLaunchKernelGGL(k_limb_write, dim3((unsigned)n), dim3(256), (size_t)h->p.width, h->stream, h->tview(), dw, perm, rowLp, n_multi,
                       h->ws_limb0.as<int8_t>(), h->ws_limbhot.as<int8_t>());
    hipLaunchKernelGGL(k_tile_limbs, dim3((unsigned)((ntiles + 255) / 256)), dim3(256), 0, h->stream, rowLp, n,
                       tileL);
    CMS_HIP(h->ws_nsq.ensure(sizeof(double) * (size_t)n * (size_t)h->p.depth));
    hipLaunchKernelGGL(k_perm_norms, dim3(grid), dim3(256), 0, h->stream, h->d_norm_sqrt, perm, n, h->p.depth,
                       h->ws_nsq.as<double>());
    if (n > f0) {
      // whole kImgBlk-row blocks; the last block's padding rows are zero
      const int64_t blocks = (n - f0 + kImgBlk - 1) / kImgBlk;
      CMS_HIP(h->ws_f4.ensure((size_t)blocks * kImgBlk * (size_t)(dw / 2)));
      CMS_HIP(hipMemsetAsync(h->ws_f4.as<uint8_t>() + (size_t)(blocks - 1) * kImgBlk * (dw / 2), 0,
                             (size_t)kImgBlk * (dw / 2), h->stream));
      hipLaunchKernelGGL(k_f4_write, dim3((unsigned)(n - f0)), dim3(256), (size_t)h->p.width, h->stream, h->tview(), dw, perm, f0,
                         h->ws_f4.as<uint8_t>(), h->sym_sw);
    }
    CMS_HIP(hipGetLastError());
  }
  h->tile_limbs.resize(ntiles);
  h->h_perm.resize(n);
  h->h_inv.resize(n);
  CMS_HIP(hipMemcpyAsync(h->tile_limbs.data(), tileL, ntiles, hipMemcpyDeviceToHost, h->stream));
  CMS_HIP(hipMemcpyAsync(h->h_perm.data(), perm, sizeof(int64_t) * n, hipMemcpyDeviceToHost, h->stream));
  CMS_HIP(hipMemcpyAsync(h->h_inv.data(), inv, sizeof(int64_t) * n, hipMemcpyDeviceToHost, h->stream));
  CMS_HIP(hipStreamSynchronize(h->stream));
  // virtual limb rows for the multi-limb x single-limb blocks (k_cosine_big<., LS>):
  // 4 slots for the 3-4-limb owners, 2 slots for the 2-limb ones
  h->vl_ok = n_five == 0;
  const int64_t bounds[3] = {0, n_deep, n_multi};
  const int32_t slots[2] = {4, 2};
  for (int gi = 0; gi < 2; ++gi) {
    auto& G = h->vl[gi];
    G.o0 = bounds[gi];
    G.o1 = bounds[gi + 1];
    G.ls = slots[gi];
    const int per = 32 / G.ls;  // owners per 32-row block
    G.rows = (G.o1 - G.o0 + per - 1) / per * 32;
    G.bready = false;
    if (!h->vl_ok || G.rows == 0) continue;
    CMS_HIP(G.buf.ensure((size_t)G.rows * (size_t)dw));
    TimedScope ts(h, "limb_prep");
    hipLaunchKernelGGL(k_vl_build, dim3((unsigned)G.rows), dim3(256), 0, h->stream, h->ws_limb0.as<int8_t>(),
                       h->ws_limbhot.as<int8_t>(), rowLp, G.o0, G.o1, dw, G.ls, G.buf.as<int8_t>());
    CMS_HIP(hipGetLastError());
  }
  h->mfma_ready = true;
  return CMS_OK;
}

const int64_t* cosine_perm_device(cms_handle* h) { return h->ws_limbmeta.as<int64_t>(); }

bool mfma_eligible(cms_handle* h) { return !h->f64 && (h->p.width % kBK) == 0; }

// Similarities of the owners at PERMUTED positions [q0, q0+qc) against every
// owner into slab [qc][n] (fp64, column = permuted position; owner row =
// perm[column]).  q0 must be a multiple of kTile.
// Launch shape of k_cosine_big for this table: stage depth and ring size
// that fit 160 KiB of LDS beside the panel norms.
struct BigCfg {
  int bk = 128, nstage = 0;
  size_t norms = 0;
};

static BigCfg big_config(cms_handle* h, int force_bk = 0) {
  BigCfg c;
  if (force_bk) c.bk = force_bk;
  c.norms = (size_t)h->p.depth * (kTA + kTB) * sizeof(double) + (kTA + kTB) * sizeof(__half);
#ifdef CMS_SCREEN_PROBE
  constexpr size_t kLdsMax = 160 * 1024 - 2048;  // the probe's static LDS (2-stage ring)
#else
  constexpr size_t kLdsMax = 160 * 1024;
#endif
  // 128-B K slices (one cache line per row) in a 3- or 2-deep ring; 64-B
  // slices in a 6-deep ring measured slower (twice the line requests per
  // byte, twice the barriers)
#ifdef CMS_BOUND_ANALYSIS
  if (const char* e = getenv("CMS_COS_BK")) c.bk = atoi(e) == 64 ? 64 : 128;
#endif
  if (c.bk == 64) {
    c.nstage = 6 * 384 * 64 + c.norms <= kLdsMax ? 6 : 4 * 384 * 64 + c.norms <= kLdsMax ? 4 : 0;
    if (!c.nstage) c.bk = 128;
  }
  if (c.bk == 128) c.nstage = 3 * 384 * 128 + c.norms <= kLdsMax ? 3 : 2 * 384 * 128 + c.norms <= kLdsMax ? 2 : 0;
  static bool attr = [] {
    const void* fns[] = {(const void*)k_cosine_tile<false>,      (const void*)k_cosine_tile<true>,
                         (const void*)k_cosine_big<2, 1, 128>,   (const void*)k_cosine_big<3, 1, 128>,
                         (const void*)k_cosine_big<2, 2, 128>,   (const void*)k_cosine_big<3, 2, 128>,
                         (const void*)k_cosine_big<2, 4, 128>,   (const void*)k_cosine_big<3, 4, 128>,
                         (const void*)k_cosine_big<4, 1, 64>,    (const void*)k_cosine_big<6, 1, 64>,
                         (const void*)k_cosine_big<4, 2, 64>,    (const void*)k_cosine_big<6, 2, 64>,
                         (const void*)k_cosine_big<4, 4, 64>,    (const void*)k_cosine_big<6, 4, 64>,
                         (const void*)k_cosine_big<2, 1, 128, 1>, (const void*)k_cosine_big<3, 1, 128, 1>,
                         (const void*)k_cosine_big<4, 1, 64, 1>,  (const void*)k_cosine_big<6, 1, 64, 1>};
    for (const void* f : fns) (void)hipFuncSetAttribute(f, hipFuncAttributeMaxDynamicSharedMemorySize, (int)kLdsMax);
    return true;
  }();
  (void)attr;
  return c;
}

// One k_cosine_big launch.  Rectangular mode: A owners x B rows; symmetric
// mode (g.sym): sym_pairs block pairs of the wave, two workgroups each.
static int launch_big(cms_handle* h, const BigCfg& c, BigArgs g, int ls, int64_t sym_pairs = 0, int fmt = 0) {
  if (g.sym) {
    g.tilesB = 2;
    g.nblk = (int)(2 * g.band * sym_pairs);
    if (g.rect) {
      g.njc = (g.si + g.band - 1 + g.sj - 1) / g.sj;
      g.nblk = (int)(((sym_pairs + g.si - 1) / g.si) * g.njc * g.si * g.sj * 2);
    }
  } else {
    const int oa = kTA / ls;
    const int64_t tilesA = (g.a_owners + oa - 1) / oa;
    g.tilesB = (int)((g.b_rows + kTB - 1) / kTB);
    g.nblk = (int)(tilesA * g.tilesB);
  }
  if (g.nblk <= 0) return CMS_OK;
  const size_t bytes = (size_t)c.nstage * 384 * c.bk + c.norms;
  const dim3 grid((unsigned)g.nblk), blk(512);
  if (fmt == 1) {  // fp4 operands: single-limb sym waves, 128-B stages
    if (c.bk == 64) {
      if (c.nstage == 6) hipLaunchKernelGGL((k_cosine_big<6, 1, 64, 1>), grid, blk, bytes, h->stream, g);
      else hipLaunchKernelGGL((k_cosine_big<4, 1, 64, 1>), grid, blk, bytes, h->stream, g);
    } else if (c.nstage == 3) {
      hipLaunchKernelGGL((k_cosine_big<3, 1, 128, 1>), grid, blk, bytes, h->stream, g);
    } else {
      hipLaunchKernelGGL((k_cosine_big<2, 1, 128, 1>), grid, blk, (size_t)2 * 384 * 128 + c.norms, h->stream, g);
    }
    CMS_HIP(hipGetLastError());
    return CMS_OK;
  }
#define CMS_BIG(NS, L, K) hipLaunchKernelGGL((k_cosine_big<NS, L, K>), grid, blk, bytes, h->stream, g)
#define CMS_BIG_LS(NS, K)              \
  do {                                 \
    if (ls == 1) CMS_BIG(NS, 1, K);      \
    else if (ls == 2) CMS_BIG(NS, 2, K); \
    else CMS_BIG(NS, 4, K);            \
  } while (0)
  if (c.bk == 64) {
    if (c.nstage == 6) CMS_BIG_LS(6, 64);
    else CMS_BIG_LS(4, 64);
  } else {
    if (c.nstage == 3) CMS_BIG_LS(3, 128);
    else CMS_BIG_LS(2, 128);
  }
#undef CMS_BIG_LS
#undef CMS_BIG
  CMS_HIP(hipGetLastError());
  return CMS_OK;
}

static BigArgs big_base(cms_handle* h) {
  BigArgs b{};
#ifdef CMS_BOUND_ANALYSIS
  b.noscreen = getenv("CMS_NO_SCREEN") ? 1 : 0;
  if (const char* m = getenv("CMS_COS_MODE")) b.mode = atoi(m);
#endif
  b.perm = h->ws_limbmeta.as<int64_t>();
  b.nsq_t = h->ws_nsq.as<double>();
  b.n = h->n;
  b.ldo = h->n;
  b.dw = h->dw;
  b.w = h->p.width;
  b.depth = h->p.depth;
  b.weighted = h->p.weighting == CMS_WEIGHTED;
  b.rs = h->dw;
  b.kw = h->p.width;
  return b;
}

// The K-blocked copy of the single-limb int8 image (positions [n_multi, n))
// that the int8 symmetric waves and k_cosine_mls read, when the device has
// room for it next to everything else.
static bool ensure_i8blk(cms_handle* h) {
  if (h->i8blk_ready) return true;
  const int64_t nm = h->n_hot_limb, ns = h->n - nm;
  if (ns <= 0) return false;
  const int64_t blocks = (ns + kImgBlk - 1) / kImgBlk;
  const size_t bytes = (size_t)blocks * kImgBlk * (size_t)h->dw;
  size_t free_b = 0, total_b = 0;
  if (hipMemGetInfo(&free_b, &total_b) != hipSuccess || free_b <= bytes + ((size_t)4 << 30) ||
      h->ws_i8blk.ensure(bytes) != hipSuccess)
    return false;
  TimedScope ts(h, "limb_prep");
  hipLaunchKernelGGL(k_i8blk_write, dim3((unsigned)(blocks * kImgBlk)), dim3(256), 0, h->stream, h->ws_limb0.as<int8_t>(),
                     h->dw, nm, ns, h->ws_i8blk.as<int8_t>(), h->sym_sw);
  if (hipGetLastError() != hipSuccess) return false;
  h->i8blk_ready = true;
  return true;
}

int cosine_slab(cms_handle* h, int64_t q0, int64_t qc, double* d_out) {
  int rc = cosine_prepare(h);
  if (rc) return rc;
  const int64_t n = h->n, dw = h->dw;
  const int64_t nbs = (n + 4095) / 4096 + 1;
  CosArgs a;
  a.limb0 = h->ws_limb0.as<int8_t>();
  a.hl = h->ws_limbhot.as<int8_t>();
  a.perm = h->ws_limbmeta.as<int64_t>();
  a.rowL = reinterpret_cast<const uint8_t*>(reinterpret_cast<const uint32_t*>(a.perm + 2 * n) + 2 * n + nbs) + n;
  a.tileL = a.rowL + n;
  a.n_multi = h->n_hot_limb;
  a.nsqrt = h->d_norm_sqrt;
  a.n = n;
  a.dw = dw;
  a.w = h->p.width;
  a.depth = h->p.depth;
  a.q0 = q0;
  a.qcount = qc;
  a.ldo = n;
  a.out = d_out;
  a.weighted = h->p.weighting == CMS_WEIGHTED;
  const int64_t ntiles = (n + kTile - 1) / kTile;
  const int64_t trows = (qc + kTile - 1) / kTile;
  a.tiles_x = (int)ntiles;
  const int64_t nm = a.n_multi;
  const BigCfg cfg = big_config(h);
  const size_t lds = 4 * kTile * kBK + 2 * kTile * sizeof(double);  // 2 buffers x (A + B) + norms
  const int64_t qend = q0 + qc;

  if (cfg.nstage && (nm == 0 || h->vl_ok)) {
    // Four blocks of the slab in permuted coordinates (M = multi-limb owners
    // [0, nm), S = the rest):  S x S and M x S / S x M on k_cosine_big,
    // M x M on the int64-folding MULTI tile kernel.
    auto launch = [&](const BigArgs& g, int ls) { return launch_big(h, cfg, g, ls); };
    BigArgs base = big_base(h);
    base.out = d_out;
    base.q0 = q0;
    base.qcount = qc;
    const int64_t slo = std::max(q0, nm);  // single-limb query rows [slo, qend)
    // candidate column ranges: every column, or (a refresh's untouched
    // multi-limb rows) the caller's ranges; the other columns are left alone
    std::vector<std::pair<int64_t, int64_t>> cols = h->slab_cols;
    if (cols.empty()) cols.push_back({0, n});
    else if (slo < qend) return set_error(CMS_E_STATE, "column-restricted slab with single-limb query rows");
    if (slo < qend && nm < n) {  // S x S
      BigArgs g = base;
      g.A = a.limb0 + slo * dw;
      g.a_vrows = g.a_owners = qend - slo;
      g.a_pos0 = slo;
      g.B = a.limb0 + nm * dw;
      g.b_pos0 = nm;
      g.b_rows = n - nm;
      TimedScope ts(h, "cosine_mfma");
      if ((rc = launch(g, 1))) return rc;
    }
    for (int gi = 0; gi < 2 && nm > 0; ++gi) {
      const auto& G = h->vl[gi];
      if (G.o1 <= G.o0) continue;
      const int ls = G.ls, per = 32 / ls;
      const int8_t* vl = G.buf.as<int8_t>();
      TimedScope ts(h, "cosine_mfma_limbs");
      if (q0 < G.o1 && qend > G.o0 && nm < n && h->i8blk_ready && mls_eligible(h) && h->tune.mls) {
        // M x S on k_cosine_mls (256 x 192 tiles from the K-blocked images):
        // from the 64-row image block holding the slab's first owner of the group
        if ((rc = vl_blk_prepare(h, gi))) return rc;
        const int64_t oa0 = G.o0 + (std::max(q0, G.o0) - G.o0) / (2 * per) * (2 * per);
        const int64_t vrow0 = (oa0 - G.o0) / per * 32;
        for (const auto& cr : cols) {
        const int64_t lo = std::max(cr.first, nm), hi = std::min(cr.second, n);
        if (lo >= hi) continue;
        const int64_t blo = nm + (lo - nm) / kImgBlk * kImgBlk;  // image blocks start every kImgBlk rows from nm
        MlsArgs m{};
        m.A = G.bbuf.as<int8_t>() + vrow0 * dw;
        m.a_vrows = G.rows - vrow0;
        m.a_pos0 = oa0;
        m.a_owners = std::min(qend, G.o1) - oa0;
        m.B = h->ws_i8blk.as<int8_t>();
        m.b_img0 = nm;
        m.b_pos0 = blo;
        m.b_rows = hi - blo;
        m.rs = dw;
        m.kw = h->p.width;
        m.depth = h->p.depth;
        m.nsq_t = h->ws_nsq.as<double>();
        m.n = n;
        m.out = d_out;
        m.ldo = n;
        m.q0 = q0;
        m.qcount = qc;
        m.weighted = h->p.weighting == CMS_WEIGHTED;
        if ((rc = launch_mls(h, m, ls))) return rc;
        }
      } else if (q0 < G.o1 && qend > G.o0 && nm < n) {  // M x S: multi-limb queries against single-limb candidates
        const int64_t oa0 = G.o0 + (std::max(q0, G.o0) - G.o0) / per * per;
        const int64_t blk = (oa0 - G.o0) / per;
        for (const auto& cr : cols) {
          const int64_t lo = std::max(cr.first, nm), hi = std::min(cr.second, n);
          if (lo >= hi) continue;
          BigArgs g = base;
          g.A = vl + blk * 32 * dw;
          g.a_vrows = G.rows - blk * 32;
          g.a_pos0 = oa0;
          g.a_owners = std::min(qend, G.o1) - oa0;
          g.B = a.limb0 + lo * dw;
          g.b_pos0 = lo;
          g.b_rows = hi - lo;
          if ((rc = launch(g, ls))) return rc;
        }
      }
      if (slo < qend) {  // S x M, computed as M x S and written transposed
        BigArgs g = base;
        g.A = vl;
        g.a_vrows = G.rows;
        g.a_pos0 = G.o0;
        g.a_owners = G.o1 - G.o0;
        g.B = a.limb0 + slo * dw;
        g.b_pos0 = slo;
        g.b_rows = qend - slo;
        g.trans = 1;
        if ((rc = launch(g, ls))) return rc;
      }
    }
    // M x M: the 128-tiles holding multi-limb queries and multi-limb candidates
    std::vector<int2> multi;
    auto col_tile = [&](int64_t tc) {  // the 128-column tile meets a candidate range
      for (const auto& cr : cols)
        if (cr.first < (tc + 1) * kTile && cr.second > tc * kTile) return true;
      return false;
    };
    for (int64_t tr = 0; q0 + tr * kTile < std::min(qend, nm); ++tr)
      for (int64_t tc = 0; tc * kTile < nm; ++tc)
        if (col_tile(tc)) multi.push_back(make_int2((int)tc, (int)tr));
    if (!multi.empty()) {
      CMS_HIP(h->ws_tiles.ensure(sizeof(int2) * multi.size()));
      CMS_HIP(hipMemcpyAsync(h->ws_tiles.ptr, multi.data(), sizeof(int2) * multi.size(), hipMemcpyHostToDevice,
                             h->stream));
      TimedScope ts(h, "cosine_mfma_multi");
      hipLaunchKernelGGL(k_cosine_tile<true>, dim3((unsigned)multi.size()), dim3(256), lds, h->stream, a,
                         h->ws_tiles.as<int2>(), (int32_t)multi.size());
      CMS_HIP(hipGetLastError());
      CMS_HIP(hipStreamSynchronize(h->stream));  // the host tile list must outlive the copy
    }
    return CMS_OK;
  }

  // Legacy 128 x 128 path (depth > 21, or owners needing 5 limbs): the fast
  // kernel skips tiles touching a multi-limb owner, MULTI takes them.
  {
    TimedScope ts(h, "cosine_mfma");
    hipLaunchKernelGGL(k_cosine_tile<false>, dim3((unsigned)ntiles, (unsigned)trows), dim3(256), lds, h->stream, a,
                       (const int2*)nullptr, 0);
    CMS_HIP(hipGetLastError());
  }
  std::vector<int2> multi;
  for (int64_t tr = 0; tr < trows; ++tr)
    for (int64_t tc = 0; tc < ntiles; ++tc)
      if (h->tile_limbs[(q0 / kTile) + tr] > 1 || h->tile_limbs[tc] > 1) multi.push_back(make_int2((int)tc, (int)tr));
  if (!multi.empty()) {
    CMS_HIP(h->ws_tiles.ensure(sizeof(int2) * multi.size()));
    CMS_HIP(hipMemcpyAsync(h->ws_tiles.ptr, multi.data(), sizeof(int2) * multi.size(), hipMemcpyHostToDevice,
                           h->stream));
    TimedScope ts(h, "cosine_mfma_multi");
    hipLaunchKernelGGL(k_cosine_tile<true>, dim3((unsigned)multi.size()), dim3(256), lds, h->stream, a,
                       h->ws_tiles.as<int2>(), (int32_t)multi.size());
    CMS_HIP(hipGetLastError());
    CMS_HIP(hipStreamSynchronize(h->stream));  // the host tile list must outlive the copy
  }
  return CMS_OK;
}

// fp32 copies of admission thresholds, rounded toward -inf (never above)
__global__ void k_thr_f32(const double* thr, float* t32, int64_t n) {
  for (int64_t i = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; i < n; i += (int64_t)gridDim.x * blockDim.x)
    t32[i] = __double2float_rd(thr[i]);
}

// Refresh: admission thresholds of the untouched owners' lists from their
// kept lists (position p holds owner row perm[p]); a kept list that holds
// every candidate (full) or none keeps -inf.
__global__ void k_rf_seed_thr(int64_t n, int32_t D, const int64_t* perm, const uint8_t* touch, const int32_t* kcnt,
                              const double* ksc, const uint8_t* kfull, double* thr) {
  for (int64_t p = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; p < n; p += (int64_t)gridDim.x * blockDim.x) {
    const int64_t r = perm[p];
    const int32_t c = kcnt[r];
    if (!touch[r] && !kfull[r] && c > 0) thr[p] = ksc[r * D + c - 1];
  }
}

// ---------------------------------------------- all-pairs top-k, streaming --
// TopItems.getTopUsers for EVERY owner (T/impl/recommender/TopItems.java:91-136,
// one GenericUserBasedRecommender.mostSimilarUserIDs per owner) without an
// n x n slab and with each unordered single-limb pair computed ONCE:
//   1. multi-limb rows (M): exact slab top-k (slab_top_k_positions);
//   2. single-limb rows (S) x M candidates: k_cosine_big in candidate mode,
//      M owners as virtual limb rows, offered to the S rows' lists;
//   3. S x S: symmetric waves -- wave w computes block pairs {I, I+w mod nb}
//      of 256 rows, each similarity offered to BOTH rows' lists;
//   4. lists compacted to the first k of (score desc, owner row asc) --
//      SimilarUser.compareTo -- whenever a pass could overflow them; the
//      k-th score becomes the row's admission threshold (score >= thr,
//      ties admitted, so the order among equal scores stays exact).
// A row receives at most 512 offers per wave (its block as A, and as B), and
// a list is compacted before a pass whenever it holds more than cap - 512, so
// lists cannot overflow; should one ever do, the row is recomputed exactly.
// Shard `shard` of `nshards` computes a disjoint share of the pairs (M rows
// p % nshards, S x M chunks, waves w % nshards) and leaves PARTIAL lists:
// for every owner the first k of the candidates it saw, sorted.  The union
// over shards is every pair once, so merging the partial lists
// (top_k_merge) gives the exact result.  nshards == 1 is the whole job.
int top_k_all(cms_handle* h, int32_t k, int64_t* d_ids, double* d_scores, int32_t* d_counts, int32_t shard,
              int32_t nshards) {
  if (h->per_owner) {  // asymmetric similarities: every row scans every candidate
    if (nshards == 1) return top_k_rows(h, 0, h->n, k, d_ids, d_scores, d_counts);
    // G ranks: every rank holds the whole DataModel (u1's preferences are
    // hashed at each candidate's shape), so the job shards by QUERY rows --
    // chunks of kPoShardRows rows round-robin (a Zipf model's costly rows
    // spread over the ranks); the other rows' lists stay empty (count 0) and
    // the collective merge (top_k_all_job) takes each row's list from the
    // rank that computed it
    constexpr int64_t kPoShardRows = 256;
    CMS_HIP(hipMemsetAsync(d_counts, 0, sizeof(int32_t) * h->n, h->stream));
    for (int64_t r0 = (int64_t)shard * kPoShardRows; r0 < h->n; r0 += (int64_t)nshards * kPoShardRows) {
      const int64_t rc0 = std::min<int64_t>(kPoShardRows, h->n - r0);
      if (int rc = top_k_rows(h, r0, rc0, k, d_ids + r0 * k, d_scores + r0 * k, d_counts + r0)) return rc;
    }
    return CMS_OK;
  }
  if (h->f64) {  // fp64 counters: the exact sequential kernels, one slab of query rows at a time
    if (nshards == 1) return top_k_rows(h, 0, h->n, k, d_ids, d_scores, d_counts);
    CMS_HIP(hipMemsetAsync(d_counts, 0, sizeof(int32_t) * h->n, h->stream));
    for (int64_t r0 = shard; r0 < h->n; r0 += nshards) {
      if (int rc = top_k_rows(h, r0, 1, k, d_ids + r0 * k, d_scores + r0 * k, d_counts + r0)) return rc;
    }
    return CMS_OK;
  }
  int rc = cosine_prepare(h);
  if (rc) return rc;
  const int64_t n = h->n;
  const BigCfg cfg = big_config(h);
  const int64_t nm = h->n_hot_limb, ns = n - nm;
  if (!cfg.nstage || (nm > 0 && !h->vl_ok) || h->n_inexact_rows != 0 || k > kCandCap / 2) {
    if (nshards == 1) return top_k_rows(h, 0, n, k, d_ids, d_scores, d_counts);  // per-row slab path
    // per-row slab path for this shard's rows only; the other rows stay empty
    CMS_HIP(hipMemsetAsync(d_counts, 0, sizeof(int32_t) * n, h->stream));
    for (int64_t r0 = shard; r0 < n; r0 += nshards) {
      if ((rc = top_k_rows(h, r0, 1, k, d_ids + r0 * k, d_scores + r0 * k, d_counts + r0))) return rc;
    }
    return CMS_OK;
  }
  CMS_HIP(hipMemsetAsync(d_counts, 0, sizeof(int32_t) * n, h->stream));
  // symmetric waves on k_cosine_sym (256 x 192 tiles, 768-row blocks) when
  // the table allows it and the images are staged 64 B deep
  int32_t rb8 = 0, rb4 = 0;
  const bool sym_img = h->sym_sw == sym_stage_bytes();
  const bool sym8 = sym_img && sym_eligible(h, 0, &rb8);
  const bool sym4 = sym_img && sym_eligible(h, 1, &rb4);
  const int32_t cap = (sym8 || sym4) ? kCandCapSym : kCandCap;
  DevBuf& ws = h->ws_cand;
  const size_t off_cidx = (sizeof(uint32_t) * (size_t)n + 255) & ~size_t(255);
  const size_t off_cval = off_cidx + ((sizeof(uint32_t) * (size_t)n * cap + 255) & ~size_t(255));
  const size_t off_thr = off_cval + sizeof(double) * (size_t)n * cap;
  const size_t off_ovf = off_thr + sizeof(double) * (size_t)n;
  const size_t off_list = off_ovf + sizeof(uint32_t) * (size_t)n;
  const size_t off_ln = off_list + sizeof(uint32_t) * (size_t)n;
  const size_t off_t32 = (off_ln + 256 + 255) & ~size_t(255);
  CMS_HIP(ws.ensure(off_t32 + sizeof(float) * (size_t)n + 256));
  float* thr32 = reinterpret_cast<float*>(ws.as<char>() + off_t32);
  char* wsb = ws.as<char>();
  CandBufs cb;
  cb.ccnt = reinterpret_cast<uint32_t*>(wsb);
  cb.cidx = reinterpret_cast<uint32_t*>(wsb + off_cidx);
  cb.cval = reinterpret_cast<double*>(wsb + off_cval);
  cb.thr = reinterpret_cast<double*>(wsb + off_thr);
  cb.ovf = reinterpret_cast<uint32_t*>(wsb + off_ovf);
  cb.list = reinterpret_cast<uint32_t*>(wsb + off_list);
  cb.list_n = reinterpret_cast<uint32_t*>(wsb + off_ln);
  cb.cap = cap;
  CMS_HIP(hipMemsetAsync(cb.ccnt, 0, sizeof(uint32_t) * n, h->stream));
  CMS_HIP(hipMemsetAsync(cb.ovf, 0, sizeof(uint32_t) * n, h->stream));
  {
    std::vector<double> ninf(1 << 16, -__builtin_inf());
    for (int64_t o = 0; o < n; o += (int64_t)ninf.size())
      CMS_HIP(hipMemcpyAsync(cb.thr + o, ninf.data(), sizeof(double) * std::min<int64_t>(ninf.size(), n - o),
                             hipMemcpyHostToDevice, h->stream));
    if (h->rf_restrict) {
      // refresh: an untouched owner's fold keeps only the merged entries at or
      // above its kept list's last score (k_rf_fold's valid prefix), so its
      // list here admits nothing below that score
      const unsigned grid = (unsigned)std::min<int64_t>((n + 255) / 256, 4096);
      hipLaunchKernelGGL(k_rf_seed_thr, dim3(grid), dim3(256), 0, h->stream, n, h->rf_depth, cosine_perm_device(h),
                         h->rf_touch.as<uint8_t>(), h->rf_cnt.as<int32_t>(), h->rf_sc.as<double>(),
                         h->rf_full.as<uint8_t>(), cb.thr);
      CMS_HIP(hipGetLastError());
    }
    CMS_HIP(hipStreamSynchronize(h->stream));
  }
  BigArgs base = big_base(h);
  base.thr = cb.thr;
  base.ccnt = cb.ccnt;
  base.cidx = cb.cidx;
  base.cval = cb.cval;
  base.cap = cap;
  const int8_t* limb0 = h->ws_limb0.as<int8_t>();
  // 1 + 2. multi-limb rows in chunks: one slab each (M x S as
  // virtual limb rows, M x M on the MULTI tiles) gives their exact top-k AND
  // the M candidates of every single-limb row -- each (M, S) pair once
  if (nm > 0) {
    if (ns > 0) (void)ensure_i8blk(h);  // k_cosine_mls's candidate operand (and the int8 waves')
    TimedScope ts(h, "topk_all_multi_rows");
    // chunk: a slab of qc rows offers qc similarities to every S list, so a
    // chunk must leave room in a list compacted to cap - qc entries
    // (the lists are offered the slab cap/2 rows at a time: multi_rows_slab_offer)
    const int64_t chunk = multi_slab_rows(h, n);
    if (!h->rf_restrict) {
      for (int64_t m0 = (int64_t)shard * chunk; m0 < nm; m0 += (int64_t)nshards * chunk) {
        const int64_t qc = std::min<int64_t>(chunk, nm - m0);
        if ((rc = multi_rows_slab_offer(h, cb, m0, qc, nm, n, k, d_ids, d_scores, d_counts))) return rc;
      }
    } else {
      // refresh: touched multi-limb rows (first in each limb group) against
      // every column; untouched ones only against the touched owners' columns
      // (multi-limb, int8 and fp4 ranges), the only pairs of theirs that changed
      const int64_t nd = h->rf_nd;
      const std::vector<std::pair<int64_t, int64_t>> touched = {
          {0, h->rf_td}, {nd, nd + h->rf_tm}, {nm, nm + h->rf_t8}, {nm + h->rf_s8, nm + h->rf_s8 + h->rf_t4}};
      const struct {
        int64_t lo, hi;
        bool all;
      } runs[4] = {{0, h->rf_td, true}, {nd, nd + h->rf_tm, true}, {h->rf_td, nd, false}, {nd + h->rf_tm, nm, false}};
      int64_t ctr = 0;
      for (const auto& ru : runs)
        for (int64_t m0 = ru.lo; m0 < ru.hi; m0 += chunk) {
          if (ctr++ % nshards != shard) continue;
          const int64_t qc = std::min<int64_t>(chunk, ru.hi - m0);
          if ((rc = multi_rows_slab_offer(h, cb, m0, qc, nm, n, k, d_ids, d_scores, d_counts,
                                          ru.all ? nullptr : &touched)))
            return rc;
        }
    }
  }
  // 3. S x S symmetric waves.  With fp4 owners (positions [f0, n), whole
  // 256-row blocks from fblk0 on): waves over the fp4 region on the fp4 image,
  // then waves over all S blocks restricted to pairs with a block below fblk0
  // on int8 -- every unordered pair once either way.
  if (ns > 0) {
    const int64_t nb = (ns + kTA - 1) / kTA;
    const int64_t f0 = h->f4_pos0;
    const int64_t fblk0 = f0 < n ? (f0 - nm) / kTA : nb;  // first block of fp4 owners only
    // Weighted similarities are all +-1: thresholds never tighten, so every
    // later candidate is admitted and only single waves are safe.
    const bool weighted = h->p.weighting == CMS_WEIGHTED;
    int64_t ramp = 25, lmax = 32;
#ifdef CMS_BOUND_ANALYSIS
    if (const char* e = getenv("CMS_BAND")) sscanf(e, "%ld,%ld", &ramp, &lmax);
#endif
    // Bands of waves per launch.  A row takes up to 512 offers per wave, but
    // once its list has seen m columns its threshold admits about k*512/m of
    // them; bands grow with the wave index so a launch brings ~25 expected
    // offers per row (lists are compacted to cap/2 before each band; an
    // overflow would flag the row for an exact recompute).  Each band reads
    // its panels from HBM once and reuses them 2*band times from L2.
    auto band_list = [&](int64_t nbk) {
      std::vector<std::pair<int64_t, int64_t>> bands;  // (first wave, waves)
      for (int64_t wv = 0; wv <= nbk / 2;) {
        int64_t L = (wv < 8 || weighted) ? 1 : std::max<int64_t>(1, std::min<int64_t>(lmax, wv * ramp / std::max(1, k)));
        L = std::min<int64_t>(L, nbk / 2 - wv + 1);
        bands.push_back({wv, L});
        wv += L;
      }
      return bands;
    };
    // The int8 waves read their operands from a K-blocked copy of the
    // single-limb image (a stage of a block is one contiguous run) when the
    // device has room for it next to everything else
    const bool i8blk = fblk0 > 0 && ensure_i8blk(h);
    const BigCfg scfg = big_config(h, h->sym_sw);  // the blocked images' stage depth
    // pass 0: fp4 x fp4 block pairs; pass 1: the rest (all S when no fp4 region).
    // Each pass picks its kernel: k_cosine_sym (768-row blocks) or
    // k_cosine_big (256-row blocks); the passes' row sets do not depend on it.
    int64_t shard_ctr = 0;
    for (int pass = 0; pass < 2; ++pass) {
      const bool fp4 = pass == 0;
      if (fp4 && fblk0 >= nb) continue;
      if (!fp4 && fblk0 == 0) continue;
      const bool use_sym = fp4 ? sym4 : (sym8 && i8blk);
      const int64_t blk = use_sym ? kSymBlk : kTA;
      const int64_t nb_s = (ns + blk - 1) / blk;                        // blocks of the whole S region
      const int64_t fb0 = f0 < n ? (f0 - nm) / blk : nb_s;              // first block of fp4 owners only
      const int64_t nbk = fp4 ? (n - f0 + blk - 1) / blk : nb_s;
      for (const auto& bd : band_list(nbk)) {
        if (shard_ctr++ % nshards != shard) continue;
        const int64_t wv = bd.first, L = bd.second;
        // a row takes up to 2 * blk offers per wave (its block as A and as B)
        const uint32_t limit = L == 1 ? (uint32_t)(cap - 2 * blk) : (uint32_t)cap / 2;
        if ((rc = cand_compact(h, cb, nm, ns, limit, k))) return rc;
        // wide bands of plain (non-fsel) waves: rectangle enumeration
        const int rect = (L >= 8 && !(fp4 ? false : fb0 < nb_s)) ? 1 : 0;
        TimedScope ts(h, "topk_all_waves");
        TimedScope tsub(h, fp4 ? "topk_all_waves_f4" : "topk_all_waves_i8");
        if (use_sym) {
          SymArgs g{};
          g.img = fp4 ? h->ws_f4.as<int8_t>() : h->ws_i8blk.as<int8_t>();
          g.img0 = g.s0 = fp4 ? f0 : nm;
          g.s_rows = fp4 ? n - f0 : ns;
          g.rs = fp4 ? h->dw / 2 : h->dw;
          g.kw = fp4 ? h->p.width / 2 : h->p.width;
          g.depth = h->p.depth;
          g.nsq_t = h->ws_nsq.as<double>();
          g.n = n;
          g.nb = (int32_t)nbk;
          g.wave = (int32_t)wv;
          g.band = (int32_t)L;
          g.rect = rect;
          g.si = 8;  // 8 A blocks x 2 J chunks: fp4 waves -5 % against 4 x 4 (8 x 1, 16 x 2 within 1 %)
          g.sj = 2;
          g.xchunk = 32;  // the XCDs side by side (xcd_chunk_map): int8 waves -7%, fp4 waves unchanged
          g.thr = cb.thr;
          g.ccnt = cb.ccnt;
          g.cidx = cb.cidx;
          g.cval = cb.cval;
          g.cap = cap;
          g.rbits = fp4 ? rb4 : rb8;
          if (h->rf_restrict) {  // refresh: the touched rows are two position ranges; keep their blocks' pairs
            auto blocks = [&](int64_t lo, int64_t hi, int32_t* b0, int32_t* b1) {
              lo = std::max<int64_t>(lo, g.s0);
              hi = std::min<int64_t>(hi, g.s0 + g.s_rows);
              *b0 = *b1 = 0;
              if (hi > lo) {
                *b0 = (int32_t)((lo - g.s0) / kSymBlk);
                *b1 = (int32_t)((hi - g.s0 + kSymBlk - 1) / kSymBlk);
              }
            };
            g.tsel = 1;
            blocks(nm, nm + h->rf_t8, &g.ts0, &g.ts1);
            blocks(nm + h->rf_s8, nm + h->rf_s8 + h->rf_t4, &g.ts2, &g.ts3);
          }
          int64_t slots = nbk;
          if (!fp4 && fb0 < nb_s) {
            g.fsel = 1;
            g.fblk0 = (int32_t)fb0;
            slots = 2 * fb0;
          }
          if (g.tsel) {
            int32_t a0 = g.ts0, a1 = g.ts1, b0 = g.ts2, b1 = g.ts3;
            if (a0 == a1) {
              a0 = b0;
              a1 = b1;
              b0 = b1 = 0;
            }
            if (a0 == a1) continue;  // no touched owner in this pass's region: no pair to recompute
            // touched blocks [0, P): enumerate only the pairs with a block
            // below P (dense, as the fsel waves); otherwise every pair of the
            // pass is enumerated and the untouched ones leave at once, with the
            // workgroups spread round-robin over the XCDs (identity map) so the
            // ones that stay are not all on one XCD
            if (a0 == 0 && (b0 == b1 || b0 <= a1) && !g.fsel) {
              const int32_t P = std::max(a1, b0 == b1 ? a1 : b1);
              if (2 * (int64_t)P < nbk) {
                g.tsel = 0;
                g.fsel = 1;
                g.fblk0 = P;
                slots = 2 * (int64_t)P;
              }
              g.rect = 0;
            } else {
              g.rect = 0;
            }
          }
          {  // the admission thresholds as fp32 rounded down, for the tiles' LDS-DMA
            const unsigned tg = (unsigned)std::min<int64_t>((g.s_rows + 255) / 256, 4096);
            hipLaunchKernelGGL(k_thr_f32, dim3(tg), dim3(256), 0, h->stream, cb.thr + g.s0, thr32 + g.s0, g.s_rows);
            CMS_HIP(hipGetLastError());
            g.thr32 = thr32;
          }
          if ((rc = launch_sym(h, g, fp4 ? 1 : 0, slots))) return rc;
          continue;
        }
        BigArgs g = base;
        g.sym = 1;
        g.wave = (int32_t)wv;
        g.band = (int32_t)L;
        g.nb = (int32_t)nbk;
        g.append_a = g.append_b = 1;
        g.rect = rect;
        g.si = 4;
        g.sj = 4;
        if (fp4) {
          g.A = g.B = h->ws_f4.as<int8_t>();
          g.img0 = g.s0 = f0;
          g.s_rows = n - f0;
          g.rs = h->dw / 2;
          g.kw = h->p.width / 2;
          if ((rc = launch_big(h, scfg, g, 1, nbk, 1))) return rc;
        } else {
          g.A = g.B = limb0;
          if (i8blk) {  // the K-blocked copy, positions from nm
            g.A = g.B = h->ws_i8blk.as<int8_t>();
            g.img0 = nm;
            g.blk = 1;
          }
          g.s0 = nm;
          g.s_rows = ns;
          int64_t slots = nbk;
          if (fb0 < nb_s) {
            g.fsel = 1;
            g.fblk0 = (int32_t)fb0;
            slots = 2 * fb0;
          }
          if ((rc = launch_big(h, i8blk ? scfg : cfg, g, 1, slots))) return rc;
        }
      }
    }
    // 4. final lists -> outputs
    if ((rc = cand_compact(h, cb, nm, ns, 0, k))) return rc;
    if ((rc = cand_emit(h, cb, nm, ns, k, d_ids, d_scores, d_counts))) return rc;
#ifdef CMS_SCREEN_PROBE
    {
      unsigned long long pr[4][32][2];
      CMS_HIP(hipMemcpyFromSymbol(pr, HIP_SYMBOL(g_probe), sizeof(pr), 0, hipMemcpyDeviceToHost));
      for (int f = 0; f < 4; ++f)
        for (int r = 0; r < h->p.depth; ++r) {
          const unsigned long long dead = pr[f][r][0], live = pr[f][r][1];
          fprintf(stderr, "probe %s %s row %d: dead %llu alive %llu (%.1f%% dead)\n", f / 2 ? "fp4" : "i8",
                  f % 2 ? "WG" : "wave", r, dead, live, 100.0 * dead / (double)std::max(1ULL, dead + live));
        }
    }
#endif
  }
  // rows whose list overflowed (not expected): exact per-row recompute (whole
  // row, so a sharded job's merge still sees every pair once per shard at most:
  // the row's other partial lists are subsets of this exact list)
  std::vector<uint32_t> ovf(ns > 0 ? ns : 1);
  if (ns > 0) CMS_HIP(hipMemcpyAsync(ovf.data(), cb.ovf + nm, sizeof(uint32_t) * ns, hipMemcpyDeviceToHost, h->stream));
  CMS_HIP(hipStreamSynchronize(h->stream));
  std::vector<int64_t> pos, outp;
  for (int64_t i = 0; i < ns; ++i)
    if (ovf[i]) {
      pos.push_back(nm + i);
      outp.push_back(h->h_perm[nm + i]);
    }
  h->topk_redo += (int64_t)pos.size();
  if (!pos.empty() && (rc = slab_top_k_positions(h, pos, outp, k, d_ids, d_scores, d_counts))) return rc;
  return CMS_OK;
}

}  // namespace cms
