// cms_cosine_mls.hip -- multi-limb owners x single-limb owners on 256 x 192
// tiles: the M x S block of the all-pairs job's multi-limb slabs (config 4;
// DoubleCountMinSketch.cosine, T/impl/common/DoubleCountMinSketch.java:114-149,
// for every pair of a multi-limb owner with every other owner, the rows the
// TopItems.getTopUsers ranking of those owners needs, TopItems.java:91-136).
//
// A multi-limb owner has a counter >= 128, so its row does not fit one int8
// limb: it is split into LS 7-bit limbs (LS = 2, or 4 for counters >= 2^14)
// stored as "virtual limb rows" -- within each 32-row MFMA block, row 8g + i
// holds limb g % LS of owner (g / LS) * 8 + i, so the LS limbs of an owner land
// in accumulator elements e, e + 4, ... of one lane and fold exactly in
// registers (dot = sum_l acc_l << 7 l, < 2^49).  k_cosine_big ran this block
// on 256 x 128 tiles out of a 3-deep ring of 48 KiB stages (27 % MFMA busy):
// here the geometry is k_cosine_sym's -- 256 x 192 tiles, 8 waves of 64 x 96,
// a 5-deep ring of 64-B K stages filled by LDS-DMA from K-blocked images (the
// group's virtual limb rows re-laid by k_vl_blk, and the single-limb int8
// image the symmetric waves read) -- and the running minimum is the packed
// (exact dot << 5 | sketch row) state: rows are compared by fp32 estimates,
// in fp64 (__dmul_rn / __ddiv_rn, as Java) inside a 2^-17 margin, and the
// value is divided out once, exactly, at the end.  Each pair's similarity
// goes to the slab (the multi-limb owner's exact top-k and the single-limb
// owners' candidate offers are read from it, cms_topk.hip).
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cfloat>

#include "cms_device.h"
#include "cms_internal.h"
#include "cms_mfma.h"

namespace cms {

constexpr int kMA = 256, kMB = 192;  // A panel (virtual limb rows) x B panel (owners)
constexpr int kMNS = 5, kMBK = 64;   // ring depth, K bytes per row per stage

// Virtual limb rows (row-major, k_vl_build) -> the K-blocked image of
// cms_mfma.h (kImgBlk-row blocks, kMBK-byte slices); padding rows are zero.
__global__ __launch_bounds__(256) void k_vl_blk(const int8_t* vl, int64_t rows, int64_t dw, int8_t* img) {
  const int64_t r = blockIdx.x;
  const int8_t* src = r < rows ? vl + r * dw : nullptr;
  for (int64_t j = threadIdx.x * 16; j < dw; j += 256 * 16) {
    const int4 v = src ? *reinterpret_cast<const int4*>(src + j) : make_int4(0, 0, 0, 0);
    *reinterpret_cast<int4*>(img + blk_off(r, j, dw, kMBK)) = v;
  }
}

// the q-th workgroup of XCD x takes tile (q / C) * 8C + x C + q % C: the 8
// XCDs work on 8 neighbouring runs of C tiles at any time
__device__ __forceinline__ int mls_map(int bx, int C) {
  const int q = bx >> 3;
  return (q / C) * 8 * C + (bx & 7) * C + q % C;
}

template <int LS>
__global__ __launch_bounds__(512, 1) void k_cosine_mls(MlsArgs g) {
  constexpr int NSTAGE = kMNS, BK = kMBK, NW = 8;
  constexpr int OA = kMA / LS;  // owners per A panel
  constexpr int OG = 4 / LS;    // owner groups per 32-row block in one lane
  constexpr int kStageA = kMA * BK, kStageB = kMB * BK, kStage = kStageA + kStageB;
  constexpr int RPI = 1024 / BK;                 // rows per 1-KiB LDS-DMA instruction
  constexpr int OPA = kMA / RPI / NW;            // A instructions per wave per stage
  constexpr int RB = kMB / RPI;                  // B instructions per stage (all waves)
  constexpr int OPB_HI = (RB + NW - 1) / NW, OPB_LO = RB / NW;
  extern __shared__ __align__(16) unsigned char lds[];
  const int depth = g.depth;
  double* s_sa = reinterpret_cast<double*>(lds + NSTAGE * kStage);  // [depth][OA]
  double* s_sb = s_sa + depth * OA;                                   // [depth][192]

  // ---- tile: runs of ga x gb tiles (A panels fastest), B runs fastest ----
  const int C = g.ga * g.gb;
  const int lin = mls_map((int)blockIdx.x, C);
  if (lin >= g.nblk) return;
  const int gi = lin / C, l = lin - gi * C;
  const int ngb = (g.tilesB + g.gb - 1) / g.gb;
  const int ta = (gi / ngb) * g.ga + l % g.ga;
  const int tb = (gi % ngb) * g.gb + l / g.ga;
  if (ta >= g.tilesA || tb >= g.tilesB) return;  // the whole workgroup leaves before any barrier
  const int64_t a_own = min<int64_t>(OA, g.a_owners - (int64_t)ta * OA);
  const int64_t a_pos = g.a_pos0 + (int64_t)ta * OA;
  const int64_t b_pos = g.b_pos0 + (int64_t)tb * kMB;
  const int64_t b_n = min<int64_t>(kMB, g.b_rows - (int64_t)tb * kMB);
  if (a_own <= 0 || b_n <= 0) return;

  const int tid = threadIdx.x, lane = tid & 63, wid = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int wr = wid >> 1, wc = wid & 1;  // wave rows [wr * 64, +64), columns [wc * 96, +96)
  const int64_t rs = g.rs;
  const int cstages = g.kw / BK;
  const int total = depth * cstages;

  // sqrt norms of the panels' owners by LDS-DMA (32 doubles per instruction;
  // past-the-end owners land as zeros)
  constexpr int kPartsA = OA / 32, kParts = kPartsA + kMB / 32;
  for (int k = wid; k < kParts * depth; k += NW) {
    const int r = k / kParts, part = k % kParts;
    const bool isA = part < kPartsA;
    const int64_t first = isA ? part * 32 : (part - kPartsA) * 32;
    const int64_t cnt = max<int64_t>(0, min<int64_t>(32, (isA ? a_own : b_n) - first));
    const double* src = g.nsq_t + (int64_t)r * g.n + (isA ? a_pos : b_pos) + first;
    const __amdgpu_buffer_rsrc_t rsn = __builtin_amdgcn_make_buffer_rsrc((void*)src, (short)0, (int)(cnt * 8), 0x00020000);
    double* dst = isA ? s_sa + r * OA + first : s_sb + r * kMB + first;
    __builtin_amdgcn_raw_ptr_buffer_load_lds(rsn, (__attribute__((address_space(3))) void*)dst, 4, lane * 4, 0, 0, 0);
  }

  // ---- operand fills: K-blocked images, panels start on a kImgBlk block ----
  const int64_t a_vr = min<int64_t>(kMA, g.a_vrows - (int64_t)ta * kMA);
  const int64_t recA = (a_vr + kImgBlk - 1) / kImgBlk * kImgBlk * rs;
  const int64_t recB = (b_n + kImgBlk - 1) / kImgBlk * kImgBlk * rs;
  const __amdgpu_buffer_rsrc_t rsA =
      __builtin_amdgcn_make_buffer_rsrc((void*)(g.A + (int64_t)ta * kMA * rs), (short)0, (int)recA, 0x00020000);
  const __amdgpu_buffer_rsrc_t rsB =
      __builtin_amdgcn_make_buffer_rsrc((void*)(g.B + (b_pos - g.b_img0) * rs), (short)0, (int)recB, 0x00020000);
  constexpr int CPR = BK / 16;
  const int srow = wid * RPI + lane / CPR;
  const int slot = lane % CPR;
  const int32_t chunk = (slot ^ ((srow >> 2) & 3)) << 4;  // lds_off_bk<64>'s swizzle
  const int32_t bstep = kImgBlk * (int32_t)rs;
  const int32_t vo = (srow / kImgBlk) * bstep + (srow % kImgBlk) * BK + chunk;
  constexpr int UROWS = NW * RPI;
  static_assert(UROWS % kImgBlk == 0, "rounds start on image blocks");
  const int opb = wid < (RB % NW == 0 ? NW : RB % NW) ? OPB_HI : OPB_LO;
  auto issue = [&](int s, int slot_, int part) {
    const int32_t koff = s * (kImgBlk * BK);
    unsigned char* st = lds + (slot_ % NSTAGE) * kStage;
    if (part & 1) {
#pragma unroll
      for (int u = 0; u < OPA; ++u)
        __builtin_amdgcn_raw_ptr_buffer_load_lds(rsA, (__attribute__((address_space(3))) void*)(st + (wid + NW * u) * 1024),
                                                 16, vo + (u * UROWS / kImgBlk) * bstep, koff, 0, 0);
#pragma unroll
      for (int u = 0; u < OPB_LO; ++u)
        __builtin_amdgcn_raw_ptr_buffer_load_lds(
            rsB, (__attribute__((address_space(3))) void*)(st + kStageA + (wid + NW * u) * 1024), 16,
            vo + (u * UROWS / kImgBlk) * bstep, koff, 0, 0);
    }
    if ((part & 2) && OPB_HI > OPB_LO && opb == OPB_HI)
      __builtin_amdgcn_raw_ptr_buffer_load_lds(
          rsB, (__attribute__((address_space(3))) void*)(st + kStageA + (wid + NW * OPB_LO) * 1024), 16,
          vo + (OPB_LO * UROWS / kImgBlk) * bstep, koff, 0, 0);
  };

  i32x16 acc[2][3];
  // running Math.min per owner pair: (exact dot << 5 | sketch row), ~0 = none yet
  uint64_t mn[2][3][4 * OG];
#pragma unroll
  for (int i = 0; i < 2; ++i)
#pragma unroll
    for (int j = 0; j < 3; ++j) {
#pragma unroll
      for (int e = 0; e < 16; ++e) acc[i][j][e] = 0;
#pragma unroll
      for (int e = 0; e < 4 * OG; ++e) mn[i][j][e] = ~0ULL;
    }

  // the five fragments of k-step ks of a stage
  auto frags = [&](const unsigned char* A, int ks, i8x16* fa, i8x16* fb) {
    const int ch = 2 * ks + (lane >> 5);
#pragma unroll
    for (int j = 0; j < 3; ++j)
      fb[j] = *reinterpret_cast<const i8x16*>(A + kStageA + lds_off_bk<BK>(wc * 96 + j * 32 + (lane & 31), ch));
#pragma unroll
    for (int i = 0; i < 2; ++i)
      fa[i] = *reinterpret_cast<const i8x16*>(A + lds_off_bk<BK>(wr * 64 + i * 32 + (lane & 31), ch));
  };
  // k_cosine_sym's schedule (CMS_SYM_SCHED 3): the barrier between a stage's
  // two k-steps, the next stage's first fragments read behind the second
  // k-step's MFMAs, the slot just finished refilled at once
  constexpr int NVB = OPA + OPB_LO;
#pragma unroll
  for (int s = 0; s < NSTAGE; ++s) issue(min(s, total - 1), s, 3);  // every iteration issues: one vmcnt count
  if (opb == OPB_HI) wait_vmcnt<(OPA + OPB_HI) * (NSTAGE - 1)>();
  else wait_vmcnt<(OPA + OPB_LO) * (NSTAGE - 1)>();
  asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
  __builtin_amdgcn_s_barrier();
  asm volatile("" ::: "memory");
  i8x16 fa0[2], fb0[3];
  frags(lds, 0, fa0, fb0);

  int s_in_row = 0, r_next = 0;  // stage within the current sketch row, and that row (no per-stage division)
  for (int s = 0; s < total; ++s) {
    {
      const unsigned char* A = lds + (s % NSTAGE) * kStage;
      i8x16 fa1[2], fb1[3];
      frags(A, 1, fa1, fb1);
#pragma unroll
      for (int i = 0; i < 2; ++i)
#pragma unroll
        for (int j = 0; j < 3; ++j) acc[i][j] = __builtin_amdgcn_mfma_i32_32x32x32_i8(fa0[i], fb0[j], acc[i][j], 0, 0, 0);
#pragma unroll
      for (int m = 0; m < 6; ++m) {
        __builtin_amdgcn_sched_group_barrier(0x008, 1, 0);
        if (m < 5) __builtin_amdgcn_sched_group_barrier(0x100, 1, 0);
      }
      asm volatile("" ::: "memory");
      if (opb == OPB_HI) wait_vmcnt<(OPA + OPB_HI) * (NSTAGE - 2)>();
      else wait_vmcnt<(OPA + OPB_LO) * (NSTAGE - 2)>();
      asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
      __builtin_amdgcn_s_barrier();
      asm volatile("" ::: "memory");
      const int sn = min(s + NSTAGE, total - 1);
      issue(sn, s, 1);
      frags(lds + ((s + 1) % NSTAGE) * kStage, 0, fa0, fb0);
#pragma unroll
      for (int i = 0; i < 2; ++i)
#pragma unroll
        for (int j = 0; j < 3; ++j) acc[i][j] = __builtin_amdgcn_mfma_i32_32x32x32_i8(fa1[i], fb1[j], acc[i][j], 0, 0, 0);
#pragma unroll
      for (int m = 0; m < 6; ++m) {
        __builtin_amdgcn_sched_group_barrier(0x008, 1, 0);
        if (m < NVB) __builtin_amdgcn_sched_group_barrier(0x020, 1, 0);
        if (m >= 1 && m < 6) __builtin_amdgcn_sched_group_barrier(0x100, 1, 0);
      }
      issue(sn, s, 2);
    }
    if (++s_in_row != cstages) continue;
    s_in_row = 0;
    const int r = r_next++;
    // ---- sketch row r done (DoubleCountMinSketch.java:139-147) ----
    const double* sa_r = s_sa + r * OA;
    const double* sb_r = s_sb + r * kMB;
#pragma unroll
    for (int j = 0; j < 3; ++j) {
      const int col = wc * 96 + j * 32 + (lane & 31);
      const double sb = sb_r[col];
      if (sb == 0.0) continue;  // den == 0: this sketch row does not qualify
      const float rb = __builtin_amdgcn_rcpf((float)sb);
#pragma unroll
      for (int i = 0; i < 2; ++i)
#pragma unroll
        for (int og = 0; og < OG; ++og)
#pragma unroll
          for (int q = 0; q < 4; ++q) {
            const int ol = (wr * 64 + i * 32) / LS + og * 8 + q + 4 * (lane >> 5);
            const double sa = sa_r[ol];
            if (sa == 0.0) continue;
            int64_t dot = 0;
#pragma unroll
            for (int lb = 0; lb < LS; ++lb) dot += (int64_t)acc[i][j][q + 4 * (og * LS + lb)] << (7 * lb);
            uint64_t& m = mn[i][j][og * 4 + q];
            bool take = m == ~0ULL;
            if (!take) {
              const int r0 = (int)(m & 31ULL);
              const int64_t d0 = (int64_t)(m >> 5);
              const double sa0 = s_sa[r0 * OA + ol], sb0 = s_sb[r0 * kMB + col];
              const float est = (float)dot * __builtin_amdgcn_rcpf((float)sa) * rb;
              const float est0 = (float)d0 * __builtin_amdgcn_rcpf((float)sa0) * __builtin_amdgcn_rcpf((float)sb0);
              if (est < est0 * (1.0f - 0x1p-17f)) {
                take = true;
              } else if (est <= est0 * (1.0f + 0x1p-17f)) {  // too close for fp32: the exact values
                take = __ddiv_rn((double)dot, __dmul_rn(sa, sb)) < __ddiv_rn((double)d0, __dmul_rn(sa0, sb0));
              }
            }
            if (take) m = ((uint64_t)dot << 5) | (uint64_t)r;
          }
    }
#pragma unroll
    for (int i = 0; i < 2; ++i)
#pragma unroll
      for (int j = 0; j < 3; ++j)
#pragma unroll
        for (int e = 0; e < 16; ++e) acc[i][j][e] = 0;
  }
  wait_vmcnt<0>();  // the repeat loads land before the workgroup's LDS is released

  // ---- NaN when no row qualified, then normalizeWeightResult; the slab ----
#pragma unroll
  for (int j = 0; j < 3; ++j) {
    const int col = wc * 96 + j * 32 + (lane & 31);
    if (col >= b_n) continue;
    const int64_t bp = b_pos + col;
#pragma unroll
    for (int i = 0; i < 2; ++i)
#pragma unroll
      for (int og = 0; og < OG; ++og)
#pragma unroll
        for (int q = 0; q < 4; ++q) {
          const int ol = (wr * 64 + i * 32) / LS + og * 8 + q + 4 * (lane >> 5);
          if (ol >= a_own) continue;
          const int64_t ap = a_pos + ol;
          if (ap < g.q0 || ap >= g.q0 + g.qcount) continue;
          const uint64_t m = mn[i][j][og * 4 + q];
          double rr = __builtin_nan("");
          if (m != ~0ULL) {
            const int r0 = (int)(m & 31ULL);
            rr = __ddiv_rn((double)(int64_t)(m >> 5), __dmul_rn(s_sa[r0 * OA + ol], s_sb[r0 * kMB + col]));
            if (g.weighted) rr = rr < 0.0 ? -1.0 : 1.0;  // scaleFactor 1 - 1/(0+1) = 0
            if (rr > 1.0) rr = 1.0;
          }
          g.out[(ap - g.q0) * g.ldo + bp] = rr;
        }
  }
}

size_t mls_lds_bytes(int depth) {
  return (size_t)kMNS * (kMA + kMB) * kMBK + (size_t)depth * (kMA + kMB) * sizeof(double);
}

bool mls_eligible(cms_handle* h) {
  return h->p.depth <= 32 && (h->p.width % kMBK) == 0 && h->sym_sw == kMBK && mls_lds_bytes(h->p.depth) <= 160 * 1024;
}

int vl_blk_prepare(cms_handle* h, int gi) {
  auto& G = h->vl[gi];
  if (G.bready) return CMS_OK;
  const int64_t rows = (G.rows + kImgBlk - 1) / kImgBlk * kImgBlk;
  CMS_HIP(G.bbuf.ensure((size_t)rows * (size_t)h->dw));
  TimedScope ts(h, "limb_prep");
  hipLaunchKernelGGL(k_vl_blk, dim3((unsigned)rows), dim3(256), 0, h->stream, G.buf.as<int8_t>(), G.rows, h->dw,
                     G.bbuf.as<int8_t>());
  CMS_HIP(hipGetLastError());
  G.bready = true;
  return CMS_OK;
}

int launch_mls(cms_handle* h, MlsArgs g, int ls) {
  const int64_t vneed = (g.a_owners * ls + 31) / 32 * 32;  // virtual rows holding the launch's owners
  g.tilesA = (int32_t)((std::min<int64_t>(vneed, g.a_vrows) + kMA - 1) / kMA);
  g.tilesB = (int32_t)((g.b_rows + kMB - 1) / kMB);
  if (g.tilesA <= 0 || g.tilesB <= 0) return CMS_OK;
  // runs of ga A panels x gb B panels (32 tiles: an XCD's workgroups at once)
  g.ga = std::min<int32_t>(8, g.tilesA);
  g.gb = std::max<int32_t>(1, 32 / g.ga);
  const int64_t C = (int64_t)g.ga * g.gb;
  const int64_t groups = (int64_t)((g.tilesA + g.ga - 1) / g.ga) * ((g.tilesB + g.gb - 1) / g.gb);
  const int64_t nblk = groups * C;
  if (nblk >= (int64_t)1 << 31) return CMS_E_PARAM;
  g.nblk = (int32_t)nblk;
  const int64_t grid = (nblk + 8 * C - 1) / (8 * C) * (8 * C);
  const size_t bytes = mls_lds_bytes(g.depth);
  static bool attr = [] {
    (void)hipFuncSetAttribute((const void*)k_cosine_mls<2>, hipFuncAttributeMaxDynamicSharedMemorySize, 160 * 1024);
    (void)hipFuncSetAttribute((const void*)k_cosine_mls<4>, hipFuncAttributeMaxDynamicSharedMemorySize, 160 * 1024);
    return true;
  }();
  (void)attr;
  if (ls == 2) hipLaunchKernelGGL(k_cosine_mls<2>, dim3((unsigned)grid), dim3(512), bytes, h->stream, g);
  else if (ls == 4) hipLaunchKernelGGL(k_cosine_mls<4>, dim3((unsigned)grid), dim3(512), bytes, h->stream, g);
  else return CMS_E_PARAM;
  CMS_HIP(hipGetLastError());
  return CMS_OK;
}

}  // namespace cms
