// cms_cosine_sym.hip -- the all-pairs top-k's symmetric waves with 256 x 192
// tiles (config 4's hot loop; DoubleCountMinSketch.cosine,
// T/impl/common/DoubleCountMinSketch.java:114-149, offered to both owners'
// candidate lists as TopItems.getTopUsers would rank them, TopItems.java:91-136).
//
// Why a second kernel.  k_cosine_big's 256 x 128 tile keeps every pair's
// running Math.min as an fp64 value (2 registers per output, 128 of its 234
// VGPRs).  Its waves are bound by the rate at which a CU can pull operand
// bytes into LDS (~30 B/clk from L2), so the lever is bytes per MFMA, i.e. a
// bigger tile -- which the fp64 state does not leave room for.  Here the state
// is ONE register per output: the sketch row r* that holds the minimum so far
// and its exact integer dot AB* (u32: AB* << rbits | r*).  The row cosine is
// AB / (sqrt(A) * sqrt(B)) with sqrt(A), sqrt(B) in LDS for every sketch row,
// so any state value can be re-derived exactly:
//   - at each row boundary the new row's value and the stored one are first
//     compared by fp32 estimates (relative error < 2^-20 each); only when the
//     two lie within 2^-17 of each other are both recomputed in fp64
//     (__dmul_rn / __ddiv_rn, as Java does) and compared exactly;
//   - the admitted value is recomputed once at the end from (r*, AB*).
// So the minimum, and the value reported, are the reference's exactly.  The
// same fp32 estimate drives the threshold screening (a pair whose estimate is
// below both owners' admission thresholds can never be admitted).
//
// Geometry.  Blocks of kSymBlk = 768 rows; a block pair {I, J} is 3 x 4
// workgroups (A panels of 256 rows, B panels of 192); 8 waves in 4 x 2, each
// 64 x 96 outputs = 2 x 3 MFMA 32x32 tiles (96 accumulators + 96 states per
// lane).  K is staged 64 B per row per stage by buffer LDS-DMA from the
// K-blocked images (kImgBlk-row blocks, a stage of a panel is a few
// contiguous runs) into a 5-deep ring of 28 KiB stages.
#include <hip/hip_fp16.h>
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cfloat>
#include <cmath>

#include "cms_device.h"
#include "cms_internal.h"
#include "cms_mfma.h"

#ifndef CMS_SYM_PROBE
// bound analysis builds only (build_lib.py --define), bit flags: 1 every
// workgroup loads the same panels, 2 no row-boundary work, 4 no MFMAs
#define CMS_SYM_PROBE 0
#endif
#ifndef CMS_SYM_SCHED
// 0: refill loads before the MFMAs, 1: interleaved with them, 2: also the next
// k-step's fragments, 3: the barrier between the two k-steps (f4 -4 %, i8 -6 % over 2)
#define CMS_SYM_SCHED 3
#endif

namespace cms {

#ifndef CMS_SYM_WAVES
#define CMS_SYM_WAVES 8
#endif
constexpr int kSymNW = CMS_SYM_WAVES;  // waves per workgroup (8: two per SIMD, 4: one)
// A panel rows x B panel rows per workgroup: 256 x 192 on 8 waves (64 x 96 per
// wave), 192 x 192 on 4 waves (96 x 96 per wave, 512 registers)
constexpr int kSA = kSymNW == 4 ? 192 : 256, kSB = 192;
constexpr int kPA = kSymBlk / kSA;   // 3 A panels per block
constexpr int kPB = kSymBlk / kSB;   // 4 B panels per block
constexpr int kSub = kPA * kPB;      // 12 workgroups per block pair
constexpr uint32_t kEmpty = 0xFFFFFFFFu;  // no sketch row qualified yet (NaN)

__device__ __forceinline__ uint32_t block_map(int bx, int nblk) {
  // contiguous ranges of the linear index per XCD (workgroup bx runs on XCD bx % 8)
  const int xcd = bx & 7, q8 = nblk >> 3, r8 = nblk & 7;
  return (uint32_t)((xcd < r8 ? xcd * (q8 + 1) : r8 * (q8 + 1) + (xcd - r8) * q8) + (bx >> 3));
}

// the XCDs side by side: the q-th workgroup of XCD x takes tile
// (q / C) * 8C + x C + q % C, so at any time the 8 XCDs work on neighbouring
// runs of C tiles (one rectangle of block pairs) -- each XCD's run shares its
// panels in its own L2, the 8 runs share theirs in the Infinity Cache.  The
// grid is rounded up to 8C; tiles past the end leave at once.
__device__ __forceinline__ uint32_t xcd_chunk_map(int bx, int C) {
  const int q = bx >> 3;
  return (uint32_t)((q / C) * 8 * C + (bx & 7) * C + q % C);
}

// Row cosines as the reference forms them: v = AB / (sa * sb), both fp64
// operations rounded (DoubleCountMinSketch.java:139-147).  Whether v < v0
// without the two divisions: rounding is monotonic, so AB / D < AB0 / D0
// exactly (D = rn(sa sb), D0 = rn(sa0 sb0) > 0) implies v <= v0, equal only
// when both round to the same double -- either row then yields the same
// minimum.  AB * D0 < AB0 * D is decided exactly on the FMA-split products
// (p + e, |e| <= ulp(p) / 2; p1 < p2 implies p1 + e1 <= p2 + e2).
__device__ __forceinline__ bool exact_less(double ab, double sa, double sb, double ab0, double sa0, double sb0) {
  const double D = __dmul_rn(sa, sb), D0 = __dmul_rn(sa0, sb0);
  const double p1 = __dmul_rn(ab, D0), e1 = __fma_rn(ab, D0, -p1);
  const double p2 = __dmul_rn(ab0, D), e2 = __fma_rn(ab0, D, -p2);
  return p1 < p2 || (p1 == p2 && e1 < e2);
}

template <int FMT>
__device__ __forceinline__ typename AccOf<FMT>::type sym_mma(const i8x16& a, const i8x16& b,
                                                             typename AccOf<FMT>::type c) {
#if CMS_SYM_PROBE & 4  // bound analysis: the fragments are consumed, no MFMA issued
  c[0] += (int)a[0] ^ (int)b[0];
  return c;
#else
  return mfma_step<FMT>(a, b, c);
#endif
}

template <int NSTAGE, int BK, int FMT, int NW>
__device__ __forceinline__ void sym_tile(SymArgs g, int bx) {
  using AccT = typename AccOf<FMT>::type;
  // NW waves in (NW/2) x 2; a wave holds TI x 3 MFMA tiles (TI = 2 at 8 waves;
  // 3 at 4 waves: one wave per SIMD with 512 registers, 6 fragments per 9 MFMAs)
  constexpr int TI = kSA / (NW / 2) / 32, WROWS = 32 * TI, NAW = (TI * 48 + 31) / 32;
  static_assert(NW == 4 || NW == 8, "4 or 8 waves");
  constexpr int kStageA = kSA * BK, kStageB = kSB * BK, kStage = kStageA + kStageB;
  constexpr int RPI = 1024 / BK;                 // rows per 1-KiB LDS-DMA instruction
  constexpr int OPA = kSA / RPI / NW;            // A instructions per wave per stage
  constexpr int RB = kSB / RPI;                  // B instructions per stage (all waves)
  constexpr int OPB_HI = (RB + NW - 1) / NW, OPB_LO = RB / NW;  // waves < RB % NW issue one more
  static_assert(kSA % (NW * RPI) == 0, "A rows per round");
  extern __shared__ __align__(16) unsigned char lds[];
  const int depth = g.depth;
  double* s_sa = reinterpret_cast<double*>(lds + NSTAGE * kStage);  // [depth][256]
  double* s_sb = s_sa + depth * kSA;                                  // [depth][192]
  float* s_ta = reinterpret_cast<float*>(s_sb + depth * kSB);        // admission thresholds, rounded down
  float* s_tb = s_ta + kSA;

  // ---- which tile: band of waves, block pair {I, J}, A panel, B panel ----
  // a refresh's sparse pair set (tsel) is spread over the XCDs round-robin
  const int lin = g.tsel ? bx : (g.xchunk ? (int)xcd_chunk_map(bx, g.xchunk) : (int)block_map(bx, g.nblk));
  if (lin >= g.nblk) return;
  int c, sub, wv;
  if (g.rect) {
    const int per = kSub * g.si * g.sj;
    const int blk = lin / per, loc = lin - blk * per;
    const int ib = blk / g.njc, jc = blk - ib * g.njc;
    sub = loc % kSub;
    const int rest = loc / kSub;
    const int li = rest / g.sj, lj = rest - li * g.sj;
    c = ib * g.si + li;
    if (c >= g.nb) return;
    wv = ib * g.si + g.wave + jc * g.sj + lj - c;  // unwrapped J' - I
    if (wv < g.wave || wv >= g.wave + g.band) return;
  } else {
    const int per = kSub * g.band;
    c = lin / per;
    const int rem = lin - c * per;
    sub = rem % kSub;
    wv = g.wave + rem / kSub;
  }
  int I = c;
  if (g.fsel) {  // only pairs with a block below fblk0 (see k_cosine_big)
    if (c >= g.fblk0) {
      I = ((c - g.fblk0 - wv) % g.nb + g.nb) % g.nb;
      if (I < g.fblk0) return;
    }
  }
  if ((g.nb & 1) == 0 && 2 * wv == g.nb && 2 * I >= g.nb) return;  // {I, I + nb/2} once
  const int J = (I + wv) % g.nb;
  if (g.tsel) {  // incremental refresh: block pairs holding a touched owner only
    auto touched = [&](int b) { return (b >= g.ts0 && b < g.ts1) || (b >= g.ts2 && b < g.ts3); };
    if (!touched(I) && !touched(J)) return;
  }
  const bool diag = I == J;
  const int pa = sub / kPB, pb = sub - pa * kPB;
  const int64_t a_pos0 = g.s0 + (int64_t)I * kSymBlk + pa * kSA;
  const int64_t b_pos0 = g.s0 + (int64_t)J * kSymBlk + pb * kSB;
  const int64_t a_rows = min<int64_t>(kSA, g.s0 + g.s_rows - a_pos0);
  const int64_t b_rows = min<int64_t>(kSB, g.s0 + g.s_rows - b_pos0);
  if (a_rows <= 0 || b_rows <= 0) return;          // the whole workgroup leaves before any barrier
  if (diag && a_pos0 >= b_pos0 + kSB - 1) return;  // every pair of the tile has a >= b

  const int tid = threadIdx.x, lane = tid & 63, wid = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int wr = wid >> 1, wc = wid & 1;  // wave rows [wr * WROWS, +WROWS), columns [wc * 96, +96)
  const int64_t rs = g.rs;
  const int cstages = g.kw / BK;
  const int total = depth * cstages;

  // sqrt norms of the panels' owners by LDS-DMA (256 B = 32 doubles per
  // instruction; past-the-end owners land as zeros), thresholds as fp16
  // rounded toward -inf (never above the threshold)
  constexpr int kPartsA = kSA / 32, kParts = (kSA + kSB) / 32;
  for (int k = wid; k < kParts * depth; k += NW) {
    const int r = k / kParts, part = k % kParts;
    const bool isA = part < kPartsA;
    const int64_t first = isA ? part * 32 : (part - kPartsA) * 32;
    const int64_t lim = isA ? a_rows : b_rows;
    const int64_t cnt = max<int64_t>(0, min<int64_t>(32, lim - first));
    const double* src = g.nsq_t + (int64_t)r * g.n + (isA ? a_pos0 : b_pos0) + first;
    const __amdgpu_buffer_rsrc_t rsn = __builtin_amdgcn_make_buffer_rsrc((void*)src, (short)0, (int)(cnt * 8), 0x00020000);
    double* dst = isA ? s_sa + r * kSA + first : s_sb + r * kSB + first;
    __builtin_amdgcn_raw_ptr_buffer_load_lds(rsn, (__attribute__((address_space(3))) void*)dst, 4, lane * 4, 0, 0, 0);
  }
  // thresholds: the launch's fp32 copy (rounded toward -inf) by LDS-DMA too,
  // 256 B per instruction, so no load latency stands before the ring's fill
  // (past-the-end owners land as 0: their rows never qualify, den == 0)
  constexpr int kTIA = kSA / 64, kTI = (kSA + kSB) / 64;
  for (int k = wid; k < kTI; k += NW) {
    const bool isA = k < kTIA;
    const int64_t first = (isA ? k : k - kTIA) * 64;
    const int64_t cnt = max<int64_t>(0, min<int64_t>(64, (isA ? a_rows : b_rows) - first));
    const float* src = g.thr32 + (isA ? a_pos0 : b_pos0) + first;
    const __amdgpu_buffer_rsrc_t rst = __builtin_amdgcn_make_buffer_rsrc((void*)src, (short)0, (int)(cnt * 4), 0x00020000);
    float* dst = (isA ? s_ta : s_tb) + first;
    __builtin_amdgcn_raw_ptr_buffer_load_lds(rst, (__attribute__((address_space(3))) void*)dst, 4, lane * 4, 0, 0, 0);
  }

  // ---- operand fills: K-blocked images, panels start on a kImgBlk block ----
  const int64_t recA = (a_rows + kImgBlk - 1) / kImgBlk * kImgBlk * rs;
  const int64_t recB = (b_rows + kImgBlk - 1) / kImgBlk * kImgBlk * rs;
#if CMS_SYM_PROBE & 1  // bound analysis: every workgroup streams the image's first panels (L2-resident)
  const int64_t a_img = 0, b_img = 0;
#else
  const int64_t a_img = a_pos0 - g.img0, b_img = b_pos0 - g.img0;
#endif
  const __amdgpu_buffer_rsrc_t rsA =
      __builtin_amdgcn_make_buffer_rsrc((void*)(g.img + a_img * rs), (short)0, (int)recA, 0x00020000);
  const __amdgpu_buffer_rsrc_t rsB =
      __builtin_amdgcn_make_buffer_rsrc((void*)(g.img + b_img * rs), (short)0, (int)recB, 0x00020000);
  // instruction u of wave wid fills panel rows [(wid + NW u) RPI, +RPI); lane i
  // lands at byte 16 i (row (wid + 8u) RPI + i / CPR, slot i % CPR) and
  // fetches the chunk the XOR swizzle puts there
  constexpr int CPR = BK / 16;
  const int srow = wid * RPI + lane / CPR;
  const int slot = lane % CPR;
  const int32_t chunk = (BK == 128 ? (slot ^ ((srow >> 1) & 7)) : (slot ^ ((srow >> 2) & 3))) << 4;
  const int32_t bstep = kImgBlk * (int32_t)rs;
  const int32_t vo = (srow / kImgBlk) * bstep + (srow % kImgBlk) * BK + chunk;
  constexpr int UROWS = NW * RPI;  // panel rows per round of instructions (a multiple of kImgBlk)
  static_assert(UROWS % kImgBlk == 0, "rounds start on image blocks");
  const int opb = wid < (RB % NW == 0 ? NW : RB % NW) ? OPB_HI : OPB_LO;
  // stage s's data into ring slot `slot`; `part` 1: the loads every wave
  // issues, 2: the extra B load of waves < RB % NW, 3: both
  auto issue = [&](int s, int slot, int part) {
    const int32_t koff = s * (kImgBlk * BK);
    unsigned char* st = lds + (slot % NSTAGE) * kStage;
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

  AccT acc[TI][3];
  uint32_t st[TI][3][16];
  uint32_t alive[NAW];  // bit (i*3+j)*16 + e: the pair may still be admitted
#pragma unroll
  for (int w = 0; w < NAW; ++w) alive[w] = ~0u;
#pragma unroll
  for (int i = 0; i < TI; ++i)
#pragma unroll
    for (int j = 0; j < 3; ++j)
#pragma unroll
      for (int e = 0; e < 16; ++e) {
        acc[i][j][e] = 0;
        st[i][j][e] = kEmpty;
      }
  const uint32_t rbits = (uint32_t)g.rbits, rmask = (1u << rbits) - 1u;
  // The running minimum of an output (kEmpty: no row qualified yet) is kept
  // in one of two forms.  Estimate form (bit 31 clear): the fp32 estimate
  // AB*/(sa* sb*) with its low rbits mantissa bits replaced by the row r*;
  // its relative error is <= 2^-21 (two rcp, two products) + 2^(rbits-23),
  // so AB* = rint(est * sa* * sb*) is exact while AB* <= ab_est_max, and a
  // row boundary compares against it without looking row r* up.  Exact form
  // (bit 31 set): AB* << rbits | r*, for larger dots (int8 rows; fp4 rows
  // always take the estimate form, sym_eligible checks their bound).
  const float ab_est_max = floorf(0.5f / (0x1p-21f + __builtin_ldexpf(1.0f, (int)rbits - 23)));
#if CMS_SYM_PROBE & 2
  float probe_sink = 0.0f;
#endif

  // the five fragments of k-step ks of a stage
  auto frags = [&](const unsigned char* A, int ks, i8x16* fa, i8x16* fb) {
    const int ch = 2 * ks + (lane >> 5);
#pragma unroll
    for (int j = 0; j < 3; ++j)
      fb[j] = *reinterpret_cast<const i8x16*>(A + kStageA + lds_off_bk<BK>(wc * 96 + j * 32 + (lane & 31), ch));
#pragma unroll
    for (int i = 0; i < TI; ++i)
      fa[i] = *reinterpret_cast<const i8x16*>(A + lds_off_bk<BK>(wr * WROWS + i * 32 + (lane & 31), ch));
  };
#if CMS_SYM_SCHED == 3
  // Barrier between a stage's two k-steps: the first k-step's MFMAs run
  // through the wait for the NEXT stage, whose first fragments are then read
  // behind the second k-step's MFMAs -- no fragment-read bubble after the
  // barrier, and the slot just finished is refilled at once (every slot of
  // the ring is in flight or being read).
  static_assert(BK == 64, "two k-steps per stage");
  constexpr int NVB = OPA + OPB_LO;
#pragma unroll
  for (int s = 0; s < NSTAGE; ++s) issue(min(s, total - 1), s, 3);  // every iteration issues: one vmcnt count
  if (opb == OPB_HI) wait_vmcnt<(OPA + OPB_HI) * (NSTAGE - 1)>();
  else wait_vmcnt<(OPA + OPB_LO) * (NSTAGE - 1)>();
  asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
  __builtin_amdgcn_s_barrier();
  asm volatile("" ::: "memory");
  i8x16 fa0[TI], fb0[3];
  frags(lds, 0, fa0, fb0);
#else
#pragma unroll
  for (int s = 0; s < NSTAGE - 1; ++s)
#if CMS_SYM_SCHED
    issue(min(s, total - 1), s, 3);  // every iteration issues: one vmcnt count for all stages
#else
    if (s < total) issue(s, s, 3);
#endif
#endif

  int s_in_row = 0, r_next = 0;  // stage within the current sketch row, and that row (no per-stage division)
  for (int s = 0; s < total; ++s) {
#if CMS_SYM_SCHED == 3
    {
      const unsigned char* A = lds + (s % NSTAGE) * kStage;
      i8x16 fa1[TI], fb1[3];
      frags(A, 1, fa1, fb1);
#pragma unroll
      for (int i = 0; i < TI; ++i)
#pragma unroll
        for (int j = 0; j < 3; ++j) acc[i][j] = sym_mma<FMT>(fa0[i], fb0[j], acc[i][j]);
#pragma unroll
      for (int m = 0; m < TI * 3; ++m) {
        __builtin_amdgcn_sched_group_barrier(0x008, 1, 0);
        if (m < TI + 3) __builtin_amdgcn_sched_group_barrier(0x100, 1, 0);
      }
      // stage s+1 landed (the NSTAGE-2 younger stages stay in flight); every
      // wave's reads of slot s are done past the barrier
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
      for (int i = 0; i < TI; ++i)
#pragma unroll
        for (int j = 0; j < 3; ++j) acc[i][j] = sym_mma<FMT>(fa1[i], fb1[j], acc[i][j]);
#pragma unroll
      for (int m = 0; m < TI * 3; ++m) {
        __builtin_amdgcn_sched_group_barrier(0x008, 1, 0);
        if (m < NVB) __builtin_amdgcn_sched_group_barrier(0x020, 1, 0);
        if (m >= 1 && m < TI + 4) __builtin_amdgcn_sched_group_barrier(0x100, 1, 0);
      }
      issue(sn, s, 2);
    }
#else
    // stage s landed: at most the (NSTAGE-2) younger stages stay in flight
    asm volatile("" ::: "memory");
#if CMS_SYM_SCHED
    if (opb == OPB_HI) wait_vmcnt<(OPA + OPB_HI) * (NSTAGE - 2)>();
    else wait_vmcnt<(OPA + OPB_LO) * (NSTAGE - 2)>();
#else
    if (s + NSTAGE - 2 < total) {
      if (opb == OPB_HI) wait_vmcnt<(OPA + OPB_HI) * (NSTAGE - 2)>();
      else wait_vmcnt<(OPA + OPB_LO) * (NSTAGE - 2)>();
    } else {
      wait_vmcnt<0>();
    }
#endif
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
    __builtin_amdgcn_s_barrier();
    asm volatile("" ::: "memory");
    const unsigned char* A = lds + (s % NSTAGE) * kStage;
    const unsigned char* B = A + kStageA;
#if CMS_SYM_SCHED
    // refill the slot read in iteration s-1 (past the last stage: a repeat of
    // it into that free slot, so every iteration issues the same loads), the
    // common loads between the first k-step's MFMAs, the extra one after the MFMAs
    {
      const int sn = min(s + NSTAGE - 1, total - 1);
#pragma unroll
      for (int ks = 0; ks < BK / 32; ++ks) {
        const int ch = 2 * ks + (lane >> 5);
        i8x16 fb[3], fa[TI];
#pragma unroll
        for (int j = 0; j < 3; ++j)
          fb[j] = *reinterpret_cast<const i8x16*>(B + lds_off_bk<BK>(wc * 96 + j * 32 + (lane & 31), ch));
#pragma unroll
        for (int i = 0; i < TI; ++i)
          fa[i] = *reinterpret_cast<const i8x16*>(A + lds_off_bk<BK>(wr * WROWS + i * 32 + (lane & 31), ch));
#pragma unroll
        for (int i = 0; i < TI; ++i)
#pragma unroll
          for (int j = 0; j < 3; ++j) acc[i][j] = sym_mma<FMT>(fa[i], fb[j], acc[i][j]);
        if (ks == 0) issue(sn, s + NSTAGE - 1, 1);
      }
      constexpr int NV = OPA + OPB_LO, NF = TI + 3, NM = TI * 3, KS = BK / 32;
      static_assert(NV <= NM * KS && NF >= 3 && NM >= 4, "schedule shape");
      // per k-step: its MFMAs one at a time, the refill loads one after each
      // MFMA from the first on; CMS_SYM_SCHED 2 also reads the next k-step's
      // fragments behind the last four MFMAs (as the registers they replace free up)
      __builtin_amdgcn_sched_group_barrier(0x100, NF, 0);  // k-step 0 fragments
#pragma unroll
      for (int ks = 0; ks < KS; ++ks) {
#pragma unroll
        for (int m = 0; m < NM; ++m) {
          __builtin_amdgcn_sched_group_barrier(0x008, 1, 0);
          if (ks * NM + m < NV) __builtin_amdgcn_sched_group_barrier(0x020, 1, 0);
          if (CMS_SYM_SCHED == 2 && ks + 1 < KS && m >= NM - 4) {
            if (m == NM - 1) __builtin_amdgcn_sched_group_barrier(0x100, NF - 3, 0);
            else __builtin_amdgcn_sched_group_barrier(0x100, 1, 0);
          }
        }
        if (CMS_SYM_SCHED != 2 && ks + 1 < KS) __builtin_amdgcn_sched_group_barrier(0x100, NF, 0);
      }
      issue(sn, s + NSTAGE - 1, 2);
    }
#else
    if (s + NSTAGE - 1 < total) issue(s + NSTAGE - 1, s + NSTAGE - 1, 3);  // refill the slot read in iteration s-1
#pragma unroll
    for (int ks = 0; ks < BK / 32; ++ks) {
      // the k-step's five fragments first, then its six MFMAs
      const int ch = 2 * ks + (lane >> 5);
      i8x16 fb[3], fa[TI];
#pragma unroll
      for (int j = 0; j < 3; ++j)
        fb[j] = *reinterpret_cast<const i8x16*>(B + lds_off_bk<BK>(wc * 96 + j * 32 + (lane & 31), ch));
#pragma unroll
      for (int i = 0; i < TI; ++i)
        fa[i] = *reinterpret_cast<const i8x16*>(A + lds_off_bk<BK>(wr * WROWS + i * 32 + (lane & 31), ch));
#pragma unroll
      for (int i = 0; i < TI; ++i)
#pragma unroll
        for (int j = 0; j < 3; ++j) acc[i][j] = sym_mma<FMT>(fa[i], fb[j], acc[i][j]);
    }
#endif
#endif  // CMS_SYM_SCHED == 3
    if (++s_in_row != cstages) continue;
    s_in_row = 0;
    const int r = r_next++;
#if CMS_SYM_PROBE & 2  // bound analysis: no row-boundary screening / minimum (the MFMAs stay live)
#pragma unroll
    for (int i = 0; i < TI; ++i)
#pragma unroll
      for (int j = 0; j < 3; ++j) probe_sink += (float)acc[i][j][0];
    continue;
#endif
    // ---- sketch row r done (DoubleCountMinSketch.java:139-147) ----
    const double* sa_r = s_sa + r * kSA;
    const double* sb_r = s_sb + r * kSB;
    uint32_t any_alive = 0u;
#pragma unroll
    for (int w = 0; w < NAW; ++w) any_alive |= alive[w];
    if constexpr (FMT == 1) {
      // fp4: the running minimum is kept as its fp32 estimate (low rbits of
      // the mantissa replaced by the row), from which the exact dot AB* is
      // recovered at the end (sym_eligible bounds the error below 1/2).  So a
      // row boundary needs no LDS lookups of the state's row and runs
      // branch-free over the 96 outputs; only near ties (within 2^-17) take
      // the exact fp64 comparison, in a second pass few waves enter.
      if (__any(any_alive != 0u)) {
#pragma unroll
        for (int j = 0; j < 3; ++j) {
          const int col = wc * 96 + j * 32 + (lane & 31);
          const double sb = sb_r[col];
          const float rb = __builtin_amdgcn_rcpf((float)sb);
          const float tb = s_tb[col];
#pragma unroll
          for (int i = 0; i < TI; ++i) {
            const int g0 = (i * 3 + j) * 16;  // the 16 outputs of MFMA tile (i, j): one test when the wave's are all dead
            if (!__any(((alive[g0 >> 5] >> (g0 & 31)) & 0xFFFFu) != 0u)) continue;
#pragma unroll
            for (int e = 0; e < 16; ++e) {
              const int bit = (i * 3 + j) * 16 + e;
              const uint32_t m = 1u << (bit & 31);
              if (!(alive[bit >> 5] & m)) continue;
              const int row = wr * WROWS + i * 32 + (e & 3) + 8 * (e >> 2) + 4 * (lane >> 5);
              const double sa = sa_r[row];
              if (sa == 0.0 || sb == 0.0) continue;  // den == 0: this sketch row does not qualify
              const float est = (float)acc[i][j][e] * __builtin_amdgcn_rcpf((float)sa) * rb;
              if (est < fminf(s_ta[row], tb) - 4e-6f) {  // can never be admitted
                alive[bit >> 5] &= ~m;
                continue;
              }
              uint32_t& sv = st[i][j][e];
              const float est0 = __uint_as_float(sv & ~rmask);  // NaN when empty
              bool take = sv == kEmpty || est < est0 * (1.0f - 0x1p-17f);
              if (!take && est <= est0 * (1.0f + 0x1p-17f)) {  // too close for fp32: the exact values
                const int rr = (int)(sv & rmask);
                const double sa0 = s_sa[rr * kSA + row], sb0 = s_sb[rr * kSB + col];
                take = exact_less((double)acc[i][j][e], sa, sb, rint((double)est0 * sa0 * sb0), sa0, sb0);
              }
              if (take) sv = (__float_as_uint(est) & ~rmask) | (uint32_t)r;
            }
          }
        }
      }
    } else if (__any(any_alive != 0u)) {  // int8: estimate or exact form
#pragma unroll
      for (int j = 0; j < 3; ++j) {
        const int col = wc * 96 + j * 32 + (lane & 31);
        const double sb = sb_r[col];
        const float rb = __builtin_amdgcn_rcpf((float)sb);
        const float tb = s_tb[col];
#pragma unroll
        for (int i = 0; i < TI; ++i) {
          const int g0 = (i * 3 + j) * 16;
          if (!__any(((alive[g0 >> 5] >> (g0 & 31)) & 0xFFFFu) != 0u)) continue;
#pragma unroll
          for (int e = 0; e < 16; ++e) {
            const int bit = (i * 3 + j) * 16 + e;
            const uint32_t m = 1u << (bit & 31);
            if (!(alive[bit >> 5] & m)) continue;
            const int row = wr * WROWS + i * 32 + (e & 3) + 8 * (e >> 2) + 4 * (lane >> 5);
            const double sa = sa_r[row];
            if (sa == 0.0 || sb == 0.0) continue;  // den == 0: this sketch row does not qualify
            const uint32_t ab = (uint32_t)acc[i][j][e];
            const float est = (float)ab * __builtin_amdgcn_rcpf((float)sa) * rb;
            if (est < fminf(s_ta[row], tb) - 4e-6f) {  // can never be admitted
              alive[bit >> 5] &= ~m;
              continue;
            }
            uint32_t& sv = st[i][j][e];
            bool take = sv == kEmpty;
            if (!take) {
              const int rr = (int)(sv & rmask);
              float est0;
              if (!(sv >> 31)) {
                est0 = __uint_as_float(sv & ~rmask);  // estimate form: no lookup of row rr
              } else {
                est0 = (float)((sv & 0x7FFFFFFFu) >> rbits) * __builtin_amdgcn_rcpf((float)s_sa[rr * kSA + row]) *
                       __builtin_amdgcn_rcpf((float)s_sb[rr * kSB + col]);
              }
              if (est < est0 * (1.0f - 0x1p-17f)) {
                take = true;
              } else if (est <= est0 * (1.0f + 0x1p-17f)) {  // too close for fp32: the exact values
                const double sa0 = s_sa[rr * kSA + row], sb0 = s_sb[rr * kSB + col];
                const double ab0 =
                    (sv >> 31) ? (double)((sv & 0x7FFFFFFFu) >> rbits) : rint((double)est0 * sa0 * sb0);
                take = exact_less((double)ab, sa, sb, ab0, sa0, sb0);
              }
            }
            if (take) sv = (float)ab <= ab_est_max ? (__float_as_uint(est) & ~rmask) | (uint32_t)r
                                                                 : 0x80000000u | (ab << rbits) | (uint32_t)r;
          }
        }
      }
    }
#pragma unroll
    for (int i = 0; i < TI; ++i)
#pragma unroll
      for (int j = 0; j < 3; ++j)
#pragma unroll
        for (int e = 0; e < 16; ++e) acc[i][j][e] = 0;
  }
#if CMS_SYM_SCHED
  wait_vmcnt<0>();  // the repeat loads land before the workgroup's LDS is released
#endif
#if CMS_SYM_PROBE & 2
  if (probe_sink == 1234.5f) g.ccnt[tid] = 7u;  // never true in practice: keeps the sums (and MFMAs) live
#endif

  // ---- the exact value of each surviving pair, offered to both lists ----
#pragma unroll
  for (int j = 0; j < 3; ++j) {
    const int col = wc * 96 + j * 32 + (lane & 31);
    const int64_t bp = b_pos0 + col;
    const double tb = col < b_rows ? g.thr[bp] : 0.0;
#pragma unroll
    for (int i = 0; i < TI; ++i)
#pragma unroll
      for (int e = 0; e < 16; ++e) {
        const int bit = (i * 3 + j) * 16 + e;
        if (!((alive[bit >> 5] >> (bit & 31)) & 1u)) continue;
        const uint32_t sv = st[i][j][e];
        if (sv == kEmpty) continue;  // NaN: never offered
        const int row = wr * WROWS + i * 32 + (e & 3) + 8 * (e >> 2) + 4 * (lane >> 5);
        if (row >= a_rows || col >= b_rows) continue;
        const int64_t ap = a_pos0 + row;
        if (ap == bp || (diag && ap > bp)) continue;
        const int rr = (int)(sv & rmask);
        const double sa = s_sa[rr * kSA + row], sb = s_sb[rr * kSB + col];
        // the exact dot: packed, or recovered from the fp32 estimate
        const double ab = (FMT == 0 && (sv >> 31)) ? (double)((sv & 0x7FFFFFFFu) >> rbits)
                                                   : rint((double)__uint_as_float(sv & ~rmask) * sa * sb);
        double v = __ddiv_rn(ab, __dmul_rn(sa, sb));
        if (v > 1.0) v = 1.0;  // normalizeWeightResult, unweighted (values are >= 0)
        if (v >= g.thr[ap]) {
          const uint32_t slot = atomicAdd(&g.ccnt[ap], 1u);
          if (slot < (uint32_t)g.cap) {
            g.cidx[ap * g.cap + slot] = (uint32_t)bp;
            g.cval[ap * g.cap + slot] = v;
          }
        }
        if (v >= tb) {
          const uint32_t slot = atomicAdd(&g.ccnt[bp], 1u);
          if (slot < (uint32_t)g.cap) {
            g.cidx[bp * g.cap + slot] = (uint32_t)ap;
            g.cval[bp * g.cap + slot] = v;
          }
        }
      }
  }
}

template <int NSTAGE, int BK, int FMT, int NW>
__global__ __launch_bounds__(64 * NW, 1) void k_cosine_sym(SymArgs g) {
  sym_tile<NSTAGE, BK, FMT, NW>(g, (int)blockIdx.x);
}

#ifndef CMS_SYM_NS
#define CMS_SYM_NS 5
#endif
#ifndef CMS_SYM_BK
#define CMS_SYM_BK 64
#endif
constexpr int kSymNS = CMS_SYM_NS, kSymBK = CMS_SYM_BK;  // ring depth, bytes per row per stage

int sym_stage_bytes() { return kSymBK; }

size_t sym_lds_bytes(int depth) {
  return (size_t)kSymNS * (kSA + kSB) * kSymBK + (size_t)depth * (kSA + kSB) * sizeof(double) +
         (kSA + kSB) * sizeof(float);
}

bool sym_eligible(cms_handle* h, int fmt, int32_t* rbits) {
  int rb = 0;
  while ((1 << rb) < h->p.depth) ++rb;
  rb = std::max(rb, 1);
  // largest exact dot of one sketch row: fp4 counters <= 4, int8 limbs <= 127
  const double max_ab = (fmt == 1 ? 16.0 : 16129.0) * (double)h->p.width;
  *rbits = rb;
  // the exact form of the running minimum packs AB* << rb | r* below bit 31;
  // fp4 rows keep the estimate form only: relative error <= 2^-21 (two rcp,
  // two products) + 2^(rb-23) (the replaced bits), and the dot recovered from
  // it is exact while max_ab times that error stays below 1/2
  if (fmt == 1 && max_ab * (std::ldexp(1.0, -21) + std::ldexp(1.0, rb - 23)) >= 0.5) return false;
  return h->p.weighting != CMS_WEIGHTED && max_ab < (double)((1ULL << (31 - rb)) - 1) &&
         sym_lds_bytes(h->p.depth) <= 160 * 1024 && (h->p.width % (fmt == 1 ? 2 * kSymBK : kSymBK)) == 0;
}

int launch_sym(cms_handle* h, SymArgs g, int fmt, int64_t pair_slots) {
  g.nblk = (int32_t)(kSub * g.band * pair_slots);
  if (g.rect) {
    g.njc = (g.si + g.band - 1 + g.sj - 1) / g.sj;
    g.nblk = (int32_t)(((pair_slots + g.si - 1) / g.si) * g.njc * g.si * g.sj * kSub);
  }
  if (g.nblk <= 0) return CMS_OK;
  if (g.tsel) g.xchunk = 0;
  int64_t grid = g.xchunk ? (g.nblk + 8LL * g.xchunk - 1) / (8LL * g.xchunk) * 8LL * g.xchunk : g.nblk;
  const size_t bytes = sym_lds_bytes(g.depth);
  static bool attr = [] {
    (void)hipFuncSetAttribute((const void*)k_cosine_sym<kSymNS, kSymBK, 0, kSymNW>, hipFuncAttributeMaxDynamicSharedMemorySize,
                              160 * 1024);
    (void)hipFuncSetAttribute((const void*)k_cosine_sym<kSymNS, kSymBK, 1, kSymNW>, hipFuncAttributeMaxDynamicSharedMemorySize,
                              160 * 1024);
    return true;
  }();
  (void)attr;
  if (fmt == 1) hipLaunchKernelGGL((k_cosine_sym<kSymNS, kSymBK, 1, kSymNW>), dim3((unsigned)grid), dim3(64 * kSymNW), bytes, h->stream, g);
  else hipLaunchKernelGGL((k_cosine_sym<kSymNS, kSymBK, 0, kSymNW>), dim3((unsigned)grid), dim3(64 * kSymNW), bytes, h->stream, g);
  CMS_HIP(hipGetLastError());
  return CMS_OK;
}

}  // namespace cms
