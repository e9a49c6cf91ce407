// cms_partition.hip -- unordered COO stream -> CSR keys grouped by owner row.
//
// The reference never sees an unordered stream: its DataModel hands CosineCM
// one PreferenceArray per owner (T/impl/similarity/CosineCM.java:49-56).  A
// streaming ingest has to group the pairs itself before the LDS row build
// (cms_build.hip).  Two MSD passes, fan-out <= 4096 each:
//   pass 1: coarse bin = row >> s2   (writes the key token + u16 fine index)
//   pass 2: fine bin   = row & (2^s2 - 1), segmented per coarse bin
//           (writes the key at its final CSR position; the scan of pass 2 also
//            yields the CSR row offsets)
// Each scatter stages a 4096-pair tile in LDS sorted by bin and writes it out
// as contiguous per-bin runs, so global writes coalesce instead of landing as
// isolated 8-byte stores.  Counts come from per-block LDS histograms and a
// device-wide scan -- no global atomics on hot rows.
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cstdlib>

#include "cms_device.h"
#include "cms_internal.h"

namespace cms {

constexpr int kPartThreads = 512;
#ifndef CMS_PART_PER
#define CMS_PART_PER 8
#endif
constexpr int kPartPer = CMS_PART_PER;  // pairs per thread per tile
constexpr int kPartTile = kPartThreads * kPartPer;  // pairs staged per tile
constexpr int kMaxBins = 4096;

// aggregation rounds per LDS histogram (lds_bin_add); 0 = plain atomics
#ifndef CMS_PEEL_P1H
#define CMS_PEEL_P1H 0
#endif
#ifndef CMS_PEEL_P1S
#define CMS_PEEL_P1S 0
#endif
#ifndef CMS_PEEL_P2H
#define CMS_PEEL_P2H 1
#endif
#ifndef CMS_PEEL_P2S
#define CMS_PEEL_P2S 0
#endif
// fine bits of the two-pass split (pass 2 fan-out 2^CMS_PART_S2)
#ifndef CMS_PART_S2
#define CMS_PART_S2 10
#endif
// pass-1 stream chunks (workgroups) for large batches
#ifndef CMS_P1_BLOCKS
#define CMS_P1_BLOCKS 2048
#endif
// largest pass-1 tile, in rounds of kPartTile pairs (k_p1_scatter<R>: the
// largest R <= CMS_P1_ROUNDS whose tile fits the LDS)
#ifndef CMS_P1_ROUNDS
#define CMS_P1_ROUNDS 4
#endif
// the next tile's first round is loaded as the last round of this tile is
// binned (before the scan, placement and write-out), not after the placement
#ifndef CMS_PART_EARLY_NEXT
#define CMS_PART_EARLY_NEXT 1
#endif
// pass 2: the next virtual block's first round and cursors loaded during this
// block's last round (k_p2_scatter)
#ifndef CMS_P1_NT
#define CMS_P1_NT 0
#endif
#ifndef CMS_P2_AHEAD
#define CMS_P2_AHEAD 1
#endif
// pass-2 tile in rounds of kPartTile pairs (1, 2 or 4: a block's chunk is
// four rounds; 4 = one 16384-pair tile per block: config-3 partition
// 5.30-5.34 -> 5.08-5.11 ms in two A/B runs, profiles/r04/ab_*)
#ifndef CMS_P2_ROUNDS
#define CMS_P2_ROUNDS 4
#endif

// LDS histogram increment aggregated across the wave.  Zipf streams put most
// lanes of a wave on the same few bins (the head items: 3/4 of config 2's
// pairs fall in coarse bin 0), and same-address LDS atomics serialise lane by
// lane.  kPeel times, the pending lanes that share the bin of the lowest
// pending lane are counted by one atomic of their population count; the rest
// then increment one by one.  With kRank the lane's rank within its bin is
// returned (unique and contiguous per bin, as a plain atomicAdd's would be).
// Call from converged code: the ballots see only the active lanes.
template <int kPeel, bool kRank>
__device__ __forceinline__ uint32_t lds_bin_add(uint32_t* hist, uint32_t bin, bool active) {
  uint32_t rank = 0;
  bool pending = active;
  const int lane = (int)__lane_id();
#pragma unroll
  for (int r = 0; r < kPeel; ++r) {
    const unsigned long long pm = __ballot(pending);
    if (pm == 0ULL) return rank;
    const int lead = __builtin_ctzll(pm);
    const uint32_t b0 = (uint32_t)__builtin_amdgcn_readlane((int)bin, lead);
    const bool mine = pending && bin == b0;
    const unsigned long long m = __ballot(mine);
    uint32_t base = 0;
    if (lane == lead) {
      if (kRank) base = atomicAdd(&hist[b0], (uint32_t)__popcll(m));
      else atomicAdd(&hist[b0], (uint32_t)__popcll(m));
    }
    if (kRank) {
      base = (uint32_t)__builtin_amdgcn_readlane((int)base, lead);
      if (mine) rank = base + __builtin_amdgcn_mbcnt_hi((uint32_t)(m >> 32), __builtin_amdgcn_mbcnt_lo((uint32_t)m, 0u));
    }
    pending = pending && !mine;
  }
  if (pending) {
    if (kRank) rank = atomicAdd(&hist[bin], 1u);
    else atomicAdd(&hist[bin], 1u);
  }
  return rank;
}

// ---- hot-owner routing (partition_to_spans) ----
// A Zipf stream puts most pairs on a few owners (config 2: the top ~1000 of
// 100K items hold ~3/4 of the pairs).  Those owners get bins of their own in
// pass 1, so their keys land at their final place at once and only the other
// pairs take pass 2.  The hot set comes from a strided sample: every owner
// with >= tau sample hits bids for slot hslot(owner) of a kHotBins-entry
// table, the one with the most hits wins (ties: larger owner; an owner that
// loses its slot simply stays on the two-pass path -- correctness never
// depends on who is hot).
#ifndef CMS_HOT_LOG
#define CMS_HOT_LOG 10
#endif
constexpr int kHotLog = CMS_HOT_LOG, kHotBins = 1 << kHotLog;
__device__ __forceinline__ uint32_t hslot(int64_t o) {
  return (uint32_t)(((uint64_t)o * 0x9E3779B97F4A7C15ULL) >> (64 - kHotLog));  // top kHotLog bits
}

// Sample counts: each block counts its share of the strided sample in an LDS
// hash table first (a Zipf head owner takes a good part of every block's
// samples, and same-address global atomics serialise at the memory side),
// then adds each owner's block count with one global atomic.
constexpr int kSampleTab = 4096;  // LDS entries (owner + 1, count)
constexpr int kSamplePerBlock = 4096;
__global__ __launch_bounds__(256) void k_hot_sample(const int64_t* row, int64_t stride, int64_t S, int64_t nrows,
                                                    uint32_t* cnt) {
  __shared__ uint32_t tkey[kSampleTab], tcnt[kSampleTab];
  for (int i = threadIdx.x; i < kSampleTab; i += blockDim.x) tkey[i] = tcnt[i] = 0u;
  __syncthreads();
  const int64_t s0 = (int64_t)blockIdx.x * kSamplePerBlock, s1 = min(S, s0 + kSamplePerBlock);
  for (int64_t i = s0 + threadIdx.x; i < s1; i += blockDim.x) {
    const int64_t r = row[i * stride];
    if (r < 0 || r >= nrows) continue;
    const uint32_t k = (uint32_t)r + 1u;
    uint32_t slot = (uint32_t)(((uint64_t)r * 0x9E3779B97F4A7C15ULL) >> 52) & (kSampleTab - 1);
    bool done = false;
    for (int probe = 0; probe < 32 && !done; ++probe) {
      const uint32_t old = atomicCAS(&tkey[slot], 0u, k);
      if (old == 0u || old == k) {
        atomicAdd(&tcnt[slot], 1u);
        done = true;
      }
      slot = (slot + 1) & (kSampleTab - 1);
    }
    if (!done) atomicAdd(&cnt[r], 1u);  // table crowded: count directly
  }
  __syncthreads();
  for (int i = threadIdx.x; i < kSampleTab; i += blockDim.x)
    if (tkey[i]) atomicAdd(&cnt[tkey[i] - 1u], tcnt[i]);
}

__global__ __launch_bounds__(256) void k_hot_claim(const uint32_t* cnt, int64_t nrows, uint32_t tau,
                                                   unsigned long long* slotkey) {
  for (int64_t o = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; o < nrows; o += (int64_t)gridDim.x * blockDim.x) {
    const uint32_t c = cnt[o];
    if (c >= tau) atomicMax(&slotkey[hslot(o)], ((unsigned long long)c << 32) | (unsigned long long)(o + 1));
  }
}

// LDS copy of the hot table (owner + 1 per slot, 0 = empty); bin of a row:
// its hot bin P1 + slot, else its coarse bin.
__device__ __forceinline__ void load_hot_table(const unsigned long long* slotkey, uint32_t* tab) {
  for (int t = threadIdx.x; t < kHotBins; t += blockDim.x) tab[t] = (uint32_t)slotkey[t];
}
__device__ __forceinline__ uint32_t bin_of(uint32_t r, int s2, int P1, const uint32_t* tab) {
  if (tab) {
    const uint32_t t = hslot(r);
    if (tab[t] == r + 1u) return (uint32_t)P1 + t;
  }
  return r >> s2;
}

// Pass-1 work is cut into tiles of kPartTile pairs, and block b takes tiles
// b, b + NB, b + 2 NB, ... (the same assignment in k_p1_hist and
// k_p1_scatter): at any moment the blocks stream one contiguous window of the
// stream instead of NB separate regions (DRAM page locality; the contiguous
// per-block chunks streamed the owner column at ~3.4 TB/s).
template <int R>
__global__ __launch_bounds__(256) void k_p1_hist(const int64_t* row, int64_t n, int s2, int P1, int64_t nrows,
                                                 uint32_t* H1, int NB, uint32_t* flags,
                                                 const unsigned long long* hotkey) {
  extern __shared__ uint32_t lh[];
  const int P = P1 + (hotkey ? kHotBins : 0);  // bins: coarse, then hot
  uint32_t* tab = hotkey ? lh + P : nullptr;
  for (int b = threadIdx.x; b < P; b += blockDim.x) lh[b] = 0;
  if (tab) load_hot_table(hotkey, tab);
  __syncthreads();
  bool bad = false;
  // tiles of R * kPartTile pairs (k_p1_scatter<R>'s), each counted as R
  // sub-tiles of kPartTile
  const int64_t ntiles = (n + (int64_t)R * kPartTile - 1) / ((int64_t)R * kPartTile);
  const bool vec = (reinterpret_cast<uintptr_t>(row) & 15) == 0;
  // 256 threads x 8 16-byte loads = one 4096-pair sub-tile, all loads in flight;
  // whole waves step together so the aggregated increments see converged lanes
  constexpr int kL = kPartTile / 2 / 256;
  static_assert(kL * 2 * 256 == kPartTile, "tile = 256 threads x kL pair loads");
  for (int64_t t = blockIdx.x; t < ntiles; t += NB)
  for (int sub = 0; sub < R; ++sub) {
    const int64_t t0 = (t * R + sub) * kPartTile, tn = min<int64_t>(kPartTile, n - t0);
    if (tn <= 0) break;
    longlong2 v[kL];
#pragma unroll
    for (int u = 0; u < kL; ++u) {
      const int64_t i = 2 * ((int64_t)u * 256 + threadIdx.x);  // pair index within the tile
      if (vec && i + 1 < tn) {
        v[u] = *reinterpret_cast<const longlong2*>(row + t0 + i);
      } else {
        v[u].x = i < tn ? row[t0 + i] : -1;
        v[u].y = i + 1 < tn ? row[t0 + i + 1] : -1;
      }
    }
#pragma unroll
    for (int u = 0; u < kL; ++u) {
      const int64_t i = 2 * ((int64_t)u * 256 + threadIdx.x);
      const bool okx = v[u].x >= 0 && v[u].x < nrows, oky = v[u].y >= 0 && v[u].y < nrows;
      if ((i < tn && !okx) || (i + 1 < tn && !oky)) bad = true;
      lds_bin_add<CMS_PEEL_P1H, false>(lh, okx ? bin_of((uint32_t)v[u].x, s2, P1, tab) : 0u, okx);
      lds_bin_add<CMS_PEEL_P1H, false>(lh, oky ? bin_of((uint32_t)v[u].y, s2, P1, tab) : 0u, oky);
    }
  }
  if (bad) atomicOr(flags, kFlagBadRow);
  __syncthreads();
  for (int b = threadIdx.x; b < P; b += blockDim.x) H1[(int64_t)blockIdx.x * P + b] = lh[b];  // block-major, coalesced
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
  uint32_t* key;  // key tokens (make_token)
  float* val;
  uint16_t* fine;
  uint16_t* bin;
  uint32_t* cursor;
  uint32_t* hist;
  uint32_t* off;
  uint32_t* scr;
};

// LDS image of a tile: keys, then values and fine indices only when the pass
// carries them (a smaller image lets more workgroups share a CU).
__device__ __forceinline__ TileLds carve(unsigned char* smem, int P, bool has_val, bool has_fine, int tile = kPartTile) {
  TileLds t;
  unsigned char* q = smem;
  t.key = reinterpret_cast<uint32_t*>(q);
  q += sizeof(uint32_t) * tile;
  t.val = reinterpret_cast<float*>(q);
  if (has_val) q += sizeof(float) * tile;
  t.fine = reinterpret_cast<uint16_t*>(q);
  if (has_fine) q += sizeof(uint16_t) * tile;
  t.bin = reinterpret_cast<uint16_t*>(q);
  q += sizeof(uint16_t) * tile;
  t.cursor = reinterpret_cast<uint32_t*>(q);
  t.hist = t.cursor + P;
  t.off = t.hist + P;
  t.scr = t.off + P;
  return t;
}

static size_t tile_lds_bytes(int P, bool has_val, bool has_fine, bool hot = false, int tile = kPartTile) {
  return (size_t)tile * (4 + (has_val ? 4 : 0) + (has_fine ? 2 : 0) + 2) + (size_t)3 * P * 4 + 64 * 4 +
         (hot ? sizeof(uint32_t) * kHotBins : 0);
}

// Pass 1: block b owns tiles b, b + NB, ... of the stream; output region of
// (coarse bin, block) starts at O1[bin*NB + b].
// With hotkey: bins [P1, P1 + kHotBins) are hot owners, whose keys (and
// values) go straight to okey_hot / oval_hot -- their final place.  Keys
// leave as u32 tokens (make_token: the key itself below 2^31, else its
// index in this batch).
//
// A tile is R rounds of kPartTile pairs.  Each round's pairs are binned and
// ranked as they arrive (the next round's loads already in flight) and kept
// in registers as (token, rank|bin, fine); one scan and one LDS placement per
// tile then write the tile out as per-bin runs.  The runs are what the
// partition pays for: a bin's run is a few keys at 4096 pairs per tile (config
// 3: ~1500 bins), and each one costs about one partial-line write, so R = 4
// (16384-pair tiles) writes a quarter of the runs.
template <int R, bool HV>
__global__ __launch_bounds__(kPartThreads) void k_p1_scatter(const int64_t* row, const int64_t* key, const float* val,
                                                             int64_t n, int s2, int P1, int64_t nrows,
                                                             const uint32_t* O1, int NB, uint16_t* ofine,
                                                             uint32_t* okey, float* oval,
                                                             const unsigned long long* hotkey, uint32_t* okey_hot,
                                                             float* oval_hot) {
  constexpr int TILE = R * kPartTile;  // pairs per tile
  constexpr int NP = R * kPartPer;     // pairs per thread per tile
  extern __shared__ __align__(16) unsigned char smem[];
  const int P = P1 + (hotkey ? kHotBins : 0);
  TileLds L = carve(smem, P, HV, true, TILE);
  uint32_t* tab = hotkey ? L.scr + 64 : nullptr;
  const int tid = threadIdx.x;
  if (tab) load_hot_table(hotkey, tab);
  for (int b = tid; b < P; b += kPartThreads) L.cursor[b] = O1[(int64_t)blockIdx.x * P + b];
  const uint32_t fmask = (1u << s2) - 1u;
  for (int b = tid; b < P; b += kPartThreads) L.hist[b] = 0;
  // tiles blockIdx.x, + NB, + 2 NB, ... (k_p1_hist<R>'s assignment)
  const int64_t ntiles = (n + TILE - 1) / TILE;
  // two load buffers: round u + 1's loads are issued before round u is binned,
  // and the next tile's first round before this tile's write-out
  int64_t rr[2][kPartPer], kk[2][kPartPer];
  float vv[2][kPartPer];
  auto load = [&](int64_t t, int u, int buf) {
    const int64_t tb = t * TILE + (int64_t)u * kPartTile;
#pragma unroll
    for (int q = 0; q < kPartPer; ++q) {
      const int64_t e = tb + tid + (int64_t)q * kPartThreads;
      rr[buf][q] = -1;
      if (e < n) {
#if CMS_P1_NT  // the stream read once: non-temporal loads (the runs' partial lines keep L2)
        rr[buf][q] = __builtin_nontemporal_load(row + e);
        kk[buf][q] = __builtin_nontemporal_load(key + e);
        if (HV) vv[buf][q] = __builtin_nontemporal_load(val + e);
#else
        rr[buf][q] = row[e];
        kk[buf][q] = key[e];
        if (HV) vv[buf][q] = val[e];
#endif
      }
    }
  };
  uint32_t tk[NP], rb[NP], ff[NP / 2];  // token; rank << 12 | bin (~0: none); two fine indices
  float va[HV ? NP : 1];
  if ((int64_t)blockIdx.x < ntiles) load(blockIdx.x, 0, 0);
  __syncthreads();
  for (int64_t t = blockIdx.x; t < ntiles; t += NB) {
#pragma unroll
    for (int u = 0; u < R; ++u) {
      if (u + 1 < R) load(t, u + 1, (u + 1) & 1);
      // the last round: the next tile's first round into the other buffer
      // (free: its round was binned), in flight through the epilogue
      else if (CMS_PART_EARLY_NEXT && (R % 2) == 0 && t + NB < ntiles) load(t + NB, 0, 0);
      const int cb = u & 1;
#pragma unroll
      for (int q = 0; q < kPartPer; ++q) {
        const int x = u * kPartPer + q;
        const bool ok = rr[cb][q] >= 0 && rr[cb][q] < nrows;
        const uint32_t r32 = ok ? (uint32_t)rr[cb][q] : 0u;
        const uint32_t bin = ok ? bin_of(r32, s2, P1, tab) : 0u;
        const uint32_t rank = lds_bin_add<CMS_PEEL_P1S, true>(L.hist, bin, ok);
        rb[x] = ok ? (rank << 12 | bin) : 0xFFFFFFFFu;
        tk[x] = make_token(kk[cb][q], t * TILE + (int64_t)u * kPartTile + tid + (int64_t)q * kPartThreads);
        const uint32_t f = r32 & fmask;
        ff[x >> 1] = (x & 1) ? (ff[x >> 1] | f << 16) : f;
        if (HV) va[x] = vv[cb][q];
      }
    }
    lds_barrier();
    const uint32_t cnt = scan_bins(L.hist, L.off, P, L.scr);
    lds_barrier();
#pragma unroll
    for (int x = 0; x < NP; ++x) {
      if (rb[x] != 0xFFFFFFFFu) {
        const uint32_t bin = rb[x] & 0xFFFu;
        const uint32_t p = L.off[bin] + (rb[x] >> 12);
        L.key[p] = tk[x];
        if (HV) L.val[p] = va[x];
        L.fine[p] = (uint16_t)(ff[x >> 1] >> ((x & 1) << 4));
        L.bin[p] = (uint16_t)bin;
      }
    }
    if (!(CMS_PART_EARLY_NEXT && (R % 2) == 0) && t + NB < ntiles) load(t + NB, 0, 0);
    lds_barrier();
    for (uint32_t i = tid; i < cnt; i += kPartThreads) {
      uint32_t bin = L.bin[i];
      uint32_t g = L.cursor[bin] + (i - L.off[bin]);
#ifdef CMS_PART_LINEAR  // bound analysis only: contiguous instead of per-bin destinations
      g = (uint32_t)(t * TILE + i);
#endif
#ifdef CMS_PART_NOWRITE  // bound analysis only: no global stores
      if (g != 0xFFFFFFFFu) continue;
#endif
      if ((int)bin >= P1) {  // hot owner: final place
        okey_hot[g] = L.key[i];
        if (HV) oval_hot[g] = L.val[i];
        continue;
      }
      okey[g] = L.key[i];
      ofine[g] = L.fine[i];
      if (HV) oval[g] = L.val[i];
    }
    lds_barrier();
    for (int b = tid; b < P; b += kPartThreads) {
      L.cursor[b] += L.hist[b];
      L.hist[b] = 0;
    }
    lds_barrier();
  }
}

// bs1[b] = first position of pass-1 bin b (b <= P1: bs1[P1] = end of the
// coarse bins); binStart = bs1[0..P1], blkStart = exclusive scan of
// ceil(size_b / CH2).  One block.
__global__ __launch_bounds__(1024) void k_p2_plan(const uint32_t* bs1, int P1, int64_t CH2, uint32_t* binStart,
                                                  uint32_t* blkStart) {
  __shared__ uint32_t sc[1024 / 64 + 1];
  int per = (P1 + 1023) / 1024;
  int lo = threadIdx.x * per, hi = min(P1, lo + per);
  uint32_t s = 0;
  for (int b = lo; b < hi; ++b) {
    binStart[b] = bs1[b];
    s += (uint32_t)((bs1[b + 1] - bs1[b] + CH2 - 1) / CH2);
  }
  uint32_t tot;
  uint32_t off = block_excl_scan_u32(s, sc, &tot);
  for (int b = lo; b < hi; ++b) {
    blkStart[b] = off;
    off += (uint32_t)((bs1[b + 1] - bs1[b] + CH2 - 1) / CH2);
  }
  if (threadIdx.x == 0) {
    blkStart[P1] = tot;
    binStart[P1] = bs1[P1];
  }
}

// Pass-2 block order: workgroup bx runs on XCD bx % 8, and each XCD takes a
// contiguous range of the logical blocks, in order -- so the blocks of one
// coarse bin (adjacent output regions: fine bin f of block k ends where that
// of block k + 1 starts, a few keys long) run together on ONE XCD, and the
// short runs they write into a coarse bin's ~2 MB of output meet in that
// XCD's L2 instead of leaving as partial lines from eight L2s.
__device__ __forceinline__ uint32_t p2_block(uint32_t bx, uint32_t nblk) {
  const uint32_t xcd = bx & 7u, q8 = nblk >> 3, r8 = nblk & 7u;
  return (xcd < r8 ? xcd * (q8 + 1) : r8 * (q8 + 1) + (xcd - r8) * q8) + (bx >> 3);
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
  const uint32_t nblk = blkStart[P1];
  // persistent over the device-side block count (the host's bound on it is
  // loose: a launch of that many workgroups mostly dispatches empty ones);
  // the grid is a multiple of 8, so every virtual block vb runs on XCD vb % 8
  for (uint32_t vb = blockIdx.x; vb < nblk; vb += gridDim.x) {
  const uint32_t lb = p2_block(vb, nblk);
  int b = find_bin(blkStart, P1, lb);
  for (int f = threadIdx.x; f < P2; f += blockDim.x) lh[f] = 0;
  __syncthreads();
  int64_t lo = binStart[b] + (int64_t)(lb - blkStart[b]) * CH2;
  int64_t hi = min((int64_t)binStart[b + 1], lo + CH2);
  // 8 fine indices per 16-byte load; the unaligned head and tail one by one
  const int64_t a0 = min(hi, (lo + 7) & ~int64_t(7));
  const int64_t nv = (hi - a0) / 8;
  const int64_t a1 = a0 + nv * 8;
  if ((int64_t)threadIdx.x < a0 - lo) atomicAdd(&lh[fine[lo + threadIdx.x]], 1u);
  if ((int64_t)threadIdx.x < hi - a1) atomicAdd(&lh[fine[a1 + threadIdx.x]], 1u);
  const uint4* f8 = reinterpret_cast<const uint4*>(fine + a0);
  const int64_t nstep = (nv + blockDim.x - 1) / blockDim.x * blockDim.x;
  for (int64_t i = threadIdx.x; i < nstep; i += blockDim.x) {
    const bool in = i < nv;
    const uint4 v = in ? f8[i] : make_uint4(0, 0, 0, 0);
    const uint32_t w[4] = {v.x, v.y, v.z, v.w};
#pragma unroll
    for (int c = 0; c < 4; ++c) {
      lds_bin_add<CMS_PEEL_P2H, false>(lh, w[c] & 0xFFFFu, in);
      lds_bin_add<CMS_PEEL_P2H, false>(lh, w[c] >> 16, in);
    }
  }
  __syncthreads();
  for (int f = threadIdx.x; f < P2; f += blockDim.x) H2[(int64_t)lb * P2 + f] = lh[f];
  __syncthreads();  // lh read out before the next block zeroes it
  }
}

// Offsets of (pass-2 block, fine bin) and the CSR row starts, in three
// kernels so that no single workgroup walks a Zipf-heavy coarse bin's whole
// column of block histograms: each coarse bin's blocks are cut into
// kP2Split chunks whose column sums are taken in parallel (k_p2_colsum), one
// workgroup per bin scans the bin's totals over fine bins and turns the chunk
// sums into chunk prefixes (k_p2_scan), and the chunks write their blocks'
// offsets in parallel (k_p2_offsets).
constexpr int kP2Split = 16;

template <int SPLIT>
__device__ __forceinline__ void p2_chunk(const uint32_t* blkStart, int b, int c, uint32_t& ka, uint32_t& kb) {
  const uint32_t k0 = blkStart[b], k1 = blkStart[b + 1];
  const uint32_t per = (k1 - k0 + SPLIT - 1) / SPLIT;
  ka = min(k1, k0 + (uint32_t)c * per);
  kb = min(k1, ka + per);
}

template <int SPLIT>
__global__ __launch_bounds__(1024) void k_p2_colsum(const uint32_t* H2, const uint32_t* blkStart, int P2,
                                                    uint32_t* PS) {
  const int b = blockIdx.x / SPLIT, c = blockIdx.x % SPLIT;
  uint32_t ka, kb;
  p2_chunk<SPLIT>(blkStart, b, c, ka, kb);
  for (int f = threadIdx.x; f < P2; f += blockDim.x) {
    uint32_t T = 0;
#pragma unroll 8
    for (uint32_t k = ka; k < kb; ++k) T += H2[(int64_t)k * P2 + f];
    PS[(int64_t)blockIdx.x * P2 + f] = T;
  }
}

__global__ __launch_bounds__(1024) void k_p2_scan(const uint32_t* binStart, int P1, int P2, int64_t nrows,
                                                  uint32_t* PS, int64_t* row_start) {
  __shared__ uint32_t sc[1024 / 64 + 1];
  __shared__ uint32_t tots[kMaxBins];
  const int b = blockIdx.x;
  uint32_t* ps = PS + (int64_t)b * kP2Split * P2;
  for (int f = threadIdx.x; f < P2; f += blockDim.x) {
    uint32_t T = 0;
#pragma unroll
    for (int c = 0; c < kP2Split; ++c) T += ps[(int64_t)c * P2 + f];
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
    const uint32_t base = binStart[b] + tots[f];
    const int64_t r = (int64_t)b * P2 + f;
    if (r < nrows) row_start[r] = base;
    uint32_t run = base;  // chunk sums -> chunk prefixes, in place
#pragma unroll
    for (int c = 0; c < kP2Split; ++c) {
      const uint32_t t = ps[(int64_t)c * P2 + f];
      ps[(int64_t)c * P2 + f] = run;
      run += t;
    }
  }
  if (b == P1 - 1 && threadIdx.x == 0) row_start[nrows] = binStart[P1];
}

// Pass 1 has ONE segment of NB blocks over P bins: the bin totals' exclusive
// scan gives bs1[0..P] (bs1[P] = every valid pair), and the chunk sums become
// chunk prefixes for k_p2_offsets.  One block.
constexpr int kP1Split = 16;  // pass-1 chunks of the block column (NB <= 2048 rows: 128 per chunk)
__global__ __launch_bounds__(1024) void k_p1_scan(int P, uint32_t* PS, uint32_t* bs1) {
  __shared__ uint32_t sc[1024 / 64 + 1];
  __shared__ uint32_t tots[kMaxBins];
  for (int f = threadIdx.x; f < P; f += blockDim.x) {
    uint32_t T = 0;
#pragma unroll
    for (int c = 0; c < kP1Split; ++c) T += PS[(int64_t)c * P + f];
    tots[f] = T;
  }
  __syncthreads();
  const int per = (P + 1023) / 1024;
  const int f0 = threadIdx.x * per, f1 = min(P, f0 + per);
  uint32_t s = 0;
  for (int f = f0; f < f1; ++f) s += tots[f];
  uint32_t total;
  uint32_t ex = block_excl_scan_u32(s, sc, &total);
  for (int f = f0; f < f1; ++f) {
    uint32_t t = tots[f];
    tots[f] = ex;
    ex += t;
  }
  __syncthreads();
  for (int f = threadIdx.x; f < P; f += blockDim.x) {
    const uint32_t base = tots[f];
    bs1[f] = base;
    uint32_t run = base;
#pragma unroll 8
    for (int c = 0; c < kP1Split; ++c) {
      const uint32_t t = PS[(int64_t)c * P + f];
      PS[(int64_t)c * P + f] = run;
      run += t;
    }
  }
  if (threadIdx.x == 0) bs1[P] = total;
}

template <int SPLIT>
__global__ __launch_bounds__(1024) void k_p2_offsets(const uint32_t* H2, const uint32_t* blkStart, int P2,
                                                     const uint32_t* PS, uint32_t* O2) {
  const int b = blockIdx.x / SPLIT, c = blockIdx.x % SPLIT;
  uint32_t ka, kb;
  p2_chunk<SPLIT>(blkStart, b, c, ka, kb);
  for (int f = threadIdx.x; f < P2; f += blockDim.x) {
    uint32_t run = PS[(int64_t)blockIdx.x * P2 + f];
    uint32_t k = ka;
    for (; k + 8 <= kb; k += 8) {  // the counts' loads in flight together
      uint32_t cnt[8];
#pragma unroll
      for (int u = 0; u < 8; ++u) cnt[u] = H2[(int64_t)(k + u) * P2 + f];
#pragma unroll
      for (int u = 0; u < 8; ++u) {
        O2[(int64_t)(k + u) * P2 + f] = run;
        run += cnt[u];
      }
    }
    for (; k < kb; ++k) {
      const uint32_t cnt = H2[(int64_t)k * P2 + f];
      O2[(int64_t)k * P2 + f] = run;
      run += cnt;
    }
  }
}

// Pass 2: block lb takes its coarse bin's pairs [lo, lo + CH2) in tiles of R
// rounds of kPartTile pairs (k_p1_scatter's scheme: binned and ranked from
// registers, one scan and one LDS placement per tile), fine bin = owner.
template <int R, bool HV>
__global__ __launch_bounds__(kPartThreads) void k_p2_scatter(const uint16_t* fine, const uint32_t* key1,
                                                             const float* val1, const uint32_t* binStart,
                                                             const uint32_t* blkStart, int P1, int64_t CH2, int P2,
                                                             const uint32_t* O2, uint32_t* okey, float* oval,
                                                             int32_t* orow) {
  constexpr int TILE = R * kPartTile, NP = R * kPartPer;
  extern __shared__ __align__(16) unsigned char smem[];
  const uint32_t nblk = blkStart[P1];
  TileLds L = carve(smem, P2, HV, false, TILE);
  const int tid = threadIdx.x;
  // persistent over the device-side block count (k_p2_hist).  With
  // CMS_P2_AHEAD the next virtual block's first round and its row of
  // cursors are loaded while this block's last round is binned, so they are
  // in flight through this block's epilogue (a block is one tile at the
  // default CH2: without this, every block started with two exposed loads).
  constexpr bool kAhead = CMS_P2_AHEAD && (R % 2) == 0;
  constexpr int kCurPer = kMaxBins / kPartThreads;  // cursor words per thread (P2 <= kMaxBins)
  uint32_t kk[2][kPartPer], ff[2][kPartPer];
  float vv[2][kPartPer];
  auto load = [&](int64_t tb, int buf, int64_t end) {
#pragma unroll
    for (int q = 0; q < kPartPer; ++q) {
      const int64_t e = tb + tid + (int64_t)q * kPartThreads;
      ff[buf][q] = 0xFFFFFFFFu;
      if (e < end) {
        ff[buf][q] = fine[e];
        kk[buf][q] = key1[e];
        if (HV) vv[buf][q] = val1[e];
      }
    }
  };
  struct Blk {
    uint32_t lb;
    int b;
    int64_t lo, hi;
  };
  auto block_of = [&](uint32_t vb) {
    Blk k;
    k.lb = p2_block(vb, nblk);
    k.b = find_bin(blkStart, P1, k.lb);
    k.lo = binStart[k.b] + (int64_t)(k.lb - blkStart[k.b]) * CH2;
    k.hi = min((int64_t)binStart[k.b + 1], k.lo + CH2);
    return k;
  };
  uint32_t cur[kCurPer];
  auto load_cursors = [&](uint32_t lb) {
#pragma unroll
    for (int c = 0; c < kCurPer; ++c) {
      const int f = tid + c * kPartThreads;
      if (f < P2) cur[c] = O2[(int64_t)lb * P2 + f];
    }
  };
  Blk nx{};
  if (kAhead && blockIdx.x < nblk) {
    nx = block_of(blockIdx.x);
    load_cursors(nx.lb);
    if (nx.lo < nx.hi) load(nx.lo, 0, nx.hi);
  }
  for (uint32_t vb = blockIdx.x; vb < nblk; vb += gridDim.x) {
  const Blk blk = kAhead ? nx : block_of(vb);
  const uint32_t lb = blk.lb;
  const int b = blk.b;
  const int64_t lo = blk.lo, hi = blk.hi;
  if (kAhead) {
#pragma unroll
    for (int c = 0; c < kCurPer; ++c) {
      const int f = tid + c * kPartThreads;
      if (f < P2) L.cursor[f] = cur[c];
    }
  } else {
    for (int f = tid; f < P2; f += kPartThreads) L.cursor[f] = O2[(int64_t)lb * P2 + f];
  }
  for (int f = tid; f < P2; f += kPartThreads) L.hist[f] = 0;
  uint32_t tk[NP], rf[NP];  // key token; rank << 12 | fine bin (~0: none)
  float va[HV ? NP : 1];
  if (!kAhead && lo < hi) load(lo, 0, hi);
  __syncthreads();
  for (int64_t tb = lo; tb < hi; tb += TILE) {
#pragma unroll
    for (int u = 0; u < R; ++u) {
      if (u + 1 < R) {
        load(tb + (int64_t)(u + 1) * kPartTile, (u + 1) & 1, hi);
      } else if (kAhead) {
        if (tb + TILE < hi) {
          load(tb + TILE, 0, hi);  // the next tile of this block (k_p1_scatter)
        } else if (vb + gridDim.x < nblk) {
          nx = block_of(vb + gridDim.x);  // the next block's first round and cursors
          load_cursors(nx.lb);
          if (nx.lo < nx.hi) load(nx.lo, 0, nx.hi);
        }
      }
      const int cb = u & 1;
#pragma unroll
      for (int q = 0; q < kPartPer; ++q) {
        const int x = u * kPartPer + q;
        const bool ok = ff[cb][q] != 0xFFFFFFFFu;
        const uint32_t rank = lds_bin_add<CMS_PEEL_P2S, true>(L.hist, ok ? ff[cb][q] : 0u, ok);
        rf[x] = ok ? (rank << 12 | ff[cb][q]) : 0xFFFFFFFFu;
        tk[x] = kk[cb][q];
        if (HV) va[x] = vv[cb][q];
      }
    }
    lds_barrier();
    const uint32_t cnt = scan_bins(L.hist, L.off, P2, L.scr);
    lds_barrier();
#pragma unroll
    for (int x = 0; x < NP; ++x) {
      if (rf[x] != 0xFFFFFFFFu) {
        const uint32_t f = rf[x] & 0xFFFu;
        const uint32_t p = L.off[f] + (rf[x] >> 12);
        L.key[p] = tk[x];
        if (HV) L.val[p] = va[x];
        L.bin[p] = (uint16_t)f;
      }
    }
    if (!kAhead && tb + TILE < hi) load(tb + TILE, 0, hi);
    lds_barrier();
    for (uint32_t i = tid; i < cnt; i += kPartThreads) {
      uint32_t f = L.bin[i];
      uint32_t g = L.cursor[f] + (i - L.off[f]);
#ifdef CMS_PART_LINEAR  // bound analysis only: contiguous instead of per-bin destinations
      g = (uint32_t)(tb + i);
#endif
#ifdef CMS_PART_NOWRITE  // bound analysis only: no global stores
      if (g != 0xFFFFFFFFu) continue;
#endif
      okey[g] = L.key[i];
      if (HV) oval[g] = L.val[i];
      if (orow) orow[g] = b * P2 + (int32_t)f;
    }
    lds_barrier();
    for (int f = tid; f < P2; f += kPartThreads) {
      L.cursor[f] += L.hist[f];
      L.hist[f] = 0;
    }
    lds_barrier();
  }
  if (kAhead && lo >= hi && vb + gridDim.x < nblk) {  // an empty block had no last round
    nx = block_of(vb + gridDim.x);
    load_cursors(nx.lb);
    if (nx.lo < nx.hi) load(nx.lo, 0, nx.hi);
  }
  __syncthreads();  // this block's LDS use ends before the next block's cursors are stored
  }
}

static int ceil_log2(int64_t v) {
  int b = 0;
  while ((int64_t(1) << b) < v) ++b;
  return b;
}

// Spans of the hot owners (their bins of pass 1) and the end of every other
// owner's CSR range; hot owners have empty ranges in the two-pass CSR.
__global__ void k_spans_hi(const int64_t* coff, int64_t nrows, int64_t* hi) {
  for (int64_t r = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; r < nrows; r += (int64_t)gridDim.x * blockDim.x)
    hi[r] = coff[r + 1];
}
__global__ void k_spans_hot(const unsigned long long* slotkey, const uint32_t* bs1, int P1, int64_t* lo, int64_t* hi) {
  const int t = blockIdx.x * blockDim.x + threadIdx.x;
  if (t >= kHotBins) return;
  const uint32_t o1 = (uint32_t)slotkey[t];
  if (o1 == 0) return;
  lo[o1 - 1] = bs1[P1 + t];
  hi[o1 - 1] = bs1[P1 + t + 1];
}

static int partition_impl(cms_handle* h, const int64_t* d_row, const int64_t* d_key, const float* d_val, int64_t npairs,
                          bool hot, int64_t** out_lo, int64_t** out_hi, uint32_t** out_tok, float** out_val,
                          int32_t* out_rows) {
  const int64_t n = h->n;
  const int B = std::max(1, ceil_log2(n));
  // fine bits: 11 for 2^19+ owners (config 3, 1M owners: 489 coarse bins give
  // the cold pairs' pass-1 runs twice the length of 977; partition 6.18 ->
  // 5.79 ms), else CMS_PART_S2 (10)
  int s2 = std::min(B, B >= 20 ? 11 : CMS_PART_S2);
  if (B - s2 > 12) s2 = B - 12;
  const int P2 = 1 << s2;
  const int P1 = (int)((n + P2 - 1) / P2);
  if (P1 > kMaxBins || P2 > kMaxBins)
    return set_error(CMS_E_PARAM, "num_owners %lld too large for the partition", (long long)n);
  if (hot && (P1 + kHotBins > kMaxBins || out_rows || n >= (int64_t(1) << 31))) return kNoSpans;
  const int P = P1 + (hot ? kHotBins : 0);  // pass-1 bins
  // pass-1 tile: the most rounds whose LDS image fits a workgroup
  int R = CMS_P1_ROUNDS;
  while (R > 1 && tile_lds_bytes(P, d_val != nullptr, true, hot, R * kPartTile) > 160 * 1024) R >>= 1;
  const int64_t tile1 = (int64_t)R * kPartTile;
  const int NB = (int)std::max<int64_t>(1, std::min<int64_t>(CMS_P1_BLOCKS, (npairs + tile1 - 1) / tile1));
  const int64_t CH2 = 4 * kPartTile;
  const int64_t nb2max = npairs / CH2 + P1 + 1;

  CMS_HIP(h->ws_p1_row.ensure(sizeof(uint16_t) * (size_t)npairs));
  CMS_HIP(h->ws_p1_key.ensure(sizeof(uint32_t) * (size_t)npairs));
  if (d_val) CMS_HIP(h->ws_p1_val.ensure(sizeof(float) * (size_t)npairs));
  CMS_HIP(h->ws_csr_key.ensure(sizeof(uint32_t) * (size_t)npairs));
  if (d_val) CMS_HIP(h->ws_csr_val.ensure(sizeof(float) * (size_t)npairs));
  CMS_HIP(h->ws_csr_off.ensure(sizeof(int64_t) * (size_t)(n + 1)));
  if (hot) {
    CMS_HIP(h->ws_csr_hi.ensure(sizeof(int64_t) * (size_t)n));
    CMS_HIP(h->ws_hotpart.ensure(sizeof(unsigned long long) * kHotBins + sizeof(uint32_t) * (size_t)n));
  }
  const int64_t L1 = (int64_t)P * NB, L2 = nb2max * P2;
  const size_t hist_words = (size_t)(2 * L1 + 2 * L2 + 2 * (P1 + 1) + 64) + (size_t)P1 * kP2Split * P2 +
                            (size_t)kP1Split * P + (P + 1) + 2;
  CMS_HIP(h->ws_hist.ensure(sizeof(uint32_t) * hist_words));
  uint32_t* H1 = h->ws_hist.as<uint32_t>();
  uint32_t* O1 = H1 + L1;
  uint32_t* H2 = O1 + L1;
  uint32_t* O2 = H2 + L2;
  uint32_t* binStart = O2 + L2;
  uint32_t* blkStart = binStart + (P1 + 1);
  uint32_t* PS = blkStart + (P1 + 1) + 64;  // [P1][kP2Split][P2] chunk column sums / prefixes
  uint32_t* PS1 = PS + (size_t)P1 * kP2Split * P2;  // [kP1Split][P] pass-1 chunk sums / prefixes
  uint32_t* bs1 = PS1 + (size_t)kP1Split * P;     // [P + 1] pass-1 bin starts
  uint32_t* seg1 = bs1 + (P + 1);                 // {0, NB}: pass 1 is one segment of NB blocks

  uint16_t* fine = h->ws_p1_row.as<uint16_t>();
  uint32_t* key1 = h->ws_p1_key.as<uint32_t>();
  float* val1 = d_val ? h->ws_p1_val.as<float>() : nullptr;
  uint32_t* ckey = h->ws_csr_key.as<uint32_t>();
  float* cval = d_val ? h->ws_csr_val.as<float>() : nullptr;
  int64_t* coff = h->ws_csr_off.as<int64_t>();
  unsigned long long* slotkey = hot ? h->ws_hotpart.as<unsigned long long>() : nullptr;
  static bool lds_attr = [] {
    const void* fs[] = {(const void*)k_p1_scatter<1, false>, (const void*)k_p1_scatter<1, true>,
                        (const void*)k_p1_scatter<2, false>, (const void*)k_p1_scatter<2, true>,
                        (const void*)k_p1_scatter<4, false>, (const void*)k_p1_scatter<4, true>,
                        (const void*)k_p2_scatter<1, false>, (const void*)k_p2_scatter<1, true>,
                        (const void*)k_p2_scatter<2, false>, (const void*)k_p2_scatter<2, true>,
                        (const void*)k_p2_scatter<4, false>, (const void*)k_p2_scatter<4, true>};
    for (const void* f : fs) (void)hipFuncSetAttribute(f, hipFuncAttributeMaxDynamicSharedMemorySize, 160 * 1024);
    return true;
  }();
  (void)lds_attr;
  {
    TimedScope ts(h, "partition");
    if (hot) {
      // strided sample of up to 2^18 pairs; an owner is a candidate when its
      // hits predict >= kHotMinPairs pairs
      constexpr int64_t kSample = int64_t(1) << 18, kHotMinPairs = 2048;
      const int64_t S = std::min(npairs, kSample), stride = npairs / S;
      const uint32_t tau = (uint32_t)std::max<int64_t>(2, (kHotMinPairs * S + npairs - 1) / npairs);
      uint32_t* cnt = reinterpret_cast<uint32_t*>(slotkey + kHotBins);
      CMS_HIP(hipMemsetAsync(slotkey, 0, sizeof(unsigned long long) * kHotBins + sizeof(uint32_t) * (size_t)n,
                             h->stream));
      hipLaunchKernelGGL(k_hot_sample, dim3((unsigned)((S + kSamplePerBlock - 1) / kSamplePerBlock)), dim3(256), 0,
                         h->stream, d_row, stride, S, n, cnt);
      hipLaunchKernelGGL(k_hot_claim, dim3((unsigned)std::min<int64_t>((n + 255) / 256, 4096)), dim3(256), 0,
                         h->stream, cnt, n, tau, slotkey);
    }
    auto hist = R == 4 ? k_p1_hist<4> : R == 2 ? k_p1_hist<2> : k_p1_hist<1>;
    hipLaunchKernelGGL(hist, dim3(NB), dim3(256), sizeof(uint32_t) * (P + (hot ? kHotBins : 0)), h->stream, d_row,
                       npairs, s2, P1, n, H1, NB, h->d_flags, slotkey);
    // block-major (block, bin) offsets: chunked column sums, one scan over
    // the bins, chunk prefixes (the pass-2 kernels with one segment)
    CMS_HIP(hipMemsetD32Async(reinterpret_cast<hipDeviceptr_t>(seg1), 0, 1, h->stream));
    CMS_HIP(hipMemsetD32Async(reinterpret_cast<hipDeviceptr_t>(seg1 + 1), NB, 1, h->stream));
    hipLaunchKernelGGL(k_p2_colsum<kP1Split>, dim3(kP1Split), dim3(1024), 0, h->stream, H1, seg1, P, PS1);
    hipLaunchKernelGGL(k_p1_scan, dim3(1), dim3(1024), 0, h->stream, P, PS1, bs1);
    hipLaunchKernelGGL(k_p2_offsets<kP1Split>, dim3(kP1Split), dim3(1024), 0, h->stream, H1, seg1, P, PS1, O1);
    auto scat = d_val ? (R == 4 ? k_p1_scatter<4, true> : R == 2 ? k_p1_scatter<2, true> : k_p1_scatter<1, true>)
                      : (R == 4 ? k_p1_scatter<4, false> : R == 2 ? k_p1_scatter<2, false> : k_p1_scatter<1, false>);
    hipLaunchKernelGGL(scat, dim3(NB), dim3(kPartThreads), tile_lds_bytes(P, d_val != nullptr, true, hot, (int)tile1),
                       h->stream, d_row, d_key, d_val, npairs, s2, P1, n, O1, NB, fine, key1, val1, slotkey,
                       ckey, cval);
    // the hot-routed owners' keys are in place now (their pass-1 bins are
    // their final spans): the build may start on them beside pass 2
    h->p1_event = false;
    if (hot && h->tune.early_slices && h->plan_side_request && h->side_stream3 && !d_val && !h->plan_side_active) {
      CMS_HIP(hipEventRecord(h->ev_p1, h->stream));
      h->p1_event = true;
      h->p1_slotkey = slotkey;
      h->p1_bs1 = bs1;
      h->p1_P1 = P1;
      h->p1_nslots = kHotBins;
    }
    hipLaunchKernelGGL(k_p2_plan, dim3(1), dim3(1024), 0, h->stream, bs1, P1, CH2, binStart, blkStart);
    const int64_t g2h = std::min<int64_t>((nb2max + 7) & ~int64_t(7), (int64_t)h->num_cus * 8);
    hipLaunchKernelGGL(k_p2_hist, dim3((unsigned)g2h), dim3(256), sizeof(uint32_t) * P2, h->stream, fine,
                       binStart, blkStart, P1, CH2, P2, H2);
    hipLaunchKernelGGL(k_p2_colsum<kP2Split>, dim3(P1 * kP2Split), dim3(1024), 0, h->stream, H2, blkStart, P2, PS);
    hipLaunchKernelGGL(k_p2_scan, dim3(P1), dim3(1024), 0, h->stream, binStart, P1, P2, n, PS, coff);
    hipLaunchKernelGGL(k_p2_offsets<kP2Split>, dim3(P1 * kP2Split), dim3(1024), 0, h->stream, H2, blkStart, P2, PS, O2);
    int R2 = CMS_P2_ROUNDS;
    while (R2 > 1 && tile_lds_bytes(P2, d_val != nullptr, false, false, R2 * kPartTile) > 160 * 1024) R2 >>= 1;
    auto scat2 = d_val ? (R2 == 4 ? k_p2_scatter<4, true> : R2 == 2 ? k_p2_scatter<2, true> : k_p2_scatter<1, true>)
                       : (R2 == 4 ? k_p2_scatter<4, false> : R2 == 2 ? k_p2_scatter<2, false> : k_p2_scatter<1, false>);
    // one pass-2 workgroup per CU fits its LDS tile; a few per CU keep the
    // dispatcher ahead of the exits (multiple of 8: XCD-contiguous blocks)
    const int64_t g2s = std::min<int64_t>((nb2max + 7) & ~int64_t(7), (int64_t)h->num_cus * 2);
    // the owner spans need only the offsets: computed before the last
    // scatter, and marked so the build plan can run beside it
    if (hot) {
      int64_t* chi = h->ws_csr_hi.as<int64_t>();
      hipLaunchKernelGGL(k_spans_hi, dim3((unsigned)std::min<int64_t>((n + 255) / 256, 4096)), dim3(256), 0,
                         h->stream, coff, n, chi);
      hipLaunchKernelGGL(k_spans_hot, dim3(kHotBins / 256), dim3(256), 0, h->stream, slotkey, bs1, P1, coff, chi);
      *out_hi = chi;
    } else {
      *out_hi = coff + 1;
    }
    h->spans_event = false;
    if (h->plan_side_active) return set_error(CMS_E_STATE, "internal: partition inside the plan's swapped-stream section");
    if (h->plan_side_request && h->side_stream && !d_val) {
      CMS_HIP(hipEventRecord(h->ev_spans, h->stream));
      h->spans_event = true;
    }
    hipLaunchKernelGGL(scat2, dim3((unsigned)g2s), dim3(kPartThreads),
                       tile_lds_bytes(P2, d_val != nullptr, false, false, R2 * kPartTile), h->stream, fine, key1, val1,
                       binStart, blkStart, P1, CH2, P2, O2, ckey, cval, out_rows);
    CMS_HIP(hipGetLastError());
  }
  *out_lo = coff;
  *out_tok = ckey;
  *out_val = cval;
  return CMS_OK;
}

int partition_to_csr(cms_handle* h, const int64_t* d_row, const int64_t* d_key, const float* d_val, int64_t npairs,
                     int64_t** out_off, uint32_t** out_tok, float** out_val, int32_t* out_rows) {
  int64_t* hi;
  return partition_impl(h, d_row, d_key, d_val, npairs, false, out_off, &hi, out_tok, out_val, out_rows);
}

int partition_to_spans(cms_handle* h, const int64_t* d_row, const int64_t* d_key, const float* d_val, int64_t npairs,
                       int64_t** out_lo, int64_t** out_hi, uint32_t** out_tok, float** out_val) {
  return partition_impl(h, d_row, d_key, d_val, npairs, true, out_lo, out_hi, out_tok, out_val, nullptr);
}

}  // namespace cms
