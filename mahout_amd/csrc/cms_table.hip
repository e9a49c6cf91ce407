// cms_table.hip -- layout of the sketch table: u16 narrow slots (holding u16,
// u8 or nibble rows) + u32 hot slots.
//
// DoubleCountMinSketch keeps fp64 counters (T/impl/common/DoubleCountMinSketch.java:21);
// with integer increments every counter is an integer no larger than its
// owner's total increment (the row mass).  Rows whose mass stays below 2^16
// -- at config 2 all but the ~70 head items of the Zipf stream -- are stored
// as u16, the rest in a growable table of u32 rows ("hot slots").  A writer
// that could lift a row's mass to 2^16 promotes the row first (promote_rows),
// so no u16 counter can overflow and every stored value is the exact counter.
#include <hip/hip_runtime.h>

#include <algorithm>
#include <chrono>

#include "cms_internal.h"

namespace cms {

// claim >= 0: the list entry i also takes slot claim + i here (the caller
// reserved `reserved` slots, a proven bound), so the promotion needs no count
// on the host; a broken bound flags an overflow instead of writing past them.
__global__ void k_promote_list(const uint64_t* bound, const uint8_t* force, int32_t* hidx, int64_t n,
                               uint32_t* cnt, int32_t* list, int64_t claim, int64_t reserved, uint32_t* flags) {
  for (int64_t r = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; r < n; r += (int64_t)gridDim.x * blockDim.x) {
    if (hidx[r] >= 0) continue;
    const bool need = (bound && bound[r] >= kNarrowLimit) || (force && force[r]);
    if (need) {
      const uint32_t i = atomicAdd(cnt, 1u);
      if (claim >= 0 && (int64_t)i >= reserved) {
        atomicOr(flags, kFlagOverflow);
        continue;
      }
      list[i] = (int32_t)r;
      if (claim >= 0) hidx[r] = (int32_t)(claim + i);
    }
  }
}

// one workgroup per promoted row: slot base + i, old narrow counters copied
// (or zeros); dcount != nullptr: the list length is read on the device.
// whole_bound > 0 (a fresh build whose single-slice owners store their rows
// whole, k_build_slices): rows of bound <= whole_bound are not zeroed.
__global__ __launch_bounds__(256) void k_promote_rows(const int32_t* list, int64_t count, const uint32_t* dcount,
                                                      int64_t base, TableView tv, int32_t* hidx, int copy_old,
                                                      const uint64_t* bound, uint64_t whole_bound) {
  if (dcount) count = min<int64_t>(count, (int64_t)*dcount);
  for (int64_t i = blockIdx.x; i < count; i += gridDim.x) {
    const int64_t r = list[i];
    const int64_t slot = base + i;
    uint32_t* dst = tv.hot + slot * tv.dw;
    const bool skip = !copy_old && whole_bound > 0 && bound && bound[r] <= whole_bound;
    if (!skip)
      for (int64_t j = threadIdx.x; j < tv.dw; j += 256) dst[j] = copy_old ? tv.get(r, j) : 0u;  // any narrow form
    __syncthreads();  // every lane has read the row through its old form before the form changes
    if (threadIdx.x == 0) hidx[r] = (int32_t)slot;
  }
}

static int grow_hot(cms_handle* h, int64_t need) {
  if (need <= h->hot_cap) return CMS_OK;
  // (early slices may still be writing slots on their own stream: the copy
  // below must see their rows, and the old table outlive them)
  CMS_HIP(hipDeviceSynchronize());
  {  // grow: new slot table, live slots copied over
    // at least `need` (reserved-but-unclaimed slots can make it exceed n)
    const int64_t cap =
        std::max<int64_t>(need, std::min<int64_t>(h->n, std::max<int64_t>({need, h->hot_cap + h->hot_cap / 2, 64})));
    DevBuf nb;
    CMS_HIP(nb.ensure(sizeof(uint32_t) * (size_t)cap * (size_t)h->dw));
    if (h->hot_used > 0)
      CMS_HIP(hipMemcpyAsync(nb.ptr, h->hot_tab.ptr, sizeof(uint32_t) * (size_t)h->hot_used * (size_t)h->dw,
                             hipMemcpyDeviceToDevice, h->stream));
    CMS_HIP(hipStreamSynchronize(h->stream));
    h->hot_tab = std::move(nb);
    h->hot_cap = cap;
  }
  return CMS_OK;
}

int reserve_hot_slots(cms_handle* h, int64_t count, int64_t* base) {
  if (int rc = grow_hot(h, h->hot_used + count)) return rc;
  *base = h->hot_used;
  h->hot_used += count;
  return CMS_OK;
}

int promote_rows(cms_handle* h, const uint64_t* d_bound, const uint8_t* d_force, bool copy_old, int64_t max_new,
                 uint64_t whole_bound) {
  const int64_t n = h->n;
  CMS_HIP(h->ws_plist.ensure(sizeof(int32_t) * (size_t)(n + 1)));
  int32_t* list = h->ws_plist.as<int32_t>();
  uint32_t* cnt = reinterpret_cast<uint32_t*>(list + n);
  const unsigned g = (unsigned)std::max<int64_t>(1, std::min<int64_t>((n + 255) / 256, 8192));
  if (max_new >= 0) {
    // The caller bounds the rows this call can promote: reserve that many
    // slots, claim them on the device -- no host round trip inside the build.
    // Unclaimed reserved slots stay unused until the next layout reset.
    max_new = std::min<int64_t>(max_new, n);
    if (max_new == 0) return CMS_OK;
    if (h->hot_used + max_new > n) return promote_rows(h, d_bound, d_force, copy_old, -1, whole_bound);  // reservations spent
    int rc = grow_hot(h, h->hot_used + max_new);
    if (rc) return rc;
    CMS_HIP(hipMemsetAsync(cnt, 0, sizeof(uint32_t), h->stream));
    hipLaunchKernelGGL(k_promote_list, dim3(g), dim3(256), 0, h->stream, d_bound, d_force, h->d_hidx, n, cnt, list,
                       h->hot_used, max_new, h->d_flags);
    hipLaunchKernelGGL(k_promote_rows, dim3((unsigned)std::min<int64_t>(max_new, 65536)), dim3(256), 0, h->stream,
                       list, max_new, cnt, h->hot_used, h->tview(), h->d_hidx, copy_old ? 1 : 0, d_bound, whole_bound);
    CMS_HIP(hipGetLastError());
    h->hot_used += max_new;
    return CMS_OK;
  }
  CMS_HIP(hipMemsetAsync(cnt, 0, sizeof(uint32_t), h->stream));
  hipLaunchKernelGGL(k_promote_list, dim3(g), dim3(256), 0, h->stream, d_bound, d_force, h->d_hidx, n, cnt, list,
                     (int64_t)-1, (int64_t)0, h->d_flags);
  CMS_HIP(hipGetLastError());
  uint32_t c = 0;
  CMS_HIP(hipMemcpyAsync(&c, cnt, sizeof(uint32_t), hipMemcpyDeviceToHost, h->stream));
  CMS_HIP(hipStreamSynchronize(h->stream));
  if (c == 0) return CMS_OK;
  const int64_t need = h->hot_used + c;
  int rc = grow_hot(h, need);
  if (rc) return rc;
  hipLaunchKernelGGL(k_promote_rows, dim3((unsigned)std::min<int64_t>(c, 65536)), dim3(256), 0, h->stream, list,
                     (int64_t)c, (const uint32_t*)nullptr, h->hot_used, h->tview(), h->d_hidx, copy_old ? 1 : 0, d_bound,
                     whole_bound);
  CMS_HIP(hipGetLastError());
  h->hot_used = need;
  return CMS_OK;
}

// ---- narrow forms (u8 / 4-bit / 2-bit / 1-bit and list rows inside their u16 slots) ----

// Rows to widen before a write (see widen_rows in cms_internal.h).  With span
// bounds (lo, hi: the accumulate build's owner spans) a row is touched when it
// has keys -- the build rewrites every such row through its u16 / u32 image
// even when all its increments are 0 (no mass added).  A listed row's cbound
// becomes its bound after the write, which picks the form it widens to.
__device__ __forceinline__ int form_bits(int32_t f) {  // counter bits of a form (0: a list row)
  return f == kFormList ? 0 : f == kFormU1 ? 1 : f == kFormU2 ? 2 : f == kFormU4 ? 4 : f == kFormU8 ? 8 : 16;
}

// The form a listed row is rewritten in: the narrowest form wider than its
// own whose capacity holds its new bound nb (u16 for an accumulate build) --
// a 2-bit row that one more pair lifts to 4 becomes a 4-bit row.  The zero
// row counts as a list row (it holds nothing of its own).
// the smallest place a moved row takes (kCap class): a mover whose target
// form fits a u8 row takes a u8 place, one past it a whole slot.  With the
// rows' bounds from their tracked maxima most rows never pass u8: after the
// 1B-pair config-5 stream 78.7 GB in use against 102 GB with whole slots
// for every mover (scripts/stream_compact_probe.py)
#ifndef CMS_MOVE_CLASS
#define CMS_MOVE_CLASS 4
#endif
// widening bounds from the tracked row maxima (0: the accumulated cbound alone)
#ifndef CMS_WIDEN_ROWMAX
#define CMS_WIDEN_ROWMAX 1
#endif
__device__ __forceinline__ int32_t widen_target(int32_t f, uint32_t nb, int to_u16, int w) {
  if (to_u16) return kFormU16;
  if (f == kFormList && nb <= 1u && (w & 127) == 0) return kFormU1;
  if (form_bits(f) < 2 && nb <= 3u && (w & 63) == 0) return kFormU2;
  if (form_bits(f) < 4 && nb <= 15u) return kFormU4;
  if (form_bits(f) < 8 && nb <= 255u) return kFormU8;
  return kFormU16;
}

// A listed row is rewritten in place when its place holds the target form
// (its kCap class), else it moves to a place of class CMS_MOVE_CLASS (or a
// whole slot) at the arena's end (mv[i]: its offset in kRowAlign units among
// the cnt[1] units the movers take) -- places sized to each target form left
// a row moving once per widening (a 1B-pair stream then held 151 GB).  A
// touched row on the zero row is always listed.
__global__ void k_widen_mark(const uint64_t* bound, const uint64_t* old_mass, const int64_t* lo, const int64_t* hi,
                             const int32_t* hidx, const int64_t* off, uint32_t* cbound, const uint32_t* rowmax,
                             int64_t n, int all_touched, int to_u16, int w, int64_t dw, int32_t* list, int32_t* mv,
                             int8_t* tfa, uint32_t* cnt) {
  for (int64_t r = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; r < n; r += (int64_t)gridDim.x * blockDim.x) {
    const int32_t f = hidx[r];
    if (f >= 0) continue;
    const int64_t o = off[r];
    const int cc = (int)(o & kCapMask);
    if (f == kFormU16 && cc == kCapU16) continue;  // a u16 row in a whole slot takes its adds in place
    bool need = true;
    uint32_t nbv = cbound[r];
    if (bound) {
      const uint64_t b = bound[r], m = old_mass ? old_mass[r] : 0ULL;
      const bool has_keys = lo && hi[r] > lo[r];
      if (b <= m && !has_keys) continue;  // no update lands on this row
      // the row's current largest counter (rowmax, exact while the norms
      // are tracked) bounds it more tightly than the accumulated cbound
      const uint64_t cur = rowmax ? min<uint64_t>(cbound[r], rowmax[r]) : (uint64_t)cbound[r];
      const uint64_t nb = cur + (b - m);
      need = all_touched || nb > (uint64_t)form_cap(f) || o == 0;
      nbv = (uint32_t)min<uint64_t>(nb, 0xFFFFFFFFull);
      cbound[r] = nbv;  // <= the capacity of the form it keeps or takes
    }
    if (need) {
      const int32_t tf = widen_target(o == 0 ? kFormList : f, nbv, to_u16, w);
      const int tc = form_class(tf);
      const uint32_t i = atomicAdd(cnt, 1u);
      list[i] = (int32_t)r;
      tfa[i] = (int8_t)tf;
      const int mc = tc >= CMS_MOVE_CLASS ? kCapU16 : CMS_MOVE_CLASS;  // the class of a mover's new place
      mv[i] = (o != 0 && cc >= tc) ? -1 : (int32_t)atomicAdd(cnt + 1, (uint32_t)(class_units(mc, dw) / kRowAlign));
    }
  }
}

// 16 counters v[0..16) packed at 32 / C bits into C-counter words at w32[j / C ...]
template <int C>
__device__ __forceinline__ void pack16(const uint32_t (&v)[16], uint32_t* w32, int64_t j) {
#pragma unroll
  for (int q = 0; q < 16; q += C) {
    uint32_t word = 0;
#pragma unroll
    for (int k = 0; k < C; ++k) word |= v[q + k] << (k * (32 / C));
    w32[(j + q) / C] = word;
  }
}

// One workgroup per listed row, rewritten (in place, or into a mover's new
// slot at base + mv[i] * kRowAlign) in its target form tfa[i] (widen_target:
// the narrowest form
// wider than its own whose capacity holds its new bound (cbound), u16 for an
// accumulate build (to_u16) -- a 2-bit row that one more pair lifts to 4
// becomes a 4-bit row (half the bytes of u8, a quarter of u16).
//  * dense forms: the image of counters [c0, c1) at tb >= sb bits covers
//    bytes [c0 tb/8, c1 tb/8), which hold only old bytes of counters >= c0;
//    so chunks of 4096 counters go from the top down, each read completely
//    (16 counters per lane) before any lane writes it.
//  * list rows: every entry is read first (at most 32 per lane: d <= 32,
//    m <= 256), then each sketch row is counted in LDS (u8 counters, four per
//    word: a list row's counters are < 2^8) and leaves packed.
__global__ __launch_bounds__(256) void k_widen_rows(const int32_t* list, const int32_t* mv, const int8_t* tfa,
                                                    const uint32_t* dcount, TableView tv, int64_t* off_w, int64_t base,
                                                    int32_t* hidx) {
  extern __shared__ uint32_t lc[];  // [w / 4] (list rows)
  const int64_t count = *dcount;
  const int64_t dw = tv.dw;
  const int w = tv.w;
  constexpr int64_t kChunk = 256 * 16;
  for (int64_t i = blockIdx.x; i < count; i += gridDim.x) {
    const int64_t r = list[i];
    const int32_t f = hidx[r];
    const int32_t tf = tfa[i];
    const int tb = form_bits(tf);
    const uint16_t* src = tv.row16(r);
    const int64_t dst_off = mv[i] >= 0 ? base + (int64_t)mv[i] * kRowAlign : tv.base(r);
    const uint8_t* p8 = reinterpret_cast<const uint8_t*>(src);
    uint32_t* w32 = reinterpret_cast<uint32_t*>(tv.t16 + dst_off);
    if (f == kFormList) {
      const uint32_t m = tv.list_m(r);
      const uint32_t ne = (uint32_t)(dw / w) * m;
      uint32_t ent[32];
#pragma unroll
      for (int q = 0; q < 32; ++q) {
        const uint32_t t = threadIdx.x + 256u * q;
        ent[q] = 0xFFFFFFFFu;
        if (t < ne) ent[q] = (t / m) << 16 | src[1 + t];  // sketch row, bucket
      }
      const int cpw = 32 / tb;  // counters per output word
      for (int rr = 0; (int64_t)rr * w < dw; ++rr) {
        for (int j = threadIdx.x; j < (w >> 2); j += 256) lc[j] = 0u;
        __syncthreads();  // (the first pass: every entry is also read before any store below)
#pragma unroll
        for (int q = 0; q < 32; ++q)
          if (ent[q] != 0xFFFFFFFFu && (int)(ent[q] >> 16) == rr)
            atomicAdd(&lc[(ent[q] & 0xFFFFu) >> 2], 1u << ((ent[q] & 3u) * 8u));
        __syncthreads();
        const uint8_t* c8 = reinterpret_cast<const uint8_t*>(lc);
        for (int q = threadIdx.x; q < w / cpw; q += 256) {
          uint32_t word = 0;
          for (int k = 0; k < cpw; ++k) word |= (uint32_t)c8[q * cpw + k] << (k * tb);
          w32[((int64_t)rr * w) / cpw + q] = word;
        }
        __syncthreads();  // the counts are packed before the next sketch row zeroes them
      }
    } else {
      for (int64_t c0 = ((dw - 1) / kChunk) * kChunk; c0 >= 0; c0 -= kChunk) {
        const int64_t j = c0 + (int64_t)threadIdx.x * 16;  // this lane's 16 counters
        uint32_t v[16];
        if (j < dw) {
          if (f == kFormU16) {  // a mover's u16 row (the zero row): copied
            const uint4 x0 = *reinterpret_cast<const uint4*>(src + j);
            const uint4 x1 = *reinterpret_cast<const uint4*>(src + j + 8);
            const uint32_t wv[8] = {x0.x, x0.y, x0.z, x0.w, x1.x, x1.y, x1.z, x1.w};
#pragma unroll
            for (int q = 0; q < 16; ++q) v[q] = (wv[q >> 1] >> ((q & 1) * 16)) & 0xFFFFu;
          } else if (f == kFormU8) {
            const uint4 x = *reinterpret_cast<const uint4*>(p8 + j);
            const uint32_t wv[4] = {x.x, x.y, x.z, x.w};
#pragma unroll
            for (int q = 0; q < 16; ++q) v[q] = (wv[q >> 2] >> ((q & 3) * 8)) & 255u;
          } else if (f == kFormU2) {
            const uint32_t x = *reinterpret_cast<const uint32_t*>(p8 + (j >> 2));
#pragma unroll
            for (int q = 0; q < 16; ++q) v[q] = (x >> (q * 2)) & 3u;
          } else if (f == kFormU1) {
            const uint32_t x = *reinterpret_cast<const uint16_t*>(p8 + (j >> 3));
#pragma unroll
            for (int q = 0; q < 16; ++q) v[q] = (x >> q) & 1u;
          } else {
            const uint2 x = *reinterpret_cast<const uint2*>(p8 + (j >> 1));
            const uint32_t wv[2] = {x.x, x.y};
#pragma unroll
            for (int q = 0; q < 16; ++q) v[q] = (wv[q >> 3] >> ((q & 7) * 4)) & 15u;
          }
        }
        __syncthreads();  // the whole chunk is read before any lane overwrites it
        if (j < dw) {  // 16 counters at tb bits: tb / 2 words from word j tb / 32
          if (tb == 2) pack16<16>(v, w32, j);
          else if (tb == 4) pack16<8>(v, w32, j);
          else if (tb == 8) pack16<4>(v, w32, j);
          else pack16<2>(v, w32, j);
        }
        __syncthreads();  // the next (lower) chunk's old bytes are read after these stores
      }
    }
    if (threadIdx.x == 0) {
      hidx[r] = tf;
      if (mv[i] >= 0) off_w[r] = dst_off | (form_class(tf) >= CMS_MOVE_CLASS ? kCapU16 : CMS_MOVE_CLASS);  // (k_widen_mark)
    }
  }
}

int widen_rows(cms_handle* h, const uint64_t* d_bound, const uint64_t* old_mass, bool all_touched, const int64_t* d_lo,
               const int64_t* d_hi) {
  if (!h->forms_ok) return CMS_OK;  // (every row in a full slot, u16)
  TimedScope ts(h, "widen_rows");
  const int64_t n = h->n;
  CMS_HIP(h->ws_plist.ensure(sizeof(int32_t) * (size_t)(n + 1)));
  CMS_HIP(h->ws_layout.ensure(sizeof(int32_t) * (size_t)(n + 4) + (size_t)n));
  int32_t* list = h->ws_plist.as<int32_t>();
  int32_t* mv = h->ws_layout.as<int32_t>();
  uint32_t* cnt = reinterpret_cast<uint32_t*>(mv + n);  // [0] listed rows, [1] the movers' kRowAlign units
  int8_t* tfa = reinterpret_cast<int8_t*>(mv + n + 4);  // [n] target forms
  CMS_HIP(hipMemsetAsync(cnt, 0, 2 * sizeof(uint32_t), h->stream));
  const unsigned g = (unsigned)std::max<int64_t>(1, std::min<int64_t>((n + 255) / 256, 8192));
  // u16 for an accumulate build or when no bound is known
  const int to_u16 = (all_touched || !d_bound) ? 1 : 0;
  // (the row maxima are current when the norms are: every writer tracks them then)
  const uint32_t* rmax = h->norms_valid && CMS_WIDEN_ROWMAX ? h->d_rowmax : nullptr;
  hipLaunchKernelGGL(k_widen_mark, dim3(g), dim3(256), 0, h->stream, d_bound, old_mass, d_lo, d_hi, h->d_hidx,
                     h->d_off, h->d_cbound, rmax, n, all_touched ? 1 : 0, to_u16, h->p.width, h->dw, list, mv, tfa,
                     cnt);
  CMS_HIP(hipGetLastError());
  // movers take whole slots at the arena's end: the units they need size it
  // (a handle without compact rows has no movers and skips the read-back)
  int64_t base = h->t16_used;
  if (h->compact) {
    CMS_HIP(hipMemcpyAsync(h->h_pin + 8, cnt + 1, sizeof(uint32_t), hipMemcpyDeviceToHost, h->stream));
    CMS_HIP(hipStreamSynchronize(h->stream));
    const int64_t units = (int64_t)h->h_pin[8] * kRowAlign;
    if (units > 0) {
      int rc = arena_reserve(h, h->t16_used + units, true);
      if (rc) return rc;
      h->t16_used += units;
    }
  }
  // one workgroup per row, looping: the row count stays on the device
  hipLaunchKernelGGL(k_widen_rows, dim3((unsigned)std::min<int64_t>(n, 8192)), dim3(256), (size_t)h->p.width,
                     h->stream, list, mv, tfa, cnt, h->tview(), h->d_off, base, h->d_hidx);
  CMS_HIP(hipGetLastError());
  return CMS_OK;
}

// [0..5] hot, u16, u8, 4-bit, 2-bit, 1-bit rows, [6] list rows, [7] their
// bytes, [8] u16 rows on the shared zero row (counted in [1] too)
__global__ void k_count_forms(TableView tv, int64_t n, unsigned long long* out) {
  uint32_t c[8] = {0, 0, 0, 0, 0, 0, 0, 0};
  unsigned long long lb = 0;
  const uint64_t d = (uint64_t)(tv.dw / tv.w);
  for (int64_t r = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; r < n; r += (int64_t)gridDim.x * blockDim.x) {
    const int32_t f = tv.hidx[r];
    c[f >= 0 ? 0 : f == kFormU16 ? 1 : f == kFormU8 ? 2 : f == kFormU4 ? 3 : f == kFormU2 ? 4 : f == kFormU1 ? 5 : 6] += 1;
    if (f == kFormList) lb += 2 + 2 * d * tv.list_m(r);
    if (f == kFormU16 && tv.off[r] == 0) c[7] += 1;
  }
  for (int q = 0; q < 7; ++q)
    if (c[q]) atomicAdd(out + q, (unsigned long long)c[q]);
  if (lb) atomicAdd(out + 7, lb);
  if (c[7]) atomicAdd(out + 8, (unsigned long long)c[7]);
}

int count_forms(cms_handle* h, int64_t out[9]) {
  DevBuf tmp;
  CMS_HIP(tmp.ensure(9 * sizeof(unsigned long long)));
  CMS_HIP(hipMemsetAsync(tmp.ptr, 0, 9 * sizeof(unsigned long long), h->stream));
  const unsigned g = (unsigned)std::max<int64_t>(1, std::min<int64_t>((h->n + 255) / 256, 4096));
  hipLaunchKernelGGL(k_count_forms, dim3(g), dim3(256), 0, h->stream, h->tview(), h->n, tmp.as<unsigned long long>());
  CMS_HIP(hipGetLastError());
  unsigned long long c[9];
  CMS_HIP(hipMemcpyAsync(c, tmp.ptr, sizeof(c), hipMemcpyDeviceToHost, h->stream));
  CMS_HIP(hipStreamSynchronize(h->stream));
  for (int q = 0; q < 9; ++q) out[q] = (int64_t)c[q];
  return CMS_OK;
}

__global__ void k_count_hot(const int32_t* hidx, int64_t n, unsigned long long* out) {
  uint32_t c = 0;
  for (int64_t r = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; r < n; r += (int64_t)gridDim.x * blockDim.x)
    c += hidx[r] >= 0;
  if (c) atomicAdd(out, (unsigned long long)c);
}

int count_hot_rows(cms_handle* h, int64_t* out) {
  DevBuf tmp;
  CMS_HIP(tmp.ensure(sizeof(unsigned long long)));
  CMS_HIP(hipMemsetAsync(tmp.ptr, 0, sizeof(unsigned long long), h->stream));
  const unsigned g = (unsigned)std::max<int64_t>(1, std::min<int64_t>((h->n + 255) / 256, 4096));
  hipLaunchKernelGGL(k_count_hot, dim3(g), dim3(256), 0, h->stream, h->d_hidx, h->n, tmp.as<unsigned long long>());
  CMS_HIP(hipGetLastError());
  unsigned long long c = 0;
  CMS_HIP(hipMemcpyAsync(&c, tmp.ptr, sizeof(c), hipMemcpyDeviceToHost, h->stream));
  CMS_HIP(hipStreamSynchronize(h->stream));
  *out = (int64_t)c;
  return CMS_OK;
}

// counters of rows [r0, r0 + rc) as u32, [rc][dw] (cms_read_counters_device)
__global__ void k_read_u32(TableView tv, int64_t r0, int64_t rc, uint32_t* out, int vec) {
  const int64_t total = rc * tv.dw;
  for (int64_t i = (blockIdx.x * (int64_t)blockDim.x + threadIdx.x) * 4; i < total;
       i += (int64_t)gridDim.x * blockDim.x * 4) {
    const int64_t r = i / tv.dw, j = i - r * tv.dw;
    if (vec) {
      *reinterpret_cast<uint4*>(out + i) =
          tv.hidx[r0 + r] == kFormList ? make_uint4(0, 0, 0, 0) : tv.get4(r0 + r, j);  // lists: k_read_lists
    } else {
      for (int64_t e = i; e < min(i + 4, total); ++e) {
        const int64_t re = e / tv.dw;
        out[e] = tv.hidx[r0 + re] == kFormList ? 0u : tv.get(r0 + re, e - re * tv.dw);
      }
    }
  }
}

// list rows of [r0, r0 + rc): their entries added into the zeros k_read_u32 left
__global__ void k_read_lists(TableView tv, int64_t r0, int64_t rc, uint32_t* out) {
  for (int64_t r = blockIdx.x; r < rc; r += gridDim.x) {
    if (tv.hidx[r0 + r] != kFormList) continue;
    const uint32_t m = tv.list_m(r0 + r);
    const int64_t ne = (tv.dw / tv.w) * (int64_t)m;
    const uint16_t* e = tv.row16(r0 + r) + 1;
    for (int64_t t = threadIdx.x; t < ne; t += blockDim.x)
      atomicAdd(out + r * tv.dw + (t / m) * tv.w + e[t], 1u);
  }
}

int read_counters_device(cms_handle* h, int64_t r0, int64_t rc, uint32_t* d_out) {
  if (rc <= 0) return CMS_OK;
  if (h->empty) {
    CMS_HIP(hipMemsetAsync(d_out, 0, sizeof(uint32_t) * (size_t)rc * (size_t)h->dw, h->stream));
    return CMS_OK;
  }
  const int64_t quads = (rc * h->dw + 3) / 4;
  const unsigned g = (unsigned)std::max<int64_t>(1, std::min<int64_t>((quads + 255) / 256, 65536));
  const int vec = (h->dw & 3) == 0 && ((uintptr_t)d_out & 15) == 0;
  hipLaunchKernelGGL(k_read_u32, dim3(g), dim3(256), 0, h->stream, h->tview(), r0, rc, d_out, vec);
  if (h->forms_ok)
    hipLaunchKernelGGL(k_read_lists, dim3((unsigned)std::min<int64_t>(rc, 65536)), dim3(256), 0, h->stream,
                       h->tview(), r0, rc, d_out);
  CMS_HIP(hipGetLastError());
  return CMS_OK;
}

int reset_table_layout(cms_handle* h) {
  CMS_HIP(hipMemsetAsync(h->d_hidx, 0xff, sizeof(int32_t) * (size_t)h->n, h->stream));
  h->hot_used = 0;
  return CMS_OK;
}

// ---- the narrow-row arena (cms_internal.h TableView) ----

__global__ void k_off_identity(int64_t* off, int64_t n, int64_t su) {
  for (int64_t r = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; r < n; r += (int64_t)gridDim.x * blockDim.x)
    off[r] = (su + r * su) | kCapU16;
}

// Virtual arena: physical chunks mapped at the end of the reserved range.
static int arena_map(cms_handle* h, size_t want) {
  hipMemAllocationProp prop = {};
  prop.type = hipMemAllocationTypePinned;
  prop.location.type = hipMemLocationTypeDevice;
  prop.location.id = h->device;
  const size_t g = h->arena_gran;
  const auto t0 = std::chrono::steady_clock::now();
  const size_t bytes = std::min(h->arena_va_bytes - h->arena_mapped, (want - h->arena_mapped + g - 1) / g * g);
  if (h->arena_mapped + bytes < want) return set_error(CMS_E_OOM, "row arena: %.2f GB exceeds its reserved range", 1e-9 * want);
  hipMemGenericAllocationHandle_t mem;
  hipError_t e = hipMemCreate(&mem, bytes, &prop, 0);
  const auto t1 = std::chrono::steady_clock::now();
  if (e != hipSuccess) {
    (void)hipGetLastError();
    return set_error(CMS_E_OOM, "row arena chunk of %.2f GB: %s", 1e-9 * bytes, hipGetErrorString(e));
  }
  char* at = static_cast<char*>(h->arena_va) + h->arena_mapped;
  hipMemAccessDesc acc = {};
  acc.location = prop.location;
  acc.flags = hipMemAccessFlagsProtReadWrite;
  // (access is set over the whole mapped range from the reservation's start:
  // on this ROCm a sub-range starting inside it is refused once other
  // allocations exist -- scripts/vmm_probe.cpp)
  std::chrono::steady_clock::time_point t2;
  if ((e = hipMemMap(at, bytes, 0, mem, 0)) != hipSuccess || (t2 = std::chrono::steady_clock::now(), false) ||
      (e = hipMemSetAccess(h->arena_va, h->arena_mapped + bytes, &acc, 1)) != hipSuccess) {
    (void)hipMemUnmap(at, bytes);
    (void)hipMemRelease(mem);
    (void)hipGetLastError();
    return set_error(CMS_E_HIP, "row arena map: %s", hipGetErrorString(e));
  }
  h->arena_chunks.push_back({mem, bytes});
  h->arena_mapped += bytes;
  if (h->timing) {  // host time of the mapping (cms_get_timing "arena_map"; its create / map / access parts)
    const auto t3 = std::chrono::steady_clock::now();
    auto add = [h](const char* name, double ms) {
      auto& a = h->timing_acc[name];
      a.total_ms += ms;
      a.launches += 1;
    };
    using ms = std::chrono::duration<double, std::milli>;
    add("arena_map", ms(t3 - t0).count());
    add("arena_map_create", ms(t1 - t0).count());
    add("arena_map_map", ms(t2 - t1).count());
    add("arena_map_access", ms(t3 - t2).count());
  }
  return CMS_OK;
}

// unmaps trailing chunks wholly above `keep_bytes` (the caller has drained the stream)
static void arena_unmap_above(cms_handle* h, size_t keep_bytes) {
  while (!h->arena_chunks.empty()) {
    const auto c = h->arena_chunks.back();
    if (h->arena_mapped - c.bytes < keep_bytes) break;
    char* at = static_cast<char*>(h->arena_va) + (h->arena_mapped - c.bytes);
    (void)hipMemUnmap(at, c.bytes);
    (void)hipMemRelease(c.mem);
    h->arena_chunks.pop_back();
    h->arena_mapped -= c.bytes;
  }
}

void arena_release(cms_handle* h) {
  if (h->arena_va) {
    arena_unmap_above(h, 0);
    (void)hipMemAddressFree(h->arena_va, h->arena_va_bytes);
    h->arena_va = nullptr;
    h->d_t16 = nullptr;  // (not a hipMalloc pointer)
  } else if (h->d_t16) {
    (void)hipFree(h->d_t16);
    h->d_t16 = nullptr;
  }
}

int arena_reserve(cms_handle* h, int64_t need, bool keep) {
  const int64_t su = slot_units(h->dw);
  need = std::max(need, su);
  // A re-laid-out table gives back what it no longer needs -- once three
  // layouts in a row wanted under a quarter of the arena: a multi-rank step
  // alternates a small local build with the larger merged layout, and
  // unmapping and mapping that difference every step would cost more than
  // it frees.
  bool shrink = false;
  if (!keep) {
    const int64_t have = h->arena_va ? (int64_t)(h->arena_mapped / sizeof(uint16_t)) : h->t16_cap;
    h->arena_small_layouts = have > 4 * need + (int64_t)(h->arena_gran / sizeof(uint16_t)) ? h->arena_small_layouts + 1 : 0;
    shrink = h->arena_small_layouts >= 3;
    if (shrink) h->arena_small_layouts = 0;
  }
  if (h->arena_va) {
    const size_t want = sizeof(uint16_t) * (size_t)need;
    if (shrink) {
      CMS_HIP(hipDeviceSynchronize());
      arena_unmap_above(h, want);
    }
    if (want > h->arena_mapped) {
      const bool first = h->arena_mapped == 0;
      // a growing table (rows moving to slots) maps a quarter more than it needs
      const size_t ask = std::max(keep ? std::min(h->arena_va_bytes, want + want / 4) : want, want);
      int rc = arena_map(h, ask);
      if (rc && ask > want) rc = arena_map(h, want);  // (short of memory: without the headroom)
      if (rc) return rc;
      if (first) CMS_HIP(hipMemsetAsync(h->arena_va, 0, sizeof(uint16_t) * (size_t)su, h->stream));  // the zero row
    }
    h->t16_cap = (int64_t)(h->arena_mapped / sizeof(uint16_t));
    return CMS_OK;
  }
  if (shrink) {  // (its rows are dead: a smaller arena)
    CMS_HIP(hipFree(h->d_t16));
    h->d_t16 = nullptr;
    h->t16_cap = 0;
  }
  if (need <= h->t16_cap) return CMS_OK;
  // a growing arena takes some headroom (bounded by every row in a slot of its own)
  int64_t cap = need;
  if (keep) cap = std::max(need, std::min<int64_t>(h->t16_cap + h->t16_cap / 2, su * (h->n + 1) + h->t16_used));
  uint16_t* nb = nullptr;
  hipError_t e = hipMalloc((void**)&nb, sizeof(uint16_t) * (size_t)cap);
  if (e != hipSuccess) {
    (void)hipGetLastError();
    return set_error(CMS_E_OOM, "row arena of %.2f GB: %s", 2e-9 * (double)cap, hipGetErrorString(e));
  }
  if (keep && h->t16_used > 0) {
    CMS_HIP(hipMemcpyAsync(nb, h->d_t16, sizeof(uint16_t) * (size_t)h->t16_used, hipMemcpyDeviceToDevice, h->stream));
  } else {
    CMS_HIP(hipMemsetAsync(nb, 0, sizeof(uint16_t) * (size_t)su, h->stream));  // the zero row
  }
  CMS_HIP(hipStreamSynchronize(h->stream));
  if (h->d_t16) CMS_HIP(hipFree(h->d_t16));
  h->d_t16 = nb;
  h->t16_cap = cap;
  return CMS_OK;
}

int init_row_offsets(cms_handle* h) {
  const int64_t su = slot_units(h->dw);
  if (h->compact && !h->tune.no_vmm) {
    // the virtual range: room for a compact layout plus every row moved once
    // to a whole slot of its own (2 x a slot per row); physical chunks map on demand
    hipMemAllocationProp prop = {};
    prop.type = hipMemAllocationTypePinned;
    prop.location.type = hipMemLocationTypeDevice;
    prop.location.id = h->device;
    size_t g = 0;
    if (hipMemGetAllocationGranularity(&g, &prop, hipMemAllocationGranularityRecommended) == hipSuccess && g > 0) {
      // map in chunks of 64 MB multiples (a small table: 1/64 of its slot layout)
      const size_t slots = sizeof(uint16_t) * (size_t)su * (size_t)(h->n + 1);
      g = std::max(g, std::min<size_t>(size_t(64) << 20, (slots / 64 + g - 1) / g * g));
      const size_t va = ((size_t)4 * sizeof(uint16_t) * (size_t)su * (size_t)(h->n + 1) + 2 * g) / g * g;
      void* p = nullptr;
      if (hipMemAddressReserve(&p, va, g, nullptr, 0) == hipSuccess) {
        h->arena_va = p;
        h->arena_va_bytes = va;
        h->arena_gran = g;
        h->d_t16 = static_cast<uint16_t*>(p);
      }
    }
    (void)hipGetLastError();  // (no virtual memory API: the hipMalloc arena)
  }
  if (h->compact) {  // every row on the zero row until a build lays it out
    int rc = arena_reserve(h, su, false);
    if (rc) return rc;
    CMS_HIP(hipMemsetAsync(h->d_off, 0, sizeof(int64_t) * (size_t)h->n, h->stream));
    h->t16_used = su;
  } else {  // a full slot per row, in row order
    int rc = arena_reserve(h, su * (h->n + 1), false);
    if (rc) return rc;
    const unsigned g = (unsigned)std::max<int64_t>(1, std::min<int64_t>((h->n + 255) / 256, 8192));
    hipLaunchKernelGGL(k_off_identity, dim3(g), dim3(256), 0, h->stream, h->d_off, h->n, su);
    CMS_HIP(hipGetLastError());
    h->t16_used = su * (h->n + 1);
  }
  CMS_HIP(hipStreamSynchronize(h->stream));
  return CMS_OK;
}

int reset_rows_zero(cms_handle* h) {
  const int64_t su = slot_units(h->dw);
  if (h->compact) {
    CMS_HIP(hipMemsetAsync(h->d_off, 0, sizeof(int64_t) * (size_t)h->n, h->stream));
    h->t16_used = su;
  } else {
    CMS_HIP(hipMemsetAsync(h->d_t16 + su, 0, sizeof(uint16_t) * (size_t)(su * h->n), h->stream));
  }
  return reset_table_layout(h);
}

// off[r] from the rows' capacities (128-B units): the rows follow the zero
// row in row order; a row of capacity 0 (a hot row) points at the zero row
__global__ void k_row_offsets(const uint32_t* caps, const uint32_t* ex, int64_t n, int64_t su, int64_t dw, int64_t* off,
                              uint32_t* total) {
  for (int64_t r = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; r < n; r += (int64_t)gridDim.x * blockDim.x) {
    const uint32_t c = caps[r];
    off[r] = c ? (su + (int64_t)ex[r] * kRowAlign) | class_of_units((int64_t)c * kRowAlign, dw) : 0;
    if (r == n - 1) *total = ex[r] + c;
  }
}

int row_layout(cms_handle* h, const uint32_t* d_caps, uint32_t* d_scratch) {
  const int64_t n = h->n, su = slot_units(h->dw);
  if (n <= 0) return CMS_OK;
  uint32_t* ex = d_scratch;           // [n]
  uint32_t* total = d_scratch + n;    // [1]
  uint32_t* bsum = d_scratch + n + 4; // [n / 4096 + 1]
  int rc = scan_exclusive_u32(h, d_caps, ex, n, bsum);
  if (rc) return rc;
  const unsigned g = (unsigned)std::max<int64_t>(1, std::min<int64_t>((n + 255) / 256, 8192));
  hipLaunchKernelGGL(k_row_offsets, dim3(g), dim3(256), 0, h->stream, d_caps, ex, n, su, h->dw, h->d_off, total);
  CMS_HIP(hipGetLastError());
  CMS_HIP(hipMemcpyAsync(h->h_pin + 8, total, sizeof(uint32_t), hipMemcpyDeviceToHost, h->stream));
  CMS_HIP(hipStreamSynchronize(h->stream));
  const int64_t used = su + (int64_t)h->h_pin[8] * kRowAlign;
  const int64_t want = used + used / 16;  // (a little headroom for the next build)
  if ((rc = arena_reserve(h, want, false))) return rc;  // (an arena grown by earlier writers shrinks back)
  h->t16_used = used;
  return CMS_OK;
}

}  // namespace cms
