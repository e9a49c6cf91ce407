// cms_merge.hip -- counter-width-adaptive merge of per-rank sketch tables.
//
// Each rank holds a full-shape partial table built from its user-hash shard of
// the stream; the merged table is the elementwise sum (counters are linear).
// Summing the u32 table as is moves 4 B per counter over xGMI.  Most of it is
// headroom: a merged counter of owner o can never exceed
//     bound(o) = min(sum_g mass_g(o), sum_g max_g(o))
// (mass = the owner's total increment, max = its largest local counter), and
// both sums are one small all-reduce of 2n words.  So each owner's counters
// travel as b(o) = bit_length(bound(o)) -bit fields packed floor(64/b) to a
// u64 word (no field straddles a word; field f of word i is counter f*NW + i), and the packed words are all-reduced
// as plain u64 sums: every partial sum of a field is <= its final value <
// 2^b, so no carry ever crosses a field and the packed sum IS the packed
// merged table, bit for bit.  Owners with bound 0 send nothing.
//
// The unpack writes the merged u32 table and, in the same pass, the exact
// per-row norms and row maxima the cosine needs (no second table read).
#include <hip/hip_runtime.h>

#include <algorithm>
#include <vector>

#include "cms_device.h"
#include "cms_internal.h"

namespace cms {

typedef unsigned short u16x2 __attribute__((ext_vector_type(2)));

// [0, n): local row mass (copied in), [n, 2n): local row max, widened to u64.
__global__ void k_merge_bounds_in(const uint64_t* mass, const uint32_t* rowmax, int64_t n, uint64_t* out) {
  for (int64_t i = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; i < n; i += (int64_t)gridDim.x * blockDim.x) {
    out[i] = mass[i];
    out[n + i] = rowmax[i];
  }
}

// After the bounds all-reduce: merged mass back into row_mass (overflow check:
// a row whose total increment reaches 2^32 could overflow a u32 counter).
__global__ void k_merge_bounds_out(const uint64_t* sums, int64_t n, uint64_t* mass, uint32_t* flags) {
  for (int64_t i = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; i < n; i += (int64_t)gridDim.x * blockDim.x) {
    mass[i] = sums[i];
    if (sums[i] >= (1ULL << 32)) atomicOr(flags, kFlagOverflow);
  }
}

struct PackLayout {
  const uint8_t* bits;   // [n] field width per owner (0: owner sends nothing)
  const int64_t* woff;   // [n+1] first packed word per owner
};

// One workgroup per owner.  Field f of the owner's word i holds counter
// f*NW + i (NW = the owner's word count): both the pack's reads and the
// unpack's word reads are then consecutive across the lanes of a wave.
// use_img: a narrow owner's d x w counters are first staged in LDS with
// 16-byte loads, and the words are assembled from there.
__global__ __launch_bounds__(256) void k_merge_pack(TableView tv, int64_t n, int64_t dw, PackLayout L,
                                                   uint64_t* words, int use_img) {
  extern __shared__ __align__(16) uint16_t img[];  // [dw] (use_img)
  for (int64_t o = blockIdx.x; o < n; o += gridDim.x) {
    const int b = L.bits[o];
    if (b == 0) continue;
    const int F = 64 / b;
    const int64_t w0 = L.woff[o], nw = L.woff[o + 1] - w0;
    const int32_t slot = tv.hidx[o];
    const uint32_t* s32 = slot >= 0 ? tv.hot + (int64_t)slot * dw : nullptr;
    const uint16_t* s16 = tv.row16(o);
    if (use_img && (slot == kFormU16 || slot == kFormList)) {
      uint4* l4 = reinterpret_cast<uint4*>(img);
      if (slot == kFormList) {  // zeros, then each entry adds 1 into its half of an LDS word (counts < 2^8)
        for (int64_t j = threadIdx.x; j < (dw >> 3); j += 256) l4[j] = make_uint4(0, 0, 0, 0);
        __syncthreads();
        const uint32_t m = tv.list_m(o);
        const int64_t ne = (dw / tv.w) * (int64_t)m;
        uint32_t* i32 = reinterpret_cast<uint32_t*>(img);
        for (int64_t t = threadIdx.x; t < ne; t += 256) {
          const uint32_t idx = (uint32_t)((t / m) * tv.w + s16[1 + t]);
          atomicAdd(i32 + (idx >> 1), 1u << ((idx & 1u) << 4));
        }
      } else {
        const uint4* g4 = reinterpret_cast<const uint4*>(s16);
        for (int64_t j = threadIdx.x; j < (dw >> 3); j += 256) l4[j] = g4[j];
      }
      __syncthreads();
      for (int64_t i = threadIdx.x; i < nw; i += 256) {
        uint64_t wv = 0;
        int64_t idx = i;
        for (int f = 0; f < F && idx < dw; ++f, idx += nw) wv |= (uint64_t)img[idx] << (f * b);
        words[w0 + i] = wv;
      }
      __syncthreads();
      continue;
    }
    for (int64_t i = threadIdx.x; i < nw; i += 256) {
      uint64_t wv = 0;
      for (int f = 0; f < F; ++f) {
        const int64_t idx = (int64_t)f * nw + i;
        if (idx < dw)  // u8 / nibble rows through the view
          wv |= (uint64_t)(s32 ? s32[idx] : slot == kFormU16 ? (uint32_t)s16[idx] : tv.get(o, idx)) << (f * b);
      }
      words[w0 + i] = wv;
    }
  }
}

// Merged words -> u32 table, with the exact per-row sum of squares and the
// owner's largest counter (as k_norms computes them).  use_img: a narrow
// owner's fields are first scattered into an LDS image of its d x w u16
// counters (one word read per F counters, no per-counter division), which
// then leaves as 16-byte row-major stores while the norms are summed.
// mforms (compact rows, row_layout by k_merge_caps): a narrow owner whose
// field width b <= 8 (so every merged counter < 2^b) leaves as a u8 row, b <= 4
// as a 4-bit row; an owner of b = 0 stays on the zero row.
__global__ void k_merge_caps(const uint8_t* bits, const int32_t* hidx, int64_t n, int64_t dw, int mforms,
                             uint32_t* caps) {
  const uint32_t full = (uint32_t)(slot_units(dw) / kRowAlign);
  for (int64_t o = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; o < n; o += (int64_t)gridDim.x * blockDim.x) {
    const int b = bits[o];
    const int64_t u16s = !mforms || b > 8 ? slot_units(dw) : b > 4 ? dw / 2 : dw / 4;
    caps[o] = hidx[o] >= 0 || b == 0 ? 0u : u16s == slot_units(dw) ? full : (uint32_t)((u16s + kRowAlign - 1) / kRowAlign);
  }
}

__global__ __launch_bounds__(256) void k_merge_unpack(const uint64_t* words, int64_t n, HashParams hp, PackLayout L,
                                                      TableView tv, uint64_t* norm, uint32_t* rowmax, int use_img,
                                                      int32_t* hidx_w, uint32_t* cbound, int mforms) {
  extern __shared__ __align__(16) uint16_t img[];  // [dw] (use_img)
  __shared__ uint64_t red[4];
  __shared__ uint32_t smax[4];
  __shared__ unsigned long long s_sq[CMS_MAX_DEPTH];
  const int w = (int)hp.width;
  const int64_t dw = (int64_t)hp.depth * w;
  for (int64_t o = blockIdx.x; o < n; o += gridDim.x) {
    const int b = L.bits[o];
    const int32_t slot = tv.hidx[o];  // rows whose merged mass reaches 2^16 were promoted
    uint32_t* dst = slot >= 0 ? tv.hot + (int64_t)slot * dw : nullptr;
    uint16_t* dst16 = tv.row16(o);
    if (b == 0) {  // every rank's counters of this owner are zero (a compact row: the zero row)
      if (dst || tv.off[o] != 0)
        for (int64_t i = threadIdx.x; i < dw; i += 256) {
          if (dst) dst[i] = 0u;
          else dst16[i] = 0;
        }
      if (threadIdx.x < hp.depth) norm[o * hp.depth + threadIdx.x] = 0;
      if (threadIdx.x == 0) {
        rowmax[o] = 0;
        if (slot < 0) hidx_w[o] = kFormU16;
      }
      __syncthreads();
      continue;
    }
    const uint32_t nw = (uint32_t)(L.woff[o + 1] - L.woff[o]);
    const uint64_t mask = b >= 64 ? ~0ULL : ((1ULL << b) - 1);
    const uint64_t* src = words + L.woff[o];
    uint32_t vmax = 0;
    if (use_img && !dst) {  // narrow owner: merged counters < 2^16, so b <= 16
      const int F = 64 / b;
      for (uint32_t i0 = threadIdx.x; i0 < nw; i0 += 4 * 256) {  // four word loads in flight per lane
        uint64_t wv[4];
#pragma unroll
        for (int u = 0; u < 4; ++u) {
          const uint32_t i = i0 + u * 256;
          wv[u] = i < nw ? src[i] : 0ULL;
        }
#pragma unroll
        for (int u = 0; u < 4; ++u) {
          const uint32_t i = i0 + u * 256;
          if (i >= nw) break;
          uint32_t idx = i;
          for (int f = 0; f < F && idx < (uint32_t)dw; ++f, idx += nw)
            img[idx] = (uint16_t)((wv[u] >> (f * b)) & mask);
        }
      }
      if (threadIdx.x < hp.depth) s_sq[threadIdx.x] = 0;
      __syncthreads();
      // a narrow row's sum of squares is at most mass * max < 2^32: u32 partial
      // sums by v_dot2_u32_u16 are exact; one wave atomic per row, one barrier
      u16x2 pm = {0, 0};
      const int fm = mforms ? (b <= 4 ? 4 : b <= 8 ? 8 : 16) : 16;  // the stored form's counter bits
      for (int d = 0; d < hp.depth; ++d) {
        uint32_t sq = 0;
        const uint4* r4 = reinterpret_cast<const uint4*>(img + (int64_t)d * w);
        uint4* g4 = reinterpret_cast<uint4*>(dst16 + (int64_t)d * w);
        uint2* g2 = reinterpret_cast<uint2*>(reinterpret_cast<uint8_t*>(dst16) + (int64_t)d * w);
        uint32_t* g1 = reinterpret_cast<uint32_t*>(dst16) + (int64_t)d * (w >> 3);
        for (int j = threadIdx.x; j < (w >> 3); j += 256) {
          const uint4 v = r4[j];  // counters 8j .. 8j + 7 of sketch row d
          if (fm == 16) {
            g4[j] = v;
          } else if (fm == 8) {  // counter c at byte c
            auto b4 = [](uint32_t x, uint32_t y) {
              return (x & 0xFFu) | ((x >> 16) & 0xFFu) << 8 | (y & 0xFFu) << 16 | ((y >> 16) & 0xFFu) << 24;
            };
            g2[j] = make_uint2(b4(v.x, v.y), b4(v.z, v.w));
          } else {  // counter c in bits 4 (c & 7) of word c / 8
            const uint32_t x[4] = {v.x, v.y, v.z, v.w};
            uint32_t q = 0;
#pragma unroll
            for (int k = 0; k < 4; ++k) q |= ((x[k] & 0xFu) | ((x[k] >> 16) & 0xFu) << 4) << (8 * k);
            g1[j] = q;
          }
          const u16x2 a = __builtin_bit_cast(u16x2, v.x), bq = __builtin_bit_cast(u16x2, v.y),
                      c = __builtin_bit_cast(u16x2, v.z), e = __builtin_bit_cast(u16x2, v.w);
          sq = __builtin_amdgcn_udot2(a, a, sq, false);
          sq = __builtin_amdgcn_udot2(bq, bq, sq, false);
          sq = __builtin_amdgcn_udot2(c, c, sq, false);
          sq = __builtin_amdgcn_udot2(e, e, sq, false);
          pm = __builtin_elementwise_max(pm, __builtin_elementwise_max(__builtin_elementwise_max(a, bq),
                                                                       __builtin_elementwise_max(c, e)));
        }
        const uint32_t tot = wave_sum_u32(sq);
        if ((threadIdx.x & 63) == 0 && tot) atomicAdd(&s_sq[d], (unsigned long long)tot);
      }
      vmax = max((uint32_t)pm.x, (uint32_t)pm.y);
      __syncthreads();
      if (threadIdx.x < hp.depth) norm[o * hp.depth + threadIdx.x] = s_sq[threadIdx.x];
      if (threadIdx.x == 0 && fm < 16) hidx_w[o] = fm == 8 ? kFormU8 : kFormU4;  // (after the U16 default below)
    } else {
    for (int d = 0; d < hp.depth; ++d) {
      uint64_t sq = 0;
      for (int j = threadIdx.x; j < w; j += 256) {
        const uint32_t idx = (uint32_t)(d * w + j);
        const uint32_t f = idx / nw, wi = idx - f * nw;
        const uint32_t c = (uint32_t)((src[wi] >> (f * (uint32_t)b)) & mask);
        if (dst) dst[idx] = c;
        else dst16[idx] = (uint16_t)c;
        sq = sat_add(sq, (uint64_t)c * c);
        vmax = max(vmax, c);
      }
      const uint64_t tot = block_sum_u64_sat(sq, red);
      if (threadIdx.x == 0) norm[o * hp.depth + d] = tot;
    }
    }
#pragma unroll
    for (int s = 32; s > 0; s >>= 1) vmax = max(vmax, (uint32_t)__shfl_xor((int)vmax, s, 64));
    if ((threadIdx.x & 63) == 0) smax[threadIdx.x >> 6] = vmax;
    __syncthreads();
    if (threadIdx.x == 0) {
      const uint32_t rm = max(max(smax[0], smax[1]), max(smax[2], smax[3]));
      rowmax[o] = rm;
      // a narrow row holds u16 merged counters, or (mforms) the u8 / 4-bit form set above
      if (slot < 0 && !(mforms && use_img && b <= 8)) hidx_w[o] = kFormU16;
      if (slot < 0) cbound[o] = rm;
    }
    __syncthreads();
  }
}

int merge_packed(cms_handle* h, const AllReduceU64& allreduce) {
  const int64_t n = h->n, dw = h->dw;
  // 1. local row maxima (the build passes leave them current with the norms)
  int rc;
  if (!h->norms_valid && (rc = local_norms(h))) return rc;
  // 2. one all-reduce of (mass, max) per owner
  DevBuf& bnd = h->ws_mbnd;  // merge scratch stays allocated across steps
  CMS_HIP(bnd.ensure(sizeof(uint64_t) * 2 * n));
  const unsigned g = (unsigned)std::min<int64_t>((n + 255) / 256, 8192);
  hipLaunchKernelGGL(k_merge_bounds_in, dim3(g), dim3(256), 0, h->stream, h->d_row_mass, h->d_rowmax, n,
                     bnd.as<uint64_t>());
  CMS_HIP(hipGetLastError());
  {
    TimedScope ts(h, "merge_bounds");
    if ((rc = allreduce(bnd.as<uint64_t>(), 2 * n))) return rc;
  }
  hipLaunchKernelGGL(k_merge_bounds_out, dim3(g), dim3(256), 0, h->stream, bnd.as<uint64_t>(), n, h->d_row_mass,
                     h->d_flags);
  CMS_HIP(hipGetLastError());
  // 3. field widths and word offsets (identical on every rank: same sums)
  std::vector<uint64_t> sums(2 * n);
  CMS_HIP(hipMemcpyAsync(sums.data(), bnd.ptr, sizeof(uint64_t) * 2 * n, hipMemcpyDeviceToHost, h->stream));
  CMS_HIP(hipStreamSynchronize(h->stream));
  std::vector<uint8_t> bits(n);
  std::vector<int64_t> woff(n + 1);
  int64_t words = 0;
  for (int64_t o = 0; o < n; ++o) {
    const uint64_t bound = std::min(sums[o], sums[n + o]);
    const int b = bound == 0 ? 0 : 64 - __builtin_clzll(bound);
    bits[o] = (uint8_t)b;
    woff[o] = words;
    if (b) words += (dw + (64 / b) - 1) / (64 / b);
  }
  woff[n] = words;
  h->merge_words = words;
  DevBuf& d_bits = h->ws_mbits;
  DevBuf& d_woff = h->ws_mwoff;
  DevBuf& packed = h->ws_mpacked;
  CMS_HIP(d_bits.ensure(std::max<int64_t>(n, 1)));
  CMS_HIP(d_woff.ensure(sizeof(int64_t) * (n + 1)));
  CMS_HIP(packed.ensure(sizeof(uint64_t) * std::max<int64_t>(words, 1)));
  CMS_HIP(hipMemcpyAsync(d_bits.ptr, bits.data(), n, hipMemcpyHostToDevice, h->stream));
  CMS_HIP(hipMemcpyAsync(d_woff.ptr, woff.data(), sizeof(int64_t) * (n + 1), hipMemcpyHostToDevice, h->stream));
  CMS_HIP(hipStreamSynchronize(h->stream));  // bits / woff are host locals (the stream is idle here anyway)
  PackLayout L{d_bits.as<uint8_t>(), d_woff.as<int64_t>()};
  const unsigned go = (unsigned)std::min<int64_t>(n, 65536);
  // LDS image path for narrow owners when the image leaves room for 2 blocks per CU
  const size_t img = sizeof(uint16_t) * (size_t)dw;
  const int use_img = (h->p.width % 8 == 0 && img <= 80 * 1024) ? 1 : 0;
  static bool attr = [] {
    (void)hipFuncSetAttribute((const void*)k_merge_pack, hipFuncAttributeMaxDynamicSharedMemorySize, 80 * 1024);
    (void)hipFuncSetAttribute((const void*)k_merge_unpack, hipFuncAttributeMaxDynamicSharedMemorySize, 80 * 1024);
    return true;
  }();
  (void)attr;
  {
    TimedScope ts(h, "merge_pack");
    hipLaunchKernelGGL(k_merge_pack, dim3(go), dim3(256), use_img ? img : 0, h->stream, h->tview(), n, dw, L,
                       packed.as<uint64_t>(), use_img);
    CMS_HIP(hipGetLastError());
  }
  {
    TimedScope ts(h, "allreduce");
    if (words > 0 && (rc = allreduce(packed.as<uint64_t>(), words))) return rc;
  }
  // rows whose merged mass reaches 2^16 need u32 slots (row_mass is merged)
  if ((rc = promote_rows(h, h->d_row_mass, nullptr, false))) return rc;
  // compact rows: the table's bytes now live in the packed words, so the
  // narrow rows are laid out anew by their merged field widths
  const int mforms = h->compact && use_img ? 1 : 0;
  if (h->compact) {
    CMS_HIP(h->ws_layout.ensure(sizeof(uint32_t) * (size_t)(2 * n + n / 4096 + 16)));
    uint32_t* caps = h->ws_layout.as<uint32_t>();
    hipLaunchKernelGGL(k_merge_caps, dim3(g), dim3(256), 0, h->stream, d_bits.as<uint8_t>(), h->d_hidx, n, dw, mforms,
                       caps);
    CMS_HIP(hipGetLastError());
    if ((rc = row_layout(h, caps, caps + n))) return rc;
  }
  {
    TimedScope ts(h, "merge_unpack");
    hipLaunchKernelGGL(k_merge_unpack, dim3(go), dim3(256), use_img ? img : 0, h->stream, packed.as<uint64_t>(), n,
                       h->hp, L, h->tview(), h->d_norm, h->d_rowmax, use_img, h->d_hidx, h->d_cbound, mforms);
    CMS_HIP(hipGetLastError());
  }
  h->norms_valid = true;  // the unpack wrote the merged norms
  return CMS_OK;
}

}  // namespace cms
