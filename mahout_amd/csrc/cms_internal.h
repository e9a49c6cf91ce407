// cms_internal.h -- handle state and kernel launchers shared by the
// libmahout_cms.so translation units.  Not part of the ABI.
#pragma once
#include <hip/hip_runtime.h>
#include <rccl/rccl.h>

#include <functional>
#include <map>
#include <mutex>
#include <shared_mutex>
#include <string>
#include <vector>

#include "../../include/mahout_cms.h"
#include "cms_hash.h"

namespace cms {

// Device error flags (one u32 word per handle).
enum : uint32_t {
  kFlagBadRow = 1u << 0,    // owner row outside [0, n)
  kFlagBadValue = 1u << 1,  // increment not a non-negative integer (u32 counters)
  kFlagOverflow = 1u << 2,  // a row's total mass reached 2^32
};

// Growable device scratch buffer (grown outside any capture region).
struct DevBuf {
  void* ptr = nullptr;
  size_t bytes = 0;
  DevBuf() = default;
  DevBuf(const DevBuf&) = delete;
  DevBuf& operator=(const DevBuf&) = delete;
  DevBuf(DevBuf&& o) noexcept : ptr(o.ptr), bytes(o.bytes) {
    o.ptr = nullptr;
    o.bytes = 0;
  }
  DevBuf& operator=(DevBuf&& o) noexcept {
    if (this != &o) {
      release();
      ptr = o.ptr;
      bytes = o.bytes;
      o.ptr = nullptr;
      o.bytes = 0;
    }
    return *this;
  }
  ~DevBuf() { release(); }  // scoped scratch frees itself (hipFree waits for the device)
  hipError_t ensure(size_t need);
  template <class T>
  T* as() const { return reinterpret_cast<T*>(ptr); }
  void release();
};

struct TimingAcc {
  double total_ms = 0.0;
  int64_t launches = 0;
};

struct PendingEvent {
  std::string name;
  hipEvent_t start, stop;
};

// The sketch table.  A counter never exceeds its owner's total increment
// (row mass), so rows whose mass bound is below 2^16 are stored as u16 and
// only the others ("hot" rows: mass >= 2^16, or split over several build
// workgroups) get a u32 row in the slot table -- at config 2 that halves the
// bytes the row build writes.  Writers promote a row to a slot before its
// bound can reach 2^16 (promote_rows), so a u16 counter never overflows.
//
// ROW STORAGE: the narrow rows live in one arena (t16) at per-row offsets
// (off[row], u16 units, 128-B aligned; bits 0-2: kCap*, the widest form the
// row's place holds).  Offset 0 is a shared row of zeros that every row of an
// empty table points to.  A fresh build with forms lays the rows out
// compactly (row_layout: each row gets what its class's kernel can store -- a
// list row its entries, a byte-class row its u8 image, a mid row a whole
// slot); a writer widens a row in place when its place holds the new form,
// else moves it to a whole u16 slot at the arena's end (widen_rows), and the
// zero row always moves first -- so in-place adds only ever touch a row's
// own place.  Handles without forms keep every row in a
// whole u16 slot.
//
// Narrow FORMS: a fresh build stores a row whose counters are all below 2^8
// as u8 (dw bytes at its offset), one whose counters are all below 2^4 as
// packed nibbles (counter j in bits 4*(j&1) of byte j/2; dw/2 bytes), one
// whose counters are all below 2^2 as 2-bit counters (counter j in bits
// 2*(j&3) of byte j/4; dw/4 bytes), and one whose counters are all 0 or 1 as
// bits (counter j in bit j&7 of byte j/8; dw/8 bytes) -- at config 3 most of
// the 1M owners, so the build writes a fraction of the u16 bytes.  hidx[row]
// names the form (< 0) or the hot slot (>= 0).  cbound[row] (u32) bounds a
// form row's counters; a writer widens a form row (widen_rows: in place in a
// whole slot, else into a new one) before its bound could pass the form's
// capacity.  Forms exist only when dw % 32 == 0 (every row then starts
// 64-byte aligned, every nibble row holds whole 16-B words).
//
// LIST rows (kFormList): the smallest owners of a fresh build with unit
// increments are stored sparse -- row[0] = m, the owner's key count, then
// for each sketch row r the m buckets its keys hash to, row[1 + r m + t]
// (u16, unsorted, repeats allowed): counter (r, j) is the number of entries
// of row r equal to j.  2 + 2 d m bytes instead of a dense row (config 3: an
// owner of 100 keys takes 1 KB instead of the 10 KB of its 2-bit rows).  A
// list row takes no in-place adds (capacity 0: any write widens it to u16
// first); whole-row readers expand it per sketch row (list_* helpers).
constexpr uint64_t kNarrowLimit = 1ULL << 16;
constexpr int32_t kFormU16 = -1, kFormU8 = -2, kFormU4 = -3, kFormU2 = -4, kFormU1 = -5, kFormList = -6;
constexpr uint32_t form_cap(int32_t form) {
  return form == kFormList ? 0u : form == kFormU1 ? 1u : form == kFormU2 ? 3u : form == kFormU4 ? 15u
       : form == kFormU8 ? 255u : 65535u;
}

constexpr int64_t kRowAlign = 64;  // u16 units (128 B: an L2 line, so no two rows share one) per arena allocation unit
__host__ __device__ constexpr int64_t slot_units(int64_t dw) { return (dw + kRowAlign - 1) / kRowAlign * kRowAlign; }
// off[row] bits 0-2 (the offset is a multiple of kRowAlign): the widest form
// the row's place holds -- a row is written in place only in a form no wider.
// kCapNone: a list row's place, or the shared zero row (offset 0).
constexpr int64_t kCapMask = 7;
enum : int { kCapNone = 0, kCapU1 = 1, kCapU2 = 2, kCapU4 = 3, kCapU8 = 4, kCapU16 = 5 };
__host__ __device__ constexpr int form_class(int32_t f) {
  return f == kFormU1 ? kCapU1 : f == kFormU2 ? kCapU2 : f == kFormU4 ? kCapU4 : f == kFormU8 ? kCapU8
       : f == kFormU16 ? kCapU16 : kCapNone;
}
// u16 units a form's row takes in the arena (rounded to kRowAlign)
__host__ __device__ constexpr int64_t class_units(int c, int64_t dw) {
  return c == kCapU16 ? slot_units(dw)
       : ((c == kCapU8 ? dw / 2 : c == kCapU4 ? dw / 4 : c == kCapU2 ? dw / 8 : c == kCapU1 ? dw / 16 : 0) +
          kRowAlign - 1) / kRowAlign * kRowAlign;
}
// the widest form a place of `units` u16 holds
__host__ __device__ constexpr int class_of_units(int64_t units, int64_t dw) {
  return units >= class_units(kCapU16, dw) ? kCapU16 : units >= class_units(kCapU8, dw) ? kCapU8
       : units >= class_units(kCapU4, dw) ? kCapU4 : units >= class_units(kCapU2, dw) ? kCapU2
       : units >= class_units(kCapU1, dw) && dw >= 16 ? kCapU1 : kCapNone;
}

struct TableView {
  uint16_t* t16;        // the narrow-row arena (row r at off[r] & ~kCapMask)
  uint32_t* hot;        // [hot_cap][dw] u32 rows
  const int32_t* hidx;  // [n] slot of a hot row, or the narrow form (kForm*)
  int64_t dw;
  int32_t w;            // sketch row width (list rows)
  const int64_t* off;   // [n] arena offset of each narrow row (u16 units) | its place's form class (kCap*)
  __device__ __forceinline__ int64_t base(int64_t row) const { return off[row] & ~kCapMask; }
  __device__ __forceinline__ uint16_t* row16(int64_t row) const { return t16 + base(row); }
  // list row: key count and the entries of sketch row r
  __device__ __forceinline__ uint32_t list_m(int64_t row) const { return t16[base(row)]; }
  __device__ __forceinline__ const uint16_t* list_row(int64_t row, int64_t r, uint32_t m) const {
    return row16(row) + 1 + r * (int64_t)m;
  }
  __device__ __forceinline__ uint32_t get(int64_t row, int64_t j) const {
    const int32_t s = hidx[row];
    if (s >= 0) return hot[(int64_t)s * dw + j];
    if (s == kFormU16) return (uint32_t)t16[base(row) + j];
    if (s == kFormList) {  // O(m): point queries; whole-row readers expand instead
      const uint32_t m = list_m(row);
      const int64_t r = j / w;
      const uint32_t b = (uint32_t)(j - r * w);
      const uint16_t* e = list_row(row, r, m);
      uint32_t c = 0;
      for (uint32_t t = 0; t < m; ++t) c += e[t] == b;
      return c;
    }
    const uint8_t* p = reinterpret_cast<const uint8_t*>(row16(row));
    if (s == kFormU8) return p[j];
    if (s == kFormU2) return (uint32_t)(p[j >> 2] >> ((j & 3) << 1)) & 3u;
    if (s == kFormU1) return (uint32_t)(p[j >> 3] >> (j & 7)) & 1u;
    return (uint32_t)(p[j >> 1] >> ((j & 1) << 2)) & 15u;
  }
  // counters j..j+3 of a row (j % 4 == 0 and dw % 4 == 0: aligned vector loads)
  __device__ __forceinline__ uint4 get4(int64_t row, int64_t j) const {
    const int32_t s = hidx[row];
    if (s >= 0) return *reinterpret_cast<const uint4*>(hot + (int64_t)s * dw + j);
    if (s == kFormU16) {
      const ushort4 v = *reinterpret_cast<const ushort4*>(row16(row) + j);
      return make_uint4(v.x, v.y, v.z, v.w);
    }
    if (s == kFormList) {  // O(m), w % 4 == 0: the four counters share a sketch row
      const uint32_t m = list_m(row);
      const int64_t r = j / w;
      const uint32_t b = (uint32_t)(j - r * w);
      const uint16_t* e = list_row(row, r, m);
      uint4 c = make_uint4(0, 0, 0, 0);
      for (uint32_t t = 0; t < m; ++t) {
        const uint32_t q = (uint32_t)e[t] - b;
        c.x += q == 0u;
        c.y += q == 1u;
        c.z += q == 2u;
        c.w += q == 3u;
      }
      return c;
    }
    const uint8_t* p = reinterpret_cast<const uint8_t*>(row16(row));
    if (s == kFormU8) {
      const uint32_t v = *reinterpret_cast<const uint32_t*>(p + j);
      return make_uint4(v & 255u, (v >> 8) & 255u, (v >> 16) & 255u, v >> 24);
    }
    if (s == kFormU2) {
      const uint32_t v = p[j >> 2];
      return make_uint4(v & 3u, (v >> 2) & 3u, (v >> 4) & 3u, v >> 6);
    }
    if (s == kFormU1) {
      const uint32_t v = (uint32_t)p[j >> 3] >> (j & 4);
      return make_uint4(v & 1u, (v >> 1) & 1u, (v >> 2) & 1u, (v >> 3) & 1u);
    }
    const uint32_t v = *reinterpret_cast<const uint16_t*>(p + (j >> 1));
    return make_uint4(v & 15u, (v >> 4) & 15u, (v >> 8) & 15u, v >> 12);
  }
};

// Row-build tuning: pairs per build work item.
#ifndef CMS_SLICE
#define CMS_SLICE 8192  // keys per row-build workgroup of a split (hot) owner
#endif
constexpr int64_t kSlice = CMS_SLICE;
#ifndef CMS_BUILD_THREADS
#define CMS_BUILD_THREADS 256
#endif
constexpr int kBuildThreads = CMS_BUILD_THREADS;

}  // namespace cms

namespace cms {
// Scratch of one concurrent query (similarity / point query / estimate): its
// own stream and buffers, taken from the handle's pool for the call.
struct QueryCtx {
  hipStream_t stream = nullptr;
  DevBuf q, o, r, x, y, z;
};
}  // namespace cms

namespace cms {
// Tunables read ONCE, from the environment, when the handle is created
// (include/mahout_cms.h lists them); nothing in the library reads the
// environment after cms_create.
struct Tunables {
  int bit_keys = 64;       // CMS_BIT_KEYS: byte-class owners of <= this many keys try 1-bit rows first
  int crumb_keys = 256;    // CMS_CRUMB_KEYS: ... of <= this many keys 2-bit rows
  int list_keys = 256;     // CMS_LIST_KEYS: ... of <= this many keys (unit increments) list rows; 0: none
  // mid-class owners start at the form their key count suggests: a Zipf key
  // set repeats its most popular key about n / 40 times, so a counter passes
  // 15 past a few hundred keys and 255 past ten thousand -- the 4-bit (and u8)
  // attempts would only be thrown away (the escalation stays as the safety net)
  int mid_u4_keys = 768;    // CMS_MID_U4_KEYS: more keys start at u8 (list-row owners always try 4-bit)
  int mid_u8_keys = 12288;  // CMS_MID_U8_KEYS: more keys start at u16
  int nib_persist = 0;      // CMS_NIB_PERSIST=1: k_build_nibbles as persistent waves (else one owner per wave)
  int plan_side = 1;        // CMS_PLAN_SIDE=0: the build plan after the whole partition on the handle's stream
  int build_streams = 3;    // CMS_BUILD_STREAMS=2: the mid class after the byte class on one side stream
  int mid_image = 0;        // CMS_MID_IMAGE=1: mid owners through the one-pass u16 image (k_build_image; slower on MI355X)
  int po_dense_x4 = 4;      // CMS_PO_DENSE_X4: group kernel's dense dots when 4 w <= this x nnz(u1)
  int po_bound_part2 = 1;   // CMS_PO_BOUND_PART2=0: the widest narrow part through the group kernel, unbounded
  int po_bound_rows = 1;    // CMS_PO_BOUND_ROWS: sketch rows of the wide owners' upper bound (1 or 2)
  int po_no_prune = 0;      // CMS_PO_NO_PRUNE=1: every (query, wide owner) pair through k_po_pairs (no row-0 bound)
  int po_no_bigq = 0;       // CMS_PO_NO_BIGQ=1: per-owner all-pairs without k_po_bigq (every query in the group kernel)
  int mid_u8_image = 0;     // CMS_MID_U8_IMAGE=1: mid owners starting at u8 count all sketch rows in one [d][w] u8 image
  int nib_rows_once = 0;    // CMS_NIB_ROWS_ONCE=1: a byte-class wave hashes its first key slot's d rows up front (d = 4 or 5)
  int mid_threads = 256;    // CMS_MID_THREADS=128: k_build_mid owners on 2-wave workgroups (twice as many in flight)
  int split_keys = 0;       // CMS_SPLIT_KEYS: rows with more keys get a u32 slot and k_build_slices (0: 8192, 16384 at w >= 8192)
  int mid_waves = 0;        // CMS_MID_WAVES=<k>: mid owners one wave each (k_build_mid_waves), k persistent 4-wave workgroups per CU; 0: k_build_mid
  int slice_reduce = 0;     // CMS_SLICE_REDUCE=1: split owners' slices leave u16 images summed by k_slice_reduce (no slot atomics)
  int early_slices = 0;     // CMS_EARLY_SLICES=1: the hot-routed split owners are built beside pass 2 of the partition
  bool forms = true;       // CMS_NO_FORMS=1: every narrow row stays u16 (no 1/2/4/8-bit forms)
  bool no_compact = false; // CMS_NO_COMPACT=1: every narrow row keeps a whole u16 slot (no compact layout)
  bool no_vmm = false;     // CMS_NO_VMM=1: the compact arena as one hipMalloc grown by copying (no virtual range)
  bool hot_routing = true; // CMS_NO_HOT_ROUTING=1: the partition sends every owner through both passes
  bool fp4 = true;         // CMS_NO_FP4=1: no e2m1 operand image (every single-limb pair on int8)
  bool mls = true;         // CMS_NO_MLS=1: multi-limb slabs on the 128-tile kernel instead of k_cosine_mls
};
}  // namespace cms

struct cms_handle {
  cms_params p{};
  cms::Tunables tune;
  int device = 0;
  int num_cus = 256;  // compute units of the device (persistent grids)
  hipStream_t stream = nullptr;
  // side stream of the row build: the hot owners' slices run beside the row
  // kernels (ordered by ev_fork / ev_join on the handle's stream)
  hipStream_t side_stream = nullptr;
  hipEvent_t ev_fork = nullptr, ev_join = nullptr;    // slices experiment (CMS_SLICES_SIDE)
  hipEvent_t ev_fork2 = nullptr, ev_join2 = nullptr;  // byte / mid class kernels beside the slot rows
  hipStream_t side_stream2 = nullptr;                 // the mid class beside the byte class (Tunables::build_streams 3)
  hipEvent_t ev_join3 = nullptr;
  // the owner spans of a partition are ready (recorded before its last
  // scatter): the build plan may start on the side stream meanwhile
  hipEvent_t ev_spans = nullptr, ev_plan = nullptr;
  // early slices (Tunables::early_slices): pass 1 of the partition has placed
  // the hot-routed owners' keys (ev_p1); their build runs on side_stream3,
  // ev_e1 marks their rows claimed (hidx, early flags), ev_early its end
  hipStream_t side_stream3 = nullptr;
  hipEvent_t ev_p1 = nullptr, ev_e1 = nullptr, ev_early = nullptr;
  bool p1_event = false;
  const unsigned long long* p1_slotkey = nullptr;  // hot slot t -> owner row + 1 (0: free)
  const uint32_t* p1_bs1 = nullptr;                // pass-1 bin starts: hot slot t spans [bs1[P1 + t], bs1[P1 + t + 1])
  int p1_P1 = 0, p1_nslots = 0;
  bool spans_event = false, plan_side_request = false;
  bool plan_side_active = false;  // h->stream and h->side_stream are swapped (the build plan's section)
  // Writers (ingest, finalize, reset, top-k passes, ...) hold mu exclusively;
  // the point queries after cms_finalize hold it shared and run concurrently,
  // each on a QueryCtx of its own (the table and norms are read-only then).
  std::shared_mutex mu;
  std::mutex pool_mu;
  std::vector<cms::QueryCtx*> qpool;

  int64_t a[CMS_MAX_DEPTH] = {};  // HashFunctionBuilder parameters as drawn
  int64_t b[CMS_MAX_DEPTH] = {};
  cms::HashParams hp{};

  int64_t n = 0;       // rows
  int64_t dw = 0;      // d*w counters per row
  uint16_t* d_t16 = nullptr;        // arena of the narrow rows (TableView; [0, slot_units(dw)) the zero row)
  int64_t t16_cap = 0, t16_used = 0;  // arena capacity and end of the allocated part (u16 units)
  int64_t* d_off = nullptr;         // [n] arena offset of each narrow row | its place's form class (kCap*)
  // compact handles: the arena is a reserved virtual range whose physical
  // memory is mapped (and unmapped) in chunks at its end -- growing never
  // copies and the base never moves (arena_reserve); without the virtual
  // memory API it is one hipMalloc grown by copying
  struct ArenaChunk {
    hipMemGenericAllocationHandle_t mem;
    size_t bytes;
  };
  void* arena_va = nullptr;
  size_t arena_va_bytes = 0, arena_mapped = 0, arena_gran = 0;
  int arena_small_layouts = 0;  // consecutive layouts that wanted under a quarter of the arena (arena_reserve)
  std::vector<ArenaChunk> arena_chunks;
  bool compact = false;             // forms_ok: fresh builds lay the rows out compactly (row_layout)
  bool f64 = false;                 // CMS_COUNTER_F64: fp64 counters in d_t64 (cms_f64.hip), no u16/u32 table
  double* d_t64 = nullptr;          // [n][d][w] fp64 counters
  int32_t* d_hidx = nullptr;        // [n] hot slot, or the narrow form (kFormU16 / kFormU8 / kFormU4 / kFormU2 / kFormU1)
  uint32_t* d_cbound = nullptr;     // [n] bound of a form row's counters (maintained for form rows only)
  bool forms_ok = false;            // dw % 32 == 0: fresh builds may store u8 / nibble forms
  cms::DevBuf hot_tab;              // [hot_cap][d][w] u32 counters of the hot rows
  cms::DevBuf ws_bound, ws_force, ws_plist;  // promotion scratch: u64 [n], u8 [n], i32 [n] + count
  cms::DevBuf ws_blist;                      // row build: slot-row and mid-class row lists + counts
  cms::DevBuf ws_layout;                     // row layout: capacities / scan (u32 [2n + ...]); widen: movers
  cms::DevBuf ws_early;                      // early slices: spans i64 [2n], flags u8 [n], HotInfo / slice map
  int64_t hot_cap = 0, hot_used = 0;
  cms::TableView tview() const {
    return cms::TableView{d_t16, hot_tab.as<uint32_t>(), d_hidx, dw, p.width, d_off};
  }
  uint64_t* d_row_mass = nullptr;   // [n] total increment mass per row
  uint64_t* d_norm = nullptr;       // [n][d] exact sum of squares (saturating)
  double* d_norm_sqrt = nullptr;    // [n][d] Math.sqrt((double) norm)
  uint32_t* d_rowmax = nullptr;     // [n] largest counter of the owner (valid with the norms)
  uint32_t* d_flags = nullptr;      // error flags word + counters
  uint32_t* h_pin = nullptr;        // pinned host words: flag read-back without a staged copy
  bool stale_possible = true;       // an incremental ingest may have raised flags[2] since the last check
  bool inexact_zero = true;         // flags[1] (inexact-norm count) is known to be 0 on the device
  int64_t* d_owner_ids = nullptr;   // [n] sorted IDs (null => identity)
  std::vector<int64_t> h_owner_ids;

  bool empty = true;         // every counter is zero (next large batch builds rows)
  bool norms_valid = false;  // d_norm matches d_table
  bool finalized = false;
  // all-pairs (MFMA) operands, derived lazily from the finalized table
  bool mfma_ready = false;
  uint32_t n_hot_limb = 0;      // owners with counters >= 128 (multi-limb)
  uint32_t n_inexact_rows = 0;  // owners with a norm >= 2^53
  std::vector<uint8_t> tile_limbs;   // per permuted 128-row tile: max limb count
  // virtual limb rows of the multi-limb owners, two groups by limb count:
  // [0] positions [0, n4) with 3-4 limbs (4 slots), [1] [n4, n_multi) with 2 (2 slots)
  struct VLGroup {
    int64_t o0 = 0, o1 = 0;  // permuted positions
    int32_t ls = 0;          // limb slots
    int64_t rows = 0;        // virtual rows in buf
    cms::DevBuf buf;
    cms::DevBuf bbuf;        // the same rows K-blocked (k_cosine_mls operands), valid when bready
    bool bready = false;
  } vl[2];
  int64_t n_f4 = 0;     // single-limb owners whose counters are all <= 4 (fp4-exact)
  int64_t f4_pos0 = 0;  // first permuted position of the fp4 image (ws_f4); n if none
  int32_t sym_sw = 128;      // K slice width (bytes) of the K-blocked images = the symmetric waves' stage depth
  bool i8blk_ready = false;  // ws_i8blk holds the K-blocked int8 image of positions [n_multi, n)
  bool vl_ok = false;           // every multi-limb owner fits 4 limbs (else the legacy 128x128 path)
  int64_t topk_redo = 0;        // top-k rows the sampled threshold missed (radix-select redo)
  std::vector<int64_t> h_perm, h_inv;  // permuted position <-> owner row
  // incremental all-pairs top-k (cms_top_k_refresh): exact lists of depth
  // rf_depth >= k per owner row (candidate rows, scores, valid prefix length,
  // "holds every candidate" flag) for the table as it was, minus the owners
  // marked touched by COO ingests since (rf_touch).
  bool rf_valid = false;
  int32_t rf_k = 0, rf_depth = 0;
  cms::DevBuf rf_ids, rf_sc, rf_cnt, rf_full, rf_touch, rf_new, rf_redo, rf_perm;
  // set by cms_top_k_refresh around its job: cosine_prepare orders touched
  // single-limb owners first within their class, top_k_all's symmetric waves
  // keep only block pairs holding a touched owner
  bool rf_restrict = false;
  int64_t rf_t8 = 0, rf_t4 = 0, rf_s8 = 0;  // touched int8 / fp4 single-limb owners; int8-class size
  int64_t rf_td = 0, rf_tm = 0, rf_nd = 0;  // touched 3+-limb / 2-limb owners (first in their group); 3+-limb owners
  // column ranges (permuted positions [lo, hi)) a slab is restricted to; empty: every column
  std::vector<std::pair<int64_t, int64_t>> slab_cols;
  int64_t rf_stat_touched = 0, rf_stat_redo = 0, rf_stat_full = 0;
  // owners of the last all-pairs job per operand class (multi-limb, int8,
  // fp4) and, for an incremental refresh, how many of each were touched
  int64_t rf_stat_class[6] = {0, 0, 0, 0, 0, 0};
  int64_t pairs_ingested = 0;
  int32_t exact_norms = 1;

  // scratch
  cms::DevBuf ws_in_row, ws_in_key, ws_in_val;   // host-ingest staging
  cms::DevBuf ws_p1_row, ws_p1_key, ws_p1_val;   // pass-1 partition output
  cms::DevBuf ws_mbnd, ws_mbits, ws_mwoff, ws_mpacked;  // packed multi-rank merge (bounds, layout, words)
  cms::DevBuf ws_csr_key, ws_csr_val, ws_csr_off, ws_csr_hi;
  cms::DevBuf ws_hotpart;  // hot-owner routing of the partition: slot keys [1024] u64, sample counts [n] u32
  cms::DevBuf ws_hist, ws_small, ws_partials, ws_hot;
  cms::DevBuf ws_slicepart;  // row build: u16 [mapped slices][d*w] slice images of split owners (k_slice_reduce)
  cms::DevBuf ws_query, ws_query2, ws_out, ws_srow, ws_f4, ws_i8blk;
  cms::DevBuf ws_limb0, ws_limbmeta, ws_limbhot, ws_hotlist, ws_tiles, ws_slab, ws_topq, ws_nsq, ws_cand;

  // communicator: RCCL (cms_comm_init) or a caller transport (cms_comm_init_transport)
  ncclComm_t comm = nullptr;
  int32_t rank = 0, world = 1;
  cms_allreduce_fn x_allreduce = nullptr;  // caller transport (ext_comm)
  cms_allgather_fn x_allgather = nullptr;
  void* x_user = nullptr;
  bool ext_comm = false;
  int64_t coll_calls = 0;  // collectives issued through the communicator (cms_stats.collective_calls)
  // the multi-rank data path: a communicator is attached and either there are
  // several ranks or the handle asked for the collective path at one rank
  bool multi() const {
    return (world > 1 || (p.flags & CMS_FLAG_COLLECTIVE_SINGLE_RANK)) && (comm != nullptr || ext_comm);
  }
  // After the first multi-rank finalize every rank holds the summed table; later
  // COO batches are logged here and only the logs are exchanged at the next
  // finalize (each rank applies the other ranks' batches).
  bool merged = false;
  bool ext_merged = false;  // merged through cms_finalize_with (no delta log: refuse later ingests)
  int64_t merge_words = 0;  // u64 words the last packed merge moved
  int64_t dlog_n = 0, dlog_cap = 0;
  cms::DevBuf dlog_row, dlog_key, dlog_val, dlog_cnt, dlog_all;

  // per-owner shapes (CosineCM with its CountMinSketchConfig, cms_create_per_owner):
  // the DataModel stays resident as CSR and each owner carries its own (d, w);
  // userSimilarity(u1, u2) hashes u1's preferences at u2's shape on the fly
  bool per_owner = false;
  bool po_loaded = false, po_configured = false;
  int64_t po_npairs = 0;
  int32_t po_max_w = 0, po_max_d = 0;
  std::vector<int64_t> h_po_off;                 // [n+1] CSR offsets (DataModel)
  std::vector<double> h_po_delta, h_po_eps;      // CountMinSketchConfig.getDelta/getEpsilon
  std::vector<int32_t> h_po_w, h_po_d;           // AbstractCountMinSketch(delta, epsilon) shape; 0 = CMException
  cms::DevBuf po_off, po_kp, po_inc;             // CSR offsets, keys mod p, u32 increments
  cms::DevBuf po_v64;                            // fp64 counters: (double) preferences in CSR order
  cms::DevBuf po_shape;                          // PoShape [n]
  cms::DevBuf po_sk, po_norm, po_nsq;            // own sketches [sum d*w] u32; norms [sum d] u64 / f64 sqrt
  cms::DevBuf po_scratch;                        // per-block bucket rows for widths beyond LDS
  // candidates grouped by shape class for the all-pairs slabs (po_allpairs_slab):
  // PoGroup [po_ngroups] (LDS-sized groups of one (w, d) class, then the wide
  // owners one per group), po_cmem the owner rows in group order
  cms::DevBuf po_groups, po_cmem, po_redo;
  int64_t po_ngroups = 0, po_nnarrow = 0, po_wide0 = 0;  // groups, narrow groups, first wide member in po_cmem
  int32_t po_gmax_lds = 0;                       // LDS of a group workgroup (bytes)
  int64_t po_nnarrow_part[3] = {};               // narrow groups of width <= 512, <= 1024, <= 2048 (in that order)
  int32_t po_hist_w = 1;                         // widest narrow class (the waves' LDS bucket rows)
  // the narrow classes whole (one PoGroup each, po_classes) with their
  // members' sketches transposed, [class][d * w][members] (po_skT): the
  // big-query kernel's coalesced operand
  cms::DevBuf po_classes, po_skT;
  int64_t po_nclasses = 0;
  int32_t po_class_maxdw = 0;
  // the wide owners by width (po_wrows) and every preference's row-0 residue
  // (a_0 k + b_0) mod p (po_s0): k_po_wide_bound's operands; the top-k
  // threshold scratch and the surviving (query, wide owner) pairs
  cms::DevBuf po_wrows, po_s0, ws_pothr, ws_posurv;
  int64_t po_nbound = 0, po_nbound_narrow = 0;   // k_po_wide_bound's candidates (po_wrows), narrow ones among them
  int32_t po_s0_rows = 1;                        // sketch rows in po_s0 (the bound's rows)
  int64_t po_wide_pairs = 0, po_wide_exact = 0;  // (query, wide owner) pairs bounded / computed exactly

  // instrumentation
  int timing = 0;  // 0 off, 1 the roofline kernels' scopes only, 2 every scope (phase breakdown)
  std::map<std::string, cms::TimingAcc> timing_acc;
  std::vector<cms::PendingEvent> pending;
  std::vector<hipEvent_t> event_pool;  // recycled timing events (no create/destroy per scope)
  hipEvent_t order_ev = nullptr;       // cms_wait_stream / cms_release_to_stream (timing disabled)
};

namespace cms {

// error plumbing (cms_api.hip)
int set_error(int code, const char* fmt, ...);
int hip_fail(hipError_t e, const char* what);
#define CMS_HIP(call)                                  \
  do {                                                 \
    hipError_t _e = (call);                            \
    if (_e != hipSuccess) return cms::hip_fail(_e, #call); \
  } while (0)

// timing scopes on the handle stream
struct TimedScope {
  cms_handle* h;
  hipEvent_t start = nullptr;
  const char* name;
  TimedScope(cms_handle* hh, const char* nm, bool on = true);
  ~TimedScope();
};

// ---- launchers (cms_ingest.hip) ----
// COO -> table. rows are dense row indices (validated on device).
int ingest_coo_device(cms_handle* h, const int64_t* d_row, const int64_t* d_key, const float* d_val, int64_t n);
// CSR (offsets int64 [n+1]) -> table.
int ingest_csr_device(cms_handle* h, const int64_t* d_off, const int64_t* d_key, const float* d_val, int64_t npairs);
// owner spans -> table: row r's keys are d_key[d_lo[r], d_hi[r]) (the spans
// need not be in row order; a CSR is d_lo = off, d_hi = off + 1).
// d_tok: the partition's key tokens (cms_device.h Keys), d_key then the
// batch's keys they escape into; null for a caller CSR (keys in d_key).
int ingest_spans_device(cms_handle* h, const int64_t* d_lo, const int64_t* d_hi, const int64_t* d_key,
                        const uint32_t* d_tok, const float* d_val, int64_t npairs);
// owner IDs -> rows by binary search over h->d_owner_ids.
int map_owner_ids(cms_handle* h, const int64_t* d_ids, int64_t n, int64_t* d_rows);
int compute_norms(cms_handle* h);
// norms + row maxima of the local table (k_norms)
int local_norms(cms_handle* h);
// Every row whose bound[r] (a u64 upper bound of its counters after the
// coming write, in counter units; or any row with force[r]) reaches 2^16
// gets a hot slot; copy_old copies its narrow counters into the slot (else the
// slot is zeroed).  bound may be null when only force is used.
// max_new >= 0: a proven bound on the rows this call can promote (no host
// round trip: that many slots are reserved and claimed on the device).
int promote_rows(cms_handle* h, const uint64_t* d_bound, const uint8_t* d_force, bool copy_old, int64_t max_new = -1,
                 uint64_t whole_bound = 0);
// count consecutive hot slots for the caller's rows (host bookkeeping; the
// table grows first if needed): [*base, *base + count)
int reserve_hot_slots(cms_handle* h, int64_t count, int64_t* base);
// rows holding a u32 slot (synchronises the stream)
int count_hot_rows(cms_handle* h, int64_t* out);
// rows per storage form: [0] hot, [1] u16, [2] u8, [3] nibble (synchronises)
int count_forms(cms_handle* h, int64_t out[9]);  // hot, u16, u8, 4-bit, 2-bit, 1-bit, list rows, list bytes, zero rows
// Form rows that a coming write could push past their capacity become u16 in
// place: with d_bound (a u64 upper bound of each row's mass after the write)
// and old_mass, a touched form row (bound > old mass) is widened when
// cbound + (bound - old_mass) exceeds its form's capacity, and its cbound grows
// by the batch's mass; all_touched widens every touched form row (with d_lo /
// d_hi, the build's owner spans, a row with keys counts as touched even when
// its increments add no mass); d_bound null widens every form row.
int widen_rows(cms_handle* h, const uint64_t* d_bound, const uint64_t* old_mass, bool all_touched,
               const int64_t* d_lo = nullptr, const int64_t* d_hi = nullptr);
// per-row counter bounds after a CSR batch (mass in counter units + old_mass)
// and the rows split over more than `slice` keys (cms_build.hip)
int row_bounds(cms_handle* h, const int64_t* d_lo, const int64_t* d_hi, const float* d_val, const uint64_t* old_mass,
               int64_t slice, uint64_t* bound, uint8_t* force);
// counters of rows [r0, r0 + rc) as u32 into a device buffer (stream-ordered)
int read_counters_device(cms_handle* h, int64_t r0, int64_t rc, uint32_t* d_out);
// all rows narrow and zero-able again (empty table)
int reset_table_layout(cms_handle* h);
// every row back to zeros: compact handles point every row at the arena's
// zero row (nothing is cleared), the others zero their full slots
int reset_rows_zero(cms_handle* h);
// the arena holds at least need u16 units; keep: its allocated part
// [0, t16_used) is copied over (else the table is dead: only the zero row
// is restored)
int arena_reserve(cms_handle* h, int64_t need, bool keep);
// the arena and off[] of a new handle (cms_create)
int init_row_offsets(cms_handle* h);
// unmaps and frees the arena (cms_destroy)
void arena_release(cms_handle* h);
// Compact layout of a fresh build (cms_build.hip): caps[r] (128-B units) ->
// off[] after the zero row; returns the arena units in use.  Synchronises
// h->stream (the plan's stream) to size the arena.
int row_layout(cms_handle* h, const uint32_t* d_caps, uint32_t* d_scratch);
// ---- collectives over the handle's communicator (cms_api.hip) ----
// in-place u64 sum over all ranks (RCCL all-reduce or the caller transport)
int coll_allreduce_u64(cms_handle* h, uint64_t* d_buf, int64_t count);
// recv = the `bytes` of every rank's send, concatenated in rank order
int coll_allgather(cms_handle* h, const void* d_send, void* d_recv, int64_t bytes);
// ---- cms_merge.hip ----
// in-place u64 sum over all ranks of count words of a device buffer
using AllReduceU64 = std::function<int(uint64_t*, int64_t)>;
// merge the per-rank tables (and row masses) through the counter-width-adaptive
// packed all-reduce; leaves the merged table, norms and row maxima
int merge_packed(cms_handle* h, const AllReduceU64& allreduce);
// flags rows outside [0,n) and increments the counter type cannot hold.
int validate_batch(cms_handle* h, const int64_t* d_rows, const float* d_val, int64_t n);
// offsets[0] == 0 and non-decreasing (flags kFlagBadRow otherwise)
int check_offsets_device(cms_handle* h, const int64_t* d_off);
int hash_keys_device(cms_handle* h, const int64_t* d_keys, int64_t n, int32_t* d_out);
int scan_exclusive_u32(cms_handle* h, const uint32_t* in, uint32_t* out, int64_t L, uint32_t* bsum);
// List rows (kFormList) may be stored: forms, the tunable, and a d x w u16
// image that fits the merge's LDS (k_merge_pack expands them there).
inline bool lists_allowed(const cms_handle* h) {
  return h->forms_ok && h->tune.list_keys > 0 && h->p.width % 8 == 0 && (size_t)h->dw * 2 <= 80 * 1024;
}
// ---- cms_partition.hip ----
// COO -> CSR grouped by row; outputs live in handle scratch.
// Keys come out as u32 tokens (cms_device.h make_token / Keys) that escape
// into d_key.
int partition_to_csr(cms_handle* h, const int64_t* d_row, const int64_t* d_key, const float* d_val, int64_t npairs,
                     int64_t** out_off, uint32_t** out_tok, float** out_val,
                     int32_t* out_rows = nullptr);
// COO -> owner spans with the hottest owners routed straight to their final
// place by pass 1 (only the other pairs take pass 2).  Returns kNoSpans when
// the shape does not allow it (the caller then uses partition_to_csr).
constexpr int kNoSpans = 1;
int partition_to_spans(cms_handle* h, const int64_t* d_row, const int64_t* d_key, const float* d_val, int64_t npairs,
                       int64_t** out_lo, int64_t** out_hi, uint32_t** out_tok, float** out_val);

// ---- launchers (cms_query.hip) ----
// s: the stream to launch on (null = the handle's stream; a query context's
// stream is never timed)
int pair_cosines(cms_handle* h, int64_t q_row, const int64_t* d_rows, int64_t m, double* d_out,
                 hipStream_t s = nullptr);
int point_queries(cms_handle* h, int64_t row, const int64_t* d_keys, int64_t m, double* d_out, hipStream_t s = nullptr);
int pair_cosines_many(cms_handle* h, const int64_t* d_qrows, const int64_t* d_rows, int64_t m, double* d_out,
                      hipStream_t s);
int estimate_preferences_batch(cms_handle* h, const int64_t* d_user_rows, const int64_t* d_nb_off,
                               const int64_t* d_nb_rows, const double* d_sims, const int32_t* d_item_user,
                               const int64_t* d_items, int64_t q, int use_capper, float lo, float hi, float* d_out,
                               hipStream_t s);
int estimate_preferences(cms_handle* h, int64_t user_row, const int64_t* d_nb_rows, const double* d_sims, int64_t m,
                         const int64_t* d_items, int64_t q, int use_capper, float lo, float hi, float* d_out,
                         hipStream_t s = nullptr);
int top_k_rows(cms_handle* h, int64_t row_begin, int64_t row_count, int32_t k, int64_t* d_ids, double* d_scores,
               int32_t* d_counts);
// exact top-k (slab path) of the owners at PERMUTED positions pos, written at out_pos
int slab_top_k_positions(cms_handle* h, const std::vector<int64_t>& pos, const std::vector<int64_t>& out_pos,
                         int32_t k, int64_t* d_ids, double* d_scores, int32_t* d_counts);
// candidate lists of the streaming all-pairs top-k
constexpr int kCandCap = 1024;  // entries per row
constexpr int kCandCapSym = 2048;  // entries per row with the 768-row symmetric blocks (up to 1536 offers per wave)
struct CandBufs {
  uint32_t* ccnt;  // [n]
  uint32_t* cidx;  // [n][cap]
  double* cval;    // [n][cap]
  double* thr;     // [n]
  uint32_t* ovf;   // [n]
  uint32_t* list;  // [n]
  uint32_t* list_n;
  int32_t cap;
};
int cand_compact(cms_handle* h, const CandBufs& cb, int64_t p0, int64_t np, uint32_t limit, int32_t k);
int cand_emit(cms_handle* h, const CandBufs& cb, int64_t p0, int64_t np, int32_t k, int64_t* d_ids, double* d_scores,
              int32_t* d_counts);
// slab of positions [m0, m0+qc) against everyone: exact top-k of those rows,
// and their similarities offered to the lists of columns [c0, c1)
int multi_rows_slab_offer(cms_handle* h, const CandBufs& cb, int64_t m0, int64_t qc, int64_t c0, int64_t c1, int32_t k,
                          int64_t* d_ids, double* d_scores, int32_t* d_counts,
                          const std::vector<std::pair<int64_t, int64_t>>* cols = nullptr);
int top_k_all(cms_handle* h, int32_t k, int64_t* d_ids, double* d_scores, int32_t* d_counts, int32_t shard = 0,
              int32_t nshards = 1);
// merge nparts partial top-k lists ([nparts][n][k] ids by owner ID, scores; [nparts][n] counts)
int top_k_merge(cms_handle* h, int32_t k, int32_t nparts, const int64_t* d_ids, const double* d_scores,
                const int32_t* d_counts, int64_t* d_out_ids, double* d_out_scores, int32_t* d_out_counts);
// ---- incremental refresh (cms_topk.hip) ----
// mark the owner rows of a COO batch touched (rf_touch) when refresh lists are live
int refresh_mark(cms_handle* h, const int64_t* d_row, int64_t npairs);
// fold a refresh job's lists (rows, depth rf_depth) into the kept lists: touched
// rows take the new list, untouched rows the first rf_depth of new + kept
// (kept entries of touched candidates dropped), valid up to the kept boundary;
// rows left with fewer than k valid entries are listed in redo ([0] = count)
int refresh_fold(cms_handle* h, const int64_t* d_new_ids, const double* d_new_sc, const int32_t* d_new_cnt,
                 int32_t k, uint32_t* d_redo);
// first k of the kept lists -> outputs (owner IDs through d_owner_ids)
int refresh_emit(cms_handle* h, int32_t k, int64_t* d_ids, double* d_scores, int32_t* d_counts);
// kept lists' "holds every candidate" flags from their counts (after a full job)
int refresh_set_full(cms_handle* h);
// the same for the rows of d_list ([0] = count, rows from [1])
int refresh_set_full_list(cms_handle* h, const uint32_t* d_list, int64_t m);
// the whole-table job of cms_top_k_all on device outputs (multi-rank: shard,
// all-gather, merge)
int top_k_all_job(cms_handle* h, int32_t k, int64_t* d_ids, double* d_scores, int32_t* d_counts);
// ---- cms_profiles.hip (per-owner shapes) ----
struct PoShape {
  int64_t soff;      // first counter of the owner's own sketch
  int64_t roff;      // first (owner, row) norm slot
  uint64_t barrett;  // floor((2^64-1)/w)
  int32_t w, d;      // 0 when the owner's (delta, epsilon) raise CMException
};
// Candidates of one shape class (w, d) whose own sketches share a workgroup's
// LDS (cnt <= kPoGroupMax), or one wide owner (wide = 1: sketch read from HBM)
struct PoGroup {
  uint64_t barrett;  // floor((2^64-1)/w)
  int32_t w, d;
  int32_t m0, cnt;   // members po_cmem[m0, m0 + cnt)
  int32_t wide, pad;
};
int po_load_csr(cms_handle* h, const int64_t* d_off, const int64_t* d_key, const float* d_val, int64_t npairs,
                const int64_t* h_off);
int po_finalize(cms_handle* h);
// similarities of (qrows[i / m], crows[i % m]) into out[i] (crows null: identity)
int po_pair_cosines(cms_handle* h, const int64_t* d_qrows, int64_t nq, const int64_t* d_crows, int64_t m, double* d_out,
                    hipStream_t s = nullptr);
int po_point_queries(cms_handle* h, int64_t row, const int64_t* d_keys, int64_t m, double* d_out,
                     hipStream_t s = nullptr);
int po_estimate_preferences(cms_handle* h, int64_t user_row, const int64_t* d_nb_rows, const double* d_sims, int64_t m,
                            const int64_t* d_items, int64_t q, int use_capper, float lo, float hi, float* d_out,
                            hipStream_t s = nullptr);
int po_top_k_rows(cms_handle* h, int64_t row_begin, int64_t row_count, int32_t k, int64_t* d_ids, double* d_scores,
                  int32_t* d_counts);
// shape check of every owner in rows (all owners when rows is null)
int po_require_shapes(cms_handle* h, const int64_t* rows, int64_t m);
// the per-owner pair kernel needs the handle's global scratch (fp64, or widths past LDS)
bool po_shared_scratch(cms_handle* h);
// ---- cms_topk.hip (shared by both modes) ----
struct TopQuery {
  int64_t slab_row;  // row of the slab holding this query's similarities
  int64_t self_col;  // slab column of the query itself (excluded)
  int64_t out_pos;   // output slot
};
int launch_top_k(cms_handle* h, const double* slab, const std::vector<TopQuery>& qs, int32_t k, const int64_t* d_perm,
                 int64_t* d_ids, double* d_scores, int32_t* d_counts);
int64_t slab_rows_for(int64_t n);
// slab rows of one multi-limb chunk of the all-pairs job (memory permitting, up to 4096 at 1M)
int64_t multi_slab_rows(cms_handle* h, int64_t n);
// ---- cms_f64.hip (CMS_COUNTER_F64) ----
int f64_ingest_csr(cms_handle* h, const int64_t* d_off, const int64_t* d_key, const float* d_val);
int f64_ingest_coo_host(cms_handle* h, const int64_t* owner, const int64_t* key, const float* val, int64_t np);
// per-owner shapes on fp64 counters
int po_f64_load(cms_handle* h, const int64_t* d_key, const float* d_val, int64_t npairs);
int po_f64_finalize(cms_handle* h, int64_t total_counters, int64_t total_rows);
int po_f64_pair_cosines(cms_handle* h, const int64_t* d_qrows, int64_t nq, const int64_t* d_crows, int64_t m,
                        double* d_out, hipStream_t s);
int po_f64_point_queries(cms_handle* h, int64_t row, const int64_t* d_keys, int64_t m, double* d_out, hipStream_t s);
int po_f64_estimate_preferences(cms_handle* h, int64_t user_row, const int64_t* d_nb_rows, const double* d_sims,
                                int64_t m, const int64_t* d_items, int64_t q, int use_capper, float lo, float hi,
                                float* d_out, hipStream_t s);
int f64_norms(cms_handle* h);
int f64_pair_cosines(cms_handle* h, int64_t q_row, const int64_t* d_rows, int64_t m, double* d_out, hipStream_t s);
int f64_slab(cms_handle* h, int64_t q0, int64_t qc, double* d_slab);
int f64_point_queries(cms_handle* h, int64_t row, const int64_t* d_keys, int64_t m, double* d_out, hipStream_t s);
int f64_estimate_preferences(cms_handle* h, int64_t user_row, const int64_t* d_nb_rows, const double* d_sims,
                             int64_t m, const int64_t* d_items, int64_t q, int use_capper, float lo, float hi,
                             float* d_out, hipStream_t s);
// ---- cms_output.cpp ----
int java_double_to_string(double v, char* out, int cap);
// cms_recommend.cpp: GenericUserBasedRecommender's host logic (FastIDSet
// candidates, TopItems.getTopItems) around the device estimates
void recommend_candidates(const int64_t* nb_rows, int64_t m, int64_t user_row, const int64_t* pref_offsets,
                          const int64_t* pref_items, bool include_known, std::vector<int64_t>& out);
int32_t recommend_top_items(int32_t how_many, const int64_t* items, const float* est, int64_t q, int64_t* out_items,
                            float* out_values);
void parallel_users(int64_t n, int threads, const std::function<void(int64_t)>& fn);
int write_similar_items(cms_handle* h, const char* path, int32_t k, int32_t as_float);
int write_similarities(cms_handle* h, const char* path, int32_t k, int32_t format, double threshold);
// ---- cms_cosine_sym.hip: symmetric all-pairs waves, 256 x 192 tiles ----
struct SymArgs {
  const int8_t* img;  // K-blocked operand image (int8 limb 0 or fp4), row 0 = position img0
  int64_t img0;
  int64_t rs;         // bytes per image row
  int32_t kw;         // bytes per sketch row in the image
  int32_t depth;
  const double* nsq_t;  // [d][n] sqrt norms by permuted position
  int64_t n;
  int64_t s0, s_rows;   // the region's positions; blocks of kSymBlk rows from s0
  int32_t nb, wave, band, nblk;
  int32_t fsel, fblk0;              // only block pairs with a block below fblk0
  int32_t tsel, ts0, ts1, ts2, ts3;  // refresh: only block pairs with a block in [ts0, ts1) or [ts2, ts3)
  int32_t rect, si, sj, njc;        // band enumerated by si x sj block rectangles
  const double* thr;                // candidate lists (CandBufs)
  const float* thr32;               // the same thresholds as fp32 rounded toward -inf (k_thr_f32)
  uint32_t* ccnt;
  uint32_t* cidx;
  double* cval;
  int32_t cap;
  int32_t rbits;  // bits of the sketch-row index in the packed running-min state
  int32_t xchunk; // > 0: runs of xchunk consecutive tiles per XCD, the 8 XCDs side by side (0: one contiguous range per XCD)
};
// the kernel can run this table's waves (unweighted, its exact dot fits the
// packed state, LDS budget); fmt 0 int8, 1 fp4
bool sym_eligible(cms_handle* h, int fmt, int32_t* rbits);
// ---- cms_cosine_mls.hip: multi-limb x single-limb slab block on 256 x 192 tiles ----
struct MlsArgs {
  const int8_t* A;      // K-blocked virtual limb rows, row 0 = the launch's first (a multiple of kImgBlk in the group)
  int64_t a_vrows;      // rows available from A
  int64_t a_pos0;       // permuted position of the owner of A's row 0
  int64_t a_owners;     // owners from a_pos0 (the group's, up to the slab's end)
  const int8_t* B;      // K-blocked int8 image of the single-limb owners, row 0 = position b_img0
  int64_t b_img0, b_pos0, b_rows;  // candidates: positions [b_pos0, b_pos0 + b_rows), b_pos0 - b_img0 a multiple of kImgBlk
  int64_t rs;           // bytes per image row
  int32_t kw, depth;    // bytes per sketch row, sketch rows
  const double* nsq_t;  // [d][n] sqrt norms by permuted position
  int64_t n;
  double* out;          // slab [qcount][ldo], row = position - q0, column = position
  int64_t ldo, q0, qcount;
  int32_t weighted;
  int32_t tilesA, tilesB, ga, gb, nblk;  // set by launch_mls
};
bool mls_eligible(cms_handle* h);
int vl_blk_prepare(cms_handle* h, int gi);
int launch_mls(cms_handle* h, MlsArgs g, int ls);
int launch_sym(cms_handle* h, SymArgs g, int fmt, int64_t pair_slots);
int sym_stage_bytes();  // k_cosine_sym's K slice per stage = the images' slice width
// ---- cms_cosine_mfma.hip ----
const int64_t* cosine_perm_device(cms_handle* h);
// ---- cms_cosine_mfma.hip ----
int cosine_prepare(cms_handle* h);
bool mfma_eligible(cms_handle* h);
int cosine_slab(cms_handle* h, int64_t q0, int64_t qc, double* d_out);

}  // namespace cms
