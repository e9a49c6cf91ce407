// cms_mfma.h -- gfx950 MFMA helpers shared by the all-pairs cosine kernels
// (cms_cosine_mfma.hip, cms_cosine_sym.hip).  Not part of the ABI.
#pragma once
#include <hip/hip_runtime.h>

#include <cstdint>

namespace cms {

typedef int8_t i8x16 __attribute__((ext_vector_type(16)));
typedef int32_t i32x16 __attribute__((ext_vector_type(16)));

// K-blocked layout: the image is cut into blocks of kImgBlk rows, and inside a
// block every sw-byte K slice of its rows is one contiguous run
// ([slice][row][sw B], 8 KiB at sw = 128); a stage of an operand panel is then
// a few contiguous runs instead of one line per row a row stride apart (DRAM
// page locality for the symmetric waves' fills).  Panels start on a block
// (64 rows: the 256- and 192-row panels of both symmetric kernels).  Rows
// past the end of the image (the last block's padding) are zero.
constexpr int kImgBlk = 64;
// symmetric-wave blocks: 256 rows (k_cosine_big, 256 x 128 tiles) and 768
// rows (k_cosine_sym, 3 x 4 tiles of 256 x 192); the single-limb image
// regions start on a multiple of both
constexpr int kSymBlk = 768;
// sw: K slice width in bytes (the symmetric waves' stage depth, 128 or 64)
__device__ __forceinline__ int64_t blk_off(int64_t row, int64_t kb, int64_t rs, int sw = 128) {
  return (row / kImgBlk) * (kImgBlk * rs) + (kb / sw) * (kImgBlk * sw) + (row % kImgBlk) * sw + (kb % sw);
}

// LDS image of a BK-byte K slice of R rows: row-major, the 16-B chunk index
// XOR-swizzled so that each 16-lane ds_read_b128 group (16 consecutive rows,
// one chunk) hits 16 distinct 16-B slots of a 256-B bank line.
template <int BK>
__device__ __forceinline__ int lds_off_bk(int row, int ch) {
  if constexpr (BK == 128) return row * 128 + ((ch ^ ((row >> 1) & 7)) << 4);
  else return row * 64 + ((ch ^ ((row >> 2) & 3)) << 4);  // BK == 64
}

// s_waitcnt vmcnt(N) alone (expcnt / lgkmcnt fields at their maxima), gfx9 encoding.
template <int N>
__device__ __forceinline__ void wait_vmcnt() {
  static_assert(N >= 0 && N < 64, "vmcnt range");
  __builtin_amdgcn_s_waitcnt((N & 15) | ((N >> 4) << 14) | (7 << 4) | (15 << 8));
}

typedef float f32x16 __attribute__((ext_vector_type(16)));
typedef int32_t i32x4 __attribute__((ext_vector_type(4)));
typedef int32_t i32x8 __attribute__((ext_vector_type(8)));

// FMT 0: int8 limbs, v_mfma_i32_32x32x32_i8.  FMT 1: fp4 (e2m1) counters
// <= 4, v_mfma_f32_32x32x64_f8f6f4 (unscaled): the same 16 B per lane per
// fragment carries 32 counters instead of 16, so a stage holds twice the K
// at the same MFMA cycles.  Products <= 16 and row sums <= 16 * 32768 < 2^24
// keep the f32 accumulation exact.
template <int FMT>
struct AccOf {
  typedef i32x16 type;
};
template <>
struct AccOf<1> {
  typedef f32x16 type;
};

template <int FMT>
__device__ __forceinline__ typename AccOf<FMT>::type mfma_step(const i8x16& a, const i8x16& b,
                                                               typename AccOf<FMT>::type c) {
  if constexpr (FMT == 0) {
    return __builtin_amdgcn_mfma_i32_32x32x32_i8(a, b, c, 0, 0, 0);
  } else {
    const i32x4 a4 = __builtin_bit_cast(i32x4, a), b4 = __builtin_bit_cast(i32x4, b);
    const i32x4 z = {0, 0, 0, 0};
    const i32x8 a8 = __builtin_shufflevector(a4, z, 0, 1, 2, 3, 4, 5, 6, 7);
    const i32x8 b8 = __builtin_shufflevector(b4, z, 0, 1, 2, 3, 4, 5, 6, 7);
    return __builtin_amdgcn_mfma_scale_f32_32x32x64_f8f6f4(a8, b8, c, 4, 4, 0, 0, 0, 0);  // cbsz/blgp 4: e2m1
  }
}

}  // namespace cms
