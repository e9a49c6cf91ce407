// cms_hash.h -- exact count-min-sketch hash for gfx950 (and the host).
//
// Restates HashFunction.hash (T/impl/common/HashFunction.java:31-34):
//     ((a * key + b) mod p) mod w,   p = 2^63 - 25  (HashFunctionBuilder.java:24)
// evaluated by the reference in java.math.BigInteger (non-negative mod).
//
// The GPU form never builds a 128-bit signed value: a, b and key are reduced
// into [0, p) once (a, b on the host, key once per pair), the product a'*k'
// (< 2^126) is folded with 2^63 == 25 (mod p) twice, and the final "mod w" is a
// mask for power-of-two widths or a Barrett reduction with a precomputed
// reciprocal otherwise.  Every step is exact integer arithmetic, so the
// bucket equals the BigInteger result bit-for-bit for every int64 key
// (negative keys included).
#pragma once
#include <stdint.h>

#ifndef CMS_HD
#define CMS_HD __host__ __device__ __forceinline__
#endif

#define CMS_MAX_DEPTH 32

namespace cms {

constexpr uint64_t kPrime = 9223372036854775783ULL;  // 2^63 - 25
constexpr uint64_t kMask63 = 0x7FFFFFFFFFFFFFFFULL;

// Per-handle hash state passed to kernels by value (kernarg segment -> SGPRs).
struct HashParams {
  uint64_t ap[CMS_MAX_DEPTH];  // a_i mod p
  uint64_t bp[CMS_MAX_DEPTH];  // b_i mod p
  uint64_t barrett;            // floor((2^64-1)/w) for non-power-of-two w
  uint32_t width;
  uint32_t wmask;              // w-1 when w is a power of two
  int32_t depth;
  int32_t pow2;
  int32_t frac_bits;           // counters hold preference * 2^frac_bits
};

// key mod p in [0, p) for any signed 64-bit key.
CMS_HD uint64_t reduce_key(int64_t k) {
  const int64_t P = (int64_t)kPrime;
  if (k >= 0) return (uint64_t)(k >= P ? k - P : k);
  int64_t t = k + P;  // k >= -2^63 so t >= -25
  if (t < 0) t += P;
  return (uint64_t)t;
}

// (x * y) mod p for x, y in [0, p).
CMS_HD uint64_t mulmod_p(uint64_t x, uint64_t y) {
  unsigned __int128 prod = (unsigned __int128)x * y;  // < 2^126
  uint64_t lo = (uint64_t)prod;
  uint64_t hi = (uint64_t)(prod >> 64);
  uint64_t H = (hi << 1) | (lo >> 63);  // prod >> 63   (< 2^63)
  uint64_t L = lo & kMask63;            // prod mod 2^63
  // prod == H*2^63 + L == 25*H + L (mod p);  25*H < 2^68
  unsigned __int128 t = (unsigned __int128)H * 25u;
  uint64_t tH = (uint64_t)(t >> 63);  // < 25
  uint64_t tL = (uint64_t)t & kMask63;
  uint64_t z = tL + L;  // < 2^64
  if (z >= kPrime) z -= kPrime;
  if (z >= kPrime) z -= kPrime;
  z += tH * 25u;  // < p + 625
  if (z >= kPrime) z -= kPrime;
  return z;
}

// (x * y) mod p for x in [0, p) and y < 2^32 (keys of the usual ID ranges):
// the product is < 2^95, so one fold of 2^63 == 25 leaves z < 2p and one
// conditional subtract finishes -- two 32x32 multiplies instead of four.
CMS_HD uint64_t mulmod_p_small(uint64_t x, uint32_t y) {
  const uint64_t p0 = (uint64_t)(uint32_t)x * y;
  const uint64_t p1 = (x >> 32) * (uint64_t)y;  // < 2^63
  const uint64_t lo = p0 + (p1 << 32);
  const uint64_t hi = (p1 >> 32) + (lo < p0 ? 1u : 0u);  // prod >> 64 (< 2^31)
  const uint64_t H = (hi << 1) | (lo >> 63);             // prod >> 63 (< 2^32)
  uint64_t z = (lo & kMask63) + H * 25u;                  // < 2^63 + 2^37 < 2p
  if (z >= kPrime) z -= kPrime;
  return z;
}

// Bucket of a reduced key in sketch row r.
CMS_HD uint32_t bucket(const HashParams& hp, int r, uint64_t kp) {
  uint64_t s = ((kp >> 32) == 0 ? mulmod_p_small(hp.ap[r], (uint32_t)kp) : mulmod_p(hp.ap[r], kp)) + hp.bp[r];  // < 2p
  if (s >= kPrime) s -= kPrime;
  if (hp.pow2) return (uint32_t)(s & hp.wmask);
  uint64_t q = (uint64_t)(((unsigned __int128)s * hp.barrett) >> 64);
  uint64_t rem = s - q * hp.width;
  while (rem >= hp.width) rem -= hp.width;
  return (uint32_t)rem;
}

// Bucket for an arbitrary width w with its Barrett constant floor((2^64-1)/w)
// (per-owner sketch shapes: CosineCM hashes u1 at u2's width).
CMS_HD uint32_t bucket_wb(const HashParams& hp, int r, uint64_t kp, uint32_t w, uint64_t barrett) {
  uint64_t s = mulmod_p(hp.ap[r], kp) + hp.bp[r];
  if (s >= kPrime) s -= kPrime;
  uint64_t q = (uint64_t)(((unsigned __int128)s * barrett) >> 64);
  uint64_t rem = s - q * w;
  while (rem >= w) rem -= w;
  return (uint32_t)rem;
}

}  // namespace cms
