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
//
// Power-of-two widths (every fixed-shape config) take a cheaper exact route
// for reduced keys below 2^32 (bucket_q): with X = a'k' + b' and
// q = floor(X / p), s = X - q p == X + 25 q (mod 2^m) because p == -25
// (mod 2^m) for m <= 63, so the bucket needs only q and the low m bits of
// a', k', b' (24-bit multiplies).  q comes from one fp64 FMA,
// y = fma(a'/p, k', b'/p) (both quotients rounded once on the host); its error
// is below 2^-20 (a'/p within 2^-53 times k' < 2^32, plus the FMA's rounding
// at y < 2^32), so floor(y) == q whenever y's fractional part lies in
// [2^-16, 1 - 2^-16] -- otherwise (about 1 hash in 30,000) the folding
// route above decides.  Either way the bucket is the BigInteger one.
#pragma once
#include <math.h>
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
  int32_t fastq;               // bucket_q applies: power-of-two width <= 2^24
  double qa[CMS_MAX_DEPTH];    // a'/p rounded to double (bucket_q)
  double qb[CMS_MAX_DEPTH];    // b'/p rounded to double
#ifdef CMS_BUILD_GATHERHASH    // bound analysis only: [2^24] x 16 B per-key bucket table (contents unset)
  const uint4* gtab;
#endif
};

// The derived fields of a HashParams whose ap, bp, width and depth are set.
inline void hash_finish(HashParams& hp) {
  hp.pow2 = hp.width != 0 && (hp.width & (hp.width - 1)) == 0;
  hp.wmask = hp.pow2 ? hp.width - 1u : 0u;
  hp.barrett = hp.pow2 ? 0 : (~0ULL) / (uint64_t)hp.width;
  hp.fastq = hp.pow2 && hp.width <= (1u << 24);
  for (int i = 0; i < CMS_MAX_DEPTH; ++i) {
    // x87 long double holds a', b' and p exactly; the quotient rounds once
    // to 64 bits, then to 53 (error < 2^-53 relative, far inside the margin)
    hp.qa[i] = i < hp.depth ? (double)((long double)hp.ap[i] / (long double)kPrime) : 0.0;
    hp.qb[i] = i < hp.depth ? (double)((long double)hp.bp[i] / (long double)kPrime) : 0.0;
  }
}

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

// Bucket of a reduced key in sketch row r, by the folding route.
CMS_HD uint32_t bucket_exact(const HashParams& hp, int r, uint64_t kp) {
  uint64_t s = ((kp >> 32) == 0 ? mulmod_p_small(hp.ap[r], (uint32_t)kp) : mulmod_p(hp.ap[r], kp)) + hp.bp[r];  // < 2p
  if (s >= kPrime) s -= kPrime;
  if (hp.pow2) return (uint32_t)(s & hp.wmask);
  uint64_t q = (uint64_t)(((unsigned __int128)s * hp.barrett) >> 64);
  uint64_t rem = s - q * hp.width;
  while (rem >= hp.width) rem -= hp.width;
  return (uint32_t)rem;
}

#if defined(__HIP_DEVICE_COMPILE__)
#define CMS_MUL24(x, y) __umul24((x), (y))
#else
#define CMS_MUL24(x, y) (((x) & 0xFFFFFFu) * ((y) & 0xFFFFFFu))
#endif
constexpr double kQEps = 1.0 / 65536.0;  // fractional-part margin of bucket_q (error < 2^-20)

// bucket_q (header comment): hp.fastq, kp < 2^32; kf = (double)kp,
// km = kp & wmask.  The low m bits: a'k' + b' + 25 q (mod 2^m), m <= 24, by
// 24-bit multiplies (q's low 24 bits suffice).  Inside the margin the
// estimate q0 = floor(y) is off by at most one, in the direction the
// fractional part says, and the wrapping 64-bit residue s = X - q0 p
// (mod 2^64) settles it: s < p exactly when q0 is right.
CMS_HD uint32_t bucket_q(const HashParams& hp, int r, uint64_t kp, double kf, uint32_t km) {
  const double y = fma(hp.qa[r], kf, hp.qb[r]);
  const double fl = floor(y);
  const double fr = y - fl;  // exact
  union {
    double d;
    uint64_t u;
  } qb;
  qb.d = fl + 4503599627370496.0;  // 2^52: the integer q0 <= 2^32 in the low mantissa bits
  uint32_t q = (uint32_t)qb.u;
  if (!(fr >= kQEps && fr <= 1.0 - kQEps)) {  // about 1 hash in 30,000
    // q0 needs 33 bits here: y can round up to exactly 2^32 (true q 2^32 - 1)
    const uint64_t q0 = qb.u & 0xFFFFFFFFFFFFFULL;
    const uint64_t x = hp.ap[r] * kp + hp.bp[r];    // X mod 2^64
    const uint64_t s = x - ((q0 << 63) - 25u * q0);  // X - q0 p mod 2^64 (p = 2^63 - 25)
    if (s >= kPrime) q = fr < 0.5 ? q - 1u : q + 1u;
  }
  const uint32_t xm = CMS_MUL24((uint32_t)hp.ap[r] & hp.wmask, km) + (uint32_t)hp.bp[r];
  return (xm + CMS_MUL24(q, 25u)) & hp.wmask;
}

// Bucket of a reduced key in sketch row r.
CMS_HD uint32_t bucket(const HashParams& hp, int r, uint64_t kp) {
  if (hp.fastq && (kp >> 32) == 0) return bucket_q(hp, r, kp, (double)(uint32_t)kp, (uint32_t)kp & hp.wmask);
  return bucket_exact(hp, r, kp);
}

// All d buckets of one reduced key: f(r, bucket).  D > 0: the handle's depth
// is exactly D and the rows unroll (their constants stay in scalar registers
// across a key loop instead of being reloaded per row; a key below 2^32 at a
// power-of-two width converts once for all rows).  D == 0: any depth.
template <int D, typename F>
CMS_HD void each_bucket(const HashParams& hp, uint64_t kp, F&& f) {
#ifdef CMS_BUILD_CHEAPHASH  // bound analysis only: a trivial hash instead of the exact mod-p one
  if (D > 0) {
#pragma unroll
    for (int r = 0; r < D; ++r) f(r, (uint32_t)((kp >> r) & hp.wmask));
  } else {
    for (int r = 0; r < hp.depth; ++r) f(r, (uint32_t)((kp >> r) & hp.wmask));
  }
  return;
#endif
#ifdef CMS_BUILD_GATHERHASH  // bound analysis only: one 16-B gather per key instead of d mod-p hashes
  {
    const uint4 e = hp.gtab[kp & 0xFFFFFFu];
    const uint32_t v[4] = {e.x, e.y, e.z, e.w};
    for (int r = 0; r < (D > 0 ? D : hp.depth); ++r) f(r, (v[(r >> 1) & 3] >> ((r & 1) << 4)) & hp.wmask);
    return;
  }
#endif
  if (D > 0) {
    if (hp.fastq && (kp >> 32) == 0) {
      const double kf = (double)(uint32_t)kp;
      const uint32_t km = (uint32_t)kp & hp.wmask;
#pragma unroll
      for (int r = 0; r < D; ++r) f(r, bucket_q(hp, r, kp, kf, km));
    } else {
#pragma unroll
      for (int r = 0; r < D; ++r) f(r, bucket_exact(hp, r, kp));
    }
  } else {
    for (int r = 0; r < hp.depth; ++r) f(r, bucket(hp, r, kp));
  }
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

// bucket_wb for a reduced key below 2^32 (the usual DataModel IDs), without
// the 128-bit fold: q0 = floor(fma(a'/p, k', b'/p)) is q or q +- 1 (its error
// is below 2^-20), the wrapping 64-bit residue s = a'k' + b' - q0 p (mod 2^64)
// is then < p exactly when q0 = q, and one add or subtract of p repairs it
// otherwise (direction from the fractional part); Barrett mod w as bucket_wb.
// residue_wbq is the width-independent part, (a_r k + b_r) mod p.
CMS_HD uint64_t residue_wbq(const HashParams& hp, int r, uint64_t kp) {
  if ((kp >> 32) != 0) {
    uint64_t s = mulmod_p(hp.ap[r], kp) + hp.bp[r];
    if (s >= kPrime) s -= kPrime;
    return s;
  }
  const double y = fma(hp.qa[r], (double)(uint32_t)kp, hp.qb[r]);
  const double fl = floor(y);
  const double fr = y - fl;
  union {
    double d;
    uint64_t u;
  } qb;
  qb.d = fl + 4503599627370496.0;  // 2^52
  const uint64_t q = qb.u & 0xFFFFFFFFFFFFFULL;  // q0 <= 2^32: y can round up to exactly 2^32
  uint64_t s = hp.ap[r] * kp + hp.bp[r] - ((q << 63) - 25u * q);  // X - q0 p (mod 2^64)
  if (s >= kPrime) s = fr < 0.5 ? s + kPrime : s - kPrime;
  return s;
}

// s mod w for s < 2^63 by the Barrett constant floor((2^64-1)/w)
CMS_HD uint32_t mod_barrett(uint64_t s, uint32_t w, uint64_t barrett) {
  const uint64_t qq = (uint64_t)(((unsigned __int128)s * barrett) >> 64);
  uint64_t rem = s - qq * w;
  while (rem >= w) rem -= w;
  return (uint32_t)rem;
}

CMS_HD uint32_t bucket_wbq(const HashParams& hp, int r, uint64_t kp, uint32_t w, uint64_t barrett) {
  return mod_barrett(residue_wbq(hp, r, kp), w, barrett);
}

}  // namespace cms
