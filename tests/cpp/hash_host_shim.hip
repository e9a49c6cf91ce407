// Host-side build of the product's hash (mahout_amd/csrc/cms_hash.h) for the
// CPU test tests/test_hash_host.py.  The kernels include the same header.
#include <hip/hip_runtime.h>
#include "../../mahout_amd/csrc/cms_hash.h"

extern "C" void host_buckets(const int64_t* a, const int64_t* b, int depth, int width, const int64_t* keys, int64_t n,
                             int32_t* out) {
  cms::HashParams hp{};
  for (int i = 0; i < depth; ++i) {
    hp.ap[i] = cms::reduce_key(a[i]);
    hp.bp[i] = cms::reduce_key(b[i]);
  }
  hp.width = (uint32_t)width;
  hp.depth = depth;
  cms::hash_finish(hp);
  for (int64_t i = 0; i < n; ++i) {
    uint64_t kp = cms::reduce_key(keys[i]);
    for (int r = 0; r < depth; ++r) out[i * depth + r] = (int32_t)cms::bucket(hp, r, kp);
  }
}

// The same keys through each_bucket (the kernels' unrolled form) and through
// the folding route alone; fallbacks[0] counts the bucket_q hashes whose
// fractional part fell inside the margin (decided by the folding route).
extern "C" void host_buckets_modes(const int64_t* a, const int64_t* b, int depth, int width, const int64_t* keys,
                                   int64_t n, int32_t* out_each, int32_t* out_exact, int64_t* fallbacks) {
  cms::HashParams hp{};
  for (int i = 0; i < depth; ++i) {
    hp.ap[i] = cms::reduce_key(a[i]);
    hp.bp[i] = cms::reduce_key(b[i]);
  }
  hp.width = (uint32_t)width;
  hp.depth = depth;
  cms::hash_finish(hp);
  int64_t fb = 0;
  for (int64_t i = 0; i < n; ++i) {
    uint64_t kp = cms::reduce_key(keys[i]);
    auto put = [&](int r, uint32_t c) { out_each[i * depth + r] = (int32_t)c; };
    if (depth == 4) cms::each_bucket<4>(hp, kp, put);
    else if (depth == 5) cms::each_bucket<5>(hp, kp, put);
    else if (depth == 6) cms::each_bucket<6>(hp, kp, put);
    else cms::each_bucket<0>(hp, kp, put);
    for (int r = 0; r < depth; ++r) {
      out_exact[i * depth + r] = (int32_t)cms::bucket_exact(hp, r, kp);
      if (hp.fastq && (kp >> 32) == 0) {
        const double y = fma(hp.qa[r], (double)(uint32_t)kp, hp.qb[r]);
        const double fr = y - floor(y);
        if (!(fr >= cms::kQEps && fr <= 1.0 - cms::kQEps)) ++fb;
      }
    }
  }
  fallbacks[0] = fb;
}

// bucket_wbq (the per-owner kernels' route for keys below 2^32) against
// bucket_wb, any width: out_q / out_w [n][depth]
extern "C" void host_buckets_wb(const int64_t* a, const int64_t* b, int depth, int width, const int64_t* keys,
                                int64_t n, int32_t* out_q, int32_t* out_w) {
  cms::HashParams hp{};
  for (int i = 0; i < depth; ++i) {
    hp.ap[i] = cms::reduce_key(a[i]);
    hp.bp[i] = cms::reduce_key(b[i]);
  }
  hp.width = 1;
  hp.depth = depth;
  cms::hash_finish(hp);
  const uint64_t barrett = (~0ULL) / (uint64_t)width;
  for (int64_t i = 0; i < n; ++i) {
    const uint64_t kp = cms::reduce_key(keys[i]);
    for (int r = 0; r < depth; ++r) {
      out_q[i * depth + r] = (int32_t)cms::bucket_wbq(hp, r, kp, (uint32_t)width, barrett);
      out_w[i * depth + r] = (int32_t)cms::bucket_wb(hp, r, kp, (uint32_t)width, barrett);
    }
  }
}
