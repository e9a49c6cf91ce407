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
  hp.pow2 = (width & (width - 1)) == 0;
  hp.wmask = hp.pow2 ? (uint32_t)(width - 1) : 0u;
  hp.barrett = hp.pow2 ? 0 : (~0ULL) / (uint64_t)width;
  for (int64_t i = 0; i < n; ++i) {
    uint64_t kp = cms::reduce_key(keys[i]);
    for (int r = 0; r < depth; ++r) out[i * depth + r] = (int32_t)cms::bucket(hp, r, kp);
  }
}
