// Host build of the recommender's host logic (mahout_amd/csrc/cms_recommend.cpp)
// for the CPU test tests/test_recommend_host.py: FastIDSet candidate order
// and TopItems.getTopItems, compared with the Python restatement in
// mahout_amd/taste.py.
#include <cstdint>
#include <vector>

#include "../../mahout_amd/csrc/cms_internal.h"

extern "C" int64_t host_candidates(const int64_t* nb_rows, int64_t m, int64_t user_row, const int64_t* pref_offsets,
                                   const int64_t* pref_items, int include_known, int64_t* out, int64_t cap) {
  std::vector<int64_t> c;
  cms::recommend_candidates(nb_rows, m, user_row, pref_offsets, pref_items, include_known != 0, c);
  for (size_t i = 0; i < c.size() && (int64_t)i < cap; ++i) out[i] = c[i];
  return (int64_t)c.size();
}

extern "C" int32_t host_top_items(int32_t how_many, const int64_t* items, const float* est, int64_t q,
                                  int64_t* out_items, float* out_values) {
  return cms::recommend_top_items(how_many, items, est, q, out_items, out_values);
}
