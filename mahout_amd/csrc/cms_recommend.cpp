// cms_recommend.cpp -- GenericUserBasedRecommender.recommend for a batch of
// users (T/impl/recommender/GenericUserBasedRecommender.java:84-105) around
// the device estimates: the candidate set in FastIDSet iteration order
// (getAllOtherItems, :187-198), every candidate's estimate in ONE
// cms_estimate_preferences_batch, then TopItems.getTopItems
// (TopItems.java:47-88) with java.util.PriorityQueue's sift order.
//
// The candidate order and the heap order are what decide which of several
// equal estimates are recommended and in which order, so both are restated
// exactly: FastIDSet (T/impl/common/FastIDSet.java: double hashing, REMOVED
// markers, twin-prime table sizes, float load-factor arithmetic) and the
// JDK's binary heap (siftUpUsingComparator / siftDownUsingComparator).
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cmath>
#include <cstdint>
#include <thread>
#include <vector>

#include "cms_internal.h"

namespace cms {
namespace {

// Deterministic Miller-Rabin for n < 2^32 (bases 2, 3, 5, 7 suffice below
// 3,215,031,751); table sizes stay below RandomUtils.MAX_INT_SMALLER_TWIN_PRIME.
bool is_prime(uint64_t n) {
  if (n < 2) return false;
  for (uint64_t p : {2ull, 3ull, 5ull, 7ull, 11ull, 13ull}) {
    if (n % p == 0) return n == p;
  }
  uint64_t d = n - 1;
  int s = 0;
  while ((d & 1) == 0) {
    d >>= 1;
    ++s;
  }
  auto mulmod = [n](uint64_t a, uint64_t b) { return (uint64_t)((unsigned __int128)a * b % n); };
  for (uint64_t a : {2ull, 3ull, 5ull, 7ull, 11ull}) {
    uint64_t x = 1, b = a % n, e = d;
    while (e) {
      if (e & 1) x = mulmod(x, b);
      b = mulmod(b, b);
      e >>= 1;
    }
    if (x == 1 || x == n - 1) continue;
    bool comp = true;
    for (int r = 1; r < s && comp; ++r) {
      x = mulmod(x, x);
      if (x == n - 1) comp = false;
    }
    if (comp) return false;
  }
  return true;
}

// commons-math3 Primes.nextPrime: the smallest prime >= n
int64_t next_prime(int64_t n) {
  if (n < 2) n = 2;
  while (!is_prime((uint64_t)n)) ++n;
  return n;
}

// RandomUtils.nextTwinPrime (math/.../common/RandomUtils.java:86-98)
int32_t next_twin_prime(int32_t n) {
  if (n <= 3) return 5;
  int64_t next = next_prime(n);
  while (!is_prime((uint64_t)(next + 2))) next = next_prime(next + 4);
  return (int32_t)(next + 2);
}

constexpr int64_t kNull = INT64_MIN, kRemoved = INT64_MAX;

// FastIDSet with DEFAULT_LOAD_FACTOR 1.5f
struct FastIdSet {
  std::vector<int64_t> keys;
  float lf = 1.5f;
  int32_t entries = 0, slots_used = 0;

  explicit FastIdSet(int32_t size = 2) { keys.assign((size_t)next_twin_prime((int32_t)(lf * (float)size)), kNull); }

  static int32_t hash_of(int64_t key) { return (int32_t)key & 0x7FFFFFFF; }  // (int) key & 0x7FFFFFFF

  int32_t find(int64_t key) const {
    const int32_t hc = hash_of(key), n = (int32_t)keys.size();
    const int32_t jump = 1 + hc % (n - 2);
    int32_t index = hc % n;
    int64_t cur = keys[(size_t)index];
    while (cur != kNull && key != cur) {  // true when cur == REMOVED
      index -= index < jump ? jump - n : jump;
      cur = keys[(size_t)index];
    }
    return index;
  }

  int32_t find_for_add(int64_t key) const {
    const int32_t hc = hash_of(key), n = (int32_t)keys.size();
    const int32_t jump = 1 + hc % (n - 2);
    int32_t index = hc % n;
    int64_t cur = keys[(size_t)index];
    while (cur != kNull && cur != kRemoved && key != cur) {
      index -= index < jump ? jump - n : jump;
      cur = keys[(size_t)index];
    }
    if (cur != kRemoved) return index;
    const int32_t add_index = index;
    while (cur != kNull && key != cur) {
      index -= index < jump ? jump - n : jump;
      cur = keys[(size_t)index];
    }
    return key == cur ? index : add_index;
  }

  void rehash(int32_t new_size) {
    std::vector<int64_t> old;
    old.swap(keys);
    entries = slots_used = 0;
    keys.assign((size_t)new_size, kNull);
    for (int64_t k : old)
      if (k != kNull && k != kRemoved) add(k);
  }

  bool add(int64_t key) {
    if ((float)slots_used * lf >= (float)keys.size()) {
      if ((float)entries * lf >= (float)slots_used) rehash(next_twin_prime((int32_t)(lf * (float)keys.size())));
      else rehash(next_twin_prime((int32_t)(lf * (float)entries)));
    }
    const int32_t index = find_for_add(key);
    const int64_t old = keys[(size_t)index];
    if (old == key) return false;
    keys[(size_t)index] = key;
    ++entries;
    if (old == kNull) ++slots_used;
    return true;
  }

  bool remove(int64_t key) {
    if (key == kNull || key == kRemoved) return false;
    const int32_t index = find(key);
    if (keys[(size_t)index] == kNull) return false;
    keys[(size_t)index] = kRemoved;
    --entries;
    return true;
  }

  void add_all(const FastIdSet& o) {
    for (int64_t k : o.keys)
      if (k != kNull && k != kRemoved) add(k);
  }
  void remove_all(const FastIdSet& o) {
    for (int64_t k : o.keys)
      if (k != kNull && k != kRemoved) remove(k);
  }
};

// GenericDataModel.getItemIDsFromUser (GenericDataModel.java:219-227): a
// FastIDSet sized to the user's preference count, items added in order
FastIdSet item_set(const int64_t* items, int64_t m) {
  FastIdSet s((int32_t)m);
  for (int64_t i = 0; i < m; ++i) s.add(items[i]);
  return s;
}

struct Rec {
  int64_t item;
  float value;
};

// java.util.PriorityQueue under Collections.reverseOrder(
// ByValueRecommendedItemComparator): the head is the lowest value
struct RecHeap {
  std::vector<Rec> q;
  static int cmp(const Rec& a, const Rec& b) { return a.value < b.value ? -1 : a.value > b.value ? 1 : 0; }
  void add(Rec x) {
    size_t k = q.size();
    q.push_back(x);
    while (k > 0) {
      const size_t parent = (k - 1) >> 1;
      if (cmp(x, q[parent]) >= 0) break;
      q[k] = q[parent];
      k = parent;
    }
    q[k] = x;
  }
  void poll() {
    const Rec x = q.back();
    q.pop_back();
    const size_t n = q.size();
    if (!n) return;
    size_t k = 0;
    const size_t half = n >> 1;
    while (k < half) {
      size_t child = 2 * k + 1;
      Rec c = q[child];
      const size_t right = child + 1;
      if (right < n && cmp(c, q[right]) > 0) c = q[child = right];
      if (cmp(x, c) <= 0) break;
      q[k] = c;
      k = child;
    }
    q[k] = x;
  }
};

}  // namespace

// Candidate items of one user: getAllOtherItems over the neighbourhood
// (FastIDSet iteration order).  pref_items of model row r:
// pref_items[pref_offsets[r] .. pref_offsets[r + 1]).
void recommend_candidates(const int64_t* nb_rows, int64_t m, int64_t user_row, const int64_t* pref_offsets,
                          const int64_t* pref_items, bool include_known, std::vector<int64_t>& out) {
  FastIdSet possible;
  for (int64_t j = 0; j < m; ++j) {
    const int64_t r = nb_rows[j];
    possible.add_all(item_set(pref_items + pref_offsets[r], pref_offsets[r + 1] - pref_offsets[r]));
  }
  if (!include_known && user_row >= 0)
    possible.remove_all(item_set(pref_items + pref_offsets[user_row], pref_offsets[user_row + 1] - pref_offsets[user_row]));
  out.clear();
  out.reserve((size_t)possible.entries);
  for (int64_t k : possible.keys)
    if (k != kNull && k != kRemoved) out.push_back(k);
}

// TopItems.getTopItems with no rescorer; returns the list length (<= how_many)
int32_t recommend_top_items(int32_t how_many, const int64_t* items, const float* est, int64_t q, int64_t* out_items,
                            float* out_values) {
  RecHeap heap;
  heap.q.reserve((size_t)how_many + 1);
  bool full = false;
  double lowest = -INFINITY;
  for (int64_t i = 0; i < q; ++i) {
    const double pref = (double)est[i];
    if (std::isnan(pref) || (full && !(pref > lowest))) continue;
    heap.add(Rec{items[i], (float)pref});
    if (full) {
      heap.poll();
    } else if ((int64_t)heap.q.size() > how_many) {
      full = true;
      heap.poll();
    }
    lowest = (double)heap.q[0].value;
  }
  std::vector<Rec> res = heap.q;  // Collections.sort (stable) by value, descending
  std::stable_sort(res.begin(), res.end(), [](const Rec& a, const Rec& b) { return a.value > b.value; });
  for (size_t i = 0; i < res.size(); ++i) {
    out_items[i] = res[i].item;
    out_values[i] = res[i].value;
  }
  return (int32_t)res.size();
}

// Run fn(u) for u in [0, n) on up to `threads` host threads.
void parallel_users(int64_t n, int threads, const std::function<void(int64_t)>& fn) {
  threads = (int)std::max<int64_t>(1, std::min<int64_t>(threads, n));
  if (threads == 1) {
    for (int64_t u = 0; u < n; ++u) fn(u);
    return;
  }
  std::vector<std::thread> pool;
  for (int t = 0; t < threads; ++t)
    pool.emplace_back([&, t] {
      for (int64_t u = t; u < n; u += threads) fn(u);
    });
  for (auto& th : pool) th.join();
}

}  // namespace cms
