// cms_output.cpp -- FileSimilarItemsWriter-format output of the all-pairs
// top-k (T/impl/similarity/precompute/FileSimilarItemsWriter.java:50-61):
// one line "itemID,similarItemID,similarity" per similar item, items in
// ascending ID order, each item's list most similar first.  The similarity
// is written like Java's String.valueOf(double) (Double.toString, shortest
// uniquely-distinguishing digits as specified since JDK 19).  With as_float
// the value is first narrowed to float, as RecommendedItem.getValue() does for
// the SimilarItems that MultithreadedBatchItemSimilarities collects
// (SimilarItems.java:36-47).
#include <hip/hip_runtime.h>

#include <charconv>
#include <cmath>
#include <algorithm>
#include <cstdio>
#include <cstring>
#include <limits>
#include <string>
#include <vector>

#include "cms_internal.h"

namespace cms {

// Double.toString: NaN / Infinity; plain notation for 1e-3 <= |v| < 1e7
// (at least one fractional digit), else d.ddd...E[-]n.
int java_double_to_string(double v, char* out, int cap) {
  std::string s;
  if (std::isnan(v)) {
    s = "NaN";
  } else if (std::isinf(v)) {
    s = v > 0 ? "Infinity" : "-Infinity";
  } else if (v == 0.0) {
    s = std::signbit(v) ? "-0.0" : "0.0";
  } else {
    char buf[64];
    auto r = std::to_chars(buf, buf + sizeof(buf), v, std::chars_format::scientific);
    *r.ptr = 0;
    // buf = [-]d[.ddd]e[+-]XX
    const char* p = buf;
    if (*p == '-') {
      s += '-';
      ++p;
    }
    std::string digits;
    while (*p && *p != 'e') {
      if (*p != '.') digits += *p;
      ++p;
    }
    const int e10 = std::atoi(p + 1);  // value = d.ddd * 10^e10
    const double a = std::fabs(v);
    if (a >= 1e-3 && a < 1e7) {
      if (e10 >= 0) {
        std::string ip = digits.substr(0, std::min<size_t>(digits.size(), e10 + 1));
        while ((int)ip.size() < e10 + 1) ip += '0';
        std::string fp = (int)digits.size() > e10 + 1 ? digits.substr(e10 + 1) : "0";
        s += ip + "." + fp;
      } else {
        s += "0." + std::string(-e10 - 1, '0') + digits;
      }
    } else {
      s += digits.substr(0, 1) + "." + (digits.size() > 1 ? digits.substr(1) : "0") + "E" + std::to_string(e10);
    }
  }
  if ((int)s.size() + 1 > cap) return -1;
  std::memcpy(out, s.c_str(), s.size() + 1);
  return (int)s.size();
}

namespace {

struct OutBuf {
  FILE* f = nullptr;
  std::vector<char> buf;
  bool ok = true;
  void put(const char* p, size_t len) {
    buf.insert(buf.end(), p, p + len);
    if (buf.size() > (1u << 22)) flush();
  }
  void put_id(int64_t v) {
    char num[32];
    const int len = std::snprintf(num, sizeof(num), "%lld", (long long)v);
    put(num, (size_t)len);
  }
  void put_double(double v) {
    char num[64];
    const int len = java_double_to_string(v, num, sizeof(num));
    put(num, (size_t)len);
  }
  void flush() {
    if (!buf.empty() && std::fwrite(buf.data(), 1, buf.size(), f) != buf.size()) ok = false;
    buf.clear();
  }
};

}  // namespace

// The all-pairs lists on the host: ids/scores [n][k] (owner IDs), counts [n].
static int host_lists(cms_handle* h, int32_t k, std::vector<int64_t>& ids, std::vector<double>& sc,
                      std::vector<int32_t>& cnt) {
  const int64_t n = h->n;
  DevBuf o_ids, o_sc, o_cnt;
  CMS_HIP(o_ids.ensure(sizeof(int64_t) * n * k));
  CMS_HIP(o_sc.ensure(sizeof(double) * n * k));
  CMS_HIP(o_cnt.ensure(sizeof(int32_t) * n));
  int rc = top_k_all(h, k, o_ids.as<int64_t>(), o_sc.as<double>(), o_cnt.as<int32_t>());
  if (rc) return rc;
  ids.resize((size_t)n * k);
  sc.resize((size_t)n * k);
  cnt.resize(n);
  CMS_HIP(hipMemcpyAsync(ids.data(), o_ids.ptr, sizeof(int64_t) * n * k, hipMemcpyDeviceToHost, h->stream));
  CMS_HIP(hipMemcpyAsync(sc.data(), o_sc.ptr, sizeof(double) * n * k, hipMemcpyDeviceToHost, h->stream));
  CMS_HIP(hipMemcpyAsync(cnt.data(), o_cnt.ptr, sizeof(int32_t) * n, hipMemcpyDeviceToHost, h->stream));
  CMS_HIP(hipStreamSynchronize(h->stream));
  return CMS_OK;
}

// ItemSimilarityJob's result (T/hadoop/similarity/item/ItemSimilarityJob.java:181-233):
// every pair of a top-k list as (min ID, max ID) (:214-220), one line per
// distinct pair (the reducer keeps the first value, :226-231), in
// EntityEntityWritable order (aID, then bID; EntityEntityWritable.java:64-71),
// "aID\tbID\tsimilarity" with DoubleWritable's Double.toString.
static int write_item_similarity_job(cms_handle* h, OutBuf& o, int32_t k, const std::vector<int64_t>& ids,
                                     const std::vector<double>& sc, const std::vector<int32_t>& cnt, double thr) {
  struct P {
    int64_t a, b;
    double v;
  };
  std::vector<P> pairs;
  for (int64_t r = 0; r < h->n; ++r) {
    const int64_t owner = h->h_owner_ids.empty() ? r : h->h_owner_ids[r];
    for (int32_t i = 0; i < cnt[r]; ++i) {
      const int64_t other = ids[(size_t)r * k + i];
      const double v = sc[(size_t)r * k + i];
      // TopSimilarItemsQueue admits only similarity > its sentinel's
      // Double.MIN_VALUE (zero is not a non-zero of the similarity vector anyway)
      if (!(v > std::numeric_limits<double>::denorm_min()) || v < thr) continue;
      pairs.push_back(P{std::min(owner, other), std::max(owner, other), v});
    }
  }
  // stable: for a pair listed by both owners the lower ID's list comes first
  std::stable_sort(pairs.begin(), pairs.end(), [](const P& x, const P& y) {
    return x.a != y.a ? x.a < y.a : x.b < y.b;
  });
  for (size_t i = 0; i < pairs.size(); ++i) {
    if (i > 0 && pairs[i].a == pairs[i - 1].a && pairs[i].b == pairs[i - 1].b) continue;
    o.put_id(pairs[i].a);
    o.put("\t", 1);
    o.put_id(pairs[i].b);
    o.put("\t", 1);
    o.put_double(pairs[i].v);
    o.put("\n", 1);
  }
  return CMS_OK;
}

// spark-itemsimilarity's TextDelimitedIndexedDatasetWriter with the default
// write schema (spark/.../drivers/TextDelimitedReaderWriter.scala:244-303,
// math-scala/.../indexeddataset/Schema.scala:62-66): per owner
// "ID\tID1:s1 ID2:s2 ..." over the non-zero similarities sorted by strength
// descending (stable: ties stay in list order), a bare "ID" when none.
static int write_spark_itemsimilarity(cms_handle* h, OutBuf& o, int32_t k, const std::vector<int64_t>& ids,
                                      const std::vector<double>& sc, const std::vector<int32_t>& cnt, double thr) {
  for (int64_t r = 0; r < h->n; ++r) {
    const int64_t owner = h->h_owner_ids.empty() ? r : h->h_owner_ids[r];
    o.put_id(owner);
    bool first = true;
    for (int32_t i = 0; i < cnt[r]; ++i) {
      const double v = sc[(size_t)r * k + i];
      if (v == 0.0 || v < thr) continue;  // not a non-zero of the similarity vector / below the threshold
      o.put(first ? "\t" : " ", 1);
      first = false;
      o.put_id(ids[(size_t)r * k + i]);
      o.put(":", 1);
      o.put_double(v);
    }
    o.put("\n", 1);
  }
  return CMS_OK;
}

int write_similarities(cms_handle* h, const char* path, int32_t k, int32_t format, double threshold) {
  std::vector<int64_t> ids;
  std::vector<double> sc;
  std::vector<int32_t> cnt;
  int rc = host_lists(h, k, ids, sc, cnt);
  if (rc) return rc;
  OutBuf o;
  o.f = std::fopen(path, "wb");
  if (!o.f) return set_error(CMS_E_PARAM, "cannot open %s for writing", path);
  o.buf.reserve(1 << 22);
  rc = format == CMS_FORMAT_ITEM_SIMILARITY_JOB ? write_item_similarity_job(h, o, k, ids, sc, cnt, threshold)
                                                : write_spark_itemsimilarity(h, o, k, ids, sc, cnt, threshold);
  o.flush();
  const bool closed = std::fclose(o.f) == 0;
  if (rc) return rc;
  if (!o.ok || !closed) return set_error(CMS_E_PARAM, "short write to %s", path);
  return CMS_OK;
}

int write_similar_items(cms_handle* h, const char* path, int32_t k, int32_t as_float) {
  const int64_t n = h->n;
  DevBuf o_ids, o_sc, o_cnt;
  CMS_HIP(o_ids.ensure(sizeof(int64_t) * n * k));
  CMS_HIP(o_sc.ensure(sizeof(double) * n * k));
  CMS_HIP(o_cnt.ensure(sizeof(int32_t) * n));
  int rc = top_k_all(h, k, o_ids.as<int64_t>(), o_sc.as<double>(), o_cnt.as<int32_t>());
  if (rc) return rc;
  std::vector<int64_t> ids((size_t)n * k);
  std::vector<double> sc((size_t)n * k);
  std::vector<int32_t> cnt(n);
  CMS_HIP(hipMemcpyAsync(ids.data(), o_ids.ptr, sizeof(int64_t) * n * k, hipMemcpyDeviceToHost, h->stream));
  CMS_HIP(hipMemcpyAsync(sc.data(), o_sc.ptr, sizeof(double) * n * k, hipMemcpyDeviceToHost, h->stream));
  CMS_HIP(hipMemcpyAsync(cnt.data(), o_cnt.ptr, sizeof(int32_t) * n, hipMemcpyDeviceToHost, h->stream));
  CMS_HIP(hipStreamSynchronize(h->stream));
  FILE* f = std::fopen(path, "wb");
  if (!f) return set_error(CMS_E_PARAM, "cannot open %s for writing", path);
  std::vector<char> buf;
  buf.reserve(1 << 22);
  char num[64];
  for (int64_t r = 0; r < n; ++r) {
    const int64_t owner = h->h_owner_ids.empty() ? r : h->h_owner_ids[r];
    for (int32_t i = 0; i < cnt[r]; ++i) {
      double v = sc[(size_t)r * k + i];
      if (as_float) v = (double)(float)v;
      int len = std::snprintf(num, sizeof(num), "%lld,%lld,", (long long)owner, (long long)ids[(size_t)r * k + i]);
      buf.insert(buf.end(), num, num + len);
      len = java_double_to_string(v, num, sizeof(num));
      buf.insert(buf.end(), num, num + len);
      buf.push_back('\n');
      if (buf.size() > (1u << 22)) {
        if (std::fwrite(buf.data(), 1, buf.size(), f) != buf.size()) {
          std::fclose(f);
          return set_error(CMS_E_PARAM, "short write to %s", path);
        }
        buf.clear();
      }
    }
  }
  bool ok = std::fwrite(buf.data(), 1, buf.size(), f) == buf.size();
  ok = (std::fclose(f) == 0) && ok;
  if (!ok) return set_error(CMS_E_PARAM, "short write to %s", path);
  return CMS_OK;
}

}  // namespace cms
