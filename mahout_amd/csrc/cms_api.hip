// cms_api.hip -- extern "C" entry points of libmahout_cms.so (see
// include/mahout_cms.h for the reference interface each one replaces).
#include <hip/hip_runtime.h>

#include <atomic>
#include <chrono>
#include <rccl/rccl.h>

#include <algorithm>
#include <thread>
#include <cmath>
#include <cstdarg>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <new>
#include <vector>

#include "cms_internal.h"

namespace cms {

static thread_local char g_err[512] = "";

int set_error(int code, const char* fmt, ...) {
  va_list ap;
  va_start(ap, fmt);
  vsnprintf(g_err, sizeof(g_err), fmt, ap);
  va_end(ap);
  return code;
}

int hip_fail(hipError_t e, const char* what) {
  if (e == hipErrorOutOfMemory) return set_error(CMS_E_OOM, "out of device memory in %s", what);
  return set_error(CMS_E_HIP, "%s failed: %s", what, hipGetErrorString(e));
}

// host time spent in device allocations (process-wide; cms_get_timing's
// "host_alloc" scope): a first all-pairs job allocates its operand images and
// candidate lists, tens of GB at config 4
static std::atomic<int64_t> g_alloc_ns{0}, g_alloc_calls{0}, g_free_ns{0}, g_alloc_bytes{0}, g_alloc_max_ns{0},
    g_alloc_max_bytes{0};

static int64_t ns_since(std::chrono::steady_clock::time_point t0) {
  return std::chrono::duration_cast<std::chrono::nanoseconds>(std::chrono::steady_clock::now() - t0).count();
}

hipError_t DevBuf::ensure(size_t need) {
  if (need <= bytes && ptr) return hipSuccess;
  if (ptr) {  // hipFree waits for the device's queued work: timed apart from the allocation
    const auto t0 = std::chrono::steady_clock::now();
    hipError_t e = hipFree(ptr);
    g_free_ns += ns_since(t0);
    if (e != hipSuccess) return e;
    ptr = nullptr;
    bytes = 0;
  }
  size_t alloc = std::max<size_t>(need, 256);
  const auto t0 = std::chrono::steady_clock::now();
  hipError_t e = hipMalloc(&ptr, alloc);
  const int64_t dt = ns_since(t0);
  g_alloc_ns += dt;
  if (dt > g_alloc_max_ns.load()) {  // the slowest single allocation (diagnostic; races only blur it)
    g_alloc_max_ns = dt;
    g_alloc_max_bytes = (int64_t)alloc;
  }
  ++g_alloc_calls;
  if (e == hipSuccess) {
    bytes = alloc;
    g_alloc_bytes += (int64_t)alloc;
  }
  return e;
}

void DevBuf::release() {
  if (ptr) (void)hipFree(ptr);
  ptr = nullptr;
  bytes = 0;
}

// Phase scopes of the ingest step whose events are recorded only at timing
// level 2: every timing event is a marker in the stream that costs the GPU a
// few microseconds, so the timed bench steps (level 1) bracket the roofline
// kernels alone.
static bool fine_scope(const char* nm) {
  static const char* const kFine[] = {"partition", "build_plan", "hot_norms", "norms", "reduce_hot",
                                      "merge_bounds", "merge_pack", "merge_unpack"};
  for (const char* f : kFine)
    if (!strcmp(nm, f)) return true;
  return false;
}

static hipEvent_t pooled_event(cms_handle* h) {
  hipEvent_t e = nullptr;
  if (!h->event_pool.empty()) {
    e = h->event_pool.back();
    h->event_pool.pop_back();
  } else if (hipEventCreate(&e) != hipSuccess) {
    e = nullptr;
  }
  return e;
}

TimedScope::TimedScope(cms_handle* hh, const char* nm, bool on) : h(hh), name(nm) {
  if (on && h->timing >= (fine_scope(nm) ? 2 : 1)) {
    start = pooled_event(h);
    if (start) (void)hipEventRecord(start, h->stream);
  }
}

TimedScope::~TimedScope() {
  if (!start) return;
  hipEvent_t stop = pooled_event(h);
  if (!stop) return;
  (void)hipEventRecord(stop, h->stream);
  h->pending.push_back(PendingEvent{name, start, stop});
}

// java.util.Random restated for HashFunctionBuilder (HashFunctionBuilder.java:23-61):
// (a_i, b_i) = (Math.abs(nextLong()), Math.abs(nextLong())) for i = 0..d-1.
static void java_hash_params(int64_t seed, int depth, int64_t* a, int64_t* b) {
  const uint64_t mult = 0x5DEECE66DULL, add = 0xBULL, mask = (1ULL << 48) - 1;
  uint64_t s = ((uint64_t)seed ^ mult) & mask;
  auto next32 = [&]() -> int64_t {
    s = (s * mult + add) & mask;
    return (int64_t)(int32_t)(uint32_t)(s >> 16);
  };
  auto next_long = [&]() -> int64_t {
    int64_t hi = next32();
    int64_t lo = next32();
    return (int64_t)((uint64_t)hi << 32) + lo;
  };
  auto jabs = [](int64_t v) -> int64_t { return v < 0 ? (int64_t)(0 - (uint64_t)v) : v; };
  for (int i = 0; i < depth; ++i) {
    a[i] = jabs(next_long());
    b[i] = jabs(next_long());
  }
}

static int flags_error(cms_handle* h, uint32_t f, bool by_id);

static int check_flags(cms_handle* h, bool by_id) {
  uint32_t f = 0;
  CMS_HIP(hipMemcpy(&f, h->d_flags, sizeof(uint32_t), hipMemcpyDeviceToHost));
  return flags_error(h, f, by_id);
}

// error flags word f (already read back): clear it on the device and report
static int flags_error(cms_handle* h, uint32_t f, bool by_id) {
  if (f == 0) return CMS_OK;
  CMS_HIP(hipMemset(h->d_flags, 0, sizeof(uint32_t)));
  if (f & kFlagBadRow)
    return by_id ? set_error(CMS_E_NO_SUCH_ID, "owner ID not in the owner universe")
                 : set_error(CMS_E_PARAM, "owner row outside [0, num_owners)");
  if (f & kFlagBadValue) return set_error(CMS_E_VALUE, "u32 counters need non-negative integer increments");
  return set_error(CMS_E_OVERFLOW, "a row's total increment reached 2^32 (u32 counters)");
}

static int resolve_timing(cms_handle* h) {
  for (auto& pe : h->pending) {
    float ms = 0.f;
    CMS_HIP(hipEventSynchronize(pe.stop));
    CMS_HIP(hipEventElapsedTime(&ms, pe.start, pe.stop));
    auto& acc = h->timing_acc[pe.name];
    acc.total_ms += ms;
    acc.launches += 1;
    h->event_pool.push_back(pe.start);
    h->event_pool.push_back(pe.stop);
  }
  h->pending.clear();
  return CMS_OK;
}

static int row_of(cms_handle* h, int64_t id, int64_t* row) {
  if (h->h_owner_ids.empty()) {
    if (id < 0 || id >= h->n) return set_error(CMS_E_NO_SUCH_ID, "no such owner ID %lld", (long long)id);
    *row = id;
    return CMS_OK;
  }
  auto it = std::lower_bound(h->h_owner_ids.begin(), h->h_owner_ids.end(), id);
  if (it == h->h_owner_ids.end() || *it != id) return set_error(CMS_E_NO_SUCH_ID, "no such owner ID %lld", (long long)id);
  *row = it - h->h_owner_ids.begin();
  return CMS_OK;
}

struct Guard {
  cms_handle* h;
  explicit Guard(cms_handle* hh) : h(hh) {
    h->mu.lock();
    (void)hipSetDevice(h->device);
  }
  ~Guard() { h->mu.unlock(); }
};

// Point queries after cms_finalize: shared with each other, exclusive of writers.
struct SharedGuard {
  cms_handle* h;
  explicit SharedGuard(cms_handle* hh) : h(hh) {
    h->mu.lock_shared();
    (void)hipSetDevice(h->device);
  }
  ~SharedGuard() { h->mu.unlock_shared(); }
};

// A query context (stream + scratch) leased from the handle's pool for one call.
struct CtxLease {
  cms_handle* h;
  QueryCtx* c = nullptr;
  explicit CtxLease(cms_handle* hh) : h(hh) {
    std::lock_guard<std::mutex> g(h->pool_mu);
    if (!h->qpool.empty()) {
      c = h->qpool.back();
      h->qpool.pop_back();
    }
  }
  int ready() {
    if (c) return CMS_OK;
    c = new (std::nothrow) QueryCtx();
    if (!c) return set_error(CMS_E_OOM, "host allocation failed");
    CMS_HIP(hipStreamCreateWithFlags(&c->stream, hipStreamNonBlocking));
    return CMS_OK;
  }
  ~CtxLease() {
    if (!c) return;
    std::lock_guard<std::mutex> g(h->pool_mu);
    h->qpool.push_back(c);
  }
};

static void free_query_pool(cms_handle* h) {
  for (QueryCtx* c : h->qpool) {
    if (c->stream) (void)hipStreamDestroy(c->stream);
    delete c;
  }
  h->qpool.clear();
}

static int refuse_per_owner(cms_handle* h, const char* what) {
  if (h->per_owner)
    return set_error(CMS_E_STATE, "%s: not available on a per-owner-shape handle (cms_create_per_owner)", what);
  return CMS_OK;
}

static int require_finalized(cms_handle* h) {
  if (!h->finalized) return set_error(CMS_E_STATE, "call cms_finalize before queries");
  return CMS_OK;
}

int coll_allreduce_u64(cms_handle* h, uint64_t* d_buf, int64_t count) {
  if (count <= 0) return CMS_OK;
  ++h->coll_calls;
  if (h->ext_comm) {
    CMS_HIP(hipStreamSynchronize(h->stream));
    const int r = h->x_allreduce(d_buf, count, h->x_user);
    if (r != 0) return set_error(CMS_E_RCCL, "caller all-reduce returned %d", r);
    return CMS_OK;
  }
  ncclResult_t r = ncclAllReduce(d_buf, d_buf, (size_t)count, ncclUint64, ncclSum, h->comm, h->stream);
  if (r != ncclSuccess) return set_error(CMS_E_RCCL, "ncclAllReduce: %s", ncclGetErrorString(r));
  return CMS_OK;
}

int coll_allgather(cms_handle* h, const void* d_send, void* d_recv, int64_t bytes) {
  if (bytes <= 0) return CMS_OK;
  ++h->coll_calls;
  if (h->ext_comm) {
    CMS_HIP(hipStreamSynchronize(h->stream));
    const int r = h->x_allgather(d_send, d_recv, bytes, h->x_user);
    if (r != 0) return set_error(CMS_E_RCCL, "caller all-gather returned %d", r);
    return CMS_OK;
  }
  ncclResult_t r = ncclAllGather(d_send, d_recv, (size_t)bytes, ncclUint8, h->comm, h->stream);
  if (r != ncclSuccess) return set_error(CMS_E_RCCL, "ncclAllGather: %s", ncclGetErrorString(r));
  return CMS_OK;
}

}  // namespace cms

using namespace cms;

extern "C" {

int cms_abi_version(void) { return CMS_ABI_VERSION; }

const char* cms_last_error(void) { return g_err; }

int cms_params_init(cms_params* p) {
  if (!p) return set_error(CMS_E_PARAM, "null params");
  std::memset(p, 0, sizeof(*p));
  p->struct_size = sizeof(cms_params);
  p->depth = 5;
  p->width = 4096;
  p->counter_type = CMS_COUNTER_U32;
  p->seed = 42;
  p->num_owners = 0;
  p->weighting = CMS_UNWEIGHTED;
  p->device = -1;
  return CMS_OK;
}

int cms_shape_from_delta_epsilon(double delta, double epsilon, int32_t* width, int32_t* depth) {
  if (!width || !depth) return set_error(CMS_E_PARAM, "null output");
  if (delta <= 0 || delta > std::exp(-1.0))
    return set_error(CMS_E_PARAM, "CountMinSketch: delta must be between 0 and 1, exclusive");
  if (epsilon <= 0 || epsilon > std::exp(1.0))
    return set_error(CMS_E_PARAM, "CountMinSketch: epsilon must be between 0 and 1, exclusive");
  *width = (int32_t)std::ceil(std::exp(1.0) / epsilon);
  *depth = (int32_t)std::ceil(std::log(1.0 / delta));
  return CMS_OK;
}

static int create_impl(const cms_params* p, bool per_owner, cms_handle** out) {
  if (!p || !out) return set_error(CMS_E_PARAM, "null argument");
  if (p->struct_size != sizeof(cms_params)) return set_error(CMS_E_PARAM, "cms_params ABI mismatch");
  if (!per_owner) {
    if (p->depth < 1 || p->depth > CMS_MAX_DEPTH)
      return set_error(CMS_E_PARAM, "depth must be in [1, %d]", CMS_MAX_DEPTH);
    // u32 counters: LDS-staged sketch rows up to 32768 counters; fp64
    // counters (DoubleCountMinSketch's own type, any width the reference's
    // constructor takes) up to 2^20, rows past the LDS built in place
    const int32_t wmax = p->counter_type == CMS_COUNTER_F64 ? (1 << 20) : (1 << 15);
    if (p->width < 1 || p->width > wmax) return set_error(CMS_E_PARAM, "width must be in [1, %d]", wmax);
  }
  if (p->num_owners < 1 || p->num_owners > (int64_t(1) << 24))
    return set_error(CMS_E_PARAM, "num_owners must be in [1, 2^24]");
  if (p->counter_type != CMS_COUNTER_U32 && p->counter_type != CMS_COUNTER_F64)
    return set_error(CMS_E_PARAM, "unsupported counter type");
  const bool f64 = p->counter_type == CMS_COUNTER_F64;
  if (p->frac_bits < 0 || p->frac_bits > 31) return set_error(CMS_E_PARAM, "frac_bits must be in [0, 31]");
  if (p->flags & ~CMS_FLAG_COLLECTIVE_SINGLE_RANK) return set_error(CMS_E_PARAM, "unknown flags 0x%x", p->flags);
  if (f64 && (p->flags & CMS_FLAG_COLLECTIVE_SINGLE_RANK))
    return set_error(CMS_E_PARAM, "fp64 counters are single-GPU: no collective path");
  cms_handle* h = new (std::nothrow) cms_handle();
  if (!h) return set_error(CMS_E_OOM, "host allocation failed");
  h->p = *p;
  {  // tunables: the environment is read here and nowhere else
    auto flag = [](const char* name) { const char* e = getenv(name); return e && *e && std::strcmp(e, "0") != 0; };
    auto num = [](const char* name, int dflt) { const char* e = getenv(name); return e && *e ? atoi(e) : dflt; };
    h->tune.bit_keys = num("CMS_BIT_KEYS", h->tune.bit_keys);
    h->tune.crumb_keys = num("CMS_CRUMB_KEYS", h->tune.crumb_keys);
    h->tune.list_keys = std::max(0, std::min(256, num("CMS_LIST_KEYS", h->tune.list_keys)));
    h->tune.mid_u4_keys = num("CMS_MID_U4_KEYS", h->tune.mid_u4_keys);
    h->tune.mid_u8_keys = num("CMS_MID_U8_KEYS", h->tune.mid_u8_keys);
    h->tune.mid_u8_image = num("CMS_MID_U8_IMAGE", h->tune.mid_u8_image);
    h->tune.nib_persist = num("CMS_NIB_PERSIST", h->tune.nib_persist);
    h->tune.mid_image = num("CMS_MID_IMAGE", h->tune.mid_image);
    h->tune.build_streams = num("CMS_BUILD_STREAMS", h->tune.build_streams);
    h->tune.plan_side = num("CMS_PLAN_SIDE", h->tune.plan_side);
    h->tune.slice_reduce = num("CMS_SLICE_REDUCE", h->tune.slice_reduce);
    h->tune.mid_waves = num("CMS_MID_WAVES", h->tune.mid_waves);
    h->tune.split_keys = num("CMS_SPLIT_KEYS", h->tune.split_keys);
    h->tune.mid_threads = num("CMS_MID_THREADS", h->tune.mid_threads);
    h->tune.nib_rows_once = num("CMS_NIB_ROWS_ONCE", h->tune.nib_rows_once);
    h->tune.po_no_prune = num("CMS_PO_NO_PRUNE", h->tune.po_no_prune);
    h->tune.po_bound_rows = num("CMS_PO_BOUND_ROWS", h->tune.po_bound_rows);
    h->tune.po_bound_part2 = num("CMS_PO_BOUND_PART2", h->tune.po_bound_part2);
    h->tune.po_dense_x4 = num("CMS_PO_DENSE_X4", h->tune.po_dense_x4);
    h->tune.po_no_bigq = num("CMS_PO_NO_BIGQ", h->tune.po_no_bigq);
    h->tune.forms = !flag("CMS_NO_FORMS");
    h->tune.no_compact = flag("CMS_NO_COMPACT");
    h->tune.no_vmm = flag("CMS_NO_VMM");
    h->tune.early_slices = flag("CMS_EARLY_SLICES") ? 1 : 0;
    h->tune.hot_routing = !flag("CMS_NO_HOT_ROUTING");
    h->tune.fp4 = !flag("CMS_NO_FP4");
    h->tune.mls = !flag("CMS_NO_MLS");
  }
  h->per_owner = per_owner;
  h->f64 = f64;
  if (f64) h->p.frac_bits = 0;  // raw (double) float preferences
  if (per_owner) {  // every owner may use up to CMS_MAX_DEPTH rows; no shared table
    h->p.depth = CMS_MAX_DEPTH;
    h->p.width = 1;
  }
  int dev = p->device;
  if (dev < 0) {
    if (hipGetDevice(&dev) != hipSuccess) dev = 0;
  }
  h->device = dev;
  hipError_t e = hipSetDevice(dev);
  if (e != hipSuccess) {
    delete h;
    return hip_fail(e, "hipSetDevice");
  }
  {
    int cus = 0;
    if (hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev) == hipSuccess && cus > 0)
      h->num_cus = cus;
  }
  h->n = p->num_owners;
  h->dw = (int64_t)p->depth * p->width;
  java_hash_params(p->seed, h->p.depth, h->a, h->b);
  HashParams& hp = h->hp;
  std::memset(&hp, 0, sizeof(hp));
  for (int i = 0; i < h->p.depth; ++i) {
    hp.ap[i] = reduce_key(h->a[i]);
    hp.bp[i] = reduce_key(h->b[i]);
  }
  hp.width = (uint32_t)h->p.width;
  hp.depth = h->p.depth;
  hp.frac_bits = p->frac_bits;
  hash_finish(hp);
  if (per_owner) h->dw = 0;

  size_t tbytes = sizeof(uint16_t) * (size_t)h->n * (size_t)h->dw;
  if ((e = hipStreamCreateWithFlags(&h->stream, hipStreamDefault)) != hipSuccess ||
      (e = hipStreamCreateWithFlags(&h->side_stream, hipStreamNonBlocking)) != hipSuccess ||
      (e = hipStreamCreateWithFlags(&h->side_stream2, hipStreamNonBlocking)) != hipSuccess ||
      (e = hipStreamCreateWithFlags(&h->side_stream3, hipStreamNonBlocking)) != hipSuccess ||
      (e = hipEventCreateWithFlags(&h->ev_p1, hipEventDisableTiming)) != hipSuccess ||
      (e = hipEventCreateWithFlags(&h->ev_e1, hipEventDisableTiming)) != hipSuccess ||
      (e = hipEventCreateWithFlags(&h->ev_early, hipEventDisableTiming)) != hipSuccess ||
      (e = hipEventCreateWithFlags(&h->ev_join3, hipEventDisableTiming)) != hipSuccess ||
      (e = hipEventCreateWithFlags(&h->ev_spans, hipEventDisableTiming)) != hipSuccess ||
      (e = hipEventCreateWithFlags(&h->ev_plan, hipEventDisableTiming)) != hipSuccess ||
      (e = hipEventCreateWithFlags(&h->ev_fork, hipEventDisableTiming)) != hipSuccess ||
      (e = hipEventCreateWithFlags(&h->ev_join, hipEventDisableTiming)) != hipSuccess ||
      (e = hipEventCreateWithFlags(&h->ev_fork2, hipEventDisableTiming)) != hipSuccess ||
      (e = hipEventCreateWithFlags(&h->ev_join2, hipEventDisableTiming)) != hipSuccess ||
#ifdef CMS_BUILD_GATHERHASH  // bound analysis only (cms_hash.h): the gathered table, contents unset
      (e = hipMalloc((void**)&h->hp.gtab, sizeof(uint4) << 24)) != hipSuccess ||
#endif
      (!per_owner && !f64 && (e = hipMalloc(&h->d_off, sizeof(int64_t) * h->n)) != hipSuccess) ||
      (f64 && (e = hipMalloc(&h->d_t64, 4 * tbytes)) != hipSuccess) ||
      (!per_owner && (e = hipMalloc(&h->d_hidx, sizeof(int32_t) * h->n)) != hipSuccess) ||
      (!per_owner && (e = hipMemset(h->d_hidx, 0xff, sizeof(int32_t) * h->n)) != hipSuccess) ||
      (!per_owner && !f64 && (e = hipMalloc(&h->d_cbound, sizeof(uint32_t) * h->n)) != hipSuccess) ||
      (e = hipMalloc(&h->d_row_mass, sizeof(uint64_t) * h->n)) != hipSuccess ||
      (!per_owner && (e = hipMalloc(&h->d_norm, sizeof(uint64_t) * h->n * p->depth)) != hipSuccess) ||
      (!per_owner && (e = hipMalloc(&h->d_norm_sqrt, sizeof(double) * h->n * p->depth)) != hipSuccess) ||
      (e = hipMalloc(&h->d_rowmax, sizeof(uint32_t) * h->n)) != hipSuccess ||
      (e = hipMalloc(&h->d_flags, 64 * sizeof(uint32_t))) != hipSuccess ||
      (e = hipHostMalloc((void**)&h->h_pin, 16 * sizeof(uint32_t), hipHostMallocDefault)) != hipSuccess ||
      (e = hipMemset(h->d_flags, 0, 64 * sizeof(uint32_t))) != hipSuccess ||
      (e = hipMemset(h->d_row_mass, 0, sizeof(uint64_t) * h->n)) != hipSuccess) {
    int rc = hip_fail(e, "cms_create allocation");
    cms_destroy(h);
    return rc;
  }
  h->empty = true;
  h->norms_valid = false;
  // u8 / nibble row forms need 64-B aligned slots and 16-B nibble rows
  // (the byte-class and mid kernels store whole 16-B words of a 4-bit sketch
  // row: w % 32 == 0)
  h->forms_ok = !per_owner && !f64 && h->p.width % 32 == 0 && h->tune.forms;
  // compact rows (cms_internal.h TableView) when the layout's 128-B units fit
  // the u32 scan; the arena then starts as the zero row alone
  h->compact = h->forms_ok && !h->tune.no_compact &&
               (double)h->n * (double)(slot_units(h->dw) / kRowAlign + 1) < 4.0e9;
  if (!per_owner && !f64) {
    if (int rc = init_row_offsets(h)) {
      cms_destroy(h);
      return rc;
    }
  }
  *out = h;
  return CMS_OK;
}

int cms_create(const cms_params* p, cms_handle** out) { return create_impl(p, false, out); }

int cms_create_per_owner(const cms_params* p, cms_handle** out) { return create_impl(p, true, out); }

void cms_destroy(cms_handle* h) {
  if (!h) return;
  (void)hipSetDevice(h->device);
  if (h->stream) (void)hipStreamSynchronize(h->stream);
  for (auto& pe : h->pending) {
    (void)hipEventDestroy(pe.start);
    (void)hipEventDestroy(pe.stop);
  }
  for (hipEvent_t e : h->event_pool) (void)hipEventDestroy(e);
  if (h->order_ev) (void)hipEventDestroy(h->order_ev);
  if (h->side_stream) (void)hipStreamSynchronize(h->side_stream);
  if (h->side_stream2) (void)hipStreamSynchronize(h->side_stream2);
  if (h->side_stream3) (void)hipStreamSynchronize(h->side_stream3);
  for (hipEvent_t ev : {h->ev_p1, h->ev_e1, h->ev_early})
    if (ev) (void)hipEventDestroy(ev);
  if (h->ev_join3) (void)hipEventDestroy(h->ev_join3);
  if (h->ev_spans) (void)hipEventDestroy(h->ev_spans);
  if (h->ev_plan) (void)hipEventDestroy(h->ev_plan);
  if (h->ev_fork) (void)hipEventDestroy(h->ev_fork);
  if (h->ev_join) (void)hipEventDestroy(h->ev_join);
  if (h->ev_fork2) (void)hipEventDestroy(h->ev_fork2);
  if (h->ev_join2) (void)hipEventDestroy(h->ev_join2);
  free_query_pool(h);
  if (h->comm) (void)ncclCommDestroy(h->comm);
  arena_release(h);
  void* bufs[] = {h->d_off, h->d_t64, h->d_hidx, h->d_cbound, h->d_row_mass, h->d_norm, h->d_norm_sqrt, h->d_rowmax, h->d_flags, h->d_owner_ids};
  for (void* b : bufs)
    if (b) (void)hipFree(b);
  if (h->h_pin) (void)hipHostFree(h->h_pin);
  DevBuf* ws[] = {&h->ws_in_row, &h->ws_in_key, &h->ws_in_val, &h->ws_p1_row, &h->ws_p1_key, &h->ws_p1_val,
                  &h->ws_csr_key, &h->ws_csr_val, &h->ws_csr_off, &h->ws_csr_hi, &h->ws_hotpart, &h->ws_hist, &h->ws_small, &h->ws_partials, &h->ws_slicepart,
                  &h->ws_hot, &h->ws_query, &h->ws_out, &h->ws_limb0, &h->ws_limbmeta, &h->ws_limbhot,
                  &h->ws_hotlist, &h->ws_tiles, &h->ws_slab, &h->ws_topq, &h->vl[0].buf, &h->vl[1].buf, &h->ws_nsq, &h->ws_cand,
                  &h->dlog_row, &h->dlog_key, &h->dlog_val, &h->dlog_cnt, &h->dlog_all, &h->ws_srow,
                  &h->ws_f4, &h->ws_i8blk, &h->po_off, &h->po_kp, &h->po_inc, &h->po_shape, &h->po_sk, &h->po_norm, &h->po_nsq,
                  &h->po_scratch, &h->po_wrows, &h->po_s0, &h->ws_pothr, &h->ws_posurv, &h->hot_tab, &h->ws_bound, &h->ws_force, &h->ws_plist, &h->ws_blist,
                  &h->ws_mbnd, &h->ws_mbits, &h->ws_mwoff, &h->ws_mpacked, &h->rf_ids, &h->rf_sc, &h->rf_cnt,
                  &h->rf_full, &h->rf_touch, &h->rf_new, &h->rf_redo, &h->rf_perm};
  for (DevBuf* b : ws) b->release();
  if (h->stream) (void)hipStreamDestroy(h->stream);
  if (h->side_stream) (void)hipStreamDestroy(h->side_stream);
  if (h->side_stream2) (void)hipStreamDestroy(h->side_stream2);
  if (h->side_stream3) (void)hipStreamDestroy(h->side_stream3);
  delete h;
}

int cms_set_owner_ids(cms_handle* h, const int64_t* ids, int64_t n) {
  if (!h || !ids) return set_error(CMS_E_PARAM, "null argument");
  Guard g(h);
  if (n != h->n) return set_error(CMS_E_PARAM, "expected %lld owner IDs, got %lld", (long long)h->n, (long long)n);
  for (int64_t i = 1; i < n; ++i)
    if (ids[i] <= ids[i - 1]) return set_error(CMS_E_PARAM, "owner IDs must be strictly ascending");
  h->h_owner_ids.assign(ids, ids + n);
  if (!h->d_owner_ids) CMS_HIP(hipMalloc(&h->d_owner_ids, sizeof(int64_t) * n));
  CMS_HIP(hipMemcpy(h->d_owner_ids, ids, sizeof(int64_t) * n, hipMemcpyHostToDevice));
  return CMS_OK;
}

int cms_hash_params(cms_handle* h, int64_t* a, int64_t* b) {
  if (!h || !a || !b) return set_error(CMS_E_PARAM, "null argument");
  for (int i = 0; i < h->p.depth; ++i) {
    a[i] = h->a[i];
    b[i] = h->b[i];
  }
  return CMS_OK;
}

int cms_set_hash_params(cms_handle* h, const int64_t* a, const int64_t* b, int32_t count) {
  if (!h || !a || !b) return set_error(CMS_E_PARAM, "null argument");
  Guard g(h);
  if (count != h->p.depth)
    return set_error(CMS_E_PARAM, "expected %d (a, b) pairs, got %d", (int)h->p.depth, (int)count);
  if (!h->empty || h->pairs_ingested != 0 || h->po_loaded)
    return set_error(CMS_E_STATE, "hash parameters must be set before the first ingest (or after cms_reset)");
  for (int i = 0; i < count; ++i) {
    h->a[i] = a[i];
    h->b[i] = b[i];
    h->hp.ap[i] = reduce_key(a[i]);  // any int64, as BigInteger.valueOf(a).mod(p) takes it
    h->hp.bp[i] = reduce_key(b[i]);
  }
  hash_finish(h->hp);
  return CMS_OK;
}

int cms_hash_keys(cms_handle* h, const int64_t* keys, int64_t n, int32_t* out) {
  if (!h || (n > 0 && (!keys || !out))) return set_error(CMS_E_PARAM, "null argument");
  if (int rc0 = refuse_per_owner(h, "cms_hash_keys")) return rc0;
  if (n <= 0) return CMS_OK;
  Guard g(h);
  CMS_HIP(h->ws_in_key.ensure(sizeof(int64_t) * n));
  CMS_HIP(h->ws_out.ensure(sizeof(int32_t) * n * h->p.depth));
  CMS_HIP(hipMemcpyAsync(h->ws_in_key.ptr, keys, sizeof(int64_t) * n, hipMemcpyHostToDevice, h->stream));
  int rc = hash_keys_device(h, h->ws_in_key.as<int64_t>(), n, h->ws_out.as<int32_t>());
  if (rc) return rc;
  CMS_HIP(hipMemcpyAsync(out, h->ws_out.ptr, sizeof(int32_t) * n * h->p.depth, hipMemcpyDeviceToHost, h->stream));
  CMS_HIP(hipStreamSynchronize(h->stream));
  return CMS_OK;
}

namespace {

// Delta log of a merged multi-rank handle (cms_internal.h).  Grows by copy.
int dlog_reserve(cms_handle* h, int64_t need) {
  if (need <= h->dlog_cap) return CMS_OK;
  const int64_t cap = std::max<int64_t>({need, 2 * h->dlog_cap, int64_t(1) << 16});
  cms::DevBuf nr, nk, nv;
  CMS_HIP(nr.ensure(sizeof(int64_t) * cap));
  CMS_HIP(nk.ensure(sizeof(int64_t) * cap));
  CMS_HIP(nv.ensure(sizeof(float) * cap));
  if (h->dlog_n > 0) {
    CMS_HIP(hipMemcpyAsync(nr.ptr, h->dlog_row.ptr, sizeof(int64_t) * h->dlog_n, hipMemcpyDeviceToDevice, h->stream));
    CMS_HIP(hipMemcpyAsync(nk.ptr, h->dlog_key.ptr, sizeof(int64_t) * h->dlog_n, hipMemcpyDeviceToDevice, h->stream));
    CMS_HIP(hipMemcpyAsync(nv.ptr, h->dlog_val.ptr, sizeof(float) * h->dlog_n, hipMemcpyDeviceToDevice, h->stream));
  }
  CMS_HIP(hipStreamSynchronize(h->stream));
  h->dlog_row.release();
  h->dlog_key.release();
  h->dlog_val.release();
  std::swap(h->dlog_row, nr);
  std::swap(h->dlog_key, nk);
  std::swap(h->dlog_val, nv);
  h->dlog_cap = cap;
  return CMS_OK;
}

// Log a batch (rows already resolved) that went into a merged multi-rank table.
int dlog_append(cms_handle* h, const int64_t* d_row, const int64_t* d_key, const float* d_val, int64_t n) {
  if (!(h->merged && h->multi()) || n <= 0) return CMS_OK;
  int rc = dlog_reserve(h, h->dlog_n + n);
  if (rc) return rc;
  const int64_t o = h->dlog_n;
  CMS_HIP(hipMemcpyAsync(h->dlog_row.as<int64_t>() + o, d_row, sizeof(int64_t) * n, hipMemcpyDeviceToDevice, h->stream));
  CMS_HIP(hipMemcpyAsync(h->dlog_key.as<int64_t>() + o, d_key, sizeof(int64_t) * n, hipMemcpyDeviceToDevice, h->stream));
  if (d_val)
    CMS_HIP(hipMemcpyAsync(h->dlog_val.as<float>() + o, d_val, sizeof(float) * n, hipMemcpyDeviceToDevice, h->stream));
  else
    CMS_HIP(hipMemsetD32Async((hipDeviceptr_t)(h->dlog_val.as<float>() + o), 0x3F800000u, (size_t)n, h->stream));
  h->dlog_n += n;
  return CMS_OK;
}

// Exchange the logs of every rank and apply the other ranks' batches.
int dlog_exchange(cms_handle* h) {
  const int G = h->world;
  CMS_HIP(h->dlog_cnt.ensure(sizeof(int64_t) * (G + 1)));
  int64_t* cnt = h->dlog_cnt.as<int64_t>();
  CMS_HIP(hipMemcpyAsync(cnt, &h->dlog_n, sizeof(int64_t), hipMemcpyHostToDevice, h->stream));
  int rc = coll_allgather(h, cnt, cnt + 1, sizeof(int64_t));
  if (rc) return rc;
  std::vector<int64_t> counts(G);
  CMS_HIP(hipMemcpyAsync(counts.data(), cnt + 1, sizeof(int64_t) * G, hipMemcpyDeviceToHost, h->stream));
  CMS_HIP(hipStreamSynchronize(h->stream));
  const int64_t m = *std::max_element(counts.begin(), counts.end());
  if (m == 0) return CMS_OK;
  rc = dlog_reserve(h, m);  // the send buffers are read to length m
  if (rc) return rc;
  const size_t per = sizeof(int64_t) * 2 + sizeof(float);
  CMS_HIP(h->dlog_all.ensure(per * (size_t)G * (size_t)m));
  int64_t* g_row = h->dlog_all.as<int64_t>();
  int64_t* g_key = g_row + (size_t)G * m;
  float* g_val = reinterpret_cast<float*>(g_key + (size_t)G * m);
  if ((rc = coll_allgather(h, h->dlog_row.ptr, g_row, (int64_t)sizeof(int64_t) * m)) ||
      (rc = coll_allgather(h, h->dlog_key.ptr, g_key, (int64_t)sizeof(int64_t) * m)) ||
      (rc = coll_allgather(h, h->dlog_val.ptr, g_val, (int64_t)sizeof(float) * m)))
    return rc;
  for (int q = 0; q < G; ++q) {
    if (q == h->rank || counts[q] == 0) continue;
    const size_t o = (size_t)q * m;
    if ((rc = ingest_coo_device(h, g_row + o, g_key + o, g_val + o, counts[q]))) return rc;
  }
  h->dlog_n = 0;
  return CMS_OK;
}

}  // namespace

int cms_ingest(cms_handle* h, const int64_t* owner, const int64_t* key, const float* val, int64_t n) {
  if (h && h->ext_merged)
    return set_error(CMS_E_STATE, "table merged through cms_finalize_with: cms_reset starts a new epoch");
  if (!h || (n > 0 && (!owner || !key))) return set_error(CMS_E_PARAM, "null argument");
  if (int rc0 = refuse_per_owner(h, "COO ingest (per-owner mode takes the DataModel as CSR)")) return rc0;
  if (n <= 0) return CMS_OK;
  Guard g(h);
  if (h->f64) return f64_ingest_coo_host(h, owner, key, val, n);
  CMS_HIP(h->ws_in_row.ensure(sizeof(int64_t) * n));
  CMS_HIP(h->ws_in_key.ensure(sizeof(int64_t) * n));
  if (val) CMS_HIP(h->ws_in_val.ensure(sizeof(float) * n));
  int64_t* d_row = h->ws_in_row.as<int64_t>();
  CMS_HIP(hipMemcpyAsync(d_row, owner, sizeof(int64_t) * n, hipMemcpyHostToDevice, h->stream));
  CMS_HIP(hipMemcpyAsync(h->ws_in_key.ptr, key, sizeof(int64_t) * n, hipMemcpyHostToDevice, h->stream));
  if (val) CMS_HIP(hipMemcpyAsync(h->ws_in_val.ptr, val, sizeof(float) * n, hipMemcpyHostToDevice, h->stream));
  const bool by_id = !h->h_owner_ids.empty();
  int rc;
  if (by_id) {
    rc = map_owner_ids(h, d_row, n, d_row);  // in place: each thread reads then writes its own slot
    if (rc) return rc;
  }
  // all-or-nothing: reject unknown owners / bad increments before touching the table
  if ((rc = validate_batch(h, by_id ? nullptr : d_row, val ? h->ws_in_val.as<float>() : nullptr, n))) return rc;
  CMS_HIP(hipStreamSynchronize(h->stream));
  if ((rc = check_flags(h, by_id))) return rc;
  rc = ingest_coo_device(h, d_row, h->ws_in_key.as<int64_t>(), val ? h->ws_in_val.as<float>() : nullptr, n);
  if (rc) return rc;
  if ((rc = dlog_append(h, d_row, h->ws_in_key.as<int64_t>(), val ? h->ws_in_val.as<float>() : nullptr, n))) return rc;
  CMS_HIP(hipStreamSynchronize(h->stream));
  h->finalized = false;
  rc = check_flags(h, by_id);
  if (rc == CMS_OK) h->pairs_ingested += n;
  return rc;
}

int cms_ingest_device_rows(cms_handle* h, const int64_t* d_row, const int64_t* d_key, const float* d_val, int64_t n) {
  if (h && h->ext_merged)
    return set_error(CMS_E_STATE, "table merged through cms_finalize_with: cms_reset starts a new epoch");
  if (!h || (n > 0 && (!d_row || !d_key))) return set_error(CMS_E_PARAM, "null argument");
  if (int rc0 = refuse_per_owner(h, "COO ingest (per-owner mode takes the DataModel as CSR)")) return rc0;
  if (n <= 0) return CMS_OK;
  Guard g(h);
  if (h->f64)
    return set_error(CMS_E_STATE, "fp64 counters take the owners' order from CSR or host COO ingest, not from an "
                                  "unordered device stream");
  int rc = ingest_coo_device(h, d_row, d_key, d_val, n);
  if (rc == CMS_OK) rc = dlog_append(h, d_row, d_key, d_val, n);
  if (rc == CMS_OK) {
    h->pairs_ingested += n;
    h->finalized = false;
  }
  return rc;
}

int cms_ingest_csr(cms_handle* h, const int64_t* offsets, const int64_t* keys, const float* vals) {
  if (h && h->ext_merged)
    return set_error(CMS_E_STATE, "table merged through cms_finalize_with: cms_reset starts a new epoch");
  if (!h || !offsets) return set_error(CMS_E_PARAM, "null argument");
  const int64_t n = h->n;
  if (offsets[0] != 0) return set_error(CMS_E_PARAM, "offsets[0] must be 0");
  for (int64_t r = 0; r < n; ++r)
    if (offsets[r + 1] < offsets[r]) return set_error(CMS_E_PARAM, "offsets must be non-decreasing");
  const int64_t np = offsets[n];
  if (np > 0 && !keys) return set_error(CMS_E_PARAM, "null keys");
  Guard g(h);
  if (h->merged && h->multi())
    return set_error(CMS_E_STATE, "CSR bulk ingest into a merged multi-rank table: cms_reset first, or use COO ingest");
  CMS_HIP(h->ws_in_row.ensure(sizeof(int64_t) * (n + 1)));
  CMS_HIP(h->ws_in_key.ensure(sizeof(int64_t) * std::max<int64_t>(np, 1)));
  if (vals) CMS_HIP(h->ws_in_val.ensure(sizeof(float) * std::max<int64_t>(np, 1)));
  CMS_HIP(hipMemcpyAsync(h->ws_in_row.ptr, offsets, sizeof(int64_t) * (n + 1), hipMemcpyHostToDevice, h->stream));
  if (np > 0)
    CMS_HIP(hipMemcpyAsync(h->ws_in_key.ptr, keys, sizeof(int64_t) * np, hipMemcpyHostToDevice, h->stream));
  if (vals && np > 0)
    CMS_HIP(hipMemcpyAsync(h->ws_in_val.ptr, vals, sizeof(float) * np, hipMemcpyHostToDevice, h->stream));
  int rc;
  if (h->per_owner) {  // the DataModel itself stays resident; sketches are built at finalize
    rc = po_load_csr(h, h->ws_in_row.as<int64_t>(), h->ws_in_key.as<int64_t>(), vals ? h->ws_in_val.as<float>() : nullptr,
                     np, offsets);
    if (rc) return rc;
    CMS_HIP(hipStreamSynchronize(h->stream));
    if ((rc = check_flags(h, false))) {
      h->po_loaded = false;
      return rc;
    }
    h->pairs_ingested = np;
    return CMS_OK;
  }
  if (h->f64) {  // any float preference; the CSR order is the update order
    if ((rc = f64_ingest_csr(h, h->ws_in_row.as<int64_t>(), h->ws_in_key.as<int64_t>(),
                             vals ? h->ws_in_val.as<float>() : nullptr)))
      return rc;
    CMS_HIP(hipStreamSynchronize(h->stream));
    h->finalized = false;
    h->pairs_ingested += np;
    return CMS_OK;
  }
  if (vals && (rc = validate_batch(h, nullptr, h->ws_in_val.as<float>(), np))) return rc;
  CMS_HIP(hipStreamSynchronize(h->stream));
  if ((rc = check_flags(h, false))) return rc;
  rc = ingest_csr_device(h, h->ws_in_row.as<int64_t>(), h->ws_in_key.as<int64_t>(),
                         vals ? h->ws_in_val.as<float>() : nullptr, np);
  if (rc) return rc;
  CMS_HIP(hipStreamSynchronize(h->stream));
  h->finalized = false;
  rc = check_flags(h, false);
  if (rc == CMS_OK) h->pairs_ingested += np;
  return rc;
}

int cms_ingest_csr_device(cms_handle* h, const int64_t* d_offsets, const int64_t* d_keys, const float* d_vals) {
  if (h && h->ext_merged)
    return set_error(CMS_E_STATE, "table merged through cms_finalize_with: cms_reset starts a new epoch");
  if (!h || !d_offsets) return set_error(CMS_E_PARAM, "null argument");
  Guard g(h);
  if (h->merged && h->multi())
    return set_error(CMS_E_STATE, "CSR bulk ingest into a merged multi-rank table: cms_reset first, or use COO ingest");
  int64_t np = 0;
  if (!h->per_owner) {  // the build reads keys[offsets[r] .. offsets[r+1]): check the offsets first
    int rc0 = check_offsets_device(h, d_offsets);
    if (rc0) return rc0;
  }
  CMS_HIP(hipMemcpyAsync(&np, d_offsets + h->n, sizeof(int64_t), hipMemcpyDeviceToHost, h->stream));
  CMS_HIP(hipStreamSynchronize(h->stream));
  if (!h->per_owner) {
    if (int rc0 = check_flags(h, false)) return set_error(rc0, "CSR offsets must start at 0 and be non-decreasing");
  }
  if (h->per_owner) {
    std::vector<int64_t> off(h->n + 1);
    CMS_HIP(hipMemcpy(off.data(), d_offsets, sizeof(int64_t) * (h->n + 1), hipMemcpyDeviceToHost));
    if (off[0] != 0) return set_error(CMS_E_PARAM, "offsets[0] must be 0");
    for (int64_t r = 0; r < h->n; ++r)
      if (off[r + 1] < off[r]) return set_error(CMS_E_PARAM, "offsets must be non-decreasing");
    int rc = po_load_csr(h, d_offsets, d_keys, d_vals, np, off.data());
    if (rc) return rc;
    CMS_HIP(hipStreamSynchronize(h->stream));
    if ((rc = check_flags(h, false))) {
      h->po_loaded = false;
      return rc;
    }
    h->pairs_ingested = np;
    return CMS_OK;
  }
  h->rf_valid = false;  // CSR ingest does not mark touched owners: the next refresh is a full job
  int rc = h->f64 ? f64_ingest_csr(h, d_offsets, d_keys, d_vals) : ingest_csr_device(h, d_offsets, d_keys, d_vals, np);
  if (rc == CMS_OK) {
    h->pairs_ingested += np;
    h->finalized = false;
  }
  return rc;
}

int cms_reset(cms_handle* h) {
  if (!h) return set_error(CMS_E_PARAM, "null handle");
  Guard g(h);
  h->po_loaded = false;
  CMS_HIP(hipMemsetAsync(h->d_row_mass, 0, sizeof(uint64_t) * h->n, h->stream));
  h->empty = true;
  h->norms_valid = false;
  h->finalized = false;
  h->pairs_ingested = 0;
  h->merged = false;
  h->ext_merged = false;
  h->dlog_n = 0;
  h->rf_valid = false;
  return CMS_OK;
}

int cms_release_scratch(cms_handle* h) {
  if (!h) return set_error(CMS_E_PARAM, "null handle");
  Guard g(h);
  CMS_HIP(hipStreamSynchronize(h->stream));
  DevBuf* ws[] = {&h->ws_in_row, &h->ws_in_key, &h->ws_in_val, &h->ws_p1_row, &h->ws_p1_key, &h->ws_p1_val,
                  &h->ws_csr_key, &h->ws_csr_val, &h->ws_csr_off, &h->ws_csr_hi, &h->ws_hotpart, &h->ws_hist, &h->ws_hot, &h->ws_slicepart, &h->ws_query,
                  &h->ws_out, &h->ws_slab, &h->ws_topq, &h->ws_tiles, &h->ws_cand, &h->ws_srow,
                  &h->ws_mbnd, &h->ws_mbits, &h->ws_mwoff, &h->ws_mpacked, &h->rf_ids, &h->rf_sc, &h->rf_cnt,
                  &h->rf_full, &h->rf_touch, &h->rf_new, &h->rf_redo, &h->rf_perm};
  for (DevBuf* b : ws) b->release();
  // the kept refresh lists and touched marks are gone: the next COO ingest must not mark
  // into rf_touch, and the next cms_top_k_refresh is a whole job
  h->rf_valid = false;
  return CMS_OK;
}

int cms_comm_unique_id(void* out) {
  if (!out) return set_error(CMS_E_PARAM, "null argument");
  ncclUniqueId id;
  ncclResult_t r = ncclGetUniqueId(&id);
  if (r != ncclSuccess) return set_error(CMS_E_RCCL, "ncclGetUniqueId: %s", ncclGetErrorString(r));
  static_assert(sizeof(ncclUniqueId) == 128, "ncclUniqueId size");
  std::memcpy(out, &id, sizeof(id));
  return CMS_OK;
}

int cms_comm_init(cms_handle* h, const void* unique_id, int32_t rank, int32_t world) {
  if (!h || !unique_id) return set_error(CMS_E_PARAM, "null argument");
  if (world < 1 || rank < 0 || rank >= world) return set_error(CMS_E_PARAM, "bad rank/world");
  if (h->f64 && world > 1)
    return set_error(CMS_E_STATE, "fp64 counters are single-GPU: shard sums would not round in the reference's order");
  Guard g(h);
  if (h->comm) {
    (void)ncclCommDestroy(h->comm);
    h->comm = nullptr;
  }
  h->ext_comm = false;
  h->rank = rank;
  h->world = world;
  if (world == 1 && !(h->p.flags & CMS_FLAG_COLLECTIVE_SINGLE_RANK)) return CMS_OK;  // detached: single-GPU path
  ncclUniqueId id;
  std::memcpy(&id, unique_id, sizeof(id));
  ncclResult_t r = ncclCommInitRank(&h->comm, world, id, rank);
  if (r != ncclSuccess) return set_error(CMS_E_RCCL, "ncclCommInitRank: %s", ncclGetErrorString(r));
  return CMS_OK;
}

int cms_comm_init_transport(cms_handle* h, int32_t rank, int32_t world, cms_allreduce_fn allreduce,
                            cms_allgather_fn allgather, void* user) {
  if (!h) return set_error(CMS_E_PARAM, "null handle");
  if (world < 1 || rank < 0 || rank >= world) return set_error(CMS_E_PARAM, "bad rank/world");
  // every argument check precedes any state change: a rejected call leaves
  // the handle's communicator, rank and world as they were
  if ((world > 1 || (h->p.flags & CMS_FLAG_COLLECTIVE_SINGLE_RANK)) && (!allreduce || !allgather))
    return set_error(CMS_E_PARAM, "null transport function");
  if (h->f64 && world > 1)
    return set_error(CMS_E_STATE, "fp64 counters are single-GPU: shard sums would not round in the reference's order");
  Guard g(h);
  if (h->comm) {
    (void)ncclCommDestroy(h->comm);
    h->comm = nullptr;
  }
  h->rank = world > 1 ? rank : 0;
  h->world = world;
  h->ext_comm = world > 1 || (h->p.flags & CMS_FLAG_COLLECTIVE_SINGLE_RANK);
  h->x_allreduce = allreduce;
  h->x_allgather = allgather;
  h->x_user = user;
  return CMS_OK;
}

// splitmix64 finalizer of the key, modulo world.
int32_t cms_shard_of_key(int64_t key, int32_t world) {
  if (world <= 1) return 0;
  uint64_t z = (uint64_t)key + 0x9E3779B97F4A7C15ULL;
  z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ULL;
  z = (z ^ (z >> 27)) * 0x94D049BB133111EBULL;
  z ^= z >> 31;
  return (int32_t)(z % (uint64_t)world);
}

int cms_finalize(cms_handle* h) {
  if (!h) return set_error(CMS_E_PARAM, "null handle");
  Guard g(h);
  if (h->per_owner) {
    int rc = po_finalize(h);
    if (rc) return rc;
    if ((rc = check_flags(h, false))) return rc;
    h->finalized = true;
    return CMS_OK;
  }
  if (h->f64) {
    if (h->empty) {
      CMS_HIP(hipMemsetAsync(h->d_t64, 0, sizeof(double) * h->n * h->dw, h->stream));
      h->empty = false;
      h->norms_valid = false;
    }
    int rc = h->norms_valid ? CMS_OK : f64_norms(h);
    if (rc) return rc;
    CMS_HIP(hipStreamSynchronize(h->stream));
    if ((rc = check_flags(h, false))) return rc;
    h->finalized = true;
    return CMS_OK;
  }
  if (h->empty) {
    if (int rc0 = reset_rows_zero(h)) return rc0;
    h->empty = false;
    h->norms_valid = false;
  }
  if (h->multi() && h->merged) {
    TimedScope ts(h, "delta_exchange");
    int rc = dlog_exchange(h);
    if (rc) return rc;
  } else if (h->multi()) {
    // counter-width-adaptive packed sums over RCCL / the transport (cms_merge.hip)
    auto sum = [h](uint64_t* buf, int64_t count) -> int { return coll_allreduce_u64(h, buf, count); };
    int rc = merge_packed(h, sum);
    if (rc) return rc;
    h->rf_valid = false;  // every rank's table changed wholesale
    h->merged = true;
    h->dlog_n = 0;
  }
  int rc = compute_norms(h);
  if (rc) return rc;
  // error word and inexact-norm count in one pinned read-back: the step's only sync
  CMS_HIP(hipMemcpyAsync(h->h_pin, h->d_flags, 2 * sizeof(uint32_t), hipMemcpyDeviceToHost, h->stream));
  CMS_HIP(hipStreamSynchronize(h->stream));
  const uint32_t inexact = h->h_pin[1];
  h->inexact_zero = inexact == 0;
  rc = flags_error(h, h->h_pin[0], false);
  if (rc) return rc;
  h->exact_norms = inexact == 0;
  h->mfma_ready = false;
  h->i8blk_ready = false;
  h->finalized = true;
  return CMS_OK;
}

int cms_finalize_with(cms_handle* h, cms_allreduce_fn fn, void* user) {
  if (!h || !fn) return set_error(CMS_E_PARAM, "null argument");
  if (int rc0 = refuse_per_owner(h, "cms_finalize_with")) return rc0;
  if (h->f64) return set_error(CMS_E_STATE, "fp64 counters are single-GPU: use cms_finalize");
  Guard g(h);
  if (h->comm || h->ext_comm) return set_error(CMS_E_STATE, "handle has a communicator: use cms_finalize");
  if (h->ext_merged) return set_error(CMS_E_STATE, "already merged: cms_reset starts a new epoch");
  if (h->empty) {
    if (int rc0 = reset_rows_zero(h)) return rc0;
    h->empty = false;
    h->norms_valid = false;
  }
  auto ext = [h, fn, user](uint64_t* buf, int64_t count) -> int {
    CMS_HIP(hipStreamSynchronize(h->stream));
    const int r = fn(buf, count, user);
    if (r != 0) return set_error(CMS_E_RCCL, "caller all-reduce returned %d", r);
    return CMS_OK;
  };
  int rc = merge_packed(h, ext);
  if (rc) return rc;
  h->rf_valid = false;  // the table is now the cross-rank sum: kept lists describe the local table
  h->ext_merged = true;
  if ((rc = compute_norms(h))) return rc;
  CMS_HIP(hipStreamSynchronize(h->stream));
  if ((rc = check_flags(h, false))) return rc;
  uint32_t inexact = 0;
  CMS_HIP(hipMemcpy(&inexact, h->d_flags + 1, sizeof(uint32_t), hipMemcpyDeviceToHost));
  h->inexact_zero = inexact == 0;
  h->exact_norms = inexact == 0;
  h->mfma_ready = false;
  h->i8blk_ready = false;
  h->finalized = true;
  return CMS_OK;
}

int cms_synchronize(cms_handle* h) {
  if (!h) return set_error(CMS_E_PARAM, "null handle");
  Guard g(h);
  CMS_HIP(hipStreamSynchronize(h->stream));
  return check_flags(h, false);
}

static int order_streams(cms_handle* h, hipStream_t from, hipStream_t to) {
  if (!h->order_ev) CMS_HIP(hipEventCreateWithFlags(&h->order_ev, hipEventDisableTiming));
  CMS_HIP(hipEventRecord(h->order_ev, from));
  CMS_HIP(hipStreamWaitEvent(to, h->order_ev, 0));
  return CMS_OK;
}

int cms_wait_stream(cms_handle* h, void* stream) {
  if (!h) return set_error(CMS_E_PARAM, "null handle");
  Guard g(h);
  return order_streams(h, (hipStream_t)stream, h->stream);
}

int cms_release_to_stream(cms_handle* h, void* stream) {
  if (!h) return set_error(CMS_E_PARAM, "null handle");
  Guard g(h);
  return order_streams(h, h->stream, (hipStream_t)stream);
}

// userSimilarity(id1, ids2[i]) on stream st with scratch (qb, ob)
static int similarities_on(cms_handle* h, int64_t id1, const int64_t* ids2, int64_t n, double* out, hipStream_t st,
                           DevBuf& qb, DevBuf& ob, bool shared) {
  int rc = require_finalized(h);
  if (rc) return rc;
  int64_t q;
  if ((rc = row_of(h, id1, &q))) return rc;
  if (n <= 0) return CMS_OK;
  std::vector<int64_t> rows(n);
  for (int64_t i = 0; i < n; ++i)
    if ((rc = row_of(h, ids2[i], &rows[i]))) return rc;
  CMS_HIP(qb.ensure(sizeof(int64_t) * (n + 1)));
  CMS_HIP(ob.ensure(sizeof(double) * n));
  hipStream_t ks = shared ? st : nullptr;  // kernels on the context's stream (untimed) or the handle's
  if (h->per_owner) {  // u2's shape decides each pair (CosineCM.java:86)
    if ((rc = po_require_shapes(h, rows.data(), n))) return rc;
    rows.push_back(q);
    CMS_HIP(hipMemcpyAsync(qb.ptr, rows.data(), sizeof(int64_t) * (n + 1), hipMemcpyHostToDevice, st));
    rc = po_pair_cosines(h, qb.as<int64_t>() + n, 1, qb.as<int64_t>(), n, ob.as<double>(), ks);
  } else {
    CMS_HIP(hipMemcpyAsync(qb.ptr, rows.data(), sizeof(int64_t) * n, hipMemcpyHostToDevice, st));
    rc = pair_cosines(h, q, qb.as<int64_t>(), n, ob.as<double>(), ks);
  }
  if (rc) return rc;
  CMS_HIP(hipMemcpyAsync(out, ob.ptr, sizeof(double) * n, hipMemcpyDeviceToHost, st));
  CMS_HIP(hipStreamSynchronize(st));
  return CMS_OK;
}

int cms_similarities(cms_handle* h, int64_t id1, const int64_t* ids2, int64_t n, double* out) {
  if (!h || (n > 0 && (!ids2 || !out))) return set_error(CMS_E_PARAM, "null argument");
  {
    SharedGuard g(h);
    if (!po_shared_scratch(h)) {  // concurrent readers, each on its own stream and scratch
      CtxLease L(h);
      if (int rc = L.ready()) return rc;
      return similarities_on(h, id1, ids2, n, out, L.c->stream, L.c->q, L.c->o, true);
    }
  }
  Guard g(h);
  return similarities_on(h, id1, ids2, n, out, h->stream, h->ws_query, h->ws_small, false);
}

int cms_similarity(cms_handle* h, int64_t id1, int64_t id2, double* out) {
  return cms_similarities(h, id1, &id2, 1, out);
}

static int estimate_on(cms_handle* h, int64_t user_id, const int64_t* neighbor_ids, int64_t m,
                       const int64_t* item_keys, int64_t q, int32_t use_capper, float cap_min, float cap_max,
                       float* out, hipStream_t st, QueryCtx& c, bool shared) {
  int rc = require_finalized(h);
  if (rc) return rc;
  int64_t urow;
  if ((rc = row_of(h, user_id, &urow))) return rc;
  std::vector<int64_t> rows(m);
  for (int64_t i = 0; i < m; ++i)
    if ((rc = row_of(h, neighbor_ids[i], &rows[i]))) return rc;
  if (q == 0) return CMS_OK;
  hipStream_t ks = shared ? st : nullptr;
  // c.r: neighbour rows then the user's row; c.x: similarities; c.q: item keys; c.o: estimates
  CMS_HIP(c.r.ensure(sizeof(int64_t) * (size_t)(m + 1)));
  CMS_HIP(c.x.ensure(sizeof(double) * (size_t)std::max<int64_t>(m, 1)));
  CMS_HIP(c.q.ensure(sizeof(int64_t) * (size_t)q));
  CMS_HIP(c.o.ensure(sizeof(float) * (size_t)q));
  rows.push_back(urow);
  CMS_HIP(hipMemcpyAsync(c.r.ptr, rows.data(), sizeof(int64_t) * (size_t)(m + 1), hipMemcpyHostToDevice, st));
  CMS_HIP(hipMemcpyAsync(c.q.ptr, item_keys, sizeof(int64_t) * q, hipMemcpyHostToDevice, st));
  int64_t* d_rows = c.r.as<int64_t>();
  double* d_sims = c.x.as<double>();
  if (h->per_owner) {
    std::vector<int64_t> others;  // every neighbour but the user needs its own profile (:154-156)
    for (int64_t i = 0; i < m; ++i)
      if (rows[i] != urow) others.push_back(rows[i]);
    if ((rc = po_require_shapes(h, others.data(), (int64_t)others.size()))) return rc;
    if ((rc = po_pair_cosines(h, d_rows + m, 1, d_rows, m, d_sims, ks))) return rc;
    rc = po_estimate_preferences(h, urow, d_rows, d_sims, m, c.q.as<int64_t>(), q, use_capper, cap_min, cap_max,
                                 c.o.as<float>(), ks);
  } else {
    if ((rc = pair_cosines(h, urow, d_rows, m, d_sims, ks))) return rc;
    rc = estimate_preferences(h, urow, d_rows, d_sims, m, c.q.as<int64_t>(), q, use_capper, cap_min, cap_max,
                              c.o.as<float>(), ks);
  }
  if (rc) return rc;
  CMS_HIP(hipMemcpyAsync(out, c.o.ptr, sizeof(float) * q, hipMemcpyDeviceToHost, st));
  CMS_HIP(hipStreamSynchronize(st));
  return CMS_OK;
}

int cms_estimate_preferences(cms_handle* h, int64_t user_id, const int64_t* neighbor_ids, int64_t m,
                             const int64_t* item_keys, int64_t q, int32_t use_capper, float cap_min, float cap_max,
                             float* out) {
  if (!h || m < 0 || q < 0 || (m > 0 && !neighbor_ids) || (q > 0 && (!item_keys || !out)))
    return set_error(CMS_E_PARAM, "null argument");
  {
    SharedGuard g(h);
    if (!po_shared_scratch(h)) {
      CtxLease L(h);
      if (int rc = L.ready()) return rc;
      return estimate_on(h, user_id, neighbor_ids, m, item_keys, q, use_capper, cap_min, cap_max, out, L.c->stream,
                         *L.c, true);
    }
  }
  Guard g(h);
  QueryCtx tmp;  // exclusive path: the handle's stream, call-local scratch
  return estimate_on(h, user_id, neighbor_ids, m, item_keys, q, use_capper, cap_min, cap_max, out, h->stream, tmp,
                     false);
}

// cms_estimate_preferences_batch on a fixed-shape table, under the shared
// guard: c.r rows, c.y neighbour offsets, c.x similarities, c.q item keys,
// c.z candidate -> user, c.o estimates, all on c.stream.
static int estimate_batch_on(cms_handle* h, int64_t n, const int64_t* user_ids, const int64_t* nb_offsets,
                             const int64_t* neighbor_ids, const int64_t* item_offsets, const int64_t* item_keys,
                             int32_t use_capper, float cap_min, float cap_max, float* out, QueryCtx& c) {
  int rc = require_finalized(h);
  if (rc) return rc;
  const int64_t M = nb_offsets[n], Q = item_offsets[n];
  // rows: users [n], then per pair (user row, neighbour row) [M] x 2; the
  // owner of every candidate [Q]
  std::vector<int64_t> rows((size_t)(n + 2 * M));
  std::vector<int32_t> item_user((size_t)Q);
  for (int64_t u = 0; u < n; ++u) {
    if ((rc = row_of(h, user_ids[u], &rows[(size_t)u]))) return rc;
    for (int64_t j = nb_offsets[u]; j < nb_offsets[u + 1]; ++j) {
      rows[(size_t)(n + j)] = rows[(size_t)u];
      if ((rc = row_of(h, neighbor_ids[j], &rows[(size_t)(n + M + j)]))) return rc;
    }
    for (int64_t i = item_offsets[u]; i < item_offsets[u + 1]; ++i) item_user[(size_t)i] = (int32_t)u;
  }
  if (Q == 0) return CMS_OK;
  DevBuf &d_rows = c.r, &d_off = c.y, &d_sims = c.x, &d_items = c.q, &d_iu = c.z, &d_out = c.o;
  CMS_HIP(d_rows.ensure(sizeof(int64_t) * rows.size()));
  CMS_HIP(d_off.ensure(sizeof(int64_t) * (size_t)(n + 1)));
  CMS_HIP(d_sims.ensure(sizeof(double) * (size_t)std::max<int64_t>(M, 1)));
  CMS_HIP(d_items.ensure(sizeof(int64_t) * (size_t)Q));
  CMS_HIP(d_iu.ensure(sizeof(int32_t) * (size_t)Q));
  CMS_HIP(d_out.ensure(sizeof(float) * (size_t)Q));
  hipStream_t st = c.stream;
  CMS_HIP(hipMemcpyAsync(d_rows.ptr, rows.data(), sizeof(int64_t) * rows.size(), hipMemcpyHostToDevice, st));
  CMS_HIP(hipMemcpyAsync(d_off.ptr, nb_offsets, sizeof(int64_t) * (size_t)(n + 1), hipMemcpyHostToDevice, st));
  CMS_HIP(hipMemcpyAsync(d_items.ptr, item_keys, sizeof(int64_t) * (size_t)Q, hipMemcpyHostToDevice, st));
  CMS_HIP(hipMemcpyAsync(d_iu.ptr, item_user.data(), sizeof(int32_t) * (size_t)Q, hipMemcpyHostToDevice, st));
  const int64_t* dr = d_rows.as<int64_t>();
  // userSimilarity(user, neighbour) for every pair of the batch (:162)
  if ((rc = pair_cosines_many(h, dr + n, dr + n + M, M, d_sims.as<double>(), st))) return rc;
  if ((rc = estimate_preferences_batch(h, dr, d_off.as<int64_t>(), dr + n + M, d_sims.as<double>(), d_iu.as<int32_t>(),
                                       d_items.as<int64_t>(), Q, use_capper, cap_min, cap_max, d_out.as<float>(),
                                       st)))
    return rc;
  CMS_HIP(hipMemcpyAsync(out, d_out.ptr, sizeof(float) * (size_t)Q, hipMemcpyDeviceToHost, st));
  CMS_HIP(hipStreamSynchronize(st));
  return CMS_OK;
}

int cms_estimate_preferences_batch(cms_handle* h, int64_t n, const int64_t* user_ids, const int64_t* nb_offsets,
                                   const int64_t* neighbor_ids, const int64_t* item_offsets, const int64_t* item_keys,
                                   int32_t use_capper, float cap_min, float cap_max, float* out) {
  if (!h || n < 0 || (n > 0 && (!user_ids || !nb_offsets || !item_offsets)))
    return set_error(CMS_E_PARAM, "null argument");
  if (n == 0) return CMS_OK;
  if (nb_offsets[0] != 0 || item_offsets[0] != 0) return set_error(CMS_E_PARAM, "offsets must start at 0");
  for (int64_t u = 0; u < n; ++u)
    if (nb_offsets[u + 1] < nb_offsets[u] || item_offsets[u + 1] < item_offsets[u])
      return set_error(CMS_E_PARAM, "offsets must not decrease");
  const int64_t M = nb_offsets[n], Q = item_offsets[n];
  if ((M > 0 && !neighbor_ids) || (Q > 0 && (!item_keys || !out))) return set_error(CMS_E_PARAM, "null argument");
  if (Q >= (int64_t(1) << 31)) return set_error(CMS_E_PARAM, "too many candidate items in one batch");
  if (!h->per_owner && !h->f64) {
    // fixed-shape u32 table: one batched pass, shared with other readers, on
    // a leased stream and scratch (no per-call hipMalloc)
    SharedGuard g(h);
    CtxLease L(h);
    if (int rc = L.ready()) return rc;
    return estimate_batch_on(h, n, user_ids, nb_offsets, neighbor_ids, item_offsets, item_keys, use_capper, cap_min,
                             cap_max, out, *L.c);
  }
  Guard g(h);
  int rc = require_finalized(h);
  if (rc) return rc;
  QueryCtx tmp;  // per-user estimates (their own kernels), one user after another
  for (int64_t u = 0; u < n; ++u)
    if ((rc = estimate_on(h, user_ids[u], neighbor_ids + nb_offsets[u], nb_offsets[u + 1] - nb_offsets[u],
                          item_keys + item_offsets[u], item_offsets[u + 1] - item_offsets[u], use_capper, cap_min,
                          cap_max, out + item_offsets[u], h->stream, tmp, false)))
      return rc;
  return CMS_OK;
}

int cms_recommend_batch(cms_handle* h, int64_t n, const int64_t* user_ids, const int64_t* nb_offsets,
                        const int64_t* neighbor_ids, int64_t n_model_users, const int64_t* model_user_ids,
                        const int64_t* pref_offsets, const int64_t* pref_items, int32_t how_many,
                        int32_t include_known, int32_t use_capper, float cap_min, float cap_max, int32_t* out_counts,
                        int64_t* out_items, float* out_values) {
  if (!h || n < 0 || n_model_users < 0 || (n > 0 && (!user_ids || !nb_offsets || !out_counts || !out_items ||
                                                     !out_values)) ||
      (n_model_users > 0 && (!model_user_ids || !pref_offsets)))
    return set_error(CMS_E_PARAM, "null argument");
  if (how_many < 1) return set_error(CMS_E_PARAM, "howMany must be at least 1");
  if (n == 0) return CMS_OK;
  if (nb_offsets[0] != 0) return set_error(CMS_E_PARAM, "nb_offsets must start at 0");
  for (int64_t u = 0; u < n; ++u)
    if (nb_offsets[u + 1] < nb_offsets[u]) return set_error(CMS_E_PARAM, "nb_offsets must not decrease");
  if (nb_offsets[n] > 0 && !neighbor_ids) return set_error(CMS_E_PARAM, "null argument");
  if (n_model_users > 0) {
    if (pref_offsets[0] != 0) return set_error(CMS_E_PARAM, "pref_offsets must start at 0");
    for (int64_t r = 0; r < n_model_users; ++r) {
      if (pref_offsets[r + 1] < pref_offsets[r]) return set_error(CMS_E_PARAM, "pref_offsets must not decrease");
      if (r > 0 && model_user_ids[r] <= model_user_ids[r - 1])
        return set_error(CMS_E_PARAM, "model_user_ids must be strictly ascending");
    }
    if (pref_offsets[n_model_users] > 0 && !pref_items) return set_error(CMS_E_PARAM, "null argument");
  }
  const int64_t* mb = model_user_ids;
  const int64_t* me = model_user_ids + n_model_users;
  auto model_row = [&](int64_t id) -> int64_t {
    const int64_t* it = std::lower_bound(mb, me, id);
    return it != me && *it == id ? it - mb : -1;
  };
  // neighbourhood rows in the model (a neighbour the model lacks would throw
  // NoSuchUserException from getItemIDsFromUser)
  std::vector<int64_t> nb_rows((size_t)nb_offsets[n]);
  std::vector<int64_t> user_rows((size_t)n);
  for (int64_t u = 0; u < n; ++u) {
    const bool empty = nb_offsets[u + 1] == nb_offsets[u];
    user_rows[(size_t)u] = model_row(user_ids[u]);
    if (!empty && !include_known && user_rows[(size_t)u] < 0)
      return set_error(CMS_E_NO_SUCH_ID, "no such user ID %lld in the data model", (long long)user_ids[u]);
    for (int64_t j = nb_offsets[u]; j < nb_offsets[u + 1]; ++j)
      if ((nb_rows[(size_t)j] = model_row(neighbor_ids[j])) < 0)
        return set_error(CMS_E_NO_SUCH_ID, "no such user ID %lld in the data model", (long long)neighbor_ids[j]);
  }
  // candidates per user (host threads), then one concatenated estimate batch
  std::vector<std::vector<int64_t>> cand((size_t)n);
  const int threads = (int)std::min<unsigned>(16u, std::max(1u, std::thread::hardware_concurrency()));
  parallel_users(n, threads, [&](int64_t u) {
    if (nb_offsets[u + 1] == nb_offsets[u]) return;  // recommend(): an empty neighbourhood recommends nothing
    recommend_candidates(nb_rows.data() + nb_offsets[u], nb_offsets[u + 1] - nb_offsets[u], user_rows[(size_t)u],
                         pref_offsets, pref_items, include_known != 0, cand[(size_t)u]);
  });
  std::vector<int64_t> it_off((size_t)n + 1, 0);
  for (int64_t u = 0; u < n; ++u) it_off[(size_t)u + 1] = it_off[(size_t)u] + (int64_t)cand[(size_t)u].size();
  std::vector<int64_t> keys((size_t)it_off[(size_t)n]);
  for (int64_t u = 0; u < n; ++u) std::copy(cand[(size_t)u].begin(), cand[(size_t)u].end(), keys.begin() + it_off[(size_t)u]);
  std::vector<float> est(keys.size());
  if (int rc = cms_estimate_preferences_batch(h, n, user_ids, nb_offsets, neighbor_ids, it_off.data(), keys.data(),
                                              use_capper, cap_min, cap_max, est.data()))
    return rc;
  parallel_users(n, threads, [&](int64_t u) {
    const int64_t o = it_off[(size_t)u];
    out_counts[u] = recommend_top_items(how_many, keys.data() + o, est.data() + o, it_off[(size_t)u + 1] - o,
                                        out_items + u * (int64_t)how_many, out_values + u * (int64_t)how_many);
  });
  return CMS_OK;
}

int cms_point_query(cms_handle* h, int64_t id, int64_t key, double* out) {
  if (!h || !out) return set_error(CMS_E_PARAM, "null argument");
  SharedGuard g(h);
  int rc = require_finalized(h);
  if (rc) return rc;
  int64_t row;
  if ((rc = row_of(h, id, &row))) return rc;
  CtxLease L(h);
  if ((rc = L.ready())) return rc;
  QueryCtx& c = *L.c;
  CMS_HIP(c.q.ensure(sizeof(int64_t)));
  CMS_HIP(c.o.ensure(sizeof(double)));
  CMS_HIP(hipMemcpyAsync(c.q.ptr, &key, sizeof(int64_t), hipMemcpyHostToDevice, c.stream));
  if (h->per_owner) {
    if ((rc = po_require_shapes(h, &row, 1))) return rc;
    rc = po_point_queries(h, row, c.q.as<int64_t>(), 1, c.o.as<double>(), c.stream);
  } else {
    rc = point_queries(h, row, c.q.as<int64_t>(), 1, c.o.as<double>(), c.stream);
  }
  if (rc) return rc;
  CMS_HIP(hipMemcpyAsync(out, c.o.ptr, sizeof(double), hipMemcpyDeviceToHost, c.stream));
  CMS_HIP(hipStreamSynchronize(c.stream));
  return CMS_OK;
}

static int top_k_host(cms_handle* h, int64_t row_begin, int64_t row_count, int32_t k, int64_t* ids, double* scores,
                      int32_t* counts) {
  DevBuf o_ids, o_sc, o_cnt;
  CMS_HIP(o_ids.ensure(sizeof(int64_t) * row_count * k));
  CMS_HIP(o_sc.ensure(sizeof(double) * row_count * k));
  CMS_HIP(o_cnt.ensure(sizeof(int32_t) * row_count));
  int rc = top_k_rows(h, row_begin, row_count, k, o_ids.as<int64_t>(), o_sc.as<double>(), o_cnt.as<int32_t>());
  if (rc == CMS_OK) {
    hipError_t e = hipMemcpyAsync(ids, o_ids.ptr, sizeof(int64_t) * row_count * k, hipMemcpyDeviceToHost, h->stream);
    if (e == hipSuccess && scores)
      e = hipMemcpyAsync(scores, o_sc.ptr, sizeof(double) * row_count * k, hipMemcpyDeviceToHost, h->stream);
    if (e == hipSuccess)
      e = hipMemcpyAsync(counts, o_cnt.ptr, sizeof(int32_t) * row_count, hipMemcpyDeviceToHost, h->stream);
    if (e == hipSuccess) e = hipStreamSynchronize(h->stream);
    if (e != hipSuccess) rc = hip_fail(e, "top-k copy-out");
  }
  o_ids.release();
  o_sc.release();
  o_cnt.release();
  return rc;
}

int cms_most_similar(cms_handle* h, int64_t id, int32_t k, int64_t* out_ids, double* out_scores, int32_t* count) {
  if (!h || !out_ids || !count) return set_error(CMS_E_PARAM, "null argument");
  Guard g(h);
  int rc = require_finalized(h);
  if (rc) return rc;
  int64_t row;
  if ((rc = row_of(h, id, &row))) return rc;
  return top_k_host(h, row, 1, k, out_ids, out_scores, count);
}

int cms_top_k_rows(cms_handle* h, int64_t row_begin, int64_t row_count, int32_t k, int64_t* ids, double* scores,
                   int32_t* counts) {
  if (!h || !ids || !counts) return set_error(CMS_E_PARAM, "null argument");
  Guard g(h);
  int rc = require_finalized(h);
  if (rc) return rc;
  if (row_begin < 0 || row_count < 0 || row_begin + row_count > h->n) return set_error(CMS_E_PARAM, "row range");
  if (row_count == 0) return CMS_OK;
  return top_k_host(h, row_begin, row_count, k, ids, scores, counts);
}

extern "C++" {
namespace cms {
int top_k_all_job(cms_handle* h, int32_t k, int64_t* d_ids, double* d_scores, int32_t* d_counts) {
  const int64_t n = h->n;
  if (!h->multi()) return top_k_all(h, k, d_ids, d_scores, d_counts);
  // one process per GPU: rank r computes shard r of the pairs, then one
  // all-gather of the partial lists over xGMI and an exact merge (in rounds
  // of kCandCap / k lists when world * k exceeds a merge workgroup's LDS)
  const int G = h->world;
  DevBuf g_ids, g_sc, g_cnt;
  CMS_HIP(g_ids.ensure(sizeof(int64_t) * n * k * G));
  CMS_HIP(g_sc.ensure(sizeof(double) * n * k * G));
  CMS_HIP(g_cnt.ensure(sizeof(int32_t) * n * G));
  int rc = top_k_all(h, k, d_ids, d_scores, d_counts, h->rank, G);
  if (rc) return rc;
  {
    TimedScope ts(h, "topk_allgather");
    if ((rc = coll_allgather(h, d_ids, g_ids.ptr, (int64_t)sizeof(int64_t) * n * k)) ||
        (rc = coll_allgather(h, d_scores, g_sc.ptr, (int64_t)sizeof(double) * n * k)) ||
        (rc = coll_allgather(h, d_counts, g_cnt.ptr, (int64_t)sizeof(int32_t) * n)))
      return rc;
  }
  rc = top_k_merge(h, k, G, g_ids.as<int64_t>(), g_sc.as<double>(), g_cnt.as<int32_t>(), d_ids, d_scores, d_counts);
  if (rc == CMS_OK) {
    const hipError_t e = hipStreamSynchronize(h->stream);  // the gather buffers free on return
    if (e != hipSuccess) rc = hip_fail(e, "top-k merge");
  }
  return rc;
}
}  // namespace cms
}

// Padding of the [n][k] list outputs: entries past counts[r] hold ID -1 and a
// NaN score (all-ones bytes), written before the job so the kernels' valid
// prefixes overwrite it (include/mahout_cms.h, cms_top_k_all).
static int pad_lists(cms_handle* h, int64_t k, int64_t* d_ids, double* d_sc) {
  const size_t cells = (size_t)h->n * (size_t)k;
  CMS_HIP(hipMemsetAsync(d_ids, 0xFF, sizeof(int64_t) * cells, h->stream));
  if (d_sc) CMS_HIP(hipMemsetAsync(d_sc, 0xFF, sizeof(double) * cells, h->stream));
  return CMS_OK;
}

static int copy_out_lists(cms_handle* h, int64_t k, const DevBuf& o_ids, const DevBuf& o_sc, const DevBuf& o_cnt,
                          int64_t* ids, double* scores, int32_t* counts) {
  const int64_t n = h->n;
  hipError_t e = hipMemcpyAsync(ids, o_ids.ptr, sizeof(int64_t) * n * k, hipMemcpyDeviceToHost, h->stream);
  if (e == hipSuccess && scores)
    e = hipMemcpyAsync(scores, o_sc.ptr, sizeof(double) * n * k, hipMemcpyDeviceToHost, h->stream);
  if (e == hipSuccess) e = hipMemcpyAsync(counts, o_cnt.ptr, sizeof(int32_t) * n, hipMemcpyDeviceToHost, h->stream);
  if (e == hipSuccess) e = hipStreamSynchronize(h->stream);
  if (e != hipSuccess) return hip_fail(e, "top-k copy-out");
  return CMS_OK;
}

static int check_k(int32_t k) {
  if (k < 1 || k > kCandCap / 2) return set_error(CMS_E_PARAM, "k must be in [1, %d]", kCandCap / 2);
  return CMS_OK;
}

int cms_top_k_all(cms_handle* h, int32_t k, int64_t* ids, double* scores, int32_t* counts) {
  if (!h || !ids || !counts) return set_error(CMS_E_PARAM, "null argument");
  if (int rc0 = check_k(k)) return rc0;
  Guard g(h);
  int rc = require_finalized(h);
  if (rc) return rc;
  const int64_t n = h->n;
  DevBuf o_ids, o_sc, o_cnt;
  CMS_HIP(o_ids.ensure(sizeof(int64_t) * n * k));
  CMS_HIP(o_sc.ensure(sizeof(double) * n * k));
  CMS_HIP(o_cnt.ensure(sizeof(int32_t) * n));
  if ((rc = pad_lists(h, k, o_ids.as<int64_t>(), o_sc.as<double>()))) return rc;
  rc = top_k_all_job(h, k, o_ids.as<int64_t>(), o_sc.as<double>(), o_cnt.as<int32_t>());
  if (rc == CMS_OK) rc = copy_out_lists(h, k, o_ids, o_sc, o_cnt, ids, scores, counts);
  return rc;
}

int cms_top_k_all_device(cms_handle* h, int32_t k, int64_t* d_ids, double* d_scores, int32_t* d_counts) {
  if (!h || !d_ids || !d_scores || !d_counts) return set_error(CMS_E_PARAM, "null argument");
  if (int rc0 = check_k(k)) return rc0;
  Guard g(h);
  int rc = require_finalized(h);
  if (rc) return rc;
  if ((rc = pad_lists(h, k, d_ids, d_scores))) return rc;
  if ((rc = top_k_all_job(h, k, d_ids, d_scores, d_counts))) return rc;
  CMS_HIP(hipStreamSynchronize(h->stream));
  return check_flags(h, false);
}

// Incremental all-pairs top-k (the periodic refresh of a streaming table):
// the result of cms_top_k_all on the current table, computed from the lists
// the previous refresh kept plus the pairs with an owner a COO batch touched
// since (cms_topk.hip, k_rf_fold, states the exactness argument).  Writes the
// k-deep answer into the device buffers o_* (already padded).
static int top_k_refresh_job(cms_handle* h, int32_t k, int64_t* o_ids, double* o_sc, int32_t* o_cnt) {
  const int64_t n = h->n;
  int rc = CMS_OK;
  if (h->per_owner || h->f64)  // no kept lists for these modes: the whole job
    return top_k_all_job(h, k, o_ids, o_sc, o_cnt);
  // kept lists are twice as deep as the answer, so a few candidates of an
  // untouched owner may leave before its list must be recomputed
  const int32_t D = std::min(2 * k, kCandCap / 2);
  // the job and the redo emit owner ROWS (the kept lists' candidates)
  struct RowsOut {
    cms_handle* h;
    int64_t* saved;
    ~RowsOut() { h->d_owner_ids = saved; }
  } rows_out{h, h->d_owner_ids};
  h->d_owner_ids = nullptr;
  const bool full = !h->rf_valid || h->rf_k != k || h->rf_depth != D;
  // Until this call completes the kept lists are not trusted: a failure at any
  // step below (after the fold has rewritten some lists, say) leaves rf_valid
  // false, so the next refresh is a whole job and no COO ingest marks into
  // the touched-owner array meanwhile.
  h->rf_valid = false;
  if (full) {
    CMS_HIP(h->rf_ids.ensure(sizeof(int64_t) * (size_t)n * D));
    CMS_HIP(h->rf_sc.ensure(sizeof(double) * (size_t)n * D));
    CMS_HIP(h->rf_cnt.ensure(sizeof(int32_t) * (size_t)n));
    CMS_HIP(h->rf_full.ensure((size_t)n));
    CMS_HIP(h->rf_touch.ensure((size_t)n));
    h->rf_depth = D;
    h->rf_k = k;
    TimedScope ts(h, "refresh_full");
    if ((rc = top_k_all_job(h, D, h->rf_ids.as<int64_t>(), h->rf_sc.as<double>(), h->rf_cnt.as<int32_t>())))
      return rc;
    if ((rc = refresh_set_full(h))) return rc;
    {
      const int64_t nm = h->n_hot_limb, nf = h->n_f4;
      const int64_t cls[6] = {nm, n - nm - nf, nf, nm, n - nm - nf, nf};
      std::copy(cls, cls + 6, h->rf_stat_class);
    }
    h->rf_stat_full += 1;
    h->rf_stat_touched = n;
    h->rf_stat_redo = 0;
  } else {
    // touched owners since the kept lists were made
    std::vector<uint8_t> touch(n);
    CMS_HIP(hipMemcpyAsync(touch.data(), h->rf_touch.ptr, (size_t)n, hipMemcpyDeviceToHost, h->stream));
    CMS_HIP(hipStreamSynchronize(h->stream));
    int64_t nt = 0;
    for (int64_t r = 0; r < n; ++r) nt += touch[r];
    h->rf_stat_touched = nt;
    h->rf_stat_redo = 0;
    if (nt == 0) {  // nothing recomputed: the class counts say so (not the previous refresh's)
      const int64_t nm = h->n_hot_limb, nf = h->n_f4;
      const int64_t cls[6] = {nm, n - nm - nf, nf, 0, 0, 0};
      std::copy(cls, cls + 6, h->rf_stat_class);
    }
    if (nt > 0) {
      CMS_HIP(h->rf_new.ensure((sizeof(int64_t) + sizeof(double)) * (size_t)n * D + sizeof(int32_t) * (size_t)n));
      int64_t* n_ids = h->rf_new.as<int64_t>();
      double* n_sc = reinterpret_cast<double*>(n_ids + (size_t)n * D);
      int32_t* n_cnt = reinterpret_cast<int32_t*>(n_sc + (size_t)n * D);
      // the operands are re-laid out with the touched owners first
      h->mfma_ready = false;
      h->i8blk_ready = false;
      h->rf_restrict = true;
      {
        TimedScope ts(h, "refresh_job");
        rc = top_k_all_job(h, D, n_ids, n_sc, n_cnt);
      }
      h->rf_restrict = false;
      if (rc) return rc;
      {  // touched owners per operand class (positions: multi-limb, int8, fp4)
        const int64_t nm = h->n_hot_limb, nf = h->n_f4;
        int64_t tm = 0;
        for (int64_t r = 0; r < n; ++r) tm += touch[r] && h->h_inv[r] < nm;
        const int64_t cls[6] = {nm, n - nm - nf, nf, tm, h->rf_t8, h->rf_t4};
        std::copy(cls, cls + 6, h->rf_stat_class);
      }
      CMS_HIP(h->rf_redo.ensure(sizeof(uint32_t) * ((size_t)n + 1)));
      uint32_t* redo = h->rf_redo.as<uint32_t>();
      {
        TimedScope ts(h, "refresh_fold");
        if ((rc = refresh_fold(h, n_ids, n_sc, n_cnt, k, redo))) return rc;
      }
      uint32_t nredo = 0;
      CMS_HIP(hipMemcpyAsync(&nredo, redo, sizeof(uint32_t), hipMemcpyDeviceToHost, h->stream));
      CMS_HIP(hipStreamSynchronize(h->stream));
      h->rf_stat_redo = nredo;
      if (nredo > 0) {  // lists an untouched owner could not keep exact: whole-row recompute
        std::vector<uint32_t> rows(nredo);
        CMS_HIP(hipMemcpyAsync(rows.data(), redo + 1, sizeof(uint32_t) * nredo, hipMemcpyDeviceToHost, h->stream));
        CMS_HIP(hipStreamSynchronize(h->stream));
        std::vector<int64_t> pos(nredo), outp(nredo);
        for (uint32_t i = 0; i < nredo; ++i) {
          outp[i] = rows[i];
          pos[i] = h->h_inv[rows[i]];
        }
        TimedScope ts(h, "refresh_redo");
        if ((rc = slab_top_k_positions(h, pos, outp, D, h->rf_ids.as<int64_t>(), h->rf_sc.as<double>(),
                                       h->rf_cnt.as<int32_t>())))
          return rc;
        // a recomputed list holds every candidate iff it is shorter than D
        if ((rc = refresh_set_full_list(h, redo, nredo))) return rc;
      }
    }
  }
  CMS_HIP(hipMemsetAsync(h->rf_touch.ptr, 0, (size_t)n, h->stream));
  h->rf_valid = true;
  h->d_owner_ids = rows_out.saved;
  return refresh_emit(h, k, o_ids, o_sc, o_cnt);
}

int cms_top_k_refresh(cms_handle* h, int32_t k, int64_t* ids, double* scores, int32_t* counts) {
  if (!h || !ids || !counts) return set_error(CMS_E_PARAM, "null argument");
  if (int rc0 = check_k(k)) return rc0;
  Guard g(h);
  int rc = require_finalized(h);
  if (rc) return rc;
  const int64_t n = h->n;
  DevBuf o_ids, o_sc, o_cnt;
  CMS_HIP(o_ids.ensure(sizeof(int64_t) * n * k));
  CMS_HIP(o_sc.ensure(sizeof(double) * n * k));
  CMS_HIP(o_cnt.ensure(sizeof(int32_t) * n));
  if ((rc = pad_lists(h, k, o_ids.as<int64_t>(), o_sc.as<double>()))) return rc;
  if ((rc = top_k_refresh_job(h, k, o_ids.as<int64_t>(), o_sc.as<double>(), o_cnt.as<int32_t>()))) return rc;
  return copy_out_lists(h, k, o_ids, o_sc, o_cnt, ids, scores, counts);
}

int cms_top_k_refresh_device(cms_handle* h, int32_t k, int64_t* d_ids, double* d_scores, int32_t* d_counts) {
  if (!h || !d_ids || !d_scores || !d_counts) return set_error(CMS_E_PARAM, "null argument");
  if (int rc0 = check_k(k)) return rc0;
  Guard g(h);
  int rc = require_finalized(h);
  if (rc) return rc;
  if ((rc = pad_lists(h, k, d_ids, d_scores))) return rc;
  if ((rc = top_k_refresh_job(h, k, d_ids, d_scores, d_counts))) return rc;
  CMS_HIP(hipStreamSynchronize(h->stream));
  return check_flags(h, false);
}

int cms_refresh_stats(cms_handle* h, int64_t* touched, int64_t* redone, int64_t* full_jobs) {
  if (!h || !touched || !redone || !full_jobs) return set_error(CMS_E_PARAM, "null argument");
  Guard g(h);
  *touched = h->rf_stat_touched;
  *redone = h->rf_stat_redo;
  *full_jobs = h->rf_stat_full;
  return CMS_OK;
}

int cms_refresh_classes(cms_handle* h, int64_t* out6) {
  if (!h || !out6) return set_error(CMS_E_PARAM, "null argument");
  Guard g(h);
  std::copy(h->rf_stat_class, h->rf_stat_class + 6, out6);
  return CMS_OK;
}

int cms_top_k_all_partial(cms_handle* h, int32_t k, int32_t shard, int32_t nshards, int64_t* ids, double* scores,
                          int32_t* counts) {
  if (!h || !ids || !scores || !counts) return set_error(CMS_E_PARAM, "null argument");
  if (int rc0 = refuse_per_owner(h, "cms_top_k_all_partial")) return rc0;
  if (k < 1 || k > kCandCap / 2) return set_error(CMS_E_PARAM, "k must be in [1, %d]", kCandCap / 2);
  if (nshards < 1 || shard < 0 || shard >= nshards) return set_error(CMS_E_PARAM, "shard %d of %d", shard, nshards);
  Guard g(h);
  int rc = require_finalized(h);
  if (rc) return rc;
  const int64_t n = h->n;
  DevBuf o_ids, o_sc, o_cnt;
  CMS_HIP(o_ids.ensure(sizeof(int64_t) * n * k));
  CMS_HIP(o_sc.ensure(sizeof(double) * n * k));
  CMS_HIP(o_cnt.ensure(sizeof(int32_t) * n));
  rc = top_k_all(h, k, o_ids.as<int64_t>(), o_sc.as<double>(), o_cnt.as<int32_t>(), shard, nshards);
  if (rc) return rc;
  CMS_HIP(hipMemcpyAsync(ids, o_ids.ptr, sizeof(int64_t) * n * k, hipMemcpyDeviceToHost, h->stream));
  CMS_HIP(hipMemcpyAsync(scores, o_sc.ptr, sizeof(double) * n * k, hipMemcpyDeviceToHost, h->stream));
  CMS_HIP(hipMemcpyAsync(counts, o_cnt.ptr, sizeof(int32_t) * n, hipMemcpyDeviceToHost, h->stream));
  CMS_HIP(hipStreamSynchronize(h->stream));
  return CMS_OK;
}

int cms_top_k_merge(cms_handle* h, int32_t k, int32_t nparts, const int64_t* ids, const double* scores,
                    const int32_t* counts, int64_t* out_ids, double* out_scores, int32_t* out_counts) {
  if (!h || !ids || !scores || !counts || !out_ids || !out_scores || !out_counts)
    return set_error(CMS_E_PARAM, "null argument");
  if (k < 1 || k > kCandCap / 2 || nparts < 1)
    return set_error(CMS_E_PARAM, "need k in [1, %d] and nparts >= 1", kCandCap / 2);
  Guard g(h);
  const int64_t n = h->n;
  DevBuf i_ids, i_sc, i_cnt, o_ids, o_sc, o_cnt;
  CMS_HIP(i_ids.ensure(sizeof(int64_t) * n * k * nparts));
  CMS_HIP(i_sc.ensure(sizeof(double) * n * k * nparts));
  CMS_HIP(i_cnt.ensure(sizeof(int32_t) * n * nparts));
  CMS_HIP(o_ids.ensure(sizeof(int64_t) * n * k));
  CMS_HIP(o_sc.ensure(sizeof(double) * n * k));
  CMS_HIP(o_cnt.ensure(sizeof(int32_t) * n));
  CMS_HIP(hipMemcpyAsync(i_ids.ptr, ids, sizeof(int64_t) * n * k * nparts, hipMemcpyHostToDevice, h->stream));
  CMS_HIP(hipMemcpyAsync(i_sc.ptr, scores, sizeof(double) * n * k * nparts, hipMemcpyHostToDevice, h->stream));
  CMS_HIP(hipMemcpyAsync(i_cnt.ptr, counts, sizeof(int32_t) * n * nparts, hipMemcpyHostToDevice, h->stream));
  int rc = top_k_merge(h, k, nparts, i_ids.as<int64_t>(), i_sc.as<double>(), i_cnt.as<int32_t>(), o_ids.as<int64_t>(),
                       o_sc.as<double>(), o_cnt.as<int32_t>());
  if (rc) return rc;
  CMS_HIP(hipMemcpyAsync(out_ids, o_ids.ptr, sizeof(int64_t) * n * k, hipMemcpyDeviceToHost, h->stream));
  CMS_HIP(hipMemcpyAsync(out_scores, o_sc.ptr, sizeof(double) * n * k, hipMemcpyDeviceToHost, h->stream));
  CMS_HIP(hipMemcpyAsync(out_counts, o_cnt.ptr, sizeof(int32_t) * n, hipMemcpyDeviceToHost, h->stream));
  CMS_HIP(hipStreamSynchronize(h->stream));
  return CMS_OK;
}

int cms_write_similar_items(cms_handle* h, const char* path, int32_t k, int32_t as_float) {
  if (!h || !path) return set_error(CMS_E_PARAM, "null argument");
  if (k < 1 || k > kCandCap / 2) return set_error(CMS_E_PARAM, "k must be in [1, %d]", kCandCap / 2);
  Guard g(h);
  int rc = require_finalized(h);
  if (rc) return rc;
  return write_similar_items(h, path, k, as_float);
}

int cms_write_similarities(cms_handle* h, const char* path, int32_t k, int32_t format) {
  return cms_write_similarities_threshold(h, path, k, format, -__builtin_inf());
}

int cms_write_similarities_threshold(cms_handle* h, const char* path, int32_t k, int32_t format, double threshold) {
  if (!h || !path) return set_error(CMS_E_PARAM, "null argument");
  if (threshold != threshold) return set_error(CMS_E_PARAM, "threshold is NaN");
  if (k < 1 || k > kCandCap / 2) return set_error(CMS_E_PARAM, "k must be in [1, %d]", kCandCap / 2);
  if (format != CMS_FORMAT_ITEM_SIMILARITY_JOB && format != CMS_FORMAT_SPARK_ITEMSIMILARITY)
    return set_error(CMS_E_PARAM, "unknown output format %d", format);
  Guard g(h);
  int rc = require_finalized(h);
  if (rc) return rc;
  return write_similarities(h, path, k, format, threshold);
}

int cms_format_java_double(double v, char* buf, int32_t cap) {
  if (!buf || cap <= 0) return -1;
  return java_double_to_string(v, buf, cap);
}

int cms_read_counters(cms_handle* h, int64_t row_begin, int64_t row_count, double* out) {
  if (!h || !out) return set_error(CMS_E_PARAM, "null argument");
  if (int rc0 = refuse_per_owner(h, "cms_read_counters (use cms_read_owner_sketch)")) return rc0;
  Guard g(h);
  if (row_begin < 0 || row_count < 0 || row_begin + row_count > h->n) return set_error(CMS_E_PARAM, "row range");
  size_t cnt = (size_t)(row_count * h->dw);
  CMS_HIP(hipStreamSynchronize(h->stream));
  if (h->empty) {
    std::fill(out, out + cnt, 0.0);
    return CMS_OK;
  }
  if (h->f64) {
    if (cnt) CMS_HIP(hipMemcpy(out, h->d_t64 + row_begin * h->dw, sizeof(double) * cnt, hipMemcpyDeviceToHost));
    return CMS_OK;
  }
  // every storage form (u32 slots, u16 / u8 / nibble rows) through the
  // device read, in chunks of at most 256 MB of u32 counters
  const int64_t chunk = std::max<int64_t>(1, std::min<int64_t>(row_count, (int64_t(1) << 26) / std::max<int64_t>(h->dw, 1)));
  DevBuf tmp;
  std::vector<uint32_t> host;
  if (row_count > 0) {
    CMS_HIP(tmp.ensure(sizeof(uint32_t) * (size_t)(chunk * h->dw)));
    host.resize((size_t)(chunk * h->dw));
  }
  for (int64_t r0 = 0; r0 < row_count; r0 += chunk) {
    const int64_t rc = std::min(chunk, row_count - r0);
    int rc1 = read_counters_device(h, row_begin + r0, rc, tmp.as<uint32_t>());
    if (rc1) return rc1;
    CMS_HIP(hipMemcpyAsync(host.data(), tmp.ptr, sizeof(uint32_t) * (size_t)(rc * h->dw), hipMemcpyDeviceToHost,
                           h->stream));
    CMS_HIP(hipStreamSynchronize(h->stream));
    double* o = out + r0 * h->dw;
    for (int64_t j = 0; j < rc * h->dw; ++j) o[j] = std::ldexp((double)host[j], -h->p.frac_bits);
  }
  return CMS_OK;
}

int cms_read_counters_device(cms_handle* h, int64_t row_begin, int64_t row_count, uint32_t* d_out) {
  if (!h || (row_count > 0 && !d_out)) return set_error(CMS_E_PARAM, "null argument");
  if (int rc0 = refuse_per_owner(h, "cms_read_counters_device")) return rc0;
  if (h->f64) return set_error(CMS_E_STATE, "fp64 counters: use cms_read_counters");
  Guard g(h);
  if (row_begin < 0 || row_count < 0 || row_begin + row_count > h->n) return set_error(CMS_E_PARAM, "row range");
  return read_counters_device(h, row_begin, row_count, d_out);
}

int cms_owner_forms(cms_handle* h, int64_t row_begin, int64_t row_count, int32_t* out_form, uint32_t* out_bound) {
  if (!h) return set_error(CMS_E_PARAM, "null argument");
  if (int rc0 = refuse_per_owner(h, "cms_owner_forms")) return rc0;
  if (h->f64) return set_error(CMS_E_STATE, "fp64 counters have one form");
  Guard g(h);
  if (row_begin < 0 || row_count < 0 || row_begin + row_count > h->n) return set_error(CMS_E_PARAM, "row range");
  if (row_count == 0) return CMS_OK;
  std::vector<int32_t> hx((size_t)row_count);
  CMS_HIP(hipMemcpyAsync(hx.data(), h->d_hidx + row_begin, sizeof(int32_t) * (size_t)row_count, hipMemcpyDeviceToHost,
                         h->stream));
  if (out_bound)
    CMS_HIP(hipMemcpyAsync(out_bound, h->d_cbound + row_begin, sizeof(uint32_t) * (size_t)row_count,
                           hipMemcpyDeviceToHost, h->stream));
  CMS_HIP(hipStreamSynchronize(h->stream));
  for (int64_t i = 0; i < row_count; ++i) {
    const int32_t s = hx[(size_t)i];
    const int32_t f = s >= 0 ? CMS_FORM_U32 : s == kFormU16 ? CMS_FORM_U16 : s == kFormU8 ? CMS_FORM_U8
                    : s == kFormU4 ? CMS_FORM_U4 : s == kFormU2 ? CMS_FORM_U2 : s == kFormU1 ? CMS_FORM_U1 : CMS_FORM_LIST;
    if (out_form) out_form[i] = f;
    if (out_bound && s >= 0) out_bound[i] = 0;
  }
  return CMS_OK;
}

int cms_read_owner_sketch(cms_handle* h, int64_t id, double* out, int64_t capacity, int32_t* width, int32_t* depth) {
  if (!h) return set_error(CMS_E_PARAM, "null argument");
  if (!h->per_owner) return set_error(CMS_E_STATE, "fixed-shape handle: use cms_read_counters");
  Guard g(h);
  int rc = require_finalized(h);
  if (rc) return rc;
  int64_t row;
  if ((rc = row_of(h, id, &row))) return rc;
  if ((rc = po_require_shapes(h, &row, 1))) return rc;
  const int64_t w = h->h_po_w[row], d = h->h_po_d[row];
  if (width) *width = (int32_t)w;
  if (depth) *depth = (int32_t)d;
  if (!out) return CMS_OK;
  if (capacity < w * d) return set_error(CMS_E_PARAM, "capacity %lld < %lld counters", (long long)capacity, (long long)(w * d));
  int64_t soff = 0;
  for (int64_t r = 0; r < row; ++r) soff += (int64_t)h->h_po_w[r] * h->h_po_d[r];
  if (h->f64) {
    CMS_HIP(hipMemcpy(out, h->po_sk.as<double>() + soff, sizeof(double) * w * d, hipMemcpyDeviceToHost));
    return CMS_OK;
  }
  std::vector<uint32_t> tmp(w * d);
  CMS_HIP(hipMemcpy(tmp.data(), h->po_sk.as<uint32_t>() + soff, sizeof(uint32_t) * w * d, hipMemcpyDeviceToHost));
  for (int64_t i = 0; i < w * d; ++i) out[i] = std::ldexp((double)tmp[i], -h->p.frac_bits);
  return CMS_OK;
}

int cms_get_stats(cms_handle* h, cms_stats* out) {
  if (!h || !out) return set_error(CMS_E_PARAM, "null argument");
  const uint32_t want = out->struct_size;
  if (want < offsetof(cms_stats, pairs_ingested) + sizeof(int64_t))
    return set_error(CMS_E_PARAM, "cms_stats.struct_size %u too small (set it to sizeof(cms_stats))", want);
  cms_stats full;
  std::memset(&full, 0, sizeof(full));
  cms_stats* const dst = out;
  out = &full;
  Guard g(h);
  out->pairs_ingested = h->pairs_ingested;
  out->num_owners = h->n;
  out->depth = h->per_owner ? h->po_max_d : h->p.depth;
  out->width = h->per_owner ? h->po_max_w : h->p.width;
  out->exact_norms = h->exact_norms;
  out->world = h->world;
  out->rank = h->rank;
  int64_t forms[9] = {0, 0, 0, 0, 0, 0, 0, 0, 0};  // hot, u16, u8, 4-bit, 2-bit, 1-bit, list rows, list bytes, zero rows
  if (!h->per_owner && !h->f64 && h->d_hidx) {
    int rc = count_forms(h, forms);
    if (rc) return rc;
  }
  const int64_t hot_rows = forms[0];
  out->table_bytes = h->per_owner ? (int64_t)h->po_sk.bytes
                    : h->f64      ? (int64_t)sizeof(double) * h->n * h->dw
                                  : (int64_t)sizeof(uint16_t) * h->t16_used + (int64_t)sizeof(uint32_t) * hot_rows * h->dw;
  out->multi_limb_owners = h->mfma_ready ? (int64_t)h->n_hot_limb : -1;
  out->topk_redo = h->topk_redo;
  out->deep_limb_owners = h->mfma_ready ? h->vl[0].o1 - h->vl[0].o0 : -1;
  out->fp4_owners = h->mfma_ready ? h->n_f4 : -1;
  out->merge_words = h->merge_words;
  out->hot_rows = hot_rows;
  out->stored_bytes = h->per_owner ? (int64_t)h->po_sk.bytes
                     : h->f64      ? (int64_t)sizeof(double) * h->n * h->dw
                                   : 4 * forms[0] * h->dw + 2 * (forms[1] - forms[8]) * h->dw + forms[2] * h->dw +
                                    forms[3] * (h->dw / 2) + forms[4] * (h->dw / 4) + forms[5] * (h->dw / 8) +
                                    forms[7];
  out->u8_rows = forms[2];
  out->nibble_rows = forms[3];
  out->crumb_rows = forms[4];
  out->bit_rows = forms[5];
  out->collective_calls = h->coll_calls;
  out->comm_kind = h->comm ? 1 : h->ext_comm ? 2 : 0;
  out->device = h->device;
  out->list_rows = forms[6];
  out->po_wide_pairs = h->po_wide_pairs;
  out->po_wide_exact = h->po_wide_exact;
  out->struct_size = (uint32_t)std::min<size_t>(want, sizeof(cms_stats));
  std::memcpy(dst, out, out->struct_size);  // the fields the caller's struct has room for
  return CMS_OK;
}

int cms_set_timing(cms_handle* h, int32_t enabled) {
  if (!h) return set_error(CMS_E_PARAM, "null handle");
  h->timing = enabled <= 0 ? 0 : enabled == 1 ? 1 : 2;
  return CMS_OK;
}

int cms_get_timing(cms_handle* h, const char* name, double* total_ms, int64_t* launches) {
  if (!h || !name || !total_ms || !launches) return set_error(CMS_E_PARAM, "null argument");
  Guard g(h);
  int rc = resolve_timing(h);
  if (rc) return rc;
  if (std::strcmp(name, "host_alloc") == 0) {  // process-wide host time in hipMalloc (launches = calls)
    *total_ms = (double)g_alloc_ns.load() * 1e-6;
    *launches = g_alloc_calls.load();
    return CMS_OK;
  }
  if (std::strcmp(name, "host_alloc_bytes") == 0) {  // ... bytes allocated (in total_ms, as a count)
    *total_ms = (double)g_alloc_bytes.load();
    *launches = g_alloc_calls.load();
    return CMS_OK;
  }
  if (std::strcmp(name, "host_alloc_max") == 0) {  // the slowest single hipMalloc: ms, and its bytes in launches
    *total_ms = (double)g_alloc_max_ns.load() * 1e-6;
    *launches = g_alloc_max_bytes.load();
    return CMS_OK;
  }
  if (std::strcmp(name, "host_free") == 0) {  // process-wide host time in the hipFree of a growing buffer
    *total_ms = (double)g_free_ns.load() * 1e-6;
    *launches = 0;
    return CMS_OK;
  }
  auto it = h->timing_acc.find(name);
  *total_ms = it == h->timing_acc.end() ? 0.0 : it->second.total_ms;
  *launches = it == h->timing_acc.end() ? 0 : it->second.launches;
  return CMS_OK;
}

int cms_reset_timing(cms_handle* h) {
  if (!h) return set_error(CMS_E_PARAM, "null handle");
  Guard g(h);
  int rc = resolve_timing(h);
  h->timing_acc.clear();
  g_alloc_ns = 0;
  g_alloc_calls = 0;
  g_free_ns = 0;
  g_alloc_bytes = 0;
  g_alloc_max_ns = 0;
  g_alloc_max_bytes = 0;
  return rc;
}

}  // extern "C"
