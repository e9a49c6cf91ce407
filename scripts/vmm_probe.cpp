// Probe of the HIP virtual memory calls the compact row arena uses
// (cms_table.hip arena_map): chunks mapped one after another at the end of
// one reserved range, with ordinary allocations in between (a sub-range
// hipMemSetAccess is refused then; the whole range from the start is not),
// and what mapping costs: hipMemCreate / hipMemMap / hipMemSetAccess times
// for growing chunk sizes against hipMalloc of the same bytes.
#include <hip/hip_runtime.h>
#include <chrono>
#include <cstdio>
#define P(x) do { hipError_t e_ = (x); printf("%-72s -> %s\n", #x, hipGetErrorString(e_)); } while (0)
static double now_ms() {
  return std::chrono::duration<double, std::milli>(std::chrono::steady_clock::now().time_since_epoch()).count();
}
int main() {
  hipMemAllocationProp prop = {};
  prop.type = hipMemAllocationTypePinned;
  prop.location.type = hipMemLocationTypeDevice;
  prop.location.id = 0;
  hipMemAccessDesc acc = {};
  acc.location = prop.location;
  acc.flags = hipMemAccessFlagsProtReadWrite;
  const size_t g = 64 << 20, va_bytes = size_t(2048) * g;  // 128 GB of range
  void* va = nullptr;
  P(hipMemAddressReserve(&va, va_bytes, g, nullptr, 0));
  void* other = nullptr;
  P(hipMalloc(&other, g));
  size_t mapped = 0;
  const size_t chunks[] = {g, 16 * g, 64 * g, 256 * g};  // 64 MB .. 16 GB
  for (size_t c : chunks) {
    hipMemGenericAllocationHandle_t m;
    double t0 = now_ms();
    hipError_t e1 = hipMemCreate(&m, c, &prop, 0);
    double t1 = now_ms();
    hipError_t e2 = hipMemMap((char*)va + mapped, c, 0, m, 0);
    double t2 = now_ms();
    hipError_t e3 = hipMemSetAccess(va, mapped + c, &acc, 1);
    double t3 = now_ms();
    mapped += c;
    printf("chunk %6.2f GB: create %8.2f ms (%s) map %7.2f ms (%s) access(whole %6.2f GB) %8.2f ms (%s)\n", c / 1e9,
           t1 - t0, hipGetErrorString(e1), t2 - t1, hipGetErrorString(e2), mapped / 1e9, t3 - t2, hipGetErrorString(e3));
  }
  double t0 = now_ms();
  P(hipMemsetD8((hipDeviceptr_t)va, 1, mapped));
  P(hipDeviceSynchronize());
  printf("memset %.2f GB over the mapped range: %.2f ms\n", mapped / 1e9, now_ms() - t0);
  for (size_t c : {16 * g, 256 * g}) {
    void* p = nullptr;
    double a = now_ms();
    hipError_t e = hipMalloc(&p, c);
    double b = now_ms();
    hipMemsetD8((hipDeviceptr_t)p, 1, c);
    hipDeviceSynchronize();
    double d = now_ms();
    printf("hipMalloc %6.2f GB: %8.2f ms (%s), memset %.2f ms\n", c / 1e9, b - a, hipGetErrorString(e), d - b);
    hipFree(p);
  }
  return 0;
}
