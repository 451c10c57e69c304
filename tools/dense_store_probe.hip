// dense_store_probe.hip — what the TX fill's checksum stores cost in
// sendTCPBatch's dense header layout, written three ways
// after a 1.5 GB read has evicted every cache (as in the product, where the
// payload stream runs between a tile's header reads and the next tile's):
//   sparse    2M 2-byte stores, two per 54-B slot (the product's stores:
//             relaxed agent-scope, written through)
//   rewrite   every slot's bytes read back and written whole (16-B loads and
//             stores over the 57 MB header region), the two fields patched
//   overwrite the same 16-B stores without the read (a floor: not correct)
// Each variant: 10 rounds of [read 1.5 GB, then the stores], the stores
// timed alone by an event pair around them.  ./dense_store_probe
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cstdint>
#include <cstdio>
#include <vector>

#define CK(x)                                                                         \
  do {                                                                                \
    hipError_t e_ = (x);                                                              \
    if (e_ != hipSuccess) {                                                           \
      std::fprintf(stderr, "%s:%d %s\n", __FILE__, __LINE__, hipGetErrorString(e_)); \
      return 1;                                                                       \
    }                                                                                 \
  } while (0)

namespace {

constexpr uint32_t kSlot = 54, kIp = 24, kTcp = 50;

__global__ __launch_bounds__(256) void stream_read(const uint4* __restrict__ p, uint64_t n, uint32_t* __restrict__ sink) {
  uint32_t s = 0;
  for (uint64_t i = (uint64_t)blockIdx.x * 256 + threadIdx.x; i < n; i += (uint64_t)gridDim.x * 256) {
    const uint4 v = p[i];
    s += v.x ^ v.y ^ v.z ^ v.w;
  }
  if (s == 0x12345678u) sink[0] = s;  // never, but the loads stay live
}

__global__ __launch_bounds__(256) void sparse_stores(uint8_t* __restrict__ hdr, uint32_t n) {
  const uint32_t i = blockIdx.x * 256 + threadIdx.x;
  if (i >= n) return;
  uint16_t* a = reinterpret_cast<uint16_t*>(hdr + (uint64_t)i * kSlot + kIp);
  uint16_t* b = reinterpret_cast<uint16_t*>(hdr + (uint64_t)i * kSlot + kTcp);
  __hip_atomic_store(a, (uint16_t)i, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  __hip_atomic_store(b, (uint16_t)~i, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}

template <bool READ>
__global__ __launch_bounds__(256) void rewrite(uint4* __restrict__ hdr, uint64_t nchunks) {
  const uint64_t i = (uint64_t)blockIdx.x * 256 + threadIdx.x;
  if (i >= nchunks) return;
  uint4 v = READ ? hdr[i] : make_uint4((uint32_t)i, 0, 0, 0);
  v.x += 1;  // stands for the patched fields
  hdr[i] = v;
}

}  // namespace

int main() {
  const uint32_t n = 1u << 20;
  const uint64_t hdr_bytes = ((uint64_t)n * kSlot + 4095) / 4096 * 4096;
  const uint64_t pay_bytes = (uint64_t)n * 1460;
  uint8_t* arena = nullptr;
  uint32_t* sink = nullptr;
  CK(hipMalloc(&arena, hdr_bytes + pay_bytes));
  CK(hipMalloc(&sink, 64));
  CK(hipMemset(arena, 7, hdr_bytes + pay_bytes));
  hipStream_t s;
  CK(hipStreamCreate(&s));
  hipEvent_t a, b;
  CK(hipEventCreate(&a));
  CK(hipEventCreate(&b));
  const uint64_t pay16 = pay_bytes / 16, hdr16 = hdr_bytes / 16;
  const char* names[3] = {"sparse", "rewrite", "overwrite"};
  std::printf("{\n \"header_region_MB\": %.1f, \"payload_MB\": %.1f,\n", hdr_bytes / 1e6, pay_bytes / 1e6);
  for (int v = 0; v < 3; ++v) {
    std::vector<float> t;
    for (int r = 0; r < 11; ++r) {
      hipLaunchKernelGGL(stream_read, dim3(4096), dim3(256), 0, s, reinterpret_cast<const uint4*>(arena + hdr_bytes),
                         pay16, sink);
      CK(hipEventRecord(a, s));
      if (v == 0) hipLaunchKernelGGL(sparse_stores, dim3(n / 256), dim3(256), 0, s, arena, n);
      if (v == 1) hipLaunchKernelGGL(rewrite<true>, dim3((uint32_t)((hdr16 + 255) / 256)), dim3(256), 0, s,
                                     reinterpret_cast<uint4*>(arena), hdr16);
      if (v == 2) hipLaunchKernelGGL(rewrite<false>, dim3((uint32_t)((hdr16 + 255) / 256)), dim3(256), 0, s,
                                     reinterpret_cast<uint4*>(arena), hdr16);
      CK(hipEventRecord(b, s));
      CK(hipEventSynchronize(b));
      float ms = 0;
      CK(hipEventElapsedTime(&ms, a, b));
      if (r) t.push_back(ms * 1000.0f);
    }
    std::sort(t.begin(), t.end());
    std::printf(" \"%s_us\": {\"median\": %.1f, \"min\": %.1f, \"max\": %.1f}%s\n", names[v], t[t.size() / 2], t[0],
                t.back(), v < 2 ? "," : "");
  }
  std::printf("}\n");
  CK(hipFree(arena));
  return 0;
}
