// Probe: cost of small in-place stores into a large packet arena on MI355X.
// 2M stores at the TX checksum positions (packet stride 1504 B, bytes 10 and
// 36) with different widths, each after (or without) a streaming read of the
// arena, to see whether sub-sector writes pay a read-modify-write in HBM.
//   hipcc -O3 --offload-arch=gfx950 tools/store_probe.hip -o tools/store_probe
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdint>
#include <vector>

#define CK(x) do { hipError_t e = (x); if (e != hipSuccess) { printf("%s\n", hipGetErrorString(e)); return 1; } } while (0)

constexpr uint64_t N = 1 << 20, STRIDE = 1504;

// W = bytes written per store: 1 (two byte stores), 2, 16, 32, 64 (aligned
// segment holding the field; rewrites the bytes it read), 128
template <int W>
__global__ void store_k(uint8_t* a) {
  const uint64_t j = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (j >= 2 * N) return;
  const uint64_t at = (j >> 1) * STRIDE + ((j & 1) ? 36 : 10);
  if constexpr (W == 1) {
    a[at] = (uint8_t)j; a[at + 1] = (uint8_t)(j >> 8);
  } else if constexpr (W == 2) {
    *reinterpret_cast<uint16_t*>(a + at) = (uint16_t)j;
  } else {
    // only the even j (the byte-10 field) so two stores never share a segment
    if (j & 1) return;
    const uint64_t s = at & ~(uint64_t)(W - 1);
    uint4* p = reinterpret_cast<uint4*>(a + s);
#pragma unroll
    for (int k = 0; k < W / 16; ++k) { uint4 v = p[k]; v.x ^= 1; p[k] = v; }
  }
}

__global__ void read_k(const uint4* a, uint64_t n16, uint32_t* out) {
  uint32_t acc = 0;
  for (uint64_t k = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; k < n16; k += (uint64_t)gridDim.x * blockDim.x) {
    uint4 v = a[k];
    acc += v.x ^ v.y ^ v.z ^ v.w;
  }
  if (acc == 0x12345678) out[0] = acc;
}

template <int W>
float time_store(uint8_t* a, hipEvent_t e0, hipEvent_t e1) {
  const uint32_t grid = (uint32_t)((2 * N + 255) / 256);
  store_k<W><<<grid, 256>>>(a);
  hipEventRecord(e0);
  for (int r = 0; r < 20; ++r) store_k<W><<<grid, 256>>>(a);
  hipEventRecord(e1);
  hipEventSynchronize(e1);
  float ms = 0;
  hipEventElapsedTime(&ms, e0, e1);
  return ms / 20 * 1e3f;
}

int main() {
  uint8_t* a;
  uint32_t* o;
  const uint64_t bytes = N * STRIDE;
  CK(hipMalloc(&a, bytes));
  CK(hipMalloc(&o, 64));
  CK(hipMemset(a, 1, bytes));
  hipEvent_t e0, e1;
  hipEventCreate(&e0);
  hipEventCreate(&e1);
  printf("store-only us per 2M-position pass (W=64/128/16/32: 1M stores):\n");
  printf("  W=1  (2 byte stores) %8.1f\n", time_store<1>(a, e0, e1));
  printf("  W=2  (u16)           %8.1f\n", time_store<2>(a, e0, e1));
  printf("  W=16 seg (1M)        %8.1f\n", time_store<16>(a, e0, e1));
  printf("  W=32 seg (1M)        %8.1f\n", time_store<32>(a, e0, e1));
  printf("  W=64 seg (1M)        %8.1f\n", time_store<64>(a, e0, e1));
  printf("  W=128 seg (1M)       %8.1f\n", time_store<128>(a, e0, e1));
  // streaming read of the arena, then read + stores (same stream, serial)
  read_k<<<4096, 256>>>((const uint4*)a, bytes / 16, o);
  hipEventRecord(e0);
  for (int r = 0; r < 20; ++r) read_k<<<4096, 256>>>((const uint4*)a, bytes / 16, o);
  hipEventRecord(e1);
  hipEventSynchronize(e1);
  float ms;
  hipEventElapsedTime(&ms, e0, e1);
  printf("read-only pass %8.1f us\n", ms / 20 * 1e3f);
  CK(hipDeviceSynchronize());
  return 0;
}
