// server_probe.hip — how fast a resident workgroup answers a small request,
// against a launch per request.  One wave polls a
// doorbell word in fine-grained VRAM that the host writes through the BAR;
// on a new sequence number it (optionally) sums a 1500-B payload staged in
// VRAM and answers with a system-scope release store into coherent host
// memory, which the host spins on.  The server exits on a quit word, after
// `idle` without a request, or after `life` in all, whichever comes first,
// so no wave outlives the probe.  Median and p99 over many requests:
//   server            doorbell -> answer
//   server+1500B      ... with the payload summed before answering
//   launch+flag       one tiny kernel per request ending in the same answer
//   ./server_probe [iters]
#include <hip/hip_runtime.h>

#include <algorithm>
#include <chrono>
#include <cstdint>
#include <cstdio>
#include <cstdlib>
#include <vector>

#define CK(x)                                                                         \
  do {                                                                                \
    hipError_t e_ = (x);                                                              \
    if (e_ != hipSuccess) {                                                           \
      std::fprintf(stderr, "%s:%d %s\n", __FILE__, __LINE__, hipGetErrorString(e_)); \
      std::exit(1);                                                                   \
    }                                                                                 \
  } while (0)

namespace {

constexpr uint32_t kQuit = 0xFFFFFFFFu;

double now_us() {
  return std::chrono::duration<double, std::micro>(std::chrono::steady_clock::now().time_since_epoch()).count();
}

__device__ __forceinline__ uint32_t sum_bytes(const uint8_t* p, uint32_t n) {
  uint32_t s = 0;
  for (uint32_t i = threadIdx.x * 16; i + 16 <= n; i += 64 * 16) {
    const uint4 v = *reinterpret_cast<const uint4*>(p + i);
    s += __builtin_amdgcn_sad_u8(v.x, 0u, 0u) + __builtin_amdgcn_sad_u8(v.y, 0u, 0u) +
         __builtin_amdgcn_sad_u8(v.z, 0u, 0u) + __builtin_amdgcn_sad_u8(v.w, 0u, 0u);
  }
  for (int o = 32; o > 0; o >>= 1) s += __shfl_xor(s, o, 64);
  return s;
}

// One wave.  Every lane runs the same loop on wave-uniform values, so every
// lane reaches the exit together.  100 MHz s_memrealtime ticks.
__global__ __launch_bounds__(64) void server(const uint32_t* db, uint32_t* reply, const uint8_t* payload,
                                            uint32_t nbytes, uint64_t idle, uint64_t life) {
  const uint64_t start = __builtin_amdgcn_s_memrealtime();
  uint64_t last_act = start;
  uint32_t last = 0;
  while (true) {
    uint32_t v = 0;
    if (threadIdx.x == 0) v = __hip_atomic_load(db, __ATOMIC_ACQUIRE, __HIP_MEMORY_SCOPE_SYSTEM);
    v = __shfl(v, 0, 64);
    const uint64_t now = __builtin_amdgcn_s_memrealtime();
    if (v == kQuit || now - start > life || now - last_act > idle) break;
    if (v != last) {
      last = v;
      uint32_t s = nbytes ? sum_bytes(payload, nbytes) : 0u;
      if (threadIdx.x == 0) {
        reply[1] = s;
        __hip_atomic_store(reply, v, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_SYSTEM);
      }
      last_act = now;
    } else {
      __builtin_amdgcn_s_sleep(1);
    }
  }
}

__global__ __launch_bounds__(64) void tiny(uint32_t* reply, const uint8_t* payload, uint32_t nbytes, uint32_t seq) {
  uint32_t s = nbytes ? sum_bytes(payload, nbytes) : 0u;
  if (threadIdx.x == 0) {
    reply[1] = s;
    __hip_atomic_store(reply, seq, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_SYSTEM);
  }
}

struct Stat {
  double med, p99;
  int lost;
};

Stat stats(std::vector<double>& t, int lost) {
  std::sort(t.begin(), t.end());
  if (t.empty()) return {0, 0, lost};
  return {t[t.size() / 2], t[(size_t)(t.size() * 0.99)], lost};
}

// Spin until reply[0] == seq, at most 50 ms; false if it never came.
bool wait_reply(volatile uint32_t* reply, uint32_t seq) {
  const double t0 = now_us();
  while (__atomic_load_n(const_cast<uint32_t*>(reply), __ATOMIC_ACQUIRE) != seq)
    if (now_us() - t0 > 50000) return false;
  return true;
}

}  // namespace

int main(int argc, char** argv) {
  const int iters = argc > 1 ? std::atoi(argv[1]) : 3000;
  int large_bar = 0;
  CK(hipDeviceGetAttribute(&large_bar, hipDeviceAttributeIsLargeBar, 0));
  uint32_t* db = nullptr;  // the doorbell: VRAM the host writes through the BAR (else mapped host memory)
  if (large_bar) {
    CK(hipExtMallocWithFlags(reinterpret_cast<void**>(&db), 256, hipDeviceMallocFinegrained));
  } else {
    CK(hipHostMalloc(reinterpret_cast<void**>(&db), 256, hipHostMallocMapped | hipHostMallocCoherent));
  }
  uint32_t* reply = nullptr;
  uint32_t* reply_dev = nullptr;
  CK(hipHostMalloc(reinterpret_cast<void**>(&reply), 256, hipHostMallocMapped | hipHostMallocCoherent));
  CK(hipHostGetDevicePointer(reinterpret_cast<void**>(&reply_dev), reply, 0));
  uint8_t* payload = nullptr;
  CK(hipMalloc(reinterpret_cast<void**>(&payload), 4096));
  std::vector<uint8_t> hp(4096);
  for (size_t i = 0; i < hp.size(); ++i) hp[i] = (uint8_t)(i * 131 + 7);
  CK(hipMemcpy(payload, hp.data(), hp.size(), hipMemcpyHostToDevice));
  uint32_t want1500 = 0;
  for (int i = 0; i < 1488; ++i) want1500 += hp[i];  // the lanes' whole 16-B chunks of 1500 B
  hipStream_t s;
  CK(hipStreamCreateWithFlags(&s, hipStreamNonBlocking));
  volatile uint32_t* rep = reply;
  std::printf("{\n \"large_bar\": %d,\n", large_bar);
  uint32_t seq = 0;
  int bad_sum = 0;
  for (uint32_t nbytes : {0u, 1500u}) {
    __atomic_store_n(db, 0u, __ATOMIC_RELEASE);
    __builtin_ia32_sfence();
    __atomic_store_n(reply, 0u, __ATOMIC_RELEASE);
    seq = 0;
    // idle 20 ms, life 3 s (100 MHz ticks)
    hipLaunchKernelGGL(server, dim3(1), dim3(64), 0, s, db, reply_dev, payload, nbytes, 2000000ull, 300000000ull);
    CK(hipGetLastError());
    std::vector<double> t;
    int lost = 0;
    for (int k = 0; k < iters + 100; ++k) {
      ++seq;
      const double a = now_us();
      __atomic_store_n(db, seq, __ATOMIC_RELEASE);
      __builtin_ia32_sfence();
      if (!wait_reply(rep, seq)) {
        ++lost;
        break;  // the server is gone (timed out): stop this variant
      }
      const double b = now_us();
      if (nbytes && rep[1] != want1500) ++bad_sum;
      if (k >= 100) t.push_back(b - a);
    }
    __atomic_store_n(db, kQuit, __ATOMIC_RELEASE);
    __builtin_ia32_sfence();
    CK(hipStreamSynchronize(s));
    const Stat st = stats(t, lost);
    std::printf(" \"server_%uB\": {\"med_us\": %.2f, \"p99_us\": %.2f, \"lost\": %d, \"n\": %zu},\n", nbytes, st.med,
                st.p99, st.lost, t.size());
  }
  for (uint32_t nbytes : {0u, 1500u}) {
    std::vector<double> t;
    int lost = 0;
    for (int k = 0; k < iters + 100; ++k) {
      ++seq;
      const double a = now_us();
      hipLaunchKernelGGL(tiny, dim3(1), dim3(64), 0, s, reply_dev, payload, nbytes, seq);
      if (!wait_reply(rep, seq)) {
        ++lost;
        break;
      }
      const double b = now_us();
      if (nbytes && rep[1] != want1500) ++bad_sum;
      if (k >= 100) t.push_back(b - a);
    }
    CK(hipStreamSynchronize(s));
    const Stat st = stats(t, lost);
    std::printf(" \"launch_%uB\": {\"med_us\": %.2f, \"p99_us\": %.2f, \"lost\": %d, \"n\": %zu},\n", nbytes, st.med,
                st.p99, st.lost, t.size());
  }
  std::printf(" \"bad_sums\": %d\n}\n", bad_sum);
  CK(hipStreamDestroy(s));
  return bad_sum != 0;
}
