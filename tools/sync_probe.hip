// sync_probe.hip — where a synchronous small call's ~18 us round trip goes,
// on one MI355X.  Each variant launches one tiny kernel (one workgroup that
// reads a few bytes from mapped host memory and writes a result back) and
// waits for it; median and p99 over many calls after warm-up:
//   launch+streamsync      hipLaunchKernelGGL + hipStreamSynchronize
//   launch+eventsync       ... + hipEventRecord + hipEventSynchronize
//   launch+query-spin      ... + hipStreamQuery in a spin loop
//   launch+flag-spin       the kernel ends with a system-scope release store
//                          of a sequence number into fine-grained host memory;
//                          the host spins on it (no HIP wait call at all)
//   graph+flag-spin        the same kernel as a one-node hipGraph
//   spin-sched             launch+streamsync under hipDeviceScheduleSpin
//   ./sync_probe [iters]
#include <hip/hip_runtime.h>

#include <algorithm>
#include <atomic>
#include <chrono>
#include <cstdint>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <functional>
#include <vector>

#define CK(x)                                                                    \
  do {                                                                           \
    hipError_t e_ = (x);                                                         \
    if (e_ != hipSuccess) {                                                      \
      std::fprintf(stderr, "%s:%d %s\n", __FILE__, __LINE__, hipGetErrorString(e_)); \
      std::exit(1);                                                              \
    }                                                                            \
  } while (0)

namespace {

double now_us() {
  return std::chrono::duration<double, std::micro>(std::chrono::steady_clock::now().time_since_epoch()).count();
}

// Reads n bytes of mapped host memory, writes their byte sum to res[0], then
// (if flag) publishes seq with a system-scope release store (a vector store).
__global__ void tiny(const uint8_t* __restrict__ in, uint32_t n, uint32_t* __restrict__ res,
                     uint32_t* __restrict__ flag, uint32_t seq) {
  __shared__ uint32_t tot;
  if (threadIdx.x == 0) tot = 0;
  __syncthreads();
  uint32_t s = 0;
  for (uint32_t i = threadIdx.x; i < n; i += blockDim.x) s += in[i];
  atomicAdd(&tot, s);
  __syncthreads();
  if (threadIdx.x == 0) {
    res[0] = tot;
    if (flag) __hip_atomic_store(flag, seq, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_SYSTEM);
  }
}

// One 16-B descriptor {off, len} then its payload, 16-B chunks, all from
// mapped host memory (two dependent PCIe round trips), or the descriptor by
// value in the kernel arguments (one): res[0] = byte sum, then the flag.
struct Desc {
  uint64_t off;
  uint32_t len, pad;
};
template <bool BYVAL>
__global__ void desc_then_payload(const uint8_t* __restrict__ base, const Desc* __restrict__ dptr, Desc dval,
                                  uint32_t* __restrict__ res, uint32_t* __restrict__ flag, uint32_t seq) {
  __shared__ uint32_t tot;
  if (threadIdx.x == 0) tot = 0;
  const Desc d = BYVAL ? dval : dptr[0];
  __syncthreads();
  uint32_t s = 0;
  const uint4* p = reinterpret_cast<const uint4*>(base + d.off);
  for (uint32_t i = threadIdx.x; i < d.len / 16; i += blockDim.x) {
    const uint4 v = p[i];
    s += __builtin_amdgcn_sad_u8(v.x, 0u, 0u) + __builtin_amdgcn_sad_u8(v.y, 0u, 0u) +
         __builtin_amdgcn_sad_u8(v.z, 0u, 0u) + __builtin_amdgcn_sad_u8(v.w, 0u, 0u);
  }
  atomicAdd(&tot, s);
  __syncthreads();
  if (threadIdx.x == 0) {
    res[0] = tot;
    __hip_atomic_store(flag, seq, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_SYSTEM);
  }
}

// Publishes seq into fine-grained host memory (system-scope release).
__global__ void signal(uint32_t* __restrict__ flag, uint32_t seq) {
  if (threadIdx.x == 0) __hip_atomic_store(flag, seq, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_SYSTEM);
}

struct Stat {
  double med, p99;
};

Stat time_calls(int iters, const std::function<void()>& f) {
  for (int i = 0; i < 100; ++i) f();
  std::vector<double> t(iters);
  for (int i = 0; i < iters; ++i) {
    const double a = now_us();
    f();
    t[i] = now_us() - a;
  }
  std::sort(t.begin(), t.end());
  return {t[iters / 2], t[(size_t)(iters * 0.99)]};
}

}  // namespace

int main(int argc, char** argv) {
  const int iters = argc > 1 ? std::atoi(argv[1]) : 2000;
  const bool spin_sched = argc > 2 && argv[2][0] == 's';
  if (spin_sched) CK(hipSetDeviceFlags(hipDeviceScheduleSpin));
  CK(hipSetDevice(0));
  hipStream_t s;
  CK(hipStreamCreateWithFlags(&s, hipStreamNonBlocking));
  hipEvent_t ev;
  CK(hipEventCreateWithFlags(&ev, hipEventDisableTiming));
  uint8_t* in = nullptr;  // coarse-grained mapped staging, as the library's zero-copy path
  CK(hipHostMalloc(reinterpret_cast<void**>(&in), 1 << 16, hipHostMallocMapped | hipHostMallocNonCoherent));
  uint32_t* res = nullptr;
  uint32_t* flag = nullptr;  // fine-grained (coherent) host memory for the flag
  CK(hipHostMalloc(reinterpret_cast<void**>(&res), 64, hipHostMallocMapped | hipHostMallocCoherent));
  CK(hipHostMalloc(reinterpret_cast<void**>(&flag), 64, hipHostMallocMapped | hipHostMallocCoherent));
  for (int i = 0; i < (1 << 16); ++i) in[i] = (uint8_t)(i * 7);
  uint8_t* din;
  uint32_t *dres, *dflag;
  CK(hipHostGetDevicePointer(reinterpret_cast<void**>(&din), in, 0));
  CK(hipHostGetDevicePointer(reinterpret_cast<void**>(&dres), res, 0));
  CK(hipHostGetDevicePointer(reinterpret_cast<void**>(&dflag), flag, 0));
  const uint32_t n = 1500;
  uint32_t want = 0;
  for (uint32_t i = 0; i < n; ++i) want += in[i];
  uint32_t seq = 0;
  long bad = 0;
  auto check = [&] {
    if (__atomic_load_n(res, __ATOMIC_ACQUIRE) != want) ++bad;
  };
  auto spin_flag = [&](uint32_t q) {
    const double t0 = now_us();
    while (__atomic_load_n(flag, __ATOMIC_ACQUIRE) != q) {
      if (now_us() - t0 > 2e6) {
        std::fprintf(stderr, "flag timeout\n");
        std::exit(2);
      }
    }
  };

  std::printf("{\n \"schedule\": \"%s\", \"bytes\": %u, \"iters\": %d,\n", spin_sched ? "spin" : "auto", n, iters);
  Stat a = time_calls(iters, [&] {
    hipLaunchKernelGGL(tiny, dim3(1), dim3(256), 0, s, din, n, dres, nullptr, 0u);
    CK(hipStreamSynchronize(s));
    check();
  });
  std::printf(" \"launch_streamsync\": {\"med_us\": %.2f, \"p99_us\": %.2f},\n", a.med, a.p99);
  Stat b = time_calls(iters, [&] {
    hipLaunchKernelGGL(tiny, dim3(1), dim3(256), 0, s, din, n, dres, nullptr, 0u);
    CK(hipEventRecord(ev, s));
    CK(hipEventSynchronize(ev));
    check();
  });
  std::printf(" \"launch_eventsync\": {\"med_us\": %.2f, \"p99_us\": %.2f},\n", b.med, b.p99);
  Stat c = time_calls(iters, [&] {
    hipLaunchKernelGGL(tiny, dim3(1), dim3(256), 0, s, din, n, dres, nullptr, 0u);
    while (hipStreamQuery(s) == hipErrorNotReady) {
    }
    check();
  });
  std::printf(" \"launch_query_spin\": {\"med_us\": %.2f, \"p99_us\": %.2f},\n", c.med, c.p99);
  Stat d = time_calls(iters, [&] {
    ++seq;
    hipLaunchKernelGGL(tiny, dim3(1), dim3(256), 0, s, din, n, dres, dflag, seq);
    spin_flag(seq);
    check();
  });
  std::printf(" \"launch_flag_spin\": {\"med_us\": %.2f, \"p99_us\": %.2f},\n", d.med, d.p99);
  Stat d2 = time_calls(iters, [&] {
    ++seq;
    hipLaunchKernelGGL(tiny, dim3(1), dim3(256), 0, s, din, n, dres, nullptr, 0u);
    hipLaunchKernelGGL(signal, dim3(1), dim3(64), 0, s, dflag, seq);
    spin_flag(seq);
    check();
  });
  std::printf(" \"launch_signal_kernel_spin\": {\"med_us\": %.2f, \"p99_us\": %.2f},\n", d2.med, d2.p99);
  {
    Desc* hd = nullptr;  // coarse-grained mapped, as the library's pass table
    CK(hipHostMalloc(reinterpret_cast<void**>(&hd), 64, hipHostMallocMapped | hipHostMallocNonCoherent));
    Desc* ddv;
    CK(hipHostGetDevicePointer(reinterpret_cast<void**>(&ddv), hd, 0));
    hd->off = 0;
    hd->len = 1504;
    uint32_t w2 = 0;
    for (uint32_t i = 0; i < 1504; ++i) w2 += in[i];
    long bad2 = 0;
    Stat x = time_calls(iters, [&] {
      ++seq;
      hipLaunchKernelGGL((desc_then_payload<false>), dim3(1), dim3(128), 0, s, din, ddv, Desc{}, dres, dflag, seq);
      spin_flag(seq);
      if (__atomic_load_n(res, __ATOMIC_ACQUIRE) != w2) ++bad2;
    });
    std::printf(" \"desc_in_host_memory_then_payload\": {\"med_us\": %.2f, \"p99_us\": %.2f},\n", x.med, x.p99);
    Stat y = time_calls(iters, [&] {
      ++seq;
      hipLaunchKernelGGL((desc_then_payload<true>), dim3(1), dim3(128), 0, s, din, nullptr, *hd, dres, dflag, seq);
      spin_flag(seq);
      if (__atomic_load_n(res, __ATOMIC_ACQUIRE) != w2) ++bad2;
    });
    std::printf(" \"desc_by_value_then_payload\": {\"med_us\": %.2f, \"p99_us\": %.2f},\n", y.med, y.p99);
    bad += bad2;
    CK(hipStreamSynchronize(s));
    CK(hipHostFree(hd));
  }
  {
    // Fine-grained device memory the CPU writes through the BAR: the
    // descriptor and the payload staged in HBM by host stores, read by the
    // kernel from local memory (no PCIe read round trip).
    uint8_t* vram = nullptr;
    hipError_t e = hipExtMallocWithFlags(reinterpret_cast<void**>(&vram), 1 << 16, hipDeviceMallocFinegrained);
    hipPointerAttribute_t at{};
    // argv[3] == "direct": dereference the device address on the host (SVM
    // over a large BAR); a fault ends only this process
    const bool direct = argc > 3 && argv[3][0] == 'd';
    const bool ok = e == hipSuccess && hipPointerGetAttributes(&at, vram) == hipSuccess && (at.hostPointer || direct);
    std::printf(" \"vram_finegrained_host_ptr\": %s, \"direct\": %s,\n", at.hostPointer ? "true" : "false",
                direct ? "true" : "false");
    std::fflush(stdout);
    if (ok) {
      uint8_t* hv = at.hostPointer ? static_cast<uint8_t*>(at.hostPointer) : vram;
      Desc* vd = reinterpret_cast<Desc*>(hv + 4096);
      uint32_t w3 = 0;
      for (uint32_t i = 0; i < 1504; ++i) w3 += in[i];
      long bad3 = 0;
      // freshness: every call stages different bytes (the previous call's
      // lines may sit in the GPU's L2); the kernel must sum the new ones
      std::vector<uint8_t> pat(1504);
      Stat zf = time_calls(iters, [&] {
        ++seq;
        uint32_t w = 0;
        for (uint32_t i = 0; i < 1504; ++i) w += (pat[i] = (uint8_t)(seq * 131u + i * 7u));
        std::memcpy(hv, pat.data(), 1504);
        vd->off = 0;
        vd->len = 1504;
        std::atomic_thread_fence(std::memory_order_seq_cst);
        hipLaunchKernelGGL((desc_then_payload<false>), dim3(1), dim3(128), 0, s, vram,
                           reinterpret_cast<const Desc*>(vram + 4096), Desc{}, dres, dflag, seq);
        spin_flag(seq);
        if (__atomic_load_n(res, __ATOMIC_ACQUIRE) != w) ++bad3;
      });
      std::printf(" \"vram_staged_fresh_bytes_each_call\": {\"med_us\": %.2f, \"wrong\": %ld},\n", zf.med, bad3);
      Stat z = time_calls(iters, [&] {
        ++seq;
        std::memcpy(hv, in, 1504);  // the staging copy, into HBM
        vd->off = 0;
        vd->len = 1504;
        std::atomic_thread_fence(std::memory_order_seq_cst);
        hipLaunchKernelGGL((desc_then_payload<false>), dim3(1), dim3(128), 0, s, vram,
                           reinterpret_cast<const Desc*>(vram + 4096), Desc{}, dres, dflag, seq);
        spin_flag(seq);
        if (__atomic_load_n(res, __ATOMIC_ACQUIRE) != w3) ++bad3;
      });
      std::printf(" \"vram_staged_desc_and_payload\": {\"med_us\": %.2f, \"p99_us\": %.2f, \"wrong\": %ld},\n",
                  z.med, z.p99, bad3);
      std::vector<uint8_t> big(1 << 16, 7);
      const double tw0 = now_us();
      for (int r = 0; r < 100; ++r) std::memcpy(hv, big.data(), 1 << 16);
      std::atomic_thread_fence(std::memory_order_seq_cst);
      std::printf(" \"cpu_write_to_vram_GBps\": %.2f,\n", 100.0 * 65536 / (now_us() - tw0) / 1e3);
      CK(hipStreamSynchronize(s));
      CK(hipFree(vram));
    } else {
      (void)hipGetLastError();
    }
  }
  Stat wv = time_calls(iters, [&] {
    ++seq;
    hipLaunchKernelGGL(tiny, dim3(1), dim3(256), 0, s, din, n, dres, nullptr, 0u);
    CK(hipStreamWriteValue32(s, dflag, seq, 0));
    spin_flag(seq);
    check();
  });
  std::printf(" \"launch_streamwritevalue_spin\": {\"med_us\": %.2f, \"p99_us\": %.2f},\n", wv.med, wv.p99);
  Stat d5 = time_calls(iters, [&] {
    ++seq;
    hipLaunchKernelGGL(tiny, dim3(1), dim3(256), 0, s, din, n, dres, nullptr, 0u);
    hipLaunchKernelGGL(signal, dim3(1), dim3(64), 0, s, dflag, seq);
    spin_flag(seq);
    CK(hipStreamSynchronize(s));
    check();
  });
  std::printf(" \"launch_signal_kernel_spin_then_streamsync\": {\"med_us\": %.2f, \"p99_us\": %.2f},\n", d5.med, d5.p99);
  Stat d6 = time_calls(iters, [&] {
    ++seq;
    hipLaunchKernelGGL(tiny, dim3(1), dim3(256), 0, s, din, n, dres, dflag, seq);
    spin_flag(seq);
    CK(hipStreamSynchronize(s));
    check();
  });
  std::printf(" \"launch_flag_spin_then_streamsync\": {\"med_us\": %.2f, \"p99_us\": %.2f},\n", d6.med, d6.p99);
  Stat d3 = time_calls(iters, [&] {
    ++seq;
    hipLaunchKernelGGL(tiny, dim3(1), dim3(256), 0, s, din, 0u, dres, dflag, seq);
    spin_flag(seq);
  });
  std::printf(" \"no_read_flag_spin\": {\"med_us\": %.2f, \"p99_us\": %.2f},\n", d3.med, d3.p99);
  Stat d4 = time_calls(iters, [&] {
    hipLaunchKernelGGL(tiny, dim3(1), dim3(256), 0, s, din, 0u, dres, nullptr, 0u);
    CK(hipStreamSynchronize(s));
  });
  std::printf(" \"no_read_streamsync\": {\"med_us\": %.2f, \"p99_us\": %.2f},\n", d4.med, d4.p99);
  // launch cost alone (no wait), amortised over a burst
  CK(hipStreamSynchronize(s));
  const double t0 = now_us();
  for (int i = 0; i < 200; ++i) hipLaunchKernelGGL(tiny, dim3(1), dim3(256), 0, s, din, n, dres, nullptr, 0u);
  const double t1 = now_us();
  CK(hipStreamSynchronize(s));
  const double t2 = now_us();
  std::printf(" \"launch_cpu_us\": %.2f, \"burst_gpu_us_per_kernel\": %.2f,\n", (t1 - t0) / 200, (t2 - t0) / 200);
  // one-node graph whose kernel args carry a fixed seq: re-instantiate per
  // seq would dominate, so the graph writes a constant and the host resets it
  hipGraph_t g;
  hipGraphExec_t ge;
  CK(hipStreamBeginCapture(s, hipStreamCaptureModeThreadLocal));
  hipLaunchKernelGGL(tiny, dim3(1), dim3(256), 0, s, din, n, dres, dflag, 0xFFFFFFFFu);
  CK(hipStreamEndCapture(s, &g));
  CK(hipGraphInstantiate(&ge, g, nullptr, nullptr, 0));
  Stat e = time_calls(iters, [&] {
    __atomic_store_n(flag, 0u, __ATOMIC_RELEASE);
    CK(hipGraphLaunch(ge, s));
    spin_flag(0xFFFFFFFFu);
    check();
  });
  CK(hipStreamSynchronize(s));
  std::printf(" \"graph_flag_spin\": {\"med_us\": %.2f, \"p99_us\": %.2f},\n", e.med, e.p99);
  std::printf(" \"wrong\": %ld\n}\n", bad);
  CK(hipGraphExecDestroy(ge));
  CK(hipGraphDestroy(g));
  CK(hipStreamDestroy(s));
  return bad ? 1 : 0;
}
