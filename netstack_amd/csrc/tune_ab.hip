// tune_ab.hip — NOT part of the product ABI.  A small A/B library with the
// same entry points as libns_tune.so (nsk_tune_count / _name / _launch), so
// tools/tune.py --lib can time a handful of kernel variants without building
// the full tuning library (which instantiates every probe: ~8 minutes).
#include "csum_kernels.hip"

namespace nsk {

// Production launch (the launcher's own TP rule) and fixed-TP instances.
template <int QS, int AUXB = 2>
hipError_t ab_auto(const uint8_t* arena, uint64_t arena_bytes, const void* desc, uint32_t n, uint16_t* out,
                   unsigned long long* err, hipStream_t s) {
  return launch_hyb<8, 16, 4, AUXB, 0, 2, QS>(arena, arena_bytes, desc, n, out, nullptr, err, s, kBigChunks);
}
template <int TP, int QS>
hipError_t ab_tp(const uint8_t* arena, uint64_t arena_bytes, const void* desc, uint32_t n, uint16_t* out,
                 unsigned long long* err, hipStream_t s) {
  const uint32_t grid = (uint32_t)(((uint64_t)n + TP - 1) / TP);
  hipLaunchKernelGGL((csum_hyb<256, TP, 8, 16, 4, 2, 0, false, 2, QS, false>), dim3(grid), dim3(256), 0, s, arena,
                     arena_bytes, reinterpret_cast<const uint4*>(desc), n, out, nullptr, err, kBigChunks, 0u,
                     nullptr, nullptr, 0u, 0u);
  return hipGetLastError();
}

typedef hipError_t (*ab_fn)(const uint8_t*, uint64_t, const void*, uint32_t, uint16_t*, unsigned long long*,
                            hipStream_t);
struct AbVariant {
  const char* name;
  ab_fn fn;
};
static const AbVariant kAb[] = {
    {"prod", ab_auto<0>},
    {"big_sc1nt", ab_auto<0, 18>},
    {"big_sc0nt", ab_auto<0, 3>},
    {"big_sc0sc1nt", ab_auto<0, 19>},
    {"big_sc1", ab_auto<0, 16>},
    {"small_sc1", ab_auto<16 << 10>},
    {"small_sc0", ab_auto<1 << 10>},
    {"small_nt", ab_auto<2 << 10>},
    {"small_sc1nt", ab_auto<18 << 10>},
};

}  // namespace nsk

extern "C" {
int nsk_tune_count(void) { return (int)(sizeof(nsk::kAb) / sizeof(nsk::kAb[0])); }
const char* nsk_tune_name(int v) { return v >= 0 && v < nsk_tune_count() ? nsk::kAb[v].name : ""; }
int nsk_tune_launch(int v, const void* arena, uint64_t arena_bytes, const void* desc, uint32_t n, void* out,
                    void* err, void* stream) {
  if (v < 0 || v >= nsk_tune_count() || n == 0) return -1;
  return nsk::kAb[v].fn((const uint8_t*)arena, arena_bytes, desc, n, (uint16_t*)out, (unsigned long long*)err,
                        (hipStream_t)stream) == hipSuccess
             ? 0
             : -5;
}
}
