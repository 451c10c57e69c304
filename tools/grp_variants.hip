// grp_variants.hip — the receive ring's shape for descriptor tables
// (tbl_ring.hip, one 8-lane group per descriptor) beside csum_hyb's
// big-packet instance, for tools/grp_probe.py.  grpv_launch(k, ...):
//   0 tbl_ring     1 csum_hyb<...,8,16,4,2,0,2> (what launch_batch runs for
//   such tables)     2 tbl_ring with no descriptor read (packets at i * 1504,
//   1500 B: timing only, the floor of its payload loads)     3 the same over
//   contiguous 1460-B packets (the TX payload's layout)     4 2 with an
//   8-waves/SIMD register floor
// Not part of the product ABI.
#include "../netstack_amd/csrc/csum_kernels.hip"
#include "tbl_ring.hip"

extern "C" int grpv_launch(int k, const uint8_t* arena, uint64_t bytes, const void* desc, uint32_t n, uint16_t* out,
                           unsigned long long* err, void* stream) {
  hipStream_t s = (hipStream_t)stream;
  switch (k) {
    case 1:
      return (int)nsk::launch_hyb<8, 16, 4, 2, 0, 2>(arena, bytes, desc, n, out, nullptr, err, s, nsk::kBigChunks,
                                                      bytes, nsk::kTileBytes);
    case 2: {
      hipLaunchKernelGGL((nsk::tbl_ring<13, 1504>), dim3((n + 31) / 32), dim3(256), 0, s, arena, bytes,
                         reinterpret_cast<const uint4*>(desc), n, out, err);
      return (int)hipGetLastError();
    }
    case 3: {  // contiguous 1460-B packets (the TX payload's layout) over the same arena
      const uint32_t m = (uint32_t)(bytes / 1460);
      hipLaunchKernelGGL((nsk::tbl_ring<13, 1460, 1, 1460>), dim3((m + 31) / 32), dim3(256), 0, s, arena, bytes,
                         reinterpret_cast<const uint4*>(desc), m < n ? m : n, out, err);
      return (int)hipGetLastError();
    }
    case 4: {  // 2 with an 8-waves/SIMD register floor
      hipLaunchKernelGGL((nsk::tbl_ring<13, 1504, 8>), dim3((n + 31) / 32), dim3(256), 0, s, arena, bytes,
                         reinterpret_cast<const uint4*>(desc), n, out, err);
      return (int)hipGetLastError();
    }

    default:
      return (int)nsk::launch_tbl_ring(arena, bytes, desc, n, out, err, s);
  }
}
