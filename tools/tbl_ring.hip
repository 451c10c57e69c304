// tbl_ring.hip — a candidate shape for ns_csum_batch_dev's tables of
// MTU-sized packets: the receive ring's (rx_ring.hip).  Measured, not taken:
// on cfg2 (1M x 1500 B, two rotating batches; tools/grp_probe.py) it runs
// 222.5 us against 218.7 us for csum_hyb's big-packet instance, and 218.2 us
// even with no descriptor read at all.  It is built only
// into the timing-variants library (tools/grp_variants.hip).
//
// One wave takes 8 consecutive descriptors, one 8-lane group per packet (4
// waves per workgroup).  The group's load instruction k reads the packet's
// k-th 128-B HBM line whole (lane i: 16 B at line + 16 i), line 0 with the
// default cache policy (its first bytes belong to the packet before, which
// another group reads), the others nontemporal.  The descriptor alone
// decides which chunks exist, so all NB loads of a packet are issued at once;
// a chunk past the packet reads the buffer resource's out-of-range zeros
// (its offset is the resource's own size).  Every loaded chunk is summed
// whole except two: the chunk holding the packet's first byte is masked
// below it, and the chunk holding its last byte is re-read (an L2 hit,
// issued with the others) by the lane that loaded it, which takes the bytes
// past the end back out.  One 3-step DPP reduction gives the group its sum.
// Packets longer than NB lines take further batches of 4 lines.
//
// The hypothesis it tested: csum_hyb's big-packet shape splits each packet
// into whole lines for 8-lane groups and edge lines for single lanes, with a
// tile-wide scan; this shape reads the TX payload at 7.35 TB/s (§4.7) with
// no LDS, no scan and no barrier.  On descriptor tables it ties csum_hyb at
// best.
//
// Arithmetic: csum_kernels.hip's.  Packets of at most kGrpWOnlyMax bytes
// accumulate only the little-endian word sum W (s_class); a wave holding a
// longer one accumulates the exact (T, W) pair (s_of), so every result is
// Go's for any length.  Each packet's result is fold1(initial + S), as
// csum_hyb's finish_tile writes it for an unchained tile.
#include <hip/hip_runtime.h>
#include <stdint.h>

#include <algorithm>

#include "csum_kernels.h"

namespace nsk {
namespace {

constexpr uint32_t kGrpPerWave = 8;  // packets per wave
constexpr uint32_t kGrpWaves = 4;    // waves per workgroup
// W-only is exact up to 8190 chunks per packet (csum_kernels.hip
// kWOnlyMaxChunks); a packet of this many bytes spans at most that many.
constexpr uint32_t kGrpWOnlyMax = 8190u * 16u - 15u;
constexpr uint64_t kGrpMaxSrd = 0xFFFF0000ull;  // a buffer resource's reach (csum_kernels.hip kMaxSrdBytes)

__device__ __forceinline__ uint32_t g_fold1(uint32_t v) {  // ChecksumCombine, checksum.go:104-107
  const uint32_t s = (v & 0xFFFFu) + (v >> 16);
  return (s + (s >> 16)) & 0xFFFFu;
}

__device__ __forceinline__ uint32_t g_below(int c) {  // bytes [0, c) of a dword, c clamped to [0, 4]
  c = c < 0 ? 0 : (c > 4 ? 4 : c);
  return c >= 4 ? 0xFFFFFFFFu : ((1u << (8 * c)) - 1u);
}

__device__ __forceinline__ uint4 g_from(const uint4 v, int c) {  // bytes [c, 16) of a chunk
  return make_uint4(v.x & ~g_below(c), v.y & ~g_below(c - 4), v.z & ~g_below(c - 8), v.w & ~g_below(c - 12));
}

template <int AUX>
__device__ __forceinline__ uint4 g_load(__amdgpu_buffer_rsrc_t r, uint32_t off) {
  auto x = __builtin_amdgcn_raw_buffer_load_b128(r, (int)off, 0, AUX);
  return *reinterpret_cast<uint4*>(&x);
}

// The accumulator: W only, or the exact pair (T = byte sum, W).
template <bool EX>
struct Acc {
  uint32_t T = 0, W = 0;
  __device__ __forceinline__ void add(const uint4 v) {
    W = __builtin_amdgcn_sad_u16(v.x, 0u, W);
    W = __builtin_amdgcn_sad_u16(v.y, 0u, W);
    W = __builtin_amdgcn_sad_u16(v.z, 0u, W);
    W = __builtin_amdgcn_sad_u16(v.w, 0u, W);
    if constexpr (EX) {
      T = __builtin_amdgcn_sad_u8(v.x, 0u, T);
      T = __builtin_amdgcn_sad_u8(v.y, 0u, T);
      T = __builtin_amdgcn_sad_u8(v.z, 0u, T);
      T = __builtin_amdgcn_sad_u8(v.w, 0u, T);
    }
  }
  __device__ __forceinline__ void sub(const uint4 v) {
    Acc<EX> x;
    x.add(v);
    W -= x.W;
    if constexpr (EX) T -= x.T;
  }
};

__device__ __forceinline__ uint32_t g_group_sum(uint32_t s) {  // over the 8 lanes of a group
  s += (uint32_t)__builtin_amdgcn_update_dpp(0, (int)s, 0xB1, 0xF, 0xF, false);   // quad_perm 1,0,3,2
  s += (uint32_t)__builtin_amdgcn_update_dpp(0, (int)s, 0x4E, 0xF, 0xF, false);   // quad_perm 2,3,0,1
  s += (uint32_t)__builtin_amdgcn_update_dpp(0, (int)s, 0x141, 0xF, 0xF, false);  // row_half_mirror
  return s;
}

// One packet per group: bytes [pa, pe) of the resource (pa, pe relative to
// its 128-B-aligned base).  Returns the group's exact-or-W-only S value for
// phase `phase` (the packet's first byte's position parity, odd carry-in
// included), in every lane of the group.
template <int NB, bool EX>
__device__ __forceinline__ uint32_t grp_packet(__amdgpu_buffer_rsrc_t r, uint32_t nrec, uint32_t pa, uint32_t len,
                                               uint32_t li, uint32_t phase) {
  const uint32_t pe = pa + len;
  const uint32_t cl = (pa & ~127u) + 16u * li;  // lane li's chunk of line 0
  // lines k >= 1 start past pa: the lane's chunk there holds packet bytes
  // iff it starts before pe (k <= klast)
  const uint32_t klast = len && pe > cl ? (pe - 1u - cl) >> 7 : 0u;
  const uint32_t cl1 = len && pe > cl + 128u ? cl : nrec;
  const bool in0 = len && cl + 16u > pa && cl < pe;
  const uint32_t tc = (pe - 1u) & ~15u;  // the chunk holding the last byte
  const bool owner = len && ((tc >> 4) & 7u) == li;
  uint4 v[NB];
  v[0] = g_load<0>(r, in0 ? cl : nrec);
  const uint4 t = g_load<0>(r, owner ? tc : nrec);
#pragma unroll
  for (int k = 1; k < NB; ++k) v[k] = g_load<2>(r, ((uint32_t)k <= klast ? cl1 : nrec) + 128u * k);
  Acc<EX> a;
  a.add(g_from(v[0], pa > cl ? (int)(pa - cl) : 0));
#pragma unroll
  for (int k = 1; k < NB; ++k) a.add(v[k]);
  // packets longer than NB lines: the rest in batches of 4 lines
  for (uint32_t k0 = NB; __builtin_amdgcn_ballot_w64(k0 <= klast) != 0; k0 += 4) {
#pragma unroll
    for (int k = 0; k < 4; ++k) a.add(g_load<2>(r, ((k0 + k) <= klast ? cl1 : nrec) + 128u * (k0 + k)));
  }
  // the bytes [pe, tc + 16) were summed with the last chunk (none when pe
  // ends a chunk); the first chunk's bytes below pa were masked, so if it is
  // also the last, what is taken out lies above pa
  if (owner) a.sub(g_from(t, (int)(pe - tc)));
  const uint32_t W = g_group_sum(a.W);
  if constexpr (EX) {
    const uint32_t T = g_group_sum(a.T);
    return phase ? W : (257u * T - W);  // s_of: Go's S mod 2^32
  } else {
    const uint32_t w = g_fold1(W);  // s_class
    return phase ? w : g_fold1(w << 8);
  }
}

// FX > 0 (timing probes only, tools/grp_variants.hip): no descriptor read,
// packet i at arena byte i * FX, 1,500 B long — the payload loads' floor
// without the descriptor -> payload dependency.
// OCC: a waves-per-SIMD floor for the register allocator (timing probes).
template <int NB, int FX = 0, int OCC = 1, int FL = 1500>
__global__ __launch_bounds__(64 * kGrpWaves) __attribute__((amdgpu_waves_per_eu(OCC))) void tbl_ring(const uint8_t* __restrict__ arena, uint64_t arena_bytes,
                                                           const uint4* __restrict__ desc, uint32_t n,
                                                           uint16_t* __restrict__ out,
                                                           unsigned long long* __restrict__ err) {
  const uint32_t lane = threadIdx.x & 63u, grp = lane >> 3, li = lane & 7u;
  const uint32_t wv = (uint32_t)__builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  const uint64_t i0 = ((uint64_t)blockIdx.x * kGrpWaves + wv) * kGrpPerWave;  // the wave's first descriptor
  if (i0 >= n) return;  // a whole wave leaves together
  const uint64_t i = i0 + grp;
  const bool live = i < n;
  // every lane of the group loads its packet's descriptor (8 descriptors =
  // 128 B per wave instruction)
  const uint4 raw = !live ? make_uint4(0, 0, 0, 0)
                   : FX ? make_uint4((uint32_t)(i * FX), (uint32_t)((i * FX) >> 32), (uint32_t)FL, 0u)
                        : desc[i];
  const uint64_t off = (uint64_t)raw.x | ((uint64_t)raw.y << 32);
  uint32_t len = raw.z;
  if (live && (off > arena_bytes || (uint64_t)len > arena_bytes - off)) {  // csum_hyb decode()
    len = 0;
    if (li == 0) atomicAdd(err, 1ull);
  }
  const uint32_t init = raw.w & 0xFFFFu, odd = (raw.w >> 16) & 1u;
  // one resource over the arena from its 128-B line (the launcher keeps the
  // arena below kMaxSrdBytes), rounded up to whole 16-B chunks: the chunk
  // holding a packet's last byte lies inside it (its bytes past the arena's
  // end are in the same aligned chunk, never another page)
  const uint64_t a0 = (uint64_t)(uintptr_t)arena;
  const uint64_t base = a0 & ~127ull;
  const uint32_t nrec = (uint32_t)((a0 + arena_bytes - base + 15u) & ~15ull);
  const uint32_t lo = (uint32_t)__builtin_amdgcn_readfirstlane((uint32_t)base);
  const uint32_t hi = (uint32_t)__builtin_amdgcn_readfirstlane((uint32_t)(base >> 32));
  const __amdgpu_buffer_rsrc_t r = __builtin_amdgcn_make_buffer_rsrc(
      (void*)(((uint64_t)hi << 32) | (uint64_t)lo), (short)0, (int)__builtin_amdgcn_readfirstlane(nrec), 0x00020000);
  const uint32_t pa = len ? (uint32_t)(a0 + off - base) : 0u;
  const uint32_t phase = (uint32_t)((a0 + off + odd) & 1u);
  const uint32_t s = __builtin_amdgcn_ballot_w64(len > kGrpWOnlyMax) != 0
                         ? grp_packet<NB, true>(r, nrec, pa, len, li, phase)
                         : grp_packet<NB, false>(r, nrec, pa, len, li, phase);
  if (li == 0 && live) out[i] = (uint16_t)g_fold1(init + s);
}

template <int NB>
hipError_t launch_tbl_ring_t(const uint8_t* arena, uint64_t arena_bytes, const void* desc, uint32_t n, uint16_t* out,
                        unsigned long long* err, hipStream_t stream) {
  const uint64_t per_wg = (uint64_t)kGrpWaves * kGrpPerWave;
  hipLaunchKernelGGL((tbl_ring<NB>), dim3((uint32_t)((n + per_wg - 1) / per_wg)), dim3(64 * kGrpWaves), 0, stream,
                     arena, arena_bytes, reinterpret_cast<const uint4*>(desc), n, out, err);
  return hipGetLastError();
}

}  // namespace

bool tbl_ring_eligible(const uint8_t* arena, uint64_t arena_bytes, uint32_t n, uint64_t sizing_bytes) {
  if (!arena || n == 0) return false;
  const uint64_t avg = sizing_bytes / n;
  return avg >= kGrpMinAvg && avg <= kGrpMaxAvg && ((uintptr_t)arena & 127u) + arena_bytes + 64 < kGrpMaxSrd;
}

hipError_t launch_tbl_ring(const uint8_t* arena, uint64_t arena_bytes, const void* desc, uint32_t n, uint16_t* out,
                      unsigned long long* err, hipStream_t stream, uint32_t lines) {
  if (n == 0) return hipSuccess;
  if (lines == 0) {  // lines per batch for the average packet from any offset: 13 for 1500 B
    const uint64_t avg = arena_bytes / n;
    lines = (uint32_t)std::min<uint64_t>(16, (avg + 127 + 127) / 128);
  }
  if (lines <= 8) return launch_tbl_ring_t<8>(arena, arena_bytes, desc, n, out, err, stream);
  if (lines <= 13) return launch_tbl_ring_t<13>(arena, arena_bytes, desc, n, out, err, stream);
  return launch_tbl_ring_t<16>(arena, arena_bytes, desc, n, out, err, stream);
}

}  // namespace nsk
