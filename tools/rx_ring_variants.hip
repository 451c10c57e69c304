// rx_ring_variants.hip — timing variants of the receive-ring kernel
// (rx_ring.hip) that the product library does not carry, for
// tools/rx_ring_probe.py.  rxv_launch(geo, stream, k):
//   0 the product shape <13, default line 0, nt rest, 4 waves/WG>
//   1 every line default policy      2 every line nontemporal
//   3 2 waves/WG   4 8 waves/WG   5 1 wave/WG
//   6 16 lines per batch   7 8 lines per batch (two batches for 1500 B)
//   8 the product shape with a 6-waves/SIMD register floor
//   9 12 lines per batch
//  10 every chunk range-checked (F = 0: round 5's first product shape)
//  11 F with 8 lines per batch
//  12 / 13 line 0 / lines 0-1 loaded before the slot's length arrives
//  14 the product shape with each group's lines >= 2 in a rotated order
//  20-23 buffer lists (LIST = 1, g.off set): the product shape, then lines
//        >= 1 with the policy nt sc1 / default / sc1 instead of nt
//  24-29 buffer lists with each packet's last line at the default policy
//        (LL), the other lines >= 1 nt / nt sc1 / sc0 nt / sc0 sc1 /
//        sc0 nt sc1 / sc0
//  30    buffer lists sorted into address buckets first (rx_bk_count,
//        rx_bk_place, then the parse over the sorted list: LIST = 2)
//  31    30 with the outputs written in sorted order (timing only: wrong
//        places)   32  30 with the list index loaded with the entry
//  33    the sort alone (rx_bk_count + rx_bk_place)   34  rx_bk_count alone
//  50    the layout's read floor (rx_floor: the frames' lines, no parse;
//        timing only)
//  40 / 41 / 42  4-lane groups (16 packets per wave, 64-B units), 4 / 8 / 16
//        units per batch (rings of short frames)
// Every variant but 31, 33 and 34 computes the product's verdicts and sums.
// Not part of the ABI.
#include "../netstack_amd/csrc/rx_ring.hip"

namespace nsk {
// Sorting a buffer list into address buckets (variants 30-34, LIST = 2).
// A pool hands its buffers out in any order; verified in that order,
// neighbouring buffers' shared edge lines are read twice and the reads
// scatter over the whole pool.
// Two passes over the list, 4,096 entries per workgroup, bring it into
// bucket order (bucket = off >> bk_shift; order inside a bucket arbitrary):
// rx_bk_count histograms its entries in LDS and reserves each bucket's run
// with one atomic per bucket (bk_wgoff: where its run starts in the bucket);
// rx_bk_place turns the bucket totals into starts and writes each entry's
// (off, len, index) at start + run offset + its LDS rank.
constexpr uint32_t kBkChunk = 4096, kBkMax = 128, kBkPer = kBkChunk / 256;

__device__ __forceinline__ uint32_t rx_bk_of(const RxGeo& g, uint32_t o) {
  const uint32_t b = o >> g.bk_shift;
  return b < g.bk_nb ? b : g.bk_nb - 1u;
}

__global__ __launch_bounds__(256) void rx_bk_count(RxGeo g) {
  __shared__ uint32_t h[kBkMax];
  const uint32_t t = threadIdx.x;
  if (t < kBkMax) h[t] = 0u;
  __syncthreads();
  const uint64_t c0 = (uint64_t)blockIdx.x * kBkChunk;
  uint32_t o[kBkPer];
#pragma unroll
  for (uint32_t j = 0; j < kBkPer; ++j) {
    const uint64_t i = c0 + t + 256u * j;
    o[j] = i < g.n ? g.off[i] : 0u;
  }
#pragma unroll
  for (uint32_t j = 0; j < kBkPer; ++j)
    if (c0 + t + 256u * j < g.n) atomicAdd(&h[rx_bk_of(g, o[j])], 1u);
  __syncthreads();
  if (t < g.bk_nb) {
    const uint32_t c = h[t];
    g.bk_wgoff[(uint64_t)blockIdx.x * g.bk_nb + t] = c ? atomicAdd(&g.bk_total[t], c) : 0u;
  }
}

__global__ __launch_bounds__(256) void rx_bk_place(RxGeo g) {
  __shared__ uint32_t sc[kBkMax], cur[kBkMax];
  const uint32_t t = threadIdx.x;
  const uint64_t c0 = (uint64_t)blockIdx.x * kBkChunk;
  uint32_t o[kBkPer], l[kBkPer];
#pragma unroll
  for (uint32_t j = 0; j < kBkPer; ++j) {
    const uint64_t i = c0 + t + 256u * j;
    o[j] = i < g.n ? g.off[i] : 0u;
    l[j] = i < g.n ? g.len[i] : 0u;
  }
  const uint32_t tot = t < g.bk_nb ? g.bk_total[t] : 0u;
  if (t < kBkMax) sc[t] = tot;
  __syncthreads();
  for (uint32_t d = 1; d < kBkMax; d <<= 1) {  // inclusive scan of the totals
    const uint32_t x = t < kBkMax && t >= d ? sc[t - d] : 0u;
    __syncthreads();
    if (t < kBkMax) sc[t] += x;
    __syncthreads();
  }
  if (t < g.bk_nb) cur[t] = sc[t] - tot + g.bk_wgoff[(uint64_t)blockIdx.x * g.bk_nb + t];
  __syncthreads();
#pragma unroll
  for (uint32_t j = 0; j < kBkPer; ++j) {
    const uint64_t i = c0 + t + 256u * j;
    if (i < g.n) {
      const uint32_t at = atomicAdd(&cur[rx_bk_of(g, o[j])], 1u);
      g.bk_tup[at] = make_uint4(o[j], l[j], (uint32_t)i, 0u);
    }
  }
}

// The sorted list's parse: the product shape over bk_tup.
template <int NB, int L = 2>
static hipError_t launch_rx_bufs_sorted_t(const RxGeo& g, hipStream_t stream) {
  const uint32_t wgs = (uint32_t)((g.n + kBkChunk - 1) / kBkChunk);
  hipLaunchKernelGGL(rx_bk_count, dim3(wgs), dim3(256), 0, stream, g);
  hipLaunchKernelGGL(rx_bk_place, dim3(wgs), dim3(256), 0, stream, g);
  return launch_rx_ring_t<NB, 0, 2, kWaves, 1, 1, 0, L>(g, stream);
}

static hipError_t launch_rx_bufs_sorted(const RxGeo& g, hipStream_t stream) {
  if (g.n == 0) return hipSuccess;
  switch (rx_batch_lines(g)) {
    case 2: return launch_rx_bufs_sorted_t<2>(g, stream);
    case 4: return launch_rx_bufs_sorted_t<4>(g, stream);
    case 8: return launch_rx_bufs_sorted_t<8>(g, stream);
    default: return launch_rx_bufs_sorted_t<13>(g, stream);
  }
}

// Variant 50: the read floor of a ring layout -- each 8-lane group reads the
// lines holding its slot's received bytes (len[s] from the slot's start),
// sums them and writes one byte; no parse.  Timing only.
template <int NB>
__global__ __launch_bounds__(256) void rx_floor(RxGeo g) {
  const uint32_t lane = threadIdx.x & 63u, grp = lane >> 3, li = lane & 7u;
  const uint32_t wv = (uint32_t)__builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  const uint64_t s0 = ((uint64_t)blockIdx.x * 4u + wv) * 8u;
  if (s0 >= g.n) return;
  const uint64_t s = s0 + grp;
  const uint64_t wbase = (g.ring + s0 * g.stride) & ~127ull;
  const uint64_t s_end = s0 + 8u < g.n ? s0 + 8u : g.n;
  const uint32_t nrec = (uint32_t)(g.ring + s_end * g.stride - wbase);
  const __amdgpu_buffer_rsrc_t r = rx_srd(wbase, nrec);
  const uint32_t len = s < g.n ? g.len[s] : 0u;
  const uint32_t pa = (uint32_t)(g.ring + s * g.stride - wbase);
  const uint32_t cl = (pa & ~127u) + 16u * li;
  uint32_t w = 0;
  for (uint32_t k0 = 0; __builtin_amdgcn_ballot_w64(s < g.n && 128u * k0 < len + (pa & 127u)) != 0; k0 += NB) {
    uint4 v[NB];
#pragma unroll
    for (int k = 0; k < NB; ++k) {
      const uint32_t o = cl + 128u * (k0 + k);
      v[k] = rx_load<2>(r, s < g.n && o + 16u > pa && o < pa + len ? o : nrec);
    }
#pragma unroll
    for (int k = 0; k < NB; ++k) w = rx_wsum4(v[k]) + w;
  }
  w += (uint32_t)__builtin_amdgcn_update_dpp(0, (int)w, 0xB1, 0xF, 0xF, false);
  w += (uint32_t)__builtin_amdgcn_update_dpp(0, (int)w, 0x4E, 0xF, 0xF, false);
  w += (uint32_t)__builtin_amdgcn_update_dpp(0, (int)w, 0x141, 0xF, 0xF, false);
  if (li == 0 && s < g.n) g.verdict[s] = (uint8_t)w;
}

}  // namespace nsk

extern "C" int rxv_launch(const nsk::RxGeo* g, void* stream, int k) {
  hipStream_t s = (hipStream_t)stream;
  switch (k) {
    case 1: return (int)nsk::launch_rx_ring_t<13, 0, 0>(*g, s);
    case 2: return (int)nsk::launch_rx_ring_t<13, 2, 2>(*g, s);
    case 3: return (int)nsk::launch_rx_ring_t<13, 0, 2, 2>(*g, s);
    case 4: return (int)nsk::launch_rx_ring_t<13, 0, 2, 8>(*g, s);
    case 5: return (int)nsk::launch_rx_ring_t<13, 0, 2, 1>(*g, s);
    case 6: return (int)nsk::launch_rx_ring_t<16>(*g, s);
    case 7: return (int)nsk::launch_rx_ring_t<8>(*g, s);
    case 8: return (int)nsk::launch_rx_ring_t<13, 0, 2, 4, 6>(*g, s);
    case 9: return (int)nsk::launch_rx_ring_t<12>(*g, s);
    case 10: return (int)nsk::launch_rx_ring_t<13, 0, 2, 4, 1, 0>(*g, s);
    case 11: return (int)nsk::launch_rx_ring_t<8, 0, 2, 4, 1, 1>(*g, s);
    case 12: return (int)nsk::launch_rx_ring_t<13, 0, 2, 4, 1, 1, 1>(*g, s);
    case 13: return (int)nsk::launch_rx_ring_t<13, 0, 2, 4, 1, 1, 2>(*g, s);
    case 14: return (int)nsk::launch_rx_ring_t<13, 0, 2, 4, 1, 1, 0, 0, 1>(*g, s);
    case 20: return (int)nsk::launch_rx_ring_t<13, 0, 2, 4, 1, 1, 0, 1>(*g, s);
    case 21: return (int)nsk::launch_rx_ring_t<13, 0, 18, 4, 1, 1, 0, 1>(*g, s);
    case 22: return (int)nsk::launch_rx_ring_t<13, 0, 0, 4, 1, 1, 0, 1>(*g, s);
    case 23: return (int)nsk::launch_rx_ring_t<13, 0, 16, 4, 1, 1, 0, 1>(*g, s);
    case 24: return (int)nsk::launch_rx_ring_t<13, 0, 2, 4, 1, 1, 0, 1, 0, 1>(*g, s);
    case 25: return (int)nsk::launch_rx_ring_t<13, 0, 18, 4, 1, 1, 0, 1, 0, 1>(*g, s);
    case 26: return (int)nsk::launch_rx_ring_t<13, 0, 3, 4, 1, 1, 0, 1, 0, 1>(*g, s);
    case 27: return (int)nsk::launch_rx_ring_t<13, 0, 17, 4, 1, 1, 0, 1, 0, 1>(*g, s);
    case 28: return (int)nsk::launch_rx_ring_t<13, 0, 19, 4, 1, 1, 0, 1, 0, 1>(*g, s);
    case 29: return (int)nsk::launch_rx_ring_t<13, 0, 1, 4, 1, 1, 0, 1, 0, 1>(*g, s);
    case 40: return (int)nsk::launch_rx_ring_t<4, 0, 2, 4, 1, 1, 0, 0, 0, 0, 4>(*g, s);
    case 41: return (int)nsk::launch_rx_ring_t<8, 0, 2, 4, 1, 1, 0, 0, 0, 0, 4>(*g, s);
    case 42: return (int)nsk::launch_rx_ring_t<16, 0, 2, 4, 1, 1, 0, 0, 0, 0, 4>(*g, s);
    case 30: return (int)nsk::launch_rx_bufs_sorted(*g, s);
    case 50: {
      hipLaunchKernelGGL(nsk::rx_floor<13>, dim3((uint32_t)((g->n + 31) / 32)), dim3(256), 0, s, *g);
      return (int)hipGetLastError();
    }
    case 31: return (int)nsk::launch_rx_bufs_sorted_t<13, 3>(*g, s);
    case 32: return (int)nsk::launch_rx_bufs_sorted_t<13, 4>(*g, s);
    case 33: case 34: {
      const uint32_t wgs = (uint32_t)((g->n + nsk::kBkChunk - 1) / nsk::kBkChunk);
      hipLaunchKernelGGL(nsk::rx_bk_count, dim3(wgs), dim3(256), 0, s, *g);
      if (k == 33) hipLaunchKernelGGL(nsk::rx_bk_place, dim3(wgs), dim3(256), 0, s, *g);
      hipMemsetAsync(g->bk_total, 0, 4 * g->bk_nb, s);
      return (int)hipGetLastError();
    }
    default: return (int)nsk::launch_rx_ring_t<13>(*g, s);
  }
}
