// tx_variants.hip — timing variants of the structured TX kernel (tcp_tx.hip)
// that the product library does not carry, for tools/tx_struct_probe.py:
//   txv_launch(geo, stream, k): 0 = production shape, 1 = no segment
//   reductions (wrong sums), 2 = 8 windows in flight, 3 = 4 windows in
//   flight, 4 = production without the header write-back (fields unwritten),
//   5 = neither reductions nor write-back (the bare stream + header reads),
//   6 = 12 windows in flight, 7 = 6 without the write-back; 8 / 9 / 10 = the
//   two-pass shape (g->xs set) with 12 / 16 / 8 windows in flight; 11 = the
//   two passes with no header write-back (fields unwritten); (8-17 with
//   the windowed payload pass, round 4's); 12 / 13 / 14 =
//   the two passes with the persistent header pass at 4 / 16 / 2 waves per CU
//   (the product runs 24); 15 = the two passes, one-shot header pass;
//   16 / 17 = the persistent header pass at 24 / 32 waves per CU;
//   18 = the persistent header pass alone (the payload values left in g.xs);
//   19 / 20 / 21 = floors over the header slots' bytes [hdr, hdr + n slot):
//   copied onto themselves (read + write), read only, written only (16-B
//   lane accesses, 4 per lane, one-shot grid); 22-24 / 25-27 = written only /
//   copied with store cache policy 1 / 2 / 3; 28 / 29 = the payload pass
//   alone, in 8-lane groups (product) / windowed (round 4); 93 = the payload
//   pass alone in 4-lane groups (16 segments per wave); 30 / 31 / 32 =
//   both passes with the group payload pass all nontemporal / with
//   nontemporal header stores / both; 33 = the all-nontemporal group
//   payload pass alone; 34 / 35 = both passes, windowed / group payload
//   pass (whatever the product's default); 36 / 37 / 38 = the floors of
//   19 / 20 / 21 with lane-consecutive chunks (1 KiB per wave instruction);
//   39 = 36 with nt sc1 stores;
//   40-43 = the persistent header pass alone at 8 / 16 / 32 / 48 waves per
//   CU, 44 = the one-shot header pass alone (htile: the header tile);
//   70-76 = the persistent header pass alone, store policies (tx_store_aux);
//   77 / 78 = one pass in the group shape, slots written through / default;
//   90 = the production header pass alone at g->pad waves per CU; 91 = the
//   same with 3 tiles in flight per wave; 92 = one tile per wave, one-shot.
// Not part of the product ABI.
#include "../netstack_amd/csrc/tcp_tx.hip"


// Measured (round 6, bench.py --config 8, two rotating batches, three
// interleaved runs each; profiles/r06/tx_onepass/): 265.8 us with
// written-through slot stores, 279 us with default-policy ones, against
// 235.6-236.2 us for the two passes: the slot writes interleaved with the
// payload stream cost ~56 us, write-through or not.  The product keeps two
// passes.
namespace nsk {
// One pass in the group shape (timing variants 77 / 78; round 6): tcp_tx_pay's payload loop,
// then the wave finishes its own 8 segments' header slots, which sit back to
// back (8 x slot bytes from a 16-B-aligned start): the slot chunks are loaded
// with the payload (lane c: chunk c), parked in the wave's LDS row after the
// payload sums, segment g's fields computed by lane 8g from there (its
// group's W in registers: no payload value goes through memory), and the
// chunks written back with store policy SP.  For regions of at most 1 KiB
// (slot <= 128) that start 16-B aligned; the last wave's ragged end is
// written byte by byte.
template <int NB, int SP>
__global__ __launch_bounds__(256) void tcp_tx_payhdr(TxGeo g) {
  __shared__ uint4 ph_lds[4][64];
  const uint32_t lane = threadIdx.x & 63u, grp = lane >> 3, li = lane & 7u;
  const uint32_t wv = (uint32_t)__builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  const uint64_t s0 = ((uint64_t)blockIdx.x * 4u + wv) * 8u;
  if (s0 >= g.n) return;  // a whole wave leaves together
  const uint64_t s = s0 + grp;
  const uint64_t tail0 = (g.n - 1) * (uint64_t)g.mss;
  const uint32_t sz = s < g.n ? (s + 1 < g.n ? g.mss : (uint32_t)(g.size - tail0)) : 0u;
  const uint64_t wbase = (g.pay + s0 * g.mss) & ~127ull;
  const uint64_t s_end = s0 + 8u < g.n ? s0 + 8u : g.n;
  const uint32_t nseg = (uint32_t)(s_end - s0);
  const uint64_t w_end = g.pay + (s_end < g.n ? s_end * (uint64_t)g.mss : g.size);
  const uint32_t nrec = (uint32_t)((w_end - wbase + 15u) & ~15ull);
  const __amdgpu_buffer_rsrc_t r = tx_srd(wbase, nrec);
  // the wave's header slots: chunk `lane` (the last chunk may reach up to 15
  // bytes past the region, inside its own aligned 16 B)
  const uint64_t h_lo = g.hdr + s0 * g.slot;
  const uint32_t hbytes = nseg * g.slot, hchunks = (hbytes + 15u) >> 4;
  const __amdgpu_buffer_rsrc_t hr = tx_srd(h_lo, hchunks * 16u);
  const uint4 hv = tx_load<0>(hr, lane < hchunks ? lane * 16u : hchunks * 16u);
  const uint32_t pa = sz ? (uint32_t)(g.pay + s * g.mss - wbase) : 0u;
  const uint32_t pe = pa + sz;
  const uint32_t cl = (pa & ~127u) + 16u * li;
  const uint32_t klast = sz && pe > cl ? (pe - 1u - cl) >> 7 : 0u;
  const uint32_t cl1 = sz && pe > cl + 128u ? cl : nrec;
  const bool in0 = sz && cl + 16u > pa && cl < pe;
  const uint32_t tc = (pe - 1u) & ~15u;
  const bool owner = sz && ((tc >> 4) & 7u) == li;
  uint4 v[NB];
  v[0] = tx_load<0>(r, in0 ? cl : nrec);
  const uint4 t = tx_load<0>(r, owner ? tc : nrec);
#pragma unroll
  for (int k = 1; k < NB; ++k) v[k] = tx_load<2>(r, ((uint32_t)k <= klast ? cl1 : nrec) + 128u * k);
  uint32_t w = tx_bytes_from(v[0], pa > cl ? (int)(pa - cl) : 0);
#pragma unroll
  for (int k = 1; k < NB; ++k) w = wsum4(v[k], w);
  for (uint32_t k0 = NB; __builtin_amdgcn_ballot_w64(k0 <= klast) != 0; k0 += 4) {
#pragma unroll
    for (int k = 0; k < 4; ++k) w = wsum4(tx_load<2>(r, ((k0 + k) <= klast ? cl1 : nrec) + 128u * (k0 + k)), w);
  }
  if (owner) w -= tx_bytes_from(t, (int)(pe - tc));
  w += (uint32_t)__builtin_amdgcn_update_dpp(0, (int)w, 0xB1, 0xF, 0xF, false);
  w += (uint32_t)__builtin_amdgcn_update_dpp(0, (int)w, 0x4E, 0xF, 0xF, false);
  w += (uint32_t)__builtin_amdgcn_update_dpp(0, (int)w, 0x141, 0xF, 0xF, false);
  // the slots into the wave's LDS row
  uint4* L4 = ph_lds[wv];
  uint8_t* L = reinterpret_cast<uint8_t*>(L4);
  if (lane < hchunks) L4[lane] = hv;
  __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
  __builtin_amdgcn_wave_barrier();
  __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
  if (li == 0 && s < g.n) {  // tcp_tx_hdr's arithmetic for segment s
    const uint32_t o = grp * g.slot;
    uint32_t ipv = 0;
    if (g.mode & kTxIp) {
      const uint32_t a = o + g.ip_at;
      ipv = tx_fold(tx_class(lds_wsum_loop(L, a, g.ip_len, a + 10u), a & 1u));  // Checksum(ip[:IHL], 0)
      lds_put_be16(L, a + 10u, ~ipv & 0xFFFFu);
    }
    uint32_t x = tx_fold(g.addr_sum + ((g.tcp_len + sz) & 0xFFFFu));  // PseudoHeaderChecksum
    x = tx_fold(x + g.proto);
    const uint32_t a = o + g.tcp_at;
    x = tx_fold(x + tx_class(w, (uint32_t)((g.pay + s * g.mss) & 1u)));       // ChecksumVVWithOffset
    x = tx_fold(x + tx_class(lds_wsum_loop(L, a, g.tcp_len, a + 16u), a & 1u));  // CalculateChecksum
    lds_put_be16(L, a + 16u, ~x & 0xFFFFu);
    if (g.out) *reinterpret_cast<uint32_t*>(g.out + 2 * s) = ipv | (x << 16);
  }
  __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
  __builtin_amdgcn_wave_barrier();
  __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
  const uint32_t full = hbytes >> 4;
  const __amdgpu_buffer_rsrc_t hw = tx_srd(h_lo, full * 16u);
  const uint4 xv = L4[lane < hchunks ? lane : 0u];
  __builtin_amdgcn_raw_buffer_store_b128(*reinterpret_cast<const __attribute__((ext_vector_type(4))) uint32_t*>(&xv),
                                         hw, (int)(lane < full ? lane * 16u : full * 16u), 0, tx_store_aux(SP));
  if (full < hchunks && lane < (hbytes & 15u))  // the last wave's ragged end
    reinterpret_cast<uint8_t*>((uintptr_t)(h_lo + full * 16u))[lane] = L[full * 16u + lane];
}

template <int NB, int SP>
static hipError_t launch_tx_payhdr_t(const TxGeo& g, hipStream_t stream) {
  const uint64_t wgs = (g.n + 31) / 32;
  hipLaunchKernelGGL((tcp_tx_payhdr<NB, SP>), dim3((uint32_t)wgs), dim3(256), 0, stream, g);
  return hipGetLastError();
}

// 77 / 78's conditions: full TCP mode with whole slots written back, each
// wave's 8 slots 16-B aligned and at most 1 KiB, d_out 4-B aligned.
static bool tx_payhdr_ok(const TxGeo& g) {
  return (g.mode & kTxTcpFull) && !(g.mode & kTxFieldsOnly) && !(g.hdr & 15) && (8u * g.slot) % 16 == 0 &&
         g.slot <= 128 && !((uintptr_t)g.out & 3) && (g.n + 31) / 32 < (1ull << 31);
}

template <int SP>
static hipError_t launch_payhdr(const TxGeo& g, hipStream_t stream) {
  if (g.n == 0) return hipSuccess;
  switch (tx_pay_lines(g.mss)) {
    case 2: return launch_tx_payhdr_t<2, SP>(g, stream);
    case 4: return launch_tx_payhdr_t<4, SP>(g, stream);
    case 8: return launch_tx_payhdr_t<8, SP>(g, stream);
    case 13: return launch_tx_payhdr_t<13, SP>(g, stream);
    default: return launch_tx_payhdr_t<16, SP>(g, stream);
  }
}

}  // namespace nsk

namespace {
// FL: 0 read + write back, 1 read only (one dword per wave out), 2 write only
template <int FL, int SA = 0>
__global__ __launch_bounds__(256) void slot_floor(uint64_t base, uint32_t bytes, uint32_t* sink) {
  const uint32_t c0 = (blockIdx.x * 256u + threadIdx.x) * 4u;
  const __amdgpu_buffer_rsrc_t r = nsk::tx_srd(base, bytes);
  __attribute__((ext_vector_type(4))) uint32_t v[4];
#pragma unroll
  for (int i = 0; i < 4; ++i) {
    const uint32_t o = (c0 + (uint32_t)i) * 16u;
    if (FL != 2) v[i] = __builtin_amdgcn_raw_buffer_load_b128(r, (int)o, 0, 0);
    else v[i] = (__attribute__((ext_vector_type(4))) uint32_t){o, o, o, o};
  }
  if (FL == 1) {
    uint32_t a = 0;
#pragma unroll
    for (int i = 0; i < 4; ++i) a ^= v[i].x ^ v[i].y ^ v[i].z ^ v[i].w;
    if (a == 0x9E3779B9u) sink[0] = a;  // keeps the loads; never true on the probe's data
    return;
  }
#pragma unroll
  for (int i = 0; i < 4; ++i) __builtin_amdgcn_raw_buffer_store_b128(v[i], r, (int)((c0 + (uint32_t)i) * 16u), 0, SA);
}

// The same with each store / load instruction covering 1 KiB contiguous per
// wave (lane-consecutive chunks; slot_floor gives each lane 4 consecutive
// chunks, so one instruction touches 4 KiB at a 64-B stride).
template <int FL>
__global__ __launch_bounds__(256) void slot_floor_co(uint64_t base, uint32_t bytes, uint32_t* sink) {
  const __amdgpu_buffer_rsrc_t r = nsk::tx_srd(base, bytes);
  __attribute__((ext_vector_type(4))) uint32_t v[4];
#pragma unroll
  for (int i = 0; i < 4; ++i) {
    const uint32_t o = ((blockIdx.x * 4u + (uint32_t)i) * 256u + threadIdx.x) * 16u;
    if (FL < 2 || FL == 4) v[i] = __builtin_amdgcn_raw_buffer_load_b128(r, (int)o, 0, 0);
    else v[i] = (__attribute__((ext_vector_type(4))) uint32_t){o, o, o, o};
  }
  if (FL == 1) {
    uint32_t a = 0;
#pragma unroll
    for (int i = 0; i < 4; ++i) a ^= v[i].x ^ v[i].y ^ v[i].z ^ v[i].w;
    if (a == 0x9E3779B9u) sink[0] = a;
    return;
  }
#pragma unroll
  for (int i = 0; i < 4; ++i)
    __builtin_amdgcn_raw_buffer_store_b128(v[i], r, (int)(((blockIdx.x * 4u + (uint32_t)i) * 256u + threadIdx.x) * 16u),
                                           0, FL == 3 ? 2 : FL == 4 ? 18 : 0);
}

template <int FL>
hipError_t launch_floor_co(const nsk::TxGeo& g, hipStream_t s) {
  const uint32_t bytes = (uint32_t)((g.n * (uint64_t)g.slot) & ~15ull);
  const uint32_t chunks = bytes / 16u;
  hipLaunchKernelGGL((slot_floor_co<FL>), dim3((chunks + 1023u) / 1024u), dim3(256), 0, s, g.hdr & ~15ull, bytes,
                     reinterpret_cast<uint32_t*>(g.out));
  return hipGetLastError();
}

template <int FL, int SA = 0>
hipError_t launch_floor(const nsk::TxGeo& g, hipStream_t s) {
  const uint32_t bytes = (uint32_t)((g.n * (uint64_t)g.slot) & ~15ull);
  const uint32_t chunks = bytes / 16u;
  hipLaunchKernelGGL((slot_floor<FL, SA>), dim3((chunks + 1023u) / 1024u), dim3(256), 0, s, g.hdr & ~15ull, bytes,
                     reinterpret_cast<uint32_t*>(g.out));
  return hipGetLastError();
}
}  // namespace

extern "C" int txv_launch(const nsk::TxGeo* g, void* stream, int k) {
  hipStream_t s = (hipStream_t)stream;
  hipError_t e;
  switch (k) {
    case 1: e = nsk::launch_tcp_tx_t<16, 2, 0, 2>(*g, s); break;
    case 2: e = nsk::launch_tcp_tx_t<8, 2, 0, 1>(*g, s); break;
    case 3: e = nsk::launch_tcp_tx_t<4, 2, 0, 1>(*g, s); break;
    case 4: e = nsk::launch_tcp_tx_t<16, 2, 0, 1, 1>(*g, s); break;
    case 5: e = nsk::launch_tcp_tx_t<16, 2, 0, 2, 1>(*g, s); break;
    case 6: e = nsk::launch_tcp_tx_t<12, 2, 0, 1>(*g, s); break;
    case 7: e = nsk::launch_tcp_tx_t<12, 2, 0, 1, 1>(*g, s); break;
    case 8: e = nsk::launch_passes<12, 2, 0, 1, 1, 0>(*g, s); break;
    case 9: e = nsk::launch_passes<16, 2, 0, 1, 1, 0>(*g, s); break;
    case 10: e = nsk::launch_passes<8, 2, 0, 1, 1, 0>(*g, s); break;
    case 11: {  // the two passes, the header pass without its write-back (timing only)
      nsk::TxGeo h = *g;
      h.tile = g->htile;
      e = nsk::launch_tcp_tx_t<16, 2, 0, 1, 0, 1>(*g, s);
      if (e == hipSuccess) e = nsk::launch_tcp_tx_t<16, 2, 0, 1, 1, 2>(h, s);
      break;
    }
    case 12: e = nsk::launch_passes<16, 2, 0, 1, 1, 0>(*g, s, 4); break;
    case 13: e = nsk::launch_passes<16, 2, 0, 1, 1, 0>(*g, s, 16); break;
    case 14: e = nsk::launch_passes<16, 2, 0, 1, 1, 0>(*g, s, 2); break;
    case 15: e = nsk::launch_passes<16, 2, 0, 1, 0, 0>(*g, s); break;
    case 16: e = nsk::launch_passes<16, 2, 0, 1, 1, 0>(*g, s, 24); break;
    case 17: e = nsk::launch_passes<16, 2, 0, 1, 1, 0>(*g, s, 32); break;
    case 18: {
      nsk::TxGeo h = *g;
      h.tile = g->htile;
      e = nsk::launch_header_pass<0>(h, s, 0);
      break;
    }
    case 19: e = launch_floor<0>(*g, s); break;
    case 20: e = launch_floor<1>(*g, s); break;
    case 21: e = launch_floor<2>(*g, s); break;
    case 22: e = launch_floor<2, 1>(*g, s); break;
    case 23: e = launch_floor<2, 2>(*g, s); break;
    case 24: e = launch_floor<2, 3>(*g, s); break;
    case 25: e = launch_floor<0, 1>(*g, s); break;
    case 26: e = launch_floor<0, 2>(*g, s); break;
    case 27: e = launch_floor<0, 3>(*g, s); break;
    case 28: e = nsk::launch_payload_pass<16, 2, 0, 1, 1>(*g, s); break;
    case 93: {  // the payload pass in 4-lane groups (16 segments per wave, 64-B units)
      const uint32_t u = (g->mss + 63u + 63u) / 64u;
      e = u <= 2 ? nsk::launch_tx_pay_t<2, 0, 4>(*g, s) : u <= 4 ? nsk::launch_tx_pay_t<4, 0, 4>(*g, s)
        : u <= 8 ? nsk::launch_tx_pay_t<8, 0, 4>(*g, s) : nsk::launch_tx_pay_t<16, 0, 4>(*g, s);
      break;
    }
    case 29: e = nsk::launch_payload_pass<16, 2, 0, 1, 0>(*g, s); break;
    case 30: e = nsk::launch_passes<16, 2, 0, 1, 1, 2>(*g, s); break;
    case 31: e = nsk::launch_passes<16, 2, 1, 1, 1, 1>(*g, s); break;
    case 32: e = nsk::launch_passes<16, 2, 1, 1, 1, 2>(*g, s); break;
    case 33: e = nsk::launch_payload_pass<16, 2, 0, 1, 2>(*g, s); break;
    case 34: e = nsk::launch_passes<16, 2, 0, 1, 1, 0>(*g, s); break;
    case 40: case 41: case 42: case 43: case 45: {  // the persistent header pass alone at 8 / 16 / 32 / 48 / 12 waves per CU
      nsk::TxGeo h = *g;
      h.tile = g->htile;
      const uint32_t pc[] = {8, 16, 32, 48, 0, 12};
      e = nsk::launch_header_pass<0>(h, s, pc[k - 40]);
      break;
    }
    case 46: {  // the persistent header pass alone, nontemporal stores
      nsk::TxGeo h = *g;
      h.tile = g->htile;
      e = nsk::launch_header_pass<1>(h, s, 0);
      break;
    }
    case 47: e = launch_floor_co<3>(*g, s); break;  // written only, lane-consecutive, nontemporal
    case 44: {  // the one-shot header pass alone (round 4's)
      nsk::TxGeo h = *g;
      h.tile = g->htile;
      e = nsk::launch_tcp_tx_t<16, 2, 0, 1, 0, 2>(h, s);
      break;
    }
    case 36: e = launch_floor_co<0>(*g, s); break;
    case 37: e = launch_floor_co<1>(*g, s); break;
    case 38: e = launch_floor_co<2>(*g, s); break;
    case 39: e = launch_floor_co<4>(*g, s); break;  // copied onto themselves, lane-consecutive, nt sc1 stores
    case 35: e = nsk::launch_passes<16, 2, 0, 1, 1, 1>(*g, s); break;
    case 92: {  // one tile per wave on a one-shot grid (register-staged)
      nsk::TxGeo h = *g;
      h.tile = g->htile;
      e = nsk::launch_header_pass<4, 1>(h, s, g->pad);  // g->pad: waves per workgroup (0: the launcher's)
      break;
    }
    case 91: {  // the same with 3 tiles in flight per wave
      nsk::TxGeo h = *g;
      h.tile = g->htile;
      e = nsk::launch_header_pass<4, 3>(h, s, g->pad);
      break;
    }
    case 90: {  // the production header pass (nt sc1 stores) at g->pad waves per CU (0: 24), tile g->htile
      nsk::TxGeo h = *g;
      h.tile = g->htile;
      e = nsk::launch_header_pass<4>(h, s, g->pad);
      break;
    }
    // 77 / 78: one pass, the group payload loop + the wave's own slots,
    // written through (nt sc1) / default policy (falls back to production
    // where its conditions fail)
    case 77: e = nsk::tx_payhdr_ok(*g) ? nsk::launch_payhdr<4>(*g, s) : nsk::launch_tcp_tx(*g, s, 0); break;
    case 78: e = nsk::tx_payhdr_ok(*g) ? nsk::launch_payhdr<0>(*g, s) : nsk::launch_tcp_tx(*g, s, 0); break;
    // 70-76: the persistent header pass alone with store policy SP = k - 70
    // (tcp_tx.hip tx_store_aux: default, nt, sc1, sc0 sc1, nt sc1, sc0,
    // sc0 nt sc1)
    case 70: case 71: case 72: case 73: case 74: case 75: case 76: {
      nsk::TxGeo h = *g;
      h.tile = g->htile;
      const int sp = k - 70;
      e = sp == 0 ? nsk::launch_header_pass<0>(h, s, 0) : sp == 1 ? nsk::launch_header_pass<1>(h, s, 0)
        : sp == 2 ? nsk::launch_header_pass<2>(h, s, 0) : sp == 3 ? nsk::launch_header_pass<3>(h, s, 0)
        : sp == 4 ? nsk::launch_header_pass<4>(h, s, 0) : sp == 5 ? nsk::launch_header_pass<5>(h, s, 0)
        : nsk::launch_header_pass<6>(h, s, 0);
      break;
    }
    default: e = nsk::launch_tcp_tx_t<16, 2, 0, 1>(*g, s); break;
  }
  return (int)e;
}
