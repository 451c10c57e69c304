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
//   alone, in 8-lane groups (product) / windowed (round 4); 30 / 31 / 32 =
//   both passes with the group payload pass all nontemporal / with
//   nontemporal header stores / both; 33 = the all-nontemporal group
//   payload pass alone; 34 / 35 = both passes, windowed / group payload
//   pass (whatever the product's default); 36 / 37 / 38 = the floors of
//   19 / 20 / 21 with lane-consecutive chunks (1 KiB per wave instruction);
//   40-43 = the persistent header pass alone at 8 / 16 / 32 / 48 waves per
//   CU, 44 = the one-shot header pass alone (htile: the header tile);
//   70-76 = the persistent header pass alone, store policies (tx_store_aux).
// Not part of the product ABI.
#include "../netstack_amd/csrc/tcp_tx.hip"

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
    if (FL < 2) v[i] = __builtin_amdgcn_raw_buffer_load_b128(r, (int)o, 0, 0);
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
                                           0, FL == 3 ? 2 : 0);
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
    case 35: e = nsk::launch_passes<16, 2, 0, 1, 1, 1>(*g, s); break;
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
