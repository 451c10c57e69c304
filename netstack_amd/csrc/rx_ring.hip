// rx_ring.hip — receive-side verification of a fixed-stride ring of received
// frames, parsed on the device (ns_csum_rx_ring, include/netstack_csum.h;
// DESIGN.md §4.8).  The receive mirror of tcp_tx.hip: no descriptor table and
// no host planning; the kernel reads each slot's received length, parses the
// frame's headers itself and gives the verdict ns_csum_packet_buffers
// (NS_PKB_VERIFY) gives for the same packet.
//
// What one slot goes through, as the reference does it:
//   link     recvMMsgDispatcher.dispatch (link/fdbased/packet_dispatchers.go:
//            258-317): a frame of n <= hdrSize bytes is dropped; Ethernet picks
//            the network protocol by EtherType, a headerless link (TUN) by the
//            IP version nibble (others dropped); Data = the frame's views
//            (BufConfig, :30) with the link header trimmed.
//   IPv4     HandlePacket (network/ipv4/ipv4.go:341-394) + IsValid (header/
//            ipv4.go:280-296): length checks against the FIRST view; trim to
//            [IHL*4, TotalLength); a fragment without payload or whose uint16
//            offset + size - 1 wraps is malformed, any other fragment goes to
//            reassembly (its transport checksum is checked only after that).
//   IPv6     HandlePacket (network/ipv6/ipv6.go:168-188) + IsValid (header/
//            ipv6.go:207-222); trim to [40, 40 + PayloadLength).
//   TCP      segment.parse (transport/tcp/segment.go:145-181): DataOffset
//            checked against the first view; xsum = PseudoHeaderChecksum(6,
//            src, dst, size) + header + payload, valid iff 0xffff.
//   ICMPv4   handleICMP echo request (network/ipv4/icmp.go:60-80).
//   ICMPv6   handleICMP (network/ipv6/icmp.go:62-84, ICMPv6Checksum
//            header/icmpv6.go:202-221).
// oracle/packets.py (verify, verify_frame) restates the same rules on the CPU.
//
// Shape.  A wave owns 8 consecutive slots, one 8-lane group per packet.  The
// group's instruction k reads the packet's k-th 128-B HBM line whole (lane i:
// 16 B at line + 16 i), so every load instruction reads exactly one line per
// group: line 0 with the default cache policy (its first bytes may belong to
// the slot before), the rest nontemporal.  All of a packet's loads are issued
// at once from its received length, before anything is known about its
// headers.  Lines 0 and 1 then go to an LDS row (the first 96 B of the IP
// packet); every lane of the group parses the headers from it (the same LDS
// reads in each lane: broadcasts), so each lane knows the byte range to sum
// and the field to read as zero without any cross-lane step.  The lanes mask
// their chunks to that range (only edge chunks need a mask), sum little-endian
// words with v_sad_u16, and one 3-step DPP reduction gives the group its W.
//
// Arithmetic.  Slots are 16-B aligned and the IP packet starts at an even
// offset, so every summed range starts at an even address: Go's big-endian
// word sum S satisfies S == 256 W (mod 65535) and S == 0 iff W == 0, and no
// range is longer than 65,575 B, so no uint32 wraps (tcp_tx.hip, csum_kernels
// W-only accumulation): the folded results are bit-exact with the Go code.
#include <hip/hip_runtime.h>
#include <stdint.h>

#include "csum_kernels.h"

namespace nsk {
namespace {

constexpr uint32_t kRowBytes = 96;  // LDS bytes per packet: [floor16(pa), +96)
constexpr uint32_t kPerWave = 8;    // packets per wave
constexpr uint32_t kWaves = 4;      // waves per workgroup
constexpr uint32_t kMaxIp = 65576;  // the longest IP packet any header can describe (40 + 65535), + 1

constexpr uint32_t kInvalid = 0, kValid = 1, kUnchecked = 2, kMalformed = 3;  // NS_PKB_*

__device__ __forceinline__ uint32_t rx_fold(uint32_t v) {  // ChecksumCombine, checksum.go:104-107
  const uint32_t s = (v & 0xFFFFu) + (v >> 16);
  return (s + (s >> 16)) & 0xFFFFu;
}

// A W total of a range starting at an even address, as a value with the fold
// behaviour of Go's S (the byte swap of W, mod 65535; zero iff W is).
__device__ __forceinline__ uint32_t rx_class(uint32_t W) { return rx_fold(rx_fold(W) << 8); }

__device__ __forceinline__ uint32_t rx_wsum4(const uint4 v) {
  uint32_t acc = __builtin_amdgcn_sad_u16(v.x, 0u, 0u);
  acc = __builtin_amdgcn_sad_u16(v.y, 0u, acc);
  acc = __builtin_amdgcn_sad_u16(v.z, 0u, acc);
  return __builtin_amdgcn_sad_u16(v.w, 0u, acc);
}

__device__ __forceinline__ uint32_t rx_below(int c) {  // bytes [0, c) of a dword, c clamped to [0, 4]
  c = c < 0 ? 0 : (c > 4 ? 4 : c);
  return c >= 4 ? 0xFFFFFFFFu : ((1u << (8 * c)) - 1u);
}

// Bytes [lo, hi) of a 16-B chunk, without [zl, zl + 2).
__device__ __forceinline__ uint32_t rx_dmask(int lo, int hi, int zl, int d) {
  const int b = 4 * d;
  return rx_below(hi - b) & ~rx_below(lo - b) & ~(rx_below(zl + 2 - b) & ~rx_below(zl - b));
}

__device__ __forceinline__ uint32_t rx_masked(uint4 v, int lo, int hi, int zl) {
  v.x &= rx_dmask(lo, hi, zl, 0);
  v.y &= rx_dmask(lo, hi, zl, 1);
  v.z &= rx_dmask(lo, hi, zl, 2);
  v.w &= rx_dmask(lo, hi, zl, 3);
  return rx_wsum4(v);
}

// One chunk's contribution: its bytes inside [a, b) minus the field at z,
// where r is the chunk's offset from the IP packet's first byte.
__device__ __forceinline__ uint32_t rx_chunk(const uint4 v, int r, int a, int b, int z) {
  const int lo = a - r, hi = b - r, zl = z - r;
  const bool full = (lo <= 0) & (hi >= 16) & ((zl >= 16) | (zl <= -2));
  if (full) return rx_wsum4(v);
  if ((hi <= 0) | (lo >= 16)) return 0u;
  return rx_masked(v, lo, hi, zl);
}

// The W sum of LDS bytes [a, a + len) (4-B-aligned row, len <= 4 * MAXD - 3).
template <int MAXD>
__device__ __forceinline__ uint32_t rx_lds_wsum(const uint8_t* row, uint32_t a, uint32_t len) {
  const uint32_t* D = reinterpret_cast<const uint32_t*>(row);
  const uint32_t d0 = a >> 2;
  const uint32_t nd = ((a + len + 3) >> 2) - d0;
  uint32_t w = 0;
#pragma unroll
  for (int k = 0; k < MAXD; ++k) {
    if ((uint32_t)k < nd) {
      const int b = (int)(4 * (d0 + k));
      w = __builtin_amdgcn_sad_u16(D[d0 + k] & rx_below((int)(a + len) - b) & ~rx_below((int)a - b), 0u, w);
    }
  }
  return w;
}

__device__ __forceinline__ __amdgpu_buffer_rsrc_t rx_srd(uint64_t base, uint32_t nrec) {
  const uint32_t lo = (uint32_t)__builtin_amdgcn_readfirstlane((uint32_t)base);
  const uint32_t hi = (uint32_t)__builtin_amdgcn_readfirstlane((uint32_t)(base >> 32));
  return __builtin_amdgcn_make_buffer_rsrc((void*)(((uint64_t)hi << 32) | (uint64_t)lo), (short)0,
                                           (int)__builtin_amdgcn_readfirstlane(nrec), 0x00020000);
}

template <int AUX>
__device__ __forceinline__ uint4 rx_load(__amdgpu_buffer_rsrc_t r, uint32_t off) {
  auto x = __builtin_amdgcn_raw_buffer_load_b128(r, (int)off, 0, AUX);
  return *reinterpret_cast<uint4*>(&x);
}

}  // namespace

// NB = lines per load batch (line 0 included); a packet longer than NB lines
// takes further batches of NB nontemporal lines.
template <int NB>
__global__ __launch_bounds__(256) void rx_ring(RxGeo g) {
  __shared__ uint4 rx_lds[kWaves * kPerWave * kRowBytes / 16];
  const uint32_t lane = threadIdx.x & 63u, grp = lane >> 3, li = lane & 7u;
  const uint32_t wv = (uint32_t)__builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  const uint64_t s0 = ((uint64_t)blockIdx.x * kWaves + wv) * kPerWave;  // the wave's first slot
  if (s0 >= g.n) return;  // a whole wave leaves together
  const uint64_t s = s0 + grp;
  const bool live = s < g.n;

  // The frame: recvmmsg's length, less the bytes before the frame (a virtio-
  // net header) and the link header.  A slot longer than the ring's stride is
  // malformed and counted (ns_csum_sync), a frame of no more than its link
  // header is dropped by the link (packet_dispatchers.go:268-270).
  const uint32_t rlen = live ? g.len[s] : 0u;
  const bool over = (uint64_t)rlen > g.stride;
  const uint32_t pre = g.frame_at + g.link;
  const uint32_t P = (!over && rlen > pre) ? rlen - pre : 0u;       // Data.Size()
  const uint32_t Pl = P < kMaxIp ? P : kMaxIp;                       // bytes any header can cover
  const uint64_t pa = g.ring + s * g.stride + pre;                   // the IP packet's first byte
  const uint64_t l0 = pa >> 7;
  const uint32_t nl = Pl ? (uint32_t)(((pa + Pl - 1) >> 7) - l0 + 1) : 0u;  // its HBM lines

  // One buffer resource over the wave's slots (< 8 strides + a line).
  const uint64_t wbase = (g.ring + s0 * g.stride + pre) & ~127ull;
  const uint64_t s_end = s0 + kPerWave < g.n ? s0 + kPerWave : g.n;
  const uint32_t nrec = (uint32_t)(g.ring + s_end * g.stride - wbase);
  const __amdgpu_buffer_rsrc_t rsrc = rx_srd(wbase, nrec);
  const uint64_t pe = pa + Pl;
  // chunk li of line k: loaded only where it holds packet bytes, else the
  // range check returns zeros without touching memory
  auto off_of = [&](uint32_t k) -> uint32_t {
    const uint64_t c = ((l0 + k) << 7) + 16u * li;
    return (k < nl && c + 16 > pa && c < pe) ? (uint32_t)(c - wbase) : nrec;
  };

  uint4 v[NB];
  v[0] = rx_load<0>(rsrc, off_of(0));
#pragma unroll
  for (int k = 1; k < NB; ++k) v[k] = rx_load<2>(rsrc, off_of((uint32_t)k));
  uint32_t etype = 0;
  if (g.link && P) {
    const uint8_t* e = reinterpret_cast<const uint8_t*>((uintptr_t)(g.ring + s * g.stride + g.frame_at + 12));
    etype = ((uint32_t)e[0] << 8) | e[1];
  }

  // The first 96 B from floor16(pa) into the group's LDS row.
  uint8_t* row = reinterpret_cast<uint8_t*>(rx_lds) + (wv * kPerWave + grp) * kRowBytes;
  const uint64_t f16 = pa & ~15ull;
#pragma unroll
  for (int k = 0; k < 2; ++k) {
    const uint64_t c = ((l0 + k) << 7) + 16u * li;
    if (c >= f16 && c < f16 + kRowBytes) *reinterpret_cast<uint4*>(row + (c - f16)) = v[k];
  }
  __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
  __builtin_amdgcn_wave_barrier();
  __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");

  // Parse (every lane of the group, same LDS bytes).  h(i) = IP byte i.
  const uint32_t po = (uint32_t)(pa & 15u);
  auto h = [&](uint32_t i) -> uint32_t { return row[po + i]; };
  const uint32_t first = g.view0 && g.view0 < P ? g.view0 : P;  // the first view's length
  uint32_t verdict = kMalformed, net = 0, init = 0, want = 0, kind = 0;
  int a = 0, b = 0, z = -64;  // sum [a, b) but [z, z + 2) as zeros
  do {
    if (P == 0) break;
    const uint32_t ver = h(0) >> 4;
    const uint32_t np = g.link ? (etype == 0x0800u ? 4u : etype == 0x86DDu ? 6u : 0u) : ver;
    if (g.link && np == 0) {  // not IP: nothing the reference checksums
      verdict = kUnchecked;
      break;
    }
    uint32_t proto, asum, tend, tb;
    if (np == 4) {
      if (first < 20) break;
      const uint32_t hlen = (h(0) & 15u) * 4u, tlen = (h(2) << 8) | h(3);
      // hlen > first is not in IsValid (tests/golden/rx_choices.json)
      if (hlen < 20 || hlen > tlen || tlen > P || hlen > first || ver != 4) break;
      net = rx_class(rx_lds_wsum<16>(row, po, hlen));  // IPv4.CalculateChecksum (ipv4.go:251-253)
      const uint32_t more = h(6) & 0x20u;
      const uint32_t foff = ((((h(6) & 0x1Fu) << 8) | h(7)) << 3) & 0xFFFFu;
      if (more || foff) {  // ipv4.go:355-385
        const uint32_t size = tlen - hlen;
        verdict = (size == 0 || ((foff + (size & 0xFFFFu) - 1u) & 0xFFFFu) < foff) ? kMalformed : kUnchecked;
        break;
      }
      proto = h(9);
      asum = rx_class(rx_lds_wsum<3>(row, po + 12, 8));
      tb = hlen;
      tend = tlen;
    } else if (np == 6) {
      if (first < 40) break;
      const uint32_t plen = (h(4) << 8) | h(5);
      if (plen > P - 40 || ver != 6) break;
      proto = h(6);
      asum = rx_class(rx_lds_wsum<9>(row, po + 8, 32));
      tb = 40;
      tend = 40 + plen;
    } else {
      break;  // a headerless link drops other versions
    }
    const uint32_t tsize = tend - tb;
    const uint32_t tfl = (first < tend ? first : tend) - tb;  // the transport's first view
    verdict = kUnchecked;
    if (proto == 6) {  // segment.parse (segment.go:160-180)
      const uint32_t off = (h(tb + 12) >> 4) * 4u;
      if (tfl < 20 || off < 20 || off > tfl) {
        verdict = kMalformed;
        break;
      }
      kind = 1;
      init = rx_fold(asum + (tsize & 0xFFFFu) + 6u);  // PseudoHeaderChecksum (checksum.go:112-122)
    } else if (proto == 1 && np == 4) {  // handleICMP: echo requests only
      if (tfl < 8) {
        verdict = kMalformed;
        break;
      }
      if (h(tb) != 8) break;
      kind = 2;
      want = (h(tb + 2) << 8) | h(tb + 3);
      z = (int)tb + 2;
    } else if (proto == 58 && np == 6) {  // ICMPv6Checksum
      if (tfl < 4) {
        verdict = kMalformed;
        break;
      }
      kind = 3;
      want = (h(tb + 2) << 8) | h(tb + 3);
      z = (int)tb + 2;
      init = rx_fold(asum + tsize + 58u);
    } else {
      break;
    }
    a = (int)tb;
    b = (int)tend;
  } while (false);

  // The transport range, masked chunk by chunk.
  uint32_t w = 0;
  const int r0 = (int)((int64_t)((l0 << 7) + 16u * li) - (int64_t)pa);  // chunk offset of line 0
#pragma unroll
  for (int k = 0; k < NB; ++k) w += rx_chunk(v[k], r0 + 128 * k, a, b, z);
  for (uint32_t k0 = NB; __builtin_amdgcn_ballot_w64(k0 < nl && (int)(r0 + 128 * k0) < b) != 0; k0 += NB) {
#pragma unroll
    for (int k = 0; k < NB; ++k) v[k] = rx_load<2>(rsrc, off_of(k0 + k));
#pragma unroll
    for (int k = 0; k < NB; ++k) w += rx_chunk(v[k], r0 + 128 * (int)(k0 + k), a, b, z);
  }
  w += (uint32_t)__builtin_amdgcn_update_dpp(0, (int)w, 0xB1, 0xF, 0xF, false);   // quad_perm 1,0,3,2
  w += (uint32_t)__builtin_amdgcn_update_dpp(0, (int)w, 0x4E, 0xF, 0xF, false);   // quad_perm 2,3,0,1
  w += (uint32_t)__builtin_amdgcn_update_dpp(0, (int)w, 0x141, 0xF, 0xF, false);  // row_half_mirror

  if (li == 0 && live) {
    uint32_t tr = 0;
    if (kind == 1) {  // xsum == 0xffff (segment.go:180)
      tr = rx_fold(init + rx_class(w));
      verdict = tr == 0xFFFFu ? kValid : kInvalid;
    } else if (kind == 2) {  // ^ChecksumVV(data with the field zeroed) == the field (icmp.go:72-80)
      tr = rx_class(w);
      verdict = (~tr & 0xFFFFu) == want ? kValid : kInvalid;
    } else if (kind == 3) {  // ICMPv6Checksum == the field (ipv6/icmp.go:76-84)
      tr = rx_fold(init + rx_class(w));
      verdict = (~tr & 0xFFFFu) == want ? kValid : kInvalid;
    }
    if (g.verdict) g.verdict[s] = (uint8_t)verdict;
    if (g.sums) {
      g.sums[2 * s] = (uint16_t)net;
      g.sums[2 * s + 1] = (uint16_t)tr;
    }
    if (over) atomicAdd(g.err, 1ull);
  }
}

// Lines per batch for the ring's longest frame: every line of an MTU packet
// (1,500 B from any offset: 13 lines) in one batch, 16 at most.
static int rx_batch_lines(const RxGeo& g) {
  const uint64_t longest = g.stride < (uint64_t)kMaxIp + g.frame_at + g.link ? g.stride : (uint64_t)kMaxIp + g.frame_at + g.link;
  const uint64_t lines = (longest + 15 + 127) / 128 + 1;
  return lines <= 2 ? 2 : lines <= 4 ? 4 : lines <= 8 ? 8 : lines <= 13 ? 13 : 16;
}

hipError_t launch_rx_ring(const RxGeo& g, hipStream_t stream) {
  if (g.n == 0) return hipSuccess;
  const uint64_t per_wg = (uint64_t)kWaves * kPerWave;
  const dim3 grid((uint32_t)((g.n + per_wg - 1) / per_wg)), block(64 * kWaves);
  switch (rx_batch_lines(g)) {
    case 2: hipLaunchKernelGGL(rx_ring<2>, grid, block, 0, stream, g); break;
    case 4: hipLaunchKernelGGL(rx_ring<4>, grid, block, 0, stream, g); break;
    case 8: hipLaunchKernelGGL(rx_ring<8>, grid, block, 0, stream, g); break;
    case 13: hipLaunchKernelGGL(rx_ring<13>, grid, block, 0, stream, g); break;
    default: hipLaunchKernelGGL(rx_ring<16>, grid, block, 0, stream, g); break;
  }
  return hipGetLastError();
}

}  // namespace nsk
