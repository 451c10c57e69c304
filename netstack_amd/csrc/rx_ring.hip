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
// A buffer list (ns_csum_rx_bufs, LIST = 1) is the same parse over buffers at
// per-packet offsets in one arena (a NIC's buffer pool) instead of slots.
//
// Shape.  A wave owns 8 consecutive slots, one 8-lane group per packet (16
// slots and 4-lane groups reading 64-B units on rings of short slots, G = 4:
// there the per-packet parse, not memory, is the cost).  The
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

// The W sum of row bytes [x, y) of a packet's LDS row (x even; y may be
// odd): dwords with halfword masks, the odd last byte on its own.  Every
// range the receive path sums from the row starts at an even offset, so a
// boundary never splits a halfword except at an odd end.
template <int MAXD>
__device__ __forceinline__ uint32_t rx_row_wsum(const uint8_t* row, uint32_t x, uint32_t y) {
  const uint32_t* D = reinterpret_cast<const uint32_t*>(row);
  const uint32_t ye = y & ~1u;
  const uint32_t len = ye > x ? ye - x : 0u;
  const uint32_t d0 = x >> 2;
  const uint32_t nd = len ? ((ye + 3) >> 2) - d0 : 0u;
  uint32_t w = 0;
  // a wave-uniform trip count (the longest lane's), the lanes past their own
  // end masked: no divergent branch per dword
  for (uint32_t k = 0; k < MAXD && __builtin_amdgcn_ballot_w64(k < nd) != 0; ++k) {
    const uint32_t o = 4u * (d0 + k);
    const uint32_t m = ((o - x) < len ? 0x0000FFFFu : 0u) | ((o + 2u - x) < len ? 0xFFFF0000u : 0u);
    w = __builtin_amdgcn_sad_u16(D[k < nd ? d0 + k : 0u] & m, 0u, w);
  }
  if ((y & 1u) && y > x) w += row[y - 1];  // a lone byte at an even offset: the low byte of its word
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
// takes further batches of NB lines.  A0 / AN = the cache policy of line 0 /
// of the others (0 default, 2 nontemporal), WV = waves per workgroup, OCC =
// a waves-per-SIMD floor for the register allocator (1: none).  F = 1: the
// lines past line 1 are summed whole, as they arrive, with no per-chunk range
// check (the chunk holding the transport's end is corrected by the lane that
// re-reads it); a wave with a frame padded past its transport's end beyond
// line 1 re-reads those lines with the range check.  F = 0: every chunk
// range-checked.  The product runs <NB, 0, 2, 4, 1, 1>;
// tools/rx_ring_variants.hip times the others.
// LIST = 1: a buffer list (g.off): packet s's buffer at g.ring + g.off[s]; one
// buffer resource over the whole arena (< 4 GiB, 32-bit offsets).  A buffer
// that is misaligned or not inside the arena is malformed and counted.
// ROT = 1 (timing variant, tools/rx_ring_variants.hip): load slot k >= 2 of
// group g reads line 2 + (k - 2 + 3 g) mod (NB - 2), so the eight groups of
// a wave do not all ask for line k of their slots at once (the same lines
// are loaded and summed whole: the sums do not change).
// LIST = 2 (timing variant, tools/rx_ring_variants.hip 30-32): a buffer list
// already sorted into address buckets (g.bk_tup: off, len, list index), the
// outputs written at the list index; 3: at the sorted position (timing only);
// 4: 2 with the index loaded with the entry.  It lost.
// LL = 1 (timing variant, tools/rx_ring_variants.hip): the packet's last
// line (the one it may share with the next buffer) with the default cache
// policy, its other lines >= 1 with AN, through two predicated loads of which
// one reads nothing; only lines NB - 2 and NB - 1 (where an MTU frame ends)
// get the pair.
template <int NB, int A0 = 0, int AN = 2, int WV = kWaves, int OCC = 1, int F = 1, int SPEC = 0, int LIST = 0,
          int ROT = 0, int LL = 0, int G = 8>
__global__ __launch_bounds__(64 * WV) __attribute__((amdgpu_waves_per_eu(OCC))) void rx_ring(RxGeo g) {
  // G lanes per packet: a load unit of U = 16 G bytes per group instruction
  // (G = 8: a 128-B line), KR units holding the LDS row, PW packets per wave
  static_assert(G == 8 || (G == 4 && LIST == 0 && ROT == 0 && LL == 0 && SPEC == 0 && F == 1 && NB >= 3),
                "4-lane groups: rings only, the product shape");
  constexpr uint32_t U = 16u * G, US = G == 8 ? 7u : 6u, KR = G == 8 ? 2u : 3u, PW = 64u / G;
  __shared__ uint4 rx_lds[WV * PW * kRowBytes / 16];
  const uint32_t lane = threadIdx.x & 63u, grp = lane / G, li = lane & (G - 1u);
  const uint32_t wv = (uint32_t)__builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  const uint64_t s0 = ((uint64_t)blockIdx.x * WV + wv) * PW;  // the wave's first slot
  if (s0 >= g.n) return;  // a whole wave leaves together
  const uint64_t s = s0 + grp;
  const bool live = s < g.n;

  // The frame: recvmmsg's length, less the bytes before the frame (a virtio-
  // net header) and the link header.  A slot longer than the ring's stride is
  // malformed and counted (ns_csum_sync), a frame of no more than its link
  // header is dropped by the link (packet_dispatchers.go:268-270).
  if constexpr (LIST >= 2) {  // leave the bucket totals zero for the next sort
    if (blockIdx.x == 0 && threadIdx.x < g.bk_nb) g.bk_total[threadIdx.x] = 0u;
  }
  // LIST = 2: (off, len) from the sorted list; its list index (where the
  // outputs go) is read again at the end rather than held
  const uint32_t* tup32 = reinterpret_cast<const uint32_t*>(g.bk_tup);
  uint32_t rlen = live ? (LIST >= 2 ? tup32[4 * s + 1] : g.len[s]) : 0u;
  // LIST = 4 (timing): the list index read with the entry
  const uint32_t idx4 = LIST == 4 && live ? tup32[4 * s + 2] : 0u;
  const uint32_t pre = g.frame_at + g.link;
  uint64_t slot;
  uint64_t wbase;
  uint32_t nrec;
  bool bad = false;  // LIST: a buffer not 16-B aligned or not inside the arena
  if constexpr (LIST) {
    const uint32_t o = live ? (LIST >= 2 ? tup32[4 * s] : g.off[s]) : 0u;
    bad = live && ((o & 15u) || (uint64_t)o + g.stride > g.limit);
    if (bad) rlen = 0;  // parsed as an empty frame: malformed
    slot = g.ring + (bad ? 0u : o);
    // arena-relative 32-bit coordinates: one resource over the whole arena
    wbase = g.ring & ~127ull;
    nrec = (uint32_t)(g.ring + g.limit - wbase);
  } else {
    slot = g.ring + s * g.stride;
    // Wave-relative 32-bit coordinates: one buffer resource from the 128-B
    // line of the wave's first packet over its slots (< 8 strides + a line).
    wbase = (g.ring + s0 * g.stride + pre) & ~127ull;
    const uint64_t s_end = s0 + PW < g.n ? s0 + PW : g.n;
    nrec = (uint32_t)(g.ring + s_end * g.stride - wbase);
  }
  const __amdgpu_buffer_rsrc_t rsrc = rx_srd(wbase, nrec);
  const uint32_t pa = (uint32_t)(slot + pre - wbase);  // the IP packet's first byte
  const uint32_t po = pa & 15u;                         // its offset in its 16-B chunk (even)
  const uint32_t cl = (pa & ~(U - 1u)) + 16u * li;      // lane li's chunk of line (unit) 0
  uint4 v[NB];
  // SPEC (timing variants): line 0 (1: and line 1, 2) loaded before the
  // length arrives: bytes past the frame only ever reach the LDS row, whose
  // reads the parse gates by the lengths, and the sums range-check lines 0-1
  if constexpr (SPEC >= 1) v[0] = rx_load<A0>(rsrc, live ? cl : nrec);
  if constexpr (SPEC >= 2) v[1] = rx_load<AN>(rsrc, live ? cl + 128u : nrec);
  if constexpr (SPEC >= 1) __builtin_amdgcn_sched_barrier(0);
  const bool over = (uint64_t)rlen > g.stride;
  const uint32_t P = (!over && rlen > pre) ? rlen - pre : 0u;  // Data.Size()
  const uint32_t Pl = P < kMaxIp ? P : kMaxIp;                  // bytes any header can cover
  // chunk at o: loaded only where it holds packet bytes, else the range
  // check returns zeros without touching memory
  const uint32_t lim = Pl ? Pl + 15u : 0u;
  auto off_of = [&](uint32_t o) -> uint32_t { return (o + 15u - pa) < lim ? o : nrec; };
  // F: lines k >= 1 start past pa, so a chunk there holds packet bytes iff
  // it starts before pe: k <= klast.  The voffset is cl (or nrec) and the
  // line's 128 k goes in the instruction's offset field.
  const uint32_t pe = pa + Pl;
  const uint32_t klast = Pl && pe > cl ? (pe - 1u - cl) >> US : 0u;
  const bool any1 = Pl && pe > cl + U;  // some line k >= 1 holds packet bytes for this lane
  const uint32_t cl1 = any1 ? cl : nrec;

  if constexpr (SPEC < 1 && LIST && A0 == 0) {
    // a buffer list: line 0 nontemporal for a buffer that starts a line and
    // whose packet starts in that line (no other buffer can share it), with
    // the default policy otherwise; the other load reads nothing (offset
    // nrec: the resource's out-of-range zeros)
    const bool alone = (slot & 127u) == 0 && pre < 128u;
    const uint4 a = rx_load<0>(rsrc, alone ? nrec : off_of(cl));
    const uint4 b = rx_load<2>(rsrc, alone ? off_of(cl) : nrec);
    v[0] = make_uint4(a.x | b.x, a.y | b.y, a.z | b.z, a.w | b.w);
  } else if constexpr (SPEC < 1) {
    v[0] = rx_load<A0>(rsrc, off_of(cl));
  }
  const uint32_t rot = ROT && NB > 3 ? (3u * grp) % (uint32_t)(NB > 3 ? NB - 2 : 1) : 0u;
  // LL: the group's last line holding packet bytes
  const uint32_t kgl = LL && Pl ? (pe - 1u - (pa & ~127u)) >> 7 : 0xFFFFFFFFu;
  auto line = [&](int k) {
    if constexpr (F && LL) if (k >= NB - 2) {  // (the lines an MTU frame can end in: a probe)
      const uint32_t o = ((uint32_t)k <= klast ? cl1 : nrec) + 128u * k;
      const bool last = (uint32_t)k == kgl;
      const uint4 x = rx_load<AN>(rsrc, last ? nrec + 128u * k : o);
      const uint4 y = rx_load<0>(rsrc, last ? o : nrec + 128u * k);
      v[k] = make_uint4(x.x | y.x, x.y | y.y, x.z | y.z, x.w | y.w);
      return;
    }
    if constexpr (F && ROT && NB > 3) {
      if (k >= 2) {
        uint32_t kk = (uint32_t)k + rot;
        if (kk >= (uint32_t)NB) kk -= (uint32_t)(NB - 2);
        v[k] = rx_load<AN>(rsrc, (kk <= klast ? cl1 : nrec) + 128u * kk);
        return;
      }
    }
    if constexpr (F) v[k] = rx_load<AN>(rsrc, ((uint32_t)k <= klast ? cl1 : nrec) + U * k);
    else v[k] = rx_load<AN>(rsrc, off_of(cl + U * k));
  };
  if constexpr (SPEC < 2) line(1);
  // The EtherType (the link header's bytes 12-13, pa - 2): a buffer load on
  // a resource one line lower (pa - 2 may precede wbase), issued after the
  // lines the parse reads, so waiting for it waits for nothing more.
  uint32_t etype = 0;
  if (g.link) {
    const __amdgpu_buffer_rsrc_t re = rx_srd(wbase - 128u, nrec + 128u);
    const uint32_t e = (uint32_t)__builtin_amdgcn_raw_buffer_load_b16(re, (int)(P ? pa + 126u : nrec + 128u), 0, 0);
    etype = ((e & 0xFFu) << 8) | ((e >> 8) & 0xFFu);
  }
#pragma unroll
  for (int k = 2; k < NB; ++k) line(k);
  uint32_t w2 = 0;  // F: every loaded chunk of lines >= KR
  if constexpr (F) {
#pragma unroll
    for (int k = KR; k < NB; ++k) {
      w2 = __builtin_amdgcn_sad_u16(v[k].x, 0u, w2);
      w2 = __builtin_amdgcn_sad_u16(v[k].y, 0u, w2);
      w2 = __builtin_amdgcn_sad_u16(v[k].z, 0u, w2);
      w2 = __builtin_amdgcn_sad_u16(v[k].w, 0u, w2);
    }
  }

  // The first 96 B from the packet's 16-B chunk into the group's LDS row.
  uint8_t* row = reinterpret_cast<uint8_t*>(rx_lds) + (wv * PW + grp) * kRowBytes;
  const uint32_t f16 = pa & ~15u;
#pragma unroll
  for (int k = 0; k < (int)KR; ++k) {
    const uint32_t o = cl + U * k - f16;
    if (o < kRowBytes) *reinterpret_cast<uint4*>(row + o) = v[k];
  }
  __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
  __builtin_amdgcn_wave_barrier();
  __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");

  // Parse (every lane of the group, same LDS bytes).  h(i) = IP byte i.  The
  // rules are evaluated side by side and combined with selects (one path for
  // every packet kind: no divergent branches, few scalar instructions); every
  // byte read lies in the row, and a field only decides anything where the
  // rule that reads it has passed its length checks.
  auto h = [&](uint32_t i) -> uint32_t { return row[po + i]; };
  const uint32_t first = g.view0 && g.view0 < P ? g.view0 : P;  // the first view's length
  const uint32_t h0 = h(0), h2 = h(2), h3 = h(3), h4 = h(4), h5 = h(5), h6 = h(6), h7 = h(7), h9 = h(9);
  const uint32_t ver = h0 >> 4;
  const uint32_t np = g.link ? (etype == 0x0800u ? 4u : etype == 0x86DDu ? 6u : 0u) : ver;
  // IPv4 HandlePacket + IsValid (ipv4.go:341-353, header/ipv4.go:280-296);
  // hlen > first is not in IsValid (tests/golden/rx_choices.json)
  const uint32_t hlen = (h0 & 15u) * 4u, tlen = (h2 << 8) | h3;
  const bool v4 = P && np == 4 && first >= 20 && hlen >= 20 && hlen <= tlen && tlen <= P && hlen <= first && ver == 4;
  const uint32_t foff = ((((h6 & 0x1Fu) << 8) | h7) << 3) & 0xFFFFu;
  const bool frag = v4 && ((h6 & 0x20u) || foff);  // ipv4.go:355-385
  const uint32_t fsize = (tlen - hlen) & 0xFFFFu;
  const bool fragbad = tlen == hlen || ((foff + fsize - 1u) & 0xFFFFu) < foff;
  // IPv6 HandlePacket + IsValid (ipv6.go:168-177, header/ipv6.go:207-222)
  const uint32_t plen = (h4 << 8) | h5;
  const bool v6 = P && np == 6 && first >= 40 && plen <= P - 40 && ver == 6;
  const bool ip = (v4 && !frag) || v6;
  const uint32_t proto = v4 ? h9 : h6;
  const uint32_t a = v4 ? hlen : 40u;                  // the transport range [a, tend)
  const uint32_t tend = v4 ? tlen : 40u + plen;
  const uint32_t tsize = tend - a;
  const uint32_t tfl = (first < tend ? first : tend) - a;  // the transport's first view
  const uint32_t ta = h(a), toff = (h(a + 12) >> 4) * 4u;
  const uint32_t want = (h(a + 2) << 8) | h(a + 3);
  const bool tcp = ip && proto == 6, udp = ip && proto == 17, icmp4 = ip && v4 && proto == 1,
             icmp6 = ip && !v4 && proto == 58;
  // The minimum sizes, each against the transport's first view: TCP 20 and
  // UDP 8 (stack/nic.go:851, header/tcp.go:169, header/udp.go:56), ICMPv4 8
  // (ipv4/icmp.go:60, header/icmpv4.go:32), ICMPv6 8 (ipv6/icmp.go:68,
  // ICMPv6MinimumSize, header/icmpv6.go:35).
  const bool tcp_bad = tfl < 20 || toff < 20 || toff > tfl;  // + segment.parse (segment.go:159)
  // kind: 1 TCP, 2 ICMPv4 echo request (handleICMP, icmp.go:60-80), 3 ICMPv6
  const uint32_t kind = tcp && !tcp_bad ? 1u : icmp4 && tfl >= 8 && ta == 8 ? 2u : icmp6 && tfl >= 8 ? 3u : 0u;
  const bool malformed = !P || (g.link ? np != 0 && !v4 && !v6 : !v4 && !v6) || (frag && fragbad) ||
                         (tcp && tcp_bad) || (udp && tfl < 8) || (icmp4 && tfl < 8) || (icmp6 && tfl < 8);
  uint32_t verdict = malformed ? kMalformed : kUnchecked;  // the checked kinds are decided below
  const uint32_t b = kind ? tend : 0u;
  const uint32_t asz = v4 ? 8u : 32u;

  // The transport range splits at 16-B chunk boundaries (offsets r with
  // (r + po) % 16 == 0) into a head [hx, min(b, A)) summed from the LDS row
  // (after the ICMP field), whole chunks [A, B) summed from the registers, and
  // a tail [B, b) re-read by one lane.
  const uint32_t hs = kind == 0 ? 0u : kind == 1 ? a : a + 4u;
  const uint32_t A = ((hs + po + 15u) & ~15u) - po, B = ((b + po) & ~15u) - po;
  const uint32_t span = kind && B > A ? B - A : 0u;
  // lanes 0, 1, 2: the IPv4 header, the pseudo-header's addresses, the head
  uint32_t x = 0, y = 0;
  if (li == 0 && v4) {
    x = po;
    y = po + hlen;
  } else if (li == 1 && kind) {
    x = po + (asz == 8 ? 12u : 8u);
    y = x + asz;
  } else if (li == 2 && kind) {
    x = po + hs;
    y = po + (b < A ? b : A);
  }
  // The last loaded chunk (its offset from pa) and the first of line 2.
  const uint32_t rl = Pl ? ((pa + Pl - 1u) & ~15u) - pa : 0u;
  const uint32_t r2 = (pa & ~(U - 1u)) + KR * U - pa;
  // F: a frame padded past its transport's end with loaded chunks beyond the
  // transport's last chunk in lines >= 2 (their bytes are in w2; the chunk at
  // B is corrected below only if it holds transport bytes): the whole wave
  // sums lines >= 2 again with the range check.
  const bool slow = F && kind && rl >= r2 && (rl > B || (rl == B && b == B));
  const bool wslow = F && __builtin_amdgcn_ballot_w64(slow) != 0;
  uint32_t tail = 0;
  if (li == 3 && kind && b > B && B >= A) {  // bytes [B, b): one 16-B chunk, an L2 hit
    const uint4 t = rx_load<0>(rsrc, pa + B);  // a buffer load: no wait on the LDS traffic
    const int c = (int)(b - B);
    tail = rx_wsum4(make_uint4(t.x & rx_below(c), t.y & rx_below(c - 4), t.z & rx_below(c - 8),
                               t.w & rx_below(c - 12)));
    // F: in line >= 2 this chunk is in w2 whole; take its bytes past b back out
    if (F && B >= r2 && !wslow) tail -= rx_wsum4(t);
  }
  uint32_t rs = rx_row_wsum<16>(row, x, y);
  if (li == 2 && kind >= 2) rs += *reinterpret_cast<const uint16_t*>(row + po + a);  // ICMP bytes [a, a + 2)

  // The whole chunks: chunk at o (lane li, line k) counts iff A <= o - pa < B.
  uint32_t w = (li == 2 ? rs : 0u) + tail;
  const uint32_t d = cl - pa - A;
#pragma unroll
  for (int k = 0; k < (F ? (int)KR : NB); ++k) {
    const uint32_t t = rx_wsum4(v[k]);
    w += (d + U * k) < span ? t : 0u;
  }
  if constexpr (F) {
    // (both loops below take 4 lines at a time: their registers are not the
    // kernel's peak, and they run only for long or padded frames)
    if (wslow) {  // a padded frame in this wave: lines >= 2 re-read, range-checked
      w2 = 0;
      for (uint32_t k0 = KR; __builtin_amdgcn_ballot_w64((d + U * k0) < span) != 0; k0 += 4) {
#pragma unroll
        for (int k = 0; k < 4; ++k) {
          const uint32_t t = rx_wsum4(rx_load<AN>(rsrc, off_of(cl + U * (k0 + k))));
          w2 += (d + U * (k0 + k)) < span ? t : 0u;
        }
      }
    } else {
      for (uint32_t k0 = NB; __builtin_amdgcn_ballot_w64(k0 <= klast && kind) != 0; k0 += 4) {
#pragma unroll
        for (int k = 0; k < 4; ++k) {
          const uint4 x4 = rx_load<AN>(rsrc, ((k0 + k) <= klast ? cl1 : nrec) + U * (k0 + k));
          w2 = __builtin_amdgcn_sad_u16(x4.x, 0u, w2);
          w2 = __builtin_amdgcn_sad_u16(x4.y, 0u, w2);
          w2 = __builtin_amdgcn_sad_u16(x4.z, 0u, w2);
          w2 = __builtin_amdgcn_sad_u16(x4.w, 0u, w2);
        }
      }
    }
    w += w2;
  } else {
    for (uint32_t k0 = NB; __builtin_amdgcn_ballot_w64((d + U * k0) < span) != 0; k0 += NB) {
#pragma unroll
      for (int k = 0; k < NB; ++k) v[k] = rx_load<AN>(rsrc, off_of(cl + U * (k0 + k)));
#pragma unroll
      for (int k = 0; k < NB; ++k) {
        const uint32_t t = rx_wsum4(v[k]);
        w += (d + U * (k0 + k)) < span ? t : 0u;
      }
    }
  }
  w += (uint32_t)__builtin_amdgcn_update_dpp(0, (int)w, 0xB1, 0xF, 0xF, false);   // quad_perm 1,0,3,2
  w += (uint32_t)__builtin_amdgcn_update_dpp(0, (int)w, 0x4E, 0xF, 0xF, false);   // quad_perm 2,3,0,1
  if constexpr (G == 8) w += (uint32_t)__builtin_amdgcn_update_dpp(0, (int)w, 0x141, 0xF, 0xF, false);  // row_half_mirror
  const uint32_t addr = (uint32_t)__builtin_amdgcn_mov_dpp((int)rs, 0x55, 0xF, 0xF, false);  // lane 1's

  if (li == 0 && live) {
    // LIST = 3 (timing only: outputs in sorted order, not the list's)
    const uint64_t os = LIST == 2 ? (uint64_t)tup32[4 * s + 2] : LIST == 4 ? (uint64_t)idx4 : s;
    uint32_t tr = 0;
    if (kind == 1) {  // PseudoHeaderChecksum (checksum.go:112-122), then xsum == 0xffff (segment.go:180)
      tr = rx_fold(rx_fold(rx_class(addr) + (tsize & 0xFFFFu) + 6u) + rx_class(w));
      verdict = tr == 0xFFFFu ? kValid : kInvalid;
    } else if (kind == 2) {  // ^ChecksumVV(data with the field zeroed) == the field (icmp.go:72-80)
      tr = rx_class(w);
      verdict = (~tr & 0xFFFFu) == want ? kValid : kInvalid;
    } else if (kind == 3) {  // ICMPv6Checksum == the field (ipv6/icmp.go:76-84)
      tr = rx_fold(rx_fold(rx_class(addr) + tsize + 58u) + rx_class(w));
      verdict = (~tr & 0xFFFFu) == want ? kValid : kInvalid;
    }
    if (g.verdict) g.verdict[os] = (uint8_t)verdict;
    if (g.sums) {
      g.sums[2 * os] = (uint16_t)(v4 ? rx_class(rs) : 0u);
      g.sums[2 * os + 1] = (uint16_t)tr;
    }
    if (over || bad) atomicAdd(g.err, 1ull);
  }
}

// Lines per batch for the ring's longest frame: every line of an MTU packet
// (1,500 B from any offset: 13 lines) in one batch, 16 at most.  A slot's
// bytes [pa, slot + stride) start at most 126 B into a line (pa is even), so
// they span at most (stride + 126 + 127) / 128 lines.  A buffer list's
// stride is the buffers' capacity, not the frames' length (2-KiB buffers
// holding MTU frames): it takes 13 at most, and longer frames take further
// batches (measured on 1536- to 2048-B pools of MTU frames: no change in
// time, fewer registers held).
static int rx_batch_lines(const RxGeo& g) {
  const uint64_t longest = g.stride < (uint64_t)kMaxIp + g.frame_at + g.link ? g.stride : (uint64_t)kMaxIp + g.frame_at + g.link;
  uint64_t lines = (longest + 126 + 127) / 128;
  if (g.off && lines > 13) lines = 13;
  return lines <= 2 ? 2 : lines <= 4 ? 4 : lines <= 8 ? 8 : lines <= 13 ? 13 : 16;
}

template <int NB, int A0 = 0, int AN = 2, int WV = kWaves, int OCC = 1, int F = 1, int SPEC = 0, int LIST = 0,
          int ROT = 0, int LL = 0, int G = 8>
static hipError_t launch_rx_ring_t(const RxGeo& g, hipStream_t stream) {
  if (g.n == 0) return hipSuccess;
  const uint64_t per_wg = (uint64_t)WV * (64u / G);
  hipLaunchKernelGGL((rx_ring<NB, A0, AN, WV, OCC, F, SPEC, LIST, ROT, LL, G>),
                     dim3((uint32_t)((g.n + per_wg - 1) / per_wg)), dim3(64 * WV), 0, stream, g);
  return hipGetLastError();
}

// 4-lane groups (G = 4: 16 packets per wave, 64-B load units) for a ring
// whose frames span at most 8 units: the per-packet parse is the kernel's
// cost below a few hundred bytes, and a wave then parses twice the packets.
// 0: not eligible (a longer stride or a buffer list).
static int rx_batch_units4(const RxGeo& g) {
  if (g.off) return 0;
  const uint64_t longest = g.stride < (uint64_t)kMaxIp + g.frame_at + g.link ? g.stride : (uint64_t)kMaxIp + g.frame_at + g.link;
  const uint64_t units = (longest + 62 + 63) / 64;
  return units <= 4 ? 4 : units <= 8 ? 8 : 0;
}

template <int LIST, int A0 = 0>
static hipError_t launch_rx_ring_l(const RxGeo& g, hipStream_t stream) {
  switch (rx_batch_lines(g)) {
    case 2: return launch_rx_ring_t<2, A0, 2, kWaves, 1, 1, 0, LIST>(g, stream);
    case 4: return launch_rx_ring_t<4, A0, 2, kWaves, 1, 1, 0, LIST>(g, stream);
    case 8: return launch_rx_ring_t<8, A0, 2, kWaves, 1, 1, 0, LIST>(g, stream);
    case 13: return launch_rx_ring_t<13, A0, 2, kWaves, 1, 1, 0, LIST>(g, stream);
    default: return launch_rx_ring_t<16, A0, 2, kWaves, 1, 1, 0, LIST>(g, stream);
  }
}

// Line 0 takes the default cache policy because its first bytes may be the
// slot before's last ones.  A ring of line-aligned slots whose IP packets
// start in their slot's first line shares no line between slots: line 0
// goes nontemporal too (1536-B slots: 236.5 -> 234.2 us per 1M frames,
// tools/rx_ring_probe.py --stride 1536) -- but not where the stride is a
// multiple of 1 KiB (2048-B slots: 233.3-240.1 us nontemporal against
// 221.0-229.4 default; 1024, 3072, 4096 no better; profiles/r06/rxpow2/).
// Rings of short slots take 4-lane groups (rx_batch_units4; tools/
// rx_size_probe.py --variants 40,41, profiles/r06/rxg4/: per ring of ~1.5 GB,
// 64-B frames 903.9 -> 509.5 us, 128-B 665.3 -> 424.2, 256-B 369.9 -> 332.7;
// 576-B frames lose, 315.5 against 241.7, and keep 8-lane groups).
hipError_t launch_rx_ring(const RxGeo& g, hipStream_t stream) {
  if (g.off) return launch_rx_ring_l<1>(g, stream);
  switch (rx_batch_units4(g)) {
    case 4: return launch_rx_ring_t<4, 0, 2, kWaves, 1, 1, 0, 0, 0, 0, 4>(g, stream);
    case 8: return launch_rx_ring_t<8, 0, 2, kWaves, 1, 1, 0, 0, 0, 0, 4>(g, stream);
    default: break;
  }
  if ((g.ring & 127) == 0 && (g.stride & 127) == 0 && (g.stride & 1023) != 0 && g.frame_at + g.link < 128)
    return launch_rx_ring_l<0, 2>(g, stream);
  return launch_rx_ring_l<0>(g, stream);
}

}  // namespace nsk
