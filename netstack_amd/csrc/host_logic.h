// host_logic.h — the HIP-free host logic of the C ABI (csum_api.cpp), kept
// in one header so it also builds on its own for the sanitizer tests
// (tests/cpp/host_logic_test.cc under -fsanitize=address,undefined and
// -fsanitize=thread; `make -C netstack_amd/csrc sanitize`):
//   - clip_views: ChecksumVVWithOffset's view walk (checksum.go:72-96);
//   - ChainBuilder: chains of restart/continue pieces -> ns_pkt_desc runs;
//   - PacketBytes / plan_packet: tcpip.PacketBuffer checksum steps;
//   - cut_chunk: the host pipeline's chunking of a descriptor table;
//   - shard_plan: byte-balanced contiguous shards;
//   - ScratchRegistry: per-stream scratch bookkeeping (LRU, pins, release);
//   - FlatCombiner: flat combining of concurrent small synchronous calls.
// Plumbing only: no checksum arithmetic happens here (pseudo-header length
// and protocol words are folded with the reference's ChecksumCombine).
#pragma once

#include <stdint.h>

#include <algorithm>
#include <atomic>
#include <chrono>
#include <condition_variable>
#include <cstring>
#include <mutex>
#include <thread>
#include <utility>
#include <vector>

#include "netstack_csum.h"

namespace nsh {

// Largest run of VectorisedView pieces that may be merged into ONE descriptor
// and still equal Go's per-view chain (checksum.go:89): with initial <= 0xFFFF
// and L <= 131072 bytes the uint32 accumulator cannot wrap, neither in the
// chain nor in the merged sum (65535 * (1 + 65536) = 2^32 - 1).  A single
// piece is never split (its own wrap is reproduced exactly by the kernel).
constexpr uint64_t kMergeMax = 131072;

// ChecksumCombine (checksum.go:104-107).
inline uint16_t combine(uint16_t a, uint16_t b) {
  const uint32_t v = (uint32_t)a + (uint32_t)b;
  return (uint16_t)(v + (v >> 16));
}

inline bool any_cont(const ns_pkt_desc* d, uint32_t n) {
  for (uint32_t i = 0; i < n; ++i)
    if (d[i].flags & NS_DESC_CONT) return true;
  return false;
}

// Clip a VectorisedView to [off, off+size) exactly like checksum.go:72-96.
inline int clip_views(const ns_view* views, uint32_t nviews, int64_t off, int64_t size,
                      std::vector<std::pair<const uint8_t*, uint64_t>>* pieces) {
  if (off < 0 || size < 0) return NS_EINVAL;
  pieces->clear();
  uint64_t o = (uint64_t)off, s = (uint64_t)size;
  for (uint32_t k = 0; k < nviews; ++k) {
    const uint64_t vl = views[k].len;
    if (vl == 0) continue;  // :73-75
    if (!views[k].data) return NS_EINVAL;
    if (o >= vl) {  // :77-80
      o -= vl;
      continue;
    }
    const uint64_t l = std::min<uint64_t>(vl - o, s);  // :81-87
    if (l > 0xFFFFFFFFull) return NS_EINVAL;
    pieces->emplace_back(views[k].data + o, l);
    s -= l;  // :91-94
    if (s == 0) break;
    o = 0;
  }
  return NS_OK;
}

// One piece of a checksum chain: `restart` = a fresh Checksum(piece, xsum)
// (alignment restarts, checksum.go:52-55); otherwise the piece continues the
// previous piece's byte stream with its odd-byte carry (the view chaining of
// ChecksumVVWithOffset, checksum.go:89).
struct Piece {
  const uint8_t* p;
  uint64_t len;
  bool restart;
};

// Builds descriptors from chains of pieces.  Sink::append(p, len) makes the
// bytes part of the arena and returns their arena offset.
template <class Sink>
struct ChainBuilder {
  Sink& bytes;
  std::vector<ns_pkt_desc> desc;
  std::vector<uint32_t> result_at;  // index of the descriptor holding each chain's result
  std::vector<Piece> scratch;       // plan_packet's piece list, its capacity kept across packets
  explicit ChainBuilder(Sink& s) : bytes(s) {}

  // One chain (include/netstack_csum.h, ns_csum_chains): sum = initial,
  // odd = false; per piece (sum, odd) = calculateChecksum(piece, odd', sum)
  // with odd' = false on a restart piece.  A piece that follows the open
  // descriptor's bytes in the arena merges into it, up to kMergeMax bytes
  // (exact, see kMergeMax): a continue piece always, a restart piece when the
  // open descriptor ends on an even byte count (its first byte is then the
  // high byte of a word either way, and Go's fold between the two calls
  // gives the same value as summing on — DESIGN.md §2).  Otherwise a restart
  // piece opens a new descriptor with odd = 0.  Empty pieces are skipped
  // (checksum.go:73-75; Checksum(empty, x) == x), an empty restart piece
  // still clearing the odd carry.  A piece is never split.
  void chain(const Piece* p, size_t np, uint16_t initial) {
    bool first_desc = true;
    uint32_t parity = 0;  // odd flag carried to the next continue piece
    ns_pkt_desc cur{};
    bool open = false;
    auto close = [&]() {
      if (!open) return;
      desc.push_back(cur);
      open = false;
    };
    for (size_t k = 0; k < np; ++k) {
      const uint64_t len = p[k].len;
      if (len == 0) {
        if (p[k].restart) {
          close();
          parity = 0;
        }
        continue;
      }
      const bool big = len > kMergeMax;
      const uint64_t at = bytes.append(p[k].p, len);
      if (p[k].restart && parity != 0) close();  // odd carry pending: a new descriptor at odd = 0
      if (p[k].restart) parity = 0;
      if (open && (big || cur.len + len > kMergeMax || at != cur.off + cur.len)) close();
      if (!open) {
        cur.off = at;
        cur.len = 0;
        cur.initial = first_desc ? initial : 0;
        cur.flags = (uint16_t)((first_desc ? 0u : NS_DESC_CONT) | (parity ? NS_DESC_ODD : 0u));
        first_desc = false;
        open = true;
      }
      cur.len += (uint32_t)len;
      parity ^= (uint32_t)(len & 1);
      if (big) close();
    }
    close();
    if (first_desc) {  // no bytes at all: result = initial (checksum.go:97)
      ns_pkt_desc z{};
      z.initial = initial;
      desc.push_back(z);
    }
    result_at.push_back((uint32_t)desc.size() - 1);
  }

  // ChecksumVVWithOffset's view walk over already clipped pieces: the first
  // restarts, the rest continue (checksum.go:69-98).
  void segment(const std::vector<std::pair<const uint8_t*, uint64_t>>& pieces, uint16_t initial) {
    std::vector<Piece> ps;
    ps.reserve(pieces.size());
    for (size_t k = 0; k < pieces.size(); ++k) ps.push_back(Piece{pieces[k].first, pieces[k].second, k == 0});
    chain(ps.data(), ps.size(), initial);
  }

  // Each view its own calculateChecksum with odd=false, chained
  // (xsum = Checksum(v, xsum): udp/endpoint.go:811-813).
  void restart_chain(const std::vector<std::pair<const uint8_t*, uint64_t>>& pieces, uint16_t initial) {
    std::vector<Piece> ps;
    ps.reserve(pieces.size());
    for (const auto& pc : pieces) ps.push_back(Piece{pc.first, pc.second, true});
    chain(ps.data(), ps.size(), initial);
  }
};

// A vector whose first N elements live inline: a packet of a handful of views
// needs no heap allocation (two per packet were ~a third of the planning
// time of a recvmmsg batch; tools/plan_cost.cc).
template <class T, size_t N>
class InlineVec {
 public:
  void reserve(size_t) {}
  void push_back(const T& v) {
    if (n_ < N) {
      inl_[n_] = v;
    } else {
      if (n_ == N) heap_.assign(inl_, inl_ + N);
      heap_.push_back(v);
    }
    ++n_;
  }
  template <class... A>
  void emplace_back(A&&... a) {
    push_back(T{std::forward<A>(a)...});
  }
  size_t size() const { return n_; }
  const T& operator[](size_t i) const { return n_ <= N ? inl_[i] : heap_[i]; }
  const T* begin() const { return n_ <= N ? inl_ : heap_.data(); }
  const T* end() const { return begin() + n_; }

 private:
  T inl_[N];
  std::vector<T> heap_;
  size_t n_ = 0;
};

// ---- tcpip.PacketBuffer batches (ns_csum_packet_buffers) -------------------
// A packet as one byte stream: its Header bytes, then its Data views clipped
// to Data.Size() (packet_buffer.go:25-50).  The host reads header fields from
// it (plumbing: lengths, positions of the addresses, protocol numbers) and
// cuts it into the pieces of each reference call sequence; every sum is
// computed by the kernel.
struct PacketBytes {
  InlineVec<std::pair<const uint8_t*, uint64_t>, 8> seg;  // non-empty segments in order
  InlineVec<uint64_t, 8> at;                              // byte offset of each segment
  uint64_t size = 0;
  uint64_t hdr_len = 0;  // bytes [0, hdr_len) are the Header's (writable)

  int init(const ns_pkt_buf& pk) {
    if (pk.hdr_len && !pk.hdr) return NS_EINVAL;
    if (pk.ndata && !pk.data) return NS_EINVAL;
    // A piece is one descriptor (u32 length), as in every other entry point.
    if (pk.hdr_len > 0xFFFFFFFFull) return NS_EINVAL;
    hdr_len = pk.hdr_len;
    seg.reserve((size_t)pk.ndata + 1);
    at.reserve((size_t)pk.ndata + 1);
    add(pk.hdr, pk.hdr_len);
    uint64_t left = pk.data_size;
    for (uint32_t k = 0; k < pk.ndata && left; ++k) {
      const uint64_t l = std::min<uint64_t>(pk.data[k].len, left);
      if (l && !pk.data[k].data) return NS_EINVAL;
      if (l > 0xFFFFFFFFull) return NS_EINVAL;
      add(pk.data[k].data, l);
      left -= l;
    }
    return NS_OK;
  }
  void add(const uint8_t* p, uint64_t l) {
    if (!l) return;
    seg.emplace_back(p, l);
    at.push_back(size);
    size += l;
  }
  // Segment holding byte k (k < size).
  size_t seg_of(uint64_t k) const {
    if (seg.size() < 2 || k < at[1]) return 0;  // the headers: nearly every lookup
    size_t lo = 1, hi = seg.size();
    while (hi - lo > 1) {
      const size_t mid = (lo + hi) / 2;
      if (at[mid] <= k) lo = mid;
      else hi = mid;
    }
    return lo;
  }
  // End of the segment (view) holding byte k: "Data.First()" after a trim to k.
  uint64_t seg_end(uint64_t k) const {
    if (k >= size) return size;
    const size_t s = seg_of(k);
    return at[s] + seg[s].second;
  }
  bool read(uint64_t k, uint8_t* out, uint64_t n) const {
    if (k > size || n > size - k) return false;
    while (n) {
      const size_t s = seg_of(k);
      const uint64_t o = k - at[s], l = std::min<uint64_t>(n, seg[s].second - o);
      std::memcpy(out, seg[s].first + o, l);
      out += l;
      k += l;
      n -= l;
    }
    return true;
  }
  uint8_t* mut(uint64_t k) const {  // address of byte k (a Header byte for stores)
    const size_t s = seg_of(k);
    return const_cast<uint8_t*>(seg[s].first) + (k - at[s]);
  }
  // Pieces covering [a, b), cut at view boundaries: the first `first_restart`,
  // then each next view restarting (`per_view`, the `xsum = Checksum(v, xsum)`
  // loops) or continuing (ChecksumVV's view walk).
  void pieces(uint64_t a, uint64_t b, bool first_restart, bool per_view, std::vector<Piece>* out) const {
    bool first = true;
    while (a < b) {
      const size_t s = seg_of(a);
      const uint64_t o = a - at[s], l = std::min<uint64_t>(b - a, seg[s].second - o);
      out->push_back(Piece{seg[s].first + o, l, first ? first_restart : per_view});
      first = false;
      a += l;
    }
  }
};

constexpr uint8_t kProtoICMPv4 = 1, kProtoTCP = 6, kProtoUDP = 17, kProtoICMPv6 = 58;

// One packet's plan: up to two chains (network header, transport) and where
// their results go.
struct PacketPlan {
  int net_chain = -1, tr_chain = -1;  // result indices in the builder
  uint8_t verdict = NS_PKB_UNCHECKED;
  uint8_t kind = 0;                   // transport protocol for the verdict
  uint64_t net_store = UINT64_MAX, tr_store = UINT64_MAX;  // FILL: field offsets
  uint16_t field = 0;                 // VERIFY (ICMP): the received checksum field
};

// The IP layer of a packet: header length, transport range and protocol, the
// pseudo-header address bytes.  parse_ip returns false for what IPv4/IPv6
// IsValid (header/ipv4.go:280-296, ipv6.go:207-222) and HandlePacket reject.
struct IpInfo {
  bool v4 = false;
  uint64_t hlen = 0, tbeg = 0, tend = 0, addr = 0, addr_len = 0;
  uint8_t proto = 0;
  bool fragment = false;
  uint16_t frag_off = 0;  // IPv4 FragmentOffset() in bytes (header/ipv4.go:167-169)
};

inline bool parse_ip(const PacketBytes& pb, bool rx, IpInfo* ip) {
  uint8_t h[40];
  if (pb.size < 1 || !pb.read(0, h, 1)) return false;
  const uint8_t ver = h[0] >> 4;
  // RX: the network header lies in Data.First() (packet_buffer.go:27-29);
  // IsValid looks at that view alone.
  const uint64_t first = pb.seg_end(0);
  if (ver == 4) {
    if ((rx && first < 20) || !pb.read(0, h, 20)) return false;
    ip->v4 = true;
    ip->hlen = (uint64_t)(h[0] & 0xF) * 4;
    const uint64_t tlen = ((uint64_t)h[2] << 8) | h[3];
    if (rx) {
      // IsValid (header/ipv4.go:280-296), plus `hlen > first`: where the
      // reference reslices past the first view or panics (ipv4.go:348), the
      // packet is MALFORMED (tests/golden/rx_choices.json).
      if (ip->hlen < 20 || ip->hlen > tlen || tlen > pb.size || ip->hlen > first) return false;
      ip->tend = tlen;  // Data.CapLength(tlen - hlen), ipv4.go:353
    } else {
      if (ip->hlen < 20 || ip->hlen > pb.size) return false;
      ip->tend = pb.size;
    }
    ip->proto = h[9];
    ip->addr = 12;
    ip->addr_len = 8;
    ip->frag_off = (uint16_t)((((h[6] & 0x1F) << 8) | h[7]) << 3);
    ip->fragment = (h[6] & 0x20) || ip->frag_off;  // MF or a fragment offset (ipv4.go:355-356)
  } else if (ver == 6) {
    if ((rx && first < 40) || !pb.read(0, h, 40)) return false;
    ip->hlen = 40;
    const uint64_t plen = ((uint64_t)h[4] << 8) | h[5];
    if (rx) {
      if (plen > pb.size - 40) return false;
      ip->tend = 40 + plen;  // Data.CapLength(PayloadLength), ipv6.go:177
    } else {
      ip->tend = pb.size;
    }
    ip->proto = h[6];
    ip->addr = 8;
    ip->addr_len = 32;
  } else {
    return false;
  }
  ip->tbeg = ip->hlen;
  return true;
}

// Builds one packet's chains.  RX (NS_PKB_VERIFY) mirrors the receive path's
// checks; TX (NS_PKB_FILL) the transmit path's sums (include/netstack_csum.h).
template <class Builder>
int plan_packet(Builder& g, const PacketBytes& pb, uint32_t op, PacketPlan* pp) {
  IpInfo ip;
  const bool rx = op == NS_PKB_VERIFY;
  if (!parse_ip(pb, rx, &ip)) {
    if (rx) {
      pp->verdict = NS_PKB_MALFORMED;
      return NS_OK;
    }
    return NS_EINVAL;
  }
  std::vector<Piece>& ps = g.scratch;  // capacity kept across the packets of a batch
  ps.clear();
  auto add_chain = [&](uint16_t init) {
    g.chain(ps.data(), ps.size(), init);
    ps.clear();
    return (int)g.result_at.size() - 1;
  };
  if (ip.v4) {
    // TX: the IPv4 checksum field is written into Header, so the whole IP
    // header must lie there (addIPHeader prepends it, ipv4.go:217-238); a
    // header reaching into Data (borrowed, read-only bytes) is NS_EINVAL.
    if (!rx && ip.hlen > pb.hdr_len) return NS_EINVAL;
    // TX: addIPHeader's ip.SetChecksum(^ip.CalculateChecksum()) (ipv4.go:236),
    // CalculateChecksum = Checksum(b[:HeaderLength()], 0) (ipv4.go:251-253).
    // RX: not verified on receive in the reference; reported for the caller.
    pb.pieces(0, ip.hlen, true, false, &ps);
    pp->net_chain = add_chain(0);
    if (!rx) pp->net_store = 10;
  }
  const uint64_t t0 = ip.tbeg, te = ip.tend, tl = te - t0;
  const uint64_t first_end = std::min(pb.seg_end(t0), te);  // Data.First() after the IP trim
  pp->kind = ip.proto;
  auto pseudo = [&](uint8_t proto, uint64_t len, bool icmpv6) -> uint16_t {
    // PseudoHeaderChecksum (checksum.go:112-122) / ICMPv6Checksum's
    // pseudo-header (icmpv6.go:204-210): the addresses in place, the length
    // and protocol words as the initial.  The pieces are all even-length
    // restarts, so any grouping of them gives Go's value (both
    // are fold1 of the same total, and 0 only when every piece is 0).
    pb.pieces(ip.addr, ip.addr + ip.addr_len, true, false, &ps);
    if (icmpv6) return combine(combine((uint16_t)(len >> 16), (uint16_t)len), proto);
    return combine((uint16_t)len, proto);
  };
  if (rx) {
    if (ip.fragment) {
      // ipv4.go:357-373: a fragment with no payload, or whose uint16
      // `last = FragmentOffset() + size - 1` wraps below its offset, is
      // dropped as malformed.  Any other fragment is reassembled before the
      // transport layer sees it (:375-385): UNCHECKED, its checksum is
      // verified after reassembly (receive contract).
      const uint16_t last = (uint16_t)(ip.frag_off + (uint16_t)tl - 1);
      if (tl == 0 || last < ip.frag_off) pp->verdict = NS_PKB_MALFORMED;
      return NS_OK;
    }
    if (ip.proto == kProtoTCP) {
      // stack.DeliverTransportPacket: First() >= TCPMinimumSize; segment.parse
      // (segment.go:145-181): offset in [20, len(First())]
      uint8_t h[13];
      if (first_end - t0 < 20 || !pb.read(t0, h, 13)) {
        pp->verdict = NS_PKB_MALFORMED;
        return NS_OK;
      }
      const uint64_t off = (uint64_t)(h[12] >> 4) * 4;
      if (off < 20 || off > first_end - t0) {
        pp->verdict = NS_PKB_MALFORMED;
        return NS_OK;
      }
      const uint16_t init = pseudo(kProtoTCP, (uint16_t)tl, false);  // :176 PseudoHeaderChecksum(data.Size())
      pb.pieces(t0, t0 + off, true, false, &ps);                     // :177 h.CalculateChecksum(xsum)
      pb.pieces(t0 + off, te, true, false, &ps);                     // :179 ChecksumVV(s.data, xsum)
      pp->tr_chain = add_chain(init);
      pp->verdict = NS_PKB_INVALID;  // decided from the result (:180)
    } else if (ip.proto == kProtoICMPv4 && ip.v4) {
      // handleICMP (network/ipv4/icmp.go:60-80): echo requests only
      uint8_t h[4];
      if (first_end - t0 < 8 || !pb.read(t0, h, 4)) {
        pp->verdict = NS_PKB_MALFORMED;
        return NS_OK;
      }
      if (h[0] != 8) return NS_OK;
      pp->field = (uint16_t)((h[2] << 8) | h[3]);
      // h.SetChecksum(0); ^ChecksumVV(pkt.Data, 0): bytes [2, 4) as zeros
      pb.pieces(t0, t0 + 2, true, false, &ps);
      pb.pieces(t0 + 4, te, false, false, &ps);
      pp->tr_chain = add_chain(0);
      pp->verdict = NS_PKB_INVALID;
    } else if (ip.proto == kProtoICMPv6 && !ip.v4) {
      // handleICMP (network/ipv6/icmp.go:62-84): h = the first view, payload
      // = the other views, ICMPv6Checksum (header/icmpv6.go:202-221); a first
      // view under ICMPv6MinimumSize (8, header/icmpv6.go:35) is dropped (:68)
      uint8_t h[4];
      if (first_end - t0 < 8 || !pb.read(t0, h, 4)) {
        pp->verdict = NS_PKB_MALFORMED;
        return NS_OK;
      }
      pp->field = (uint16_t)((h[2] << 8) | h[3]);
      const uint16_t init = pseudo(kProtoICMPv6, tl, true);
      pb.pieces(first_end, te, true, true, &ps);        // for v in vv.Views(): Checksum(v, xsum)
      pb.pieces(t0, t0 + 2, true, false, &ps);          // Checksum(h with h[2:4] = 0, xsum)
      pb.pieces(t0 + 4, first_end, false, false, &ps);
      pp->tr_chain = add_chain(init);
      pp->verdict = NS_PKB_INVALID;
    } else if (ip.proto == kProtoUDP && first_end - t0 < 8) {
      // stack.DeliverTransportPacket: First() >= UDPMinimumSize (stack/nic.go:
      // 851); UDP takes no checksum on receive otherwise (UNCHECKED)
      pp->verdict = NS_PKB_MALFORMED;
    }
    return NS_OK;
  }
  // TX of an IPv4 fragment: writePacketFragments (ipv4.go:119-212) writes only
  // each fragment's IP header checksum (:159-160); the transport checksum was
  // computed over the whole segment before it was cut, and a later fragment
  // carries no transport header at all.
  if (ip.fragment) return NS_OK;
  // TX: the transport header follows the IP header in Header; its checksum
  // field must lie in Header (it is written there).
  const uint64_t hdr_end = pb.hdr_len;
  auto need = [&](uint64_t field_end) { return field_end <= hdr_end; };
  if (ip.proto == kProtoTCP) {
    uint8_t h[13];
    if (!pb.read(t0, h, 13)) return NS_EINVAL;
    const uint64_t thl = (uint64_t)(h[12] >> 4) * 4;
    if (thl < 20 || t0 + thl > te || !need(t0 + 18)) return NS_EINVAL;
    // buildTCPHdr (connect.go:653-663): PseudoHeaderChecksum(length),
    // ChecksumVVWithOffset(payload), tcp.CalculateChecksum(xsum) = Checksum(tcp[:DataOffset])
    const uint16_t init = pseudo(kProtoTCP, (uint16_t)tl, false);
    pb.pieces(t0 + thl, te, true, false, &ps);
    pb.pieces(t0, t0 + thl, true, false, &ps);
    pp->tr_chain = add_chain(init);
    pp->tr_store = t0 + 16;
  } else if (ip.proto == kProtoUDP) {
    if (t0 + 8 > te || !need(t0 + 8)) return NS_EINVAL;
    // sendUDP (udp/endpoint.go:808-815): per-view restart, then the header
    const uint16_t init = pseudo(kProtoUDP, (uint16_t)tl, false);
    pb.pieces(t0 + 8, te, true, true, &ps);
    pb.pieces(t0, t0 + 8, true, false, &ps);
    pp->tr_chain = add_chain(init);
    pp->tr_store = t0 + 6;
  } else if (ip.proto == kProtoICMPv4 && ip.v4) {
    // the echo reply (network/ipv4/icmp.go:96-100): pkt = the ICMP bytes in
    // Header, SetChecksum(0), ^Checksum(pkt, ChecksumVV(vv, 0))
    if (!need(t0 + 4)) return NS_EINVAL;
    pb.pieces(hdr_end, te, true, false, &ps);
    pb.pieces(t0, t0 + 2, true, false, &ps);
    pb.pieces(t0 + 4, hdr_end, false, false, &ps);
    pp->tr_chain = add_chain(0);
    pp->tr_store = t0 + 2;
  } else if (ip.proto == kProtoICMPv6 && !ip.v4) {
    // ICMPv6Checksum(h = the ICMP bytes in Header, src, dst, Data) (icmpv6.go:202-221)
    if (!need(t0 + 4)) return NS_EINVAL;
    const uint16_t init = pseudo(kProtoICMPv6, tl, true);
    pb.pieces(hdr_end, te, true, true, &ps);
    pb.pieces(t0, t0 + 2, true, false, &ps);
    pb.pieces(t0 + 4, hdr_end, false, false, &ps);
    pp->tr_chain = add_chain(init);
    pp->tr_store = t0 + 2;
  }
  return NS_OK;
}

// After the device pass: FILL writes SetChecksum(^sum) big-endian into each
// packet's Header; VERIFY turns the sums into verdicts (TCP: xsum == 0xffff,
// segment.go:180; ICMP: ^sum == the received field).
inline void finish_packet(const PacketBytes& pb, PacketPlan& p, uint32_t op, const uint16_t* res, uint16_t* sums2,
                          uint8_t* verdict) {
  const uint16_t net = p.net_chain >= 0 ? res[(size_t)p.net_chain] : 0;
  const uint16_t tr = p.tr_chain >= 0 ? res[(size_t)p.tr_chain] : 0;
  if (sums2) {
    sums2[0] = net;
    sums2[1] = tr;
  }
  if (op == NS_PKB_FILL) {
    auto put = [&](uint64_t at, uint16_t v) {
      uint8_t* q = pb.mut(at);
      q[0] = (uint8_t)(v >> 8);
      q[1] = (uint8_t)v;
    };
    if (p.net_store != UINT64_MAX) put(p.net_store, (uint16_t)~net);
    if (p.tr_store != UINT64_MAX) put(p.tr_store, (uint16_t)~tr);
  } else if (verdict) {
    if (p.tr_chain >= 0) {
      const bool ok = p.kind == kProtoTCP ? tr == 0xFFFF : (uint16_t)~tr == p.field;
      p.verdict = ok ? NS_PKB_VALID : NS_PKB_INVALID;
    }
    *verdict = p.verdict;
  }
}

// ---- the host pipeline's chunking (ns_csum_batch_host) ---------------------
// The next chunk starting at descriptor k: grows while its byte span stays
// within `budget` and it holds at most `max_desc` descriptors (so the CPU's
// table copy of one chunk overlaps the other chunk's transfers), never ending
// inside a NS_DESC_CONT run of a chained table; a single run larger than the
// budget becomes one chunk.  Descriptors are range-checked on the way.
// Returns NS_OK with [k, *cut) and its byte span [*lo, *hi) (0, 0 if empty),
// or NS_ERANGE for a descriptor past the arena.
inline int cut_chunk(const ns_pkt_desc* d, uint32_t n, uint32_t k, uint64_t arena_bytes, uint64_t budget,
                     uint32_t max_desc, bool chained, uint32_t* cut_out, uint64_t* lo_out, uint64_t* hi_out) {
  uint64_t lo = UINT64_MAX, hi = 0;
  uint32_t j = k;
  uint32_t cut = k;  // last index (exclusive) at which we may cut
  uint64_t cut_lo = 0, cut_hi = 0;
  while (j < n) {
    const uint64_t off = d[j].off, len = d[j].len;
    if (off > arena_bytes || len > arena_bytes - off) return NS_ERANGE;
    uint64_t nlo = lo, nhi = hi;  // empty descriptors do not widen the span
    if (len) {
      nlo = std::min(lo, off);
      nhi = std::max(hi, off + len);
    }
    if (j > k && cut > k && ((nlo != UINT64_MAX && nhi - nlo > budget) || j - k >= max_desc)) break;
    lo = nlo;
    hi = nhi;
    ++j;
    if (j == n || !(chained && (d[j].flags & NS_DESC_CONT))) {
      cut = j;
      cut_lo = lo;
      cut_hi = hi;
    }
  }
  if (cut == k) {  // only possible at the end: take everything left
    cut = j;
    cut_lo = lo;
    cut_hi = hi;
  }
  if (cut_lo == UINT64_MAX || cut_hi < cut_lo) cut_lo = cut_hi = 0;
  *cut_out = cut;
  *lo_out = cut_lo;
  *hi_out = cut_hi;
  return NS_OK;
}

// ---- sharding (ns_csum_shard_plan) -------------------------------------------
// Splits n descriptors into `parts` contiguous ranges with near-equal payload
// bytes (cut at byte quantiles of the prefix sum of len), never inside a
// NS_DESC_CONT run; first[parts] = n.
inline void shard_plan(const ns_pkt_desc* d, uint32_t n, uint32_t parts, uint32_t* first) {
  uint64_t total = 0;
  for (uint32_t i = 0; i < n; ++i) total += d[i].len;
  first[0] = 0;
  uint64_t run = 0;
  uint32_t i = 0;
  for (uint32_t p = 1; p < parts; ++p) {
    // Cut at the first descriptor whose prefix reaches p/parts of the bytes;
    // with all-empty tables fall back to equal descriptor counts.
    const uint64_t target = total ? (total * p + parts - 1) / parts : 0;
    if (total == 0) {
      i = (uint32_t)(((uint64_t)n * p) / parts);
    } else {
      while (i < n && run + d[i].len <= target) run += d[i++].len;
    }
    while (i > 0 && i < n && (d[i].flags & NS_DESC_CONT)) run += d[i++].len;  // never split a chained run
    first[p] = std::max(i, first[p - 1]);
  }
  first[parts] = n;
}

// ---- per-stream scratch registry (ns_csum_batch_dev, ns_csum_stream_release)
// The device-resident API keeps scratch per caller stream (csum_api.cpp
// StreamScratch).  This is its bookkeeping, HIP-free so the sanitizer tests
// cover it: entries keyed by (stream handle, thread — hipStreamPerThread
// names a different stream in every thread), pinned while a call grows or
// launches with one, at most `max` kept (a new key evicts the least recently
// used unpinned entry), released on request.  `make()` builds an entry
// (nullptr on failure); `retire(e)` frees one and is called with the
// registry lock held, never for a pinned entry.
struct ScratchKey {
  const void* stream = nullptr;
  std::thread::id thread{};
  bool operator==(const ScratchKey& o) const { return stream == o.stream && thread == o.thread; }
};
struct ScratchSlot {
  ScratchKey key;
  int pins = 0;
  uint64_t tick = 0;
};

template <class Entry>
class ScratchRegistry {
 public:
  explicit ScratchRegistry(size_t max) : max_(max) {}

  template <class Make, class Retire>
  Entry* pin(const ScratchKey& k, Make&& make, Retire&& retire) {
    std::lock_guard<std::mutex> lk(mu_);
    Entry* e = nullptr;
    for (Entry* x : v_)
      if (x->key == k) e = x;
    if (!e) {
      if (v_.size() >= max_) {
        size_t lru = SIZE_MAX;
        for (size_t i = 0; i < v_.size(); ++i)
          if (v_[i]->pins == 0 && (lru == SIZE_MAX || v_[i]->tick < v_[lru]->tick)) lru = i;
        if (lru != SIZE_MAX) {
          Entry* old = v_[lru];
          v_.erase(v_.begin() + (long)lru);
          retire(old);
        }
      }
      e = make();
      if (!e) return nullptr;
      e->key = k;
      v_.push_back(e);
    }
    e->pins++;
    e->tick = ++tick_;
    return e;
  }

  void unpin(Entry* e) {
    std::lock_guard<std::mutex> lk(mu_);
    e->pins--;
  }

  // NS_EINVAL if the key's entry is pinned (a call on it is running).
  template <class Retire>
  int release(const ScratchKey& k, Retire&& retire) {
    std::lock_guard<std::mutex> lk(mu_);
    for (size_t i = 0; i < v_.size(); ++i) {
      if (!(v_[i]->key == k)) continue;
      if (v_[i]->pins) return NS_EINVAL;
      Entry* old = v_[i];
      v_.erase(v_.begin() + (long)i);
      retire(old);
      break;
    }
    return NS_OK;
  }

  template <class Retire>
  void clear(Retire&& retire) {
    std::lock_guard<std::mutex> lk(mu_);
    for (Entry* e : v_) retire(e);
    v_.clear();
  }

  size_t size() {
    std::lock_guard<std::mutex> lk(mu_);
    return v_.size();
  }

 private:
  const size_t max_;
  std::mutex mu_;
  std::vector<Entry*> v_;
  uint64_t tick_ = 0;
};

// ---- flat combining of concurrent small synchronous calls ------------------
// netstack calls the checksum from every endpoint's goroutine at once
// (SURVEY.md §8(b)); one launch + wait costs ~15-20 us whatever its size, so
// serialising calls would cap a context at ~50K calls/s.  A caller queues its
// request; if no pass is running it becomes the combiner: it takes queued
// requests (while their table bytes fit `pass_bytes`), runs them as ONE pass,
// hands out the results and repeats while requests remain (up to kMaxPasses
// passes, so back-to-back passes do not wait for a sleeping thread to wake).
// Everyone else spins briefly, then sleeps until its request is done.
// Req needs: uint64_t table_bytes() const; int rc; std::atomic<bool> done.
template <class Req>
class FlatCombiner {
 public:
  explicit FlatCombiner(uint64_t pass_bytes) : pass_bytes_(pass_bytes) {}

  // run(Req* const* reqs, size_t n) executes one pass and returns its status.
  template <class Run>
  int submit(Req* req, Run&& run) {
    constexpr int kMaxPasses = 8;
    std::unique_lock<std::mutex> ql(mu_);
    pending_.push_back(req);
    while (!req->done.load(std::memory_order_acquire)) {
      if (combining_) {
        // Spin briefly (a pass is ~20-60 us) before sleeping: a woken thread
        // costs more than the spin.
        ql.unlock();
        const auto t0 = std::chrono::steady_clock::now();
        while (!req->done.load(std::memory_order_acquire) &&
               std::chrono::steady_clock::now() - t0 < std::chrono::microseconds(50))
          std::this_thread::yield();
        ql.lock();
        if (req->done.load(std::memory_order_acquire)) break;
        if (combining_) cv_.wait(ql);
        continue;
      }
      combining_ = true;
      for (int pass = 0; pass < kMaxPasses && !pending_.empty(); ++pass) {
        std::vector<Req*> take;
        uint64_t staged = 0;
        size_t i = 0;
        for (; i < pending_.size(); ++i) {
          const uint64_t sz = pending_[i]->table_bytes();
          if (!take.empty() && staged + sz > pass_bytes_) break;
          take.push_back(pending_[i]);
          staged += sz;
        }
        pending_.erase(pending_.begin(), pending_.begin() + (long)i);
        ql.unlock();
        const int rc = run(take.data(), take.size());
        for (Req* t : take) {
          t->rc = rc;
          t->done.store(true, std::memory_order_release);
        }
        ql.lock();
        cv_.notify_all();
        if (req->done.load(std::memory_order_relaxed) && pass + 1 >= kMaxPasses) break;
      }
      combining_ = false;
      cv_.notify_all();  // a waiter takes the role over if requests remain
    }
    return req->rc;
  }

 private:
  const uint64_t pass_bytes_;
  std::mutex mu_;
  std::condition_variable cv_;
  std::vector<Req*> pending_;
  bool combining_ = false;
};

// ns_csum_tcp_tx's geometry, validated (include/netstack_csum.h): the
// segment count n = ceil(size / mss) (connect.go:675) and what the passes
// compute (tcp_tx.hip kTx* bits: 1 IPv4, 2 full TCP, 4 pseudo-header only,
// 8 field-only stores).  NS_OK with n = 0 or mode & 7 = 0: nothing to fill.
struct TxPlan {
  uint64_t n = 0;
  uint32_t mode = 0;
};
inline int tx_plan(const ns_tcp_tx& t, uint64_t arena_bytes, TxPlan* out) {
  if (t.mss == 0 || t.mss > 0xFFFFu || t.slot == 0 || t.slot > 4096) return NS_EINVAL;
  const bool partial = (t.flags & NS_TX_TCP_PARTIAL) != 0, none = (t.flags & NS_TX_TCP_NONE) != 0;
  if ((partial && none) || (t.flags & ~(NS_TX_TCP_PARTIAL | NS_TX_TCP_NONE | NS_TX_FIELDS_ONLY))) return NS_EINVAL;
  if (t.ip_len && (t.ip_len < 12 || t.ip_len > 60 || (uint32_t)t.ip_at + t.ip_len > t.slot)) return NS_EINVAL;
  if (!none && (t.tcp_len < 18 || t.tcp_len > 60 || (uint32_t)t.tcp_at + t.tcp_len > t.slot)) return NS_EINVAL;
  // PseudoHeaderChecksum takes uint8(protocol) (checksum.go:121): a wider
  // value has no reference meaning.
  if (t.protocol > 0xFFu) return NS_EINVAL;
  // The two headers are summed from one copy of the slot, each with the
  // other's field already written: they must not share bytes (the reference
  // prepends them one before the other, ipv4.go:217-238).
  if (t.ip_len && !none && (uint32_t)t.ip_at < (uint32_t)t.tcp_at + t.tcp_len &&
      (uint32_t)t.tcp_at < (uint32_t)t.ip_at + t.ip_len)
    return NS_EINVAL;
  const uint64_t n = t.size / t.mss + (t.size % t.mss != 0);
  if (n >= (1ull << 32)) return NS_EINVAL;
  const uint32_t mode = (t.ip_len ? 1u : 0u) | (none ? 0u : partial ? 4u : 2u) |
                        ((t.flags & NS_TX_FIELDS_ONLY) ? 8u : 0u);
  out->n = n;
  out->mode = mode;
  if (n == 0 || !(mode & 7u)) return NS_OK;
  const uint64_t hdr_bytes = n * t.slot;
  if (t.hdr_off > arena_bytes || hdr_bytes > arena_bytes - t.hdr_off) return NS_ERANGE;
  if (t.pay_off > arena_bytes || t.size > arena_bytes - t.pay_off) return NS_ERANGE;
  // The payload is read while other waves write slots back: they must not meet.
  if ((mode & 2u) && t.pay_off < t.hdr_off + hdr_bytes && t.hdr_off < t.pay_off + t.size) return NS_EINVAL;
  return NS_OK;
}

// Two interval lists merged into one sorted by lo.  Callers usually pack
// their calls side by side, so each list is sorted only if it is not already:
// O(n) instead of a sort for packed calls (23,832 calls: a 4-5 ms plan).
template <typename Iv>
inline void merge_by_lo(std::vector<Iv>& a, std::vector<Iv>& b, std::vector<Iv>* out) {
  auto lt = [](const Iv& x, const Iv& y) { return x.lo < y.lo; };
  if (!std::is_sorted(a.begin(), a.end(), lt)) std::sort(a.begin(), a.end(), lt);
  if (!std::is_sorted(b.begin(), b.end(), lt)) std::sort(b.begin(), b.end(), lt);
  out->resize(a.size() + b.size());
  std::merge(a.begin(), a.end(), b.begin(), b.end(), out->begin(), lt);
}

// ns_csum_tcp_tx_multi: every call checked as above, then the ranges the
// one launch touches: no call's slots may overlap another's slots, nor any
// payload a full-mode call reads (waves of other calls write slots back while
// it streams).  Payloads may overlap each other (they are only read).
inline int tx_multi_plan(const ns_tcp_tx* t, uint32_t count, uint64_t arena_bytes, std::vector<TxPlan>* plans) {
  plans->assign(count, TxPlan{});
  struct Iv {
    uint64_t lo, hi;
    bool slots;
  };
  std::vector<Iv> sl, pl, iv;
  sl.reserve(count);
  for (uint32_t k = 0; k < count; ++k) {
    const int rc = tx_plan(t[k], arena_bytes, &(*plans)[k]);
    if (rc != NS_OK) return rc;
    const TxPlan& p = (*plans)[k];
    if (p.n == 0 || !(p.mode & 7u)) continue;
    sl.push_back({t[k].hdr_off, t[k].hdr_off + p.n * t[k].slot, true});
    if ((p.mode & 2u) && t[k].size) pl.push_back({t[k].pay_off, t[k].pay_off + t[k].size, false});
  }
  merge_by_lo(sl, pl, &iv);
  uint64_t slot_end = 0, pay_end = 0;
  for (const Iv& v : iv) {
    if (v.slots) {
      if (v.lo < slot_end || v.lo < pay_end) return NS_EINVAL;
      slot_end = std::max(slot_end, v.hi);
    } else {
      if (v.lo < slot_end) return NS_EINVAL;
      pay_end = std::max(pay_end, v.hi);
    }
  }
  return NS_OK;
}

// ns_csum_tcp_tx_host's plan (sendTCPBatch calls over host memory).  The
// geometry is affine in the segment index (segment i's payload starts at
// pay_off + i*mss, its slot at hdr_off + i*slot; connect.go:679-691), so a run
// [a, b) of one call's segments is itself a call — hdr_off + a*slot, pay_off +
// a*mss, size min(size - a*mss, (b-a)*mss) — with the same segment lengths,
// pseudo-header length words and sums.  Each call is cut into such pieces of
// at most `budget` bytes (its slots plus the payload a full-mode call reads;
// one segment may exceed it), consecutive pieces are grouped into chunks of
// at most kMaxTxHostPieces pieces whose staging is at most `budget` bytes
// (a one-piece chunk excepted), and a chunk uploads its pieces' byte ranges
// merged where they overlap or lie within kTxHostGap bytes of each other —
// the gap bytes travel and count against the budget.  Each merged range goes to the chunk's staging at its
// arena offset modulo 256, so the kernel meets the alignments it would meet
// in the arena.
constexpr uint64_t kTxHostGap = 4096;
constexpr uint32_t kMaxTxHostPieces = 1u << 16;
struct TxPiece {
  ns_tcp_tx t;       // the run as a call (arena offsets)
  uint64_t nseg;     // its segments
  uint64_t out0;     // its first segment's index over all calls' segments
  uint32_t mode;     // TxPlan::mode
};
struct TxRange {
  uint64_t lo, hi;  // arena bytes [lo, hi)
  uint64_t at;      // their staging offset
};
struct TxChunk {
  uint32_t p0 = 0, np = 0;  // pieces [p0, p0 + np)
  uint32_t r0 = 0, nr = 0;  // ranges [r0, r0 + nr), sorted by lo
  uint64_t staging = 0;     // staging bytes the ranges take
  uint64_t out0 = 0;        // its pieces' segments are [out0, out0 + nout) over all calls
  uint64_t nout = 0;
};
struct TxHostPlan {
  std::vector<TxPiece> pieces;
  std::vector<TxRange> ranges;
  std::vector<TxChunk> chunks;
  // calls with segments but nothing to compute (TX offload, no IPv4
  // header): their sums are 0, as ns_csum_tcp_tx_multi writes them
  std::vector<std::pair<uint64_t, uint64_t>> zeros;  // (first segment, segments)
  uint64_t nseg = 0;                                 // all calls' segments

  // The staging offset of arena byte x, which lies in one of chunk c's ranges.
  uint64_t map(const TxChunk& c, uint64_t x) const {
    const TxRange* b = ranges.data() + c.r0;
    const TxRange* e = b + c.nr;
    const TxRange* r = std::upper_bound(b, e, x, [](uint64_t v, const TxRange& q) { return v < q.lo; }) - 1;
    return r->at + (x - r->lo);
  }
};

// Segments [a, a + nseg) of call c as a call of their own.
inline ns_tcp_tx tx_run(const ns_tcp_tx& c, uint64_t a, uint64_t nseg) {
  ns_tcp_tx r = c;
  r.hdr_off = c.hdr_off + a * c.slot;
  r.pay_off = c.pay_off + a * c.mss;
  r.size = std::min<uint64_t>(c.size - a * c.mss, nseg * c.mss);
  return r;
}

// ns_csum_tcp_tx_host_multi's split: the calls (checked by tx_multi_plan)
// cut into `parts` consecutive lists of runs, balanced by the bytes each
// uploads (slots, and the payload of full-mode calls): a list ends once it
// holds ceil(total / parts) bytes, cutting a call between segments where
// needed.  Calls with nothing to compute stay whole in the list they fall
// in.  seg0[p] = the index over all calls' segments of list p's first
// segment, so list p's sums are h_out[2 seg0[p] ...].  Lists may be empty.
inline void tx_shard_calls(const ns_tcp_tx* t, uint32_t count, const std::vector<TxPlan>& plans, uint32_t parts,
                           std::vector<std::vector<ns_tcp_tx>>* out, std::vector<uint64_t>* seg0) {
  out->assign(parts, {});
  seg0->assign(parts, 0);
  auto per_seg = [&](uint32_t k) {
    return (plans[k].n && (plans[k].mode & 7u)) ? (uint64_t)t[k].slot + ((plans[k].mode & 2u) ? t[k].mss : 0u) : 0u;
  };
  uint64_t total = 0;
  for (uint32_t k = 0; k < count; ++k)
    if (per_seg(k)) total += plans[k].n * t[k].slot + ((plans[k].mode & 2u) ? t[k].size : 0u);
  const uint64_t quota = std::max<uint64_t>(1, (total + parts - 1) / parts);
  uint32_t p = 0;
  uint64_t have = 0, seg = 0;
  for (uint32_t k = 0; k < count; ++k) {
    const uint64_t n = plans[k].n, b = per_seg(k);
    if (!b) {  // whole, wherever it falls
      (*out)[p].push_back(t[k]);
      seg += n;
      continue;
    }
    for (uint64_t a = 0; a < n;) {
      if (have >= quota && p + 1 < parts) {
        ++p;
        have = 0;
        (*seg0)[p] = seg;
      }
      // segments that fit the part's quota (at least one; the last part takes the rest)
      const uint64_t room = p + 1 < parts ? (quota - have + b - 1) / b : n - a;
      const uint64_t m = std::min<uint64_t>(n - a, std::max<uint64_t>(1, room));
      const ns_tcp_tx r = tx_run(t[k], a, m);
      (*out)[p].push_back(r);
      have += m * t[k].slot + ((plans[k].mode & 2u) ? r.size : 0u);
      a += m;
      seg += m;
    }
  }
  for (uint32_t q = p + 1; q < parts; ++q) (*seg0)[q] = seg;
}

inline int tx_host_plan(const ns_tcp_tx* t, uint32_t count, uint64_t arena_bytes, uint64_t budget,
                        TxHostPlan* out) {
  std::vector<TxPlan> plans;
  const int vr = tx_multi_plan(t, count, arena_bytes, &plans);
  if (vr != NS_OK) return vr;
  if (budget == 0) return NS_EINVAL;
  out->pieces.clear();
  out->ranges.clear();
  out->chunks.clear();
  out->zeros.clear();
  uint64_t seg = 0;
  std::vector<uint64_t> bytes;  // per piece
  for (uint32_t k = 0; k < count; ++k) {
    const ns_tcp_tx& c = t[k];
    const TxPlan& p = plans[k];
    if (p.n && !(p.mode & 7u)) out->zeros.emplace_back(seg, p.n);
    if (p.n && (p.mode & 7u)) {
      const bool full = (p.mode & 2u) != 0;
      const uint64_t per = (uint64_t)c.slot + (full ? c.mss : 0u);
      const uint64_t run = std::max<uint64_t>(1, budget / per);
      for (uint64_t a = 0; a < p.n; a += run) {
        TxPiece q;
        q.nseg = std::min(run, p.n - a);
        q.t = tx_run(c, a, q.nseg);
        q.out0 = seg + a;
        q.mode = p.mode;
        out->pieces.push_back(q);
        bytes.push_back(q.nseg * c.slot + (full ? q.t.size : 0u));
      }
    }
    seg += p.n;
  }
  out->nseg = seg;
  std::vector<TxRange> sl, pl, iv;
  // The staging pieces [p0, p1) take: their ranges merged (the bytes of the
  // gaps merged in count) at their offsets modulo 256 (the alignment counts);
  // `emit` appends the ranges to the plan.
  auto staging_of = [&](uint32_t p0, uint32_t p1, bool emit) -> uint64_t {
    sl.clear();
    pl.clear();
    for (uint32_t j = p0; j < p1; ++j) {
      const TxPiece& q = out->pieces[j];
      sl.push_back({q.t.hdr_off, q.t.hdr_off + q.nseg * q.t.slot, 0});
      if ((q.mode & 2u) && q.t.size) pl.push_back({q.t.pay_off, q.t.pay_off + q.t.size, 0});
    }
    merge_by_lo(sl, pl, &iv);
    uint64_t at = 0;
    for (size_t j = 0; j < iv.size();) {
      TxRange m = iv[j++];
      while (j < iv.size() && iv[j].lo <= m.hi + kTxHostGap) m.hi = std::max(m.hi, iv[j++].hi);
      m.at = ((at + 255) & ~255ull) + (m.lo & 255u);
      at = m.at + (m.hi - m.lo);
      if (emit) out->ranges.push_back(m);
    }
    return at;
  };
  const uint32_t np = (uint32_t)out->pieces.size();
  for (uint32_t i = 0; i < np;) {
    TxChunk ch;
    ch.p0 = i;
    uint64_t sum = 0;
    while (i < np && ch.np < kMaxTxHostPieces && (ch.np == 0 || sum + bytes[i] <= budget)) {
      sum += bytes[i++];
      ++ch.np;
    }
    // The pieces' own bytes fit the budget; with the gaps and alignment the
    // staging may not: keep the longest prefix whose staging fits (a single
    // piece always goes, and may exceed the budget by its own gap and
    // alignment, under 4.6 KiB).
    if (ch.np > 1 && staging_of(ch.p0, i, false) > budget) {
      uint32_t lo = 1, hi = ch.np - 1;  // lo: taken; counts above hi: too big
      while (lo < hi) {
        const uint32_t mid = lo + (hi - lo + 1) / 2;
        if (staging_of(ch.p0, ch.p0 + mid, false) <= budget) lo = mid;
        else hi = mid - 1;
      }
      ch.np = lo;
      i = ch.p0 + lo;
    }
    ch.r0 = (uint32_t)out->ranges.size();
    ch.staging = staging_of(ch.p0, i, true);
    ch.nr = (uint32_t)(out->ranges.size() - ch.r0);
    const TxPiece& last = out->pieces[i - 1];
    ch.out0 = out->pieces[ch.p0].out0;
    ch.nout = last.out0 + last.nseg - ch.out0;
    out->chunks.push_back(ch);
  }
  return NS_OK;
}

// ns_csum_rx_ring's geometry, validated (include/netstack_csum.h).  `base`
// is the device address of the arena (its alignment matters: 16-B loads).
inline int rx_plan(const ns_rx_ring& r, uint64_t base, uint64_t arena_bytes) {
  if (r.flags || r.stride == 0 || r.stride >= (1ull << 24) || (r.stride & 15u) || ((base + r.ring_off) & 15u))
    return NS_EINVAL;
  if ((r.link_hdr != 0 && r.link_hdr != 14) || ((r.frame_at + r.link_hdr) & 1u) || r.frame_at >= r.stride)
    return NS_EINVAL;
  if (r.first_view && ((r.first_view & 1u) || r.first_view < (uint32_t)r.link_hdr + 64u)) return NS_EINVAL;
  const uint64_t bytes = (uint64_t)r.n * r.stride;
  if (r.ring_off > arena_bytes || bytes > arena_bytes - r.ring_off) return NS_ERANGE;
  return NS_OK;
}

}  // namespace nsh
