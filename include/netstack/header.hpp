// netstack/header.hpp — C++ mirror of google/netstack tcpip/header checksum
// entry points (tcpip/header/checksum.go:52-122), every sum computed by the
// MI355X engine through the C ABI (include/netstack_csum.h).  Same names,
// argument meaning and un-complemented results as the Go functions.
//
// Error behaviour: where Go panics (negative off/size) these throw
// std::out_of_range; a HIP failure throws netstack::header::ChecksumError.
// There is no host fallback.
#pragma once

#include <cstdint>
#include <stdexcept>
#include <string>
#include <vector>

#include "netstack/buffer.hpp"
#include "netstack/packet_buffer.hpp"
#include "netstack_csum.h"

namespace netstack {
namespace header {

class ChecksumError : public std::runtime_error {
 public:
  ChecksumError(int status, const std::string& what)
      : std::runtime_error(what + ": " + ns_csum_strerror(status)), status_(status) {}
  int status() const { return status_; }

 private:
  int status_;
};

// The process-wide engine context for `device` (created once, like the Go
// shim's sync.Once).
ns_csum_ctx* Engine(int device = 0);

// checksum.go:52-55
uint16_t Checksum(const buffer::View& buf, uint16_t initial);
uint16_t Checksum(const std::vector<uint8_t>& buf, uint16_t initial);
// checksum.go:61-63
uint16_t ChecksumVV(const buffer::VectorisedView& vv, uint16_t initial);
// checksum.go:69-98
uint16_t ChecksumVVWithOffset(const buffer::VectorisedView& vv, uint16_t initial, long long off,
                              long long size);
// checksum.go:104-107
uint16_t ChecksumCombine(uint16_t a, uint16_t b);
// checksum.go:112-122 (addresses are raw 4- or 16-byte tcpip.Address strings)
uint16_t PseudoHeaderChecksum(uint32_t protocol, const std::string& srcAddr,
                              const std::string& dstAddr, uint16_t totalLen);

// One segment of a batched payload checksum: the Off/Size of a
// stack.PacketDescriptor (stack/route.go:174-178) plus its pseudo-header sum.
struct SegDesc {
  long long Off;
  long long Size;
  uint16_t Initial;
};
// n x ChecksumVVWithOffset in one device pass (sendTCPBatch,
// transport/tcp/connect.go:668-702).
std::vector<uint16_t> ChecksumVVBatch(const buffer::VectorisedView& vv,
                                      const std::vector<SegDesc>& segs);
// xsum = initial; for v in views: xsum = Checksum(v, xsum)
// (transport/udp/endpoint.go:811-813, header/icmpv4.go:158-160).
uint16_t ChecksumViews(const std::vector<buffer::View>& views, uint16_t initial);

// Batched checksum steps over tcpip.PacketBuffer (ns_csum_packet_buffers),
// one device pass per call.  Receive (a recvmmsg batch, Data = the IP
// packet): the verdict per packet — TCP segment.parse (segment.go:174-180),
// ICMPv4 echo (network/ipv4/icmp.go:72-80), ICMPv6 (network/ipv6/icmp.go:
// 76-84) — one of the constants below.  Transmit (Header = IP + transport
// headers, Data = payload): the transport checksum (buildTCPHdr, sendUDP,
// the ICMP echo reply, ICMPv6Checksum) and the IPv4 header checksum
// (addIPHeader) are written into each Header.
enum PacketVerdict : uint8_t {
  PacketChecksumInvalid = NS_PKB_INVALID,
  PacketChecksumValid = NS_PKB_VALID,
  PacketChecksumUnchecked = NS_PKB_UNCHECKED,
  PacketMalformed = NS_PKB_MALFORMED,
};
std::vector<uint8_t> VerifyPacketBuffers(const std::vector<tcpip::PacketBuffer>& pkts);
void FillPacketBuffers(std::vector<tcpip::PacketBuffer>& pkts);

}  // namespace header
}  // namespace netstack
