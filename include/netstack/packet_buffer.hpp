// netstack/packet_buffer.hpp — C++ mirror of google/netstack
// tcpip.PacketBuffer (tcpip/packet_buffer.go:25-50): the packet as it moves
// through the stack.  The batched checksum steps over these are
// netstack::header::VerifyPacketBuffers / FillPacketBuffers (header.hpp).
#pragma once

#include "netstack/buffer.hpp"

namespace netstack {
namespace tcpip {

struct PacketBuffer {
  // Data holds the payload; for inbound packets also the headers, consumed
  // as the packet moves up the stack (packet_buffer.go:27-33).
  buffer::VectorisedView Data;
  // Header holds the headers of outbound packets; each layer prepends
  // (packet_buffer.go:35-37).
  buffer::Prependable Header;
  buffer::View LinkHeader;
  buffer::View NetworkHeader;
  buffer::View TransportHeader;

  // packet_buffer.go:55-58: a new VectorisedView over the same bytes.
  PacketBuffer Clone() const { return *this; }
};

}  // namespace tcpip
}  // namespace netstack
