// Copyright 2026 netstack-csum-mi355x authors.
//
// The link side of the receive contract (INTEGRATION.md §2, "Receive"):
// recvMMsgDispatcher.dispatch (packet_dispatchers.go:258-317, patched by
// go/netstack-hipcsum.patch) hands each recvmmsg batch here before
// delivering it.  One engine pass verifies every packet's transport checksum
// as segment.parse and handleICMP would (header.VerifyPacketBuffers); the
// verdict goes into PacketBuffer.RXChecksum, which segment.parse honours.
//
// The endpoint never advertises stack.CapabilityRXChecksumOffload for this:
// that bit is link-wide (segment.go:166-173), and a fragment cannot be
// verified before reassembly (ipv4.go:355-385).  Fragments and anything the
// pass does not check stay RXChecksumUnknown and are verified by the stack
// as usual; invalid packets are delivered too, so the stack drops and counts
// them where the reference does (tcp/endpoint.go:2108-2114).  Only batches
// of at least header.VerifyOffloadMinBytes go to the engine (see below).

// +build linux,hipcsum

package fdbased

import (
	"github.com/google/netstack/tcpip"
	"github.com/google/netstack/tcpip/header"
	"github.com/google/netstack/tcpip/stack"
)

func verifyRXChecksums(e *endpoint, pkts []tcpip.PacketBuffer) {
	if len(pkts) == 0 || e.Capabilities()&stack.CapabilityRXChecksumOffload != 0 {
		return // the NIC / host kernel verified them already
	}
	// Below header.VerifyOffloadMinBytes one core verifies the batch sooner
	// than one engine call (INTEGRATION.md §2): leave every packet
	// RXChecksumUnknown, and segment.parse verifies it as the reference does.
	// With MaxMsgsPerRecv = 8 that takes packets of 24,000 B on average (a
	// large-MTU link); 8 x 1500 B never reaches it.
	total := 0
	for i := range pkts {
		total += pkts[i].Data.Size()
	}
	if total < header.VerifyOffloadMinBytes {
		return
	}
	var verdict [MaxMsgsPerRecv]uint8
	if err := header.VerifyPacketBuffersErr(pkts, verdict[:len(pkts)]); err != nil {
		// The engine could not run the pass (counted in
		// header.EngineFallbacks): every packet stays RXChecksumUnknown and
		// segment.parse verifies it, as in the default build.
		return
	}
	for i := range pkts {
		switch verdict[i] {
		case header.PacketChecksumValid:
			pkts[i].RXChecksum = tcpip.RXChecksumValid
		case header.PacketChecksumInvalid:
			pkts[i].RXChecksum = tcpip.RXChecksumInvalid
		}
	}
}
