// Copyright 2026 netstack-csum-mi355x authors.
//
// sendTCPBatch's per-segment checksum as the reference computes it in
// buildTCPHdr (connect.go:661-663), shared by both builds: the default build's
// finishTCPBatchChecksums (csum_batch_go.go) is this loop, and the hipcsum
// build runs it when the engine cannot (csum_batch_hip.go).  Only the
// reference's own header functions are called.

package tcp

import (
	"github.com/google/netstack/tcpip/buffer"
	"github.com/google/netstack/tcpip/header"
	"github.com/google/netstack/tcpip/stack"
)

func tcpBatchChecksumsRef(hdrs []stack.PacketDescriptor, data buffer.VectorisedView, pseudo []uint16) {
	for i := range hdrs {
		xsum := header.ChecksumVVWithOffset(data, pseudo[i], hdrs[i].Off, hdrs[i].Size)
		tcp := header.TCP(hdrs[i].Hdr.View())
		tcp.SetChecksum(^tcp.CalculateChecksum(xsum))
	}
}
