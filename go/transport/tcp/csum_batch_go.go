// Copyright 2026 netstack-csum-mi355x authors.
//
// The default build's side of csum_batch_hip.go (see there): with
// deferTCPBatchChecksums false, sendTCPBatch never defers, and buildTCPHdr
// computes every segment's checksum itself exactly as the reference does
// (connect.go:661-663).  finishTCPBatchChecksums is that same per-segment
// computation (tcpBatchChecksumsRef, csum_batch_ref.go), for completeness.

// +build !hipcsum

package tcp

import (
	"github.com/google/netstack/tcpip/buffer"
	"github.com/google/netstack/tcpip/stack"
)

func deferTCPBatchChecksums(payload int) bool {
	return false
}

func finishTCPBatchChecksums(hdrs []stack.PacketDescriptor, data buffer.VectorisedView, pseudo []uint16) {
	tcpBatchChecksumsRef(hdrs, data, pseudo)
}
