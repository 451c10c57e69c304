// Copyright 2026 netstack-csum-mi355x authors.
//
// sendTCPBatch's n segment checksums in one engine call (SURVEY.md §8(f)
// rank 1).  ADDED to the reference's tcpip/transport/tcp together with
// go/netstack-hipcsum.patch, which makes sendTCPBatch (connect.go:668-702)
// defer the checksum of every segment to finishTCPBatchChecksums when this
// file is compiled in (-tags hipcsum).  csum_batch_go.go is the same
// function for the default build: the reference's per-segment loop.

// +build hipcsum

package tcp

import (
	"github.com/google/netstack/tcpip/buffer"
	"github.com/google/netstack/tcpip/header"
	"github.com/google/netstack/tcpip/stack"
)

// deferTCPBatchChecksums tells sendTCPBatch whether to defer its checksums
// here: only for a payload of at least header.ChainsOffloadMinBytes, where
// one engine call beats one core doing the segments' sums (INTEGRATION.md
// §2).  The reference's own sendTCPBatch payload is one GSO packet of at
// most 64 KiB (stack/registration.go:522-524), so with its settings this
// never defers and buildTCPHdr sums every segment as before.
func deferTCPBatchChecksums(payload int) bool {
	return payload >= header.ChainsOffloadMinBytes
}

// finishTCPBatchChecksums writes every segment's checksum into its TCP
// header: for segment i, buildTCPHdr's
//   xsum = ChecksumVVWithOffset(data, pseudo[i], Off, Size)   (connect.go:662)
//   tcp.SetChecksum(^tcp.CalculateChecksum(xsum))             (connect.go:663)
// as one chain per segment — the payload views (the first a restart, the
// rest continuing its odd-byte carry, checksum.go:69-98), then the header
// (a restart, tcp.go:259-262) — and all n chains in one device pass.  If the
// engine fails, the default build's loop computes them instead.
func finishTCPBatchChecksums(hdrs []stack.PacketDescriptor, data buffer.VectorisedView, pseudo []uint16) {
	chains := make([]header.ChecksumChain, len(hdrs))
	views := data.Views()
	for i := range hdrs {
		tcp := header.TCP(hdrs[i].Hdr.View())
		pieces := payloadPieces(views, hdrs[i].Off, hdrs[i].Size)
		pieces = append(pieces, header.ChecksumPiece{Buf: tcp[:tcp.DataOffset()], Restart: true})
		chains[i] = header.ChecksumChain{Initial: pseudo[i], Pieces: pieces}
	}
	sums := make([]uint16, len(hdrs))
	if err := header.ChecksumChainsErr(chains, sums); err != nil {
		// The engine could not run the call (counted in
		// header.EngineFallbacks): the reference's own per-segment loop, as
		// the default build runs it (csum_batch_ref.go).
		tcpBatchChecksumsRef(hdrs, data, pseudo)
		return
	}
	for i := range hdrs {
		header.TCP(hdrs[i].Hdr.View()).SetChecksum(^sums[i])
	}
}

// payloadPieces clips the views to [off, off+size) as ChecksumVVWithOffset
// walks them (checksum.go:72-96): empty views skipped, the first piece a
// restart, the others continuing it.
func payloadPieces(views []buffer.View, off, size int) []header.ChecksumPiece {
	var out []header.ChecksumPiece
	for _, v := range views {
		if len(v) == 0 {
			continue
		}
		if off >= len(v) {
			off -= len(v)
			continue
		}
		v = v[off:]
		if len(v) > size {
			v = v[:size]
		}
		out = append(out, header.ChecksumPiece{Buf: v, Restart: len(out) == 0})
		size -= len(v)
		if size == 0 {
			break
		}
		off = 0
	}
	return out
}
