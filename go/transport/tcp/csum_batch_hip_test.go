// Copyright 2026 netstack-csum-mi355x authors.
//
// The engine path of sendTCPBatch's deferred checksums (csum_batch_hip.go)
// at the reference's own sizes: the test opens header.ChainsOffloadMinBytes,
// which otherwise keeps every GSO payload (<= 64 KiB) on the CPU, and checks
// finishTCPBatchChecksums byte for byte against the reference's own loop
// (tcpBatchChecksumsRef: buildTCPHdr's ChecksumVVWithOffset +
// CalculateChecksum, connect.go:661-663) over the same segments.

// +build hipcsum

package tcp

import (
	"bytes"
	"math/rand"
	"testing"

	"github.com/google/netstack/tcpip"
	"github.com/google/netstack/tcpip/buffer"
	"github.com/google/netstack/tcpip/header"
	"github.com/google/netstack/tcpip/stack"
)

// tcpBatch builds a sendTCPBatch call as connect.go:668-702 lays it out: one
// payload VectorisedView (views of uneven lengths) cut at mss, a TCP header
// prepended in each of NewPacketDescriptors' slots, each segment's
// pseudo-header sum.  The same seed gives the same call.
func tcpBatch(seed int64, size, mss int) ([]stack.PacketDescriptor, buffer.VectorisedView, []uint16) {
	rng := rand.New(rand.NewSource(seed))
	var views []buffer.View
	for left := size; left > 0; {
		l := 1 + rng.Intn(3001)
		if l > left {
			l = left
		}
		v := buffer.NewView(l)
		rng.Read(v)
		views = append(views, v)
		left -= l
	}
	data := buffer.NewVectorisedView(size, views)
	n := (size + mss - 1) / mss
	hdrs := stack.NewPacketDescriptors(n, header.TCPMinimumSize)
	pseudo := make([]uint16, n)
	src, dst := tcpip.Address("\xc0\xa8\x01\x07"), tcpip.Address("\x0a\xc8\x03\x63")
	for i := range hdrs {
		off := i * mss
		sz := mss
		if size-off < sz {
			sz = size - off
		}
		hdrs[i].Off, hdrs[i].Size = off, sz
		tcp := header.TCP(hdrs[i].Hdr.Prepend(header.TCPMinimumSize))
		tcp.Encode(&header.TCPFields{
			SrcPort:    80,
			DstPort:    uint16(1000 + i),
			SeqNum:     rng.Uint32(),
			AckNum:     rng.Uint32(),
			DataOffset: header.TCPMinimumSize,
			Flags:      header.TCPFlagAck,
			WindowSize: uint16(rng.Intn(65536)),
		})
		pseudo[i] = header.PseudoHeaderChecksum(header.TCPProtocolNumber, src, dst, uint16(header.TCPMinimumSize+sz))
	}
	return hdrs, data, pseudo
}

func TestDeferGateOpensOnlyWhenSet(t *testing.T) {
	defer func(v int) { header.ChainsOffloadMinBytes = v }(header.ChainsOffloadMinBytes)
	if deferTCPBatchChecksums(64 << 10) {
		t.Fatalf("a 64 KiB GSO payload must stay on the CPU at the measured gate (%d B)", header.ChainsOffloadMinBytes)
	}
	header.ChainsOffloadMinBytes = 0
	if !deferTCPBatchChecksums(1) {
		t.Fatal("with the gate open every payload defers")
	}
}

func TestFinishTCPBatchChecksumsMatchesTheReferenceLoop(t *testing.T) {
	defer func(v int) { header.ChainsOffloadMinBytes = v }(header.ChainsOffloadMinBytes)
	header.ChainsOffloadMinBytes = 0
	for _, c := range []struct{ size, mss int }{
		{64 << 10, 1460},   // one GSO write, netstack's MSS
		{1460*3 + 1, 1460}, // a 1-byte last segment
		{7001, 7},          // many segments per view, odd MSS
		{1000, 1460},       // one short segment
	} {
		before := header.EngineFallbacks()
		got, data, pseudo := tcpBatch(int64(c.size), c.size, c.mss)
		finishTCPBatchChecksums(got, data, pseudo)
		if header.EngineFallbacks() != before {
			t.Fatalf("size %d mss %d: the engine did not run the call (fallback counted)", c.size, c.mss)
		}
		want, wdata, wpseudo := tcpBatch(int64(c.size), c.size, c.mss)
		tcpBatchChecksumsRef(want, wdata, wpseudo)
		for i := range got {
			if g, w := got[i].Hdr.View(), want[i].Hdr.View(); !bytes.Equal(g, w) {
				t.Fatalf("size %d mss %d segment %d: header %x, the reference's %x", c.size, c.mss, i, g, w)
			}
		}
	}
}
