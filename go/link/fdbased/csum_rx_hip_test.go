// Copyright 2026 netstack-csum-mi355x authors.
//
// The engine path of the link's receive verification (csum_rx_hip.go) at
// the reference's own batch size: the test opens
// header.VerifyOffloadMinBytes, which otherwise keeps every 8-message
// recvmmsg batch on the CPU, and checks the verdicts written into
// PacketBuffer.RXChecksum against what segment.parse decides
// (segment.go:174-180: PseudoHeaderChecksum + the segment's sum == 0xffff).

// +build linux,hipcsum

package fdbased

import (
	"math/rand"
	"testing"

	"github.com/google/netstack/tcpip"
	"github.com/google/netstack/tcpip/buffer"
	"github.com/google/netstack/tcpip/header"
)

// rxPacket is an IPv4/TCP packet as recvmmsg leaves it in BufConfig's views
// (128 B, then the rest), both checksums set as a sender's stack sets them;
// corrupt flips one payload byte afterwards.
func rxPacket(rng *rand.Rand, payload int, corrupt bool) tcpip.PacketBuffer {
	src, dst := tcpip.Address("\x0a\x00\x00\x01"), tcpip.Address("\x0a\x00\x00\x02")
	total := header.IPv4MinimumSize + header.TCPMinimumSize + payload
	b := make([]byte, total)
	ip := header.IPv4(b)
	ip.Encode(&header.IPv4Fields{
		IHL:         header.IPv4MinimumSize,
		TotalLength: uint16(total),
		ID:          uint16(rng.Intn(65536)),
		TTL:         64,
		Protocol:    uint8(header.TCPProtocolNumber),
		SrcAddr:     src,
		DstAddr:     dst,
	})
	ip.SetChecksum(^ip.CalculateChecksum())
	tcp := header.TCP(b[header.IPv4MinimumSize:])
	tcp.Encode(&header.TCPFields{
		SrcPort:    uint16(1024 + rng.Intn(60000)),
		DstPort:    80,
		SeqNum:     rng.Uint32(),
		AckNum:     rng.Uint32(),
		DataOffset: header.TCPMinimumSize,
		Flags:      header.TCPFlagAck,
		WindowSize: 65535,
	})
	data := tcp[header.TCPMinimumSize:]
	rng.Read(data)
	xsum := header.PseudoHeaderChecksum(header.TCPProtocolNumber, src, dst, uint16(len(tcp)))
	xsum = header.Checksum(data, xsum)
	tcp.SetChecksum(^tcp.CalculateChecksum(xsum))
	if corrupt {
		data[rng.Intn(len(data))] ^= 0x40
	}
	views := []buffer.View{buffer.NewViewFromBytes(b[:128]), buffer.NewViewFromBytes(b[128:])}
	return tcpip.PacketBuffer{Data: buffer.NewVectorisedView(total, views)}
}

func TestVerifyRXChecksumsWithTheGateOpen(t *testing.T) {
	defer func(v int) { header.VerifyOffloadMinBytes = v }(header.VerifyOffloadMinBytes)
	rng := rand.New(rand.NewSource(7))
	pkts := make([]tcpip.PacketBuffer, MaxMsgsPerRecv)
	bad := map[int]bool{2: true, 5: true}
	for i := range pkts {
		pkts[i] = rxPacket(rng, 1460, bad[i])
	}
	// at the measured gate an 8 x 1500-B batch stays with segment.parse
	verifyRXChecksums(&endpoint{}, pkts)
	for i := range pkts {
		if pkts[i].RXChecksum != tcpip.RXChecksumUnknown {
			t.Fatalf("packet %d: %v below the gate", i, pkts[i].RXChecksum)
		}
	}
	header.VerifyOffloadMinBytes = 0
	before := header.EngineFallbacks()
	verifyRXChecksums(&endpoint{}, pkts)
	if header.EngineFallbacks() != before {
		t.Fatal("the engine did not run the batch (fallback counted)")
	}
	for i := range pkts {
		want := tcpip.RXChecksumValid
		if bad[i] {
			want = tcpip.RXChecksumInvalid
		}
		if pkts[i].RXChecksum != want {
			t.Fatalf("packet %d: %v, segment.parse would decide %v", i, pkts[i].RXChecksum, want)
		}
	}
}
