// Copyright 2026 netstack-csum-mi355x authors.
//
// FillTCPBatches (ns_csum_tcp_tx_host) against the reference's own Go
// computation of the same fields (fillTCPBatchGo: buildTCPHdr's
// PseudoHeaderChecksum, ChecksumVVWithOffset and TCP.CalculateChecksum,
// connect.go:652-663; addIPHeader's IPv4 CalculateChecksum, ipv4.go:236),
// byte for byte over whole slot buffers: many batches in one call, IPv4 and
// IPv6 routes, odd MSS and slot sizes, TCP options, payloads split over
// several views, CHECKSUM_PARTIAL and TX offload, no engine fallback counted.
// ADDED to the reference's tcpip/header; compiled only with -tags hipcsum.

// +build hipcsum

package header

import (
	"bytes"
	"math/rand"
	"testing"

	"github.com/google/netstack/tcpip"
	"github.com/google/netstack/tcpip/buffer"
)

func randomTCPBatch(r *rand.Rand, size, mss, slot, ipLen, tcpLen, mode int, v6 bool) TCPBatch {
	b := TCPBatch{SlotSize: slot, MSS: mss, TCPLen: tcpLen, Protocol: 6, Mode: mode}
	// the headers at the end of each slot, as Prependable leaves them
	b.TCPAt = slot - tcpLen
	if ipLen > 0 {
		b.IPAt, b.IPLen = b.TCPAt-ipLen, ipLen
	}
	src, dst := make([]byte, 4), make([]byte, 4)
	if v6 {
		src, dst = make([]byte, 16), make([]byte, 16)
	}
	r.Read(src)
	r.Read(dst)
	b.Src, b.Dst = tcpip.Address(src), tcpip.Address(dst)
	n := (size + mss - 1) / mss
	b.Slots = make([]byte, n*slot)
	r.Read(b.Slots)
	for i := 0; i < n; i++ {
		s := b.Slots[i*slot:][:slot]
		TCP(s[b.TCPAt:]).SetChecksum(0)
		s[b.TCPAt+12] = byte(tcpLen/4) << 4 // DataOffset
		if ipLen > 0 {
			s[b.IPAt] = 0x40 | byte(ipLen/4) // version 4, IHL
			IPv4(s[b.IPAt:]).SetChecksum(0)
		}
	}
	// the payload over several views of random lengths
	var views []buffer.View
	for left := size; left > 0; {
		l := 1 + r.Intn(3*mss)
		if l > left {
			l = left
		}
		v := buffer.NewView(l)
		r.Read(v)
		views = append(views, v)
		left -= l
	}
	b.Payload = buffer.NewVectorisedView(size, views)
	return b
}

func cloneTCPBatch(b TCPBatch) TCPBatch {
	c := b
	c.Slots = append([]byte(nil), b.Slots...)
	return c
}

func TestFillTCPBatchesMatchesReferenceGo(t *testing.T) {
	r := rand.New(rand.NewSource(42))
	var got, want []TCPBatch
	add := func(b TCPBatch) {
		got = append(got, b)
		want = append(want, cloneTCPBatch(b))
	}
	for rep := 0; rep < 3; rep++ {
		add(randomTCPBatch(r, 65536, 1460, 54+40, 20, 20, TxCsumFull, false)) // netstack's 64 KiB GSO write
		add(randomTCPBatch(r, 1461*7+3, 1461, 75, 0, 32, TxCsumFull, true))  // IPv6 route, TCP options
		add(randomTCPBatch(r, 999, 1460, 94, 20, 20, TxCsumFull, false))     // one short segment
		add(randomTCPBatch(r, 7*300+5, 7, 61, 24, 20, TxCsumFull, false))    // MSS 7, IPv4 options
		add(randomTCPBatch(r, 9000*3+1, 9000, 94, 20, 20, TxCsumPartial, false))
		add(randomTCPBatch(r, 1460*4, 1460, 94, 20, 20, TxCsumOffload, false))
	}
	before := EngineFallbacks()
	if err := FillTCPBatchesErr(got); err != nil {
		t.Fatalf("FillTCPBatchesErr: %v", err)
	}
	if f := EngineFallbacks(); f != before {
		t.Fatalf("engine fallbacks %d -> %d", before, f)
	}
	for i := range want {
		fillTCPBatchGo(&want[i])
		if !bytes.Equal(got[i].Slots, want[i].Slots) {
			t.Errorf("batch %d: slots differ from the reference's fill", i)
		}
	}
	// refilling filled slots is idempotent (both fields are summed as zero)
	if err := FillTCPBatchesErr(got); err != nil {
		t.Fatalf("refill: %v", err)
	}
	for i := range want {
		if !bytes.Equal(got[i].Slots, want[i].Slots) {
			t.Errorf("batch %d: refill changed the slots", i)
		}
	}
}

// FillTCPBatches itself: below TxBatchOffloadMinBytes the reference's code
// runs (no engine call); with the gate opened the engine fills the same
// bytes.  The gate is restored afterwards.
func TestFillTCPBatchesGate(t *testing.T) {
	defer func(v int) { TxBatchOffloadMinBytes = v }(TxBatchOffloadMinBytes)
	r := rand.New(rand.NewSource(7))
	for _, gate := range []int{1 << 30, 0} {
		TxBatchOffloadMinBytes = gate
		got := []TCPBatch{randomTCPBatch(r, 65536, 1460, 94, 20, 20, TxCsumFull, false),
			randomTCPBatch(r, 1460*3+1, 1460, 74, 0, 20, TxCsumFull, true)}
		want := []TCPBatch{cloneTCPBatch(got[0]), cloneTCPBatch(got[1])}
		before := EngineFallbacks()
		FillTCPBatches(got)
		if f := EngineFallbacks(); f != before {
			t.Fatalf("gate %d: engine fallbacks %d -> %d", gate, before, f)
		}
		for i := range want {
			fillTCPBatchGo(&want[i])
			if !bytes.Equal(got[i].Slots, want[i].Slots) {
				t.Errorf("gate %d, batch %d: slots differ from the reference's fill", gate, i)
			}
		}
	}
}
