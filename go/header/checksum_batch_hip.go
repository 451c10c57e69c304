// Copyright 2026 netstack-csum-mi355x authors.
//
// Batched checksum entry points for google/netstack's package header,
// computed by the MI355X (gfx950) engine behind include/netstack_csum.h
// through cgo.
//
// This file is ADDED to the reference's tcpip/header next to checksum.go,
// which stays untouched: the single-buffer functions (Checksum, ChecksumVV,
// ChecksumVVWithOffset, ChecksumCombine, PseudoHeaderChecksum,
// checksum.go:52-122) remain the reference's own Go code, because one GPU
// round trip (~11 us) costs far more than a 20-60-B header sum.  The callers'
// batches come here instead (SURVEY.md §8(b)): sendTCPBatch's n segments
// (tcp/connect.go:668-702), a recvmmsg batch of packet buffers
// (link/fdbased/packet_dispatchers.go:258-317), WritePackets' headers
// (network/ipv4/ipv4.go:271-285).  None of the names below exists in the
// reference's package header.
//
// Written for the reference's Go (<= 1.14: tcpip/time_unsafe.go:15-16):
// no runtime.Pinner, unsafe.Slice, unsafe.Add or generics.  cgo forbids
// passing C memory that holds Go pointers, so every byte the engine reads
// through a table is first copied into a staging buffer the engine leases
// (ns_csum_stage_acquire); the engine reads it there in place, and the tables
// handed to C hold only C pointers.  Contiguous Go buffers (ChecksumBatch)
// are passed directly, as cgo allows.
//
// Compiled only with -tags hipcsum; include and library paths come from
// CGO_CFLAGS / CGO_LDFLAGS (INTEGRATION.md §2).

// +build hipcsum

package header

/*
#cgo LDFLAGS: -lnetstack_csum
#include <stdint.h>
#include "netstack_csum.h"
*/
import "C"

import (
	"fmt"
	"reflect"
	"sync"
	"unsafe"

	"github.com/google/netstack/tcpip"
	"github.com/google/netstack/tcpip/buffer"
)

var (
	csumOnce sync.Once
	csumCtx  *C.ns_csum_ctx
	csumErr  C.int
	csumABI  C.int
)

// csumEngine returns the process-wide engine context for device 0, created
// once.  It refuses a library whose C ABI differs from the header this file
// was compiled against (a stale libnetstack_csum.so).
func csumEngine() *C.ns_csum_ctx {
	csumOnce.Do(func() {
		csumABI = C.ns_csum_abi_version()
		if csumABI != C.NS_CSUM_ABI_VERSION {
			return
		}
		var opts C.ns_csum_opts
		csumErr = C.ns_csum_init(&opts, &csumCtx)
	})
	if csumABI != C.NS_CSUM_ABI_VERSION {
		panic(fmt.Sprintf("netstack_csum: libnetstack_csum.so has C ABI %d, netstack_csum.h has %d: rebuild the library",
			int(csumABI), int(C.NS_CSUM_ABI_VERSION)))
	}
	if csumErr != C.NS_OK {
		// No host fallback: these batch functions exist only in the hipcsum
		// build, and a missing GPU is fatal like a slice-bound panic.
		panic(fmt.Sprintf("netstack_csum: ns_csum_init: %s", C.GoString(C.ns_csum_strerror(csumErr))))
	}
	return csumCtx
}

func csumMust(rc C.int, what string) {
	if rc != C.NS_OK {
		panic(fmt.Sprintf("netstack_csum: %s: %s", what, C.GoString(C.ns_csum_strerror(rc))))
	}
}

// csumStage is a leased engine staging buffer: pinned host memory the GPU
// reads in place.  mem is the same C memory as a Go slice.
type csumStage struct {
	base *C.uint8_t
	mem  []byte
	used int
}

func acquireStage(n int) *csumStage {
	if n < 1 {
		n = 1
	}
	s := &csumStage{}
	csumMust(C.ns_csum_stage_acquire(csumEngine(), C.uint64_t(n), &s.base), "ns_csum_stage_acquire")
	h := (*reflect.SliceHeader)(unsafe.Pointer(&s.mem))
	h.Data = uintptr(unsafe.Pointer(s.base))
	h.Len = n
	h.Cap = n
	return s
}

func (s *csumStage) release() {
	csumMust(C.ns_csum_stage_release(csumEngine(), s.base), "ns_csum_stage_release")
}

// put copies b into the stage; it returns b's C address there (nil if empty)
// and its offset.
func (s *csumStage) put(b []byte) (*C.uint8_t, int) {
	at := s.used
	if len(b) == 0 {
		return nil, at
	}
	copy(s.mem[at:], b)
	s.used += len(b)
	return (*C.uint8_t)(unsafe.Pointer(&s.mem[at])), at
}

// views reserves an 8-byte-aligned table of n ns_view in the stage (C
// memory, so a table that C reads through another table's pointer).
func (s *csumStage) views(n int) (*C.ns_view, []C.ns_view) {
	s.used = (s.used + 7) &^ 7
	if n == 0 {
		return nil, nil
	}
	if n > 1<<26 { // the array type below; a VectorisedView never gets near it
		panic("netstack_csum: more than 1<<26 views in one packet")
	}
	p := unsafe.Pointer(&s.mem[s.used])
	s.used += n * int(unsafe.Sizeof(C.ns_view{}))
	return (*C.ns_view)(p), (*[1 << 26]C.ns_view)(p)[:n:n]
}

func viewBytes(vs []buffer.View) int {
	n := 0
	for _, v := range vs {
		n += len(v)
	}
	return n
}

const viewEntry = int(unsafe.Sizeof(C.ns_view{}))

// SegDesc is one segment of a batched payload checksum: the Off/Size of a
// stack.PacketDescriptor (stack/route.go:174-178) and its pseudo-header sum.
type SegDesc struct {
	Off, Size int
	Initial   uint16
}

// ChecksumVVBatch sets out[i] = ChecksumVVWithOffset(vv, segs[i].Initial,
// segs[i].Off, segs[i].Size) (checksum.go:69-98) for every segment in one
// device pass: the n per-MSS payload sums of sendTCPBatch
// (transport/tcp/connect.go:668-702).
func ChecksumVVBatch(vv buffer.VectorisedView, segs []SegDesc, out []uint16) {
	if len(out) < len(segs) {
		panic("ChecksumVVBatch: out too short")
	}
	if len(segs) == 0 {
		return
	}
	for _, s := range segs {
		if s.Off < 0 || s.Size < 0 {
			panic("slice bounds out of range") // as v[off:] / v[:l] would in checksum.go
		}
	}
	vs := vv.Views()
	st := acquireStage(viewBytes(vs))
	defer st.release()
	tab := make([]C.ns_view, len(vs)) // Go memory holding only C pointers
	for i, v := range vs {
		p, _ := st.put(v)
		tab[i].data = p
		tab[i].len = C.uint64_t(len(v))
	}
	cs := make([]C.ns_seg, len(segs))
	for i, s := range segs {
		cs[i].off = C.int64_t(s.Off)
		cs[i].size = C.int64_t(s.Size)
		cs[i].initial = C.uint16_t(s.Initial)
	}
	var tp *C.ns_view
	if len(tab) > 0 {
		tp = &tab[0]
	}
	csumMust(C.ns_csum_vv_batch(csumEngine(), tp, C.uint32_t(len(tab)), &cs[0], C.uint32_t(len(cs)),
		(*C.uint16_t)(unsafe.Pointer(&out[0]))), "ChecksumVVBatch")
}

// ChecksumPiece is one buffer of a checksum chain.  Restart = a fresh
// Checksum(Buf, xsum) call (alignment restarts, checksum.go:52-55); otherwise
// the piece continues the previous one's byte stream with its odd-byte carry
// (ChecksumVVWithOffset's view chaining, checksum.go:89).
type ChecksumPiece struct {
	Buf     []byte
	Restart bool
}

// ChecksumChain is `xsum := Initial; for each piece: xsum = ...`.
type ChecksumChain struct {
	Initial uint16
	Pieces  []ChecksumPiece
}

// ChecksumChains evaluates every chain in one device pass (ns_csum_chains);
// out[i] is chain i's un-complemented sum.  One chain holds a whole TCP
// segment checksum — pseudo-header fields, payload views, the TCP header —
// so sendTCPBatch (connect.go:668-702) and a recvmmsg batch of segment.parse
// checks (segment.go:174-180) each take one call.
func ChecksumChains(chains []ChecksumChain, out []uint16) {
	if len(out) < len(chains) {
		panic("ChecksumChains: out too short")
	}
	if len(chains) == 0 {
		return
	}
	n, bytes := 0, 0
	for _, ch := range chains {
		if len(ch.Pieces) == 0 {
			n++
		}
		n += len(ch.Pieces)
		for _, pc := range ch.Pieces {
			bytes += len(pc.Buf)
		}
	}
	st := acquireStage(bytes)
	defer st.release()
	tab := make([]C.ns_piece, n) // Go memory holding only C pointers
	k := 0
	for _, ch := range chains {
		pieces := ch.Pieces
		if len(pieces) == 0 {
			pieces = []ChecksumPiece{{Restart: true}}
		}
		for j, pc := range pieces {
			p, _ := st.put(pc.Buf)
			tab[k].data = p
			tab[k].len = C.uint64_t(len(pc.Buf))
			if j == 0 {
				tab[k].initial = C.uint16_t(ch.Initial)
			}
			if pc.Restart {
				tab[k].flags |= C.NS_PIECE_RESTART
			}
			if j == len(pieces)-1 {
				tab[k].flags |= C.NS_PIECE_END
			}
			k++
		}
	}
	csumMust(C.ns_csum_chains(csumEngine(), &tab[0], C.uint32_t(n), (*C.uint16_t)(unsafe.Pointer(&out[0])),
		C.uint32_t(len(chains))), "ChecksumChains")
}

// BatchDesc is one packet of a contiguous batch: ns_pkt_desc (16 bytes) —
// stack.PacketDescriptor's Off/Size (route.go:174-178) plus the packet's
// pseudo-header sum and the NS_DESC_* flags (1: odd carry-in, 2: chained to
// the previous descriptor).
type BatchDesc struct {
	Off     uint64
	Len     uint32
	Initial uint16
	Flags   uint16
}

// ChecksumBatch sets out[i] to calculateChecksum(arena[d.Off:d.Off+d.Len],
// d.Flags&1 != 0, d.Initial), folded (checksum.go:26-46), for every
// descriptor in one device pass (chained runs with flag 2 when chained).
// arena and descs are contiguous Go memory without Go pointers, so they are
// passed to C directly.
func ChecksumBatch(arena []byte, descs []BatchDesc, out []uint16, chained bool) {
	if len(out) < len(descs) {
		panic("ChecksumBatch: out too short")
	}
	if len(descs) == 0 {
		return
	}
	var flags C.uint32_t
	if chained {
		flags = C.NS_BATCH_CHAINED
	}
	var ap *C.uint8_t
	if len(arena) > 0 {
		ap = (*C.uint8_t)(unsafe.Pointer(&arena[0]))
	}
	csumMust(C.ns_csum_batch_host(csumEngine(), ap, C.uint64_t(len(arena)),
		(*C.ns_pkt_desc)(unsafe.Pointer(&descs[0])), C.uint32_t(len(descs)),
		(*C.uint16_t)(unsafe.Pointer(&out[0])), flags), "ChecksumBatch")
}

// Verdicts of VerifyPacketBuffers (NS_PKB_*).
const (
	PacketChecksumInvalid   = 0
	PacketChecksumValid     = 1
	PacketChecksumUnchecked = 2 // nothing the reference verifies on receive
	PacketMalformed         = 3 // dropped by IsValid / the length checks first
)

// Offload thresholds.  A synchronous engine call costs one GPU round trip
// (~11 us) plus its bytes; below these sizes one core running the
// reference's own loop (checksum.go:26-46) on the same bytes finishes first
// (tools/crossover.cc on MI355X, profiles/r04/crossover.json; INTEGRATION.md
// §2 "When offload pays").  The build-tagged callers offload only calls at
// or above them; smaller calls take the reference's unmodified Go code.
const (
	// ChainsOffloadMinBytes is the payload of one sendTCPBatch
	// (ChecksumChains): at 64 KiB the engine took 1.57x one core's time,
	// at 128 KiB 0.91x, at 256 KiB 0.57x.
	ChainsOffloadMinBytes = 128 << 10
	// VerifyOffloadMinBytes is the Data bytes of one recvmmsg batch
	// (VerifyPacketBuffers): 64 x 1500 B took 1.31x one core's time,
	// 128 x 1500 B 0.88x, 256 x 1500 B 0.70x.
	VerifyOffloadMinBytes = 128 * 1500
)

// VerifyPacketBuffers runs the receive path's checksum checks over a batch
// of packets as the link layer delivers them (recvMMsgDispatcher,
// link/fdbased/packet_dispatchers.go:258-317: Data holds the IP packet over
// BufConfig views) in one device pass: TCP segment.parse
// (transport/tcp/segment.go:174-180), ICMPv4 echo (network/ipv4/icmp.go:
// 72-80), ICMPv6 (network/ipv6/icmp.go:76-84).  verdict[i] is one of the
// constants above.
func VerifyPacketBuffers(pkts []tcpip.PacketBuffer, verdict []uint8) {
	if len(verdict) < len(pkts) {
		panic("VerifyPacketBuffers: verdict too short")
	}
	packetBuffers(pkts, C.NS_PKB_VERIFY, verdict)
}

// FillPacketBuffers writes the checksums of a batch of outbound packets whose
// Header holds the IP header and the transport header (Data the payload), in
// one device pass: the transport checksum as buildTCPHdr
// (transport/tcp/connect.go:653-663), sendUDP (transport/udp/endpoint.go:
// 808-815), the ICMPv4 echo reply (network/ipv4/icmp.go:96-100) or
// ICMPv6Checksum (icmpv6.go:202-221) compute it, and the IPv4 header
// checksum of addIPHeader (network/ipv4/ipv4.go:236).
func FillPacketBuffers(pkts []tcpip.PacketBuffer) {
	packetBuffers(pkts, C.NS_PKB_FILL, nil)
}

func packetBuffers(pkts []tcpip.PacketBuffer, op C.uint32_t, verdict []uint8) {
	n := len(pkts)
	if n == 0 {
		return
	}
	need := 8
	for i := range pkts {
		need += pkts[i].Header.UsedLength() + pkts[i].Data.Size()
		need += (len(pkts[i].Data.Views()) + 1) * viewEntry
		need += 8
	}
	st := acquireStage(need)
	defer st.release()
	tab := make([]C.ns_pkt_buf, n) // Go memory holding only C pointers
	hdrAt := make([]int, n)
	for i := range pkts {
		hv := pkts[i].Header.View()
		p, at := st.put(hv)
		tab[i].hdr = p
		tab[i].hdr_len = C.uint64_t(len(hv))
		hdrAt[i] = at
		// Data's views, clipped to Data.Size() (the C side clips too)
		vs := pkts[i].Data.Views()
		left := pkts[i].Data.Size()
		type span struct {
			p *C.uint8_t
			l int
		}
		spans := make([]span, 0, len(vs))
		for _, v := range vs {
			if left <= 0 {
				break
			}
			l := len(v)
			if l > left {
				l = left
			}
			q, _ := st.put(v[:l])
			spans = append(spans, span{q, l})
			left -= l
		}
		vp, vt := st.views(len(spans))
		for j, s := range spans {
			vt[j].data = s.p
			vt[j].len = C.uint64_t(s.l)
		}
		tab[i].data = vp
		tab[i].ndata = C.uint32_t(len(spans))
		tab[i].data_size = C.uint64_t(pkts[i].Data.Size() - left)
	}
	var vp *C.uint8_t
	if verdict != nil {
		vp = (*C.uint8_t)(unsafe.Pointer(&verdict[0]))
	}
	csumMust(C.ns_csum_packet_buffers(csumEngine(), &tab[0], C.uint32_t(n), op, nil, vp), "ns_csum_packet_buffers")
	if op == C.NS_PKB_FILL {
		// the checksum fields were written into the staged Header bytes
		for i := range pkts {
			hv := pkts[i].Header.View()
			copy(hv, st.mem[hdrAt[i]:hdrAt[i]+len(hv)])
		}
	}
}
