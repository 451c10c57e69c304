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
// Errors (SURVEY.md §8(b)): the exported batch functions keep no-error
// signatures.  When the engine cannot run a call (no device, an allocation
// or HIP failure, a stale library), the call is computed by the reference's
// own Go code in this package instead — calculateChecksum, Checksum,
// ChecksumVVWithOffset and the header types' CalculateChecksum /
// SetChecksum, in the callers' order — and EngineFallbacks() counts it.  The
// result is the same either way.  The ...Err variants the build-tagged
// callers use report the failure instead, so those callers run their
// default-build path (csum_batch_go.go, csum_rx_go.go).  Only argument misuse
// the reference would also trip over (an out slice too short, a negative
// slice bound) panics.
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
	"reflect"
	"sync"
	"sync/atomic"
	"unsafe"

	"github.com/google/netstack/tcpip"
	"github.com/google/netstack/tcpip/buffer"
)

var (
	csumOnce sync.Once
	csumCtx  *C.ns_csum_ctx
	csumErr  C.int
	csumABI  C.int

	engineFallbacks uint64 // calls computed by the Go code instead (atomic)
	engineLastRC    int32  // the last failing status (atomic)
)

// EngineFallbacks returns how many batch calls the engine could not run and
// the reference's Go code computed instead (see the file comment).
func EngineFallbacks() uint64 {
	return atomic.LoadUint64(&engineFallbacks)
}

// EngineError is an engine call's failure: the operation and its NS_E*
// status (include/netstack_csum.h).
type EngineError struct {
	Op     string
	Status int
}

func (e *EngineError) Error() string {
	return "netstack_csum: " + e.Op + ": " + C.GoString(C.ns_csum_strerror(C.int(e.Status)))
}

// engineFailed counts one call that falls back and returns its error.
func engineFailed(op string, rc C.int) error {
	atomic.AddUint64(&engineFallbacks, 1)
	atomic.StoreInt32(&engineLastRC, int32(rc))
	return &EngineError{Op: op, Status: int(rc)}
}

// csumEngine returns the process-wide engine context for device 0, created
// once.  A library whose C ABI differs from the header this file was
// compiled against (a stale libnetstack_csum.so), or a failed init, is an
// engine failure like any other: every call falls back.
func csumEngine() (*C.ns_csum_ctx, C.int) {
	csumOnce.Do(func() {
		csumABI = C.ns_csum_abi_version()
		if csumABI != C.NS_CSUM_ABI_VERSION {
			csumErr = C.NS_EINVAL
			return
		}
		var opts C.ns_csum_opts
		csumErr = C.ns_csum_init(&opts, &csumCtx)
	})
	if csumErr != C.NS_OK {
		return nil, csumErr
	}
	return csumCtx, C.NS_OK
}

// csumStage is a leased engine staging buffer: pinned host memory the GPU
// reads in place.  mem is the same C memory as a Go slice.
type csumStage struct {
	ctx  *C.ns_csum_ctx
	base *C.uint8_t
	mem  []byte
	used int
}

func acquireStage(ctx *C.ns_csum_ctx, n int) (*csumStage, C.int) {
	if n < 1 {
		n = 1
	}
	s := &csumStage{ctx: ctx}
	if rc := C.ns_csum_stage_acquire(ctx, C.uint64_t(n), &s.base); rc != C.NS_OK {
		return nil, rc
	}
	h := (*reflect.SliceHeader)(unsafe.Pointer(&s.mem))
	h.Data = uintptr(unsafe.Pointer(s.base))
	h.Len = n
	h.Cap = n
	return s, C.NS_OK
}

func (s *csumStage) release() {
	// a stage the engine does not know is a library bug, not a call's
	// failure: the call's results stand
	_ = C.ns_csum_stage_release(s.ctx, s.base)
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
	for _, s := range segs {
		if s.Off < 0 || s.Size < 0 {
			panic("slice bounds out of range") // as v[off:] / v[:l] would in checksum.go
		}
	}
	if len(segs) == 0 || checksumVVBatch(vv, segs, out) == nil {
		return
	}
	for i, s := range segs { // the reference's own function, segment by segment
		out[i] = ChecksumVVWithOffset(vv, s.Initial, s.Off, s.Size)
	}
}

func checksumVVBatch(vv buffer.VectorisedView, segs []SegDesc, out []uint16) error {
	ctx, rc := csumEngine()
	if rc != C.NS_OK {
		return engineFailed("ns_csum_init", rc)
	}
	vs := vv.Views()
	st, rc := acquireStage(ctx, viewBytes(vs))
	if rc != C.NS_OK {
		return engineFailed("ns_csum_stage_acquire", rc)
	}
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
	if rc := C.ns_csum_vv_batch(ctx, tp, C.uint32_t(len(tab)), &cs[0], C.uint32_t(len(cs)),
		(*C.uint16_t)(unsafe.Pointer(&out[0]))); rc != C.NS_OK {
		return engineFailed("ns_csum_vv_batch", rc)
	}
	return nil
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
	if err := ChecksumChainsErr(chains, out); err != nil {
		checksumChainsGo(chains, out)
	}
}

// ChecksumChainsErr is ChecksumChains without the fallback: on an engine
// failure it returns the error (counted in EngineFallbacks) and out is
// undefined; the caller computes the sums its own way.
func ChecksumChainsErr(chains []ChecksumChain, out []uint16) error {
	if len(out) < len(chains) {
		panic("ChecksumChains: out too short")
	}
	if len(chains) == 0 {
		return nil
	}
	ctx, rc := csumEngine()
	if rc != C.NS_OK {
		return engineFailed("ns_csum_init", rc)
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
	st, rc := acquireStage(ctx, bytes)
	if rc != C.NS_OK {
		return engineFailed("ns_csum_stage_acquire", rc)
	}
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
	if rc := C.ns_csum_chains(ctx, &tab[0], C.uint32_t(n), (*C.uint16_t)(unsafe.Pointer(&out[0])),
		C.uint32_t(len(chains))); rc != C.NS_OK {
		return engineFailed("ns_csum_chains", rc)
	}
	return nil
}

// checksumChainsGo is a chain evaluated by the reference's own functions: a
// restart piece is Checksum(buf, xsum) (checksum.go:52-55), a continuing one
// carries the odd byte on, as ChecksumVVWithOffset chains views
// (checksum.go:89); empty continuing pieces are skipped like empty views
// (:73-75).
func checksumChainsGo(chains []ChecksumChain, out []uint16) {
	for i, ch := range chains {
		xsum, odd := ch.Initial, false
		for _, pc := range ch.Pieces {
			if pc.Restart {
				xsum, odd = calculateChecksum(pc.Buf, false, uint32(xsum))
			} else if len(pc.Buf) > 0 {
				xsum, odd = calculateChecksum(pc.Buf, odd, uint32(xsum))
			}
		}
		out[i] = xsum
	}
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
	if len(descs) == 0 || checksumBatch(arena, descs, out, chained) == nil {
		return
	}
	var prev uint16
	for i, d := range descs { // calculateChecksum (checksum.go:26-46) per descriptor
		init := d.Initial
		if chained && d.Flags&2 != 0 {
			init = prev
		}
		b := arena[d.Off : d.Off+uint64(d.Len)] // past the arena: a slice-bound panic, as in Go
		prev, _ = calculateChecksum(b, d.Flags&1 != 0 && len(b) > 0, uint32(init))
		out[i] = prev
	}
}

func checksumBatch(arena []byte, descs []BatchDesc, out []uint16, chained bool) error {
	ctx, rc := csumEngine()
	if rc != C.NS_OK {
		return engineFailed("ns_csum_init", rc)
	}
	var flags C.uint32_t
	if chained {
		flags = C.NS_BATCH_CHAINED
	}
	var ap *C.uint8_t
	if len(arena) > 0 {
		ap = (*C.uint8_t)(unsafe.Pointer(&arena[0]))
	}
	if rc := C.ns_csum_batch_host(ctx, ap, C.uint64_t(len(arena)),
		(*C.ns_pkt_desc)(unsafe.Pointer(&descs[0])), C.uint32_t(len(descs)),
		(*C.uint16_t)(unsafe.Pointer(&out[0])), flags); rc != C.NS_OK {
		return engineFailed("ns_csum_batch_host", rc)
	}
	return nil
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
// (tools/crossover.cc on MI355X, profiles/r05/crossover.json; INTEGRATION.md
// §2 "When offload pays").  The build-tagged callers offload only calls at
// or above them; smaller calls take the reference's unmodified Go code.
// Variables, not constants, so the callers' tests can open the gates and
// run the engine path at the reference's own sizes (set them before any
// traffic; they are read without synchronisation).
var (
	// ChainsOffloadMinBytes is the payload of one sendTCPBatch
	// (ChecksumChains; medians of six runs): at 64 KiB the engine took 1.70x
	// one core's time, at 128 KiB 0.98x, at 256 KiB 0.62x.
	ChainsOffloadMinBytes = 128 << 10
	// VerifyOffloadMinBytes is the Data bytes of one recvmmsg batch
	// (VerifyPacketBuffers): 64 x 1500 B took 1.41x one core's time,
	// 128 x 1500 B 0.98x, 256 x 1500 B 0.74x.
	VerifyOffloadMinBytes = 128 * 1500
	// TxBatchOffloadMinBytes is the payload of all the batches one
	// FillTCPBatches call fills (profiles/r05/crossover.json "tx_host",
	// 64 KiB sendTCPBatch calls, stage copies included): 2 calls took 1.32x
	// one core's time, 4 calls (256 KiB) 0.82x, 64 calls 0.39x.
	TxBatchOffloadMinBytes = 256 << 10
)

// VerifyPacketBuffers runs the receive path's checksum checks over a batch
// of packets as the link layer delivers them (recvMMsgDispatcher,
// link/fdbased/packet_dispatchers.go:258-317: Data holds the IP packet over
// BufConfig views) in one device pass: TCP segment.parse
// (transport/tcp/segment.go:174-180), ICMPv4 echo (network/ipv4/icmp.go:
// 72-80), ICMPv6 (network/ipv6/icmp.go:76-84).  verdict[i] is one of the
// constants above.
func VerifyPacketBuffers(pkts []tcpip.PacketBuffer, verdict []uint8) {
	if err := VerifyPacketBuffersErr(pkts, verdict); err != nil {
		// Nothing verified: the stack's own checks (segment.parse, handleICMP)
		// run on every packet, as the reference's receive path does.
		for i := range pkts {
			verdict[i] = PacketChecksumUnchecked
		}
	}
}

// VerifyPacketBuffersErr is VerifyPacketBuffers without the fallback: on an
// engine failure it returns the error (counted in EngineFallbacks) and
// verdict is undefined.
func VerifyPacketBuffersErr(pkts []tcpip.PacketBuffer, verdict []uint8) error {
	if len(verdict) < len(pkts) {
		panic("VerifyPacketBuffers: verdict too short")
	}
	return packetBuffers(pkts, C.NS_PKB_VERIFY, verdict)
}

// FillPacketBuffers writes the checksums of a batch of outbound packets whose
// Header holds the IP header and the transport header (Data the payload), in
// one device pass: the transport checksum as buildTCPHdr
// (transport/tcp/connect.go:653-663), sendUDP (transport/udp/endpoint.go:
// 808-815), the ICMPv4 echo reply (network/ipv4/icmp.go:96-100) or
// ICMPv6Checksum (icmpv6.go:202-221) compute it, and the IPv4 header
// checksum of addIPHeader (network/ipv4/ipv4.go:236).
func FillPacketBuffers(pkts []tcpip.PacketBuffer) {
	if packetBuffers(pkts, C.NS_PKB_FILL, nil) != nil {
		for i := range pkts {
			fillPacketGo(&pkts[i])
		}
	}
}

// fillPacketGo writes one packet's fields with the reference's own functions,
// in its callers' order (the engine's NS_PKB_FILL rules): the transport
// checksum unless the packet is an IPv4 fragment (writePacketFragments,
// ipv4.go:159-160), then the IPv4 header checksum over the header as encoded.
func fillPacketGo(pkt *tcpip.PacketBuffer) {
	h := pkt.Header.View()
	if len(h) == 0 {
		return
	}
	var src, dst tcpip.Address
	var proto uint8
	var t []byte
	v4 := IPVersion(h) == IPv4Version
	frag := false
	if v4 {
		ip := IPv4(h)
		src, dst, proto, t = ip.SourceAddress(), ip.DestinationAddress(), ip.Protocol(), h[ip.HeaderLength():]
		frag = ip.Flags()&IPv4FlagMoreFragments != 0 || ip.FragmentOffset() != 0
	} else {
		ip := IPv6(h)
		src, dst, proto, t = ip.SourceAddress(), ip.DestinationAddress(), ip.NextHeader(), h[IPv6MinimumSize:]
	}
	length := uint16(len(t) + pkt.Data.Size())
	switch {
	case frag:
	case proto == uint8(TCPProtocolNumber): // buildTCPHdr (connect.go:653-663)
		tcp := TCP(t)
		xsum := PseudoHeaderChecksum(TCPProtocolNumber, src, dst, length)
		xsum = ChecksumVV(pkt.Data, xsum)
		tcp.SetChecksum(^tcp.CalculateChecksum(xsum))
	case proto == uint8(UDPProtocolNumber): // sendUDP (udp/endpoint.go:808-815)
		udp := UDP(t)
		xsum := PseudoHeaderChecksum(UDPProtocolNumber, src, dst, length)
		for _, v := range pkt.Data.Views() {
			xsum = Checksum(v, xsum)
		}
		udp.SetChecksum(^udp.CalculateChecksum(xsum))
	case proto == uint8(ICMPv4ProtocolNumber) && v4: // the echo reply (ipv4/icmp.go:96-100)
		icmp := ICMPv4(t)
		icmp.SetChecksum(0)
		icmp.SetChecksum(^Checksum(icmp, ChecksumVV(pkt.Data, 0)))
	case proto == uint8(ICMPv6ProtocolNumber) && !v4:
		icmp := ICMPv6(t)
		icmp.SetChecksum(ICMPv6Checksum(icmp, src, dst, pkt.Data))
	}
	if v4 { // addIPHeader (ipv4.go:236)
		ip := IPv4(h)
		ip.SetChecksum(^ip.CalculateChecksum())
	}
}

func packetBuffers(pkts []tcpip.PacketBuffer, op C.uint32_t, verdict []uint8) error {
	n := len(pkts)
	if n == 0 {
		return nil
	}
	ctx, rc := csumEngine()
	if rc != C.NS_OK {
		return engineFailed("ns_csum_init", rc)
	}
	need := 8
	for i := range pkts {
		need += pkts[i].Header.UsedLength() + pkts[i].Data.Size()
		need += (len(pkts[i].Data.Views()) + 1) * viewEntry
		need += 8
	}
	st, rc := acquireStage(ctx, need)
	if rc != C.NS_OK {
		return engineFailed("ns_csum_stage_acquire", rc)
	}
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
	if rc := C.ns_csum_packet_buffers(ctx, &tab[0], C.uint32_t(n), op, nil, vp); rc != C.NS_OK {
		return engineFailed("ns_csum_packet_buffers", rc)
	}
	if op == C.NS_PKB_FILL {
		// the checksum fields were written into the staged Header bytes
		for i := range pkts {
			hv := pkts[i].Header.View()
			copy(hv, st.mem[hdrAt[i]:hdrAt[i]+len(hv)])
		}
	}
	return nil
}

// TCPBatch is one sendTCPBatch call's checksum work (connect.go:668-702) in
// the form ns_csum_tcp_tx_host takes it: Slots is the call's
// NewPacketDescriptors buffer (n slots of SlotSize bytes, route.go:181-188),
// each holding the segment's encoded headers — the IPv4 header at IPAt (IPLen
// bytes, IHL*4; 0: none, as before WritePackets or on an IPv6 route) and the
// TCP header at TCPAt (TCPLen = DataOffset) — and Payload is the data view,
// cut into MSS-byte segments (:679-691).  Src and Dst are the route's
// addresses (4 or 16 bytes), Protocol its transport protocol (6), Mode what
// buildTCPHdr does with the TCP field (:652-663).
type TCPBatch struct {
	Slots                      []byte
	SlotSize                   int
	Payload                    buffer.VectorisedView
	MSS                        int
	IPAt, IPLen, TCPAt, TCPLen int
	Src, Dst                   tcpip.Address
	Protocol                   tcpip.TransportProtocolNumber
	Mode                       int
}

// TCPBatch.Mode: the full checksum (buildTCPHdr's default), the
// pseudo-header sum only (gso.NeedsCsum, CHECKSUM_PARTIAL), or nothing
// (CapabilityTXChecksumOffload); the IPv4 field is filled in every mode.
const (
	TxCsumFull    = 0
	TxCsumPartial = 1
	TxCsumOffload = 2
)

// FillTCPBatches writes the checksum fields of every segment of every batch —
// buildTCPHdr's TCP checksum (connect.go:652-663) and addIPHeader's IPv4
// header checksum (ipv4.go:236) — in one engine call, ns_csum_tcp_tx_host:
// the batches' slots and payloads are packed into one engine stage, the fields
// are computed on the device and written into the stage, and each batch's
// slots are copied back.  Many connections' sendTCPBatch calls can go in
// one call; that is the shape the engine pays off for at netstack's 64 KiB
// GSO writes (INTEGRATION.md §2).  Fields are summed as zero, as freshly
// encoded headers hold them.  Below TxBatchOffloadMinBytes of payload in
// all, and whenever the engine cannot run the call (counted in
// EngineFallbacks), the same fields are computed by the reference's Go code
// (fillTCPBatchGo).
func FillTCPBatches(batches []TCPBatch) {
	total := 0
	for i := range batches {
		total += batches[i].Payload.Size()
	}
	// below the measured crossover one core is faster: the reference's code
	if total < TxBatchOffloadMinBytes {
		for i := range batches {
			fillTCPBatchGo(&batches[i])
		}
		return
	}
	if err := FillTCPBatchesErr(batches); err != nil {
		for i := range batches {
			fillTCPBatchGo(&batches[i])
		}
	}
}

// FillTCPBatchesErr is FillTCPBatches without the fallback: on an engine
// failure nothing is written and the error is returned (and counted).
func FillTCPBatchesErr(batches []TCPBatch) error {
	if len(batches) == 0 {
		return nil
	}
	ctx, rc := csumEngine()
	if rc != C.NS_OK {
		return engineFailed("ns_csum_init", rc)
	}
	need := 0
	for i := range batches {
		b := &batches[i]
		need += tcpBatchSegments(b)*b.SlotSize + b.Payload.Size()
	}
	st, rc := acquireStage(ctx, need)
	if rc != C.NS_OK {
		return engineFailed("ns_csum_stage_acquire", rc)
	}
	defer st.release()
	txs := make([]C.ns_tcp_tx, len(batches))
	slotAt := make([]int, len(batches))
	for i := range batches {
		b := &batches[i]
		n := tcpBatchSegments(b)
		_, slotAt[i] = st.put(b.Slots[:n*b.SlotSize])
		payAt := st.used
		for _, v := range b.Payload.Views() {
			st.put(v)
		}
		var flags C.uint32_t
		switch b.Mode {
		case TxCsumPartial:
			flags = C.NS_TX_TCP_PARTIAL
		case TxCsumOffload:
			flags = C.NS_TX_TCP_NONE
		}
		// Checksum(dst, Checksum(src, 0)): PseudoHeaderChecksum's address part
		// (checksum.go:113-114); the kernel adds the protocol and length words
		txs[i] = C.ns_tcp_tx{hdr_off: C.uint64_t(slotAt[i]), pay_off: C.uint64_t(payAt),
			size: C.uint64_t(b.Payload.Size()), mss: C.uint32_t(b.MSS), slot: C.uint32_t(b.SlotSize),
			ip_at: C.uint16_t(b.IPAt), ip_len: C.uint16_t(b.IPLen), tcp_at: C.uint16_t(b.TCPAt),
			tcp_len: C.uint16_t(b.TCPLen), addr_sum: C.uint16_t(Checksum([]byte(b.Dst), Checksum([]byte(b.Src), 0))),
			protocol: C.uint16_t(b.Protocol), flags: flags}
	}
	if rc := C.ns_csum_tcp_tx_host(ctx, st.base, C.uint64_t(st.used), &txs[0], C.uint32_t(len(txs)), nil); rc != C.NS_OK {
		return engineFailed("ns_csum_tcp_tx_host", rc)
	}
	for i := range batches {
		b := &batches[i]
		n := tcpBatchSegments(b) * b.SlotSize
		copy(b.Slots[:n], st.mem[slotAt[i]:slotAt[i]+n])
	}
	return nil
}

// tcpBatchSegments is sendTCPBatch's n = ceil(data.Size() / mss)
// (connect.go:675); 0 for an MSS the engine refuses anyway.
func tcpBatchSegments(b *TCPBatch) int {
	if b.MSS <= 0 {
		return 0
	}
	return (b.Payload.Size() + b.MSS - 1) / b.MSS
}

// fillTCPBatchGo is the reference's own computation of the same fields, in
// its order: per segment, buildTCPHdr's PseudoHeaderChecksum, then
// ChecksumVVWithOffset over the payload and TCP.CalculateChecksum
// (connect.go:652-663), then addIPHeader's IPv4 CalculateChecksum
// (ipv4.go:236).  Both fields are cleared first, as Encode leaves them.
func fillTCPBatchGo(b *TCPBatch) {
	n := tcpBatchSegments(b)
	size, off := b.Payload.Size(), 0
	for i := 0; i < n; i++ {
		slot := b.Slots[i*b.SlotSize:][:b.SlotSize]
		packetSize := b.MSS
		if packetSize > size {
			packetSize = size
		}
		size -= packetSize
		if b.Mode != TxCsumOffload {
			tcp := TCP(slot[b.TCPAt:][:b.TCPLen])
			tcp.SetChecksum(0)
			xsum := PseudoHeaderChecksum(b.Protocol, b.Src, b.Dst, uint16(b.TCPLen+packetSize))
			if b.Mode == TxCsumPartial {
				tcp.SetChecksum(xsum)
			} else {
				xsum = ChecksumVVWithOffset(b.Payload, xsum, off, packetSize)
				tcp.SetChecksum(^tcp.CalculateChecksum(xsum))
			}
		}
		if b.IPLen > 0 {
			ip := IPv4(slot[b.IPAt:][:b.IPLen])
			ip.SetChecksum(0)
			ip.SetChecksum(^ip.CalculateChecksum())
		}
		off += packetSize
	}
}

// RxRing is a receive ring resident in device memory (ns_rx_ring): n slots
// of Stride bytes from the arena's RingOff, the frame at FrameAt of a slot,
// LinkHdr 0 (TUN) or 14 (Ethernet), FirstView the link's first buffer view
// (BufConfig[0], packet_dispatchers.go:30; 0: one view).
type RxRing struct {
	RingOff, Stride  uint64
	N                uint32
	FrameAt, LinkHdr uint16
	FirstView        uint32
}

// VerifyRingDevice verifies a ring of received frames that a GPU-attached
// receive path left in device memory (ns_csum_rx_ring): every slot's verdict
// (the constants above) and its two sums go to device memory, asynchronously
// on stream (a hipStream_t, 0 = the null stream).  arena, lens, sums (or 0)
// and verdict (or 0) are device addresses.  There is nothing to fall back to
// on the host for bytes that live on the device: the error is returned
// (and counted in EngineFallbacks), and the caller delivers the frames
// unverified (RXChecksumUnknown), as the default build does.
func VerifyRingDevice(arena uintptr, arenaBytes uint64, r RxRing, lens, sums, verdict, stream uintptr) error {
	ctx, rc := csumEngine()
	if rc != C.NS_OK {
		return engineFailed("ns_csum_init", rc)
	}
	cr := C.ns_rx_ring{ring_off: C.uint64_t(r.RingOff), stride: C.uint64_t(r.Stride), n: C.uint32_t(r.N),
		frame_at: C.uint16_t(r.FrameAt), link_hdr: C.uint16_t(r.LinkHdr), first_view: C.uint32_t(r.FirstView)}
	if rc := C.ns_csum_rx_ring(ctx, (*C.uint8_t)(unsafe.Pointer(arena)), C.uint64_t(arenaBytes), &cr,
		(*C.uint32_t)(unsafe.Pointer(lens)), (*C.uint16_t)(unsafe.Pointer(sums)),
		(*C.uint8_t)(unsafe.Pointer(verdict)), unsafe.Pointer(stream)); rc != C.NS_OK {
		return engineFailed("ns_csum_rx_ring", rc)
	}
	return nil
}

// VerifyBufsDevice is VerifyRingDevice over buffers at per-packet offsets
// of one device arena (a GPU-attached NIC's buffer pool; ns_csum_rx_bufs):
// packet k's frame is in the buffer at arena + r.RingOff + offs[k], of
// r.Stride bytes (the buffers' capacity).  offs, lens, sums (or 0) and
// verdict (or 0) are device addresses.  Errors as for VerifyRingDevice.
func VerifyBufsDevice(arena uintptr, arenaBytes uint64, r RxRing, offs, lens, sums, verdict, stream uintptr) error {
	ctx, rc := csumEngine()
	if rc != C.NS_OK {
		return engineFailed("ns_csum_init", rc)
	}
	cr := C.ns_rx_ring{ring_off: C.uint64_t(r.RingOff), stride: C.uint64_t(r.Stride), n: C.uint32_t(r.N),
		frame_at: C.uint16_t(r.FrameAt), link_hdr: C.uint16_t(r.LinkHdr), first_view: C.uint32_t(r.FirstView)}
	if rc := C.ns_csum_rx_bufs(ctx, (*C.uint8_t)(unsafe.Pointer(arena)), C.uint64_t(arenaBytes), &cr,
		(*C.uint32_t)(unsafe.Pointer(offs)), (*C.uint32_t)(unsafe.Pointer(lens)), (*C.uint16_t)(unsafe.Pointer(sums)),
		(*C.uint8_t)(unsafe.Pointer(verdict)), unsafe.Pointer(stream)); rc != C.NS_OK {
		return engineFailed("ns_csum_rx_bufs", rc)
	}
	return nil
}

// VerifyRingHost is VerifyRingDevice for a ring in host memory: arena holds
// r.N slots of r.Stride bytes from r.RingOff (recvmmsg's buffers laid out
// at a fixed stride), lens their received lengths; verdict (or nil) and sums
// (or nil, 2 per slot) receive the results (ns_csum_rx_ring_host).  The parse
// runs on the device: no per-packet host planning, unlike
// VerifyPacketBuffers.  On an error (counted in EngineFallbacks) the outputs
// are not to be used: the caller delivers the frames unverified
// (RXChecksumUnknown), as the default build does.
func VerifyRingHost(arena []byte, r RxRing, lens []uint32, sums []uint16, verdict []uint8) error {
	n := int(r.N)
	if len(lens) < n || (sums != nil && len(sums) < 2*n) || (verdict != nil && len(verdict) < n) {
		panic("netstack_csum: VerifyRingHost: lens, sums or verdict too short")
	}
	if n == 0 {
		return nil
	}
	ctx, rc := csumEngine()
	if rc != C.NS_OK {
		return engineFailed("ns_csum_init", rc)
	}
	cr := C.ns_rx_ring{ring_off: C.uint64_t(r.RingOff), stride: C.uint64_t(r.Stride), n: C.uint32_t(r.N),
		frame_at: C.uint16_t(r.FrameAt), link_hdr: C.uint16_t(r.LinkHdr), first_view: C.uint32_t(r.FirstView)}
	var ap *C.uint8_t
	if len(arena) > 0 {
		ap = (*C.uint8_t)(unsafe.Pointer(&arena[0]))
	}
	var sp *C.uint16_t
	if sums != nil {
		sp = (*C.uint16_t)(unsafe.Pointer(&sums[0]))
	}
	var vp *C.uint8_t
	if verdict != nil {
		vp = (*C.uint8_t)(unsafe.Pointer(&verdict[0]))
	}
	if rc := C.ns_csum_rx_ring_host(ctx, ap, C.uint64_t(len(arena)), &cr, (*C.uint32_t)(unsafe.Pointer(&lens[0])),
		sp, vp); rc != C.NS_OK {
		return engineFailed("ns_csum_rx_ring_host", rc)
	}
	return nil
}
