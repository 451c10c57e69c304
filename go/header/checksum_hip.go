// Copyright 2026 netstack-csum-mi355x authors.
//
// cgo shim: google/netstack's tcpip/header checksum entry points, same Go
// signatures (tcpip/header/checksum.go:52-122), computed by the MI355X (gfx950)
// engine behind include/netstack_csum.h.  Built only with `-tags hipcsum`;
// without the tag the reference's pure-Go checksum.go is used unchanged.
//
// This file is written for the reference tree (it replaces checksum.go in
// package header when the tag is set; checksum.go gets `// +build !hipcsum`).
// It cannot be compiled in the build container (no Go toolchain); see
// INTEGRATION.md.

// +build hipcsum

package header

/*
#cgo CFLAGS: -I${SRCDIR}/../../include
#cgo LDFLAGS: -L${SRCDIR}/../../netstack_amd/lib -lnetstack_csum -Wl,-rpath,${SRCDIR}/../../netstack_amd/lib
#include <stdlib.h>
#include "netstack_csum.h"
*/
import "C"

import (
	"encoding/binary"
	"fmt"
	"runtime"
	"sync"
	"unsafe"

	"github.com/google/netstack/tcpip"
	"github.com/google/netstack/tcpip/buffer"
)

var (
	ctxOnce sync.Once
	ctx     *C.ns_csum_ctx
	ctxErr  C.int
)

// engine returns the process-wide context for device 0 (created once).
func engine() *C.ns_csum_ctx {
	ctxOnce.Do(func() {
		var opts C.ns_csum_opts
		opts.device = 0
		ctxErr = C.ns_csum_init(&opts, &ctx)
	})
	if ctxErr != C.NS_OK {
		// No fallback: the reference signatures have no error return, so a
		// missing GPU is fatal exactly like a Go slice-bound panic.
		panic(fmt.Sprintf("netstack_csum: ns_csum_init: %s", C.GoString(C.ns_csum_strerror(ctxErr))))
	}
	return ctx
}

func must(rc C.int, what string) {
	if rc != C.NS_OK {
		panic(fmt.Sprintf("netstack_csum: %s: %s", what, C.GoString(C.ns_csum_strerror(rc))))
	}
}

func bytePtr(b []byte) *C.uint8_t {
	if len(b) == 0 {
		return nil
	}
	return (*C.uint8_t)(unsafe.Pointer(&b[0]))
}

// cViews copies the view headers into C memory (cgo forbids passing Go memory
// that holds Go pointers); the bytes themselves are borrowed for the call and
// pinned while their addresses sit in C memory (runtime.Pinner, Go 1.21+).
func cViews(views []buffer.View) (*C.ns_view, func()) {
	n := len(views)
	if n == 0 {
		return nil, func() {}
	}
	var pin runtime.Pinner
	p := (*C.ns_view)(C.malloc(C.size_t(n) * C.size_t(unsafe.Sizeof(C.ns_view{}))))
	arr := (*[1 << 28]C.ns_view)(unsafe.Pointer(p))[:n:n]
	for i, v := range views {
		if len(v) > 0 {
			pin.Pin(&v[0])
		}
		arr[i].data = bytePtr(v)
		arr[i].len = C.uint64_t(len(v))
	}
	return p, func() { pin.Unpin(); C.free(unsafe.Pointer(p)) }
}

// Checksum calculates the checksum (as defined in RFC 1071) of the bytes in the
// given byte array.  checksum.go:52-55.
func Checksum(buf []byte, initial uint16) uint16 {
	var out C.uint16_t
	must(C.ns_csum_checksum(engine(), bytePtr(buf), C.uint64_t(len(buf)), C.uint16_t(initial), &out), "Checksum")
	return uint16(out)
}

// ChecksumVV calculates the checksum of the bytes in the given
// VectorizedView.  checksum.go:61-63.
func ChecksumVV(vv buffer.VectorisedView, initial uint16) uint16 {
	return ChecksumVVWithOffset(vv, initial, 0, vv.Size())
}

// ChecksumVVWithOffset calculates the checksum of bytes [off, off+size) of the
// given VectorizedView.  checksum.go:69-98.
func ChecksumVVWithOffset(vv buffer.VectorisedView, initial uint16, off int, size int) uint16 {
	if off < 0 || size < 0 {
		panic("slice bounds out of range") // as v[off:] / v[:l] would in checksum.go
	}
	views, free := cViews(vv.Views())
	defer free()
	var out C.uint16_t
	must(C.ns_csum_vv_with_offset(engine(), views, C.uint32_t(len(vv.Views())), C.uint16_t(initial),
		C.int64_t(off), C.int64_t(size), &out), "ChecksumVVWithOffset")
	return uint16(out)
}

// ChecksumCombine combines the two uint16 to form their checksum.
// checksum.go:104-107.
func ChecksumCombine(a, b uint16) uint16 {
	return uint16(C.ns_csum_combine(C.uint16_t(a), C.uint16_t(b)))
}

// PseudoHeaderChecksum calculates the pseudo-header checksum.
// checksum.go:112-122.
func PseudoHeaderChecksum(protocol tcpip.TransportProtocolNumber, srcAddr tcpip.Address, dstAddr tcpip.Address, totalLen uint16) uint16 {
	src, dst := []byte(srcAddr), []byte(dstAddr)
	var out C.uint16_t
	must(C.ns_csum_pseudo_header(engine(), C.uint32_t(protocol), bytePtr(src), C.uint32_t(len(src)),
		bytePtr(dst), C.uint32_t(len(dst)), C.uint16_t(totalLen), &out), "PseudoHeaderChecksum")
	return uint16(out)
}

// SegDesc is one segment of a batched payload checksum: the Off/Size of a
// stack.PacketDescriptor (stack/route.go:174-178) and its pseudo-header sum.
type SegDesc struct {
	Off, Size int
	Initial   uint16
}

// ChecksumVVBatch computes out[i] = ChecksumVVWithOffset(vv, segs[i].Initial,
// segs[i].Off, segs[i].Size) for every segment in one device pass — the n
// per-MSS calls of sendTCPBatch (transport/tcp/connect.go:668-702).
func ChecksumVVBatch(vv buffer.VectorisedView, segs []SegDesc, out []uint16) {
	if len(out) < len(segs) {
		panic("ChecksumVVBatch: out too short")
	}
	if len(segs) == 0 {
		return
	}
	views, free := cViews(vv.Views())
	defer free()
	cs := (*C.ns_seg)(C.malloc(C.size_t(len(segs)) * C.size_t(unsafe.Sizeof(C.ns_seg{}))))
	defer C.free(unsafe.Pointer(cs))
	arr := (*[1 << 28]C.ns_seg)(unsafe.Pointer(cs))[:len(segs):len(segs)]
	for i, s := range segs {
		arr[i].off = C.int64_t(s.Off)
		arr[i].size = C.int64_t(s.Size)
		arr[i].initial = C.uint16_t(s.Initial)
	}
	must(C.ns_csum_vv_batch(engine(), views, C.uint32_t(len(vv.Views())), cs, C.uint32_t(len(segs)),
		(*C.uint16_t)(unsafe.Pointer(&out[0]))), "ChecksumVVBatch")
}

// ChecksumViews is the per-view-restart loop of sendUDP
// (transport/udp/endpoint.go:811-813): xsum = Checksum(v, xsum) per view.
func ChecksumViews(views []buffer.View, initial uint16) uint16 {
	cv, free := cViews(views)
	defer free()
	var out C.uint16_t
	must(C.ns_csum_views_restart(engine(), cv, C.uint32_t(len(views)), C.uint16_t(initial), &out), "ChecksumViews")
	return uint16(out)
}

// ChecksumPiece is one buffer of a checksum chain.  Restart = a fresh
// Checksum(Buf, xsum) call (alignment restarts, checksum.go:52-55); otherwise
// the piece continues the previous one's byte stream with its odd-byte carry
// (ChecksumVVWithOffset's view chaining, checksum.go:89).
type ChecksumPiece struct {
	Buf     []byte
	Restart bool
}

// ChecksumChain is `xsum := Initial; for p := range Pieces { ... }`.
type ChecksumChain struct {
	Initial uint16
	Pieces  []ChecksumPiece
}

// ChecksumChains evaluates every chain in one device pass (ns_csum_chains);
// out[i] is chain i's un-complemented sum.  One chain can hold a whole TCP
// segment checksum — pseudo-header fields, payload views, the TCP header —
// so sendTCPBatch (connect.go:668-702) and a recvmmsg batch of
// segment.parse checks (segment.go:174-180) each take one call.
func ChecksumChains(chains []ChecksumChain, out []uint16) {
	if len(out) < len(chains) {
		panic("ChecksumChains: out too short")
	}
	if len(chains) == 0 {
		return
	}
	n := 0
	for _, ch := range chains {
		if len(ch.Pieces) == 0 {
			n++
		}
		n += len(ch.Pieces)
	}
	var pin runtime.Pinner
	defer pin.Unpin()
	cp := (*C.ns_piece)(C.malloc(C.size_t(n) * C.size_t(unsafe.Sizeof(C.ns_piece{}))))
	defer C.free(unsafe.Pointer(cp))
	arr := (*[1 << 28]C.ns_piece)(unsafe.Pointer(cp))[:n:n]
	k := 0
	for _, ch := range chains {
		pieces := ch.Pieces
		if len(pieces) == 0 {
			pieces = []ChecksumPiece{{Restart: true}}
		}
		for j, pc := range pieces {
			if len(pc.Buf) > 0 {
				pin.Pin(&pc.Buf[0])
			}
			arr[k] = C.ns_piece{data: bytePtr(pc.Buf), len: C.uint64_t(len(pc.Buf))}
			if j == 0 {
				arr[k].initial = C.uint16_t(ch.Initial)
			}
			if pc.Restart {
				arr[k].flags |= C.NS_PIECE_RESTART
			}
			if j == len(pieces)-1 {
				arr[k].flags |= C.NS_PIECE_END
			}
			k++
		}
	}
	must(C.ns_csum_chains(engine(), cp, C.uint32_t(n), (*C.uint16_t)(unsafe.Pointer(&out[0])),
		C.uint32_t(len(chains))), "ChecksumChains")
}

var _ = binary.BigEndian // keep the reference file's import set
