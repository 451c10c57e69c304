// Copyright 2026 netstack-csum-mi355x authors.
//
// The default build's side of csum_rx_hip.go: the link verifies nothing,
// every PacketBuffer.RXChecksum stays RXChecksumUnknown, and segment.parse
// verifies each segment as the reference does (segment.go:174-180).

// +build linux,!hipcsum

package fdbased

import "github.com/google/netstack/tcpip"

func verifyRXChecksums(e *endpoint, pkts []tcpip.PacketBuffer) {}
