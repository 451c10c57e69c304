"""Synthetic packet batches for the BASELINE.json configurations.

Bytes come from splitmix64 (state_i = seed + (i+1)*0x9E3779B97F4A7C15, output
little-endian), generated either with numpy on the host or with torch int64
arithmetic directly in HBM — both produce the same bytes, so a device-generated
arena can be checked against the host oracle on the same inputs.

Layouts (BASELINE.md "CPU-baseline and measurement plan"):
  cfg1  one 65,536-B buffer, seed 1, initial 0 (host only)
  cfg2  1,048,576 x 1500 B, seed 2, 16-B-aligned starts (stride 1504)
  cfg3  1,048,576 x 64 B, seed 3 (stride 64)
  cfg4  1,048,576 packets, L = 64 + r, P(r) ~ (r+1)^-1.1, r in [0, 8936], seed 4
  cfg5  8,388,608 x 1500 B, seed 5 (sharded over GPUs)
Per-packet `initial` is a random uint16 (a stand-in for the pseudo-header sum)
drawn from an independent splitmix64 stream.  Padding bytes between packets
are random too, so a kernel that sums them fails parity.
"""
from __future__ import annotations

from dataclasses import dataclass

import numpy as np

GAMMA = 0x9E3779B97F4A7C15
M1 = 0xBF58476D1CE4E5B9
M2 = 0x94D049BB133111EB
MASK64 = (1 << 64) - 1

DESC_DTYPE = np.dtype(
    [("off", "<u8"), ("len", "<u4"), ("initial", "<u2"), ("flags", "<u2")], align=False)


def splitmix64(seed: int, n: int, start: int = 0) -> np.ndarray:
    """n outputs of splitmix64 starting at index `start` (numpy, host)."""
    i = np.arange(start + 1, start + n + 1, dtype=np.uint64)
    with np.errstate(over="ignore"):
        z = i * np.uint64(GAMMA) + np.uint64(seed & MASK64)
        z = (z ^ (z >> np.uint64(30))) * np.uint64(M1)
        z = (z ^ (z >> np.uint64(27))) * np.uint64(M2)
        z = z ^ (z >> np.uint64(31))
    return z


def random_bytes(seed: int, nbytes: int, chunk: int = 1 << 24, start_word: int = 0) -> np.ndarray:
    """nbytes of splitmix64 output (host) from word `start_word` on, generated
    in chunks of `chunk` words."""
    words = (nbytes + 7) // 8
    out = np.empty(words * 8, dtype=np.uint8)
    o64 = out.view(np.uint64)
    for s in range(0, words, chunk):
        e = min(words, s + chunk)
        o64[s:e] = splitmix64(seed, e - s, start_word + s)
    return out[:nbytes]


def _s64(x: int) -> int:
    x &= MASK64
    return x - (1 << 64) if x >> 63 else x


def random_bytes_torch(seed: int, nbytes: int, device, chunk: int = 1 << 26, start_word: int = 0):
    """Same bytes as random_bytes(), generated in HBM with torch int64 ops
    (two's-complement wrap; logical shifts emulated with masks)."""
    import torch

    words = (nbytes + 7) // 8
    out = torch.empty(words * 8, dtype=torch.uint8, device=device)
    o64 = out.view(torch.int64)
    g, m1, m2, sd = _s64(GAMMA), _s64(M1), _s64(M2), _s64(seed)

    def lsr(z, k):
        return (z >> k) & ((1 << (64 - k)) - 1)

    for s in range(0, words, chunk):
        e = min(words, s + chunk)
        z = torch.arange(start_word + s + 1, start_word + e + 1, dtype=torch.int64, device=device)
        z = z * g + sd
        z = (z ^ lsr(z, 30)) * m1
        z = (z ^ lsr(z, 27)) * m2
        o64[s:e] = z ^ lsr(z, 31)
    return out[:nbytes]


def zipf_lengths(seed: int, n: int, lo: int = 64, hi: int = 9000, alpha: float = 1.1) -> np.ndarray:
    """L = lo + r, r in [0, hi-lo], P(r) ~ (r+1)^-alpha, by inverse CDF."""
    r = np.arange(hi - lo + 1, dtype=np.float64)
    w = (r + 1.0) ** (-alpha)
    cdf = np.cumsum(w)
    cdf /= cdf[-1]
    u = (splitmix64(seed ^ 0x5A5A5A5A, n) >> np.uint64(11)).astype(np.float64) * (1.0 / (1 << 53))
    idx = np.searchsorted(cdf, u, side="right")
    idx = np.minimum(idx, len(cdf) - 1)
    return (lo + idx).astype(np.uint32)


@dataclass
class Batch:
    """A packet batch: descriptor table + how to make its arena."""

    name: str
    seed: int
    desc: np.ndarray  # DESC_DTYPE
    arena_bytes: int
    base: int = 0  # byte offset of this arena in the seed's byte stream (multiple of 8)

    @property
    def n(self) -> int:
        return len(self.desc)

    @property
    def payload_bytes(self) -> int:
        return int(self.desc["len"].sum(dtype=np.uint64))

    @property
    def algorithmic_bytes(self) -> int:
        """Σlen + 18·N: payload read + 16-B descriptor read + 2-B result
        write."""
        return self.payload_bytes + 18 * self.n

    def arena_host(self) -> np.ndarray:
        return random_bytes(self.seed, self.arena_bytes, start_word=self.base // 8)

    def arena_device(self, device):
        return random_bytes_torch(self.seed, self.arena_bytes, device, start_word=self.base // 8)

    def host_bytes(self, lo: int, hi: int) -> np.ndarray:
        """Arena bytes [lo, hi) on the host, without generating the rest."""
        w0 = (self.base + lo) // 8
        skip = (self.base + lo) - 8 * w0
        return random_bytes(self.seed, hi - lo + skip, start_word=w0)[skip:]

    def shard(self, part: int, parts: int) -> "Batch":
        """Packets [part*n/parts, (part+1)*n/parts) as a batch of their own
        (contiguous packet ranges, offsets rebased, no
        collective).  The shard's arena is the same bytes as the whole
        batch's arena over its range, so results equal the unsharded ones."""
        n = self.n
        a, b = part * n // parts, (part + 1) * n // parts
        d = self.desc[a:b].copy()
        if len(d) == 0:
            return Batch(f"{self.name}_s{part}of{parts}", self.seed, d, 0, self.base)
        lo = (int(d["off"][0]) // 16) * 16
        hi = int((d["off"] + d["len"].astype(np.uint64)).max())
        d["off"] -= np.uint64(lo)
        return Batch(f"{self.name}_s{part}of{parts}", self.seed, d, ((hi - lo + 15) // 16) * 16,
                     self.base + lo)


def make_desc(lengths: np.ndarray, initial: np.ndarray, align: int = 16, base: int = 0,
              flags: np.ndarray | None = None) -> tuple[np.ndarray, int]:
    """Pack packets back to back with starts aligned to `align` bytes."""
    n = len(lengths)
    lengths = lengths.astype(np.uint64)
    stride = ((lengths + np.uint64(align - 1)) // np.uint64(align)) * np.uint64(align) if align > 1 else lengths
    off = np.zeros(n, dtype=np.uint64)
    if n:
        off[1:] = np.cumsum(stride[:-1], dtype=np.uint64)
    off += np.uint64(base)
    d = np.zeros(n, dtype=DESC_DTYPE)
    d["off"] = off
    d["len"] = lengths.astype(np.uint32)
    d["initial"] = initial.astype(np.uint16)
    if flags is not None:
        d["flags"] = flags.astype(np.uint16)
    end = int(off[-1] + lengths[-1]) if n else base
    return d, end


def _initials(seed: int, n: int) -> np.ndarray:
    return (splitmix64(seed ^ 0x1D1D1D1D, n) >> np.uint64(48)).astype(np.uint16)


def uniform(name: str, seed: int, n: int, length: int, align: int = 16) -> Batch:
    lengths = np.full(n, length, dtype=np.uint32)
    d, end = make_desc(lengths, _initials(seed, n), align)
    return Batch(name, seed, d, ((end + 15) // 16) * 16)


def zipf(name: str, seed: int, n: int, align: int = 16) -> Batch:
    lengths = zipf_lengths(seed, n)
    d, end = make_desc(lengths, _initials(seed, n), align)
    return Batch(name, seed, d, ((end + 15) // 16) * 16)


def config(k: int, n: int | None = None) -> Batch:
    """BASELINE.json configs[k-1] (k = 1..5; 6 = bulk 64 KiB GSO buffers, not
    a BASELINE config); `n` overrides the packet count
    (for parity-test subsets with the same layout rule)."""
    if k == 1:
        b = uniform("cfg1_64KiB", 1, 1, 65536)
        b.desc["initial"] = 0
        return b
    if k == 2:
        return uniform("cfg2_1Mx1500", 2, n or (1 << 20), 1500)
    if k == 3:
        return uniform("cfg3_1Mx64", 3, n or (1 << 20), 64)
    if k == 4:
        return zipf("cfg4_1Mzipf", 4, n or (1 << 20))
    if k == 5:
        return uniform("cfg5_8Mx1500", 5, n or (8 << 20), 1500)
    if k == 6:
        # Not a BASELINE config: 64 KiB GSO payloads (sendTCPBatch's largest
        # write, connect.go:668-702) in bulk — the large-packet tile sizing case.
        return uniform("gso_16Kx64KiB", 6, n or (16 << 10), 65536)
    raise ValueError(k)


# ---------------------------------------------------------------------------
# Received IPv4/TCP packets for device-resident RX verification (SURVEY.md
# §8(f) rank 2: segment.parse's csumValid, transport/tcp/segment.go:166-181,
# and the IPv4 header check of ipv4.go's IsValid/checker.go:51-53).
# ---------------------------------------------------------------------------
RX_PKT = 1500      # IPv4 total length
RX_STRIDE = 1504   # 16-B-aligned packet starts
RX_IHL = 20
RX_TCP = RX_PKT - RX_IHL  # TCP header + payload bytes (1480)


def _fold_np(s):
    s = (s & 0xFFFF) + (s >> 16)
    return (s & 0xFFFF) + (s >> 16)


def _tcp_packets(n: int, seed: int, device):
    """n 1500-B IPv4/TCP packets at RX_STRIDE (splitmix64 bytes with fixed
    header fields), both checksum fields zero.  Returns (arena, packet view)."""
    arena = random_bytes_torch(seed, n * RX_STRIDE, device)
    p = arena.view(n, RX_STRIDE)[:, :RX_PKT]
    p[:, 0] = 0x45
    p[:, 1] = 0
    p[:, 2] = RX_PKT >> 8
    p[:, 3] = RX_PKT & 0xFF
    p[:, 6] = 0x40
    p[:, 7] = 0
    p[:, 8] = 64
    p[:, 9] = 6
    p[:, 10:12] = 0
    p[:, 32] = 0x50  # data offset 5 words
    p[:, 33] = 0x18  # PSH | ACK
    p[:, 36:40] = 0  # checksum, urgent pointer
    return arena, p


def _tcp_desc(n: int, fused: bool = True) -> np.ndarray:
    """The descriptor table over _tcp_packets (see rx_batch); per packet:

    fused (2 independent descriptors):
      2i    IPv4 header [0, 20), initial 0                  -> must sum to 0xffff
      2i+1  [12, 1500): the pseudo-header addresses (in place in the packet)
            followed directly by the TCP header and payload, initial =
            ChecksumCombine(1480, 6), the length and protocol words
    chained (3 descriptors, the second and third one NS_DESC_CONT run):
      3i    IPv4 header [0, 20)
      3i+1  src+dst addresses [12, 20), initial = ChecksumCombine(1480, 6)
      3i+2  TCP header + payload [20, 1500), NS_DESC_CONT

    Both compute segment.parse's xsum (segment.go:174-180): PseudoHeaderChecksum
    then Checksum(h[:offset]) then ChecksumVV(payload) are restarts at even
    offsets over contiguous bytes, and without a uint32 wrap (< 128 KiB) the
    sum of the concatenation folds to the same value as the chain of folds
    (both are fold1 of the same total, 0 only if every piece is
    0).  The fused table needs no run folding."""
    base = np.arange(n, dtype=np.uint64) * np.uint64(RX_STRIDE)
    if fused:
        d = np.zeros(2 * n, dtype=DESC_DTYPE)
        d["off"][0::2] = base
        d["len"][0::2] = RX_IHL
        d["off"][1::2] = base + np.uint64(12)
        d["len"][1::2] = RX_PKT - 12
        d["initial"][1::2] = RX_TCP + 6  # ChecksumCombine(1480, 6): no carry
        return d
    d = np.zeros(3 * n, dtype=DESC_DTYPE)
    d["off"][0::3] = base
    d["len"][0::3] = RX_IHL
    d["off"][1::3] = base + np.uint64(12)
    d["len"][1::3] = 8
    d["initial"][1::3] = RX_TCP + 6  # ChecksumCombine(1480, 6): no carry
    d["off"][2::3] = base + np.uint64(RX_IHL)
    d["len"][2::3] = RX_TCP
    d["flags"][2::3] = 2  # NS_DESC_CONT
    return d


def per_packet(fused: bool) -> int:
    """Descriptors per packet of _tcp_desc: the IPv4 header result is
    out[0::k], the TCP result out[k-1::k]."""
    return 2 if fused else 3


def rx_batch(n: int, seed: int, device, corrupt_every: int = 0, fused: bool = True):
    """n received 1500-B IPv4/TCP packets packed at RX_STRIDE in HBM, with
    valid IPv4 and TCP checksums (RFC 1071, computed here with torch integer
    ops as plain data generation), and the descriptor table that verifies
    them (_tcp_desc: the IPv4 header must sum to 0xffff, and so must the TCP
    segment with its pseudo-header — PseudoHeaderChecksum, checksum.go:
    112-122: the length and protocol words are host-known, the addresses are
    in the packet).
    With corrupt_every = k > 0, one payload byte of every k-th packet is
    flipped after its checksum was written (tcp_test.go:3246-3254): exactly
    those TCP sums fail.  Returns (arena uint8 tensor, desc, bad indices)."""
    import torch

    arena, p = _tcp_packets(n, seed, device)

    def be_sum(lo, hi):
        w = p[:, lo:hi].to(torch.int64)
        return (w[:, 0::2] * 256 + w[:, 1::2]).sum(dim=1)

    ip = (~_fold_np(be_sum(0, RX_IHL))) & 0xFFFF
    p[:, 10] = (ip >> 8).to(torch.uint8)
    p[:, 11] = (ip & 0xFF).to(torch.uint8)
    tcp = (~_fold_np(be_sum(RX_IHL, RX_PKT) + be_sum(12, 20) + RX_TCP + 6)) & 0xFFFF
    p[:, 36] = (tcp >> 8).to(torch.uint8)
    p[:, 37] = (tcp & 0xFF).to(torch.uint8)
    bad = np.arange(0, n, corrupt_every, dtype=np.int64) if corrupt_every > 0 else np.zeros(0, np.int64)
    if bad.size:
        idx = torch.from_numpy(bad).to(device)
        p[idx, 100] ^= 0x5A
    return arena, _tcp_desc(n, fused), bad


def rx_ring_batch(n: int, seed: int, device, corrupt_every: int = 0):
    """rx_batch's packets as a receive ring (ns_csum_rx_ring): the same n
    valid 1500-B IPv4/TCP packets, one per RX_STRIDE slot, and the n received
    lengths (int32 CUDA tensor) in place of a descriptor table; with
    corrupt_every = k > 0 one payload byte of every k-th packet is flipped.
    Returns (arena, lens, bad indices)."""
    import torch

    arena, _, bad = rx_batch(n, seed, device, corrupt_every)
    lens = torch.full((n,), RX_PKT, dtype=torch.int32, device=device)
    return arena, lens, bad


def rx_ring_batch_v6(n: int, seed: int, device, corrupt_every: int = 0):
    """rx_ring_batch over IPv6: n 1500-B IPv6/TCP packets (a 40-B header,
    PayloadLength 1460, NextHeader 6, random addresses) with valid TCP
    checksums, one per RX_STRIDE slot; with corrupt_every = k > 0 one payload
    byte of every k-th packet is flipped.  Returns (arena, lens, bad)."""
    arena, lens, bad, _ = rx_ring_batch_sized(n, RX_PKT, seed, device, v6=True, corrupt_every=corrupt_every,
                                              stride=RX_STRIDE)
    return arena, lens, bad


def rx_ring_batch_sized(n: int, frame: int, seed: int, device, v6: bool = False, corrupt_every: int = 0,
                        eth: bool = False, stride: int = 0):
    """rx_ring_batch / rx_ring_batch_v6 at any frame length (IPv4 or IPv6
    TCP packets of `frame` bytes, e.g. 9000-B jumbo frames), one per slot of
    `stride` bytes (0: round_up(frame [+ 14], 16) + 16); eth: each packet
    behind a 14-B Ethernet header (EtherType 0x0800 / 0x86DD; ring link_hdr
    14, lengths frame + 14).  Returns (arena, lens, bad, stride)."""
    import torch

    lh = 14 if eth else 0
    stride = stride or (frame + lh + 15) // 16 * 16 + 16
    arena = random_bytes_torch(seed, n * stride, device)
    if eth:
        e = arena.view(n, stride)[:, :14]
        e[:, 12] = 0x86 if v6 else 0x08
        e[:, 13] = 0xDD if v6 else 0x00
    p = arena.view(n, stride)[:, lh:lh + frame]
    ipl = 40 if v6 else RX_IHL
    tl = frame - ipl
    if v6:
        p[:, 0] = 0x60
        p[:, 1:4] = 0
        p[:, 4] = tl >> 8
        p[:, 5] = tl & 0xFF
        p[:, 6] = 6
        p[:, 7] = 64
    else:
        p[:, 0] = 0x45
        p[:, 1] = 0
        p[:, 2] = frame >> 8
        p[:, 3] = frame & 0xFF
        p[:, 6] = 0x40
        p[:, 7] = 0
        p[:, 8] = 64
        p[:, 9] = 6
        p[:, 10:12] = 0
    p[:, ipl + 12] = 0x50
    p[:, ipl + 13] = 0x18
    p[:, ipl + 16:ipl + 20] = 0

    def be_sum(lo, hi):
        w = p[:, lo:hi].to(torch.int64)
        return (w[:, 0::2] * 256 + w[:, 1::2]).sum(dim=1)

    if not v6:
        ip = (~_fold_np(be_sum(0, RX_IHL))) & 0xFFFF
        p[:, 10] = (ip >> 8).to(torch.uint8)
        p[:, 11] = (ip & 0xFF).to(torch.uint8)
    addr = be_sum(8, 40) if v6 else be_sum(12, 20)
    tcp = (~_fold_np(_fold_np(be_sum(ipl, frame) + addr + tl + 6))) & 0xFFFF
    p[:, ipl + 16] = (tcp >> 8).to(torch.uint8)
    p[:, ipl + 17] = (tcp & 0xFF).to(torch.uint8)
    bad = np.arange(0, n, corrupt_every, dtype=np.int64) if corrupt_every > 0 else np.zeros(0, np.int64)
    if bad.size:
        idx = torch.from_numpy(bad).to(device)
        p[idx, frame - 3] ^= 0x5A
    lens = torch.full((n,), frame + lh, dtype=torch.int32, device=device)
    return arena, lens, bad, stride


TX_IP_CSUM = 10   # header.IPv4 checksum field (ipv4.go:35 checksum offset)
TX_TCP_CSUM = 16  # header.TCP checksum field, from the TCP header start


def tx_desc(n: int, fused: bool = True) -> np.ndarray:
    """rx_batch's table with the stores of the transmit side (flags for
    ns_csum_batch_dev_store): the IPv4 run stores ^sum at byte 10
    (addIPHeader: ip.SetChecksum(^ip.CalculateChecksum()), ipv4.go:236) and
    the pseudo-header + TCP run stores ^sum at TCP byte 16 (buildTCPHdr:
    tcp.SetChecksum(^tcp.CalculateChecksum(xsum)), connect.go:662-663)."""
    d = _tcp_desc(n, fused)
    k = per_packet(fused)
    d["flags"][0::k] |= 0x4 | (TX_IP_CSUM << 4)
    # the TCP checksum field: TCP byte 16 = packet byte 36, from the TCP
    # descriptor's start (byte 12 fused, byte 20 chained)
    d["flags"][k - 1::k] |= 0x4 | ((RX_IHL + TX_TCP_CSUM - (12 if fused else RX_IHL)) << 4)
    return d


def tx_batch(n: int, seed: int, device, fused: bool = True):
    """The transmit side of rx_batch: the same n packets with both checksum
    fields zero, and tx_desc(n).  One ns_csum_batch_dev_store launch (with
    NS_BATCH_CHAINED for the chained table) fills the fields in place;
    afterwards the arena equals rx_batch(n, seed)'s byte for byte.  Returns
    (arena, desc)."""
    arena, _ = _tcp_packets(n, seed, device)
    return arena, tx_desc(n, fused)


# ---------------------------------------------------------------------------
# Transmit batches laid out as sendTCPBatch builds them (transport/tcp/
# connect.go:668-702).  stack.NewPacketDescriptors(n, hdrSize) allocates ONE
# buffer of n * hdrSize bytes and gives segment i a Prependable over slot i
# (stack/route.go:181-188); buildTCPHdr prepends the TCP header at the slot's
# end, addIPHeader the IPv4 header before it (the link header's room comes
# first); the payload is one VectorisedView, segment i at Off = i * MSS.  In
# HBM: [n header slots | payload], one arena.  Per packet (3 descriptors,
# NS_BATCH_CHAINED):
#   3i    the IPv4 header [slot+14, +20)                       store ^sum at +10
#   3i+1  the payload [P + i*MSS, +MSS), initial = ChecksumCombine(1480, 6)
#   3i+2  src+dst addresses and the TCP header [slot+26, +28), NS_DESC_CONT:
#         the run's final value (PseudoHeaderChecksum, ChecksumVVWithOffset,
#         CalculateChecksum: restarts at even offsets, no uint32 wrap, so the
#         order of the pieces does not change the folded sum)
#                                                              store ^sum at +24
# = TCP byte 16.  The checksum fields are dense (two per 54-B slot), where in
# the wire layout (tx_batch) they sit one packet stride apart.
# ---------------------------------------------------------------------------
TX_HDR = 54     # TCPMinimumSize + MaxHeaderLength (IPv4 20 + Ethernet 14), no options
TX_MSS = RX_TCP - 20  # 1460
TX_IP_AT = 14   # the IPv4 header's offset in a slot
TX_TCP_AT = 34  # the TCP header's offset in a slot
TX_SRC = bytes([10, 0, 0, 1])  # the route's addresses (every segment of one
TX_DST = bytes([10, 0, 0, 2])  # sendTCPBatch call shares them, route.go:93-95)


def tx_split_layout(n: int) -> tuple[int, int]:
    """(payload region offset, arena bytes) of the sendTCPBatch layout."""
    pay = (n * TX_HDR + 4095) // 4096 * 4096
    return pay, pay + n * TX_MSS


def tx_split_desc(n: int, store: bool = True, paired: bool = False) -> np.ndarray:
    """The table over the sendTCPBatch layout.  Chained (NS_BATCH_CHAINED):
    per packet [IPv4 header, payload, addresses + TCP header (CONT)].  Paired
    (NS_BATCH_PAIRED, n even): per two packets 2k, 2k+1
        6k    payload of 2k       6k+1  addresses + TCP header of 2k (CONT)
        6k+2  IPv4 header of 2k   6k+3  IPv4 header of 2k+1
        6k+4  payload of 2k+1     6k+5  addresses + TCP header of 2k+1 (CONT)
    so every pair starts at an even index and each packet's descriptors stay
    together.  tx_split_order(n, paired) maps packets to their results."""
    d = _tx_split_chained(n, store)
    if not paired:
        return d
    if n % 2:
        raise ValueError("the paired table needs an even packet count")
    ip, pay_, tcp = d[0::3].reshape(-1, 2), d[1::3].reshape(-1, 2), d[2::3].reshape(-1, 2)
    p = np.zeros(3 * n, dtype=DESC_DTYPE).reshape(-1, 6)
    p[:, 0], p[:, 1] = pay_[:, 0], tcp[:, 0]
    p[:, 2], p[:, 3] = ip[:, 0], ip[:, 1]
    p[:, 4], p[:, 5] = pay_[:, 1], tcp[:, 1]
    return p.reshape(-1)


def tx_split_order(n: int, paired: bool) -> tuple[np.ndarray, np.ndarray]:
    """(index of each packet's IPv4 result, index of its TCP result) in the
    results of tx_split_desc(n, paired=...)."""
    i = np.arange(n)
    if not paired:
        return 3 * i, 3 * i + 2
    k, odd = i // 2, i % 2
    return 6 * k + 2 + odd, 6 * k + 1 + 4 * odd


def _tx_split_chained(n: int, store: bool) -> np.ndarray:
    pay, _ = tx_split_layout(n)
    slot = np.arange(n, dtype=np.uint64) * np.uint64(TX_HDR)
    d = np.zeros(3 * n, dtype=DESC_DTYPE)
    d["off"][0::3] = slot + np.uint64(TX_IP_AT)
    d["len"][0::3] = RX_IHL
    d["off"][1::3] = np.uint64(pay) + np.arange(n, dtype=np.uint64) * np.uint64(TX_MSS)
    d["len"][1::3] = TX_MSS
    d["initial"][1::3] = RX_TCP + 6  # ChecksumCombine(1480, 6): no carry
    d["off"][2::3] = slot + np.uint64(TX_IP_AT + 12)
    d["len"][2::3] = 8 + 20
    d["flags"][2::3] = 2  # NS_DESC_CONT
    if store:
        d["flags"][0::3] |= 0x4 | (TX_IP_CSUM << 4)
        d["flags"][2::3] |= 0x4 | ((TX_TCP_AT - (TX_IP_AT + 12) + TX_TCP_CSUM) << 4)
    return d


def _split_packets(n: int, seed: int, device):
    """The sendTCPBatch-layout arena (splitmix64 bytes with fixed header
    fields, both checksum fields zero) and views of its header slots and
    payloads."""
    import torch

    pay, total = tx_split_layout(n)
    arena = random_bytes_torch(seed, total, device)
    h = arena[:n * TX_HDR].view(n, TX_HDR)
    ip = h[:, TX_IP_AT:TX_IP_AT + RX_IHL]
    ip[:, 0] = 0x45
    ip[:, 1] = 0
    ip[:, 2] = RX_PKT >> 8
    ip[:, 3] = RX_PKT & 0xFF
    ip[:, 6] = 0x40
    ip[:, 7] = 0
    ip[:, 8] = 64
    ip[:, 9] = 6
    ip[:, 10:12] = 0
    ip[:, 12:16] = torch.tensor(list(TX_SRC), dtype=torch.uint8, device=arena.device)
    ip[:, 16:20] = torch.tensor(list(TX_DST), dtype=torch.uint8, device=arena.device)
    t = h[:, TX_TCP_AT:TX_TCP_AT + 20]
    t[:, 12] = 0x50
    t[:, 13] = 0x18
    t[:, 16:20] = 0
    return arena, h, arena[pay:pay + n * TX_MSS].view(n, TX_MSS)


def tx_struct_geometry(n: int) -> dict:
    """The geometry of the sendTCPBatch-layout arena (_split_packets) for
    ns_csum_tcp_tx: the same fill as tx_split_desc's table, taken from the
    layout itself (Engine.tcp_tx)."""
    pay, _ = tx_split_layout(n)
    return dict(hdr_off=0, pay_off=pay, size=n * TX_MSS, mss=TX_MSS, slot=TX_HDR, ip_at=TX_IP_AT, ip_len=RX_IHL,
                tcp_at=TX_TCP_AT, tcp_len=20, src=TX_SRC, dst=TX_DST, protocol=6)


def tx_split_batch(n: int, seed: int, device):
    """n outbound IPv4/TCP segments in the sendTCPBatch layout with both
    checksum fields zero, and tx_split_desc(n).  One ns_csum_batch_dev_store
    launch with NS_BATCH_CHAINED fills them; afterwards the arena equals
    tx_split_expected(n, seed)'s.  Returns (arena, desc)."""
    arena, _, _ = _split_packets(n, seed, device)
    return arena, tx_split_desc(n)


def tx_split_expected(n: int, seed: int, device, chunk: int = 1 << 16):
    """The same arena with both checksum fields written (RFC 1071 sums with
    torch integer ops, as plain data generation, per chunk of packets)."""
    import torch

    arena, h, p = _split_packets(n, seed, device)

    def be_sum(x):
        w = x.to(torch.int64)
        return (w[:, 0::2] * 256 + w[:, 1::2]).sum(dim=1)

    for a in range(0, n, chunk):
        b = min(n, a + chunk)
        hh, pp = h[a:b], p[a:b]
        ip = (~_fold_np(be_sum(hh[:, TX_IP_AT:TX_IP_AT + RX_IHL]))) & 0xFFFF
        hh[:, TX_IP_AT + 10] = (ip >> 8).to(torch.uint8)
        hh[:, TX_IP_AT + 11] = (ip & 0xFF).to(torch.uint8)
        tcp = (~_fold_np(be_sum(hh[:, TX_IP_AT + 12:TX_TCP_AT + 20]) + be_sum(pp) + RX_TCP + 6)) & 0xFFFF
        hh[:, TX_TCP_AT + 16] = (tcp >> 8).to(torch.uint8)
        hh[:, TX_TCP_AT + 17] = (tcp & 0xFF).to(torch.uint8)
    return arena
