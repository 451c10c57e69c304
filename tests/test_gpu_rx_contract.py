"""GPU: the receive contract (netstack_amd/rx.py) and the
fragment cases, through ns_csum_packet_buffers, against the reference's own
fixtures (tests/golden/rx_fixtures.json) and the oracle:

* TestInvalidFragments' packets (ipv4_test.go:360-455): the engine's verdicts
  and sums equal oracle/packets.py's, packet by packet;
* TestFragmentation's shapes (ipv4_test.go:257-270): fragments filled by the
  engine equal writePacketFragments' headers byte for byte;
* a recvmmsg batch holding a corrupted *fragmented* TCP segment: the link's
  pass cannot check it (UNCHECKED), the contract verifies it after
  reassembly, and ChecksumErrors counts it — with the reference's
  TestReceivedIncorrectChecksumIncrement segment (tcp_test.go:3232-3259)
  and intact segments, fragmented or not, in the same batch.
"""
import random

import numpy as np
import pytest

import rxcases as R

pytestmark = pytest.mark.gpu

BUF_CONFIG = [128, 256, 256, 512, 1024, 2048, 4096, 8192, 16384, 32768]  # packet_dispatchers.go:30


def _rx_pk(b: bytes, link_hdr: int = 14):
    """recvMMsgDispatcher's views (BufConfig, capped, link header trimmed)."""
    from netstack_amd.buffer import NewVectorisedView, View
    from netstack_amd.packet import PacketBuffer

    frame = bytes(link_hdr) + b
    views, c = [], 0
    for s in BUF_CONFIG:
        views.append(View(bytearray(frame[c:c + s])))
        c += s
        if c >= len(frame):
            break
    vv = NewVectorisedView(len(frame), views)
    vv.TrimFront(link_hdr)
    return PacketBuffer(Data=vv)


def test_invalid_fragments_verdicts_match_the_oracle(engine):
    import packets as P

    from netstack_amd.packet import verify_packet_buffers

    fx = R.fixtures()
    raw = [bytes.fromhex(p) for c in fx["invalid_fragments"] for p in c["packets"]]
    pkts = [_rx_pk(b, k % 2 * 14) for k, b in enumerate(raw)]
    verdict, sums = verify_packet_buffers(pkts, engine)
    for i, b in enumerate(raw):
        want = P.verify(b"", [b], len(b))
        assert (int(verdict[i]), int(sums[2 * i]), int(sums[2 * i + 1])) == want, (i, b.hex())
    assert P.MALFORMED in verdict.tolist() and P.UNCHECKED in verdict.tolist()


def test_fragments_filled_as_write_packet_fragments_writes_them(engine):
    from netstack_amd.buffer import NewPrependableFromView, NewVectorisedView, View
    from netstack_amd.packet import PacketBuffer, fill_packet_buffers

    rnd = random.Random(270)
    pkts, want = [], []
    for row in R.fixtures()["fragmentation"]:
        sizes = R.view_sizes(row["views"])
        rest = bytes(rnd.getrandbits(8) for _ in range(row["hdr_length"]))
        views = [bytes(rnd.getrandbits(8) for _ in range(s)) for s in sizes]
        ip = R.build_segment(b"\x10\0\0\1", b"\x10\0\0\2", 1, 2, 3, 4, 0x10, 5, b"", ttl=42, ident=9)[:20]
        ip[2:4] = (20 + len(rest) + sum(sizes)).to_bytes(2, "big")
        filled = R.write_packet_fragments(bytes(ip) + rest, views, row["mtu"])
        bare = R.write_packet_fragments(bytes(ip) + rest, views, row["mtu"], set_checksums=False)
        if len(filled) == 1:
            continue  # not a fragment: a whole packet whose "TCP header" is random bytes
        for (h, d), (h0, d0) in zip(filled, bare):
            assert d == d0
            pkts.append(PacketBuffer(Data=NewVectorisedView(sum(map(len, d0)), [View(bytearray(v)) for v in d0]),
                                     Header=NewPrependableFromView(View(bytearray(h0)))))
            want.append(h)
    assert len(pkts) > 60
    fill_packet_buffers(pkts, engine)
    for i, pk in enumerate(pkts):
        assert bytes(pk.Header.View()) == want[i], i


def _segment(fx, payload, ident):
    c = fx["incorrect_checksum"]
    return R.build_segment(bytes.fromhex(c["src"]), bytes.fromhex(c["dst"]), c["src_port"], c["dst_port"], c["seq"],
                           c["ack"], c["flags"], c["window"], payload, ttl=c["ttl"], ident=ident)


@pytest.mark.parametrize("mtu", [300, 800, 1500])
def test_corrupted_fragmented_segment_fails_after_reassembly(engine, mtu):
    from netstack_amd.rx import RX_CHECKSUM_INVALID, RX_CHECKSUM_UNKNOWN, RX_CHECKSUM_VALID, ReceivePath

    fx = R.fixtures()
    c = fx["incorrect_checksum"]
    rng = np.random.default_rng(mtu)
    data = bytes(i & 0xFF for i in range(4000))  # testBrokenUpWrite's data[i] = byte(i) (tcp_test.go:2214-2216)
    good = _segment(fx, data, 101)
    bad = _segment(fx, data, 102)
    frags_good = R.write_packet_fragments(bytes(good[:20]), [bytes(good[20:])], mtu)
    frags_bad = R.write_packet_fragments(bytes(bad[:20]), [bytes(bad[20:])], mtu)
    assert len(frags_good) > 2
    # one payload byte of the second fragment flipped: every IPv4 header stays valid
    wire_bad = [h + b"".join(dd) for h, dd in frags_bad]
    k = 20 + int(rng.integers(0, len(wire_bad[1]) - 20))
    wb = bytearray(wire_bad[1])
    wb[k] ^= 0x5A
    wire_bad[1] = bytes(wb)
    # TestReceivedIncorrectChecksumIncrement's segment, corrupted and intact
    ref_payload = bytes.fromhex(c["payload"])
    ref_bad = _segment(fx, ref_payload, 0)
    ref_good = bytes(ref_bad)
    ref_bad[40 + c["corrupt_payload_byte"]] = c["corrupt_value"]
    wires = [h + b"".join(dd) for h, dd in frags_good] + wire_bad + [bytes(ref_bad), ref_good]
    order = list(range(len(wires)))
    random.Random(mtu).shuffle(order)  # fragments of both datagrams interleaved
    pkts = [_rx_pk(wires[i]) for i in order]
    rp = ReceivePath(engine)
    out = rp.deliver(pkts)
    # link verdicts: the fragments UNKNOWN, the whole segments VALID / INVALID
    by_wire = {order[j]: pkts[j].RXChecksum for j in range(len(pkts))}
    nf = len(frags_good) + len(frags_bad)
    assert all(by_wire[i] == RX_CHECKSUM_UNKNOWN for i in range(nf))
    assert by_wire[nf] == RX_CHECKSUM_INVALID and by_wire[nf + 1] == RX_CHECKSUM_VALID
    # delivered: the intact reassembled segment and the intact reference segment, nothing else
    assert sorted(o[2] for o in out) == sorted([bytes(good[20:]), ref_good[20:]])
    s = rp.stats
    assert s.TCPChecksumErrors == 2 and s.EndpointChecksumErrors == 2  # the fragmented one and the reference one
    assert s.TCPValidSegmentsReceived == 2 and s.IPMalformedPacketsReceived == 0
