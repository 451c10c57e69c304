"""CPU: the tcpip/buffer mirror keeps view.go semantics (view_test.go:89-235
style tables for TrimFront / CapLength / ToView)."""
from netstack_amd.buffer import NewVectorisedView, NewView, NewViewFromBytes, View


def vv(size, *pieces):
    # view_test.go:36-43 helper
    return NewVectorisedView(size, [NewViewFromBytes(p.encode()) for p in pieces])


def flat(v):
    return b"".join(bytes(x) for x in v.Views())


def _same(a, b):
    return a.Size() == b.Size() and flat(a) == flat(b) and len(a.Views()) == len(b.Views())


def test_cap_length():
    # view_test.go:44-97 capLengthTestCases
    cases = [
        ("Simple case", vv(2, "12"), 1, vv(1, "1")),
        ("Case spanning across two Views", vv(4, "123", "4"), 2, vv(2, "12")),
        ("Corner case with negative length", vv(1, "1"), -1, vv(0)),
        ("Corner case with length = 0", vv(3, "12", "3"), 0, vv(0)),
        ("Corner case with length = size", vv(1, "1"), 1, vv(1, "1")),
        ("Corner case with length > size", vv(1, "1"), 2, vv(1, "1")),
    ]
    for name, v, n, want in cases:
        v.CapLength(n)
        assert _same(v, want), name


def test_trim_front():
    # view_test.go:99-160 trimFrontTestCases
    cases = [
        ("Simple case", vv(2, "12"), 1, vv(1, "2")),
        ("Case where we trim an entire View", vv(2, "1", "2"), 1, vv(1, "2")),
        ("Case spanning across two Views", vv(3, "1", "23"), 2, vv(1, "3")),
        ("Corner case with negative count", vv(1, "1"), -1, vv(1, "1")),
        ("Corner case with count = 0", vv(1, "1"), 0, vv(1, "1")),
        ("Corner case with count = size", vv(1, "1"), 1, vv(0)),
        ("Corner case with count > size", vv(1, "1"), 2, vv(0)),
    ]
    for name, v, n, want in cases:
        v.TrimFront(n)
        assert _same(v, want), name


def test_to_view():
    # view_test.go:162-190 toViewCases
    for v, want in [(vv(2, "12"), b"12"), (vv(2, "1", "2"), b"12"), (vv(0), b"")]:
        assert bytes(v.ToView()) == want


def test_to_view_and_append():
    v = vv(4, "12", "34")
    assert bytes(v.ToView()) == b"1234"
    v.Append(vv(2, "56"))
    assert v.Size() == 6 and bytes(v.ToView()) == b"123456"
    assert bytes(vv(1, "1").ToView()) == b"1"


def test_view_aliases_backing_bytes():
    b = bytearray(b"abcdef")
    v = View(b)
    v.TrimFront(2)
    b[3] = ord("X")
    assert bytes(v) == b"cXef"
    n = NewView(3)
    assert bytes(n) == b"\0\0\0"


def test_prependable_grows_backwards():
    """buffer.Prependable (prependable.go): Prepend reserves bytes in front,
    View is the used part and aliases the backing buffer, Prepend past the
    available space returns nil; TrimBack; the FromView constructors."""
    from netstack_amd.buffer import NewEmptyPrependableFromView, NewPrependable, NewPrependableFromView, View

    p = NewPrependable(10)
    assert p.UsedLength() == 0 and p.AvailableLength() == 10 and len(p.View()) == 0
    p.Prepend(4)[:] = b"tcp!"
    p.Prepend(2)[:] = b"ip"
    assert bytes(p.View()) == b"iptcp!" and p.UsedLength() == 6 and p.AvailableLength() == 4
    assert p.Prepend(5) is None and p.UsedLength() == 6
    v = p.View()
    v.memory[0] = ord("I")  # aliases the backing bytes
    assert bytes(p.View()) == b"Iptcp!"
    q = p.DeepCopy()
    q.View().memory[0] = ord("x")
    assert bytes(p.View()) == b"Iptcp!" and bytes(q.View()) == b"xptcp!"
    p.TrimBack(1)
    assert bytes(p.View()) == b"Iptcp"
    full = NewPrependableFromView(View(bytearray(b"abc")))
    assert full.UsedLength() == 3 and full.Prepend(1) is None
    empty = NewEmptyPrependableFromView(View(bytearray(b"abc")))
    assert empty.UsedLength() == 0 and empty.AvailableLength() == 3


def test_packet_buffer_clone_copies_the_vv_not_the_bytes():
    """PacketBuffer.Clone (packet_buffer.go:55-58): Data is a new
    VectorisedView over the same bytes; trimming the clone leaves the
    original's views alone."""
    from netstack_amd.buffer import NewVectorisedView, View
    from netstack_amd.packet import PacketBuffer

    b = bytearray(b"0123456789")
    pk = PacketBuffer(Data=NewVectorisedView(10, [View(b)]))
    c = pk.Clone()
    c.Data.TrimFront(3)
    assert pk.Data.Size() == 10 and bytes(pk.Data.First()) == b"0123456789"
    b[5] = ord("X")
    assert bytes(c.Data.First()) == b"34X6789"
