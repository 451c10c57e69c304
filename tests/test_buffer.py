"""CPU: the tcpip/buffer mirror keeps view.go semantics (view_test.go:89-235
style tables for TrimFront / CapLength / ToView)."""
from netstack_amd.buffer import NewVectorisedView, NewView, NewViewFromBytes, View


def vv(size, *pieces):
    # view_test.go:36-43 helper
    return NewVectorisedView(size, [NewViewFromBytes(p.encode()) for p in pieces])


def flat(v):
    return b"".join(bytes(x) for x in v.Views())


def test_cap_length():
    cases = [
        (vv(2, "12"), 1, vv(1, "1")),
        (vv(2, "12"), 0, vv(0)),
        (vv(2, "12"), 2, vv(2, "12")),
        (vv(4, "12", "34"), 3, vv(3, "12", "3")),
        (vv(4, "12", "34"), 2, vv(2, "12")),
        (vv(4, "12", "34"), 5, vv(4, "12", "34")),
        (vv(4, "12", "34"), -1, vv(0)),
    ]
    for v, n, want in cases:
        v.CapLength(n)
        assert v.Size() == want.Size() and flat(v) == flat(want) and len(v.Views()) == len(want.Views())


def test_trim_front():
    cases = [
        (vv(2, "12"), 1, vv(1, "2")),
        (vv(2, "12"), 2, vv(0)),
        (vv(4, "12", "34"), 1, vv(3, "2", "34")),
        (vv(4, "12", "34"), 2, vv(2, "34")),
        (vv(4, "12", "34"), 3, vv(1, "4")),
        (vv(4, "12", "34"), 5, vv(0)),
    ]
    for v, n, want in cases:
        v.TrimFront(n)
        assert v.Size() == want.Size() and flat(v) == flat(want)


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
