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
