"""Mirror of google/netstack ``tcpip/buffer`` (view.go, prependable.go) — the
checksum's input layout.

``View`` is a byte slice with ``TrimFront``/``CapLength`` (view.go:18-51),
``VectorisedView`` a list of views plus a size (view.go:53-158) and
``Prependable`` the outbound header buffer that grows backwards
(prependable.go:17-85).  The methods
keep the Go names and semantics so tests read like the reference's own
(tcpip/buffer/view_test.go, tcpip/header/checksum_test.go).  No copies are made
when trimming: views are memoryviews over the caller's bytes, exactly as Go
slices alias their backing array.  The gather of these views into the
device-staged layout (pinned arena + 16-byte descriptor table) is done natively
by the C ABI (netstack_amd/csrc/csum_api.cpp).
"""
from __future__ import annotations


class View:
    """buffer.View (view.go:19): a slice of a byte buffer."""

    __slots__ = ("_m",)

    def __init__(self, data=b""):
        m = data._m if isinstance(data, View) else memoryview(data)
        self._m = m.cast("B") if m.format != "B" or m.ndim != 1 else m

    def TrimFront(self, count: int) -> None:  # view.go:34-36
        if count < 0 or count > len(self._m):
            raise IndexError("slice bounds out of range")
        self._m = self._m[count:]

    def CapLength(self, length: int) -> None:  # view.go:40-46
        if length < 0 or length > len(self._m):
            raise IndexError("slice bounds out of range")
        self._m = self._m[:length]

    def ToVectorisedView(self) -> "VectorisedView":  # view.go:49-51
        return NewVectorisedView(len(self), [self])

    def __len__(self) -> int:
        return len(self._m)

    def __bytes__(self) -> bytes:
        return self._m.tobytes()

    def __getitem__(self, k):
        r = self._m[k]
        return View(r) if isinstance(k, slice) else r

    def __buffer__(self, flags):  # pragma: no cover - py>=3.12
        return self._m.__buffer__(flags)

    @property
    def memory(self) -> memoryview:
        return self._m

    def __eq__(self, other) -> bool:
        return bytes(self) == bytes(other)

    def __repr__(self) -> str:
        return f"View({bytes(self)!r})"


def NewView(size: int) -> View:  # view.go:23-25
    return View(bytearray(size))


def NewViewFromBytes(b) -> View:  # view.go:28-30
    return View(bytearray(bytes(b)))


class VectorisedView:
    """buffer.VectorisedView (view.go:57-60): views + size."""

    __slots__ = ("views", "size")

    def __init__(self, views=None, size: int = 0):
        self.views = list(views or [])
        self.size = size

    def TrimFront(self, count: int) -> None:  # view.go:69-79
        while count > 0 and self.views:
            if count < len(self.views[0]):
                self.size -= count
                self.views[0].TrimFront(count)
                return
            count -= len(self.views[0])
            self.RemoveFirst()

    def CapLength(self, length: int) -> None:  # view.go:82-103
        if length < 0:
            length = 0
        if self.size < length:
            return
        self.size = length
        for i, v in enumerate(self.views):
            if len(v) >= length:
                if length == 0:
                    self.views = self.views[:i]
                else:
                    v.CapLength(length)
                    self.views = self.views[: i + 1]
                return
            length -= len(v)

    def Clone(self, buffer=None) -> "VectorisedView":  # view.go:108-110
        return VectorisedView([View(v) for v in self.views], self.size)

    def First(self):  # view.go:113-118
        return self.views[0] if self.views else None

    def RemoveFirst(self) -> None:  # view.go:121-127
        if not self.views:
            return
        self.size -= len(self.views[0])
        self.views = self.views[1:]

    def Size(self) -> int:  # view.go:130-132
        return self.size

    def ToView(self) -> View:  # view.go:138-147
        if len(self.views) == 1:
            return self.views[0]
        return View(bytearray(b"".join(bytes(v) for v in self.views)))

    def Views(self):  # view.go:150-152
        return self.views

    def Append(self, vv2: "VectorisedView") -> None:  # view.go:155-158
        self.views.extend(vv2.views)
        self.size += vv2.size


def NewVectorisedView(size: int, views) -> VectorisedView:  # view.go:64-66
    return VectorisedView([v if isinstance(v, View) else View(v) for v in views], size)


class Prependable:
    """buffer.Prependable (prependable.go:22-28): a buffer that grows
    backwards; each layer prepends its header in front of the one above.
    ``View()`` aliases the backing bytes, as the Go slice does."""

    __slots__ = ("buf", "usedIdx")

    def __init__(self, buf: View | None = None, usedIdx: int = 0):
        self.buf = buf if buf is not None else View(bytearray())
        self.usedIdx = usedIdx

    def View(self) -> View:  # prependable.go:56-58
        return self.buf[self.usedIdx:]

    def UsedLength(self) -> int:  # prependable.go:61-63
        return len(self.buf) - self.usedIdx

    def AvailableLength(self) -> int:  # prependable.go:66-68
        return self.usedIdx

    def TrimBack(self, size: int) -> None:  # prependable.go:71-73
        self.buf = self.buf[: len(self.buf) - size]

    def Prepend(self, size: int):  # prependable.go:77-84
        """The reserved `size` bytes in front (a writable memoryview), or
        None if they do not fit."""
        if size > self.usedIdx:
            return None
        self.usedIdx -= size
        return self.View().memory[:size]

    def DeepCopy(self) -> "Prependable":  # prependable.go:87-90
        return Prependable(View(bytearray(bytes(self.buf))), self.usedIdx)


def NewPrependable(size: int) -> Prependable:  # prependable.go:31-33
    return Prependable(NewView(size), size)


def NewPrependableFromView(v: View) -> Prependable:  # prependable.go:40-42
    return Prependable(v if isinstance(v, View) else View(v), 0)


def NewEmptyPrependableFromView(v: View) -> Prependable:  # prependable.go:45-47
    v = v if isinstance(v, View) else View(v)
    return Prependable(v, len(v))
