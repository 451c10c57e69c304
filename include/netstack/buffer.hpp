// netstack/buffer.hpp — C++ mirror of google/netstack tcpip/buffer (view.go,
// prependable.go), the checksum's input layout.  Same type and method names
// as the Go package (View, VectorisedView, Prependable, TrimFront, CapLength,
// ToView, Prepend, ...), same semantics;
// views alias their backing bytes exactly like Go slices (no copies on trim).
// Out-of-range slicing throws std::out_of_range where Go panics.
#pragma once

#include <cstddef>
#include <cstdint>
#include <memory>
#include <stdexcept>
#include <vector>

namespace netstack {
namespace buffer {

// View (view.go:19): a slice of a byte buffer.
class View {
 public:
  View() = default;
  // Borrow `len` bytes at `data` (the caller keeps them alive).
  View(const uint8_t* data, size_t len) : data_(data), len_(len) {}
  // Own a copy of the bytes.
  explicit View(std::vector<uint8_t> bytes)
      : own_(std::make_shared<std::vector<uint8_t>>(std::move(bytes))),
        data_(own_->data()),
        len_(own_->size()) {}

  // view.go:34-36
  void TrimFront(size_t count) {
    if (count > len_) throw std::out_of_range("View.TrimFront: slice bounds out of range");
    data_ += count;
    len_ -= count;
  }
  // view.go:40-46
  void CapLength(size_t length) {
    if (length > len_) throw std::out_of_range("View.CapLength: slice bounds out of range");
    len_ = length;
  }
  const uint8_t* data() const { return data_; }
  size_t size() const { return len_; }
  uint8_t operator[](size_t i) const { return data_[i]; }

 private:
  std::shared_ptr<std::vector<uint8_t>> own_;
  const uint8_t* data_ = nullptr;
  size_t len_ = 0;
};

// NewView (view.go:23-25)
inline View NewView(size_t size) { return View(std::vector<uint8_t>(size, 0)); }
// NewViewFromBytes (view.go:28-30)
inline View NewViewFromBytes(std::vector<uint8_t> b) { return View(std::move(b)); }

// VectorisedView (view.go:57-60)
class VectorisedView {
 public:
  VectorisedView() = default;
  VectorisedView(size_t size, std::vector<View> views) : views_(std::move(views)), size_(size) {}

  // view.go:69-79 (a count <= 0 leaves the view unchanged, as in Go)
  void TrimFront(long long count) {
    while (count > 0 && !views_.empty()) {
      if ((size_t)count < views_[0].size()) {
        size_ -= count;
        views_[0].TrimFront((size_t)count);
        return;
      }
      count -= (long long)views_[0].size();
      RemoveFirst();
    }
  }
  // view.go:82-103 (a negative length clamps to 0 as in Go)
  void CapLength(long long length) {
    if (length < 0) length = 0;
    if ((long long)size_ < length) return;
    size_ = (size_t)length;
    for (size_t i = 0; i < views_.size(); ++i) {
      if ((long long)views_[i].size() >= length) {
        if (length == 0) {
          views_.resize(i);
        } else {
          views_[i].CapLength((size_t)length);
          views_.resize(i + 1);
        }
        return;
      }
      length -= (long long)views_[i].size();
    }
  }
  // view.go:121-127
  void RemoveFirst() {
    if (views_.empty()) return;
    size_ -= views_[0].size();
    views_.erase(views_.begin());
  }
  // view.go:113-118
  View First() const { return views_.empty() ? View() : views_[0]; }
  // view.go:130-132
  size_t Size() const { return size_; }
  // view.go:150-152
  const std::vector<View>& Views() const { return views_; }
  // view.go:138-147
  View ToView() const {
    if (views_.size() == 1) return views_[0];
    std::vector<uint8_t> u;
    u.reserve(size_);
    for (const View& v : views_) u.insert(u.end(), v.data(), v.data() + v.size());
    return View(std::move(u));
  }
  // view.go:155-158
  void Append(const VectorisedView& vv2) {
    views_.insert(views_.end(), vv2.views_.begin(), vv2.views_.end());
    size_ += vv2.size_;
  }

 private:
  std::vector<View> views_;
  size_t size_ = 0;
};

// NewVectorisedView (view.go:64-66)
inline VectorisedView NewVectorisedView(size_t size, std::vector<View> views) {
  return VectorisedView(size, std::move(views));
}

// Prependable (prependable.go:22-28): a buffer that grows backwards; each
// protocol prepends its header in front of the one above.  The bytes are
// shared by copies of the value, as a Go slice's backing array is.
class Prependable {
 public:
  Prependable() = default;
  Prependable(std::shared_ptr<std::vector<uint8_t>> buf, size_t used_idx)
      : buf_(std::move(buf)), end_(buf_ ? buf_->size() : 0), used_(used_idx) {}

  // prependable.go:56-58: the used part (aliases the bytes).
  buffer::View View() const { return buffer::View(base() + used_, end_ - used_); }
  // The used part, writable (header fields are set through it).
  uint8_t* Data() { return base() + used_; }
  // prependable.go:61-63, 66-68
  size_t UsedLength() const { return end_ - used_; }
  size_t AvailableLength() const { return used_; }
  // prependable.go:71-73
  void TrimBack(size_t size) {
    if (size > end_ - used_) throw std::out_of_range("Prependable.TrimBack: slice bounds out of range");
    end_ -= size;
  }
  // prependable.go:77-84: the reserved bytes in front, or nullptr if they do
  // not fit (Go returns nil).
  uint8_t* Prepend(size_t size) {
    if (size > used_) return nullptr;
    used_ -= size;
    return base() + used_;
  }
  // prependable.go:87-90
  Prependable DeepCopy() const {
    auto b = std::make_shared<std::vector<uint8_t>>(base(), base() + end_);
    Prependable p(std::move(b), used_);
    return p;
  }

 private:
  uint8_t* base() const { return buf_ ? buf_->data() : nullptr; }
  std::shared_ptr<std::vector<uint8_t>> buf_;
  size_t end_ = 0;
  size_t used_ = 0;
};

// prependable.go:31-33
inline Prependable NewPrependable(size_t size) {
  return Prependable(std::make_shared<std::vector<uint8_t>>(size, 0), size);
}
// prependable.go:40-42 (takes ownership of the bytes)
inline Prependable NewPrependableFromView(std::vector<uint8_t> v) {
  return Prependable(std::make_shared<std::vector<uint8_t>>(std::move(v)), 0);
}
// prependable.go:45-47
inline Prependable NewEmptyPrependableFromView(std::vector<uint8_t> v) {
  const size_t n = v.size();
  return Prependable(std::make_shared<std::vector<uint8_t>>(std::move(v)), n);
}

}  // namespace buffer
}  // namespace netstack
