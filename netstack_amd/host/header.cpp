// header.cpp — C++ mirror of tcpip/header's checksum functions over the C ABI
// (see include/netstack/header.hpp).  Only marshalling happens here.
#include "netstack/header.hpp"

#include <mutex>

namespace netstack {
namespace header {
namespace {

std::vector<ns_view> to_views(const std::vector<buffer::View>& vs) {
  std::vector<ns_view> out;
  out.reserve(vs.size());
  for (const buffer::View& v : vs) out.push_back(ns_view{v.data(), (uint64_t)v.size()});
  return out;
}

void check(int rc, const char* what) {
  if (rc == NS_OK) return;
  if (rc == NS_EINVAL) throw std::out_of_range(std::string(what) + ": slice bounds out of range");
  throw ChecksumError(rc, what);
}

}  // namespace

ns_csum_ctx* Engine(int device) {
  static std::mutex mu;
  static std::vector<ns_csum_ctx*> ctxs;
  std::lock_guard<std::mutex> lk(mu);
  if ((size_t)device >= ctxs.size()) ctxs.resize(device + 1, nullptr);
  if (!ctxs[device]) {
    ns_csum_opts o{};
    o.device = device;
    check(ns_csum_init(&o, &ctxs[device]), "ns_csum_init");
  }
  return ctxs[device];
}

uint16_t Checksum(const buffer::View& buf, uint16_t initial) {
  uint16_t r = 0;
  check(ns_csum_checksum(Engine(), buf.data(), buf.size(), initial, &r), "Checksum");
  return r;
}

uint16_t Checksum(const std::vector<uint8_t>& buf, uint16_t initial) {
  return Checksum(buffer::View(buf.data(), buf.size()), initial);
}

uint16_t ChecksumVV(const buffer::VectorisedView& vv, uint16_t initial) {
  return ChecksumVVWithOffset(vv, initial, 0, (long long)vv.Size());
}

uint16_t ChecksumVVWithOffset(const buffer::VectorisedView& vv, uint16_t initial, long long off,
                              long long size) {
  std::vector<ns_view> v = to_views(vv.Views());
  uint16_t r = 0;
  check(ns_csum_vv_with_offset(Engine(), v.data(), (uint32_t)v.size(), initial, off, size, &r),
        "ChecksumVVWithOffset");
  return r;
}

uint16_t ChecksumCombine(uint16_t a, uint16_t b) { return ns_csum_combine(a, b); }

uint16_t PseudoHeaderChecksum(uint32_t protocol, const std::string& srcAddr,
                              const std::string& dstAddr, uint16_t totalLen) {
  uint16_t r = 0;
  check(ns_csum_pseudo_header(Engine(), protocol, (const uint8_t*)srcAddr.data(),
                              (uint32_t)srcAddr.size(), (const uint8_t*)dstAddr.data(),
                              (uint32_t)dstAddr.size(), totalLen, &r),
        "PseudoHeaderChecksum");
  return r;
}

std::vector<uint16_t> ChecksumVVBatch(const buffer::VectorisedView& vv,
                                      const std::vector<SegDesc>& segs) {
  std::vector<ns_view> v = to_views(vv.Views());
  std::vector<ns_seg> s;
  s.reserve(segs.size());
  for (const SegDesc& d : segs) s.push_back(ns_seg{d.Off, d.Size, d.Initial, 0, 0});
  std::vector<uint16_t> out(segs.size());
  if (!segs.empty())
    check(ns_csum_vv_batch(Engine(), v.data(), (uint32_t)v.size(), s.data(), (uint32_t)s.size(),
                           out.data()),
          "ChecksumVVBatch");
  return out;
}

uint16_t ChecksumViews(const std::vector<buffer::View>& views, uint16_t initial) {
  std::vector<ns_view> v = to_views(views);
  uint16_t r = 0;
  check(ns_csum_views_restart(Engine(), v.data(), (uint32_t)v.size(), initial, &r), "ChecksumViews");
  return r;
}

}  // namespace header
}  // namespace netstack
