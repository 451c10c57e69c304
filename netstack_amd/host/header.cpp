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

namespace {
// ns_pkt_buf table over the packets' own bytes (Header's used part, Data's
// views); `views` keeps each packet's ns_view array alive.
std::vector<ns_pkt_buf> to_pkt_bufs(const std::vector<tcpip::PacketBuffer>& pkts,
                                    std::vector<std::vector<ns_view>>* views) {
  std::vector<ns_pkt_buf> t(pkts.size());
  views->resize(pkts.size());
  for (size_t i = 0; i < pkts.size(); ++i) {
    const tcpip::PacketBuffer& p = pkts[i];
    (*views)[i] = to_views(p.Data.Views());
    const buffer::View hv = p.Header.View();
    t[i].hdr = const_cast<uint8_t*>(hv.data());
    t[i].hdr_len = hv.size();
    t[i].data = (*views)[i].data();
    t[i].ndata = (uint32_t)(*views)[i].size();
    t[i].flags = 0;
    t[i].data_size = p.Data.Size();
  }
  return t;
}
}  // namespace

std::vector<uint8_t> VerifyPacketBuffers(const std::vector<tcpip::PacketBuffer>& pkts) {
  std::vector<std::vector<ns_view>> keep;
  std::vector<ns_pkt_buf> t = to_pkt_bufs(pkts, &keep);
  std::vector<uint8_t> verdict(pkts.size());
  if (!pkts.empty())
    check(ns_csum_packet_buffers(Engine(), t.data(), (uint32_t)t.size(), NS_PKB_VERIFY, nullptr, verdict.data()),
          "VerifyPacketBuffers");
  return verdict;
}

void FillPacketBuffers(std::vector<tcpip::PacketBuffer>& pkts) {
  std::vector<std::vector<ns_view>> keep;
  std::vector<ns_pkt_buf> t = to_pkt_bufs(pkts, &keep);
  if (!pkts.empty())
    check(ns_csum_packet_buffers(Engine(), t.data(), (uint32_t)t.size(), NS_PKB_FILL, nullptr, nullptr),
          "FillPacketBuffers");
}

}  // namespace header
}  // namespace netstack
