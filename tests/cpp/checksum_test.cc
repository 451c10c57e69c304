// C++ mirror of the reference's own tests for this path, through the C++
// host mirror (include/netstack/{buffer,header}.hpp) and the HIP engine:
//   tcpip/header/checksum_test.go:26-109   TestChecksumVVWithOffset
//   tcpip/buffer/view_test.go:89-235       CapLength / TrimFront tables
// plus invariants the reference's protocol tests rely on.
// Usage: checksum_test [--cpu-only]   (exit status 0 = all passed)
#include <cstdio>
#include <cstring>
#include <string>
#include <vector>

#include "netstack/buffer.hpp"
#include "netstack/header.hpp"

using netstack::buffer::NewVectorisedView;
using netstack::buffer::NewViewFromBytes;
using netstack::buffer::VectorisedView;
using netstack::buffer::View;
namespace header = netstack::header;

static int g_fail = 0, g_run = 0;
#define EXPECT_EQ(got, want, name)                                                        \
  do {                                                                                    \
    ++g_run;                                                                              \
    auto g__ = (got);                                                                     \
    auto w__ = (want);                                                                    \
    if (!(g__ == w__)) {                                                                  \
      ++g_fail;                                                                           \
      std::printf("FAIL %s:%d %s: got %lld want %lld\n", __FILE__, __LINE__, (name),      \
                  (long long)g__, (long long)w__);                                        \
    }                                                                                     \
  } while (0)

static std::string flat(const VectorisedView& vv) {
  std::string s;
  for (const View& v : vv.Views()) s.append((const char*)v.data(), v.size());
  return s;
}

static VectorisedView vv(size_t size, std::vector<std::string> pieces) {
  // view_test.go:36-43 helper
  std::vector<View> views;
  for (auto& p : pieces) views.push_back(NewViewFromBytes(std::vector<uint8_t>(p.begin(), p.end())));
  return NewVectorisedView(size, views);
}

static void TestCapLength() {  // view_test.go:44-97 (capLengthTestCases)
  struct C {
    const char* name;
    VectorisedView in;
    long long length;
    VectorisedView want;
  } cases[] = {
      {"Simple case", vv(2, {"12"}), 1, vv(1, {"1"})},
      {"Case spanning across two Views", vv(4, {"123", "4"}), 2, vv(2, {"12"})},
      {"Corner case with negative length", vv(1, {"1"}), -1, vv(0, {})},
      {"Corner case with length = 0", vv(3, {"12", "3"}), 0, vv(0, {})},
      {"Corner case with length = size", vv(1, {"1"}), 1, vv(1, {"1"})},
      {"Corner case with length > size", vv(1, {"1"}), 2, vv(1, {"1"})},
  };
  for (auto& c : cases) {
    c.in.CapLength(c.length);
    EXPECT_EQ(c.in.Size(), c.want.Size(), c.name);
    EXPECT_EQ(flat(c.in) == flat(c.want), true, c.name);
    EXPECT_EQ(c.in.Views().size(), c.want.Views().size(), c.name);
  }
}

static void TestTrimFront() {  // view_test.go:99-160 (trimFrontTestCases)
  struct C {
    const char* name;
    VectorisedView in;
    long long count;
    VectorisedView want;
  } cases[] = {
      {"Simple case", vv(2, {"12"}), 1, vv(1, {"2"})},
      {"Case where we trim an entire View", vv(2, {"1", "2"}), 1, vv(1, {"2"})},
      {"Case spanning across two Views", vv(3, {"1", "23"}), 2, vv(1, {"3"})},
      {"Corner case with negative count", vv(1, {"1"}), -1, vv(1, {"1"})},
      {"Corner case with count = 0", vv(1, {"1"}), 0, vv(1, {"1"})},
      {"Corner case with count = size", vv(1, {"1"}), 1, vv(0, {})},
      {"Corner case with count > size", vv(1, {"1"}), 2, vv(0, {})},
  };
  for (auto& c : cases) {
    c.in.TrimFront(c.count);
    EXPECT_EQ(c.in.Size(), c.want.Size(), c.name);
    EXPECT_EQ(flat(c.in) == flat(c.want), true, c.name);
    EXPECT_EQ(c.in.Views().size(), c.want.Views().size(), c.name);
  }
}

static void TestToView() {  // view_test.go:162-190 (toViewCases)
  struct C {
    VectorisedView in;
    std::string want;
  } cases[] = {{vv(2, {"12"}), "12"}, {vv(2, {"1", "2"}), "12"}, {vv(0, {}), ""}};
  for (auto& c : cases) {
    View v = c.in.ToView();
    EXPECT_EQ(std::string((const char*)v.data(), v.size()) == c.want, true, "ToView");
  }
}

static void TestChecksumVVWithOffset() {  // checksum_test.go:26-109
  struct C {
    const char* name;
    VectorisedView vv;
    long long off, size;
    uint16_t initial;
    uint16_t want;
  };
  auto V = [](std::vector<uint8_t> b) { return NewViewFromBytes(std::move(b)); };
  C cases[] = {
      {"empty", NewVectorisedView(0, {V({1, 9, 0, 5, 4})}), 0, 0, 0, 0},
      {"OneView", NewVectorisedView(0, {V({1, 9, 0, 5, 4})}), 0, 5, 0, 1294},
      {"TwoViews", NewVectorisedView(0, {V({1, 9, 0, 5, 4}), V({4, 3, 7, 1, 2, 123})}), 0, 11, 0, 33819},
      {"TwoViewsWithOffset", NewVectorisedView(0, {V({98, 1, 9, 0, 5, 4}), V({4, 3, 7, 1, 2, 123})}), 1,
       11, 0, 33819},
      {"ThreeViewsWithOffset",
       NewVectorisedView(0, {V({98, 1, 9, 0, 5, 4}), V({98, 1, 9, 0, 5, 4}), V({4, 3, 7, 1, 2, 123})}), 7,
       11, 0, 33819},
      {"ThreeViewsWithInitial",
       NewVectorisedView(0, {V({77, 11, 33, 0, 55, 44}), V({98, 1, 9, 0, 5, 4}), V({4, 3, 7, 1, 2, 123, 99})}),
       7, 11, 77, 33896},
  };
  for (auto& tc : cases) {
    EXPECT_EQ(header::ChecksumVVWithOffset(tc.vv, tc.initial, tc.off, tc.size), tc.want, tc.name);
    View v = tc.vv.ToView();
    v.TrimFront((size_t)tc.off);
    v.CapLength((size_t)tc.size);
    EXPECT_EQ(header::Checksum(v, tc.initial), tc.want, tc.name);
  }
}

static void TestInvariants() {
  // IPv4 header with a correct checksum field sums to 0xffff (ipv4_test.go:140-142).
  std::vector<uint8_t> ip = {0x45, 0x00, 0x00, 0x73, 0x00, 0x00, 0x40, 0x00, 0x40, 0x11,
                             0xb8, 0x61, 0xc0, 0xa8, 0x00, 0x01, 0xc0, 0xa8, 0x00, 0xc7};
  EXPECT_EQ(header::Checksum(ip, 0), 0xffff, "ipv4 header");
  // RFC 1071 section 3 example.
  EXPECT_EQ(header::Checksum(std::vector<uint8_t>{0x00, 0x01, 0xf2, 0x03, 0xf4, 0xf5, 0xf6, 0xf7}, 0),
            0xddf2, "rfc1071");
  // uint32 wrap quirk.
  EXPECT_EQ(header::Checksum(std::vector<uint8_t>(200000, 0xff), 0), 0xfffe, "wrap");
  // TCP segment: sender writes ^sum, receiver verifies 0xffff, one corrupted
  // payload byte fails (tcp_test.go:2214-2245, 3246-3254).
  std::string src("\x0a\x00\x00\x01", 4), dst("\x0a\x00\x00\x02", 4);
  std::vector<uint8_t> payload(1000), hdr(20, 0);
  for (size_t i = 0; i < payload.size(); ++i) payload[i] = (uint8_t)i;
  hdr[12] = 5 << 4;
  const uint16_t len = (uint16_t)(hdr.size() + payload.size());
  uint16_t x = header::PseudoHeaderChecksum(6, src, dst, len);
  x = header::Checksum(payload, x);
  x = header::Checksum(hdr, x);
  const uint16_t c = (uint16_t)~x;
  hdr[16] = c >> 8;
  hdr[17] = c & 0xff;
  uint16_t r = header::Checksum(payload, header::Checksum(hdr, header::PseudoHeaderChecksum(6, src, dst, len)));
  EXPECT_EQ(r, 0xffff, "tcp verify");
  payload[0] = 0x4;
  r = header::Checksum(payload, header::Checksum(hdr, header::PseudoHeaderChecksum(6, src, dst, len)));
  EXPECT_EQ(r != 0xffff, true, "tcp corrupt");
  // ChecksumVVBatch == per-segment ChecksumVVWithOffset (sendTCPBatch).
  std::vector<View> views;
  std::vector<uint8_t> seed(9000);
  for (size_t i = 0; i < seed.size(); ++i) seed[i] = (uint8_t)(i * 131 + 7);
  size_t pos = 0;
  for (size_t k : {1000u, 1u, 3333u, 7u, 4659u}) {
    views.push_back(View(seed.data() + pos, k));
    pos += k;
  }
  VectorisedView big = NewVectorisedView(pos, views);
  std::vector<header::SegDesc> segs;
  for (long long off = 0; off < (long long)pos; off += 1460)
    segs.push_back({off, std::min<long long>(1460, (long long)pos - off), (uint16_t)(off * 7)});
  std::vector<uint16_t> got = header::ChecksumVVBatch(big, segs);
  for (size_t i = 0; i < segs.size(); ++i)
    EXPECT_EQ(got[i], header::ChecksumVVWithOffset(big, segs[i].Initial, segs[i].Off, segs[i].Size), "vv batch");
  // Go panics on a negative slice bound; the mirror throws.
  bool threw = false;
  try {
    header::ChecksumVVWithOffset(big, 0, 0, -1);
  } catch (const std::out_of_range&) {
    threw = true;
  }
  EXPECT_EQ(threw, true, "negative size throws");
  EXPECT_EQ(header::ChecksumCombine(0xffff, 1), 1, "combine");
}

static void TestPrependable() {  // prependable.go
  netstack::buffer::Prependable p = netstack::buffer::NewPrependable(10);
  EXPECT_EQ(p.UsedLength(), 0u, "prependable empty");
  std::memcpy(p.Prepend(4), "tcp!", 4);
  std::memcpy(p.Prepend(2), "ip", 2);
  View v = p.View();
  EXPECT_EQ(std::string((const char*)v.data(), v.size()) == "iptcp!", true, "prepend order");
  EXPECT_EQ(p.AvailableLength(), 4u, "available");
  EXPECT_EQ(p.Prepend(5) == nullptr, true, "prepend past the front is nil");
  netstack::buffer::Prependable q = p.DeepCopy();
  q.Data()[0] = 'x';
  EXPECT_EQ(p.View()[0], 'i', "deep copy does not alias");
  p.TrimBack(1);
  EXPECT_EQ(p.UsedLength(), 5u, "trim back");
}

// A TCP/IPv4 packet filled by FillPacketBuffers verifies with
// VerifyPacketBuffers; one corrupted payload byte fails (tcp_test.go:3246-3254).
static void TestPacketBuffers() {
  using netstack::tcpip::PacketBuffer;
  std::vector<uint8_t> payload(2000);
  for (size_t i = 0; i < payload.size(); ++i) payload[i] = (uint8_t)(i * 29 + 1);
  const uint8_t ip[20] = {0x45, 0, 0x08, 0x04, 0, 7, 0, 0, 64, 6, 0, 0, 10, 0, 0, 1, 10, 0, 0, 2};  // 2052 B
  uint8_t tcp[32] = {0, 80, 0x1f, 0x90, 0, 0, 0, 1, 0, 0, 0, 2, 0x80, 0x18, 0xff, 0xff};         // offset 32
  PacketBuffer out;
  out.Header = netstack::buffer::NewPrependable(64);
  std::memcpy(out.Header.Prepend(sizeof tcp), tcp, sizeof tcp);
  std::memcpy(out.Header.Prepend(sizeof ip), ip, sizeof ip);
  out.Data = NewVectorisedView(payload.size(), {View(payload.data(), 777), View(payload.data() + 777, 1223)});
  std::vector<PacketBuffer> tx = {out};
  header::FillPacketBuffers(tx);
  View h = tx[0].Header.View();
  EXPECT_EQ(header::Checksum(h, 0) != 0, true, "filled");
  std::vector<uint8_t> wire(h.data(), h.data() + h.size());
  wire.insert(wire.end(), payload.begin(), payload.end());
  EXPECT_EQ(header::Checksum(std::vector<uint8_t>(wire.begin(), wire.begin() + 20), 0), 0xffff, "ipv4 header");
  std::vector<uint8_t> bad = wire;
  bad[1500] ^= 0x20;
  std::vector<PacketBuffer> rx(2);
  rx[0].Data = NewVectorisedView(wire.size(), {View(wire.data(), 128), View(wire.data() + 128, wire.size() - 128)});
  rx[1].Data = NewVectorisedView(bad.size(), {View(bad.data(), bad.size())});
  std::vector<uint8_t> v = header::VerifyPacketBuffers(rx);
  EXPECT_EQ(v[0], header::PacketChecksumValid, "tcp valid");
  EXPECT_EQ(v[1], header::PacketChecksumInvalid, "tcp corrupted");
}

int main(int argc, char** argv) {
  const bool cpu_only = argc > 1 && std::strcmp(argv[1], "--cpu-only") == 0;
  TestCapLength();
  TestTrimFront();
  TestToView();
  TestPrependable();
  if (!cpu_only) {
    TestChecksumVVWithOffset();
    TestInvariants();
    TestPacketBuffers();
  }
  std::printf("%d checks, %d failed%s\n", g_run, g_fail, cpu_only ? " (cpu-only)" : "");
  return g_fail ? 1 : 0;
}
