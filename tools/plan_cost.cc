// plan_cost.cc — host time of ns_csum_packet_buffers' planning, without the
// GPU: what csum_api.cpp does per call around the device pass (PacketBytes
// per packet, the chain builder over a copying sink, plan_packet,
// finish_packet), over recvmmsg-shaped batches of 1500-B IPv4/TCP packets in
// BufConfig views.  CPU only; links nothing but host_logic.h.
//   make -C netstack_amd/csrc  ->  netstack_amd/lib/plan_cost
#include <algorithm>
#include <chrono>
#include <cstdio>
#include <cstring>
#include <vector>

#include "host_logic.h"

namespace {

struct FlatSink {  // a preallocated staging buffer, as the leased gather stage is
  std::vector<uint8_t> a;
  uint64_t n = 0;
  uint64_t append(const uint8_t* p, uint64_t len) {
    const uint64_t at = n;
    std::memcpy(a.data() + n, p, len);
    n += len;
    return at;
  }
};

double now_us() {
  return std::chrono::duration<double, std::micro>(std::chrono::steady_clock::now().time_since_epoch()).count();
}

}  // namespace

int main() {
  const uint32_t cuts[5] = {128, 256, 256, 512, 348};
  for (uint32_t n : {8u, 64u, 256u, 2048u}) {
    std::vector<uint8_t> pk((size_t)n * 1500);
    for (size_t i = 0; i < pk.size(); ++i) pk[i] = (uint8_t)(i * 2654435761u >> 13);
    std::vector<ns_view> views((size_t)n * 5);
    std::vector<ns_pkt_buf> pkts(n);
    for (uint32_t i = 0; i < n; ++i) {
      uint8_t* p = pk.data() + (size_t)i * 1500;
      const uint8_t ip[20] = {0x45, 0, 0x05, 0xDC, 0, 0, 0x40, 0, 64, 6, 0, 0, 10, 0, 0, 1, 10, 0, 0, 2};
      std::memcpy(p, ip, 20);
      p[32] = 0x50;
      uint32_t o = 0;
      for (int k = 0; k < 5; ++k) {
        views[(size_t)i * 5 + k] = ns_view{p + o, cuts[k]};
        o += cuts[k];
      }
      pkts[i] = ns_pkt_buf{nullptr, 0, &views[(size_t)i * 5], 5, 0, 1500};
    }
    FlatSink sink;
    sink.a.resize((size_t)n * 1600 + 4096);
    std::vector<uint8_t> verdict(n);
    const int reps = std::max(50, 200000 / (int)n);
    double best = 1e30;
    for (int r = 0; r < 5; ++r) {
      const double t0 = now_us();
      for (int q = 0; q < reps; ++q) {
        sink.n = 0;
        std::vector<nsh::PacketBytes> pb(n);
        for (uint32_t i = 0; i < n; ++i) pb[i].init(pkts[i]);
        nsh::ChainBuilder<FlatSink> gt(sink);
        gt.desc.reserve((size_t)n * 4);
        gt.result_at.reserve((size_t)n * 2);
        std::vector<nsh::PacketPlan> plan(n);
        for (uint32_t i = 0; i < n; ++i) nsh::plan_packet(gt, pb[i], NS_PKB_VERIFY, &plan[i]);
        std::vector<uint16_t> res(gt.result_at.size(), 0xFFFF);
        for (uint32_t i = 0; i < n; ++i) nsh::finish_packet(pb[i], plan[i], NS_PKB_VERIFY, res.data(), nullptr, &verdict[i]);
      }
      best = std::min(best, (now_us() - t0) / reps);
    }
    // for scale: the reference's own verify loop over the same bytes (2 B per
    // iteration, as calculateChecksum; segment.parse's pseudo-header + segment)
    double cbest = 1e30;
    volatile uint32_t keep = 0;
    for (int r = 0; r < 5; ++r) {
      const double t0 = now_us();
      for (int q = 0; q < reps; ++q)
        for (uint32_t i = 0; i < n; ++i) {
          const uint8_t* b = pk.data() + (size_t)i * 1500 + 20;
          uint32_t v = 0x1234;
          for (int j = 0; j < 1480; j += 2) {
            v += ((uint32_t)b[j] << 8) + b[j + 1];
            __asm__ volatile("" : "+r"(v));  // keep it scalar, as Go emits it
          }
          keep += v;
        }
      cbest = std::min(cbest, (now_us() - t0) / reps);
    }
    std::printf("packets %5u: plan %.2f us per call (%.1f ns per packet), scalar verify %.2f us; %zu bytes staged\n",
                n, best, best * 1e3 / n, cbest, (size_t)sink.n);
  }
  return 0;
}
