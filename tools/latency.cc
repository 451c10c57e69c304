// latency.cc — per-call wall latency of the synchronous, reference-shaped
// entry points (the calls a cgo shim makes), on one MI355X:
//   ns_csum_checksum      one 1500-B segment            (header.Checksum)
//   ns_csum_vv_batch      sendTCPBatch: 64 KiB GSO payload, MSS 1460 (45 segs)
//   ns_csum_chains        45 TCP segments: pseudo-header + payload + header
//   ns_csum_batch_host    1024 x 1500 B from pinned host memory
// Median and p99 over many calls after warm-up; a scalar 2-B/iteration loop
// (checksum.go:41-43) on the same bytes is timed beside each for scale.
//   ./latency [iters]
#include <algorithm>
#include <chrono>
#include <cstdint>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <functional>
#include <vector>

#include "netstack_csum.h"

namespace {

double now_us() {
  return std::chrono::duration<double, std::micro>(std::chrono::steady_clock::now().time_since_epoch()).count();
}

struct Stat {
  double med, p99;
};

Stat time_calls(int iters, const std::function<void()>& f) {
  for (int i = 0; i < 50; ++i) f();
  std::vector<double> t(iters);
  for (int i = 0; i < iters; ++i) {
    const double a = now_us();
    f();
    t[i] = now_us() - a;
  }
  std::sort(t.begin(), t.end());
  return {t[iters / 2], t[(size_t)(iters * 0.99)]};
}

// The scalar loop of checksum.go:26-46, for scale only.
uint16_t scalar(const uint8_t* b, size_t n, uint32_t v) {
  for (size_t i = 0; i + 1 < n; i += 2) v += ((uint32_t)b[i] << 8) | b[i + 1];
  if (n & 1) v += (uint32_t)b[n - 1] << 8;
  v = (v & 0xFFFF) + (v >> 16);
  return (uint16_t)(v + (v >> 16));
}

void check(int rc, const char* what) {
  if (rc != NS_OK) {
    std::fprintf(stderr, "%s: %s\n", what, ns_csum_strerror(rc));
    std::exit(1);
  }
}

}  // namespace

int main(int argc, char** argv) {
  const int iters = argc > 1 ? std::atoi(argv[1]) : 2000;
  ns_csum_ctx* ctx = nullptr;
  check(ns_csum_init(nullptr, &ctx), "init");
  std::vector<uint8_t> payload(1 << 20);
  for (size_t i = 0; i < payload.size(); ++i) payload[i] = (uint8_t)(i * 2654435761u >> 13);
  volatile uint32_t sink = 0;
  std::printf("{\n");

  {  // header.Checksum of one MTU payload
    uint16_t r = 0;
    const Stat g = time_calls(iters, [&] { check(ns_csum_checksum(ctx, payload.data(), 1500, 0x1234, &r), "checksum"); });
    const Stat c = time_calls(iters, [&] { sink += scalar(payload.data(), 1500, 0x1234); });
    std::printf(" \"checksum_1500B\": {\"gpu_med_us\": %.2f, \"gpu_p99_us\": %.2f, \"scalar_med_us\": %.3f},\n",
                g.med, g.p99, c.med);
  }
  {  // sendTCPBatch: 64 KiB payload in one view, 45 MSS segments
    const int mss = 1460, total = 65536;
    ns_view v{payload.data(), (uint64_t)total};
    std::vector<ns_seg> segs;
    for (int off = 0; off < total; off += mss) segs.push_back(ns_seg{off, std::min(mss, total - off), 0x4321, 0, 0});
    std::vector<uint16_t> out(segs.size());
    const Stat g = time_calls(iters, [&] {
      check(ns_csum_vv_batch(ctx, &v, 1, segs.data(), (uint32_t)segs.size(), out.data()), "vv_batch");
    });
    const Stat c = time_calls(iters, [&] {
      for (const auto& s : segs) sink += scalar(payload.data() + s.off, (size_t)s.size, s.initial);
    });
    std::printf(" \"vv_batch_64KiB_45segs\": {\"gpu_med_us\": %.2f, \"gpu_p99_us\": %.2f, \"scalar_med_us\": %.3f},\n",
                g.med, g.p99, c.med);
  }
  {  // 45 TCP segments as chains: pseudo-header fields, payload, 20-B header
    const int mss = 1460, total = 65536;
    uint8_t ph[12] = {10, 0, 0, 1, 10, 0, 0, 2, 0, 6, 0, 0};
    uint8_t hdr[20] = {0};
    std::vector<ns_piece> pcs;
    int nseg = 0;
    for (int off = 0; off < total; off += mss, ++nseg) {
      pcs.push_back(ns_piece{ph, 12, 0, NS_PIECE_RESTART, 0});
      pcs.push_back(ns_piece{payload.data() + off, (uint64_t)std::min(mss, total - off), 0, NS_PIECE_RESTART, 0});
      pcs.push_back(ns_piece{hdr, 20, 0, NS_PIECE_RESTART | NS_PIECE_END, 0});
    }
    std::vector<uint16_t> out(nseg);
    const Stat g = time_calls(iters, [&] {
      check(ns_csum_chains(ctx, pcs.data(), (uint32_t)pcs.size(), out.data(), (uint32_t)nseg), "chains");
    });
    std::printf(" \"chains_45_tcp_segments\": {\"gpu_med_us\": %.2f, \"gpu_p99_us\": %.2f},\n", g.med, g.p99);
  }
  {  // 1024 x 1500 B from host memory
    const uint32_t n = 1024;
    std::vector<ns_pkt_desc> d(n);
    for (uint32_t i = 0; i < n; ++i) d[i] = ns_pkt_desc{(uint64_t)i * 1504, 1500, (uint16_t)i, 0};
    std::vector<uint16_t> out(n);
    const Stat g = time_calls(iters / 4, [&] {
      check(ns_csum_batch_host(ctx, payload.data(), (uint64_t)n * 1504, d.data(), n, out.data(), 0), "batch_host");
    });
    const Stat c = time_calls(iters / 4, [&] {
      for (uint32_t i = 0; i < n; ++i) sink += scalar(payload.data() + d[i].off, 1500, d[i].initial);
    });
    std::printf(" \"batch_host_1024x1500B\": {\"gpu_med_us\": %.2f, \"gpu_p99_us\": %.2f, \"scalar_med_us\": %.3f}\n",
                g.med, g.p99, c.med);
  }
  std::printf("}\n");
  ns_csum_destroy(ctx);
  return sink == 0xFFFFFFFFu;
}
