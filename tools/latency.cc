// latency.cc — per-call wall latency of the synchronous, reference-shaped
// entry points (the calls a cgo shim makes), on one MI355X:
//   ns_csum_checksum      one 1500-B segment            (header.Checksum)
//   ns_csum_vv_batch      sendTCPBatch: 64 KiB GSO payload, MSS 1460 (45 segs)
//   ns_csum_chains        45 TCP segments: pseudo-header + payload + header
//   ns_csum_batch_host    1024 x 1500 B from host memory
//   concurrency           T threads issuing sendTCPBatch-shaped vv_batch calls
//                         on one context (flat-combined into shared launches)
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
#include <thread>
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
  std::vector<uint8_t> payload(4 << 20);
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
  {  // recvmmsg batches of received IPv4/TCP packets as PacketBuffers (NS_PKB_VERIFY):
     // 1500-B packets in BufConfig views (128+256+256+512+348), valid checksums
    const uint32_t cuts[5] = {128, 256, 256, 512, 348};
    auto be16 = [](uint8_t* p, uint32_t v) { p[0] = (uint8_t)(v >> 8); p[1] = (uint8_t)v; };
    std::printf(" \"packet_buffers_verify\": [");
    const uint32_t counts[] = {8, 64};
    for (int qi = 0; qi < 2; ++qi) {
      const uint32_t n = counts[qi];
      std::vector<uint8_t> pk((size_t)n * 1500);
      std::vector<ns_view> views((size_t)n * 5);
      std::vector<ns_pkt_buf> pb(n);
      for (uint32_t i = 0; i < n; ++i) {
        uint8_t* p = pk.data() + (size_t)i * 1500;
        std::memcpy(p + 40, payload.data() + (size_t)i * 1460, 1460);
        const uint8_t ip[20] = {0x45, 0, 0x05, 0xDC, (uint8_t)(i >> 8), (uint8_t)i, 0x40, 0, 64, 6, 0, 0,
                                10, 0, 0, 1, 10, 0, 0, 2};
        std::memcpy(p, ip, 20);
        be16(p + 10, ~scalar(p, 20, 0) & 0xFFFF);
        uint8_t* t = p + 20;
        std::memset(t, 0, 20);
        be16(t, 40000 + i);
        be16(t + 2, 443);
        t[12] = 5 << 4;
        t[13] = 0x10;
        be16(t + 14, 65535);
        const uint8_t ph[12] = {10, 0, 0, 1, 10, 0, 0, 2, 0, 6, 0x05, 0xC8};  // pseudo-header, length 1480
        uint16_t x = scalar(ph, 12, 0);
        x = scalar(t, 20, x);
        x = scalar(p + 40, 1460, x);
        be16(t + 16, ~x & 0xFFFF);
        uint32_t o = 0;
        for (int k = 0; k < 5; ++k) {
          views[(size_t)i * 5 + k] = ns_view{p + o, cuts[k]};
          o += cuts[k];
        }
        pb[i] = ns_pkt_buf{nullptr, 0, &views[(size_t)i * 5], 5, 0, 1500};
      }
      std::vector<uint8_t> verdict(n);
      check(ns_csum_packet_buffers(ctx, pb.data(), n, NS_PKB_VERIFY, nullptr, verdict.data()), "packet_buffers");
      uint32_t valid = 0;
      for (uint8_t v : verdict) valid += v == NS_PKB_VALID;
      const Stat g = time_calls(std::max(20, iters / 2), [&] {
        check(ns_csum_packet_buffers(ctx, pb.data(), n, NS_PKB_VERIFY, nullptr, verdict.data()), "packet_buffers");
      });
      std::printf("%s{\"packets\": %u, \"gpu_med_us\": %.2f, \"gpu_p99_us\": %.2f, \"valid\": %u}", qi ? ", " : "",
                  n, g.med, g.p99, valid);
    }
    std::printf("],\n");
  }
  {  // host batches of growing size: zero-copy below kStageBytes (1 MiB), DMA above
    std::printf(" \"batch_host_sizes\": [");
    const uint32_t ns[] = {43, 170, 680, 2720};
    for (int qi = 0; qi < 4; ++qi) {
      const uint32_t n = ns[qi];
      std::vector<ns_pkt_desc> d(n);
      for (uint32_t i = 0; i < n; ++i) d[i] = ns_pkt_desc{(uint64_t)i * 1504, 1500, (uint16_t)i, 0};
      std::vector<uint16_t> out(n);
      const Stat g = time_calls(std::max(20, iters / 8), [&] {
        check(ns_csum_batch_host(ctx, payload.data(), (uint64_t)n * 1504, d.data(), n, out.data(), 0), "batch_host");
      });
      std::printf("%s{\"packets\": %u, \"bytes\": %u, \"gpu_med_us\": %.2f, \"GBps\": %.2f}", qi ? ", " : "", n,
                  n * 1504, g.med, n * 1504 / g.med / 1e3);
    }
    std::printf("],\n");
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
    std::printf(" \"batch_host_1024x1500B\": {\"gpu_med_us\": %.2f, \"gpu_p99_us\": %.2f, \"scalar_med_us\": %.3f},\n",
                g.med, g.p99, c.med);
  }
  {  // large gathers: one VectorisedView batch of 64 MiB in 1 MiB views, 64 KiB segments
    const uint64_t total = 64ull << 20, vsz = 1ull << 20;
    std::vector<uint8_t> big(total);
    for (size_t i = 0; i < big.size(); ++i) big[i] = (uint8_t)(i * 2654435761u >> 11);
    std::vector<ns_view> views;
    for (uint64_t o = 0; o < total; o += vsz) views.push_back(ns_view{big.data() + o, vsz});
    std::vector<ns_seg> segs;
    for (uint64_t o = 0; o < total; o += 65536) segs.push_back(ns_seg{(int64_t)o, 65536, 0x77, 0, 0});
    std::vector<uint16_t> out(segs.size());
    const Stat g = time_calls(20, [&] {
      check(ns_csum_vv_batch(ctx, views.data(), (uint32_t)views.size(), segs.data(), (uint32_t)segs.size(),
                             out.data()), "vv_batch");
    });
    bool ok = true;
    for (size_t k = 0; k < segs.size(); k += 97) ok = ok && out[k] == scalar(big.data() + segs[k].off, 65536, 0x77);
    std::printf(" \"vv_batch_64MiB_1024segs\": {\"gpu_med_us\": %.1f, \"GBps\": %.2f, \"ok\": %s},\n", g.med,
                total / g.med / 1e3, ok ? "true" : "false");
  }
  {  // T threads x sendTCPBatch calls on one context
    const int mss = 1460, total = 65536;
    std::vector<ns_seg> segs;
    for (int off = 0; off < total; off += mss) segs.push_back(ns_seg{off, std::min(mss, total - off), 0, 0, 0});
    std::vector<uint16_t> want(segs.size());
    ns_view v0{payload.data(), (uint64_t)total};
    check(ns_csum_vv_batch(ctx, &v0, 1, segs.data(), (uint32_t)segs.size(), want.data()), "vv_batch");
    std::printf(" \"concurrent_vv_batch_64KiB\": [");
    const int threads[] = {1, 2, 4, 8, 16, 32};
    for (int ti = 0; ti < 6; ++ti) {
      const int T = threads[ti], per = std::max(20, iters / 8);
      std::vector<std::thread> th;
      std::vector<int> bad(T, 0);
      const double a = now_us();
      for (int t = 0; t < T; ++t)
        th.emplace_back([&, t] {
          // each thread its own payload window (distinct bytes, same shape)
          ns_view v{payload.data() + 4096 * (t % 64), (uint64_t)total};
          std::vector<ns_seg> sg = segs;
          for (auto& x : sg) x.initial = (uint16_t)t;
          std::vector<uint16_t> out(sg.size());
          std::vector<uint16_t> ref(sg.size());
          for (size_t k = 0; k < sg.size(); ++k)
            ref[k] = scalar(payload.data() + 4096 * (t % 64) + sg[k].off, (size_t)sg[k].size, (uint16_t)t);
          for (int i = 0; i < per; ++i) {
            check(ns_csum_vv_batch(ctx, &v, 1, sg.data(), (uint32_t)sg.size(), out.data()), "vv_batch");
            bad[t] += out != ref;  // every call checked (a vector compare, not a re-sum)
          }
        });
      for (auto& x : th) x.join();
      const double el = now_us() - a;
      int nbad = 0;
      for (int b : bad) nbad += b;
      const double calls = (double)T * per;
      std::printf("%s{\"threads\": %d, \"calls_per_s\": %.0f, \"payload_GiBps\": %.3f, \"us_per_call_per_thread\": %.2f, \"wrong\": %d}",
                  ti ? ", " : "", T, calls / el * 1e6, calls * total / el * 1e6 / (1 << 30), el / per, nbad);
    }
    std::printf("]\n");
  }
  std::printf("}\n");
  ns_csum_destroy(ctx);
  return sink == 0xFFFFFFFFu;
}
