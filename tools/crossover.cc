// crossover.cc — where a synchronous engine call starts to beat one CPU core
// doing the reference's own loop (checksum.go:26-46) on the same bytes.  The
// Go callers (go/transport/tcp/csum_batch_hip.go, go/link/fdbased/
// csum_rx_hip.go) offload only calls above the sizes this reports; below
// them the default build's Go code runs ("When offload
// pays").
//
// Per call shape, per size: the median wall time of the engine call (the
// caller's thread is busy for all of it: it copies the views into staging
// and spins on the completion word) and of the scalar loop doing what the
// reference does for the same call, on one core:
//   checksum      header.Checksum(buf)                       one buffer
//   vv_batch      ChecksumVVWithOffset per MSS segment         sendTCPBatch payload
//   chains        pseudo-header + payload + TCP header chains  finishTCPBatchChecksums
//   verify        segment.parse's check per received packet    recvmmsg batch (VerifyPacketBuffers)
//   verify_ring_host  the same packets copied into a 1504-B-stride ring
//                 stage, parsed on the device (ns_csum_rx_ring_host)
//   tx_host       K sendTCPBatch calls of 64 KiB (45 segments, 54-B slots),
//                 both fields of every segment (FillTCPBatches: the calls
//                 copied into an engine stage, ns_csum_tcp_tx_host, the slots
//                 copied back) against buildTCPHdr + addIPHeader per segment
// The scalar loop is compiled without auto-vectorisation, as the Go compiler
// emits it.  Output: one JSON object; "crossover" is the smallest size from
// which the engine is faster at every larger size measured (null if never).
//   ./crossover [iters]
#include <algorithm>
#include <chrono>
#include <cstdint>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <functional>
#include <string>
#include <vector>

#include "netstack_csum.h"

namespace {

double now_us() {
  return std::chrono::duration<double, std::micro>(std::chrono::steady_clock::now().time_since_epoch()).count();
}

double median_us(int iters, const std::function<void()>& f) {
  for (int i = 0; i < std::max(5, iters / 10); ++i) f();
  std::vector<double> t(iters);
  for (int i = 0; i < iters; ++i) {
    const double a = now_us();
    f();
    t[i] = now_us() - a;
  }
  std::sort(t.begin(), t.end());
  return t[iters / 2];
}

// calculateChecksum (checksum.go:26-46): 2 bytes per iteration, never folded
// inside the loop; returns the folded sum and the odd carry.
__attribute__((noinline, optimize("no-tree-vectorize"))) uint16_t go_sum(const uint8_t* b, size_t n, bool odd,
                                                                           uint32_t v, bool* odd_out) {
  if (odd && n) {
    v += b[0];
    ++b;
    --n;
  }
  size_t l = n;
  const bool o = (l & 1) != 0;
  if (o) {
    --l;
    v += (uint32_t)b[l] << 8;
  }
  for (size_t i = 0; i < l; i += 2) v += ((uint32_t)b[i] << 8) + b[i + 1];
  if (odd_out) *odd_out = o;
  v = (v & 0xFFFF) + (v >> 16);
  return (uint16_t)(v + (v >> 16));
}

// ChecksumVVWithOffset over views (checksum.go:69-98).
uint16_t go_vv(const std::pair<const uint8_t*, size_t>* views, int nviews, uint16_t initial) {
  bool odd = false;
  uint16_t x = initial;
  for (int k = 0; k < nviews; ++k) x = go_sum(views[k].first, views[k].second, odd, x, &odd);
  return x;
}

void check(int rc, const char* what) {
  if (rc != NS_OK) {
    std::fprintf(stderr, "%s: %s\n", what, ns_csum_strerror(rc));
    std::exit(1);
  }
}

volatile uint32_t g_sink = 0;

struct Point {
  uint64_t size;  // bytes (or packets, for verify)
  uint64_t bytes;
  double gpu_us, cpu_us;
};

void emit(const char* name, const char* unit, const std::vector<Point>& pts, bool last) {
  // crossover: smallest size from which gpu < cpu at every larger size
  long x = -1;
  for (long i = (long)pts.size() - 1; i >= 0 && pts[i].gpu_us < pts[i].cpu_us; --i) x = i;
  std::printf(" \"%s\": {\"unit\": \"%s\", \"points\": [", name, unit);
  for (size_t i = 0; i < pts.size(); ++i)
    std::printf("%s{\"%s\": %llu, \"bytes\": %llu, \"gpu_med_us\": %.2f, \"cpu_1core_med_us\": %.2f, \"gpu_over_cpu\": %.3f}",
                i ? ", " : "", unit, (unsigned long long)pts[i].size, (unsigned long long)pts[i].bytes,
                pts[i].gpu_us, pts[i].cpu_us, pts[i].gpu_us / pts[i].cpu_us);
  if (x < 0)
    std::printf("], \"crossover\": null}%s\n", last ? "" : ",");
  else
    std::printf("], \"crossover\": {\"%s\": %llu, \"bytes\": %llu}}%s\n", unit, (unsigned long long)pts[x].size,
                (unsigned long long)pts[x].bytes, last ? "" : ",");
}

}  // namespace

int main(int argc, char** argv) {
  const int iters = argc > 1 ? std::atoi(argv[1]) : 400;
  ns_csum_ctx* ctx = nullptr;
  check(ns_csum_init(nullptr, &ctx), "init");
  std::vector<uint8_t> payload(8 << 20);
  for (size_t i = 0; i < payload.size(); ++i) payload[i] = (uint8_t)(i * 2654435761u >> 13);
  const uint64_t sizes[] = {4096, 8192, 16384, 32768, 65536, 131072, 262144, 524288, 1u << 20, 2u << 20, 4u << 20};
  std::printf("{\n");

  {  // header.Checksum of one buffer
    std::vector<Point> pts;
    for (uint64_t n : sizes) {
      uint16_t r = 0;
      const double g = median_us(iters, [&] { check(ns_csum_checksum(ctx, payload.data(), n, 0x1234, &r), "checksum"); });
      if (r != go_sum(payload.data(), n, false, 0x1234, nullptr)) check(NS_EHIP, "checksum parity");
      const double c = median_us(iters, [&] { g_sink += go_sum(payload.data(), n, false, 0x1234, nullptr); });
      pts.push_back({n, n, g, c});
    }
    emit("checksum", "bytes", pts, false);
  }
  const int mss = 1460;
  {  // sendTCPBatch's payload: one view, MSS segments, ChecksumVVWithOffset each
    std::vector<Point> pts;
    for (uint64_t n : sizes) {
      ns_view v{payload.data(), n};
      std::vector<ns_seg> segs;
      for (uint64_t off = 0; off < n; off += mss)
        segs.push_back(ns_seg{(int64_t)off, (int64_t)std::min<uint64_t>(mss, n - off), 0x4321, 0, 0});
      std::vector<uint16_t> out(segs.size());
      const double g = median_us(iters, [&] {
        check(ns_csum_vv_batch(ctx, &v, 1, segs.data(), (uint32_t)segs.size(), out.data()), "vv_batch");
      });
      for (size_t k = 0; k < segs.size(); ++k)
        if (out[k] != go_sum(payload.data() + segs[k].off, (size_t)segs[k].size, false, 0x4321, nullptr))
          check(NS_EHIP, "vv_batch parity");
      const double c = median_us(iters, [&] {
        for (const auto& s : segs) g_sink += go_sum(payload.data() + s.off, (size_t)s.size, false, s.initial, nullptr);
      });
      pts.push_back({n, n, g, c});
    }
    emit("vv_batch", "bytes", pts, false);
  }
  {  // finishTCPBatchChecksums: per segment, pseudo-header sum, payload, 20-B header
    std::vector<Point> pts;
    uint8_t ph[12] = {10, 0, 0, 1, 10, 0, 0, 2, 0, 6, 0x05, 0xC8};
    uint8_t hdr[20] = {0x9C, 0x40, 0x01, 0xBB, 0, 0, 0, 1, 0, 0, 0, 2, 0x50, 0x10, 0xFF, 0xFF, 0, 0, 0, 0};
    for (uint64_t n : sizes) {
      std::vector<ns_piece> pcs;
      uint32_t nseg = 0;
      for (uint64_t off = 0; off < n; off += mss, ++nseg) {
        pcs.push_back(ns_piece{ph, 12, 0, NS_PIECE_RESTART, 0});
        pcs.push_back(ns_piece{payload.data() + off, std::min<uint64_t>(mss, n - off), 0, NS_PIECE_RESTART, 0});
        pcs.push_back(ns_piece{hdr, 20, 0, NS_PIECE_RESTART | NS_PIECE_END, 0});
      }
      std::vector<uint16_t> out(nseg);
      const double g = median_us(iters, [&] {
        check(ns_csum_chains(ctx, pcs.data(), (uint32_t)pcs.size(), out.data(), nseg), "chains");
      });
      auto cpu = [&](uint32_t k) {
        uint16_t x = go_sum(ph, 12, false, 0, nullptr);  // Route.PseudoHeaderChecksum
        x = go_sum(pcs[3 * k + 1].data, pcs[3 * k + 1].len, false, x, nullptr);  // ChecksumVVWithOffset
        return go_sum(hdr, 20, false, x, nullptr);  // tcp.CalculateChecksum
      };
      for (uint32_t k = 0; k < nseg; ++k)
        if (out[k] != cpu(k)) check(NS_EHIP, "chains parity");
      const double c = median_us(iters, [&] {
        for (uint32_t k = 0; k < nseg; ++k) g_sink += cpu(k);
      });
      pts.push_back({n, n, g, c});
    }
    emit("chains", "bytes", pts, false);
  }
  {  // recvmmsg batches of received 1500-B IPv4/TCP packets in BufConfig views
    const uint32_t cuts[5] = {128, 256, 256, 512, 348};
    auto be16 = [](uint8_t* p, uint32_t v) {
      p[0] = (uint8_t)(v >> 8);
      p[1] = (uint8_t)v;
    };
    std::vector<Point> pts, rpts;
    const uint32_t counts[] = {1, 2, 4, 8, 16, 32, 64, 128, 256, 512, 1024, 2048};
    for (uint32_t n : counts) {
      std::vector<uint8_t> pk((size_t)n * 1500);
      std::vector<ns_view> views((size_t)n * 5);
      std::vector<ns_pkt_buf> pb(n);
      for (uint32_t i = 0; i < n; ++i) {
        uint8_t* p = pk.data() + (size_t)i * 1500;
        std::memcpy(p + 40, payload.data() + (size_t)i * 1460, 1460);
        const uint8_t ip[20] = {0x45, 0, 0x05, 0xDC, (uint8_t)(i >> 8), (uint8_t)i, 0x40, 0, 64, 6, 0, 0,
                                10, 0, 0, 1, 10, 0, 0, 2};
        std::memcpy(p, ip, 20);
        be16(p + 10, ~go_sum(p, 20, false, 0, nullptr) & 0xFFFF);
        uint8_t* t = p + 20;
        std::memset(t, 0, 20);
        be16(t, 40000 + (i & 0x3FFF));
        be16(t + 2, 443);
        t[12] = 5 << 4;
        t[13] = 0x10;
        be16(t + 14, 65535);
        const uint8_t ph[12] = {10, 0, 0, 1, 10, 0, 0, 2, 0, 6, 0x05, 0xC8};
        uint16_t x = go_sum(ph, 12, false, 0, nullptr);
        x = go_sum(t, 20, false, x, nullptr);
        x = go_sum(p + 40, 1460, false, x, nullptr);
        be16(t + 16, ~x & 0xFFFF);
        uint32_t o = 0;
        for (int k = 0; k < 5; ++k) {
          views[(size_t)i * 5 + k] = ns_view{p + o, cuts[k]};
          o += cuts[k];
        }
        pb[i] = ns_pkt_buf{nullptr, 0, &views[(size_t)i * 5], 5, 0, 1500};
      }
      std::vector<uint8_t> verdict(n);
      const double g = median_us(std::max(20, iters / 2), [&] {
        check(ns_csum_packet_buffers(ctx, pb.data(), n, NS_PKB_VERIFY, nullptr, verdict.data()), "packet_buffers");
      });
      for (uint8_t v : verdict)
        if (v != NS_PKB_VALID) check(NS_EHIP, "verify parity");
      // segment.parse per packet (segment.go:174-180): the pseudo-header sum
      // (route.go:93-95), then ChecksumVV over the segment's views past the
      // 20-B IP header, == 0xffff.
      const double c = median_us(std::max(20, iters / 2), [&] {
        uint32_t ok = 0;
        for (uint32_t i = 0; i < n; ++i) {
          const uint8_t* p = pk.data() + (size_t)i * 1500;
          const uint8_t ph[12] = {p[12], p[13], p[14], p[15], p[16], p[17], p[18], p[19], 0, 6, 0x05, 0xC8};
          std::pair<const uint8_t*, size_t> vs[5] = {{p + 20, cuts[0] - 20}};
          uint32_t o = cuts[0];
          for (int k = 1; k < 5; ++k) {
            vs[k] = {p + o, cuts[k]};
            o += cuts[k];
          }
          ok += go_vv(vs, 5, go_sum(ph, 12, false, 0, nullptr)) == 0xFFFF;
        }
        g_sink += ok;
      });
      pts.push_back({n, (uint64_t)n * 1500, g, c});
      // the same packets as a receive ring in an engine stage: each packet's
      // views copied into its 1504-B slot (what a caller does with recvmmsg's
      // buffers), then ns_csum_rx_ring_host parses and verifies them on the
      // device, no host planning
      uint8_t* stage = nullptr;
      check(ns_csum_stage_acquire(ctx, (uint64_t)n * 1504, &stage), "stage_acquire");
      std::vector<uint32_t> lens(n, 1500);
      std::vector<uint8_t> rv(n);
      const ns_rx_ring ring{0, 1504, n, 0, 0, 128, 0};
      const double gr = median_us(std::max(20, iters / 2), [&] {
        for (uint32_t i = 0; i < n; ++i) {
          uint8_t* dst = stage + (size_t)i * 1504;
          for (int k = 0; k < 5; ++k) {
            const ns_view& v = views[(size_t)i * 5 + k];
            std::memcpy(dst, v.data, v.len);
            dst += v.len;
          }
        }
        check(ns_csum_rx_ring_host(ctx, stage, (uint64_t)n * 1504, &ring, lens.data(), nullptr, rv.data()),
              "rx_ring_host");
      });
      for (uint8_t v : rv)
        if (v != NS_PKB_VALID) check(NS_EHIP, "ring verify parity");
      check(ns_csum_stage_release(ctx, stage), "stage_release");
      rpts.push_back({n, (uint64_t)n * 1500, gr, c});
    }
    emit("verify", "packets", pts, false);
    emit("verify_ring_host", "packets", rpts, false);
  }
  {  // FillTCPBatches: K connections' 64 KiB sendTCPBatch calls in one engine call
    const uint32_t slot = 54, ip_at = 14, tcp_at = 34, seg = 45, csize = 65536;
    const uint32_t per = seg * slot + csize;  // one call's slots, then its payload
    auto be16 = [](uint8_t* p, uint32_t v) {
      p[0] = (uint8_t)(v >> 8);
      p[1] = (uint8_t)v;
    };
    const uint8_t src[4] = {10, 0, 0, 1}, dst[4] = {10, 0, 0, 2};
    const uint16_t addr_sum = go_sum(dst, 4, false, go_sum(src, 4, false, 0, nullptr), nullptr);
    std::vector<Point> pts;
    const uint32_t counts[] = {1, 2, 4, 8, 16, 32, 64, 128, 256, 512, 1024};
    for (uint32_t k : counts) {
      // the callers' memory: K calls side by side, fresh headers (fields 0)
      std::vector<uint8_t> mem((size_t)k * per);
      for (uint32_t c = 0; c < k; ++c) {
        uint8_t* base = mem.data() + (size_t)c * per;
        for (uint32_t i = 0; i < seg; ++i) {
          uint8_t* s = base + i * slot;
          std::memset(s, 0, slot);
          const uint8_t ip[20] = {0x45, 0, 0x05, 0xDC, (uint8_t)(c >> 8), (uint8_t)c, 0x40, 0, 64, 6, 0, 0,
                                  10, 0, 0, 1, 10, 0, 0, 2};
          std::memcpy(s + ip_at, ip, 20);
          be16(s + tcp_at, 40000 + (c & 0x3FFF));
          be16(s + tcp_at + 2, 443);
          be16(s + tcp_at + 4, i);
          s[tcp_at + 12] = 5 << 4;
          s[tcp_at + 13] = 0x10;
          be16(s + tcp_at + 14, 65535);
        }
        std::memcpy(base + seg * slot, payload.data() + (size_t)(c % 64) * 4096, csize);
      }
      std::vector<ns_tcp_tx> txs(k);
      for (uint32_t c = 0; c < k; ++c)
        txs[c] = ns_tcp_tx{(uint64_t)c * per, (uint64_t)c * per + seg * slot, csize, 1460, slot, ip_at, 20, tcp_at, 20,
                           addr_sum, 6, 0};
      uint8_t* stage = nullptr;
      check(ns_csum_stage_acquire(ctx, mem.size(), &stage), "stage_acquire");
      const double g = median_us(std::max(20, iters / 4), [&] {
        for (uint32_t c = 0; c < k; ++c)  // the shim packs each call into the stage
          std::memcpy(stage + (size_t)c * per, mem.data() + (size_t)c * per, per);
        check(ns_csum_tcp_tx_host(ctx, stage, mem.size(), txs.data(), k, nullptr), "tcp_tx_host");
        for (uint32_t c = 0; c < k; ++c)  // and copies the slots back
          std::memcpy(mem.data() + (size_t)c * per, stage + (size_t)c * per, seg * slot);
      });
      // buildTCPHdr (connect.go:652-663) and addIPHeader (ipv4.go:236) per
      // segment, on the callers' memory
      auto cpu = [&](uint8_t* m) {
        for (uint32_t c = 0; c < k; ++c) {
          uint8_t* base = m + (size_t)c * per;
          for (uint32_t i = 0; i < seg; ++i) {
            uint8_t* s = base + i * slot;
            const uint32_t len = std::min<uint32_t>(1460, csize - i * 1460);
            s[tcp_at + 16] = s[tcp_at + 17] = 0;
            const uint8_t lw[4] = {0, 6, (uint8_t)((20 + len) >> 8), (uint8_t)(20 + len)};
            uint16_t x = go_sum(lw, 4, false, addr_sum, nullptr);  // PseudoHeaderChecksum
            x = go_sum(base + seg * slot + i * 1460, len, false, x, nullptr);  // ChecksumVVWithOffset
            be16(s + tcp_at + 16, ~go_sum(s + tcp_at, 20, false, x, nullptr) & 0xFFFF);
            s[ip_at + 10] = s[ip_at + 11] = 0;
            be16(s + ip_at + 10, ~go_sum(s + ip_at, 20, false, 0, nullptr) & 0xFFFF);
          }
        }
      };
      std::vector<uint8_t> ref = mem;
      cpu(ref.data());
      if (ref != mem) check(NS_EHIP, "tx_host parity");
      const double c = median_us(std::max(20, iters / 4), [&] { cpu(ref.data()); });
      check(ns_csum_stage_release(ctx, stage), "stage_release");
      pts.push_back({k, (uint64_t)k * csize, g, c});
    }
    emit("tx_host", "calls", pts, true);
  }
  std::printf("}\n");
  ns_csum_destroy(ctx);
  return g_sink == 0xFFFFFFFFu;
}
