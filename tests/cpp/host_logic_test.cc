// The HIP-free host logic of the C ABI (netstack_amd/csrc/host_logic.h)
// under sanitizers — built by `make -C netstack_amd/csrc sanitize` twice:
// with -fsanitize=address,undefined and with -fsanitize=thread — and run by
// tests/test_host_sanitizers.py (CPU only).  Results are checked against the
// oracle's C restatement of checksum.go (oracle/csum_oracle.c, test
// infrastructure), everything else against the invariants the C ABI relies
// on:
//   ChainBuilder  chains of restart/continue pieces (copied or adopted in
//                 place) -> descriptors whose chained sums equal Go's chain;
//   clip_views    == ChecksumVVWithOffset (checksum.go:69-98);
//   plan_packet   random and garbage packets, both directions: no memory
//                 error, fields written only inside Header, filled TCP
//                 packets verify;
//   cut_chunk     chunks tile the table, never end inside a chained run,
//                 spans within budget, NS_ERANGE on a bad descriptor;
//   shard_plan    contiguous, ordered, whole runs, byte-balanced;
//   tx_plan, tx_multi_plan, rx_plan  geometry checks: whatever they accept
//                 stays inside the arena and apart where the kernels need it;
//   tx_host_plan  pieces tile each call's segments as valid calls, chunks
//                 within budget, the staged ranges hold every byte read;
//   tx_shard_calls  parts tile the calls' segments in order, balanced;
//   FlatCombiner  many threads x many requests: every request done once
//                 with its own result (the point of the -fsanitize=thread
//                 build).
// Usage: host_logic_test [--quick]   (exit status 0 = all passed)
#include <atomic>
#include <chrono>
#include <cstdio>
#include <cstring>
#include <random>
#include <thread>
#include <vector>

#include "csum_oracle.h"
#include "host_logic.h"

static std::atomic<int> g_fail{0}, g_run{0};  // CHECK runs in worker threads too
#define CHECK(cond, ...)                                         \
  do {                                                           \
    ++g_run;                                                     \
    if (!(cond)) {                                               \
      ++g_fail;                                                  \
      std::printf("FAIL %s:%d: %s: ", __FILE__, __LINE__, #cond); \
      std::printf(__VA_ARGS__);                                  \
      std::printf("\n");                                         \
    }                                                            \
  } while (0)

using Rng = std::mt19937_64;

// Copying sink: the arena is a vector.
struct VecSink {
  std::vector<uint8_t> a;
  uint64_t append(const uint8_t* p, uint64_t len) {
    const uint64_t at = a.size();
    a.insert(a.end(), p, p + len);
    return at;
  }
};
// Adopting sink: the pieces already lie in `base` (a caller's stage).
struct AdoptSink {
  const uint8_t* base;
  uint64_t n = 0;
  uint64_t append(const uint8_t* p, uint64_t len) {
    const uint64_t at = len ? (uint64_t)(p - base) : n;
    n = std::max(n, at + len);
    return at;
  }
};

// Go's chain over pieces: xsum = initial, odd = false; each piece through
// calculateChecksum (checksum.go:26-46), odd reset on a restart; empty
// pieces skipped.
static uint16_t go_chain(const std::vector<nsh::Piece>& ps, uint16_t initial) {
  uint32_t x = initial;
  int odd = 0;
  for (const nsh::Piece& p : ps) {
    if (p.restart) odd = 0;
    if (!p.len) continue;
    int o2 = 0;
    x = oracle_calculate_checksum(p.p, p.len, odd, x, &o2);
    odd = o2;
  }
  return (uint16_t)x;
}

template <class Sink>
static std::vector<uint16_t> eval(const Sink& s, const uint8_t* arena, uint64_t arena_bytes,
                                  const nsh::ChainBuilder<Sink>& b) {
  std::vector<uint16_t> res(b.desc.size());
  const int bad = oracle_batch(arena, arena_bytes, reinterpret_cast<const oracle_desc*>(b.desc.data()),
                               (uint32_t)b.desc.size(), res.data(), 1);
  CHECK(bad == 0, "%d out-of-range descriptors", bad);
  std::vector<uint16_t> out;
  for (uint32_t r : b.result_at) out.push_back(res[r]);
  (void)s;
  return out;
}

static void TestChains(Rng& rng, int rounds) {
  std::vector<uint8_t> pool(1 << 20);
  for (auto& b : pool) b = (uint8_t)rng();
  for (int round = 0; round < rounds; ++round) {
    const int nch = 1 + (int)(rng() % 40);
    std::vector<std::vector<nsh::Piece>> chains(nch);
    std::vector<uint16_t> inits(nch), want(nch);
    for (int c = 0; c < nch; ++c) {
      const int np = (int)(rng() % 7);
      for (int k = 0; k < np; ++k) {
        uint64_t len = rng() % 4 == 0 ? 0 : rng() % 3000;
        if (rng() % 50 == 0) len = 131072 + rng() % 20000;  // above the merge limit
        const uint64_t off = rng() % (pool.size() - len);
        // sometimes the next piece continues the previous one's bytes in place
        const uint8_t* p = pool.data() + off;
        if (k > 0 && rng() % 3 == 0) {
          const nsh::Piece& prev = chains[c].back();
          if (prev.p + prev.len + len <= pool.data() + pool.size()) p = prev.p + prev.len;
        }
        chains[c].push_back(nsh::Piece{p, len, k == 0 || rng() % 3 == 0});
      }
      inits[c] = (uint16_t)rng();
      want[c] = go_chain(chains[c], inits[c]);
    }
    VecSink vs;
    nsh::ChainBuilder<VecSink> bv(vs);
    AdoptSink as{pool.data()};
    nsh::ChainBuilder<AdoptSink> ba(as);
    for (int c = 0; c < nch; ++c) {
      bv.chain(chains[c].data(), chains[c].size(), inits[c]);
      ba.chain(chains[c].data(), chains[c].size(), inits[c]);
    }
    for (const ns_pkt_desc& d : bv.desc) CHECK(d.off + d.len <= vs.a.size(), "descriptor inside the arena");
    for (const ns_pkt_desc& d : ba.desc) CHECK(d.off + d.len <= pool.size(), "adopted descriptor inside the stage");
    const auto gv = eval(vs, vs.a.data(), vs.a.size(), bv);
    const auto ga = eval(as, pool.data(), pool.size(), ba);
    for (int c = 0; c < nch; ++c) {
      CHECK(gv[c] == want[c], "copied chain %d: %04x vs %04x", c, gv[c], want[c]);
      CHECK(ga[c] == want[c], "adopted chain %d: %04x vs %04x", c, ga[c], want[c]);
    }
  }
}

static void TestClipViews(Rng& rng, int rounds) {
  std::vector<uint8_t> pool(200000);
  for (auto& b : pool) b = (uint8_t)rng();
  for (int round = 0; round < rounds; ++round) {
    const uint32_t nv = (uint32_t)(rng() % 8);
    std::vector<ns_view> views(nv);
    std::vector<const uint8_t*> vp(nv);
    std::vector<uint64_t> vl(nv);
    uint64_t total = 0;
    for (uint32_t k = 0; k < nv; ++k) {
      const uint64_t len = rng() % 5 == 0 ? 0 : rng() % 5000;
      const uint64_t off = rng() % (pool.size() - len);
      views[k] = ns_view{pool.data() + off, len};
      vp[k] = views[k].data;
      vl[k] = len;
      total += len;
    }
    const int64_t off = (int64_t)(rng() % (total + 10));
    const int64_t size = (int64_t)(rng() % (total + 10));
    std::vector<std::pair<const uint8_t*, uint64_t>> pieces;
    CHECK(nsh::clip_views(views.data(), nv, off, size, &pieces) == NS_OK, "clip");
    VecSink vs;
    nsh::ChainBuilder<VecSink> b(vs);
    const uint16_t init = (uint16_t)rng();
    b.segment(pieces, init);
    uint16_t want = 0;
    oracle_vv_with_offset(vp.data(), vl.data(), nv, init, off, size, &want);
    const auto got = eval(vs, vs.a.data(), vs.a.size(), b);
    CHECK(got[0] == want, "vv_with_offset %04x vs %04x", got[0], want);
  }
  std::vector<std::pair<const uint8_t*, uint64_t>> pieces;
  CHECK(nsh::clip_views(nullptr, 0, -1, 0, &pieces) == NS_EINVAL, "negative off");
  CHECK(nsh::clip_views(nullptr, 0, 0, -1, &pieces) == NS_EINVAL, "negative size");
}

// A random, often broken, packet: IPv4 or IPv6 (or garbage), a transport
// header of a random protocol, random lengths, split into random views.
struct RandPacket {
  std::vector<uint8_t> bytes;
  size_t hdr_len = 0;
  std::vector<size_t> cuts;  // data view boundaries after hdr_len
};

static RandPacket make_packet(Rng& rng, bool tx) {
  RandPacket rp;
  const int kind = (int)(rng() % 10);
  const uint8_t protos[] = {6, 17, 1, 58, 6, 6, 99};
  const uint8_t proto = protos[rng() % 7];
  const size_t payload = rng() % 3 == 0 ? rng() % 8 : rng() % 2000;
  std::vector<uint8_t>& b = rp.bytes;
  size_t ihl = 20, thl = proto == 6 ? 20 + 4 * (rng() % 11) : proto == 17 ? 8 : 8 + 4 * (rng() % 5);
  if (kind < 6) {  // IPv4
    if (rng() % 6 == 0) ihl = 4 * (rng() % 16);
    b.assign(std::max<size_t>(ihl, 20) + thl + payload, 0);
    for (auto& x : b) x = (uint8_t)rng();
    b[0] = (uint8_t)(0x40 | (ihl / 4));
    const size_t tlen = rng() % 8 == 0 ? rng() % 70000 : b.size();
    b[2] = (uint8_t)(tlen >> 8);
    b[3] = (uint8_t)tlen;
    b[6] = rng() % 10 == 0 ? 0x20 : 0;
    b[7] = rng() % 10 == 0 ? (uint8_t)rng() : 0;
    b[9] = proto;
    if (ihl >= 20 && proto == 6 && ihl + 12 < b.size()) b[ihl + 12] = (uint8_t)((thl / 4) << 4);
  } else if (kind < 9) {  // IPv6
    b.assign(40 + thl + payload, 0);
    for (auto& x : b) x = (uint8_t)rng();
    b[0] = 0x60;
    const size_t plen = rng() % 8 == 0 ? rng() % 70000 : b.size() - 40;
    b[4] = (uint8_t)(plen >> 8);
    b[5] = (uint8_t)plen;
    b[6] = proto;
    if (proto == 6) b[40 + 12] = (uint8_t)((thl / 4) << 4);
  } else {  // garbage, possibly tiny
    b.assign(rng() % 64, 0);
    for (auto& x : b) x = (uint8_t)rng();
  }
  const size_t ipl = b.empty() ? 0 : ((b[0] >> 4) == 6 ? 40 : (size_t)(b[0] & 0xF) * 4);
  if (tx && kind < 9) {
    // as Encode leaves them (checksum fields 0): a filled packet then verifies
    if ((b[0] >> 4) == 4 && b.size() >= 12) b[10] = b[11] = 0;
    if (ipl + 18 <= b.size()) b[ipl + 16] = b[ipl + 17] = 0;
  }
  if (rng() % 12 == 0 && !b.empty()) b.resize(rng() % b.size());  // truncated
  rp.hdr_len = tx ? std::min(b.size(), ipl + thl + (rng() % 4 == 0 ? rng() % 16 : 0)) : 0;
  for (size_t p = rp.hdr_len; p < b.size();) {
    p += 1 + rng() % 700;
    if (p < b.size()) rp.cuts.push_back(p);
  }
  return rp;
}

static void TestPackets(Rng& rng, int rounds) {
  int valid_tcp = 0;
  for (int round = 0; round < rounds; ++round) {
    for (uint32_t op : {NS_PKB_VERIFY, NS_PKB_FILL}) {
      RandPacket rp = make_packet(rng, op == NS_PKB_FILL);
      std::vector<uint8_t> before = rp.bytes;
      std::vector<ns_view> views;
      size_t prev = rp.hdr_len;
      for (size_t c : rp.cuts) {
        views.push_back(ns_view{rp.bytes.data() + prev, c - prev});
        prev = c;
      }
      views.push_back(ns_view{rp.bytes.data() + prev, rp.bytes.size() - prev});
      ns_pkt_buf pk{};
      pk.hdr = rp.hdr_len ? rp.bytes.data() : nullptr;
      pk.hdr_len = rp.hdr_len;
      pk.data = views.data();
      pk.ndata = (uint32_t)views.size();
      pk.data_size = rp.bytes.size() - rp.hdr_len - (rng() % 5 == 0 && rp.bytes.size() > rp.hdr_len ? 1 : 0);
      nsh::PacketBytes pb;
      CHECK(pb.init(pk) == NS_OK, "init");
      VecSink vs;
      nsh::ChainBuilder<VecSink> b(vs);
      nsh::PacketPlan plan;
      const int rc = nsh::plan_packet(b, pb, op, &plan);
      CHECK(rc == NS_OK || (op == NS_PKB_FILL && rc == NS_EINVAL), "plan rc %d", rc);
      if (rc != NS_OK) {
        CHECK(rp.bytes == before, "a rejected packet is not written");
        continue;
      }
      std::vector<uint16_t> res(b.result_at.size());
      if (!res.empty()) res = eval(vs, vs.a.data(), vs.a.size(), b);
      uint16_t sums[2] = {0, 0};
      uint8_t verdict = 0xEE;
      nsh::finish_packet(pb, plan, op, res.data(), sums, &verdict);
      if (op == NS_PKB_FILL) {
        // only the checksum fields inside Header may change
        for (size_t k = 0; k < rp.bytes.size(); ++k) {
          const bool field = k == plan.net_store || k == plan.net_store + 1 || k == plan.tr_store ||
                             k == plan.tr_store + 1;
          if (rp.bytes[k] != before[k]) CHECK(field && k < rp.hdr_len, "byte %zu written", k);
        }
        // a filled TCP packet (whole, one view) verifies on receive
        const bool ipv4 = !rp.bytes.empty() && (rp.bytes[0] >> 4) == 4;
        const bool tcp = ipv4 && rp.bytes.size() > 9 && rp.bytes[9] == 6;
        const size_t tlen = rp.bytes.size() >= 4 ? ((size_t)rp.bytes[2] << 8 | rp.bytes[3]) : 0;
        if (tcp && !(rp.bytes[6] & 0x3F) && !rp.bytes[7] && tlen == rp.bytes.size() &&
            pk.data_size + rp.hdr_len == rp.bytes.size() && plan.tr_store != UINT64_MAX) {
          ns_view one{rp.bytes.data(), rp.bytes.size()};
          ns_pkt_buf rx{};
          rx.data = &one;
          rx.ndata = 1;
          rx.data_size = rp.bytes.size();
          nsh::PacketBytes pr;
          pr.init(rx);
          VecSink v2;
          nsh::ChainBuilder<VecSink> b2(v2);
          nsh::PacketPlan p2;
          CHECK(nsh::plan_packet(b2, pr, NS_PKB_VERIFY, &p2) == NS_OK, "verify plan");
          std::vector<uint16_t> r2 = eval(v2, v2.a.data(), v2.a.size(), b2);
          uint8_t v = 0xEE;
          nsh::finish_packet(pr, p2, NS_PKB_VERIFY, r2.data(), nullptr, &v);
          if (p2.verdict != NS_PKB_MALFORMED) {
            CHECK(v == NS_PKB_VALID, "filled TCP packet verdict %d", v);
            ++valid_tcp;
          }
        }
      } else {
        CHECK(verdict <= NS_PKB_MALFORMED, "verdict %d", verdict);
        CHECK(rp.bytes == before, "verify writes nothing");
      }
    }
  }
  CHECK(valid_tcp > 0 || rounds < 50, "no filled TCP packet was checked");
  // A Header or Data view of 4 GiB or more is NS_EINVAL (a descriptor's length
  // is a u32); init reads no bytes, so no such buffer is needed.
  {
    uint8_t b[64] = {0x45};
    ns_view big{b, 1ull << 32};
    ns_pkt_buf pk{};
    pk.data = &big;
    pk.ndata = 1;
    pk.data_size = 1ull << 32;
    nsh::PacketBytes pb;
    CHECK(pb.init(pk) == NS_EINVAL, "a 4 GiB data view");
    pk.data_size = 64;
    nsh::PacketBytes pc;
    CHECK(pc.init(pk) == NS_OK, "the same view clipped to 64 bytes");
    ns_pkt_buf ph{};
    ph.hdr = b;
    ph.hdr_len = 1ull << 32;
    nsh::PacketBytes pd;
    CHECK(pd.init(ph) == NS_EINVAL, "a 4 GiB header");
  }
}

static void TestCutChunk(Rng& rng, int rounds) {
  for (int round = 0; round < rounds; ++round) {
    const uint32_t n = (uint32_t)(rng() % 3000);
    std::vector<ns_pkt_desc> d(n);
    uint64_t pos = 0;
    for (uint32_t i = 0; i < n; ++i) {
      d[i].len = rng() % 6 == 0 ? 0 : (uint32_t)(rng() % 3000);
      d[i].off = rng() % 10 == 0 ? rng() % (pos + 1) : pos;  // mostly packed, some overlap
      d[i].flags = (uint16_t)(i && rng() % 3 == 0 ? NS_DESC_CONT : 0);
      pos = std::max<uint64_t>(pos, d[i].off + d[i].len) + rng() % 16;
    }
    const uint64_t arena = pos + 16;
    const uint64_t budget = 1 + rng() % 200000;
    const uint32_t max_desc = 1 + (uint32_t)(rng() % 500);
    const bool chained = rng() % 2;
    uint32_t k = 0;
    while (k < n) {
      uint32_t cut = 0;
      uint64_t lo = 0, hi = 0;
      CHECK(nsh::cut_chunk(d.data(), n, k, arena, budget, max_desc, chained, &cut, &lo, &hi) == NS_OK, "cut");
      CHECK(cut > k && cut <= n, "progress %u -> %u", k, cut);
      if (cut <= k || cut > n) break;
      if (chained && cut < n) CHECK(!(d[cut].flags & NS_DESC_CONT), "chunk ends inside a run at %u", cut);
      uint64_t l = UINT64_MAX, h = 0;
      bool run_start = true;  // whether [k, cut) holds more than one run
      uint32_t heads = 0;
      for (uint32_t i = k; i < cut; ++i) {
        if (d[i].len) {
          l = std::min<uint64_t>(l, d[i].off);
          h = std::max<uint64_t>(h, d[i].off + d[i].len);
        }
        if (i == k || !(chained && (d[i].flags & NS_DESC_CONT))) ++heads;
      }
      (void)run_start;
      if (l == UINT64_MAX) l = h = 0;
      CHECK(lo == l && hi == h, "span [%llu, %llu) vs [%llu, %llu)", (unsigned long long)lo,
            (unsigned long long)hi, (unsigned long long)l, (unsigned long long)h);
      if (heads > 1) CHECK(hi - lo <= budget && cut - k <= max_desc, "chunk over budget");
      k = cut;
    }
    if (n) {
      std::vector<ns_pkt_desc> bad = d;
      bad[n / 2].off = arena + 1;
      bad[n / 2].len = 1;
      uint32_t kk = 0, cut = 0;
      uint64_t lo, hi;
      int rc = NS_OK;
      while (kk < n && (rc = nsh::cut_chunk(bad.data(), n, kk, arena, budget, max_desc, chained, &cut, &lo, &hi)) ==
                           NS_OK)
        kk = cut;
      CHECK(rc == NS_ERANGE, "bad descriptor -> NS_ERANGE (%d)", rc);
    }
  }
}

static void TestShardPlan(Rng& rng, int rounds) {
  for (int round = 0; round < rounds; ++round) {
    const uint32_t n = (uint32_t)(rng() % 5000);
    const uint32_t parts = 1 + (uint32_t)(rng() % 9);
    std::vector<ns_pkt_desc> d(n);
    uint64_t total = 0;
    for (uint32_t i = 0; i < n; ++i) {
      d[i].len = (uint32_t)(rng() % 9000);
      d[i].flags = (uint16_t)(i && rng() % 4 == 0 ? NS_DESC_CONT : 0);
      total += d[i].len;
    }
    std::vector<uint32_t> first(parts + 1);
    nsh::shard_plan(d.data(), n, parts, first.data());
    CHECK(first[0] == 0 && first[parts] == n, "ends");
    for (uint32_t p = 0; p < parts; ++p) {
      CHECK(first[p] <= first[p + 1], "ordered");
      if (first[p] < n && p > 0 && first[p] > 0) CHECK(!(d[first[p]].flags & NS_DESC_CONT), "whole runs");
    }
    (void)total;
  }
}

struct Req {
  uint64_t in = 0, out = 0;
  uint32_t ndesc = 1;
  int rc = NS_OK;
  std::atomic<bool> done{false};
  uint64_t table_bytes() const { return (uint64_t)ndesc * 18 + 16; }
};

static void TestCombiner(int threads, int per_thread) {
  nsh::FlatCombiner<Req> fc(4096);
  std::atomic<uint64_t> passes{0}, served{0};
  std::atomic<int> in_pass{0}, overlap{0};
  std::atomic<size_t> max_batch{0};
  auto run = [&](Req* const* rs, size_t n) {
    if (in_pass.fetch_add(1) != 0) overlap.fetch_add(1);  // passes never overlap
    // a pass takes a while (a GPU round trip): callers queue up meanwhile
    const auto t0 = std::chrono::steady_clock::now();
    while (std::chrono::steady_clock::now() - t0 < std::chrono::microseconds(20)) {
    }
    for (size_t i = 0; i < n; ++i) rs[i]->out = rs[i]->in * 2654435761ull + 7;
    if (n > max_batch.load()) max_batch.store(n);
    passes.fetch_add(1);
    served.fetch_add(n);
    in_pass.fetch_sub(1);
    return NS_OK;
  };
  std::atomic<int> wrong{0};
  std::vector<std::thread> th;
  for (int t = 0; t < threads; ++t) {
    th.emplace_back([&, t]() {
      Rng r((uint64_t)t * 7919 + 1);
      for (int k = 0; k < per_thread; ++k) {
        Req q;
        q.in = r();
        q.ndesc = 1 + (uint32_t)(r() % 100);
        const int rc = fc.submit(&q, run);
        if (rc != NS_OK || q.out != q.in * 2654435761ull + 7 || !q.done.load()) wrong.fetch_add(1);
      }
    });
  }
  for (auto& x : th) x.join();
  CHECK(wrong.load() == 0, "%d wrong results", wrong.load());
  CHECK(served.load() == (uint64_t)threads * per_thread, "served %llu", (unsigned long long)served.load());
  CHECK(overlap.load() == 0, "passes overlapped");
  std::printf("combiner: %d threads x %d requests in %llu passes (largest %zu requests)\n", threads, per_thread,
              (unsigned long long)passes.load(), max_batch.load());
}

// ScratchRegistry (per-stream scratch of ns_csum_batch_dev): `threads`
// threads each pin, use and unpin scratch for random streams out of
// `streams` handles (half of them through a per-thread key, as
// hipStreamPerThread is), releasing some; checks that an entry is never
// retired while pinned, that one key maps to one live entry, that at most
// `max` entries live, and that every entry made is retired exactly once.
struct FakeScratch : nsh::ScratchSlot {
  std::atomic<int> users{0};
  bool retired = false;
};

static void TestScratchRegistry(int threads, int streams, int per_thread) {
  const size_t kMax = 64;
  nsh::ScratchRegistry<FakeScratch> reg(kMax);
  std::atomic<uint64_t> made{0}, retired{0}, busy_release{0};
  std::mutex gm;
  std::vector<FakeScratch*> graveyard;  // retired entries, deleted at the end
  auto make = [&]() {
    made++;
    return new FakeScratch();
  };
  auto retire = [&](FakeScratch* e) {
    CHECK(e->pins == 0 && e->users.load() == 0, "retired while in use");
    CHECK(!e->retired, "retired twice");
    e->retired = true;
    retired++;
    std::lock_guard<std::mutex> lk(gm);
    graveyard.push_back(e);
  };
  std::vector<std::thread> th;
  for (int t = 0; t < threads; ++t) {
    th.emplace_back([&, t]() {
      Rng r((uint64_t)t * 7919 + 1);
      for (int i = 0; i < per_thread; ++i) {
        const uintptr_t h = 0x1000 + 16 * (uintptr_t)(r() % (uint64_t)streams);
        nsh::ScratchKey k;
        k.stream = reinterpret_cast<const void*>(h);
        if (h & 16) k.thread = std::this_thread::get_id();  // a per-thread stream handle
        if (r() % 8 == 0) {
          if (reg.release(k, retire) == NS_EINVAL) busy_release++;
          continue;
        }
        FakeScratch* e = reg.pin(k, make, retire);
        CHECK(e != nullptr, "pin");
        if (!e) continue;
        CHECK(!e->retired && e->key == k, "pinned entry");
        e->users++;
        if (r() % 4 == 0) std::this_thread::yield();
        CHECK(!e->retired, "retired during use");
        e->users--;
        reg.unpin(e);
        CHECK(reg.size() <= kMax + (size_t)threads, "registry size");
      }
    });
  }
  for (auto& x : th) x.join();
  CHECK(reg.size() <= kMax, "registry above its bound when idle");
  reg.clear(retire);
  CHECK(made.load() == retired.load(), "made %llu retired %llu", (unsigned long long)made.load(),
        (unsigned long long)retired.load());
  for (FakeScratch* e : graveyard) delete e;
  std::printf("scratch registry: %d threads, %d streams, %llu entries made and retired, %llu busy releases\n",
              threads, streams, (unsigned long long)made.load(), (unsigned long long)busy_release.load());
}

// nsh::tx_plan (ns_csum_tcp_tx's geometry check): random geometries, fuzzed
// near every bound.  Whatever it accepts with work to do, every slot, header,
// field and payload byte the kernels touch lies in the arena, the fields in
// their headers, and the payload (when read) apart from the slots; the
// segment count is connect.go:675's.
static void TestTxPlan(Rng& rng, int rounds) {
  auto pick = [&](uint64_t lo, uint64_t hi) { return lo + rng() % (hi - lo + 1); };
  int accepted = 0;
  for (int round = 0; round < rounds * 50; ++round) {
    ns_tcp_tx t{};
    const uint64_t arena = pick(0, 1u << 22);
    t.mss = (uint32_t)(rng() % 8 == 0 ? pick(0, 70000) : pick(1, 3000));
    t.slot = (uint32_t)(rng() % 8 == 0 ? pick(0, 5000) : pick(40, 120));
    t.ip_at = (uint16_t)pick(0, 70);
    t.ip_len = (uint16_t)(rng() % 4 == 0 ? 0 : pick(8, 64));
    t.tcp_at = (uint16_t)pick(0, 90);
    t.tcp_len = (uint16_t)pick(14, 64);
    t.size = rng() % 16 == 0 ? 0 : pick(1, 1u << 20);
    t.hdr_off = pick(0, arena + 100);
    t.pay_off = pick(0, arena + 100);
    t.flags = (uint32_t)(rng() % 16 == 0 ? rng() : rng() % 8);
    nsh::TxPlan p;
    const int rc = nsh::tx_plan(t, arena, &p);
    CHECK(rc == NS_OK || rc == NS_EINVAL || rc == NS_ERANGE, "rc %d", rc);
    if (rc != NS_OK) continue;
    CHECK(t.mss >= 1 && t.mss <= 65535 && t.slot >= 1 && t.slot <= 4096, "accepted mss %u slot %u", t.mss, t.slot);
    CHECK(p.n == (t.size + t.mss - 1) / t.mss, "segment count");
    if (p.n == 0 || !(p.mode & 7u)) continue;
    ++accepted;
    CHECK(t.hdr_off + p.n * t.slot <= arena, "slots inside the arena");
    CHECK(t.pay_off + t.size <= arena, "payload inside the arena");
    if (p.mode & 1u) CHECK(t.ip_len >= 12 && (uint32_t)t.ip_at + t.ip_len <= t.slot, "IPv4 header and field in a slot");
    if (p.mode & 6u) CHECK(t.tcp_len >= 18 && (uint32_t)t.tcp_at + t.tcp_len <= t.slot, "TCP header and field in a slot");
    if (p.mode & 2u)
      CHECK(t.pay_off >= t.hdr_off + p.n * t.slot || t.hdr_off >= t.pay_off + t.size, "payload apart from the slots");
    if ((p.mode & 1u) && (p.mode & 6u))
      CHECK((uint32_t)t.ip_at + t.ip_len <= t.tcp_at || (uint32_t)t.tcp_at + t.tcp_len <= t.ip_at,
            "IPv4 and TCP headers apart");
  }
  CHECK(accepted > 0, "no geometry accepted");
  // the reference's own shape: 45 segments of a 64 KiB GSO write
  ns_tcp_tx t{};
  t.size = 65536, t.mss = 1460, t.slot = 54, t.ip_at = 14, t.ip_len = 20, t.tcp_at = 34, t.tcp_len = 20;
  t.hdr_off = 0, t.pay_off = 45 * 54;
  nsh::TxPlan p;
  CHECK(nsh::tx_plan(t, t.pay_off + t.size, &p) == NS_OK && p.n == 45 && p.mode == 3u, "sendTCPBatch 64 KiB");
  CHECK(nsh::tx_plan(t, t.pay_off + t.size - 1, &p) == NS_ERANGE, "payload one byte past the arena");
  t.pay_off = 100;
  CHECK(nsh::tx_plan(t, 1 << 20, &p) == NS_EINVAL, "payload over the slots");
  t.flags = NS_TX_TCP_PARTIAL;
  CHECK(nsh::tx_plan(t, 1 << 20, &p) == NS_OK && p.mode == 5u, "CHECKSUM_PARTIAL reads no payload");
  t.protocol = 256;  // PseudoHeaderChecksum takes uint8(protocol)
  CHECK(nsh::tx_plan(t, 1 << 20, &p) == NS_EINVAL, "protocol above 255");
  t.protocol = 6;
  t.tcp_at = 30;  // TCP header over the IPv4 header's last 4 bytes
  CHECK(nsh::tx_plan(t, 1 << 20, &p) == NS_EINVAL, "overlapping headers");
  t.flags = NS_TX_TCP_NONE;  // no TCP field written: only the IPv4 header matters
  CHECK(nsh::tx_plan(t, 1 << 20, &p) == NS_OK && p.mode == 1u, "overlap irrelevant under TX offload");
}

// nsh::rx_plan (ns_csum_rx_ring's geometry check): random rings.  Whatever it
// accepts: 16-B-aligned slots of a stride below 2^24, an even IP packet start,
// a first view the parse can rely on, and every slot inside the arena.
static void TestRxPlan(Rng& rng, int rounds) {
  auto pick = [&](uint64_t lo, uint64_t hi) { return lo + rng() % (hi - lo + 1); };
  int accepted = 0;
  for (int round = 0; round < rounds * 50; ++round) {
    ns_rx_ring r{};
    const uint64_t base = rng() % 4 == 0 ? pick(0, 64) : 256 * pick(0, 1000);
    const uint64_t arena = pick(0, 1u << 24);
    r.ring_off = rng() % 2 ? 16 * pick(0, 4096) : pick(0, 1u << 16);
    r.stride = rng() % 8 == 0 ? pick(0, 1u << 25) : 16 * pick(0, 200);
    r.n = (uint32_t)pick(0, 5000);
    r.frame_at = (uint16_t)pick(0, 40);
    r.link_hdr = (uint16_t)(rng() % 4 == 0 ? pick(0, 20) : 14 * (rng() % 2));
    r.first_view = (uint32_t)(rng() % 2 ? 0 : pick(0, 300));
    r.flags = rng() % 16 == 0 ? 1u : 0u;
    const int rc = nsh::rx_plan(r, base, arena);
    CHECK(rc == NS_OK || rc == NS_EINVAL || rc == NS_ERANGE, "rc %d", rc);
    if (rc != NS_OK) continue;
    ++accepted;
    CHECK(r.stride && r.stride < (1u << 24) && r.stride % 16 == 0 && (base + r.ring_off) % 16 == 0, "slot shape");
    CHECK((r.link_hdr == 0 || r.link_hdr == 14) && (r.frame_at + r.link_hdr) % 2 == 0 && r.frame_at < r.stride,
          "frame placement");
    CHECK(r.first_view == 0 || (r.first_view % 2 == 0 && r.first_view >= r.link_hdr + 64u), "first view");
    CHECK(r.ring_off + (uint64_t)r.n * r.stride <= arena, "ring inside the arena");
    CHECK(r.flags == 0, "flags");
  }
  CHECK(accepted > 0, "no ring accepted");
  ns_rx_ring r{};
  r.stride = 1504, r.n = 1000, r.first_view = 128, r.link_hdr = 14;
  CHECK(nsh::rx_plan(r, 4096, 1504000) == NS_OK, "an MTU ring");
  CHECK(nsh::rx_plan(r, 4096, 1503999) == NS_ERANGE, "one byte short");
  CHECK(nsh::rx_plan(r, 4104, 1504000) == NS_EINVAL, "8-B-aligned arena");
  r.first_view = 76;
  CHECK(nsh::rx_plan(r, 4096, 1504000) == NS_EINVAL, "first view below 64 B of IP");
}

// nsh::tx_multi_plan: random sets of calls; whatever it accepts, no call's
// slots overlap another call's slots or a payload a full-mode call reads.
static void TestTxMultiPlan(Rng& rng, int rounds) {
  int accepted = 0;
  for (int round = 0; round < rounds * 20; ++round) {
    const uint32_t count = (uint32_t)(rng() % 6);
    std::vector<ns_tcp_tx> t(count);
    const uint64_t arena = 1u << 20;
    for (auto& x : t) {
      x = ns_tcp_tx{};
      x.mss = 100 + (uint32_t)(rng() % 1400);
      x.slot = 54;
      x.ip_at = 14, x.ip_len = 20, x.tcp_at = 34, x.tcp_len = 20;
      x.size = rng() % 20000;
      x.hdr_off = rng() % (arena - 20000);
      x.pay_off = rng() % (arena - 20000);
      x.flags = (uint32_t)(rng() % 3);
    }
    std::vector<nsh::TxPlan> p;
    const int rc = nsh::tx_multi_plan(t.data(), count, arena, &p);
    if (rc != NS_OK) continue;
    ++accepted;
    for (uint32_t a = 0; a < count; ++a) {
      if (!p[a].n || !(p[a].mode & 7u)) continue;
      const uint64_t alo = t[a].hdr_off, ahi = alo + p[a].n * t[a].slot;
      for (uint32_t b = 0; b < count; ++b) {
        if (!p[b].n || !(p[b].mode & 7u)) continue;
        if (b != a) {
          const uint64_t blo = t[b].hdr_off, bhi = blo + p[b].n * t[b].slot;
          CHECK(ahi <= blo || bhi <= alo, "slots of calls %u and %u overlap", a, b);
        }
        if ((p[b].mode & 2u) && t[b].size)
          CHECK(ahi <= t[b].pay_off || t[b].pay_off + t[b].size <= alo, "slots of %u over payload of %u", a, b);
      }
    }
  }
  CHECK(accepted > 0, "no call set accepted");
  ns_tcp_tx two[2]{};
  for (auto& x : two) x.mss = 1460, x.slot = 54, x.ip_at = 14, x.ip_len = 20, x.tcp_at = 34, x.tcp_len = 20;
  two[0].size = two[1].size = 14600;  // 10 segments each
  two[0].hdr_off = 0, two[0].pay_off = 4096, two[1].hdr_off = 540, two[1].pay_off = 20000;
  std::vector<nsh::TxPlan> p;
  CHECK(nsh::tx_multi_plan(two, 2, 1 << 20, &p) == NS_OK, "adjacent slot regions");
  two[1].hdr_off = 539;
  CHECK(nsh::tx_multi_plan(two, 2, 1 << 20, &p) == NS_EINVAL, "slot regions overlap by one byte");
  two[1].hdr_off = 4096 + 14599;
  CHECK(nsh::tx_multi_plan(two, 2, 1 << 20, &p) == NS_EINVAL, "slots over another call's payload");
  two[1].flags = NS_TX_TCP_NONE;  // that call's payload is not read; call 0's still is
  CHECK(nsh::tx_multi_plan(two, 2, 1 << 20, &p) == NS_EINVAL, "slots over a read payload");
  two[0].flags = NS_TX_TCP_PARTIAL;  // now no payload is read
  CHECK(nsh::tx_multi_plan(two, 2, 1 << 20, &p) == NS_OK, "no payload read");
}

// nsh::tx_host_plan (ns_csum_tcp_tx_host): random call sets and staging
// budgets.  The pieces tile each call's segments in order, each a valid call
// with the segment lengths of the run it stands for; chunks tile the pieces
// within the budget; and a staging buffer filled from the chunk's ranges
// holds, at map(x), arena byte x for every slot and payload byte a piece
// reads, at the arena's alignment modulo 256.
static void TestTxHostPlan(Rng& rng, int rounds) {
  int accepted = 0, multi_chunk = 0, split = 0;
  for (int round = 0; round < rounds * 10; ++round) {
    const uint32_t count = (uint32_t)(rng() % 7);
    const uint64_t arena = 1u << 18;
    std::vector<uint8_t> a(arena);
    for (auto& b : a) b = (uint8_t)rng();
    std::vector<ns_tcp_tx> t(count);
    uint64_t pos = rng() % 300;
    for (auto& x : t) {  // side by side with random gaps, as a caller packs them
      x = ns_tcp_tx{};
      x.mss = rng() % 4 == 0 ? 1 + (uint32_t)(rng() % 16) : 100 + (uint32_t)(rng() % 1500);
      x.slot = 40 + (uint32_t)(rng() % 40);
      x.ip_at = 0, x.ip_len = (uint16_t)(rng() % 4 == 0 ? 0 : 20), x.tcp_at = 20, x.tcp_len = 20;
      x.size = rng() % 8 == 0 ? 0 : rng() % 12000;
      x.flags = (uint32_t)(rng() % 3);
      const uint64_t n = (x.size + x.mss - 1) / x.mss;
      const bool pay_first = rng() % 2;
      if (pay_first) {
        x.pay_off = pos, x.hdr_off = pos + x.size + rng() % 6000;
        pos = x.hdr_off + n * x.slot + rng() % 9000;
      } else {
        x.hdr_off = pos, x.pay_off = pos + n * x.slot + rng() % 6000;
        pos = x.pay_off + x.size + rng() % 9000;
      }
    }
    if (pos > arena) continue;
    const uint64_t budget = rng() % 3 == 0 ? 1 + rng() % 3000 : 1 + rng() % 60000;
    nsh::TxHostPlan plan;
    const int rc = nsh::tx_host_plan(t.data(), count, arena, budget, &plan);
    CHECK(rc == NS_OK, "rc %d for a packed call set", rc);
    if (rc != NS_OK) continue;
    ++accepted;
    multi_chunk += plan.chunks.size() > 1;
    // pieces tile every call's segments
    std::vector<uint64_t> bytes;
    size_t pi = 0;
    uint64_t seg = 0, zeros = 0;
    for (uint32_t k = 0; k < count; ++k) {
      nsh::TxPlan p;
      CHECK(nsh::tx_plan(t[k], arena, &p) == NS_OK, "call %u", k);
      if (p.n && !(p.mode & 7u)) {
        CHECK(zeros < plan.zeros.size() && plan.zeros[zeros].first == seg && plan.zeros[zeros].second == p.n,
              "zero sums of call %u", k);
        ++zeros;
      }
      if (p.n && (p.mode & 7u)) {
        uint64_t next = 0;
        int pieces = 0;
        while (next < p.n) {
          CHECK(pi < plan.pieces.size(), "pieces end inside call %u", k);
          if (pi >= plan.pieces.size()) return;
          const nsh::TxPiece& q = plan.pieces[pi++];
          ++pieces;
          CHECK(q.out0 == seg + next && q.mode == p.mode, "piece of call %u at segment %llu", k,
                (unsigned long long)next);
          const uint64_t want = next + q.nseg == p.n ? t[k].size - next * t[k].mss : q.nseg * t[k].mss;
          CHECK(q.nseg >= 1 && next + q.nseg <= p.n && q.t.size == want, "piece size");
          CHECK(q.t.hdr_off == t[k].hdr_off + next * t[k].slot && q.t.pay_off == t[k].pay_off + next * t[k].mss,
                "piece offsets");
          nsh::TxPlan qp;
          CHECK(nsh::tx_plan(q.t, arena, &qp) == NS_OK && qp.n == q.nseg && qp.mode == q.mode, "piece as a call");
          const uint64_t b = q.nseg * q.t.slot + ((q.mode & 2u) ? q.t.size : 0u);
          CHECK(b <= budget || q.nseg == 1, "piece of %llu bytes over budget %llu", (unsigned long long)b,
                (unsigned long long)budget);
          bytes.push_back(b);
          next += q.nseg;
        }
        split += pieces > 1;
      }
      seg += p.n;
    }
    CHECK(pi == plan.pieces.size() && zeros == plan.zeros.size() && plan.nseg == seg, "no stray pieces");
    // chunks tile the pieces; the staging image matches the arena
    uint32_t next = 0;
    for (const nsh::TxChunk& c : plan.chunks) {
      CHECK(c.p0 == next && c.np >= 1 && c.np <= nsh::kMaxTxHostPieces, "chunk pieces");
      next = c.p0 + c.np;
      uint64_t sum = 0;
      for (uint32_t j = c.p0; j < next; ++j) sum += bytes[j];
      CHECK(sum <= budget || c.np == 1, "chunk over budget");
      // the staging (merged gaps and alignment included) fits too; a
      // one-piece chunk by at most its own gap and two ranges' alignment
      CHECK(c.staging <= budget || (c.np == 1 && c.staging <= sum + nsh::kTxHostGap + 512),
            "chunk staging %llu over budget %llu", (unsigned long long)c.staging, (unsigned long long)budget);
      std::vector<uint8_t> st(c.staging + 16, 0xEE);
      uint64_t end = 0;
      for (uint32_t j = c.r0; j < c.r0 + c.nr; ++j) {
        const nsh::TxRange& r = plan.ranges[j];
        CHECK(r.lo < r.hi && r.hi <= arena && (r.at & 255u) == (r.lo & 255u) && r.at >= end, "range");
        if (j > c.r0) CHECK(r.lo > plan.ranges[j - 1].hi + nsh::kTxHostGap, "ranges merged");
        std::memcpy(st.data() + r.at, a.data() + r.lo, r.hi - r.lo);
        end = r.at + (r.hi - r.lo);
      }
      CHECK(end == c.staging, "staging size");
      const nsh::TxPiece& last = plan.pieces[next - 1];
      CHECK(c.out0 == plan.pieces[c.p0].out0 && c.nout == last.out0 + last.nseg - c.out0, "chunk sums");
      for (uint32_t j = c.p0; j < next; ++j) {
        const nsh::TxPiece& q = plan.pieces[j];
        auto same = [&](uint64_t lo, uint64_t len) {
          const uint64_t m = plan.map(c, lo);
          return m + len <= c.staging && std::memcmp(st.data() + m, a.data() + lo, len) == 0;
        };
        CHECK(same(q.t.hdr_off, q.nseg * q.t.slot), "slots staged");
        if (q.mode & 2u) CHECK(same(q.t.pay_off, q.t.size), "payload staged");
      }
    }
    CHECK(next == plan.pieces.size(), "chunks tile the pieces");
  }
  CHECK(accepted > 0 && multi_chunk > 0 && split > 0, "coverage: %d accepted, %d multi-chunk, %d split", accepted,
        multi_chunk, split);
  // refused as tx_multi_plan refuses, and a zero budget
  ns_tcp_tx two[2]{};
  for (auto& x : two) x.mss = 1460, x.slot = 54, x.ip_at = 14, x.ip_len = 20, x.tcp_at = 34, x.tcp_len = 20;
  two[0].size = two[1].size = 14600;
  two[0].hdr_off = 0, two[0].pay_off = 4096, two[1].hdr_off = 539, two[1].pay_off = 20000;
  nsh::TxHostPlan plan;
  CHECK(nsh::tx_host_plan(two, 2, 1 << 20, 1 << 20, &plan) == NS_EINVAL, "overlapping slots");
  two[1].hdr_off = 540;
  CHECK(nsh::tx_host_plan(two, 2, 1 << 20, 0, &plan) == NS_EINVAL, "zero budget");
  CHECK(nsh::tx_host_plan(two, 2, 1 << 20, 1 << 20, &plan) == NS_OK && plan.chunks.size() == 1 &&
            plan.pieces.size() == 2 && plan.nseg == 20,
        "two calls, one chunk");
}

// nsh::tx_shard_calls (ns_csum_tcp_tx_host_multi): random call sets and part
// counts.  The parts, in order, hold every call's segments in order as runs
// that are valid calls, seg0 follows the segment counts, and every part but
// the last stays within one segment of the byte quota.
static void TestTxShardCalls(Rng& rng, int rounds) {
  int checked = 0;
  for (int round = 0; round < rounds * 10; ++round) {
    const uint32_t count = (uint32_t)(rng() % 9);
    const uint64_t arena = 1u << 20;
    std::vector<ns_tcp_tx> t(count);
    uint64_t pos = 0;
    for (auto& x : t) {
      x = ns_tcp_tx{};
      x.mss = rng() % 4 == 0 ? 1 + (uint32_t)(rng() % 16) : 100 + (uint32_t)(rng() % 1500);
      x.slot = 40 + (uint32_t)(rng() % 40);
      x.ip_at = 0, x.ip_len = (uint16_t)(rng() % 4 == 0 ? 0 : 20), x.tcp_at = 20, x.tcp_len = 20;
      x.size = rng() % 8 == 0 ? 0 : rng() % 40000;
      x.flags = (uint32_t)(rng() % 3);
      const uint64_t n = (x.size + x.mss - 1) / x.mss;
      x.hdr_off = pos, x.pay_off = pos + n * x.slot + rng() % 100;
      pos = x.pay_off + x.size + rng() % 100;
    }
    if (pos > arena) continue;
    std::vector<nsh::TxPlan> plans;
    CHECK(nsh::tx_multi_plan(t.data(), count, arena, &plans) == NS_OK, "packed calls");
    const uint32_t parts = 1 + (uint32_t)(rng() % 9);
    std::vector<std::vector<ns_tcp_tx>> out;
    std::vector<uint64_t> seg0;
    nsh::tx_shard_calls(t.data(), count, plans, parts, &out, &seg0);
    CHECK(out.size() == parts && seg0.size() == parts, "part count");
    uint64_t total = 0, maxper = 0;
    for (uint32_t k = 0; k < count; ++k)
      if (plans[k].n && (plans[k].mode & 7u)) {
        total += plans[k].n * t[k].slot + ((plans[k].mode & 2u) ? t[k].size : 0u);
        maxper = std::max<uint64_t>(maxper, t[k].slot + ((plans[k].mode & 2u) ? t[k].mss : 0u));
      }
    const uint64_t quota = std::max<uint64_t>(1, (total + parts - 1) / parts);
    // walk the parts against the calls
    uint32_t k = 0;
    uint64_t a = 0, seg = 0, sum = 0;
    for (uint32_t p = 0; p < parts; ++p) {
      CHECK(seg0[p] == seg, "seg0 of part %u", p);
      uint64_t bytes = 0;
      for (const ns_tcp_tx& r : out[p]) {
        while (k < count && a == plans[k].n && !(plans[k].n == 0 && a == 0 && r.hdr_off == t[k].hdr_off &&
                                                  r.size == t[k].size)) {
          ++k;
          a = 0;
        }
        CHECK(k < count, "run past the calls");
        if (k >= count) return;
        const bool work = plans[k].n && (plans[k].mode & 7u);
        nsh::TxPlan rp;
        CHECK(nsh::tx_plan(r, arena, &rp) == NS_OK && rp.mode == plans[k].mode, "run as a call");
        const ns_tcp_tx want = nsh::tx_run(t[k], a, rp.n);
        CHECK(r.hdr_off == want.hdr_off && r.pay_off == want.pay_off && r.size == want.size, "run %llu of call %u",
              (unsigned long long)a, k);
        CHECK(work || (a == 0 && rp.n == plans[k].n), "a call without work stays whole");
        if (work) bytes += rp.n * r.slot + ((rp.mode & 2u) ? r.size : 0u);
        a += rp.n;
        seg += rp.n;
        if (plans[k].n == 0) {  // no segments: one run, then the next call
          ++k;
          a = 0;
        }
      }
      if (p + 1 < parts) CHECK(bytes <= quota + maxper, "part %u: %llu bytes, quota %llu", p,
                               (unsigned long long)bytes, (unsigned long long)quota);
      sum += bytes;
    }
    while (k < count && a == plans[k].n) {
      ++k;
      a = 0;
    }
    CHECK(k == count && sum == total, "every segment placed once");
    ++checked;
  }
  CHECK(checked > 0, "no call set checked");
}

int main(int argc, char** argv) {
  const bool quick = argc > 1 && std::strcmp(argv[1], "--quick") == 0;
  Rng rng(20261016);
  const int r = quick ? 20 : 200;
  TestChains(rng, r);
  TestClipViews(rng, 5 * r);
  TestPackets(rng, 10 * r);
  TestCutChunk(rng, r);
  TestShardPlan(rng, r);
  TestTxPlan(rng, r);
  TestTxMultiPlan(rng, r);
  TestTxHostPlan(rng, r);
  TestTxShardCalls(rng, r);
  TestRxPlan(rng, r);
  TestCombiner(16, quick ? 200 : 2000);
  TestScratchRegistry(8, 1000, quick ? 2000 : 20000);
  std::printf("%d checks, %d failed\n", g_run.load(), g_fail.load());
  return g_fail ? 1 : 0;
}
