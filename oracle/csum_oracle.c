/*
 * ORACLE — TEST INFRASTRUCTURE ONLY.  Not part of the product.
 *
 * A plain-C restatement of google/netstack's RFC 1071 checksum
 * (tcpip/header/checksum.go) used as the parity checker for the HIP engine
 * and, timed on host cores, as bench.py's `cpu_baseline` ("kind": "port").
 * Only tests/, __graft_entry__.smoke() and bench.py's cpu_baseline leg may
 * load this library.  The reference is Go and cannot be built in this image
 * (no Go toolchain; package header also imports the un-vendored
 * github.com/google/btree, tcpip/header/tcp.go:20), so the restatement is
 * pinned by the reference's own known-answer tests
 * (tcpip/header/checksum_test.go:34-94) plus public RFC 1071 vectors — see
 * tests/golden/ and DESIGN.md §Oracle.
 *
 * Built with -O2 -fno-tree-vectorize so that the scalar 2-bytes-per-iteration
 * loop stays scalar, like Go gc's code for checksum.go:41-43.
 */
#include "csum_oracle.h"

#include <pthread.h>
#include <stdlib.h>
#include <string.h>

/* checksum.go:104-107 — one end-around carry. */
uint16_t oracle_combine(uint16_t a, uint16_t b) {
  uint32_t v = (uint32_t)a + (uint32_t)b;
  return (uint16_t)(v + (v >> 16));
}

/* checksum.go:26-46 — calculateChecksum(buf, odd, initial) (uint16, bool).
 * v is a uint32 that wraps mod 2^32 and is never folded inside the loop. */
uint16_t oracle_calculate_checksum(const uint8_t* buf, uint64_t len, int odd,
                                   uint32_t initial, int* odd_out) {
  uint32_t v = initial;
  if (odd) {                       /* :29-32 — odd byte is the LOW byte */
    v += (uint32_t)buf[0];
    buf += 1;
    len -= 1;
  }
  uint64_t l = len;
  int odd_now = (int)(l & 1);      /* :34-39 — trailing byte is the HIGH byte */
  if (odd_now) {
    l--;
    v += (uint32_t)buf[l] << 8;
  }
  for (uint64_t i = 0; i < l; i += 2) {  /* :41-43 — big-endian words */
    v += ((uint32_t)buf[i] << 8) + (uint32_t)buf[i + 1];
  }
  if (odd_out) *odd_out = odd_now;
  return oracle_combine((uint16_t)v, (uint16_t)(v >> 16)); /* :45 */
}

/* checksum.go:52-55 */
uint16_t oracle_checksum(const uint8_t* buf, uint64_t len, uint16_t initial) {
  return oracle_calculate_checksum(buf, len, 0, (uint32_t)initial, NULL);
}

/* checksum.go:69-98 — walk the views, skip empties (:73-75), consume `off`
 * across views (:77-81), clip to the remaining size (:83-87), chain the
 * folded sum and the odd flag (:89), stop when size reaches 0 (:91-94). */
int oracle_vv_with_offset(const uint8_t* const* views, const uint64_t* lens,
                          uint32_t nviews, uint16_t initial, int64_t off,
                          int64_t size, uint16_t* out) {
  if (off < 0 || size < 0) return -1; /* Go panics on a negative bound */
  int odd = 0;
  uint16_t sum = initial;
  for (uint32_t k = 0; k < nviews; k++) {
    uint64_t vl = lens[k];
    const uint8_t* v = views[k];
    if (vl == 0) continue;
    if ((uint64_t)off >= vl) {
      off -= (int64_t)vl;
      continue;
    }
    v += off;
    vl -= (uint64_t)off;
    uint64_t l = vl;
    if (l > (uint64_t)size) l = (uint64_t)size;
    if (l == 0) {
      /* calculateChecksum over an empty slice with odd=false leaves the sum;
       * with odd=true Go would index buf[0] and panic — unreachable, since
       * size==0 only happens before the first piece (break at :91-94). */
      sum = oracle_calculate_checksum(v, 0, 0, sum, &odd);
    } else {
      sum = oracle_calculate_checksum(v, l, odd, sum, &odd);
    }
    size -= (int64_t)l;
    if (size == 0) break;
    off = 0;
  }
  *out = sum;
  return 0;
}

/* transport/udp/endpoint.go:811-813, header/icmpv4.go:158-160:
 * xsum = Checksum(v, xsum) per view — alignment restarts at every view. */
uint16_t oracle_views_restart(const uint8_t* const* views, const uint64_t* lens,
                              uint32_t nviews, uint16_t initial) {
  uint16_t x = initial;
  for (uint32_t k = 0; k < nviews; k++) x = oracle_checksum(views[k], lens[k], x);
  return x;
}

/* checksum.go:112-122 */
uint16_t oracle_pseudo_header(uint32_t protocol, const uint8_t* src,
                              uint32_t src_len, const uint8_t* dst,
                              uint32_t dst_len, uint16_t total_len) {
  uint16_t x = oracle_checksum(src, src_len, 0);
  x = oracle_checksum(dst, dst_len, x);
  uint8_t tmp[2] = {(uint8_t)(total_len >> 8), (uint8_t)total_len};
  x = oracle_checksum(tmp, 2, x);
  uint8_t pr[2] = {0, (uint8_t)protocol};
  return oracle_checksum(pr, 2, x);
}

/* The batch contract of include/netstack_csum.h restated over
 * calculateChecksum: each descriptor is one call; CONT chains the result. */
int oracle_batch(const uint8_t* arena, uint64_t arena_bytes,
                 const oracle_desc* d, uint32_t n, uint16_t* out, int chained) {
  int bad = 0;
  uint16_t prev = 0;
  for (uint32_t i = 0; i < n; i++) {
    uint16_t init = (chained && (d[i].flags & 2u)) ? prev : d[i].initial;
    uint64_t len = d[i].len;
    if (d[i].off > arena_bytes || len > arena_bytes - d[i].off) {
      len = 0;
      bad++;
    }
    int odd = (d[i].flags & 1u) && len > 0;
    prev = oracle_calculate_checksum(arena + (len ? d[i].off : 0), len, odd,
                                     init, NULL);
    out[i] = prev;
  }
  return bad;
}

/* ---- packet-parallel CPU baseline (independent descriptors only) -------- */
typedef struct {
  const uint8_t* arena;
  const oracle_desc* d;
  uint16_t* out;
  uint32_t lo, hi;
} mt_job;

static void* mt_worker(void* p) {
  mt_job* j = (mt_job*)p;
  for (uint32_t i = j->lo; i < j->hi; i++) {
    j->out[i] = oracle_calculate_checksum(j->arena + j->d[i].off, j->d[i].len,
                                          (j->d[i].flags & 1u) && j->d[i].len,
                                          j->d[i].initial, NULL);
  }
  return NULL;
}

int oracle_batch_mt(const uint8_t* arena, const oracle_desc* d, uint32_t n,
                    uint16_t* out, int nthreads) {
  if (nthreads < 1) nthreads = 1;
  if (nthreads > 256) nthreads = 256;
  pthread_t th[256];
  mt_job jobs[256];
  for (int t = 0; t < nthreads; t++) {
    jobs[t].arena = arena;
    jobs[t].d = d;
    jobs[t].out = out;
    jobs[t].lo = (uint32_t)(((uint64_t)n * t) / nthreads);
    jobs[t].hi = (uint32_t)(((uint64_t)n * (t + 1)) / nthreads);
  }
  for (int t = 1; t < nthreads; t++) pthread_create(&th[t], NULL, mt_worker, &jobs[t]);
  mt_worker(&jobs[0]);
  for (int t = 1; t < nthreads; t++) pthread_join(th[t], NULL);
  return 0;
}

/* transport/tcp/connect.go:668-702 (sendTCPBatch) with buildTCPHdr
 * (:634-666) per segment, then network/ipv4/ipv4.go:217-238 (addIPHeader)
 * per segment as WritePackets (:271-285) runs it.  The headers are already
 * encoded in the slots (tcp.Encode / ip.Encode, checksum fields zero: a fresh
 * Prependable is zeroed); what remains are the checksum steps:
 *   length := uint16(hdr.UsedLength() + packetSize)        connect.go:652
 *   xsum := r.PseudoHeaderChecksum(ProtocolNumber, length)  :653, route.go:93-95
 *   CHECKSUM_PARTIAL: tcp.SetChecksum(xsum)                 :655-660
 *   else: xsum = ChecksumVVWithOffset(data, xsum, off, packetSize)   :662
 *         tcp.SetChecksum(^tcp.CalculateChecksum(xsum))     :663, tcp.go:259-262
 *   ip.SetChecksum(^ip.CalculateChecksum())                 ipv4.go:236, :251-253
 * The payload is one view (data flattened), so ChecksumVVWithOffset is called
 * on it with the segment's offset, as the Go loop does (off += packetSize). */
static void put_be16(uint8_t* p, uint16_t v) {
  p[0] = (uint8_t)(v >> 8);
  p[1] = (uint8_t)v;
}

uint64_t oracle_send_tcp_batch(uint8_t* arena, uint64_t hdr_off, uint64_t pay_off,
                               uint64_t size, uint32_t mss, uint32_t slot,
                               uint32_t ip_at, uint32_t ip_len, uint32_t tcp_at,
                               uint32_t tcp_len, uint32_t protocol,
                               const uint8_t* src, uint32_t src_len,
                               const uint8_t* dst, uint32_t dst_len, int mode,
                               uint16_t* out) {
  const uint64_t n = (size + mss - 1) / mss; /* connect.go:675 */
  const uint8_t* view = arena + pay_off;
  const uint64_t vlen = size;
  uint64_t left = size, off = 0;
  for (uint64_t i = 0; i < n; i++) {
    uint64_t packet_size = mss;
    if (packet_size > left) packet_size = left;
    left -= packet_size;
    uint8_t* hdr = arena + hdr_off + i * slot;
    uint16_t tsum = 0, isum = 0;
    if (mode != 2) {
      uint8_t* tcp = hdr + tcp_at;
      put_be16(tcp + 16, 0);
      const uint16_t length = (uint16_t)(tcp_len + packet_size);
      uint16_t xsum = oracle_pseudo_header(protocol, src, src_len, dst, dst_len, length);
      if (mode == 1) {
        put_be16(tcp + 16, xsum);
      } else {
        oracle_vv_with_offset(&view, &vlen, 1, xsum, (int64_t)off, (int64_t)packet_size, &xsum);
        xsum = oracle_checksum(tcp, tcp_len, xsum);
        put_be16(tcp + 16, (uint16_t)~xsum);
      }
      tsum = xsum;
    }
    if (ip_len) {
      uint8_t* ip = hdr + ip_at;
      put_be16(ip + 10, 0);
      isum = oracle_checksum(ip, ip_len, 0);
      put_be16(ip + 10, (uint16_t)~isum);
    }
    if (out) {
      out[2 * i] = isum;
      out[2 * i + 1] = tsum;
    }
    off += packet_size;
  }
  return n;
}

/* ---- the receive path over a ring of recvmmsg slots ----------------------
 * One slot as the reference handles it, call for call:
 *   recvMMsgDispatcher.dispatch (link/fdbased/packet_dispatchers.go:258-317):
 *     views = BufConfig buffers (:30; the first of first_view bytes, 0: one
 *     view) capped to the frame (capViews :214-224); n <= hdrSize: dropped;
 *     protocol by EtherType, or by the version nibble without a link header
 *     (:283-296); Data.TrimFront(hdrSize) (:304).
 *   IPv4 HandlePacket (network/ipv4/ipv4.go:341-394), IsValid (header/
 *     ipv4.go:280-296); IPv6 HandlePacket (network/ipv6/ipv6.go:168-188),
 *     IsValid (header/ipv6.go:207-222).
 *   segment.parse (transport/tcp/segment.go:145-181); handleICMP (network/
 *     ipv4/icmp.go:60-80, network/ipv6/icmp.go:62-84, header/icmpv6.go:
 *     202-221).
 * Verdicts and sums as oracle/packets.py verify (0 invalid, 1 valid,
 * 2 unchecked, 3 malformed). */
typedef struct {
  const uint8_t* p;
  uint64_t n;
} o_view;
typedef struct {
  o_view v[16];
  uint32_t k;
} o_vv;

static uint64_t ovv_size(const o_vv* vv) {
  uint64_t s = 0;
  for (uint32_t i = 0; i < vv->k; i++) s += vv->v[i].n;
  return s;
}

/* VectorisedView.TrimFront (tcpip/buffer/view.go:69-79) */
static void ovv_trim_front(o_vv* vv, uint64_t count) {
  while (count > 0 && vv->k > 0) {
    if (count < vv->v[0].n) {
      vv->v[0].p += count;
      vv->v[0].n -= count;
      return;
    }
    count -= vv->v[0].n;
    memmove(&vv->v[0], &vv->v[1], (vv->k - 1) * sizeof(o_view));
    vv->k--;
  }
}

/* VectorisedView.CapLength (view.go:82-103) */
static void ovv_cap(o_vv* vv, uint64_t length) {
  uint64_t left = length;
  for (uint32_t i = 0; i < vv->k; i++) {
    if (left == 0) {
      vv->k = i;
      return;
    }
    if (vv->v[i].n > left) vv->v[i].n = left;
    left -= vv->v[i].n;
  }
}

/* ChecksumVV (checksum.go:61-63) */
static uint16_t ovv_checksum(const o_vv* vv, uint16_t initial) {
  const uint8_t* ptrs[16];
  uint64_t lens[16];
  for (uint32_t i = 0; i < vv->k; i++) {
    ptrs[i] = vv->v[i].p;
    lens[i] = vv->v[i].n;
  }
  uint16_t out = initial;
  oracle_vv_with_offset(ptrs, lens, vv->k, initial, 0, (int64_t)ovv_size(vv), &out);
  return out;
}

static const uint32_t kBufConfig[10] = {128, 256, 256, 512, 1024, 2048, 4096, 8192, 16384, 32768};

int oracle_rx_verify(const uint8_t* slot, uint64_t slot_bytes, uint64_t rlen, uint32_t frame_at,
                     uint32_t link_hdr, uint32_t first_view, uint16_t* net_out, uint16_t* tr_out) {
  *net_out = *tr_out = 0;
  if (rlen > slot_bytes || rlen <= frame_at) return 3;
  const uint8_t* f = slot + frame_at;
  const uint64_t n = rlen - frame_at;
  if (n <= link_hdr) return 3; /* packet_dispatchers.go:268-270 */
  o_vv vv = {0};
  if (first_view == 0) {
    vv.v[0].p = f;
    vv.v[0].n = n;
    vv.k = 1;
  } else {
    uint64_t at = 0;
    for (int i = 0; i < 10 && at < n; i++) {
      const uint64_t sz = i ? kBufConfig[i] : first_view;
      vv.v[vv.k].p = f + at;
      vv.v[vv.k].n = n - at < sz ? n - at : sz;
      vv.k++;
      at += sz;
    }
  }
  int np = -1;
  if (link_hdr) {
    const uint32_t et = ((uint32_t)f[12] << 8) | f[13];
    np = et == 0x0800 ? 4 : et == 0x86DD ? 6 : 0;
    ovv_trim_front(&vv, link_hdr);
  }
  const uint64_t size = n - link_hdr; /* pkt.Data.Size() */
  if (vv.k == 0 || vv.v[0].n == 0) return 3;
  const o_view first = vv.v[0];
  const int ver = first.p[0] >> 4;
  if (np == 0) return 2; /* not IP: nothing the reference checksums */
  if (np > 0 && ver != np) return 3; /* IsValid's version check */
  const uint8_t *src, *dst;
  uint32_t alen, proto;
  uint16_t net = 0;
  if (ver == 4) {
    if (first.n < 20) return 3;
    const uint32_t hlen = (first.p[0] & 0xFu) * 4u, tlen = ((uint32_t)first.p[2] << 8) | first.p[3];
    /* hlen > len(first): not in IsValid; MALFORMED here */
    if (hlen < 20 || hlen > tlen || tlen > size || hlen > first.n) return 3;
    net = oracle_checksum(first.p, hlen, 0); /* IPv4.CalculateChecksum, reported only */
    *net_out = net;
    src = first.p + 12;
    dst = first.p + 16;
    alen = 4;
    proto = first.p[9];
    const int more = (first.p[6] & 0x20) != 0;
    const uint16_t foff = (uint16_t)(((((uint32_t)first.p[6] & 0x1Fu) << 8) | first.p[7]) << 3);
    ovv_trim_front(&vv, hlen);
    ovv_cap(&vv, tlen - hlen);
    if (more || foff) { /* ipv4.go:355-385 */
      const uint64_t ts = ovv_size(&vv);
      if (ts == 0) return 3;
      const uint16_t last = (uint16_t)(foff + (uint16_t)ts - 1);
      return last < foff ? 3 : 2;
    }
  } else if (ver == 6) {
    if (first.n < 40) return 3;
    const uint32_t plen = ((uint32_t)first.p[4] << 8) | first.p[5];
    if ((uint64_t)plen > size - 40) return 3;
    src = first.p + 8;
    dst = first.p + 24;
    alen = 16;
    proto = first.p[6];
    ovv_trim_front(&vv, 40);
    ovv_cap(&vv, plen);
  } else {
    return 3;
  }
  const o_view tfirst = vv.k ? vv.v[0] : (o_view){NULL, 0};
  if (proto == 6) { /* segment.parse */
    if (tfirst.n < 20) return 3;
    const uint32_t off = (uint32_t)(tfirst.p[12] >> 4) * 4u;
    if (off < 20 || off > tfirst.n) return 3;
    uint16_t xsum = oracle_pseudo_header(6, src, alen, dst, alen, (uint16_t)ovv_size(&vv));
    xsum = oracle_checksum(tfirst.p, off, xsum);
    ovv_trim_front(&vv, off);
    xsum = ovv_checksum(&vv, xsum);
    *tr_out = xsum;
    return xsum == 0xFFFF ? 1 : 0;
  }
  if (proto == 1 && ver == 4) { /* handleICMP, echo requests */
    if (tfirst.n < 8) return 3;
    if (tfirst.p[0] != 8) return 2;
    const uint16_t want = (uint16_t)(((uint32_t)tfirst.p[2] << 8) | tfirst.p[3]);
    uint8_t* h = (uint8_t*)malloc(tfirst.n);
    memcpy(h, tfirst.p, tfirst.n);
    h[2] = h[3] = 0; /* h.SetChecksum(0) */
    vv.v[0].p = h;
    const uint16_t s = ovv_checksum(&vv, 0);
    free(h);
    *tr_out = s;
    return (uint16_t)~s == want ? 1 : 0;
  }
  if (proto == 58 && ver == 6) { /* ICMPv6Checksum(h, src, dst, the other views) */
    if (tfirst.n < 8) return 3; /* ICMPv6MinimumSize (ipv6/icmp.go:68, header/icmpv6.go:35) */
    const uint16_t want = (uint16_t)(((uint32_t)tfirst.p[2] << 8) | tfirst.p[3]);
    const uint64_t total = ovv_size(&vv);
    uint16_t xsum = oracle_checksum(src, 16, 0);
    xsum = oracle_checksum(dst, 16, xsum);
    const uint8_t l4[4] = {(uint8_t)(total >> 24), (uint8_t)(total >> 16), (uint8_t)(total >> 8), (uint8_t)total};
    xsum = oracle_checksum(l4, 4, xsum);
    const uint8_t nh[4] = {0, 0, 0, 58};
    xsum = oracle_checksum(nh, 4, xsum);
    for (uint32_t i = 1; i < vv.k; i++) xsum = oracle_checksum(vv.v[i].p, vv.v[i].n, xsum);
    uint8_t* h = (uint8_t*)malloc(tfirst.n);
    memcpy(h, tfirst.p, tfirst.n);
    h[2] = h[3] = 0;
    const uint16_t got = (uint16_t)~oracle_checksum(h, tfirst.n, xsum);
    free(h);
    *tr_out = (uint16_t)~got;
    return got == want ? 1 : 0;
  }
  if (proto == 17 && tfirst.n < 8) return 3; /* UDPMinimumSize (stack/nic.go:851) */
  return 2;
}

typedef struct {
  const uint8_t* ring;
  uint64_t stride;
  const uint32_t* lens;
  uint32_t frame_at, link_hdr, first_view;
  uint8_t* verdict;
  uint16_t* sums;
  uint32_t lo, hi;
} rx_job;

static void* rx_worker(void* p) {
  rx_job* j = (rx_job*)p;
  for (uint32_t s = j->lo; s < j->hi; s++) {
    uint16_t net, tr;
    j->verdict[s] = (uint8_t)oracle_rx_verify(j->ring + (uint64_t)s * j->stride, j->stride, j->lens[s], j->frame_at,
                                              j->link_hdr, j->first_view, &net, &tr);
    j->sums[2 * (uint64_t)s] = net;
    j->sums[2 * (uint64_t)s + 1] = tr;
  }
  return NULL;
}

int oracle_rx_ring(const uint8_t* ring, uint64_t stride, uint32_t n, const uint32_t* lens, uint32_t frame_at,
                   uint32_t link_hdr, uint32_t first_view, uint8_t* verdict, uint16_t* sums, int nthreads) {
  if (nthreads < 1) nthreads = 1;
  if (nthreads > 256) nthreads = 256;
  pthread_t th[256];
  rx_job jobs[256];
  for (int t = 0; t < nthreads; t++) {
    jobs[t] = (rx_job){ring, stride, lens, frame_at, link_hdr, first_view, verdict, sums,
                       (uint32_t)(((uint64_t)n * t) / nthreads), (uint32_t)(((uint64_t)n * (t + 1)) / nthreads)};
  }
  for (int t = 1; t < nthreads; t++) pthread_create(&th[t], NULL, rx_worker, &jobs[t]);
  rx_worker(&jobs[0]);
  for (int t = 1; t < nthreads; t++) pthread_join(th[t], NULL);
  return 0;
}
