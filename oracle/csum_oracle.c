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
