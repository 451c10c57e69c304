/* ORACLE — TEST INFRASTRUCTURE ONLY (see csum_oracle.c). */
#ifndef CSUM_ORACLE_H_
#define CSUM_ORACLE_H_
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

/* Same 16-byte layout as ns_pkt_desc (include/netstack_csum.h). */
typedef struct oracle_desc {
  uint64_t off;
  uint32_t len;
  uint16_t initial;
  uint16_t flags; /* bit0 odd, bit1 chain */
} oracle_desc;

uint16_t oracle_combine(uint16_t a, uint16_t b);
uint16_t oracle_calculate_checksum(const uint8_t* buf, uint64_t len, int odd,
                                   uint32_t initial, int* odd_out);
uint16_t oracle_checksum(const uint8_t* buf, uint64_t len, uint16_t initial);
int oracle_vv_with_offset(const uint8_t* const* views, const uint64_t* lens,
                          uint32_t nviews, uint16_t initial, int64_t off,
                          int64_t size, uint16_t* out);
uint16_t oracle_views_restart(const uint8_t* const* views, const uint64_t* lens,
                              uint32_t nviews, uint16_t initial);
uint16_t oracle_pseudo_header(uint32_t protocol, const uint8_t* src,
                              uint32_t src_len, const uint8_t* dst,
                              uint32_t dst_len, uint16_t total_len);
int oracle_batch(const uint8_t* arena, uint64_t arena_bytes,
                 const oracle_desc* d, uint32_t n, uint16_t* out, int chained);
int oracle_batch_mt(const uint8_t* arena, const oracle_desc* d, uint32_t n,
                    uint16_t* out, int nthreads);
/* sendTCPBatch's checksum steps over its header slots and payload view
 * (mode: 0 full, 1 CHECKSUM_PARTIAL, 2 none for TCP); writes the fields into
 * `arena` and the un-complemented sums into out[2n] (or NULL).  Returns the
 * segment count. */
uint64_t oracle_send_tcp_batch(uint8_t* arena, uint64_t hdr_off, uint64_t pay_off,
                               uint64_t size, uint32_t mss, uint32_t slot,
                               uint32_t ip_at, uint32_t ip_len, uint32_t tcp_at,
                               uint32_t tcp_len, uint32_t protocol,
                               const uint8_t* src, uint32_t src_len,
                               const uint8_t* dst, uint32_t dst_len, int mode,
                               uint16_t* out);

/* The receive path of one recvmmsg slot (link dispatch, IPv4/IPv6
 * HandlePacket, segment.parse, handleICMP): returns the verdict (0 invalid,
 * 1 valid, 2 unchecked, 3 malformed) and the IPv4 / transport sums. */
int oracle_rx_verify(const uint8_t* slot, uint64_t slot_bytes, uint64_t rlen, uint32_t frame_at,
                     uint32_t link_hdr, uint32_t first_view, uint16_t* net_out, uint16_t* tr_out);
/* ... over n slots of `stride` bytes from `ring`, slot-parallel over nthreads. */
int oracle_rx_ring(const uint8_t* ring, uint64_t stride, uint32_t n, const uint32_t* lens, uint32_t frame_at,
                   uint32_t link_hdr, uint32_t first_view, uint8_t* verdict, uint16_t* sums, int nthreads);

#ifdef __cplusplus
}
#endif
#endif
