/*
 * netstack_csum.h — C ABI of the MI355X (gfx950) Internet-checksum engine.
 *
 * This is the drop-in boundary for google/netstack's checksum hot path.  A cgo
 * shim in package `header` binds exactly these symbols;
 * nothing here uses torch or HIP types (streams are passed as `void*`, which is
 * a hipStream_t; NULL = the HIP null stream, as in the HIP runtime API).
 *
 * Reference interfaces replaced (google/netstack @ /root/reference):
 *   header.Checksum              tcpip/header/checksum.go:52-55   -> ns_csum_checksum
 *   header.ChecksumVV            tcpip/header/checksum.go:61-63   -> ns_csum_vv_with_offset(off=0,size=Size())
 *   header.ChecksumVVWithOffset  tcpip/header/checksum.go:69-98   -> ns_csum_vv_with_offset
 *   header.ChecksumCombine       tcpip/header/checksum.go:104-107 -> ns_csum_combine
 *   header.PseudoHeaderChecksum  tcpip/header/checksum.go:112-122 -> ns_csum_pseudo_header
 *   per-view restart loops       transport/udp/endpoint.go:811-813,
 *                                header/icmpv4.go:158-160, icmpv6.go:210-212
 *                                                                 -> ns_csum_views_restart
 *   n x ChecksumVVWithOffset in  transport/tcp/connect.go:668-702 (sendTCPBatch,
 *   buildTCPHdr :662) over stack.PacketDescriptor{Off,Size}
 *   (stack/route.go:174-188)                                      -> ns_csum_vv_batch
 *   the per-packet calculateChecksum (checksum.go:26-46) over a
 *   device-resident batch                                         -> ns_csum_batch_dev / _host
 *   ... and the header write that follows it, SetChecksum(^xsum)
 *   (connect.go:663, ipv4.go:236; tcp.go:252, ipv4.go:223)        -> ns_csum_batch_dev_store
 *   sendTCPBatch's whole batch from its geometry: buildTCPHdr for every
 *   segment (connect.go:668-702) and addIPHeader (ipv4.go:217-238)  -> ns_csum_tcp_tx
 *   ... for calls in host memory, many at once                    -> ns_csum_tcp_tx_host
 *   any composition of Checksum(v, xsum) / view chaining (a whole
 *   TCP/UDP/ICMP/IPv4 checksum per chain)                         -> ns_csum_chains
 *   the checksum steps of a batch of tcpip.PacketBuffer
 *   (tcpip/packet_buffer.go:25-50): receive — segment.parse
 *   (tcp/segment.go:166-181), ICMPv4/v6 handleICMP
 *   (network/ipv4/icmp.go:60-80, network/ipv6/icmp.go:62-84);
 *   transmit — buildTCPHdr (tcp/connect.go:653-663), sendUDP
 *   (udp/endpoint.go:808-815), the ICMP echo reply
 *   (network/ipv4/icmp.go:96-100), ICMPv6Checksum (icmpv6.go:202-221),
 *   addIPHeader (network/ipv4/ipv4.go:217-238)                  -> ns_csum_packet_buffers
 *   the same receive checks for a recvmmsg ring resident in HBM, parsed on
 *   the device: recvMMsgDispatcher.dispatch (link/fdbased/
 *   packet_dispatchers.go:258-317), IPv4/IPv6 HandlePacket + IsValid
 *   (network/ipv4/ipv4.go:341-394, header/ipv4.go:280-296; network/ipv6/
 *   ipv6.go:168-188, header/ipv6.go:207-222), segment.parse
 *   (tcp/segment.go:145-181), handleICMP                         -> ns_csum_rx_ring
 *   ... for a ring in host memory                                 -> ns_csum_rx_ring_host
 *
 * Semantics (bit-exact with checksum.go, including its un-folded uint32 wrap for
 * buffers > 128 KiB): every descriptor d is one calculateChecksum call over
 * arena[d.off, d.off+d.len) with odd = (d.flags & NS_DESC_ODD) and
 * initial = d.initial, returning ChecksumCombine(uint16(v), uint16(v>>16)).
 * A descriptor with NS_DESC_CONT takes as its initial the result of the
 * descriptor before it (the `sum` chaining of checksum.go:89 / the
 * `xsum = Checksum(v, xsum)` loops); its own `initial` field is ignored.
 * Results are the UN-complemented sum, exactly like the Go functions; callers
 * apply `^` (connect.go:663) or compare with 0xffff (segment.go:180).
 *
 * Errors: every function returns NS_OK (0) or a negative NS_E* code; nothing is
 * silently recomputed on the host.  There is no CPU fallback in this library.
 */
#ifndef NETSTACK_CSUM_H_
#define NETSTACK_CSUM_H_

#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

#define NS_CSUM_ABI_VERSION 9  /* 2: ns_csum_batch_dev_store, NS_DESC_STORE*;
                                  3: ns_csum_stage_*, ns_csum_packet_buffers;
                                  4: ns_csum_stream_release, _scratch_count;
                                  5: ns_csum_get_stats;
                                  6: ns_csum_tcp_tx;
                                  7: ns_csum_tcp_tx_multi;
                                  8: ns_csum_rx_ring, ns_csum_set_tx_tuning;
                                  9: ns_csum_tcp_tx_host, _host_multi,
                                     ns_csum_rx_ring_host, ns_csum_rx_bufs */

/* ---- status codes ------------------------------------------------------- */
#define NS_OK 0
#define NS_EINVAL (-1)     /* bad argument (negative size, NULL pointer, ...)  */
#define NS_ERANGE (-2)     /* a descriptor reaches past the arena              */
#define NS_ENODEV (-3)     /* no HIP device / device id out of range           */
#define NS_ENOMEM (-4)     /* device or pinned allocation failed               */
#define NS_EHIP (-5)       /* any other HIP runtime error                      */

/* ---- descriptor --------------------------------------------------------- */
/* bit 0: the previous piece ended mid-word; this piece's first byte is the
 *        LOW byte of a big-endian word (calculateChecksum's `odd` argument,
 *        checksum.go:29-32).                                                 */
#define NS_DESC_ODD 0x1u
/* bit 1: chain: initial := result of the previous descriptor (checksum.go:89). */
#define NS_DESC_CONT 0x2u
/* bit 2: store: once this descriptor's result r is final (after its chain),
 *        write ^r big-endian at arena[off + NS_DESC_STORE_AT(flags)], i.e.
 *        the header's SetChecksum(^CalculateChecksum(xsum)) (tcp.go:252,
 *        connect.go:663; ipv4.go:223, :236).  Honoured only by
 *        ns_csum_batch_dev_store (a writable arena); ignored elsewhere.
 * bit 3: with bit 2, store r itself, not ^r: the CHECKSUM_PARTIAL
 *        pseudo-header sum of a GSO segment (connect.go:655-660).
 * bits 4-15: the store offset from `off` (0..4095); the 2 bytes must lie in
 *        the arena (else the store is dropped and counted by ns_csum_sync).
 *        Every sum of the batch sees the arena as it was before the call
 *        provided no descriptor reads stored bytes other than the storing
 *        descriptor itself (unchained) or any descriptor (NS_BATCH_CHAINED:
 *        stores happen after all reads, in the run-folding pass).          */
#define NS_DESC_STORE 0x4u
#define NS_DESC_STORE_RAW 0x8u
#define NS_DESC_STORE_SHIFT 4
#define NS_DESC_STORE_AT(flags) ((uint32_t)(flags) >> NS_DESC_STORE_SHIFT)

/* One packet (or one piece of a chained packet).  16 bytes, little-endian,
 * naturally aligned: maps 1:1 onto stack.PacketDescriptor{Off,Size}
 * (stack/route.go:174-178) plus the pseudo-header sum as `initial`
 * (stack/route.go:93-95) — the device-staged layout of tcpip/buffer.        */
typedef struct ns_pkt_desc {
  uint64_t off;     /* byte offset of the piece in the arena          */
  uint32_t len;     /* byte length (0 allowed: result = initial)      */
  uint16_t initial; /* starting sum (pseudo-header), ignored if CONT  */
  uint16_t flags;   /* NS_DESC_*                                       */
} ns_pkt_desc;

/* batch_flags for ns_csum_batch_*: the table contains NS_DESC_CONT entries.
 * Without it CONT bits are an error-free no-op (each entry is independent). */
#define NS_BATCH_CHAINED 0x1u
/* batch_flags for ns_csum_batch_dev / _dev_store only: runs are pairs.  An
 * odd-indexed NS_DESC_CONT descriptor continues the descriptor before it (its
 * initial := that one's result, checksum.go:89), exactly as NS_BATCH_CHAINED
 * would fold it; NS_DESC_CONT on an even-indexed descriptor is ignored.  The
 * pair is folded inside the checksum kernel: no scratch, no fold pass.  Meant
 * for two-piece sums whose pieces are not contiguous, e.g. a TCP segment whose
 * header lies in sendTCPBatch's header slots and whose payload lies in its
 * payload view (workloads.tx_split_desc).  NS_EINVAL together
 * with NS_BATCH_CHAINED, and on the host-memory entry points.               */
#define NS_BATCH_PAIRED 0x2u

/* A borrowed host byte range: one buffer.View (tcpip/buffer/view.go:19). */
typedef struct ns_view {
  const uint8_t* data;
  uint64_t len;
} ns_view;

/* One segment of a VectorisedView batch: the (Off, Size) of a
 * stack.PacketDescriptor (route.go:174-178) plus its pseudo-header sum.     */
typedef struct ns_seg {
  int64_t off;
  int64_t size;
  uint16_t initial;
  uint16_t pad0;
  uint32_t pad1;
} ns_seg;

/* ---- context -------------------------------------------------------------*/
typedef struct ns_csum_ctx ns_csum_ctx;

typedef struct ns_csum_opts {
  int32_t device;          /* HIP device ordinal                            */
  uint32_t flags;          /* 0, or NS_OPT_* below (others: NS_EINVAL)      */
  uint64_t staging_bytes;  /* pinned host staging per buffer (0 = 64 MiB)   */
} ns_csum_opts;
/* Tests only: chained batches fold their runs with no look-back, every
 * block deriving its carry-in by walking its run (the path a block takes
 * when a predecessor is not running).  Results are the same.               */
#define NS_OPT_FOLD_WALK 0x1u

int ns_csum_abi_version(void);
/* hipError_t of the last failed HIP call on this thread (0 if none); set
 * NS_CSUM_DEBUG=1 in the environment to also print it to stderr.          */
int ns_csum_last_hip_error(void);
const char* ns_csum_strerror(int status);
int ns_csum_device_count(int* count);

int ns_csum_init(const ns_csum_opts* opts, ns_csum_ctx** out);
void ns_csum_destroy(ns_csum_ctx* ctx);

/* Blocks until `stream` is idle (NULL: the whole device); returns the
 * number of out-of-range descriptors (and dropped stores) counted since the
 * last call in *bad (descriptors past `arena_bytes` are summed as empty and
 * counted).  The count is read and reset in one device atomic: counts from
 * kernels still running on other streams are reported by a later call.      */
int ns_csum_sync(ns_csum_ctx* ctx, void* stream, uint64_t* bad);

/* ---- device-resident batch (the hot path) --------------------------------
 * d_arena/d_desc/d_out are device pointers on ctx's device; the call only
 * enqueues kernels on `stream` and returns (asynchronous).  With
 * NS_BATCH_CHAINED, or when descriptors average >= 1 MiB (arena_bytes / n:
 * then each is spread over many workgroups), the call uses device scratch
 * that the context keeps per stream: calls on different streams of one
 * context run concurrently, calls on one stream are ordered by it.  (For
 * hipStreamPerThread the scratch is per calling thread as well.)  Growing it
 * is stream-ordered and never waits for the device; at most 64 streams keep
 * scratch, the least recently used giving it up when another needs it.
 * A 16-B-aligned arena of exactly n slots of 16, 32, 48 or 64 bytes (a ring
 * of fixed-size receive buffers, packet k in slot k) lets the kernel load
 * each packet beside its descriptor instead of after it; any other layout
 * gives the same results.                                                    */
int ns_csum_batch_dev(ns_csum_ctx* ctx, const uint8_t* d_arena,
                      uint64_t arena_bytes, const ns_pkt_desc* d_desc,
                      uint32_t n, uint16_t* d_out, uint32_t batch_flags,
                      void* stream);

/* ns_csum_batch_dev over a writable arena, honouring NS_DESC_STORE: the
 * device-resident transmit path writes every checksum field in place
 * (buildTCPHdr connect.go:653-663 and addIPHeader ipv4.go:217-238 for a whole
 * batch, without the packets leaving HBM).  Results also go to d_out.       */
int ns_csum_batch_dev_store(ns_csum_ctx* ctx, uint8_t* d_arena,
                            uint64_t arena_bytes, const ns_pkt_desc* d_desc,
                            uint32_t n, uint16_t* d_out, uint32_t batch_flags,
                            void* stream);

/* ---- sendTCPBatch from its geometry (no descriptor table) ----------------
 * The transmit checksums of one sendTCPBatch call (transport/tcp/connect.go:
 * 668-702) and of addIPHeader for its segments (network/ipv4/ipv4.go:217-238),
 * over the layout sendTCPBatch builds, resident in d_arena:
 * NewPacketDescriptors' one buffer of n header slots (stack/route.go:181-188)
 * and the payload view.  n = ceil(size / mss) segments (connect.go:675);
 * segment i's payload is [pay_off + i*mss, + min(mss, size - i*mss))
 * (:679-691), its headers lie in slot i = [hdr_off + i*slot, + slot).
 * Per segment, as buildTCPHdr and addIPHeader compute them:
 *   TCP field (tcp_at + 16) := ^Checksum(tcp[:tcp_len], ChecksumVVWithOffset(
 *       payload, PseudoHeaderChecksum(protocol, src, dst, tcp_len + size)))
 *       (connect.go:652-663); with NS_TX_TCP_PARTIAL the pseudo-header sum
 *       itself (gso.NeedsCsum, :655-660); NS_TX_TCP_NONE leaves it alone
 *       (CapabilityTXChecksumOffload, :661);
 *   IPv4 field (ip_at + 10) := ^Checksum(ip[:ip_len], 0) (ipv4.go:236);
 *       ip_len = 0: no IPv4 header (an IPv6 route).
 * Both fields are summed as zero, as freshly encoded headers hold them.  The
 * pseudo-header's addresses enter as addr_sum = Checksum(dst, Checksum(src,
 * 0)), the route's (route.go:93-95, checksum.go:113-114); tcp_len is the
 * header's DataOffset (tcp.go:259-262) and the length word is
 * uint16(tcp_len + size) (connect.go:652).
 * The call owns the header slots until it completes: it writes them back whole
 * (unchanged bytes included), unless NS_TX_FIELDS_ONLY (2-byte stores).
 * Asynchronous on `stream`.  d_out (2n u16, or NULL): [2i] the IPv4 sum,
 * [2i+1] the TCP sum, un-complemented (0 where not computed).
 * NS_EINVAL: mss 0 or > 65535, slot 0 or > 4096, a header longer than 60 B
 * or not inside the slot, a field not inside its header (ip_len < 12,
 * tcp_len < 18), NS_TX_TCP_PARTIAL with NS_TX_TCP_NONE, n >= 2^32, payload
 * and slots overlapping.  NS_ERANGE: slots or payload past the arena.
 * Bytes per segment read: its payload and its slot; written: its slot.     */
typedef struct ns_tcp_tx {
  uint64_t hdr_off;   /* arena offset of header slot 0                        */
  uint64_t pay_off;   /* arena offset of the payload's first byte              */
  uint64_t size;      /* data.Size()                                           */
  uint32_t mss;       /* gso.MSS                                               */
  uint32_t slot;      /* hdrSize: TCPMinimumSize + MaxHeaderLength + optLen    */
  uint16_t ip_at;     /* the IPv4 header's offset in a slot                    */
  uint16_t ip_len;    /* its length, IHL * 4 (0: none)                         */
  uint16_t tcp_at;    /* the TCP header's offset in a slot                     */
  uint16_t tcp_len;   /* its length, DataOffset (20 + options)                 */
  uint16_t addr_sum;  /* Checksum(dst, Checksum(src, 0))                       */
  uint16_t protocol;  /* 6 (header.TCPProtocolNumber)                          */
  uint32_t flags;     /* NS_TX_*                                               */
} ns_tcp_tx;
#define NS_TX_TCP_PARTIAL 0x1u
#define NS_TX_TCP_NONE 0x2u
#define NS_TX_FIELDS_ONLY 0x4u
int ns_csum_tcp_tx(ns_csum_ctx* ctx, uint8_t* d_arena, uint64_t arena_bytes,
                   const ns_tcp_tx* tx, uint16_t* d_out, void* stream);
/* Many sendTCPBatch calls (one per connection, say) over one arena in one
 * launch: txs[0..count) (host memory) as for ns_csum_tcp_tx, each checked
 * the same way; d_out (or NULL) holds call k's 2 n_k sums from
 * 2 * (n_0 + ... + n_{k-1}).  One fused pass for all of them.  NS_EINVAL
 * also when one call's slots overlap another's slots or a payload a
 * full-mode call reads.  Asynchronous on `stream`; the geometry table is
 * uploaded through the stream's scratch (released by ns_csum_stream_release).*/
int ns_csum_tcp_tx_multi(ns_csum_ctx* ctx, uint8_t* d_arena, uint64_t arena_bytes,
                         const ns_tcp_tx* txs, uint32_t count, uint16_t* d_out,
                         void* stream);
/* The same calls over HOST memory (sendTCPBatch as netstack runs it: the
 * header slots and payload views in host memory, possibly many connections'
 * calls at once): h_arena as d_arena above, txs[0..count) checked as for
 * ns_csum_tcp_tx_multi.  Synchronous.  The bytes the calls read (their slots,
 * and the payload of full-mode calls) go to the device in chunks of at most
 * the context's staging size (ns_csum_opts.staging_bytes; a call larger than
 * that is split by segments), four chunks in flight; ranges closer than 4 KiB
 * travel together, so bytes between them are uploaded too (and count
 * against the staging size; only a chunk of one call's run of segments can
 * exceed it, by that gap and 512 B of alignment).  Each segment's
 * fields are then written into h_arena's slots, the same values
 * ns_csum_tcp_tx_multi stores: only the 2-byte fields change, every other
 * byte is left as it was.  h_out (2 * sum n_k u16, or NULL) gets the sums as
 * d_out does.  Pinned memory (ns_csum_stage_acquire) is copied by DMA
 * directly; pageable memory is bounced by the HIP runtime.  Errors as for
 * ns_csum_tcp_tx_multi, returned before any byte is written; on an engine
 * error later (NS_ENOMEM, NS_EHIP) some fields may already be written.
 * Like ns_csum_rx_ring_host it waits for a host pipeline call running on the
 * same context, small calls (within 1 MiB, no DMA) included.               */
int ns_csum_tcp_tx_host(ns_csum_ctx* ctx, uint8_t* h_arena, uint64_t arena_bytes,
                        const ns_tcp_tx* txs, uint32_t count, uint16_t* h_out);

/* Frees the scratch the context keeps for `stream` (see ns_csum_batch_dev),
 * after the stream's last launch that used it; nothing waits.  Call it
 * before destroying a stream that ran chained or huge-descriptor batches
 * (otherwise the scratch is reclaimed only when 64 other streams need some).
 * NS_EINVAL if another thread is launching on that stream right now; NS_OK
 * if the stream has no scratch.  ns_csum_scratch_count: streams holding some. */
int ns_csum_stream_release(ns_csum_ctx* ctx, void* stream);
int ns_csum_scratch_count(ns_csum_ctx* ctx, uint32_t* count);

/* Host-memory batch: H2D of arena and table, kernels writing the results
 * into mapped pinned memory, pipelined in chunks over the context's streams
 * (four in flight); synchronous.  Pageable host memory is bounced through
 * the context's pinned staging.                                             */
int ns_csum_batch_host(ns_csum_ctx* ctx, const uint8_t* h_arena,
                       uint64_t arena_bytes, const ns_pkt_desc* h_desc,
                       uint32_t n, uint16_t* h_out, uint32_t batch_flags);

/* ---- reference-shaped entry points (synchronous, device-computed) ------- */
/* header.Checksum(buf, initial)                    checksum.go:52-55        */
int ns_csum_checksum(ns_csum_ctx* ctx, const uint8_t* buf, uint64_t len,
                     uint16_t initial, uint16_t* out);
/* header.ChecksumVVWithOffset(vv, initial, off, size) checksum.go:69-98.
 * ChecksumVV(vv, initial) == this with off = 0, size = vv.Size().
 * size < 0 or off < 0 -> NS_EINVAL (Go panics on a negative slice bound). */
int ns_csum_vv_with_offset(ns_csum_ctx* ctx, const ns_view* views,
                           uint32_t nviews, uint16_t initial, int64_t off,
                           int64_t size, uint16_t* out);
/* n x ChecksumVVWithOffset(vv, segs[i].initial, segs[i].off, segs[i].size)
 * in one device pass (sendTCPBatch, connect.go:668-702).                    */
int ns_csum_vv_batch(ns_csum_ctx* ctx, const ns_view* views, uint32_t nviews,
                     const ns_seg* segs, uint32_t nsegs, uint16_t* out);
/* xsum = initial; for v in views: xsum = Checksum(v, xsum)
 * (udp/endpoint.go:811-813, icmpv4.go:158-160): alignment restarts per view. */
int ns_csum_views_restart(ns_csum_ctx* ctx, const ns_view* views,
                          uint32_t nviews, uint16_t initial, uint16_t* out);
/* header.PseudoHeaderChecksum(protocol, src, dst, totalLen) checksum.go:112-122 */
int ns_csum_pseudo_header(ns_csum_ctx* ctx, uint32_t protocol,
                          const uint8_t* src, uint32_t src_len,
                          const uint8_t* dst, uint32_t dst_len,
                          uint16_t total_len, uint16_t* out);
/* Chains of pieces: the general form every caller above reduces to.  A chain
 * is a run of pieces ending with one flagged NS_PIECE_END; its result is
 * emitted to out[] in chain order.  Per chain: sum = first piece's initial,
 * odd = false; for each piece (sum, odd) = calculateChecksum(piece, odd', sum)
 * (checksum.go:26-46) with odd' = false for a NS_PIECE_RESTART piece (the
 * semantics of Checksum(v, sum), checksum.go:52-55) and odd' = odd otherwise
 * (ChecksumVVWithOffset's view chaining, checksum.go:89; empty continue
 * pieces are skipped as empty views are, :73-75).  One chain can therefore
 * hold a TCP/UDP segment's whole checksum: pseudo-header fields (restart),
 * payload views (first restart, then continue), transport header (restart) —
 * buildTCPHdr (tcp/connect.go:634-666) and segment.parse (tcp/segment.go:
 * 174-180) — and all chains of a batch run in one device pass.              */
#define NS_PIECE_RESTART 0x1u
#define NS_PIECE_END 0x2u
typedef struct ns_piece {
  const uint8_t* data;
  uint64_t len;
  uint16_t initial; /* used by the first piece of a chain */
  uint16_t flags;   /* NS_PIECE_* */
  uint32_t pad;
} ns_piece;
int ns_csum_chains(ns_csum_ctx* ctx, const ns_piece* pieces, uint32_t npieces,
                   uint16_t* out, uint32_t nout);

/* ---- caller-filled staging ----------------------------------------------
 * A pinned, device-mapped host buffer of at least `bytes` bytes leased from
 * the context (released with ns_csum_stage_release).  Every entry point that
 * takes host byte pointers (ns_csum_checksum, _vv_with_offset, _vv_batch,
 * _views_restart, _chains, _packet_buffers) reads them IN PLACE, without a
 * copy, when all of a call's bytes lie inside one acquired stage: a host that
 * must not hand the library pointers into its own heap (Go: cgo forbids C
 * memory holding Go pointers) copies its views into a stage once and passes
 * pointers into it.  One call at a time per stage.                          */
int ns_csum_stage_acquire(ns_csum_ctx* ctx, uint64_t bytes, uint8_t** base);
int ns_csum_stage_release(ns_csum_ctx* ctx, uint8_t* base);

/* ---- tcpip.PacketBuffer batches --------------------------------------------
 * One tcpip.PacketBuffer (tcpip/packet_buffer.go:25-50): the packet's bytes
 * are its Header's used part (buffer.Prependable View(), prependable.go:
 * 55-58) followed by its Data views clipped to Data.Size().  The network
 * header (IPv4 or IPv6, no extension headers) is the packet's first byte.  */
typedef struct ns_pkt_buf {
  uint8_t* hdr;        /* Header.View(); NS_PKB_FILL writes checksum fields here */
  uint64_t hdr_len;
  const ns_view* data; /* Data.Views()                                        */
  uint32_t ndata;
  uint32_t flags;      /* reserved, 0                                         */
  uint64_t data_size;  /* Data.Size() (<= the views' total: CapLength)       */
} ns_pkt_buf;

/* NS_PKB_VERIFY — a received batch (a recvmmsg batch as the link layer
 * delivers it: Data holds the IP packet, Header is empty), the checksum steps
 * of the receive path after IPv4/IPv6 HandlePacket's checks and trims:
 *   TCP: segment.parse (segment.go:174-180), valid iff the sum is 0xffff;
 *   ICMPv4 echo request: handleICMP's ^ChecksumVV(Data with the field
 *     zeroed) == the field (network/ipv4/icmp.go:72-80);
 *   ICMPv6: ICMPv6Checksum(first view, src, dst, the other views) == the
 *     field (network/ipv6/icmp.go:76-84).
 * verdict[i]: NS_PKB_VALID / NS_PKB_INVALID; NS_PKB_UNCHECKED where the
 * reference verifies nothing on receive (UDP, other protocols, ICMPv4 other
 * than echo) and for IPv4 fragments, whose transport checksum can only be
 * checked after reassembly (ipv4.go:375-385; the receive contract in
 * INTEGRATION.md §2 says who checks it then); NS_PKB_MALFORMED where IsValid,
 * HandlePacket's fragment checks (no payload, or a uint16
 * FragmentOffset() + size - 1 that wraps: ipv4.go:357-373) or the
 * transport's length checks drop the packet first: a transport first view
 * under 20 B for TCP (or a DataOffset outside [20, that view]) and under 8 B
 * for UDP (stack/nic.go:851, segment.go:159), ICMPv4 (ipv4/icmp.go:60) and
 * ICMPv6 (ICMPv6MinimumSize, ipv6/icmp.go:68; not the 4-B ICMPv6HeaderSize).
 * NS_PKB_FILL — a batch to transmit: Header holds the IP header and the
 * transport header (Data the payload); writes ^sum into the transport
 * checksum field — TCP buildTCPHdr (connect.go:653-663), UDP sendUDP
 * (udp/endpoint.go:808-815), ICMPv4 echo reply (icmp.go:96-100), ICMPv6
 * ICMPv6Checksum — and into the IPv4 header checksum (addIPHeader,
 * ipv4.go:236).  An IPv4 fragment (MF set or a fragment offset) gets only
 * its IP header checksum, as writePacketFragments writes it (ipv4.go:159-160).
 * NS_EINVAL for a Header or a clipped Data view of 4 GiB or more (one
 * descriptor's length is a u32, as for every view-taking entry point).
 * NS_EINVAL if a field to write lies outside Header (for IPv4, the whole IP
 * header must lie in Header).
 * sums (2n, or NULL): [2i] the IPv4 header sum (0 for IPv6), [2i+1] the
 * transport chain's un-complemented sum (0 when there is none).
 * All sums of the batch are one device pass.                                */
#define NS_PKB_VERIFY 1u
#define NS_PKB_FILL 2u
#define NS_PKB_INVALID 0u
#define NS_PKB_VALID 1u
#define NS_PKB_UNCHECKED 2u
#define NS_PKB_MALFORMED 3u
int ns_csum_packet_buffers(ns_csum_ctx* ctx, const ns_pkt_buf* pkts, uint32_t n,
                           uint32_t op, uint16_t* sums, uint8_t* verdict);

/* ---- a receive ring in HBM, verified without host planning ---------------
 * The receive mirror of ns_csum_tcp_tx: n slots of `stride` bytes from
 * d_arena + ring_off, slot s holding one frame as recvmmsg wrote it (its
 * length d_len[s], u32 device memory, counts from the slot's first byte).
 * The kernel parses every frame itself and gives, per slot, exactly the
 * verdict and sums ns_csum_packet_buffers(NS_PKB_VERIFY) gives for that
 * packet delivered the way the link delivers it:
 *   recvMMsgDispatcher.dispatch (link/fdbased/packet_dispatchers.go:258-317):
 *     the frame is [frame_at, len) of the slot (frame_at: bytes before it,
 *     e.g. a 10-B virtio-net header); a frame of no more than link_hdr bytes
 *     is dropped (MALFORMED); link_hdr = 14 (Ethernet) picks IPv4/IPv6 by
 *     EtherType (0x0800 / 0x86dd; any other: UNCHECKED, nothing the reference
 *     checksums), link_hdr = 0 (TUN) by the version nibble (others dropped:
 *     MALFORMED); Data = the frame less its link header, in views whose first
 *     holds first_view - link_hdr bytes (BufConfig[0] = 128, :30; the later
 *     views, all of even length, do not change any sum), first_view = 0: one
 *     view;
 *   then the rules of NS_PKB_VERIFY above (IsValid against the first view,
 *   fragments UNCHECKED or MALFORMED, segment.parse, ICMPv4 echo, ICMPv6).
 * d_verdict[s] (u8, or NULL) gets NS_PKB_*; d_sums (2n u16, or NULL) [2s] the
 * IPv4 header sum, [2s+1] the transport sum, as ns_csum_packet_buffers.
 * A slot whose length exceeds the stride is MALFORMED and counted
 * (ns_csum_sync).  Asynchronous on `stream`; no scratch, no host work per
 * packet.  Bytes read per slot: its frame (up to the IP packet's 65,575-B
 * limit) and its length; written: 1 + 4.
 * NS_EINVAL: d_arena + ring_off or stride not 16-B aligned, stride 0 or
 * >= 2^24, frame_at + link_hdr odd or frame_at >= stride, link_hdr not 0 or 14,
 * first_view neither 0 nor an even length with first_view - link_hdr >= 64,
 * flags != 0, NULL d_len (n > 0), both outputs NULL.
 * NS_ERANGE: the ring past the arena.                                       */
typedef struct ns_rx_ring {
  uint64_t ring_off;    /* arena offset of slot 0                            */
  uint64_t stride;      /* bytes per slot                                    */
  uint32_t n;           /* slots                                             */
  uint16_t frame_at;    /* where the link frame starts in a slot              */
  uint16_t link_hdr;    /* 0 (TUN) or 14 (Ethernet)                          */
  uint32_t first_view;  /* the link's first buffer view (128), 0: one view   */
  uint32_t flags;       /* reserved, 0                                       */
} ns_rx_ring;
int ns_csum_rx_ring(ns_csum_ctx* ctx, const uint8_t* d_arena, uint64_t arena_bytes,
                    const ns_rx_ring* ring, const uint32_t* d_len, uint16_t* d_sums,
                    uint8_t* d_verdict, void* stream);
/* The same checks over buffers at per-packet offsets in one device arena
 * (a NIC's buffer pool, not a fixed-stride ring): packet k's frame is in the
 * buffer at d_arena + ring->ring_off + d_off[k] (16-B aligned) of
 * ring->stride bytes (the buffers' capacity, a multiple of 16), with d_len[k]
 * bytes received; the other ns_rx_ring fields as above (n, frame_at,
 * link_hdr, first_view).  arena_bytes - ring_off must be below 4 GiB - 512
 * (32-bit offsets).  A buffer not 16-B aligned or not inside the arena gets
 * NS_PKB_MALFORMED and sums 0, and is counted by ns_csum_sync.  Asynchronous
 * on `stream`.                                                              */
int ns_csum_rx_bufs(ns_csum_ctx* ctx, const uint8_t* d_arena, uint64_t arena_bytes,
                    const ns_rx_ring* ring, const uint32_t* d_off, const uint32_t* d_len,
                    uint16_t* d_sums, uint8_t* d_verdict, void* stream);
/* The same ring in HOST memory (recvmmsg's buffers as the link endpoint
 * fills them): h_arena, h_len, h_sums and h_verdict are host pointers, the
 * ring's own alignment is free (ring_off need not be 16-B aligned; the stride
 * still must be a multiple of 16).  The slots go to the device in chunks of
 * whole slots (up to the context's staging size), four in flight; verdicts
 * and sums come back through mapped memory.  No host planning: the parse
 * runs on the device.  Synchronous.  Errors as for ns_csum_rx_ring.
 * Calls on one context share its host pipeline: a ring (even one small
 * enough for the BAR stage, within 1 MiB) waits for any ns_csum_batch_host,
 * _tcp_tx_host or _rx_ring_host call already running on that context; the
 * zero-copy passes of the single-buffer calls do not.  Use a context per
 * thread where that wait matters.                                           */
int ns_csum_rx_ring_host(ns_csum_ctx* ctx, const uint8_t* h_arena, uint64_t arena_bytes,
                         const ns_rx_ring* ring, const uint32_t* h_len, uint16_t* h_sums,
                         uint8_t* h_verdict);

/* header.ChecksumCombine(a, b)                     checksum.go:104-107      */
uint16_t ns_csum_combine(uint16_t a, uint16_t b);

/* ---- multi-GPU sharding -------------------------------------------------
 * ns_csum_batch_multi: one host batch over nctx contexts (normally one per
 * device): the table is split by ns_csum_shard_plan, each shard runs
 * ns_csum_batch_host on its own context from its own host thread, results
 * land in h_out in table order.  Shards are independent (per-packet
 * arithmetic): no collective, no peer traffic.  Synchronous.                */
int ns_csum_batch_multi(ns_csum_ctx* const* ctxs, uint32_t nctx,
                        const uint8_t* h_arena, uint64_t arena_bytes,
                        const ns_pkt_desc* h_desc, uint32_t n, uint16_t* h_out,
                        uint32_t batch_flags);
/* ns_csum_tcp_tx_host_multi: ns_csum_tcp_tx_host's calls over nctx contexts
 * (normally one per device, each with its own PCIe link): the calls are cut
 * into nctx consecutive parts balanced by the bytes each uploads (a call may
 * be split between segments), each part runs ns_csum_tcp_tx_host on its own
 * context from its own host thread, and h_out (or NULL) holds the sums in
 * call order as for one context.  No collective.  Synchronous.             */
int ns_csum_tcp_tx_host_multi(ns_csum_ctx* const* ctxs, uint32_t nctx,
                              uint8_t* h_arena, uint64_t arena_bytes,
                              const ns_tcp_tx* txs, uint32_t count,
                              uint16_t* h_out);

/* ---- (sharding plan) ----------------------------------------------------
 * Splits n descriptors into `parts` contiguous ranges with near-equal payload
 * bytes (prefix sum of len, cut at byte quantiles).  first[p] = index of the
 * first descriptor of part p; first[parts] = n.  Pure host arithmetic.      */
int ns_csum_shard_plan(const ns_pkt_desc* h_desc, uint32_t n, uint32_t parts,
                       uint32_t* first);

/* ---- diagnostics ----------------------------------------------------------
 * Where a context's host time went, so a slow synchronous call can be placed
 * on one path (no reference counterpart: instrumentation of this boundary).
 * Times are host wall-clock nanoseconds.  ns_csum_get_stats copies the
 * counters; with reset != 0 it also zeroes them.                            */
typedef struct ns_csum_stats {
  uint64_t calls;            /* synchronous calls returned (ns_csum_checksum,
                                _vv_*, _views_restart, _pseudo_header, _chains,
                                _packet_buffers, _batch_host)                  */
  uint64_t call_ns_max;      /* the longest of them, entry to return          */
  uint64_t lock_ns_max;      /* longest wait for the context lock by a pass   */
  uint64_t zc_passes;        /* zero-copy passes run                          */
  uint64_t zc_late;          /* ...whose completion word was not in after
                                2 ms (the caller then waited on the stream);
                                also counts the small host-ring / host-TX
                                passes (ns_csum_rx_ring_host, _tcp_tx_host
                                within 1 MiB) that were late the same way    */
  uint64_t zc_pass_ns_max;   /* longest pass, launch to results               */
  uint64_t growths;          /* stream-ordered scratch growths (batch_dev)    */
  uint64_t growth_ns_total;  /* host time in hipFreeAsync/hipMallocAsync/
                                hipMemsetAsync for them                       */
  uint64_t growth_ns_max;
  uint64_t retires;          /* scratch entries retired (LRU bound, release)  */
  uint64_t retire_ns_max;    /* longest retire, incl. creating its stream     */
  uint64_t stage_allocs;     /* staging buffers allocated (pool was empty)    */
  uint64_t stage_alloc_ns_max;
} ns_csum_stats;
int ns_csum_get_stats(ns_csum_ctx* ctx, ns_csum_stats* out, int reset);

/* A/B and test knobs of ns_csum_tcp_tx on this context (no reference
 * counterpart; every result is the same whatever they are): variant (0 =
 * production: the payload pass in 8-lane groups, header stores written
 * through; 1 one fused pass; with the windowed payload pass: 2 nontemporal
 * write-back, 3 segments reduced over the wave, 4 the one-shot header pass;
 * 5 the group pass with default-policy header stores; 6 round 5's
 * production, windowed with default-policy stores; 7 production with the
 * persistent header pass),
 * tile / htile (segments per wave of the fused pass or the windowed payload
 * pass — a tile set here selects the windowed pass — and of the header
 * pass; 0 = the launcher's choice), passes (0 = by
 * size, 1 = fused, 2 = two passes).  Read by each call without a lock; set
 * them while no ns_csum_tcp_tx call runs on the context.  ns_csum_init takes
 * their initial values from NS_CSUM_TX_VARIANT / _TILE / _HTILE / _PASSES,
 * once.  NS_EINVAL for a variant above 7 or passes above 2.                 */
int ns_csum_set_tx_tuning(ns_csum_ctx* ctx, uint32_t variant, uint32_t tile, uint32_t htile,
                          uint32_t passes);

#ifdef __cplusplus
}
#endif
#endif /* NETSTACK_CSUM_H_ */
