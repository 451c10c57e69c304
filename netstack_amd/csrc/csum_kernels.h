// Internal launcher interface between the C ABI (csum_api.cpp) and the gfx950
// kernels (csum_kernels.hip).  Not installed; the public boundary is
// include/netstack_csum.h.
#pragma once
#include <hip/hip_runtime_api.h>
#include <stdint.h>

namespace nsk {

// Enqueue the checksum of n descriptors (16-byte ns_pkt_desc, device memory)
// over `arena` on `stream`.  With `chain` set (a chained-batch scratch, layout
// below) the per-descriptor partial sums and continuation flags go there and
// a fold pass folds NS_DESC_CONT runs into `out`; otherwise every descriptor
// is independent.
// Out-of-range descriptors are summed as empty and counted in *err.
// `sizing_bytes` (0: arena_bytes) is the byte count the launcher sizes tiles
// by — the payload of a batch whose "arena" is the whole address space
// (arena = nullptr, descriptors holding absolute addresses).
// `store`: descriptors flagged NS_DESC_STORE write their final result into
// the (then writable) arena.
// `split`: scratch for csum_split (see below), or nullptr.
//
// Chained-batch scratch: `partial`, chain_scratch_words(n) u32 — the n
// partial sums, then their u16 flags from chain_flag_word(n) (16-B aligned);
// and `status`, chain_blocks(n) u64 fold statuses (one per kFoldBlock
// descriptors, csum_kernels.hip run folding) in a buffer of their own that
// holds nothing but status words.  Statuses are tagged with a process-wide
// launch generation, so stale ones are ignored; the status buffer is zeroed
// when it is allocated, so no word in it can carry a live generation (a
// status array that shared its buffer with the partials could land on a
// previous launch's partials).  Neither needs clearing between launches.
// Concurrent chained launches need distinct scratch (csum_api.cpp keys it by
// stream).
constexpr uint32_t kFoldPer = 8;                 // descriptors per thread
constexpr uint32_t kFoldBlock = 256 * kFoldPer;  // descriptors per workgroup
constexpr uint64_t chain_flag_word(uint64_t n) { return (n + 3) & ~3ull; }
constexpr uint64_t chain_blocks(uint64_t n) { return (n + kFoldBlock - 1) / kFoldBlock; }
constexpr uint64_t chain_scratch_words(uint64_t n) { return (chain_flag_word(n) + ((n + 7) & ~7ull) / 2 + 3) & ~3ull; }

struct ChainScratch {
  uint32_t* partial = nullptr;  // chain_scratch_words(n) u32
  uint64_t* status = nullptr;   // chain_blocks(n) u64, zeroed at allocation
  bool walk = false;            // NS_OPT_FOLD_WALK (tests): no look-back, every carry-in walked
};

// A self-signalling launch (`zc.flag` set; unchained checksum tiles only, no
// `chain` and no `split`): results are written through to `out` (coherent
// host memory) and the launch's last workgroup stores `zc.seq` into
// `*zc.flag` (coherent host memory) once every result is complete; `zc.ctr`
// is a device counter that is zero between launches (each launch leaves it
// so).  The caller spins on the flag instead of launching a signal kernel.
struct ZcSignal {
  uint32_t* ctr = nullptr;
  uint32_t* flag = nullptr;
  uint32_t seq = 0;
};

// `store`: bit 0 = honour NS_DESC_STORE (ns_csum_batch_dev_store); bit 1 =
// NS_BATCH_PAIRED (an odd-indexed NS_DESC_CONT descriptor continues the one
// before it, folded inside the tile; not with `chain`, `split` or `zc`);
// bit 2 = plain write-back stores (A/B diagnostics).
hipError_t launch_batch(const uint8_t* arena, uint64_t arena_bytes,
                        const void* desc, uint32_t n, uint16_t* out,
                        ChainScratch chain, unsigned long long* err,
                        hipStream_t stream, uint64_t sizing_bytes = 0, uint32_t store = 0,
                        uint32_t* split = nullptr, ZcSignal zc = {});

// *taken = the error count, which is reset to 0 in the same atomic exchange
// (counts added by kernels still running on other streams are never lost).
// `taken` must be device-visible (mapped host memory).
hipError_t launch_take_err(unsigned long long* err, unsigned long long* taken, hipStream_t stream);

// Store `seq` into *flag (mapped fine-grained host memory) with a
// system-scope release once the stream's earlier work is done: the completion
// word a zero-copy pass's caller spins on.
hipError_t launch_signal(uint32_t* flag, uint32_t seq, hipStream_t stream);

// Rewrite n device-resident descriptors' offsets relative to `bias` (empty
// descriptors get 0): the host pipeline's per-chunk table rebase.
hipError_t launch_rebase(void* desc, uint32_t n, uint64_t bias, hipStream_t stream);

// Batches of few descriptors averaging >= split_min_avg() bytes take the
// split kernel when launch_batch gets `split`: a scratch of split_words(n)
// u32, zeroed once at allocation (every launch leaves it zero).
constexpr uint64_t split_min_avg() { return 1u << 20; }
constexpr uint64_t split_words(uint64_t n) { return 2 * n; }

// sendTCPBatch's transmit checksums from the batch geometry (tcp_tx.hip,
// ns_csum_tcp_tx).  Absolute device addresses; validated by the caller:
// n = ceil(size / mss) >= 1, mss <= 65535, every slot and the payload inside
// the arena, the headers inside a slot (each <= 60 B), the fields inside the
// headers, slots and payload disjoint.  tile = segments per wave (0: the
// launcher picks; at most 64 and 12 KiB of slots); lds_rows and lds_wave
// are set by the launcher.  out (or nullptr): [2i] the IPv4 sum, [2i+1] the TCP sum, both
// un-complemented.
constexpr uint32_t kTxIp = 1u;           // fill the IPv4 header checksum
constexpr uint32_t kTxTcpFull = 2u;      // fill ^(pseudo + payload + TCP header)
constexpr uint32_t kTxTcpPartial = 4u;   // fill the pseudo-header sum (CHECKSUM_PARTIAL)
constexpr uint32_t kTxFieldsOnly = 8u;   // store the 2-byte fields, not whole slots
struct TxGeo {
  uint64_t hdr, pay, size, n;
  uint32_t mss, slot, tile, lds_wave;
  uint32_t ip_at, ip_len, tcp_at, tcp_len;
  uint32_t addr_sum, proto, mode, lds_rows;
  uint16_t* out;
  uint32_t wpg, pad;  // waves (tiles) per workgroup, set by the launcher
  uint16_t* xs;          // the two-pass shape's payload values (xs[i * xstride]), or nullptr
  uint32_t htile;        // the header pass's tile (0: the launcher's choice)
  uint32_t xstride;      // 1 (scratch) or 2 (parked in out[2i + 1])
};
// A batch whose payload needs reading takes two passes (a payload pass, then
// a header pass: g.xs set) from this many payload bytes, one fused pass below
// (g.xs = nullptr).  tools/tx_struct_probe.py, 1460-B segments, two passes
// against one: 16 MB 15.5 vs 13.1 us, 191 MB 41.2 vs 42.5, 383 MB 72.2 vs
// 76.6, 1.5 GB 246 vs 271 (profiles/r04/tx_struct/sizes/).
constexpr uint64_t kTxTwoPassMinBytes = 64ull << 20;
// variant (A/B diagnostics; 0 = production: the payload pass in 8-lane
// groups, the header pass's stores nt sc1): 1 = one fused pass, 2 = windowed
// payload pass + nontemporal write-back, 3 = windowed, segments reduced over
// the wave in the loop, 4 = windowed + the one-shot header pass (tcp_tx
// PH = 2), 5 = group payload pass + default-policy header stores, 6 =
// round 5's production (windowed + default-policy stores), 7 = production
// with the persistent header pass (2 tiles per wave in flight).
hipError_t launch_tcp_tx(TxGeo g, hipStream_t stream, uint32_t variant = 0);
// Many batches in one fused launch (ns_csum_tcp_tx_multi).  calls[] (host)
// hold each batch's geometry with n, mode and out set; tx_multi_prepare sets
// their tiles, fills first[ncalls + 1] and the launch-wide shape, and returns
// the grid (0: more than 2^31 tiles).  The launch reads calls[] and first[]
// from device memory (d_calls, d_first: copies of them).
uint32_t tx_multi_prepare(TxGeo* calls, uint32_t ncalls, TxGeo* launch, uint32_t* first);
hipError_t launch_tcp_tx_multi(const TxGeo& launch, uint32_t grid, const TxGeo* d_calls, const uint32_t* d_first,
                               uint32_t ncalls, hipStream_t stream);

// The receive ring's shape for descriptor tables (tbl_ring.hip): one 8-lane
// group per descriptor.  Measured against csum_hyb's big-packet instance on
// cfg2 and not taken (tools/grp_probe.py); built only into
// the timing-variants library.
bool tbl_ring_eligible(const uint8_t* arena, uint64_t arena_bytes, uint32_t n, uint64_t sizing_bytes);
hipError_t launch_tbl_ring(const uint8_t* arena, uint64_t arena_bytes, const void* desc, uint32_t n, uint16_t* out,
                      unsigned long long* err, hipStream_t stream, uint32_t lines = 0);
constexpr uint64_t kGrpMinAvg = 1024, kGrpMaxAvg = 16384;

// A receive ring verified on the device (rx_ring.hip, ns_csum_rx_ring).
// Absolute device addresses; validated by the caller: ring and stride
// 16-B aligned, stride < 2^24, frame_at + link even, view0 = 0 or >= 64 and
// even.  Per slot s: the received length len[s] (bytes from the slot's first
// byte); verdict[s] (NS_PKB_*) and sums[2s], sums[2s + 1] (or nullptr).
struct RxGeo {
  uint64_t ring, stride;
  const uint32_t* len;
  uint16_t* sums;
  uint8_t* verdict;
  unsigned long long* err;
  uint32_t n;
  uint32_t frame_at;  // bytes before the link frame in a slot (a virtio-net header)
  uint32_t link;      // 0: the frame is the IP packet; 14: Ethernet
  uint32_t view0;     // the IP packet's first view (BufConfig[0] - link), 0: one view
  // A buffer list instead of a ring (ns_csum_rx_bufs): packet s in the buffer
  // at ring + off[s] (16-B aligned) of `stride` bytes, inside `limit` bytes
  // from `ring` (< 4 GiB); nullptr: the ring's slots.
  const uint32_t* off;
  uint64_t limit;
  // Timing variants only (tools/rx_ring_variants.hip 30-34; zero in the
  // product): a buffer list sorted into bk_nb buckets of 2^bk_shift arena
  // bytes first (bk_tup[j] = (off, len, list index, 0), bucket by bucket),
  // the parse then run over bk_tup (LIST = 2).  bk_total (bk_nb words) is
  // zero before the sort and left zero by the parse; bk_wgoff holds bk_nb
  // words per 4,096 list entries.
  uint4* bk_tup;
  uint32_t* bk_total;
  uint32_t* bk_wgoff;
  uint32_t bk_shift, bk_nb;
};
hipError_t launch_rx_ring(const RxGeo& g, hipStream_t stream);

}  // namespace nsk
