// tcp_tx.hip — the transmit checksums of sendTCPBatch (transport/tcp/
// connect.go:668-702) taken from the batch's geometry instead of a
// descriptor table (ns_csum_tcp_tx, include/netstack_csum.h).
//
// The layout is the one sendTCPBatch builds.  stack.NewPacketDescriptors(n,
// hdrSize) allocates ONE buffer of n slots of hdrSize bytes (stack/route.go:
// 181-188); buildTCPHdr prepends the TCP header in slot i and addIPHeader the
// IPv4 header before it; the payload is one VectorisedView, segment i at
// Off = i * MSS, Size = min(MSS, what is left) (connect.go:679-692).  Per
// segment the reference computes
//   tcp: xsum = PseudoHeaderChecksum(6, src, dst, tcp_len + size)    checksum.go:112-122
//        xsum = ChecksumVVWithOffset(data, xsum, off, size)           connect.go:662
//        field = ^Checksum(tcp[:DataOffset], xsum)                    connect.go:663, tcp.go:259-262
//        (or field = xsum of the pseudo-header alone: CHECKSUM_PARTIAL, connect.go:655-660)
//   ip:  field = ^Checksum(ip[:IHL], 0)                               ipv4.go:236, :251-253
// with both fields zero while they are summed (freshly encoded headers).
//
// One wave owns a tile of `tile` consecutive segments: their payload bytes
// are one contiguous span and their header slots one contiguous region.
//   1. The wave starts an LDS-DMA copy of its header region (no registers).
//   2. It streams the payload span in aligned 1-KiB windows (lane l reads
//      16 B at window + 16 l, nontemporal: every 128-B line consumed by one
//      instruction), U windows in flight.  Each lane keeps the little-endian
//      word sum W of its bytes (one v_sad_u16 per dword).  Segment ends are
//      wave-uniform: a window holding one splits the straddling lane's chunk
//      with scalar byte masks, and each lane parks its partial in the
//      finished segment's LDS row; lane j sums row j at the end.
//   3. Lane j sums its slot's IPv4 and TCP headers from LDS (the fields read
//      as zero), folds everything as the Go code does, and writes the two
//      fields into the LDS copy.
//   4. The wave writes its header region back whole (16-B stores of full
//      chunks; byte stores where a chunk is shared with a neighbouring
//      tile): whole-line writes instead of 2M scattered 2-byte stores
//      (tools/dense_store_probe.hip).
// Batches of 64 MiB of payload or more split that into two kernels (PH): a
// payload pass (step 2, each segment's payload value to g.xs) and a header
// pass (steps 1, 3, 4), because the slot writes cost ~45 us per 1M segments
// when they are interleaved with the payload stream and ~12 us on their own.
// A header pass's lanes loop over up to 256 segments per wave.
//
// Arithmetic.  A segment holds at most 65,535 bytes, so no sum here wraps a
// uint32 and each folded value depends on W only through W mod 65535 and
// whether it is zero (csum_kernels.hip, kWOnlyMaxChunks / s_class): the
// result is bit-exact with the Go code for every byte pattern.
#include <hip/hip_runtime.h>
#include <stdint.h>

#include <algorithm>

#include "csum_kernels.h"

namespace nsk {
namespace {

// ChecksumCombine(uint16(v), uint16(v>>16)) — checksum.go:45, :104-107.
__device__ __forceinline__ uint32_t tx_fold(uint32_t v) {
  const uint32_t s = (v & 0xFFFFu) + (v >> 16);
  return (s + (s >> 16)) & 0xFFFFu;
}

// A W total as a value with the fold behaviour of Go's S for a piece whose
// first byte is at an address of parity `phase` (csum_kernels.hip s_class).
__device__ __forceinline__ uint32_t tx_class(uint32_t W, uint32_t phase) {
  const uint32_t w = tx_fold(W);
  return phase ? w : tx_fold(w << 8);
}

__device__ __forceinline__ uint32_t wsum4(const uint4 v, uint32_t acc) {
  acc = __builtin_amdgcn_sad_u16(v.x, 0u, acc);
  acc = __builtin_amdgcn_sad_u16(v.y, 0u, acc);
  acc = __builtin_amdgcn_sad_u16(v.z, 0u, acc);
  return __builtin_amdgcn_sad_u16(v.w, 0u, acc);
}

__device__ __forceinline__ uint32_t below(int c) {  // bytes [0, c) of a dword, c clamped to [0, 4]
  c = c < 0 ? 0 : (c > 4 ? 4 : c);
  return c >= 4 ? 0xFFFFFFFFu : ((1u << (8 * c)) - 1u);
}

// Sum over the 64 lanes of the wave; every lane gets the (uniform) total.
__device__ __forceinline__ uint32_t wave_total(uint32_t s) {
  s += (uint32_t)__builtin_amdgcn_update_dpp(0, (int)s, 0xB1, 0xF, 0xF, false);   // quad_perm 1,0,3,2
  s += (uint32_t)__builtin_amdgcn_update_dpp(0, (int)s, 0x4E, 0xF, 0xF, false);   // quad_perm 2,3,0,1
  s += (uint32_t)__builtin_amdgcn_update_dpp(0, (int)s, 0x141, 0xF, 0xF, false);  // row_half_mirror
  s += (uint32_t)__builtin_amdgcn_update_dpp(0, (int)s, 0x140, 0xF, 0xF, false);  // row_mirror
  return (uint32_t)__builtin_amdgcn_readlane((int)s, 0) + (uint32_t)__builtin_amdgcn_readlane((int)s, 16) +
         (uint32_t)__builtin_amdgcn_readlane((int)s, 32) + (uint32_t)__builtin_amdgcn_readlane((int)s, 48);
}

__device__ __forceinline__ __amdgpu_buffer_rsrc_t tx_srd(uint64_t base, uint32_t nrec) {
  // readfirstlane returns int: widen through uint32_t
  const uint32_t lo = (uint32_t)__builtin_amdgcn_readfirstlane((uint32_t)base);
  const uint32_t hi = (uint32_t)__builtin_amdgcn_readfirstlane((uint32_t)(base >> 32));
  return __builtin_amdgcn_make_buffer_rsrc((void*)(((uint64_t)hi << 32) | (uint64_t)lo), (short)0,
                                           (int)__builtin_amdgcn_readfirstlane(nrec), 0x00020000);
}

template <int AUX>
__device__ __forceinline__ uint4 tx_load(__amdgpu_buffer_rsrc_t r, uint32_t off) {
  auto x = __builtin_amdgcn_raw_buffer_load_b128(r, (int)off, 0, AUX);
  return *reinterpret_cast<uint4*>(&x);
}

// The W sum of LDS bytes [a, a + len) (len <= 60), dword reads with masks;
// `zero` (an offset inside the range, or ~0u) is a 2-byte field read as zero.
template <int MAXD>
__device__ __forceinline__ uint32_t lds_wsum(const uint8_t* L, uint32_t a, uint32_t len, uint32_t zero) {
  const uint32_t* D = reinterpret_cast<const uint32_t*>(L);
  const uint32_t d0 = a >> 2;
  const uint32_t nd = ((a + len + 3) >> 2) - d0;
  uint32_t w = 0;
#pragma unroll
  for (int k = 0; k < MAXD; ++k) {
    if ((uint32_t)k < nd) {
      const int b = (int)(4 * (d0 + k));
      uint32_t m = below((int)(a + len) - b) & ~below((int)a - b);
      if (zero != ~0u) m &= ~(below((int)(zero + 2) - b) & ~below((int)zero - b));
      w = __builtin_amdgcn_sad_u16(D[d0 + k] & m, 0u, w);
    }
  }
  return w;
}

// lds_wsum as a loop (no unrolling): fewer registers where two tiles are in
// flight (tcp_tx_hdr).
__device__ __forceinline__ uint32_t lds_wsum_loop(const uint8_t* L, uint32_t a, uint32_t len, uint32_t zero) {
  const uint32_t* D = reinterpret_cast<const uint32_t*>(L);
  const uint32_t d0 = a >> 2;
  const uint32_t nd = ((a + len + 3) >> 2) - d0;
  uint32_t w = 0;
#pragma nounroll
  for (uint32_t k = 0; k < nd; ++k) {
    const int b = (int)(4 * (d0 + k));
    uint32_t m = below((int)(a + len) - b) & ~below((int)a - b);
    m &= ~(below((int)(zero + 2) - b) & ~below((int)zero - b));
    w = __builtin_amdgcn_sad_u16(D[d0 + k] & m, 0u, w);
  }
  return w;
}

__device__ __forceinline__ void lds_put_be16(uint8_t* L, uint32_t at, uint32_t v) {
  L[at] = (uint8_t)(v >> 8);
  L[at + 1] = (uint8_t)v;
}

// A relaxed agent-scope 2-byte store (written through), or two byte stores
// at an odd address (csum_kernels.hip store_result).
__device__ __forceinline__ void tx_store_be16(uint64_t addr, uint32_t v) {
  uint8_t* p = reinterpret_cast<uint8_t*>((uintptr_t)addr);
  if (!(addr & 1u)) {
    __hip_atomic_store(reinterpret_cast<uint16_t*>(p), (uint16_t)(((v & 0xFFu) << 8) | ((v >> 8) & 0xFFu)),
                       __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  } else {
    p[0] = (uint8_t)(v >> 8);
    p[1] = (uint8_t)v;
  }
}

// The header pass's store cache policy (SP): 0 default, 1 nt, then the
// scope bits, A/B only: 2 sc1, 3 sc0 sc1, 4 nt sc1, 5 sc0, 6 sc0 nt sc1
// (buffer aux: 1 = sc0, 2 = nt, 16 = sc1).
constexpr int tx_store_aux(int sp) {
  return sp == 1 ? 2 : sp == 2 ? 16 : sp == 3 ? 17 : sp == 4 ? 18 : sp == 5 ? 1 : sp == 6 ? 19 : 0;
}

}  // namespace

// Step 3 of a tile (below): lane l finishes segments s0 + l, s0 + l + 64, ...
// of the tile whose slots sit in LDS from byte `ho` (h_lo - h_base): sums
// the IPv4 and TCP headers (the fields read as zero), folds them with the
// pseudo-header and the payload value (wres, or g.xs in the header pass), as
// the Go code does, and writes both fields into the LDS copy (and d_out; or
// straight to the slots with kTxFieldsOnly).
template <int PH>
__device__ __forceinline__ void tx_fields(const TxGeo& g, uint64_t s0, uint32_t nseg, uint8_t* L, uint32_t ho,
                                          uint32_t lane, uint32_t wres) {
  const uint64_t h_lo = g.hdr + s0 * g.slot;
  for (uint32_t j = lane; j < nseg; j += 64) {
    const uint32_t o = ho + j * g.slot;  // slot j in LDS
    const uint64_t si = s0 + j;
    const uint32_t size = si + 1 < g.n ? g.mss : (uint32_t)(g.size - (g.n - 1) * (uint64_t)g.mss);
    uint32_t ipv = 0, tcpv = 0;
    if (g.mode & kTxIp) {
      const uint32_t a = o + g.ip_at;
      ipv = tx_fold(tx_class(lds_wsum<16>(L, a, g.ip_len, a + 10u), a & 1u));  // Checksum(ip[:IHL], 0)
      lds_put_be16(L, a + 10u, ~ipv & 0xFFFFu);
    }
    if (g.mode & (kTxTcpFull | kTxTcpPartial)) {
      uint32_t x = tx_fold(g.addr_sum + ((g.tcp_len + size) & 0xFFFFu));  // PseudoHeaderChecksum
      x = tx_fold(x + g.proto);
      const uint32_t a = o + g.tcp_at;
      if (g.mode & kTxTcpFull) {
        // PH 3: the payload value itself was handed in as wres (one segment per lane)
        const uint32_t pv = PH == 2 ? (uint32_t)g.xs[si * g.xstride]
                            : PH == 3 ? wres
                                      : tx_class(wres, (uint32_t)((g.pay + si * g.mss) & 1u));
        x = tx_fold(x + pv);                                                            // ChecksumVVWithOffset
        x = tx_fold(x + tx_class(lds_wsum<16>(L, a, g.tcp_len, a + 16u), a & 1u));     // CalculateChecksum
        lds_put_be16(L, a + 16u, ~x & 0xFFFFu);
      } else {
        lds_put_be16(L, a + 16u, x);
      }
      tcpv = x;
    }
    if (g.out) {
      g.out[2 * si] = (uint16_t)ipv;
      g.out[2 * si + 1] = (uint16_t)tcpv;
    }
    if (g.mode & kTxFieldsOnly) {  // only the 2-byte fields, as csum_hyb stores them
      const uint64_t slot = h_lo + (uint64_t)j * g.slot;
      if (g.mode & kTxIp) tx_store_be16(slot + g.ip_at + 10u, ~ipv & 0xFFFFu);
      if (g.mode & kTxTcpFull) tx_store_be16(slot + g.tcp_at + 16u, ~tcpv & 0xFFFFu);
      if (g.mode & kTxTcpPartial) tx_store_be16(slot + g.tcp_at + 16u, tcpv);
    }
  }
}

// Step 4: the tile's region [h_lo, h_hi) back from LDS, whole (16-B stores of
// full chunks; byte stores where a chunk is shared with a neighbouring tile).
template <int SP>
__device__ __forceinline__ void tx_writeback(const uint8_t* L, uint64_t h_lo, uint64_t h_hi, uint64_t h_base,
                                             uint32_t h_chunks, uint32_t lane) {
  const uint4* L4 = reinterpret_cast<const uint4*>(L);
  for (uint32_t c = lane; c < h_chunks; c += 64) {
    const uint64_t at = h_base + (uint64_t)c * 16u;
    if (at >= h_lo && at + 16 <= h_hi) {
      uint4* p = reinterpret_cast<uint4*>((uintptr_t)at);
      if constexpr (SP == 1) {
        const uint4 x = L4[c];
        uint32_t* q = reinterpret_cast<uint32_t*>(p);
        __builtin_nontemporal_store(x.x, q);
        __builtin_nontemporal_store(x.y, q + 1);
        __builtin_nontemporal_store(x.z, q + 2);
        __builtin_nontemporal_store(x.w, q + 3);
      } else {
        *p = L4[c];
      }
    } else {  // a chunk shared with the neighbouring tile: only this tile's bytes
      for (uint32_t k = 0; k < 16; ++k)
        if (at + k >= h_lo && at + k < h_hi) reinterpret_cast<uint8_t*>((uintptr_t)at)[k] = L[c * 16u + k];
    }
  }
}

// Step 4 through the tile's buffer resource (hr: [h_base, h_base + 16
// h_chunks)): buffer stores, which count in vmcnt only.  A flat store would
// make every later LDS access wait for all of the wave's memory operations
// (flat_* complete out of order: vmcnt(0) and lgkmcnt(0)), which in a loop
// over tiles drains the next tile's prefetch too.
template <int SP>
__device__ __forceinline__ void tx_writeback_buf(const uint8_t* L, __amdgpu_buffer_rsrc_t hr, uint64_t h_lo,
                                                 uint64_t h_hi, uint64_t h_base, uint32_t h_chunks, uint32_t lane) {
  const uint4* L4 = reinterpret_cast<const uint4*>(L);
  const uint32_t lo = (uint32_t)(h_lo - h_base), hi = (uint32_t)(h_hi - h_base);
  for (uint32_t c = lane; c < h_chunks; c += 64) {
    const uint32_t at = c * 16u;
    if (at >= lo && at + 16 <= hi) {
      const uint4 x = L4[c];
      __builtin_amdgcn_raw_buffer_store_b128(*reinterpret_cast<const __attribute__((ext_vector_type(4))) uint32_t*>(&x),
                                             hr, (int)at, 0, tx_store_aux(SP));
    } else {  // a chunk shared with the neighbouring tile: only this tile's bytes
      for (uint32_t k = 0; k < 16; ++k)
        if (at + k >= lo && at + k < hi) __builtin_amdgcn_raw_buffer_store_b8(L[at + k], hr, (int)(at + k), 0, 0);
    }
  }
}

// U = payload windows (1 KiB per wave each) in flight; AUX = payload load
// policy (2 = nontemporal); SP = header write-back policy (0 plain, 1 nt);
// RED = how a finished segment's lane sums meet: 0 = reduced over the wave
// at once (DPP + readlane), 1 = each lane's partial parked in an LDS row of
// the segment, summed by the segment's lane at the end (no cross-lane
// dependency inside the stream loop), 2 = not at all (timing probes only:
// wrong sums); XF & 1 (timing probes only): no write-back.
// PH = the pass: 0 = everything in one kernel; 1 = the payload pass (each
// segment's payload value to g.xs, no headers); 2 = the header pass (the
// payload values from g.xs, no payload read).
// One wave's tile: segments [s0, s0 + tile) of batch g, its LDS share L
// (header region, then `rows`).
template <int U, int AUX, int SP, int RED, int XF, int PH>
__device__ __forceinline__ void tx_tile(const TxGeo& g, uint64_t s0, uint8_t* L, uint32_t* rows, uint32_t lane) {
  if (s0 >= g.n) return;  // a whole wave leaves together
  const uint32_t nseg = g.n - s0 < g.tile ? (uint32_t)(g.n - s0) : g.tile;

  // 1. the header region, into LDS by DMA
  const uint64_t h_lo = g.hdr + s0 * g.slot, h_hi = h_lo + (uint64_t)nseg * g.slot;
  const uint64_t h_base = h_lo & ~15ull;
  const uint32_t h_chunks = (uint32_t)((h_hi - h_base + 15) >> 4);
  const __amdgpu_buffer_rsrc_t hr = tx_srd(h_base, h_chunks * 16u);
  for (uint32_t c = 0; PH != 1 && c < h_chunks; c += 64) {
    const uint32_t o = (c + lane) * 16u;
    __builtin_amdgcn_raw_ptr_buffer_load_lds(hr, (__attribute__((address_space(3))) void*)(L + c * 16u), 16,
                                             o < h_chunks * 16u ? o : h_chunks * 16u, 0, 0, 0);
  }

  // 2. the payload span: lane j ends up with segment j's W total
  uint32_t wres = 0;
  if (PH != 2 && (g.mode & kTxTcpFull)) {
    const uint64_t p_lo = g.pay + s0 * g.mss;
    const uint64_t p_end = g.pay + g.size;
    const uint64_t p_hi = p_lo + (uint64_t)nseg * g.mss < p_end ? p_lo + (uint64_t)nseg * g.mss : p_end;
    const uint64_t p_base = p_lo & ~15ull;
    const uint32_t span = (uint32_t)(p_hi - p_base);  // < 2^32: tile * mss <= 64 * 65535
    const uint32_t nrec = (span + 15u) & ~15u;
    const __amdgpu_buffer_rsrc_t pr = tx_srd(p_base, nrec);
    const uint32_t nwin = (nrec / 16u + 63u) / 64u;
    // Segment ends, relative to p_base (uniform).  "Segment -1" ends where
    // the tile's first segment starts, and "segment nseg" holds what follows
    // the last one in its chunk: those bytes belong to the neighbouring
    // tiles and are dropped.
    int seg = -1;
    uint32_t nb = (uint32_t)(p_lo - p_base);  // where segment `seg` ends
    uint32_t pc = 0;                           // where the previous one ended
    uint32_t acc = 0;
    for (uint32_t w0 = 0; w0 < nwin; w0 += U) {
      uint4 v[U];
#pragma unroll
      for (int j = 0; j < U; ++j) {
        const uint32_t o = ((w0 + j) * 64u + lane) * 16u;
        v[j] = tx_load<AUX>(pr, o < nrec ? o : nrec);
      }
#pragma unroll
      for (int j = 0; j < U; ++j) {
        // (windows past the span read zeros and hold no segment end)
        uint32_t w = wsum4(v[j], 0u);
        const uint32_t wbase = (w0 + j) * 1024u;
        while (RED != 2 && nb < wbase + 1024u) {
          // lane lb holds the segment's last bytes [lo, cut) of its chunk
          const uint32_t c = nb - wbase, lb = c >> 4, cut = c & 15u;
          const uint32_t lo = ((pc >> 4) == (nb >> 4) && seg >= 0) ? (pc & 15u) : 0u;
          const uint32_t m0 = below((int)cut) & ~below((int)lo), m1 = below((int)cut - 4) & ~below((int)lo - 4),
                         m2 = below((int)cut - 8) & ~below((int)lo - 8), m3 = below((int)cut - 12) & ~below((int)lo - 12);
          const uint32_t part = wsum4(make_uint4(v[j].x & m0, v[j].y & m1, v[j].z & m2, v[j].w & m3), 0u);
          const uint32_t vc = lane < lb ? w : (lane == lb ? part : 0u);
          if constexpr (RED == 0) {
            const uint32_t tot = wave_total(acc + vc);
            if ((int)lane == seg) wres = tot;
          } else if constexpr (RED == 1) {
            if (seg >= 0) rows[(uint32_t)seg * 64u + lane] = acc + vc;
          }
          acc = 0;
          w -= vc;
          pc = nb;
          ++seg;
          // the last segment ends at the span's end: the rest of its last
          // chunk belongs to the next tile
          nb = (uint32_t)seg < nseg ? min(nb + g.mss, span) : 0xFFFFFFFFu;
        }
        acc += w;
      }
    }
    if constexpr (RED == 0) {
      const uint32_t tot = wave_total(acc);
      if ((int)lane == seg) wres = tot;
    } else if constexpr (RED == 1) {
      if ((uint32_t)seg < nseg) rows[(uint32_t)seg * 64u + lane] = acc;
      __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
      __builtin_amdgcn_wave_barrier();
      if (lane < nseg) {
        const uint4* r = reinterpret_cast<const uint4*>(rows + lane * 64u);
#pragma unroll
        for (int k = 0; k < 16; ++k) {
          const uint4 x = r[k];
          wres += x.x + x.y + x.z + x.w;
        }
      }
    } else {
      wres = acc;
    }
  }

  if constexpr (PH == 1) {  // the payload pass ends here
    if (lane < nseg) {
      const uint64_t si = s0 + lane;
      g.xs[si * g.xstride] = (uint16_t)tx_class(wres, (uint32_t)((g.pay + si * g.mss) & 1u));
    }
    return;
  }

  // 3. headers, then the fields: lane l takes segments s0 + l, s0 + l + 64, ...
  // (a pass that reads payload has at most 64, so lane j = segment j)
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");  // the LDS-DMA copy is in
  __builtin_amdgcn_wave_barrier();
  tx_fields<PH>(g, s0, nseg, L, (uint32_t)(h_lo - h_base), lane, wres);
  if (g.mode & kTxFieldsOnly) return;
  if constexpr ((XF & 1) != 0) return;
  __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
  __builtin_amdgcn_wave_barrier();
  // 4. the header region back, whole
  tx_writeback<SP>(L, h_lo, h_hi, h_base, h_chunks, lane);
}

template <int U, int AUX, int SP, int RED, int XF = 0, int PH = 0>
__global__ __launch_bounds__(256) void tcp_tx(TxGeo g) {
  extern __shared__ uint4 tx_lds[];
  const uint32_t lane = threadIdx.x & 63u;
  const uint32_t wv = (uint32_t)__builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  uint8_t* L = reinterpret_cast<uint8_t*>(tx_lds) + (size_t)wv * g.lds_wave;
  uint32_t* rows = reinterpret_cast<uint32_t*>(L + g.lds_rows);  // RED 1: [tile][64] partials
  tx_tile<U, AUX, SP, RED, XF, PH>(g, ((uint64_t)blockIdx.x * g.wpg + wv) * g.tile, L, rows, lane);
}

// The header pass as a persistent grid: wave W takes tiles W, W + NW, ...
// with two tiles' slot regions in flight in registers (plain buffer loads,
// CPL 16-B chunks per lane, plus the tile's payload values, one segment per
// lane) while it finishes a third from LDS: the one-shot header pass (tcp_tx
// PH = 2) does one memory round per wave, its DMA, the wait, then the stores
// (22-28 us where the writes alone take ~12).
// Every memory operation of an iteration is a buffer operation issued
// unconditionally (out-of-range offsets where there is nothing to do; a
// resource of 0 bytes where a fetch runs past the last tile), so the
// compiler knows how many are younger than the registers it waits for: the
// wait for tile t's region leaves tile t+1's fetch and tile t-1's stores in
// flight.  A flat store, or a store count it cannot know, would make it wait
// for all of them.  For tiles that start 16-B aligned (hdr, tile * slot) and
// hold at most 64 segments and 64 CPL chunks; the last tile's unaligned end
// is written with byte stores as the wave's last act.
// DEP = tiles in flight per wave (2; 3 as a timing variant); 1: one tile
// per wave on a one-shot grid (register-staged, no persistence).
template <int CPL, int SP, int DEP = 2>
__global__ __launch_bounds__(256) void tcp_tx_hdr(TxGeo g, uint32_t ntiles) {
  extern __shared__ uint4 tx_lds[];
  const uint32_t lane = threadIdx.x & 63u;
  const uint32_t wv = (uint32_t)__builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  uint8_t* L = reinterpret_cast<uint8_t*>(tx_lds) + (size_t)wv * g.lds_wave;
  uint4* L4 = reinterpret_cast<uint4*>(L);
  const uint32_t NW = gridDim.x * g.wpg;
  const uint32_t t0 = blockIdx.x * g.wpg + wv;
  if (t0 >= ntiles) return;  // a whole wave leaves together
  const uint32_t region = g.tile * g.slot;  // bytes of a full tile (a multiple of 16)
  const uint64_t end = g.hdr + g.n * (uint64_t)g.slot;
  // the payload values and the sums, through resources of their own
  const __amdgpu_buffer_rsrc_t xr = tx_srd((uint64_t)(uintptr_t)g.xs, (uint32_t)(g.n * g.xstride * 2u));
  const __amdgpu_buffer_rsrc_t orr = tx_srd((uint64_t)(uintptr_t)g.out, g.out ? (uint32_t)(g.n * 4u) : 0u);
  auto fetch = [&](uint32_t tt, uint4* v, uint32_t& pv) {
    const bool live = tt < ntiles;
    const uint64_t lo = g.hdr + (uint64_t)(live ? tt : 0u) * region;
    const uint32_t bytes = live ? (uint32_t)(end - lo < region ? ((end - lo + 15) & ~15ull) : region) : 0u;
    const __amdgpu_buffer_rsrc_t hr = tx_srd(lo, bytes);
#pragma unroll
    for (int i = 0; i < CPL; ++i) v[i] = tx_load<0>(hr, (lane + 64u * i) * 16u);
    const uint64_t si = (uint64_t)tt * g.tile + lane;
    pv = __builtin_amdgcn_raw_buffer_load_b16(xr, (int)(live && si < g.n ? si * g.xstride * 2u : 0xFFFFFFF0u), 0, 0);
  };
  auto finish = [&](uint32_t t, const uint4* v, uint32_t pv) {
    const uint64_t s0 = (uint64_t)t * g.tile;
    const uint32_t nseg = g.n - s0 < g.tile ? (uint32_t)(g.n - s0) : g.tile;
    const uint64_t lo = g.hdr + s0 * g.slot, hi = lo + (uint64_t)nseg * g.slot;
    const uint32_t chunks = (uint32_t)((hi - lo + 15) >> 4);
#pragma unroll
    for (int i = 0; i < CPL; ++i)
      if (lane + 64u * i < chunks) L4[lane + 64u * i] = v[i];
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
    __builtin_amdgcn_wave_barrier();
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
    // the fields (tx_fields' arithmetic for the lane's one segment)
    uint32_t ipv = 0, tcpv = 0;
    if (lane < nseg) {
      const uint32_t o = lane * g.slot;
      const uint64_t si = s0 + lane;
      const uint32_t size = si + 1 < g.n ? g.mss : (uint32_t)(g.size - (g.n - 1) * (uint64_t)g.mss);
      if (g.mode & kTxIp) {
        const uint32_t a = o + g.ip_at;
        ipv = tx_fold(tx_class(lds_wsum_loop(L, a, g.ip_len, a + 10u), a & 1u));  // Checksum(ip[:IHL], 0)
        lds_put_be16(L, a + 10u, ~ipv & 0xFFFFu);
      }
      uint32_t x = tx_fold(g.addr_sum + ((g.tcp_len + size) & 0xFFFFu));  // PseudoHeaderChecksum
      x = tx_fold(x + g.proto);
      const uint32_t a = o + g.tcp_at;
      x = tx_fold(x + (pv & 0xFFFFu));                                               // ChecksumVVWithOffset
      x = tx_fold(x + tx_class(lds_wsum_loop(L, a, g.tcp_len, a + 16u), a & 1u));    // CalculateChecksum
      lds_put_be16(L, a + 16u, ~x & 0xFFFFu);
      tcpv = x;
    }
    __builtin_amdgcn_raw_buffer_store_b32(ipv | (tcpv << 16), orr, (int)(lane < nseg ? (s0 + lane) * 4u : 0xFFFFFFF0u), 0,
                                          0);
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
    __builtin_amdgcn_wave_barrier();
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
    // the region back, whole chunks (the tile's own: it starts 16-B aligned)
    const uint32_t full = (uint32_t)((hi - lo) >> 4);
    const __amdgpu_buffer_rsrc_t hr = tx_srd(lo, full * 16u);
#pragma unroll
    for (int i = 0; i < CPL; ++i) {
      const uint32_t c = lane + 64u * i;
      const uint4 x = L4[c < chunks ? c : 0u];
      __builtin_amdgcn_raw_buffer_store_b128(*reinterpret_cast<const __attribute__((ext_vector_type(4))) uint32_t*>(&x),
                                             hr, (int)(c * 16u), 0, tx_store_aux(SP));
    }
    return full < chunks;  // an unaligned end: the last tile
  };
  auto tail = [&](uint32_t t) {  // the last tile's partial chunk, byte by byte
    const uint64_t s0 = (uint64_t)t * g.tile;
    const uint32_t nseg = (uint32_t)(g.n - s0);
    const uint64_t lo = g.hdr + s0 * g.slot, hi = lo + (uint64_t)nseg * g.slot;
    const uint32_t full = (uint32_t)((hi - lo) >> 4);
    if (lane < (uint32_t)((hi - lo) & 15u)) reinterpret_cast<uint8_t*>((uintptr_t)(lo + full * 16u))[lane] = L[full * 16u + lane];
  };
  uint4 x[CPL], y[CPL];
  uint32_t px = 0, py = 0;
  fetch(t0, x, px);
  if constexpr (DEP == 1) {  // one tile per wave (a one-shot grid, NW = ntiles)
    if (finish(t0, x, px)) tail(t0);
    return;
  }
  fetch(t0 + NW, y, py);
  if constexpr (DEP == 3) {
    uint4 z[CPL];
    uint32_t pz = 0;
    fetch(t0 + 2 * NW, z, pz);
    for (uint32_t t = t0;; t += 3 * NW) {
      if (finish(t, x, px)) {
        tail(t);
        break;
      }
      fetch(t + 3 * NW, x, px);
      if (t + NW >= ntiles) break;
      if (finish(t + NW, y, py)) {
        tail(t + NW);
        break;
      }
      fetch(t + 4 * NW, y, py);
      if (t + 2 * NW >= ntiles) break;
      if (finish(t + 2 * NW, z, pz)) {
        tail(t + 2 * NW);
        break;
      }
      fetch(t + 5 * NW, z, pz);
      if (t + 3 * NW >= ntiles) break;
    }
    return;
  }
  for (uint32_t t = t0;; t += 2 * NW) {
    // tile t from x, then tile t + 2 NW's fetch into x (x is in LDS by then)
    bool ragged = finish(t, x, px);
    if (ragged) {
      tail(t);
      break;
    }
    fetch(t + 2 * NW, x, px);
    if (t + NW >= ntiles) break;
    ragged = finish(t + NW, y, py);
    if (ragged) {
      tail(t + NW);
      break;
    }
    fetch(t + 3 * NW, y, py);
    if (t + 2 * NW >= ntiles) break;
  }
}

// Many batches (sendTCPBatch calls) in one launch, one fused pass each:
// wave T takes tile T of the concatenation; first[c] is call c's first tile
// (first[ncalls] the total), calls[c] its geometry.  g holds the launch-wide
// LDS shape (the largest call's) and waves per workgroup.
__global__ __launch_bounds__(256) __attribute__((amdgpu_waves_per_eu(6))) void tcp_tx_multi(TxGeo g, const TxGeo* __restrict__ calls,
                                                    const uint32_t* __restrict__ first, uint32_t ncalls) {
  extern __shared__ uint4 tx_lds[];
  const uint32_t lane = threadIdx.x & 63u;
  const uint32_t wv = (uint32_t)__builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  uint8_t* L = reinterpret_cast<uint8_t*>(tx_lds) + (size_t)wv * g.lds_wave;
  uint32_t* rows = reinterpret_cast<uint32_t*>(L + g.lds_rows);
  const uint32_t T = blockIdx.x * g.wpg + wv;
  if (T >= first[ncalls]) return;
  uint32_t lo = 0, hi = ncalls;  // first[lo] <= T < first[hi]
  while (hi - lo > 1) {
    const uint32_t mid = (lo + hi) >> 1;
    if (first[mid] <= T) lo = mid;
    else hi = mid;
  }
  lo = (uint32_t)__builtin_amdgcn_readfirstlane(lo);
  const TxGeo c = calls[lo];
  tx_tile<16, 2, 0, 1, 0, 0>(c, (uint64_t)(T - first[lo]) * c.tile, L, rows, lane);
}

// Segments per wave for a pass.  A pass that reads payload: about 12 KiB of
// it per wave, at most 32 segments (1M x 1460 B, payload pass: 218 us at 8
// segments, 222-228 at 4 / 16 / 32; tools/tx_struct_probe.py).  A header
// pass: 64 segments (28 us at 64, 36 at 32, 58 at 8).  Fewer when the batch
// would not give ~2,048 waves, and at most ~8 KiB of header slots.
static uint32_t tx_tile(const TxGeo& g, bool pay) {
  uint32_t t = pay ? (uint32_t)std::min<uint64_t>(32, std::max<uint64_t>(1, (12u << 10) / std::max<uint32_t>(g.mss, 1)))
                   : 64u;
  const uint64_t per = (g.n + 2047) / 2048;
  if (per < t) t = (uint32_t)std::max<uint64_t>(1, per);
  while (t > 1 && (uint64_t)t * g.slot > (8u << 10)) t /= 2;
  return t;
}

// Tile, LDS and workgroup shape of a pass (g.tile = 0: tx_tile's choice).
static hipError_t tx_shape(TxGeo& g, int ph, uint32_t* grid) {
  const bool pay = ph != 2 && (g.mode & kTxTcpFull), hdr = ph != 1;
  if (g.tile == 0) g.tile = tx_tile(g, pay);
  // (a lane holds a payload-reading pass's segment; a header pass loops)
  if (g.tile > (pay ? 64u : 256u) || (uint64_t)g.tile * g.slot > (12u << 10)) return hipErrorInvalidValue;
  // The LDS-DMA copy writes whole 64-chunk (1 KiB) rows, zeros past the
  // region included: each wave's share is rounded up to whole rows; then the
  // segments' rows of lane partials (passes that read payload).
  g.lds_rows = hdr ? (uint32_t)(((uint64_t)g.tile * g.slot + 30) / 16 + 63) / 64 * 1024 : 0u;
  g.lds_wave = g.lds_rows + (pay ? g.tile * 256u : 0u);
  // 4 waves (tiles) per workgroup, fewer where their LDS would pass 64 KiB
  g.wpg = g.lds_wave <= (16u << 10) ? 4u : g.lds_wave <= (32u << 10) ? 2u : 1u;
  const uint64_t tiles = (g.n + g.tile - 1) / g.tile;
  *grid = (uint32_t)((tiles + g.wpg - 1) / g.wpg);
  return hipSuccess;
}

template <int U, int AUX, int SP, int RED, int XF = 0, int PH = 0>
static hipError_t launch_tcp_tx_t(TxGeo g, hipStream_t stream) {
  if (g.n == 0) return hipSuccess;
  uint32_t grid = 0;
  const hipError_t e = tx_shape(g, PH, &grid);
  if (e != hipSuccess) return e;
  hipLaunchKernelGGL((tcp_tx<U, AUX, SP, RED, XF, PH>), dim3(grid), dim3(64 * g.wpg), (size_t)g.lds_wave * g.wpg,
                     stream, g);
  return hipGetLastError();
}

// The payload pass in the receive ring's shape (rx_ring.hip; round 5): a wave
// takes 8 consecutive segments, one 8-lane group per segment, and the group's
// load instruction k reads its segment's k-th 128-B line whole (lane i: 16 B
// at line + 16 i), line 0 with the default policy (its first bytes belong to
// the segment before), the others nontemporal.  The segment's byte range
// alone decides which chunks exist, so all NB loads are issued at once; a
// chunk past the segment reads the buffer resource's out-of-range zeros.
// Every loaded chunk is summed whole (4 v_sad_u16) except two: the chunk
// holding the segment's first byte is masked below it, and the chunk holding
// its last byte is re-read (an L2 hit, issued with the others) by the lane
// that loaded it, which takes the bytes past the end back out.  One 3-step
// DPP reduction gives the group its W; lane 0 writes the payload value.  No
// LDS, no cross-group step, no per-window segment bookkeeping.
__device__ __forceinline__ uint32_t tx_bytes_from(const uint4 v, int c) {  // W of bytes [c, 16)
  return wsum4(make_uint4(v.x & ~below(c), v.y & ~below(c - 4), v.z & ~below(c - 8), v.w & ~below(c - 12)), 0u);
}

// G lanes per segment: 8 (a 128-B line per group instruction) or 4 (64-B
// units, 16 segments per wave: short segments, where the per-segment work and
// not memory is the cost).
template <int NB, int A0 = 0, int G = 8>
__global__ __launch_bounds__(256) void tcp_tx_pay(TxGeo g) {
  static_assert(G == 8 || G == 4, "8- or 4-lane groups");
  constexpr uint32_t U = 16u * G, US = G == 8 ? 7u : 6u, PW = 64u / G;
  const uint32_t lane = threadIdx.x & 63u, grp = lane / G, li = lane & (G - 1u);
  const uint32_t wv = (uint32_t)__builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  const uint64_t s0 = ((uint64_t)blockIdx.x * 4u + wv) * PW;  // the wave's first segment
  if (s0 >= g.n) return;  // a whole wave leaves together
  const uint64_t s = s0 + grp;
  const uint64_t tail0 = (g.n - 1) * (uint64_t)g.mss;  // where the last segment starts
  const uint32_t sz = s < g.n ? (s + 1 < g.n ? g.mss : (uint32_t)(g.size - tail0)) : 0u;
  // wave-relative 32-bit coordinates: one resource over the wave's bytes
  // (< 8 * 65,535 + 144), rounded up to whole 16-B chunks: a load whose 16 B
  // reach past the resource's end reads zeros, so the chunk holding the last
  // byte must lie inside it (its bytes past the end are in the same aligned
  // chunk, never another page)
  const uint64_t wbase = (g.pay + s0 * g.mss) & ~127ull;
  const uint64_t s_end = s0 + PW < g.n ? s0 + PW : g.n;
  const uint64_t w_end = g.pay + (s_end < g.n ? s_end * (uint64_t)g.mss : g.size);
  const uint32_t nrec = (uint32_t)((w_end - wbase + 15u) & ~15ull);
  const __amdgpu_buffer_rsrc_t r = tx_srd(wbase, nrec);
  const uint32_t pa = sz ? (uint32_t)(g.pay + s * g.mss - wbase) : 0u;  // the segment's first byte
  const uint32_t pe = pa + sz;
  const uint32_t cl = (pa & ~(U - 1u)) + 16u * li;  // lane li's chunk of line (unit) 0
  // lines k >= 1 start past pa: the lane's chunk there holds segment bytes
  // iff it starts before pe (k <= klast)
  const uint32_t klast = sz && pe > cl ? (pe - 1u - cl) >> US : 0u;
  const uint32_t cl1 = sz && pe > cl + U ? cl : nrec;
  const bool in0 = sz && cl + 16u > pa && cl < pe;
  // the chunk holding the last byte, re-read by the lane that loads it
  const uint32_t tc = (pe - 1u) & ~15u;
  const bool owner = sz && ((tc >> 4) & (G - 1u)) == li;
  uint4 v[NB];
  v[0] = tx_load<A0>(r, in0 ? cl : nrec);
  const uint4 t = tx_load<0>(r, owner ? tc : nrec);
#pragma unroll
  for (int k = 1; k < NB; ++k) v[k] = tx_load<2>(r, ((uint32_t)k <= klast ? cl1 : nrec) + U * k);
  uint32_t w = tx_bytes_from(v[0], pa > cl ? (int)(pa - cl) : 0);
#pragma unroll
  for (int k = 1; k < NB; ++k) w = wsum4(v[k], w);
  // segments longer than NB lines: the rest in batches of 4 lines
  for (uint32_t k0 = NB; __builtin_amdgcn_ballot_w64(k0 <= klast) != 0; k0 += 4) {
#pragma unroll
    for (int k = 0; k < 4; ++k) w = wsum4(tx_load<2>(r, ((k0 + k) <= klast ? cl1 : nrec) + U * (k0 + k)), w);
  }
  // the bytes [pe, tc + 16) were summed whole with the last chunk (none when
  // pe ends a chunk); the first chunk's bytes below pa were masked, so if it
  // is also the last, what is taken out lies above pa
  if (owner) w -= tx_bytes_from(t, (int)(pe - tc));
  w += (uint32_t)__builtin_amdgcn_update_dpp(0, (int)w, 0xB1, 0xF, 0xF, false);   // quad_perm 1,0,3,2
  w += (uint32_t)__builtin_amdgcn_update_dpp(0, (int)w, 0x4E, 0xF, 0xF, false);   // quad_perm 2,3,0,1
  if constexpr (G == 8) w += (uint32_t)__builtin_amdgcn_update_dpp(0, (int)w, 0x141, 0xF, 0xF, false);  // row_half_mirror
  if (li == 0 && s < g.n) g.xs[s * g.xstride] = (uint16_t)tx_class(w, (uint32_t)((g.pay + s * g.mss) & 1u));
}

// Lines per load batch for a segment of `mss` bytes from any offset.
static int tx_pay_lines(uint32_t mss) {
  const uint64_t lines = ((uint64_t)mss + 127 + 127) / 128;
  return lines <= 2 ? 2 : lines <= 4 ? 4 : lines <= 8 ? 8 : lines <= 13 ? 13 : 16;
}

template <int NB, int A0, int G = 8>
static hipError_t launch_tx_pay_t(const TxGeo& g, hipStream_t stream) {
  const uint64_t per = 4u * (64u / G);  // 4 waves x 8 (16) segments
  const uint64_t wgs = (g.n + per - 1) / per;
  hipLaunchKernelGGL((tcp_tx_pay<NB, A0, G>), dim3((uint32_t)wgs), dim3(256), 0, stream, g);
  return hipGetLastError();
}

// The payload pass: the group shape above (GP = 1; GP = 2: line 0
// nontemporal too, A/B only), or tcp_tx PH = 1 (GP = 0, the round-4 shape,
// kept for A/B).
template <int U, int AUX, int SP, int RED, int GP = 1>
static hipError_t launch_payload_pass(const TxGeo& g, hipStream_t stream) {
  if (g.n == 0) return hipSuccess;
  // a tile forced through ns_csum_set_tx_tuning selects the windowed pass
  // (the group pass's shape is fixed: 8 segments per wave)
  if (!GP || g.tile || (g.n + 31) / 32 >= (1ull << 31)) return launch_tcp_tx_t<U, AUX, SP, RED, 0, 1>(g, stream);
  constexpr int A0 = GP == 2 ? 2 : 0;
  switch (tx_pay_lines(g.mss)) {
    case 2: return launch_tx_pay_t<2, A0>(g, stream);
    case 4: return launch_tx_pay_t<4, A0>(g, stream);
    case 8: return launch_tx_pay_t<8, A0>(g, stream);
    case 13: return launch_tx_pay_t<13, A0>(g, stream);
    default: return launch_tx_pay_t<16, A0>(g, stream);
  }
}

// Compute units of the current device (cached per device ordinal).
static uint32_t tx_cu_count() {
  static uint32_t cus[64] = {};
  int dev = 0;
  if (hipGetDevice(&dev) != hipSuccess || dev < 0 || dev >= 64) return 256;
  if (!cus[dev]) {
    int c = 0;
    if (hipDeviceGetAttribute(&c, hipDeviceAttributeMultiprocessorCount, dev) != hipSuccess || c <= 0) c = 256;
    cus[dev] = (uint32_t)c;
  }
  return cus[dev];
}

// The header pass on a persistent grid (tcp_tx_hdr), `per_cu` waves per CU
// (0: 24; tools/tx_struct_probe.py, 1M x 1460-B segments, both passes: 244.1
// us at 24, 245.2 at 32, 245.6 at 16, 250.7 at 8, 254.6 at 4, against 248.3
// for the one-shot header pass; profiles/r05/tx_hdr/), or the one-shot
// kernel where tcp_tx_hdr's conditions do not hold.
template <int SP, int DEP = 2>
static hipError_t launch_header_pass(TxGeo h, hipStream_t stream, uint32_t per_cu) {
  if (h.n == 0) return hipSuccess;
  uint32_t grid = 0;
  hipError_t e = tx_shape(h, 2, &grid);
  if (e != hipSuccess) return e;
  // tcp_tx_hdr's conditions: full TCP mode with whole write-back, tiles of
  // <= 64 segments starting 16-B aligned, <= 8 KiB of slots each (CPL = 4,
  // 5, 6 or 8 chunks per lane: IPv4's 54-B slots take 4, an IPv6 route's
  // 74-B slots 5; 6 and 8 on the one-shot grid only), d_out 4-B aligned
  const uint64_t region = (uint64_t)h.tile * h.slot;
  if (h.tile > 64 || region > 8192 || region % 16 || (h.hdr & 15) || !(h.mode & kTxTcpFull) ||
      (h.mode & kTxFieldsOnly) || ((uintptr_t)h.out & 3) || h.xs == nullptr)
    return launch_tcp_tx_t<16, 2, SP, 1, 0, 2>(h, stream);
  const uint64_t tiles = (h.n + h.tile - 1) / h.tile;
  if (DEP == 1 && per_cu >= 1 && per_cu <= 4) h.wpg = per_cu;  // one-shot: per_cu = waves per workgroup (A/B)
  const uint64_t waves = DEP == 1 ? tiles : std::min<uint64_t>(tiles, (uint64_t)tx_cu_count() * (per_cu ? per_cu : 24u));
  const uint32_t wgs = (uint32_t)((waves + h.wpg - 1) / h.wpg);
  const size_t lds = (size_t)h.lds_wave * h.wpg;
  const uint32_t cpl = (uint32_t)((region + 1023) / 1024);
  if (cpl <= 4) {
    hipLaunchKernelGGL((tcp_tx_hdr<4, SP, DEP>), dim3(wgs), dim3(64 * h.wpg), lds, stream, h, (uint32_t)tiles);
  } else if (cpl == 5) {
    hipLaunchKernelGGL((tcp_tx_hdr<5, SP, DEP>), dim3(wgs), dim3(64 * h.wpg), lds, stream, h, (uint32_t)tiles);
  } else if constexpr (DEP == 1) {  // (2-3 tiles in flight at 6-8 chunks per lane: 5 waves per SIMD or fewer)
    if (cpl == 6) hipLaunchKernelGGL((tcp_tx_hdr<6, SP, 1>), dim3(wgs), dim3(64 * h.wpg), lds, stream, h, (uint32_t)tiles);
    else hipLaunchKernelGGL((tcp_tx_hdr<8, SP, 1>), dim3(wgs), dim3(64 * h.wpg), lds, stream, h, (uint32_t)tiles);
  } else {
    return launch_tcp_tx_t<16, 2, SP, 1, 0, 2>(h, stream);
  }
  return hipGetLastError();
}

// The production shape: a batch that needs its payload read takes two passes
// when it has scratch for the payload values (g.xs): the payload pass streams
// only payload, the header pass then reads, fills and writes back the slots
// (interleaving the slot write-back with the payload stream
// cost ~45 us on 1M segments).  One fused pass otherwise.  HP: the header
// pass one tile per wave on a one-shot grid, register-staged (2, production:
// tcp_tx_hdr DEP = 1), persistent (1: DEP = 2) or round 4's LDS-DMA one-shot
// (0: tcp_tx PH = 2).  In situ after the payload pass over fresh slots
// (profiles/r06/tx_drain/header_oneshot.jsonl): 25.7-26.1 us at 4 waves per
// workgroup against 27.9-28.3 persistent and 22.2 for a plain copy of the
// slots with the same stores.
// GP: the payload pass windowed (0) or in 8-lane groups (1, production).
// SP: the header pass's store policy (tx_store_aux; production 4, nt sc1).
// With default-policy stores the header pass's 57 MB of slots leave L2
// within its own dispatch (WRITE_SIZE, profiles/r06/tx_drain/) but stay
// dirty in the die-level Infinity Cache, which writes them to HBM only when
// the next call's payload stream evicts them: that pass then takes 244 us
// instead of 208 over fresh slots (idle time between calls does not help; a
// 1 GiB read in between takes the cost instead).  nt sc1 stores write them
// through: the payload pass stays at 211 us and both passes take 237 against
// 251 for round 5's windowed pass with default stores (which absorbed the
// eviction 6% below the read ceiling).  tools/tx_drain_probe.py.
template <int U, int AUX, int SP, int RED, int HP = 1, int GP = 0>
static hipError_t launch_passes(TxGeo g, hipStream_t stream, uint32_t per_cu = 0) {
  if (!(g.mode & kTxTcpFull) || g.xs == nullptr) return launch_tcp_tx_t<U, AUX, SP, RED>(g, stream);
  TxGeo h = g;
  h.tile = g.htile;
  hipError_t e = launch_payload_pass<U, AUX, SP, RED, GP>(g, stream);
  if (e == hipSuccess)
    e = HP == 2 ? launch_header_pass<SP, 1>(h, stream, 0)
        : HP    ? launch_header_pass<SP>(h, stream, per_cu)
                : launch_tcp_tx_t<U, AUX, SP, RED, 0, 2>(h, stream);
  return e;
}

// ns_csum_tcp_tx_multi's plan: each call's tile (tx_tile's rule without the
// per-call wave floor: the launch has every call's waves), first[c] = call
// c's first tile, first[ncalls] the total; the launch-wide LDS shape and
// waves per workgroup in *launch.  Returns the grid (0: too many tiles).
uint32_t tx_multi_prepare(TxGeo* calls, uint32_t ncalls, TxGeo* launch, uint32_t* first) {
  uint64_t tiles = 0, max_hdr = 0;
  uint32_t max_tile = 1;
  for (uint32_t c = 0; c < ncalls; ++c) {
    TxGeo& g = calls[c];
    uint32_t t = (uint32_t)std::min<uint64_t>(32, std::max<uint64_t>(1, (12u << 10) / std::max<uint32_t>(g.mss, 1)));
    while (t > 1 && (uint64_t)t * g.slot > (8u << 10)) t /= 2;
    g.tile = t;
    g.xs = nullptr;
    first[c] = (uint32_t)tiles;
    tiles += (g.n + t - 1) / t;
    if (tiles >= (1ull << 31)) return 0;
    max_tile = std::max(max_tile, t);
    max_hdr = std::max<uint64_t>(max_hdr, (uint64_t)t * g.slot);
  }
  first[ncalls] = (uint32_t)tiles;
  *launch = TxGeo{};
  launch->lds_rows = (uint32_t)((max_hdr + 30) / 16 + 63) / 64 * 1024;
  launch->lds_wave = launch->lds_rows + max_tile * 256u;
  launch->wpg = launch->lds_wave <= (16u << 10) ? 4u : launch->lds_wave <= (32u << 10) ? 2u : 1u;
  return (uint32_t)((tiles + launch->wpg - 1) / launch->wpg);
}

hipError_t launch_tcp_tx_multi(const TxGeo& launch, uint32_t grid, const TxGeo* d_calls, const uint32_t* d_first,
                               uint32_t ncalls, hipStream_t stream) {
  if (grid == 0) return hipSuccess;
  hipLaunchKernelGGL(tcp_tx_multi, dim3(grid), dim3(64 * launch.wpg), (size_t)launch.lds_wave * launch.wpg, stream,
                     launch, d_calls, d_first, ncalls);
  return hipGetLastError();
}

hipError_t launch_tcp_tx(TxGeo g, hipStream_t stream, uint32_t variant) {
  switch (variant) {
    case 1: g.xs = nullptr; return launch_tcp_tx_t<16, 2, 0, 1>(g, stream);  // one fused pass
    case 2: return launch_passes<16, 2, 1, 1>(g, stream);
    case 3: return launch_passes<16, 2, 0, 0>(g, stream);
    case 4: return launch_passes<16, 2, 0, 1, 0>(g, stream);  // the one-shot header pass (round 4)
    case 5: return launch_passes<16, 2, 0, 1, 1, 1>(g, stream);  // group payload pass, default-policy stores
    case 6: return launch_passes<16, 2, 0, 1, 1, 0>(g, stream);  // round 5's: windowed, default-policy stores
    case 7: return launch_passes<16, 2, 4, 1, 1, 1>(g, stream);  // the header pass persistent (2 tiles per wave in flight)
    default: return launch_passes<16, 2, 4, 1, 2, 1>(g, stream);  // group payload pass, one-shot header pass, nt sc1 stores
  }
}

}  // namespace nsk
