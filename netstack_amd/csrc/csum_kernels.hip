// csum_kernels.hip — gfx950 (MI355X / CDNA4) kernels for netstack's RFC 1071
// checksum hot path (tcpip/header/checksum.go:26-46 applied per packet).
//
// Arithmetic.  calculateChecksum (checksum.go:26-46) adds big-endian 16-bit
// words into a uint32 that wraps mod 2^32 and folds once at the end
// (ChecksumCombine, :104-107).  Every byte therefore contributes
// byte*256 (high byte of a word) or byte*1 (low byte), decided by the parity
// of its position in the piece, shifted by one when `odd` is set (:29-32).
// In absolute device addresses: with phase = (addr(first byte) + odd) & 1,
// the byte at address A is a high byte iff (A & 1) == phase.  Summing
//     S = 256*E + O  (phase 0)   or   E + 256*O  (phase 1)
// with E/O = sums of the bytes at even/odd addresses, all mod 2^32, gives the
// Go accumulator exactly (uint32 addition is associative and commutative, so
// any reduction order is bit-exact, including the > 128 KiB wrap quirk).
//
// Layout.  Packets are byte ranges of one arena in HBM, described by a table of
// 16-byte ns_pkt_desc {u64 off, u32 len, u16 initial, u16 flags}.  The kernel
// reads only whole, naturally aligned 16-byte chunks (global_load_dwordx4):
// a packet covers chunks [addr>>4, (addr+len-1)>>4] and its first/last chunk
// is byte-masked.  An aligned 16-byte chunk never crosses a page, and each
// chunk read holds at least one byte of the packet, so no read can fault.
//
// Work decomposition.  A 256-thread workgroup owns a tile of P = 256*D
// descriptors (D = 1 for MTU-sized packets, 4 for small ones).  The prologue
// reads the tile's descriptors once, scans them in LDS and picks one of two
// block-uniform paths:
//
//  * dense path — the tile's packets are sorted and non-overlapping in the
//    arena with little padding (a packed batch, what tcpip/buffer staging and
//    the benchmarks produce).  The tile's byte span is streamed directly:
//    every lane owns runs of UD consecutive 16-byte chunks (a wave-instruction's
//    lanes 64 B apart, which streams at the coalesced rate on gfx950), loads are
//    nontemporal and software-pipelined one step ahead because their addresses
//    do not depend on any lookup; packet attribution (a binary search of the
//    packets' end offsets in LDS, then a forward walk with byte masks) runs
//    while the next step's loads are in flight.
//  * general path — any table (unsorted, overlapping, sparse, giant
//    descriptors): the tile's chunk counts are scanned into a virtual chunk
//    space; each lane takes UG consecutive virtual chunks, finds their packet
//    by binary search and loads them.
//
// Both paths split each chunk into even/odd byte lanes of packed 2x16-bit
// accumulators, flush a packet's 32-bit partial into an LDS accumulator
// (ds_add_u32) when the lane moves past it, and the epilogue folds
// initial + partial and writes one u16 per packet (coalesced).  No MFMA: this
// is a byte sum, HBM-bound.
#include <hip/hip_runtime.h>
#include <stdint.h>

#include "csum_kernels.h"

#include <algorithm>
#include <map>
#include <mutex>

namespace nsk {

// ChecksumCombine(uint16(v), uint16(v>>16)) — checksum.go:45, :104-107.
__device__ __forceinline__ uint32_t fold1(uint32_t v) {
  const uint32_t s = (v & 0xFFFFu) + (v >> 16);
  return (s + (s >> 16)) & 0xFFFFu;
}

// Byte mask of dword j (bytes 4j..4j+3) of a 16-byte chunk restricted to
// bytes [lo, hi).
__device__ __forceinline__ uint32_t dword_mask(int lo, int hi, int j) {
  const int a = max(lo - 4 * j, 0);
  const int b = min(hi - 4 * j, 4);
  if (b <= a) return 0u;
  const uint32_t below_b = (b >= 4) ? 0xFFFFFFFFu : ((1u << (8 * b)) - 1u);
  return below_b & (0xFFFFFFFFu << (8 * a));
}

// Packed even/odd byte accumulation of one 16-byte chunk:
//   e: bytes at even addresses (dword bytes 0 and 2) in two 16-bit lanes
//   o: bytes at odd addresses  (dword bytes 1 and 3) in two 16-bit lanes
__device__ __forceinline__ void acc_chunk(const uint4 w, uint32_t& e, uint32_t& o) {
  e += (w.x & 0x00FF00FFu) + (w.y & 0x00FF00FFu);
  e += (w.z & 0x00FF00FFu) + (w.w & 0x00FF00FFu);
  o += ((w.x >> 8) & 0x00FF00FFu) + ((w.y >> 8) & 0x00FF00FFu);
  o += ((w.z >> 8) & 0x00FF00FFu) + ((w.w >> 8) & 0x00FF00FFu);
}

// Packet partial S (mod 2^32) from packed accumulators and the phase.
__device__ __forceinline__ uint32_t partial_of(uint32_t e, uint32_t o, uint32_t phase) {
  const uint32_t E = (e & 0xFFFFu) + (e >> 16);
  const uint32_t O = (o & 0xFFFFu) + (o >> 16);
  return phase ? (E + (O << 8)) : ((E << 8) + O);
}

// meta word (general path): bits 0-3 = first byte within first chunk,
// 4-7 = last byte within last chunk, bit 8 = phase.  Dense path: bit 8 only.
constexpr uint32_t kPhaseBit = 1u << 8;

template <bool NT>
__device__ __forceinline__ uint4 load16(const uint4* p) {
  if constexpr (NT) {
    uint4 v;
    v.x = __builtin_nontemporal_load(&p->x);
    v.y = __builtin_nontemporal_load(&p->y);
    v.z = __builtin_nontemporal_load(&p->z);
    v.w = __builtin_nontemporal_load(&p->w);
    return v;
  } else {
    return *p;
  }
}

__device__ __forceinline__ uint4 mask_chunk(uint4 w, int lo, int hi) {
  w.x &= dword_mask(lo, hi, 0);
  w.y &= dword_mask(lo, hi, 1);
  w.z &= dword_mask(lo, hi, 2);
  w.w &= dword_mask(lo, hi, 3);
  return w;
}

__device__ __forceinline__ void flush(uint32_t* s_acc, const uint32_t* s_meta, int pk,
                                      uint32_t e, uint32_t o) {
  if (e | o) atomicAdd(&s_acc[pk], partial_of(e, o, s_meta[pk] & kPhaseBit));
}

// ---- general path: virtual chunk space ------------------------------------
template <int P, int U, bool NT>
__device__ __forceinline__ void general_step(const uint4* __restrict__ chunks,
                                             const uint64_t* __restrict__ s_cstart,
                                             const uint64_t* __restrict__ s_cbase,
                                             const uint32_t* __restrict__ s_meta,
                                             uint32_t* __restrict__ s_acc, uint64_t C,
                                             uint64_t c0, int& pk_floor) {
  constexpr int LOGP = __builtin_ctz(P);
  // Largest pk with s_cstart[pk] <= c0 (that packet is non-empty); the lane's
  // packet only moves forward, so search [pk_floor, P).
  int lo = pk_floor, hi = P;
#pragma unroll
  for (int s = 0; s < LOGP; ++s) {
    const int mid = (lo + hi) >> 1;
    if (hi - lo > 1) {
      if (s_cstart[mid] <= c0) lo = mid; else hi = mid;
    }
  }
  int pk = lo;
  pk_floor = lo;
  uint64_t pstart = s_cstart[pk], pend = s_cstart[pk + 1], pbase = s_cbase[pk];
  uint4 v[U];
  int pid[U];
  uint32_t firstm = 0, lastm = 0;
#pragma unroll
  for (int u = 0; u < U; ++u) {
    const uint64_t c = c0 + u;
    pid[u] = -1;
    v[u] = make_uint4(0, 0, 0, 0);
    if (c < C) {
      while (c >= pend) {
        ++pk;
        pstart = pend;
        pend = s_cstart[pk + 1];
        pbase = s_cbase[pk];
      }
      pid[u] = pk;
      if (c == pstart) firstm |= 1u << u;
      if (c + 1 == pend) lastm |= 1u << u;
      v[u] = load16<NT>(chunks + (pbase + c));
    }
  }
  int cur = pid[0];
  uint32_t e = 0, o = 0;
#pragma unroll
  for (int u = 0; u < U; ++u) {
    if (pid[u] < 0) break;
    if (pid[u] != cur) {
      flush(s_acc, s_meta, cur, e, o);
      e = 0;
      o = 0;
      cur = pid[u];
    }
    uint4 w = v[u];
    if ((firstm | lastm) & (1u << u)) {
      const uint32_t m = s_meta[cur];
      const int blo = (firstm >> u) & 1u ? (int)(m & 15u) : 0;
      const int bhi = (lastm >> u) & 1u ? (int)((m >> 4) & 15u) + 1 : 16;
      w = mask_chunk(w, blo, bhi);
    }
    acc_chunk(w, e, o);
  }
  flush(s_acc, s_meta, cur, e, o);
}

// ---- dense path: stream the tile's byte span --------------------------------
// Loads go through a buffer resource (SRD) whose range is the tile span:
// measured on MI355X, per-lane runs of 4 chunks stream at 6.26 TB/s through
// buffer_load_dwordx4 but only 5.46 TB/s through global_load_dwordx4, and the
// SRD range check returns zeros past the span (no clamping, no branches).
// AUX = cache-policy bits (0 default; 2 nt helps only fully coalesced reads).
template <int U, int AUX>
__device__ __forceinline__ void dense_load(__amdgpu_buffer_rsrc_t rsrc, uint32_t q0, uint4 (&v)[U]) {
#pragma unroll
  for (int u = 0; u < U; ++u) {
    auto x = __builtin_amdgcn_raw_buffer_load_b128(rsrc, (int)((q0 + u) * 16u), 0, AUX);
    v[u] = *reinterpret_cast<uint4*>(&x);
  }
}

// Attribute one lane run [16*q0, 16*(q0+U)) of the tile span to packets.
// s_S/s_E: packet start/end byte offsets in the span (both non-decreasing;
// empty packets have S == E).
template <int P, int U>
__device__ __forceinline__ void dense_consume(const uint4 (&v)[U], uint32_t q0, uint32_t C,
                                              const uint32_t* __restrict__ s_S,
                                              const uint32_t* __restrict__ s_E,
                                              const uint32_t* __restrict__ s_meta,
                                              uint32_t* __restrict__ s_acc, int& pk_floor) {
  constexpr int LOGP = __builtin_ctz(P);
  if (q0 >= C) return;
  const uint32_t rb = q0 * 16u;
  // First packet with E > rb, in [pk_floor, P].
  int lo = pk_floor, hi = P;
#pragma unroll
  for (int s = 0; s <= LOGP; ++s) {
    if (lo < hi) {
      const int mid = (lo + hi) >> 1;
      if (s_E[mid] > rb) hi = mid; else lo = mid + 1;
    }
  }
  int cur = lo;
  pk_floor = lo;
  if (cur >= P) return;
  uint32_t S = s_S[cur], E = s_E[cur];
  uint32_t e = 0, o = 0;
#pragma unroll
  for (int u = 0; u < U; ++u) {
    const uint32_t cb = rb + 16u * u;
    if (q0 + u >= C) break;
    const uint4 w = v[u];
    while (S < cb + 16u) {
      if (S <= cb && E >= cb + 16u) {
        acc_chunk(w, e, o);  // the whole chunk belongs to `cur`
      } else {
        const int blo = (int)(max(S, cb) - cb);
        const int bhi = (int)(min(E, cb + 16u) - cb);
        if (bhi > blo) acc_chunk(mask_chunk(w, blo, bhi), e, o);
      }
      if (E > cb + 16u) break;  // `cur` continues into the next chunk
      flush(s_acc, s_meta, cur, e, o);
      e = 0;
      o = 0;
      if (++cur >= P) break;
      S = s_S[cur];
      E = s_E[cur];
    }
    if (cur >= P) break;
  }
  if (cur < P) flush(s_acc, s_meta, cur, e, o);
}

// ---- dense path, LDS-DMA ring variant ---------------------------------------
// Each wave streams its share of the tile span in windows of 64*U chunks.  A
// window is fetched by U global_load_lds_dwordx4 (1 KiB each, fully coalesced,
// nontemporal) into a wave-private ring slot, NB slots deep, then every lane
// reads its run of U consecutive chunks back with ds_read_b128.  The source
// permutation below makes those reads bank-conflict-free: LDS position
// p = m + (64/U)*j of block b holds window chunk b*64 + U*m + j, so the 16
// lanes of a ds_read_b128 group hit 16 distinct 16-byte bank slots.
template <int U>
__device__ __forceinline__ uint32_t ring_src(int u, int lane) {
  constexpr int G = 64 / U;
  return (uint32_t)(u * 64 + U * (lane % G) + lane / G);
}
template <int U>
__device__ __forceinline__ uint32_t ring_pos(int lane, int j) {
  constexpr int G = 64 / U;
  return (uint32_t)(((lane * U) / 64) * 64 + (lane % G) + G * j);
}

// One 16-byte-per-lane LDS-DMA (global_load_lds_dwordx4): lane i's 16 bytes
// land at lds_dst + 16*i.  Issued from inline asm so that hipcc does not
// count it: otherwise it drains every in-flight DMA (vmcnt(0)) in front of any
// LDS store or atomic it cannot prove disjoint from the ring.  Completion is
// waited for explicitly with wait_vmcnt<N>() (cdna_hip_programming.md §5.7).
template <bool NT>
__device__ __forceinline__ void glds16(const void* gsrc, uint32_t lds_dst) {
  unsigned keep;
  if constexpr (NT) {
    asm volatile(
        "s_mov_b32 %0, m0\n\ts_mov_b32 m0, %2\n\ts_nop 0\n\t"
        "global_load_lds_dwordx4 %1, off nt\n\ts_mov_b32 m0, %0"
        : "=&s"(keep)
        : "v"(gsrc), "s"(lds_dst)
        : "memory");
  } else {
    asm volatile(
        "s_mov_b32 %0, m0\n\ts_mov_b32 m0, %2\n\ts_nop 0\n\t"
        "global_load_lds_dwordx4 %1, off\n\ts_mov_b32 m0, %0"
        : "=&s"(keep)
        : "v"(gsrc), "s"(lds_dst)
        : "memory");
  }
}

template <int N>
__device__ __forceinline__ void wait_vmcnt() {
  static_assert(N >= 0 && N < 64, "vmcnt is 6 bits");
  asm volatile("s_waitcnt vmcnt(%0)" ::"i"(N) : "memory");
}

// Template parameters: WG threads, D descriptors per thread (tile P = WG*D),
// UG / UD chunks per lane run on the general / dense path, NT nontemporal
// loads (each byte is read exactly once).
template <int WG, int D, int UG, int UD, bool NT, int DM = 0, int NB = 3>
__global__ __launch_bounds__(WG) void csum_batch(
    const uint8_t* __restrict__ arena, uint64_t arena_bytes,
    const uint4* __restrict__ desc, uint32_t n, uint16_t* __restrict__ out,
    uint32_t* __restrict__ partial, unsigned long long* __restrict__ err) {
  constexpr int P = WG * D;
  constexpr int NW = WG / 64;
  static_assert((P & (P - 1)) == 0, "tile must be a power of two");
  static_assert(UG * 1020 < 65536 && UD * 1020 < 65536, "packed 16-bit lanes would overflow");
  __shared__ uint64_t s_cstart[P + 1];  // general: virtual chunk start per packet
  __shared__ uint64_t s_cbase[P];       // general: chunk index - s_cstart; dense: S|E
  __shared__ uint32_t s_meta[P];
  __shared__ uint32_t s_acc[P];
  __shared__ uint64_t s_wsum[NW], s_wmax[NW], s_wmin[NW], s_wpay[NW];
  // dense path ring (DM == 1): NW waves x NB slots x 64*UD chunks
  __shared__ uint4 s_ring[DM == 1 ? NW * NB * 64 * UD : 1];

  const int t = threadIdx.x;
  const int lane = t & 63;
  const int wv = t >> 6;
  const uint64_t i0 = (uint64_t)blockIdx.x * P + (uint64_t)t * D;
  const uint64_t abase = (uint64_t)(uintptr_t)arena & 15u;  // arena-aligned coordinates

  uint64_t a[D], nch[D];
  uint32_t len[D], meta[D], init[D];
  uint64_t tsum = 0, tpay = 0, tmax = 0, tmin = ~0ull;
  bool sorted = true;
#pragma unroll
  for (int k = 0; k < D; ++k) {
    a[k] = 0;
    nch[k] = 0;
    len[k] = 0;
    meta[k] = 0;
    init[k] = 0;
    const uint64_t i = i0 + k;
    if (i < n) {
      const uint4 raw = desc[i];
      const uint64_t off = (uint64_t)raw.x | ((uint64_t)raw.y << 32);
      uint32_t l = raw.z;
      init[k] = raw.w & 0xFFFFu;
      const uint32_t odd = (raw.w >> 16) & 1u;
      if (off > arena_bytes || (uint64_t)l > arena_bytes - off) {
        l = 0;
        atomicAdd(err, 1ull);
      }
      if (l) {
        const uint64_t s = abase + off;
        const uint64_t last = s + l - 1;
        a[k] = s;
        len[k] = l;
        nch[k] = (last >> 4) - (s >> 4) + 1;
        meta[k] = (uint32_t)(s & 15u) | ((uint32_t)(last & 15u) << 4) |
                  ((uint32_t)((s + odd) & 1u) << 8);
        sorted = sorted && (s >= tmax);
        tmax = s + l;
        tmin = min(tmin, s);
        tpay += l;
      }
    }
    tsum += nch[k];
  }

  // Wave scans (sum of chunk counts, max of ends) and reductions.
  uint64_t isum = tsum, imax = tmax, rmin = tmin, rpay = tpay;
#pragma unroll
  for (int d = 1; d < 64; d <<= 1) {
    const uint64_t ys = __shfl_up(isum, d, 64);
    const uint64_t ym = __shfl_up(imax, d, 64);
    if (lane >= d) {
      isum += ys;
      imax = max(imax, ym);
    }
    rmin = min(rmin, __shfl_xor(rmin, d, 64));
    rpay += __shfl_xor(rpay, d, 64);
  }
  // Exclusive max of ends before this thread, within the wave.
  uint64_t xmax = __shfl_up(imax, 1, 64);
  if (lane == 0) xmax = 0;
  if (lane == 63) {
    s_wsum[wv] = isum;
    s_wmax[wv] = imax;
    s_wmin[wv] = rmin;
    s_wpay[wv] = rpay;
  }
  // First non-empty start of this thread vs everything before it.
  uint64_t first = ~0ull;
#pragma unroll
  for (int k = D - 1; k >= 0; --k)
    if (len[k]) first = a[k];
  __syncthreads();
  uint64_t run = isum - tsum, tot = 0, maxend = 0, minstart = ~0ull, pay = 0;
#pragma unroll
  for (int w = 0; w < NW; ++w) {
    if (w < wv) {
      run += s_wsum[w];
      xmax = max(xmax, s_wmax[w]);
    }
    tot += s_wsum[w];
    maxend = max(maxend, s_wmax[w]);
    minstart = min(minstart, s_wmin[w]);
    pay += s_wpay[w];
  }
  if (first != ~0ull && first < xmax) sorted = false;
  const bool all_sorted = __syncthreads_and(sorted);
  const uint64_t tbase = (minstart == ~0ull) ? 0 : (minstart & ~15ull);
  const uint64_t span = (minstart == ~0ull) ? 0 : maxend - tbase;
  const bool dense = all_sorted && pay != 0 && span < (1ull << 31) &&
                     span <= pay + (pay >> 3) + 64ull * P;

  uint32_t* s_S = reinterpret_cast<uint32_t*>(s_cbase);
  uint32_t* s_E = s_S + P;
  if (dense) {
    uint64_t rm = xmax;  // running max end before descriptor k
#pragma unroll
    for (int k = 0; k < D; ++k) {
      const int idx = t * D + k;
      if (len[k]) {
        s_S[idx] = (uint32_t)(a[k] - tbase);
        s_E[idx] = (uint32_t)(a[k] + len[k] - tbase);
        rm = a[k] + len[k];
      } else {
        const uint32_t z = rm > tbase ? (uint32_t)(rm - tbase) : 0u;
        s_S[idx] = z;
        s_E[idx] = z;
      }
      s_meta[idx] = meta[k] & kPhaseBit;
      s_acc[idx] = 0u;
    }
  } else {
#pragma unroll
    for (int k = 0; k < D; ++k) {
      const int idx = t * D + k;
      s_cstart[idx] = run;
      s_cbase[idx] = (len[k] ? (a[k] >> 4) : 0) - run;
      s_meta[idx] = meta[k];
      s_acc[idx] = 0u;
      run += nch[k];
    }
    if (t == WG - 1) s_cstart[P] = run;
  }
  __syncthreads();

  const uint4* __restrict__ chunks = reinterpret_cast<const uint4*>(arena - abase);
  if (dense && DM == 1) {
    const uint32_t C = (uint32_t)((span + 15) >> 4);
    const uint4* __restrict__ tb = chunks + (tbase >> 4);
    constexpr uint32_t WIN = 64u * UD;
    const uint32_t nwin = (C + WIN - 1) / WIN;
    const int w = __builtin_amdgcn_readfirstlane(wv);
    const uint32_t k0 = (uint32_t)(((uint64_t)nwin * w) / NW);
    const uint32_t k1 = (uint32_t)(((uint64_t)nwin * (w + 1)) / NW);
    uint4* ring = s_ring + (size_t)w * NB * WIN;
    // LDS byte offset of this wave's ring (wave-uniform, in an SGPR).
    const uint32_t ring_lds = (uint32_t)(uintptr_t)(__attribute__((address_space(3))) uint4*)ring;
    auto issue = [&](uint32_t k) {
      const uint32_t slot = __builtin_amdgcn_readfirstlane(ring_lds + (k % NB) * WIN * 16u);
#pragma unroll
      for (int u = 0; u < UD; ++u) {
        // Out-of-range lanes re-read the last chunk instead of being masked
        // off, so every wave-instruction issues and the vmcnt counts hold.
        const uint32_t src = min(k * WIN + ring_src<UD>(u, lane), C - 1);
        glds16<NT>(tb + src, slot + u * 1024u);
      }
    };
#pragma unroll
    for (int a0 = 0; a0 < NB - 1; ++a0)
      if (k0 + a0 < k1) issue(k0 + a0);
    int pk_floor = 0;
    for (uint32_t k = k0; k < k1; ++k) {
      if (k + NB - 1 < k1) {
        issue(k + NB - 1);
        wait_vmcnt<(NB - 1) * UD>();
      } else {
        wait_vmcnt<0>();
      }
      const uint4* slot = ring + (k % NB) * WIN;
      uint4 v[UD];
#pragma unroll
      for (int j = 0; j < UD; ++j) v[j] = slot[ring_pos<UD>(lane, j)];
      dense_consume<P, UD>(v, k * WIN + (uint32_t)lane * UD, C, s_S, s_E, s_meta, s_acc, pk_floor);
    }
  } else if (dense) {
    const uint32_t C = (uint32_t)((span + 15) >> 4);
    // Wave-uniform SRD over the tile span (readfirstlane: T20, no waterfall).
    const uint64_t tbp = (uint64_t)(uintptr_t)(chunks + (tbase >> 4));
    const uint32_t lo32 = __builtin_amdgcn_readfirstlane((uint32_t)tbp);
    const uint32_t hi32 = __builtin_amdgcn_readfirstlane((uint32_t)(tbp >> 32));
    const uint32_t nrec = __builtin_amdgcn_readfirstlane(C * 16u);
    const __amdgpu_buffer_rsrc_t rsrc = __builtin_amdgcn_make_buffer_rsrc(
        (void*)(((uint64_t)hi32 << 32) | lo32), (short)0, (int)nrec, 0x00020000);
    constexpr uint32_t STEP = (uint32_t)WG * UD;
    constexpr int AUX = NT ? 2 : 0;
    int pk_floor = 0;
    uint4 va[UD], vb[UD];
    uint32_t q = (uint32_t)t * UD;
    dense_load<UD, AUX>(rsrc, q, va);
    while (q < C) {
      dense_load<UD, AUX>(rsrc, q + STEP, vb);
      dense_consume<P, UD>(va, q, C, s_S, s_E, s_meta, s_acc, pk_floor);
      q += STEP;
      if (q >= C) break;
      dense_load<UD, AUX>(rsrc, q + STEP, va);
      dense_consume<P, UD>(vb, q, C, s_S, s_E, s_meta, s_acc, pk_floor);
      q += STEP;
    }
  } else {
    int pk_floor = 0;
    for (uint64_t c0 = (uint64_t)t * UG; c0 < tot; c0 += (uint64_t)WG * UG)
      general_step<P, UG, NT>(chunks, s_cstart, s_cbase, s_meta, s_acc, tot, c0, pk_floor);
  }
  __syncthreads();

#pragma unroll
  for (int k = 0; k < D; ++k) {
    const uint64_t i = i0 + k;
    if (i < n) {
      const uint32_t sacc = s_acc[t * D + k];
      if (partial) partial[i] = sacc;
      else out[i] = (uint16_t)fold1(init[k] + sacc);
    }
  }
}

// ===========================================================================
// csum_runs — the production kernel (arena < 4 GiB).
//
// Each packet is split into   head | body | tail:
//   head = its first 16-byte chunk if the packet does not start on a chunk
//          boundary (byte-masked), tail = its last chunk if it does not end on
//          one (byte-masked); a packet inside one chunk is a lone head;
//   body = the chunks it covers completely — no masking.
// Body chunks are cut into packet-aligned runs of U chunks (a packet with no
// full chunk gets one empty run).  The tile's runs are scanned into LDS and
// each lane takes one run per step: a branch-free binary search for its
// packet, U buffer_load_dwordx4 of consecutive chunks (lanes U*16 B apart: the
// run shape that streams at ~6.3 TB/s through buffer loads on MI355X), plus —
// only on the packet's first / last run — the head / tail chunk, adjacent in
// address and time so its 128-B line is fetched once.  Then 2 VALU per dword:
//   T += v_sad_u8(w, 0)   (sum of the 4 bytes)
//   W += v_sad_u16(w, 0)  (sum of the 2 little-endian 16-bit words)
// and the big-endian word sum of checksum.go:41-43 is
//   S = 256*E + O = 257*T - W   (first byte at an even address, phase 0)
//   S = E + 256*O = W           (phase 1)
// with E/O the bytes at even/odd addresses — all mod 2^32, so bit-exact
// including the > 128 KiB wrap.  A run never crosses a packet, so each run
// ends in exactly one ds_add_u32 into its packet's LDS accumulator.  Runs are
// software-pipelined one step deep (PIPE).
// Out-of-range slots load from offset num_records (the SRD's own size): out of
// range under both "offset >= size" and "offset + 16 > size" checks and far
// from 32-bit wrap, so the hardware returns zeros without touching memory.
// (An offset near 2^32 is NOT safe: offset + 16 wraps and passes the check.)
// ===========================================================================
constexpr uint64_t kMaxSrdBytes = 0xFFFF0000ull;  // arenas at or above: launch_general

template <int AUX = 0>
__device__ __forceinline__ uint4 bload(__amdgpu_buffer_rsrc_t r, uint32_t off) {
  auto x = __builtin_amdgcn_raw_buffer_load_b128(r, (int)off, 0, AUX);
  return *reinterpret_cast<uint4*>(&x);
}

__device__ __forceinline__ void sad_chunk(const uint4 w, uint32_t& T, uint32_t& W) {
  T = __builtin_amdgcn_sad_u8(w.x, 0u, T);
  W = __builtin_amdgcn_sad_u16(w.x, 0u, W);
  T = __builtin_amdgcn_sad_u8(w.y, 0u, T);
  W = __builtin_amdgcn_sad_u16(w.y, 0u, W);
  T = __builtin_amdgcn_sad_u8(w.z, 0u, T);
  W = __builtin_amdgcn_sad_u16(w.z, 0u, W);
  T = __builtin_amdgcn_sad_u8(w.w, 0u, T);
  W = __builtin_amdgcn_sad_u16(w.w, 0u, W);
}

__device__ __forceinline__ uint32_t s_of(uint32_t T, uint32_t W, uint32_t phase) {
  return phase ? W : (257u * T - W);
}

// Per-packet edge word (LDS): bit 0 head, bit 1 tail, head bytes [hlo, hhi),
// tail bytes [0, thi), bit 31 phase.
__device__ __forceinline__ uint32_t edge_word(uint32_t has_h, uint32_t has_t, uint32_t hlo,
                                              uint32_t hhi, uint32_t thi, uint32_t phase) {
  return has_h | (has_t << 1) | (hlo << 2) | (hhi << 7) | (thi << 12) | (phase << 31);
}

template <int U>
struct RunStage {
  uint4 v[U];
  uint4 h, tl;   // head / tail chunk (zeros unless this run carries them)
  uint32_t ew;   // the packet's edge word, with bits 0/1 cleared unless carried here
  int pk;
};

// PERSIST: the grid is sized to the resident workgroup slots and workgroup w
// owns descriptors [n*w/G, n*(w+1)/G), walked in sub-tiles of WG: every
// workgroup ends together (no under-filled last round of tiles).
template <int WG, int U, bool PIPE = true, bool PERSIST = false>
__global__ __launch_bounds__(WG) void csum_runs(
    const uint8_t* __restrict__ arena, uint64_t arena_bytes,
    const uint4* __restrict__ desc, uint32_t n, uint16_t* __restrict__ out,
    uint32_t* __restrict__ partial, unsigned long long* __restrict__ err) {
  constexpr int P = WG;
  constexpr int NW = WG / 64;
  static_assert((P & (P - 1)) == 0, "tile must be a power of two");
  __shared__ uint64_t s_rstart[P + 1];  // first run of each packet (tile-relative)
  __shared__ uint32_t s_body[P];        // SRD byte offset of the packet's first body chunk
  __shared__ uint32_t s_nb[P];          // body chunks
  __shared__ uint32_t s_edge[P];        // edge word
  __shared__ uint32_t s_acc[P];
  __shared__ uint64_t s_wtot[NW];

  const int t = threadIdx.x;
  const int lane = t & 63;
  const int wv = t >> 6;

  // SRD over the whole arena, from its 16-byte-aligned base (the launcher
  // guarantees the rounded size is below kMaxSrdBytes).
  const uint64_t abase = (uint64_t)(uintptr_t)arena & 15u;
  const uint64_t sb = (uint64_t)(uintptr_t)arena - abase;
  const uint32_t nrec = (uint32_t)((abase + arena_bytes + 15) & ~15ull);
  // readfirstlane returns int: widen through uint32_t (a sign-extended low
  // word would corrupt the base's high bits).
  const uint32_t sb_lo = (uint32_t)__builtin_amdgcn_readfirstlane((uint32_t)sb);
  const uint32_t sb_hi = (uint32_t)__builtin_amdgcn_readfirstlane((uint32_t)(sb >> 32));
  const __amdgpu_buffer_rsrc_t rsrc = __builtin_amdgcn_make_buffer_rsrc(
      (void*)(((uint64_t)sb_hi << 32) | (uint64_t)sb_lo), (short)0,
      (int)__builtin_amdgcn_readfirstlane(nrec), 0x00020000);
  const uint32_t oob = (uint32_t)__builtin_amdgcn_readfirstlane(nrec);

  uint64_t tile_lo, tile_end;
  if constexpr (PERSIST) {
    tile_lo = (uint64_t)n * blockIdx.x / gridDim.x;
    tile_end = (uint64_t)n * (blockIdx.x + 1) / gridDim.x;
  } else {
    tile_lo = (uint64_t)blockIdx.x * P;
    tile_end = min<uint64_t>(tile_lo + P, n);
  }
  for (; tile_lo < tile_end; tile_lo += P) {
  const uint64_t i = tile_lo + t;
  const uint64_t lim = min<uint64_t>(tile_end, tile_lo + P);
  uint32_t init = 0, nb = 0, body = 0, ew = 0, nr = 0;
  if (i < lim) {
    const uint4 raw = desc[i];
    const uint64_t off = (uint64_t)raw.x | ((uint64_t)raw.y << 32);
    uint32_t len = raw.z;
    init = raw.w & 0xFFFFu;
    const uint32_t odd = (raw.w >> 16) & 1u;
    if (off > arena_bytes || (uint64_t)len > arena_bytes - off) {
      len = 0;
      atomicAdd(err, 1ull);
    }
    if (len) {
      const uint32_t a = (uint32_t)(abase + off);
      const uint32_t e = a + len;  // exclusive end
      const uint32_t cf = a >> 4, cl = (e - 1) >> 4;
      const uint32_t lo = a & 15u, hiex = ((e - 1) & 15u) + 1u;
      const uint32_t phase = (a + odd) & 1u;
      if (cf == cl) {  // inside one chunk: a lone head
        ew = edge_word(1u, 0u, lo, hiex, 16u, phase);
        body = (cf + 1u) * 16u;
        nb = 0;
      } else {
        const uint32_t hh = lo ? 1u : 0u, ht = hiex != 16u ? 1u : 0u;
        ew = edge_word(hh, ht, lo, 16u, hiex, phase);
        const uint32_t bf = cf + hh;
        nb = (cl - ht) + 1u - bf;
        body = bf * 16u;
      }
      nr = nb ? (nb + (U - 1)) / U : 1u;
    }
  }

  // Block-wide exclusive scan of run counts.
  uint64_t incl = nr;
#pragma unroll
  for (int d = 1; d < 64; d <<= 1) {
    const uint64_t y = __shfl_up(incl, d, 64);
    if (lane >= d) incl += y;
  }
  if (lane == 63) s_wtot[wv] = incl;
  __syncthreads();
  uint64_t excl = incl - nr;
#pragma unroll
  for (int w = 0; w < NW; ++w)
    if (w < wv) excl += s_wtot[w];
  s_rstart[t] = excl;
  s_body[t] = body;
  s_nb[t] = nb;
  s_edge[t] = ew;
  s_acc[t] = 0u;
  if (t == WG - 1) s_rstart[P] = excl + nr;
  __syncthreads();

  const uint64_t R = s_rstart[P];
  auto stage = [&](uint64_t q, RunStage<U>& st) {
    // Largest p with s_rstart[p] <= q (that packet has a run q): fixed-step,
    // branch-free search (s_rstart[0] = 0 <= q always holds).
    int lo = 0;
#pragma unroll
    for (int step = P / 2; step >= 1; step >>= 1)
      lo = (s_rstart[lo + step] <= q) ? lo + step : lo;
    const uint64_t r0 = s_rstart[lo];
    const uint32_t k = (uint32_t)(q - r0);
    const uint32_t last = (uint32_t)(s_rstart[lo + 1] - r0) - 1u;
    const uint32_t nbp = s_nb[lo];
    const uint32_t c0 = k * U;
    const uint32_t nvalid = nbp > c0 ? min((uint32_t)U, nbp - c0) : 0u;
    const uint32_t bo = s_body[lo];
    const uint32_t base = bo + c0 * 16u;
#pragma unroll
    for (int j = 0; j < U; ++j) st.v[j] = bload(rsrc, (uint32_t)j < nvalid ? base + 16u * j : oob);
    uint32_t e = s_edge[lo];
    if (k != 0) e &= ~1u;
    if (k != last) e &= ~2u;
    st.h = make_uint4(0, 0, 0, 0);
    st.tl = make_uint4(0, 0, 0, 0);
    if (e & 1u) st.h = bload(rsrc, bo - 16u);
    if (e & 2u) st.tl = bload(rsrc, bo + nbp * 16u);
    st.ew = e;
    st.pk = lo;
  };
  auto consume = [&](const RunStage<U>& st) {
    uint32_t T = 0, W = 0;
#pragma unroll
    for (int j = 0; j < U; ++j) sad_chunk(st.v[j], T, W);
    const uint32_t e = st.ew;
    if (e & 3u) {
      sad_chunk(mask_chunk(st.h, (int)((e >> 2) & 31u), (int)((e >> 7) & 31u)), T, W);
      sad_chunk(mask_chunk(st.tl, 0, (int)((e >> 12) & 31u)), T, W);
    }
    atomicAdd(&s_acc[st.pk], s_of(T, W, e >> 31));
  };
  if constexpr (PIPE) {
    // Software pipeline: run q+WG is looked up and its loads issued before
    // run q is consumed (two register stages, unrolled by 2).
    RunStage<U> sa, sbg;
    uint64_t q = (uint64_t)t;
    if (q < R) stage(q, sa);
    while (q < R) {
      if (q + WG < R) stage(q + WG, sbg);
      consume(sa);
      q += WG;
      if (q >= R) break;
      if (q + WG < R) stage(q + WG, sa);
      consume(sbg);
      q += WG;
    }
  } else {
    for (uint64_t q = (uint64_t)t; q < R; q += WG) {
      RunStage<U> st;
      stage(q, st);
      consume(st);
    }
  }
  __syncthreads();

  if (i < lim) {
    const uint32_t sacc = s_acc[t];
    if (partial) partial[i] = sacc;
    else out[i] = (uint16_t)fold1(init + sacc);
  }
  }  // sub-tiles
}

// ===========================================================================
// csum_grp — lane groups over a packet's chunks (arena < 4 GiB).
//
// A packet covers chunks [cf, cl] of the arena (16-B aligned address space);
// they are cut into packet-aligned runs of G*U chunks and a run belongs to a
// group of G adjacent lanes: lane li loads chunks li, li+G, ..., li+(U-1)G of
// the run, so every load instruction reads G*16 contiguous bytes per group —
// for G = 8 one full 128-B line, the fully coalesced shape rather than the
// per-lane run shape (lanes U*16 B apart) of csum_runs.  The packet's first
// and last chunk are byte-masked where they are loaded (no separate edge
// loads); the group's partials are summed with DPP (S is linear in T and W
// for a fixed phase) and lane 0 of the group issues the one ds_add_u32.
// ===========================================================================
template <int G>
__device__ __forceinline__ uint32_t group_sum(uint32_t s) {
  static_assert(G == 1 || G == 2 || G == 4 || G == 8 || G == 16, "group of 1..16 lanes");
  if constexpr (G >= 2) s += (uint32_t)__builtin_amdgcn_update_dpp(0, (int)s, 0xB1, 0xF, 0xF, false);   // quad_perm 1,0,3,2
  if constexpr (G >= 4) s += (uint32_t)__builtin_amdgcn_update_dpp(0, (int)s, 0x4E, 0xF, 0xF, false);   // quad_perm 2,3,0,1
  if constexpr (G >= 8) s += (uint32_t)__builtin_amdgcn_update_dpp(0, (int)s, 0x141, 0xF, 0xF, false);  // row_half_mirror
  if constexpr (G >= 16) s += (uint32_t)__builtin_amdgcn_update_dpp(0, (int)s, 0x140, 0xF, 0xF, false); // row_mirror
  return s;
}

template <int U>
struct GrpStage {
  uint4 v[U];
  uint32_t ci0;  // chunk index (within the packet) of v[0]
  uint32_t nch;  // the packet's chunk count
  uint32_t ew;   // lo | hiex << 5 | phase << 31
  int pk;
};

template <int WG, int G, int U, bool PIPE, int AUX = 0>
__global__ __launch_bounds__(WG) void csum_grp(
    const uint8_t* __restrict__ arena, uint64_t arena_bytes,
    const uint4* __restrict__ desc, uint32_t n, uint16_t* __restrict__ out,
    uint32_t* __restrict__ partial, unsigned long long* __restrict__ err) {
  constexpr int P = WG;
  constexpr int NW = WG / 64;
  constexpr int NG = WG / G;     // groups per workgroup
  constexpr uint32_t RC = G * U; // chunks per run
  static_assert((P & (P - 1)) == 0, "tile must be a power of two");
  __shared__ uint64_t s_rstart[P + 1];
  __shared__ uint32_t s_first[P];  // SRD byte offset of chunk cf
  __shared__ uint32_t s_nch[P];
  __shared__ uint32_t s_edge[P];
  __shared__ uint32_t s_acc[P];
  __shared__ uint64_t s_wtot[NW];

  const int t = threadIdx.x;
  const int lane = t & 63;
  const int wv = t >> 6;
  const int grp = t / G;
  const uint32_t li = (uint32_t)(t % G);

  const uint64_t abase = (uint64_t)(uintptr_t)arena & 15u;
  const uint64_t sb = (uint64_t)(uintptr_t)arena - abase;
  const uint32_t nrec = (uint32_t)((abase + arena_bytes + 15) & ~15ull);
  const uint32_t sb_lo = (uint32_t)__builtin_amdgcn_readfirstlane((uint32_t)sb);
  const uint32_t sb_hi = (uint32_t)__builtin_amdgcn_readfirstlane((uint32_t)(sb >> 32));
  const __amdgpu_buffer_rsrc_t rsrc = __builtin_amdgcn_make_buffer_rsrc(
      (void*)(((uint64_t)sb_hi << 32) | (uint64_t)sb_lo), (short)0,
      (int)__builtin_amdgcn_readfirstlane(nrec), 0x00020000);
  const uint32_t oob = (uint32_t)__builtin_amdgcn_readfirstlane(nrec);

  const uint64_t tile_lo = (uint64_t)blockIdx.x * P;
  const uint64_t i = tile_lo + t;
  const uint64_t lim = min<uint64_t>(tile_lo + P, n);
  uint32_t init = 0, nch = 0, first = 0, ew = 0, nr = 0;
  if (i < lim) {
    const uint4 raw = desc[i];
    const uint64_t off = (uint64_t)raw.x | ((uint64_t)raw.y << 32);
    uint32_t len = raw.z;
    init = raw.w & 0xFFFFu;
    const uint32_t odd = (raw.w >> 16) & 1u;
    if (off > arena_bytes || (uint64_t)len > arena_bytes - off) {
      len = 0;
      atomicAdd(err, 1ull);
    }
    if (len) {
      const uint32_t a = (uint32_t)(abase + off);
      const uint32_t e = a + len;
      const uint32_t cf = a >> 4, cl = (e - 1) >> 4;
      nch = cl - cf + 1u;
      first = cf * 16u;
      ew = (a & 15u) | ((((e - 1) & 15u) + 1u) << 5) | (((a + odd) & 1u) << 31);
      nr = (nch + RC - 1) / RC;
    }
  }

  uint64_t incl = nr;
#pragma unroll
  for (int d = 1; d < 64; d <<= 1) {
    const uint64_t y = __shfl_up(incl, d, 64);
    if (lane >= d) incl += y;
  }
  if (lane == 63) s_wtot[wv] = incl;
  __syncthreads();
  uint64_t excl = incl - nr;
#pragma unroll
  for (int w = 0; w < NW; ++w)
    if (w < wv) excl += s_wtot[w];
  s_rstart[t] = excl;
  s_first[t] = first;
  s_nch[t] = nch;
  s_edge[t] = ew;
  s_acc[t] = 0u;
  if (t == WG - 1) s_rstart[P] = excl + nr;
  __syncthreads();

  const uint64_t R = s_rstart[P];
  auto stage = [&](uint64_t q, GrpStage<U>& st) {
    int lo = 0;
#pragma unroll
    for (int step = P / 2; step >= 1; step >>= 1)
      lo = (s_rstart[lo + step] <= q) ? lo + step : lo;
    const uint32_t k = (uint32_t)(q - s_rstart[lo]);
    const uint32_t nc = s_nch[lo];
    const uint32_t ci0 = k * RC + li;
    const uint32_t base = s_first[lo] + ci0 * 16u;
#pragma unroll
    for (int j = 0; j < U; ++j)
      st.v[j] = bload<AUX>(rsrc, ci0 + (uint32_t)(G * j) < nc ? base + (uint32_t)(16 * G * j) : oob);
    st.ci0 = ci0;
    st.nch = nc;
    st.ew = s_edge[lo];
    st.pk = lo;
  };
  auto consume = [&](const GrpStage<U>& st) {
    uint32_t T = 0, W = 0;
    const uint32_t lastc = st.nch - 1u;
#pragma unroll
    for (int j = 0; j < U; ++j) {
      const uint32_t ci = st.ci0 + (uint32_t)(G * j);
      uint4 w = st.v[j];
      if (ci == 0u || ci == lastc)
        w = mask_chunk(w, ci == 0u ? (int)(st.ew & 31u) : 0, ci == lastc ? (int)((st.ew >> 5) & 31u) : 16);
      sad_chunk(w, T, W);
    }
    const uint32_t s = group_sum<G>(s_of(T, W, st.ew >> 31));
    if (li == 0) atomicAdd(&s_acc[st.pk], s);
  };
  if constexpr (PIPE) {
    GrpStage<U> sa, sbg;
    uint64_t q = (uint64_t)grp;
    if (q < R) stage(q, sa);
    while (q < R) {
      if (q + NG < R) stage(q + NG, sbg);
      consume(sa);
      q += NG;
      if (q >= R) break;
      if (q + NG < R) stage(q + NG, sa);
      consume(sbg);
      q += NG;
    }
  } else {
    for (uint64_t q = (uint64_t)grp; q < R; q += NG) {
      GrpStage<U> st;
      stage(q, st);
      consume(st);
    }
  }
  __syncthreads();

  if (i < lim) {
    const uint32_t sacc = s_acc[t];
    if (partial) partial[i] = sacc;
    else out[i] = (uint16_t)fold1(init + sacc);
  }
}

// ===========================================================================
// csum_hyb — two lane shapes in one tile, chosen per packet.
//
// Nontemporal loads stream at ~6.8 TB/s on MI355X when every 128-B line is
// consumed by ONE wave instruction (groups of 16 lanes = 256 contiguous bytes
// per instruction), and lose badly when a line is split across instructions
// (the evicted line is fetched again).  So a packet of at least `big_chunks`
// chunks goes to a group of GB = 16 lanes (runs of GB*UB chunks, nt loads),
// and a smaller one to a single lane (runs of US consecutive chunks, default
// policy — its lines are shared with neighbouring packets and must stay in L2).
// One prologue scans both run counts (packed in a u64); two loops follow.
//
// LA: a big packet's body is cut at 128-B line boundaries — chunks [0, h) and
// [ts, nch) (the partial lines it shares with its neighbours) go to the
// default-policy lane runs, [h, ts) to the nontemporal groups, so every nt
// instruction reads whole lines no other packet touches.
//
// UD > 0 adds a direct path for tiles of small packets: when every packet of
// the tile spans at most UD chunks (a block-wide vote), each lane loads its
// own packet right after its descriptor — no scan, no search, no LDS atomics.
// PERSIST sizes the grid to the resident workgroup slots; workgroup w owns
// descriptors [n*w/G, n*(w+1)/G) in sub-tiles, and the next sub-tile's
// descriptors are loaded while the current one streams.
// ===========================================================================

// One descriptor, decoded: the chunks [cf, cf + nch) it covers (first = cf*16,
// the SRD offset), its edge word (lo | hiex << 5 | phase << 31) and initial.
struct PktInfo {
  uint32_t init, nch, first, ew;
};

__device__ __forceinline__ PktInfo pkt_info(uint4 raw, bool mine, uint64_t abase,
                                            uint64_t arena_bytes, unsigned long long* err) {
  PktInfo p{0u, 0u, 0u, 0u};
  if (!mine) return p;
  const uint64_t off = (uint64_t)raw.x | ((uint64_t)raw.y << 32);
  uint32_t len = raw.z;
  p.init = raw.w & 0xFFFFu;
  const uint32_t odd = (raw.w >> 16) & 1u;
  if (off > arena_bytes || (uint64_t)len > arena_bytes - off) {
    len = 0;
    atomicAdd(err, 1ull);
  }
  if (len) {
    const uint32_t a = (uint32_t)(abase + off);
    const uint32_t e = a + len;
    const uint32_t cf = a >> 4, cl = (e - 1) >> 4;
    p.nch = cl - cf + 1u;
    p.first = cf * 16u;
    p.ew = (a & 15u) | ((((e - 1) & 15u) + 1u) << 5) | (((a + odd) & 1u) << 31);
  }
  return p;
}

__device__ __forceinline__ uint4 edge_mask(uint4 w, uint32_t ci, uint32_t lastc, uint32_t e) {
  if (ci == 0u || ci == lastc)
    w = mask_chunk(w, ci == 0u ? (int)(e & 31u) : 0, ci == lastc ? (int)((e >> 5) & 31u) : 16);
  return w;
}

__device__ __forceinline__ void put_result(const PktInfo& p, uint32_t sacc, uint64_t i,
                                           uint16_t* out, uint32_t* partial) {
  if (partial) partial[i] = sacc;
  else out[i] = (uint16_t)fold1(p.init + sacc);
}

template <int P, bool LA>
struct HybLds {
  uint32_t rb[P + 1];   // first big run of each packet
  uint32_t rs[P + 1];   // first small run of each packet
  uint32_t first[P];
  uint32_t nch[P];
  uint32_t edge[P];
  uint32_t acc[P];
  uint32_t hts[LA ? P : 1];  // LA: split | h << 1 | ts << 4 (0: not split)
  uint64_t wtot[P / 64];
};

struct Srd {
  __amdgpu_buffer_rsrc_t rsrc;
  uint32_t oob;    // an offset the range check rejects: the SRD's own size
  uint32_t sb_lo;  // low word of the 16-B-aligned base (128-B line phase)
  uint64_t abase;  // arena - base (0..15)
};

__device__ __forceinline__ Srd make_srd(const uint8_t* arena, uint64_t arena_bytes) {
  Srd r;
  r.abase = (uint64_t)(uintptr_t)arena & 15u;
  const uint64_t sb = (uint64_t)(uintptr_t)arena - r.abase;
  const uint32_t nrec = (uint32_t)((r.abase + arena_bytes + 15) & ~15ull);
  // readfirstlane returns int: widen through uint32_t (a sign-extended low
  // word would corrupt the base's high bits).
  r.sb_lo = (uint32_t)__builtin_amdgcn_readfirstlane((uint32_t)sb);
  const uint32_t sb_hi = (uint32_t)__builtin_amdgcn_readfirstlane((uint32_t)(sb >> 32));
  r.rsrc = __builtin_amdgcn_make_buffer_rsrc((void*)(((uint64_t)sb_hi << 32) | (uint64_t)r.sb_lo),
                                             (short)0, (int)__builtin_amdgcn_readfirstlane(nrec),
                                             0x00020000);
  r.oob = (uint32_t)__builtin_amdgcn_readfirstlane(nrec);
  return r;
}

// The direct path's per-lane sum of one packet of at most UD chunks.
template <int UD>
__device__ __forceinline__ void direct_load(const Srd& r, const PktInfo& p, uint4 (&v)[UD]) {
#pragma unroll
  for (int j = 0; j < UD; ++j) v[j] = bload(r.rsrc, (uint32_t)j < p.nch ? p.first + 16u * j : r.oob);
}

template <int UD>
__device__ __forceinline__ uint32_t direct_sum(const PktInfo& p, const uint4 (&v)[UD]) {
  uint32_t T = 0, W = 0;
#pragma unroll
  for (int j = 0; j < UD; ++j) sad_chunk(edge_mask(v[j], (uint32_t)j, p.nch - 1u, p.ew), T, W);
  return s_of(T, W, p.ew >> 31);
}

// One tile of WG descriptors through the scan path (thread t holds packet p of
// global index i).  Every thread of the block must call it.
template <int WG, int GB, int UB, int US, int AUXB, bool LA>
__device__ __forceinline__ void hyb_scan_tile(HybLds<WG, LA>& L, const Srd& r, const PktInfo& p,
                                              bool mine, uint64_t i, uint16_t* __restrict__ out,
                                              uint32_t* __restrict__ partial, uint32_t big_chunks) {
  constexpr int P = WG;
  constexpr int NW = WG / 64;
  constexpr int NG = WG / GB;
  constexpr uint32_t RB = GB * UB;
  const int t = threadIdx.x;
  const int lane = t & 63;
  const int wv = t >> 6;
  const uint32_t li = (uint32_t)(t % GB);
  const uint32_t nch = p.nch;

  uint32_t h = nch, ts = nch;
  if (LA && nch >= big_chunks) {
    const uint32_t cph = ((r.sb_lo >> 4) + (p.first >> 4)) & 7u;  // chunk slot in its 128-B line
    h = (8u - cph) & 7u;
    ts = ((cph + nch) & ~7u) - cph;
  }
  // arena < 4 GiB: at most 2^28 chunks per packet, so a tile's big-run total
  // stays below 2^32; small packets have < big_chunks chunks.
  const uint64_t nr = nch == 0 ? 0ull
                      : !LA ? (nch >= big_chunks ? (uint64_t)((nch + RB - 1) / RB)
                                                 : ((uint64_t)((nch + US - 1) / US) << 32))
                      : nch >= big_chunks
                          ? ((uint64_t)((ts - h + RB - 1) / RB) |
                             ((uint64_t)((h + US - 1) / US + (nch - ts + US - 1) / US) << 32))
                          : ((uint64_t)((nch + US - 1) / US) << 32);
  uint64_t incl = nr;
#pragma unroll
  for (int d = 1; d < 64; d <<= 1) {
    const uint64_t y = __shfl_up(incl, d, 64);
    if (lane >= d) incl += y;
  }
  if (lane == 63) L.wtot[wv] = incl;
  __syncthreads();
  uint64_t excl = incl - nr;
#pragma unroll
  for (int w = 0; w < NW; ++w)
    if (w < wv) excl += L.wtot[w];
  L.rb[t] = (uint32_t)excl;
  L.rs[t] = (uint32_t)(excl >> 32);
  L.first[t] = p.first;
  L.nch[t] = nch;
  L.edge[t] = p.ew;
  if constexpr (LA) L.hts[t] = (nch >= big_chunks) ? (1u | (h << 1) | (ts << 4)) : 0u;
  L.acc[t] = 0u;
  if (t == WG - 1) {
    L.rb[P] = (uint32_t)(excl + nr);
    L.rs[P] = (uint32_t)((excl + nr) >> 32);
  }
  __syncthreads();

  auto search = [&](const uint32_t* s_r, uint32_t q) {
    int lo = 0;
#pragma unroll
    for (int step = P / 2; step >= 1; step >>= 1)
      lo = (s_r[lo + step] <= q) ? lo + step : lo;
    return lo;
  };

  // Big packets: groups of GB lanes, lane li takes chunks li + GB*j of a run.
  const uint32_t RBt = L.rb[P];
  for (uint32_t q = (uint32_t)(t / GB); q < RBt; q += NG) {
    const int pk = search(L.rb, q);
    const uint32_t nc = L.nch[pk];
    uint32_t ci0 = (q - L.rb[pk]) * RB + li, cend = nc;
    if constexpr (LA) {  // every big packet is split: body [h, ts)
      const uint32_t hts = L.hts[pk];
      ci0 += (hts >> 1) & 7u;
      cend = hts >> 4;
    }
    const uint32_t base = L.first[pk] + ci0 * 16u;
    uint4 v[UB];
#pragma unroll
    for (int j = 0; j < UB; ++j)
      v[j] = bload<AUXB>(r.rsrc, ci0 + (uint32_t)(GB * j) < cend ? base + (uint32_t)(16 * GB * j) : r.oob);
    const uint32_t e = L.edge[pk];
    uint32_t T = 0, W = 0;
#pragma unroll
    for (int j = 0; j < UB; ++j) sad_chunk(edge_mask(v[j], ci0 + (uint32_t)(GB * j), nc - 1u, e), T, W);
    const uint32_t sg = group_sum<GB>(s_of(T, W, e >> 31));
    if (li == 0) atomicAdd(&L.acc[pk], sg);
  }

  // Small packets (and split packets' edge lines): one lane per run of US
  // consecutive chunks.
  const uint32_t RSt = L.rs[P];
  for (uint32_t q = (uint32_t)t; q < RSt; q += WG) {
    const int pk = search(L.rs, q);
    const uint32_t nc = L.nch[pk];
    uint32_t ci0 = (q - L.rs[pk]) * US, cend = nc;
    if constexpr (LA) {  // split big packet: head runs cover [0, h), tail runs [ts, nc)
      const uint32_t hts = L.hts[pk];
      if (hts & 1u) {
        const uint32_t hh = (hts >> 1) & 7u, nh = (hh + US - 1) / US;
        const uint32_t k = q - L.rs[pk];
        if (k < nh) cend = hh;
        else ci0 = (hts >> 4) + (k - nh) * US;
      }
    }
    const uint32_t base = L.first[pk] + ci0 * 16u;
    uint4 v[US];
#pragma unroll
    for (int j = 0; j < US; ++j) v[j] = bload(r.rsrc, ci0 + (uint32_t)j < cend ? base + 16u * j : r.oob);
    const uint32_t e = L.edge[pk];
    uint32_t T = 0, W = 0;
#pragma unroll
    for (int j = 0; j < US; ++j) sad_chunk(edge_mask(v[j], ci0 + (uint32_t)j, nc - 1u, e), T, W);
    atomicAdd(&L.acc[pk], s_of(T, W, e >> 31));
  }
  __syncthreads();

  if (mine) put_result(p, L.acc[t], i, out, partial);
}

template <int WG, int GB, int UB, int US, int AUXB, int UD = 0, bool PERSIST = false, bool LA = false>
__global__ __launch_bounds__(WG) void csum_hyb(
    const uint8_t* __restrict__ arena, uint64_t arena_bytes,
    const uint4* __restrict__ desc, uint32_t n, uint16_t* __restrict__ out,
    uint32_t* __restrict__ partial, unsigned long long* __restrict__ err, uint32_t big_chunks) {
  constexpr int P = WG;
  static_assert((P & (P - 1)) == 0, "tile must be a power of two");
  __shared__ HybLds<P, LA> L;
  const int t = threadIdx.x;
  const Srd r = make_srd(arena, arena_bytes);

  uint64_t tile_lo, tile_end;
  if constexpr (PERSIST) {
    tile_lo = (uint64_t)n * blockIdx.x / gridDim.x;
    tile_end = (uint64_t)n * (blockIdx.x + 1) / gridDim.x;
  } else {
    tile_lo = (uint64_t)blockIdx.x * P;
    tile_end = min<uint64_t>(tile_lo + P, n);
  }
  uint4 raw = make_uint4(0, 0, 0, 0);
  if (tile_lo + t < tile_end) raw = desc[tile_lo + t];
  if (tile_lo >= tile_end) return;
  do {
    const uint64_t i = tile_lo + t;
    const bool mine = i < min<uint64_t>(tile_end, tile_lo + P);
    const PktInfo p = pkt_info(raw, mine, r.abase, arena_bytes, err);
    if constexpr (PERSIST) {  // prefetch the next sub-tile's descriptor
      const uint64_t nx = tile_lo + P + t;
      raw = nx < tile_end ? desc[nx] : make_uint4(0, 0, 0, 0);
    }
    bool done = false;
    if constexpr (UD > 0) {
      if (__syncthreads_and(p.nch <= (uint32_t)UD)) {
        uint4 v[UD];
        direct_load<UD>(r, p, v);
        const uint32_t sacc = direct_sum<UD>(p, v);
        if (mine) put_result(p, sacc, i, out, partial);
        done = true;
      }
    }
    if (!done) hyb_scan_tile<WG, GB, UB, US, AUXB, LA>(L, r, p, mine, i, out, partial, big_chunks);
    tile_lo += P;
  } while (PERSIST && tile_lo < tile_end);
}

// Sequential chain fix-up for NS_DESC_CONT runs (checksum.go:89 / the
// `xsum = Checksum(v, xsum)` loops): out[k] = fold1(out[k-1] + S_k).
__global__ void csum_chain(const uint4* __restrict__ desc, uint32_t n,
                           const uint32_t* __restrict__ partial,
                           uint16_t* __restrict__ out) {
  const uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n) return;
  const uint32_t w = desc[i].w;
  const bool cont = (w >> 16) & 2u;
  if (cont && i > 0) return;  // not a run head
  uint32_t s = fold1((cont ? 0u : (w & 0xFFFFu)) + partial[i]);
  out[i] = (uint16_t)s;
  for (uint64_t k = i + 1; k < n; ++k) {
    if (!((desc[k].w >> 16) & 2u)) break;
    s = fold1(s + partial[k]);
    out[k] = (uint16_t)s;
  }
}

}  // namespace nsk

// ---- launchers (C++ linkage, used by csum_api.cpp) ------------------------
namespace nsk {

// Resident workgroup slots of a kernel on the current device (cached per
// device and kernel; hipOccupancy... is a host-side query, no launch).
static uint32_t resident_slots(const void* kernel, int slot_id) {
  static std::mutex mu;
  static std::map<std::pair<int, int>, uint32_t> cache;
  int dev = 0;
  if (hipGetDevice(&dev) != hipSuccess) return 0;
  std::lock_guard<std::mutex> lk(mu);
  auto it = cache.find({dev, slot_id});
  if (it != cache.end()) return it->second;
  int per_cu = 0, cus = 0;
  if (hipOccupancyMaxActiveBlocksPerMultiprocessor(&per_cu, kernel, 256, 0) != hipSuccess) per_cu = 0;
  if (hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev) != hipSuccess) cus = 0;
  const uint32_t slots = (uint32_t)(per_cu > 0 && cus > 0 ? per_cu * cus : 0);
  cache[{dev, slot_id}] = slots;
  return slots;
}

template <int U, bool PIPE, bool PERSIST>
static hipError_t launch_runs(const uint8_t* arena, uint64_t arena_bytes, const void* desc,
                              uint32_t n, uint16_t* out, uint32_t* partial,
                              unsigned long long* err, hipStream_t stream) {
  constexpr int WG = 256;
  const auto kfn = csum_runs<WG, U, PIPE, PERSIST>;
  uint32_t grid = (uint32_t)(((uint64_t)n + WG - 1) / WG);
  if (PERSIST) {
    const uint32_t slots = resident_slots((const void*)kfn, U * 4 + (PIPE ? 1 : 0));
    if (slots) grid = std::min(grid, slots);
  }
  hipLaunchKernelGGL(kfn, dim3(grid), dim3(WG), 0, stream, arena, arena_bytes,
                     reinterpret_cast<const uint4*>(desc), n, out, partial, err);
  return hipGetLastError();
}

template <int G, int U, bool PIPE, int AUX = 0>
static hipError_t launch_grp(const uint8_t* arena, uint64_t arena_bytes, const void* desc,
                             uint32_t n, uint16_t* out, uint32_t* partial,
                             unsigned long long* err, hipStream_t stream) {
  constexpr int WG = 256;
  const uint32_t grid = (uint32_t)(((uint64_t)n + WG - 1) / WG);
  hipLaunchKernelGGL((csum_grp<WG, G, U, PIPE, AUX>), dim3(grid), dim3(WG), 0, stream, arena, arena_bytes,
                     reinterpret_cast<const uint4*>(desc), n, out, partial, err);
  return hipGetLastError();
}

template <int GB, int UB, int US, int AUXB, int UD = 0, bool PERSIST = false, bool LA = false>
static hipError_t launch_hyb(const uint8_t* arena, uint64_t arena_bytes, const void* desc,
                             uint32_t n, uint16_t* out, uint32_t* partial,
                             unsigned long long* err, hipStream_t stream, uint32_t big_chunks) {
  constexpr int WG = 256;
  const auto kfn = csum_hyb<WG, GB, UB, US, AUXB, UD, PERSIST, LA>;
  uint32_t grid = (uint32_t)(((uint64_t)n + WG - 1) / WG);
  if (PERSIST) {
    const uint32_t slots = resident_slots((const void*)kfn, 1000 + GB * 100 + UB * 10 + US + UD * 7);
    if (slots) grid = std::min(grid, slots);
  }
  hipLaunchKernelGGL(kfn, dim3(grid), dim3(WG), 0, stream, arena, arena_bytes,
                     reinterpret_cast<const uint4*>(desc), n, out, partial, err, big_chunks);
  return hipGetLastError();
}

static hipError_t launch_general(const uint8_t* arena, uint64_t arena_bytes, const void* desc,
                                 uint32_t n, uint16_t* out, uint32_t* partial,
                                 unsigned long long* err, hipStream_t stream) {
  constexpr int WG = 256;
  const uint32_t tiles = (uint32_t)(((uint64_t)n + WG - 1) / WG);
  hipLaunchKernelGGL((csum_batch<WG, 1, 2, 4, false>), dim3(tiles), dim3(WG), 0, stream, arena,
                     arena_bytes, reinterpret_cast<const uint4*>(desc), n, out, partial, err);
  return hipGetLastError();
}

hipError_t launch_batch(const uint8_t* arena, uint64_t arena_bytes,
                        const void* desc, uint32_t n, uint16_t* out,
                        uint32_t* partial, unsigned long long* err,
                        hipStream_t stream) {
  if (n == 0) return hipSuccess;
  hipError_t e;
  if (arena_bytes + 64 >= kMaxSrdBytes) {
    // Arenas of 4 GiB and more: 64-bit addressing, global loads.
    e = launch_general(arena, arena_bytes, desc, n, out, partial, err, stream);
  } else if (arena_bytes / n >= 256) {
    // Packets of >= 64 chunks (~1 KiB): their whole 128-B lines to 8-lane
    // groups (one full line per group per load instruction, 16 loads per lane
    // in flight) with nontemporal loads; their partial edge lines and all
    // smaller packets to per-lane runs of 4 (tools/tune.py on MI355X: 227 us
    // on 1M x 1500 B = 87.6% of 8 TB/s, 110 us on the Zipf batch;
    // profiles/r01/tune_*.json).
    e = launch_hyb<8, 16, 4, 2, 0, false, true>(arena, arena_bytes, desc, n, out, partial, err, stream, 64u);
  } else {
    // Small packets: the same kernel plus the direct path — a tile whose
    // packets all span <= 5 chunks (any <= 65-B packet) has each lane read its
    // own packet with no scan (16.9 us on 1M x 64 B vs 17.7 for the best
    // run-based variant).
    e = launch_hyb<16, 8, 4, 2, 5, false, true>(arena, arena_bytes, desc, n, out, partial, err, stream, 64u);
  }
  if (e != hipSuccess || partial == nullptr) return e;
  const uint32_t blocks = (n + 255) / 256;
  hipLaunchKernelGGL(csum_chain, dim3(blocks), dim3(256), 0, stream,
                     reinterpret_cast<const uint4*>(desc), n, partial, out);
  return hipGetLastError();
}

}  // namespace nsk
