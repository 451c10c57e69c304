// csum_kernels.hip — gfx950 (MI355X / CDNA4) kernels for netstack's RFC 1071
// checksum hot path (tcpip/header/checksum.go:26-46 applied per packet).
//
// Arithmetic.  calculateChecksum (checksum.go:26-46) adds big-endian 16-bit
// words into a uint32 that wraps mod 2^32 and folds once at the end
// (ChecksumCombine, :104-107).  Every byte therefore contributes
// byte*256 (high byte of a word) or byte*1 (low byte), decided by the parity
// of its position in the piece, shifted by one when `odd` is set (:29-32).
// In absolute device addresses: with phase = (addr(first byte) + odd) & 1,
// the byte at address A is a high byte iff (A & 1) == phase.  With E/O the
// sums of the bytes at even/odd addresses, the kernel accumulates
//     T = E + O        (v_sad_u8(w, 0) per dword)
//     W = E + 256*O    (v_sad_u16(w, 0): the little-endian word sum)
// and Go's accumulator is
//     S = 256*E + O = 257*T - W   (phase 0)    S = E + 256*O = W   (phase 1)
// all mod 2^32.  uint32 addition is associative and commutative, so any split
// of a packet across lanes, groups and waves is bit-exact, including the
// > 128 KiB wrap quirk.
//
// Layout.  Packets are byte ranges of one arena in HBM, described by a table
// of 16-byte ns_pkt_desc {u64 off, u32 len, u16 initial, u16 flags}.  The
// kernel reads only whole, naturally aligned 16-byte chunks: a packet covers
// chunks [A >> 4, (A + len - 1) >> 4] and its first/last chunk is byte-masked.
// An aligned chunk never crosses a page and holds at least one byte of the
// packet, so no read can fault.  No MFMA: this is a byte sum, HBM-bound
// (DESIGN.md §4).
//
// Kernels.  csum_hyb: tiles of TP descriptors per workgroup, the hot path
// (DESIGN.md §4.1-4.3).  fold_scan: NS_DESC_CONT runs of a chained batch,
// a one-pass segmented scan (§4.4).  csum_split: batches of a few huge
// descriptors, each cut into pieces over many workgroups (§4.6).  Stores of
// NS_DESC_STORE results into the packets happen in csum_hyb (unchained),
// fold_scan (chained) or csum_split (§4.5).
#include <hip/hip_runtime.h>
#include <stdint.h>

#include <algorithm>
#include <atomic>
#include <type_traits>

#include "csum_kernels.h"

namespace nsk {

// Per-workgroup finish stamps, in the tuning library only (tune.hip defines
// NSK_TIMELINE before including this file; tools/timeline.py): the low word
// of s_memrealtime (100 MHz) when a workgroup's thread 0 ends, stored when a
// buffer is set.  The product library compiles them out.  Nothing more: a
// start stamp, or the counter's high word, or the XCD id, each made the
// compiler hold uniform values in VGPRs (72 -> 86 VGPRs, 7 -> 5 waves per
// SIMD), which would time a different kernel.
#ifdef NSK_TIMELINE
__device__ uint32_t* nsk_timeline = nullptr;
#define NSK_TL_BEGIN
#define NSK_TL_END                                                                                      \
  {                                                                                                     \
    uint32_t* nsk_p = *(uint32_t* volatile*)&nsk_timeline;                                              \
    if (nsk_p != nullptr && threadIdx.x == 0) nsk_p[blockIdx.x] = (uint32_t)__builtin_amdgcn_s_memrealtime(); \
  }
#else
#define NSK_TL_BEGIN
#define NSK_TL_END
#endif

// ChecksumCombine(uint16(v), uint16(v>>16)) — checksum.go:45, :104-107.
__device__ __forceinline__ uint32_t fold1(uint32_t v) {
  const uint32_t s = (v & 0xFFFFu) + (v >> 16);
  return (s + (s >> 16)) & 0xFFFFu;
}

// Buffer resources cover < 4 GiB: a tile whose packets span more takes the
// 64-bit-addressed path.
constexpr uint64_t kMaxSrdBytes = 0xFFFF0000ull;

// buffer_load_dwordx4 through an SRD.  AUX = cache-policy bits (2 = nt).  An
// offset at or past num_records returns zeros without touching memory; an
// offset near 2^32 is NOT safe (offset + 16 wraps and passes the check), so
// out-of-range slots use num_records itself.
template <int AUX = 0>
__device__ __forceinline__ uint4 bload(__amdgpu_buffer_rsrc_t r, uint32_t off) {
  auto x = __builtin_amdgcn_raw_buffer_load_b128(r, (int)off, 0, AUX);
  return *reinterpret_cast<uint4*>(&x);
}

// global_load_dwordx4 from a 64-bit address (the > 4 GiB-span fallback).
typedef __attribute__((address_space(1))) const uint32_t gu32;
template <bool NT>
__device__ __forceinline__ uint4 gload(uint64_t addr) {
  gu32* p = (gu32*)addr;
  uint4 v;
  if constexpr (NT) {
    v.x = __builtin_nontemporal_load(p);
    v.y = __builtin_nontemporal_load(p + 1);
    v.z = __builtin_nontemporal_load(p + 2);
    v.w = __builtin_nontemporal_load(p + 3);
  } else {
    v.x = p[0];
    v.y = p[1];
    v.z = p[2];
    v.w = p[3];
  }
  return v;
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

// Lane jj of each quad, broadcast to the quad (DPP quad_perm; jj folds to a
// constant once the caller's loop is unrolled).
__device__ __forceinline__ uint32_t quad_bcast(uint32_t x, int jj) {
  switch (jj & 3) {
    case 0: return (uint32_t)__builtin_amdgcn_mov_dpp((int)x, 0x00, 0xF, 0xF, false);
    case 1: return (uint32_t)__builtin_amdgcn_mov_dpp((int)x, 0x55, 0xF, 0xF, false);
    case 2: return (uint32_t)__builtin_amdgcn_mov_dpp((int)x, 0xAA, 0xF, 0xF, false);
    default: return (uint32_t)__builtin_amdgcn_mov_dpp((int)x, 0xFF, 0xF, 0xF, false);
  }
}

// Sum over an aligned group of G lanes (DPP; every lane gets the total).
template <int G>
__device__ __forceinline__ uint32_t group_sum(uint32_t s) {
  static_assert(G == 1 || G == 2 || G == 4 || G == 8 || G == 16, "group of 1..16 lanes");
  if constexpr (G >= 2) s += (uint32_t)__builtin_amdgcn_update_dpp(0, (int)s, 0xB1, 0xF, 0xF, false);   // quad_perm 1,0,3,2
  if constexpr (G >= 4) s += (uint32_t)__builtin_amdgcn_update_dpp(0, (int)s, 0x4E, 0xF, 0xF, false);   // quad_perm 2,3,0,1
  if constexpr (G >= 8) s += (uint32_t)__builtin_amdgcn_update_dpp(0, (int)s, 0x141, 0xF, 0xF, false);  // row_half_mirror
  if constexpr (G >= 16) s += (uint32_t)__builtin_amdgcn_update_dpp(0, (int)s, 0x140, 0xF, 0xF, false); // row_mirror
  return s;
}

// ===========================================================================
// csum_hyb — the checksum kernel.  One 256-thread workgroup owns a tile of
// TP <= 256 descriptors (about 64 KiB of payload, launch_hyb); packets of at
// most 8190 chunks accumulate only the little-endian word sum W (see
// kWOnlyMaxChunks), longer ones the exact (T, W) pair.
//
// Two lane shapes, chosen per packet.  Nontemporal loads stream at ~6.8 TB/s
// on MI355X when every 128-B line is consumed by ONE wave instruction, and
// lose badly when a line is split across instructions (the evicted line is
// fetched again).  So a packet of at least `big_chunks` chunks is split at
// 128-B line boundaries: its whole lines go to groups of GB lanes (runs
// of GB*UB chunks, lane li loads chunks li, li+GB, ...: one whole line per
// group per load for GB = 8), and the partial lines it shares with its
// neighbours — plus every smaller packet — go to single lanes (runs of US
// consecutive chunks, default policy, so a shared line stays in L2 for the
// neighbour's lane).  One prologue scans both run counts (packed in a u64);
// two loops follow, each ending in one ds_add_u32 per run.
//
// Window.  The tile's SRD covers only the tile's own byte span (from its
// lowest first chunk to its highest packet end), so any arena size works;
// a tile spanning 4 GiB or more (a scattered table over a huge arena) takes
// the same scan path with 64-bit global loads.
//
// UD > 0 adds a direct path for tiles of small packets: when every packet of
// the tile spans at most UD chunks, each lane loads its own packet right
// after its descriptor — no scan, no search, no LDS atomics.
// ===========================================================================

// One validated descriptor.
struct Pkt {
  uint64_t A;  // absolute address of the first byte
  uint32_t len, init, odd, cont;
};

__device__ __forceinline__ Pkt decode(uint4 raw, bool mine, uint64_t arena_abs,
                                      uint64_t arena_bytes, unsigned long long* err) {
  Pkt d{0ull, 0u, 0u, 0u, 0u};
  if (!mine) return d;
  const uint64_t off = (uint64_t)raw.x | ((uint64_t)raw.y << 32);
  uint32_t len = raw.z;
  d.init = raw.w & 0xFFFFu;
  d.odd = (raw.w >> 16) & 1u;
  d.cont = (raw.w >> 17) & 1u;
  if (off > arena_bytes || (uint64_t)len > arena_bytes - off) {
    len = 0;
    atomicAdd(err, 1ull);
  }
  d.A = arena_abs + off;
  d.len = len;
  return d;
}

__device__ __forceinline__ uint32_t chunks_of(const Pkt& d) {
  return d.len ? (uint32_t)(((d.A + d.len - 1) >> 4) - (d.A >> 4) + 1) : 0u;
}

// A packet as the loops see it: chunks [0, nch) starting at absolute address
// g (16-B aligned), first = g - window base (SRD offset), line slot of chunk 0
// (lp), edge word (lo | hiex << 5 | phase << 31).
struct PktInfo {
  uint64_t g;
  uint32_t init, nch, first, ew, lp;
};

__device__ __forceinline__ PktInfo pkt_info(const Pkt& d, uint64_t wbase) {
  PktInfo p{0ull, d.init, 0u, 0u, 0u, 0u};
  if (d.len) {
    const uint64_t last = d.A + d.len - 1;
    p.nch = chunks_of(d);
    p.g = d.A & ~15ull;
    p.first = (uint32_t)(p.g - wbase);
    p.lp = (uint32_t)(d.A >> 4) & 7u;
    p.ew = (uint32_t)(d.A & 15u) | ((uint32_t)((last & 15u) + 1u) << 5) |
           ((uint32_t)((d.A + d.odd) & 1u) << 31);
  }
  return p;
}

// W-only accumulation.  The result fold1(initial + S) depends on S only
// through S mod 65535 and whether initial + S == 0, as long as Go's uint32
// accumulator does not wrap (initial + S < 2^32, i.e. packets of at most
// 8190 chunks = 131,040 bytes).  Since 2^16 == 1 (mod 65535), the big-endian
// word sum is S == 256*W (phase 0) or W (phase 1) (mod 65535), and S == 0 iff
// every byte is 0 iff W == 0.  So those packets need only W — one v_sad_u16
// per dword — and s_class() turns a packet's W total into a value with the
// same fold1 behaviour as S (also as a chain partial: a chained run adds it to
// a u16).  Tiles holding a longer packet accumulate the exact S (EX = true).
constexpr uint32_t kWOnlyMaxChunks = 8190;

__device__ __forceinline__ uint32_t s_class(uint32_t W, uint32_t phase) {
  const uint32_t w = fold1(W);
  return phase ? w : fold1(w << 8);
}

template <bool EX>
__device__ __forceinline__ void acc_chunk(const uint4 w, uint32_t& T, uint32_t& W) {
  if constexpr (EX) {
    sad_chunk(w, T, W);
  } else {
    W = __builtin_amdgcn_sad_u16(w.x, 0u, W);
    W = __builtin_amdgcn_sad_u16(w.y, 0u, W);
    W = __builtin_amdgcn_sad_u16(w.z, 0u, W);
    W = __builtin_amdgcn_sad_u16(w.w, 0u, W);
  }
}

template <bool EX>
__device__ __forceinline__ uint32_t run_value(uint32_t T, uint32_t W, uint32_t phase) {
  if constexpr (EX) return s_of(T, W, phase);
  else return W;
}

// The bytes of a run that lie outside its packet: [0, lo) of the packet's
// first chunk and [hiex, 16) of its last (edge word e).  A run sums its chunks
// unmasked and subtracts these (S is linear in T and W for a fixed phase):
// one masked chunk per partial edge, in a branch taken only by lanes whose run
// holds such an edge — a 16-B-aligned packet start never has one, so no run
// masks its chunks one by one.
__device__ __forceinline__ uint32_t bytes_below(int c) {  // bytes [0, c) of a dword, c clamped to [0, 4]
  c = min(max(c, 0), 4);
  return c >= 4 ? 0xFFFFFFFFu : ((1u << (8 * c)) - 1u);
}

template <bool EX, int U>
__device__ __forceinline__ void sub_edges(const uint4 (&v)[U], uint32_t ci0, uint32_t lastc, uint32_t e,
                                          uint32_t& T, uint32_t& W) {
  const int lo = (int)(e & 31u), hx = (int)((e >> 5) & 31u);
  uint32_t Tx = 0, Wx = 0;
  if (ci0 == 0u && lo != 0) {
    const uint4 w = v[0];
    acc_chunk<EX>(make_uint4(w.x & bytes_below(lo), w.y & bytes_below(lo - 4), w.z & bytes_below(lo - 8),
                             w.w & bytes_below(lo - 12)),
                  Tx, Wx);
  }
  const uint32_t jl = lastc - ci0;
  if (jl < (uint32_t)U && hx != 16) {
    // The last chunk, picked with AND/OR masks (an if-chain on jl becomes a
    // switch that LLVM lowers to a scratch-memory lookup of v[jl]).
    uint4 w = make_uint4(0, 0, 0, 0);
#pragma unroll
    for (int j = 0; j < U; ++j) {
      const uint32_t m = 0u - (uint32_t)(jl == (uint32_t)j);
      w.x |= v[j].x & m;
      w.y |= v[j].y & m;
      w.z |= v[j].z & m;
      w.w |= v[j].w & m;
    }
    acc_chunk<EX>(make_uint4(w.x & ~bytes_below(hx), w.y & ~bytes_below(hx - 4), w.z & ~bytes_below(hx - 8),
                             w.w & ~bytes_below(hx - 12)),
                  Tx, Wx);
  }
  T -= Tx;
  W -= Wx;
}

// Edge word bits: lo (0-4) | hiex (5-9) | h (10-13) | split (14) | phase (31).
constexpr uint32_t kSplitBit = 1u << 14;

template <int P>
struct HybLds {
  uint4 info[P];        // {SRD offset of chunk 0, nch, edge word, ts}
  uint64_t g[P];        // absolute address of chunk 0 (64-bit path)
  uint64_t wtot[P / 64];
  uint64_t wmin[P / 64], wmax[P / 64];
  uint32_t rb[P + 1];   // first big run of each packet
  uint32_t rs[P + 1];   // first small run of each packet
  uint32_t acc[P];
  uint32_t wsmall[P / 64];
  uint32_t wex[P / 64];
  uint32_t wsch[P / 64];  // QS & 8: each wave's small-run chunks
  // NS_DESC_STORE launches only: each lane's validated store word and
  // address (written at decode, read back by the same lane after the scan).
  uint64_t sat[P];
  uint32_t stw[P];
};

struct Srd {
  __amdgpu_buffer_rsrc_t rsrc;
  uint32_t oob;  // an offset the range check rejects: the SRD's own size
};

__device__ __forceinline__ Srd make_srd(uint64_t base, uint64_t span) {
  Srd r;
  const uint32_t nrec = (uint32_t)((span + 15) & ~15ull);
  // readfirstlane returns int: widen through uint32_t (a sign-extended low
  // word would corrupt the base's high bits).
  const uint32_t lo = (uint32_t)__builtin_amdgcn_readfirstlane((uint32_t)base);
  const uint32_t hi = (uint32_t)__builtin_amdgcn_readfirstlane((uint32_t)(base >> 32));
  r.rsrc = __builtin_amdgcn_make_buffer_rsrc((void*)(((uint64_t)hi << 32) | (uint64_t)lo), (short)0,
                                             (int)__builtin_amdgcn_readfirstlane(nrec), 0x00020000);
  r.oob = (uint32_t)__builtin_amdgcn_readfirstlane(nrec);
  return r;
}

extern "C" __device__ unsigned long __ockl_wfred_min_u64(unsigned long);
extern "C" __device__ unsigned long __ockl_wfred_max_u64(unsigned long);

// Block-wide: lowest packet start, highest packet end, and whether every
// packet spans at most `ud` chunks.
struct Win {
  uint64_t base, span;
  bool small;
};

template <int WG>
__device__ __forceinline__ Win tile_window(HybLds<WG>& L, const Pkt& d, uint32_t nch, uint32_t ud) {
  constexpr int NW = WG / 64;
  const int lane = threadIdx.x & 63, wv = threadIdx.x >> 6;
  // DPP wave reductions (device library), no LDS round trips.
  uint64_t mn = __ockl_wfred_min_u64(d.len ? d.A : ~0ull);
  uint64_t mx = __ockl_wfred_max_u64(d.len ? d.A + d.len : 0ull);
  const int sm = __all(nch <= ud);
  if (lane == 0) {
    L.wmin[wv] = mn;
    L.wmax[wv] = mx;
    L.wsmall[wv] = (uint32_t)sm;
  }
  __syncthreads();
  Win w{0ull, 0ull, true};
  mn = ~0ull;
  mx = 0ull;
#pragma unroll
  for (int k = 0; k < NW; ++k) {
    mn = min(mn, L.wmin[k]);
    mx = max(mx, L.wmax[k]);
    w.small = w.small && L.wsmall[k];
  }
  if (mx != 0ull) {  // at least one non-empty packet
    w.base = mn & ~15ull;
    w.span = mx - w.base;
  }
  return w;
}

// The direct path: one lane, one packet of at most UD chunks.
template <int UD>
__device__ __forceinline__ uint32_t direct_sum(const Srd& r, const PktInfo& p) {
  uint4 v[UD];
#pragma unroll
  for (int j = 0; j < UD; ++j) {
    // Chunks past the 4th only when some lane of the wave has them (a 64-B
    // packet at a 16-B-aligned start spans exactly 4): an out-of-range load
    // touches no memory but still costs issue and address slots.
    v[j] = make_uint4(0, 0, 0, 0);
    if (j < 4 || __any((uint32_t)j < p.nch)) v[j] = bload(r.rsrc, (uint32_t)j < p.nch ? p.first + 16u * j : r.oob);
  }
  uint32_t T = 0, W = 0;
#pragma unroll
  for (int j = 0; j < UD; ++j) acc_chunk<false>(v[j], T, W);
  sub_edges<false>(v, 0u, p.nch - 1u, p.ew, T, W);
  return s_class(W, p.ew >> 31);
}

// The quad-lane direct path: a wave whose 64 packets all span <= 4 chunks
// (any alignment and length; every 16-B-aligned packet of <= 64 B).  Load
// instruction j of the wave reads packets 16 j .. 16 j + 15 — lane l takes
// chunk l % 4 of packet 16 j + l / 4, so dense packets give whole 128-B
// lines per instruction and the loads are nontemporal (cdna: a line split
// across instructions must stay cached).  Each packet's
// geometry reaches its quad by __shfl, a lane masks only its own chunk's edge
// bytes, a quad DPP sum gives the packet's W, and the W totals shuffle back to
// one per lane.  1M x 64 B: 14.7 vs 16.3 us for the lane-per-packet path
// (tools/tune.py, profiles/r02/tune_cfg3_quad.log).
//
// This path is VALU-bound, not memory-bound, at 1M x 64 B: with 8 one-wave
// tiles per SIMD each issuing ~420 VALU instructions, every wave was issuing
// VALU for 14.8% of its life (SQ_ACTIVE_INST_VALU / SQ_WAVE_CYCLES,
// profiles/r03/sq_summary.json): 8 waves x 14.8% fills the SIMD; the floor
// kernel issues 72 per wave.  So a chunk is masked only when it needs it —
// the packet's first chunk with a partial start, its last with a partial
// end, a chunk past its last (the "need" bits, computed once by the packet's
// own lane) — in a branch the lanes of whole aligned chunks skip, and the
// W-only class value (s_class) is taken once per packet by its own lane after
// one shuffle back, not by all four lanes of its quad before four.
__device__ __forceinline__ uint32_t quad_geo(const PktInfo& p) {
  // nch (3 bits) | lo (4) | hiex (5) | phase (1) | need (4: bit c = chunk c is masked)
  const uint32_t nc = p.nch, lo = p.ew & 15u, hx = (p.ew >> 5) & 31u;
  uint32_t need = 0xFu & ~((1u << min(nc, 4u)) - 1u);  // past the last chunk
  if (lo != 0u) need |= 1u;
  if (nc != 0u && hx != 16u) need |= 1u << ((nc - 1u) & 3u);
  return nc | (lo << 3) | (hx << 7) | ((p.ew >> 31) << 12) | (need << 13);
}

// The quad layout's sums: v[j] holds chunk l % 4 of packet 16 j + l / 4 and
// g[j] that packet's geometry; a chunk past the packet's last is masked out
// (it reads zeros in quad_sum, the next packet's bytes in a speculative load).
// `phase` is the lane's own packet's byte phase (pkt_info's edge word).
__device__ __forceinline__ uint32_t quad_reduce(const uint4 (&v)[4], const uint32_t (&g)[4], uint32_t phase) {
  const uint32_t l = threadIdx.x & 63u, c = l & 3u;
  uint32_t sv[4];
#pragma unroll
  for (int j = 0; j < 4; ++j) {
    const uint32_t gj = g[j];
    uint4 w = v[j];
    if ((gj >> (13u + c)) & 1u) {  // an edge chunk, or one past the packet
      const uint32_t nc = gj & 7u;
      const int lo_b = c == 0 ? (int)((gj >> 3) & 15u) : 0;
      const int hi_b = c + 1 == nc ? (int)((gj >> 7) & 31u) : (c < nc ? 16 : 0);
      w.x &= bytes_below(hi_b) & ~bytes_below(lo_b);
      w.y &= bytes_below(hi_b - 4) & ~bytes_below(lo_b - 4);
      w.z &= bytes_below(hi_b - 8) & ~bytes_below(lo_b - 8);
      w.w &= bytes_below(hi_b - 12) & ~bytes_below(lo_b - 12);
    }
    uint32_t T = 0, W = 0;
    acc_chunk<false>(w, T, W);
    sv[j] = group_sum<4>(W);  // the packet's W, in all four lanes of its quad
  }
  // lane 4k + c keeps packet 16 c + k's total; lane l reads its own packet
  // (16 (l >> 4) + (l & 15)) from lane 4 (l & 15) + (l >> 4): one shuffle
  const uint32_t mine = c == 0u ? sv[0] : c == 1u ? sv[1] : c == 2u ? sv[2] : sv[3];
  const uint32_t W = (uint32_t)__shfl((int)mine, (int)(4u * (l & 15u) + (l >> 4)), 64);
  return s_class(W, phase);
}

__device__ __forceinline__ uint32_t quad_sum(const Srd& r, const PktInfo& p) {
  const uint32_t l = threadIdx.x & 63u, c = l & 3u;
  const uint32_t geo = quad_geo(p);
  uint4 v[4];
  uint32_t g[4];
#pragma unroll
  for (int j = 0; j < 4; ++j) {
    const int src = (int)(16 * j + (l >> 2));
    g[j] = (uint32_t)__shfl((int)geo, src, 64);
    const uint32_t f = (uint32_t)__shfl((int)p.first, src, 64);
    v[j] = bload<2>(r.rsrc, c < (g[j] & 7u) ? f + 16u * c : r.oob);
  }
  return quad_reduce(v, g, p.ew >> 31);
}

// Speculative quad loads (one-wave small-packet tiles; launch_batch sets
// `spec` only for a 16-B-aligned arena of exactly n * spec bytes, spec a
// multiple of 16 up to 64): packet k predicted at arena byte k * spec, its 4
// chunks loaded in quad_sum's layout together with the descriptors instead of
// after them.  spec_check: every packet of the wave is where predicted and
// spans <= 4 chunks (then the loaded chunks cover it), else the wave takes
// quad_sum / direct_sum as without speculation.
// (32-bit arithmetic: the arena is n * spec bytes under one SRD, < 4 GiB,
// and a tile's first packet index is below n.)
__device__ __forceinline__ void spec_load(const Srd& r, uint64_t tile0, uint32_t n, uint32_t spec, uint4 (&v)[4]) {
  const uint32_t l = threadIdx.x & 63u, c = l & 3u;
#pragma unroll
  for (int j = 0; j < 4; ++j) {
    const uint32_t k = (uint32_t)tile0 + 16u * j + (l >> 2);
    v[j] = bload<2>(r.rsrc, k < n ? k * spec + 16u * c : r.oob);
  }
}

__device__ __forceinline__ bool spec_check(const PktInfo& p, uint64_t i, uint32_t spec) {
  return __all(p.nch == 0u || (p.nch <= 4u && p.first == (uint32_t)i * spec)) != 0;
}

// quad_reduce for a wave in which no chunk needs a mask (every packet whole
// 16-B-aligned chunks, 4 of them: cfg3's dense 64-B slots): no geometry
// shuffles and no per-chunk mask tests (round 5: a first SQ pass put cfg3's
// distance to its floor kernels on VALU issue; a second did not confirm it,
// DESIGN.md §4.2b).
__device__ __forceinline__ uint32_t quad_reduce_whole(const uint4 (&v)[4], uint32_t phase) {
  const uint32_t l = threadIdx.x & 63u, c = l & 3u;
  uint32_t sv[4];
#pragma unroll
  for (int j = 0; j < 4; ++j) {
    uint32_t T = 0, W = 0;
    acc_chunk<false>(v[j], T, W);
    sv[j] = group_sum<4>(W);
  }
  const uint32_t mine = c == 0u ? sv[0] : c == 1u ? sv[1] : c == 2u ? sv[2] : sv[3];
  const uint32_t W = (uint32_t)__shfl((int)mine, (int)(4u * (l & 15u) + (l >> 4)), 64);
  return s_class(W, phase);
}

__device__ __forceinline__ uint32_t spec_sum(const PktInfo& p, const uint4 (&v)[4]) {
  const uint32_t l = threadIdx.x & 63u;
  const uint32_t geo = quad_geo(p);
  if (!__any(geo >> 13)) return quad_reduce_whole(v, p.ew >> 31);  // no packet's chunk needs a mask
  uint32_t g[4];
#pragma unroll
  for (int j = 0; j < 4; ++j) g[j] = (uint32_t)__shfl((int)geo, (int)(16 * j + (l >> 2)), 64);
  return quad_reduce(v, g, p.ew >> 31);
}

// One tile through the scan path (thread t holds packet p of global index i).
// GL = 64-bit global loads (tile span >= 4 GiB) instead of the window SRD.
// Every thread of the block must call it.
// Returns this thread's packet sum (finish_tile turns it into the result).
// FX = always the exact (T, W) accumulator (csum_split: its pieces' sums are
// added, so they must be exact mod 2^32, not W-only class values).
// QS = quad-lane small runs (US = 4, SRD path only; 1: nontemporal loads, 2:
// the default policy; | 4: two sets of 64 runs per iteration; | 8: only in
// tiles whose small runs fill >= 7/8 of their quads, the others take the
// lane runs; | 64, without the quad loop: lean load addressing; | 128: the
// run words exchanged within quads by DPP): a wave takes 64
// consecutive small runs per iteration, lane l looking up run l and quad q of
// load instruction j loading run 16 j + q, one chunk per lane; consecutive
// runs lie back to back in memory when packets are packed, so one
// instruction reads ~1 KiB contiguous and the loads are nontemporal.
// Staged small runs (QS & 256, SRD path): the 128-B lines the tile's small
// runs read are fetched whole, nontemporal, by LDS-DMA into a line buffer of
// SLN lines, and the lane runs sum from LDS.  Per packet, its small-run lines
// (every line of a small packet; the head and tail line of a split one) take
// consecutive slots, a line equal to the previous packet's last one sharing
// its slot, so a packet's chunk ci sits at LDS chunk lb + ci (lb: its first
// slot * 8 + line position; the tail of a split packet has its own base).
template <int N>
struct SlLds {
  uint4 line[N * 8];  // N staged 128-B lines
  uint32_t la[N];     // SRD offset of each staged line
  uint32_t nlt;       // lines the tile stages
};
template <>
struct SlLds<0> {
  uint32_t nlt;
};

template <int WG, int TP, int GB, int UB, int US, int AUXB, bool GL, int SU, bool FX = false, int QS = 0>
__device__ __forceinline__ uint32_t hyb_scan_tile(HybLds<WG>& L, const Srd& r, const PktInfo& p,
                                                  uint32_t big_chunks) {
  constexpr int P = WG;
  constexpr int NW = WG / 64;
  constexpr int NG = WG / GB;
  constexpr uint32_t RB = GB * UB;
  constexpr bool SL = (QS & 256) != 0 && !GL && !FX;
  constexpr int SAUX = (QS >> 10) & 31;  // tuning only: the lane runs' cache-policy bits (0 = default)
  constexpr uint32_t SLN = (QS & 512) ? 96u : 80u;
  __shared__ SlLds<SL ? (int)SLN : 0> S;
  const int t = threadIdx.x;
  const int lane = t & 63;
  const int wv = t >> 6;
  const uint32_t li = (uint32_t)(t % GB);
  const uint32_t nch = p.nch;

  // LA split of a big packet: lane runs over chunks [0, h) and [ts, nch), the
  // partial first and last 128-B lines; groups over the whole lines [h, ts).
  // The body holds only whole chunks of the packet, so the group loop needs
  // no byte masks: a partial first (last) chunk sends its whole line to the
  // lane runs — a line it shares with the neighbouring packet anyway.
  uint32_t h = nch, ts = nch;
  const bool split = nch >= big_chunks;
  if (split) {
    h = (8u - p.lp) & 7u;
    ts = ((p.lp + nch) & ~7u) - p.lp;
    if (h == 0u && (p.ew & 31u) != 0u) h = 8u;
    if (ts == nch && ((p.ew >> 5) & 31u) != 16u) ts -= 8u;
  }
  // At most 2^28 chunks per packet (len is a u32), so a tile's big-run total
  // stays below 2^32 with RB >= 16; small runs per packet are bounded by
  // big_chunks / US + 4.
  uint64_t nr = nch == 0 ? 0ull
                : split ? ((uint64_t)((ts - h + RB - 1) / RB) |
                           ((uint64_t)((h + US - 1) / US + (nch - ts + US - 1) / US) << 32))
                        : ((uint64_t)((nch + US - 1) / US) << 32);
  // SL: the packet's staged lines (nl, the first of them deduplicated against
  // the previous lane's last) ride in bits 48-63 of the scan; small runs stay
  // below 2^16 per tile (<= big_chunks / US + 4 per packet).
  [[maybe_unused]] uint32_t sl_nl = 0u, sl_dup = 0u, sl_span = 0u;
  if constexpr (SL) {
    uint32_t fl = 0u, ll = 0u;
    if (nch) {
      const uint32_t l0 = (uint32_t)(p.g >> 7), ln = (uint32_t)((p.g + 16ull * (nch - 1u)) >> 7);
      const bool hh = h > 0u, ht = ts < nch;
      sl_span = ln - l0;
      sl_nl = split ? (uint32_t)hh + (uint32_t)ht : sl_span + 1u;
      fl = (split && !hh) ? ln : l0;
      ll = (split && !ht) ? l0 : ln;
    }
    const uint32_t pnl = (uint32_t)__shfl_up((int)sl_nl, 1, 64);
    const uint32_t pll = (uint32_t)__shfl_up((int)ll, 1, 64);
    sl_dup = (lane > 0 && sl_nl && pnl && pll == fl) ? 1u : 0u;
    nr |= (uint64_t)(sl_nl - sl_dup) << 48;
  }
  uint64_t incl = nr;
#pragma unroll
  for (int d = 1; d < 64; d <<= 1) {
    const uint64_t y = __shfl_up(incl, d, 64);
    if (lane >= d) incl += y;
  }
  const int wex = FX || __any(nch > kWOnlyMaxChunks);
  uint32_t sch = 0u;  // QS & 8: chunks in small runs (the quads they fill)
  if constexpr ((QS & 8) != 0) {
    sch = split ? h + nch - ts : nch;
#pragma unroll
    for (int d = 1; d < 64; d <<= 1) sch += __shfl_xor(sch, d, 64);
  }
  if (lane == 63) {
    L.wtot[wv] = incl;
    L.wex[wv] = (uint32_t)wex;
    if constexpr ((QS & 8) != 0) L.wsch[wv] = sch;
  }
  __syncthreads();
  uint64_t excl = incl - nr;
  bool exact = false;
  uint32_t scht = 0u;
#pragma unroll
  for (int w = 0; w < NW; ++w) {
    if (w < wv) excl += L.wtot[w];
    exact = exact || L.wex[w];
    if constexpr ((QS & 8) != 0) scht += L.wsch[w];
  }
  constexpr uint32_t kRsMask = SL ? 0xFFFFu : 0xFFFFFFFFu;
  L.rb[t] = (uint32_t)excl;
  L.rs[t] = (uint32_t)(excl >> 32) & kRsMask;
  if constexpr (GL) L.g[t] = p.g;
  L.info[t] = make_uint4(p.first, nch, p.ew | (split ? (kSplitBit | (h << 10)) : 0u), ts);
  L.acc[t] = 0u;
  if (t == WG - 1) {
    L.rb[P] = (uint32_t)(excl + nr);
    L.rs[P] = (uint32_t)((excl + nr) >> 32) & kRsMask;
    if constexpr (SL) S.nlt = (uint32_t)((excl + nr) >> 48);
  }
  if constexpr (SL) {
    // this packet's line slots and the LDS chunk bases of its runs (in L.g,
    // which only the 64-bit path uses otherwise)
    const uint32_t hh = (split && h > 0u) ? 1u : 0u;
    const uint32_t base = (uint32_t)(excl >> 48) - sl_dup;
    const uint32_t lof = p.first - 16u * p.lp;  // SRD offset of the first line (may wrap below 0)
    for (uint32_t j = sl_dup; j < sl_nl; ++j) {
      const uint32_t rel = split ? ((j == 0u && hh) ? 0u : sl_span) : j;
      if (base + j < SLN) S.la[base + j] = lof + 128u * rel;
    }
    L.g[t] = (uint64_t)(base * 8u + p.lp) | ((uint64_t)((base + hh) * 8u - ts) << 32);
  }
  __syncthreads();

  auto search = [&](const uint32_t* s_r, uint32_t q) {
    // Largest pk < TP with s_r[pk] <= q: fixed-step, branch-free
    // (s_r[0] = 0 <= q; threads past TP hold no packet and no runs).
    int lo = 0;
#pragma unroll
    for (int step = TP / 2; step >= 1; step >>= 1)
      lo = (s_r[lo + step] <= q) ? lo + step : lo;
    return lo;
  };
  const uint32_t RBt = L.rb[P];
  const uint32_t RSt = L.rs[P];
  // SL: issue the staging loads before the big loop's, 8 lanes per line (one
  // wave instruction = 8 whole lines = 1 KiB of LDS, lane-linear); a tile
  // with more than SLN lines takes the lane runs from memory.
  [[maybe_unused]] bool staged = false;
  if constexpr (SL) {
    const uint32_t nlt = S.nlt;
    staged = nlt <= SLN;
    if (staged) {
      const uint32_t l8 = (uint32_t)t & 7u;
      for (uint32_t s0 = (uint32_t)wv * 8u; s0 < nlt; s0 += (uint32_t)WG / 8u) {
        const uint32_t s = s0 + ((uint32_t)lane >> 3);
        const uint32_t o = s < nlt ? S.la[s] + 16u * l8 : r.oob;
        __builtin_amdgcn_raw_ptr_buffer_load_lds(r.rsrc, (__attribute__((address_space(3))) void*)&S.line[s0 * 8u],
                                                 16, o < r.oob ? o : r.oob, 0, 0, 2);
      }
    }
  }

  // The loops, with the exact (T, W) or the W-only accumulator for the whole
  // tile.  Every load offset is a select (out-of-range slots read r.oob, which
  // the buffer range check turns into zeros), so the descriptor fields come
  // from one ds_read_b128 per run and no load sits behind a branch.
  auto loops = [&](auto ex_tag) {
    constexpr bool EX = decltype(ex_tag)::value;
    // Small packets (and split packets' edge lines): one lane per run of US
    // consecutive chunks.  A run is issued (search + loads) by small_issue and
    // consumed by small_sum, so its loads can be in flight while other work
    // runs: SU runs are issued per iteration of the small loop.
    struct SRun {
      int pk;
      uint32_t ci0, lastc, ew;
      bool act;
    };
    auto small_issue = [&](uint32_t q, uint4 (&v)[US]) -> SRun {
      SRun sr{0, 0u, 0u, 0u, q < RSt};
      uint32_t cend = 0u, base = 0u;
      uint64_t gb = 0ull;
      if (sr.act) {
        sr.pk = search(L.rs, q);
        const uint32_t k = q - L.rs[sr.pk];
        const uint4 inf = L.info[sr.pk];
        sr.ci0 = k * US;
        sr.lastc = inf.y - 1u;
        sr.ew = inf.z;
        cend = inf.y;
        if (inf.z & kSplitBit) {  // head runs cover [0, h), tail runs [ts, nch)
          const uint32_t hh = (inf.z >> 10) & 15u, nh = (hh + US - 1) / US;
          if (k < nh) cend = hh;
          else sr.ci0 = inf.w + (k - nh) * US;
        }
        if constexpr (GL) gb = L.g[sr.pk] + (uint64_t)sr.ci0 * 16u;
        else base = inf.x + sr.ci0 * 16u;
      }
      if constexpr ((QS & 64) != 0 && !GL) {
        // QS & 64: the valid slots counted once, each load's select on the
        // base alone (the chunk step folds into the instruction's offset)
        const uint32_t kv = sr.ci0 < cend ? min(cend - sr.ci0, (uint32_t)US) : 0u;
#pragma unroll
        for (int j = 0; j < US; ++j) v[j] = bload(r.rsrc, ((uint32_t)j < kv ? base : r.oob) + 16u * j);
      } else {
#pragma unroll
        for (int j = 0; j < US; ++j) {
          const bool valid = sr.ci0 + (uint32_t)j < cend;
          if constexpr (GL) v[j] = valid ? gload<false>(gb + 16u * j) : make_uint4(0, 0, 0, 0);
          else v[j] = bload<SAUX>(r.rsrc, valid ? base + 16u * j : r.oob);
        }
      }
      return sr;
    };
    auto small_sum = [&](const SRun& sr, const uint4 (&v)[US]) {
      if (!sr.act) return;
      uint32_t T = 0, W = 0;
#pragma unroll
      for (int j = 0; j < US; ++j) acc_chunk<EX>(v[j], T, W);
      sub_edges<EX>(v, sr.ci0, sr.lastc, sr.ew, T, W);
      atomicAdd(&L.acc[sr.pk], run_value<EX>(T, W, sr.ew >> 31));
    };

    // Big packets: groups of GB lanes, lane li takes chunks li + GB*j of a run.
    for (uint32_t q = (uint32_t)(t / GB); q < RBt; q += NG) {
      const int pk = search(L.rb, q);
      const uint4 inf = L.info[pk];
      // every big packet is split: the body [h, ts)
      const uint32_t ci0 = (q - L.rb[pk]) * RB + li + ((inf.z >> 10) & 15u), cend = inf.w;
      uint4 v[UB];
      if constexpr (GL) {
        const uint64_t g0 = L.g[pk] + (uint64_t)ci0 * 16u;
#pragma unroll
        for (int j = 0; j < UB; ++j)
          v[j] = ci0 + (uint32_t)(GB * j) < cend ? gload<AUXB != 0>(g0 + 16u * GB * j) : make_uint4(0, 0, 0, 0);
      } else {
        const uint32_t b0 = inf.x + ci0 * 16u;
        if constexpr ((QS & 64) != 0) {
          const uint32_t kv = ci0 < cend ? min((cend - ci0 + GB - 1u) / GB, (uint32_t)UB) : 0u;
#pragma unroll
          for (int j = 0; j < UB; ++j) v[j] = bload<AUXB>(r.rsrc, ((uint32_t)j < kv ? b0 : r.oob) + 16u * GB * j);
        } else {
#pragma unroll
          for (int j = 0; j < UB; ++j)
            v[j] = bload<AUXB>(r.rsrc, ci0 + (uint32_t)(GB * j) < cend ? b0 + 16u * GB * j : r.oob);
        }
      }
      uint32_t T = 0, W = 0;
#pragma unroll
      for (int j = 0; j < UB; ++j)
        acc_chunk<EX>(v[j], T, W);  // body chunks are whole chunks of the packet
      const uint32_t sg = group_sum<GB>(run_value<EX>(T, W, inf.z >> 31));
      if (li == 0) atomicAdd(&L.acc[pk], sg);
    }

    if constexpr ((QS & 3) != 0 && !GL) {
      static_assert(US == 4, "quad-lane small runs are runs of 4 chunks");
      if ((QS & 8) && scht * 8u < RSt * 28u) goto lane_runs;  // | 8: only when the quads are >= 7/8 full
      constexpr int QN = (QS & 4) ? 2 : 1;  // sets of 64 runs per wave per iteration
      constexpr int QP = (QS & 3) == 1 ? 2 : 0;  // load policy: nontemporal or default
      const uint32_t c = (uint32_t)lane & 3u;
      for (uint32_t qb = (uint32_t)wv * 64u * QN; qb < RSt; qb += (uint32_t)NW * 64u * QN) {
        // lane l describes run qb + 64 s + l: SRD offset of its first chunk
        // and a meta word nvalid (3 bits) | lo (4) | last chunk in run (1) |
        // its index (2) | hiex (5) | phase (1) | packet (8)
        uint32_t roff[QN], meta[QN];
#pragma unroll
        for (int s = 0; s < QN; ++s) {
          // | 128: lane 4 q + c describes run 16 c + q, so that quad q finds
          // instruction j's run in its own lane j (a DPP broadcast)
          const uint32_t q = qb + 64u * s +
                             ((QS & 128) ? 16u * ((uint32_t)lane & 3u) + ((uint32_t)lane >> 2) : (uint32_t)lane);
          roff[s] = r.oob;
          meta[s] = 0u;
          if (q < RSt) {
            const int pk = search(L.rs, q);
            const uint32_t k = q - L.rs[pk];
            const uint4 inf = L.info[pk];
            uint32_t ci0 = k * 4u, cend = inf.y;
            if (inf.z & kSplitBit) {  // head runs cover [0, h), tail runs [ts, nch)
              const uint32_t hh = (inf.z >> 10) & 15u, nh = (hh + 3u) / 4u;
              if (k < nh) cend = hh;
              else ci0 = inf.w + (k - nh) * 4u;
            }
            const uint32_t nv = min(cend - ci0, 4u);
            const uint32_t lo = ci0 == 0u ? (inf.z & 15u) : 0u;
            const uint32_t jl = inf.y - 1u - ci0;
            const uint32_t has_last = jl < nv ? 1u : 0u;
            meta[s] = nv | (lo << 3) | (has_last << 7) | ((jl & 3u) << 8) | (((inf.z >> 5) & 31u) << 10) |
                      ((inf.z >> 31) << 15) | ((uint32_t)pk << 16);
            roff[s] = inf.x + ci0 * 16u;
          }
        }
        uint4 v[4 * QN];
        uint32_t mj[4 * QN];
#pragma unroll
        for (int j = 0; j < 4 * QN; ++j) {
          uint32_t o;
          if constexpr ((QS & 128) != 0) {
            mj[j] = quad_bcast(meta[j >> 2], j & 3);
            o = quad_bcast(roff[j >> 2], j & 3);
          } else {
            const int src = (int)(16 * (j & 3) + (lane >> 2));
            mj[j] = (uint32_t)__shfl((int)meta[j >> 2], src, 64);
            o = (uint32_t)__shfl((int)roff[j >> 2], src, 64);
          }
          v[j] = bload<QP>(r.rsrc, c < (mj[j] & 7u) ? o + 16u * c : r.oob);
        }
#pragma unroll
        for (int j = 0; j < 4 * QN; ++j) {
          const uint32_t m = mj[j];
          const int lo_b = c == 0u ? (int)((m >> 3) & 15u) : 0;
          const int hi_b = ((m >> 7) & 1u) && c == ((m >> 8) & 3u) ? (int)((m >> 10) & 31u) : 16;
          uint4 w = v[j];
          if (lo_b != 0 || hi_b != 16) {  // an edge chunk (slots past the run read zeros)
            w.x &= bytes_below(hi_b) & ~bytes_below(lo_b);
            w.y &= bytes_below(hi_b - 4) & ~bytes_below(lo_b - 4);
            w.z &= bytes_below(hi_b - 8) & ~bytes_below(lo_b - 8);
            w.w &= bytes_below(hi_b - 12) & ~bytes_below(lo_b - 12);
          }
          uint32_t T = 0, W = 0;
          acc_chunk<EX>(w, T, W);
          const uint32_t val = group_sum<4>(run_value<EX>(T, W, (m >> 15) & 1u));
          if (c == 0u && (m & 7u)) atomicAdd(&L.acc[m >> 16], val);
        }
      }
      return;
    }
  lane_runs:
    static_assert(SU == 1 || SU == 2, "the small loop issues one or two runs per iteration");
    if constexpr (SL) {
      if (staged) {
        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");  // this wave's staging loads have landed
        __syncthreads();                                   // ... and every other wave's
        auto sl_issue = [&](uint32_t q, uint4 (&v)[US]) -> SRun {
          SRun sr{0, 0u, 0u, 0u, q < RSt};
          uint32_t cend = 0u, lb = 0u;
          if (sr.act) {
            sr.pk = search(L.rs, q);
            const uint32_t k = q - L.rs[sr.pk];
            const uint4 inf = L.info[sr.pk];
            const uint64_t lbs = L.g[sr.pk];
            sr.ci0 = k * US;
            sr.lastc = inf.y - 1u;
            sr.ew = inf.z;
            cend = inf.y;
            lb = (uint32_t)lbs;
            if (inf.z & kSplitBit) {
              const uint32_t hh = (inf.z >> 10) & 15u, nh = (hh + US - 1) / US;
              if (k < nh) {
                cend = hh;
              } else {
                sr.ci0 = inf.w + (k - nh) * US;
                lb = (uint32_t)(lbs >> 32);
              }
            }
          }
#pragma unroll
          for (int j = 0; j < US; ++j)
            v[j] = sr.ci0 + (uint32_t)j < cend ? S.line[lb + sr.ci0 + (uint32_t)j] : make_uint4(0, 0, 0, 0);
          return sr;
        };
        for (uint32_t q = (uint32_t)t; q < RSt; q += SU * WG) {
          uint4 va[US];
          const SRun ra = sl_issue(q, va);
          if constexpr (SU == 2) {
            uint4 vb[US];
            const SRun rb = sl_issue(q + WG, vb);
            small_sum(ra, va);
            small_sum(rb, vb);
          } else {
            small_sum(ra, va);
          }
        }
        return;
      }
    }
    for (uint32_t q = (uint32_t)t; q < RSt; q += SU * WG) {
      uint4 va[US];
      const SRun ra = small_issue(q, va);
      if constexpr (SU == 2) {
        uint4 vb[US];
        const SRun rb = small_issue(q + WG, vb);
        small_sum(ra, va);
        small_sum(rb, vb);
      } else {
        small_sum(ra, va);
      }
    }
  };
  if (exact) loops(std::true_type{});
  else loops(std::false_type{});
  __syncthreads();
  const uint32_t acc = L.acc[t];
  return exact ? acc : s_class(acc, p.ew >> 31);
}

// The tile's results.  Unchained: fold1(initial + s).  Chained (CH,
// NS_DESC_CONT runs): a run head stores its folded value fold1(initial + s)
// (descriptor 0 heads its run with initial 0), a continuation its s, each
// with a u16 continuation flag after the n partials (u16, not u8: a wave's
// 64 flags then fill a whole 128-B line — byte flags cost 8.5 us more on 3M
// descriptors, profiles/r01/tune_chained_b2b.log); fold_scan folds the runs
// from those alone (6 bytes per descriptor, no descriptor re-read).
// NS_DESC_STORE: a run's final result r goes into the packet, big-endian,
// as ^r (SetChecksum(^xsum): connect.go:663, ipv4.go:236) or, with
// NS_DESC_STORE_RAW, as r (the CHECKSUM_PARTIAL pseudo-header sum,
// connect.go:660).  One u16 store, or two byte stores at an odd address.
//
// The aligned store is a relaxed agent-scope store (global_store_short sc1:
// written through, the line dropped from L2) rather than a plain one that
// leaves a partially dirty line in L2 to be written back during the next
// launch's stream: TX fill 285-286 vs 290-292 us (nontemporal: 292),
// bench.py --config 8, two interleaved rounds on one box
// (profiles/r02/tx_store_policy.txt).
__device__ __forceinline__ void store_result(uint64_t addr, uint32_t r, uint32_t stw, bool wb = false) {
  const uint32_t v = (stw & 2u) ? r : (~r & 0xFFFFu);
  uint8_t* p = reinterpret_cast<uint8_t*>((uintptr_t)addr);
  if (wb && !(addr & 1u)) {  // A/B (store bit 2): a plain, write-back store
    *reinterpret_cast<uint16_t*>(p) = (uint16_t)(((v & 0xFFu) << 8) | (v >> 8));
  } else if (!(addr & 1u)) {
    __hip_atomic_store(reinterpret_cast<uint16_t*>(p), (uint16_t)(((v & 0xFFu) << 8) | (v >> 8)), __ATOMIC_RELAXED,
                       __HIP_MEMORY_SCOPE_AGENT);
  } else {
    p[0] = (uint8_t)(v >> 8);
    p[1] = (uint8_t)v;
  }
}

// The store word (flags bits 2-15: NS_DESC_STORE | STORE_RAW | offset << 2)
// and its absolute address are validated at decode and parked in LDS for
// the lane's finish: carrying them through the scan loops in registers cost
// every kernel 10-20 VGPRs and a wave per SIMD, and re-reading the
// descriptor after the scan put a dependent global load at the end of every
// tile (+25 us on 3M descriptors).  A store that would land past the arena
// is dropped and counted as an error.
template <int P>
__device__ __forceinline__ void park_store(HybLds<P>& L, uint32_t store, uint4 raw, bool mine,
                                           uint64_t arena_abs, uint64_t arena_bytes,
                                           unsigned long long* err) {
  if (!store) return;
  uint32_t stw = (mine && (store & 1u)) ? (raw.w >> 18) & 0x3FFFu : 0u;
  const uint64_t at = ((uint64_t)raw.x | ((uint64_t)raw.y << 32)) + (stw >> 2);
  if (!(stw & 1u)) {  // NS_DESC_STORE_RAW counts only with NS_DESC_STORE
    stw = 0;
  } else if (at > arena_bytes || arena_bytes - at < 2) {
    atomicAdd(err, 1ull);
    stw = 0;
  }
  // NS_BATCH_PAIRED: the descriptor's CONT bit rides along at bit 14, so the
  // decoded flag need not stay live in a register through the scan.
  if (store & 2u) stw |= ((raw.w >> 17) & 1u) << 14;
  L.stw[threadIdx.x] = stw;
  L.sat[threadIdx.x] = arena_abs + at;
}

template <int P, bool CH>
__device__ __forceinline__ void finish_tile(HybLds<P>& L, uint32_t s, const Pkt& d, bool mine, uint64_t i,
                                            uint64_t n, uint16_t* __restrict__ out,
                                            uint32_t* __restrict__ partial, uint32_t store, bool wt = false) {
  const int t = threadIdx.x;
  if constexpr (CH) {
    const bool head = !d.cont || i == 0;
    const uint32_t v = head ? fold1((d.cont ? 0u : d.init) + s) : s;
    // Chained stores wait for fold_scan, which knows the final run value:
    // the flag word carries the store word.  (An in-tile fold that stored
    // runs lying inside the tile from this kernel measured 4-6 us slower on
    // the TX batch: 2M scattered 2-byte stores cost the same ~50 us of HBM
    // read-modify-write wherever they are issued, and issuing them here
    // holds every workgroup until its stores drain.)
    const uint32_t stw = ((store & 1u) && mine) ? L.stw[t] : 0u;
    if (!mine) return;
    partial[i] = v;
    reinterpret_cast<uint16_t*>(partial + chain_flag_word(n))[i] = (uint16_t)((head ? 0u : 1u) | (stw << 1));
  } else {
    uint32_t r = fold1(d.init + s);
    if (store & 2u) {
      // NS_BATCH_PAIRED: an odd-indexed NS_DESC_CONT descriptor continues the
      // one before it — Go's `Checksum(v, xsum)` chaining, exactly: the uint32
      // add wraps as Go's accumulator does, and a W-only class value (s_class)
      // behaves as S does.  Tiles hold an even number of descriptors, so lane
      // t - 1 of this wave holds it; every lane of the wave is here.
      // row_shr:1 — lane t takes lane t - 1's value (odd lanes never start a DPP row)
      const uint32_t prev = (uint32_t)__builtin_amdgcn_update_dpp(0, (int)r, 0x111, 0xF, 0xF, false);
      if ((t & 1) && (L.stw[t] >> 14)) r = fold1(prev + s);
    }
    if (!mine) return;
    if (wt)  // a self-signalling launch (zc_complete): results written through to the host
      __hip_atomic_store(out + i, (uint16_t)r, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
    else
      out[i] = (uint16_t)r;
    if (store & 1u) {
      const uint32_t stw = L.stw[t] & 0x3FFFu;
      if (stw) store_result(L.sat[t], r, stw, (store & 4u) != 0);
    }
  }
}

// Completion word of a self-signalling launch (an unchained zero-copy pass,
// csum_api.cpp run_zero_copy).  The caller, a CPU thread, spins on `flag` in
// coherent host memory and then reads the results; what makes a host reader
// that sees `seq` also see every result is the memory model's release/acquire
// chain (HSA / LLVM AMDGPU scoped model), not the hardware's store order:
//   1. every wave waits for its own result stores (vmcnt 0; MI355X_MICROARCH
//      "Valid forms": every storing wave, then the workgroup barrier);
//   2. lane 0: a SYSTEM-scope release fence (the host is a system-scope
//      observer), then the count on the device counter — release fence +
//      relaxed RMW = a release of everything this workgroup stored;
//   3. the workgroup whose add returns gridDim.x - 1 read the value written by
//      the RMW chain every other workgroup's release heads, so an acquire
//      fence (agent scope: all workgroups share the agent) makes their results
//      happen-before what it does next;
//   4. it resets the counter for the next pass, then a SYSTEM-scope release
//      fence and the store of `seq`: the host's acquire load of `flag`
//      (csum_api.cpp) synchronizes with it, so by transitivity it sees every
//      workgroup's results.
// Each fence is followed by an explicit `s_waitcnt vmcnt(0)`: ROCm 7.2 can
// drop a release fence's own wait when the wave's counter is provably empty
// (here: after a returned atomic), letting the next store overtake the L2
// write-back (MI355X_MICROARCH.md "Compiler hazard").
__device__ __forceinline__ void zc_complete(uint32_t* __restrict__ ctr, uint32_t* __restrict__ flag, uint32_t seq) {
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");  // 1
  __syncthreads();
  if (threadIdx.x == 0) {
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "");  // 2: system scope
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    const uint32_t prev = __hip_atomic_fetch_add(ctr, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    if (prev == gridDim.x - 1u) {
      __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "agent");  // 3
      __hip_atomic_store(ctr, 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      __builtin_amdgcn_fence(__ATOMIC_RELEASE, "");  // 4: system scope
      asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
      __hip_atomic_store(flag, seq, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
    }
  }
}

// WIN = false (arenas below 4 GiB): one SRD over the whole arena, no window
// reduction — it costs a block barrier and ~1 us on latency-bound
// small-packet batches.
// TP = descriptors per tile (<= WG): large packets get fewer per workgroup so
// a batch of 64 KiB GSO buffers still spreads over every CU.
// SU = small runs issued per lane per iteration; CH = chained batch
// (finish_tile writes partials and continuation flags for fold_scan).
template <int WG, int TP, int GB, int UB, int US, int AUXB, int UD = 0, bool WIN = false,
          int SU = 1, int QS = 0, bool CH = false>
// QS & 32 (tuning only): at least 8 waves per SIMD (<= 64 VGPRs).
__global__ __launch_bounds__(WG) __attribute__((amdgpu_waves_per_eu((QS & 32) ? 8 : (QS & 256) ? 7 : 1))) void csum_hyb(
    const uint8_t* __restrict__ arena, uint64_t arena_bytes,
    const uint4* __restrict__ desc, uint32_t n, uint16_t* __restrict__ out,
    uint32_t* __restrict__ partial, unsigned long long* __restrict__ err, uint32_t big_chunks,
    uint32_t store, uint32_t* __restrict__ zc_ctr, uint32_t* __restrict__ zc_flag, uint32_t zc_seq,
    uint32_t spec) {
  static_assert((WG & (WG - 1)) == 0, "tile must be a power of two");
  NSK_TL_BEGIN
  __shared__ HybLds<WG> L;
  const bool wt = zc_flag != nullptr;
  const int t = threadIdx.x;
  // QS & 16: XCD-aware tiles — the blocks one XCD runs (b, b + 8, ...) take
  // consecutive tiles, so the line two neighbouring tiles share is read
  // through one L2 (bijective for any grid).
  uint32_t tid = blockIdx.x;
  if constexpr ((QS & 16) != 0) {
    const uint32_t g = gridDim.x, q = g >> 3, r = g & 7u, x = blockIdx.x & 7u, k = blockIdx.x >> 3;
    tid = x < r ? x * (q + 1u) + k : r * (q + 1u) + (x - r) * q + k;
  }
  constexpr int QL = QS & ~(16 | 32);
  const uint64_t i = (uint64_t)tid * TP + t;
  const bool mine = t < TP && i < n;
  const uint64_t arena_abs = (uint64_t)(uintptr_t)arena;
  // Speculative payload loads beside the descriptor loads (spec_load), in
  // the one-wave small-packet tiles.  There every lane loads its descriptor
  // (the tail wave's spare lanes re-read the last one; the launcher never
  // launches n = 0) and selects afterwards: a load behind a branch is waited
  // for at the branch's end, before the speculative loads could be issued.
  constexpr bool kSpec = !WIN && UD > 0 && WG == 64 && TP == WG;
  [[maybe_unused]] uint4 sv[4];
  uint4 raw;
  if constexpr (kSpec) {
    const uint4 rawl = desc[min(i, (uint64_t)n - 1u)];
    // branch-free: with spec = 0 every slot is out of range (no memory access)
    spec_load(make_srd(arena_abs & ~15ull, arena_abs + arena_bytes - (arena_abs & ~15ull)),
              (uint64_t)tid * TP, spec ? n : 0u, spec, sv);
    __builtin_amdgcn_sched_barrier(0);  // all four issued before anything waits for the descriptor
    raw = mine ? rawl : make_uint4(0, 0, 0, 0);
  } else {
    raw = mine ? desc[i] : make_uint4(0, 0, 0, 0);
  }
  const Pkt d = decode(raw, mine, arena_abs, arena_bytes, err);
  park_store(L, store, raw, mine, arena_abs, arena_bytes, err);
  Win w;
  if constexpr (WIN) {
    w = tile_window<WG>(L, d, chunks_of(d), (uint32_t)UD);
  } else {
    w.base = arena_abs & ~15ull;
    w.span = arena_abs + arena_bytes - w.base;
    w.small = false;
  }

  auto tile = [&]() {
  if constexpr (!WIN && UD > 0) {
    // Small-packet tiles, decided per wave: a wave whose packets all span
    // <= UD chunks sums them directly and finishes at once — the quad-lane
    // shape when all span <= 4 (a full tile: lane t holds packet
    // blockIdx.x * WG + t), else one lane per packet — without waiting for
    // the other waves (a block-wide vote before the loads held every wave
    // of the tile until the slowest descriptor arrived).  Only if some wave
    // of the tile has a longer packet does the block run the scan path,
    // the finished waves taking part with no packets.
    const Srd r = make_srd(w.base, w.span);
    const PktInfo p = pkt_info(d, w.base);
    const bool small = __all(p.nch <= (uint32_t)UD) != 0;
    if (small) {
      bool done = false;
      uint32_t s = 0;
      if constexpr (kSpec) {
        if (spec && spec_check(p, i, spec)) {
          s = spec_sum(p, sv);
          done = true;
        }
      }
      if (!done) s = (TP == WG && __all(p.nch <= 4u)) ? quad_sum(r, p) : direct_sum<UD ? UD : 1>(r, p);
      finish_tile<WG, CH>(L, s, d, mine, i, n, out, partial, store, wt);
    }
    if (!__syncthreads_or(!small)) return;
    const uint32_t s =
        hyb_scan_tile<WG, TP, GB, UB, US, AUXB, false, SU, false, QL>(L, r, small ? PktInfo{} : p, big_chunks);
    if (!small) finish_tile<WG, CH>(L, s, d, mine, i, n, out, partial, store, wt);
    return;
  }

  if (!WIN || w.span + 64 < kMaxSrdBytes) {
    const Srd r = make_srd(w.base, w.span);
    const PktInfo p = pkt_info(d, w.base);
    if (UD > 0 && w.small) {
      // per wave: the quad-lane shape when every packet spans <= 4 chunks
      // (a full tile: lane t holds packet blockIdx.x * WG + t), else one lane
      // per packet
      const uint32_t s = (TP == WG && __all(p.nch <= 4u)) ? quad_sum(r, p) : direct_sum<UD ? UD : 1>(r, p);
      finish_tile<WG, CH>(L, s, d, mine, i, n, out, partial, store, wt);
      return;
    }
    const uint32_t s = hyb_scan_tile<WG, TP, GB, UB, US, AUXB, false, SU, false, QL>(L, r, p, big_chunks);
    finish_tile<WG, CH>(L, s, d, mine, i, n, out, partial, store, wt);
  } else if constexpr (WIN) {
    // The tile spans >= 4 GiB: 64-bit global loads, fewer in flight per lane
    // so this rarely taken path does not raise the kernel's register count.
    const Srd r = make_srd(0ull, 0ull);
    const PktInfo p = pkt_info(d, 0ull);
    const uint32_t s = hyb_scan_tile<WG, TP, 16, 4, 4, AUXB, true, 1>(L, r, p, big_chunks);
    finish_tile<WG, CH>(L, s, d, mine, i, n, out, partial, store, wt);
  }
  };
  tile();
  if (wt) zc_complete(zc_ctr, zc_flag, zc_seq);
  NSK_TL_END
}

// ---- descriptors far larger than a tile: csum_split -----------------------
// The tile kernel gives one workgroup to each descriptor of >= 64 KiB, which
// leaves most of the chip idle on a batch of a few huge descriptors (one
// 1 GiB buffer: one workgroup, 41 GB/s).  csum_split cuts each descriptor
// into `per` pieces of whole 128-B lines (even offsets from the packet
// start, so every piece keeps the packet's byte phase) and runs each piece
// through the tile kernel's own scan as a one-packet tile, always with the
// exact accumulator.  A piece adds its sum mod 2^32 — Go's uint32
// accumulator wraps the same way — to the descriptor's accumulator; the
// last piece to finish folds and writes the result (unchained) or the
// partial and flag (chained), as finish_tile does.  (A plain grid-stride
// streaming kernel in its place reached only 3.0-4.1 TB/s.)
constexpr uint64_t kSplitAvg = split_min_avg();  // launch_batch: the average size that selects it
constexpr uint32_t kSplitMaxN = 160;  // ... for fewer descriptors than this (more fill the chip as tiles)
constexpr uint32_t kSplitWGs = 256;   // pieces over the whole batch: one per CU (tools/split_probe.py)

template <int GB, int UB, int US, int AUXB, int SU>
__global__ __launch_bounds__(256) void csum_split(const uint8_t* __restrict__ arena, uint64_t arena_bytes,
                                                  const uint4* __restrict__ desc, uint32_t n, uint32_t per,
                                                  uint16_t* __restrict__ out, uint32_t* __restrict__ partial,
                                                  uint32_t* __restrict__ acc, unsigned long long* __restrict__ err,
                                                  uint32_t store, uint32_t big_chunks) {
  __shared__ HybLds<256> L;
  const uint32_t i = blockIdx.x / per, y = blockIdx.x % per;
  const int t = threadIdx.x;
  const uint4 raw = desc[i];
  const uint64_t off = (uint64_t)raw.x | ((uint64_t)raw.y << 32);
  uint64_t len = raw.z;
  const bool bad = off > arena_bytes || len > arena_bytes - off;
  if (bad) len = 0;
  if (bad && y == 0 && t == 0) atomicAdd(err, 1ull);
  const uint64_t arena_abs = (uint64_t)(uintptr_t)arena;
  const uint64_t piece = (((len + per - 1) / per) + 127) & ~127ull;
  const uint64_t r0 = min(len, (uint64_t)y * piece), r1 = min(len, r0 + piece);
  Pkt d{0ull, 0u, 0u, 0u, 0u};
  if (t == 0 && r1 > r0) {
    d.A = arena_abs + off + r0;
    d.len = (uint32_t)(r1 - r0);
    d.odd = (raw.w >> 16) & 1u;
  }
  // The piece's own SRD window (uniform over the block: it depends only on
  // the descriptor and blockIdx), so the arena may be any size; launch_batch
  // keeps every piece below 2^31 + 128 bytes.
  const uint64_t base = (arena_abs + off + r0) & ~15ull;
  const Srd r = make_srd(base, r1 > r0 ? arena_abs + off + r1 - base : 0ull);
  const PktInfo p = pkt_info(d, base);
  const uint32_t s = hyb_scan_tile<256, 1, GB, UB, US, AUXB, false, SU, true>(L, r, p, big_chunks);
  if (t != 0) return;
  atomicAdd(&acc[i], s);
  __threadfence();
  if (atomicAdd(&acc[n + i], 1u) != per - 1) return;
  // the last piece: finish descriptor i
  __threadfence();
  // (and leave its accumulator and counter zero for the next launch: the
  // scratch is zeroed once, at allocation, instead of per launch)
  const uint32_t sum = __hip_atomic_exchange(&acc[i], 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  __hip_atomic_store(&acc[n + i], 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  const uint32_t init = raw.w & 0xFFFFu, cont = (raw.w >> 17) & 1u;
  uint32_t stw = store ? (raw.w >> 18) & 0x3FFFu : 0u;
  const uint64_t at = off + (stw >> 2);
  if (!(stw & 1u)) {  // NS_DESC_STORE_RAW counts only with NS_DESC_STORE
    stw = 0;
  } else if (at > arena_bytes || arena_bytes - at < 2) {
    atomicAdd(err, 1ull);
    stw = 0;
  }
  if (partial) {
    const bool head = !cont || i == 0;
    partial[i] = head ? fold1((cont ? 0u : init) + sum) : sum;
    reinterpret_cast<uint16_t*>(partial + chain_flag_word(n))[i] = (uint16_t)((head ? 0u : 1u) | (stw << 1));
  } else {
    const uint32_t res = fold1(init + sum);
    out[i] = (uint16_t)res;
    if (stw) store_result(arena_abs + at, res, stw);
  }
}

// ---- run folding (NS_DESC_CONT chains) -------------------------------------
// After the CH kernel, descriptor k holds partial p_k and flag f_k (bit 0:
// continuation; bits 1-15: the store word).  Go's chaining (checksum.go:89,
// the `xsum = Checksum(v, xsum)` loops) is x_k = fold1(x_{k-1} + p_k) along a
// run, x_head = p_head (already folded with its initial).
//
// As a scan.  While x + p cannot wrap 2^32 (x <= 0xFFFF, so only p >=
// 0xFFFF0001 can), fold1(x + p) == x + p (mod 65535), and it is 0 iff x == 0
// and p == 0, else in [1, 0xFFFF].  So x is exactly described by
// (r = x mod 65535, z = x is 0), and a continuation acts as
// (r, z) -> (r + p mod 65535, z && p == 0): an associative segmented scan in
// which a head resets the state.  fold_scan is one pass (decoupled look-back):
// each workgroup scans kFoldBlock descriptors, publishes its aggregate (or,
// holding a head, its inclusive state) and takes its carry-in from its
// predecessors' statuses.  O(n) for any run length: one thread per head
// walking its run cost 183 ms on a 1M-descriptor run
// (profiles/r01/chain_fold.txt).  A block holding a continuation that could
// wrap folds its descriptors sequentially from the exact carry-in, as Go does,
// and publishes only its (exact) inclusive state.
//
// State word: bits 0-15 r, bit 16 z, bit 17 "a run head inside".
constexpr uint32_t kFZ = 1u << 16, kFH = 1u << 17, kFIdent = kFZ, kFMask = (1u << 18) - 1;
constexpr uint32_t kFAgg = 1u, kFIncl = 2u;  // status kinds

__device__ __forceinline__ uint32_t mod65535(uint32_t v) {
  v = (v & 0xFFFFu) + (v >> 16);
  v = (v & 0xFFFFu) + (v >> 16);
  return v == 0xFFFFu ? 0u : v;
}

__device__ __forceinline__ uint32_t fold_state(uint32_t x) {  // a head with value x
  return (x == 0xFFFFu ? 0u : x) | (x == 0 ? kFZ : 0u) | kFH;
}

__device__ __forceinline__ uint32_t fold_elem(uint32_t p, uint32_t f) {
  return (f & 1u) ? (mod65535(p) | (p == 0 ? kFZ : 0u)) : fold_state(p);
}

__device__ __forceinline__ uint32_t fold_combine(uint32_t a, uint32_t b) {  // a, then b
  if (b & kFH) return b;
  uint32_t r = (a & 0xFFFFu) + (b & 0xFFFFu);
  r = r >= 65535u ? r - 65535u : r;
  return r | (a & b & kFZ) | (a & kFH);
}

__device__ __forceinline__ uint32_t fold_value(uint32_t st) {
  return (st & kFZ) ? 0u : ((st & 0xFFFFu) == 0 ? 0xFFFFu : (st & 0xFFFFu));
}

__device__ __forceinline__ void fold_publish(uint64_t* st, uint32_t gen, uint32_t kind, uint32_t state) {
  // Relaxed: a status word carries all it says (no other data is published
  // through it), and a release/acquire pair at agent scope would write back /
  // invalidate the XCD's whole L2 per block.
  __hip_atomic_store(st, ((uint64_t)gen << 32) | ((uint64_t)kind << 30) | state, __ATOMIC_RELAXED,
                     __HIP_MEMORY_SCOPE_AGENT);
}

constexpr uint32_t kFoldSpins = 4096;

// The state just before descriptor k0 > 0, by Go's own sequential fold from
// the head of the run k0 falls in (exact; the look-back's fallback).
__device__ __noinline__ uint32_t fold_carry_walk(const uint32_t* __restrict__ partial,
                                                 const uint16_t* __restrict__ flags, uint64_t k0) {
  uint64_t h = k0 - 1;
  while (h > 0 && (flags[h] & 1u)) --h;
  uint32_t x = partial[h];
  for (uint64_t k = h + 1; k < k0; ++k) x = fold1(x + partial[k]);
  return fold_state(x);
}

// SPINS: polls of a predecessor's status before deriving the carry-in
// directly (the tuning library builds SPINS = 0 to test that path).
template <uint32_t SPINS = kFoldSpins>
__global__ __launch_bounds__(256) void fold_scan(const uint32_t* __restrict__ partial,
                                                 const uint16_t* __restrict__ flags, uint32_t n,
                                                 uint64_t* __restrict__ status, uint32_t gen,
                                                 uint16_t* __restrict__ out, const uint4* __restrict__ desc,
                                                 const uint8_t* __restrict__ arena) {
  __shared__ uint32_t sh[4];
  __shared__ uint32_t s_carry;
  __shared__ uint32_t lx[kFoldBlock];  // results + flags (wrap path; store transposition)
  const int t = threadIdx.x, lane = t & 63, w = t >> 6;
  // The look-back below waits only on lower-numbered blocks, which the
  // dispatcher starts first; should one not be running (or be slow), the
  // waiter stops after kFoldSpins polls and derives its carry-in itself
  // (fold_carry_walk), so no schedule can deadlock.  (An atomic ticket for
  // the block order instead cost 17 us on 1,536 blocks: one contended
  // device-scope atomic per block.)
  const uint32_t blk = blockIdx.x;
  const uint64_t b0 = (uint64_t)blk * kFoldBlock;
  const uint64_t base = b0 + (uint64_t)t * kFoldPer;

  // Scan phase: each thread owns 8 consecutive descriptors (3 vector loads).
  uint32_t p[kFoldPer], f[kFoldPer];
  if (base + kFoldPer <= n) {
    const uint4 a = *reinterpret_cast<const uint4*>(partial + base);
    const uint4 b = *reinterpret_cast<const uint4*>(partial + base + 4);
    const uint4 c = *reinterpret_cast<const uint4*>(flags + base);
    p[0] = a.x; p[1] = a.y; p[2] = a.z; p[3] = a.w;
    p[4] = b.x; p[5] = b.y; p[6] = b.z; p[7] = b.w;
    f[0] = c.x & 0xFFFFu; f[1] = c.x >> 16; f[2] = c.y & 0xFFFFu; f[3] = c.y >> 16;
    f[4] = c.z & 0xFFFFu; f[5] = c.z >> 16; f[6] = c.w & 0xFFFFu; f[7] = c.w >> 16;
  } else {
#pragma unroll
    for (uint32_t j = 0; j < kFoldPer; ++j) {
      const bool in = base + j < n;
      p[j] = in ? partial[base + j] : 0u;
      f[j] = in ? flags[base + j] : 1u;  // past the end: an empty continuation
    }
  }
  uint32_t e[kFoldPer];
  uint32_t a = kFIdent;
  bool wraps = false;
#pragma unroll
  for (uint32_t j = 0; j < kFoldPer; ++j) {
    e[j] = fold_elem(p[j], f[j]);
    a = fold_combine(a, e[j]);
    wraps |= (f[j] & 1u) && p[j] >= 0xFFFF0001u;
  }
  // ordered inclusive scan of the thread totals: within the wave, then the waves
  uint32_t v = a;
  for (int d = 1; d < 64; d <<= 1) {
    const uint32_t o = __shfl_up(v, d, 64);
    if (lane >= d) v = fold_combine(o, v);
  }
  if (lane == 63) sh[w] = v;
  const bool seq = __syncthreads_or(wraps) != 0;
  const uint32_t total = fold_combine(fold_combine(sh[0], sh[1]), fold_combine(sh[2], sh[3]));

  if (t == 0) {
    const bool incl = blk == 0 || (total & kFH);
    if (!seq) fold_publish(&status[blk], gen, incl ? kFIncl : kFAgg, total);
    uint32_t carry = kFIdent;
    // A block whose first descriptor heads a run needs no carry-in (every
    // state in it starts at or after that head): only its statuses matter.
    if (blk > 0 && (f[0] & 1u)) {
      // Walk back to the nearest inclusive status; the aggregates passed on
      // the way hold no head and no wrap, so they combine as residue adds.
      uint32_t run = kFIdent;
      for (uint32_t j = blk - 1;; --j) {
        uint64_t sw = 0;
        bool ready = false;
        for (uint32_t spins = 0; spins < SPINS; ++spins) {
          sw = __hip_atomic_load(&status[j], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
          if ((uint32_t)(sw >> 32) == gen && ((sw >> 30) & 3u)) {
            ready = true;
            break;
          }
          __builtin_amdgcn_s_sleep(2);
        }
        if (!ready) {
          carry = fold_carry_walk(partial, flags, b0);
          break;
        }
        const uint32_t val = (uint32_t)sw & kFMask;
        if (((sw >> 30) & 3u) == kFIncl) {
          carry = fold_combine(val, run);
          break;
        }
        run = fold_combine(val, run);
      }
    }
    if (blk > 0 && !seq && !incl) fold_publish(&status[blk], gen, kFIncl, fold_combine(carry, total));
    s_carry = carry;
  }
  __syncthreads();
  const uint32_t carry = s_carry;

  uint32_t x[kFoldPer];
  if (!seq) {
    uint32_t st = carry;
    for (int q = 0; q < w; ++q) st = fold_combine(st, sh[q]);
    const uint32_t before = __shfl_up(v, 1, 64);
    if (lane > 0) st = fold_combine(st, before);
#pragma unroll
    for (uint32_t j = 0; j < kFoldPer; ++j) {
      st = fold_combine(st, e[j]);
      x[j] = fold_value(st);
    }
  } else {
    // Go's own sequential fold over the block, from the exact carry-in (a
    // head-holding state, or nothing before descriptor 0).
    if (t == 0) {
      uint32_t xv = fold_value(carry);
      const uint64_t cnt = min<uint64_t>(kFoldBlock, n - b0);
      for (uint32_t k = 0; k < cnt; ++k) {
        const uint32_t pk = partial[b0 + k];
        const uint32_t fk = flags[b0 + k];
        xv = (fk & 1u) ? fold1(xv + pk) : pk;
        lx[k] = xv | (fk << 16);
      }
      fold_publish(&status[blk], gen, kFIncl, fold_state(xv));
    }
    __syncthreads();
#pragma unroll
    for (uint32_t j = 0; j < kFoldPer; ++j) x[j] = lx[t * kFoldPer + j] & 0xFFFFu;
  }
  uint32_t mine_st = 0;
#pragma unroll
  for (uint32_t j = 0; j < kFoldPer; ++j) mine_st |= (f[j] >> 1) & 1u;
  const bool stores = __syncthreads_or(mine_st) != 0;

  if (base + kFoldPer <= n && ((uintptr_t)(out + base) & 15u) == 0) {
    uint4 o;
    o.x = x[0] | (x[1] << 16); o.y = x[2] | (x[3] << 16);
    o.z = x[4] | (x[5] << 16); o.w = x[6] | (x[7] << 16);
    *reinterpret_cast<uint4*>(out + base) = o;
  } else {
#pragma unroll
    for (uint32_t j = 0; j < kFoldPer; ++j)
      if (base + j < n) out[base + j] = (uint16_t)x[j];
  }
  if (!stores) return;

  // In-packet stores (NS_DESC_STORE), transposed through LDS: round j covers
  // descriptors b0 + 256 j + t, so each store instruction of a round writes
  // neighbouring packets (the partial-sector read-modify-writes then stay in
  // nearby HBM rows: 11 us less per 2M stores than descriptors 8 apart per
  // instruction).
  if (!seq) {
#pragma unroll
    for (uint32_t j = 0; j < kFoldPer; ++j) lx[t * kFoldPer + j] = x[j] | (f[j] << 16);
  }
  __syncthreads();
  uint32_t xf[kFoldPer];
  uint4 dk[kFoldPer];
#pragma unroll
  for (uint32_t j = 0; j < kFoldPer; ++j) {
    const uint64_t k = b0 + 256u * j + t;
    xf[j] = k < n ? lx[256u * j + t] : 0u;
    dk[j] = ((xf[j] >> 17) & 1u) ? desc[k] : make_uint4(0, 0, 0, 0);
  }
#pragma unroll
  for (uint32_t j = 0; j < kFoldPer; ++j) {
    const uint32_t stw = xf[j] >> 17;
    if (stw & 1u)
      store_result((uint64_t)(uintptr_t)arena + ((uint64_t)dk[j].x | ((uint64_t)dk[j].y << 32)) + (stw >> 2),
                   xf[j] & 0xFFFFu, stw);
  }
}

// Rebase a host-pipeline chunk's descriptor table on the device: offsets
// relative to the chunk's first byte (and 0 for empty descriptors), so the
// host copies the caller's table verbatim instead of rewriting it.
__global__ __launch_bounds__(256) void rebase_desc(uint4* __restrict__ d, uint32_t n, uint64_t bias) {
  const uint64_t i = (uint64_t)blockIdx.x * 256 + threadIdx.x;
  if (i >= n) return;
  uint4 v = d[i];
  const uint64_t off = v.z ? (((uint64_t)v.x | ((uint64_t)v.y << 32)) - bias) : 0ull;
  v.x = (uint32_t)off;
  v.y = (uint32_t)(off >> 32);
  d[i] = v;
}

}  // namespace nsk

// ---- launchers (C++ linkage, used by csum_api.cpp) ------------------------
namespace nsk {

template <uint32_t SPINS = kFoldSpins>
static void launch_fold(ChainScratch ch, uint32_t n, uint16_t* out, const void* desc, const uint8_t* arena,
                        hipStream_t stream) {
  static std::atomic<uint32_t> gen_counter{0};
  uint32_t gen = ++gen_counter;
  if (gen == 0) gen = ++gen_counter;  // 0 never tags a status
  const uint32_t nb = (uint32_t)chain_blocks(n);
  const uint16_t* flags = reinterpret_cast<const uint16_t*>(ch.partial + chain_flag_word(n));
  hipLaunchKernelGGL(fold_scan<SPINS>, dim3(nb), dim3(256), 0, stream, ch.partial, flags, n, ch.status, gen, out,
                     reinterpret_cast<const uint4*>(desc), arena);
}

template <int TP, int GB, int UB, int US, int AUXB, int UD, int SU = 1, int QS = 0, int WG = 256>
static hipError_t launch_hyb_tp(const uint8_t* arena, uint64_t arena_bytes, const void* desc,
                                uint32_t n, uint16_t* out, uint32_t* partial,
                                unsigned long long* err, hipStream_t stream, uint32_t big_chunks,
                                uint32_t store = 0, ZcSignal zc = {}, uint32_t spec = 0) {
  static_assert(TP <= WG, "a tile holds at most one descriptor per thread");
  const uint32_t grid = (uint32_t)(((uint64_t)n + TP - 1) / TP);
  const uint4* d = reinterpret_cast<const uint4*>(desc);
  // One SRD over the whole arena when it fits (arena base rounded down to 16 B
  // plus the arena), else per-tile windows.
  const bool win = ((uintptr_t)arena & 15u) + arena_bytes + 64 >= kMaxSrdBytes;
#define NSK_LAUNCH(W, C)                                                                              \
  hipLaunchKernelGGL((csum_hyb<WG, TP, GB, UB, US, AUXB, UD, W, SU, QS, C>), dim3(grid), dim3(WG), 0, \
                     stream, arena, arena_bytes, d, n, out, partial, err, big_chunks, store, zc.ctr, zc.flag, zc.seq, spec)
  if (partial) {
    if (win) NSK_LAUNCH(true, true);
    else NSK_LAUNCH(false, true);
  } else {
    if (win) NSK_LAUNCH(true, false);
    else NSK_LAUNCH(false, false);
  }
#undef NSK_LAUNCH
  return hipGetLastError();
}

// Descriptors per workgroup: the largest power of two <= kTileBytes of
// payload per workgroup, clamped to [1, 256].  Tiles of 32-64 KiB balance the
// tail best; below ~32 KiB per workgroup the prologue dominates (tools/tune.py
// on MI355X, profiles/r01/tune_tile_bytes.log: 1M x 1500 B 218 us at 32
// descriptors vs 221 at 64 and 244 at 16; the Zipf batch 103 us at 64 vs 107
// at 128 and 114 at 32; 64 KiB GSO buffers flat).
constexpr uint64_t kTileBytes = 64u << 10;
constexpr uint32_t kBigChunks = 40;  // packets of >= this many 16-B chunks take the 8-lane groups
// ... in a zero-copy pass: 32 KiB, what one workgroup's lane loop covers in
// one iteration (256 lanes x 2 runs x 4 chunks); a larger packet's body goes
// to the groups, 64 KiB per iteration (one 64 KiB Checksum: 19.4 us that
// way, 26.8 us through the lane runs)
constexpr uint32_t kZeroCopyBigChunks = 2048;
constexpr uint64_t kZeroCopyTileBytes = 16u << 10;  // ... and its tiles
template <int GB, int UB, int US, int AUXB, int UD = 0, int SU = 1, int QS = 0>
static hipError_t launch_hyb(const uint8_t* arena, uint64_t arena_bytes, const void* desc,
                             uint32_t n, uint16_t* out, uint32_t* partial,
                             unsigned long long* err, hipStream_t stream, uint32_t big_chunks,
                             uint64_t sizing_bytes = 0, uint64_t tile_bytes = kTileBytes, uint32_t store = 0,
                             ZcSignal zc = {}, uint32_t spec = 0) {
  const uint64_t avg = std::max<uint64_t>((sizing_bytes ? sizing_bytes : arena_bytes) / n, 1);
  const uint64_t want = tile_bytes / avg;
#define NSK_TP(tp) \
  if (want >= tp)              \
  return launch_hyb_tp<tp, GB, UB, US, AUXB, UD, SU, QS>(arena, arena_bytes, desc, n, out, partial, err, stream, big_chunks, store, zc)
  if constexpr (UD > 0) {
    // The small-packet variant (launch_batch: < 256 B per descriptor) keeps
    // full tiles of one-wave workgroups: its direct path is one packet per
    // lane, and a one-wave workgroup retires (and frees its slot for the next
    // tile) as soon as its own packets are done.  1M x 64 B with the
    // descriptor tables rotated past the MALL, as bench.py runs it: 15.5-15.7
    // vs 16.7 us for 256-thread tiles (tools/tune.py --rot-desc,
    // profiles/r02/tune_small_wg_rotdesc.log; 128-B packets -1%, 192-B +2%).
    return launch_hyb_tp<64, GB, UB, US, AUXB, UD, SU, QS, 64>(arena, arena_bytes, desc, n, out, partial, err,
                                                               stream, big_chunks, store, zc, spec);
  } else {
    NSK_TP(256);
    NSK_TP(128);
    NSK_TP(64);
    NSK_TP(32);
    NSK_TP(16);
    NSK_TP(8);
    NSK_TP(4);
    NSK_TP(2);
    if (store & 2u)  // NS_BATCH_PAIRED: a pair never straddles two tiles
      return launch_hyb_tp<2, GB, UB, US, AUXB, UD, SU, QS>(arena, arena_bytes, desc, n, out, partial, err, stream,
                                                            big_chunks, store, zc);
    return launch_hyb_tp<1, GB, UB, US, AUXB, UD, SU, QS>(arena, arena_bytes, desc, n, out, partial, err, stream,
                                                          big_chunks, store, zc);
  }
#undef NSK_TP
}

hipError_t launch_rebase(void* desc, uint32_t n, uint64_t bias, hipStream_t stream) {
  if (n == 0) return hipSuccess;
  hipLaunchKernelGGL(rebase_desc, dim3((n + 255) / 256), dim3(256), 0, stream, reinterpret_cast<uint4*>(desc), n,
                     bias);
  return hipGetLastError();
}

// The error-count exchange of ns_csum_sync: one atomic, so a kernel still
// running on another stream never has its count wiped by a separate reset.
__global__ void take_err(unsigned long long* __restrict__ err, unsigned long long* __restrict__ taken) {
  if (threadIdx.x == 0) *taken = atomicExch(err, 0ull);
}

__global__ void signal_host(uint32_t* __restrict__ flag, uint32_t seq) {
  if (threadIdx.x == 0) __hip_atomic_store(flag, seq, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_SYSTEM);
}

hipError_t launch_signal(uint32_t* flag, uint32_t seq, hipStream_t stream) {
  hipLaunchKernelGGL(signal_host, dim3(1), dim3(64), 0, stream, flag, seq);
  return hipGetLastError();
}

hipError_t launch_take_err(unsigned long long* err, unsigned long long* taken, hipStream_t stream) {
  hipLaunchKernelGGL(take_err, dim3(1), dim3(64), 0, stream, err, taken);
  return hipGetLastError();
}

hipError_t launch_batch(const uint8_t* arena, uint64_t arena_bytes,
                        const void* desc, uint32_t n, uint16_t* out,
                        ChainScratch chain, unsigned long long* err,
                        hipStream_t stream, uint64_t sizing_bytes, uint32_t store,
                        uint32_t* split, ZcSignal zc) {
  uint32_t* part = chain.partial;  // the chained scratch (layout: csum_kernels.h)
  if (zc.flag && (part || split || !zc.ctr)) return hipErrorInvalidValue;  // unchained tiles only
  if (n == 0) return hipSuccess;
  hipError_t e;
  if (sizing_bytes == 0) sizing_bytes = arena_bytes;
  if ((store & 2u) && (part || split || zc.flag)) return hipErrorInvalidValue;  // pairs: plain tiles only
  if (split && sizing_bytes / n >= kSplitAvg && n < kSplitMaxN) {
    // A few huge descriptors: spread each over many workgroups.  (`split`
    // holds zeros between launches: csum_split leaves it so.)  Each piece
    // reads through its own SRD window, so arenas of any size qualify; in one
    // of 4 GiB or more, at least two pieces per descriptor keep a piece of a
    // u32-length descriptor below the window limit.  (Before the windows such
    // arenas took one workgroup per descriptor: 64-bit loads, ~0.1 s for a
    // 4 GiB descriptor.)
    const bool huge_arena = ((uintptr_t)arena & 15u) + arena_bytes + 64 >= kMaxSrdBytes;
    const uint32_t per = std::max<uint32_t>(huge_arena ? 2u : 1u, kSplitWGs / n);
    hipLaunchKernelGGL((csum_split<8, 16, 4, 2, 2>), dim3(n * per), dim3(256), 0, stream, arena, arena_bytes,
                       reinterpret_cast<const uint4*>(desc), n, per, out, part, split, err, store, 64u);
    e = hipGetLastError();
  } else if (sizing_bytes / n >= 256) {
    // Packets of >= 40 chunks (~640 B): their whole 128-B lines to 8-lane
    // groups (one full line per group per load instruction, 16 loads per lane
    // in flight) with nontemporal loads; their partial edge lines and all
    // smaller packets to per-lane runs of 4, two runs issued per lane per
    // iteration (tools/tune.py on MI355X: 220.6 us on 1M x 1500 B = 90.2% of
    // 8 TB/s, 107 us on the Zipf batch; profiles/r01/tune_*.json).  The
    // group threshold, swept over uniform 576-960-B packets
    // (profiles/r01/tune_bc_*.log): 40 chunks beats 64 by up to 15% on
    // 704-960-B packets (960 B: 219.8 vs 253.5 us per 1.5 GB) and ties it
    // elsewhere; at 36 chunks and below the groups lose (576 B: 277.7 vs
    // 253.4 us).
    // A zero-copy pass (arena == nullptr: descriptors hold absolute addresses
    // of mapped host memory, csum_api.cpp run_zero_copy) is PCIe-latency
    // bound, not bandwidth bound: it sends packets below 32 KiB through the
    // lane runs (the group loop and the lane loop are two dependent PCIe
    // round trips per tile, the lane loop alone one) and cuts 16 KiB tiles
    // (more workgroups, so a 64 KiB call's lane runs are all in flight at
    // once).  tools/latency.cc, same box, against groups and 64 KiB tiles:
    // Checksum(1500 B) 12.7-13.1 vs 14.8-14.9 us, the 45-segment VV batch
    // 15.8-16.0 vs 18.9-19.5, 45 chained segments 14.9-15.5 vs 18.2,
    // 1 MiB of packets 44.7-45.3 vs 50.7-50.9 (profiles/r02/latency_zc_ab.txt).
    e = launch_hyb<8, 16, 4, 2, 0, 2>(arena, arena_bytes, desc, n, out, part, err, stream,
                                      arena ? kBigChunks : kZeroCopyBigChunks, sizing_bytes,
                                      arena ? kTileBytes : kZeroCopyTileBytes, store, zc);
  } else {
    // Small packets: the same kernel plus the direct path — a tile whose
    // packets all span <= 5 chunks (any <= 65-B packet) has each lane read its
    // own packet with no scan; 16 x 8 groups keep the register count (and the
    // occupancy this latency-bound case needs) lower.
    // Fixed-stride tables (every packet in a slot of `spec` bytes: an arena
    // of exactly n slots, as a receive ring of fixed-size buffers) get the
    // speculative payload loads (spec_load): the descriptor -> payload
    // dependency is what this latency-bound case waits on.
    // A table that only looks fixed-stride costs one wasted load round per
    // wave; results never depend on the prediction.
    uint32_t spec = 0;
    if (arena && ((uintptr_t)arena & 15u) == 0 && arena_bytes % n == 0) {
      const uint64_t st = arena_bytes / n;
      if (st % 16 == 0 && st >= 16 && st <= 64) spec = (uint32_t)st;
    }
    e = launch_hyb<16, 8, 4, 2, 5>(arena, arena_bytes, desc, n, out, part, err, stream, 64u, 0, kTileBytes,
                                   store, zc, spec);
  }
  if (e != hipSuccess || part == nullptr) return e;
  // run folding: one pass over 6 B per descriptor, any run length
  if (chain.walk) launch_fold<0>(chain, n, out, desc, arena, stream);
  else launch_fold<>(chain, n, out, desc, arena, stream);
  return hipGetLastError();
}

}  // namespace nsk
