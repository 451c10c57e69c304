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
// Work decomposition ("chunk stream").  A 256-thread workgroup owns a tile of
// 256 descriptors.  It scans their chunk counts into a virtual chunk space of
// the tile (LDS), then streams that space: each lane takes U consecutive
// chunks per step (so a lane's chunks almost always belong to one packet and
// are summed in registers), finds their packet by a binary search of the
// scan, issues all U 16-byte loads, then masks / splits the bytes into E/O
// lanes of a packed 2x16-bit accumulator (v_and / v_perm / v_add3) and, on a
// packet change, adds the packet's 32-bit partial into an LDS accumulator
// (ds_add_u32).  The tile epilogue folds initial+acc and writes one u16 per
// packet (coalesced).  No MFMA: this is a byte sum, HBM-bound.
#include <hip/hip_runtime.h>
#include <stdint.h>

#include "csum_kernels.h"

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

// meta word: bits 0-3 = first byte within first chunk, 4-7 = last byte within
// last chunk, bit 8 = phase.
template <int WG, int U>
__global__ __launch_bounds__(WG) void csum_tiles(
    const uint8_t* __restrict__ arena, uint64_t arena_bytes,
    const uint4* __restrict__ desc, uint32_t n, uint16_t* __restrict__ out,
    uint32_t* __restrict__ partial, unsigned long long* __restrict__ err) {
  constexpr int P = WG;  // descriptors per tile
  constexpr int NW = WG / 64;
  static_assert(U * 1020 < 65536, "packed 16-bit lanes would overflow");
  __shared__ uint64_t s_cstart[P + 1];  // virtual chunk start per packet
  __shared__ uint64_t s_cbase[P];       // absolute chunk index - s_cstart
  __shared__ uint32_t s_meta[P];
  __shared__ uint32_t s_acc[P];
  __shared__ uint64_t s_wtot[NW];

  const int t = threadIdx.x;
  const int lane = t & 63;
  const int wv = t >> 6;
  const uint64_t i = (uint64_t)blockIdx.x * P + t;

  uint64_t nch = 0, cb = 0;
  uint32_t meta = 0, init = 0;
  if (i < n) {
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
      // chunk coordinates relative to the 16-byte-aligned arena base (keeps
      // the loads in the global address space; parity is unchanged).
      const uint64_t a = ((uint64_t)(uintptr_t)arena & 15u) + off;
      const uint64_t last = a + len - 1;
      nch = (last >> 4) - (a >> 4) + 1;
      cb = a >> 4;
      meta = (uint32_t)(a & 15u) | ((uint32_t)(last & 15u) << 4) |
             ((uint32_t)((a + odd) & 1u) << 8);
    }
  }

  // Block-wide exclusive scan of the chunk counts.
  uint64_t incl = nch;
#pragma unroll
  for (int d = 1; d < 64; d <<= 1) {
    const uint64_t y = __shfl_up(incl, d, 64);
    if (lane >= d) incl += y;
  }
  if (lane == 63) s_wtot[wv] = incl;
  s_acc[t] = 0u;
  __syncthreads();
  uint64_t wbase = 0;
#pragma unroll
  for (int w = 0; w < NW; ++w)
    if (w < wv) wbase += s_wtot[w];
  const uint64_t excl = wbase + incl - nch;
  s_cstart[t] = excl;
  s_cbase[t] = cb - excl;
  s_meta[t] = meta;
  if (t == P - 1) s_cstart[P] = excl + nch;
  __syncthreads();

  const uint4* __restrict__ chunks =
      reinterpret_cast<const uint4*>(arena - ((uintptr_t)arena & 15u));
  const uint64_t C = s_cstart[P];
  for (uint64_t base = 0; base < C; base += (uint64_t)WG * U) {
    const uint64_t c0 = base + (uint64_t)t * U;
    if (c0 >= C) break;
    // Largest pk with s_cstart[pk] <= c0 (that packet is non-empty).
    int lo = 0, hi = P;
#pragma unroll
    for (int s = 0; s < 8; ++s) {  // log2(P) steps (P = 256)
      const int mid = (lo + hi) >> 1;
      if (s_cstart[mid] <= c0) lo = mid; else hi = mid;
    }
    int pk = lo;
    uint64_t pstart = s_cstart[pk];
    uint64_t pend = s_cstart[pk + 1];
    uint64_t pbase = s_cbase[pk];

    uint4 v[U];
    int pid[U];
    uint32_t firstm = 0, lastm = 0;
#pragma unroll
    for (int u = 0; u < U; ++u) {
      const uint64_t c = c0 + u;
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
        v[u] = chunks[pbase + c];
      } else {
        pid[u] = -1;
        v[u] = make_uint4(0, 0, 0, 0);
      }
    }

    int cur = pid[0];
    uint32_t e = 0, o = 0;
#pragma unroll
    for (int u = 0; u < U; ++u) {
      if (pid[u] < 0) break;
      if (pid[u] != cur) {
        atomicAdd(&s_acc[cur], partial_of(e, o, (s_meta[cur] >> 8) & 1u));
        e = 0;
        o = 0;
        cur = pid[u];
      }
      uint4 w = v[u];
      if ((firstm | lastm) & (1u << u)) {
        const uint32_t m = s_meta[cur];
        const int blo = (firstm >> u) & 1u ? (int)(m & 15u) : 0;
        const int bhi = (lastm >> u) & 1u ? (int)((m >> 4) & 15u) + 1 : 16;
        w.x &= dword_mask(blo, bhi, 0);
        w.y &= dword_mask(blo, bhi, 1);
        w.z &= dword_mask(blo, bhi, 2);
        w.w &= dword_mask(blo, bhi, 3);
      }
      acc_chunk(w, e, o);
    }
    atomicAdd(&s_acc[cur], partial_of(e, o, (s_meta[cur] >> 8) & 1u));
  }
  __syncthreads();

  if (i < n) {
    const uint32_t s = s_acc[t];
    if (partial) partial[i] = s;
    else out[i] = (uint16_t)fold1(init + s);
  }
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

static constexpr int kWG = 256;
static constexpr int kU = 8;

hipError_t launch_batch(const uint8_t* arena, uint64_t arena_bytes,
                        const void* desc, uint32_t n, uint16_t* out,
                        uint32_t* partial, unsigned long long* err,
                        hipStream_t stream) {
  if (n == 0) return hipSuccess;
  const uint32_t tiles = (n + kWG - 1) / kWG;
  hipLaunchKernelGGL((csum_tiles<kWG, kU>), dim3(tiles), dim3(kWG), 0, stream,
                     arena, arena_bytes, reinterpret_cast<const uint4*>(desc), n,
                     out, partial, err);
  hipError_t e = hipGetLastError();
  if (e != hipSuccess || partial == nullptr) return e;
  const uint32_t blocks = (n + 255) / 256;
  hipLaunchKernelGGL(csum_chain, dim3(blocks), dim3(256), 0, stream,
                     reinterpret_cast<const uint4*>(desc), n, partial, out);
  return hipGetLastError();
}

}  // namespace nsk
