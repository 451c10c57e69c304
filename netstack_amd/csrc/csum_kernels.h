// Internal launcher interface between the C ABI (csum_api.cpp) and the gfx950
// kernels (csum_kernels.hip).  Not installed; the public boundary is
// include/netstack_csum.h.
#pragma once
#include <hip/hip_runtime_api.h>
#include <stdint.h>

namespace nsk {

// Enqueue the checksum of n descriptors (16-byte ns_pkt_desc, device memory)
// over `arena` on `stream`.  With `partial` != nullptr (room for n u32 plus
// n u16) the per-descriptor partial sums and continuation flags go there
// and a chain pass folds NS_DESC_CONT runs into `out`; otherwise every
// descriptor is independent.
// Out-of-range descriptors are summed as empty and counted in *err.
// `sizing_bytes` (0: arena_bytes) is the byte count the launcher sizes tiles
// by — the payload of a batch whose "arena" is the whole address space
// (arena = nullptr, descriptors holding absolute addresses).
// `store`: descriptors flagged NS_DESC_STORE write their final result into
// the (then writable) arena.
hipError_t launch_batch(const uint8_t* arena, uint64_t arena_bytes,
                        const void* desc, uint32_t n, uint16_t* out,
                        uint32_t* partial, unsigned long long* err,
                        hipStream_t stream, uint64_t sizing_bytes = 0, uint32_t store = 0);

}  // namespace nsk
