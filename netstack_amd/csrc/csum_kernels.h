// Internal launcher interface between the C ABI (csum_api.cpp) and the gfx950
// kernels (csum_kernels.hip).  Not installed; the public boundary is
// include/netstack_csum.h.
#pragma once
#include <hip/hip_runtime_api.h>
#include <stdint.h>

namespace nsk {

// Enqueue the checksum of n descriptors (16-byte ns_pkt_desc, device memory)
// over `arena` on `stream`.  With `partial` != nullptr (a chained-batch
// scratch of chain_scratch_words(n) u32, layout below) the per-descriptor
// partial sums and continuation flags go there and a fold pass folds
// NS_DESC_CONT runs into `out`; otherwise every
// descriptor is independent.
// Out-of-range descriptors are summed as empty and counted in *err.
// `sizing_bytes` (0: arena_bytes) is the byte count the launcher sizes tiles
// by — the payload of a batch whose "arena" is the whole address space
// (arena = nullptr, descriptors holding absolute addresses).
// `store`: descriptors flagged NS_DESC_STORE write their final result into
// the (then writable) arena.
// `split`: scratch for csum_split (see below), or nullptr.
// Chained-batch scratch layout, in u32 words: the n partial sums, their u16
// flags from chain_flag_word(n) (16-B aligned), then one 8-B fold status per
// kFoldBlock descriptors from chain_status_word(n) (csum_kernels.hip, run
// folding).  Statuses are tagged with a launch generation, so stale ones are
// ignored; a fresh scratch is zeroed so that no garbage word can carry a
// live generation.
constexpr uint32_t kFoldPer = 8;                 // descriptors per thread
constexpr uint32_t kFoldBlock = 256 * kFoldPer;  // descriptors per workgroup
constexpr uint64_t chain_flag_word(uint64_t n) { return (n + 3) & ~3ull; }
constexpr uint64_t chain_status_word(uint64_t n) { return (chain_flag_word(n) + ((n + 7) & ~7ull) / 2 + 1) & ~1ull; }
constexpr uint64_t chain_blocks(uint64_t n) { return (n + kFoldBlock - 1) / kFoldBlock; }
constexpr uint64_t chain_scratch_words(uint64_t n) { return chain_status_word(n) + 2 * chain_blocks(n); }

hipError_t launch_batch(const uint8_t* arena, uint64_t arena_bytes,
                        const void* desc, uint32_t n, uint16_t* out,
                        uint32_t* partial, unsigned long long* err,
                        hipStream_t stream, uint64_t sizing_bytes = 0, uint32_t store = 0,
                        uint32_t* split = nullptr);

// Rewrite n device-resident descriptors' offsets relative to `bias` (empty
// descriptors get 0): the host pipeline's per-chunk table rebase.
hipError_t launch_rebase(void* desc, uint32_t n, uint64_t bias, hipStream_t stream);

// Batches of few descriptors averaging >= split_min_avg() bytes take the
// split kernel when launch_batch gets `split`: a scratch of split_words(n)
// u32, zeroed once at allocation (every launch leaves it zero).
constexpr uint64_t split_min_avg() { return 1u << 20; }
constexpr uint64_t split_words(uint64_t n) { return 2 * n; }

}  // namespace nsk
