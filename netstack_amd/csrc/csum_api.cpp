// csum_api.cpp — the C ABI of include/netstack_csum.h on top of the gfx950
// kernels.  Host-side work here is plumbing only: argument validation, the
// gather of tcpip/buffer views into a pinned, contiguous staging arena plus a
// descriptor table (the "device-staged layout" of north_star), H2D/D2H copies
// and launches.  Every checksum is computed on the GPU; there is no host
// fallback — a HIP failure is returned as a negative status.
#include <hip/hip_runtime_api.h>

#include <algorithm>
#include <atomic>
#include <condition_variable>
#include <cstdio>
#include <cstdlib>
#include <chrono>
#include <cstring>
#include <mutex>
#include <new>
#include <thread>
#include <vector>

#include "csum_kernels.h"
#include "host_logic.h"
#include "netstack_csum.h"

static_assert(sizeof(ns_pkt_desc) == 16, "ns_pkt_desc must be 16 bytes");
static_assert(sizeof(ns_seg) == 24, "ns_seg layout");
static_assert(sizeof(ns_piece) == 24, "ns_piece layout");
static_assert(sizeof(ns_pkt_buf) == 40, "ns_pkt_buf layout");

namespace {

using nsh::any_cont;
using nsh::clip_views;
using nsh::Piece;

constexpr uint64_t kDefaultStaging = 64ull << 20;
// Small host calls (bytes up to kStageBytes, below) run zero-copy: the kernel
// reads the table and the bytes from mapped pinned host memory over PCIe and
// writes the results there, so a small synchronous call is one CPU copy, one
// launch and one wait instead of three DMA operations, a launch and a wait
// (tools/latency.cc).

thread_local hipError_t g_last_hip = hipSuccess;

// Records the failing HIP call (ns_csum_last_hip_error) and, with
// NS_CSUM_DEBUG set in the environment, prints it.
int report_hip(hipError_t e, const char* expr, const char* file, int line);

#define HIP_TRY(expr)                                                        \
  do {                                                                       \
    hipError_t e__ = (expr);                                                 \
    if (e__ != hipSuccess) return report_hip(e__, #expr, __FILE__, __LINE__); \
  } while (0)

int map_hip_error(hipError_t e) {
  if (e == hipErrorOutOfMemory) return NS_ENOMEM;
  if (e == hipErrorNoDevice || e == hipErrorInvalidDevice) return NS_ENODEV;
  return NS_EHIP;
}

int report_hip(hipError_t e, const char* expr, const char* file, int line) {
  g_last_hip = e;
  static const bool dbg = std::getenv("NS_CSUM_DEBUG") != nullptr;
  if (dbg) std::fprintf(stderr, "netstack_csum: %s:%d: %s -> %s\n", file, line, expr, hipGetErrorString(e));
  return map_hip_error(e);
}

template <typename T>
struct DevBuf {
  T* p = nullptr;
  size_t cap = 0;  // elements
  // zero = clear a fresh allocation (the chained-batch scratch: see
  // csum_kernels.h).
  int ensure(size_t n, bool zero = false) {
    if (n <= cap) return NS_OK;
    if (p) (void)hipFree(p);
    p = nullptr;
    cap = 0;
    size_t want = std::max<size_t>(n, 1);
    HIP_TRY(hipMalloc(reinterpret_cast<void**>(&p), want * sizeof(T)));
    if (zero) HIP_TRY(hipMemset(p, 0, want * sizeof(T)));
    cap = want;
    return NS_OK;
  }
  void release() {
    if (p) (void)hipFree(p);
    p = nullptr;
    cap = 0;
  }
  // Stream-ordered growth for per-stream scratch: the old buffer is freed
  // after the work already queued on `s` (hipFreeAsync), the new one is
  // allocated and cleared in stream order.  Unlike hipFree, nothing waits for
  // the device, so a growing batch on one stream never stalls another.
  int ensure_async(size_t n, bool zero, hipStream_t s) {
    if (n <= cap) return NS_OK;
    if (p) (void)hipFreeAsync(p, s);
    p = nullptr;
    cap = 0;
    size_t want = std::max<size_t>(n, 1);
    HIP_TRY(hipMallocAsync(reinterpret_cast<void**>(&p), want * sizeof(T), s));
    if (zero) HIP_TRY(hipMemsetAsync(p, 0, want * sizeof(T), s));
    cap = want;
    return NS_OK;
  }
  void release_async(hipStream_t s) {
    if (p) (void)hipFreeAsync(p, s);
    p = nullptr;
    cap = 0;
  }
};

template <typename T, unsigned FLAGS = hipHostMallocDefault>
struct PinBuf {
  T* p = nullptr;
  T* dev = nullptr;  // the same memory as a device pointer (mapped)
  size_t cap = 0;
  int ensure(size_t n) {
    if (n <= cap) return NS_OK;
    if (p) (void)hipHostFree(p);
    p = dev = nullptr;
    cap = 0;
    size_t want = std::max<size_t>(n, 1);
    HIP_TRY(hipHostMalloc(reinterpret_cast<void**>(&p), want * sizeof(T), FLAGS));
    HIP_TRY(hipHostGetDevicePointer(reinterpret_cast<void**>(&dev), p, 0));
    cap = want;
    return NS_OK;
  }
  void release() {
    if (p) (void)hipHostFree(p);
    p = dev = nullptr;
    cap = 0;
  }
};

// Mapped, all-device pinned memory that the kernel reads and writes over PCIe
// with ordinary loads and stores (zero-copy).  It is coarse-grained
// (hipHostMallocNonCoherent): device writes become visible to the host at
// kernel completion, and host writes to a kernel at its dispatch.  That is
// all the zero-copy path needs — the host fills the table and bytes before
// the launch and reads results only after hipStreamSynchronize — but it is
// not safe for polling a buffer while a kernel runs.
using MappedPin = PinBuf<uint8_t, hipHostMallocMapped | hipHostMallocNonCoherent | hipHostMallocPortable>;
// Mapped, fine-grained (coherent) host memory: device stores reach it
// uncached, in order, so the host may poll it while kernels run.  A zero-copy
// pass writes its results here and then a completion word (from the checksum
// launch's last workgroup, nsk::ZcSignal, or a signal kernel behind a chained
// pass's fold), which the caller spins on instead of hipStreamSynchronize:
// the stream's own completion arrives ~10 us after the kernel's last store
// (tools/sync_probe.hip).
using CoherentPin = PinBuf<uint8_t, hipHostMallocMapped | hipHostMallocCoherent | hipHostMallocPortable>;

// What a zero-copy pass reads: its descriptor table and the bytes small
// calls gather.  On a large-BAR part (the whole VRAM mapped into the CPU's
// address space, hipDeviceAttributeIsLargeBar) they are fine-grained device
// memory the host writes through the BAR at the same address, so the
// kernel's dependent reads are local instead of PCIe round trips; elsewhere
// mapped host memory.  The host only ever writes these buffers (reads
// through the BAR are uncached and slow), and drains its write-combined
// stores (sfence) before the work is launched.
struct BarBuf {
  uint8_t* p = nullptr;    // host view
  uint8_t* dev = nullptr;  // device view (the same address in VRAM)
  size_t cap = 0;
  bool vram = false;
  MappedPin host;
  int ensure(size_t n, bool want_vram) {
    if (n <= cap) return NS_OK;
    release();
    if (want_vram) {
      void* q = nullptr;
      if (hipExtMallocWithFlags(&q, n, hipDeviceMallocFinegrained) == hipSuccess) {
        p = dev = static_cast<uint8_t*>(q);
        cap = n;
        vram = true;
        return NS_OK;
      }
      (void)hipGetLastError();
    }
    const int rc = host.ensure(n);
    if (rc != NS_OK) return rc;
    p = host.p;
    dev = host.dev;
    cap = n;
    return NS_OK;
  }
  void release() {
    if (vram && p) (void)hipFree(p);
    host.release();
    p = dev = nullptr;
    cap = 0;
    vram = false;
  }
};

// Chained-batch scratch (csum_kernels.h ChainScratch): partials + flags, and
// the fold statuses in a buffer of their own, zeroed once at allocation.
struct ChainBuf {
  DevBuf<uint32_t> part;
  DevBuf<uint64_t> status;
  int ensure(uint64_t n) {
    int rc = part.ensure((size_t)nsk::chain_scratch_words(n));
    if (rc == NS_OK) rc = status.ensure((size_t)nsk::chain_blocks(n), true);
    return rc;
  }
  int ensure_async(uint64_t n, hipStream_t s) {
    int rc = part.ensure_async((size_t)nsk::chain_scratch_words(n), false, s);
    if (rc == NS_OK) rc = status.ensure_async((size_t)nsk::chain_blocks(n), true, s);
    return rc;
  }
  nsk::ChainScratch get(bool walk = false) const { return nsk::ChainScratch{part.p, status.p, walk}; }
  void release() {
    part.release();
    status.release();
  }
  void release_async(hipStream_t s) {
    part.release_async(s);
    status.release_async(s);
  }
};

// Scratch of the device-resident API for one caller stream: chained batches
// and huge-descriptor splits on different streams of one context run
// concurrently, each on its own scratch (the same stream orders its own).
// The bookkeeping (keys, pins, LRU bound, release) is nsh::ScratchRegistry.
// `last` marks the stream's last launch that used the scratch, so the
// buffers can be freed after it even once the stream itself is gone
// (retire_scratch).
struct StreamScratch : nsh::ScratchSlot {
  ChainBuf chain;
  DevBuf<uint32_t> split;  // csum_split accumulators (zero between launches)
  DevBuf<uint16_t> txpay;  // ns_csum_tcp_tx: per-segment payload values between its passes
  // ns_csum_tcp_tx_multi: the calls' table on the device (stream-ordered:
  // one suffices) and a ring of pinned host copies, each with the event
  // after which its upload has run and it may be rewritten
  DevBuf<uint8_t> txtab;
  struct TabSlot {
    uint8_t* h = nullptr;
    size_t cap = 0;
    hipEvent_t ev = nullptr;
  };
  static constexpr uint32_t kTabSlots = 8;
  TabSlot tab[kTabSlots];
  uint32_t tab_next = 0;
  hipEvent_t last = nullptr;
  std::mutex mu;  // held while growing it and launching with it
};
constexpr size_t kMaxStreamScratch = 64;

// One small synchronous call's batch: `ndesc` descriptors over bytes
// [lo, lo + nbytes) of the caller's arena, staged in mapped memory whose
// device address is `dbytes` (= byte lo).
struct SmallReq {
  const uint8_t* dbytes = nullptr;
  uint64_t nbytes = 0, lo = 0;
  const ns_pkt_desc* desc = nullptr;
  uint32_t ndesc = 0;
  uint16_t* res = nullptr;
  bool chained = false;  // NS_DESC_CONT runs are chains (else the flag is ignored)
  int rc = NS_OK;
  std::atomic<bool> done{false};  // set (release) once rc and the results are in
  // bytes this request takes in a pass's table buffer (table + results)
  uint64_t table_bytes() const { return (uint64_t)ndesc * (sizeof(ns_pkt_desc) + 2) + 16; }
};

// A small call's bytes live in one staging buffer of kStageBytes leased from
// the context's pool for the duration of the call, so concurrent callers
// gather in parallel straight into memory the kernel reads.
constexpr uint64_t kStageBytes = 1ull << 20;
// A gather that outgrows its stage moves to a larger one leased from a second
// pool (powers of two up to kZeroCopyMax) and stays zero-copy; only beyond
// that does it take the DMA pipeline.  On MI355X (large BAR) a gather stage is
// device memory the host writes through the BAR at ~23 GB/s, where the DMA
// pipeline first gathers into pinned memory and then copies it: 2-4 MiB calls
// ran at 13-15 GB/s there (tools/crossover.cc, profiles/r04/crossover.json).
constexpr uint64_t kZeroCopyMax = 16ull << 20;
// A pass's [table | results] buffer; a pass takes queued requests while they fit.
constexpr uint64_t kPassTableBytes = 1ull << 20;
// The "arena" of a zero-copy pass is the address space: descriptors hold
// absolute device addresses (the kernel's per-tile windows take it from there).
constexpr uint64_t kWholeSpace = 1ull << 60;

// Diagnostic counters of one context (ns_csum_get_stats), updated lock-free.
struct StatCounters {
  std::atomic<uint64_t> calls{0}, call_ns_max{0}, lock_ns_max{0}, zc_passes{0}, zc_late{0}, zc_pass_ns_max{0},
      growths{0}, growth_ns_total{0}, growth_ns_max{0}, retires{0}, retire_ns_max{0}, stage_allocs{0},
      stage_alloc_ns_max{0};
};

uint64_t now_ns() {
  return (uint64_t)std::chrono::duration_cast<std::chrono::nanoseconds>(
             std::chrono::steady_clock::now().time_since_epoch())
      .count();
}

void bump_max(std::atomic<uint64_t>& m, uint64_t v) {
  uint64_t c = m.load(std::memory_order_relaxed);
  while (v > c && !m.compare_exchange_weak(c, v, std::memory_order_relaxed)) {
  }
}

}  // namespace

// The host-batch pipeline's shape: chunks in flight and descriptors per chunk
// (cfg3, 1M x 64 B, two slots with a D2H copy per chunk: 64K 3.11 ms, 128K
// 2.18, 256K 2.16, 512K 2.52 ms per call).  Results written straight to
// mapped memory, 128K-descriptor chunks (round 5, profiles/r05/host/): 2 /
// 3 / 4 slots 1.86 / 1.80 / 1.72 ms per call, against 2.03 / 1.90 / 1.88 ms
// with the D2H copy.
constexpr uint32_t kMaxHostSlots = 4;
constexpr uint32_t kHostSlots = 4;
constexpr uint32_t kHostChunkDesc = 1u << 17;

struct ns_csum_ctx {
  int device = 0;
  bool fold_walk = false;  // NS_OPT_FOLD_WALK
  uint64_t staging = kDefaultStaging;
  // The host-batch DMA pipeline (ns_csum_batch_host, gathers above
  // kZeroCopyMax): its streams, slots and g_arena, under pmu.  It never
  // takes mu, so a 1.5 GB host batch does not hold up the zero-copy passes
  // of small synchronous calls (a 29 ms head-of-line block).
  // nslots chunks in flight (one stream each), chunk_desc descriptors per
  // chunk at most: set once at init (NS_CSUM_HOST_SLOTS / _CHUNK, A/B only).
  uint32_t nslots = kHostSlots;
  uint32_t chunk_desc = kHostChunkDesc;
  hipStream_t stream[kMaxHostSlots] = {};
  hipEvent_t done[kMaxHostSlots] = {};
  std::mutex pmu;
  // Zero-copy passes and ns_csum_sync run on zstream, a stream of their own
  // at the greatest priority like the pipeline's, under mu.  That puts it on
  // a hardware queue apart from callers' (normal-priority) streams, but with
  // four pipeline streams at that priority and GPU_MAX_HW_QUEUES = 4 it
  // shares one with a pipeline stream: a pass may run behind one chunk's
  // copy and kernel there.  Measured (profiles/r06/latency/, 1 KiB passes
  // during 0.6 GB host TX calls): longest pass 29.5-81.8 us with 4 slots,
  // 33.3-36.3 us with 3 (NS_CSUM_HOST_SLOTS=3), no late pass either way;
  // tests/test_gpu_tx_host.py asserts the longest pass under 1 ms.
  hipStream_t zstream = nullptr;
  unsigned long long* d_err = nullptr;
  std::mutex mu;  // guards everything below but the pipeline's state

  // device-resident API scratch, one per caller stream (allocated on first
  // use), under its own lock: growing one never holds up synchronous calls
  nsh::ScratchRegistry<StreamScratch> scratch{kMaxStreamScratch};
  std::mutex rmu;                // guards retire
  hipStream_t retire = nullptr;  // frees retired scratch after its last use
  // ns_csum_sync's exchanged error count (mapped: written by take_err)
  MappedPin err_taken;
  ChainBuf z_chain;  // a chained zero-copy pass's scratch
  // host-path slots (nslots in flight; pmu)
  DevBuf<uint8_t> d_arena[kMaxHostSlots];
  DevBuf<ns_pkt_desc> d_desc[kMaxHostSlots];
  DevBuf<uint16_t> d_out[kMaxHostSlots];
  ChainBuf d_chain[kMaxHostSlots];
  PinBuf<ns_pkt_desc> h_desc[kMaxHostSlots];
  // results: written by the kernel straight into mapped pinned memory (no
  // D2H copy on the DMA engine; NS_CSUM_HOST_D2H=1 copies them instead, A/B)
  PinBuf<uint16_t, hipHostMallocMapped | hipHostMallocNonCoherent | hipHostMallocPortable> h_out[kMaxHostSlots];
  bool host_d2h = false;
  // ns_csum_tcp_tx_host: each slot's geometry table (TxGeo[] + first[]),
  // pinned for its upload and on the device
  PinBuf<uint8_t> h_txtab[kMaxHostSlots];
  DevBuf<uint8_t> d_txtab[kMaxHostSlots];
  // ns_csum_rx_ring_host: each slot's received lengths on the device and its
  // verdicts (mapped, written by the kernel; the sums go to h_out)
  DevBuf<uint32_t> d_len[kMaxHostSlots];
  MappedPin h_verd[kMaxHostSlots];
  // the small host paths' results and completion word (coherent: written
  // through, visible once the signal is; pmu)
  CoherentPin p_res;
  CoherentPin p_done;
  uint32_t p_seq = 0;
  // zero-copy pass buffers for small calls: the table (read by the kernel),
  // the results and the completion word (written by it)
  BarBuf z_buf;
  bool bar_table = false;  // large BAR: z_buf in device memory
  CoherentPin z_res;
  CoherentPin z_done;
  DevBuf<uint32_t> z_ctr;  // a self-signalling pass's workgroup counter (zero between passes)
  uint32_t z_seq = 0;
  // flat combining of concurrent small calls (nsh::FlatCombiner)
  nsh::FlatCombiner<SmallReq> combiner{kPassTableBytes};
  // the pool of staging buffers small calls gather into (BarBuf: device
  // memory behind the BAR where possible), and the pool of mapped host
  // buffers callers acquire (ns_csum_stage_acquire); guarded by qmu
  std::mutex qmu;
  std::vector<BarBuf*> gstage_free;
  std::vector<BarBuf*> gstage_all;
  std::vector<BarBuf*> gbig_free;  // gather stages above kStageBytes (in gstage_all too)
  std::vector<MappedPin*> stage_free;
  std::vector<MappedPin*> stage_all;
  std::vector<MappedPin*> big_free;  // pooled caller stages above kStageBytes
  std::vector<MappedPin*> leased;    // stages a caller holds (ns_csum_stage_acquire)
  // gather staging for the VectorisedView entry points above kZeroCopyMax (pmu)
  PinBuf<uint8_t> g_arena;
  std::vector<ns_pkt_desc> g_desc;
  StatCounters st;
  // ns_csum_set_tx_tuning's knobs (A/B and tests), read by ns_csum_tcp_tx
  std::atomic<uint32_t> tx_variant{0}, tx_tile{0}, tx_htile{0}, tx_passes{0};
};

namespace {

// Frees a scratch entry the registry dropped: its buffers are freed on the
// context's retire stream after the last launch that used them (its event),
// so neither the host nor the device waits, and the entry's own stream may
// already be destroyed.
void retire_scratch(ns_csum_ctx* ctx, StreamScratch* sc) {
  const uint64_t t0 = now_ns();
  std::lock_guard<std::mutex> lk(ctx->rmu);
  if (!ctx->retire && hipStreamCreateWithFlags(&ctx->retire, hipStreamNonBlocking) != hipSuccess) ctx->retire = nullptr;
  if (ctx->retire && hipStreamWaitEvent(ctx->retire, sc->last, 0) == hipSuccess) {
    sc->chain.release_async(ctx->retire);
    sc->split.release_async(ctx->retire);
    sc->txpay.release_async(ctx->retire);
    sc->txtab.release_async(ctx->retire);
  } else {  // no retire stream: free once its last launch is done
    (void)hipGetLastError();
    (void)hipEventSynchronize(sc->last);
    sc->chain.release();
    sc->split.release();
    sc->txpay.release();
    sc->txtab.release();
  }
  for (StreamScratch::TabSlot& t : sc->tab) {  // host memory: free once its last copy has run
    if (t.ev) (void)hipEventSynchronize(t.ev);
    if (t.h) (void)hipHostFree(t.h);
    if (t.ev) (void)hipEventDestroy(t.ev);
  }
  (void)hipEventDestroy(sc->last);
  delete sc;
  ctx->st.retires.fetch_add(1, std::memory_order_relaxed);
  bump_max(ctx->st.retire_ns_max, now_ns() - t0);
}

// Times one synchronous entry point, entry to return (ns_csum_stats.calls,
// call_ns_max).
struct CallClock {
  ns_csum_ctx* ctx;
  uint64_t t0;
  explicit CallClock(ns_csum_ctx* c) : ctx(c), t0(now_ns()) {}
  ~CallClock() {
    ctx->st.calls.fetch_add(1, std::memory_order_relaxed);
    bump_max(ctx->st.call_ns_max, now_ns() - t0);
  }
  CallClock(const CallClock&) = delete;
  CallClock& operator=(const CallClock&) = delete;
};

// Times a staging allocation (a pool was empty).
struct AllocClock {
  ns_csum_ctx* ctx;
  uint64_t t0;
  explicit AllocClock(ns_csum_ctx* c) : ctx(c), t0(now_ns()) {}
  ~AllocClock() {
    ctx->st.stage_allocs.fetch_add(1, std::memory_order_relaxed);
    bump_max(ctx->st.stage_alloc_ns_max, now_ns() - t0);
  }
};

StreamScratch* make_scratch() {
  StreamScratch* sc = new (std::nothrow) StreamScratch();
  if (sc && hipEventCreateWithFlags(&sc->last, hipEventDisableTiming) != hipSuccess) {
    (void)hipGetLastError();
    delete sc;
    sc = nullptr;
  }
  return sc;
}

nsh::ScratchKey scratch_key(hipStream_t s) {
  nsh::ScratchKey k;
  k.stream = (const void*)s;
  if (s == hipStreamPerThread) k.thread = std::this_thread::get_id();
  return k;
}

struct DeviceGuard {
  int prev = -1;
  explicit DeviceGuard(int dev) {
    if (hipGetDevice(&prev) != hipSuccess) prev = -1;
    if (prev != dev) (void)hipSetDevice(dev);
  }
  ~DeviceGuard() {
    int cur = -1;
    if (prev >= 0 && hipGetDevice(&cur) == hipSuccess && cur != prev) (void)hipSetDevice(prev);
  }
};

// Validates a host table against its arena and returns the byte span its
// non-empty descriptors cover ([0, 0) if none).
int table_span(const ns_pkt_desc* d, uint32_t n, uint64_t arena_bytes, uint64_t* lo, uint64_t* hi) {
  uint64_t l = UINT64_MAX, h = 0;
  for (uint32_t i = 0; i < n; ++i) {
    const uint64_t off = d[i].off, len = d[i].len;
    if (off > arena_bytes || len > arena_bytes - off) return NS_ERANGE;
    if (len) {
      l = std::min(l, off);
      h = std::max(h, off + len);
    }
  }
  if (l == UINT64_MAX) l = h = 0;
  *lo = l;
  *hi = h;
  return NS_OK;
}

bool zero_copy_enabled() {
  // NS_CSUM_NO_ZERO_COPY=1 forces the DMA pipeline (A/B diagnostics only).
  static const bool off = std::getenv("NS_CSUM_NO_ZERO_COPY") != nullptr;
  return !off;
}

// Zero-copy pass over one or more small requests (caller holds ctx->mu and
// the device guard): one table of all their descriptors with absolute device
// addresses into their mapped staging, results beside it, one launch that
// reads both over PCIe, one wait.  Requests never share a NS_DESC_CONT run: a
// request's first descriptor is made a run head.
int run_zero_copy(ns_csum_ctx* ctx, SmallReq* const* reqs, size_t nreq) {
  uint64_t nd = 0, nb = 0;
  bool chained = false;
  for (size_t r = 0; r < nreq; ++r) {
    nd += reqs[r]->ndesc;
    nb += reqs[r]->nbytes;
    chained = chained || reqs[r]->chained;
  }
  if (nd == 0) return NS_OK;
  int rc;
  if ((rc = ctx->z_buf.ensure(std::max<uint64_t>(kPassTableBytes, nd * sizeof(ns_pkt_desc)), ctx->bar_table)) !=
      NS_OK)
    return rc;
  if ((rc = ctx->z_res.ensure(std::max<uint64_t>(kPassTableBytes / 8, nd * 2))) != NS_OK) return rc;
  if (ctx->z_done.cap == 0) {  // zeroed once: no stale word may equal a pass's sequence number
    if ((rc = ctx->z_done.ensure(64)) != NS_OK) return rc;
    __atomic_store_n(reinterpret_cast<uint32_t*>(ctx->z_done.p), 0u, __ATOMIC_RELEASE);
  }
  if (chained && (rc = ctx->z_chain.ensure(nd)) != NS_OK) return rc;
  if ((rc = ctx->z_ctr.ensure(1, true)) != NS_OK) return rc;
  uint8_t* z = ctx->z_buf.p;
  ns_pkt_desc* zd = reinterpret_cast<ns_pkt_desc*>(z);
  uint64_t k = 0;
  for (size_t r = 0; r < nreq; ++r) {
    const SmallReq& q = *reqs[r];
    const uint64_t base = (uint64_t)(uintptr_t)q.dbytes;
    for (uint32_t i = 0; i < q.ndesc; ++i, ++k) {
      // built in a register and written once: the table may be device memory
      // behind the BAR, which the host must never read back
      ns_pkt_desc d = q.desc[i];
      d.off = d.len ? base + (d.off - q.lo) : 0;
      if (!q.chained) {
        d.flags &= (uint16_t)~NS_DESC_CONT;  // independent in an unchained batch
      } else if (i == 0 && (d.flags & NS_DESC_CONT)) {
        // A batch's first descriptor heads its run even when flagged CONT
        // (with initial 0, fold_scan): keep that inside a combined pass.
        d.flags &= (uint16_t)~NS_DESC_CONT;
        d.initial = 0;
      }
      zd[k] = d;
    }
  }
  // BAR writes are write-combined: drain them before the launch's doorbell.
  __builtin_ia32_sfence();
  hipStream_t s = ctx->zstream;
  // Completion: the pass's sequence number lands in coherent host memory once
  // every result is there — stored by the checksum launch's last workgroup
  // (unchained passes: the results are written through, nsk::ZcSignal) or by
  // a one-wave kernel behind the fold pass (chained).  The caller spins for
  // it, and only if it is late (a fault, or a busy device) waits on the
  // stream itself, which also reports a failed kernel.
  uint32_t seq = ++ctx->z_seq;
  if (seq == 0) seq = ++ctx->z_seq;
  uint32_t* done = reinterpret_cast<uint32_t*>(ctx->z_done.p);
  uint32_t* done_dev = reinterpret_cast<uint32_t*>(ctx->z_done.dev);
  // NS_CSUM_SIGNAL_KERNEL=1: the signal kernel for unchained passes too (A/B only)
  static const bool sig_kernel = std::getenv("NS_CSUM_SIGNAL_KERNEL") != nullptr;
  const bool self = !chained && !sig_kernel;
  nsk::ZcSignal zc{};
  if (self) zc = nsk::ZcSignal{ctx->z_ctr.p, done_dev, seq};
  HIP_TRY(nsk::launch_batch(nullptr, kWholeSpace, ctx->z_buf.dev, (uint32_t)nd,
                            reinterpret_cast<uint16_t*>(ctx->z_res.dev),
                            chained ? ctx->z_chain.get(ctx->fold_walk) : nsk::ChainScratch{}, ctx->d_err, s,
                            std::max<uint64_t>(nb, 1), 0, nullptr, zc));
  if (!self) HIP_TRY(nsk::launch_signal(done_dev, seq, s));
  ctx->st.zc_passes.fetch_add(1, std::memory_order_relaxed);
  const uint64_t pass_t0 = now_ns();
  const auto t0 = std::chrono::steady_clock::now();
  for (uint32_t spin = 0; __atomic_load_n(done, __ATOMIC_ACQUIRE) != seq; ++spin) {
    if ((spin & 255u) == 255u && std::chrono::steady_clock::now() - t0 > std::chrono::milliseconds(2)) {
      ctx->st.zc_late.fetch_add(1, std::memory_order_relaxed);
      HIP_TRY(hipStreamSynchronize(s));
      if (__atomic_load_n(done, __ATOMIC_ACQUIRE) != seq) {
        // The pass ended without its last workgroup's word: its counter may
        // be left nonzero, which would keep every later pass from
        // signalling.  Reset it before the next pass can run.
        if (self) {
          HIP_TRY(hipMemsetAsync(ctx->z_ctr.p, 0, sizeof(uint32_t), s));
          HIP_TRY(hipStreamSynchronize(s));
        }
        if (std::getenv("NS_CSUM_DEBUG")) std::fprintf(stderr, "netstack_csum: pass %u signalled no completion\n", seq);
        return NS_EHIP;
      }
      break;
    }
  }
  bump_max(ctx->st.zc_pass_ns_max, now_ns() - pass_t0);
  const uint16_t* res = reinterpret_cast<const uint16_t*>(ctx->z_res.p);
  for (size_t r = 0; r < nreq; ++r) {
    std::memcpy(reqs[r]->res, res, (size_t)reqs[r]->ndesc * 2);
    res += reqs[r]->ndesc;
  }
  return NS_OK;
}

// Lease a mapped staging buffer of kStageBytes from the context's pool
// (ns_csum_stage_acquire; ns_csum_stage_release returns it).
MappedPin* lease_stage(ns_csum_ctx* ctx, int* rc) {
  {
    std::lock_guard<std::mutex> ql(ctx->qmu);
    if (!ctx->stage_free.empty()) {
      MappedPin* b = ctx->stage_free.back();
      ctx->stage_free.pop_back();
      return b;
    }
  }
  AllocClock clk(ctx);
  MappedPin* b = new (std::nothrow) MappedPin();
  if (!b) {
    *rc = NS_ENOMEM;
    return nullptr;
  }
  {
    DeviceGuard g(ctx->device);
    if ((*rc = b->ensure(kStageBytes)) != NS_OK) {
      delete b;
      return nullptr;
    }
  }
  std::lock_guard<std::mutex> ql(ctx->qmu);
  ctx->stage_all.push_back(b);
  return b;
}

// Lease / return a gather stage (device memory behind the BAR on large-BAR
// parts) of at least `bytes`: kStageBytes from the context's pool, or above
// that the smallest pooled big stage that fits (new ones are powers of two).
BarBuf* lease_gather_stage(ns_csum_ctx* ctx, int* rc, uint64_t bytes = kStageBytes) {
  uint64_t cap = kStageBytes;
  {
    std::lock_guard<std::mutex> ql(ctx->qmu);
    if (bytes <= kStageBytes) {
      if (!ctx->gstage_free.empty()) {
        BarBuf* b = ctx->gstage_free.back();
        ctx->gstage_free.pop_back();
        return b;
      }
    } else {
      size_t best = ctx->gbig_free.size();
      for (size_t i = 0; i < ctx->gbig_free.size(); ++i)
        if (ctx->gbig_free[i]->cap >= bytes && (best == ctx->gbig_free.size() || ctx->gbig_free[i]->cap < ctx->gbig_free[best]->cap))
          best = i;
      if (best < ctx->gbig_free.size()) {
        BarBuf* b = ctx->gbig_free[best];
        ctx->gbig_free.erase(ctx->gbig_free.begin() + (long)best);
        return b;
      }
      while (cap < bytes) cap *= 2;
    }
  }
  AllocClock clk(ctx);
  BarBuf* b = new (std::nothrow) BarBuf();
  if (!b) {
    *rc = NS_ENOMEM;
    return nullptr;
  }
  {
    DeviceGuard g(ctx->device);
    if ((*rc = b->ensure(cap, ctx->bar_table)) != NS_OK) {
      delete b;
      return nullptr;
    }
  }
  std::lock_guard<std::mutex> ql(ctx->qmu);
  ctx->gstage_all.push_back(b);
  return b;
}

void return_gather_stage(ns_csum_ctx* ctx, BarBuf* b) {
  if (!b) return;
  std::lock_guard<std::mutex> ql(ctx->qmu);
  (b->cap == kStageBytes ? ctx->gstage_free : ctx->gbig_free).push_back(b);
}

// Flat combining of concurrent small synchronous calls (nsh::FlatCombiner):
// concurrent callers' requests run as one zero-copy pass.  Each caller has
// already gathered its bytes into its own leased staging, so the only serial
// host work per request is copying its descriptors.  Results are identical
// to separate calls (descriptors are independent; chains never cross
// requests).
int submit_small(ns_csum_ctx* ctx, SmallReq* req) {
  // This thread's gather may have gone to device memory through the BAR:
  // drain its write-combined stores before another thread launches the pass.
  __builtin_ia32_sfence();
  return ctx->combiner.submit(req, [ctx](SmallReq* const* reqs, size_t nreq) {
    const uint64_t t0 = now_ns();
    std::lock_guard<std::mutex> lk(ctx->mu);
    bump_max(ctx->st.lock_ns_max, now_ns() - t0);
    DeviceGuard g(ctx->device);
    return run_zero_copy(ctx, reqs, nreq);
  });
}

// Host batch core, caller holds ctx->pmu and the device guard.  Pipelines
// chunks of the descriptor table over the context's slots/streams: H2D of
// chunk k+1 overlaps the kernel of chunk k.  Chunks never split a
// NS_DESC_CONT run.

// Whether [p, p + bytes) is page-locked host memory the DMA engines read
// directly (hipHostMalloc, hipHostRegister, torch pin_memory).  A pageable
// pointer makes hipPointerGetAttributes fail; that error is cleared so no
// later hipGetLastError sees it.
bool host_pinned(const void* p, uint64_t bytes) {
  if (!p || !bytes) return false;
  for (const void* q : {p, static_cast<const void*>(static_cast<const uint8_t*>(p) + bytes - 1)}) {
    hipPointerAttribute_t a{};
    if (hipPointerGetAttributes(&a, q) != hipSuccess) {
      (void)hipGetLastError();
      return false;
    }
    if (a.type != hipMemoryTypeHost) return false;
  }
  return true;
}

int run_host_batch(ns_csum_ctx* ctx, const uint8_t* h_arena, uint64_t arena_bytes,
                   const ns_pkt_desc* h_desc, uint32_t n, uint16_t* h_out,
                   bool chained) {
  if (n == 0) return NS_OK;
  const uint64_t budget = ctx->staging;
  // A pinned table goes to the device straight from the caller's memory; a
  // pageable one is copied into pinned staging chunk by chunk first (1M x
  // 64 B: that copy, 16 MB per call on one core, was as long as the chunks'
  // DMA).
  const bool desc_pinned = host_pinned(h_desc, (uint64_t)n * sizeof(ns_pkt_desc));
  struct Pending {
    bool live = false;
    uint32_t first = 0, count = 0;
  } pend[kMaxHostSlots];
  const uint32_t nslots = ctx->nslots;
  // Drain whatever is in flight (on an error return too: the staging
  // buffers must be idle before the next call reuses them).
  auto drain = [&](int slot) -> int {
    for (uint32_t s = 0; s < nslots; ++s) {
      const int sl = (int)((slot + s) % nslots);
      if (pend[sl].live) {
        HIP_TRY(hipEventSynchronize(ctx->done[sl]));
        std::memcpy(h_out + pend[sl].first, ctx->h_out[sl].p, pend[sl].count * sizeof(uint16_t));
        pend[sl].live = false;
      }
    }
    return NS_OK;
  };
  uint32_t k = 0;
  int slot = 0;
  while (k < n) {
    // The next chunk (nsh::cut_chunk): at most kHostChunkDesc descriptors
    // and `budget` bytes of span, never inside a chained run; descriptors are
    // range-checked on the way.  1M x 64 B: 4.27 ms -> 2.15 ms per call with
    // this, the skipped span pass and the device-side table rebase
    // (profiles/r01/bench_host3.json).
    uint32_t cut = k;
    uint64_t cut_lo = 0, cut_hi = 0;
    const int crc = nsh::cut_chunk(h_desc, n, k, arena_bytes, budget, ctx->chunk_desc, chained, &cut, &cut_lo,
                                   &cut_hi);
    if (crc != NS_OK) {
      const int rc = drain(slot);
      return rc != NS_OK ? rc : crc;
    }
    const uint32_t cnt = cut - k;
    const uint64_t span = cut_hi - cut_lo;

    // Retire the slot's previous chunk before reusing its staging.
    if (pend[slot].live) {
      HIP_TRY(hipEventSynchronize(ctx->done[slot]));
      std::memcpy(h_out + pend[slot].first, ctx->h_out[slot].p, pend[slot].count * sizeof(uint16_t));
      pend[slot].live = false;
    }
    // Everything that can fail for this chunk; on failure the other slot's
    // transfers are drained before returning (the next call reuses the
    // pinned buffers they read and write).
    auto enqueue = [&]() -> int {
      int rc;
      if ((rc = ctx->d_arena[slot].ensure(std::max<uint64_t>(span, 16))) != NS_OK) return rc;
      if ((rc = ctx->d_desc[slot].ensure(cnt)) != NS_OK) return rc;
      if (ctx->host_d2h && (rc = ctx->d_out[slot].ensure(cnt)) != NS_OK) return rc;
      if (!desc_pinned && (rc = ctx->h_desc[slot].ensure(cnt)) != NS_OK) return rc;
      if ((rc = ctx->h_out[slot].ensure(cnt)) != NS_OK) return rc;
      if (chained && (rc = ctx->d_chain[slot].ensure(cnt)) != NS_OK) return rc;
      // The table goes over verbatim (from the caller's pinned table, or one
      // memcpy into pinned staging) and is rebased to the chunk on the
      // device: a per-descriptor rewrite on the CPU was the limit of
      // small-packet batches.
      const ns_pkt_desc* hd = h_desc + k;
      if (!desc_pinned) {
        std::memcpy(ctx->h_desc[slot].p, hd, (size_t)cnt * sizeof(ns_pkt_desc));
        hd = ctx->h_desc[slot].p;
      }
      hipStream_t s = ctx->stream[slot];
      if (span) HIP_TRY(hipMemcpyAsync(ctx->d_arena[slot].p, h_arena + cut_lo, span, hipMemcpyHostToDevice, s));
      HIP_TRY(hipMemcpyAsync(ctx->d_desc[slot].p, hd, cnt * sizeof(ns_pkt_desc), hipMemcpyHostToDevice, s));
      HIP_TRY(nsk::launch_rebase(ctx->d_desc[slot].p, cnt, cut_lo, s));
      // The results go straight to mapped host memory: a D2H copy would sit
      // on the DMA engine's ring waiting for this kernel, and every later
      // chunk's H2D copies queue behind it (a rocprofv3 copy trace of cfg3
      // showed the slots' streams fully serialised that way).
      uint16_t* dst = ctx->host_d2h ? ctx->d_out[slot].p : ctx->h_out[slot].dev;
      HIP_TRY(nsk::launch_batch(ctx->d_arena[slot].p, span, ctx->d_desc[slot].p, cnt, dst,
                                chained ? ctx->d_chain[slot].get(ctx->fold_walk) : nsk::ChainScratch{}, ctx->d_err, s));
      if (ctx->host_d2h)
        HIP_TRY(hipMemcpyAsync(ctx->h_out[slot].p, ctx->d_out[slot].p, cnt * sizeof(uint16_t), hipMemcpyDeviceToHost,
                               s));
      HIP_TRY(hipEventRecord(ctx->done[slot], s));
      return NS_OK;
    };
    const int rc = enqueue();
    if (rc != NS_OK) {
      (void)drain(slot);
      return rc;
    }
    pend[slot].live = true;
    pend[slot].first = k;
    pend[slot].count = cnt;
    k = cut;
    slot = (int)((slot + 1) % nslots);
  }
  return drain(slot);
}

inline void put_be16(uint8_t* p, uint32_t v) {
  p[0] = (uint8_t)(v >> 8);
  p[1] = (uint8_t)v;
}

// ns_csum_tcp_tx_host's pipeline over nsh::tx_host_plan's chunks, nslots in
// flight on the host pipeline's streams.  Per chunk: one H2D copy per merged
// byte range into the slot's staging, the geometry table, and one
// tcp_tx_multi launch (fields-only: its stores stay in the staging) whose sums
// go straight to mapped pinned memory.  When a chunk is done the host writes
// its fields into the caller's slots from those sums, the values the kernel
// stores (2 x 2 B per segment instead of copying the slots back), while the
// later chunks are in flight.
// A finished chunk's fields, written into the caller's slots from the sums
// the kernel left in `res` (the values it stores), and its sums to h_out.
void patch_tx_fields(const nsh::TxHostPlan& plan, const nsh::TxChunk& c, const uint16_t* res, uint8_t* h_arena,
                     uint16_t* h_out) {
  for (uint32_t j = c.p0; j < c.p0 + c.np; ++j) {
    const nsh::TxPiece& q = plan.pieces[j];
    const uint16_t* r = res + 2 * (q.out0 - c.out0);
    uint8_t* s = h_arena + q.t.hdr_off;
    for (uint64_t i = 0; i < q.nseg; ++i, s += q.t.slot) {
      if (q.mode & nsk::kTxIp) put_be16(s + q.t.ip_at + 10u, ~r[2 * i] & 0xFFFFu);
      if (q.mode & nsk::kTxTcpFull) put_be16(s + q.t.tcp_at + 16u, ~r[2 * i + 1] & 0xFFFFu);
      if (q.mode & nsk::kTxTcpPartial) put_be16(s + q.t.tcp_at + 16u, r[2 * i + 1]);
    }
    if (h_out) std::memcpy(h_out + 2 * q.out0, r, 4 * q.nseg);
  }
}

// Chunk c's geometry table for tcp_tx_multi over staging at device address
// `base`, sums to `out`: calls[np] and first[np + 1], the launch shape; the
// grid (0: too many tiles).
uint32_t tx_chunk_table(const nsh::TxHostPlan& plan, const nsh::TxChunk& c, uint64_t base, uint16_t* out,
                        std::vector<nsk::TxGeo>* calls, std::vector<uint32_t>* first, nsk::TxGeo* launch) {
  calls->assign(c.np, nsk::TxGeo{});
  for (uint32_t j = 0; j < c.np; ++j) {
    const nsh::TxPiece& q = plan.pieces[c.p0 + j];
    nsk::TxGeo& geo = (*calls)[j];
    geo.hdr = base + plan.map(c, q.t.hdr_off);
    // a payload only full-mode pieces read (and upload)
    geo.pay = (q.mode & nsk::kTxTcpFull) ? base + plan.map(c, q.t.pay_off) : geo.hdr;
    geo.size = q.t.size;
    geo.n = q.nseg;
    geo.mss = q.t.mss;
    geo.slot = q.t.slot;
    geo.ip_at = q.t.ip_at;
    geo.ip_len = q.t.ip_len;
    geo.tcp_at = q.t.tcp_at;
    geo.tcp_len = q.t.tcp_len;
    geo.addr_sum = q.t.addr_sum;
    geo.proto = q.t.protocol;
    geo.mode = q.mode | nsk::kTxFieldsOnly;
    geo.out = out + 2 * (q.out0 - c.out0);
  }
  first->assign(c.np + 1, 0);
  *launch = nsk::TxGeo{};
  return nsk::tx_multi_prepare(calls->data(), c.np, launch, first->data());
}

// Host TX calls whose bytes and table fit kHostSmallBytes take no DMA: the
// ranges and the table are written through the BAR into a leased gather
// stage (fine-grained VRAM on large-BAR parts), one launch reads them there
// and writes its sums to mapped memory, then one wait, as the small checksum
// calls do.  Above that size the DMA pipeline's ~55 GB/s beats the BAR's ~23.
constexpr uint64_t kHostSmallBytes = 1ull << 20;

// Completes a small host-path launch on stream s (pmu held): a one-wave
// kernel behind it stores this call's sequence number into coherent host
// memory and the caller spins on that word, as the zero-copy passes do (the
// stream's own completion arrives some microseconds later).
// Past 2 ms it waits on the stream, which also reports a failed kernel.
int wait_small(ns_csum_ctx* ctx, hipStream_t s) {
  int rc;
  if (ctx->p_done.cap == 0) {  // zeroed once: no stale word may equal a sequence number
    if ((rc = ctx->p_done.ensure(64)) != NS_OK) return rc;
    __atomic_store_n(reinterpret_cast<uint32_t*>(ctx->p_done.p), 0u, __ATOMIC_RELEASE);
  }
  uint32_t seq = ++ctx->p_seq;
  if (seq == 0) seq = ++ctx->p_seq;
  uint32_t* done = reinterpret_cast<uint32_t*>(ctx->p_done.p);
  HIP_TRY(nsk::launch_signal(reinterpret_cast<uint32_t*>(ctx->p_done.dev), seq, s));
  const auto t0 = std::chrono::steady_clock::now();
  for (uint32_t spin = 0; __atomic_load_n(done, __ATOMIC_ACQUIRE) != seq; ++spin) {
    if ((spin & 255u) == 255u && std::chrono::steady_clock::now() - t0 > std::chrono::milliseconds(2)) {
      ctx->st.zc_late.fetch_add(1, std::memory_order_relaxed);  // counted like a late zero-copy pass
      HIP_TRY(hipStreamSynchronize(s));
      if (__atomic_load_n(done, __ATOMIC_ACQUIRE) != seq) return NS_EHIP;
      break;
    }
  }
  return NS_OK;
}

int run_tx_small(ns_csum_ctx* ctx, uint8_t* h_arena, const nsh::TxHostPlan& plan, uint16_t* h_out) {
  const nsh::TxChunk& c = plan.chunks[0];
  int rc = NS_OK;
  if ((rc = ctx->p_res.ensure(4 * c.nout)) != NS_OK) return rc;
  uint16_t* res = reinterpret_cast<uint16_t*>(ctx->p_res.p);
  const uint64_t tab_at = (c.staging + 255) & ~255ull;
  const size_t tab = ((size_t)c.np * sizeof(nsk::TxGeo) + 15) & ~(size_t)15;
  const uint64_t need = tab_at + tab + ((size_t)c.np + 1) * sizeof(uint32_t);
  BarBuf* st = lease_gather_stage(ctx, &rc, need);
  if (!st) return rc;
  for (uint32_t j = c.r0; j < c.r0 + c.nr; ++j) {
    const nsh::TxRange& r = plan.ranges[j];
    std::memcpy(st->p + r.at, h_arena + r.lo, r.hi - r.lo);
  }
  std::vector<nsk::TxGeo> calls;
  std::vector<uint32_t> first;
  nsk::TxGeo launch{};
  const uint32_t grid = tx_chunk_table(plan, c, (uint64_t)(uintptr_t)st->dev,
                                       reinterpret_cast<uint16_t*>(ctx->p_res.dev), &calls, &first, &launch);
  if (grid == 0) {
    return_gather_stage(ctx, st);
    return NS_EINVAL;
  }
  // written once, never read back (the stage may be VRAM behind the BAR)
  std::memcpy(st->p + tab_at, calls.data(), (size_t)c.np * sizeof(nsk::TxGeo));
  std::memcpy(st->p + tab_at + tab, first.data(), first.size() * sizeof(uint32_t));
  __builtin_ia32_sfence();  // drain the write-combined BAR stores before the launch
  hipStream_t s = ctx->stream[0];
  const hipError_t e = nsk::launch_tcp_tx_multi(launch, grid, reinterpret_cast<const nsk::TxGeo*>(st->dev + tab_at),
                                                reinterpret_cast<const uint32_t*>(st->dev + tab_at + tab), c.np, s);
  rc = e == hipSuccess ? wait_small(ctx, s) : report_hip(e, "run_tx_small", __FILE__, __LINE__);
  return_gather_stage(ctx, st);
  if (rc != NS_OK) return rc;
  patch_tx_fields(plan, c, res, h_arena, h_out);
  return NS_OK;
}

int run_tx_host(ns_csum_ctx* ctx, uint8_t* h_arena, const nsh::TxHostPlan& plan, uint16_t* h_out) {
  if (plan.chunks.size() == 1 && zero_copy_enabled()) {
    // (within the context's staging budget too: a context created with a
    // small budget sends everything through the pipeline)
    const nsh::TxChunk& c = plan.chunks[0];
    const uint64_t tab = ((uint64_t)c.np * sizeof(nsk::TxGeo) + 15) & ~15ull;
    const uint64_t need = ((c.staging + 255) & ~255ull) + tab + 4ull * (c.np + 1);
    if (need <= std::min<uint64_t>(kHostSmallBytes, ctx->staging)) return run_tx_small(ctx, h_arena, plan, h_out);
  }
  const uint32_t nslots = ctx->nslots;
  int64_t pend[kMaxHostSlots];
  std::fill(pend, pend + kMaxHostSlots, (int64_t)-1);
  auto finish = [&](uint32_t sl) -> int {
    if (pend[sl] < 0) return NS_OK;
    const nsh::TxChunk& c = plan.chunks[(size_t)pend[sl]];
    pend[sl] = -1;
    HIP_TRY(hipEventSynchronize(ctx->done[sl]));
    patch_tx_fields(plan, c, ctx->h_out[sl].p, h_arena, h_out);
    return NS_OK;
  };
  std::vector<nsk::TxGeo> calls;
  std::vector<uint32_t> first;
  auto enqueue = [&](const nsh::TxChunk& c, uint32_t sl) -> int {
    int rc;
    if ((rc = ctx->d_arena[sl].ensure(c.staging + 256)) != NS_OK) return rc;
    if ((rc = ctx->h_out[sl].ensure(2 * c.nout)) != NS_OK) return rc;
    nsk::TxGeo launch{};
    const uint32_t grid = tx_chunk_table(plan, c, (uint64_t)(uintptr_t)ctx->d_arena[sl].p, ctx->h_out[sl].dev,
                                         &calls, &first, &launch);
    if (grid == 0) return NS_EINVAL;  // more than 2^31 tiles
    const size_t tab = ((size_t)c.np * sizeof(nsk::TxGeo) + 15) & ~(size_t)15;
    const size_t bytes = tab + first.size() * sizeof(uint32_t);
    if ((rc = ctx->h_txtab[sl].ensure(bytes)) != NS_OK) return rc;
    if ((rc = ctx->d_txtab[sl].ensure(bytes)) != NS_OK) return rc;
    std::memcpy(ctx->h_txtab[sl].p, calls.data(), (size_t)c.np * sizeof(nsk::TxGeo));
    std::memcpy(ctx->h_txtab[sl].p + tab, first.data(), first.size() * sizeof(uint32_t));
    hipStream_t s = ctx->stream[sl];
    for (uint32_t j = c.r0; j < c.r0 + c.nr; ++j) {
      const nsh::TxRange& r = plan.ranges[j];
      HIP_TRY(hipMemcpyAsync(ctx->d_arena[sl].p + r.at, h_arena + r.lo, r.hi - r.lo, hipMemcpyHostToDevice, s));
    }
    HIP_TRY(hipMemcpyAsync(ctx->d_txtab[sl].p, ctx->h_txtab[sl].p, bytes, hipMemcpyHostToDevice, s));
    HIP_TRY(nsk::launch_tcp_tx_multi(launch, grid, reinterpret_cast<const nsk::TxGeo*>(ctx->d_txtab[sl].p),
                                     reinterpret_cast<const uint32_t*>(ctx->d_txtab[sl].p + tab), c.np, s));
    HIP_TRY(hipEventRecord(ctx->done[sl], s));
    return NS_OK;
  };
  int rc = NS_OK;
  uint32_t slot = 0;
  for (size_t ci = 0; ci < plan.chunks.size(); ++ci) {
    if ((rc = finish(slot)) != NS_OK) break;
    if ((rc = enqueue(plan.chunks[ci], slot)) != NS_OK) {
      // copies of this chunk may be in flight: the caller's memory and the
      // staging must be idle before returning
      (void)hipStreamSynchronize(ctx->stream[slot]);
      (void)hipGetLastError();
      break;
    }
    pend[slot] = (int64_t)ci;
    slot = (slot + 1) % nslots;
  }
  for (uint32_t k = 0; k < nslots; ++k) {
    const int r = finish((slot + k) % nslots);
    if (rc == NS_OK) rc = r;
  }
  return rc;
}

// ns_csum_rx_ring_host's pipeline: the ring in chunks of whole slots (as
// many as the staging budget holds), nslots in flight on the host pipeline's
// streams.  Per chunk: the slots and their lengths go to the device, rx_ring
// parses and verifies them there and writes verdicts and sums straight to
// mapped pinned memory; when the chunk is done they are copied to the
// caller's arrays while later chunks are in flight.  No host planning.
// A small ring (its slots and lengths within kHostSmallBytes and the staging
// budget) takes no DMA either: written through the BAR into a gather stage,
// one launch, one wait.
int run_rx_small(ns_csum_ctx* ctx, const uint8_t* h_arena, const ns_rx_ring& r, const uint32_t* h_len,
                 uint16_t* h_sums, uint8_t* h_verdict) {
  const uint64_t bytes = (uint64_t)r.n * r.stride, len_at = (bytes + 255) & ~255ull;
  int rc = NS_OK;
  // results: the sums, then the verdicts
  if ((rc = ctx->p_res.ensure(5 * (size_t)r.n)) != NS_OK) return rc;
  BarBuf* st = lease_gather_stage(ctx, &rc, len_at + 4ull * r.n);
  if (!st) return rc;
  std::memcpy(st->p, h_arena + r.ring_off, bytes);
  std::memcpy(st->p + len_at, h_len, 4 * (size_t)r.n);
  __builtin_ia32_sfence();  // drain the write-combined BAR stores before the launch
  nsk::RxGeo geo{};
  geo.ring = (uint64_t)(uintptr_t)st->dev;
  geo.stride = r.stride;
  geo.len = reinterpret_cast<const uint32_t*>(st->dev + len_at);
  geo.sums = reinterpret_cast<uint16_t*>(ctx->p_res.dev);
  geo.verdict = ctx->p_res.dev + 4 * (size_t)r.n;
  geo.err = ctx->d_err;
  geo.n = r.n;
  geo.frame_at = r.frame_at;
  geo.link = r.link_hdr;
  geo.view0 = r.first_view ? r.first_view - r.link_hdr : 0u;
  hipStream_t s = ctx->stream[0];
  const hipError_t e = nsk::launch_rx_ring(geo, s);
  rc = e == hipSuccess ? wait_small(ctx, s) : report_hip(e, "run_rx_small", __FILE__, __LINE__);
  return_gather_stage(ctx, st);
  if (rc != NS_OK) return rc;
  if (h_sums) std::memcpy(h_sums, ctx->p_res.p, 4 * (size_t)r.n);
  if (h_verdict) std::memcpy(h_verdict, ctx->p_res.p + 4 * (size_t)r.n, r.n);
  return NS_OK;
}

int run_rx_host(ns_csum_ctx* ctx, const uint8_t* h_arena, const ns_rx_ring& r, const uint32_t* h_len,
                uint16_t* h_sums, uint8_t* h_verdict) {
  const uint64_t small = (((uint64_t)r.n * r.stride + 255) & ~255ull) + 4ull * r.n;
  if (zero_copy_enabled() && small <= std::min<uint64_t>(kHostSmallBytes, ctx->staging))
    return run_rx_small(ctx, h_arena, r, h_len, h_sums, h_verdict);
  const uint32_t nslots = ctx->nslots;
  const uint32_t per = (uint32_t)std::min<uint64_t>(std::max<uint64_t>(1, ctx->staging / r.stride), 1u << 24);
  struct Pending {
    bool live = false;
    uint32_t first = 0, count = 0;
  } pend[kMaxHostSlots];
  auto finish = [&](uint32_t sl) -> int {
    if (!pend[sl].live) return NS_OK;
    pend[sl].live = false;
    HIP_TRY(hipEventSynchronize(ctx->done[sl]));
    if (h_sums) std::memcpy(h_sums + 2 * (uint64_t)pend[sl].first, ctx->h_out[sl].p, 4 * (size_t)pend[sl].count);
    if (h_verdict) std::memcpy(h_verdict + pend[sl].first, ctx->h_verd[sl].p, pend[sl].count);
    return NS_OK;
  };
  auto enqueue = [&](uint32_t first, uint32_t cnt, uint32_t sl) -> int {
    int rc;
    const uint64_t bytes = (uint64_t)cnt * r.stride;
    if ((rc = ctx->d_arena[sl].ensure(bytes)) != NS_OK) return rc;
    if ((rc = ctx->d_len[sl].ensure(cnt)) != NS_OK) return rc;
    if ((rc = ctx->h_out[sl].ensure(2 * (size_t)cnt)) != NS_OK) return rc;
    if ((rc = ctx->h_verd[sl].ensure(cnt)) != NS_OK) return rc;
    hipStream_t s = ctx->stream[sl];
    HIP_TRY(hipMemcpyAsync(ctx->d_arena[sl].p, h_arena + r.ring_off + (uint64_t)first * r.stride, bytes,
                           hipMemcpyHostToDevice, s));
    HIP_TRY(hipMemcpyAsync(ctx->d_len[sl].p, h_len + first, 4 * (size_t)cnt, hipMemcpyHostToDevice, s));
    nsk::RxGeo geo{};
    geo.ring = (uint64_t)(uintptr_t)ctx->d_arena[sl].p;
    geo.stride = r.stride;
    geo.len = ctx->d_len[sl].p;
    geo.sums = ctx->h_out[sl].dev;
    geo.verdict = ctx->h_verd[sl].dev;
    geo.err = ctx->d_err;
    geo.n = cnt;
    geo.frame_at = r.frame_at;
    geo.link = r.link_hdr;
    geo.view0 = r.first_view ? r.first_view - r.link_hdr : 0u;
    HIP_TRY(nsk::launch_rx_ring(geo, s));
    HIP_TRY(hipEventRecord(ctx->done[sl], s));
    return NS_OK;
  };
  int rc = NS_OK;
  uint32_t slot = 0;
  for (uint64_t f = 0; f < r.n; f += per) {  // 64-bit: first + per may pass 2^32
    const uint32_t first = (uint32_t)f;
    const uint32_t cnt = (uint32_t)std::min<uint64_t>(per, r.n - f);
    if ((rc = finish(slot)) != NS_OK) break;
    if ((rc = enqueue(first, cnt, slot)) != NS_OK) {
      (void)hipStreamSynchronize(ctx->stream[slot]);
      (void)hipGetLastError();
      break;
    }
    pend[slot].live = true;
    pend[slot].first = first;
    pend[slot].count = cnt;
    slot = (slot + 1) % nslots;
  }
  for (uint32_t k = 0; k < nslots; ++k) {
    const int e = finish((slot + k) % nslots);
    if (rc == NS_OK) rc = e;
  }
  return rc;
}

// Caller-acquired staging (ns_csum_stage_acquire): mapped pinned buffers a
// caller fills itself — the Go shim, which may not hand C memory holding Go
// pointers to the library, copies its views there once.  Gathers whose bytes
// all lie in one acquired stage read them in place (ByteSink adopt mode).
// Buffers above kStageBytes come from a second pool (big_free).
MappedPin* lease_big(ns_csum_ctx* ctx, uint64_t bytes, int* rc) {
  {
    std::lock_guard<std::mutex> ql(ctx->qmu);
    for (size_t i = 0; i < ctx->big_free.size(); ++i) {
      if (ctx->big_free[i]->cap >= bytes) {
        MappedPin* b = ctx->big_free[i];
        ctx->big_free.erase(ctx->big_free.begin() + (long)i);
        return b;
      }
    }
  }
  AllocClock clk(ctx);
  MappedPin* b = new (std::nothrow) MappedPin();
  if (!b) {
    *rc = NS_ENOMEM;
    return nullptr;
  }
  {
    DeviceGuard g(ctx->device);
    // whole MiB, so a pooled buffer fits the next call of a similar size
    if ((*rc = b->ensure((bytes + (1ull << 20) - 1) & ~((1ull << 20) - 1))) != NS_OK) {
      delete b;
      return nullptr;
    }
  }
  std::lock_guard<std::mutex> ql(ctx->qmu);
  ctx->stage_all.push_back(b);
  return b;
}

// The acquired stage holding every byte of [lo, hi), or nullptr.
MappedPin* find_acquired(ns_csum_ctx* ctx, uintptr_t lo, uintptr_t hi) {
  std::lock_guard<std::mutex> ql(ctx->qmu);
  for (MappedPin* b : ctx->leased) {
    const uintptr_t a = (uintptr_t)b->p;
    if (lo >= a && hi <= a + b->cap) return b;
  }
  return nullptr;
}

// The byte span of a call's inputs, to decide whether they all lie in one
// acquired stage.
struct SpanProbe {
  uintptr_t lo = UINTPTR_MAX, hi = 0;
  void add(const uint8_t* p, uint64_t len) {
    if (!len || !p) return;
    lo = std::min(lo, (uintptr_t)p);
    hi = std::max(hi, (uintptr_t)p + (uintptr_t)len);
  }
  MappedPin* stage(ns_csum_ctx* ctx) const { return hi ? find_acquired(ctx, lo, hi) : nullptr; }
};

// Where a gather assembles its bytes.  Small gathers go to a mapped staging
// buffer leased from the context's pool (the kernel reads it in place).  A
// gather that outgrows it moves, under the context lock it then keeps until
// the call ends, into the pipeline's pinned arena `g_arena` (grown by doubling
// and kept between calls) and takes the DMA pipeline: one CPU copy per byte
// either way (a 64 MiB VectorisedView batch went from 31 ms through a
// growing std::vector to a few ms; tools/latency.cc).  A gather whose bytes
// already lie in a caller's acquired stage copies nothing: its descriptors
// address that stage (adopt mode).
struct ByteSink {
  ns_csum_ctx* ctx;
  BarBuf* stage = nullptr;       // leased from the pool (copy mode)
  MappedPin* adopted = nullptr;  // the caller's acquired stage (adopt mode)
  std::unique_lock<std::mutex> big;  // ctx->pmu, held once the bytes live in ctx->g_arena
  uint64_t n = 0;  // copy: bytes appended; adopt: end of the highest byte used
  int rc = NS_OK;
  // the pieces copied into the stage so far: a move to g_arena copies them
  // again from their sources, never back out of the stage (device memory
  // behind the BAR reads at PCIe-latency speed)
  std::vector<std::pair<const uint8_t*, uint64_t>> staged;
  explicit ByteSink(ns_csum_ctx* c, MappedPin* adopt = nullptr) : ctx(c), adopted(adopt) {
    if (adopted) return;
    if (zero_copy_enabled()) stage = lease_gather_stage(ctx, &rc);
    if (!stage) rc = to_big(0);
    else staged.reserve(64);
  }
  ~ByteSink() { return_gather_stage(ctx, stage); }
  ByteSink(const ByteSink&) = delete;
  ByteSink& operator=(const ByteSink&) = delete;
  bool in_big() const { return big.owns_lock(); }
  uint64_t size() const { return n; }
  uint8_t* base() const { return adopted ? adopted->p : in_big() ? ctx->g_arena.p : stage->p; }
  // g_arena with room for `need` bytes, keeping its first `keep` bytes.
  int reserve_big(uint64_t need, uint64_t keep) {
    PinBuf<uint8_t>& g = ctx->g_arena;
    if (need <= g.cap) return NS_OK;
    PinBuf<uint8_t> fresh;
    DeviceGuard dg(ctx->device);
    const int r = fresh.ensure(std::max<uint64_t>(need, 2 * (uint64_t)g.cap));
    if (r != NS_OK) return r;
    if (keep) std::memcpy(fresh.p, g.p, keep);
    g.release();
    g = fresh;
    return NS_OK;
  }
  // Move to a larger gather stage with room for `need` bytes (<=
  // kZeroCopyMax), copying what is staged again from its sources.
  int grow_stage(uint64_t need) {
    int r = NS_OK;
    BarBuf* nb = lease_gather_stage(ctx, &r, std::max<uint64_t>(need, 2 * stage->cap));
    if (!nb) return r != NS_OK ? r : NS_ENOMEM;
    uint64_t at = 0;
    for (const auto& pc : staged) {
      std::memcpy(nb->p + at, pc.first, pc.second);
      at += pc.second;
    }
    return_gather_stage(ctx, stage);
    stage = nb;
    return NS_OK;
  }
  // Move to g_arena (taking the pipeline lock) with room for `need` bytes.
  int to_big(uint64_t need) {
    big = std::unique_lock<std::mutex>(ctx->pmu);
    const int r = reserve_big(std::max<uint64_t>(need, 1ull << 20), 0);
    if (r != NS_OK) return r;
    uint64_t at = 0;
    for (const auto& pc : staged) {
      std::memcpy(ctx->g_arena.p + at, pc.first, pc.second);
      at += pc.second;
    }
    staged.clear();
    return NS_OK;
  }
  // Makes bytes [p, p + len) part of the arena; returns their arena offset.
  uint64_t append(const uint8_t* p, uint64_t len) {
    if (adopted) {
      const uint64_t at = len ? (uint64_t)(p - adopted->p) : n;
      n = std::max(n, at + len);
      return at;
    }
    const uint64_t at = n;
    if (!len || rc != NS_OK) return at;
    if (!in_big() && n + len > stage->cap) rc = n + len <= kZeroCopyMax ? grow_stage(n + len) : to_big(n + len);
    else if (in_big()) rc = reserve_big(n + len, n);
    if (rc != NS_OK) return at;
    std::memcpy(base() + n, p, len);
    if (!in_big()) staged.emplace_back(p, len);
    n += len;
    return at;
  }
};

// ---- gather of VectorisedView pieces (tcpip/buffer -> staging arena) -----
// The descriptors come from nsh::ChainBuilder (host_logic.h) over a ByteSink.
struct SinkHolder {
  ByteSink sink;  // assembled in mapped staging (or spilled host memory), or adopted in place
  SinkHolder(ns_csum_ctx* c, MappedPin* adopt) : sink(c, adopt) {}
};
struct Gather : SinkHolder, nsh::ChainBuilder<ByteSink> {  // the sink is constructed first
  ns_csum_ctx* ctx;
  explicit Gather(ns_csum_ctx* c, MappedPin* adopt = nullptr)
      : SinkHolder(c, adopt), nsh::ChainBuilder<ByteSink>(sink), ctx(c) {}

  int run(uint16_t* out) {
    if (sink.rc != NS_OK) return sink.rc;
    std::vector<uint16_t> res(desc.size());
    int rc;
    const bool chained = any_cont(desc.data(), (uint32_t)desc.size());
    if (sink.adopted && !(zero_copy_enabled() && sink.size() <= kStageBytes)) {
      // A large caller stage: pinned already, so the DMA pipeline reads it.
      std::lock_guard<std::mutex> lk(ctx->pmu);
      DeviceGuard g(ctx->device);
      rc = run_host_batch(ctx, sink.base(), sink.size(), desc.data(), (uint32_t)desc.size(), res.data(), chained);
    } else if (!sink.in_big()) {
      // Small: zero-copy from the leased (or the caller's) staging, combined
      // with concurrent calls.
      SmallReq rq;
      rq.dbytes = sink.adopted ? sink.adopted->dev : sink.stage->dev;
      rq.nbytes = sink.size();
      rq.desc = desc.data();
      rq.ndesc = (uint32_t)desc.size();
      rq.res = res.data();
      rq.chained = chained;
      rc = submit_small(ctx, &rq);
    } else {
      // Large: the bytes are in the pinned g_arena and ctx->pmu is held.
      DeviceGuard g(ctx->device);
      rc = run_host_batch(ctx, ctx->g_arena.p, sink.size(), desc.data(), (uint32_t)desc.size(), res.data(),
                          chained);
    }
    if (rc != NS_OK) return rc;
    for (size_t q = 0; q < result_at.size(); ++q) out[q] = res[result_at[q]];
    return NS_OK;
  }
};

}  // namespace

extern "C" {

int ns_csum_abi_version(void) { return NS_CSUM_ABI_VERSION; }

int ns_csum_last_hip_error(void) { return (int)g_last_hip; }

const char* ns_csum_strerror(int status) {
  switch (status) {
    case NS_OK: return "ok";
    case NS_EINVAL: return "invalid argument";
    case NS_ERANGE: return "descriptor outside the arena";
    case NS_ENODEV: return "no HIP device";
    case NS_ENOMEM: return "out of memory";
    case NS_EHIP: return "HIP runtime error";
    default: return "unknown status";
  }
}

int ns_csum_device_count(int* count) {
  if (!count) return NS_EINVAL;
  *count = 0;
  int c = 0;
  hipError_t e = hipGetDeviceCount(&c);
  if (e != hipSuccess) return (e == hipErrorNoDevice) ? NS_ENODEV : map_hip_error(e);
  *count = c;
  return NS_OK;
}

uint16_t ns_csum_combine(uint16_t a, uint16_t b) {  // checksum.go:104-107
  const uint32_t v = (uint32_t)a + (uint32_t)b;
  return (uint16_t)(v + (v >> 16));
}

int ns_csum_init(const ns_csum_opts* opts, ns_csum_ctx** out) {
  if (!out) return NS_EINVAL;
  *out = nullptr;
  int ndev = 0;
  int rc = ns_csum_device_count(&ndev);
  if (rc != NS_OK) return rc;
  if (opts && (opts->flags & ~NS_OPT_FOLD_WALK)) return NS_EINVAL;
  const int dev = opts ? opts->device : 0;
  if (dev < 0 || dev >= ndev) return NS_ENODEV;
  ns_csum_ctx* ctx = new (std::nothrow) ns_csum_ctx();
  if (!ctx) return NS_ENOMEM;
  ctx->device = dev;
  if (opts && opts->staging_bytes) ctx->staging = opts->staging_bytes;
  ctx->fold_walk = opts && (opts->flags & NS_OPT_FOLD_WALK);
  DeviceGuard g(dev);
  // The context's own streams serve synchronous callers only (zero-copy
  // passes, the DMA pipeline, ns_csum_sync), so they take the device's
  // greatest priority.  HIP pools hardware queues per priority
  // (GPU_MAX_HW_QUEUES=4 each): at normal priority a pass could share a
  // queue with a caller's stream and wait behind its whole backlog (round 3's
  // 21-43 ms stalls, every one a pass whose completion was late; DESIGN.md
  // §4.4).  NS_CSUM_NORMAL_PRIORITY=1 creates them at normal priority (A/B
  // diagnostics only).
  int least = 0, greatest = 0;
  if (hipDeviceGetStreamPriorityRange(&least, &greatest) != hipSuccess) {
    least = greatest = 0;
    (void)hipGetLastError();
  }
  (void)least;
  if (std::getenv("NS_CSUM_NORMAL_PRIORITY")) greatest = 0;
  // the pipeline's shape (A/B diagnostics; read here once, never per call)
  if (const char* v = std::getenv("NS_CSUM_HOST_SLOTS")) {
    const long x = std::strtol(v, nullptr, 10);
    if (x >= 1 && x <= (long)kMaxHostSlots) ctx->nslots = (uint32_t)x;
  }
  ctx->host_d2h = std::getenv("NS_CSUM_HOST_D2H") != nullptr;
  if (const char* v = std::getenv("NS_CSUM_HOST_CHUNK")) {
    const long x = std::strtol(v, nullptr, 10);
    if (x >= 1024 && x <= (1l << 22)) ctx->chunk_desc = (uint32_t)x;
  }
  hipError_t e = hipSuccess;
  for (uint32_t s = 0; s < ctx->nslots && e == hipSuccess; ++s) {
    e = hipStreamCreateWithPriority(&ctx->stream[s], hipStreamNonBlocking, greatest);
    if (e == hipSuccess) e = hipEventCreateWithFlags(&ctx->done[s], hipEventDisableTiming);
  }
  if (e == hipSuccess) e = hipStreamCreateWithPriority(&ctx->zstream, hipStreamNonBlocking, greatest);
  if (e == hipSuccess) e = hipMalloc(reinterpret_cast<void**>(&ctx->d_err), sizeof(unsigned long long));
  if (e == hipSuccess) e = hipMemset(ctx->d_err, 0, sizeof(unsigned long long));
  if (e != hipSuccess) {
    ns_csum_destroy(ctx);
    return report_hip(e, "ns_csum_init", __FILE__, __LINE__);
  }
  if ((rc = ctx->err_taken.ensure(sizeof(unsigned long long))) != NS_OK) {
    ns_csum_destroy(ctx);
    return rc;
  }
  // Zero-copy pass tables in device memory written through the BAR when the
  // whole VRAM is CPU-mapped (NS_CSUM_NO_BAR_TABLE=1: mapped host memory, for
  // A/B diagnostics only).
  int large_bar = 0;
  if (hipDeviceGetAttribute(&large_bar, hipDeviceAttributeIsLargeBar, dev) != hipSuccess) {
    large_bar = 0;
    (void)hipGetLastError();
  }
  ctx->bar_table = large_bar != 0 && std::getenv("NS_CSUM_NO_BAR_TABLE") == nullptr;
  // ns_csum_tcp_tx's A/B knobs, read from the environment once, here (the
  // tools set them per process; tests use ns_csum_set_tx_tuning).
  auto knob = [](const char* name) -> uint32_t {
    const char* v = std::getenv(name);
    return v ? (uint32_t)std::strtoul(v, nullptr, 10) : 0u;
  };
  ctx->tx_variant = knob("NS_CSUM_TX_VARIANT");
  ctx->tx_tile = knob("NS_CSUM_TX_TILE");
  ctx->tx_htile = knob("NS_CSUM_TX_HTILE");
  ctx->tx_passes = knob("NS_CSUM_TX_PASSES");
  *out = ctx;
  return NS_OK;
}

void ns_csum_destroy(ns_csum_ctx* ctx) {
  if (!ctx) return;
  {
    DeviceGuard g(ctx->device);
    for (uint32_t s = 0; s < kMaxHostSlots; ++s)
      if (ctx->stream[s]) (void)hipStreamSynchronize(ctx->stream[s]);
    if (ctx->zstream) (void)hipStreamSynchronize(ctx->zstream);
    ctx->scratch.clear([&](StreamScratch* sc) { retire_scratch(ctx, sc); });
    if (ctx->retire) {
      (void)hipStreamSynchronize(ctx->retire);
      (void)hipStreamDestroy(ctx->retire);
    }
    ctx->err_taken.release();
    ctx->z_buf.release();
    ctx->z_res.release();
    ctx->z_done.release();
    ctx->z_ctr.release();
    for (MappedPin* b : ctx->stage_all) {
      b->release();
      delete b;
    }
    ctx->stage_all.clear();
    ctx->stage_free.clear();
    for (BarBuf* b : ctx->gstage_all) {
      b->release();
      delete b;
    }
    ctx->gstage_all.clear();
    ctx->gstage_free.clear();
    for (uint32_t s = 0; s < kMaxHostSlots; ++s) {
      ctx->d_arena[s].release();
      ctx->d_desc[s].release();
      ctx->d_out[s].release();
      ctx->d_chain[s].release();
      ctx->h_desc[s].release();
      ctx->h_out[s].release();
      ctx->h_txtab[s].release();
      ctx->d_txtab[s].release();
      ctx->d_len[s].release();
      ctx->h_verd[s].release();
      if (s == 0) {
        ctx->p_res.release();
        ctx->p_done.release();
      }
      if (ctx->done[s]) (void)hipEventDestroy(ctx->done[s]);
      if (ctx->stream[s]) (void)hipStreamDestroy(ctx->stream[s]);
    }
    ctx->g_arena.release();
    ctx->z_chain.release();
    if (ctx->zstream) (void)hipStreamDestroy(ctx->zstream);
    if (ctx->d_err) (void)hipFree(ctx->d_err);
  }
  delete ctx;
}

int ns_csum_sync(ns_csum_ctx* ctx, void* stream, uint64_t* bad) {
  if (!ctx) return NS_EINVAL;
  DeviceGuard g(ctx->device);
  if (stream) {
    HIP_TRY(hipStreamSynchronize((hipStream_t)stream));
  } else {
    HIP_TRY(hipDeviceSynchronize());
  }
  unsigned long long v = 0;
  {
    // Read and reset in one device atomic (take_err): a separate copy and
    // memset would lose counts that kernels on other streams add in between.
    std::lock_guard<std::mutex> lk(ctx->mu);
    unsigned long long* taken = reinterpret_cast<unsigned long long*>(ctx->err_taken.p);
    HIP_TRY(nsk::launch_take_err(ctx->d_err, reinterpret_cast<unsigned long long*>(ctx->err_taken.dev),
                                 ctx->zstream));
    HIP_TRY(hipStreamSynchronize(ctx->zstream));
    v = *reinterpret_cast<volatile unsigned long long*>(taken);
  }
  if (bad) *bad = v;
  return NS_OK;
}

namespace {
int batch_dev(ns_csum_ctx* ctx, const uint8_t* d_arena, uint64_t arena_bytes, const ns_pkt_desc* d_desc,
              uint32_t n, uint16_t* d_out, uint32_t batch_flags, void* stream, bool store) {
  if (!ctx || (n && (!d_desc || !d_out)) || (arena_bytes && !d_arena)) return NS_EINVAL;
  if (n == 0) return NS_OK;
  const bool need_chain = (batch_flags & NS_BATCH_CHAINED) != 0;
  const bool paired = (batch_flags & NS_BATCH_PAIRED) != 0;
  if (paired && need_chain) return NS_EINVAL;
  DeviceGuard g(ctx->device);
  hipStream_t s = (hipStream_t)stream;  // NULL = the HIP null stream
  // NS_CSUM_STORE_WB=1: in-place stores of unchained tiles as plain
  // write-back stores (A/B diagnostics only)
  static const uint32_t wb = std::getenv("NS_CSUM_STORE_WB") ? 4u : 0u;
  if (paired) {  // plain tiles, pairs folded in the kernel (no scratch)
    HIP_TRY(nsk::launch_batch(d_arena, arena_bytes, d_desc, n, d_out, nsk::ChainScratch{}, ctx->d_err, s, 0,
                              (store ? 1u | wb : 0u) | 2u, nullptr));
    return NS_OK;
  }
  const bool need_split = arena_bytes / n >= nsk::split_min_avg();
  if (!need_chain && !need_split) {
    HIP_TRY(nsk::launch_batch(d_arena, arena_bytes, d_desc, n, d_out, nsk::ChainScratch{}, ctx->d_err, s, 0,
                              store ? 1u | wb : 0u, nullptr));
    return NS_OK;
  }
  StreamScratch* sc = ctx->scratch.pin(scratch_key(s), make_scratch,
                                       [&](StreamScratch* old) { retire_scratch(ctx, old); });
  if (!sc) return NS_ENOMEM;
  int rc = NS_OK;
  {
    std::lock_guard<std::mutex> lk(sc->mu);
    nsk::ChainScratch chain{};
    uint32_t* split = nullptr;
    const size_t caps = sc->chain.part.cap + sc->chain.status.cap + sc->split.cap;
    const uint64_t t0 = now_ns();
    if (need_chain && (rc = sc->chain.ensure_async(n, s)) == NS_OK) chain = sc->chain.get(ctx->fold_walk);
    // split accumulators: zero once, the kernel leaves them so
    if (rc == NS_OK && need_split && (rc = sc->split.ensure_async(nsk::split_words(n), true, s)) == NS_OK)
      split = sc->split.p;
    if (sc->chain.part.cap + sc->chain.status.cap + sc->split.cap != caps) {
      const uint64_t dt = now_ns() - t0;
      ctx->st.growths.fetch_add(1, std::memory_order_relaxed);
      ctx->st.growth_ns_total.fetch_add(dt, std::memory_order_relaxed);
      bump_max(ctx->st.growth_ns_max, dt);
    }
    if (rc == NS_OK) {
      hipError_t e = nsk::launch_batch(d_arena, arena_bytes, d_desc, n, d_out, chain, ctx->d_err, s, 0,
                                       store ? 1u : 0u, split);
      if (e == hipSuccess) e = hipEventRecord(sc->last, s);
      if (e != hipSuccess) rc = report_hip(e, "launch_batch", __FILE__, __LINE__);
    }
  }
  ctx->scratch.unpin(sc);
  return rc;
}
}  // namespace

int ns_csum_stream_release(ns_csum_ctx* ctx, void* stream) {
  if (!ctx) return NS_EINVAL;
  DeviceGuard g(ctx->device);
  return ctx->scratch.release(scratch_key((hipStream_t)stream),
                              [&](StreamScratch* sc) { retire_scratch(ctx, sc); });
}

int ns_csum_scratch_count(ns_csum_ctx* ctx, uint32_t* count) {
  if (!ctx || !count) return NS_EINVAL;
  *count = (uint32_t)ctx->scratch.size();
  return NS_OK;
}

int ns_csum_batch_dev(ns_csum_ctx* ctx, const uint8_t* d_arena, uint64_t arena_bytes,
                      const ns_pkt_desc* d_desc, uint32_t n, uint16_t* d_out,
                      uint32_t batch_flags, void* stream) {
  return batch_dev(ctx, d_arena, arena_bytes, d_desc, n, d_out, batch_flags, stream, false);
}

int ns_csum_batch_dev_store(ns_csum_ctx* ctx, uint8_t* d_arena, uint64_t arena_bytes,
                            const ns_pkt_desc* d_desc, uint32_t n, uint16_t* d_out,
                            uint32_t batch_flags, void* stream) {
  return batch_dev(ctx, d_arena, arena_bytes, d_desc, n, d_out, batch_flags, stream, true);
}

int ns_csum_tcp_tx(ns_csum_ctx* ctx, uint8_t* d_arena, uint64_t arena_bytes, const ns_tcp_tx* tx,
                   uint16_t* d_out, void* stream) {
  if (!ctx || !tx || (arena_bytes && !d_arena)) return NS_EINVAL;
  const ns_tcp_tx& t = *tx;
  nsh::TxPlan plan;
  const int vr = nsh::tx_plan(t, arena_bytes, &plan);
  if (vr != NS_OK) return vr;
  const uint64_t n = plan.n;
  const uint32_t mode = plan.mode;
  static_assert(nsk::kTxIp == 1u && nsk::kTxTcpFull == 2u && nsk::kTxTcpPartial == 4u && nsk::kTxFieldsOnly == 8u,
                "nsh::tx_plan's mode bits");
  if (n == 0) return NS_OK;
  if (!(mode & (nsk::kTxIp | nsk::kTxTcpFull | nsk::kTxTcpPartial))) {  // nothing to fill: the sums are 0
    if (d_out) {
      DeviceGuard g(ctx->device);
      HIP_TRY(hipMemsetAsync(d_out, 0, 4 * n, (hipStream_t)stream));
    }
    return NS_OK;
  }
  DeviceGuard g(ctx->device);
  nsk::TxGeo geo{};
  const uint64_t base = (uint64_t)(uintptr_t)d_arena;
  geo.hdr = base + t.hdr_off;
  geo.pay = base + t.pay_off;
  geo.size = t.size;
  geo.n = n;
  geo.mss = t.mss;
  geo.slot = t.slot;
  geo.ip_at = t.ip_at;
  geo.ip_len = t.ip_len;
  geo.tcp_at = t.tcp_at;
  geo.tcp_len = t.tcp_len;
  geo.addr_sum = t.addr_sum;
  geo.proto = t.protocol;
  geo.mode = mode;
  geo.out = d_out;
  // A/B and test knobs (ns_csum_set_tx_tuning): a variant of the kernel
  // (csum_kernels.h launch_tcp_tx); segments per wave of the payload (or the
  // only) pass and of the header pass instead of the launcher's choice; the
  // fused or the two-pass shape whatever the payload size.
  const uint32_t variant = ctx->tx_variant.load(std::memory_order_relaxed);
  geo.tile = ctx->tx_tile.load(std::memory_order_relaxed);
  geo.htile = ctx->tx_htile.load(std::memory_order_relaxed);
  const uint32_t passes = ctx->tx_passes.load(std::memory_order_relaxed);
  const bool two = passes ? passes == 2 : t.size >= nsk::kTxTwoPassMinBytes;
  hipStream_t s = (hipStream_t)stream;
  if (!(mode & nsk::kTxTcpFull) || !two) {  // one pass (no scratch)
    HIP_TRY(nsk::launch_tcp_tx(geo, s, variant));
    return NS_OK;
  }
  if (d_out) {
    // The payload pass parks each segment's payload value in d_out[2i + 1],
    // which the header pass then overwrites with the TCP sum: no scratch, and
    // no event to record (an event per call put ~6 us between calls).
    geo.xs = d_out + 1;
    geo.xstride = 2;
    HIP_TRY(nsk::launch_tcp_tx(geo, s, variant));
    return NS_OK;
  }
  // The payload pass leaves each segment's payload value in per-stream
  // scratch (2 B per segment) for the header pass.
  StreamScratch* sc = ctx->scratch.pin(scratch_key(s), make_scratch,
                                       [&](StreamScratch* old) { retire_scratch(ctx, old); });
  if (!sc) return NS_ENOMEM;
  int rc = NS_OK;
  {
    std::lock_guard<std::mutex> lk(sc->mu);
    const size_t cap = sc->txpay.cap;
    const uint64_t t0 = now_ns();
    rc = sc->txpay.ensure_async((size_t)n, false, s);
    if (sc->txpay.cap != cap) {
      const uint64_t dt = now_ns() - t0;
      ctx->st.growths.fetch_add(1, std::memory_order_relaxed);
      ctx->st.growth_ns_total.fetch_add(dt, std::memory_order_relaxed);
      bump_max(ctx->st.growth_ns_max, dt);
    }
    if (rc == NS_OK) {
      geo.xs = sc->txpay.p;
      geo.xstride = 1;
      hipError_t e = nsk::launch_tcp_tx(geo, s, variant);
      if (e == hipSuccess) e = hipEventRecord(sc->last, s);
      if (e != hipSuccess) rc = report_hip(e, "launch_tcp_tx", __FILE__, __LINE__);
    }
  }
  ctx->scratch.unpin(sc);
  return rc;
}

int ns_csum_tcp_tx_multi(ns_csum_ctx* ctx, uint8_t* d_arena, uint64_t arena_bytes, const ns_tcp_tx* txs,
                         uint32_t count, uint16_t* d_out, void* stream) {
  if (!ctx || (count && !txs) || (arena_bytes && !d_arena)) return NS_EINVAL;
  std::vector<nsh::TxPlan> plans;
  const int vr = nsh::tx_multi_plan(txs, count, arena_bytes, &plans);
  if (vr != NS_OK) return vr;
  DeviceGuard g(ctx->device);
  hipStream_t s = (hipStream_t)stream;
  const uint64_t base = (uint64_t)(uintptr_t)d_arena;
  std::vector<nsk::TxGeo> calls;
  calls.reserve(count);
  uint64_t seg = 0;
  for (uint32_t k = 0; k < count; ++k) {
    const ns_tcp_tx& t = txs[k];
    const nsh::TxPlan& p = plans[k];
    if (p.n && !(p.mode & 7u) && d_out) HIP_TRY(hipMemsetAsync(d_out + 2 * seg, 0, 4 * p.n, s));  // nothing to fill
    if (p.n && (p.mode & 7u)) {
      nsk::TxGeo geo{};
      geo.hdr = base + t.hdr_off;
      geo.pay = base + t.pay_off;
      geo.size = t.size;
      geo.n = p.n;
      geo.mss = t.mss;
      geo.slot = t.slot;
      geo.ip_at = t.ip_at;
      geo.ip_len = t.ip_len;
      geo.tcp_at = t.tcp_at;
      geo.tcp_len = t.tcp_len;
      geo.addr_sum = t.addr_sum;
      geo.proto = t.protocol;
      geo.mode = p.mode;
      geo.out = d_out ? d_out + 2 * seg : nullptr;
      calls.push_back(geo);
    }
    seg += p.n;
  }
  if (calls.empty()) return NS_OK;
  const uint32_t nc = (uint32_t)calls.size();
  std::vector<uint32_t> first(nc + 1);
  nsk::TxGeo launch{};
  const uint32_t grid = nsk::tx_multi_prepare(calls.data(), nc, &launch, first.data());
  if (grid == 0) return NS_EINVAL;  // more than 2^31 tiles
  const size_t tab = ((size_t)nc * sizeof(nsk::TxGeo) + 15) & ~(size_t)15;
  const size_t bytes = tab + first.size() * sizeof(uint32_t);
  StreamScratch* sc = ctx->scratch.pin(scratch_key(s), make_scratch,
                                       [&](StreamScratch* old) { retire_scratch(ctx, old); });
  if (!sc) return NS_ENOMEM;
  int rc = NS_OK;
  {
    std::lock_guard<std::mutex> lk(sc->mu);
    rc = sc->txtab.ensure_async(bytes, false, s);
    // The next pinned copy of the ring.  Its previous upload was enqueued
    // kTabSlots calls ago on this stream: waiting for it here (only when the
    // device is that far behind) is back-pressure, not a per-call stall.
    StreamScratch::TabSlot& ts = sc->tab[sc->tab_next++ % StreamScratch::kTabSlots];
    if (rc == NS_OK && !ts.ev && hipEventCreateWithFlags(&ts.ev, hipEventDisableTiming) != hipSuccess) {
      ts.ev = nullptr;
      rc = NS_EHIP;
    }
    if (rc == NS_OK) {
      if (hipEventQuery(ts.ev) != hipSuccess) {
        (void)hipGetLastError();
        (void)hipEventSynchronize(ts.ev);
      }
      if (ts.cap < bytes) {
        if (ts.h) (void)hipHostFree(ts.h);
        ts.h = nullptr;
        ts.cap = 0;
        const size_t cap = std::max<size_t>(bytes, 64u << 10);
        if (hipHostMalloc(reinterpret_cast<void**>(&ts.h), cap, hipHostMallocDefault) != hipSuccess) {
          ts.h = nullptr;
          rc = NS_ENOMEM;
        } else {
          ts.cap = cap;
        }
      }
    }
    if (rc == NS_OK) {
      std::memcpy(ts.h, calls.data(), (size_t)nc * sizeof(nsk::TxGeo));
      std::memcpy(ts.h + tab, first.data(), first.size() * sizeof(uint32_t));
      hipError_t e = hipMemcpyAsync(sc->txtab.p, ts.h, bytes, hipMemcpyHostToDevice, s);
      if (e == hipSuccess) e = hipEventRecord(ts.ev, s);
      if (e == hipSuccess)
        e = nsk::launch_tcp_tx_multi(launch, grid, reinterpret_cast<const nsk::TxGeo*>(sc->txtab.p),
                                     reinterpret_cast<const uint32_t*>(sc->txtab.p + tab), nc, s);
      if (e == hipSuccess) e = hipEventRecord(sc->last, s);
      if (e != hipSuccess) rc = report_hip(e, "launch_tcp_tx_multi", __FILE__, __LINE__);
    }
  }
  ctx->scratch.unpin(sc);
  return rc;
}

int ns_csum_tcp_tx_host(ns_csum_ctx* ctx, uint8_t* h_arena, uint64_t arena_bytes, const ns_tcp_tx* txs,
                        uint32_t count, uint16_t* h_out) {
  if (!ctx || (count && !txs) || (arena_bytes && !h_arena)) return NS_EINVAL;
  CallClock clk(ctx);
  nsh::TxHostPlan plan;
  const int vr = nsh::tx_host_plan(txs, count, arena_bytes, ctx->staging, &plan);
  if (vr != NS_OK) return vr;
  if (h_out)
    for (const auto& z : plan.zeros) std::memset(h_out + 2 * z.first, 0, 4 * z.second);
  if (plan.chunks.empty()) return NS_OK;
  std::lock_guard<std::mutex> lk(ctx->pmu);
  DeviceGuard g(ctx->device);
  return run_tx_host(ctx, h_arena, plan, h_out);
}

int ns_csum_set_tx_tuning(ns_csum_ctx* ctx, uint32_t variant, uint32_t tile, uint32_t htile, uint32_t passes) {
  if (!ctx || variant > 7 || passes > 2) return NS_EINVAL;
  ctx->tx_variant = variant;
  ctx->tx_tile = tile;
  ctx->tx_htile = htile;
  ctx->tx_passes = passes;
  return NS_OK;
}

int ns_csum_rx_ring(ns_csum_ctx* ctx, const uint8_t* d_arena, uint64_t arena_bytes, const ns_rx_ring* ring,
                    const uint32_t* d_len, uint16_t* d_sums, uint8_t* d_verdict, void* stream) {
  if (!ctx || !ring || (arena_bytes && !d_arena) || (!d_sums && !d_verdict)) return NS_EINVAL;
  const ns_rx_ring& r = *ring;
  if (r.n && !d_len) return NS_EINVAL;
  const uint64_t base = (uint64_t)(uintptr_t)d_arena;
  const int vr = nsh::rx_plan(r, base, arena_bytes);
  if (vr != NS_OK) return vr;
  if (r.n == 0) return NS_OK;
  DeviceGuard g(ctx->device);
  nsk::RxGeo geo{};
  geo.ring = base + r.ring_off;
  geo.stride = r.stride;
  geo.len = d_len;
  geo.sums = d_sums;
  geo.verdict = d_verdict;
  geo.err = ctx->d_err;
  geo.n = r.n;
  geo.frame_at = r.frame_at;
  geo.link = r.link_hdr;
  geo.view0 = r.first_view ? r.first_view - r.link_hdr : 0u;
  HIP_TRY(nsk::launch_rx_ring(geo, (hipStream_t)stream));
  return NS_OK;
}

int ns_csum_rx_bufs(ns_csum_ctx* ctx, const uint8_t* d_arena, uint64_t arena_bytes, const ns_rx_ring* ring,
                    const uint32_t* d_off, const uint32_t* d_len, uint16_t* d_sums, uint8_t* d_verdict, void* stream) {
  if (!ctx || !ring || (arena_bytes && !d_arena) || (!d_sums && !d_verdict)) return NS_EINVAL;
  const ns_rx_ring& r = *ring;
  if (r.n && (!d_len || !d_off)) return NS_EINVAL;
  const uint64_t base = (uint64_t)(uintptr_t)d_arena;
  if (r.ring_off > arena_bytes) return NS_ERANGE;
  // the ring's shape rules with no slots to place (the buffers are wherever
  // the offsets say; the kernel checks each against the arena)
  ns_rx_ring r0 = r;
  r0.n = 0;
  const int vr = nsh::rx_plan(r0, base, arena_bytes);
  if (vr != NS_OK) return vr;
  const uint64_t limit = arena_bytes - r.ring_off;
  if (limit > (1ull << 32) - 512) return NS_EINVAL;  // 32-bit offsets under one buffer resource
  if (r.n == 0) return NS_OK;
  DeviceGuard g(ctx->device);
  nsk::RxGeo geo{};
  geo.ring = base + r.ring_off;
  geo.stride = r.stride;
  geo.len = d_len;
  geo.sums = d_sums;
  geo.verdict = d_verdict;
  geo.err = ctx->d_err;
  geo.n = r.n;
  geo.frame_at = r.frame_at;
  geo.link = r.link_hdr;
  geo.view0 = r.first_view ? r.first_view - r.link_hdr : 0u;
  geo.off = d_off;
  geo.limit = limit;
  HIP_TRY(nsk::launch_rx_ring(geo, (hipStream_t)stream));
  return NS_OK;
}

int ns_csum_rx_ring_host(ns_csum_ctx* ctx, const uint8_t* h_arena, uint64_t arena_bytes, const ns_rx_ring* ring,
                         const uint32_t* h_len, uint16_t* h_sums, uint8_t* h_verdict) {
  if (!ctx || !ring || (arena_bytes && !h_arena) || (!h_sums && !h_verdict)) return NS_EINVAL;
  const ns_rx_ring& r = *ring;
  if (r.n && !h_len) return NS_EINVAL;
  if (r.ring_off > arena_bytes) return NS_ERANGE;
  // the slots go to 16-B-aligned staging: the host ring's own alignment is free
  ns_rx_ring r0 = r;
  r0.ring_off = 0;
  const int vr = nsh::rx_plan(r0, 0, arena_bytes - r.ring_off);
  if (vr != NS_OK) return vr;
  CallClock clk(ctx);
  if (r.n == 0) return NS_OK;
  std::lock_guard<std::mutex> lk(ctx->pmu);
  DeviceGuard g(ctx->device);
  return run_rx_host(ctx, h_arena, r, h_len, h_sums, h_verdict);
}

int ns_csum_batch_host(ns_csum_ctx* ctx, const uint8_t* h_arena, uint64_t arena_bytes,
                       const ns_pkt_desc* h_desc, uint32_t n, uint16_t* h_out,
                       uint32_t batch_flags) {
  if (!ctx || (n && (!h_desc || !h_out)) || (arena_bytes && !h_arena)) return NS_EINVAL;
  if (batch_flags & NS_BATCH_PAIRED) return NS_EINVAL;  // device-resident batches only
  CallClock clk(ctx);
  if (n == 0) return NS_OK;
  // The zero-copy pass needs the table's byte span first; an arena larger
  // than one staging buffer goes straight to the DMA pipeline, which checks
  // the descriptors as it cuts chunks (a separate pass over a 1M-descriptor
  // table cost ~1 ms of a 2.9 ms call).
  const bool maybe_small = zero_copy_enabled() && arena_bytes <= kStageBytes;
  uint64_t lo = 0, hi = 0;
  if (maybe_small) {
    const int vr = table_span(h_desc, n, arena_bytes, &lo, &hi);
    if (vr != NS_OK) return vr;
  }
  if (maybe_small && hi - lo <= kStageBytes) {
    int rc = NS_OK;
    BarBuf* st = lease_gather_stage(ctx, &rc);
    if (!st) return rc;
    if (hi > lo) std::memcpy(st->p, h_arena + lo, hi - lo);
    SmallReq rq;
    rq.dbytes = st->dev;
    rq.nbytes = hi - lo;
    rq.lo = lo;
    rq.desc = h_desc;
    rq.ndesc = n;
    rq.res = h_out;
    rq.chained = (batch_flags & NS_BATCH_CHAINED) != 0;
    rc = submit_small(ctx, &rq);
    return_gather_stage(ctx, st);
    return rc;
  }
  std::lock_guard<std::mutex> lk(ctx->pmu);
  DeviceGuard g(ctx->device);
  return run_host_batch(ctx, h_arena, arena_bytes, h_desc, n, h_out,
                        (batch_flags & NS_BATCH_CHAINED) != 0);
}

int ns_csum_checksum(ns_csum_ctx* ctx, const uint8_t* buf, uint64_t len, uint16_t initial,
                     uint16_t* out) {
  if (!ctx || !out || (len && !buf) || len > 0xFFFFFFFFull) return NS_EINVAL;
  CallClock clk(ctx);
  SpanProbe pr;
  pr.add(buf, len);
  Gather gt(ctx, pr.stage(ctx));
  const Piece pc{buf, len, true};  // one piece, odd = false: checksum.go:52-55
  gt.chain(&pc, 1, initial);
  return gt.run(out);
}

int ns_csum_vv_with_offset(ns_csum_ctx* ctx, const ns_view* views, uint32_t nviews,
                           uint16_t initial, int64_t off, int64_t size, uint16_t* out) {
  if (!ctx || !out || (nviews && !views)) return NS_EINVAL;
  CallClock clk(ctx);
  std::vector<std::pair<const uint8_t*, uint64_t>> pieces;
  int rc = clip_views(views, nviews, off, size, &pieces);
  if (rc != NS_OK) return rc;
  SpanProbe pr;
  for (const auto& pc : pieces) pr.add(pc.first, pc.second);
  Gather gt(ctx, pr.stage(ctx));
  gt.segment(pieces, initial);
  return gt.run(out);
}

int ns_csum_vv_batch(ns_csum_ctx* ctx, const ns_view* views, uint32_t nviews,
                     const ns_seg* segs, uint32_t nsegs, uint16_t* out) {
  if (!ctx || (nsegs && (!segs || !out)) || (nviews && !views)) return NS_EINVAL;
  CallClock clk(ctx);
  if (nsegs == 0) return NS_OK;
  // Every segment's clipped views as one flat list of chain pieces (a
  // segment's first piece restarts, the others continue it), so a
  // sendTCPBatch-sized call makes a few allocations, not two per segment.
  std::vector<Piece> ps;
  std::vector<uint32_t> start(nsegs + 1);
  std::vector<std::pair<const uint8_t*, uint64_t>> clipped;
  ps.reserve((size_t)nsegs * 2);
  SpanProbe pr;
  for (uint32_t q = 0; q < nsegs; ++q) {
    int rc = clip_views(views, nviews, segs[q].off, segs[q].size, &clipped);
    if (rc != NS_OK) return rc;
    start[q] = (uint32_t)ps.size();
    for (size_t k = 0; k < clipped.size(); ++k) {
      ps.push_back(Piece{clipped[k].first, clipped[k].second, k == 0});
      pr.add(clipped[k].first, clipped[k].second);
    }
  }
  start[nsegs] = (uint32_t)ps.size();
  Gather gt(ctx, pr.stage(ctx));
  for (uint32_t q = 0; q < nsegs; ++q) gt.chain(ps.data() + start[q], start[q + 1] - start[q], segs[q].initial);
  return gt.run(out);
}

int ns_csum_views_restart(ns_csum_ctx* ctx, const ns_view* views, uint32_t nviews,
                          uint16_t initial, uint16_t* out) {
  if (!ctx || !out || (nviews && !views)) return NS_EINVAL;
  CallClock clk(ctx);
  std::vector<std::pair<const uint8_t*, uint64_t>> pieces;
  SpanProbe pr;
  for (uint32_t k = 0; k < nviews; ++k) {
    if (views[k].len && !views[k].data) return NS_EINVAL;
    if (views[k].len > 0xFFFFFFFFull) return NS_EINVAL;
    pieces.emplace_back(views[k].data, views[k].len);
    pr.add(views[k].data, views[k].len);
  }
  Gather gt(ctx, pr.stage(ctx));
  gt.restart_chain(pieces, initial);
  return gt.run(out);
}

int ns_csum_chains(ns_csum_ctx* ctx, const ns_piece* pieces, uint32_t npieces, uint16_t* out,
                   uint32_t nout) {
  if (!ctx || (npieces && !pieces)) return NS_EINVAL;
  CallClock clk(ctx);
  uint32_t chains = 0;
  SpanProbe pr;
  for (uint32_t k = 0; k < npieces; ++k) {
    if (pieces[k].len && !pieces[k].data) return NS_EINVAL;
    if (pieces[k].len > 0xFFFFFFFFull) return NS_EINVAL;
    if (pieces[k].flags & NS_PIECE_END) ++chains;
    pr.add(pieces[k].data, pieces[k].len);
  }
  if (npieces && !(pieces[npieces - 1].flags & NS_PIECE_END)) return NS_EINVAL;  // unterminated
  if (chains > nout || (chains && !out)) return NS_EINVAL;
  if (chains == 0) return NS_OK;
  Gather gt(ctx, pr.stage(ctx));
  std::vector<Piece> ps;
  uint32_t start = 0;
  for (uint32_t k = 0; k < npieces; ++k) {
    ps.push_back(Piece{pieces[k].data, pieces[k].len, (pieces[k].flags & NS_PIECE_RESTART) != 0});
    if (pieces[k].flags & NS_PIECE_END) {
      ps[0].restart = true;  // a chain starts fresh: sum = initial, odd = false
      gt.chain(ps.data(), ps.size(), pieces[start].initial);
      ps.clear();
      start = k + 1;
    }
  }
  return gt.run(out);
}

int ns_csum_pseudo_header(ns_csum_ctx* ctx, uint32_t protocol, const uint8_t* src,
                          uint32_t src_len, const uint8_t* dst, uint32_t dst_len,
                          uint16_t total_len, uint16_t* out) {
  if (!ctx || !out || (src_len && !src) || (dst_len && !dst)) return NS_EINVAL;
  CallClock clk(ctx);
  // checksum.go:112-122: four chained Checksum calls, each restarting alignment.
  const uint8_t lenbe[2] = {(uint8_t)(total_len >> 8), (uint8_t)total_len};
  const uint8_t proto[2] = {0, (uint8_t)protocol};
  std::vector<std::pair<const uint8_t*, uint64_t>> pieces = {
      {src, src_len}, {dst, dst_len}, {lenbe, 2}, {proto, 2}};
  Gather gt(ctx);
  gt.restart_chain(pieces, 0);
  return gt.run(out);
}

int ns_csum_stage_acquire(ns_csum_ctx* ctx, uint64_t bytes, uint8_t** base) {
  if (!ctx || !base) return NS_EINVAL;
  *base = nullptr;
  int rc = NS_OK;
  MappedPin* b = bytes <= kStageBytes ? lease_stage(ctx, &rc) : lease_big(ctx, bytes, &rc);
  if (!b) return rc != NS_OK ? rc : NS_ENOMEM;
  {
    std::lock_guard<std::mutex> ql(ctx->qmu);
    ctx->leased.push_back(b);
  }
  *base = b->p;
  return NS_OK;
}

int ns_csum_stage_release(ns_csum_ctx* ctx, uint8_t* base) {
  if (!ctx || !base) return NS_EINVAL;
  std::lock_guard<std::mutex> ql(ctx->qmu);
  for (size_t i = 0; i < ctx->leased.size(); ++i) {
    MappedPin* b = ctx->leased[i];
    if (b->p != base) continue;
    ctx->leased.erase(ctx->leased.begin() + (long)i);
    if (b->cap == kStageBytes) ctx->stage_free.push_back(b);
    else ctx->big_free.push_back(b);
    return NS_OK;
  }
  return NS_EINVAL;
}

int ns_csum_packet_buffers(ns_csum_ctx* ctx, const ns_pkt_buf* pkts, uint32_t n, uint32_t op,
                           uint16_t* sums, uint8_t* verdict) {
  if (!ctx || (n && !pkts) || (op != NS_PKB_VERIFY && op != NS_PKB_FILL)) return NS_EINVAL;
  CallClock clk(ctx);
  if (n == 0) return NS_OK;
  std::vector<nsh::PacketBytes> pb(n);
  SpanProbe pr;
  for (uint32_t i = 0; i < n; ++i) {
    const int rc = pb[i].init(pkts[i]);
    if (rc != NS_OK) return rc;
    for (const auto& sg : pb[i].seg) pr.add(sg.first, sg.second);
  }
  Gather gt(ctx, pr.stage(ctx));
  gt.desc.reserve((size_t)n * 4);  // IP header + transport chain pieces, typically
  gt.result_at.reserve((size_t)n * 2);
  std::vector<nsh::PacketPlan> plan(n);
  for (uint32_t i = 0; i < n; ++i) {
    const int rc = nsh::plan_packet(gt, pb[i], op, &plan[i]);
    if (rc != NS_OK) return rc;
  }
  std::vector<uint16_t> res(gt.result_at.size());
  if (!res.empty()) {
    const int rc = gt.run(res.data());
    if (rc != NS_OK) return rc;
  }
  for (uint32_t i = 0; i < n; ++i)
    nsh::finish_packet(pb[i], plan[i], op, res.data(), sums ? sums + 2 * i : nullptr, verdict ? verdict + i : nullptr);
  return NS_OK;
}

int ns_csum_batch_multi(ns_csum_ctx* const* ctxs, uint32_t nctx, const uint8_t* h_arena,
                        uint64_t arena_bytes, const ns_pkt_desc* h_desc, uint32_t n,
                        uint16_t* h_out, uint32_t batch_flags) {
  if (!ctxs || nctx == 0 || (n && (!h_desc || !h_out)) || (arena_bytes && !h_arena)) return NS_EINVAL;
  for (uint32_t c = 0; c < nctx; ++c)
    if (!ctxs[c]) return NS_EINVAL;
  for (uint32_t i = 0; i < n; ++i) {
    const uint64_t off = h_desc[i].off, len = h_desc[i].len;
    if (off > arena_bytes || len > arena_bytes - off) return NS_ERANGE;
  }
  std::vector<uint32_t> first(nctx + 1);
  int rc = ns_csum_shard_plan(h_desc, n, nctx, first.data());
  if (rc != NS_OK) return rc;
  // One host thread per shard (per device context); each runs the pipelined
  // host path on its own streams.  Shards are independent: no collective.
  std::vector<int> status(nctx, NS_OK);
  std::vector<std::thread> th;
  th.reserve(nctx);
  for (uint32_t c = 0; c < nctx; ++c) {
    th.emplace_back([&, c]() {
      const uint32_t lo = first[c], hi = first[c + 1];
      if (hi <= lo) return;
      status[c] = ns_csum_batch_host(ctxs[c], h_arena, arena_bytes, h_desc + lo, hi - lo,
                                     h_out + lo, batch_flags);
    });
  }
  for (auto& t : th) t.join();
  for (uint32_t c = 0; c < nctx; ++c)
    if (status[c] != NS_OK) return status[c];
  return NS_OK;
}

int ns_csum_tcp_tx_host_multi(ns_csum_ctx* const* ctxs, uint32_t nctx, uint8_t* h_arena, uint64_t arena_bytes,
                              const ns_tcp_tx* txs, uint32_t count, uint16_t* h_out) {
  if (!ctxs || nctx == 0 || (count && !txs) || (arena_bytes && !h_arena)) return NS_EINVAL;
  for (uint32_t c = 0; c < nctx; ++c)
    if (!ctxs[c]) return NS_EINVAL;
  std::vector<nsh::TxPlan> plans;
  const int vr = nsh::tx_multi_plan(txs, count, arena_bytes, &plans);
  if (vr != NS_OK) return vr;
  std::vector<std::vector<ns_tcp_tx>> parts;
  std::vector<uint64_t> seg0;
  nsh::tx_shard_calls(txs, count, plans, nctx, &parts, &seg0);
  // One host thread per part (per device context), each running the host TX
  // pipeline on its own context's streams.  Parts are independent (each
  // segment's fields depend on its own bytes): no collective.
  std::vector<int> status(nctx, NS_OK);
  std::vector<std::thread> th;
  th.reserve(nctx);
  for (uint32_t c = 0; c < nctx; ++c) {
    if (parts[c].empty()) continue;
    th.emplace_back([&, c]() {
      status[c] = ns_csum_tcp_tx_host(ctxs[c], h_arena, arena_bytes, parts[c].data(), (uint32_t)parts[c].size(),
                                      h_out ? h_out + 2 * seg0[c] : nullptr);
    });
  }
  for (auto& t : th) t.join();
  for (uint32_t c = 0; c < nctx; ++c)
    if (status[c] != NS_OK) return status[c];
  return NS_OK;
}

int ns_csum_get_stats(ns_csum_ctx* ctx, ns_csum_stats* out, int reset) {
  if (!ctx || !out) return NS_EINVAL;
  StatCounters& c = ctx->st;
  std::atomic<uint64_t>* src[] = {&c.calls,          &c.call_ns_max,   &c.lock_ns_max,    &c.zc_passes, &c.zc_late,
                                  &c.zc_pass_ns_max, &c.growths,       &c.growth_ns_total, &c.growth_ns_max,
                                  &c.retires,        &c.retire_ns_max, &c.stage_allocs,   &c.stage_alloc_ns_max};
  static_assert(sizeof(ns_csum_stats) == sizeof(src) / sizeof(src[0]) * sizeof(uint64_t), "ns_csum_stats fields");
  uint64_t* dst = reinterpret_cast<uint64_t*>(out);
  for (size_t i = 0; i < sizeof(src) / sizeof(src[0]); ++i)
    dst[i] = reset ? src[i]->exchange(0, std::memory_order_relaxed) : src[i]->load(std::memory_order_relaxed);
  return NS_OK;
}

int ns_csum_shard_plan(const ns_pkt_desc* h_desc, uint32_t n, uint32_t parts, uint32_t* first) {
  if (!first || parts == 0 || (n && !h_desc)) return NS_EINVAL;
  nsh::shard_plan(h_desc, n, parts, first);
  return NS_OK;
}

}  // extern "C"
