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
#include "netstack_csum.h"

static_assert(sizeof(ns_pkt_desc) == 16, "ns_pkt_desc must be 16 bytes");
static_assert(sizeof(ns_seg) == 24, "ns_seg layout");
static_assert(sizeof(ns_piece) == 24, "ns_piece layout");
static_assert(sizeof(ns_pkt_buf) == 40, "ns_pkt_buf layout");

namespace {

// Largest run of VectorisedView pieces that may be merged into ONE descriptor
// and still equal Go's per-view chain (checksum.go:89): with initial <= 0xFFFF
// and L <= 131072 bytes the uint32 accumulator cannot wrap, neither in the
// chain nor in the merged sum (65535 * (1 + 65536) = 2^32 - 1).  A single
// piece is never split (its own wrap is reproduced exactly by the kernel).
constexpr uint64_t kMergeMax = 131072;
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
  nsk::ChainScratch get() const { return nsk::ChainScratch{part.p, status.p}; }
  void release() {
    part.release();
    status.release();
  }
};

// Scratch of the device-resident API for one caller stream: chained batches
// and huge-descriptor splits on different streams of one context run
// concurrently, each on its own scratch (the same stream orders its own).
struct StreamScratch {
  hipStream_t stream = nullptr;
  ChainBuf chain;
  DevBuf<uint32_t> split;  // csum_split accumulators (zero between launches)
};

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
// A pass's [table | results] buffer; a pass takes queued requests while they fit.
constexpr uint64_t kPassTableBytes = 1ull << 20;
// The "arena" of a zero-copy pass is the address space: descriptors hold
// absolute device addresses (the kernel's per-tile windows take it from there).
constexpr uint64_t kWholeSpace = 1ull << 60;

}  // namespace

struct ns_csum_ctx {
  int device = 0;
  uint64_t staging = kDefaultStaging;
  hipStream_t stream[2] = {nullptr, nullptr};
  hipEvent_t done[2] = {nullptr, nullptr};
  unsigned long long* d_err = nullptr;
  std::mutex mu;  // guards everything below

  // device-resident API scratch, one per caller stream (allocated on first use)
  std::vector<StreamScratch*> scratch;
  // ns_csum_sync's exchanged error count (mapped: written by take_err)
  MappedPin err_taken;
  // host-path slots (double-buffered)
  DevBuf<uint8_t> d_arena[2];
  DevBuf<ns_pkt_desc> d_desc[2];
  DevBuf<uint16_t> d_out[2];
  ChainBuf d_chain[2];
  PinBuf<ns_pkt_desc> h_desc[2];
  PinBuf<uint16_t> h_out[2];
  // zero-copy pass buffer for small calls: [table | results]
  MappedPin z_buf;
  // flat combining of concurrent small calls (submit_small) and the pool of
  // mapped staging buffers they gather into; guarded by qmu
  std::mutex qmu;
  std::condition_variable qcv;
  std::vector<SmallReq*> pending;
  bool combining = false;
  std::vector<MappedPin*> stage_free;
  std::vector<MappedPin*> stage_all;
  std::vector<MappedPin*> big_free;  // pooled caller stages above kStageBytes
  std::vector<MappedPin*> leased;    // stages a caller holds (ns_csum_stage_acquire)
  // gather staging for the VectorisedView entry points
  PinBuf<uint8_t> g_arena;
  std::vector<ns_pkt_desc> g_desc;
};

namespace {

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

bool any_cont(const ns_pkt_desc* d, uint32_t n) {
  for (uint32_t i = 0; i < n; ++i)
    if (d[i].flags & NS_DESC_CONT) return true;
  return false;
}

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
  const uint64_t o_off = nd * sizeof(ns_pkt_desc);
  int rc;
  if ((rc = ctx->z_buf.ensure(std::max<uint64_t>(kPassTableBytes, o_off + nd * 2))) != NS_OK) return rc;
  if (chained && (rc = ctx->d_chain[0].ensure(nd)) != NS_OK) return rc;
  uint8_t* z = ctx->z_buf.p;
  ns_pkt_desc* zd = reinterpret_cast<ns_pkt_desc*>(z);
  uint64_t k = 0;
  for (size_t r = 0; r < nreq; ++r) {
    const SmallReq& q = *reqs[r];
    const uint64_t base = (uint64_t)(uintptr_t)q.dbytes;
    for (uint32_t i = 0; i < q.ndesc; ++i, ++k) {
      zd[k] = q.desc[i];
      zd[k].off = zd[k].len ? base + (zd[k].off - q.lo) : 0;
      if (!q.chained) {
        zd[k].flags &= (uint16_t)~NS_DESC_CONT;  // independent in an unchained batch
      } else if (i == 0 && (zd[k].flags & NS_DESC_CONT)) {
        // A batch's first descriptor heads its run even when flagged CONT
        // (with initial 0, fold_scan): keep that inside a combined pass.
        zd[k].flags &= (uint16_t)~NS_DESC_CONT;
        zd[k].initial = 0;
      }
    }
  }
  uint8_t* zdev = ctx->z_buf.dev;
  hipStream_t s = ctx->stream[0];
  HIP_TRY(nsk::launch_batch(nullptr, kWholeSpace, zdev, (uint32_t)nd, reinterpret_cast<uint16_t*>(zdev + o_off),
                            chained ? ctx->d_chain[0].get() : nsk::ChainScratch{}, ctx->d_err, s,
                            std::max<uint64_t>(nb, 1)));
  HIP_TRY(hipStreamSynchronize(s));
  const uint16_t* res = reinterpret_cast<const uint16_t*>(z + o_off);
  for (size_t r = 0; r < nreq; ++r) {
    std::memcpy(reqs[r]->res, res, (size_t)reqs[r]->ndesc * 2);
    res += reqs[r]->ndesc;
  }
  return NS_OK;
}

// Lease / return a mapped staging buffer of kStageBytes from the context's pool.
MappedPin* lease_stage(ns_csum_ctx* ctx, int* rc) {
  {
    std::lock_guard<std::mutex> ql(ctx->qmu);
    if (!ctx->stage_free.empty()) {
      MappedPin* b = ctx->stage_free.back();
      ctx->stage_free.pop_back();
      return b;
    }
  }
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

void return_stage(ns_csum_ctx* ctx, MappedPin* b) {
  if (!b) return;
  std::lock_guard<std::mutex> ql(ctx->qmu);
  ctx->stage_free.push_back(b);
}

// Flat combining of concurrent small synchronous calls.  netstack calls the
// checksum from every endpoint's goroutine at once; one
// launch + wait costs ~15-20 us whatever its size, so serialising calls on
// the context would cap a context at ~50K calls/s.  Instead a caller queues
// its request; if no pass is running it becomes the combiner: it takes every
// queued request (while their tables fit kPassTableBytes), runs them as ONE
// zero-copy pass, hands out the results and repeats while requests remain.
// Each caller has already gathered its bytes into its own leased staging, so
// the only serial host work per request is copying its descriptors.
// Everyone else sleeps until its request is done.  Results are identical to
// separate calls (descriptors are independent; chains never cross requests).
int submit_small(ns_csum_ctx* ctx, SmallReq* req) {
  // A combiner keeps serving queued requests after its own is done, up to
  // kMaxPasses passes, so back-to-back passes do not wait for a sleeping
  // thread to wake up and take the role over.
  constexpr int kMaxPasses = 8;
  std::unique_lock<std::mutex> ql(ctx->qmu);
  ctx->pending.push_back(req);
  while (!req->done.load(std::memory_order_acquire)) {
    if (ctx->combining) {
      // Spin briefly (a pass is ~20-60 us) before sleeping: a woken thread
      // costs more than the spin.
      ql.unlock();
      const auto t0 = std::chrono::steady_clock::now();
      while (!req->done.load(std::memory_order_acquire) &&
             std::chrono::steady_clock::now() - t0 < std::chrono::microseconds(50))
        std::this_thread::yield();
      ql.lock();
      if (req->done.load(std::memory_order_acquire)) break;
      if (ctx->combining) ctx->qcv.wait(ql);
      continue;
    }
    ctx->combining = true;
    for (int pass = 0; pass < kMaxPasses && !ctx->pending.empty(); ++pass) {
      std::vector<SmallReq*> take;
      uint64_t staged = 0;
      size_t i = 0;
      for (; i < ctx->pending.size(); ++i) {
        const uint64_t sz = ctx->pending[i]->table_bytes();
        if (!take.empty() && staged + sz > kPassTableBytes) break;
        take.push_back(ctx->pending[i]);
        staged += sz;
      }
      ctx->pending.erase(ctx->pending.begin(), ctx->pending.begin() + (long)i);
      ql.unlock();
      int rc;
      {
        std::lock_guard<std::mutex> lk(ctx->mu);
        DeviceGuard g(ctx->device);
        rc = run_zero_copy(ctx, take.data(), take.size());
      }
      for (SmallReq* t : take) {
        t->rc = rc;
        t->done.store(true, std::memory_order_release);
      }
      ql.lock();
      ctx->qcv.notify_all();
      if (req->done.load(std::memory_order_relaxed) && pass + 1 >= kMaxPasses) break;
    }
    ctx->combining = false;
    ctx->qcv.notify_all();  // a waiter takes the role over if requests remain
  }
  return req->rc;
}

// Host batch core, caller holds ctx->mu and the device guard.  Pipelines
// chunks of the descriptor table over the two slots/streams: H2D of chunk k+1
// overlaps the kernel of chunk k.  Chunks never split a NS_DESC_CONT run.
// Descriptors per host-pipeline chunk (cfg3, 1M x 64 B: 64K 3.11 ms, 128K
// 2.18, 256K 2.16, 512K 2.52 ms per call).
constexpr uint32_t kHostChunkDesc = 1u << 17;

int run_host_batch(ns_csum_ctx* ctx, const uint8_t* h_arena, uint64_t arena_bytes,
                   const ns_pkt_desc* h_desc, uint32_t n, uint16_t* h_out,
                   bool chained) {
  if (n == 0) return NS_OK;
  const uint64_t budget = ctx->staging;
  struct Pending {
    bool live = false;
    uint32_t first = 0, count = 0;
  } pend[2];
  // Drain whatever is in flight (on an error return too: the staging
  // buffers must be idle before the next call reuses them).
  auto drain = [&](int slot) -> int {
    for (int s = 0; s < 2; ++s) {
      const int sl = slot ^ s ^ 1;  // older chunk first
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
    // Grow the chunk while its byte span stays within budget and it holds at
    // most kHostChunkDesc descriptors (so that the CPU's table copy of one
    // chunk overlaps the other chunk's transfers).  Descriptors are
    // range-checked on the way.  1M x 64 B: 4.27 ms -> 2.15 ms per call
    // with this, the skipped span pass and the device-side table rebase
    // (profiles/r01/bench_host3.json).
    uint64_t lo = UINT64_MAX, hi = 0;
    uint32_t j = k;
    uint32_t cut = k;  // last index (exclusive) at which we may cut
    uint64_t cut_lo = 0, cut_hi = 0;
    while (j < n) {
      const uint64_t off = h_desc[j].off, len = h_desc[j].len;
      if (off > arena_bytes || len > arena_bytes - off) {
        const int rc = drain(slot);
        return rc != NS_OK ? rc : NS_ERANGE;
      }
      uint64_t nlo = lo, nhi = hi;  // empty descriptors do not widen the span
      if (len) {
        nlo = std::min(lo, off);
        nhi = std::max(hi, off + len);
      }
      if (j > k && cut > k && ((nlo != UINT64_MAX && nhi - nlo > budget) || j - k >= kHostChunkDesc)) break;
      lo = nlo;
      hi = nhi;
      ++j;
      if (j == n || !(chained && (h_desc[j].flags & NS_DESC_CONT))) {
        cut = j;
        cut_lo = lo;
        cut_hi = hi;
      }
    }
    if (cut == k) {  // only possible at the end: take everything left
      cut = j;
      cut_lo = lo;
      cut_hi = hi;
    }
    const uint32_t cnt = cut - k;
    if (cut_lo == UINT64_MAX || cut_hi < cut_lo) cut_lo = cut_hi = 0;
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
      if ((rc = ctx->d_out[slot].ensure(cnt)) != NS_OK) return rc;
      if ((rc = ctx->h_desc[slot].ensure(cnt)) != NS_OK) return rc;
      if ((rc = ctx->h_out[slot].ensure(cnt)) != NS_OK) return rc;
      if (chained && (rc = ctx->d_chain[slot].ensure(cnt)) != NS_OK) return rc;
      // The table goes over verbatim (one memcpy into pinned memory) and is
      // rebased to the chunk on the device: a per-descriptor rewrite on the
      // CPU was the limit of small-packet batches.
      ns_pkt_desc* hd = ctx->h_desc[slot].p;
      std::memcpy(hd, h_desc + k, (size_t)cnt * sizeof(ns_pkt_desc));
      hipStream_t s = ctx->stream[slot];
      if (span) HIP_TRY(hipMemcpyAsync(ctx->d_arena[slot].p, h_arena + cut_lo, span, hipMemcpyHostToDevice, s));
      HIP_TRY(hipMemcpyAsync(ctx->d_desc[slot].p, hd, cnt * sizeof(ns_pkt_desc), hipMemcpyHostToDevice, s));
      HIP_TRY(nsk::launch_rebase(ctx->d_desc[slot].p, cnt, cut_lo, s));
      HIP_TRY(nsk::launch_batch(ctx->d_arena[slot].p, span, ctx->d_desc[slot].p, cnt, ctx->d_out[slot].p,
                                chained ? ctx->d_chain[slot].get() : nsk::ChainScratch{}, ctx->d_err, s));
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
    slot ^= 1;
  }
  return drain(slot);
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
// the call ends, into the context's pinned arena `g_arena` (grown by doubling
// and kept between calls) and takes the DMA pipeline: one CPU copy per byte
// either way (a 64 MiB VectorisedView batch went from 31 ms through a
// growing std::vector to a few ms; tools/latency.cc).  A gather whose bytes
// already lie in a caller's acquired stage copies nothing: its descriptors
// address that stage (adopt mode).
struct ByteSink {
  ns_csum_ctx* ctx;
  MappedPin* stage = nullptr;    // leased from the pool (copy mode)
  MappedPin* adopted = nullptr;  // the caller's acquired stage (adopt mode)
  std::unique_lock<std::mutex> big;  // held once the bytes live in ctx->g_arena
  uint64_t n = 0;  // copy: bytes appended; adopt: end of the highest byte used
  int rc = NS_OK;
  explicit ByteSink(ns_csum_ctx* c, MappedPin* adopt = nullptr) : ctx(c), adopted(adopt) {
    if (adopted) return;
    if (zero_copy_enabled()) stage = lease_stage(ctx, &rc);
    if (!stage) rc = to_big(0);
  }
  ~ByteSink() { return_stage(ctx, stage); }
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
  // Move to g_arena (taking the context lock) with room for `need` bytes.
  int to_big(uint64_t need) {
    big = std::unique_lock<std::mutex>(ctx->mu);
    const int r = reserve_big(std::max<uint64_t>(need, 1ull << 20), 0);
    if (r == NS_OK && n) std::memcpy(ctx->g_arena.p, stage->p, n);
    return r;
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
    if (!in_big() && n + len > stage->cap) rc = to_big(n + len);
    else if (in_big()) rc = reserve_big(n + len, n);
    if (rc != NS_OK) return at;
    std::memcpy(base() + n, p, len);
    n += len;
    return at;
  }
};

// One piece of a checksum chain: `restart` = a fresh Checksum(piece, xsum)
// (alignment restarts, checksum.go:52-55); otherwise the piece continues the
// previous piece's byte stream with its odd-byte carry (the view chaining of
// ChecksumVVWithOffset, checksum.go:89).
struct Piece {
  const uint8_t* p;
  uint64_t len;
  bool restart;
};

// ---- gather of VectorisedView pieces (tcpip/buffer -> staging arena) -----
struct Gather {
  ns_csum_ctx* ctx;
  ByteSink bytes;  // assembled in mapped staging (or spilled host memory)
  std::vector<ns_pkt_desc> desc;
  std::vector<uint32_t> result_at;  // index of the descriptor holding each result
  explicit Gather(ns_csum_ctx* c, MappedPin* adopt = nullptr) : ctx(c), bytes(c, adopt) {}

  // One chain (include/netstack_csum.h, ns_csum_chains): sum = initial,
  // odd = false; per piece (sum, odd) = calculateChecksum(piece, odd', sum)
  // with odd' = false on a restart piece.  Continue pieces that follow each
  // other in the arena merge into the open descriptor up to kMergeMax bytes
  // (exact, see kMergeMax); a restart piece opens a new descriptor with
  // odd = 0; empty pieces are skipped (checksum.go:73-75; Checksum(empty, x)
  // == x).  A piece is never split: its own > 128 KiB wrap is reproduced
  // exactly by the kernel.
  void chain(const Piece* p, size_t np, uint16_t initial) {
    bool first_desc = true;
    uint32_t parity = 0;  // odd flag carried to the next continue piece
    ns_pkt_desc cur{};
    bool open = false;
    auto close = [&]() {
      if (!open) return;
      desc.push_back(cur);
      open = false;
    };
    for (size_t k = 0; k < np; ++k) {
      const uint64_t len = p[k].len;
      if (p[k].restart) {
        close();
        parity = 0;
      }
      if (len == 0) continue;
      const bool big = len > kMergeMax;
      const uint64_t at = bytes.append(p[k].p, len);
      if (open && (big || cur.len + len > kMergeMax || at != cur.off + cur.len)) close();
      if (!open) {
        cur.off = at;
        cur.len = 0;
        cur.initial = first_desc ? initial : 0;
        cur.flags = (uint16_t)((first_desc ? 0u : NS_DESC_CONT) | (parity ? NS_DESC_ODD : 0u));
        first_desc = false;
        open = true;
      }
      cur.len += (uint32_t)len;
      parity ^= (uint32_t)(len & 1);
      if (big) close();
    }
    close();
    if (first_desc) {  // no bytes at all: result = initial (checksum.go:97)
      ns_pkt_desc z{};
      z.initial = initial;
      desc.push_back(z);
    }
    result_at.push_back((uint32_t)desc.size() - 1);
  }

  // ChecksumVVWithOffset's view walk over already clipped pieces: the first
  // restarts, the rest continue (checksum.go:69-98).
  void segment(const std::vector<std::pair<const uint8_t*, uint64_t>>& pieces, uint16_t initial) {
    std::vector<Piece> ps;
    ps.reserve(pieces.size());
    for (size_t k = 0; k < pieces.size(); ++k) ps.push_back(Piece{pieces[k].first, pieces[k].second, k == 0});
    chain(ps.data(), ps.size(), initial);
  }

  // Each view its own calculateChecksum with odd=false, chained
  // (xsum = Checksum(v, xsum): udp/endpoint.go:811-813).
  void restart_chain(const std::vector<std::pair<const uint8_t*, uint64_t>>& pieces, uint16_t initial) {
    std::vector<Piece> ps;
    ps.reserve(pieces.size());
    for (const auto& pc : pieces) ps.push_back(Piece{pc.first, pc.second, true});
    chain(ps.data(), ps.size(), initial);
  }

  int run(uint16_t* out) {
    if (bytes.rc != NS_OK) return bytes.rc;
    std::vector<uint16_t> res(desc.size());
    int rc;
    const bool chained = any_cont(desc.data(), (uint32_t)desc.size());
    if (bytes.adopted && !(zero_copy_enabled() && bytes.size() <= kStageBytes)) {
      // A large caller stage: pinned already, so the DMA pipeline reads it.
      std::lock_guard<std::mutex> lk(ctx->mu);
      DeviceGuard g(ctx->device);
      rc = run_host_batch(ctx, bytes.base(), bytes.size(), desc.data(), (uint32_t)desc.size(), res.data(),
                          chained);
    } else if (!bytes.in_big()) {
      // Small: zero-copy from the leased (or the caller's) staging, combined
      // with concurrent calls.
      SmallReq rq;
      rq.dbytes = bytes.adopted ? bytes.adopted->dev : bytes.stage->dev;
      rq.nbytes = bytes.size();
      rq.desc = desc.data();
      rq.ndesc = (uint32_t)desc.size();
      rq.res = res.data();
      rq.chained = chained;
      rc = submit_small(ctx, &rq);
    } else {
      // Large: the bytes are in the pinned g_arena and ctx->mu is held.
      DeviceGuard g(ctx->device);
      rc = run_host_batch(ctx, ctx->g_arena.p, bytes.size(), desc.data(), (uint32_t)desc.size(), res.data(),
                          chained);
    }
    if (rc != NS_OK) return rc;
    for (size_t q = 0; q < result_at.size(); ++q) out[q] = res[result_at[q]];
    return NS_OK;
  }
};

// Clip a VectorisedView to [off, off+size) exactly like checksum.go:72-96.
int clip_views(const ns_view* views, uint32_t nviews, int64_t off, int64_t size,
               std::vector<std::pair<const uint8_t*, uint64_t>>* pieces) {
  if (off < 0 || size < 0) return NS_EINVAL;
  pieces->clear();
  uint64_t o = (uint64_t)off, s = (uint64_t)size;
  for (uint32_t k = 0; k < nviews; ++k) {
    const uint64_t vl = views[k].len;
    if (vl == 0) continue;  // :73-75
    if (!views[k].data) return NS_EINVAL;
    if (o >= vl) {  // :77-80
      o -= vl;
      continue;
    }
    const uint64_t l = std::min<uint64_t>(vl - o, s);  // :81-87
    if (l > 0xFFFFFFFFull) return NS_EINVAL;
    pieces->emplace_back(views[k].data + o, l);
    s -= l;  // :91-94
    if (s == 0) break;
    o = 0;
  }
  return NS_OK;
}

// ---- tcpip.PacketBuffer batches (ns_csum_packet_buffers) -------------------
// A packet as one byte stream: its Header bytes, then its Data views clipped
// to Data.Size() (packet_buffer.go:25-50).  The host reads header fields from
// it (plumbing: lengths, addresses' positions, protocol numbers) and cuts it
// into the pieces of each reference call sequence; every sum is computed by
// the kernel.
struct PacketBytes {
  std::vector<std::pair<const uint8_t*, uint64_t>> seg;  // non-empty segments in order
  std::vector<uint64_t> at;                             // byte offset of each segment
  uint64_t size = 0;
  uint64_t hdr_len = 0;  // bytes [0, hdr_len) are the Header's (writable)

  int init(const ns_pkt_buf& pk) {
    if (pk.hdr_len && !pk.hdr) return NS_EINVAL;
    hdr_len = pk.hdr_len;
    if (pk.ndata && !pk.data) return NS_EINVAL;
    add(pk.hdr, pk.hdr_len);
    uint64_t left = pk.data_size;
    for (uint32_t k = 0; k < pk.ndata && left; ++k) {
      const uint64_t l = std::min<uint64_t>(pk.data[k].len, left);
      if (l && !pk.data[k].data) return NS_EINVAL;
      add(pk.data[k].data, l);
      left -= l;
    }
    return NS_OK;
  }
  void add(const uint8_t* p, uint64_t l) {
    if (!l) return;
    seg.emplace_back(p, l);
    at.push_back(size);
    size += l;
  }
  // Segment holding byte k (k < size).
  size_t seg_of(uint64_t k) const {
    size_t lo = 0, hi = seg.size();
    while (hi - lo > 1) {
      const size_t mid = (lo + hi) / 2;
      if (at[mid] <= k) lo = mid;
      else hi = mid;
    }
    return lo;
  }
  // End of the segment (view) holding byte k: "Data.First()" after a trim to k.
  uint64_t seg_end(uint64_t k) const {
    if (k >= size) return size;
    const size_t s = seg_of(k);
    return at[s] + seg[s].second;
  }
  bool read(uint64_t k, uint8_t* out, uint64_t n) const {
    if (k + n > size) return false;
    while (n) {
      const size_t s = seg_of(k);
      const uint64_t o = k - at[s], l = std::min<uint64_t>(n, seg[s].second - o);
      std::memcpy(out, seg[s].first + o, l);
      out += l;
      k += l;
      n -= l;
    }
    return true;
  }
  uint8_t* mut(uint64_t k) const {  // address of byte k (a Header byte for stores)
    const size_t s = seg_of(k);
    return const_cast<uint8_t*>(seg[s].first) + (k - at[s]);
  }
  // Pieces covering [a, b), cut at view boundaries: the first `first_restart`,
  // then each next view restarting (`per_view`, the `xsum = Checksum(v, xsum)`
  // loops) or continuing (ChecksumVV's view walk).
  void pieces(uint64_t a, uint64_t b, bool first_restart, bool per_view, std::vector<Piece>* out) const {
    bool first = true;
    while (a < b) {
      const size_t s = seg_of(a);
      const uint64_t o = a - at[s], l = std::min<uint64_t>(b - a, seg[s].second - o);
      out->push_back(Piece{seg[s].first + o, l, first ? first_restart : per_view});
      first = false;
      a += l;
    }
  }
};

constexpr uint8_t kProtoICMPv4 = 1, kProtoTCP = 6, kProtoUDP = 17, kProtoICMPv6 = 58;

// One packet's plan: up to two chains (network header, transport) and where
// their results go.
struct PacketPlan {
  int net_chain = -1, tr_chain = -1;  // result indices in the Gather
  uint8_t verdict = NS_PKB_UNCHECKED;
  uint8_t kind = 0;                   // transport protocol for the verdict
  uint64_t net_store = UINT64_MAX, tr_store = UINT64_MAX;  // FILL: field offsets
  uint16_t field = 0;                 // VERIFY (ICMP): the received checksum field
};

// ChecksumCombine (checksum.go:104-107): folds the pseudo-header's length and
// protocol words into the initial of the address piece.  The pseudo-header
// pieces are all even-length restarts, so any grouping of them gives Go's
// value (both are fold1 of the same total, and 0 only when all
// pieces are 0).
uint16_t combine(uint16_t a, uint16_t b) { return ns_csum_combine(a, b); }

// The IP layer of a packet: header length, transport range and protocol, the
// pseudo-header address bytes.  Returns false for what IPv4/IPv6 IsValid
// (header/ipv4.go:280-296, ipv6.go:207-222) and HandlePacket reject.
struct IpInfo {
  bool v4 = false;
  uint64_t hlen = 0, tbeg = 0, tend = 0, addr = 0, addr_len = 0;
  uint8_t proto = 0;
  bool fragment = false;
};

bool parse_ip(const PacketBytes& pb, bool rx, IpInfo* ip) {
  uint8_t h[40];
  if (pb.size < 1 || !pb.read(0, h, 1)) return false;
  const uint8_t ver = h[0] >> 4;
  // RX: the network header lies in Data.First() (packet_buffer.go:27-29);
  // IsValid looks at that view alone.
  const uint64_t first = pb.seg_end(0);
  if (ver == 4) {
    if ((rx && first < 20) || !pb.read(0, h, 20)) return false;
    ip->v4 = true;
    ip->hlen = (uint64_t)(h[0] & 0xF) * 4;
    const uint64_t tlen = ((uint64_t)h[2] << 8) | h[3];
    if (rx) {
      if (ip->hlen < 20 || ip->hlen > tlen || tlen > pb.size || ip->hlen > first) return false;
      ip->tend = tlen;  // Data.CapLength(tlen - hlen), ipv4.go:353
    } else {
      if (ip->hlen < 20 || ip->hlen > pb.size) return false;
      ip->tend = pb.size;
    }
    ip->proto = h[9];
    ip->addr = 12;
    ip->addr_len = 8;
    ip->fragment = (h[6] & 0x20) || (((h[6] & 0x1F) << 8) | h[7]);  // MF or a fragment offset
  } else if (ver == 6) {
    if ((rx && first < 40) || !pb.read(0, h, 40)) return false;
    ip->hlen = 40;
    const uint64_t plen = ((uint64_t)h[4] << 8) | h[5];
    if (rx) {
      if (plen > pb.size - 40) return false;
      ip->tend = 40 + plen;  // Data.CapLength(PayloadLength), ipv6.go:177
    } else {
      ip->tend = pb.size;
    }
    ip->proto = h[6];
    ip->addr = 8;
    ip->addr_len = 32;
  } else {
    return false;
  }
  ip->tbeg = ip->hlen;
  return true;
}

// Builds one packet's chains into g.  RX (NS_PKB_VERIFY) mirrors the receive
// path's checks; TX (NS_PKB_FILL) the transmit path's sums (see the header).
int plan_packet(Gather& g, const PacketBytes& pb, uint32_t op, PacketPlan* pp) {
  IpInfo ip;
  const bool rx = op == NS_PKB_VERIFY;
  if (!parse_ip(pb, rx, &ip)) {
    if (rx) {
      pp->verdict = NS_PKB_MALFORMED;
      return NS_OK;
    }
    return NS_EINVAL;
  }
  std::vector<Piece> ps;
  const int nres = (int)g.result_at.size();
  auto add_chain = [&](uint16_t init) {
    g.chain(ps.data(), ps.size(), init);
    ps.clear();
    return (int)g.result_at.size() - 1;
  };
  if (ip.v4 && !rx) {
    // addIPHeader: ip.SetChecksum(^ip.CalculateChecksum()) (ipv4.go:236),
    // CalculateChecksum = Checksum(b[:HeaderLength()], 0) (ipv4.go:251-253)
    pb.pieces(0, ip.hlen, true, false, &ps);
    pp->net_chain = add_chain(0);
    pp->net_store = 10;
  } else if (ip.v4) {
    // not verified on receive in the reference; reported for the caller
    pb.pieces(0, ip.hlen, true, false, &ps);
    pp->net_chain = add_chain(0);
  }
  (void)nres;
  const uint64_t t0 = ip.tbeg, te = ip.tend, tl = te - t0;
  const uint64_t first_end = std::min(pb.seg_end(t0), te);  // Data.First() after the IP trim
  pp->kind = ip.proto;
  auto pseudo = [&](uint8_t proto, uint64_t len, bool icmpv6) -> uint16_t {
    // PseudoHeaderChecksum (checksum.go:112-122) / ICMPv6Checksum's
    // pseudo-header (icmpv6.go:204-210): the addresses in place, the length
    // and protocol words as the initial.
    pb.pieces(ip.addr, ip.addr + ip.addr_len, true, false, &ps);
    if (icmpv6) return combine(combine((uint16_t)(len >> 16), (uint16_t)len), proto);
    return combine((uint16_t)len, proto);
  };
  if (rx) {
    if (ip.fragment) return NS_OK;  // reassembled before the transport layer sees it
    if (ip.proto == kProtoTCP) {
      // stack.DeliverTransportPacket: First() >= TCPMinimumSize; segment.parse
      // (segment.go:145-181): offset in [20, len(First())]
      uint8_t h[13];
      if (first_end - t0 < 20 || !pb.read(t0, h, 13)) {
        pp->verdict = NS_PKB_MALFORMED;
        return NS_OK;
      }
      const uint64_t off = (uint64_t)(h[12] >> 4) * 4;
      if (off < 20 || off > first_end - t0) {
        pp->verdict = NS_PKB_MALFORMED;
        return NS_OK;
      }
      const uint16_t init = pseudo(kProtoTCP, (uint16_t)tl, false);  // :176 PseudoHeaderChecksum(data.Size())
      pb.pieces(t0, t0 + off, true, false, &ps);                     // :177 h.CalculateChecksum(xsum)
      pb.pieces(t0 + off, te, true, false, &ps);                     // :179 ChecksumVV(s.data, xsum)
      pp->tr_chain = add_chain(init);
      pp->verdict = NS_PKB_INVALID;  // decided from the result (:180)
    } else if (ip.proto == kProtoICMPv4 && ip.v4) {
      // handleICMP (network/ipv4/icmp.go:60-80): echo requests only
      uint8_t h[4];
      if (first_end - t0 < 8 || !pb.read(t0, h, 4)) {
        pp->verdict = NS_PKB_MALFORMED;
        return NS_OK;
      }
      if (h[0] != 8) return NS_OK;
      pp->field = (uint16_t)((h[2] << 8) | h[3]);
      // h.SetChecksum(0); ^ChecksumVV(pkt.Data, 0): bytes [2, 4) as zeros
      pb.pieces(t0, t0 + 2, true, false, &ps);
      pb.pieces(t0 + 4, te, false, false, &ps);
      pp->tr_chain = add_chain(0);
      pp->verdict = NS_PKB_INVALID;
    } else if (ip.proto == kProtoICMPv6 && !ip.v4) {
      // handleICMP (network/ipv6/icmp.go:62-84): h = the first view, payload
      // = the other views, ICMPv6Checksum (header/icmpv6.go:202-221)
      uint8_t h[4];
      if (first_end - t0 < 4 || !pb.read(t0, h, 4)) {
        pp->verdict = NS_PKB_MALFORMED;
        return NS_OK;
      }
      pp->field = (uint16_t)((h[2] << 8) | h[3]);
      const uint16_t init = pseudo(kProtoICMPv6, tl, true);
      pb.pieces(first_end, te, true, true, &ps);        // for v in vv.Views(): Checksum(v, xsum)
      pb.pieces(t0, t0 + 2, true, false, &ps);          // Checksum(h with h[2:4] = 0, xsum)
      pb.pieces(t0 + 4, first_end, false, false, &ps);
      pp->tr_chain = add_chain(init);
      pp->verdict = NS_PKB_INVALID;
    }
    return NS_OK;
  }
  // TX: the transport header follows the IP header in Header; its checksum
  // field must lie in Header (it is written there).
  const uint64_t hdr_end = pb.hdr_len;
  auto need = [&](uint64_t field_end) { return field_end <= hdr_end; };
  if (ip.proto == kProtoTCP) {
    uint8_t h[13];
    if (!pb.read(t0, h, 13)) return NS_EINVAL;
    const uint64_t thl = (uint64_t)(h[12] >> 4) * 4;
    if (thl < 20 || t0 + thl > te || !need(t0 + 18)) return NS_EINVAL;
    // buildTCPHdr (connect.go:653-663): PseudoHeaderChecksum(length),
    // ChecksumVVWithOffset(payload), tcp.CalculateChecksum(xsum) = Checksum(tcp[:DataOffset])
    const uint16_t init = pseudo(kProtoTCP, (uint16_t)tl, false);
    pb.pieces(t0 + thl, te, true, false, &ps);
    pb.pieces(t0, t0 + thl, true, false, &ps);
    pp->tr_chain = add_chain(init);
    pp->tr_store = t0 + 16;
  } else if (ip.proto == kProtoUDP) {
    if (t0 + 8 > te || !need(t0 + 8)) return NS_EINVAL;
    // sendUDP (udp/endpoint.go:808-815): per-view restart, then the header
    const uint16_t init = pseudo(kProtoUDP, (uint16_t)tl, false);
    pb.pieces(t0 + 8, te, true, true, &ps);
    pb.pieces(t0, t0 + 8, true, false, &ps);
    pp->tr_chain = add_chain(init);
    pp->tr_store = t0 + 6;
  } else if (ip.proto == kProtoICMPv4 && ip.v4) {
    // the echo reply (network/ipv4/icmp.go:96-100): pkt = the ICMP bytes in
    // Header, SetChecksum(0), ^Checksum(pkt, ChecksumVV(vv, 0))
    if (!need(t0 + 4)) return NS_EINVAL;
    pb.pieces(hdr_end, te, true, false, &ps);
    pb.pieces(t0, t0 + 2, true, false, &ps);
    pb.pieces(t0 + 4, hdr_end, false, false, &ps);
    pp->tr_chain = add_chain(0);
    pp->tr_store = t0 + 2;
  } else if (ip.proto == kProtoICMPv6 && !ip.v4) {
    // ICMPv6Checksum(h = the ICMP bytes in Header, src, dst, Data) (icmpv6.go:202-221)
    if (!need(t0 + 4)) return NS_EINVAL;
    const uint16_t init = pseudo(kProtoICMPv6, tl, true);
    pb.pieces(hdr_end, te, true, true, &ps);
    pb.pieces(t0, t0 + 2, true, false, &ps);
    pb.pieces(t0 + 4, hdr_end, false, false, &ps);
    pp->tr_chain = add_chain(init);
    pp->tr_store = t0 + 2;
  }
  return NS_OK;
}

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
  const int dev = opts ? opts->device : 0;
  if (dev < 0 || dev >= ndev) return NS_ENODEV;
  ns_csum_ctx* ctx = new (std::nothrow) ns_csum_ctx();
  if (!ctx) return NS_ENOMEM;
  ctx->device = dev;
  if (opts && opts->staging_bytes) ctx->staging = opts->staging_bytes;
  DeviceGuard g(dev);
  hipError_t e = hipSuccess;
  for (int s = 0; s < 2 && e == hipSuccess; ++s) {
    e = hipStreamCreateWithFlags(&ctx->stream[s], hipStreamNonBlocking);
    if (e == hipSuccess) e = hipEventCreateWithFlags(&ctx->done[s], hipEventDisableTiming);
  }
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
  *out = ctx;
  return NS_OK;
}

void ns_csum_destroy(ns_csum_ctx* ctx) {
  if (!ctx) return;
  {
    DeviceGuard g(ctx->device);
    for (int s = 0; s < 2; ++s)
      if (ctx->stream[s]) (void)hipStreamSynchronize(ctx->stream[s]);
    for (StreamScratch* sc : ctx->scratch) {
      sc->chain.release();
      sc->split.release();
      delete sc;
    }
    ctx->scratch.clear();
    ctx->err_taken.release();
    ctx->z_buf.release();
    for (MappedPin* b : ctx->stage_all) {
      b->release();
      delete b;
    }
    ctx->stage_all.clear();
    ctx->stage_free.clear();
    for (int s = 0; s < 2; ++s) {
      ctx->d_arena[s].release();
      ctx->d_desc[s].release();
      ctx->d_out[s].release();
      ctx->d_chain[s].release();
      ctx->h_desc[s].release();
      ctx->h_out[s].release();
      if (ctx->done[s]) (void)hipEventDestroy(ctx->done[s]);
      if (ctx->stream[s]) (void)hipStreamDestroy(ctx->stream[s]);
    }
    ctx->g_arena.release();
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
                                 ctx->stream[0]));
    HIP_TRY(hipStreamSynchronize(ctx->stream[0]));
    v = *reinterpret_cast<volatile unsigned long long*>(taken);
  }
  if (bad) *bad = v;
  return NS_OK;
}

namespace {
// The scratch of `s` (caller holds ctx->mu).  Growing a buffer frees the old
// one with hipFree, which waits for the device, so no launch still uses it.
StreamScratch* stream_scratch(ns_csum_ctx* ctx, hipStream_t s) {
  for (StreamScratch* sc : ctx->scratch)
    if (sc->stream == s) return sc;
  StreamScratch* sc = new (std::nothrow) StreamScratch();
  if (!sc) return nullptr;
  sc->stream = s;
  ctx->scratch.push_back(sc);
  return sc;
}

int batch_dev(ns_csum_ctx* ctx, const uint8_t* d_arena, uint64_t arena_bytes, const ns_pkt_desc* d_desc,
              uint32_t n, uint16_t* d_out, uint32_t batch_flags, void* stream, bool store) {
  if (!ctx || (n && (!d_desc || !d_out)) || (arena_bytes && !d_arena)) return NS_EINVAL;
  if (n == 0) return NS_OK;
  DeviceGuard g(ctx->device);
  hipStream_t s = (hipStream_t)stream;  // NULL = the HIP null stream
  nsk::ChainScratch chain{};
  uint32_t* split = nullptr;
  if ((batch_flags & NS_BATCH_CHAINED) || arena_bytes / n >= nsk::split_min_avg()) {
    std::lock_guard<std::mutex> lk(ctx->mu);
    StreamScratch* sc = stream_scratch(ctx, s);
    if (!sc) return NS_ENOMEM;
    if (batch_flags & NS_BATCH_CHAINED) {
      int rc = sc->chain.ensure(n);
      if (rc != NS_OK) return rc;
      chain = sc->chain.get();
    }
    if (arena_bytes / n >= nsk::split_min_avg()) {
      int rc = sc->split.ensure(nsk::split_words(n), true);  // zero once; the kernel keeps it so
      if (rc != NS_OK) return rc;
      split = sc->split.p;
    }
  }
  HIP_TRY(nsk::launch_batch(d_arena, arena_bytes, d_desc, n, d_out, chain, ctx->d_err, s, 0, store ? 1u : 0u,
                            split));
  return NS_OK;
}
}  // namespace

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

int ns_csum_batch_host(ns_csum_ctx* ctx, const uint8_t* h_arena, uint64_t arena_bytes,
                       const ns_pkt_desc* h_desc, uint32_t n, uint16_t* h_out,
                       uint32_t batch_flags) {
  if (!ctx || (n && (!h_desc || !h_out)) || (arena_bytes && !h_arena)) return NS_EINVAL;
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
    MappedPin* st = lease_stage(ctx, &rc);
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
    return_stage(ctx, st);
    return rc;
  }
  std::lock_guard<std::mutex> lk(ctx->mu);
  DeviceGuard g(ctx->device);
  return run_host_batch(ctx, h_arena, arena_bytes, h_desc, n, h_out,
                        (batch_flags & NS_BATCH_CHAINED) != 0);
}

int ns_csum_checksum(ns_csum_ctx* ctx, const uint8_t* buf, uint64_t len, uint16_t initial,
                     uint16_t* out) {
  if (!ctx || !out || (len && !buf) || len > 0xFFFFFFFFull) return NS_EINVAL;
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
  if (nsegs == 0) return NS_OK;
  std::vector<std::vector<std::pair<const uint8_t*, uint64_t>>> clipped(nsegs);
  SpanProbe pr;
  for (uint32_t q = 0; q < nsegs; ++q) {
    int rc = clip_views(views, nviews, segs[q].off, segs[q].size, &clipped[q]);
    if (rc != NS_OK) return rc;
    for (const auto& pc : clipped[q]) pr.add(pc.first, pc.second);
  }
  Gather gt(ctx, pr.stage(ctx));
  for (uint32_t q = 0; q < nsegs; ++q) gt.segment(clipped[q], segs[q].initial);
  return gt.run(out);
}

int ns_csum_views_restart(ns_csum_ctx* ctx, const ns_view* views, uint32_t nviews,
                          uint16_t initial, uint16_t* out) {
  if (!ctx || !out || (nviews && !views)) return NS_EINVAL;
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
  if (n == 0) return NS_OK;
  std::vector<PacketBytes> pb(n);
  SpanProbe pr;
  for (uint32_t i = 0; i < n; ++i) {
    const int rc = pb[i].init(pkts[i]);
    if (rc != NS_OK) return rc;
    for (const auto& sg : pb[i].seg) pr.add(sg.first, sg.second);
  }
  Gather gt(ctx, pr.stage(ctx));
  std::vector<PacketPlan> plan(n);
  for (uint32_t i = 0; i < n; ++i) {
    const int rc = plan_packet(gt, pb[i], op, &plan[i]);
    if (rc != NS_OK) return rc;
  }
  std::vector<uint16_t> res(gt.result_at.size());
  if (!res.empty()) {
    const int rc = gt.run(res.data());
    if (rc != NS_OK) return rc;
  }
  for (uint32_t i = 0; i < n; ++i) {
    PacketPlan& p = plan[i];
    const uint16_t net = p.net_chain >= 0 ? res[(size_t)p.net_chain] : 0;
    const uint16_t tr = p.tr_chain >= 0 ? res[(size_t)p.tr_chain] : 0;
    if (sums) {
      sums[2 * i] = net;
      sums[2 * i + 1] = tr;
    }
    if (op == NS_PKB_FILL) {
      // SetChecksum(^sum), big-endian, into the packet's Header
      auto put = [&](uint64_t at, uint16_t v) {
        uint8_t* q = pb[i].mut(at);
        q[0] = (uint8_t)(v >> 8);
        q[1] = (uint8_t)v;
      };
      if (p.net_store != UINT64_MAX) put(p.net_store, (uint16_t)~net);
      if (p.tr_store != UINT64_MAX) put(p.tr_store, (uint16_t)~tr);
    } else if (verdict) {
      if (p.tr_chain >= 0) {
        // TCP: xsum == 0xffff (segment.go:180); ICMP: ^sum == the received field
        const bool ok = p.kind == kProtoTCP ? tr == 0xFFFF : (uint16_t)~tr == p.field;
        p.verdict = ok ? NS_PKB_VALID : NS_PKB_INVALID;
      }
      verdict[i] = p.verdict;
    }
  }
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

int ns_csum_shard_plan(const ns_pkt_desc* h_desc, uint32_t n, uint32_t parts, uint32_t* first) {
  if (!first || parts == 0 || (n && !h_desc)) return NS_EINVAL;
  uint64_t total = 0;
  for (uint32_t i = 0; i < n; ++i) total += h_desc[i].len;
  first[0] = 0;
  uint64_t run = 0;
  uint32_t i = 0;
  for (uint32_t p = 1; p < parts; ++p) {
    // Cut at the first descriptor whose prefix reaches p/parts of the bytes;
    // with all-empty tables fall back to equal descriptor counts.
    const uint64_t target = total ? (total * p + parts - 1) / parts : 0;
    if (total == 0) {
      i = (uint32_t)(((uint64_t)n * p) / parts);
    } else {
      while (i < n && run + h_desc[i].len <= target) run += h_desc[i++].len;
    }
    // never split a chained run
    while (i > 0 && i < n && (h_desc[i].flags & NS_DESC_CONT)) run += h_desc[i++].len;
    first[p] = std::max(i, first[p - 1]);
  }
  first[parts] = n;
  return NS_OK;
}

}  // extern "C"
