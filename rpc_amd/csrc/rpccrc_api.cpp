// rpc_amd/csrc/rpccrc_api.cpp -- C-ABI host layer of librpccrc (include/rpccrc.h).
//
// Owns per-device state, built once per device with std::call_once so the
// drop-in calls stay thread-safe without an init call (SURVEY.md 8b
// "Threading"):
//  * the table images in HBM;
//  * pools that lend resources to one call at a time and take them back when
//    the call returns -- device workspaces and pinned staging (BlockPool), the
//    drop-in scalar path's streams and staging (ScalarCtx), the host-batch
//    pipelines (HostPipeline).  Nothing is per thread, so a thread-per-
//    connection server that exits threads leaks nothing, and the memory held
//    is bounded by the peak number of concurrent calls.
// Every CRC value this library returns is computed by the HIP kernels in
// crc32_kernels.hip / frames.hip; there is no CPU CRC implementation in the
// product path.
#include <hip/hip_runtime.h>

#include <errno.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>
#include <time.h>

#include <algorithm>
#include <atomic>
#include <deque>
#include <functional>
#include <mutex>
#include <vector>

#include "../../include/rpccrc.h"
#include "crc32_gf2.h"
#include "crc32_kernels.h"
#include "crc32_layout.h"
#include "crc32_service_math.h"
#include "frames.h"

namespace rpccrc {
namespace {

constexpr int kMaxDevices = 64;

int map_hip(hipError_t e) {
  if (e == hipSuccess) return RPCCRC_OK;
  if (e == hipErrorOutOfMemory) return RPCCRC_ENOMEM;
  if (e == hipErrorNoDevice || e == hipErrorInvalidDevice) return RPCCRC_ENODEV;
  if (e == hipErrorInvalidValue) return RPCCRC_EINVAL;
  return RPCCRC_EIO;
}

#define RPCCRC_TRY(expr)                      \
  do {                                        \
    const hipError_t _e = (expr);             \
    if (_e != hipSuccess) return map_hip(_e); \
  } while (0)

// ---- pools -----------------------------------------------------------------

// A cached block of device memory (or pinned host memory) lent to one call at
// a time.  `ev` is recorded on the stream of the block's last use when the
// call returns it.  The next borrower orders itself after that use: a device
// block through hipStreamWaitEvent on its own stream (no host wait, and valid
// even if the earlier stream has been destroyed since -- the event outlives
// it), a pinned block through hipEventSynchronize (the host is about to write
// it).  Replaces per-call hipMallocAsync/hipFreeAsync, whose free blocked the
// calling thread until the GPU reached it (profiles/r01h_*), and the r01
// per-thread cache that hipFree'd on every stream switch.
struct Block {
  void *p = nullptr;
  size_t cap = 0;
  hipEvent_t ev = nullptr;
  bool used = false;
};

class BlockPool {
 public:
  BlockPool(bool pinned, size_t keep) : pinned_(pinned), keep_(keep) {}

  int acquire(size_t bytes, hipStream_t s, Block *out) {
    {
      std::lock_guard<std::mutex> g(mu_);
      int best = -1;
      for (int i = 0; i < (int)free_.size(); ++i)
        if (free_[i].cap >= bytes && (best < 0 || free_[i].cap < free_[best].cap)) best = i;
      if (best >= 0) {
        *out = free_[best];
        free_.erase(free_.begin() + best);
        cached_ -= out->cap;
      }
    }
    if (out->p) {
      if (out->used) RPCCRC_TRY(pinned_ ? hipEventSynchronize(out->ev) : hipStreamWaitEvent(s, out->ev, 0));
      return RPCCRC_OK;
    }
    size_t cap = pinned_ ? (64u << 10) : (1u << 20);
    while (cap < bytes) cap <<= 1;
    Block b;
    hipError_t e = pinned_ ? hipHostMalloc(&b.p, cap, hipHostMallocDefault) : hipMalloc(&b.p, cap);
    if (e != hipSuccess) {
      b.p = nullptr;
      return map_hip(e);
    }
    e = hipEventCreateWithFlags(&b.ev, hipEventDisableTiming);
    if (e != hipSuccess) {
      (void)(pinned_ ? hipHostFree(b.p) : hipFree(b.p));
      return map_hip(e);
    }
    b.cap = cap;
    *out = b;
    return RPCCRC_OK;
  }

  // Returns the block after the call has enqueued its last use on stream s.
  // recorded: the call's last kernel already recorded b.ev as its completion
  // signal (hipExtLaunchKernel stopEvent), so no marker packet is needed here.
  void release(Block &b, hipStream_t s, bool recorded = false) {
    if (!b.p) return;
    b.used = recorded || hipEventRecord(b.ev, s) == hipSuccess;
    if (!b.used) (void)hipStreamSynchronize(s); // no event: make the block idle now
    std::vector<Block> evict;
    {
      std::lock_guard<std::mutex> g(mu_);
      free_.push_back(b);
      cached_ += b.cap;
      // Over the keep limit: drop the largest idle blocks (rare; e.g. after a
      // one-off huge batch).
      while (cached_ > keep_ && !free_.empty()) {
        auto it = std::max_element(free_.begin(), free_.end(),
                                   [](const Block &x, const Block &y) { return x.cap < y.cap; });
        cached_ -= it->cap;
        evict.push_back(*it);
        free_.erase(it);
      }
    }
    for (Block &x : evict) {
      if (x.used) (void)hipEventSynchronize(x.ev);
      (void)(pinned_ ? hipHostFree(x.p) : hipFree(x.p));
      (void)hipEventDestroy(x.ev);
    }
    b = Block();
  }

 private:
  std::mutex mu_;
  std::vector<Block> free_;
  size_t cached_ = 0;
  const bool pinned_;
  const size_t keep_;
};

// A block borrowed for the duration of one call (returned by the destructor,
// after the call has enqueued all its work on `s`).
struct Lease {
  BlockPool *pool = nullptr;
  Block b;
  hipStream_t s = nullptr;
  bool recorded = false; // the call's last launch recorded b.ev (done_event())
  Lease() = default;
  Lease(const Lease &) = delete;
  Lease &operator=(const Lease &) = delete;
  ~Lease() {
    if (pool) pool->release(b, s, recorded);
  }
  // The block's event, for the call's LAST launch on s to record as its own
  // completion (then set `recorded`).
  hipEvent_t done_event() const { return b.ev; }
  int get(BlockPool *p, size_t bytes, hipStream_t stream) {
    pool = p;
    s = stream;
    return p->acquire(bytes, stream, &b);
  }
  uint8_t *ptr() const { return static_cast<uint8_t *>(b.p); }
};

// Two-word device counters for the rows kernel's tail stealing (crc32_rows.h
// kStealAhead).  A launch leases one; the launch's last workgroup resets it
// to zero, and the next lessee orders itself after that launch through the
// slot's event (hipStreamWaitEvent: no host wait).  Slots are 256 B apart and
// leased least-recently-used first, so back-to-back launches find their
// slot's last use finished and skip the wait: a wait per launch put ~5 us
// between back-to-back C1 kernels (profiles/r02/r02af_c1_kernel_stats.csv
// vs r02af_bench_c1.log).
class StealPool {
 public:
  struct Slot {
    uint32_t *p = nullptr;
    hipEvent_t ev = nullptr;
    bool used = false;
  };
  // The lessee gets the Slot itself (taken under mu_), so no lookup of the
  // slot storage happens outside the lock while grow() may be extending it
  // (deque operator[] outside mu_ raced with push_back).
  int acquire(hipStream_t s, Slot **out) {
    Slot *x = nullptr;
    {
      std::lock_guard<std::mutex> g(mu_);
      if (free_.size() < kMinFree)
        if (const int rc = grow()) return rc;
      x = free_.front();
      free_.pop_front();
    }
    if (x->used && hipEventQuery(x->ev) != hipSuccess) RPCCRC_TRY(hipStreamWaitEvent(s, x->ev, 0));
    *out = x;
    return RPCCRC_OK;
  }
  // recorded: the launch recorded the slot's event as its completion signal
  // (launch_rows steal_done).  Otherwise the slot may have been used by a
  // launch without it (ext_event() off): record it here, a marker packet.
  void release(Slot *x, hipStream_t s, bool recorded, bool dealt) {
    if (recorded) {
      x->used = true;
    } else if (dealt) {
      x->used = hipEventRecord(x->ev, s) == hipSuccess;
      if (!x->used) (void)hipStreamSynchronize(s);
    } // else the launch did not touch the slot: its last use (and event) stand
    std::lock_guard<std::mutex> g(mu_);
    free_.push_back(x);
  }

 private:
  static constexpr int kChunk = 64;
  static constexpr size_t kMinFree = 16; // grow early: a slot rests >= 16 leases before reuse
  int grow() { // under mu_
    uint8_t *mem = nullptr;
    RPCCRC_TRY(hipMalloc(reinterpret_cast<void **>(&mem), kChunk * 256));
    RPCCRC_TRY(hipMemset(mem, 0, kChunk * 256));
    for (int i = 0; i < kChunk; ++i) {
      Slot x;
      x.p = reinterpret_cast<uint32_t *>(mem + 256 * i);
      RPCCRC_TRY(hipEventCreateWithFlags(&x.ev, hipEventDisableTiming));
      all_.push_back(x);
      free_.push_back(&all_.back());
    }
    return RPCCRC_OK;
  }
  std::mutex mu_;
  std::deque<Slot> all_;   // element addresses stay valid as it grows; touched only under mu_
  std::deque<Slot *> free_; // FIFO: least recently used first
};

// A simple free list of T (one borrower at a time, created on demand).
template <class T>
class ObjPool {
 public:
  T *acquire() {
    {
      std::lock_guard<std::mutex> g(mu_);
      if (!free_.empty()) {
        T *t = free_.back();
        free_.pop_back();
        return t;
      }
    }
    return new T();
  }
  void release(T *t) {
    std::lock_guard<std::mutex> g(mu_);
    free_.push_back(t);
  }

 private:
  std::mutex mu_;
  std::vector<T *> free_;
};

// Drop-in scalar path: a non-blocking stream plus pinned staging.
struct ScalarCtx {
  hipStream_t stream = nullptr;
  uint8_t *pin = nullptr;   // pinned input staging, device-readable (zero-copy)
  uint32_t *pout = nullptr; // pinned result (rows kernel path)
  uint64_t *pres = nullptr; // pinned {crc, seq} of the one-wave kernel (polled)
  // Error word of this context's rows / large-body launches (pinned, coherent:
  // pres[1]).  A drop-in call checks its own word after its sync, so one failed
  // launch elsewhere on the device never takes the drop-in calls down with it.
  uint32_t *perr = nullptr;
  uint32_t seq = 0;
};

// rpc_crc32_batch: two slots, each a stream with a device stage and pinned
// metadata, so one group's H2D overlaps the previous group's kernel.
constexpr uint64_t kStageBytes = 256ull << 20; // device staging per pipeline slot
constexpr uint64_t kStageMaxBodies = 1ull << 20;
struct HostSlot {
  hipStream_t stream = nullptr;
  uint8_t *dbuf = nullptr;  // device copy of the group's span
  uint64_t *doff = nullptr; // rebased offsets
  uint32_t *dlen = nullptr;
  uint32_t *dout = nullptr;
  uint64_t *hoff = nullptr; // pinned staging for metadata
  uint32_t *hlen = nullptr;
  uint32_t *hout = nullptr;
  uint64_t first = 0, count = 0; // bodies of the group in flight
  bool busy = false;
};
struct HostPipeline {
  HostSlot slot[2];
  uint32_t *perr = nullptr; // error word of this call's launches (pinned, coherent)
  bool ok = false;
};

// Drop-in service (crc32_service.hip): one resident workgroup answers drop-in
// calls of <= kSvcMaxLen bytes through request slots in pinned coherent host
// memory, so a call costs PCIe round trips instead of a kernel launch.
struct Service {
  SvcShared *sh = nullptr;     // pinned, coherent (hipHostMallocCoherent)
  uint32_t *kshift = nullptr;  // device: 3 x 64 per-lane merge shifts
  const uint32_t *tq = nullptr;
  hipStream_t stream = nullptr;
  std::mutex launch_mu;
  std::atomic<uint32_t> launched{0}; // instances launched (written under launch_mu); instance k stores k when it leaves
  // Slot k is held while bit k is set: a lock-free claim (a std::mutex free
  // list put 10 concurrent callers to sleep on each other, r04d: 28 us a call).
  // A thread first tries the slot it held last (the same wave, k % kSvcWaves).
  // Each hot word has a cache line of its own: the claim mask (every caller's
  // CAS), the degraded flag (every caller reads it), and each slot's host state
  // (written only by the slot's holder).  Round 6's first version kept the
  // slots' shadows and an `answered` counter that every call incremented on
  // shared lines: 68-B calls on 10 threads took 7.6 us against 6.3 for round 5
  // on one box (profiles/r06x).
  alignas(64) std::atomic<uint32_t> busy{0};
  // Set when a request was given up (no answer in kSvcWaitNs), cleared by the
  // next answered one.  While set, a call whose instance has not started yet
  // (still queued behind other kernels) takes the launch path without posting,
  // and a posted call waits kSvcWaitShortNs, not kSvcWaitNs (one
  // slow call, not a 2-s stall per call).
  alignas(64) std::atomic<bool> degraded{false};
  alignas(64) std::atomic<uint64_t> fallbacks_full{0}, fallbacks_short{0}, bypassed{0};
  struct alignas(128) Slot {
    uint32_t seq = 0; // last request seq (written by the slot's holder)
    // Host copy of the slot's inline bytes (kSvcInline, as the request block
    // holds them): the tag's check sum covers all of them (svc::block_sum), and
    // reading them back from the coherent (uncached) block would cost a
    // PCIe-speed read per word.
    uint32_t inl[kSvcInline / 4] = {};
    std::atomic<uint64_t> answered{0}; // (one writer at a time: the holder)
  };
  Slot slot[kSvcSlots];
  bool ok = false;
};

struct DeviceCtx {
  int device = -1;
  int cus = 0;
  uint4 *img = nullptr; // LDS table image (rows kernel layout, 155 KiB)
  uint4 *img_round = nullptr; // the same with the round maps in ZI[11..14] (crc32_layout.h kLdsRoundMaps)
  uint4 *img_span = nullptr;  // the same with the dense span pass's maps over ZI / TQ16 (kLdsSpanM4)
  uint32_t *tq = nullptr;
  uint4 *shift_nib = nullptr; // NIB[k][i][j] = A_{2^k bytes}(j << 4i) (chunk combine)
  uint32_t *big_dbl = nullptr; // the big-body fold's doubling maps per chunk class (build_big_dbl)
  uint4 *scalar_tab = nullptr; // one-wave scalar kernel's table image (kScalarTabWords)
  uint32_t *dense_tab = nullptr; // the dense span fold's maps (kDenseTabWords, build_dense_tab)
  // Device error word (pinned, coherent host memory) of the ASYNCHRONOUS calls
  // (device batches, large bodies, frames): the rows kernel stores kErr* here
  // when a bounded wait runs out (crc32_rows.h).  Once it is non-zero, every
  // asynchronous call on this device returns RPCCRC_EIO until the caller clears
  // it (rpc_crc32_device_clear_status) -- CRCs of the failed launch may be
  // stale, and an asynchronous call has no later point at which to report it.
  // The synchronous calls (drop-in, host batch) use a word of their own per
  // call and are not affected by it.
  uint32_t *err = nullptr;
  int status = RPCCRC_ENODEV;
  char name[128] = {0};
  char arch[64] = {0};
  // Pools (never destroyed: a static destructor would run after the HIP
  // runtime's own teardown; the process exit releases everything).
  BlockPool *ws = nullptr;  // device workspaces (keeps <= 1 GiB idle)
  BlockPool *pin = nullptr; // pinned staging (keeps <= 256 MiB idle)
  ObjPool<ScalarCtx> *scalar = nullptr;
  ObjPool<HostPipeline> *pipes = nullptr;
  StealPool *steal = nullptr;
  Service *svc = nullptr;       // built on the first drop-in call (svc_once)
  std::once_flag svc_once;
  // The stream-read probe's output sink (its kernel stores nothing that is
  // read): one device block for the context, not a workspace lease per call --
  // a lease orders itself after the block's last use with an event wait, a
  // gap between back-to-back probe launches the product's launches do not have.
  uint32_t *probe_sink = nullptr;
  std::once_flag probe_once;
};

DeviceCtx g_dev[kMaxDevices];
std::once_flag g_once[kMaxDevices];

// Process-wide knobs (written by rpc_crc32_set_*, read by every call).
std::atomic<int> g_nontemporal{1}; // streamed once: non-temporal loads (measured faster)
std::atomic<int> g_max_blocks{0};
std::atomic<int> g_ragged_path{RPCCRC_RAGGED_AUTO};
// Large-body chunk (rpc_crc32_device_large, chunk_bytes = 0).  C4 per call
// (profiles/r01c4_*): 4 KiB 697 us (rows kernel fastest, combine 27 us),
// 16 KiB 673 us, 64 KiB 689 us (each wave streams its own 64 KiB).
// Tuning override: RPCCRC_LARGE_CHUNK (bytes, multiple of 16).
const uint64_t g_large_chunk = [] {
  const char *e = getenv("RPCCRC_LARGE_CHUNK");
  const unsigned long long v = e ? strtoull(e, nullptr, 10) : 0ull;
  return (v >= 16 && v % 16 == 0 && v <= (1ull << 31)) ? (uint64_t)v : (uint64_t)16384;
}();
const bool g_large_chunk_env = getenv("RPCCRC_LARGE_CHUNK") != nullptr;
// Ragged bodies of at least this many bytes take the on-device chunk route
// (DESIGN.md 4.6).  Tuning override: RPCCRC_BIG_MIN (bytes, >= 16 KiB).
const uint32_t g_big_min_env = [] {
  const char *e = getenv("RPCCRC_BIG_MIN");
  const unsigned long long v = e ? strtoull(e, nullptr, 10) : 0ull;
  return (v >= 16384 && v <= 0xFFFFFFFFull) ? (uint32_t)v : 0u;
}();
// A batch that the route can hold whole (n <= kBigMaxBodies) has too few
// bodies to keep the chip busy with one wave per body: a 255 KiB body was one
// wave's 64-row walk, 87 us of the 1024 lifted-cap frames' 760 us
// (profiles/r03/r03b_frames_kernel_stats.csv).  Such batches route every body
// of >= 16 KiB (at most 4 rows stay on one wave); large batches keep 256 KiB.
constexpr uint32_t kBigMinSmallBatch = 16384;
uint32_t big_min_for(uint64_t n) {
  if (g_big_min_env) return g_big_min_env;
  return n <= kBigMaxBodies ? kBigMinSmallBatch : kBigMin;
}
// Chunks of the big-body route: address-aligned power-of-two
// chunks by default (RPCCRC_BIG_ALIGNED=0: the end-aligned 2^k * 4096 - 16-byte
// chunks of rounds 2-3).  The plan doubles the size until the chunks fit
// kBigMaxChunks.  Tuning override: RPCCRC_BIG_CHUNK (bytes: a power of two
// >= 4096 aligned, 2^k * 4096 - 16 end-aligned).
const bool g_big_aligned = [] {
  const char *e = getenv("RPCCRC_BIG_ALIGNED");
  return !(e && e[0] == '0');
}();
const uint64_t g_big_chunk = [] {
  const char *e = getenv("RPCCRC_BIG_CHUNK");
  const unsigned long long v = e ? strtoull(e, nullptr, 10) : 0ull;
  if (g_big_aligned) return (v >= 4096 && v <= (1ull << 30) && (v & (v - 1)) == 0) ? (uint64_t)v : kBigMinChunkAligned;
  const unsigned long long p = v + 16;
  return (v >= 4096 - 16 && p <= (1ull << 30) && (p & (p - 1)) == 0) ? (uint64_t)v : kBigMinChunk;
}();
constexpr uint32_t kRowsGroupShift = 0;           // rows kernel group dealing, G = 2^shift
constexpr uint64_t kSplitMinFrames = 16384;       // fewer frames: one wave per body (rows kernel)
constexpr uint64_t kRouteAllMax = 2048;           // lifted-cap frames batches up to this size: route-all
// Route-all span mode (BigRoute): on by default; RPCCRC_BIG_SPAN=0
// keeps every body on the chunk route.  Streams below kSpanMinBytes keep it too.
const bool g_big_span = [] {
  const char *e = getenv("RPCCRC_BIG_SPAN");
  return !(e && e[0] == '0');
}();
constexpr uint64_t kSpanMinBytes = 1ull << 20;
// Round values for one-row chunks of contiguous large bodies (device_large):
// on by default; RPCCRC_ROUND_COMBINE=0 folds the per-chunk CRCs.
const bool g_round_combine = [] {
  const char *e = getenv("RPCCRC_ROUND_COMBINE");
  return !(e && e[0] == '0');
}();
constexpr bool kAutoSplitFrames = true;           // AUTO frames batches: split (true) or packed (false)
constexpr uint64_t kPackedMaxSlices = 1ull << 21; // slice-table cap (8 MiB)
// Chunks per packed slice, at least: a slice switch costs the wave two scalar
// loads it waits on.  Tuning override: RPCCRC_PACKED_MIN_SLICE.
uint64_t packed_min_slice() {
  static const uint64_t v = [] {
    const char *e = getenv("RPCCRC_PACKED_MIN_SLICE");
    const long long x = e ? atoll(e) : 0;
    return x > 0 ? (uint64_t)x : (uint64_t)32;
  }();
  return v;
}

void init_device(int dev) {
  DeviceCtx &c = g_dev[dev];
  c.device = dev;
  hipDeviceProp_t prop;
  if (hipGetDeviceProperties(&prop, dev) != hipSuccess) {
    c.status = RPCCRC_ENODEV;
    return;
  }
  c.cus = prop.multiProcessorCount;
  snprintf(c.name, sizeof c.name, "%s", prop.name);
  snprintf(c.arch, sizeof c.arch, "%s", prop.gcnArchName);
  if (prop.sharedMemPerBlock < kLdsBytesV3) { // needs the 160 KiB LDS of gfx950
    fprintf(stderr, "rpccrc: device %d (%s) has %zu B LDS per block, need %u\n", dev, c.arch,
            (size_t)prop.sharedMemPerBlock, kLdsBytesV3);
    c.status = RPCCRC_ENODEV;
    return;
  }
  std::vector<uint32_t> img(kLdsBytesV3 / 4), tq(kTqEntries), nib(kShiftNibWords), stab(kScalarTabWords);
  build_tq(tq.data());
  build_scalar_tab(stab.data());
  uint32_t sq = kX0 >> 8; // x^8 (one zero byte); squared: x^(8 * 2^k)
  for (uint32_t k = 0; k < 64; ++k) {
    for (uint32_t i = 0; i < 8; ++i)
      for (uint32_t j = 0; j < 16; ++j) nib[k * 128 + i * 16 + j] = gf2_mulmod(sq, j << (4 * i));
    sq = gf2_mulmod(sq, sq);
  }
  int prev = 0;
  (void)hipGetDevice(&prev);
  (void)hipSetDevice(dev);
  hipError_t e = hipSuccess;
  e = (e == hipSuccess) ? hipMalloc(&c.img, kImgHbmBytes) : e;
  e = (e == hipSuccess) ? hipMalloc(&c.img_round, kImgHbmBytes) : e;
  e = (e == hipSuccess) ? hipMalloc(&c.img_span, kImgHbmBytes) : e;
  e = (e == hipSuccess) ? hipMalloc(&c.tq, kTqEntries * 4) : e;
  e = (e == hipSuccess) ? hipMalloc(&c.shift_nib, kShiftNibWords * 4) : e;
  e = (e == hipSuccess) ? hipMalloc(&c.big_dbl, kBigDblWords * 4) : e;
  e = (e == hipSuccess) ? hipMalloc(&c.scalar_tab, kScalarTabWords * 4) : e;
  e = (e == hipSuccess) ? hipMalloc(&c.dense_tab, kDenseTabWords * 4) : e;
  e = (e == hipSuccess) ? hipHostMalloc(reinterpret_cast<void **>(&c.err), 64, hipHostMallocCoherent) : e;
  if (e == hipSuccess) *reinterpret_cast<volatile uint32_t *>(c.err) = 0;
  if (e == hipSuccess) {
    build_lds_image_v2(img.data());
    std::vector<uint32_t> img_round(img);
    for (uint32_t l = 1; l <= 4; ++l) // A_{4096 * 2^l} = NIB[12 + l]
      std::copy(nib.begin() + (12 + l) * 128, nib.begin() + (13 + l) * 128,
                img_round.begin() + kLdsRoundMaps / 4 + (l - 1) * 128);
    auto upload = [&](uint4 *dst, const std::vector<uint32_t> &src) {
      if (!kImgCompact) return hipMemcpy(dst, src.data(), kLdsBytesV3, hipMemcpyHostToDevice);
      std::vector<uint32_t> compact(kImgCompactBytes / 4);
      build_lds_image_compact(src.data(), compact.data());
      return hipMemcpy(dst, compact.data(), kImgCompactBytes, hipMemcpyHostToDevice);
    };
    e = upload(c.img, img);
    if (e == hipSuccess) e = upload(c.img_round, img_round);
    std::vector<uint32_t> img_span(img);
    build_lds_image_span(img_span.data());
    if (e == hipSuccess) e = upload(c.img_span, img_span);
  }
  if (e == hipSuccess) e = hipMemcpy(c.tq, tq.data(), kTqEntries * 4, hipMemcpyHostToDevice);
  if (e == hipSuccess) e = hipMemcpy(c.shift_nib, nib.data(), kShiftNibWords * 4, hipMemcpyHostToDevice);
  if (e == hipSuccess) {
    std::vector<uint32_t> dbl(kBigDblWords);
    build_big_dbl(dbl.data());
    e = hipMemcpy(c.big_dbl, dbl.data(), kBigDblWords * 4, hipMemcpyHostToDevice);
  }
  if (e == hipSuccess) e = hipMemcpy(c.scalar_tab, stab.data(), kScalarTabWords * 4, hipMemcpyHostToDevice);
  if (e == hipSuccess) {
    std::vector<uint32_t> dt(kDenseTabWords);
    build_dense_tab(dt.data());
    e = hipMemcpy(c.dense_tab, dt.data(), kDenseTabWords * 4, hipMemcpyHostToDevice);
  }
  (void)hipSetDevice(prev);
  c.ws = new BlockPool(false, 1ull << 30);
  c.pin = new BlockPool(true, 256ull << 20);
  c.scalar = new ObjPool<ScalarCtx>();
  c.steal = new StealPool();
  c.pipes = new ObjPool<HostPipeline>();
  c.status = map_hip(e);
}

// A kernel-reported error in the word w (a device's or a call's own).
int word_error(const uint32_t *w) {
  return (w != nullptr && *reinterpret_cast<const volatile uint32_t *>(w) != 0u) ? RPCCRC_EIO : RPCCRC_OK;
}
int device_error(const DeviceCtx &c) { return word_error(c.err); }

// Context of the calling thread's current device (its initialisation status).
int get_ctx(DeviceCtx **out) {
  int dev = -1;
  if (hipGetDevice(&dev) != hipSuccess || dev < 0 || dev >= kMaxDevices) return RPCCRC_ENODEV;
  int count = 0;
  if (hipGetDeviceCount(&count) != hipSuccess || count <= 0) return RPCCRC_ENODEV;
  std::call_once(g_once[dev], init_device, dev);
  *out = &g_dev[dev];
  return g_dev[dev].status;
}

// The same for an asynchronous call: RPCCRC_EIO while the device error word
// holds an uncleared error (DeviceCtx::err).
int get_async_ctx(DeviceCtx **out) {
  const int rc = get_ctx(out);
  return rc ? rc : device_error(**out);
}

// Test hook, compiled into the test build only (librpccrc_test.so,
// -DRPCCRC_TEST_HOOKS; ADVICE r03: the shipping library must not read it):
// RPCCRC_TEST_STEAL_GIVEUP=K makes the next K tail-stealing launches give up
// every pool-round wait (ItemsArgs.test_giveup), to exercise the error words.
uint32_t take_test_giveup() {
#ifdef RPCCRC_TEST_HOOKS
  static std::atomic<long> left{[] {
    const char *e = getenv("RPCCRC_TEST_STEAL_GIVEUP");
    return e ? atol(e) : 0L;
  }()};
  return left.fetch_sub(1) > 0 ? 1u : 0u;
#else
  return 0u;
#endif
}

// Test hook (test build only): RPCCRC_TEST_DENSE_ONLY=1 leaves out the plain
// rows pass of ragged batches, so a dense batch's CRCs can only come from the
// span pass and the fold, and a batch that does not take the dense step (the
// plan refuses it, or it is too small for it) keeps its output as it was
// (tests/test_gpu_parity.py test_dense_mode_covers_every_crc).
bool test_dense_only() {
#ifdef RPCCRC_TEST_HOOKS
  static const bool v = [] {
    const char *e = getenv("RPCCRC_TEST_DENSE_ONLY");
    return e && e[0] == '1';
  }();
  return v;
#else
  return false;
#endif
}

int max_blocks_for(const DeviceCtx &c) {
  // One 1024-thread workgroup per CU (156 KiB LDS each).
  int mb = c.cus > 0 ? c.cus : 256;
  const int cap = g_max_blocks.load(std::memory_order_relaxed);
  if (cap > 0) mb = std::min(mb * 8, cap);
  return mb;
}

bool nontemporal() { return g_nontemporal.load(std::memory_order_relaxed) != 0; }

ItemsArgs items_args(const DeviceCtx &c, const uint8_t *base, const uint64_t *offsets, const uint32_t *lengths,
                     uint64_t n, uint64_t stride, uint32_t len, uint32_t mode, uint32_t *out) {
  ItemsArgs a;
  a.base = base;
  a.offsets = offsets;
  a.lengths = lengths;
  a.n_items = n;
  a.stride = stride;
  a.len = len;
  a.mode = mode;
  a.lds_image = c.img;
  a.tq = c.tq;
  a.out = out;
  a.gshift = kRowsGroupShift;
  a.err = c.err;
  return a;
}

// A tail-stealing counter for a rows launch of n items that deals its rounds
// dynamically (QB = 1, at least 8 rounds per workgroup; crc32_kernels.hip
// launch_rows), released after the launch is enqueued.  Used for uniform
// batches of one-row bodies (north star NS -4.3 %, C3); ragged batches (C2
// +0.7 %) and the 16 KiB chunks of large bodies (C4 +1.3 %) measured slower
// with it (profiles/r02/r02w_steal_fraction_ab.txt).
// The slot's event is bound to the kernel's completion (launch_rows
// steal_done, hipExtLaunchKernel): a separate hipEventRecord after each launch
// is a marker packet between back-to-back kernels (+4 us per C1 step with
// per-step events, profiles/r02/r02aj_step_events_ab.txt).
// RPCCRC_STEAL_EXT_EVENT=0 records it separately (A/B only).
bool steal_ext_event() {
  static const bool v = [] {
    const char *e = getenv("RPCCRC_STEAL_EXT_EVENT");
    return !(e && e[0] == '0');
  }();
  return v;
}
struct StealLease {
  StealPool *pool = nullptr;
  StealPool::Slot *slot = nullptr;
  hipStream_t s = nullptr;
  uint32_t *p = nullptr;
  bool recorded = false; // the launch recorded the slot's event itself
  StealLease() = default;
  StealLease(const StealLease &) = delete;
  StealLease &operator=(const StealLease &) = delete;
  ~StealLease() {
    if (pool) pool->release(slot, s, recorded, !steal_ext_event());
  }
  int get(const DeviceCtx &c, uint64_t n, int QB, hipStream_t stream) {
    const uint64_t tasks = QB == 4 ? (n + 3) / 4 : n;
    if (tasks < 8ull * dyn_round(QB) * (uint64_t)max_blocks_for(c)) return RPCCRC_OK; // launch_rows: not DYN
    if (const int rc = c.steal->acquire(stream, &slot)) return rc;
    p = slot->p;
    pool = c.steal;
    s = stream;
    return RPCCRC_OK;
  }
  hipEvent_t done_event() const { return steal_ext_event() && slot ? slot->ev : nullptr; }
};

// Tail stealing for ragged rows passes: on since round 5's two-phase loop
// (crc32_rows.h; a 3 % pool, crc32_kernels.hip steal_frac): C2 -0.5 to -0.9 %
// against no pool, rotated (profiles/r05z).  Before it, the pool protocol in
// the one loop made every row dearer and stealing cost C2 +0.7 % (round 2),
// +2.3 % (round 3), +1.8 % (round 5, r05w).  RPCCRC_RAGGED_STEAL=0 turns it off.
bool ragged_steal() {
  static const bool v = [] {
    const char *e = getenv("RPCCRC_RAGGED_STEAL");
    return !(e && e[0] == '0');
  }();
  return v;
}

// Dense span mode for ragged device batches.  RPCCRC_DENSE=0
// turns it off (the rows pass only, as in rounds 1-5).
bool dense_enabled() {
  static const bool v = [] {
    const char *e = getenv("RPCCRC_DENSE");
    return !(e && e[0] == '0');
  }();
  return v;
}

// err: the error word of the call's launches (nullptr: the device's, for the
// asynchronous entry points; the synchronous ones pass a word of their own).
int items(const DeviceCtx &c, const uint8_t *base, const uint64_t *offsets, const uint32_t *lengths, uint64_t n,
          uint64_t stride, uint32_t len, uint32_t mode, uint32_t *out, int QB, hipStream_t s, uint32_t *err = nullptr) {
  ItemsArgs a = items_args(c, base, offsets, lengths, n, stride, len, mode, out);
  if (err) a.err = err;
  StealLease sl;
  if (offsets == nullptr && len <= 4096)
    if (const int rc = sl.get(c, n, QB, s)) return rc;
  a.steal = sl.p;
  if (a.steal) a.test_giveup = take_test_giveup();
  return map_hip(launch_rows(a, QB, nontemporal(), max_blocks_for(c), s, sl.done_event(), &sl.recorded));
}

// A ragged batch on the device.
//  * Kernel: AUTO frames (bodies capped at MAX_BODY_LEN = 1 KiB, rpc.h:17)
//    take the split path (bodies <= 1 KiB four per row through the QB = 4
//    rows kernel: 1M frames 334 us vs 481 packed, 565 rows),
//    other batches the rows kernel (one wave per body; ahead on C2's
//    64 B - 64 KiB mix).
//  * route: bodies of >= kBigMin bytes go through the big-body chunk route
//    (classify before, chunks + fold after) so a long body
//    does not stream through a single wave.  Not with the packed kernel.
//  * span_bytes (frames calls: the stream length; 0 otherwise): a route-all
//    batch over a 4 KiB-aligned base may take the route's span mode (BigRoute).
//  * cmp (frames verify): in route-all mode the fold writes the verdicts too
//    and *compared is set (the caller then skips its compare launch).
struct FramesCmp {
  const uint32_t *expected;
  const uint8_t *pre;
  uint8_t *verdict;
};
int ragged(const DeviceCtx &c, const uint8_t *base, const uint64_t *offsets, const uint32_t *lengths, uint64_t n,
           uint32_t mode, uint32_t *out, hipStream_t s, bool small_bodies, bool route, uint32_t *err = nullptr,
           uint64_t span_bytes = 0, const FramesCmp *cmp = nullptr, bool *compared = nullptr,
           const FramesParse *fparse = nullptr, const FramesStamp *fstamp = nullptr, bool *stamped = nullptr,
           uint32_t max_len = 0) {
  const int path = g_ragged_path.load(std::memory_order_relaxed);
  const bool nt = nontemporal();
  const int mb = max_blocks_for(c);
  const bool fits = n < (1ull << 27); // the packed kernel's metadata window: 8-B offsets in a 1 GiB buffer range
  // AUTO frames batches split only when they are large: the split's flag /
  // scan / scatter passes and second rows launch cost ~20 us, which only a
  // batch of many frames repays (1M frames: 334 vs 565 us); a
  // small batch (e.g. 1024 lifted-cap frames) takes the rows kernel directly.
  const bool auto_frames = path == RPCCRC_RAGGED_AUTO && small_bodies && n >= kSplitMinFrames;
  const bool packed = fits && (path == RPCCRC_RAGGED_PACKED || (auto_frames && !kAutoSplitFrames));
  const bool split = !packed && n <= kMaxLaunchItems && (path == RPCCRC_RAGGED_SPLIT || (auto_frames && kAutoSplitFrames));
  route = route && !packed && mode == kModeFinal && n <= kMaxLaunchItems;
  // Route-all: a lifted-cap frames batch of at most kRouteAllMax frames sends
  // every body through the chunk route (no classify pass and no plain rows
  // pass, whose longest non-routed body -- up to the 16 KiB small-batch
  // threshold, one wave -- set its duration: 15 us of a 1024-frame verify).
  // Bounded because the fold spends a block-wide reduction per body (1024
  // blocks): a few bodies per block cost less than the passes they replace.
  const bool route_all = route && small_bodies && !split && n <= kRouteAllMax && !g_big_min_env;
  // fparse (frames verify): the route-all aligned plan parses the headers
  // itself; any other path needs them parsed before its first launch.
  const bool fuse_parse = fparse && route_all && g_big_aligned;
  if (fparse && !fuse_parse)
    RPCCRC_TRY(launch_frames_parse(fparse->stream, fparse->stream_bytes, fparse->frame_off, n, fparse->flags,
                                   fparse->body_off, fparse->body_len, fparse->hdr_crc, fparse->pre, s));
  // fstamp (frames stamp): likewise the stamp's bounds / cap check, and the fold
  // then writes the headers (*stamped set; the caller skips its stamp launch).
  const bool fuse_stamp = fstamp && route_all && g_big_aligned;
  if (fstamp && !fuse_stamp) RPCCRC_TRY(launch_frames_stamp_prep(*fstamp, n, s));
  ItemsArgs a = items_args(c, base, offsets, lengths, n, 0, 0, mode, out);
  if (err) a.err = err;
  if (packed) {
    const uint64_t ms = std::min<uint64_t>(kPackedMaxSlices, std::max<uint64_t>(8192, 4 * n));
    size_t bytes = 0;
    RPCCRC_TRY(packed_workspace_bytes(n, ms, &bytes));
    Lease ws;
    if (const int rc = ws.get(c.ws, bytes, s)) return rc;
    PackedBatch p;
    p.base = base;
    p.offsets = offsets;
    p.lengths = lengths;
    p.n = n;
    p.mode = mode;
    p.lds_image = c.img;
    p.tq = c.tq;
    p.out = out;
    p.ws = ws.ptr();
    p.ws_bytes = bytes;
    p.max_slices = ms;
    p.min_slice = packed_min_slice();
    return map_hip(launch_packed_batch(p, nt, mb, s));
  }
  size_t split_bytes = 0;
  if (split) RPCCRC_TRY(split_workspace_bytes(n, &split_bytes));
  split_bytes = (split_bytes + 255) & ~(size_t)255;
  // Span mode (route-all over a 4 KiB-aligned stream of >= kSpanMinBytes; the
  // plan still falls back to chunks when the bodies are sparse in it).
  const uint64_t span_rows = (route_all && g_big_span && g_big_aligned && ((uintptr_t)base & 4095u) == 0 &&
                              span_bytes >= kSpanMinBytes && (span_bytes >> 12) <= kSpanMaxRows)
                                 ? span_bytes >> 12
                                 : 0;
  const size_t route_bytes = route ? big_route_workspace_bytes(n, span_rows) : 0;
  Lease ws;
  if (split_bytes + route_bytes > 0)
    if (const int rc = ws.get(c.ws, split_bytes + route_bytes, s)) return rc;
  // Dense span mode: a ragged batch of many bodies whose bound
  // (or, unbounded, the mode's own 1 MiB body limit) allows it.  The plan
  // decides on the device whether the bodies lie back to back in order with
  // 64 B .. 1 MiB each; then the span pass and the fold compute every CRC, and
  // the rows pass and the big-body route's classify pass (so the whole route)
  // have nothing to do (DenseCtl::skip); otherwise the span pass and the fold
  // exit at once.
  // nb_cap: the blocks the workspace holds (20 B each) -- by the bound, or for an
  // unbounded call by a 64 KiB average body (a longer stream is refused by the
  // plan and takes the rows pass and the route: exact, as without the mode)
  const uint64_t dense_len = max_len ? max_len : kDenseMaxBody;
  const uint64_t nb_cap = std::min<uint64_t>(n * (max_len ? max_len : 65536u) / 4096u + 2u, kDenseMaxBlocks);
  const bool dense = dense_enabled() && !route_all && !split && !small_bodies && mode == kModeFinal &&
                     n >= kDenseMinN && n <= kDenseMaxN && dense_len >= kDenseMinBody && dense_len <= kDenseMaxBody &&
                     nb_cap >= 8ull * dyn_round(1) * (uint64_t)mb;
  Lease dws;
  DenseArgs dn{};
  StealLease dsl; // the span pass's steal counter
  if (dense) {
    if (const int rc = dws.get(c.ws, dense_workspace_bytes(n, nb_cap), s)) return rc;
    dn = dense_carve(dws.ptr(), n, nb_cap);
    dn.base = base;
    dn.offsets = offsets;
    dn.lengths = lengths;
    dn.out = out;
    dn.tq = c.tq;
    dn.tab = c.dense_tab;
    RPCCRC_TRY(launch_dense_plan(dn, s));
    a.skip_dev = &dn.ctl->skip;
  }
  BigRoute r{};
  StealLease sl;  // the route's chunk pass deals its tail from this counter (device-counted)
  StealLease ssl; // ... and its span pass from this one
  if (route) {
    r = big_route_carve(ws.ptr() + split_bytes, n, span_rows);
    r.min_chunk = g_big_chunk;
    r.aligned = g_big_aligned;
    r.tq = c.tq;
    r.dbl = c.big_dbl;
    r.tab4 = c.scalar_tab;
    // span pass round values: only when it deals in DYN rounds
    if (!(span_rows && g_round_combine && span_rows >= 256ull * (uint64_t)mb)) r.rnd = nullptr;
    r.rnd_image = c.img_round;
    if (route_all) {
      r.all_n = (uint32_t)n;
      // (the verdicts come from the aligned route's fold only: the end-aligned
      // fold, big_combine_kernel, writes CRCs -- with RPCCRC_BIG_ALIGNED=0 the
      // caller's compare launch writes them)
      if (cmp && g_big_aligned) {
        r.cmp_expected = cmp->expected;
        r.cmp_pre = cmp->pre;
        r.cmp_verdict = cmp->verdict;
        if (compared) *compared = true;
      }
      if (fuse_parse) r.parse = *fparse;
      if (fuse_stamp) {
        r.stamp = *fstamp;
        if (stamped) *stamped = true;
      }
    } else {
      const uint32_t big_min = big_min_for(n);
      if (dense) r.skip = &dn.ctl->skip;
      RPCCRC_TRY(launch_big_classify(lengths, n, big_min, r, s));
      a.routed = r.routed;
      a.big_min = big_min;
    }
    if (const int rc = c.steal->acquire(s, &sl.slot)) return rc;
    sl.p = sl.slot->p;
    sl.pool = c.steal;
    sl.s = s;
    if (span_rows)
      if (const int rc = ssl.get(c, span_rows, 1, s)) return rc;
    a.test_giveup = take_test_giveup(); // (the route's chunk pass; the plain rows pass takes its own below)
  }
  StealLease rsl; // the plain rows pass deals its tail from a steal counter too (RPCCRC_RAGGED_STEAL=0: not)
  if (split) {
    RPCCRC_TRY(launch_split_batch(a, ws.ptr(), split_bytes, nt, mb, s));
  } else if (!route_all && !test_dense_only()) {
    if (ragged_steal()) {
      if (const int rc = rsl.get(c, n, 1, s)) return rc;
      a.steal = rsl.p;
    }
    const uint32_t route_giveup = a.test_giveup;
    a.test_giveup = a.steal ? take_test_giveup() : 0u;
    RPCCRC_TRY(launch_rows(a, 1, nt, mb, s, rsl.done_event(), &rsl.recorded));
    a.steal = nullptr;
    a.test_giveup = route_giveup;
  }
  if (dense) {
    ItemsArgs sp = items_args(c, nullptr, nullptr, nullptr, nb_cap, 4096, 4096, kModeRaw, dn.W);
    if (err) sp.err = err;
    sp.n_dev = &dn.ctl->nblocks;
    sp.lds_image = c.img_span;
    sp.span_ctl = dn.ctl;
    sp.span_rec = dn.rec;
    sp.span_bpos = dn.bpos;
    sp.span_bnd = dn.bnd;
    if (const int rc = dsl.get(c, nb_cap, 1, s)) return rc;
    sp.steal = dsl.p;
    RPCCRC_TRY(launch_rows(sp, 1, nt, mb, s, dsl.done_event(), &dsl.recorded));
    RPCCRC_TRY(launch_dense_fold(dn, c.cus, s));
  }
  if (route) {
    StealArgs span;
    span.p = ssl.p;
    span.done = ssl.done_event();
    span.recorded = &ssl.recorded;
    RPCCRC_TRY(launch_big_route(a, r, c.shift_nib, nt, mb, s, sl.p, sl.done_event(), &sl.recorded, span));
  }
  return RPCCRC_OK;
}

// ---- large bodies: chunk expansion + combine --------------------------------

using BodyDesc = LargeBody;

template <class Bodies>
__device__ __forceinline__ void expand_chunks(const Bodies &bodies, uint64_t nb, uint64_t chunk, uint64_t total_chunks,
                                              uint64_t *item_off, uint32_t *item_len, uint64_t *lens, uint64_t *firsts,
                                              uint32_t *out) {
  const uint64_t t = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (t < nb) {
    lens[t] = bodies[t].len;
    firsts[t] = bodies[t].chunk_first;
    out[t] = 0; // the combine XORs its partials in
  }
  if (t >= total_chunks) return;
  uint64_t lo = 0, hi = nb; // last body with chunk_first <= t
  while (hi - lo > 1) {
    const uint64_t mid = (lo + hi) / 2;
    if (bodies[mid].chunk_first <= t) lo = mid; else hi = mid;
  }
  const BodyDesc b = bodies[lo];
  const uint64_t nch = (b.len + chunk - 1) / chunk;
  const uint64_t k = t - b.chunk_first;
  const uint64_t end = b.len - (nch - 1 - k) * chunk;
  const uint64_t start = end > chunk ? end - chunk : 0;
  item_off[t] = b.off + start;
  item_len[t] = (uint32_t)(end - start);
}

__global__ void expand_chunks_kernel(const BodyDesc *bodies, uint64_t nb, uint64_t chunk, uint64_t total_chunks,
                                     uint64_t *item_off, uint32_t *item_len, uint64_t *lens, uint64_t *firsts,
                                     uint32_t *out) {
  expand_chunks(bodies, nb, chunk, total_chunks, item_off, item_len, lens, firsts, out);
}

__global__ void expand_chunks_inline_kernel(InlineBodies bodies, uint64_t nb, uint64_t chunk, uint64_t total_chunks,
                                            uint64_t *item_off, uint32_t *item_len, uint64_t *lens, uint64_t *firsts,
                                            uint32_t *out) {
  expand_chunks(bodies.b, nb, chunk, total_chunks, item_off, item_len, lens, firsts, out);
}

// Large bodies: end-aligned chunks, CRC'd by the rows kernel in RAW mode, then
// folded per body by the chunk combine.
//  * Contiguous fast path: when the bodies lie back to back and every length
//    is a multiple of the chunk, the chunks of all bodies are one uniform
//    batch (base + off_0 + i * chunk): the rows kernel runs the north-star
//    pattern and no chunk table is built.  With the default chunk (0) the
//    largest of 16/8/4 KiB dividing every length is taken.
//  * Otherwise expand_chunks writes each chunk's (offset, length) and the rows
//    kernel runs ragged.
// <= 32 bodies travel in the kernel arguments; bodies of <= 64Ki chunks get
// one 1024-thread combine block each (plain store), longer ones several
// blocks that XOR into the zeroed output.  The workspace comes from the
// device's pool (stream-ordered reuse, no free on this path).
int device_large(const DeviceCtx &c, const uint8_t *d_base, const uint64_t *h_offsets, const uint64_t *h_lengths,
                 uint64_t n, uint32_t *d_out, uint64_t chunk, hipStream_t s, uint32_t *err = nullptr) {
  if (chunk % 16 != 0 || chunk > (1ull << 31)) return RPCCRC_EINVAL;
  if (n == 0) return RPCCRC_OK;
  const bool inl = n <= kInlineBodies;
  bool contiguous = inl;
  uint64_t lens_or = 0;
  for (uint64_t i = 0; i < n && contiguous; ++i) {
    lens_or |= h_lengths[i];
    if (i + 1 < n && h_offsets[i + 1] != h_offsets[i] + h_lengths[i]) contiguous = false;
  }
  bool equal = true;
  for (uint64_t i = 1; i < n && equal; ++i) equal = h_lengths[i] == h_lengths[0];
  if (chunk == 0) {
    chunk = g_large_chunk;
    // Back-to-back equal bodies of a multiple of 16 MiB: one-row 4 KiB chunks,
    // dealt with tail stealing and folded by the contiguous-run combine
    // (C4 640 -> 618 us, profiles/r02/r02ac_*).
    if (contiguous && equal && n <= 1024 && h_lengths[0] != 0 && h_lengths[0] % (4096ull * 4096ull) == 0 &&
        h_lengths[0] / 4096 <= 16ull * 4096ull && !g_large_chunk_env)
      chunk = 4096;
    else if (contiguous && lens_or % chunk != 0 && !g_large_chunk_env)
      for (uint64_t cand : {8192ull, 4096ull})
        if (lens_or % cand == 0) {
          chunk = cand;
          break;
        }
  }
  // power-of-two chunk: every length is a multiple of it iff their OR is
  const bool pow2 = (chunk & (chunk - 1)) == 0;
  uint64_t total = 0, max_nch = 0;
  InlineBodies ib;
  BodyDesc *bd = ib.b;
  Lease stage; // pinned body table for > kInlineBodies bodies
  if (!inl) {
    if (const int rc = stage.get(c.pin, n * sizeof(BodyDesc), s)) return rc;
    bd = reinterpret_cast<BodyDesc *>(stage.ptr());
  }
  bool multiple = true;
  uint64_t min_nch = ~0ull;
  for (uint64_t i = 0; i < n; ++i) {
    bd[i].off = h_offsets[i];
    bd[i].len = h_lengths[i];
    bd[i].chunk_first = total;
    const uint64_t nch = (h_lengths[i] + chunk - 1) / chunk;
    total += nch;
    max_nch = std::max(max_nch, nch);
    min_nch = std::min(min_nch, nch);
    if (!pow2 && h_lengths[i] % chunk != 0) multiple = false;
  }
  if (pow2) multiple = lens_or % chunk == 0;
  if (total == 0) { // all bodies empty
    RPCCRC_TRY(hipMemsetAsync(d_out, 0, n * 4, s));
    return RPCCRC_OK;
  }
  uint64_t splits = 1; // combine blocks per body
  if (max_nch > 65536) {
    splits = (max_nch + 1023) / 1024;
    splits = std::max<uint64_t>(1, std::min<uint64_t>(splits, (1ull << 20) / n));
  }
  const bool fast = contiguous && multiple && splits == 1;
  // Equal bodies of 4096 * S power-of-two chunks (S <= 16) on the fast path:
  // the contiguous-run combine with S blocks per body (the rows pass zeroes out).
  const uint64_t cs = max_nch / 4096;
  const bool contig = fast && min_nch == max_nch && max_nch % 4096 == 0 && cs >= 1 && cs <= 16 &&
                      (chunk & (chunk - 1)) == 0 && n <= 1024;
  // One-row chunks of a contiguous batch: the rows pass also stores each round's
  // crc0 (32 chunks = 128 KiB, ItemsArgs.round_out) and the combine folds those
  // -- 1/32 of the values (RPCCRC_ROUND_COMBINE=0: the per-chunk fold).  The
  // launch must deal in DYN rounds (launch_rows: >= 8 rounds per workgroup),
  // and the base must be 16-byte aligned: the round maps sit in the image's ZI
  // slots of trailing pads 12..15, which a misaligned base's items would read.
  const bool rounds = contig && chunk == 4096 && g_round_combine && total >= 8ull * 32 * (uint64_t)max_blocks_for(c) &&
                      (reinterpret_cast<uintptr_t>(d_base + h_offsets[0]) & 15u) == 0;
  const size_t ws_bytes = fast ? total * 4 + (rounds ? total / 8 : 0) + 64
                               : n * sizeof(BodyDesc) + n * 16 + total * (8 + 4 + 4) + 64;
  Lease wsl;
  if (const int rc = wsl.get(c.ws, ws_bytes, s)) return rc;
  uint8_t *ws = wsl.ptr();
  uint32_t *d_raw = reinterpret_cast<uint32_t *>(ws);
  uint64_t *d_lens = nullptr, *d_firsts = nullptr;
  if (fast) {
    ItemsArgs k = items_args(c, d_base + h_offsets[0], nullptr, nullptr, total, chunk, (uint32_t)chunk, kModeRaw, d_raw);
    if (err) k.err = err;
    StealLease sl; // one-row chunks deal like the north star (items())
    if (chunk <= 4096)
      if (const int rc = sl.get(c, total, 1, s)) return rc;
    k.steal = sl.p;
    if (k.steal) k.test_giveup = take_test_giveup();
    if (contig) {
      k.zero_out = d_out;
      k.zero_n = (uint32_t)n;
    }
    if (rounds) {
      k.round_out = d_raw + total;
      k.lds_image = c.img_round;
    }
    RPCCRC_TRY(launch_rows(k, 1, nontemporal(), max_blocks_for(c), s, sl.done_event(), &sl.recorded));
  } else {
    BodyDesc *d_bodies = reinterpret_cast<BodyDesc *>(ws);
    d_lens = reinterpret_cast<uint64_t *>(ws + n * sizeof(BodyDesc));
    d_firsts = d_lens + n;
    uint64_t *d_ioff = d_firsts + n;
    uint32_t *d_ilen = reinterpret_cast<uint32_t *>(d_ioff + total);
    d_raw = d_ilen + total;
    if (!inl) RPCCRC_TRY(hipMemcpyAsync(d_bodies, bd, n * sizeof(BodyDesc), hipMemcpyHostToDevice, s));
    const uint64_t threads = std::max<uint64_t>(total, n);
    const dim3 eg((unsigned)((threads + 255) / 256));
    if (inl)
      hipLaunchKernelGGL(expand_chunks_inline_kernel, eg, dim3(256), 0, s, ib, n, chunk, total, d_ioff, d_ilen, d_lens,
                         d_firsts, d_out);
    else
      hipLaunchKernelGGL(expand_chunks_kernel, eg, dim3(256), 0, s, d_bodies, n, chunk, total, d_ioff, d_ilen, d_lens,
                         d_firsts, d_out);
    RPCCRC_TRY(hipGetLastError());
    ItemsArgs k = items_args(c, d_base, d_ioff, d_ilen, total, 0, 0, kModeRaw, d_raw);
    if (err) k.err = err;
    RPCCRC_TRY(launch_rows(k, 1, nontemporal(), max_blocks_for(c), s));
  }
  CombineArgs ca;
  ca.raw = d_raw;
  ca.lengths = d_lens;
  ca.chunk_first = d_firsts;
  ca.shift_nib = c.shift_nib;
  ca.n_bodies = n;
  ca.chunk = chunk;
  ca.out = d_out;
  ca.splits = (uint32_t)splits;
  if (contig) {
    ca.contig = true;
    ca.splits = (uint32_t)cs;
  }
  if (rounds) { // 128 * S round values per body: one block each
    ca.raw = d_raw + total;
    ca.chunk = chunk * 32;
    ca.splits = 1;
  }
  ca.inline_bodies = inl;
  if (inl) ca.bodies = ib;
  if (steal_ext_event()) {
    const hipError_t e = launch_chunk_combine(ca, s, wsl.done_event());
    wsl.recorded = e == hipSuccess;
    return map_hip(e);
  }
  return map_hip(launch_chunk_combine(ca, s));
}

// ---- drop-in scalar path ------------------------------------------------------

[[noreturn]] void die(const char *what, int rc) {
  fprintf(stderr, "rpccrc: %s failed (%s); librpccrc requires a usable HIP device and has no CPU fallback\n", what,
          rpc_crc32_strerror(rc));
  abort();
}

constexpr size_t kScalarZeroCopyMax = 64 << 10;  // read straight from pinned memory
constexpr uint64_t kScalarChunkedMin = 8 << 20;  // chunk + combine above this

int scalar_ctx_init(ScalarCtx &t) {
  if (t.stream) return RPCCRC_OK;
  RPCCRC_TRY(hipStreamCreateWithFlags(&t.stream, hipStreamNonBlocking));
  RPCCRC_TRY(hipHostMalloc(reinterpret_cast<void **>(&t.pout), 64, hipHostMallocDefault));
  // Coherent: the host polls this word while the kernel may still be running.
  RPCCRC_TRY(hipHostMalloc(reinterpret_cast<void **>(&t.pres), 64, hipHostMallocCoherent));
  *reinterpret_cast<volatile uint64_t *>(t.pres) = 0;
  t.perr = reinterpret_cast<uint32_t *>(t.pres + 1);
  *reinterpret_cast<volatile uint32_t *>(t.perr) = 0;
  RPCCRC_TRY(hipHostMalloc(reinterpret_cast<void **>(&t.pin), kScalarZeroCopyMax, hipHostMallocDefault));
  return RPCCRC_OK;
}

// Bodies <= kScalarMaxLen: the one-wave kernel, and the host polls the
// pinned result word for this call's sequence number -- no stream
// synchronisation (~3 us less per call: tools/latency_probe.hip,
// profiles/r02/r02n_*).  A call whose result has not arrived after
// kScalarSpinNs falls back to hipStreamSynchronize, which also surfaces a
// device error.
constexpr uint64_t kScalarSpinNs = 200000;

uint64_t mono_ns() {
  timespec ts;
  clock_gettime(CLOCK_MONOTONIC, &ts);
  return (uint64_t)ts.tv_sec * 1000000000ull + (uint64_t)ts.tv_nsec;
}

uint32_t scalar_small(const DeviceCtx &c, ScalarCtx &t, const uint8_t *src, uint32_t len) {
  const uint32_t vbytes = 64u << scalar_seg_log2(len);
  if (len) memcpy(t.pin + (vbytes - len), src, len);
  if (++t.seq == 0) t.seq = 1; // 0 is the result word's initial value
  const uint32_t seq = t.seq;
  if (launch_scalar(t.pin, len, c.scalar_tab, c.tq, t.pres, seq, t.stream) != hipSuccess)
    die("kernel launch", RPCCRC_EIO);
  const volatile uint64_t *res = t.pres;
  uint64_t v = *res;
  if ((uint32_t)(v >> 32) != seq) {
    const uint64_t t0 = mono_ns();
    for (uint32_t spin = 1;; ++spin) {
      v = *res;
      if ((uint32_t)(v >> 32) == seq) break;
      if ((spin & 255u) == 0 && mono_ns() - t0 > kScalarSpinNs) {
        if (hipStreamSynchronize(t.stream) != hipSuccess) die("stream sync", RPCCRC_EIO);
        v = *res;
        if ((uint32_t)(v >> 32) != seq) die("scalar result", RPCCRC_EIO);
        break;
      }
    }
  }
  return (uint32_t)v;
}

// ---- drop-in service host side ---------------------------------

// RPCCRC_SERVICE=0 turns the service off (every drop-in call launches a kernel).
bool service_enabled() {
  static const bool v = [] {
    const char *e = getenv("RPCCRC_SERVICE");
    return !(e && e[0] == '0');
  }();
  return v;
}
constexpr uint64_t kSvcIdleTicks = 200000;   // 2 ms without a request (s_memrealtime, 100 MHz)
constexpr uint64_t kSvcLifeTicks = 2000000;  // 20 ms per instance: bounds what a device-wide sync waits for
// A call with no answer after kSvcWaitNs gives its request up and takes the
// launch-per-call path instead (VERDICT / ADVICE r04: the service may not be
// placed while other kernels fill the GPU; that path then waits on its own
// stream, and surfaces a real device error).  The abandoned request is safe to
// leave: nobody waits for its seq, and the slot's next request carries a new one.
constexpr uint64_t kSvcWaitNs = 2000000000;
// After a request was given up, the next posted calls wait this long (the
// instance has started by then, so an answer normally takes microseconds).
constexpr uint64_t kSvcWaitShortNs = 2000000;
constexpr uint64_t kSvcWaitMutedNs = 20000000; // the test build's muted requests

// Test hook, compiled into the test build only (librpccrc_test.so):
// RPCCRC_TEST_SVC_MUTE=K makes the next K inline service requests unanswerable
// (their tag never matches) and their first wait 20 ms, to exercise the fallback.
bool take_test_svc_mute() {
#ifdef RPCCRC_TEST_HOOKS
  static std::atomic<long> left{[] {
    const char *e = getenv("RPCCRC_TEST_SVC_MUTE");
    return e ? atol(e) : 0L;
  }()};
  return left.fetch_sub(1) > 0;
#else
  return false;
#endif
}

std::vector<Service *> g_services; // for the exit handler (under g_services_mu)
std::mutex g_services_mu;

bool svc_running(const Service &v) {
  return *reinterpret_cast<const volatile uint32_t *>(&v.sh->ctl[kSvcExited]) !=
         v.launched.load(std::memory_order_acquire);
}

// Asks every running instance to leave and waits for all of them together
// (bounded: 200 ms), then clears the stop words so the next drop-in call's
// instance serves as usual (unless `keep_stopped`, at exit).  g_services_mu is
// held only to copy the list, and each launch_mu only to set / clear the word
// (the waits no longer add up per device, and a first drop-in call
// on another device does not block behind them).
int svc_stop_list(bool keep_stopped) {
  std::vector<Service *> vs;
  {
    std::lock_guard<std::mutex> g(g_services_mu);
    vs = g_services;
  }
  std::vector<Service *> told;
  for (Service *v : vs) {
    std::lock_guard<std::mutex> lg(v->launch_mu);
    if (!svc_running(*v)) continue;
    reinterpret_cast<volatile uint32_t *>(v->sh->ctl)[kSvcStop] = 1u;
    told.push_back(v);
  }
  const uint64_t t0 = mono_ns();
  bool left = false;
  while (!left && mono_ns() - t0 < 200000000ull) {
    left = true;
    for (Service *v : told) left = left && !svc_running(*v);
  }
  int rc = RPCCRC_OK;
  for (Service *v : told) {
    std::lock_guard<std::mutex> lg(v->launch_mu);
    if (svc_running(*v)) rc = RPCCRC_EIO;
    if (!keep_stopped) reinterpret_cast<volatile uint32_t *>(v->sh->ctl)[kSvcStop] = 0u;
  }
  return rc;
}

// At process exit: every running instance leaves, so no service wave outlives
// the process's last HIP call.
void stop_services() { (void)svc_stop_list(true); }

void svc_init(DeviceCtx &c) {
  Service *v = new Service();
  int prev = 0;
  (void)hipGetDevice(&prev);
  (void)hipSetDevice(c.device);
  hipError_t e = hipHostMalloc(reinterpret_cast<void **>(&v->sh), sizeof(SvcShared), hipHostMallocCoherent);
  if (e == hipSuccess) {
    memset(v->sh, 0, sizeof(SvcShared));
    std::vector<uint32_t> k(3 * 64);
    const uint32_t segs[3] = {4, 8, 16};
    for (int cl = 0; cl < 3; ++cl)
      for (uint32_t L = 0; L < 64; ++L) k[cl * 64 + L] = gf2_xpow(8ull * segs[cl] * (63u - L));
    e = hipMalloc(&v->kshift, k.size() * 4);
    if (e == hipSuccess) e = hipMemcpy(v->kshift, k.data(), k.size() * 4, hipMemcpyHostToDevice);
  }
  if (e == hipSuccess) e = hipStreamCreateWithFlags(&v->stream, hipStreamNonBlocking);
  (void)hipSetDevice(prev);
  v->tq = c.tq;
  v->ok = e == hipSuccess;
  if (v->ok) {
    std::lock_guard<std::mutex> g(g_services_mu);
    if (g_services.empty()) atexit(stop_services);
    g_services.push_back(v);
  }
  c.svc = v;
}

// rpc_crc32_service_stop: the running instances leave now.
int svc_stop_all() { return svc_stop_list(false); }

// Launches an instance unless one is running (the new one queues behind a
// leaving one on the service stream).
bool svc_ensure(DeviceCtx &c, Service &v) {
  if (svc_running(v)) return true;
  std::lock_guard<std::mutex> g(v.launch_mu);
  if (svc_running(v)) return true;
  int prev = 0;
  (void)hipGetDevice(&prev);
  if (prev != c.device) (void)hipSetDevice(c.device);
  const uint32_t next = v.launched.load(std::memory_order_relaxed) + 1;
  const hipError_t e = launch_service(v.sh, v.tq, v.kshift, kSvcIdleTicks, kSvcLifeTicks, next, v.stream);
  if (prev != c.device) (void)hipSetDevice(prev);
  if (e != hipSuccess) return false;
  v.launched.store(next, std::memory_order_release);
  return true;
}

// One drop-in CRC through the service; false when the service is off, busy
// (every slot held), failed to launch, or gave the request up -- the caller then
// launches a kernel.
bool svc_crc(DeviceCtx &c, const uint8_t *src, uint32_t len, uint32_t *crc) {
  if (!service_enabled() || len > kSvcMaxLen) return false;
  std::call_once(c.svc_once, svc_init, std::ref(c));
  Service &v = *c.svc;
  if (!v.ok) return false;
  SvcShared *sh = v.sh;
  // After a request went unanswered: while the latest instance has not started
  // (queued behind kernels that fill the GPU), take the launch path at once.
  const bool degraded = v.degraded.load(std::memory_order_relaxed);
  if (degraded && *reinterpret_cast<const volatile uint32_t *>(&sh->ctl[kSvcStarted]) !=
                      v.launched.load(std::memory_order_acquire)) {
    v.bypassed.fetch_add(1, std::memory_order_relaxed);
    return false;
  }
  // claim a slot: this thread's last one if free, else the lowest free one
  thread_local int last_slot = -1;
  int slot = -1;
  for (uint32_t m = v.busy.load(std::memory_order_relaxed);;) {
    const uint32_t free = ~m & ((1u << kSvcSlots) - 1u);
    if (free == 0) return false;
    const int k = (last_slot >= 0 && ((free >> last_slot) & 1u)) ? last_slot : __builtin_ctz(free);
    if (v.busy.compare_exchange_weak(m, m | (1u << k), std::memory_order_acquire, std::memory_order_relaxed)) {
      slot = k;
      break;
    }
  }
  last_slot = slot;
  SvcReq &rq = sh->rq[slot];
  Service::Slot &hs = v.slot[slot];
  uint32_t q = ++hs.seq;
  if (q == 0) q = ++hs.seq; // 0: the answered seq of a fresh slot
  const bool mute = len <= kSvcInline && take_test_svc_mute();
  const uint64_t wait_ns = degraded ? kSvcWaitShortNs : mute ? kSvcWaitMutedNs : kSvcWaitNs;
  // the tag: the check sum of the block's len, seq and inline words (the
  // request's new bytes written into the shadow first), and of a longer body's
  // masked words (crc32_kernels.h SvcReq)
  uint32_t tag;
  if (len <= kSvcInline) { // in the request block, ending at its inline byte 116
    uint8_t *shadow = reinterpret_cast<uint8_t *>(hs.inl);
    memcpy(shadow + kSvcInline - len, src, len);
    memcpy(rq.inl + kSvcInline - len, src, len);
    tag = svc::block_sum(len, q, hs.inl);
  } else {
    const uint32_t seg = svc::seg_of(len);
    memcpy(sh->body[slot] + 64u * seg - len, src, len);
    tag = svc::block_sum(len, q, hs.inl) ^ svc::body_sum(src, len);
  }
  std::atomic_thread_fence(std::memory_order_release); // the bytes before the tag (x86: a compiler barrier)
  *reinterpret_cast<volatile uint32_t *>(&rq.tag) = mute ? tag ^ 0x80000000u : tag;
  std::atomic_thread_fence(std::memory_order_release); // the tag before the request word
  *reinterpret_cast<volatile uint64_t *>(&rq.req) = (uint64_t)len | ((uint64_t)q << 32);
  bool ok = svc_ensure(c, v);
  const volatile uint64_t *res = &sh->res[slot][0];
  uint64_t r = *res;
  if (ok && (uint32_t)(r >> 32) != q) {
    const uint64_t t0 = mono_ns();
    for (uint32_t spin = 1;; ++spin) {
      r = *res;
      if ((uint32_t)(r >> 32) == q) break;
      if ((spin & 63u) == 0) {
        // an instance that left just before our request: start the next one
        if (!svc_ensure(c, v)) {
          ok = false;
          break;
        }
        if ((spin & 1023u) == 0 && mono_ns() - t0 > wait_ns) { // give the request up (above)
          (degraded ? v.fallbacks_short : v.fallbacks_full).fetch_add(1, std::memory_order_relaxed);
          v.degraded.store(true, std::memory_order_relaxed);
          ok = false;
          break;
        }
      }
    }
  }
  if (ok) hs.answered.store(hs.answered.load(std::memory_order_relaxed) + 1, std::memory_order_relaxed);
  v.busy.fetch_and(~(1u << slot), std::memory_order_release);
  if (ok) {
    *crc = (uint32_t)r;
    if (degraded) v.degraded.store(false, std::memory_order_relaxed);
  }
  return ok;
}

// One CRC through the GPU.  The context (stream + staging) is borrowed from
// the device's pool for the call: concurrent callers get distinct contexts,
// and a context is reused by the next call of any thread.
uint32_t scalar_crc(const void *data, uint32_t len) {
  DeviceCtx *c = nullptr;
  int rc = get_ctx(&c);
  if (rc) die("device init", rc);
  uint32_t svc_r = 0;
  if (svc_crc(*c, static_cast<const uint8_t *>(data), len, &svc_r)) return svc_r;
  ScalarCtx *t = c->scalar->acquire();
  if ((rc = scalar_ctx_init(*t))) die("scalar context", rc);
  const uint8_t *src = static_cast<const uint8_t *>(data);
  if (len <= kScalarMaxLen) {
    const uint32_t r = scalar_small(*c, *t, src, len);
    c->scalar->release(t);
    return r;
  }
  if (len <= kScalarZeroCopyMax) {
    memcpy(t->pin, src, len);
    rc = items(*c, t->pin, nullptr, nullptr, 1, 0, len, kModeFinal, t->pout, 1, t->stream, t->perr);
    if (rc) die("kernel launch", rc);
  } else {
    // Device staging borrowed from the device's workspace pool (stream-ordered
    // reuse: no hipMalloc / hipFree -- a hipFree synchronises the whole device
    // and stalls every other thread's stream).  The CRC lands
    // in a device word at the end of the lease and comes back by a 4-byte D2H
    // copy: the chunk combine XORs its partials in with device atomics, which
    // must not target host memory.
    const size_t body = (len + 255) & ~(size_t)255;
    Lease stage;
    if ((rc = stage.get(c->ws, body + 256, t->stream))) die("device staging", rc);
    uint8_t *dbuf = stage.ptr();
    uint32_t *dword = reinterpret_cast<uint32_t *>(dbuf + body);
    if (hipMemcpyAsync(dbuf, src, len, hipMemcpyHostToDevice, t->stream) != hipSuccess) die("H2D copy", RPCCRC_EIO);
    if (len >= kScalarChunkedMin) {
      const uint64_t off = 0, l64 = len;
      rc = device_large(*c, dbuf, &off, &l64, 1, dword, 0, t->stream, t->perr);
    } else {
      rc = items(*c, dbuf, nullptr, nullptr, 1, 0, len, kModeFinal, dword, 1, t->stream, t->perr);
    }
    if (rc) die("kernel launch", rc);
    if (hipMemcpyAsync(t->pout, dword, 4, hipMemcpyDeviceToHost, t->stream) != hipSuccess) die("D2H copy", RPCCRC_EIO);
  } // the lease returns the staging block here, after its last use was enqueued
  if (hipStreamSynchronize(t->stream) != hipSuccess) die("stream sync", RPCCRC_EIO);
  if ((rc = word_error(t->perr))) die("kernel (call error word)", rc);
  const uint32_t r = *t->pout;
  c->scalar->release(t);
  return r;
}

// ---- host-buffer batch pipeline ----------------------------------------------

int pipe_init(HostPipeline &p) {
  if (p.ok) return RPCCRC_OK;
  if (!p.perr) RPCCRC_TRY(hipHostMalloc(reinterpret_cast<void **>(&p.perr), 64, hipHostMallocCoherent));
  for (HostSlot &s : p.slot) {
    if (!s.stream) RPCCRC_TRY(hipStreamCreateWithFlags(&s.stream, hipStreamNonBlocking));
    if (!s.dbuf) RPCCRC_TRY(hipMalloc(&s.dbuf, kStageBytes));
    if (!s.doff) RPCCRC_TRY(hipMalloc(&s.doff, kStageMaxBodies * 8));
    if (!s.dlen) RPCCRC_TRY(hipMalloc(&s.dlen, kStageMaxBodies * 4));
    if (!s.dout) RPCCRC_TRY(hipMalloc(&s.dout, kStageMaxBodies * 4));
    if (!s.hoff) RPCCRC_TRY(hipHostMalloc(reinterpret_cast<void **>(&s.hoff), kStageMaxBodies * 8, hipHostMallocDefault));
    if (!s.hlen) RPCCRC_TRY(hipHostMalloc(reinterpret_cast<void **>(&s.hlen), kStageMaxBodies * 4, hipHostMallocDefault));
    if (!s.hout) RPCCRC_TRY(hipHostMalloc(reinterpret_cast<void **>(&s.hout), kStageMaxBodies * 4, hipHostMallocDefault));
  }
  p.ok = true;
  return RPCCRC_OK;
}

int slot_drain(HostSlot &s, uint32_t *out) {
  if (!s.busy) return RPCCRC_OK;
  s.busy = false;
  RPCCRC_TRY(hipStreamSynchronize(s.stream));
  memcpy(out + s.first, s.hout, s.count * 4);
  return RPCCRC_OK;
}

int host_batch_run(const DeviceCtx &c, HostPipeline &p, const uint8_t *base, const uint64_t *offsets,
                   const uint32_t *lengths, uint64_t n, uint32_t *out) {
  int rc = pipe_init(p);
  if (rc) return rc;
  *reinterpret_cast<volatile uint32_t *>(p.perr) = 0; // this call's launches report here
  uint64_t i = 0;
  int which = 0;
  while (i < n) {
    // Bodies larger than a stage go through the chunked large path on their own.
    if ((uint64_t)lengths[i] > kStageBytes) {
      for (HostSlot &s : p.slot)
        if ((rc = slot_drain(s, out))) return rc;
      HostSlot &s = p.slot[0];
      const uint64_t L = lengths[i];
      {
        Lease tmp;
        if ((rc = tmp.get(c.ws, L, s.stream))) return rc;
        RPCCRC_TRY(hipMemcpyAsync(tmp.ptr(), base + offsets[i], L, hipMemcpyHostToDevice, s.stream));
        const uint64_t zero = 0;
        if ((rc = device_large(c, tmp.ptr(), &zero, &L, 1, s.dout, 0, s.stream, p.perr))) return rc;
      }
      RPCCRC_TRY(hipMemcpyAsync(s.hout, s.dout, 4, hipMemcpyDeviceToHost, s.stream));
      s.first = i;
      s.count = 1;
      s.busy = true;
      if ((rc = slot_drain(s, out))) return rc;
      ++i;
      continue;
    }
    // Greedy group of consecutive bodies whose byte span fits one stage.
    uint64_t lo = offsets[i], hi = offsets[i] + lengths[i];
    uint64_t k = i + 1;
    while (k < n && k - i < kStageMaxBodies && (uint64_t)lengths[k] <= kStageBytes) {
      const uint64_t nlo = std::min(lo, offsets[k]);
      const uint64_t nhi = std::max(hi, offsets[k] + lengths[k]);
      if (nhi - nlo > kStageBytes) break;
      lo = nlo;
      hi = nhi;
      ++k;
    }
    HostSlot &s = p.slot[which];
    which ^= 1;
    if ((rc = slot_drain(s, out))) return rc;
    const uint64_t cnt = k - i;
    for (uint64_t q = 0; q < cnt; ++q) {
      s.hoff[q] = offsets[i + q] - lo;
      s.hlen[q] = lengths[i + q];
    }
    if (hi > lo) RPCCRC_TRY(hipMemcpyAsync(s.dbuf, base + lo, hi - lo, hipMemcpyHostToDevice, s.stream));
    RPCCRC_TRY(hipMemcpyAsync(s.doff, s.hoff, cnt * 8, hipMemcpyHostToDevice, s.stream));
    RPCCRC_TRY(hipMemcpyAsync(s.dlen, s.hlen, cnt * 4, hipMemcpyHostToDevice, s.stream));
    rc = ragged(c, s.dbuf, s.doff, s.dlen, cnt, kModeFinal, s.dout, s.stream, false, true, p.perr);
    if (rc) return rc;
    RPCCRC_TRY(hipMemcpyAsync(s.hout, s.dout, cnt * 4, hipMemcpyDeviceToHost, s.stream));
    s.first = i;
    s.count = cnt;
    s.busy = true;
    i = k;
  }
  for (HostSlot &s : p.slot)
    if ((rc = slot_drain(s, out))) return rc;
  return RPCCRC_OK;
}

int host_batch(DeviceCtx &c, const uint8_t *base, const uint64_t *offsets, const uint32_t *lengths, uint64_t n,
               uint32_t *out) {
  HostPipeline *p = c.pipes->acquire();
  int rc = host_batch_run(c, *p, base, offsets, lengths, n, out);
  if (rc == RPCCRC_OK) rc = word_error(p->perr); // every launch of this call has completed
  if (rc) // leave the pipeline idle for its next borrower
    for (HostSlot &s : p->slot)
      if (s.busy) {
        (void)hipStreamSynchronize(s.stream);
        s.busy = false;
      }
  c.pipes->release(p);
  return rc;
}

bool frames_flags_ok(int flags) {
  const int role = flags & (RPC_FRAMES_SERVER | RPC_FRAMES_CLIENT);
  return (flags & ~(RPC_FRAMES_SERVER | RPC_FRAMES_CLIENT | RPC_FRAMES_LIFT_CAP)) == 0 &&
         (role == RPC_FRAMES_SERVER || role == RPC_FRAMES_CLIENT);
}

constexpr size_t align256(size_t x) { return (x + 255) & ~(size_t)255; }

} // namespace
} // namespace rpccrc

using namespace rpccrc;

extern "C" {

uint32_t rpc_crc32(const void *data, size_t len) {
  const uint32_t len32 = (uint32_t)len; // zlib uInt length (crc.c:7)
  if (data == nullptr || len32 == 0) return 0u;
  return scalar_crc(data, len32);
}

bool rpc_crc32_verify(const void *data, size_t len, uint32_t expected_crc) {
  return rpc_crc32(data, len) == expected_crc;
}

int rpc_crc32_batch(const uint8_t *base, const uint64_t *offsets, const uint32_t *lengths, size_t n,
                    uint32_t *out_crc, int flags) {
  if (flags != 0) return RPCCRC_EINVAL;
  if (n == 0) return RPCCRC_OK;
  if (!offsets || !lengths || !out_crc) return RPCCRC_EINVAL;
  if (!base) { // zlib: Z_NULL buffer -> 0
    memset(out_crc, 0, n * 4);
    return RPCCRC_OK;
  }
  DeviceCtx *c = nullptr;
  int rc = get_ctx(&c);
  if (rc) return rc;
  return host_batch(*c, base, offsets, lengths, n, out_crc);
}

int64_t rpc_crc32_verify_batch(const uint8_t *base, const uint64_t *offsets, const uint32_t *lengths,
                               const uint32_t *expected, size_t n, uint8_t *ok) {
  if (n == 0) return 0;
  if (!expected || !ok) return RPCCRC_EINVAL;
  std::vector<uint32_t> crc(n);
  const int rc = rpc_crc32_batch(base, offsets, lengths, n, crc.data(), 0);
  if (rc) return rc;
  int64_t bad = 0;
  for (size_t i = 0; i < n; ++i) {
    ok[i] = crc[i] == expected[i];
    bad += !ok[i];
  }
  return bad;
}

int rpc_crc32_device_batch(const uint8_t *d_base, const uint64_t *d_offsets, const uint32_t *d_lengths, uint64_t n,
                           uint32_t *d_out, void *stream) {
  return rpc_crc32_device_batch_bounded(d_base, d_offsets, d_lengths, n, 0, d_out, stream);
}

int rpc_crc32_device_batch_bounded(const uint8_t *d_base, const uint64_t *d_offsets, const uint32_t *d_lengths,
                                   uint64_t n, uint32_t max_len, uint32_t *d_out, void *stream) {
  if (n == 0) return RPCCRC_OK;
  if (!d_base || !d_offsets || !d_lengths || !d_out) return RPCCRC_EINVAL;
  DeviceCtx *c = nullptr;
  int rc = get_async_ctx(&c);
  if (rc) return rc;
  // A bound below the route threshold: no body can take the big-body route, so
  // its passes (classify before the rows pass; plan, expand, chunk rows and
  // fold after it: ~30 us of launches, profiles/r02final4/c2_kernel_stats.csv)
  // are not launched.  A body over a wrong bound is still CRC'd correctly by
  // the rows pass (one wave for the whole body): the hint is about speed only.
  const bool route = max_len == 0 || max_len >= big_min_for(n);
  return ragged(*c, d_base, d_offsets, d_lengths, n, kModeFinal, d_out, static_cast<hipStream_t>(stream), false, route,
                nullptr, 0, nullptr, nullptr, nullptr, nullptr, nullptr, max_len);
}

int rpc_crc32_device_uniform(const uint8_t *d_base, uint64_t n, uint32_t body_len, uint64_t stride, uint32_t *d_out,
                             void *stream) {
  if (n == 0) return RPCCRC_OK;
  if (!d_base || !d_out) return RPCCRC_EINVAL;
  DeviceCtx *c = nullptr;
  int rc = get_async_ctx(&c);
  if (rc) return rc;
  // Four bodies per 4 KiB row when every body plus its pad to a 16-byte end
  // fits a 1 KiB quarter (QB = 4); otherwise one body per row sequence.
  const uint32_t zmax = (stride % 16 == 0) ? (uint32_t)(0u - (uint32_t)(uintptr_t)(d_base + body_len)) & 15u : 15u;
  const int QB = (body_len + zmax <= 1024) ? 4 : 1;
  return items(*c, d_base, nullptr, nullptr, n, stride, body_len, kModeFinal, d_out, QB,
               static_cast<hipStream_t>(stream));
}

int rpc_crc32_device_large(const uint8_t *d_base, const uint64_t *h_offsets, const uint64_t *h_lengths, uint64_t n,
                           uint32_t *d_out, uint64_t chunk_bytes, void *stream) {
  if (n == 0) return RPCCRC_OK;
  if (!d_base || !h_offsets || !h_lengths || !d_out) return RPCCRC_EINVAL;
  DeviceCtx *c = nullptr;
  int rc = get_async_ctx(&c);
  if (rc) return rc;
  return device_large(*c, d_base, h_offsets, h_lengths, n, d_out, chunk_bytes, static_cast<hipStream_t>(stream));
}

int rpc_frames_verify_device(const uint8_t *d_stream, uint64_t stream_bytes, const uint64_t *d_frame_offsets,
                             uint64_t n, int flags, uint8_t *d_verdict, uint32_t *d_crc, void *stream) {
  if (!frames_flags_ok(flags)) return RPCCRC_EINVAL;
  if (n == 0) return RPCCRC_OK;
  if (!d_stream || !d_frame_offsets || !d_verdict || n >= 0xFFFFFFFFull) return RPCCRC_EINVAL;
  DeviceCtx *c = nullptr;
  int rc = get_async_ctx(&c);
  if (rc) return rc;
  hipStream_t s = static_cast<hipStream_t>(stream);
  Lease wsl;
  const size_t ws_bytes = align256(n * 8) + 3 * align256(n * 4) + align256(n);
  if ((rc = wsl.get(c->ws, ws_bytes, s))) return rc;
  uint8_t *ws = wsl.ptr();
  uint64_t *boff = reinterpret_cast<uint64_t *>(ws);
  uint32_t *blen = reinterpret_cast<uint32_t *>(ws + align256(n * 8));
  uint32_t *bexp = reinterpret_cast<uint32_t *>(ws + align256(n * 8) + align256(n * 4));
  uint32_t *bcrc = d_crc ? d_crc : reinterpret_cast<uint32_t *>(ws + align256(n * 8) + 2 * align256(n * 4));
  uint8_t *pre = ws + align256(n * 8) + 3 * align256(n * 4);
  FramesParse fp; // (launched by ragged(), or fused into the route's plan)
  fp.stream = d_stream;
  fp.stream_bytes = stream_bytes;
  fp.frame_off = d_frame_offsets;
  fp.flags = flags;
  fp.body_off = boff;
  fp.body_len = blen;
  fp.hdr_crc = bexp;
  fp.pre = pre;
  const bool lift = (flags & RPC_FRAMES_LIFT_CAP) != 0;
  const FramesCmp cmp{bexp, pre, d_verdict};
  bool compared = false;
  if ((rc = ragged(*c, d_stream, boff, blen, n, kModeFinal, bcrc, s, true, lift, nullptr, stream_bytes, &cmp, &compared,
                   &fp)))
    return rc;
  if (compared) return RPCCRC_OK; // (route-all: the fold wrote the verdicts)
  return map_hip(launch_frames_compare(bcrc, bexp, pre, n, d_verdict, s));
}

int rpc_frames_stamp_device(uint8_t *d_stream, uint64_t stream_bytes, const uint64_t *d_frame_offsets,
                            const uint32_t *d_body_lens, uint64_t n, uint16_t version, uint16_t type, int flags,
                            uint8_t *d_verdict, void *stream) {
  if ((flags & ~(RPC_FRAMES_SERVER | RPC_FRAMES_CLIENT | RPC_FRAMES_LIFT_CAP)) != 0) return RPCCRC_EINVAL;
  if (n == 0) return RPCCRC_OK;
  if (!d_stream || !d_frame_offsets || !d_body_lens || n >= 0xFFFFFFFFull) return RPCCRC_EINVAL;
  DeviceCtx *c = nullptr;
  int rc = get_async_ctx(&c);
  if (rc) return rc;
  hipStream_t s = static_cast<hipStream_t>(stream);
  Lease wsl;
  const size_t ws_bytes = align256(n * 8) + 2 * align256(n * 4) + align256(n);
  if ((rc = wsl.get(c->ws, ws_bytes, s))) return rc;
  uint8_t *ws = wsl.ptr();
  uint64_t *boff = reinterpret_cast<uint64_t *>(ws);
  uint32_t *blen = reinterpret_cast<uint32_t *>(ws + align256(n * 8));
  uint32_t *bcrc = reinterpret_cast<uint32_t *>(ws + align256(n * 8) + align256(n * 4));
  uint8_t *pre = d_verdict ? d_verdict : ws + align256(n * 8) + 2 * align256(n * 4);
  FramesStamp st; // (the check launched by ragged(), or fused into the route's plan; the headers likewise)
  st.stream = d_stream;
  st.stream_bytes = stream_bytes;
  st.frame_off = d_frame_offsets;
  st.body_len = d_body_lens;
  st.flags = flags;
  st.version = version;
  st.type = type;
  st.body_off = boff;
  st.len_eff = blen;
  st.pre = pre;
  const bool lift = (flags & RPC_FRAMES_LIFT_CAP) != 0;
  bool stamped = false;
  if ((rc = ragged(*c, d_stream, boff, blen, n, kModeFinal, bcrc, s, true, lift, nullptr, stream_bytes, nullptr,
                   nullptr, nullptr, &st, &stamped)))
    return rc;
  if (stamped) return RPCCRC_OK; // (route-all: the fold wrote the headers)
  return map_hip(launch_frames_stamp(st, bcrc, n, s));
}

uint32_t rpc_crc32_combine(uint32_t crc1, uint32_t crc2, uint64_t len2) { return crc32_combine(crc1, crc2, len2); }

int rpc_crc32_fill_random_device(void *d_dst, uint64_t nbytes, uint64_t seed, void *stream) {
  if (nbytes == 0) return RPCCRC_OK;
  if (!d_dst || nbytes % 8 != 0) return RPCCRC_EINVAL;
  return map_hip(launch_splitmix_fill(d_dst, nbytes, seed, static_cast<hipStream_t>(stream)));
}

int rpc_crc32_stream_read_device(const void *d_src, uint64_t nbytes, int pattern, int nontemporal, void *stream) {
  if (!d_src || nbytes % 4096 != 0 || pattern < 0 || pattern > 2) return RPCCRC_EINVAL;
  DeviceCtx *c = nullptr;
  int rc = get_async_ctx(&c);
  if (rc) return rc;
  hipStream_t s = static_cast<hipStream_t>(stream);
  if (pattern == 2) { // the rows kernel's dealing and load shape (launch_stream_rows)
    const uint64_t n = nbytes / 4096;
    StealLease sl;
    if ((rc = sl.get(*c, n, 1, s))) return rc;
    if (!sl.p) return RPCCRC_EINVAL; // too small to deal dynamically
    std::call_once(c->probe_once, [c] {
      int prev = 0;
      (void)hipGetDevice(&prev);
      (void)hipSetDevice(c->device);
      void *p = nullptr; // one uint32 per wave of a full grid (kRowsAblNoStore writes at most a.out[gw])
      if (hipMalloc(&p, 16 * 4 * 8 * (size_t)std::max(c->cus, 256)) == hipSuccess) c->probe_sink = static_cast<uint32_t *>(p);
      (void)hipSetDevice(prev);
    });
    if (!c->probe_sink) return RPCCRC_ENOMEM;
    ItemsArgs a = items_args(*c, static_cast<const uint8_t *>(d_src), nullptr, nullptr, n, 4096, 4096, kModeFinal,
                             c->probe_sink);
    a.steal = sl.p;
    return map_hip(launch_stream_rows(a, max_blocks_for(*c), s, sl.done_event(), &sl.recorded));
  }
  return map_hip(launch_stream_read(d_src, nbytes, pattern, nontemporal != 0, max_blocks_for(*c), nullptr, s));
}

int rpc_crc32_set_options(int nontemporal, int max_blocks) {
  if (max_blocks < 0) return RPCCRC_EINVAL;
  g_nontemporal.store(nontemporal ? 1 : 0);
  g_max_blocks.store(max_blocks);
  return RPCCRC_OK;
}

int rpc_crc32_set_ragged_path(int path) {
  if (path != RPCCRC_RAGGED_AUTO && path != RPCCRC_RAGGED_ROWS && path != RPCCRC_RAGGED_PACKED &&
      path != RPCCRC_RAGGED_SPLIT)
    return RPCCRC_EINVAL;
  g_ragged_path.store(path);
  return RPCCRC_OK;
}

int rpc_crc32_device_status(void) {
  DeviceCtx *c = nullptr;
  return get_async_ctx(&c);
}

int rpc_crc32_service_stop(void) { return svc_stop_all(); }

int rpc_crc32_service_stats(rpccrc_service_stats_t *out) {
  if (!out) return RPCCRC_EINVAL;
  memset(out, 0, sizeof(*out));
  std::vector<Service *> vs;
  {
    std::lock_guard<std::mutex> g(g_services_mu);
    vs = g_services;
  }
  for (Service *v : vs) {
    out->services += 1;
    out->running += svc_running(*v) ? 1 : 0;
    out->launched += v->launched.load(std::memory_order_acquire);
    for (const Service::Slot &hs : v->slot) out->answered += hs.answered.load(std::memory_order_relaxed);
    out->fallbacks_full += v->fallbacks_full.load(std::memory_order_relaxed);
    out->fallbacks_short += v->fallbacks_short.load(std::memory_order_relaxed);
    out->bypassed += v->bypassed.load(std::memory_order_relaxed);
  }
  return RPCCRC_OK;
}

int rpc_crc32_device_clear_status(void) {
  DeviceCtx *c = nullptr;
  const int rc = get_ctx(&c);
  if (rc) return rc;
  const int was = device_error(*c);
  *reinterpret_cast<volatile uint32_t *>(c->err) = 0u;
  return was;
}

const char *rpc_crc32_strerror(int err) {
  switch (err) {
  case RPCCRC_OK: return "ok";
  case RPCCRC_EINVAL: return "invalid argument";
  case RPCCRC_ENODEV: return "no usable HIP device (gfx950 with 160 KiB LDS required)";
  case RPCCRC_ENOMEM: return "out of device or pinned memory";
  case RPCCRC_EIO: return "HIP runtime error";
  case RPCCRC_EAGAIN: return "no free receive-ring segment (poll first)";
  default: return "unknown error";
  }
}

int rpc_crc32_device_info(char *buf, size_t buflen) {
  if (!buf || buflen == 0) return RPCCRC_EINVAL;
  DeviceCtx *c = nullptr;
  const int rc = get_ctx(&c);
  if (rc) return rc;
  snprintf(buf, buflen, "device=%s arch=%s cus=%d", c->name, c->arch, c->cus);
  return RPCCRC_OK;
}

} // extern "C"
