// rpc_amd/csrc/rpccrc_api.cpp -- C-ABI host layer of librpccrc (include/rpccrc.h).
//
// Owns per-device state (table images in HBM, built once per device with
// std::call_once so the drop-in calls stay thread-safe without an init call,
// SURVEY.md 8b "Threading"), per-thread staging for the drop-in scalar path, and
// the host-buffer pipeline of rpc_crc32_batch.  Every CRC value this library
// returns is computed by the HIP kernels in crc32_kernels.hip / frames.hip;
// there is no CPU CRC implementation in the product path.
#include <hip/hip_runtime.h>

#include <errno.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>

#include <algorithm>
#include <mutex>
#include <vector>

#include "../../include/rpccrc.h"
#include "crc32_gf2.h"
#include "crc32_kernels.h"
#include "crc32_layout.h"
#include "frames.h"

namespace rpccrc {
namespace {

constexpr int kMaxDevices = 64;

struct DeviceCtx {
  int device = -1;
  int cus = 0;
  uint4 *img = nullptr;   // LDS table image (v2 layout, 160 KiB)
  uint32_t *tq = nullptr;
  uint4 *shift_nib = nullptr; // NIB[k][i][j] = A_{2^k bytes}(j << 4i) (chunk combine)
  int status = RPCCRC_ENODEV;
  char name[128] = {0};
  char arch[64] = {0};
};

DeviceCtx g_dev[kMaxDevices];
std::once_flag g_once[kMaxDevices];

int g_nontemporal = 1; // streamed once: non-temporal loads (measured faster)
int g_max_blocks = 0;
int g_ragged_path = RPCCRC_RAGGED_AUTO;
// Large-body chunk (rpc_crc32_device_large, chunk_bytes = 0).  C4 per call
// (profiles/r01c4_*): 4 KiB 697 us (rows kernel fastest, combine 27 us),
// 16 KiB 673 us, 64 KiB 689 us (each wave streams its own 64 KiB).
// Tuning override: RPCCRC_LARGE_CHUNK (bytes, multiple of 16).
const uint64_t g_large_chunk = [] {
  const char *e = getenv("RPCCRC_LARGE_CHUNK");
  const unsigned long long v = e ? strtoull(e, nullptr, 10) : 0ull;
  return (v >= 16 && v % 16 == 0 && v <= (1ull << 31)) ? (uint64_t)v : (uint64_t)16384;
}();
constexpr uint32_t kRowsGroupShift = 0;           // rows kernel group dealing, G = 2^shift
constexpr uint64_t kPackedMinBodies = 64;         // fewer frames: one wave per body (rows kernel)
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

int map_hip(hipError_t e) {
  if (e == hipSuccess) return RPCCRC_OK;
  if (e == hipErrorOutOfMemory) return RPCCRC_ENOMEM;
  if (e == hipErrorNoDevice || e == hipErrorInvalidDevice) return RPCCRC_ENODEV;
  if (e == hipErrorInvalidValue) return RPCCRC_EINVAL;
  return RPCCRC_EIO;
}

#define RPCCRC_TRY(expr)                  \
  do {                                    \
    const hipError_t _e = (expr);         \
    if (_e != hipSuccess) return map_hip(_e); \
  } while (0)

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
  if (prop.sharedMemPerBlock < kLdsBytesV2) { // needs the 160 KiB LDS of gfx950
    fprintf(stderr, "rpccrc: device %d (%s) has %zu B LDS per block, need %u\n", dev, c.arch,
            (size_t)prop.sharedMemPerBlock, kLdsBytesV2);
    c.status = RPCCRC_ENODEV;
    return;
  }
  std::vector<uint32_t> img(kLdsBytesV2 / 4), tq(kTqEntries), nib(kShiftNibWords);
  build_tq(tq.data());
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
  e = (e == hipSuccess) ? hipMalloc(&c.img, kLdsBytesV2) : e;
  e = (e == hipSuccess) ? hipMalloc(&c.tq, kTqEntries * 4) : e;
  e = (e == hipSuccess) ? hipMalloc(&c.shift_nib, kShiftNibWords * 4) : e;
  if (e == hipSuccess) {
    build_lds_image_v2(img.data());
    e = hipMemcpy(c.img, img.data(), kLdsBytesV2, hipMemcpyHostToDevice);
  }
  if (e == hipSuccess) e = hipMemcpy(c.tq, tq.data(), kTqEntries * 4, hipMemcpyHostToDevice);
  if (e == hipSuccess) e = hipMemcpy(c.shift_nib, nib.data(), kShiftNibWords * 4, hipMemcpyHostToDevice);
  (void)hipSetDevice(prev);
  c.status = map_hip(e);
}

// Context of the calling thread's current device.
int get_ctx(DeviceCtx **out) {
  int dev = -1;
  if (hipGetDevice(&dev) != hipSuccess || dev < 0 || dev >= kMaxDevices) return RPCCRC_ENODEV;
  int count = 0;
  if (hipGetDeviceCount(&count) != hipSuccess || count <= 0) return RPCCRC_ENODEV;
  std::call_once(g_once[dev], init_device, dev);
  *out = &g_dev[dev];
  return g_dev[dev].status;
}

int max_blocks_for(const DeviceCtx &c) {
  // One 1024-thread workgroup per CU (156 KiB LDS each).
  int mb = c.cus > 0 ? c.cus : 256;
  if (g_max_blocks > 0) mb = std::min(mb * 8, g_max_blocks);
  return mb;
}

int items(const DeviceCtx &c, const uint8_t *base, const uint64_t *offsets, const uint32_t *lengths, uint64_t n,
          uint64_t stride, uint32_t len, uint32_t mode, uint32_t *out, int QB, hipStream_t s) {
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
  return map_hip(launch_rows(a, QB, g_nontemporal != 0, max_blocks_for(c), s));
}

// A ragged batch on the device.  AUTO: frames (bodies capped at MAX_BODY_LEN =
// 1 KiB, rpc.h:17) take the split path (bodies <= 1 KiB four per row through
// the QB = 4 rows kernel: 1M frames 334 us vs 481 packed, 565 rows, DESIGN.md
// 4.2), other batches the rows kernel (one wave per body; ahead on C2's
// 64 B - 64 KiB mix).
int ragged(const DeviceCtx &c, const uint8_t *base, const uint64_t *offsets, const uint32_t *lengths, uint64_t n,
           uint32_t mode, uint32_t *out, hipStream_t s, bool small_bodies = false) {
  const bool fits = n < (1ull << 27); // the packed kernel's metadata window: 8-B offsets in a 1 GiB buffer range
  const bool auto_frames = g_ragged_path == RPCCRC_RAGGED_AUTO && small_bodies && n >= kPackedMinBodies;
  const bool packed = fits && (g_ragged_path == RPCCRC_RAGGED_PACKED || (auto_frames && !kAutoSplitFrames));
  const bool split = !packed && n < 0xFFFFFFFFull &&
                     (g_ragged_path == RPCCRC_RAGGED_SPLIT || (auto_frames && kAutoSplitFrames));
  if (split) {
    size_t bytes = 0;
    RPCCRC_TRY(split_workspace_bytes(n, &bytes));
    void *ws = nullptr;
    RPCCRC_TRY(hipMallocAsync(&ws, bytes, s));
    ItemsArgs a;
    a.base = base;
    a.offsets = offsets;
    a.lengths = lengths;
    a.n_items = n;
    a.mode = mode;
    a.lds_image = c.img;
    a.tq = c.tq;
    a.out = out;
    a.gshift = kRowsGroupShift;
    const int r = map_hip(launch_split_batch(a, ws, bytes, g_nontemporal != 0, max_blocks_for(c), s));
    (void)hipFreeAsync(ws, s);
    return r;
  }
  if (!packed) return items(c, base, offsets, lengths, n, 0, 0, mode, out, 1, s);
  const uint64_t ms = std::min<uint64_t>(kPackedMaxSlices, std::max<uint64_t>(8192, 4 * n));
  size_t bytes = 0;
  RPCCRC_TRY(packed_workspace_bytes(n, ms, &bytes));
  void *ws = nullptr;
  RPCCRC_TRY(hipMallocAsync(&ws, bytes, s));
  PackedBatch p;
  p.base = base;
  p.offsets = offsets;
  p.lengths = lengths;
  p.n = n;
  p.mode = mode;
  p.lds_image = c.img;
  p.tq = c.tq;
  p.out = out;
  p.ws = ws;
  p.ws_bytes = bytes;
  p.max_slices = ms;
  p.min_slice = packed_min_slice();
  const int r = map_hip(launch_packed_batch(p, g_nontemporal != 0, max_blocks_for(c), s));
  (void)hipFreeAsync(ws, s);
  return r;
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

struct PinnedStage {
  void *ptr = nullptr;
  size_t cap = 0;
  hipEvent_t ready = nullptr; // last async consumer of ptr
  bool pending = false;
  int reserve(size_t bytes) {
    if (pending) {
      (void)hipEventSynchronize(ready);
      pending = false;
    }
    if (bytes <= cap) return RPCCRC_OK;
    if (ptr) (void)hipHostFree(ptr);
    ptr = nullptr;
    cap = 0;
    size_t want = std::max<size_t>(bytes, 1 << 16);
    RPCCRC_TRY(hipHostMalloc(&ptr, want, hipHostMallocDefault));
    cap = want;
    if (!ready) RPCCRC_TRY(hipEventCreateWithFlags(&ready, hipEventDisableTiming));
    return RPCCRC_OK;
  }
  void mark(hipStream_t s) {
    (void)hipEventRecord(ready, s);
    pending = true;
  }
};

thread_local PinnedStage t_large_stage;

// Per-thread device workspace, reused by the next call on the same stream
// (stream order makes the reuse safe) and grown when too small.  A
// hipFreeAsync per call blocked the calling thread until the GPU reached it
// and left a ~6 us gap in the stream before the next call's first kernel
// (rocprofv3 --hip-runtime-trace, profiles/r01h_*).  Released when the thread
// switches stream or device or needs more; a thread's last workspace is kept
// until the process ends.
struct StreamWorkspace {
  int dev = -1;
  hipStream_t stream = nullptr;
  void *p = nullptr;
  size_t cap = 0;
  int get(int device, hipStream_t s, size_t bytes, void **out) {
    if (p && (dev != device || stream != s || cap < bytes)) {
      // hipFree, not hipFreeAsync on the old stream: the caller may have
      // destroyed that stream by now.  hipFree waits for the device, so no
      // queued work still uses the old workspace (only on a switch or growth).
      int cur = -1;
      (void)hipGetDevice(&cur);
      if (cur != dev) (void)hipSetDevice(dev);
      (void)hipFree(p);
      if (cur != dev) (void)hipSetDevice(cur);
      p = nullptr;
      cap = 0;
    }
    if (!p) {
      const size_t want = std::max<size_t>(bytes, 1u << 20);
      RPCCRC_TRY(hipMallocAsync(&p, want, s));
      cap = want;
      dev = device;
      stream = s;
    }
    *out = p;
    return RPCCRC_OK;
  }
};
thread_local StreamWorkspace t_large_ws;

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
// blocks that XOR into the zeroed output.
int device_large(const DeviceCtx &c, const uint8_t *d_base, const uint64_t *h_offsets, const uint64_t *h_lengths,
                 uint64_t n, uint32_t *d_out, uint64_t chunk, hipStream_t s) {
  if (chunk % 16 != 0 || chunk > (1ull << 31)) return RPCCRC_EINVAL;
  if (n == 0) return RPCCRC_OK;
  const bool inl = n <= kInlineBodies;
  bool contiguous = inl;
  uint64_t lens_or = 0;
  for (uint64_t i = 0; i < n && contiguous; ++i) {
    lens_or |= h_lengths[i];
    if (i + 1 < n && h_offsets[i + 1] != h_offsets[i] + h_lengths[i]) contiguous = false;
  }
  if (chunk == 0) {
    chunk = g_large_chunk;
    if (contiguous && lens_or % chunk != 0 && !getenv("RPCCRC_LARGE_CHUNK"))
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
  if (!inl) {
    const int rc = t_large_stage.reserve(n * sizeof(BodyDesc));
    if (rc) return rc;
    bd = static_cast<BodyDesc *>(t_large_stage.ptr);
  }
  bool multiple = true;
  for (uint64_t i = 0; i < n; ++i) {
    bd[i].off = h_offsets[i];
    bd[i].len = h_lengths[i];
    bd[i].chunk_first = total;
    const uint64_t nch = (h_lengths[i] + chunk - 1) / chunk;
    total += nch;
    max_nch = std::max(max_nch, nch);
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
  const size_t ws_bytes = fast ? total * 4 + 64 : n * sizeof(BodyDesc) + n * 16 + total * (8 + 4 + 4) + 64;
  uint8_t *ws = nullptr;
  if (const int rc = t_large_ws.get(c.device, s, ws_bytes, reinterpret_cast<void **>(&ws))) return rc;
  int r = RPCCRC_OK;
  uint32_t *d_raw = reinterpret_cast<uint32_t *>(ws);
  uint64_t *d_lens = nullptr, *d_firsts = nullptr;
  if (fast) {
    r = items(c, d_base + h_offsets[0], nullptr, nullptr, total, chunk, (uint32_t)chunk, kModeRaw, d_raw, 1, s);
  } else {
    BodyDesc *d_bodies = reinterpret_cast<BodyDesc *>(ws);
    d_lens = reinterpret_cast<uint64_t *>(ws + n * sizeof(BodyDesc));
    d_firsts = d_lens + n;
    uint64_t *d_ioff = d_firsts + n;
    uint32_t *d_ilen = reinterpret_cast<uint32_t *>(d_ioff + total);
    d_raw = d_ilen + total;
    hipError_t e = hipSuccess;
    if (!inl) {
      e = hipMemcpyAsync(d_bodies, bd, n * sizeof(BodyDesc), hipMemcpyHostToDevice, s);
      t_large_stage.mark(s);
      if (e != hipSuccess) {
        // the workspace stays cached for the next call on this stream
        return map_hip(e);
      }
    }
    const uint64_t threads = std::max<uint64_t>(total, n);
    const dim3 eg((unsigned)((threads + 255) / 256));
    if (inl)
      hipLaunchKernelGGL(expand_chunks_inline_kernel, eg, dim3(256), 0, s, ib, n, chunk, total, d_ioff, d_ilen, d_lens,
                         d_firsts, d_out);
    else
      hipLaunchKernelGGL(expand_chunks_kernel, eg, dim3(256), 0, s, d_bodies, n, chunk, total, d_ioff, d_ilen, d_lens,
                         d_firsts, d_out);
    r = map_hip(hipGetLastError());
    if (r == RPCCRC_OK) r = items(c, d_base, d_ioff, d_ilen, total, 0, 0, kModeRaw, d_raw, 1, s);
  }
  if (r == RPCCRC_OK) {
    CombineArgs ca;
    ca.raw = d_raw;
    ca.lengths = d_lens;
    ca.chunk_first = d_firsts;
    ca.shift_nib = c.shift_nib;
    ca.n_bodies = n;
    ca.chunk = chunk;
    ca.out = d_out;
    ca.splits = (uint32_t)splits;
    ca.inline_bodies = inl;
    if (inl) ca.bodies = ib;
    r = map_hip(launch_chunk_combine(ca, s));
  }
  // the workspace stays cached for the next call on this stream (no hipFreeAsync)
  return r;
}

// ---- per-thread staging for the drop-in scalar path --------------------------

struct ScalarCtx {
  int device = -1;
  hipStream_t stream = nullptr;
  uint8_t *pin = nullptr; // pinned input staging, device-readable
  size_t cap = 0;
  uint32_t *pout = nullptr; // pinned result
  uint8_t *dbuf = nullptr; // device staging for large bodies
  size_t dcap = 0;
};
thread_local ScalarCtx t_scalar;

[[noreturn]] void die(const char *what, int rc) {
  fprintf(stderr, "rpccrc: %s failed (%s); librpccrc requires a usable HIP device and has no CPU fallback\n", what,
          rpc_crc32_strerror(rc));
  abort();
}

constexpr size_t kScalarZeroCopyMax = 64 << 10;  // read straight from pinned memory
constexpr uint64_t kScalarChunkedMin = 8 << 20;  // chunk + combine above this

uint32_t scalar_crc(const void *data, uint32_t len) {
  DeviceCtx *c = nullptr;
  int rc = get_ctx(&c);
  if (rc) die("device init", rc);
  ScalarCtx &t = t_scalar;
  int dev = 0;
  (void)hipGetDevice(&dev);
  if (t.device != dev) {
    t.device = dev;
    if (hipStreamCreateWithFlags(&t.stream, hipStreamNonBlocking) != hipSuccess) die("stream create", RPCCRC_EIO);
    if (hipHostMalloc(reinterpret_cast<void **>(&t.pout), 64, hipHostMallocDefault) != hipSuccess)
      die("pinned alloc", RPCCRC_ENOMEM);
    t.pin = nullptr;
    t.cap = 0;
    t.dbuf = nullptr;
    t.dcap = 0;
  }
  const uint8_t *src = static_cast<const uint8_t *>(data);
  if (len <= kScalarZeroCopyMax) {
    if (t.cap < len || !t.pin) {
      if (t.pin) (void)hipHostFree(t.pin);
      t.cap = kScalarZeroCopyMax;
      if (hipHostMalloc(reinterpret_cast<void **>(&t.pin), t.cap, hipHostMallocDefault) != hipSuccess)
        die("pinned alloc", RPCCRC_ENOMEM);
    }
    memcpy(t.pin, src, len);
    rc = items(*c, t.pin, nullptr, nullptr, 1, 0, len, kModeFinal, t.pout, 1, t.stream);
  } else {
    if (t.dcap < len) {
      if (t.dbuf) (void)hipFree(t.dbuf);
      t.dbuf = nullptr;
      if (hipMalloc(reinterpret_cast<void **>(&t.dbuf), len) != hipSuccess) die("device alloc", RPCCRC_ENOMEM);
      t.dcap = len;
    }
    if (hipMemcpyAsync(t.dbuf, src, len, hipMemcpyHostToDevice, t.stream) != hipSuccess) die("H2D copy", RPCCRC_EIO);
    if (len >= kScalarChunkedMin) {
      const uint64_t off = 0, l64 = len;
      rc = device_large(*c, t.dbuf, &off, &l64, 1, t.pout, 0, t.stream);
    } else {
      rc = items(*c, t.dbuf, nullptr, nullptr, 1, 0, len, kModeFinal, t.pout, 1, t.stream);
    }
  }
  if (rc) die("kernel launch", rc);
  if (hipStreamSynchronize(t.stream) != hipSuccess) die("stream sync", RPCCRC_EIO);
  return *t.pout;
}

// ---- host-buffer batch pipeline ----------------------------------------------

constexpr uint64_t kStageBytes = 256ull << 20; // device staging per pipeline slot
constexpr uint64_t kStageMaxBodies = 1ull << 20;

struct HostSlot {
  hipStream_t stream = nullptr;
  uint8_t *dbuf = nullptr;   // device copy of the group's span
  uint64_t *doff = nullptr;  // rebased offsets
  uint32_t *dlen = nullptr;
  uint32_t *dout = nullptr;
  uint64_t *hoff = nullptr;  // pinned staging for metadata
  uint32_t *hlen = nullptr;
  uint32_t *hout = nullptr;
  uint64_t first = 0, count = 0; // bodies of the group in flight
  bool busy = false;
};

struct HostPipeline {
  int device = -1;
  HostSlot slot[2];
  bool ok = false;
};
thread_local HostPipeline t_pipe;

int pipe_init(HostPipeline &p, int dev) {
  if (p.device == dev && p.ok) return RPCCRC_OK;
  p.device = dev;
  p.ok = false;
  for (HostSlot &s : p.slot) {
    RPCCRC_TRY(hipStreamCreateWithFlags(&s.stream, hipStreamNonBlocking));
    RPCCRC_TRY(hipMalloc(&s.dbuf, kStageBytes));
    RPCCRC_TRY(hipMalloc(&s.doff, kStageMaxBodies * 8));
    RPCCRC_TRY(hipMalloc(&s.dlen, kStageMaxBodies * 4));
    RPCCRC_TRY(hipMalloc(&s.dout, kStageMaxBodies * 4));
    RPCCRC_TRY(hipHostMalloc(reinterpret_cast<void **>(&s.hoff), kStageMaxBodies * 8, hipHostMallocDefault));
    RPCCRC_TRY(hipHostMalloc(reinterpret_cast<void **>(&s.hlen), kStageMaxBodies * 4, hipHostMallocDefault));
    RPCCRC_TRY(hipHostMalloc(reinterpret_cast<void **>(&s.hout), kStageMaxBodies * 4, hipHostMallocDefault));
  }
  p.ok = true;
  return RPCCRC_OK;
}

int slot_drain(HostSlot &s, uint32_t *out) {
  if (!s.busy) return RPCCRC_OK;
  RPCCRC_TRY(hipStreamSynchronize(s.stream));
  memcpy(out + s.first, s.hout, s.count * 4);
  s.busy = false;
  return RPCCRC_OK;
}

int host_batch(const DeviceCtx &c, const uint8_t *base, const uint64_t *offsets, const uint32_t *lengths, uint64_t n,
               uint32_t *out) {
  int dev = 0;
  (void)hipGetDevice(&dev);
  int rc = pipe_init(t_pipe, dev);
  if (rc) return rc;
  HostPipeline &p = t_pipe;
  uint64_t i = 0;
  int which = 0;
  while (i < n) {
    // Bodies larger than a stage go through the chunked large path on their own.
    if ((uint64_t)lengths[i] > kStageBytes) {
      for (HostSlot &s : p.slot)
        if ((rc = slot_drain(s, out))) return rc;
      HostSlot &s = p.slot[0];
      uint8_t *dtmp = nullptr;
      const uint64_t L = lengths[i];
      RPCCRC_TRY(hipMallocAsync(reinterpret_cast<void **>(&dtmp), L, s.stream));
      RPCCRC_TRY(hipMemcpyAsync(dtmp, base + offsets[i], L, hipMemcpyHostToDevice, s.stream));
      const uint64_t zero = 0;
      rc = device_large(c, dtmp, &zero, &L, 1, s.dout, 0, s.stream);
      (void)hipFreeAsync(dtmp, s.stream);
      if (rc) return rc;
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
    rc = ragged(c, s.dbuf, s.doff, s.dlen, cnt, kModeFinal, s.dout, s.stream);
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
  if (n == 0) return RPCCRC_OK;
  if (!d_base || !d_offsets || !d_lengths || !d_out) return RPCCRC_EINVAL;
  DeviceCtx *c = nullptr;
  int rc = get_ctx(&c);
  if (rc) return rc;
  return ragged(*c, d_base, d_offsets, d_lengths, n, kModeFinal, d_out, static_cast<hipStream_t>(stream));
}

int rpc_crc32_device_uniform(const uint8_t *d_base, uint64_t n, uint32_t body_len, uint64_t stride, uint32_t *d_out,
                             void *stream) {
  if (n == 0) return RPCCRC_OK;
  if (!d_base || !d_out) return RPCCRC_EINVAL;
  DeviceCtx *c = nullptr;
  int rc = get_ctx(&c);
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
  int rc = get_ctx(&c);
  if (rc) return rc;
  return device_large(*c, d_base, h_offsets, h_lengths, n, d_out, chunk_bytes, static_cast<hipStream_t>(stream));
}

int rpc_frames_verify_device(const uint8_t *d_stream, const uint64_t *d_frame_offsets, uint64_t n, uint8_t *d_ok,
                             uint32_t *d_crc, void *stream) {
  if (n == 0) return RPCCRC_OK;
  if (!d_stream || !d_frame_offsets || !d_ok) return RPCCRC_EINVAL;
  DeviceCtx *c = nullptr;
  int rc = get_ctx(&c);
  if (rc) return rc;
  hipStream_t s = static_cast<hipStream_t>(stream);
  uint8_t *ws = nullptr;
  const size_t ws_bytes = n * (8 + 4 + 4 + 4);
  RPCCRC_TRY(hipMallocAsync(reinterpret_cast<void **>(&ws), ws_bytes, s));
  uint64_t *boff = reinterpret_cast<uint64_t *>(ws);
  uint32_t *blen = reinterpret_cast<uint32_t *>(boff + n);
  uint32_t *bexp = blen + n;
  uint32_t *bcrc = d_crc ? d_crc : bexp + n;
  rc = map_hip(launch_frames_parse(d_stream, d_frame_offsets, n, boff, blen, bexp, s));
  if (rc == RPCCRC_OK) rc = ragged(*c, d_stream, boff, blen, n, kModeFinal, bcrc, s, true);
  if (rc == RPCCRC_OK) rc = map_hip(launch_frames_compare(bcrc, bexp, n, d_ok, s));
  (void)hipFreeAsync(ws, s);
  return rc;
}

int rpc_frames_stamp_device(uint8_t *d_stream, const uint64_t *d_frame_offsets, const uint32_t *d_body_lens,
                            uint64_t n, uint16_t version, uint16_t type, void *stream) {
  if (n == 0) return RPCCRC_OK;
  if (!d_stream || !d_frame_offsets || !d_body_lens) return RPCCRC_EINVAL;
  DeviceCtx *c = nullptr;
  int rc = get_ctx(&c);
  if (rc) return rc;
  hipStream_t s = static_cast<hipStream_t>(stream);
  uint8_t *ws = nullptr;
  RPCCRC_TRY(hipMallocAsync(reinterpret_cast<void **>(&ws), n * (8 + 4), s));
  uint64_t *boff = reinterpret_cast<uint64_t *>(ws);
  uint32_t *bcrc = reinterpret_cast<uint32_t *>(boff + n);
  rc = map_hip(launch_frames_body_offsets(d_frame_offsets, n, boff, s));
  if (rc == RPCCRC_OK) rc = ragged(*c, d_stream, boff, d_body_lens, n, kModeFinal, bcrc, s, true);
  if (rc == RPCCRC_OK)
    rc = map_hip(launch_frames_stamp(d_stream, d_frame_offsets, d_body_lens, bcrc, n, version, type, s));
  (void)hipFreeAsync(ws, s);
  return rc;
}

uint32_t rpc_crc32_combine(uint32_t crc1, uint32_t crc2, uint64_t len2) { return crc32_combine(crc1, crc2, len2); }

int rpc_crc32_fill_random_device(void *d_dst, uint64_t nbytes, uint64_t seed, void *stream) {
  if (nbytes == 0) return RPCCRC_OK;
  if (!d_dst || nbytes % 8 != 0) return RPCCRC_EINVAL;
  return map_hip(launch_splitmix_fill(d_dst, nbytes, seed, static_cast<hipStream_t>(stream)));
}

int rpc_crc32_stream_read_device(const void *d_src, uint64_t nbytes, int pattern, int nontemporal, void *stream) {
  if (!d_src || nbytes % 4096 != 0 || (pattern != 0 && pattern != 1)) return RPCCRC_EINVAL;
  DeviceCtx *c = nullptr;
  int rc = get_ctx(&c);
  if (rc) return rc;
  return map_hip(launch_stream_read(d_src, nbytes, pattern, nontemporal != 0, max_blocks_for(*c), nullptr,
                                    static_cast<hipStream_t>(stream)));
}

int rpc_crc32_set_options(int nontemporal, int max_blocks) {
  if (max_blocks < 0) return RPCCRC_EINVAL;
  g_nontemporal = nontemporal ? 1 : 0;
  g_max_blocks = max_blocks;
  return RPCCRC_OK;
}

int rpc_crc32_set_ragged_path(int path) {
  if (path != RPCCRC_RAGGED_AUTO && path != RPCCRC_RAGGED_ROWS && path != RPCCRC_RAGGED_PACKED &&
      path != RPCCRC_RAGGED_SPLIT)
    return RPCCRC_EINVAL;
  g_ragged_path = path;
  return RPCCRC_OK;
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
