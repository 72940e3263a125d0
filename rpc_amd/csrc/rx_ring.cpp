// rpc_amd/csrc/rx_ring.cpp -- batched server receive ring.
//
// The reference server handles one frame at a time: a blocking recv of the
// 12-byte header, a recv loop for the body, rpc_crc32_verify, dispatch
// (server/rpc_server_main.c:135-238; verify at :227).  The ring lets a receive
// loop land many frames -- from any number of connections -- directly in
// pinned host SEGMENTS (rpc_rx_ring_reserve hands out the destination for
// recv()), and verifies a whole segment with one H2D copy, one
// rpc_frames_verify_device launch (header parse with the reference's type / cap
// rules, CRC kernels, compare) and one D2H copy of the verdicts, while the next
// segment fills.  Results come
// back in arrival order with the caller's tag (e.g. the connection fd), so the
// dispatch step stays as it is.
//
// Segment life cycle: FREE -> FILLING (reserve/commit) -> INFLIGHT (submit, or
// a reserve that does not fit) -> returned by poll -> FREE at the next poll.
// A ring belongs to one thread (like the reference's single-threaded server
// loop); distinct rings are independent.
#include <hip/hip_runtime.h>

#include <stdlib.h>
#include <string.h>

#include <new>
#include <vector>

#include "../../include/rpccrc.h"

namespace {

constexpr size_t kHdr = 12; // RPC_HEADER_LEN (rpc.h:15)

uint32_t be32(const uint8_t *p) {
  return ((uint32_t)p[0] << 24) | ((uint32_t)p[1] << 16) | ((uint32_t)p[2] << 8) | (uint32_t)p[3];
}
uint16_t be16(const uint8_t *p) { return (uint16_t)(((uint32_t)p[0] << 8) | (uint32_t)p[1]); }

int map_hip(hipError_t e) {
  if (e == hipSuccess) return RPCCRC_OK;
  if (e == hipErrorOutOfMemory) return RPCCRC_ENOMEM;
  if (e == hipErrorNoDevice || e == hipErrorInvalidDevice) return RPCCRC_ENODEV;
  if (e == hipErrorInvalidValue) return RPCCRC_EINVAL;
  return RPCCRC_EIO;
}

enum SegState { kFree, kFilling, kInflight };

struct Segment {
  uint8_t *h_buf = nullptr;  // pinned frames, back to back
  uint64_t *h_off = nullptr; // pinned frame offsets
  uint8_t *h_verdict = nullptr; // pinned verdicts (D2H)
  uint32_t *h_crc = nullptr; // pinned body CRCs (D2H)
  uint8_t *d_buf = nullptr;
  uint64_t *d_off = nullptr;
  uint8_t *d_verdict = nullptr;
  uint32_t *d_crc = nullptr;
  std::vector<uint64_t> tags;
  size_t used = 0, nframes = 0;
  hipEvent_t done = nullptr;
  SegState state = kFree;
};

// Runs with the ring's device current, restoring the caller's afterwards.
struct DeviceGuard {
  int prev = -1;
  explicit DeviceGuard(int dev) {
    (void)hipGetDevice(&prev);
    if (prev != dev) (void)hipSetDevice(dev);
  }
  ~DeviceGuard() {
    int cur = -1;
    (void)hipGetDevice(&cur);
    if (prev >= 0 && cur != prev) (void)hipSetDevice(prev);
  }
};

} // namespace

struct rpc_rx_ring {
  int device = -1;
  int flags = 0; // RPC_FRAMES_* (role, LIFT_CAP)
  hipStream_t stream = nullptr;
  size_t seg_bytes = 0, max_frames = 0;
  std::vector<Segment> seg;
  size_t fill = 0;              // segment being filled (or the next one to fill)
  size_t head = 0;              // oldest segment not yet fully returned by poll
  size_t head_pos = 0;          // frames of `head` already returned
  bool release_head = false;    // head fully returned: free it at the next poll
  uint8_t *reserved = nullptr;  // outstanding reservation
  size_t reserved_len = 0;
};

namespace {

void free_ring(rpc_rx_ring *r) {
  if (!r) return;
  DeviceGuard g(r->device);
  if (r->stream) (void)hipStreamSynchronize(r->stream);
  for (Segment &s : r->seg) {
    if (s.h_buf) (void)hipHostFree(s.h_buf);
    if (s.h_off) (void)hipHostFree(s.h_off);
    if (s.h_verdict) (void)hipHostFree(s.h_verdict);
    if (s.h_crc) (void)hipHostFree(s.h_crc);
    if (s.d_buf) (void)hipFree(s.d_buf);
    if (s.d_off) (void)hipFree(s.d_off);
    if (s.d_verdict) (void)hipFree(s.d_verdict);
    if (s.d_crc) (void)hipFree(s.d_crc);
    if (s.done) (void)hipEventDestroy(s.done);
  }
  if (r->stream) (void)hipStreamDestroy(r->stream);
  delete r;
}

// Send the filling segment to the GPU: H2D of its frames and offsets, frames
// verify, D2H of the verdicts and CRCs, all stream-ordered.
int submit_fill(rpc_rx_ring *r) {
  Segment &s = r->seg[r->fill];
  if (s.state != kFilling || s.nframes == 0) return RPCCRC_OK;
  hipError_t e = hipMemcpyAsync(s.d_buf, s.h_buf, s.used, hipMemcpyHostToDevice, r->stream);
  if (e == hipSuccess) e = hipMemcpyAsync(s.d_off, s.h_off, s.nframes * 8, hipMemcpyHostToDevice, r->stream);
  if (e != hipSuccess) return map_hip(e);
  const int rc =
      rpc_frames_verify_device(s.d_buf, s.used, s.d_off, s.nframes, r->flags, s.d_verdict, s.d_crc, r->stream);
  if (rc != RPCCRC_OK) return rc;
  e = hipMemcpyAsync(s.h_verdict, s.d_verdict, s.nframes, hipMemcpyDeviceToHost, r->stream);
  if (e == hipSuccess) e = hipMemcpyAsync(s.h_crc, s.d_crc, s.nframes * 4, hipMemcpyDeviceToHost, r->stream);
  if (e == hipSuccess) e = hipEventRecord(s.done, r->stream);
  if (e != hipSuccess) return map_hip(e);
  s.state = kInflight;
  r->fill = (r->fill + 1) % r->seg.size();
  return RPCCRC_OK;
}

} // namespace

extern "C" {

int rpc_rx_ring_create(rpc_rx_ring_t **ring, size_t segment_bytes, size_t max_frames, int nsegments, int flags) {
  if (!ring) return RPCCRC_EINVAL;
  *ring = nullptr;
  if (segment_bytes < kHdr || max_frames == 0 || nsegments < 2 || nsegments > 64) return RPCCRC_EINVAL;
  const int role = flags & (RPC_FRAMES_SERVER | RPC_FRAMES_CLIENT);
  if ((flags & ~(RPC_FRAMES_SERVER | RPC_FRAMES_CLIENT | RPC_FRAMES_LIFT_CAP)) != 0 ||
      (role != RPC_FRAMES_SERVER && role != RPC_FRAMES_CLIENT))
    return RPCCRC_EINVAL;
  int dev = -1, count = 0;
  if (hipGetDeviceCount(&count) != hipSuccess || count <= 0 || hipGetDevice(&dev) != hipSuccess)
    return RPCCRC_ENODEV;
  rpc_rx_ring *r = new (std::nothrow) rpc_rx_ring;
  if (!r) return RPCCRC_ENOMEM;
  r->device = dev;
  r->flags = flags;
  r->seg_bytes = segment_bytes;
  r->max_frames = max_frames;
  r->seg.resize((size_t)nsegments);
  hipError_t e = hipStreamCreateWithFlags(&r->stream, hipStreamNonBlocking);
  for (Segment &s : r->seg) {
    if (e == hipSuccess) e = hipHostMalloc(reinterpret_cast<void **>(&s.h_buf), segment_bytes, hipHostMallocDefault);
    if (e == hipSuccess) e = hipHostMalloc(reinterpret_cast<void **>(&s.h_off), max_frames * 8, hipHostMallocDefault);
    if (e == hipSuccess) e = hipHostMalloc(reinterpret_cast<void **>(&s.h_verdict), max_frames, hipHostMallocDefault);
    if (e == hipSuccess) e = hipHostMalloc(reinterpret_cast<void **>(&s.h_crc), max_frames * 4, hipHostMallocDefault);
    if (e == hipSuccess) e = hipMalloc(reinterpret_cast<void **>(&s.d_buf), segment_bytes);
    if (e == hipSuccess) e = hipMalloc(reinterpret_cast<void **>(&s.d_off), max_frames * 8);
    if (e == hipSuccess) e = hipMalloc(reinterpret_cast<void **>(&s.d_verdict), max_frames);
    if (e == hipSuccess) e = hipMalloc(reinterpret_cast<void **>(&s.d_crc), max_frames * 4);
    if (e == hipSuccess) e = hipEventCreateWithFlags(&s.done, hipEventDisableTiming);
    if (e == hipSuccess) s.tags.reserve(max_frames);
  }
  if (e != hipSuccess) {
    free_ring(r);
    return map_hip(e);
  }
  *ring = r;
  return RPCCRC_OK;
}

void rpc_rx_ring_destroy(rpc_rx_ring_t *ring) { free_ring(ring); }

int rpc_rx_ring_reserve(rpc_rx_ring_t *r, size_t frame_len, uint8_t **dst) {
  if (!r || !dst) return RPCCRC_EINVAL;
  *dst = nullptr;
  if (frame_len < kHdr || frame_len > r->seg_bytes) return RPCCRC_EINVAL;
  DeviceGuard g(r->device);
  Segment *s = &r->seg[r->fill];
  if (s->state == kFilling && (s->used + frame_len > r->seg_bytes || s->nframes == r->max_frames)) {
    const int rc = submit_fill(r); // the full segment goes to the GPU; fill the next one
    if (rc != RPCCRC_OK) return rc;
    s = &r->seg[r->fill];
  }
  if (s->state == kInflight) return RPCCRC_EAGAIN; // every segment busy: poll first
  if (s->state == kFree) {
    s->state = kFilling;
    s->used = 0;
    s->nframes = 0;
    s->tags.clear();
  }
  r->reserved = s->h_buf + s->used;
  r->reserved_len = frame_len;
  *dst = r->reserved;
  return RPCCRC_OK;
}

int rpc_rx_ring_commit(rpc_rx_ring_t *r, uint64_t tag) {
  if (!r || !r->reserved) return RPCCRC_EINVAL;
  Segment &s = r->seg[r->fill];
  const uint8_t *h = r->reserved;
  const size_t len = r->reserved_len;
  r->reserved = nullptr;
  r->reserved_len = 0;
  // The landed length must be exactly what the reference reads for this
  // header: the header alone for a control frame (rpc_server_main.c:172-187
  // PING at the server, rpc_async.c:303-309 PONG at the client) or a data
  // frame over the cap (rpc_server_main.c:189-195, rpc_async.c:312: dropped
  // before the body) -- any bytes after such a header are the NEXT frame's to
  // the reference, so a landing that includes them is refused -- else the
  // header plus body_len bytes (rpc.h:6).
  const uint64_t bl = be32(h + 4);
  const uint16_t type = be16(h + 2);
  const bool control = (type == RPC_FRAME_TYPE_PING && (r->flags & RPC_FRAMES_SERVER)) ||
                       (type == RPC_FRAME_TYPE_PONG && (r->flags & RPC_FRAMES_CLIENT));
  const bool over_cap = bl > RPC_MAX_BODY_LEN && !(r->flags & RPC_FRAMES_LIFT_CAP);
  const uint64_t want = (control || over_cap) ? kHdr : bl + kHdr;
  if (len != want) return RPCCRC_EINVAL;
  s.h_off[s.nframes] = s.used;
  s.tags.push_back(tag);
  s.used += len;
  s.nframes += 1;
  return RPCCRC_OK;
}

int rpc_rx_ring_push(rpc_rx_ring_t *r, const void *frame, size_t frame_len, uint64_t tag) {
  if (!frame) return RPCCRC_EINVAL;
  uint8_t *dst = nullptr;
  const int rc = rpc_rx_ring_reserve(r, frame_len, &dst);
  if (rc != RPCCRC_OK) return rc;
  memcpy(dst, frame, frame_len);
  return rpc_rx_ring_commit(r, tag);
}

int rpc_rx_ring_submit(rpc_rx_ring_t *r) {
  if (!r) return RPCCRC_EINVAL;
  DeviceGuard g(r->device);
  r->reserved = nullptr; // an uncommitted reservation is dropped
  r->reserved_len = 0;
  return submit_fill(r);
}

int64_t rpc_rx_ring_poll(rpc_rx_ring_t *r, rpc_rx_frame_t *out, size_t max_frames, int wait) {
  if (!r || (!out && max_frames)) return RPCCRC_EINVAL;
  DeviceGuard g(r->device);
  if (r->release_head) { // its frames were returned by the previous poll
    r->seg[r->head].state = kFree;
    r->head = (r->head + 1) % r->seg.size();
    r->head_pos = 0;
    r->release_head = false;
  }
  Segment &h = r->seg[r->head];
  if (h.state != kInflight || max_frames == 0) return 0;
  if (wait) {
    const hipError_t e = hipEventSynchronize(h.done);
    if (e != hipSuccess) return map_hip(e);
  } else {
    const hipError_t e = hipEventQuery(h.done);
    if (e == hipErrorNotReady) return 0;
    if (e != hipSuccess) return map_hip(e);
  }
  size_t n = h.nframes - r->head_pos;
  if (n > max_frames) n = max_frames;
  for (size_t i = 0; i < n; ++i) {
    const size_t k = r->head_pos + i;
    const uint8_t *f = h.h_buf + h.h_off[k];
    rpc_rx_frame_t &o = out[i];
    o.tag = h.tags[k];
    o.frame = f;
    o.body_len = be32(f + 4); // the header field (a control / over-cap frame landed no body)
    o.version = be16(f);
    o.type = be16(f + 2);
    o.header_crc = be32(f + 8);
    o.crc = h.h_crc[k];
    o.verdict = h.h_verdict[k];
    o.ok = (o.verdict == RPC_FRAME_OK || o.verdict == RPC_FRAME_CONTROL) ? 1 : 0;
  }
  r->head_pos += n;
  if (r->head_pos == h.nframes) r->release_head = true;
  return (int64_t)n;
}

} // extern "C"
