// rpc_amd/csrc/frames.h -- wire-frame helpers around the CRC kernels.
// Frame = 12-byte packed big-endian rpc_header_t (reference rpc.h:3-8,15)
// followed by body_len bytes.
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

#include "../../include/rpccrc.h"

namespace rpccrc {

constexpr uint32_t kFrameHeaderLen = 12; // RPC_HEADER_LEN, rpc.h:15
constexpr uint8_t kFramePending = 0xFF;  // data frame whose body CRC decides

__device__ __forceinline__ uint32_t be32(const uint8_t *p) {
  return ((uint32_t)p[0] << 24) | ((uint32_t)p[1] << 16) | ((uint32_t)p[2] << 8) | (uint32_t)p[3];
}
__device__ __forceinline__ uint32_t be16(const uint8_t *p) { return ((uint32_t)p[0] << 8) | (uint32_t)p[1]; }
// Does [off, off + len) lie inside a stream of `bytes` bytes (no wrap-around)?
__device__ __forceinline__ bool inside(uint64_t off, uint64_t len, uint64_t bytes) {
  return off <= bytes && len <= bytes - off;
}

// The header parse of a verify call: frame i's body offset / effective length,
// header crc32 and verdict so far.
struct FramesParse {
  const uint8_t *stream = nullptr;
  uint64_t stream_bytes = 0;
  const uint64_t *frame_off = nullptr; // nullptr: no parse requested
  int flags = 0;
  uint64_t *body_off = nullptr;
  uint32_t *body_len = nullptr;
  uint32_t *hdr_crc = nullptr;
  uint8_t *pre = nullptr;
};
// The reference's decision order for a received header: type (rpc_server_main.c:172
// PING, rpc_async.c:303 PONG), then the body_len cap (rpc_server_main.c:189,
// rpc_async.c:312), then the body is read and its CRC checked
// (rpc_server_main.c:227, rpc_async.c:219).  A frame whose body is not read gets
// length 0 here (its CRC is then 0) and its final verdict now; data frames get
// kFramePending and are decided by the compare (frames_compare_kernel, or the
// route's fold).  The client never verifies a data frame with body_len 0: its
// BODY state recv()s 0 bytes, which returns 0 as soon as anything more (or a
// FIN) is pending on the socket, taken for a closed peer (rpc_async.c:330-349
// -> RPC_RECV_ERR): RPC_FRAME_RECV_ERR.
// A parsed frame's body as stored (the plan uses the values without reading its
// own stores back: one memory round trip less on its critical path).
struct FrameBody {
  uint64_t off;
  uint32_t len;
};
__device__ __forceinline__ FrameBody frames_parse_one(const FramesParse &p, uint64_t i) {
  const uint64_t off = p.frame_off[i];
  uint8_t v = kFramePending;
  uint32_t len = 0, crc = 0;
  if (!inside(off, kFrameHeaderLen, p.stream_bytes)) {
    v = RPC_FRAME_MALFORMED;
  } else {
    const uint8_t *h = p.stream + off;
    const uint32_t type = be16(h + 2); // rpc.h:5
    const uint32_t bl = be32(h + 4);   // rpc.h:6
    crc = be32(h + 8);                 // rpc.h:7
    if ((type == RPC_FRAME_TYPE_PING && (p.flags & RPC_FRAMES_SERVER)) ||
        (type == RPC_FRAME_TYPE_PONG && (p.flags & RPC_FRAMES_CLIENT)))
      v = RPC_FRAME_CONTROL;
    else if (bl > RPC_MAX_BODY_LEN && !(p.flags & RPC_FRAMES_LIFT_CAP))
      v = RPC_FRAME_TOO_LARGE;
    else if (bl == 0 && (p.flags & RPC_FRAMES_CLIENT))
      v = RPC_FRAME_RECV_ERR;
    else if (!inside(off + kFrameHeaderLen, bl, p.stream_bytes))
      v = RPC_FRAME_MALFORMED;
    else
      len = bl;
  }
  const uint64_t boff = (v == kFramePending) ? off + kFrameHeaderLen : 0; // unread bodies: an in-range empty body
  p.body_off[i] = boff;
  p.body_len[i] = len;
  p.hdr_crc[i] = crc;
  p.pre[i] = v;
  return FrameBody{boff, len};
}

// Reads each header (as rpc_server_main.c:165-169 does with ntohs/ntohl) and
// applies the reference's type / cap / bounds rules (frames.hip): the body
// offset and effective length (0 when the body is not read), the header crc32
// and the verdict so far (RPC_FRAME_* or kFramePending).
// The stamp side of a call: frame i's body offset / effective length and its
// verdict (the bounds and the cap, rpc_async.c:499-501), then the 12-byte
// big-endian header of every OK frame (rpc_async.c:521-530: htons / htonl).
struct FramesStamp {
  uint8_t *stream = nullptr;
  uint64_t stream_bytes = 0;
  const uint64_t *frame_off = nullptr; // nullptr: no stamp requested
  const uint32_t *body_len = nullptr;
  int flags = 0;
  uint16_t version = 0, type = 0;
  uint64_t *body_off = nullptr;
  uint32_t *len_eff = nullptr;
  uint8_t *pre = nullptr; // the verdict: OK (stamped), TOO_LARGE or MALFORMED
};
__device__ __forceinline__ FrameBody frames_stamp_prep_one(const FramesStamp &p, uint64_t i) {
  const uint64_t off = p.frame_off[i];
  const uint32_t bl = p.body_len[i];
  uint8_t v = RPC_FRAME_OK;
  if (!inside(off, kFrameHeaderLen, p.stream_bytes) || !inside(off + kFrameHeaderLen, bl, p.stream_bytes))
    v = RPC_FRAME_MALFORMED;
  else if (bl > RPC_MAX_BODY_LEN && !(p.flags & RPC_FRAMES_LIFT_CAP))
    v = RPC_FRAME_TOO_LARGE;
  const FrameBody b{(v == RPC_FRAME_OK) ? off + kFrameHeaderLen : 0, (v == RPC_FRAME_OK) ? bl : 0u};
  p.body_off[i] = b.off;
  p.len_eff[i] = b.len;
  p.pre[i] = v;
  return b;
}
__device__ __forceinline__ void put_be16(uint8_t *p, uint16_t v) {
  p[0] = (uint8_t)(v >> 8);
  p[1] = (uint8_t)v;
}
__device__ __forceinline__ void put_be32(uint8_t *p, uint32_t v) {
  p[0] = (uint8_t)(v >> 24);
  p[1] = (uint8_t)(v >> 16);
  p[2] = (uint8_t)(v >> 8);
  p[3] = (uint8_t)v;
}
// (only header bytes are written: no body's CRC depends on them)
__device__ __forceinline__ void frames_stamp_one(const FramesStamp &p, uint64_t i, uint32_t crc) {
  if (p.pre[i] != RPC_FRAME_OK) return;
  uint8_t *h = p.stream + p.frame_off[i];
  put_be16(h + 0, p.version);
  put_be16(h + 2, p.type);
  put_be32(h + 4, p.body_len[i]);
  put_be32(h + 8, crc);
}

hipError_t launch_frames_parse(const uint8_t *stream, uint64_t stream_bytes, const uint64_t *frame_off, uint64_t n,
                               int flags, uint64_t *body_off, uint32_t *body_len, uint32_t *hdr_crc, uint8_t *pre,
                               hipStream_t s);
// verdict[i] = pre[i], or for pending data frames OK / BAD_CRC by crc == expected.
hipError_t launch_frames_compare(const uint32_t *crc, const uint32_t *expected, const uint8_t *pre, uint64_t n,
                                 uint8_t *verdict, hipStream_t s);
// Stamp side: bounds + cap (rpc_async.c:499-501) -> body offset, effective
// length, OK / TOO_LARGE / MALFORMED (frames_stamp_prep_one); then the header of
// every OK frame (frames_stamp_one).
hipError_t launch_frames_stamp_prep(const FramesStamp &p, uint64_t n, hipStream_t s);
hipError_t launch_frames_stamp(const FramesStamp &p, const uint32_t *crc, uint64_t n, hipStream_t s);

} // namespace rpccrc
