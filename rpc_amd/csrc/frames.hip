// rpc_amd/csrc/frames.hip -- batched frame verify / stamp helpers (SURVEY.md 8f
// rows 1 and 3).  Header parse and stamp are tiny byte kernels; the body CRCs
// come from the same ragged path as every other batch (rows kernel, plus the
// chunk route for large bodies when the MAX_BODY_LEN cap is lifted).
#include "../../include/rpccrc.h"
#include "frames.h"

namespace rpccrc {

namespace {
__device__ __forceinline__ uint32_t be32(const uint8_t *p) {
  return ((uint32_t)p[0] << 24) | ((uint32_t)p[1] << 16) | ((uint32_t)p[2] << 8) | (uint32_t)p[3];
}
__device__ __forceinline__ uint32_t be16(const uint8_t *p) { return ((uint32_t)p[0] << 8) | (uint32_t)p[1]; }
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

// Does [off, off + len) lie inside a stream of `bytes` bytes (no wrap-around)?
__device__ __forceinline__ bool inside(uint64_t off, uint64_t len, uint64_t bytes) {
  return off <= bytes && len <= bytes - off;
}

// The reference's decision order for a received header: type (rpc_server_main.c:172
// PING, rpc_async.c:303 PONG), then the body_len cap (rpc_server_main.c:189,
// rpc_async.c:312), then the body is read and its CRC checked
// (rpc_server_main.c:227, rpc_async.c:219).  A frame whose body is not read gets
// length 0 here (its CRC is then 0) and its final verdict now; data frames get
// kFramePending and are decided by frames_compare_kernel.  The client never
// verifies a data frame with body_len 0: its BODY state recv()s 0 bytes, which
// returns 0 as soon as anything more (or a FIN) is pending on the socket, taken
// for a closed peer (rpc_async.c:330-349 -> RPC_RECV_ERR): RPC_FRAME_RECV_ERR.
__global__ void frames_parse_kernel(const uint8_t *stream, uint64_t stream_bytes, const uint64_t *frame_off,
                                    uint64_t n, int flags, uint64_t *body_off, uint32_t *body_len, uint32_t *hdr_crc,
                                    uint8_t *pre) {
  const uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n) return;
  const uint64_t off = frame_off[i];
  uint8_t v = kFramePending;
  uint32_t len = 0, crc = 0;
  if (!inside(off, kFrameHeaderLen, stream_bytes)) {
    v = RPC_FRAME_MALFORMED;
  } else {
    const uint8_t *h = stream + off;
    const uint32_t type = be16(h + 2); // rpc.h:5
    const uint32_t bl = be32(h + 4);   // rpc.h:6
    crc = be32(h + 8);                 // rpc.h:7
    if ((type == RPC_FRAME_TYPE_PING && (flags & RPC_FRAMES_SERVER)) ||
        (type == RPC_FRAME_TYPE_PONG && (flags & RPC_FRAMES_CLIENT)))
      v = RPC_FRAME_CONTROL;
    else if (bl > RPC_MAX_BODY_LEN && !(flags & RPC_FRAMES_LIFT_CAP))
      v = RPC_FRAME_TOO_LARGE;
    else if (bl == 0 && (flags & RPC_FRAMES_CLIENT))
      v = RPC_FRAME_RECV_ERR;
    else if (!inside(off + kFrameHeaderLen, bl, stream_bytes))
      v = RPC_FRAME_MALFORMED;
    else
      len = bl;
  }
  body_off[i] = (v == kFramePending) ? off + kFrameHeaderLen : 0; // unread bodies: an in-range empty body
  body_len[i] = len;
  hdr_crc[i] = crc;
  pre[i] = v;
}

__global__ void frames_compare_kernel(const uint32_t *crc, const uint32_t *expected, const uint8_t *pre, uint64_t n,
                                      uint8_t *verdict) {
  const uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n) return;
  const uint8_t p = pre[i];
  verdict[i] = (p != kFramePending) ? p : (crc[i] == expected[i] ? RPC_FRAME_OK : RPC_FRAME_BAD_CRC);
}

// Stamp side: the body of frame i must lie inside the stream, and without
// LIFT_CAP be at most MAX_BODY_LEN (rpc_async.c:499-501 refuses to send it).
__global__ void frames_stamp_prep_kernel(uint64_t stream_bytes, const uint64_t *frame_off, const uint32_t *body_len,
                                         uint64_t n, int flags, uint64_t *body_off, uint32_t *len_eff, uint8_t *pre) {
  const uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n) return;
  const uint64_t off = frame_off[i];
  const uint32_t bl = body_len[i];
  uint8_t v = RPC_FRAME_OK;
  if (!inside(off, kFrameHeaderLen, stream_bytes) || !inside(off + kFrameHeaderLen, bl, stream_bytes))
    v = RPC_FRAME_MALFORMED;
  else if (bl > RPC_MAX_BODY_LEN && !(flags & RPC_FRAMES_LIFT_CAP))
    v = RPC_FRAME_TOO_LARGE;
  body_off[i] = (v == RPC_FRAME_OK) ? off + kFrameHeaderLen : 0;
  len_eff[i] = (v == RPC_FRAME_OK) ? bl : 0u;
  pre[i] = v;
}

__global__ void frames_stamp_kernel(uint8_t *stream, const uint64_t *frame_off, const uint32_t *body_len,
                                    const uint32_t *crc, const uint8_t *pre, uint64_t n, uint16_t version,
                                    uint16_t type) {
  const uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n || pre[i] != RPC_FRAME_OK) return;
  uint8_t *h = stream + frame_off[i];
  put_be16(h + 0, version);
  put_be16(h + 2, type);
  put_be32(h + 4, body_len[i]);
  put_be32(h + 8, crc[i]);
}

dim3 grid_for(uint64_t n) { return dim3((unsigned)((n + 255) / 256)); }
} // namespace

hipError_t launch_frames_parse(const uint8_t *stream, uint64_t stream_bytes, const uint64_t *frame_off, uint64_t n,
                               int flags, uint64_t *body_off, uint32_t *body_len, uint32_t *hdr_crc, uint8_t *pre,
                               hipStream_t s) {
  hipLaunchKernelGGL(frames_parse_kernel, grid_for(n), dim3(256), 0, s, stream, stream_bytes, frame_off, n, flags,
                     body_off, body_len, hdr_crc, pre);
  return hipGetLastError();
}

hipError_t launch_frames_compare(const uint32_t *crc, const uint32_t *expected, const uint8_t *pre, uint64_t n,
                                 uint8_t *verdict, hipStream_t s) {
  hipLaunchKernelGGL(frames_compare_kernel, grid_for(n), dim3(256), 0, s, crc, expected, pre, n, verdict);
  return hipGetLastError();
}

hipError_t launch_frames_stamp_prep(uint64_t stream_bytes, const uint64_t *frame_off, const uint32_t *body_len,
                                    uint64_t n, int flags, uint64_t *body_off, uint32_t *len_eff, uint8_t *pre,
                                    hipStream_t s) {
  hipLaunchKernelGGL(frames_stamp_prep_kernel, grid_for(n), dim3(256), 0, s, stream_bytes, frame_off, body_len, n,
                     flags, body_off, len_eff, pre);
  return hipGetLastError();
}

hipError_t launch_frames_stamp(uint8_t *stream, const uint64_t *frame_off, const uint32_t *body_len,
                               const uint32_t *crc, const uint8_t *pre, uint64_t n, uint16_t version, uint16_t type,
                               hipStream_t s) {
  hipLaunchKernelGGL(frames_stamp_kernel, grid_for(n), dim3(256), 0, s, stream, frame_off, body_len, crc, pre, n,
                     version, type);
  return hipGetLastError();
}

} // namespace rpccrc
