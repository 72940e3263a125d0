// rpc_amd/csrc/frames.hip -- batched frame verify / stamp helpers (SURVEY.md 8f
// rows 1 and 3).  Header parse and stamp are tiny byte kernels; the body CRCs
// come from the same ragged path as every other batch (rows kernel, plus the
// chunk route for large bodies when the MAX_BODY_LEN cap is lifted).
#include "../../include/rpccrc.h"
#include "frames.h"

namespace rpccrc {

namespace {
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

// (the rule: frames.h frames_parse_one)
__global__ void frames_parse_kernel(FramesParse p, uint64_t n) {
  const uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i < n) frames_parse_one(p, i);
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
  FramesParse p;
  p.stream = stream;
  p.stream_bytes = stream_bytes;
  p.frame_off = frame_off;
  p.flags = flags;
  p.body_off = body_off;
  p.body_len = body_len;
  p.hdr_crc = hdr_crc;
  p.pre = pre;
  hipLaunchKernelGGL(frames_parse_kernel, grid_for(n), dim3(256), 0, s, p, n);
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
