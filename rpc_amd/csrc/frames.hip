// rpc_amd/csrc/frames.hip -- batched frame verify / stamp helpers (SURVEY.md 8f
// row 1).  Header parse and stamp are tiny byte kernels; the body CRCs come from
// the same items kernel as every other path.
#include "frames.h"

namespace rpccrc {

namespace {
__device__ __forceinline__ uint32_t be32(const uint8_t *p) {
  return ((uint32_t)p[0] << 24) | ((uint32_t)p[1] << 16) | ((uint32_t)p[2] << 8) | (uint32_t)p[3];
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

__global__ void frames_parse_kernel(const uint8_t *stream, const uint64_t *frame_off, uint64_t n, uint64_t *body_off,
                                    uint32_t *body_len, uint32_t *hdr_crc) {
  const uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n) return;
  const uint8_t *h = stream + frame_off[i];
  body_off[i] = frame_off[i] + kFrameHeaderLen;
  body_len[i] = be32(h + 4); // rpc.h:6 body_len
  hdr_crc[i] = be32(h + 8);  // rpc.h:7 crc32
}

__global__ void frames_compare_kernel(const uint32_t *crc, const uint32_t *expected, uint64_t n, uint8_t *ok) {
  const uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i < n) ok[i] = crc[i] == expected[i] ? 1 : 0;
}

__global__ void frames_body_offsets_kernel(const uint64_t *frame_off, uint64_t n, uint64_t *body_off) {
  const uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i < n) body_off[i] = frame_off[i] + kFrameHeaderLen;
}

__global__ void frames_stamp_kernel(uint8_t *stream, const uint64_t *frame_off, const uint32_t *body_len,
                                    const uint32_t *crc, uint64_t n, uint16_t version, uint16_t type) {
  const uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n) return;
  uint8_t *h = stream + frame_off[i];
  put_be16(h + 0, version);
  put_be16(h + 2, type);
  put_be32(h + 4, body_len[i]);
  put_be32(h + 8, crc[i]);
}

dim3 grid_for(uint64_t n) { return dim3((unsigned)((n + 255) / 256)); }
} // namespace

hipError_t launch_frames_parse(const uint8_t *stream, const uint64_t *frame_off, uint64_t n, uint64_t *body_off,
                               uint32_t *body_len, uint32_t *hdr_crc, hipStream_t s) {
  hipLaunchKernelGGL(frames_parse_kernel, grid_for(n), dim3(256), 0, s, stream, frame_off, n, body_off, body_len,
                     hdr_crc);
  return hipGetLastError();
}

hipError_t launch_frames_compare(const uint32_t *crc, const uint32_t *expected, uint64_t n, uint8_t *ok,
                                 hipStream_t s) {
  hipLaunchKernelGGL(frames_compare_kernel, grid_for(n), dim3(256), 0, s, crc, expected, n, ok);
  return hipGetLastError();
}

hipError_t launch_frames_body_offsets(const uint64_t *frame_off, uint64_t n, uint64_t *body_off, hipStream_t s) {
  hipLaunchKernelGGL(frames_body_offsets_kernel, grid_for(n), dim3(256), 0, s, frame_off, n, body_off);
  return hipGetLastError();
}

hipError_t launch_frames_stamp(uint8_t *stream, const uint64_t *frame_off, const uint32_t *body_len,
                               const uint32_t *crc, uint64_t n, uint16_t version, uint16_t type, hipStream_t s) {
  hipLaunchKernelGGL(frames_stamp_kernel, grid_for(n), dim3(256), 0, s, stream, frame_off, body_len, crc, n, version,
                     type);
  return hipGetLastError();
}

} // namespace rpccrc
