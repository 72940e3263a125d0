// rpc_amd/csrc/frames.hip -- batched frame verify / stamp helpers (SURVEY.md 8f
// rows 1 and 3).  Header parse and stamp are tiny byte kernels; the body CRCs
// come from the same ragged path as every other batch (rows kernel, plus the
// chunk route for large bodies when the MAX_BODY_LEN cap is lifted).
#include "../../include/rpccrc.h"
#include "frames.h"

namespace rpccrc {

namespace {
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

// Stamp side (the rules: frames.h frames_stamp_prep_one / frames_stamp_one).
__global__ void frames_stamp_prep_kernel(FramesStamp p, uint64_t n) {
  const uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i < n) frames_stamp_prep_one(p, i);
}
__global__ void frames_stamp_kernel(FramesStamp p, const uint32_t *crc, uint64_t n) {
  const uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i < n) frames_stamp_one(p, i, crc[i]);
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

hipError_t launch_frames_stamp_prep(const FramesStamp &p, uint64_t n, hipStream_t s) {
  hipLaunchKernelGGL(frames_stamp_prep_kernel, grid_for(n), dim3(256), 0, s, p, n);
  return hipGetLastError();
}

hipError_t launch_frames_stamp(const FramesStamp &p, const uint32_t *crc, uint64_t n, hipStream_t s) {
  hipLaunchKernelGGL(frames_stamp_kernel, grid_for(n), dim3(256), 0, s, p, crc, n);
  return hipGetLastError();
}

} // namespace rpccrc
