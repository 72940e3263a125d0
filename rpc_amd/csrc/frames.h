// rpc_amd/csrc/frames.h -- wire-frame helpers around the CRC kernels.
// Frame = 12-byte packed big-endian rpc_header_t (reference rpc.h:3-8,15)
// followed by body_len bytes.
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

namespace rpccrc {

constexpr uint32_t kFrameHeaderLen = 12; // RPC_HEADER_LEN, rpc.h:15
constexpr uint8_t kFramePending = 0xFF;  // data frame whose body CRC decides

// Reads each header (as rpc_server_main.c:165-169 does with ntohs/ntohl) and
// applies the reference's type / cap / bounds rules (frames.hip): the body
// offset and effective length (0 when the body is not read), the header crc32
// and the verdict so far (RPC_FRAME_* or kFramePending).
hipError_t launch_frames_parse(const uint8_t *stream, uint64_t stream_bytes, const uint64_t *frame_off, uint64_t n,
                               int flags, uint64_t *body_off, uint32_t *body_len, uint32_t *hdr_crc, uint8_t *pre,
                               hipStream_t s);
// verdict[i] = pre[i], or for pending data frames OK / BAD_CRC by crc == expected.
hipError_t launch_frames_compare(const uint32_t *crc, const uint32_t *expected, const uint8_t *pre, uint64_t n,
                                 uint8_t *verdict, hipStream_t s);
// Stamp side: bounds + cap (rpc_async.c:499-501) -> body offset, effective length, OK / TOO_LARGE / MALFORMED.
hipError_t launch_frames_stamp_prep(uint64_t stream_bytes, const uint64_t *frame_off, const uint32_t *body_len,
                                    uint64_t n, int flags, uint64_t *body_off, uint32_t *len_eff, uint8_t *pre,
                                    hipStream_t s);
// Writes the header of every OK frame as rpc_async.c:521-530 does (htons/htonl + memcpy).
hipError_t launch_frames_stamp(uint8_t *stream, const uint64_t *frame_off, const uint32_t *body_len,
                               const uint32_t *crc, const uint8_t *pre, uint64_t n, uint16_t version, uint16_t type,
                               hipStream_t s);

} // namespace rpccrc
