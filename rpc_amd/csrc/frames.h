// rpc_amd/csrc/frames.h -- wire-frame helpers around the CRC items kernel.
// Frame = 12-byte packed big-endian rpc_header_t (reference rpc.h:3-8,15)
// followed by body_len bytes.
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

namespace rpccrc {

constexpr uint32_t kFrameHeaderLen = 12; // RPC_HEADER_LEN, rpc.h:15

// Reads each header (as rpc_server_main.c:165-169 does with ntohs/ntohl) and
// writes the body offset (frame offset + 12), body_len and header crc32.
hipError_t launch_frames_parse(const uint8_t *stream, const uint64_t *frame_off, uint64_t n, uint64_t *body_off,
                               uint32_t *body_len, uint32_t *hdr_crc, hipStream_t s);
// ok[i] = crc[i] == expected[i]
hipError_t launch_frames_compare(const uint32_t *crc, const uint32_t *expected, uint64_t n, uint8_t *ok,
                                 hipStream_t s);
hipError_t launch_frames_body_offsets(const uint64_t *frame_off, uint64_t n, uint64_t *body_off, hipStream_t s);
// Writes the header as rpc_async.c:521-530 does (htons/htonl + memcpy).
hipError_t launch_frames_stamp(uint8_t *stream, const uint64_t *frame_off, const uint32_t *body_len,
                               const uint32_t *crc, uint64_t n, uint16_t version, uint16_t type, hipStream_t s);

} // namespace rpccrc
