/*
 * include/rpccrc.h -- C-ABI of librpccrc, the MI355X-native body-checksum
 * library that replaces KlinLike/RPC's crc.c.
 *
 * Drop-in part (exact reference signatures, C linkage, no new types):
 *   rpc_crc32         replaces reference crc.c:4-9   (declared crc.h:8)
 *   rpc_crc32_verify  replaces reference crc.c:11-14 (declared crc.h:11)
 * Callers that keep working unchanged: client/rpc_async.c:219,525 and
 * server/rpc_server_main.c:227,249 (and the unbuilt client/rpc_client.c:60,154).
 * Link librpccrc.so in place of crc.c (CMakeLists.txt:14,25).  The library
 * does NOT define zlib's global `crc32`, so it never interposes on -lz.
 *
 * Additive part (SURVEY.md 8b "New (additive) batched ABI"): many-buffer CRC
 * over host or device (HBM-resident) buffers, computed by hand-written HIP
 * kernels for gfx950.  Plain pointers and sizes only; the caller owns every
 * buffer.  `stream` arguments are hipStream_t passed as void* (NULL = the
 * default stream of the calling thread's current HIP device).
 *
 * Semantics are bit-exact to zlib crc32 as called by crc.c:6-7:
 *   CRC-32/ISO-HDLC, poly 0xEDB88320 (reflected), init/xorout 0xFFFFFFFF;
 *   rpc_crc32(NULL, n) == 0; rpc_crc32(p, 0) == 0;
 *   len is reduced modulo 2^32 (zlib's uInt len, crc.c:7 passes size_t).
 *
 * Error convention for the int-returning batched calls: 0 (or a non-negative
 * count where stated) on success, a negative errno-style code on failure
 * (RPCCRC_E*).  The two drop-in calls have no error channel in the reference
 * (crc.h:8,11); if no HIP device is usable they print a diagnostic to stderr and
 * abort() -- they never fall back to a CPU implementation.
 */
#pragma once

#include <stdbool.h>
#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

#if defined(__GNUC__)
#define RPCCRC_API __attribute__((visibility("default")))
#else
#define RPCCRC_API
#endif

#define RPCCRC_OK 0
#define RPCCRC_EINVAL (-22) /* bad argument (NULL buffer with n>0, bad size, ...) */
#define RPCCRC_ENODEV (-19) /* no usable HIP device */
#define RPCCRC_ENOMEM (-12) /* device or pinned allocation failed */
#define RPCCRC_EIO (-5)     /* HIP runtime / kernel launch error, or a kernel-reported
                               error (rpc_crc32_device_status) */
#define RPCCRC_EAGAIN (-11) /* receive ring: no free segment yet, poll first */

/* ---- drop-in (reference crc.h) ---------------------------------------- */

/* reference crc.h:8 / crc.c:4-9.  CRC of `len` bytes at `data`. */
RPCCRC_API uint32_t rpc_crc32(const void *data, size_t len);

/* reference crc.h:11 / crc.c:11-14.  expected_crc in host byte order. */
RPCCRC_API bool rpc_crc32_verify(const void *data, size_t len, uint32_t expected_crc);

/* ---- batched, host buffers -------------------------------------------- */

/* out_crc[i] = rpc_crc32(base + offsets[i], lengths[i]) for i < n.  Buffers are
 * host memory (pinned memory is used in place; pageable memory is staged).
 * flags must be 0.  Returns RPCCRC_OK or a negative code. */
RPCCRC_API int rpc_crc32_batch(const uint8_t *base, const uint64_t *offsets, const uint32_t *lengths, size_t n,
                    uint32_t *out_crc, int flags);

/* Batched rpc_crc32_verify: ok[i] = (crc == expected[i]).  Returns the number
 * of mismatching bodies (>= 0) or a negative code. */
RPCCRC_API int64_t rpc_crc32_verify_batch(const uint8_t *base, const uint64_t *offsets, const uint32_t *lengths,
                               const uint32_t *expected, size_t n, uint8_t *ok);

/* ---- batched, device (HBM-resident) buffers ---------------------------- */

/* Ragged batch: body i = d_base[d_offsets[i] .. + d_lengths[i]).  All pointers
 * are device pointers on the current device.  Asynchronous on `stream`.
 * Bodies of >= 256 KiB (>= 16 KiB in batches of <= 16384 bodies) are cut into
 * chunks on the device and folded with the GF(2) combine, so one long body does
 * not serialise the batch on one wave.  A batch of >= 65536 bodies that lie back
 * to back in batch order (each 64 B - 1 MiB; decided on the device) is CRC'd as
 * one stream of 4 KiB blocks and folded per body (dense span mode, DESIGN.md 4.9;
 * RPCCRC_DENSE=0 turns it off).  Same results either way. */
RPCCRC_API int rpc_crc32_device_batch(const uint8_t *d_base, const uint64_t *d_offsets, const uint32_t *d_lengths,
                           uint64_t n, uint32_t *d_out, void *stream);

/* rpc_crc32_device_batch with a length bound the caller knows (e.g. MAX_BODY_LEN,
 * rpc.h:17, or a workload's maximum): max_len >= every d_lengths[i], 0 = none.
 * With a bound below the big-body route threshold the route is never needed
 * and its passes are not launched.  The threshold depends on the batch size:
 * 16 KiB for n <= 16384 bodies, 256 KiB above (RPCCRC_BIG_MIN overrides both).
 * Results never depend on the hint: a body longer than a wrong bound is still
 * CRC'd exactly (by one wavefront, so slowly). */
RPCCRC_API int rpc_crc32_device_batch_bounded(const uint8_t *d_base, const uint64_t *d_offsets,
                                              const uint32_t *d_lengths, uint64_t n, uint32_t max_len,
                                              uint32_t *d_out, void *stream);

/* Equal-length batch: body i = d_base[i*stride .. + body_len). */
RPCCRC_API int rpc_crc32_device_uniform(const uint8_t *d_base, uint64_t n, uint32_t body_len, uint64_t stride,
                             uint32_t *d_out, void *stream);

/* Large bodies (any size): body i = d_base[h_offsets[i] .. + h_lengths[i]),
 * offsets/lengths in HOST memory.  Each body is split into chunk_bytes chunks
 * (multiple of 16; 0 = default: 16 KiB, or 8/4 KiB when that divides every
 * length of back-to-back bodies) processed in parallel and merged with the
 * GF(2) combine (zlib crc32_combine semantics).  Back-to-back bodies whose
 * lengths are chunk multiples run as one uniform batch.  Stream-ordered; the
 * call returns once the work is enqueued. */
RPCCRC_API int rpc_crc32_device_large(const uint8_t *d_base, const uint64_t *h_offsets, const uint64_t *h_lengths,
                           uint64_t n, uint32_t *d_out, uint64_t chunk_bytes, void *stream);

/* ---- frames (rpc.h:3-8 wire format) ------------------------------------ */

/* Reference wire constants (rpc.h:11-18). */
#define RPC_HEADER_LEN_BYTES 12u /* RPC_HEADER_LEN, rpc.h:15 */
#define RPC_MAX_BODY_LEN 1024u   /* MAX_BODY_LEN, rpc.h:17 */
#define RPC_FRAME_TYPE_DATA 0u   /* RPC_TYPE_DATA, rpc.h:11 */
#define RPC_FRAME_TYPE_PING 1u   /* RPC_TYPE_PING, rpc.h:12 */
#define RPC_FRAME_TYPE_PONG 2u   /* RPC_TYPE_PONG, rpc.h:13 */

/* Per-frame verdict (one byte per frame), in the order the reference decides:
 * type first, then the body-length cap, then the CRC. */
#define RPC_FRAME_BAD_CRC 0u   /* data frame, body CRC != header crc32: the server
                                  closes the connection (rpc_server_main.c:227-233),
                                  the client reports RPC_CRC_ERR (rpc_async.c:219-222) */
#define RPC_FRAME_OK 1u        /* data frame, body CRC == header crc32 */
#define RPC_FRAME_CONTROL 2u   /* heartbeat answered from the header alone, whatever
                                  its crc32 / body_len fields hold: PING at the server
                                  (rpc_server_main.c:172-187), PONG at the client
                                  (rpc_async.c:303-309); no body is read */
#define RPC_FRAME_TOO_LARGE 3u /* body_len > MAX_BODY_LEN with the cap in force: the
                                  peer is dropped before its body is read
                                  (rpc_server_main.c:189-195, rpc_async.c:312) */
#define RPC_FRAME_MALFORMED 4u /* header or body extends past the stream: not read */
#define RPC_FRAME_RECV_ERR 5u  /* client role only: a non-PONG frame with body_len 0.
                                  The reference client's BODY state calls
                                  recv(fd, buf, 0) on its non-blocking socket; once
                                  any further byte (or the peer's FIN) is pending that
                                  returns 0, taken for a closed peer
                                  (rpc_async.c:330-349): the connection is dropped and
                                  the call ends with RPC_RECV_ERR (rpc_types.h:26,
                                  rpc_async.c:377-386).  (On an idle socket recv
                                  returns EAGAIN and the client waits until more
                                  arrives, or the call times out.)  The empty body is
                                  never verified (rpc_async.c:219 is not reached).
                                  The server reads an empty body and verifies it
                                  (rpc_server_main.c:198-227), so a server-role frame
                                  with body_len 0 is OK / BAD_CRC by its crc32 field. */

/* Frame-call flags.  The role picks which heartbeat type is a control frame
 * (the other one is an ordinary data frame, as in the reference). */
#define RPC_FRAMES_SERVER 0x1   /* PING is control (rpc_server_main.c:172) */
#define RPC_FRAMES_CLIENT 0x2   /* PONG is control (rpc_async.c:303) */
#define RPC_FRAMES_LIFT_CAP 0x4 /* no MAX_BODY_LEN cap; bodies of any
                                   size, the large ones chunked + GF(2)-combined */

/* Verify n frames of a device stream of stream_bytes bytes.  Frame i starts at
 * d_stream + d_frame_offsets[i] with a 12-byte big-endian rpc_header_t {u16
 * version, u16 type, u32 body_len, u32 crc32} (rpc.h:3-8, parsed as
 * rpc_server_main.c:165-169) followed by body_len body bytes.  Writes
 * d_verdict[i] (RPC_FRAME_*) and, if d_crc is not NULL, the body CRC (0 for
 * frames whose body is not read).  Nothing outside [d_stream, d_stream +
 * stream_bytes) is read.  flags: exactly one role bit, optionally LIFT_CAP. */
RPCCRC_API int rpc_frames_verify_device(const uint8_t *d_stream, uint64_t stream_bytes, const uint64_t *d_frame_offsets,
                             uint64_t n, int flags, uint8_t *d_verdict, uint32_t *d_crc, void *stream);

/* Stamp headers: for each frame i whose body d_stream[d_frame_offsets[i] + 12
 * .. + d_body_lens[i]) lies inside the stream, write its 12-byte header
 * (version, type, body_len, crc32 big-endian, as rpc_async.c:521-530).
 * Without RPC_FRAMES_LIFT_CAP a body over MAX_BODY_LEN is not stamped (the
 * reference client refuses to send it, rpc_async.c:499-501).  d_verdict
 * (optional): RPC_FRAME_OK (stamped), _TOO_LARGE or _MALFORMED.  Role bits are
 * ignored. */
RPCCRC_API int rpc_frames_stamp_device(uint8_t *d_stream, uint64_t stream_bytes, const uint64_t *d_frame_offsets,
                            const uint32_t *d_body_lens, uint64_t n, uint16_t version, uint16_t type, int flags,
                            uint8_t *d_verdict, void *stream);

/* ---- batched server receive ring -------------------
 * Replaces the one-frame-at-a-time verify of the reference server loop
 * (server/rpc_server_main.c:135-238, verify at :227) for a receive loop that
 * batches: frames from any connections are landed straight into pinned host
 * segments (recv() into the pointer rpc_rx_ring_reserve returns, then
 * rpc_rx_ring_commit), a full segment -- or one flushed by rpc_rx_ring_submit
 * -- is verified on the GPU (one H2D copy, rpc_frames_verify_device, one D2H
 * copy of the verdicts) while the next one fills, and rpc_rx_ring_poll returns
 * the verdicts in arrival order with the caller's tag.  A ring is used by one
 * thread; it works on the HIP device current at creation. */
typedef struct rpc_rx_ring rpc_rx_ring_t;

typedef struct {
  uint64_t tag;         /* the caller's tag from rpc_rx_ring_commit / _push */
  const uint8_t *frame; /* the frame (12-byte header + body) in the ring's pinned
                           memory; valid until the next rpc_rx_ring_poll */
  uint32_t body_len;    /* header fields, host order (rpc.h:3-8) */
  uint16_t version;
  uint16_t type;
  uint32_t header_crc;  /* the crc32 the sender stamped */
  uint32_t crc;         /* rpc_crc32 of the body, computed on the GPU (0 if not read) */
  uint8_t ok;           /* verdict is RPC_FRAME_OK or RPC_FRAME_CONTROL */
  uint8_t verdict;      /* RPC_FRAME_* */
} rpc_rx_frame_t;

/* nsegments (2..64) segments of segment_bytes bytes and max_frames frames each;
 * flags as rpc_frames_verify_device (one role bit, optionally LIFT_CAP). */
RPCCRC_API int rpc_rx_ring_create(rpc_rx_ring_t **ring, size_t segment_bytes, size_t max_frames, int nsegments,
                                  int flags);
RPCCRC_API void rpc_rx_ring_destroy(rpc_rx_ring_t *ring);
/* *dst = where to land a frame of frame_len bytes (header + body).  A segment
 * that cannot take it is submitted first; RPCCRC_EAGAIN when every segment is
 * still in flight or unpolled (call rpc_rx_ring_poll). */
RPCCRC_API int rpc_rx_ring_reserve(rpc_rx_ring_t *ring, size_t frame_len, uint8_t **dst);
/* Accepts the reserved frame; RPCCRC_EINVAL (frame dropped) unless the landed
 * length is exactly what the reference reads for that header: 12 + body_len for
 * a data frame, the 12-byte header alone for a control frame or a data frame over
 * the cap (the reference reads no body for either, rpc_server_main.c:172-195,
 * rpc_async.c:303-315; the bytes after such a header belong to the next frame). */
RPCCRC_API int rpc_rx_ring_commit(rpc_rx_ring_t *ring, uint64_t tag);
/* reserve + memcpy + commit. */
RPCCRC_API int rpc_rx_ring_push(rpc_rx_ring_t *ring, const void *frame, size_t frame_len, uint64_t tag);
/* Sends the partly filled segment to the GPU now (e.g. when the socket loop idles). */
RPCCRC_API int rpc_rx_ring_submit(rpc_rx_ring_t *ring);
/* Up to max_frames verdicts of the oldest submitted segment, in arrival order;
 * returns their count (0 if none is ready and wait == 0) or a negative code. */
RPCCRC_API int64_t rpc_rx_ring_poll(rpc_rx_ring_t *ring, rpc_rx_frame_t *out, size_t max_frames, int wait);

/* ---- helpers ----------------------------------------------------------- */

/* zlib crc32_combine (zlib.h:1750): crc(A||B) from crc(A), crc(B), |B|. */
RPCCRC_API uint32_t rpc_crc32_combine(uint32_t crc1, uint32_t crc2, uint64_t len2);

/* Fill d_dst with the counter-based splitmix64 stream used by tests/bench
 * (word k = mix64(seed + (k+1)*0x9E3779B97F4A7C15), little-endian).
 * nbytes must be a multiple of 8. */
RPCCRC_API int rpc_crc32_fill_random_device(void *d_dst, uint64_t nbytes, uint64_t seed, void *stream);

/* HBM read probe over nbytes (multiple of 4096): pattern 0 = coalesced 16-B
 * lanes, 1 = the CRC kernel's 64-B-per-lane segments (both a plain grid-stride
 * loop), 2 = the rows kernel itself with its CRC work compiled out: the same
 * dealing (workgroup rounds + tail stealing), loads (4 x 16 B non-temporal per
 * lane, a row ahead) and launch shape, i.e. the ceiling of the product's memory
 * stream (nbytes >= 256 MiB on 256 CUs; `nontemporal` is ignored). */
RPCCRC_API int rpc_crc32_stream_read_device(const void *d_src, uint64_t nbytes, int pattern, int nontemporal, void *stream);

/* Tuning knobs (process-wide): nontemporal loads (0/1, default 1) and the
 * persistent-grid size cap in workgroups (0 = one per CU). */
RPCCRC_API int rpc_crc32_set_options(int nontemporal, int max_blocks);

/* Kernel for ragged device batches (process-wide; used by rpc_crc32_device_batch,
 * rpc_crc32_batch and the frames calls).  Results are identical either way.
 *   RPCCRC_RAGGED_AUTO   frames calls (bodies <= MAX_BODY_LEN): split;
 *                        other batches: rows (default)
 *   RPCCRC_RAGGED_ROWS   one wavefront per body, 4 KiB rows
 *   RPCCRC_RAGGED_PACKED 1 KiB chunks of consecutive bodies packed four per
 *                        row, balanced by chunk count
 *   RPCCRC_RAGGED_SPLIT  bodies of <= 1 KiB (with their 16-B end pad) four per
 *                        row, the rest one wavefront per body
 * Returns RPCCRC_EINVAL for any other value. */
#define RPCCRC_RAGGED_AUTO 0
#define RPCCRC_RAGGED_ROWS 1
#define RPCCRC_RAGGED_PACKED 2
#define RPCCRC_RAGGED_SPLIT 3
RPCCRC_API int rpc_crc32_set_ragged_path(int path);

/* Human-readable text for a negative return code. */
RPCCRC_API const char *rpc_crc32_strerror(int err);

/* Writes "device=<name> arch=<gcn> cus=<n>" for the current device. */
RPCCRC_API int rpc_crc32_device_info(char *buf, size_t buflen);

/* Device error status of the current device: RPCCRC_OK, or RPCCRC_EIO once a
 * kernel launched by an ASYNCHRONOUS call (device batches, large bodies, frames,
 * the receive ring) has stored into the device's error word -- a bounded wait of
 * the rows kernel's dealing protocol ran out (after 30 s), so CRCs of that launch
 * may be stale.  While it is set, every asynchronous call on the device returns
 * RPCCRC_EIO.  Device calls are asynchronous: check after synchronising the
 * stream.  The synchronous calls (rpc_crc32, rpc_crc32_verify, rpc_crc32_batch,
 * rpc_crc32_verify_batch) report their own launches' errors in their own return
 * (the drop-in calls abort) and are neither affected by nor recorded in it. */
RPCCRC_API int rpc_crc32_device_status(void);

/* Clears the current device's error word so asynchronous calls work again, and
 * returns what rpc_crc32_device_status returned before (RPCCRC_OK or
 * RPCCRC_EIO).  Call it after synchronising every stream whose results are in
 * doubt: outputs of the launch that failed are not repaired. */
RPCCRC_API int rpc_crc32_device_clear_status(void);

/* Stops the resident drop-in service kernel (the one that answers rpc_crc32 /
 * rpc_crc32_verify calls of <= 1 KiB without a launch) on every
 * device this process has used, and waits (up to 200 ms each) until it has left.
 * A device-wide synchronise (hipDeviceSynchronize, torch.cuda.synchronize())
 * otherwise waits for the service: up to ~2 ms after the last drop-in call
 * (INTEGRATION.md 5).  The next drop-in call starts it again.  Call it with no
 * drop-in call in flight: one racing it waits for its answer (up to 2 s) and then
 * launches a kernel instead.  Returns RPCCRC_OK, or RPCCRC_EIO if an instance did
 * not leave in time (it was still queued behind other work; it then runs and
 * serves calls as usual).  Not part of crc.h; the reference has no counterpart. */
RPCCRC_API int rpc_crc32_service_stop(void);

/* Counters of the drop-in service, summed over every device this process has
 * used (no device needed; all zero before the first drop-in call).  A request
 * that gets no answer in 2 s is given up and the call launches a kernel
 * instead; after that, while the device's latest service instance has not
 * started (queued behind other kernels), drop-in calls launch a kernel without
 * posting (`bypassed`), and posted calls wait 2 ms, not 2 s (`fallbacks_short`),
 * until one is answered again.  Not part of crc.h. */
typedef struct rpccrc_service_stats {
  uint64_t services;        /* devices with a drop-in service */
  uint64_t running;         /* of them, with an instance running or queued */
  uint64_t launched;        /* instances launched */
  uint64_t answered;        /* drop-in calls the service answered */
  uint64_t fallbacks_full;  /* requests given up after the full 2-s wait */
  uint64_t fallbacks_short; /* requests given up after the 2-ms wait that follows a give-up */
  uint64_t bypassed;        /* calls that did not post (instance not started after a give-up) */
} rpccrc_service_stats_t;
RPCCRC_API int rpc_crc32_service_stats(rpccrc_service_stats_t *out);

#ifdef __cplusplus
}
#endif
