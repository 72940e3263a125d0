// rpc_amd/csrc/crc32_kernels.h -- internal (C++) interface between the C-ABI
// host layer (rpccrc_api.cpp) and the HIP kernels (crc32_kernels.hip).
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

#include "crc32_layout.h"
#include "frames.h"

namespace rpccrc {

// Output modes of the items kernel.
constexpr uint32_t kModeFinal = 0; // crc(M) = ~U(F, M)           (rpc_crc32 value)
constexpr uint32_t kModeRaw = 1;   // crc0(M)                      (chunk partials)
constexpr uint32_t kModeInit = 2;  // U(F, M), no final complement (diagnostic)

struct ItemsArgs {
  const uint8_t *base;      // device (or host-mapped) byte buffer
  const uint64_t *offsets;  // nullptr -> item i at i * stride
  const uint32_t *lengths;  // nullptr -> every item has length len
  uint64_t n_items;
  uint64_t stride;
  uint32_t len;
  uint32_t mode;
  const uint4 *lds_image;   // LDS table image (v2 layout, kLdsBytesV2 bytes)
  const uint32_t *tq;       // Tq[q] = A_q(0xFFFFFFFF), q = 0..4096
  uint32_t *out;            // n_items CRCs
  uint32_t gshift;          // group dealing: each wave takes 2^gshift consecutive tasks per round
  // Split ragged batches (launch_split_batch): the item count is read on the
  // device (n_items is then only the upper bound the grid is sized for) and
  // item i's CRC goes to out[out_idx[i]].
  const uint64_t *n_dev = nullptr;
  const uint32_t *out_idx = nullptr;
  // Big-body route (QB = 1 ragged only): a body with length >= big_min whose
  // bit is set in `routed` (indexed by its batch index, out_idx[i] or i) is
  // taken as empty here; launch_big_route computes its CRC afterwards.
  const uint32_t *routed = nullptr;
  uint32_t big_min = 0xFFFFFFFFu;
  // Tail stealing (QB = 1, DYN launches of host-counted batches): a leased
  // two-word device counter, zero at launch and reset to zero by the launch's
  // last workgroup (crc32_rows.h kStealAhead).  nullptr: static rounds only.
  // steal_s is set by launch_rows.
  uint32_t *steal = nullptr;
  uint32_t steal_s = 0;         // kStealOnDevice: the kernel sizes the pool from the device count
  uint32_t steal_permille = 80;  // pool share of the rounds (steal_s on the device)
  uint32_t steal_max_wg = 48;     // ... at most this many pool rounds per workgroup
  // Words zeroed by workgroup 0 at launch (<= 1024; the contiguous chunk
  // combine XORs into them afterwards).
  uint32_t *zero_out = nullptr;
  uint32_t zero_n = 0;
  // Round values (uniform QB = 1 DYN launches of 4096-byte RAW items whose
  // lds_image carries the round maps, crc32_rows.h kRowsRoundOut): crc0 of
  // round r's 32 items at round_out[r].  launch_rows refuses it otherwise.
  uint32_t *round_out = nullptr;
  // Device error word of the launch's device (pinned host memory, zero while
  // all is well).  A wave whose bounded wait in the DYN / tail-stealing
  // protocol runs out stores kErr* into it (crc32_rows.h); the host turns a
  // non-zero word into RPCCRC_EIO (sticky per device, rpc_crc32_device_status).
  uint32_t *err = nullptr;
  // Test-only (RPCCRC_TEST_STEAL_GIVEUP=1 in the environment): every pool-round
  // wait gives up at once, so the error path can be exercised deliberately.
  uint32_t test_giveup = 0;
  // Dense span mode (crc32_rows.h kRowsSpanBnd): the span pass
  // reads its stream base and length from span_ctl (the plan's output), each
  // block's boundary record from span_rec, and stores per-boundary values into
  // span_bnd.  nullptr: not a span pass.
  const struct DenseCtl *span_ctl = nullptr;
  const uint4 *span_rec = nullptr;
  const uint16_t *span_bpos = nullptr;
  uint2 *span_bnd = nullptr;
  // Non-zero *skip_dev: the launch exits at once (the ragged rows pass of a
  // batch the dense plan took; decided on the device).
  const uint32_t *skip_dev = nullptr;
};

// ---- dense span mode -----------------------------------------
// A ragged device batch whose bodies lie back to back in order, each of
// kDenseMinBody .. kDenseMaxBody bytes (C2's layout), is CRC'd as ONE uniform
// stream of 4 KiB blocks (the north star's kernel and rate) plus per-boundary
// values, then folded per body -- instead of one wave walking each body's own
// end-aligned rows (C2: 12.47M row steps against 9.66M blocks).  Decided on the
// device by dense_plan_kernel; a batch that is not dense runs the rows pass.
constexpr uint32_t kDenseMinBody = 64;          // at most one boundary per 64-B segment of a block
constexpr uint32_t kDenseMaxBody = 1u << 20;    // the fold's thread-per-body Horner (<= 257 blocks)
constexpr uint64_t kDenseMinN = 1u << 16;       // smaller batches stay on the rows path
constexpr uint64_t kDenseMaxN = (1u << 25) - 2; // boundary indices fit 25 bits of a block record
constexpr uint64_t kDenseMaxBlocks = 1ull << 24; // 64 GiB of stream per call
constexpr uint32_t kDenseInline = 6;            // boundary offsets carried in a block record
// Plan output (device).  nblocks = 0: the batch is not dense (the rows pass
// runs; the span and fold passes exit at once).
struct DenseCtl {
  uint64_t anchor;  // stream base: the first body's address rounded down to 16 B
  uint64_t bytes;   // anchor .. the last body's end
  uint64_t nblocks; // 4 KiB blocks of the stream (the span pass's device count)
  uint32_t skip;    // 1 when dense: the rows pass exits at once
  uint32_t pad;
};
// Block record (every block of the stream): x = first boundary index in the
// block | count << 25; y, z, w = the block offsets (12 bits, as u16) of its
// first kDenseInline boundaries.
// Boundary g (body g's start; g = n: the last body's end) at stream offset
// rel_g: bpos[g] = rel_g & 4095.  Span pass output per boundary:
// bnd[g] = {P1 ^ A_{64(15-lo)}(A_{4(16-tb)}(cap)), Qp} (tests/test_dense_emu.py
// names them): crc0 of the boundary's quarter up to it, shifted to the quarter's
// end, and the quarters before it shifted to the block's end.
struct DenseArgs {
  const uint8_t *base;
  const uint64_t *offsets;
  const uint32_t *lengths;
  uint64_t n;
  uint64_t nb_cap;    // records / W words in the workspace
  DenseCtl *ctl;
  uint4 *rec;         // nb_cap
  uint16_t *bpos;     // n + 1
  uint2 *bnd;         // n + 1
  uint32_t *W;        // nb_cap: crc0 of each block (the span pass's out)
  uint32_t *flags;    // dense_plan_blocks(n): the plan's per-workgroup "not dense" flags
  uint32_t *out;      // n CRCs
  const uint32_t *tq; // Tq[q] = A_q(0xFFFFFFFF)
  const uint32_t *tab; // kDenseTabWords: the fold's maps (crc32_layout.h)
};
size_t dense_workspace_bytes(uint64_t n, uint64_t nb_cap);
DenseArgs dense_carve(void *ws, uint64_t n, uint64_t nb_cap);
inline uint64_t dense_plan_blocks(uint64_t n) { return (n + 1 + 255) / 256; } // 4 waves of 64 boundaries each
// The plan (dense_plan_kernel) and the decision (dense_decide_kernel: DenseCtl).
hipError_t launch_dense_plan(const DenseArgs &d, hipStream_t s);
hipError_t launch_dense_fold(const DenseArgs &d, int cus, hipStream_t s);

constexpr uint32_t kStealOnDevice = 0xFFFFFFFFu; // ItemsArgs.steal_s: computed in the kernel (device-counted n)

// Device error bits (ItemsArgs.err).
constexpr uint32_t kErrStealWait = 1u; // a wave gave up waiting for a stolen round: its tasks were not run
constexpr uint32_t kErrRingWait = 2u;  // a wave gave up waiting for an output-ring slot: CRCs may be stale

// ---- big bodies of a ragged batch ----------------------------
// One wave per body would leave a long body streaming through a single wave
// while the rest of the chip idles.  Bodies of >= kBigMin bytes (up to
// kBigMaxBodies per batch; any further ones keep one wave each) are cut into
// chunks on the device, CRC'd by the rows kernel (RAW) and folded per body.
constexpr uint32_t kBigMin = 256u << 10;
constexpr uint32_t kBigMaxBodies = 16384;
constexpr uint64_t kBigMaxChunks = 1ull << 20;
// Default first chunk size: two-row chunks (8176 B: with the body's end pad
// z <= 15 a chunk still fits two 4 KiB rows), dealt with tail stealing.
// 1024 lifted-cap frames of 1 B - 64 MiB (bench extra.frames_lifted), verify
// per call on one box: 4080 B 622-634 us, 8176 B 590-596 us, 16368 B 602-609 us
// (profiles/r03d/frames_chunks.txt); 16 KiB chunks until round 3.
// The plan grows it as (chunk + 16) * 2 - 16 until the chunks fit kBigMaxChunks.
constexpr uint64_t kBigMinChunk = 8192 - 16;       // end-aligned chunks (BigRoute.aligned = false)
constexpr uint64_t kBigMinChunkAligned = 8192;     // address-aligned chunks (the default)
struct BigRoute {
  uint32_t *routed;  // bit i: body i takes the route (ceil(n / 64) * 2 words, all written)
  uint64_t *meta;    // [0] bodies claimed, [1] their bytes, [2] chunks, [3] chunk bytes,
                     // [4] span rows, [5] span mode on (route-all span mode, below)
  uint32_t *b_idx;   // kBigMaxBodies: batch index of each routed body
  uint64_t *b_first; // kBigMaxBodies + 1: first chunk of each routed body
  uint64_t *c_off;   // kBigMaxChunks: chunk offsets / lengths / crc0
  uint32_t *c_len;
  uint32_t *c_raw;
  uint64_t min_chunk = kBigMinChunk; // the plan's starting chunk size (aligned: a power of two; else 2^k 4096 - 16)
  // Address-aligned chunks (round 4): a body's pieces between multiples of the
  // power-of-two chunk (interior chunks: whole aligned blocks, aligned rows).
  // false: end-aligned chunks of 2^k * 4096 - 16 bytes (rounds 2-3).
  bool aligned = true;
  // Route-all mode (all_n > 0): every body of a batch of all_n <= kBigMaxBodies
  // takes the route, body b = batch index b (no classify pass, no b_idx list,
  // no plain rows pass); the plan sums the lengths itself.
  uint32_t all_n = 0;
  // Dense span mode beside the route: non-zero *skip (the dense
  // plan's DenseCtl::skip) makes the classify pass route no body, so the route's
  // later passes find nothing to do.  nullptr: no dense plan.
  const uint32_t *skip = nullptr;
  const uint32_t *tq = nullptr;  // Tq[q] = A_q(0xFFFFFFFF): the combine seeds chunk 0 with it
  // Span mode (route-all only; span_rows_max > 0, the batch base 4 KiB-aligned):
  // when the plan finds the bodies dense in [base, base + 4096 * span_rows_max)
  // (meta[5] = 1), the UNIFORM rows pass CRCs every whole 4 KiB block below the
  // last body end into blk[] (meta[4] blocks), the ragged chunk pass has no
  // chunks, and the fold takes a body's interior blocks from blk[] and CRCs its
  // first / last partial blocks itself.
  uint32_t *blk = nullptr;
  uint64_t span_rows_max = 0;
  const uint4 *tab4 = nullptr; // span mode: the slice-by-4 tables (scalar table image, first 4 KiB)
  // Span mode with round values (ItemsArgs.round_out): the span pass also stores
  // the crc0 of every whole 32-block round (128 KiB) at rnd[round], and the fold
  // takes a body's whole rounds from there.  rnd_image: the table image with the
  // round maps (kLdsRoundMaps).  Set by the host only when the span pass deals in
  // DYN rounds (span_rows_max >= 256 * max_blocks).
  uint32_t *rnd = nullptr;
  const uint4 *rnd_image = nullptr;
  // Frames verify in route-all mode: the fold also decides each frame's verdict
  // (frames_compare_kernel's rule: the parse's pre-verdict, else crc == the
  // header's crc32), so the compare launch is skipped.  nullptr: no verdicts.
  const uint32_t *cmp_expected = nullptr;
  const uint8_t *cmp_pre = nullptr;
  uint8_t *cmp_verdict = nullptr;
  // ... and the aligned plan parses the headers first (parse.frame_off set:
  // the batch's offsets / lengths are the parse's outputs), so the parse
  // launch is skipped too.
  FramesParse parse;
  // Frames stamp in route-all mode: the plan runs the stamp's bounds / cap
  // check (stamp.frame_off set), and the fold writes each OK frame's header.
  FramesStamp stamp;
  const uint32_t *dbl = nullptr; // kBigDblWords: the fold's doubling maps per chunk class (build_big_dbl)
};
// (The fold's doubling maps per chunk class: crc32_layout.h build_big_dbl.)
// span_rows: the span pass's block table (span mode, 0: off)
size_t big_route_workspace_bytes(uint64_t n, uint64_t span_rows = 0);
BigRoute big_route_carve(void *ws, uint64_t n, uint64_t span_rows = 0);
// Before the rows pass: flags and lists the big bodies (route.routed goes into
// the rows pass's ItemsArgs).  Stream-ordered, no host round trip.
// big_min: bodies of at least this many bytes are routed (kBigMin by default).
hipError_t launch_big_classify(const uint32_t *lengths, uint64_t n, uint32_t big_min, const BigRoute &r,
                               hipStream_t s);
// After the rows pass (route-all: instead of it): chunk plan, chunk CRCs (rows
// kernel, RAW), per-body fold into out[batch index].
// steal: a leased zeroed two-word counter for the chunk pass's tail stealing
// (nullptr: static rounds); its event is recorded as the chunk pass's
// completion (steal_done, *steal_recorded) like launch_rows.
// span: the span pass's steal counter and event (span mode only).
struct StealArgs {
  uint32_t *p = nullptr;
  hipEvent_t done = nullptr;
  bool *recorded = nullptr;
};
hipError_t launch_big_route(const ItemsArgs &proto, const BigRoute &r, const uint4 *shift_nib, bool nt, int max_blocks,
                            hipStream_t s, uint32_t *steal = nullptr, hipEvent_t steal_done = nullptr,
                            bool *steal_recorded = nullptr, StealArgs span = StealArgs());
// Most 4 KiB blocks of a span-mode route (16 GiB of stream per call).
constexpr uint64_t kSpanMaxRows = 1ull << 22;

constexpr uint32_t kShiftNibWords = 64u * 8u * 16u; // 32 KiB: the chunk combine's shift maps

// ---- drop-in scalar calls (crc32_scalar.hip) ------------------
// One wave CRCs one body of <= kScalarMaxLen bytes from pinned host staging
// (the body right-aligned at offset 64 * 2^scalar_seg_log2(len) - len) and
// stores {crc, seq} (crc in the low half) to pinned `result`.  Table image:
// crc32_layout.h (kScalarTabWords).
uint32_t scalar_seg_log2(uint32_t len);
hipError_t launch_scalar(const uint8_t *stage, uint32_t len, const uint4 *tab, const uint32_t *tq, uint64_t *result,
                         uint32_t seq, hipStream_t stream);

// ---- drop-in service (crc32_service.hip) ---------------------
// A resident one-workgroup kernel answers drop-in calls of <= kSvcMaxLen bytes
// through request slots in pinned, coherent host memory: no launch per call.
constexpr uint32_t kSvcWaves = 8;                      // waves of the service workgroup (2 per SIMD)
constexpr uint32_t kSvcPer = 2;                        // slots per wave: wave w owns slots w + 8 i
constexpr uint32_t kSvcSlots = kSvcWaves * kSvcPer;    // concurrent drop-in calls served
constexpr uint32_t kSvcMaxLen = 1024;                  // MAX_BODY_LEN (rpc.h:17)
constexpr uint32_t kSvcStop = 0, kSvcExited = 1, kSvcStarted = 2; // SvcShared::ctl words
constexpr uint32_t kSvcInline = 116;                   // bodies up to this length travel in the request block
// A slot's request block: two 64-B lines the service reads in ONE poll.
//   line 0: req = {len (low), seq (high)}, then inline bytes 0..55
//   line 1: inline bytes 56..115, then tag
// An inline body (len <= kSvcInline) ends at inline byte 116, so its CRC needs no
// second PCIe round trip; longer bodies go to SvcShared::body.  The host writes
// the bytes, then line 1's tag, then line 0's req word.
// Check (round 6, crc32_service_math.h word_hash): tag = XOR over the block's
// dwords 0..30 (len, seq, the 29 inline words) of word_hash(dword, position),
// XOR -- for a longer body -- the same sum over every masked word of the body's
// virtual buffer (svc::body_sum).  The service answers a request only when its
// own sum over what it read equals the tag it read: a poll or body read that
// combined stale and current words (its pieces arrive in an order the memory
// system chooses) fails with probability 1 - 2^-32 whatever the bodies, and is
// retried.  Rounds 4-5 summed the words with a plain XOR (and mixed only len and
// seq): two stale words with equal old -> new deltas cancelled, and requests over
// 116 B had no check at all.
struct SvcReq {
  uint64_t req;
  uint8_t inl[kSvcInline];
  uint32_t tag;
};
static_assert(sizeof(SvcReq) == 128, "two lines per request block");
static_assert(kSvcInline % 4 == 0 && kSvcInline / 4 == 29, "inline bytes as 29 whole words");
struct SvcShared {
  // one block per slot (a shared line was written by up to 8 caller threads
  // while 8 waves polled it: 10 callers took 30 us a call, r04c)
  SvcReq rq[kSvcSlots];
  uint64_t res[kSvcSlots][8];         // device: {crc, seq} (crc in the low half), one 64-B line per slot
  uint32_t ctl[16];                   // [kSvcStop] host: leave now; [kSvcExited] / [kSvcStarted] device: last instance that left / started
  uint8_t body[kSvcSlots][kSvcMaxLen]; // host: the body, right-aligned in 64 * seg bytes (seg 4 / 8 / 16)
};
// kshift: 3 x 64 words, kshift[c][L] = x^(8 * seg_c * (63 - L)) mod P for seg 4, 8, 16.
// The kernel leaves after idle_ticks (s_memrealtime, 100 MHz) without a
// request or after life_ticks in all; it stores `instance` into
// ctl[kSvcStarted] when it starts and into ctl[kSvcExited] when it leaves.
hipError_t launch_service(SvcShared *sh, const uint32_t *tq, const uint32_t *kshift, uint64_t idle_ticks,
                          uint64_t life_ticks, uint32_t instance, hipStream_t stream);

// A large body of rpc_crc32_device_large: bytes [off, off + len) of the base
// buffer, its end-aligned chunks at raw[chunk_first ...].
struct LargeBody {
  uint64_t off;
  uint64_t len;
  uint64_t chunk_first;
};
// Up to kInlineBodies bodies travel in the kernel arguments (no H2D copy).
constexpr uint64_t kInlineBodies = 32;
struct InlineBodies {
  LargeBody b[kInlineBodies];
};

struct CombineArgs {
  const uint32_t *raw;          // per-chunk crc0 values
  const uint64_t *lengths;      // body lengths (bytes); unused when inline
  const uint64_t *chunk_first;  // index into raw of each body's chunk 0; unused when inline
  const uint4 *shift_nib;       // NIB[k][i][j] = A_{2^k bytes}(j << 4i), k < 64, i < 8, j < 16
  uint64_t n_bodies;
  uint64_t chunk;               // chunk size in bytes (multiple of 16)
  uint32_t *out;                // splits > 1: zeroed before the launch, blocks XOR their partials in
  uint32_t splits = 1;          // blocks per body (each folds a contiguous run of chunks)
  // Equal bodies of 4096 * splits power-of-two chunks, 16-B aligned raw, out
  // zeroed by the rows pass: the contiguous-run kernel (4 chunks per thread).
  bool contig = false;
  bool inline_bodies = false;   // body table from `bodies` below (n_bodies <= kInlineBodies)
  InlineBodies bodies;
};

// Tasks per dealing round of the rows kernel's workgroup-dynamic dealing
// (crc32_rows.h DYN).
constexpr uint32_t kDynRound = 32;
// QB = 4 rounds may be shorter: a round of 16 four-body tasks is still 64
// whole CRCs (two 128-B lines), and the tail -- the last claimed round per
// workgroup -- is one task per wave instead of two.
#ifndef RPCCRC_DYN_ROUND_QB4
#define RPCCRC_DYN_ROUND_QB4 32
#endif
constexpr uint32_t dyn_round(int QB) { return QB == 4 ? (uint32_t)RPCCRC_DYN_ROUND_QB4 : kDynRound; }
static_assert(RPCCRC_DYN_ROUND_QB4 == 16 || RPCCRC_DYN_ROUND_QB4 == 32, "QB = 4 round: 16 or 32 tasks");

// Most items one rows-kernel launch takes (it indexes them in 32 bits);
// launch_rows splits larger host-counted batches.
constexpr uint64_t kMaxLaunchItems = 1ull << 30;

// QB = 1: rows of 4 KiB of one item (any length); QB = 4: four items per row,
// each with len + ((-(end address)) & 15) <= 1024.
// steal_done: the steal-counter slot's event.  A launch that deals from the
// counter (a.steal) records it as the kernel's own completion signal
// (hipExtLaunchKernel stopEvent: no marker packet between back-to-back
// launches) and sets *steal_recorded.
hipError_t launch_rows(const ItemsArgs &a, int QB, bool nt, int max_blocks, hipStream_t stream,
                       hipEvent_t steal_done = nullptr, bool *steal_recorded = nullptr);
// done: optional event recorded as the combine kernel's completion signal.
hipError_t launch_chunk_combine(const CombineArgs &a, hipStream_t stream, hipEvent_t done = nullptr);

// Packed ragged batches (crc32_packed.h): 1 KiB chunks of consecutive bodies,
// four per row, balanced by chunk count; n < 2^32 - 1.  ws must hold
// packed_workspace_bytes(n, max_slices) bytes of device memory, stream-ordered
// with the launch (count, scan, plan and CRC kernels all run on `stream`).
struct PackedBatch {
  const uint8_t *base;
  const uint64_t *offsets;
  const uint32_t *lengths;
  uint64_t n;
  uint32_t mode;
  const uint4 *lds_image;
  const uint32_t *tq;
  uint32_t *out;
  void *ws;
  size_t ws_bytes;
  uint64_t max_slices; // slice-table capacity (balance granularity)
  uint64_t min_slice;  // chunks per slice, at least
};
hipError_t packed_workspace_bytes(uint64_t n, uint64_t max_slices, size_t *bytes);
hipError_t launch_packed_batch(const PackedBatch &p, bool nt, int max_blocks, hipStream_t stream);
// Split ragged batches (crc32_kernels.hip): small bodies (len + end pad <= 1 KiB)
// through the QB = 4 rows kernel, the rest through QB = 1; n < 2^32 - 1.  proto
// carries the batch (offsets / lengths required); ws must hold
// split_workspace_bytes(n) bytes of device memory, stream-ordered with the launch.
struct SplitLists {
  uint64_t *counts; // [small, big]
  uint64_t *s_off, *b_off;
  uint32_t *s_len, *s_idx, *b_len, *b_idx;
};
hipError_t split_workspace_bytes(uint64_t n, size_t *bytes);
hipError_t launch_split_batch(const ItemsArgs &proto, void *ws, size_t ws_bytes, bool nt, int max_blocks,
                              hipStream_t stream);
// Small bodies only (len + end pad <= 1 KiB each; crc32_small.h), CRC i to
// out[out_idx[i]] (out_idx non-null) or out[i]; the count from *n_dev when set
// (n_items: its upper bound).
hipError_t launch_small(const ItemsArgs &a, bool nt, int max_blocks, hipStream_t stream);
bool small_kernel_on();
hipError_t launch_splitmix_fill(void *dst, uint64_t nbytes, uint64_t seed, hipStream_t stream);
hipError_t launch_stream_read(const void *p, uint64_t nbytes, int pattern, bool nt, int max_blocks, uint32_t *out,
                              hipStream_t stream);
// The rows kernel's memory stream alone (uniform 4 KiB rows, DYN + tail
// stealing from a.steal, CRC work compiled out; a.out: >= 16 * max_blocks words
// the kernel never stores in practice).  Only for batches large enough to deal
// dynamically with a steal pool.
hipError_t launch_stream_rows(const ItemsArgs &a, int max_blocks, hipStream_t stream, hipEvent_t steal_done = nullptr,
                              bool *steal_recorded = nullptr);

} // namespace rpccrc
