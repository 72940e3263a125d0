// rpc_amd/csrc/crc32_packed.h -- the "packed" ragged-batch kernel (device code).
//
// Ragged batches (config C2: 4M bodies, 64 B - 64 KiB) waste much of the QB = 1
// rows kernel: every body starts with a partial 4 KiB row (on average 2 KiB of
// dead lanes per body), a small body takes a whole row, and dealing bodies by
// count leaves waves ~1.2x unbalanced.  This kernel cuts every body into 1 KiB
// CHUNKS whose windows end at the body's 16-B-aligned virtual end (only the
// first chunk is partial, only the last one carries the z pad), concatenates
// the chunks of consecutive bodies into one stream, and packs that stream four
// chunks per 4 KiB row: a row may hold quarters of up to four bodies.
//
// Balance: the plan kernels (crc32_kernels.hip) split the chunk stream into
// SLICES of S chunks; a body belongs to the slice its first chunk lies in and
// slice_rec[s] holds the first body of slice s.  Slices are dealt round-robin
// over the workgroups (a moving window over HBM, like the rows kernel), the
// waves of a workgroup take its slices from an LDS counter, and a wave
// walks the bodies of its slices with a scalar cursor, packing chunks across
// body and slice boundaries.  A body is always processed start to end by ONE
// wave (past its slice's end if need be), so the Horner chain across rows stays
// inside the wave: no cross-wave combine and no buffer sized by the chunk count.
//
// Row algebra (crc32_gf2.h notation).  After the chain and merge step 1 every
// lane of 16-lane row hi holds q_hi = crc0 of quarter hi (a body's first chunk
// also XORs in its zlib seed A_{first}(0xFFFFFFFF)).  Consecutive quarters of
// one body form a RUN [s, e].  One distributed ds_read per lane shifts each
// quarter to the end of its run, X_hi = A_{1024*(e-hi)}(q_hi) (ST2 entry
// 3-(e-hi)); in the same read lanes 8..15 of row 0 shift the register W of a
// body continuing from the previous row by A_{1024*(e_0+1)} (ST2 entry 2-e_0,
// or RW for a whole row).  The runs are then XORed in scalar registers.  A run
// ending on its body's last chunk is a finished body: the ZI_z undo of its pad
// is one more distributed step (up to four bodies at once, one per row), then
// the final complement; a run reaching the row end continues as W.
#pragma once
#include "crc32_rows.h"

namespace rpccrc {

struct PackedArgs {
  const uint8_t *base;
  const uint64_t *offsets;    // body i = base[offsets[i], + lengths[i])
  const uint32_t *lengths;
  uint64_t n_items;           // < 2^32 - 1 (slice records hold u32 body indices)
  const uint4 *slice_rec;     // [nslices + 1] SliceRec, written by the plan kernel
  const uint64_t *plan;       // plan[0] = nslices, plan[1] = S (device-written)
  uint32_t mode;
  const uint4 *lds_image;
  const uint32_t *tq;         // Tq[q] = A_q(0xFFFFFFFF), q = 0..4096
  uint32_t *out;
};

namespace packed {

constexpr uint32_t kChunk = 1024;

// Plan record of slice s: its first body and that body's offset / length, so a
// wave enters a slice with one scalar load (prefetched a slice ahead) instead
// of a chain slice table -> body table.  Record nslices is the sentinel {n}.
struct SliceRec {
  uint32_t b;
  uint32_t len;
  uint64_t off;
};
static_assert(sizeof(SliceRec) == 16, "one uint4 per record");

// Chunks of a body of `len` bytes ending at address `end`: windows end at the
// virtual end end + z, z = (-end) mod 16.  Empty bodies have no chunks.
__host__ __device__ __forceinline__ uint32_t body_chunks(uint64_t end, uint32_t len) {
  const uint32_t z = (uint32_t)(0u - (uint32_t)end) & 15u;
  return len ? (uint32_t)(((uint64_t)len + z + kChunk - 1) / kChunk) : 0u;
}

// Quarter descriptor, carried from issue to compute (wave-uniform).
constexpr uint32_t kQFirst = 1u << 15, kQLast = 1u << 16, kQValid = 1u << 17;
struct Quarter {
  uint32_t info; // clen (bits 0-10) | z << 11 | first << 15 | last << 16 | valid << 17
  uint32_t body;
  uint32_t seed; // A_{clen+z}(0xFFFFFFFF) on a body's first chunk (kModeFinal), else 0
};
__device__ __forceinline__ uint32_t q_clen(uint32_t i) { return i & 0x7FFu; }
__device__ __forceinline__ uint32_t q_z(uint32_t i) { return (i >> 11) & 15u; }

// The wave's scalar cursor.  Body b+1's metadata and the next slice's record
// are loaded one step ahead, so moving to a new body or slice issues loads but
// never waits on one in the issue path.
struct Cursor {
  uint64_t s;      // current slice
  uint64_t p0;     // start address of body b
  uint32_t b;      // current body
  uint32_t bend;   // first body of the next slice (bodies [., bend) are ours)
  uint32_t k;      // next chunk of body b
  uint32_t nch;    // chunks of body b
  uint32_t len;
  uint32_t z;
  uint64_t nb_off; // body b+1 (prefetched)
  uint32_t nb_len;
  uint64_t ns_s;   // the wave's next slice,
  SliceRec ns;     // its record (prefetched) and its end body
  uint32_t ns_end;
  bool done;
};

} // namespace packed

template <bool NT>
__global__ void __launch_bounds__(1024, 4) crc32_packed_kernel(PackedArgs a) {
  using namespace rows;
  using namespace packed;
  __shared__ __attribute__((aligned(16))) uint32_t s_lds[kLdsBytesV2 / 4];
  // Workgroup-dynamic slice dealing (as the rows kernel's DYN): workgroup vb
  // owns rounds of 16 consecutive slices, round r = slices (r * blocks + vb) * 16
  // + [0, 16), and its waves take the next slice from this LDS counter, so they
  // finish together and neighbouring bodies (and their metadata cache lines)
  // are walked by one CU at about the same time.
  __shared__ uint32_t s_grab;
  if (threadIdx.x == 0) s_grab = 0;
  copy_lds_image<kLdsBytesV2>(a.lds_image, reinterpret_cast<uint4 *>(s_lds));
  __syncthreads();
  const uint8_t *lds = reinterpret_cast<const uint8_t *>(s_lds);

  const uint32_t lane = threadIdx.x & 63u;
  const uint32_t lane4 = (lane & 31u) * 4u;
  const uint32_t lsel = lane4 | ((lane4 + 128u) << 8) | (1u << 16);  // MAIN tables
  const uint32_t lsel1 = lane4 | ((lane4 + 128u) << 8) | (2u << 16); // ST1
  const uint32_t hi = lane >> 4, lo = lane & 15u;
  const uint32_t pofs = 16u * piece_of_lane(lane);
  // distributed-step lane constants (the lane looks up nibble lo & 7)
  const uint32_t nshift = 4u * (lo & 7u);
  const uint32_t n256 = (lo & 7u) * 256u, n64 = (lo & 7u) * 64u;
  const bool own = lo < 8u;                // looks up its own row's value
  const bool wlane = hi == 0u && lo >= 8u; // looks up the carried W
  const uint32_t hi8 = 8u * hi;

  const uint32_t nblk = gridDim.x;
  // XCD-aware wave numbering (see crc32_rows_kernel): neighbouring slices, and
  // so neighbouring outputs, live on one XCD.
  const uint32_t vb = (nblk % 8u == 0u) ? (blockIdx.x % 8u) * (nblk / 8u) + blockIdx.x / 8u : blockIdx.x;
  const uint64_t nslices = ld_const(a.plan, 0);
  const uint32_t mode = a.mode;
  auto grab = [&]() -> uint32_t { // lane 0 holds the grabbed k; read a step later
    uint32_t k = 0;
    if (lane == 0) k = __hip_atomic_fetch_add(&s_grab, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
    return k;
  };
  auto slice_of = [&](uint32_t k) -> uint64_t { return ((uint64_t)(k >> 4) * nblk + vb) * 16u + (k & 15u); };
  const uint64_t s0 = slice_of((uint32_t)__builtin_amdgcn_readfirstlane((int)grab()));
  if (s0 >= nslices) return;
  uint32_t pend = grab();

  Cursor cur;
  const uint64_t last_body = a.n_items - 1;
  const uint32_t *recw = reinterpret_cast<const uint32_t *>(a.slice_rec);
  auto rec = [&](uint64_t sl) -> SliceRec { // one s_load_dwordx4
    SliceRec x;
    x.b = ld_const(recw, 4 * sl);
    x.len = ld_const(recw, 4 * sl + 1);
    x.off = (uint64_t)ld_const(recw, 4 * sl + 2) | ((uint64_t)ld_const(recw, 4 * sl + 3) << 32);
    return x;
  };
  auto prefetch_body = [&]() { // body b+1 (an in-range index either way)
    const uint64_t nb = (uint64_t)cur.b + 1 <= last_body ? (uint64_t)cur.b + 1 : last_body;
    cur.nb_off = ld_const(a.offsets, nb);
    cur.nb_len = ld_const(a.lengths, nb);
  };
  auto prefetch_slice = [&]() { // the wave's next slice (grabbed a step ago) and its record
    cur.ns_s = slice_of((uint32_t)__builtin_amdgcn_readfirstlane((int)pend));
    if (cur.ns_s < nslices) pend = grab();
    const uint64_t sl = cur.ns_s < nslices ? cur.ns_s : nslices - 1;
    cur.ns = rec(sl);
    cur.ns_end = ld_const(recw, 4 * (sl + 1));
  };
  auto enter = [&](uint64_t off, uint32_t len) { // body b with this metadata becomes current
    cur.len = len;
    cur.p0 = (uint64_t)(uintptr_t)a.base + off;
    cur.z = (uint32_t)(0u - (uint32_t)(cur.p0 + len)) & 15u;
    cur.nch = body_chunks(cur.p0 + len, len);
    cur.k = 0;
  };
  // Move the cursor onto its next chunk (next body, next slice of this wave);
  // false once the wave's slices are exhausted.
  auto settle = [&]() -> bool {
    if (cur.done) return false;
    while (cur.k >= cur.nch) {
      if (cur.b + 1u < cur.bend) { // next body of this slice
        ++cur.b;
        enter(cur.nb_off, cur.nb_len);
        prefetch_body();
      } else { // next slice of this wave
        cur.s = cur.ns_s;
        if (cur.s >= nslices) {
          cur.done = true;
          return false;
        }
        cur.b = cur.ns.b;
        cur.bend = cur.ns_end;
        if (cur.b < cur.bend) enter(cur.ns.off, cur.ns.len);
        else cur.nch = cur.k = 0; // empty slice (inside a long body of an earlier one)
        prefetch_body();
        prefetch_slice();
      }
    }
    return true;
  };

  {
    const SliceRec r0 = rec(s0);
    cur.s = s0;
    cur.b = r0.b;
    cur.bend = ld_const(recw, 4 * (s0 + 1));
    cur.done = false;
    if (cur.b < cur.bend) enter(r0.off, r0.len);
    else cur.nch = cur.k = 0;
    prefetch_body();
    prefetch_slice();
  }
  if (!settle()) return;
  const uint64_t safe = cur.p0 & ~(uint64_t)15; // 16-B block of a byte this wave reads

  // The next chunk of the wave's stream as one quarter of the row being issued.
  auto take = [&](Quarter &q, uint64_t &qp0) {
    if (!settle()) {
      q.info = 0;
      q.body = 0;
      q.seed = 0;
      qp0 = safe;
      return;
    }
    const uint64_t v = (uint64_t)cur.len + cur.z;
    const uint64_t wend = cur.p0 + v - (uint64_t)(cur.nch - 1u - cur.k) * kChunk; // 16-B aligned
    const bool first = cur.k == 0, last = cur.k + 1u == cur.nch;
    const uint64_t rs = first ? cur.p0 : wend - kChunk; // real bytes [rs, re)
    const uint64_t re = last ? cur.p0 + cur.len : wend;
    const uint32_t clen = (uint32_t)(re - rs);
    const uint32_t z = last ? cur.z : 0u;
    q.info = clen | (z << 11) | (first ? kQFirst : 0u) | (last ? kQLast : 0u) | kQValid;
    q.body = cur.b;
    q.seed = (first && mode != kModeRaw) ? ld_const(a.tq, clen + z) : 0u;
    qp0 = rs;
    ++cur.k;
  };

  auto issue = [&](Quarter (&q)[4], u32x4 (&buf)[4]) {
    uint64_t p[4];
    bool full;
    if (settle() && cur.k + 4u <= cur.nch) {
      // Common case: the next four chunks all belong to the current body.
      // Only quarter 0 can be its first chunk and only quarter 3 its last.
      const uint64_t wend0 = cur.p0 + (uint64_t)cur.len + cur.z - (uint64_t)(cur.nch - 1u - cur.k) * kChunk;
      const bool first = cur.k == 0, last = cur.k + 4u == cur.nch;
      const uint32_t c0 = first ? (uint32_t)(wend0 - cur.p0) : kChunk;
      const uint32_t c3 = last ? kChunk - cur.z : kChunk;
      const uint32_t z3 = last ? cur.z : 0u;
      q[0].info = c0 | (first ? kQFirst : 0u) | kQValid;
      q[0].seed = (first && mode != kModeRaw) ? ld_const(a.tq, c0) : 0u;
      q[1].info = kChunk | kQValid;
      q[1].seed = 0;
      q[2].info = kChunk | kQValid;
      q[2].seed = 0;
      q[3].info = c3 | (z3 << 11) | (last ? kQLast : 0u) | kQValid;
      q[3].seed = 0;
#pragma unroll
      for (int b = 0; b < 4; ++b) q[b].body = cur.b;
      p[0] = first ? cur.p0 : wend0 - kChunk;
      p[1] = wend0;
      p[2] = wend0 + kChunk;
      p[3] = wend0 + 2 * kChunk;
      cur.k += 4u;
      full = !first && !last;
    } else {
      // Body or slice boundary inside the row: one chunk at a time (one copy
      // of the cursor code; the quarter index only selects registers).
      full = true;
#pragma nounroll
      for (int b = 0; b < 4; ++b) {
        Quarter t;
        uint64_t tp;
        take(t, tp);
        full = full && q_clen(t.info) == kChunk;
        if (b == 0) { q[0] = t; p[0] = tp; }
        else if (b == 1) { q[1] = t; p[1] = tp; }
        else if (b == 2) { q[2] = t; p[2] = tp; }
        else { q[3] = t; p[3] = tp; }
      }
    }
    (void)full;
    // One load path for every row (a separate path for whole rows made the
    // compiler's vmcnt accounting wait for the row just issued): the window of
    // quarter b starts d bytes from the 16-B block holding the chunk's first
    // byte; pieces before that block read as zeros without touching memory.
#pragma unroll
    for (int b = 0; b < 4; ++b) {
      const uint32_t clen = q_clen(q[b].info);
      const uint64_t base = clen ? (p[b] & ~(uint64_t)15) : safe;
      const int32_t d = clen ? (int32_t)(clen + q_z(q[b].info)) - (int32_t)kChunk + (int32_t)(p[b] & 15) : INT32_MIN / 2;
      buf[b] = ldb16_or_zero<NT>(row_rsrc(base), d + (int32_t)pofs);
    }
  };

  // Transpose + chain + merge step 1: every lane of 16-lane row hi gets crc0
  // of quarter hi (crc32_rows.h).
  auto quarter_crcs = [&](u32x4 (&buf)[4]) -> uint32_t {
    transpose(buf);
    return merge_lo(lds, seg_crc(lds, buf, lsel), lsel1);
  };

  uint32_t W = 0; // register of the body continuing into the next row (uniform)
  // Finished CRCs parked one per lane (value + body index), stored <= 64 at a time.
  uint32_t outv = 0, outi = 0, ocount = 0;
  auto flush = [&]() {
    if (lane < ocount) a.out[outi] = outv;
    ocount = 0;
  };

  auto compute = [&](const Quarter (&q)[4], u32x4 (&buf)[4]) {
    uint32_t sl = 0;
#pragma unroll
    for (int b = 0; b < 4; ++b) {
      const uint32_t clen = q_clen(q[b].info), z = q_z(q[b].info);
      const int32_t vstart = (int32_t)(clen + z) - (int32_t)kChunk;
      if (vstart < 0 || z != 0u) buf[b] = mask_piece32(buf[b], vstart + (int32_t)pofs, (int32_t)clen);
      sl = (hi == (uint32_t)b) ? q[b].seed : sl;
    }
    const uint32_t v = quarter_crcs(buf) ^ sl; // row hi: q_hi (^ seed on a first chunk)

    // Quarter b ends a run if it is its body's last chunk, invalid, or b = 3.
    bool endq[4], lastq[4];
#pragma unroll
    for (int b = 0; b < 4; ++b) {
      lastq[b] = (q[b].info & (kQLast | kQValid)) == (kQLast | kQValid);
      endq[b] = b == 3 || (q[b].info & (kQLast | kQValid)) != kQValid;
    }
    uint32_t e[4];
    e[3] = 3u;
    e[2] = endq[2] ? 2u : 3u;
    e[1] = endq[1] ? 1u : e[2];
    e[0] = endq[0] ? 0u : e[1];
    const uint32_t dpack = e[0] | ((e[1] - 1u) << 8) | ((e[2] - 2u) << 16); // d = e(hi) - hi
    const bool cont = (q[0].info & (kQFirst | kQValid)) == kQValid;        // quarter 0 continues W
    uint32_t addr;
    {
      const uint32_t d = (dpack >> hi8) & 3u;
      const uint32_t nib = ((own ? v : W) >> nshift) & 15u;
      uint32_t a_w;
      if (!cont) a_w = kLdsZero;
      else if (e[0] == 3u) a_w = kLdsRW2 + n64 + nib * 4u;            // A_4096
      else a_w = kLdsST2 + n256 + (2u - e[0]) * 4u + nib * 16u;       // A_{1024*(e0+1)}
      const uint32_t a_own = kLdsST2 + n256 + (3u - d) * 4u + nib * 16u; // A_{1024*d}
      addr = own ? a_own : (wlane ? a_w : kLdsZero);
    }
    const uint32_t t = dist_reduce8(lds_ld(lds, addr));
    uint32_t X[4];
#pragma unroll
    for (int b = 0; b < 4; ++b) X[b] = (uint32_t)__builtin_amdgcn_readlane((int)t, 16 * b + 4);
    const uint32_t wsh = (uint32_t)__builtin_amdgcn_readlane((int)t, 12);

    // Runs, in scalar registers.
    uint32_t acc = cont ? wsh : 0u;
    uint32_t fin[4];
    uint32_t fmask = 0, zmask = 0;
#pragma unroll
    for (int b = 0; b < 4; ++b) {
      acc ^= X[b];
      fin[b] = acc;
      if (lastq[b]) {
        fmask |= 1u << b;
        if (q_z(q[b].info) != 0u) zmask |= 1u << b;
      }
      if (endq[b]) {
        if (b == 3 && !lastq[3]) W = acc;
        acc = 0u;
      }
    }
    if (fmask == 0u) return;
    if (zmask != 0u) {
      // ZI_z undo of the finished bodies' pads, row b working on quarter b's body.
      uint32_t fv = fin[0], zl = q_z(q[0].info);
#pragma unroll
      for (int b = 1; b < 4; ++b) {
        fv = (hi == (uint32_t)b) ? fin[b] : fv;
        zl = (hi == (uint32_t)b) ? q_z(q[b].info) : zl;
      }
      const bool zrow = ((zmask >> hi) & 1u) != 0u;
      const uint32_t nib = (fv >> nshift) & 15u;
      const uint32_t za = (own && zrow) ? kLdsZI2 + (zl - 1u) * 512u + n64 + nib * 4u : kLdsZero;
      const uint32_t tz = dist_reduce8(lds_ld(lds, za));
#pragma unroll
      for (int b = 0; b < 4; ++b)
        if ((zmask >> b) & 1u) fin[b] = (uint32_t)__builtin_amdgcn_readlane((int)tz, 16 * b + 4);
    }
    if (ocount > 60u) flush();
#pragma unroll
    for (int b = 0; b < 4; ++b) {
      if ((fmask >> b) & 1u) {
        const uint32_t r = (mode == kModeFinal) ? ~fin[b] : fin[b];
        outv = (lane == ocount) ? r : outv;
        outi = (lane == ocount) ? q[b].body : outi;
        ++ocount;
      }
    }
  };

  // One row of loads in flight ahead of the row being computed; one exit at
  // the bottom (see crc32_rows_kernel).  Rows past the wave's stream are
  // all-invalid: safe loads, no run finishes.
  Quarter qa[4], qb[4];
  u32x4 bufA[4], bufB[4];
  issue(qa, bufA);
  do {
    issue(qb, bufB);
    compute(qa, bufA);
    issue(qa, bufA);
    compute(qb, bufB);
  } while ((qa[0].info & kQValid) != 0u);
  flush();
}

} // namespace rpccrc
