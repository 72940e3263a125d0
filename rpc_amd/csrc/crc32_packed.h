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
// waves of a workgroup take its slices from an LDS counter, and a wave walks
// the bodies of its slices through a 64-body metadata WINDOW (one body per
// lane, loaded a row ahead with vector loads; a prefix scan of the chunk
// counts and one ballot per quarter find the body of each chunk), packing
// chunks across body and slice boundaries.  A body is always processed start to end by ONE
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

// Plan record of slice s: its first body (the kernel reads only .b; the
// body's offset / length ride along for tools).  Record nslices is the
// sentinel {n}.
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
constexpr uint32_t kQLive = 1u << 18; // quarter 0 only: the wave's stream was not finished at issue
struct Quarter {
  uint32_t info; // clen (bits 0-10) | z << 11 | first << 15 | last << 16 | valid << 17
  uint32_t body;
  uint32_t lane; // window lane of the body (its seed is read from that lane)
};
__device__ __forceinline__ uint32_t q_clen(uint32_t i) { return i & 0x7FFu; }
__device__ __forceinline__ uint32_t q_z(uint32_t i) { return (i >> 11) & 15u; }

// Exclusive prefix sum over the 64 lanes: row_shr 1/2/4/8 inside each 16-lane
// row (bound_ctrl: lanes shifted in read 0), then the row totals by readlane.
__device__ __forceinline__ uint32_t wave_excl_scan(uint32_t x, uint32_t lane) {
  uint32_t v = x;
  v += (uint32_t)__builtin_amdgcn_mov_dpp((int)v, 0x111, 0xF, 0xF, true);
  v += (uint32_t)__builtin_amdgcn_mov_dpp((int)v, 0x112, 0xF, 0xF, true);
  v += (uint32_t)__builtin_amdgcn_mov_dpp((int)v, 0x114, 0xF, 0xF, true);
  v += (uint32_t)__builtin_amdgcn_mov_dpp((int)v, 0x118, 0xF, 0xF, true);
  const uint32_t r0 = (uint32_t)__builtin_amdgcn_readlane((int)v, 15);
  const uint32_t r1 = r0 + (uint32_t)__builtin_amdgcn_readlane((int)v, 31);
  const uint32_t r2 = r1 + (uint32_t)__builtin_amdgcn_readlane((int)v, 47);
  const uint32_t add = lane >= 48u ? r2 : lane >= 32u ? r1 : lane >= 16u ? r0 : 0u;
  return v + add - x;
}

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
  copy_lds_image<kLdsBytesV2>(a.lds_image, s_lds);
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
  const uint32_t n64 = (lo & 7u) * 64u;
  const bool own = lo < 8u;                // looks up its own row's value
  const bool wlane = hi == 0u && lo >= 8u; // looks up the carried W
  const uint32_t hi8 = 8u * hi;

  const uint32_t nblk = gridDim.x;
  // XCD-aware wave numbering (see crc32_rows_kernel): neighbouring slices, and
  // so neighbouring outputs, live on one XCD.
  const uint32_t vb = (nblk % 8u == 0u) ? (blockIdx.x % 8u) * (nblk / 8u) + blockIdx.x / 8u : blockIdx.x;
  const uint64_t nslices = ld_const(a.plan, 0);
  const uint32_t mode = a.mode;
  const uint64_t base = (uint64_t)(uintptr_t)a.base;
  auto grab = [&]() -> uint32_t { // lane 0 holds the grabbed k; read a step later
    uint32_t k = 0;
    if (lane == 0) k = __hip_atomic_fetch_add(&s_grab, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
    return k;
  };
  auto slice_of = [&](uint32_t k) -> uint64_t { return ((uint64_t)(k >> 4) * nblk + vb) * 16u + (k & 15u); };
  const uint32_t *recw = reinterpret_cast<const uint32_t *>(a.slice_rec);

  // The wave's stream is the concatenation of the bodies of its slices.  It
  // keeps two slices: the current one, bodies [wb0, cb1) still to walk, and the
  // next one, [nb0, nb1) (empty once the wave's slices are exhausted).
  uint32_t pend = grab();
  uint32_t wb0 = 0, cb1 = 0, nb0 = 0, nb1 = 0;
  bool more_slices = true;
  auto fetch_next = [&]() { // next non-empty slice of this wave into [nb0, nb1)
    nb0 = nb1 = 0;
    while (more_slices) {
      const uint64_t sl = slice_of((uint32_t)__builtin_amdgcn_readfirstlane((int)pend));
      if (sl >= nslices) {
        more_slices = false;
        break;
      }
      pend = grab();
      nb0 = ld_const(recw, 4 * sl);
      nb1 = ld_const(recw, 4 * (sl + 1));
      if (nb0 < nb1) break;
    }
  };
  auto advance = [&]() { // the next slice becomes current
    wb0 = nb0;
    cb1 = nb1;
    fetch_next();
  };
  fetch_next();
  advance();
  if (wb0 >= cb1) return; // no slice for this wave
  uint32_t wk0 = 0;       // chunk of body wb0 where the next row starts

  // WINDOW: the next 64 bodies of the stream, one per lane (lane l < kw: body
  // wb0 + l of the current slice; lane l >= kw: body nb0 + l - kw of the next
  // one), loaded a row ahead with two vector loads and decoded with ballots
  // and readlanes -- no scalar body walk.  Lanes past the stream read zeros.
  const auto off_rsrc = row_rsrc((uint64_t)(uintptr_t)a.offsets);
  const auto len_rsrc = row_rsrc((uint64_t)(uintptr_t)a.lengths);
  const auto tq_rsrc = row_rsrc((uint64_t)(uintptr_t)a.tq);
  uint32_t w_kw = 0, w_b0 = 0, w_n0 = 0, w_n1 = 0; // the window's layout, fixed when it was loaded
  uint32_t w_offlo = 0, w_offhi = 0, w_len = 0;
  auto load_window = [&]() {
    w_kw = (cb1 - wb0) < 64u ? cb1 - wb0 : 64u;
    w_b0 = wb0;
    w_n0 = nb0;
    w_n1 = nb1;
    const uint32_t idx = lane < w_kw ? w_b0 + lane : w_n0 + (lane - w_kw);
    const bool ok = lane < w_kw || idx < w_n1;
    const auto o = __builtin_amdgcn_raw_buffer_load_b64(off_rsrc, ok ? (int)(idx * 8u) : (int)kOobOffset, 0, 0);
    w_offlo = o[0];
    w_offhi = o[1];
    w_len = __builtin_amdgcn_raw_buffer_load_b32(len_rsrc, ok ? (int)(idx * 4u) : (int)kOobOffset, 0, 0);
  };
  load_window();

  auto issue = [&](Quarter (&q)[4], u32x4 (&buf)[4], uint32_t &seedv) {
    // Decode the window: pads, chunk counts and each body's first chunk in
    // window chunk coordinates (body wb0's chunk 0 = position 0).
    const uint32_t endlo = (uint32_t)base + w_offlo + w_len;
    const uint32_t zl = (0u - endlo) & 15u;
    const uint32_t vl = w_len + zl;
    const uint32_t nchl = w_len ? (vl + kChunk - 1u) >> 10 : 0u;
    const uint32_t cst = wave_excl_scan(nchl, lane);
    const bool has = nchl != 0u;
    // zlib seed of the body's first chunk, A_{first window fill}(0xFFFFFFFF)
    seedv = __builtin_amdgcn_raw_buffer_load_b32(tq_rsrc, has ? (int)((vl - ((nchl - 1u) << 10)) * 4u) : (int)kOobOffset,
                                                 0, 0);
    uint32_t nvalid = 4u;
    uint64_t p[4];
    auto locate = [&](uint32_t pos, uint32_t &m, uint32_t &c, uint32_t &nc) -> bool { // body lane holding pos
      const uint64_t m64 = __builtin_amdgcn_ballot_w64(has && cst <= pos);
      m = m64 ? 63u - (uint32_t)__builtin_clzll(m64) : 0u;
      c = (uint32_t)__builtin_amdgcn_readlane((int)cst, m);
      nc = (uint32_t)__builtin_amdgcn_readlane((int)nchl, m);
      return m64 != 0u && pos - c < nc;
    };
    auto body_p0 = [&](uint32_t m, uint32_t &len, uint32_t &z) -> uint64_t {
      len = (uint32_t)__builtin_amdgcn_readlane((int)w_len, m);
      const uint64_t p0 = base + ((uint64_t)(uint32_t)__builtin_amdgcn_readlane((int)w_offhi, m) << 32 |
                                  (uint32_t)__builtin_amdgcn_readlane((int)w_offlo, m));
      z = (uint32_t)(0u - (uint32_t)(p0 + len)) & 15u;
      return p0;
    };
    uint32_t m0, c0, nc0;
    const bool v0 = locate(wk0, m0, c0, nc0);
    const uint32_t body0 = m0 < w_kw ? w_b0 + m0 : w_n0 + (m0 - w_kw);
    bool known = false; // the next row starts inside body m0
    if (v0 && wk0 - c0 + 4u <= nc0) {
      // Common case: the four chunks all belong to one body.  Only quarter 0
      // can be its first chunk and only quarter 3 its last.
      uint32_t len, z;
      const uint64_t p0 = body_p0(m0, len, z);
      const uint32_t j = wk0 - c0;
      const uint64_t wend0 = p0 + len + z - (uint64_t)(nc0 - 1u - j) * kChunk; // end of chunk j's window
      const bool first = j == 0u, last = j + 4u == nc0;
      q[0].info = (first ? (uint32_t)(wend0 - p0) : kChunk) | (first ? kQFirst : 0u) | kQValid;
      q[1].info = kChunk | kQValid;
      q[2].info = kChunk | kQValid;
      q[3].info = (last ? kChunk - z : kChunk) | ((last ? z : 0u) << 11) | (last ? kQLast : 0u) | kQValid;
#pragma unroll
      for (int b = 0; b < 4; ++b) {
        q[b].body = body0;
        q[b].lane = m0;
      }
      p[0] = first ? p0 : wend0 - kChunk;
      p[1] = wend0;
      p[2] = wend0 + kChunk;
      p[3] = wend0 + 2 * kChunk;
      known = !last;
    } else {
      // Body boundaries inside the row (or the end of the stream).
#pragma unroll
      for (int b = 0; b < 4; ++b) {
        const uint32_t pos = wk0 + (uint32_t)b;
        uint32_t m = m0, c = c0, nc = nc0;
        bool valid = v0;
        if (b > 0) valid = nvalid == 4u && locate(pos, m, c, nc);
        if (!valid) {
          if (nvalid == 4u) nvalid = (uint32_t)b;
          q[b].info = 0;
          q[b].body = 0;
          q[b].lane = 0;
          p[b] = base;
          continue;
        }
        uint32_t len, z;
        const uint64_t p0 = body_p0(m, len, z);
        const uint32_t j = pos - c;
        const uint64_t wend = p0 + len + z - (uint64_t)(nc - 1u - j) * kChunk; // 16-B aligned
        const bool first = j == 0u, last = j + 1u == nc;
        const uint64_t rs = first ? p0 : wend - kChunk; // real bytes [rs, re)
        const uint64_t re = last ? p0 + len : wend;
        q[b].info = (uint32_t)(re - rs) | ((last ? z : 0u) << 11) | (first ? kQFirst : 0u) | (last ? kQLast : 0u) | kQValid;
        q[b].body = m < w_kw ? w_b0 + m : w_n0 + (m - w_kw);
        q[b].lane = m;
        p[b] = rs;
      }
    }
    if (wb0 < cb1 || nb0 < nb1) q[0].info |= kQLive;

    // Where the next row starts: the body holding position wk0 + nvalid, or
    // (window exhausted: every lane's chunks taken) the body after the window.
    {
      const uint32_t pos = wk0 + nvalid;
      uint32_t skip; // bodies of the stream before the next row's body
      uint32_t m = m0, c = c0, nc;
      if (known || locate(pos, m, c, nc)) {
        skip = m;
        wk0 = pos - c;
      } else {
        skip = 64u;
        wk0 = 0;
      }
      if (skip < cb1 - wb0) {
        wb0 += skip;
      } else {
        // the current slice is used up; rest bodies into the next
        uint32_t rest = skip - (cb1 - wb0);
        advance();
        while (wb0 < cb1 && rest >= cb1 - wb0) { // the window ran past the next slice too
          rest = 0;
          advance();
        }
        wb0 += rest;
      }
      if (wb0 >= cb1) { // stream finished: later windows are empty
        wb0 = cb1 = 0;
        nb0 = nb1 = 0;
      }
    }
    load_window(); // for the next row

    // One load path for every row (a separate path for whole rows made the
    // compiler's vmcnt accounting wait for the row just issued): the window of
    // quarter b starts d bytes from the 16-B block holding the chunk's first
    // byte; pieces before that block read as zeros without touching memory.
#pragma unroll
    for (int b = 0; b < 4; ++b) {
      const uint32_t clen = q_clen(q[b].info);
      const int32_t d = clen ? (int32_t)(clen + q_z(q[b].info)) - (int32_t)kChunk + (int32_t)(p[b] & 15) : INT32_MIN / 2;
      buf[b] = ldb16_or_zero<NT>(row_rsrc(p[b] & ~(uint64_t)15), d + (int32_t)pofs);
    }
  };

  // Transpose + chain + merge step 1: every lane of 16-lane row hi gets crc0
  // of quarter hi (crc32_rows.h).
  auto quarter_crcs = [&](u32x4 (&buf)[4]) -> uint32_t {
    transpose(buf);
    return row_quarters(lds, buf, lsel, lsel1, (lane & 16u) != 0);
  };

  uint32_t W = 0; // register of the body continuing into the next row (uniform)
  // Finished CRCs parked one per lane (value + body index), stored <= 64 at a time.
  uint32_t outv = 0, outi = 0, ocount = 0;
  auto flush = [&]() {
    if (lane < ocount) a.out[outi] = outv;
    ocount = 0;
  };

  auto compute = [&](const Quarter (&q)[4], u32x4 (&buf)[4], uint32_t seedv) {
    uint32_t sl = 0;
#pragma unroll
    for (int b = 0; b < 4; ++b) {
      const uint32_t clen = q_clen(q[b].info), z = q_z(q[b].info);
      // the quarter's first real byte sits at window offset kChunk - clen - z
      fix_quarter(buf[b], lane, kChunk - clen - z, z);
      const bool seeded = (q[b].info & kQFirst) != 0u && mode != kModeRaw;
      const uint32_t seed = seeded ? (uint32_t)__builtin_amdgcn_readlane((int)seedv, q[b].lane) : 0u;
      sl = (hi == (uint32_t)b) ? seed : sl;
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
      else a_w = st2_byte(lo & 7u, nib, 2u - e[0]);                   // A_{1024*(e0+1)}
      const uint32_t a_own = st2_byte(lo & 7u, nib, 3u - d);              // A_{1024*d}
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
  // all-invalid: out-of-range loads, no run finishes.
  Quarter qa[4], qb[4];
  u32x4 bufA[4], bufB[4];
  uint32_t seedA, seedB;
  issue(qa, bufA, seedA);
  do {
    issue(qb, bufB, seedB);
    compute(qa, bufA, seedA);
    issue(qa, bufA, seedA);
    compute(qb, bufB, seedB);
  } while ((qa[0].info & kQLive) != 0u);
  flush();
}

} // namespace rpccrc
