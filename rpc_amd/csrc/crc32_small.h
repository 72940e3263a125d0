// rpc_amd/csrc/crc32_small.h -- the small-body kernel (device code, round 5).
//
// Ragged batches of SMALL bodies -- len + end pad z <= 1 KiB, four per 4 KiB
// row as in the rows kernel's QB = 4 (one body per 1 KiB quarter) -- are bound
// by latency, not by bytes: C2's 1.67M small bodies carry 0.57 GB, and the rows
// kernel's QB = 4 loop over a list of them ran at ~1.2 TB/s (a wave took ~5-7
// us per row: the row's metadata came from scalar loads issued with the row,
// so every row waited for a metadata round trip AND a data round trip, one
// row of data in flight).  Here a wave walks a contiguous range of the list in
// ITERATIONS of 16 bodies (4 rows):
//   * metadata by VECTOR loads, 16 lanes per iteration (offset, length, output
//     index), two iterations ahead -- in the vmcnt queue with the rows, so a
//     wait for them never waits for an LDS lookup (scalar loads share lgkmcnt
//     with the chain's ds_reads and return out of order);
//   * each body's zlib seed Tq[len + z] gathered per lane one iteration ahead;
//   * row data THREE rows ahead (four row buffers, 64 VGPRs);
//   * a row's quarter bases and windows from v_readlane of the metadata;
//   * every iteration issues the same 21 vector-memory instructions (offsets,
//     lengths, indices, seeds, 16 row loads, one CRC store), invalid lanes
//     through out-of-range buffer offsets, so the compiler's vmcnt counts are
//     exact and the prefetch is never drained.
// The row arithmetic is the rows kernel's QB = 4 row (crc32_rows.h): edge fix
// per quarter, transpose, chain, merge step 1, seed, ZI pad undo.
// Reference: every body's CRC is crc.c:4-9 (zlib crc32 of the body).
#pragma once
#include "crc32_rows.h"

namespace rpccrc {

namespace small {

constexpr uint32_t kIter = 16; // bodies per iteration (4 rows of 4 quarters)

// An iteration's metadata: lane j < 16 holds body i0 + j (other lanes zeros).
struct Meta {
  uint32_t olo, ohi; // offset
  uint32_t len;      // length (after derive: (len << 4) | z)
  uint32_t idx;      // output slot
  uint32_t seed;     // after derive: Tq[len + z] (0 for an empty body or RAW mode)
};

// Buffer descriptor for a metadata array slice (range 1 GiB, zeros past it).
__device__ __forceinline__ __amdgpu_buffer_rsrc_t meta_rsrc(const void *p) {
  return __builtin_amdgcn_make_buffer_rsrc(const_cast<void *>(p), (short)0, (int)rows::kRsrcRange, 0x00020000);
}

} // namespace small

// IDX: CRC i goes to out[out_idx[i]] (split lists); else out[i].
template <bool NT, bool IDX>
__global__ void __launch_bounds__(1024, 4) crc32_small_kernel(ItemsArgs a) {
  using namespace rows;
  using namespace small;
  __shared__ __attribute__((aligned(16))) uint32_t s_lds[kLdsBytesV2 / 4];
  // Edge masks of a quarter's two edge pieces, one 16-B row per case: [f] keeps
  // bytes >= f of the piece holding the body's first byte, [16 + z] bytes below
  // 16 - z of the window's last piece (its z pad).  Four scalar masks per fix
  // cost ~16 SALU; a row has up to eight fixes, and one scalar unit serves the
  // CU's 16 waves (the kernel was SALU-bound: 310 SALU per row, profiles/r05u).
  __shared__ __attribute__((aligned(16))) uint32_t s_mask[2 * 16 * 4];
  static_assert(sizeof(s_lds) + sizeof(s_mask) <= kRowsLdsMax, "leave a CU room for the drop-in service");
  const uint64_t n = a.n_dev ? ld_const(a.n_dev, 0) : a.n_items;
  if (n == 0) return; // (block-uniform: before the image copy)
  if (threadIdx.x < 128u) {
    const uint32_t t = threadIdx.x, k = (t >> 2) & 15u, d = t & 3u;
    s_mask[t] = (t < 64u) ? keep_front_dword(k, d) : keep_end_dword(16u - k, d);
  }
  copy_lds_image<kLdsBytesV2>(a.lds_image, s_lds);
  __syncthreads();
  const uint8_t *lds = reinterpret_cast<const uint8_t *>(s_lds);

  const uint32_t lane = threadIdx.x & 63u;
  const uint32_t lane4 = (lane & 31u) * 4u;
  const uint32_t lsel = lane4 | ((lane4 + 128u) << 8) | (1u << 16);  // MAIN tables
  const uint32_t lsel1 = lane4 | ((lane4 + 128u) << 8) | (2u << 16); // ST1
  const uint32_t hi = lane >> 4;
  const bool upper = (lane & 16u) != 0;
  const uint32_t pofs = 16u * piece_of_lane(lane);
  const DistLane dl = dist_lane(lane);
  const uint32_t mode = a.mode;

  // Static contiguous ranges of whole iterations per wave (byte balance: a
  // wave's share holds hundreds of bodies, and a small body's row costs about
  // the same whatever its length).
  const uint32_t wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  const uint64_t nwaves = (uint64_t)gridDim.x * 16u;
  const uint64_t gw = (uint64_t)blockIdx.x * 16u + wave;
  const uint64_t n_it = (n + kIter - 1) / kIter;
  const uint64_t it_lo = n_it * gw / nwaves, it_hi = n_it * (gw + 1) / nwaves;
  if (it_lo >= it_hi) return;

  const uint64_t ubase = (uint64_t)(uintptr_t)a.base;
  const __amdgpu_buffer_rsrc_t tq_rsrc = meta_rsrc(a.tq);

  // Metadata loads of iteration `it` (lanes 0..15; past the range: nothing read).
  auto meta_load = [&](uint64_t it, Meta &m) {
    const uint64_t i0 = it * kIter;
    const bool in = it < it_hi; // uniform
    // the slice's first element (uniform: readfirstlane keeps the descriptor
    // in SGPRs -- a select merged into the lanes' validity test made it a VGPR
    // value and every load a waterfall loop)
    const uint32_t s0 = (uint32_t)__builtin_amdgcn_readfirstlane((int)(in ? (uint32_t)i0 : 0u));
    const uint32_t s1 = (uint32_t)__builtin_amdgcn_readfirstlane((int)(in ? (uint32_t)(i0 >> 32) : 0u));
    const uint64_t first = ((uint64_t)s1 << 32) | s0;
    const bool ok = in & (lane < kIter) & (i0 + lane < n);
    const uint32_t o8 = ok ? lane * 8u : kOobOffset, o4 = ok ? lane * 4u : kOobOffset;
    const __amdgpu_buffer_rsrc_t ro = meta_rsrc(a.offsets + first);
    const __amdgpu_buffer_rsrc_t rl = meta_rsrc(a.lengths + first);
    m.olo = __builtin_amdgcn_raw_buffer_load_b32(ro, (int)o8, 0, 0);
    m.ohi = __builtin_amdgcn_raw_buffer_load_b32(ro, (int)(ok ? o8 + 4u : kOobOffset), 0, 0);
    m.len = __builtin_amdgcn_raw_buffer_load_b32(rl, (int)o4, 0, 0);
    if constexpr (IDX) {
      const __amdgpu_buffer_rsrc_t ri = meta_rsrc(a.out_idx + first);
      m.idx = __builtin_amdgcn_raw_buffer_load_b32(ri, (int)o4, 0, 0);
    } else {
      m.idx = (uint32_t)i0 + lane;
    }
  };
  // After the loads: (len << 4) | z per lane, and the seed gather.
  auto derive = [&](Meta &m) {
    const uint32_t z = (0u - ((uint32_t)ubase + m.olo + m.len)) & 15u;
    const bool live = m.len != 0u && mode != kModeRaw;
    m.seed = __builtin_amdgcn_raw_buffer_load_b32(tq_rsrc, (int)(live ? (m.len + z) * 4u : kOobOffset), 0, 0);
    m.len = m.len == 0u ? 0u : ((m.len << 4) | z);
  };
  // Row k (0..3) of an iteration: quarter b <- body lane 4k + b.
  auto issue = [&](const Meta &m, uint32_t k, u32x4 (&buf)[4]) {
#pragma unroll
    for (uint32_t b = 0; b < 4; ++b) {
      const uint32_t src = 4u * k + b;
      const uint32_t olo = __builtin_amdgcn_readlane(m.olo, src);
      const uint32_t ohi = __builtin_amdgcn_readlane(m.ohi, src);
      const uint32_t lz = __builtin_amdgcn_readlane(m.len, src);
      const uint64_t p = ubase + (((uint64_t)ohi << 32) | olo);
      const uint32_t len = lz >> 4, z = lz & 15u;
      const bool live = len != 0u;
      const uint64_t base = live ? (p & ~(uint64_t)15) : ubase;
      // window = the 1 KiB ending at the body's 16-B-rounded end
      const int32_t o = (int32_t)(len + z) - (int32_t)kQuarter + (int32_t)(p & 15u) + (int32_t)pofs;
      const uint32_t off = live ? min((uint32_t)o, kOobOffset) : kOobOffset;
      buf[b] = ldb16<NT>(row_rsrc(base), off);
    }
  };
  // Row k's four CRCs into lanes 4k .. 4k + 3 of outv.
  auto compute = [&](const Meta &m, uint32_t k, u32x4 (&buf)[4], uint32_t &outv) {
    uint32_t lz[4], zany = 0, zl = 0, sl = 0;
    const uint32_t e_end = (lane == lane_of_piece(63u)) ? 0u : 0xFFFFFFFFu; // the window's last piece
#pragma unroll
    for (uint32_t b = 0; b < 4; ++b) {
      lz[b] = __builtin_amdgcn_readlane(m.len, 4u * k + b);
      const uint32_t len = lz[b] >> 4, z = lz[b] & 15u;
      // both edge fixes, unconditionally (rows::fix_quarter's arithmetic with the
      // masks from s_mask; an aligned front or z = 0 reads an all-ones row, and
      // an empty quarter's pieces are zeros already)
      const uint32_t front = kQuarter - len - z; // < 1024 for a live body
      const u32x4 mf = *reinterpret_cast<const u32x4 *>(s_mask + 4u * (front & 15u));
      const u32x4 me = *reinterpret_cast<const u32x4 *>(s_mask + 64u + 4u * z);
      const uint32_t e_front = (lane == lane_of_piece((front >> 4) & 63u)) ? 0u : 0xFFFFFFFFu;
#pragma unroll
      for (uint32_t d = 0; d < 4; ++d)
        buf[b][d] = and_or_keep(and_or_keep(buf[b][d], mf[d], e_front), me[d], e_end);
      zany |= z;
      zl = (hi == b) ? z : zl;
      const uint32_t sd = __builtin_amdgcn_readlane(m.seed, 4u * k + b);
      sl = (hi == b) ? sd : sl;
    }
    transpose(buf);
    uint32_t res = row_quarters(lds, buf, lsel, lsel1, upper) ^ sl; // 16-lane row b: body 4k + b
    if (zany != 0u) {
      const uint32_t nib = (res >> dl.shift) & 15u;
      const uint32_t t = dist_reduce8(lds_ld(lds, kLdsZI2 + (zl - 1u) * 512u + dl.n64 + nib * 4u));
      res = (zl != 0u) ? t : res; // valid in lanes 4..7 of each row
    }
    if (mode == kModeFinal) res = ~res;
#pragma unroll
    for (uint32_t b = 0; b < 4; ++b) {
      uint32_t v = __builtin_amdgcn_readlane(res, 16u * b + 4u);
      if (lz[b] == 0u) v = 0u;
      outv = (lane == 4u * k + b) ? v : outv;
    }
  };
  // The iteration's 16 CRCs (lanes past the range store nothing).
  auto store = [&](const Meta &m, uint64_t it, uint32_t outv) {
    const bool ok = lane < kIter && it * kIter + lane < n;
    if (ok) a.out[m.idx] = outv;
  };

  Meta m0, m1, m2;
  u32x4 B0[4], B1[4], B2[4], B3[4];
  meta_load(it_lo, m0);
  meta_load(it_lo + 1, m1);
  derive(m0);
  issue(m0, 0, B0);
  issue(m0, 1, B1);
  issue(m0, 2, B2);
  for (uint64_t it = it_lo; it < it_hi; ++it) {
    uint32_t outv = 0;
    meta_load(it + 2, m2);
    issue(m0, 3, B3);
    compute(m0, 0, B0, outv);
    derive(m1);
    issue(m1, 0, B0);
    compute(m0, 1, B1, outv);
    issue(m1, 1, B1);
    compute(m0, 2, B2, outv);
    issue(m1, 2, B2);
    compute(m0, 3, B3, outv);
    store(m0, it, outv);
    m0 = m1;
    m1 = m2;
  }
}

} // namespace rpccrc
