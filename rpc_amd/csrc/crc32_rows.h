// rpc_amd/csrc/crc32_rows.h -- batched CRC-32 "rows" kernel (device code).
//
// A wavefront processes ROWS of 4 KiB, held as 16 B per lane per slot:
//   load:      4 coalesced global_load_dwordx4 (non-temporal by default); load
//              b covers the 1 KiB quarter b of the row and lane L reads piece
//              p(L) = ((L & 15) << 2) | (L >> 4) of it, so piece q = 64b + p(L)
//              has slot bits (q7 q6) and lane bits (q1 q0 | q5 q4 q3 q2).
//   transpose: v_permlane16_swap on slot pairs (0,1),(2,3) swaps slot bit 0
//              with lane bit 4; v_permlane32_swap on (0,2),(1,3) swaps slot
//              bit 1 with lane bit 5.  Lane L' then holds the contiguous 64-B
//              segment s = L' of the row, slots in byte order.  16 VALU per row.
//   chain:     16 slice-by-4 steps per lane: v_perm_b32 forms each LDS address,
//              4 ds_read_b32 (bank-conflict-free: 32 replicated copies), two
//              v_bitop3_b32 (3-way XOR) fold the lookups and the next dword.
//   merge:     crc0(row) = XOR_L' A_{64*(63-L')} c_L'
//                        = XOR_hi A_{1024*(3-hi)} XOR_lo A_{64*(15-lo)} c_{hi,lo},
//              hi = L' >> 4 (the quarter), lo = L' & 15: nibble step ST1
//              (per lane), DPP quad + row_ror reduction over lo, nibble step
//              ST2 (per row), permlane16/32-swap reductions over hi.  All
//              reductions are VALU; no LDS traffic besides the 16 nibble reads.
// QB = 1: the row is 4 KiB of one item (items of any length, end-aligned rows,
//         Horner across rows with RW, Tq pre-conditioning, ZI trailing-pad undo).
// QB = 4: the row holds four items of <= 1 KiB each (item = quarter = hi), so
//         the merge stops after the lo reduction (no ST2 step).
//
// LDS image (crc32_layout.h "v3"):
//   MAIN [0,128K)  slice-by-4 tables x32 copies (two tables per 256-B row)
//   ST1  16 KiB    ST1[n][nib][c]  = A_{64*(15-(c&15))}(nib<<4n), c = lane&31
//   ST2  2 KiB     ST2[n][nib][hi] = A_{1024*(3-hi)}(nib<<4n)
//   RW   512 B     RW[n][nib]      = A_4096(nib<<4n)
//   ZI   7.5 KiB   ZI[z-1][n][nib] = A_z^-1(nib<<4n)
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

#include <type_traits>

#include "crc32_gf2.h"
#include "crc32_kernels.h"
#include "crc32_layout.h"

namespace rpccrc {

namespace rows {

constexpr uint32_t kRow = 4096;
constexpr uint32_t kQuarter = 1024;

__device__ __forceinline__ uint32_t lds_ld(const uint8_t *lds, uint32_t byte_addr) {
  return *reinterpret_cast<const uint32_t *>(lds + byte_addr);
}

__device__ __forceinline__ uint32_t slice4(const uint8_t *lds, uint32_t x, uint32_t lsel) {
  const uint32_t a3 = __builtin_amdgcn_perm(x, lsel, 0x0C0C0400u);
  const uint32_t a2 = __builtin_amdgcn_perm(x, lsel, 0x0C0C0501u);
  const uint32_t a1 = __builtin_amdgcn_perm(x, lsel, 0x0C020600u);
  const uint32_t a0 = __builtin_amdgcn_perm(x, lsel, 0x0C020701u);
  return lds_ld(lds, a3) ^ lds_ld(lds, a2) ^ lds_ld(lds, a1) ^ lds_ld(lds, a0);
}

// One slice-by-4 step fused with the next data word: A_4(x) ^ w.
__device__ __forceinline__ uint32_t slice4w(const uint8_t *lds, uint32_t x, uint32_t w, uint32_t lsel) {
  const uint32_t a3 = __builtin_amdgcn_perm(x, lsel, 0x0C0C0400u);
  const uint32_t a2 = __builtin_amdgcn_perm(x, lsel, 0x0C0C0501u);
  const uint32_t a1 = __builtin_amdgcn_perm(x, lsel, 0x0C020600u);
  const uint32_t a0 = __builtin_amdgcn_perm(x, lsel, 0x0C020701u);
  const uint32_t t3 = lds_ld(lds, a3), t2 = lds_ld(lds, a2), t1 = lds_ld(lds, a1), t0 = lds_ld(lds, a0);
  return __builtin_amdgcn_bitop3_b32(__builtin_amdgcn_bitop3_b32(t3, t2, t1, 0x96), t0, w, 0x96);
}

template <uint32_t STRIDE, uint32_t SHIFT>
__device__ __forceinline__ uint32_t nib_map(const uint8_t *lds, uint32_t s, uint32_t base) {
  uint32_t r = 0;
#pragma unroll
  for (uint32_t n = 0; n < 8; ++n) r ^= lds_ld(lds, base + n * STRIDE + (((s >> (4 * n)) & 15u) << SHIFT));
  return r;
}

// DPP lane moves (all lanes active, every source valid).
__device__ __forceinline__ uint32_t dpp_xor1(uint32_t v) { // quad_perm [1,0,3,2]
  return (uint32_t)__builtin_amdgcn_mov_dpp((int)v, 0xB1, 0xF, 0xF, false);
}
__device__ __forceinline__ uint32_t dpp_xor2(uint32_t v) { // quad_perm [2,3,0,1]
  return (uint32_t)__builtin_amdgcn_mov_dpp((int)v, 0x4E, 0xF, 0xF, false);
}
__device__ __forceinline__ uint32_t dpp_ror4(uint32_t v) { // row_ror:4
  return (uint32_t)__builtin_amdgcn_mov_dpp((int)v, 0x124, 0xF, 0xF, false);
}
__device__ __forceinline__ uint32_t dpp_ror8(uint32_t v) { // row_ror:8
  return (uint32_t)__builtin_amdgcn_mov_dpp((int)v, 0x128, 0xF, 0xF, false);
}
__device__ __forceinline__ uint32_t swz_xor16(uint32_t v) { // ds_swizzle bit mode, xor 16
  return (uint32_t)__builtin_amdgcn_ds_swizzle((int)v, 0x401F);
}
__device__ __forceinline__ uint32_t shfl_xor32(uint32_t v) {
  return (uint32_t)__shfl_xor((int)v, 32, 64);
}

typedef unsigned int u32x4 __attribute__((ext_vector_type(4)));

template <bool NT>
__device__ __forceinline__ u32x4 ld16(const uint8_t *p) {
  const u32x4 *q = reinterpret_cast<const u32x4 *>(p);
  if constexpr (NT)
    return __builtin_nontemporal_load(q);
  else
    return *q;
}

// Zero bytes of a 16-byte piece (virtual offset v relative to the item start)
// that lie before the item (pos < 0) or at/after its end (pos >= len).
__device__ __forceinline__ u32x4 mask_piece(u32x4 x, int64_t v, int64_t len) {
#pragma unroll
  for (int d = 0; d < 4; ++d) {
    const int64_t lo = v + 4 * d;
    uint32_t m = 0xFFFFFFFFu;
    if (lo < 0) m = (lo <= -4) ? 0u : (m << (8 * (uint32_t)(-lo)));
    const int64_t over = lo + 4 - len;
    if (over > 0) m &= (over >= 4) ? 0u : (0xFFFFFFFFu >> (8 * (uint32_t)over));
    x[d] &= m;
  }
  return x;
}

// Lane that loads piece p of a quarter / piece loaded by lane L (involution-free
// bijection on 0..63): p(L) = ((L & 15) << 2) | (L >> 4).
__device__ __forceinline__ uint32_t piece_of_lane(uint32_t L) { return ((L & 15u) << 2) | (L >> 4); }

// Transpose 4 slots x 64 lanes of 16-B pieces (see header comment).
__device__ __forceinline__ void transpose(u32x4 (&p)[4]) {
#pragma unroll
  for (int d = 0; d < 4; ++d) {
    auto a = __builtin_amdgcn_permlane16_swap(p[0][d], p[1][d], false, false);
    p[0][d] = a[0];
    p[1][d] = a[1];
    auto b = __builtin_amdgcn_permlane16_swap(p[2][d], p[3][d], false, false);
    p[2][d] = b[0];
    p[3][d] = b[1];
  }
#pragma unroll
  for (int d = 0; d < 4; ++d) {
    auto a = __builtin_amdgcn_permlane32_swap(p[0][d], p[2][d], false, false);
    p[0][d] = a[0];
    p[2][d] = a[1];
    auto b = __builtin_amdgcn_permlane32_swap(p[1][d], p[3][d], false, false);
    p[1][d] = b[0];
    p[3][d] = b[1];
  }
}

// XOR over lane bit 4 / lane bit 5 (every lane gets the pair's XOR).
__device__ __forceinline__ uint32_t xor_lanebit4(uint32_t v) {
  auto a = __builtin_amdgcn_permlane16_swap(v, v, false, false);
  return a[0] ^ a[1];
}
__device__ __forceinline__ uint32_t xor_lanebit5(uint32_t v) {
  auto a = __builtin_amdgcn_permlane32_swap(v, v, false, false);
  return a[0] ^ a[1];
}

__device__ __forceinline__ uint32_t xor3(uint32_t a, uint32_t b, uint32_t c) {
  return __builtin_amdgcn_bitop3_b32(a, b, c, 0x96);
}

// crc0 contribution of this lane's 64-byte segment: 16 slice-by-4 steps.
__device__ __forceinline__ uint32_t seg_crc(const uint8_t *lds, const u32x4 (&p)[4], uint32_t lsel) {
  uint32_t x = p[0][0];
#pragma unroll
  for (int k = 0; k < 4; ++k)
#pragma unroll
    for (int d = 0; d < 4; ++d) {
      if (k == 0 && d == 0) continue;
      x = slice4w(lds, x, p[k][d], lsel);
    }
  return slice4(lds, x, lsel);
}

struct RowTask {
  const uint8_t *p0; // item start
  uint64_t item;
  uint64_t lp;       // len + z (end 16-byte aligned)
  uint32_t len;
  uint32_t nrows;
  uint32_t r;
  uint32_t z;
  uint32_t w0;
  uint32_t valid;
};

} // namespace rows

// Ablation bits (measurement builds in tools/probe_kernels.hip only; product = 0).
constexpr int kRowsAblNoCompute = 1; // XOR fold instead of the slice-by-4 chain
constexpr int kRowsAblNoMerge = 2;   // skip the per-lane shift / reductions
constexpr int kRowsAblNoLoad = 4;    // synthesize row data instead of loading it

namespace rows {

// Two independent chains interleaved step by step (2x LDS reads in flight).
__device__ __forceinline__ void seg_crc2(const uint8_t *lds, const u32x4 (&p)[4], const u32x4 (&q)[4],
                                         uint32_t lsel, uint32_t &s0, uint32_t &s1) {
  uint32_t x = p[0][0], y = q[0][0];
#pragma unroll
  for (int k = 0; k < 4; ++k)
#pragma unroll
    for (int d = 0; d < 4; ++d) {
      if (k == 0 && d == 0) continue;
      const uint32_t nx = slice4w(lds, x, p[k][d], lsel);
      const uint32_t ny = slice4w(lds, y, q[k][d], lsel);
      x = nx;
      y = ny;
    }
  s0 = slice4(lds, x, lsel);
  s1 = slice4(lds, y, lsel);
}

__device__ __forceinline__ uint32_t xor_fold(const u32x4 (&p)[4]) {
  uint32_t r = 0;
#pragma unroll
  for (int k = 0; k < 4; ++k) r ^= p[k][0] ^ p[k][1] ^ p[k][2] ^ p[k][3];
  return r;
}

// Per-row merge (see header): ST1 per lane, reduce over lo (lane bits 0-3),
// then for QB = 1 ST2 per 16-lane row and reduce over hi (lane bits 4-5).
template <int QB>
__device__ __forceinline__ uint32_t merge(const uint8_t *lds, uint32_t s, uint32_t st1_base, uint32_t st2_base) {
  s = nib_map<2048u, 7u>(lds, s, st1_base); // A_{64*(15-lo)}
  s ^= dpp_xor1(s);
  s ^= dpp_xor2(s);
  s ^= dpp_ror4(s);
  s ^= dpp_ror8(s);
  if constexpr (QB == 1) {
    s = nib_map<256u, 4u>(lds, s, st2_base); // A_{1024*(3-hi)}
    s = xor_lanebit4(s);
    s = xor_lanebit5(s);
  }
  return s;
}

template <int QB>
__device__ __forceinline__ void merge2(const uint8_t *lds, uint32_t &s0, uint32_t &s1, uint32_t st1_base,
                                       uint32_t st2_base) {
  s0 = nib_map<2048u, 7u>(lds, s0, st1_base);
  s1 = nib_map<2048u, 7u>(lds, s1, st1_base);
  s0 ^= dpp_xor1(s0);
  s1 ^= dpp_xor1(s1);
  s0 ^= dpp_xor2(s0);
  s1 ^= dpp_xor2(s1);
  s0 ^= dpp_ror4(s0);
  s1 ^= dpp_ror4(s1);
  s0 ^= dpp_ror8(s0);
  s1 ^= dpp_ror8(s1);
  if constexpr (QB == 1) {
    s0 = nib_map<256u, 4u>(lds, s0, st2_base);
    s1 = nib_map<256u, 4u>(lds, s1, st2_base);
    s0 = xor_lanebit4(s0);
    s1 = xor_lanebit4(s1);
    s0 = xor_lanebit5(s0);
    s1 = xor_lanebit5(s1);
  }
}

// QB = 4 task: item group g = items [4g, 4g+4); quarter b <-> item 4g+b.  Only
// the group index is carried; per-quarter facts are re-derived (scalar loads)
// where needed, which keeps the task in a few SGPRs.
struct QuadTask {
  uint64_t g;
  uint32_t nvalid; // valid items in the group (0..4); 0 = no task
};

struct QuarterInfo {
  const uint8_t *p0;
  uint32_t len;
  uint32_t z;
  int64_t vstart; // 1 KiB window start relative to the item start (<= 0)
};

} // namespace rows

// QB = 1: rows of one item.  QB = 4: four items (<= 1 KiB each) per row.
// PAIR = 2: two rows computed together (two interleaved lookup chains).
// WAVES = wavefronts per (one-per-CU) workgroup; PAIR = 2 needs the larger
// register budget of 12 waves (3 per SIMD).
template <int QB, bool NT, int PAIR = 2, int ABL = 0, int WAVES = (PAIR == 2 ? 12 : 16)>
__global__ void __launch_bounds__(WAVES * 64, WAVES / 4) crc32_rows_kernel(ItemsArgs a) {
  using namespace rows;
  __shared__ __attribute__((aligned(16))) uint32_t s_lds[kLdsBytesV2 / 4];
  {
    const uint4 *src = a.lds_image;
    uint4 *dst = reinterpret_cast<uint4 *>(s_lds);
    for (uint32_t k = threadIdx.x; k < kLdsBytesV2 / 16; k += blockDim.x) dst[k] = src[k];
  }
  __syncthreads();
  const uint8_t *lds = reinterpret_cast<const uint8_t *>(s_lds);

  const uint32_t lane = threadIdx.x & 63u;
  const uint32_t lane4 = (lane & 31u) * 4u;
  const uint32_t lsel = lane4 | ((lane4 + 128u) << 8) | (1u << 16);
  const uint32_t hi = lane >> 4;               // quarter / row of 16 lanes after the transpose
  const uint32_t pofs = 16u * piece_of_lane(lane); // byte offset of this lane's piece in a quarter
  const uint32_t st1_base = kLdsST1 + lane4;
  const uint32_t st2_base = kLdsST2 + hi * 4u;
  const uint32_t wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  const uint32_t wpb = blockDim.x >> 6;
  const uint64_t nwaves = (uint64_t)gridDim.x * wpb;
  const uint64_t gw = (uint64_t)blockIdx.x * wpb + wave;
  const uint32_t mode = a.mode;

  auto synth = [&](uint64_t key, u32x4 (&buf)[4]) {
#pragma unroll
    for (int b = 0; b < 4; ++b) {
      const uint32_t v = (uint32_t)key * 0x9E3779B1u + (uint32_t)b * 0x85EBCA6Bu + lane;
      buf[b] = u32x4{v, v ^ 0x5bd1e995u, v + 0x68e31da4u, ~v};
    }
  };
  auto chain1 = [&](const u32x4 (&buf)[4]) -> uint32_t {
    if constexpr ((ABL & kRowsAblNoCompute) != 0) return xor_fold(buf);
    else return seg_crc(lds, buf, lsel);
  };
  auto chain2 = [&](const u32x4 (&p)[4], const u32x4 (&q)[4], uint32_t &s0, uint32_t &s1) {
    if constexpr ((ABL & kRowsAblNoCompute) != 0) {
      s0 = xor_fold(p);
      s1 = xor_fold(q);
    } else {
      seg_crc2(lds, p, q, lsel, s0, s1);
    }
  };
  auto do_merge1 = [&](uint32_t s) -> uint32_t {
    if constexpr ((ABL & kRowsAblNoMerge) != 0) return s;
    else return merge<QB>(lds, s, st1_base, st2_base);
  };
  auto do_merge2 = [&](uint32_t &s0, uint32_t &s1) {
    if constexpr ((ABL & kRowsAblNoMerge) == 0) merge2<QB>(lds, s0, s1, st1_base, st2_base);
  };

  // ---- task policies ----------------------------------------------------------
  // QB = 1
  auto load_item = [&](uint64_t item, RowTask &t) {
    for (;;) {
      if (item >= a.n_items) {
        t.valid = 0u;
        return;
      }
      const uint64_t off = a.offsets ? a.offsets[item] : item * a.stride;
      const uint32_t len = a.lengths ? a.lengths[item] : a.len;
      if (len == 0) {
        if (lane == 0) a.out[item] = 0u;
        item += nwaves;
        continue;
      }
      t.valid = 1u;
      t.item = item;
      t.p0 = a.base + off;
      t.len = len;
      t.z = (uint32_t)(0u - (uint32_t)(uintptr_t)(t.p0 + len)) & 15u;
      t.lp = (uint64_t)len + t.z;
      t.nrows = (uint32_t)((t.lp + kRow - 1) / kRow);
      t.r = 0;
      const uint32_t first = (uint32_t)(t.lp - (uint64_t)(t.nrows - 1) * kRow);
      t.w0 = (mode == kModeRaw) ? 0u : a.tq[first];
      return;
    }
  };
  // QB = 4
  const uint64_t ngroups = (a.n_items + 3) / 4;
  auto load_group = [&](uint64_t g, QuadTask &q) {
    q.g = g;
    q.nvalid = 0;
    if (g >= ngroups) return;
    const uint64_t left = a.n_items - 4 * g;
    q.nvalid = left >= 4 ? 4u : (uint32_t)left;
  };
  auto quarter = [&](const QuadTask &q, int b) -> QuarterInfo {
    QuarterInfo r;
    const uint64_t item = 4 * q.g + b;
    const bool ok = (uint32_t)b < q.nvalid;
    const uint64_t off = !ok ? 0 : a.offsets ? a.offsets[item] : item * a.stride;
    r.len = !ok ? 0u : a.lengths ? a.lengths[item] : a.len;
    r.p0 = a.base + off;
    r.z = (uint32_t)(0u - (uint32_t)(uintptr_t)(r.p0 + r.len)) & 15u;
    r.vstart = (int64_t)r.len + r.z - (int64_t)kQuarter;
    return r;
  };
  using Task = typename std::conditional<QB == 1, RowTask, QuadTask>::type;
  auto first_task = [&](Task &t) {
    if constexpr (QB == 1) load_item(gw, t);
    else load_group(gw, t);
  };
  auto valid = [&](const Task &t) -> bool {
    if constexpr (QB == 1) return t.valid != 0u;
    else return t.nvalid != 0u;
  };
  auto next_task = [&](const Task &c, Task &n) {
    if constexpr (QB == 1) {
      if (c.r + 1 < c.nrows) {
        n = c;
        n.r = c.r + 1;
      } else {
        load_item(c.item + nwaves, n);
      }
    } else {
      load_group(c.g + nwaves, n);
    }
  };
  auto row_start = [&](const RowTask &t) -> int64_t {
    return (int64_t)t.lp - (int64_t)(t.nrows - t.r) * (int64_t)kRow;
  };
  auto issue = [&](const Task &t, u32x4 (&buf)[4]) {
    if constexpr ((ABL & kRowsAblNoLoad) != 0) {
      if constexpr (QB == 1) synth(t.item * 131u + t.r, buf);
      else synth(t.g, buf);
    } else if constexpr (QB == 1) {
      const int64_t rs = row_start(t);
      if (rs >= 0) {
#pragma unroll
        for (int b = 0; b < 4; ++b) buf[b] = ld16<NT>(t.p0 + rs + b * kQuarter + pofs);
      } else {
#pragma unroll
        for (int b = 0; b < 4; ++b) {
          const int64_t v = rs + b * kQuarter + (int64_t)pofs;
          buf[b] = (v + 16 > 0) ? ld16<NT>(t.p0 + v) : u32x4{0u, 0u, 0u, 0u};
        }
      }
    } else {
#pragma unroll
      for (int b = 0; b < 4; ++b) {
        const QuarterInfo qi = quarter(t, b);
        const int64_t v = qi.vstart + (int64_t)pofs;
        buf[b] = (qi.len != 0 && v + 16 > 0) ? ld16<NT>(qi.p0 + v) : u32x4{0u, 0u, 0u, 0u};
      }
    }
  };
  // mask + transpose
  auto prep = [&](const Task &t, u32x4 (&buf)[4]) {
    if constexpr (QB == 1) {
      const int64_t rs = row_start(t);
      if (rs < 0 || (t.r + 1 == t.nrows && t.z != 0)) {
#pragma unroll
        for (int b = 0; b < 4; ++b) buf[b] = mask_piece(buf[b], rs + b * kQuarter + (int64_t)pofs, t.len);
      }
    } else {
#pragma unroll
      for (int b = 0; b < 4; ++b) {
        const QuarterInfo qi = quarter(t, b);
        if (qi.vstart < 0 || qi.z != 0) buf[b] = mask_piece(buf[b], qi.vstart + (int64_t)pofs, qi.len);
      }
    }
    transpose(buf);
  };
  uint32_t W = 0; // QB = 1 Horner accumulator (wave-uniform)
  auto finish = [&](const Task &t, uint32_t s) {
    if constexpr (QB == 1) {
      W = (t.r == 0) ? t.w0 : nib_map<64u, 2u>(lds, W, kLdsRW2);
      W ^= s;
      if (t.r + 1 == t.nrows) {
        uint32_t res = W;
        if (t.z != 0) res = nib_map<64u, 2u>(lds, res, kLdsZI2 + (t.z - 1u) * 512u);
        if (mode == kModeFinal) res = ~res;
        if (lane == 0) a.out[t.item] = res;
      }
    } else {
      uint32_t z = 0, len = 0;
#pragma unroll
      for (int b = 0; b < 4; ++b) {
        const QuarterInfo qi = quarter(t, b);
        if (hi == (uint32_t)b) {
          z = qi.z;
          len = qi.len;
        }
      }
      const uint32_t w0 = (mode == kModeRaw || len == 0) ? 0u : a.tq[len + z];
      uint32_t res = w0 ^ s;
      if (z != 0) res = nib_map<64u, 2u>(lds, res, kLdsZI2 + (z - 1u) * 512u);
      if (mode == kModeFinal) res = ~res;
      if (len == 0) res = 0u;
      if ((lane & 15u) == 0 && hi < t.nvalid) a.out[4 * t.g + hi] = res;
    }
  };

  if constexpr (PAIR == 1) {
    Task cur, nxt;
    u32x4 bufA[4], bufB[4];
    first_task(cur);
    if (valid(cur)) issue(cur, bufA);
    auto step = [&](u32x4 (&cb)[4], u32x4 (&nb)[4]) {
      next_task(cur, nxt);
      if (valid(nxt)) issue(nxt, nb);
      prep(cur, cb);
      finish(cur, do_merge1(chain1(cb)));
      cur = nxt;
    };
    for (;;) {
      if (!valid(cur)) break;
      step(bufA, bufB);
      if (!valid(cur)) break;
      step(bufB, bufA);
    }
  } else {
    // Two rows per step; the next two rows load while these two compute.
    Task c0, c1, n0, n1;
    u32x4 A0[4], A1[4], B0[4], B1[4];
    first_task(c0);
    if (valid(c0)) {
      issue(c0, A0);
      next_task(c0, c1);
      if (valid(c1)) issue(c1, A1);
    } else {
      c1 = c0;
    }
    auto step = [&](u32x4 (&p0)[4], u32x4 (&p1)[4], u32x4 (&q0)[4], u32x4 (&q1)[4]) {
      if (valid(c1)) {
        next_task(c1, n0);
        if (valid(n0)) {
          issue(n0, q0);
          next_task(n0, n1);
          if (valid(n1)) issue(n1, q1);
        } else {
          n1 = n0;
        }
      } else {
        n0 = c1;
        n1 = c1;
      }
      prep(c0, p0);
      prep(c1, p1);
      uint32_t s0, s1;
      chain2(p0, p1, s0, s1);
      do_merge2(s0, s1);
      finish(c0, s0);
      if (valid(c1)) finish(c1, s1);
      c0 = n0;
      c1 = n1;
    };
    for (;;) {
      if (!valid(c0)) break;
      step(A0, A1, B0, B1);
      if (!valid(c0)) break;
      step(B0, B1, A0, A1);
    }
  }
}

} // namespace rpccrc
