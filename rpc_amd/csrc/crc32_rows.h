// rpc_amd/csrc/crc32_rows.h -- batched CRC-32 kernel v2 ("rows" kernel), device code.
//
// A wavefront processes ROWS of 4 KiB.  Row layout in registers:
//   load:      4 coalesced global_load_dwordx4 (optionally non-temporal); load
//              b covers the 1 KiB quarter b of the row, lane L its 16-B piece L
//              -> piece q = 64b + L sits in (slot b, lane L).
//   transpose: two DPP lane-pair exchanges (slot bit0 <-> lane bit0, slot bit1
//              <-> lane bit1) move piece q to (slot q&3, lane 4*((q>>2)&15) +
//              (q>>8... )), i.e. lane' = 4*lo + hi holds the contiguous 64-B
//              segment s = 16*hi + lo of the row, slots in byte order.
//   chain:     16 slice-by-4 steps per lane (v_perm_b32 address + 4 ds_read_b32,
//              bank-conflict-free through 32 replicated copies).
//   merge:     crc0(row) = XOR_s A_{64*(63-s)} c_s
//                        = XOR_lo A_{64*(15-lo)} XOR_hi A_{1024*(3-hi)} c_{hi,lo}
//              -> hi step (SH nibble table), DPP quad reduce, lo step (SL nibble
//              table), DPP row_ror reduce + 2 cross-row swizzles.
// QB = 1: the row is 4 KiB of one item (items of any length, end-aligned rows,
//         Horner across rows, Tq pre-conditioning, ZI trailing-pad undo).
// QB = 4: the row is four items of <= 1 KiB each (one per quarter; hi = item),
//         the hi step is skipped.
//
// LDS image (crc32_layout.h, v2):
//   MAIN [0,128K)  slice-by-4 tables x32 copies (as v1)
//   SH   16 KiB    SH[n][nib][c]  = A_{1024*(3-(c&3))}(nib<<4n), c = lane&31
//   SL   8 KiB     SL[n][nib][lo] = A_{64*(15-lo)}(nib<<4n), lo = 0..15
//   RW   512 B     RW[n][nib]     = A_4096(nib<<4n)
//   ZI   7.5 KiB   ZI[z-1][n][nib] = A_z^-1(nib<<4n)
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

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

// Exchange slot bit <-> lane bit between partner lanes (DPP): pairs (x, y)
// where x has slot bit 0 and y slot bit 1.  c = this lane's lane bit.
template <int XOR>
__device__ __forceinline__ void exch(u32x4 &x, u32x4 &y, bool c) {
#pragma unroll
  for (int d = 0; d < 4; ++d) {
    const uint32_t send = c ? x[d] : y[d];
    const uint32_t recv = (XOR == 1) ? dpp_xor1(send) : dpp_xor2(send);
    const uint32_t nx = c ? recv : x[d];
    const uint32_t ny = c ? y[d] : recv;
    x[d] = nx;
    y[d] = ny;
  }
}

// Transpose 4 slots x 64 lanes of 16-B pieces: see header comment.
__device__ __forceinline__ void transpose(u32x4 (&p)[4], uint32_t lane) {
  const bool l0 = (lane & 1u) != 0, l1 = (lane & 2u) != 0;
  exch<1>(p[0], p[1], l0);
  exch<1>(p[2], p[3], l0);
  exch<2>(p[0], p[2], l1);
  exch<2>(p[1], p[3], l1);
}

// crc0 contribution of this lane's 64-byte segment: 16 slice-by-4 steps.
__device__ __forceinline__ uint32_t seg_crc(const uint8_t *lds, const u32x4 (&p)[4], uint32_t lsel) {
  uint32_t x = p[0][0];
#pragma unroll
  for (int k = 0; k < 4; ++k)
#pragma unroll
    for (int d = 0; d < 4; ++d) {
      if (k == 0 && d == 0) continue;
      x = slice4(lds, x, lsel) ^ p[k][d];
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

// QB = 1: rows of one item.  QB = 4: four items (<= 1 KiB each) per row.
template <int QB, bool NT>
__global__ void __launch_bounds__(1024, 4) crc32_rows_kernel(ItemsArgs a) {
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
  const uint32_t hi = lane & 3u;
  const uint32_t lo = lane >> 2;
  const uint32_t sh_base = kLdsSH + lane4;
  const uint32_t sl_base = kLdsSL + lo * 4u;
  const uint32_t wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  const uint32_t wpb = blockDim.x >> 6;
  const uint64_t nwaves = (uint64_t)gridDim.x * wpb;
  const uint64_t gw = (uint64_t)blockIdx.x * wpb + wave;
  const uint32_t mode = a.mode;

  if constexpr (QB == 1) {
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
    auto next_task = [&](const RowTask &c, RowTask &n) {
      if (c.r + 1 < c.nrows) {
        n = c;
        n.r = c.r + 1;
      } else {
        load_item(c.item + nwaves, n);
      }
    };
    auto row_start = [&](const RowTask &t) -> int64_t {
      return (int64_t)t.lp - (int64_t)(t.nrows - t.r) * (int64_t)kRow;
    };
    auto issue = [&](const RowTask &t, u32x4 (&buf)[4]) {
      const int64_t rs = row_start(t);
      if (rs >= 0) {
#pragma unroll
        for (int b = 0; b < 4; ++b) buf[b] = ld16<NT>(t.p0 + rs + b * kQuarter + 16 * lane);
      } else {
#pragma unroll
        for (int b = 0; b < 4; ++b) {
          const int64_t v = rs + b * kQuarter + 16 * (int64_t)lane;
          buf[b] = (v + 16 > 0) ? ld16<NT>(t.p0 + v) : u32x4{0u, 0u, 0u, 0u};
        }
      }
    };
    uint32_t W = 0;
    auto compute = [&](const RowTask &t, u32x4 (&buf)[4]) {
      const int64_t rs = row_start(t);
      const bool last = t.r + 1 == t.nrows;
      if (rs < 0 || (last && t.z != 0)) {
#pragma unroll
        for (int b = 0; b < 4; ++b) buf[b] = mask_piece(buf[b], rs + b * kQuarter + 16 * (int64_t)lane, t.len);
      }
      transpose(buf, lane);
      uint32_t s = seg_crc(lds, buf, lsel);
      s = nib_map<2048u, 7u>(lds, s, sh_base); // A_{1024*(3-hi)}
      s ^= dpp_xor1(s);
      s ^= dpp_xor2(s);
      s = nib_map<1024u, 6u>(lds, s, sl_base); // A_{64*(15-lo)}
      s ^= dpp_ror4(s);
      s ^= dpp_ror8(s);
      s ^= swz_xor16(s);
      s ^= shfl_xor32(s);
      W = (t.r == 0) ? t.w0 : nib_map<64u, 2u>(lds, W, kLdsRW2);
      W ^= s;
      if (last) {
        uint32_t res = W;
        if (t.z != 0) res = nib_map<64u, 2u>(lds, res, kLdsZI2 + (t.z - 1u) * 512u);
        if (mode == kModeFinal) res = ~res;
        if (lane == 0) a.out[t.item] = res;
      }
    };
    RowTask cur, nxt;
    u32x4 bufA[4], bufB[4];
    load_item(gw, cur);
    if (cur.valid) issue(cur, bufA);
    for (;;) {
      if (!cur.valid) break;
      next_task(cur, nxt);
      if (nxt.valid) issue(nxt, bufB);
      compute(cur, bufA);
      cur = nxt;
      if (!cur.valid) break;
      next_task(cur, nxt);
      if (nxt.valid) issue(nxt, bufA);
      compute(cur, bufB);
      cur = nxt;
    }
  } else {
    // QB == 4: item group g = items [4g, 4g+4); quarter b <-> item 4g+b (len <= 1 KiB).
    struct Quad {
      const uint8_t *wnd[4]; // 1 KiB window start (16-B aligned) per quarter
      int64_t vstart[4];     // window start relative to the item start (<= 0)
      uint32_t len[4];
      uint32_t z[4];
      uint32_t w0[4];
      uint32_t nvalid;       // number of valid items in the group (0..4)
      uint64_t g;
    };
    const uint64_t ngroups = (a.n_items + 3) / 4;
    auto load_group = [&](uint64_t g, Quad &q) {
      q.g = g;
      q.nvalid = 0;
      if (g >= ngroups) return;
#pragma unroll
      for (int b = 0; b < 4; ++b) {
        const uint64_t item = 4 * g + b;
        uint32_t len = 0;
        uint64_t off = 0;
        if (item < a.n_items) {
          off = a.offsets ? a.offsets[item] : item * a.stride;
          len = a.lengths ? a.lengths[item] : a.len;
          q.nvalid = b + 1;
        }
        const uint8_t *p0 = a.base + off;
        const uint32_t z = (uint32_t)(0u - (uint32_t)(uintptr_t)(p0 + len)) & 15u;
        q.len[b] = len;
        q.z[b] = z;
        q.vstart[b] = (int64_t)len + z - (int64_t)kQuarter;
        q.wnd[b] = p0 + q.vstart[b];
        q.w0[b] = (mode == kModeRaw || len == 0) ? 0u : a.tq[len + z];
      }
    };
    auto issue = [&](const Quad &q, u32x4 (&buf)[4]) {
#pragma unroll
      for (int b = 0; b < 4; ++b) {
        const int64_t v = q.vstart[b] + 16 * (int64_t)lane;
        buf[b] = ((uint32_t)b < q.nvalid && q.len[b] != 0 && v + 16 > 0) ? ld16<NT>(q.wnd[b] + 16 * lane)
                                                                          : u32x4{0u, 0u, 0u, 0u};
      }
    };
    auto compute = [&](const Quad &q, u32x4 (&buf)[4]) {
#pragma unroll
      for (int b = 0; b < 4; ++b)
        if (q.vstart[b] < 0 || q.z[b] != 0)
          buf[b] = mask_piece(buf[b], q.vstart[b] + 16 * (int64_t)lane, q.len[b]);
      transpose(buf, lane);
      uint32_t s = seg_crc(lds, buf, lsel);
      s = nib_map<1024u, 6u>(lds, s, sl_base); // A_{64*(15-lo)}
      s ^= dpp_ror4(s);
      s ^= dpp_ror8(s);
      s ^= swz_xor16(s);
      s ^= shfl_xor32(s);
      // lanes with hi = b now hold crc0 of item 4g+b
      const uint32_t w0 = hi == 0 ? q.w0[0] : hi == 1 ? q.w0[1] : hi == 2 ? q.w0[2] : q.w0[3];
      const uint32_t z = hi == 0 ? q.z[0] : hi == 1 ? q.z[1] : hi == 2 ? q.z[2] : q.z[3];
      const uint32_t len = hi == 0 ? q.len[0] : hi == 1 ? q.len[1] : hi == 2 ? q.len[2] : q.len[3];
      uint32_t res = w0 ^ s;
      if (z != 0) res = nib_map<64u, 2u>(lds, res, kLdsZI2 + (z - 1u) * 512u);
      if (mode == kModeFinal) res = ~res;
      if (len == 0) res = 0u;
      if (lane < q.nvalid) a.out[4 * q.g + lane] = res;
    };
    Quad cur, nxt;
    u32x4 bufA[4], bufB[4];
    load_group(gw, cur);
    if (cur.nvalid) issue(cur, bufA);
    for (;;) {
      if (!cur.nvalid) break;
      load_group(cur.g + nwaves, nxt);
      if (nxt.nvalid) issue(nxt, bufB);
      compute(cur, bufA);
      cur = nxt;
      if (!cur.nvalid) break;
      load_group(cur.g + nwaves, nxt);
      if (nxt.nvalid) issue(nxt, bufA);
      compute(cur, bufB);
      cur = nxt;
    }
  }
}

} // namespace rpccrc
