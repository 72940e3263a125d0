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
//              hi = L' >> 4 (the quarter), lo = L' & 15.  Step 1 (per lane):
//              ST1 shift, 8 lookups each formed by ONE v_perm_b32 from the
//              even/odd nibble vectors; DPP quad + row_ror XOR over lo.
//              Step 2 (values now uniform per 16-lane row): "distributed" --
//              lane lo < 8 looks up nibble lo of its row's value in ST2, and in
//              the same ds_read lanes 8..15 of row 0 look up the nibbles of the
//              running item CRC W in RW (Horner A_4096); DPP + permlane-swap
//              reductions, readlane 4 / 12 -> crc0(row), A_4096(W) as SGPRs.
//              Seeds A_first(0xFFFFFFFF) are scalar loads from the global Tq
//              table; the trailing-pad undo ZI is another distributed step.
// QB = 1: the row is 4 KiB of one item (items of any length, end-aligned rows,
//         Horner across rows with RW, Tq pre-conditioning, ZI trailing-pad undo).
// QB = 4: the row holds four items of <= 1 KiB each (item = quarter = hi), so
//         the merge stops after the lo reduction (no ST2 step).
//
// LDS image (crc32_layout.h "v3"):
//   MAIN [0,128K)  slice-by-4 tables x32 copies (two tables per 256-B row)
//   ST1  16 KiB    A_{64*(15-(c&15))}(nib<<4n), c = lane&31, perm-addressable
//   ST2  2 KiB     ST2(n, nib, hi) = A_{1024*(3-hi)}(nib<<4n), one bank per (n, hi) (st2_byte)
//   RW   512 B     RW[n][nib]      = A_4096(nib<<4n)
//   ZI   7.5 KiB   ZI[z-1][n][nib] = A_z^-1(nib<<4n)
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

#include <type_traits>

#include "crc32_edge.h"
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


// DPP lane moves (all lanes active, every source valid).  bound_ctrl is set
// even where every source lane is valid: only then does the DPP combiner fold
// the move into the consuming v_xor (one VALU instead of two).
__device__ __forceinline__ uint32_t dpp_xor1(uint32_t v) { // quad_perm [1,0,3,2]
  return (uint32_t)__builtin_amdgcn_mov_dpp((int)v, 0xB1, 0xF, 0xF, true);
}
__device__ __forceinline__ uint32_t dpp_xor2(uint32_t v) { // quad_perm [2,3,0,1]
  return (uint32_t)__builtin_amdgcn_mov_dpp((int)v, 0x4E, 0xF, 0xF, true);
}
__device__ __forceinline__ uint32_t dpp_ror4(uint32_t v) { // row_ror:4
  return (uint32_t)__builtin_amdgcn_mov_dpp((int)v, 0x124, 0xF, 0xF, true);
}
__device__ __forceinline__ uint32_t dpp_ror8(uint32_t v) { // row_ror:8
  return (uint32_t)__builtin_amdgcn_mov_dpp((int)v, 0x128, 0xF, 0xF, true);
}
__device__ __forceinline__ uint32_t dpp_shr4(uint32_t v) { // row_shr:4, zeros shifted in
  return (uint32_t)__builtin_amdgcn_mov_dpp((int)v, 0x114, 0xF, 0xF, true);
}
__device__ __forceinline__ uint32_t swz_xor16(uint32_t v) { // ds_swizzle bit mode, xor 16
  return (uint32_t)__builtin_amdgcn_ds_swizzle((int)v, 0x401F);
}
__device__ __forceinline__ uint32_t shfl_xor32(uint32_t v) {
  return (uint32_t)__shfl_xor((int)v, 32, 64);
}

typedef unsigned int u32x4 __attribute__((ext_vector_type(4)));

// 16-byte global load.  The pointer is cast to the global address space so a
// selected / integer-derived address still compiles to global_load (in-order
// vmcnt accounting) rather than flat_load (which also ties up lgkmcnt).
template <bool NT>
__device__ __forceinline__ u32x4 ld16(const uint8_t *p) {
  const __attribute__((address_space(1))) u32x4 *q = (const __attribute__((address_space(1))) u32x4 *)(p);
  if constexpr (NT)
    return __builtin_nontemporal_load(q);
  else
    return *q;
}

// 16-byte load from a wave-uniform base plus a 32-bit per-lane offset, as a
// raw buffer load: the base lives in an SGPR descriptor (2 SALU to build), the
// lane offset in a VGPR and the quarter offset in the immediate -- no 64-bit
// per-lane address arithmetic per row (a global_load shared with the masked
// path was compiled with per-lane 64-bit addresses).  aux 2 = nt.
// Descriptor range: offsets >= kRsrcRange fail the raw-buffer range check and
// read as zeros WITHOUT a memory access; kOobOffset is such an offset.  Every
// in-range offset of the kernels is below 8 KiB.
constexpr uint32_t kRsrcRange = 0x40000000u;
constexpr uint32_t kOobOffset = 0x7FFFFFF0u;
static_assert(kOobOffset >= kRsrcRange, "the out-of-range offset must fail the range check");
// Flags 0x00020000: DATA_FORMAT 32 (a descriptor with format 0, "invalid",
// reads zeros).
__device__ __forceinline__ __amdgpu_buffer_rsrc_t row_rsrc(uint64_t base, uint32_t range = kRsrcRange) {
  return __builtin_amdgcn_make_buffer_rsrc(reinterpret_cast<void *>(base), (short)0, (int)range, 0x00020000);
}
// Cache-policy bits of the non-temporal row loads (the builtin's aux operand;
// 2 = nt).  RPCCRC_ROW_AUX overrides them for A/B builds only: sc0|nt, sc1|nt
// and sc0|sc1|nt measured the same as nt on NS and C2, sc1 alone +11 % / +6 %
// (profiles/r05n/row_load_cache_policy_ab.txt).
#ifndef RPCCRC_ROW_AUX
#define RPCCRC_ROW_AUX 2
#endif
template <bool NT>
__device__ __forceinline__ u32x4 ldb16(__amdgpu_buffer_rsrc_t rsrc, uint32_t off) {
  return __builtin_amdgcn_raw_buffer_load_b128(rsrc, (int)off, 0, NT ? RPCCRC_ROW_AUX : 0);
}
// A 16-B piece at signed offset `off` from a uniform base; pieces with off < 0
// (before the data) are not read at all and come back as zeros: their offset
// is replaced by one past the descriptor's range (raw buffer range check).
template <bool NT>
__device__ __forceinline__ u32x4 ldb16_or_zero(__amdgpu_buffer_rsrc_t rsrc, int32_t off) {
  return __builtin_amdgcn_raw_buffer_load_b128(rsrc, (int)min((uint32_t)off, kOobOffset), 0, NT ? RPCCRC_ROW_AUX : 0);
}

// Edge fix of one quarter of 16-B pieces (replaces a per-lane byte mask of
// every piece: ~250 VALU per partial row, measured on 1M x 3 KiB bodies).
// Pieces wholly before the body already read as zeros (out-of-range loads),
// so only two pieces of a window can hold foreign bytes: the one holding the
// body's first byte (window offset `front`, its front & 15 leading bytes are
// foreign) and the window's last piece when it ends in the z pad (its last z
// bytes).  `front` >= 1024 (or a multiple of 16) and z = 0 disable a fix.
// x & (m | e) in one v_bitop3_b32 (truth table 0xE0): m is the scalar dword
// mask, e is all-ones in every lane but the edge lane.
__device__ __forceinline__ uint32_t and_or_keep(uint32_t x, uint32_t m, uint32_t e) {
  return __builtin_amdgcn_bitop3_b32(x, m, e, 0xE0);
}
template <bool NATURAL = false>
__device__ __forceinline__ void fix_quarter(u32x4 &x, uint32_t lane, uint32_t front, uint32_t z) {
  auto lane_of = [](uint32_t p) { return NATURAL ? p : lane_of_piece(p); };
  if ((front & 15u) != 0u && front < 1024u) {
    const uint32_t e = (lane == lane_of(front >> 4)) ? 0u : 0xFFFFFFFFu;
    const uint32_t f = front & 15u;
#pragma unroll
    for (uint32_t d = 0; d < 4; ++d) x[d] = and_or_keep(x[d], keep_front_dword(f, d), e);
  }
  if (z != 0u) {
    const uint32_t e = (lane == lane_of(63u)) ? 0u : 0xFFFFFFFFu;
#pragma unroll
    for (uint32_t d = 0; d < 4; ++d) x[d] = and_or_keep(x[d], keep_end_dword(16u - z, d), e);
  }
}

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

// Two independent chains per lane (kTwoChains): a = crc0 of the segment's
// first 32 bytes (slots 0, 1), b = crc0 of its last 32 bytes (slots 2, 3).
// Their LDS round trips interleave, so a segment costs 8 dependent steps
// instead of 16 (the chain is latency-bound: 4 waves per SIMD).
struct Seg2 {
  uint32_t a, b;
};
__device__ __forceinline__ Seg2 seg_crc2(const uint8_t *lds, const u32x4 (&p)[4], uint32_t lsel) {
  uint32_t xa = p[0][0], xb = p[2][0];
#pragma unroll
  for (int k = 0; k < 2; ++k)
#pragma unroll
    for (int d = 0; d < 4; ++d) {
      if (k == 0 && d == 0) continue;
      xa = slice4w(lds, xa, p[k][d], lsel);
      xb = slice4w(lds, xb, p[k + 2][d], lsel);
    }
  return Seg2{slice4(lds, xa, lsel), slice4(lds, xb, lsel)};
}

// The value of lane L ^ 16 (swap across lane bit 4), `upper` = lane & 16.
__device__ __forceinline__ uint32_t swap_lanebit4(uint32_t v, bool upper) {
  auto a = __builtin_amdgcn_permlane16_swap(v, v, false, false);
  return upper ? a[0] : a[1];
}

// Workgroup copy of the kBytes LDS table image (1024 threads) from its HBM
// form (crc32_layout.h kImgCompact): img_load issues all of a thread's global
// loads at once into registers, img_store writes LDS.  Compact form: the
// thread's 8 MAIN pieces (16 B = 4 copies of one table word each; lanes of a
// wave write consecutive pieces, so the stores are bank-conflict-free) come
// from 8 dword loads of the 4 KiB single-copy tables, the rest of the image is
// copied.  Whole iterations and the partial one are separate so every value
// stays in a register (a conditionally written local array went to scratch:
// 176 B per lane, the image loaded twice).
template <uint32_t kBytes>
struct ImgRegs {
  static constexpr uint32_t kTail = (kBytes - kLdsST1) / 16, kTailIt = (kTail + 1023) / 1024; // compact
  static constexpr uint32_t kFull = kBytes / 16 / 1024, kRem = (kBytes / 16) % 1024;          // full
  uint32_t t[kImgCompact ? 8 : 1];
  u32x4 p[kImgCompact ? kTailIt : kFull + 1];
};
template <uint32_t kBytes>
__device__ __forceinline__ void img_load(const uint4 *src, ImgRegs<kBytes> &r) {
  using R = ImgRegs<kBytes>;
  const uint32_t tid = threadIdx.x;
  if constexpr (kImgCompact) {
    const uint32_t *w = reinterpret_cast<const uint32_t *>(src);
#pragma unroll
    for (uint32_t k = 0; k < 8; ++k) { // MAIN piece q: region q >> 12, row (q >> 4) & 255, half (q >> 3) & 1
      const uint32_t q = tid + 1024u * k;
      r.t[k] = w[(((q >> 12) << 1) | ((q >> 3) & 1u)) * 256u + ((q >> 4) & 255u)];
    }
    const u32x4 *tail = reinterpret_cast<const u32x4 *>(reinterpret_cast<const uint8_t *>(src) + kImgTailOfs);
#pragma unroll
    for (uint32_t i = 0; i < R::kTailIt; ++i) {
      const uint32_t q = tid + 1024u * i;
      r.p[i] = (i + 1 < R::kTailIt || q < R::kTail) ? tail[q] : u32x4{0u, 0u, 0u, 0u};
    }
  } else {
    const u32x4 *s4 = reinterpret_cast<const u32x4 *>(src);
#pragma unroll
    for (uint32_t i = 0; i < R::kFull; ++i) r.p[i] = s4[tid + i * 1024u];
    r.p[R::kFull] = (R::kRem != 0 && tid < R::kRem) ? s4[R::kFull * 1024u + tid] : u32x4{0u, 0u, 0u, 0u};
  }
}
template <uint32_t kBytes>
__device__ __forceinline__ void img_store(const ImgRegs<kBytes> &r, uint32_t *lds) {
  using R = ImgRegs<kBytes>;
  const uint32_t tid = threadIdx.x;
  u32x4 *d4 = reinterpret_cast<u32x4 *>(lds);
  if constexpr (kImgCompact) {
#pragma unroll
    for (uint32_t k = 0; k < 8; ++k) d4[tid + 1024u * k] = u32x4{r.t[k], r.t[k], r.t[k], r.t[k]};
#pragma unroll
    for (uint32_t i = 0; i < R::kTailIt; ++i) {
      const uint32_t q = tid + 1024u * i;
      if (i + 1 < R::kTailIt || q < R::kTail) d4[kLdsST1 / 16u + q] = r.p[i];
    }
  } else {
#pragma unroll
    for (uint32_t i = 0; i < R::kFull; ++i) d4[tid + i * 1024u] = r.p[i];
    if (R::kRem != 0 && tid < R::kRem) d4[R::kFull * 1024u + tid] = r.p[R::kFull];
  }
}
template <uint32_t kBytes>
__device__ __forceinline__ void copy_lds_image(const uint4 *src, uint32_t *dst) {
  ImgRegs<kBytes> r;
  img_load<kBytes>(src, r);
  img_store<kBytes>(r, dst);
}

// Read-only kernel inputs through the constant address space: uniform indices
// then compile to scalar loads (s_load, counted by lgkmcnt) instead of vector
// loads that would sit in the vmcnt queue in front of the row prefetch.
template <typename T>
__device__ __forceinline__ T ld_const(const T *p, uint64_t i) {
  return ((const __attribute__((address_space(4))) T *)(p))[i];
}

// Per-lane ST1 step A_{64*(15-lo)}(s): the nibbles of s are split into two
// byte vectors (even / odd nibbles) so that ONE v_perm_b32 per lookup forms
// the address {copy | (nibble << 8) | (2 << 16)} exactly like the main tables
// (ST1 sits at 2 << 16); the nibble pair index rides in the immediate offset.
__device__ __forceinline__ uint32_t st1_map(const uint8_t *lds, uint32_t s, uint32_t lsel1) {
  const uint32_t xl = s & 0x0F0F0F0Fu, xh = (s >> 4) & 0x0F0F0F0Fu;
  uint32_t t[8];
#pragma unroll
  for (uint32_t k = 0; k < 4; ++k) {
    t[2 * k] = lds_ld(lds, __builtin_amdgcn_perm(xl, lsel1, 0x0C020400u + (k << 8)) + k * 4096u);
    t[2 * k + 1] = lds_ld(lds, __builtin_amdgcn_perm(xh, lsel1, 0x0C020401u + (k << 8)) + k * 4096u);
  }
  return xor3(xor3(t[0], t[1], t[2]), xor3(t[3], t[4], t[5]), t[6] ^ t[7]);
}

// "Distributed" nibble steps for values that are uniform over a 16-lane row
// (or the whole wave): lane n = lane & 7 of the row looks up nibble n only, one
// ds_read per lane instead of eight, and a 3-step DPP XOR (quad xor1, xor2,
// row_shr 4) leaves the 8-lane sums in lanes 4..7 (and 12..15) of each row.
__device__ __forceinline__ uint32_t dist_reduce8(uint32_t t) {
  t ^= dpp_xor1(t);
  t ^= dpp_xor2(t);
  return t ^ dpp_shr4(t);
}

// Per-lane constants of the distributed steps (computed once per kernel).
struct DistLane {
  uint32_t shift;  // 4 * (lane & 7): which nibble this lane looks up
  uint32_t n64;    // (lane & 7) * 64: nibble-table row ([n][nib] tables, 64 B per n)
  uint32_t row_base; // merge step: lo < 8 -> st2_byte(lo, 0, hi); hi == 0, lo >= 8 -> RW2 + (lo-8)*64; else kLdsZero
  uint32_t row_mul;  // merge step: nibble stride (128 for ST2, 4 for RW2, 0 for the zero lanes)
  bool own;          // merge step: lane looks up its own row's value (lo < 8)
};

__device__ __forceinline__ DistLane dist_lane(uint32_t lane) {
  DistLane d;
  const uint32_t lo = lane & 15u, hi = lane >> 4;
  d.shift = 4u * (lane & 7u);
  d.n64 = (lane & 7u) * 64u;
  d.own = lo < 8u;
  d.row_base = d.own ? st2_byte(lo, 0u, hi) : (hi == 0u ? kLdsRW2 + (lo - 8u) * 64u : kLdsZero);
  d.row_mul = d.own ? st2_byte(0u, 1u, 0u) - st2_byte(0u, 0u, 0u) : (hi == 0u ? 4u : 0u);
  return d;
}

// Nibble map of a wave-uniform value u by a [n][nib] table at `table`
// (RW2 / ZI2 layout); result is wave-uniform (read from lane 4).
__device__ __forceinline__ uint32_t dist_uniform(const uint8_t *lds, uint32_t u, uint32_t table, const DistLane &d) {
  const uint32_t nib = (u >> d.shift) & 15u;
  const uint32_t t = dist_reduce8(lds_ld(lds, table + d.n64 + nib * 4u));
  return (uint32_t)__builtin_amdgcn_readlane((int)t, 4);
}

} // namespace rows

// Ablation bits (measurement builds in tools/probe_kernels.hip only; product = 0).
constexpr int kRowsAblNoCompute = 1; // XOR fold instead of the slice-by-4 chain
constexpr int kRowsAblNoMerge = 2;   // skip the per-lane shift / reductions
constexpr int kRowsAblNoLoad = 4;    // synthesize row data instead of loading it
constexpr int kRowsAblNaturalOrder = 8; // lane L loads piece L (timing only: wrong CRCs)
constexpr int kRowsAblNoStore = 16;     // results never stored (timing / codegen only)
constexpr int kRowsAblNoTranspose = 32; // skip the permlane transposes (timing only)
constexpr int kRowsAblLdsSeed = 64;     // QB = 1 seeds from LDS TQ16 (+ ZI) instead of scalar loads (exact)
constexpr int kRowsAblNoFastLoad = 128; // always the per-lane address path (exact)
constexpr int kRowsAblNoImage = 256;    // no LDS image copy (timing only; with NoCompute|NoMerge)
// Per-wave timeline (exact results): s_memrealtime (100 MHz) at entry, after
// the LDS image, and at exit, stored by lane 0 at times[4*gw + 0..2] together
// with the wave's task count; times = a.offsets (unused by uniform batches).
constexpr int kRowsAblTimes = 512;
constexpr int kRowsAblNtStore = 2048; // non-temporal CRC stores (DYN paths; exact)
// Chain only slots 2-3 (8 slice-by-4 steps per lane, the last 2 KiB of the row):
// the instruction cost of a half-width row (timing only: wrong CRCs).
constexpr int kRowsAblHalfChain = 8192;
constexpr int kRowsAblNoSub = 16384; // ragged QB = 1 without the quarter / half first rows (exact)
// Ragged QB = 1 lane-Horner pipeline (the C2 loop: loads two rows ahead) with
// the chain, the per-lane Horner and the merge replaced by an XOR fold: its
// memory stream and control path alone (timing only: wrong CRCs).
constexpr int kRowsAblPipeMem = 65536;
// Feature bit (product, not an ablation): uniform QB = 1 DYN launches of
// 4096-byte RAW items also store each whole round's crc0 -- the 32 items as one
// 128 KiB run -- at a.round_out[round] (rpc_crc32_device_large's contiguous
// path folds those instead of the per-chunk CRCs).  The lane tree's maps
// A_{8 KiB .. 64 KiB} sit in the image's ZI slots z = 12..15 (kLdsRoundMaps),
// which such launches never read (16-byte aligned items of 4096 bytes have no
// trailing pad; the host requires the aligned base).
constexpr int kRowsRoundOut = 32768;
// Feature bit (product): the dense span pass (ItemsArgs.span_*).
// Uniform QB = 1 RAW rows over one stream of 4 KiB blocks (base and length
// from the plan's DenseCtl, the last block range-checked at the stream's end);
// a block whose record lists body boundaries also stores, per boundary, the
// in-quarter prefix P1, the chain state cap at the boundary's dword and the
// quarter prefix Qp (tests/test_dense_emu.py), from values the lanes hold.
constexpr int kRowsSpanBnd = 131072;
// A/B builds of the span pass: RPCCRC_SPAN_TWO_PHASE=1 runs it as two phases
// (the plain loop, then the pool loop) like host-counted stealing launches --
// 2.5 % SLOWER than the one loop (5817 vs 5675 us per C2 span pass, rocprof,
// rotated A/B, profiles/r06sp), where C3 gained 2.3 % from two phases;
// RPCCRC_SPAN_ABL=1 never takes the boundary path, 2 also skips the record
// load (timing only: wrong CRCs).
#ifndef RPCCRC_SPAN_TWO_PHASE
#define RPCCRC_SPAN_TWO_PHASE 0
#endif
#ifndef RPCCRC_SPAN_ABL
#define RPCCRC_SPAN_ABL 0
#endif
// QB = 1 software pipeline over rows (chain of row r+1 beside the merge of row r).
#ifndef RPCCRC_ROWS_PIPE
#define RPCCRC_ROWS_PIPE 1
#endif
constexpr bool kRowsPipe = RPCCRC_ROWS_PIPE != 0;
// Ragged QB = 1: first rows of <= 1 / 2 KiB as quarter / half rows (rows::quarter_row_segs,
// rows::half_row_segs).
#ifndef RPCCRC_SUBROWS
#define RPCCRC_SUBROWS 1
#endif
constexpr bool kSubRows = RPCCRC_SUBROWS != 0;
// Ragged QB = 1 pipeline: Horner across a body's rows per lane (rows::rw_map)
// and one merge per body, instead of a merge and a scalar Horner step per row.
// C2 -0.5 % on two boxes (profiles/r03o, r03p).
#ifndef RPCCRC_LANE_HORNER
#define RPCCRC_LANE_HORNER 1
#endif
constexpr bool kLaneHorner = RPCCRC_LANE_HORNER != 0;
// Ragged DYN QB = 1: tasks are groups of 4 items, and the group's items that
// fit a 1 KiB quarter share one row (round 5, crc32_rows_kernel kSB).  Exact
// (82 ragged / frames GPU tests green with it, profiles/r05m) but C2 ran 11 %
// SLOWER (6784 vs 6115 us, rotated A/B on one box): the extra row kind and the
// group state in the three unrolled pipeline steps took the kernel from 10 to
// 56 SGPR spills (~160 v_readlane per step) -- more than the 1.2M row steps it
// saves.  Off; kept as the measured alternative.
#ifndef RPCCRC_SMALL_GROUPS
#define RPCCRC_SMALL_GROUPS 0
#endif
// Ragged QB = 1: an item's offset and length loads issued together, then one
// wait (round 4).  The compiler had sunk the offset load below the length's
// route test: two serial scalar-load round trips per item (ISA).
#ifndef RPCCRC_META_COISSUE
#define RPCCRC_META_COISSUE 1
#endif
constexpr bool kMetaCoissue = RPCCRC_META_COISSUE != 0;
// Ragged QB = 1: zlib seeds from the LDS image (TQ16 + a distributed ZI step)
// instead of a scalar load of Tq[hd] per item.  Any scalar load in flight makes
// the chain's next LDS wait an lgkmcnt(0) (SMEM returns out of order), so the
// seed load issued with the next item's metadata stalled the current row's
// chain.
#ifndef RPCCRC_LDS_SEED
#define RPCCRC_LDS_SEED 0
#endif

namespace rows {

__device__ __forceinline__ uint32_t xor_fold(const u32x4 (&p)[4]) {
  uint32_t r = 0;
#pragma unroll
  for (int k = 0; k < 4; ++k) r ^= p[k][0] ^ p[k][1] ^ p[k][2] ^ p[k][3];
  return r;
}

// Merge step 1 (see header): ST1 per lane, then XOR over lo (lane bits 0-3).
// Every lane of 16-lane row hi then holds v_hi = crc0 of quarter hi.
__device__ __forceinline__ uint32_t merge_lo(const uint8_t *lds, uint32_t s, uint32_t lsel1) {
  s = st1_map(lds, s, lsel1); // A_{64*(15-lo)}
  s ^= dpp_xor1(s);
  s ^= dpp_xor2(s);
  s ^= dpp_ror4(s);
  return s ^ dpp_ror8(s);
}

// Merge step 1 for two chains: the segment's crc0 is A_{S+32}(a) ^ A_S(b),
// S = 64*(15-lo).  A lane reads ST1 only in its own bank (conflict-free), and
// bank c holds shift S + 32*((c >> 4) & 1): lanes with lane bit 4 clear hold
// S, their partners L ^ 16 (same lo) hold S + 32.  So each lane shifts its own
// value of its bank's kind and its partner's value of the same kind, then
// hands the partner's result back: two ST1 passes, two lane-bit-4 swaps.
__device__ __forceinline__ uint32_t merge_lo2(const uint8_t *lds, Seg2 c, uint32_t lsel1, bool upper) {
  const uint32_t own = upper ? c.a : c.b;
  const uint32_t other = swap_lanebit4(upper ? c.b : c.a, upper);
  const uint32_t t_own = st1_map(lds, own, lsel1);
  const uint32_t t_other = st1_map(lds, other, lsel1);
  uint32_t s = t_own ^ swap_lanebit4(t_other, upper);
  s ^= dpp_xor1(s);
  s ^= dpp_xor2(s);
  s ^= dpp_ror4(s);
  return s ^ dpp_ror8(s);
}

// Transposed row -> every lane of 16-lane row hi holds crc0 of quarter hi.
__device__ __forceinline__ uint32_t row_quarters(const uint8_t *lds, const u32x4 (&p)[4], uint32_t lsel,
                                                 uint32_t lsel1, bool upper) {
  if constexpr (kTwoChains) return merge_lo2(lds, seg_crc2(lds, p, lsel), lsel1, upper);
  else return merge_lo(lds, seg_crc(lds, p, lsel), lsel1);
}

// Merge step 2 for QB = 1 fused with the Horner step of the previous rows:
// one ds_read per lane serves both the per-quarter ST2 shift A_{1024*(3-hi)}
// of v_hi (lanes lo < 8, nibble lo) and RW(u) = A_4096(u) of the wave-uniform
// running CRC u (lanes 8..15 of row 0, nibble lo - 8); other lanes read zero.
// After dist_reduce8 and the hi reduction, lane 4 holds crc0(row) and lane 12
// holds A_4096(u).
struct RowMerge {
  uint32_t crc;  // crc0 of the 4 KiB row (uniform)
  uint32_t rwu;  // A_4096(u) (uniform)
};
__device__ __forceinline__ RowMerge merge_row(const uint8_t *lds, uint32_t v, uint32_t u, const DistLane &d) {
  const uint32_t src = d.own ? v : u;
  const uint32_t nib = (src >> d.shift) & 15u;
  uint32_t t = dist_reduce8(lds_ld(lds, d.row_base + nib * d.row_mul));
  t = xor_lanebit4(t);
  t = xor_lanebit5(t);
  RowMerge m;
  m.crc = (uint32_t)__builtin_amdgcn_readlane((int)t, 4);
  m.rwu = (uint32_t)__builtin_amdgcn_readlane((int)t, 12);
  return m;
}

// ---- sub-row first rows (ragged QB = 1; crc32_layout.h SQ) ----
// A body's first row holds its first hd <= 4096 bytes (end-aligned rows), so
// a first row of hd <= 1 KiB has data in load 3 only, and one of hd <= 2 KiB in
// loads 2 and 3; the pieces before the body read as zeros (out of range).  The
// full row spends 16 chain steps per lane on them anyway.  These variants
// spread the live bytes over all 64 lanes instead (4 or 8 chain steps), shift
// the pieces to their 64-B segment's end with one per-lane SQ lookup pass,
// and leave the full-row layout (lane L' = crc0 of 64-B segment L', zero for
// the empty segments), so merge_lo / merge_row are shared.  C2: 2.15M of its
// 12.47M rows are quarter rows and 0.85M half rows.
// s -> A_{16*(3-j)}(s), jb = (j * 64) * 0x01010101 (this lane's j):
// 8 lookups, each address one v_perm_b32 {byte j*64 + nib*4 | kLdsSQ}.
__device__ __forceinline__ uint32_t sq_map(const uint8_t *lds, uint32_t s, uint32_t jb) {
  const uint32_t xl4 = ((s << 2) & 0x3C3C3C3Cu) | jb, xh4 = ((s >> 2) & 0x3C3C3C3Cu) | jb;
  uint32_t t[8];
#pragma unroll
  for (uint32_t k = 0; k < 4; ++k) {
    t[2 * k] = lds_ld(lds, __builtin_amdgcn_perm(xl4, kLdsSQ, 0x0C020104u + k) + k * 512u);
    t[2 * k + 1] = lds_ld(lds, __builtin_amdgcn_perm(xh4, kLdsSQ, 0x0C020104u + k) + k * 512u + 256u);
  }
  return xor3(xor3(t[0], t[1], t[2]), xor3(t[3], t[4], t[5]), t[6] ^ t[7]);
}
// Quarter row: lane L holds piece 4*(L&15) + (L>>4) of the row's last 1 KiB
// (no transpose), i.e. 16-B piece hi = L>>4 of 64-B segment 48 + lo.  4 chain
// steps, A_{16*(3-hi)} to the segment's end, XOR over lane bits 4 and 5, and
// only row hi = 3 keeps it (m3: all-ones in lanes 48..63).
__device__ __forceinline__ uint32_t quarter_row_segs(const uint8_t *lds, const u32x4 (&p)[4], uint32_t lsel,
                                                     uint32_t jbq, uint32_t m3) {
  uint32_t x = p[3][0];
#pragma unroll
  for (int d = 1; d < 4; ++d) x = slice4w(lds, x, p[3][d], lsel);
  uint32_t a = sq_map(lds, slice4(lds, x, lsel), jbq);
  a = xor_lanebit4(a);
  a = xor_lanebit5(a);
  return a & m3;
}
// Half row: the transpose's permlane16 stage on slots (2, 3) only leaves lane
// L with the 32-B half (L >> 5) of 64-B segment 32 + (L & 31) in slots 2, 3.
// 8 chain steps; the first halves (lower lanes) are shifted by A_32 and moved
// to their upper partners by one permlane32_swap into a zero register:
// upper lanes (mU all-ones) end with c ^ A_32(c_partner), lower lanes with 0.
__device__ __forceinline__ uint32_t half_row_segs(const uint8_t *lds, u32x4 (&p)[4], uint32_t lsel, uint32_t mU) {
#pragma unroll
  for (int d = 0; d < 4; ++d) {
    auto b = __builtin_amdgcn_permlane16_swap(p[2][d], p[3][d], false, false);
    p[2][d] = b[0];
    p[3][d] = b[1];
  }
  uint32_t x = p[2][0];
#pragma unroll
  for (int k = 2; k < 4; ++k)
#pragma unroll
    for (int d = 0; d < 4; ++d) {
      if (k == 2 && d == 0) continue;
      x = slice4w(lds, x, p[k][d], lsel);
    }
  const uint32_t c = slice4(lds, x, lsel);
  const uint32_t a = sq_map(lds, c, 0x40404040u); // j = 1: A_32
  auto w = __builtin_amdgcn_permlane32_swap(0u, a, false, false); // w[0]: upper lanes <- a of lower lanes
  return __builtin_amdgcn_bitop3_b32(c, mU, w[0], 0x6A);          // (c & mU) ^ w
}

// Per-lane A_4096 (lane Horner, kLaneHorner): each lane advances its own
// segment accumulator by one row, from the single-copy RW table ([n][nib] at
// kLdsRW2 + n*64 + nib*4: the 16 words of one n sit on 16 banks, lanes with
// equal nibbles share a word).  One v_perm_b32 per address, n in the immediate.
__device__ __forceinline__ uint32_t rw_map(const uint8_t *lds, uint32_t s) {
  static_assert((kLdsRW2 & 255u) == 0, "RW must be 256-B aligned for the perm-formed address");
  const uint32_t xl4 = (s << 2) & 0x3C3C3C3Cu, xh4 = (s >> 2) & 0x3C3C3C3Cu;
  uint32_t t[8];
#pragma unroll
  for (uint32_t k = 0; k < 4; ++k) {
    t[2 * k] = lds_ld(lds, __builtin_amdgcn_perm(xl4, kLdsRW2, 0x0C020104u + k) + k * 128u);
    t[2 * k + 1] = lds_ld(lds, __builtin_amdgcn_perm(xh4, kLdsRW2, 0x0C020104u + k) + k * 128u + 64u);
  }
  return xor3(xor3(t[0], t[1], t[2]), xor3(t[3], t[4], t[5]), t[6] ^ t[7]);
}

// Per-lane A_{4096 * 2^l} (kRowsRoundOut's tree): l = 0 is rw_map; l = 1..4
// read the [n][nib] maps at kLdsRoundMaps + (l - 1) * 512 (same addressing).
template <uint32_t TAB>
__device__ __forceinline__ uint32_t nib_map_at(const uint8_t *lds, uint32_t s) {
  static_assert((TAB & 255u) == 0 && TAB < (1u << 24), "256-B aligned for the perm-formed address");
  const uint32_t xl4 = (s << 2) & 0x3C3C3C3Cu, xh4 = (s >> 2) & 0x3C3C3C3Cu;
  uint32_t t[8];
#pragma unroll
  for (uint32_t k = 0; k < 4; ++k) {
    t[2 * k] = lds_ld(lds, __builtin_amdgcn_perm(xl4, TAB, 0x0C020104u + k) + k * 128u);
    t[2 * k + 1] = lds_ld(lds, __builtin_amdgcn_perm(xh4, TAB, 0x0C020104u + k) + k * 128u + 64u);
  }
  return xor3(xor3(t[0], t[1], t[2]), xor3(t[3], t[4], t[5]), t[6] ^ t[7]);
}

// ---- dense span rows (kRowsSpanBnd) ----
// The chain of seg_crc, also capturing cap = X_tb ^ (w_tb & nm): the state
// after the boundary's dword tb (X_0 = w_0, X_t = A_4(X_{t-1}) ^ w_t) with the
// dword's bytes at or after the boundary (nm) taken out again.  tb = 16 in
// lanes without a boundary (cap stays 0).
__device__ __forceinline__ uint32_t seg_crc_cap(const uint8_t *lds, const u32x4 (&p)[4], uint32_t lsel, uint32_t tb,
                                                uint32_t nm, uint32_t &cap) {
  uint32_t x = p[0][0];
  uint32_t c = (tb == 0u) ? (x & ~nm) : 0u;
#pragma unroll
  for (int k = 0; k < 4; ++k)
#pragma unroll
    for (int d = 0; d < 4; ++d) {
      if (k == 0 && d == 0) continue;
      x = slice4w(lds, x, p[k][d], lsel);
      c = (tb == (uint32_t)(4 * k + d)) ? __builtin_amdgcn_bitop3_b32(p[k][d], nm, x, 0x6A) : c; // (w & nm) ^ x
    }
  cap = c;
  return slice4(lds, x, lsel);
}
// A_{4(16-tb)}(s): a boundary's captured chain state shifted to its segment's
// end (the span image's maps at kLdsSpanM4, word (n * 16 + nib) * 17 + tb).
__device__ __forceinline__ uint32_t span_m4(const uint8_t *lds, uint32_t s, uint32_t tb) {
  uint32_t t[8];
#pragma unroll
  for (uint32_t k = 0; k < 8; ++k)
    t[k] = lds_ld(lds, kLdsSpanM4 + 4u * ((k * 16u + ((s >> (4u * k)) & 15u)) * kSpanM4Stride + tb));
  return xor3(xor3(t[0], t[1], t[2]), xor3(t[3], t[4], t[5]), t[6] ^ t[7]);
}
// Inclusive XOR scan over the 16 lanes of each DPP row (row_shr, zeros shifted in).
__device__ __forceinline__ uint32_t row_xor_scan(uint32_t v) {
  v ^= (uint32_t)__builtin_amdgcn_mov_dpp((int)v, 0x111, 0xF, 0xF, true); // row_shr:1
  v ^= (uint32_t)__builtin_amdgcn_mov_dpp((int)v, 0x112, 0xF, 0xF, true); // row_shr:2
  v ^= (uint32_t)__builtin_amdgcn_mov_dpp((int)v, 0x114, 0xF, 0xF, true); // row_shr:4
  return v ^ (uint32_t)__builtin_amdgcn_mov_dpp((int)v, 0x118, 0xF, 0xF, true); // row_shr:8
}
// merge_row's distributed ST2 step without the cross-row XOR: the four
// shifted quarter values Vs_h = A_{1024(3-h)}(v_h) as scalars (lane 16h + 4).
struct RowQuarterVals {
  uint32_t vs[4];
};
__device__ __forceinline__ RowQuarterVals merge_quarters(const uint8_t *lds, uint32_t v, const DistLane &d) {
  const uint32_t nib = ((d.own ? v : 0u) >> d.shift) & 15u;
  const uint32_t t = dist_reduce8(lds_ld(lds, d.row_base + nib * d.row_mul));
  RowQuarterVals r;
#pragma unroll
  for (int h = 0; h < 4; ++h) r.vs[h] = (uint32_t)__builtin_amdgcn_readlane((int)t, 16 * h + 4);
  return r;
}

struct QuarterInfo {
  const uint8_t *p0;
  uint32_t len;
  uint32_t z;
  int64_t vstart; // 1 KiB window start relative to the item start (<= 0)
};

} // namespace rows

// QB = 1: rows of one item.  QB = 4: four items (<= 1 KiB each) per row.
// One 1024-thread workgroup (16 waves) per CU; each wave walks its tasks with
// one row of loads in flight ahead of the row it computes.  Every row issues
// exactly 4 loads and 1 store so the compiler can count vmcnt exactly (the
// prefetch is never drained early).  Per-task state is plain wave-uniform
// scalars (SGPRs); item metadata comes from scalar loads.
// RAGGED: items come from the offsets / lengths arrays (both non-null);
// otherwise item i is [base + i * stride, + len).
// DYN (QB = 1): workgroup-dynamic dealing.  A workgroup owns ROUNDS of 32
// consecutive tasks (round r of workgroup vb: tasks [(r * blocks + vb) * 32, +32))
// and its 16 waves take the tasks one at a time from an LDS counter, so they
// all finish within a task of each other.  (Static dealing leaves the waves
// of a SIMD finishing ~10 % apart, youngest last: measured per-slot exit
// times, tools/probe.py --mode timeline.)  Finished CRCs go to an LDS ring of
// kDynSlots rounds; the wave completing a round stores its 32 CRCs as one
// whole 128-B line.
// kDynRound / dyn_round(QB): crc32_kernels.h (the host sizes launches with them).
// Rounds the LDS output ring holds: a wave that finishes a task of round r
// waits until round r - kDynSlots has been stored.  QB = 1: 8 (was 4): C2
// -1.0 %, NS -0.25 % (profiles/r02/r02bx_dyn_slots_ab.txt).  QB = 4: 6 (its
// ring is 512 B a slot): with 8 the kernel took 163040 B of LDS, and a CU
// running one of its workgroups had no room left for the drop-in service's
// (kRowsLdsMax below) -- a C1 batch beside a busy service ran 251 us against
// 161 with 6 slots, while C1 alone measured the same (157.1 / 157.3 us,
// profiles/r04za).
#ifndef RPCCRC_DYN_SLOTS
#define RPCCRC_DYN_SLOTS 6
#endif
#ifndef RPCCRC_DYN_SLOTS_QB1
#define RPCCRC_DYN_SLOTS_QB1 8
#endif
// LDS one rows workgroup may take: the rest of the CU's 160 KiB stays free for
// the drop-in service's workgroup (crc32_service.hip, 476 B; LDS is granted in
// 1 KiB steps as measured: 162016 B left room for it, 163040 B did not).
constexpr uint32_t kRowsLdsMax = 163840u - 1024u;
constexpr uint32_t dyn_slots(int QB) { return QB == 1 ? RPCCRC_DYN_SLOTS_QB1 : RPCCRC_DYN_SLOTS; }
// Tail stealing (DYN with a.steal_s > 0): workgroup vb keeps only its first
// steal_s local rounds static (global rounds r * blocks + vb); the remaining
// global rounds form a pool that workgroups claim one round at a time from a
// device-scope counter (a.steal[0]), so XCDs that stream faster take more of
// it (per-XCD exit medians differ by up to 20 % with static rounds,
// profiles/r02/r02t_*).  A claim is issued kStealAhead local rounds ahead, by
// the wave taking a round's first task, and published into an LDS queue; the
// workgroup consumes its claimed rounds in publication order, so a claim that
// returns late is never lost.  A wave never waits (for a queue entry or a
// ring slot) while it holds an unpublished claim.
// Ragged QB = 1: a multi-row item's next row reuses its metadata (no
// offset / length reload and wait per row).
#ifndef RPCCRC_META_REUSE
#define RPCCRC_META_REUSE 1
#endif
constexpr bool kRowsMetaReuse = RPCCRC_META_REUSE != 0;
// Ragged QB = 1 pipeline: row loads issued two rows ahead instead of one.
#ifndef RPCCRC_RAGGED_AHEAD2
#define RPCCRC_RAGGED_AHEAD2 1
#endif
constexpr bool kRaggedAhead2 = RPCCRC_RAGGED_AHEAD2 != 0;
// First row's loads issued under the LDS image copy (crc32_rows_kernel kEarly).
// On since round 4: with the compact image (33 KiB read per workgroup) the
// overlap pays -- rotated-order A/B on one box: NS -0.5 %, C1 -0.6 %, C4
// -0.25 %, C2 -0.1 % (profiles/r04k/ab2, ab3); round 3 (155 KiB image): +-1 %.
#ifndef RPCCRC_EARLY_ROW
#define RPCCRC_EARLY_ROW 1
#endif
constexpr bool kEarlyRow = RPCCRC_EARLY_ROW != 0;
#ifndef RPCCRC_LDS_MASKS
#define RPCCRC_LDS_MASKS 1
#endif
constexpr bool kLdsMasks = RPCCRC_LDS_MASKS != 0;
// Uniform QB = 1 batches through the ragged pipeline (loads two rows ahead,
// chain of row C beside the merge of row P): A/B builds only.  Round 5, rotated,
// one box: NS +0.8 %, C3 +0.6 %, C4 +1.5 % against the plain loop
// (profiles/r05upipe; every uniform / stealing test green with it).
#ifndef RPCCRC_UNIFORM_PIPE
#define RPCCRC_UNIFORM_PIPE 0
#endif
constexpr bool kUniformPipe = RPCCRC_UNIFORM_PIPE != 0;
#ifndef RPCCRC_RAGGED_Q3_TEMPORAL
#define RPCCRC_RAGGED_Q3_TEMPORAL 0
#endif
constexpr bool kRaggedQ3Temporal = RPCCRC_RAGGED_Q3_TEMPORAL != 0;
#ifndef RPCCRC_TWO_PHASE
#define RPCCRC_TWO_PHASE 1
#endif
constexpr bool kTwoPhase = RPCCRC_TWO_PHASE != 0;
#ifndef RPCCRC_QB4_TWO_PHASE
#define RPCCRC_QB4_TWO_PHASE 0
#endif
constexpr bool kQb4TwoPhase = RPCCRC_QB4_TWO_PHASE != 0;
#ifndef RPCCRC_STEAL_EXIT_ACQREL
#define RPCCRC_STEAL_EXIT_ACQREL 0
#endif
#ifndef RPCCRC_STEAL_AHEAD
#define RPCCRC_STEAL_AHEAD 1
#endif
constexpr uint32_t kStealAhead = RPCCRC_STEAL_AHEAD;
// The task of a local round whose taker issues the claim (0: the round's first).
// A later task commits less work ahead of the pool's end (the drain) but leaves
// the claim less time to return before the next round needs it.
#ifndef RPCCRC_STEAL_CLAIM_AT
#define RPCCRC_STEAL_CLAIM_AT 0
#endif
constexpr uint32_t kStealClaimAt = RPCCRC_STEAL_CLAIM_AT;
constexpr uint32_t kStealQ = 16;                      // LDS queue ring
// Queue capacity.  A wave that grabbed its next task (one ahead) in pool round
// R maps it to a queue entry only at its next item switch; meanwhile the other
// waves can start tasks up to round R + kDynSlots (the output ring stops them
// only at their OUTPUT) and claim kStealAhead rounds past that.  Entry R of
// the ring must not be overwritten by then, or the lagging wave never finds
// its claim: it spins until its wait cap, its round is never stored, and every
// wave waiting for that ring slot caps too (RPCCRC_EIO).  That is what failed
// in round 4's pool-UNIT variant (RPCCRC_STEAL_SPLIT, profiles/r04b/split_ab.txt):
// units of 1/2 or 1/4 round made the lead 2 or 4 times as many queue entries
// (~20 or ~40 against 16) while the whole-round pool's lead is ~10 (DESIGN.md
// 4.1).  Rebuilt in round 5 with a queue sized for it, the units passed every
// test and still ran slower (C1 +4 %, NS +1.5 %, profiles/r05d).
static_assert(kStealQ >= dyn_slots(1) + kStealAhead + 2 && kStealQ >= dyn_slots(4) + kStealAhead + 2,
              "steal queue shorter than the rounds a workgroup can run ahead of a lagging wave");
constexpr uint32_t kStealCtlWords = 3 + 2 * kStealQ;  // tail, done, inflight, tags[Q], ids[Q]
// Bounded waits.  Both waits end by protocol (a claim is published by the wave
// holding it at the end of its current row, before it waits on anything, and
// an output-ring slot is freed by the wave finishing its round's last task),
// so these caps never trigger in a healthy launch.  If one does, the wave
// stores kErrStealWait / kErrRingWait into the launch's error word a.err and
// moves on -- the host then reports RPCCRC_EIO instead of returning stale CRCs
// silently (VERDICT / ADVICE r02), and no wait can turn into a hang.
// The cap must outlast any healthy wait: a ring slot waits for the slowest
// task of the round 8 rounds back, and one task may be a body of up to 4 GiB
// walked by ONE wave (a ragged batch whose length bound skips the big-body
// route) -- ~1-3 s at one wave's rate.  Round 3's cap of 2^21 short sleeps
// (~0.1 s) fired on such a healthy launch.  The first 1024 spins
// sleep briefly (a healthy wait is usually microseconds), later ones
// s_sleep 127 (~8K cycles, >= 3.4 us): 2^23 spins are >= ~28 s.  (A wall-time
// cap from s_memrealtime kept 64-bit timestamps live: SGPR spills in the hot
// loops went 2 -> 7 on the north-star kernel.)
constexpr uint32_t kWaitSpinMax = 1u << 23;
__device__ __forceinline__ bool wait_spin(uint32_t spin) { // sleeps; true once the cap has passed
  if (spin >= kWaitSpinMax) return true;
  if (spin < 1024u) __builtin_amdgcn_s_sleep(2);
  else __builtin_amdgcn_s_sleep(127);
  return false;
}
// DYN control block: [0] task counter, kDynSlots done counts, kDynSlots slot
// generations (slot s starts at round s), then the CRC ring (QB CRCs per task,
// kRound tasks per slot).
constexpr uint32_t dyn_gen_ofs(int QB) { return 1 + dyn_slots(QB); }
constexpr uint32_t dyn_ringbuf_ofs(int QB) { return dyn_gen_ofs(QB) + dyn_slots(QB); }
constexpr uint32_t dyn_ring_words(int QB) { return dyn_ringbuf_ofs(QB) + dyn_slots(QB) * dyn_round(QB) * (uint32_t)QB; }
constexpr uint32_t dyn_ctl_words(int QB) { return dyn_ring_words(QB) + kStealCtlWords; }

template <int QB, bool NT, bool RAGGED = false, int ABL = 0, int DEPTH = 1, bool DYN = false, bool STEAL = false>
__global__ void __launch_bounds__(1024, 4) crc32_rows_kernel(ItemsArgs a) {
  using namespace rows;
  static_assert(!DYN || DEPTH == 1, "DYN: DEPTH = 1");
  static_assert(!STEAL || DYN, "stealing: DYN launches");
  constexpr uint32_t kRound = dyn_round(QB); // tasks per dealing round
  constexpr uint32_t kDynSlots = dyn_slots(QB);
  constexpr uint32_t kGen = dyn_gen_ofs(QB), kRingBuf = dyn_ringbuf_ofs(QB);
  constexpr bool kLdsSeed = (ABL & kRowsAblLdsSeed) != 0 || (RPCCRC_LDS_SEED != 0 && QB == 1 && RAGGED);
  // sub-row first rows: ragged QB = 1 with the plain chain (image V3 adds SQ)
  constexpr bool kSub = kSubRows && QB == 1 && RAGGED && !kTwoChains &&
                        (ABL & (kRowsAblNoCompute | kRowsAblNoMerge | kRowsAblNoTranspose | kRowsAblHalfChain | kRowsAblNoSub)) == 0;
  constexpr uint32_t kImgBytes = kSub ? kLdsBytesV3 : kLdsBytesV2;
  // Ragged DYN QB = 1 (the C2 path): small items four per row (see kSB's loop)
  constexpr bool kSB = RPCCRC_SMALL_GROUPS != 0 && QB == 1 && RAGGED && DYN && !STEAL && DEPTH == 1 && kSub &&
                       kLaneHorner && kRowsPipe && kRaggedAhead2 && (ABL & ~kRowsAblNoStore) == 0;
  __shared__ __attribute__((aligned(16))) uint32_t s_lds[kImgBytes / 4];
  // DYN control block (dyn_ring_words): task counter, done counts, slot
  // generations (slot s starts at round s), CRC ring.
  __shared__ uint32_t s_ctl[DYN ? (STEAL ? dyn_ctl_words(QB) : dyn_ring_words(QB)) : 1];
  // Ragged QB = 1 (RPCCRC_LDS_MASKS): the edge fixes' byte masks as a table, as
  // crc32_small_kernel's s_mask (row f: bytes >= f of the first piece; row
  // 16 + z: bytes below 16 - z of the last) -- 16 SALU per fix saved.
  constexpr bool kMaskTab = kLdsMasks && QB == 1 && RAGGED && (ABL & kRowsAblNaturalOrder) == 0;
  __shared__ __attribute__((aligned(16))) uint32_t s_mask[kMaskTab ? 128 : 4];
  static_assert(sizeof(s_lds) + sizeof(s_ctl) + (kMaskTab ? sizeof(s_mask) : 0) <= kRowsLdsMax,
                "leave a CU room for the drop-in service");
  if constexpr (kMaskTab) {
    if (threadIdx.x < 128u) {
      const uint32_t t = threadIdx.x, k = (t >> 2) & 15u, d = t & 3u;
      s_mask[t] = (t < 64u) ? keep_front_dword(k, d) : keep_end_dword(16u - k, d);
    }
  }
  // kEarlyRow: each wave's first task is static (DYN: counter index = wave, so
  // the LDS counter starts at 16), and its first row's loads are issued between
  // the image's global loads and its LDS stores -- the row's HBM latency then
  // overlaps the image copy instead of following the barrier.
  constexpr bool kEarly = kEarlyRow && (ABL & kRowsAblTimes) == 0;
  if constexpr (DYN) {
    if (threadIdx.x < kRingBuf)
      s_ctl[threadIdx.x] = (threadIdx.x >= kGen) ? threadIdx.x - kGen : ((threadIdx.x == 0u && kEarly) ? 16u : 0u);
    if (STEAL && threadIdx.x < 3 + kStealQ) s_ctl[dyn_ring_words(QB) + threadIdx.x] = 0u; // tail/done/inflight/tags
  }
  // Device-side item counts (split lists, big-body chunks) may be 0: leave
  // before the 155 KiB image copy (block-uniform).
  if (blockIdx.x == 0 && threadIdx.x < a.zero_n) a.zero_out[threadIdx.x] = 0u;
  if (a.n_dev != nullptr && ld_const(a.n_dev, 0) == 0) return;
  if (a.skip_dev != nullptr && ld_const(a.skip_dev, 0) != 0u) return; // (a dense batch: the span pass has it)
  uint64_t t_entry = 0, t_image = 0, c_entry = 0;
  if constexpr ((ABL & kRowsAblTimes) != 0) { // (+ the shader clock: s_memtime ticks shader cycles)
    t_entry = __builtin_amdgcn_s_memrealtime();
    c_entry = __builtin_amdgcn_s_memtime();
    __builtin_amdgcn_s_waitcnt(0xC07F); // lgkmcnt(0)
  }
  // All of this thread's image loads in flight at once (a rolled loop would
  // pay one L2 round trip per 16 KiB before the first HBM byte is read).
  // kEarly: the image in registers until the first row's loads are issued
  // (native vectors: HIP's uint4 struct copies became memcpys through a
  // private-memory array -- 160 B of scratch per lane).
  ImgRegs<kImgBytes> img;
  if constexpr (!kEarly) {
    if constexpr ((ABL & kRowsAblNoImage) == 0) copy_lds_image<kImgBytes>(a.lds_image, s_lds);
    __syncthreads();
    if constexpr ((ABL & kRowsAblTimes) != 0) t_image = __builtin_amdgcn_s_memrealtime();
  } else if constexpr ((ABL & kRowsAblNoImage) == 0) {
    img_load<kImgBytes>(a.lds_image, img);
  }
  // LDS stores of the image + the barrier (kEarly: after the first row's loads
  // are issued; the loads above were issued first, so waiting for them does
  // not wait for the row).  A macro, not a lambda: a lambda capturing `img` by
  // reference kept it in memory -- 160 B of scratch per lane, the image
  // round-tripped through HBM on every launch (+70 MB per launch, NS 602 ->
  // 645 us; -Rpass-analysis=kernel-resource-usage).
#define RPCCRC_ROWS_IMAGE_READY()                                                                          \
  do {                                                                                                     \
    __builtin_amdgcn_sched_barrier(0);                                                                     \
    if constexpr ((ABL & kRowsAblNoImage) == 0) img_store<kImgBytes>(img, s_lds);                          \
    __syncthreads();                                                                                       \
    if constexpr ((ABL & kRowsAblTimes) != 0) t_image = __builtin_amdgcn_s_memrealtime();                  \
  } while (0)
  // (!kEarly: the image is in LDS already, above)
  const uint8_t *lds = reinterpret_cast<const uint8_t *>(s_lds);

  const uint32_t lane = threadIdx.x & 63u;
  const uint32_t lane4 = (lane & 31u) * 4u;
  const uint32_t lsel = lane4 | ((lane4 + 128u) << 8) | (1u << 16);  // MAIN tables
  const uint32_t lsel1 = lane4 | ((lane4 + 128u) << 8) | (2u << 16); // ST1
  const uint32_t hi = lane >> 4;                   // 16-lane row = quarter after the transpose
  const bool upper = (lane & 16u) != 0;            // lane bit 4 (two-chain merge)
  // byte offset of this lane's piece in a quarter
  const uint32_t pofs = 16u * (((ABL & kRowsAblNaturalOrder) != 0) ? lane : piece_of_lane(lane));
  const DistLane dl = dist_lane(lane);
  // sub-row constants: quarter rows' SQ index j = hi, their kept row hi = 3;
  // half rows' upper lanes
  const uint32_t sub_jbq = (hi * 64u) * 0x01010101u;
  const uint32_t sub_m3 = (hi == 3u) ? 0xFFFFFFFFu : 0u;
  const uint32_t sub_mu = (lane & 32u) ? 0xFFFFFFFFu : 0u;
  const uint32_t wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  // Task / item indices are 32-bit (launch_rows keeps every launch below 2^30
  // items): SALU has no 64-bit ordered compare, so 64-bit indices put every
  // `task < n` test (and its operand copies) on the VALU.
  const uint32_t nwaves = gridDim.x * 16u;
  // Tasks (QB = 1: items, QB = 4: groups of 4 items) are dealt round-robin in
  // groups of G (below): all waves stream one moving window of HBM (blocked
  // ranges put 4096 streams 1 MiB apart in lockstep: measured 6 % slower).
  // gw is XCD-aware: workgroups are dispatched round-
  // robin over the 8 XCDs, so virtual block vb = (b % 8) * (blocks / 8) + b / 8
  // makes the 32 waves whose CRCs share a 128-B output line live on one XCD,
  // whose L2 assembles the whole line (measured: strided 4-B stores from two
  // XCDs per line cost 3.5 % of the kernel).
  const uint32_t nblk = gridDim.x;
  const uint32_t vb = (nblk % 8u == 0u) ? (blockIdx.x % 8u) * (nblk / 8u) + blockIdx.x / 8u : blockIdx.x;
  const uint32_t gw = vb * 16u + wave;
  const uint32_t mode = a.mode;
  const uint32_t n = (uint32_t)(a.n_dev ? ld_const(a.n_dev, 0) : a.n_items);
  // Dense span pass (kRowsSpanBnd): item j is block j of the plan's stream.
  constexpr bool kSpan = (ABL & kRowsSpanBnd) != 0 && QB == 1 && !RAGGED;
  const uint64_t span_base = kSpan ? ld_const(reinterpret_cast<const uint64_t *>(a.span_ctl), 0) : 0u;
  const uint64_t span_end = kSpan ? span_base + ld_const(reinterpret_cast<const uint64_t *>(a.span_ctl), 1) : 0u;
  auto oidx = [&](uint32_t i) -> uint32_t { return a.out_idx ? a.out_idx[i] : i; }; // output slot
  auto store_out = [&](uint32_t *p, uint32_t v) {
    if constexpr ((ABL & kRowsAblNtStore) != 0) __builtin_nontemporal_store(v, p);
    else *p = v;
  };
  const uint32_t n_tasks = (QB == 4 || kSB) ? (n + 3) / 4 : n; // (kSB: groups of 4 items)
  // Group dealing, G = 2^a.gshift: in each whole round of nwaves * G tasks,
  // wave gw takes the G consecutive tasks [gw * G, gw * G + G), so its results
  // of a round are G consecutive outputs (G = 32: the wave writes whole 128-B
  // lines).  Tasks past the last whole round are dealt round-robin.
  const uint32_t gshift = a.gshift;
  const uint32_t gmask = (1u << gshift) - 1;
  const uint32_t tail_base = n_tasks / (nwaves << gshift) * (nwaves << gshift);
  const uint32_t jg = tail_base / nwaves; // tasks per wave dealt in groups
  auto task_of = [&](uint32_t j) -> uint32_t { // the wave's j-th task
    return j < jg ? ((((j >> gshift) * nwaves + gw) << gshift) | (j & gmask)) : tail_base + gw + (j - jg) * nwaves;
  };
  auto next_task = [&](uint32_t t) -> uint32_t { // the wave's task after task t
    if (t >= tail_base) return t + nwaves;
    if (((t + 1) & gmask) != 0) return t + 1;
    const uint32_t u = t + 1 + ((nwaves - 1) << gshift);
    return u < tail_base ? u : tail_base + gw;
  };
  // DYN: a wave's next task comes from the workgroup's LDS counter.  The
  // atomic is issued a task ahead; its result is read at the next item switch.
  auto dyn_grab = [&]() -> uint32_t { // lane 0 holds the grabbed index
    uint32_t c = 0;
    if (lane == 0) c = __hip_atomic_fetch_add(&s_ctl[0], 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
    return c;
  };
  auto dyn_task = [&](uint32_t c) -> uint32_t { return (((c / kRound) * nblk + vb) * kRound) | (c % kRound); };
  // ---- tail stealing (see kStealAhead) ----
  // Static local rounds per workgroup.  Device-counted launches (a.n_dev: the
  // big-body route's chunk pass) size the pool here, as launch_rows does on
  // the host; too few rounds -> no pool (then `steal` is false and the
  // STEAL instantiation deals like plain DYN).
  const uint32_t steal_s = [&]() -> uint32_t {
    if constexpr (!STEAL) return 0u;
    if (a.steal_s != kStealOnDevice) return a.steal_s;
    const uint32_t rounds = (n_tasks + kRound - 1) / kRound;
    uint32_t st = (uint32_t)(((uint64_t)rounds * (1000u - a.steal_permille)) / 1000u) / nblk;
    if (rounds / nblk > st + a.steal_max_wg) st = rounds / nblk - a.steal_max_wg; // (launch_rows' cap)
    return (st >= kStealAhead && st * nblk < rounds) ? st : 0u;
  }();
  const bool steal = STEAL && steal_s != 0u;
  const uint32_t pool_first = steal_s * nblk; // first pool (global) round
  const uint32_t pool_n = steal ? (n_tasks + kRound - 1) / kRound - pool_first : 0u;
  uint32_t *q_ctl = s_ctl + (STEAL ? dyn_ring_words(QB) : 0u);
  uint32_t *q_tail = q_ctl, *q_done = q_ctl + 1, *q_inflight = q_ctl + 2;
  uint32_t *q_tag = q_ctl + 3, *q_id = q_ctl + 3 + kStealQ;
  bool has_claim = false; // wave-uniform: this wave holds an unpublished claim
  uint32_t claim_v = 0;   // lane 0: the device counter's answer
  // Device error word (pinned host memory): one vector store from the lane that
  // ran out of patience; the host maps a non-zero word to RPCCRC_EIO.
  auto report_err = [&](uint32_t bits) {
    if (a.err != nullptr) __hip_atomic_store(a.err, bits, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
  };
  // Lane 0: wait until output-ring slot `slot` is free for round `rnd` (bounded).
  auto ring_wait = [&](const uint32_t *gen, uint32_t slot, uint32_t rnd) {
    for (uint32_t spin = 0; __hip_atomic_load(&gen[slot], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP) != rnd; ++spin) {
      if (wait_spin(spin)) {
        report_err(kErrRingWait);
        break;
      }
    }
  };
  auto lds_ld_acq = [](uint32_t *p) { return __hip_atomic_load(p, __ATOMIC_ACQUIRE, __HIP_MEMORY_SCOPE_WORKGROUP); };
  auto publish = [&]() { // uniform
    if (!has_claim) return;
    if (lane == 0) {
      uint32_t id = claim_v;
      // keeps the use (and its wait for the atomic) here: hoisted out of a
      // wait loop it made every pool round's first task wait for its own claim
      __asm__ volatile("" : "+v"(id));
      if (id < pool_n) {
        const uint32_t slot = __hip_atomic_fetch_add(q_tail, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
        q_id[slot % kStealQ] = id;
        __hip_atomic_store(&q_tag[slot % kStealQ], slot + 1u, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_WORKGROUP);
      } else {
        __hip_atomic_store(q_done, 1u, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_WORKGROUP);
      }
      __hip_atomic_fetch_sub(q_inflight, 1u, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_WORKGROUP);
    }
    has_claim = false;
  };
  // The wave taking local round r's first task claims a pool round for the
  // workgroup (for use kStealAhead rounds later).
  auto claim_if_first = [&](uint32_t c) { // uniform
    if (!steal || c % kRound != kStealClaimAt || c / kRound + kStealAhead < steal_s) return;
    publish(); // at most one claim in flight per wave
    uint32_t go = 0;
    if (lane == 0 && lds_ld_acq(q_done) == 0u) {
      go = 1;
      __hip_atomic_fetch_add(q_inflight, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
      // the in-flight count is visible before the device counter moves: a
      // wave that then sees done && inflight == 0 has seen every claim that
      // can still return a pool round
      __builtin_amdgcn_s_waitcnt(0xC07F); // lgkmcnt(0)
      claim_v = __hip_atomic_fetch_add(a.steal, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    }
    has_claim = __builtin_amdgcn_readfirstlane((int)go) != 0;
  };
  // Counter index -> global task.  more = false: the workgroup has no work left
  // (returns n_tasks).  Static rounds as dyn_task; pool rounds from the queue.
  auto dyn_map = [&](uint32_t c, bool &more) -> uint32_t {
    const uint32_t r = c / kRound;
    more = true;
    if (!steal || r < steal_s) return dyn_task(c);
    const uint32_t q = r - steal_s, k = q % kStealQ;
    if (a.test_giveup != 0u) { // test-only: take the give-up path below deterministically
      if (lane == 0) report_err(kErrStealWait);
      more = false;
      return n_tasks;
    }
    for (uint32_t spin = 0;; ++spin) {
      uint32_t st = 0, id = 0;
      if (lane == 0) {
        if (lds_ld_acq(&q_tag[k]) == q + 1u) {
          st = 1;
        } else if (lds_ld_acq(q_done) != 0u && lds_ld_acq(q_inflight) == 0u) {
          st = (lds_ld_acq(&q_tag[k]) == q + 1u) ? 1u : 2u; // every claim is published: final answer
        }
        if (st == 1u) id = q_id[k];
      }
      st = (uint32_t)__builtin_amdgcn_readfirstlane((int)st);
      if (st == 1u) return ((pool_first + (uint32_t)__builtin_amdgcn_readfirstlane((int)id)) * kRound) | (c % kRound);
      if (st == 2u) break;
      publish(); // never wait holding a claim
      if (wait_spin(spin)) { // never in a healthy launch: fail loudly, do not hang
        if (lane == 0) report_err(kErrStealWait);
        break;
      }
    }
    more = false;
    return n_tasks;
  };
  // Every workgroup passes here once at the end; the last one resets the
  // device counter for the next launch that leases it.  Relaxed: a workgroup
  // gets here only after every claim it issued has returned (performed), so
  // the last arrival's reset follows every claim of the launch; the next
  // launch sees the zeros through the kernel boundary's release.  (acq_rel /
  // release put an L2 writeback + invalidate, buffer_wbl2 / buffer_inv sc1,
  // into every workgroup's exit -- RPCCRC_STEAL_EXIT_ACQREL=1 restores it.)
  auto steal_exit = [&]() {
    if (!steal) return;
    __syncthreads();
    if (threadIdx.x == 0) {
#if RPCCRC_STEAL_EXIT_ACQREL
      const uint32_t old = __hip_atomic_fetch_add(a.steal + 1, 1u, __ATOMIC_ACQ_REL, __HIP_MEMORY_SCOPE_AGENT);
#else
      const uint32_t old = __hip_atomic_fetch_add(a.steal + 1, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
#endif
      if (old + 1u == nblk) {
        // No fence here (ADVICE r02 asked for an acquire fence on this path).
        // At agent scope on gfx950 that fence is an L2 invalidate. It is not
        // needed for the reset to be ordered: the claims, the
        // exit increments and this reset all touch the same two words as
        // agent-scope atomics, so they are performed at one coherence point.
        // Each workgroup's increment is issued after its claims have returned,
        // and this store is issued after the increment that returned nblk - 1,
        // so it lands after every claim of the launch.
        __hip_atomic_store(a.steal, 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        __hip_atomic_store(a.steal + 1, 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      }
    }
  };
  uint32_t first_c = 0, first_task;
  if constexpr (DYN) {
    first_c = kEarly ? wave : (uint32_t)__builtin_amdgcn_readfirstlane((int)dyn_grab());
    first_task = dyn_task(first_c);
  } else {
    first_task = task_of(0);
  }
  if (first_task >= n_tasks) { // (never with stealing: local round 0 is static and full)
    if constexpr (kEarly) RPCCRC_ROWS_IMAGE_READY(); // every wave of the workgroup reaches the barrier once
    return;
  }
  // After the first row's loads are issued (kEarly), the image and the LDS
  // control block become usable: RPCCRC_ROWS_BEGIN() at each first issue.
#define RPCCRC_ROWS_BEGIN()                             \
  do {                                                  \
    if constexpr (kEarly) RPCCRC_ROWS_IMAGE_READY();    \
    claim_if_first(first_c);                            \
  } while (0)
  if constexpr (!kEarly) RPCCRC_ROWS_BEGIN();

  auto synth = [&](uint32_t key, u32x4 (&buf)[4]) {
#pragma unroll
    for (int b = 0; b < 4; ++b) {
      const uint32_t v = (uint32_t)key * 0x9E3779B1u + (uint32_t)b * 0x85EBCA6Bu + lane;
      buf[b] = u32x4{v, v ^ 0x5bd1e995u, v + 0x68e31da4u, ~v};
    }
  };
  // Transpose + chain + merge step 1: every lane of 16-lane row hi returns
  // crc0 of quarter hi of the row.
  auto quarter_crcs = [&](u32x4 (&buf)[4]) -> uint32_t {
    if constexpr ((ABL & kRowsAblNoTranspose) == 0) transpose(buf);
    if constexpr ((ABL & kRowsAblHalfChain) != 0) {
      uint32_t x = buf[2][0];
#pragma unroll
      for (int k = 2; k < 4; ++k)
#pragma unroll
        for (int d = 0; d < 4; ++d) {
          if (k == 2 && d == 0) continue;
          x = slice4w(lds, x, buf[k][d], lsel);
        }
      return merge_lo(lds, slice4(lds, x, lsel), lsel1);
    }
    if constexpr ((ABL & (kRowsAblNoCompute | kRowsAblNoMerge)) == 0) return row_quarters(lds, buf, lsel, lsel1, upper);
    uint32_t s;
    if constexpr ((ABL & kRowsAblNoCompute) != 0) s = xor_fold(buf);
    else s = seg_crc(lds, buf, lsel);
    if constexpr ((ABL & kRowsAblNoMerge) == 0) s = merge_lo(lds, s, lsel1);
    return s;
  };

  if constexpr (QB == 1) {
    // Item metadata (wave-uniform).  item must be < n.
    // The zlib seed A_first(0xFFFFFFFF) of the item's first row is a scalar
    // load from the global Tq table, issued here -- a task ahead of its use.
    // hd = bytes of the item's first row (1..4096; 0 for an empty item) after
    // the z pad: row r starts at item offset r * 4096 + hd - 4096, so only row
    // 0 can start before the item (when hd < 4096).
    auto meta = [&](uint32_t item, uint64_t &p0, uint32_t &hd, uint32_t &len, uint32_t &z, uint32_t &nr,
                    uint32_t &seed) {
      if constexpr (kSpan) { // one 4 KiB block, no pad, RAW
        p0 = span_base + (uint64_t)item * kRow;
        len = kRow;
        z = 0u;
        nr = 1u;
        hd = kRow;
        seed = 0u;
        return;
      }
      uint64_t off = RAGGED ? ld_const(a.offsets, item) : (uint64_t)item * a.stride;
      len = RAGGED ? ld_const(a.lengths, item) : a.len;
      if constexpr (RAGGED && kMetaCoissue) __asm__ volatile("" : "+s"(off), "+s"(len)); // both loads, one wait
      if constexpr (RAGGED) {
        // a routed big body is empty here (launch_big_route computes it)
        if (len >= a.big_min && a.routed != nullptr) {
          const uint32_t bi = a.out_idx ? ld_const(a.out_idx, item) : item;
          if ((ld_const(a.routed, bi >> 5) >> (bi & 31u)) & 1u) len = 0;
        }
      }
      p0 = (uint64_t)(uintptr_t)a.base + off;
      z = (uint32_t)(0u - (uint32_t)(p0 + len)) & 15u;
      // rows and first-row bytes of lp = len + z in 32-bit scalar ops (lp may
      // pass 2^32): lp = 4096 a + b with b <= 4110, so the rows are a + cb,
      // cb = ceil(b / 4096) in {0, 1, 2}, and hd = b + 4096 (1 - cb)
      const uint32_t ra = len >> 12, rb = (len & (kRow - 1u)) + z, cb = (rb + kRow - 1u) >> 12;
      nr = ra + cb;
      hd = rb + kRow - cb * kRow;
      if (nr == 0u) { // zero-length items: one fully masked row
        nr = 1u;
        hd = 0u;
      }
      if constexpr (kLdsSeed)
        seed = hd; // resolved in compute / lane_horner_p
      else
        seed = (mode == kModeRaw) ? 0u : ld_const(a.tq, hd);
    };
    auto issue = [&](uint64_t p0, uint32_t hd, uint32_t nr, uint32_t r, bool ok, uint64_t safe, u32x4 (&buf)[4]) {
      if constexpr ((ABL & kRowsAblNoLoad) != 0) {
        synth((uint32_t)p0 + r, buf);
      } else {
        const bool fp = r == 0 && hd < kRow; // a first row that starts before the item
        // One load sequence for every row (loads issued from two paths broke
        // the compiler's vmcnt accounting: the row just issued was waited for).
        // Whole rows: scalar row base + the lane's constant offsets.  A first
        // row starting before the item: base = the item's first 16-B block,
        // pieces before it read as zeros; invalid rows read nothing.
        uint64_t base;
        uint32_t off[4];
        if (ok && !fp && (ABL & kRowsAblNoFastLoad) == 0) {
          base = p0 + (uint64_t)r * kRow + hd - kRow;
#pragma unroll
          for (int b = 0; b < 4; ++b) off[b] = pofs + b * kQuarter;
        } else {
          base = ok ? (p0 & ~(uint64_t)15) : safe;
          const int32_t d = ok ? (int32_t)(r * kRow + hd) - (int32_t)kRow + (int32_t)(p0 & 15) : INT32_MIN / 2;
#pragma unroll
          for (int b = 0; b < 4; ++b) // negative offsets (pieces before the item) -> kOobOffset: one v_min_u32
            off[b] = min((uint32_t)(d + (int32_t)(pofs + b * kQuarter)), kOobOffset);
        }
        // (span pass: the stream's last block reads zeros past its end, rounded
        // up to 16 B -- inside the 16-B block holding the last body byte)
        const uint64_t rem = span_end - base;
        const __amdgpu_buffer_rsrc_t row =
            row_rsrc(base, (kSpan && rem < kRow) ? (uint32_t)((rem + 15u) & ~(uint64_t)15) : kRsrcRange);
#pragma unroll
        for (int b = 0; b < 4; ++b) {
          // RPCCRC_RAGGED_Q3_TEMPORAL (A/B): a ragged row's last quarter through
          // L2 at normal priority, so the line it shares with the next row
          // (rows end at the body's 16-B end) is there when that row loads it
          if (RAGGED && kRaggedQ3Temporal && b == 3) buf[b] = ldb16<false>(row, off[b]);
          else buf[b] = ldb16<NT>(row, off[b]);
        }
      }
    };
    uint32_t W = 0; // running crc0 (Horner over rows) of the current item, wave-uniform
    // Finished CRCs are parked in one VGPR (lane k = this wave's k-th pending
    // item, item = gw + (j0 + k) * nwaves) and stored 64 at a time: a per-row
    // store would make the compiler drain vmcnt (store-data WAR) every row.
    uint32_t outv = 0, ocount = 0;
    uint32_t j0 = 0;
    uint32_t sink = 0;
    auto flush = [&]() {
      if constexpr ((ABL & kRowsAblNoStore) == 0) {
        if (lane < ocount) a.out[oidx(task_of(j0 + lane))] = outv;
      } else {
        sink ^= outv;
      }
      j0 += ocount;
      ocount = 0;
    };
    auto park = [&](uint32_t res) {
      outv = (lane == ocount) ? res : outv;
      if (++ocount == 64u) flush();
    };
    // DYN output: CRC of the task with counter index c into the LDS ring; the
    // wave completing a round stores the round's CRCs as one whole line.
    auto dyn_out = [&](uint32_t c, uint32_t tsk, uint32_t res) {
      const uint32_t rnd = c / kRound, idx = c % kRound, slot = rnd % kDynSlots;
      uint32_t *done = s_ctl + 1 + slot, *gen = s_ctl + kGen, *ring = s_ctl + kRingBuf;
      uint32_t old = 0;
      publish(); // the ring wait below must not hold a claim
      if (lane == 0) {
        // the slot still holds an older round that a slow wave has not finished
        ring_wait(gen, slot, rnd);
        ring[slot * kRound + idx] = res;
        old = __hip_atomic_fetch_add(done, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
      }
      old = (uint32_t)__builtin_amdgcn_readfirstlane((int)old);
      // the round's first global task (rounds are aligned)
      const uint32_t base = tsk & ~(kRound - 1u);
      const uint32_t cnt = (n_tasks - base < kRound) ? n_tasks - base : kRound;
      if (old + 1u == cnt) { // this wave completed the round
        const uint32_t v = ring[slot * kRound + (lane % kRound)];
        if constexpr ((ABL & kRowsAblNoStore) == 0) {
          if (lane < cnt) store_out(a.out + oidx(base + lane), v);
        } else {
          sink ^= v;
        }
        if (lane == 0) {
          *done = 0;
          __hip_atomic_store(&gen[slot], rnd + kDynSlots, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
        }
        if constexpr ((ABL & kRowsRoundOut) != 0 && QB == 1 && !RAGGED) {
          // the round's crc0: a 5-level lane tree (lanes 32..63 repeat 0..31);
          // at level l the earlier 2^l-item run is shifted past the later one
          if (cnt == kRound) {
            uint32_t x = v;
#pragma unroll
            for (uint32_t l = 0; l < 5; ++l) {
              uint32_t sh;
              if (l == 0) sh = rw_map(lds, x);
              else if (l == 1) sh = nib_map_at<kLdsRoundMaps>(lds, x);
              else if (l == 2) sh = nib_map_at<kLdsRoundMaps + 512u>(lds, x);
              else if (l == 3) sh = nib_map_at<kLdsRoundMaps + 1024u>(lds, x);
              else sh = nib_map_at<kLdsRoundMaps + 1536u>(lds, x);
              const uint32_t mine = ((lane >> l) & 1u) ? x : sh;
              x = mine ^ (uint32_t)__shfl_xor((int)mine, 1 << l, 64);
            }
            if (lane == 0) a.round_out[base / kRound] = x;
          }
        }
        j0 += cnt;
      }
    };
    auto fix_row = [&](uint32_t hd, uint32_t z, uint32_t nr, uint32_t r, u32x4 (&buf)[4]) {
      const bool fp = r == 0 && hd < kRow;
      const bool last = r + 1 == nr;
      if (fp || (last && z != 0)) {
        // the body's first byte sits at row offset 4096 - hd (first row only)
        const uint32_t front = fp ? kRow - hd : kRow;
        constexpr bool kNat = (ABL & kRowsAblNaturalOrder) != 0;
#pragma unroll
        for (uint32_t b = 0; b < 4; ++b) {
          const uint32_t fb = front - b * kQuarter; // wraps (>= 1024) outside quarter b
          const uint32_t zb = (b == 3 && last) ? z : 0u;
          if constexpr (kMaskTab) {
            if ((fb & 15u) != 0u && fb < kQuarter) {
              const u32x4 mf = *reinterpret_cast<const u32x4 *>(s_mask + 4u * (fb & 15u));
              const uint32_t e = (lane == lane_of_piece(fb >> 4)) ? 0u : 0xFFFFFFFFu;
#pragma unroll
              for (uint32_t d = 0; d < 4; ++d) buf[b][d] = and_or_keep(buf[b][d], mf[d], e);
            }
            if (zb != 0u) {
              const u32x4 me = *reinterpret_cast<const u32x4 *>(s_mask + 64u + 4u * zb);
              const uint32_t e = (lane == lane_of_piece(63u)) ? 0u : 0xFFFFFFFFu;
#pragma unroll
              for (uint32_t d = 0; d < 4; ++d) buf[b][d] = and_or_keep(buf[b][d], me[d], e);
            }
          } else {
            fix_quarter<kNat>(buf[b], lane, fb, zb);
          }
        }
      }
    };
    // Horner step and result of a row whose merge is done.
    auto finish = [&](bool valid, uint32_t len, uint32_t z, uint32_t nr, uint32_t r, uint32_t seed, uint32_t cidx,
                      uint32_t tsk, RowMerge m) {
      const bool last = r + 1 == nr;
      // Horner over rows: A_4096(W), or the zlib seed on the item's first row.
      if constexpr (kLdsSeed) {
        if (r == 0) {
          const uint32_t first = seed, up = (first + 15u) & ~15u;
          uint32_t w = lds_ld(lds, kLdsTQ16 + up / 4u);
          if (up != first) w = dist_uniform(lds, w, kLdsZI2 + (up - first - 1u) * 512u, dl);
          seed = (mode == kModeRaw) ? 0u : (uint32_t)__builtin_amdgcn_readfirstlane((int)w);
        }
      }
      W = ((r == 0) ? seed : m.rwu) ^ m.crc;
      if (last) {
        uint32_t res = W;
        if (z != 0) res = dist_uniform(lds, res, kLdsZI2 + (z - 1u) * 512u, dl);
        if (mode == kModeFinal) res = ~res;
        if constexpr (DYN) {
          if (valid) dyn_out(cidx, tsk, res);
        } else {
          if (valid) park(res);
        }
      }
    };
    auto compute = [&](bool valid, uint32_t hd, uint32_t len, uint32_t z, uint32_t nr, uint32_t r, uint32_t seed,
                       uint32_t cidx, uint32_t tsk, u32x4 (&buf)[4]) {
      fix_row(hd, z, nr, r, buf);
      uint32_t v;
      if (kSub && r == 0 && hd <= kQuarter) v = merge_lo(lds, quarter_row_segs(lds, buf, lsel, sub_jbq, sub_m3), lsel1);
      else if (kSub && r == 0 && hd <= 2 * kQuarter) v = merge_lo(lds, half_row_segs(lds, buf, lsel, sub_mu), lsel1);
      else v = quarter_crcs(buf);
      RowMerge m;
      if constexpr ((ABL & kRowsAblNoMerge) == 0) {
        m = merge_row(lds, v, W, dl);
      } else {
        m.crc = (uint32_t)__builtin_amdgcn_readfirstlane((int)v);
        m.rwu = W;
      }
      finish(valid, len, z, nr, r, seed, cidx, tsk, m);
    };

    // ---- dense span pass (kSpan) ----
    // Block j's record {first | cnt << 25, offsets of its first kDenseInline
    // boundaries} comes with the block's row loads as a VECTOR load (one 16-B
    // request, every lane the same address): a scalar load in flight would make
    // each chain step's LDS wait an lgkmcnt(0) (SMEM returns out of order).
    // (A separate count array, one byte a block, measured the span pass +3.4 %
    // for the second load per row: profiles/r06d.)
    auto span_record = [&](uint32_t item) -> u32x4 {
      const __amdgpu_buffer_rsrc_t rr = row_rsrc((uint64_t)(uintptr_t)a.span_rec);
      return __builtin_amdgcn_raw_buffer_load_b128(rr, 0, (int)(item * 16u), 0);
    };
    // A block without boundaries: the plain row (W only).  With boundaries:
    // lane k's segment holds at most one (bodies are >= 64 B); occ marks those
    // segments and the boundary in segment k is the block's src-th, src = the
    // bits of occ below k (mbcnt).  The chain also captures cap at the
    // boundary's dword; P1 = the exclusive in-quarter XOR scan of the ST1-shifted
    // segment CRCs; Qp = the XOR of the shifted quarters before this one.
    auto compute_span = [&](bool valid, uint32_t cidx, uint32_t tsk, uint32_t item, u32x4 (&buf)[4],
                            const u32x4 &recv) {
      const uint32_t r0 = (uint32_t)__builtin_amdgcn_readfirstlane((int)recv[0]);
      const uint32_t first = r0 & 0x1FFFFFFu, cnt = RPCCRC_SPAN_ABL ? 0u : r0 >> 25;
      transpose(buf);
      RowMerge m;
      m.rwu = 0u;
      if (cnt == 0u || !valid) {
        m.crc = merge_row(lds, merge_lo(lds, seg_crc(lds, buf, lsel), lsel1), 0u, dl).crc;
      } else {
        const uint32_t rw[3] = {(uint32_t)__builtin_amdgcn_readfirstlane((int)recv[1]),
                                (uint32_t)__builtin_amdgcn_readfirstlane((int)recv[2]),
                                (uint32_t)__builtin_amdgcn_readfirstlane((int)recv[3])};
        uint64_t occ = 0;
        uint32_t pos_l = 0; // > kDenseInline boundaries: lane L < cnt holds boundary L's block offset
        if (cnt <= kDenseInline) {
#pragma unroll
          for (uint32_t i = 0; i < kDenseInline; ++i)
            if (i < cnt) occ |= 1ull << (((rw[i >> 1] >> (16u * (i & 1u))) & 0xFFFu) >> 6);
        } else {
          pos_l = lane < cnt ? (uint32_t)a.span_bpos[first + lane] : 0u;
          uint32_t ol = 0, oh = 0;
          if (lane < cnt) {
            const uint32_t k = pos_l >> 6;
            ol = k < 32u ? 1u << k : 0u;
            oh = k >= 32u ? 1u << (k - 32u) : 0u;
          }
#pragma unroll
          for (int mm = 1; mm < 64; mm <<= 1) {
            ol |= (uint32_t)__shfl_xor((int)ol, mm, 64);
            oh |= (uint32_t)__shfl_xor((int)oh, mm, 64);
          }
          occ = ((uint64_t)(uint32_t)__builtin_amdgcn_readfirstlane((int)oh) << 32) |
                (uint32_t)__builtin_amdgcn_readfirstlane((int)ol);
        }
        const bool has = ((occ >> lane) & 1u) != 0u;
        const uint32_t src = __builtin_amdgcn_mbcnt_hi((uint32_t)(occ >> 32), __builtin_amdgcn_mbcnt_lo((uint32_t)occ, 0u));
        uint32_t pos;
        if (cnt <= kDenseInline) {
          const uint32_t w = src < 2u ? rw[0] : (src < 4u ? rw[1] : rw[2]);
          pos = ((src & 1u) ? (w >> 16) : w) & 0xFFFu;
        } else {
          pos = (uint32_t)__builtin_amdgcn_ds_bpermute((int)(src * 4u), (int)pos_l);
        }
        const uint32_t rr = pos & 63u;
        uint32_t cap;
        const uint32_t c = seg_crc_cap(lds, buf, lsel, has ? rr >> 2 : 16u, 0xFFFFFFFFu << (8u * (rr & 3u)), cap);
        const uint32_t d1 = st1_map(lds, c, lsel1); // A_{64(15-lo)}
        const uint32_t p1 = row_xor_scan(d1) ^ d1;  // exclusive in-quarter prefix
        uint32_t v = d1 ^ dpp_xor1(d1);
        v ^= dpp_xor2(v);
        v ^= dpp_ror4(v);
        v ^= dpp_ror8(v);
        const RowQuarterVals q = merge_quarters(lds, v, dl);
        m.crc = (q.vs[0] ^ q.vs[1]) ^ (q.vs[2] ^ q.vs[3]);
        const uint32_t qp = (hi > 0u ? q.vs[0] : 0u) ^ (hi > 1u ? q.vs[1] : 0u) ^ (hi > 2u ? q.vs[2] : 0u);
        // the boundary's quarter up to it, shifted to the quarter's end:
        // P1 ^ A_{64(15-lo)}(A_{4(16-tb)}(cap)) (cap = 0 in the other lanes)
        const uint32_t eq = p1 ^ st1_map(lds, span_m4(lds, cap, has ? rr >> 2 : 0u), lsel1);
        if (has) a.span_bnd[first + src] = make_uint2(eq, qp);
      }
      finish(valid, kRow, 0u, 1u, 0u, 0u, cidx, tsk, m);
    };

    if constexpr (kSB) {
      // ---- small-body groups (kSB, round 5) ----
      // Tasks are groups of 4 consecutive items.  The items of a group whose
      // end-padded length fits a 1 KiB quarter ("small") share ONE row, one
      // quarter each, computed as a QB = 4 row (P row); the group's other
      // items take their own rows as before (sub-row heads, lane Horner).
      // C2's 1.67M small bodies cost ~420 us of its ~6.2 ms as one row each
      // (tools/c2_subsets.py, profiles/r05j).  Each wave keeps its group's 4
      // CRCs in lanes 0..3 of `gres` and stores them (4 lanes, 16 B) once the
      // group's last row is merged -- no output ring (a group's rows are one
      // wave's, in order).
      const uint32_t ngroups = n_tasks;
      auto item_ol = [&](uint32_t item, uint64_t &off, uint32_t &len) __attribute__((always_inline)) { // (meta()'s loads and routing)
        off = ld_const(a.offsets, item);
        len = ld_const(a.lengths, item);
        if constexpr (kMetaCoissue) __asm__ volatile("" : "+s"(off), "+s"(len));
        if (len >= a.big_min && a.routed != nullptr) {
          const uint32_t bi = a.out_idx ? ld_const(a.out_idx, item) : item;
          if ((ld_const(a.routed, bi >> 5) >> (bi & 31u)) & 1u) len = 0;
        }
      };
      // generator (the producer of stage-m rows): its group, that group's small
      // items (P row) and items with rows of their own (bit b = item 4g + b)
      uint32_t gg = first_task, gsm = 0, gns = 0, gdone = 0;
      uint32_t pend = 0;
      // P row of a group: one descriptor at B (the first small item's 16-B
      // block); quarter b reads item b's 1 KiB window at per-lane offsets
      // d_b + pofs, pieces wholly before the item (pofs + 16 <= front_b) none.
      // (four named scalars each, not arrays: an array a lambda captures by
      // reference went to scratch, and its values to VGPRs -- "illegal VGPR to
      // SGPR copy" for the descriptor base)
      struct Q4 {
        uint32_t v0, v1, v2, v3;
        __device__ uint32_t get(uint32_t b) const { return b == 0 ? v0 : b == 1 ? v1 : b == 2 ? v2 : v3; }
        __device__ void set(uint32_t b, uint32_t x) {
          if (b == 0) v0 = x;
          else if (b == 1) v1 = x;
          else if (b == 2) v2 = x;
          else v3 = x;
        }
      };
      uint64_t pB = 0;
      Q4 pd{0, 0, 0, 0}, pfront{kQuarter, kQuarter, kQuarter, kQuarter};
      uint32_t plzA = 0, plzB = 0;
      // one small-item candidate b: fills its P-row quarter or marks it for rows of its own
      auto classify = [&](uint32_t g, uint32_t b) __attribute__((always_inline)) {
        // (no early returns: the compiler merged `gns |= ` / `gsm |= ` on
        // different paths into a store through a pointer phi -- both went to
        // scratch)
        const bool exists = 4u * g + b < n;
        uint64_t off = 0;
        uint32_t len = 0;
        if (exists) item_ol(4u * g + b, off, len);
        const uint64_t p = (uint64_t)(uintptr_t)a.base + off;
        const uint32_t zb = (uint32_t)(0u - (uint32_t)(p + len)) & 15u;
        const bool fits = exists && len + zb <= kQuarter;
        const uint64_t B = (gsm == 0u) ? (p & ~(uint64_t)15) : pB; // the first small item's 16-B block
        const uint64_t rel = p - B; // items outside [B, B + 1 GiB - 2048) take rows of their own
        const bool small = fits && (rel >> 30) == 0u && (uint32_t)rel < (1u << 30) - 2048u;
        if (small && gsm == 0u) pB = B;
        const uint32_t bit = 1u << b;
        gsm |= small ? bit : 0u;
        gns |= (exists && !small) ? bit : 0u;
        if (small && len != 0u) { // (an empty item: no loads, lz = 0 -> CRC 0 by the algebra)
          pfront.set(b, kQuarter - len - zb);
          pd.set(b, (uint32_t)rel + len + zb - kQuarter);
          const uint32_t lz = (len << 4) | zb;
          if (b < 2) plzA |= lz << (16u * b);
          else plzB |= lz << (16u * (b - 2u));
        }
      };
      auto load_group = [&](uint32_t g) __attribute__((always_inline)) {
        gsm = gns = 0;
        plzA = plzB = 0;
        pd = Q4{0, 0, 0, 0};
        pfront = Q4{kQuarter, kQuarter, kQuarter, kQuarter};
        classify(g, 0);
        classify(g, 1);
        classify(g, 2);
        classify(g, 3);
      };
      // Rows through the pipeline: (item, r, nr, lp, len, z, seed, p0).
      //   item rows: nr >= 1, lp = hd | kGLast on the group's last row.
      //   P rows:    nr = 0, item = 4g, lp = the small mask | kGLast, len / z
      //              = the packed lz words (lz = len << 4 | z, 16 bits each).
      //   invalid:   nr = kNone (past the wave's last group; loads from safe_sb).
      // (No separate ok / flag fields: every SGPR counts -- an earlier version
      // spilled 129 SGPRs and ran 11 % slower, profiles/r05l.)
      constexpr uint32_t kGLast = 0x80000000u, kNone = 0xFFFFFFFFu;
      auto gen = [&](uint32_t pitem, uint32_t pr, uint32_t pnr, uint64_t pp0, uint32_t plp, uint32_t plen,
                     uint32_t pz, uint32_t pseed, uint32_t &item, uint32_t &r, uint32_t &nr, uint64_t &p0,
                     uint32_t &lp, uint32_t &len, uint32_t &z, uint32_t &seed) __attribute__((always_inline)) {
        item = pitem;
        p0 = pp0;
        len = plen;
        z = pz;
        seed = pseed;
        r = 0;
        if (pnr != kNone && pnr != 0u && pr + 1u < pnr) { // the item's next row (metadata reused)
          r = pr + 1u;
          nr = pnr;
          const uint32_t b = pitem & 3u;
          lp = (plp & ~kGLast) | ((r + 1u == nr && (gns >> (b + 1u)) == 0u) ? kGLast : 0u);
          return;
        }
        uint32_t rest = 0;
        if (pnr != kNone) rest = (pnr == 0u) ? gns : (gns & ~((2u << (pitem & 3u)) - 1u));
        nr = kNone;
        lp = 0;
        if (rest == 0u && gdone == 0u) { // the next group
          const uint32_t c = (uint32_t)__builtin_amdgcn_readfirstlane((int)pend);
          gg = dyn_task(c);
          if (gg < ngroups) {
            pend = dyn_grab();
            load_group(gg);
            rest = gns;
            if (gsm != 0u) { // its P row
              item = 4u * gg;
              nr = 0;
              p0 = pB;
              lp = gsm | ((gns == 0u) ? kGLast : 0u);
              len = plzA;
              z = plzB;
              return;
            }
          } else {
            gdone = 1;
          }
        }
        if (rest == 0u) return; // nothing left: an invalid row
        const uint32_t b = (uint32_t)__builtin_ctz(rest);
        item = 4u * gg + b;
        meta(item, p0, lp, len, z, nr, seed);
        lp |= (nr == 1u && (gns >> (b + 1u)) == 0u) ? kGLast : 0u;
      };
      uint64_t safe_sb = 0; // 16-B block of this wave's first bytes: invalid rows load from it
      auto issue_sb = [&](uint64_t p0, uint32_t lp, uint32_t nr, uint32_t r, u32x4 (&buf)[4]) __attribute__((always_inline)) {
        // one load sequence (see issue): whole rows, P rows, first / invalid rows
        const uint32_t hd = lp & ~kGLast;
        uint64_t base;
        uint32_t off[4];
        if (nr != kNone && nr != 0u && !(r == 0u && hd < kRow)) {
          base = p0 + (uint64_t)r * kRow + hd - kRow;
#pragma unroll
          for (int b = 0; b < 4; ++b) off[b] = pofs + b * kQuarter;
        } else if (nr == 0u) {
          base = p0;
#pragma unroll
          for (uint32_t b = 0; b < 4; ++b) off[b] = (pofs + 16u > pfront.get(b)) ? pd.get(b) + pofs : kOobOffset;
        } else {
          const bool ok = nr != kNone;
          base = ok ? (p0 & ~(uint64_t)15) : safe_sb;
          const int32_t d = ok ? (int32_t)(r * kRow + hd) - (int32_t)kRow + (int32_t)(p0 & 15) : INT32_MIN / 2;
#pragma unroll
          for (int b = 0; b < 4; ++b) off[b] = min((uint32_t)(d + (int32_t)(pofs + b * kQuarter)), kOobOffset);
        }
        const __amdgpu_buffer_rsrc_t row = row_rsrc(base);
#pragma unroll
        for (int b = 0; b < 4; ++b) buf[b] = ldb16<NT>(row, off[b]);
      };
      // A P row, all of it (stage c): per 16-lane row hi its item's CRC, valid
      // in lanes 4..7 -- QB = 4's algebra (fix, chain, merge step 1, zlib seed
      // A_{len+z}(F) = ZI_{up-q}(TQ16[up / 16]) with q = len + z, ZI_z, ~).
      auto p_row = [&](uint32_t lzA, uint32_t lzB, u32x4 (&cb)[4]) __attribute__((always_inline)) -> uint32_t {
#pragma unroll
        for (uint32_t b = 0; b < 4; ++b) {
          const uint32_t lz = ((b < 2u ? lzA : lzB) >> (16u * (b & 1u))) & 0xFFFFu;
          const uint32_t len_b = lz >> 4, z_b = lz & 15u;
          if (len_b != 0u) fix_quarter<false>(cb[b], lane, kQuarter - len_b - z_b, z_b);
        }
        transpose(cb);
        const uint32_t ch = row_quarters(lds, cb, lsel, lsel1, upper);
        const uint32_t lzr = ((hi < 2u ? lzA : lzB) >> (16u * (hi & 1u))) & 0xFFFFu;
        const uint32_t q = (lzr >> 4) + (lzr & 15u), up = (q + 15u) & ~15u, zq = up - q, zl = lzr & 15u;
        uint32_t w = lds_ld(lds, kLdsTQ16 + up / 4u);
        {
          const uint32_t nib = (w >> dl.shift) & 15u;
          const uint32_t t = dist_reduce8(lds_ld(lds, kLdsZI2 + (zq != 0u ? zq - 1u : 0u) * 512u + dl.n64 + nib * 4u));
          // lanes 4..7 / 12..15 of each row hold the row's value; row_shl:4 brings it to 0..3 / 8..11
          const uint32_t tb = (uint32_t)__builtin_amdgcn_mov_dpp((int)t, 0x104, 0xF, 0xF, true);
          w = (zq != 0u) ? ((lane & 4u) ? t : tb) : w;
        }
        uint32_t res = ch ^ ((mode == kModeRaw) ? 0u : w);
        {
          const uint32_t nib = (res >> dl.shift) & 15u;
          const uint32_t t = dist_reduce8(lds_ld(lds, kLdsZI2 + (zl != 0u ? zl - 1u : 0u) * 512u + dl.n64 + nib * 4u));
          res = (zl != 0u) ? t : res; // valid in lanes 4..7 of each row
        }
        return (mode == kModeFinal) ? ~res : res;
      };
      uint32_t lacc = 0, gres = 0;
      // stage p: a P row's CRCs into gres, or an item row's lane-Horner step
      // (its CRC on its last row); the group's CRCs stored on its last row
      auto retire = [&](uint32_t item, uint32_t r, uint32_t nr, uint32_t lp, uint32_t z, uint32_t seed,
                        uint32_t chain) __attribute__((always_inline)) {
        if (nr == kNone) return;
        if (nr == 0u) {
          const uint32_t v = (uint32_t)__shfl((int)chain, (int)(16u * (lane & 3u) + 4u), 64);
          if (lane < 4u && ((lp >> lane) & 1u) != 0u) gres = v;
        } else {
          if (r != 0u) {
            lacc = rw_map(lds, lacc) ^ chain;
          } else { // a body's first row starts the accumulator (zlib's seed in lane 63)
            lacc = chain ^ ((lane == 63u) ? seed : 0u);
          }
          if (r + 1u == nr) {
            const RowMerge m = merge_row(lds, merge_lo(lds, lacc, lsel1), 0u, dl);
            uint32_t res = m.crc;
            if (z != 0u) res = dist_uniform(lds, res, kLdsZI2 + (z - 1u) * 512u, dl);
            if (mode == kModeFinal) res = ~res;
            if (lane == (item & 3u)) gres = res;
          }
        }
        if ((lp & kGLast) != 0u) { // the group's last row: its CRCs, 4 lanes
          const uint32_t it = (item & ~3u) + lane;
          if constexpr ((ABL & kRowsAblNoStore) == 0) {
            if (lane < 4u && it < n) store_out(a.out + oidx(it), gres);
          } else {
            sink ^= gres;
          }
        }
      };
      uint32_t c_item = 0, c_r = 0, c_nr = kNone, c_lp = 0, c_len = 0, c_z = 0, c_seed = 0;
      uint32_t n_item, n_r, n_nr, n_lp, n_len, n_z, n_seed;
      uint32_t p_item = 0, p_r = 0, p_nr = kNone, p_lp = 0, p_z = 0, p_seed = 0, p_chain = 0;
      uint64_t c_p0 = 0, n_p0;
      // the first group (gg = first_task): its first row
      load_group(gg);
      gdone = 0;
      if (gsm != 0u) {
        c_item = 4u * gg;
        c_nr = 0;
        c_p0 = pB;
        c_lp = gsm | ((gns == 0u) ? kGLast : 0u);
        c_len = plzA;
        c_z = plzB;
      } else {
        const uint32_t b = (uint32_t)__builtin_ctz(gns);
        c_item = 4u * gg + b;
        meta(c_item, c_p0, c_lp, c_len, c_z, c_nr, c_seed);
        c_lp |= (c_nr == 1u && (gns >> (b + 1u)) == 0u) ? kGLast : 0u;
      }
      safe_sb = c_p0 & ~(uint64_t)15;
      u32x4 bufA[4], bufB[4], bufC[4];
      issue_sb(c_p0, c_lp, c_nr, c_r, bufA);
      if constexpr (kEarly) RPCCRC_ROWS_BEGIN();
      pend = dyn_grab();
      gen(c_item, c_r, c_nr, c_p0, c_lp, c_len, c_z, c_seed, n_item, n_r, n_nr, n_p0, n_lp, n_len, n_z, n_seed);
      issue_sb(n_p0, n_lp, n_nr, n_r, bufB);
      auto step = [&](u32x4 (&cb)[4], u32x4 (&mb)[4]) __attribute__((always_inline)) {
        uint32_t m_item, m_r, m_nr, m_lp, m_len, m_z, m_seed;
        uint64_t m_p0;
        gen(n_item, n_r, n_nr, n_p0, n_lp, n_len, n_z, n_seed, m_item, m_r, m_nr, m_p0, m_lp, m_len, m_z, m_seed);
        issue_sb(m_p0, m_lp, m_nr, m_r, mb);
        uint32_t ch;
        const uint32_t c_hd = c_lp & ~kGLast;
        if (c_nr == 0u) { // P row: four small items, one per quarter (QB = 4 row)
          ch = p_row(c_len, c_z, cb);
        } else {
          fix_row(c_hd, c_z, c_nr, c_r, cb);
          if (c_r == 0 && c_hd <= kQuarter) {
            ch = quarter_row_segs(lds, cb, lsel, sub_jbq, sub_m3);
          } else if (c_r == 0 && c_hd <= 2 * kQuarter) {
            ch = half_row_segs(lds, cb, lsel, sub_mu);
          } else {
            transpose(cb);
            ch = seg_crc(lds, cb, lsel);
          }
        }
        retire(p_item, p_r, p_nr, p_lp, p_z, p_seed, p_chain);
        p_item = c_item;
        p_r = c_r;
        p_nr = c_nr;
        p_lp = c_lp;
        p_z = c_z;
        p_seed = c_seed;
        p_chain = ch;
        c_item = n_item;
        c_r = n_r;
        c_nr = n_nr;
        c_p0 = n_p0;
        c_lp = n_lp;
        c_len = n_len;
        c_z = n_z;
        c_seed = n_seed;
        n_item = m_item;
        n_r = m_r;
        n_nr = m_nr;
        n_p0 = m_p0;
        n_lp = m_lp;
        n_len = m_len;
        n_z = m_z;
        n_seed = m_seed;
      };
      do {
        step(bufA, bufC);
        step(bufB, bufA);
        step(bufC, bufB);
      } while (p_nr != kNone);
    } else {
    // Stealing launches run in two phases (round 5): phase 1 -- the loop
    // compiled WITHOUT the pool protocol -- takes the static rounds up to the
    // one whose first task claims from the pool; phase 2 (the full protocol)
    // starts from the task phase 1 grabbed last and takes the rest.  The pool
    // bookkeeping in the item switch (claims, queue lookups, publishing) then
    // costs only the last ~8 % of a launch: in one loop it made the ragged
    // (C2) kernel's loop 30 % larger and C2 1.8 % slower with stealing than
    // without (profiles/r05w), so C2 ran without it and its exit spread, 380
    // us (odd XCDs ~130 us behind even ones, profiles/r05v), stayed.
    uint32_t pend = 0; // DYN: lane 0 holds the counter index grabbed a task ahead
    const uint32_t p1_lim = steal ? (steal_s - kStealAhead) * kRound : 0xFFFFFFFFu;
    auto rows_phase = [&](auto ph) {
      // 1: plain loop (all of a launch without a pool), 2: pool phase, 3: one
      // loop with the protocol (RPCCRC_TWO_PHASE=0, rounds 2-4)
      constexpr int kPh = decltype(ph)::value;
      constexpr bool kS = STEAL && kPh >= 2; // the pool protocol compiled in
      uint32_t c_item = first_task;
      uint32_t c_c = first_c, m_c = 0; // DYN: counter index of the current / successor item
      // more: the wave may still get work (stealing: a task past n inside a
      // pool round is skipped, not the end).  Invalid rows take one step each.
      bool c_ok = true, c_more = true;
      if constexpr (kPh == 2) { // phase 2 starts at the task phase 1 grabbed and left
        c_c = (uint32_t)__builtin_amdgcn_readfirstlane((int)pend);
        claim_if_first(c_c);
        bool more = false;
        const uint32_t t0 = dyn_map(c_c, more);
        more = __builtin_amdgcn_readfirstlane((int)more) != 0;
        c_more = more;
        c_ok = more && t0 < n;
        if (c_ok) c_item = t0; // (else the first task's metadata: an in-range address)
        if (more) pend = dyn_grab();
      }
      uint64_t c_p0;
      uint32_t c_lp, c_len, c_z, c_nr, c_seed, c_r = 0; // c_lp: the item's first-row bytes (hd)
      meta(c_item, c_p0, c_lp, c_len, c_z, c_nr, c_seed);
      const uint64_t safe = c_p0 & ~(uint64_t)15; // 16-B block holding this wave's first byte
      // Successor of task (item, r) with metadata nr: same item next row, or the
      // wave's next item.  Invalid successors carry the wave's first item's
      // (in-range) metadata and load from `safe`; their results are dropped.
      // After the first row's loads: the image / barrier (kEarly), then the grab
      // of the task after the first one (phase 2 has done both).
#define RPCCRC_ROWS_START()                          \
    do {                                               \
      if constexpr (kPh != 2) {                        \
        if constexpr (kEarly) RPCCRC_ROWS_BEGIN();     \
        if constexpr (DYN) pend = dyn_grab();          \
      }                                                \
    } while (0)
      // cur_*: the current row's item metadata, reused for the item's next row
      // (RAGGED: no reload of its offset / length -- a scalar-load wait in
      // front of every row's loads otherwise).
      auto succ = [&](bool ok, bool more, uint32_t item, uint32_t r, uint32_t nr, uint32_t &s_item, uint32_t &s_r,
                      bool &s_ok, bool &s_more, uint64_t &p0, uint32_t &lp, uint32_t &len, uint32_t &z,
                      uint32_t &snr, uint32_t &seed, uint64_t cur_p0, uint32_t cur_lp, uint32_t cur_len,
                      uint32_t cur_z, uint32_t cur_seed) {
        const bool adv = r + 1 < nr;
        if constexpr (kS) {
          if (adv) {
            s_item = item;
            m_c = c_c;
            // (`ok && s_item < n`, though implied by ok: written as `ok` it made
            // the compiler treat the row base as divergent -- a waterfall loop
            // around every buffer load, ISA)
            s_ok = ok && s_item < n;
            s_more = more;
          } else {
            s_item = n;
            s_more = false;
            if (more) {
              m_c = (uint32_t)__builtin_amdgcn_readfirstlane((int)pend);
              claim_if_first(m_c);
              s_item = dyn_map(m_c, s_more);
              if (s_more) pend = dyn_grab();
            }
            s_ok = s_more && s_item < n;
          }
        } else {
          if constexpr (DYN) {
            if (adv) {
              s_item = item;
              m_c = c_c;
            } else {
              m_c = (uint32_t)__builtin_amdgcn_readfirstlane((int)pend);
              s_item = dyn_task(m_c);
              // phase 1 of a stealing launch ends at the rounds that claim or
              // come from the pool: that task (left in pend) starts phase 2
              if constexpr (STEAL) if (m_c >= p1_lim) s_item = n;
              if (ok && s_item < n) pend = dyn_grab(); // no more grabs once the wave is done
            }
          } else {
            s_item = adv ? item : next_task(item);
          }
          s_ok = ok && s_item < n;
          s_more = s_ok;
        }
        if (kRowsMetaReuse && RAGGED && adv) {
          p0 = cur_p0;
          lp = cur_lp;
          len = cur_len;
          z = cur_z;
          snr = nr;
          seed = cur_seed;
        } else {
          meta(s_ok ? s_item : first_task, p0, lp, len, z, snr, seed);
        }
        if (steal && !s_ok) snr = 1u;
        s_r = adv ? r + 1 : 0u;
      };
      // The unrolled loops have ONE exit, at the bottom: a mid-body break edge
      // (structurized back through the loop header) would carry the first
      // half's in-flight prefetch into the header, and the compiler would then
      // drain vmcnt before every prefetch (measured: rows fully serialised on
      // half the iterations).  Trailing steps past the wave's last task run on
      // invalid tasks (c_ok false): safe loads, no result parked.
      // Ragged batches only: C2 -1.6 %, while uniform batches (north star
      // +-0.5 %, C4's chunks +0.6 %) keep the plain loop
      // (profiles/r02/r02r_rows_pipeline_ab.txt).
      constexpr bool kPipe = kRowsPipe && (RAGGED || kUniformPipe) && !kTwoChains &&
                             (ABL & (kRowsAblNoCompute | kRowsAblNoMerge | kRowsAblNoTranspose)) == 0;
      // Row C's chain (full / half / quarter row, rows::*_row_segs) and row P's
      // merge, inside each arm so the scheduler overlaps it with C's chain (P's
      // merge before or after the arms: C2 +1.3 % with the max-ilp scheduler,
      // profiles/r03m).
#define RPCCRC_CHAIN_MERGE(cb, ch, pm)                                                   \
    do {                                                                                   \
      if (kSub && c_r == 0 && c_lp <= kQuarter) {                                          \
        ch = quarter_row_segs(lds, cb, lsel, sub_jbq, sub_m3);                             \
        pm = merge_row(lds, merge_lo(lds, p_chain, lsel1), W, dl);                         \
      } else if (kSub && c_r == 0 && c_lp <= 2 * kQuarter) {                               \
        ch = half_row_segs(lds, cb, lsel, sub_mu);                                         \
        pm = merge_row(lds, merge_lo(lds, p_chain, lsel1), W, dl);                         \
      } else {                                                                             \
        transpose(cb);                                                                     \
        ch = seg_crc(lds, cb, lsel);                                                       \
        pm = merge_row(lds, merge_lo(lds, p_chain, lsel1), W, dl);                         \
      }                                                                                    \
    } while (0)
      // Lane Horner (kLH): C's chain only, then row P joins its body's per-lane
      // accumulator (A_4096 on every row but the first; zlib's seed enters in
      // lane 63, whose merge shift is A_0), and the body's last row is merged
      // once: crc0(body) = XOR_L' A_{64(63-L')}(acc_L').
      constexpr bool kLH = kLaneHorner && kSub;
      uint32_t lacc = 0; // kLH: this wave's per-lane accumulator of row P's body
      // (row P's lane-Horner step after C's arms: inside each arm measured
      // -0.2 % against -0.5 % here, profiles/r03p)
#define RPCCRC_CHAIN_ONLY(cb, ch)                                                        \
    do {                                                                                   \
      if constexpr ((ABL & kRowsAblPipeMem) != 0) {                                        \
        ch = xor_fold(cb);                                                                 \
      } else if (kSub && c_r == 0 && c_lp <= kQuarter) {                                   \
        ch = quarter_row_segs(lds, cb, lsel, sub_jbq, sub_m3);                             \
      } else if (kSub && c_r == 0 && c_lp <= 2 * kQuarter) {                               \
        ch = half_row_segs(lds, cb, lsel, sub_mu);                                         \
      } else {                                                                             \
        transpose(cb);                                                                     \
        ch = seg_crc(lds, cb, lsel);                                                       \
      }                                                                                    \
      lane_horner_p(p_ok, p_z, p_nr, p_r, p_seed, p_c, p_item, p_chain);                   \
    } while (0)
      auto lane_horner_p = [&](bool ok, uint32_t z, uint32_t nr, uint32_t r, uint32_t seed, uint32_t cidx,
                               uint32_t tsk, uint32_t chain) {
        if constexpr ((ABL & kRowsAblPipeMem) != 0) {
          lacc = (r != 0 ? lacc : seed) ^ chain;
          if (r + 1 == nr) {
            const uint32_t res = (uint32_t)__builtin_amdgcn_readfirstlane((int)lacc);
            if constexpr (DYN) {
              if (ok) dyn_out(cidx, tsk, res);
            } else {
              if (ok) park(res);
            }
          }
          return;
        }
        if (r != 0) {
          lacc = rw_map(lds, lacc) ^ chain;
        } else { // a body's first row starts the accumulator (zlib's seed in lane 63)
          if constexpr (kLdsSeed) { // seed holds hd: A_hd(F) = ZI_{up - hd}(TQ16[up / 16])
            const uint32_t up = (seed + 15u) & ~15u;
            uint32_t w = lds_ld(lds, kLdsTQ16 + up / 4u);
            if (up != seed) w = dist_uniform(lds, w, kLdsZI2 + (up - seed - 1u) * 512u, dl);
            seed = (mode == kModeRaw) ? 0u : (uint32_t)__builtin_amdgcn_readfirstlane((int)w);
          }
          lacc = chain ^ ((lane == 63u) ? seed : 0u);
        }
        if (r + 1 == nr) {
          const RowMerge m = merge_row(lds, merge_lo(lds, lacc, lsel1), 0u, dl);
          uint32_t res = m.crc;
          if (z != 0) res = dist_uniform(lds, res, kLdsZI2 + (z - 1u) * 512u, dl);
          if (mode == kModeFinal) res = ~res;
          if constexpr (DYN) {
            if (ok) dyn_out(cidx, tsk, res);
          } else {
            if (ok) park(res);
          }
        }
      };
      if constexpr (DEPTH == 1 && kPipe && kRaggedAhead2) {
        // The pipeline below with loads two rows ahead: one step issues row M's
        // loads while row N's (the row after C) are in flight, chains row C and
        // merges row P.  A wave then keeps a row of loads in flight while it
        // computes, also across item switches (C2's memory-only variant runs
        // 5.79 ms against 6.33 for the product with one row ahead).
        u32x4 bufA[4], bufB[4], bufC[4];
        issue(c_p0, c_lp, c_nr, c_r, c_ok, safe, bufA);
        RPCCRC_ROWS_START();
        uint32_t n_item, n_lp, n_r, n_len, n_z, n_nr, n_seed, n_c;
        uint64_t n_p0;
        bool n_ok, n_more;
        succ(c_ok, c_more, c_item, c_r, c_nr, n_item, n_r, n_ok, n_more, n_p0, n_lp, n_len, n_z, n_nr, n_seed, c_p0,
             c_lp, c_len, c_z, c_seed);
        n_c = m_c;
        issue(n_p0, n_lp, n_nr, n_r, n_ok, safe, bufB);
        bool p_ok = false; // no row pending before the first step
        uint32_t p_len = 0, p_z = 0, p_nr = 1, p_r = 0, p_seed = 0, p_c = 0, p_item = 0, p_chain = 0;
        auto step = [&](u32x4 (&cb)[4], u32x4 (&mb)[4]) {
          uint32_t m_item, m_lp;
          uint64_t m_p0;
          uint32_t m_r, m_len, m_z, m_nr, m_seed;
          bool m_ok, m_more;
          // succ() tracks the DYN counter index of the row it is given in c_c
          // and leaves the successor's in m_c
          const uint32_t cc = c_c;
          c_c = n_c;
          succ(n_ok, n_more, n_item, n_r, n_nr, m_item, m_r, m_ok, m_more, m_p0, m_lp, m_len, m_z, m_nr, m_seed, n_p0,
               n_lp, n_len, n_z, n_seed);
          c_c = cc;
          issue(m_p0, m_lp, m_nr, m_r, m_ok, safe, mb);
          fix_row(c_lp, c_z, c_nr, c_r, cb);
          uint32_t ch;
          if constexpr (kLH) {
            RPCCRC_CHAIN_ONLY(cb, ch);
          } else {
            RowMerge pm;
            RPCCRC_CHAIN_MERGE(cb, ch, pm);
            finish(p_ok, p_len, p_z, p_nr, p_r, p_seed, p_c, p_item, pm);
          }
          publish();
          p_ok = c_ok;
          p_len = c_len;
          p_z = c_z;
          p_nr = c_nr;
          p_r = c_r;
          p_seed = c_seed;
          p_c = c_c;
          p_item = c_item;
          p_chain = ch;
          c_c = n_c;
          c_ok = n_ok;
          c_more = n_more;
          c_seed = n_seed;
          c_item = n_item;
          c_r = n_r;
          c_p0 = n_p0;
          c_lp = n_lp;
          c_len = n_len;
          c_z = n_z;
          c_nr = n_nr;
          n_c = m_c;
          n_ok = m_ok;
          n_more = m_more;
          n_seed = m_seed;
          n_item = m_item;
          n_r = m_r;
          n_p0 = m_p0;
          n_lp = m_lp;
          n_len = m_len;
          n_z = m_z;
          n_nr = m_nr;
        };
        do {
          step(bufA, bufC);
          step(bufB, bufA);
          step(bufC, bufB);
        } while ((kS && steal) ? (n_more || c_more || p_ok) : p_ok);
      } else if constexpr (DEPTH == 1 && kPipe) {
        // Software pipeline over rows: one step issues row M's loads, runs row
        // C's edge fix, transpose and chain, and merges row P (the row before C,
        // whose chain the previous step computed).  C's chain and P's merge are
        // independent and share one basic block, so the scheduler overlaps P's
        // dependent merge lookups with C's chain.  Rows still finish in order
        // (Horner across rows needs that).
        u32x4 bufA[4], bufB[4];
        issue(c_p0, c_lp, c_nr, c_r, c_ok, safe, bufA);
        RPCCRC_ROWS_START();
        bool p_ok = false; // no row pending before the first step
        uint32_t p_len = 0, p_z = 0, p_nr = 1, p_r = 0, p_seed = 0, p_c = 0, p_item = 0, p_chain = 0;
        auto step = [&](u32x4 (&cb)[4], u32x4 (&nb)[4]) {
          uint32_t m_item, m_lp;
          uint64_t m_p0;
          uint32_t m_r, m_len, m_z, m_nr, m_seed;
          bool m_ok, m_more;
          succ(c_ok, c_more, c_item, c_r, c_nr, m_item, m_r, m_ok, m_more, m_p0, m_lp, m_len, m_z, m_nr, m_seed, c_p0,
               c_lp, c_len, c_z, c_seed);
          issue(m_p0, m_lp, m_nr, m_r, m_ok, safe, nb);
          fix_row(c_lp, c_z, c_nr, c_r, cb);
          uint32_t ch;
          if constexpr (kLH) {
            RPCCRC_CHAIN_ONLY(cb, ch);
          } else {
            RowMerge pm;
            RPCCRC_CHAIN_MERGE(cb, ch, pm);
            finish(p_ok, p_len, p_z, p_nr, p_r, p_seed, p_c, p_item, pm);
          }
          publish();
          p_ok = c_ok;
          p_len = c_len;
          p_z = c_z;
          p_nr = c_nr;
          p_r = c_r;
          p_seed = c_seed;
          p_c = c_c;
          p_item = c_item;
          p_chain = ch;
          c_c = m_c;
          c_ok = m_ok;
          c_more = m_more;
          c_seed = m_seed;
          c_item = m_item;
          c_r = m_r;
          c_p0 = m_p0;
          c_lp = m_lp;
          c_len = m_len;
          c_z = m_z;
          c_nr = m_nr;
        };
        do {
          step(bufA, bufB);
          step(bufB, bufA);
        } while ((kS && steal) ? (c_more || p_ok) : p_ok);
      } else if constexpr (DEPTH == 1) {
        u32x4 bufA[4], bufB[4];
        u32x4 recA = {0u, 0u, 0u, 0u}, recB = {0u, 0u, 0u, 0u}; // kSpan: the rows' block records
        issue(c_p0, c_lp, c_nr, c_r, c_ok, safe, bufA);
        if constexpr (kSpan && RPCCRC_SPAN_ABL < 2) recA = span_record(c_ok ? c_item : first_task);
        RPCCRC_ROWS_START();
        auto step = [&](u32x4 (&cb)[4], u32x4 (&nb)[4], u32x4 &crec, u32x4 &nrec) {
          uint32_t m_item, m_lp;
          uint64_t m_p0;
          uint32_t m_r, m_len, m_z, m_nr, m_seed;
          bool m_ok, m_more;
          succ(c_ok, c_more, c_item, c_r, c_nr, m_item, m_r, m_ok, m_more, m_p0, m_lp, m_len, m_z, m_nr, m_seed, c_p0,
               c_lp, c_len, c_z, c_seed);
          issue(m_p0, m_lp, m_nr, m_r, m_ok, safe, nb);
          if constexpr (kSpan) {
            if constexpr (RPCCRC_SPAN_ABL < 2) nrec = span_record(m_ok ? m_item : first_task);
            compute_span(c_ok, c_c, c_item, c_item, cb, crec);
          } else {
            compute(c_ok, c_lp, c_len, c_z, c_nr, c_r, c_seed, c_c, c_item, cb);
          }
          publish();
          c_c = m_c;
          c_ok = m_ok;
          c_more = m_more;
          c_seed = m_seed;
          c_item = m_item;
          c_r = m_r;
          c_p0 = m_p0;
          c_lp = m_lp;
          c_len = m_len;
          c_z = m_z;
          c_nr = m_nr;
        };
        do {
          step(bufA, bufB, recA, recB);
          step(bufB, bufA, recB, recA);
        } while ((kS && steal) ? c_more : c_ok);
      } else {
        // DEPTH = 2: the next two rows' loads are in flight while one computes.
        u32x4 bufA[4], bufB[4], bufC[4];
        uint32_t n_item, n_lp;
        uint64_t n_p0;
        uint32_t n_r, n_len, n_z, n_nr, n_seed;
        bool n_ok, n_more;
        issue(c_p0, c_lp, c_nr, c_r, c_ok, safe, bufA);
        RPCCRC_ROWS_START();
        succ(true, true, c_item, c_r, c_nr, n_item, n_r, n_ok, n_more, n_p0, n_lp, n_len, n_z, n_nr, n_seed, c_p0, c_lp,
             c_len, c_z, c_seed);
        issue(n_p0, n_lp, n_nr, n_r, n_ok, safe, bufB);
        auto step = [&](u32x4 (&cb)[4], u32x4 (&fb)[4]) {
          uint32_t m_item, m_lp;
          uint64_t m_p0;
          uint32_t m_r, m_len, m_z, m_nr, m_seed;
          bool m_ok, m_more;
          succ(n_ok, n_more, n_item, n_r, n_nr, m_item, m_r, m_ok, m_more, m_p0, m_lp, m_len, m_z, m_nr, m_seed, n_p0,
               n_lp, n_len, n_z, n_seed);
          issue(m_p0, m_lp, m_nr, m_r, m_ok, safe, fb);
          compute(c_ok, c_lp, c_len, c_z, c_nr, c_r, c_seed, 0, c_item, cb);
          c_ok = n_ok;
          c_seed = n_seed;
          n_seed = m_seed;
          c_item = n_item;
          c_r = n_r;
          c_lp = n_lp;
          c_len = n_len;
          c_z = n_z;
          c_nr = n_nr;
          n_ok = m_ok;
          n_item = m_item;
          n_r = m_r;
          n_p0 = m_p0;
          n_lp = m_lp;
          n_len = m_len;
          n_z = m_z;
          n_nr = m_nr;
        };
        do {
          step(bufA, bufC);
          step(bufB, bufA);
          step(bufC, bufB);
        } while (c_ok);
      }
    };
    if constexpr (STEAL && (!kTwoPhase || (kSpan && !RPCCRC_SPAN_TWO_PHASE))) { // (the span pass is device-counted: one loop)
      rows_phase(std::integral_constant<int, 3>{});
    } else if constexpr (STEAL && kSpan) {
      // the dense span pass (device-counted, its pool sized in the kernel): two
      // phases, and only those two compiled (phase 3 beside them took the
      // kernel to 128 VGPRs and scratch; these two: 103 VGPRs, no scratch)
      rows_phase(std::integral_constant<int, 1>{});
      if (steal) rows_phase(std::integral_constant<int, 2>{});
    } else if constexpr (STEAL) {
      // Device-counted launches (the big-body route's chunk and span passes)
      // keep one loop, as in rounds 2-4: lifted-cap frames ran 1-2 % slower with
      // two phases (profiles/r05fl2).
      if (a.steal_s == kStealOnDevice) {
        rows_phase(std::integral_constant<int, 3>{});
      } else {
        rows_phase(std::integral_constant<int, 1>{});
        if (steal) rows_phase(std::integral_constant<int, 2>{});
      }
    } else {
      rows_phase(std::integral_constant<int, 1>{});
    }
    } // (!kSB)
    publish();
    flush();
    if constexpr ((ABL & kRowsAblNoStore) != 0)
      if (sink == 0x9E3779B9u) a.out[gw] = sink; // keeps the results live
    if constexpr ((ABL & kRowsAblTimes) != 0) {
      // (ragged batches need their offsets: the probe passes the times array in round_out)
      uint64_t *times = RAGGED ? reinterpret_cast<uint64_t *>(a.round_out) : const_cast<uint64_t *>(a.offsets);
      const uint64_t t_exit = __builtin_amdgcn_s_memrealtime();
      const uint64_t c_exit = __builtin_amdgcn_s_memtime();
      if (lane == 0) {
        times[4 * gw + 0] = t_entry;
        times[4 * gw + 1] = t_image;
        times[4 * gw + 2] = t_exit;
        times[4 * gw + 3] = (uint64_t)j0 | ((c_exit - c_entry) << 24); // tasks | shader cycles
      }
    }
  } else {
    // QB = 4: group g = items [4g, 4g+4), quarter b <-> item 4g+b (len + pad <= 1 KiB).
    const uint32_t ngroups = (n + 3) / 4;
    auto quarter = [&](uint32_t g, int b) -> QuarterInfo {
      QuarterInfo r;
      const uint32_t item = 4 * g + b;
      const bool ok = item < n;
      const uint32_t it = ok ? item : 0;
      const uint64_t off = RAGGED ? ld_const(a.offsets, it) : (uint64_t)it * a.stride;
      const uint32_t len = RAGGED ? ld_const(a.lengths, it) : a.len;
      r.len = ok ? len : 0u;
      r.p0 = a.base + off;
      r.z = (uint32_t)(0u - (uint32_t)(uintptr_t)(r.p0 + r.len)) & 15u;
      r.vstart = (int64_t)r.len + r.z - (int64_t)kQuarter;
      return r;
    };
    // issue() loads group g's row and returns what compute() needs, so item
    // metadata is read once per group, a row ahead of its use: per quarter
    // lz[b] = (len << 4) | z (len 0 = no item), and the lane-selected zlib
    // seeds A_{len_b+z_b}(0xFFFFFFFF) (scalar loads from the global Tq table).
    struct QuadMeta {
      uint32_t lz[4];
      uint32_t sl;
    };
    // Uniform batches with stride % 4 == 0: quarter b of group g is item 4g+b
    // at base + (4g+b) * stride, and its end pad z_b = -(base + b*stride +
    // len) mod 16 is the same for every g (4 * stride is a multiple of 16).
    // So lz[b], the seeds and `full` are computed once, and a group whose four
    // items all exist costs one 64-bit multiply instead of four quarter()
    // calls and four seed loads (C1: the QB = 4 rows were bound by the scalar
    // unit, PMC ~2.7x the SALU of a QB = 1 row).
    const bool affine = !RAGGED && (a.stride % 4u) == 0;
    QuadMeta aqm;
    aqm.sl = 0;
    // Uniform batches (round 4): ONE buffer descriptor per row, at B = the 16-B
    // block holding body 4g's first byte.  Quarter b reads body 4g+b's window
    // (the 1 KiB ending at the body's 16-B-rounded end) at offsets
    // (p_b - B) - front_b + 16k, front_b = 1024 - len - z_b the window offset of
    // the body's first byte; pieces wholly before the body get the out-of-range
    // offset (zeros), exactly as with a descriptor per quarter (rounds 1-3: four
    // descriptors, 16 SGPRs, and per-quarter 64-bit bases kept live -- the C1
    // kernel spilled 31 SGPRs).  Affine batches (stride % 4 == 0, so 4 * stride
    // keeps the 16-B phase): the offsets do not depend on g, one VGPR each.
    uint32_t aoff[4] = {kOobOffset, kOobOffset, kOobOffset, kOobOffset};
    if constexpr (!RAGGED) {
      const uint32_t ph = (uint32_t)(uintptr_t)a.base & 15u;
#pragma unroll
      for (int b = 0; b < 4; ++b) {
        const uint32_t z = (uint32_t)(0u - (uint32_t)((uintptr_t)a.base + (uint64_t)b * a.stride + a.len)) & 15u;
        const uint32_t front = kQuarter - a.len - z; // window offset of the body's first byte
        aoff[b] = (a.len == 0u || pofs + 16u <= front) ? kOobOffset : ph + (uint32_t)b * (uint32_t)a.stride + pofs - front;
        aqm.lz[b] = (a.len << 4) | z;
        const uint32_t seed = (mode == kModeRaw) ? 0u : ld_const(a.tq, a.len + z);
        aqm.sl = (hi == (uint32_t)b) ? seed : aqm.sl;
      }
    }
    auto issue = [&](uint32_t g, bool ok, uint64_t safe, u32x4 (&buf)[4]) -> QuadMeta {
      QuadMeta qm;
      qm.sl = 0;
      if constexpr (!RAGGED) {
        uint64_t B = safe;
        uint32_t off[4] = {kOobOffset, kOobOffset, kOobOffset, kOobOffset};
#pragma unroll
        for (int b = 0; b < 4; ++b) qm.lz[b] = 0u;
        if (ok) {
          const uint64_t p0 = (uint64_t)(uintptr_t)a.base + (uint64_t)g * 4u * a.stride;
          B = p0 & ~(uint64_t)15;
          if (affine && 4 * g + 4 <= n) {
#pragma unroll
            for (int b = 0; b < 4; ++b) off[b] = aoff[b];
            qm = aqm;
          } else { // a last partial group, or a stride that moves the 16-B phase
#pragma unroll
            for (int b = 0; b < 4; ++b) {
              const bool live = 4 * g + b < n && a.len != 0u;
              const uint32_t rel = (uint32_t)(p0 & 15u) + (uint32_t)b * (uint32_t)a.stride; // p_b - B
              const uint32_t z = (uint32_t)(0u - (uint32_t)(p0 + (uint64_t)b * a.stride + a.len)) & 15u;
              const uint32_t front = kQuarter - a.len - z;
              off[b] = (!live || pofs + 16u <= front) ? kOobOffset : rel + pofs - front;
              qm.lz[b] = live ? (a.len << 4) | z : 0u;
              const uint32_t seed = (mode == kModeRaw || !live) ? 0u : ld_const(a.tq, a.len + z);
              qm.sl = (hi == (uint32_t)b) ? seed : qm.sl;
            }
          }
        }
        if constexpr ((ABL & kRowsAblNoLoad) != 0) {
          synth(g, buf);
        } else {
          const __amdgpu_buffer_rsrc_t row = row_rsrc(B);
#pragma unroll
          for (int b = 0; b < 4; ++b) buf[b] = ldb16<NT>(row, off[b]);
        }
        return qm;
      }
      QuarterInfo qi[4];
      bool full = ok;
#pragma unroll
      for (int b = 0; b < 4; ++b) {
        qi[b] = quarter(g, b);
        full = full && qi[b].vstart == 0 && qi[b].len != 0;
        qm.lz[b] = (qi[b].len << 4) | qi[b].z;
        const uint32_t seed = (mode == kModeRaw) ? 0u : ld_const(a.tq, qi[b].len + qi[b].z);
        qm.sl = (hi == (uint32_t)b) ? seed : qm.sl;
      }
      if constexpr ((ABL & kRowsAblNoLoad) != 0) {
        synth(g, buf);
      } else {
        // One load sequence (see QB = 1): per quarter a uniform base (the item's
        // first 16-B block) and per-lane offsets, zeros before the item.
        uint64_t base[4];
        uint32_t off[4];
        if (full) { // four whole 1 KiB items: scalar bases, constant lane offset
#pragma unroll
          for (int b = 0; b < 4; ++b) {
            base[b] = (uint64_t)(uintptr_t)qi[b].p0;
            off[b] = pofs;
          }
        } else {
#pragma unroll
          for (int b = 0; b < 4; ++b) {
            const uint64_t p = (uint64_t)(uintptr_t)qi[b].p0;
            const bool live = ok && qi[b].len != 0;
            base[b] = live ? (p & ~(uint64_t)15) : safe;
            const int32_t o = live ? (int32_t)(qi[b].vstart + (int64_t)(p & 15)) + (int32_t)pofs : -1;
            off[b] = min((uint32_t)o, kOobOffset);
          }
        }
#pragma unroll
        for (int b = 0; b < 4; ++b) buf[b] = ldb16<NT>(row_rsrc(base[b]), off[b]);
      }
      return qm;
    };
    // Parked results: lane k = item 4 * (gw + (j0 + k / 4) * nwaves) + k % 4 (see QB = 1).
    uint32_t outv = 0, ocount = 0;
    uint32_t j0 = 0;
    // DYN output (see QB = 1): the 4 CRCs of group task c into the LDS ring; the
    // wave completing a round stores its (up to) 128 CRCs as two 256-B stores.
    auto dyn_out4 = [&](uint32_t c, uint32_t tsk, const uint32_t (&v)[4]) {
      constexpr uint32_t kW = kRound * 4; // CRCs per round (64 or 128)
      const uint32_t rnd = (uint32_t)(c / kRound), idx = (uint32_t)(c % kRound), slot = rnd % kDynSlots;
      uint32_t *done = s_ctl + 1 + slot, *gen = s_ctl + kGen;
      uint32_t *ring = s_ctl + kRingBuf + slot * kW;
      uint32_t old = 0;
      publish(); // the ring wait below must not hold a claim
      if (lane == 0) {
        ring_wait(gen, slot, rnd);
#pragma unroll
        for (int b = 0; b < 4; ++b) ring[idx * 4 + b] = v[b];
        old = __hip_atomic_fetch_add(done, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
      }
      old = (uint32_t)__builtin_amdgcn_readfirstlane((int)old);
      // first group of the round (rounds are aligned)
      const uint32_t base = tsk & ~(kRound - 1u);
      const uint32_t cnt = (ngroups - base < kRound) ? (uint32_t)(ngroups - base) : kRound;
      if (old + 1u == cnt) {
        const uint32_t ibase = 4 * base;
        const uint32_t nit = (n - ibase < kW) ? (uint32_t)(n - ibase) : kW;
        const uint32_t v0 = ring[lane];
        if (lane < nit) store_out(a.out + oidx(ibase + lane), v0);
        if constexpr (kW > 64) {
          const uint32_t v1 = ring[64 + lane];
          if (64 + lane < nit) store_out(a.out + oidx(ibase + 64 + lane), v1);
        }
        if (lane == 0) {
          *done = 0;
          __hip_atomic_store(&gen[slot], rnd + kDynSlots, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
        }
        j0 += cnt;
      }
    };
    auto flush = [&]() {
      const uint32_t item = 4 * task_of(j0 + lane / 4u) + (lane & 3u);
      if (lane < ocount && item < n) a.out[oidx(item)] = outv;
      j0 += ocount / 4u;
      ocount = 0;
    };
    auto compute = [&](const QuadMeta &qm, bool valid, uint32_t cidx, uint32_t tsk, u32x4 (&buf)[4]) {
      uint32_t zl = 0, zany = 0;
#pragma unroll
      for (int b = 0; b < 4; ++b) {
        const uint32_t len = qm.lz[b] >> 4, z = qm.lz[b] & 15u;
        // the item's first byte sits at quarter offset kQuarter - len - z (empty
        // quarters read zeros: out-of-range loads)
        if (len != 0u) fix_quarter<(ABL & kRowsAblNaturalOrder) != 0>(buf[b], lane, kQuarter - len - z, z);
        zany |= z;
        zl = (hi == (uint32_t)b) ? z : zl;
      }
      uint32_t res = quarter_crcs(buf) ^ qm.sl; // 16-lane row b: item 4g+b
      if (zany != 0) {
        // Undo the z_b pad bytes of each row's item: distributed nibble step
        // within each row (rows with z_b = 0 keep res; their lookup hits RW2).
        const uint32_t nib = (res >> dl.shift) & 15u;
        const uint32_t t = dist_reduce8(lds_ld(lds, kLdsZI2 + (zl - 1u) * 512u + dl.n64 + nib * 4u));
        res = (zl != 0u) ? t : res; // valid in lanes 4..7 of each row
      }
      if (mode == kModeFinal) res = ~res;
      uint32_t vals[4];
#pragma unroll
      for (int b = 0; b < 4; ++b) {
        uint32_t v = __builtin_amdgcn_readlane(res, 16 * b + 4);
        if ((qm.lz[b] >> 4) == 0) v = 0u;
        vals[b] = v;
      }
      if (!valid) return; // a trailing step past the wave's last group
      if constexpr (DYN) {
        dyn_out4(cidx, tsk, vals);
      } else {
#pragma unroll
        for (int b = 0; b < 4; ++b) outv = (lane == ocount + (uint32_t)b) ? vals[b] : outv;
        ocount += 4;
        if (ocount == 64u) flush();
      }
    };
    uint32_t g = first_task;
    const uint64_t safe = (uint64_t)(uintptr_t)quarter(g, 0).p0 & ~(uint64_t)15;
    if constexpr (DEPTH == 1) {
      // Stealing launches in two phases as QB = 1 (the loop without the pool
      // protocol, then the one with it) only with RPCCRC_QB4_TWO_PHASE=1: C1's
      // launches are 32 rounds a workgroup, and the pipeline drain and refill
      // at the phase switch cost more than the cheaper static loop saves (C1
      // +0.5 %, profiles/r05zc).  Phase 3: one loop with the protocol.
      uint32_t pend = 0;
      const uint32_t p1_lim = steal ? (steal_s - kStealAhead) * kRound : 0xFFFFFFFFu;
      const uint32_t g0 = g;
      auto rows_phase4 = [&](auto ph) {
        constexpr int kPh = decltype(ph)::value;
        constexpr bool kS = STEAL && kPh >= 2;
        u32x4 bufA[4], bufB[4];
        uint32_t c_c = first_c;
        bool c_ok = true;   // the group being computed next is real
        bool c_more = true; // stealing: the wave may still get groups (a group past the end is skipped)
        QuadMeta c_qm;
        if constexpr (kPh == 2) { // from the task phase 1 grabbed and left
          c_c = (uint32_t)__builtin_amdgcn_readfirstlane((int)pend);
          claim_if_first(c_c);
          bool more = false;
          const uint32_t t0 = dyn_map(c_c, more);
          more = __builtin_amdgcn_readfirstlane((int)more) != 0;
          c_more = more;
          c_ok = more && t0 < ngroups;
          g = c_ok ? t0 : g0;
          if (more) pend = dyn_grab();
          c_qm = issue(g, c_ok, safe, bufA);
        } else {
          c_qm = issue(g, true, safe, bufA);
          if constexpr (kEarly) RPCCRC_ROWS_BEGIN();
          if constexpr (DYN) pend = dyn_grab();
        }
        // One exit, at the bottom (see QB = 1): a mid-body break made the
        // compiler drain vmcnt before the next group's loads on every step
        // (ISA: s_waitcnt vmcnt(0) ahead of the offset of the 4th quarter load).
        // Steps past the wave's last group load nothing and store nothing.
        auto step = [&](u32x4 (&cb)[4], u32x4 (&nb)[4]) {
          uint32_t ng, n_c = 0;
          bool ok, more = false;
          if constexpr (kS) {
            ng = ngroups;
            if (c_more) {
              n_c = (uint32_t)__builtin_amdgcn_readfirstlane((int)pend);
              claim_if_first(n_c);
              ng = dyn_map(n_c, more);
              if (more) pend = dyn_grab();
            }
            // uniform again after the lane-0 grab (else the compiler carried
            // `more` as a lane mask and the group index went to VGPRs)
            more = __builtin_amdgcn_readfirstlane((int)more) != 0;
            ok = more && ng < ngroups;
          } else {
            if constexpr (DYN) {
              n_c = (uint32_t)__builtin_amdgcn_readfirstlane((int)pend);
              ng = dyn_task(n_c);
              if constexpr (STEAL) if (n_c >= p1_lim) ng = ngroups; // phase 1 ends (as QB = 1)
            } else {
              ng = next_task(g);
            }
            ok = c_ok && ng < ngroups;
            // the next group as an SGPR before the lane-0 grab: the compiler
            // otherwise sank its select into the grab's exec-masked region
            // and carried the group index in a VGPR (the loop's SALU work
            // went to the VALU, ISA)
            uint32_t gn = ok ? ng : g;
            __asm__ volatile("" : "+s"(gn));
            ng = gn;
            if constexpr (DYN)
              if (ok) pend = dyn_grab();
          }
          if constexpr (kS) ng = ok ? ng : g;
          const QuadMeta n_qm = issue(ng, ok, safe, nb);
          compute(c_qm, c_ok, c_c, g, cb);
          publish();
          c_qm = n_qm;
          g = ng;
          c_c = n_c;
          c_ok = ok;
          c_more = more;
        };
        do {
          step(bufA, bufB);
          step(bufB, bufA);
        } while ((kS && steal) ? c_more : c_ok);
      };
      if constexpr (STEAL && !kQb4TwoPhase) {
        rows_phase4(std::integral_constant<int, 3>{});
      } else {
        rows_phase4(std::integral_constant<int, 1>{});
        if constexpr (STEAL)
          if (steal) rows_phase4(std::integral_constant<int, 2>{});
      }
    } else {
      u32x4 bufA[4], bufB[4], bufC[4];
      QuadMeta c_qm = issue(g, true, safe, bufA), n_qm;
      if constexpr (kEarly) RPCCRC_ROWS_BEGIN();
      uint32_t gn = next_task(g);
      n_qm = issue(gn < ngroups ? gn : g, gn < ngroups, safe, bufB);
      auto step = [&](u32x4 (&cb)[4], u32x4 (&fb)[4]) -> bool {
        const uint32_t g2 = next_task(gn);
        const bool ok2 = g2 < ngroups;
        const QuadMeta m_qm = issue(ok2 ? g2 : g, ok2, safe, fb);
        compute(c_qm, true, 0, g, cb);
        c_qm = n_qm;
        n_qm = m_qm;
        g = gn;
        gn = g2;
        return g < ngroups;
      };
      for (;;) {
        if (!step(bufA, bufC)) break;
        if (!step(bufB, bufA)) break;
        if (!step(bufC, bufB)) break;
      }
    }
    publish();
    flush();
    if constexpr ((ABL & kRowsAblTimes) != 0) {
      // (ragged batches need their offsets: the probe passes the times array in round_out)
      uint64_t *times = RAGGED ? reinterpret_cast<uint64_t *>(a.round_out) : const_cast<uint64_t *>(a.offsets);
      const uint64_t t_exit = __builtin_amdgcn_s_memrealtime();
      const uint64_t c_exit = __builtin_amdgcn_s_memtime();
      if (lane == 0) {
        times[4 * gw + 0] = t_entry;
        times[4 * gw + 1] = t_image;
        times[4 * gw + 2] = t_exit;
        times[4 * gw + 3] = (uint64_t)j0 | ((c_exit - c_entry) << 24); // tasks | shader cycles
      }
    }
  }
  steal_exit();
#undef RPCCRC_ROWS_START
#undef RPCCRC_ROWS_BEGIN
#undef RPCCRC_ROWS_IMAGE_READY
}

} // namespace rpccrc
