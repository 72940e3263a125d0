// tests/cpu_emu/rows_emu.cpp -- CPU emulation of crc32_rows_kernel lane by lane
// (TEST CODE): permuted coalesced piece loads, the v_permlane16/32_swap
// transpose, the slice-by-4 chain on the rows LDS image, the perm-addressed
// ST1 step with the exact DPP quad/row_ror reductions, the distributed
// ST2 + Horner step (row_shr 4 with zero fill, permlane-swap reductions,
// readlane 4 / 12), global Tq seeds and the distributed ZI steps.  Compared
// with the oracle by tests/test_kernel_emu.py.  Not the product path.
//
// stdin:  QB misalign n  then n lengths; bodies are splitmix bytes (seed 7)
//         back to back from byte `misalign` of a 16-aligned buffer.  QB = 1 is
//         QB = 1 with sub-row first rows, QB = 6 the same with the ragged kernel's
//         per-lane Horner (one merge per body), QB = 5 QB = 1 with full rows.
//         QB = 2 is the packed ragged kernel (crc32_packed.h) and reads
//         "nwaves min_slice max_slices" after n.
// stdout: one CRC (hex) per body.
#include "../../rpc_amd/csrc/crc32_gf2.h"
#include "../../rpc_amd/csrc/crc32_layout.h"

#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>
#include <algorithm>
#include <vector>

using namespace rpccrc;

static std::vector<uint32_t> g_img, g_tq;
static uint32_t ld(uint32_t a) {
  if (a % 4 || a >= kLdsBytesV3) { fprintf(stderr, "bad lds addr %u\n", a); exit(2); }
  return g_img[a / 4];
}
static uint32_t perm(uint32_t s0, uint32_t s1, uint32_t sel) {
  uint64_t data = ((uint64_t)s0 << 32) | s1;
  uint32_t r = 0;
  for (int b = 0; b < 4; ++b) {
    uint32_t sb = (sel >> (8 * b)) & 0xFF;
    uint32_t out = sb >= 13 ? 0xFF : sb == 12 ? 0 : sb <= 7 ? (uint32_t)(data >> (8 * sb)) & 0xFF : 0;
    r |= out << (8 * b);
  }
  return r;
}
static uint32_t slice4(uint32_t x, uint32_t lsel) {
  return ld(perm(x, lsel, 0x0C0C0400u)) ^ ld(perm(x, lsel, 0x0C0C0501u)) ^ ld(perm(x, lsel, 0x0C020600u)) ^
         ld(perm(x, lsel, 0x0C020701u));
}
typedef uint32_t Wave[64];
static void quad_perm(const Wave in, Wave out, const int p[4]) {
  for (int l = 0; l < 64; ++l) out[l] = in[(l & ~3) | p[l & 3]];
}
static void row_ror(const Wave in, Wave out, int n) { // dst[i] = src[(i - n) mod 16] within each row
  for (int l = 0; l < 64; ++l) out[l] = in[(l & ~15) | (((l & 15) - n) & 15)];
}
static void row_shr_zero(const Wave in, Wave out, int n) { // dst[i] = src[i - n] within the row, else 0
  for (int l = 0; l < 64; ++l) out[l] = ((l & 15) >= n) ? in[l - n] : 0u;
}
// dist_reduce8: quad xor1, quad xor2, row_shr 4 (zero fill), each XORed in.
static void dist_reduce8(Wave t) {
  static const int px1[4] = {1, 0, 3, 2}, px2[4] = {2, 3, 0, 1};
  Wave u;
  quad_perm(t, u, px1); for (int l = 0; l < 64; ++l) t[l] ^= u[l];
  quad_perm(t, u, px2); for (int l = 0; l < 64; ++l) t[l] ^= u[l];
  row_shr_zero(t, u, 4); for (int l = 0; l < 64; ++l) t[l] ^= u[l];
}

struct Piece { uint32_t d[4]; };

// dist_uniform: lane n = lane & 7 looks up nibble n of the uniform u in a
// [n][nib] table; the result is read from lane 4.
static uint32_t dist_uniform(uint32_t u, uint32_t table) {
  Wave t;
  for (int l = 0; l < 64; ++l) t[l] = ld(table + (uint32_t)(l & 7) * 64u + ((u >> (4 * (l & 7))) & 15u) * 4u);
  dist_reduce8(t);
  return t[4];
}

static uint32_t piece_of_lane(uint32_t L) { return ((L & 15u) << 2) | (L >> 4); }

// v_permlane16_swap vdst, vsrc: odd rows of vdst <-> even rows of vsrc.
static void permlane16_swap(Wave x, Wave y) {
  Wave nx, ny;
  for (int l = 0; l < 64; ++l) { nx[l] = x[l]; ny[l] = y[l]; }
  for (int l = 0; l < 64; ++l) {
    if ((l >> 4) & 1) nx[l] = y[l - 16];   // odd row of vdst <- even row of vsrc
    else ny[l] = x[l + 16];                // even row of vsrc <- odd row of vdst
  }
  for (int l = 0; l < 64; ++l) { x[l] = nx[l]; y[l] = ny[l]; }
}
// v_permlane32_swap vdst, vsrc: upper half of vdst <-> lower half of vsrc.
static void permlane32_swap(Wave x, Wave y) {
  Wave nx, ny;
  for (int l = 0; l < 64; ++l) { nx[l] = x[l]; ny[l] = y[l]; }
  for (int l = 0; l < 32; ++l) { nx[l + 32] = y[l]; ny[l] = x[l + 32]; }
  for (int l = 0; l < 64; ++l) { x[l] = nx[l]; y[l] = ny[l]; }
}

static Wave g_chain_b; // two-chain mode: each lane's second chain value (row_chain -> merge_lo)

// One 4 KiB row: P[b][lane] = the piece lane loaded in load b (already masked).
// Returns the per-lane chain value after the transpose.
static void row_chain(Piece P[4][64], Wave s_out) {
  for (int d = 0; d < 4; ++d) {
    Wave w[4];
    for (int b = 0; b < 4; ++b) for (int l = 0; l < 64; ++l) w[b][l] = P[b][l].d[d];
    permlane16_swap(w[0], w[1]);
    permlane16_swap(w[2], w[3]);
    permlane32_swap(w[0], w[2]);
    permlane32_swap(w[1], w[3]);
    for (int b = 0; b < 4; ++b) for (int l = 0; l < 64; ++l) P[b][l].d[d] = w[b][l];
  }
  for (int l = 0; l < 64; ++l) {
    uint32_t lane4 = (uint32_t)(l & 31) * 4u, lsel = lane4 | ((lane4 + 128u) << 8) | (1u << 16);
    if (kTwoChains) { // seg_crc2: slots 0-1 and 2-3 as two chains; s_out = a, s_out2 = b
      uint32_t xa = P[0][l].d[0], xb = P[2][l].d[0];
      for (int k = 0; k < 2; ++k)
        for (int d = 0; d < 4; ++d) {
          if (!k && !d) continue;
          xa = slice4(xa, lsel) ^ P[k][l].d[d];
          xb = slice4(xb, lsel) ^ P[k + 2][l].d[d];
        }
      s_out[l] = slice4(xa, lsel);
      g_chain_b[l] = slice4(xb, lsel);
      continue;
    }
    uint32_t x = P[0][l].d[0];
    for (int k = 0; k < 4; ++k)
      for (int d = 0; d < 4; ++d) {
        if (!k && !d) continue;
        x = slice4(x, lsel) ^ P[k][l].d[d];
      }
    s_out[l] = slice4(x, lsel);
  }
}

static void xor_lanebit(Wave s, int bit) {
  Wave a, b;
  for (int l = 0; l < 64; ++l) { a[l] = s[l]; b[l] = s[l]; }
  if (bit == 4) permlane16_swap(a, b); else permlane32_swap(a, b);
  for (int l = 0; l < 64; ++l) s[l] = a[l] ^ b[l];
}

// ST1 (perm-addressed) + reduce over lane bits 0-3 (quad_perm xor1, xor2, row_ror 4, 8).
static uint32_t st1_map(uint32_t s, uint32_t lane) {
  const uint32_t lane4 = (lane & 31u) * 4u, lsel1 = lane4 | ((lane4 + 128u) << 8) | (2u << 16);
  const uint32_t xl = s & 0x0F0F0F0Fu, xh = (s >> 4) & 0x0F0F0F0Fu;
  uint32_t r = 0;
  for (uint32_t k = 0; k < 4; ++k) {
    r ^= ld(perm(xl, lsel1, 0x0C020400u + (k << 8)) + k * 4096u);
    r ^= ld(perm(xh, lsel1, 0x0C020401u + (k << 8)) + k * 4096u);
  }
  return r;
}
// swap_lanebit4 of the kernel: both results of v_permlane16_swap(v, v), then
// upper lanes take the first, lower lanes the second.
static void swap_lanebit4(const Wave v, Wave out) {
  Wave a, b;
  for (int l = 0; l < 64; ++l) { a[l] = v[l]; b[l] = v[l]; }
  permlane16_swap(a, b);
  for (int l = 0; l < 64; ++l) out[l] = (l & 16) ? a[l] : b[l];
}
static void merge_lo(Wave s) {
  static const int px1[4] = {1, 0, 3, 2}, px2[4] = {2, 3, 0, 1};
  Wave t;
  if (kTwoChains) { // merge_lo2: s = chain a, g_chain_b = chain b
    Wave own, sel, other, t_own, t_other, back;
    for (int l = 0; l < 64; ++l) {
      const bool up = (l & 16) != 0;
      own[l] = up ? s[l] : g_chain_b[l];
      sel[l] = up ? g_chain_b[l] : s[l];
    }
    swap_lanebit4(sel, other);
    for (int l = 0; l < 64; ++l) {
      t_own[l] = st1_map(own[l], (uint32_t)l);
      t_other[l] = st1_map(other[l], (uint32_t)l);
    }
    swap_lanebit4(t_other, back);
    for (int l = 0; l < 64; ++l) s[l] = t_own[l] ^ back[l];
  } else {
    for (int l = 0; l < 64; ++l) s[l] = st1_map(s[l], (uint32_t)l);
  }
  quad_perm(s, t, px1); for (int l = 0; l < 64; ++l) s[l] ^= t[l];
  quad_perm(s, t, px2); for (int l = 0; l < 64; ++l) s[l] ^= t[l];
  row_ror(s, t, 4); for (int l = 0; l < 64; ++l) s[l] ^= t[l];
  row_ror(s, t, 8); for (int l = 0; l < 64; ++l) s[l] ^= t[l];
}

// Sub-row first rows (ragged QB = 1, crc32_rows.h sub_chain): per-lane SQ
// shift A_{16*(3-j)} with the perm-formed address {j*64 + nib*4 | kLdsSQ},
// nibble n's 256-B block in the immediate.
static uint32_t sq_map(uint32_t s, uint32_t j) {
  const uint32_t jb = (j * 64u) * 0x01010101u;
  const uint32_t xl4 = ((s << 2) & 0x3C3C3C3Cu) | jb, xh4 = ((s >> 2) & 0x3C3C3C3Cu) | jb;
  uint32_t r = 0;
  for (uint32_t k = 0; k < 4; ++k) {
    r ^= ld(perm(xl4, kLdsSQ, 0x0C020104u + k) + k * 512u);
    r ^= ld(perm(xh4, kLdsSQ, 0x0C020104u + k) + k * 512u + 256u);
  }
  return r;
}
static uint32_t chain_slots(const Piece *slots, int nslots, uint32_t lane) {
  const uint32_t lane4 = (lane & 31u) * 4u, lsel = lane4 | ((lane4 + 128u) << 8) | (1u << 16);
  uint32_t x = slots[0].d[0];
  for (int k = 0; k < nslots; ++k)
    for (int d = 0; d < 4; ++d) {
      if (!k && !d) continue;
      x = slice4(x, lsel) ^ slots[k].d[d];
    }
  return slice4(x, lsel);
}
// Quarter row (hd <= 1 KiB: only load 3 holds data): no transpose, 4 chain
// steps on slot 3, A_{16*(3-hi)}, XOR over lane bits 4 and 5, rows hi < 3 zeroed.
// Half row (hd <= 2 KiB: loads 2, 3): the transpose's permlane16 stage on
// slots (2, 3) only -- lane L then holds the 32-B half (L >> 5) of 64-B
// segment 32 + (L & 31); 8 chain steps; lower lanes' A_32 moved up by one
// permlane32_swap into a zero register and XORed into the upper lanes.
// Both leave the full-row layout (lane L' = 64-B segment L') for merge_lo.
static void sub_chain(Piece P[4][64], bool quarter, Wave v) {
  if (quarter) {
    Wave a;
    for (int l = 0; l < 64; ++l) a[l] = sq_map(chain_slots(&P[3][l], 1, (uint32_t)l), (uint32_t)l >> 4);
    xor_lanebit(a, 4);
    xor_lanebit(a, 5);
    for (int l = 0; l < 64; ++l) v[l] = ((l >> 4) == 3) ? a[l] : 0u;
    return;
  }
  for (int d = 0; d < 4; ++d) {
    Wave w2, w3;
    for (int l = 0; l < 64; ++l) { w2[l] = P[2][l].d[d]; w3[l] = P[3][l].d[d]; }
    permlane16_swap(w2, w3);
    for (int l = 0; l < 64; ++l) { P[2][l].d[d] = w2[l]; P[3][l].d[d] = w3[l]; }
  }
  Wave c, a, zr;
  for (int l = 0; l < 64; ++l) {
    Piece sl[2] = {P[2][l], P[3][l]};
    c[l] = chain_slots(sl, 2, (uint32_t)l);
    a[l] = sq_map(c[l], 1u);
    zr[l] = 0u;
  }
  permlane32_swap(zr, a);
  for (int l = 0; l < 64; ++l) v[l] = ((l & 32) ? c[l] : 0u) ^ zr[l];
}

static bool g_subrows = true; // QB code 1: sub-row first rows (the ragged kernel); 5: full rows only
static bool g_lane_horner = false; // QB code 6: sub-rows + per-lane Horner (RPCCRC_LANE_HORNER)
static uint32_t rw_map_emu(uint32_t s) {
  const uint32_t xl4 = (s << 2) & 0x3C3C3C3Cu, xh4 = (s >> 2) & 0x3C3C3C3Cu;
  uint32_t r = 0;
  for (uint32_t k = 0; k < 4; ++k) {
    r ^= ld(perm(xl4, kLdsRW2, 0x0C020104u + k) + k * 128u);
    r ^= ld(perm(xh4, kLdsRW2, 0x0C020104u + k) + k * 128u + 64u);
  }
  return r;
}

static void mask_piece(Piece &p, int64_t v, int64_t len) {
  for (int d = 0; d < 4; ++d) {
    int64_t lo = v + 4 * d;
    uint32_t m = 0xFFFFFFFFu;
    if (lo < 0) m = (lo <= -4) ? 0u : (m << (8 * (uint32_t)(-lo)));
    int64_t over = lo + 4 - len;
    if (over > 0) m &= (over >= 4) ? 0u : (0xFFFFFFFFu >> (8 * (uint32_t)over));
    p.d[d] &= m;
  }
}
static Piece load_piece(const uint8_t *p) {
  if (((uintptr_t)p) & 15u) { fprintf(stderr, "misaligned load\n"); exit(3); }
  Piece r;
  memcpy(r.d, p, 16);
  return r;
}

static uint32_t emu_qb1(const uint8_t *p0, uint32_t len) {
  if (len == 0) return 0;
  const uint32_t z = (uint32_t)(0u - (uint32_t)(uintptr_t)(p0 + len)) & 15u;
  const uint64_t lp = (uint64_t)len + z;
  const uint32_t nrows = (uint32_t)((lp + 4095) / 4096);
  const uint32_t first = (uint32_t)(lp - (uint64_t)(nrows - 1) * 4096);
  uint32_t W = 0;
  static Piece P[4][64];
  for (uint32_t r = 0; r < nrows; ++r) {
    int64_t rs = (int64_t)lp - (int64_t)(nrows - r) * 4096;
    bool last = r + 1 == nrows;
    for (int b = 0; b < 4; ++b)
      for (int L = 0; L < 64; ++L) {
        int64_t v = rs + b * 1024 + 16 * (int64_t)piece_of_lane((uint32_t)L);
        P[b][L] = (v + 16 > 0) ? load_piece(p0 + v) : Piece{{0, 0, 0, 0}};
        if (rs < 0 || (last && z)) mask_piece(P[b][L], v, len);
      }
    Wave s;
    const uint32_t hd = r == 0 ? first : 4096u;
    if (g_subrows && !kTwoChains && hd <= 2048u) sub_chain(P, hd <= 1024u, s);
    else row_chain(P, s);
    if (g_lane_horner) { // per-lane Horner across rows (rw_map), one merge per body
      static Wave acc;
      for (int l = 0; l < 64; ++l) {
        uint32_t a = (r == 0) ? 0u : rw_map_emu(acc[l]);
        a ^= s[l];
        if (r == 0 && l == 63) a ^= g_tq[first];
        acc[l] = a;
      }
      if (!last) continue;
      for (int l = 0; l < 64; ++l) s[l] = acc[l];
      merge_lo(s);
      Wave t;
      for (int l = 0; l < 64; ++l) {
        const uint32_t lo = l & 15, hi = l >> 4;
        const bool own = lo < 8;
        const uint32_t base = own ? st2_byte(lo, 0u, hi) : kLdsZero;
        const uint32_t mul = own ? st2_byte(0u, 1u, 0u) - st2_byte(0u, 0u, 0u) : 0u;
        t[l] = ld(base + ((s[l] >> (4 * (l & 7))) & 15u) * mul);
      }
      dist_reduce8(t);
      xor_lanebit(t, 4);
      xor_lanebit(t, 5);
      W = t[4];
      continue;
    }
    merge_lo(s);
    for (int h = 0; h < 4; ++h)
      for (int l = 16 * h; l < 16 * h + 16; ++l)
        if (s[l] != s[16 * h]) { fprintf(stderr, "row not uniform\n"); exit(4); }
    // distributed ST2 (lanes lo < 8, own row value) + RW of W (row 0, lanes 8..15)
    Wave t;
    for (int l = 0; l < 64; ++l) {
      const uint32_t lo = l & 15, hi = l >> 4;
      const bool own = lo < 8;
      const uint32_t base = own ? st2_byte(lo, 0u, hi) : (hi == 0 ? kLdsRW2 + (lo - 8u) * 64u : kLdsZero);
      const uint32_t mul = own ? st2_byte(0u, 1u, 0u) - st2_byte(0u, 0u, 0u) : (hi == 0 ? 4u : 0u);
      const uint32_t src = own ? s[l] : W;
      t[l] = ld(base + ((src >> (4 * (l & 7))) & 15u) * mul);
    }
    dist_reduce8(t);
    xor_lanebit(t, 4);
    xor_lanebit(t, 5);
    const uint32_t rowcrc = t[4], rwu = t[12];
    W = ((r == 0) ? g_tq[first] : rwu) ^ rowcrc;
  }
  if (z) W = dist_uniform(W, kLdsZI2 + (z - 1) * 512);
  return ~W;
}

// Four items (<= 1 KiB each incl. end pad) in one row; returns 4 CRCs.
static void emu_qb4(const uint8_t *const p0[4], const uint32_t len[4], int nvalid, uint32_t out[4]) {
  static Piece P[4][64];
  uint32_t z[4], w0[4];
  for (int b = 0; b < 4; ++b) {
    uint32_t L = b < nvalid ? len[b] : 0;
    const uint8_t *q = b < nvalid ? p0[b] : p0[0];
    z[b] = (uint32_t)(0u - (uint32_t)(uintptr_t)(q + L)) & 15u;
    int64_t vstart = (int64_t)L + z[b] - 1024;
    w0[b] = g_tq[L + z[b]];
    for (int Ln = 0; Ln < 64; ++Ln) {
      int64_t v = vstart + 16 * (int64_t)piece_of_lane((uint32_t)Ln);
      P[b][Ln] = (b < nvalid && L != 0 && v + 16 > 0) ? load_piece(q + v) : Piece{{0, 0, 0, 0}};
      if (vstart < 0 || z[b]) mask_piece(P[b][Ln], v, L);
    }
  }
  Wave s;
  row_chain(P, s);
  merge_lo(s);
  for (int h = 0; h < 4; ++h)
    for (int l = 16 * h; l < 16 * h + 16; ++l)
      if (s[l] != s[16 * h]) { fprintf(stderr, "row not uniform\n"); exit(4); }
  Wave res;
  for (int l = 0; l < 64; ++l) res[l] = w0[l >> 4] ^ s[l];
  if (z[0] | z[1] | z[2] | z[3]) {
    Wave t;
    for (int l = 0; l < 64; ++l) {
      const uint32_t zl = z[l >> 4];
      const uint32_t table = kLdsZI2 + (zl - 1u) * 512u; // zl = 0: lands in RW2, discarded
      t[l] = ld(table + (uint32_t)(l & 7) * 64u + ((res[l] >> (4 * (l & 7))) & 15u) * 4u);
    }
    dist_reduce8(t);
    for (int l = 0; l < 64; ++l) if (z[l >> 4]) res[l] = t[l];
  }
  for (int h = 0; h < 4; ++h) {
    uint32_t r = ~res[16 * h + 4];
    if (h >= nvalid || len[h] == 0) r = 0;
    out[h] = r;
  }
}

// ---- packed ragged kernel (crc32_packed.h) ------------------------------------
// The plan (chunk counts, exclusive scan, slice table), every wave's 64-body
// metadata window over its slices (prefix scan + ballots), rows of four 1 KiB chunks, the distributed run shift
// (ST2 / RW), the scalar run XOR and the distributed ZI step of finished bodies.
// Checks that every slice is planned once and every body is written once.

static uint32_t pk_body_chunks(uint64_t end, uint32_t len) {
  const uint32_t z = (uint32_t)(0u - (uint32_t)end) & 15u;
  return len ? (uint32_t)(((uint64_t)len + z + 1023) / 1024) : 0u;
}

struct PkQuarter {
  uint32_t clen = 0, z = 0, body = 0, seed = 0;
  bool first = false, last = false, valid = false;
  const uint8_t *p = nullptr;
};

static void emu_packed(const std::vector<const uint8_t *> &ptr, const std::vector<uint32_t> &lens, uint64_t nwaves,
                       uint64_t min_slice, uint64_t max_slices, std::vector<uint32_t> &out) {
  const uint64_t n = lens.size();
  std::vector<uint32_t> cnt(n);
  std::vector<uint64_t> cfirst(n);
  std::vector<int> written(n, 0);
  uint64_t total = 0;
  for (uint64_t i = 0; i < n; ++i) { // packed_count_kernel + exclusive scan
    cnt[i] = pk_body_chunks((uint64_t)(uintptr_t)ptr[i] + lens[i], lens[i]);
    cfirst[i] = total;
    total += cnt[i];
    if (lens[i] == 0) {
      out[i] = 0;
      written[i] = 1;
    }
  }
  uint64_t S = (total + max_slices - 1) / max_slices;
  if (S < min_slice) S = min_slice;
  const uint64_t nslices = (total + S - 1) / S;
  std::vector<uint32_t> sb(nslices + 1, 0xFFFFFFFFu);
  for (uint64_t i = 0; i <= n; ++i) { // packed_plan_kernel, thread i
    const uint64_t s_lo = i == 0 ? 0 : cfirst[i - 1] / S + 1;
    uint64_t s_hi = i < n ? cfirst[i] / S : nslices;
    if (s_hi > nslices) s_hi = nslices;
    for (uint64_t s = s_lo; s <= s_hi; ++s) {
      if (sb[s] != 0xFFFFFFFFu) { fprintf(stderr, "slice %llu planned twice\n", (unsigned long long)s); exit(5); }
      sb[s] = (uint32_t)i;
    }
  }
  for (uint64_t s = 0; s <= nslices; ++s)
    if (sb[s] == 0xFFFFFFFFu) { fprintf(stderr, "slice %llu unplanned\n", (unsigned long long)s); exit(5); }

  for (uint64_t gw = 0; gw < nwaves && gw < nslices; ++gw) {
    // The wave's stream (crc32_packed.h): current slice [wb0, cb1), next
    // slice [nb0, nb1); slices dealt round-robin here (the kernel deals them
    // dynamically; any order gives the same CRCs).
    uint64_t snext = gw;
    bool more = true;
    uint32_t wb0 = 0, cb1 = 0, nb0 = 0, nb1 = 0, wk0 = 0;
    auto fetch_next = [&]() {
      nb0 = nb1 = 0;
      while (more) {
        if (snext >= nslices) {
          more = false;
          break;
        }
        const uint64_t sl = snext;
        snext += nwaves;
        nb0 = sb[sl];
        nb1 = sb[sl + 1];
        if (nb0 < nb1) break;
      }
    };
    auto advance = [&]() {
      wb0 = nb0;
      cb1 = nb1;
      fetch_next();
    };
    fetch_next();
    advance();
    if (wb0 >= cb1) continue;
    uint32_t W = 0;
    for (;;) {
      // window: 64 bodies of the stream, one per lane
      const uint32_t kw = std::min<uint32_t>(64u, cb1 - wb0), wn0 = nb0, wn1 = nb1, w0 = wb0;
      uint32_t idx[64], wl[64], nchl[64], cst[64];
      bool has[64];
      uint32_t run = 0;
      for (uint32_t l = 0; l < 64; ++l) {
        idx[l] = l < kw ? w0 + l : wn0 + (l - kw);
        const bool ok = l < kw || idx[l] < wn1;
        wl[l] = ok ? lens[idx[l]] : 0u;
        const uint32_t z = ok ? (uint32_t)(0u - (uint32_t)((uintptr_t)ptr[idx[l]] + wl[l])) & 15u : 0u;
        nchl[l] = wl[l] ? (wl[l] + z + 1023u) >> 10 : 0u;
        has[l] = nchl[l] != 0;
        cst[l] = run;
        run += nchl[l];
      }
      auto find = [&](uint32_t pos, uint32_t &m) -> bool { // last nonempty lane with cst <= pos
        int mm = -1;
        for (int l = 0; l < 64; ++l)
          if (has[l] && cst[l] <= pos) mm = l;
        m = mm < 0 ? 0u : (uint32_t)mm;
        return mm >= 0 && pos - cst[m] < nchl[m];
      };
      PkQuarter q[4];
      uint32_t nvalid = 4;
      for (int bq = 0; bq < 4; ++bq) {
        uint32_t m;
        const uint32_t pos = wk0 + (uint32_t)bq;
        if (nvalid != 4 || !find(pos, m)) {
          if (nvalid == 4) nvalid = (uint32_t)bq;
          continue;
        }
        const uint32_t j = pos - cst[m], nc = nchl[m], len = wl[m];
        const uint8_t *p0 = ptr[idx[m]];
        const uint32_t z = (uint32_t)(0u - (uint32_t)((uintptr_t)p0 + len)) & 15u;
        const uint8_t *wend = p0 + len + z - (uint64_t)(nc - 1 - j) * 1024;
        const bool first = j == 0, last = j + 1 == nc;
        const uint8_t *rs = first ? p0 : wend - 1024;
        const uint8_t *re = last ? p0 + len : wend;
        q[bq].clen = (uint32_t)(re - rs);
        q[bq].z = last ? z : 0;
        q[bq].first = first;
        q[bq].last = last;
        q[bq].valid = true;
        q[bq].body = idx[m];
        // seed: the first window fill of lane m's body (kernel: tq gather per lane)
        q[bq].seed = first ? g_tq[len + z - (nc - 1) * 1024] : 0;
        q[bq].p = rs;
      }
      const bool live = wb0 < cb1 || nb0 < nb1;
      { // next row start
        uint32_t m, skip;
        const uint32_t pos = wk0 + nvalid;
        if (find(pos, m)) {
          skip = m;
          wk0 = pos - cst[m];
        } else {
          skip = 64;
          wk0 = 0;
        }
        if (skip < cb1 - wb0) {
          wb0 += skip;
        } else {
          uint32_t rest = skip - (cb1 - wb0);
          advance();
          while (wb0 < cb1 && rest >= cb1 - wb0) {
            rest = 0;
            advance();
          }
          wb0 += rest;
        }
        if (wb0 >= cb1) wb0 = cb1 = nb0 = nb1 = 0;
      }
      if (!live) break;
      static Piece P[4][64];
      for (int bq = 0; bq < 4; ++bq) {
        const int64_t vstart = (int64_t)q[bq].clen + q[bq].z - 1024;
        for (int L = 0; L < 64; ++L) {
          const int64_t v = vstart + 16 * (int64_t)piece_of_lane((uint32_t)L);
          P[bq][L] = (q[bq].valid && q[bq].clen && v + 16 > 0) ? load_piece(q[bq].p + v) : Piece{{0, 0, 0, 0}};
          if (vstart < 0 || q[bq].z) mask_piece(P[bq][L], v, q[bq].clen);
        }
      }
      Wave sv;
      row_chain(P, sv);
      merge_lo(sv);
      for (int h = 0; h < 4; ++h)
        for (int l = 16 * h; l < 16 * h + 16; ++l)
          if (sv[l] != sv[16 * h]) { fprintf(stderr, "row not uniform\n"); exit(4); }
      bool endq[4], lastq[4];
      for (int bq = 0; bq < 4; ++bq) {
        lastq[bq] = q[bq].valid && q[bq].last;
        endq[bq] = bq == 3 || !q[bq].valid || q[bq].last;
      }
      uint32_t e[4];
      e[3] = 3;
      e[2] = endq[2] ? 2 : 3;
      e[1] = endq[1] ? 1 : e[2];
      e[0] = endq[0] ? 0 : e[1];
      const bool cont = q[0].valid && !q[0].first;
      Wave t;
      for (int l = 0; l < 64; ++l) {
        const uint32_t lo = l & 15, hi = l >> 4, n8 = lo & 7;
        const bool own = lo < 8, wl = hi == 0 && lo >= 8;
        const uint32_t v = sv[l] ^ q[hi].seed;
        const uint32_t nib = ((own ? v : W) >> (4 * n8)) & 15u;
        const uint32_t d = e[hi] - hi;
        const uint32_t a_w = !cont ? kLdsZero
                             : (e[0] == 3 ? kLdsRW2 + n8 * 64 + nib * 4 : st2_byte(n8, nib, 2 - e[0]));
        const uint32_t a_own = st2_byte(n8, nib, 3 - d);
        t[l] = ld(own ? a_own : (wl ? a_w : kLdsZero));
      }
      dist_reduce8(t);
      uint32_t acc = cont ? t[12] : 0, fin[4] = {0, 0, 0, 0};
      for (int bq = 0; bq < 4; ++bq) {
        acc ^= t[16 * bq + 4];
        fin[bq] = acc;
        if (endq[bq]) {
          if (bq == 3 && !lastq[3]) W = acc;
          acc = 0;
        }
      }
      bool zrow[4], any = false;
      for (int bq = 0; bq < 4; ++bq) {
        zrow[bq] = lastq[bq] && q[bq].z;
        any = any || zrow[bq];
      }
      if (any) {
        Wave tz;
        for (int l = 0; l < 64; ++l) {
          const uint32_t lo = l & 15, hi = l >> 4, n8 = lo & 7;
          const uint32_t nib = (fin[hi] >> (4 * n8)) & 15u;
          tz[l] = ld((lo < 8 && zrow[hi]) ? kLdsZI2 + (q[hi].z - 1) * 512 + n8 * 64 + nib * 4 : kLdsZero);
        }
        dist_reduce8(tz);
        for (int bq = 0; bq < 4; ++bq)
          if (zrow[bq]) fin[bq] = tz[16 * bq + 4];
      }
      for (int bq = 0; bq < 4; ++bq)
        if (lastq[bq]) {
          if (written[q[bq].body]++) { fprintf(stderr, "body %u written twice\n", q[bq].body); exit(6); }
          out[q[bq].body] = ~fin[bq];
        }
    }
  }
  for (uint64_t i = 0; i < n; ++i)
    if (!written[i]) { fprintf(stderr, "body %llu never written\n", (unsigned long long)i); exit(7); }
}

int main() {
  int QB, mis;
  unsigned long n;
  unsigned long long pk_nwaves = 1, pk_min_slice = 8, pk_max_slices = 1 << 20;
  if (scanf("%d %d %lu", &QB, &mis, &n) != 3) return 1;
  if (QB == 2 && scanf("%llu %llu %llu", &pk_nwaves, &pk_min_slice, &pk_max_slices) != 3) return 1;
  std::vector<uint32_t> lens(n);
  uint64_t total = 0;
  for (unsigned long i = 0; i < n; ++i) {
    if (scanf("%u", &lens[i]) != 1) return 1;
    total += lens[i];
  }
  g_img.resize(kLdsBytesV3 / 4);
  build_lds_image_v2(g_img.data());
  g_tq.resize(kTqEntries);
  build_tq(g_tq.data());
  // guard bands: loads may touch the 16-B blocks around a body, never further
  std::vector<uint8_t> raw(total + mis + 8192);
  uint8_t *buf = raw.data() + 4096;
  while ((uintptr_t)buf & 15u) ++buf;
  auto mix = [](uint64_t zz) {
    zz = (zz ^ (zz >> 30)) * 0xBF58476D1CE4E5B9ull;
    zz = (zz ^ (zz >> 27)) * 0x94D049BB133111EBull;
    return zz ^ (zz >> 31);
  };
  for (uint64_t i = 0; i < total + mis; ++i) {
    uint64_t w = mix(7 + (i / 8 + 1) * 0x9E3779B97F4A7C15ull);
    buf[i] = (uint8_t)(w >> (8 * (i % 8)));
  }
  std::vector<const uint8_t *> ptr(n);
  uint64_t off = (uint64_t)mis;
  for (unsigned long i = 0; i < n; ++i) {
    ptr[i] = buf + off;
    off += lens[i];
  }
  if (QB == 6) { // QB = 1, sub-rows, per-lane Horner
    QB = 1;
    g_lane_horner = true;
  }
  if (QB == 5) { // QB = 1 with full rows only
    QB = 1;
    g_subrows = false;
  }
  if (QB == 1) {
    for (unsigned long i = 0; i < n; ++i) printf("%08x\n", emu_qb1(ptr[i], lens[i]));
  } else if (QB == 2) { // packed ragged kernel
    std::vector<uint32_t> out(n);
    emu_packed(ptr, lens, pk_nwaves, pk_min_slice, pk_max_slices, out);
    for (unsigned long i = 0; i < n; ++i) printf("%08x\n", out[i]);
  } else {
    for (unsigned long g = 0; g < n; g += 4) {
      int nv = (int)((n - g) < 4 ? n - g : 4);
      const uint8_t *pp[4];
      uint32_t ll[4], out[4];
      for (int b = 0; b < 4; ++b) {
        pp[b] = b < nv ? ptr[g + b] : ptr[g];
        ll[b] = b < nv ? lens[g + b] : 0;
      }
      emu_qb4(pp, ll, nv, out);
      for (int b = 0; b < nv; ++b) printf("%08x\n", out[b]);
    }
  }
  return 0;
}
