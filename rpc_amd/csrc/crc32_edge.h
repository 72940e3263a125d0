// rpc_amd/csrc/crc32_edge.h -- lane <-> piece map and the scalar byte masks of
// a window's edge pieces (host + device: tests/cpu_emu/edge_emu.cpp checks
// them on the CPU against a per-byte mask).
#pragma once
#include <stdint.h>

#include "crc32_gf2.h" // RPCCRC_HD

namespace rpccrc {

// Lane that loads piece p of a quarter / piece loaded by lane L (involution-free
// bijection on 0..63): p(L) = ((L & 15) << 2) | (L >> 4).
RPCCRC_HD uint32_t piece_of_lane(uint32_t L) { return ((L & 15u) << 2) | (L >> 4); }
RPCCRC_HD uint32_t lane_of_piece(uint32_t p) { return ((p & 3u) << 4) | (p >> 2); }

// Mask of dword d of a 16-byte piece keeping the piece bytes [lo, hi)
// (0 <= lo, hi <= 16; wave-uniform, scalar arithmetic).
RPCCRC_HD uint32_t keep_dword(uint32_t lo, uint32_t hi, uint32_t d) {
  const uint32_t s = lo > 4u * d ? (lo - 4u * d < 4u ? lo - 4u * d : 4u) : 0u;
  const uint32_t e = hi > 4u * d ? (hi - 4u * d < 4u ? hi - 4u * d : 4u) : 0u;
  return e > s ? (uint32_t)(((1ull << (8u * e)) - 1u) & ~((1ull << (8u * s)) - 1u)) : 0u;
}

// The two masks the kernels use, with fewer scalar ops than keep_dword (~4 per
// dword: one clamped shift amount and one 64-bit shift, whose low half is 0
// for a shift of 32):
//   keep_front_dword(f, d) == keep_dword(f, 16, d)      (bytes >= f kept, f < 16)
//   keep_end_dword(k, d)   == keep_dword(0, k, d)       (bytes <  k kept, k <= 16)
RPCCRC_HD uint32_t keep_front_dword(uint32_t f, uint32_t d) {
  const int32_t t = (int32_t)(8u * f) - (int32_t)(32u * d); // foreign bits at the dword's low end
  return t <= 0 ? 0xFFFFFFFFu : (t >= 32 ? 0u : 0xFFFFFFFFu << (uint32_t)t);
}
RPCCRC_HD uint32_t keep_end_dword(uint32_t k, uint32_t d) {
  const int32_t t = (int32_t)(32u * d + 32u) - (int32_t)(8u * k); // foreign bits at the dword's high end
  return t <= 0 ? 0xFFFFFFFFu : (t >= 32 ? 0u : 0xFFFFFFFFu >> (uint32_t)t);
}

} // namespace rpccrc
