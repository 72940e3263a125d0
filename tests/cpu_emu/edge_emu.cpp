// tests/cpu_emu/edge_emu.cpp -- TEST CODE.  Checks the kernels' edge fix
// (crc32_rows.h fix_quarter, masks from crc32_edge.h) against a per-byte mask:
// a 1 KiB window whose real bytes are [front, 1024 - z) is loaded as 64 pieces
// of 16 B, lane L holding piece p(L); pieces wholly before the 16-B block of
// byte `front` read as zeros (out-of-range loads), every other piece reads
// memory (foreign bytes included).  After the fix, each piece must equal the
// window with every foreign byte zeroed.  Exit status 0 = all cases pass.
#include "../../rpc_amd/csrc/crc32_edge.h"

#include <stdio.h>
#include <string.h>

using namespace rpccrc;

int main() {
  // the kernels' cheaper mask forms equal the general keep_dword
  for (uint32_t f = 0; f < 16; ++f)
    for (uint32_t d = 0; d < 4; ++d)
      if (keep_front_dword(f, d) != keep_dword(f, 16u, d)) {
        printf("keep_front_dword(%u, %u) %08x != %08x\n", f, d, keep_front_dword(f, d), keep_dword(f, 16u, d));
        return 1;
      }
  for (uint32_t k = 0; k <= 16; ++k)
    for (uint32_t d = 0; d < 4; ++d)
      if (keep_end_dword(k, d) != keep_dword(0u, k, d)) {
        printf("keep_end_dword(%u, %u) %08x != %08x\n", k, d, keep_end_dword(k, d), keep_dword(0u, k, d));
        return 1;
      }
  uint8_t mem[1024];
  for (int i = 0; i < 1024; ++i) mem[i] = (uint8_t)(i * 37 + 11) | 1u; // no zero bytes
  long cases = 0;
  for (uint32_t front = 0; front <= 1024; ++front) {
    for (uint32_t z = 0; z < 16; ++z) {
      if (front + z > 1024) continue;
      if ((front + 16 - (front & 15)) % 16 != 0) return 2;
      uint32_t piece[64][4];
      for (uint32_t L = 0; L < 64; ++L) { // load
        const uint32_t p = piece_of_lane(L);
        const bool oob = 16 * p + 16 <= (front & ~15u);
        for (uint32_t d = 0; d < 4; ++d) {
          uint32_t w = 0;
          if (!oob) memcpy(&w, mem + 16 * p + 4 * d, 4);
          piece[L][d] = w;
        }
      }
      // the fix (same steps as fix_quarter, lane-parallel)
      for (uint32_t L = 0; L < 64; ++L) {
        if ((front & 15u) != 0u && front < 1024u && L == lane_of_piece(front >> 4))
          for (uint32_t d = 0; d < 4; ++d) piece[L][d] &= keep_front_dword(front & 15u, d);
        if (z != 0u && L == lane_of_piece(63u))
          for (uint32_t d = 0; d < 4; ++d) piece[L][d] &= keep_end_dword(16u - z, d);
      }
      for (uint32_t L = 0; L < 64; ++L) {
        const uint32_t p = piece_of_lane(L);
        for (uint32_t d = 0; d < 4; ++d) {
          uint32_t want = 0;
          for (uint32_t k = 0; k < 4; ++k) {
            const uint32_t pos = 16 * p + 4 * d + k;
            if (pos >= front && pos < 1024 - z) want |= (uint32_t)mem[pos] << (8 * k);
          }
          if (piece[L][d] != want) {
            printf("front %u z %u lane %u dword %u: %08x != %08x\n", front, z, L, d, piece[L][d], want);
            return 1;
          }
        }
      }
      ++cases;
    }
  }
  printf("ok %ld\n", cases);
  return 0;
}
