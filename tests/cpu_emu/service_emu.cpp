// tests/cpu_emu/service_emu.cpp -- CPU run of the drop-in service kernel's lane
// algebra (TEST CODE): the SAME functions the kernel calls
// (rpc_amd/csrc/crc32_service_math.h: the bit-serial chain, the per-lane shift
// multiply, the masks; bitop3 / sbfe evaluated from the same immediates), lane
// by lane over the kernel's virtual buffer, with stale bytes before the body.
// Compared with zlib by tests/test_kernel_emu.py.  Not the product path.
//
// stdin:  n, then n lengths (1..1024); body k = splitmix-like bytes (seed k).
// stdout: one CRC (hex) per body.
#include "../../rpc_amd/csrc/crc32_service_math.h"

#include <stdint.h>
#include <stdio.h>
#include <string.h>

using namespace rpccrc;

static uint64_t mix(uint64_t z) {
  z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ull;
  z = (z ^ (z >> 27)) * 0x94D049BB133111EBull;
  return z ^ (z >> 31);
}

int main() {
  int n = 0;
  if (scanf("%d", &n) != 1) return 2;
  for (int k = 0; k < n; ++k) {
    unsigned len = 0;
    if (scanf("%u", &len) != 1 || len == 0 || len > 1024) return 2;
    const uint32_t seg = svc::seg_of(len);
    uint8_t V[1024];
    for (uint32_t i = 0; i < 64 * seg; ++i) V[i] = (uint8_t)(0xA5 ^ i); // stale staging
    const uint32_t off0 = 64 * seg - len;
    for (uint32_t i = 0; i < len; ++i) V[off0 + i] = (uint8_t)mix(0x5E17C0DEull + (uint64_t)k * 4096 + i);
    uint32_t c0 = 0;
    for (uint32_t L = 0; L < 64; ++L) {
      uint32_t s = 0;
      for (uint32_t d = 0; d < seg / 4; ++d) {
        uint32_t w;
        memcpy(&w, V + L * seg + 4 * d, 4);
        s = svc::crc0_word(s ^ (w & svc::keep_mask(L * seg + 4 * d, off0)));
      }
      c0 ^= svc::mulmod(s, gf2_xpow(8ull * seg * (63u - L))); // the host's kshift table entry
    }
    const uint32_t tq = gf2_shift_bytes(0xFFFFFFFFu, len); // Tq[len]
    printf("%08x\n", ~(tq ^ c0));
  }
  return 0;
}
