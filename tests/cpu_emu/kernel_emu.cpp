// tests/cpu_emu/kernel_emu.cpp -- CPU emulation of crc32_items_kernel's exact
// arithmetic (TEST CODE).  It reads the same LDS image (crc32_tables.cpp), forms
// LDS addresses with an emulated v_perm_b32, runs the same per-lane segment CRC,
// nibble-table lane shifts, XOR "shuffles", row Horner, Tq pre-conditioning and
// ZI trailing-pad undo, for groups of G lanes, and prints one CRC per body.
// tests/test_kernel_emu.py compares its output with the oracle, so table layout
// and index math are checked without a GPU.  It is not the product path.
//
// stdin:  G misalign n  then n lines "len"; bodies are splitmix bytes (seed 7)
//         laid back to back starting at byte offset `misalign` of a 16-aligned buffer.
// stdout: one CRC (hex) per body.
#include "../../rpc_amd/csrc/crc32_gf2.h"
#include "../../rpc_amd/csrc/crc32_layout.h"

#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>
#include <vector>

using namespace rpccrc;

static uint32_t perm(uint32_t s0, uint32_t s1, uint32_t sel) {
  uint64_t data = ((uint64_t)s0 << 32) | s1;
  uint32_t r = 0;
  for (int b = 0; b < 4; ++b) {
    uint32_t sb = (sel >> (8 * b)) & 0xFF, out;
    if (sb >= 13) out = 0xFF;
    else if (sb == 12) out = 0;
    else if (sb <= 7) out = (uint32_t)(data >> (8 * sb)) & 0xFF;
    else out = 0; // sign-replicate selectors unused
    r |= out << (8 * b);
  }
  return r;
}

static std::vector<uint32_t> g_img;
static std::vector<uint32_t> g_tq;
static uint32_t ld(uint32_t a) {
  if (a % 4 || a >= kLdsBytes) { fprintf(stderr, "bad lds addr %u\n", a); exit(2); }
  return g_img[a / 4];
}
static uint32_t slice4(uint32_t x, uint32_t lsel) {
  return ld(perm(x, lsel, 0x0C0C0400u)) ^ ld(perm(x, lsel, 0x0C0C0501u)) ^ ld(perm(x, lsel, 0x0C020600u)) ^
         ld(perm(x, lsel, 0x0C020701u));
}
static uint32_t nib_map(uint32_t s, uint32_t base, uint32_t stride, uint32_t shift) {
  uint32_t r = 0;
  for (uint32_t n = 0; n < 8; ++n) r ^= ld(base + n * stride + (((s >> (4 * n)) & 15u) << shift));
  return r;
}

// Emulates one group (G lanes at wave lanes [g0, g0+G)) on one body.
static uint32_t emu_body(int G, const uint8_t *buf, uint64_t off, uint32_t len, uint32_t mode) {
  if (len == 0) return 0;
  const uint32_t ROW = (uint32_t)G * 64;
  const uint8_t *p0 = buf + off;
  const uint32_t z = (uint32_t)(0u - (uint32_t)(uintptr_t)(p0 + len)) & 15u;
  const uint64_t lp = (uint64_t)len + z;
  const uint32_t nrows = (uint32_t)((lp + ROW - 1) / ROW);
  const uint32_t first = (uint32_t)(lp - (uint64_t)(nrows - 1) * ROW);
  uint32_t W = 0;
  for (uint32_t r = 0; r < nrows; ++r) {
    std::vector<uint32_t> s(64, 0);
    // Wave lanes: this group occupies lanes [0, G) (lane-dependent tables use lane & 31, lane >> 3).
    for (int lane = 0; lane < G; ++lane) {
      const uint32_t j = (uint32_t)lane & (uint32_t)(G - 1);
      const int64_t seg = (int64_t)lp - (int64_t)(nrows - r) * ROW + 64 * (int64_t)j;
      if ((((uintptr_t)(p0 + seg)) & 15u) != 0) { fprintf(stderr, "misaligned segment\n"); exit(3); }
      uint32_t w[16];
      for (int d = 0; d < 16; ++d) {
        uint32_t v = 0;
        for (int b = 0; b < 4; ++b) {
          int64_t pos = seg + 4 * d + b;
          // the kernel loads whole 16-B blocks that contain a valid byte, then masks
          uint8_t byte = (pos >= 0 && pos < (int64_t)len) ? p0[pos] : 0;
          v |= (uint32_t)byte << (8 * b);
        }
        w[d] = v;
      }
      const uint32_t lane4 = ((uint32_t)lane & 31u) * 4u;
      const uint32_t lsel = lane4 | ((lane4 + 128u) << 8) | (1u << 16);
      uint32_t acc = 0;
      if (seg + 64 > 0) {
        uint32_t x = w[0];
        for (int d = 0; d < 15; ++d) x = slice4(x, lsel) ^ w[d + 1];
        acc = slice4(x, lsel);
      }
      s[lane] = nib_map(acc, kLdsS1 + lane4, 2048, 7);
    }
    // XOR-reduce over lane groups of 8, then step 2, then across the group.
    std::vector<uint32_t> t(64, 0);
    for (int lane = 0; lane < G; ++lane) {
      uint32_t v = 0;
      for (int m = 0; m < 8; ++m) v ^= s[(lane & ~7) + m];
      t[lane] = nib_map(v, kLdsS2 + ((uint32_t)lane >> 3) * 4u, 512, 5);
    }
    uint32_t rowcrc = 0;
    for (int lane = 0; lane < G; lane += 8) rowcrc ^= t[lane];
    W = (r == 0) ? (mode == 1 ? 0u : g_tq[first]) : nib_map(W, kLdsRW, 64, 2);
    W ^= rowcrc;
  }
  if (z) W = nib_map(W, kLdsZI + (z - 1) * 512, 64, 2);
  return mode == 0 ? ~W : W;
}

int main() {
  int G, mis;
  unsigned long n;
  if (scanf("%d %d %lu", &G, &mis, &n) != 3) return 1;
  std::vector<uint32_t> lens(n);
  uint64_t total = 0;
  for (unsigned long i = 0; i < n; ++i) {
    if (scanf("%u", &lens[i]) != 1) return 1;
    total += lens[i];
  }
  g_img.resize(kLdsWords);
  build_lds_image(G, g_img.data());
  g_tq.resize(kTqEntries);
  build_tq(g_tq.data());
  std::vector<uint8_t> raw(total + mis + 64 + 16);
  uint8_t *buf = raw.data();
  while ((uintptr_t)buf & 15u) ++buf;
  // splitmix bytes, seed 7 (same generator as oracle_splitmix_fill)
  auto mix = [](uint64_t z) {
    z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ull;
    z = (z ^ (z >> 27)) * 0x94D049BB133111EBull;
    return z ^ (z >> 31);
  };
  for (uint64_t i = 0; i < total + mis; ++i) {
    uint64_t w = mix(7 + (i / 8 + 1) * 0x9E3779B97F4A7C15ull);
    buf[i] = (uint8_t)(w >> (8 * (i % 8)));
  }
  uint64_t off = (uint64_t)mis;
  for (unsigned long i = 0; i < n; ++i) {
    printf("%08x\n", emu_body(G, buf, off, lens[i], 0));
    off += lens[i];
  }
  return 0;
}
