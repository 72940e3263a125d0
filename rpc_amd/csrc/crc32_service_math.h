// rpc_amd/csrc/crc32_service_math.h -- the drop-in service kernel's per-lane
// CRC arithmetic (crc32_service.hip), written once for the device and for the
// host: tests/cpu_emu/service_emu.cpp compiles this header with g++ (the two
// gfx950 instructions it uses are emulated bit for bit below) and checks the
// lane algebra against zlib -- including the bitop3 truth tables, which the
// host build evaluates from the same immediates.
#pragma once
#include <stdint.h>

#include "crc32_gf2.h"

namespace rpccrc {
namespace svc {

// v_bfe_i32 x, i, 1: all ones iff bit i of x.
RPCCRC_HD uint32_t sext_bit(uint32_t x, int i) {
#if defined(__HIP_DEVICE_COMPILE__)
  return (uint32_t)__builtin_amdgcn_sbfe((int)x, i, 1);
#else
  return ((x >> i) & 1u) ? 0xFFFFFFFFu : 0u;
#endif
}

// v_bitop3_b32 a, b, c, TT: bit k of the result is bit (a_k << 2 | b_k << 1 | c_k) of TT.
template <uint32_t TT>
RPCCRC_HD uint32_t bitop3(uint32_t a, uint32_t b, uint32_t c) {
#if defined(__HIP_DEVICE_COMPILE__)
  return __builtin_amdgcn_bitop3_b32(a, b, c, TT);
#else
  uint32_t r = 0;
  for (int k = 0; k < 32; ++k) {
    const uint32_t idx = (((a >> k) & 1u) << 2) | (((b >> k) & 1u) << 1) | ((c >> k) & 1u);
    r |= ((TT >> idx) & 1u) << k;
  }
  return r;
#endif
}

// (m & b) ^ p in one instruction (truth table 0x6A = (a & b) ^ c).
RPCCRC_HD uint32_t and_xor(uint32_t m, uint32_t b, uint32_t p) { return bitop3<0x6A>(m, b, p); }

// crc0 of one 32-bit word x (the state already XORed in): 32 steps of
// x <- x * x mod P, 3 VALU per bit (a table of the 32 single-bit results would
// take 2 per bit but keep 32 constants live).
RPCCRC_HD uint32_t crc0_word(uint32_t x) {
  for (int i = 0; i < 32; ++i) x = and_xor(sext_bit(x, 0), kPoly, x >> 1); // (x >> 1) ^ (P if bit 0)
  return x;
}

// a * b mod P (reflected: bit 31 = x^0), bit-serial over a; `a` is shifted
// along rather than tested bit by bit (independent bit tests were hoisted, one
// live VGPR each).
RPCCRC_HD uint32_t mulmod(uint32_t a, uint32_t b) {
#if defined(__HIP_DEVICE_COMPILE__)
  // b * x^i does not depend on a: without this barrier the 32 powers of each
  // per-lane constant were precomputed outside the service's poll loop
  __asm__ volatile("" : "+v"(b));
#endif
  uint32_t p = 0;
  for (int i = 0; i < 32; ++i) {
    p = and_xor((uint32_t)((int32_t)a >> 31), b, p); // p ^= b if bit 31 of a
    a <<= 1;
    b = and_xor(sext_bit(b, 0), kPoly, b >> 1); // b *= x
  }
  return p;
}

// The dword at virtual offset pos of V keeps only the bytes at or after off0
// (the body's first byte; stale staging bytes before it read as zeros).
RPCCRC_HD uint32_t keep_mask(uint32_t pos, uint32_t off0) {
  return pos >= off0 ? 0xFFFFFFFFu : (pos + 4 <= off0 ? 0u : 0xFFFFFFFFu << (8 * (off0 - pos)));
}

// Size class of a body of len bytes: seg bytes per lane (4, 8 or 16) and the
// class index of the per-lane shift constants.
RPCCRC_HD uint32_t seg_of(uint32_t len) { return len <= 256u ? 4u : len <= 512u ? 8u : 16u; }

// ---- request check (crc32_kernels.h SvcReq, round 6) -------------------------
// Every dword the service uses for an answer -- the request block's len, seq and
// inline words, and for a longer body every masked word of its virtual buffer --
// enters the request's check sum through word_hash(word, position): fmix32
// (MurmurHash3's finalizer) of the word XOR a per-position constant, XORed over
// the positions.  The host stores the sum as the block's tag; the service
// answers only when its own sum over what it read equals the tag.
//
// Why non-linear and position-dependent: a poll reads the
// 32 block dwords in pieces of the memory system's choosing, so it may combine
// current and stale words.  Under a plain XOR sum (rounds 4-5), two stale words
// whose old -> new deltas are equal cancel -- JSON-RPC bodies on one slot where
// "id":1 -> 2 and a parameter digit 1 -> 2 fall in the same byte lane of two
// dwords pass the check, and the service would answer the CRC of a mix of two
// bodies.  Through word_hash each stale word changes the sum by an unrelated
// 32-bit value (h(new, p) ^ h(old, p)), so a torn read passes with probability
// ~2^-32 per torn poll whatever the structure of the bodies, and no read
// granularity of the PCIe / memory path is assumed.  tests/test_kernel_emu.py
// checks it exhaustively over the stale-word subsets of structured request
// pairs (tests/cpu_emu/svc_check_emu.cpp).
constexpr uint32_t kHashBodyPos = 32; // body word j hashes at position 32 + j (block words at 0..30)
RPCCRC_HD uint32_t word_hash(uint32_t w, uint32_t pos) {
  uint32_t h = w ^ (pos * 0x9E3779B1u + 0x6A09E667u);
  h ^= h >> 16;
  h *= 0x85EBCA6Bu;
  h ^= h >> 13;
  h *= 0xC2B2AE35u;
  return h ^ (h >> 16);
}

// Host side: the check sum of a request block's first 31 dwords (len, seq, the
// 29 inline words; the 32nd is the tag itself).
inline uint32_t block_sum(uint32_t len, uint32_t seq, const uint32_t *inl_words29) {
  uint32_t x = word_hash(len, 0) ^ word_hash(seq, 1);
  for (uint32_t k = 0; k < 29; ++k) x ^= word_hash(inl_words29[k], 2 + k);
  return x;
}

// Host side: the check sum of a longer body as the service reads it -- the
// 64 * seg-byte virtual buffer with the body right-aligned and every byte before
// it masked to zero (keep_mask), word j at position kHashBodyPos + j.
inline uint32_t body_sum(const uint8_t *src, uint32_t len) {
  const uint32_t seg = seg_of(len), nw = 16u * seg, off0 = 64u * seg - len;
  uint32_t x = 0, j = 0;
  for (; 4u * j + 4u <= off0; ++j) x ^= word_hash(0u, kHashBodyPos + j); // wholly before the body
  if (4u * j < off0) { // the word holding the body's first byte
    uint32_t w = 0;
    for (uint32_t b = off0 - 4u * j; b < 4; ++b) w |= (uint32_t)src[4u * j + b - off0] << (8 * b);
    x ^= word_hash(w, kHashBodyPos + j);
    ++j;
  }
  for (; j < nw; ++j) { // whole body words (little-endian, as the service loads them)
    const uint8_t *p = src + 4u * j - off0;
    const uint32_t w = (uint32_t)p[0] | (uint32_t)p[1] << 8 | (uint32_t)p[2] << 16 | (uint32_t)p[3] << 24;
    x ^= word_hash(w, kHashBodyPos + j);
  }
  return x;
}

} // namespace svc
} // namespace rpccrc
