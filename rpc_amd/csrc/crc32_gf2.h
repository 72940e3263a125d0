// rpc_amd/csrc/crc32_gf2.h -- GF(2) arithmetic for reflected CRC-32 (ISO-HDLC).
//
// The reference checksum (crc.c:4-9) is zlib crc32(): reflected polynomial
// 0xEDB88320, init/xorout 0xFFFFFFFF.  In the reflected representation bit
// (31-k) of a 32-bit word is the coefficient of x^k, so ">> 1" multiplies by x.
//
// Notation used throughout the library and DESIGN.md:
//   crc0(M)   raw register after M from state 0 (linear in M; leading zero
//             bytes do not change it)
//   A_n(s)    state s advanced through n zero bytes = s * x^(8n) mod P
//   U(s, M)   = A_|M|(s) ^ crc0(M)          (register after M from state s)
//   crc(M)    = ~U(0xFFFFFFFF, M)           (what rpc_crc32 returns)
//   crc(A||B) = A_|B|(crc(A)) ^ crc(B)      (zlib crc32_combine, zlib.h:1750)
//
// Everything here is constexpr-friendly plain C++ usable from host code and
// from HIP device code (RPCCRC_HD).
#pragma once
#include <stdint.h>

#if defined(__HIPCC__)
#include <hip/hip_runtime.h>
#define RPCCRC_HD __host__ __device__ __forceinline__
#else
#define RPCCRC_HD inline
#endif

namespace rpccrc {

constexpr uint32_t kPoly = 0xEDB88320u;
constexpr uint32_t kX0 = 0x80000000u; // the polynomial "1" (x^0)

// a(x) * b(x) mod P  (zlib multmodp).
RPCCRC_HD constexpr uint32_t gf2_mulmod(uint32_t a, uint32_t b) {
  uint32_t m = kX0, p = 0;
  for (int i = 0; i < 32; ++i) {
    if (a & m) p ^= b;
    m >>= 1;
    b = (b & 1u) ? (b >> 1) ^ kPoly : (b >> 1);
  }
  return p;
}

// x^n mod P by square-and-multiply over the bits of n (n in bits).
RPCCRC_HD constexpr uint32_t gf2_xpow(uint64_t n) {
  uint32_t result = kX0;
  uint32_t sq = kX0 >> 1; // x^1
  while (n) {
    if (n & 1u) result = gf2_mulmod(result, sq);
    sq = gf2_mulmod(sq, sq);
    n >>= 1;
  }
  return result;
}

// A_nbytes(s): advance state s through nbytes zero bytes.
RPCCRC_HD constexpr uint32_t gf2_shift_bytes(uint32_t s, uint64_t nbytes) {
  return gf2_mulmod(gf2_xpow(8ull * nbytes), s);
}

// Multiply by x^-1 (inverse of one zero bit).  P has a constant term, so the
// bit that left on the x-multiply is recoverable from bit 31 of the result.
RPCCRC_HD constexpr uint32_t gf2_mul_xinv(uint32_t c) {
  return (c & 0x80000000u) ? (((c ^ kPoly) << 1) | 1u) : (c << 1);
}

// A_nbytes^-1(s): undo nbytes trailing zero bytes.
RPCCRC_HD constexpr uint32_t gf2_unshift_bytes(uint32_t s, uint32_t nbytes) {
  for (uint32_t i = 0; i < 8u * nbytes; ++i) s = gf2_mul_xinv(s);
  return s;
}

// zlib crc32_combine semantics: crc(A||B) from crc(A), crc(B), |B|.
RPCCRC_HD constexpr uint32_t crc32_combine(uint32_t crc1, uint32_t crc2, uint64_t len2) {
  return gf2_shift_bytes(crc1, len2) ^ crc2;
}

// Byte table entry: crc0 of the single byte v (zlib crc_table[0][v]).
RPCCRC_HD constexpr uint32_t crc_byte_entry(uint32_t v) {
  uint32_t c = v;
  for (int k = 0; k < 8; ++k) c = (c & 1u) ? (c >> 1) ^ kPoly : (c >> 1);
  return c;
}

// Slice table T_k[v] = A_k(T_0[v]) = crc0 of byte v followed by k zero bytes.
RPCCRC_HD constexpr uint32_t crc_slice_entry(int k, uint32_t v) {
  uint32_t c = crc_byte_entry(v);
  for (int i = 0; i < k; ++i) c = (c >> 8) ^ crc_byte_entry(c & 0xFFu);
  return c;
}

} // namespace rpccrc
