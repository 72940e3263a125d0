// rpc_amd/csrc/crc32_tables.cpp -- builds the LDS image and the Tq table once
// per device context (host code; uploaded to HBM, copied to LDS per workgroup).
#include "crc32_gf2.h"
#include "crc32_layout.h"

#include <string.h>

namespace rpccrc {

namespace {
// Nibble table of the linear map s -> A_nbytes(s): N[n][nib] = A(nib << 4n).
void nibble_table(uint32_t nbytes, uint32_t out[8][16]) {
  const uint32_t xp = gf2_xpow(8ull * nbytes);
  for (int n = 0; n < 8; ++n)
    for (uint32_t nib = 0; nib < 16; ++nib)
      out[n][nib] = gf2_mulmod(xp, nib << (4 * n));
}
void nibble_table_inverse(uint32_t nbytes, uint32_t out[8][16]) {
  for (int n = 0; n < 8; ++n)
    for (uint32_t nib = 0; nib < 16; ++nib)
      out[n][nib] = gf2_unshift_bytes(nib << (4 * n), nbytes);
}
} // namespace

void build_lds_image_v2(uint32_t *img) {
  memset(img, 0, kLdsBytesV3);
  uint8_t *b = reinterpret_cast<uint8_t *>(img);
  auto put = [&](uint32_t byte_addr, uint32_t v) { memcpy(b + byte_addr, &v, 4); };
  for (uint32_t v = 0; v < 256; ++v) {
    const uint32_t t0 = crc_slice_entry(0, v), t1 = crc_slice_entry(1, v);
    const uint32_t t2 = crc_slice_entry(2, v), t3 = crc_slice_entry(3, v);
    for (uint32_t c = 0; c < 32; ++c) {
      put(kLdsMain + v * 256 + c * 4, t3);
      put(kLdsMain + v * 256 + 128 + c * 4, t2);
      put(kLdsMainRegion1 + v * 256 + c * 4, t1);
      put(kLdsMainRegion1 + v * 256 + 128 + c * 4, t0);
    }
  }
  uint32_t nt[8][16];
  for (uint32_t c = 0; c < 32; ++c) { // lo = c & 15; banks 16..31 add the first half-segment's A_32
    nibble_table(64u * (15u - (c & 15u)) + (kTwoChains ? 32u * ((c >> 4) & 1u) : 0u), nt);
    for (int n = 0; n < 8; ++n)
      for (uint32_t nib = 0; nib < 16; ++nib)
        put(kLdsST1 + (n >> 1) * 4096 + nib * 256 + (n & 1) * 128 + c * 4, nt[n][nib]);
  }
  for (uint32_t hi = 0; hi < 4; ++hi) {
    nibble_table(1024u * (3u - hi), nt);
    for (int n = 0; n < 8; ++n)
      for (uint32_t nib = 0; nib < 16; ++nib) put(st2_byte(n, nib, hi), nt[n][nib]);
  }
  nibble_table(4096u, nt);
  for (int n = 0; n < 8; ++n)
    for (uint32_t nib = 0; nib < 16; ++nib) put(kLdsRW2 + n * 64 + nib * 4, nt[n][nib]);
  for (uint32_t z = 1; z <= 15; ++z) {
    nibble_table_inverse(z, nt);
    for (int n = 0; n < 8; ++n)
      for (uint32_t nib = 0; nib < 16; ++nib) put(kLdsZI2 + (z - 1) * 512 + n * 64 + nib * 4, nt[n][nib]);
  }
  for (uint32_t k = 0; k <= 256; ++k) put(kLdsTQ16 + 4 * k, gf2_shift_bytes(0xFFFFFFFFu, 16ull * k));
  for (uint32_t j = 0; j < 4; ++j) { // sub-row shifts A_{16*(3-j)} (crc32_layout.h SQ)
    nibble_table(16u * (3u - j), nt);
    for (uint32_t n = 0; n < 8; ++n)
      for (uint32_t nib = 0; nib < 16; ++nib) put(sq_byte(j, n, nib), nt[n][nib]);
  }
}

void build_big_dbl(uint32_t *tab) {
  for (uint32_t m = 0; m < kBigChunkClasses; ++m)
    for (uint32_t i = 0; i < kBigDbl; ++i) {
      const uint64_t nbytes = ((4096ull << m) - 16) << i;
      const uint32_t xp = gf2_xpow(8ull * nbytes);
      for (uint32_t n = 0; n < 8; ++n)
        for (uint32_t j = 0; j < 16; ++j) tab[(m * kBigDbl + i) * 128 + n * 16 + j] = gf2_mulmod(xp, j << (4 * n));
    }
}

void build_dense_tab(uint32_t *tab) {
  auto put = [&](uint32_t map, uint32_t xp) { // [n][nib][map] of s -> s * xp mod P (crc32_layout.h)
    for (uint32_t n = 0; n < 8; ++n)
      for (uint32_t j = 0; j < 16; ++j) tab[(n * 16 + j) * kDenseMaps + map] = gf2_mulmod(xp, j << (4 * n));
  };
  for (uint32_t h = 0; h < 4; ++h) put(kDenseMQ + h, gf2_xpow(8ull * 1024 * h));
  for (uint32_t k = 0; k < 16; ++k) { // x^(-8 k unit) mod P: undo k units of zero bytes
    put(kDenseMI0 + k, gf2_unshift_bytes(kX0, k));
    put(kDenseMI1 + k, gf2_unshift_bytes(kX0, 16 * k));
    put(kDenseMI2 + k, gf2_unshift_bytes(kX0, 256 * k));
  }
  for (uint32_t k = 0; k < 16; ++k) put(kDenseMB0 + k, gf2_xpow(8ull * 4096 * k));
  for (uint32_t k = 0; k <= 16; ++k) put(kDenseMB1 + k, gf2_xpow(8ull * 65536 * k));
}

void build_lds_image_span(uint32_t *img) {
  uint8_t *b = reinterpret_cast<uint8_t *>(img);
  for (uint32_t tb = 0; tb < 16; ++tb) {
    const uint32_t xp = gf2_xpow(8ull * 4 * (16 - tb));
    for (uint32_t n = 0; n < 8; ++n)
      for (uint32_t j = 0; j < 16; ++j) {
        const uint32_t v = gf2_mulmod(xp, j << (4 * n));
        memcpy(b + kLdsSpanM4 + 4 * ((n * 16 + j) * kSpanM4Stride + tb), &v, 4);
      }
  }
}

void build_scalar_tab(uint32_t *tab) {
  for (int k = 0; k < 4; ++k)
    for (uint32_t v = 0; v < 256; ++v) tab[256 * k + v] = crc_slice_entry(k, v);
  for (uint32_t k = kScalarNibK0; k < kScalarNibK0 + 10; ++k)
    nibble_table(1u << k, reinterpret_cast<uint32_t(*)[16]>(tab + 1024 + (k - kScalarNibK0) * 128));
}

void build_lds_image_compact(const uint32_t *img, uint32_t *compact) {
  const uint8_t *b = reinterpret_cast<const uint8_t *>(img);
  for (uint32_t tbl = 0; tbl < 4; ++tbl)
    for (uint32_t v = 0; v < 256; ++v) // copy 0 of table tbl, row v
      memcpy(compact + tbl * 256 + v, b + (tbl >> 1) * kLdsMainRegion1 + v * 256 + (tbl & 1) * 128, 4);
  memcpy(reinterpret_cast<uint8_t *>(compact) + kImgTailOfs, b + kLdsST1, kLdsBytesV3 - kLdsST1);
}

void build_tq(uint32_t *tq) {
  for (uint32_t q = 0; q < kTqEntries; ++q) tq[q] = gf2_shift_bytes(0xFFFFFFFFu, q);
}

} // namespace rpccrc
