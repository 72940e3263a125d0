// rpc_amd/csrc/crc32_layout.h -- LDS table image layout of the rows kernel.
//
// One persistent 1024-thread workgroup per CU owns 155 KiB of LDS holding every
// table the kernel looks up.  All lookups are ds_read_b32 whose bank is
// (byte_addr/4) mod 32 (MI355X_MICROARCH.md, LDS table): a table replicated 32
// times with copy c = lane & 31 at bank c is conflict-free for ANY indices.
//
//   MAIN   [0, 128 KiB)  slice-by-4 byte tables, 32 copies, two tables per
//                        256-byte row so that one v_perm_b32 forms the address:
//                        region 0: row v = { T3[v] x32 | T2[v] x32 }
//                        region 1: row v = { T1[v] x32 | T0[v] x32 } (+64 KiB)
//   then the shift tables listed below (ST1, ST2, RW, ZI, TQ16).
#pragma once
#include <stdint.h>

namespace rpccrc {

constexpr uint32_t kLdsMain = 0;
constexpr uint32_t kLdsMainRegion1 = 65536;
constexpr uint32_t kLdsBytesV2 = 158736;     // rows-kernel image (155 KiB)
constexpr uint32_t kMaxRow = 4096;           // 64 lanes x 64-byte segments
constexpr uint32_t kTqEntries = kMaxRow + 1; // Tq[q] = A_q(0xFFFFFFFF), q=0..4096

// Two independent slice-by-4 chains per lane (crc32_rows.h seg_crc2 /
// merge_lo2): each lane's 64-B segment is CRC'd as two 32-B halves whose
// dependent LDS round trips interleave; the ST1 copies of banks 16..31 then
// carry the extra A_32 of the first half.  Off: measured slower (NS 640 vs 622 us,
// C2 7200 vs 6890 us, one box, profiles/r02/r02d_two_chains_ab.txt) -- the kernel
// is bound by board power (instructions per byte), not by the chain latency.
#ifndef RPCCRC_TWO_CHAINS
#define RPCCRC_TWO_CHAINS 0
#endif
constexpr bool kTwoChains = RPCCRC_TWO_CHAINS != 0;

// ---- rows-kernel image (crc32_rows.h): main tables as above, then
//   ST1 16 KiB  A_{64*(15-(c&15)) + (kTwoChains ? 32*((c>>4)&1) : 0)}(nib << 4n), c = lane & 31, at
//               ST1 + (n/2)*4096 + nib*256 + (n%2)*128 + c*4: one v_perm_b32 of
//               the masked nibble vector forms the address (like MAIN), the
//               n/2 part rides in the ds_read immediate offset
//   ST2  2 KiB  ST2(n, nib, hi) = A_{1024*(3-hi)}(nib << 4n),    hi = 0..3 (st2_byte)
//   RW  512 B   RW[n][nib]      = A_4096(nib << 4n)
//   ZI  7.5 KiB ZI[z-1][n][nib] = A_z^-1(nib << 4n)
//   TQ16 1 KiB  TQ16[k]         = A_{16k}(0xFFFFFFFF), k = 0..256
constexpr uint32_t kLdsST1 = 131072;
constexpr uint32_t kLdsST2 = kLdsST1 + 16384; // 147456
constexpr uint32_t kLdsRW2 = kLdsST2 + 2048;  // 149504
// ST2 word of entry (n, nib, k) (k = the shift's quarter index): the 16 nibbles of
// (n, k) share ONE bank, 2n + (k & 1) + 16 (k >> 1), so the rows kernel's
// distributed step -- lane (lo = n, hi = k) looks up its own (n, k) -- is
// bank-conflict-free whatever the nibbles (the [n][nib][k] layout put lanes
// with equal nibbles on one bank).
constexpr uint32_t st2_byte(uint32_t n, uint32_t nib, uint32_t k) {
  return kLdsST2 + 4u * (nib * 32u + 2u * n + (k & 1u) + 16u * (k >> 1));
}
constexpr uint32_t kLdsZI2 = kLdsRW2 + 512;   // 150016
// TQ16[k] = A_{16k}(0xFFFFFFFF), k = 0..256: zlib pre-conditioning seeds for
// first rows of 16k bytes (other lengths: round up, undo with ZI).
constexpr uint32_t kLdsTQ16 = kLdsZI2 + 15 * 512; // 157696
// kRowsRoundOut launches (crc32_rows.h): A_{4096 * 2^l}, l = 1..4, in [n][nib]
// layout over ZI[11..14] (pads z = 12..15, which 16-B aligned 4096-byte items never have).
constexpr uint32_t kLdsRoundMaps = kLdsZI2 + 11 * 512;
static_assert(kLdsRoundMaps % 256 == 0 && kLdsRoundMaps + 4 * 512 <= kLdsTQ16, "round maps inside ZI");
// A zero dword (TQ16's 12-byte tail pad): lanes with nothing to look up read it.
constexpr uint32_t kLdsZero = kLdsTQ16 + 1028;
// The dense span pass's image (crc32_rows.h kRowsSpanBnd; RAW 4096-byte rows
// never read ZI or TQ16): over ZI..TQ16, the maps A_{4(16-tb)}, tb = 0..15 --
// a boundary's chain state cap shifted to its 64-B segment's end -- word
// (n * 16 + nib) * 17 + tb (stride 17: the lanes of one lookup, each with its
// own tb, spread over the banks), below kLdsZero.
constexpr uint32_t kLdsSpanM4 = kLdsZI2;
constexpr uint32_t kSpanM4Stride = 17;
static_assert(kLdsSpanM4 + 128 * kSpanM4Stride * 4 <= kLdsZero, "span maps below the zero dword");
void build_lds_image_span(uint32_t *img /* a V2 image: the maps go over its ZI / TQ16 */);
static_assert(kLdsTQ16 + 1040 == kLdsBytesV2, "rows image size");
static_assert(kLdsBytesV2 % 16 == 0 && kLdsBytesV2 <= 163840, "fits the 160 KiB LDS");
// ---- sub-row shifts (ragged QB = 1 kernels only: image V3 = V2 + pad + SQ) ----
//   SQ  2 KiB   SQ(j, n, nib) = A_{16*(3-j)}(nib << 4n), j = 0..3, at byte
//               kLdsSQ + n*256 + j*64 + nib*4.  A first row of <= 1 KiB ("quarter
//               row") shifts lane L's 16-B piece by A_{16*(3-(L>>4))}; a first
//               row of <= 2 KiB ("half row") shifts the first 32-B half of each
//               64-B segment by A_32 (j = 1).  Bank = 16*(j&1) + nib: the lanes
//               of one half-wave (j in {0,1} or {2,3}) never collide, lanes with
//               equal (j, nib) read one word (broadcast).  256-B aligned so one
//               v_perm_b32 forms {j*64 + nib*4 | base}; n rides in the immediate.
constexpr uint32_t kLdsSQ = (kLdsBytesV2 + 255u) & ~255u; // 158976
constexpr uint32_t kLdsBytesV3 = kLdsSQ + 2048u;         // 161024
static_assert(kLdsBytesV3 % 16 == 0 && kLdsBytesV3 <= 163840, "fits the 160 KiB LDS");
constexpr uint32_t sq_byte(uint32_t j, uint32_t n, uint32_t nib) { return kLdsSQ + n * 256u + j * 64u + nib * 4u; }
void build_lds_image_v2(uint32_t *img /* kLdsBytesV3 bytes: V2 + the SQ tables */);

// Compact HBM form of the image (round 4): MAIN is 32 copies of the four
// slice-by-4 tables, so HBM holds them once -- word tbl * 256 + v, tbl = 0..3
// for T3, T2, T1, T0 (MAIN's regions / halves in order) -- followed by the
// image bytes from kLdsST1 on.  Each workgroup reads ~38 KiB instead of 157 KiB
// and writes the 128 KiB of copies into LDS itself (crc32_rows.h
// img_load / img_store): 256 workgroups had read 40 MB from L2 per launch.
// RPCCRC_IMG_COMPACT=0 keeps the full 157 KiB image in HBM (A/B only).
#ifndef RPCCRC_IMG_COMPACT
#define RPCCRC_IMG_COMPACT 1
#endif
constexpr bool kImgCompact = RPCCRC_IMG_COMPACT != 0;
constexpr uint32_t kImgTailOfs = 4096; // compact form: where image byte kLdsST1 sits
constexpr uint32_t kImgCompactBytes = kImgTailOfs + (kLdsBytesV3 - kLdsST1);
constexpr uint32_t kImgHbmBytes = kImgCompact ? kImgCompactBytes : kLdsBytesV3; // what the device context uploads
void build_lds_image_compact(const uint32_t *img /* kLdsBytesV3 bytes */, uint32_t *compact /* kImgCompactBytes */);

// Host-side builder (crc32_tables.cpp).
void build_tq(uint32_t *tq /* kTqEntries */);

// The big-body route fold's maps (crc32_kernels.hip big_combine_kernel), built
// once per device on the host: for chunk class m (chunk = 4096 * 2^m - 16
// bytes, m < kBigChunkClasses) and i < kBigDbl,
// DBL[m][i][n][j] = A_{chunk * 2^i}(j << 4n).  (Round 3 first built them in every
// fold block from the 32 KiB A_{2^k} maps: ~10 us of a 24 us fold.)
constexpr uint32_t kBigChunkClasses = 19; // 4080 B .. 1 GiB - 16
constexpr uint32_t kBigDbl = 11;          // i = 10: A_{1024 * chunk}, the Horner step
constexpr uint32_t kBigDblWords = kBigChunkClasses * kBigDbl * 128;
void build_big_dbl(uint32_t *tab /* kBigDblWords */);

// The dense span fold's maps (crc32_kernels.hip dense_fold_kernel, DESIGN.md
// 4.9), stored [n][nib][map] (word (n * 16 + nib) * kDenseMaps + map: the
// lanes of one lookup, each with its own map, spread over all 32 banks; a
// [map][n][nib] layout put one lookup on 16 banks): A_{1024h} (h = 0..3),
// A_{-z0}, A_{-16 z1}, A_{-256 z2} (0..15 each), A_{4096 d0} (d0 = 0..15),
// A_{65536 d1} (d1 = 0..16).
constexpr uint32_t kDenseMQ = 0, kDenseMI0 = 4, kDenseMI1 = 20, kDenseMI2 = 36, kDenseMB0 = 52, kDenseMB1 = 68,
                   kDenseMaps = 85;
constexpr uint32_t kDenseTabWords = kDenseMaps * 128;
void build_dense_tab(uint32_t *tab /* kDenseTabWords */);

// One-wave scalar kernel (crc32_scalar.hip): bodies of <= kScalarMaxLen
// bytes.  Table image of kScalarTabWords words: T_k[256] slice-by-4 tables,
// k = 0..3, then NIB[k - kScalarNibK0][i][j] = A_{2^k bytes}(j << 4i) for
// k = 2..11.
constexpr uint32_t kScalarMaxLen = 4096;
constexpr uint32_t kScalarNibK0 = 2;
constexpr uint32_t kScalarTabWords = 1024 + 10 * 128;
void build_scalar_tab(uint32_t *tab /* kScalarTabWords */);

} // namespace rpccrc
