// rpc_amd/csrc/crc32_kernels.hip -- batched CRC-32 (zlib / ISO-HDLC) for gfx950.
//
// Replaces the arithmetic behind rpc_crc32() (reference crc.c:4-9 -> zlib crc32)
// with a many-buffer device path:
//
//  * crc32_rows_kernel (crc32_rows.h): persistent grid, one 1024-thread
//    workgroup (16 waves) per CU with the 155 KiB table image in LDS; a wave
//    CRCs one 4 KiB row per step (QB = 1: rows of one body, end-aligned, Horner
//    across rows; QB = 4: four <= 1 KiB bodies per row).  Coalesced 16-B
//    non-temporal loads, permlane transpose, slice-by-4 lookups, GF(2) merge.
//  * crc32_chunk_combine_kernel (below): folds chunk CRCs of large bodies
//    (zlib crc32_combine algebra), several blocks per body.
//  * splitmix_fill_kernel / stream_read_kernel: synthetic data and the
//    achievable-HBM-read probe used by bench.py.
//  No MFMA: this is a byte scan.
#include <hip/hip_ext.h>
#include <hip/hip_runtime.h>
#include <stdint.h>
#include <stdlib.h>

#include <algorithm>

#include <rocprim/device/device_scan.hpp>
#include <rocprim/iterator/counting_iterator.hpp>
#include <rocprim/iterator/transform_iterator.hpp>

#include "crc32_gf2.h"
#include "crc32_kernels.h"
#include "crc32_layout.h"
#include "crc32_packed.h"
#include "crc32_small.h"
#include "crc32_rows.h"
#include "frames.h"
#include "../../include/rpccrc.h"

namespace rpccrc {

// ---------------------------------------------------------------------------
// Chunk combine for large bodies: body b's chunk CRCs raw[cfirst[b] + k],
// k = 0..nch-1 (end-aligned chunks of `chunk` bytes, all crc0) are folded into
// crc(body) = ~(A_L(F) ^ XOR_k A_{(nch-1-k)*chunk}(raw_k)).
// ---------------------------------------------------------------------------
// A_n(v) for n = sum of 2^k bytes, applied map by map from the nibble tables
// NIB[k][i][j] = A_{2^k}(j << 4i) (64 maps x 8 nibble positions x 16, in LDS):
// 8 lookups per set bit of n, instead of a bit-serial gf2_mulmod for x^(8n)
// and another for the product (~30 of those per thread for C4's shifts).
__device__ __forceinline__ uint32_t nib_apply(const uint32_t *nib, uint32_t k, uint32_t v) {
  const uint32_t *m = nib + k * 128u;
  uint32_t r = 0;
#pragma unroll
  for (uint32_t i = 0; i < 8; ++i) r ^= m[i * 16u + ((v >> (4u * i)) & 15u)];
  return r;
}
__device__ __forceinline__ uint32_t nib_shift(const uint32_t *nib, uint64_t nbytes, uint32_t v) {
  while (nbytes) {
    const uint32_t k = (uint32_t)__builtin_ctzll(nbytes);
    v = nib_apply(nib, k, v);
    nbytes &= nbytes - 1;
  }
  return v;
}

// `splits` blocks per body; block s folds a contiguous run [c0, c1) of the
// body's chunks.  Thread t takes chunks c0 + t, c0 + t + NT, ... (the raw
// loads of a wave are coalesced): Horner with the step map A_{NT*chunk} (one
// nibble map when NT and chunk are powers of two), then a shift of the
// partial from its last chunk to the body end.  The block XORs its threads'
// partials.  splits == 1 (the common case: up to 64Ki chunks per body, NT =
// 1024) stores ~(A_L(F) ^ XOR) directly; splits > 1 atomically XORs into
// the zeroed out[b] (block 0 adds the ~A_L(0xFFFFFFFF) term).
template <uint32_t NT>
__global__ void __launch_bounds__(NT) crc32_chunk_combine_kernel(CombineArgs a) {
  __shared__ __attribute__((aligned(16))) uint32_t nib[kShiftNibWords];
  __shared__ uint32_t part[NT / 64];
  const uint64_t b = blockIdx.x / a.splits;
  const uint32_t s = blockIdx.x % a.splits;
  const uint32_t t = threadIdx.x;
  const uint64_t L = a.inline_bodies ? a.bodies.b[b].len : a.lengths[b];
  const uint64_t first = a.inline_bodies ? a.bodies.b[b].chunk_first : a.chunk_first[b];
  const uint64_t nch = (L + a.chunk - 1) / a.chunk;
  const uint64_t pb = (nch + a.splits - 1) / a.splits;
  const uint64_t c0 = s * pb, c1 = (c0 + pb < nch) ? c0 + pb : nch;
  if (c0 >= c1) { // (block-uniform) no chunks here
    if (a.splits == 1 && t == 0) a.out[b] = 0u; // empty body
    return;
  }
  const uint64_t step = (uint64_t)NT * a.chunk;
  const uint32_t *raw = a.raw + first;
  // The raw loads of a batch of 16 chunks are issued together, the first
  // batch before the table copy, so the two memory round trips overlap.
  constexpr uint32_t kB = 16;
  uint32_t r[kB];
  uint64_t k = c0 + t;
  auto load_batch = [&]() {
#pragma unroll
    for (uint32_t i = 0; i < kB; ++i) r[i] = (k + i * NT < c1) ? raw[k + i * NT] : 0u;
  };
  load_batch();
  {
    uint4 *dst = reinterpret_cast<uint4 *>(nib);
#pragma unroll
    for (uint32_t q = 0; q < kShiftNibWords / 4 / NT; ++q) dst[q * NT + t] = a.shift_nib[q * NT + t];
  }
  __syncthreads();
  uint32_t acc = 0;
  while (k < c1) {
#pragma unroll
    for (uint32_t i = 0; i < kB; ++i)
      if (k + i * NT < c1) acc = nib_shift(nib, step, acc) ^ r[i];
    k += (uint64_t)kB * NT;
    if (k < c1) load_batch();
  }
  if (c0 + t < c1) { // shift from this thread's last chunk to the body end
    const uint64_t kl = c0 + t + (c1 - 1 - (c0 + t)) / NT * NT;
    acc = nib_shift(nib, (nch - 1 - kl) * a.chunk, acc);
  }
  for (int m = 1; m < 64; m <<= 1) acc ^= (uint32_t)__shfl_xor((int)acc, m, 64);
  if ((t & 63u) == 0) part[t >> 6] = acc;
  __syncthreads();
  if (t == 0) {
    for (uint32_t w = 1; w < NT / 64; ++w) acc ^= part[w];
    if (s == 0) acc ^= ~nib_shift(nib, L, 0xFFFFFFFFu);
    if (a.splits == 1) a.out[b] = acc;
    else atomicXor(a.out + b, acc);
  }
}

// Bodies of equal length, a multiple of 4096 power-of-two chunks (C4: 256 MiB
// in 4 KiB or 16 KiB chunks): a.splits blocks per body, 1024 threads each,
// thread t of block s folding the CONTIGUOUS run of 4 chunks starting at
// chunk 4 * (s * 1024 + t) (one 16-B load, three Horner maps), shifted to the
// body end; the block XORs its threads' runs into out[b], which the rows
// pass zeroed (ItemsArgs.zero_out).  The combine is bound by LDS lookups (8
// per map): one block per body (16 CUs for C4) took 21-23 us at 4 KiB
// chunks, 16 blocks per body spread it over the chip (profiles/r02/r02ab_*).
// Round values (ItemsArgs.round_out: one crc0 per 128 KiB, chunk = 131072):
// 128 * S values per body, one block per body, the threads past them idle.
__global__ void __launch_bounds__(1024) crc32_chunk_combine_contig_kernel(CombineArgs a) {
  __shared__ __attribute__((aligned(16))) uint32_t nib[kShiftNibWords];
  __shared__ uint32_t part[16];
  const uint64_t b = blockIdx.x / a.splits;
  const uint32_t s = blockIdx.x % a.splits;
  const uint32_t t = threadIdx.x;
  const uint64_t L = a.inline_bodies ? a.bodies.b[b].len : a.lengths[b];
  const uint64_t nch = L / a.chunk;                       // 4096 * splits (round values: 128 * S, splits = 1)
  const uint64_t first = b * nch;                         // equal bodies back to back
  const uint64_t k0 = 4ull * ((uint64_t)s * 1024u + t); // this thread's first chunk
  const bool live = k0 < nch;
  const uint4 v = live ? *reinterpret_cast<const uint4 *>(a.raw + first + k0) : make_uint4(0u, 0u, 0u, 0u);
  {
    uint4 *dst = reinterpret_cast<uint4 *>(nib);
#pragma unroll
    for (uint32_t q = 0; q < kShiftNibWords / 4 / 1024; ++q) dst[q * 1024 + t] = a.shift_nib[q * 1024 + t];
  }
  __syncthreads();
  const uint32_t ks = (uint32_t)__builtin_ctzll(a.chunk); // A_chunk = one nibble map
  uint32_t acc = nib_apply(nib, ks, nib_apply(nib, ks, nib_apply(nib, ks, v.x) ^ v.y) ^ v.z) ^ v.w;
  acc = nib_shift(nib, live ? (nch - k0 - 4) * a.chunk : 0ull, acc);
  for (int m = 1; m < 64; m <<= 1) acc ^= (uint32_t)__shfl_xor((int)acc, m, 64);
  if ((t & 63u) == 0) part[t >> 6] = acc;
  __syncthreads();
  if (t == 0) {
    for (uint32_t w = 1; w < 16; ++w) acc ^= part[w];
    if (s == 0) acc ^= ~nib_shift(nib, L, 0xFFFFFFFFu);
    atomicXor(a.out + b, acc);
  }
}

// ---------------------------------------------------------------------------
// Synthetic data: counter-based splitmix64 words (same stream as
// oracle_splitmix_fill): word k = mix64(seed + (k+1) * golden), little-endian.
// ---------------------------------------------------------------------------
__device__ __forceinline__ uint64_t mix64(uint64_t z) {
  z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ull;
  z = (z ^ (z >> 27)) * 0x94D049BB133111EBull;
  return z ^ (z >> 31);
}

__global__ void __launch_bounds__(256) splitmix_fill_kernel(uint64_t *dst, uint64_t nwords, uint64_t seed,
                                                             uint64_t word_offset) {
  const uint64_t stride = (uint64_t)gridDim.x * blockDim.x * 2;
  for (uint64_t k = ((uint64_t)blockIdx.x * blockDim.x + threadIdx.x) * 2; k < nwords; k += stride) {
    const uint64_t g = k + word_offset;
    const uint64_t w0 = mix64(seed + (g + 1) * 0x9E3779B97F4A7C15ull);
    if (k + 1 < nwords) {
      const uint64_t w1 = mix64(seed + (g + 2) * 0x9E3779B97F4A7C15ull);
      reinterpret_cast<ulonglong2 *>(dst)[k / 2] = make_ulonglong2(w0, w1);
    } else {
      dst[k] = w0;
    }
  }
}

// ---------------------------------------------------------------------------
// Stream-read probe (bench / DESIGN.md): the achievable HBM read rate for the
// two access shapes the CRC kernel could use over the same buffer.  PATTERN 0:
// lane reads 16 B at lane*16 + b*1024 (fully coalesced); PATTERN 1: lane reads
// its own 64 B segment (lane*64 + b*16), the CRC kernel's shape.
// ---------------------------------------------------------------------------
template <int PATTERN, bool NT>
__global__ void __launch_bounds__(1024, 4) stream_read_kernel(const uint4 *p, uint64_t ntiles, uint32_t *out) {
  const uint32_t lane = threadIdx.x & 63u;
  const uint64_t gw = (uint64_t)blockIdx.x * (blockDim.x >> 6) + (threadIdx.x >> 6);
  const uint64_t nw = (uint64_t)gridDim.x * (blockDim.x >> 6);
  uint32_t acc = 0;
  for (uint64_t t = gw; t < ntiles; t += nw) {
    const uint4 *tile = p + t * 256;
    uint4 v[4];
#pragma unroll
    for (int b = 0; b < 4; ++b) {
      const uint4 *src = tile + (PATTERN == 0 ? (b * 64 + lane) : (lane * 4 + b));
      const rows::u32x4 x = rows::ld16<NT>(reinterpret_cast<const uint8_t *>(src));
      v[b] = make_uint4(x[0], x[1], x[2], x[3]);
    }
#pragma unroll
    for (int b = 0; b < 4; ++b) acc ^= v[b].x ^ v[b].y ^ v[b].z ^ v[b].w;
  }
  if (acc == 0x9E3779B9u) out[0] = acc; // keeps the loads live; practically never stores
}

// ---------------------------------------------------------------------------
// Host-side launchers.
// ---------------------------------------------------------------------------
static constexpr int kBlock = 1024;

// Fraction of a launch's rounds dealt from the steal pool (RPCCRC_STEAL_FRAC,
// 0 disables stealing; NS r02w: 0.08 / 0.15 / 0.25 -> -3.9 / -4.3 / -3.2 %).
// QB = 4 launches (C1) may take their own (RPCCRC_STEAL_FRAC_QB4): 0.08 and
// 0.15 measured the same on C1 with the run order rotated (0.25 +1.3 %;
// profiles/r04k/c1_steal_ab.txt, ab2).
static double env_frac(const char *name, double dflt) {
  const char *e = getenv(name);
  const double v = e ? atof(e) : dflt;
  return (v >= 0.0 && v < 1.0) ? v : dflt;
}
// Round 4 (final tree): 0.08 instead of 0.15 -- NS -1.15 / -0.1 %, C4 -0.7 /
// -0.9 %, C1 -0.45 % on two boxes, rotated (profiles/r04zi, r04zj); 0.05 was
// better still for NS / C4 on one box but +1.5 % for C1, 0.03 +1.5-2 % for all.
// Ragged QB = 1 launches (C2) take a smaller pool (RPCCRC_STEAL_FRAC_RAGGED):
// with the two-phase loop their pool rounds still cost ~30 % more than static
// ones (the protocol at every item switch; a C2 item averages 2.6 rows), so
// the pool is sized to the exit spread it absorbs (~6 % without a pool,
// profiles/r05v) and no larger: C2 rotated A/B on one box, no pool 6073 / 6100
// / 6102 us, 2 % 6069 / 6078 / 6087, 3 % 6041 / 6048 / 6069, 5 % 6052 / 6076 /
// 6079, 8 % 6046 / 6064 / 6066 (profiles/r05x, r05z).
// Uniform QB = 1 (NS, C3, C4's chunks) 6.5 % since the two-phase loop.  Rotated
// A/Bs on three boxes: 5 % beat 8 % on one (NS 593.0 / 594.3 against 597.5 /
// 599.8 us, profiles/r05zb), 6.5 % beat 5 % on the next (NS 596.6-598.1 against
// 601.1-608.1, C4 the same, 4 % worse; r05frac) and matched 8 % on the third
// (r05frac2); 3 % cost 1-2 %.  QB = 4 (C1) keeps 8 % (5 % +1-3 %, 3 % +4-7 %).
static double steal_frac(int QB = 1, bool ragged = false) {
  static const double f1 = env_frac("RPCCRC_STEAL_FRAC", 0.065);
  static const double f4 = env_frac("RPCCRC_STEAL_FRAC_QB4", 0.08);
  static const double fr = env_frac("RPCCRC_STEAL_FRAC_RAGGED", 0.03);
  return QB == 4 ? f4 : ragged ? fr : f1;
}
// Device-counted launches (the big-body route's chunk and span passes, sized in
// the kernel) keep the round-4 pool of 8 %: lifted-cap frames verify 543-545 us
// with it against 554-567 with 5 % (rotated, one box, profiles/r05fl2).
static double steal_frac_dev() {
  static const double f = env_frac("RPCCRC_STEAL_FRAC_DEV", 0.08);
  return f;
}
// ... but at most this many pool rounds per workgroup: the pool has to absorb
// the workgroups' spread in finishing time, not a share of an ever larger
// batch, and every pool round costs a device-scope claim.  C3 (8M x 4 KiB,
// 1024 rounds per workgroup): 15 % 4778 us, 5 % 4724 us, 30 % 4846 us
// (profiles/r04zf, rotated); with this cap of 48 (4.7 %) 4752 against 4789 us
// uncapped (r04zg); caps of 16 / 24 / 32 were within that box's noise (r04zh).
// The north star (128 rounds per workgroup, 19 in the pool) and smaller
// launches are below the cap.  RPCCRC_STEAL_MAX_PER_WG overrides it (A/B).
static uint32_t steal_max_per_wg() {
  static const uint32_t v = [] {
    const char *e = getenv("RPCCRC_STEAL_MAX_PER_WG");
    const long x = e ? atol(e) : 0;
    return x > 0 ? (uint32_t)x : 48u;
  }();
  return v;
}

hipError_t launch_rows(const ItemsArgs &a, int QB, bool nt, int max_blocks, hipStream_t stream, hipEvent_t steal_done,
                       bool *steal_recorded) {
  if (a.n_items == 0) return hipSuccess;
  // The kernel indexes items and tasks in 32 bits: launches of at most
  // kMaxLaunchItems (a multiple of 4: QB = 4 groups never straddle launches).
  if (a.n_items > kMaxLaunchItems) {
    if (a.n_dev != nullptr || a.out_idx != nullptr || a.routed != nullptr || a.round_out != nullptr)
      return hipErrorInvalidValue;
    for (uint64_t s0 = 0; s0 < a.n_items; s0 += kMaxLaunchItems) {
      ItemsArgs b = a;
      b.n_items = std::min<uint64_t>(kMaxLaunchItems, a.n_items - s0);
      if (b.offsets) {
        b.offsets += s0;
        b.lengths += s0;
      } else {
        b.base += s0 * a.stride;
      }
      b.out += s0;
      const hipError_t e = launch_rows(b, QB, nt, max_blocks, stream, steal_done, steal_recorded);
      if (e != hipSuccess) return e;
    }
    return hipSuccess;
  }
  // One row per step (PAIR = 1), 16-wave (1024-thread) workgroups, one per CU.
  constexpr int kWaves = 16;
  const uint64_t per_wave = (QB == 4) ? 4 : 1;
  const uint64_t waves = (a.n_items + per_wave - 1) / per_wave;
  uint64_t blocks = (waves + kWaves - 1) / kWaves;
  if (blocks > (uint64_t)max_blocks) blocks = (uint64_t)max_blocks;
  const dim3 grid((unsigned)blocks), block(kWaves * 64);
  const bool ragged = a.offsets != nullptr;
  if (ragged != (a.lengths != nullptr)) return hipErrorInvalidValue;
  // Workgroup-dynamic dealing (crc32_rows.h DYN) once every workgroup has
  // several rounds of 32 tasks; small batches (e.g. the chunks of a few large
  // bodies) keep the static one-task-per-wave dealing.
  const uint64_t n_tasks = (QB == 4) ? (a.n_items + 3) / 4 : a.n_items;
  const uint64_t round = dyn_round(QB);
  const bool dyn = n_tasks >= 8ull * round * blocks;
  // Tail stealing (DYN, host-counted): the last steal_frac of the
  // rounds go to the device-counter pool, the rest stay static per workgroup.
  ItemsArgs k = a;
  k.steal_s = 0;
  k.steal_permille = (uint32_t)(steal_frac_dev() * 1000.0 + 0.5); // (device-counted launches only)
  k.steal_max_wg = steal_max_per_wg();
  if (dyn && a.steal != nullptr && a.n_dev == nullptr) {
    const uint64_t rounds = (n_tasks + round - 1) / round;
    uint64_t st = (uint64_t)((double)rounds * (1.0 - steal_frac(QB, ragged))) / blocks;
    if (rounds / blocks > st + k.steal_max_wg) st = rounds / blocks - k.steal_max_wg; // the cap
    if (st >= kStealAhead && st * blocks < rounds) k.steal_s = (uint32_t)st;
  } else if (dyn && a.steal != nullptr && k.steal_permille > 0) {
    k.steal_s = kStealOnDevice; // device-counted: the kernel sizes the pool from *n_dev
  }
  if (k.steal_s == 0) k.steal = nullptr;
  if (a.span_ctl != nullptr) { // kRowsSpanBnd: the dense span pass (DYN, 4096-byte uniform RAW items, device count)
    if (QB != 1 || ragged || !dyn || a.len != 4096 || a.stride != 4096 || a.mode != kModeRaw || a.n_dev == nullptr ||
        a.out_idx != nullptr || a.span_rec == nullptr || a.span_bnd == nullptr || a.span_bpos == nullptr)
      return hipErrorInvalidValue;
#define RPCCRC_ROWS_SPAN(N)                                                                                       \
  do {                                                                                                            \
    if (k.steal_s && steal_done) {                                                                                \
      hipExtLaunchKernelGGL((crc32_rows_kernel<1, N, false, kRowsSpanBnd, 1, true, true>), grid, block, 0, stream, \
                            nullptr, steal_done, 0, k);                                                           \
      if (steal_recorded) *steal_recorded = true;                                                                 \
    } else if (k.steal_s) {                                                                                       \
      hipLaunchKernelGGL((crc32_rows_kernel<1, N, false, kRowsSpanBnd, 1, true, true>), grid, block, 0, stream, k); \
    } else {                                                                                                      \
      hipLaunchKernelGGL((crc32_rows_kernel<1, N, false, kRowsSpanBnd, 1, true>), grid, block, 0, stream, k);    \
    }                                                                                                             \
  } while (0)
    if (nt) RPCCRC_ROWS_SPAN(true); else RPCCRC_ROWS_SPAN(false);
#undef RPCCRC_ROWS_SPAN
    return hipGetLastError();
  }
  if (a.round_out != nullptr) { // kRowsRoundOut: whole DYN rounds of 4096-byte uniform RAW items
    if (QB != 1 || ragged || !dyn || a.len != 4096 || a.stride != 4096 || a.mode != kModeRaw ||
        a.out_idx != nullptr || (reinterpret_cast<uintptr_t>(a.base) & 15u) != 0)
      return hipErrorInvalidValue;
#define RPCCRC_ROWS_ROUND(N)                                                                                      \
  do {                                                                                                            \
    if (k.steal_s && steal_done) {                                                                                \
      hipExtLaunchKernelGGL((crc32_rows_kernel<1, N, false, kRowsRoundOut, 1, true, true>), grid, block, 0, stream, \
                            nullptr, steal_done, 0, k);                                                           \
      if (steal_recorded) *steal_recorded = true;                                                                 \
    } else if (k.steal_s) {                                                                                       \
      hipLaunchKernelGGL((crc32_rows_kernel<1, N, false, kRowsRoundOut, 1, true, true>), grid, block, 0, stream, k); \
    } else {                                                                                                      \
      hipLaunchKernelGGL((crc32_rows_kernel<1, N, false, kRowsRoundOut, 1, true>), grid, block, 0, stream, k);    \
    }                                                                                                             \
  } while (0)
    if (nt) RPCCRC_ROWS_ROUND(true); else RPCCRC_ROWS_ROUND(false);
#undef RPCCRC_ROWS_ROUND
    return hipGetLastError();
  }
#define RPCCRC_ROWS(Q, N, R)                                                                      \
  do {                                                                                            \
    if (dyn && k.steal_s) {                                                                       \
      if (steal_done) {                                                                           \
        hipExtLaunchKernelGGL((crc32_rows_kernel<Q, N, R, 0, 1, true, true>), grid, block, 0, stream, nullptr, \
                              steal_done, 0, k);                                                  \
        if (steal_recorded) *steal_recorded = true;                                               \
      } else {                                                                                    \
        hipLaunchKernelGGL((crc32_rows_kernel<Q, N, R, 0, 1, true, true>), grid, block, 0, stream, k); \
      }                                                                                           \
    }                                                                                             \
    else if (dyn) hipLaunchKernelGGL((crc32_rows_kernel<Q, N, R, 0, 1, true>), grid, block, 0, stream, k); \
    else hipLaunchKernelGGL((crc32_rows_kernel<Q, N, R>), grid, block, 0, stream, k);             \
  } while (0)
  if (QB == 4) {
    if (ragged) {
      if (nt) RPCCRC_ROWS(4, true, true); else RPCCRC_ROWS(4, false, true);
    } else {
      if (nt) RPCCRC_ROWS(4, true, false); else RPCCRC_ROWS(4, false, false);
    }
  } else {
    if (ragged) {
      if (nt) RPCCRC_ROWS(1, true, true); else RPCCRC_ROWS(1, false, true);
    } else {
      if (nt) RPCCRC_ROWS(1, true, false); else RPCCRC_ROWS(1, false, false);
    }
  }
#undef RPCCRC_ROWS
  return hipGetLastError();
}

hipError_t launch_chunk_combine(const CombineArgs &a, hipStream_t stream, hipEvent_t done) {
  if (a.n_bodies == 0) return done ? hipEventRecord(done, stream) : hipSuccess;
  const uint64_t blocks = a.n_bodies * a.splits;
  if (a.splits == 0 || blocks >= (1ull << 31)) return hipErrorInvalidValue;
  if (a.inline_bodies && a.n_bodies > kInlineBodies) return hipErrorInvalidValue;
  if (a.contig)
    hipExtLaunchKernelGGL(crc32_chunk_combine_contig_kernel, dim3((unsigned)blocks), dim3(1024), 0, stream, nullptr,
                          done, 0, a);
  else if (a.splits == 1)
    hipExtLaunchKernelGGL(crc32_chunk_combine_kernel<1024>, dim3((unsigned)blocks), dim3(1024), 0, stream, nullptr,
                          done, 0, a);
  else
    hipExtLaunchKernelGGL(crc32_chunk_combine_kernel<256>, dim3((unsigned)blocks), dim3(256), 0, stream, nullptr,
                          done, 0, a);
  return hipGetLastError();
}

// ---------------------------------------------------------------------------
// Packed ragged batches (crc32_packed.h): per-body chunk counts, their
// exclusive scan (rocPRIM), the slice plan, then the packed kernel.  All four
// are stream-ordered; nothing here waits on the device.
// ---------------------------------------------------------------------------
namespace {

__global__ void __launch_bounds__(256) packed_count_kernel(const uint8_t *base, const uint64_t *offsets,
                                                           const uint32_t *lengths, uint64_t n, uint32_t *cnt,
                                                           uint32_t *out) {
  const uint64_t i = (uint64_t)blockIdx.x * 256u + threadIdx.x;
  if (i >= n) return;
  const uint32_t len = lengths[i];
  cnt[i] = packed::body_chunks((uint64_t)(uintptr_t)base + offsets[i] + len, len);
  if (len == 0) out[i] = 0u; // empty bodies never enter the chunk stream (zlib: crc of nothing = 0)
}

// Thread i = 0..n writes the record {i, lengths[i], offsets[i]} of every slice
// whose first chunk s*S lies in (cfirst[i-1], cfirst[i]] (thread n, the
// sentinel {n, 0, 0}, up to nslices).
__global__ void __launch_bounds__(256) packed_plan_kernel(const uint64_t *cfirst, const uint32_t *cnt,
                                                          const uint64_t *offsets, const uint32_t *lengths, uint64_t n,
                                                          uint64_t max_slices, uint64_t min_slice, uint4 *slice_rec,
                                                          uint64_t *plan) {
  const uint64_t i = (uint64_t)blockIdx.x * 256u + threadIdx.x;
  if (i > n) return;
  const uint64_t total = cfirst[n - 1] + cnt[n - 1];
  uint64_t S = (total + max_slices - 1) / max_slices;
  if (S < min_slice) S = min_slice;
  const uint64_t nslices = (total + S - 1) / S;
  if (i == 0) {
    plan[0] = nslices;
    plan[1] = S;
  }
  const uint64_t s_lo = (i == 0) ? 0 : cfirst[i - 1] / S + 1;
  uint64_t s_hi = (i < n) ? cfirst[i] / S : nslices;
  if (s_hi > nslices) s_hi = nslices;
  if (s_lo > s_hi) return;
  const uint64_t off = (i < n) ? offsets[i] : 0;
  const uint4 r = make_uint4((uint32_t)i, (i < n) ? lengths[i] : 0u, (uint32_t)off, (uint32_t)(off >> 32));
  for (uint64_t s = s_lo; s <= s_hi; ++s) slice_rec[s] = r;
}

constexpr size_t align256(size_t x) { return (x + 255) & ~(size_t)255; }

hipError_t packed_scan(void *tmp, size_t &bytes, const uint32_t *cnt, uint64_t *cfirst, uint64_t n, hipStream_t s) {
  return rocprim::exclusive_scan(tmp, bytes, cnt, cfirst, (uint64_t)0, (size_t)n, rocprim::plus<uint64_t>(), s);
}
} // namespace

hipError_t packed_workspace_bytes(uint64_t n, uint64_t max_slices, size_t *bytes) {
  size_t scan = 0;
  const hipError_t e = packed_scan(nullptr, scan, nullptr, nullptr, n, nullptr);
  if (e != hipSuccess) return e;
  *bytes = align256(n * 4) + align256(n * 8) + align256((max_slices + 1) * 16) + align256(16) + align256(scan);
  return hipSuccess;
}

hipError_t launch_packed_batch(const PackedBatch &p, bool nt, int max_blocks, hipStream_t s) {
  if (p.n == 0) return hipSuccess;
  if (p.n >= 0xFFFFFFFFull || p.max_slices == 0 || p.min_slice == 0) return hipErrorInvalidValue;
  uint8_t *w = static_cast<uint8_t *>(p.ws);
  uint32_t *cnt = reinterpret_cast<uint32_t *>(w);
  w += align256(p.n * 4);
  uint64_t *cfirst = reinterpret_cast<uint64_t *>(w);
  w += align256(p.n * 8);
  uint4 *slices = reinterpret_cast<uint4 *>(w);
  w += align256((p.max_slices + 1) * 16);
  uint64_t *plan = reinterpret_cast<uint64_t *>(w);
  w += align256(16);
  const size_t used = (size_t)(w - static_cast<uint8_t *>(p.ws));
  if (used > p.ws_bytes) return hipErrorInvalidValue;
  size_t scan = p.ws_bytes - used;
  hipLaunchKernelGGL(packed_count_kernel, dim3((unsigned)((p.n + 255) / 256)), dim3(256), 0, s, p.base, p.offsets,
                     p.lengths, p.n, cnt, p.out);
  hipError_t e = hipGetLastError();
  if (e != hipSuccess) return e;
  e = packed_scan(w, scan, cnt, cfirst, p.n, s);
  if (e != hipSuccess) return e;
  hipLaunchKernelGGL(packed_plan_kernel, dim3((unsigned)((p.n + 1 + 255) / 256)), dim3(256), 0, s, cfirst, cnt,
                     p.offsets, p.lengths, p.n, p.max_slices, p.min_slice, slices, plan);
  e = hipGetLastError();
  if (e != hipSuccess) return e;
  PackedArgs a;
  a.base = p.base;
  a.offsets = p.offsets;
  a.lengths = p.lengths;
  a.n_items = p.n;
  a.slice_rec = slices;
  a.plan = plan;
  a.mode = p.mode;
  a.lds_image = p.lds_image;
  a.tq = p.tq;
  a.out = p.out;
  // One 1024-thread workgroup per CU; waves beyond the slice count exit at once.
  uint64_t blocks = (p.max_slices + 15) / 16;
  if (blocks > (uint64_t)max_blocks) blocks = (uint64_t)max_blocks;
  if (nt)
    hipLaunchKernelGGL((crc32_packed_kernel<true>), dim3((unsigned)blocks), dim3(1024), 0, s, a);
  else
    hipLaunchKernelGGL((crc32_packed_kernel<false>), dim3((unsigned)blocks), dim3(1024), 0, s, a);
  return hipGetLastError();
}

// ---------------------------------------------------------------------------
// Split ragged batches: bodies whose bytes plus 16-B end pad fit a 1 KiB
// quarter ("small") go four to a row through the QB = 4 rows kernel, the rest
// one body per row sequence (QB = 1).  An exclusive scan (rocPRIM) of the small
// flags, computed as it reads them, and an order-preserving scatter build both
// lists and their counts on the device (no host round trip); each rows kernel reads its count from the
// device and writes CRC i to out[idx[i]].  Frames batches (bodies <= 1 KiB,
// rpc.h:17) take this path: almost every body is small.
// ---------------------------------------------------------------------------
namespace {

__device__ __forceinline__ bool small_body(const uint8_t *base, uint64_t off, uint32_t len) {
  const uint32_t z = (uint32_t)(0u - (uint32_t)((uint64_t)(uintptr_t)base + off + len)) & 15u;
  return len + z <= 1024u;
}

// Item i's small flag, computed where the scan reads it (round 5: the flags
// were a kernel and an array of their own, 5 us and a launch per call).
struct SmallFlag {
  const uint8_t *base;
  const uint64_t *offsets;
  const uint32_t *lengths;
  __host__ __device__ uint32_t operator()(uint64_t i) const {
#if defined(__HIP_DEVICE_COMPILE__)
    return small_body(base, offsets[i], lengths[i]) ? 1u : 0u;
#else
    return 0u; // (the host never evaluates it)
#endif
  }
};
using SmallFlags = rocprim::transform_iterator<rocprim::counting_iterator<uint64_t>, SmallFlag, uint32_t>;

// Item i goes to slot pos[i] of the small list or slot i - pos[i] of the big
// one (stable: both lists keep batch order, so consecutive tasks stay
// neighbours in memory).  Thread n - 1 publishes both counts.
__global__ void __launch_bounds__(256) split_scatter_kernel(const uint8_t *base, const uint64_t *offsets,
                                                            const uint32_t *lengths, uint64_t n, const uint32_t *pos,
                                                            SplitLists l) {
  const uint64_t i = (uint64_t)blockIdx.x * 256u + threadIdx.x;
  if (i >= n) return;
  const uint64_t off = offsets[i];
  const uint32_t len = lengths[i];
  const uint32_t f = small_body(base, off, len) ? 1u : 0u, p = pos[i];
  if (f) {
    l.s_off[p] = off;
    l.s_len[p] = len;
    l.s_idx[p] = (uint32_t)i;
  } else {
    const uint64_t q = i - p;
    l.b_off[q] = off;
    l.b_len[q] = len;
    l.b_idx[q] = (uint32_t)i;
  }
  if (i == n - 1) {
    l.counts[0] = p + f;
    l.counts[1] = n - (p + f);
  }
}

hipError_t split_scan(void *tmp, size_t &bytes, const SmallFlag &f, uint32_t *pos, uint64_t n, hipStream_t s) {
  const SmallFlags flags(rocprim::counting_iterator<uint64_t>(0), f);
  return rocprim::exclusive_scan(tmp, bytes, flags, pos, 0u, (size_t)n, rocprim::plus<uint32_t>(), s);
}
} // namespace

// The small-body kernel (crc32_small.h) for split lists; RPCCRC_SMALL_KERNEL=0
// restores the rows kernel's QB = 4 loop (A/B).
bool small_kernel_on() {
  static const bool on = [] {
    const char *e = getenv("RPCCRC_SMALL_KERNEL");
    return e == nullptr || atoi(e) != 0;
  }();
  return on;
}

hipError_t launch_small(const ItemsArgs &a, bool nt, int max_blocks, hipStream_t s) {
  if (a.n_items == 0) return hipSuccess;
  if (a.offsets == nullptr || a.lengths == nullptr || a.n_items > kMaxLaunchItems) return hipErrorInvalidValue;
  // every wave at least a few iterations of 16 bodies
  const uint64_t want = (a.n_items + 16 * 16 * 4 - 1) / (16 * 16 * 4);
  const uint64_t blocks = std::max<uint64_t>(1, std::min<uint64_t>(want, (uint64_t)max_blocks));
  const dim3 grid((unsigned)blocks), block(kBlock);
#define RPCCRC_SMALL(N, I) hipLaunchKernelGGL((crc32_small_kernel<N, I>), grid, block, 0, s, a)
  if (nt) {
    if (a.out_idx) RPCCRC_SMALL(true, true); else RPCCRC_SMALL(true, false);
  } else {
    if (a.out_idx) RPCCRC_SMALL(false, true); else RPCCRC_SMALL(false, false);
  }
#undef RPCCRC_SMALL
  return hipGetLastError();
}

hipError_t split_workspace_bytes(uint64_t n, size_t *bytes) {
  size_t scan = 0;
  const hipError_t e = split_scan(nullptr, scan, SmallFlag{}, nullptr, n, nullptr);
  if (e != hipSuccess) return e;
  *bytes = align256(n * 4) + align256(16) + 2 * (align256(n * 8) + 2 * align256(n * 4)) + align256(scan);
  return hipSuccess;
}

hipError_t launch_split_batch(const ItemsArgs &proto, void *ws, size_t ws_bytes, bool nt, int max_blocks,
                              hipStream_t s) {
  const uint64_t n = proto.n_items;
  if (n == 0) return hipSuccess;
  if (n > kMaxLaunchItems || proto.offsets == nullptr || proto.lengths == nullptr) return hipErrorInvalidValue;
  uint8_t *w = static_cast<uint8_t *>(ws);
  auto take = [&](size_t bytes) {
    uint8_t *r = w;
    w += align256(bytes);
    return r;
  };
  uint32_t *pos = reinterpret_cast<uint32_t *>(take(n * 4));
  SplitLists l;
  l.counts = reinterpret_cast<uint64_t *>(take(16));
  l.s_off = reinterpret_cast<uint64_t *>(take(n * 8));
  l.s_len = reinterpret_cast<uint32_t *>(take(n * 4));
  l.s_idx = reinterpret_cast<uint32_t *>(take(n * 4));
  l.b_off = reinterpret_cast<uint64_t *>(take(n * 8));
  l.b_len = reinterpret_cast<uint32_t *>(take(n * 4));
  l.b_idx = reinterpret_cast<uint32_t *>(take(n * 4));
  const size_t used = (size_t)(w - static_cast<uint8_t *>(ws));
  if (used > ws_bytes) return hipErrorInvalidValue;
  size_t scan = ws_bytes - used;
  const dim3 g((unsigned)((n + 255) / 256));
  hipError_t e = split_scan(w, scan, SmallFlag{proto.base, proto.offsets, proto.lengths}, pos, n, s);
  if (e != hipSuccess) return e;
  hipLaunchKernelGGL(split_scatter_kernel, g, dim3(256), 0, s, proto.base, proto.offsets, proto.lengths, n, pos, l);
  e = hipGetLastError();
  if (e != hipSuccess) return e;
  ItemsArgs a = proto; // small bodies, four per row
  a.offsets = l.s_off;
  a.lengths = l.s_len;
  a.n_dev = l.counts;
  a.out_idx = l.s_idx;
  e = small_kernel_on() ? launch_small(a, nt, max_blocks, s) : launch_rows(a, 4, nt, max_blocks, s);
  if (e != hipSuccess) return e;
  a.offsets = l.b_off; // the rest, one body per row sequence
  a.lengths = l.b_len;
  a.n_dev = l.counts + 1;
  a.out_idx = l.b_idx;
  return launch_rows(a, 1, nt, max_blocks, s);
}

// ---------------------------------------------------------------------------
// Big bodies of a ragged batch (crc32_kernels.h BigRoute): a
// classify pass before the rows pass claims up to kBigMaxBodies bodies of
// >= kBigMin bytes (the rows pass then takes them as empty), and after it a
// one-block plan picks a power-of-two chunk so the chunks fit kBigMaxChunks,
// an expand pass writes the chunk table, the rows kernel CRCs the chunks
// (RAW) and a persistent combine folds them per body.  Every count stays on
// the device; the host only launches.
// ---------------------------------------------------------------------------
namespace {

__global__ void __launch_bounds__(256) big_classify_kernel(const uint32_t *lengths, uint64_t n, uint32_t big_min,
                                                             BigRoute r) {
  const uint64_t i = (uint64_t)blockIdx.x * 256u + threadIdx.x;
  const uint32_t lane = threadIdx.x & 63u;
  const bool dense = r.skip != nullptr && *r.skip != 0u; // (uniform) the dense step has every body
  const uint32_t len = (i < n) ? lengths[i] : 0u;
  const bool big = !dense && i < n && len >= big_min;
  const uint64_t m = __builtin_amdgcn_ballot_w64(big);
  uint64_t routed = 0;
  if (m != 0) { // wave-uniform: one slot claim per wave
    unsigned long long base = 0;
    if (lane == 0) base = atomicAdd(reinterpret_cast<unsigned long long *>(&r.meta[0]), (unsigned long long)__popcll(m));
    base = __shfl(base, 0, 64);
    const uint64_t slot = base + (uint64_t)__popcll(m & ((1ull << lane) - 1ull));
    const bool take = big && slot < kBigMaxBodies;
    if (take) {
      r.b_idx[slot] = (uint32_t)i;
      atomicAdd(reinterpret_cast<unsigned long long *>(&r.meta[1]), (unsigned long long)len);
    }
    routed = __builtin_amdgcn_ballot_w64(take);
  }
  const uint64_t w0 = i - lane; // the wave's first item (a multiple of 64): its two bitmap words
  if (w0 < n) {
    if (lane == 0) r.routed[w0 >> 5] = (uint32_t)routed;
    if (lane == 32) r.routed[(w0 >> 5) + 1] = (uint32_t)(routed >> 32);
  }
}

__device__ __forceinline__ uint64_t big_count(const BigRoute &r) {
  if (r.all_n) return r.all_n;
  const uint64_t c = r.meta[0];
  return c < kBigMaxBodies ? c : kBigMaxBodies;
}
__device__ __forceinline__ uint32_t big_body(const BigRoute &r, uint64_t b) { return r.all_n ? (uint32_t)b : r.b_idx[b]; }

// One block: chunk size, per-body chunk counts and their exclusive scan
// (route-all: also the routed bytes, which classify sums otherwise).
__global__ void __launch_bounds__(1024) big_plan_kernel(const uint32_t *lengths, BigRoute r) {
  __shared__ unsigned long long wsum[16];
  __shared__ unsigned long long run;
  const uint64_t nb = big_count(r);
  const uint32_t t = threadIdx.x, lane = t & 63u, w = t >> 6;
  if (nb == 0) {
    if (t == 0) {
      r.meta[2] = 0;
      r.meta[3] = r.min_chunk;
    }
    return;
  }
  uint64_t bytes;
  if (r.all_n) {
    unsigned long long x = 0;
    for (uint64_t b = t; b < nb; b += 1024) x += lengths[b];
    for (int m = 32; m >= 1; m >>= 1) x += __shfl_xor(x, m, 64);
    if (lane == 0) wsum[w] = x;
    __syncthreads();
    bytes = 0;
    for (uint32_t k = 0; k < 16; ++k) bytes += wsum[k];
    __syncthreads();
  } else {
    bytes = r.meta[1];
  }
  // Chunks of (2^k) * 4096 - 16 bytes: end-aligned chunks all share their body's
  // end pad z < 16, so each takes exactly 2^k rows (a 4096-byte chunk with
  // z != 0 would take two).  sum ceil(len / chunk) <= bytes / chunk + 1 + nb
  uint64_t chunk = r.min_chunk;
  while (bytes / chunk + 1 + nb > kBigMaxChunks) chunk = ((chunk + 16) << 1) - 16;
  if (t == 0) run = 0;
  __syncthreads();
  for (uint64_t base = 0; base < nb; base += 1024) {
    const uint64_t b = base + t;
    const unsigned long long c = (b < nb) ? ((uint64_t)lengths[big_body(r, b)] + chunk - 1) / chunk : 0ull;
    unsigned long long x = c; // inclusive wave scan
    for (int d = 1; d < 64; d <<= 1) {
      const unsigned long long y = __shfl_up(x, d, 64);
      if (lane >= (uint32_t)d) x += y;
    }
    if (lane == 63) wsum[w] = x;
    __syncthreads();
    unsigned long long pre = run;
    for (uint32_t k = 0; k < w; ++k) pre += wsum[k];
    if (b < nb) r.b_first[b] = pre + x - c;
    __syncthreads();
    if (t == 1023) run = pre + x;
    __syncthreads();
  }
  if (t == 0) {
    r.b_first[nb] = run;
    r.meta[2] = run;
    r.meta[3] = chunk;
  }
}

// Chunk table: end-aligned chunks of each routed body (the first one partial).
// Block k takes bodies k, k + grid, ...; its threads stride over the body's
// chunks (round 2 searched the body of every chunk: ~9 dependent global loads
// per chunk, 20 us for 0.9M chunks).
__global__ void __launch_bounds__(256) big_expand_kernel(const uint64_t *offsets, const uint32_t *lengths, BigRoute r) {
  const uint64_t nb = big_count(r), chunk = r.meta[3];
  for (uint64_t b = blockIdx.x; b < nb; b += gridDim.x) {
    const uint32_t i = big_body(r, b);
    const uint64_t L = lengths[i], first = r.b_first[b], nch = r.b_first[b + 1] - first, off = offsets[i];
    for (uint64_t k = threadIdx.x; k < nch; k += 256) {
      const uint64_t end = L - (nch - 1 - k) * chunk;
      const uint64_t start = end > chunk ? end - chunk : 0;
      r.c_off[first + k] = off + start;
      r.c_len[first + k] = (uint32_t)(end - start);
    }
  }
}

// Persistent fold: block b takes routed bodies b, b + grid, ...: thread t runs
// Horner over chunks t, t + 1024, ... with the step map A_{1024 * chunk},
// shifts its partial by A_{j * chunk} to the body end (j = chunks after its
// last one, < 1024: one map per set bit of j from the doubling tables
// A_{chunk * 2^i}), and the block XOR-reduces:
//   crc = ~(XOR_k A_{(nch-1-k) chunk}(raw_k)),  raw_0 ^= A_{len_0}(F):
// the zlib pre-conditioning enters with chunk 0 (Tq for len_0 <= 4096), so no
// shift by the whole body length follows the reduction.  (The chunk is
// 2^k * 4096 - 16 bytes, not a power of two: the maps are built per block.)
__device__ __forceinline__ uint32_t nib_map(const uint32_t *m, uint32_t v) {
  uint32_t r = 0;
#pragma unroll
  for (uint32_t i = 0; i < 8; ++i) r ^= m[i * 16u + ((v >> (4u * i)) & 15u)];
  return r;
}
__global__ void __launch_bounds__(1024) big_combine_kernel(const uint32_t *lengths, BigRoute r, const uint4 *shift_nib,
                                                           uint32_t *out) {
  constexpr uint32_t kHiMaps = 20;                // A_{2^k}, k = 12..31: the seed's shift by len0 & ~4095
  __shared__ uint32_t nibhi[kHiMaps * 128];
  __shared__ uint32_t part[16];
  __shared__ uint32_t dbl[kBigDbl * 128];         // [i][n][j] = A_{chunk * 2^i}(j << 4n), the chunk's class
  const uint64_t nb = big_count(r);
  if (blockIdx.x >= nb) return;
  const uint32_t t = threadIdx.x;
  const uint64_t chunk = r.meta[3];
  const uint32_t m = (uint32_t)__builtin_ctzll((chunk + 16) >> 12); // chunk = 4096 * 2^m - 16
  {
    const uint32_t *src = reinterpret_cast<const uint32_t *>(shift_nib) + 12u * 128u;
    for (uint32_t e = t; e < kHiMaps * 128; e += 1024) nibhi[e] = src[e];
    for (uint32_t e = t; e < kBigDbl * 128; e += 1024) dbl[e] = r.dbl[m * kBigDbl * 128 + e];
  }
  __syncthreads();
  const uint32_t *stepnib = dbl + 10 * 128; // A_{1024 * chunk}
  for (uint64_t b = blockIdx.x; b < nb; b += gridDim.x) {
    const uint32_t i = big_body(r, b);
    const uint64_t L = lengths[i], first = r.b_first[b], nch = r.b_first[b + 1] - first;
    uint32_t acc = 0;
    // zlib's pre-conditioning, carried in from the body's first byte by chunk 0
    // (thread 0): A_{len0}(F) = A_{4096 q}(Tq[len0 mod 4096]), one map for q = 1
    uint32_t seed = 0;
    if (t == 0 && nch != 0) {
      const uint64_t len0 = L - (nch - 1) * chunk;
      seed = r.tq[len0 & 4095u];
      for (uint64_t q = len0 >> 12; q; q &= q - 1) seed = nib_map(nibhi + 128u * (uint32_t)__builtin_ctzll(q), seed);
    }
    // The thread's raw CRCs are loaded kB at a time ahead of the Horner chain
    // (one dependent global load per step left the fold latency-bound).
    constexpr uint32_t kB = 8;
    for (uint64_t k0 = t; k0 < nch; k0 += (uint64_t)kB * 1024u) {
      uint32_t rv[kB];
#pragma unroll
      for (uint32_t q = 0; q < kB; ++q) rv[q] = (k0 + q * 1024u < nch) ? r.c_raw[first + k0 + q * 1024u] : 0u;
#pragma unroll
      for (uint32_t q = 0; q < kB; ++q)
        if (k0 + q * 1024u < nch) acc = nib_map(stepnib, acc) ^ rv[q] ^ (k0 + q == 0 ? seed : 0u);
    }
    if (t < nch) {
      uint32_t j = (uint32_t)((nch - 1 - t) % 1024u); // chunks after this thread's last one
      while (j) {
        acc = nib_map(dbl + 128u * (uint32_t)__builtin_ctz(j), acc);
        j &= j - 1;
      }
    }
    for (int m = 1; m < 64; m <<= 1) acc ^= (uint32_t)__shfl_xor((int)acc, m, 64);
    if ((t & 63u) == 0) part[t >> 6] = acc;
    __syncthreads();
    if (t == 0) {
      for (uint32_t w = 1; w < 16; ++w) acc ^= part[w];
      out[i] = nch ? ~acc : 0u; // an empty body: crc32 = 0
    }
    __syncthreads();
  }
}

// ---- address-aligned chunks (round 4; BigRoute.aligned) ----------------------
// The chunks of a routed body [s, e) (absolute addresses) are its pieces
// between multiples of the power-of-two chunk C: [max(s, jC), min(e, jC + C)).
// Interior chunks are then whole, aligned C-byte blocks: their rows are
// aligned 4 KiB rows with no edge masks and no 128-B line shared with another
// chunk.  End-aligned chunks of C - 16 bytes (rounds 2-3) put every row at an
// arbitrary 16-B offset: 33 lines per 4 KiB row, the shared ones fetched twice,
// and a front mask on every chunk.  The fold:
//   crc = ~(A_t(G) ^ raw_last),  G = XOR_{k < nch-1} A_{(nch-2-k) C}(raw_k)
// with raw_0 seeded with A_{len_0}(F) (zlib's pre-conditioning) and t the last
// chunk's length; one chunk: crc = ~(raw_0 ^ A_{len_0}(F)).  Every map is a
// power-of-two shift A_{2^k} (shift_nib), so no per-class tables are needed.
__device__ __forceinline__ uint64_t aligned_nch(uint64_t s, uint64_t L, uint32_t lc) {
  return L == 0 ? 0 : ((s + L - 1) >> lc) - (s >> lc) + 1;
}

__global__ void __launch_bounds__(1024) big_plan_aligned_kernel(const uint8_t *base, const uint64_t *offsets,
                                                                const uint32_t *lengths, BigRoute r) {
  __shared__ unsigned long long wsum[16];
  __shared__ unsigned long long run;
  const uint64_t nb = big_count(r);
  const uint32_t t = threadIdx.x, lane = t & 63u, w = t >> 6;
  if (nb == 0) {
    if (t == 0) {
      r.meta[2] = 0;
      r.meta[3] = r.min_chunk;
    }
    return;
  }
  // One pass over the bodies (route-all: the routed bytes; span mode: also the
  // last body end and the bytes of the whole blocks inside bodies, the blocks
  // the fold takes from the span pass), then one block reduction.  A fused
  // frames parse or stamp check (BigRoute.parse / .stamp) produces each body's
  // offset / length here.
  unsigned long long x = 0, hi = 0, inner = 0, disorder = 0;
  const bool sums = r.all_n != 0, span = r.span_rows_max != 0;
  if (sums || r.parse.frame_off != nullptr || r.stamp.frame_off != nullptr) {
    for (uint64_t b = t; b < nb; b += 1024) {
      uint64_t s0, L;
      if (r.parse.frame_off != nullptr) {
        const FrameBody fb = frames_parse_one(r.parse, b);
        s0 = fb.off;
        L = fb.len;
      } else if (r.stamp.frame_off != nullptr) {
        const FrameBody fb = frames_stamp_prep_one(r.stamp, b);
        s0 = fb.off;
        L = fb.len;
        // Span mode's fold reads the partial blocks while it writes headers:
        // only frames in stream order, none overlapping the next, keep every
        // header out of every body (else the chunk route: all CRCs first).
        if (b + 1 < nb && r.stamp.frame_off[b] + kFrameHeaderLen + L > r.stamp.frame_off[b + 1]) disorder = 1;
      } else {
        s0 = span ? offsets[b] : 0;
        L = lengths[b];
      }
      x += L;
      if (span && L != 0) {
        const uint64_t e = s0 + L, j0 = s0 >> 12, j1 = (e - 1) >> 12;
        hi = e > hi ? e : hi;
        inner += (j1 > j0 + 1) ? (j1 - j0 - 1) << 12 : 0ull;
      }
    }
  }
  for (int m = 32; m >= 1; m >>= 1) {
    x += __shfl_xor(x, m, 64);
    const unsigned long long h = __shfl_xor(hi, m, 64);
    hi = h > hi ? h : hi;
    inner += __shfl_xor(inner, m, 64);
    disorder |= __shfl_xor(disorder, m, 64);
  }
  __shared__ unsigned long long wred[4][16];
  if (lane == 0) {
    wred[0][w] = x;
    wred[1][w] = hi;
    wred[2][w] = inner;
    wred[3][w] = disorder;
  }
  __syncthreads(); // (also orders the parse's stores before the chunk scan below reads them)
  unsigned long long x_all = 0, hi_all = 0, inner_all = 0, disorder_all = 0;
  for (uint32_t k = 0; k < 16; ++k) {
    x_all += wred[0][k];
    hi_all = wred[1][k] > hi_all ? wred[1][k] : hi_all;
    inner_all += wred[2][k];
    disorder_all |= wred[3][k];
  }
  const uint64_t bytes = sums ? x_all : r.meta[1];
  if (span) { // span mode (route-all, base 4 KiB-aligned; BigRoute)
    // Dense: the span pass reads at most 1/16 more than the interior blocks (+ 1 MiB).
    const uint64_t rows = hi_all >> 12;
    const bool dense =
        rows <= r.span_rows_max && (rows << 12) <= inner_all + inner_all / 16 + (1ull << 20) && disorder_all == 0;
    if (t == 0) {
      r.meta[4] = dense ? rows : 0;
      r.meta[5] = dense ? 1 : 0;
      if (dense) {
        r.meta[2] = 0; // no chunks for the ragged chunk pass
        r.meta[3] = 4096;
      }
    }
    if (dense) return;
  }
  // sum over bodies of (L / C + 2) bounds the chunks
  uint64_t chunk = r.min_chunk;
  while (bytes / chunk + 2 * nb > kBigMaxChunks) chunk <<= 1;
  const uint32_t lc = (uint32_t)__builtin_ctzll(chunk);
  const uint64_t b0 = (uint64_t)(uintptr_t)base;
  if (t == 0) run = 0;
  __syncthreads();
  for (uint64_t bb = 0; bb < nb; bb += 1024) {
    const uint64_t b = bb + t;
    unsigned long long c = 0;
    if (b < nb) {
      const uint32_t i = big_body(r, b);
      c = aligned_nch(b0 + offsets[i], lengths[i], lc);
    }
    unsigned long long x = c; // inclusive wave scan
    for (int d = 1; d < 64; d <<= 1) {
      const unsigned long long y = __shfl_up(x, d, 64);
      if (lane >= (uint32_t)d) x += y;
    }
    if (lane == 63) wsum[w] = x;
    __syncthreads();
    unsigned long long pre = run;
    for (uint32_t k = 0; k < w; ++k) pre += wsum[k];
    if (b < nb) r.b_first[b] = pre + x - c;
    __syncthreads();
    if (t == 1023) run = pre + x;
    __syncthreads();
  }
  if (t == 0) {
    r.b_first[nb] = run;
    r.meta[2] = run;
    r.meta[3] = chunk;
  }
}

__global__ void __launch_bounds__(256) big_expand_aligned_kernel(const uint8_t *base, const uint64_t *offsets,
                                                                 const uint32_t *lengths, BigRoute r) {
  if (r.span_rows_max != 0 && r.meta[5] != 0) return; // span mode: no chunk table
  const uint64_t nb = big_count(r), chunk = r.meta[3];
  const uint64_t b0 = (uint64_t)(uintptr_t)base;
  for (uint64_t b = blockIdx.x; b < nb; b += gridDim.x) {
    const uint32_t i = big_body(r, b);
    const uint64_t s = b0 + offsets[i], e = s + lengths[i], first = r.b_first[b], nch = r.b_first[b + 1] - first;
    const uint64_t blk0 = s & ~(chunk - 1);
    for (uint64_t k = threadIdx.x; k < nch; k += 256) {
      const uint64_t lo = blk0 + k * chunk;
      const uint64_t cs = lo > s ? lo : s, ce = lo + chunk < e ? lo + chunk : e;
      r.c_off[first + k] = cs - b0;
      r.c_len[first + k] = (uint32_t)(ce - cs);
    }
  }
}

// ---- span mode (BigRoute.span_rows_max; route-all batches) --------------------
// A body [s, e) (offsets from the 4 KiB-aligned base) covers blocks j0..j1: its
// chunks are the aligned chunks of C = 4096 -- the first and last partial
// blocks, which the fold CRCs itself (span_piece_wave, one wave each), and the
// interior blocks j0 < j < j1, whose crc0 the span pass (uniform rows, RAW)
// left in blk[j].  (Round 4 tried the two pieces as a window over all 1024
// threads with two block-wide reductions -- fold 43.6 us for 1024 frames -- and
// as items of the ragged chunk pass -- 16.4 us for that pass:
// profiles/r04e, r04f prof_frames.)
//
// crc0 of a piece [ps, pe) of <= 4096 bytes by ONE wave: the piece right-
// aligned in a 4096-byte window (leading zeros leave crc0 unchanged), lane L
// takes window bytes [64 L, 64 L + 64): 16 slice-by-4 steps from T (the
// scalar kernel's tables, T_k at T + 256 k), then six pair levels, the left
// group shifted past the right one's 64 * 2^b bytes by NIB[6 + b].  The words
// come from 17 aligned dword loads per lane through a buffer resource based at
// ps & ~3 and v_alignbyte; a dword before the resource gets kOobOffset (reads
// 0 without an access) -- not its wrapped offset, which with constant-adjacent
// offsets merged two loads into one partly out-of-range load that read 0 for
// the in-range dword too (r04e); bytes before ps are masked.
constexpr uint32_t kFoldThreads = 256, kFoldLog2 = 8, kFoldWaves = kFoldThreads / 64;
// Raw chunk CRCs each thread loads before its Horner steps (a 64 MiB body in
// 4 KiB span blocks is 64 steps per thread: 2 round trips, 8 with 8 in flight).
constexpr uint32_t kFoldBatch = 32;
// BigRoute.cmp_*: frames_compare_kernel's rule, in the fold (route-all frames verify).
__device__ __forceinline__ void fold_verdict(const BigRoute &r, uint32_t i, uint32_t crc) {
  const uint8_t p = r.cmp_pre[i];
  r.cmp_verdict[i] = (p != kFramePending) ? p : (crc == r.cmp_expected[i] ? RPC_FRAME_OK : RPC_FRAME_BAD_CRC);
}
static_assert((1u << kFoldLog2) == kFoldThreads && kFoldThreads == 256, "T4 load: one uint4 per thread");

__device__ __forceinline__ uint32_t span_piece_wave(const uint8_t *base, uint64_t ps, uint64_t pe, uint32_t lane,
                                                    const uint32_t *T, const uint32_t *nib) {
  const uint64_t B = ps & ~3ull;
  const uint32_t span = (uint32_t)(pe - B); // <= 4099
  const uint32_t lim = (span + 3u) & ~3u;
  const uint32_t r = (uint32_t)pe & 3u;
  const __amdgpu_buffer_rsrc_t rs =
      __builtin_amdgcn_make_buffer_rsrc(const_cast<uint8_t *>(base + B), (short)0, (int)lim, 0x00020000);
  const uint32_t a0 = span - 4096u + 64u * lane - r; // aligned; wraps before B
  const int kmin = (int)(4096u - (uint32_t)(pe - ps)); // window bytes before the piece
  uint32_t d[17];
#pragma unroll
  for (uint32_t k = 0; k < 17; ++k) {
    const uint32_t off = a0 + 4u * k;
    d[k] = (uint32_t)__builtin_amdgcn_raw_buffer_load_b32(rs, (int)(off < lim ? off : rows::kOobOffset), 0, 0);
  }
  uint32_t sv = 0;
#pragma unroll
  for (uint32_t k = 0; k < 16; ++k) {
    const uint32_t wd = __builtin_amdgcn_alignbyte(d[k + 1], d[k], r);
    const int dd = kmin - (int)(64u * lane + 4u * k); // bytes of this word before ps
    const uint32_t keep = dd <= 0 ? 0xFFFFFFFFu : (dd >= 4 ? 0u : (0xFFFFFFFFu << (8 * dd)));
    const uint32_t x = sv ^ (wd & keep);
    sv = T[768 + (x & 0xFFu)] ^ T[512 + ((x >> 8) & 0xFFu)] ^ T[256 + ((x >> 16) & 0xFFu)] ^ T[x >> 24];
  }
#pragma unroll
  for (uint32_t b = 0; b < 6; ++b) {
    const uint32_t sh = nib_map(nib + 128u * (6u + b), sv);
    const uint32_t mine = ((lane >> b) & 1u) ? sv : sh;
    sv = mine ^ (uint32_t)__shfl_xor((int)mine, 1 << b, 64);
  }
  return sv;
}

// Block b folds routed bodies b, b + grid, ...: thread t runs Horner over
// chunks t, t + T, ... of the first nch - 1 with the step map A_{T C} (T =
// kFoldThreads), shifts its partial by A_{j C} (j < T chunks after its last
// one), and the block XOR-reduces into G; thread 0 adds the last chunk.  All
// maps are the power-of-two shifts NIB[k] = A_{2^k bytes} (32 KiB, in LDS).
// T = 256 (round 4; 1024 before): a block's cost is mostly fixed -- the map
// table, the two partial blocks (span mode), thread 0's final shifts -- and a
// frames batch has one body per block, so 4x more resident blocks beat 4x
// longer Horner chains on the few long bodies (1024 frames: fold 35.9 us at
// 1024 threads, profiles/r04h prof_frames).
__global__ void __launch_bounds__(kFoldThreads) big_combine_aligned_kernel(const uint8_t *base, const uint64_t *offsets,
                                                                   const uint32_t *lengths, BigRoute r,
                                                                   const uint4 *shift_nib, uint32_t *out) {
  __shared__ __attribute__((aligned(16))) uint32_t nib[kShiftNibWords];
  __shared__ __attribute__((aligned(16))) uint32_t T4[1024]; // span mode: slice-by-4 tables (r.tab4)
  __shared__ uint32_t part[kFoldWaves], praw[2];
  const uint64_t nb = big_count(r);
  if (blockIdx.x >= nb) return;
  const uint32_t t = threadIdx.x, lane = t & 63u, w = t >> 6;
  const bool span = r.span_rows_max != 0 && r.meta[5] != 0; // (span mode: chunk = 4096)
  const uint64_t chunk = r.meta[3];
  const uint32_t lc = (uint32_t)__builtin_ctzll(chunk);
  {
    uint4 *dst = reinterpret_cast<uint4 *>(nib);
#pragma unroll
    for (uint32_t q = 0; q < kShiftNibWords / 4 / kFoldThreads; ++q)
      dst[q * kFoldThreads + t] = shift_nib[q * kFoldThreads + t];
    if (span) reinterpret_cast<uint4 *>(T4)[t] = r.tab4[t];
  }
  __syncthreads();
  auto apply = [&](uint64_t nbytes, uint32_t v) { // A_nbytes(v): one map per set bit
    for (; nbytes; nbytes &= nbytes - 1) v = nib_map(nib + 128u * (uint32_t)__builtin_ctzll(nbytes), v);
    return v;
  };
  const uint32_t *stepnib = nib + 128u * (lc + kFoldLog2); // A_{kFoldThreads C}
  const uint64_t b0 = (uint64_t)(uintptr_t)base;
  for (uint64_t b = blockIdx.x; span && b < nb; b += gridDim.x) { // span mode (block-uniform)
    const uint32_t i = (uint32_t)b; // route-all: body b
    const uint64_t s = offsets[i], L = lengths[i], e = s + L;
    const uint64_t j0 = s >> 12, j1 = L ? (e - 1) >> 12 : j0, nch = L ? j1 - j0 + 1 : 0;
    const uint64_t h_end = nch == 1 ? e : (j0 + 1) << 12;
    // waves 0 / 1: the first / last partial block, while the others fold the
    // interior blocks (G' below leaves chunk 0, the head, to thread 0 at the end)
    if (w < 2u) {
      uint32_t v = 0;
      if (w == 0u && nch != 0) v = span_piece_wave(base, s, h_end, lane, T4, nib);
      if (w == 1u && nch > 1) v = span_piece_wave(base, j1 << 12, e, lane, T4, nib);
      if (lane == 0) praw[w] = v;
    }
    const uint64_t m = nch ? nch - 1 : 0; // chunks folded into G: the head, then blocks j0 + 1 ..
    uint32_t acc = 0;
    constexpr uint32_t kB = kFoldBatch;
    // G' = crc0 of the interior blocks [ja, jb) (jb = j1), shifted to jb.  With
    // round values: the whole rounds [ra, rb) from rnd[], the <= 31 blocks before
    // them (wave 2) and after them (wave 3) from blk[], each shifted to jb.
    const uint64_t ja = j0 + 1, jb = j1, ra = (ja + 31) >> 5, rb = jb >> 5;
    if (r.rnd != nullptr && m > 1 && ra < rb) {
      const uint64_t nA = (ra << 5) - ja, nR = rb - ra, nC = jb - (rb << 5);
      const uint32_t *rstep = nib + 128u * (17u + kFoldLog2); // A_{T * 128 KiB}
      for (uint64_t k0 = t; k0 < nR; k0 += (uint64_t)kB * kFoldThreads) {
        uint32_t rv[kB];
#pragma unroll
        for (uint32_t q = 0; q < kB; ++q) {
          const uint64_t k = k0 + q * kFoldThreads;
          rv[q] = (k < nR) ? r.rnd[ra + k] : 0u;
        }
#pragma unroll
        for (uint32_t q = 0; q < kB; ++q)
          if (k0 + q * kFoldThreads < nR) acc = nib_map(rstep, acc) ^ rv[q];
      }
      if (t < nR) // from this thread's last round to the end of the rounds, then past C
        acc = apply((((nR - 1 - t) % kFoldThreads) << 17) + (nC << 12), acc);
      const uint32_t u = t & 63u;
      if (w == 2u && u < nA) acc ^= apply((jb - 1 - (ja + u)) << 12, r.blk[ja + u]);
      if (w == 3u && u < nC) acc ^= apply((nC - 1 - u) << 12, r.blk[(rb << 5) + u]);
    } else {
      for (uint64_t k0 = t; k0 < m; k0 += (uint64_t)kB * kFoldThreads) {
        uint32_t rv[kB];
#pragma unroll
        for (uint32_t q = 0; q < kB; ++q) {
          const uint64_t k = k0 + q * kFoldThreads;
          rv[q] = (k != 0 && k < m) ? r.blk[j0 + k] : 0u;
        }
#pragma unroll
        for (uint32_t q = 0; q < kB; ++q)
          if (k0 + q * kFoldThreads < m) acc = nib_map(stepnib, acc) ^ rv[q];
      }
      if (t < m) {
        for (uint32_t j = (uint32_t)((m - 1 - t) % kFoldThreads); j; j &= j - 1)
          acc = nib_map(nib + 128u * (lc + (uint32_t)__builtin_ctz(j)), acc);
      }
    }
    for (int d = 1; d < 64; d <<= 1) acc ^= (uint32_t)__shfl_xor((int)acc, d, 64);
    if (lane == 0) part[w] = acc;
    __syncthreads();
    if (t == 0) {
      for (uint32_t k = 1; k < kFoldWaves; ++k) acc ^= part[k];
      // zlib's pre-conditioning enters with the head: A_{len0}(F)
      const uint64_t len0 = h_end - s;
      const uint32_t head = praw[0] ^ apply(len0 & ~4095ull, r.tq[len0 & 4095u]);
      uint32_t crc = 0;
      if (nch == 1) {
        crc = ~head;
      } else if (nch > 1) {
        const uint32_t g = acc ^ apply((m - 1) << 12, head); // + the head, m - 1 chunks before the last of G
        crc = ~(apply(e - (j1 << 12), g) ^ praw[1]);
      }
      out[i] = crc; // an empty body: crc32 = 0
      if (r.cmp_verdict) fold_verdict(r, i, crc);
      if (r.stamp.frame_off) frames_stamp_one(r.stamp, i, crc);
    }
    __syncthreads();
  }
  for (uint64_t b = blockIdx.x; !span && b < nb; b += gridDim.x) {
    const uint32_t i = big_body(r, b);
    const uint64_t s = b0 + offsets[i], L = lengths[i], first = r.b_first[b], nch = r.b_first[b + 1] - first;
    const uint64_t e = s + L;
    // zlib's pre-conditioning, carried in by chunk 0 (thread 0): A_{len0}(F)
    uint32_t seed = 0;
    if (t == 0 && nch != 0) {
      const uint64_t end0 = (s & ~(chunk - 1)) + chunk;
      const uint64_t len0 = (end0 < e ? end0 : e) - s;
      seed = apply(len0 & ~4095ull, r.tq[len0 & 4095u]); // A_{4096 q} after Tq[len0 mod 4096]
    }
    const uint64_t m = nch ? nch - 1 : 0; // chunks folded into G
    uint32_t acc = 0;
    constexpr uint32_t kB = kFoldBatch;
    for (uint64_t k0 = t; k0 < m; k0 += (uint64_t)kB * kFoldThreads) {
      uint32_t rv[kB];
#pragma unroll
      for (uint32_t q = 0; q < kB; ++q) rv[q] = (k0 + q * kFoldThreads < m) ? r.c_raw[first + k0 + q * kFoldThreads] : 0u;
#pragma unroll
      for (uint32_t q = 0; q < kB; ++q)
        if (k0 + q * kFoldThreads < m) acc = nib_map(stepnib, acc) ^ rv[q] ^ (k0 + q == 0 ? seed : 0u);
    }
    if (t < m) { // chunks between this thread's last one and chunk m - 1
      for (uint32_t j = (uint32_t)((m - 1 - t) % kFoldThreads); j; j &= j - 1)
        acc = nib_map(nib + 128u * (lc + (uint32_t)__builtin_ctz(j)), acc);
    }
    for (int d = 1; d < 64; d <<= 1) acc ^= (uint32_t)__shfl_xor((int)acc, d, 64);
    if ((t & 63u) == 0) part[t >> 6] = acc;
    __syncthreads();
    if (t == 0) {
      for (uint32_t w = 1; w < kFoldWaves; ++w) acc ^= part[w];
      uint32_t crc = 0;
      if (nch == 1) {
        crc = ~(r.c_raw[first] ^ seed);
      } else if (nch > 1) {
        const uint64_t last_lo = (e - 1) & ~(chunk - 1);
        crc = ~(apply(e - last_lo, acc) ^ r.c_raw[first + nch - 1]);
      }
      out[i] = crc; // an empty body: crc32 = 0
      if (r.cmp_verdict) fold_verdict(r, i, crc);
      if (r.stamp.frame_off) frames_stamp_one(r.stamp, i, crc);
    }
    __syncthreads();
  }
}

} // namespace

size_t big_route_workspace_bytes(uint64_t n, uint64_t span_rows) {
  return align256((n + 63) / 64 * 8) + align256(64) + align256(kBigMaxBodies * 4) +
         align256((kBigMaxBodies + 1) * 8) + align256(kBigMaxChunks * 8) + 2 * align256(kBigMaxChunks * 4) +
         (span_rows ? align256((span_rows + 1) * 4) + align256((span_rows / 32 + 1) * 4) : 0);
}

BigRoute big_route_carve(void *ws, uint64_t n, uint64_t span_rows) {
  uint8_t *w = static_cast<uint8_t *>(ws);
  auto take = [&](size_t bytes) {
    uint8_t *p = w;
    w += align256(bytes);
    return p;
  };
  BigRoute r;
  r.routed = reinterpret_cast<uint32_t *>(take((n + 63) / 64 * 8));
  r.meta = reinterpret_cast<uint64_t *>(take(64));
  r.b_idx = reinterpret_cast<uint32_t *>(take(kBigMaxBodies * 4));
  r.b_first = reinterpret_cast<uint64_t *>(take((kBigMaxBodies + 1) * 8));
  r.c_off = reinterpret_cast<uint64_t *>(take(kBigMaxChunks * 8));
  r.c_len = reinterpret_cast<uint32_t *>(take(kBigMaxChunks * 4));
  r.c_raw = reinterpret_cast<uint32_t *>(take(kBigMaxChunks * 4));
  if (span_rows) {
    r.blk = reinterpret_cast<uint32_t *>(take((span_rows + 1) * 4)); // (+1: the fold's idle loads read blk[j0])
    r.rnd = reinterpret_cast<uint32_t *>(take((span_rows / 32 + 1) * 4)); // (the host clears it when unused)
    r.span_rows_max = span_rows;
  }
  return r;
}

hipError_t launch_big_classify(const uint32_t *lengths, uint64_t n, uint32_t big_min, const BigRoute &r,
                               hipStream_t s) {
  if (n == 0) return hipSuccess;
  if (n > kMaxLaunchItems) return hipErrorInvalidValue;
  hipError_t e = hipMemsetAsync(r.meta, 0, 32, s);
  if (e != hipSuccess) return e;
  hipLaunchKernelGGL(big_classify_kernel, dim3((unsigned)((n + 255) / 256)), dim3(256), 0, s, lengths, n, big_min, r);
  return hipGetLastError();
}

hipError_t launch_big_route(const ItemsArgs &proto, const BigRoute &r, const uint4 *shift_nib, bool nt, int max_blocks,
                            hipStream_t s, uint32_t *steal, hipEvent_t steal_done, bool *steal_recorded,
                            StealArgs span) {
  if (proto.n_items == 0) return hipSuccess;
  if (proto.mode != kModeFinal || proto.offsets == nullptr || proto.lengths == nullptr || !r.tq) return hipErrorInvalidValue;
  // span mode: route-all over a 4 KiB-aligned base, aligned chunks, a block table
  if (r.span_rows_max != 0 && (!r.all_n || !r.aligned || !r.blk || !r.tab4 || ((uintptr_t)proto.base & 4095u) != 0 ||
                               r.span_rows_max > kSpanMaxRows))
    return hipErrorInvalidValue;
  hipError_t e;
  if (r.aligned) {
    // address-aligned power-of-two chunks (>= 4 KiB; the fold's step map is
    // A_{1024 C}, so C <= 2^53)
    if (r.min_chunk < 4096 || (r.min_chunk & (r.min_chunk - 1)) != 0 || r.min_chunk > (1ull << 40))
      return hipErrorInvalidValue;
    hipLaunchKernelGGL(big_plan_aligned_kernel, dim3(1), dim3(1024), 0, s, proto.base, proto.offsets, proto.lengths, r);
    e = hipGetLastError();
    if (e != hipSuccess) return e;
    hipLaunchKernelGGL(big_expand_aligned_kernel, dim3(128), dim3(256), 0, s, proto.base, proto.offsets, proto.lengths,
                       r);
  } else {
    // The fold indexes its maps by chunk class: chunk = 4096 * 2^m - 16 (the plan
    // only doubles it), m < kBigChunkClasses; r.dbl must be set.
    const uint64_t p = r.min_chunk + 16;
    if (p < 4096 || (p & (p - 1)) != 0 || (p >> 12) >= (1ull << kBigChunkClasses) || !r.dbl)
      return hipErrorInvalidValue;
    hipLaunchKernelGGL(big_plan_kernel, dim3(1), dim3(1024), 0, s, proto.lengths, r);
    e = hipGetLastError();
    if (e != hipSuccess) return e;
    hipLaunchKernelGGL(big_expand_kernel, dim3(512), dim3(256), 0, s, proto.offsets, proto.lengths, r);
  }
  e = hipGetLastError();
  if (e != hipSuccess) return e;
  ItemsArgs a = proto; // the chunks: rows kernel, RAW, count on the device
  a.offsets = r.c_off;
  a.lengths = r.c_len;
  a.n_items = kBigMaxChunks;
  a.n_dev = r.meta + 2;
  a.out_idx = nullptr;
  a.routed = nullptr;
  a.big_min = 0xFFFFFFFFu;
  a.mode = kModeRaw;
  a.out = r.c_raw;
  // The tail is dealt from the steal counter, the pool sized in the kernel
  // from the device count (crc32_rows.h steal_s).
  a.steal = steal;
  e = launch_rows(a, 1, nt, max_blocks, s, steal_done, steal_recorded);
  if (e != hipSuccess) return e;
  if (r.span_rows_max != 0) {
    // the span pass: every whole 4 KiB block below the last body end, uniform
    // rows (RAW), count on the device (0 unless the plan chose span mode)
    ItemsArgs u = proto;
    u.offsets = nullptr;
    u.lengths = nullptr;
    u.n_items = r.span_rows_max;
    u.stride = 4096;
    u.len = 4096;
    u.n_dev = r.meta + 4;
    u.out_idx = nullptr;
    u.routed = nullptr;
    u.big_min = 0xFFFFFFFFu;
    u.mode = kModeRaw;
    u.out = r.blk;
    if (r.rnd != nullptr) { // round values (crc32_rows.h kRowsRoundOut)
      if (!r.rnd_image || r.span_rows_max < 256ull * (uint64_t)max_blocks) return hipErrorInvalidValue;
      u.round_out = r.rnd;
      u.lds_image = r.rnd_image;
    }
    u.steal = span.p;
    e = launch_rows(u, 1, nt, max_blocks, s, span.done, span.recorded);
    if (e != hipSuccess) return e;
  }
  // 1024 blocks (blocks past the routed-body count leave at once): a block folds
  // one body at a time, so the count bounds the serial bodies per block.
  if (r.aligned)
    hipLaunchKernelGGL(big_combine_aligned_kernel, dim3(2048), dim3(kFoldThreads), 0, s, proto.base, proto.offsets,
                       proto.lengths, r, shift_nib, proto.out);
  else
    hipLaunchKernelGGL(big_combine_kernel, dim3(1024), dim3(1024), 0, s, proto.lengths, r, shift_nib, proto.out);
  return hipGetLastError();
}

hipError_t launch_splitmix_fill(void *dst, uint64_t nbytes, uint64_t seed, hipStream_t stream) {
  if (nbytes == 0) return hipSuccess;
  if (nbytes % 8 != 0) return hipErrorInvalidValue;
  const uint64_t nwords = nbytes / 8;
  uint64_t blocks = (nwords / 2 + 255) / 256;
  if (blocks > 65536) blocks = 65536;
  if (blocks == 0) blocks = 1;
  hipLaunchKernelGGL(splitmix_fill_kernel, dim3((unsigned)blocks), dim3(256), 0, stream,
                     reinterpret_cast<uint64_t *>(dst), nwords, seed, (uint64_t)0);
  return hipGetLastError();
}

// Stream-read probe with the rows kernel's own memory stream (pattern 2): the
// product kernel (uniform 4 KiB rows, DYN rounds + tail stealing, 4 x 16 B NT
// buffer loads per lane issued a row ahead, one exit at the bottom) with every
// CRC instruction compiled out -- no LDS image, no transpose, no chain, no
// merge, no stores.  This is the ceiling the product's dealing and load shape
// can reach on the buffer; the plain grid-stride probe above has no tail
// dealing, and the product beat it.
constexpr int kStreamRowsAbl = kRowsAblNoCompute | kRowsAblNoMerge | kRowsAblNoTranspose | kRowsAblNoStore |
                               kRowsAblNoImage;
hipError_t launch_stream_rows(const ItemsArgs &a, int max_blocks, hipStream_t stream, hipEvent_t steal_done,
                              bool *steal_recorded) {
  if (a.n_items == 0) return hipSuccess;
  if (a.offsets != nullptr || a.len != 4096 || a.stride != 4096 || a.n_items > kMaxLaunchItems || a.out == nullptr)
    return hipErrorInvalidValue;
  uint64_t blocks = (a.n_items + 15) / 16;
  if (blocks > (uint64_t)max_blocks) blocks = (uint64_t)max_blocks;
  const uint64_t round = dyn_round(1);
  if (a.n_items < 8ull * round * blocks || a.steal == nullptr) return hipErrorInvalidValue; // DYN + stealing only
  ItemsArgs k = a;
  const uint64_t rounds = (a.n_items + round - 1) / round;
  const uint64_t st = (uint64_t)((double)rounds * (1.0 - steal_frac())) / blocks;
  if (!(st >= kStealAhead && st * blocks < rounds)) return hipErrorInvalidValue;
  k.steal_s = (uint32_t)st;
  const dim3 grid((unsigned)blocks), block(1024);
  if (steal_done) {
    hipExtLaunchKernelGGL((crc32_rows_kernel<1, true, false, kStreamRowsAbl, 1, true, true>), grid, block, 0, stream,
                          nullptr, steal_done, 0, k);
    if (steal_recorded) *steal_recorded = true;
  } else {
    hipLaunchKernelGGL((crc32_rows_kernel<1, true, false, kStreamRowsAbl, 1, true, true>), grid, block, 0, stream, k);
  }
  return hipGetLastError();
}

hipError_t launch_stream_read(const void *p, uint64_t nbytes, int pattern, bool nt, int max_blocks, uint32_t *out,
                              hipStream_t stream) {
  const uint64_t ntiles = nbytes / 4096;
  if (ntiles == 0) return hipSuccess;
  const dim3 grid((unsigned)max_blocks), block(kBlock);
  const uint4 *q = reinterpret_cast<const uint4 *>(p);
  if (pattern == 0) {
    if (nt)
      hipLaunchKernelGGL((stream_read_kernel<0, true>), grid, block, 0, stream, q, ntiles, out);
    else
      hipLaunchKernelGGL((stream_read_kernel<0, false>), grid, block, 0, stream, q, ntiles, out);
  } else {
    if (nt)
      hipLaunchKernelGGL((stream_read_kernel<1, true>), grid, block, 0, stream, q, ntiles, out);
    else
      hipLaunchKernelGGL((stream_read_kernel<1, false>), grid, block, 0, stream, q, ntiles, out);
  }
  return hipGetLastError();
}

// ---- dense span mode (tests/test_dense_emu.py restates it) ----

size_t dense_workspace_bytes(uint64_t n, uint64_t nb_cap) {
  return align256(sizeof(DenseCtl)) + align256(nb_cap * 16) + align256((n + 1) * 2) + align256((n + 1) * 8) +
         align256(nb_cap * 4) + align256(dense_plan_blocks(n) * 4);
}

DenseArgs dense_carve(void *ws, uint64_t n, uint64_t nb_cap) {
  uint8_t *w = static_cast<uint8_t *>(ws);
  auto take = [&](size_t bytes) {
    uint8_t *p = w;
    w += align256(bytes);
    return p;
  };
  DenseArgs d{};
  d.n = n;
  d.nb_cap = nb_cap;
  d.ctl = reinterpret_cast<DenseCtl *>(take(sizeof(DenseCtl)));
  d.rec = reinterpret_cast<uint4 *>(take(nb_cap * 16));
  d.bpos = reinterpret_cast<uint16_t *>(take((n + 1) * 2));
  d.bnd = reinterpret_cast<uint2 *>(take((n + 1) * 8));
  d.W = reinterpret_cast<uint32_t *>(take(nb_cap * 4));
  d.flags = reinterpret_cast<uint32_t *>(take(dense_plan_blocks(n) * 4));
  return d;
}

namespace {

__device__ __forceinline__ uint64_t shfl64(uint64_t v, int src) {
  const uint32_t lo = (uint32_t)__shfl((int)(uint32_t)v, src, 64), hi = (uint32_t)__shfl((int)(uint32_t)(v >> 32), src, 64);
  return ((uint64_t)hi << 32) | lo;
}
__device__ __forceinline__ uint64_t ballot64(bool p) { return (uint64_t)__builtin_amdgcn_ballot_w64(p); }
// Lane-to-lane words through LDS inside one wave: atomic (relaxed, wavefront
// scope) stores and loads with a wave barrier between the phases.  Plain ones
// are a data race to the compiler: it forwarded a lane's own earlier store to
// its load where the other lanes' stores were to reach it (owner marks read as
// 0: wrong dense CRCs, found by tests/test_gpu_parity.py test_dense_span_mode).
__device__ __forceinline__ void lane_st(uint32_t *p, uint32_t v) {
  __hip_atomic_store(p, v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WAVEFRONT);
}
__device__ __forceinline__ uint32_t lane_ld(uint32_t *p) {
  return __hip_atomic_load(p, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WAVEFRONT);
}

// Inclusive wave scans on the VALU: row_shr 1, 2, 4, 8 (DPP) inside each
// 16-lane row, then the row totals (lanes 15, 31, 47) read as scalars and
// added to the rows after them (gfx950 has no DPP row_bcast 15 / 31: the
// first version of this scan used them and came out wrong).  A ds_bpermute
// per step cost LDS issue slots the fold's lookups need.
template <bool MAX>
__device__ __forceinline__ uint32_t wave_incl_scan(uint32_t v) {
  auto op = [](uint32_t a, uint32_t b) { return MAX ? max(a, b) : a + b; };
  v = op(v, (uint32_t)__builtin_amdgcn_mov_dpp((int)v, 0x111, 0xF, 0xF, true)); // row_shr:1 (zeros shifted in)
  v = op(v, (uint32_t)__builtin_amdgcn_mov_dpp((int)v, 0x112, 0xF, 0xF, true)); // row_shr:2 (zeros shifted in)
  v = op(v, (uint32_t)__builtin_amdgcn_mov_dpp((int)v, 0x114, 0xF, 0xF, true)); // row_shr:4 (zeros shifted in)
  v = op(v, (uint32_t)__builtin_amdgcn_mov_dpp((int)v, 0x118, 0xF, 0xF, true)); // row_shr:8 (zeros shifted in)
  const uint32_t r0 = (uint32_t)__builtin_amdgcn_readlane((int)v, 15);
  const uint32_t r1 = op(r0, (uint32_t)__builtin_amdgcn_readlane((int)v, 31));
  const uint32_t r2 = op(r1, (uint32_t)__builtin_amdgcn_readlane((int)v, 47));
  const uint32_t row = (threadIdx.x & 63u) >> 4;
  const uint32_t add = row == 0u ? 0u : (row == 1u ? r0 : (row == 2u ? r1 : r2));
  return row == 0u ? v : op(v, add);
}

// Decides whether the batch is dense -- every body kDenseMinBody ..
// kDenseMaxBody bytes and starting where the previous one ends -- and writes
// the span pass's inputs: per boundary its block offset (bpos), per block its
// record (first boundary, count, the first kDenseInline offsets; a block
// without a boundary: count 0).  One wave per window of 64 boundaries g0 ..
// g0 + 63 (lane L: boundary g0 + L), all its loads issued at once (loads under
// per-lane branches had each waited out its own round trip: 190 us for C2);
// it looks at the next window too (a block holds at most 64 boundaries, so a
// run that starts in the window ends before the next window's end).  The
// first boundary of each block writes its record, and the records of the
// empty blocks before it (inside the previous body) are dealt over the wave's
// lanes.  Each workgroup stores whether it found the batch not dense
// (dense_decide_kernel reads them).
__global__ __launch_bounds__(256) void dense_plan_kernel(DenseArgs d) {
  __shared__ uint32_t s_own[4 * 64];
  const uint64_t n = d.n;
  const uint64_t base = (uint64_t)(uintptr_t)d.base;
  const uint64_t anchor = (base + d.offsets[0]) & ~(uint64_t)15;
  const uint64_t rel_n = base + d.offsets[n - 1] + d.lengths[n - 1] - anchor;
  const uint64_t nblocks = (rel_n + 4095u) >> 12;
  constexpr uint64_t kNone = ~(uint64_t)0; // past boundary n: a block of its own
  bool bad = nblocks > d.nb_cap || nblocks > kDenseMaxBlocks;
  // records are written below rec_lim only: the array holds nb_cap of them, and
  // a batch the plan refuses (a longer stream than the bound allowed, or bodies
  // before the first one: offsets that wrap below the anchor) must not write
  // past it -- its records are never read
  const uint64_t rec_lim = min(nblocks, (uint64_t)d.nb_cap);
  const uint32_t lane = threadIdx.x & 63u;
  const uint64_t w = (uint64_t)blockIdx.x * (blockDim.x / 64u) + (threadIdx.x >> 6);
  const uint64_t g0 = 64u * w, g = g0 + lane;
  if (g0 <= n) { // (wave-uniform)
    // every load at once, indices clamped; selects after
    const uint64_t oa = d.offsets[min(g, n - 1)], ob = d.offsets[min(g + 64u, n - 1)];
    const uint32_t L = d.lengths[min(g, n - 1)];
    const uint64_t op = d.offsets[g0 == 0 ? 0 : g0 - 1]; // (lane 0's previous boundary)
    const bool va = g <= n;
    const uint64_t ra = g < n ? base + oa - anchor : (g == n ? rel_n : kNone);
    const uint64_t rb = g + 64u < n ? base + ob - anchor : (g + 64u == n ? rel_n : kNone); // the next window
    uint64_t rp = shfl64(ra, (int)((lane + 63u) & 63u)); // the previous boundary
    if (lane == 0u) rp = g0 == 0 ? 0u : base + op - anchor;
    const uint64_t rn_b = shfl64(rb, 0);
    uint64_t rn = shfl64(ra, (int)((lane + 1u) & 63u)); // the next boundary
    if (lane == 63u) rn = rn_b;
    if (g < n && (L < kDenseMinBody || L > kDenseMaxBody || rn - ra != L)) bad = true;
    if (va) d.bpos[g] = (uint16_t)(ra & 4095u);
    const uint64_t ja = ra >> 12, jp = rp >> 12, jb = rb >> 12;
    const bool first = g == 0 || ja != jp; // (the first lane past boundary n counts as one: it ends the run)
    if (va && g != 0 && ja != jp && (ja < jp || ja - jp > (kDenseMaxBody >> 12) + 2)) bad = true; // out of order
    // boundaries of this lane's block from this lane on: to the next first lane,
    // else through lane 63 and on into the next window
    const uint64_t F = ballot64(first);
    const uint64_t ja63 = shfl64(ja, 63);
    const uint64_t B = ballot64(jb != ja63);
    const uint64_t after = lane == 63u ? 0u : F >> (lane + 1u);
    const uint32_t cnt = after ? (uint32_t)__builtin_ctzll(after) + 1u
                               : 64u - lane + (B ? (uint32_t)__builtin_ctzll(B) : 64u);
    if (va && first && cnt > 64u) bad = true; // (bodies under 64 B: caught above as well)
    uint32_t o[kDenseInline];
#pragma unroll
    for (uint32_t i = 0; i < kDenseInline; ++i) {
      const uint32_t src = lane + i;
      const uint32_t qa = (uint32_t)__shfl((int)(uint32_t)(ra & 4095u), (int)(src & 63u), 64);
      const uint32_t qb = (uint32_t)__shfl((int)(uint32_t)(rb & 4095u), (int)(src & 63u), 64);
      o[i] = i < cnt ? (src < 64u ? qa : qb) : 0u;
    }
    if (va && first && ja < rec_lim)
      d.rec[ja] = make_uint4((uint32_t)g | (min(cnt, 64u) << 25), o[0] | (o[1] << 16), o[2] | (o[3] << 16),
                             o[4] | (o[5] << 16));
    // empty blocks (jp, ja) before a first boundary: k records, dealt over the wave
    uint32_t k = 0;
    if (va && first && g != 0 && ja > jp + 1u && ja - jp <= (kDenseMaxBody >> 12) + 2)
      k = (uint32_t)(min(ja, rec_lim) > jp + 1u ? min(ja, rec_lim) - jp - 1u : 0u);
    const uint32_t incl = wave_incl_scan<false>(k);
    const uint32_t K = (uint32_t)__builtin_amdgcn_readlane((int)incl, 63);
    // the first pass's owners by marks and a max-scan (fold kernel), later
    // passes by a search
    uint32_t *own_mark = s_own + (threadIdx.x >> 6) * 64u;
    lane_st(&own_mark[lane], 0u);
    __builtin_amdgcn_wave_barrier();
    if (k != 0u && incl - k < 64u) lane_st(&own_mark[incl - k], lane);
    __builtin_amdgcn_wave_barrier();
    const uint32_t own0 = wave_incl_scan<true>(lane_ld(&own_mark[lane]));
    __builtin_amdgcn_wave_barrier();
    for (uint32_t q0 = 0; q0 < K; q0 += 64u) {
      const uint32_t q = q0 + lane;
      uint32_t own = own0;
      if (q0 != 0u) { // (the first lane whose inclusive sum passes q)
        own = 0;
#pragma unroll
        for (uint32_t step = 32; step; step >>= 1) {
          const uint32_t v = (uint32_t)__shfl((int)incl, (int)(own + step - 1u), 64);
          if (v <= q) own += step;
        }
        own = min(own, 63u);
      }
      const uint64_t jp_o = shfl64(jp, (int)own);
      const uint32_t ex_o = (uint32_t)__shfl((int)(incl - k), (int)own, 64);
      const uint64_t j = jp_o + 1u + (q - ex_o);
      if (q < K && j < rec_lim) d.rec[j] = make_uint4((uint32_t)(g0 + own), 0u, 0u, 0u);
    }
  }
  const int any_bad = __syncthreads_or(bad ? 1 : 0);
  if (threadIdx.x == 0) d.flags[blockIdx.x] = any_bad ? 1u : 0u; // (every word written: no clearing)
}

// One workgroup: ORs the plan's per-workgroup flags and writes DenseCtl
// (nblocks = 0 unless dense).  (The plan's workgroups had each counted
// themselves done on one device atomic, 16K of them: 1.4 ms.)
__global__ __launch_bounds__(1024) void dense_decide_kernel(DenseArgs d, uint32_t plan_blocks) {
  uint32_t bad = 0;
  for (uint32_t i = threadIdx.x; i < plan_blocks; i += 1024u) bad |= d.flags[i];
  bad = __syncthreads_or((int)bad);
  if (threadIdx.x == 0) {
    const uint64_t n = d.n;
    const uint64_t base = (uint64_t)(uintptr_t)d.base;
    const uint64_t anchor = (base + d.offsets[0]) & ~(uint64_t)15;
    const uint64_t rel_n = base + d.offsets[n - 1] + d.lengths[n - 1] - anchor;
    const uint64_t nblocks = (rel_n + 4095u) >> 12;
    const bool dense = bad == 0u && nblocks <= d.nb_cap && nblocks <= kDenseMaxBlocks && n >= 1 && n <= kDenseMaxN;
    d.ctl->anchor = anchor;
    d.ctl->bytes = rel_n;
    d.ctl->nblocks = dense ? nblocks : 0u;
    d.ctl->skip = dense ? 1u : 0u;
  }
}

// Nibble map `map` of x from the LDS copy of the maps (crc32_layout.h
// kDenseTabWords: word (n * 16 + nib) * kDenseMaps + map).
__device__ __forceinline__ uint32_t dense_map(const uint32_t *t, uint32_t map, uint32_t x) {
  uint32_t v[8];
#pragma unroll
  for (uint32_t k = 0; k < 8; ++k) v[k] = t[(k * 16u + ((x >> (4u * k)) & 15u)) * kDenseMaps + map];
  // three-way XORs (v_bitop3_b32): 4 VALU for the 8 lookups instead of 7
  auto x3 = [](uint32_t a, uint32_t b, uint32_t c) { return __builtin_amdgcn_bitop3_b32(a, b, c, 0x96); };
  return x3(x3(v[0], v[1], v[2]), x3(v[3], v[4], v[5]), v[6] ^ v[7]);
}

// Per boundary g: E = crc0(its block with the bytes from g on zeroed)
//   = A_{1024(3-hi)}(bnd.x) ^ bnd.y  (the span pass stored the quarter part).
// Per body g over blocks j .. j1 (D = j1 - j):
//   j1 = j:  Y = Tq[4096 - off] ^ E(g) ^ E_end
//   j1 > j:  Y = A_{4096 D}(Tq[4096 - off] ^ W[j] ^ E(g)) ^ X ^ E_end,
//            X = XOR over the blocks i in between of A_{4096 (j1 - i)}(W[i])
// with E_end = E(g + 1), or W[j1] when the body ends its block; then
// crc = ~A_{-z}(Y), z = 4096 - e_off (the bytes of j1 after the body).  A wave
// takes boundaries 63 w .. 63 w + 63 and bodies 63 w .. 63 w + 62 (body g's
// end boundary is lane g + 1's); the in-between blocks of its bodies are dealt
// over its lanes (one block each per pass, XORed into an LDS word per body),
// so a long body does not hold the wave for a Horner step per block.
__global__ __launch_bounds__(1024) void dense_fold_kernel(DenseArgs d) {
  __shared__ uint32_t s_tab[kDenseTabWords];
  __shared__ uint32_t s_x[16 * 64];
  __shared__ uint32_t s_own[16 * 64];
  if (d.ctl->nblocks == 0u) return; // (block-uniform) not dense: the rows pass did it
  for (uint32_t i = threadIdx.x; i < kDenseTabWords; i += 1024u) s_tab[i] = d.tab[i];
  __syncthreads();
  const uint32_t lane = threadIdx.x & 63u, wave = threadIdx.x >> 6;
  uint32_t *x_acc = s_x + wave * 64u;
  const uint64_t n = d.n, nw = (n + 62) / 63, last_w = d.nb_cap - 1;
  const uint64_t base = (uint64_t)(uintptr_t)d.base, anchor = d.ctl->anchor, rel_n = d.ctl->bytes;
  // round trip 1 of a window: boundary g's offset and values, body g's length
  // (every index clamped, no load under a branch); issued a window ahead, so
  // it overlaps the current window's second round trip
  const uint64_t wstep = (uint64_t)gridDim.x * 16u;
  uint64_t w = (uint64_t)blockIdx.x * 16u + wave;
  uint64_t nx_o = 0;
  uint32_t nx_L = 0;
  uint2 nx_b = make_uint2(0u, 0u);
  auto fetch = [&](uint64_t ww) {
    const uint64_t gg = 63u * min(ww, nw - 1) + lane;
    nx_o = d.offsets[min(gg, n - 1)];
    nx_L = d.lengths[min(gg, n - 1)];
    nx_b = d.bnd[min(gg, n)];
  };
  if (w < nw) fetch(w);
  for (; w < nw; w += wstep) {
    const uint64_t g = 63u * w + lane;
    const uint64_t o = nx_o;
    const uint32_t L = nx_L;
    const uint2 b = nx_b;
    fetch(w + wstep); // (clamped: the last window again at the end)
    const bool body = lane < 63u && g < n;
    const uint64_t rs = g < n ? base + o - anchor : rel_n; // stream offset of boundary g
    const uint64_t j = rs >> 12;
    const uint32_t off = (uint32_t)(rs & 4095u);
    const uint64_t re = rs + L; // body g's end
    const uint64_t j1 = (re - 1) >> 12;
    const uint32_t e_off = (uint32_t)(re - j1 * 4096u); // 1 .. 4096
    // the blocks in between: m per body, dealt over the wave's lanes
    const uint32_t m = (body && j1 > j + 1u) ? (uint32_t)(j1 - j - 1u) : 0u;
    const uint32_t incl = wave_incl_scan<false>(m);
    const uint32_t K = (uint32_t)__builtin_amdgcn_readlane((int)incl, 63);
    // lane q's in-between block for pass q0: its body (owner), index and distance
    auto deal_from = [&](uint32_t q, uint32_t own, uint64_t &i, uint32_t &dist) {
      const uint32_t jo = (uint32_t)__shfl((int)(uint32_t)j, (int)own, 64); // (blocks < 2^24)
      const uint32_t j1o = (uint32_t)__shfl((int)(uint32_t)j1, (int)own, 64);
      const uint32_t exo = (uint32_t)__shfl((int)(incl - m), (int)own, 64);
      i = q < K ? (uint64_t)jo + 1u + (q - exo) : 0u;
      dist = q < K ? j1o - (uint32_t)i : 0u; // 1 .. 256
    };
    auto deal = [&](uint32_t q0, uint64_t &i, uint32_t &dist, uint32_t &own) { // (passes past the first)
      const uint32_t q = q0 + lane;
      own = 0; // the first lane whose inclusive sum passes q
#pragma unroll
      for (uint32_t step = 32; step; step >>= 1) {
        const uint32_t v = (uint32_t)__shfl((int)incl, (int)(own + step - 1u), 64);
        if (v <= q) own += step;
      }
      own = min(own, 63u);
      deal_from(q, own, i, dist);
    };
    // the first pass: each owner marks the slot of its first block, a max-scan
    // spreads the marks (an LDS store and load instead of a 6-step search)
    uint32_t *own_mark = s_own + wave * 64u;
    lane_st(&own_mark[lane], 0u);
    __builtin_amdgcn_wave_barrier();
    if (m != 0u && incl - m < 64u) lane_st(&own_mark[incl - m], lane);
    __builtin_amdgcn_wave_barrier();
    const uint32_t own0 = wave_incl_scan<true>(lane_ld(&own_mark[lane]));
    uint64_t i0;
    uint32_t dist0;
    deal_from(lane, own0, i0, dist0);
    // round trip 2: seed, first / last block CRCs, the first pass's blocks
    const uint32_t tqv = d.tq[4096u - off];
    const uint32_t wj = d.W[body ? min(j, last_w) : 0u];
    const uint32_t wj1 = d.W[body ? min(j1, last_w) : 0u];
    const uint32_t wi0 = d.W[min(i0, last_w)];
    lane_st(&x_acc[lane], 0u);
    __builtin_amdgcn_wave_barrier();
    const uint32_t hi = off >> 10;
    const uint32_t E = dense_map(s_tab, kDenseMQ + (3u - hi), b.x) ^ b.y;
    const uint32_t En = (uint32_t)__shfl_down((int)E, 1, 64);
    // (A_{65536 k} with k = 0 is the identity: its 8 lookups are skipped when no
    // lane of the wave needs k > 0 -- a block distance or body span of >= 16
    // blocks, i.e. a body over 60 KiB)
    if (lane < K) {
      uint32_t c = dense_map(s_tab, kDenseMB0 + (dist0 & 15u), wi0);
      if (ballot64(dist0 >= 16u) != 0u) c = dense_map(s_tab, kDenseMB1 + (dist0 >> 4), c);
      __hip_atomic_fetch_xor(&x_acc[own0], c, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WAVEFRONT);
    }
    for (uint32_t q0 = 64u; q0 < K; q0 += 64u) { // (long bodies)
      uint64_t i;
      uint32_t dist, own;
      deal(q0, i, dist, own);
      const uint32_t wi = d.W[min(i, last_w)];
      if (q0 + lane < K) {
        uint32_t c = dense_map(s_tab, kDenseMB0 + (dist & 15u), wi);
        if (ballot64(dist >= 16u) != 0u) c = dense_map(s_tab, kDenseMB1 + (dist >> 4), c);
        __hip_atomic_fetch_xor(&x_acc[own], c, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WAVEFRONT);
      }
    }
    __builtin_amdgcn_wave_barrier();
    const uint32_t X = lane_ld(&x_acc[lane]);
    if (body) {
      const uint32_t Ee = e_off == 4096u ? wj1 : En;
      uint32_t acc = tqv ^ E;
      if (j1 == j) {
        acc ^= Ee;
      } else {
        const uint32_t D = (uint32_t)(j1 - j); // 1 .. 257
        acc = dense_map(s_tab, kDenseMB0 + (D & 15u), acc ^ wj);
        if (ballot64(D >= 16u) != 0u) acc = dense_map(s_tab, kDenseMB1 + (D >> 4), acc);
        acc ^= X ^ Ee;
      }
      const uint32_t z = 4096u - e_off;
      acc = dense_map(s_tab, kDenseMI0 + (z & 15u), acc);
      acc = dense_map(s_tab, kDenseMI1 + ((z >> 4) & 15u), acc);
      acc = dense_map(s_tab, kDenseMI2 + (z >> 8), acc);
      d.out[g] = ~acc;
    }
  }
}

} // namespace

hipError_t launch_dense_plan(const DenseArgs &d, hipStream_t s) {
  if (d.n == 0 || d.n > kDenseMaxN || d.flags == nullptr) return hipErrorInvalidValue;
  const uint64_t blocks = dense_plan_blocks(d.n); // one wave per 64 boundaries
  hipLaunchKernelGGL(dense_plan_kernel, dim3((unsigned)blocks), dim3(256), 0, s, d);
  hipError_t e = hipGetLastError();
  if (e != hipSuccess) return e;
  hipLaunchKernelGGL(dense_decide_kernel, dim3(1), dim3(1024), 0, s, d, (uint32_t)blocks);
  return hipGetLastError();
}

hipError_t launch_dense_fold(const DenseArgs &d, int cus, hipStream_t s) {
  const uint64_t nw = (d.n + 62) / 63;
  const uint64_t blocks = std::max<uint64_t>(1, std::min<uint64_t>((nw + 15) / 16, 2ull * (uint64_t)std::max(cus, 1)));
  hipLaunchKernelGGL(dense_fold_kernel, dim3((unsigned)blocks), dim3(1024), 0, s, d);
  return hipGetLastError();
}

} // namespace rpccrc
