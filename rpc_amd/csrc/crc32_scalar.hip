// rpc_amd/csrc/crc32_scalar.hip -- one drop-in rpc_crc32 call (crc.h:8,
// crc.c:4-9) on a body of <= 4 KiB: the in-product RPC bodies (<= 1 KiB,
// rpc.h:17) and the captured 68-B request.  The rows kernel would spend a
// whole CU copying its 155 KiB LDS image to CRC one row; this kernel is ONE
// wave with a 9 KiB table.
//
// The body is right-aligned in a virtual buffer V of 64 * seg bytes (seg =
// bytes per lane, a power of two 4..64): lane L owns V[L*seg, +seg).  Bytes
// before the body count as zeros, and leading zeros leave a zero-initialised
// CRC unchanged, so crc0(V) = crc0(body).
//   load:   every lane reads its dwords straight from the caller's pinned
//           staging (host memory; the host copied the body to offset
//           64*seg - len) and masks the bytes before the body.  The table
//           image is read from HBM into LDS meanwhile.
//   chain:  seg/4 slice-by-4 steps per lane from LDS (one table copy; a
//           single wave, bank conflicts do not matter here).
//   merge:  six levels of pairs: A_{seg*2^b}(left) ^ right, the shift applied
//           by 8 nibble lookups, one lane exchange per level.
//   result: crc = ~(A_len(0xFFFFFFFF) ^ crc0(V)) (zlib pre/post conditioning,
//           the seed from the Tq table), stored by lane 0 as one 64-bit word
//           {crc, seq} to pinned host memory with system-scope release, so the
//           host can poll for it instead of synchronising the stream.
#include "crc32_kernels.h"
#include "crc32_layout.h"

namespace rpccrc {

namespace {

template <uint32_t SEG_LOG2>
__global__ __launch_bounds__(64) void crc32_scalar_kernel(const uint8_t *stage, uint32_t len, const uint4 *tab,
                                                           const uint32_t *tq, uint64_t *result, uint32_t seq) {
  constexpr uint32_t kSeg = 1u << SEG_LOG2;
  constexpr uint32_t kWords = kSeg / 4;
  constexpr uint32_t kTabPieces = kScalarTabWords / 4; // 16-B pieces
  static_assert(kTabPieces % 64 == 0, "whole pieces per lane");
  __shared__ uint4 lds4[kTabPieces];
  const uint32_t lane = threadIdx.x;

  uint4 t[kTabPieces / 64];
#pragma unroll
  for (uint32_t k = 0; k < kTabPieces / 64; ++k) t[k] = tab[lane + 64 * k];
  const uint32_t seed = tq[len];

  const uint32_t off0 = 64u * kSeg - len; // V offset of the body's first byte
  const uint32_t base = lane * kSeg;
  // Every lane loads (the staging is always readable; stale bytes before the
  // body are masked): no branch, so the data and table loads fly together.
  uint32_t w[kWords];
  const uint8_t *p = stage + base;
  if constexpr (kWords >= 4) {
#pragma unroll
    for (uint32_t q = 0; q < kWords / 4; ++q) {
      const uint4 v = reinterpret_cast<const uint4 *>(p)[q];
      w[4 * q] = v.x;
      w[4 * q + 1] = v.y;
      w[4 * q + 2] = v.z;
      w[4 * q + 3] = v.w;
    }
  } else if constexpr (kWords == 2) {
    const uint2 v = *reinterpret_cast<const uint2 *>(p);
    w[0] = v.x;
    w[1] = v.y;
  } else {
    w[0] = *reinterpret_cast<const uint32_t *>(p);
  }
#pragma unroll
  for (uint32_t d = 0; d < kWords; ++d) {
    const uint32_t pos = base + 4 * d;
    const uint32_t keep = pos >= off0 ? 0xFFFFFFFFu : (pos + 4 <= off0 ? 0u : 0xFFFFFFFFu << (8 * (off0 - pos)));
    w[d] &= keep;
  }

#pragma unroll
  for (uint32_t k = 0; k < kTabPieces / 64; ++k) lds4[lane + 64 * k] = t[k];
  __syncthreads();
  const uint32_t *T = reinterpret_cast<const uint32_t *>(lds4);

  // crc0 of the lane's segment: slice-by-4, T_k at T + 256 k (T_3 takes byte 0).
  uint32_t s = 0;
#pragma unroll
  for (uint32_t d = 0; d < kWords; ++d) {
    const uint32_t x = s ^ w[d];
    s = T[768 + (x & 0xFFu)] ^ T[512 + ((x >> 8) & 0xFFu)] ^ T[256 + ((x >> 16) & 0xFFu)] ^ T[x >> 24];
  }

  // Pair levels: groups of 2^b lanes hold crc0 of seg * 2^b bytes each.
#pragma unroll
  for (uint32_t b = 0; b < 6; ++b) {
    const uint32_t *nib = T + 1024 + (SEG_LOG2 + b - kScalarNibK0) * 128; // A_{2^(SEG_LOG2+b) bytes}
    uint32_t sh = 0;
#pragma unroll
    for (uint32_t i = 0; i < 8; ++i) sh ^= nib[i * 16 + ((s >> (4 * i)) & 15u)];
    const uint32_t mine = (lane >> b) & 1u ? s : sh; // left half shifted past the right half
    s = mine ^ __shfl_xor(mine, 1 << b);
  }

  if (lane == 0) {
    const uint64_t v = (uint64_t)(~(seed ^ s)) | ((uint64_t)seq << 32);
    __hip_atomic_store(result, v, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_SYSTEM);
  }
}

} // namespace

uint32_t scalar_seg_log2(uint32_t len) {
  uint32_t g = 2;
  while ((64u << g) < len) ++g;
  return g;
}

hipError_t launch_scalar(const uint8_t *stage, uint32_t len, const uint4 *tab, const uint32_t *tq, uint64_t *result,
                         uint32_t seq, hipStream_t stream) {
  if (len > kScalarMaxLen) return hipErrorInvalidValue;
  switch (scalar_seg_log2(len)) {
    case 2: crc32_scalar_kernel<2><<<1, 64, 0, stream>>>(stage, len, tab, tq, result, seq); break;
    case 3: crc32_scalar_kernel<3><<<1, 64, 0, stream>>>(stage, len, tab, tq, result, seq); break;
    case 4: crc32_scalar_kernel<4><<<1, 64, 0, stream>>>(stage, len, tab, tq, result, seq); break;
    case 5: crc32_scalar_kernel<5><<<1, 64, 0, stream>>>(stage, len, tab, tq, result, seq); break;
    default: crc32_scalar_kernel<6><<<1, 64, 0, stream>>>(stage, len, tab, tq, result, seq); break;
  }
  return hipGetLastError();
}

} // namespace rpccrc
