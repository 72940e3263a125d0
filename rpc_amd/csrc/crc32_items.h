// rpc_amd/csrc/crc32_items.h -- the batched CRC-32 items kernel (device code).
//
// Included by crc32_kernels.hip (product instantiations) and by
// tools/probe_kernels.hip (ablation variants for measurement only).  See the
// design notes at the top of crc32_kernels.hip and DESIGN.md section 3.
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

#include "crc32_gf2.h"
#include "crc32_kernels.h"
#include "crc32_layout.h"

namespace rpccrc {

// Ablation bits (probe builds only; the product uses 0).
constexpr int kAblNoCompute = 1; // replace the slice-by-4 chain by an XOR fold
constexpr int kAblNoCombine = 2; // skip the per-lane shift / shuffle merge
constexpr int kAblNoLoad = 4;    // synthesize data instead of loading it

namespace detail {

__device__ __forceinline__ uint32_t lds_ld(const uint8_t *lds, uint32_t byte_addr) {
  return *reinterpret_cast<const uint32_t *>(lds + byte_addr);
}

// One slice-by-4 step: returns A_4(x) = T3[b0]^T2[b1]^T1[b2]^T0[b3].
// v_perm_b32 builds each LDS byte address {copy, byte of x, region, 0}.
__device__ __forceinline__ uint32_t slice4(const uint8_t *lds, uint32_t x, uint32_t lsel) {
  const uint32_t a3 = __builtin_amdgcn_perm(x, lsel, 0x0C0C0400u); // T3[x.b0]
  const uint32_t a2 = __builtin_amdgcn_perm(x, lsel, 0x0C0C0501u); // T2[x.b1]
  const uint32_t a1 = __builtin_amdgcn_perm(x, lsel, 0x0C020600u); // T1[x.b2]
  const uint32_t a0 = __builtin_amdgcn_perm(x, lsel, 0x0C020701u); // T0[x.b3]
  const uint32_t t3 = lds_ld(lds, a3), t2 = lds_ld(lds, a2);
  const uint32_t t1 = lds_ld(lds, a1), t0 = lds_ld(lds, a0);
  return t3 ^ t2 ^ t1 ^ t0;
}

// Linear map s -> XOR_n TAB[n][(s >> 4n) & 15] with TAB at base, row stride
// STRIDE bytes per nibble position and entry stride (1 << SHIFT) bytes.
template <uint32_t STRIDE, uint32_t SHIFT>
__device__ __forceinline__ uint32_t nib_map(const uint8_t *lds, uint32_t s, uint32_t base) {
  uint32_t r = 0;
#pragma unroll
  for (uint32_t n = 0; n < 8; ++n) {
    const uint32_t nib = (s >> (4 * n)) & 15u;
    r ^= lds_ld(lds, base + n * STRIDE + (nib << SHIFT));
  }
  return r;
}

__device__ __forceinline__ uint32_t xshfl(uint32_t v, int mask) {
  return (uint32_t)__shfl_xor((int)v, mask, 64);
}

struct Task {
  const uint8_t *p0; // body start
  uint64_t item;
  uint64_t lp;       // length incl. z trailing pad (multiple of 16 end)
  uint32_t len;
  uint32_t nrows;
  uint32_t r;
  uint32_t z;
  uint32_t w0;       // initial Horner value (A_q(F) or 0)
  uint32_t valid;    // 32-bit on purpose: no padding bytes to copy
};

typedef unsigned int u32x4 __attribute__((ext_vector_type(4)));

template <bool NT>
__device__ __forceinline__ uint4 ld16(const uint4 *p) {
  if constexpr (NT) {
    const u32x4 v = __builtin_nontemporal_load(reinterpret_cast<const u32x4 *>(p));
    return make_uint4(v.x, v.y, v.z, v.w);
  } else {
    return *p;
  }
}

} // namespace detail

template <int G, bool NT, int ABL = 0, int DEPTH = 1>
__global__ void __launch_bounds__(1024, 4) crc32_items_kernel(ItemsArgs a) {
  using namespace detail;
  __shared__ __attribute__((aligned(16))) uint32_t s_lds[kLdsWords];
  {
    const uint4 *src = a.lds_image;
    uint4 *dst = reinterpret_cast<uint4 *>(s_lds);
    for (uint32_t k = threadIdx.x; k < kLdsBytes / 16; k += blockDim.x) dst[k] = src[k];
  }
  __syncthreads();
  const uint8_t *lds = reinterpret_cast<const uint8_t *>(s_lds);

  constexpr uint32_t ROW = (uint32_t)G * kSegBytes;
  constexpr uint32_t GPW = 64 / G; // item groups per wavefront
  const uint32_t lane = threadIdx.x & 63u;
  const uint32_t lane4 = (lane & 31u) * 4u;
  const uint32_t lsel = lane4 | ((lane4 + 128u) << 8) | (1u << 16);
  const uint32_t s1base = kLdsS1 + lane4;
  const uint32_t s2base = kLdsS2 + (lane >> 3) * 4u;
  const uint32_t j = lane & (uint32_t)(G - 1);
  const uint32_t wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  const uint32_t waves_per_block = blockDim.x >> 6;
  const uint64_t nslots = (uint64_t)gridDim.x * waves_per_block * GPW;
  const uint64_t slot0 = ((uint64_t)blockIdx.x * waves_per_block + wave) * GPW + (GPW > 1 ? lane / (uint32_t)G : 0u);
  const uint32_t mode = a.mode;

  auto load_item = [&](uint64_t item, Task &t) {
    for (;;) {
      if (item >= a.n_items) {
        t.valid = 0u;
        return;
      }
      const uint64_t off = a.offsets ? a.offsets[item] : item * a.stride;
      const uint32_t len = a.lengths ? a.lengths[item] : a.len;
      if (len == 0) {
        if (j == 0) a.out[item] = 0u;
        item += nslots;
        continue;
      }
      t.valid = 1u;
      t.item = item;
      t.p0 = a.base + off;
      t.len = len;
      const uint32_t z = (uint32_t)(0u - (uint32_t)(uintptr_t)(t.p0 + len)) & 15u;
      t.z = z;
      t.lp = (uint64_t)len + z;
      t.nrows = (uint32_t)((t.lp + ROW - 1) / ROW);
      t.r = 0;
      const uint32_t first = (uint32_t)(t.lp - (uint64_t)(t.nrows - 1) * ROW);
      t.w0 = (mode == kModeRaw) ? 0u : a.tq[first];
      return;
    }
  };
  auto next_task = [&](const Task &c, Task &n) {
    if (c.r + 1 < c.nrows) {
      n = c;
      n.r = c.r + 1;
    } else {
      load_item(c.item + nslots, n);
    }
  };
  auto seg_of = [&](const Task &t) -> int64_t {
    return (int64_t)t.lp - (int64_t)(t.nrows - t.r) * (int64_t)ROW + (int64_t)(64u * j);
  };
  auto issue = [&](const Task &t, uint4 (&buf)[4]) {
    const int64_t seg = seg_of(t);
    if constexpr ((ABL & kAblNoLoad) != 0) {
#pragma unroll
      for (int b = 0; b < 4; ++b) {
        const uint32_t v = (uint32_t)seg * 0x9E3779B1u + (uint32_t)b;
        buf[b] = make_uint4(v, v ^ 0x5bd1e995u, v + 0x68e31da4u, ~v);
      }
      return;
    }
    const uint4 *p = reinterpret_cast<const uint4 *>(t.p0 + seg);
    if (seg >= 0) {
#pragma unroll
      for (int b = 0; b < 4; ++b) buf[b] = ld16<NT>(p + b);
    } else {
#pragma unroll
      for (int b = 0; b < 4; ++b)
        buf[b] = (seg + 16 * b + 16 > 0) ? ld16<NT>(p + b) : make_uint4(0u, 0u, 0u, 0u);
    }
  };
  uint32_t W = 0;
  auto compute = [&](const Task &t, const uint4 (&buf)[4]) {
    const int64_t seg = seg_of(t);
    uint32_t w[16];
#pragma unroll
    for (int b = 0; b < 4; ++b) {
      w[4 * b + 0] = buf[b].x;
      w[4 * b + 1] = buf[b].y;
      w[4 * b + 2] = buf[b].z;
      w[4 * b + 3] = buf[b].w;
    }
    if (t.r == 0 && seg < 0) { // bytes before the body start are zero padding
#pragma unroll
      for (int d = 0; d < 16; ++d) {
        const int64_t v = seg + 4 * d;
        if (v < 0) {
          const int64_t cut = -v;
          w[d] = cut >= 4 ? 0u : (w[d] & (0xFFFFFFFFu << (8 * (uint32_t)cut)));
        }
      }
    }
    if (t.z != 0 && t.r + 1 == t.nrows) { // bytes past the body end (pad to 16)
#pragma unroll
      for (int d = 0; d < 16; ++d) {
        const int64_t e = seg + 4 * d + 4 - (int64_t)t.len;
        if (e > 0) w[d] = e >= 4 ? 0u : (w[d] & (0xFFFFFFFFu >> (8 * (uint32_t)e)));
      }
    }
    uint32_t s = 0;
    if constexpr ((ABL & kAblNoCompute) != 0) {
#pragma unroll
      for (int d = 0; d < 16; ++d) s ^= w[d];
    } else if (seg + 64 > 0) {
      uint32_t x = w[0];
#pragma unroll
      for (int d = 0; d < 15; ++d) x = slice4(lds, x, lsel) ^ w[d + 1];
      s = slice4(lds, x, lsel);
    }
    if constexpr ((ABL & kAblNoCombine) == 0) {
      // Per-lane shift A_{64*(G-1-j)} in two nibble steps + XOR shuffles.
      s = nib_map<2048u, 7u>(lds, s, s1base);
      s ^= xshfl(s, 1);
      s ^= xshfl(s, 2);
      s ^= xshfl(s, 4);
      s = nib_map<512u, 5u>(lds, s, s2base);
      s ^= xshfl(s, 8);
      if constexpr (G == 64) {
        s ^= xshfl(s, 16);
        s ^= xshfl(s, 32);
      }
    }
    W = (t.r == 0) ? t.w0 : nib_map<64u, 2u>(lds, W, kLdsRW);
    W ^= s;
    if (t.r + 1 == t.nrows) {
      uint32_t res = W;
      if (t.z != 0) res = nib_map<64u, 2u>(lds, res, kLdsZI + (t.z - 1u) * 512u);
      if (mode == kModeFinal) res = ~res;
      if (j == 0) a.out[t.item] = res;
    }
  };

  if constexpr (DEPTH == 1) {
    // One row in flight ahead of the row being computed (2 register buffers).
    Task cur, nxt;
    uint4 bufA[4], bufB[4];
    load_item(slot0, cur);
    if (cur.valid) issue(cur, bufA);
    for (;;) {
      if (!cur.valid) break;
      next_task(cur, nxt);
      if (nxt.valid) issue(nxt, bufB);
      compute(cur, bufA);
      cur = nxt;
      if (!cur.valid) break;
      next_task(cur, nxt);
      if (nxt.valid) issue(nxt, bufA);
      compute(cur, bufB);
      cur = nxt;
    }
  } else {
    // Two rows in flight (3 rotating register buffers).
    Task cur, n1, n2;
    uint4 bufA[4], bufB[4], bufC[4];
    load_item(slot0, cur);
    if (cur.valid) issue(cur, bufA);
    if (cur.valid) next_task(cur, n1); else n1.valid = 0u;
    if (n1.valid) issue(n1, bufB);
    for (;;) {
      if (!cur.valid) break;
      if (n1.valid) next_task(n1, n2); else n2.valid = 0u;
      if (n2.valid) issue(n2, bufC);
      compute(cur, bufA);
      cur = n1; n1 = n2;
      if (!cur.valid) break;
      if (n1.valid) next_task(n1, n2); else n2.valid = 0u;
      if (n2.valid) issue(n2, bufA);
      compute(cur, bufB);
      cur = n1; n1 = n2;
      if (!cur.valid) break;
      if (n1.valid) next_task(n1, n2); else n2.valid = 0u;
      if (n2.valid) issue(n2, bufB);
      compute(cur, bufC);
      cur = n1; n1 = n2;
    }
  }
}

} // namespace rpccrc
