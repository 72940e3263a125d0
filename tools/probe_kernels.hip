// tools/probe_kernels.hip -- MEASUREMENT ONLY: ablation / tuning variants of the
// rows kernel (rpc_amd/csrc/crc32_rows.h), built into tools/libprobe.so by
// tools/Makefile and driven by tools/probe.py --mode ablate.  Outputs of
// ablated variants are wrong by construction; only their timing is used.
#include <hip/hip_runtime.h>

#include <vector>

#include "crc32_rows.h"

using namespace rpccrc;

namespace {
uint4 *g_img = nullptr;
uint32_t *g_tq = nullptr;

int ensure_tables() {
  if (g_img) return 0;
  std::vector<uint32_t> img(kLdsBytesV3 / 4), compact(kImgCompactBytes / 4), tq(kTqEntries);
  build_lds_image_v2(img.data());
  build_lds_image_compact(img.data(), compact.data());
  build_tq(tq.data());
  if (hipMalloc(&g_img, kImgHbmBytes) != hipSuccess) return -1;
  if (hipMalloc(&g_tq, kTqEntries * 4) != hipSuccess) return -1;
  if (hipMemcpy(g_img, kImgCompact ? compact.data() : img.data(), kImgHbmBytes, hipMemcpyHostToDevice) != hipSuccess)
    return -1;
  if (hipMemcpy(g_tq, tq.data(), kTqEntries * 4, hipMemcpyHostToDevice) != hipSuccess) return -1;
  return 0;
}

// abl bit 1024 (not a kernel ABL bit) selects the workgroup-dynamic dealing (DYN);
// 4096 (with 1024) adds the product's tail stealing (15 % of the rounds in the
// pool, a probe-owned counter that each launch's last workgroup resets).
constexpr int kProbeDyn = 1024;
constexpr int kProbeSteal = 4096;
uint32_t *g_steal = nullptr;
template <int QB, bool NT, int ABL, int DEPTH>
void go(const ItemsArgs &a, int blocks, hipStream_t s) {
  if constexpr ((ABL & kProbeSteal) != 0) {
    if (!g_steal) {
      if (hipMalloc(&g_steal, 256) != hipSuccess || hipMemset(g_steal, 0, 256) != hipSuccess) return;
    }
    ItemsArgs k = a;
    const uint64_t tasks = QB == 4 ? (a.n_items + 3) / 4 : a.n_items;
    const uint64_t rounds = (tasks + dyn_round(QB) - 1) / dyn_round(QB);
    const uint64_t st = (uint64_t)((double)rounds * 0.85) / (uint64_t)blocks;
    k.steal = g_steal;
    k.steal_s = (uint32_t)st;
    hipLaunchKernelGGL((crc32_rows_kernel<QB, NT, false, (ABL & ~(kProbeDyn | kProbeSteal)), DEPTH, true, true>),
                       dim3(blocks), dim3(1024), 0, s, k);
  } else if constexpr ((ABL & kProbeDyn) != 0)
    hipLaunchKernelGGL((crc32_rows_kernel<QB, NT, false, (ABL & ~kProbeDyn), DEPTH, true>), dim3(blocks), dim3(1024),
                       0, s, a);
  else
    hipLaunchKernelGGL((crc32_rows_kernel<QB, NT, false, ABL, DEPTH>), dim3(blocks), dim3(1024), 0, s, a);
}
} // namespace

#define V(QB, NT, ABL, D)                                                             \
  if (qb == QB && nt == NT && abl == ABL && depth == D) {                             \
    go<QB, NT, ABL, D>(a, blocks, s);                                                 \
    return hipGetLastError() == hipSuccess ? 0 : -5;                                  \
  }

extern "C" __attribute__((visibility("default"))) int probe_rows_times(const uint8_t *d_base, uint64_t n,
                                                                        uint32_t len, uint64_t stride, uint32_t *d_out,
                                                                        int qb, int pair, int nt, int abl, int depth,
                                                                        int blocks, void *stream, uint64_t *d_times,
                                                                        int gshift) {
  if (ensure_tables()) return -12;
  ItemsArgs a;
  a.base = d_base;
  a.offsets = d_times; // kRowsAblTimes variants only (uniform batches never read offsets)
  a.lengths = nullptr;
  a.n_items = n;
  a.stride = stride;
  a.len = len;
  a.mode = kModeFinal;
  a.lds_image = g_img;
  a.tq = g_tq;
  a.out = d_out;
  a.gshift = (uint32_t)gshift;
  hipStream_t s = static_cast<hipStream_t>(stream);
  V(1, 1, 0, 1) V(1, 0, 0, 1) V(1, 1, 1, 1) V(1, 1, 2, 1) V(1, 1, 3, 1) V(1, 1, 4, 1) V(1, 1, 6, 1)
  V(1, 1, 0, 2) V(1, 0, 0, 2) V(1, 1, 3, 2) V(1, 1, 8, 1) V(1, 1, 11, 1) V(1, 1, 9, 1) V(1, 0, 11, 1) V(1, 0, 3, 1) V(1, 1, 16, 1) V(1, 1, 19, 1) V(1, 1, 32, 1) V(1, 1, 35, 1) V(1, 1, 51, 1) V(1, 1, 64, 1) V(1, 1, 128, 1) V(1, 1, 192, 1) V(1, 1, 67, 1) V(1, 1, 131, 1) V(1, 1, 195, 1)
  V(4, 1, 0, 1) V(4, 0, 0, 1) V(4, 1, 3, 1) V(4, 1, 4, 1) V(4, 1, 6, 1) V(4, 1, 0, 2) V(4, 1, 3, 2)
  V(1, 1, 259, 1) V(1, 1, 275, 1) V(1, 1, 512, 1) V(4, 1, 512, 1)
  V(1, 1, 5632, 1) V(4, 1, 5632, 1)
  V(1, 1, 1024, 1) V(1, 1, 1027, 1) V(1, 1, 1043, 1) V(1, 1, 1536, 1) V(4, 1, 1024, 1) V(4, 1, 1536, 1)
  V(1, 1, 1025, 1) V(1, 1, 1026, 1) V(1, 1, 1028, 1) V(1, 1, 1056, 1) V(1, 1, 1059, 1)
  V(1, 1, 9216, 1) V(4, 1, 1027, 1) V(4, 1, 1043, 1) V(4, 1, 1028, 1) V(1, 1, 3072, 1) V(4, 1, 3072, 1) V(1, 1, 1040, 1) V(4, 1, 1040, 1)
  return -22;
}

extern "C" __attribute__((visibility("default"))) int probe_rows(const uint8_t *d_base, uint64_t n, uint32_t len,
                                                                  uint64_t stride, uint32_t *d_out, int qb, int pair,
                                                                  int nt, int abl, int depth, int blocks,
                                                                  void *stream) {
  return probe_rows_times(d_base, n, len, stride, d_out, qb, pair, nt, abl, depth, blocks, stream, nullptr,
                          pair >> 8);
}

// Ragged QB = 1 DYN rows kernel (the C2 path, static rounds) under ablation
// bits: 0 product, kRowsAblNoSub full first rows, 3 memory only, 4 compute
// only (synthesized rows, metadata still read), 16 no stores, 2 no merge.
template <int ABL>
void go_ragged(const ItemsArgs &a, int blocks, hipStream_t s) {
  hipLaunchKernelGGL((crc32_rows_kernel<1, true, true, ABL, 1, true>), dim3(blocks), dim3(1024), 0, s, a);
}
extern "C" __attribute__((visibility("default"))) int probe_rows_ragged(const uint8_t *d_base, const uint64_t *d_offs,
                                                                         const uint32_t *d_lens, uint64_t n,
                                                                         uint32_t *d_out, int abl, int blocks,
                                                                         void *stream) {
  if (ensure_tables()) return -12;
  ItemsArgs a;
  a.base = d_base;
  a.offsets = d_offs;
  a.lengths = d_lens;
  a.n_items = n;
  a.stride = 0;
  a.len = 0;
  a.mode = kModeFinal;
  a.lds_image = g_img;
  a.tq = g_tq;
  a.out = d_out;
  a.gshift = 0;
  hipStream_t s = static_cast<hipStream_t>(stream);
  switch (abl) {
  case 0: go_ragged<0>(a, blocks, s); break;
  case kRowsAblNoSub: go_ragged<kRowsAblNoSub>(a, blocks, s); break;
  case 3: go_ragged<3>(a, blocks, s); break;
  case 4: go_ragged<4>(a, blocks, s); break;
  case 16: go_ragged<16>(a, blocks, s); break;
  case 2: go_ragged<2>(a, blocks, s); break;
  case 3 | 16: go_ragged<3 | 16>(a, blocks, s); break;
  case kRowsAblPipeMem: go_ragged<kRowsAblPipeMem>(a, blocks, s); break;
  default: return -22;
  }
  return hipGetLastError() == hipSuccess ? 0 : -5;
}

// The same kernel with the per-wave timeline (kRowsAblTimes; exact results):
// d_times (4 words per wave) travels in round_out, unused by ragged batches.
extern "C" __attribute__((visibility("default"))) int probe_rows_ragged_times(const uint8_t *d_base, const uint64_t *d_offs,
                                                                               const uint32_t *d_lens, uint64_t n,
                                                                               uint32_t *d_out, int blocks, void *stream,
                                                                               uint64_t *d_times, int steal) {
  if (ensure_tables()) return -12;
  ItemsArgs a;
  a.base = d_base;
  a.offsets = d_offs;
  a.lengths = d_lens;
  a.n_items = n;
  a.stride = 0;
  a.len = 0;
  a.mode = kModeFinal;
  a.lds_image = g_img;
  a.tq = g_tq;
  a.out = d_out;
  a.gshift = 0;
  a.round_out = reinterpret_cast<uint32_t *>(d_times);
  hipStream_t s = static_cast<hipStream_t>(stream);
  if (steal) { // the product's pool sizing (launch_rows): steal % of the rounds, at most 48 per workgroup
    static uint32_t *ctr = nullptr;
    if (!ctr && hipMalloc(&ctr, 64) != hipSuccess) return -12;
    if (hipMemsetAsync(ctr, 0, 64, s) != hipSuccess) return -5;
    const uint64_t rounds = (n + kDynRound - 1) / kDynRound;
    uint64_t st = (uint64_t)((double)rounds * (1.0 - steal / 100.0)) / (uint64_t)blocks;
    if (rounds / blocks > st + 48) st = rounds / blocks - 48;
    a.steal = ctr;
    a.steal_s = (uint32_t)st;
    hipLaunchKernelGGL((crc32_rows_kernel<1, true, true, kRowsAblTimes, 1, true, true>), dim3(blocks), dim3(1024), 0,
                       s, a);
  } else {
    hipLaunchKernelGGL((crc32_rows_kernel<1, true, true, kRowsAblTimes, 1, true>), dim3(blocks), dim3(1024), 0, s, a);
  }
  return hipGetLastError() == hipSuccess ? 0 : -5;
}

// ---------------------------------------------------------------------------
// Row-shape stream probes (MEASUREMENT ONLY): does a wave-iteration cost track
// the bytes it reads or the load instructions it issues?  Tile t of TB bytes
// (t = gw + k * nwaves, all waves one moving window), NT buffer loads of 1 KiB
// per instruction (lane L at 16 L):
//   MODE 0: 4 loads, TB = 4 KiB          MODE 1: 3 loads + 1 out-of-range, TB = 3 KiB
//   MODE 2: 3 loads, TB = 3 KiB          MODE 3: 8 loads, TB = 8 KiB
// ---------------------------------------------------------------------------
template <int MODE>
__global__ void __launch_bounds__(1024, 4) stream_rows_probe(const uint8_t *p, uint64_t ntiles, uint32_t *out) {
  constexpr uint32_t TB = MODE == 0 ? 4096 : MODE == 3 ? 8192 : 3072;
  constexpr int NL = MODE == 3 ? 8 : MODE == 2 ? 3 : 4;
  const uint32_t lane = threadIdx.x & 63u;
  const uint64_t gw = (uint64_t)blockIdx.x * 16u + (threadIdx.x >> 6);
  const uint64_t nw = (uint64_t)gridDim.x * 16u;
  uint32_t acc = 0;
  for (uint64_t t = gw; t < ntiles; t += nw) {
    const auto rs = rows::row_rsrc((uint64_t)(uintptr_t)(p + t * TB));
    rows::u32x4 v[NL];
#pragma unroll
    for (int b = 0; b < NL; ++b) {
      const uint32_t off = (MODE == 1 && b == 3) ? rows::kOobOffset : (uint32_t)(b * 1024 + 16 * lane);
      v[b] = rows::ldb16<true>(rs, off);
    }
#pragma unroll
    for (int b = 0; b < NL; ++b) acc ^= v[b][0] ^ v[b][1] ^ v[b][2] ^ v[b][3];
  }
  if (acc == 0x9E3779B9u) out[0] = acc;
}

extern "C" __attribute__((visibility("default"))) int probe_stream_rows(const uint8_t *d_base, uint64_t nbytes, int mode,
                                                                         int blocks, uint32_t *d_out, void *stream) {
  hipStream_t s = static_cast<hipStream_t>(stream);
  const uint64_t tb = mode == 0 ? 4096 : mode == 3 ? 8192 : 3072;
  const uint64_t nt = nbytes / tb;
  switch (mode) {
  case 0: hipLaunchKernelGGL(stream_rows_probe<0>, dim3(blocks), dim3(1024), 0, s, d_base, nt, d_out); break;
  case 1: hipLaunchKernelGGL(stream_rows_probe<1>, dim3(blocks), dim3(1024), 0, s, d_base, nt, d_out); break;
  case 2: hipLaunchKernelGGL(stream_rows_probe<2>, dim3(blocks), dim3(1024), 0, s, d_base, nt, d_out); break;
  case 3: hipLaunchKernelGGL(stream_rows_probe<3>, dim3(blocks), dim3(1024), 0, s, d_base, nt, d_out); break;
  default: return -22;
  }
  return hipGetLastError() == hipSuccess ? 0 : -5;
}
