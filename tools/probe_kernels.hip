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
  std::vector<uint32_t> img(kLdsBytesV2 / 4), tq(kTqEntries);
  build_lds_image_v2(img.data());
  build_tq(tq.data());
  if (hipMalloc(&g_img, kLdsBytesV2) != hipSuccess) return -1;
  if (hipMalloc(&g_tq, kTqEntries * 4) != hipSuccess) return -1;
  if (hipMemcpy(g_img, img.data(), kLdsBytesV2, hipMemcpyHostToDevice) != hipSuccess) return -1;
  if (hipMemcpy(g_tq, tq.data(), kTqEntries * 4, hipMemcpyHostToDevice) != hipSuccess) return -1;
  return 0;
}

// abl bit 1024 (not a kernel ABL bit) selects the workgroup-dynamic dealing (DYN).
constexpr int kProbeDyn = 1024;
template <int QB, bool NT, int ABL, int DEPTH>
void go(const ItemsArgs &a, int blocks, hipStream_t s) {
  if constexpr ((ABL & kProbeDyn) != 0)
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
  V(1, 1, 1024, 1) V(1, 1, 1027, 1) V(1, 1, 1043, 1) V(1, 1, 1536, 1) V(4, 1, 1024, 1) V(4, 1, 1536, 1)
  return -22;
}

extern "C" __attribute__((visibility("default"))) int probe_rows(const uint8_t *d_base, uint64_t n, uint32_t len,
                                                                  uint64_t stride, uint32_t *d_out, int qb, int pair,
                                                                  int nt, int abl, int depth, int blocks,
                                                                  void *stream) {
  return probe_rows_times(d_base, n, len, stride, d_out, qb, pair, nt, abl, depth, blocks, stream, nullptr,
                          pair >> 8);
}
