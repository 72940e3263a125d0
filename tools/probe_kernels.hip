// tools/probe_kernels.hip -- MEASUREMENT ONLY: ablation / tuning variants of the
// items kernel (rpc_amd/csrc/crc32_items.h), built into tools/libprobe.so by
// tools/Makefile and driven by tools/probe.py.  Results of ablated variants are
// wrong by construction; only their timing is used.  Not part of the product.
#include <hip/hip_runtime.h>

#include <vector>

#include "crc32_items.h"

using namespace rpccrc;

namespace {
uint4 *g_img = nullptr;
uint32_t *g_tq = nullptr;

int ensure_tables() {
  if (g_img) return 0;
  std::vector<uint32_t> img(kLdsWords), tq(kTqEntries);
  build_lds_image(64, img.data());
  build_tq(tq.data());
  if (hipMalloc(&g_img, kLdsBytes) != hipSuccess) return -1;
  if (hipMalloc(&g_tq, kTqEntries * 4) != hipSuccess) return -1;
  if (hipMemcpy(g_img, img.data(), kLdsBytes, hipMemcpyHostToDevice) != hipSuccess) return -1;
  if (hipMemcpy(g_tq, tq.data(), kTqEntries * 4, hipMemcpyHostToDevice) != hipSuccess) return -1;
  return 0;
}

template <bool NT, int ABL, int DEPTH>
void launch(const ItemsArgs &a, int blocks, hipStream_t s) {
  hipLaunchKernelGGL((crc32_items_kernel<64, NT, ABL, DEPTH>), dim3(blocks), dim3(1024), 0, s, a);
}

template <bool NT, int ABL>
int by_depth(const ItemsArgs &a, int depth, int blocks, hipStream_t s) {
  if (depth == 1) launch<NT, ABL, 1>(a, blocks, s);
  else if (depth == 2) launch<NT, ABL, 2>(a, blocks, s);
  else return -22;
  return 0;
}

template <bool NT>
int by_abl(const ItemsArgs &a, int abl, int depth, int blocks, hipStream_t s) {
  switch (abl) {
  case 0: return by_depth<NT, 0>(a, depth, blocks, s);
  case 1: return by_depth<NT, 1>(a, depth, blocks, s);
  case 2: return by_depth<NT, 2>(a, depth, blocks, s);
  case 3: return by_depth<NT, 3>(a, depth, blocks, s);
  case 4: return by_depth<NT, 4>(a, depth, blocks, s);
  case 6: return by_depth<NT, 6>(a, depth, blocks, s);
  default: return -22;
  }
}
} // namespace

extern "C" __attribute__((visibility("default"))) int probe_uniform(const uint8_t *d_base, uint64_t n, uint32_t len,
                                                                     uint32_t *d_out, int nt, int abl, int depth,
                                                                     int blocks, void *stream) {
  if (ensure_tables()) return -12;
  ItemsArgs a;
  a.base = d_base;
  a.offsets = nullptr;
  a.lengths = nullptr;
  a.n_items = n;
  a.stride = len;
  a.len = len;
  a.mode = kModeFinal;
  a.lds_image = g_img;
  a.tq = g_tq;
  a.out = d_out;
  hipStream_t s = static_cast<hipStream_t>(stream);
  int rc = nt ? by_abl<true>(a, abl, depth, blocks, s) : by_abl<false>(a, abl, depth, blocks, s);
  if (rc) return rc;
  return hipGetLastError() == hipSuccess ? 0 : -5;
}
