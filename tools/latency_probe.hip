// tools/latency_probe.hip -- MEASUREMENT ONLY: where the ~16 us of one drop-in
// rpc_crc32 call (crc.h:8) goes.  Each line times N back-to-back calls of one
// building block on a non-blocking stream and prints microseconds per call:
//   launch_sync     empty 1-wave kernel + hipStreamSynchronize
//   launch_spin     1-wave kernel that stores a sequence number to pinned host
//                   memory; the host spins on it (no hipStreamSynchronize)
//   image_sync      1024-thread kernel copying the 155 KiB LDS table image
//                   (what the rows kernel does first) + sync
//   pinned_rd_sync  1-wave kernel reading 68 B of pinned host memory and
//                   writing 4 B back to pinned memory + sync
//   rpc_crc32_68 / rpc_crc32_1k   the library's drop-in call
// usage: latency_probe [iters]     prints one JSON object
#include <hip/hip_runtime.h>
#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>
#include <time.h>

#include "rpccrc.h"

#define CK(x)                                                                              \
  do {                                                                                     \
    hipError_t e_ = (x);                                                                   \
    if (e_ != hipSuccess) {                                                                \
      fprintf(stderr, "%s:%d %s: %s\n", __FILE__, __LINE__, #x, hipGetErrorString(e_));    \
      exit(1);                                                                             \
    }                                                                                      \
  } while (0)

static double now(void) {
  struct timespec ts;
  clock_gettime(CLOCK_MONOTONIC, &ts);
  return ts.tv_sec + ts.tv_nsec * 1e-9;
}

constexpr uint32_t kImageBytes = 158736; // crc32_layout.h kLdsBytesV2

__global__ void k_empty() {}

__global__ void k_flag(volatile uint32_t *flag, uint32_t seq) {
  if (threadIdx.x == 0) {
    __hip_atomic_store(flag, seq, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_SYSTEM);
  }
}

__global__ __launch_bounds__(1024) void k_image(const uint4 *src, uint32_t *out) {
  extern __shared__ uint4 lds[];
  for (uint32_t i = threadIdx.x; i < kImageBytes / 16; i += 1024) lds[i] = src[i];
  __syncthreads();
  if (threadIdx.x == 0) out[0] = lds[(kImageBytes / 16) - 1].x;
}

__global__ void k_pinned_rd(const uint32_t *in, uint32_t n_words, uint32_t *out) {
  uint32_t v = threadIdx.x < n_words ? in[threadIdx.x] : 0u;
  for (int o = 32; o > 0; o >>= 1) v ^= __shfl_xor(v, o);
  if (threadIdx.x == 0) out[0] = v;
}

int main(int argc, char **argv) {
  const int iters = argc > 1 ? atoi(argv[1]) : 20000;
  hipStream_t s;
  CK(hipStreamCreateWithFlags(&s, hipStreamNonBlocking));
  uint32_t *pin = nullptr, *dout = nullptr;
  uint4 *img = nullptr;
  CK(hipHostMalloc(reinterpret_cast<void **>(&pin), 4096, hipHostMallocDefault));
  CK(hipMalloc(reinterpret_cast<void **>(&img), kImageBytes));
  CK(hipMalloc(reinterpret_cast<void **>(&dout), 64));
  CK(hipMemset(img, 0x5a, kImageBytes));
  CK(hipFuncSetAttribute(reinterpret_cast<const void *>(k_image), hipFuncAttributeMaxDynamicSharedMemorySize,
                         kImageBytes));
  memset(pin, 0, 4096);
  uint8_t body[1024];
  for (int i = 0; i < 1024; ++i) body[i] = (uint8_t)(i * 131 + 7);

  printf("{\"iters\": %d", iters);
  for (int rep = 0; rep < 2; ++rep) { // rep 0 warms up; rep 1 is printed
    double t0, us;
    t0 = now();
    for (int i = 0; i < iters; ++i) {
      k_empty<<<1, 64, 0, s>>>();
      CK(hipStreamSynchronize(s));
    }
    us = (now() - t0) / iters * 1e6;
    if (rep) printf(", \"launch_sync_us\": %.2f", us);

    volatile uint32_t *flag = pin + 512;
    t0 = now();
    for (int i = 0; i < iters; ++i) {
      const uint32_t seq = (uint32_t)(rep * iters + i + 1);
      k_flag<<<1, 64, 0, s>>>(flag, seq);
      while (*flag != seq) {
      }
    }
    us = (now() - t0) / iters * 1e6;
    CK(hipStreamSynchronize(s));
    if (rep) printf(", \"launch_spin_us\": %.2f", us);

    t0 = now();
    for (int i = 0; i < iters; ++i) {
      k_image<<<1, 1024, kImageBytes, s>>>(img, dout);
      CK(hipStreamSynchronize(s));
    }
    us = (now() - t0) / iters * 1e6;
    if (rep) printf(", \"image_sync_us\": %.2f", us);

    t0 = now();
    for (int i = 0; i < iters; ++i) {
      memcpy(pin, body, 68);
      k_pinned_rd<<<1, 64, 0, s>>>(pin, 17, pin + 256);
      CK(hipStreamSynchronize(s));
    }
    us = (now() - t0) / iters * 1e6;
    if (rep) printf(", \"pinned_rd_sync_us\": %.2f", us);

    const size_t lens[2] = {68, 1024};
    const char *names[2] = {"rpc_crc32_68_us", "rpc_crc32_1k_us"};
    for (int k = 0; k < 2; ++k) {
      uint32_t acc = 0;
      t0 = now();
      for (int i = 0; i < iters; ++i) acc ^= rpc_crc32(body, lens[k]);
      us = (now() - t0) / iters * 1e6;
      if (rep) printf(", \"%s\": %.2f, \"%s_acc\": %u", names[k], us, names[k], acc);
    }
  }
  printf("}\n");
  return 0;
}
