// rpc_amd/csrc/crc32_service.hip -- the drop-in rpc_crc32 (crc.h:8, crc.c:4-9)
// without a kernel launch per call: a small resident SERVICE kernel (one
// workgroup of kSvcWaves waves) polls request slots in pinned host memory and
// answers each with one wave.
//
// Why: a launch + completion costs ~6.6 us of the 8.3 us a one-wave-kernel
// call took (tools/latency_probe.hip, profiles/r02/r02n_*), against 0.025 us
// for the reference crc.c on a 68-B body.  The reference's callers make one
// call per RPC (client stamp rpc_async.c:525, recv verify :219; server verify
// rpc_server_main.c:227, stamp :249), from up to 10 threads.
//
// Protocol (SvcShared, hipHostMallocCoherent: every access below bypasses the
// GPU caches -- sc0 sc1 loads / stores, no cache-wide fence):
//   host   writes a body of <= kSvcInline bytes into the slot's request block
//          (SvcReq: the bytes, ending at inline byte 116, then the tag), a
//          longer one right-aligned into body[slot] (virtual buffer of 64 * seg
//          bytes, seg = 4 / 8 / 16 bytes per lane by length), then
//          rq[slot].req = {len, seq} as ONE 64-bit store (x86 stores stay in order);
//   wave   polls the request blocks of its kSvcPer slots (one dword per lane,
//          both blocks in one round trip); a seq it has not answered is a
//          request once its check sum matches the tag (crc32_kernels.h SvcReq:
//          a non-linear, position-dependent sum over every word used).  An
//          inline body is already in registers; a longer one is read (every
//          lane its seg bytes; the loads of all its pending slots in flight
//          together) and its words enter the sum.  It computes the CRC and
//          stores {crc, seq} into res[slot] (one 64-bit store);
//   host   spins on res[slot] until the seq matches.
// The waves share the time of the last request in LDS (4 bytes) and all leave
// after idle_ticks without one, after the kernel's lifetime cap, or when the
// host sets ctl[kSvcStop] -- together: the first wave to decide sets s_leave,
// which every wave checks before each poll; the last wave out stores its instance number into
// ctl[kSvcExited], so the host knows when to launch a new instance (a request
// that arrives while an instance is leaving is picked up by the next one:
// pending = seq not yet answered in res).
//
// Resources: no table image in LDS (476 B: the Tq words of the inline
// lengths) and few registers (37 VGPRs; built without the library's max-ilp
// scheduler, Makefile), so the kernel can sit on a CU next to a rows-kernel
// workgroup (155-159 KiB LDS each, one per CU, a persistent grid over all CUs;
// crc32_rows.h kRowsLdsMax keeps 1 KiB free for it): the CRC is bit-serial --
//   chain: crc0 of each 32-bit word by the bit loop (3 VALU per bit);
//   merge: lane L's segment crc0 times x^(8 * seg * (63 - L)) mod P (per-lane
//          constant from the host, kSvcShift), bit-serial, then an XOR over
//          the 64 lanes;
//   final: ~(Tq[len] ^ crc0), Tq[len] = A_len(0xFFFFFFFF) (zlib's conditioning).
#include <hip/hip_runtime.h>

#include "crc32_gf2.h"
#include "crc32_kernels.h"
#include "crc32_layout.h"
#include "crc32_service_math.h"

namespace rpccrc {

namespace {

// 16-B load that bypasses the GPU caches (sc0 sc1: system coherence), from a
// wave-uniform base + lane offset; offsets past the range read zeros.
__device__ __forceinline__ uint4 ld_sys16(const void *base, uint32_t range, uint32_t off) {
  const __amdgpu_buffer_rsrc_t r =
      __builtin_amdgcn_make_buffer_rsrc(const_cast<void *>(base), (short)0, (int)range, 0x00020000);
  typedef unsigned int u32x4 __attribute__((ext_vector_type(4)));
  const u32x4 v = __builtin_amdgcn_raw_buffer_load_b128(r, (int)off, 0, 1 | 16);
  return make_uint4(v[0], v[1], v[2], v[3]);
}
__device__ __forceinline__ uint32_t ld_sys32(const uint32_t *p) {
  return __hip_atomic_load(p, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
}

// A request's body words: lane L's seg bytes of V = body + 64*seg - len..., as
// dwords (the words past seg/4 are zero).  Issued for every pending slot of the
// wave before any is computed, so their PCIe round trips overlap.
struct Body {
  uint32_t w[4];
};
__device__ __forceinline__ Body load_body(const uint8_t *body, uint32_t seg, uint32_t lane) {
  Body b;
  const uint32_t *p = reinterpret_cast<const uint32_t *>(body + lane * seg);
  if (seg == 16u) {
    const uint4 v = ld_sys16(body, 64u * 16u, lane * 16u);
    b.w[0] = v.x;
    b.w[1] = v.y;
    b.w[2] = v.z;
    b.w[3] = v.w;
  } else {
    b.w[0] = ld_sys32(p);
    b.w[1] = seg == 8u ? ld_sys32(p + 1) : 0u;
    b.w[2] = 0u;
    b.w[3] = 0u;
  }
  return b;
}

// crc0 of V: the lane's chain over its seg / 4 words (bytes before the body
// masked), shifted to V's end by the lane's constant, XORed over the wave; and
// the request check's sum over the same masked words (svc::word_hash at
// position kHashBodyPos + word index, XORed over the wave).
struct BodySums {
  uint32_t c0, h;
};
__device__ __forceinline__ BodySums body_crc0(const Body &b, uint32_t seg, uint32_t len, uint32_t lane,
                                              uint32_t kshift) {
  const uint32_t off0 = 64u * seg - len; // V offset of the body's first byte
  uint32_t s = 0, h = 0;
#pragma unroll
  for (uint32_t d = 0; d < 4; ++d)
    if (4u * d < seg) {
      const uint32_t w = b.w[d] & svc::keep_mask(lane * seg + 4u * d, off0);
      s = svc::crc0_word(s ^ w);
      h ^= svc::word_hash(w, svc::kHashBodyPos + lane * (seg >> 2) + d);
    }
  s = svc::mulmod(s, kshift);
#pragma unroll
  for (int m = 1; m < 64; m <<= 1) {
    s ^= (uint32_t)__shfl_xor((int)s, m, 64);
    h ^= (uint32_t)__shfl_xor((int)h, m, 64);
  }
  return BodySums{s, h};
}

__global__ __launch_bounds__(64 * kSvcWaves) __attribute__((amdgpu_waves_per_eu(8, 8))) void crc32_service_kernel(
    SvcShared *sh, const uint32_t *tq, const uint32_t *kshift, uint64_t idle_ticks, uint64_t life_ticks,
    uint32_t instance) {
  __shared__ uint32_t s_last;  // low 32 bits of the last request's s_memrealtime
  __shared__ uint32_t s_alive; // waves still in the loop
  __shared__ uint32_t s_leave; // set by the first wave that decides to leave: all leave
  // Tq of the inline lengths: an LDS read instead of a dependent global load per
  // request (476 B of LDS still fits beside any rows workgroup: <= 163040 B)
  __shared__ uint32_t s_tq[kSvcInline + 1];
  const uint32_t lane = threadIdx.x & 63u;
  const uint32_t wave = threadIdx.x >> 6;
  const uint64_t t_start = __builtin_amdgcn_s_memrealtime();
  if (threadIdx.x == 0) {
    s_last = (uint32_t)t_start;
    s_alive = kSvcWaves;
    s_leave = 0u;
    // the host sees this instance running (a vector store): until then, after a
    // request that went unanswered, its calls take the launch path
    __hip_atomic_store(&sh->ctl[kSvcStarted], instance, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
  }
  for (uint32_t k = threadIdx.x; k <= kSvcInline; k += 64 * kSvcWaves) s_tq[k] = tq[k];
  __syncthreads();
  static_assert(kSvcPer == 2, "one poll: 2 request blocks x 32 dwords");
  // per-lane constants: shift of this lane's segment to V's end, per seg class
  const uint32_t k4 = kshift[0 * 64 + lane], k8 = kshift[1 * 64 + lane], k16 = kshift[2 * 64 + lane];
  // wave w owns slots w + kSvcWaves * i (i < kSvcPer): the host hands slots out
  // lowest first, so concurrent callers land on different waves.  Poll: lane
  // 32 i + d reads dword d of slot i's request block.
  const uint32_t pslot = wave + kSvcWaves * (lane >> 5);
  const uint32_t *pblk = reinterpret_cast<const uint32_t *>(&sh->rq[pslot]) + (lane & 31u);
  // the seq this wave last answered for its slot i (wave-uniform)
  uint32_t served[kSvcPer];
#pragma unroll
  for (uint32_t i = 0; i < kSvcPer; ++i)
    served[i] = (uint32_t)(__hip_atomic_load(&sh->res[wave + kSvcWaves * i][0], __ATOMIC_RELAXED,
                                             __HIP_MEMORY_SCOPE_SYSTEM) >> 32);
  // An inline body ends at block byte 124: V byte v (V = 256 B, seg 4) is block
  // byte v - 132, so lane L's word is block dword L - 33 (lanes >= 33).
  const int src0 = (int)lane - 33;
  for (uint32_t poll = 0;; ++poll) {
    // one wave decided to leave: all leave together (a wave that stayed would
    // keep the instance alive while the departed wave's slots went unanswered)
    if (__hip_atomic_load(&s_leave, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP) != 0u) break;
    const uint32_t pv = ld_sys32(pblk); // both blocks, one round trip
    // the request check (crc32_kernels.h SvcReq): lane 32 i + d hashes block
    // dword d at position d (d < 31), lane 32 i + 31 holds the tag as read; the
    // XOR over each block's 32 lanes is 0 for a whole, current inline request
    const uint32_t bd = lane & 31u;
    uint32_t xs = bd == 31u ? pv : svc::word_hash(pv, bd);
    xs ^= (uint32_t)__builtin_amdgcn_mov_dpp((int)xs, 0xB1, 0xF, 0xF, true);  // quad_perm [1,0,3,2]
    xs ^= (uint32_t)__builtin_amdgcn_mov_dpp((int)xs, 0x4E, 0xF, 0xF, true);  // quad_perm [2,3,0,1]
    xs ^= (uint32_t)__builtin_amdgcn_mov_dpp((int)xs, 0x124, 0xF, 0xF, true); // row_ror:4
    xs ^= (uint32_t)__builtin_amdgcn_mov_dpp((int)xs, 0x128, 0xF, 0xF, true); // row_ror:8
    {
      const auto sw = __builtin_amdgcn_permlane16_swap(xs, xs, false, false); // lane bit 4
      xs = sw[0] ^ sw[1];
    }
    uint32_t lens[kSvcPer], seqs[kSvcPer], xsum[kSvcPer];
    bool pend[kSvcPer], inl[kSvcPer];
    bool any = false;
#pragma unroll
    for (uint32_t i = 0; i < kSvcPer; ++i) {
      lens[i] = (uint32_t)__builtin_amdgcn_readlane((int)pv, (int)(32 * i + 0));
      seqs[i] = (uint32_t)__builtin_amdgcn_readlane((int)pv, (int)(32 * i + 1));
      xsum[i] = (uint32_t)__builtin_amdgcn_readlane((int)xs, (int)(32 * i));
      if (lens[i] > kSvcMaxLen) lens[i] = kSvcMaxLen; // (the host never sends more; the check then fails)
      inl[i] = lens[i] <= kSvcInline;
      // an inline request counts once its block's sum matches; a longer one is
      // read first and counts once the block's and the body's sums match the tag
      pend[i] = seqs[i] != served[i] && (!inl[i] || xsum[i] == 0u);
      any = any || pend[i];
    }
    if (any) {
      // the longer bodies' loads first (a second round trip, both slots' in
      // flight together), then the CRCs
      Body body[kSvcPer];
#pragma unroll
      for (uint32_t i = 0; i < kSvcPer; ++i) {
        if (pend[i] && !inl[i]) {
          body[i] = load_body(sh->body[wave + kSvcWaves * i], svc::seg_of(lens[i]), lane);
        } else {
          // (every lane runs the shuffle: a lane outside the exec mask is not a
          // source -- a shuffle under `src0 >= 0` read zeros from lanes 0..30)
          const int src = src0 >= 0 ? (int)(32 * i) + src0 : (int)lane;
          const uint32_t wv = (uint32_t)__shfl((int)pv, src, 64);
          body[i].w[0] = src0 >= 0 ? wv : 0u; // (lanes < 33: before V's body, masked anyway)
          body[i].w[1] = body[i].w[2] = body[i].w[3] = 0u;
        }
      }
#pragma unroll
      for (uint32_t i = 0; i < kSvcPer; ++i) {
        if (!pend[i]) continue;
        const uint32_t len = lens[i], seg = svc::seg_of(len);
        const BodySums bs = body_crc0(body[i], seg, len, lane, seg == 4u ? k4 : seg == 8u ? k8 : k16);
        // a longer body: its words as read must match the tag too (a torn
        // {len, seq} pair or body read fails here; the next poll retries)
        if (!inl[i] && (xsum[i] ^ bs.h) != 0u) continue;
        const uint32_t crc = len == 0u ? 0u : ~((inl[i] ? s_tq[len] : tq[len]) ^ bs.c0);
        if (lane == 0)
          __hip_atomic_store(&sh->res[wave + kSvcWaves * i][0], (uint64_t)crc | ((uint64_t)seqs[i] << 32),
                             __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
        served[i] = seqs[i];
      }
      if (lane == 0)
        __hip_atomic_store(&s_last, (uint32_t)__builtin_amdgcn_s_memrealtime(), __ATOMIC_RELAXED,
                           __HIP_MEMORY_SCOPE_WORKGROUP);
      continue;
    }
    const uint64_t now = __builtin_amdgcn_s_memrealtime();
    const uint32_t last = __hip_atomic_load(&s_last, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
    bool leave = (uint32_t)now - last > (uint32_t)idle_ticks || now - t_start > life_ticks;
    if ((poll & 63u) == 63u) leave = leave || ld_sys32(&sh->ctl[kSvcStop]) != 0u;
    if (leave) {
      if (lane == 0) __hip_atomic_store(&s_leave, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
      break;
    }
    __builtin_amdgcn_s_sleep(1);
  }
  // the last wave out tells the host this instance is gone (a vector store)
  if (lane == 0) {
    const uint32_t left = __hip_atomic_fetch_sub(&s_alive, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
    if (left == 1u) __hip_atomic_store(&sh->ctl[kSvcExited], instance, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
  }
}

} // namespace

hipError_t launch_service(SvcShared *sh, const uint32_t *tq, const uint32_t *kshift, uint64_t idle_ticks,
                          uint64_t life_ticks, uint32_t instance, hipStream_t stream) {
  hipLaunchKernelGGL(crc32_service_kernel, dim3(1), dim3(64 * kSvcWaves), 0, stream, sh, tq, kshift, idle_ticks,
                     life_ticks, instance);
  return hipGetLastError();
}

} // namespace rpccrc
