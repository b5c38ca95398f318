// Diagnostic streaming-read probes (not used by the CRC path): what HBM read
// rate can a gfx950 kernel reach with a given access shape and cache
// policy?  They bound the tiled kernel's roofline empirically.
//
// probe2_kernel<NLOAD, AUX, LDSDMA, ORDER>: a wave reads NLOAD KiB
// contiguous per round (NLOAD buffer_load_dwordx4, 1 KiB each, all in
// flight), then XORs them.  AUX = cache-policy bits of the load (gfx940+:
// 1 sc0, 2 nt, 16 sc1).  LDSDMA: global_load_lds_dwordx4 into LDS instead of
// VGPRs.  ORDER 0: rounds interleaved over all waves of the grid;
// ORDER 1: each workgroup owns a contiguous slice, its waves interleave
// rounds inside it; ORDER 2: as 0 with workgroups dealt XCD-major (the tiled
// CRC kernel's schedule-3 pattern).
#include <hip/hip_runtime.h>

#include <cstdint>

namespace hdfs_crc32c {

typedef uint32_t p32x4 __attribute__((ext_vector_type(4)));

template <int NLOAD, int AUX, int LDSDMA, int ORDER>
__global__ __launch_bounds__(1024) void probe2_kernel(const uint8_t *__restrict__ p, uint64_t nbytes,
                                                      uint32_t *__restrict__ out) {
  __shared__ __attribute__((aligned(16))) uint32_t lds[LDSDMA ? 16 * NLOAD * 256 : 4];
  const uint32_t lane = threadIdx.x & 63u, wave = threadIdx.x >> 6, wpb = blockDim.x >> 6;
  constexpr uint64_t rb = NLOAD * 1024ull;
  const uint64_t nr = nbytes / rb;
  uint64_t r, r1, step;
  if (ORDER == 0) {
    r = uint64_t(blockIdx.x) * wpb + wave;
    r1 = nr;
    step = uint64_t(gridDim.x) * wpb;
  } else if (ORDER == 2) {
    // as ORDER 0 but blocks dealt XCD-major (XCD = blockIdx % 8): each XCD
    // sweeps a contiguous run of gridDim/8 blocks' rounds per step
    const uint32_t G = gridDim.x, b = blockIdx.x;
    const uint32_t vb = (G % 8u) == 0 ? (b % 8u) * (G / 8u) + b / 8u : b;
    r = uint64_t(vb) * wpb + wave;
    r1 = nr;
    step = uint64_t(G) * wpb;
  } else {
    const uint64_t b0 = nr * blockIdx.x / gridDim.x, b1 = nr * (blockIdx.x + 1) / gridDim.x;
    r = b0 + wave;
    r1 = b1;
    step = wpb;
  }
  p32x4 acc = {0u, 0u, 0u, 0u};
  for (; r < r1; r += step) {
    const uint8_t *base = p + r * rb;
    if constexpr (LDSDMA) {
#pragma unroll
      for (int k = 0; k < NLOAD; k++)
        __builtin_amdgcn_global_load_lds(
            (const __attribute__((address_space(1))) void *)(base + k * 1024 + lane * 16),
            (__attribute__((address_space(3))) void *)(&lds[(wave * NLOAD + k) * 256]), 16, 0, AUX);
      __builtin_amdgcn_s_waitcnt(0);
      acc.x ^= lds[(wave * NLOAD) * 256 + lane];
    } else {
      const __amdgpu_buffer_rsrc_t rs =
          __builtin_amdgcn_make_buffer_rsrc(const_cast<uint8_t *>(base), 0, static_cast<int>(rb), 0x00020000);
      p32x4 v[NLOAD];
#pragma unroll
      for (int k = 0; k < NLOAD; k++) v[k] = __builtin_amdgcn_raw_buffer_load_b128(rs, k * 1024 + lane * 16, 0, AUX);
#pragma unroll
      for (int k = 0; k < NLOAD; k++) acc ^= v[k];
    }
  }
  const uint32_t v = acc.x ^ acc.y ^ acc.z ^ acc.w;
  if (v == 0x9E3779B9u) out[0] = v;  // keeps the loads live
}

// probe3_kernel<NLOAD, DEPTH>: software-pipelined like the tiled CRC kernel:
// a wave's rounds are NLOAD KiB (NLOAD nontemporal buffer_load_dwordx4),
// DEPTH rounds in register buffers, DEPTH-1 always in flight while one is
// consumed; rounds dealt to waves grid-interleaved with workgroups taken
// XCD-major.  The closest pure-read model of the tiled kernel's stream.
template <int NLOAD, int DEPTH>
__global__ __launch_bounds__(1024) void probe3_kernel(const uint8_t *__restrict__ p, uint64_t nbytes,
                                                      uint32_t *__restrict__ out) {
  const uint32_t lane = threadIdx.x & 63u, wave = threadIdx.x >> 6, wpb = blockDim.x >> 6;
  constexpr uint64_t rb = NLOAD * 1024ull;
  const uint64_t nr = nbytes / rb;
  const uint32_t G = gridDim.x, b = blockIdx.x;
  const uint32_t vb = (G % 8u) == 0 ? (b % 8u) * (G / 8u) + b / 8u : b;
  const uint64_t step = uint64_t(G) * wpb;
  uint64_t r = uint64_t(vb) * wpb + wave;
  p32x4 buf[DEPTH][NLOAD];
  p32x4 acc = {0u, 0u, 0u, 0u};
  auto issue = [&](p32x4 (&v)[NLOAD], uint64_t rr) {
    const uint64_t rc = rr < nr ? rr : nr - 1;  // clamp: loads stay unconditional, vmcnt counted
    const __amdgpu_buffer_rsrc_t rs =
        __builtin_amdgcn_make_buffer_rsrc(const_cast<uint8_t *>(p + rc * rb), 0, static_cast<int>(rb), 0x00020000);
#pragma unroll
    for (int k = 0; k < NLOAD; k++) v[k] = __builtin_amdgcn_raw_buffer_load_b128(rs, k * 1024 + lane * 16, 0, 2);
  };
  if (r >= nr) return;
#pragma unroll
  for (int d = 0; d < DEPTH; d++) issue(buf[d], r + d * step);
  for (;;) {
#pragma unroll
    for (int d = 0; d < DEPTH; d++) {
#pragma unroll
      for (int k = 0; k < NLOAD; k++) acc ^= buf[d][k];
      issue(buf[d], r + DEPTH * step);
      r += step;
    }
    if (r >= nr) break;
  }
  const uint32_t v = acc.x ^ acc.y ^ acc.z ^ acc.w;
  if (v == 0x9E3779B9u) out[0] = v;  // keeps the loads live
}

#define P3(N, D) \
  hipLaunchKernelGGL((probe3_kernel<N, D>), dim3(grid), dim3(block), 0, stream, p, nbytes, out)

#define P2(N, A, L, O) \
  hipLaunchKernelGGL((probe2_kernel<N, A, L, O>), dim3(grid), dim3(block), 0, stream, p, nbytes, out)

// variant 10..: see the table in DESIGN.md / tools/exp_probe.py
hipError_t launch_probe2(const uint8_t *p, uint64_t nbytes, uint32_t *out, int grid, int block, int variant,
                         hipStream_t stream) {
  switch (variant) {
    case 10: P2(8, 0, 0, 0); break;
    case 11: P2(8, 2, 0, 0); break;
    case 12: P2(8, 16, 0, 0); break;
    case 13: P2(8, 18, 0, 0); break;
    case 14: P2(16, 2, 0, 0); break;
    case 15: P2(8, 2, 0, 1); break;
    case 16: P2(16, 2, 0, 1); break;
    case 17: P2(8, 2, 1, 0); break;
    case 18: P2(8, 2, 1, 1); break;
    case 19: P2(4, 2, 0, 1); break;
    case 20: P2(8, 17, 0, 0); break;
    case 21: P2(8, 0, 0, 1); break;
    case 22: P2(4, 2, 1, 1); break;
    case 23: P2(16, 0, 0, 0); break;
    case 24: P2(16, 2, 0, 2); break;  // XCD-major, 16 KiB per wave round, nt
    case 25: P2(8, 2, 0, 2); break;
    case 26: P2(8, 2, 1, 2); break;   // XCD-major LDS-DMA
    case 27: P2(4, 2, 1, 2); break;
    case 30: P3(4, 3); break;  // the tiled kernel's shape: 4 KiB rounds, 3 deep
    case 31: P3(4, 4); break;
    case 32: P3(8, 3); break;
    case 33: P3(4, 2); break;
    default: return hipErrorInvalidValue;
  }
  return hipGetLastError();
}

}  // namespace hdfs_crc32c
