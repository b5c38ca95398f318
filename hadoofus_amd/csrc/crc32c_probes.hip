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
// rounds inside it (the tiled CRC kernel's pattern).
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
    default: return hipErrorInvalidValue;
  }
  return hipGetLastError();
}

}  // namespace hdfs_crc32c
