// Probe (GPU box): can the host write device memory directly (large-BAR
// fine-grained VRAM), and how fast is a 64 KiB memcpy into it compared with
// pinned host memory?  Prints one JSON line.  Exits non-zero if the
// allocation or the host access is refused.
#include <hip/hip_runtime.h>
#include <chrono>
#include <cstdio>
#include <cstring>
#include <vector>

__global__ void sum_kernel(const unsigned *p, unsigned n, unsigned *out) {
  unsigned s = 0;
  for (unsigned i = threadIdx.x; i < n; i += blockDim.x) s += p[i];
  atomicAdd(out, s);
}

int main() {
  const size_t n = 65536;
  void *dv = nullptr;
  hipError_t e = hipExtMallocWithFlags(&dv, n, hipDeviceMallocFinegrained);
  if (e != hipSuccess) { std::printf("{\"alloc\": \"%s\"}\n", hipGetErrorString(e)); return 2; }
  hipPointerAttribute_t a;
  (void)hipPointerGetAttributes(&a, dv);
  std::vector<unsigned char> src(n);
  for (size_t i = 0; i < n; i++) src[i] = (unsigned char)(i * 7);
  // host write through the pointer
  std::memcpy(dv, src.data(), n);
  unsigned *out;
  (void)hipMalloc(&out, 4);
  (void)hipMemset(out, 0, 4);
  hipLaunchKernelGGL(sum_kernel, dim3(1), dim3(256), 0, 0, (const unsigned *)dv, (unsigned)(n / 4), out);
  unsigned got = 0;
  (void)hipMemcpy(&got, out, 4, hipMemcpyDeviceToHost);
  unsigned want = 0;
  for (size_t i = 0; i < n / 4; i++) { unsigned w; std::memcpy(&w, src.data() + 4 * i, 4); want += w; }
  // timing: memcpy into VRAM vs into pinned host memory
  void *pin;
  (void)hipHostMalloc(&pin, n, hipHostMallocCoherent | hipHostMallocMapped);
  auto t = [&](void *dst) {
    double best = 1e9;
    for (int r = 0; r < 200; r++) {
      auto t0 = std::chrono::steady_clock::now();
      std::memcpy(dst, src.data(), n);
      __builtin_ia32_sfence();
      double us = std::chrono::duration<double, std::micro>(std::chrono::steady_clock::now() - t0).count();
      if (us < best) best = us;
    }
    return best;
  };
  const double tv = t(dv), tp = t(pin);
  // host read of VRAM (uncached over BAR)
  auto t0 = std::chrono::steady_clock::now();
  std::memcpy(src.data(), dv, 4096);
  double rd = std::chrono::duration<double, std::micro>(std::chrono::steady_clock::now() - t0).count();
  std::printf("{\"alloc\": \"ok\", \"type\": %d, \"host_write_visible\": %s, \"memcpy64k_vram_us\": %.2f, "
              "\"memcpy64k_pinned_us\": %.2f, \"read4k_vram_us\": %.2f}\n",
              (int)a.type, got == want ? "true" : "false", tv, tp, rd);
  return 0;
}
