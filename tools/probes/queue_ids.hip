// Do the AQL queue's write / read dispatch ids (amd_queue_t, read through
// the kernel's queue pointer) show a packet queued behind a running kernel?
// A spinning kernel records {write, read} at its start, then polls write
// until it moves (or 20 ms pass); the host enqueues a second kernel on the
// same stream 2 ms after the first.  Prints the snapshots and times.
#include <hip/hip_runtime.h>
#include <hsa/amd_hsa_queue.h>

#include <chrono>
#include <cstddef>
#include <cstdio>
#include <thread>

__device__ inline unsigned long long qload(unsigned off) {
  const char *q = (const char *)(unsigned long long)(__builtin_amdgcn_queue_ptr());
  return *(volatile const unsigned long long *)(q + off);
}

__global__ void spin(unsigned long long *out) {
  if (threadIdx.x) return;
  const unsigned W = offsetof(amd_queue_t, write_dispatch_id), R = offsetof(amd_queue_t, read_dispatch_id);
  const unsigned long long w0 = qload(W), r0 = qload(R);
  const unsigned long long t0 = __builtin_amdgcn_s_memrealtime();
  unsigned long long w = w0, t = t0;
  while (w == w0 && t - t0 < 2000000ull) {  // 20 ms at 100 MHz
    __builtin_amdgcn_s_sleep(8);
    w = qload(W);
    t = __builtin_amdgcn_s_memrealtime();
  }
  const unsigned long long rl = qload(R);
  volatile unsigned long long *o = out;
  o[0] = w0; o[1] = r0; o[2] = w; o[3] = rl; o[4] = (t - t0) / 100ull;  // us
}

__global__ void tiny(unsigned long long *out) {
  if (threadIdx.x == 0) out[5] = 1;
}

int main() {
  unsigned long long *d = nullptr, h[6] = {};
  if (hipMalloc(&d, 64) != hipSuccess) return 1;
  hipStream_t s;
  if (hipStreamCreateWithFlags(&s, hipStreamNonBlocking) != hipSuccess) return 1;
  for (int rep = 0; rep < 3; rep++) {
    if (hipMemsetAsync(d, 0, 64, s) != hipSuccess) return 1;
    if (hipStreamSynchronize(s) != hipSuccess) return 1;
    const auto t0 = std::chrono::steady_clock::now();
    hipLaunchKernelGGL(spin, dim3(1), dim3(64), 0, s, d);
    std::this_thread::sleep_for(std::chrono::milliseconds(2));
    hipLaunchKernelGGL(tiny, dim3(1), dim3(64), 0, s, d);
    if (hipStreamSynchronize(s) != hipSuccess) return 1;
    const double ms = std::chrono::duration<double, std::milli>(std::chrono::steady_clock::now() - t0).count();
    if (hipMemcpy(h, d, sizeof(h), hipMemcpyDeviceToHost) != hipSuccess) return 1;
    std::printf("{\"rep\": %d, \"w0\": %llu, \"r0\": %llu, \"w_end\": %llu, \"r_end\": %llu, \"spin_us\": %llu, "
                "\"tiny_ran\": %llu, \"host_ms\": %.3f}\n", rep, h[0], h[1], h[2], h[3], h[4], h[5], ms);
  }
  return 0;
}
