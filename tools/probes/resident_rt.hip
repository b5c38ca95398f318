// Probe (GPU box): what a grid-wide resident kernel would save a block-sized
// call over a launch.  Both sides do no work; they measure the fixed path of
// a call that needs every CU:
//   launch:   hipLaunchKernelGGL of a 256 x 1024 grid holding 150 KiB of LDS
//             per workgroup (one per CU, as the verify kernels), whose last
//             workgroup to finish writes the call's sequence number to pinned
//             memory; the host spins on it.
//   resident: the same grid launched once; workgroup 0 polls a pinned request
//             word and relays it through device memory to the others, every
//             workgroup counts itself in, the last one writes the sequence
//             number to pinned memory; the host writes the request and spins.
// Every workgroup leaves on a quit request or after 2 s without one.
//   hipcc --offload-arch=gfx950 -O3 -o tools/probes/resident_rt tools/probes/resident_rt.hip
#include <hip/hip_runtime.h>

#include <algorithm>
#include <chrono>
#include <cstdio>
#include <cstdlib>
#include <vector>

#define CHK(x)                                                                          \
  do {                                                                                  \
    hipError_t e_ = (x);                                                                \
    if (e_ != hipSuccess) {                                                             \
      std::fprintf(stderr, "%s: %s\n", #x, hipGetErrorString(e_));                      \
      std::exit(1);                                                                     \
    }                                                                                   \
  } while (0)

constexpr int kLdsWords = 150 * 1024 / 4;
constexpr unsigned kQuit = 0xFFFFFFFFu;

__global__ __launch_bounds__(1024) void launched(unsigned *done, unsigned *hout, unsigned seq) {
  __shared__ unsigned lds[kLdsWords];
  lds[threadIdx.x] = threadIdx.x;
  __syncthreads();
  if (threadIdx.x == 0) {
    const unsigned n = __hip_atomic_fetch_add(done, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    if (n + 1u == gridDim.x + lds[5] - 5u) {
      __hip_atomic_store(done, 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      __hip_atomic_store(hout, seq, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
    }
  }
}

__global__ __launch_bounds__(1024) void resident(const unsigned *req, unsigned *go, unsigned *done, unsigned *hout) {
  __shared__ unsigned lds[kLdsWords];
  __shared__ unsigned cur;
  lds[threadIdx.x] = threadIdx.x;
  unsigned last = 0;
  for (;;) {
    if (threadIdx.x == 0) {
      const unsigned long long t0 = __builtin_amdgcn_s_memrealtime();
      unsigned v = last;
      for (;;) {
        if (blockIdx.x == 0) {
          v = *(const volatile unsigned *)req;  // pinned host memory, system-coherent
          if (v != last) {
            __hip_atomic_store(go, v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
            break;
          }
        } else {
          v = __hip_atomic_load(go, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
          if (v != last) break;
        }
        if (__builtin_amdgcn_s_memrealtime() - t0 > 200000000ull) {  // 2 s idle
          v = kQuit;
          if (blockIdx.x == 0) __hip_atomic_store(go, kQuit, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
          break;
        }
        __builtin_amdgcn_s_sleep(1);
      }
      cur = v;
    }
    __syncthreads();
    const unsigned v = cur;
    if (v == kQuit) break;
    last = v;
    if (threadIdx.x == 0) {  // one counter per request parity: reset long before its next use
      unsigned *d = done + (v & 1u);
      const unsigned n = __hip_atomic_fetch_add(d, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      if (n + 1u == gridDim.x + lds[5] - 5u) {
        __hip_atomic_store(d, 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        __hip_atomic_store(hout, v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
      }
    }
    __syncthreads();
  }
}

static double now_us() {
  return std::chrono::duration<double, std::micro>(std::chrono::steady_clock::now().time_since_epoch()).count();
}

static void spin(volatile unsigned *w, unsigned v) {
  const double t0 = now_us();
  while (*w != v)
    if (now_us() - t0 > 2e6) {
      std::fprintf(stderr, "timeout waiting for %u\n", v);
      std::exit(2);
    }
}

int main(int argc, char **argv) {
  const int n = argc > 1 ? std::atoi(argv[1]) : 200;
  const int grid = argc > 2 ? std::atoi(argv[2]) : 256;
  unsigned *hreq = nullptr, *hout = nullptr, *go = nullptr, *done = nullptr;
  CHK(hipHostMalloc(&hreq, 64, hipHostMallocCoherent | hipHostMallocMapped));
  CHK(hipHostMalloc(&hout, 64, hipHostMallocCoherent | hipHostMallocMapped));
  CHK(hipMalloc(&go, 64));
  CHK(hipMalloc(&done, 64));
  CHK(hipMemset(go, 0, 64));
  CHK(hipMemset(done, 0, 64));
  *(volatile unsigned *)hreq = 0;
  *(volatile unsigned *)hout = 0;
  hipStream_t st;
  CHK(hipStreamCreateWithFlags(&st, hipStreamNonBlocking));
  std::vector<double> tl, tr;
  unsigned seq = 0;
  for (int i = 0; i < n + 10; i++) {  // launch path
    seq++;
    const double t0 = now_us();
    hipLaunchKernelGGL(launched, dim3(grid), dim3(1024), 0, st, done, hout, seq);
    spin(hout, seq);
    if (i >= 10) tl.push_back(now_us() - t0);
  }
  CHK(hipStreamSynchronize(st));
  hipLaunchKernelGGL(resident, dim3(grid), dim3(1024), 0, st, hreq, go, done, hout);
  CHK(hipGetLastError());
  for (int i = 0; i < n + 10; i++) {  // resident path
    seq++;
    const double t0 = now_us();
    __atomic_store_n(hreq, seq, __ATOMIC_RELEASE);
    spin(hout, seq);
    if (i >= 10) tr.push_back(now_us() - t0);
  }
  __atomic_store_n(hreq, kQuit, __ATOMIC_RELEASE);
  CHK(hipStreamSynchronize(st));
  std::sort(tl.begin(), tl.end());
  std::sort(tr.begin(), tr.end());
  std::printf("{\"grid\": %d, \"calls\": %d, \"launch_us\": {\"min\": %.2f, \"median\": %.2f}, "
              "\"resident_us\": {\"min\": %.2f, \"median\": %.2f}}\n",
              grid, n, tl[0], tl[tl.size() / 2], tr[0], tr[tr.size() / 2]);
  return 0;
}
