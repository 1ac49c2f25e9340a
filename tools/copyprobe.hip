// Fabric-traffic calibration (profiling aid): a plain 16-byte-per-lane streaming copy of 750 MB,
// nt and default stores. Under `rocprofv3 --pmc TCC_EA0_WRREQ_64B` / `TCC_EA0_RDREQ_128B` it shows
// what the counters report for a copy whose bytes are known exactly.
// Build: hipcc --offload-arch=gfx950 -O3 -o /tmp/copyprobe tools/copyprobe.hip
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdint>

typedef unsigned int u32x4 __attribute__((ext_vector_type(4)));

template <bool NT>
__global__ void __launch_bounds__(256) k_copy(const u32x4 *__restrict__ in, u32x4 *__restrict__ out, size_t n) {
  for (size_t i = blockIdx.x * (size_t)256 + threadIdx.x; i < n; i += (size_t)gridDim.x * 256) {
    const u32x4 v = in[i];
    if (NT) __builtin_nontemporal_store(v, out + i);
    else out[i] = v;
  }
}

int main() {
  const size_t bytes = 750000000 / 16 * 16, n = bytes / 16;
  u32x4 *a, *b;
  if (hipMalloc(&a, bytes) != hipSuccess || hipMalloc(&b, bytes) != hipSuccess) return 1;
  hipMemset(a, 1, bytes);
  hipMemset(b, 0, bytes);
  hipDeviceSynchronize();
  hipEvent_t e0, e1;
  hipEventCreate(&e0);
  hipEventCreate(&e1);
  for (int nt = 0; nt < 2; ++nt)
    for (int rep = 0; rep < 3; ++rep) {
      hipEventRecord(e0);
      if (nt) k_copy<true><<<8192, 256>>>(a, b, n);
      else k_copy<false><<<8192, 256>>>(a, b, n);
      hipEventRecord(e1);
      hipEventSynchronize(e1);
      float ms = 0;
      hipEventElapsedTime(&ms, e0, e1);
      printf("nt=%d rep=%d %.4f ms %.1f GB/s (read+write)\n", nt, rep, ms, 2.0 * bytes / ms / 1e6);
    }
  return 0;
}
