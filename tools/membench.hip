// Store-pattern microbenchmark (profiling aid): how much do partially written 128-byte lines
// cost when their pieces come from different workgroups / XCDs?
//   full      : each wave writes whole lines (dword per lane, consecutive)
//   halves_x  : the two 64-byte halves of every line written by blocks on different XCDs
//   halves_s  : the two halves written by blocks on the same XCD (block ids 8 apart)
//   rec75_x   : 75-byte records, one per lane group, neighbours' records from other XCDs,
//               byte stores at record edges (the output pattern of per-read writers)
//   memcpy    : hipMemcpyAsync device-to-device of the same size
// Build: hipcc --offload-arch=gfx950 -O3 -o /tmp/membench tools/membench.hip
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdint>

#define CK(x) do { hipError_t e = (x); if (e != hipSuccess) { printf("%s: %s\n", #x, hipGetErrorString(e)); return 1; } } while (0)

constexpr size_t kBytes = size_t(768) << 20;

__global__ void k_full(uint32_t *out, size_t n_dw) {
  for (size_t i = blockIdx.x * (size_t)blockDim.x + threadIdx.x; i < n_dw; i += (size_t)gridDim.x * blockDim.x)
    out[i] = (uint32_t)i;
}

// line pairs: block b writes half (b & 1) of lines belonging to block-pair b >> 1 (xcd_split) or
// half ((b >> 3) & 1) of lines of block-pair (b & 7) + 8 * (b >> 4) (same XCD).
__global__ void k_halves(uint32_t *out, size_t n_lines, int same_xcd) {
  const int b = blockIdx.x;
  int half, pair;
  if (same_xcd) {
    half = (b >> 3) & 1;
    pair = (b & 7) + 8 * (b >> 4);
  } else {
    half = b & 1;
    pair = b >> 1;
  }
  const int n_pairs = gridDim.x / 2;
  // each pair handles lines pair, pair + n_pairs, ...; a block writes 16 dwords per line
  for (size_t line = pair + (threadIdx.x >> 4) * (size_t)n_pairs; line < n_lines; line += (size_t)n_pairs * (blockDim.x >> 4)) {
    out[line * 32 + half * 16 + (threadIdx.x & 15)] = (uint32_t)line;
  }
}

// 75-byte records; record r written by block (r % grid) — neighbours on other XCDs. Each record
// is written by 19 lanes: whole dwords inside it, bytes at its edges.
__global__ void k_rec75(uint8_t *out, size_t n_rec) {
  const int lane = threadIdx.x & 31, grp = threadIdx.x >> 5, gpb = blockDim.x >> 5;
  for (size_t r = blockIdx.x + (size_t)grp * gridDim.x; r < n_rec; r += (size_t)gridDim.x * gpb) {
    const size_t R0 = r * 75, R1 = R0 + 75;
    const size_t D = (R0 & ~size_t(3)) + 4 * lane;
    if (D >= R1) continue;
    const size_t lo = D > R0 ? D : R0, hi = D + 4 < R1 ? D + 4 : R1;
    if (lo == D && hi == D + 4) *reinterpret_cast<uint32_t *>(out + D) = (uint32_t)r;
    else for (size_t x = lo; x < hi; ++x) out[x] = (uint8_t)r;
  }
}

int main() {
  uint8_t *src, *dst;
  CK(hipMalloc(&src, kBytes));
  CK(hipMalloc(&dst, kBytes));
  CK(hipMemset(src, 1, kBytes));
  hipEvent_t e0, e1;
  CK(hipEventCreate(&e0));
  CK(hipEventCreate(&e1));
  auto timeit = [&](const char *name, auto launch) {
    for (int i = 0; i < 3; ++i) launch();
    hipEventRecord(e0);
    const int reps = 10;
    for (int i = 0; i < reps; ++i) launch();
    hipEventRecord(e1);
    hipEventSynchronize(e1);
    float ms = 0;
    hipEventElapsedTime(&ms, e0, e1);
    ms /= reps;
    printf("{\"pattern\": \"%s\", \"ms\": %.4f, \"write_GBps\": %.1f}\n", name, ms, kBytes / (ms * 1e-3) / 1e9);
  };
  const size_t n_dw = kBytes / 4, n_lines = kBytes / 128, n_rec = kBytes / 75;
  timeit("full", [&] { k_full<<<8192, 256>>>(reinterpret_cast<uint32_t *>(dst), n_dw); });
  timeit("halves_x", [&] { k_halves<<<8192, 256>>>(reinterpret_cast<uint32_t *>(dst), n_lines, 0); });
  timeit("halves_s", [&] { k_halves<<<8192, 256>>>(reinterpret_cast<uint32_t *>(dst), n_lines, 1); });
  timeit("rec75_x", [&] { k_rec75<<<8192, 256>>>(dst, n_rec); });
  timeit("memcpy", [&] { hipMemcpyAsync(dst, src, kBytes, hipMemcpyDeviceToDevice, 0); });
  CK(hipDeviceSynchronize());
  return 0;
}
