// tools/randread.hip — memory-system microbenchmarks for the roofline discussion:
// random aligned reads of W bytes from a table of T bytes (the LP probe's table access pattern,
// without the probe logic) and a streaming copy (the achievable HBM ceiling).
// Build: hipcc --offload-arch=gfx950 -O3 -o tools/randread tools/randread.hip
#include <hip/hip_runtime.h>

#include <cstdio>
#include <cstdlib>

#define CK(x)                                                                   \
  do {                                                                          \
    hipError_t e = (x);                                                         \
    if (e != hipSuccess) {                                                      \
      printf("HIP error %s at %s:%d\n", hipGetErrorString(e), __FILE__, __LINE__); \
      exit(1);                                                                  \
    }                                                                           \
  } while (0)

__device__ __forceinline__ uint64_t mix(uint64_t z) {
  z = (z ^ (z >> 30)) * 0xbf58476d1ce4e5b9ULL;
  z = (z ^ (z >> 27)) * 0x94d049bb133111ebULL;
  return z ^ (z >> 31);
}

// Each thread performs `per` independent random reads of W bytes (W/16 dwordx4, or one 8-B load).
template <int W, int PER>
__global__ void rand_read(const int64_t *table, uint64_t n_units, uint64_t n_threads, unsigned long long *sink) {
  const uint64_t t = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (t >= n_threads) return;
  int64_t acc = 0;
  int64_t v[PER][W >= 16 ? W / 8 : 1];
#pragma unroll
  for (int k = 0; k < PER; ++k) {
    const uint64_t u = mix(t * PER + k + 12345) % n_units;
    const int64_t *p = table + u * (W / 8 > 0 ? W / 8 : 1);
    if (W >= 16) {
#pragma unroll
      for (int q = 0; q < W / 16; ++q) {
        const longlong2 x = reinterpret_cast<const longlong2 *>(p)[q];
        v[k][2 * q] = x.x;
        v[k][2 * q + 1] = x.y;
      }
    } else {
      v[k][0] = p[0];
    }
  }
#pragma unroll
  for (int k = 0; k < PER; ++k)
#pragma unroll
    for (int q = 0; q < (W >= 16 ? W / 8 : 1); ++q) acc ^= v[k][q];
  if (acc == 0x1234567) atomicAdd(sink, 1ull);
}

__global__ void copy_stream(const int4 *src, int4 *dst, uint64_t n) {
  for (uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (uint64_t)gridDim.x * blockDim.x)
    dst[i] = src[i];
}

template <int W, int PER>
void run_rand(const int64_t *table, uint64_t table_bytes, unsigned long long *sink, uint64_t reads) {
  const uint64_t n_units = table_bytes / (W >= 8 ? W : 8);
  const uint64_t n_threads = reads / PER;
  hipEvent_t a, b;
  CK(hipEventCreate(&a));
  CK(hipEventCreate(&b));
  const unsigned grid = (unsigned)((n_threads + 255) / 256);
  hipLaunchKernelGGL((rand_read<W, PER>), dim3(grid), dim3(256), 0, 0, table, n_units, n_threads, sink);
  CK(hipEventRecord(a));
  for (int i = 0; i < 3; ++i)
    hipLaunchKernelGGL((rand_read<W, PER>), dim3(grid), dim3(256), 0, 0, table, n_units, n_threads, sink);
  CK(hipEventRecord(b));
  CK(hipEventSynchronize(b));
  float ms;
  CK(hipEventElapsedTime(&ms, a, b));
  ms /= 3;
  printf("{\"test\": \"rand_read\", \"width_B\": %d, \"per_thread\": %d, \"table_MiB\": %llu, \"reads\": %llu, "
         "\"ms\": %.3f, \"Greads_per_s\": %.2f, \"useful_GBps\": %.1f}\n",
         W, PER, (unsigned long long)(table_bytes >> 20), (unsigned long long)reads, ms, reads / ms / 1e6,
         reads * (double)W / ms / 1e6);
}

int main() {
  const uint64_t tbytes = 2ull << 30;
  int64_t *table;
  unsigned long long *sink;
  CK(hipMalloc(&table, tbytes));
  CK(hipMemset(table, 1, tbytes));
  CK(hipMalloc(&sink, 8));
  const uint64_t reads = 1ull << 28;
  run_rand<8, 4>(table, tbytes, sink, reads);
  run_rand<8, 8>(table, tbytes, sink, reads);
  run_rand<32, 4>(table, tbytes, sink, reads);
  run_rand<64, 2>(table, tbytes, sink, reads);
  run_rand<128, 1>(table, tbytes, sink, reads);
  run_rand<8, 4>(table, 128ull << 20, sink, reads);   // fits the Infinity Cache
  run_rand<32, 4>(table, 128ull << 20, sink, reads);
  run_rand<32, 4>(table, 2ull << 20, sink, reads);    // fits L2
  // streaming copy ceiling
  const uint64_t n = (4ull << 30) / 16;
  int4 *src, *dst;
  CK(hipMalloc(&src, n * 16));
  CK(hipMalloc(&dst, n * 16));
  CK(hipMemset(src, 3, n * 16));
  hipEvent_t a, b;
  CK(hipEventCreate(&a));
  CK(hipEventCreate(&b));
  hipLaunchKernelGGL(copy_stream, dim3(256 * 16), dim3(256), 0, 0, src, dst, n);
  CK(hipEventRecord(a));
  for (int i = 0; i < 3; ++i) hipLaunchKernelGGL(copy_stream, dim3(256 * 16), dim3(256), 0, 0, src, dst, n);
  CK(hipEventRecord(b));
  CK(hipEventSynchronize(b));
  float ms;
  CK(hipEventElapsedTime(&ms, a, b));
  ms /= 3;
  printf("{\"test\": \"stream_copy\", \"bytes_moved\": %llu, \"ms\": %.3f, \"GBps\": %.1f}\n",
         (unsigned long long)(2 * n * 16), ms, 2.0 * n * 16 / ms / 1e6);
  return 0;
}
